# Round 4 A/B on one box: back-to-back 20-step calls (tools/ubench_call.py) of the current tree,
# its knobs, and the round-3 library (tools/libbprmf_r3.so), then bench.py K=20 three times each.
#   gpurun --timeout 900 -- 'bash tools/gpu/r4_ab.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 400 python tools/ubench_call.py --ab "UB_VARIANT=current" "BPRMF_K2_ITEM_LG=0" \
  "BPRMF_SAMPLE_TREE=0" "BPRMF_DIAG_LIB=tools/libbprmf_r3.so" "UB_VARIANT=current2" > "$out/ab.log" 2>&1
rc=$?
cat "$out/ab.log" | cut -c1-400
[ $rc -eq 0 ] || exit $rc
for v in cur r3 cur r3 cur r3; do
  if [ $v = r3 ]; then export BPRMF_DIAG_LIB=tools/libbprmf_r3.so; else unset BPRMF_DIAG_LIB; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-profile > "$out/bench_$v.log" 2>&1 || exit 1
  echo "$v $(grep '^{' $out/bench_$v.log | cut -c90-140)" | tee -a "$out/bench_ab.txt"
done
