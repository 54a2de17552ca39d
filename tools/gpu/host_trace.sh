# bench.py at the driver's settings with BPRMF_HOST_TRACE=1, R times: host timestamps (us from the
# call's start) of each call's phases: build launch issued, returned, all launches enqueued, done.
#   gpurun --timeout 600 -- 'bash tools/gpu/host_trace.sh <tag> [R]'
set -o pipefail
tag="$1"; R="${2:-3}"
out="gpurun_out/$tag"
mkdir -p "$out"
for r in $(seq 1 "$R"); do
  BPRMF_HOST_TRACE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/b$r.log" 2> "$out/t$r.log" || { tail -5 "$out/t$r.log"; exit 1; }
  echo "run $r: $(grep '^{' "$out/b$r.log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  grep "host trace" "$out/t$r.log" | head -4
done
