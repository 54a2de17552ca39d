# Evidence run: -m gpu suite, smoke(), bench lines at the driver's settings (3 runs) and the
# defaults, rocprofv3 --stats of a K=20 run and its call timeline.
#   gpurun --timeout 1200 -- 'bash tools/gpu/evidence.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -3 "$out/gpu_tests.log"
grep -q "illegal memory\|APERTURE\|Aborted\|core dumped" "$out/gpu_tests.log" && exit 3
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -5 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench20_$r.log" 2>&1 || { tail -5 "$out/bench20_$r.log"; exit 1; }
  grep '^{' "$out/bench20_$r.log" >> "$out/bench20.jsonl"
done
timeout -k 10 240 python bench.py --no-cpu-baseline > "$out/bench.log" 2>&1 || { tail -5 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" > "$out/bench.json"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --semantics hogwild --no-cpu-baseline > "$out/bench20_hog.log" 2>&1 || { tail -5 "$out/bench20_hog.log"; exit 1; }
grep '^{' "$out/bench20_hog.log" > "$out/bench20_hog.json"
timeout -k 10 240 python bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline > "$out/bench20_sh.log" 2>&1 || { tail -5 "$out/bench20_sh.log"; exit 1; }
grep '^{' "$out/bench20_sh.log" > "$out/bench20_sh.json"
python3 - "$out" <<'PY'
import json, sys
for f in ("bench20.jsonl", "bench.json", "bench20_hog.json", "bench20_sh.json"):
    for line in open(sys.argv[1] + "/" + f):
        d = json.loads(line)
        print(f, d["value"], d["ms_per_step"], d["roofline"]["avg_us_per_step"], d["roofline"]["frac"])
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_k20" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/prof_k20.log" 2>&1 || exit 1
find "$out/prof_k20" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats_k20.csv" \;
find "$out/prof_k20" -name '*kernel_trace.csv' -exec cp {} "$out/kernel_trace_k20.csv" \;
cut -c1-150 "$out/kernel_stats_k20.csv" | head -12
exit $rc
