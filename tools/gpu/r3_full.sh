# Round-3 evidence run: the whole -m gpu suite, smoke(), bench lines (driver settings, exact and
# hogwild; defaults), rocprofv3 --stats of the K=20 exact and hogwild runs.
#   gpurun --timeout 1500 -- 'bash tools/gpu/r3_full.sh <tag>'
set -o pipefail
tag="$1"
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -4 "$out/gpu_tests.log"
grep -q "illegal memory\|APERTURE\|Aborted\|core dumped" "$out/gpu_tests.log" && exit 3
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -5 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$out/bench20.log" 2>&1 || { tail -5 "$out/bench20.log"; exit 1; }
grep '^{' "$out/bench20.log" > "$out/bench20.json"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --semantics hogwild --no-cpu-baseline > "$out/bench20_hog.log" 2>&1 || { tail -5 "$out/bench20_hog.log"; exit 1; }
grep '^{' "$out/bench20_hog.log" > "$out/bench20_hog.json"
timeout -k 10 240 python bench.py --no-cpu-baseline > "$out/bench.log" 2>&1 || { tail -5 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" > "$out/bench.json"
timeout -k 10 240 python bench.py --no-cpu-baseline --semantics hogwild > "$out/bench_hog.log" 2>&1 || { tail -5 "$out/bench_hog.log"; exit 1; }
grep '^{' "$out/bench_hog.log" > "$out/bench_hog.json"
cut -c1-200 "$out"/bench*.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_k20" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/prof_k20.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_hog" -o run --output-format csv -- python bench.py --steps 2000 --warmup 100 --no-cpu-baseline --semantics hogwild > "$out/prof_hog.log" 2>&1 || exit 1
timeout -k 10 400 python tools/hr_modes.py --seeds 11,12 --epochs 10 > "$out/hr_modes.jsonl" 2>&1 || exit 1
cat "$out/hr_modes.jsonl" | grep '^{' | cut -c1-200
exit $rc
