# NCF row (C4) evaluation on one box: the NCF GPU tests, the lazy-Adam check against the oracle,
# tools/bench_ncf.py, and a rocprofv3 --kernel-trace --stats run of it (per-kernel averages).
#   gpurun --timeout 900 -- 'bash tools/gpu/ncf_eval.sh <tag> [bench args]'
set -o pipefail
tag="$1"; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ncf.py \
  tests/test_gpu_configs.py -k "ncf or c4" > "$out/tests.log" 2>&1 &&
timeout -k 10 120 python3 -u tools/dbg/ncf_lazy_check.py > "$out/check.json" 2>&1 &&
timeout -k 10 200 python3 -u tools/bench_ncf.py "$@" > "$out/bench.json" 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- \
  python3 "$R/tools/bench_ncf.py" --no-cpu-baseline --steps 200 --warmup 10 > "$out/prof.log" 2>&1 &&
cd "$R" && tail -n 3 "$out/tests.log" && grep '^{' "$out/bench.json" | cut -c1-700 &&
python3 tools/kstats.py "$(find "$out/prof" -name "*kernel_stats.csv")" > "$out/kstats.txt" && head -n 8 "$out/kstats.txt"
