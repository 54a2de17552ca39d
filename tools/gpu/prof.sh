# rocprofv3 kernel trace + stats of one bench.py invocation; output under gpurun_out/<tag>/.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash tools/gpu/prof.sh <tag> [bench.py args...]'
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
tag="$1"; shift
out="$R/gpurun_out/$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$out/bench_prof.log" 2>&1 || { tail -20 "$out/bench_prof.log"; exit 1; }
grep '^{' "$out/bench_prof.log"
find "$out/prof" -name '*kernel_stats.csv' -exec cp {} "$out/kernel_stats.csv" \;
head -20 "$out/kernel_stats.csv"
