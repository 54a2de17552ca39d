# Round-end evidence of a tree: the -m gpu suite, smoke(), the driver's bench line three times,
# the defaults, rocprofv3 --stats of the driver's command, and the PMC traffic passes of the
# headline fused step and of the local mode.   gpurun --timeout 1200 -- 'bash tools/gpu/final.sh <tag>'
set -o pipefail
tag="$1"
R=${GRAFT_REPO_ROOT:-$(pwd)}
out="$R/gpurun_out/$tag"
mkdir -p "$out"
step() {  # name, timeout, command...
  local name="$1" to="$2"; shift 2
  echo "== $name"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -n 2 "$out/$name.log" | cut -c1-300
  return $rc
}
step gpu_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread &&
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench20a 240 python bench.py --steps 20 --warmup 5 &&
step bench20b 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline &&
step bench20c 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline &&
step bench_defaults 300 python bench.py --no-cpu-baseline --no-relaxed &&
cd /tmp && export TMPDIR=/tmp &&
step prof 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline &&
cd "$R" &&
step pmc_headline 400 bash tools/gpu/pmc.sh "$tag/pmc_h" ml20m_d128_B4096 1 --steps 200 --warmup 20 &&
step pmc_local 400 bash tools/gpu/pmc.sh "$tag/pmc_l" ml20m_d128_B4096_local 128 --semantics local --steps 1024 --warmup 256
