# narrow default: GPU suite, local/hogwild HR, bench lines
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$out/gpu_suite.log" 2>&1 &&
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m,f5 --modes local,hogwild --seeds 11,12 > "$out/hr.log" 2>&1 &&
timeout -k 10 300 python3 bench.py --semantics local > "$out/bench_local.log" 2>&1 &&
timeout -k 10 300 python3 bench.py --semantics hogwild --no-cpu-baseline > "$out/bench_hog.log" 2>&1
rc=$?
tail -1 "$out/gpu_suite.log"; cut -c1-260 "$out/hr.log" | grep "{"; tail -1 "$out/bench_local.log" | cut -c1-200; tail -1 "$out/bench_hog.log" | cut -c1-200
exit $rc
