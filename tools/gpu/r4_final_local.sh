set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$out/gpu_suite.log" 2>&1 &&
timeout -k 10 300 python3 bench.py --semantics local > "$out/bench_local.log" 2>&1 &&
timeout -k 10 300 python3 bench.py --semantics local --steps 20 --warmup 5 > "$out/bench_local_k20.log" 2>&1
rc=$?
tail -2 "$out/gpu_suite.log"; tail -1 "$out/bench_local.log" | cut -c1-300; tail -1 "$out/bench_local_k20.log" | cut -c1-300
exit $rc
