# GPU-box check of the tree: pytest -m gpu, then one default bench line.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/check.sh'
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 240 python bench.py "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
