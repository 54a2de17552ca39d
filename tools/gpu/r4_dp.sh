# semantics "local" at world W (replicated item table): tests, merge-kernel durations, HR@10
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_local_dp.py > "$out/tests.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o dp -- python3 tools/ubench_local_dp.py 8 256 64 > "$out/ubench8.log" 2>&1 &&
timeout -k 10 200 python3 tools/ubench_local_dp.py 2 256 64 > "$out/ubench2.log" 2>&1 &&
timeout -k 10 600 python3 tools/hr_modes.py --which f5 --modes local_dp8,local_dp2 --seeds 11,12,13 > "$out/hr_f5.log" 2>&1 &&
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes local_dp8 --seeds 11 > "$out/hr_ml20m.log" 2>&1
rc=$?
tail -3 "$out/tests.log"; grep -h "{" "$out"/ubench*.log "$out"/hr_*.log | cut -c1-400
find "$out/prof" -name "*kernel_stats.csv" | head -2
exit $rc
