set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_local_dp.py tests/test_gpu_hogwild.py > "$out/tests.log" 2>&1 &&
timeout -k 10 600 python3 tools/hr_modes.py --which f5 --modes local_dp8 --seeds 11,12,13 --dp-overlap > "$out/hr_f5_ov.log" 2>&1 &&
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes local_dp8 --seeds 11 --dp-steps 64 --dp-overlap > "$out/hr_ml_ov64.log" 2>&1 &&
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes local_dp8 --seeds 11 --dp-steps 256 --dp-overlap > "$out/hr_ml_ov256.log" 2>&1
rc=$?
tail -2 "$out/tests.log"; grep -h "{" "$out"/hr_*.log | cut -c1-330
exit $rc
