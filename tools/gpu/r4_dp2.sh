# replicated-item mode: merge kernels at world 2 (csv stats), HR@10 vs merge period, full GPU suite
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o w2 --output-format csv -- python3 tools/ubench_local_dp.py 2 256 64 > "$out/ubench2.log" 2>&1 &&
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes local_dp8 --seeds 11 --dp-steps 256 > "$out/hr_256.log" 2>&1 &&
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes local_dp8 --seeds 11 --dp-steps 1024 > "$out/hr_1024.log" 2>&1 &&
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes exact,local --seeds 11 > "$out/hr_ref.log" 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$out/gpu_suite.log" 2>&1
rc=$?
grep -h "{" "$out"/ubench2.log "$out"/hr_*.log | cut -c1-330
tail -3 "$out/gpu_suite.log"
exit $rc
