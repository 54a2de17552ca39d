# local mode at local_steps 128: more seeds
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m,f5 --modes local --seeds 12,13 --local-steps 128 > "$out/hr_128.log" 2>&1 &&
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes local_dp8 --seeds 11 --local-steps 128 --dp-steps 256 --dp-overlap > "$out/hr_dp8.log" 2>&1
rc=$?
cut -c1-250 "$out"/hr_*.log
exit $rc
