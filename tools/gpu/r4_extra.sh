# extra evidence: 8-rank local mode HR@10 seeds 12/13 (dp 256, overlapped); the local mode at the
# C5 shape on one GPU (tables far past the MALL)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes local_dp8 --seeds 12,13 --dp-steps 256 --dp-overlap > "$out/hr_dp8.log" 2>&1 || exit 1
grep -h "{" "$out/hr_dp8.log" | cut -c1-260
timeout -k 10 1000 python3 bench.py --semantics local --users 10000000 --items 100000000 --positives 150000000 --factor 256 --steps 1024 --warmup 128 --no-cpu-baseline > "$out/c5_local.log" 2>&1
rc=$?
tail -1 "$out/c5_local.log" | cut -c1-400
exit $rc
