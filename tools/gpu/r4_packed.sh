# packed sampler reads: A/B of the driver-shaped call, then the whole GPU suite
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 600 python tools/ubench_call.py --ab "BPRMF_SAMPLE_PACKED=0" "BPRMF_SAMPLE_PACKED=1" "BPRMF_SAMPLE_PACKED=0" "BPRMF_SAMPLE_PACKED=1" > "$out/ab.log" 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$out/gpu_suite.log" 2>&1
rc=$?
cut -c1-330 "$out/ab.log"; tail -2 "$out/gpu_suite.log"
exit $rc
