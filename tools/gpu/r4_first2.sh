# first-call penalty: runtime pre-warm launches, no torch sync around calls, host trace
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 600 python tools/ubench_call.py --ab "UB_X=0" "BPRMF_DIAG_PREWARM=64" "BPRMF_DIAG_PREWARM=1024" "UB_NOSYNC=1" "UB_X=1" "BPRMF_DIAG_PREWARM=1024" > "$out/ab.log" 2>&1
rc=$?
cut -c1-420 "$out/ab.log"
exit $rc
