# The first-call penalty: per-call GPU span vs wall (call stamps) and host phase times
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 200 python tools/ubench_call_stamps.py 10 > "$out/stamps.log" 2>&1 &&
BPRMF_HOST_TRACE=1 timeout -k 10 200 python tools/ubench_call.py 20 12 > "$out/host.log" 2>&1 &&
UB_WARM=25 timeout -k 10 200 python tools/ubench_call.py 20 12 > "$out/warm25.log" 2>&1
rc=$?
python3 -c "
import json
t=open('$out/stamps.log').read(); d=json.loads(t[t.index('{'):])
for c in d['per_call']: print(c)
"
grep -h "host trace\|first_calls" "$out/host.log" | cut -c1-300
grep -h "first_calls" "$out/warm25.log" | cut -c1-300
exit $rc
