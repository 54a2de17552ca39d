# the first timed call: Python garbage collection off inside the timed calls (UB_GC=0) vs on
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 900 python tools/ubench_call.py --ab "UB_GC=1" "UB_GC=0" "UB_GC=1" "UB_GC=0" "UB_GC=1" "UB_GC=0" > "$out/ab.log" 2>&1
rc=$?
python3 -c "
import json
for l in open('$out/ab.log'):
    k,v=l.split('] ',1); d=json.loads(v)
    print(k, 'first', d['first_calls_us_per_step'][:2], 'py', d['first_calls_python_call_us'][:2], 'lib', d['first_calls_library_us_per_step'][:2], 'median', d['us_per_step_median'])
"
exit $rc
