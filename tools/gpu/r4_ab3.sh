# A/B of HIP runtime knobs on back-to-back 20-step calls (kernel arguments in device memory)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 500 python tools/ubench_call.py --ab "UB_VARIANT=default" "HIP_FORCE_DEV_KERNARG=1" \
  "HIP_FORCE_DEV_KERNARG=0" "UB_VARIANT=default2" "HIP_FORCE_DEV_KERNARG=1 UB_V=2" > "$out/ab.log" 2>&1
rc=$?
python3 -c "
import json,sys
for l in open('$out/ab.log'):
    if '{' in l: c=l[:l.index('{')]; d=json.loads(l[l.index('{'):]); print(c, d['us_per_step_median'], d['us_per_step_min'], d['library_us_per_step_median'], d['first_calls_us_per_step'][:3])
    else: print(l.strip()[:300])"
exit $rc
