# A/B: current vs no build-failure check (diag) vs round-3 library, back-to-back 20-step calls
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 500 python tools/ubench_call.py --ab "UB_VARIANT=current" \
  "BPRMF_DIAG_LIB=tools/libbprmf_nodead.so" "BPRMF_DIAG_LIB=tools/libbprmf_nodead.so BPRMF_K2_ITEM_LG=0" \
  "BPRMF_DIAG_LIB=tools/libbprmf_r3.so" "UB_VARIANT=current2" "BPRMF_DIAG_LIB=tools/libbprmf_nodead.so UB_V=2" \
  "BPRMF_DIAG_LIB=tools/libbprmf_r3.so UB_V=2" > "$out/ab.log" 2>&1
rc=$?
python3 -c "
import json,sys
for l in open('$out/ab.log'):
    if '{' in l: c=l[:l.index('{')]; d=json.loads(l[l.index('{'):]); print(c, d['us_per_step_median'], d['us_per_step_min'], d['library_us_per_step_median'])
    else: print(l.strip()[:300])"
exit $rc
