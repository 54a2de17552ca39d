# K2 item lane groups per 1024 triplets (BPRMF_K2_ITEM_LG): 20-step call A/B
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 900 python tools/ubench_call.py --ab "BPRMF_K2_ITEM_LG=384" "BPRMF_K2_ITEM_LG=256" "BPRMF_K2_ITEM_LG=512" "BPRMF_K2_ITEM_LG=768" "BPRMF_K2_ITEM_LG=384" "BPRMF_K2_ITEM_LG=256" "BPRMF_K2_ITEM_LG=512" "BPRMF_K2_ITEM_LG=768" > "$out/ab.log" 2>&1
rc=$?
python3 -c "
import json
for l in open('$out/ab.log'):
    k,v=l.split('] ',1); d=json.loads(v)
    print(k, d['us_per_step_median'], d['us_per_step_min'], d['first_calls_us_per_step'][:2])
"
[ $rc = 0 ] || exit $rc
timeout -k 10 900 python3 tools/hr_modes.py --which ml20m --modes exact_b32768 --seeds 11 > "$out/hr_b32k.log" 2>&1
rc2=$?
grep -h "{" "$out/hr_b32k.log" | cut -c1-300
exit $rc2
