# exact kernels at 16 lanes x 2 stripes (BPRMF_GEOM_NARROW=1): parity tests first, then the A/B
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
BPRMF_GEOM_NARROW=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_build_tags.py tests/test_gpu_configs.py > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 600 python tools/ubench_call.py --ab "BPRMF_GEOM_NARROW=0" "BPRMF_GEOM_NARROW=1" "BPRMF_GEOM_NARROW=0" "BPRMF_GEOM_NARROW=1" > "$out/ab.log" 2>&1
rc=$?
python3 -c "
import json
for l in open('$out/ab.log'):
    k,v=l.split('] ',1); d=json.loads(v)
    print(k, d['us_per_step_median'], d['us_per_step_min'], d['first_calls_us_per_step'][:2])
"
exit $rc
