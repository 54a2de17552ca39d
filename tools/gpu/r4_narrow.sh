# hogwild/local kernel: narrow lane groups (G4/2, 2 stripes) A/B, and its tests
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
BPRMF_HOGWILD_NARROW=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hogwild.py tests/test_gpu_local_dp.py > "$out/tests.log" 2>&1 || { tail -20 "$out/tests.log"; exit 1; }
for v in 0 1 0 1; do
  BPRMF_HOGWILD_NARROW=$v timeout -k 10 300 python3 bench.py --semantics local --no-cpu-baseline > "$out/bench_$v.log" 2>&1 || exit 1
  BPRMF_HOGWILD_NARROW=$v timeout -k 10 300 python3 bench.py --semantics hogwild --no-cpu-baseline > "$out/bench_hog_$v.log" 2>&1 || exit 1
  python3 -c "
import json
b=json.loads(open('$out/bench_$v.log').read().strip().splitlines()[-1]); h=json.loads(open('$out/bench_hog_$v.log').read().strip().splitlines()[-1])
print('narrow $v local', b['value'], b['roofline']['avg_us_per_step'], 'hogwild', h['value'], h['roofline']['avg_us_per_step'])
"
done
tail -1 "$out/tests.log"
