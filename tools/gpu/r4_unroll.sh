# hogwild/local kernel: triplets per lane group per round (kHwUnroll 2 / 3 / 4 builds)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for v in 2 3 4 2 3 4; do
  if [ $v = 2 ]; then unset BPRMF_DIAG_LIB; else export BPRMF_DIAG_LIB=tools/libbprmf_unr$v.so; fi
  timeout -k 10 300 python3 bench.py --semantics local --no-cpu-baseline --steps 2000 --warmup 256 > "$out/local_$v.log" 2>&1 || exit 1
  timeout -k 10 300 python3 bench.py --semantics hogwild --no-cpu-baseline --steps 2000 --warmup 256 > "$out/hog_$v.log" 2>&1 || exit 1
  python3 -c "
import json
a=json.loads(open('$out/local_$v.log').read().strip().splitlines()[-1]); b=json.loads(open('$out/hog_$v.log').read().strip().splitlines()[-1])
print('unroll $v local', a['value'], a['roofline']['avg_us_per_step'], 'hogwild', b['value'], b['roofline']['avg_us_per_step'])
"
done
