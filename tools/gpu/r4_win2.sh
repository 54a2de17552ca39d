# local mode (128-step periods, narrow lane groups): in-flight window x triplets per wave
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for cfg in "0 0" "53000 0" "106000 0" "212000 0" "106000 32" "212000 32"; do
  set -- $cfg
  if [ "$1" = 0 ]; then unset BPRMF_HOGWILD_WINDOW; else export BPRMF_HOGWILD_WINDOW=$1; fi
  if [ "$2" = 0 ]; then unset BPRMF_HOGWILD_TPW; else export BPRMF_HOGWILD_TPW=$2; fi
  timeout -k 10 300 python3 bench.py --semantics local --no-cpu-baseline --steps 2000 --warmup 256 > "$out/bench_$1_$2.log" 2>&1 || exit 1
  python3 -c "
import json
b=json.loads(open('$out/bench_$1_$2.log').read().strip().splitlines()[-1])
print('window $1 tpw $2', b['value'], b['roofline']['avg_us_per_step'], b['roofline']['frac'])
"
done
