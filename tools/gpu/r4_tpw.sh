# local mode: throughput and HR@10 against triplets per wave (more waves in flight)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for cfg in "64 0" "32 0" "64 212000"; do
  set -- $cfg
  export BPRMF_HOGWILD_TPW=$1
  if [ "$2" = 0 ]; then unset BPRMF_HOGWILD_WINDOW; else export BPRMF_HOGWILD_WINDOW=$2; fi
  tag="$1_$2"
  timeout -k 10 300 python3 bench.py --semantics local --no-cpu-baseline > "$out/bench_$tag.log" 2>&1 || exit 1
  timeout -k 10 600 python3 tools/hr_modes.py --which ml20m --modes local --seeds 11 > "$out/hr_$tag.log" 2>&1 || exit 1
  python3 -c "
import json
b=json.loads(open('$out/bench_$tag.log').read().strip().splitlines()[-1]); h=json.loads(open('$out/hr_$tag.log').read().strip().splitlines()[-1])
print('$tag', b['value'], b['roofline']['avg_us_per_step'], b['roofline']['frac'], h['hr10'], h['ndcg10'], h['final_loss'])
"
done
