# local mode: throughput and HR@10 against the in-flight window (BPRMF_HOGWILD_WINDOW)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for w in 0 53000 106000 212000; do
  if [ "$w" = 0 ]; then unset BPRMF_HOGWILD_WINDOW; else export BPRMF_HOGWILD_WINDOW=$w; fi
  timeout -k 10 300 python3 bench.py --semantics local --no-cpu-baseline > "$out/bench_$w.log" 2>&1 || exit 1
  timeout -k 10 600 python3 tools/hr_modes.py --which ml20m --modes local --seeds 11 > "$out/hr_$w.log" 2>&1 || exit 1
  python3 -c "
import json
b=json.loads(open('$out/bench_$w.log').read().strip().splitlines()[-1]); h=json.loads(open('$out/hr_$w.log').read().strip().splitlines()[-1])
print('$w', b['value'], b['roofline']['avg_us_per_step'], b['roofline']['frac'], h['hr10'], h['ndcg10'], h['final_loss'])
"
done
