# local mode: HR@10 and throughput against the merge period (local_steps)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for ls in 32 64 128 256; do
  timeout -k 10 300 python3 bench.py --semantics local --local-steps $ls --no-cpu-baseline > "$out/bench_$ls.log" 2>&1 || exit 1
  BPRMF_LOCAL_STEPS_HR=$ls timeout -k 10 600 python3 tools/hr_modes.py --which ml20m,f5 --modes local --seeds 11 --local-steps $ls > "$out/hr_$ls.log" 2>&1 || exit 1
  python3 -c "
import json
b=json.loads(open('$out/bench_$ls.log').read().strip().splitlines()[-1])
hs=[json.loads(l) for l in open('$out/hr_$ls.log') if l.startswith('{')]
print('ls $ls', b['value'], b['roofline']['avg_us_per_step'], b['roofline']['frac'], [(h['workload'][:6], h['hr10'], h['ndcg10']) for h in hs])
"
done
