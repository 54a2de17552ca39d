# local mode: merge period sweep (local_steps) at the default triplets per wave
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for ls in 16 32 64; do
  timeout -k 10 300 python3 bench.py --semantics local --local-steps $ls --no-cpu-baseline > "$out/bench_$ls.log" 2>&1 || exit 1
  python3 -c "
import json
b=json.loads(open('$out/bench_$ls.log').read().strip().splitlines()[-1])
print('ls $ls', b['value'], b['roofline']['avg_us_per_step'], b['roofline']['frac'])
"
done
