# bench.py at the driver's settings, five runs (GC paused inside the timed region), plus the
# ubench GC A/B
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for n in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/b$n.log" 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$out/b$n.log').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'])
"
done
bash tools/gpu/r4_gc.sh "$1/ub"
