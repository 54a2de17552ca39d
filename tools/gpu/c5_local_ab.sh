# A/B of the local mode at the C5 shape on one GPU (10M x 100M, d = 256) between environment
# variants, interleaved, one bench.py process per run (settings read at set_train).
#   gpurun --timeout 1200 -- 'bash tools/gpu/c5_local_ab.sh <tag> <repeats> "name:ENV=v,..." ...'
set -o pipefail
tag="$1"; reps="$2"; shift 2
out="gpurun_out/$tag"
mkdir -p "$out"
C5="--users 10000000 --items 100000000 --positives 150000000 --factor 256"
for r in $(seq 1 "$reps"); do
  for spec in "$@"; do
    name="${spec%%:*}"; envs="${spec#*:}"
    ( [ "$envs" != "$spec" ] && [ -n "$envs" ] && for kv in ${envs//,/ }; do export "$kv"; done
      timeout -k 10 500 python3 bench.py $C5 --semantics local --steps 1024 --warmup 256 \
        --no-cpu-baseline --no-relaxed > "$out/${name}_$r.log" 2>&1 ) || { echo "variant $name failed"; tail -n 5 "$out/${name}_$r.log"; exit 1; }
    python3 -c "
import json
d=json.loads(open('$out/${name}_$r.log').read().strip().splitlines()[-1]); ro=d['roofline']
print('$name', $r, d['value'], ro['avg_us_per_step'], ro['frac'])
" | tee -a "$out/summary.txt"
  done
done
