# the ml-1m shape (d=64): capped vs full K2 item grid (BPRMF_K2_ITEM_LG=0), twice each
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for v in 384 0 384 0; do
  BPRMF_K2_ITEM_LG=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --users 6040 --items 3706 --positives 575000 --factor 64 > "$out/lg$v.log" 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$out/lg$v.log').read().strip().splitlines()[-1]); r=d['roofline']
print('lg $v', d['value'], r['avg_us_per_step'], r['frac'])
"
done
