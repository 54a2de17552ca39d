# shader clock per launch (diagnostic call-stamp build): the first 20-step call after the warm-up
# against later ones
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
timeout -k 10 200 python tools/ubench_call_stamps.py 10 > "$out/stamps.log" 2>&1
rc=$?
python3 -c "
import json
t=open('$out/stamps.log').read(); d=json.loads(t[t.index('{'):])
for c in d['per_call']: print(c)
" || tail -20 "$out/stamps.log"
exit $rc
