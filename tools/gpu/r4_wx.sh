# local mode with the 4x window: HR@10 (F5 three seeds, ml-20m two) against 1x, and the bench
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
for wx in 4 1; do
  BPRMF_HOGWILD_LOCAL_WX=$wx timeout -k 10 900 python3 tools/hr_modes.py --which f5,ml20m --modes local --seeds 11,12,13 > "$out/hr_$wx.log" 2>&1 || exit 1
  BPRMF_HOGWILD_LOCAL_WX=$wx timeout -k 10 300 python3 bench.py --semantics local > "$out/bench_$wx.log" 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hogwild.py tests/test_gpu_local_dp.py > "$out/tests.log" 2>&1
rc=$?
for wx in 4 1; do python3 -c "
import json
b=json.loads(open('$out/bench_$wx.log').read().strip().splitlines()[-1])
print('wx $wx', b['value'], b['roofline']['avg_us_per_step'], b['roofline']['frac'])
for l in open('$out/hr_$wx.log'):
    if l.startswith('{'):
        h=json.loads(l); print('   ', h['workload'][:6], h['seed'], h['hr10'], h['ndcg10'], h['final_loss'])
"; done
tail -1 "$out/tests.log"
exit $rc
