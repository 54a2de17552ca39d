set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_local_dp.py tests/test_gpu_hogwild.py > "$out/tests.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o w2 --output-format csv -- python3 tools/ubench_local_dp.py 2 256 64 > "$out/ubench2.log" 2>&1
rc=$?
tail -2 "$out/tests.log"; grep -h "{" "$out"/ubench2.log | cut -c1-330
python3 -c "
import csv
for r in csv.DictReader(open('$out/prof/w2_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1000,2), round(float(r['MinNs'])/1000,2))
"
exit $rc
