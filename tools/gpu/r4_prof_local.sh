# rocprofv3 --stats of the local mode's bench line (every launch a 128-step period)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python3 bench.py --semantics local --no-cpu-baseline --steps 2048 --warmup 256 > "$out/bench.log" 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$out/prof" -o run --output-format csv -- python3 "$R/bench.py" --semantics local --no-cpu-baseline --steps 2048 --warmup 256 > "$R/$out/prof.log" 2>&1
rc=$?
cd "$R"
tail -1 "$out/bench.log" | cut -c1-200
python3 -c "
import csv
for r in csv.DictReader(open('$out/prof/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,2))
" | head -6
exit $rc
