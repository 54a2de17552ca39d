# hogwild kernel with in-kernel sampling vs replaying pre-sampled triplets (k_sample first)
set -o pipefail
out="gpurun_out/$1"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/p0" -o run --output-format csv -- python3 bench.py --semantics hogwild --no-cpu-baseline --no-profile --steps 2000 --warmup 200 > "$out/b0.log" 2>&1 &&
BPRMF_HOGWILD_PRESAMPLE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/p1" -o run --output-format csv -- python3 bench.py --semantics hogwild --no-cpu-baseline --no-profile --steps 2000 --warmup 200 > "$out/b1.log" 2>&1
rc=$?
for v in 0 1; do echo "== presample $v"; python3 -c "
import csv
for r in csv.DictReader(open('$out/p$v/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,2), round(float(r['TotalDurationNs'])/1e6,3))
" | head -5; done
exit $rc
