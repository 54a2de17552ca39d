# The owner plan at world 8 (in-process loopback shards on the one GPU, ml-20m per-rank shape)
# under rocprofv3 for each environment variant given (default: the list-pair form
# BPRMF_PLAN_PAIRS=1, the lane form, the sequential form BPRMF_PLAN_LANES=0); the sharded and IPC
# tests first, with the list-pair form.
#   gpurun --timeout 900 -- 'bash tools/gpu/plan_w8.sh <tag> ["ENV=a" ...]'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag="$1"; shift
[ $# -gt 0 ] || set -- "BPRMF_PLAN_PAIRS=1" "X=1" "BPRMF_PLAN_LANES=0"
out="$R/gpurun_out/$tag"
mkdir -p "$out"
cd "$R"
BPRMF_PLAN_PAIRS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_ipc.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/sh_tests.log" 2>&1
rc=$?
tail -2 "$out/sh_tests.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
n=0
for v in "$@"; do
  n=$((n + 1))
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/p$n" -o run --output-format csv -- python3 "$R/tools/ubench_plan_w8.py" 8 20 3 > "$out/p$n.log" 2>&1 || { tail -20 "$out/p$n.log"; exit 1; }
  f=$(find "$out/p$n" -name '*kernel_stats.csv' | head -1)
  echo "[$v]"; grep -E "plan" "$f" | python3 -c "
import sys, csv
for r in csv.reader(sys.stdin):
    print('  %-28s calls %5s avg %8.2f us' % (r[0].split('(')[0][-28:], r[1], float(r[3]) / 1e3))"
done
