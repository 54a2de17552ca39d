#!/bin/bash
# GPU box: Item2Vec GPU tests, bench line and a rocprofv3 kernel summary (outputs under gpurun_out/sgns)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sgns
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgns.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -12 $O/tests.log
if [ -f tools/bench_sgns.py ]; then
  timeout -k 10 200 python -u tools/bench_sgns.py "$@" > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 1; }
  cat $O/bench.json
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/tools/bench_sgns.py --epochs 1 --cpu-steps 1 "$@" > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
  f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
  cut -d, -f1-4 "$f" | head -12
fi
