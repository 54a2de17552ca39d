#!/bin/bash
# GPU box: FETCH_SIZE and WRITE_SIZE passes (separate runs, kernel trace only) over the BPR-FM and
# Item2Vec bench tools; CSVs under gpurun_out/pmc_sib/<tool>_<counter>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_sib
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for tool in bench_bprfm bench_sgns; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${tool}_$c -o run --output-format csv -- python3 $R/tools/$tool.py --epochs 1 --cpu-steps 1 > $O/${tool}_$c.out 2>&1 || { tail -5 $O/${tool}_$c.out; exit 1; }
  done
done
echo done
