#!/bin/bash
# GPU box: FETCH_SIZE and WRITE_SIZE passes (separate runs) of the fused step at the C5 shape on one
# GPU (10M users x 100M items, d=256: 112.6 GB of tables, far past the 256 MiB MALL, so the L2-miss
# traffic these counters report is HBM traffic), then tools/pmc_traffic.py.
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/gpu/pmc_c5.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_c5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 $R/bench.py --users 10000000 --items 100000000 --positives 150000000 --factor 256 --steps 100 --warmup 20 --no-cpu-baseline --no-profile > $O/$c.out 2>&1 || { tail -5 $O/$c.out; exit 1; }
done
cd $R && python3 tools/pmc_traffic.py c5_d256_B4096 $O/FETCH_SIZE $O/WRITE_SIZE --factor 256 --out gpurun_out/pmc_c5/pmc_traffic_c5.json
