#!/bin/bash
# GPU box: FETCH_SIZE and WRITE_SIZE passes (separate runs) of the local mode's kernels at the C5
# shape on one GPU (112.6 GB of tables, far past the MALL: L2-miss traffic is HBM traffic); every
# launch a 128-step period.   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu/pmc_c5_local.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_c5_local
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 500 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 $R/bench.py --semantics local --users 10000000 --items 100000000 --positives 150000000 --factor 256 --steps 256 --warmup 128 --no-cpu-baseline --no-profile > $O/$c.out 2>&1 || { tail -5 $O/$c.out; exit 1; }
done
cd $R && python3 tools/pmc_traffic.py c5_d256_B4096_local $O/FETCH_SIZE $O/WRITE_SIZE --factor 256 --steps-per-launch 128 --out gpurun_out/pmc_c5_local/pmc_traffic_c5_local.json && python3 -c "
import json
d=json.load(open('gpurun_out/pmc_c5_local/pmc_traffic_c5_local.json'))['c5_d256_B4096_local']
print({k:v for k,v in d.items() if k!='kernels'})
"
