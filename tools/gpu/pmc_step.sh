#!/bin/bash
# GPU box: FETCH_SIZE and WRITE_SIZE passes (separate runs) over a short bench.py run at the
# headline shape; CSVs under gpurun_out/pmc_step/<counter>, then tools/pmc_traffic.py.
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'bash tools/gpu/pmc_step.sh'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_step
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-profile > $O/$c.out 2>&1 || { tail -5 $O/$c.out; exit 1; }
done
cd $R && python3 tools/pmc_traffic.py ml20m_d128_B4096 $O/FETCH_SIZE $O/WRITE_SIZE --out gpurun_out/pmc_step/pmc_traffic.json
