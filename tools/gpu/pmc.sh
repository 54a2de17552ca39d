# FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 --pmc runs, the MI355X_MICROARCH.md recipe)
# over one bench.py invocation, then tools/pmc_traffic.py: HBM bytes per step under <key>.
#   gpurun --timeout 1200 -- 'bash tools/gpu/pmc.sh <tag> <key> <steps-per-launch> [bench.py args...]'
# e.g. headline:  bash tools/gpu/pmc.sh pmc ml20m_d128_B4096 1 --steps 200 --warmup 20
#      local C5:  bash tools/gpu/pmc.sh pmc5 c5_d256_B4096_local 128 --semantics local --users 10000000 \
#                   --items 100000000 --positives 150000000 --factor 256 --steps 256 --warmup 128
set -o pipefail
tag="$1"; key="$2"; spl="$3"; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
fac=128
for ((a = 1; a <= $#; a++)); do [ "${!a}" = "--factor" ] && { b=$((a + 1)); fac="${!b}"; }; done
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 500 rocprofv3 --pmc $c -d "$O/$c" -o run --output-format csv -- python3 "$R/bench.py" \
    --no-cpu-baseline --no-profile --no-relaxed "$@" > "$O/$c.out" 2>&1 || { tail -n 5 "$O/$c.out"; exit 1; }
done
cd "$R" && python3 tools/pmc_traffic.py "$key" "$O/FETCH_SIZE" "$O/WRITE_SIZE" --factor "$fac" \
  --steps-per-launch "$spl" --out "$O/pmc_traffic.json" &&
python3 -c "
import json
d=json.load(open('$O/pmc_traffic.json'))['$key']
print({k: v for k, v in d.items() if k != 'kernels'})"
