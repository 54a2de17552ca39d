# tools/local_sweep.py on the box: the local mode's kernel under launch-setting variants, at one
# shape, in one process.   gpurun --timeout 1200 -- 'bash tools/gpu/local_sweep.sh <tag> <shape> "name:ENV=v" ...'
set -o pipefail
tag="$1"; shape="$2"; shift 2
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 1000 python -u tools/local_sweep.py --shape "$shape" --reps 2 "$@" > "$out/sweep.jsonl" 2> "$out/sweep.err" || { tail -n 20 "$out/sweep.err"; exit 1; }
cut -c1-300 "$out/sweep.jsonl"
