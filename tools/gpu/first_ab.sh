# First-call A/B: ubench_call processes alternating the variants given (each prints its first six
# calls and the steady median), R rounds.
#   gpurun --timeout 900 -- 'bash tools/gpu/first_ab.sh <tag> <R> "ENV=a" "ENV=b" ...'
set -o pipefail
tag="$1"; R="$2"; shift 2
out="gpurun_out/$tag"
mkdir -p "$out"
for r in $(seq 1 "$R"); do
  timeout -k 10 400 python -u tools/ubench_call.py --ab "$@" >> "$out/ab.log" 2>&1 || { tail -20 "$out/ab.log"; exit 1; }
done
python3 - "$out/ab.log" <<'PY'
import json, sys, collections
by = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if not line.startswith("["):
        continue
    cfg, js = line.split("] ", 1)
    d = json.loads(js)
    by[cfg[1:]].append(d)
for cfg, ds in by.items():
    first = [d["first_calls_us_per_step"][0] for d in ds]
    second = [d["first_calls_us_per_step"][1] for d in ds]
    med = [d["us_per_step_median"] for d in ds]
    print(f"{cfg:40s} first {sorted(first)} second {sorted(second)} steady {sorted(med)}")
PY
