"""Summarise tools/gpu/pmc_sq.sh passes: per kernel name, mean of each SQ counter per dispatch,
and the wave-cycle split (SQ_* cycle counters are quad-cycles, MI355X_MICROARCH.md).
   python tools/pmc_sq.py gpurun_out/pmc_sq/<tag>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0][:60]
                acc[k][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    out = {}
    for k, m in acc.items():
        per = defaultdict(list)
        for (c, _), v in m.items():
            per[c].append(sum(v))  # summed over the dispatch's XCD/SE instances
        out[k] = {c: sum(v) / len(v) for c, v in per.items()} | {"dispatches": max(len(v) for v in per.values())}
    return out


def main():
    d = sys.argv[1]
    res = {}
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        if os.path.isdir(p):
            for k, v in load(p).items():
                res.setdefault(k, {}).update(v)
    for k, v in sorted(res.items()):
        print(k, json.dumps({c: round(x, 1) for c, x in sorted(v.items())}))
    with open(os.path.join(d, "pmc_sq.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
