"""Short summary of rocprofv3 `--stats` kernel tables (kernel_stats.csv): one line per kernel,
name shortened to its template head, calls and average/min/max microseconds.

  python tools/kstats.py <kernel_stats.csv> [...]        # every kernel
  python tools/kstats.py --only k_fused_step,k_user_step <csv> [...]   # the named kernels, one line per file
"""
import csv
import re
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)  # drop the argument list
    n = n.replace("void ", "").replace("bprmf::", "")
    return n


def read(path):
    rows = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            rows[short(r["Name"])] = dict(calls=int(r["Calls"]), avg=float(r["AverageNs"]) / 1e3,
                                          min=float(r["MinNs"]) / 1e3, max=float(r["MaxNs"]) / 1e3)
    return rows


def main(argv):
    only = None
    if argv and argv[0] == "--only":
        only = argv[1].split(",")
        argv = argv[2:]
    for p in argv:
        rows = read(p)
        if only:
            parts = []
            for k in only:
                hit = [(n, v) for n, v in rows.items() if re.sub(r"<.*", "", n) == k]
                for n, v in hit:
                    parts.append(f"{k} {v['avg']:.3f} us x{v['calls']}")
            print(f"{p}: " + "; ".join(parts))
        else:
            print(f"== {p}")
            for n, v in sorted(rows.items(), key=lambda kv: -kv[1]["avg"] * kv[1]["calls"]):
                print(f"  {n[:70]:70s} x{v['calls']:<6d} avg {v['avg']:8.3f}  min {v['min']:8.3f}  max {v['max']:8.3f} us")


if __name__ == "__main__":
    main(sys.argv[1:])
