"""Per-step L2<->fabric traffic of the step kernels from rocprofv3 PMC CSVs.

  python tools/pmc_traffic.py KEY FETCH_DIR WRITE_DIR [--out profiles/pmc_traffic.json]

FETCH_SIZE and WRITE_SIZE (KB per dispatch) are averaged per kernel over all dispatches; the step
traffic is one fused launch's (single GPU, fused step), else the sum over the step kernels
(user_step + item_step; + owner-side kernels when sharded).  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly half the bytes
of a wide coalesced (16 B/lane) read, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
Infinity-Cache hits are counted by these counters (they are L2-miss requests), so for tables that
fit the 256 MiB MALL this is L2-miss traffic, not strictly DRAM bytes.
"""
import argparse
import collections
import csv
import glob
import json
import os

STEP_KERNELS = ("k_fused_step", "k_user_step", "k_item_step", "k_gather_rows", "k_add_rows",
                "k_apply_rows", "k_hogwild", "k_local_merge")


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            for k in STEP_KERNELS:
                if f"bprmf::{k}" in name:
                    acc[k].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("key")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--factor", type=int, default=128)
    ap.add_argument("--steps-per-launch", type=int, default=0,
                    help="relaxed modes: steps one k_hogwild launch covers (its bytes and one merge's "
                         "are divided by it)")
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_dir, "FETCH_SIZE")
    write = per_kernel(a.write_dir, "WRITE_SIZE")
    kernels = {k: dict(fetch_kb_raw=round(fetch.get(k, 0.0), 1), write_kb=round(write.get(k, 0.0), 1),
                       bytes=round((2 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024))
               for k in sorted(set(fetch) | set(write))}
    # single GPU, fused (default): one k_fused_step launch = K2 of a step + K1 of the next, so
    # one launch's traffic is one step's (the chunk's lone K1 and K2 launches are its two ends)
    if "k_fused_step" in kernels:
        total = kernels["k_fused_step"]["bytes"]
    elif "k_hogwild" in kernels and a.steps_per_launch > 0:  # relaxed: per launch (+ its merge) / steps
        total = round((kernels["k_hogwild"]["bytes"] + kernels.get("k_local_merge", {}).get("bytes", 0))
                      / a.steps_per_launch)
    else:
        total = sum(v["bytes"] for v in kernels.values())
    alg = a.batch * (24 * a.factor + 12)
    entry = dict(hbm_bytes_per_step=total, algorithmic_bytes_per_step=alg,
                 ratio_to_algorithmic=round(total / alg, 3), kernels=kernels,
                 method="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); "
                        "bytes = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024 (gfx950 FETCH_SIZE halving); "
                        "L2-miss traffic incl. Infinity-Cache hits")
    data = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            data = json.load(f)
    data[a.key] = entry
    with open(a.out, "w") as f:
        json.dump(data, f, indent=1)
    print(json.dumps({a.key: entry}, indent=1))


if __name__ == "__main__":
    main()
