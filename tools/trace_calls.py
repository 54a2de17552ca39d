"""Per-call GPU time by kernel from a rocprofv3 kernel trace: calls start at each sampler launch
(k_sample), and every kernel up to the next one belongs to that call.  Prints, per call, its
GPU span and the summed duration of each kernel kind, in microseconds.

  python tools/trace_calls.py gpurun_out/<tag>/prof/run_kernel_trace.csv [max calls]
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
limit = int(sys.argv[2]) if len(sys.argv) > 2 else 12
calls, cur = [], None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bprmf::", "")
    name = name.split("<")[0]
    if name == "k_sample":
        cur = {"t0": int(r["Start_Timestamp"]), "t1": 0, "k": collections.OrderedDict(), "n": 0}
        calls.append(cur)
    if cur is None:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    cur["t1"] = max(cur["t1"], e)
    cur["k"][name] = cur["k"].get(name, 0.0) + (e - s) / 1e3
    cur["n"] += 1
for c, x in enumerate(calls[:limit]):
    parts = " ".join(f"{k}={v:.1f}" for k, v in x["k"].items())
    print(f"call {c}: span {(x['t1'] - x['t0']) / 1e3:7.1f} us, {x['n']} kernels: {parts}")
