"""GPU-side timeline of the last library call in a rocprofv3 kernel trace (from its sampler or,
without one, its batch-builder launch on): start, duration and the gap before each kernel, in
microseconds.

  python tools/trace_call.py gpurun_out/<tag>/prof/run_kernel_trace.csv
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [k for k, r in enumerate(rows) if "k_build_batches" in r["Kernel_Name"] or "k_build_split" in r["Kernel_Name"]]
first = starts[-1]
if first > 0 and "k_sample" in rows[first - 1]["Kernel_Name"]:
    first -= 1
t0 = prev = int(rows[first]["Start_Timestamp"])
for r in rows[first:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bprmf::", "")[:44]
    print(f"{(s - t0) / 1e3:8.2f} {(e - s) / 1e3:7.2f} gap {(s - prev) / 1e3:6.2f}  {name}")
    prev = e
print(f"total {(prev - t0) / 1e3:.2f} us")
