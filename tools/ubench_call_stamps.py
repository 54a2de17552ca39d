"""The GPU timeline of one 20-step library call without a profiler: a diagnostic build
(-DBPRMF_CALL_STAMPS) records, per launch, the earliest workgroup start and the latest workgroup
end with s_memrealtime (100 MHz); this prints start / duration / gap before each launch, in us
from the call's first launch, median over calls (ml-20m shape, d=128, B=4096, the bench's setup).

  python tools/ubench_call_stamps.py build     # here: compile tools/libbprmf_cstamps.so
  python tools/ubench_call_stamps.py [calls]   # GPU box
Env knobs pass through (e.g. BPRMF_SPLIT_SAMPLE=0) for A/B.
"""
import ctypes
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.environ.get("UB_LIB", os.path.join(ROOT, "tools", "libbprmf_cstamps.so"))
SLOTS = {0: "build", 1: "k_sample", 2: "K1 (k_user_step)", 62: "last K2 (k_item_step)", 63: "k_status_out"}
SLOTS.update({3 + r: f"fused {r}" for r in range(19)})

if len(sys.argv) > 1 and sys.argv[1] == "build":
    b = importlib.import_module("recommend-lib_amd.build")
    print(b.build(force=True, defines=("BPRMF_CALL_STAMPS",), out=LIB))
    sys.exit(0)

os.environ["BPRMF_DIAG_LIB"] = LIB
rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
L = rl._lib.load()
readers = []
for tu in ("seg", "step", "ker"):
    f = getattr(L, f"bprmf_debug_call_stamps_{tu}")
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    readers.append(f)
calls = int(sys.argv[1]) if len(sys.argv) > 1 else 8
pos = syn.make_positives(138493, 26744, 10_000_000, 20261015)
m = rl.BPRMF(138493, 26744, 128, lr=0.01, wd=0.001, batch_size=4096, num_ng=4, seed=20261015)
m.set_train(pos)
m.train_steps(0, 0, 5)  # the bench's warm-up call
clk_step = L.bprmf_debug_clk_step
clk_step.argtypes = [ctypes.c_void_p]
clk_seg = L.bprmf_debug_clk_seg
clk_seg.argtypes = [ctypes.c_void_p]
rows, walls, mhz = [], [], []
import time  # noqa: E402
for c in range(calls):
    for f in readers:
        assert f(None, 1) == 0
    t0 = time.perf_counter()
    m.train_steps(0, 5 + 20 * c, 20)
    walls.append((time.perf_counter() - t0) * 1e6)
    tab = {}
    for f in readers:
        a = np.zeros((64, 2, 64), np.uint64)
        assert f(a.ctypes.data, 0) == 0
        for slot in range(64):
            st, en = a[slot, 0].min(), a[slot, 1].max()
            if st != np.iinfo(np.uint64).max and en:
                tab[slot] = (int(st), int(en))
    rows.append(tab)
    # shader clock during each fused launch (workgroup 0: s_memtime ticks per 10 ns of s_memrealtime)
    ck = np.zeros((64, 4), np.uint64)
    assert clk_step(ck.ctypes.data) == 0
    fs = [(int(ck[s, 2]) - int(ck[s, 0])) / max(1, int(ck[s, 3]) - int(ck[s, 1])) * 100.0
          for s in range(3, 22) if int(ck[s, 3]) > int(ck[s, 1])]
    cb = np.zeros((64, 4), np.uint64)
    assert clk_seg(cb.ctypes.data) == 0
    b = (int(cb[0, 2]) - int(cb[0, 0])) / max(1, int(cb[0, 3]) - int(cb[0, 1])) * 100.0 if int(cb[0, 3]) > int(cb[0, 1]) else None
    mhz.append({"fused_mhz_mean": round(float(np.mean(fs)), 1) if fs else None,
                "fused_mhz_first": round(fs[0], 1) if fs else None, "build_mhz": round(b, 1) if b else None})
t0s = [min(v[0] for v in tab.values()) for tab in rows]
out = {"wall_us_per_call": [round(w, 1) for w in walls], "launches": []}
order = sorted(rows[-1], key=lambda s: rows[-1][s][0])
prev_end = None
for slot in order:
    st = np.median([(tab[slot][0] - t0) * 0.01 for tab, t0 in zip(rows, t0s) if slot in tab])
    en = np.median([(tab[slot][1] - t0) * 0.01 for tab, t0 in zip(rows, t0s) if slot in tab])
    gap = st - prev_end if prev_end is not None else 0.0
    out["launches"].append({"launch": SLOTS.get(slot, str(slot)), "start_us": round(float(st), 2),
                            "dur_us": round(float(en - st), 2), "gap_before_us": round(float(gap), 2)})
    prev_end = en
out["span_us"] = round(float(prev_end), 2)
# per call: its GPU span, the build, the mean fused body, and the wall clock (the first calls
# after the warm-up are the bench's timed call)
per = []
for tab, t0, w in zip(rows, t0s, walls):
    end = max(v[1] for v in tab.values())
    fused = [tab[s][1] - tab[s][0] for s in range(3, 22) if s in tab]
    per.append({"wall_us": round(w, 1), "span_us": round((end - t0) * 0.01, 2),
                "build_us": round((tab[0][1] - tab[0][0]) * 0.01, 2) if 0 in tab else None,
                "fused_mean_us": round(float(np.mean(fused)) * 0.01, 2) if fused else None})
out["per_call"] = per
for p_, m_ in zip(per, mhz):
    p_.update(m_)
print(json.dumps(out, indent=1))
