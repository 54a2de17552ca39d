"""Phase timing of the batch builder (k_build_batches) from a diagnostic build with s_memrealtime
stamps (-DBPRMF_BUILD_STAMPS): the first workgroup's time per phase, ml-20m shape, B = 4096.

  python tools/ubench_build.py build          # here: compile tools/libbprmf_stamps.so
  python tools/ubench_build.py                # GPU box: run and print the phase table
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.environ.get("UB_LIB", os.path.join(ROOT, "tools", "libbprmf_stamps.so"))
PHASES = ["loads", "user sort", "user segments", "item keys+sort", "item heads/refs",
          "slot prefix", "item records", "triplet records"]

if len(sys.argv) > 1 and sys.argv[1] == "build":
    b = importlib.import_module("recommend-lib_amd.build")
    extra = tuple(a for a in sys.argv[2:] if a != "--split")  # further diagnostic defines
    # the step kernels never run on a diagnostic build's batches (some are wrong on purpose),
    # except in the split builder's form (--split: its batches are the shipped ones)
    if "--split" not in sys.argv:
        extra += ("BPRMF_DIAG_BUILD_ONLY",)
    print(b.build(force=True, defines=("BPRMF_BUILD_STAMPS",) + extra, out=LIB))
    sys.exit(0)

os.environ["BPRMF_DIAG_LIB"] = LIB
import ctypes  # noqa: E402

import numpy as np  # noqa: E402

rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
L = rl._lib.load()
L.bprmf_debug_build_stamps.argtypes = [ctypes.c_void_p]
pos = syn.make_positives(138493, 26744, 10_000_000, 20261015)
res = {}
if "--split" in sys.argv:  # the split builder (k_build_split): user workgroup, first / last item part
    m = rl.BPRMF(138493, 26744, 128, batch_size=4096, seed=1, device=0)
    m.set_train(pos)
    rows = []
    for rep in range(8):
        m.train_steps(0, 20 * rep, 20)
        st = np.zeros(32, np.uint64)
        assert L.bprmf_debug_build_stamps(st.ctypes.data) == 0
        rows.append((st.astype(np.int64) - int(st[0])) * 0.01)  # us from the user workgroup's start
    med = np.median(np.array(rows[2:]), axis=0)
    names_u = ["start", "loads", "user sort", "segments", "end"]
    names_i = ["start", "loads", "user sort", "ref keys", "sparse sort", "heads/refs", "exchange", "end"]
    res["user workgroup (us from its start)"] = {n: round(float(med[k]), 2) for k, n in enumerate(names_u)}
    res["first item part"] = {n: round(float(med[8 + k]), 2) for k, n in enumerate(names_i)}
    res["last item part"] = {n: round(float(med[16 + k]), 2) for k, n in enumerate(names_i)}
    # every workgroup of the last call's launch: start / end spread, per role, per batch
    L.bprmf_debug_split_se.argtypes = [ctypes.c_void_p]
    se = np.zeros((4096, 2), np.uint64)
    assert L.bprmf_debug_split_se(se.ctypes.data) == 0
    se = se[:20 * 9].astype(np.int64)
    t0 = se[:, 0].min()
    st, en = (se[:, 0] - t0) * 0.01, (se[:, 1] - t0) * 0.01
    role = np.arange(len(se)) % 9
    res["all workgroups (us from the first start)"] = {
        "start (median, max)": [round(float(np.median(st)), 2), round(float(st.max()), 2)],
        "user workgroup end (median, max)": [round(float(np.median(en[role == 0])), 2), round(float(en[role == 0].max()), 2)],
        "item part end (median, p90, max)": [round(float(np.median(en[role > 0])), 2),
                                             round(float(np.percentile(en[role > 0], 90)), 2), round(float(en[role > 0].max()), 2)],
        "slowest batch's ends": [round(float(x), 2) for x in en.reshape(20, 9)[int(np.argmax(en.reshape(20, 9).max(1)))]],
        "item part duration (median, max)": [round(float(np.median((en - st)[role > 0])), 2), round(float((en - st)[role > 0].max()), 2)],
    }
    print(json.dumps(res, indent=1))
    sys.exit(0)
for radix in ("0",) if "--quick" in sys.argv else ("0", "1"):
    for split in ("1",) if "--quick" in sys.argv else ("1", "0"):
        os.environ["BPRMF_SPLIT_BUILD"] = split
        if radix == "1":
            os.environ["BPRMF_RADIX_BUILD"] = "1"
        else:
            os.environ.pop("BPRMF_RADIX_BUILD", None)
        m = rl.BPRMF(138493, 26744, 128, batch_size=4096, seed=1, device=0)
        m.set_train(pos)
        rows = []
        for rep in range(5):
            try:
                m.train_steps(0, 20 * rep, 20)
            except rl.BprmfError:  # diagnostic builds that break the batches: stamps still valid
                pass
            st = np.zeros(32, np.uint64)
            assert L.bprmf_debug_build_stamps(st.ctypes.data) == 0
            d = np.diff(st[:9].astype(np.int64)) * 0.01  # 100 MHz -> us
            x = st.astype(np.int64)
            sub = np.diff(np.concatenate([x[3:4], x[9:14]])) * 0.01 if radix == "0" else np.zeros(5)
            usub = np.diff(np.concatenate([x[1:2], x[16:21]])) * 0.01 if radix == "0" else np.zeros(5)
            rows.append(np.concatenate([d, sub, usub]))
        med = np.median(np.array(rows[1:]), axis=0)
        key = f"radix={radix} split={split}"
        res[key] = {p: round(float(v), 2) for p, v in zip(PHASES, med[:8])}
        res[key]["total"] = round(float(med[:8].sum()), 2)
        if radix == "0":  # the item bucket sort's own phases
            res[key]["item sort phases"] = {p: round(float(v), 2) for p, v in zip(
                ("keys+count", "scan", "scatter", "rank", "gather"), med[8:13])}
            res[key]["user sort phases"] = {p: round(float(v), 2) for p, v in zip(
                ("count", "scan", "scatter", "rank", "gather"), med[13:18])}
        m.close()
print(json.dumps(res, indent=1))
