"""Per-step, per-workgroup timing of the persistent step (step.hip k_persist_steps) from a
diagnostic build with s_memrealtime stamps (-DBPRMF_PERSIST_STAMPS): ml-20m shape, d = 128,
B = 4096, 20-step calls (the driver's bench setting).  Per step k and workgroup: after its gate,
after its body, after its arrival.  Printed per step: when the last K1 workgroup of step k
arrived (the gate both K2 of k and K1 of k+1 wait for), how long after that the waiters passed
their gates, how long K2's roles and K1 took, and the step period.

  python tools/ubench_persist_stamps.py build    # here: compile tools/libbprmf_pstamps.so
  python tools/ubench_persist_stamps.py          # GPU box
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "tools", "libbprmf_pstamps.so")
# --plain: the diagnostic variant whose persistent step reads with plain loads (WRONG results,
# timing only: what the sc1 loads cost)
PLAIN = "--plain" in sys.argv
if PLAIN:
    LIB = os.path.join(ROOT, "tools", "libbprmf_pstamps_plain.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    b = importlib.import_module("recommend-lib_amd.build")
    defs = ("BPRMF_PERSIST_STAMPS",) + (("BPRMF_PERSIST_PLAIN",) if PLAIN else ())
    print(b.build(force=True, defines=defs, out=LIB))
    sys.exit(0)

os.environ["BPRMF_DIAG_LIB"] = LIB
os.environ["BPRMF_PERSIST"] = "1"  # opt-in (capi.cpp persist_enabled)
import ctypes  # noqa: E402

import numpy as np  # noqa: E402

rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
L = rl._lib.load()
L.bprmf_debug_persist_stamps.argtypes = [ctypes.c_void_p]
L.bprmf_debug_persist_k1wait.argtypes = [ctypes.c_void_p]
L.bprmf_debug_persist_knobs.argtypes = [ctypes.c_void_p]
# --knobs a,b,c: extra s_sleep 4 iterations per stamp poll, K2 wave priority, extra per gate poll
KN = [0, 0, 0, 0]
for x in sys.argv:
    if x.startswith("--knobs="):
        KN[:3] = [int(v) for v in x.split("=", 1)[1].split(",")]
kn = (ctypes.c_int * 4)(*KN)
assert L.bprmf_debug_persist_knobs(kn) == 0
U, I, d, B = 138493, 26744, 128, 4096
pos = syn.make_positives(U, I, 10_000_000, 20261015)
m = rl.BPRMF(U, I, d, batch_size=B, seed=1, device=0)
m.set_train(pos)
for c in range(6):
    m.train_steps(0, 20 * c, 20)
total = m.debug_persist_grid()
assert total > 0, total
k1_blocks = B // (256 // 32)
k2_blocks = total - k1_blocks
NG = 256 // 32
lb = (B + 255) // 256
lg = 384
item_blocks = min((2 * B + NG - 1) // NG, max((2 * B + 6 * NG - 1) // (6 * NG), (B * lg // 1024 + NG - 1) // NG))
long_blocks = k2_blocks - lb - item_blocks - ((min(B // 2, B // 8) + NG - 1) // NG)
roles = {"loss": (0, lb), "hot": (lb, lb + long_blocks), "items": (lb + long_blocks, lb + long_blocks + item_blocks),
         "users": (lb + long_blocks + item_blocks, k2_blocks)}
us = lambda x: round(float(x) * 0.01, 2)  # 100 MHz ticks -> us
out = {"knobs": KN, "grid": dict(total=total, k1=k1_blocks, k2=k2_blocks, roles={k: v[1] - v[0] for k, v in roles.items()})}
for rep in range(3):
    m_t0 = m.steps_taken
    m.train_steps(0, 200 + 20 * rep, 20)
    st = np.zeros((32, 2048, 3), np.uint64)
    assert L.bprmf_debug_persist_stamps(st.ctypes.data) == 0
    st = st.astype(np.int64)
    kw = np.zeros((32, 1024, 32), np.uint64)
    assert L.bprmf_debug_persist_k1wait(kw.ctypes.data) == 0
    kflags = (kw >> np.uint64(60)).astype(np.int64)
    kw = (kw & np.uint64((1 << 60) - 1)).astype(np.int64)
    k2 = st[:20, :k2_blocks]
    k1 = st[:20, k2_blocks:total]
    T0 = k1[0, :, 0].min()
    steps = []
    for k in range(1, 19):
        last_k1 = k1[k, :, 2].max()  # K1 of step k: every workgroup arrived
        row = dict(k=k, k1_done=us(last_k1 - T0))
        row["period"] = us(last_k1 - k1[k - 1, :, 2].max())
        g2 = k2[k, :, 0] - last_k1
        row["K2 gate after last K1 (min, med, max)"] = [us(g2.min()), us(np.median(g2)), us(g2.max())]
        for name, (a, b) in roles.items():
            body = k2[k, a:b, 1] - k2[k, a:b, 0]
            row[f"K2 {name} body (med, max)"] = [us(np.median(body)), us(body.max())]
            row[f"K2 {name} end after last K1"] = us(k2[k, a:b, 1].max() - last_k1)
        g1 = k1[k + 1, :, 0] - last_k1
        row["K1(k+1) gate after last K1(k) (min, med, max)"] = [us(g1.min()), us(np.median(g1)), us(g1.max())]
        b1 = k1[k + 1, :, 1] - k1[k + 1, :, 0]
        row["K1(k+1) body (med, p90, max)"] = [us(np.median(b1)), us(np.percentile(b1, 90)), us(b1.max())]
        a1 = k1[k + 1, :, 2] - k1[k + 1, :, 1]
        row["K1(k+1) arrive (med, max)"] = [us(np.median(a1)), us(a1.max())]
        tk = (int(m_t0) + k + 2) & 31  # global step of K1(k+1)
        w = kw[tk, :k1_blocks, :32 // 4 * 1]  # 8 triplet slots per workgroup at d = 128
        w = w[:, :8]
        wmax = np.where(w > 0, w, 0).max(axis=1)
        ok = wmax > k1[k + 1, :, 0] - 100
        row["K1(k+1) waits done after its gate (med, p90, max)"] = [
            us(np.median((wmax - k1[k + 1, :, 0])[ok])), us(np.percentile((wmax - k1[k + 1, :, 0])[ok], 90)),
            us((wmax - k1[k + 1, :, 0])[ok].max())]
        row["K1(k+1) body end after waits (med, p90, max)"] = [
            us(np.median((k1[k + 1, :, 1] - wmax)[ok])), us(np.percentile((k1[k + 1, :, 1] - wmax)[ok], 90)),
            us((k1[k + 1, :, 1] - wmax)[ok].max())]
        row["K1(k+1) last waits done after last K1(k)"] = us(wmax[ok].max() - last_k1)
        steps.append(row)
    out[f"rep{rep}"] = steps
print(json.dumps(out, indent=1))
