"""Per-workgroup phase timing of the two step kernels from a diagnostic build with
s_memrealtime stamps (-DBPRMF_STEP_STAMPS): ml-20m shape, d = 128, B = 4096, the last step of a
64-step chunk.  Stamps: entry, record loaded, rows loaded / contributions summed, stores drained
(thread 0 of each workgroup waits for its own memory operations before each stamp).

  python tools/ubench_step_stamps.py build    # here: compile tools/libbprmf_step_stamps.so
  python tools/ubench_step_stamps.py          # GPU box
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "tools", "libbprmf_step_stamps.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    b = importlib.import_module("recommend-lib_amd.build")
    # fused launches only: the chunk's epilogue K2 would overwrite the last fused launch's K2
    print(b.build(force=True, defines=("BPRMF_STEP_STAMPS", "BPRMF_FUSED_STAMPS_ONLY=1"), out=LIB))
    sys.exit(0)

os.environ["BPRMF_DIAG_LIB"] = LIB
import ctypes  # noqa: E402

import numpy as np  # noqa: E402

rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
L = rl._lib.load()
L.bprmf_debug_step_stamps.argtypes = [ctypes.c_void_p]
U, I, d, B = 138493, 26744, 128, 4096
pos = syn.make_positives(U, I, 10_000_000, 20261015)
m = rl.BPRMF(U, I, d, batch_size=B, seed=1, device=0)
m.set_train(pos)
m.train_steps(0, 0, 256)
out = {}
samples = []
for rep in range(8):
    m.train_steps(0, 256 + 64 * rep, 64)
    st = np.zeros((2, 8192, 6), np.uint64)
    assert L.bprmf_debug_step_stamps(st.ctypes.data) == 0
    samples.append(st.astype(np.int64))
roles = {1: "long item", 2: "item", 3: "multi user"}


def summarize(st, k1_blocks, k2_blocks):
    res = {}
    k1 = st[0, :k1_blocks]
    k2 = st[1, :k2_blocks]
    # fused launch: K2 (step t) and K1 (step t+1) share the launch; time from its first start
    t0 = min(k1[:, 0].min(), k2[k2[:, 0] > 0][:, 0].min())
    us = lambda x: round(float(x) * 0.01, 2)  # 100 MHz ticks -> us
    res["K1 first start"] = us(k1[:, 0].min() - t0)
    res["K1 first start -> last start"] = us(k1[:, 0].max() - k1[:, 0].min())
    res["K1 record (median, max)"] = [us(np.median(k1[:, 1] - k1[:, 0])), us((k1[:, 1] - k1[:, 0]).max())]
    res["K1 wait (median, max)"] = [us(np.median(k1[:, 4] - k1[:, 1])), us((k1[:, 4] - k1[:, 1]).max())]
    res["K1 rows (median, max)"] = [us(np.median(k1[:, 2] - k1[:, 4])), us((k1[:, 2] - k1[:, 4]).max())]
    res["K1 stores (median, max)"] = [us(np.median(k1[:, 3] - k1[:, 2])), us((k1[:, 3] - k1[:, 2]).max())]
    res["K1 last end"] = us(k1[:, 3].max() - t0)
    res["K2 first start"] = us(k2[:, 0].min() - t0)
    res["K2 last start"] = us(k2[:, 0].max() - t0)
    for r, name in roles.items():
        sel = k2[:, 5] == r
        if not sel.any():
            continue
        x = k2[sel]
        live = x[:, 3] >= x[:, 0]
        if not live.any():
            continue
        x = x[live]
        res[f"K2 {name}: n"] = int(live.sum())
        res[f"K2 {name}: record (median, max)"] = [us(np.median(x[:, 1] - x[:, 0])), us((x[:, 1] - x[:, 0]).max())]
        res[f"K2 {name}: sums (median, max)"] = [us(np.median(x[:, 2] - x[:, 1])), us((x[:, 2] - x[:, 1]).max())]
        res[f"K2 {name}: stores (median, max)"] = [us(np.median(x[:, 3] - x[:, 2])), us((x[:, 3] - x[:, 2]).max())]
        res[f"K2 {name}: last end"] = us(x[:, 3].max() - t0)
    return res


k1_blocks = B // (256 // 32)
KB = 256  # K2 workgroup size (step.hip)
NG = KB // 32
lb = (B + KB - 1) // KB
k2_users = min(B // 2, B // 8)
# the item workgroups as step.hip k2_grid sizes them for the single-GPU step (capped: up to 6
# segments per lane group, kK2ItemLg = 384 lane groups per 1024 triplets)
lg = 384
item_blocks = (2 * B + NG - 1) // NG
if lg > 0:
    need = (2 * B + 6 * NG - 1) // (6 * NG)
    item_blocks = min(item_blocks, max(need, (B * lg // 1024 + NG - 1) // NG))
k2_blocks = lb + 64 + item_blocks + (k2_users + NG - 1) // NG
def by_len(st, k2_blocks):
    k2 = st[1, :k2_blocks]
    sel = (k2[:, 5] == 2) & (k2[:, 3] >= k2[:, 0]) & (k2[:, 2] > 0)
    x = k2[sel]
    t0 = st[0, :, 0][st[0, :, 0] > 0].min()
    out = {}
    for lo, hi in ((1, 4), (5, 8), (9, 12), (13, 16), (17, 10**6)):
        m = (x[:, 4] >= lo) & (x[:, 4] <= hi)
        if m.any():
            out[f"len {lo}-{hi}"] = dict(n=int(m.sum()), sums_med=round(float(np.median(x[m, 2] - x[m, 1])) * 0.01, 2),
                                         sums_max=round(float((x[m, 2] - x[m, 1]).max()) * 0.01, 2),
                                         end_max=round(float(x[m, 3].max() - t0) * 0.01, 2))
    return out


for n, st in enumerate(samples[2:]):
    # the last step's stamps: clear stale rows (their stamps are older than this K1's start)
    st = st.copy()
    # the last launch: K1 stamps of its step; K2 stamps of the same launch (within ~50 us)
    t0 = st[0, :k1_blocks, 0].min()
    st[1, :k2_blocks][st[1, :k2_blocks, 0] < t0 - 500] = 0
    out[f"rep{n}"] = summarize(st, k1_blocks, k2_blocks)
    out[f"rep{n}"]["items by length"] = by_len(st, k2_blocks)
print(json.dumps(out, indent=1))
