"""Wall time of short library calls at the driver's bench shape (ml-20m, d=128, B=4096): each
call is timed like bench.py's timed region (device synchronise, call, synchronise), many times,
so one-call noise averages out.  Variants are environment settings, each in its own process.

  python tools/ubench_call.py [steps per call] [calls]          # one variant (current env)
  python tools/ubench_call.py --ab "ENV=.. ENV2=.." "ENV=.." ...  # several, one process each
"""
import importlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if len(sys.argv) > 1 and sys.argv[1] == "--ab":
    for cfg in sys.argv[2:]:
        env = dict(os.environ)
        for kv in cfg.split():
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True,
                           text=True, timeout=300)
        if r.returncode != 0:
            print(cfg, "FAILED", r.stderr[-2000:])
            sys.exit(1)
        print(f"[{cfg}] {r.stdout.strip().splitlines()[-1]}", flush=True)
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
U, I, d, B = 138493, 26744, 128, 4096
pos = syn.make_positives(U, I, 10_000_000, 20260101)
m = rl.BPRMF(U, I, d, lr=0.01, wd=0.001, batch_size=B, num_ng=4, seed=20260101, device=0)
m.set_train(pos)
n_steps = m.epoch_size()[1]
W = int(os.environ.get("UB_WARM", "5"))
if os.environ.get("UB_WARM_SPLIT"):  # the same W warm-up steps as two calls
    m.train_steps(0, 0, W // 2)
    m.train_steps(0, W // 2, W - W // 2)
else:
    m.train_steps(0, 0, W)
first, walls, inner, calls = W, [], [], []
if os.environ.get("UB_SPIN"):  # busy the GPU for ~UB_SPIN ms of unrelated work before the first call
    x = torch.randn(2048, 2048, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < float(os.environ["UB_SPIN"]) * 1e-3:
        x = x @ x
        x = x / x.norm()
        torch.cuda.synchronize()
if os.environ.get("UB_GC") == "0":  # no Python garbage collection inside the timed calls
    import gc
    gc.collect()
    gc.disable()
for c in range(N):
    if os.environ.get("UB_SPINCPU"):  # busy the host core for UB_SPINCPU ms before the call
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < float(os.environ["UB_SPINCPU"]) * 1e-3:
            pass
    e, s = divmod(first, n_steps)
    if s + K > n_steps:
        e, s = e + 1, 0
    nosync = os.environ.get("UB_NOSYNC") == "1"  # the library's own wait only
    if not nosync:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = m.train_steps(e, s, K)
    t1 = time.perf_counter()
    if not nosync:
        torch.cuda.synchronize()
    walls.append(time.perf_counter() - t0)
    calls.append(t1 - t0)
    inner.append(st["seconds"])
    first = e * n_steps + s + K
w = np.array(walls[5:]) * 1e6 / K
i = np.array(inner[5:]) * 1e6 / K
first_calls = [round(x * 1e6 / K, 2) for x in walls[:6]]
first_inner = [round(x * 1e6 / K, 2) for x in inner[:6]]
print(json.dumps({"steps_per_call": K, "calls": len(w), "first_calls_us_per_step": first_calls,
                  "first_calls_library_us_per_step": first_inner,
                  "first_calls_python_call_us": [round(x * 1e6, 1) for x in calls[:6]],
                  "first_calls_wall_us": [round(x * 1e6, 1) for x in walls[:6]],
                  "us_per_step_median": round(float(np.median(w)), 3),
                  "us_per_step_min": round(float(w.min()), 3),
                  "library_us_per_step_median": round(float(np.median(i)), 3)}))
