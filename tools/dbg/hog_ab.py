"""A/B of hogwild launch knobs on the bench workload (ml-20m shape, d=128, B=4096), one process.
Prints per config: K=20 call time per step (wall, like bench.py) and a 1000-step call."""
import importlib, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
U, I, d, B = 138493, 26744, 128, 4096
pos = syn.make_positives(U, I, 10_000_000, 20261015)
configs = [c.split("=", 1) if c else [] for c in (sys.argv[1:] or [""])]
KNOBS = ("BPRMF_HOGWILD_TPW", "BPRMF_HOGWILD_PLAIN", "BPRMF_HOGWILD_BLOCKS", "BPRMF_HOGWILD_WINDOW",
         "BPRMF_HOGWILD_PRESAMPLE", "BPRMF_HOGWILD_DIAG")
for cfg in sys.argv[1:] or ["exact"]:
    for k in KNOBS:
        os.environ.pop(k, None)
    sem = "hogwild"
    for kv in cfg.split(","):
        if kv == "exact":
            sem = "exact"
        elif "=" in kv:
            k, v = kv.split("=")
            os.environ[k] = v
    m = rl.BPRMF(U, I, d, batch_size=B, seed=20261015, semantics=sem)
    m.set_train(pos)
    m.train_steps(0, 0, 5)
    ts = []
    for r in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.train_steps(0, 5 + 20 * r, 20)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / 20 * 1e6)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.train_steps(0, 200, 1000)
    torch.cuda.synchronize()
    tl = (time.perf_counter() - t0) / 1000 * 1e6
    print(json.dumps(dict(cfg=cfg, k20_us_per_step=[round(x, 2) for x in ts], k20_rate=round(B / np.median(ts) * 1e6, 1),
                          long_us_per_step=round(tl, 2), long_rate=round(B / tl * 1e6, 1))), flush=True)
    m.close()
