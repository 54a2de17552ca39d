"""First timed call after the warm-up: does splitting the W warm-up steps into several calls
change the timed call (exact mode, bench workload)?  argv: warm-up pattern, e.g. 5 or 1,1,1,1,1"""
import importlib, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
pos = syn.make_positives(138493, 26744, 10_000_000, 20261015)
m = rl.BPRMF(138493, 26744, 128, batch_size=4096, seed=20261015)
m.set_train(pos)
pat = [int(x) for x in sys.argv[1].split(",")]
s = 0
for w in pat:
    m.train_steps(0, s, w)
    s += w
out = []
for r in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.train_steps(0, s, 20)
    torch.cuda.synchronize()
    out.append(round((time.perf_counter() - t0) / 20 * 1e6, 2))
    s += 20
print(json.dumps(dict(warm=sys.argv[1], us_per_step=out)))
