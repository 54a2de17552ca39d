"""Debug: does hogwild learn?  ml-100k positives, d=32, B=4096: per-epoch loss for exact and for
hogwild at several grid caps (BPRMF_HOGWILD_BLOCKS) and the serial build."""
import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa
rl = importlib.import_module("recommend-lib_amd")
f = np.load(os.path.join(ROOT, "tests", "golden", "bpr_ml100k_replay.npz"))
pos = f["positives"].astype(np.int64)
U, I = int(f["U"]), int(f["I"])
for name, sem, env in [("exact", "exact", {}), ("hog", "hogwild", {}),
                       ("hog blocks=64", "hogwild", {"BPRMF_HOGWILD_BLOCKS": "64"}),
                       ("hog blocks=8", "hogwild", {"BPRMF_HOGWILD_BLOCKS": "8"}),
                       ("hog serial", "hogwild", {"BPRMF_HOGWILD_SERIAL": "1"})]:
    for k in ("BPRMF_HOGWILD_BLOCKS", "BPRMF_HOGWILD_SERIAL"):
        os.environ.pop(k, None)
    os.environ.update(env)
    m = rl.BPRMF(U, I, 32, batch_size=4096, seed=11, semantics=sem)
    m.set_train(pos)
    ls = []
    for e in range(5 if "serial" in name else 10):
        ls.append(m.train_epoch()["loss"])
    P, Q = m.get_weights()
    print(f"{name:16s} " + " ".join(f"{x:.0f}" for x in ls) + f"  |P| {np.abs(P).mean():.4f} |Q| {np.abs(Q).mean():.4f}", flush=True)
