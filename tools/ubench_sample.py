"""Time the grid-wide sampler (k_sample) on the driver's short chunk: 20 batches x 4096 triplets,
ml-20m shape.  Run once per library variant (BPRMF_DIAG_LIB selects a diagnostic build).

  python tools/ubench_sample.py [lib.so ...]     # GPU box; no argument = the product library
Prints one JSON line per library: median us per 81,920-slot chunk over 200 chunks.
"""
import ctypes
import importlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if len(sys.argv) > 1 and sys.argv[1] != "--child":
    for lib in sys.argv[1:]:  # one child process per library (each loads its own .so)
        env = dict(os.environ, BPRMF_DIAG_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

rl = importlib.import_module("recommend-lib_amd")
syn = importlib.import_module("recommend-lib_amd.synthetic")
pos = syn.make_positives(138493, 26744, 10_000_000, 20261015)
m = rl.BPRMF(138493, 26744, 128, batch_size=4096, seed=1, device=0)
m.set_train(pos)
n = 20 * 4096
N = m.epoch_size()[0]
buf = torch.empty(3, n, dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
m.set_stream(s.cuda_stream)
L = m._L
times = []
with torch.cuda.stream(s):
    for rep in range(220):
        first = (rep * n) % (N - n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        rc = L.bprmf_dist_sample_dev(m._h, 0, first, n, ctypes.c_void_p(buf[0].data_ptr()),
                                     ctypes.c_void_p(buf[1].data_ptr()), ctypes.c_void_p(buf[2].data_ptr()))
        e1.record(s)
        assert rc == 0
        s.synchronize()
        if rep >= 20:
            times.append(e0.elapsed_time(e1) * 1e3)
m.set_stream(None)
print(json.dumps({"lib": os.path.basename(os.environ.get("BPRMF_DIAG_LIB", "libbprmf_amd.so")),
                  "us_per_chunk_median": round(float(np.median(times)), 2),
                  "us_min": round(float(np.min(times)), 2)}), flush=True)
m.close()
