"""Benchmark: BPR triplets/sec on the ml-20m-shaped workload (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W [--batch-size B]

A "step" = one BPR-MF training step over one batch of B triplets per GPU: on-device negative
sampling (amortised: the sampler fills whole chunks of steps), gather + dots + sigmoid + gradient
scatter (fwd_scatter), and the lazy-decay SGD update of every referenced row (apply).
Workload: 138,493 users x 26,744 items (ml-20m shape, data/ml-20m/README.txt:4), ~1e7 synthetic
positives (lognormal degree, Zipf items), d=128, num_ng=4, lr=0.01, wd=0.001 (reference CLI
defaults, BPRMFRecommender.py:53-116).  N>1: one process per GPU (torchrun), users and items
row-sharded, item rows/grads exchanged by RCCL all-to-all every step.

Prints ONE JSON line (rank 0).  roofline: algorithmic bytes of fwd_scatter = B*(24d+12) per launch
(3 rows read + 3 rows of f32 atomic adds + 3 int32 ids) / its live HIP-event average duration.
cpu_baseline: the oracle's C port of the reference step (dense grads + dense weight decay, as
torch does) plus the C port of the sampler, timed on this host on a bounded sample.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

U_ML20M, I_ML20M, NPOS_ML20M = 138493, 26744, 10_000_000
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def bytes_per_triplet(d):
    return 24 * d + 12


def cpu_baseline(pos, U, I, d, B, budget_s=12.0, seed=1):
    """Oracle C port (test infrastructure), bounded sample: dense reference steps + sampler."""
    from oracle import bpr_oracle as O
    from oracle import c_oracle as C
    g = np.random.default_rng(seed)
    P = (0.01 * g.standard_normal((U, d))).astype(np.float32)
    Q = (0.01 * g.standard_normal((I, d))).astype(np.float32)
    indptr, indices = O.build_csr(pos[:, 0], pos[:, 1], U)
    # sampler: one chunk of 2M triplets
    n_s = 2_000_000
    t0 = time.perf_counter()
    u, i, j = C.sample(pos[:, 0], pos[:, 1], indptr, indices, I, 4, seed, 0, 0, n_s)
    t_s = time.perf_counter() - t0
    T = C.DenseTrainer(P, Q, 0.01, 0.001)
    steps = 0
    t0 = time.perf_counter()
    while True:
        s = (steps * B) % (n_s - B)
        T.step(u[s:s + B], i[s:s + B], j[s:s + B])
        steps += 1
        el = time.perf_counter() - t0
        if el > budget_s * 0.8 or steps >= 2000:
            break
    step_rate = steps * B / el
    samp_rate = n_s / t_s
    combined = 1.0 / (1.0 / step_rate + 1.0 / samp_rate)
    return dict(value=combined, unit="triplets/s", cores=C.threads(), kind="port",
                sample=f"{steps} dense reference steps of B={B} (d={d}, full {U}x{I} tables, "
                       f"dense grads + dense weight decay as torch SGD does) = {step_rate:.4g} "
                       f"triplets/s, and {n_s} sampled triplets = {samp_rate:.4g} triplets/s; "
                       f"value = 1/(1/step + 1/sampler)")


def load_traffic(cfg_key):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    e = d.get(cfg_key)
    return None if e is None else e.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--batch-size", type=int, default=4096)
    ap.add_argument("--factor", type=int, default=128)
    ap.add_argument("--users", type=int, default=U_ML20M)
    ap.add_argument("--items", type=int, default=I_ML20M)
    ap.add_argument("--positives", type=int, default=NPOS_ML20M)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="no live per-kernel events")
    ap.add_argument("--seed", type=int, default=20261015)
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("run N>1 under torch.distributed.run (one process per GPU)")
    import torch
    rl = importlib.import_module("recommend-lib_amd")
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    U, I, d, B = a.users, a.items, a.factor, a.batch_size
    pos = syn.make_positives(U, I, a.positives, a.seed)
    if world == 1:
        m = rl.BPRMF(U, I, d, lr=0.01, wd=0.001, batch_size=B, num_ng=4, seed=a.seed, device=local)
        m.set_train(pos)
        n_trip, n_steps = m.epoch_size()

        def run(first, k):
            done = 0
            while done < k:
                e, s = divmod(first + done, n_steps)
                c = min(k - done, n_steps - s)
                m.train_steps(e, s, c)
                done += c
    else:
        sh = importlib.import_module("recommend-lib_amd.sharded")
        m = sh.ShardedBPRMF(U, I, d, lr=0.01, wd=0.001, batch_size=B, num_ng=4, seed=a.seed,
                            device=local, group=None)
        m.set_train(pos)
        n_steps = m.steps_per_epoch

        def run(first, k):
            for s in range(first, first + k):
                e, st = divmod(s, n_steps)
                m.step(e, st)

    run(0, a.warmup)
    torch.cuda.synchronize()
    if not a.no_profile:
        m.profile(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.warmup, a.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    kp = m.profile_read() if not a.no_profile else None
    m.profile(False)
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total = a.steps * B * world
    value = total / el
    out = None
    if rank == 0:
        roof = None
        if kp and kp["fwd_scatter"]["count"]:
            avg_s = kp["fwd_scatter"]["ms"] / kp["fwd_scatter"]["count"] * 1e-3
            ach = B * bytes_per_triplet(d) / avg_s / 1e9
            cfg_key = f"ml20m_d{d}_B{B}"
            roof = dict(bound="hbm", kernel="fwd_scatter", achieved=round(ach, 1), peak=HBM_PEAK_GBS,
                        unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4), traffic=load_traffic(cfg_key),
                        algorithmic_bytes_per_launch=B * bytes_per_triplet(d),
                        avg_launch_us=round(avg_s * 1e6, 3),
                        kernels_us={k: round(v["ms"] / max(v["count"], 1) * 1e3, 3) for k, v in kp.items()})
        cpu = None
        if not a.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(pos, U, I, d, B)
        out = {"metric": "BPR triplets/sec ml-20m d=128 (HR@10 parity vs ref: tests/test_gpu_parity.py)",
               "value": round(value, 1), "unit": "triplets/s", "n_gpus": world, "steps": a.steps,
               "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 5),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic ml-20m-shaped positives (lognormal user degree, Zipf items), "
                       "random N(0,0.01^2) init; no dataset download",
               "config": {"workload": "BPR-MF training, ml-20m shape", "users": U, "items": I,
                          "positives": int(len(pos)), "factor_num": d, "batch_size_per_gpu": B,
                          "global_batch": B * world, "num_ng": 4, "lr": 0.01, "wd": 0.001,
                          "parallelism": f"users+items row-sharded x{world}" if world > 1 else "single GPU",
                          "semantics": "exact batch-synchronous SGD (reference step), lazy weight decay"},
               "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
