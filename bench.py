"""Benchmark: BPR triplets/sec on the ml-20m-shaped workload (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W [--batch-size B]

A "step" = one BPR-MF training step over one batch of B triplets per GPU: on-device negative
sampling + batch build (amortised: one build launch per chunk of steps, inside the timed region),
then user_step (gathers, dots, sigmoid, user update, c*P_u per triplet) and item_step (per-item
fixed-order gradient sum, item update).  N>1: one process per GPU (torch.distributed.run), users
and items row-sharded; every step the owners' item rows go to the requesting ranks and their
gradients come back, both exchanges issued by the library (IPC peer writes over xGMI, or RCCL).
Workload: 138,493 users x 26,744 items (ml-20m shape, data/ml-20m/README.txt:4), ~1e7 synthetic
positives (lognormal degree, Zipf items), d=128, num_ng=4, lr=0.01, wd=0.001, B=4096 (the
reference CLI defaults, BPRMFRecommender.py:53-116).

Prints ONE JSON line (rank 0).
roofline: algorithmic bytes per step = B*(24d+12) (3 rows read + 3 rows written + 3 int32 ids per
  triplet) over the live HIP-event time of the step's two kernels (user_step +
  item_step, which together do that gather/scatter), peak 8 TB/s HBM3E.  The event pass runs right
  after the timed region over the same number of steps (per-launch events perturb the timing, so
  they are kept out of the timed region); rocprofv3 summaries of the same command: profiles/.
cpu_baseline: the oracle's C port of the reference step (dense grads + dense weight decay, as torch
  does) and of the sampler, timed on this host on a bounded sample; the reference's own torch-CPU
  step (measured in the build container) is quoted beside it.
--semantics hogwild: the opt-in relaxed mode (csrc/hogwild.hip; not the reference step) on the
  same workload, labelled as such in config.semantics; the default line is the exact step.
--semantics local: hot items in per-XCD replicas; at N > 1 also the item table
  replicated on every rank and merged by an RCCL all-reduce every --dp-steps steps (§5d).  Opt-in,
  labelled; never the headline.
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
# what `achieved` / `frac` divide by: this run's own HIP events around the step launches (a
# process cannot read its own rocprofv3 summary; the same kernel's rocprofv3 averages, which run
# ~3 % longer than the events, are in profiles/ and DESIGN.md §5)
FRAC_BASIS = ("events: live HIP-event time per step of this run (rocprofv3 kernel averages of the "
              "same command: profiles/, DESIGN.md §5)")


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
    return dict(value=round(combined, 1), unit="triplets/s", cores=C.threads(), kind="port",
                sample=f"{steps} dense reference steps of B={B} (d={d}, full {U}x{I} tables, "
                       f"dense grads + dense weight decay as torch SGD does) = {step_rate:.4g} "
                       f"triplets/s, and {n_s} sampled triplets = {samp_rate:.4g} triplets/s; "
                       f"value = 1/(1/step + 1/sampler)")


# the reference's own torch-CPU BPR step at the ml-20m shape, d=128, B=4096 (SURVEY.md
# §6): measured in the build container, not on the GPU box (the reference does not travel there)
REFERENCE_CPU_QUOTED = {"value": 179000.0, "unit": "triplets/s", "threads": 8,
                        "source": "BASELINE.md: reference torch-CPU step (BPRMFRecommender.py:172-176), "
                                  "ml-20m shape d=128 B=4096, 8-core build container, not this host"}


def load_traffic(cfg_key):
    """Bytes per step from rocprofv3 PMC counters (profiles/pmc_traffic.json): a STATIC number from
    an earlier profiled run, labelled as such in the line (traffic_source)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        e = json.load(f).get(cfg_key)
    if e is None:
        return None, None
    src = ("profiles/pmc_traffic.json (static, from an earlier rocprofv3 --pmc run of this kernel; "
           "L2<->fabric bytes, Infinity-Cache hits included)")
    return e.get("hbm_bytes_per_step"), src


def relaxed_local(rl, pos, U, I, d, B, seed, local_steps, steps, warmup, traffic_key=None):
    """The opt-in relaxed mode (semantics="local") on the same workload, as a
    labelled sub-object of the exact line: its own model, warm-up and timed
    region (whole merge periods: `steps` >= 1024), live HIP-event roofline, its own PMC key.  NOT
    the reference step, never the headline `value`."""
    import torch
    m = rl.BPRMF(U, I, d, lr=0.01, wd=0.001, batch_size=B, num_ng=4, seed=seed, device=0,
                 semantics="local", local_steps=local_steps)
    m.set_train(pos)
    n_steps = m.epoch_size()[1]

    def run(first, k):
        done = 0
        while done < k:
            e, s = divmod(first + done, n_steps)
            c = min(k - done, n_steps - s)
            m.train_steps(e, s, c)
            done += c

    run(0, warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(warmup, steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    m.profile(True)
    run(warmup + steps, steps)
    torch.cuda.synchronize()
    kp = m.profile_read()
    m.profile(False)
    roof = None
    if kp and kp["step_graph"]["count"]:
        step_us = kp["step_graph"]["ms"] / kp["step_graph"]["count"] * 1e3
        ach = B * bytes_per_triplet(d) / (step_us * 1e-6) / 1e9
        if traffic_key is None and (U, I) == (U_ML20M, I_ML20M):
            traffic_key = f"ml20m_d{d}_B{B}_local"
        traffic, tsrc = load_traffic(traffic_key) if traffic_key else (None, None)
        roof = dict(bound="hbm", kernel=("k_hogwild<LOCAL> (in-kernel sampling + gather + dots + "
                                         "sigmoid + SGD scatter, hot items in per-XCD replicas) + "
                                         "k_local_merge every period"),
                    achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(ach / HBM_PEAK_GBS, 4), frac_basis=FRAC_BASIS,
                    traffic=traffic, traffic_source=tsrc,
                    algorithmic_bytes_per_step=B * bytes_per_triplet(d),
                    avg_us_per_step=round(step_us, 3))
    del m
    return {"semantics": ("relaxed (local: hogwild for users and cold items, the hot items in one "
                          "replica per XCD merged every local_steps steps; NOT the reference step; "
                          "opt-in, never the headline)"),
            "value": round(steps * B / el, 1), "unit": "triplets/s", "steps": steps,
            "warmup": warmup, "ms_per_step": round(el / steps * 1e3, 5), "local_steps": local_steps,
            "timed_region": "one train_steps call per epoch segment, synchronised on both sides",
            "roofline": roof,
            "quality": "HR@10 / NDCG@10 against the exact step: DESIGN.md §5c, tools/hr_modes.py"}


# the HBM-resident shape of the relaxed_local_hbm sub-object: tables of
# (U + I) * d * 4 B = 1.54 GB at d = 128, 6x the 256 MiB Infinity Cache (MALL), so the rows come
# from HBM rather than from the on-die cache that holds the ml-20m shape's 85 MB of tables
U_HBM, I_HBM, NPOS_HBM = 2_000_000, 1_000_000, 20_000_000


def relaxed_local_hbm(rl, syn, d, B, seed, local_steps, steps, warmup):
    """relaxed_local at an HBM-resident shape: its own positives (synthetic.make_positives of
    (U_HBM, I_HBM, NPOS_HBM)), model, warm-up, timed region and event roofline.  NOT the
    reference step, never the headline."""
    t0 = time.perf_counter()
    pos = syn.make_positives(U_HBM, I_HBM, NPOS_HBM, seed + 1)
    r = relaxed_local(rl, pos, U_HBM, I_HBM, d, B, seed, local_steps, steps, warmup,
                      traffic_key=f"hbm2m1m_d{d}_B{B}_local")
    r["config"] = {"users": U_HBM, "items": I_HBM, "positives": int(len(pos)), "factor_num": d,
                   "batch_size": B, "table_bytes": (U_HBM + I_HBM) * d * 4,
                   "mall_bytes": 256 << 20,
                   "why": "tables 6x the 256 MiB Infinity Cache: rows served from HBM"}
    r["wall_s"] = round(time.perf_counter() - t0, 1)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--warmup", type=int, default=400)
    ap.add_argument("--batch-size", type=int, default=4096)
    ap.add_argument("--factor", type=int, default=128)
    ap.add_argument("--users", type=int, default=U_ML20M)
    ap.add_argument("--items", type=int, default=I_ML20M)
    ap.add_argument("--positives", type=int, default=NPOS_ML20M)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the live per-kernel event pass")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--chunk", type=int, default=0,
                    help="steps per library call (0: up to the end of the epoch)")
    ap.add_argument("--sharded", action="store_true",
                    help="use the sharded RCCL path even at one rank (exercises it on one GPU)")
    ap.add_argument("--transport", default="auto", choices=["auto", "ipc", "rccl"],
                    help="sharded runner exchange: IPC peer writes (auto: unless a rank cannot map "
                         "its peers) or RCCL send/recv")
    ap.add_argument("--python-orchestration", action="store_true",
                    help="sharded: per-step Python orchestration over torch.distributed instead of "
                         "the library's runner")
    ap.add_argument("--semantics", default="exact", choices=["exact", "hogwild", "local", "stale1"],
                    help="exact: the reference's batch-synchronous step (default, the headline); "
                         "hogwild: opt-in relaxed synchronisation (a separate, labelled line)")
    ap.add_argument("--local-steps", type=int, default=0,
                    help="--semantics local: steps between the XCD replicas' merges (0: 128)")
    ap.add_argument("--dp-steps", type=int, default=0,
                    help="--semantics local, N > 1: steps between the ranks' item-table merges (0: 256)")
    ap.add_argument("--dp-overlap", action="store_true",
                    help="--semantics local, N > 1: each merge's all-reduce beside the next period")
    ap.add_argument("--step", default="segmented", choices=["segmented", "atomic"],
                    help="exact step's duplicate-row sums: segmented (sorted, one writer per row, "
                         "bitwise reproducible; the headline) or atomic (f32 atomics; a labelled line)")
    ap.add_argument("--no-relaxed", action="store_true",
                    help="N=1 exact line: skip its relaxed_local sub-object")
    ap.add_argument("--relaxed-steps", type=int, default=2048,
                    help="timed steps of the relaxed_local sub-object (whole 128-step periods)")
    ap.add_argument("--pg-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group backend (gloo: rehearse several ranks on one GPU, IPC "
                         "transport; RCCL refuses two ranks on one device)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and a.gpus > 1:
        raise SystemExit("run N>1 under torch.distributed.run (one process per GPU)")
    import torch
    rl = importlib.import_module("recommend-lib_amd")
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    local = local % max(1, torch.cuda.device_count())  # ranks beyond the GPUs: rehearsal only
    torch.cuda.set_device(local)
    dist = None
    sharded = world > 1 or a.sharded or a.semantics == "stale1"  # stale1: the sharded runner only
    hog = a.semantics in ("hogwild", "local")
    if a.semantics == "hogwild" and sharded:
        raise SystemExit("--semantics hogwild is single-GPU (run N independent replicas instead)")
    # users sharded, item table replicated and merged (§5d): only with peers to merge with (a
    # one-rank --sharded handle runs the single-GPU local path unless BPRMF_DP_ONE_RANK is set)
    dpi = a.semantics == "local" and sharded and (world > 1 or os.environ.get("BPRMF_DP_ONE_RANK") == "1")
    if a.semantics in ("local", "stale1") and a.python_orchestration:
        raise SystemExit("--semantics local runs through the library runner only (per-step Python "
                         "orchestration addresses items by owner)")
    if a.step == "atomic" and (sharded or hog):
        raise SystemExit("--step atomic is the single-GPU exact step's alternative")
    if sharded:
        import torch.distributed as dist
        if "RANK" not in os.environ:  # --sharded without a launcher: a one-rank group
            os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=os.environ.get("MASTER_PORT", "29529"))
        if a.pg_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    U, I, d, B = a.users, a.items, a.factor, a.batch_size
    pos = syn.make_positives(U, I, a.positives, a.seed)
    if not sharded:
        m = rl.BPRMF(U, I, d, lr=0.01, wd=0.001, batch_size=B, num_ng=4, seed=a.seed, device=local,
                     semantics=a.semantics, step=a.step, local_steps=a.local_steps)
        m.set_train(pos)
        n_steps = m.epoch_size()[1]

        def run(first, k):
            done = 0
            while done < k:
                e, s = divmod(first + done, n_steps)
                c = min(k - done, n_steps - s)
                m.train_steps(e, s, c)
                done += c
    else:
        m = rl.ShardedBPRMF(U, I, d, lr=0.01, wd=0.001, batch_size=B, num_ng=4, seed=a.seed,
                            device=local, semantics=a.semantics, local_steps=a.local_steps,
                            dp_steps=a.dp_steps, dp_overlap=a.dp_overlap)
        n_steps = m.set_train(pos)
        if a.python_orchestration:
            def run(first, k):
                for s in range(first, first + k):
                    e, st = divmod(s, n_steps)
                    m.step(e, st)
        else:  # the library's runner: chunks of steps, exchanges issued from C++
            m.attach_runner(a.transport)

            def run(first, k):
                done = 0
                while done < k:
                    e, s = divmod(first + done, n_steps)
                    c = min(k - done, n_steps - s)
                    m.train_steps(e, s, c)
                    done += c

    # the timing barriers: the ranks of one node meet on shared memory (bprmf_node_barrier_*,
    # ~1 us); a process group's barrier (gloo sockets, or the nccl group's device all-reduce plus a
    # synchronisation) costs ~0.1 ms that would land inside the timed region.  Ranks on several
    # nodes: a gloo group's barrier.
    bar = dist.new_group(backend="gloo") if dist and a.pg_backend == "nccl" else None
    nb, nb_path = None, None
    if dist and world > 1 and int(os.environ.get("LOCAL_WORLD_SIZE", "0")) == world:
        tok = [f"/dev/shm/bprmf_bench_{os.getpid()}_{time.time_ns()}" if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0, group=bar)
        nb_path = tok[0]
        if rank == 0:
            nb = rl.sharded.NodeBarrier(nb_path, world, rank, create=True)
        dist.barrier(group=bar)
        if rank != 0:
            nb = rl.sharded.NodeBarrier(nb_path, world, rank, create=False)
        dist.barrier(group=bar)

    def barrier():
        if nb is not None:
            nb.wait()
        elif dist and world > 1:  # (one rank: nothing to wait for)
            dist.barrier(group=bar)

    def timed(first, k):
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(first, k)
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], dtype=torch.float64,
                             device="cuda" if a.pg_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    run(0, a.warmup)
    xs0 = m.exchange_stats() if sharded and not a.python_orchestration else None
    el = timed(a.warmup, a.steps)
    xs1 = m.exchange_stats() if xs0 is not None else None
    kp = None
    if not a.no_profile:  # live per-kernel HIP events over the same number of steps
        m.profile(True)
        timed(a.warmup + a.steps, a.steps)
        kp = m.profile_read()
        m.profile(False)
    value = a.steps * B * world / el
    out = None
    if rank == 0:
        roof = None
        if kp and (kp["step_graph"]["count"] or kp["user_step"]["count"]):
            us = {k: v["ms"] / v["count"] * 1e3 for k, v in kp.items() if v["count"]}
            if ("step_graph" in us and sharded and world == 1 and not a.python_orchestration
                    and a.semantics == "exact"):
                # one rank: the runner dispatches to the single-GPU fused step (nothing to exchange)
                step_us, what = us["step_graph"], ("world 1: the single-GPU fused step launches (the "
                                                   "runner has no peer to exchange with)")
            elif "step_graph" in us and dpi:  # one pair per call: periods + merges (per rank)
                step_us, what = us["step_graph"], ("per rank: k_hogwild<LOCAL> on the rank's users + "
                                                   "k_local_merge every local_steps + the item-table "
                                                   "merge (k_dp_delta, all-reduce, k_dp_apply) every "
                                                   "dp_steps")
            elif "step_graph" in us and a.semantics == "local":  # periods: k_hogwild + k_local_merge
                step_us, what = us["step_graph"], ("k_hogwild<LOCAL> (in-kernel sampling + gather + dots "
                                                   "+ sigmoid + SGD scatter, hot items in per-XCD replicas) "
                                                   "+ k_local_merge every period")
            elif "step_graph" in us and a.semantics == "stale1":
                step_us, what = us["step_graph"], ("stale1 sharded step, per rank: K1 beside the owners' "
                                                   "apply of the step before and gather of the step after "
                                                   "(ipc: one launch, device flags) or beside the owner "
                                                   "stream's exchanges (rccl: two streams), then K2")
            elif "step_graph" in us and sharded:  # events around each chunk's steps (per rank)
                step_us, what = us["step_graph"], ("sharded step, per rank: owner gather + row exchange + "
                                                   "user_step + item_step + grad exchange + owner apply")
            elif "step_graph" in us and hog:  # one k_hogwild launch per chunk
                step_us, what = us["step_graph"], ("k_hogwild (in-kernel sampling + gather + dots + "
                                                   "sigmoid + SGD scatter, one launch per chunk)")
            elif "step_graph" in us:  # events around each chunk's step launches (GPU-bound)
                step_us, what = us["step_graph"], ("fused step launches (K2 of step t + K1 of step "
                                                   "t+1 per launch; a chunk is K1, n-1 fused, K2)")
            elif a.step == "atomic" and "user_step" in us:  # fwd_scatter + apply_refs per step
                step_us, what = us["user_step"] + us["item_step"], ("atomic step: k_fwd_scatter (gathers, "
                                                                    "dots, f32-atomic gradient scatter) + "
                                                                    "k_apply_refs (decay + SGD per touched row)")
            else:  # eager (sharded): events around the two kernels of sampled steps
                step_us, what = us["user_step"] + us["item_step"], "user_step + item_step"
            ach = B * bytes_per_triplet(d) / (step_us * 1e-6) / 1e9
            # PMC bytes only for the kernel they were counted on: the single-GPU fused step (or
            # the hogwild kernel); a sharded line (world > 1) gets them only from an entry measured
            # on the sharded kernels themselves, keyed by world size
            tkey = (f"ml20m_d{d}_B{B}" + (f"_{a.semantics}" if hog else "")
                    + ("_atomic" if a.step == "atomic" else ""))
            if sharded and not (world == 1 and not a.python_orchestration):
                tkey = f"sharded_w{world}_ml20m_d{d}_B{B}"
            traffic, tsrc = load_traffic(tkey) if (U, I) == (U_ML20M, I_ML20M) else (None, None)
            if traffic is None and sharded:
                tsrc = ("none: no rocprofv3 --pmc pass has counted the sharded kernels at this world "
                        "size (a single-GPU figure would describe other kernels)")
            roof = dict(bound="hbm", kernel=what, achieved=round(ach, 1), peak=HBM_PEAK_GBS,
                        unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4), frac_basis=FRAC_BASIS,
                        traffic=traffic, traffic_source=tsrc,
                        algorithmic_bytes_per_launch=B * bytes_per_triplet(d),
                        avg_us_per_step=round(step_us, 3),
                        avg_launch_us={k: round(v, 3) for k, v in us.items()})
            if sharded:
                # per rank: `achieved` counts this rank's algorithmic bytes (its B triplets' rows
                # and ids) over its own step time; the exchange bytes below are separate (xGMI
                # link traffic, not HBM reads of this rank's step)
                roof["bytes_counted"] = ("per rank: B*(24d+12) algorithmic bytes of the rank's own "
                                         "batch per step; exchange bytes reported separately")
        xch = None
        if xs0 is not None and xs1 is not None:
            ns = max(1, xs1["steps"] - xs0["steps"])
            xch = {k: (xs1[k] - xs0[k]) // ns for k in ("row_bytes", "grad_bytes", "id_bytes")}
            xch = {"per_rank_per_step": xch, "peer_links": world - 1, "steps": xs1["steps"] - xs0["steps"],
                   "note": ("bytes this rank sent to its peers per step as the transport moved them "
                            "(padded to the chunk's exchange capacity; world 1 sends nothing)"
                            if not dpi else
                            "grad_bytes: the item-table merges' all-reduce, 2(W-1)/W of the table per "
                            "merge per rank (a ring's volume), averaged per step")}
        rlx = rlx_hbm = None
        if (world == 1 and not sharded and a.semantics == "exact" and a.step == "segmented"
                and not a.no_relaxed):
            del m  # the exact model's tables and buffers are not needed any more
            rlx = relaxed_local(rl, pos, U, I, d, B, a.seed, a.local_steps or 128,
                                max(1024, a.relaxed_steps), 256)
            rlx_hbm = relaxed_local_hbm(rl, syn, d, B, a.seed, a.local_steps or 128,
                                        max(1024, a.relaxed_steps), 256)
        cpu = None
        if not a.no_cpu_baseline and world == 1 and not sharded:
            cpu = cpu_baseline(pos, U, I, d, B)
            cpu["reference_cpu_quoted"] = REFERENCE_CPU_QUOTED
        out = {"metric": "BPR triplets/sec ml-20m d=128 (HR@10 parity vs ref: tests/test_gpu_parity.py)",
               "value": round(value, 1), "unit": "triplets/s", "n_gpus": world, "steps": a.steps,
               "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 5),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic ml-20m-shaped positives (lognormal user degree, Zipf items), "
                       "random N(0,0.01^2) init; no dataset download",
               "config": {"workload": "BPR-MF training, ml-20m shape", "users": U, "items": I,
                          **({"local_steps": a.local_steps or 128} if a.semantics == "local" else {}),
                          **({"dp_steps": a.dp_steps or 256, "dp_overlap": a.dp_overlap} if dpi else {}),
                          "positives": int(len(pos)), "factor_num": d, "batch_size_per_gpu": B,
                          "global_batch": B * world, "num_ng": 4, "lr": 0.01, "wd": 0.001,
                          "parallelism": (f"users row-sharded x{world}, item table replicated, merged "
                                          f"every dp_steps by {m.runner} all-reduce" if dpi else
                                          f"users+items row-sharded x{world}, "
                                          f"{'python/torch.distributed' if a.python_orchestration else m.runner} exchange"
                                          if sharded else "single GPU"),
                          "semantics": ("relaxed (hogwild: per-triplet lock-free updates, weight decay "
                                        "once per row per step, staleness bounded by the launch's "
                                        "in-flight window; NOT the reference step)" if a.semantics == "hogwild" else
                                        "relaxed (local: hogwild for users and cold items, the hot items "
                                        "in one replica per XCD merged every local_steps steps; NOT the "
                                        "reference step)" if a.semantics == "local" else
                                        "relaxed (stale1: the exact sharded step with the item rows one "
                                        "step stale, the exchange of step k beside the compute of step "
                                        "k+1; NOT the reference step)" if a.semantics == "stale1" else
                                        "exact batch-synchronous SGD (reference step), lazy weight decay, "
                                        "duplicate rows summed by f32 atomics (not bitwise reproducible)"
                                        if a.step == "atomic" else
                                        "exact batch-synchronous SGD (reference step), lazy weight decay")},
               "roofline": roof, "cpu_baseline": cpu}
        if rlx is not None:
            out["relaxed_local"] = rlx
        if rlx_hbm is not None:
            out["relaxed_local_hbm"] = rlx_hbm
        if sharded:
            out["exchange"] = xch
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        if nb is not None:
            nb.close()
            if rank == 0:
                try:
                    os.unlink(nb_path)
                except OSError:
                    pass
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
