"""GPU: the library's IPC transport (kernels writing straight into the peers' buffers, flags for
completion) between two PROCESSES sharing the box's one GPU (tests/ipc_worker.py, gloo process
group for the handle exchange).  The sharded result equals the dense oracle on the union batches
and, bit for bit, the in-process loopback transport."""
import os
import socket
import subprocess
import sys
import threading

import numpy as np
import pytest

from conftest import ROOT
from oracle import bpr_oracle as O

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_workers(tmp_path, spec, mode, world=2, timeout=300, extra_env=None):
    """Start `world` worker processes, each logging to its own file; poll them together and stop
    the rest as soon as one fails, so a crash on one rank reports that rank's log instead of a
    peer's timeout (and no pipe can fill while another worker is being waited on)."""
    import time
    spec_path = str(tmp_path / f"spec_{mode}.npz")
    np.savez(spec_path, **spec)
    port = _free_port()
    procs, outs, logs = [], [], []
    for r in range(world):
        out = str(tmp_path / f"out_{mode}_{r}.npz")
        outs.append(out)
        log = str(tmp_path / f"log_{mode}_{r}.txt")
        logs.append(log)
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(world), LOCAL_RANK="0", IPC_SPEC=spec_path, **(extra_env or {}))
        with open(log, "w") as lf:
            procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "ipc_worker.py"),
                                           out, mode], env=env, stdout=lf, stderr=subprocess.STDOUT))

    def tail(r):
        with open(logs[r]) as f:
            return f.read()[-3000:]

    deadline = time.monotonic() + timeout
    failed = None
    try:
        while time.monotonic() < deadline:
            codes = [p.poll() for p in procs]
            bad = [r for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    if failed is not None:
        raise AssertionError(f"worker {failed} exited {procs[failed].returncode}:\n{tail(failed)}")
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"worker {r} did not finish in {timeout} s:\n{tail(r)}"
    return [dict(np.load(o)) for o in outs]


def _loopback(rl, world, spec, mode, key):
    sh = rl.sharded
    grp = sh.ThreadGroup(world)
    out, errs = [None] * world, []
    U, I, D, B = (int(spec[k]) for k in ("U", "I", "D", "B"))

    def run(r):
        try:
            m = sh.ShardedBPRMF(U, I, D, lr=float(spec["lr"]), wd=float(spec["wd"]), batch_size=B,
                                seed=int(spec["seed"]), device=0, comm=sh.ThreadComm(grp, r))
            if mode == "replay":
                m.set_weights(sh.shard_rows(spec["P0"], r, world), sh.shard_rows(spec["Q0"], r, world))
                m.attach_runner("loopback", key=key)
                batches = [(spec["u"][k], spec["i"][k], spec["j"][k]) for k in range(spec["u"].shape[0])]
                m.train_replay(batches)
                m.train_replay(batches)
            else:
                S = m.set_train(spec["pos"])
                m.attach_runner("loopback", key=key)
                m.train_steps(0, 0, S)
                m.train_steps(1, 0, 5)
            out[r] = m.get_weights()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(world)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    if errs:
        raise errs[0]
    return out


@pytest.mark.parametrize("world,fuse", [(1, "auto"), (2, "auto"), (3, "auto"), (4, "auto"),
                                        (2, "1"), (3, "1")])
def test_ipc_replay_equals_dense_oracle_and_loopback(rl, tmp_path, world, fuse):
    """fuse "1": the fused two-launch step (owner phase beside K1, K2 straight into the owners'
    landing buffers; the default with one rank per GPU) forced on although the ranks share the
    box's one GPU; "auto": the shared-device default (every exchange a push kernel plus a receive
    copy into cached buffers)."""
    U, I, D, GB, steps = 301, 157, 128, 512, 6
    g = np.random.default_rng(11)
    u = g.integers(0, U, (steps, GB)).astype(np.int32)
    i = g.integers(0, I, (steps, GB)).astype(np.int32)
    j = g.integers(0, I, (steps, GB)).astype(np.int32)
    i[:, :40] = 7  # a hot item
    spec = dict(U=U, I=I, D=D, B=GB, lr=0.05, wd=0.01, seed=3, u=u, i=i, j=j,
                P0=(0.05 * g.standard_normal((U, D))).astype(np.float32),
                Q0=(0.05 * g.standard_normal((I, D))).astype(np.float32))
    res = _run_workers(tmp_path, spec, "replay", world,
                       extra_env=None if fuse == "auto" else {"BPRMF_DIST_FUSE": fuse})
    sh = rl.sharded
    P = sh.unshard_rows([r["P"] for r in res], U)
    Q = sh.unshard_rows([r["Q"] for r in res], I)
    Pr, Qr = spec["P0"].copy(), spec["Q0"].copy()
    loss = 0.0
    for _ in range(2):
        for k in range(steps):
            loss += O.bpr_step_dense(Pr, Qr, u[k], i[k], j[k], 0.05, 0.01)
    np.testing.assert_allclose(P, Pr, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Q, Qr, rtol=1e-5, atol=1e-6)
    assert sum(int(r["triplets"]) for r in res) == 2 * steps * GB
    got = sum(float(r["loss"]) for r in res)
    assert abs(got - loss) <= 1e-4 * abs(loss)
    lb = _loopback(rl, world, spec, "replay", key=4000 + world)
    for r in range(world):
        assert np.array_equal(res[r]["P"], lb[r][0]) and np.array_equal(res[r]["Q"], lb[r][1])


@pytest.mark.parametrize("world,fuse", [(1, "1"), (2, "1"), (3, "1"), (1, "auto")])
def test_ipc_stale1_device_flags_match_oracle_and_two_stream_form(rl, tmp_path, world, fuse):
    """semantics "stale1" over the IPC transport: the device-flag form (dist.cpp
    enqueue_stale1_ipc: front k = the owners' apply of step k-1 and gather of step k+1 beside
    K1(k), back k = K2(k) pushing its gradients; two landing parities, no cross-stream events),
    forced on the shared GPU (BPRMF_DIST_FUSE=1); "auto": attach_runner("auto") at one rank per
    GPU picks it by itself.  Against the spec
    (oracle/bpr_oracle.py:sharded_stale1_serial; each call is one runner chunk) at the stale1
    tolerance, and bit for bit against the two-stream form over the in-process loopback
    transport."""
    U, I, D, GB, steps = 301, 157, 64, 512, 6
    g = np.random.default_rng(41 + world)
    u = g.integers(0, U, (steps, GB)).astype(np.int32)
    i = g.integers(0, I, (steps, GB)).astype(np.int32)
    j = g.integers(0, I, (steps, GB)).astype(np.int32)
    i[:, :40] = 7  # a hot item, touched by every step
    j[:, 40:45] = i[:, 40:45]  # i == j
    spec = dict(U=U, I=I, D=D, B=GB, lr=0.05, wd=0.01, seed=3, u=u, i=i, j=j,
                P0=(0.05 * g.standard_normal((U, D))).astype(np.float32),
                Q0=(0.05 * g.standard_normal((I, D))).astype(np.float32))
    if fuse == "auto":
        res = _run_workers(tmp_path, spec, "stale1_auto", world)
        assert all(str(r["runner"]) == "ipc" for r in res)
    else:
        res = _run_workers(tmp_path, spec, "stale1", world, extra_env={"BPRMF_DIST_FUSE": fuse})
    sh = rl.sharded
    P = sh.unshard_rows([r["P"] for r in res], U)
    Q = sh.unshard_rows([r["Q"] for r in res], I)
    batches = [(u[k], i[k], j[k]) for k in range(steps)]
    Pr, Qr = spec["P0"].copy(), spec["Q0"].copy()
    losses = np.concatenate([O.sharded_stale1_serial(Pr, Qr, batches, 0.05, 0.01, steps)
                             for _ in range(2)])
    np.testing.assert_allclose(P, Pr, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(Q, Qr, rtol=1e-5, atol=1e-6)
    assert sum(float(r["loss"]) for r in res) == pytest.approx(losses.sum(), rel=1e-5)
    # the two-stream form (rccl / loopback transports) computes the same rows in the same order
    grp = sh.ThreadGroup(world)
    out, errs = [None] * world, []

    def run(r):
        try:
            m = sh.ShardedBPRMF(U, I, D, lr=0.05, wd=0.01, batch_size=GB, seed=3, device=0,
                                comm=sh.ThreadComm(grp, r), semantics="stale1")
            m.set_weights(sh.shard_rows(spec["P0"], r, world), sh.shard_rows(spec["Q0"], r, world))
            m.attach_runner("loopback", key=8900 + world)
            m.train_replay(batches)
            m.train_replay(batches)
            out[r] = m.get_weights()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(world)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    if errs:
        raise errs[0]
    for r in range(world):
        assert np.array_equal(res[r]["P"], out[r][0]) and np.array_equal(res[r]["Q"], out[r][1])


def test_ipc_sampler_training_equals_loopback(rl, golden, tmp_path):
    f = golden("bpr_ml100k_replay.npz")
    pos = f["positives"].astype(np.int64)
    spec = dict(U=int(f["U"]), I=int(f["I"]), D=64, B=1024, lr=0.01, wd=0.001, seed=9, pos=pos)
    res = _run_workers(tmp_path, spec, "sampler")
    lb = _loopback(rl, 2, spec, "sampler", key=4010)
    for r in range(2):
        assert np.array_equal(res[r]["P"], lb[r][0]) and np.array_equal(res[r]["Q"], lb[r][1])


@pytest.mark.parametrize("world,overlap", [(2, False), (3, True)])
def test_ipc_local_semantics_all_reduce_equals_loopback(rl, tmp_path, monkeypatch, world, overlap):
    """semantics "local" across processes: the IPC transport's all-reduce
    (reduce-scatter + all-gather pushes over the full mesh) against the in-process loopback
    transport's rank-order sum, the SERIAL build on both sides: bit for bit, and every rank ends
    with the same item table."""
    U, I, D, B, steps = 61, 47, 32, 64, 7
    g = np.random.default_rng(23 + world)
    rows = [(uu, it) for uu in range(U) for it in range(I) if g.random() < 0.2 / (1 + it % 5)]
    pos = np.unique(np.array(rows, np.int64), axis=0).astype(np.int32)
    us, is_, js = [], [], []
    for k in range(steps):  # each rank's share of a step: exactly B triplets
        parts = [g.choice(np.arange(r, U, world), B) for r in range(world)]
        us.append(np.concatenate(parts))
        is_.append(g.integers(0, I, world * B))
        js.append(g.integers(0, I, world * B))
    spec = dict(U=U, I=I, D=D, B=B, lr=0.05, wd=0.01, seed=5, pos=pos, period=2, dp=3,
                overlap=int(overlap), u=np.array(us, np.int32), i=np.array(is_, np.int32),
                j=np.array(js, np.int32),
                P0=(0.1 * g.standard_normal((U, D))).astype(np.float32),
                Q0=(0.1 * g.standard_normal((I, D))).astype(np.float32))
    env = {"BPRMF_HOGWILD_SERIAL": "1", "BPRMF_LOCAL_HOT": "4"}
    res = _run_workers(tmp_path, spec, "local", world, extra_env=env)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sh = rl.sharded
    grp = sh.ThreadGroup(world)
    out, errs = [None] * world, []

    def run(r):
        try:
            m = sh.ShardedBPRMF(U, I, D, lr=0.05, wd=0.01, batch_size=B, seed=5, device=0,
                                comm=sh.ThreadComm(grp, r), semantics="local", local_steps=2,
                                dp_steps=3, dp_overlap=overlap)
            m.set_train(pos)
            m.set_weights(sh.shard_rows(spec["P0"], r, world), spec["Q0"])
            m.attach_runner("loopback", key=8800 + world)
            batches = [(spec["u"][k], spec["i"][k], spec["j"][k]) for k in range(steps)]
            m.train_replay(batches)
            m.train_replay(batches)
            out[r] = m.get_weights()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            grp.barrier.abort()

    ts = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(world)]
    [t.start() for t in ts]
    [t.join(timeout=300) for t in ts]
    if errs:
        raise errs[0]
    for r in range(world):
        assert np.array_equal(res[r]["Q"], res[0]["Q"])
        assert np.array_equal(res[r]["P"], out[r][0]), r
        assert np.array_equal(res[r]["Q"], out[r][1]), r
