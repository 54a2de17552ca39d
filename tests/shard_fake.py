"""Test double of sharded.HipShard on CPU torch tensors (TEST INFRASTRUCTURE ONLY).

It implements the same step phases as the C ABI's bprmf_dist_* with the reference's dense
semantics (every local row decays every step, BPRMFRecommender.py:154,176), so the orchestrator's
exchange logic (ShardedBPRMF + TorchComm over gloo) can be tested on CPU with world_size > 1.
Only replay plans are supported (no sampler here).
"""
import numpy as np
import torch


class FakeShard:
    def __init__(self, user_num, item_num, d, lr, wd, batch_size, rank, world, P_local, Q_local):
        self.U, self.I, self.d = user_num, item_num, d
        self.lr, self.wd = np.float32(lr), np.float32(wd)
        self.batch_size, self.rank, self.world = batch_size, rank, world
        self.ld = d
        self.device = torch.device("cpu")
        self.P = np.array(P_local, dtype=np.float32)
        self.Q = np.array(Q_local, dtype=np.float32)
        self.iloc = (item_num + world - 1) // world
        self.steps = []
        self.cur = None

    def set_train(self, pos):
        pos = np.asarray(pos)
        n = int(((pos[:, 0] % self.world) == self.rank).sum()) * 4
        return (n + self.batch_size - 1) // self.batch_size

    def plan(self, epoch, first_step, n_steps):
        raise NotImplementedError("FakeShard supports replay plans only")

    def plan_replay(self, U, I, J, n_steps):
        B, W = self.batch_size, self.world
        counts = np.zeros((n_steps, W), dtype=np.int32)
        self.steps = []
        for k in range(n_steps):
            u, i, j = U[k * B:(k + 1) * B], I[k * B:(k + 1) * B], J[k * B:(k + 1) * B]
            keep = u >= 0
            u, i, j = u[keep].astype(np.int64), i[keep].astype(np.int64), j[keep].astype(np.int64)
            keys = np.unique(np.concatenate([(i % W) * self.iloc + i // W, (j % W) * self.iloc + j // W]))
            slot = {int(kk): s for s, kk in enumerate(keys)}
            si = np.array([slot[int((x % W) * self.iloc + x // W)] for x in i], dtype=np.int64)
            sj = np.array([slot[int((x % W) * self.iloc + x // W)] for x in j], dtype=np.int64)
            owners = keys // self.iloc
            counts[k] = np.bincount(owners, minlength=W)
            self.steps.append(dict(ul=u // W, si=si, sj=sj, ukey=(keys % self.iloc).astype(np.int32)))
        return counts

    def request_ids(self, k, ids, n):
        ids[:n] = torch.from_numpy(self.steps[k]["ukey"][:n])

    def gather_items(self, rows, n, out):
        out[:n] = torch.from_numpy(self.Q[rows[:n].numpy()])

    def user_step(self, k, item_rows):
        st = self.steps[k]
        rows = item_rows.numpy()
        pu = self.P[st["ul"]]
        qi, qj = rows[st["si"]], rows[st["sj"]]
        x = (pu * qi).sum(1) - (pu * qj).sum(1)
        c = (1.0 / (1.0 + np.exp(x))).astype(np.float32)
        gP = np.zeros_like(self.P)
        np.add.at(gP, st["ul"], -c[:, None] * (qi - qj))
        st["contrib"] = c[:, None] * pu
        self.P -= self.lr * (gP + self.wd * self.P)

    def item_grads(self, k, grads):
        st = self.steps[k]
        n = len(st["ukey"])
        g = np.zeros((n, self.d), dtype=np.float32)
        np.add.at(g, st["si"], -st["contrib"])
        np.add.at(g, st["sj"], st["contrib"])
        grads[:n] = torch.from_numpy(g)

    def apply_items(self, rows, grads, n):
        gQ = np.zeros_like(self.Q)
        np.add.at(gQ, rows[:n].numpy(), grads[:n].numpy())
        self.Q -= self.lr * (gQ + self.wd * self.Q)

    def end_step(self, want_loss=False):
        return None

    def get_weights(self):
        return self.P.copy(), self.Q.copy()
