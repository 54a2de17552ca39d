"""ORACLE — CPU restatement of the reference BPR-MF training path, for TESTS ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker.  The product path (recommend-lib_amd) never calls it.

Two parts:

1. The reference training step, restated densely and literally (numpy float32):
   BPRMFRecommender.py:42-50  forward   pred_i = <P_u,Q_i>, pred_j = <P_u,Q_j>
   BPRMFRecommender.py:174    loss      L = -sum(log(sigmoid(pred_i - pred_j)))   (a SUM)
   BPRMFRecommender.py:175    backward  dense embedding grads, duplicates summed
   BPRMFRecommender.py:154,176 SGD      W <- W - lr*(G + wd*W) over EVERY row (weight decay is dense)
   Pinned against tests/golden/bpr_step_tiny.npz (F1) and bpr_ml100k_replay.npz (F2), which were
   produced by the reference itself (tests/golden/make_golden.py).

2. The on-device sampler's specification (util/data_loader.py:680-700 semantics, our RNG):
   the reference draws `num_ng` negatives per positive with MT19937 + rejection against the train
   set (data_loader.py:684-689) and the DataLoader shuffles the triplets
   (BPRMFRecommender.py:141-142).  A data-dependent MT19937 stream cannot be parallelised, so the
   product uses a counter-based equivalent with the SAME distribution:
     * triplet q = p*num_ng + r  <->  positive p = features[p], r-th negative   (data_loader.py:684-690)
     * negative j = k-th item NOT in the user's train set, k ~ U[0, I - deg(u)) (exactly uniform over
       non-positives, like rejection sampling, but one draw and one binary search)
     * the epoch's triplet order is a keyed Feistel permutation of [0, N) (cycle-walking), standing in
       for the DataLoader's torch.randperm shuffle
     * randomness: Philox4x32-10 (Salmon et al., SC'11), key = 64-bit seed, counter = (q, epoch, tag)
   This module restates that spec independently of the HIP code; GPU output must match it bit-for-bit.
   Distributional parity with the reference sampler is pinned by tests/golden/ng_sample_ml100k.npz (F3).
"""
import math

import numpy as np

# ----------------------------------------------------------------------------------------------
# 1. dense reference step
# ----------------------------------------------------------------------------------------------


def bpr_step_dense(P, Q, u, i, j, lr, wd):
    """In-place reference step on float32 tables P [U,d], Q [I,d]; returns the loss (float64).

    Follows BPRMFRecommender.py:172-176 with torch's single-tensor SGD (torch/optim/sgd.py):
    d_p = grad + wd*p ; p = p - lr*d_p, applied to every row because nn.Embedding grads are dense.
    """
    f32 = np.float32
    lr = f32(lr)
    wd = f32(wd)
    u = np.asarray(u, dtype=np.int64)
    i = np.asarray(i, dtype=np.int64)
    j = np.asarray(j, dtype=np.int64)
    pu, qi, qj = P[u], Q[i], Q[j]
    x = (pu * qi).sum(-1, dtype=f32) - (pu * qj).sum(-1, dtype=f32)
    s = (f32(1) / (f32(1) + np.exp(-x, dtype=f32))).astype(f32)
    with np.errstate(divide="ignore"):
        loss = float(-np.log(s.astype(np.float64)).sum())
    c = (f32(1) - s).astype(f32)  # -dL/dx
    gP = np.zeros_like(P)
    gQ = np.zeros_like(Q)
    np.add.at(gP, u, (-c)[:, None] * qi + c[:, None] * qj)
    np.add.at(gQ, i, (-c)[:, None] * pu)
    np.add.at(gQ, j, c[:, None] * pu)
    for W, G in ((P, gP), (Q, gQ)):
        dp = G + wd * W
        W -= lr * dp
    return loss


def train_replay(P, Q, triplets, bounds, lr, wd):
    """Replay a sequence of reference batches (triplets [3,N], batch boundaries)."""
    losses = []
    for b in range(len(bounds) - 1):
        s, e = bounds[b], bounds[b + 1]
        losses.append(bpr_step_dense(P, Q, triplets[0, s:e], triplets[1, s:e], triplets[2, s:e], lr, wd))
    return np.array(losses)


def bpr_step_stale(P, Q, Qs, u, i, j, lr, wd):
    """One step of the reference (bpr_step_dense) whose forward and gradients read the item rows
    Qs instead of Q (the rows a stale-1 sharded step receives, see sharded_stale1_serial); the
    update is applied to the current P and Q (their weight decay included), exactly torch's SGD
    given those gradients.  In place; returns the loss."""
    f32 = np.float32
    lr = f32(lr)
    wd = f32(wd)
    u = np.asarray(u, dtype=np.int64)
    i = np.asarray(i, dtype=np.int64)
    j = np.asarray(j, dtype=np.int64)
    pu, qi, qj = P[u], Qs[i], Qs[j]
    x = (pu * qi).sum(-1, dtype=f32) - (pu * qj).sum(-1, dtype=f32)
    s = (f32(1) / (f32(1) + np.exp(-x, dtype=f32))).astype(f32)
    with np.errstate(divide="ignore"):
        loss = float(-np.log(s.astype(np.float64)).sum())
    c = (f32(1) - s).astype(f32)
    gP = np.zeros_like(P)
    gQ = np.zeros_like(Q)
    np.add.at(gP, u, (-c)[:, None] * qi + c[:, None] * qj)
    np.add.at(gQ, i, (-c)[:, None] * pu)
    np.add.at(gQ, j, c[:, None] * pu)
    for W, G in ((P, gP), (Q, gQ)):
        W -= lr * (G + wd * W)
    return loss


def sharded_stale1_serial(P, Q, batches, lr, wd, chunk):
    """The opt-in stale-1 sharded step (semantics "stale1", csrc/dist.cpp enqueue_stale1), as one
    table: the spec, NOT the reference step.  The runner overlaps step k's gradient exchange and
    the owners' apply with step k+1's compute, so the item rows a step reads miss the previous
    step's gradients: step t reads Q_{t-2} (the table after step t-2) brought to step t-1 by the
    weight decay alone, i.e. a * Q_{t-2} (a = 1 - lr wd; the owners' gather decays rows to the
    consuming step, dist_body.h owner_gather_body).  Users are owned by their rank and stay exact:
    P is current.  The first step of every runner chunk (`chunk` steps; the plans change there)
    reads the current table.  The update is the reference's SGD on the current P and Q with the
    gradients taken at those rows (bpr_step_stale).  With chunk = 1 every step is the reference
    step.  batches: the union batch of every step (u, i, j).  In place; returns per-step losses."""
    a = np.float32(1) - np.float32(lr) * np.float32(wd)
    losses = []
    prev = None  # the table before the previous step's update (a step that was not a chunk start)
    for k, (u, i, j) in enumerate(batches):
        if k % chunk == 0:
            Qs = Q.copy()
        else:
            Qs = (prev * a).astype(np.float32)
        prev = Q.copy()
        losses.append(bpr_step_stale(P, Q, Qs, u, i, j, lr, wd))
    return np.array(losses)


def hogwild_serial(P, Q, u, i, j, lr, wd, B, t0=0, sP=None, sQ=None):
    """The opt-in relaxed mode (semantics "hogwild", csrc/hogwild.hip) run serially: the spec its
    SERIAL test build (BPRMF_HOGWILD_SERIAL=1: one lane group, slot order) must reproduce.
    NOT the reference step (BPRMFRecommender.py:172-176 sums a batch's gradients before one
    update); this applies each triplet on its own, keeping the reference's per-step weight decay:
      slot s belongs to step t = t0 + 1 + s // B; a row with stamp st < t is first brought to step
      t - 1 (x (1 - lr wd)^(t-1-st)) and takes the wd term, its stamp becomes t; a row with
      st >= t (already updated in step t) takes neither;
      x = <P_u,Q_i> - <P_u,Q_j>, c = sigmoid(-x); g_u = -c (Q_i - Q_j), g_i = -c P_u, g_j = c P_u,
      all from the values read before the triplet's stores; i == j: the one row takes g_i + g_j
      (as the reference's summed dense gradient does).
    In place on float32 P, Q; stamps sP, sQ (int arrays, default all t0) are updated too.
    Returns the loss sum of -log sigmoid(x) (float64)."""
    P_, Q_ = P, Q
    sP = np.full(P.shape[0], t0, np.int64) if sP is None else sP
    sQ = np.full(Q.shape[0], t0, np.int64) if sQ is None else sQ
    log2a = math.log2(1.0 - float(lr) * float(wd))
    lr32, wd32 = np.float32(lr), np.float32(wd)
    loss = 0.0

    def bring(W, st, r, t):
        if st[r] < t:
            f = np.float32(2.0 ** np.float32((t - 1 - st[r]) * log2a)) if t - 1 - st[r] > 0 else np.float32(1)
            return (W[r] * f).astype(np.float32), True
        return W[r].copy(), False

    for s in range(len(u)):
        t = t0 + 1 + s // B
        uu, ii, jj = int(u[s]), int(i[s]), int(j[s])
        pu, fu = bring(P_, sP, uu, t)
        vi, fi = bring(Q_, sQ, ii, t)
        vj, fj = bring(Q_, sQ, jj, t)
        x = np.float32(np.dot(pu.astype(np.float64), vi.astype(np.float64)) -
                       np.dot(pu.astype(np.float64), vj.astype(np.float64)))
        c = np.float32(1.0) / (np.float32(1.0) + np.float32(np.exp(np.float64(x))))
        loss += float(np.logaddexp(0.0, -float(x)))
        gu, gi, gj = -c * (vi - vj), -c * pu, c * pu
        P_[uu] = pu - lr32 * (gu + (wd32 if fu else np.float32(0)) * pu)
        if ii == jj:
            Q_[ii] = vi - lr32 * ((gi + gj) + (wd32 if fi else np.float32(0)) * vi)
        else:
            Q_[ii] = vi - lr32 * (gi + (wd32 if fi else np.float32(0)) * vi)
            Q_[jj] = vj - lr32 * (gj + (wd32 if fj else np.float32(0)) * vj)
        if fu:
            sP[uu] = t
        if fi:
            sQ[ii] = t
        if fj:
            sQ[jj] = t
    return loss, sP, sQ


def local_serial(P, Q, u, i, j, lr, wd, B, hot, period, t0=0):
    """The opt-in bounded-staleness mode (semantics "local", csrc/hogwild.hip LOCAL + k_local_merge)
    run serially on ONE XCD (its SERIAL test build: one lane group, slot order, so one replica
    changes): the spec that build must reproduce.  NOT the reference step.
      users and cold items: exactly hogwild_serial's rule (stamps, per-step weight decay);
      hot items (`hot`: item ids): read and written in the XCD's replica, which starts each period
      equal to the base row b0 (current at the period's first step t_a); a replica update is
      W - lr g (no weight-decay term, no stamp);
      a period ends every `period` steps and at the end of the slots: the base row becomes
      fma(b0, (1 - lr wd)^(t_b - t_a), replica - b0) (the other XCDs' replicas add exactly 0),
      current at t_b, and the replica restarts from it.
    In place on float32 P, Q.  Returns (loss, sP, sQ)."""
    sP = np.full(P.shape[0], t0, np.int64)
    sQ = np.full(Q.shape[0], t0, np.int64)
    hot = set(int(x) for x in hot)
    log2a = math.log2(1.0 - float(lr) * float(wd))
    lr32, wd32 = np.float32(lr), np.float32(wd)

    def dec(k):
        return np.float32(2.0 ** np.float32(k * log2a)) if k > 0 else np.float32(1)

    def bring(W, st, r, t):
        if st[r] < t:
            return (W[r] * dec(t - 1 - st[r])).astype(np.float32), True
        return W[r].copy(), False

    rep = {h: Q[h].copy() for h in hot}  # base rows current at t0 (stamps t0)
    t_a = t0
    loss = 0.0
    n = len(u)
    for s in range(n):
        t = t0 + 1 + s // B
        uu, ii, jj = int(u[s]), int(i[s]), int(j[s])
        pu, fu = bring(P, sP, uu, t)
        vi, fi = (rep[ii].copy(), False) if ii in hot else bring(Q, sQ, ii, t)
        vj, fj = (rep[jj].copy(), False) if jj in hot else bring(Q, sQ, jj, t)
        x = np.float32(np.dot(pu.astype(np.float64), vi.astype(np.float64)) -
                       np.dot(pu.astype(np.float64), vj.astype(np.float64)))
        c = np.float32(1.0) / (np.float32(1.0) + np.float32(np.exp(np.float64(x))))
        loss += float(np.logaddexp(0.0, -float(x)))
        gu, gi, gj = -c * (vi - vj), -c * pu, c * pu
        P[uu] = pu - lr32 * (gu + (wd32 if fu else np.float32(0)) * pu)
        if fu:
            sP[uu] = t
        upd = [(ii, vi, gi + gj, fi)] if ii == jj else [(ii, vi, gi, fi), (jj, vj, gj, fj)]
        for r, v, g, f in upd:
            new = v - lr32 * (g + (wd32 if f else np.float32(0)) * v)
            if r in hot:
                rep[r] = new
            else:
                Q[r] = new
                if f:
                    sQ[r] = t
        last = s + 1 == n
        if last or ((s + 1) % B == 0 and t - t_a >= period):
            t_b = t
            fk = dec(t_b - t_a)
            for h in hot:
                b0 = Q[h].copy()  # stamp t_a
                Q[h] = (b0.astype(np.float64) * np.float64(fk) +
                        (rep[h] - b0).astype(np.float64)).astype(np.float32)
                sQ[h] = t_b
                rep[h] = Q[h].copy()
            t_a = t_b
    return loss, sP, sQ


def local_dp_serial(P_parts, Q, trips, lr, wd, B, hots, period, dp_period, world, overlap=False):
    """semantics "local" at world > 1 (csrc/dist.cpp dp_run / dp_merge, hogwild.hip k_dp_delta /
    k_dp_apply), each rank run serially on one XCD (the SERIAL test build): the spec, NOT the
    reference step.
      rank r trains its users' rows P_parts[r] (row = u // world) and its own copy of the whole
      item table with local_serial on trips[r] = (u, i, j) (B triplets per step, global ids; hot
      set hots[r]);
      every dp_period steps and at the end: each copy is brought to t1 (rows decayed from their
      stamps), delta_r = copy - base * a^(t1 - tm) (base: the table of the last merge, current at
      tm); every copy and the base become base * a^(t1 - tm) + sum of the deltas in rank order.
      overlap (dp_overlap): at a merge other than the last, the sum is only started; each rank
      goes on from its own copy.  At the next merge (step t1, the sum started at tp lands): the
      base becomes base * a^(tp - tm) + sum (current at tp), the copy adds the other ranks' part
      (sum - delta_r) * a^(t1 - tp), and the new delta is taken against the new base decayed to
      t1.  The last merge is blocking as above.
    P_parts updated in place, rows current at the returned stamps.  Returns (loss, sPs, Q at T)."""
    log2a = math.log2(1.0 - float(lr) * float(wd))

    def dec(k):
        return np.float32(2.0 ** np.float32(k * log2a)) if k > 0 else np.float32(1)

    steps = len(trips[0][0]) // B
    base = Q.astype(np.float32).copy()
    copies = [base.copy() for _ in range(world)]
    sPs = [np.zeros(p.shape[0], np.int64) for p in P_parts]
    pend = None  # (tp, sum, deltas) of a started all-reduce
    loss = 0.0
    tm = 0
    ts = 0  # the step every copy is current at
    while ts < steps:
        t1 = min(steps, ts + dp_period)
        last = t1 == steps
        mats = []
        for r in range(world):
            Pr = P_parts[r]
            for x in range(Pr.shape[0]):  # local_serial starts every row at t0 = ts
                Pr[x] = Pr[x] * dec(ts - sPs[r][x])
            Qr = copies[r]
            u, i, j = (np.asarray(v)[ts * B:t1 * B] for v in trips[r])
            lo, sP, sQ = local_serial(Pr, Qr, u // world, i, j, lr, wd, B, hots[r], period, t0=ts)
            loss += lo
            sPs[r] = sP
            mats.append(np.stack([Qr[x] * dec(t1 - sQ[x]) for x in range(Qr.shape[0])]).astype(np.float64))
        if pend is not None:
            tp, ssum, dl = pend
            g = base.astype(np.float64) * np.float64(dec(tp - tm)) + ssum
            for r in range(world):
                mats[r] = mats[r] + (ssum - dl[r]) * np.float64(dec(t1 - tp))
            base = g.astype(np.float32)
            tm = tp
            pend = None
        gd = base.astype(np.float64) * np.float64(dec(t1 - tm))
        deltas = [mats[r] - gd for r in range(world)]
        ssum = np.zeros_like(gd)
        for r in range(world):
            ssum += deltas[r]
        if overlap and not last:
            pend = (t1, ssum, deltas)
            copies = [mats[r].astype(np.float32) for r in range(world)]
        else:
            base = (gd + ssum).astype(np.float32)
            tm = t1
            copies = [base.copy() for _ in range(world)]
        ts = t1
    return loss, sPs, base


# ----------------------------------------------------------------------------------------------
# 2. sampler specification (bit-exact target for the HIP sampler)
# ----------------------------------------------------------------------------------------------
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK32 = np.uint64(0xFFFFFFFF)
TAG_NEG = 0x4E470000   # counter word 3 for negative draws ('NG'), low 16 bits = attempt
TAG_PERM = 0x50520000  # counter word 3 for Feistel round keys ('PR'), low 16 bits = round
FEISTEL_ROUNDS = 6


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10.  Counter words are uint32 arrays (or scalars); key two uint32."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & _MASK32 for c in (c0, c1, c2, c3))
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0)), lo1, (hi0 ^ c3 ^ np.uint64(k1)), lo0
        k0 = (k0 + _W0) & 0xFFFFFFFF
        k1 = (k1 + _W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def _seed_key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, seed >> 32


def feistel_dims(n):
    """Domain Z_a x Z_c of the Feistel permutation: c = ceil(sqrt(n)), a = ceil(n / c)."""
    n = int(n)
    if n <= 1:
        return 1, 1
    c = math.isqrt(n)
    if c * c < n:
        c += 1
    return (n + c - 1) // c, c


def permute(q, n, seed, epoch):
    """Keyed bijection of [0,n): 6-round alternating Feistel on Z_a x Z_c + cycle-walking.

    x = L*c + R (feistel_dims); even rounds L = (L + (F(R)*a >> 32)) mod a, odd rounds
    R = (R + (F(L)*c >> 32)) mod c, F = Philox4x32-10 word 0 of (half, round, epoch, tag|round)."""
    k0, k1 = _seed_key(seed)
    fa, fc = feistel_dims(n)
    ua, uc = np.uint64(fa), np.uint64(fc)
    x = np.asarray(q, dtype=np.uint64).copy()
    todo = np.ones(x.shape, dtype=bool)
    while todo.any():
        y = x[todo]
        L = y // uc
        R = y % uc
        for r in range(FEISTEL_ROUNDS):
            src = L if r & 1 else R
            f = philox4x32_10(src & np.uint64(0xFFFFFFFF), np.uint64(r), np.uint64(epoch),
                              np.uint64(TAG_PERM | r), k0, k1)[0]
            if r & 1:
                R = (R + ((f * uc) >> np.uint64(32))) % uc
            else:
                L = (L + ((f * ua) >> np.uint64(32))) % ua
        y = L * uc + R
        x[todo] = y
        todo[todo] = y >= np.uint64(n)
    return x.astype(np.int64)


def _bounded(q, epoch, n, k0, k1):
    """Unbiased Lemire reduction of Philox output into [0,n) for each triplet q (n>0 per element)."""
    q = np.asarray(q, dtype=np.uint64)
    n = np.asarray(n, dtype=np.uint64)
    out = np.zeros(q.shape, dtype=np.uint64)
    att = np.zeros(q.shape, dtype=np.uint64)
    todo = np.ones(q.shape, dtype=bool)
    thresh = ((np.uint64(1 << 32) - n) % n)  # (2^32 - n) mod n
    while todo.any():
        qq = q[todo]
        r = philox4x32_10(qq & _MASK32, qq >> np.uint64(32), np.uint64(epoch),
                          np.uint64(TAG_NEG) | att[todo], k0, k1)[0]
        m = r * n[todo]
        lo = m & _MASK32
        ok = lo >= thresh[todo]
        idx = np.flatnonzero(todo)
        out[idx[ok]] = m[ok] >> np.uint64(32)
        att[idx[~ok]] += np.uint64(1)
        todo[idx[ok]] = False
    return out.astype(np.int64)


def build_csr(users, items, user_num):
    """Per-user sorted, de-duplicated positive lists (the dok_matrix of data_loader.py:538-545)."""
    users = np.asarray(users, dtype=np.int64)
    items = np.asarray(items, dtype=np.int64)
    key = np.unique(users * (1 << 32) + items)
    uu = key >> 32
    ii = key & 0xFFFFFFFF
    indptr = np.zeros(user_num + 1, dtype=np.int64)
    np.add.at(indptr, uu + 1, 1)
    return np.cumsum(indptr), ii.astype(np.int32)


def kth_nonmember(indptr, indices, u, k):
    """j = the k-th (0-based) item id not in the sorted list of user u.  Vectorised binary search
    for m = #{idx : a[idx] - idx <= k}; then j = k + m."""
    u = np.asarray(u, dtype=np.int64)
    k = np.asarray(k, dtype=np.int64)
    lo = np.zeros(u.shape, dtype=np.int64)
    hi = indptr[u + 1] - indptr[u]
    base = indptr[u]
    while True:
        act = lo < hi
        if not act.any():
            break
        mid = (lo + hi) >> 1
        a = np.where(act, indices[np.where(act, base + mid, 0)].astype(np.int64) - mid, 0)
        go_right = act & (a <= k)
        lo = np.where(go_right, mid + 1, lo)
        hi = np.where(act & ~go_right, mid, hi)
    return k + lo


def sample_triplets(pos_u, pos_i, indptr, indices, item_num, num_ng, seed, epoch, first, count):
    """Triplet slots [first, first+count) of an epoch -> (u, i, j) int32 arrays.

    slot s -> q = permute(s) -> positive p = q // num_ng -> (u,i) = pos[p]; j via kth_nonmember.
    """
    n = len(pos_u) * num_ng
    s = np.arange(first, first + count, dtype=np.int64)
    q = permute(s, n, seed, epoch)
    p = q // num_ng
    u = np.asarray(pos_u, dtype=np.int64)[p]
    i = np.asarray(pos_i, dtype=np.int64)[p]
    deg = indptr[u + 1] - indptr[u]
    free = item_num - deg
    if (free <= 0).any():
        raise ValueError("user with no negative item (reference ng_sample would loop forever)")
    k0, k1 = _seed_key(seed)
    k = _bounded(q, epoch, free, k0, k1)
    j = kth_nonmember(indptr, indices, u, k)
    return u.astype(np.int32), i.astype(np.int32), j.astype(np.int32)


# ----------------------------------------------------------------------------------------------
# 3. metrics (restated from util/metrics.py:99-195 for host-only KAT cross-checks)
# ----------------------------------------------------------------------------------------------
def hr_ndcg_from_scores(test_users, test_items, scores, gt, k=10):
    """Final KPI of BPRMFRecommender.py:196-229: per user rank candidates by score, take top-k,
    HR = sum hits / sum |gt| (metrics.py:159-167), NDCG = mean DCG/IDCG (metrics.py:169-195)."""
    order = np.lexsort((-scores, test_users))
    tu = test_users[order]
    ti = test_items[order]
    starts = np.flatnonzero(np.r_[True, tu[1:] != tu[:-1]])
    ends = np.r_[starts[1:], len(tu)]
    hits = denom = 0
    ndcgs = []
    for s, e in zip(starts, ends):
        u = int(tu[s])
        top = ti[s:min(e, s + k)]
        g = gt[u]
        r = np.array([1.0 if int(x) in g else 0.0 for x in top])
        hits += r.sum()
        denom += len(g)
        disc = 1.0 / np.log2(np.arange(2, len(r) + 2))
        dcg = ((2 ** r - 1) * disc).sum()
        rs = np.sort(r)[::-1]
        idcg = ((2 ** rs - 1) * disc).sum()
        ndcgs.append(dcg / idcg if idcg else 0.0)
    return hits / denom, float(np.mean(ndcgs))
