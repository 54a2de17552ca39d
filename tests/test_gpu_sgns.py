"""GPU: the Item2Vec path (include/sgns.h, sgns.hip) through the Item2Vec / SGNS drop-ins, against
the reference module's own steps (tests/golden/sgns_cases.npz: Item2Vec + SGNS + Adam run with
torch's RNG, negatives recorded) and the float64 oracle (oracle/sgns_oracle.py).

The drop-in's Item2Vec draws its initial tables from torch's RNG exactly as the reference does, so
the fixtures replay from the same seed.  Tolerances: float32 on both sides, different summation
orders (f32 atomics for the centre-row gradient, an sgemm for the context rows), then Adam, whose
first updates are ~lr * m / (|g| + eps): PARAM_ATOL on the tables, MOM_RTOL of scale on the
moments, LOSS_RTOL on the losses."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import sgns_oracle as O

pytestmark = pytest.mark.gpu

F = np.load(os.path.join(GOLDEN, "sgns_cases.npz"))
CASES = [str(c) for c in F["cases"]]
SEEDS = {"uni": 1, "wtd": 2, "e300": 3}
PARAM_ATOL = 1e-5
MOM_RTOL = 1e-4
LOSS_RTOL = 1e-5


def case(name):
    return {k[len(name) + 1:]: F[k] for k in F.files if k.startswith(name + "_")}


def make(rl, c, seed=None):
    import torch
    torch.manual_seed(SEEDS.get(seed, 0) if isinstance(seed, str) else 0)
    V, E = int(c["V"]), int(c["E"])
    m = rl.Item2Vec(vocab_size=V, embedding_size=E)
    noise = c["noise"] if int(c["weighted"]) else None
    s = rl.SGNS(embedding=m, vocab_size=V, n_negs=int(c["n_negs"]), weights=noise,
                context=int(c["C"]), max_batch=int(c["B"]), seed=11)
    return m, s


@pytest.mark.parametrize("name", CASES)
def test_steps_match_reference_module(rl, name):
    c = case(name)
    m, s = make(rl, c, name)
    sd = s.state_dict()
    np.testing.assert_array_equal(sd["embedding.ivectors.weight"], c["init_i"])
    np.testing.assert_array_equal(sd["embedding.ovectors.weight"], c["init_o"])
    for k in range(int(c["steps"])):
        loss = s.train_examples(c["iwords"][k], c["owords"][k], c["nwords"][k], batch_size=int(c["B"]))
        assert loss == pytest.approx(float(c["loss"][k]), rel=LOSS_RTOL)
    sd = s.state_dict()
    np.testing.assert_allclose(sd["embedding.ivectors.weight"], c["final_i"], rtol=0, atol=PARAM_ATOL)
    np.testing.assert_allclose(sd["embedding.ovectors.weight"], c["final_o"], rtol=0, atol=PARAM_ATOL)
    assert not sd["embedding.ivectors.weight"][0].any() and not sd["embedding.ovectors.weight"][0].any()
    st = s.optimizer_state_dict()["state"]
    assert st[0]["step"] == int(c["steps"])
    for q, key in ((0, "i"), (1, "o")):
        for mom, ref in ((st[q]["exp_avg"], c["adam_m_" + key]), (st[q]["exp_avg_sq"], c["adam_v_" + key])):
            np.testing.assert_allclose(mom, ref, rtol=0, atol=MOM_RTOL * np.abs(ref).max())


def test_larger_vocab_against_oracle(rl):
    """V = 2000, E = 300 (the reference default), window 5, 20 negatives, 3 steps of B = 256."""
    g = np.random.default_rng(9)
    V, E, C, n, B = 2000, 300, 10, 20, 256
    import torch
    torch.manual_seed(4)
    m = rl.Item2Vec(V, E)
    s = rl.SGNS(m, V, n_negs=n, context=C, max_batch=B)
    st = O.State(*m._init)
    for k in range(3):
        iw = g.integers(1, V, B)
        iw[:20] = 7  # a hot centre word
        ow = g.integers(0, V, (B, C))
        nw = s.negatives(B)
        assert nw.min() >= 0 and nw.max() <= V - 2
        want = O.step(st, iw, ow, nw)
        got = s.train_examples(iw, ow)  # negatives drawn on the device: the ones returned above
        assert got == pytest.approx(want, rel=LOSS_RTOL)
    sd = s.state_dict()
    np.testing.assert_allclose(sd["embedding.ivectors.weight"], st.I, rtol=0, atol=PARAM_ATOL)
    np.testing.assert_allclose(sd["embedding.ovectors.weight"], st.O, rtol=0, atol=PARAM_ATOL)
    np.testing.assert_allclose(m.forward_i([7, 3]), st.I[[7, 3]], rtol=0, atol=PARAM_ATOL)
    np.testing.assert_allclose(m.forward_o(np.array([[1, 2]])), st.O[[[1, 2]]], rtol=0, atol=PARAM_ATOL)


def test_negative_distributions(rl):
    c = case("wtd")
    _, s = make(rl, c)
    V = int(c["V"])
    import torch
    torch.manual_seed(0)
    su = rl.SGNS(rl.Item2Vec(V, 8), V, n_negs=50, context=10, max_batch=4096)
    x = su.negatives(4096).reshape(-1)
    assert x.min() == 0 and x.max() == V - 2  # uniform_(0, V - 1).long()
    h = np.bincount(x, minlength=V)[: V - 1] / len(x)
    assert np.abs(h - 1.0 / (V - 1)).max() < 0.1 / (V - 1)
    sw = rl.SGNS(rl.Item2Vec(V, 8), V, n_negs=50, context=10, max_batch=4096,
                 weights=c["noise"])
    y = sw.negatives(4096).reshape(-1)
    p = np.power(c["noise"], 0.75)
    p /= p.sum()
    hy = np.bincount(y, minlength=V) / len(y)
    assert np.abs(hy - p).max() < 0.1 * p.max()
    # a step consumes its draws: the next step draws anew, deterministically
    a = su.negatives(64)
    assert np.array_equal(a, su.negatives(64))
    su.train_examples(np.ones(64, np.int32), np.ones((64, 10), np.int32))
    assert (su.negatives(64) != a).mean() > 0.9


def test_resume_from_state_dicts(rl):
    c = case("uni")
    g = np.random.default_rng(2)
    V, B, C = int(c["V"]), int(c["B"]), int(c["C"])
    batches = [(g.integers(0, V, B), g.integers(0, V, (B, C))) for _ in range(3)]
    _, s1 = make(rl, c, "uni")
    for iw, ow in batches[:2]:
        s1.train_examples(iw, ow)
    sd, osd = s1.state_dict(), s1.optimizer_state_dict()
    _, s2 = make(rl, c)
    s2.load_state_dict(sd)
    s2.load_optimizer_state_dict(osd)
    assert s2.steps == 2
    nw = s1.negatives(B)
    s1.train_examples(*batches[2], nwords=nw)
    s2.train_examples(*batches[2], nwords=nw)
    a, b = s1.state_dict(), s2.state_dict()
    for k in a:
        np.testing.assert_allclose(a[k], b[k], rtol=0, atol=1e-7)


def test_epoch_over_corpus_and_bad_inputs(rl):
    import pandas as pd
    g = np.random.default_rng(1)
    df = pd.DataFrame({"user": g.integers(0, 30, 600), "item": g.integers(0, 90, 600)})
    pre = rl.BuildCorpus(df, window=2, max_vocab=100).build()
    data = rl.PermutedSubsampledCorpus(pre.convert(df, 0))
    V = len(pre.idx2word)
    m = rl.Item2Vec(V, 32)
    s = rl.SGNS(m, V, n_negs=5, context=4, max_batch=128)
    loss = s.train_epoch(data, 128)
    assert np.isfinite(loss) and s.last_stats["steps"] == (len(data) + 127) // 128
    with pytest.raises(ValueError):
        s.train_examples([V], np.zeros((1, 4)))
    with pytest.raises(ValueError):
        s.train_examples([1], np.full((1, 4), -1))
    with pytest.raises(ValueError):
        s.train_examples([1], np.zeros((1, 4)), batch_size=129)
    assert s.train_examples(np.zeros(0), np.zeros((0, 4))) == 0.0


@pytest.mark.parametrize("E,C,n", [(1, 2, 1), (64, 4, 0), (130, 6, 3), (1024, 2, 2)])
def test_embedding_widths_against_oracle(rl, E, C, n):
    """Every lanes-per-wave width (ceil(E/64) = 1, 1, 3, 16), no negatives, odd widths."""
    import torch
    g = np.random.default_rng(E)
    V, B = 90, 40
    torch.manual_seed(E)
    m = rl.Item2Vec(V, E)
    s = rl.SGNS(m, V, n_negs=n, context=C, max_batch=B)
    st = O.State(*m._init)
    for _ in range(2):
        iw, ow = g.integers(0, V, B), g.integers(0, V, (B, C))
        nw = s.negatives(B) if n else np.zeros((B, 0), np.int64)
        want = O.step(st, iw, ow, nw)
        got = s.train_examples(iw, ow)
        assert got == pytest.approx(want, rel=LOSS_RTOL)
    sd = s.state_dict()
    np.testing.assert_allclose(sd["embedding.ivectors.weight"], st.I, rtol=0, atol=PARAM_ATOL)
    np.testing.assert_allclose(sd["embedding.ovectors.weight"], st.O, rtol=0, atol=PARAM_ATOL)
