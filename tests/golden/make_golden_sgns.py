"""Generate the Item2Vec / SGNS fixtures by IMPORTING the reference's classes in the build
container and driving them as its script does:

* corpus: `util.data_loader.BuildCorpus` (util/data_loader.py:1118-1171) on a small synthetic
  ratings frame; build() gives the vocabulary (idx2word) and convert() the skip-gram rows.  Both
  write pickles into ./data/<dataset>/ relative to the working directory: this script runs them in
  a temporary directory and captures the objects handed to pickle.dump instead of reading any
  pickle back.
* steps: `Item2VecRecommender.Item2Vec` + `SGNS` (:39-97) with `optim.Adam(sgns.parameters())`
  (:272), loss / zero_grad / backward / step (:282-286).  SGNS.forward draws its negatives from
  torch's global RNG first thing; the script draws the same numbers beforehand from a saved RNG
  state and records them, so a checker can replay the exact negatives.  Uniform negatives
  (`weights=None`, the script's default) and weighted ones (`--weights`: wf^0.75).

sgns_cases.npz, per case c: V, E, C, n_negs, B, steps, weighted, noise (weights or empty),
iwords [steps, B], owords [steps, B, C], nwords [steps, B, C * n_negs], init_i / init_o,
loss [steps], grad0_i / grad0_o (first step), final_i / final_o, adam_m_i, adam_v_i, adam_m_o,
adam_v_o (after the last step).  corpus_*: the BuildCorpus fixture.
Run:  python tests/golden/make_golden_sgns.py
"""
import os
import pickle
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def corpus_fixture(out):
    import pandas as pd
    from util import data_loader as D
    g = np.random.default_rng(3)
    n = 400
    df = pd.DataFrame({"user": g.integers(0, 25, n), "item": (g.zipf(1.6, n) - 1) % 60,
                       "rating": g.integers(1, 6, n).astype(float), "timestamp": np.arange(n)})
    captured = []
    real_dump = pickle.dump
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "data", "toy"))
        os.chdir(tmp)
        try:
            pickle.dump = lambda obj, f, *a, **k: captured.append(obj)
            pre = D.BuildCorpus(df, window=3, max_vocab=40, unk="<UNK>", dataset="toy")
            pre.build()
            train = df.iloc[: 300]
            pre.convert(train, 0)
        finally:
            pickle.dump = real_dump
            os.chdir(cwd)
    wc, vocab, idx2word, word2idx, data = captured
    out["corpus_user"] = df.user.values.astype(np.int64)
    out["corpus_item"] = df.item.values.astype(np.int64)
    out["corpus_train_rows"] = np.array(300)
    out["corpus_window"] = np.array(3)
    out["corpus_max_vocab"] = np.array(40)
    # the UNK token as -1 (idx2word holds it at 0 and, as wc counts it once, again further down)
    out["corpus_idx2word"] = np.array([-1 if w == "<UNK>" else int(w) for w in idx2word], np.int64)
    wcount = np.array([wc[w] for w in idx2word], np.int64)
    out["corpus_wc"] = wcount
    out["corpus_iwords"] = np.array([d[0] for d in data], np.int64)
    out["corpus_owords"] = np.array([d[1] for d in data], np.int64)


def steps_fixture(out, name, V, E, C, n_negs, B, steps, weighted, seed):
    import torch
    from Item2VecRecommender import Item2Vec, SGNS
    torch.manual_seed(seed)
    g = np.random.default_rng(seed)
    noise = None
    if weighted:
        noise = g.integers(1, 50, V).astype(np.float64)
    model = Item2Vec(vocab_size=V, embedding_size=E)
    sgns = SGNS(embedding=model, vocab_size=V, n_negs=n_negs, weights=noise)
    opt = torch.optim.Adam(sgns.parameters())
    init_i = model.ivectors.weight.detach().numpy().copy()
    init_o = model.ovectors.weight.detach().numpy().copy()
    iw = g.integers(0, V, (steps, B))
    ow = g.integers(0, V, (steps, B, C))
    ow[:, :, 0] = 0  # UNK padding contexts, as skipgram() makes at sentence ends
    iw[0, :3] = iw[0, 0]  # a repeated centre word
    nw, losses = [], []
    for s in range(steps):
        st = torch.get_rng_state()
        if weighted:
            draw = torch.multinomial(sgns.weights, B * C * n_negs, replacement=True).view(B, -1)
        else:
            draw = torch.FloatTensor(B, C * n_negs).uniform_(0, V - 1).long()
        torch.set_rng_state(st)
        nw.append(draw.numpy().copy())
        loss = sgns(torch.from_numpy(iw[s]), torch.from_numpy(ow[s]))
        opt.zero_grad()
        loss.backward()
        if s == 0:
            grad0_i = model.ivectors.weight.grad.detach().numpy().copy()
            grad0_o = model.ovectors.weight.grad.detach().numpy().copy()
        opt.step()
        losses.append(float(loss.detach()))
    state = opt.state_dict()["state"]
    c = dict(V=V, E=E, C=C, n_negs=n_negs, B=B, steps=steps, weighted=int(weighted),
             noise=noise if weighted else np.zeros(0), iwords=iw.astype(np.int32),
             owords=ow.astype(np.int32), nwords=np.stack(nw).astype(np.int32), init_i=init_i,
             init_o=init_o, loss=np.array(losses), grad0_i=grad0_i, grad0_o=grad0_o,
             final_i=model.ivectors.weight.detach().numpy(),
             final_o=model.ovectors.weight.detach().numpy(),
             adam_m_i=state[0]["exp_avg"].numpy(), adam_v_i=state[0]["exp_avg_sq"].numpy(),
             adam_m_o=state[1]["exp_avg"].numpy(), adam_v_o=state[1]["exp_avg_sq"].numpy())
    for key, v in c.items():
        out[f"{name}_{key}"] = np.asarray(v)


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import torch
    torch.set_num_threads(1)
    out = {}
    corpus_fixture(out)
    cases = [("uni", 50, 16, 4, 5, 32, 4, False, 1), ("wtd", 80, 24, 6, 3, 48, 3, True, 2),
             ("e300", 120, 300, 10, 20, 64, 2, False, 3)]
    for cs in cases:
        steps_fixture(out, *cs)
    out["cases"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(OUT, "sgns_cases.npz"), **out)


if __name__ == "__main__":
    main()
