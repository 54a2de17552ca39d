"""CPU: the host side of the Item2Vec path (recommend-lib_amd/item2vec.py) against the reference's
own outputs (tests/golden/sgns_cases.npz, made by running BuildCorpus and Item2Vec): the corpus
(vocabulary and skip-gram rows, bit-exact) and the initial tables drawn from torch's RNG."""
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN

F = np.load(os.path.join(GOLDEN, "sgns_cases.npz"))


def test_build_corpus_matches_reference(rl):
    df = pd.DataFrame({"user": F["corpus_user"], "item": F["corpus_item"]})
    pre = rl.BuildCorpus(df, window=int(F["corpus_window"]), max_vocab=int(F["corpus_max_vocab"]))
    pre.build()
    got = [-1 if w == "<UNK>" else int(w) for w in pre.idx2word]
    np.testing.assert_array_equal(got, F["corpus_idx2word"])
    np.testing.assert_array_equal(pre.word_counts(), F["corpus_wc"])
    iw, ow = pre.convert(df.iloc[: int(F["corpus_train_rows"])], 0)
    np.testing.assert_array_equal(iw, F["corpus_iwords"])
    np.testing.assert_array_equal(ow, F["corpus_owords"])


def test_subsampled_corpus_keeps_by_python_random(rl):
    import random
    iw = np.arange(1, 201, dtype=np.int32) % 7
    ow = np.zeros((200, 4), np.int32)
    ws = np.linspace(0.0, 0.9, 7)
    random.seed(5)
    d = rl.PermutedSubsampledCorpus((iw, ow), ws)
    random.seed(5)
    keep = [w for w in iw if random.random() > ws[w]]
    np.testing.assert_array_equal(d.iwords, keep)
    assert len(rl.PermutedSubsampledCorpus((iw, ow))) == 200


@pytest.mark.parametrize("name", [str(c) for c in F["cases"]])
def test_initial_tables_match_reference_draws(rl, name):
    import torch
    seed = {"uni": 1, "wtd": 2, "e300": 3}[name]
    torch.manual_seed(seed)
    m = rl.Item2Vec(int(F[name + "_V"]), int(F[name + "_E"]))
    np.testing.assert_array_equal(m._init[0], F[name + "_init_i"])
    np.testing.assert_array_equal(m._init[1], F[name + "_init_o"])
