"""CPU: ratings ingestion.  The oracle (oracle/ingest_oracle.py) and the
product (libbprmf_amd.so `bprmf_dataset_*` through recommend-lib_amd/ingest.py, host C++ that
needs no GPU) against tests/golden/ingest_ml100k_slice.npz, made by the reference's own
load_rate / load_mat (tests/golden/make_golden_ingest.py).

Deterministic outputs are compared exactly: load_rate's rows for the three file formats and the
k-core filters, codes, user_num / item_num, the loo split, the cv folds, train_mat sizes and the
loo ground truth.  Where the reference orders equal timestamps at random (fo / tfo) the test checks
what is determined: the timestamp sequence and the rows of every timestamp except the one the
split cuts through."""
import os

import numpy as np
import pytest

from oracle import ingest_oracle as O

FIX = "ingest_ml100k_slice.npz"


def _write(raw, tmp, src):
    """The slice in the file format of `src` (as make_golden_ingest.py writes it)."""
    half = (raw[:, 3] % 2 == 1) & (raw[:, 2] < 5)
    d = os.path.join(tmp, src)
    os.makedirs(d, exist_ok=True)
    if src == "ml-100k":
        p = os.path.join(d, "u.data")
        lines = [f"{u}\t{i}\t{r}\t{t}\n" for u, i, r, t in raw]
    elif src == "ml-20m":
        p = os.path.join(d, "ratings.csv")
        lines = ["userId,movieId,rating,timestamp\n"] + [
            f"{u},{i},{r + 0.5 if h else float(r)},{t}\n" for (u, i, r, t), h in zip(raw, half)]
    else:
        p = os.path.join(d, "ratings.dat")
        lines = [f"{u}::{i}::{r}::{t}\n" for u, i, r, t in raw]
    with open(p, "w") as f:
        f.writelines(lines)
    return p


@pytest.fixture(scope="module")
def fx(golden):
    return golden(FIX)


@pytest.fixture(scope="module")
def data_dir(fx, tmp_path_factory):
    tmp = str(tmp_path_factory.mktemp("data"))
    for src in ("ml-100k", "ml-1m", "ml-20m"):
        _write(fx["raw"], tmp, src)
    return tmp


RATE_CASES = [("ml-100k", "origin", 0.0, 0), ("ml-100k", "5core", 0.0, 5),
              ("ml-100k", "10core", 0.0, 10), ("ml-1m", "origin", 4.0, 0),
              ("ml-20m", "origin", 4.0, 0)]


# ---- oracle vs the reference's outputs -------------------------------------------------------
@pytest.mark.parametrize("src,pre,mr,core", RATE_CASES)
def test_oracle_load_rate(fx, src, pre, mr, core):
    raw = fx["raw"].copy()
    if src == "ml-20m":  # the csv form carries half-star ratings; the >= 4 filter sees them
        half = (raw[:, 3] % 2 == 1) & (raw[:, 2] < 5)
        raw = raw.astype(np.float64)
        raw[half, 2] += 0.5
    rows = O.load_rate_rows(raw, mr, core)
    assert np.array_equal(rows, fx[f"rate_{src}_{pre}_rows"])


def test_oracle_load_mat_loo_cv(fx):
    m = O.load_mat(fx["raw"], "loo", "cv")
    assert [m["user_num"], m["item_num"]] == fx["loo_cv_shape"].tolist()
    assert np.array_equal(np.concatenate(m["folds_va"]), fx["loo_cv_val"])
    assert [len(f) for f in m["folds_va"]] == fx["loo_cv_val_len"].tolist()
    assert [len(f) for f in m["folds_tr"]] == fx["loo_cv_train_len"].tolist()
    gt = np.stack([m["users"][m["is_test"]], m["items"][m["is_test"]]], 1)
    assert np.array_equal(gt, fx["loo_cv_test_gt"])


def _ts_of(m):
    """(user, item) -> timestamp of the coded rows."""
    return {(int(u), int(i)): int(t) for u, i, t in zip(m["users"], m["items"], m["ts"])}


def _same_up_to_tie(ours, ref, ts, cut_ts=None):
    """Pair lists in time order that may differ only in the order of equal timestamps, and in
    which rows of timestamp `cut_ts` made it in."""
    t_o = np.array([ts[tuple(x)] for x in ours.tolist()])
    t_r = np.array([ts[tuple(x)] for x in ref.tolist()])
    assert np.array_equal(t_o, t_r)
    assert np.all(np.diff(t_o) >= 0)
    keep_o, keep_r = t_o != cut_ts, t_r != cut_ts
    so = sorted(map(tuple, ours[keep_o].tolist()))
    sr = sorted(map(tuple, ref[keep_r].tolist()))
    assert so == sr


def test_oracle_load_mat_fo(fx):
    for val in ("tfo", "cv"):
        m = O.load_mat(fx["raw"], "fo", val)
        assert [m["user_num"], m["item_num"]] == fx[f"fo_{val}_shape"].tolist()
        ts = _ts_of(m)
        cut = int(np.sort(m["ts"])[len(m["train"]) - 1])  # the timestamp the 80% split cuts
        assert [len(f) for f in m["folds_tr"]] == fx[f"fo_{val}_train_len"].tolist()
        assert [len(f) for f in m["folds_va"]] == fx[f"fo_{val}_val_len"].tolist()
        if val == "tfo":
            ref = np.concatenate([fx["fo_tfo_train"], fx["fo_tfo_val"]])
            _same_up_to_tie(np.concatenate([m["folds_tr"][0], m["folds_va"][0]]), ref, ts, cut)
        else:
            _same_up_to_tie(np.concatenate(m["folds_va"]), fx["fo_cv_val"], ts, cut)


# ---- product vs the reference and the oracle ---------------------------------------------------
@pytest.mark.parametrize("src,pre,mr,core", RATE_CASES)
@pytest.mark.parametrize("threads", [1, 4])
def test_load_rate_matches_reference(rl, fx, data_dir, src, pre, mr, core, threads):
    df = rl.ingest.load_rate(src, pre, data_dir=data_dir, threads=threads)
    raw = fx["raw"]
    rows = fx[f"rate_{src}_{pre}_rows"]
    assert np.array_equal(df["user"].to_numpy(), raw[rows, 0])
    assert np.array_equal(df["item"].to_numpy(), raw[rows, 1])
    assert np.array_equal(df["timestamp"].to_numpy(), raw[rows, 3])
    want = raw[rows, 2].astype(np.float64)
    if src == "ml-20m":
        want = want + np.where((raw[rows, 3] % 2 == 1) & (raw[rows, 2] < 5), 0.5, 0.0)
    assert np.array_equal(df["rating"].to_numpy(np.float64), want)


def test_load_mat_loo_cv_matches_reference(rl, fx, data_dir):
    tr, test, U, I, mats, ur, va = rl.load_mat("ml-100k", data_dir=data_dir, as_lists=False)
    assert [U, I] == fx["loo_cv_shape"].tolist()
    assert np.array_equal(np.concatenate(va), fx["loo_cv_val"])
    assert [len(f) for f in va] == fx["loo_cv_val_len"].tolist()
    assert [len(f) for f in tr] == fx["loo_cv_train_len"].tolist()
    for f in range(5):
        assert np.array_equal(tr[f], np.concatenate(va[:f] + va[f + 1:]))
    assert [m.nnz for m in mats] == fx["loo_cv_mat_nnz"].tolist()
    assert len(test) == int(fx["loo_cv_test_len"])
    assert np.array_equal(test[::1000], fx["loo_cv_test_gt"])
    assert {u: {i} for u, i in fx["loo_cv_test_gt"].tolist()} == dict(ur)
    # a train_mat is the fold's positives
    d = mats[0]
    assert d.shape == (U, I) and all(d[u, i] == 1.0 for u, i in tr[0][:50].tolist())


def test_load_mat_lists_mirror_reference_types(rl, data_dir):
    tr, test, U, I, mats, ur, va = rl.load_mat("ml-100k", data_dir=data_dir)
    assert isinstance(tr, list) and isinstance(tr[0], list) and isinstance(tr[0][0], list)
    assert isinstance(test, list) and len(test[0]) == 2
    import scipy.sparse as sp
    assert isinstance(mats[0], sp.dok_matrix) and mats[0].dtype == np.float32


def test_loo_negatives_properties(rl, fx, data_dir):
    r = rl.ingest.read_ratings(os.path.join(data_dir, "ml-100k", "u.data"))
    rated = {}
    for u, i in zip(r.users.tolist(), r.items.tolist()):
        rated.setdefault(u, set()).add(i)
    t = r.split(rl.ingest.LOO)
    u, i = r.candidates(t, rl.ingest.LOO, 999, seed=3)
    assert len(u) == 1000 * r.user_num
    for s in range(0, len(u), 1000):
        uu = int(u[s])
        assert np.all(u[s:s + 1000] == uu)
        negs = i[s + 1:s + 1000]
        assert np.all(np.diff(negs) > 0)  # distinct, ascending
        assert not (set(negs.tolist()) & rated[uu])
        assert negs.min() >= 0 and negs.max() < r.item_num
    u2, i2 = r.candidates(t, rl.ingest.LOO, 999, seed=3)
    assert np.array_equal(i, i2)  # a function of the seed
    _, i3 = r.candidates(t, rl.ingest.LOO, 999, seed=4)
    assert not np.array_equal(i, i3)
    r.close()


def test_load_mat_fo_matches_reference(rl, fx, data_dir):
    for val in ("tfo", "cv"):
        tr, test, U, I, mats, ur, va = rl.load_mat("ml-100k", data_split="fo", val_method=val,
                                                   data_dir=data_dir, as_lists=False, seed=1)
        m = O.load_mat(fx["raw"], "fo", val)
        assert [U, I] == fx[f"fo_{val}_shape"].tolist()
        # deterministic tie order: identical to the oracle
        for a, b in zip(tr + va, m["folds_tr"] + m["folds_va"]):
            assert np.array_equal(a, b)
        assert [mm.nnz for mm in mats] == fx[f"fo_{val}_mat_nnz"].tolist()
        assert len(test) == int(fx[f"fo_{val}_test_len"])
        if val != "tfo":
            continue
        ts = _ts_of(m)
        cut = int(np.sort(m["ts"])[len(m["train"]) - 1])
        ref = np.concatenate([fx["fo_tfo_train"], fx["fo_tfo_val"]])
        _same_up_to_tie(np.concatenate([tr[0], va[0]]), ref, ts, cut)
        # ground truth: equal for every user, up to the rows at the cut timestamp
        off = np.concatenate([[0], np.cumsum(fx["fo_tfo_ur_len"])])
        ref_ur = {int(u): set(fx["fo_tfo_ur_item"][off[k]:off[k + 1]].tolist())
                  for k, u in enumerate(fx["fo_tfo_ur_user"])}
        for u in set(ref_ur) | set(ur):
            a = {i for i in ur.get(u, set()) if ts[(u, i)] != cut}
            b = {i for i in ref_ur.get(u, set()) if ts[(u, i)] != cut}
            assert a == b, u
        # test lists: per user, all of its ground truth plus unseen items, 1000 rows per user
        train_items = {}
        for u, i in tr[0].tolist() + va[0].tolist():
            train_items.setdefault(u, set()).add(i)
        users = list(dict.fromkeys(test[:, 0].tolist()))
        assert len(test) == 1000 * len(users) and set(users) == set(ur)
        for u in users:
            lst = test[test[:, 0] == u, 1]
            assert len(lst) == 1000 and len(set(lst.tolist())) == 1000
            assert ur[u] <= set(lst.tolist())
            assert not (set(lst.tolist()) - ur[u]) & train_items.get(u, set())


def test_val_methods_loo_tloo(rl, data_dir):
    for val in ("tloo", "loo"):
        tr, test, U, I, mats, ur, va = rl.load_mat("ml-100k", val_method=val, data_dir=data_dir,
                                                   as_lists=False)
        assert len(tr) == 1 and len(va) == 1
        assert len(np.unique(va[0][:, 0])) == len(va[0])  # one validation row per user
        both = np.concatenate([tr[0], va[0]])
        assert len({tuple(x) for x in both.tolist()}) == len(both)
        assert mats[0].nnz == len(tr[0])


# ---- formats and edge cases -----------------------------------------------------------------
def _load(rl, tmp_path, text, name="r.txt", **kw):
    p = tmp_path / name
    p.write_bytes(text.encode() if isinstance(text, str) else text)
    return rl.ingest.read_ratings(str(p), **kw)


def test_empty_and_header_only(rl, tmp_path):
    r = _load(rl, tmp_path, "")
    assert (r.n, r.user_num, r.item_num) == (0, 0, 0)
    r = _load(rl, tmp_path, "userId,movieId,rating,timestamp\n", name="h.csv")
    assert r.n == 0
    assert r.candidates(r.split(0), 0, 5)[0].size == 0


def test_crlf_blank_lines_and_no_trailing_newline(rl, tmp_path):
    r = _load(rl, tmp_path, "3\t10\t4\t100\r\n\r\n1\t20\t5\t50\r\n2\t10\t3\t70")
    assert r.n == 3
    assert r.user_ids.tolist() == [1, 2, 3] and r.item_ids.tolist() == [10, 20]
    assert r.users.tolist() == [0, 1, 2] and r.items.tolist() == [1, 0, 0]
    assert r.timestamps.tolist() == [50, 70, 100]


def test_sparse_huge_ids_and_ties(rl, tmp_path):
    # ids far apart (sorted-unique coding, not the direct table); duplicate (user, item) rows
    lines = ["1000000000000::7::4::5", "5::900000000000::5::3", "5::7::4::9", "5::7::4::2",
             "1000000000000::7::3::5"]
    r = _load(rl, tmp_path, "\n".join(lines) + "\n")
    assert r.user_ids.tolist() == [5, 1000000000000] and r.item_ids.tolist() == [7, 900000000000]
    assert list(zip(r.users.tolist(), r.items.tolist(), r.timestamps.tolist())) == [
        (0, 0, 2), (0, 0, 9), (0, 1, 3), (1, 0, 5), (1, 0, 5)]
    assert r.ratings.tolist() == [4.0, 4.0, 5.0, 4.0, 3.0]  # the full tie keeps file order


def test_parallel_parse_equals_serial(rl, tmp_path):
    g = np.random.default_rng(0)
    n = 400_000  # > 1 MiB of text: the multi-threaded parse path
    u = g.integers(1, 5000, n)
    i = g.integers(1, 3000, n)
    rt = g.integers(1, 11, n) / 2
    t = g.integers(0, 10**9, n)
    text = "".join(f"{a},{b},{c},{d}\n" for a, b, c, d in zip(u, i, rt, t))
    r1 = _load(rl, tmp_path, "userId,movieId,rating,timestamp\n" + text, name="a.csv",
               min_rating=4.0, threads=1)
    r8 = _load(rl, tmp_path, "userId,movieId,rating,timestamp\n" + text, name="b.csv",
               min_rating=4.0, threads=8)
    for k in ("users", "items", "ratings", "timestamps", "user_ids", "item_ids"):
        assert np.array_equal(getattr(r1, k), getattr(r8, k)), k
    keep = rt >= 4.0
    m = O.load_rate_rows(np.stack([u, i, rt, t], 1)[keep], 0.0)
    src = np.stack([u, i, rt, t], 1)[keep][m]
    assert np.array_equal(r1.user_ids[r1.users], src[:, 0])
    assert np.array_equal(r1.item_ids[r1.items], src[:, 1])
    assert np.array_equal(r1.timestamps, src[:, 3])
    for method in (0, 1):  # splits on all threads equal the oracle's
        t_p = r8.split(method)
        t_o = (O.split_loo(r8.users, r8.timestamps) if method == 0
               else O.split_fo(r8.timestamps)[0])
        assert np.array_equal(t_p, t_o)


def test_errors(rl, tmp_path):
    with pytest.raises(FileNotFoundError):
        rl.ingest.read_ratings(str(tmp_path / "missing.dat"))
    with pytest.raises(ValueError, match="Invalid Dataset"):
        rl.load_rate("netflix", data_dir=str(tmp_path))
    with pytest.raises(ValueError):
        rl.load_rate("ml-100k", prepro="3core", data_dir=str(tmp_path))
    # a user who rated every item but 2 cannot get 999 negatives (random.sample raises there)
    text = "".join(f"1\t{i}\t5\t{i}\n" for i in range(1, 20)) + "2\t1\t5\t1\n"
    r = _load(rl, tmp_path, text)
    with pytest.raises(ValueError, match="population"):
        r.candidates(r.split(0), 0, 999)
    with pytest.raises(ValueError):
        r.split(1, 1.5)
