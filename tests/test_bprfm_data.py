"""CPU: BPRFMData (recommend-lib_amd/bprfm.py), the host side of the BPR-FM path, against the
reference's sampling loop (util/data_loader.py:574-627) restated inline."""
import numpy as np


def test_data_loader_mirrors_reference_sampling(rl):
    """BPRFMData: feature mapping and the reference's rejection sampling order."""
    import pandas as pd
    df = pd.DataFrame({"user": [0, 0, 1, 2, 2, 2], "item": [0, 1, 1, 2, 3, 0],
                       "rating": [5.0] * 6, "timestamp": list(range(6))})
    fid = {"user": 0, "item": 3}
    fmap = {x: x for x in range(7)}
    d = rl.BPRFMData(df.drop(columns=["timestamp"]).copy(), fid, fmap, 4, num_ng=3,
                     is_training=True)
    np.random.seed(11)
    d.ng_sample()
    u, i, j = d.triplets()
    assert len(u) == len(d) == 18
    np.testing.assert_array_equal(u, np.repeat([0, 0, 1, 2, 2, 2], 3))
    np.testing.assert_array_equal(i, np.repeat([3, 4, 4, 5, 6, 3], 3))
    # the same draws, replayed as the reference's loop makes them
    np.random.seed(11)
    train = set(zip(df.user, df.item))
    for q, uu in enumerate(np.repeat([0, 0, 1, 2, 2, 2], 3)):
        jj = np.random.randint(4)
        while (uu, jj) in train:
            jj = np.random.randint(4)
        assert j[q] == jj + 3
