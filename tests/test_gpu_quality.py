"""GPU: the relaxed modes' training quality against the exact step on data with structure
(DESIGN.md §5c "Quality").

The ml-20m-shaped synthetic set of the bench has no taste structure beyond item popularity, so
every mode's HR@10 there equals the popularity ranking's and tells nothing.  Here the positives
are drawn from a planted rank-8 model plus Zipf popularity (synthetic.make_planted, ml-20m shape,
~10M positives), one random positive per user is held out and ranked against 99 non-positives
(tools/hr_modes.py "planted"): a model has to learn the user-item structure to beat popularity.
Measured (profiles/r05_hr_modes_planted.jsonl, seeds 11-13, 10 epochs): popularity HR@10 0.705;
exact 0.9124 +- 0.0004; local 0.9063 (-0.006); hogwild 0.8905 (-0.022); final-table loss local
+13.5 %, hogwild +19 % over exact.  The relaxed modes are a measured quality / speed trade, not
parity: these bounds pin the trade (twice the measured gap fails) and that every mode learns."""
import importlib.util
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _hr_modes():
    spec = importlib.util.spec_from_file_location("hr_modes", os.path.join(ROOT, "tools", "hr_modes.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_planted_structure_separates_modes_and_beats_popularity(rl):
    H = _hr_modes()
    res = {mode: H.planted(rl, mode, 11, 10, 20000) for mode in ("popularity", "exact", "local", "hogwild")}
    pop, ex, lo, hw = (res[m] for m in ("popularity", "exact", "local", "hogwild"))
    # every trained mode learns the planted structure, far beyond popularity
    for r in (ex, lo, hw):
        assert r["hr10"] >= pop["hr10"] + 0.15, (r["mode"], r["hr10"], pop["hr10"])
        assert r["ndcg10"] >= pop["ndcg10"] + 0.15, (r["mode"], r["ndcg10"], pop["ndcg10"])
    assert ex["hr10"] >= 0.90, ex
    # the relaxed modes' measured cost (local -0.006 / +13.5 %, hogwild -0.022 / +19 %), bounded
    assert lo["hr10"] >= ex["hr10"] - 0.012, (lo["hr10"], ex["hr10"])
    assert hw["hr10"] >= ex["hr10"] - 0.045, (hw["hr10"], ex["hr10"])
    assert lo["eval_loss_per_1e6"] <= 1.27 * ex["eval_loss_per_1e6"], (lo, ex)
    assert hw["eval_loss_per_1e6"] <= 1.38 * ex["eval_loss_per_1e6"], (hw, ex)
    # and the exact step is the best fit of the three (the relaxation is not free)
    assert ex["eval_loss_per_1e6"] < min(lo["eval_loss_per_1e6"], hw["eval_loss_per_1e6"])
