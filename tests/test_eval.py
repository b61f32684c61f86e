"""Evaluators (`Server/similarity_analysis.py:15-82`, `Server/utility_analysis.py:15-119`):
metric definitions and the reference quirks, checked against SciPy / scikit-learn directly."""
import numpy as np
import pandas as pd
import pytest
from scipy.spatial import distance
from scipy.stats import wasserstein_distance

from fed_tgan_amd.eval.similarity import column_jsd, column_similarity, column_wd, stat_sim
from fed_tgan_amd.eval.utility import utility_difference


def test_jsd_base2_over_real_categories_with_missing_double_count():
    real = pd.Series(["a"] * 50 + ["b"] * 30 + ["c"] * 20)
    fake = pd.Series(["a"] * 60 + ["b"] * 40)
    # real categories sorted; the missing "c" contributes 0 and is appended a second time
    rv = [0.5, 0.3, 0.2, 0.2]
    fv = [0.6, 0.4, 0.0, 0.0]
    assert column_jsd(real, fake) == pytest.approx(distance.jensenshannon(rv, fv, base=2.0), rel=1e-9)


def test_jsd_ignores_synthetic_only_categories_and_identity():
    real = pd.Series(["x"] * 70 + ["y"] * 30)
    fake = pd.Series(["x"] * 60 + ["y"] * 20 + ["z"] * 20)   # "z" never seen in the real table
    rv, fv = [0.7, 0.3], [0.6, 0.2]
    assert column_jsd(real, fake) == pytest.approx(distance.jensenshannon(rv, fv, base=2.0), rel=1e-9)
    assert column_jsd(real, real.sample(frac=1.0, random_state=0)) == pytest.approx(0.0, abs=1e-12)


def test_wd_after_minmax_fitted_on_real():
    rng = np.random.default_rng(0)
    real = pd.Series(rng.normal(10, 3, 2000))
    fake = pd.Series(rng.normal(11, 4, 1500))
    lo, hi = real.min(), real.max()
    want = wasserstein_distance((real - lo) / (hi - lo), (fake - lo) / (hi - lo))
    assert column_wd(real, fake) == pytest.approx(want, rel=1e-9)


def test_stat_sim_means_and_per_column_table():
    rng = np.random.default_rng(1)
    real = pd.DataFrame({"c1": rng.choice(["p", "q", "r"], 500), "n1": rng.normal(0, 1, 500),
                         "c2": rng.choice(["u", "v"], 500), "n2": rng.exponential(2, 500)})
    fake = pd.DataFrame({"c1": rng.choice(["p", "q"], 400), "n1": rng.normal(0.5, 1, 400),
                         "c2": rng.choice(["u", "v", "w"], 400), "n2": rng.exponential(3, 400)})
    jsd, wd = stat_sim(real, fake, ["c1", "c2"])
    assert jsd == pytest.approx(np.mean([column_jsd(real.c1, fake.c1), column_jsd(real.c2, fake.c2)]))
    assert wd == pytest.approx(np.mean([column_wd(real.n1, fake.n1), column_wd(real.n2, fake.n2)]))
    tab = column_similarity(real, fake, ["c1", "c2"])
    assert list(tab["metric"]) == ["JSD", "WD", "JSD", "WD"]


def test_utility_difference_is_zero_for_a_copy_of_train():
    rng = np.random.default_rng(2)
    n = 600
    x1 = rng.normal(0, 1, n)
    cat = rng.choice(["a", "b", "c"], n)
    y = ((x1 + (cat == "a") * 1.5 + rng.normal(0, 0.5, n)) > 0.5).astype(int)
    df = pd.DataFrame({"x1": x1, "x2": rng.normal(0, 1, n), "cat": cat, "label": y})
    train, test = df.iloc[:400], df.iloc[400:]
    diff, mean_f1 = utility_difference(train, test, train.copy(), "label", ["cat"], verbose=False)
    assert diff.shape == (4, 2)                  # LR / DT / RF / MLP x (accuracy, weighted F1)
    assert np.allclose(diff, 0.0) and mean_f1 == pytest.approx(0.0)
    noise = train.copy()
    noise["label"] = rng.permutation(noise["label"].values)   # labels unrelated to the features
    diff2, mean2 = utility_difference(train, test, noise, "label", ["cat"], verbose=False)
    assert mean2 > 0.05
