"""Federated statistics (vocab merge, JSD / W1 client distances, aggregation weights) vs the reference math."""
import numpy as np
import pytest
from scipy.spatial import distance
from scipy.stats import wasserstein_distance

from fed_tgan_amd.fed.stats import (aggregation_weights, jensenshannon, merge_categorical_metas,
                                    normalise_over_clients, softmax, uniform_weights, wasserstein_1d)


def test_jsd_matches_scipy():
    rng = np.random.default_rng(0)
    for _ in range(20):
        p, q = rng.random(7), rng.random(7)
        q[rng.integers(0, 7)] = 0
        assert jensenshannon(p, q) == pytest.approx(distance.jensenshannon(p, q), abs=1e-12)
        assert jensenshannon(p, q, 2.0) == pytest.approx(distance.jensenshannon(p, q, 2.0), abs=1e-12)


def test_w1_matches_scipy():
    rng = np.random.default_rng(1)
    for n, m in ((10, 10), (100, 37), (1000, 2000)):
        u, v = rng.normal(size=n), rng.normal(1, 2, size=m)
        assert wasserstein_1d(u, v) == pytest.approx(wasserstein_distance(u, v), rel=1e-10)


def _device_pool_case(dev):
    import torch
    from fed_tgan_amd.fed.stats import continuous_client_distances, continuous_client_distances_device
    rng = np.random.default_rng(2)
    parts = [[rng.normal(i, 1 + j, size=n) for j in range(3)] for i, n in enumerate((500, 1300, 40))]
    pooled = [np.concatenate([p[j] for p in parts]) for j in range(3)]
    off = np.concatenate([[0], np.cumsum([len(p[0]) for p in parts])]).tolist()
    want = continuous_client_distances(pooled, parts)
    got = continuous_client_distances_device(torch.as_tensor(np.stack(pooled), device=dev), off)
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12)


def test_w1_rows_and_device_distances_match_numpy():
    """The batched device W1 (sort + merged grid, fed/stats.py) = the numpy/SciPy one per row."""
    import torch
    from fed_tgan_amd.fed.stats import wasserstein_1d_rows
    rng = np.random.default_rng(3)
    u, v = rng.normal(size=(4, 900)), rng.gamma(2.0, size=(4, 333))
    got = wasserstein_1d_rows(torch.as_tensor(u), torch.as_tensor(v)).numpy()
    np.testing.assert_allclose(got, [wasserstein_distance(a, b) for a, b in zip(u, v)], rtol=1e-10)
    _device_pool_case("cpu")


@pytest.mark.gpu
def test_device_distances_on_gpu():
    _device_pool_case("cuda:0")


def test_sample_pool_layout_and_moments():
    """sample_pool: client i's draws of column j sit in columns off[i]:off[i+1] of row j, with that
    client's mixture moments."""
    from fed_tgan_amd.features.gmm import VGMBank, sample_pool
    k = 10

    def bank(mu):
        a = np.full((2, k), 1.0)
        w = np.zeros((2, k))
        w[:, :2] = [[5.0, 1e-9], [2.0, 2.0]]
        means = np.zeros((2, k))
        means[:, 0], means[:, 1] = mu, mu + 4
        return VGMBank(w + 1e-12, a, a, means, a + 5, np.full((2, k), 0.25))
    banks = [bank(0.0), bank(10.0)]
    pool, off = sample_pool(banks, [20000, 5000], np.random.default_rng(0), "cpu", seed=1)
    assert tuple(pool.shape) == (2, 25000) and off == [0, 20000, 25000]
    p = pool.numpy()
    for i, b in enumerate(banks):
        for j in range(2):
            x = p[j, off[i]:off[i + 1]]
            w = b.weights[j]
            mean = float(np.sum(w * b.means[j]))
            assert abs(x.mean() - mean) < 0.05, (i, j)


def _meta(counts):
    return {"columns": [{"column_name": "c", "type": "categorical", "i2s": counts},
                        {"column_name": "x", "type": "continous"}]}


def test_vocab_merge_order_and_weights():
    m1 = _meta({"a": 5, "b": 3})
    m2 = _meta({"b": 6, "c": 1})
    merged, vocabs, d_hat = merge_categorical_metas([m1, m2])
    assert merged["columns"][0]["i2s"] == ["b", "a", "c"]       # by global frequency
    assert vocabs[0].tolist() == ["a", "b", "c"]                # label codes alphabetical
    glob = np.array([5, 9, 1.0])
    d1 = distance.jensenshannon(glob, [5, 3, 0])
    d2 = distance.jensenshannon(glob, [0, 6, 1])
    assert d_hat[:, 0] == pytest.approx([d1 / (d1 + d2), d2 / (d1 + d2)])


def test_identical_clients_uniform():
    m = _meta({"a": 5, "b": 3})
    _, _, d_hat = merge_categorical_metas([m, m, m])
    assert np.allclose(d_hat, 1.0 / 3)                         # all-zero column -> 1/K
    e_hat = normalise_over_clients(np.zeros((3, 2)), zero_fill_uniform=False)
    w = aggregation_weights(d_hat, e_hat, [100, 100, 100])
    assert np.allclose(w, 1.0 / 3)


def test_aggregation_weight_formula():
    d_hat = np.array([[0.2, 0.5], [0.8, 0.5]])
    e_hat = np.array([[0.3], [0.7]])
    rows = [300, 100]
    s = e_hat.sum(1) + d_hat.sum(1)
    raw = (1 - s / s.sum()) * np.array([0.75, 0.25])
    assert aggregation_weights(d_hat, e_hat, rows) == pytest.approx(np.exp(raw) / np.exp(raw).sum())
    assert softmax(np.array([0.0, 0.0])) == pytest.approx([0.5, 0.5])
    assert uniform_weights(4) == pytest.approx([0.25] * 4)


def test_unequal_client_aggregate_matches_reference():
    """The unequal-client FedAvg against the reference's own code.  Fixture
    tests/golden/unequal_agg.npz (tools/make_unequal_fixture.py): the reference's MDGANClient.train_model(1) on the
    Adult Dirichlet(0.3) split's two clients (11 and 20 steps per epoch), their state dicts, the federator's
    distances and weights (`Server/dtds/distributed.py:767-783`) and its aggregate (`average_model`, `:86-106`,
    loaded into the generator as at `:811`).  This framework's weights (fed/stats.py) and its aggregation
    (FedRuntime.aggregate: one pre-scaled all-reduce of the flat buffer -- every parameter AND the BatchNorm running
    statistics -- plus num_batches_tracked = the truncated weighted sum of 2 x steps) must give the same model."""
    import os
    import threading

    import torch

    from fed_tgan_amd.features.transformer import SpanLayout
    from fed_tgan_amd.fed.local import LocalGroup, ThreadComm
    from fed_tgan_amd.fed.runtime import FedRuntime
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig

    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "unequal_agg.npz"))
    w = aggregation_weights(fx["d_hat"], fx["e_hat"], fx["rows"])
    np.testing.assert_allclose(w, fx["weights"], rtol=1e-12)
    assert fx["steps"].tolist() == [11, 20]
    info = [(int(a), "tanh" if k == 0 else "softmax") for a, k in zip(fx["span_width"], fx["span_kind"])]
    dims = tuple(int(x) for x in fx["dims"])
    cfg = EngineConfig(gen_dims=dims, dis_dims=dims)
    k = 2
    engines = []
    for i in range(k):
        e = CTGANEngine(SpanLayout.from_output_info(info), cfg, "cpu", backend="torch", seed=100 + i)
        e.load_g_state_dict({key: torch.from_numpy(fx[f"G{i}|{key}"]) for key in fx["G_keys"]})
        e.load_d_state_dict({key: torch.from_numpy(fx[f"D{i}|{key}"]) for key in fx["D_keys"]})
        assert e.bn_batches == 2 * int(fx["steps"][i])
        engines.append(e)
    group = LocalGroup(k)

    class _Cfg:
        phase_detail = False

    def client(i):
        rt = FedRuntime.__new__(FedRuntime)
        rt.cfg, rt.comm, rt.engine = _Cfg(), ThreadComm(group, i, torch.device("cpu")), engines[i]
        rt.weights, rt.is_client, rt.is_fed, rt.federator = w, True, i == 0, 0
        rt.steps, rt._epoch_done, rt._pipe = [int(s) for s in fx["steps"]], 1, False
        rt.aggregate()

    ts = [threading.Thread(target=client, args=(i,)) for i in range(k)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in engines:
        got_g, got_d = e.g_state_dict(), e.d_state_dict()
        for key in fx["G_keys"]:
            want = fx[f"Gagg|{key}"]
            if key.endswith("num_batches_tracked"):
                assert int(got_g[key]) == int(want) == 32          # int(0.4307 * 22 + 0.5693 * 40)
            else:
                np.testing.assert_allclose(got_g[key].numpy(), want, rtol=2e-6, atol=1e-7, err_msg=key)
        for key in fx["D_keys"]:
            np.testing.assert_allclose(got_d[key].numpy(), fx[f"Dagg|{key}"], rtol=2e-6, atol=1e-7, err_msg=key)
