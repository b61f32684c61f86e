"""Initialisation-path HIP kernels (csrc/kernels/init_ops.hip) against their torch / numpy formulations: the CSR
real-row index of an encoded table (`Server/dtds/synthesizers/ctgan.py:205-217`), the federator's pooled GMM sample
(`Server/dtds/distributed.py:731-735`) and the fit's row centring."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


class _Layout:
    def __init__(self, widths):
        self.cond_width = np.asarray(widths, dtype=np.int32)
        self.n_col = len(widths)


@pytest.mark.parametrize("n", [1, 300, 10000])
def test_csr_rows_matches_torch_index(n):
    from fed_tgan_amd.features.encode_gpu import row_index_on_device, row_index_torch
    from fed_tgan_amd.ops import native
    native.require()
    rng = np.random.default_rng(n)
    widths = [1, 2, 7, 64, 301, 3]
    # skewed options (many repeats inside every 256-row batch) and unused options
    opt = np.stack([np.minimum(rng.geometric(0.3, n) - 1, w - 1) for w in widths], axis=1).astype(np.int32)
    opt[:, 4] = np.where(opt[:, 4] % 3 == 0, opt[:, 4], 299)
    lay = _Layout(widths)
    t = torch.as_tensor(opt, device=DEV)
    got, cnt = row_index_on_device(t, lay)
    want, cnt_w = row_index_torch(t, lay)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(cnt, cnt_w)
    for k in ("row_offset", "row_count", "rows"):
        assert torch.equal(got[k], want[k]), k
    again, _ = row_index_on_device(t, lay)
    assert torch.equal(again["rows"], got["rows"])           # deterministic


def test_pool_sample_layout_and_moments():
    from fed_tgan_amd.features.gmm import VGMBank, sample_pool
    from fed_tgan_amd.ops import native
    native.require()
    K = 10

    def bank(mu):
        w = np.zeros((2, K))
        w[:, :2] = [[0.3, 0.7], [0.5, 0.5]]
        a = 1 + w * 1e4
        b = 1e-3 + (1 - np.cumsum(w, axis=1)) * 1e4
        means = np.tile(np.arange(K, dtype=np.float64) * 10 + mu, (2, 1))
        return VGMBank(wc_a=a, wc_b=b, mean_precision=np.ones((2, K)), means=means, dof=np.ones((2, K)) * 3,
                       covariances=np.full((2, K), 0.25))
    banks = [bank(0.0), bank(1000.0)]
    pool, off = sample_pool(banks, [30000, 10000], np.random.default_rng(0), DEV, seed=3)
    p = pool.cpu().numpy()
    assert p.shape == (2, 40000) and off == [0, 30000, 40000]
    a, b = p[:, :30000], p[:, 30000:]
    assert (a < 500).all() and (b > 500).all()                    # client blocks in order
    for blk, mu in ((a, 0.0), (b, 1000.0)):
        lo = blk[blk < mu + 5]                                      # component 0: mean mu, sd 0.5
        assert abs(lo.mean() - mu) < 0.02 and abs(lo.std() - 0.5) < 0.02
    pool2, _ = sample_pool(banks, [30000, 10000], np.random.default_rng(0), DEV, seed=3)
    assert torch.equal(pool, pool2)


def test_row_center_matches_numpy():
    from fed_tgan_amd.ops import native
    L = native.require()
    x = torch.randn(5, 12345, dtype=torch.float64, device=DEV) * 3 + torch.arange(5, device=DEV, dtype=torch.float64)[:, None]
    ref = x.cpu().numpy()
    shift = torch.empty(5, dtype=torch.float64, device=DEV)
    L.row_center(x, shift)
    np.testing.assert_allclose(shift.cpu().numpy(), ref.mean(1), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(x.cpu().numpy(), ref - ref.mean(1, keepdims=True), rtol=1e-12, atol=1e-12)
