"""GEMM tile / split-K planner (host-side, no GPU)."""
def test_split_planner_keeps_bursts_per_split_bounded():
    """Long-K skinny GEMMs split until each slice is at most ~8 K-bursts (capped by the slab
    budget and the epilogue's 64 slabs); the measured Intrusion plans stay as they were."""
    from fed_tgan_amd.ops.hip import GEMM_MAX_SPLITS, _effective_splits, _plan
    assert _plan(150, 256, 6280) == (32, 13) and _plan(50, 256, 6280) == (32, 25)
    assert _plan(1000, 256, 431) == (32, 1)
    for M, K in ((150, 137800), (50, 137800), (1000, 6890)):
        tile, sk = _plan(M, 256, K)
        n = _effective_splits(K, sk, 128)
        # (plenty of workgroups at this K: 64-tiles, which re-read the long operands half as often)
        assert tile == 64 and 1 < n <= GEMM_MAX_SPLITS
        assert -(-K // n) <= 128 * 27       # was 83 bursts per split for D0 of the wide table


def test_planner_counts_clients_of_a_batched_launch():
    """A batched multi-client launch fills the chip with clients x tiles: less split-K for the same shape,
    and no 128-row tiles over fewer than 128 rows."""
    from fed_tgan_amd.ops.hip import _plan
    t1, s1 = _plan(150, 256, 5860)
    t2, s2 = _plan(150, 256, 5860, clients=2)
    t8, s8 = _plan(150, 256, 5860, clients=8)
    assert t1 == t2 == t8 == 32 and s8 < s2 < s1
    assert _plan(50, 5860, 256, clients=8)[0] != 128
    assert _plan(40000, 256, 658)[0] == 128
    # D0's weight gradient (K = the 150 stacked rows): 64-tiles for one client, 128-tiles for 8
    assert _plan(256, 6200, 150) == (64, 1)
    assert _plan(256, 6200, 150, clients=8) == (128, 1)
