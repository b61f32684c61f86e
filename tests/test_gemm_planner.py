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
        assert tile == 32 and 1 < n <= GEMM_MAX_SPLITS
        assert -(-K // n) <= 128 * 27       # was 83 bursts per split for D0 of the wide table
