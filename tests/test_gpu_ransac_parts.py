"""findEssentialMat's RANSAC pieces on the device against their sequential
restatement (visual_odometry_v3.py:297 -> ptsetreg.cpp
RANSACPointSetRegistrator::run): the subsets getSubset draws from
cv::RNG((uint64)-1) (wave-parallel assembly with rejection redraws), and the
best-model / niters / stop bookkeeping over per-hypothesis model counts
(event-parallel replay).  Bit-exact, including rounds past the 1024-hypothesis
replay chunk."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m", [6, 7, 9, 50, 871, 5000])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4096])
def test_subsets_equal_get_subset(gpu_ctx, oracle_mod, m, n):
    from droplet_visual_odometry_amd import ops
    np.testing.assert_array_equal(ops.test_ransac_subsets(m, n, ctx=gpu_ctx), oracle_mod.ransac_subsets(m, n))


def _counts(rng, n, m, regime):
    nmod = rng.choice([0, 1, 1, 1, 2, 3, 4, 10], n).astype(np.int32)
    if regime == "rising":      # slowly improving models: many events, niters shrinking late
        base = np.minimum(m, (np.arange(n) * m // (2 * n)) + rng.integers(0, 5, n))
        cnt = np.clip(base[:, None] + rng.integers(-3, 4, (n, 10)), 0, m)
    elif regime == "early":     # a very good model early: niters collapses
        cnt = rng.integers(0, m // 4, (n, 10))
        cnt[3, 0] = int(0.9 * m)
    elif regime == "flat":      # nothing beats 4: no event at all
        cnt = rng.integers(0, 5, (n, 10))
    else:                       # ties and plateaus
        cnt = rng.choice([3, 10, 50, 50, 51, m // 2], (n, 10))
    return nmod, cnt.astype(np.int32)


@pytest.mark.parametrize("regime", ["rising", "early", "flat", "ties"])
@pytest.mark.parametrize("n,max_iters", [(5, 1000), (64, 1000), (936, 1000), (1024, 4096), (1500, 4096),
                                         (4096, 4096)])
def test_replay_equals_sequential_loop(gpu_ctx, oracle_mod, regime, n, max_iters):
    from droplet_visual_odometry_amd import ops
    for seed in range(3):
        rng = np.random.default_rng(seed * 100 + n)
        m = int(rng.integers(6, 3000))
        nmod, cnt = _counts(rng, n, m, regime)
        want = oracle_mod.ransac_replay(nmod, cnt, m, 0.999, max_iters)
        got = ops.test_ransac_replay(nmod, cnt, m, 0.999, max_iters, ctx=gpu_ctx)
        assert got == want, (seed, m, got, want)
