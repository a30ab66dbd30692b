"""On-device Philox normal / gamma variates (dc:104,126,142,150,158,163,170 sites):
moments and Kolmogorov-Smirnov against the exact distributions, at every gamma
shape the sweep uses, plus counter-addressing properties."""
import numpy as np
import pytest
from scipy import stats

pytestmark = pytest.mark.gpu

N = 200_000


def test_normal_moments_and_ks(dcfm):
    x = dcfm.rng_fill("normal", N, seed=123, site=1, shard=5, iteration=7)
    assert abs(x.mean()) < 5 / np.sqrt(N)
    assert abs(x.var() - 1) < 5 * np.sqrt(2 / N)
    assert stats.kstest(x, "norm").pvalue > 1e-4


@pytest.mark.parametrize("shape", [0.3, 0.75, 1.0, 1.5, 2.0, 3.5, 501.0, 4682.0])
def test_gamma_moments_and_ks(dcfm, shape):
    """Shapes below 1 (hyper-parameters other than dc:62-65's) come from the boost
    Ga(a) = Ga(a+1) U^(1/a)."""
    x = dcfm.rng_fill("gamma", N, seed=99, shape=shape, site=4, shard=2, iteration=3)
    assert np.all(x > 0)
    sd = np.sqrt(shape)
    assert abs(x.mean() - shape) < 5 * sd / np.sqrt(N)
    # sampling sd of the variance ratio: sqrt((excess kurtosis 6/a + 2) / N)
    assert abs(x.var() / shape - 1) < max(0.05, 6 * np.sqrt((6 / shape + 2) / N))
    assert stats.kstest(x, "gamma", args=(shape,)).pvalue > 1e-4


def test_counter_addressing(dcfm):
    a = dcfm.rng_fill("normal", 4096, seed=1, site=3, shard=0, iteration=1)
    b = dcfm.rng_fill("normal", 4096, seed=1, site=3, shard=0, iteration=1)
    c = dcfm.rng_fill("normal", 4096, seed=1, site=3, shard=1, iteration=1)
    e = dcfm.rng_fill("normal", 4096, seed=1, site=3, shard=0, iteration=2)
    f = dcfm.rng_fill("normal", 4096, seed=2, site=3, shard=0, iteration=1)
    assert np.array_equal(a, b)
    for o in (c, e, f):
        assert not np.array_equal(a, o)
        assert abs(np.corrcoef(a, o)[0, 1]) < 0.06
