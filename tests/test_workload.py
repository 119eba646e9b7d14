"""Device workload generators (sherman_amd/workload.py) against the
reference's distributions (test/zipf.h via the oracle restatement), on CPU."""
import numpy as np
import torch

from oracle.pyoracle import zipf_fill
from sherman_amd.workload import Zipf, op_is_get, pow_approx, pow_approx_scalar, zeta


def _pow_approx_ref(a, b):
    # zipf.h:65-91 transcribed on numpy words (hi word interpolation)
    e = int(b)
    w = np.array([a], dtype=np.float64).view(np.int32).copy()
    w[1] = np.int32(int((b - e) * float(int(w[1]) - 1072632447) + 1072632447.0))
    w[0] = 0
    d = float(w.view(np.float64)[0])
    r = 1.0
    while e:
        if e & 1:
            r *= a
        a *= a
        e >>= 1
    return r * d


def test_pow_approx_restatement():
    xs = [1.0, 1.5, 2.0, 3.7, 1e-3, 0.5, 0.999, 12345.0]
    for b in (0.99, 0.01, 0.5, 100.0000000000001, 2.25):
        t = pow_approx(torch.tensor(xs, dtype=torch.float64), b).tolist()
        for x, y in zip(xs, t):
            r = _pow_approx_ref(x, b)
            assert y == r and pow_approx_scalar(x, b) == r, (x, b, y, r)


def test_zeta_matches_direct_sum():
    n, th = 10000, 0.99
    ref = sum(1.0 / _pow_approx_ref(float(i), th) for i in range(1, n + 1))
    assert abs(zeta(n, th, "cpu", chunk=777) - ref) < 1e-9 * ref


def test_zipf_distribution_matches_reference_generator():
    """Same n and theta: item frequencies of the bulk generator and of the
    reference's sequential mehcached generator agree within sampling noise."""
    n, th, count = 1 << 12, 0.99, 400000
    ref = zipf_fill(n, th, 12345, count).astype(np.int64)
    g = torch.Generator().manual_seed(7)
    ours = Zipf(n, th, "cpu").sample(count, g).numpy()
    assert ours.min() >= 0 and ours.max() < n
    for top in (0, 1, 2, 10):
        p_ref = np.mean(ref == top)
        p_ours = np.mean(ours == top)
        sd = np.sqrt(p_ref * (1 - p_ref) / count)
        assert abs(p_ref - p_ours) < 6 * sd + 2e-3, (top, p_ref, p_ours)
    # head mass (items < 64) and a tail quantile
    assert abs(np.mean(ref < 64) - np.mean(ours < 64)) < 0.01
    assert abs(np.quantile(ref, 0.9) - np.quantile(ours, 0.9)) <= 0.05 * n


def test_uniform_and_op_mix():
    g = torch.Generator().manual_seed(1)
    u = Zipf(1000, 0.0, "cpu").sample(100000, g).numpy()
    assert u.min() >= 0 and u.max() < 1000
    assert abs(u.mean() - 499.5) < 5
    m = op_is_get(100000, 50, "cpu", g)
    assert abs(m.float().mean().item() - 0.5) < 0.01
