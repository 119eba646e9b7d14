"""Device-side workload generators for the benchmark configs.

The reference benchmark draws `dis = mehcached_zipf_next(&state)` and uses
`key = to_key(dis)` (test/benchmark.cpp:165-173). The op is a GET iff
`rand_r(&seed) % 100 < kReadRatio` (benchmark.cpp:176).

Here the same distributions are drawn on the GPU in bulk:
  * zipf: J. Gray et al. (SIGMOD'94) exactly as test/zipf.h:163-203 computes
    it, including mehcached_pow_approx (zipf.h:65-91). That approximation
    reshapes the distribution noticeably: at theta 0.99, n = 4096, items 0
    and 1 get 14.7 % and 11.9 % instead of 11.1 % and 5.6 %. It is restated
    here bit for bit, so the skew matches the reference benchmark's.
    theta = 0 gives uniform (u64)(n * u), as zipf.h:185-187.
  * keys: to_key through the device CityHash64 (Tree.hash_keys).

These streams have the reference's distribution, not its exact sequence.
Parity tests that need the exact sequence take it from the oracle's bit-exact
restatement (tests/ only).
"""
import torch


def pow_approx_scalar(a, b):
    """mehcached_pow_approx (zipf.h:65-91) on one double."""
    import struct
    e = int(b)
    lo, hi = struct.unpack("<ii", struct.pack("<d", a))
    hi = int((b - e) * float(hi - 1072632447) + 1072632447.0)
    (d,) = struct.unpack("<d", struct.pack("<ii", 0, hi))
    r = 1.0
    while e:
        if e & 1:
            r *= a
        a *= a
        e >>= 1
    return r * d


def pow_approx(a, b):
    """mehcached_pow_approx on a float64 tensor of positive values, scalar b:
    exponent-field interpolation for frac(b), squaring for int(b)."""
    e = int(b)
    hi = a.view(torch.int64) >> 32
    hi = ((b - e) * (hi.to(torch.float64) - 1072632447.0) + 1072632447.0).to(torch.int64)
    d = (hi << 32).view(torch.float64)
    r = torch.ones_like(a)
    x = a.clone()
    while e:
        if e & 1:
            r = r * x
        x = x * x
        e >>= 1
    return r * d


def zeta(n, theta, device, chunk=1 << 24):
    """sum_{i=1..n} 1 / pow_approx(i, theta) in float64 (zipf.h:149-160)."""
    total = torch.zeros((), dtype=torch.float64, device=device)
    for lo in range(1, n + 1, chunk):
        i = torch.arange(lo, min(n + 1, lo + chunk), dtype=torch.float64, device=device)
        total += (1.0 / pow_approx(i, theta)).sum()
    return float(total)


class Zipf:
    """Draws item indices in [0, n) like mehcached_zipf_next (zipf.h:163-203)."""

    def __init__(self, n, theta, device):
        assert theta == 0.0 or 0.0 < theta < 1.0, "theta in {0} U (0, 1)"
        self.n, self.theta, self.device = n, theta, device
        if theta > 0.0:
            self.zetan = zeta(n, theta, device)
            self.alpha = 1.0 / (1.0 - theta)
            self.thres = 1.0 + pow_approx_scalar(0.5, theta)
            zeta2 = 1.0 + 1.0 / pow_approx_scalar(2.0, theta)
            self.eta = ((1.0 - pow_approx_scalar(2.0 / n, 1.0 - theta)) /
                        (1.0 - zeta2 / self.zetan))

    def sample(self, count, generator=None):
        u = torch.rand(count, dtype=torch.float64, device=self.device, generator=generator)
        if self.theta == 0.0:
            return (u * self.n).to(torch.int64)
        v = (self.n * pow_approx(self.eta * (u - 1.0) + 1.0, self.alpha)).to(torch.int64)
        uz = u * self.zetan
        v = torch.where(uz < self.thres, torch.ones_like(v), v)
        v = torch.where(uz < 1.0, torch.zeros_like(v), v)
        return v.clamp_(0, self.n - 1)


def op_is_get(count, read_ratio, device, generator=None):
    """GET iff r % 100 < read_ratio (benchmark.cpp:176), r uniform."""
    r = torch.randint(0, 100, (count,), device=device, generator=generator)
    return r < read_ratio
