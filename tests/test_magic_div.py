"""CPU: exact division by the launch's runtime divisors (kernels.h
MagicDiv / magic_div, used by the path and stream kernels for tiles_x,
num_slots and batch): q = mulhi(n, m) >> sh equals n // d for every n < 2^31.
The restatement below follows magic_div line by line; the check covers every
divisor up to 4096 against the numerators where the floor changes (k d - 1,
k d) near 0 and near 2^31, and random divisors up to 2^31 (num_slots is
owned tiles x 4096)."""
import numpy as np

from helpers import SEED


def magic_div(d):
    if d <= 1:
        return 0, 0
    l = 0
    while (1 << l) < d:
        l += 1
    p = 1 << (31 + l)
    return (p + d - 1) // d, l - 1


def mdiv(n, m, sh):
    return n if m == 0 else ((n * m) >> 32) >> sh


def _check(d, ns):
    m, sh = magic_div(d)
    assert m < 1 << 32
    for n in ns:
        assert mdiv(n, m, sh) == n // d, (d, n, m, sh)


def test_small_divisors_at_every_floor_step():
    top = (1 << 31) - 1
    for d in range(1, 4097):
        k_top = top // d
        ns = [0, 1, d - 1, d, d + 1, 2 * d - 1, 2 * d, top, top - 1]
        ns += [k * d + e for k in (k_top - 1, k_top) for e in (-1, 0) if 0 <= k * d + e <= top]
        _check(d, ns)


def test_random_divisors():
    rng = np.random.default_rng(SEED)
    top = (1 << 31) - 1
    for d in list(rng.integers(2, 1 << 31, 2000)) + [4096 * k for k in (1, 2, 3, 255, 510, 2040)]:
        d = int(d)
        ns = [int(x) for x in rng.integers(0, top, 50)] + [top, top // d * d, top // d * d - 1, d - 1, d]
        _check(d, [n for n in ns if 0 <= n <= top])
