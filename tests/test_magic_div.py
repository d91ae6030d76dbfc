"""CPU: exact division by the launch's runtime divisors (kernels.h
MagicDiv / magic_div, used by the path and stream kernels for tiles_x,
num_slots and batch): q = mulhi(n, m) >> sh equals n // d for every n < 2^31.
The check runs through libmrt itself (test entry mrt_debug_magic_div: the
compiled magic_div and the kernels' mulhi + shift restated in kernels.h, the
same functions draw_n checks every launch's divisors with), over every
divisor up to 4096 at the numerators where the floor changes (k d - 1, k d)
near 0 and near 2^31, and random divisors up to 2^31 (num_slots is owned
tiles x 4096)."""
import numpy as np

from helpers import SEED

TOP = (1 << 31) - 1


def _check(mrt_mod, d, ns):
    ns = np.array(sorted(set(n for n in ns if 0 <= n <= TOP)), np.uint32)
    q = mrt_mod.debug_magic_div(d, ns)
    want = ns.astype(np.uint64) // d
    bad = np.nonzero(q != want)[0]
    assert len(bad) == 0, (d, ns[bad[:5]], q[bad[:5]], want[bad[:5]])


def test_small_divisors_at_every_floor_step(mrt_mod):
    for d in range(1, 4097):
        k_top = TOP // d
        ns = [0, 1, d - 1, d, d + 1, 2 * d - 1, 2 * d, TOP, TOP - 1]
        ns += [k * d + e for k in (k_top - 1, k_top) for e in (-1, 0)]
        ns += list(range(0, min(TOP, 64 * d), max(1, d // 3)))
        _check(mrt_mod, d, ns)


def test_random_divisors(mrt_mod):
    rng = np.random.default_rng(SEED)
    for d in list(rng.integers(2, 1 << 31, 2000)) + [4096 * k for k in (1, 2, 3, 255, 510, 2040)]:
        d = int(d)
        ns = [int(x) for x in rng.integers(0, TOP, 200)] + [TOP, TOP // d * d, TOP // d * d - 1, d - 1, d]
        _check(mrt_mod, d, ns)


def test_zero_divisor_rejected(mrt_mod):
    import pytest
    with pytest.raises(mrt_mod.MrtError):
        mrt_mod.debug_magic_div(0, [1, 2])
