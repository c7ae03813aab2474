"""unrank_colex (csrc/cbic_dev.h): element i of the set with colex rank r is
the largest c with C(c, i) <= r below the previous element.  The kernel
estimates it as e = floor((r i!)^(1/i) + (i-1)/2) + 1 in float32, reads
C(e+1, i) (guard), C(e, i), C(e-1, i), C(e-2, i) at once, and falls back to
the table scan when the guard fires or none of the three fits -- so lists
never depend on the estimate, only the speed does.  This test restates the
arithmetic in numpy float32 and checks, at every boundary rank C(c, i) and
C(c+1, i) - 1 for c < 64, i <= 8 (the largest and smallest r with answer c),
that the answer lies in [e - 2, e]: the fast path covers them all, and a
full unrank with the fallback equals the plain scan."""
import math

import numpy as np

FACT = [1, 1, 2, 6, 24, 120, 720, 5040, 40320]


def estimate(r, i, c_hi):
    if i == 1:
        return min(r, c_hi)
    x = np.float32(r) * np.float32(FACT[i])
    lg = np.log2(x) if x > 0 else np.float32(-np.inf)
    g = np.exp2(np.float32(lg) * np.float32(1.0 / i)).astype(np.float32)
    e = int(np.float32(g + np.float32(0.5 * (i - 1)))) + 1
    return max(min(e, c_hi), i - 1)


def unrank(r, l, U):
    mask, c = 0, U - 1
    for i in range(l, 0, -1):
        e = estimate(r, i, c)
        low = e < c and math.comb(e + 1, i) <= r
        cands = [x for x in (e, e - 1, e - 2) if x >= 0 and math.comb(x, i) <= r]
        cc = cands[0] if cands and not low else None
        if cc is None:
            cc = c if low else e - 3
            while cc >= 0 and math.comb(cc, i) > r:
                cc -= 1
        mask |= 1 << cc
        r -= math.comb(cc, i)
        c = cc - 1
    return mask


def unrank_scan(r, l, U):
    mask, c = 0, U - 1
    for i in range(l, 0, -1):
        while c >= 0 and math.comb(c, i) > r:
            c -= 1
        mask |= 1 << c
        r -= math.comb(c, i)
        c -= 1
    return mask


def test_estimate_brackets_every_boundary_rank():
    for i in range(1, 9):
        for c in range(i - 1, 64):
            for r in {math.comb(c, i), math.comb(c + 1, i) - 1}:
                e = estimate(r, i, 63)
                assert e - 2 <= c <= e, (i, c, r, e)


def test_unrank_equals_scan():
    rng = np.random.default_rng(5)
    for _ in range(3000):
        U = int(rng.integers(1, 64))
        l = int(rng.integers(0, min(8, U) + 1))
        r = int(rng.integers(0, math.comb(U, l)))
        assert unrank(r, l, U) == unrank_scan(r, l, U)
