"""The list packing of the bit-sliced walk (cbic_dev.h walk_sliced, round 6).

find_best_subset_score (BIC_OLS.cpp:125-172) passes each call a
parent list: the caller's entries other than the removed one u, in order,
the first j of them for the j-th call, zero-padded to the callee's length
(the zero-initialised vector, N3).  walk_sliced packs a node's entries other
than u once per expansion instead of testing every entry per call.  The
packing relies on the lists' shape: an optional leading 0 (variable 0, a
member of P in phase 0), then distinct nonzero entries, then zero padding.
This test walks every list the recursion can build for layers 1..8, both
phases (data-independent: every call is taken), checks the shape, and checks
the device code's packing (restated in `_packed`) against the generic one.
"""
import pytest


def _packed(pv, M, idx):
    """cbic_dev.h walk_sliced, ULG_WALK_LOOPCOND 2: (rest, cnt) from the
    4-bit entries of pv, with u = entry idx."""
    u = (pv >> (4 * idx)) & 15
    if u != 0:
        lo = (1 << (4 * idx)) - 1
        return ((pv & lo) | ((pv >> 4) & ~lo)) & 0xFFFFFFFF, M - 1
    lm = 0xFFFFFFFF if M >= 8 else (1 << (4 * M)) - 1
    nz = (pv | (pv >> 1) | (pv >> 2) | (pv >> 3)) & 0x11111111 & lm
    return (pv >> 4 if (pv & 15) == 0 else pv), bin(nz).count("1")


def _entries(pv, M):
    return [(pv >> (4 * i)) & 15 for i in range(M)]


def _shape_ok(lst):
    i = 1 if lst and lst[0] == 0 else 0
    nz = []
    while i < len(lst) and lst[i] != 0:
        nz.append(lst[i])
        i += 1
    return all(x == 0 for x in lst[i:]) and len(set(nz)) == len(nz)


def _walk(pv, M, lo, hi, seen):
    if (pv, M, lo, hi) in seen:
        return 0
    seen.add((pv, M, lo, hi))
    lst = _entries(pv, M)
    assert _shape_ok(lst), lst
    n = 0
    for idx in range(lo, hi):
        if M == 1:
            continue
        u = lst[idx]
        gen = [p for p in lst if p != u]
        rest, cnt = _packed(pv, M, idx)
        assert cnt == len(gen), (lst, idx)
        assert _entries(rest, cnt) == gen, (lst, idx)
        for j in range(1, cnt + 1):
            npv = rest & ((1 << (4 * j)) - 1)
            clo, chi = (0, min(M - 1, 2)) if j == 1 else (j - 1, j)
            n += 1 + _walk(npv, M - 1, clo, chi, seen)
    return n


@pytest.mark.parametrize("L", range(1, 9))
@pytest.mark.parametrize("phase", [0, 1])
def test_walk_list_packing_every_list(L, phase):
    first = 0 if phase == 0 else 1
    pvtop = 0
    for i in range(L):
        pvtop |= (i + first) << (4 * i)
    calls = _walk(pvtop, L, 0, L, set())
    assert calls >= 0
