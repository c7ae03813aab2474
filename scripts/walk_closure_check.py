#!/usr/bin/env python3
"""Checks walk_may_hit (csrc/cbic_dev.h) against find_best_subset_score's
recursion (BIC_OLS.cpp:125-172 as walk_sliced replays it: zero-padded parent
vector, XOR toggle, `checked`, the no-op re-tests skipped) on random
presence / hi patterns: every node the recursion tests lies in the closure's
tested set (P itself aside, never a key), so "no key >= -ts in the closure"
implies "the walk stores P".  The closure is restated here word by word
(64-bit words, the device's operations).

    python scripts/walk_closure_check.py [--trials 100000]
"""
import argparse
import random

M64 = (1 << 64) - 1
KM = [0xAAAAAAAAAAAAAAAA, 0xCCCCCCCCCCCCCCCC, 0xF0F0F0F0F0F0F0F0, 0xFF00FF00FF00FF00, 0xFFFF0000FFFF0000,
      0xFFFFFFFF00000000]


def walk(T, pv, M, present, hi, checked, tested, lo, hi_idx):
    """The recursion; returns True on a hit (the walk's decision: pruned)."""
    for idx in range(lo, hi_idx):
        u = (pv >> (4 * idx)) & 15
        T2 = T ^ (1 << u)
        tested.add(T2)
        if T2 in checked:
            continue
        if present[T2]:
            if hi[T2]:
                return True
            continue
        if M > 1:
            npv, j = 0, 0
            for i in range(M):
                pi = (pv >> (4 * i)) & 15
                if pi == u:
                    continue
                npv |= pi << (4 * j)
                j += 1
                if walk(T2, npv, M - 1, present, hi, checked, tested, 0 if j == 1 else j - 1,
                        (min(2, M - 1) if j == 1 else j)):
                    return True
                checked.add(T2)
    return False


def bits_words(L):
    return 1 if L + 1 <= 6 else 1 << (L + 1 - 6)


def walk_may_hit(L, phase, pres, hiw):
    """cbic_dev.h walk_may_hit on lists of W 64-bit words; also returns the tested words."""
    W = bits_words(L)
    Q = L if phase == 0 else L + 1
    root = (1 << L) - 1 if phase == 0 else ((1 << L) - 1) << 1

    def bitw(t, j):
        return 1 << (t & 63) if t >> 6 == j else 0
    absent, tested, reach = [0] * W, [0] * W, [0] * W
    for j in range(W):
        valid = (M64 if j < (1 << (Q - 6)) else 0) if Q >= 6 else ((1 << (1 << Q)) - 1 if j == 0 else 0)
        first = 0
        for b in (range(0, L) if phase == 0 else range(1, L + 1)):
            first |= bitw(root ^ (1 << b), j)
        notkey = bitw(root, j) | (bitw(root | 1, j) if phase == 1 else 0)
        absent[j] = ~pres[j] & valid & ~notkey & M64
        tested[j] = first
        reach[j] = first & absent[j]

    def closure():
        for j in range(W):
            c = (((reach[j] & 0x5555555555555555) << 1) | ((reach[j] & 0xAAAAAAAAAAAAAAAA) >> 1)) & M64
            tested[j] |= c
            reach[j] |= c & absent[j]
    closure()
    for e in range(L - 1 if phase == 0 else L, 0, -1):
        n = [0] * W
        for j in range(W):
            if e < 6:
                n[j] = (reach[j] & KM[e]) >> (1 << e)
            else:
                s = 1 << (e - 6)
                n[j] = reach[j + s] if j + s < W and ((j >> (e - 6)) & 1) == 0 else 0
        for j in range(W):
            tested[j] |= n[j]
            reach[j] |= n[j] & absent[j]
        closure()
    hit = False
    for j in range(W):
        notkey = bitw(root, j) | (bitw(root | 1, j) if phase == 1 else 0)
        tested[j] &= ~notkey & M64
        hit |= (tested[j] & hiw[j]) != 0
    return hit, tested


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=100000)
    ap.add_argument("--seed", type=int, default=5)
    a = ap.parse_args()
    random.seed(a.seed)
    bad = stored = proved = 0
    for _ in range(a.trials):
        L = random.randint(1, 6)
        phase = random.randint(0, 1)
        Q = L if phase == 0 else L + 1
        root = (1 << L) - 1 if phase == 0 else ((1 << L) - 1) << 1
        pp, ph = random.random(), random.random() * 0.3
        present = [random.random() < pp for _ in range(1 << Q)]
        hi = [present[t] and random.random() < ph for t in range(1 << Q)]
        for t in (0, root, root | 1):
            if t < (1 << Q):
                present[t] = hi[t] = False
        pvtop = 0
        for i in range(L):
            pvtop |= (i + (0 if phase == 0 else 1)) << (4 * i)
        tested = set()
        dom = walk(root, pvtop, L, present, hi, {0}, tested, 0, L)
        W = bits_words(L)
        pres = [sum(1 << (t & 63) for t in range(1 << Q) if present[t] and t >> 6 == j) for j in range(W)]
        hiw = [sum(1 << (t & 63) for t in range(1 << Q) if hi[t] and t >> 6 == j) for j in range(W)]
        may, tw = walk_may_hit(L, phase, pres, hiw)
        missing = [t for t in tested if t not in (0, root, root | 1) and not (tw[t >> 6] >> (t & 63)) & 1]
        if missing or (dom and not may):
            bad += 1
        if not dom:
            stored += 1
            proved += not may
    print(f"trials {a.trials}: violations {bad}; walk stores {stored}, the closure proves {proved} of them")
    raise SystemExit(1 if bad else 0)


if __name__ == "__main__":
    main()
