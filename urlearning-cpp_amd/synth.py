"""Seeded synthetic inputs for the cBIC + A* path.

The reference's own generators (score/generate_chain.cpp:86) seed from the
wall clock, so the benchmark and the tests use this seeded linear-Gaussian
structural equation model instead: random topological order, edge i->j with
probability 2d/(n-1) (d = 2), weights +-U[0.5, 1.5], noise N(0, 1).
"""
from __future__ import annotations

import numpy as np


def gaussian_sem(n: int, N: int, seed: int, d: float = 2.0):
    """Returns (X [N x n] float64, W [n x n] with W[i, j] != 0 iff i -> j)."""
    rng = np.random.default_rng(seed)
    order = rng.permutation(n)
    p = min(1.0, 2.0 * d / max(n - 1, 1))
    W = np.zeros((n, n))
    for a in range(n):
        for b in range(a + 1, n):
            if rng.random() < p:
                W[order[a], order[b]] = rng.uniform(0.5, 1.5) * (1.0 if rng.random() < 0.5 else -1.0)
    X = np.zeros((N, n))
    for j in order:
        X[:, j] = X @ W[:, j] + rng.standard_normal(N)
    return X, W


def full_skeleton(n: int):
    """n x n all-ones matrix (README.md:16-24): every variable a candidate."""
    allm = (1 << n) - 1
    return [allm] * n


def true_skeleton_edges(W: np.ndarray, extra_frac: float = 0.0, seed: int = 0):
    """Symmetric skeleton rows (bit j of row i = edge i-j) from the true DAG,
    plus extra_frac * |E| random extra edges (the C4 stand-in for MMPC)."""
    n = W.shape[0]
    A = (W != 0) | (W.T != 0)
    if extra_frac > 0:
        rng = np.random.default_rng(seed)
        extra = int(round(extra_frac * A.sum() / 2))
        while extra > 0:
            i, j = rng.integers(0, n, 2)
            if i != j and not A[i, j]:
                A[i, j] = A[j, i] = True
                extra -= 1
    rows = []
    for i in range(n):
        r = 1 << i  # the reference's matrices carry the diagonal (README.md:16-24)
        for j in range(n):
            if A[i, j]:
                r |= 1 << j
        rows.append(r)
    return rows


def write_csv(path: str, X: np.ndarray):
    np.savetxt(path, X, fmt="%.17g", delimiter=",")


def write_skeleton(path: str, rows, n: int):
    with open(path, "w") as f:
        for i in range(n):
            f.write(",".join("1" if (rows[i] >> j) & 1 else "0" for j in range(n)) + "\n")
