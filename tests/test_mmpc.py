"""The MMPC skeleton producer (ulg_mmpc / bin/mmpc).  The reference takes the
skeleton from outside (README.md:16), so parity is unpinned: the HIP driver
is checked against the oracle's restatement of the same rules
(oracle/ora_mmpc.c), and the oracle against the independences a chain and
a collider imply."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG
import synth

MMPC = os.path.join(PKG, "bin", "mmpc")


def test_norm_quantile(oracle_built):
    L = oracle_built.lib()
    assert abs(L.ora_norm_quantile(0.975) - 1.959963984540054) < 1e-12
    assert abs(L.ora_norm_quantile(0.995) - 2.5758293035489004) < 1e-12
    assert abs(L.ora_norm_quantile(0.5)) < 1e-15


def test_oracle_chain_and_collider(oracle_built):
    """x0 -> x1 -> x2 (x0 _||_ x2 | x1) and x3 -> x5 <- x4 (x3 _||_ x4)."""
    rng = np.random.default_rng(0)
    N = 20000
    x0 = rng.standard_normal(N)
    x1 = 0.9 * x0 + rng.standard_normal(N)
    x2 = 0.9 * x1 + rng.standard_normal(N)
    x3 = rng.standard_normal(N)
    x4 = rng.standard_normal(N)
    x5 = 0.8 * x3 - 0.8 * x4 + rng.standard_normal(N)
    rows = oracle_built.Dataset(np.stack([x0, x1, x2, x3, x4, x5], 1)).mmpc(0.01)
    edges = {(i, j) for i in range(6) for j in range(6) if i < j and (rows[i] >> j) & 1}
    assert edges == {(0, 1), (1, 2), (3, 5), (4, 5)}


def test_oracle_skeleton_shape(oracle_built):
    X, _ = synth.gaussian_sem(15, 4000, 9810)
    rows = oracle_built.Dataset(X).mmpc(0.05)
    for i in range(15):
        assert not (rows[i] >> i) & 1
        for j in range(15):
            assert ((rows[i] >> j) & 1) == ((rows[j] >> i) & 1)


def test_cli_help():
    r = subprocess.run([MMPC, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--alpha" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,N,alpha,max_cond", [
    (9811, 12, 2000, 0.05, -1), (9812, 20, 5000, 0.01, -1), (9813, 20, 5000, 0.05, 2),
    (9814, 30, 100000, 0.01, -1), (9815, 30, 20000, 0.05, 3)])
def test_gpu_mmpc_matches_oracle(ulg_ctx, oracle_built, seed, n, N, alpha, max_cond):
    X, _ = synth.gaussian_sem(n, N, seed)
    ulg_ctx.load(X, 2.0)
    got = ulg_ctx.mmpc(alpha, max_cond)
    ref = oracle_built.Dataset(X).mmpc(alpha, max_cond)
    assert got == ref


@pytest.mark.gpu
def test_cli_mmpc_feeds_score_and_astar(tmp_path, oracle_built):
    """mmpc -> score -k -> astar -k: the C4 pipeline shape (n=30, N=100k) at k=4."""
    X, _ = synth.gaussian_sem(30, 100000, 9816)
    data = tmp_path / "d.csv"
    synth.write_csv(str(data), X)
    skel = tmp_path / "skel.csv"
    r = subprocess.run([MMPC, str(data), str(skel), "--alpha", "0.01"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    M = np.loadtxt(skel, delimiter=",", dtype=int)
    ref = oracle_built.Dataset(X).mmpc(0.01)
    assert [int(sum(int(b) << j for j, b in enumerate(row))) for row in M] == ref
    pss = tmp_path / "s.pss"
    r = subprocess.run([os.path.join(PKG, "bin", "score"), str(data), str(pss), "-f", "cBIC", "--lambda", "2",
                        "-p", "4", "-k", str(skel)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    net = tmp_path / "net"
    r = subprocess.run([os.path.join(PKG, "bin", "astar"), str(pss), "-k", str(skel), "-n", str(net)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    ref_net = tmp_path / "ref_net"
    subprocess.run([oracle_built.REF_ASTAR, str(pss), "-k", str(skel), "-n", str(ref_net)], check=True,
                   stdout=subprocess.DEVNULL)
    assert net.read_text() == ref_net.read_text()
