"""calc_dag_score (astar/calc_dag_score.cpp): the drop-in command against the
oracle's restatement and the reference's Figure 3/4 fixtures (edge counts,
CPU), and the GPU-batched scores against the oracle's list scans (GPU)."""
import csv
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG
import synth

CDS = os.path.join(PKG, "bin", "calc_dag_score")
FIG3 = os.path.join(GOLDEN, "fig3")


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return r.stdout


def _parse(out):
    toks = out.split()
    res, i = [], 0
    while i < len(toks):
        name, score, _, edges = toks[i:i + 4]
        i += 4
        rm = None
        if i < len(toks) and toks[i] == "remove":
            rm = int(toks[i + 1])
            i += 2
        res.append((name, score, int(edges), rm))
    return res


def test_fig3_edges_match_fig4_without_scores(oracle_built, tmp_path):
    rows = list(csv.DictReader(open(os.path.join(GOLDEN, "fig4_edge_true_astar_ges_10k_group2_lambda1.csv"))))
    files = [os.path.join(FIG3, f"astar2_N10000_{r['seqnum']}.csv") for r in rows]
    missing = str(tmp_path / "none.pss")
    out = _run([CDS, missing] + files)
    ref = _run([oracle_built.REF_DAGSCORE, missing] + files)
    assert out == ref
    got = _parse(out)
    assert [g[0] for g in got] == [f"ASTAR2_N10000_{r['seqnum']}" for r in rows]
    assert [g[2] for g in got] == [int(r["astar_edges"]) for r in rows]
    assert all(g[1] == "0.000000" for g in got)


def test_unreadable_model_counts_as_empty(tmp_path):
    out = _run([CDS, str(tmp_path / "none.pss"), os.path.join(FIG3, "astar2_N10000_9200.csv"),
                str(tmp_path / "nope.csv")])
    assert _parse(out)[1] == ("NOPE", "0.000000", 0, 0)


@pytest.mark.gpu
def test_gpu_scores_match_oracle(oracle_built, tmp_path):
    """Scores of the A* DAG, the generating DAG (both orientations), random
    DAGs and the empty DAG, from a .pss the oracle wrote: the product's
    batched GPU lookups print exactly the oracle's line."""
    o = oracle_built
    n = 12
    X, W = synth.gaussian_sem(n, 3000, 9500)
    data = tmp_path / "d.csv"
    synth.write_csv(str(data), X)
    pss = tmp_path / "s.pss"
    subprocess.run([o.REF_SCORE, str(data), str(pss), "-f", "cBIC", "--lambda", "1", "-p", "4"], check=True,
                   stdout=subprocess.DEVNULL)
    net = tmp_path / "astar_net"
    subprocess.run([o.REF_ASTAR, str(pss), "-n", str(net)], check=True, stdout=subprocess.DEVNULL)
    dags = [str(net) + ".csv"]
    rng = np.random.default_rng(1)
    mats = {"true_dag": (W != 0).astype(int), "true_dag_t": (W != 0).astype(int).T,
            "empty": np.zeros((n, n), dtype=int)}
    for r in range(4):
        M = np.tril((rng.random((n, n)) < 0.2).astype(int), -1)
        perm = rng.permutation(n)
        mats[f"random_{r}"] = M[perm][:, perm]
    for name, M in mats.items():
        p = tmp_path / f"{name}.csv"
        np.savetxt(p, M, fmt="%d", delimiter=",")
        dags.append(str(p))
    out = _run([CDS, str(pss)] + dags)
    ref = _run([o.REF_DAGSCORE, str(pss)] + dags)
    assert out == ref
    got = _parse(out)
    assert got[0][0] == "ASTAR_NET" and float(got[0][1]) <= min(float(g[1]) for g in got[1:]) + 1e-3
