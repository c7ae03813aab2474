"""CPU tests: the oracle against the reference's own golden fixtures, and
the oracle's internal invariants that the HIP design relies on."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, TRIPLET_SKELETON, fig_dag, fig_mec, load_fig, read_matrix

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "urlearning-cpp_amd"))
import synth  # noqa: E402


FIG_CSV = {1: "fig1_raw_data_8000.csv", 2: "fig2_raw_data_5000.csv"}


@pytest.mark.parametrize("fig", [1, 2])
@pytest.mark.parametrize("lam", ["0.5", "1", "2"])
def test_oracle_cli_reproduces_astar_dag(oracle_built, tmp_path, fig, lam):
    """ref_score -> .pss -> ref_astar reproduces triplet_data/Figure_*/astar_dag_*.csv."""
    o = oracle_built
    skel = tmp_path / "full4.csv"
    skel.write_text("1,1,1,1\n1,1,1,1\n1,1,1,1\n1,1,1,1\n")
    pss = tmp_path / "s.pss"
    net = tmp_path / "net"
    subprocess.run([o.REF_SCORE, os.path.join(GOLDEN, FIG_CSV[fig]), str(pss), "-f", "cBIC", "--lambda", lam,
                    "-k", str(skel)], check=True, stdout=subprocess.DEVNULL)
    out = subprocess.run([o.REF_ASTAR, str(pss), "-k", str(skel), "-n", str(net)], check=True,
                         capture_output=True, text=True).stdout
    assert "Nodes expanded" in out
    assert read_matrix(str(net) + ".csv") == fig_dag(fig)
    text = (tmp_path / "net").read_text().splitlines()
    assert text[0] == "NumVars 4"
    assert all(line.startswith("Var ") for line in text[1:])


def test_pss_header_and_blocks(oracle_built, tmp_path):
    o = oracle_built
    pss = tmp_path / "s.pss"
    csv = os.path.join(GOLDEN, FIG_CSV[1])
    subprocess.run([o.REF_SCORE, csv, str(pss), "-f", "cBIC", "--lambda", "2"], check=True, stdout=subprocess.DEVNULL)
    lines = pss.read_text().split("\n")
    # score_main.cpp:387-388
    assert lines[:7] == ["META pss_version = 0.1", f"META input_file={csv}", "META num_records=5000",
                         "META parent_limit=3", "META score_type=cbic", "META ess=1", ""]
    assert lines[7] == "VAR Variable_0"
    assert lines[8] == "META arity=5000"
    assert lines[9] == "-0.000000 "  # the empty set: -0.0f printed with "%f "


def test_quantize_matches_printf_round_trip(oracle_built):
    o = oracle_built
    rng = np.random.default_rng(1)
    vals = np.concatenate([rng.normal(0, 1e4, 2000), rng.normal(0, 1, 2000), [0.0078125, 0.0234375, -0.0078125,
                                                                             -1e-9, 1e-9, 0.0, -0.0, 5e-7, -5e-7]])
    for x in vals.astype(np.float32):
        expect = np.float32(-1.0 * float("%f" % float(x)))
        assert np.float32(o.quantize(float(x))).tobytes() == expect.tobytes() or (expect == 0 and o.quantize(float(x)) == 0)


def test_two_phase_schedule_equivalence(oracle_built):
    """per layer, [sets containing variable 0] then [the rest], in any
    order within a phase, stores exactly the sets the sequential Gosper order
    stores.  The HIP scorer's two launches per layer rely on this."""
    o = oracle_built
    for seed in range(4):
        n = 9
        X, _ = synth.gaussian_sem(n, 1500, 9300 + seed)
        ds = o.Dataset(X)
        for v in range(n):
            a = ds.score_variable(2.0, v, (1 << n) - 1, 5)
            b = ds.score_variable_sched(2.0, v, (1 << n) - 1, 5, 1)
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_empty_set_always_stored_and_sorted(oracle_built):
    o = oracle_built
    X = load_fig(2)
    ds = o.Dataset(X)
    offs, sets, scores = ds.score_all(1.0, [0xF] * 4, 3)
    for v in range(4):
        s = sets[offs[v]:offs[v + 1]]
        assert s[0] == 0 and np.float32(scores[offs[v]]).tobytes() == np.float32(-0.0).tobytes()
        keys = [(bin(int(x)).count("1"), int(x)) for x in s]
        assert keys == sorted(keys)
        assert all(not (int(x) >> v) & 1 for x in s)


def test_oracle_astar_api_matches_cli(oracle_built):
    o = oracle_built
    X = load_fig(1)
    ds = o.Dataset(X)
    offs, sets, scores = ds.score_all(2.0, [0xF] * 4, 3)
    costs = np.array([o.quantize(float(s)) for s in scores], dtype=np.float32)
    srch = o.Search(4, offs, sets, costs)
    res = srch.astar(edges=[0xF] * 4)
    assert res["rc"] == 0
    M = o.dag_matrix(res["vpar"], 4).tolist()
    assert M == fig_dag(1)


def test_pdb_groups_split(oracle_built):
    """static_pattern_database.cpp:95-120: consecutive variables, ceil(n/2) per group."""
    o = oracle_built
    n = 7
    X, _ = synth.gaussian_sem(n, 800, 9400)
    ds = o.Dataset(X)
    offs, sets, scores = ds.score_all(2.0, [(1 << n) - 1] * n, 3)
    costs = np.array([o.quantize(float(s)) for s in scores], dtype=np.float32)
    srch = o.Search(n, offs, sets, costs)
    srch.pdb_build(2)
    assert srch.pdb_groups() == [0b0001111, 0b1110000]
    h, comp = srch.pdb_h(0)
    assert comp == 0 and h <= 0
    h, comp = srch.pdb_h((1 << n) - 1)
    assert comp == 1 and h == 0


@pytest.mark.parametrize("fig", [1, 2])
@pytest.mark.parametrize("lam", ["0.5", "1", "2"])
def test_oracle_cli_reproduces_triplet_mec(oracle_built, tmp_path, fig, lam):
    """ref_score -> .pss -> ref_triplet reproduces triplet_data/Figure_*/triplet_mec_*.csv
    (astar/triplet_astar.cpp:991-1687; netFile.csv = directed_graph, netFile left empty)."""
    o = oracle_built
    skel = tmp_path / "skel.csv"
    skel.write_text(TRIPLET_SKELETON[fig])
    pss = tmp_path / "s.pss"
    net = tmp_path / "net"
    subprocess.run([o.REF_SCORE, os.path.join(GOLDEN, FIG_CSV[fig]), str(pss), "-f", "cBIC", "--lambda", lam,
                    "-k", str(skel)], check=True, stdout=subprocess.DEVNULL)
    subprocess.run([o.REF_TRIPLET, str(pss), "-k", str(skel), "-n", str(net)], check=True, capture_output=True)
    assert read_matrix(str(net) + ".csv") == fig_mec(fig)
    assert net.read_text() == ""
    # the same skeleton also reproduces the plain A* fixture
    subprocess.run([o.REF_ASTAR, str(pss), "-k", str(skel), "-n", str(tmp_path / "a")], check=True,
                   stdout=subprocess.DEVNULL)
    assert read_matrix(str(tmp_path / "a.csv")) == fig_dag(fig)


def test_oracle_triplet_api_memoizes_clusters(oracle_built):
    """Every triple on a 4-variable full skeleton sorts into the one cluster
    {0,1,2,3}: one distinct A* search, many memoized runs."""
    o = oracle_built
    ds = o.Dataset(load_fig(1))
    offs, sets, scores = ds.score_all(2.0, [0xF] * 4, 3)
    costs = np.array([o.quantize(float(s)) for s in scores], dtype=np.float32)
    res = o.triplet(o.Search(4, offs, sets, costs), edges=[0xF] * 4)
    assert res["rc"] == 0 and res["distinct"] == 1 and res["runs"] > 1
    assert res["mec"].tolist() == fig_mec(1)


def test_single_set_decision_matches_full_runs(oracle_built):
    """ora_decide (one set against a finished run's cache, seen as it stood
    under the two-phase layer order) reproduces every store decision and value
    of the oracle's own sequential runs -- the check the full-size GPU test
    applies to a C3 run."""
    from itertools import combinations
    o = oracle_built
    n = 10
    X, _ = synth.gaussian_sem(n, 2000, 9900)
    ds = o.Dataset(X)
    for v in (0, 3, 9):
        sets, scores = ds.score_variable(2.0, v, ((1 << n) - 1) & ~(1 << v), 5)
        cache = o.Cache(sets, scores)
        stored = {int(s): np.float32(f) for s, f in zip(sets, scores)}
        for L in range(6):
            for comb in combinations([u for u in range(n) if u != v], L):
                P = sum(1 << u for u in comb)
                st, val = ds.decide(2.0, v, P, cache)
                assert st == (P in stored), (v, P)
                if st:
                    assert np.float32(val).tobytes() == stored[P].tobytes()
