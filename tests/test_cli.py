"""The drop-in command lines (urlearning-cpp_amd/bin/score, bin/astar,
bin/triplet_astar): option
handling on the CPU, and the end-to-end CSV -> .pss -> netFile path on the
GPU against the oracle's command lines and the golden DAGs."""
import os
import subprocess

import pytest

from conftest import GOLDEN, PKG, TRIPLET_SKELETON, fig_dag, fig_mec, read_matrix

SCORE = os.path.join(PKG, "bin", "score")
ASTAR = os.path.join(PKG, "bin", "astar")
TRIPLET = os.path.join(PKG, "bin", "triplet_astar")
FIG_CSV = {1: "fig1_raw_data_8000.csv", 2: "fig2_raw_data_5000.csv"}


def _run(cmd, **kw):
    return subprocess.run(cmd, capture_output=True, text=True, **kw)


def test_cli_binaries_built():
    assert os.access(SCORE, os.X_OK) and os.access(ASTAR, os.X_OK) and os.access(TRIPLET, os.X_OK)


def test_triplet_help_and_option_errors(tmp_path):
    r = _run([TRIPLET, "--help"])
    assert r.returncode == 0 and "--skeleton" in r.stdout
    r = _run([TRIPLET, str(tmp_path / "x.pss"), "-e", "dynamic"])
    assert r.returncode == 2 and "static" in r.stderr
    r = _run([TRIPLET, str(tmp_path / "missing.pss")])
    assert r.returncode == 1 and "Could not open the score cache file" in r.stderr


def test_score_rejects_other_scoring_functions():
    r = _run([SCORE, "in.csv", "out.pss", "-f", "BDeu"])
    assert r.returncode == 2 and "cBIC" in r.stderr


def test_score_and_astar_help():
    assert _run([SCORE, "--help"]).returncode == 0
    r = _run([ASTAR, "--help"])
    assert r.returncode == 0 and "--mode" in r.stdout


def test_astar_rejects_unknown_calculator(tmp_path):
    r = _run([ASTAR, str(tmp_path / "x.pss"), "-b", "heap"])
    assert r.returncode == 2 and "Invalid BestScore" in r.stderr


def test_astar_missing_pss_fails_before_gpu(tmp_path):
    r = _run([ASTAR, str(tmp_path / "missing.pss")])
    assert r.returncode == 1 and "Could not open the score cache file" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("fig", [1, 2])
@pytest.mark.parametrize("lam", ["0.5", "2"])
def test_cli_end_to_end_matches_oracle_and_golden(tmp_path, oracle_built, fig, lam):
    o = oracle_built
    csv = os.path.join(GOLDEN, FIG_CSV[fig])
    skel = tmp_path / "full4.csv"
    skel.write_text("1,1,1,1\n1,1,1,1\n1,1,1,1\n1,1,1,1\n")
    pss, ref_pss = tmp_path / "gpu.pss", tmp_path / "ref.pss"
    r = _run([SCORE, csv, str(pss), "-f", "cBIC", "--lambda", lam, "-k", str(skel)])
    assert r.returncode == 0, r.stderr
    m = _metrics(r.stderr)
    assert m["tool"] == "score" and m["n"] == 4 and m["stored"] > 0 and m["scored"] == 4 * 8
    subprocess.run([o.REF_SCORE, csv, str(ref_pss), "-f", "cBIC", "--lambda", lam, "-k", str(skel)], check=True,
                   stdout=subprocess.DEVNULL)
    # the .pss text is the reference's format; same sets, same "%f" scores
    assert pss.read_text() == ref_pss.read_text()
    for mode in ("exact", "gpu"):
        net = tmp_path / f"net_{mode}"
        r = _run([ASTAR, str(pss), "-k", str(skel), "-n", str(net), "--mode", mode])
        assert r.returncode == 0, r.stderr
        m = _metrics(r.stderr)
        assert m["tool"] == "astar" and m["mode"] == mode and m["expanded"] > 0
        if mode == "exact":
            assert read_matrix(str(net) + ".csv") == fig_dag(fig)
            ref_net = tmp_path / "ref_net"
            subprocess.run([o.REF_ASTAR, str(pss), "-k", str(skel), "-n", str(ref_net)], check=True,
                           stdout=subprocess.DEVNULL)
            assert net.read_text() == ref_net.read_text()


def _metrics(stderr):
    """The command lines' one machine-readable line (stderr, 'ulg_metrics {json}')."""
    import json
    lines = [ln for ln in stderr.splitlines() if ln.startswith("ulg_metrics ")]
    assert len(lines) == 1, stderr
    return json.loads(lines[0][len("ulg_metrics "):])


@pytest.mark.parametrize("bad", ["1,x", ",1", "1,", "a"])
def test_astar_invalid_csv_fails_before_gpu(tmp_path, oracle_built, bad):
    """setFromCsv (typedefs.h:737-754) rejects a token atoi reads as 0 that
    does not start with '0'; both command lines refuse it before any search."""
    o = oracle_built
    pss = tmp_path / "x.pss"
    o.write_pss(str(pss), ["a", "b", "c"], [1, 1, 1], [0, 1, 2, 3], [0, 0, 0], [0.0, 0.0, 0.0])
    r = _run([ASTAR, str(pss), "-s", bad, "-p", "0"])
    assert r.returncode == 1 and "Invalid csv string" in r.stderr
    r = _run([o.REF_ASTAR, str(pss), "-s", "1,2", "-p", bad])
    assert r.returncode == 1 and "Invalid csv string" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("fig", [1, 2])
@pytest.mark.parametrize("ps", [("0", "1,2,3"), ("", "0,,2"), ("2", "0,1")])
def test_astar_cli_ancestors_scc_matches_oracle(tmp_path, oracle_built, fig, ps):
    o = oracle_built
    csv = os.path.join(GOLDEN, FIG_CSV[fig])
    pss = tmp_path / "gpu.pss"
    r = _run([SCORE, csv, str(pss), "-f", "cBIC", "--lambda", "1"])
    assert r.returncode == 0, r.stderr
    net, ref_net = tmp_path / "net", tmp_path / "ref_net"
    r = _run([ASTAR, str(pss), "-n", str(net), "-p", ps[0], "-s", ps[1]])
    assert r.returncode == 0, r.stderr
    subprocess.run([o.REF_ASTAR, str(pss), "-n", str(ref_net), "-p", ps[0], "-s", ps[1]], check=True,
                   stdout=subprocess.DEVNULL)
    assert net.read_text() == ref_net.read_text()
    assert read_matrix(str(net) + ".csv") == read_matrix(str(ref_net) + ".csv")


@pytest.mark.gpu
@pytest.mark.parametrize("fig", [1, 2])
@pytest.mark.parametrize("lam", ["0.5", "1", "2"])
def test_triplet_cli_reproduces_mec(tmp_path, oracle_built, fig, lam):
    """score -> .pss -> triplet_astar: netFile.csv is the triplet_mec fixture,
    netFile is left empty, and the oracle's ref_triplet agrees on the same .pss."""
    o = oracle_built
    csv = os.path.join(GOLDEN, FIG_CSV[fig])
    skel = tmp_path / "skel.csv"
    skel.write_text(TRIPLET_SKELETON[fig])
    pss = tmp_path / "gpu.pss"
    r = _run([SCORE, csv, str(pss), "-f", "cBIC", "--lambda", lam, "-k", str(skel)])
    assert r.returncode == 0, r.stderr
    net, ref_net = tmp_path / "net", tmp_path / "ref_net"
    r = _run([TRIPLET, str(pss), "-k", str(skel), "-n", str(net)])
    assert r.returncode == 0, r.stderr
    assert read_matrix(str(net) + ".csv") == fig_mec(fig)
    assert net.read_text() == ""
    subprocess.run([o.REF_TRIPLET, str(pss), "-k", str(skel), "-n", str(ref_net)], check=True, stdout=subprocess.DEVNULL)
    assert (tmp_path / "net.csv").read_text() == (tmp_path / "ref_net.csv").read_text()


@pytest.mark.gpu
def test_cli_c1_hepatitis_default_parent_limit(tmp_path):
    """Config C1 (BASELINE.json configs[0]) through the drop-in command lines
    on the GPU: data/hepatitis.clean.csv, --lambda 2, full skeleton, default
    -p = n - 1 = 19 (score_main.cpp:296-298; the scorer's wide layers).  The
    1.26 GB .pss must be byte-identical to the oracle's command line output
    and the netFile / netFile.csv identical to its A*
    (tests/golden/make_c1_cli.sh wrote the fixture)."""
    import hashlib
    import json
    with open(os.path.join(GOLDEN, "c1_hepatitis_cli.json")) as f:
        ref = json.load(f)
    skel = tmp_path / "full20.csv"
    skel.write_text("\n".join([",".join(["1"] * 20)] * 20) + "\n")
    pss = tmp_path / "c1.pss"
    r = _run([SCORE, ref["csv"], str(pss), "-f", "cBIC", "--lambda", ref["lambda"], "-k", str(skel)],
             cwd=GOLDEN)  # relative input path, as the fixture was made (the header records it)
    assert r.returncode == 0, r.stderr
    assert os.path.getsize(pss) == ref["pss_bytes"]
    h = hashlib.sha256()
    with open(pss, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 24), b""):
            h.update(chunk)
    assert h.hexdigest() == ref["pss_sha256"]
    for mode in ("exact", "gpu"):
        net = tmp_path / f"net_{mode}"
        r = _run([ASTAR, str(pss), "-k", str(skel), "-n", str(net), "--mode", mode])
        assert r.returncode == 0, r.stderr
        cost = float(r.stdout.split("Found solution:")[1].split()[0])
        ref_cost = float(ref["solution"].split(":")[1])
        # the batched search sums g in layer order, not the reference's path
        # order: the optimal cost up to float rounding (1e-6 relative)
        assert abs(cost - ref_cost) <= 1e-6 * abs(ref_cost), (mode, cost, ref_cost)
        if mode == "exact":  # the exact-order replay: the reference's DAG and its printed cost
            assert ref["solution"] in r.stdout
            assert net.read_text() == ref["net"]
            assert (tmp_path / "net_exact.csv").read_text() == ref["net_csv"]
    os.remove(pss)


def test_triplet_cli_accepts_running_time():
    """triplet_astar -r is the reference's flag (triplet_astar.cpp:1647,
    1674-1681): accepted and announced as the reference does, before the
    score file is read."""
    r = subprocess.run([os.path.join(PKG, "bin", "triplet_astar"), "missing.pss", "-r", "5"], capture_output=True,
                       text=True, timeout=60)
    assert "Maximum running time: 5" in r.stdout
    assert r.returncode == 1 and "not supported" not in r.stderr
