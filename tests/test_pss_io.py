"""The .pss text path: the parallel drop-in reader (host/io.cpp read_pss via
bin/pss_dump) against the oracle's sequential ScoreCache::read restatement
on quirky files (CPU), and the GPU "%f" formatter (ulg_pss_format*) against
glibc printf through the oracle's writer, special values included (GPU)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG

DUMP = os.path.join(PKG, "bin", "pss_dump")

QUIRKY = (
    "META pss_version = 0.1\r\n"
    "# a comment\n"
    "META input_file=x.csv\n"
    "\n"
    "VAR a\n"
    "META arity=3\n"
    "-0.000000 \n"
    "-12.500000 b \n"
    "-3.250000   b    c\t\n"          # runs of spaces, a tab in the last token
    "   \n"                            # whitespace only: an empty-set entry, atof("") = 0
    "-7.000000 b \n"                   # repeated set: first position, last value
    "-1.5 zz \n"                       # unknown name -> variable 0
    "-9.0 metabolite \n"               # contains "meta": skipped
    "#-4.0 c\n"
    "VAR b\r\n"
    "meta arity=2\n"
    "1e3 a c \r\n"
    "-2.000000 a \n"
    "VAR nosuch\n"                     # unknown variable: entries go to variable 0
    "-8.25 c \n"
    "VAR c\n"
    "-0.125 a b \n"
    "-0.5 a\n"                         # last line, no newline
)


def _dump(path, threads):
    env = dict(os.environ, ULG_THREADS=str(threads))
    r = subprocess.run([DUMP, str(path)], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    names = lines[0].split()[1:]
    ent = [tuple(x.split()) for x in lines[1:]]
    return names, [(int(v), int(s), c) for v, s, c in ent]


def _oracle_entries(o, path):
    names, offs, sets, costs = o.read_pss(str(path))
    ent = []
    for v in range(len(names)):
        for i in range(offs[v], offs[v + 1]):
            ent.append((v, int(sets[i]), "%08x" % np.float32(costs[i]).view(np.uint32)))
    return names, ent


@pytest.mark.parametrize("threads", [1, 3, 7, 16])
def test_reader_matches_oracle_on_quirks(oracle_built, tmp_path, threads):
    p = tmp_path / "q.pss"
    p.write_bytes(QUIRKY.encode())
    names, ent = _dump(p, threads)
    onames, oent = _oracle_entries(oracle_built, p)
    assert names == onames == ["a", "b", "nosuch", "c"]
    assert ent == oent
    # the repeated {b} of variable a: second position, last value (-7 -> cost 7)
    a_b = [e for e in ent if e[0] == 0 and e[1] == 0b10]
    assert len(a_b) == 1 and a_b[0][2] == "%08x" % np.float32(7.0).view(np.uint32)


@pytest.mark.parametrize("threads", [1, 5])
def test_reader_matches_oracle_on_generated_file(oracle_built, tmp_path, threads):
    """A few thousand lines from the oracle's writer, split over several threads."""
    o = oracle_built
    rng = np.random.default_rng(3)
    n = 9
    names = [f"Variable_{i}" for i in range(n)]
    offs = [0]
    sets, scores = [], []
    for v in range(n):
        cnt = int(rng.integers(50, 400))
        for _ in range(cnt):
            s = int(rng.integers(0, 1 << n)) & ~(1 << v)
            sets.append(s)
            scores.append(np.float32(rng.normal(0, 1e4)))
        offs.append(len(sets))
    p = tmp_path / "g.pss"
    o.write_pss(str(p), names, [5] * n, offs, sets, scores)
    assert _dump(p, threads) == _oracle_entries(o, p)


def test_reader_rejects_bad_meta(tmp_path):
    p = tmp_path / "bad.pss"
    p.write_text("META a=1\nhello\nVAR a\n-1.0 \n")
    r = subprocess.run([DUMP, str(p)], capture_output=True, text=True)
    assert r.returncode == 1 and "Expected META line or Variable" in r.stderr


SPECIAL = [-0.0, 0.0, 1e-7, -1e-7, 4.9999997e-7, 5e-7, -5e-7, 1.5e-6, 2.5e-6, 0.0000125, 123456.5, -98765.4375,
           16777216.0, 16777218.0, -3.4028235e38, 1e30, 2.0 ** -149, 1.0 / 3, 2.0 / 3, -2.0 / 3, 9.9999999e9,
           1.8446744e19, 3.6893488e19, float("inf"), float("-inf"), float("nan")]


@pytest.mark.gpu
def test_gpu_pss_format_matches_glibc(ulg_ctx, oracle_built, tmp_path):
    o = oracle_built
    rng = np.random.default_rng(4)
    n = 6
    names = ["alpha", "b", "Variable_2", "x3", "long_variable_name_4", "v5"]
    vals = np.concatenate([np.array(SPECIAL, dtype=np.float32),
                           rng.normal(0, 1e5, 3000).astype(np.float32),
                           (rng.normal(0, 1, 3000) * 10.0 ** rng.integers(-8, 8, 3000)).astype(np.float32)])
    vals = np.concatenate([vals, -vals])
    neg_nan = np.array([0xFFC00000], dtype=np.uint32).view(np.float32)
    vals = np.concatenate([vals, neg_nan])
    per = len(vals) // n + 1
    offs, sets, scores = [0], [], []
    k = 0
    for v in range(n):
        for _ in range(per):
            if k >= len(vals):
                break
            sets.append(int(rng.integers(0, 1 << n)) & ~(1 << v))
            scores.append(vals[k])
            k += 1
        offs.append(len(sets))
    # an empty list as well
    offs.append(offs[-1])
    names.append("empty")
    ref = tmp_path / "ref.pss"
    o.write_pss(str(ref), names, list(range(1, n + 2)), offs, sets, scores, num_records=5000)
    ref_text = ref.read_bytes()
    header = ref_text[: ref_text.index(b"VAR ")].decode()
    got = ulg_ctx.pss_format_lists(header, names, list(range(1, n + 2)), offs, sets, scores)
    assert got == ref_text


@pytest.mark.gpu
def test_gpu_pss_format_of_scored_lists(ulg_ctx, oracle_built, tmp_path):
    """ulg_pss_format on the device lists of a scoring run equals the oracle's
    writer on the same (fetched) lists."""
    from conftest import load_fig
    X = load_fig(1)
    n = X.shape[1]
    ulg_ctx.load(X, 1.0)
    st, sc = ulg_ctx.score(list(range(n)), [(1 << n) - 1] * n, 3)
    offs, sets, scores = ulg_ctx.fetch(st)
    names = [f"Variable_{i}" for i in range(n)]
    ref = tmp_path / "ref.pss"
    oracle_built.write_pss(str(ref), names, [5000] * n, offs, sets, scores, num_records=5000)
    ref_text = ref.read_bytes()
    header = ref_text[: ref_text.index(b"VAR ")].decode()
    assert ulg_ctx.pss_format(header, names, [5000] * n) == ref_text
