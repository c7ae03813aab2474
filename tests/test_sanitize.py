"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

`make sanitize` builds, with -fsanitize=address,undefined and no recovery:
  * urlearning-cpp_amd/bin/san/heap_check: the two replays of the reference's
    priority queue (csrc/exact_heap.h) run side by side on random push / pop /
    decrease-key sequences, including sub-FLT_EPSILON near-ties that make the
    reference's __down_heap move and leave stale pqPos values; every pop,
    heap slot and position must agree;
  * urlearning-cpp_amd/bin/san/pss_dump: the parallel .pss reader (host/io.cpp);
  * oracle/build/san/ref_{score,astar,triplet}: the CPU oracle's command lines.
Any sanitizer report aborts the program, so a zero exit status is the check."""
import os
import subprocess

import pytest

from conftest import GOLDEN, ORACLE, PKG, TRIPLET_SKELETON

SAN = os.path.join(PKG, "bin", "san")
OSAN = os.path.join(ORACLE, "build", "san")


@pytest.fixture(scope="module")
def san_built():
    import fcntl
    # one builder at a time (pytest-xdist workers share the output tree)
    with open(os.path.join(PKG, ".sanitize.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", PKG, "sanitize"], check=True, stdout=subprocess.DEVNULL)
        subprocess.run(["make", "-C", ORACLE, "sanitize"], check=True, stdout=subprocess.DEVNULL)


def _run(cmd, **extra_env):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", **extra_env)
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (cmd, r.stdout[-2000:], r.stderr[-4000:])
    return r


@pytest.mark.parametrize("seed,ops,bits", [(1, 1500000, 8), (4, 2000000, 8), (7, 600000, 12), (11, 400000, 15)])
def test_heap_replays_agree_under_sanitizers(san_built, seed, ops, bits):
    r = _run([os.path.join(SAN, "heap_check"), str(seed), str(ops), str(bits)])
    assert "heap_check ok" in r.stdout


def test_pss_reader_under_sanitizers(san_built, tmp_path):
    from test_pss_io import QUIRKY
    p = tmp_path / "q.pss"
    p.write_bytes(QUIRKY.encode())
    for threads in ("1", "3", "16"):
        r = _run([os.path.join(SAN, "pss_dump"), str(p)], ULG_THREADS=threads)
        assert r.stdout.startswith("names a b nosuch c")
    bad = tmp_path / "bad.pss"
    bad.write_text("META arity=x\nVAR a\n-1.0 \n")
    subprocess.run([os.path.join(SAN, "pss_dump"), str(bad)], capture_output=True, timeout=60)


@pytest.mark.parametrize("fig", [1, 2])
def test_oracle_command_lines_under_sanitizers(san_built, tmp_path, fig):
    csv = os.path.join(GOLDEN, {1: "fig1_raw_data_8000.csv", 2: "fig2_raw_data_5000.csv"}[fig])
    pss = tmp_path / "f.pss"
    skel = tmp_path / "skel.csv"
    skel.write_text(TRIPLET_SKELETON[fig])
    _run([os.path.join(OSAN, "ref_score"), csv, str(pss), "-f", "cBIC", "--lambda", "2", "-p", "3"])
    _run([os.path.join(OSAN, "ref_astar"), str(pss), "-k", str(skel), "-n", str(tmp_path / "net")])
    _run([os.path.join(OSAN, "ref_triplet"), str(pss), "-k", str(skel), "-n", str(tmp_path / "mec")])
    assert (tmp_path / "net.csv").exists() and (tmp_path / "mec").exists()
