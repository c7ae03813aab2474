import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "urlearning-cpp_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")

for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libulg.so on cuda:0)")


@pytest.fixture(scope="session")
def oracle_built():
    subprocess.run(["make", "-C", ORACLE], check=True, stdout=subprocess.DEVNULL)
    import oracle
    return oracle


@pytest.fixture(scope="session")
def ulg_ctx():
    """A libulg context on GPU 0 (gpu tests only)."""
    import ulg
    ctx = ulg.Context(0)
    yield ctx
    ctx.close()


def read_matrix(path):
    rows = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line:
                rows.append([int(x) for x in line.replace(" ", "").split(",") if x != ""])
    return rows


def load_fig(fig):
    import numpy as np
    name = {1: "fig1_raw_data_8000.csv", 2: "fig2_raw_data_5000.csv"}[fig]
    return np.loadtxt(os.path.join(GOLDEN, name), delimiter=",")


def fig_dag(fig):
    name = {1: "fig1_astar_dag_8000.csv", 2: "fig2_astar_dag_5000.csv"}[fig]
    return read_matrix(os.path.join(GOLDEN, name))


def fig_mec(fig):
    name = {1: "fig1_triplet_mec_8000.csv", 2: "fig2_triplet_mec_5000.csv"}[fig]
    return read_matrix(os.path.join(GOLDEN, name))


# The skeleton each triplet_mec fixture is reproduced with.  The fixtures do not
# record it; Figure 1's fully oriented MEC needs the all-ones matrix (diagonal
# included: the degenerate triples (i, i, k) orient every A* edge), Figure 2's
# CPDAG-shaped MEC needs the off-diagonal skeleton.  Both give the A* DAG fixture.
TRIPLET_SKELETON = {1: "1,1,1,1\n1,1,1,1\n1,1,1,1\n1,1,1,1\n",
                    2: "0,1,1,1\n1,0,1,1\n1,1,0,1\n1,1,1,0\n"}
