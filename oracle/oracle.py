"""ctypes wrapper of the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path.  See ora.h for the
reference functions each entry point restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(BUILD, "liboracle.so")
REF_SCORE = os.path.join(BUILD, "ref_score")
REF_ASTAR = os.path.join(BUILD, "ref_astar")
REF_TRIPLET = os.path.join(BUILD, "ref_triplet")
REF_DAGSCORE = os.path.join(BUILD, "ref_calc_dag_score")

_lib = None


def build(quiet: bool = True):
    subprocess.run(["make", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P, I, I64, D, F, U64 = C.c_void_p, C.c_int, C.c_int64, C.c_double, C.c_float, C.c_uint64
        L.ora_dataset_from_colmajor.argtypes = [P, I64, I]
        L.ora_dataset_from_colmajor.restype = P
        L.ora_dataset_from_csv.argtypes = [C.c_char_p]
        L.ora_dataset_from_csv.restype = P
        L.ora_dataset_free.argtypes = [P]
        L.ora_dataset_N.argtypes = [P]
        L.ora_dataset_N.restype = I64
        L.ora_dataset_n.argtypes = [P]
        L.ora_dataset_norm.argtypes = [P]
        L.ora_dataset_norm.restype = C.POINTER(C.c_double)
        L.ora_cbic_raw.argtypes = [P, D, I, U64]
        L.ora_cbic_raw.restype = F
        L.ora_score_variable.argtypes = [P, D, I, U64, I, P, P, I64]
        L.ora_score_variable.restype = I64
        L.ora_score_variable_sched.argtypes = [P, D, I, U64, I, I, P, P, I64]
        L.ora_score_variable_sched.restype = I64
        L.ora_score_all.argtypes = [P, D, P, I, I, P, P, P, P]
        L.ora_score_sample.argtypes = [P, D, P, I, P, I, D, I]
        L.ora_score_sample.restype = I64
        L.ora_quantize_cost.argtypes = [F]
        L.ora_quantize_cost.restype = F
        L.ora_search_create.argtypes = [I, P, P, P]
        L.ora_search_create.restype = P
        L.ora_search_free.argtypes = [P]
        L.ora_search_set_time_limit.argtypes = [P, D]
        L.ora_search_out_of_time.argtypes = [P]
        L.ora_search_last_open.argtypes = [P]
        L.ora_search_last_open.restype = I64
        L.ora_bestscore.argtypes = [P, I, U64, C.POINTER(U64)]
        L.ora_bestscore.restype = F
        L.ora_pdb_build.argtypes = [P, I, U64, U64]
        L.ora_pdb_h.argtypes = [P, U64, C.POINTER(I)]
        L.ora_pdb_h.restype = F
        L.ora_pdb_groups.argtypes = [P, P, I]
        L.ora_pdb_value.argtypes = [P, I, U64]
        L.ora_pdb_value.restype = F
        L.ora_astar.argtypes = [P, P, I, P, P, C.POINTER(F), C.POINTER(I64), C.c_char_p, I64]
        L.ora_astar_scc.argtypes = [P, P, I, U64, U64, P, P, C.POINTER(F), C.POINTER(I64), C.c_char_p, I64]
        L.ora_mmpc.argtypes = [P, D, I, P]
        L.ora_cache_create.argtypes = [P, P, I64]
        L.ora_cache_create.restype = P
        L.ora_cache_free.argtypes = [P]
        L.ora_decide.argtypes = [P, D, I, U64, P, C.POINTER(F)]
        L.ora_norm_quantile.argtypes = [D]
        L.ora_norm_quantile.restype = D
        L.ora_partial_z.argtypes = [P, I, D, I, I, P, I]
        L.ora_partial_z.restype = D
        L.ora_triplet_astar.argtypes = [P, P, I, P, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def binom(m, k):
    from math import comb
    return comb(m, k) if 0 <= k <= m else 0


class Dataset:
    def __init__(self, X=None, csv_path=None):
        L = lib()
        if csv_path is not None:
            self.h = L.ora_dataset_from_csv(csv_path.encode())
        else:
            x = np.asarray(X, dtype=np.float64)
            flat = np.ascontiguousarray(x.T.reshape(-1))
            self.h = L.ora_dataset_from_colmajor(_p(flat), x.shape[0], x.shape[1])
        if not self.h:
            raise RuntimeError("oracle dataset load failed")
        self.n = L.ora_dataset_n(self.h)
        self.N = L.ora_dataset_N(self.h)

    def __del__(self):
        try:
            lib().ora_dataset_free(self.h)
        except Exception:
            pass

    def norm(self):
        p = lib().ora_dataset_norm(self.h)
        return np.ctypeslib.as_array(p, shape=(self.n * self.N,)).reshape(self.n, self.N).T.copy()

    def cbic_raw(self, lam, v, parents):
        return lib().ora_cbic_raw(self.h, float(lam), int(v), int(parents))

    def decide(self, lam, v, P, cache):
        """ora_decide -> (stored, value) for one set against a cache handle."""
        val = C.c_float()
        st = lib().ora_decide(self.h, float(lam), int(v), int(P), cache.h, C.byref(val))
        return bool(st), val.value

    def mmpc(self, alpha=0.05, max_cond=-1):
        """ora_mmpc -> skeleton rows (bit j of row i = edge i-j)."""
        rows = np.zeros(64, dtype=np.uint64)
        lib().ora_mmpc(self.h, float(alpha), int(max_cond), _p(rows))
        return [int(x) for x in rows[:self.n]]

    def score_variable(self, lam, v, candidates, k):
        m = bin(int(candidates) & ~(1 << v)).count("1")
        cap = sum(binom(m, L) for L in range(0, k + 1)) + 1
        sets = np.empty(cap, dtype=np.uint64)
        scores = np.empty(cap, dtype=np.float32)
        c = lib().ora_score_variable(self.h, float(lam), int(v), int(candidates), int(k), _p(sets), _p(scores), cap)
        if c < 0:
            raise RuntimeError("oracle capacity")
        return sets[:c].copy(), scores[:c].copy()

    def score_variable_sched(self, lam, v, candidates, k, sched):
        m = bin(int(candidates) & ~(1 << v)).count("1")
        cap = sum(binom(m, L) for L in range(0, k + 1)) + 1
        sets = np.empty(cap, dtype=np.uint64)
        scores = np.empty(cap, dtype=np.float32)
        c = lib().ora_score_variable_sched(self.h, float(lam), int(v), int(candidates), int(k), int(sched),
                                           _p(sets), _p(scores), cap)
        if c < 0:
            raise RuntimeError("oracle capacity")
        return sets[:c].copy(), scores[:c].copy()

    def score_all(self, lam, candidates, k, threads=1):
        n = self.n
        cands = np.asarray([int(c) for c in candidates], dtype=np.uint64)
        caps = np.asarray([sum(binom(bin(int(cands[v]) & ~(1 << v)).count("1"), L) for L in range(0, k + 1)) + 1
                           for v in range(n)], dtype=np.int64)
        sets = np.empty(int(caps.sum()), dtype=np.uint64)
        scores = np.empty(int(caps.sum()), dtype=np.float32)
        offs = np.empty(n + 1, dtype=np.int64)
        rc = lib().ora_score_all(self.h, float(lam), _p(cands), int(k), int(threads), _p(caps), _p(sets),
                                 _p(scores), _p(offs))
        if rc != 0:
            raise RuntimeError("oracle score_all failed")
        return offs, sets[:offs[n]].copy(), scores[:offs[n]].copy()


def score_sample(ds, lam, variables, candidates, k, frac, threads):
    v = np.ascontiguousarray(variables, dtype=np.int32)
    c = np.ascontiguousarray([int(x) for x in candidates], dtype=np.uint64)
    return lib().ora_score_sample(ds.h, float(lam), _p(v), len(v), _p(c), int(k), float(frac), int(threads))


def quantize(score: float) -> float:
    return lib().ora_quantize_cost(float(score))


class Search:
    """BestScore lists + static PDB + exact-order A* (astar_main.cpp)."""

    def __init__(self, n, offsets, sets, costs):
        self.n = n
        self.offs = np.ascontiguousarray(offsets, dtype=np.int64)
        self.sets = np.ascontiguousarray(sets, dtype=np.uint64)
        self.costs = np.ascontiguousarray(costs, dtype=np.float32)
        self.h = lib().ora_search_create(n, _p(self.offs), _p(self.sets), _p(self.costs))

    def __del__(self):
        try:
            lib().ora_search_free(self.h)
        except Exception:
            pass

    def bestscore(self, v, S):
        par = C.c_uint64()
        c = lib().ora_bestscore(self.h, int(v), int(S), C.byref(par))
        return c, par.value

    def pdb_build(self, pd_count=2, ancestors=0, scc=None):
        if scc is None:
            scc = (1 << self.n) - 1
        return lib().ora_pdb_build(self.h, pd_count, ancestors, scc)

    def pdb_h(self, S):
        comp = C.c_int(0)
        h = lib().ora_pdb_h(self.h, int(S), C.byref(comp))
        return h, comp.value

    def pdb_groups(self):
        g = np.zeros(64, dtype=np.uint64)
        k = lib().ora_pdb_groups(self.h, _p(g), 64)
        return [int(x) for x in g[:k]]

    def astar(self, edges=None, pd_count=2, ancestors=None, scc=None, time_limit_s=0.0):
        """time_limit_s > 0: the reference's -r watchdog; the result's
        out_of_time says the search stopped on it (expanded = pops so far)."""
        n = self.n
        lib().ora_search_set_time_limit(self.h, float(time_limit_s))
        vpar = np.zeros(n, dtype=np.uint64)
        order = np.zeros(n, dtype=np.int32)
        cost = C.c_float()
        exp = C.c_int64()
        buf = C.create_string_buffer(1 << 16)
        e = None
        if edges is not None:
            e = np.ascontiguousarray(edges, dtype=np.uint64)
        if ancestors is None and scc is None:
            rc = lib().ora_astar(self.h, _p(e) if e is not None else None, pd_count, _p(vpar), _p(order),
                                 C.byref(cost), C.byref(exp), buf, len(buf))
        else:
            rc = lib().ora_astar_scc(self.h, _p(e) if e is not None else None, pd_count, int(ancestors or 0),
                                     int(scc) if scc is not None else (1 << n) - 1, _p(vpar), _p(order),
                                     C.byref(cost), C.byref(exp), buf, len(buf))
        return {"rc": rc, "vpar": vpar, "order": order, "cost": cost.value, "expanded": exp.value,
                "net_text": buf.value.decode(), "out_of_time": bool(lib().ora_search_out_of_time(self.h)),
                "open_list": lib().ora_search_last_open(self.h)}


def triplet(search, edges=None, pd_count=2):
    n = search.n
    dg = np.zeros(n * n, dtype=np.int32)
    runs, distinct, exp = C.c_int64(), C.c_int64(), C.c_int64()
    e = None
    if edges is not None:
        e = np.ascontiguousarray([int(x) for x in edges], dtype=np.uint64)
    rc = lib().ora_triplet_astar(search.h, _p(e) if e is not None else None, pd_count, _p(dg), C.byref(runs),
                                 C.byref(distinct), C.byref(exp))
    return {"rc": rc, "mec": dg.reshape(n, n), "runs": runs.value, "distinct": distinct.value,
            "expanded": exp.value}


class _OraPss(C.Structure):
    _fields_ = [("n", C.c_int), ("names", C.POINTER(C.c_char_p)), ("offsets", C.POINTER(C.c_int64)),
                ("sets", C.POINTER(C.c_uint64)), ("costs", C.POINTER(C.c_float))]


def write_pss(path, names, arity, offsets, sets, scores, input_file="x.csv", num_records=0, parent_limit=3,
              score_type="cbic"):
    """ora_pss_write: glibc printf("%f ") lines (score_main.cpp:173-203,383-389)."""
    L = lib()
    L.ora_pss_write.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                C.c_void_p, C.c_char_p, C.c_int64, C.c_int, C.c_char_p]
    n = len(names)
    stride = max(len(x) for x in names) + 1
    blob = b"".join(x.encode().ljust(stride, b"\0") for x in names)
    ar = np.ascontiguousarray(arity, dtype=np.int32)
    offs = np.ascontiguousarray(offsets, dtype=np.int64)
    st = np.ascontiguousarray(sets, dtype=np.uint64)
    sc = np.ascontiguousarray(scores, dtype=np.float32)
    rc = L.ora_pss_write(path.encode(), n, blob, stride, _p(ar), _p(offs), _p(st), _p(sc), input_file.encode(),
                         int(num_records), int(parent_limit), score_type.encode())
    if rc != 0:
        raise OSError(path)


def read_pss(path):
    """ora_pss_read (ScoreCache::read restatement) -> (names, offsets, sets, costs) or None."""
    L = lib()
    L.ora_pss_read.argtypes = [C.c_char_p, C.POINTER(_OraPss)]
    L.ora_pss_free.argtypes = [C.POINTER(_OraPss)]
    p = _OraPss()
    if L.ora_pss_read(path.encode(), C.byref(p)) != 0:
        return None
    n = p.n
    names = [p.names[i].decode() for i in range(n)]
    offs = np.array([p.offsets[i] for i in range(n + 1)], dtype=np.int64)
    tot = int(offs[-1])
    sets = np.array([p.sets[i] for i in range(tot)], dtype=np.uint64)
    costs = np.array([p.costs[i] for i in range(tot)], dtype=np.float32)
    L.ora_pss_free(C.byref(p))
    return names, offs, sets, costs


class Cache:
    """ora_cache over one variable's stored (set, score) list."""

    def __init__(self, sets, scores):
        self._s = np.ascontiguousarray(sets, dtype=np.uint64)
        self._f = np.ascontiguousarray(scores, dtype=np.float32)
        self.h = lib().ora_cache_create(_p(self._s), _p(self._f), len(self._s))

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_cache_free(self.h)
            self.h = None


def dag_matrix(vpar, n):
    """netFile.csv matrix: row v, column i = 1 iff i -> v."""
    M = np.zeros((n, n), dtype=np.int64)
    for v in range(n):
        for i in range(n):
            if (int(vpar[v]) >> i) & 1:
                M[v, i] = 1
    return M
