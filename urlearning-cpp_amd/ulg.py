"""ctypes binding of libulg.so (include/ulg.h) -- the HIP hot path.

This module is plumbing for tests, bench.py and scripts: every compute call
goes through the C ABI into the gfx950 kernels.  There is no CPU fallback:
if libulg.so is missing, or no HIP device is present, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ULG_LIB", os.path.join(HERE, "libulg.so"))  # ULG_LIB: A/B builds
HEADER = os.path.join(os.path.dirname(HERE), "include", "ulg.h")

_lib = None


class ULGError(RuntimeError):
    pass


def lib():
    """Load libulg.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ULGError(f"{LIB_PATH} not built: run __graft_entry__.build() or make -C urlearning-cpp_amd")
        L = C.CDLL(LIB_PATH)
        P, I, I64, D, F = C.c_void_p, C.c_int, C.c_int64, C.c_double, C.c_float
        L.ulg_create.argtypes = [C.POINTER(I), I, C.POINTER(P)]
        L.ulg_destroy.argtypes = [P]
        L.ulg_last_error.argtypes = [P]
        L.ulg_last_error.restype = C.c_char_p
        L.ulg_version.restype = C.c_char_p
        L.ulg_cbic_load.argtypes = [P, P, I64, I, D]
        L.ulg_cbic_gram.argtypes = [P, P]
        L.ulg_cbic_score.argtypes = [P, P, I, P, I, C.POINTER(I64), C.POINTER(I64)]
        L.ulg_cbic_score_async.argtypes = [P, P, I, P, I]
        L.ulg_cbic_score_finish.argtypes = [P, C.POINTER(I64), C.POINTER(I64)]
        L.ulg_cbic_fetch.argtypes = [P, P, P, P, I]
        L.ulg_cbic_score_vars.argtypes = [P, P, I, P, I, P, P, P, I64]
        L.ulg_cbic_score_sets.argtypes = [P, I64, P, P, P]
        L.ulg_quantize_costs.argtypes = [P, P, P, I64]
        L.ulg_search_load.argtypes = [P, I, P, P, P]
        L.ulg_search_from_scores.argtypes = [P]
        L.ulg_search_load_scores.argtypes = [P, I, P, P, P, I]
        L.ulg_bestscore_query.argtypes = [P, I64, P, P, P, P]
        L.ulg_pdb_build.argtypes = [P, I, C.c_uint64, C.c_uint64]
        L.ulg_pdb_query.argtypes = [P, I64, P, P, P]
        L.ulg_astar.argtypes = [P, P, I, I, P, P, C.POINTER(F), C.POINTER(I64), C.c_char_p, I64]
        L.ulg_triplet_astar.argtypes = [P, P, I, P, P]
        L.ulg_triplet_clusters.argtypes = [P, P, P, I64, C.POINTER(I64)]
        L.ulg_triplet_solve.argtypes = [P, P, I64, I, P, P]
        L.ulg_triplet_memo_put.argtypes = [P, P, I64, I, P]
        L.ulg_mmpc.argtypes = [P, D, I, P]
        L.ulg_pss_format.argtypes = [P, C.c_char_p, P, P, C.POINTER(C.c_void_p), C.POINTER(I64)]
        L.ulg_pss_format_lists.argtypes = [P, I, P, P, P, C.c_char_p, P, P, C.POINTER(C.c_void_p), C.POINTER(I64)]
        L.ulg_astar_scc.argtypes = [P, P, I, I, C.c_uint64, C.c_uint64, P, P, C.POINTER(F), C.POINTER(I64),
                                    C.c_char_p, I64]
        L.ulg_sweep_shard_begin.argtypes = [P, C.c_uint64, C.POINTER(I64)]
        L.ulg_sweep_shard_layer.argtypes = [P, I, P]
        L.ulg_sweep_shard_commit.argtypes = [P, I, P]
        L.ulg_sweep_shard_end.argtypes = [P, P, P, C.POINTER(F), C.POINTER(I64)]
        L.ulg_set_option.argtypes = [P, C.c_char_p, I64]
        L.ulg_get_info.argtypes = [P, C.c_char_p, C.POINTER(I64)]
        L.ulg_profile_enable.argtypes = [P, I]
        L.ulg_profile_get.argtypes = [P, C.c_char_p, C.POINTER(D), C.POINTER(I64), C.POINTER(D)]
        L.ulg_profile_dump.argtypes = [P, C.c_char_p, I64]
        L.ulg_profile_reset.argtypes = [P]
        L.ulg_profile_select.argtypes = [P, C.c_char_p]
        L.ulg_diag_pdb_host.argtypes = [P, C.c_uint64, I, I, P]
        _lib = L
    return _lib


def header_symbols():
    """Every function the C ABI header declares."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(ulg_[a-z0-9_]+)\s*\(", txt)))


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class Context:
    """One ulg_ctx on one GPU (one process per GPU for multi-GPU work)."""

    def __init__(self, device: int = 0):
        L = lib()
        self._h = C.c_void_p()
        dev = (C.c_int * 1)(device)
        rc = L.ulg_create(dev, 1, C.byref(self._h))
        if rc != 0:
            raise ULGError(f"ulg_create(device={device}) failed with status {rc}")
        self.device = device
        self.n = None

    def close(self):
        if self._h:
            lib().ulg_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = lib().ulg_last_error(self._h).decode()
            raise ULGError(f"{what}: status {rc}: {msg}")

    # ---- cBIC -------------------------------------------------------------
    def load(self, data: np.ndarray, lam: float):
        """data: N x n array (rows = records).  Stored column-major."""
        x = np.asfortranarray(np.asarray(data, dtype=np.float64))
        N, n = x.shape
        flat = np.ascontiguousarray(x.T.reshape(-1))  # column-major flatten
        self._check(lib().ulg_cbic_load(self._h, _ptr(flat), N, n, float(lam)), "ulg_cbic_load")
        self.n = n
        self.N = N

    def mmpc(self, alpha=0.05, max_cond=-1):
        """ulg_mmpc on the loaded data -> skeleton rows (bit j of row i = edge i-j)."""
        rows = np.zeros(64, dtype=np.uint64)
        self._check(lib().ulg_mmpc(self._h, float(alpha), int(max_cond), _ptr(rows)), "ulg_mmpc")
        return [int(x) for x in rows[:self.n]]

    def gram(self) -> np.ndarray:
        g = np.empty((self.n, self.n), dtype=np.float64)
        self._check(lib().ulg_cbic_gram(self._h, _ptr(g)), "ulg_cbic_gram")
        return g

    def score(self, variables, candidates, max_parents: int):
        """Returns (total_stored, total_scored); results stay on the GPU."""
        v = np.ascontiguousarray(variables, dtype=np.int32)
        c = np.ascontiguousarray(candidates, dtype=np.uint64)
        st, sc = C.c_int64(), C.c_int64()
        self._check(lib().ulg_cbic_score(self._h, _ptr(v), len(v), _ptr(c), int(max_parents),
                                         C.byref(st), C.byref(sc)), "ulg_cbic_score")
        self._nv = len(v)
        return st.value, sc.value

    def score_async(self, variables, candidates, max_parents: int):
        """ulg_cbic_score_async: queues the scoring call; score_finish() waits for it."""
        v = np.ascontiguousarray(variables, dtype=np.int32)
        c = np.ascontiguousarray(candidates, dtype=np.uint64)
        self._check(lib().ulg_cbic_score_async(self._h, _ptr(v), len(v), _ptr(c), int(max_parents)),
                    "ulg_cbic_score_async")
        self._nv = len(v)

    def score_finish(self):
        """-> (total_stored, total_scored) of the last (async) scoring call."""
        st, sc = C.c_int64(), C.c_int64()
        self._check(lib().ulg_cbic_score_finish(self._h, C.byref(st), C.byref(sc)), "ulg_cbic_score_finish")
        return st.value, sc.value

    def fetch(self, total_stored: int):
        sets = np.empty(max(total_stored, 1), dtype=np.uint64)
        scores = np.empty(max(total_stored, 1), dtype=np.float32)
        offs = np.empty(self._nv + 1, dtype=np.int64)
        self._check(lib().ulg_cbic_fetch(self._h, _ptr(sets), _ptr(scores), _ptr(offs), 0), "ulg_cbic_fetch")
        return offs, sets[:total_stored], scores[:total_stored]

    def stream_wait_event(self, event):
        """ulg_stream_wait_event: this context's stream waits for a
        torch.cuda.Event (or a raw hipEvent_t handle) recorded on another
        stream of the same device."""
        h = event.cuda_event if hasattr(event, "cuda_event") else int(event)
        self._check(lib().ulg_stream_wait_event(self._h, C.c_void_p(h)), "ulg_stream_wait_event")

    def fetch_device(self, sets_ptr: int, scores_ptr: int, offsets_ptr: int):
        """Copy results into caller-owned device buffers (e.g. torch tensors).
        Synchronous on the context's stream; see ulg.h's stream contract."""
        self._check(lib().ulg_cbic_fetch(self._h, C.c_void_p(sets_ptr), C.c_void_p(scores_ptr),
                                         C.c_void_p(offsets_ptr), 1), "ulg_cbic_fetch")

    def score_all(self, variables, candidates, max_parents: int):
        st, _ = self.score(variables, candidates, max_parents)
        return self.fetch(st)

    def score_sets(self, variables, parents) -> np.ndarray:
        """ScoringFunction::calculateScore's value per (variable, parent mask) pair (ulg_cbic_score_sets)."""
        v = np.ascontiguousarray(variables, dtype=np.int32)
        p = np.ascontiguousarray(parents, dtype=np.uint64)
        if v.shape != p.shape:
            raise ValueError("score_sets: variables and parents differ in length")
        out = np.empty(max(len(v), 1), dtype=np.float32)
        self._check(lib().ulg_cbic_score_sets(self._h, len(v), _ptr(v), _ptr(p), _ptr(out)), "ulg_cbic_score_sets")
        return out[:len(v)]

    def quantize(self, scores: np.ndarray) -> np.ndarray:
        s = np.ascontiguousarray(scores, dtype=np.float32)
        out = np.empty_like(s)
        self._check(lib().ulg_quantize_costs(self._h, _ptr(s), _ptr(out), s.size), "ulg_quantize_costs")
        return out

    # ---- search side -------------------------------------------------------
    ASTAR_EXACT = 0
    ASTAR_GPU = 1

    def search_load(self, offsets, sets, costs):
        o = np.ascontiguousarray(offsets, dtype=np.int64)
        s = np.ascontiguousarray(sets, dtype=np.uint64)
        c = np.ascontiguousarray(costs, dtype=np.float32)
        if s.size == 0:
            s = np.zeros(1, dtype=np.uint64)
            c = np.zeros(1, dtype=np.float32)
        self._check(lib().ulg_search_load(self._h, len(o) - 1, _ptr(o), _ptr(s), _ptr(c)), "ulg_search_load")
        self.search_n = len(o) - 1

    def search_from_scores(self):
        self._check(lib().ulg_search_from_scores(self._h), "ulg_search_from_scores")
        self.search_n = self.n

    def search_load_scores(self, offsets, sets, scores, device_ptrs=False):
        """ulg_search_load_scores: per-variable .pss-score lists in variable
        order (offsets[n+1] on the host).  device_ptrs: sets/scores are
        device addresses (ints, e.g. tensor.data_ptr()); else numpy arrays."""
        o = np.ascontiguousarray(offsets, dtype=np.int64)
        if device_ptrs:
            sp, cp = C.c_void_p(int(sets)), C.c_void_p(int(scores))
            keep = None
        else:
            s = np.ascontiguousarray(sets, dtype=np.uint64)
            c = np.ascontiguousarray(scores, dtype=np.float32)
            if s.size == 0:
                s, c = np.zeros(1, dtype=np.uint64), np.zeros(1, dtype=np.float32)
            sp, cp, keep = _ptr(s), _ptr(c), (s, c)
        self._check(lib().ulg_search_load_scores(self._h, len(o) - 1, _ptr(o), sp, cp, 1 if device_ptrs else 0),
                    "ulg_search_load_scores")
        del keep
        self.search_n = len(o) - 1

    def bestscore(self, variables, S):
        v = np.ascontiguousarray(variables, dtype=np.int32)
        s = np.ascontiguousarray([int(x) for x in S], dtype=np.uint64)
        costs = np.empty(len(v), dtype=np.float32)
        par = np.empty(len(v), dtype=np.uint64)
        self._check(lib().ulg_bestscore_query(self._h, len(v), _ptr(v), _ptr(s), _ptr(costs), _ptr(par)),
                    "ulg_bestscore_query")
        return costs, par

    def pdb_build(self, pd_count=2, ancestors=0, scc=None):
        if scc is None:
            scc = (1 << self.search_n) - 1
        self._check(lib().ulg_pdb_build(self._h, int(pd_count), int(ancestors), int(scc)), "ulg_pdb_build")

    def pdb_h(self, S):
        s = np.ascontiguousarray([int(x) for x in S], dtype=np.uint64)
        h = np.empty(len(s), dtype=np.float32)
        comp = np.empty(len(s), dtype=np.int32)
        self._check(lib().ulg_pdb_query(self._h, len(s), _ptr(s), _ptr(h), _ptr(comp)), "ulg_pdb_query")
        return h, comp

    def astar(self, edges=None, pd_count=2, mode=0, net_text=True, ancestors=None, scc=None):
        n = self.search_n
        vpar = np.zeros(n, dtype=np.uint64)
        order = np.zeros(n, dtype=np.int32)
        cost = C.c_float()
        exp = C.c_int64()
        buf = C.create_string_buffer(1 << 16) if net_text else None
        e = None
        if edges is not None:
            e = np.ascontiguousarray([int(x) for x in edges], dtype=np.uint64)
        if ancestors is None and scc is None:
            self._check(lib().ulg_astar(self._h, _ptr(e) if e is not None else None, int(pd_count), int(mode),
                                        _ptr(vpar), _ptr(order), C.byref(cost), C.byref(exp), buf,
                                        len(buf) if buf is not None else 0), "ulg_astar")
        else:
            anc = int(ancestors or 0)
            sc = int(scc) if scc is not None else (1 << n) - 1
            self._check(lib().ulg_astar_scc(self._h, _ptr(e) if e is not None else None, int(pd_count), int(mode),
                                            anc, sc, _ptr(vpar), _ptr(order), C.byref(cost), C.byref(exp), buf,
                                            len(buf) if buf is not None else 0), "ulg_astar_scc")
        return {"vpar": vpar, "order": order, "cost": cost.value, "expanded": exp.value,
                "net_text": buf.value.decode() if buf is not None else None}

    def sweep_shard_begin(self, own: int) -> int:
        """This rank's tables and sweep slices for the variables in `own`
        (ulg_sweep_shard_begin); returns the largest layer's node count."""
        mx = C.c_int64()
        self._check(lib().ulg_sweep_shard_begin(self._h, int(own), C.byref(mx)), "ulg_sweep_shard_begin")
        return mx.value

    def sweep_shard_layer(self, layer: int, keys_ptr: int):
        self._check(lib().ulg_sweep_shard_layer(self._h, int(layer), C.c_void_p(keys_ptr)), "ulg_sweep_shard_layer")

    def sweep_shard_commit(self, layer: int, keys_ptr: int):
        self._check(lib().ulg_sweep_shard_commit(self._h, int(layer), C.c_void_p(keys_ptr)), "ulg_sweep_shard_commit")

    def sweep_shard_end(self):
        n = self.search_n
        vpar = np.zeros(n, dtype=np.uint64)
        order = np.zeros(n, dtype=np.int32)
        cost = C.c_float()
        exp = C.c_int64()
        self._check(lib().ulg_sweep_shard_end(self._h, _ptr(vpar), _ptr(order), C.byref(cost), C.byref(exp)),
                    "ulg_sweep_shard_end")
        return {"vpar": vpar, "order": order, "cost": cost.value, "expanded": exp.value}

    def _names_arg(self, names):
        arr = (C.c_char_p * len(names))(*[x.encode() for x in names])
        return arr

    def pss_format(self, header: str, names, arity) -> bytes:
        """ulg_pss_format: the .pss text of the last score() call (every variable)."""
        nm = self._names_arg(names)
        ar = np.ascontiguousarray(arity, dtype=np.int32)
        text, ln = C.c_void_p(), C.c_int64()
        self._check(lib().ulg_pss_format(self._h, header.encode(), C.cast(nm, C.c_void_p), _ptr(ar), C.byref(text),
                                         C.byref(ln)), "ulg_pss_format")
        return C.string_at(text.value, ln.value)

    def pss_format_lists(self, header: str, names, arity, offsets, sets, scores) -> bytes:
        nm = self._names_arg(names)
        ar = np.ascontiguousarray(arity, dtype=np.int32)
        offs = np.ascontiguousarray(offsets, dtype=np.int64)
        st = np.ascontiguousarray(sets, dtype=np.uint64)
        sc = np.ascontiguousarray(scores, dtype=np.float32)
        text, ln = C.c_void_p(), C.c_int64()
        self._check(lib().ulg_pss_format_lists(self._h, len(names), _ptr(offs), _ptr(st), _ptr(sc), header.encode(),
                                               C.cast(nm, C.c_void_p), _ptr(ar), C.byref(text), C.byref(ln)),
                    "ulg_pss_format_lists")
        return C.string_at(text.value, ln.value)

    def triplet(self, edges=None, pd_count=2):
        """ulg_triplet_astar -> {"mec": n x n int32 (i -> j at [i, j]), "runs", "distinct", "expanded"}."""
        n = self.search_n
        dg = np.zeros(n * n, dtype=np.int32)
        stats = np.zeros(3, dtype=np.int64)
        e = None
        if edges is not None:
            e = np.ascontiguousarray([int(x) for x in edges], dtype=np.uint64)
        self._check(lib().ulg_triplet_astar(self._h, _ptr(e) if e is not None else None, int(pd_count), _ptr(dg),
                                            _ptr(stats)), "ulg_triplet_astar")
        return {"mec": dg.reshape(n, n), "runs": int(stats[0]), "distinct": int(stats[1]), "expanded": int(stats[2])}

    def triplet_clusters(self, edges=None):
        """ulg_triplet_clusters -> uint64 array of the first sweep's distinct clusters."""
        e = None if edges is None else np.ascontiguousarray([int(x) for x in edges], dtype=np.uint64)
        cnt = C.c_int64()
        self._check(lib().ulg_triplet_clusters(self._h, _ptr(e) if e is not None else None, None, 0,
                                               C.byref(cnt)), "ulg_triplet_clusters")
        out = np.zeros(max(cnt.value, 1), dtype=np.uint64)
        self._check(lib().ulg_triplet_clusters(self._h, _ptr(e) if e is not None else None, _ptr(out), len(out),
                                               C.byref(cnt)), "ulg_triplet_clusters")
        return out[:cnt.value]

    def triplet_solve(self, clusters, pd_count=2):
        """ulg_triplet_solve -> (parents [nc, n] uint64, {"runs", "distinct", "expanded"})."""
        cl = np.ascontiguousarray(clusters, dtype=np.uint64)
        par = np.zeros((max(len(cl), 1), self.search_n), dtype=np.uint64)
        stats = np.zeros(3, dtype=np.int64)
        self._check(lib().ulg_triplet_solve(self._h, _ptr(cl), len(cl), int(pd_count), _ptr(par), _ptr(stats)),
                    "ulg_triplet_solve")
        return par[:len(cl)], {"runs": int(stats[0]), "distinct": int(stats[1]), "expanded": int(stats[2])}

    def triplet_memo_put(self, clusters, parents, pd_count=2):
        cl = np.ascontiguousarray(clusters, dtype=np.uint64)
        par = np.ascontiguousarray(parents, dtype=np.uint64).reshape(len(cl), self.search_n) if len(cl) else \
            np.zeros((1, self.search_n), dtype=np.uint64)
        self._check(lib().ulg_triplet_memo_put(self._h, _ptr(cl), len(cl), int(pd_count), _ptr(par)),
                    "ulg_triplet_memo_put")

    def set_option(self, name: str, value: int):
        self._check(lib().ulg_set_option(self._h, name.encode(), int(value)), "ulg_set_option")

    def diag_pdb_host(self, cluster: int, pd_count: int = 2, cancel_preset: bool = False):
        """ulg_diag_pdb_host (tests): -> (built, cancelled, entries, entries equal to the device PDB's)."""
        out = np.zeros(4, dtype=np.int64)
        self._check(lib().ulg_diag_pdb_host(self._h, C.c_uint64(int(cluster)), int(pd_count), int(bool(cancel_preset)),
                                            _ptr(out)), "ulg_diag_pdb_host")
        return tuple(int(x) for x in out)

    def info(self, name: str) -> int:
        """ulg_get_info: "out_of_time", "highest_completed_layer", "score_error_word",
        "exact_cycles", "exact_instructions", "exact_cache_misses"."""
        v = C.c_int64()
        self._check(lib().ulg_get_info(self._h, name.encode(), C.byref(v)), "ulg_get_info")
        return v.value

    # ---- profiling ----------------------------------------------------------
    def profile(self, on: bool = True):
        self._check(lib().ulg_profile_enable(self._h, 1 if on else 0), "ulg_profile_enable")

    def profile_select(self, names=None):
        """Time only these kernels (None = all)."""
        arg = ",".join(names).encode() if names else None
        self._check(lib().ulg_profile_select(self._h, arg), "ulg_profile_select")

    def profile_reset(self):
        self._check(lib().ulg_profile_reset(self._h), "ulg_profile_reset")

    def profile_get(self, name: str):
        avg, tot = C.c_double(), C.c_double()
        cnt = C.c_int64()
        rc = lib().ulg_profile_get(self._h, name.encode(), C.byref(avg), C.byref(cnt), C.byref(tot))
        if rc != 0:
            return None
        return {"avg_ms": avg.value, "count": cnt.value, "total_ms": tot.value}

    def profile_dump(self) -> dict:
        buf = C.create_string_buffer(1 << 16)
        self._check(lib().ulg_profile_dump(self._h, buf, len(buf)), "ulg_profile_dump")
        out = {}
        for line in buf.value.decode().splitlines():
            name, cnt, tot = line.split()
            out[name] = {"count": int(cnt), "total_ms": float(tot)}
        return out


def candidates_from_edges(edges, n: int):
    """2-hop candidate sets N(v) U N(N(v)) (score_main.cpp:146-153)."""
    allm = (1 << n) - 1
    if edges is None:
        return [allm] * n
    out = []
    for v in range(n):
        nb = int(edges[v])
        for j in range(n):
            if (int(edges[v]) >> j) & 1 and j != v:
                nb |= int(edges[j])
        out.append(nb)
    return out
