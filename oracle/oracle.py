"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end for oracle/liboracle.so, the plain-C restatement of cover/cover.go and
prog/prio.go (see oracle.h for the file:line map). Imported only by tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg. The product package syzkaller_amd never
imports this module.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_f32p = ctypes.POINTER(ctypes.c_float)
_szp = ctypes.POINTER(ctypes.c_size_t)

OPS = {"difference": 0, "symmetric_difference": 1, "union": 2, "intersection": 3}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so not built (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        L.oracle_canonicalize.argtypes = [_u32p, ctypes.c_size_t, _szp]
        L.oracle_setop.argtypes = [ctypes.c_int, _u32p, ctypes.c_size_t, _u32p, ctypes.c_size_t, _u32p,
                                   ctypes.c_size_t, _szp]
        L.oracle_minimize.argtypes = [_u32p, _u64p, ctypes.c_size_t, _i64p, _szp]
        L.oracle_minimize_grouped.argtypes = [_u32p, _u64p, _u32p, ctypes.c_size_t, ctypes.c_uint32, _i64p,
                                              _u64p]
        L.oracle_minimize_order.argtypes = [_u64p, ctypes.c_size_t, _i64p]
        L.oracle_set_go_sort_leaf.argtypes = [ctypes.c_int]
        L.oracle_dynamic_prio.argtypes = [_u16p, ctypes.c_size_t, ctypes.c_int32, _f32p]
        L.oracle_call_cooccurrence.argtypes = [_u16p, _u64p, ctypes.c_size_t, ctypes.c_int32,
                                               ctypes.POINTER(ctypes.c_int32)]
        L.oracle_normalize_prio.argtypes = [_f32p, ctypes.c_int32]
        L.oracle_normalize_prio.restype = None
        L.oracle_calculate_priorities.argtypes = [_f32p, _u16p, ctypes.c_size_t, ctypes.c_int32, _f32p]
        L.oracle_build_choice_table.argtypes = [_f32p, _u8p, ctypes.c_int32, _i64p, _u8p]
        L.oracle_novelty.argtypes = [_u32p, _u64p, _u32p, ctypes.c_size_t, ctypes.c_uint32, _u32p, _u64p,
                                     _u32p, ctypes.c_size_t, _u8p, _u32p, _u64p, ctypes.c_size_t]
        L.oracle_prog_scan.argtypes = [_u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), _u8p]
        L.oracle_prog_scan.restype = None
        L.oracle_sha1.argtypes = [_u8p, ctypes.c_size_t, _u8p]
        L.oracle_sha1.restype = None
        L.oracle_cover_stats.argtypes = [_u32p, _u64p, _u32p, ctypes.c_size_t, ctypes.c_uint32, _u64p, _u64p,
                                         _u64p, _u64p, _u32p]
        L.oracle_corpus_cover.argtypes = [_u32p, _u64p, _u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int64,
                                          ctypes.c_int, _u32p, ctypes.c_size_t, _szp]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError("oracle %s failed: status %d" % (what, rc))


def canonicalize(cov):
    a = np.ascontiguousarray(np.asarray(cov, dtype=np.uint32)).copy()
    n = ctypes.c_size_t()
    _check(lib().oracle_canonicalize(_p(a, _u32p), a.size, ctypes.byref(n)), "canonicalize")
    return a[: n.value].copy()


def setop(op, a, b):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.uint32))
    b = np.ascontiguousarray(np.asarray(b, dtype=np.uint32))
    out = np.empty(a.size + b.size + 1, dtype=np.uint32)
    n = ctypes.c_size_t()
    _check(lib().oracle_setop(OPS[op], _p(a, _u32p), a.size, _p(b, _u32p), b.size, _p(out, _u32p), out.size,
                              ctypes.byref(n)), op)
    return out[: n.value].copy()


def to_csr(covers):
    off = np.zeros(len(covers) + 1, dtype=np.uint64)
    for i, c in enumerate(covers):
        off[i + 1] = off[i] + len(c)
    pcs = np.concatenate([np.asarray(c, dtype=np.uint32) for c in covers]) if covers else np.zeros(0, np.uint32)
    return np.ascontiguousarray(pcs, dtype=np.uint32), off


def minimize(covers=None, pcs=None, off=None):
    if covers is not None:
        pcs, off = to_csr(covers)
    n = off.size - 1
    out = np.empty(max(n, 1), dtype=np.int64)
    m = ctypes.c_size_t()
    _check(lib().oracle_minimize(_p(pcs, _u32p), _p(off, _u64p), n, _p(out, _i64p), ctypes.byref(m)), "minimize")
    return out[: m.value].copy()


def minimize_grouped(pcs, off, group, ngroups):
    n = off.size - 1
    group = np.ascontiguousarray(group, dtype=np.uint32)
    out = np.empty(max(n, 1), dtype=np.int64)
    goff = np.zeros(ngroups + 1, dtype=np.uint64)
    _check(lib().oracle_minimize_grouped(_p(pcs, _u32p), _p(off, _u64p), _p(group, _u32p), n, ngroups,
                                         _p(out, _i64p), _p(goff, _u64p)), "minimize_grouped")
    return out[: int(goff[-1])].copy(), goff


def minimize_grouped_mt(pcs, off, group, ngroups, nthreads):
    n = off.size - 1
    group = np.ascontiguousarray(group, dtype=np.uint32)
    out = np.empty(max(n, 1), dtype=np.int64)
    goff = np.zeros(ngroups + 1, dtype=np.uint64)
    f = lib().oracle_minimize_grouped_mt
    f.argtypes = [_u32p, _u64p, _u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int, _i64p, _u64p]
    _check(f(_p(pcs, _u32p), _p(off, _u64p), _p(group, _u32p), n, ngroups, int(nthreads), _p(out, _i64p),
             _p(goff, _u64p)), "minimize_grouped_mt")
    return out[: int(goff[-1])].copy(), goff


def set_go_sort_leaf(leaf):
    """The leaf form of the restated Go quickSort: 12 (default) or 7 (gosort.h)."""
    if lib().oracle_set_go_sort_leaf(int(leaf)) != 0:
        raise ValueError("leaf form must be 12 or 7")


def minimize_order(lens):
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    perm = np.empty(max(lens.size, 1), dtype=np.int64)
    _check(lib().oracle_minimize_order(_p(lens, _u64p), lens.size, _p(perm, _i64p)), "minimize_order")
    return perm[: lens.size].copy()


def dynamic_prio(prog_len, C):
    prog_len = np.ascontiguousarray(prog_len, dtype=np.uint16)
    out = np.empty((C, C), dtype=np.float32)
    _check(lib().oracle_dynamic_prio(_p(prog_len, _u16p), prog_len.size, C, _p(out, _f32p)), "dynamic_prio")
    return out


def call_cooccurrence(calls, off, C):
    """The call-ID form of prio.go:142-151: int32 C x C pair counts."""
    calls = np.ascontiguousarray(calls, dtype=np.uint16)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    out = np.empty((C, C), dtype=np.int32)
    _check(lib().oracle_call_cooccurrence(_p(calls, _u16p), _p(off, _u64p), off.size - 1, C,
                                          out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), "call_cooccurrence")
    return out


def normalize_prio(m):
    m = np.ascontiguousarray(m, dtype=np.float32).copy()
    lib().oracle_normalize_prio(_p(m, _f32p), m.shape[0])
    return m


def calculate_priorities(static, prog_len):
    static = np.ascontiguousarray(static, dtype=np.float32)
    C = static.shape[0]
    prog_len = np.ascontiguousarray(prog_len, dtype=np.uint16)
    out = np.empty((C, C), dtype=np.float32)
    _check(lib().oracle_calculate_priorities(_p(static, _f32p), _p(prog_len, _u16p), prog_len.size, C,
                                             _p(out, _f32p)), "calculate_priorities")
    return out


def static_priorities(uses, key_order=None, exact=False):
    """calcStaticPriorities (prio.go:40-135) of a nkeys x C usage matrix (oracle_static_priorities)."""
    uses = np.ascontiguousarray(uses, dtype=np.float32)
    nkeys, C = uses.shape
    ko = None if key_order is None else np.ascontiguousarray(key_order, dtype=np.int64)
    out = np.empty((C, C), dtype=np.float32)
    f = lib().oracle_static_priorities
    f.argtypes = [_f32p, ctypes.c_size_t, ctypes.c_int32, _i64p, ctypes.c_int, _f32p]
    _check(f(_p(uses, _f32p), nkeys, C, None if ko is None else _p(ko, _i64p), int(bool(exact)), _p(out, _f32p)),
           "static_priorities")
    return out


def build_choice_table(prios, enabled=None):
    prios = np.ascontiguousarray(prios, dtype=np.float32)
    C = prios.shape[0]
    run = np.empty((C, C), dtype=np.int64)
    present = np.empty(C, dtype=np.uint8)
    en = None if enabled is None else np.ascontiguousarray(enabled, dtype=np.uint8)
    _check(lib().oracle_build_choice_table(_p(prios, _f32p), None if en is None else _p(en, _u8p), C,
                                           _p(run, _i64p), _p(present, _u8p)), "build_choice_table")
    return run, present


def novelty(pcs, off, group, ngroups, mc, mc_off, flakes):
    n = off.size - 1
    group = np.ascontiguousarray(group, dtype=np.uint32)
    mc = np.ascontiguousarray(mc, dtype=np.uint32)
    mc_off = np.ascontiguousarray(mc_off, dtype=np.uint64)
    flakes = np.ascontiguousarray(flakes, dtype=np.uint32)
    is_new = np.zeros(max(n, 1), dtype=np.uint8)
    cap = int(mc.size + pcs.size + 1)
    out_mc = np.empty(cap, dtype=np.uint32)
    out_off = np.zeros(ngroups + 1, dtype=np.uint64)
    _check(lib().oracle_novelty(_p(pcs, _u32p), _p(off, _u64p), _p(group, _u32p), n, ngroups, _p(mc, _u32p),
                                _p(mc_off, _u64p), _p(flakes, _u32p), flakes.size, _p(is_new, _u8p),
                                _p(out_mc, _u32p), _p(out_off, _u64p), cap), "novelty")
    return is_new[:n].copy(), out_mc[: int(out_off[-1])].copy(), out_off


def novelty_mt(pcs, off, group, ngroups, mc, mc_off, flakes, nthreads=16):
    """oracle_novelty for canonical inputs, per-call first occurrence over nthreads host threads."""
    n = off.size - 1
    group = np.ascontiguousarray(group, dtype=np.uint32)
    mc = np.ascontiguousarray(mc, dtype=np.uint32)
    mc_off = np.ascontiguousarray(mc_off, dtype=np.uint64)
    flakes = np.ascontiguousarray(flakes, dtype=np.uint32)
    is_new = np.zeros(max(n, 1), dtype=np.uint8)
    cap = int(mc.size + pcs.size + 1)
    out_mc = np.empty(cap, dtype=np.uint32)
    out_off = np.zeros(ngroups + 1, dtype=np.uint64)
    f = lib().oracle_novelty_mt
    f.argtypes = [_u32p, _u64p, _u32p, ctypes.c_size_t, ctypes.c_uint32, _u32p, _u64p, _u32p, ctypes.c_size_t,
                  ctypes.c_int, _u8p, _u32p, _u64p, ctypes.c_size_t]
    _check(f(_p(pcs, _u32p), _p(off, _u64p), _p(group, _u32p), n, ngroups, _p(mc, _u32p), _p(mc_off, _u64p),
             _p(flakes, _u32p), flakes.size, int(nthreads), _p(is_new, _u8p), _p(out_mc, _u32p),
             _p(out_off, _u64p), cap), "novelty_mt")
    return is_new[:n].copy(), out_mc[: int(out_off[-1])].copy(), out_off


def prog_scan(data, off):
    """(ncalls u32[n], status u8[n]) per program of a CSR byte blob (oracle_prog_scan)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    n = off.size - 1
    nc = np.zeros(max(n, 1), np.uint32)
    st = np.zeros(max(n, 1), np.uint8)
    L = lib()
    base = data.ctypes.data
    for i in range(n):
        b = int(off[i])
        L.oracle_prog_scan(ctypes.cast(base + b, _u8p), int(off[i + 1]) - b,
                           ctypes.cast(nc.ctypes.data + 4 * i, ctypes.POINTER(ctypes.c_uint32)),
                           ctypes.cast(st.ctypes.data + i, _u8p))
    return nc[:n].copy(), st[:n].copy()


def sha1(data, off):
    """sigs u8[n, 20] (oracle_sha1 per program)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    n = off.size - 1
    sig = np.zeros((max(n, 1), 20), np.uint8)
    L = lib()
    base = data.ctypes.data
    for i in range(n):
        b = int(off[i])
        L.oracle_sha1(ctypes.cast(base + b, _u8p), int(off[i + 1]) - b, ctypes.cast(sig.ctypes.data + 20 * i, _u8p))
    return sig[:n].copy()


def cover_stats(pcs, off, group, ngroups):
    """syz-manager/html.go analytics (see oracle_cover_stats): dict of numpy arrays."""
    pcs = np.ascontiguousarray(pcs, dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    group = np.ascontiguousarray(group, dtype=np.uint32)
    n = off.size - 1
    ci, cc, cu = (np.zeros(max(ngroups, 1), dtype=np.uint64) for _ in range(3))
    tot = np.zeros(3, dtype=np.uint64)
    iu = np.zeros(max(n, 1), dtype=np.uint32)
    _check(lib().oracle_cover_stats(_p(pcs, _u32p), _p(off, _u64p), _p(group, _u32p), n, ngroups, _p(ci, _u64p),
                                    _p(cc, _u64p), _p(cu, _u64p), _p(tot, _u64p), _p(iu, _u32p)), "cover_stats")
    return dict(call_inputs=ci[:ngroups], call_cover=cc[:ngroups], call_unique=cu[:ngroups], totals=tot,
                input_unique=iu[:n])


def corpus_cover(pcs, off, group, ngroups, call, unique):
    pcs = np.ascontiguousarray(pcs, dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    group = np.ascontiguousarray(group, dtype=np.uint32)
    out = np.empty(pcs.size + 1, dtype=np.uint32)
    m = ctypes.c_size_t()
    _check(lib().oracle_corpus_cover(_p(pcs, _u32p), _p(off, _u64p), _p(group, _u32p), off.size - 1, ngroups, call,
                                     unique, _p(out, _u32p), out.size, ctypes.byref(m)), "corpus_cover")
    return out[: m.value].copy()
