"""Seeded synthetic corpora (bench / test inputs). Wraps libsyzsynth.so."""
import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class Params(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("n", ctypes.c_uint64),
        ("ngroups", ctypes.c_uint32),
        ("npcs", ctypes.c_uint32),
        ("zipf_s", ctypes.c_double),
        ("len_median", ctypes.c_double),
        ("len_sigma", ctypes.c_double),
        ("len_max", ctypes.c_uint32),
        ("prog_len_max", ctypes.c_uint32),
        ("hot_frac", ctypes.c_double),
        ("hot_space", ctypes.c_double),
        ("hot_exponent", ctypes.c_double),
        ("prog_len_p", ctypes.c_double),
    ]


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libsyzsynth.so")
        if not os.path.exists(path):
            raise RuntimeError("syzkaller_amd/libsyzsynth.so not built (run __graft_entry__.build())")
        L = ctypes.CDLL(path)
        L.syzgpu_synth_default_params.argtypes = [ctypes.POINTER(Params), ctypes.c_uint64, ctypes.c_uint64,
                                                  ctypes.c_uint32, ctypes.c_uint32]
        L.syzgpu_synth_default_params.restype = None
        L.syzgpu_synth_layout.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]
        L.syzgpu_synth_fill.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int]
        L.syzgpu_synth_fill_ids.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
        L.syzgpu_synth_prog_text.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_int]
        _LIB = L
    return _LIB


@dataclass
class Corpus:
    pcs: np.ndarray       # uint32[sum L]  concatenated sorted covers
    off: np.ndarray       # uint64[n+1]    CSR offsets
    group: np.ndarray     # uint32[n]      call (CallName) id
    prog_len: np.ndarray  # uint16[n]      len(p.Calls)
    ngroups: int

    @property
    def n(self):
        return self.off.size - 1

    def cover(self, i):
        return self.pcs[int(self.off[i]):int(self.off[i + 1])]


def params(seed, n, ngroups=289, npcs=50_000, **kw):
    p = Params()
    _lib().syzgpu_synth_default_params(ctypes.byref(p), seed, n, ngroups, npcs)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def corpus(seed, n, ngroups=289, npcs=50_000, nthreads=None, **kw):
    p = params(seed, n, ngroups, npcs, **kw)
    group = np.empty(n, dtype=np.uint32)
    off = np.empty(n + 1, dtype=np.uint64)
    plen = np.empty(n, dtype=np.uint16)
    rc = _lib().syzgpu_synth_layout(ctypes.byref(p), group.ctypes.data, off.ctypes.data, plen.ctypes.data)
    if rc:
        raise ValueError("bad synth params")
    pcs = np.empty(int(off[-1]), dtype=np.uint32)
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    rc = _lib().syzgpu_synth_fill(ctypes.byref(p), group.ctypes.data, off.ctypes.data, pcs.ctypes.data,
                                  nthreads)
    if rc:
        raise ValueError("bad synth params")
    return Corpus(pcs, off, group, plen, ngroups)


def layout(p):
    """(group u32[n], off u64[n+1], prog_len u16[n]) of the corpus described by params p."""
    n = int(p.n)
    group = np.empty(n, dtype=np.uint32)
    off = np.empty(n + 1, dtype=np.uint64)
    plen = np.empty(n, dtype=np.uint16)
    if _lib().syzgpu_synth_layout(ctypes.byref(p), group.ctypes.data, off.ctypes.data, plen.ctypes.data):
        raise ValueError("bad synth params")
    return group, off, plen


def subcorpus(p, ids, group, off, plen, nthreads=None):
    """The entries `ids` (ascending global ids) of the corpus p, as a Corpus of their own."""
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    lens = (off[1:] - off[:-1])[ids]
    soff = np.zeros(ids.size + 1, dtype=np.uint64)
    np.cumsum(lens, out=soff[1:])
    sgroup = np.ascontiguousarray(group[ids])
    pcs = np.empty(int(soff[-1]), dtype=np.uint32)
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    if _lib().syzgpu_synth_fill_ids(ctypes.byref(p), ids.ctypes.data, sgroup.ctypes.data, soff.ctypes.data,
                                    ids.size, pcs.ctypes.data, nthreads):
        raise ValueError("bad synth params")
    return Corpus(pcs, soff, sgroup, np.ascontiguousarray(plen[ids]), int(p.ngroups))


def prog_text(seed, prog_len, nthreads=None):
    """Serialized programs with exactly prog_len[i] calls each: (data uint8[], off uint64[n+1])."""
    prog_len = np.ascontiguousarray(prog_len, dtype=np.uint16)
    n = prog_len.size
    nt = nthreads or min(16, os.cpu_count() or 1)
    off = np.zeros(n + 1, dtype=np.uint64)
    L = _lib()
    if L.syzgpu_synth_prog_text(seed, prog_len.ctypes.data, n, off.ctypes.data, None, nt):
        raise RuntimeError("synth prog_text failed")
    data = np.empty(int(off[-1]) + 4, dtype=np.uint8)
    if L.syzgpu_synth_prog_text(seed, prog_len.ctypes.data, n, off.ctypes.data, data.ctypes.data, nt):
        raise RuntimeError("synth prog_text failed")
    return data[: int(off[-1])], off
