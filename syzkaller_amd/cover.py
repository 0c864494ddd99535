"""Host mirror of the reference's `cover` package (cover/cover.go) over libsyzgpu.so.

Same names and argument meaning as the Go API; every compute call runs on the MI355X:

    Canonicalize(cov)            cover.go:28   sorts + dedups IN PLACE, returns cov[:n] (aliases)
    Difference(a, b)             cover.go:42
    SymmetricDifference(a, b)    cover.go:51
    Union(a, b)                  cover.go:63
    Intersection(a, b)           cover.go:72
    Minimize(corpus)             cover.go:105  -> list of kept indices in selection order
    Copy(cov), RestorePC(pc, base)  cover.go:19-25 (trivial, host)

Batched forms serve the manager/fuzzer loops that call these per input:
    MinimizeCorpus(pcs, off, group, ngroups)   syz-manager/manager.go:507-527
    SetOpBatch(op, a_list, b_list)             one launch for many pairs
    CanonicalizeBatch(pcs, off)
    NoveltyBatch(...)                          syz-fuzzer/fuzzer.go:446-470
    CoverStore(...)                            the resident mgr.corpus: Minimize, and the manager's cover
                                               analytics CoverStats / Cover / UniqueCover (html.go)
Covers are numpy uint32 arrays. Go's nil result is returned as an empty array.
"""
import numpy as np

from . import _lib
from ._lib import ECAPACITY, check, lib, ptr

SENT = 0xFFFFFFFF  # cover.go:17


def _u32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def Copy(cov):
    return _u32(cov).copy()


def RestorePC(pc, base):
    return (int(base) << 32) + int(pc)


def Canonicalize(cov):
    """In place like Go: cov must be a writable uint32 numpy array; returns cov[:n]."""
    if not (isinstance(cov, np.ndarray) and cov.dtype == np.uint32 and cov.flags.c_contiguous):
        cov = _u32(cov).copy()
    n = np.zeros(1, dtype=np.uint64)
    check(lib().syzgpu_canonicalize(ptr(cov), cov.size, ptr(n)))
    return cov[: int(n[0])]


def _pair(fn, cap_of, a, b):
    a, b = _u32(a), _u32(b)
    cap = cap_of(a.size, b.size)
    out = np.empty(max(cap, 1), dtype=np.uint32)
    n = np.zeros(1, dtype=np.uint64)
    check(fn(ptr(a), a.size, ptr(b), b.size, ptr(out), cap, ptr(n)))
    return out[: int(n[0])].copy()


def Difference(a, b):
    return _pair(lib().syzgpu_difference, lambda x, y: x, a, b)


def SymmetricDifference(a, b):
    return _pair(lib().syzgpu_symmetric_difference, lambda x, y: x + y, a, b)


def Union(a, b):
    return _pair(lib().syzgpu_union, lambda x, y: x + y, a, b)


def Intersection(a, b):
    return _pair(lib().syzgpu_intersection, lambda x, y: min(x, y), a, b)


def to_csr(covers):
    off = np.zeros(len(covers) + 1, dtype=np.uint64)
    if covers:
        np.cumsum([len(c) for c in covers], out=off[1:])
    pcs = np.concatenate([_u32(c) for c in covers]) if covers else np.zeros(0, np.uint32)
    return np.ascontiguousarray(pcs, dtype=np.uint32), off


def SetGoSortLeaf(leaf):
    """The leaf form of the restated Go quickSort that Minimize's tie order follows (cover.go:113):
    12 (the default: `for b-a > 12`, a gap-6 shell pass, insertionSort) or 7 (`for b-a > 7`,
    insertionSort alone). Process-wide (syzgpu_set_go_sort_leaf)."""
    check(lib().syzgpu_set_go_sort_leaf(int(leaf)))


def GoSortLeaf():
    return int(lib().syzgpu_go_sort_leaf())


def Minimize(corpus):
    """cover.go:105 — corpus is a list of covers; returns the kept indices in Go's order."""
    pcs, off = to_csr(corpus)
    n = len(corpus)
    out = np.empty(max(n, 1), dtype=np.int64)
    m = np.zeros(1, dtype=np.uint64)
    check(lib().syzgpu_minimize(ptr(pcs), ptr(off), n, ptr(out), ptr(m)))
    return [int(x) for x in out[: int(m[0])]]


def MinimizeCorpus(pcs, off, group, ngroups):
    """minimizeCorpus (manager.go:507-527): returns (kept entry ids group-major, group offsets)."""
    pcs, off = _u32(pcs), np.ascontiguousarray(off, dtype=np.uint64)
    group = _u32(group)
    n = off.size - 1
    out = np.empty(max(n, 1), dtype=np.int64)
    goff = np.zeros(ngroups + 1, dtype=np.uint64)
    check(lib().syzgpu_minimize_grouped(ptr(pcs), ptr(off), ptr(group), n, ngroups, ptr(out), ptr(goff)))
    return out[: int(goff[-1])].copy(), goff


def MinimizeCorpusDev(d_pcs, d_off, d_group, n, ngroups, d_prog_len=None, C=0, d_selected=None, d_len_hist=None,
                      d_out_idx=None, d_group_out_off=None, stream=0):
    """minimizeCorpus on device-resident covers (torch tensors / device pointers), every output on the
    device: kept flags, the len(p.Calls) histogram of kept programs, and the group-major kept list in
    Go's selection order with its group offsets (syzgpu_minimize_grouped_ordered_dev)."""
    check(lib().syzgpu_minimize_grouped_ordered_dev(ptr(d_pcs), ptr(d_off), ptr(d_group), ptr(d_prog_len), n,
                                                    ngroups, C, ptr(d_selected), ptr(d_len_hist), ptr(d_out_idx),
                                                    ptr(d_group_out_off), stream))


class MultiMinimizeJob:
    """minimizeCorpus over several GPUs of one node inside the library (syzgpu_mgz_*): the library plans
    the split (call groups whole, the heaviest split by PC ranges), uploads each device's share at load,
    and runs every sub-job on a thread of its own with the exchange (peer copies + MAX) and the
    histogram sum inside. devices may repeat (two sub-jobs on device 0 exercise the exchange on one GPU)."""

    def __init__(self, devices):
        d = np.ascontiguousarray(devices, np.int32)
        h = np.zeros(1, np.uint64)
        check(lib().syzgpu_mgz_create(ptr(d), d.size, ptr(h)))
        self._h = int(h[0])
        self.ngroups = 0
        self.n = 0

    def load(self, pcs, off, group, prog_len, ngroups, split_largest=0):
        pcs = np.ascontiguousarray(pcs, np.uint32)
        off = np.ascontiguousarray(off, np.uint64)
        group = np.ascontiguousarray(group, np.uint32)
        prog_len = np.ascontiguousarray(prog_len, np.uint16)
        self.n = off.size - 1
        self.ngroups = ngroups
        check(lib().syzgpu_mgz_load(self._h, ptr(pcs), ptr(off), ptr(group), ptr(prog_len), self.n, ngroups,
                                    split_largest))

    def minimize_prio(self, C, uses=None):
        """(kept ids group-major, group offsets, len_hist, prios, run, row_present); prios/run/row_present
        are None without a usage matrix."""
        out = np.zeros(max(self.n, 1), np.int64)
        goff = np.zeros(self.ngroups + 1, np.uint64)
        hist = np.zeros(C + 1, np.int64)
        prios = run = rowp = None
        nkeys = 0
        if uses is not None:
            uses = np.ascontiguousarray(uses, np.float32)
            nkeys = uses.shape[0]
            prios = np.zeros((C, C), np.float32)
            run = np.zeros((C, C), np.int64)
            rowp = np.zeros(C, np.uint8)
        check(lib().syzgpu_mgz_minimize_prio(self._h, C, ptr(uses), nkeys, ptr(out), ptr(goff), ptr(hist),
                                             ptr(prios), ptr(run), ptr(rowp)))
        return out[:int(goff[-1])].copy(), goff, hist, prios, run, rowp

    def info(self):
        v = np.zeros(5 + 64, np.uint64)
        check(lib().syzgpu_mgz_info(self._h, ptr(v), v.size))
        nd = int(v[0])
        return {"subjobs": nd, "groups": int(v[1]), "entries": int(v[2]), "split_groups": int(v[3]),
                "exchange_bytes": int(v[4]), "subjob_entries": [int(x) for x in v[5:5 + nd]]}

    def close(self):
        if self._h:
            lib().syzgpu_mgz_destroy(self._h)
            self._h = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def plan_parts(entries, pcs, nranks, split_largest=0):
    """The library's key-space plan (host only, no device): (ranks per group, modelled cost per rank)."""
    e = np.ascontiguousarray(entries, np.int64)
    p = np.ascontiguousarray(pcs, np.float64)
    ranks = np.full((e.size, nranks), -1, np.int32)
    cost = np.zeros(nranks, np.float64)
    check(lib().syzgpu_plan_parts(ptr(e), ptr(p), e.size, nranks, split_largest, ptr(ranks), ptr(cost)))
    return [tuple(int(x) for x in row if x >= 0) for row in ranks], cost


def plan_split_bounds(pcs, off, group, g, k):
    """The library's PC bounds of group g's k parts (host only)."""
    pcs = np.ascontiguousarray(pcs, np.uint32)
    off = np.ascontiguousarray(off, np.uint64)
    group = np.ascontiguousarray(group, np.uint32)
    b = np.zeros(k + 1, np.uint64)
    check(lib().syzgpu_plan_split_bounds(ptr(pcs), ptr(off), ptr(group), off.size - 1, g, k, ptr(b)))
    return b


class MinimizeJob:
    """minimizeCorpus as a job on device-resident covers (syzgpu_mz_*): begin, an optional exchange of
    split groups' selections, end. key_lo/key_hi (per group, numpy u32) restrict this rank to a PC
    range of each group (a key part); both None = whole groups."""

    def __init__(self):
        h = np.zeros(1, np.uint64)
        check(lib().syzgpu_mz_create(ptr(h)))
        self._h = int(h[0])

    @property
    def handle(self):
        return self._h

    def begin(self, d_pcs, d_off, d_group, n, ngroups, d_prog_len=None, key_lo=None, key_hi=None, stream=0):
        self._keys = (None if key_lo is None else np.ascontiguousarray(key_lo, np.uint32),
                      None if key_hi is None else np.ascontiguousarray(key_hi, np.uint32))
        check(lib().syzgpu_mz_begin_dev(self._h, ptr(d_pcs), ptr(d_off), ptr(d_group), ptr(d_prog_len), n, ngroups,
                                        ptr(self._keys[0]), ptr(self._keys[1]), stream))

    def export_sel(self, groups, offsets, buf, stream=0):
        g, o = np.ascontiguousarray(groups, np.uint32), np.ascontiguousarray(offsets, np.uint64)
        check(lib().syzgpu_mz_export_sel_dev(self._h, ptr(g), ptr(o), g.size, ptr(buf), stream))

    def import_sel(self, groups, offsets, buf, stream=0):
        g, o = np.ascontiguousarray(groups, np.uint32), np.ascontiguousarray(offsets, np.uint64)
        check(lib().syzgpu_mz_import_sel_dev(self._h, ptr(g), ptr(o), g.size, ptr(buf), stream))

    def end(self, C=0, count_hist=None, d_selected=None, d_len_hist=None, d_out_idx=None, d_group_out_off=None,
            stream=0):
        ch = None if count_hist is None else np.ascontiguousarray(count_hist, np.uint8)
        check(lib().syzgpu_mz_end_dev(self._h, C, ptr(ch), ptr(d_selected), ptr(d_len_hist), ptr(d_out_idx),
                                      ptr(d_group_out_off), stream))

    def end_prio(self, C, d_uses, nkeys, d_static, d_prios, d_run, count_hist=None, d_selected=None,
                 d_len_hist=None, d_out_idx=None, d_group_out_off=None, d_row_present=None, stream=0):
        """minimizeCorpus's tail (manager.go:523-536): end() + calcStaticPriorities + CalculatePriorities
        + BuildChoiceTable in one call, on device buffers."""
        ch = None if count_hist is None else np.ascontiguousarray(count_hist, np.uint8)
        check(lib().syzgpu_mz_end_prio_dev(self._h, C, ptr(ch), ptr(d_selected), ptr(d_len_hist), ptr(d_out_idx),
                                           ptr(d_group_out_off), ptr(d_uses), nkeys, ptr(d_static), ptr(d_prios),
                                           ptr(d_run), ptr(d_row_present), stream))

    def fetch(self, n, ngroups):
        out = np.empty(max(n, 1), np.int64)
        goff = np.zeros(ngroups + 1, np.uint64)
        check(lib().syzgpu_mz_fetch(self._h, ptr(out), ptr(goff)))
        return out[: int(goff[-1])].copy(), goff

    def info(self):
        v = np.zeros(7, np.uint64)
        check(lib().syzgpu_mz_info(self._h, ptr(v), 7))
        return dict(zip(["entries", "groups", "pcs", "direct_windows", "hash_windows", "spec_hits", "spec_misses"],
                        (int(x) for x in v)))

    def close(self):
        if self._h:
            lib().syzgpu_mz_destroy(self._h)
            self._h = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def MinimizeOrder(lens, group_off=None):
    """cover.go:106-113: Go sort.Sort order of Minimize's inputs per group (index inside the group of
    the input at each sorted position), for cover lengths `lens` split by `group_off`."""
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    if group_off is None:
        group_off = np.array([0, lens.size], dtype=np.uint64)
    group_off = np.ascontiguousarray(group_off, dtype=np.uint64)
    perm = np.empty(max(lens.size, 1), dtype=np.int64)
    check(lib().syzgpu_minimize_order(ptr(lens), ptr(group_off), group_off.size - 1, ptr(perm)))
    return perm[: lens.size].copy()


_OPS = {"difference": _lib.DIFFERENCE, "symmetric_difference": _lib.SYMMETRIC_DIFFERENCE,
        "union": _lib.UNION, "intersection": _lib.INTERSECTION}


def SetOpBatch(op, a_list, b_list):
    """op(a_i, b_i) for every pair in one launch; returns a list of arrays."""
    code = _OPS[op] if isinstance(op, str) else int(op)
    a, aoff = to_csr(list(a_list))
    b, boff = to_csr(list(b_list))
    npairs = len(a_list)
    cap = {0: a.size, 1: a.size + b.size, 2: a.size + b.size, 3: min(a.size, b.size)}[code]
    out = np.empty(max(cap, 1), dtype=np.uint32)
    ooff = np.zeros(npairs + 1, dtype=np.uint64)
    check(lib().syzgpu_setop_batch(code, ptr(a), ptr(aoff), ptr(b), ptr(boff), npairs, ptr(out), cap, ptr(ooff)))
    return [out[int(ooff[i]):int(ooff[i + 1])].copy() for i in range(npairs)]


def SetOpBatchDev(op, a, aoff, na, b, boff, nb, npairs, out, out_cap, ooff, stream=None):
    """op(a_i, b_i) for npairs pairs of device-resident CSRs (torch tensors or device pointers):
    out / ooff on the device; returns the total output length."""
    import ctypes
    code = _OPS[op] if isinstance(op, str) else int(op)
    tot = ctypes.c_uint64(0)
    check(lib().syzgpu_setop_batch_dev(code, ptr(a), ptr(aoff), na, ptr(b), ptr(boff), nb, npairs, ptr(out),
                                       out_cap, ptr(ooff), stream, ctypes.byref(tot)))
    return int(tot.value)


def CanonicalizeBatch(pcs, off):
    """Canonicalize every cover of a CSR in place; returns the new lengths."""
    off = np.ascontiguousarray(off, dtype=np.uint64)
    n = off.size - 1
    lens = np.zeros(max(n, 1), dtype=np.uint64)
    check(lib().syzgpu_canonicalize_batch(ptr(pcs), ptr(off), n, ptr(lens)))
    return lens[:n]


def CanonicalizeBatchDev(pcs, off, ncov, out_len, stream=None):
    """Canonicalize every cover of a device-resident CSR in place (torch tensors or device pointers);
    out_len (device, u64[ncov]) receives the new lengths."""
    check(lib().syzgpu_canonicalize_batch_dev(ptr(pcs), ptr(off), ncov, ptr(out_len), stream))


def NoveltyBatch(pcs, off, group, ngroups, maxcover_pcs, maxcover_off, flakes):
    """fuzzer.go:446-470 over a batch: returns (is_new u8[n], new maxCover CSR pcs, offsets)."""
    pcs, off, group = _u32(pcs), np.ascontiguousarray(off, dtype=np.uint64), _u32(group)
    mc, mco, fl = _u32(maxcover_pcs), np.ascontiguousarray(maxcover_off, dtype=np.uint64), _u32(flakes)
    n = off.size - 1
    is_new = np.zeros(max(n, 1), dtype=np.uint8)
    cap = int(mc.size + pcs.size + 1)
    out = np.empty(cap, dtype=np.uint32)
    ooff = np.zeros(ngroups + 1, dtype=np.uint64)
    check(lib().syzgpu_novelty_batch(ptr(pcs), ptr(off), ptr(group), n, ngroups, ptr(mc), ptr(mco), ptr(fl),
                                     fl.size, ptr(is_new), ptr(out), cap, ptr(ooff)))
    return is_new[:n].copy(), out[: int(ooff[-1])].copy(), ooff


def NoveltyBatchDev(pcs, off, group, n, ngroups, mc, mc_off, mc_total, flakes, nflakes, total_pcs, is_new, out_mc,
                    out_cap, out_mc_off, stream=0):
    """NoveltyBatch on device-resident arrays (torch tensors or device pointers); outputs stay on the
    device (out_mc_off[ngroups] = the updated tables' total)."""
    check(lib().syzgpu_novelty_batch_dev(ptr(pcs), ptr(off), ptr(group), n, ngroups, ptr(mc), ptr(mc_off), mc_total,
                                         ptr(flakes), nflakes, total_pcs, ptr(is_new), ptr(out_mc), out_cap,
                                         ptr(out_mc_off), stream))


class CoverStore:
    """Device-resident corpus (the analog of syz-manager's mgr.corpus): ingest once, then Minimize
    every call group as often as the manager needs (manager.go:507-527 on each Connect / hub sync).
    Covers must be canonical (as the executor produces them)."""

    def __init__(self, pcs, off, group, ngroups, prog_len=None):
        pcs, off, group = _u32(pcs), np.ascontiguousarray(off, dtype=np.uint64), _u32(group)
        pl = None if prog_len is None else np.ascontiguousarray(prog_len, dtype=np.uint16)
        h = np.zeros(1, dtype=np.uint64)
        check(lib().syzgpu_corpus_create(ptr(pcs), ptr(off), ptr(group), ptr(pl), off.size - 1, ngroups, ptr(h)))
        self._h = int(h[0])
        self.n = off.size - 1
        self.ngroups = ngroups

    @classmethod
    def from_device(cls, d_pcs, d_off, d_group, d_prog_len, n, ngroups, stream=0):
        self = cls.__new__(cls)
        h = np.zeros(1, dtype=np.uint64)
        check(lib().syzgpu_corpus_create_dev(ptr(d_pcs), ptr(d_off), ptr(d_group), ptr(d_prog_len), n, ngroups,
                                             stream, ptr(h)))
        self._h, self.n, self.ngroups = int(h[0]), n, ngroups
        return self

    def append(self, pcs, off, group, prog_len=None):
        """mgr.corpus = append(mgr.corpus, inputs...) (NewInput, manager.go:609-616): the covers are
        appended in place on the device, O(new); Minimize then runs on the raw pipeline until a reindex."""
        pcs, off, group = _u32(pcs), np.ascontiguousarray(off, dtype=np.uint64), _u32(group)
        pl = None if prog_len is None else np.ascontiguousarray(prog_len, dtype=np.uint16)
        h = np.zeros(1, dtype=np.uint64)
        check(lib().syzgpu_corpus_append(self._h, ptr(pcs), ptr(off), ptr(group), ptr(pl), off.size - 1, ptr(h)))
        self._h = int(h[0])
        self.n += off.size - 1
        return self

    def append_device(self, d_pcs, d_off, d_group, d_prog_len, n, stream=0):
        h = np.zeros(1, dtype=np.uint64)
        check(lib().syzgpu_corpus_append_dev(self._h, ptr(d_pcs), ptr(d_off), ptr(d_group), ptr(d_prog_len), n,
                                             stream, ptr(h)))
        self._h = int(h[0])
        self.n += n
        return self

    def NewInputs(self, pcs, off, group, prog_len=None):
        """NewInput's gate (manager.go:609-616) over a batch: inputs whose cover adds a PC to corpusCover
        of their call (earlier new inputs of the batch included) are appended and unioned in. Returns
        is_new (bool per input)."""
        pcs, off, group = _u32(pcs), np.ascontiguousarray(off, dtype=np.uint64), _u32(group)
        pl = None if prog_len is None else np.ascontiguousarray(prog_len, dtype=np.uint16)
        n = off.size - 1
        is_new = np.zeros(max(n, 1), dtype=np.uint8)
        acc = np.zeros(1, dtype=np.uint64)
        check(lib().syzgpu_corpus_new_inputs(self._h, ptr(pcs), ptr(off), ptr(group), ptr(pl), n, ptr(is_new),
                                             ptr(acc)))
        self.n += int(acc[0])
        return is_new[:n].astype(bool)

    def NewInputsDevice(self, d_pcs, d_off, d_group, d_prog_len, n, d_is_new=None, stream=0):
        """NewInputs on device buffers; returns the number appended."""
        acc = np.zeros(1, dtype=np.uint64)
        check(lib().syzgpu_corpus_new_inputs_dev(self._h, ptr(d_pcs), ptr(d_off), ptr(d_group), ptr(d_prog_len), n,
                                                 ptr(d_is_new), stream, ptr(acc)))
        self.n += int(acc[0])
        return int(acc[0])

    def CorpusCover(self):
        """mgr.corpusCover (manager.go:65): per call the sorted PCs, as (pcs, off[ngroups + 1])."""
        tot = np.zeros(1, dtype=np.uint64)
        off = np.zeros(self.ngroups + 1, dtype=np.uint64)
        cap = 1 << 16
        while True:
            out = np.empty(cap, dtype=np.uint32)
            rc = lib().syzgpu_corpus_cover_union(self._h, ptr(out), ptr(off), cap, ptr(tot))
            if rc == ECAPACITY and int(tot[0]) > cap:
                cap = int(tot[0])
                continue
            check(rc)
            return out[: int(tot[0])].copy(), off

    def keep(self, idx):
        """mgr.corpus = newCorpus (manager.go:529): the corpus becomes entries idx, in that order."""
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        check(lib().syzgpu_corpus_keep(self._h, ptr(idx), idx.size))
        self.n = idx.size
        return self

    def keep_device(self, d_idx, m, stream=0):
        check(lib().syzgpu_corpus_keep_dev(self._h, ptr(d_idx), m, stream))
        self.n = m
        return self

    def MinimizeKeep(self, C=0, d_selected=None, d_len_hist=None, d_out_idx=None, d_group_out_off=None, stream=0):
        """The manager's minimizeCorpus (manager.go:507-529): Minimize every call, then keep the selected
        entries in Go's order. The optional device outputs describe the corpus before the keep."""
        kept = np.zeros(1, dtype=np.uint64)
        check(lib().syzgpu_corpus_minimize_keep_dev(self._h, C, ptr(d_selected), ptr(d_len_hist), ptr(d_out_idx),
                                                    ptr(d_group_out_off), stream, ptr(kept)))
        self.n = int(kept[0])
        return self.n

    def reindex(self, stream=0):
        check(lib().syzgpu_corpus_reindex(self._h, stream))

    @property
    def handle(self):
        return self._h

    def info(self):
        v = np.zeros(12, dtype=np.uint64)
        check(lib().syzgpu_corpus_info(self._h, ptr(v), 12))
        return dict(zip(["entries", "calls", "pcs", "ids", "work_items", "shared_tables", "vectors",
                         "big_entries", "big_pcs", "big_vecs", "big_vecs_all", "indexed"], (int(x) for x in v)))

    # ---- key-space sharding (the multi-GPU form of minimizeCorpus, syzkaller_amd/sharding.py) ----
    def set_parts(self, part, nparts, count_hist=None):
        """Keep part[g] of nparts[g] of every call group's dense-PC windows (see syzgpu.h)."""
        part = np.ascontiguousarray(part, dtype=np.uint16)
        nparts = np.ascontiguousarray(nparts, dtype=np.uint16)
        ch = None if count_hist is None else np.ascontiguousarray(count_hist, dtype=np.uint8)
        check(lib().syzgpu_corpus_set_parts(self._h, ptr(part), ptr(nparts), ptr(ch)))

    def minimize_begin(self, stream=0):
        check(lib().syzgpu_corpus_minimize_begin_dev(self._h, stream))

    def export_sel(self, groups, offsets, buf, stream=0):
        g = np.ascontiguousarray(groups, dtype=np.uint32)
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        check(lib().syzgpu_corpus_export_sel_dev(self._h, ptr(g), ptr(o), g.size, ptr(buf), stream))

    def import_sel(self, groups, offsets, buf, stream=0):
        g = np.ascontiguousarray(groups, dtype=np.uint32)
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        check(lib().syzgpu_corpus_import_sel_dev(self._h, ptr(g), ptr(o), g.size, ptr(buf), stream))

    def minimize_end(self, C, selected=None, len_hist=None, stream=0):
        check(lib().syzgpu_corpus_minimize_end_dev(self._h, C, ptr(selected), ptr(len_hist), stream))

    def Minimize(self):
        out = np.empty(max(self.n, 1), dtype=np.int64)
        goff = np.zeros(self.ngroups + 1, dtype=np.uint64)
        check(lib().syzgpu_corpus_minimize(self._h, ptr(out), ptr(goff)))
        return out[: int(goff[-1])].copy(), goff

    # ---- the manager's cover analytics (syz-manager/html.go) ----
    def CoverStats(self):
        """html.go:67-97 per call (Inputs, Cover, UniqueCover), the "cover" stat, len(uniqueCover(perCall))
        (html.go:213-237) and httpCorpus's per-input UniqueCover (html.go:158-170), in one GPU pass."""
        G, n = self.ngroups, self.n
        ci, cc, cu = (np.zeros(max(G, 1), dtype=np.uint64) for _ in range(3))
        tot = np.zeros(3, dtype=np.uint64)
        iu = np.zeros(max(n, 1), dtype=np.uint32)
        check(lib().syzgpu_corpus_cover_stats(self._h, ptr(ci), ptr(cc), ptr(cu), ptr(tot), ptr(iu)))
        return dict(call_inputs=ci[:G], call_cover=cc[:G], call_unique=cu[:G], cover=int(tot[0]),
                    unique_per_call=int(tot[1]), unique_per_input=int(tot[2]), input_unique=iu[:n])

    def Cover(self, call=-1, unique=0):
        """httpCover's PC list (html.go:186-211): call >= 0 -> that call's Union [∩ uniqueCover(unique == 1)];
        call < 0 -> the Union of all calls (unique = 0) or uniqueCover(unique == 1) itself."""
        L = lib()
        m = np.zeros(1, dtype=np.uint64)
        cap = 1 << 16
        while True:
            out = np.empty(cap, dtype=np.uint32)
            rc = L.syzgpu_corpus_cover(self._h, call, unique, ptr(out), cap, ptr(m))
            if rc == ECAPACITY and int(m[0]) > cap:
                cap = int(m[0])
                continue
            check(rc)
            return out[: int(m[0])].copy()

    def UniqueCover(self, perCall):
        """html.go:213-237 uniqueCover(perCall)."""
        return self.Cover(-1, 1 if perCall else 2)

    def close(self):
        if getattr(self, "_h", 0):
            lib().syzgpu_corpus_destroy(self._h)
            self._h = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
