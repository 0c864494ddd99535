"""The resident corpus's lifecycle, following mgr.corpus: appends on NewInput
(syz-manager/manager.go:609-616, syzgpu_corpus_append[_dev], in place), minimizeCorpus
(manager.go:507-527) and mgr.corpus = newCorpus (manager.go:529, syzgpu_corpus_keep /
_minimize_keep_dev). After every step the store's minimizeCorpus (on the stale-index raw pipeline or
on a rebuilt index) and its cover analytics must equal the oracle's over the same corpus, rebuilt
host-side by the same sequence of appends and keeps."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import cover, synth  # noqa: E402

pytestmark = pytest.mark.gpu


def _part(c, a, b):
    o = c.off[a:b + 1].astype(np.uint64)
    return c.pcs[int(o[0]):int(o[-1])], o - o[0], c.group[a:b], c.prog_len[a:b]


def _dev(a):
    import torch
    view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
    return torch.from_numpy(np.ascontiguousarray(a).view(view.get(a.dtype, a.dtype))).to("cuda:0")


def test_append_host_and_device_matches_oracle():
    import torch
    c = synth.corpus(0x5EED00A1, 30_000, 37, 200_000)
    k1, k2 = 17_000, 26_000
    st = cover.CoverStore(*_part(c, 0, k1)[:3], c.ngroups, _part(c, 0, k1)[3])
    st.append(*_part(c, k1, k2))                      # host pointers
    p, o, g, l = (_dev(x) for x in _part(c, k2, c.n))  # device pointers
    st.append_device(p, o, g, l, c.n - k2, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert st.info()["entries"] == c.n and st.info()["pcs"] == int(c.off[-1])
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    got, goff = st.Minimize()
    assert np.array_equal(wgoff, goff)
    assert np.array_equal(want, got)
    st.close()


def test_append_empty_and_to_empty():
    c = synth.corpus(0x5EED00A2, 5_000, 11, 40_000)
    st = cover.CoverStore(*_part(c, 0, 0)[:3], c.ngroups)  # an empty manager corpus
    st.append(*_part(c, 0, c.n))
    st.append(*_part(c, c.n, c.n))                         # NewInput of nothing
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    got, goff = st.Minimize()
    assert np.array_equal(want, got) and np.array_equal(wgoff, goff)
    st.close()


def test_append_rejects_bad_group_and_keeps_store():
    c = synth.corpus(0x5EED00A3, 4_000, 5, 30_000)
    st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
    before, bgoff = st.Minimize()
    pcs, off, grp, pl = _part(c, 0, 10)
    with pytest.raises(Exception):
        st.append(pcs, off, np.full_like(grp, c.ngroups), pl)
    after, agoff = st.Minimize()  # the old handle is still valid after a failed append
    assert np.array_equal(before, after) and np.array_equal(bgoff, agoff)
    st.close()


class HostCorpus:
    """The same corpus on the host (list of covers, call ids, program lengths)."""

    def __init__(self, c, a, b):
        self.covs = [c.pcs[int(c.off[i]):int(c.off[i + 1])] for i in range(a, b)]
        self.group = list(c.group[a:b])
        self.plen = list(c.prog_len[a:b])

    def append(self, c, a, b):
        other = HostCorpus(c, a, b)
        self.covs += other.covs
        self.group += other.group
        self.plen += other.plen

    def keep(self, idx):
        self.covs = [self.covs[i] for i in idx]
        self.group = [self.group[i] for i in idx]
        self.plen = [self.plen[i] for i in idx]

    def csr(self):
        pcs, off = oracle.to_csr(self.covs)
        return pcs, off, np.array(self.group, np.uint32), np.array(self.plen, np.uint16)


def _check(st, hc, G):
    pcs, off, grp, _ = hc.csr()
    want, wgoff = oracle.minimize_grouped(pcs, off, grp, G)
    got, goff = st.Minimize()
    assert np.array_equal(wgoff, goff) and np.array_equal(want, got)
    return want


def test_manager_cycle_append_minimize_keep_vs_oracle():
    import torch
    c = synth.corpus(0x5EED00A4, 60_000, 41, 300_000)
    G = c.ngroups
    C = int(c.prog_len.max())
    st = cover.CoverStore(*_part(c, 0, 20_000)[:3], G, _part(c, 0, 20_000)[3])
    hc = HostCorpus(c, 0, 20_000)
    assert st.info()["indexed"] == 1
    s = torch.cuda.current_stream().cuda_stream
    # NewInput x2 (host and device pointers): in place, the index follows (corpus_inc.hip)
    st.append(*_part(c, 20_000, 30_000))
    hc.append(c, 20_000, 30_000)
    p, o, g, l = (_dev(x) for x in _part(c, 30_000, 40_000))
    st.append_device(p, o, g, l, 10_000, s)
    hc.append(c, 30_000, 40_000)
    assert st.info()["indexed"] == 1 and st.info()["entries"] == 40_000
    _check(st, hc, G)  # on the appended index
    # minimizeCorpus + mgr.corpus = newCorpus in one call
    n0 = st.n
    sel = torch.zeros(n0, dtype=torch.uint8, device="cuda")
    hist = torch.zeros(C + 1, dtype=torch.int64, device="cuda")
    out = torch.zeros(n0, dtype=torch.int64, device="cuda")
    goff = torch.zeros(G + 1, dtype=torch.int64, device="cuda")
    kept = st.MinimizeKeep(C, sel, hist, out, goff, s)
    pcs, off, grp, pl = hc.csr()
    want, wgoff = oracle.minimize_grouped(pcs, off, grp, G)
    assert kept == want.size and np.array_equal(out.cpu().numpy()[:kept], want)
    assert np.array_equal(goff.cpu().numpy().astype(np.uint64), wgoff)
    assert np.array_equal(hist.cpu().numpy(), np.bincount(pl[want], minlength=C + 1))
    wsel = np.zeros(n0, np.uint8)
    wsel[want] = 1
    assert np.array_equal(sel.cpu().numpy(), wsel)
    hc.keep(want)
    assert st.info()["entries"] == kept and st.info()["pcs"] == sum(len(x) for x in hc.covs)
    assert st.info()["indexed"] == 1  # the keep compacted the index rather than dropping it
    _check(st, hc, G)  # the kept corpus minimizes to itself (every input was kept for a new PC)
    # more inputs after the keep, then an explicit keep in another order, then a reindex
    st.append(*_part(c, 40_000, 60_000))
    hc.append(c, 40_000, 60_000)
    _check(st, hc, G)
    perm = np.random.default_rng(1).permutation(len(hc.covs))[: len(hc.covs) // 2]
    st.keep(perm)
    hc.keep(perm)
    _check(st, hc, G)
    st.reindex()
    assert st.info()["indexed"] == 1
    _check(st, hc, G)
    # the analytics rebuild the index of the current covers themselves
    st.append(*_part(c, 0, 3_000))
    hc.append(c, 0, 3_000)
    pcs, off, grp, _ = hc.csr()
    w = oracle.cover_stats(pcs, off, grp, G)
    g = st.CoverStats()
    for k in ("call_inputs", "call_cover", "call_unique", "input_unique"):
        assert np.array_equal(np.asarray(g[k]), w[k]), k
    assert [g["cover"], g["unique_per_call"], g["unique_per_input"]] == [int(x) for x in w["totals"]]
    st.close()


@pytest.mark.parametrize("inc", [True, False])
def test_incremental_index_new_pcs_and_windows(inc, monkeypatch):
    # appends bring PCs the index has never seen (a wider PC space, few calls: their dense ids open
    # new 32K-id windows), keeps drop and reorder entries, one keep repeats an entry (the index cannot
    # follow it: it is dropped and built afresh); after every step the store minimizes like the oracle,
    # on the maintained index (inc) or on the raw pipeline (SYZGPU_NO_INC_INDEX=1)
    import torch
    if not inc:
        monkeypatch.setenv("SYZGPU_NO_INC_INDEX", "1")
    G = 5
    a = synth.corpus(0x5EED00B1, 8_000, G, 30_000)
    b = synth.corpus(0x5EED00B2, 12_000, G, 400_000)
    C = int(max(a.prog_len.max(), b.prog_len.max()))
    st = cover.CoverStore(a.pcs, a.off, a.group, G, a.prog_len)
    hc = HostCorpus(a, 0, a.n)
    s = torch.cuda.current_stream().cuda_stream
    for lo, hi in ((0, 3_000), (3_000, 3_001), (3_001, 3_001), (3_001, 9_000)):
        st.append(*_part(b, lo, hi))
        hc.append(b, lo, hi)
        assert st.info()["indexed"] == (1 if inc else 0)
        _check(st, hc, G)
    assert st.info()["entries"] == len(hc.covs)
    want = _check(st, hc, G)
    kept = st.MinimizeKeep(C, None, torch.zeros(C + 1, dtype=torch.int64, device="cuda"), None, None, s)
    assert kept == want.size
    hc.keep(want)
    _check(st, hc, G)
    st.append(*_part(b, 9_000, 12_000))
    hc.append(b, 9_000, 12_000)
    _check(st, hc, G)
    rnd = np.random.default_rng(5)
    perm = rnd.permutation(len(hc.covs))[: 2 * len(hc.covs) // 3]
    st.keep(perm)
    hc.keep(perm)
    _check(st, hc, G)
    st.append(*_part(a, 0, 500))
    hc.append(a, 0, 500)
    _check(st, hc, G)
    dup = np.concatenate([np.arange(100), [7]])  # entry 7 twice: the update fails, the index is rebuilt
    st.keep(dup)
    hc.keep(list(dup))
    _check(st, hc, G)
    st.close()


def test_keep_rejects_out_of_range_and_keeps_corpus():
    c = synth.corpus(0x5EED00A5, 3_000, 7, 20_000)
    st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
    st.append(*_part(c, 0, 100))
    before, bgoff = st.Minimize()
    with pytest.raises(Exception):
        st.keep(np.array([0, 5, c.n + 100], np.int64))
    after, agoff = st.Minimize()
    assert np.array_equal(before, after) and np.array_equal(bgoff, agoff)
    st.keep(np.zeros(0, np.int64))  # an empty corpus is a corpus
    got, goff = st.Minimize()
    assert got.size == 0 and np.array_equal(goff, np.zeros(c.ngroups + 1, np.uint64))
    st.close()


def test_key_parts_survive_append_and_keep():
    # set_parts is a property of the corpus: after an append and a keep the rebuilt index
    # still runs only this rank's windows and counts only its groups, so after the selection exchange
    # (export, MAX, import) both ranks hold the full selection and their histograms add up to the full one
    c = synth.corpus(0x5EED00A6, 40_000, 9, 200_000)
    G, C = c.ngroups, int(c.prog_len.max())
    import torch
    s = torch.cuda.current_stream().cuda_stream
    nparts = np.full(G, 2, np.uint16)
    stores = []
    for r in range(2):
        st = cover.CoverStore(*_part(c, 0, 25_000)[:3], G, _part(c, 0, 25_000)[3])
        st.set_parts(np.full(G, r, np.uint16), nparts, (np.arange(G) % 2 == r).astype(np.uint8))
        st.append(*_part(c, 25_000, 40_000))
        st.keep(np.arange(0, 40_000, 2))
        st.append(*_part(c, 1, 2))
        st.minimize_begin(s)
        stores.append(st)
    # the selection exchange of every (split) group: export, MAX across the two "ranks", import
    groups = np.arange(G, dtype=np.uint32)
    ent = np.bincount(np.concatenate([c.group[0:40_000:2], c.group[1:2]]).astype(np.int64), minlength=G)
    offs = np.zeros(G, np.uint64)
    np.cumsum(ent[:-1], out=offs[1:])
    bufs = [torch.zeros(int(ent.sum()), dtype=torch.uint8, device="cuda") for _ in range(2)]
    for st, b in zip(stores, bufs):
        st.export_sel(groups, offs, b, s)
    both = torch.maximum(bufs[0], bufs[1])
    ranks = []
    for st in stores:
        st.import_sel(groups, offs, both, s)
        sel = torch.zeros(st.n, dtype=torch.uint8, device="cuda")
        hist = torch.zeros(C + 1, dtype=torch.int64, device="cuda")
        st.minimize_end(C, sel, hist, s)
        torch.cuda.synchronize()
        ranks.append((sel.cpu().numpy(), hist.cpu().numpy()))
        st.close()
    hc = HostCorpus(c, 0, 40_000)
    hc.keep(list(range(0, 40_000, 2)))
    hc.append(c, 1, 2)
    pcs, off, grp, pl = hc.csr()
    want, _ = oracle.minimize_grouped(pcs, off, grp, G)
    wsel = np.zeros(len(hc.covs), np.uint8)
    wsel[want] = 1
    assert np.array_equal(ranks[0][0], wsel) and np.array_equal(ranks[1][0], wsel)
    assert np.array_equal(ranks[0][1] + ranks[1][1], np.bincount(pl[want], minlength=C + 1))


# ---- NewInput's corpusCover gate (manager.go:609-616, syzgpu_corpus_new_inputs[_dev]) ----------------

def _union_tables(covs, group, G):
    """corpusCover per call: the sorted union of the covers, without cover.go's sentinel."""
    per = [[] for _ in range(G)]
    for cv, g in zip(covs, group):
        per[int(g)].append(np.asarray(cv, np.uint32))
    tabs = [np.unique(np.concatenate(p)) if p else np.zeros(0, np.uint32) for p in per]
    tabs = [t[t != 0xFFFFFFFF] for t in tabs]
    off = np.zeros(G + 1, np.uint64)
    off[1:] = np.cumsum([t.size for t in tabs])
    return np.concatenate(tabs).astype(np.uint32), off


class GateModel:
    """The manager's NewInput on the host: oracle_novelty with no flakes over corpusCover, then the
    accepted inputs appended to the host corpus."""

    def __init__(self, hc, G):
        self.hc, self.G = hc, G
        self.mc, self.mco = _union_tables(hc.covs, hc.group, G)

    def new_inputs(self, pcs, off, grp, pl):
        is_new, mc, mco = oracle.novelty(pcs, off, grp, self.G, self.mc, self.mco, np.zeros(0, np.uint32))
        self.mc, self.mco = mc, mco
        for k in np.flatnonzero(is_new):
            self.hc.covs.append(pcs[int(off[k]):int(off[k + 1])])
            self.hc.group.append(grp[k])
            self.hc.plen.append(pl[k])
        return is_new.astype(bool)


def _gate_batch(c, lo, hi, extra=()):
    """Inputs lo..hi of c plus extra (cover, call) inputs, as CSR."""
    covs = [c.pcs[int(c.off[i]):int(c.off[i + 1])] for i in range(lo, hi)] + [np.asarray(x, np.uint32)
                                                                             for x, _ in extra]
    grp = np.concatenate([c.group[lo:hi], np.array([g for _, g in extra], np.uint32)]).astype(np.uint32)
    pl = np.concatenate([c.prog_len[lo:hi], np.ones(len(extra), np.uint16)]).astype(np.uint16)
    pcs, off = oracle.to_csr(covs)
    return pcs.astype(np.uint32), off.astype(np.uint64), grp, pl


def _check_gate(st, model):
    got_pcs, got_off = st.CorpusCover()
    assert np.array_equal(got_off, model.mco) and np.array_equal(got_pcs, model.mc)
    assert st.n == len(model.hc.covs)
    _check(st, model.hc, model.G)


@pytest.mark.parametrize("first", ["gate", "keep"])
def test_new_input_gate_vs_oracle_novelty(first):
    import torch
    G = 13
    a = synth.corpus(0x5EED00C1, 12_000, G, 60_000)
    b = synth.corpus(0x5EED00C2, 30_000, G, 90_000)  # a wider PC space: some inputs bring new PCs
    st = cover.CoverStore(a.pcs, a.off, a.group, G, a.prog_len)
    hc = HostCorpus(a, 0, a.n)
    if first == "keep":
        # an explicit keep before any gate: corpusCover is taken first, the dropped entries' PCs stay in it
        model = GateModel(hc, G)
        idx = np.arange(0, a.n, 3)
        st.keep(idx)
        hc.keep(list(idx))
    else:
        model = GateModel(hc, G)
    # 1: the first gate builds corpusCover; a batch of one, then a large one (the radix path), with an
    # input that repeats an earlier one of the batch, one whose only new PC is the sentinel, and an empty one
    for lo, hi in ((0, 1), (1, 1)):
        pcs, off, grp, pl = _gate_batch(b, lo, hi)
        assert np.array_equal(st.NewInputs(pcs, off, grp, pl), model.new_inputs(pcs, off, grp, pl))
    dup = b.pcs[int(b.off[5]):int(b.off[6])]
    extra = [(dup, int(b.group[5])), (np.array([0xFFFFFFFF], np.uint32), 0), (np.zeros(0, np.uint32), 1),
             (np.array([1, 2, 0xFFFFFFFF], np.uint32), 2), (np.array([1, 2], np.uint32), 2)]
    pcs, off, grp, pl = _gate_batch(b, 1, 20_000, extra)
    is_new = st.NewInputs(pcs, off, grp, pl)
    want = model.new_inputs(pcs, off, grp, pl)
    assert np.array_equal(is_new, want)
    assert 0 < want.sum() < want.size and not want[-4] and not want[-3] and want[-2] and not want[-1]
    _check_gate(st, model)
    # 2a: the same edge cases through a small batch (under 4M PCs: the batch-table path with its
    # atomicMin claims): a repeat of an earlier input of the batch, a sentinel-only cover, an empty one,
    # and a new PC pair with the sentinel followed by the same pair without it
    dup = b.pcs[int(b.off[20_005]):int(b.off[20_006])]
    extra = [(dup, int(b.group[20_005])), (np.array([0xFFFFFFFF], np.uint32), 3), (np.zeros(0, np.uint32), 4),
             (np.array([3, 4, 0xFFFFFFFF], np.uint32), 3), (np.array([3, 4], np.uint32), 3)]
    pcs, off, grp, pl = _gate_batch(b, 20_000, 20_100, extra)
    assert int(off[-1]) < (1 << 22)
    is_new = st.NewInputs(pcs, off, grp, pl)
    want = model.new_inputs(pcs, off, grp, pl)
    assert np.array_equal(is_new, want)
    assert not want[-5] and not want[-4] and not want[-3] and want[-2] and not want[-1]
    _check_gate(st, model)
    # 2b: device pointers, a small batch (the one-workgroup path)
    s = torch.cuda.current_stream().cuda_stream
    pcs, off, grp, pl = _gate_batch(b, 20_100, 20_200)
    d_new = torch.zeros(100, dtype=torch.uint8, device="cuda")
    na = st.NewInputsDevice(*(_dev(x) for x in (pcs, off, grp, pl)), 100, d_new, s)
    want = model.new_inputs(pcs, off, grp, pl)
    assert na == int(want.sum()) and np.array_equal(d_new.cpu().numpy().astype(bool), want)
    _check_gate(st, model)
    # 3: minimizeCorpus's keep leaves corpusCover as it is; an explicit keep drops entries, not PCs
    C = int(max(a.prog_len.max(), b.prog_len.max()))
    kept = st.MinimizeKeep(C, None, torch.zeros(C + 1, dtype=torch.int64, device="cuda"), None, None, s)
    pcs_h, off_h, grp_h, _ = hc.csr()
    wk, _ = oracle.minimize_grouped(pcs_h, off_h, grp_h, G)
    assert kept == wk.size
    hc.keep(list(wk))
    perm = np.random.default_rng(9).permutation(len(hc.covs))[: len(hc.covs) // 2]
    st.keep(perm)
    hc.keep(list(perm))
    _check_gate(st, model)
    # 4: an unconditional append is unioned in too; then the rest of b through the gate
    st.append(*_part(b, 20_200, 21_000))
    hc.append(b, 20_200, 21_000)
    model.mc, model.mco = _union_tables(
        [model.mc[int(model.mco[g]):int(model.mco[g + 1])] for g in range(G)]
        + [b.pcs[int(b.off[i]):int(b.off[i + 1])] for i in range(20_200, 21_000)],
        list(range(G)) + list(b.group[20_200:21_000]), G)
    pcs, off, grp, pl = _gate_batch(b, 21_000, b.n)
    assert np.array_equal(st.NewInputs(pcs, off, grp, pl), model.new_inputs(pcs, off, grp, pl))
    _check_gate(st, model)
    # 5: the same batch again adds nothing
    assert not st.NewInputs(pcs, off, grp, pl).any()
    _check_gate(st, model)
    st.close()


def test_new_input_gate_rejects_bad_batches():
    G = 5
    a = synth.corpus(0x5EED00C3, 3_000, G, 20_000)
    st = cover.CoverStore(a.pcs, a.off, a.group, G, a.prog_len)
    hc = HostCorpus(a, 0, a.n)
    model = GateModel(hc, G)
    for covs, grp in (([np.array([5, 3], np.uint32)], [0]),        # not sorted
                      ([np.array([7, 7], np.uint32)], [1]),        # a repeated PC
                      ([np.array([1 << 30], np.uint32)], [G])):    # call id >= ngroups
        pcs, off = oracle.to_csr(covs)
        with pytest.raises(Exception):
            st.NewInputs(pcs.astype(np.uint32), off.astype(np.uint64), np.array(grp, np.uint32))
        _check_gate(st, model)  # unchanged
    st.close()


def test_failed_growth_leaves_store_and_corpus_cover_unchanged():
    """A NewInput batch or an append whose store growth fails (forced through the test hook
    syzgpu_debug_fail_grow, as a device allocation failure) leaves the entries and corpusCover as they
    were, so the same batch retried afterwards is gated exactly as the oracle gates it."""
    from syzkaller_amd import _lib
    G = 7
    a = synth.corpus(0x5EED00C4, 3_000, G, 30_000)
    b = synth.corpus(0x5EED00C5, 4_000, G, 60_000)  # more PCs than the store's headroom: it must grow
    st = cover.CoverStore(a.pcs, a.off, a.group, G, a.prog_len)
    hc = HostCorpus(a, 0, a.n)
    model = GateModel(hc, G)
    _check_gate(st, model)  # builds corpusCover
    pcs, off, grp, pl = _gate_batch(b, 0, b.n)
    lib = _lib.lib()
    try:
        lib.syzgpu_debug_fail_grow(1)
        with pytest.raises(Exception):
            st.NewInputs(pcs, off, grp, pl)
        lib.syzgpu_debug_fail_grow(0)
        _check_gate(st, model)  # unchanged: no key of the failed batch entered corpusCover
        lib.syzgpu_debug_fail_grow(1)
        with pytest.raises(Exception):
            st.append(*_part(b, 0, b.n))
        lib.syzgpu_debug_fail_grow(0)
        _check_gate(st, model)
    finally:
        lib.syzgpu_debug_fail_grow(0)
    want = model.new_inputs(pcs, off, grp, pl)
    assert 0 < want.sum()
    assert np.array_equal(st.NewInputs(pcs, off, grp, pl), want)  # the retry is gated as the first try
    _check_gate(st, model)
    st.close()
