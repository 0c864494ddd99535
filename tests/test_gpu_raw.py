"""minimizeCorpus from raw device-resident covers (syzgpu_minimize_grouped_ordered_dev, panels.hip)
against the CPU oracle (oracle/oracle.c, a literal restatement of cover/cover.go:105-131 driven by
syz-manager/manager.go:507-527).

Every output is compared bit-for-bit: the group-major kept list in Go's selection order, the group
offsets, the kept flags and the len(p.Calls) histogram of the kept programs. Besides the synthetic
configs, the cases aim at each branch of the pipeline: direct and open-addressing windows (dense and
sparse PC spans), window tables that overflow and are redone in rounds, chunks split inside one
cover, call groups of one entry, empty covers, 0xFFFFFFFF, and unsorted covers (the exact-bounds
retry).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import _lib, cover, synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a device (no CPU fallback exists)"
    _lib.check(_lib.lib().syzgpu_init(0))
    return t


def _dev(torch, a):
    view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(view.get(a.dtype, a.dtype)).copy()).cuda()


def run_dev(torch, pcs, off, group, ngroups, prog_len=None, C=0):
    n = off.size - 1
    d_pcs = _dev(torch, pcs if pcs.size else np.zeros(1, np.uint32))
    d_off, d_grp = _dev(torch, off), _dev(torch, group if group.size else np.zeros(1, np.uint32))
    d_len = _dev(torch, prog_len) if prog_len is not None else None
    sel = torch.full((max(n, 1),), 7, dtype=torch.uint8, device="cuda")
    hist = torch.full((C + 1,), -1, dtype=torch.int64, device="cuda") if C else None
    out = torch.full((max(n, 1),), -1, dtype=torch.int64, device="cuda")
    goff = torch.full((ngroups + 1,), -1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    cover.MinimizeCorpusDev(d_pcs, d_off, d_grp, n, ngroups, d_len, C, sel, hist, out, goff, stream)
    torch.cuda.synchronize()
    goff_h = goff.cpu().numpy().astype(np.uint64)
    kept = out.cpu().numpy()[: int(goff_h[-1])]
    return kept, goff_h, sel.cpu().numpy()[:n], (hist.cpu().numpy() if C else None)


def check(torch, pcs, off, group, ngroups, prog_len=None, C=0):
    pcs = np.ascontiguousarray(pcs, dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    group = np.ascontiguousarray(group, dtype=np.uint32)
    want, wgoff = oracle.minimize_grouped(pcs, off, group, ngroups)
    kept, goff, sel, hist = run_dev(torch, pcs, off, group, ngroups, prog_len, C)
    assert np.array_equal(goff, wgoff)
    assert np.array_equal(kept, want)
    wsel = np.zeros(off.size - 1, np.uint8)
    wsel[want] = 1
    assert np.array_equal(sel, wsel)
    if C:
        assert np.array_equal(hist, np.bincount(prog_len[want], minlength=C + 1))
    # the host-pointer entry point runs the same pipeline
    hk, hgoff = cover.MinimizeCorpus(pcs, off, group, ngroups)
    assert np.array_equal(hk, want) and np.array_equal(hgoff, wgoff)
    return want


@pytest.mark.parametrize("seed,n,G,P", [(0x5EED0001, 10_000, 289, 50_000), (0x5EED0002, 100_000, 289, 500_000),
                                        (3, 50_000, 5, 2_000_000), (4, 20_000, 1, 30_000)])
def test_synthetic_vs_oracle(torch, seed, n, G, P):
    c = synth.corpus(seed, n, G, P)
    check(torch, c.pcs, c.off, c.group, G, c.prog_len, 64)


def test_sparse_span_hash_windows(torch):
    # PCs spread over the whole 32-bit space: every call takes wide open-addressing windows
    rnd = np.random.default_rng(5)
    covs = [np.unique(rnd.integers(0, 2**32, size=int(rnd.integers(0, 600)), dtype=np.uint64).astype(np.uint32))
            for _ in range(6000)]
    pcs, off = cover.to_csr(covs)
    group = rnd.integers(0, 9, size=len(covs)).astype(np.uint32)
    check(torch, pcs, off, group, 9)


def test_dense_span_direct_windows(torch):
    # few PCs reused by everyone in a 2M-address span: dense calls take the direct 32K tables
    rnd = np.random.default_rng(6)
    base = np.uint32(0x81000000)
    covs = [base + np.unique(rnd.integers(0, 1 << 21, size=int(rnd.integers(200, 3000)))).astype(np.uint32)
            for _ in range(12000)]
    pcs, off = cover.to_csr(covs)
    group = (rnd.random(len(covs)) < 0.9).astype(np.uint32)  # one huge call, one small one
    check(torch, pcs, off, group, 2)


def test_hash_window_overflow_rounds(torch):
    # a sparse call whose windows hold more distinct PCs than a table has slots (no PC repeats):
    # every window is redone in rounds
    rnd = np.random.default_rng(7)
    space = rnd.permutation(np.arange(0, 4 << 20, dtype=np.uint32) * 7)[: 300_000]
    covs = [np.sort(space[i * 3000:(i + 1) * 3000]) for i in range(100)]
    pcs, off = cover.to_csr(covs)
    check(torch, pcs, off, np.zeros(len(covs), np.uint32), 1)


def test_chunks_inside_long_covers(torch):
    # covers longer than a chunk (16384 PCs) and blocks of 64 members split into many chunks
    rnd = np.random.default_rng(8)
    covs = []
    for i in range(400):
        L = int(rnd.choice([1, 5, 16383, 40000, 70000])) if i % 7 == 0 else int(rnd.integers(1, 3000))
        covs.append(np.unique(rnd.integers(0, 1 << 24, size=L)).astype(np.uint32))
    pcs, off = cover.to_csr(covs)
    group = rnd.integers(0, 3, size=len(covs)).astype(np.uint32)
    check(torch, pcs, off, group, 3)


def test_lone_groups_empty_covers_sentinel(torch):
    # a one-entry call first (never sorted), empty covers, 0xFFFFFFFF counted like any PC by
    # Minimize's map (cover.go:115-127), calls with no entries at all
    c = synth.corpus(9, 30_000, 4, 40_000)
    group = c.group.copy() + 2
    group[0] = 0  # call 0: one entry; call 1: none
    lens = np.diff(c.off).astype(np.int64)
    covs = [c.cover(i).copy() for i in range(c.n)]
    for i in range(0, c.n, 13):
        covs[i] = np.zeros(0, np.uint32)
    for i in range(5, c.n, 17):
        if covs[i].size:
            covs[i] = np.append(covs[i][:-1], np.uint32(0xFFFFFFFF))
    covs[1] = np.array([0xFFFFFFFF], np.uint32)
    pcs, off = cover.to_csr(covs)
    check(torch, pcs, off, group, 6, c.prog_len, 40)
    del lens


def test_unsorted_covers_exact_bounds_retry(torch):
    # Minimize's map does not need sorted covers: the pipeline's first/last-PC bounds do, so an
    # unsorted cover with a PC outside them sends the call through the exact-bounds retry
    rnd = np.random.default_rng(10)
    covs = [rnd.permutation(np.unique(rnd.integers(0, 1 << 22, size=int(rnd.integers(1, 400))))).astype(np.uint32)
            for _ in range(5000)]
    pcs, off = cover.to_csr(covs)
    group = rnd.integers(0, 4, size=len(covs)).astype(np.uint32)
    check(torch, pcs, off, group, 4)


def test_duplicates_inside_covers(torch):
    rnd = np.random.default_rng(11)
    covs = [np.sort(rnd.integers(0, 5000, size=int(rnd.integers(0, 300)))).astype(np.uint32) for _ in range(8000)]
    pcs, off = cover.to_csr(covs)
    check(torch, pcs, off, rnd.integers(0, 3, size=len(covs)).astype(np.uint32), 3)


def test_empty_corpus_and_all_empty_covers(torch):
    kept, goff, _, _ = run_dev(torch, np.zeros(0, np.uint32), np.zeros(1, np.uint64), np.zeros(0, np.uint32), 3)
    assert kept.size == 0 and np.array_equal(goff, np.zeros(4, np.uint64))
    off = np.zeros(101, np.uint64)
    check(torch, np.zeros(0, np.uint32), off, np.arange(100, dtype=np.uint32) % 5, 5)


def test_reuse_across_layouts(torch):
    # the context caches the Go-sort plan of the last layout: alternate two corpora
    a = synth.corpus(12, 20_000, 17, 100_000)
    b = synth.corpus(13, 25_000, 17, 100_000)
    for c in (a, b, a):
        check(torch, c.pcs, c.off, c.group, 17)


def test_len_hist_rejects_long_programs(torch):
    c = synth.corpus(14, 2000, 5, 10_000)
    pl = c.prog_len.copy()
    pl[:] = 99  # every kept program is longer than C
    with pytest.raises(_lib.SyzGpuError):
        run_dev(torch, c.pcs, c.off, c.group, 5, pl, 40)


def test_end_prio_fused_tail_matches_oracle(torch):
    # syzgpu_mz_end_prio_dev: minimizeCorpus's tail (manager.go:523-536) in one call — kept list, flags
    # and length histogram of the job, calcStaticPriorities of the bundled sys/ usage matrix, then
    # CalculatePriorities + BuildChoiceTable — against the oracle of each piece
    from syzkaller_amd import sysdesc
    u = sysdesc.bundled()
    C = u.C
    c = synth.corpus(0x5EED0021, 30_000, 97, 200_000)
    want_kept, want_goff = oracle.minimize_grouped(c.pcs, c.off, c.group, 97)
    want_hist = np.bincount(c.prog_len[want_kept], minlength=C + 1).astype(np.int64)
    st = oracle.static_priorities(u.weights, exact=True)
    want_p = oracle.calculate_priorities(st, c.prog_len[want_kept])
    want_run, want_pres = oracle.build_choice_table(want_p)
    s = torch.cuda.current_stream().cuda_stream
    d = [_dev(torch, x) for x in (c.pcs, c.off, c.group, c.prog_len)]
    sel = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    hist = torch.zeros(C + 1, dtype=torch.int64, device="cuda")
    out = torch.zeros(c.n, dtype=torch.int64, device="cuda")
    goff = torch.zeros(98, dtype=torch.int64, device="cuda")
    d_w = torch.from_numpy(u.weights).cuda()
    d_st = torch.empty((C, C), dtype=torch.float32, device="cuda")
    d_p = torch.empty((C, C), dtype=torch.float32, device="cuda")
    d_run = torch.empty((C, C), dtype=torch.int64, device="cuda")
    d_pres = torch.empty(C, dtype=torch.uint8, device="cuda")
    job = cover.MinimizeJob()
    for _ in range(2):  # the second step reuses the job and the lane's streams
        job.begin(d[0], d[1], d[2], c.n, 97, d[3], stream=s)
        job.end_prio(C, d_w, u.weights.shape[0], d_st, d_p, d_run, None, sel, hist, out, goff, d_pres, s)
        torch.cuda.synchronize()
        g = goff.cpu().numpy().astype(np.uint64)
        assert np.array_equal(g, want_goff)
        assert np.array_equal(out.cpu().numpy()[: int(g[-1])], want_kept)
        assert np.array_equal(hist.cpu().numpy(), want_hist)
        assert np.array_equal(d_st.cpu().numpy().view(np.uint32), st.view(np.uint32))
        assert np.array_equal(d_p.cpu().numpy().view(np.uint32), want_p.view(np.uint32))
        assert np.array_equal(d_run.cpu().numpy(), want_run)
        assert np.array_equal(d_pres.cpu().numpy(), want_pres)
    # the deferred checks still raise: a kept program longer than C, and a non-finite usage weight
    long_len = _dev(torch, np.full(c.n, C + 5, np.uint16))
    job.begin(d[0], d[1], d[2], c.n, 97, long_len, stream=s)
    with pytest.raises(_lib.SyzGpuError):
        job.end_prio(C, d_w, u.weights.shape[0], d_st, d_p, d_run, None, sel, hist, out, goff, d_pres, s)
    bad = u.weights.copy()
    bad[0, 0] = np.nan
    d_bad = torch.from_numpy(bad).cuda()
    job.begin(d[0], d[1], d[2], c.n, 97, d[3], stream=s)
    with pytest.raises(_lib.SyzGpuError):
        job.end_prio(C, d_bad, u.weights.shape[0], d_st, d_p, d_run, None, sel, hist, out, goff, d_pres, s)
