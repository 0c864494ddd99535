"""Reentrancy of the C ABI (SURVEY.md §8b "Threading"): callers arrive concurrently — fuzzer procs under
coverMu's read lock (syz-fuzzer/fuzzer.go:448-456), manager RPC goroutines — so two threads that
interleave syzgpu_minimize_grouped_dev / _fetch on different corpora must each get their own result,
and jobs / stores used from several threads must keep their state apart. ctypes releases the GIL
during foreign calls, so the Python threads below really run inside the library at the same time.
Also the job API's key parts (the multi-GPU split of one call group by PC range):
partial selections OR-ed together equal the oracle's selection.
"""
import os
import sys
import threading

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


def test_two_threads_interleave_dev_and_fetch(torch):
    corpora = [synth.corpus(21, 40_000, 31, 200_000), synth.corpus(22, 55_000, 17, 300_000)]
    wants = [oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups) for c in corpora]
    dev = [[_dev(torch, c.pcs), _dev(torch, c.off), _dev(torch, c.group)] for c in corpora]
    barrier = threading.Barrier(2)
    errors = []

    def worker(i):
        try:
            c = corpora[i]
            L = _lib.lib()
            s = torch.cuda.Stream()
            for it in range(6):
                barrier.wait()  # both threads enter the library together
                with torch.cuda.stream(s):
                    _lib.check(L.syzgpu_minimize_grouped_dev(dev[i][0].data_ptr(), dev[i][1].data_ptr(),
                                                             dev[i][2].data_ptr(), None, c.n, c.ngroups, 0, None,
                                                             None, s.cuda_stream))
                barrier.wait()  # the other thread's minimize ran in between
                out = np.empty(c.n, np.int64)
                goff = np.zeros(c.ngroups + 1, np.uint64)
                _lib.check(L.syzgpu_minimize_grouped_fetch(out.ctypes.data, goff.ctypes.data, c.n, c.ngroups))
                want, wgoff = wants[i]
                assert np.array_equal(goff, wgoff), (i, it)
                assert np.array_equal(out[:int(goff[-1])], want), (i, it)
        except Exception as e:  # noqa: BLE001
            errors.append((i, repr(e)))
            barrier.abort()

    th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_threads_share_nothing_through_jobs_and_stores(torch):
    # four threads, each with its own job and store, hammering the library at once
    corpora = [synth.corpus(30 + i, 20_000 + 5_000 * i, 13, 100_000) for i in range(4)]
    wants = [oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups) for c in corpora]
    errors = []

    def worker(i):
        try:
            c = corpora[i]
            d = [_dev(torch, c.pcs), _dev(torch, c.off), _dev(torch, c.group)]
            s = torch.cuda.Stream()
            job = cover.MinimizeJob()
            st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
            want, wgoff = wants[i]
            for _ in range(4):
                job.begin(d[0], d[1], d[2], c.n, c.ngroups, stream=s.cuda_stream)
                job.end(stream=s.cuda_stream)
                got, goff = job.fetch(c.n, c.ngroups)
                assert np.array_equal(goff, wgoff) and np.array_equal(got, want)
                sgot, sgoff = st.Minimize()
                assert np.array_equal(sgoff, wgoff) and np.array_equal(sgot, want)
                hk, hg = cover.MinimizeCorpus(c.pcs, c.off, c.group, c.ngroups)
                assert np.array_equal(hg, wgoff) and np.array_equal(hk, want)
            job.close()
            st.close()
        except Exception as e:  # noqa: BLE001
            errors.append((i, repr(e)))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_fetch_on_another_thread_is_rejected(torch):
    c = synth.corpus(40, 5000, 7, 20_000)
    d = [_dev(torch, c.pcs), _dev(torch, c.off), _dev(torch, c.group)]
    L = _lib.lib()
    _lib.check(L.syzgpu_minimize_grouped_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), None, c.n,
                                             c.ngroups, 0, None, None, 0))
    torch.cuda.synchronize()
    res = []

    def other():
        out = np.empty(c.n, np.int64)
        goff = np.zeros(c.ngroups + 1, np.uint64)
        res.append(L.syzgpu_minimize_grouped_fetch(out.ctypes.data, goff.ctypes.data, c.n, c.ngroups))

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert res == [_lib.EINVAL]


@pytest.mark.parametrize("k", [2, 3, 5])
def test_key_parts_or_to_full_selection(torch, k):
    # one rank per part, all on this GPU: every group split into k PC ranges at sample quantiles
    c = synth.corpus(50 + k, 60_000, 9, 400_000)
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    d = [_dev(torch, c.pcs), _dev(torch, c.off), _dev(torch, c.group), _dev(torch, c.prog_len)]
    G = c.ngroups
    qs = np.quantile(c.pcs.astype(np.float64), np.linspace(0, 1, k + 1)[1:-1]).astype(np.uint64)
    b = np.concatenate([[0], np.maximum.accumulate(qs), [1 << 32]]).astype(np.uint64)
    ent = np.bincount(c.group, minlength=G)
    goff_in = np.zeros(G, np.uint64)
    goff_in[1:] = np.cumsum(ent)[:-1]
    groups = np.arange(G, dtype=np.uint32)
    buf = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    jobs = []
    C = 40
    for j in range(k):
        lo = np.full(G, b[j], np.uint32)
        hi = np.full(G, min(int(b[j + 1]) - 1, 0xFFFFFFFF), np.uint32)
        job = cover.MinimizeJob()
        job.begin(d[0], d[1], d[2], c.n, G, d[3], lo, hi)
        part = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
        job.export_sel(groups, goff_in, part)
        buf = torch.maximum(buf, part)  # the MAX all-reduce
        jobs.append(job)
    hists = []
    for j, job in enumerate(jobs):
        job.import_sel(groups, goff_in, buf)
        hist = torch.zeros(C + 1, dtype=torch.int64, device="cuda")
        count = np.full(G, 1 if j == 0 else 0, np.uint8)  # one rank counts each group
        out = torch.zeros(c.n, dtype=torch.int64, device="cuda")
        go = torch.zeros(G + 1, dtype=torch.int64, device="cuda")
        job.end(C, count, None, hist, out, go)
        torch.cuda.synchronize()
        goh = go.cpu().numpy().astype(np.uint64)
        assert np.array_equal(goh, wgoff)
        assert np.array_equal(out.cpu().numpy()[:int(goh[-1])], want)
        hists.append(hist.cpu().numpy())
    assert np.array_equal(sum(hists), np.bincount(c.prog_len[want], minlength=C + 1))
