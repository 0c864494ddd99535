"""BASELINE.json's configs at their full size, against the CPU oracle.

configs[3] (1M programs, 2M-PC space, 289 calls, C = 1159: the bench workload) and configs[4] (the
hub merge of 8 managers' corpora, 8M programs, on one GPU) run minimizeCorpus
(syz-manager/manager.go:507-527 over cover/cover.go:105-131) from the raw covers and from the resident
store, then CalculatePriorities + BuildChoiceTable (prog/prio.go:29-38,137-228) on the kept programs.
Every output is compared bit-for-bit with oracle/oracle.c: the group-major kept list in selection
order, the group offsets, the kept flags, the len(p.Calls) histogram, the float32 priorities and the
ChoiceTable's run matrix. The oracle runs its per-call Minimize over 16 host threads
(oracle_minimize_grouped_mt: the same selection as the serial restatement, tests/test_oracle.py).

configs[2] (the fuzzer's triage batch, 1M fresh covers against maxCover) is checked at full size in
tests/test_gpu_novelty.py::test_novelty_config3_full_size.
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

C = 1159          # calls of sys/*.txt (BASELINE.json configs[3])
G = 289           # call groups of the synthetic corpus
THREADS = 16      # the GPU box's host share


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a device (no CPU fallback exists)"
    _lib.check(_lib.lib().syzgpu_init(0))
    return t


def _dev(torch, a):
    view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(view.get(a.dtype, a.dtype))).cuda()


def _static(seed=7):
    rnd = np.random.default_rng(seed)
    s = (rnd.random((C, C)) * 0.9 + 0.1).astype(np.float32)
    np.fill_diagonal(s, s.max(axis=1))
    return s


def _raw_then_prio(torch, c, static):
    """The bench's step: raw minimizeCorpus, then prio + ChoiceTable from the kept-length histogram."""
    L = _lib.lib()
    d_pcs, d_off, d_grp, d_len = (_dev(torch, x) for x in (c.pcs, c.off, c.group, c.prog_len))
    sel = torch.full((c.n,), 7, dtype=torch.uint8, device="cuda")
    hist = torch.full((C + 1,), -1, dtype=torch.int64, device="cuda")
    out = torch.full((c.n,), -1, dtype=torch.int64, device="cuda")
    goff = torch.full((G + 1,), -1, dtype=torch.int64, device="cuda")
    prios = torch.empty((C, C), dtype=torch.float32, device="cuda")
    run = torch.empty((C, C), dtype=torch.int64, device="cuda")
    pres = torch.empty(C, dtype=torch.uint8, device="cuda")
    d_static = torch.from_numpy(static).cuda()
    s = torch.cuda.current_stream().cuda_stream
    job = cover.MinimizeJob()
    job.begin(d_pcs, d_off, d_grp, c.n, G, d_len, stream=s)
    job.end(C, None, sel, hist, out, goff, s)
    _lib.check(L.syzgpu_prio_choice_dev(d_static.data_ptr(), hist.data_ptr(), C, None, prios.data_ptr(),
                                        run.data_ptr(), pres.data_ptr(), s))
    torch.cuda.synchronize()
    job.close()
    goff_h = goff.cpu().numpy().astype(np.uint64)
    res = dict(kept=out.cpu().numpy()[: int(goff_h[-1])], goff=goff_h, sel=sel.cpu().numpy(),
               hist=hist.cpu().numpy(), prios=prios.cpu().numpy(), run=run.cpu().numpy(), pres=pres.cpu().numpy())
    return res, (d_pcs, d_off, d_grp, d_len)


def _store_minimize(torch, c, dbufs):
    d_pcs, d_off, d_grp, d_len = dbufs
    s = torch.cuda.current_stream().cuda_stream
    store = cover.CoverStore.from_device(d_pcs, d_off, d_grp, d_len, c.n, G, s)
    sel = torch.full((c.n,), 7, dtype=torch.uint8, device="cuda")
    hist = torch.full((C + 1,), -1, dtype=torch.int64, device="cuda")
    _lib.check(_lib.lib().syzgpu_corpus_minimize_dev(store.handle, C, sel.data_ptr(), hist.data_ptr(), s))
    torch.cuda.synchronize()
    kept, goff = store.Minimize()
    store.close()
    return kept, goff, sel.cpu().numpy(), hist.cpu().numpy()


def _check_config(torch, c):
    static = _static()
    got, dbufs = _raw_then_prio(torch, c, static)
    want, wgoff = oracle.minimize_grouped_mt(c.pcs, c.off, c.group, G, THREADS)
    assert np.array_equal(got["goff"], wgoff)
    assert np.array_equal(got["kept"], want)
    wsel = np.zeros(c.n, np.uint8)
    wsel[want] = 1
    assert np.array_equal(got["sel"], wsel)
    kept_len = c.prog_len[want]
    assert np.array_equal(got["hist"], np.bincount(kept_len, minlength=C + 1))
    wp = oracle.calculate_priorities(static, kept_len)
    assert np.array_equal(got["prios"].view(np.uint32), wp.view(np.uint32))
    wrun, wpres = oracle.build_choice_table(wp)
    assert np.array_equal(got["run"], wrun) and np.array_equal(got["pres"], wpres)
    # the resident store (dense PC ids built on the device) selects the same programs
    skept, sgoff, ssel, shist = _store_minimize(torch, c, dbufs)
    assert np.array_equal(sgoff, wgoff) and np.array_equal(skept, want)
    assert np.array_equal(ssel, wsel) and np.array_equal(shist, got["hist"])
    return want


@pytest.mark.timeout(400)
def test_config4_full_size_vs_oracle(torch):
    # configs[3] at full size: the bench's corpus (same seed and shape)
    c = synth.corpus(0x5EED0004, 1_000_000, G, 2_000_000)
    assert int(c.off[-1]) > 400_000_000
    want = _check_config(torch, c)
    assert 0.3 * c.n < want.size < c.n


@pytest.mark.timeout(900)
def test_config5_hub_merge_8m_vs_oracle(torch):
    # configs[4] on one GPU: the 8 managers' corpora merged (8M programs over the same 2M-PC kernel,
    # 3.4G PCs = 13.5 GB of covers in HBM), global Minimize + ChoiceTable rebuild
    c = synth.corpus(0x5EED0005, 8_000_000, G, 2_000_000)
    assert int(c.off[-1]) > 3 * 2**30  # element offsets past 2^31 on every path
    _check_config(torch, c)
