"""Appending to the resident store (syzgpu_corpus_append[_dev]): mgr.corpus = append(mgr.corpus, ...)
on NewInput (syz-manager/manager.go:609-616), then minimizeCorpus (manager.go:507-527) over the grown
store must equal the oracle's minimizeCorpus over the whole corpus."""
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
