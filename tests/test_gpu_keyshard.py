"""Key-space sharding of minimizeCorpus on the GPU (syzgpu_corpus_set_parts and the begin / export /
import / end halves): the partial selections of every call group's window parts, OR-ed together,
must equal the whole-store Minimize and the CPU oracle bit for bit, and the length histograms of the
parts' primaries must add up to the full one. The ranks are stand-ins inside one process: their
stores share the context's per-call scratch, so each part's first half is run again before import.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import cover, sharding, synth  # noqa: E402

pytestmark = pytest.mark.gpu

C = 1159


def _flags(n, idx):
    f = np.zeros(n, np.uint8)
    f[idx] = 1
    return f


@pytest.mark.parametrize("nparts,seed,n,G,P", [(2, 0x5EED0031, 40_000, 5, 400_000),
                                               (3, 0x5EED0032, 60_000, 9, 1_500_000),
                                               (4, 0x5EED0033, 30_000, 37, 200_000)])
def test_window_parts_or_to_the_full_selection(nparts, seed, n, G, P):
    import torch
    dev = torch.device("cuda:0")
    c = synth.corpus(seed, n, G, P)
    want_idx, _ = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    want = _flags(c.n, want_idx)
    want_hist = np.bincount(c.prog_len[want_idx], minlength=C + 1)
    groups = np.arange(G, dtype=np.uint32)  # every group split (small ones have a single window)
    ent = np.bincount(c.group, minlength=G).astype(np.uint64)
    offs = np.zeros(G, np.uint64)
    np.cumsum(ent[:-1], out=offs[1:])
    total = int(ent.sum())
    stores = []
    for p in range(nparts):
        st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
        st.set_parts(np.full(G, p, np.uint16), np.full(G, nparts, np.uint16),
                     np.full(G, 1 if p == 0 else 0, np.uint8))
        stores.append(st)
    x = torch.zeros(total, dtype=torch.uint8, device=dev)
    for st in stores:
        buf = torch.zeros(total, dtype=torch.uint8, device=dev)
        st.minimize_begin(0)
        st.export_sel(groups, offs, buf, 0)
        torch.cuda.synchronize()
        part_sel = buf.cpu().numpy()
        assert part_sel.sum() <= want.sum()
        x = torch.maximum(x, buf)
    hist_sum = np.zeros(C + 1, np.int64)
    for st in stores:
        sel = torch.zeros(c.n, dtype=torch.uint8, device=dev)
        hist = torch.zeros(C + 1, dtype=torch.int64, device=dev)
        st.minimize_begin(0)
        st.import_sel(groups, offs, x, 0)
        st.minimize_end(C, sel, hist, 0)
        torch.cuda.synchronize()
        assert np.array_equal(sel.cpu().numpy(), want)
        hist_sum += hist.cpu().numpy()
    assert np.array_equal(hist_sum, want_hist)
    # a single part is a strict subset of the selection whenever a group has several windows
    info = stores[0].info()
    assert info["work_items"] <= cover.CoverStore(c.pcs, c.off, c.group, c.ngroups).info()["work_items"]


def test_plan_on_the_bench_layout_runs_whole_and_split_groups():
    # a 4-rank plan with the two largest call groups split 3 and 2 ways, the rest whole: every
    # rank's parts OR back to the whole selection (reduced sizes, the bench's shape)
    import torch
    dev = torch.device("cuda:0")
    W = 4
    p = synth.params(0x5EED0034, 160_000, 29, 600_000)
    group, off, plen = synth.layout(p)
    e, w = sharding.layout_stats(group, off, 29)
    k = np.ones(29, np.int64)
    top = np.argsort(-e, kind="stable")
    k[top[0]], k[top[1]] = 3, 2
    ranks, cost = sharding._assign(e, w, k, W)
    plan = sharding.KeyPlan(ranks, cost, e)
    assert plan.split_groups()[0].size == 2
    c = synth.corpus(0x5EED0034, 160_000, 29, 600_000)
    want_idx, _ = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    want = _flags(c.n, want_idx)
    split_g, split_off, split_bytes = plan.split_groups()
    x = torch.zeros(max(split_bytes, 1), dtype=torch.uint8, device=dev)
    ranks = []
    for r in range(W):
        ids = plan.local_entries(group, r)
        sub = synth.subcorpus(p, ids, group, off, plen)
        st = cover.CoverStore(sub.pcs, sub.off, sub.group, sub.ngroups, sub.prog_len)
        st.set_parts(*plan.store_parts(r))
        held = plan.held(r)
        xg, xo = split_g[held[split_g]], split_off[held[split_g]]
        buf = torch.zeros_like(x)
        st.minimize_begin(0)
        if xg.size:
            st.export_sel(xg, xo, buf, 0)
        x = torch.maximum(x, buf)
        ranks.append((ids, st, xg, xo))
    got = np.zeros(c.n, np.uint8)
    for ids, st, xg, xo in ranks:
        sel = torch.zeros(ids.size, dtype=torch.uint8, device=dev)
        st.minimize_begin(0)
        if xg.size:
            st.import_sel(xg, xo, x, 0)
        st.minimize_end(C, sel, None, 0)
        torch.cuda.synchronize()
        got[ids] |= sel.cpu().numpy()
    assert np.array_equal(got, want)
