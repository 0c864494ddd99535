"""PC-range shards of the new-coverage check on the HIP path.

Every rank's slice of a config-3-shaped batch (fuzzer.go:446-470 per cover, in order) runs through
syzgpu_novelty_batch — the ranks one after another in this process — and the results are combined
exactly as sharding.novelty_shard combines them over RCCL: the MAX of the ranks' n + G flag bytes
(sharding.novelty_flags) and each call's table parts concatenated in PC-range order
(sharding.novelty_merge). The combined result must equal the per-call first-occurrence oracle on the
whole batch (oracle_novelty_mt, pinned to the literal oracle_novelty in tests/test_oracle.py).
The multi-process form of the same exchange runs under gloo in tests/test_sharding.py.
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

G = 289


def _maxcover_of(c):
    # maxCover0: the union of a seed corpus's covers per call (sorted, as the fuzzer keeps it)
    lens = np.diff(c.off).astype(np.int64)
    ent = np.repeat(np.arange(c.n), lens)
    keys = np.unique((c.group[ent].astype(np.uint64) << np.uint64(32)) | c.pcs.astype(np.uint64))
    g = (keys >> np.uint64(32)).astype(np.int64)
    mco = np.zeros(G + 1, np.uint64)
    np.cumsum(np.bincount(g, minlength=G), out=mco[1:])
    return (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), mco


@pytest.fixture(scope="module")
def batch():
    # configs[2]'s shape at 200k fresh covers: maxCover0 of a 10k corpus over a 500k-PC space, 5k flakes
    seedc = synth.corpus(0x5EED0003, 10_000, G, 500_000)
    mcp, mco = _maxcover_of(seedc)
    fresh = synth.corpus(0x5EED0103, 200_000, G, 500_000)
    flakes = np.unique(np.random.default_rng(3).choice(fresh.pcs, size=5000)).astype(np.uint32)
    want = oracle.novelty_mt(fresh.pcs, fresh.off, fresh.group, G, mcp, mco, flakes, 16)
    return fresh, mcp, mco, flakes, want


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3, 8])
def test_novelty_pc_shards_on_gpu(batch, world):
    fresh, mcp, mco, flakes, (w_new, w_mc, w_off) = batch
    sample = fresh.pcs[::97]
    bounds = sharding.pc_bounds(sample, world)
    flags = np.zeros(fresh.n + G, np.uint8)
    parts = []
    for r in range(world):
        lo, hi = int(bounds[r]), int(bounds[r + 1]) - 1
        p_r, o_r, m_r, mo_r, f_r = sharding.novelty_slice(fresh.pcs, fresh.off, mcp, mco, flakes, lo, hi)
        assert p_r.size < fresh.pcs.size  # a real slice
        is_new_r, tab_r, toff_r = cover.NoveltyBatch(p_r, o_r, fresh.group, G, m_r, mo_r, f_r)
        flags = np.maximum(flags, sharding.novelty_flags(is_new_r, fresh.group, G))
        parts.append((tab_r, toff_r))
    g_new, g_mc, g_off = sharding.novelty_merge(flags, parts, fresh.n, G)
    assert np.array_equal(g_off, w_off)
    assert np.array_equal(g_mc, w_mc)
    assert np.array_equal(g_new, w_new)
    assert 0 < g_new.sum() < fresh.n


def test_novelty_pc_shards_sentinel_tables():
    # the sentinel lives in the last PC range only: a call updated on ANY rank loses it, a call no
    # rank updated keeps it (cover.go:63-70 Union drops it over the whole table)
    S = 0xFFFFFFFF
    covs = [np.array([10, 20], np.uint32), np.array([3_000_000_000], np.uint32), np.array([5], np.uint32)]
    grp = np.array([0, 1, 2], np.uint32)
    mc = [np.array([1, S], np.uint32), np.array([7, S], np.uint32), np.array([5, S], np.uint32)]
    pcs, off = oracle.to_csr(covs)
    mcp, mco = oracle.to_csr(mc)
    flakes = np.zeros(0, np.uint32)
    w_new, w_mc, w_off = oracle.novelty(pcs, off, grp, 3, mcp, mco, flakes)
    bounds = np.array([0, 1 << 31, 1 << 32], np.uint64)
    flags = np.zeros(3 + 3, np.uint8)
    parts = []
    for r in range(2):
        p_r, o_r, m_r, mo_r, f_r = sharding.novelty_slice(pcs, off, mcp, mco, flakes, int(bounds[r]),
                                                          int(bounds[r + 1]) - 1)
        is_new_r, tab_r, toff_r = cover.NoveltyBatch(p_r, o_r, grp, 3, m_r, mo_r, f_r)
        flags = np.maximum(flags, sharding.novelty_flags(is_new_r, grp, 3))
        parts.append((tab_r, toff_r))
    g_new, g_mc, g_off = sharding.novelty_merge(flags, parts, 3, 3)
    assert np.array_equal(g_new, w_new) and np.array_equal(g_mc, w_mc) and np.array_equal(g_off, w_off)
