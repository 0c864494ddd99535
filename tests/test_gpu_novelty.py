"""Parity of the batch new-coverage check (syz-fuzzer/fuzzer.go:446-470 execute; manager.go:609-616
NewInput) on the MI355X against the oracle's literal restatement (oracle.c oracle_novelty).

Bit-exact: is_new flags and every updated maxCover table. BASELINE.json configs[2] ("1M fresh
execution covers diffed against maxCover") is covered at full size (1M covers) against the
per-call first-occurrence oracle and at reduced sizes against the literal one, plus
the edge cases foreach gives the path: the 0xFFFFFFFF sentinel (dropped by Difference and by Union),
flakes, empty covers, empty tables.
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


@pytest.fixture(autouse=True, params=["windows", "hwindows", "table", "keys", "sort"])
def strategy(request, monkeypatch):
    """Every device strategy: PC windows on the Minimize pipeline (the default: direct windows while
    the PC span fits 1024 windows of 32K addresses, hashed windows beyond), the hashed windows forced
    whatever the span, the keyed first-occurrence table over G x (P+1) (the default for G > 4096),
    the keyed table over per-call keys, and the stable radix sort (when no table fits). A forced
    windows strategy fails rather than fall back. SYZGPU_NOVELTY is read by the library on every call."""
    monkeypatch.setenv("SYZGPU_NOVELTY", request.param)
    return request.param


def _check(pcs, off, grp, G, mcp, mco, flakes):
    w_new, w_mc, w_off = oracle.novelty(pcs, off, grp, G, mcp, mco, flakes)
    g_new, g_mc, g_off = cover.NoveltyBatch(pcs, off, grp, G, mcp, mco, flakes)
    assert np.array_equal(w_off, g_off)
    assert np.array_equal(w_mc, g_mc)
    assert np.array_equal(w_new, g_new)
    return g_new


@pytest.mark.parametrize("seed", range(6))
def test_novelty_random_small(seed):
    rnd = np.random.default_rng(seed)
    G = 4
    for _ in range(20):
        n = int(rnd.integers(0, 60))
        covs = [np.unique(rnd.integers(0, 80, size=int(rnd.integers(0, 12)))).astype(np.uint32) for _ in range(n)]
        grp = rnd.integers(0, G, size=n).astype(np.uint32)
        mc = [np.unique(rnd.integers(0, 80, size=int(rnd.integers(0, 20)))).astype(np.uint32) for _ in range(G)]
        flakes = np.unique(rnd.integers(0, 80, size=int(rnd.integers(0, 8)))).astype(np.uint32)
        pcs, off = oracle.to_csr(covs)
        mcp, mco = oracle.to_csr(mc)
        _check(pcs, off, grp, G, mcp, mco, flakes)


def test_novelty_sentinel_flakes_empty():
    S = 0xFFFFFFFF
    covs = [[1, 2, S], [S], [], [3, 4], [4, 5], [7], [1, S], [9, S]]
    grp = [0, 1, 1, 2, 2, 3, 0, 3]
    mc = [[1, 2], [S], [3, S], [S], []]  # group 1 never updated (keeps S); group 2/3 updated (lose S)
    flakes = [5, 9]
    covs = [np.array(c, np.uint32) for c in covs]
    pcs, off = oracle.to_csr(covs)
    mcp, mco = oracle.to_csr([np.array(m, np.uint32) for m in mc])
    new = _check(pcs, off, np.array(grp, np.uint32), 5, mcp, mco, np.array(flakes, np.uint32))
    assert list(new) == [0, 0, 0, 1, 0, 1, 0, 0]


def _maxcover_of(c):
    lens = np.diff(c.off).astype(np.int64)
    ent = np.repeat(np.arange(c.n), lens)
    keys = np.unique((c.group[ent].astype(np.uint64) << np.uint64(32)) | c.pcs.astype(np.uint64))
    g = (keys >> np.uint64(32)).astype(np.int64)
    mco = np.zeros(c.ngroups + 1, np.uint64)
    np.cumsum(np.bincount(g, minlength=c.ngroups), out=mco[1:])
    return (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), mco


def _config3(n_seed, n_fresh, P):
    G = 289
    seedc = synth.corpus(0x5EED0003, n_seed, G, P)
    mcp, mco = _maxcover_of(seedc)
    fresh = synth.corpus(0x5EED0103, n_fresh, G, P)
    rnd = np.random.default_rng(3)
    flakes = np.unique(rnd.choice(fresh.pcs, size=5000)).astype(np.uint32)
    return fresh, mcp, mco, flakes


def test_novelty_config3_shape_vs_oracle():
    # configs[2] at a size the literal oracle (O(|maxCover|) merges per cover, like Go) finishes in
    # seconds: maxCover0 from a seeded corpus, a fresh batch, 5k flakes
    fresh, mcp, mco, flakes = _config3(1_000, 8_000, 100_000)
    new = _check(fresh.pcs, fresh.off, fresh.group, 289, mcp, mco, flakes)
    assert 0 < new.sum() < fresh.n


def test_novelty_config3_property_large():
    # size-independent characterisation at a larger size (the oracle would take minutes):
    #   cover k is new  <=>  some pc of cov_k \ flakes \ {0xFFFFFFFF} \ maxCover0[g] occurs first in cov_k
    #   table_out[g]    == maxCover0[g] u (covers of g \ flakes \ {0xFFFFFFFF})   (no sentinel in this data)
    fresh, mcp, mco, flakes = _config3(10_000, 200_000, 500_000)
    G = 289
    new, out, ooff = cover.NoveltyBatch(fresh.pcs, fresh.off, fresh.group, G, mcp, mco, flakes)
    lens = np.diff(fresh.off).astype(np.int64)
    ent = np.repeat(np.arange(fresh.n), lens)
    key = (fresh.group[ent].astype(np.uint64) << np.uint64(32)) | fresh.pcs.astype(np.uint64)
    mg = np.repeat(np.arange(G), np.diff(mco).astype(np.int64)).astype(np.uint64)
    mkey = (mg << np.uint64(32)) | mcp.astype(np.uint64)
    keep = ~np.isin(fresh.pcs, flakes) & ~np.isin(key, mkey)
    uk, first = np.unique(key[keep], return_index=True)
    want_new = np.zeros(fresh.n, np.uint8)
    want_new[ent[keep][first]] = 1
    assert np.array_equal(new, want_new)
    want_keys = np.union1d(mkey, uk)
    og = np.repeat(np.arange(G), np.diff(ooff).astype(np.int64)).astype(np.uint64)
    assert np.array_equal((og << np.uint64(32)) | out.astype(np.uint64), want_keys)


@pytest.mark.timeout(300)
def test_novelty_config3_full_size():
    # configs[2] at full size (the bench leg's shape): maxCover0 of a 100k-program corpus, 1M fresh
    # covers (422M PCs) over a 2M-PC space, 5k flakes; checked against the per-call first-occurrence
    # oracle (oracle_novelty_mt, pinned to the literal oracle_novelty in tests/test_oracle.py)
    fresh, mcp, mco, flakes = _config3(100_000, 1_000_000, 2_000_000)
    w_new, w_mc, w_off = oracle.novelty_mt(fresh.pcs, fresh.off, fresh.group, 289, mcp, mco, flakes, 16)
    g_new, g_mc, g_off = cover.NoveltyBatch(fresh.pcs, fresh.off, fresh.group, 289, mcp, mco, flakes)
    assert np.array_equal(w_off, g_off)
    assert np.array_equal(w_mc, g_mc)
    assert np.array_equal(w_new, g_new)
    assert 0 < g_new.sum() < fresh.n


def _scopes(fn):
    """Run fn with the library's profiling scopes on; the set of scope names it recorded."""
    import ctypes
    L = _lib.lib()
    L.syzgpu_profile_only(None)
    L.syzgpu_profile_enable(1)
    try:
        res = fn()
    finally:
        cap = 4096
        names = ctypes.create_string_buffer(48 * cap)
        ms = np.zeros(cap, np.float32)
        by = np.zeros(cap, np.uint64)
        k = L.syzgpu_profile_read(names, ms.ctypes.data, by.ctypes.data, cap)
        L.syzgpu_profile_enable(0)
    return res, {names.raw[48 * i:48 * (i + 1)].split(b"\0")[0].decode() for i in range(k)}


def _stretch(pcs, base, k, add=0):
    """The monotone map base + (pc - base) * k + add (keeps every list strictly increasing)."""
    return (np.uint64(add) + np.uint64(base) + (pcs.astype(np.uint64) - np.uint64(base)) * np.uint64(k)).astype(np.uint32)


def _with_extremes(mcp, mco):
    """The tables with PC 0 first in call 0's and 0xFFFFFFFE last in the last call's."""
    add0 = not (mco[1] > 0 and mcp[0] == 0)
    out = np.concatenate([np.zeros(int(add0), np.uint32), mcp, np.array([0xFFFFFFFE], np.uint32)])
    mco = mco.copy()
    mco[1:] += np.uint64(add0)
    mco[-1] += np.uint64(1)
    return out, mco


def test_novelty_mixed_windows_vs_literal_oracle(strategy):
    # a narrow span (4 direct windows) where one call is dense (direct windows) and the others hold
    # fewer than NW_HSPARSE PCs per direct window (hashed windows): both kernels in one batch, the
    # updated tables interleaved by call in the output, bit-exact against the literal oracle
    if strategy != "windows":
        pytest.skip("the default strategy's per-call window choice")
    rnd = np.random.default_rng(51)
    base = 0x81000000
    pool = (base + 4 * np.arange(16_000)).astype(np.uint32)  # 64K addresses
    G = 5
    covs, grp = [], []
    for _ in range(1_500):  # call 2: ~600K PCs, dense
        covs.append(np.unique(rnd.choice(pool, size=400)))
        grp.append(2)
    for g in (0, 1, 3, 4):
        for _ in range(int(rnd.integers(20, 60))):
            covs.append(np.unique(rnd.choice(pool, size=int(rnd.integers(0, 40)))))
            grp.append(g)
    order = rnd.permutation(len(covs))
    covs = [covs[i].astype(np.uint32) for i in order]
    grp = np.array(grp, np.uint32)[order]
    mc = [np.unique(rnd.choice(pool, size=int(rnd.integers(0, 1_000)))).astype(np.uint32) for _ in range(G)]
    flakes = np.unique(rnd.choice(pool, size=200)).astype(np.uint32)
    pcs, off = oracle.to_csr(covs)
    mcp, mco = oracle.to_csr(mc)
    new, sc = _scopes(lambda: _check(pcs, off, grp, G, mcp, mco, flakes))
    assert "novelty_min" in sc and "novelty_min_hash" in sc
    assert 0 < new.sum() < len(covs)


@pytest.mark.parametrize("span", ["256M", "u32"])
def test_novelty_wide_span_small_vs_literal_oracle(span, strategy):
    # configs[2]-shaped data spread over a 280M-address span (past the direct windows' 32M) and over
    # the whole u32 space (0 and 0xFFFFFFFE held): the default strategy must stay on the windows
    # (hashed) and match the literal oracle
    if strategy not in ("windows", "hwindows"):
        pytest.skip("the windowed strategies' span coverage")
    fresh, mcp, mco, flakes = _config3(1_000, 8_000, 100_000)
    base = 0x81000000
    if span == "256M":
        f = lambda a: _stretch(a, base, 700)
    else:  # v = (pc - base) / 4 in [0, 100000) -> v * 42949: [0, 0xFFFE...]
        f = lambda a: ((a.astype(np.uint64) - np.uint64(base)) // np.uint64(4) * np.uint64(42949)).astype(np.uint32)
    pcs, mcp2, fl2 = f(fresh.pcs), f(mcp), f(flakes)
    mcp2, mco2 = _with_extremes(mcp2, mco)
    lo, hi = int(min(pcs.min(), mcp2.min())), int(max(pcs.max(), mcp2.max()))
    assert hi - lo >= (256 << 20)
    if span == "u32":
        assert lo == 0 and hi == 0xFFFFFFFE
    new, sc = _scopes(lambda: _check(pcs, fresh.off, fresh.group, 289, mcp2, mco2, fl2))
    assert "novelty_min_hash" in sc and "novelty_min" not in sc
    assert 0 < new.sum() < fresh.n


@pytest.mark.timeout(300)
@pytest.mark.parametrize("span", ["256M", "u32"])
def test_novelty_config3_full_size_wide_span(span, strategy):
    # configs[2] at full size (1M fresh covers, 422M PCs) with the 2M-PC space spread over 272M
    # addresses and over the whole u32 space: hashed windows, bit-exact against oracle_novelty_mt
    if strategy != "windows":
        pytest.skip("the default strategy's span coverage")
    fresh, mcp, mco, flakes = _config3(100_000, 1_000_000, 2_000_000)
    base = 0x81000000
    if span == "256M":
        f = lambda a: _stretch(a, base, 34)
    else:  # v in [0, 2M) -> v * 2147 (<= 0xFFF...)
        f = lambda a: ((a.astype(np.uint64) - np.uint64(base)) // np.uint64(4) * np.uint64(2147)).astype(np.uint32)
    pcs, mcp2, fl2 = f(fresh.pcs), f(mcp), f(flakes)
    mco2 = mco
    if span == "u32":
        mcp2, mco2 = _with_extremes(mcp2, mco)
    lo, hi = int(min(pcs.min(), mcp2.min())), int(max(pcs.max(), mcp2.max()))
    assert hi - lo >= (256 << 20)
    w_new, w_mc, w_off = oracle.novelty_mt(pcs, fresh.off, fresh.group, 289, mcp2, mco2, fl2, 16)
    (g_new, g_mc, g_off), sc = _scopes(lambda: cover.NoveltyBatch(pcs, fresh.off, fresh.group, 289, mcp2, mco2, fl2))
    assert "novelty_min_hash" in sc
    assert np.array_equal(w_off, g_off)
    assert np.array_equal(w_mc, g_mc)
    assert np.array_equal(w_new, g_new)
    assert 0 < g_new.sum() < fresh.n


def test_novelty_full_pc_space():
    # PCs across the whole u32 space (first/last bitmap page, 0, 0xFFFFFFFE, the sentinel), several
    # batches in a row (the table strategy's bitmap and table are left clean by each call)
    rnd = np.random.default_rng(11)
    edge = np.array([0, 1, 63, 64, 32767, 32768, 0x7FFFFFFF, 0x80000000, 0xFFFF8000, 0xFFFFFFFD, 0xFFFFFFFE],
                    np.uint32)
    G = 7
    for _ in range(4):
        pool = np.unique(np.concatenate([edge, rnd.integers(0, 2**32 - 1, size=300, dtype=np.uint64)
                                         .astype(np.uint32)]))
        n = 200
        covs = [np.unique(rnd.choice(pool, size=int(rnd.integers(0, 40)))) for _ in range(n)]
        covs[3] = np.append(covs[3], np.uint32(0xFFFFFFFF))  # the pool never holds the sentinel
        grp = rnd.integers(0, G, size=n).astype(np.uint32)
        mc = [np.unique(rnd.choice(pool, size=int(rnd.integers(0, 50)))) for _ in range(G)]
        mc[2] = np.unique(np.append(mc[2], np.uint32(0xFFFFFFFF)))
        mc[5] = np.array([0xFFFFFFFF], np.uint32)
        flakes = np.unique(rnd.choice(pool, size=30))
        pcs, off = oracle.to_csr(covs)
        mcp, mco = oracle.to_csr(mc)
        _check(pcs, off, grp, G, mcp, mco, flakes)


def test_novelty_window_edges():
    # a span of exactly 1024 windows ending at the top of the u32 space: PCs on window boundaries,
    # 0xFFFFFFFE, flakes on boundaries and inside tables, a table of only the sentinel, a call with
    # only its table, covers of only the sentinel, long covers crossing chunks (> 16384 PCs)
    rnd = np.random.default_rng(21)
    base = 0xFE000000
    bounds = np.array([base, base + 32767, base + 32768, base + 65535, 0xFFFF7FFF, 0xFFFF8000, 0xFFFFFFFE],
                      np.uint32)
    G = 6
    for _ in range(3):
        pool = np.unique(np.concatenate([bounds, (base + rnd.integers(0, 2**25 - 1, size=40_000)).astype(np.uint32)]))
        n = 300
        covs = [np.unique(rnd.choice(pool, size=int(rnd.integers(0, 60)))) for _ in range(n)]
        covs[5] = np.unique(rnd.choice(pool, size=30_000))
        covs[6] = np.array([0xFFFFFFFF], np.uint32)
        covs[7] = np.append(np.unique(rnd.choice(pool, size=20)), np.uint32(0xFFFFFFFF))
        grp = rnd.integers(0, G - 1, size=n).astype(np.uint32)  # call G-1: its table only
        mc = [np.unique(rnd.choice(pool, size=int(rnd.integers(0, 3000)))) for _ in range(G)]
        mc[1] = np.append(mc[1], np.uint32(0xFFFFFFFF))
        mc[3] = np.array([0xFFFFFFFF], np.uint32)
        mc[4] = np.unique(rnd.choice(pool, size=25_000))
        flakes = np.unique(np.concatenate([bounds[:3], rnd.choice(pool, size=50), mc[0][:5]]))
        pcs, off = oracle.to_csr(covs)
        mcp, mco = oracle.to_csr(mc)
        _check(pcs, off, grp, G, mcp, mco, flakes)


def test_novelty_good_batch_after_rejected_one():
    pcs = np.array([2, 1, 3], np.uint32)  # not canonical
    off = np.array([0, 3], np.uint64)
    with pytest.raises(_lib.SyzGpuError):
        cover.NoveltyBatch(pcs, off, np.zeros(1, np.uint32), 2, np.array([4, 5], np.uint32),
                           np.array([0, 2, 2], np.uint64), np.zeros(0, np.uint32))
    fresh, mcp, mco, flakes = _config3(300, 2_000, 50_000)
    _check(fresh.pcs, fresh.off, fresh.group, 289, mcp, mco, flakes)


def test_novelty_empty_batch_and_tables():
    _check(np.zeros(0, np.uint32), np.zeros(1, np.uint64), np.zeros(0, np.uint32), 3,
           np.zeros(0, np.uint32), np.zeros(4, np.uint64), np.zeros(0, np.uint32))


@pytest.mark.parametrize("what", ["cover", "table", "flakes", "group"])
def test_novelty_rejects_bad_input(what):
    pcs = np.array([1, 2, 3], np.uint32)
    off = np.array([0, 3], np.uint64)
    grp = np.array([0], np.uint32)
    mcp = np.array([4, 5], np.uint32)
    mco = np.array([0, 2, 2], np.uint64)
    fl = np.array([7, 8], np.uint32)
    if what == "cover":
        pcs = np.array([2, 1, 3], np.uint32)
    elif what == "table":
        mcp = np.array([5, 5], np.uint32)
    elif what == "flakes":
        fl = np.array([8, 7], np.uint32)
    else:
        grp = np.array([2], np.uint32)
    with pytest.raises(_lib.SyzGpuError) as e:
        cover.NoveltyBatch(pcs, off, grp, 2, mcp, mco, fl)
    assert e.value.code == _lib.EINVAL


@pytest.mark.parametrize("where", ["cover", "table"])
@pytest.mark.parametrize("at", [1, 63, 64, 16383, 16384, 19998])
def test_novelty_rejects_unsorted_anywhere(where, at):
    # one swapped pair inside a long list: inside a 64-PC tile, across tiles, across the 16384-PC
    # chunks of the window transpose, at the end; then an equal pair (not strictly increasing)
    good = (0x81000000 + 4 * np.arange(20_000)).astype(np.uint32)
    for kind in ("swap", "dup"):
        bad = good.copy()
        if kind == "swap":
            bad[at - 1], bad[at] = bad[at], bad[at - 1]
        else:
            bad[at] = bad[at - 1]
        covs = [good[:100], bad if where == "cover" else good]
        mc = [bad if where == "table" else good[::3], np.zeros(0, np.uint32)]
        pcs, off = oracle.to_csr(covs)
        mcp, mco = oracle.to_csr(mc)
        with pytest.raises(_lib.SyzGpuError) as e:
            cover.NoveltyBatch(pcs, off, np.array([1, 0], np.uint32), 2, mcp, mco, np.zeros(0, np.uint32))
        assert e.value.code == _lib.EINVAL
    pcs, off = oracle.to_csr([good[:100], good])
    mcp, mco = oracle.to_csr([good[::3], np.zeros(0, np.uint32)])
    _check(pcs, off, np.array([1, 0], np.uint32), 2, mcp, mco, np.zeros(0, np.uint32))


def test_novelty_capacity_error():
    import ctypes
    pcs = np.array([1, 2, 3], np.uint32)
    off = np.array([0, 3], np.uint64)
    grp = np.array([0], np.uint32)
    mco = np.zeros(2, np.uint64)
    is_new = np.zeros(1, np.uint8)
    out = np.zeros(2, np.uint32)
    ooff = np.zeros(2, np.uint64)
    p = lambda a: a.ctypes.data
    rc = _lib.lib().syzgpu_novelty_batch(p(pcs), p(off), p(grp), 1, 1, p(out), p(mco), None, 0, p(is_new), p(out),
                                         2, p(ooff))
    assert rc == _lib.ECAPACITY
    del ctypes


def test_novelty_device_entry_matches_host_entry():
    import torch
    dev = torch.device("cuda:0")
    base = synth.corpus(0x5EED0041, 3_000, 31, 40_000)
    mc_new, mcp, mco = cover.NoveltyBatch(base.pcs, base.off, base.group, 31, np.zeros(0, np.uint32),
                                           np.zeros(32, np.uint64), np.zeros(0, np.uint32))
    b = synth.corpus(0x5EED0042, 20_000, 31, 40_000)
    flakes = np.unique(b.pcs[::997])
    w_new, w_mc, w_off = cover.NoveltyBatch(b.pcs, b.off, b.group, 31, mcp, mco, flakes)

    def t(a):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
        return torch.from_numpy(np.ascontiguousarray(a).view(view.get(a.dtype, a.dtype))).to(dev)
    cap = int(mcp.size + b.pcs.size + 1)
    is_new = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    out = torch.zeros(cap, dtype=torch.int32, device=dev)
    ooff = torch.zeros(32, dtype=torch.int64, device=dev)
    cover.NoveltyBatchDev(t(b.pcs), t(b.off), t(b.group), b.n, 31, t(mcp), t(mco), int(mco[-1]), t(flakes),
                          flakes.size, int(b.off[-1]), is_new, out, cap, ooff)
    torch.cuda.synchronize()
    g_off = ooff.cpu().numpy().view(np.uint64)
    assert np.array_equal(g_off, w_off)
    assert np.array_equal(out.cpu().numpy().view(np.uint32)[: int(g_off[-1])], w_mc)
    assert np.array_equal(is_new.cpu().numpy(), w_new)
    # capacity and canonical-flakes errors come back as status codes
    with pytest.raises(_lib.SyzGpuError) as e:
        cover.NoveltyBatchDev(t(b.pcs), t(b.off), t(b.group), b.n, 31, t(mcp), t(mco), int(mco[-1]), t(flakes),
                              flakes.size, int(b.off[-1]), is_new, out, 10, ooff)
    assert e.value.code == _lib.ECAPACITY
    bad = t(flakes[::-1].copy())
    with pytest.raises(_lib.SyzGpuError) as e:
        cover.NoveltyBatchDev(t(b.pcs), t(b.off), t(b.group), b.n, 31, t(mcp), t(mco), int(mco[-1]), bad,
                              flakes.size, int(b.off[-1]), is_new, out, cap, ooff)
    assert e.value.code == _lib.EINVAL


def test_novelty_identical_keys():
    # one group, every cover the same PC: every radix digit agrees, so the sort strategy runs no pass
    # and the first-occurrence rule must still pick cover 0 (and the tables' entry when present)
    pc = np.uint32(0x81234567)
    covs = [np.array([pc], np.uint32) for _ in range(3000)]
    pcs, off = oracle.to_csr(covs)
    grp = np.zeros(len(covs), np.uint32)
    for mc in ([np.zeros(0, np.uint32)], [np.array([pc], np.uint32)]):
        mcp, mco = oracle.to_csr(mc)
        new = _check(pcs, off, grp, 1, mcp, mco, np.zeros(0, np.uint32))
        assert int(new.sum()) == (0 if mcp.size else 1)


@pytest.mark.parametrize("force_sort", [False, True])
def test_novelty_clustered_pcs(strategy, force_sort, monkeypatch):
    # real kcov PCs cluster by function: dense runs of PCs at a few far-apart addresses put thousands of
    # keys into one address bucket of a hashed window, where the kept keys are ordered by a sort instead
    # of a scan of their bucket; both windowed strategies against the literal oracle
    if strategy not in ("windows", "hwindows"):
        pytest.skip("the windowed strategies' ordering")
    if force_sort:  # every sub-range through the sort (the scan path's results, another way)
        monkeypatch.setenv("SYZGPU_NWH_SORT", "1")
    rnd = np.random.default_rng(41)
    G = 3
    bases = [0x10000000, 0x80000000, 0xF0000000]
    pool = np.concatenate([b + 4 * np.arange(20_000, dtype=np.uint64) for b in bases]).astype(np.uint32)

    def draw(k):
        c = rnd.integers(0, 3)
        lo = int(rnd.integers(0, 20_000 - k))
        return np.unique(pool[c * 20_000 + lo + rnd.integers(0, 4 * k, size=k).clip(0, 20_000 - lo - 1)])
    covs = [draw(int(rnd.integers(1, 400))) for _ in range(3_000)]
    grp = rnd.integers(0, G, size=len(covs)).astype(np.uint32)
    mc = [np.unique(pool[rnd.integers(0, pool.size, size=3_000)]) for _ in range(G)]
    flakes = np.unique(pool[rnd.integers(0, pool.size, size=50)])
    pcs, off = oracle.to_csr(covs)
    mcp, mco = oracle.to_csr(mc)
    new, sc = _scopes(lambda: _check(pcs, off, grp, G, mcp, mco, flakes))
    assert "novelty_min_hash" in sc
    assert 0 < new.sum() < len(covs)
