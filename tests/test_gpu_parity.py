"""Parity of the MI355X path (libsyzgpu.so, through the C ABI) with the CPU oracle.

Bit-exact for every integer result (set ops, Canonicalize, Minimize selection and order, ChoiceTable)
and bit-exact for float32 priorities too (the north star allows 1e-6 relative; the kernels reproduce
Go's per-op float32 rounding, so the test demands identical bits). Layout mirrors
cover/cover_test.go: the known-answer tables first, then seeded random/property cases, then the
BASELINE.json configs at sizes the oracle finishes in seconds.
"""
import copy
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import _lib, cover, prog, synth  # noqa: E402

pytestmark = pytest.mark.gpu

SETOPS = {
    "difference": cover.Difference,
    "symmetric_difference": cover.SymmetricDifference,
    "union": cover.Union,
    "intersection": cover.Intersection,
}


@pytest.fixture(scope="session", autouse=True)
def device():
    n = np.zeros(1, np.int32)
    _lib.lib().syzgpu_device_count(_lib.ptr(n))
    assert n[0] >= 1, "GPU tests need a device (no CPU fallback exists)"
    _lib.check(_lib.lib().syzgpu_init(0))
    yield


# ---- cover_test.go tables ------------------------------------------------------------------------
@pytest.mark.parametrize("op", list(SETOPS))
def test_setop_golden(golden, op):
    for t in golden[op]:
        res = SETOPS[op](t["v0"], t["v1"])
        assert list(res) == t["r"], (op, t)


def test_canonicalize_golden(golden):
    for t in golden["canonicalize"]:
        buf = np.array(t["v0"], dtype=np.uint32)
        res = cover.Canonicalize(buf)
        assert list(res) == t["r"]
        if res.size:
            assert np.shares_memory(res, buf)  # Go returns cov[:i], aliasing the input (F6)


def test_minimize_golden(golden):
    for t in golden["minimize"]:
        assert cover.Minimize(t["inp"]) == t["out"], t


# ---- set operations ------------------------------------------------------------------------------
@pytest.mark.parametrize("seed", range(4))
def test_setops_random_vs_oracle(seed):
    rnd = np.random.default_rng(seed)
    a_list, b_list = [], []
    for _ in range(400):
        na, nb = int(rnd.integers(0, 50)), int(rnd.integers(0, 50))
        hi = int(rnd.choice([8, 100, 1 << 32]))
        a = np.sort(rnd.integers(0, hi, size=na, dtype=np.uint64)).astype(np.uint32)
        b = np.sort(rnd.integers(0, hi, size=nb, dtype=np.uint64)).astype(np.uint32)
        if rnd.random() < 0.15:
            a = np.append(a, np.uint32(0xFFFFFFFF))
        if rnd.random() < 0.15:
            b = np.append(b, np.uint32(0xFFFFFFFF))
        a_list.append(a)
        b_list.append(b)
    for op, fn in SETOPS.items():
        batch = cover.SetOpBatch(op, a_list, b_list)
        for a, b, got in zip(a_list, b_list, batch):
            want = oracle.setop(op, a, b)
            assert np.array_equal(got, want), (op, a, b)
        for a, b in list(zip(a_list, b_list))[:40]:
            assert np.array_equal(fn(a, b), oracle.setop(op, a, b))


def test_setops_large_lists():
    # maxCover-sized tables against execution covers (config 3 shape)
    rnd = np.random.default_rng(9)
    big = np.unique(rnd.integers(0, 1 << 24, size=300_000)).astype(np.uint32)
    covs = [np.unique(rnd.integers(0, 1 << 24, size=int(rnd.integers(1, 2000)))).astype(np.uint32)
            for _ in range(64)]
    for op in SETOPS:
        got = cover.SetOpBatch(op, covs, [big] * len(covs))
        for c, g in zip(covs, got):
            assert np.array_equal(g, oracle.setop(op, c, big)), op


def test_setop_batch_device_entry_triage_shape():
    # the device-pointer entry (bench leg setops_triage): pairs of two runs of one input's cover, the
    # second with PCs dropped (the triage loop's Intersection, fuzzer.go:389-406), and Difference /
    # Union / SymmetricDifference of the same pairs; plus empty pairs; bit-exact against the oracle
    import torch
    c = synth.corpus(0x5EED00C1, 3_000, 17, 60_000)
    rnd = np.random.default_rng(4)
    a_list = [c.cover(i) for i in range(c.n)]
    b_list = [x[rnd.random(x.size) > 0.05] for x in a_list]
    a_list[3] = np.zeros(0, np.uint32)
    b_list[5] = np.zeros(0, np.uint32)
    a, aoff = cover.to_csr(a_list)
    b, boff = cover.to_csr(b_list)

    def t(x):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
        return torch.from_numpy(np.ascontiguousarray(x).view(view.get(x.dtype, x.dtype))).to("cuda:0")
    da, dao, db, dbo = t(a), t(aoff), t(b), t(boff)
    for op in SETOPS:
        cap = a.size + b.size + 1
        out = torch.zeros(cap, dtype=torch.int32, device="cuda:0")
        ooff = torch.zeros(c.n + 1, dtype=torch.int64, device="cuda:0")
        tot = cover.SetOpBatchDev(op, da, dao, a.size, db, dbo, b.size, c.n, out, cap, ooff)
        o = out.cpu().numpy().view(np.uint32)
        oo = ooff.cpu().numpy().view(np.uint64)
        assert tot == int(oo[-1])
        for i in range(c.n):
            assert np.array_equal(o[int(oo[i]):int(oo[i + 1])], oracle.setop(op, a_list[i], b_list[i])), (op, i)


def _dev_setops(torch, a_list, b_list):
    a, aoff = cover.to_csr(a_list)
    b, boff = cover.to_csr(b_list)

    def t(x):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
        return torch.from_numpy(np.ascontiguousarray(x).view(view.get(x.dtype, x.dtype))).to("cuda:0")
    da, dao, db, dbo = t(a if a.size else np.zeros(1, np.uint32)), t(aoff), t(b if b.size else np.zeros(1, np.uint32)), t(boff)
    res = {}
    for op in SETOPS:
        cap = a.size + b.size + 1
        out = torch.zeros(cap, dtype=torch.int32, device="cuda:0")
        ooff = torch.zeros(len(a_list) + 1, dtype=torch.int64, device="cuda:0")
        tot = cover.SetOpBatchDev(op, da, dao, a.size, db, dbo, b.size, len(a_list), out, cap, ooff)
        o = out.cpu().numpy().view(np.uint32)
        oo = ooff.cpu().numpy().view(np.uint64)
        assert tot == int(oo[-1])
        res[op] = [o[int(oo[i]):int(oo[i + 1])] for i in range(len(a_list))]
    return res


def test_setop_tiles_boundaries_vs_oracle():
    # strictly increasing pairs (the merge-path tile path): merged lengths around multiples of the
    # 1024-element tile, equal values on both sides of tile cuts, identical / disjoint / one-sided
    # pairs, the sentinel at the end of either list
    import torch
    rnd = np.random.default_rng(21)
    a_list, b_list = [], []
    for m in [1, 63, 64, 1023, 1024, 1025, 2047, 2048, 2049, 5000, 20000]:
        for share in (0.0, 0.5, 1.0):
            u = np.unique(rnd.integers(0, 1 << 31, size=m)).astype(np.uint32)
            a = u[rnd.random(u.size) < 0.6]
            b = np.union1d(u[rnd.random(u.size) < 0.6], a[rnd.random(a.size) < share]).astype(np.uint32)
            a_list.append(a)
            b_list.append(b)
    a_list += [np.arange(0, 3000, 2, dtype=np.uint32), np.arange(3000, dtype=np.uint32),
               np.zeros(0, np.uint32), np.arange(1500, dtype=np.uint32)]
    b_list += [np.arange(0, 3000, 2, dtype=np.uint32), np.zeros(0, np.uint32),
               np.arange(10, 2000, 3, dtype=np.uint32), np.arange(1500, 3100, dtype=np.uint32)]
    a_list.append(np.append(np.arange(0, 2000, 2, dtype=np.uint32), np.uint32(0xFFFFFFFF)))
    b_list.append(np.append(np.arange(0, 2000, 3, dtype=np.uint32), np.uint32(0xFFFFFFFF)))
    got = _dev_setops(torch, a_list, b_list)
    for op in SETOPS:
        for i, (a, b) in enumerate(zip(a_list, b_list)):
            assert np.array_equal(got[op][i], oracle.setop(op, a, b)), (op, i)


def test_setop_batch_repeated_values_take_rank_path():
    # one pair with a repeated value (Go allows it): the whole batch takes the multiset rank path
    import torch
    rnd = np.random.default_rng(22)
    a_list = [np.unique(rnd.integers(0, 5000, size=800)).astype(np.uint32) for _ in range(50)]
    b_list = [np.unique(rnd.integers(0, 5000, size=900)).astype(np.uint32) for _ in range(50)]
    a_list[7] = np.array([1, 5, 5, 5, 9, 9], np.uint32)
    b_list[7] = np.array([5, 9, 9, 9, 12], np.uint32)
    got = _dev_setops(torch, a_list, b_list)
    for op in SETOPS:
        for i, (a, b) in enumerate(zip(a_list, b_list)):
            assert np.array_equal(got[op][i], oracle.setop(op, a, b)), (op, i)


def test_setop_batch_many_tiles_and_capacity():
    # ~40K merge tiles in one batch (the tiles' output offsets come from a look-back over all of them),
    # repeated twice (the look-back words are reused across calls), then the same batch with an output
    # capacity one short of the total: ECAPACITY, and no store past the buffer (a guard word after it)
    import torch
    c = synth.corpus(0x5EED00C7, 60_000, 31, 400_000)
    rnd = np.random.default_rng(9)
    a_list = [c.cover(i) for i in range(c.n)]
    b_list = [x[rnd.random(x.size) > 0.3] for x in a_list]
    a, aoff = cover.to_csr(a_list)
    b, boff = cover.to_csr(b_list)
    assert (a.size + b.size) // 1024 > 20_000

    def t(x):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
        return torch.from_numpy(np.ascontiguousarray(x).view(view.get(x.dtype, x.dtype))).to("cuda:0")
    da, dao, db, dbo = t(a), t(aoff), t(b), t(boff)
    aoff64, boff64 = aoff.astype(np.int64), boff.astype(np.int64)
    for op in SETOPS:
        for _ in range(2):
            cap = a.size + b.size
            out = torch.zeros(cap + 1, dtype=torch.int32, device="cuda:0")
            ooff = torch.zeros(c.n + 1, dtype=torch.int64, device="cuda:0")
            tot = cover.SetOpBatchDev(op, da, dao, a.size, db, dbo, b.size, c.n, out, cap, ooff)
            o = out.cpu().numpy().view(np.uint32)
            oo = ooff.cpu().numpy().view(np.uint64)
            want = [oracle.setop(op, a[aoff64[i]:aoff64[i + 1]], b[boff64[i]:boff64[i + 1]]) for i in range(c.n)]
            assert tot == sum(w.size for w in want) == int(oo[-1])
            assert np.array_equal(o[:tot], np.concatenate(want)), op
        guard = torch.full((tot + 8,), -7, dtype=torch.int32, device="cuda:0")
        with pytest.raises(_lib.SyzGpuError) as e:
            cover.SetOpBatchDev(op, da, dao, a.size, db, dbo, b.size, c.n, guard, tot - 1, ooff)
        assert e.value.code == _lib.ECAPACITY
        g = guard.cpu().numpy()
        assert (g[tot - 1:] == -7).all(), op


def test_setop_rejects_unsorted():
    with pytest.raises(_lib.SyzGpuError) as e:
        cover.Union([3, 1], [2])
    assert e.value.code == _lib.EINVAL


# ---- Canonicalize -----------------------------------------------------------------------------------
def test_canonicalize_random_vs_oracle():
    rnd = np.random.default_rng(1)
    covs = []
    for size in [0, 1, 2, 12, 13, 100, 1023, 1024, 1025, 16383, 16384, 16385, 40000]:
        covs.append(rnd.integers(0, max(2, size // 2), size=size, dtype=np.uint64).astype(np.uint32))
    covs.append(np.full(7, 0xFFFFFFFF, np.uint32))                       # only the sentinel -> empty
    covs.append(np.array([5, 0xFFFFFFFF, 5, 0xFFFFFFFF, 1], np.uint32))    # sentinel kept after others
    covs.append(rnd.integers(0, 1 << 32, size=5000, dtype=np.uint64).astype(np.uint32))
    pcs, off = cover.to_csr(covs)
    work = pcs.copy()
    lens = cover.CanonicalizeBatch(work, off)
    for i, c in enumerate(covs):
        want = oracle.canonicalize(c)
        got = work[int(off[i]):int(off[i]) + int(lens[i])]
        assert np.array_equal(got, want), i
        one = cover.Canonicalize(c.copy())
        assert np.array_equal(one, want), i


def test_canonicalize_batch_dev_classes_vs_oracle():
    # the device entry: every length class (<= 512 and <= 1024 one wave each, <= 2048, <= 16384,
    # <= 32768, longer), duplicates, the sentinel, empty covers; in place, lengths on the device
    import torch
    rnd = np.random.default_rng(23)
    sizes = [0, 1, 5, 63, 64, 65, 128, 129, 300, 511, 512, 513, 1000, 1024, 1025, 2048, 2049, 9000, 16384, 16385,
             20000, 32768, 32769, 33000, 70000]
    sizes += list(rnd.integers(1, 1500, size=300))
    covs = [rnd.integers(0, max(2, int(sz)), size=int(sz), dtype=np.uint64).astype(np.uint32) for sz in sizes]
    covs.append(np.full(9, 0xFFFFFFFF, np.uint32))
    covs.append(np.array([7, 0xFFFFFFFF, 3, 0xFFFFFFFF, 7], np.uint32))
    pcs, off = cover.to_csr(covs)
    d_pcs = torch.from_numpy(pcs.view(np.int32).copy()).to("cuda:0")
    d_off = torch.from_numpy(off.view(np.int64).copy()).to("cuda:0")
    d_len = torch.zeros(len(covs), dtype=torch.int64, device="cuda:0")
    cover.CanonicalizeBatchDev(d_pcs, d_off, len(covs), d_len)
    work = d_pcs.cpu().numpy().view(np.uint32)
    lens = d_len.cpu().numpy()
    for i, c in enumerate(covs):
        want = oracle.canonicalize(c)
        assert np.array_equal(work[int(off[i]):int(off[i]) + int(lens[i])], want), i


def test_canonicalize_batch_dev_canonical_fast_path_vs_oracle():
    # covers that are canonical already (the executor's dedup on) skip the sort: sorted + unique of
    # every length class, the sentinel alone (-> empty) or last (kept), empty covers; mixed with covers
    # that are one step from canonical (a repeat or an inversion at the very end of a long sorted run,
    # or at the start) and must take the full path
    import torch
    rnd = np.random.default_rng(29)
    S = 0xFFFFFFFF
    covs = []
    for sz in [0, 1, 2, 63, 64, 65, 255, 256, 257, 1000, 1024, 5000, 16384, 20000, 40000]:
        base = np.sort(rnd.choice(1 << 31, size=sz, replace=False)).astype(np.uint32)
        covs.append(base)
        if sz >= 2:
            rep = base.copy()
            rep[-1] = rep[-2]                       # a repeat at the end
            covs.append(rep)
            inv = base.copy()
            inv[-2], inv[-1] = inv[-1], inv[-2]     # an inversion at the end
            covs.append(inv)
            head = base.copy()
            head[0], head[1] = head[1], head[0]     # an inversion at the start
            covs.append(head)
    covs += [np.array([S], np.uint32), np.array([7, S], np.uint32), np.array([S, S], np.uint32),
             np.array([3, 9, S], np.uint32), np.zeros(0, np.uint32)]
    covs += [np.sort(rnd.choice(1 << 20, size=int(k), replace=False)).astype(np.uint32)
             for k in rnd.integers(1, 3000, size=200)]
    pcs, off = cover.to_csr(covs)
    d_pcs = torch.from_numpy(pcs.view(np.int32).copy()).to("cuda:0")
    d_off = torch.from_numpy(off.view(np.int64).copy()).to("cuda:0")
    d_len = torch.zeros(len(covs), dtype=torch.int64, device="cuda:0")
    cover.CanonicalizeBatchDev(d_pcs, d_off, len(covs), d_len)
    work = d_pcs.cpu().numpy().view(np.uint32)
    lens = d_len.cpu().numpy()
    for i, c in enumerate(covs):
        want = oracle.canonicalize(c)
        assert int(lens[i]) == want.size, i
        assert np.array_equal(work[int(off[i]):int(off[i]) + int(lens[i])], want), i


# ---- Minimize -----------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed", range(4))
def test_minimize_random_property(seed):
    # cover_test.go:170-205 with fixed seeds, plus exact equality with the oracle
    rnd = np.random.default_rng(seed)
    for _ in range(60):
        n = int(rnd.integers(0, 20))
        covs = [oracle.canonicalize(rnd.integers(0, 100, size=int(rnd.integers(0, 10)))) for _ in range(n)]
        got = cover.Minimize(covs)
        assert got == list(oracle.minimize(covs)) if n else got == []
        total = np.unique(np.concatenate(covs)) if n else np.zeros(0)
        mini = np.unique(np.concatenate([covs[i] for i in got])) if got else np.zeros(0)
        assert np.array_equal(total, mini)


@pytest.mark.parametrize("n,lenmax", [(13, 3), (41, 2), (200, 4), (1500, 3), (5000, 6), (30000, 5), (120000, 9)])
def test_minimize_tie_heavy_vs_oracle(n, lenmax):
    # many equal lengths: exercises every branch of the sort.Sort simulation (ninther, protect
    # pass, shell+insertion), across the finisher (<= 1024) and the level kernel (> 1024)
    rnd = np.random.default_rng(n)
    lens = rnd.integers(1, lenmax + 1, size=n)
    covs = [np.sort(rnd.choice(4 * lenmax + 40, size=int(l), replace=False)).astype(np.uint32) for l in lens]
    pcs, off = cover.to_csr(covs)
    assert np.array_equal(oracle.minimize(pcs=pcs, off=off), np.array(cover.Minimize(covs), dtype=np.int64))


def test_minimize_sort_permutation_distinct_and_sorted_lengths():
    for lens in [np.arange(3000), np.arange(3000)[::-1], np.zeros(3000, int) + 7]:
        covs = [np.arange(int(l) + 1, dtype=np.uint32) * 0 + np.uint32(i) for i, l in enumerate(lens)]
        pcs, off = cover.to_csr(covs)
        assert np.array_equal(oracle.minimize(pcs=pcs, off=off), np.array(cover.Minimize(covs), dtype=np.int64))


def _grouped_parity(c):
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    got, ggoff = cover.MinimizeCorpus(c.pcs, c.off, c.group, c.ngroups)
    assert np.array_equal(wgoff, ggoff)
    assert np.array_equal(want, got)
    # the resident store path (ingest once, minimize twice) gives the same selection
    st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
    for _ in range(2):
        sgot, sgoff = st.Minimize()
        assert np.array_equal(wgoff, sgoff)
        assert np.array_equal(want, sgot)
    st.close()
    return got


def test_minimize_corpus_config1_vs_oracle():
    # BASELINE.json configs[0]: 10k programs, ~50k PCs, 289 calls
    c = synth.corpus(0x5EED0001, 10_000, 289, 50_000)
    _grouped_parity(c)


def test_minimize_corpus_config2_vs_oracle():
    # BASELINE.json configs[1]: 100k programs, 500k PCs
    c = synth.corpus(0x5EED0002, 100_000, 289, 500_000)
    _grouped_parity(c)


def test_minimize_corpus_few_big_groups():
    # groups far above FIN_MAX (level kernel), short covers -> heavy ties, with 0xFFFFFFFF PCs
    c = synth.corpus(77, 60_000, 3, 3000, len_median=3.0, len_sigma=0.5)
    c.pcs[c.off[1:-1][::97].astype(np.int64) - 1] = 0xFFFFFFFF  # last PC of some covers
    _grouped_parity(c)


def _mirror_covers(c):
    # the same layout (entries, groups, cover lengths, PC span) with different PCs: each cover mapped by
    # pc -> lo + hi - pc and reversed, so it stays strictly increasing
    lo, hi = int(c.pcs.min()), int(c.pcs.max())
    lens = np.diff(c.off).astype(np.int64)
    ent = np.repeat(np.arange(c.n), lens)
    j = np.arange(len(c.pcs), dtype=np.int64)
    src = c.off[ent].astype(np.int64) + c.off[ent + 1].astype(np.int64) - 1 - j
    m = copy.copy(c)
    m.pcs = (np.uint64(lo + hi) - c.pcs[src].astype(np.uint64)).astype(np.uint32)
    return m


def test_minimize_speculative_plan_reuse():
    # minimize launches P on the last step's plan before it reads the layout back (panels.hip
    # begin_once): same layout (kept), same layout with other PCs (kept: the plan is a function of the
    # layout only), and another layout of the same size (the stale plan's P is discarded), alternating
    a = synth.corpus(0x5EED0011, 20_000, 289, 100_000)
    b = synth.corpus(0x5EED0012, 20_000, 289, 100_000)
    am = _mirror_covers(a)
    want = {}
    for name, c in (("a", a), ("b", b), ("am", am)):
        want[name] = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    for name in ["a", "a", "am", "b", "a", "am", "am", "b", "b", "a"]:
        c = {"a": a, "b": b, "am": am}[name]
        got, goff = cover.MinimizeCorpus(c.pcs, c.off, c.group, c.ngroups)
        assert np.array_equal(want[name][1], goff), name
        assert np.array_equal(want[name][0], got), name


def test_minimize_speculation_miss_after_miss():
    # the job speculates only once its layout repeated (panels.hip begin_once): a layout that changes on
    # every call pays at most one miss (a miss after a miss cannot happen), a corpus that grows between
    # calls (NewInputs between minimizes, manager.go:599-616) never speculates, and every call's result
    # matches the oracle through misses, re-plans and hits
    import torch
    a = synth.corpus(0x5EED0013, 20_000, 289, 100_000)
    b = synth.corpus(0x5EED0014, 20_000, 289, 100_000)
    g = synth.corpus(0x5EED0015, 22_000, 289, 100_000)
    dev = torch.device("cuda", 0)

    def t(x):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
        return torch.from_numpy(x.view(view.get(x.dtype, x.dtype))).to(dev)

    src = {k: (c, [t(c.pcs), t(c.off), t(c.group), t(c.prog_len)]) for k, c in (("a", a), ("b", b), ("g", g))}
    job = cover.MinimizeJob()
    s = torch.cuda.current_stream().cuda_stream
    want = {}
    seq = [("a", 20_000)] * 3 + [("b", 20_000)] * 3 + [("a", 20_000), ("b", 20_000), ("a", 20_000),
                                                      ("b", 20_000)] \
        + [("g", n) for n in (20_000, 20_500, 21_000, 21_500, 22_000)] + [("g", 22_000)] * 2
    hist = []
    for name, n in seq:
        c, d = src[name]
        if (name, n) not in want:
            want[name, n] = oracle.minimize_grouped(c.pcs[:int(c.off[n])], c.off[:n + 1], c.group[:n], c.ngroups)
        job.begin(d[0], d[1], d[2], n, c.ngroups, d[3], stream=s)
        got, goff = job.fetch(n, c.ngroups)
        assert np.array_equal(want[name, n][1], goff), (name, n)
        assert np.array_equal(want[name, n][0], got), (name, n)
        inf = job.info()
        hist.append((inf["spec_hits"], inf["spec_misses"]))
    hits = [h for h, _ in hist]
    misses = [m for _, m in hist]
    assert hits[2] == 1 and misses[2] == 0   # the third call on one layout kept its speculation
    assert misses[3] == 1                    # another layout of the same size: one miss
    assert hits[5] == 2 and misses[5] == 1   # ... then planned, then speculated again once it repeated
    assert misses[6] == 2                    # back to a: a miss
    assert misses[9] == 2 and hits[9] == 2   # alternating after a miss: planned steps, no miss after a miss
    assert misses[14] == 2 and hits[14] == 2  # a growing corpus: never speculated
    assert hits[-1] == 3                     # the grown corpus repeated: speculating again
    job.close()


def test_minimize_corpus_property_full_size():
    # size-independent property at the bench scale: per group, union(kept) == union(all)
    c = synth.corpus(0x5EED0004, 300_000, 289, 2_000_000)
    kept, goff = cover.MinimizeCorpus(c.pcs, c.off, c.group, c.ngroups)
    lens = np.diff(c.off).astype(np.int64)
    ent = np.repeat(np.arange(c.n), lens)
    key_all = (c.group[ent].astype(np.uint64) << np.uint64(32)) | c.pcs.astype(np.uint64)
    mask = np.zeros(c.n, bool)
    mask[kept] = True
    key_kept = key_all[mask[ent]]
    assert np.array_equal(np.unique(key_all), np.unique(key_kept))
    # selection order: within each group, kept entries have non-increasing cover length
    for g in range(c.ngroups):
        k = kept[int(goff[g]):int(goff[g + 1])]
        assert np.all(np.diff(lens[k]) <= 0)
        assert np.all(c.group[k] == g)


def test_store_many_windows_and_chunks():
    # calls with more than 32768 distinct PCs (several id windows) and windows split over chunks
    c = synth.corpus(0x5EED0005, 40_000, 2, 400_000, len_median=600.0)
    st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
    info = st.info()
    assert info["ids"] > 2 * 32768 and info["work_items"] > 2
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    got, goff = st.Minimize()
    assert np.array_equal(want, got) and np.array_equal(wgoff, goff)


def _store_parity(c):
    st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    got, goff = st.Minimize()
    assert np.array_equal(wgoff, goff)
    assert np.array_equal(want, got)
    got2, _ = st.Minimize()  # the store is reusable: same answer on every call
    assert np.array_equal(got2, got)
    return st


@pytest.mark.parametrize("seed,n,G,P", [(0x5EED0001, 10_000, 289, 50_000), (0x5EED0002, 100_000, 289, 500_000),
                                        (11, 30_000, 7, 200_000)])
def test_store_matches_oracle(seed, n, G, P):
    _store_parity(synth.corpus(seed, n, G, P))


def test_store_split_panels(monkeypatch):
    # every window's stream split over many work items -> per-window global tables + gtab_emit
    monkeypatch.setenv("SYZGPU_CHUNK_VECS", "97")
    st = _store_parity(synth.corpus(0x5EED0006, 20_000, 13, 120_000))
    assert st.info()["shared_tables"] > 10


def test_store_big_group_several_bitmap_passes():
    # one call with > 196608 entries: the LDS rank bitmap of the winners' emit takes several passes
    _store_parity(synth.corpus(0x5EED0007, 260_000, 1, 40_000, len_median=8.0, len_sigma=0.7))


def test_store_sentinel_and_empty_covers():
    c = synth.corpus(0x5EED0008, 5_000, 5, 20_000, len_median=20.0)
    covers = [c.cover(i).copy() for i in range(c.n)]
    for i in range(0, c.n, 53):
        covers[i] = np.zeros(0, np.uint32)            # empty cover: never kept
    for i in range(7, c.n, 31):
        if covers[i].size:
            covers[i][-1] = 0xFFFFFFFF                   # Minimize's map counts the sentinel (cover.go:115-127)
    pcs, off = cover.to_csr(covers)
    c2 = synth.Corpus(pcs, off, c.group, c.prog_len, c.ngroups)
    _store_parity(c2)


def test_store_resident_pipeline_matches_oracle():
    import torch
    C = 1159
    c = synth.corpus(0x5EED0009, 50_000, 289, 300_000)
    dev = torch.device("cuda:0")
    st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
    sel = torch.zeros(c.n, dtype=torch.uint8, device=dev)
    hist = torch.zeros(C + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    L = _lib.lib()
    for _ in range(2):
        _lib.check(L.syzgpu_corpus_minimize_dev(st.handle, C, sel.data_ptr(), hist.data_ptr(), stream))
    torch.cuda.synchronize()
    want_idx, _ = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    want_sel = np.zeros(c.n, np.uint8)
    want_sel[want_idx] = 1
    assert np.array_equal(sel.cpu().numpy(), want_sel)
    want_hist = np.bincount(c.prog_len[want_sel == 1], minlength=C + 1)
    assert np.array_equal(hist.cpu().numpy(), want_hist)


def test_store_rejects_non_canonical_covers():
    with pytest.raises(_lib.SyzGpuError) as e:
        cover.CoverStore(np.array([5, 5, 7], np.uint32), np.array([0, 3], np.uint64), np.array([0], np.uint32), 1)
    assert e.value.code == _lib.EINVAL


def test_minimize_rejects_bad_group():
    with pytest.raises(_lib.SyzGpuError) as e:
        cover.MinimizeCorpus(np.array([1, 2], np.uint32), np.array([0, 1, 2], np.uint64),
                             np.array([0, 5], np.uint32), 2)
    assert e.value.code == _lib.EINVAL


# ---- priorities / ChoiceTable ---------------------------------------------------------------------
def _static(C, seed):
    rnd = np.random.default_rng(seed)
    s = (rnd.random((C, C)) * 0.9 + 0.1).astype(np.float32)
    s[rnd.random((C, C)) < 0.1] = 0
    np.fill_diagonal(s, s.max(axis=1))
    return s


@pytest.mark.parametrize("C,nprogs", [(1, 5), (8, 0), (8, 50), (64, 3000), (1159, 100_000), (1536, 20_000)])
def test_priorities_bit_exact(C, nprogs):
    rnd = np.random.default_rng(C + nprogs)
    plen = rnd.integers(0, min(C, 40) + 1, size=nprogs).astype(np.uint16)
    st = _static(C, C)
    dyn_want = oracle.dynamic_prio(plen, C)
    dyn_got = prog.calcDynamicPrio(plen, C)
    assert np.array_equal(dyn_want.view(np.uint32), dyn_got.view(np.uint32))
    want = oracle.calculate_priorities(st, plen)
    got = prog.CalculatePriorities(st, plen)
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))
    for en in [None, (rnd.random(C) < 0.8).astype(np.uint8)]:
        wrun, wpres = oracle.build_choice_table(got, en)
        ct = prog.BuildChoiceTable(got, en)
        assert np.array_equal(wpres, ct.present)
        assert np.array_equal(wrun[wpres == 1], ct.run_matrix[wpres == 1])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("C,nlong", [(4096, 60), (16384, 12)])
def test_priorities_bit_exact_large_c(C, nlong):
    # a few program lengths over the whole [0, C] range, so every row's suffix sums H(k >= i) are
    # non-trivial (each row block of the fused kernel builds only its own [i, C) range); the oracle's
    # calcDynamicPrio is the literal O(sum len^2) loop, hence few long programs beside many short ones
    rnd = np.random.default_rng(C)
    plen = np.concatenate([rnd.integers(0, C + 1, size=nlong), rnd.integers(0, 41, size=20_000)]).astype(np.uint16)
    dyn_want = oracle.dynamic_prio(plen, C)
    dyn_got = prog.calcDynamicPrio(plen, C)
    assert np.array_equal(dyn_want.view(np.uint32), dyn_got.view(np.uint32))
    del dyn_want, dyn_got
    st = _static(C, C)
    want = oracle.calculate_priorities(st, plen)
    got = prog.CalculatePriorities(st, plen)
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))
    del want
    wrun, wpres = oracle.build_choice_table(got, None)
    ct = prog.BuildChoiceTable(got, None)
    assert np.array_equal(wpres, ct.present)
    assert np.array_equal(wrun, ct.run_matrix)


def test_choice_table_special_values():
    C = 16
    p = np.random.default_rng(3).random((C, C)).astype(np.float32)
    p[0, 3] = np.nan
    p[1, 1] = np.inf
    p[2, 5] = -np.inf
    p[3, 7] = 3e16        # int(p*1000) overflows int64 -> Go amd64 gives INT64_MIN
    p[4, :] = -0.7        # negative truncation toward zero
    wrun, wpres = oracle.build_choice_table(p, None)
    ct = prog.BuildChoiceTable(p, None)
    assert np.array_equal(wrun, ct.run_matrix)


def test_priorities_saturating_counts():
    # H(k) above 2^24: float32 += 1.0 sticks at 16777216 (the reference's accumulator)
    C = 4
    nprogs = (1 << 24) + 5000
    plen = np.full(nprogs, 3, np.uint16)
    got = prog.calcDynamicPrio(plen, C)
    raw = np.array([[0, 2**24, 2**24, 0], [2**24, 0, 2**24, 0], [2**24, 2**24, 0, 0], [0, 0, 0, 0]], np.float32)
    assert np.array_equal(oracle.normalize_prio(raw).view(np.uint32), got.view(np.uint32))


def test_priorities_reject_long_programs():
    with pytest.raises(_lib.SyzGpuError) as e:
        prog.calcDynamicPrio(np.array([3, 9], np.uint16), 8)
    assert e.value.code == _lib.EINVAL


# ---- device-resident pipeline (what bench.py times) -------------------------------------------------
def test_resident_pipeline_matches_oracle():
    import torch
    C = 1159
    c = synth.corpus(0x5EED0003, 20_000, 289, 100_000)
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else
                                   (a.view(np.int64) if a.dtype == np.uint64 else
                                    (a.view(np.int16) if a.dtype == np.uint16 else a))).to(dev)
    d_pcs, d_off, d_grp, d_len = t(c.pcs), t(c.off), t(c.group), t(c.prog_len)
    sel = torch.zeros(c.n, dtype=torch.uint8, device=dev)
    hist = torch.zeros(C + 1, dtype=torch.int64, device=dev)
    st = _static(C, 5)
    d_st = torch.from_numpy(st).to(dev)
    prios = torch.empty((C, C), dtype=torch.float32, device=dev)
    run = torch.empty((C, C), dtype=torch.int64, device=dev)
    pres = torch.empty(C, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    L = _lib.lib()
    _lib.check(L.syzgpu_minimize_grouped_dev(d_pcs.data_ptr(), d_off.data_ptr(), d_grp.data_ptr(), d_len.data_ptr(),
                                             c.n, c.ngroups, C, sel.data_ptr(), hist.data_ptr(), stream))
    _lib.check(L.syzgpu_prio_choice_dev(d_st.data_ptr(), hist.data_ptr(), C, None, prios.data_ptr(),
                                        run.data_ptr(), pres.data_ptr(), stream))
    torch.cuda.synchronize()
    want_idx, _ = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    want_sel = np.zeros(c.n, np.uint8)
    want_sel[want_idx] = 1
    assert np.array_equal(sel.cpu().numpy(), want_sel)
    # minimizeCorpus then CalculatePriorities(corpus) over the kept programs (manager.go:530-539)
    want_prios = oracle.calculate_priorities(st, c.prog_len[want_sel == 1])
    assert np.array_equal(want_prios.view(np.uint32), prios.cpu().numpy().view(np.uint32))
    wrun, _ = oracle.build_choice_table(want_prios, None)
    assert np.array_equal(wrun, run.cpu().numpy())
    out = np.empty(c.n, np.int64)
    goff = np.empty(c.ngroups + 1, np.uint64)
    _lib.check(L.syzgpu_minimize_grouped_fetch(out.ctypes.data, goff.ctypes.data, c.n, c.ngroups))
    assert np.array_equal(out[: int(goff[-1])], want_idx)
