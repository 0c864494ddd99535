"""The Go sort.Sort permutation of Minimize's inputs (cover/cover.go:106-113) on the MI355X, element
for element against the oracle's restatement (oracle/gosort.h, Go 1.6-1.18 quickSort).

Every path of the GPU simulation is covered: LDS packs of small call groups, global levels for groups
above 4096 entries, leaves, the ninther / medianOfThree choice, the dups probe and the protect pass
(heavy ties), and the u64 element fallback for lengths >= 2^20.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import cover  # noqa: E402

pytestmark = pytest.mark.gpu


def _pattern(kind, n, rnd):
    if kind == "few2":
        return rnd.integers(1, 3, size=n)
    if kind == "few5":
        return rnd.integers(1, 6, size=n)
    if kind == "equal":
        return np.full(n, 7)
    if kind == "asc":
        return np.arange(n) + 1
    if kind == "desc":
        return np.arange(n)[::-1] + 1
    if kind == "organ":
        h = np.arange(n) % (n // 2 + 1)
        return np.minimum(h, n - h) + 1
    if kind == "saw":
        return np.arange(n) % 17 + 1
    if kind == "wide":
        return rnd.integers(1, 1 << 30, size=n)
    if kind == "lognormal":
        return np.clip(np.exp(rnd.normal(np.log(256), 1.0, size=n)), 1, 16383).astype(np.int64)
    raise ValueError(kind)


def _check_groups(groups):
    lens = np.concatenate([np.asarray(g, np.uint64) for g in groups]) if groups else np.zeros(0, np.uint64)
    off = np.zeros(len(groups) + 1, np.uint64)
    np.cumsum([len(g) for g in groups], out=off[1:])
    got = cover.MinimizeOrder(lens, off)
    for i, g in enumerate(groups):
        want = oracle.minimize_order(np.asarray(g, np.uint64))
        a, b = int(off[i]), int(off[i + 1])
        assert np.array_equal(got[a:b], want), (i, len(g))


KINDS = ["few2", "few5", "equal", "asc", "desc", "organ", "saw", "wide", "lognormal"]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", [2, 12, 13, 40, 41, 100, 777, 4095, 4096])
def test_order_single_group_lds(kind, n):
    _check_groups([_pattern(kind, n, np.random.default_rng(n))])


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", [4097, 9000, 65_537, 250_000])
def test_order_single_group_global_levels(kind, n):
    _check_groups([_pattern(kind, n, np.random.default_rng(n + 1))])


def test_order_many_groups_packed():
    rnd = np.random.default_rng(5)
    groups = []
    for i in range(700):
        n = int(rnd.choice([0, 1, 2, 5, 12, 13, 30, 41, 200, 1000, 3000, 4096]))
        groups.append(_pattern(KINDS[i % len(KINDS)], n, rnd) if n else np.zeros(0, np.int64))
    groups += [_pattern("few5", 20_000, rnd), _pattern("lognormal", 70_000, rnd)]
    rnd.shuffle(groups)
    _check_groups(groups)


def test_order_zipf_corpus_shape():
    # the bench's shape: 289 calls, Zipf(1.1) sizes over 300k entries, lognormal lengths
    rnd = np.random.default_rng(9)
    w = 1.0 / np.arange(1, 290) ** 1.1
    sizes = rnd.multinomial(300_000, w / w.sum())
    _check_groups([_pattern("lognormal", int(s), rnd) for s in sizes])


def test_order_huge_lengths_u64_fallback():
    rnd = np.random.default_rng(11)
    g1 = rnd.integers(1, (1 << 32) - 1, size=3000)    # LDS pack with lengths >= 2^20
    g2 = rnd.integers(1 << 20, (1 << 20) + 3, size=9000)  # global levels, children bounce to u64
    _check_groups([g1, _pattern("few5", 500, rnd), g2])


def test_order_rejects_lengths_beyond_u32():
    from syzkaller_amd import _lib
    with pytest.raises(_lib.SyzGpuError) as e:
        cover.MinimizeOrder(np.array([1, 1 << 33], np.uint64))
    assert e.value.code == _lib.EINVAL


@pytest.mark.parametrize("kind", ["few5", "lognormal", "organ"])
def test_order_persistent_rounds(kind, monkeypatch):
    # the opt-in single-launch form of the global rounds (grid barriers instead of launches) must give
    # the same permutation as the graph form
    monkeypatch.setenv("SYZGPU_GR_PERSIST", "1")
    monkeypatch.setenv("SYZGPU_GR_PGRID", "64")
    rnd = np.random.default_rng(13)
    _check_groups([_pattern(kind, 250_000, rnd), _pattern("saw", 40_000, rnd), _pattern(kind, 9000, rnd)])


# ---- the other leaf form (syzgpu_set_go_sort_leaf(7): `for b-a > 7`, insertionSort alone) ----------
@pytest.fixture
def leaf7():
    cover.SetGoSortLeaf(7)
    oracle.set_go_sort_leaf(7)
    try:
        yield
    finally:
        cover.SetGoSortLeaf(12)
        oracle.set_go_sort_leaf(12)


@pytest.mark.parametrize("kind", KINDS)
def test_order_leaf7_form(kind, leaf7):
    # leaves of 2..7, the wave sorter from 8 elements, the LDS levels, the global levels' children
    rnd = np.random.default_rng(17)
    groups = [_pattern(kind, n, rnd) for n in [2, 7, 8, 9, 12, 13, 40, 41, 64, 65, 777, 4096, 9000, 65_537]]
    _check_groups(groups)


def test_minimize_corpus_leaf7_vs_oracle(leaf7):
    # the raw minimizeCorpus pipeline with the leaf-7 tie order, bit-exact: three call groups above the
    # LDS sorter's 8192 entries (global levels) and many small ones, cover lengths 1..6 (heavy ties)
    rnd = np.random.default_rng(23)
    sizes = [12_000, 9_500, 8_300] + [int(x) for x in rnd.integers(1, 300, size=40)]
    group = np.concatenate([np.full(s, g, np.uint32) for g, s in enumerate(sizes)])
    rnd.shuffle(group)
    lens = rnd.integers(1, 7, size=group.size)
    covs = [np.sort(rnd.choice(60, size=int(l), replace=False)).astype(np.uint32) + 1000 * np.uint32(g)
            for l, g in zip(lens, group)]
    pcs, off = cover.to_csr(covs)
    got, goff = cover.MinimizeCorpus(pcs, off, group, len(sizes))
    want, wgoff = oracle.minimize_grouped(pcs, off, group, len(sizes))
    assert np.array_equal(goff, wgoff)
    assert np.array_equal(got, want)
    # the two forms differ on this corpus (else the test would not tell them apart)
    cover.SetGoSortLeaf(12)
    oracle.set_go_sort_leaf(12)
    got12, _ = cover.MinimizeCorpus(pcs, off, group, len(sizes))
    assert not np.array_equal(got12, got)
