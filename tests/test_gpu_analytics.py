"""The manager's cover analytics on the resident store (syz-manager/html.go:67-97, 158-170, 186-237)
through the C ABI, bit-exact against the oracle (oracle_cover_stats / oracle_corpus_cover) on seeded
corpora, and at full size through numpy identities (distinct-PC and count==1 census of the raw
covers). Parity unpinned by reference tests (html.go has none); the oracle is cross-checked against
tests/pyref.py in tests/test_oracle_analytics.py.
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
SENT = 0xFFFFFFFF


@pytest.fixture(scope="module", autouse=True)
def device():
    _lib.check(_lib.lib().syzgpu_init(0))
    yield


def _check_stats(c, calls=None):
    st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
    got = st.CoverStats()
    want = oracle.cover_stats(c.pcs, c.off, c.group, c.ngroups)
    for k in ("call_inputs", "call_cover", "call_unique", "input_unique"):
        assert np.array_equal(got[k], want[k]), k
    assert [got["cover"], got["unique_per_call"], got["unique_per_input"]] == list(want["totals"])
    if calls is None:
        calls = sorted(set([0, c.ngroups - 1, int(np.argmax(want["call_inputs"]))]))
    for call in [-1] + list(calls):
        for u in (0, 1, 2):
            w = oracle.corpus_cover(c.pcs, c.off, c.group, c.ngroups, call, u)
            g = st.Cover(call, u)
            assert np.array_equal(g, w), (call, u)
    got2 = st.CoverStats()  # recomputed on the same store: same answer
    assert np.array_equal(got2["input_unique"], got["input_unique"])
    return st, got


@pytest.mark.parametrize("seed,n,G,P", [(0x5EED0001, 10_000, 289, 50_000), (21, 20_000, 7, 200_000)])
def test_cover_stats_vs_oracle(seed, n, G, P):
    _check_stats(synth.corpus(seed, n, G, P))


def test_cover_stats_split_panels(monkeypatch):
    # windows split over many work items: the per-id holder merges through the global table
    monkeypatch.setenv("SYZGPU_CHUNK_VECS", "97")
    st, _ = _check_stats(synth.corpus(0x5EED0006, 20_000, 13, 120_000))
    assert st.info()["shared_tables"] > 10


def test_cover_stats_many_windows():
    c = synth.corpus(0x5EED0005, 20_000, 2, 400_000, len_median=600.0)
    st, _ = _check_stats(c, calls=[0, 1])
    assert st.info()["ids"] > 2 * 32768


def test_cover_stats_sentinel_and_empty_covers():
    c = synth.corpus(0x5EED0008, 5_000, 5, 20_000, len_median=20.0)
    covers = [c.cover(i).copy() for i in range(c.n)]
    for i in range(0, c.n, 53):
        covers[i] = np.zeros(0, np.uint32)
    for i in range(7, c.n, 31):
        if covers[i].size:
            covers[i][-1] = SENT
    pcs, off = cover.to_csr(covers)
    _check_stats(synth.Corpus(pcs, off, c.group, c.prog_len, c.ngroups), calls=range(5))


@pytest.mark.parametrize("covers,calls", [
    ([[SENT]], [0]),                                  # uniqueCover = Canonicalize([sent]) = []
    ([[1, SENT], [1, 5, SENT], [7]], [0, 0, 1]),      # sent in 2 inputs of one call
    ([[1, 2], [SENT], [2]], [0, 1, 0]),               # sent alone in its call, and in uniqueCover
    ([[], [], [3]], [2, 0, 2]),                       # an unused call, empty covers
])
def test_cover_stats_edge_cases(covers, calls):
    pcs, off = cover.to_csr([np.array(x, np.uint32) for x in covers])
    G = max(calls) + 1
    c = synth.Corpus(pcs, off, np.array(calls, np.uint32), np.ones(len(covers), np.uint16), G)
    _check_stats(c, calls=range(G))


def test_cover_stats_full_size_census():
    # 300k programs, 289 calls: every statistic against a numpy census of the raw covers
    c = synth.corpus(0x5EED0004, 300_000, 289, 2_000_000)
    st = cover.CoverStore(c.pcs, c.off, c.group, c.ngroups, c.prog_len)
    got = st.CoverStats()
    pc_u, pc_n = np.unique(c.pcs, return_counts=True)            # covers are canonical: count = inputs
    key = (c.group[np.repeat(np.arange(c.n), np.diff(c.off).astype(np.int64))].astype(np.uint64) << 32) | c.pcs
    keys = np.unique(key)
    kpc = (keys & 0xFFFFFFFF).astype(np.uint32)
    kpc_u, kpc_n = np.unique(kpc, return_counts=True)              # calls per PC
    assert got["cover"] == pc_u.size
    assert got["unique_per_input"] == int(np.sum(pc_n == 1))
    assert got["unique_per_call"] == int(np.sum(kpc_n == 1))
    assert np.array_equal(got["call_inputs"], np.bincount(c.group, minlength=c.ngroups))
    assert np.array_equal(got["call_cover"], np.bincount((keys >> 32).astype(np.int64), minlength=c.ngroups))
    one_call = np.isin(kpc, kpc_u[kpc_n == 1])
    assert np.array_equal(got["call_unique"],
                          np.bincount((keys[one_call] >> 32).astype(np.int64), minlength=c.ngroups))
    assert int(got["input_unique"].sum()) == got["unique_per_input"]
    uniq = pc_u[pc_n == 1]
    assert np.array_equal(st.UniqueCover(False), uniq)
    assert np.array_equal(st.UniqueCover(True), kpc_u[kpc_n == 1])
    assert np.array_equal(st.Cover(-1, 0), pc_u)
    # httpCorpus's per-input count for a sample of inputs
    for e in range(0, c.n, 9973):
        assert got["input_unique"][e] == np.intersect1d(c.cover(e), uniq).size
