"""The oracle's restatement of syz-manager/html.go's cover analytics (oracle_cover_stats,
oracle_corpus_cover) against the independent pure-Python transliteration in tests/pyref.py.

Parity unpinned by the reference's own tests: html.go has none. Both restatements follow
html.go:67-97, 158-170, 186-237 literally (Go maps, Union grown input by input, Canonicalize).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from tests import pyref  # noqa: E402

SENT = 0xFFFFFFFF


def _corpus(seed, n, G, P, sent_every=0, empty_every=0):
    rnd = np.random.default_rng(seed)
    covers, calls = [], []
    for i in range(n):
        L = int(rnd.integers(0, 12)) if not (empty_every and i % empty_every == 0) else 0
        cov = sorted(set(int(x) for x in rnd.integers(1, P, L)))
        if sent_every and i % sent_every == 3 and cov:
            cov[-1] = SENT
        covers.append(cov)
        calls.append(int(rnd.integers(0, G)))
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(c) for c in covers])
    pcs = np.array([p for c in covers for p in c], dtype=np.uint32)
    return covers, calls, pcs, off, np.array(calls, np.uint32)


@pytest.mark.parametrize("seed,n,G,P,sent", [(1, 60, 4, 40, 0), (2, 200, 7, 300, 9), (3, 150, 1, 60, 5),
                                             (4, 40, 12, 1000, 0)])
def test_cover_stats_vs_pyref(seed, n, G, P, sent):
    covers, calls, pcs, off, grp = _corpus(seed, n, G, P, sent_every=sent, empty_every=11)
    got = oracle.cover_stats(pcs, off, grp, G)
    want = pyref.cover_stats(covers, calls, G)
    for k in ("call_inputs", "call_cover", "call_unique", "input_unique"):
        assert list(got[k]) == list(want[k]), k
    assert list(got["totals"]) == [want["cover"], want["unique_per_call"], want["unique_per_input"]]


@pytest.mark.parametrize("seed,sent", [(5, 0), (6, 4)])
def test_corpus_cover_lists_vs_pyref(seed, sent):
    G = 5
    covers, calls, pcs, off, grp = _corpus(seed, 120, G, 200, sent_every=sent)
    for per_call, u in ((True, 1), (False, 2)):
        assert list(oracle.corpus_cover(pcs, off, grp, G, -1, u)) == pyref.unique_cover(covers, calls, per_call)
    all_cov = []
    for c in covers:
        all_cov = pyref.setop("union", all_cov, c)
    assert list(oracle.corpus_cover(pcs, off, grp, G, -1, 0)) == all_cov
    for g in range(G):
        cc = []
        for c, k in zip(covers, calls):
            if k == g:
                cc = pyref.setop("union", cc, c)
        assert list(oracle.corpus_cover(pcs, off, grp, G, g, 0)) == cc
        for per_call, u in ((True, 1), (False, 2)):
            want = pyref.setop("intersection", cc, pyref.unique_cover(covers, calls, per_call))
            assert list(oracle.corpus_cover(pcs, off, grp, G, g, u)) == want


def test_unique_cover_lone_sentinel():
    # Canonicalize's `last := sent` drops 0xFFFFFFFF only when it is the sole element (cover.go:28-40)
    covers = [[1, 2], [1, 2, SENT]]
    calls = [0, 0]
    pcs = np.array([1, 2, 1, 2, SENT], np.uint32)
    off = np.array([0, 2, 5], np.uint64)
    grp = np.array(calls, np.uint32)
    assert pyref.unique_cover(covers, calls, False) == []
    assert list(oracle.corpus_cover(pcs, off, grp, 1, -1, 2)) == []
    assert oracle.cover_stats(pcs, off, grp, 1)["totals"][2] == 0
    covers2 = [[1, SENT], [1, 5, SENT], [7]]
    pcs2 = np.array([1, SENT, 1, 5, SENT, 7], np.uint32)
    off2 = np.array([0, 2, 5, 6], np.uint64)
    assert pyref.unique_cover(covers2, [0, 0, 0], False) == [5, 7]
    assert list(oracle.corpus_cover(pcs2, off2, np.zeros(3, np.uint32), 1, -1, 2)) == [5, 7]
