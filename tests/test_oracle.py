"""Pin the CPU oracle (oracle/liboracle.so) before trusting it as the parity checker.

* every known-answer table of cover/cover_test.go (:60-168), applied with runTest's rules (:31-58);
* TestMinimizeRandom's property (:170-205) with fixed, replayable seeds instead of time.Now();
* an independent pure-Python transliteration of cover.go / sort.Sort / prio.go on small cases;
* the closed forms SURVEY.md derives: Minimize == first-occurrence rule (F2) and
  calcDynamicPrio == H(max(i, j)) with a zero diagonal (F1).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from tests import pyref  # noqa: E402

SETOPS = ["difference", "symmetric_difference", "union", "intersection"]


def _is_sorted(a):
    return all(a[i] <= a[i + 1] for i in range(len(a) - 1))


@pytest.mark.parametrize("op", SETOPS)
def test_setop_tables(golden, op):
    for t in golden[op]:
        assert _is_sorted(t["v0"]) and _is_sorted(t["v1"]) and _is_sorted(t["r"])
        res = oracle.setop(op, t["v0"], t["v1"])
        assert _is_sorted(list(res))
        assert list(res) == t["r"], (op, t)


def test_canonicalize_table(golden):
    for t in golden["canonicalize"]:
        assert list(oracle.canonicalize(t["v0"])) == t["r"]


def test_minimize_table(golden):
    for t in golden["minimize"]:
        assert list(oracle.minimize(t["inp"])) == t["out"], t


@pytest.mark.parametrize("seed", range(8))
def test_minimize_random_property(seed):
    # cover_test.go:170-205 with a fixed seed: union of the minimized set == union of all
    rnd = np.random.default_rng(seed)
    for _ in range(100):
        n = int(rnd.integers(0, 20))
        covs = [oracle.canonicalize(rnd.integers(0, 100, size=int(rnd.integers(0, 10)))) for _ in range(n)]
        total = np.zeros(0, np.uint32)
        for c in covs:
            total = oracle.setop("union", total, c)
        mini = oracle.minimize(covs) if n else np.zeros(0, np.int64)
        got = np.zeros(0, np.uint32)
        for i in mini:
            got = oracle.setop("union", got, covs[i])
        assert list(total) == list(got)


@pytest.mark.parametrize("seed", range(6))
def test_oracle_matches_python_transliteration(seed):
    rnd = np.random.default_rng(100 + seed)
    for _ in range(60):
        a = np.sort(rnd.choice(64, size=int(rnd.integers(0, 20)), replace=True)).astype(np.uint32)
        b = np.sort(rnd.choice(64, size=int(rnd.integers(0, 20)), replace=True)).astype(np.uint32)
        if rnd.random() < 0.2:
            a = np.append(a, np.uint32(0xFFFFFFFF))
        for op in SETOPS:
            assert list(oracle.setop(op, a, b)) == pyref.setop(op, list(a), list(b)), op
        raw = rnd.integers(0, 40, size=int(rnd.integers(0, 60))).astype(np.uint32)
        assert list(oracle.canonicalize(raw)) == pyref.canonicalize(list(raw))
    # tie-heavy Minimize through both restatements of sort.Sort (n well above 12)
    for n in [13, 41, 100, 300, 1000]:
        lens = rnd.integers(1, 6, size=n)
        assert list(oracle.minimize_order(lens)) == pyref.minimize_order(list(lens)), n
        covs = [np.sort(rnd.choice(200, size=int(l) * 3, replace=False)).astype(np.uint32) for l in lens]
        assert list(oracle.minimize(covs)) == pyref.minimize([list(c) for c in covs])


def test_minimize_first_occurrence_rule():
    # input k (sorted position) is kept iff one of its PCs first occurs at position k
    rnd = np.random.default_rng(7)
    for _ in range(200):
        n = int(rnd.integers(1, 60))
        covs = [np.unique(rnd.integers(0, 80, size=int(rnd.integers(0, 12)))).astype(np.uint32) for _ in range(n)]
        lens = np.array([c.size for c in covs], dtype=np.uint64)
        perm = oracle.minimize_order(lens)
        first = {}
        for pos, i in enumerate(perm):
            for pc in covs[i]:
                first.setdefault(int(pc), pos)
        sel_pos = sorted(set(first.values()))
        assert list(oracle.minimize(covs)) == [int(perm[p]) for p in sel_pos]


def test_dynamic_prio_closed_form():
    # dyn[i][j] = #{p : len(p) > max(i, j)} for i != j, 0 on the diagonal (pre-normalize)
    rnd = np.random.default_rng(3)
    C = 24
    plen = rnd.integers(0, 20, size=500).astype(np.uint16)
    H = np.array([(plen > k).sum() for k in range(C)], dtype=np.float32)
    raw = np.array([[0.0 if i == j else H[max(i, j)] for j in range(C)] for i in range(C)], dtype=np.float32)
    assert np.array_equal(oracle.dynamic_prio(plen, C), oracle.normalize_prio(raw))
    assert np.array_equal(oracle.dynamic_prio(plen, C), pyref.dynamic_prio(list(plen), C))


def test_prio_and_choice_table_python_transliteration():
    rnd = np.random.default_rng(11)
    C = 17
    static = rnd.random((C, C)).astype(np.float32) * 0.9 + 0.1
    static[rnd.random((C, C)) < 0.2] = 0
    plen = rnd.integers(0, C + 1, size=300).astype(np.uint16)
    got = oracle.calculate_priorities(static, plen)
    want = pyref.calculate_priorities(static, list(plen))
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    enabled = (rnd.random(C) < 0.7).astype(np.uint8)
    for en in [None, enabled]:
        run, present = oracle.build_choice_table(got, en)
        wrun, wpresent = pyref.build_choice_table(got, None if en is None else list(en))
        assert list(present) == wpresent
        for i in range(C):
            if present[i]:
                assert list(run[i]) == wrun[i]


def test_prio_rejects_long_programs():
    with pytest.raises(RuntimeError):
        oracle.dynamic_prio(np.array([5, 9], np.uint16), 8)


def test_novelty_matches_python_transliteration():
    rnd = np.random.default_rng(5)
    G = 4
    for _ in range(30):
        n = int(rnd.integers(0, 40))
        covs = [np.unique(rnd.integers(0, 60, size=int(rnd.integers(0, 10)))).astype(np.uint32) for _ in range(n)]
        grp = rnd.integers(0, G, size=n).astype(np.uint32)
        mc = [np.unique(rnd.integers(0, 60, size=int(rnd.integers(0, 15)))).astype(np.uint32) for _ in range(G)]
        flakes = np.unique(rnd.integers(0, 60, size=5)).astype(np.uint32)
        pcs, off = oracle.to_csr(covs)
        mcp, mco = oracle.to_csr(mc)
        is_new, out_mc, out_off = oracle.novelty(pcs, off, grp, G, mcp, mco, flakes)
        w_new, w_mc = pyref.novelty([list(c) for c in covs], list(grp), [list(m) for m in mc], list(flakes))
        assert list(is_new) == w_new
        for g in range(G):
            assert list(out_mc[int(out_off[g]):int(out_off[g + 1])]) == w_mc[g]


def test_minimize_grouped_multithread_equals_serial():
    # the multi-core CPU baseline (bench.py cpu_baseline.multi_thread) computes the same selection
    from syzkaller_amd import synth
    c = synth.corpus(0x5EED0001, 10_000, 289, 50_000)
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    for nth in (1, 3, 8):
        got, goff = oracle.minimize_grouped_mt(c.pcs, c.off, c.group, c.ngroups, nth)
        assert np.array_equal(want, got) and np.array_equal(wgoff, goff)


@pytest.mark.parametrize("nth", [1, 4])
def test_novelty_first_occurrence_equals_literal(nth):
    # the full-size configs[2] checker (oracle_novelty_mt) against the literal per-cover merges, on
    # canonical batches: sentinel in covers and tables, flakes, empty covers and tables, calls with no
    # covers at all
    rnd = np.random.default_rng(17)
    S = 0xFFFFFFFF
    for it in range(40):
        G = int(rnd.integers(1, 7))
        n = int(rnd.integers(0, 80))
        covs = []
        for _ in range(n):
            c = np.unique(rnd.integers(0, 120, size=int(rnd.integers(0, 14)))).astype(np.uint32)
            if rnd.random() < 0.1:
                c = np.append(c, np.uint32(S))
            covs.append(c)
        grp = rnd.integers(0, G, size=n).astype(np.uint32)
        mc = []
        for _ in range(G):
            m = np.unique(rnd.integers(0, 120, size=int(rnd.integers(0, 30)))).astype(np.uint32)
            if rnd.random() < 0.2:
                m = np.append(m, np.uint32(S))
            mc.append(m)
        flakes = np.unique(rnd.integers(0, 120, size=int(rnd.integers(0, 10)))).astype(np.uint32)
        pcs, off = oracle.to_csr(covs)
        mcp, mco = oracle.to_csr(mc)
        w = oracle.novelty(pcs, off, grp, G, mcp, mco, flakes)
        g = oracle.novelty_mt(pcs, off, grp, G, mcp, mco, flakes, nth)
        assert np.array_equal(w[0], g[0]) and np.array_equal(w[1], g[1]) and np.array_equal(w[2], g[2]), it
    # the bench shape at a size the literal oracle finishes quickly
    from syzkaller_amd import synth
    base = synth.corpus(0x5EED0003, 500, 289, 50_000)
    lens = np.diff(base.off).astype(np.int64)
    ent = np.repeat(np.arange(base.n), lens)
    keys = np.unique((base.group[ent].astype(np.uint64) << np.uint64(32)) | base.pcs.astype(np.uint64))
    mco = np.zeros(290, np.uint64)
    np.cumsum(np.bincount((keys >> np.uint64(32)).astype(np.int64), minlength=289), out=mco[1:])
    mcp = (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    fresh = synth.corpus(0x5EED0103, 3000, 289, 50_000)
    flakes = np.unique(fresh.pcs[::97]).astype(np.uint32)
    w = oracle.novelty(fresh.pcs, fresh.off, fresh.group, 289, mcp, mco, flakes)
    g = oracle.novelty_mt(fresh.pcs, fresh.off, fresh.group, 289, mcp, mco, flakes, nth)
    assert all(np.array_equal(a, b) for a, b in zip(w, g))
    assert 0 < w[0].sum() < fresh.n


def test_oracle_call_cooccurrence_literal_pairs():
    # the oracle's pair loop against a direct Python restatement of the call-ID form of
    # prio.go:142-151 (for i0, for i1 != i0: prios[id(i0)][id(i1)] += 1)
    rnd = np.random.default_rng(9)
    C = 12
    progs = [list(rnd.integers(0, C, size=int(rnd.integers(0, 9)))) for _ in range(60)]
    want = np.zeros((C, C), np.int32)
    for p in progs:
        for i0 in range(len(p)):
            for i1 in range(len(p)):
                if i0 != i1:
                    want[p[i0], p[i1]] += 1
    off = np.zeros(len(progs) + 1, np.uint64)
    np.cumsum([len(p) for p in progs], out=off[1:])
    calls = np.array([c for p in progs for c in p], np.uint16)
    assert np.array_equal(oracle.call_cooccurrence(calls, off, C), want)


def test_go_sort_leaf_forms_oracle_vs_pyref():
    # both leaf forms of the restated quickSort (oracle/gosort.h) against the pure-Python restatement,
    # on tie-heavy lengths
    rnd = np.random.default_rng(77)
    try:
        for leaf in (7, 12):
            oracle.set_go_sort_leaf(leaf)
            for n in [1, 2, 7, 8, 9, 12, 13, 20, 41, 200, 1500]:
                for lenmax in [1, 2, 3, 6]:
                    lens = rnd.integers(0, lenmax, size=n).astype(np.uint64)
                    assert list(oracle.minimize_order(lens)) == pyref.minimize_order(list(lens), leaf=leaf), (leaf, n)
        # the forms give different tie orders (8..12 elements with ties reach a doPivot under 7 only)
        samples = [list(rnd.integers(0, 3, size=int(k))) for k in rnd.integers(8, 13, size=50)]
        assert any(pyref.minimize_order(l, leaf=12) != pyref.minimize_order(l, leaf=7) for l in samples)
        with pytest.raises(ValueError):
            oracle.set_go_sort_leaf(9)
    finally:
        oracle.set_go_sort_leaf(12)
