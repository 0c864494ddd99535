"""Signature sets (syzgpu_sigset_*) and the hub / persistent-corpus mirrors built on them
(syz-hub/state/state.go, syz-manager/manager.go:541-553 + persistent.go:91-102), on the GPU.

Exact integer/byte results: the set operations against numpy's unique/first-occurrence census of the
same signatures; the hub's Connect/Sync/pendingInputs/purgeCorpus against tests/pyref.py's literal
restatement with Go maps as dicts and hashlib SHA-1 (pendingInputs is a Go map range: compared as
sets). Parity unpinned by reference tests: syz-hub has none.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import _lib, hub, prog, synth  # noqa: E402
from tests import pyref  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def device():
    _lib.check(_lib.lib().syzgpu_init(0))
    yield


def _first_occurrence(sigs):
    v = np.ascontiguousarray(sigs).view(np.dtype((np.void, 20))).ravel()
    _, first = np.unique(v, return_index=True)
    want = np.zeros(sigs.shape[0], np.uint8)
    want[first] = 1
    return want


def test_sigset_batch_first_occurrence_and_lookup():
    rnd = np.random.default_rng(1)
    base = rnd.integers(0, 256, (50_000, 20), dtype=np.uint8)
    batch = base[rnd.integers(0, base.shape[0], 120_000)]  # many duplicates, random order
    s = hub.SigSet(16)  # grows several times
    added = s.insert(batch, seq=7)
    assert np.array_equal(added, _first_occurrence(batch))
    assert len(s) == int(added.sum())
    found, seq = s.lookup(base)
    present = np.isin(base.view(np.dtype((np.void, 20))).ravel(), batch.view(np.dtype((np.void, 20))).ravel())
    assert np.array_equal(found.astype(bool), present)
    assert np.all(seq[found == 1] == 7) and np.all(seq[found == 0] == 0)
    # a second batch: only signatures not already present are added
    more = rnd.integers(0, 256, (1000, 20), dtype=np.uint8)
    b2 = np.concatenate([batch[:5000], more, more[:10]])
    a2 = s.insert(b2, seq=8)
    assert a2[:5000].sum() == 0 and a2[5000:6000].sum() == 1000 and a2[6000:].sum() == 0
    ex, exq = s.export()
    assert ex.shape[0] == len(s)
    got = {bytes(x): int(q) for x, q in zip(ex, exq)}
    assert all(got[bytes(x)] == 8 for x in more)
    assert all(got[bytes(x)] == 7 for x in batch[:100])


def test_sigset_tag_collisions_and_probe_chains():
    # equal 64-bit tags (bytes 0..7) and equal home slots (bytes 8..15): only the last 4 bytes differ
    n = 3000
    sigs = np.zeros((n, 20), np.uint8)
    sigs[:, 16:20] = np.arange(n, dtype=np.uint32).view(np.uint8).reshape(n, 4)
    batch = np.concatenate([sigs, sigs[::-3]])
    s = hub.SigSet(1 << 14)
    added = s.insert(batch)
    assert np.array_equal(added, _first_occurrence(batch))
    assert len(s) == n
    f, _ = s.lookup(sigs)
    assert f.all()
    other = sigs.copy()
    other[:, 19] ^= 0x80  # same tag, never inserted (n < 2^31)
    f2, _ = s.lookup(other[:100])
    assert not f2.any()


def test_sigset_erase_and_revive():
    rnd = np.random.default_rng(2)
    sigs = rnd.integers(0, 256, (10_000, 20), dtype=np.uint8)
    s = hub.SigSet()
    s.insert(sigs, seq=1)
    dup_del = np.concatenate([sigs[:4000], sigs[:10]])
    er = s.erase(dup_del)
    # one item per signature erases (which one is unspecified: Go's delete reports nothing)
    assert er[10:4000].all() and np.all(er[:10] + er[4000:] == 1)
    assert len(s) == 6000
    f, _ = s.lookup(sigs)
    assert not f[:4000].any() and f[4000:].all()
    batch = np.concatenate([sigs[3000:5000], sigs[:1000]])  # 1000 erased ones again (revived), 1000 live
    a = s.insert(batch, seq=2)
    assert a[:1000].all() and not a[1000:2000].any() and a[2000:].all()
    assert int(a.sum()) == 2000
    f, q = s.lookup(sigs[:5000])
    assert f[:1000].all() and not f[1000:3000].any() and f[3000:].all()
    assert np.all(q[:1000] == 2) and np.all(q[3000:4000] == 2) and np.all(q[4000:5000] == 1)
    assert len(s) == 8000


def test_sigset_mask_skips_items():
    rnd = np.random.default_rng(3)
    sigs = rnd.integers(0, 256, (1000, 20), dtype=np.uint8)
    mask = (np.arange(1000) % 3 != 0).astype(np.uint8)
    s = hub.SigSet()
    a = s.insert(sigs, mask=mask)
    assert np.array_equal(a, mask)
    f, _ = s.lookup(sigs)
    assert np.array_equal(f, mask)


def test_hash_batch_matches_oracle_sha1_and_dedup_census():
    # 200k synthetic programs with 10% duplicates: GPU SHA-1 = oracle SHA-1, and the set's added flags
    # are the first occurrences of each distinct text
    lens = synth.corpus(0x5EED0041, 180_000, 289, 50_000).prog_len
    data, off = synth.prog_text(0x5EED0042, lens)
    rnd = np.random.default_rng(4)
    idx = np.concatenate([np.arange(lens.size), rnd.integers(0, lens.size, 20_000)])
    rnd.shuffle(idx)
    progs = [data[int(off[i]):int(off[i + 1])].tobytes() for i in idx]
    _, status, sigs = prog.ProgScan(progs, ncalls=False)
    assert not status.any()
    dblob, doff = prog._blob(progs[:3000], None)
    assert np.array_equal(sigs[:3000], oracle.sha1(dblob, doff))
    s = hub.SigSet()
    added = s.insert(sigs)
    assert np.array_equal(added, _first_occurrence(sigs))
    assert len(s) == len(set(progs))  # the generator repeats some short programs itself


def _progs(rnd, calls, n, bad_every=0):
    out = []
    for i in range(n):
        k = int(rnd.integers(1, 4))
        lines = []
        for j in range(k):
            c = calls[int(rnd.integers(0, len(calls)))]
            lines.append("r%d = %s(0x%x)" % (j, c, int(rnd.integers(0, 1 << 20))) if j % 2 else
                         "%s(0x%x, 0x%x)" % (c, int(rnd.integers(0, 8)), int(rnd.integers(0, 8))))
        if bad_every and i % bad_every == 0:
            lines.append("garbage line without bracket")
        out.append(("\n".join(lines) + "\n").encode())
    return out


def test_hub_state_vs_pyref():
    rnd = np.random.default_rng(5)
    calls = ["open", "read", "write", "close", "mmap", "ioctl", "socket"]
    want, got = pyref.HubState(), hub.State()
    pool = _progs(rnd, calls, 400, bad_every=17) + [b"# comment only\n", b"", b"x" * 70000 + b"\nopen()\n",
                                                   b"open()\n" + b"y" * 70000 + b"\n"]
    pick = lambda k: [pool[int(i)] for i in rnd.integers(0, len(pool), k)]  # noqa: E731
    mgrs = {"m0": calls, "m1": calls[:4], "m2": calls[2:]}
    for name, cl in mgrs.items():
        corpus = pick(120)
        want.connect(name, True, cl, corpus)
        got.Connect(name, True, cl, corpus)
    assert set(want.corpus) == set(bytes(x) for x in got.Corpus.export()[0])
    for step in range(12):
        name = list(mgrs)[step % 3]
        add = pick(int(rnd.integers(0, 40)))
        mine = [k.hex() for k in want.managers[name]["corpus"]]
        dels = [mine[int(i)] for i in rnd.integers(0, len(mine), 10)] if mine and step % 2 else []
        dels += ["zz", "abcd"]  # bad hashes are skipped
        w = want.sync(name, add, dels)
        g = got.Sync(name, add, dels)
        assert sorted(w) == sorted(g), step
        assert set(want.corpus) == set(bytes(x) for x in got.Corpus.export()[0]), step
        ws = {k: v[0] for k, v in want.corpus.items()}
        ex, q = got.Corpus.export()
        assert ws == {bytes(x): int(v) for x, v in zip(ex, q)}, step
    # a reconnect that is not fresh keeps the manager's seq
    c = pick(30)
    want.connect("m1", False, calls, c)
    got.Connect("m1", False, calls, c)
    add = pick(20)
    assert sorted(want.sync("m1", add, [])) == sorted(got.Sync("m1", add, []))
    got2, want2 = hub.State(), pyref.HubState()
    c = pick(50)
    want2.connect("a", True, calls, c)
    got2.Connect("a", True, calls, c)
    assert sorted(want2.sync("a", [], [])) == sorted(got2.Sync("a", [], []))


def test_persistent_minimize():
    rnd = np.random.default_rng(6)
    progs = _progs(rnd, ["open", "read"], 300)
    ps = hub.PersistentSet(progs)
    keep = [pyref.HubState()._sha1(p) for p in progs[::3]]
    a = ps.minimize(keep + [b"\x01" * 20])  # plus a "disabled hash" not in the set
    assert sorted(a) == sorted(set(progs[::3]))
