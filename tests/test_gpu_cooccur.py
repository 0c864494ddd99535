"""The call-ID co-occurrence XᵀX on int8 MFMA (syzgpu_call_cooccurrence) against the
oracle's literal pair loop (oracle_call_cooccurrence): exact int32 counts, bit-exact.

Not the reference's calcDynamicPrio (which counts call positions, tests/test_gpu_parity.py); this is
the call-ID reading of the same loop that the north_star names as the int8-MFMA contraction."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import _lib, prog  # noqa: E402

pytestmark = pytest.mark.gpu


def corpus_calls(seed, n, C, max_len=40, zipf=1.2):
    """n programs of 1 + Geometric(0.3) calls (<= max_len), call ids Zipf-distributed over [0, C)."""
    rnd = np.random.default_rng(seed)
    lens = np.minimum(1 + rnd.geometric(0.3, size=n) - 1, max_len).astype(np.uint64)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    w = 1.0 / np.arange(1, C + 1) ** zipf
    calls = rnd.choice(C, size=int(off[-1]), p=w / w.sum()).astype(np.uint16)
    return calls, off


def _check(calls, off, C):
    want = oracle.call_cooccurrence(calls, off, C)
    got = prog.CallCooccurrence(calls, off, C)
    assert np.array_equal(want, got)
    return got


@pytest.mark.parametrize("C,n", [(1, 10), (7, 0), (31, 50), (64, 1000), (129, 5000), (1159, 20_000)])
def test_cooccurrence_random(C, n):
    calls, off = corpus_calls(C * 7 + n, n, C)
    _check(calls, off, C)


def test_cooccurrence_matches_gram_form():
    # the same counts as X^T X - diag(occurrences) with X[p][c] = occurrences of call c in program p
    C, n = 40, 3000
    calls, off = corpus_calls(5, n, C)
    X = np.zeros((n, C), np.int64)
    np.add.at(X, (np.repeat(np.arange(n), np.diff(off).astype(np.int64)), calls.astype(np.int64)), 1)
    want = X.T @ X - np.diag(X.sum(axis=0))
    assert np.array_equal(_check(calls, off, C), want.astype(np.int32))


def test_cooccurrence_edges():
    C = 200
    progs = [[], [5], [5, 5], [199, 0, 199], list(range(C)) + list(range(C))[:50], [], [3] * 127]
    off = np.zeros(len(progs) + 1, np.uint64)
    np.cumsum([len(p) for p in progs], out=off[1:])
    calls = np.concatenate([np.array(p, np.uint16) for p in progs])
    got = _check(calls, off, C)
    # [3] * 127 gives 127 * 126; the 250-call program repeats calls 0..49 (two each: 2 more on each
    # of their diagonals, 2 x 2 per pair among them)
    assert got[3, 3] == 127 * 126 + 2 and got[5, 5] == 2 + 2
    assert got[199, 0] == got[0, 199] == 2 + 2 and got[199, 199] == 2 and got[100, 100] == 0


def test_cooccurrence_k_tail_and_splits(monkeypatch):
    # program counts around the 32-program K blocks, with the K split forced to several values
    # (KS a multiple of 8 takes the XCD-aware block mapping; C = 300 has 6 upper-triangle tiles)
    cases = [(96, n) for n in (31, 32, 33, 1023, 4097)] + [(300, 4097), (300, 20000)]
    for C, n in cases:
        calls, off = corpus_calls(n, n, C)
        want = oracle.call_cooccurrence(calls, off, C)
        for form in ("0", "1"):  # the direct operand loads and the LDS-staged default
            monkeypatch.setenv("SYZGPU_CO_FORM", form)
            for ks in ("1", "3", "16", "64"):
                monkeypatch.setenv("SYZGPU_CO_KS", ks)
                assert np.array_equal(prog.CallCooccurrence(calls, off, C), want)


@pytest.mark.parametrize("ks", ["1", "64"])
def test_cooccurrence_int32_overflow_is_an_error(monkeypatch, ks):
    # 140k programs of 127 calls 3: out[3][3] = 140k * 127 * 126 > 2^31 - 1. One K range: its partial
    # could wrap (sum of len^2 >= 2^31, err 4); 64 ranges: the partials are exact, the int64 sum is not
    # an int32 (err 8). Either way an error, never a wrapped count.
    n = 140_000
    off = (np.arange(n + 1, dtype=np.uint64) * 127).astype(np.uint64)
    calls = np.full(n * 127, 3, np.uint16)
    monkeypatch.setenv("SYZGPU_CO_KS", ks)
    with pytest.raises(_lib.SyzGpuError) as e:
        prog.CallCooccurrence(calls, off, 8)
    assert e.value.code == _lib.EINVAL
    # just below the limit, with the default K split: exact
    monkeypatch.delenv("SYZGPU_CO_KS")
    m = (2**31 - 1) // (127 * 126)
    got = prog.CallCooccurrence(calls[:m * 127], off[:m + 1], 8)
    assert int(got[3, 3]) == m * 127 * 126


@pytest.mark.parametrize("bad", ["call_id", "repeats"])
def test_cooccurrence_rejects(bad):
    C = 10
    progs = [[1, 2, 3], [10]] if bad == "call_id" else [[1, 2], [4] * 128]
    off = np.zeros(len(progs) + 1, np.uint64)
    np.cumsum([len(p) for p in progs], out=off[1:])
    calls = np.concatenate([np.array(p, np.uint16) for p in progs])
    with pytest.raises(_lib.SyzGpuError) as e:
        prog.CallCooccurrence(calls, off, C)
    assert e.value.code == _lib.EINVAL


@pytest.mark.timeout(300)
def test_cooccurrence_config4_size():
    # 1M programs of up to 40 calls over C = 1159 (the bench leg's shape)
    calls, off = corpus_calls(0xC0C0, 1_000_000, 1159)
    got = _check(calls, off, 1159)
    assert got.sum() == int((np.diff(off).astype(np.int64) * (np.diff(off).astype(np.int64) - 1)).sum())


def test_cooccurrence_device_entry():
    import torch
    dev = torch.device("cuda:0")
    C = 300
    calls, off = corpus_calls(77, 10_000, C)
    want = oracle.call_cooccurrence(calls, off, C)
    dc = torch.from_numpy(calls.view(np.int16)).to(dev)
    do = torch.from_numpy(off.view(np.int64)).to(dev)
    out = torch.empty((C, C), dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().syzgpu_call_cooccurrence_dev(dc.data_ptr(), do.data_ptr(), off.size - 1, C, out.data_ptr(),
                                                       torch.cuda.current_stream(dev).cuda_stream))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("world", [2, 8])
def test_cooccurrence_row_shards_on_gpu(world):
    # the north_star's multi-GPU form: corpus rows sharded over the ranks, each rank's XᵀX on the int8
    # matrix cores, one SUM all-reduce of the C x C partials (sharding.cooccurrence_shard); here the
    # ranks run one after another in this process and the partials are summed exactly as the
    # all-reduce sums them (int64, checked against int32)
    from syzkaller_amd import sharding
    C = 1159
    calls, off = corpus_calls(41, 200_000, C)
    want = oracle.call_cooccurrence(calls, off, C)
    b = sharding.cooccurrence_rows(off.size - 1, world)
    tot = np.zeros((C, C), np.int64)
    for r in range(world):
        tot += prog.CallCooccurrence(*sharding.cooccurrence_slice(calls, off, int(b[r]), int(b[r + 1])), C)
    assert tot.max() <= np.iinfo(np.int32).max
    assert np.array_equal(tot.astype(np.int32), want)
