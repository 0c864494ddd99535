"""calcStaticPriorities (prog/prio.go:40-135) on the GPU (static_prio.hip: int8-MFMA pair counts per
weight class, float64 combination, row max, normalizePrio) against oracle_static_priorities.

Bit-exact against the oracle's exact form (the same per-class-pair counts combined in the same order).
Against Go's own loop, which adds float32 products in its randomised map order, the tolerance is
1e-6 relative on the normalized priorities (BASELINE.json north_star), checked for several key orders.
The bundled matrix is the reference's sys/*.txt (1159 calls, 395 usage keys).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import _lib, prog, sysdesc  # noqa: E402

pytestmark = pytest.mark.gpu
F = np.float32
REL_TOL = 1e-6  # normalized priorities vs Go's float32 map-order sums (north_star)


@pytest.fixture(scope="module", autouse=True)
def device():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a device (no CPU fallback exists)"
    _lib.check(_lib.lib().syzgpu_init(0))


def _gpu(w):
    return prog.calcStaticPriorities(sysdesc.Usage(["c%d" % i for i in range(w.shape[1])],
                                                   ["k%d" % i for i in range(w.shape[0])], w))


def _rel(a, b):
    nan = np.isnan(b)
    assert np.array_equal(np.isnan(a), nan)  # all-equal rows normalize to 0/0 = NaN in Go too (prio.go:185)
    if not (~nan).any():
        return 0.0
    return float(np.max(np.abs(a[~nan].astype(np.float64) - b[~nan]) / np.abs(b[~nan])))


def _check(w, orders=3, seed=0, tol=None):
    """Bit-exact vs the exact form; vs Go's loop in `orders` random key orders within `tol` relative
    (default: 1e-6, or the spread between those Go orders themselves when that is larger: dense
    synthetic usage makes Go's own runs differ by more than 1e-6)."""
    got = _gpu(w)
    ex = oracle.static_priorities(w, exact=True)
    assert np.array_equal(got.view(np.uint32), ex.view(np.uint32))
    rnd = np.random.default_rng(seed)
    gos = [oracle.static_priorities(w, rnd.permutation(w.shape[0])) for _ in range(orders)]
    if tol is None:
        spread = max([_rel(a, b) for a in gos for b in gos] + [0.0])
        tol = max(REL_TOL, 1.5 * spread)
    for go in gos:
        assert _rel(go, got) <= tol
    return got


def test_bundled_sys_descriptions():
    u = sysdesc.bundled()
    got = _check(u.weights, orders=4, tol=REL_TOL)  # the north_star bound on the real descriptions
    assert got.shape == (1159, 1159)
    assert got.min() >= F(0.1) and got.max() <= F(1.0)


def _random_uses(rnd, nk, C, vals, density):
    w = np.zeros((nk, C), F)
    mask = rnd.random((nk, C)) < density
    w[mask] = rnd.choice(np.array(vals, F), size=int(mask.sum()))
    return w


@pytest.mark.parametrize("nk,C,density", [(1, 1, 1.0), (3, 2, 1.0), (31, 33, 0.3), (64, 64, 0.5),
                                          (395, 1159, 0.007), (500, 97, 0.2), (33, 300, 0.9)])
def test_random_shapes(nk, C, density):
    # tile edges (C and the key count around multiples of 32), dense and sparse usage
    rnd = np.random.default_rng(nk * 1000 + C)
    _check(_random_uses(rnd, nk, C, (0.1, 0.2, 0.5, 1.0), density), seed=C)


def test_eight_weight_classes_and_odd_values():
    rnd = np.random.default_rng(8)
    vals = (0.1, 0.2, 0.5, 1.0, 0.3, 0.7, 3.0, 1e-3)
    _check(_random_uses(rnd, 200, 150, vals, 0.2))


def test_rows_without_usage():
    # calls that share no key with any other call: a zero row, normalizePrio's max == 0 branch (all 1)
    rnd = np.random.default_rng(9)
    w = _random_uses(rnd, 50, 70, (0.1, 1.0), 0.2)
    w[:, 5] = 0
    w[:, 60:] = 0
    w[7, 60] = 1.0  # a key only call 60 uses: still no pair
    got = _check(w)
    assert np.all(got[5] == 1) and np.all(got[65] == 1)


def test_no_keys():
    got = _gpu(np.zeros((0, 40), F))
    assert np.all(got == 1)


@pytest.mark.parametrize("bad", ["nine", "nan", "inf"])
def test_rejects(bad):
    rnd = np.random.default_rng(10)
    if bad == "nine":
        w = _random_uses(rnd, 40, 30, tuple(0.1 * (i + 1) for i in range(9)), 0.9)
    else:
        w = _random_uses(rnd, 40, 30, (0.5,), 0.3)
        w[3, 4] = np.nan if bad == "nan" else np.inf
    with pytest.raises(_lib.SyzGpuError):
        _gpu(w)


def test_device_entry_feeds_calculate_priorities():
    # CalculatePriorities = normalized dynamic * static (prio.go:29-38), static from the bundled sys/
    import torch
    u = sysdesc.bundled()
    C = u.C
    s = torch.cuda.current_stream().cuda_stream
    d_w = torch.from_numpy(u.weights).cuda()
    d_static = torch.empty((C, C), dtype=torch.float32, device="cuda")
    _lib.check(_lib.lib().syzgpu_static_priorities_dev(d_w.data_ptr(), u.weights.shape[0], C, d_static.data_ptr(), s))
    lens = np.random.default_rng(11).integers(1, 30, size=20000).astype(np.uint16)
    hist = torch.from_numpy(np.bincount(lens, minlength=C + 1).astype(np.int64)).cuda()
    prios = torch.empty((C, C), dtype=torch.float32, device="cuda")
    _lib.check(_lib.lib().syzgpu_prio_choice_dev(d_static.data_ptr(), hist.data_ptr(), C, None, prios.data_ptr(),
                                                 None, None, s))
    torch.cuda.synchronize()
    st = oracle.static_priorities(u.weights, exact=True)
    assert np.array_equal(d_static.cpu().numpy().view(np.uint32), st.view(np.uint32))
    want = oracle.calculate_priorities(st, lens)
    assert np.array_equal(prios.cpu().numpy().view(np.uint32), want.view(np.uint32))
