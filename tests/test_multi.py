"""The library-owned multi-GPU minimizeCorpus (syzkaller_amd/csrc/multi.hip, syzgpu_mgz_*).

CPU: the library's key-space plan (plan_parts / split_bounds restated in C++) equals the Python planner
bench.py's torch.distributed path uses (syzkaller_amd/sharding.py) on many layouts, so both multi-GPU
forms shard the same way. GPU: two sub-jobs on device 0 through the C ABI only (no torch.distributed):
the split group's selections exchanged inside the library, the histograms summed there, and every
output bit-exact against the oracle's single-process minimizeCorpus and priorities.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from syzkaller_amd import cover, sharding, synth  # noqa: E402


def _layouts():
    rnd = np.random.default_rng(3)
    out = []
    for n, G, P in [(6_000, 37, 30_000), (100_000, 289, 500_000), (1_000_000, 289, 2_000_000)]:
        g, off, _ = synth.layout(synth.params(0x5EED0004, n, G, P))
        out.append(sharding.layout_stats(g, off, G))
    for _ in range(6):  # random skewed layouts, some groups empty
        G = int(rnd.integers(2, 60))
        e = (rnd.pareto(1.1, G) * 3000).astype(np.int64)
        e[rnd.random(G) < 0.1] = 0
        p = e * rnd.integers(50, 800, G)
        out.append((e, p.astype(np.float64)))
    return out


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_library_plan_equals_python_plan(world):
    for ent, pcs in _layouts():
        want = sharding.plan_parts(ent, pcs, world)
        got, cost = cover.plan_parts(ent, pcs, world)
        assert [tuple(r) for r in want.ranks] == got
        assert np.allclose(want.cost, cost, rtol=0, atol=1e-9)


@pytest.mark.parametrize("world,k", [(2, 2), (4, 3), (8, 8)])
def test_library_forced_split_equals_python(world, k):
    for ent, pcs in _layouts()[:3]:
        kk = np.ones(ent.size, np.int64)
        kk[int(np.argmax(ent))] = min(k, world)
        want = sharding._assign(ent, pcs, kk, world)
        got, cost = cover.plan_parts(ent, pcs, world, split_largest=k)
        assert [tuple(r) for r in want[0]] == got
        assert np.allclose(want[1], cost, rtol=0, atol=1e-9)


def test_library_split_bounds_equal_python():
    c = synth.corpus(0x5EED0010, 20_000, 37, 30_000)
    ent, pcs = sharding.layout_stats(c.group, c.off, c.ngroups)
    plan = sharding.plan_parts(ent, pcs, 4)
    kk = np.ones(c.ngroups, np.int64)
    for g in np.argsort(-ent)[:3]:
        kk[g] = 4
    plan = sharding.KeyPlan(*sharding._assign(ent, pcs, kk, 4), ent)
    for r in range(4):
        want = sharding.split_bounds(plan, c, r)
        for g, b in want.items():
            got = cover.plan_split_bounds(c.pcs, c.off, c.group, g, len(plan.ranks[g]))
            assert np.array_equal(np.asarray(b, np.uint64), got), g


@pytest.mark.gpu
@pytest.mark.parametrize("split", [0, 2])
def test_multi_device_job_two_subjobs_on_one_gpu(split):
    import oracle
    from syzkaller_amd import prog
    C = 1159
    c = synth.corpus(0x5EED0020, 60_000, 289, 300_000)
    job = cover.MultiMinimizeJob([0, 0])
    job.load(c.pcs, c.off, c.group, c.prog_len, c.ngroups, split_largest=split)
    info = job.info()
    assert info["subjobs"] == 2 and sum(info["subjob_entries"]) >= c.n
    if split:
        assert info["split_groups"] == 1 and info["exchange_bytes"] > 0
    from syzkaller_amd import sysdesc
    uses = sysdesc.bundled().weights
    static = prog.calcStaticPriorities()  # the single-device entry (oracle-checked in test_gpu_static_prio)
    want_idx, want_goff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    want_hist = np.bincount(c.prog_len[want_idx], minlength=C + 1).astype(np.int64)
    wp = oracle.calculate_priorities(static, c.prog_len[want_idx])
    wrun, wpres = oracle.build_choice_table(wp)
    for _ in range(3):  # later calls on the cached plans (speculated steps)
        got, goff, hist, prios, run, rowp = job.minimize_prio(C, uses)
        assert np.array_equal(want_goff, goff)
        assert np.array_equal(want_idx, got)
        assert np.array_equal(want_hist, hist)
        assert np.array_equal(wp.view(np.uint32), prios.view(np.uint32))
        assert np.array_equal(wrun, run) and np.array_equal(wpres, rowp)
    job.close()
