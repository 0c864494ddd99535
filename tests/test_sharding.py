"""The N>1 path of minimizeCorpus on CPU: world_size 2 and 4 over gloo (one process per rank).

Each rank takes its call-group shard (syzkaller_amd.sharding), minimizes it with the oracle standing in
for its GPU, all-reduces the kept-length histogram (the one real exchange, prio.go:29-38 over all kept
programs) and the kept ids. The result must equal the single-process minimizeCorpus bit for bit.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from syzkaller_amd import sharding, synth  # noqa: E402

C = 64


def _corpus():
    return synth.corpus(0x5EED0010, 6_000, 37, 30_000, prog_len_max=40)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = _corpus()
        owner, load = sharding.lpt_assign(sharding.group_weights(c.group, c.off, c.ngroups), world)
        ids = sharding.local_entries(c.group, owner, rank)
        sub_off = np.zeros(ids.size + 1, np.uint64)
        np.cumsum(np.diff(c.off)[ids], out=sub_off[1:])
        sub_pcs = np.concatenate([c.cover(int(i)) for i in ids]) if ids.size else np.zeros(0, np.uint32)
        kept_local, _ = oracle.minimize_grouped(sub_pcs, sub_off, c.group[ids], c.ngroups)  # GPU stand-in
        kept = ids[kept_local]
        hist = torch.from_numpy(np.bincount(c.prog_len[kept], minlength=C + 1).astype(np.int64))
        sharding.allreduce_hist(hist, dist)
        sel, goff = sharding.assemble_selection(kept, c.group, c.ngroups, dist)
        q.put((rank, hist.numpy().copy(), sel, goff, load))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_minimize_corpus_matches_single_process(world):
    import torch.multiprocessing as mp

    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = _corpus()
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    want_hist = np.bincount(c.prog_len[want], minlength=C + 1)
    for rank, hist, sel, goff, load in res:
        assert np.array_equal(hist, want_hist), rank
        assert np.array_equal(sel, want), rank
        assert np.array_equal(goff, wgoff), rank
        assert load.size == world


def test_lpt_assign_is_total_and_deterministic():
    rnd = np.random.default_rng(0)
    w = rnd.zipf(1.3, size=289).astype(np.float64)
    o1, l1 = sharding.lpt_assign(w, 8)
    o2, l2 = sharding.lpt_assign(w.copy(), 8)
    assert np.array_equal(o1, o2) and np.array_equal(l1, l2)
    assert set(o1.tolist()) <= set(range(8))
    assert np.isclose(l1.sum(), w.sum())
    for r in range(8):
        assert np.isclose(l1[r], w[o1 == r].sum())
    # LPT bound: max load <= mean + max single weight
    assert l1.max() <= w.sum() / 8 + w.max() + 1e-9


def test_local_entries_partition_the_corpus():
    c = _corpus()
    owner, _ = sharding.lpt_assign(sharding.group_weights(c.group, c.off, c.ngroups), 3)
    parts = [sharding.local_entries(c.group, owner, r) for r in range(3)]
    allids = np.sort(np.concatenate(parts))
    assert np.array_equal(allids, np.arange(c.n))
    for p in parts:
        assert np.all(np.diff(p) > 0)  # corpus order preserved inside a shard (Minimize's inputs[] order)


def test_single_rank_helpers_without_dist():
    import torch
    h = torch.arange(5, dtype=torch.int64)
    assert sharding.allreduce_hist(h) is h
    ids, goff = sharding.assemble_selection(np.array([4, 1, 2]), np.array([1, 0, 1, 0, 1]), 2)
    assert list(ids) == [1, 4, 2] and list(goff) == [0, 1, 3]


# ---- key-space sharding (groups split by PC keys over ranks) -------------------------------------
def test_plan_parts_splits_the_bottleneck_group_and_is_deterministic():
    p = synth.params(0x5EED0004, 8_000_000, 289, 2_000_000)
    group, off, _ = synth.layout(p)
    e, w = sharding.layout_stats(group, off, 289)
    plan = sharding.plan_parts(e, w, 8)
    again = sharding.plan_parts(e.copy(), w.copy(), 8)
    assert plan.ranks == again.ranks
    whole, whole_cost = sharding._assign(e, w, np.ones(289, np.int64), 8)
    assert plan.cost.max() < whole_cost.max()  # the split improves the modelled step
    gs, offs, nbytes = plan.split_groups()
    assert int(np.argmax(e)) in gs.tolist()
    assert nbytes == int(e[gs].sum())
    for g, r in enumerate(plan.ranks):
        assert (len(r) > 0) == (e[g] > 0)
        assert len(set(r)) == len(r)  # parts of a group on distinct ranks
    # every entry is held by the ranks of its group, and primaries count each group once
    counts = np.zeros(289, np.int64)
    for r in range(8):
        part, nparts, count = plan.store_parts(r)
        counts += count
        held = plan.held(r)
        assert np.array_equal(nparts[held] > 1, np.array([len(plan.ranks[g]) > 1 for g in np.nonzero(held)[0]]))
    assert np.array_equal(counts, (e > 0).astype(np.int64))


def test_plan_parts_single_rank_keeps_groups_whole():
    c = _corpus()
    e, w = sharding.layout_stats(c.group, c.off, c.ngroups)
    plan = sharding.plan_parts(e, w, 1)
    assert plan.split_groups()[0].size == 0
    assert np.array_equal(plan.local_entries(c.group, 0), np.arange(c.n))


def _partial_selection(covers, part, nparts):
    """CPU stand-in for one rank's key part of a call group's Minimize (the GPU splits by dense-PC
    windows, this by pc % nparts; the algebra is the same): byte per sorted position, 1 iff some PC
    of the part first occurs there."""
    import oracle
    lens = np.array([len(x) for x in covers], np.uint64)
    order = oracle.minimize_order(lens)  # sorted position -> input
    pcs = np.concatenate([np.asarray(covers[i], np.uint64) for i in order]) if len(covers) else np.zeros(0)
    pos = np.repeat(np.arange(len(covers)), lens[order].astype(np.int64))
    keep = (pcs % nparts) == part
    pcs, pos = pcs[keep], pos[keep]
    sel = np.zeros(len(covers), np.uint8)
    if pcs.size:
        o = np.lexsort((pos, pcs))
        first = np.ones(o.size, bool)
        first[1:] = pcs[o][1:] != pcs[o][:-1]
        sel[pos[o][first]] = 1
    return sel, order


def _keyshard_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = _corpus()
        e, w = sharding.layout_stats(c.group, c.off, c.ngroups)
        k = np.where(e >= np.sort(e)[-3], world, 1)  # the three largest groups split over all ranks
        ranks, cost = sharding._assign(e, w, k, world)
        plan = sharding.KeyPlan(ranks, cost, e)
        gs, offs, nbytes = plan.split_groups()
        buf = torch.zeros(nbytes, dtype=torch.uint8)
        final = {}
        for g in range(c.ngroups):
            r = plan.ranks[g]
            if rank not in r:
                continue
            ids = np.nonzero(c.group == g)[0]
            covers = [c.cover(int(i)) for i in ids]
            if len(r) > 1:
                sel, order = _partial_selection(covers, r.index(rank), len(r))
                j = int(np.nonzero(gs == g)[0][0])
                buf[int(offs[j]):int(offs[j]) + ids.size] = torch.from_numpy(sel)
                final[g] = (ids, order)
            else:
                sel, order = _partial_selection(covers, 0, 1)
                final[g] = (ids, order, sel)
        sharding.allreduce_max_u8(buf, dist)
        kept = {}
        for g, v in final.items():
            if len(v) == 2:
                ids, order = v
                j = int(np.nonzero(gs == g)[0][0])
                sel = buf[int(offs[j]):int(offs[j]) + ids.size].numpy()
            else:
                ids, order, sel = v
            kept[g] = np.sort(ids[order[sel == 1]])
        q.put((rank, kept))
    finally:
        dist.destroy_process_group()


def test_key_parts_or_to_the_full_minimize_world2():
    import torch.multiprocessing as mp

    import oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_keyshard_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = _corpus()
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    seen = set()
    for rank, kept in res:
        for g, ids in kept.items():
            w = np.sort(want[int(wgoff[g]):int(wgoff[g + 1])])
            assert np.array_equal(ids, w), (rank, g)
            seen.add(g)
    assert seen == set(np.unique(c.group).tolist())
