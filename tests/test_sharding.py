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


def test_cost_model_units_are_microseconds():
    # the modelled step of one rank holding the whole bench corpus (config 4: 1M programs, 422M PCs)
    # is the measured N=1 step's order, a few thousand microseconds (a 1000x unit slip shows here)
    p = synth.params(0x5EED0004, 1_000_000, 289, 2_000_000)
    group, off, _ = synth.layout(p)
    e, w = sharding.layout_stats(group, off, 289)
    cost = sharding.plan_parts(e, w, 1).cost
    assert 1_000 < float(cost.max()) < 10_000
    # and at 8 ranks over the 8M-program job every rank models a step of the same order
    p8 = synth.params(0x5EED0004, 8_000_000, 289, 2_000_000)
    g8, o8, _ = synth.layout(p8)
    e8, w8 = sharding.layout_stats(g8, o8, 289)
    c8 = sharding.plan_parts(e8, w8, 8).cost
    assert 1_000 < float(c8.min()) <= float(c8.max()) < 10_000


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


# ---- the bench's own plan: plan_parts' PC-range key split, end to end (world 2 and 4) -------------
def _split_corpus():
    # a dominant call group (17k of 30k entries): plan_parts splits it at world 2 and 4
    return synth.corpus(0x5EED0011, 30_000, 3, 100_000, prog_len_max=40)


def _raw_job_cpu(covers, lo, hi):
    """CPU restatement of one rank's MinimizeJob on a call group (panels.hip with key_lo/key_hi):
    Go-sort positions from the FULL cover lengths (every holder sorts the whole group), each cover
    restricted to PCs in [lo, hi] (k_slices), a byte per sorted position = some restricted PC first
    occurs there. Returns (sel by position, order: position -> member)."""
    import oracle
    lens = np.array([len(x) for x in covers], np.uint64)
    order = oracle.minimize_order(lens)
    sel = np.zeros(len(covers), np.uint8)
    seen = set()
    for pos, m in enumerate(order):
        cov = covers[m]
        part = cov[(cov >= lo) & (cov <= hi)]
        if any(int(x) not in seen for x in part):
            sel[pos] = 1
        seen.update(int(x) for x in part)
    return sel, order


def _plan_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = _split_corpus()
        G = c.ngroups
        # bench.py's plan, shard and key ranges
        e, w = sharding.layout_stats(c.group, c.off, G)
        plan = sharding.plan_parts(e, w, world)
        ids = plan.local_entries(c.group, rank)
        local = synth.Corpus(*_sub(c, ids), G)
        key_lo, key_hi = plan.key_ranges(rank, sharding.split_bounds(plan, local, rank))
        _, _, count_hist = plan.store_parts(rank)
        gs, offs, nbytes = plan.split_groups()
        buf = torch.zeros(max(nbytes, 1), dtype=torch.uint8)
        jobs = {}
        for g in range(G):
            if not plan.held(rank)[g]:
                continue
            mem = np.nonzero(local.group == g)[0]
            covers = [local.cover(int(i)) for i in mem]
            sel, order = _raw_job_cpu(covers, int(key_lo[g]), int(key_hi[g]))
            jobs[g] = (mem, sel, order)
            if g in gs:  # export the split group's bytes (one per group-relative rank)
                j = int(np.nonzero(gs == g)[0][0])
                buf[int(offs[j]):int(offs[j]) + mem.size] = torch.from_numpy(sel)
        sharding.allreduce_max_u8(buf, dist)
        hist = torch.zeros(C + 1, dtype=torch.int64)
        kept_primary = []
        for g, (mem, sel, order) in jobs.items():
            if g in gs:  # import: OR the other holders' bytes back
                j = int(np.nonzero(gs == g)[0][0])
                sel = np.maximum(sel, buf[int(offs[j]):int(offs[j]) + mem.size].numpy())
            kept_local = mem[order[sel == 1]]  # selection order
            if count_hist[g]:
                hist += torch.from_numpy(np.bincount(local.prog_len[kept_local], minlength=C + 1).astype(np.int64))
                kept_primary.append(ids[kept_local])
        sharding.allreduce_hist(hist, dist)
        kp = np.concatenate(kept_primary) if kept_primary else np.zeros(0, np.int64)
        sel_all, goff = sharding.assemble_selection(kp, c.group, G, dist)
        q.put((rank, hist.numpy().copy(), sel_all, goff, len(gs)))
    finally:
        dist.destroy_process_group()


def _sub(c, ids):
    lens = np.diff(c.off)[ids].astype(np.uint64)
    off = np.zeros(ids.size + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    pcs = np.concatenate([c.cover(int(i)) for i in ids]) if ids.size else np.zeros(0, np.uint32)
    return pcs, off, c.group[ids], c.prog_len[ids]


def _spawn(target, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_bench_plan_key_split_matches_single_process(world):
    import oracle
    res = _spawn(_plan_rank, world)
    c = _split_corpus()
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    want_hist = np.bincount(c.prog_len[want], minlength=C + 1)
    for rank, hist, sel, goff, nsplit in res:
        assert nsplit >= 1  # the plan really split a group
        assert np.array_equal(hist, want_hist), rank
        assert np.array_equal(goff, wgoff), rank
        assert np.array_equal(sel, want), rank


# ---- the new-coverage batch sharded by PC value (world 2 and 3) -------------------------------------
def _novelty_inputs():
    S = 0xFFFFFFFF
    base = synth.corpus(0x5EED0012, 800, 13, 20_000)
    fresh = synth.corpus(0x5EED0013, 4_000, 13, 20_000)
    mc = []
    for g in range(13):
        ids = np.nonzero(base.group == g)[0]
        t = np.unique(np.concatenate([base.cover(int(i)) for i in ids])) if ids.size else np.zeros(0, np.uint32)
        if g % 5 == 0:
            t = np.append(t[t != S], np.uint32(S))  # a table holding the sentinel
        mc.append(t.astype(np.uint32))
    import oracle
    mcp, mco = oracle.to_csr(mc)
    covs = [fresh.cover(i).copy() for i in range(fresh.n)]
    for i in range(0, fresh.n, 29):
        covs[i] = np.append(covs[i][covs[i] != S], np.uint32(S)).astype(np.uint32)
    for i in range(3, fresh.n, 31):
        covs[i] = np.zeros(0, np.uint32)
    pcs, off = oracle.to_csr(covs)
    flakes = np.unique(pcs[::53][pcs[::53] != S]).astype(np.uint32)
    return pcs, off, fresh.group, 13, mcp, mco, flakes


def _novelty_rank(rank, world, port, q):
    import torch.distributed as dist
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pcs, off, grp, G, mcp, mco, flakes = _novelty_inputs()
        bounds = sharding.pc_bounds(pcs[::7], world)
        out = sharding.novelty_shard(pcs, off, grp, G, mcp, mco, flakes, rank, world, bounds, oracle.novelty, dist)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_novelty_pc_space_shards_match_single_process(world):
    import oracle
    res = _spawn(_novelty_rank, world)
    pcs, off, grp, G, mcp, mco, flakes = _novelty_inputs()
    w_new, w_mc, w_off = oracle.novelty(pcs, off, grp, G, mcp, mco, flakes)
    assert 0 < w_new.sum() < w_new.size
    for rank, (is_new, tab, toff) in res:
        assert np.array_equal(is_new, w_new), rank
        assert np.array_equal(toff, w_off), rank
        assert np.array_equal(tab, w_mc), rank


def test_slice_csr_and_bounds():
    pcs = np.array([1, 5, 9, 2, 3, 7, 0xFFFFFFFF], np.uint32)
    off = np.array([0, 3, 3, 7], np.uint64)
    p, o = sharding.slice_csr(pcs, off, 3, 8)
    assert list(p) == [5, 3, 7] and list(o) == [0, 1, 1, 3]
    p, o = sharding.slice_csr(pcs, off, 8, 0xFFFFFFFF)
    assert list(p) == [9, 0xFFFFFFFF] and list(o) == [0, 1, 1, 2]
    b = sharding.pc_bounds(np.arange(1000), 4)
    assert b[0] == 0 and b[-1] == 1 << 32 and np.all(np.diff(b.astype(np.int64)) > 0)


# ---- the call co-occurrence sharded by corpus rows: SUM all-reduce of the C x C partials --------------
def _cooc_rank(rank, world, port, q):
    import torch.distributed as dist

    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls, off, C = _cooc_corpus()
        got = sharding.cooccurrence_shard(calls, off, C, rank, world, oracle.call_cooccurrence, dist)
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def _cooc_corpus():
    rnd = np.random.default_rng(77)
    n, C = 3000, 61
    lens = np.minimum(rnd.geometric(0.3, size=n), 40).astype(np.uint64)
    lens[::50] = 0  # empty programs
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    calls = rnd.integers(0, C, size=int(off[-1])).astype(np.uint16)
    return calls, off, C


@pytest.mark.parametrize("world", [2, 3])
def test_cooccurrence_row_shards_sum_to_the_whole(world):
    import torch.multiprocessing as mp

    import oracle
    calls, off, C = _cooc_corpus()
    want = oracle.call_cooccurrence(calls, off, C)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cooc_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(60)
    for _, got in res:
        assert np.array_equal(got, want)
