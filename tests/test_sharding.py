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
