"""The multi-GPU path of SURVEY.md §8e run for real across processes: world-2 gloo ranks, both on
cuda:0 (the bench's SYZ_BENCH_SAME_DEVICE rehearsal), each running the HIP sequence bench.py runs per
rank -- plan_parts, MinimizeJob.begin with its key ranges, export_sel -> MAX all-reduce -> import_sel,
end, the length-histogram all-reduce, then CalculatePriorities + BuildChoiceTable on the reduced
histogram (syzgpu_prio_choice_dev) -- and, for the new-coverage check, sharding.novelty_shard with
syzgpu_novelty_batch_dev on each rank's PC range. The assembled selection, histogram, priorities,
ChoiceTable, flags and tables must equal the single-process oracle bit for bit
(oracle_minimize_grouped, oracle_calculate_priorities / oracle_build_choice_table, oracle_novelty)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

pytestmark = pytest.mark.gpu

C = 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpus():
    from syzkaller_amd import synth
    # a dominant call group (17k of 30k entries): plan_parts splits it at world 2 (as in test_sharding)
    return synth.corpus(0x5EED0011, 30_000, 3, 100_000, prog_len_max=C)


def _static():
    rnd = np.random.default_rng(5)
    s = (rnd.random((C, C)) * 0.9 + 0.1).astype(np.float32)
    np.fill_diagonal(s, s.max(axis=1))
    return s


def _sub(c, ids):
    lens = np.diff(c.off)[ids].astype(np.uint64)
    off = np.zeros(ids.size + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    pcs = np.concatenate([c.cover(int(i)) for i in ids]) if ids.size else np.zeros(0, np.uint32)
    return pcs, off, c.group[ids].copy(), c.prog_len[ids].copy()


def _dev(a, dev):
    import torch
    view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
    return torch.from_numpy(np.ascontiguousarray(a).view(view.get(a.dtype, a.dtype))).to(dev)


def _minimize_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from syzkaller_amd import _lib, cover, sharding, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        L = _lib.lib()
        _lib.check(L.syzgpu_init(0))
        c = _corpus()
        G = c.ngroups
        e, w = sharding.layout_stats(c.group, c.off, G)
        plan = sharding.plan_parts(e, w, world)
        ids = plan.local_entries(c.group, rank)
        local = synth.Corpus(*_sub(c, ids), G)
        key_lo, key_hi = plan.key_ranges(rank, sharding.split_bounds(plan, local, rank))
        _, _, count_hist = plan.store_parts(rank)
        split_g, split_off, split_bytes = plan.split_groups()
        held = plan.held(rank)
        xg, xo = split_g[held[split_g]], split_off[held[split_g]]
        d_pcs, d_off, d_grp, d_len = (_dev(x, dev) for x in (local.pcs, local.off, local.group, local.prog_len))
        n = local.n
        d_sel = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        d_hist = torch.zeros(C + 1, dtype=torch.int64, device=dev)
        d_out = torch.zeros(max(n, 1), dtype=torch.int64, device=dev)
        d_goff = torch.zeros(G + 1, dtype=torch.int64, device=dev)
        d_x = torch.zeros(max(split_bytes, 1), dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        job = cover.MinimizeJob()
        parts = split_g.size > 0
        # two steps: the second runs on the job's cached plan, as the bench's timed steps do
        for _ in range(2):
            job.begin(d_pcs, d_off, d_grp, n, G, d_len, key_lo if parts else None, key_hi if parts else None, s)
            if parts:
                d_x.zero_()
                if xg.size:
                    job.export_sel(xg, xo, d_x, s)
                sharding.allreduce_max_u8(d_x, dist)
                if xg.size:
                    job.import_sel(xg, xo, d_x, s)
            d_hist.zero_()
            job.end(C, count_hist if parts else None, d_sel, d_hist, d_out, d_goff, s)
            sharding.allreduce_hist(d_hist, dist)
        d_static = _dev(_static(), dev)
        d_prios = torch.empty((C, C), dtype=torch.float32, device=dev)
        d_run = torch.empty((C, C), dtype=torch.int64, device=dev)
        d_pres = torch.empty(C, dtype=torch.uint8, device=dev)
        _lib.check(L.syzgpu_prio_choice_dev(d_static.data_ptr(), d_hist.data_ptr(), C, None, d_prios.data_ptr(),
                                            d_run.data_ptr(), d_pres.data_ptr(), s))
        torch.cuda.synchronize()
        # kept entries of the groups this rank is primary for, as global ids in selection order
        goff = d_goff.cpu().numpy()
        out = d_out.cpu().numpy()
        kept = [ids[out[int(goff[g]):int(goff[g + 1])]] for g in range(G) if count_hist[g] and held[g]]
        kp = np.concatenate(kept) if kept else np.zeros(0, np.int64)
        sel_all, sel_goff = sharding.assemble_selection(kp, c.group, G, dist)
        flags = np.zeros(c.n, np.uint8)
        flags[ids] = d_sel.cpu().numpy()[:n]
        q.put((rank, int(split_g.size), sel_all, sel_goff, flags, d_hist.cpu().numpy(),
               d_prios.cpu().numpy().view(np.uint32).copy(), d_run.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def _novelty_inputs():
    import oracle
    from syzkaller_amd import synth
    S = 0xFFFFFFFF
    base = synth.corpus(0x5EED0052, 2_000, 13, 40_000)
    fresh = synth.corpus(0x5EED0053, 20_000, 13, 40_000)
    mc = []
    for g in range(13):
        gi = np.nonzero(base.group == g)[0]
        t = np.unique(np.concatenate([base.cover(int(i)) for i in gi])) if gi.size else np.zeros(0, np.uint32)
        if g % 5 == 0:
            t = np.append(t[t != S], np.uint32(S))  # a table holding the sentinel
        mc.append(t.astype(np.uint32))
    mcp, mco = oracle.to_csr(mc)
    covs = [fresh.cover(i).copy() for i in range(fresh.n)]
    for i in range(0, fresh.n, 29):
        covs[i] = np.append(covs[i][covs[i] != S], np.uint32(S)).astype(np.uint32)
    for i in range(3, fresh.n, 31):
        covs[i] = np.zeros(0, np.uint32)
    pcs, off = oracle.to_csr(covs)
    flakes = np.unique(pcs[::53][pcs[::53] != S]).astype(np.uint32)
    return pcs.astype(np.uint32), off.astype(np.uint64), fresh.group, 13, mcp, mco, flakes


def _novelty_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from syzkaller_amd import _lib, cover, sharding
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        _lib.check(_lib.lib().syzgpu_init(0))
        pcs, off, grp, G, mcp, mco, flakes = _novelty_inputs()
        ran = []

        def run(p_r, o_r, group, ngroups, m_r, mo_r, f_r):
            # the HIP entry on this rank's slice, every buffer resident on the device
            n = o_r.size - 1
            cap = int(m_r.size + p_r.size + 1)
            d_new = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
            d_tab = torch.zeros(cap, dtype=torch.int32, device=dev)
            d_toff = torch.zeros(ngroups + 1, dtype=torch.int64, device=dev)
            s = torch.cuda.current_stream(dev).cuda_stream
            cover.NoveltyBatchDev(_dev(p_r, dev), _dev(o_r, dev), _dev(np.asarray(group, np.uint32), dev), n, ngroups,
                                  _dev(m_r, dev), _dev(mo_r, dev), int(mo_r[-1]), _dev(f_r, dev), f_r.size,
                                  int(o_r[-1]), d_new, d_tab, cap, d_toff, s)
            torch.cuda.synchronize()
            toff = d_toff.cpu().numpy().view(np.uint64)
            ran.append(int(o_r[-1]))
            return (d_new.cpu().numpy()[:n], d_tab.cpu().numpy().view(np.uint32)[:int(toff[-1])].copy(), toff.copy())

        bounds = sharding.pc_bounds(pcs[::7], world)
        out = sharding.novelty_shard(pcs, off, grp, G, mcp, mco, flakes, rank, world, bounds, run, dist)
        q.put((rank, out, ran))
    finally:
        dist.destroy_process_group()


def _spawn(target, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=100) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return res


def test_minimize_corpus_two_processes_on_the_gpu():
    import oracle
    res = _spawn(_minimize_rank, 2)
    c = _corpus()
    want, wgoff = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    want_flags = np.zeros(c.n, np.uint8)
    want_flags[want] = 1
    want_hist = np.bincount(c.prog_len[want], minlength=C + 1)
    prios = oracle.calculate_priorities(_static(), c.prog_len[want])
    run, _ = oracle.build_choice_table(prios)
    flags = np.zeros(c.n, np.uint8)
    for rank, nsplit, sel, goff, f, hist, pr, rn in res:
        assert nsplit >= 1  # the plan really split a group: the selection exchange ran
        assert np.array_equal(sel, want), rank
        assert np.array_equal(goff, wgoff), rank
        assert np.array_equal(hist, want_hist), rank
        assert np.array_equal(pr, prios.view(np.uint32)), rank
        assert np.array_equal(rn, run), rank
        flags |= f
    assert np.array_equal(flags, want_flags)


def test_novelty_pc_shards_two_processes_on_the_gpu():
    import oracle
    res = _spawn(_novelty_rank, 2)
    pcs, off, grp, G, mcp, mco, flakes = _novelty_inputs()
    w_new, w_mc, w_off = oracle.novelty(pcs, off, grp, G, mcp, mco, flakes)
    assert 0 < w_new.sum() < w_new.size
    for rank, (is_new, tab, toff), ran in res:
        assert ran and 0 < ran[0] < int(off[-1])  # each rank ran the HIP entry on a strict slice
        assert np.array_equal(is_new, w_new), rank
        assert np.array_equal(toff, w_off), rank
        assert np.array_equal(tab, w_mc), rank
