"""Multi-GPU layout of minimizeCorpus (syz-manager/manager.go:507-553) — one process per GPU.

Groups too heavy for one rank are split into key parts: PC-value ranges (split_bounds), each holder
keeping the PCs of its range only (MinimizeJob.begin key_lo/key_hi).

Every call group's Minimize is independent of every other group (manager.go:523-527 runs them one by
one), so the corpus is sharded BY CALL GROUP: no data-path collective is needed for Minimize. The one
real exchange is CalculatePriorities (prio.go:29-38) over ALL kept programs: it reads only
len(p.Calls), so ranks all-reduce a (C+1)-entry int64 histogram of the kept programs'
lengths and each rank then computes the C x C priorities / ChoiceTable itself.

The fuzzer's new-coverage check (syz-fuzzer/fuzzer.go:446-470; NewInput, manager.go:609-613) shards
the other way, by PC value (SURVEY.md §8e "shard the PC-bitmap space"): a cover is new iff one of its
PCs occurs first at it (not in maxCover, not a flake), a property of each (call, PC) key alone, so
each rank runs the batch restricted to its PC range, the per-cover flags OR together (MAX all-reduce of
one byte per cover) and the updated maxCover tables are the concatenation of the ranks' ranges
(novelty_shard).

The module holds the host logic only: group assignment, shard extraction, the histogram all-reduce
and the assembly of the global group-major selection. Compute is passed in (the GPU store path in
bench.py; tests drive the same logic with a checker on CPU under gloo).
"""
import numpy as np


def group_weights(group, off, ngroups):
    """Work of each call group: its total cover length (what Minimize streams)."""
    lens = (np.asarray(off[1:], np.int64) - np.asarray(off[:-1], np.int64)).astype(np.float64)
    return np.bincount(np.asarray(group, np.int64), weights=lens, minlength=ngroups)


def lpt_assign(weights, nranks):
    """Longest-processing-time assignment of call groups to ranks, identical on every rank.

    Returns (owner[g], load[r]). Ties break by group id (stable argsort) then by lowest rank."""
    weights = np.asarray(weights, np.float64)
    owner = np.zeros(weights.size, dtype=np.int64)
    load = np.zeros(nranks, dtype=np.float64)
    for g in np.argsort(-weights, kind="stable"):
        r = int(np.argmin(load))
        owner[g] = r
        load[r] += weights[g]
    return owner, load


# ---- key-space sharding: call groups split over ranks by dense-PC windows ----------
# Cost model of one rank's step (ms = LAT + per-entry + per-PC terms), fitted on MI355X to the 8-rank
# rehearsal of the bench workload (tools/gpu_emulate.sh 8:0..8:7, profiles/r03_emu8/: residuals
# <= 0.2 ms): a fixed 0.29 ms once a rank holds a big call group (the Go sort's dependent rounds and
# the pipeline's launches), 1.24 ns per held entry (partition, sort, ranks, selection: a split group
# costs every holder all its entries) and 4.26 ps per PC streamed (transpose + first-occurrence
# tables: a split group costs each holder only its share). Small groups (<= 8192 entries) sort in LDS
# packs and stream on the side stream, overlapped; their PCs are charged a fraction.
SMALL_GROUP = 8192
LAT_REF_N, LAT_REF_US, LAT_PER_DOUBLING_US = 203_000, 290.0, 0.0
US_PER_PC = 4.26e-6  # µs per streamed PC (4.26 ps)
US_PER_ENTRY = 1.24e-3  # µs per held entry (1.24 ns)
SMALL_PC_FRACTION = 0.3


def sort_latency_us(n):
    if n <= SMALL_GROUP:
        return 0.0
    return max(0.0, LAT_REF_US + LAT_PER_DOUBLING_US * float(np.log2(n / LAT_REF_N)))


class KeyPlan:
    """ranks[g] = tuple of the ranks holding the parts of call group g (part j on ranks[g][j]; the
    first is the group's primary: it counts the group in the length histogram and reports its
    selection). Identical on every rank (a pure function of the corpus layout)."""

    def __init__(self, ranks, cost, entries):
        self.ranks, self.cost, self.entries = ranks, np.asarray(cost), np.asarray(entries, np.int64)
        self.ngroups = len(ranks)

    def owner(self):
        """Primary rank per group (-1: empty group)."""
        return np.array([r[0] if r else -1 for r in self.ranks], np.int64)

    def held(self, rank):
        return np.array([rank in r for r in self.ranks], bool)

    def local_entries(self, group, rank):
        """Global corpus entry ids (ascending) of every group this rank holds a part of."""
        return np.nonzero(self.held(rank)[np.asarray(group, np.int64)])[0]

    def store_parts(self, rank):
        """(part u16[G], nparts u16[G], count_hist u8[G]) for CoverStore.set_parts on this rank."""
        part = np.zeros(self.ngroups, np.uint16)
        nparts = np.ones(self.ngroups, np.uint16)
        count = np.zeros(self.ngroups, np.uint8)
        for g, r in enumerate(self.ranks):
            if rank in r:
                nparts[g] = len(r)
                part[g] = r.index(rank)
                count[g] = 1 if r[0] == rank else 0
        return part, nparts, count

    def key_ranges(self, rank, bounds):
        """(key_lo u32[G], key_hi u32[G]) of this rank for MinimizeJob.begin: [0, 2^32-1] for groups held
        whole (or not held), part j of a split group g = [bounds[g][j], bounds[g][j+1] - 1]."""
        lo = np.zeros(self.ngroups, np.uint32)
        hi = np.full(self.ngroups, 0xFFFFFFFF, np.uint32)
        for g, r in enumerate(self.ranks):
            if len(r) > 1 and rank in r:
                j = r.index(rank)
                b = bounds[g]
                lo[g] = np.uint32(b[j])
                hi[g] = np.uint32(b[j + 1] - 1)
        return lo, hi

    def split_groups(self):
        """(groups, byte offsets, total bytes) of the selection exchange: every split group, one byte
        per entry, in group order — the same buffer layout on every rank."""
        gs = np.array([g for g, r in enumerate(self.ranks) if len(r) > 1], np.uint32)
        off = np.zeros(gs.size + 1, np.uint64)
        if gs.size:
            np.cumsum(self.entries[gs], out=off[1:])
        return gs, off[:-1], int(off[-1])


def _assign(entries, pcs, k, nranks):
    lat = np.array([sort_latency_us(int(n)) for n in entries])
    big = entries > SMALL_GROUP
    w = US_PER_PC * pcs * np.where(big, 1.0, SMALL_PC_FRACTION) / np.maximum(k, 1) + US_PER_ENTRY * entries
    items = [(lat[g] + w[g], g, j) for g in range(entries.size) if entries[g] > 0 for j in range(k[g])]
    items.sort(key=lambda t: (-t[0], t[1], t[2]))
    cur_lat, cur_w = np.zeros(nranks), np.zeros(nranks)
    ranks = [[] for _ in range(entries.size)]
    for _, g, j in items:
        best, best_cost = -1, None
        for r in range(nranks):
            if r in ranks[g]:
                continue
            c = max(cur_lat[r], lat[g]) + cur_w[r] + w[g]
            if best_cost is None or c < best_cost - 1e-9:
                best, best_cost = r, c
        ranks[g].append(best)
        cur_lat[best] = max(cur_lat[best], lat[g])
        cur_w[best] += w[g]
    return [tuple(r) for r in ranks], cur_lat + cur_w


def plan_parts(entries, pcs, nranks, max_rounds=24):
    """Key-space sharding plan: start with whole groups, then keep doubling the part count of the
    heaviest group on the bottleneck rank while the modelled step (max over ranks) improves."""
    entries = np.asarray(entries, np.int64)
    pcs = np.asarray(pcs, np.float64)
    k = np.ones(entries.size, np.int64)
    ranks, cost = _assign(entries, pcs, k, nranks)
    for _ in range(max_rounds):
        r = int(np.argmax(cost))
        cand = [g for g in range(entries.size) if r in ranks[g] and k[g] < nranks and entries[g] > SMALL_GROUP]
        if not cand:
            break
        g = max(cand, key=lambda x: (sort_latency_us(int(entries[x])) + US_PER_PC * pcs[x] / k[x], -x))
        k2 = k.copy()
        k2[g] = min(nranks, k[g] * 2)
        ranks2, cost2 = _assign(entries, pcs, k2, nranks)
        if cost2.max() >= cost.max() - 1e-6:
            break
        k, ranks, cost = k2, ranks2, cost2
    return KeyPlan(ranks, cost, entries)


def split_bounds(plan, corp, rank, sample_every=16):
    """PC-value boundaries of every split group this rank holds: bounds[g] = k+1 ascending values in
    [0, 2^32] (b[0] = 0, b[k] = 2^32) at equal-count quantiles of the group's PCs, so the parts hold
    about the same number of PCs. A pure function of the group's covers, which every holder has
    whole, so all holders compute the same boundaries. corp: the rank's local corpus (global group ids)."""
    bounds = {}
    grp = np.asarray(corp.group, np.int64)
    off = np.asarray(corp.off, np.int64)
    for g, r in enumerate(plan.ranks):
        if len(r) <= 1 or rank not in r:
            continue
        k = len(r)
        ent = np.nonzero(grp == g)[0][::sample_every]
        if ent.size:
            sample = np.concatenate([corp.pcs[off[e]:off[e + 1]] for e in ent]).astype(np.uint64)
        else:
            sample = np.zeros(0, np.uint64)
        b = [0]
        if sample.size:
            sample.sort()
            for j in range(1, k):
                b.append(max(b[-1] + 1, int(sample[min(sample.size - 1, (sample.size * j) // k)])))
        else:
            b += [(1 << 32) * j // k for j in range(1, k)]
        b.append(1 << 32)
        bounds[g] = np.array(b, np.uint64)
    return bounds


def layout_stats(group, off, ngroups):
    """(entries per group, PCs per group) of a CSR corpus layout."""
    g = np.asarray(group, np.int64)
    return np.bincount(g, minlength=ngroups), group_weights(group, off, ngroups)


def local_entries(group, owner, rank):
    """Global corpus entry ids (ascending, i.e. corpus order) whose call group this rank owns."""
    return np.nonzero(owner[np.asarray(group, np.int64)] == rank)[0]


def allreduce(t, dist=None, op=None):
    """In-place all-reduce of a torch tensor on any backend: RCCL takes device tensors directly, gloo
    (CPU rehearsals of the N>1 path) goes through a host copy."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return t
    op = dist.ReduceOp.SUM if op is None else op
    if t.is_cuda and dist.get_backend() == "gloo":
        tmp = t.cpu()
        dist.all_reduce(tmp, op=op)
        t.copy_(tmp)
    else:
        dist.all_reduce(t, op=op)
    return t


def allreduce_hist(hist, dist=None):
    """Sum the kept-program length histograms of all ranks in place (torch tensor, any backend)."""
    return allreduce(hist, dist)


def allreduce_max_u8(buf, dist=None):
    """The selection exchange of split groups: bytes OR-ed across ranks (MAX over 0/1 bytes)."""
    return allreduce(buf, dist, None if dist is None else dist.ReduceOp.MAX)


def assemble_selection(kept_global, group, ngroups, dist=None):
    """Group-major kept entry ids over all ranks, groups ascending (the order syzgpu_minimize_grouped
    returns; the reference concatenates groups in Go map order). Each rank passes its
    kept GLOBAL ids group-major, each group from exactly one rank (its primary); returns
    (ids, group_off) on every rank."""
    kept_global = np.asarray(kept_global, np.int64)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, kept_global)
        kept_global = np.concatenate([np.asarray(p, np.int64) for p in parts])
    g = np.asarray(group, np.int64)[kept_global]
    # a group lives on exactly one rank, so a stable sort by group keeps each group's selection order
    order = np.argsort(g, kind="stable")
    ids = kept_global[order]
    goff = np.zeros(ngroups + 1, np.uint64)
    np.cumsum(np.bincount(g, minlength=ngroups), out=goff[1:])
    return ids, goff


# ---- PC-space sharding of the new-coverage check -----------------------------------
SENTINEL = 0xFFFFFFFF


def pc_bounds(sample, nparts):
    """nparts + 1 ascending PC bounds [0, ..., 2^32] at equal-count quantiles of a PC sample (rank r
    owns PCs in [b[r], b[r+1] - 1]); a pure function of the sample, identical on every rank."""
    sample = np.sort(np.asarray(sample, np.uint64))
    b = [0]
    for j in range(1, nparts):
        q = int(sample[min(sample.size - 1, sample.size * j // nparts)]) if sample.size else (1 << 32) * j // nparts
        b.append(max(b[-1] + 1, q))
    b.append(1 << 32)
    return np.array(b, np.uint64)


def slice_csr(pcs, off, lo, hi):
    """Each (sorted) cover of a CSR batch restricted to PCs in [lo, hi]: (pcs', off')."""
    pcs = np.asarray(pcs, np.uint32)
    off = np.asarray(off, np.uint64)
    n = off.size - 1
    lens = np.diff(off).astype(np.int64)
    # covers are sorted, so (cover index, pc) is sorted over the whole batch
    key = (np.repeat(np.arange(n, dtype=np.uint64), lens) << np.uint64(32)) | pcs.astype(np.uint64)
    idx = np.arange(n, dtype=np.uint64) << np.uint64(32)
    a = np.searchsorted(key, idx | np.uint64(lo), side="left")
    b = np.searchsorted(key, idx | np.uint64(hi), side="right")
    keep = np.zeros(key.size + 1, np.int64)
    np.add.at(keep, a, 1)
    np.add.at(keep, b, -1)
    mask = np.cumsum(keep[:-1]) > 0
    off2 = np.zeros(n + 1, np.uint64)
    np.cumsum(b - a, out=off2[1:])
    return pcs[mask], off2


def novelty_slice(pcs, off, mc, mc_off, flakes, lo, hi):
    """A rank's inputs of a PC-range shard of the new-coverage check: the batch, the maxCover tables and
    the flakes restricted to PCs in [lo, hi]."""
    p_r, o_r = slice_csr(pcs, off, lo, hi)
    m_r, mo_r = slice_csr(mc, mc_off, lo, hi)
    flakes = np.asarray(flakes, np.uint32)
    return p_r, o_r, m_r, mo_r, flakes[(flakes >= lo) & (flakes <= hi)]


def novelty_flags(is_new_r, group, ngroups):
    """A rank's exchange bytes: its per-cover flags and per-call "updated" flags, u8[n + G] (the MAX
    all-reduce of these over ranks is the whole exchange of the flags)."""
    group = np.asarray(group, np.int64)
    updated = np.zeros(ngroups, np.uint8)
    if np.asarray(is_new_r).size:
        np.maximum.at(updated, group[np.asarray(is_new_r, bool)], 1)
    return np.concatenate([np.asarray(is_new_r, np.uint8), updated])


def novelty_merge(flags, parts, n, ngroups):
    """The batch's result from the MAX-reduced flags (u8[n + G]) and every rank's table part
    [(tables, offsets)] in rank (= PC range) order: each call's table is the concatenation of its
    parts, without the 0xFFFFFFFF sentinel when any rank updated it (Union drops it over the whole
    table, cover.go:63-70). Returns (is_new, tables, offsets)."""
    flags = np.asarray(flags, np.uint8)
    is_new, updated = flags[:n], flags[n:n + ngroups]
    tabs, lens = [], np.zeros(ngroups, np.int64)
    for g in range(ngroups):
        t = np.concatenate([np.asarray(p[0][int(p[1][g]):int(p[1][g + 1])], np.uint32) for p in parts])
        if updated[g]:
            t = t[t != SENTINEL]
        tabs.append(t)
        lens[g] = t.size
    toff = np.zeros(ngroups + 1, np.uint64)
    np.cumsum(lens, out=toff[1:])
    return is_new, (np.concatenate(tabs) if tabs else np.zeros(0, np.uint32)), toff


def novelty_shard(pcs, off, group, ngroups, mc, mc_off, flakes, rank, world, bounds, run, dist=None):
    """One rank's share of a new-coverage batch (fuzzer.go:446-470 per cover, in order) sharded by PC
    value: the batch, the maxCover tables and the flakes restricted to [bounds[rank], bounds[rank+1]-1]
    (novelty_slice), run(...) -> (is_new u8[n], table pcs, table offsets) on that slice (the GPU, or a
    checker), then the MAX all-reduce of the flags (novelty_flags: n + G bytes) and the ranks' table
    parts concatenated per call in PC order (novelty_merge). Returns (is_new, tables, offsets),
    identical on every rank."""
    import torch
    lo, hi = int(bounds[rank]), int(bounds[rank + 1]) - 1
    p_r, o_r, m_r, mo_r, f_r = novelty_slice(pcs, off, mc, mc_off, flakes, lo, hi)
    is_new_r, tab_r, toff_r = run(p_r, o_r, group, ngroups, m_r, mo_r, f_r)
    flags = torch.from_numpy(novelty_flags(is_new_r, group, ngroups))
    allreduce_max_u8(flags, dist)
    parts = [(tab_r, toff_r)]
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        parts = [None] * world
        dist.all_gather_object(parts, (np.asarray(tab_r, np.uint32), np.asarray(toff_r, np.uint64)))
    return novelty_merge(flags.numpy(), parts, np.asarray(is_new_r).size, ngroups)


# ---- the call co-occurrence XᵀX, sharded by corpus rows (north_star) --------------
def cooccurrence_rows(nprogs, world):
    """Row shards of the co-occurrence: rank r takes programs [b[r], b[r+1]) (equal counts, in corpus
    order). XᵀX is a sum over programs, so the shards' partial matrices add up to the whole."""
    return np.linspace(0, nprogs, world + 1).round().astype(np.int64)


def cooccurrence_slice(calls, off, lo, hi):
    """Programs [lo, hi) of the CSR (calls, off) as their own CSR."""
    off = np.asarray(off, np.uint64)
    a, b = int(off[lo]), int(off[hi])
    return np.asarray(calls)[a:b], (off[lo:hi + 1] - off[lo]).astype(np.uint64)


def cooccurrence_shard(calls, off, C, rank, world, run, dist=None):
    """One rank's share of the call co-occurrence: run(calls, off, C) -> int32 C x C on this rank's row
    shard (the GPU entry, or a checker), then one SUM all-reduce of the C x C partials. The sum is
    taken in int64 and must fit int32 like the single-device result (the entry's ERANGE): an overflow
    raises OverflowError. Returns the int32 C x C matrix, identical on every rank."""
    import torch
    b = cooccurrence_rows(np.asarray(off).size - 1, world)
    part = np.asarray(run(*cooccurrence_slice(calls, off, int(b[rank]), int(b[rank + 1])), C), np.int32)
    t = torch.from_numpy(part.astype(np.int64))
    allreduce(t, dist)
    tot = t.numpy()
    if tot.size and (tot.max() > np.iinfo(np.int32).max or tot.min() < np.iinfo(np.int32).min):
        raise OverflowError("call co-occurrence count outside int32")
    return tot.astype(np.int32)
