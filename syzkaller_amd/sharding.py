"""Multi-GPU layout of minimizeCorpus (syz-manager/manager.go:507-553) — one process per GPU.

Every call group's Minimize is independent of every other group (manager.go:523-527 runs them one by
one), so the corpus is sharded BY CALL GROUP: no data-path collective is needed for Minimize. The one
real exchange is CalculatePriorities (prio.go:29-38) over ALL kept programs: it reads only
len(p.Calls), so ranks all-reduce a (C+1)-entry int64 histogram of the kept programs'
lengths and each rank then computes the C x C priorities / ChoiceTable itself.

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


def assemble_selection(kept_global, group, ngroups, dist=None):
    """Group-major kept entry ids over all ranks, groups ascending (the order syzgpu_minimize_grouped
    returns; the reference concatenates groups in Go map order). Each rank passes its
    kept GLOBAL ids group-major; returns (ids, group_off) on every rank."""
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
