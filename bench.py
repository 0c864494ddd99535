#!/usr/bin/env python3
"""Benchmark: corpus progs/sec of syz-manager's minimizeCorpus hot path on MI355X.

One step = cover.Minimize over every call group of a device-resident corpus
(syz-manager/manager.go:507-527 -> cover/cover.go:105-131) + CalculatePriorities over the kept
programs (prog/prio.go:29-38: calcStaticPriorities :40-135 on the int8 matrix cores from the usage
matrix of sys/*.txt, calcDynamicPrio :137-192, their product) + BuildChoiceTable (prio.go:202-228),
through the C ABI of libsyzgpu.so. Inputs (covers, call ids, program lengths, the usage matrix) are
resident in HBM before the timed region; the output selection, priorities and ChoiceTable stay in HBM.

Workload (BASELINE.json configs[3], per GPU): 1M programs, 2M-PC space, 289 calls, C = 1159,
synthetic corpus from the seeded generator (SURVEY.md §8d shapes). Weak scaling: at N GPUs the
corpus has N x 1M programs; call groups go to ranks whole or, when one is heavier than a rank's share,
split by dense-PC windows over several ranks (syzkaller_amd/sharding.py plan_parts). The exchanges are
an RCCL MAX all-reduce of the split groups' selection bytes and an RCCL all-reduce of the (C+1)-entry
program-length histogram that feeds CalculatePriorities.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--progs-per-gpu 1000000]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "corpus progs/sec: cover.Minimize + calcDynamicPrio, 1M progs, 1/2/4/8 GPUs"

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s spec, 6.29 measured copy)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--progs-per-gpu", type=int, default=1_000_000)
    ap.add_argument("--ngroups", type=int, default=289)
    ap.add_argument("--npcs", type=int, default=2_000_000)
    ap.add_argument("--calls", type=int, default=1159)
    ap.add_argument("--seed", type=int, default=0x5EED0004)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 at N=1")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="programs in the CPU baseline sample")
    ap.add_argument("--profile", type=int, default=1, help="per-kernel HIP event timing in the timed region")
    ap.add_argument("--store", type=int, default=1, help="also time the resident-store side leg at N=1")
    ap.add_argument("--text", type=int, default=1, help="also time the text pass over the kept programs at N=1")
    ap.add_argument("--novelty", type=int, default=1, help="also time config 3 (triage batch): at N=1 whole, at N>1 sharded by PC range")
    ap.add_argument("--novelty-covers", type=int, default=1_000_000)
    ap.add_argument("--novelty-wide", type=int, default=1,
                    help="also time the novelty batch with its PC span stretched 34x (272M addresses)")
    ap.add_argument("--canonicalize", type=int, default=1,
                    help="also time cover.Canonicalize over 1M raw execution covers (device entry) at N=1")
    ap.add_argument("--setops", type=int, default=1,
                    help="also time the batched set ops on config-3 covers (triage pairs) at N=1")
    ap.add_argument("--hub", type=int, default=1, help="also time config 5's hub ingest (scan + SHA-1 + dedup) at N=1")
    ap.add_argument("--analytics", type=int, default=1, help="also time the manager's cover analytics at N=1")
    ap.add_argument("--analytics-cpu-sample", type=int, default=10_000)
    ap.add_argument("--append", type=int, default=10_000,
                    help="also time a NewInput append of this many programs to the store at N=1 (0: off)")
    ap.add_argument("--novelty-cpu-sample", type=int, default=20_000)
    ap.add_argument("--layout-change", type=int, default=1000,
                    help="also time minimizeCorpus when every step's corpus has this many more programs than the "
                         "step before (the manager's NewInputs between minimizes: a new group layout every call; "
                         "0: off)")
    ap.add_argument("--cooccurrence", type=int, default=1,
                    help="also time the call-ID co-occurrence X^T X on int8 MFMA (SURVEY.md F1/K9) at N=1")
    ap.add_argument("--split-largest", type=int, default=0,
                    help="rehearsal: force the largest call group into this many PC-key parts")
    ap.add_argument("--total-progs", type=int, default=0,
                    help="strong scaling: this many programs in the whole job, sharded over the N GPUs (configs[3]: "
                         "1M over 8); default 0 = weak scaling, --progs-per-gpu on every GPU (N x 1M: configs[4]'s "
                         "hub-merge shape at N = 8)")
    ap.add_argument("--emulate", default="", help="W:r — rehearsal: run rank r's shard of a W-rank job on this "
                    "one process (no collectives; the printed line is that rank's time, not a job value)")
    return ap.parse_args()


# the round's committed rocprofv3 kernel summary of this bench command (tools/gpu_final6.sh): its top
# byte-modelled kernel by total GPU time names the roofline kernel
ROCPROF_STATS = os.path.join(ROOT, "profiles", "r06_kernel_stats.csv")
# rocprofv3 kernel name -> the library's profiling scope around that kernel; the same
# names key profiles/pmc_traffic.json (tools/pmc_traffic.py)
ROCPROF_SCOPE = [("k_slab<", "k_slab"), ("k_smin_direct", "k_pmin_direct"), ("k_smin_hash<false>", "k_pmin_hash"),
                 ("k_smin_hash<true>", "k_pmin_packed")]


# the workload the committed rocprofv3 summary and PMC passes were taken on: the default bench line
PROFILED_WORKLOAD = "config4-1M"


def workload_key(args, world):
    """Short key of the workload a line measures, to match committed profiles against: the default line
    (config 4, 1M programs, 2M PCs, one GPU) is "config4-1M"."""
    if world == 1 and not args.total_progs and not args.emulate and args.progs_per_gpu == 1_000_000 \
            and args.npcs == 2_000_000 and args.ngroups == 289 and args.calls == 1159 and args.seed == 0x5EED0004:
        return PROFILED_WORKLOAD
    return "progs%d-pcs%d-groups%d-world%d%s" % (args.progs_per_gpu, args.npcs, args.ngroups, world,
                                                "-total%d" % args.total_progs if args.total_progs else "")


def rocprof_top(path=ROCPROF_STATS, workload=PROFILED_WORKLOAD):
    """(scope, kernel name) of the first row of the committed rocprofv3 --stats summary (rows are
    sorted by total duration) that is a byte-modelled kernel (ROCPROF_SCOPE), or None; None too when the
    line's workload is not the one profiled. Rows above it are latency-bound kernels without a byte model
    (round 6: the Go sort's LDS sorter, whose launches last long beside the transpose)."""
    import csv
    if workload != PROFILED_WORKLOAD:
        return None
    try:
        rows = list(csv.DictReader(open(path)))
    except OSError:
        return None
    if not rows:
        return None
    for row in rows:
        top = row["Name"]
        for pat, scope in ROCPROF_SCOPE:
            if pat in top:
                return scope, top
    return None


def dominant_kernel(kern, workload=PROFILED_WORKLOAD):
    """The step's dominant kernel: the top kernel of the committed rocprofv3 summary of this command
    (ROCPROF_STATS) when it maps to a byte-modelled scope; else the kernel scope with the most time in
    the untimed per-kernel pass among those carrying an algorithmic byte model (SURVEY.md
    §8d: a kernel's share of the algorithm's input, never the intermediate buffers it writes): k_slab
    (the transpose) 4 B per PC + 10 B per entry, k_pmin_direct / k_pmin_hash / k_pmin_packed 4 B per PC
    of the groups they walk. That pass runs the
    raw pipeline's passes one after another (syzgpu_profile_enable(2)), so each scope times its kernels
    alone. Phase scopes (gosort_*, m_big, group_partition) span several kernels and are not candidates."""
    top = rocprof_top(workload=workload)
    if top and top[0] in kern and kern[top[0]]["bytes"] > 0:
        return top[0]
    rows = [(d["ms"], name) for name, d in kern.items() if name.startswith("k_") and d["bytes"] > 0]
    return max(rows)[1] if rows else None


def roofline(name, ev, peak_gbs=None, workload=PROFILED_WORKLOAD):
    """Roofline of one kernel from its HIP events in the timed region (on its launch stream): achieved =
    its recorded algorithmic bytes / its time; traffic = HBM bytes per launch from the committed PMC
    passes (profiles/pmc_traffic.json, FETCH_SIZE doubled + WRITE_SIZE) when they name this kernel and
    were taken on this line's workload (null otherwise)."""
    d = ev.get(name)
    if not d or not d["ms"]:
        return None
    avg_ms = d["ms"] / d["launches"]
    alg = d["bytes"] / d["launches"]
    ach = alg / (avg_ms * 1e-3) / 1e9
    peak = peak_gbs or HBM_PEAK_GBS
    out = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1), "peak": peak, "unit": "GB/s",
           "frac": round(ach / peak, 4), "traffic": None, "avg_launch_ms": round(avg_ms, 4),
           "launches_per_step": None, "algorithmic_bytes_per_launch": int(alg)}
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            pm = json.load(open(tf))
            if name in pm.get("kernels", {}) and pm.get("workload") == workload:
                out["traffic"] = pm["kernels"][name]["hbm_bytes_per_launch"]
        except Exception:
            pass
    return out


def workload_label(args, world):
    """The BASELINE.json config the line measures: configs[3] (1M programs; strong scaling over N GPUs
    with --total-progs) or, weak scaling at N > 1, configs[4]'s hub-merge shape (N managers' corpora of
    --progs-per-gpu programs each)."""
    tail = "%s-PC space, %d calls, C=%d" % (("%gM" % (args.npcs / 1e6)) if args.npcs >= 1_000_000 else
                                           ("%gk" % (args.npcs / 1e3)), args.ngroups, args.calls)
    if args.total_progs:
        return "config4-%dk over %d GPU%s (strong scaling): %s" % (args.total_progs // 1000, world,
                                                                  "s" if world > 1 else "", tail)
    if world == 1:
        # BASELINE.json configs[0] / [1] / [3] by their (programs, PC space); other shapes by their numbers
        name = {(10_000, 50_000): "config1-10k", (100_000, 500_000): "config2-100k",
                (1_000_000, 2_000_000): "config4-1M",
                (8_000_000, 2_000_000): "config5-8M (hub merge of 8 managers' corpora, on 1 GPU)"}.get(
                    (args.progs_per_gpu, args.npcs), "custom")
        return "%s: %d programs on 1 GPU, %s" % (name, args.progs_per_gpu, tail)
    return ("config5-shape: %d managers' corpora of %d programs (%d programs, weak scaling: %d per GPU), %s"
            % (world, args.progs_per_gpu, args.progs_per_gpu * world, args.progs_per_gpu, tail))


def static_usage(C):
    """calcStaticPriorities' input: the usage matrix of the reference's sys/*.txt (1159 calls, bundled
    as package data by tools/gen_sys_usage.py); other call counts take a seeded matrix of the same
    density and weights."""
    from syzkaller_amd import sysdesc
    u = sysdesc.bundled()
    if u.C == C:
        return u.weights
    rnd = np.random.default_rng(7)
    w = np.zeros((u.weights.shape[0], C), np.float32)
    mask = rnd.random(w.shape) < np.count_nonzero(u.weights) / u.weights.size
    w[mask] = rnd.choice(np.array([0.1, 0.2, 0.5, 1.0], np.float32), size=int(mask.sum()))
    return w


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    emu_world, emu_rank = (int(x) for x in args.emulate.split(":")) if args.emulate else (world, rank)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("run N>1 through torch.distributed.run (one process per GPU)", file=sys.stderr)
            sys.exit(2)
    import torch
    import torch.distributed as dist

    from syzkaller_amd import _lib, cover, sharding, synth

    # SYZ_BENCH_BACKEND=gloo + SYZ_BENCH_SAME_DEVICE=1 rehearse the N>1 path with every rank on GPU 0
    # (the real run is one rank per GPU over RCCL, backend "nccl")
    backend = os.environ.get("SYZ_BENCH_BACKEND", "nccl")
    dev_index = 0 if os.environ.get("SYZ_BENCH_SAME_DEVICE") == "1" else local
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    L = _lib.lib()
    _lib.check(L.syzgpu_init(dev_index))

    # ---- corpus (synthetic, deterministic; generated on the host, then made resident) ----
    t0 = time.time()
    C, G = args.calls, args.ngroups
    job_progs = args.total_progs or args.progs_per_gpu * emu_world  # programs of the whole job
    p = synth.params(args.seed, job_progs, G, args.npcs)
    group, off, plen = synth.layout(p)
    # key-space sharding plan: call groups whole or split by PC-value ranges over ranks
    ent_g, pcs_g = sharding.layout_stats(group, off, G)
    plan = sharding.plan_parts(ent_g, pcs_g, emu_world)
    if args.split_largest > 1:
        k = np.ones(G, np.int64)
        k[int(np.argmax(ent_g))] = min(args.split_largest, emu_world)
        plan = sharding.KeyPlan(*sharding._assign(ent_g, pcs_g, k, emu_world), ent_g)
    ids = plan.local_entries(group, emu_rank)
    corp = synth.subcorpus(p, ids, group, off, plen)
    gen_s = time.time() - t0

    def dt(a):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
        return torch.from_numpy(a.view(view.get(a.dtype, a.dtype))).to(dev)

    d_pcs, d_off, d_grp, d_len = dt(corp.pcs), dt(corp.off), dt(corp.group), dt(corp.prog_len)
    uses = static_usage(C)
    d_uses = torch.from_numpy(uses).to(dev)
    d_static = torch.empty((C, C), dtype=torch.float32, device=dev)
    d_sel = torch.zeros(corp.n, dtype=torch.uint8, device=dev)
    d_hist = torch.zeros(C + 1, dtype=torch.int64, device=dev)
    d_out = torch.zeros(max(corp.n, 1), dtype=torch.int64, device=dev)
    d_goff = torch.zeros(G + 1, dtype=torch.int64, device=dev)
    d_prios = torch.empty((C, C), dtype=torch.float32, device=dev)
    d_run = torch.empty((C, C), dtype=torch.int64, device=dev)
    d_pres = torch.empty(C, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    # key parts of split groups (PC ranges, identical on every rank) and the selection exchange
    key_lo, key_hi = plan.key_ranges(emu_rank, sharding.split_bounds(plan, corp, emu_rank))
    _, _, count_hist = plan.store_parts(emu_rank)
    split_g, split_off, split_bytes = plan.split_groups()
    held = plan.held(emu_rank)
    xg, xo = split_g[held[split_g]], split_off[held[split_g]]
    d_x = torch.zeros(max(split_bytes, 1), dtype=torch.uint8, device=dev)
    job = cover.MinimizeJob()
    parts = split_g.size > 0

    def step():
        # minimizeCorpus from the raw covers in HBM: group partition, Go-sort ranks, window transpose,
        # first-occurrence tables, kept flags + length histogram + the group-major kept list
        job.begin(d_pcs, d_off, d_grp, corp.n, G, d_len, key_lo if parts else None, key_hi if parts else None, sptr)
        if parts:  # split groups: OR the partial selections across their ranks
            d_x.zero_()
            if xg.size:
                job.export_sel(xg, xo, d_x, sptr)
            sharding.allreduce_max_u8(d_x, dist)
            if xg.size:
                job.import_sel(xg, xo, d_x, sptr)
        if world == 1:
            # minimizeCorpus's tail in one call (manager.go:523-536): kept flags / list / length
            # histogram, calcStaticPriorities (int8 MFMA) beside them, CalculatePriorities +
            # BuildChoiceTable; one wait for the error checks
            job.end_prio(C, d_uses, uses.shape[0], d_static, d_prios, d_run, count_hist if parts else None,
                         d_sel, d_hist, d_out, d_goff, d_pres, sptr)
            return
        job.end(C, count_hist if parts else None, d_sel, d_hist, d_out, d_goff, sptr)
        sharding.allreduce_hist(d_hist, dist)  # kept-length histogram: (C+1) int64
        # CalculatePriorities (prio.go:29-38): calcStaticPriorities (int8 MFMA) x normalized dynamic
        _lib.check(L.syzgpu_static_priorities_dev(d_uses.data_ptr(), uses.shape[0], C, d_static.data_ptr(), sptr))
        _lib.check(L.syzgpu_prio_choice_dev(d_static.data_ptr(), d_hist.data_ptr(), C, None, d_prios.data_ptr(),
                                            d_run.data_ptr(), d_pres.data_ptr(), sptr))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    def read_prof():
        cap = 4096
        names = ctypes.create_string_buffer(48 * cap)
        ms = np.zeros(cap, np.float32)
        by = np.zeros(cap, np.uint64)
        k = L.syzgpu_profile_read(names, ms.ctypes.data, by.ctypes.data, cap)
        out, raw = {}, names.raw
        for i in range(k):
            nm = raw[48 * i:48 * (i + 1)].split(b"\0")[0].decode()
            e = out.setdefault(nm, {"ms": 0.0, "launches": 0, "bytes": 0})
            e["ms"] += float(ms[i])
            e["launches"] += 1
            e["bytes"] += int(by[i])
        return out

    # per-kernel breakdown first (untimed: events around every kernel), which names the dominant kernel
    kern = {}
    if args.profile:
        L.syzgpu_profile_only(None)
        L.syzgpu_profile_enable(2)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        kern = read_prof()
        L.syzgpu_profile_enable(0)
    wkey = workload_key(args, world)
    roof_kernel = dominant_kernel(kern, wkey) if kern else None
    # timed region: HIP events (on the launch stream) around the dominant kernel only
    if roof_kernel:
        L.syzgpu_profile_only(roof_kernel.encode())
        L.syzgpu_profile_enable(1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    roof_ev = read_prof() if roof_kernel else {}
    L.syzgpu_profile_enable(0)
    job_info = job.info()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        sharding.allreduce(t, dist, dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_progs = args.total_progs or args.progs_per_gpu * world
    sum_pcs_all = int(off[-1])  # the whole job's corpus (a split group is held by several ranks)
    ms_step = elapsed / args.steps * 1e3
    value = total_progs * args.steps / elapsed

    # configs[2] on N GPUs: every rank takes its PC range of the batch (collectives inside)
    nov_sh = None
    if world > 1 and args.novelty and not args.emulate:
        try:  # a side leg: a failure that every rank sees is reported in the line, not fatal to it
            nov_sh = novelty_leg_sharded(args, dev, L, dist, rank, world)
        except Exception as e:  # noqa: BLE001
            nov_sh = {"error": "%s: %s" % (type(e).__name__, e)}

    # the same step on a layout that changes every call (rank 0 at N = 1 only; never `value`)
    lchg = None
    if world == 1 and not args.emulate and args.layout_change:
        lchg = layout_change_leg(args, dev, corp, d_pcs, d_off, d_grp, d_len, G, C, uses, d_uses, d_static,
                                 d_prios, d_run, d_sel, d_hist, d_out, d_goff, d_pres, sptr, ms_step)

    out = None
    if rank == 0:
        # roofline of the dominant kernel: algorithmic bytes over its measured time
        roof = roofline(roof_kernel, roof_ev, workload=wkey) if roof_kernel else None
        if roof:
            roof["launches_per_step"] = round(roof_ev[roof_kernel]["launches"] / args.steps, 2)
            # the rocprofv3 kernel the library's profiling scope times (ROCPROF_SCOPE)
            roof["rocprof_kernel"] = next((pat.rstrip("<") for pat, sc in ROCPROF_SCOPE if sc == roof_kernel), None)
            roof["dominant_kernel_overall"] = max(kern.items(), key=lambda kv: kv[1]["ms"])[0]
            roof["profiled_workload"] = wkey if wkey == PROFILED_WORKLOAD else None
            top = rocprof_top(workload=wkey)
            roof["selection"] = (("the top byte-modelled kernel of the committed rocprofv3 summary %s (%s)"
                                  % (os.path.relpath(ROCPROF_STATS, ROOT), top[1][:60])) if top and top[0] == roof_kernel
                                 else "the byte-modelled kernel with the most time in the serialized per-kernel pass")
            roof["selection"] += "; achieved from its HIP events in the (concurrent) timed region"
        path_bytes = 4 * int(off[-1]) + 10 * total_progs + 16 * C * C  # SURVEY.md §8(d), whole job
        cpu = None
        if args.cpu_baseline and world == 1:
            cpu = cpu_baseline(corp, uses, min(args.cpu_sample, corp.n))
        solo = world == 1 and not args.emulate
        store_leg_res, store = (None, None)
        if solo and (args.store or args.analytics or args.append):
            store_leg_res, store = store_leg(args, L, corp, d_pcs, d_off, d_grp, d_len, d_sel, d_hist, C, G, sptr)
        tail = text_leg(args, dev, L, read_prof, corp, d_sel, sptr, ms_step) if args.text and solo else None
        nov = novelty_leg(args, dev, L, read_prof) if args.novelty and solo else None
        cooc = cooccurrence_leg(args, dev, L, read_prof, corp, C) if args.cooccurrence and solo else None
        sops = setops_leg(args, dev, L, read_prof) if args.setops and solo else None
        canon = canonicalize_leg(args, dev, L, read_prof) if args.canonicalize and solo else None
        hubr = hub_leg(args, dev, L, read_prof, corp, sptr) if args.hub and solo else None
        ana = analytics_leg(args, dev, L, read_prof, store, corp, sptr) if args.analytics and solo else None
        app = append_leg(args, dev, store, sptr, C, d_hist) if args.append and solo else None  # last: replaces
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "progs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "strong" if args.total_progs else "weak", "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: seeded generator (SURVEY.md §8d shapes); raw covers resident in HBM, every step "
                    "from the covers (no store or dictionary built ahead)",
            "config": {"workload": workload_label(args, world),
                       "progs_per_gpu": args.progs_per_gpu, "total_progs": total_progs,
                       "sum_pcs": sum_pcs_all, "ngroups": G, "npcs": args.npcs, "calls": C,
                       "step": "minimizeCorpus from raw covers (partition + Go-sort ranks + window transpose + "
                               "first-occurrence tables + kept flags/list) + CalculatePriorities + BuildChoiceTable",
                       "parallelism": "call groups sharded x%d, %d split by PC-key ranges (RCCL MAX all-reduce "
                                      "of %d selection bytes) + RCCL all-reduce of the length histogram"
                                      % (world, int(split_g.size), split_bytes),
                       "modelled_rank_us": [round(float(x), 1) for x in plan.cost],
                       "split_groups": {int(g): list(plan.ranks[g]) for g in split_g}},
            "roofline": roof,
            "path_roofline": {"bytes_per_step": path_bytes,
                              "achieved": round(path_bytes / (ms_step * 1e-3) / 1e9, 1),
                              "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                              "frac": round(path_bytes / (ms_step * 1e-3) / 1e9 / (HBM_PEAK_GBS * world), 4)},
            "kernels_ms_per_step_serialized_pass": {k: round(v["ms"] / args.steps, 4) for k, v in
                                                 sorted(kern.items(), key=lambda kv: -kv[1]["ms"])},
            "job": job_info,
            "cpu_baseline": cpu,
            "gen_s": round(gen_s, 2),
            "store_reuse": store_leg_res,
            "minimize_corpus_tail": tail,
            "novelty_config3": nov if nov is not None else nov_sh,
            "call_cooccurrence": cooc,
            "setops_triage": sops,
            "canonicalize_raw_covers": canon,
            "cover_analytics": ana,
            "hub_ingest_config5": hubr,
            "manager_cycle": app,
            "layout_change": lchg,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def layout_change_leg(args, dev, corp, d_pcs, d_off, d_grp, d_len, G, C, uses, d_uses, d_static, d_prios, d_run,
                      d_sel, d_hist, d_out, d_goff, d_pres, sptr, ms_headline):
    """Side leg (never `value`): minimizeCorpus + CalculatePriorities + BuildChoiceTable as in the headline
    step, but every step's corpus is the step before's plus --layout-change fresh programs, as when the
    manager's NewInputs (manager.go:599-616) land between the Connect-driven minimizes (manager.go:569): the
    call groups' sizes and PCs differ on every call, so the job's cached plans never match the layout. One
    corpus of 1M + (warmup + steps) x batch programs is resident; step i minimizes its first 1M + i x batch
    entries. Reports ms per step beside the headline's."""
    import torch
    from syzkaller_amd import cover, synth
    batch = args.layout_change
    nsteps = max(1, args.steps)
    extra_n = batch * (args.warmup + nsteps + 1)
    ex = synth.corpus(args.seed + 0x51, extra_n, args.ngroups, args.npcs)

    def dt(a):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
        return torch.from_numpy(a.view(view.get(a.dtype, a.dtype))).to(dev)

    n0 = corp.n
    a_pcs = torch.cat([d_pcs[:int(corp.off[-1])], dt(ex.pcs)])
    a_off = torch.cat([d_off, dt(ex.off[1:] + np.uint64(corp.off[-1]))])
    a_grp = torch.cat([d_grp, dt(ex.group)])
    a_len = torch.cat([d_len, dt(ex.prog_len)])
    sel = torch.zeros(n0 + extra_n, dtype=torch.uint8, device=dev)
    out_idx = torch.zeros(n0 + extra_n, dtype=torch.int64, device=dev)
    job = cover.MinimizeJob()
    k = [0]

    def step():
        k[0] += 1
        n = n0 + k[0] * batch
        job.begin(a_pcs, a_off, a_grp, n, G, a_len, None, None, sptr)
        job.end_prio(C, d_uses, uses.shape[0], d_static, d_prios, d_run, None, sel, d_hist, out_idx, d_goff,
                     d_pres, sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(nsteps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / nsteps * 1e3
    job.close()
    return {"what": "the headline step on a corpus that grows by %d programs per step (a new call-group layout "
                    "every call, so the cached plans never match)" % batch,
            "programs_first_timed": n0 + (args.warmup + 1) * batch, "steps": nsteps,
            "ms_per_step": round(ms, 4), "headline_ms_per_step": round(ms_headline, 4),
            "over_headline_ms": round(ms - ms_headline, 4)}


def store_leg(args, L, corp, d_pcs, d_off, d_grp, d_len, d_sel, d_hist, C, G, sptr):
    """Side leg (never the headline): the resident store (syzgpu_corpus_create_dev: per-call dense PC
    ids built once, like mgr.corpus is loaded) and minimizeCorpus re-run on it with the same covers.
    The store is what the manager's cover analytics and NewInput append work on."""
    import torch
    from syzkaller_amd import _lib, cover
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    store = cover.CoverStore.from_device(d_pcs, d_off, d_grp, d_len, corp.n, G, sptr)
    torch.cuda.synchronize()
    ingest_s = time.perf_counter() - t0
    for _ in range(2):
        _lib.check(L.syzgpu_corpus_minimize_dev(store.handle, C, d_sel.data_ptr(), d_hist.data_ptr(), sptr))
    torch.cuda.synchronize()
    steps = max(1, args.steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        _lib.check(L.syzgpu_corpus_minimize_dev(store.handle, C, d_sel.data_ptr(), d_hist.data_ptr(), sptr))
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    return {"what": "store ingest once + minimizeCorpus re-run on the unchanged store (NOT the headline: the "
                    "store build is outside this loop)",
            "ingest_s": round(ingest_s, 4), "minimize_ms": round(ms, 4), **store.info()}, store


def append_leg(args, dev, store, sptr, C, d_hist):
    """The manager's corpus cycle on the resident store. NewInput (manager.go:609-616) is the gate on
    corpusCover (syzgpu_corpus_new_inputs_dev: Difference -> skip, Union + append): `--append` fresh
    programs in batches of 1000, each batch one call; then minimizeCorpus with mgr.corpus = newCorpus
    (manager.go:507-529, syzgpu_corpus_minimize_keep_dev), then CalculatePriorities + BuildChoiceTable on
    the kept length histogram. Two cycles, the second from the first one's kept corpus. Beside them:
    single-program NewInput RPCs (gated and unconditional appends) timed one by one, and the one-time
    build of corpusCover from the store's covers (the first gate's)."""
    import torch
    from syzkaller_amd import _lib, synth
    L = _lib.lib()
    b = synth.corpus(args.seed + 0x40, args.append, args.ngroups, args.npcs)
    one = synth.corpus(args.seed + 0x41, 64, args.ngroups, args.npcs)

    def t(a):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
        return torch.from_numpy(np.ascontiguousarray(a).view(view.get(a.dtype, a.dtype))).to(dev)

    def slices(c, batch):
        out = []
        for a in range(0, c.n, batch):
            e = min(c.n, a + batch)
            o = c.off[a:e + 1].astype(np.uint64)
            out.append((t(c.pcs[int(o[0]):int(o[-1])]), t(o - o[0]), t(c.group[a:e]), t(c.prog_len[a:e]), e - a))
        return out
    batch = 1000
    parts = slices(b, batch)
    singles = slices(one, 1)
    d_new = torch.zeros(batch, dtype=torch.uint8, device=dev)
    uses = static_usage(C)
    d_uses = t(uses)
    d_static = torch.empty((C, C), dtype=torch.float32, device=dev)
    d_prios = torch.empty((C, C), dtype=torch.float32, device=dev)
    d_run = torch.empty((C, C), dtype=torch.int64, device=dev)
    empty = (t(np.zeros(1, np.uint32)), t(np.zeros(1, np.uint64)), t(np.zeros(1, np.uint32)),
             t(np.zeros(1, np.uint16)), 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    store.NewInputsDevice(*empty, None, sptr)  # corpusCover built from the store's covers
    build_ms = (time.perf_counter() - t0) * 1e3

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, r
    cycles = []
    for _ in range(2):
        n0 = store.n
        per, acc = [], 0
        for d in parts:
            ms, na = timed(lambda: store.NewInputsDevice(*d, d_new, sptr))
            per.append(ms)
            acc += na
        t1 = time.perf_counter()
        kept = store.MinimizeKeep(C, None, d_hist, None, None, sptr)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        _lib.check(L.syzgpu_static_priorities_dev(d_uses.data_ptr(), uses.shape[0], C, d_static.data_ptr(), sptr))
        _lib.check(L.syzgpu_prio_choice_dev(d_static.data_ptr(), d_hist.data_ptr(), C, None, d_prios.data_ptr(),
                                            d_run.data_ptr(), None, sptr))
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        cycles.append({"entries_before": int(n0), "offered": int(b.n), "accepted": int(acc), "kept": int(kept),
                       "new_input_ms": round(sum(per), 3),
                       "new_input_1000_ms_median": round(float(np.median(per)), 3),
                       "minimize_keep_ms": round((t2 - t1) * 1e3, 3), "prio_ms": round((t3 - t2) * 1e3, 3),
                       "cycle_ms": round(sum(per) + (t3 - t1) * 1e3, 3)})
    # single-program RPCs on the kept store: gated, then unconditional (a stale index after each)
    g1 = [timed(lambda: store.NewInputsDevice(*d, d_new, sptr))[0] for d in singles[:32]]
    u1 = [timed(lambda: store.append_device(*d, sptr))[0] for d in singles[32:]]
    u1000 = [timed(lambda: store.append_device(*d, sptr))[0] for d in parts[:5]]
    return {"what": "manager cycle on the resident store: %d gated NewInput batches of %d programs "
                    "(corpusCover Difference -> skip, Union + append), minimizeCorpus + keep "
                    "(mgr.corpus = newCorpus), CalculatePriorities + ChoiceTable; two cycles; then single-"
                    "program NewInputs (gated / unconditional append) and unconditional 1000-program appends"
                    % (len(parts), batch),
            "corpus_cover_build_ms": round(build_ms, 3), "cycles": cycles,
            "new_input_1_ms_median": round(float(np.median(g1)), 4),
            "append_1_ms_median": round(float(np.median(u1)), 4),
            "append_1000_ms_median": round(float(np.median(u1000)), 4)}


def text_leg(args, dev, L, read_prof, corp, d_sel, sptr, ms_step):
    """The rest of minimizeCorpus (manager.go:531-553) after Minimize: every kept program is
    deserialized (prog.Deserialize -> len(p.Calls), encoding.go:120-127) and hashed (hash.Hash ->
    the persistent-corpus prune, :541-550). One syzgpu_prog_scan_dev over the resident program text
    of the corpus with the step's selection bytes as the mask; synthetic text with exactly prog_len
    calls per program (synth.prog_text)."""
    import torch
    from syzkaller_amd import prog, synth
    t0 = time.perf_counter()
    data, off = synth.prog_text(args.seed + 0x40, corp.prog_len)
    gen = time.perf_counter() - t0
    n = corp.n
    td = torch.from_numpy(data).to(dev)
    to = torch.from_numpy(off.view(np.int64)).to(dev)
    nc = torch.zeros(n, dtype=torch.int32, device=dev)
    stt = torch.zeros(n, dtype=torch.uint8, device=dev)
    sg = torch.zeros((n, 20), dtype=torch.uint8, device=dev)

    def run():  # the manager needs len(p.Calls) and the signature; CallSet's checks are the hub's
        prog.ProgScanDev(td, to, n, d_sel, nc, None, sg, sptr)
    prog.ProgScanDev(td, to, n, d_sel, nc, stt, sg, sptr)  # once with the checks: a valid corpus
    torch.cuda.synchronize()
    sel = d_sel.cpu().numpy().astype(bool)
    ok = bool((nc.cpu().numpy()[sel] == corp.prog_len[sel]).all() and not stt.cpu().numpy()[sel].any())
    nc.zero_()
    run()
    torch.cuda.synchronize()
    ok = ok and bool((nc.cpu().numpy()[sel] == corp.prog_len[sel]).all())
    steps = max(1, args.steps)
    L.syzgpu_profile_only(None)
    L.syzgpu_profile_enable(1)
    t1 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t1) / steps
    ev = read_prof()
    L.syzgpu_profile_enable(0)
    kept = int(sel.sum())
    lens = np.diff(off).astype(np.int64)
    kbytes = int(lens[sel].sum())
    blocks = int(((lens[sel] + 8) // 64 + 1).sum())
    res = {"what": "prog.Deserialize len(p.Calls) + hash.Hash over the kept programs",
           "kept_programs": kept, "text_bytes": kbytes, "sha1_blocks": blocks, "ms": round(el * 1e3, 4),
           "kept_progs_per_s": round(kept / el, 1), "ncalls_match_prog_len": ok, "gen_s": round(gen, 2),
           "minimize_corpus_ms": round(ms_step + el * 1e3, 4),
           "kernels_ms": {k: round(e["ms"] / steps, 4) for k, e in ev.items()}}
    if "prog_lane" in ev:
        e = ev["prog_lane"]
        ms = e["ms"] / e["launches"]
        alg = kbytes + 16 * kept + 24 * kept  # text + offsets read; ncalls and digest written
        res["roofline"] = {"bound": "valu", "kernel": "prog_lane", "avg_launch_ms": round(ms, 4),
                           "hbm_achieved": round(alg / (ms * 1e-3) / 1e9, 1), "hbm_peak": HBM_PEAK_GBS,
                           "hbm_frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "sha1_blocks_per_s": round(blocks / (ms * 1e-3), 1)}
    if args.cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        idx = np.flatnonzero(sel)[:200_000]
        sub_off = np.zeros(idx.size + 1, np.uint64)
        sub_off[1:] = np.cumsum(lens[idx])
        sub = np.frombuffer(b"".join(data[int(off[i]):int(off[i + 1])].tobytes() for i in idx), np.uint8)
        t2 = time.perf_counter()
        oracle.prog_scan(sub, sub_off)
        oracle.sha1(sub, sub_off)
        dt = time.perf_counter() - t2
        res["cpu_baseline"] = {"value": round(idx.size / dt, 1), "unit": "kept progs/s", "cores": 1, "kind": "port",
                               "sample": "first %d kept programs; oracle_prog_scan + oracle_sha1 per program, %.2f s"
                                         % (idx.size, dt)}
    return res


def analytics_leg(args, dev, L, read_prof, store, corp, sptr):
    """syz-manager's cover analytics (html.go:67-97 httpSummary per-call table and "cover" stat,
    html.go:213-237 uniqueCover both ways, html.go:158-170 httpCorpus's per-input UniqueCover) on the
    bench's resident 1M-program store: one syzgpu_corpus_cover_stats_dev per step, outputs in HBM.
    The oracle's literal restatement (Union grown input by input, Go-map counts) is timed on a sample."""
    import torch
    G, n = corp.ngroups, corp.n
    d64 = torch.zeros(3 * G + 3, dtype=torch.int64, device=dev)
    d_iu = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    p = d64.data_ptr()

    def run():
        _lib_check(L.syzgpu_corpus_cover_stats_dev(store.handle, p, p + 8 * G, p + 16 * G, p + 24 * G,
                                                   d_iu.data_ptr(), sptr))
    run()
    torch.cuda.synchronize()
    h = d64.cpu().numpy().view(np.uint64)
    tot = [int(x) for x in h[3 * G:3 * G + 3]]
    # size-independent identities: every input counted once, every one-call PC in one call, the
    # per-input unique counts add up to uniqueCover(false) (no 0xFFFFFFFF in synthetic covers)
    ok = bool(int(h[:G].sum()) == n and int(h[2 * G:3 * G].sum()) == tot[1]
              and int(d_iu.sum().item()) == tot[2] and tot[0] >= int(h[G:2 * G].max()))
    steps = max(1, args.steps)
    L.syzgpu_profile_only(None)
    L.syzgpu_profile_enable(1)
    t1 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t1) / steps
    ev = read_prof()
    L.syzgpu_profile_enable(0)
    res = {"what": "per-call Inputs/Cover/UniqueCover, total cover, uniqueCover(true/false), per-input UniqueCover",
           "ms": round(el * 1e3, 4), "progs_per_s": round(n / el, 1), "cover": tot[0],
           "unique_per_call": tot[1], "unique_per_input": tot[2], "identities_hold": ok,
           "kernels_ms": {k: round(e["ms"] / steps, 4) for k, e in sorted(ev.items(), key=lambda kv: -kv[1]["ms"])}}
    if "cs_uniq" in ev:
        e = ev["cs_uniq"]
        ms = e["ms"] / e["launches"]
        # what the kernel reads: the store's index-resident u16 id streams (2 B per PC; 16-B vectors of 8
        # ids) and one u32 entry tag per vector, not the 4-B PCs of the raw covers
        alg = 2 * int(corp.off[-1]) + 4 * (int(corp.off[-1]) // 8)
        res["roofline"] = {"bound": "hbm", "kernel": "cs_uniq", "achieved": round(alg / (ms * 1e-3) / 1e9, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "avg_launch_ms": round(ms, 4),
                           "algorithmic_bytes_per_launch": alg,
                           "bytes": "index-resident u16 id streams (2 B per PC) + a u32 entry tag per 8 ids; the "
                                    "index build (once per store, store_reuse) is outside this leg"}
    if args.cpu_baseline and args.analytics_cpu_sample > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        k = min(args.analytics_cpu_sample, n)
        t2 = time.perf_counter()
        oracle.cover_stats(corp.pcs[:int(corp.off[k])], corp.off[:k + 1], corp.group[:k], G)
        dt = time.perf_counter() - t2
        res["cpu_baseline"] = {"value": round(k / dt, 1), "unit": "progs/s", "cores": 1, "kind": "port",
                               "sample": "first %d programs of the corpus; oracle_cover_stats (literal html.go), "
                                         "%.2f s" % (k, dt)}
    return res


def hub_leg(args, dev, L, read_prof, corp, sptr):
    """BASELINE.json configs[4]'s ingest: syz-hub receives the corpora of 8 managers (here 8 x 125k
    programs per GPU, 10% of them copies of another manager's programs) and adds them to its corpus
    (state.go:211-228 addInput: prog.CallSet checks, hash.Hash, map insert on first occurrence). One step
    = empty the hub's signature set, syzgpu_prog_scan_dev (checks + SHA-1 of every program) and
    syzgpu_sigset_insert_dev of the whole batch in order; program text resident in HBM."""
    import torch
    from syzkaller_amd import prog, synth
    n = corp.n
    t0 = time.perf_counter()
    data, off = synth.prog_text(args.seed + 0x50, corp.prog_len)
    rnd = np.random.default_rng(9)
    idx = np.arange(n)
    dup = rnd.random(n) < 0.10
    mgr = idx // max(1, n // 8)
    src = rnd.integers(0, n, int(dup.sum()))
    idx[dup] = src  # a copy of another program (mostly another manager's)
    lens = (off[1:] - off[:-1]).astype(np.int64)[idx]
    noff = np.zeros(n + 1, np.int64)
    noff[1:] = np.cumsum(lens)
    d_data = torch.from_numpy(data).to(dev)
    byte_prog = torch.repeat_interleave(torch.arange(n, device=dev), torch.from_numpy(lens).to(dev))
    starts = torch.from_numpy(off[:-1].astype(np.int64)[idx]).to(dev)
    d_noff = torch.from_numpy(noff).to(dev)
    pos = torch.arange(int(noff[-1]), device=dev, dtype=torch.int64)
    blob = d_data[starts[byte_prog] + pos - d_noff[:-1][byte_prog]].contiguous()
    del byte_prog, pos, d_data
    gen = time.perf_counter() - t0
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    sigs = torch.zeros((n, 20), dtype=torch.uint8, device=dev)
    added = torch.zeros(n, dtype=torch.uint8, device=dev)
    h = np.zeros(1, np.uint64)
    _lib_check(L.syzgpu_sigset_create(n, h.ctypes.data))
    hs = int(h[0])
    na = np.zeros(1, np.uint64)

    def run():
        _lib_check(L.syzgpu_sigset_clear(hs, sptr))
        prog.ProgScanDev(blob, d_noff, n, None, None, status, sigs, sptr)
        _lib_check(L.syzgpu_sigset_insert_dev(hs, sigs.data_ptr(), None, n, 1, added.data_ptr(), na.ctypes.data,
                                              sptr))
    run()
    torch.cuda.synchronize()
    sg = sigs.cpu().numpy()
    distinct = np.unique(sg.view(np.dtype((np.void, 20))).ravel(), return_index=True)[1]
    want = np.zeros(n, np.uint8)
    want[distinct] = 1
    ok = bool(not status.cpu().numpy().any() and np.array_equal(added.cpu().numpy(), want))
    steps = max(1, args.steps)
    L.syzgpu_profile_only(None)
    L.syzgpu_profile_enable(1)
    t1 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t1) / steps
    ev = read_prof()
    L.syzgpu_profile_enable(0)
    L.syzgpu_sigset_destroy(hs)
    res = {"workload": "config5 ingest: 8 managers x %d programs, %.1f%% copies; %d distinct added" %
                       (n // 8, 100.0 * dup.mean(), int(na[0])),
           "metric": "hub ingest progs/sec", "ms": round(el * 1e3, 4), "progs_per_s": round(n / el, 1),
           "text_bytes": int(noff[-1]), "added_first_occurrences_match": ok, "gen_s": round(gen, 2),
           "kernels_ms": {k: round(e["ms"] / steps, 4) for k, e in sorted(ev.items(), key=lambda kv: -kv[1]["ms"])}}
    if "prog_lane" in ev:
        e = ev["prog_lane"]
        ms = e["ms"] / e["launches"]
        blocks = int(((lens + 8) // 64 + 1).sum())
        res["roofline"] = {"bound": "valu", "kernel": "prog_lane", "avg_launch_ms": round(ms, 4),
                           "sha1_blocks_per_s": round(blocks / (ms * 1e-3), 1),
                           "hbm_achieved": round((int(noff[-1]) + 44 * n) / (ms * 1e-3) / 1e9, 1),
                           "hbm_peak": HBM_PEAK_GBS}
    if args.cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        k = min(200_000, n)
        hb = blob[:int(noff[k])].cpu().numpy()
        ho = noff[:k + 1].astype(np.uint64)
        t2 = time.perf_counter()
        _, st = oracle.prog_scan(hb, ho)
        sg2 = oracle.sha1(hb, ho)
        seen = set()
        for i in range(k):  # the hub's map insert (st.Corpus[sig] == nil)
            if not (int(st[i]) & ~4):
                b = sg2[i].tobytes()
                if b not in seen:
                    seen.add(b)
        dt = time.perf_counter() - t2
        res["cpu_baseline"] = {"value": round(k / dt, 1), "unit": "progs/s", "cores": 1, "kind": "port",
                               "sample": "first %d programs of the batch; oracle_prog_scan + oracle_sha1 + a "
                                         "Python set insert, %.2f s" % (k, dt)}
    return res


def _lib_check(rc):
    from syzkaller_amd import _lib
    _lib.check(rc)


I8_PEAK_TOPS = 5000.0  # MI355X dense int8 MFMA: 2x the ~2.5 PF dense BF16 rate (MI355X_MICROARCH.md, MFMA table)


def cooccurrence_leg(args, dev, L, read_prof, corp, C):
    """The call-ID co-occurrence X^T X (syzgpu_call_cooccurrence_dev, int8 MFMA; SURVEY.md F1/K9 — not the
    reference's position-indexed calcDynamicPrio) over the bench corpus's programs: len(p.Calls) from the
    corpus, call ids Zipf(1.2) over C, seeded. Roofline: the int8 ops of the upper-triangle tiles the GEMM
    runs (2 * 128^2 * Kp per tile) over its launch time against the dense int8 MFMA peak."""
    import torch
    rnd = np.random.default_rng(args.seed + 0x77)
    lens = corp.prog_len.astype(np.uint64)
    off = np.zeros(corp.n + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    w = 1.0 / np.arange(1, C + 1) ** 1.2
    calls = rnd.choice(C, size=int(off[-1]), p=w / w.sum()).astype(np.uint16)
    dc = torch.from_numpy(calls.view(np.int16)).to(dev)
    do = torch.from_numpy(off.view(np.int64)).to(dev)
    out = torch.empty((C, C), dtype=torch.int32, device=dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream

    def step():
        _lib_check(L.syzgpu_call_cooccurrence_dev(dc.data_ptr(), do.data_ptr(), corp.n, C, out.data_ptr(), sptr))
    step()
    torch.cuda.synchronize()
    steps = max(1, args.steps // 2)
    L.syzgpu_profile_only(None)
    L.syzgpu_profile_enable(1)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ev = read_prof()
    L.syzgpu_profile_enable(0)
    T = (C + 127) // 128
    Kp = (corp.n + 31) // 32 * 32
    res = {"what": "call-ID co-occurrence X^T X - diag (int32 C x C) of %d programs (%d calls, ids Zipf(1.2) over "
                   "C=%d); not the reference's position-indexed calcDynamicPrio (SURVEY.md F1)" % (corp.n, int(off[-1]), C),
           "ms": round(el / steps * 1e3, 3),
           "kernels_ms": {k: round(e["ms"] / steps, 4) for k, e in ev.items()},
           "pairs": int(out.sum().item())}
    g = ev.get("cooc_gemm")
    if g:
        ms = g["ms"] / g["launches"]
        ops = 2.0 * (T * (T + 1) // 2) * 128 * 128 * Kp  # the upper-triangle tiles the kernel runs
        res["roofline"] = {"bound": "mfma", "kernel": "cooc_gemm (v_mfma_i32_32x32x32_i8)",
                           "achieved": round(ops / (ms * 1e-3) / 1e12, 1), "peak": I8_PEAK_TOPS, "unit": "TOP/s",
                           "frac": round(ops / (ms * 1e-3) / 1e12 / I8_PEAK_TOPS, 4), "avg_launch_ms": round(ms, 4),
                           "ops_per_launch": int(ops)}
    return res


def novelty_leg(args, dev, L, read_prof):
    """BASELINE.json configs[2]: a syz-fuzzer triage batch of 1M fresh execution covers against
    maxCover (fuzzer.go:446-470 per cover, in order), maxCover0 = the union of a 100k-program corpus
    per call, 5k flakes. Device-resident inputs; one step = syzgpu_novelty_batch_dev (is_new flags and
    the updated tables). The oracle's literal per-cover merge is timed on a sample beside it."""
    import torch
    from syzkaller_amd import cover, synth
    G = args.ngroups
    base = synth.corpus(args.seed + 0x30, 100_000, G, args.npcs)
    _, mcp, mco = cover.NoveltyBatch(base.pcs, base.off, base.group, G, np.zeros(0, np.uint32),
                                     np.zeros(G + 1, np.uint64), np.zeros(0, np.uint32))
    rnd = np.random.default_rng(3)
    flakes = np.unique(rnd.choice(base.pcs, 5000, replace=False))
    b = synth.corpus(args.seed + 0x31, args.novelty_covers, G, args.npcs)

    def t(a):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
        return torch.from_numpy(np.ascontiguousarray(a).view(view.get(a.dtype, a.dtype))).to(dev)
    d = [t(b.pcs), t(b.off), t(b.group), t(mcp), t(mco), t(flakes)]
    cap = int(mcp.size + b.pcs.size + 1)
    is_new = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    out = torch.empty(cap, dtype=torch.int32, device=dev)
    ooff = torch.zeros(G + 1, dtype=torch.int64, device=dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream

    def step():
        cover.NoveltyBatchDev(d[0], d[1], d[2], b.n, G, d[3], d[4], int(mco[-1]), d[5], flakes.size,
                              int(b.off[-1]), is_new, out, cap, ooff, sptr)
    step()
    torch.cuda.synchronize()
    steps = max(1, args.steps // 2)
    L.syzgpu_profile_only(None)  # every novelty scope: events on the launch stream, inside the timed loop
    L.syzgpu_profile_enable(1)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ev = read_prof()
    L.syzgpu_profile_enable(0)
    nl = int(b.off[-1])
    # SURVEY.md §8(d) bytes of one batch: cover PCs + CSR offsets + group ids read once, is_new written,
    # maxCover0 read, the updated tables written
    alg_batch = 4 * nl + 8 * (b.n + 1) + 4 * b.n + b.n + 4 * int(mco[-1]) + 4 * int(ooff[-1].item())
    res = {"workload": "config3: 1M fresh covers (%d PCs) vs maxCover0 of a 100k corpus (%d PCs), %d flakes"
                       % (nl, int(mco[-1]), flakes.size),
           "metric": "triage covers/sec", "value": round(b.n * steps / el, 1), "ms_per_batch": round(el / steps * 1e3, 3),
           "new_covers": int(is_new.sum().item()), "maxcover_out_pcs": int(ooff[-1].item()),
           "kernels_ms_per_batch": {k: round(e["ms"] / steps, 4) for k, e in sorted(ev.items(), key=lambda x: -x[1]["ms"])},
           "path_roofline": {"bytes_per_batch": alg_batch, "achieved": round(alg_batch / (el / steps) / 1e9, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(alg_batch / (el / steps) / 1e9 / HBM_PEAK_GBS, 4)}}
    if args.novelty_wide:
        # the same batch with its PC space spread over 34x the addresses (8M -> 272M span: past the
        # direct windows' 32M, so the hashed windows run); same outputs up to the monotone map
        base = 0x81000000

        def stretch(x):
            y = (x.to(torch.int64) & 0xFFFFFFFF) - base
            return (y * 34 + base).to(torch.int32)
        dw = [stretch(d[0]), d[1], d[2], stretch(d[3]), d[4], stretch(d[5])]

        def step_w():
            cover.NoveltyBatchDev(dw[0], dw[1], dw[2], b.n, G, dw[3], dw[4], int(mco[-1]), dw[5], flakes.size,
                                  int(b.off[-1]), is_new, out, cap, ooff, sptr)
        step_w()
        torch.cuda.synchronize()
        L.syzgpu_profile_enable(1)
        t0 = time.perf_counter()
        for _ in range(steps):
            step_w()
        torch.cuda.synchronize()
        elw = time.perf_counter() - t0
        evw = read_prof()
        L.syzgpu_profile_enable(0)
        del dw
        res["wide_span"] = {"span_addresses": int(34 * (int(max(b.pcs.max(), mcp.max())) - base)),
                            "ms_per_batch": round(elw / steps * 1e3, 3),
                            "ratio_vs_default_span": round(elw / el, 3),
                            "new_covers": int(is_new.sum().item()),
                            "kernels_ms_per_batch": {k: round(e["ms"] / steps, 4)
                                                     for k, e in sorted(evw.items(), key=lambda x: -x[1]["ms"])}}
    if ev:
        dom, e = max(ev.items(), key=lambda x: x[1]["ms"])
        ms = e["ms"] / e["launches"]
        alg = e["bytes"] / e["launches"]
        res["roofline"] = {"bound": "hbm", "kernel": dom, "achieved": round(alg / (ms * 1e-3) / 1e9, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "avg_launch_ms": round(ms, 3), "algorithmic_bytes_per_launch": int(alg)}
    if args.cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        k = min(args.novelty_cpu_sample, b.n)
        off = np.ascontiguousarray(b.off[: k + 1])
        t1 = time.perf_counter()
        oracle.novelty(b.pcs[: int(off[-1])], off, b.group[:k], G, mcp, mco, flakes)
        dt = time.perf_counter() - t1
        res["cpu_baseline"] = {"value": round(k / dt, 1), "unit": "covers/s", "cores": 1, "kind": "port",
                               "sample": "first %d covers of the batch; oracle/liboracle.so literal per-cover "
                                         "Difference/Union (fuzzer.go:446-470), %.2f s" % (k, dt)}
    return res


def canonicalize_leg(args, dev, L, read_prof=None):
    """cover.Canonicalize over a batch (cover/cover.go:28-40; its caller syz-fuzzer/fuzzer.go:355 runs it
    on every input's cover): config 3's 1M fresh covers as kcov returns them when the executor's
    dedup flag is off (executor.cc:565-585), each cover's PCs in random order with ~20 % of them
    repeated; device-resident (syzgpu_canonicalize_batch_dev, in place: the raw batch is restored by an
    untimed device copy before each step). Algorithmic bytes: the raw PCs read, the canonical ones
    written, offsets read and lengths written."""
    import torch
    from syzkaller_amd import cover, synth
    G = args.ngroups
    c = synth.corpus(args.seed + 0x31, args.novelty_covers, G, args.npcs)
    n = c.n
    pcs = torch.from_numpy(c.pcs.view(np.int32)).to(dev)
    lens = torch.from_numpy(np.diff(c.off).astype(np.int64)).to(dev)
    seg = torch.repeat_interleave(torch.arange(n, device=dev, dtype=torch.int64), lens)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    dup = torch.rand(pcs.numel(), generator=gen, device=dev) < 0.2
    pcs2, seg2 = torch.cat([pcs, pcs[dup]]), torch.cat([seg, seg[dup]])
    del pcs, seg, dup
    key = (seg2 << 32) | torch.randint(0, 1 << 31, (seg2.numel(),), generator=gen, device=dev, dtype=torch.int64)
    raw = pcs2[torch.argsort(key)].contiguous()
    del key, pcs2
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(torch.bincount(seg2, minlength=n), 0, out=off[1:])
    del seg2
    work = torch.empty_like(raw)
    out_len = torch.zeros(n, dtype=torch.int64, device=dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    steps = max(1, args.steps // 2)
    tot = 0.0
    for k in range(steps + 1):
        work.copy_(raw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cover.CanonicalizeBatchDev(work, off, n, out_len, sptr)  # returns after the stream drained
        if k:
            tot += time.perf_counter() - t0
    ms = tot / steps * 1e3
    nin, nout = int(raw.numel()), int(out_len.sum().item())
    ok = nout == int(c.off[-1])  # the raw batch canonicalizes back to the distinct PCs of each cover
    kms = None
    if read_prof is not None:  # one more pass with HIP events around the phases (not timed)
        L.syzgpu_profile_only(None)
        L.syzgpu_profile_enable(1)
        work.copy_(raw)
        cover.CanonicalizeBatchDev(work, off, n, out_len, sptr)
        kms = {k: round(e["ms"], 4) for k, e in read_prof().items()}
        L.syzgpu_profile_enable(0)
    alg = 4 * nin + 4 * nout + 8 * (n + 1) + 8 * n
    res = {"workload": "config3's 1M covers as raw kcov output: %d PCs (random order, ~20%% repeated) -> %d"
                       % (nin, nout),
           "ms_per_batch": round(ms, 3), "covers_per_s": round(n / ms * 1e3, 1), "canonical_pcs_match": ok,
           "phases_ms": kms,
           "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes": int(alg)}}
    # sorted sub-leg: the same covers as the executor returns them with its dedup flag on (sorted, no
    # repeats, executor.cc:565-585): each is checked in one streaming read and left as it is
    del work
    canon = torch.from_numpy(c.pcs.view(np.int32)).to(dev)
    coff = torch.from_numpy(c.off.view(np.int64)).to(dev)
    work2 = torch.empty_like(canon)
    tot2 = 0.0
    for k in range(steps + 1):
        work2.copy_(canon)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cover.CanonicalizeBatchDev(work2, coff, n, out_len, sptr)
        if k:
            tot2 += time.perf_counter() - t0
    ms2 = tot2 / steps * 1e3
    ok2 = bool(torch.equal(work2, canon)) and int(out_len.sum().item()) == int(c.off[-1])
    kms2 = None
    if read_prof is not None:  # one more pass with HIP events around the phases (not timed)
        L.syzgpu_profile_only(None)
        L.syzgpu_profile_enable(1)
        work2.copy_(canon)
        cover.CanonicalizeBatchDev(work2, coff, n, out_len, sptr)
        kms2 = {k: round(e["ms"], 4) for k, e in read_prof().items()}
        L.syzgpu_profile_enable(0)
    alg2 = 4 * int(c.off[-1]) + 8 * (n + 1) + 8 * n  # the PCs and offsets read, the lengths written
    res["sorted"] = {"workload": "the same 1M covers already canonical (executor dedup on): %d PCs" % int(c.off[-1]),
                     "ms_per_batch": round(ms2, 3), "covers_per_s": round(n / ms2 * 1e3, 1), "unchanged": ok2,
                     "phases_ms": kms2,
                     "roofline": {"bound": "hbm", "achieved": round(alg2 / (ms2 * 1e-3) / 1e9, 1),
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(alg2 / (ms2 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                  "algorithmic_bytes": int(alg2)}}
    del work2, canon
    if args.cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        ns = min(n, 20_000)
        rh = raw[: int(off[ns].item())].cpu().numpy().view(np.uint32)
        oh = off[: ns + 1].cpu().numpy()
        t0 = time.perf_counter()
        for i in range(ns):
            oracle.canonicalize(rh[oh[i]:oh[i + 1]])
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(ns / el, 1), "unit": "covers/s", "cores": 1, "kind": "port",
                               "sample": "first %d raw covers; oracle.canonicalize per cover (Go's sort + unique), "
                                         "%.2f s" % (ns, el)}
    return res


def setops_leg(args, dev, L, read_prof=None):
    """The cover set algebra in batch (cover/cover.go:42-102; triage users fuzzer.go:374-375,
    389-406): 1M pairs (config 3's fresh covers, each against a second run of the same input with 5 %
    of its PCs missing), device-resident; one launch sequence per op over all pairs
    (syzgpu_setop_batch_dev). Algorithmic bytes: both inputs and their offsets read, the output and
    its offsets written."""
    import torch
    from syzkaller_amd import cover, synth
    G = args.ngroups
    c = synth.corpus(args.seed + 0x31, args.novelty_covers, G, args.npcs)
    n = c.n

    def t(a):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
        return torch.from_numpy(np.ascontiguousarray(a).view(view.get(a.dtype, a.dtype))).to(dev)
    da, dao = t(c.pcs), t(c.off)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    keep = torch.rand(da.numel(), generator=gen, device=dev) > 0.05
    db = da[keep].contiguous()
    cs = torch.zeros(keep.numel() + 1, dtype=torch.int64, device=dev)
    torch.cumsum(keep, 0, out=cs[1:])
    dbo = (cs[dao] - cs[dao[:1]]).contiguous()
    del keep, cs
    na, nb = int(da.numel()), int(db.numel())
    cap = na + nb + 1
    out = torch.empty(cap, dtype=torch.int32, device=dev)
    ooff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    res = {"workload": "1M pairs: config-3 covers (%d PCs) vs a second run with 5%% of the PCs dropped (%d PCs)"
                       % (na, nb), "ops": {}}
    steps = max(1, args.steps // 2)
    for op in ("intersection", "difference", "union"):
        tot = cover.SetOpBatchDev(op, da, dao, na, db, dbo, nb, n, out, cap, ooff, sptr)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            tot = cover.SetOpBatchDev(op, da, dao, na, db, dbo, nb, n, out, cap, ooff, sptr)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        kms = None
        if read_prof is not None:  # the count and emit passes alone (HIP events around each)
            L.syzgpu_profile_only(None)
            L.syzgpu_profile_enable(1)
            cover.SetOpBatchDev(op, da, dao, na, db, dbo, nb, n, out, cap, ooff, sptr)
            torch.cuda.synchronize()
            kms = {k: round(v["ms"], 3) for k, v in read_prof().items()}
            L.syzgpu_profile_enable(0)
        alg = 4 * (na + nb) + 16 * (n + 1) + 4 * tot + 8 * (n + 1)
        res["ops"][op] = {"ms_per_batch": round(ms, 3), "out_pcs": int(tot), "pairs_per_s": round(n / ms * 1e3, 1),
                          "kernels_ms": kms,
                          "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 1),
                                       "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                       "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                       "algorithmic_bytes": int(alg)}}
    return res


def novelty_leg_sharded(args, dev, L, dist, rank, world):
    """configs[2] on N GPUs (every rank runs it): the same 1M-cover batch and maxCover0 as
    novelty_leg, sharded by PC value (sharding.novelty_shard's plan: equal-count PC ranges from a
    sample, identical on every rank). Each rank holds its range's slice of the batch, of the tables and
    of the flakes in HBM (sliced on the device before the timed loop, as a PC-sharded maxCover would be
    kept); a step = syzgpu_novelty_batch_dev on the slice, the per-call "updated" flags, and one RCCL
    MAX all-reduce of n + G bytes (is_new + updated). The updated tables stay sharded (each rank's
    range is all the next batch needs). Strong scaling: the batch is fixed."""
    import torch
    from syzkaller_amd import cover, sharding, synth

    def any_failed(bad):
        # every rank reaches this collective whatever failed locally, so a failure on one rank is
        # reported by all of them instead of leaving the others blocked in a later collective
        f = torch.tensor([1 if bad else 0], dtype=torch.int32, device=dev)
        sharding.allreduce(f, dist, dist.ReduceOp.MAX)
        return int(f.item()) != 0

    try:
        prep = _novelty_shard_prepare(args, dev, rank, world)
        err = None
    except Exception as e:  # noqa: BLE001
        prep, err = None, "%s: %s" % (type(e).__name__, e)
    if any_failed(err is not None):
        return {"error": err or "another rank failed preparing its slice"}
    b, G, mco, flakes, p_r, o_r, m_r, mo_r, f_r, d_f, d_grp = prep
    g64 = d_grp.to(torch.int64)
    nl, nm = int(o_r[-1].item()), int(mo_r[-1].item())
    cap = nm + nl + 1
    flags = torch.zeros(b.n + G, dtype=torch.uint8, device=dev)
    is_new = flags[: b.n]
    out = torch.empty(cap, dtype=torch.int32, device=dev)
    ooff = torch.zeros(G + 1, dtype=torch.int64, device=dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream

    def step():
        ok = True
        try:
            cover.NoveltyBatchDev(p_r, o_r, d_grp, b.n, G, m_r, mo_r, nm, d_f, f_r.size, nl, is_new, out, cap, ooff,
                                  sptr)
            flags[b.n:].zero_()
            flags[b.n:].scatter_reduce_(0, g64, is_new, "amax")
        except Exception:  # noqa: BLE001
            ok = False
        sharding.allreduce_max_u8(flags, dist)  # reached on every rank
        return ok
    if any_failed(not step()):
        return {"error": "the sharded novelty step failed on some rank"}
    torch.cuda.synchronize()
    steps = max(1, args.steps // 2)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    sharding.allreduce(el, dist, dist.ReduceOp.MAX)
    el = float(el.item())
    new = int(is_new.sum().item())
    tab = torch.tensor([int(ooff[-1].item())], dtype=torch.int64, device=dev)
    sharding.allreduce(tab, dist)
    return {"workload": "config3: 1M fresh covers (%d PCs) vs maxCover0 of a 100k corpus (%d PCs), %d flakes; "
                        "sharded by PC range over %d ranks" % (int(b.off[-1]), int(mco[-1]), flakes.size, world),
            "metric": "triage covers/sec", "value": round(b.n * steps / el, 1), "ms_per_batch": round(el / steps * 1e3, 3),
            "scaling": "strong", "new_covers": new, "maxcover_out_pcs": int(tab.item()),
            "rank0_slice_pcs": nl, "exchange_bytes_per_batch": b.n + G,
            "exchange": "one MAX all-reduce of n + G bytes (is_new + per-call updated); tables stay sharded"}


def _novelty_shard_prepare(args, dev, rank, world):
    """This rank's PC-range slice of the config-3 batch, tables and flakes, on the device (no collectives)."""
    import torch
    from syzkaller_amd import cover, sharding, synth
    G = args.ngroups
    base = synth.corpus(args.seed + 0x30, 100_000, G, args.npcs)
    _, mcp, mco = cover.NoveltyBatch(base.pcs, base.off, base.group, G, np.zeros(0, np.uint32),
                                     np.zeros(G + 1, np.uint64), np.zeros(0, np.uint32))
    rnd = np.random.default_rng(3)
    flakes = np.unique(rnd.choice(base.pcs, 5000, replace=False))
    b = synth.corpus(args.seed + 0x31, args.novelty_covers, G, args.npcs)
    bounds = sharding.pc_bounds(b.pcs[:: max(1, b.pcs.size // 200_000)], world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1]) - 1

    def t(a):
        view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
        return torch.from_numpy(np.ascontiguousarray(a).view(view.get(a.dtype, a.dtype))).to(dev)

    def dslice(pcs, off):
        # [lo, hi] of every sorted list, on the device: mask, compaction, per-list counts
        u = pcs.to(torch.int64) & 0xFFFFFFFF
        m = (u >= lo) & (u <= hi)
        cs = torch.zeros(m.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(m, 0, out=cs[1:])
        o2 = cs[off] - cs[off[:1]]
        return pcs[m].contiguous(), o2.contiguous()
    p_r, o_r = dslice(t(b.pcs), t(b.off))
    m_r, mo_r = dslice(t(mcp), t(mco))
    f_r = flakes[(flakes >= lo) & (flakes <= hi)]
    d_f, d_grp = t(f_r), t(b.group)
    return b, G, mco, flakes, p_r, o_r, m_r, mo_r, f_r, d_f, d_grp


def cpu_baseline(corp, uses, n_sample):
    """The oracle (single-threaded C restatement of the Go path) on the first n_sample programs:
    minimizeCorpus, then CalculatePriorities (calcStaticPriorities in Go's loop form, calcDynamicPrio,
    the product) and BuildChoiceTable."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    off = np.ascontiguousarray(corp.off[: n_sample + 1])
    pcs = corp.pcs[: int(off[-1])]
    grp = np.ascontiguousarray(corp.group[:n_sample])
    t = time.perf_counter()
    kept, _ = oracle.minimize_grouped(pcs, off, grp, corp.ngroups)
    pr = oracle.calculate_priorities(oracle.static_priorities(uses), corp.prog_len[kept])
    oracle.build_choice_table(pr, None)
    dt = time.perf_counter() - t
    # SURVEY.md §8d's stronger baseline: the call groups over the host threads this job may use
    nth = max(1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1))
    t = time.perf_counter()
    kept_mt, _ = oracle.minimize_grouped_mt(pcs, off, grp, corp.ngroups, nth)
    pr = oracle.calculate_priorities(oracle.static_priorities(uses), corp.prog_len[kept_mt])
    oracle.build_choice_table(pr, None)
    dt_mt = time.perf_counter() - t
    return {"value": round(n_sample / dt, 1), "unit": "progs/s", "cores": 1, "kind": "port",
            "sample": "first %d programs of the same corpus (%d PCs); oracle/liboracle.so: Minimize + "
                      "CalculatePriorities + BuildChoiceTable, %.2f s" % (n_sample, int(off[-1]), dt),
            "cpu": _cpu_model(),
            "multi_thread": {"value": round(n_sample / dt_mt, 1), "unit": "progs/s", "cores": nth,
                             "same_selection": bool(np.array_equal(kept, kept_mt)),
                             "sample": "the same sample; call groups over %d threads, largest first "
                                       "(oracle_minimize_grouped_mt), %.2f s" % (nth, dt_mt)}}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
