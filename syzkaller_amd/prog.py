"""Host mirror of the reference's call-priority API (prog/prio.go) over libsyzgpu.so.

    calcStaticPriorities(usage=None)         prio.go:40   (usage: sysdesc.Usage, default the bundled sys/*.txt)
    CalculatePriorities(static, prog_lens)   prio.go:29   (static = calcStaticPriorities() result)
    calcDynamicPrio(prog_lens, C)            prio.go:137  (+ normalizePrio, prio.go:158)
    BuildChoiceTable(prios, enabled=None)    prio.go:202  -> ChoiceTable
    ChoiceTable.Choose(rng, call)            prio.go:230  (consumer; host-side, not part of the GPU path)
    CallCounts(data, off)                    encoding.go:120-127  len(p.Calls) of Deserialize, batched
    CallSetStatus(data, off)                 encoding.go:522-551  CallSet's checks, batched

The reference reads only len(p.Calls) of each corpus program, so programs are
passed as an array of call counts. calcStaticPriorities walks the sys.Calls type graph that sysgen
generates from sys/*.txt; sysdesc.py restates that walk on the host and hands the GPU the key-by-call
weight matrix it produces (the contraction runs on the int8 matrix cores, static_prio.hip).
"""
import numpy as np

from ._lib import check, lib, ptr


def _lens(prog_lens):
    return np.ascontiguousarray(np.asarray(prog_lens, dtype=np.uint16))


def calcDynamicPrio(prog_lens, C):
    lens = _lens(prog_lens)
    out = np.empty((C, C), dtype=np.float32)
    check(lib().syzgpu_dynamic_prio(ptr(lens), lens.size, C, ptr(out)))
    return out


def CallCooccurrence(calls, off, C):
    """The call-ID co-occurrence XᵀX on int8 MFMA (not the reference's calcDynamicPrio,
    which counts call positions): int32 C x C, [a][b] = ordered pairs of distinct positions with calls
    (a, b) in one program, summed over the programs of the CSR (calls, off)."""
    calls = np.ascontiguousarray(calls, dtype=np.uint16)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    out = np.empty((C, C), dtype=np.int32)
    check(lib().syzgpu_call_cooccurrence(ptr(calls), ptr(off), off.size - 1, C, ptr(out)))
    return out


def calcStaticPriorities(usage=None):
    """prio.go:40-135 for the calls of `usage` (sysdesc.Usage; default: the bundled sys/*.txt)."""
    if usage is None:
        from . import sysdesc
        usage = sysdesc.bundled()
    w = np.ascontiguousarray(usage.weights, dtype=np.float32)
    C = w.shape[1]
    out = np.empty((C, C), dtype=np.float32)
    check(lib().syzgpu_static_priorities(ptr(w), w.shape[0], C, ptr(out)))
    return out


def CalculatePriorities(static, prog_lens):
    static = np.ascontiguousarray(static, dtype=np.float32)
    C = static.shape[0]
    lens = _lens(prog_lens)
    out = np.empty((C, C), dtype=np.float32)
    check(lib().syzgpu_calculate_priorities(ptr(static), ptr(lens), lens.size, C, ptr(out)))
    return out


class ChoiceTable:
    """prio.go:196-200. run[i] is None for a disabled call (Go nil row, read by rand.go:406)."""

    def __init__(self, run, present, enabled):
        self.run_matrix = run
        self.present = present
        self.run = [run[i] if present[i] else None for i in range(run.shape[0])]
        self.enabled = enabled
        self.enabledCalls = [i for i in range(run.shape[0]) if enabled is None or enabled[i]]

    def Choose(self, rng, call):
        """prio.go:230-249 with a numpy Generator in place of Go's math/rand (not bit-compatible)."""
        if call < 0 or self.run[call] is None:
            return self.enabledCalls[int(rng.integers(len(self.enabledCalls)))]
        run = self.run[call]
        while True:
            x = int(rng.integers(int(run[-1])))
            i = int(np.searchsorted(run, x, side="left"))  # sort.SearchInts
            if self.enabled is None or self.enabled[i]:
                return i


def BuildChoiceTable(prios, enabled=None):
    prios = np.ascontiguousarray(prios, dtype=np.float32)
    C = prios.shape[0]
    en = None if enabled is None else np.ascontiguousarray(np.asarray(enabled, dtype=np.uint8))
    run = np.empty((C, C), dtype=np.int64)
    present = np.empty(C, dtype=np.uint8)
    check(lib().syzgpu_build_choice_table(ptr(prios), ptr(en), C, ptr(run), ptr(present)))
    return ChoiceTable(run, present, en)


# prog.CallSet errors (encoding.go:529-549) as status bits of ProgScan
NO_BRACKET, EMPTY_NAME, LINE_TOO_LONG, NO_CALLS = 1, 2, 4, 8


def _blob(data, off):
    if isinstance(data, (list, tuple)):  # [][]byte
        off = np.zeros(len(data) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(d) for d in data])
        data = np.frombuffer(b"".join(data), dtype=np.uint8) if data else np.zeros(0, np.uint8)
    return np.ascontiguousarray(data, dtype=np.uint8), np.ascontiguousarray(off, dtype=np.uint64)


def ProgScan(data, off=None, ncalls=True, status=True, sigs=True):
    """One pass over serialized programs (a list of bytes, or a CSR blob + offsets): returns
    (ncalls u32[n], status u8[n], sigs u8[n, 20]); the ones not asked for are None."""
    data, off = _blob(data, off)
    n = off.size - 1
    nc = np.zeros(max(n, 1), np.uint32) if ncalls else None
    st = np.zeros(max(n, 1), np.uint8) if status else None
    sg = np.zeros((max(n, 1), 20), np.uint8) if sigs else None
    check(lib().syzgpu_prog_scan(ptr(data), ptr(off), n, ptr(nc), ptr(st), ptr(sg)))
    return tuple(None if a is None else a[:n].copy() for a in (nc, st, sg))


def CallCounts(data, off=None):
    """len(p.Calls) of prog.Deserialize for every program (what CalculatePriorities reads)."""
    return ProgScan(data, off, status=False, sigs=False)[0]


def CallSetStatus(data, off=None):
    """0 where prog.CallSet would succeed, else an OR of NO_BRACKET / EMPTY_NAME / LINE_TOO_LONG /
    NO_CALLS."""
    return ProgScan(data, off, ncalls=False, sigs=False)[1]


def ProgScanDev(data, off, n, sel, ncalls, status, sigs, stream=0):
    """ProgScan on device-resident arrays (torch tensors or device pointers); sel (u8[n] or None)
    restricts the scan to selected programs; enqueued on `stream`."""
    check(lib().syzgpu_prog_scan_dev(ptr(data), ptr(off), n, ptr(sel), ptr(ncalls), ptr(status), ptr(sigs), stream))
