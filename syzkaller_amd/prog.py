"""Host mirror of the reference's call-priority API (prog/prio.go) over libsyzgpu.so.

    CalculatePriorities(static, prog_lens)   prio.go:29   (static = calcStaticPriorities() result)
    calcDynamicPrio(prog_lens, C)            prio.go:137  (+ normalizePrio, prio.go:158)
    BuildChoiceTable(prios, enabled=None)    prio.go:202  -> ChoiceTable
    ChoiceTable.Choose(rng, call)            prio.go:230  (consumer; host-side, not part of the GPU path)

The reference reads only len(p.Calls) of each corpus program, so programs are
passed as an array of call counts. calcStaticPriorities needs the generated sys.Calls type graph,
which the reference snapshot does not contain: its C*C result is an input.
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
