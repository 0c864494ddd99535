"""Diagnostic: run the Go-sort simulation on the bench corpus's call groups with the stats build
(libsyzgpu_dbg.so, -DSYZ_GS_STATS) and print the LDS sorter's level / cycle breakdown."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SYZGPU_LIB"] = os.path.join(ROOT, "syzkaller_amd", "libsyzgpu_dbg.so")
import numpy as np  # noqa: E402

from syzkaller_amd import _lib, cover, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
p = synth.params(int(os.environ.get("GS_SEED", "0x5EED0004"), 0), n, 289, int(os.environ.get("GS_NPCS", "2000000")))
group, off, plen = synth.layout(p)
order = np.argsort(group, kind="stable")
lens = np.diff(off)[order].astype(np.uint64)
goff = np.zeros(290, np.uint64)
np.cumsum(np.bincount(group, minlength=289), out=goff[1:])
print("largest groups", sorted(np.diff(goff).tolist())[-5:], flush=True)
L = _lib.lib()
L.syzgpu_debug_gosort_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
st = np.zeros(24, np.uint64)
for it in range(3):
    L.syzgpu_debug_gosort_stats(st.ctypes.data, 1)
    t = time.perf_counter()
    cover.MinimizeOrder(lens, goff)
    dt = time.perf_counter() - t
    L.syzgpu_debug_gosort_stats(st.ctypes.data, 1)
    names = ["packs", "levels", "cyc_total", "pivot", "part0", "probe", "part1", "children", "heaps", "heap_el",
             "max_na", "leaves"]
    print("iter %d host %.2f ms" % (it, dt * 1e3), {k: int(v) for k, v in zip(names, st)}, flush=True)
    pk = max(1, int(st[0]))
    print("  per pack: levels %.1f cycles %.0f | per level: pivot %.0f part0 %.0f probe %.0f part1 %.0f children %.0f"
          % (st[1] / pk, st[2] / pk, st[3] / max(1, st[1]), st[4] / max(1, st[1]), st[5] / max(1, st[1]),
             st[6] / max(1, st[1]), st[7] / max(1, st[1])), flush=True)
    print("  part0 per level: walk+scan %.0f bnd %.0f classify+list %.0f swap %.0f" %
          tuple(st[12 + i] / max(1, st[1]) for i in range(4)), flush=True)
    x = int(st[17])
    print("  slowest pack: %d cycles, %d levels, %d elements" % (x >> 24, (x >> 14) & 1023, x & 16383), flush=True)
