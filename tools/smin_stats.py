"""Diagnostic: where k_smin_direct's cycles go (stats build, tools/build_variant.sh smst "-DSYZ_SMIN_STATS"):
the raw minimize job on the bench corpus, one serialized step, per-workgroup means of each phase."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SYZGPU_LIB", os.path.join(ROOT, "syzkaller_amd", "libsyzgpu_smst.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from syzkaller_amd import _lib, cover, synth  # noqa: E402

L = _lib.lib()
_lib.check(L.syzgpu_init(0))
L.syzgpu_debug_smin_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
c = synth.corpus(0x5EED0004, int(os.environ.get("PM_N", "1000000")), 289, 2_000_000)


def dt(a):
    view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
    return torch.from_numpy(a.view(view.get(a.dtype, a.dtype))).cuda()


d = [dt(c.pcs), dt(c.off), dt(c.group), dt(c.prog_len)]
job = cover.MinimizeJob()
s = torch.cuda.current_stream().cuda_stream
st = np.zeros(24, np.uint64)
names = ["wgs", "cycles", "init", "walk", "emit", "batches", "ewins", "w0_steps", "batch_setup", "step_loop",
         "vectors", "runs"]
for it in range(4):
    L.syzgpu_debug_smin_stats(st.ctypes.data, 1)
    job.begin(d[0], d[1], d[2], c.n, 289, d[3], stream=s)
    torch.cuda.synchronize()
    L.syzgpu_debug_smin_stats(st.ctypes.data, 1)
    w = max(1, int(st[0]))
    print("iter", it, {k: int(v) for k, v in zip(names, st)}, flush=True)
    print("  per workgroup: cycles %.0f init %.0f walk %.0f emit %.0f | batches %.2f ewins %.2f steps %.1f "
          "setup %.0f steploop %.0f vectors %.0f runs %.0f | cycles/step %.0f" %
          (st[1] / w, st[2] / w, st[3] / w, st[4] / w, st[5] / w, st[6] / w, st[7] / w, st[8] / w, st[9] / w,
           st[10] / w, st[11] / w, st[9] / max(1, st[7])), flush=True)
    q = st[16:24]
    k = max(1, int(q[0]))
    print("  P per slab (%d): cycles %.0f | members+tiles %.0f loads+hist %.0f scan+D %.0f place %.0f pad %.0f store %.0f"
          % (k, q[1] / k, q[2] / k, q[3] / k, q[4] / k, q[5] / k, q[6] / k, q[7] / k), flush=True)
