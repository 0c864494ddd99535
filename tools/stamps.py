"""Per-workgroup phase stamps of the transpose (k_part4) and the direct walk (k_pmin_direct) from a
-DSYZ_STAMPS build (tools/build_variant.sh st "-DSYZ_STAMPS"; SYZGPU_LIB=.../libsyzgpu_st.so): one
raw minimize job on the bench corpus, serial streams; prints the mean phase durations (s_memtime
ticks), the workgroup lifetimes and how many workgroups were alive on average (dev tooling)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SYZGPU_PM_SERIAL", "1")
import torch  # noqa: E402

from syzkaller_amd import _lib, cover, synth  # noqa: E402

L = _lib.lib()
_lib.check(L.syzgpu_init(0))
n = int(os.environ.get("PM_N", "1000000"))
c = synth.corpus(0x5EED0004, n, 289, 2_000_000)


def dt(a):
    view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
    return torch.from_numpy(a.view(view.get(a.dtype, a.dtype))).cuda()


d = [dt(c.pcs), dt(c.off), dt(c.group), dt(c.prog_len)]
job = cover.MinimizeJob()
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    job.begin(d[0], d[1], d[2], c.n, 289, d[3], stream=s)
torch.cuda.synchronize()
WG = 1 << 15
for which, name, phases in ((0, "k_part4", ["meta+tiles", "loads+pass1", "scan", "pass2", "store-issue"]),
                            (1, "k_pmin_direct", ["table-init", "walk", "emit"])):
    buf = np.zeros(WG * 8, np.uint64)
    L.syzgpu_debug_stamps.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    _lib.check(L.syzgpu_debug_stamps(which, buf.ctypes.data, buf.size))
    st = buf.reshape(WG, 8).astype(np.int64)
    k = len(phases) + 1
    ok = (st[:, :k] > 0).all(axis=1)
    st = st[ok, :k]
    if not st.size:
        print(name, "no stamps")
        continue
    # the last launch only: stamps of one launch lie within its span (drop stale rows of older launches)
    t0 = st[:, 0]
    newest = t0 >= np.percentile(t0, 1) if which == 0 else np.ones(len(st), bool)
    st = st[newest]
    d_ph = np.diff(st, axis=1)
    life = st[:, -1] - st[:, 0]
    span = st[:, -1].max() - st[:, 0].min()
    print("%s: %d workgroups, span %d ticks, mean lifetime %.0f, mean alive %.1f" %
          (name, len(st), span, life.mean(), life.sum() / max(1, span)))
    for i, ph in enumerate(phases):
        print("   %-12s mean %8.0f  p50 %8.0f  p90 %8.0f" % (ph, d_ph[:, i].mean(), np.median(d_ph[:, i]),
                                                           np.percentile(d_ph[:, i], 90)))
