"""Times the raw minimize job's kernels on the bench corpus (dev tooling): per-scope HIP events."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from syzkaller_amd import _lib, cover, synth
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
def step():
    job.begin(d[0], d[1], d[2], c.n, 289, d[3], stream=s)
for _ in range(int(os.environ.get("PM_W", "3"))):
    step()
torch.cuda.synchronize()
L.syzgpu_profile_only(None)
if os.environ.get("PM_PROF", "1") == "1":
    L.syzgpu_profile_enable(1)
K = int(os.environ.get("PM_K", "5"))
t0 = time.perf_counter()
for _ in range(K):
    step()
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / K
cap = 4096
names = ctypes.create_string_buffer(48 * cap)
ms = np.zeros(cap, np.float32)
by = np.zeros(cap, np.uint64)
k = L.syzgpu_profile_read(names, ms.ctypes.data, by.ctypes.data, cap)
agg = {}
for i in range(k):
    nm = names.raw[48 * i:48 * (i + 1)].split(b"\0")[0].decode()
    agg[nm] = agg.get(nm, 0.0) + float(ms[i]) / K
print(os.environ.get("SYZGPU_PM_DBG", "0"), "step_ms %.3f" % (el * 1e3), {k2: round(v, 3) for k2, v in sorted(agg.items(), key=lambda x: -x[1])}, job.info())
