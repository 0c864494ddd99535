"""Times the resident store's NewInput paths on the bench corpus (dev tooling): the corpusCover build,
gated NewInput batches of 1 and 1000 fresh programs, unconditional appends of 1 and 1000, and the
minimizeCorpus + keep that catches the index up (after a warm-up cycle: the first minimize of a process
also pays the lazy loading of its kernels, reported as minimize_keep_first_call_ms).
SYZGPU_PHASE_TIMING=1 adds the phase split."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from syzkaller_amd import _lib, cover, synth
L = _lib.lib()
_lib.check(L.syzgpu_init(0))
n = int(os.environ.get("AT_N", "1000000"))
G = 289
c = synth.corpus(0x5EED0004, n, G, 2_000_000)
b = synth.corpus(0x5EED0044, 20_000, G, 2_000_000)


def dt(a):
    view = {np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64, np.dtype(np.uint16): np.int16}
    return torch.from_numpy(np.ascontiguousarray(a).view(view.get(a.dtype, a.dtype))).cuda()


def part(lo, hi):
    o = b.off[lo:hi + 1].astype(np.uint64)
    return dt(b.pcs[int(o[0]):int(o[-1])]), dt(o - o[0]), dt(b.group[lo:hi]), dt(b.prog_len[lo:hi]), hi - lo


s = torch.cuda.current_stream().cuda_stream
d = [dt(c.pcs), dt(c.off), dt(c.group), dt(c.prog_len)]
st = cover.CoverStore.from_device(d[0], d[1], d[2], d[3], c.n, G, s)
torch.cuda.synchronize()
C = int(max(c.prog_len.max(), b.prog_len.max()))
hist = torch.zeros(C + 1, dtype=torch.int64, device="cuda")
flag = torch.zeros(1000, dtype=torch.uint8, device="cuda")


def timed(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, r


out = {}
empty = (dt(np.zeros(1, np.uint32)), dt(np.zeros(1, np.uint64)), dt(np.zeros(1, np.uint32)), dt(np.zeros(1, np.uint16)), 0)
# the manager's steady state: minimizeCorpus has run before (the first call in a process also pays the
# lazy loading of every kernel it launches: reported apart), and one gated input has been caught up
out["minimize_keep_first_call_ms"] = timed(lambda: st.MinimizeKeep(C, None, hist, None, None, s))[0]
out["cc_build_ms"] = timed(lambda: st.NewInputsDevice(*empty, None, s))[0]
timed(lambda: st.NewInputsDevice(*part(19_999, 20_000), flag, s))
timed(lambda: st.MinimizeKeep(C, None, hist, None, None, s))
parts1 = [part(i, i + 1) for i in range(0, 40)]
parts1000 = [part(1000 + 1000 * i, 2000 + 1000 * i) for i in range(10)]
g1 = [timed(lambda: st.NewInputsDevice(*p, flag, s)) for p in parts1]
g1000 = [timed(lambda: st.NewInputsDevice(*p, flag, s)) for p in parts1000]
again = [timed(lambda: st.NewInputsDevice(*p, flag, s)) for p in parts1000[:5]]
out["gate_1_ms"] = [round(x[0], 3) for x in g1]
out["gate_1_accepted"] = sum(x[1] for x in g1)
out["gate_1000_ms"] = [round(x[0], 3) for x in g1000]
out["gate_1000_accepted"] = [x[1] for x in g1000]
out["gate_1000_seen_ms"] = [round(x[0], 3) for x in again]
out["minimize_keep_after_gates_ms"] = timed(lambda: st.MinimizeKeep(C, None, hist, None, None, s))[0]
out["minimize_keep_again_ms"] = timed(lambda: st.MinimizeKeep(C, None, hist, None, None, s))[0]
pu1 = [part(12_000 + i, 12_001 + i) for i in range(30)]
pu1000 = [part(13_000 + 1000 * i, 14_000 + 1000 * i) for i in range(5)]
u1 = [timed(lambda: st.append_device(*p, s))[0] for p in pu1]
u1000 = [timed(lambda: st.append_device(*p, s))[0] for p in pu1000]
out["append_1_ms"] = [round(x, 3) for x in u1]
out["append_1000_ms"] = [round(x, 3) for x in u1000]
out["minimize_keep_after_appends_ms"] = timed(lambda: st.MinimizeKeep(C, None, hist, None, None, s))[0]
for k in ("gate_1_ms", "gate_1000_ms", "append_1_ms", "append_1000_ms"):
    out[k.replace("_ms", "_median_ms")] = round(float(np.median(out[k])), 4)
print(out)
