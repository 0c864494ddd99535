"""Runs one bench.py side leg alone (dev tooling): python tools/leg_time.py LEG [bench args...]
LEG in setops, canonicalize, novelty; prints the leg's JSON."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
leg = sys.argv[1]
sys.argv = [sys.argv[0]] + sys.argv[2:]
import bench  # noqa: E402
args = bench.parse()
import torch  # noqa: E402
from syzkaller_amd import _lib  # noqa: E402
L = _lib.lib()
_lib.check(L.syzgpu_init(0))
dev = torch.device("cuda", 0)


def read_prof():
    import ctypes
    import numpy as np
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


if leg == "setops":
    res = bench.setops_leg(args, dev, L, read_prof)
elif leg == "canonicalize":
    res = bench.canonicalize_leg(args, dev, L, read_prof)
elif leg == "novelty":
    res = bench.novelty_leg(args, dev, L, read_prof)
else:
    raise SystemExit("unknown leg " + leg)
print(json.dumps(res))
