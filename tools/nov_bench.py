"""Config-3 novelty leg alone (bench.py novelty_leg) for quick A/B runs on the GPU box.
Usage: python tools/nov_bench.py [steps] [covers]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    from syzkaller_amd import _lib
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    covers = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    args = argparse.Namespace(ngroups=289, npcs=2_000_000, seed=0x5EED0004, novelty_covers=covers, steps=2 * steps,
                              cpu_baseline=0, novelty_cpu_sample=0,
                              novelty_wide=int(os.environ.get("NOV_WIDE", "1")))
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    _lib.check(L.syzgpu_init(0))

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
    print(json.dumps(bench.novelty_leg(args, dev, L, read_prof)), flush=True)


if __name__ == "__main__":
    main()
