"""Quick GPU sanity run: small Minimize / prio calls with progress output (for gpurun debugging)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from syzkaller_amd import cover, synth  # noqa: E402

print("golden minimize", cover.Minimize([[1, 2, 3], [4, 5, 6], [7, 8, 9]]), flush=True)
for n, G, P in [(100, 3, 500), (5000, 17, 20000), (100_000, 289, 500_000), (300_000, 5, 200_000)]:
    c = synth.corpus(n, n, G, P)
    t = time.time()
    got, goff = cover.MinimizeCorpus(c.pcs, c.off, c.group, c.ngroups)
    dt = time.time() - t
    want, _ = oracle.minimize_grouped(c.pcs, c.off, c.group, c.ngroups)
    print("n=%d G=%d kept=%d gpu=%.3fs parity=%s" % (n, G, got.size, dt, np.array_equal(got, want)), flush=True)
