"""The last minimize step's kernel timeline from a rocprofv3 --kernel-trace CSV (dev tooling).
Usage: python tools/timeline.py gpurun_out/TAG/kt [first-kernel-substring]"""
import csv
import glob
import os
import sys

root = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_grp_count"
path = [p for p in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)][0]
rows = list(csv.DictReader(open(path)))
col = lambda *names: next(k for k in rows[0] if any(n.lower() == k.lower() for n in names))
kn, ks, ke = col("Kernel_Name"), col("Start_Timestamp"), col("End_Timestamp")
kq = next((k for k in rows[0] if k.lower() in ("stream_id", "queue_id")), None)
rows.sort(key=lambda r: int(r[ks]))
starts = [i for i, r in enumerate(rows) if first in r[kn]]
rows = rows[starts[-1]:]
t0 = int(rows[0][ks])
end = max(int(r[ke]) for r in rows)
print("step: %.3f ms, %d kernels (%s)" % ((end - t0) / 1e6, len(rows), path))
agg = {}
for r in rows:
    name = r[kn].split("(")[0].replace("void ", "")[:60]
    a, b = (int(r[ks]) - t0) / 1e3, (int(r[ke]) - t0) / 1e3
    q = r[kq] if kq else "?"
    g = agg.setdefault((name, q), [0, 0.0, a, b])
    g[0] += 1
    g[1] += b - a
    g[2] = min(g[2], a)
    g[3] = max(g[3], b)
print("%-60s %5s %4s %9s %9s %9s" % ("kernel", "queue", "n", "busy_us", "first_us", "last_us"))
for (name, q), (n, busy, a, b) in sorted(agg.items(), key=lambda x: x[1][2]):
    print("%-60s %5s %4d %9.1f %9.1f %9.1f" % (name, q, n, busy, a, b))
