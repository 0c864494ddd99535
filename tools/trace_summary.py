#!/usr/bin/env python3
"""Per-dispatch timeline of one bench step from a rocprofv3 --kernel-trace CSV.

    python tools/trace_summary.py gpurun_out/<dir>/prof/run_kernel_trace.csv [first_kernel_substring]

Prints, for the LAST step (from the last dispatch whose name contains first_kernel_substring, default
k_el_init), each kernel's duration and the gap before it, then per-kernel totals for that step.
"""
import csv
import sys
from collections import defaultdict


def main(path, first="k_el_init"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    if not idx:
        print("no", first)
        return
    step = rows[idx[-1]:]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = t0
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("syz::", "")[:40]
        print("%9.1f us  +gap %7.1f  dur %8.1f  %s" % ((s - t0) / 1e3, (s - prev_end) / 1e3, (e - s) / 1e3, name))
        tot[name] += (e - s) / 1e3
        cnt[name] += 1
        prev_end = e
    print("step wall %.1f us" % ((prev_end - t0) / 1e3))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("%8.1f us  x%-3d %s" % (v, cnt[k], k))


if __name__ == "__main__":
    main(*sys.argv[1:])
