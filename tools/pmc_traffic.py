#!/usr/bin/env python3
"""Parse the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_pmc.sh into profiles/pmc_traffic.json.

FETCH_SIZE and WRITE_SIZE are KiB per dispatch; a kernel's dispatches (e.g. the two pmin classes of a
step) are averaged. On gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md §HBM), so it is doubled; WRITE_SIZE is exact for 16-B
stores and taken as is. Per kernel: the mean over its dispatches of the bench command (3 timed + 1
warmup steps), as HBM bytes per launch.
"""
import csv
import glob
import json
import os
import sys


# kernel name -> the bench's profiling scope around it (bench.py ROCPROF_SCOPE)
SCOPES = [("k_slab<", "k_slab"), ("k_smin_direct", "k_pmin_direct"), ("k_smin_hash<false>", "k_pmin_hash"),
          ("k_smin_hash<true>", "k_pmin_packed")]


def short(name, grid):
    """The bench scope of a kernel (k_smin_direct -> k_pmin_direct), else its base name
    (`void syz::k_gr_swap<true>(...)` -> `k_gr_swap`)."""
    for pat, scope in SCOPES:
        if pat in name:
            return scope
    head = name.split("(")[0]
    base = head.split("<")[0].split("::")[-1].strip()
    if base.startswith("void "):
        base = base[5:]
    return base or None


def read(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            s = short(row.get("Kernel_Name", ""), int(float(row.get("Grid_Size", 0) or 0)))
            if s:
                vals.setdefault(s, []).append(float(row["Counter_Value"]))
    return vals


def main(d, out):
    fetch, write = read(d, "FETCH_SIZE"), read(d, "WRITE_SIZE")
    res = {"workload": "config4-1M", "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes",
           "note": "FETCH_SIZE doubled (gfx950 streaming-read undercount); KiB -> bytes", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
        res["kernels"][k] = {"dispatches": len(fetch.get(k, [])), "fetch_bytes": int(2 * f * 1024),
                             "write_bytes": int(w * 1024), "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
