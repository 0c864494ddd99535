"""Regenerates syzkaller_amd/data/sys_usage.json: the calcStaticPriorities usage matrix of a syzkaller
sys/ directory (default: the reference snapshot's), parsed by syzkaller_amd/sysdesc.py.

    python tools/gen_sys_usage.py [SYSDIR]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from syzkaller_amd import sysdesc  # noqa: E402


def main():
    sysdir = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/sys"
    u = sysdesc.usage(sysdesc.load_dir(sysdir))
    obj = {"source": "sys/*.txt of the reference snapshot, parsed by syzkaller_amd/sysdesc.py "
                     "(tools/gen_sys_usage.py)", **u.to_json()}
    with open(sysdesc.DATA, "w") as f:
        json.dump(obj, f, separators=(",", ":"))
        f.write("\n")
    print("calls %d, keys %d, non-zero weights %d" % (u.C, len(u.keys), len(obj["entries"])))


if __name__ == "__main__":
    main()
