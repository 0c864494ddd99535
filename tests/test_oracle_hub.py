"""tests/pyref.py's prog.CallSet restatement (used by the hub checks) against the oracle's program scan:
CallSet fails exactly when oracle_prog_scan reports NO_BRACKET / EMPTY_NAME / NO_CALLS (a too-long line
only ends CallSet's Scan loop, encoding.go:522-551)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from tests import pyref  # noqa: E402

CASES = [b"open()\n", b"", b"\n\n", b"# c\n", b"r0 = open(0x1)\nclose(r0)\n", b"r0 =   (0)\n", b"no bracket\n",
         b"open()", b"open()\r\nread()\r\n", b"=open()\n", b"a=b=c(\n", b"x" * 70000 + b"\nopen()\n",
         b"open()\n" + b"y" * 70000 + b"\n", b"(\n", b" (\n", b"#open(\nclose(\n"]


def test_call_set_matches_oracle_status():
    off = np.zeros(len(CASES) + 1, np.uint64)
    off[1:] = np.cumsum([len(c) for c in CASES])
    blob = np.frombuffer(b"".join(CASES), np.uint8)
    _, status = oracle.prog_scan(blob, off)
    for c, st in zip(CASES, status):
        fails = bool(int(st) & ~4)
        assert (pyref.call_set(c) is None) == fails, (c[:40], st)
