#!/usr/bin/env python3
"""Regenerate tests/golden/cover_test_vectors.json from the reference's own known-answer tables.

Run in the build container only (the GPU box has no /root/reference):
    python tests/golden/make_golden.py [/root/reference]

It extracts the *data* of the table-driven tests in cover/cover_test.go —
TestCanonicalize (:60-66), TestDifference (:68-76), TestSymmetricDifference (:78-85),
TestUnion (:87-94), TestIntersection (:96-102) and TestMinimize (:104-168) — and applies the
harness rules of runTest (:31-58): symmetric ops also get the swapped cases (:32-36) and every table
gets the empty/empty case (:37). Only inputs and expected outputs are written.
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = os.path.join(REF, "cover", "cover_test.go")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cover_test_vectors.json")


def covers(s):
    return [[int(x) for x in c.split(",") if x.strip()] for c in re.findall(r"Cover\{([^}]*)\}", s)]


def table(text, fn, symmetric):
    m = re.search(r"func %s\(t \*testing\.T\) \{(.*?)\n\}" % fn, text, re.S)
    body = m.group(1)
    rows = []
    for line in body.splitlines():
        line = line.strip()
        if line.startswith("{Cover"):
            v0, v1, r = covers(line)
            rows.append({"v0": v0, "v1": v1, "r": r})
    if symmetric:
        rows += [{"v0": t["v1"], "v1": t["v0"], "r": t["r"]} for t in list(rows)]
    rows.append({"v0": [], "v1": [], "r": []})
    return rows


def minimize_table(text):
    m = re.search(r"func TestMinimize\(t \*testing\.T\) \{(.*?)\n\}", text, re.S)
    body = m.group(1)
    cases = []
    for block in re.findall(r"\[\]Cover\{(.*?)\},\s*\[\]int\{([^}]*)\}", body, re.S):
        inp = [[int(x) for x in c.split(",") if x.strip()] for c in re.findall(r"\{([^{}]*)\}", block[0])]
        out = [int(x) for x in block[1].split(",") if x.strip()]
        cases.append({"inp": inp, "out": out})
    return cases


def main():
    text = open(SRC).read()
    gold = {
        "source": "cover/cover_test.go (tables at :60-168, runTest rules :31-58)",
        "canonicalize": table(text, "TestCanonicalize", False),
        "difference": table(text, "TestDifference", False),
        "symmetric_difference": table(text, "TestSymmetricDifference", True),
        "union": table(text, "TestUnion", True),
        "intersection": table(text, "TestIntersection", True),
        "minimize": minimize_table(text),
    }
    assert len(gold["minimize"]) == 5, gold["minimize"]
    with open(OUT, "w") as f:
        json.dump(gold, f, indent=1)
    print("wrote", OUT, {k: len(v) for k, v in gold.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
