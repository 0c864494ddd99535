#!/usr/bin/env python3
"""Regenerate tests/golden/progtext_vectors.json.

Run in the build container only (the GPU box has no /root/reference):
    python tests/golden/make_golden_progtext.py [/root/reference]

* callset: the data of the table-driven TestCallSet (prog/encoding_test.go:22-75): program text,
  whether CallSet succeeds, the call names it returns.
* sha1: FIPS 180-2 known answers for sha1.Sum (hash/hash.go:13-15 wraps it): the standard's
  "abc", two-block and million-'a' messages, the empty message, plus messages around the padding
  boundaries (55/56/63/64/119/120 bytes). Digests computed with Python's hashlib here and written
  as data.
"""
import codecs
import hashlib
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = os.path.join(REF, "prog", "encoding_test.go")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "progtext_vectors.json")


def go_strings(s):
    return [codecs.decode(m, "unicode_escape") for m in re.findall(r'"((?:[^"\\]|\\.)*)"', s)]


def callset_cases(text):
    body = re.search(r"func TestCallSet\(t \*testing\.T\) \{(.*?)\n\}", text, re.S).group(1)
    table = body[body.index("}{") + 2: body.index("\n\t}\n")]
    cases = []
    for m in re.finditer(r"\{\s*((?:\"(?:[^\"\\]|\\.)*\"\s*\+?\s*)+),\s*(true|false),\s*\[\]string\{([^}]*)\},\s*\}",
                         table, re.S):
        prog = "".join(go_strings(m.group(1)))
        cases.append({"prog": prog, "ok": m.group(2) == "true", "calls": sorted(go_strings(m.group(3)))})
    return cases


def main():
    text = open(SRC).read()
    msgs = [b"", b"abc", b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq", b"a" * 1_000_000]
    msgs += [bytes((j * 7 + 3) & 0xFF for j in range(i)) for i in (55, 56, 63, 64, 119, 120)]
    out = {"source": "prog/encoding_test.go:22-75 TestCallSet; FIPS 180-2 SHA-1 examples",
           "callset": callset_cases(text),
           "sha1": [{"hex": m.hex() if len(m) < 1000 else None, "repeat_a": len(m) if len(m) >= 1000 else None,
                     "digest": hashlib.sha1(m).hexdigest()} for m in msgs]}
    assert len(out["callset"]) == 5, out["callset"]
    json.dump(out, open(OUT, "w"), indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
