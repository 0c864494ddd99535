"""Pin the oracle's program-text restatement (oracle_prog_scan, oracle_sha1) before it checks the GPU:
TestCallSet's table (prog/encoding_test.go:22-75) and the FIPS 180-2 SHA-1 examples
(tests/golden/progtext_vectors.json), hashlib on random messages, and the synthetic text generator
(its programs have exactly prog_len calls)."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import prog as sprog  # noqa: E402


@pytest.fixture(scope="module")
def vectors():
    with open(os.path.join(ROOT, "tests", "golden", "progtext_vectors.json")) as f:
        return json.load(f)


def blob(progs):
    data, off = sprog._blob([p if isinstance(p, bytes) else p.encode() for p in progs], None)
    return data, off


def callset_names(text):
    """CallSet's returned names (encoding.go:522-551) for an ok program, transliterated."""
    out = set()
    for ln in text.split("\n"):
        ln = ln[:-1] if ln.endswith("\r") else ln
        if not ln or ln[0] == "#":
            continue
        call = ln[: ln.index("(")]
        if "=" in call:
            call = call[call.index("=") + 1:].lstrip(" ")
        out.add(call)
    return sorted(out)


def test_callset_table(vectors):
    cases = vectors["callset"]
    d, o = blob([c["prog"] for c in cases])
    nc, st = oracle.prog_scan(d, o)
    for c, n, s in zip(cases, nc, st):
        assert (s == 0) == c["ok"], c
        if c["ok"]:
            assert callset_names(c["prog"]) == c["calls"]
            assert n >= len(c["calls"])
    assert list(nc) == [0, 1, 1, 1, 4]  # Deserialize's len(p.Calls) of each text


def test_sha1_known_answers(vectors):
    for v in vectors["sha1"]:
        m = bytes.fromhex(v["hex"]) if v["hex"] is not None else b"a" * v["repeat_a"]
        d, o = blob([m])
        assert bytes(oracle.sha1(d, o)[0]).hex() == v["digest"]


def test_sha1_random_vs_hashlib():
    rnd = np.random.default_rng(5)
    msgs = [rnd.integers(0, 256, size=int(k), dtype=np.uint8).tobytes() for k in range(0, 300)]
    d, o = blob(msgs)
    sig = oracle.sha1(d, o)
    for m, s in zip(msgs, sig):
        assert bytes(s) == hashlib.sha1(m).digest()


def test_line_rules():
    S = "x" * 65535
    progs = ["a()\r\nb()\r\n", "\r\n#c\r\n\r", "a(\n", "()", "r0 = =x()", "r0 =\t()", "a()\n" + S, "a()\n" + S + "x",
             S + "x\n", "#only\n\n", "f(", "   (", "=(", "x=  y()"]
    d, o = blob(progs)
    nc, st = oracle.prog_scan(d, o)
    # CallSet and Deserialize both stop at a line of >= 64 KiB (bufio.ErrTooLong): CallSet keeps the
    # calls before it, Deserialize returns a nil program; nothing after it is counted
    assert list(nc) == [2, 0, 1, 1, 1, 1, 2, 1, 0, 0, 1, 1, 1, 1]
    assert list(st) == [0, 8, 0, 2, 0, 0, 1, 4, 12, 8, 0, 0, 2, 0]


def test_synth_text_has_prog_len_calls():
    from syzkaller_amd import synth
    c = synth.corpus(9, 3000, 31, 20_000)
    d, o = synth.prog_text(11, c.prog_len)
    nc, st = oracle.prog_scan(d, o)
    assert np.array_equal(nc, c.prog_len.astype(np.uint32))
    assert not st.any()
