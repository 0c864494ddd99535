"""Parity of the program-text pass (syzgpu_prog_scan: Deserialize's len(p.Calls), CallSet's checks,
hash.Hash) on the MI355X against the pinned oracle (oracle_prog_scan, oracle_sha1): TestCallSet's table,
the FIPS SHA-1 examples, the bufio line rules (CRLF, '#', empty lines, unterminated last line,
64 KiB lines), every padding boundary, arbitrary alignments, empty programs, and a synthetic corpus;
the device entry with a selection mask."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import hash as shash  # noqa: E402
from syzkaller_amd import prog as sprog  # noqa: E402
from syzkaller_amd import synth  # noqa: E402

pytestmark = pytest.mark.gpu


def _check(progs=None, data=None, off=None):
    if progs is not None:
        data, off = sprog._blob([p if isinstance(p, bytes) else p.encode() for p in progs], None)
    nc, st, sg = sprog.ProgScan(data, off)
    wnc, wst = oracle.prog_scan(data, off)
    assert np.array_equal(nc, wnc)
    assert np.array_equal(st, wst)
    assert np.array_equal(sg, oracle.sha1(data, off))
    # the lane-per-program count (taken when no CallSet checks are asked for), alone and with SHA-1
    assert np.array_equal(sprog.CallCounts(data, off), wnc)
    nc2, st2, sg2 = sprog.ProgScan(data, off, status=False)
    assert st2 is None and np.array_equal(nc2, wnc) and np.array_equal(sg2, sg)
    return nc, st, sg, data, off


def test_callset_table_and_sha1_known_answers():
    with open(os.path.join(ROOT, "tests", "golden", "progtext_vectors.json")) as f:
        v = json.load(f)
    nc, st = _check([c["prog"] for c in v["callset"]])[:2]
    assert [s == 0 for s in st] == [c["ok"] for c in v["callset"]]
    msgs = [bytes.fromhex(x["hex"]) if x["hex"] is not None else b"a" * x["repeat_a"] for x in v["sha1"]]
    sg = _check(msgs)[2]
    assert [bytes(s).hex() for s in sg] == [x["digest"] for x in v["sha1"]]
    assert shash.Hash(b"abc").String() == "a9993e364706816aba3e25717850c26c9cd0d89d"
    assert shash.FromString(shash.Hash(b"abc").String()) == shash.Hash(b"abc")


def test_line_rules_and_long_lines():
    S = "x" * 65535
    _check(["a()\r\nb()\r\n", "\r\n#c\r\n\r", "a(\n", "()", "r0 = =x()", "r0 =\t()", "a()\n" + S, "a()\n" + S + "x",
            S + "x\n", "#only\n\n", "f(", "   (", "=(", "x=  y()", "a()\n" + S + "xx\nb()\n", "", "\n", "\r"])


def test_every_length_and_alignment():
    rnd = np.random.default_rng(1)
    alphabet = np.frombuffer(b"abc()=# \r\n\n\n$,0x", np.uint8)
    progs = [rnd.choice(alphabet, size=k).tobytes() for k in range(0, 400)]
    progs += [rnd.choice(alphabet, size=int(rnd.integers(0, 3000))).tobytes() for _ in range(300)]
    progs += [rnd.choice(np.frombuffer(b"a\r\n#", np.uint8), size=int(rnd.integers(60, 200))).tobytes() for _ in range(300)]
    rnd.shuffle(progs)
    _check(progs)


def test_count_only_mode_matches():
    # ncalls without status runs the count-only kernel (no CallSet scans); long lines go serial
    S = "x" * 65535
    progs = ["a()\n" + S + "x\nb()\n", "a()\r\n\r\n#x\nb(", "", "\n\n", "r0 = f()\n" * 300] * 3
    data, off = sprog._blob([p.encode() for p in progs], None)
    assert np.array_equal(sprog.CallCounts(data, off), oracle.prog_scan(data, off)[0])


def test_synthetic_corpus():
    c = synth.corpus(0x5EED0021, 20_000, 97, 40_000)
    d, o = synth.prog_text(0x77, c.prog_len)
    nc, st = _check(data=d, off=o)[:2]
    assert np.array_equal(nc, c.prog_len.astype(np.uint32)) and not st.any()


def test_device_entry_selection():
    import torch
    dev = torch.device("cuda:0")
    c = synth.corpus(0x5EED0022, 5_000, 31, 20_000)
    d, o = synth.prog_text(0x78, c.prog_len)
    sel = (np.random.default_rng(2).random(c.n) < 0.4).astype(np.uint8)
    td = torch.from_numpy(d.copy()).to(dev)
    to = torch.from_numpy(o.view(np.int64)).to(dev)
    ts = torch.from_numpy(sel).to(dev)
    nc = torch.full((c.n,), 0xDEAD, dtype=torch.int32, device=dev)
    st = torch.full((c.n,), 0x7F, dtype=torch.uint8, device=dev)
    sg = torch.zeros((c.n, 20), dtype=torch.uint8, device=dev)
    sprog.ProgScanDev(td, to, c.n, ts, nc, st, sg, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    wnc, wst = oracle.prog_scan(d, o)
    wsg = oracle.sha1(d, o)
    m = sel.astype(bool)
    assert np.array_equal(nc.cpu().numpy()[m], wnc[m]) and (nc.cpu().numpy()[~m] == 0xDEAD).all()
    assert np.array_equal(st.cpu().numpy()[m], wst[m]) and (st.cpu().numpy()[~m] == 0x7F).all()
    assert np.array_equal(sg.cpu().numpy()[m], wsg[m]) and not sg.cpu().numpy()[~m].any()
