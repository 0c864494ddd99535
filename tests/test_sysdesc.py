"""calcStaticPriorities' host half (syzkaller_amd/sysdesc.py: sysparser + the usage walk over the types
sysgen generates) and its CPU oracle (oracle_static_priorities), on CPU.

The reference has no test for calcStaticPriorities (prog/ has no prio_test.go), so the parser and the
walk are checked against hand-derived expectations on small descriptions that exercise every rule of
prio.go:53-104 and every sysgen construct the walk sees, and the oracle's Go-form loop against a
literal Python transliteration of prio.go:40-135. The bundled matrix must equal a fresh parse of the
reference's sys/*.txt whenever the reference is present (this container; not the GPU box).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from syzkaller_amd import sysdesc  # noqa: E402

F = np.float32

DESC = """\
# a comment
include <linux/fs.h>
define FOO	1 + 2

resource fd[int32]: 0xffffffffffffffff, AT_FDCWD
resource sock[fd]
resource sock_in[sock]
resource pid[int32]: 0
resource key[int64]

open(file filename, flags flags[open_flags], mode flags[open_mode]) fd
close(fd fd)
socket$in(domain const[2], type const[1, int32], proto int32) sock_in
bind$in(fd sock_in, addr ptr[in, sockaddr_in], len len[addr])
sendmsg(fd sock, msg ptr[in, msghdr], f flags[send_flags])
kill(pid pid, sig signalno)
mmap(addr vma, len len[addr], prot flags[open_mode], fd fd[opt], off fileoff)
keys(k ptr[out, array[key]], n len[k], s ptr[in, string[fsname]], t ptr[in, string["x"]])
blobs(a ptr[in, array[int8]], b buffer[in], c ptr[in, array[array[int8], 4]], d ptr[in, array[int32, 1:4]])
nested(u ptr[inout, opts, opt], r ptr[in, rec])

open_flags = O_RDONLY, O_RDWR
open_mode = S_IRUSR
send_flags = MSG_OOB
fsname = "ext4", "btrfs"

sockaddr_in {
	family	const[2, int16]
	port	int16be
	pad	array[int8, 8]
}

msghdr {
	addr	ptr[in, sockaddr_in, opt]
	iov	ptr[in, array[iovec]]
	pid	pid
}

iovec {
	base	buffer[in]
	len	len[base, intptr]
}

opts [
	a	sockaddr_in
	b	int32
	c	ptr[in, array[sock, 2]]
] [varlen]

rec {
	self	ptr[in, rec, opt]
	f	filename
} [packed]
"""


def usage_of(text):
    u = sysdesc.usage(sysdesc.parse(text))
    return u, {c: {k: float(u.weights[i, j]) for i, k in enumerate(u.keys) if u.weights[i, j]}
               for j, c in enumerate(u.calls)}


def test_calls_sorted_by_name_give_ids():
    u, _ = usage_of(DESC)
    assert u.calls == sorted(u.calls)
    assert u.calls[:3] == ["bind$in", "blobs", "close"]


def test_usage_rules():
    _, m = usage_of(DESC)
    f02, f01 = float(F(0.2)), float(F(0.1))
    # resources: kind chain from the root, 0.2 for prefixes and 1.0 for the full chain (prio.go:61-69);
    # the return type counts (decl.go:497-499)
    assert m["open"] == {"filename": 1.0, "res-fd": 1.0}
    assert m["close"] == {"res-fd": 1.0}
    assert m["socket$in"] == {"res-fd": f02, "res-fd-sock": f02, "res-fd-sock-sock_in": 1.0}
    # pointers to structs, the struct's fields, nested pointers; pid at 0.1 (prio.go:56-59)
    assert m["bind$in"] == {"res-fd": f02, "res-fd-sock": f02, "res-fd-sock-sock_in": 1.0, "ptrto-sockaddr_in": 1.0}
    assert m["sendmsg"] == {"res-fd": f02, "res-fd-sock": 1.0, "ptrto-msghdr": 1.0, "ptrto-sockaddr_in": 1.0,
                            "ptrto-iovec": 1.0, "respid": f01}
    assert m["kill"] == {"respid": f01, "signalno": 1.0}
    assert m["mmap"] == {"vma": 0.5, "res-fd": 1.0}
    # pointer to an array of a non-struct element: "ptrto-" + "" (the element's TypeName is empty);
    # a string from a string-flag set: str-<set> at 0.2; a literal string has no sub-kind
    assert m["keys"] == {"ptrto-": 1.0, "res-key": 1.0, "str-fsname": f02}
    # array[int8] is a blob buffer (sysgen.go:600-609): no ptrto key; an array of an unnamed type is
    # an ArrayType whose element has no name
    assert m["blobs"] == {"ptrto-": 1.0}
    # union options (a struct option is walked, but only a pointer makes a ptrto key), a recursive
    # struct (visited once), filename inside it
    assert m["nested"] == {"ptrto-opts": 1.0, "ptrto-": 1.0, "res-fd": f02,
                           "res-fd-sock": 1.0, "ptrto-rec": 1.0, "filename": 1.0}


def test_max_weight_per_key():
    # noteUsage keeps the largest weight (prio.go:48-50): sock as a prefix (0.2) and as a full chain (1.0)
    _, m = usage_of(DESC + "both(a sock_in, b sock)\n")
    assert m["both"]["res-fd-sock"] == 1.0 and m["both"]["res-fd"] == float(F(0.2))


@pytest.mark.parametrize("bad", [
    "x(a nosuchtype)\n",
    "x(a int32)\nx(b int32)\n",
    "x(a int32, a int32)\n",
    "s {\n\tf int32\n}\ns {\n\tg int32\n}\n",
    "u [\n\tf int32\n]\n",
    "s {\n\tf int32\n} [bogus]\n",
    "resource r[nosuch]\nx(a r)\n",
    "x(a string[nosuchflags])\n",
    "x(a salg_type)\n",
    "x(a int32) trailing junk(\n",
    "x(a flags[nosuchflags])\n",
])
def test_rejected_descriptions(bad):
    with pytest.raises(sysdesc.DescError):
        sysdesc.usage(sysdesc.parse(bad))


def test_parser_details():
    d = sysdesc.parse(DESC)
    assert d.includes == ["linux/fs.h"]
    assert d.defines == {"FOO": "(1+2)"}  # p.Parse(ch) skips the blanks after every character
    assert d.resources["fd"] == ("int32", ["0xffffffffffffffff", "AT_FDCWD"])
    assert d.strflags["fsname"] == ["ext4", "btrfs"]
    # nested bracketed types become unnamed types; const[...] and array[..., n] add fake flags
    assert any(v == ["array", "int8"] for v in d.unnamed.values())
    assert any(k.startswith("const_flag_") for k in d.flags)
    flds, is_union = d.structs["opts"]
    assert is_union and [f[0] for f in flds] == ["a", "b", "c"]


@pytest.mark.skipif(not os.path.isdir("/root/reference/sys"), reason="reference sys/ not present")
def test_bundled_matrix_is_the_reference_parse():
    fresh = sysdesc.usage(sysdesc.load_dir("/root/reference/sys"))
    b = sysdesc.bundled()
    assert b.calls == fresh.calls and b.keys == fresh.keys
    assert np.array_equal(b.weights, fresh.weights)


def test_bundled_matrix_shape():
    b = sysdesc.bundled()
    assert b.C == 1159 == len(set(b.calls))  # BASELINE.json configs[3]: ~1.5k calls (1159 here)
    assert sorted(set(b.weights[b.weights > 0].tolist())) == [float(F(x)) for x in (0.1, 0.2, 0.5, 1.0)]


def _go_static(uses, order):
    """prio.go:40-135 transliterated: map iteration in `order`, float32 arithmetic."""
    nk, C = uses.shape
    pr = np.zeros((C, C), F)
    for k in order:
        calls = [(c, uses[k, c]) for c in range(C) if uses[k, c] != 0]
        for c0, w0 in calls:
            for c1, w1 in calls:
                if c0 == c1:
                    continue
                pr[c0, c1] = F(pr[c0, c1] + F(w0 * w1))
    for c0 in range(C):
        mx = F(0)
        for p in pr[c0]:
            if mx < p:
                mx = p
        pr[c0, c0] = mx
    return oracle.normalize_prio(pr)


def _random_uses(rnd, nk, C, vals=(0.1, 0.2, 0.5, 1.0), density=0.05):
    w = np.zeros((nk, C), F)
    mask = rnd.random((nk, C)) < density
    w[mask] = rnd.choice(np.array(vals, F), size=int(mask.sum()))
    return w


@pytest.mark.parametrize("seed", range(3))
def test_oracle_go_form_matches_transliteration(seed):
    rnd = np.random.default_rng(seed)
    w = _random_uses(rnd, 40, 30, density=0.2)
    order = rnd.permutation(40)
    got = oracle.static_priorities(w, order)
    assert np.array_equal(got.view(np.uint32), _go_static(w, order).view(np.uint32))


def test_oracle_exact_form_within_go_rounding():
    # every map order lands within float32 rounding of the exact sum: 1e-6 relative after
    # normalisation (the north star's tolerance for normalized priorities)
    rnd = np.random.default_rng(4)
    for w in (_random_uses(rnd, 120, 90, density=0.3), sysdesc.bundled().weights):
        ex = oracle.static_priorities(w, exact=True)
        for _ in range(3):
            go = oracle.static_priorities(w, rnd.permutation(w.shape[0]))
            assert np.max(np.abs(go.astype(np.float64) - ex) / np.abs(ex)) < 1e-6
