"""CPU-side checks of the drop-in boundary: the C-ABI libraries load and export every symbol the
headers in include/ declare. No compute call is made (there is no GPU in the build container)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(syzgpu_\w+)\s*\(", text)))


def _exported(path):
    lib = ctypes.CDLL(path)
    return lib


@pytest.mark.parametrize("header,libpath", [
    ("syzgpu.h", "syzkaller_amd/libsyzgpu.so"),
    ("syzgpu_synth.h", "syzkaller_amd/libsyzsynth.so"),
])
def test_library_exports_every_declared_symbol(header, libpath):
    path = os.path.join(ROOT, libpath)
    assert os.path.exists(path), "build first: python -c 'import __graft_entry__ as g; g.build()'"
    lib = _exported(path)
    names = _declared(header)
    assert len(names) >= 3
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_abi():
    from syzkaller_amd import _lib
    declared = set(_declared("syzgpu.h"))
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_library_reports_version_without_device():
    from syzkaller_amd import _lib
    assert _lib.lib().syzgpu_version().startswith(b"syzgpu")


def test_no_oracle_in_product_package():
    # the product package must never import or link the CPU oracle
    pkg = os.path.join(ROOT, "syzkaller_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".hpp", ".h")):
                text = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "oracle" not in text.lower(), os.path.join(dirpath, f)


def test_synth_is_deterministic_and_canonical():
    from syzkaller_amd import synth
    a = synth.corpus(42, 500, 17, 4000, nthreads=1)
    b = synth.corpus(42, 500, 17, 4000, nthreads=4)
    assert np.array_equal(a.pcs, b.pcs) and np.array_equal(a.off, b.off) and np.array_equal(a.group, b.group)
    for i in range(a.n):
        c = a.cover(i)
        assert c.size >= 1 and np.all(c[1:] > c[:-1])
    assert a.prog_len.min() >= 1 and a.prog_len.max() <= 40
