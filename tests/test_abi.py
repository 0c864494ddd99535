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


def test_go_sort_leaf_setter_needs_no_device():
    from syzkaller_amd import _lib
    L = _lib.lib()
    assert L.syzgpu_go_sort_leaf() == 12
    assert L.syzgpu_set_go_sort_leaf(9) == _lib.EINVAL
    assert L.syzgpu_go_sort_leaf() == 12
    try:
        assert L.syzgpu_set_go_sort_leaf(7) == 0
        assert L.syzgpu_go_sort_leaf() == 7
    finally:
        assert L.syzgpu_set_go_sort_leaf(12) == 0


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


# The runtime options the production library reads (INTEGRATION.md "Environment"): each selects a
# strategy or a schedule and none changes a result (the -m gpu tests run the alternatives against the
# oracle). Developer switches (timing-only modes, A/B variants) are read only in the variant / dbg
# builds (dev_env, syzkaller_amd/csrc/common.hpp).
RUNTIME_OPTIONS = {
    "SYZGPU_LANES", "SYZGPU_NOVELTY", "SYZGPU_NO_INC_INDEX", "SYZGPU_NWH_SORT", "SYZGPU_PM_SERIAL",
    "SYZGPU_PM_SPEC", "SYZGPU_CHUNK_VECS", "SYZGPU_CO_FORM", "SYZGPU_CO_KS", "SYZGPU_GR_PERSIST",
    "SYZGPU_GR_PGRID",
}


def test_production_library_reads_only_documented_options():
    data = open(os.path.join(ROOT, "syzkaller_amd", "libsyzgpu.so"), "rb").read()
    names = set(m.decode() for m in re.findall(rb"SYZGPU_[A-Z0-9_]+", data))
    assert names <= RUNTIME_OPTIONS, sorted(names - RUNTIME_OPTIONS)
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert all(n in doc for n in RUNTIME_OPTIONS), [n for n in RUNTIME_OPTIONS if n not in doc]
    # the wrong-result timing switches in particular
    for n in ("SYZGPU_NW_DBG", "SYZGPU_NWH_DBG", "SYZGPU_PM_PSPLIT", "SYZGPU_SO_TWOPASS"):
        assert n.encode() not in data, n


def test_every_getenv_in_sources_is_documented_or_dev_only():
    src = os.path.join(ROOT, "syzkaller_amd", "csrc")
    seen = set()
    for f in os.listdir(src):
        text = open(os.path.join(src, f), errors="ignore").read()
        seen |= set(re.findall(r'\bgetenv\("(SYZGPU_[A-Z0-9_]+)"\)', text))
    assert seen <= RUNTIME_OPTIONS, sorted(seen - RUNTIME_OPTIONS)
