"""Host logic of bench.py's roofline: the roofline kernel is the top row of the committed rocprofv3
summary of the bench command (mapped to the library's profiling scope around that kernel), and
without that file the byte-modelled kernel scope with the most time in the serialized pass."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_rocprof_top_of_the_committed_summary():
    top = bench.rocprof_top()
    assert top is not None
    scope, name = top
    assert scope in dict((s, s) for _, s in bench.ROCPROF_SCOPE)
    assert name.split("(")[0].split("::")[-1].startswith(scope.replace("_count", ""))


def test_rocprof_scope_names_the_count_and_scatter_apart(tmp_path):
    for kernel, scope in (("void syz::k_region<512, 40, false, false>(unsigned int const*)", "k_region"),
                          ("void syz::k_region<512, 40, false, true>(unsigned int const*)", "k_region_count"),
                          ("syz::k_pmin_direct(syz::PItem const*)", "k_pmin_direct"),
                          ("void syz::k_pmin_hash<true>(syz::PItem const*)", "k_pmin_packed")):
        f = tmp_path / "stats.csv"
        f.write_text('"Name","Calls","TotalDurationNs"\n"%s",1,10\n' % kernel)
        assert bench.rocprof_top(str(f))[0] == scope
    f.write_text('"Name","Calls","TotalDurationNs"\n"void rocprim::scan(int)",1,10\n')
    assert bench.rocprof_top(str(f)) is None
    assert bench.rocprof_top(str(tmp_path / "missing.csv")) is None


def test_dominant_kernel_follows_the_summary_else_the_serialized_pass(monkeypatch, tmp_path):
    kern = {"k_region": {"ms": 1.3, "bytes": 3}, "k_pmin_direct": {"ms": 1.4, "bytes": 2},
            "gosort_level": {"ms": 9.0, "bytes": 0}, "m_big": {"ms": 5.0, "bytes": 7}}
    f = tmp_path / "stats.csv"
    f.write_text('"Name","Calls","TotalDurationNs"\n"void syz::k_region<512, 40, false, false>(int)",1,10\n')
    monkeypatch.setattr(bench, "ROCPROF_STATS", str(f))
    monkeypatch.setattr(bench.rocprof_top, "__defaults__", (str(f),))
    assert bench.dominant_kernel(kern) == "k_region"
    monkeypatch.setattr(bench.rocprof_top, "__defaults__", (str(tmp_path / "missing.csv"),))
    # phase scopes (no k_ prefix) and kernels without a byte model never name the roofline
    assert bench.dominant_kernel(kern) == "k_pmin_direct"
