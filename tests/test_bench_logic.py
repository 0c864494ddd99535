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
    assert any(pat in name and s == scope for pat, s in bench.ROCPROF_SCOPE)


def test_rocprof_scope_names_the_table_kinds_apart(tmp_path):
    for kernel, scope in (("void syz::k_slab<512, 32, false>(unsigned int const*)", "k_slab"),
                          ("syz::k_smin_direct(syz::PItem const*)", "k_pmin_direct"),
                          ("void syz::k_smin_hash<false>(syz::PItem const*)", "k_pmin_hash"),
                          ("void syz::k_smin_hash<true>(syz::PItem const*)", "k_pmin_packed")):
        f = tmp_path / "stats.csv"
        f.write_text('"Name","Calls","TotalDurationNs"\n"%s",1,10\n' % kernel)
        assert bench.rocprof_top(str(f))[0] == scope
    f.write_text('"Name","Calls","TotalDurationNs"\n"void rocprim::scan(int)",1,10\n')
    assert bench.rocprof_top(str(f)) is None
    assert bench.rocprof_top(str(tmp_path / "missing.csv")) is None


def test_dominant_kernel_follows_the_summary_else_the_serialized_pass(monkeypatch, tmp_path):
    kern = {"k_slab": {"ms": 1.3, "bytes": 3}, "k_pmin_direct": {"ms": 1.4, "bytes": 2},
            "gosort_level": {"ms": 9.0, "bytes": 0}, "m_big": {"ms": 5.0, "bytes": 7}}
    f = tmp_path / "stats.csv"
    f.write_text('"Name","Calls","TotalDurationNs"\n"void syz::k_slab<512, 32, false>(int)",1,10\n')
    monkeypatch.setattr(bench, "ROCPROF_STATS", str(f))
    monkeypatch.setattr(bench.rocprof_top, "__defaults__", (str(f), bench.PROFILED_WORKLOAD))
    assert bench.dominant_kernel(kern) == "k_slab"
    monkeypatch.setattr(bench.rocprof_top, "__defaults__", (str(tmp_path / "missing.csv"), bench.PROFILED_WORKLOAD))
    # phase scopes (no k_ prefix) and kernels without a byte model never name the roofline
    assert bench.dominant_kernel(kern) == "k_pmin_direct"


def _args(**kw):
    import types
    d = dict(progs_per_gpu=1_000_000, npcs=2_000_000, ngroups=289, calls=1159, seed=0x5EED0004, total_progs=0,
             emulate="")
    d.update(kw)
    return types.SimpleNamespace(**d)


def test_profiles_apply_only_to_the_workload_they_were_taken_on(monkeypatch, tmp_path):
    """A config-1 or config-2 line must not carry config 4's PMC traffic or rocprof selection."""
    assert bench.workload_key(_args(), 1) == bench.PROFILED_WORKLOAD
    small = bench.workload_key(_args(progs_per_gpu=10_000, npcs=50_000), 1)
    assert small != bench.PROFILED_WORKLOAD
    assert bench.workload_key(_args(), 8) != bench.PROFILED_WORKLOAD
    assert bench.workload_key(_args(total_progs=1_000_000), 1) != bench.PROFILED_WORKLOAD
    assert bench.rocprof_top(workload=small) is None
    f = tmp_path / "pmc.json"
    f.write_text('{"workload": "config4-1M", "kernels": {"k_slab": {"hbm_bytes_per_launch": 123}}}')
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    os.makedirs(tmp_path / "profiles")
    os.replace(f, tmp_path / "profiles" / "pmc_traffic.json")
    ev = {"k_slab": {"ms": 2.0, "launches": 2, "bytes": 2_000_000}}
    assert bench.roofline("k_slab", ev, workload=bench.PROFILED_WORKLOAD)["traffic"] == 123
    assert bench.roofline("k_slab", ev, workload=small)["traffic"] is None
