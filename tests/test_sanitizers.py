"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer.

oracle/sanitize_main.c drives every oracle entry point over seeded random inputs (empty and ragged
covers, the 0xFFFFFFFF sentinel, duplicates, disabled calls, over-long text lines); the multi-thread
forms (oracle_minimize_grouped_mt, oracle_novelty_mt) are checked equal to the serial ones and run
under TSan. Both binaries are built from source with gcc by oracle/Makefile here (CPU only)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def _build(target):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    r = subprocess.run(["make", "-C", ORACLE, target], capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr and "not supported" in r.stderr:
        pytest.skip("sanitizer runtime not available: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr[-2000:]


def _run(binary, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(ORACLE, "_san", binary), *args], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-1000:], r.stderr[-4000:])


def test_oracle_asan_ubsan():
    _build("asan")
    _run("oracle_asan")


def test_oracle_tsan_multithread():
    _build("tsan")
    _run("oracle_tsan", "mt")


def test_product_planners_asan_ubsan():
    # the product's host-side planners (syzkaller_amd/csrc/plan_host.cpp: plan_windows, slab_plan,
    # plan_items, gosort_segments, the multi-device plan) built with g++ under ASan + UBSan and driven over
    # random layouts by tests/planner_san.cpp
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    pkg = os.path.join(ROOT, "syzkaller_amd")
    r = subprocess.run(["make", "-C", pkg, "san"], capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr and "not supported" in r.stderr:
        pytest.skip("sanitizer runtime not available: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(pkg, "_san", "plan_san")], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.stdout[-1000:], r.stderr[-4000:])
