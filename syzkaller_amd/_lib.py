"""ctypes binding of libsyzgpu.so (the C ABI declared in include/syzgpu.h).

There is deliberately no CPU fallback: if the library or a gfx950 device is missing, every compute
call raises SyzGpuError.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SYZGPU_LIB") or os.path.join(_HERE, "libsyzgpu.so")

OK, EINVAL, ENODEV, ENOMEM, EHIP, EINTERNAL, ECAPACITY = range(7)
DIFFERENCE, SYMMETRIC_DIFFERENCE, UNION, INTERSECTION = range(4)

_c = ctypes
_vp = _c.c_void_p
_sz = _c.c_size_t

# name -> (restype, argtypes); every pointer is passed as a void* (numpy .ctypes.data / device ptr)
SIGNATURES = {
    "syzgpu_init": (_c.c_int, [_c.c_int]),
    "syzgpu_shutdown": (_c.c_int, []),
    "syzgpu_device_count": (_c.c_int, [_vp]),
    "syzgpu_last_error": (_sz, [_c.c_char_p, _sz]),
    "syzgpu_version": (_c.c_char_p, []),
    "syzgpu_canonicalize": (_c.c_int, [_vp, _sz, _vp]),
    "syzgpu_difference": (_c.c_int, [_vp, _sz, _vp, _sz, _vp, _sz, _vp]),
    "syzgpu_symmetric_difference": (_c.c_int, [_vp, _sz, _vp, _sz, _vp, _sz, _vp]),
    "syzgpu_union": (_c.c_int, [_vp, _sz, _vp, _sz, _vp, _sz, _vp]),
    "syzgpu_intersection": (_c.c_int, [_vp, _sz, _vp, _sz, _vp, _sz, _vp]),
    "syzgpu_minimize": (_c.c_int, [_vp, _vp, _sz, _vp, _vp]),
    "syzgpu_minimize_order": (_c.c_int, [_vp, _vp, _c.c_uint32, _vp]),
    "syzgpu_canonicalize_batch": (_c.c_int, [_vp, _vp, _sz, _vp]),
    "syzgpu_canonicalize_batch_dev": (_c.c_int, [_vp, _vp, _sz, _vp, _vp]),
    "syzgpu_setop_batch": (_c.c_int, [_c.c_int, _vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp]),
    "syzgpu_setop_batch_dev": (_c.c_int, [_c.c_int, _vp, _vp, _c.c_uint64, _vp, _vp, _c.c_uint64, _sz, _vp, _sz, _vp,
                                          _vp, _vp]),
    "syzgpu_minimize_grouped": (_c.c_int, [_vp, _vp, _vp, _sz, _c.c_uint32, _vp, _vp]),
    "syzgpu_novelty_batch": (_c.c_int, [_vp, _vp, _vp, _sz, _c.c_uint32, _vp, _vp, _vp, _sz, _vp, _vp, _sz,
                                        _vp]),
    "syzgpu_novelty_batch_dev": (_c.c_int, [_vp, _vp, _vp, _sz, _c.c_uint32, _vp, _vp, _sz, _vp, _sz, _sz, _vp,
                                            _vp, _sz, _vp, _vp]),
    "syzgpu_prog_scan": (_c.c_int, [_vp, _vp, _sz, _vp, _vp, _vp]),
    "syzgpu_prog_scan_dev": (_c.c_int, [_vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp]),
    "syzgpu_dynamic_prio": (_c.c_int, [_vp, _sz, _c.c_int32, _vp]),
    "syzgpu_call_cooccurrence": (_c.c_int, [_vp, _vp, _sz, _c.c_int32, _vp]),
    "syzgpu_call_cooccurrence_dev": (_c.c_int, [_vp, _vp, _sz, _c.c_int32, _vp, _vp]),
    "syzgpu_calculate_priorities": (_c.c_int, [_vp, _vp, _sz, _c.c_int32, _vp]),
    "syzgpu_static_priorities": (_c.c_int, [_vp, _sz, _c.c_int32, _vp]),
    "syzgpu_static_priorities_dev": (_c.c_int, [_vp, _sz, _c.c_int32, _vp, _vp]),
    "syzgpu_build_choice_table": (_c.c_int, [_vp, _vp, _c.c_int32, _vp, _vp]),
    "syzgpu_minimize_grouped_dev": (_c.c_int, [_vp, _vp, _vp, _vp, _sz, _c.c_uint32, _c.c_int32, _vp, _vp, _vp]),
    "syzgpu_minimize_grouped_ordered_dev": (_c.c_int, [_vp, _vp, _vp, _vp, _sz, _c.c_uint32, _c.c_int32, _vp, _vp,
                                                       _vp, _vp, _vp]),
    "syzgpu_mz_create": (_c.c_int, [_vp]),
    "syzgpu_mz_destroy": (_c.c_int, [_vp]),
    "syzgpu_mz_begin_dev": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _c.c_uint32, _vp, _vp, _vp]),
    "syzgpu_mz_export_sel_dev": (_c.c_int, [_vp, _vp, _vp, _c.c_uint32, _vp, _vp]),
    "syzgpu_mz_import_sel_dev": (_c.c_int, [_vp, _vp, _vp, _c.c_uint32, _vp, _vp]),
    "syzgpu_mz_end_dev": (_c.c_int, [_vp, _c.c_int32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "syzgpu_mz_end_prio_dev": (_c.c_int, [_vp, _c.c_int32, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp,
                                          _vp]),
    "syzgpu_mz_fetch": (_c.c_int, [_vp, _vp, _vp]),
    "syzgpu_mz_info": (_c.c_int, [_vp, _vp, _sz]),
    "syzgpu_mgz_create": (_c.c_int, [_vp, _c.c_int, _vp]),
    "syzgpu_mgz_destroy": (_c.c_int, [_vp]),
    "syzgpu_mgz_load": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _c.c_uint32, _c.c_uint32]),
    "syzgpu_mgz_minimize_prio": (_c.c_int, [_vp, _c.c_int32, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]),
    "syzgpu_mgz_info": (_c.c_int, [_vp, _vp, _sz]),
    "syzgpu_plan_parts": (_c.c_int, [_vp, _vp, _c.c_uint32, _c.c_int, _c.c_uint32, _vp, _vp]),
    "syzgpu_plan_split_bounds": (_c.c_int, [_vp, _vp, _vp, _sz, _c.c_uint32, _c.c_uint32, _vp]),
    "syzgpu_prio_choice_dev": (_c.c_int, [_vp, _vp, _c.c_int32, _vp, _vp, _vp, _vp, _vp]),
    "syzgpu_minimize_grouped_fetch": (_c.c_int, [_vp, _vp, _sz, _c.c_uint32]),
    "syzgpu_set_go_sort_leaf": (_c.c_int, [_c.c_int]),
    "syzgpu_go_sort_leaf": (_c.c_int, []),
    "syzgpu_corpus_create": (_c.c_int, [_vp, _vp, _vp, _vp, _sz, _c.c_uint32, _vp]),
    "syzgpu_corpus_create_dev": (_c.c_int, [_vp, _vp, _vp, _vp, _sz, _c.c_uint32, _vp, _vp]),
    "syzgpu_corpus_keep": (_c.c_int, [_vp, _vp, _sz]),
    "syzgpu_corpus_keep_dev": (_c.c_int, [_vp, _vp, _sz, _vp]),
    "syzgpu_corpus_minimize_ordered_dev": (_c.c_int, [_vp, _c.c_int32, _vp, _vp, _vp, _vp, _vp]),
    "syzgpu_corpus_minimize_keep_dev": (_c.c_int, [_vp, _c.c_int32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "syzgpu_corpus_reindex": (_c.c_int, [_vp, _vp]),
    "syzgpu_corpus_destroy": (_c.c_int, [_vp]),
    "syzgpu_corpus_append": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "syzgpu_corpus_append_dev": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    "syzgpu_corpus_new_inputs": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    "syzgpu_corpus_new_inputs_dev": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "syzgpu_corpus_cover_union": (_c.c_int, [_vp, _vp, _vp, _sz, _vp]),
    "syzgpu_corpus_minimize": (_c.c_int, [_vp, _vp, _vp]),
    "syzgpu_corpus_minimize_dev": (_c.c_int, [_vp, _c.c_int32, _vp, _vp, _vp]),
    "syzgpu_corpus_info": (_c.c_int, [_vp, _vp, _sz]),
    "syzgpu_corpus_set_parts": (_c.c_int, [_vp, _vp, _vp, _vp]),
    "syzgpu_corpus_minimize_begin_dev": (_c.c_int, [_vp, _vp]),
    "syzgpu_corpus_minimize_end_dev": (_c.c_int, [_vp, _c.c_int32, _vp, _vp, _vp]),
    "syzgpu_corpus_export_sel_dev": (_c.c_int, [_vp, _vp, _vp, _c.c_uint32, _vp, _vp]),
    "syzgpu_corpus_import_sel_dev": (_c.c_int, [_vp, _vp, _vp, _c.c_uint32, _vp, _vp]),
    "syzgpu_corpus_cover_stats": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "syzgpu_corpus_cover_stats_dev": (_c.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "syzgpu_corpus_cover": (_c.c_int, [_vp, _c.c_int64, _c.c_int, _vp, _sz, _vp]),
    "syzgpu_sigset_create": (_c.c_int, [_sz, _vp]),
    "syzgpu_sigset_destroy": (_c.c_int, [_vp]),
    "syzgpu_sigset_size": (_c.c_int, [_vp, _vp]),
    "syzgpu_sigset_clear": (_c.c_int, [_vp, _vp]),
    "syzgpu_sigset_insert": (_c.c_int, [_vp, _vp, _vp, _sz, _c.c_uint64, _vp, _vp]),
    "syzgpu_sigset_lookup": (_c.c_int, [_vp, _vp, _sz, _vp, _vp]),
    "syzgpu_sigset_erase": (_c.c_int, [_vp, _vp, _sz, _vp, _vp]),
    "syzgpu_sigset_export": (_c.c_int, [_vp, _vp, _vp, _sz, _vp]),
    "syzgpu_sigset_insert_dev": (_c.c_int, [_vp, _vp, _vp, _sz, _c.c_uint64, _vp, _vp, _vp]),
    "syzgpu_sigset_lookup_dev": (_c.c_int, [_vp, _vp, _sz, _vp, _vp, _vp]),
    "syzgpu_sigset_erase_dev": (_c.c_int, [_vp, _vp, _sz, _vp, _vp, _vp]),
    "syzgpu_profile_enable": (_c.c_int, [_c.c_int]),
    "syzgpu_profile_only": (_c.c_int, [_c.c_char_p]),
    "syzgpu_profile_read": (_sz, [_vp, _vp, _vp, _sz]),
    "syzgpu_debug_fail_grow": (_c.c_int, [_c.c_int]),
}


class SyzGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("syzgpu error %d: %s" % (code, msg))
        self.code = code


_LIB = None


def lib():
    """Load libsyzgpu.so (built in-tree by __graft_entry__.build()). Raises if absent."""
    global _LIB
    if _LIB is None:
        # PyTorch-ROCm ships its own libamdhip64.so.7. Importing it first makes this library's
        # NEEDED libamdhip64.so.7 resolve to that same copy (SONAME match), so the process has ONE
        # HIP runtime and torch tensors / streams are valid here. Loading us first would give two.
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(LIB_PATH):
            raise SyzGpuError(ENODEV, "libsyzgpu.so is not built (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def last_error():
    buf = ctypes.create_string_buffer(512)
    lib().syzgpu_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(rc):
    if rc != OK:
        raise SyzGpuError(rc, last_error())
    return rc


def ptr(a):
    """Address of a numpy array or a torch tensor (host or device), or None."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data
