"""ctypes binding of libdifacto_amd.so (the C-ABI declared in include/difacto_amd.h).

torch is imported BEFORE the library is opened: libdifacto_amd.so needs
``libamdhip64.so.7`` and, with torch already loaded, the dynamic loader resolves it to
torch's copy, so the library, torch tensors and torch streams share one HIP runtime.
There is no fallback: a missing library raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede CDLL, see module docstring)

LIB_PATH = os.environ.get("DFX_LIB_PATH") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libdifacto_amd.so")  # env: A/B builds

_lib = None

c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
vp = ctypes.c_void_p
i64p = ctypes.POINTER(ctypes.c_int64)
f64p = ctypes.POINTER(ctypes.c_double)


class DfxError(RuntimeError):
    pass


class Batch(ctypes.Structure):
    _fields_ = [("size", c_i64), ("nnz", c_i64), ("offset", vp), ("index", vp), ("value", vp),
                ("label", vp), ("weight", vp)]


class Progress(ctypes.Structure):
    _fields_ = [("nrows", ctypes.c_double), ("loss", ctypes.c_double), ("auc", ctypes.c_double),
                ("penalty", ctypes.c_double), ("nnz_w", ctypes.c_double)]


class HostBatch(ctypes.Structure):
    """dfx_host_batch: one pinned staging slot of a dfx_feeder"""
    _fields_ = [("offset", vp), ("index", vp), ("value", vp), ("label", vp), ("weight", vp),
                ("max_rows", c_i64), ("max_nnz", c_i64)]


# name -> (restype, argtypes)
_SIGS = {
    "dfx_last_error": (ctypes.c_char_p, []),
    "dfx_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(vp)]),
    "dfx_ctx_destroy": (ctypes.c_int, [vp]),
    "dfx_ctx_set_stream": (ctypes.c_int, [vp, vp]),
    "dfx_ctx_use_own_stream": (ctypes.c_int, [vp]),
    "dfx_ctx_set_input_stream": (ctypes.c_int, [vp, vp]),
    "dfx_prof_lanes": (ctypes.c_int, [vp, f64p]),
    "dfx_prof_counts": (ctypes.c_int, [vp, f64p]),
    "dfx_prof_host": (ctypes.c_int, [vp, f64p]),
    "dfx_ctx_vdim": (ctypes.c_int, [vp]),
    "dfx_sync": (ctypes.c_int, [vp]),
    "dfx_malloc": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.c_size_t]),
    "dfx_free": (ctypes.c_int, [vp, vp]),
    "dfx_memcpy": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, ctypes.c_int]),
    "dfx_reserve": (ctypes.c_int, [vp, c_i64, c_i64]),
    "dfx_localize": (ctypes.c_int, [vp, c_i64, c_i64, vp, vp, c_u64, vp, vp, vp, i64p]),
    "dfx_fm_predict": (ctypes.c_int, [vp, c_i64, c_i64, vp, vp, vp, vp, vp, vp, c_i64,
                                      ctypes.c_int, vp]),
    "dfx_fm_calcgrad": (ctypes.c_int, [vp, c_i64, c_i64, vp, vp, vp, vp, vp, vp, vp, vp, c_i64,
                                       ctypes.c_int, vp, vp]),
    "dfx_get_pos": (ctypes.c_int, [vp, c_i64, vp, vp, vp]),
    "dfx_evaluate": (ctypes.c_int, [vp, c_i64, vp, vp, f64p]),
    "dfx_auc": (ctypes.c_int, [vp, c_i64, vp, vp, f64p]),
    "dfx_store_pull": (ctypes.c_int, [vp, vp, c_i64, vp, vp, i64p]),
    "dfx_store_push": (ctypes.c_int, [vp, vp, c_i64, ctypes.c_int, vp, c_i64, vp]),
    "dfx_store_save": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int]),
    "dfx_store_load": (ctypes.c_int, [vp, ctypes.c_char_p]),
    "dfx_store_load_part": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]),
    "dfx_store_dump": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]),
    "dfx_store_stats": (ctypes.c_int, [vp, i64p, i64p, f64p, ctypes.POINTER(ctypes.c_uint32)]),
    "dfx_store_evaluate": (ctypes.c_int, [vp, f64p, i64p]),
    "dfx_store_reserve": (ctypes.c_int, [vp, c_i64, c_i64]),
    "dfx_store_entry": (ctypes.c_int, [vp, c_u64, vp, vp, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_int)]),
    "dfx_train_step": (ctypes.c_int, [vp, ctypes.POINTER(Batch), ctypes.c_int, ctypes.c_int,
                                      c_u64, vp]),
    "dfx_progress_read": (ctypes.c_int, [vp, ctypes.POINTER(Progress), ctypes.c_int]),
    "dfx_prof_enable": (ctypes.c_int, [vp, ctypes.c_int]),
    "dfx_prof_enable_marks": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_uint]),
    "dfx_prof_read": (ctypes.c_int, [vp, f64p, ctypes.POINTER(ctypes.c_int), f64p]),
    "dfx_feeder_create": (ctypes.c_int, [vp, c_i64, c_i64, ctypes.POINTER(vp)]),
    "dfx_feeder_destroy": (ctypes.c_int, [vp]),
    "dfx_feeder_slot": (ctypes.c_int, [vp, ctypes.POINTER(HostBatch)]),
    "dfx_feeder_submit": (ctypes.c_int, [vp, c_i64, c_i64, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(Batch)]),
    "dfx_feeder_consumed": (ctypes.c_int, [vp]),
    "dfx_feeder_create_slots": (ctypes.c_int, [vp, c_i64, c_i64, ctypes.c_int,
                                               ctypes.POINTER(vp)]),
    "dfx_feeder_consumed_back": (ctypes.c_int, [vp, ctypes.c_int]),
    "dfx_dist_record_floats": (ctypes.c_int, [vp]),
    "dfx_dist_localize": (ctypes.c_int, [vp, ctypes.POINTER(Batch), c_u64, ctypes.c_int,
                                         ctypes.c_int, vp, vp]),
    "dfx_dist_localize_wait": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, i64p, i64p]),
    "dfx_dist_owner_begin": (ctypes.c_int, [vp, ctypes.c_int, vp, i64p, ctypes.c_int, vp]),
    "dfx_dist_owner_pull": (ctypes.c_int, [vp, ctypes.c_int, vp]),
    "dfx_dist_fwd_bwd": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(Batch), vp,
                                        ctypes.c_int, vp, vp]),
    "dfx_dist_owner_push": (ctypes.c_int, [vp, ctypes.c_int, vp]),
    "dfx_dist_initv_local": (ctypes.c_int, [vp, ctypes.c_int, vp]),
    "dfx_dist_initv_draw": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int]),
    "dfx_dist_push_agg_sum": (ctypes.c_int, [vp]),
    "dfx_store_probe_stats": (ctypes.c_int, [vp, vp, vp, vp]),
    "dfx_dist_union": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp]),
    "dfx_dist_union_rows": (ctypes.c_int, [vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int,
                                           ctypes.c_int64, ctypes.c_int, ctypes.c_int, vp, vp]),
    "dfx_split_part_floats": (ctypes.c_int, [vp, ctypes.c_int]),
    "dfx_split_pxv_floats": (ctypes.c_int, [vp]),
    "dfx_split_partition": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(Batch), c_u64,
                                           ctypes.c_int, vp, vp, vp]),
    "dfx_split_partition_wait": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, i64p]),
    "dfx_split_owner_begin": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp, i64p, i64p,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int]),
    "dfx_ctx_lane_stream": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(vp)]),
    "dfx_ctx_set_lane_stream": (ctypes.c_int, [vp, ctypes.c_int, vp]),
    "dfx_split_owner_forward": (ctypes.c_int, [vp, ctypes.c_int, vp]),
    "dfx_split_owner_forward_rows": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_int, c_i64,
                                                    c_i64, c_i64]),
    "dfx_split_combine_rows": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(Batch), vp, c_i64,
                                              ctypes.c_int, vp, vp, c_i64, c_i64]),
    "dfx_split_combine": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(Batch), vp, c_i64,
                                         ctypes.c_int, vp, vp]),
    "dfx_split_owner_backward": (ctypes.c_int, [vp, ctypes.c_int, vp]),
    "dfx_split_owner_stats": (ctypes.c_int, [vp, ctypes.c_int, i64p, i64p, i64p]),
    "dfx_split_initv_local": (ctypes.c_int, [vp, ctypes.c_int, vp]),
    "dfx_split_initv_draw": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int]),
}

EXPORTED = tuple(_SIGS)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DfxError("libdifacto_amd.so is not built (%s); run `make` at the repo root"
                           % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        # an A/B run against an older build (DFX_LIB_PATH) may lack entry points it never calls
        lenient = bool(os.environ.get("DFX_LIB_PATH"))
        for name, (res, args) in _SIGS.items():
            if lenient and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().dfx_last_error()
        raise DfxError("libdifacto_amd: status %d: %s" % (rc, msg.decode() if msg else "?"))


# ---- libdfx_dist.so: the multi-GPU split driver (include/difacto_amd_dist.h) ----------------
# beside the core library it links (an A/B build's DFX_LIB_PATH brings its own driver: a
# driver from another directory would load a second, different copy of the core library)
DIST_PATH = os.path.join(os.path.dirname(os.path.abspath(LIB_PATH)), "libdfx_dist.so")
_dist = None
u32 = ctypes.c_uint32

_DIST_SIGS = {
    "dfx_dist_last_error": (ctypes.c_char_p, []),
    "dfx_dist_rccl_id_bytes": (ctypes.c_int, []),
    "dfx_dist_rccl_ids": (ctypes.c_int, [ctypes.c_int, vp]),
    "dfx_dist_rccl_comms": (ctypes.c_int, []),
    "dfx_split_store_set_slices": (ctypes.c_int, [vp, ctypes.c_int]),
    "dfx_split_store_allreduce_sum": (ctypes.c_int, [vp, f64p, ctypes.c_int]),
    "dfx_split_store_create_rccl": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, vp,
                                                   ctypes.c_int, ctypes.c_int, c_u64,
                                                   ctypes.POINTER(vp)]),
    "dfx_split_store_create_loopback": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int,
                                                       ctypes.c_int, c_u64, ctypes.POINTER(vp)]),
    "dfx_split_store_submit": (ctypes.c_int, [vp, ctypes.POINTER(Batch), ctypes.c_int,
                                              ctypes.c_int, ctypes.POINTER(vp)]),
    "dfx_split_store_flush": (ctypes.c_int, [vp]),
    "dfx_split_store_sync": (ctypes.c_int, [vp]),
    "dfx_split_store_throttle_seconds": (ctypes.c_int, [vp, f64p]),
    "dfx_split_store_set_marks": (ctypes.c_int, [vp, u32]),
    "dfx_split_store_take_marks": (ctypes.c_int, [vp, f64p, i64p]),
    "dfx_split_store_destroy": (ctypes.c_int, [vp]),
}

DIST_EXPORTED = tuple(_DIST_SIGS)


def dist_lib():
    """the split driver's library (opened after libdifacto_amd.so, which it links)"""
    global _dist
    if _dist is None:
        lib()
        if not os.path.exists(DIST_PATH):
            raise DfxError("libdfx_dist.so is not built (%s); run `make` at the repo root"
                           % DIST_PATH)
        L = ctypes.CDLL(DIST_PATH)
        for name, (res, args) in _DIST_SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _dist = L
    return _dist


def dist_check(rc):
    if rc != 0:
        msg = dist_lib().dfx_dist_last_error()
        raise DfxError("libdfx_dist: status %d: %s" % (rc, msg.decode() if msg else "?"))
