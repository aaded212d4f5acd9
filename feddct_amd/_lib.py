"""ctypes binding of libfedagg.so (include/fedagg.h).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, importing this module raises.  Build it with
``python -c "import __graft_entry__ as g; g.build()"`` (or feddct_amd.build).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

# torch first: libfedagg.so must bind to the SAME HIP runtime as PyTorch-ROCm
# (torch ships its own libamdhip64.so.7).  Loaded the other way round the
# process ends up with two runtimes and torch's stream handles / device
# pointers are not valid in ours ("no ROCm-capable device").
import torch  # noqa: F401  (load order)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfedagg.so")

FA_OK = 0
FA_E_INVAL = -1
FA_E_RANGE = -2
FA_E_ALIGN = -3
FA_E_HIP = -4
FA_E_NOMEM = -5
FA_MAX_CLIENTS = 65536
FA_INLINE_CLIENTS = 128
FA_F_BCAST = 1
FA_F_SUM_ONLY = 2
FA_F_BCAST_ONLY = 4
FA_PROX_ACCUMULATE = 1
FA_PROX_ACCUMULATE_A = 2
FA_PROX_ACCUMULATE_B = 4
FA_PLAN_GAPS_ARE_PADDING = 1
FA_PLAN_TUNE_BATCH8 = 4
FA_PLAN_TUNE_BATCH16 = 8
FA_PLAN_TUNE_NO_BALANCE = 0x10000000
# every other plan flag bit is refused by the library since r05 (fedagg.h)
FA_PLAN_FLAGS_KNOWN = FA_PLAN_GAPS_ARE_PADDING | FA_PLAN_TUNE_BATCH8 | FA_PLAN_TUNE_BATCH16 \
    | FA_PLAN_TUNE_NO_BALANCE
FA_ORDER_TORCH_CPU = 0
FA_ORDER_TORCH_GPU = 1


EXPORTS = [
    "fa_version", "fa_last_error", "fa_plan_create", "fa_plan_destroy",
    "fa_plan_get_info", "fa_plan_build_host", "fa_plan_create_from_tiles", "fa_reduce", "fa_mean_f32", "fa_weighted_f32",
    "fa_mean_i64_trunc", "fa_div_f32", "fa_div_trunc_i64", "fa_broadcast_f32",
    "fa_synth_fill_f32", "fa_synth_fill_i64", "fa_copy_f32",
    "fa_norm_plan_create", "fa_norm_plan_destroy", "fa_prox_norms", "fa_prox_grad",
    "fa_prox_grad_ex",
    "fa_read_probe_f32", "fa_write_probe_f32", "fa_tune_prox_store", "fa_tune_prox_cpw", "fa_chain_levels", "fa_reduce_chain", "fa_torch_gpu_config",
    "fa_plan_create_order", "fa_table_bytes", "fa_reduce_tab",
    "fa_plan_balance_host", "fa_plan_launch_shape", "fa_plan_launch_form",
]


class FaSeg(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_int64), ("numel", ctypes.c_int64)]


class FaPlanInfo(ctypes.Structure):
    _fields_ = [("f32_numel", ctypes.c_int64), ("i64_numel", ctypes.c_int64),
                ("ntiles", ctypes.c_int32), ("ntiles_cascade", ctypes.c_int32),
                ("ntiles_tail", ctypes.c_int32), ("tile_elems", ctypes.c_int32),
                ("cascade_elems", ctypes.c_int64), ("tail_elems", ctypes.c_int64)]


class FaTileDesc(ctypes.Structure):
    _fields_ = [("start", ctypes.c_int64), ("count", ctypes.c_int32), ("kind", ctypes.c_int32)]


class FaChain(ctypes.Structure):
    _fields_ = [("row0", ctypes.c_int), ("n_total", ctypes.c_int), ("state_in", ctypes.c_void_p),
                ("state_out", ctypes.c_void_p), ("plane", ctypes.c_int64)]


class FedaggError(RuntimeError):
    pass


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"feddct_amd: HIP library {LIB_PATH} not built (run __graft_entry__.build()); "
            "there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "fa_version": (ctypes.c_char_p, []),
        "fa_last_error": (ctypes.c_char_p, []),
        "fa_plan_create": (_I, [_P, _I, _I64, _P, _I, _I64, _I, ctypes.c_uint,
                                ctypes.POINTER(_P)]),
        "fa_plan_destroy": (_I, [_P]),
        "fa_plan_build_host": (_I, [_P, _I, _I64, _P, _I, _I64, _I, ctypes.c_uint, _P, _I,
                                    ctypes.POINTER(FaPlanInfo)]),
        "fa_plan_get_info": (_I, [_P, ctypes.POINTER(FaPlanInfo)]),
        "fa_plan_create_from_tiles": (_I, [_P, _I, _I64, _I64, _I, ctypes.c_uint,
                                           ctypes.POINTER(_P)]),
        "fa_reduce": (_I, [_P, _P, _P, _I, _P, _P, _P, ctypes.c_uint, _P]),
        "fa_table_bytes": (ctypes.c_size_t, [_I]),
        "fa_plan_balance_host": (_I, [_P, _I, _I, _I, _I, _P, _I]),
        "fa_plan_launch_shape": (_I, [_P, _I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
        "fa_plan_launch_form": (_I, [_P, _I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I),
                                     ctypes.POINTER(_I)]),
        "fa_reduce_tab": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, ctypes.c_uint, _P]),
        "fa_mean_f32": (_I, [_P, _I, _I64, _P, _P, _I, _P]),
        "fa_weighted_f32": (_I, [_P, _P, _I, _I64, _P, _P, _I, _P]),
        "fa_mean_i64_trunc": (_I, [_P, _I, _I64, _P, _P, _I, _P]),
        "fa_div_f32": (_I, [_P, ctypes.c_float, _P, _I64, _P]),
        "fa_div_trunc_i64": (_I, [_P, ctypes.c_float, _P, _I64, _P]),
        "fa_broadcast_f32": (_I, [_P, _P, _I, _I64, _P]),
        "fa_synth_fill_f32": (_I, [_P, _I64, _I, _I, ctypes.c_float, ctypes.c_float, _I, _P]),
        "fa_synth_fill_i64": (_I, [_P, _I64, _I, _I, _I, _P]),
        "fa_copy_f32": (_I, [_P, _P, _I64, _P]),
        "fa_read_probe_f32": (_I, [_P, _I64, _P, _I, _P]),
        "fa_write_probe_f32": (_I, [_P, _I, _I64, ctypes.c_uint, _P]),
        "fa_tune_prox_store": (_I, [_I]),
        "fa_tune_prox_cpw": (_I, [_I]),
        "fa_chain_levels": (ctypes.c_uint, [_I, _I]),
        "fa_torch_gpu_config": (_I, [_I, _I64, ctypes.POINTER(_I)]),
        "fa_plan_create_order": (_I, [_P, _I, _I64, _P, _I, _I64, _I, _I, ctypes.c_uint,
                                      ctypes.POINTER(_P)]),
        "fa_reduce_chain": (_I, [_P, _P, _I, _P, ctypes.POINTER(FaChain), _P, ctypes.c_uint, _P]),
        "fa_norm_plan_create": (_I, [_P, _I, _I64, ctypes.POINTER(_P)]),
        "fa_norm_plan_destroy": (_I, [_P]),
        "fa_prox_norms": (_I, [_P, _P, _P, _P, _P, _P]),
        "fa_prox_grad": (_I, [_P, _P, _P, _P, _P, ctypes.c_float, _P, _P, _P]),
        "fa_prox_grad_ex": (_I, [_P, _P, _P, _P, _P, ctypes.c_float, _P, _P, ctypes.c_uint, _P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)  # AttributeError = missing export: loud
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int, what: str = "") -> None:
    if rc != FA_OK:
        msg = lib.fa_last_error().decode(errors="replace")
        raise FedaggError(f"{what or 'fedagg'} failed ({rc}): {msg}")


def version() -> str:
    return lib.fa_version().decode()


def ptr_array(ptrs) -> ctypes.Array:
    arr = (ctypes.c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def seg_array(segs: np.ndarray):
    segs = np.ascontiguousarray(np.asarray(segs, np.int64).reshape(-1, 2))
    arr = (FaSeg * max(1, len(segs)))()
    for i, (o, n) in enumerate(segs):
        arr[i].offset = int(o)
        arr[i].numel = int(n)
    return arr, len(segs)


def build_tiles_host(segs32, f32_numel, segs64=(), i64_numel=0, tile_elems=0,
                     flags=FA_PLAN_GAPS_ARE_PADDING):
    """Tile table of a layout, computed by the library on the host (no GPU):
    returns (info dict, ndarray of (start, count, kind))."""
    a32, n32 = seg_array(segs32 if len(segs32) else np.zeros((0, 2), np.int64))
    a64, n64 = seg_array(segs64 if len(segs64) else np.zeros((0, 2), np.int64))
    info = FaPlanInfo()
    check(lib.fa_plan_build_host(a32, n32, int(f32_numel), a64, n64, int(i64_numel),
                                 int(tile_elems), flags, None, 0, ctypes.byref(info)),
          "fa_plan_build_host")
    cap = info.ntiles
    arr = (FaTileDesc * max(1, cap))()
    check(lib.fa_plan_build_host(a32, n32, int(f32_numel), a64, n64, int(i64_numel),
                                 int(tile_elems), flags, arr, cap, ctypes.byref(info)),
          "fa_plan_build_host")
    tiles = np.array([(arr[i].start, arr[i].count, arr[i].kind) for i in range(cap)],
                     np.int64).reshape(-1, 3)
    return {f: getattr(info, f) for f, _ in FaPlanInfo._fields_}, tiles


def balance_host(vec_tiles, tile_elems=2048, nscalar=0, slots=768):
    """The plan's balanced re-cut of vector tiles (fa_plan_balance_host),
    computed on the host: ndarray of (start, count, kind), or None when the
    plain cut is kept."""
    vec = np.asarray(vec_tiles, np.int64).reshape(-1, 3)
    arr = (FaTileDesc * max(1, len(vec)))()
    for i, (s, c, k) in enumerate(vec):
        arr[i].start, arr[i].count, arr[i].kind = int(s), int(c), int(k)
    cap = 2 * len(vec) + 2 * int(slots) + 16
    out = (FaTileDesc * max(1, cap))()
    rc = lib.fa_plan_balance_host(arr, len(vec), int(tile_elems), int(nscalar), int(slots),
                                  out, cap)
    if rc < 0:
        check(rc, "fa_plan_balance_host")
    if rc == 0:
        return None
    return np.array([(out[i].start, out[i].count, out[i].kind) for i in range(rc)],
                    np.int64).reshape(-1, 3)


class Plan:
    """Owning wrapper of an ``fa_plan`` (device-resident tile table); built
    from a layout's segments, or from an explicit tile subset (``tiles``)."""

    def __init__(self, segs32, f32_numel, segs64=(), i64_numel=0, tile_elems=0,
                 flags=FA_PLAN_GAPS_ARE_PADDING, tiles=None, order=FA_ORDER_TORCH_CPU, n=0):
        h = ctypes.c_void_p()
        if order != FA_ORDER_TORCH_CPU:
            a32, n32 = seg_array(segs32 if len(segs32) else np.zeros((0, 2), np.int64))
            a64, n64 = seg_array(segs64 if len(segs64) else np.zeros((0, 2), np.int64))
            check(lib.fa_plan_create_order(a32, n32, int(f32_numel), a64, n64, int(i64_numel),
                                           int(n), int(order), flags, ctypes.byref(h)),
                  "fa_plan_create_order")
        elif tiles is not None:
            tiles = np.asarray(tiles, np.int64).reshape(-1, 3)
            arr = (FaTileDesc * max(1, len(tiles)))()
            for i, (s, c, k) in enumerate(tiles):
                arr[i].start, arr[i].count, arr[i].kind = int(s), int(c), int(k)
            check(lib.fa_plan_create_from_tiles(arr, len(tiles), int(f32_numel), int(i64_numel),
                                                int(tile_elems), flags, ctypes.byref(h)),
                  "fa_plan_create_from_tiles")
        else:
            a32, n32 = seg_array(segs32 if len(segs32) else np.zeros((0, 2), np.int64))
            a64, n64 = seg_array(segs64 if len(segs64) else np.zeros((0, 2), np.int64))
            check(lib.fa_plan_create(a32, n32, int(f32_numel), a64, n64, int(i64_numel),
                                     int(tile_elems), flags, ctypes.byref(h)), "fa_plan_create")
        self.handle = h
        info = FaPlanInfo()
        check(lib.fa_plan_get_info(h, ctypes.byref(info)), "fa_plan_get_info")
        self.info = {f: getattr(info, f) for f, _ in FaPlanInfo._fields_}

    def launch_shape(self, n, weighted=False):
        """(tiles, resident-workgroup slots) a plain fa_reduce call with n
        clients launches with (the balanced table when one applies)."""
        nt, sl = _I(), _I()
        check(lib.fa_plan_launch_shape(self.handle, int(n), int(bool(weighted)), ctypes.byref(nt),
                                       ctypes.byref(sl)), "fa_plan_launch_shape")
        return nt.value, sl.value

    def launch_form(self, n, weighted=False):
        """(tile width in floats, clients per load batch, pipe) of the kernel a
        plain fa_reduce call with n clients runs (pipe 1: the client loop)."""
        te, b, p = _I(), _I(), _I()
        check(lib.fa_plan_launch_form(self.handle, int(n), int(bool(weighted)), ctypes.byref(te),
                                      ctypes.byref(b), ctypes.byref(p)), "fa_plan_launch_form")
        return te.value, b.value, p.value

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                lib.fa_plan_destroy(h)
            except Exception:
                pass
            self.handle = None
