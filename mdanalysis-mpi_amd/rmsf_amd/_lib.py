"""ctypes binding of ``librmsf_hip.so`` (the C ABI declared in include/rmsf_hip.h).

This module is the only place that touches the shared library.  It fails
loudly: there is no CPU fallback anywhere in the product path -- if the HIP
library is missing or no HIP device is visible, callers get an exception.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_size_t, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "lib", "librmsf_hip.so"))

RMSF_OK = 0
RMSF_EINVAL = -1
RMSF_EHIP = -2
RMSF_ENOMEM = -3
RMSF_EEMPTY = -4
RMSF_MODE_WELFORD = 0
RMSF_MODE_SUM = 1
RMSF_XFORM_DOUBLES = 16
RMSF_MAX_SPLIT_FRAMES = 4096  # frames per accumulate split (Welford coefficient table)
RMSF_REFINFO_DOUBLES = 2064  # 16-double record + reduction scratch
ABI_VERSION = 1


class RmsfError(RuntimeError):
    """A non-zero status returned through the C ABI."""

    def __init__(self, code: int, func: str, msg: str):
        super().__init__(f"{func} failed with status {code}: {msg}")
        self.code = code


class RmsfEmptyError(RmsfError, ZeroDivisionError):
    """No frames to reduce.  Subclasses ZeroDivisionError because RMSF.py:39
    raises exactly that when two empty partials are merged."""


# name -> (restype, argtypes); every symbol include/rmsf_hip.h declares.
P = c_void_p
SIGNATURES = {
    "rmsf_abi_version": (c_int, []),
    "rmsf_last_error": (c_char_p, []),
    "rmsf_device_count": (c_int, [POINTER(c_int)]),
    "rmsf_set_device": (c_int, [c_int]),
    "rmsf_malloc": (c_int, [POINTER(c_void_p), c_size_t]),
    "rmsf_free": (c_int, [P]),
    "rmsf_memcpy_h2d": (c_int, [P, P, c_size_t, P]),
    "rmsf_memcpy_d2h": (c_int, [P, P, c_size_t, P]),
    "rmsf_memcpy2d_d2d": (c_int, [P, c_size_t, P, c_size_t, c_size_t, c_size_t, P]),
    "rmsf_stream_synchronize": (c_int, [P]),
    "rmsf_block_range": (c_int, [c_int64, c_int, c_int, POINTER(c_int64), POINTER(c_int64)]),
    "rmsf_reference_setup": (c_int, [P, P, c_int64, P, P, P, P, P]),
    "rmsf_reference_setup_mean": (c_int, [P, c_double, c_int64, P, P, P, P, P]),
    "rmsf_fold_balanced_finalize": (c_int, [P, c_int64, c_int64, P, P, c_int64, P, P]),
    "rmsf_superpose_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "rmsf_superpose": (c_int, [P, c_int64, c_int64, c_int64, P, P, P, P, P, P, c_size_t, P]),
    "rmsf_superpose_planes": (c_int, [P, c_int64, c_int64, c_int64, c_int64, P, P, P, P, P, P, c_size_t, P]),
    "rmsf_superpose_compact": (c_int, [P, c_int64, c_int64, c_int64, P, P, P, P, P, P, c_size_t, P, c_int64, P]),
    "rmsf_accumulate_splits": (c_int, [c_int64, c_int64, c_int]),
    "rmsf_accumulate": (c_int, [P, c_int64, c_int64, c_int64, P, P, P, c_int, c_int, P, P, P]),
    "rmsf_split_count": (c_int64, [c_int64, c_int, c_int]),
    "rmsf_accumulate_balanced_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int]),
    "rmsf_accumulate_balanced": (c_int, [P, c_int64, c_int64, c_int64, P, P, P, c_int, c_int, P, c_size_t, P]),
    "rmsf_fold_balanced": (c_int, [P, c_int64, c_int, c_int64, P, P, P]),
    "rmsf_accumulate_balanced_planes": (c_int, [P, c_int64, c_int64, c_int64, c_int64, P, P, P, c_int, c_int, P,
                                                c_size_t, P]),
    "rmsf_chan_merge": (c_int, [P, P, P, c_int, c_int64, P, P, P]),
    "rmsf_chan_reduce_steps": (c_int, [c_int, c_int, P, P, c_int]),
    "rmsf_chan_reduce": (c_int, [P, P, P, c_int, c_int64, c_int, P, P, P]),
    "rmsf_chan_merge_pair": (c_int, [P, P, c_int64, P, P, c_int64, c_int64, P]),
    "rmsf_sum_splits": (c_int, [P, c_int, c_int64, P, P]),
    "rmsf_divide": (c_int, [P, c_double, c_int64, P, P]),
    "rmsf_chan_weight": (c_int, [P, c_double, c_int64, P, P]),
    "rmsf_chan_deviation": (c_int, [P, P, P, c_double, c_int64, P, P]),
    "rmsf_finalize": (c_int, [P, c_int64, c_int64, P, P]),
    "rmsf_reference_setup_sequential": (c_int, [P, P, c_double, c_int64, P, P, c_double, P, P, P, P]),
    "rmsf_superpose_sequential": (c_int, [P, c_int64, c_int64, c_int64, P, P, c_double, P, P, P, P]),
    "rmsf_reference_centre_sequential": (c_int, [P, P, c_double, c_int64, P, P, c_double, P, P, P, P]),
    "rmsf_reference_sums_sequential": (c_int, [c_int64, c_double, P, P, P]),
    "rmsf_frame_com_sequential": (c_int, [P, c_int64, c_int64, c_int64, P, P, c_double, P, P]),
    "rmsf_inner_product_sequential": (c_int, [P, c_int64, c_int64, c_int64, P, P, P, P]),
    "rmsf_superpose_sequential_qcp": (c_int, [c_int64, c_int64, P, P, P]),
    "rmsf_superpose_sequential_from_com": (c_int, [P, c_int64, c_int64, c_int64, P, P, P, P, P]),
    "rmsf_accumulate_sequential": (c_int, [P, c_int64, c_int64, c_int64, P, P, P, c_int, c_int64, P, P, P, c_size_t,
                                           P]),
    "rmsf_welford_sequential_workspace_bytes": (c_size_t, [c_int64]),
    "rmsf_welford_sequential": (c_int, [P, c_int64, c_int64, c_int64, P, c_int64, P, P, P, c_size_t, P]),
    "rmsf_chan_shift_pack": (c_int, [P, P, P, c_int, P, c_double, c_int64, P, P]),
    "rmsf_fold_balanced_shift": (c_int, [P, c_int64, c_int64, P, P, P, c_int, P, P, P]),
    "rmsf_fold_balanced_shift_sliced": (c_int, [P, c_int64, c_int64, P, P, P, c_int, P, c_int64, P, P]),
    "rmsf_chan_shift_pack_sliced": (c_int, [P, P, P, c_int, P, c_double, c_int64, c_int64, P, P]),
    "rmsf_chan_shift_finish_slice": (c_int, [P, c_int64, P, c_int, P, c_int64, c_int64, P, P, P, P]),
    "rmsf_balanced_slab_chunks": (c_int, [P, c_int64, c_int64, c_int64, P]),
    "rmsf_accumulate_balanced_slab": (c_int, [P, c_int64, c_int64, c_int64, c_int64, c_int64, P, c_size_t, P]),
    "rmsf_fold_balanced_shift_slab": (c_int, [P, c_int64, c_int64, P, P, P, c_int, P, P, c_int64, c_int64, P]),
    "rmsf_chan_shift_finish": (c_int, [P, P, c_int, P, c_int64, c_int64, P, P, P, P]),
    "rmsf_qcp_batch": (c_int, [P, P, P, c_int64, P, P, P]),
    "rmsf_calc_rmsd_rotational_matrix": (c_int, [P, P, c_int64, P, P, POINTER(c_double)]),
    "rmsf_synth_frames": (c_int, [P, c_int64, c_int64, c_int64, c_int64, c_uint64, P, P]),
    "rmsf_synth_sigma": (c_int, [P, c_int64, c_int64, c_uint64, P]),
    "rmsf_gather_frames": (c_int, [P, c_int64, P, c_int64, c_int64, P, P, P]),
    "rmsf_gather_planes": (c_int, [P, c_int64, c_int64, P, c_int64, c_int64, P, P, P]),
    "rmsf_planes_to_rows": (c_int, [P, c_int64, P, P]),
    "rmsf_stager_create": (c_int, [c_int64, c_int64, P, c_int64, c_int, c_int, POINTER(c_void_p)]),
    "rmsf_stager_destroy": (c_int, [P]),
    "rmsf_stager_stage": (c_int, [P, P, c_int64, c_int64, P, POINTER(c_int), POINTER(c_void_p)]),
    "rmsf_stager_stage_ptrs": (c_int, [P, P, c_int64, P, POINTER(c_int), POINTER(c_void_p)]),
    "rmsf_stager_stage_planes": (c_int, [P, P, c_int64, c_int64, P, POINTER(c_int), POINTER(c_void_p)]),
    "rmsf_stager_stage_xtc": (c_int, [P, P, c_int64, c_int64, c_int64, P, POINTER(c_int), POINTER(c_void_p)]),
    "rmsf_stager_release": (c_int, [P, c_int, P]),
    "rmsf_stager_synchronize": (c_int, [P]),
    "rmsf_xtc_open": (c_int, [c_char_p, POINTER(c_void_p), POINTER(c_int64), POINTER(c_int64)]),
    "rmsf_xtc_close": (c_int, [P]),
    "rmsf_xtc_frame_info": (c_int, [P, c_int64, POINTER(c_int32), POINTER(ctypes.c_float), P]),
    "rmsf_xtc_read": (c_int, [P, c_int64, c_int64, c_int64, P, c_int64, P, c_int]),
    "rmsf_xtc_write": (c_int, [c_char_p, P, c_int64, c_int64, ctypes.c_float, P, c_int]),
    "rmsf_xtc_frame_record": (c_int, [P, c_int64, POINTER(c_int64), POINTER(c_int64)]),
    "rmsf_xtcdec_create": (c_int, [P, c_int64, c_int, c_int, POINTER(c_void_p)]),
    "rmsf_xtcdec_destroy": (c_int, [P]),
    "rmsf_xtcdec_decode": (c_int, [P, c_int64, c_int64, c_int64, P, POINTER(c_int), POINTER(c_void_p)]),
    "rmsf_xtcdec_decode_into": (c_int, [P, c_int64, c_int64, c_int64, P, c_int64, P, POINTER(c_int)]),
    "rmsf_xtcdec_decode_list": (c_int, [P, P, c_int64, P, POINTER(c_int), POINTER(c_void_p)]),
    "rmsf_xtcdec_release": (c_int, [P, c_int, P]),
    "rmsf_xtcdec_synchronize": (c_int, [P]),
    "rmsf_xtc_decode_records": (c_int, [P, P, P, c_int64, c_int64, P, c_int64, P, P]),
    "rmsf_xtc_decode_records_host": (c_int, [P, P, P, c_int64, c_int64, P, c_int64, P]),
    # RMSF context (rmsf_ctx_*) and cross-rank exchange
    "rmsf_ctx_create": (c_int, [c_int, c_int64, c_int64, P, P, c_int, POINTER(c_void_p)]),
    "rmsf_ctx_destroy": (c_int, [P]),
    "rmsf_ctx_stream": (c_int, [P, POINTER(c_void_p)]),
    "rmsf_ctx_synchronize": (c_int, [P]),
    "rmsf_ctx_set_staging": (c_int, [P, c_int64, c_int, c_int]),
    "rmsf_ctx_reset": (c_int, [P, c_int]),
    "rmsf_ctx_set_timing": (c_int, [P, c_int]),
    "rmsf_ctx_collect_rmsd": (c_int, [P, c_int]),
    "rmsf_ctx_set_exact": (c_int, [P, c_int, c_double]),
    "rmsf_get_rmsd": (c_int, [P, POINTER(c_int64), P, c_int64]),
    "rmsf_ctx_kernel_time": (c_int, [P, c_int, POINTER(c_int64), POINTER(c_double), POINTER(c_double)]),
    "rmsf_set_reference": (c_int, [P, P, P]),
    "rmsf_set_reference_frame": (c_int, [P, P, c_int]),
    "rmsf_set_reference_average": (c_int, [P]),
    "rmsf_push_frames": (c_int, [P, P, c_int64, c_int64, c_int, c_int]),
    "rmsf_push_xtc": (c_int, [P, P, c_int64, c_int64, c_int64, c_int]),
    "rmsf_push_xtc_frames": (c_int, [P, P, P, c_int64, c_int]),
    "rmsf_push_frame_ptrs": (c_int, [P, P, c_int64, c_int]),
    "rmsf_push_frame_planes": (c_int, [P, P, c_int64, c_int64, c_int]),
    "rmsf_get_partial": (c_int, [P, POINTER(c_int64), P, P]),
    "rmsf_get_sum": (c_int, [P, POINTER(c_int64), P]),
    "rmsf_get_average": (c_int, [P, P]),
    "rmsf_get_rmsf": (c_int, [P, P]),
    "rmsf_set_partial": (c_int, [P, c_int64, P, P]),
    "rmsf_ctx_allreduce_sum": (c_int, [P, P, P]),
    "rmsf_ctx_chan_merge": (c_int, [P, P, P]),
    "rmsf_ctx_chan_merge_shifted": (c_int, [P, P, P]),
    "rmsf_multi_unique_id": (c_int, [P]),
    "rmsf_multi_init": (c_int, [P, P, c_int, c_int]),
    "rmsf_multi_init_all": (c_int, [P, c_int]),
    "rmsf_multi_allreduce_sum": (c_int, [P, c_int]),
    "rmsf_multi_chan_merge": (c_int, [P, c_int]),
    "rmsf_set_merge_shift_frame": (c_int, [P, P, c_int]),
    "rmsf_multi_chan_merge_root": (c_int, [P, c_int, c_int]),
    "rmsf_multi_chan_merge_exact": (c_int, [P, c_int, c_int, c_int]),
    "rmsf_multi_push_frames": (c_int, [P, c_int, P, P, c_int64, c_int, c_int, P, P, c_int]),
    "rmsf_multi_set_transport": (c_int, [P, c_int, c_int]),
}

# int (*rmsf_allreduce_fn)(double *d_buf, int64_t count, void *stream, void *user)
ALLREDUCE_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_int64, c_void_p, c_void_p)
RMSF_PUSH_WELFORD, RMSF_PUSH_ALIGN_SUM, RMSF_PUSH_ALIGN_WELFORD, RMSF_PUSH_SUM, RMSF_PUSH_EXACT = 0, 1, 2, 3, 4
RMSF_UNIQUE_ID_BYTES = 128
RMSF_TIME_ACCUMULATE, RMSF_TIME_SUPERPOSE, RMSF_TIME_MERGE = 0, 1, 2
RMSF_MULTI_RESET = 1
RMSF_TRANSPORT_AUTO, RMSF_TRANSPORT_NOOP = 0, 1
RMSF_MERGE_RANK, RMSF_MERGE_MPI4PY = 0, 1
MERGE_ORDERS = {"rank": RMSF_MERGE_RANK, "mpi4py": RMSF_MERGE_MPI4PY}


def merge_order(order) -> int:
    """``"mpi4py"`` (RMSF.py:143's comm.reduce: mpi4py's default binomial
    tree) or ``"rank"`` (rank order) -> the ABI's RMSF_MERGE_* value."""
    if isinstance(order, int) and order in MERGE_ORDERS.values():
        return order
    try:
        return MERGE_ORDERS[order]
    except (KeyError, TypeError):
        raise ValueError(f"merge_order must be one of {sorted(MERGE_ORDERS)}, got {order!r}") from None


def reduce_steps(n_parts: int, order="mpi4py") -> list[tuple[int, int]]:
    """The (dst, src) steps S[dst] = op(S[dst], S[src]) of the reduction
    (rmsf_chan_reduce_steps; host-only, no device needed)."""
    lib = load()
    o = merge_order(order)
    k = lib.rmsf_chan_reduce_steps(int(n_parts), o, None, None, 0)
    check(min(k, 0), "rmsf_chan_reduce_steps")
    d, s = (c_int * max(k, 1))(), (c_int * max(k, 1))()
    lib.rmsf_chan_reduce_steps(int(n_parts), o, d, s, k)
    return [(d[i], s[i]) for i in range(k)]

_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load the library (once) and declare every signature.

    Raises ImportError with a build hint if the .so is missing -- the product
    never falls back to a CPU path.
    """
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(
            f"librmsf_hip.so not found at {p}; build it with "
            "`make -C mdanalysis-mpi_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError = a declared symbol is missing
        fn.restype = res
        fn.argtypes = args
    v = lib.rmsf_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"librmsf_hip.so ABI {v} != expected {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(rc: int, func: str) -> None:
    if rc != RMSF_OK:
        msg = (_lib or load()).rmsf_last_error()
        msg = msg.decode(errors="replace") if msg else ""
        cls = RmsfEmptyError if rc == RMSF_EEMPTY else RmsfError
        raise cls(rc, func, msg)


def call(name: str, *args) -> int:
    lib = load()
    rc = getattr(lib, name)(*args)
    check(rc, name)
    return rc


def i64p(values) -> ctypes.Array:
    arr = (c_int64 * len(values))(*[int(v) for v in values])
    return arr


def int32_array(values) -> ctypes.Array:
    return (c_int32 * len(values))(*[int(v) for v in values])
