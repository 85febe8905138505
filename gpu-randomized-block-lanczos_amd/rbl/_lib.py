"""ctypes binding of librbl_hip.so (include/rbl_hip.h).

The library is the only compute path: if it is missing this module raises ImportError —
there is no CPU fallback anywhere in the product.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RBL_LIB: a diagnostics build of the same library (tools/build_variant.sh)
LIB_PATH = os.environ.get("RBL_LIB") or os.path.join(_HERE, "librbl_hip.so")

RBL_OK = 0
RBL_WARN_NOT_CONVERGED = 1
RBL_WARN_QR_SHIFTED = 2
RBL_ERR_INVALID = -1
RBL_ERR_HIP = -2
RBL_ERR_OOM = -3
RBL_ERR_RCCL = -4
RBL_ERR_STATE = -5
RBL_ERR_NUMERIC = -6

RBL_OPT_TIMERS = 0
RBL_OPT_REORTH_ORDER = 1
RBL_OPT_SPMM_KERNEL = 2
RBL_OPT_DEVICE_BLOCKS = 3
RBL_OPT_SPLIT_HALO = 4
RBL_OPT_KEEP_CSR = 5
RBL_OPT_FUSE = 6
RBL_OPT_HALO_OVERLAP = 7
RBL_OPT_RELABEL = 8
RBL_OPT_HALO_PUSH = 9
# rbl_path_stats entries
RBL_PATH_SPMM = 0
RBL_PATH_SPMM_LOC_FUSED = 1
RBL_PATH_LOC_SEPARATE = 2
RBL_PATH_LOC_GRAM = 3
RBL_PATH_LOCFIX_EDGES = 4
RBL_PATH_LOCFIX_REST = 5
RBL_PATH_SPMM_TWO_WAVE = 6
RBL_PATH_RITZ_PIECES = 7
RBL_PATH_NSTATS = 8
RBL_BUILD_VARIANTS = 1

_p = C.c_void_p
_i64 = C.c_int64
_u64 = C.c_uint64
_pd = C.POINTER(C.c_double)
_pi64 = C.POINTER(C.c_int64)
_pi32 = C.POINTER(C.c_int32)
_pu8 = C.POINTER(C.c_uint8)

# name -> (restype, argtypes); the complete export list of include/rbl_hip.h
SIGNATURES = {
    "rbl_abi_version": (C.c_int, []),
    "rbl_build_flags": (C.c_int, []),
    "rbl_create": (C.c_int, [C.POINTER(_p), C.c_int]),
    "rbl_get_unique_id": (C.c_int, [_pu8]),
    "rbl_create_dist": (C.c_int, [C.POINTER(_p), C.c_int, C.c_int, C.c_int, _pu8]),
    "rbl_local_group_create": (C.c_int, [C.POINTER(_p), C.c_int]),
    "rbl_local_group_free": (C.c_int, [_p]),
    "rbl_create_local": (C.c_int, [C.POINTER(_p), C.c_int, _p, C.c_int]),
    "rbl_create_shm": (C.c_int, [C.POINTER(_p), C.c_int, C.c_int, C.c_int, C.c_char_p]),
    "rbl_free": (C.c_int, [_p]),
    "rbl_last_error": (C.c_char_p, [_p]),
    "rbl_comm_info": (C.c_int, [_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_char_p, C.c_int]),
    "rbl_rccl_version": (C.c_int, [C.POINTER(C.c_int), C.c_char_p, C.c_int]),
    "rbl_set_option": (C.c_int, [_p, C.c_int, _i64]),
    "rbl_device_memory": (C.c_int, [_p, _pi64, _pi64]),
    "rbl_set_matrix_csc": (C.c_int, [_p, _i64, _i64, _pi64, _pi64, _pd, C.c_int]),
    "rbl_set_matrix_csr_rows": (C.c_int, [_p, _i64, _i64, _i64, _pi64, _pi64, _pd, C.c_int]),
    "rbl_set_matrix_dense": (C.c_int, [_p, _i64, _i64, _i64, _pd, _i64]),
    "rbl_gen_matrix_hashwindow": (C.c_int, [_p, _i64, _i64, C.c_double, _u64, C.c_int, _pd]),
    "rbl_gen_matrix_circuit": (C.c_int, [_p, _i64, _i64, C.c_double, _u64, C.c_int, _pd]),
    "rbl_gen_matrix_rmat": (C.c_int, [_p, _i64, C.c_int, _i64, C.c_double, C.c_double, C.c_double,
                                      _u64, C.c_int, _pd]),
    "rbl_matrix_info": (C.c_int, [_p, _pi64, _pi64, _pi64, _pi64]),
    "rbl_get_matrix_csr": (C.c_int, [_p, _pi64, _pi32, _pd]),
    "rbl_row_ids": (C.c_int, [_p, _pi64]),
    "rbl_apply": (C.c_int, [_p, C.c_int, _pd, _pd]),
    "rbl_spmm_kernel_for": (C.c_int, [_p, C.c_int]),
    "rbl_matrix_format": (C.c_int, [_p]),
    "rbl_start": (C.c_int, [_p, C.c_int, C.c_int, C.c_int, _pd, _u64]),
    "rbl_step": (C.c_int, [_p, C.c_int, C.c_int, _pd, _pd]),
    "rbl_step_async": (C.c_int, [_p, C.c_int, C.c_int]),
    "rbl_comm_selftest": (C.c_int, [C.c_int, C.c_char_p, C.c_int]),
    "rbl_fetch": (C.c_int, [_p, C.c_int, C.c_int, _pd, _pd, _pi32]),
    "rbl_ritz": (C.c_int, [_p, C.c_int, C.c_int, _pd, _pd]),
    "rbl_get_block": (C.c_int, [_p, C.c_int, _pd]),
    "rbl_num_blocks": (C.c_int, [_p]),
    "rbl_restart": (C.c_int, [_p, C.c_int, _pd]),
    "rbl_lock": (C.c_int, [_p, C.c_int, C.c_int, _pd]),
    "rbl_num_locked": (C.c_int, [_p]),
    "rbl_get_locked": (C.c_int, [_p, _pd]),
    "rbl_reorth_last": (C.c_int, [_p, C.c_int, C.c_int]),
    "rbl_num_stages": (C.c_int, []),
    "rbl_stage_name": (C.c_char_p, [C.c_int]),
    "rbl_timers": (C.c_int, [_p, _pd, C.c_int]),
    "rbl_reset_timers": (C.c_int, [_p]),
    "rbl_comm_stats": (C.c_int, [_p, _pi64, C.c_int, C.c_int]),
    "rbl_path_stats": (C.c_int, [_p, _pi64, C.c_int, C.c_int]),
    "rbl_allgather_host": (C.c_int, [_p, _pi64, _pi64, C.c_int]),
    "rbl_synchronize": (C.c_int, [_p]),
    "rbl_plan_row_partition": (C.c_int, [_i64, _pi64, C.c_int, _pi64]),
    "rbl_plan_halo": (C.c_int, [_i64, _pi64, _pi64, C.c_int, C.c_int, _pi64, _pi64, _pi64]),
    "rbl_hashwindow_rows_host": (C.c_int, [_i64, _i64, C.c_double, _u64, C.c_int, _pd, _i64,
                                           _i64, _pi64, _pi64, _pd]),
}


class RBLError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"librbl_hip error {code}: {msg}")
        self.code = code


def load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"librbl_hip.so not built at {LIB_PATH}; run __graft_entry__.build() "
                          "(the HIP library is the only compute path — no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = load()
# compiled with -DRBL_VARIANTS (tools/build_variant.sh): the measured-and-rejected variants and
# their A/B switches are in this copy (tests/test_gpu_variants.py runs only then)
VARIANTS = bool(lib.rbl_build_flags() & RBL_BUILD_VARIANTS)


def dptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float64 and (a.flags.c_contiguous or a.flags.f_contiguous)
    return a.ctypes.data_as(_pd)


def i64ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.int64 and a.flags.c_contiguous
    return a.ctypes.data_as(_pi64)


def i32ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_pi32)


def u8ptr(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(_pu8)


def stage_names() -> list[str]:
    return [lib.rbl_stage_name(s).decode() for s in range(lib.rbl_num_stages())]


def plan_row_partition(rowptr: np.ndarray, nranks: int) -> np.ndarray:
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    out = np.zeros(nranks + 1, dtype=np.int64)
    st = lib.rbl_plan_row_partition(len(rowptr) - 1, i64ptr(rowptr), nranks, i64ptr(out))
    if st != RBL_OK:
        raise RBLError(st, "rbl_plan_row_partition")
    return out


def plan_halo(rowptr, colind, bounds, index_base=0):
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    colind = np.ascontiguousarray(colind, dtype=np.int64)
    bounds = np.ascontiguousarray(bounds, dtype=np.int64)
    P = len(bounds) - 1
    lo = np.zeros(P, dtype=np.int64)
    hi = np.zeros(P, dtype=np.int64)
    st = lib.rbl_plan_halo(len(rowptr) - 1, i64ptr(rowptr), i64ptr(colind), index_base, P,
                           i64ptr(bounds), i64ptr(lo), i64ptr(hi))
    if st != RBL_OK:
        raise RBLError(st, "rbl_plan_halo")
    return lo, hi


def hashwindow_rows_host(n, halfwidth, density, seed, plant, row_begin, row_end):
    """Host twin of the device generator (same bits): returns (rowptr, colind, val) 0-based."""
    plant = np.ascontiguousarray(plant if plant is not None else np.zeros(0), dtype=np.float64)
    m = row_end - row_begin
    rowptr = np.zeros(m + 1, dtype=np.int64)
    pp = dptr(plant) if plant.size else None
    st = lib.rbl_hashwindow_rows_host(n, halfwidth, density, seed, plant.size, pp, row_begin,
                                      row_end, i64ptr(rowptr), None, None)
    if st != RBL_OK:
        raise RBLError(st, "rbl_hashwindow_rows_host")
    nnz = int(rowptr[-1])
    col = np.zeros(nnz, dtype=np.int64)
    val = np.zeros(nnz, dtype=np.float64)
    st = lib.rbl_hashwindow_rows_host(n, halfwidth, density, seed, plant.size, pp, row_begin,
                                      row_end, i64ptr(rowptr), i64ptr(col), dptr(val))
    if st != RBL_OK:
        raise RBLError(st, "rbl_hashwindow_rows_host")
    return rowptr, col, val
