"""ctypes binding of the in-tree libdbgpu_agg.so (include/dbgpu_agg.h).

This is the Python analog of the Rust `extern "C"` block a Databend maintainer would add
(INTEGRATION.md).  The library must be present: there is no CPU fallback in the product path —
`lib()` raises if the HIP extension was not built (run `python -c "import __graft_entry__ as g; g.build()"`).
"""
from __future__ import annotations

import ctypes as C
import os

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
# DBGPU_LIB: another in-tree build of the same library (e.g. `make TRACE=1` into a side path)
LIB_PATH = os.environ.get("DBGPU_LIB") or os.path.join(_HERE, "libdbgpu_agg.so")
_LIB = None

EXPORTED = [
    "dbg_version", "dbg_last_error", "dbg_device_count", "dbg_agg_result_type", "dbg_agg_create",
    "dbg_agg_destroy", "dbg_agg_set_stream", "dbg_agg_reset", "dbg_agg_add_groups", "dbg_agg_finalize",
    "dbg_agg_result", "dbg_agg_finalize_into", "dbg_agg_set_recycle", "dbg_agg_set_partition_keys", "dbg_agg_finalize_into_async", "dbg_agg_finalize_wait", "dbg_agg_record_width", "dbg_agg_partition", "dbg_agg_export_records",
    "dbg_agg_merge_records", "dbg_agg_export_fixed", "dbg_agg_capacity", "dbg_agg_merge_fixed", "dbg_filter_select", "dbg_take_fixed", "dbg_sort_limit_indices", "dbg_sort_limit_multi", "dbg_agg_compact", "dbg_agg_retained_bytes", "dbg_prof_enable", "dbg_prof_reset",
    "dbg_prof_get", "dbg_prof_marker", "dbg_datagen", "dbg_agg_set_strategy", "dbg_agg_get_strategy",
    "dbg_agg_record_layout", "dbg_agg_set_host_staging",
    "dbg_take_string", "dbg_legacy_hash_method", "dbg_legacy_group_hash", "dbg_agg_serialized_stride", "dbg_agg_result_serialized", "dbg_agg_merge_serialized", "dbg_comm_get_unique_id", "dbg_comm_create", "dbg_comm_destroy", "dbg_agg_exchange",
    "dbg_agg_payload_counts", "dbg_agg_payload_export", "dbg_agg_payload_import", "dbg_agg_exchange_payload",
    "dbg_payload_exchange_plan", "dbg_merge_exchange_plan", "dbg_agg_payload_counts_from", "dbg_agg_payload_export_from",
    "dbg_agg_payload_import_chunks", "dbg_agg_exchange_payload_chunk",
    "dbg_scan_create", "dbg_scan_destroy", "dbg_parquet_chunk_rows", "dbg_parquet_decode",
    "dbg_native_decode",
]


class DbgError(RuntimeError):
    """A non-OK status from the C ABI (reference: ErrorCode)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class DecimalOverflow(DbgError):
    pass


class Unsupported(DbgError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: the HIP extension was not built "
                              "(run __graft_entry__.build()); there is no CPU fallback")
        # One HIP runtime per process: torch bundles its own libamdhip64/libhsa-runtime64 (same
        # SONAME as /opt/rocm's).  Loading torch first makes the loader resolve this library's
        # libamdhip64.so.7 to the already-loaded copy; the other order would bring up a second
        # HSA runtime that cannot open the device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        P, U64, I32, VP = C.POINTER, C.c_uint64, C.c_int32, C.c_void_p
        L.dbg_version.restype = C.c_char_p
        L.dbg_last_error.restype = C.c_char_p
        L.dbg_device_count.argtypes = [P(C.c_int)]
        L.dbg_agg_result_type.argtypes = [P(abi.dbg_agg_spec), P(abi.dbg_datatype)]
        L.dbg_agg_create.argtypes = [P(abi.dbg_agg_params), P(VP)]
        L.dbg_agg_destroy.argtypes = [VP]
        L.dbg_agg_destroy.restype = None
        L.dbg_agg_set_stream.argtypes = [VP, VP]
        L.dbg_agg_reset.argtypes = [VP]
        L.dbg_agg_add_groups.argtypes = [VP, P(abi.dbg_column), P(abi.dbg_column), P(abi.dbg_filter), U64, C.c_int]
        L.dbg_agg_finalize.argtypes = [VP, P(U64), P(U64)]
        L.dbg_agg_result.argtypes = [VP, P(abi.dbg_out_column), P(abi.dbg_out_column), C.c_int]
        L.dbg_agg_finalize_into.argtypes = [VP, P(abi.dbg_out_column), P(abi.dbg_out_column), U64, P(U64), P(U64), P(U64)]
        L.dbg_agg_set_recycle.argtypes = [VP, C.c_int]
        L.dbg_agg_set_partition_keys.argtypes = [VP, C.c_int]
        L.dbg_agg_set_host_staging.argtypes = [VP, U64]
        L.dbg_comm_get_unique_id.argtypes = [VP]
        L.dbg_comm_create.argtypes = [VP, C.c_int, C.c_int, C.c_int, P(VP)]
        L.dbg_comm_destroy.argtypes = [VP]
        L.dbg_comm_destroy.restype = None
        L.dbg_agg_exchange.argtypes = [VP, VP, VP, P(abi.dbg_exchange_stats)]
        L.dbg_agg_set_strategy.argtypes = [VP, C.c_int]
        L.dbg_agg_record_layout.argtypes = [P(abi.dbg_agg_params), P(abi.dbg_record_layout)]
        L.dbg_agg_get_strategy.argtypes = [VP, P(C.c_int), P(U64)]
        L.dbg_agg_finalize_into_async.argtypes = [VP, P(abi.dbg_out_column), P(abi.dbg_out_column), U64, P(U64)]
        L.dbg_agg_finalize_wait.argtypes = [VP, P(U64), P(U64)]
        L.dbg_agg_record_width.argtypes = [VP, P(C.c_uint32)]
        L.dbg_agg_partition.argtypes = [VP, C.c_uint32, C.c_int, P(U64), P(U64)]
        L.dbg_agg_export_records.argtypes = [VP, VP, VP]
        L.dbg_agg_merge_records.argtypes = [VP, VP, VP, I32, P(U64), P(U64)]
        L.dbg_agg_export_fixed.argtypes = [VP, VP, U64]
        L.dbg_agg_capacity.argtypes = [VP, P(U64)]
        L.dbg_agg_merge_fixed.argtypes = [VP, VP, I32, U64]
        L.dbg_filter_select.argtypes = [P(abi.dbg_filter), U64, VP, P(U64), VP]
        L.dbg_take_fixed.argtypes = [P(abi.dbg_column), VP, U64, VP, VP, VP]
        L.dbg_agg_serialized_stride.argtypes = [VP, P(C.c_uint32)]
        L.dbg_agg_result_serialized.argtypes = [VP, P(abi.dbg_out_column), P(abi.dbg_out_column), C.c_int]
        L.dbg_agg_merge_serialized.argtypes = [VP, P(abi.dbg_column), P(abi.dbg_column), U64, C.c_int]
        L.dbg_legacy_hash_method.argtypes = [P(abi.dbg_datatype), C.c_int, P(C.c_int), P(C.c_uint32)]
        L.dbg_legacy_group_hash.argtypes = [P(abi.dbg_column), C.c_int, U64, VP, VP, C.c_int, VP]
        L.dbg_take_string.argtypes = [P(abi.dbg_column), VP, U64, VP, VP, U64, VP, P(U64), VP]
        L.dbg_sort_limit_indices.argtypes = [P(abi.dbg_column), U64, C.c_int, C.c_int, U64, VP, P(U64), VP]
        L.dbg_agg_compact.argtypes = [VP, P(C.c_int)]
        L.dbg_agg_retained_bytes.argtypes = [VP, P(U64)]
        L.dbg_sort_limit_multi.argtypes = [P(abi.dbg_column), C.c_int, P(C.c_int), P(C.c_int), U64, U64, VP, P(U64), VP]
        L.dbg_prof_enable.argtypes = [C.c_int]
        L.dbg_prof_get.argtypes = [C.c_int, P(C.c_char_p), P(C.c_double), P(U64)]
        L.dbg_prof_marker.argtypes = [VP]
        L.dbg_agg_payload_counts.argtypes = [VP, P(U64), P(C.c_uint32)]
        L.dbg_agg_payload_export.argtypes = [VP, C.c_uint32, VP]
        L.dbg_agg_payload_import.argtypes = [VP, C.c_uint32, C.c_uint32, P(U64), VP, VP]
        L.dbg_agg_exchange_payload.argtypes = [VP, VP, P(abi.dbg_exchange_stats)]
        L.dbg_agg_payload_counts_from.argtypes = [VP, P(C.c_uint32), P(U64), P(C.c_uint32), P(C.c_uint32)]
        L.dbg_agg_payload_export_from.argtypes = [VP, C.c_uint32, P(C.c_uint32), VP]
        L.dbg_agg_payload_import_chunks.argtypes = [VP, C.c_uint32, C.c_uint32, C.c_uint32, P(U64), P(VP), P(VP)]
        L.dbg_agg_exchange_payload_chunk.argtypes = [VP, VP, C.c_int, P(abi.dbg_exchange_stats)]
        L.dbg_payload_exchange_plan.argtypes = [P(abi.dbg_agg_params), C.c_uint32, C.c_uint32, P(C.c_uint64), P(C.c_uint32),
                                                P(C.c_uint64), P(C.c_uint64)]
        L.dbg_merge_exchange_plan.argtypes = [P(abi.dbg_agg_params), C.c_uint32, C.c_uint32, P(C.c_uint64), P(C.c_uint32),
                                              P(C.c_uint64), P(C.c_uint64), P(C.c_uint64)]
        L.dbg_scan_create.argtypes = [P(VP), VP]
        L.dbg_scan_destroy.argtypes = [VP]
        L.dbg_parquet_chunk_rows.argtypes = [P(abi.dbg_parquet_chunk), P(U64), P(C.c_uint32)]
        L.dbg_parquet_decode.argtypes = [VP, P(abi.dbg_parquet_chunk), abi.dbg_datatype, P(abi.dbg_out_column), U64, U64, P(U64),
                                         P(U64)]
        L.dbg_native_decode.argtypes = [VP, P(abi.dbg_native_column), abi.dbg_datatype, P(abi.dbg_out_column), U64, U64, P(U64),
                                        P(U64)]
        L.dbg_datagen.argtypes = [C.c_int, U64, U64, U64, P(VP), C.c_int, VP, VP]
        _LIB = L
    return _LIB


def check(rc: int):
    if rc == abi.DBG_OK:
        return
    msg = lib().dbg_last_error().decode(errors="replace")
    if rc == abi.DBG_ERR_OVERFLOW:
        raise DecimalOverflow(rc, msg)
    if rc == abi.DBG_ERR_UNSUPPORTED:
        raise Unsupported(rc, msg)
    raise DbgError(rc, msg)


def prof_enable(on: bool = True):
    check(lib().dbg_prof_enable(1 if on else 0))


def prof_reset():
    check(lib().dbg_prof_reset())


def prof_read() -> dict:
    """{kernel name: (total_ms, launches)} from the in-library HIP event timers."""
    out = {}
    i = 0
    while True:
        name, ms, n = C.c_char_p(), C.c_double(), C.c_uint64()
        if lib().dbg_prof_get(i, C.byref(name), C.byref(ms), C.byref(n)) != abi.DBG_OK:
            break
        out[name.value.decode()] = (ms.value, n.value)
        i += 1
    return out
