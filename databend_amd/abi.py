"""ctypes mirror of include/dbgpu_agg.h (the C ABI of libdbgpu_agg.so).

Plumbing only: these structs are what a Rust `extern "C"` block or this Python
host mirror hand to the library.  Keep in sync with the header; tests/test_abi.py checks sizes.
"""
import ctypes as C

DBG_OK = 0
DBG_ERR_OVERFLOW = 1
DBG_ERR_OOM = 2
DBG_ERR_UNSUPPORTED = 3
DBG_ERR_INTERNAL = 4
DBG_ERR_INVALID = 5
DBG_ERR_DEVICE = 6

# dbg_type
INT8, INT16, INT32, INT64, UINT8, UINT16, UINT32, UINT64 = range(8)
FLOAT32, FLOAT64, DECIMAL128, DATE, TIMESTAMP, STRING, BOOLEAN = range(8, 15)

# dbg_agg_kind
AGG_COUNT, AGG_SUM, AGG_MIN, AGG_MAX, AGG_AVG, AGG_AVG_SQL = range(6)

# dbg_agg_set_strategy
STRATEGY_AUTO, STRATEGY_TABLE, STRATEGY_PARTITIONED = range(3)

# dbg_cmp
CMP_EQ, CMP_NE, CMP_LT, CMP_LE, CMP_GT, CMP_GE = range(6)

# dbg_pred_op
PRED_CMP_CONST, PRED_CMP_COLS, PRED_AND, PRED_OR, PRED_NOT, PRED_IS_NULL, PRED_IS_NOT_NULL, PRED_TRUE = range(8)


class dbg_datatype(C.Structure):
    _fields_ = [("type", C.c_int32), ("precision", C.c_uint8), ("scale", C.c_uint8),
                ("nullable", C.c_uint8), ("reserved", C.c_uint8)]


class dbg_column(C.Structure):
    _fields_ = [("dt", dbg_datatype), ("data", C.c_void_p), ("offsets", C.c_void_p),
                ("validity", C.c_void_p), ("validity_offset", C.c_uint64),
                ("data_offset", C.c_uint64), ("len", C.c_uint64)]


class dbg_out_column(C.Structure):
    _fields_ = [("dt", dbg_datatype), ("data", C.c_void_p), ("offsets", C.c_void_p),
                ("validity", C.c_void_p)]


class dbg_agg_spec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("arg", dbg_datatype), ("or_null", C.c_uint8),
                ("reserved", C.c_uint8 * 3)]


class dbg_pred_node(C.Structure):
    _fields_ = [("op", C.c_int32), ("cmp", C.c_int32), ("col", C.c_int32), ("col2", C.c_int32),
                ("i64", C.c_int64), ("f64", C.c_double), ("i128_lo", C.c_uint64),
                ("i128_hi", C.c_int64), ("str", C.c_void_p), ("str_len", C.c_uint64)]


class dbg_filter(C.Structure):
    _fields_ = [("nodes", C.POINTER(dbg_pred_node)), ("n_nodes", C.c_int32),
                ("n_cols", C.c_int32), ("cols", C.POINTER(dbg_column))]


class dbg_agg_params(C.Structure):
    _fields_ = [("group_types", C.POINTER(dbg_datatype)), ("n_group_cols", C.c_int32),
                ("aggs", C.POINTER(dbg_agg_spec)), ("n_aggs", C.c_int32), ("device", C.c_int32),
                ("partial", C.c_int32), ("capacity_hint", C.c_uint64)]


class dbg_record_layout(C.Structure):
    _fields_ = [("width", C.c_uint32), ("state_off", C.c_uint32), ("key_off", C.c_uint32 * 8),
                ("validity_off", C.c_uint32 * 8), ("agg_w0", C.c_int32 * 32), ("agg_words", C.c_int32 * 32),
                ("flags_word", C.c_int32), ("n_words", C.c_int32)]


class dbg_exchange_stats(C.Structure):
    _fields_ = [("sent_bytes", C.c_uint64), ("remote_bytes", C.c_uint64), ("received_records", C.c_uint64),
                ("received_string_bytes", C.c_uint64)]


class dbg_parquet_chunk(C.Structure):  # include/dbgpu_scan.h
    _fields_ = [("host", C.c_void_p), ("device", C.c_void_p), ("len", C.c_uint64), ("physical_type", C.c_int32),
                ("type_length", C.c_int32), ("max_def_level", C.c_int32), ("codec", C.c_int32)]


class dbg_native_column(C.Structure):  # include/dbgpu_scan.h
    _fields_ = [("host", C.c_void_p), ("device", C.c_void_p), ("len", C.c_uint64), ("page_lengths", C.POINTER(C.c_uint64)),
                ("page_rows", C.POINTER(C.c_uint64)), ("n_pages", C.c_uint32), ("nullable", C.c_int32)]


# parquet physical types / codecs (dbgpu_scan.h)
PQ_BOOLEAN, PQ_INT32, PQ_INT64, PQ_INT96, PQ_FLOAT, PQ_DOUBLE, PQ_BYTE_ARRAY, PQ_FIXED_LEN_BYTE_ARRAY = range(8)
PQ_UNCOMPRESSED, PQ_SNAPPY, PQ_ZSTD, PQ_LZ4_RAW = 0, 1, 6, 7

DBG_COMM_ID_BYTES = 128

EXPECTED_SIZES = {
    "dbg_datatype": 8, "dbg_column": 56, "dbg_out_column": 32, "dbg_agg_spec": 16,
    "dbg_pred_node": 64, "dbg_filter": 24, "dbg_agg_params": 48, "dbg_record_layout": 328, "dbg_exchange_stats": 32,
    "dbg_parquet_chunk": 40, "dbg_native_column": 48,
}
