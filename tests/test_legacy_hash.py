"""Legacy HashMethod path (enable_experimental_aggregate_hashtable = 0).

CPU: the oracle's CRC32C primitive against the standard check value (CRC-32C("123456789") =
0xE3069283), the oracle's FixedKeys / SingleBinary FastHash against an independent pure-Python
restatement of build_keys_vec + _mm_crc32_u64 (EXP/kernels/group_by_hash/method_fixed_keys.rs:
74-100, 366-470; HT/traits.rs:172-330), and dbg_legacy_hash_method against
choose_hash_method_with_types (EXP/kernels/group_by.rs:48-97).  GPU: dbg_legacy_group_hash and its
hash2bucket<8, true> buckets against the oracle.  No reference test holds FastHash values: beyond
the CRC check value the hash bits are parity-unpinned (restatement only).
"""
import ctypes as C
import struct

import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.column import Column
from oracle import oracle

POLY = 0x82F63B78


def crc_py(crc, data):
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (POLY if crc & 1 else 0)
    return crc


def legacy_py(cols, i):
    if len(cols) == 1 and cols[0].dtype.type_id == abi.STRING and not cols[0].dtype.nullable:
        s = cols[0].values()[i]
        if not s:
            return (1 << 64) - 1
        v = 0xFFFFFFFF
        for o in range(0, len(s), 8):
            v = crc_py(v, s[o:o + 8].ljust(8, b"\0"))
        return v
    widths = [c.dtype.width for c in cols]
    total = sum(w + (1 if c.dtype.nullable else 0) for w, c in zip(widths, cols))
    if any(c.dtype.type_id in (abi.STRING, abi.BOOLEAN) for c in cols) or total > 32:
        # HashMethodSerializer: serialize_column_binary of every column, in order, as [u8]
        key = bytearray()
        for c in cols:
            valid = c.validity is None or not c.dtype.nullable or bool(c.validity[i])
            if c.dtype.nullable:
                key.append(1 if valid else 0)
            if not valid:
                continue
            if c.dtype.type_id == abi.STRING:
                s = c.values()[i]
                key += struct.pack("<Q", len(s)) + s
            elif c.dtype.type_id == abi.BOOLEAN:
                key.append(1 if c.values()[i] else 0)
            elif c.dtype.type_id == abi.DECIMAL128:
                key += bytes(np.asarray(c.data, np.uint8)[i * 16:(i + 1) * 16])
            else:
                w = c.dtype.width
                key += bytes(np.asarray(c.data).view(np.uint8).reshape(-1)[i * w:(i + 1) * w])
        if not key:
            return (1 << 64) - 1
        v = 0xFFFFFFFF
        for o in range(0, len(key), 8):
            v = crc_py(v, bytes(key[o:o + 8]).ljust(8, b"\0"))
        return v
    step = 1 if total == 1 else 2 if total == 2 else 4 if total <= 4 else 8 if total <= 8 else 16 if total <= 16 else 32
    key = bytearray(32)
    order = sorted(range(len(cols)), key=lambda j: -widths[j])  # stable
    off, noff = 0, sum(widths)
    for j in order:
        c = cols[j]
        w = widths[j]
        valid = c.validity is None or not c.dtype.nullable or bool(c.validity[i])
        if not valid:
            key[noff] = 1
        else:
            raw = np.asarray(c.data).view(np.uint8).reshape(-1)[i * w:(i + 1) * w] if c.dtype.type_id != abi.DECIMAL128 \
                else np.asarray(c.data, np.uint8)[i * 16:(i + 1) * 16]
            key[off:off + w] = bytes(raw)
        off += w
        if c.dtype.nullable:
            noff += 1
    v = 0xFFFFFFFF
    for wd in range(1 if step <= 8 else step // 8):
        v = crc_py(v, bytes(key[wd * 8:wd * 8 + 8]))
    return v


def test_crc32c_check_value():
    assert oracle.crc32c(b"123456789") ^ 0xFFFFFFFF == 0xE3069283
    assert crc_py(0xFFFFFFFF, b"123456789") ^ 0xFFFFFFFF == 0xE3069283


def _cases(rng, n):
    i16 = Column.from_numbers(col.Int16, rng.integers(-30000, 30000, n))
    u8 = Column.from_numbers(col.UInt8, rng.integers(0, 255, n), validity=rng.random(n) > 0.3)
    i64 = Column.from_numbers(col.Int64, rng.integers(-2**62, 2**62, n))
    i32n = Column.from_numbers(col.Int32, rng.integers(-2**31, 2**31 - 1, n), validity=rng.random(n) > 0.2)
    f64 = Column.from_numbers(col.Float64, rng.random(n) * 100)
    d = Column.from_decimals(20, 2, [int(x) * (1 << 40) for x in rng.integers(-1000, 1000, n)])
    dt = Column.from_numbers(col.Date, rng.integers(0, 20000, n))
    s = Column.from_strings([("abcdefghij"[: int(k)] * (1 + int(k) % 3)) for k in rng.integers(0, 11, n)])
    s2 = Column.from_strings(["RANF"[int(k) % 4] for k in rng.integers(0, 4, n)])
    sn = Column.from_strings([("xy" * int(k)) for k in rng.integers(0, 9, n)], validity=rng.random(n) > 0.25)
    b = Column.from_bools(rng.random(n) > 0.5)
    bn = Column.from_bools(rng.random(n) > 0.5, validity=rng.random(n) > 0.3)
    d38 = Column.from_decimals(38, 2, [int(x) * (1 << 70) for x in rng.integers(-1000, 1000, n)])
    # FixedKeys, SingleBinary, then HashMethodSerializer keys: two Strings (TPC-H Q1), String +
    # nullable Int32, one nullable String, Booleans, and more than 32 packed bytes
    return [[i16], [u8], [i16, u8], [i32n, u8, i16], [i64], [i64, i32n], [d], [d, i16], [f64, dt], [i64, d, u8],
            [d, i64, i32n], [s], [s, s2], [s2, i32n], [sn], [b], [bn, i16], [d38, d38, u8]]


def test_oracle_matches_python_restatement():
    rng = np.random.default_rng(3)
    for cols in _cases(rng, 40):
        got = oracle.legacy_group_hash(cols)
        for i in range(40):
            assert int(got[i]) == legacy_py(cols, i), (cols[0].dtype, i)


def test_hash_method_choice():
    from databend_amd.ffi import check, lib
    def kind(types):
        arr = (abi.dbg_datatype * len(types))(*[t.to_abi() for t in types])
        k, kb = C.c_int(), C.c_uint32()
        check(lib().dbg_legacy_hash_method(arr, len(types), C.byref(k), C.byref(kb)))
        return k.value, kb.value
    K = {1: "U8", 2: "U16", 3: "U32", 4: "U64", 5: "U128", 6: "U256", 7: "SingleBinary", 8: "Serializer"}
    assert K[kind([col.Int8])[0]] == "U8"
    assert kind([col.Int16, col.UInt8.wrap_nullable()]) == (3, 4)        # 2 + 1 + null byte
    assert kind([col.Int32, col.UInt8]) == (4, 5)                        # 5 bytes -> u64
    assert kind([col.Int64, col.Int64.wrap_nullable()]) == (6, 17)        # 8 + 8 + null byte -> U256
    assert K[kind([col.Decimal128(38, 2), col.Int64, col.Int64])[0]] == "U256"
    assert K[kind([col.String])[0]] == "SingleBinary"
    assert K[kind([col.String.wrap_nullable()])[0]] == "Serializer"
    assert K[kind([col.String, col.Int32])[0]] == "Serializer"
    assert K[kind([col.Boolean])[0]] == "Serializer"
    assert K[kind([col.Decimal128(38, 2), col.Decimal128(38, 2), col.Int8])[0]] == "Serializer"  # 33 bytes


@pytest.mark.gpu
def test_device_legacy_hash_and_buckets():
    import torch
    from databend_amd.device import DeviceColumn
    from databend_amd.ffi import check, lib
    rng = np.random.default_rng(4)
    n = 300_007
    for cols in _cases(rng, n):
        dev = [DeviceColumn.from_host(c) for c in cols]
        arr = (abi.dbg_column * len(dev))(*[d.to_abi() for d in dev])
        h = torch.empty(n, dtype=torch.int64, device="cuda")
        b = torch.empty(n, dtype=torch.int32, device="cuda")
        check(lib().dbg_legacy_group_hash(arr, len(dev), n, h.data_ptr(), b.data_ptr(), 8, None))
        exp = oracle.legacy_group_hash(cols)
        got = h.cpu().numpy().view(np.uint64)
        assert np.array_equal(got, exp), cols[0].dtype
        assert np.array_equal(b.cpu().numpy().view(np.uint32), ((exp >> np.uint64(24)) & np.uint64(255)).astype(np.uint32))
