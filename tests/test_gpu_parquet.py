"""GPU parity of the scan-side decode (dbg_parquet_decode, scan.hip) against the oracle
(oracle/parquet_oracle.py, pinned by pyarrow and by the reference's own expected outputs —
tests/test_parquet_oracle.py), and a Parquet -> HBM -> GROUP BY pipeline against the aggregation
oracle.  Every codec x dictionary x page version x physical type; the reference's fixture files;
multi-page chunks; malformed and unsupported chunks (errors, never faults)."""
import json
import os
import struct

import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.ffi import DbgError, Unsupported
from databend_amd.scan import ColumnChunk, ParquetChunkDecoder, deserialize_parquet_chunks
from tests.parquet_util import GOLDEN, expected_values, file_chunks, sample_table, target_of, write
from tests.test_parquet_oracle import ONTIME_COLS, _alltypes_expected, ontime_expected, oracle_values

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec():
    d = ParquetChunkDecoder()
    yield d
    d.close()


def gpu_values(dec, ch, at, nullable=True):
    t = target_of(at, nullable)
    c = dec.decode(ch, t).to_host()
    v = c.values()
    if at is not None and str(at) == "float":
        v = [None if x is None else float(struct.unpack("<f", struct.pack("<f", x))[0]) for x in v]
    return v


def check_file(dec, buf, names=None):
    n = 0
    for name, _, ch, at in file_chunks(buf):
        if names and name not in names:
            continue
        got = gpu_values(dec, ch, at)
        exp = oracle_values(ch, at)
        assert got == exp, (name, [(i, a, b) for i, (a, b) in enumerate(zip(got, exp)) if a != b][:5])
        n += 1
    return n


@pytest.mark.parametrize("comp", ["NONE", "SNAPPY", "LZ4", "ZSTD"])
@pytest.mark.parametrize("dictionary", [False, True])
@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_decode_matches_oracle(dec, comp, dictionary, version):
    t = sample_table(6_000, seed=7)
    buf = write(t, compression=comp, use_dictionary=dictionary, data_page_version=version, data_page_size=4096)
    assert check_file(dec, buf) == t.num_columns


def test_fuse_writer_shape_large(dec):
    """blocks_to_parquet's shape (one row group, PLAIN, no dictionary; parquet_rs.rs:36-44) at
    several hundred pages per chunk, every codec the GPU takes."""
    t = sample_table(400_000, seed=3).select(["i16", "i64", "s", "d20", "b"])
    for comp in ["NONE", "SNAPPY", "LZ4", "ZSTD"]:
        buf = write(t, compression=comp, use_dictionary=False, row_group_size=1 << 30)
        n = 0
        for name, _, ch, at in file_chunks(buf):  # at this size against pyarrow (which pins the oracle)
            assert gpu_values(dec, ch, at) == expected_values(t.column(name), at), (comp, name)
            n += 1
        assert n == 5


@pytest.mark.parametrize("comp", ["SNAPPY", "LZ4"])
def test_far_back_references(dec, comp):
    """Matches farther back than the inflate kernel's 32 KiB LDS ring (read back from the page's
    own output in HBM), including an LZ4 match longer than its offset: a random 40 000-byte block
    repeated, then a 60 000-byte one with a few values changed.  pyarrow's LZ4 writes the first
    page as one literal and one 119 995-byte match at offset 40 000; its Snappy skips ahead in
    random bytes and finds none (that leg checks the literal path on the same data)."""
    import pyarrow as pa
    rng = np.random.default_rng(11)
    a = rng.integers(-2**62, 2**62, 5_000)
    b = rng.integers(-2**62, 2**62, 7_500)
    b2 = b.copy()
    b2[::997] += 1
    v = np.concatenate([a, a, a, a, b, rng.integers(0, 7, 3_000), b2, a])
    t = pa.table({"x": pa.array(v, pa.int64())}, schema=pa.schema([pa.field("x", pa.int64(), nullable=False)]))
    buf = write(t, compression=comp, use_dictionary=False, data_page_size=1 << 20, row_group_size=1 << 30)
    (name, _, ch, at), = file_chunks(buf)
    assert gpu_values(dec, ch, at, nullable=False) == v.tolist()


def test_integer_decimals(dec):
    t = sample_table(5000).select(["d9", "d20"])
    buf = write(t, store_decimal_as_integer=True, compression="SNAPPY")
    assert check_file(dec, buf) == 2


def test_reference_alltypes_plain(dec):
    """alltypes_plain.parquet decoded on the GPU equals select_parquet.test:2-11."""
    buf = open(os.path.join(GOLDEN, "parquet", "alltypes_plain.parquet"), "rb").read()
    exp = _alltypes_expected()
    for name, _, ch, at in file_chunks(buf):
        got = gpu_values(dec, ch, at)
        want = exp[name]
        if name == "bool_col":
            assert got == [w == "1" for w in want]
        elif name in ("float_col", "double_col"):
            assert [round(v, 4) for v in got] == [float(w) for w in want]
        elif name in ("date_string_col", "string_col"):
            assert got == [w.encode() for w in want]
        elif name == "timestamp_col":
            assert got == oracle_values(ch, at)
        else:
            assert got == [int(w) for w in want], name


def test_reference_ontime(dec):
    """ontime_200.parquet (dictionary pages, SNAPPY) decoded on the GPU equals ontime_200.csv."""
    buf = open(os.path.join(GOLDEN, "parquet", "ontime_200.parquet"), "rb").read()
    chunks = {name: (ch, at) for name, _, ch, at in file_chunks(buf)}
    for name in ONTIME_COLS:
        ch, at = chunks[name]
        got = gpu_values(dec, ch, at)
        got = [g if not (isinstance(g, bytes) and g == b"") else None for g in got]
        assert got == ontime_expected(name, at), name
    # every other decodable column against the oracle
    n = 0
    for name, (ch, at) in chunks.items():
        try:
            target_of(at)
        except KeyError:
            continue
        assert gpu_values(dec, ch, at) == oracle_values(ch, at), name
        n += 1
    assert n > 80


def test_pipeline_parquet_to_group_by(dec):
    """Fuse-shaped Parquet of the C2 column -> HBM columns -> GPU GROUP BY == oracle."""
    import pyarrow as pa
    from databend_amd.aggregates import AggregateFunctionFactory
    from databend_amd.aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
    from databend_amd.filter import FilterProgram, cmp
    from oracle import oracle
    from tests.parity import assert_results_equal
    rng = np.random.default_rng(5)
    n = 2_000_000
    adv = np.where(rng.random(n) < 0.99, 0, rng.integers(1, 33, n)).astype(np.int16)
    uid = rng.integers(0, 1000, n)
    t = pa.table({"AdvEngineID": adv, "UserID": uid})
    buf = write(t, compression="SNAPPY", use_dictionary=False, row_group_size=1 << 30)
    fields = {0: col.Int16, 1: col.Int64}
    chunks = {i: ch for i, (name, _, ch, at) in enumerate(file_chunks(buf))}
    cols = deserialize_parquet_chunks(n, fields, chunks, dec)
    F = AggregateFunctionFactory.instance()
    fns = [F.get("count"), F.get("sum", [], [col.Int64])]
    ht = AggregateHashTable(AggregatorParams([col.Int16], fns), HashTableConfig(True))
    dadv, duid = cols[0], cols[1]
    ht.add_groups([dadv], [None, duid], rows=n, filter_program=FilterProgram(cmp(0, "<>", 0), [dadv.to_abi()]), on_device=True)
    block = ht.merge_result()
    ht.close()
    hadv, huid = col.Column.from_numbers(col.Int16, adv), col.Column.from_numbers(col.Int64, uid)
    specs = [(f.to_abi(), c) for f, c in zip(fns, [None, huid])]
    ok, oa = oracle.aggregate([hadv], specs, filter_program=FilterProgram(cmp(0, "<>", 0), [hadv.to_abi()]), threads=4)
    assert_results_equal(block.columns[2:], block.columns[:2], ok, oa)


def test_errors_not_faults(dec):
    t = sample_table(3000).select(["i64", "s"])
    buf = write(t, compression="SNAPPY", use_dictionary=False, data_page_size=4096)
    (_, _, ch, at), (_, _, chs, ats) = file_chunks(buf)
    # corrupt compressed bytes (headers intact): decode error, no fault
    pages = __import__("oracle.parquet_oracle", fromlist=["x"]).parse_pages(ch.data)
    bad = bytearray(ch.data)
    p = pages[0]
    for j in range(p.data_off + 2, p.data_off + min(p.compressed, 40)):
        bad[j] = 0xFF
    with pytest.raises(DbgError):
        dec.decode(ColumnChunk(bytes(bad), ch.physical_type, ch.max_def_level, 0, ch.codec), target_of(at))
    bad = bytearray(chs.data)
    for j in range(pages[0].data_off, min(len(bad), pages[0].data_off + 64)):
        bad[j] = 0x7F
    with pytest.raises(DbgError):
        dec.decode(ColumnChunk(bytes(bad), chs.physical_type, chs.max_def_level, 0, chs.codec), target_of(ats))
    # a Snappy literal whose 4-byte length is near 2^32: the bounds checks must not wrap (an
    # out-of-bounds device write otherwise), the page is rejected as malformed
    bad = bytearray(ch.data)
    q = p.data_off
    while bad[q] & 0x80:  # skip the uncompressed-length varint
        q += 1
    bad[q + 1:q + 6] = bytes([0xFC, 0xFE, 0xFF, 0xFF, 0xFF])
    with pytest.raises(DbgError):
        dec.decode(ColumnChunk(bytes(bad), ch.physical_type, ch.max_def_level, 0, ch.codec), target_of(at))
    # codecs the GPU does not take: the caller keeps the CPU reader
    with pytest.raises(Unsupported):
        dec.decode(ColumnChunk(ch.data, ch.physical_type, ch.max_def_level, 0, 4), target_of(at))  # BROTLI
    # a corrupted ZSTD page: an error, no fault
    tz = sample_table(3000).select(["i64", "s"])
    bz = write(tz, compression="ZSTD", use_dictionary=False, data_page_size=4096)
    (_, _, chz, atz), _ = file_chunks(bz)
    pz = __import__("oracle.parquet_oracle", fromlist=["x"]).parse_pages(chz.data)
    bad = bytearray(chz.data)
    for j in range(pz[0].data_off + 6, pz[0].data_off + min(pz[0].compressed, 60)):
        bad[j] ^= 0x5A
    with pytest.raises(DbgError):
        dec.decode(ColumnChunk(bytes(bad), chz.physical_type, chz.max_def_level, 0, chz.codec), target_of(atz))
    # a physical type that does not convert to the target
    with pytest.raises(Unsupported):
        dec.decode(ch, col.String)
    # NULLs into a non-nullable target
    t2 = sample_table(3000).select(["i16"])
    (_, _, c2, a2), = file_chunks(write(t2, compression="NONE"))
    with pytest.raises(DbgError):
        dec.decode(c2, target_of(a2, nullable=False))
    # the decoder is still usable afterwards
    assert check_file(dec, buf) == 2


@pytest.mark.parametrize("comp", ["NONE", "SNAPPY", "ZSTD"])
def test_required_plain_vectorised(dec, comp):
    """Required (non-null) PLAIN 4- and 8-byte physical values — the vectorised decode path: four
    values per lane from aligned dword loads with funnel shifts (page value sections start at any
    byte), narrowed to the target width — over many small pages, ragged page sizes and every
    narrowing the targets allow, against pyarrow."""
    import pyarrow as pa
    rng = np.random.default_rng(21)
    n = 300_007
    cols = {
        "i8": pa.array(rng.integers(-128, 128, n).astype(np.int8)),
        "u8": pa.array(rng.integers(0, 256, n).astype(np.uint8)),
        "i16": pa.array(rng.integers(-32768, 32768, n).astype(np.int16)),
        "u16": pa.array(rng.integers(0, 65536, n).astype(np.uint16)),
        "i32": pa.array(rng.integers(-2**31, 2**31, n).astype(np.int32)),
        "u32": pa.array(rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)),
        "i64": pa.array(rng.integers(-2**62, 2**62, n)),
        "f32": pa.array(rng.random(n).astype(np.float32)),
        "f64": pa.array(rng.random(n)),
    }
    schema = pa.schema([pa.field(k, v.type, nullable=False) for k, v in cols.items()])
    t = pa.table(list(cols.values()), schema=schema)
    for page in (1000, 4093, 65536):
        buf = write(t, compression=comp, use_dictionary=False, data_page_size=page, row_group_size=1 << 30)
        m = 0
        for name, _, ch, at in file_chunks(buf):
            got = gpu_values(dec, ch, at, nullable=False)
            assert got == expected_values(t.column(name), at), (comp, page, name)
            m += 1
        assert m == len(cols)
