"""CPU checks of the scan-side oracle (oracle/parquet_oracle.py) and the host half of the decoder.

The oracle restates the Parquet page decode (third-party `parquet` 52.2.0 / `snap` / `lz4_flex`
crates, absent from /root/reference).  It is pinned here by (a) pyarrow reading the files it
writes, over every codec x dictionary x page version x physical type the GPU decoder takes, and
(b) the reference's own expected outputs: select_parquet.test:2-11 for alltypes_plain.parquet and
ontime_200.csv for ontime_200.parquet (tests/golden/make_parquet_golden.py).  dbg_parquet_chunk_rows
runs on the host only (page headers), so it is checked here without a GPU.
"""
import json
import os
import struct

import pytest

from oracle import parquet_oracle as po
from tests.parquet_util import GOLDEN, expected_values, file_chunks, sample_table, write

GOLD = json.load(open(os.path.join(GOLDEN, "parquet_goldens.json")))


def oracle_values(ch, t):
    import pyarrow as pa
    rows = po.decode_chunk(ch.data, ch.physical_type, ch.codec, ch.max_def_level, ch.type_length)
    out = []
    for v in rows:
        if v is None:
            out.append(None)
        elif ch.physical_type == po.FIXED_LEN_BYTE_ARRAY:
            out.append(po.be_decimal(v))
        elif isinstance(v, float) and t == pa.float32():
            out.append(float(struct.unpack("<f", struct.pack("<f", v))[0]))
        else:
            out.append(v)
    return out


@pytest.mark.parametrize("comp", ["NONE", "SNAPPY", "LZ4"])
@pytest.mark.parametrize("dictionary", [False, True])
@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_oracle_matches_pyarrow(comp, dictionary, version):
    t = sample_table(3000)
    buf = write(t, compression=comp, use_dictionary=dictionary, data_page_version=version, data_page_size=2048)
    for name, _, ch, at in file_chunks(buf):
        got = oracle_values(ch, at)
        exp = expected_values(t.column(name), at)
        if name == "f32":
            exp = [float(struct.unpack("<f", struct.pack("<f", v))[0]) for v in exp]
        assert got == exp, (name, comp, dictionary, version)


def test_oracle_integer_decimals():
    t = sample_table(1000).select(["d9", "d20"])
    buf = write(t, store_decimal_as_integer=True, compression="SNAPPY")
    for name, _, ch, at in file_chunks(buf):
        assert ch.physical_type == (po.INT32 if name == "d9" else po.INT64) or name == "d20"
        got = oracle_values(ch, at)
        assert got == expected_values(t.column(name), at), name


def _alltypes_expected():
    g = GOLD["alltypes_plain"]
    rows = g["rows"]
    exp = {c: [r[i] for r in rows] for i, c in enumerate(g["columns"])}
    return exp


def test_oracle_alltypes_plain_matches_reference_slt():
    """select_parquet.test:2-11 — the reference's expected rows for its own fixture file."""
    buf = open(os.path.join(GOLDEN, "parquet", "alltypes_plain.parquet"), "rb").read()
    exp = _alltypes_expected()
    seen = set()
    for name, _, ch, at in file_chunks(buf):
        got = oracle_values(ch, at)
        want = exp[name]
        if name == "bool_col":
            assert got == [w == "1" for w in want]
        elif name in ("float_col", "double_col"):
            assert [round(v, 4) for v in got] == [float(w) for w in want]
        elif name in ("date_string_col", "string_col"):
            assert got == [w.encode() for w in want]
        elif name == "timestamp_col":  # INT64 nanoseconds; the SLT prints microsecond timestamps
            import datetime
            assert [datetime.datetime(1970, 1, 1) + datetime.timedelta(microseconds=v // 1000) for v in got] == \
                [datetime.datetime.strptime(w, "%Y-%m-%d %H:%M:%S.%f") for w in want]
        else:
            assert got == [int(w) for w in want], name
        seen.add(name)
    assert len(seen) == 11


ONTIME_COLS = ["Year", "Quarter", "Month", "DayofMonth", "DayOfWeek", "FlightDate", "Reporting_Airline",
               "DOT_ID_Reporting_Airline", "Tail_Number", "Flight_Number_Reporting_Airline", "OriginAirportID", "Origin",
               "OriginCityName", "DepDelay", "Distance"]


def ontime_expected(name, at):
    import pyarrow as pa
    g = GOLD["ontime_200"]
    i = g["columns"].index(name)
    raw = [r[i] for r in g["rows"]]
    if pa.types.is_string(at) or pa.types.is_large_string(at):
        return [w.encode() if w != "" else None for w in raw]
    # the file's producer stored an empty CSV number as 0 (no column of the file has NULLs)
    if pa.types.is_floating(at):
        return [float(w) if w != "" else 0.0 for w in raw]
    return [int(float(w)) if w != "" else 0 for w in raw]


def test_oracle_ontime_matches_reference_csv():
    buf = open(os.path.join(GOLDEN, "parquet", "ontime_200.parquet"), "rb").read()
    chunks = {name: (ch, at) for name, _, ch, at in file_chunks(buf)}
    for name in ONTIME_COLS:
        ch, at = chunks[name]
        got = oracle_values(ch, at)
        exp = ontime_expected(name, at)
        got = [g if not (isinstance(g, bytes) and g == b"") else None for g in got]
        assert got == exp, name


def test_chunk_rows_host_only():
    """dbg_parquet_chunk_rows parses page headers on the host: no device needed."""
    from databend_amd.scan import ParquetChunkDecoder
    t = sample_table(5000)
    for comp, ver in [("SNAPPY", "1.0"), ("NONE", "2.0"), ("LZ4", "1.0")]:
        buf = write(t, compression=comp, data_page_version=ver, data_page_size=1024)
        for name, _, ch, at in file_chunks(buf):
            assert ParquetChunkDecoder.chunk_rows(ch) == 5000, name
    buf = open(os.path.join(GOLDEN, "parquet", "ontime_200.parquet"), "rb").read()
    for name, _, ch, at in file_chunks(buf):
        assert ParquetChunkDecoder.chunk_rows(ch) == 199


def test_chunk_rows_rejects_truncated_header():
    from databend_amd.ffi import DbgError
    from databend_amd.scan import ParquetChunkDecoder
    t = sample_table(100)
    _, _, ch, _ = file_chunks(write(t, compression="NONE"))[0]
    ch.data = ch.data[:7]
    with pytest.raises(DbgError):
        ParquetChunkDecoder.chunk_rows(ch)
