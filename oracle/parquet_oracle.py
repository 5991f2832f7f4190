"""CPU restatement of the scan-side decode — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (databend_amd/csrc/scan.hip, dbg_parquet_decode) never does.

What it restates: one Parquet column chunk (the bytes a Fuse block holds for one leaf column,
BlockReader::deserialize_parquet_chunks -> column_chunks_to_record_batch,
src/query/storages/fuse/src/io/read/block/parquet/mod.rs:45-60, deserialize.rs:33-80) decoded
to a Databend column.  The decode itself lives in third-party crates that are absent from
/root/reference: `parquet` 52.2.0 (arrow-rs; Cargo.lock:11199), `snap` 1.1.1 (Cargo.lock:14017)
and `lz4_flex` 0.11.3 (Cargo.lock:9889).  Their published algorithms, restated here:
  * PageHeader in the Thrift compact protocol (parquet-format `parquet.thrift`);
  * DATA_PAGE (v1: [rep levels][def levels with a 4-byte length] then values, all compressed
    together), DATA_PAGE_V2 (levels uncompressed in front, values compressed unless
    is_compressed = false), DICTIONARY_PAGE (PLAIN values);
  * the RLE / bit-packed hybrid (definition levels; dictionary indices after a bit-width byte);
  * PLAIN: little-endian fixed width, BOOLEAN bit-packed LSB first, BYTE_ARRAY as u32 length +
    bytes, FIXED_LEN_BYTE_ARRAY big-endian decimals;
  * Snappy raw blocks and LZ4 raw blocks.
Pinning: pyarrow 25 (the Arrow C++ reader) on files it writes with every codec / encoding /
page version, and the reference's own test data files (tests/data/parquet/*.parquet, copied as
fixtures into tests/golden/parquet/), whose expected values are in
tests/golden/parquet_goldens.json (tests/golden/make_parquet_golden.py).
Pure-Python loops: small inputs only.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

# parquet::Type
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
# parquet::CompressionCodec
UNCOMPRESSED, SNAPPY, GZIP, LZO, BROTLI, LZ4, ZSTD, LZ4_RAW = range(8)
# parquet::Encoding
PLAIN, PLAIN_DICTIONARY, RLE, BIT_PACKED, DELTA_BINARY_PACKED = 0, 2, 3, 4, 5
RLE_DICTIONARY = 8
# parquet::PageType
DATA_PAGE, INDEX_PAGE, DICTIONARY_PAGE, DATA_PAGE_V2 = range(4)


# ---- Thrift compact protocol (just what PageHeader needs) ----
class _Compact:
    def __init__(self, buf: bytes, pos: int = 0):
        self.b = buf
        self.p = pos

    def byte(self) -> int:
        v = self.b[self.p]
        self.p += 1
        return v

    def varint(self) -> int:
        shift = v = 0
        while True:
            c = self.byte()
            v |= (c & 0x7F) << shift
            if not c & 0x80:
                return v
            shift += 7

    def zigzag(self) -> int:
        v = self.varint()
        return (v >> 1) ^ -(v & 1)

    def skip(self, t: int):
        if t in (1, 2):  # bool true / false (in-field)
            return
        if t == 3:
            self.p += 1
        elif t in (4, 5, 6):
            self.varint()
        elif t == 7:
            self.p += 8
        elif t == 8:
            n = self.varint()
            self.p += n
        elif t in (9, 10):
            h = self.byte()
            n = h >> 4
            if n == 15:
                n = self.varint()
            et = h & 15
            for _ in range(n):
                self.skip(et)
        elif t == 12:
            self.struct(lambda fid, ft: False)
        else:
            raise ValueError(f"thrift compact: type {t}")

    def struct(self, on_field):
        """Walk one struct; on_field(fid, ftype) reads the value and returns True, or False to skip."""
        last = 0
        while True:
            h = self.byte()
            if h == 0:
                return
            delta, t = h >> 4, h & 15
            fid = last + delta if delta else self.zigzag()
            last = fid
            if t in (1, 2):
                if not on_field(fid, t):
                    pass
                continue
            if not on_field(fid, t):
                self.skip(t)


@dataclass
class Page:
    ptype: int
    uncompressed: int
    compressed: int
    data_off: int           # offset of the page payload in the chunk
    num_values: int = 0
    encoding: int = PLAIN
    def_len: int = 0        # v2: definition level bytes
    rep_len: int = 0
    v2_compressed: bool = True


def parse_pages(chunk: bytes) -> List[Page]:
    pages = []
    pos = 0
    while pos < len(chunk):
        r = _Compact(chunk, pos)
        hdr = {}

        def sub(fields):
            def on(fid, t):
                if t in (5, 6):
                    fields[fid] = r.zigzag()
                    return True
                if t in (1, 2):
                    fields[fid] = t == 1
                    return True
                return False
            return on

        def on_top(fid, t):
            if fid in (1, 2, 3, 4) and t == 5:
                hdr[fid] = r.zigzag()
                return True
            if fid in (5, 7, 8) and t == 12:
                f = {}
                r.struct(sub(f))
                hdr[fid] = f
                return True
            return False

        r.struct(on_top)
        p = Page(hdr[1], hdr[2], hdr[3], r.p)
        if p.ptype == DATA_PAGE:
            d = hdr[5]
            p.num_values, p.encoding = d[1], d[2]
        elif p.ptype == DICTIONARY_PAGE:
            d = hdr[7]
            p.num_values, p.encoding = d[1], d[2]
        elif p.ptype == DATA_PAGE_V2:
            d = hdr[8]
            p.num_values, p.encoding = d[1], d[4]
            p.def_len, p.rep_len = d[5], d[6]
            p.v2_compressed = d.get(7, True)
        pages.append(p)
        pos = r.p + p.compressed
    return pages


# ---- codecs ----
def _uvarint(b: bytes, p: int) -> Tuple[int, int]:
    v = s = 0
    while True:
        c = b[p]
        p += 1
        v |= (c & 0x7F) << s
        if not c & 0x80:
            return v, p
        s += 7


def snappy_decompress(b: bytes) -> bytes:
    n, p = _uvarint(b, 0)
    out = bytearray()
    while p < len(b):
        tag = b[p]
        p += 1
        kind = tag & 3
        if kind == 0:  # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(b[p:p + nb], "little")
                p += nb
            ln += 1
            out += b[p:p + ln]
            p += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | b[p]
            p += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(b[p:p + 2], "little")
            p += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(b[p:p + 4], "little")
            p += 4
        for _ in range(ln):  # overlapping copies repeat the pattern
            out.append(out[-off])
    assert len(out) == n, "snappy: length mismatch"
    return bytes(out)


def lz4_raw_decompress(b: bytes, n: int) -> bytes:
    out = bytearray()
    p = 0
    while p < len(b):
        tok = b[p]
        p += 1
        ln = tok >> 4
        if ln == 15:
            while True:
                c = b[p]
                p += 1
                ln += c
                if c != 255:
                    break
        out += b[p:p + ln]
        p += ln
        if p >= len(b):
            break
        off = b[p] | (b[p + 1] << 8)
        p += 2
        ml = tok & 15
        if ml == 15:
            while True:
                c = b[p]
                p += 1
                ml += c
                if c != 255:
                    break
        ml += 4
        for _ in range(ml):
            out.append(out[-off])
    assert len(out) == n, "lz4: length mismatch"
    return bytes(out)


def decompress(codec: int, b: bytes, n: int) -> bytes:
    if codec == UNCOMPRESSED:
        return b
    if codec == SNAPPY:
        return snappy_decompress(b)
    if codec == LZ4_RAW:
        return lz4_raw_decompress(b, n)
    if codec == ZSTD:
        # Fuse's default page codec.  The reference decodes it with the `zstd` crate (0.12.4 /
        # 0.13.2 over zstd-sys, i.e. libzstd; Cargo.lock); not restated here: the checker is
        # libzstd itself, as pyarrow 25 bundles it.  The device decoder (scan.hip,
        # zstd_dev.hpp) is the independent restatement of RFC 8878 under test.
        import pyarrow as pa
        out = pa.decompress(b, decompressed_size=n, codec="zstd", asbytes=True)
        assert len(out) == n, "zstd: length mismatch"
        return out
    raise NotImplementedError(f"codec {codec}")


# ---- RLE / bit-packed hybrid ----
def rle_hybrid(b: bytes, p: int, end: int, bw: int, n: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.uint32)
    k = 0
    vb = (bw + 7) // 8
    while k < n and p < end:
        h, p = _uvarint(b, p)
        if h & 1:  # bit-packed: (h >> 1) groups of 8 values, LSB first
            cnt = (h >> 1) * 8
            nbytes = (h >> 1) * bw
            bits = int.from_bytes(b[p:p + nbytes], "little")
            p += nbytes
            for j in range(cnt):
                if k < n:
                    out[k] = (bits >> (j * bw)) & ((1 << bw) - 1)
                k += 1
        else:
            cnt = h >> 1
            v = int.from_bytes(b[p:p + vb], "little")
            p += vb
            m = min(cnt, n - k)
            out[k:k + m] = v
            k += cnt
    return out


@dataclass
class Decoded:
    values: list                         # python values per row (None = NULL)


def _plain(buf: bytes, p: int, ptype: int, tlen: int, n: int):
    vals = []
    if ptype == BOOLEAN:
        for k in range(n):
            vals.append(bool((buf[p + k // 8] >> (k % 8)) & 1))
        return vals, p + (n + 7) // 8
    if ptype == BYTE_ARRAY:
        for _ in range(n):
            ln = int.from_bytes(buf[p:p + 4], "little")
            vals.append(bytes(buf[p + 4:p + 4 + ln]))
            p += 4 + ln
        return vals, p
    if ptype == FIXED_LEN_BYTE_ARRAY:
        for _ in range(n):
            vals.append(bytes(buf[p:p + tlen]))
            p += tlen
        return vals, p
    fmt, w = {INT32: ("<i", 4), INT64: ("<q", 8), FLOAT: ("<f", 4), DOUBLE: ("<d", 8)}[ptype]
    for _ in range(n):
        vals.append(struct.unpack_from(fmt, buf, p)[0])
        p += w
    return vals, p


def decode_chunk(chunk: bytes, ptype: int, codec: int, max_def: int, tlen: int = 0) -> list:
    """Physical values per row (None for NULL), pages in order."""
    dictionary = None
    rows: list = []
    for pg in parse_pages(chunk):
        raw = chunk[pg.data_off:pg.data_off + pg.compressed]
        if pg.ptype == DICTIONARY_PAGE:
            buf = decompress(codec, raw, pg.uncompressed)
            dictionary, _ = _plain(buf, 0, ptype, tlen, pg.num_values)
            continue
        if pg.ptype == INDEX_PAGE:
            continue
        if pg.ptype == DATA_PAGE_V2:
            lv = pg.rep_len + pg.def_len
            body = raw[lv:]
            body = decompress(codec, body, pg.uncompressed - lv) if pg.v2_compressed else body
            buf = raw[:lv] + body
            dp, de = pg.rep_len, pg.rep_len + pg.def_len
            vp = lv
        else:
            buf = decompress(codec, raw, pg.uncompressed)
            p = 0
            if max_def:
                ln = int.from_bytes(buf[0:4], "little")
                dp, de = 4, 4 + ln
                vp = de
            else:
                dp = de = vp = 0
        n = pg.num_values
        defs = rle_hybrid(buf, dp, de, 1, n) if max_def else np.ones(n, dtype=np.uint32)
        nn = int(defs.sum())
        if pg.encoding in (PLAIN_DICTIONARY, RLE_DICTIONARY):
            bw = buf[vp]
            idx = rle_hybrid(buf, vp + 1, len(buf), bw, nn) if bw else np.zeros(nn, dtype=np.uint32)
            vals = [dictionary[i] for i in idx]
        elif pg.encoding == PLAIN:
            vals, _ = _plain(buf, vp, ptype, tlen, nn)
        elif pg.encoding == RLE and ptype == BOOLEAN:  # 4-byte length, then the hybrid at width 1
            ln = int.from_bytes(buf[vp:vp + 4], "little")
            vals = [bool(v) for v in rle_hybrid(buf, vp + 4, vp + 4 + ln, 1, nn)]
        else:
            raise NotImplementedError(f"encoding {pg.encoding}")
        it = iter(vals)
        rows.extend(next(it) if d else None for d in defs)
    return rows


def be_decimal(b: bytes) -> int:
    return int.from_bytes(b, "big", signed=True)
