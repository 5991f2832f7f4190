"""CPU restatement of Databend's native (strawboat) column format — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (databend_amd/csrc/scan.hip, dbg_native_decode) never does.

A Fuse table with `storage_format = 'native'` stores each leaf column of a block as pages written
by NativeWriter (src/common/arrow/src/native/write/writer.rs:113-127, common.rs:46-110: pages of
max_page_size = 131072 rows, fuse/src/constants.rs:35) and read back by NativeReader /
column_iter_to_arrays (fuse/src/io/read/block/block_reader_native_deserialize.rs:23-26).  One
page of a non-nested column (write/serialize.rs:54-150):

  [validity, Optional fields only: u32 byte length, then the definition levels as ONE bit-packed
   hybrid run — uleb128((ceil8(n) << 1) | 1) + LSB-first bitmap (parquet2 encode_bool,
   arrow/io/parquet/write/utils.rs:61-74); length 0 = no validity]
  [values]

values of an integer column (compression/integer/mod.rs:49-79): [codec u8][compressed u32]
[uncompressed u32][payload]; codecs (compression/mod.rs:34-93):
  0 None / 1 Lz4 (raw block) / 2 Zstd (frame) / 3 Snappy (raw): the little-endian values;
  10 Rle (integer/rle.rs:59-92): runs [u32 count][value], nulls extend the current run;
  11 Dict (integer/dict.rs:34-61): the u32 indices as a nested integer block (any codec but
     Dict), then [u32 count][count values];
  12 OneValue (integer/one_value.rs:58-71): one value;
  13 Freq (integer/freq.rs:33-80): top value, roaring bitmap of exceptions, nested block;
  14 Bitpacking (integer/bp.rs:40-59), 15 DeltaBitpacking (integer/delta_bp.rs:40-66): 4-byte
     values in blocks of 128, each [u8 num_bits][BitPacker4x block] (delta: from the previous
     value, the first block's from 0).
values of a String (LargeUtf8) column (compression/binary/mod.rs:37-104): Basic codecs write TWO
blocks — the (n + 1) zero-based i64 offsets, then the bytes — each [codec][comp][uncomp][payload];
OneValue (binary/one_value.rs:48-58) [u32 len][bytes]; Dict (binary/dict.rs:54-85) the nested u32
index block, [u32 count], per entry [u64 len][bytes]; Freq (binary/freq.rs).
Float32 / Float64 columns (compression/double/mod.rs:45-120) use the integer layouts of their bits
(basic, Rle, Dict, OneValue; no bit-packing) plus Freq / Patas; Boolean columns
(compression/boolean/mod.rs:35-103) the basic codecs over the LSB-first bitmap — the uncompressed
field then holds the row count — plus Rle ([u32 count][u8 value]) and OneValue (one byte).

BitPacker4x is the `bitpacking` crate (0.8.x, src/common/arrow/Cargo.toml:95; absent from
/root/reference): the simdcomp 4-lane layout — value i of a 128-value block is lane i % 4, slot
i / 4; each lane packs its 32 slots LSB-first into num_bits 32-bit words, and 128-bit output word
w holds word w of lanes 0..3; num_bits = bits of the block's OR (of the raw values, also for
delta, as delta_bp.rs:45 computes it); deltas are v[i] - v[i - 1] in value order.
The writer's choice (choose_compressor, integer/mod.rs:230-300) samples with a thread RNG, so the
bytes a reference writer produces are not reproducible; `choose_codec` restates the rule on the
full page (no sampling) and the tests also force every codec.  No reference test or fixture holds
native bytes: parity is "unpinned" beyond this restatement.  Pure-Python loops:
small inputs only.
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence, Tuple

import numpy as np

NONE, LZ4, ZSTD, SNAPPY = 0, 1, 2, 3
RLE, DICT, ONE_VALUE, FREQ, BITPACK, DELTA_BITPACK, PATAS = 10, 11, 12, 13, 14, 15, 16
BASIC = (NONE, LZ4, ZSTD, SNAPPY)
PAGE_ROWS = 131072  # DEFAULT_ROW_PER_PAGE (fuse/src/constants.rs:35)
DEFAULT_RATIO = 2.10  # block_writer.rs:83-86 (3.72 under TableCompression::Zstd)

# 16: Decimal128's i128 pages (write/primitive.rs:67-70, compress_integer over i128) as opaque
# little-endian 16-byte values
_I128 = np.dtype([("lo", "<u8"), ("hi", "<u8")])
_NP = {1: (np.int8, np.uint8), 2: (np.int16, np.uint16), 4: (np.int32, np.uint32), 8: (np.int64, np.uint64),
       16: (_I128, _I128)}


def _dtype(width: int, signed: bool):
    if width == 16:
        return _I128
    return np.dtype(_NP[width][0 if signed else 1]).newbyteorder("<")


# ---- basic codecs (pyarrow's codecs: the same lz4 block / zstd frame / snappy raw formats) ----
def _codec_name(c: int) -> str:
    return {LZ4: "lz4_raw", ZSTD: "zstd", SNAPPY: "snappy"}[c]


def basic_compress(c: int, raw: bytes) -> bytes:
    if c == NONE:
        return bytes(raw)
    import pyarrow as pa
    return pa.Codec(_codec_name(c)).compress(raw, asbytes=True)


def basic_decompress(c: int, payload: bytes, n: int) -> bytes:
    if c == NONE:
        return bytes(payload)
    import pyarrow as pa
    return pa.Codec(_codec_name(c)).decompress(payload, decompressed_size=n, asbytes=True)


def _block(codec: int, payload: bytes, uncomp: int) -> bytes:
    return struct.pack("<BII", codec, len(payload), uncomp) + payload


# ---- BitPacker4x (bitpacking crate, simdcomp layout) ----
def bp4x_pack(vals: np.ndarray, nbits: int, initial: Optional[int] = None) -> bytes:
    v = np.zeros(128, np.uint64)
    v[:len(vals)] = np.asarray(vals, np.uint64) & np.uint64(0xFFFFFFFF)
    if initial is not None:  # compress_sorted: deltas in value order, the first from `initial`
        prev = np.concatenate([[np.uint64(initial)], v[:-1]])
        v = (v - prev) & np.uint64(0xFFFFFFFF)
    out = np.zeros(4 * nbits, np.uint64)
    if nbits:
        for i in range(128):
            lane, slot = i % 4, i // 4
            bp = slot * nbits
            w, s = bp // 32, bp % 32
            out[4 * w + lane] |= (int(v[i]) << s) & 0xFFFFFFFF
            if s + nbits > 32:
                out[4 * (w + 1) + lane] |= int(v[i]) >> (32 - s)
    return (out & np.uint64(0xFFFFFFFF)).astype("<u4").tobytes()


def bp4x_unpack(buf: bytes, p: int, nbits: int, initial: Optional[int] = None) -> np.ndarray:
    words = np.frombuffer(buf, "<u4", 4 * nbits, p).astype(np.uint64) if nbits else np.zeros(0, np.uint64)
    v = np.zeros(128, np.uint64)
    mask = (1 << nbits) - 1
    for i in range(128):
        if not nbits:
            break
        lane, slot = i % 4, i // 4
        bp = slot * nbits
        w, s = bp // 32, bp % 32
        x = int(words[4 * w + lane]) >> s
        if s + nbits > 32:
            x |= int(words[4 * (w + 1) + lane]) << (32 - s)
        v[i] = x & mask
    if initial is not None:
        v = (np.cumsum(v, dtype=np.uint64) + np.uint64(initial)) & np.uint64(0xFFFFFFFF)
    return v


def _num_bits(chunk: np.ndarray) -> int:
    o = int(np.bitwise_or.reduce(np.asarray(chunk, np.uint64))) if len(chunk) else 0
    return o.bit_length()


# ---- integer blocks ----
def encode_int_block(vals: np.ndarray, width: int, codec: int, valid: Optional[np.ndarray] = None,
                     basic: int = NONE, nested: int = NONE) -> bytes:
    """[codec][compressed u32][uncompressed u32][payload] of `vals` (width bytes each)."""
    n = len(vals)
    raw = np.asarray(vals).astype(_dtype(width, True) if np.asarray(vals).dtype.kind == "i" else _dtype(width, False))
    uncomp = n * width
    if codec in BASIC:
        return _block(codec, basic_compress(codec, raw.tobytes()), uncomp)
    if codec == ONE_VALUE:
        first = next((i for i in range(n) if valid is None or valid[i]), None)
        val = raw[first:first + 1].tobytes() if first is not None else bytes(width)
        return _block(codec, val, uncomp)
    if codec == RLE:
        out = bytearray()
        cnt, last, all_null = 0, None, True
        for i in range(n):
            if valid is None or valid[i]:
                x = raw[i:i + 1].tobytes()
                if all_null:
                    all_null, last, cnt = False, x, cnt + 1
                elif x != last:
                    out += struct.pack("<I", cnt) + last
                    last, cnt = x, 1
                else:
                    cnt += 1
            else:
                cnt += 1
        if cnt:
            out += struct.pack("<I", cnt) + (last if last is not None else bytes(width))
        return _block(codec, bytes(out), uncomp)
    if codec == DICT:
        sets, index, idx = [], {}, []
        for i in range(n):
            if valid is not None and not valid[i]:
                if not idx:
                    key = bytes(width)
                else:
                    idx.append(idx[-1])
                    continue
            else:
                key = raw[i:i + 1].tobytes()
            if key not in index:
                index[key] = len(sets)
                sets.append(key)
            idx.append(index[key])
        inner = encode_int_block(np.asarray(idx, np.uint32), 4, nested)
        payload = inner + struct.pack("<I", len(sets)) + b"".join(sets)
        return _block(codec, payload, uncomp)
    if codec in (BITPACK, DELTA_BITPACK):
        assert width == 4
        u = raw.view(np.uint32).astype(np.uint64)
        out, initial = bytearray(), 0
        for b0 in range(0, n, 128):
            ch = u[b0:b0 + 128]
            nb = _num_bits(ch)
            out.append(nb)
            out += bp4x_pack(ch, nb, initial if codec == DELTA_BITPACK else None)
            initial = int(ch[-1])
        return _block(codec, bytes(out), uncomp)
    raise ValueError(f"codec {codec}")


def decode_int_block(buf: bytes, p: int, n: int, width: int, signed: bool) -> Tuple[np.ndarray, int]:
    """Decode one integer block at p -> (n values, end position)."""
    codec, comp, uncomp = struct.unpack_from("<BII", buf, p)
    q = p + 9
    end = q + comp
    dt = _dtype(width, signed)
    if codec in BASIC:
        raw = basic_decompress(codec, buf[q:end], n * width)
        return np.frombuffer(raw, dt, n).copy(), end
    if codec == ONE_VALUE:
        return np.full(n, np.frombuffer(buf, dt, 1, q)[0], dt), end
    if codec == RLE:
        out, k = [], 0
        while k < n:  # rle.rs:96-121 reads runs until n values
            cnt = struct.unpack_from("<I", buf, q)[0]
            v = np.frombuffer(buf, dt, 1, q + 4)[0]
            out.append(np.full(cnt, v, dt))
            k += cnt
            q += 4 + width
        return np.concatenate(out)[:n] if out else np.zeros(0, dt), end
    if codec == DICT:
        idx, q = decode_int_block(buf, q, n, 4, False)
        cnt = struct.unpack_from("<I", buf, q)[0]
        d = np.frombuffer(buf, dt, cnt, q + 4)
        return d[idx.astype(np.int64)].copy(), end
    if codec in (BITPACK, DELTA_BITPACK):
        out, initial = [], 0
        for _ in range(0, n, 128):
            nb = buf[q]
            v = bp4x_unpack(buf, q + 1, nb, initial if codec == DELTA_BITPACK else None)
            out.append(v)
            initial = int(v[-1])
            q += 1 + 16 * nb
        u = np.concatenate(out)[:n].astype(np.uint32)
        return u.view(dt), end
    raise NotImplementedError(f"native codec {codec} (Freq / Patas) is not restated")


# ---- String (LargeUtf8) blocks ----
def encode_binary_block(vals: Sequence[bytes], codec: int, valid: Optional[np.ndarray] = None, nested: int = NONE) -> bytes:
    n = len(vals)
    total = sum(len(v) for v in vals)
    if codec in BASIC:
        offs = np.zeros(n + 1, "<i8")
        offs[1:] = np.cumsum([len(v) for v in vals])
        return _block(codec, basic_compress(codec, offs.tobytes()), 8 * (n + 1)) + \
            _block(codec, basic_compress(codec, b"".join(vals)), total)
    if codec == ONE_VALUE:
        first = next((v for i, v in enumerate(vals) if valid is None or valid[i]), b"")
        return _block(codec, struct.pack("<I", len(first)) + first, total)
    if codec == DICT:
        sets, index, idx = [], {}, []
        for i, v in enumerate(vals):
            if valid is not None and not valid[i] and idx:
                idx.append(idx[-1])
                continue
            if v not in index:
                index[v] = len(sets)
                sets.append(v)
            idx.append(index[v])
        inner = encode_int_block(np.asarray(idx, np.uint32), 4, nested)
        payload = inner + struct.pack("<I", len(sets)) + b"".join(struct.pack("<Q", len(s)) + s for s in sets)
        return _block(codec, payload, total)
    raise ValueError(f"codec {codec}")


def decode_binary_block(buf: bytes, p: int, n: int) -> Tuple[List[bytes], int]:
    codec, comp, uncomp = struct.unpack_from("<BII", buf, p)
    q = p + 9
    if codec in BASIC:
        offs = np.frombuffer(basic_decompress(codec, buf[q:q + comp], 8 * (n + 1)), "<i8", n + 1)
        q += comp
        c2, comp2, uncomp2 = struct.unpack_from("<BII", buf, q)
        data = basic_decompress(c2, buf[q + 9:q + 9 + comp2], uncomp2)
        return [data[offs[i]:offs[i + 1]] for i in range(n)], q + 9 + comp2
    end = q + comp
    if codec == ONE_VALUE:
        ln = struct.unpack_from("<I", buf, q)[0]
        return [bytes(buf[q + 4:q + 4 + ln])] * n, end
    if codec == DICT:
        idx, q = decode_int_block(buf, q, n, 4, False)
        cnt = struct.unpack_from("<I", buf, q)[0]
        q += 4
        sets = []
        for _ in range(cnt):
            ln = struct.unpack_from("<Q", buf, q)[0]
            sets.append(bytes(buf[q + 8:q + 8 + ln]))
            q += 8 + ln
        return [sets[i] for i in idx], end
    raise NotImplementedError(f"native codec {codec} (Freq) is not restated")


# ---- Boolean blocks (compression/boolean/mod.rs:35-103, rle.rs, one_value.rs) ----
def encode_bool_block(vals, codec: int, valid: Optional[np.ndarray] = None) -> bytes:
    """[codec][compressed u32][uncompressed u32 = rows][payload]: basic codecs hold the values as an
    LSB-first bitmap; Rle runs of [u32 count][u8 value] (nulls extend the current run); OneValue
    one byte (the first valid value)."""
    v = np.asarray(vals, bool)
    n = len(v)
    if codec in BASIC:
        bm = np.packbits(v, bitorder="little").tobytes()
        return _block(codec, basic_compress(codec, bm), n)
    if codec == RLE:
        body = encode_int_block(v.astype(np.uint8), 1, RLE, valid)[9:]
        return _block(RLE, body, n)
    if codec == ONE_VALUE:
        first = next((bool(v[i]) for i in range(n) if valid is None or valid[i]), False)
        return _block(ONE_VALUE, bytes([1 if first else 0]), n)
    raise ValueError(f"codec {codec} is not a Boolean codec")


def decode_bool_block(buf: bytes, p: int, n: int) -> Tuple[np.ndarray, int]:
    codec, comp, uncomp = struct.unpack_from("<BII", buf, p)
    q = p + 9
    end = q + comp
    if codec in BASIC:
        bm = basic_decompress(codec, buf[q:end], (n + 7) // 8)
        return np.unpackbits(np.frombuffer(bm, np.uint8), bitorder="little")[:n].astype(bool), end
    if codec == RLE:
        out, k = [], 0
        while k < n:
            cnt = struct.unpack_from("<I", buf, q)[0]
            out.append(np.full(cnt, buf[q + 4] != 0, bool))
            k += cnt
            q += 5
        return (np.concatenate(out)[:n] if out else np.zeros(0, bool)), end
    if codec == ONE_VALUE:
        return np.full(n, buf[q] > 0, bool), end
    raise ValueError(f"codec {codec} is not a Boolean codec")


# ---- validity ----
def encode_validity(valid: Optional[np.ndarray], n: int) -> bytes:
    """write_validity (serialize.rs:202-217): u32 length + encode_bool of the definition levels
    (all true when the array has no validity)."""
    bits = np.ones(n, bool) if valid is None else np.asarray(valid, bool)
    groups = (n + 7) // 8
    h = (groups << 1) | 1
    hdr = bytearray()
    while True:
        b = h & 0x7F
        h >>= 7
        hdr.append(b | (0x80 if h else 0))
        if not h:
            break
    body = bytes(hdr) + np.packbits(bits, bitorder="little").tobytes()[:groups]
    return struct.pack("<I", len(body)) + body


def decode_validity(buf: bytes, p: int, n: int) -> Tuple[Optional[np.ndarray], int]:
    ln = struct.unpack_from("<I", buf, p)[0]
    q = p + 4
    if ln == 0:
        return None, q
    h = shift = 0
    r = q
    while True:
        c = buf[r]
        r += 1
        h |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            break
    assert h & 1, "read_validity: only bit-packed runs (read_basic.rs:35-42)"
    bits = np.unpackbits(np.frombuffer(buf, np.uint8, (n + 7) // 8, r), bitorder="little")[:n].astype(bool)
    return bits, q + ln


# ---- the writer's codec choice (choose_compressor, no sampling) ----
def choose_int_codec(vals: np.ndarray, width: int, valid: Optional[np.ndarray], basic: int = LZ4,
                     ratio: float = DEFAULT_RATIO, forbidden: Sequence[int] = ()) -> int:
    n = len(vals)
    if not n:
        return basic
    total = n * width
    uniq, counts = np.unique(vals, return_counts=True)
    null_count = 0 if valid is None else int((~np.asarray(valid)).sum())
    vv = vals if valid is None else vals[np.asarray(valid)]
    is_sorted = bool(np.all(vv[1:] >= vv[:-1])) if len(vv) else True
    best, best_r = basic, ratio
    mn = int(vals.min())
    cands = []
    cands.append((ONE_VALUE, float(n) if len(uniq) <= 1 else 0.0))
    mx = int(vals.max())
    if len(uniq) <= 1:
        fr = 0.0
    elif null_count / n >= 0.9:
        fr = float(n - 1)
    else:
        fr = float(n - 1) if counts.max() / n >= 0.9 and mx >= 256 else 0.0
    cands.append((FREQ, fr))
    if len(uniq) * 3 >= n:
        dr = 0.0
    else:
        after = len(uniq) * width + n * (len(uniq).bit_length() // 8) + n * 2 // 128
        dr = total / after
    cands.append((DICT, dr))
    cands.append((RLE, total / max(1, len(encode_int_block(vals, width, RLE, valid)) - 9)))
    bp_ok = mn >= 0 and width == 4 and n % 128 == 0
    bpr = total / max(1, len(encode_int_block(vals, width, BITPACK)) - 9) if bp_ok else 0.0
    cands.append((BITPACK, bpr))
    cands.append((DELTA_BITPACK, bpr * 1.5 if bp_ok and is_sorted and null_count == 0 else 0.0))
    for c, r in cands:
        if c in forbidden:
            continue
        if r > best_r:
            best, best_r = c, r
            if r == float(n):
                break
    return best


# ---- pages and columns ----
def encode_page(vals, kind: str, width: int = 0, valid: Optional[np.ndarray] = None, nullable: bool = False,
                codec: Optional[int] = None, basic: int = LZ4, nested: int = NONE) -> bytes:
    """kind 'int' (vals: numpy array of the column's width) or 'str' (vals: list of bytes)."""
    n = len(vals)
    head = encode_validity(valid, n) if nullable else b""
    if kind == "int":
        v = np.asarray(vals)
        c = codec if codec is not None else choose_int_codec(v, width, valid, basic)
        if c == FREQ:
            c = basic  # Freq (roaring exceptions) is not restated: the plain codec instead
        return head + encode_int_block(v, width, c, valid, basic, nested)
    if kind == "bool":
        return head + encode_bool_block(vals, codec if codec is not None else basic, valid)
    c = codec if codec is not None else basic
    return head + encode_binary_block(list(vals), c, valid, nested)


def decode_page(buf: bytes, p: int, n: int, kind: str, width: int = 0, signed: bool = True, nullable: bool = False):
    valid = None
    if nullable:
        valid, p = decode_validity(buf, p, n)
    if kind == "int":
        v, p = decode_int_block(buf, p, n, width, signed)
    elif kind == "bool":
        v, p = decode_bool_block(buf, p, n)
    else:
        v, p = decode_binary_block(buf, p, n)
    return v, valid, p


def write_column(vals, kind: str, width: int = 0, valid: Optional[np.ndarray] = None, nullable: bool = False,
                 page_rows: int = PAGE_ROWS, codecs: Optional[Sequence[Optional[int]]] = None, basic: int = LZ4,
                 nested: int = NONE) -> Tuple[bytes, List[int], List[int]]:
    """NativeWriter::encode_chunk for one leaf column: the page bytes, PageMeta lengths and
    num_values.  codecs[k] forces page k's codec (None: the writer's choice)."""
    n = len(vals)
    out, lens, rows = bytearray(), [], []
    for k, s in enumerate(range(0, max(n, 1), page_rows)):
        e = min(n, s + page_rows)
        if e <= s and n:
            break
        pv = vals[s:e]
        pvalid = None if valid is None else np.asarray(valid)[s:e]
        c = codecs[k % len(codecs)] if codecs else None
        pg = encode_page(pv, kind, width, pvalid, nullable, c, basic, nested)
        out += pg
        lens.append(len(pg))
        rows.append(e - s)
    return bytes(out), lens, rows


def read_column(buf: bytes, lens: Sequence[int], rows: Sequence[int], kind: str, width: int = 0, signed: bool = True,
                nullable: bool = False):
    """column_iter_to_arrays for one leaf column: values (numpy / list of bytes) and validity."""
    p, vals, valid = 0, [], []
    for ln, n in zip(lens, rows):
        v, va, q = decode_page(buf, p, n, kind, width, signed, nullable)
        vals.append(v if kind in ("int", "bool") else list(v))
        valid.append(np.ones(n, bool) if va is None else va)
        p += ln
    if kind == "bool":
        values = np.concatenate(vals) if vals else np.zeros(0, bool)
    elif kind == "int":
        values = np.concatenate(vals) if vals else np.zeros(0, _dtype(width, signed))
    else:
        values = [x for v in vals for x in v]
    return values, (np.concatenate(valid) if valid else np.zeros(0, bool))
