"""The native (strawboat) format restatement (oracle/native_oracle.py) on its own: every codec the
device reader decodes round-trips through the restated writer and reader, for every integer width,
signed and unsigned, nullable and not, and String columns; the restated codec choice picks what
the reference's rules pick on inputs where the rule is clear.  No reference test or fixture holds
native bytes, so beyond this restatement parity is unpinned."""
import numpy as np
import pytest

from oracle import native_oracle as nat

INT_CODECS = [nat.NONE, nat.LZ4, nat.ZSTD, nat.SNAPPY, nat.RLE, nat.DICT, nat.ONE_VALUE]


def _vals(rng, n, width, signed, kind):
    lo, hi = (-(1 << (8 * width - 1)), (1 << (8 * width - 1)) - 1) if signed else (0, (1 << (8 * width)) - 1)
    dt = nat._dtype(width, signed)
    if kind == "runs":
        v = np.repeat(rng.integers(max(lo, -1000), min(hi, 1000), n // 7 + 1), 7)[:n]
    elif kind == "few":
        v = rng.integers(max(lo, -5), min(hi, 5) + 1, n)
    elif kind == "const":
        v = np.full(n, min(hi, 42))
    else:
        v = rng.integers(lo, hi, n, dtype=np.int64 if signed or width < 8 else np.uint64)
    return np.asarray(v).astype(dt)


@pytest.mark.parametrize("width", [1, 2, 4, 8])
@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("codec", INT_CODECS)
@pytest.mark.parametrize("nullable", [False, True])
def test_int_codecs_round_trip(width, signed, codec, nullable):
    rng = np.random.default_rng(width * 100 + codec + 7 * nullable + 3 * signed)
    n = 1000
    v = _vals(rng, n, width, signed, "const" if codec == nat.ONE_VALUE else ("few" if codec == nat.DICT else "runs"))
    valid = rng.random(n) > 0.2 if nullable else None
    if codec == nat.ONE_VALUE and valid is not None:
        valid[0] = True
    buf, lens, rows = nat.write_column(v, "int", width, valid, nullable, page_rows=384, codecs=[codec])
    got, gv = nat.read_column(buf, lens, rows, "int", width, signed, nullable)
    ok = np.ones(n, bool) if valid is None else valid
    assert (gv == ok).all()
    assert (got[ok] == v[ok]).all()
    if not nullable or codec not in (nat.RLE, nat.DICT, nat.ONE_VALUE):
        assert (got == v).all()


@pytest.mark.parametrize("codec", [nat.BITPACK, nat.DELTA_BITPACK])
@pytest.mark.parametrize("nested_dict", [False, True])
def test_bitpacking_round_trip(codec, nested_dict):
    rng = np.random.default_rng(codec)
    n = 128 * 9
    v = np.sort(rng.integers(0, 1 << 20, n)).astype(np.uint32) if codec == nat.DELTA_BITPACK else \
        rng.integers(0, 1 << rng.integers(0, 33), n, dtype=np.uint64).astype(np.uint32)
    if nested_dict:  # Dict indices packed with this codec
        v = rng.integers(0, 50, n).astype(np.int32)
        if codec == nat.DELTA_BITPACK:  # the reference picks it only for sorted values (delta_bp.rs:82-91)
            v = np.sort(v)
        buf, lens, rows = nat.write_column(v, "int", 4, None, False, codecs=[nat.DICT], nested=codec)
        got, _ = nat.read_column(buf, lens, rows, "int", 4, True)
    else:
        buf, lens, rows = nat.write_column(v, "int", 4, None, False, codecs=[codec])
        got, _ = nat.read_column(buf, lens, rows, "int", 4, False)
    assert (got == v).all()


def test_bitpacker4x_layout():
    """value i of a block is lane i % 4, slot i // 4, LSB-first per lane (simdcomp layout)."""
    v = np.arange(128, dtype=np.uint32)
    b = nat.bp4x_pack(v, 7)
    w = np.frombuffer(b, "<u4")
    assert len(b) == 16 * 7
    assert w[0] & 0x7F == 0 and w[1] & 0x7F == 1 and w[2] & 0x7F == 2 and w[3] & 0x7F == 3
    assert (w[0] >> 7) & 0x7F == 4  # lane 0, slot 1 = value 4
    assert (nat.bp4x_unpack(b, 0, 7) == v).all()


@pytest.mark.parametrize("codec", [nat.NONE, nat.LZ4, nat.ZSTD, nat.SNAPPY, nat.ONE_VALUE, nat.DICT])
@pytest.mark.parametrize("nullable", [False, True])
def test_string_codecs_round_trip(codec, nullable):
    rng = np.random.default_rng(codec + 31 * nullable)
    n = 900
    words = [bytes(rng.integers(97, 123, rng.integers(0, 40))) for _ in range(40)]
    v = [words[0]] * n if codec == nat.ONE_VALUE else [words[i] for i in rng.integers(0, 40, n)]
    valid = rng.random(n) > 0.2 if nullable else None
    if valid is not None:
        valid[0] = True
    buf, lens, rows = nat.write_column(v, "str", 0, valid, nullable, page_rows=256, codecs=[codec])
    got, gv = nat.read_column(buf, lens, rows, "str", 0, True, nullable)
    ok = np.ones(n, bool) if valid is None else valid
    assert [g for g, k in zip(got, ok) if k] == [x for x, k in zip(v, ok) if k]


def test_codec_choice():
    rng = np.random.default_rng(1)
    n = 4096
    assert nat.choose_int_codec(np.full(n, 7, np.int64), 8, None) == nat.ONE_VALUE
    assert nat.choose_int_codec(rng.integers(0, 10, n).astype(np.int64), 8, None) == nat.DICT
    assert nat.choose_int_codec(np.repeat(rng.integers(0, 1 << 40, n // 256), 256).astype(np.int64), 8, None) in (nat.RLE, nat.DICT)
    assert nat.choose_int_codec(rng.integers(0, 1 << 62, n).astype(np.int64), 8, None) == nat.LZ4
    assert nat.choose_int_codec(np.sort(rng.integers(0, 1 << 20, n)).astype(np.int32), 4, None) == nat.DELTA_BITPACK


@pytest.mark.parametrize("codec", [nat.NONE, nat.LZ4, nat.ZSTD, nat.SNAPPY, nat.RLE, nat.ONE_VALUE])
@pytest.mark.parametrize("nullable", [False, True])
def test_bool_codecs_round_trip(codec, nullable):
    rng = np.random.default_rng(codec + 5 * nullable)
    n = 1000
    v = np.repeat(rng.random(n // 9 + 1) < 0.5, 9)[:n] if codec == nat.RLE else (
        np.ones(n, bool) if codec == nat.ONE_VALUE else rng.random(n) < 0.3)
    valid = rng.random(n) > 0.2 if nullable else None
    if valid is not None:
        valid[0] = True
    buf, lens, rows = nat.write_column(v, "bool", 0, valid, nullable, page_rows=333, codecs=[codec])
    got, gv = nat.read_column(buf, lens, rows, "bool", 0, True, nullable)
    ok = np.ones(n, bool) if valid is None else valid
    assert (gv == ok).all()
    assert (got[ok] == v[ok]).all()


def test_float_bits_round_trip():
    """Float columns store their bits in the integer layouts: every codec but the bit-packings."""
    rng = np.random.default_rng(3)
    v = rng.standard_normal(700)
    for codec in (nat.NONE, nat.LZ4, nat.RLE, nat.DICT, nat.ONE_VALUE):
        x = np.repeat(v[:100], 7) if codec in (nat.RLE, nat.DICT) else (np.full(700, 2.5) if codec == nat.ONE_VALUE else v)
        buf, lens, rows = nat.write_column(x.view(np.int64), "int", 8, page_rows=256, codecs=[codec])
        got, _ = nat.read_column(buf, lens, rows, "int", 8, True)
        assert (got.view(np.float64) == x).all()


@pytest.mark.parametrize("codec", [nat.NONE, nat.LZ4, nat.RLE, nat.DICT, nat.ONE_VALUE])
def test_decimal128_round_trip(codec):
    rng = np.random.default_rng(codec)
    n = 600
    v = np.zeros(n, nat._I128)
    v["lo"] = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    v["hi"] = rng.integers(0, 3, n, dtype=np.uint64)
    if codec in (nat.RLE, nat.DICT):
        v = np.repeat(v[:20], 30)
    if codec == nat.ONE_VALUE:
        v = np.repeat(v[:1], n)
    buf, lens, rows = nat.write_column(v, "int", 16, page_rows=250, codecs=[codec])
    got, _ = nat.read_column(buf, lens, rows, "int", 16, True)
    assert (got == v).all()
