"""One codec's Parquet chunk (bench.measure_scan's column: C2's AdvEngineID, 2^26 rows, Fuse's
parquet shape) decoded `--steps` times, for rocprofv3 counter passes over the scan kernels:

    rocprofv3 --pmc SQ_WAVES ... -d gpurun_out/pmc_scan -o sq --output-format csv -- python3 scripts/scan_run.py --codec SNAPPY
"""
import argparse
import ctypes as C
import io
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--codec", default="SNAPPY", choices=["NONE", "SNAPPY", "LZ4", "ZSTD"])
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--rows", type=int, default=1 << 26)
    p.add_argument("--no-check", action="store_true", help="experiment builds whose knobs break the output")
    p.add_argument("--time", action="store_true", help="print ms per decode (events around --steps decodes)")
    a = p.parse_args()
    import numpy as np
    import pyarrow as pa
    import pyarrow.parquet as pq
    import torch
    from databend_amd import abi
    from databend_amd import column as col
    from databend_amd.ffi import check, lib
    from databend_amd.scan import ParquetChunkDecoder
    rng = np.random.default_rng(0xC2)
    rows = a.rows
    adv = np.where(rng.random(rows) < 0.9937, 0, rng.integers(1, 33, rows)).astype(np.int16)
    t = pa.table({"a": pa.array(adv)}, schema=pa.schema([pa.field("a", pa.int16(), nullable=False)]))
    bio = io.BytesIO()
    pq.write_table(t, bio, compression=a.codec, use_dictionary=False, row_group_size=1 << 30, data_page_size=1 << 20)
    buf = bio.getvalue()
    md = pq.ParquetFile(io.BytesIO(buf)).metadata.row_group(0).column(0)
    chunk = buf[md.data_page_offset:md.data_page_offset + md.total_compressed_size]
    dchunk = torch.from_numpy(np.frombuffer(chunk, dtype=np.uint8).copy()).cuda()
    hbuf = C.create_string_buffer(chunk, len(chunk))
    c = abi.dbg_parquet_chunk()
    c.host = C.cast(hbuf, C.c_void_p)
    c.device = dchunk.data_ptr()
    c.len = len(chunk)
    c.physical_type = abi.PQ_INT32
    c.max_def_level = 0
    c.codec = {"NONE": abi.PQ_UNCOMPRESSED, "SNAPPY": abi.PQ_SNAPPY, "LZ4": abi.PQ_LZ4_RAW, "ZSTD": abi.PQ_ZSTD}[a.codec]
    out_t = torch.empty(rows * 2, dtype=torch.uint8, device="cuda")
    o = abi.dbg_out_column()
    o.data = out_t.data_ptr()
    nr, sb = C.c_uint64(), C.c_uint64()
    dec = ParquetChunkDecoder()
    call = lambda: check(lib().dbg_parquet_decode(dec.h, C.byref(c), col.Int16.to_abi(), C.byref(o), rows, 0, C.byref(nr), C.byref(sb)))
    if a.time:
        call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
    for _ in range(a.steps):
        call()
    if a.time:
        e1.record()
    torch.cuda.synchronize()
    if a.time:
        print(f"scan_run: {a.codec} {e0.elapsed_time(e1) / a.steps:.4f} ms per decode", flush=True)
    if not a.no_check:
        assert nr.value == rows and torch.equal(out_t.view(torch.int16), torch.from_numpy(adv).cuda())
    print(f"scan_run: {a.codec}, {len(chunk)} chunk bytes, {a.steps} decodes", flush=True)
    dec.close()


if __name__ == "__main__":
    main()
