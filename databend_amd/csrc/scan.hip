// scan.hip — Parquet column chunks decoded into HBM columns (include/dbgpu_scan.h).
//
// The Fuse read path hands one leaf column chunk (page headers + pages) to arrow-rs's parquet
// reader (BlockReader::deserialize_parquet_chunks -> column_chunks_to_record_batch,
// storages/fuse/src/io/read/block/parquet/mod.rs:45-60, deserialize.rs:33-80).  Here the page
// headers (Thrift compact, a few dozen bytes per page) are parsed on the host and every page is
// decoded on the device, one workgroup per page:
//
//   pq_inflate   one wave per compressed page: a SNAPPY / LZ4_RAW block decode (an UNCOMPRESSED
//                page is decoded where it lies in the chunk, page_base).  The
//                element stream is parsed by the whole wave in lockstep (uniform loads, no lane
//                divergence); literals and back-references are copied 64 bytes per step, and
//                back-references read a 64 KiB LDS ring of the page's recent output (both formats
//                reference at most 64 KiB back — an offset beyond the ring is a decode error).
//   pq_walk      one lane per BYTE_ARRAY page: the value starts of PLAIN byte arrays (u32 length
//                prefixes) — a dependent chain inside a page, parallel across pages.
//   pq_decode    one workgroup per data page: definition levels and dictionary indices through
//                the RLE / bit-packed hybrid (thread 0 parses run headers into an LDS run table,
//                all threads expand values by binary search over the runs), a block scan of the
//                definition bits gives every row its value index, then PLAIN / dictionary values
//                are converted to the Databend type and written at their row (arrow layout: NULL
//                rows hold a zero slot, validity bytes packed afterwards).
//   pq_strings   String payload gather after the offsets scan.
// All integer / byte work, HBM- or latency-bound; every device read is bounds-checked against its
// page (a malformed page sets an error bit, it never faults).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "agg.hpp"
#include "zstd_dev.hpp"
#include "../../include/dbgpu_scan.h"

int abi_fail(int code, const std::string& msg);  // abi.hip: sets dbg_last_error
void* prof_scope_begin(const char* name, hipStream_t s);  // abi.hip: dbg_prof_* event scopes
void prof_scope_end(void* p);
void launch_pack_bits(hipStream_t s, const u8* bytes, u64 n, u8* bits);
void launch_exclusive_scan(hipStream_t s, u64* data, u64 n, u64* total);

namespace {

enum { PG_DATA_V1 = 0, PG_DATA_V2 = 1, PG_DICT = 2 };
enum { ENC_PLAIN = 0, ENC_PLAIN_DICT = 2, ENC_RLE = 3, ENC_RLE_DICT = 8 };
enum { SERR_MALFORMED = 1, SERR_COUNT = 2, SERR_NULL_IN_REQUIRED = 4, SERR_DICT_RANGE = 8 };

struct ScanPage {
    u64 src;          // payload offset in the chunk
    u64 dst;          // decompressed page offset in the page buffer
    u64 row0;         // first output row (data pages)
    u64 vk0;          // first slot of this page's values in the index / value-start arrays
    u32 comp, uncomp; // payload sizes (v2: levels included)
    u32 num_values;
    u32 lv;           // v2: repetition + definition level bytes (stored uncompressed in front)
    u32 def_len;      // v2: definition level bytes
    u8 kind;          // PG_*
    u8 compressed;    // the payload after `lv` is compressed with the chunk's codec
    u8 encoding;
    u8 pad;
};

struct ScanArgs {
    const u8* chunk;
    u8* buf;           // decompressed pages
    const ScanPage* pages;
    u32 n_pages;
    int32_t ptype, tlen, max_def, codec;
    int32_t ttype;     // target dbg_type
    u32 twidth;        // target value width (bytes)
    int32_t dict_page; // index of the dictionary page, -1 none
    u64 rows;
    u8* vbytes;        // [rows] definition flags
    u32* idx;          // [rows] dictionary indices / RLE booleans by value index
    u64* vstart;       // [rows + dict values] BYTE_ARRAY value starts (page-relative)
    u32* nwalk;        // [n_pages] values found by pq_walk
    u64* sptr;         // [rows] String payload source addresses (page buffer or chunk)
    u8* out_data;      // target values (BOOLEAN: value bytes, packed afterwards)
    int32_t need_vb;   // the definition bytes are read afterwards (nullable target / NULL check)
    u64* out_offs;     // String: lengths, then the scan
    u64* err;
    u32 xflags;        // experiment builds only (DBG_X_INFLATE): 1 = no output stores, 2 = no ring reads
};

// ---------------------------------------------------------------------------------------------
// Decompression (one wave per page): the compressed stream is staged into an LDS window with
// coalesced loads and its tags parsed from there (wave-uniform); literal and match bytes are
// copied by all 64 lanes.  The last RING output bytes stay in an LDS ring for back-references;
// a farther one (Snappy / LZ4 offsets reach 64 KiB - 1) reads the page's own output in HBM.
// 32 KiB + 8 KiB of LDS per wave: four pages in flight per CU (a serial tag parse is latency-
// bound, so pages in flight is the throughput).
// ---------------------------------------------------------------------------------------------
#define RING 32768

#define IWIN (8192 - 16)  // the compressed stream's window in LDS (+ 16 bytes of over-read pad: 40 KiB per wave)
template <int CODEC>
__global__ void __launch_bounds__(64) pq_inflate_kernel(ScanArgs a) {
    __shared__ u8 ring[RING];
    __shared__ __attribute__((aligned(16))) u8 inw[IWIN + 16];  // + 16: peek's over-read
    const ScanPage pg = a.pages[blockIdx.x];
    const u32 lane = threadIdx.x;
    // an uncompressed page is decoded where it lies in the chunk (page_base): nothing to copy
    if (CODEC == DBG_PQ_UNCOMPRESSED || !pg.compressed) {
        if (pg.comp != pg.uncomp && lane == 0) atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_MALFORMED);
        return;
    }
    const u8* src = a.chunk + pg.src;
    u8* dst = a.buf + pg.dst;
    // v2 levels (uncompressed) first
    for (u32 j = lane; j < pg.lv; j += 64) dst[j] = src[j];
    const u8* s = src + pg.lv;
    u8* o = dst + pg.lv;
    const u32 sn = pg.comp - pg.lv, on = pg.uncomp - pg.lv;
    bool bad = false;
    u32 p = 0, w = 0;  // input / output cursors (uniform)
    // stream bytes [wl, wh) (offsets from s) are staged in inw; s + wl is 16-byte aligned (whole-
    // granule loads: wl may be up to 15 bytes before the payload, the chunk's own bytes); need(k)
    // restages from p when fewer than k bytes (or the end of the stream) remain staged.  32-bit
    // offsets keep the checks on the scalar unit.
    const int sa = (int)((uintptr_t)s & 15);
    int wl = 0, wh = 0;
    auto need = [&](u32 k) {
        if ((int)p >= wl && ((int)(p + k) <= wh || wh == (int)sn)) return;
        wl = (int)(((u32)p + (u32)sa) & ~15u) - sa;
        wh = (int)sn - wl <= IWIN ? (int)sn : wl + IWIN;
        const u8* g0 = s + wl;
        const u32 nb = (u32)(wh - wl), ng = nb >> 4;
        __builtin_amdgcn_wave_barrier();  // every lane is done reading the old window
        for (u32 g = lane; g < ng; g += 64) ((uint4*)inw)[g] = ((const uint4*)g0)[g];
        for (u32 j = 16 * ng + lane; j < nb; j += 64) inw[j] = g0[j];
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    };
    auto rd = [&](u32 q) -> u32 { return inw[(int)q - wl]; };
    // 8 stream bytes from q (staged) in one LDS round trip: three aligned dwords, funnel-shifted;
    // bytes past wh are garbage, every use is bounded by sn first
    auto peek = [&](u32 q) -> u64 {
        const u32 i = (u32)((int)q - wl), b = i & ~3u, sh = 8 * (i & 3);
        const u32 d0 = *(const u32*)(inw + b), d1 = *(const u32*)(inw + b + 4), d2 = *(const u32*)(inw + b + 8);
        const u64 lo = (u64)d0 | ((u64)d1 << 32);
        return sh ? (lo >> sh) | ((u64)d2 << (64 - sh)) : lo;
    };
    // bounds are compared without wrapping (p <= sn and w <= on hold throughout): a 4-byte
    // Snappy literal length near 2^32 must fail here, not wrap past the check
    auto copy_lit = [&](u64 len) {
        if (len > (u64)(sn - p) || len > (u64)(on - w)) { bad = true; return; }
        const u8* q = s + p;
        if ((int)p >= wl && (int)(p + (u32)len) <= wh) {  // staged: from LDS, no HBM round trip
            const u32 i = (u32)((int)p - wl);
            for (u32 j = lane; j < (u32)len; j += 64) {
                const u8 b = inw[i + j];
                if (!(a.xflags & 1)) o[w + j] = b;
                ring[(w + j) & (RING - 1)] = b;
            }
        } else {
            for (u32 j = lane; j < (u32)len; j += 64) {
                const u8 b = q[j];
                o[w + j] = b;
                ring[(w + j) & (RING - 1)] = b;
            }
        }
        __builtin_amdgcn_wave_barrier();
        p += (u32)len;
        w += (u32)len;
    };
    auto copy_back = [&](u32 off, u64 len) {
        if (off == 0 || off > w || len > (u64)(on - w)) { bad = true; return; }
        if (off >= RING) {
            // beyond the ring: read this wave's own output back from HBM, in segments of at most
            // `off` bytes (every source byte was written before its segment starts); the fence
            // makes the wave's earlier stores visible to its loads (L1 invalidated)
            while (len) {
                const u32 seg = (u32)(len < (u64)off ? len : (u64)off);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
                for (u32 j = lane; j < seg; j += 64) {
                    const u8 b = o[w - off + j];
                    o[w + j] = b;
                    ring[(w + j) & (RING - 1)] = b;
                }
                __builtin_amdgcn_wave_barrier();
                w += seg;
                len -= seg;
            }
            return;
        }
        // byte j repeats the last `off` bytes: out[w + j] = out[w - off + j % off], read from the
        // ring in segments of at most RING - off bytes (a longer one would overwrite ring slots it
        // still reads when off > RING / 2), 64 bytes per step, each step's reads before its writes
        auto run = [&](u32 seg) {
            for (u32 c0 = 0; c0 < seg; c0 += 64) {
                const u32 j = c0 + lane;
                u8 b = 0;
                if (j < seg && !(a.xflags & 2)) b = ring[(w - off + (j < off ? j : j % off)) & (RING - 1)];
                __builtin_amdgcn_wave_barrier();
                if (j < seg) {
                    if (!(a.xflags & 1)) o[w + j] = b;
                    ring[(w + j) & (RING - 1)] = b;
                }
                __builtin_amdgcn_wave_barrier();
            }
            w += seg;
        };
        if (len <= (u64)(RING - off)) {  // every Snappy copy (<= 64 bytes), most LZ4 matches
            run((u32)len);
            return;
        }
        while (len) {
            const u32 seg = (u32)(len < (u64)(RING - off) ? len : (u64)(RING - off));
            run(seg);
            len -= seg;
        }
    };
    if (CODEC == DBG_PQ_SNAPPY) {
        u32 n = 0, sh = 0;  // preamble: uncompressed length (varint)
        need(5);
        for (;;) {
            if (p >= sn || sh > 28) { bad = true; break; }
            const u32 c = rd(p++);
            n |= (c & 0x7F) << sh;
            sh += 7;
            if (!(c & 0x80)) break;
        }
        if (n != on) bad = true;
        while (!bad && p < sn) {
            need(5);  // a tag and its length / offset bytes, read together
            const u64 x = peek(p);
            const u32 tag = (u32)x & 0xFF;
            const u32 kind = tag & 3;
            if (kind == 0) {
                u32 len = tag >> 2;
                if (len >= 60) {
                    const u32 nb = len - 59;
                    if (p + 1 + nb > sn) { bad = true; break; }
                    len = (u32)((x >> 8) & (nb == 4 ? 0xFFFFFFFFull : ((1ull << (8 * nb)) - 1)));
                    p += 1 + nb;
                } else {
                    p += 1;
                }
                copy_lit((u64)len + 1);
            } else {
                u32 len, off;
                if (kind == 1) {
                    if (p + 2 > sn) { bad = true; break; }
                    len = ((tag >> 2) & 7) + 4;
                    off = ((tag >> 5) << 8) | ((u32)(x >> 8) & 0xFF);
                    p += 2;
                } else if (kind == 2) {
                    if (p + 3 > sn) { bad = true; break; }
                    len = (tag >> 2) + 1;
                    off = (u32)(x >> 8) & 0xFFFF;
                    p += 3;
                } else {
                    if (p + 5 > sn) { bad = true; break; }
                    len = (tag >> 2) + 1;
                    off = (u32)(x >> 8);
                    p += 5;
                }
                copy_back(off, len);
            }
        }
    } else {  // LZ4 block: [token][literal length+][literals][offset u16][match length+]
        while (!bad && p < sn) {
            need(16);
            const u64 x = peek(p);
            const u32 tok = (u32)x & 0xFF;
            p += 1;
            u64 lit = tok >> 4;
            if (lit == 15)
                for (;;) {
                    if (p >= sn) { bad = true; break; }
                    need(1);
                    const u32 c = rd(p++);
                    lit += c;
                    if (c != 255) break;
                }
            if (bad) break;
            if (lit) copy_lit(lit);
            if (bad || p >= sn) break;  // the last sequence has literals only
            if (p + 2 > sn) { bad = true; break; }
            u32 off;
            if (lit) {
                need(2);
                off = (u32)peek(p) & 0xFFFF;
            } else {  // no literals: the offset follows the token (peeked with it)
                off = (u32)(x >> 8) & 0xFFFF;
            }
            p += 2;
            u64 ml = tok & 15;
            if (ml == 15)
                for (;;) {
                    if (p >= sn) { bad = true; break; }
                    need(1);
                    const u32 c = rd(p++);
                    ml += c;
                    if (c != 255) break;
                }
            if (bad) break;
            copy_back(off, (u64)ml + 4);
        }
    }
    if ((bad || w != on) && lane == 0) atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_MALFORMED);
}

// ZSTD pages (Fuse's default TableCompression, table_compression.rs:24-31): one wave per page,
// zstd_dev.hpp.  lit: ZS_MAX_BLOCK bytes of literal scratch per page.
__global__ void __launch_bounds__(64) pq_zstd_kernel(ScanArgs a, u8* lit) {
    __shared__ ZsTables T;
    __shared__ ZsWork W;
    const ScanPage pg = a.pages[blockIdx.x];
    const u32 lane = threadIdx.x;
    if (!pg.compressed) {
        if (pg.comp != pg.uncomp && lane == 0) atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_MALFORMED);
        return;
    }
    const u8* src = a.chunk + pg.src;
    u8* dst = a.buf + pg.dst;
    for (u32 j = lane; j < pg.lv; j += 64) dst[j] = src[j];  // v2 levels (uncompressed) first
    __builtin_amdgcn_wave_barrier();
    const bool ok = pg.comp >= pg.lv && pg.uncomp >= pg.lv &&
                    zs_decode(src + pg.lv, pg.comp - pg.lv, dst + pg.lv, pg.uncomp - pg.lv, lit + (u64)blockIdx.x * ZS_MAX_BLOCK, T, W);
    if (!ok && lane == 0) atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_MALFORMED);
}

// a NULL decoded into a non-nullable target: one flag, raised on the device (no read-back of the
// validity bytes)
__global__ void __launch_bounds__(256) pq_null_check_kernel(const u8* __restrict__ vb, u64 n, u64* err) {
    bool any = false;
    for (u64 i = blockIdx.x * 256ULL + threadIdx.x; i < n; i += (u64)gridDim.x * 256) any |= vb[i] == 0;
    if (__ballot(any) && (threadIdx.x & 63) == 0) atomicOr((unsigned long long*)err, (unsigned long long)SERR_NULL_IN_REQUIRED);
}

// ---------------------------------------------------------------------------------------------
// Page-relative layout helpers
// ---------------------------------------------------------------------------------------------
// the page's uncompressed bytes: inflated into the page buffer, or in place in the chunk
__device__ __forceinline__ const u8* page_base(const ScanArgs& a, const ScanPage& pg) {
    return pg.compressed ? a.buf + pg.dst : a.chunk + pg.src;
}
// ---------------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ u32 rd_u32(const u8* p) { return (u32)p[0] | ((u32)p[1] << 8) | ((u32)p[2] << 16) | ((u32)p[3] << 24); }

// start of the values section and the definition-level byte range [d0, d1) of a data page
__device__ __forceinline__ bool page_sections(const ScanArgs& a, const ScanPage& pg, const u8* base, u32& d0, u32& d1, u32& vp) {
    d0 = d1 = vp = 0;
    if (pg.kind == PG_DICT) return true;
    if (pg.kind == PG_DATA_V2) {
        d0 = pg.lv - pg.def_len;
        d1 = pg.lv;
        vp = pg.lv;
        return pg.lv <= pg.uncomp;
    }
    if (a.max_def) {
        if (pg.uncomp < 4) return false;
        const u32 ln = rd_u32(base);
        if (ln > pg.uncomp - 4) return false;
        d0 = 4;
        d1 = 4 + ln;
        vp = d1;
    }
    return true;
}

// one lane per BYTE_ARRAY page: starts of the PLAIN values (positions of their u32 length)
__global__ void __launch_bounds__(64) pq_walk_kernel(ScanArgs a) {
    const u32 pi = blockIdx.x * 64 + threadIdx.x;
    if (pi >= a.n_pages) return;
    const ScanPage pg = a.pages[pi];
    if (pg.encoding != ENC_PLAIN && pg.kind != PG_DICT) return;
    const u8* base = page_base(a, pg);
    u32 d0, d1, vp;
    if (!page_sections(a, pg, base, d0, d1, vp)) {
        atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_MALFORMED);
        return;
    }
    u64 p = vp, k = 0;
    const u64 end = pg.uncomp, cap = pg.num_values;
    while (p + 4 <= end && k < cap) {
        const u32 len = rd_u32(base + p);
        if (p + 4 + len > end) break;
        a.vstart[pg.vk0 + k] = p;
        ++k;
        p += 4 + (u64)len;
    }
    if (p != end && k < cap) atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_MALFORMED);
    a.nwalk[pi] = (u32)k;
}

// ---------------------------------------------------------------------------------------------
// RLE / bit-packed hybrid, expanded by a whole workgroup
// ---------------------------------------------------------------------------------------------
#define DEC_NT 256
#ifndef PQ_PIECE
#define PQ_PIECE 8192  // values per y-piece of a required PLAIN page
#endif
#define RMAX 512
struct RunTable {
    u32 start[RMAX + 1];  // first value index of each run (start[nr] = end of the last one)
    u32 info[RMAX];       // bit-packed: byte offset of the packed values; RLE: the value
    u8 packed[RMAX];
    u32 nr, kend, pos, bad;
};

// Expand `n` values of bit width `bw` from [p0, p1) of `base`; put(k, v) for every k < n.
template <typename PUT>
__device__ __forceinline__ bool hybrid_expand(const u8* base, u32 p0, u32 p1, u32 bw, u32 n, RunTable& rt, PUT put) {
    if (threadIdx.x == 0) {
        rt.pos = p0;
        rt.kend = 0;
        rt.bad = bw > 32 ? 1u : 0u;
    }
    __syncthreads();
    const u32 vb = (bw + 7) / 8;
    while (true) {
        const u32 k0 = rt.kend;
        if (k0 >= n || rt.bad) break;
        __syncthreads();
        if (threadIdx.x == 0) {  // parse up to RMAX run headers
            u32 pos = rt.pos, k = k0, nr = 0;
            bool bad = false;
            while (nr < RMAX && k < n) {
                if (pos >= p1) { bad = true; break; }
                u32 h = 0, sh = 0;
                for (;;) {
                    if (pos >= p1 || sh > 28) { bad = true; break; }
                    const u32 c = base[pos++];
                    h |= (c & 0x7F) << sh;
                    sh += 7;
                    if (!(c & 0x80)) break;
                }
                if (bad) break;
                rt.start[nr] = k;
                if (h & 1) {
                    const u32 groups = h >> 1;
                    const u64 bytes = (u64)groups * bw;
                    if ((u64)pos + bytes > p1 && (u64)pos + (((u64)(n - k) * bw + 7) / 8) > p1) { bad = true; break; }
                    rt.info[nr] = pos;
                    rt.packed[nr] = 1;
                    pos += (u32)min<u64>(bytes, (u64)(p1 - pos));
                    k += groups * 8;
                } else {
                    if (pos + vb > p1) { bad = true; break; }
                    u32 v = 0;
                    for (u32 j = 0; j < vb; ++j) v |= (u32)base[pos + j] << (8 * j);
                    pos += vb;
                    rt.info[nr] = v;
                    rt.packed[nr] = 0;
                    k += h >> 1;
                    if ((h >> 1) == 0) { bad = true; break; }
                }
                ++nr;
            }
            rt.start[nr] = k;
            rt.nr = nr;
            rt.kend = min(k, n);
            rt.pos = pos;
            if (bad) rt.bad = 1;
        }
        __syncthreads();
        if (rt.bad) break;
        const u32 nr = rt.nr, ke = rt.kend;
        for (u32 k = k0 + threadIdx.x; k < ke; k += DEC_NT) {
            u32 lo = 0, hi = nr;  // last run with start <= k
            while (hi - lo > 1) {
                const u32 mid = (lo + hi) >> 1;
                if (rt.start[mid] <= k) lo = mid;
                else hi = mid;
            }
            u32 v;
            if (rt.packed[lo]) {
                const u64 bit = (u64)(k - rt.start[lo]) * bw;
                const u32 bp = rt.info[lo] + (u32)(bit >> 3);
                u64 x = 0;
                for (u32 j = 0; j < 5 && bp + j < p1; ++j) x |= (u64)base[bp + j] << (8 * j);
                v = bw ? (u32)((x >> (bit & 7)) & ((bw == 32) ? 0xFFFFFFFFull : ((1ull << bw) - 1))) : 0u;
            } else {
                v = rt.info[lo];
            }
            put(k, v);
        }
    }
    __syncthreads();
    return !rt.bad;
}

// physical value at `p` (PLAIN layout) -> target bytes at `d`
__device__ __forceinline__ void put_value(const ScanArgs& a, const u8* p, u8* d) {
    switch (a.ptype) {
        case DBG_PQ_INT32: {
            const u32 v = rd_u32(p);
            if (a.ttype == DBG_DECIMAL128) {
                const i64 x = (i64)(int32_t)v;
                ((u64*)d)[0] = (u64)x;
                ((u64*)d)[1] = x < 0 ? ~0ULL : 0ULL;
            } else {
                for (u32 j = 0; j < a.twidth; ++j) d[j] = (u8)(v >> (8 * j));
            }
            return;
        }
        case DBG_PQ_INT64: case DBG_PQ_DOUBLE: {
            u64 v = 0;
            for (int j = 0; j < 8; ++j) v |= (u64)p[j] << (8 * j);
            if (a.ttype == DBG_DECIMAL128) {
                ((u64*)d)[0] = v;
                ((u64*)d)[1] = (i64)v < 0 ? ~0ULL : 0ULL;
            } else {
                *(u64*)d = v;
            }
            return;
        }
        case DBG_PQ_FLOAT: *(u32*)d = rd_u32(p); return;
        default: {  // FIXED_LEN_BYTE_ARRAY: big-endian two's complement -> i128 LE
            u64 lo = 0, hi = 0;
            const u32 n = (u32)a.tlen;
            for (u32 j = 0; j < n; ++j) {
                const u64 b = p[n - 1 - j];
                if (j < 8) lo |= b << (8 * j);
                else hi |= b << (8 * (j - 8));
            }
            if (n < 16 && (p[0] & 0x80)) {  // sign-extend
                if (n < 8) {
                    lo |= ~0ULL << (8 * n);
                    hi = ~0ULL;
                } else {
                    hi |= n == 8 ? ~0ULL : (~0ULL << (8 * (n - 8)));
                }
            }
            ((u64*)d)[0] = lo;
            ((u64*)d)[1] = hi;
            return;
        }
    }
}

__device__ __forceinline__ u32 phys_width(const ScanArgs& a) {
    switch (a.ptype) {
        case DBG_PQ_INT32: case DBG_PQ_FLOAT: return 4;
        case DBG_PQ_INT64: case DBG_PQ_DOUBLE: return 8;
        case DBG_PQ_FIXED_LEN_BYTE_ARRAY: return (u32)a.tlen;
        default: return 0;
    }
}

__global__ void __launch_bounds__(DEC_NT) pq_decode_kernel(ScanArgs a) {
    __shared__ RunTable rt;
    __shared__ u32 wtot[DEC_NT / 64];
    __shared__ u32 s_bad;
    const ScanPage& pg = a.pages[blockIdx.x];  // read in place (uniform: scalar loads); a private copy would go to scratch
    if (pg.kind == PG_DICT) return;
    if (threadIdx.x == 0) s_bad = 0;
    __syncthreads();
    const u8* base = page_base(a, pg);
    const u32 n = pg.num_values;
    auto fail = [&](u64 bit) {
        if (threadIdx.x == 0) atomicOr((unsigned long long*)a.err, (unsigned long long)bit);
    };
    u32 d0, d1, vp;
    if (!page_sections(a, pg, base, d0, d1, vp)) return fail(SERR_MALFORMED);
    u8* vb = a.vbytes + pg.row0;
    const bool dict = pg.encoding == ENC_PLAIN_DICT || pg.encoding == ENC_RLE_DICT;
    const bool rle_bool = pg.encoding == ENC_RLE && a.ptype == DBG_PQ_BOOLEAN;
    // a required PLAIN page is elementwise (value index = row index): its rows are split over the
    // grid's y dimension; every other page is decoded by its y = 0 workgroup alone
    const bool split = !a.max_def && !dict && !rle_bool;
    if (!split && blockIdx.y) return;
    // 1. definition levels -> one byte per row
    if (split) {
        const u32 per = (n + gridDim.y - 1) / gridDim.y, lo = blockIdx.y * per, hi = min(n, lo + per);
        if (a.need_vb)
            for (u32 k = lo + threadIdx.x; k < hi; k += DEC_NT) vb[k] = 1;
    } else if (a.max_def) {
        if (!hybrid_expand(base, d0, d1, 1, n, rt, [&](u32 k, u32 v) { vb[k] = (u8)(v != 0); })) return fail(SERR_MALFORMED);
    } else {
        for (u32 k = threadIdx.x; k < n; k += DEC_NT) vb[k] = 1;
        __syncthreads();
    }
    // 2. dictionary indices (or RLE booleans) by value index
    u32* ix = a.idx + pg.vk0;
    if (dict || rle_bool) {
        u32 p0 = vp, bw = 1, p1 = pg.uncomp;
        if (dict) {
            if (vp >= pg.uncomp) {  // a page of NULLs may carry no index bytes
                p0 = p1;
                bw = 0;
            } else {
                bw = base[vp];
                p0 = vp + 1;
            }
        } else {
            if (vp + 4 > pg.uncomp) return fail(SERR_MALFORMED);
            p0 = vp + 4;
            p1 = min<u32>(pg.uncomp, p0 + rd_u32(base + vp));
        }
        // the non-null count bounds the indices; count it first (defs are in vb)
        __shared__ u32 s_nn;
        if (threadIdx.x == 0) s_nn = 0;
        __syncthreads();
        u32 c = 0;
        for (u32 k = threadIdx.x; k < n; k += DEC_NT) c += vb[k];
        if (c) atomicAdd(&s_nn, c);
        __syncthreads();
        const u32 nn = s_nn;
        if (bw == 0) {
            for (u32 k = threadIdx.x; k < nn; k += DEC_NT) ix[k] = 0;
            __syncthreads();
        } else if (!hybrid_expand(base, p0, p1, bw, nn, rt, [&](u32 k, u32 v) { ix[k] = v; })) {
            return fail(SERR_MALFORMED);
        }
    }
    // 3. values, 256 rows per round: block scan of the definition bytes -> value index
    const ScanPage* dp = a.dict_page >= 0 ? &a.pages[a.dict_page] : nullptr;
    const u8* dbase = dp ? page_base(a, *dp) : nullptr;
    const u32 dn = dp ? dp->num_values : 0;
    const u32 pw = phys_width(a);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // one row: its value (value index vi when def) converted and written; true = out of range
    auto emit = [&](u32 k, u32 vi, u32 def) -> bool {
        const u64 row = pg.row0 + k;
        bool bad = false;
        if (a.ptype == DBG_PQ_BYTE_ARRAY) {
            u64 len = 0, so = 0;
            if (def) {
                if (dict) {
                    const u32 i = ix[vi];
                    if (i >= dn || i >= a.nwalk[a.dict_page]) {
                        bad = true;
                    } else {
                        const u64 st = a.vstart[dp->vk0 + i];
                        len = rd_u32(dbase + st);
                        so = (u64)(dbase + st + 4);
                    }
                } else if (vi >= a.nwalk[blockIdx.x]) {
                    bad = true;
                } else {
                    const u64 st = a.vstart[pg.vk0 + vi];
                    len = rd_u32(base + st);
                    so = (u64)(base + st + 4);
                }
            }
            a.out_offs[row] = bad ? 0 : len;
            a.sptr[row] = so;
        } else if (a.ptype == DBG_PQ_BOOLEAN) {
            u8 v = 0;
            if (def) {
                if (rle_bool) {
                    v = (u8)(ix[vi] & 1);
                } else if (vp + (vi >> 3) < pg.uncomp) {
                    v = (base[vp + (vi >> 3)] >> (vi & 7)) & 1;
                } else {
                    bad = true;
                }
            }
            a.out_data[row] = v;
        } else {
            u8* d = a.out_data + row * a.twidth;
            const u8* sp = nullptr;
            if (def) {
                if (dict) {
                    const u32 i = ix[vi];
                    if (i < dn && (u64)(i + 1) * pw <= dp->uncomp) sp = dbase + (u64)i * pw;
                } else if ((u64)vp + (u64)(vi + 1) * pw <= pg.uncomp) {
                    sp = base + vp + (u64)vi * pw;
                }
                if (!sp) bad = true;
            }
            if (sp) put_value(a, sp, d);
            else for (u32 j = 0; j < a.twidth; ++j) d[j] = 0;
        }
        return bad;
    };
    if (split && (pw == 4 || pw == 8) && a.ptype != DBG_PQ_FIXED_LEN_BYTE_ARRAY && a.ttype != DBG_DECIMAL128 && a.twidth <= pw &&
        (u64)vp + (u64)n * pw <= pg.uncomp) {
        // required PLAIN 4- / 8-byte values into an integer / float target: 8 values per lane from
        // unaligned 16 B loads (the page's values start at any byte), narrowed to the target width
        // and stored as whole words when the row is aligned
        const u32 per = (n + gridDim.y - 1) / gridDim.y;
        const u32 lo = min(n, ((blockIdx.y * per) + 7) & ~7u), hi = min(n, (((blockIdx.y + 1) * per) + 7) & ~7u);
        const u8* vbase = base + vp;
        const u32 tw = a.twidth;
        const u64 row0 = pg.row0;  // a register copy: the lambdas below capture `pg` by reference (scratch)
        u8* const out = a.out_data;
        // load 4 values of a lane (all loads of an unrolled round are issued before its stores:
        // the output may alias the chunk as far as the compiler knows)
        auto load4 = [&](u32 k0, u64 (&v)[4]) {
            const u32 cnt = k0 < hi ? min(4u, hi - k0) : 0u;
            const u8* p = vbase + (u64)k0 * pw;
            // byte-aligned values: gfx950 global loads take unaligned addresses (the compiler emits
            // whole-dword loads for these memcpys), consecutive lanes read consecutive 16 B
            // (every index below is a constant: the arrays stay in registers, no scratch)
            v[0] = v[1] = v[2] = v[3] = 0;
            if (cnt == 4 && pw == 4) {
                u32 w[4];
                __builtin_memcpy(w, p, 16);
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = w[j];
            } else if (cnt == 4) {
                __builtin_memcpy(v, p, 32);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if ((u32)j >= cnt) continue;
                    if (pw == 4) {
                        u32 x;
                        __builtin_memcpy(&x, p + 4 * j, 4);
                        v[j] = x;
                    } else {
                        u64 x;
                        __builtin_memcpy(&x, p + 8 * j, 8);
                        v[j] = x;
                    }
                }
            }
        };
        auto store4 = [&](u32 k0, const u64 (&v)[4]) {
            if (k0 >= hi) return;
            const u32 cnt = min(4u, hi - k0);
            u8* dst = out + (row0 + k0) * (u64)tw;
            if (tw == 2 && cnt == 4 && !((uintptr_t)dst & 7)) {
                *(u64*)dst = (v[0] & 0xFFFF) | ((v[1] & 0xFFFF) << 16) | ((v[2] & 0xFFFF) << 32) | ((v[3] & 0xFFFF) << 48);
            } else if (tw == 4 && cnt == 4 && !((uintptr_t)dst & 15)) {
                typedef u32 v4u32 __attribute__((ext_vector_type(4)));
                *(v4u32*)dst = v4u32{(u32)v[0], (u32)v[1], (u32)v[2], (u32)v[3]};
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if ((u32)j >= cnt) continue;
                    u8* dj = dst + (u64)j * tw;
                    switch (tw) {
                        case 1: *dj = (u8)v[j]; break;
                        case 2: *(uint16_t*)dj = (uint16_t)v[j]; break;
                        case 4: *(u32*)dj = (u32)v[j]; break;
                        default: *(u64*)dj = v[j]; break;
                    }
                }
            }
        };
        // 8 consecutive values per lane and round (32 B read, 16 B written for Int16), two rounds'
        // loads issued before their stores
        constexpr u32 U = 2;
        for (u32 k0 = lo + 8 * threadIdx.x; k0 < hi; k0 += U * 8 * DEC_NT) {
            u64 v[U][2][4];
#pragma unroll
            for (u32 u = 0; u < U; ++u) {
                load4(k0 + u * 8 * DEC_NT, v[u][0]);
                load4(k0 + u * 8 * DEC_NT + 4, v[u][1]);
            }
#pragma unroll
            for (u32 u = 0; u < U; ++u) {
                const u32 k = k0 + u * 8 * DEC_NT;
                u8* dst = out + (row0 + k) * (u64)tw;
                if (tw == 2 && k + 8 <= hi && !((uintptr_t)dst & 15)) {
                    typedef u32 v4u32 __attribute__((ext_vector_type(4)));
                    const u64 (&x)[4] = v[u][0];
                    const u64 (&y)[4] = v[u][1];
                    *(v4u32*)dst = v4u32{(u32)((x[0] & 0xFFFF) | (x[1] << 16)), (u32)((x[2] & 0xFFFF) | (x[3] << 16)),
                                         (u32)((y[0] & 0xFFFF) | (y[1] << 16)), (u32)((y[2] & 0xFFFF) | (y[3] << 16))};
                } else {
                    store4(k, v[u][0]);
                    store4(k + 4, v[u][1]);
                }
            }
        }
        return;
    }
    if (split) {
        const u32 per = (n + gridDim.y - 1) / gridDim.y, lo = blockIdx.y * per, hi = min(n, lo + per);
        bool bad = false;
        for (u32 k = lo + threadIdx.x; k < hi; k += DEC_NT) bad |= emit(k, k, 1);
        if (bad) s_bad = 1;
        __syncthreads();
        if (s_bad) fail(SERR_DICT_RANGE);
        if (a.ptype == DBG_PQ_BYTE_ARRAY && blockIdx.y == 0 && threadIdx.x == 0 && n != a.nwalk[blockIdx.x])
            atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_COUNT);
        return;
    }
    u32 vbase = 0;
    for (u32 r0 = 0; r0 < n; r0 += DEC_NT) {
        const u32 k = r0 + threadIdx.x;
        const u32 def = k < n ? vb[k] : 0u;
        const u64 bal = __ballot(def);
        const u32 pre_w = (u32)__popcll(bal & ((1ULL << lane) - 1));
        if (lane == 0) wtot[wave] = (u32)__popcll(bal);
        __syncthreads();
        u32 pre = 0, tot = 0;
        for (int w = 0; w < DEC_NT / 64; ++w) {
            if (w < wave) pre += wtot[w];
            tot += wtot[w];
        }
        if (k < n && emit(k, vbase + pre + pre_w, def)) s_bad = 1;
        vbase += tot;
        __syncthreads();
    }
    if (s_bad) fail(SERR_DICT_RANGE);
    // PLAIN byte arrays: every value the walk found is consumed exactly once
    if (a.ptype == DBG_PQ_BYTE_ARRAY && !dict && threadIdx.x == 0 && vbase != a.nwalk[blockIdx.x])
        atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_COUNT);
    if (a.max_def == 0 && threadIdx.x == 0 && vbase != n) atomicOr((unsigned long long*)a.err, (unsigned long long)SERR_COUNT);
}

// payload gather: one lane per row
__global__ void __launch_bounds__(256) pq_strings_kernel(const u64* __restrict__ sptr, const u64* __restrict__ offs, u64 rows,
                                                         u8* __restrict__ out, u64 cap) {
    const u64 r = blockIdx.x * 256ULL + threadIdx.x;
    if (r >= rows) return;
    const u64 o = offs[r], e = offs[r + 1];
    if (e > cap || e == o) return;
    const u8* s = (const u8*)sptr[r];  // the value's bytes: page buffer or chunk
    for (u64 j = 0; j < e - o; ++j) out[o + j] = s[j];
}

// ---------------------------------------------------------------------------------------------
// Host: Thrift compact PageHeader (parquet-format parquet.thrift, fields used by the reader)
// ---------------------------------------------------------------------------------------------
struct Compact {
    const u8* b;
    u64 n, p;
    bool ok = true;
    u32 byte() {
        if (p >= n) { ok = false; return 0; }
        return b[p++];
    }
    u64 varint() {
        if (p + 10 <= n) {  // fast path: no per-byte bound checks
            u64 v = 0;
            for (int sh = 0; sh < 64; sh += 7) {
                const u32 c = b[p++];
                v |= (u64)(c & 0x7F) << sh;
                if (!(c & 0x80)) return v;
            }
            ok = false;
            return 0;
        }
        u64 v = 0;
        for (int sh = 0; sh < 64 && ok; sh += 7) {
            const u32 c = byte();
            v |= (u64)(c & 0x7F) << sh;
            if (!(c & 0x80)) return v;
        }
        ok = false;
        return 0;
    }
    i64 zigzag() {
        const u64 v = varint();
        return (i64)(v >> 1) ^ -(i64)(v & 1);
    }
    void skip(int t, int depth = 0) {
        if (depth > 16) { ok = false; return; }
        switch (t) {
            case 1: case 2: return;
            case 3: p += 1; return;
            case 4: case 5: case 6: varint(); return;
            case 7: p += 8; return;
            case 8: p += varint(); return;
            case 9: case 10: {
                const u32 h = byte();
                u64 cnt = h >> 4;
                if (cnt == 15) cnt = varint();
                for (u64 i = 0; i < cnt && ok; ++i) skip(h & 15, depth + 1);
                return;
            }
            case 12: {
                i64 last = 0;
                while (ok) {
                    const u32 h = byte();
                    if (h == 0) return;
                    last = (h >> 4) ? last + (h >> 4) : zigzag();
                    skip(h & 15, depth + 1);
                }
                return;
            }
            default: ok = false;
        }
    }
    // walk a struct: f(fid, type) returns true when it consumed the value
    template <typename F>
    void fields(F f) {
        i64 last = 0;
        while (ok) {
            const u32 h = byte();
            if (h == 0 || !ok) return;
            const int t = h & 15;
            last = (h >> 4) ? last + (h >> 4) : zigzag();
            if (!f(last, t)) skip(t);
        }
    }
};

struct HostPage {
    int type;
    i64 uncomp, comp;
    u64 data_off;
    i64 num_values = 0, encoding = 0, def_len = 0, rep_len = 0;
    bool v2_compressed = true;
};

// page type 0 DATA_PAGE, 1 INDEX_PAGE, 2 DICTIONARY_PAGE, 3 DATA_PAGE_V2
int parse_pages(const dbg_parquet_chunk& c, std::vector<HostPage>& out) {
    out.clear();
    out.reserve(std::min<u64>(c.len / 4096 + 16, 1u << 20));
    u64 pos = 0;
    // A writer's pages of one chunk usually carry byte-identical headers (same value count, sizes
    // and statistics; every page but the last of a fixed-width PLAIN column): a header whose bytes
    // equal the previous one's is that header — the parse is a function of those bytes and ends
    // where the previous one ended — so it costs one compare instead of a Thrift walk (a 2^26-row
    // chunk: 3 356 headers, 94 -> ~10 ns each).
    const u8* prev_hdr = nullptr;
    u64 prev_len = 0;
    while (pos < c.len) {
        if (prev_len && pos + prev_len <= c.len && memcmp(c.host + pos, prev_hdr, prev_len) == 0) {
            HostPage pg = out.back();
            pg.data_off = pos + prev_len;
            if (pg.data_off + (u64)pg.comp > c.len)
                return abi_fail(DBG_ERR_INVALID, "dbg_parquet: malformed page header at byte " + std::to_string(pos));
            out.push_back(pg);
            prev_hdr = c.host + pos;
            pos = pg.data_off + (u64)pg.comp;
            continue;
        }
        Compact r{c.host, c.len, pos};
        HostPage pg{-1, -1, -1, 0};
        // the nested header's integer fields (no heap allocation per page: a chunk of 2^26 rows
        // holds ~3 400 pages at the writers' 20 000-row page cap)
        struct KV {
            i64 f[16], v[16];
            int n = 0;
        };
        auto sub = [&](KV& kv) {
            r.fields([&](i64 fid, int t) {
                if ((t == 5 || t == 6) && kv.n < 16) { kv.f[kv.n] = fid; kv.v[kv.n++] = r.zigzag(); return true; }
                if ((t == 1 || t == 2) && kv.n < 16) { kv.f[kv.n] = fid; kv.v[kv.n++] = t == 1 ? 1 : 0; return true; }
                return false;
            });
        };
        auto get = [](const KV& kv, i64 f, i64 d) {
            for (int i = 0; i < kv.n; ++i) if (kv.f[i] == f) return kv.v[i];
            return d;
        };
        r.fields([&](i64 fid, int t) {
            if (fid == 1 && t == 5) { pg.type = (int)r.zigzag(); return true; }
            if (fid == 2 && t == 5) { pg.uncomp = r.zigzag(); return true; }
            if (fid == 3 && t == 5) { pg.comp = r.zigzag(); return true; }
            if ((fid == 5 || fid == 7 || fid == 8) && t == 12) {
                KV kv;
                sub(kv);
                if (fid == 5) { pg.num_values = get(kv, 1, -1); pg.encoding = get(kv, 2, -1); }
                if (fid == 7) { pg.num_values = get(kv, 1, -1); pg.encoding = get(kv, 2, -1); }
                if (fid == 8) {
                    pg.num_values = get(kv, 1, -1);
                    pg.encoding = get(kv, 4, -1);
                    pg.def_len = get(kv, 5, -1);
                    pg.rep_len = get(kv, 6, -1);
                    pg.v2_compressed = get(kv, 7, 1) != 0;
                }
                return true;
            }
            return false;
        });
        if (!r.ok || pg.type < 0 || pg.uncomp < 0 || pg.comp < 0 || r.p + (u64)pg.comp > c.len)
            return abi_fail(DBG_ERR_INVALID, "dbg_parquet: malformed page header at byte " + std::to_string(pos));
        if (pg.uncomp > 0x7FFFFFFF || pg.num_values < 0 || pg.num_values > 0x7FFFFFFF)
            return abi_fail(DBG_ERR_INVALID, "dbg_parquet: page header values out of range");
        pg.data_off = r.p;
        out.push_back(pg);
        prev_hdr = c.host + pos;
        prev_len = r.p - pos;
        pos = r.p + (u64)pg.comp;
    }
    return DBG_OK;
}

}  // namespace

struct dbg_scan_ctx {
    hipStream_t stream = nullptr;
    u8* chunk = nullptr;  // uploaded chunk bytes
    u64 chunk_cap = 0;
    u8* buf = nullptr;
    u64 buf_cap = 0;
    ScanPage* pages = nullptr;
    u64 pages_cap = 0;
    u8* vbytes = nullptr;
    u64 vbytes_cap = 0;
    u32* idx = nullptr;
    u64 idx_cap = 0;
    u64* vstart = nullptr;
    u64 vstart_cap = 0;
    u32* nwalk = nullptr;
    u64 nwalk_cap = 0;
    u64* sptr = nullptr;
    u64 sptr_cap = 0;
    u8* bools = nullptr;
    u64 bools_cap = 0;
    u64* err = nullptr;  // [0] error bits, [1] string total
    u64* herr = nullptr; // pinned
    u8* zlit = nullptr;  // ZSTD literal scratch, ZS_MAX_BLOCK per page
    u64 zlit_cap = 0;
    ScanPage* hpages = nullptr;  // pinned staging of the page table (an async upload, not a pageable copy)
    u64 hpages_cap = 0;
    // native (strawboat) pages: page descriptors and the host-built tables (Bitpacking blocks,
    // String dictionary entries)
    u8* npg = nullptr;
    u64 npg_cap = 0;
    u64* ntab = nullptr;
    u64 ntab_cap = 0;
};

namespace {
template <typename T>
int ensure(T** p, u64* cap, u64 n) {
    if (*cap >= n && *p) return DBG_OK;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const u64 want = n < 64 ? 64 : n + n / 4;
    if (hipMalloc((void**)p, want * sizeof(T)) != hipSuccess) return abi_fail(DBG_ERR_OOM, "dbg_parquet: device allocation");
    *cap = want;
    return DBG_OK;
}

bool target_ok(int ptype, int tlen, const dbg_datatype& t, u32& width) {
    width = type_width(t.type);
    switch (ptype) {
        case DBG_PQ_BOOLEAN: return t.type == DBG_BOOLEAN;
        case DBG_PQ_INT32:
            return (t.type >= DBG_INT8 && t.type <= DBG_INT32) || (t.type >= DBG_UINT8 && t.type <= DBG_UINT32) || t.type == DBG_DATE ||
                   (t.type == DBG_DECIMAL128 && t.precision <= 9);
        case DBG_PQ_INT64:
            return t.type == DBG_INT64 || t.type == DBG_UINT64 || t.type == DBG_TIMESTAMP || (t.type == DBG_DECIMAL128 && t.precision <= 18);
        case DBG_PQ_FLOAT: return t.type == DBG_FLOAT32;
        case DBG_PQ_DOUBLE: return t.type == DBG_FLOAT64;
        case DBG_PQ_BYTE_ARRAY: return t.type == DBG_STRING;
        case DBG_PQ_FIXED_LEN_BYTE_ARRAY: return t.type == DBG_DECIMAL128 && tlen >= 1 && tlen <= 16;
        default: return false;
    }
}
}  // namespace

#define SCAN_HIP(expr)                                                                                     \
    do {                                                                                                   \
        hipError_t e_ = (expr);                                                                            \
        if (e_ != hipSuccess) return abi_fail(DBG_ERR_DEVICE, std::string("dbg_parquet: ") + hipGetErrorString(e_)); \
    } while (0)
#define SCAN_RET(rc)              \
    do {                          \
        int r_ = (rc);            \
        if (r_ != DBG_OK) return r_; \
    } while (0)

extern "C" {

int dbg_scan_create(dbg_scan_ctx** out, void* stream) {
    if (!out) return abi_fail(DBG_ERR_INVALID, "dbg_scan_create: null out");
    auto* c = new dbg_scan_ctx();
    c->stream = (hipStream_t)stream;
    if (hipMalloc((void**)&c->err, 16) != hipSuccess || hipHostMalloc((void**)&c->herr, 16, hipHostMallocDefault) != hipSuccess) {
        dbg_scan_destroy(c);
        return abi_fail(DBG_ERR_OOM, "dbg_scan_create: allocation");
    }
    *out = c;
    return DBG_OK;
}

int dbg_scan_destroy(dbg_scan_ctx* c) {
    if (!c) return DBG_OK;
    void* dev[] = {c->chunk, c->buf, c->pages, c->vbytes, c->idx, c->vstart, c->nwalk, c->sptr, c->bools, c->err, c->npg, c->ntab};
    for (void* p : dev)
        if (p) hipFree(p);
    if (c->herr) hipHostFree(c->herr);
    if (c->hpages) hipHostFree(c->hpages);
    delete c;
    return DBG_OK;
}

int dbg_parquet_chunk_rows(const dbg_parquet_chunk* chunk, uint64_t* rows, uint32_t* n_pages) {
    if (!chunk || !chunk->host || !rows) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_chunk_rows: null argument");
    std::vector<HostPage> pg;
    SCAN_RET(parse_pages(*chunk, pg));
    u64 r = 0;
    for (auto& p : pg)
        if (p.type == 0 || p.type == 3) r += (u64)p.num_values;
    *rows = r;
    if (n_pages) *n_pages = (uint32_t)pg.size();
    return DBG_OK;
}

int dbg_parquet_decode(dbg_scan_ctx* ctx, const dbg_parquet_chunk* chunk, dbg_datatype target, dbg_out_column* out, uint64_t max_rows,
                       uint64_t max_string_bytes, uint64_t* rows_out, uint64_t* string_bytes) {
    if (!ctx || !chunk || !chunk->host || !out || !rows_out) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: null argument");
    *rows_out = 0;
    if (string_bytes) *string_bytes = 0;
    const dbg_parquet_chunk& c = *chunk;
    u32 tw = 0;
    if (c.max_def_level < 0 || c.max_def_level > 1) return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_parquet: nested column (definition level > 1)");
    if (c.codec != DBG_PQ_UNCOMPRESSED && c.codec != DBG_PQ_SNAPPY && c.codec != DBG_PQ_LZ4_RAW && c.codec != DBG_PQ_ZSTD)
        return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_parquet: codec " + std::to_string(c.codec) + " is decoded on the CPU");
    if (!target_ok(c.physical_type, c.type_length, target, tw))
        return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_parquet: physical type " + std::to_string(c.physical_type) + " -> target type " +
                                                 std::to_string(target.type));
    std::vector<HostPage> hp;
    SCAN_RET(parse_pages(c, hp));
    // page table, built straight into the pinned staging buffer (every call that uploads from it
    // ends synchronised, so the previous upload has finished reading it)
    if (ctx->hpages_cap < hp.size() + 2) {
        SCAN_HIP(hipStreamSynchronize(ctx->stream));
        if (ctx->hpages) SCAN_HIP(hipHostFree(ctx->hpages));
        ctx->hpages = nullptr;
        ctx->hpages_cap = 0;
        const u64 cap = hp.size() + hp.size() / 2 + 17;
        SCAN_HIP(hipHostMalloc((void**)&ctx->hpages, cap * sizeof(ScanPage), hipHostMallocDefault));
        ctx->hpages_cap = cap;
    }
    // slot 0 stages the zeroed error words (one upload resets them and ships the table)
    memset(ctx->hpages, 0, sizeof(ScanPage));
    ScanPage* const pages = ctx->hpages + 1;
    u64 n_pages = 0, maxn = 0;
    u64 dst = 0, row = 0, vk = 0;
    int dict = -1;
    bool mismatch = false;
    for (auto& p : hp) {
        if (p.type == 1) continue;  // INDEX_PAGE
        if (p.type != 0 && p.type != 2 && p.type != 3) return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_parquet: page type " + std::to_string(p.type));
        ScanPage s;
        memset(&s, 0, sizeof(s));
        s.src = p.data_off;
        s.dst = dst;
        s.comp = (u32)p.comp;
        s.uncomp = (u32)p.uncomp;
        s.num_values = (u32)p.num_values;
        s.encoding = (u8)p.encoding;
        s.compressed = (c.codec != DBG_PQ_UNCOMPRESSED) ? 1 : 0;
        if (p.type == 2) {
            if (dict >= 0) return abi_fail(DBG_ERR_INVALID, "dbg_parquet: two dictionary pages");
            if (p.encoding != ENC_PLAIN && p.encoding != ENC_PLAIN_DICT) return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_parquet: dictionary encoding");
            s.kind = PG_DICT;
            dict = (int)n_pages;
        } else {
            const bool dict_enc = p.encoding == ENC_PLAIN_DICT || p.encoding == ENC_RLE_DICT;
            if (!(p.encoding == ENC_PLAIN || dict_enc || (p.encoding == ENC_RLE && c.physical_type == DBG_PQ_BOOLEAN)))
                return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_parquet: encoding " + std::to_string(p.encoding));
            if (dict_enc && dict < 0) return abi_fail(DBG_ERR_INVALID, "dbg_parquet: dictionary-encoded page without a dictionary");
            s.kind = p.type == 3 ? PG_DATA_V2 : PG_DATA_V1;
            s.row0 = row;
            row += (u64)p.num_values;
            if (p.type == 3) {
                if (p.rep_len != 0) return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_parquet: repeated column");
                if (p.def_len < 0 || p.def_len > p.uncomp || p.def_len > p.comp) return abi_fail(DBG_ERR_INVALID, "dbg_parquet: v2 level lengths");
                s.lv = (u32)p.def_len;
                s.def_len = (u32)p.def_len;
                s.compressed = s.compressed && p.v2_compressed;
            }
        }
        s.vk0 = vk;
        vk += (u64)p.num_values;
        dst += ((u64)p.uncomp + 15) & ~15ULL;
        mismatch |= s.comp != s.uncomp;
        maxn = std::max<u64>(maxn, s.num_values);
        pages[n_pages++] = s;
    }
    // uncompressed pages are decoded where they lie; only a size mismatch is checked
    if (c.codec == DBG_PQ_UNCOMPRESSED && mismatch) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: uncompressed page sizes differ");
    *rows_out = row;
    if (row > max_rows) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: " + std::to_string(row) + " rows exceed max_rows");
    if (target.type != DBG_STRING && target.type != DBG_BOOLEAN && !out->data && row) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: null data buffer");
    hipStream_t s = ctx->stream;
    const bool upload = c.device == nullptr;
    if (upload) {
        SCAN_RET(ensure(&ctx->chunk, &ctx->chunk_cap, c.len + 16));
        SCAN_HIP(hipMemcpyAsync(ctx->chunk, c.host, c.len, hipMemcpyHostToDevice, s));
    }
    SCAN_RET(ensure(&ctx->buf, &ctx->buf_cap, dst + 16));
    SCAN_RET(ensure(&ctx->pages, &ctx->pages_cap, n_pages + 2));
    SCAN_RET(ensure(&ctx->vbytes, &ctx->vbytes_cap, row + 1));
    SCAN_RET(ensure(&ctx->idx, &ctx->idx_cap, vk + 1));
    SCAN_RET(ensure(&ctx->nwalk, &ctx->nwalk_cap, n_pages + 1));
    const bool is_str = target.type == DBG_STRING, is_bool = target.type == DBG_BOOLEAN;
    if (is_str) {
        SCAN_RET(ensure(&ctx->vstart, &ctx->vstart_cap, vk + 1));
        SCAN_RET(ensure(&ctx->sptr, &ctx->sptr_cap, row + 1));
        if (!out->offsets) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: String output needs offsets");
    }
    if (is_bool) SCAN_RET(ensure(&ctx->bools, &ctx->bools_cap, row + 1));
    if (c.codec == DBG_PQ_ZSTD) SCAN_RET(ensure(&ctx->zlit, &ctx->zlit_cap, n_pages * ZS_MAX_BLOCK + 16));
    if (target.nullable && c.max_def_level && !out->validity && row) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: null validity buffer");
    SCAN_HIP(hipMemcpyAsync(ctx->pages, ctx->hpages, (n_pages + 1) * sizeof(ScanPage), hipMemcpyHostToDevice, s));
    u64* const perr = (u64*)ctx->pages;
    if (c.physical_type == DBG_PQ_BYTE_ARRAY) SCAN_HIP(hipMemsetAsync(ctx->nwalk, 0, n_pages * 4, s));
    ScanArgs a;
    memset(&a, 0, sizeof(a));
    a.chunk = upload ? ctx->chunk : c.device;
    a.buf = ctx->buf;
    a.pages = ctx->pages + 1;
    a.n_pages = (u32)n_pages;
    a.ptype = c.physical_type;
    a.tlen = c.type_length;
    a.max_def = c.max_def_level;
    a.codec = c.codec;
    a.ttype = target.type;
    a.twidth = tw;
    a.dict_page = dict;
    a.rows = row;
    a.vbytes = ctx->vbytes;
    a.idx = ctx->idx;
    a.vstart = ctx->vstart;
    a.nwalk = ctx->nwalk;
    a.sptr = ctx->sptr;
    a.out_data = is_bool ? ctx->bools : (u8*)out->data;
    a.need_vb = (target.nullable || c.max_def_level) ? 1 : 0;
    a.out_offs = out->offsets;
    a.err = perr;
    if (const char* x = X_ENV("DBG_X_INFLATE")) a.xflags = (u32)atoi(x);  // experiment builds only
    if (n_pages) {
        const dim3 g((u32)n_pages);
        void* ps = c.codec != DBG_PQ_UNCOMPRESSED ? prof_scope_begin("pq_inflate", s) : nullptr;
        switch (c.codec) {
            case DBG_PQ_SNAPPY: hipLaunchKernelGGL(pq_inflate_kernel<DBG_PQ_SNAPPY>, g, dim3(64), 0, s, a); break;
            case DBG_PQ_LZ4_RAW: hipLaunchKernelGGL(pq_inflate_kernel<DBG_PQ_LZ4_RAW>, g, dim3(64), 0, s, a); break;
            case DBG_PQ_ZSTD: hipLaunchKernelGGL(pq_zstd_kernel, g, dim3(64), 0, s, a, ctx->zlit); break;
            default: break;
        }
        prof_scope_end(ps);
        SCAN_HIP(hipGetLastError());
        if (c.physical_type == DBG_PQ_BYTE_ARRAY) {
            hipLaunchKernelGGL(pq_walk_kernel, dim3((u32)((n_pages + 63) / 64)), dim3(64), 0, s, a);
            SCAN_HIP(hipGetLastError());
        }
        // required PLAIN pages are split over the grid's y dimension into pieces of >= 8192 values
        // (writers cap pages at 20 000 rows — pyarrow, parquet-rs — or at 1 MiB: up to 16 pieces)
        static const u64 x_piece = X_ENV("DBG_X_PQ_PIECE") ? (u64)atoll(X_ENV("DBG_X_PQ_PIECE")) : 0;  // EXPERIMENT
        const u64 piece = x_piece ? x_piece : PQ_PIECE;
        const u32 ysplit = c.max_def_level ? 1u : (u32)std::min<u64>(16, std::max<u64>(1, (maxn + piece - 1) / piece));
        ps = prof_scope_begin("pq_decode", s);
        hipLaunchKernelGGL(pq_decode_kernel, dim3((u32)n_pages, ysplit), dim3(DEC_NT), 0, s, a);
        prof_scope_end(ps);
        SCAN_HIP(hipGetLastError());
    }
    if (is_str) {
        // lengths -> offsets (exclusive scan, total into offsets[rows]), then the payload
        if (row) launch_exclusive_scan(s, out->offsets, row, out->offsets + row);
        else SCAN_HIP(hipMemsetAsync(out->offsets, 0, 8, s));
        SCAN_HIP(hipMemcpyAsync(perr + 1, out->offsets + row, 8, hipMemcpyDeviceToDevice, s));
        if (row && out->data)
            hipLaunchKernelGGL(pq_strings_kernel, dim3((u32)((row + 255) / 256)), dim3(256), 0, s, ctx->sptr, out->offsets, row,
                               (u8*)out->data, max_string_bytes);
        SCAN_HIP(hipGetLastError());
    }
    if (is_bool && row) launch_pack_bits(s, ctx->bools, row, (u8*)out->data);
    if (target.nullable && row && out->validity) launch_pack_bits(s, ctx->vbytes, row, out->validity);
    if (!target.nullable && c.max_def_level && row) {
        hipLaunchKernelGGL(pq_null_check_kernel, dim3((u32)std::min<u64>(1024, (row + 255) / 256)), dim3(256), 0, s, ctx->vbytes, row,
                           perr);
        SCAN_HIP(hipGetLastError());
    }
    SCAN_HIP(hipMemcpyAsync(ctx->herr, perr, 16, hipMemcpyDeviceToHost, s));
    SCAN_HIP(hipStreamSynchronize(s));
    const u64 e = ctx->herr[0];
    if (e & SERR_MALFORMED) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: malformed page data");
    if (e & (SERR_COUNT | SERR_DICT_RANGE)) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: value count / dictionary index out of range");
    if (is_str) {
        if (string_bytes) *string_bytes = ctx->herr[1];
        if (ctx->herr[1] > max_string_bytes)
            return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: String payload needs " + std::to_string(ctx->herr[1]) + " bytes");
    }
    if (e & SERR_NULL_IN_REQUIRED) return abi_fail(DBG_ERR_INVALID, "dbg_parquet_decode: NULL in a non-nullable column");
    return DBG_OK;
}

}  // extern "C"

// =============================================================================================
// Fuse native (strawboat) pages -> HBM columns (dbg_native_decode; include/dbgpu_scan.h).
//
// The reader this replaces: NativeReader / column_iter_to_arrays (src/common/arrow/src/native/
// read/*, compression/*), called by BlockReader::deserialize_native_chunks
// (FUSE/io/read/block/block_reader_native_deserialize.rs).  The host walks each page's structure
// — validity header, codec headers, a Dict's nested index block and entry list, Bitpacking block
// headers — bounds-checking everything against the page; basic-codec sections (Lz4 / Zstd /
// Snappy) are inflated by the Parquet path's kernels; one workgroup per page then decodes the
// values (or a Dict's indices) and the validity, and a second pass resolves dictionaries.
// Addresses in the page descriptors are tagged: bits 62-63 select the chunk, the inflate staging
// buffer or the host-built table, the rest is the byte offset in it.
// =============================================================================================
namespace {

enum { NC_NONE = 0, NC_LZ4 = 1, NC_ZSTD = 2, NC_SNAPPY = 3, NC_RLE = 10, NC_DICT = 11, NC_ONE = 12, NC_FREQ = 13, NC_BP = 14,
       NC_DBP = 15, NC_PATAS = 16 };
constexpr u64 NT_CHUNK = 0, NT_STAGE = 1ULL << 62, NT_TAB = 2ULL << 62, NT_MASK = (1ULL << 62) - 1;
enum { NC_BITMAP = 100 };  // a Boolean page's basic-codec payload: the values as an LSB-first bitmap

struct NatBlock {  // one integer block: the values, or a Dict's u32 indices
    u64 src;       // tagged: raw little-endian values (None, or inflated), OneValue's value, Rle runs, Bitpacking data
    u64 tab;       // tagged: Bitpacking / DeltaBitpacking block table, u64 per block: data offset from src | bits << 56
    u32 nrec;      // Rle runs / Bitpacking blocks
    u32 codec;     // NC_NONE (raw), NC_RLE, NC_ONE, NC_BP, NC_DBP
};
struct NatPage {
    u64 row0;
    u32 n;
    u32 kind;      // 0 integer (Float32 / Float64: their bits), 1 String, 2 Boolean (one byte per row)
    u32 tw;        // integer width (Dict indices: 4)
    u32 dict;      // values through a dictionary: `blk` holds the indices
    NatBlock blk;
    u64 valid;     // tagged bitmap (LSB first), or ~0 (no validity: all valid)
    u64 dsrc;      // Dict: integer values (tw each) / String entries in the table (tagged address, length)
    u32 dn;        // Dict entries
    u32 smode;     // String: 0 basic (offsets + bytes), 1 one value, 2 dict
    u64 soffs;     // String basic: (n + 1) zero-based u64 offsets
    u64 sdata;     // String basic: the bytes; one value: its bytes
    u64 stotal;    // String basic: the bytes' length; one value: its length
};
// SERR_* bits the inflate kernels also set: SERR_MALFORMED, SERR_COUNT (a section's size)
enum { NERR_MALFORMED = SERR_MALFORMED, NERR_NULL = SERR_NULL_IN_REQUIRED, NERR_RANGE = SERR_DICT_RANGE };

struct NatBases {
    const u8* b[3];
    __device__ __forceinline__ const u8* at(u64 x) const { return b[x >> 62] + (x & NT_MASK); }
};

__device__ __forceinline__ u64 nat_ld(const u8* p, u32 w) {  // little-endian; gfx950 global loads take byte addresses
    if (w == 8) {
        u64 x;
        __builtin_memcpy(&x, p, 8);
        return x;
    }
    if (w == 4) {
        u32 x;
        __builtin_memcpy(&x, p, 4);
        return x;
    }
    if (w == 2) {
        uint16_t x;
        __builtin_memcpy(&x, p, 2);
        return x;
    }
    return *p;
}
__device__ __forceinline__ u32 nat_ld32(const u8* p) { return (u32)nat_ld(p, 4); }
__device__ __forceinline__ void nat_st(u8* d, u64 v, u32 tw) {  // d is tw-aligned (row * tw in a torch buffer)
    if (tw == 8) *(u64*)d = v;
    else if (tw == 4) *(u32*)d = (u32)v;
    else if (tw == 2) *(uint16_t*)d = (uint16_t)v;
    else *d = (u8)v;
}

#define NAT_NT 256
#define NAT_LDS_DICT 2048  // dictionary entries staged in LDS (16 KB); larger ones are read through the caches
// block-wide inclusive scan of u64 (NAT_NT threads); `tot` receives the block total
__device__ __forceinline__ u64 nat_scan(u64 v, u64* wsum, u64& tot) {
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int d = 1; d < 64; d <<= 1) {
        const u64 y = __shfl_up(v, d);
        if ((int)lane >= d) v += y;
    }
    __syncthreads();
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    u64 pre = 0;
    tot = 0;
    for (u32 w = 0; w < NAT_NT / 64; ++w) {
        if (w < wave) pre += wsum[w];
        tot += wsum[w];
    }
    return v + pre;
}

// Decode rows [lo, hi) of integer block b (n values of width tw) with every thread of the
// workgroup, 8 consecutive rows per lane: put8(i0, cnt, v) receives rows i0 .. i0 + cnt - 1
// (cnt = 8 and i0 a multiple of 8 except at a slice's or an Rle round's edges).  lo is a multiple
// of 8.  Rle walks all runs (few) and expands only the slice; DeltaBitpacking needs the page's
// prefix sum, so its page is one slice (lo = 0, hi = n) and puts one row at a time.
// Decimal128 (16-byte values) runs twice, once per 8-byte half: vs = 16 (the value stride), vo =
// 0 / 8 (the half), tw = 8.
template <typename PUT8>
__device__ __forceinline__ void nat_block(const NatBlock& b, u32 n, u32 lo, u32 hi, u32 tw, const NatBases& B, u64* err, PUT8 put8,
                                          u32 vs = 0, u32 vo = 0) {
    __shared__ u64 wsum[NAT_NT / 64];
    __shared__ u64 rstart[NAT_NT];
    __shared__ u64 rval[NAT_NT];
    if (!vs) vs = tw;
    const u8* src = B.at(b.src);
    if (b.codec == NC_NONE) {
        for (u32 i0 = lo + 8 * threadIdx.x; i0 < hi; i0 += 8 * NAT_NT) {
            const u32 cnt = min(8u, hi - i0);
            const u8* p = src + (u64)i0 * vs + vo;
            u64 v[8];
            if (vs != tw) {
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = (u32)k < cnt ? nat_ld(p + (u64)k * vs, tw) : 0;
            } else if (cnt == 8 && tw == 1) {
                u64 x;
                __builtin_memcpy(&x, p, 8);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = (x >> (8 * k)) & 0xFF;
            } else if (cnt == 8 && tw == 2) {
                uint16_t x[8];
                __builtin_memcpy(x, p, 16);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = x[k];
            } else if (cnt == 8 && tw == 4) {
                u32 x[8];
                __builtin_memcpy(x, p, 32);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = x[k];
            } else if (cnt == 8) {
                __builtin_memcpy(v, p, 64);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = (u32)k < cnt ? nat_ld(p + (u64)k * tw, tw) : 0;
            }
            put8(i0, cnt, v);
        }
    } else if (b.codec == NC_ONE) {
        const u64 x = nat_ld(src + vo, tw);
        u64 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = x;
        for (u32 i0 = lo + 8 * threadIdx.x; i0 < hi; i0 += 8 * NAT_NT) put8(i0, min(8u, hi - i0), v);
    } else if (b.codec == NC_BITMAP) {  // 8 rows per lane from one bitmap byte (lo is a multiple of 8)
        for (u32 i0 = lo + 8 * threadIdx.x; i0 < hi; i0 += 8 * NAT_NT) {
            const u32 byte = src[i0 >> 3];
            u64 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = (byte >> k) & 1;
            put8(i0, min(8u, hi - i0), v);
        }
    } else if (b.codec == NC_RLE) {  // runs [u32 count][value]: fixed-size records, NAT_NT runs per round
        const u32 rs = 4 + vs;
        u64 row = 0;
        for (u32 r0 = 0; r0 < b.nrec && row < hi; r0 += NAT_NT) {
            const u32 r = r0 + threadIdx.x;
            const u64 cnt = r < b.nrec ? nat_ld32(src + (u64)r * rs) : 0;
            u64 tot;
            const u64 incl = nat_scan(cnt, wsum, tot);
            rstart[threadIdx.x] = row + incl - cnt;
            rval[threadIdx.x] = r < b.nrec ? nat_ld(src + (u64)r * rs + 4 + vo, tw) : 0;
            __syncthreads();
            const u64 a = row > lo ? row : lo, e = row + tot < hi ? row + tot : hi;
            for (u64 g = (a & ~7ULL) + 8 * threadIdx.x; g < e; g += 8 * NAT_NT) {
                const u64 j0 = g > a ? g : a, j1 = g + 8 < e ? g + 8 : e;
                u32 l = 0, h = NAT_NT - 1;  // the last run starting at or before j0
                while (l < h) {
                    const u32 mid = (l + h + 1) >> 1;
                    if (rstart[mid] <= j0) l = mid;
                    else h = mid - 1;
                }
                u64 v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    while (l + 1 < NAT_NT && rstart[l + 1] <= j0 + k) ++l;
                    v[k] = rval[l];
                }
                put8((u32)j0, (u32)(j1 - j0), v);
            }
            row += tot;
            __syncthreads();
        }
        if (row < hi && threadIdx.x == 0) atomicOr((unsigned long long*)err, (unsigned long long)NERR_MALFORMED);
    } else {  // Bitpacking / DeltaBitpacking: BitPacker4x blocks of 128 (simdcomp 4-lane layout)
        const u64* tab = (const u64*)B.at(b.tab);
        auto unpack = [&](u32 i) -> u64 {
            const u32 blk = i >> 7;
            if (blk >= b.nrec) return 0;
            const u64 e = tab[blk];
            const u32 bits = (u32)(e >> 56);
            if (!bits) return 0;
            const u8* d = src + (e & ((1ULL << 56) - 1));
            const u32 j = i & 127, lane = j & 3, bp = (j >> 2) * bits, w = bp >> 5, sh = bp & 31;
            u64 v = nat_ld32(d + 4 * (4 * w + lane)) >> sh;
            if (sh + bits > 32) v |= (u64)nat_ld32(d + 4 * (4 * (w + 1) + lane)) << (32 - sh);
            return v & (bits >= 32 ? 0xFFFFFFFFULL : ((1ULL << bits) - 1));
        };
        if (b.codec == NC_BP) {
            for (u32 i0 = lo + 8 * threadIdx.x; i0 < hi; i0 += 8 * NAT_NT) {
                u64 v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = unpack(i0 + k);
                put8(i0, min(8u, hi - i0), v);
            }
        } else {  // deltas in value order, the page's first from 0: a page-wide wrapping prefix sum
            u64 carry = 0;
            for (u32 i0 = 0; i0 < n; i0 += NAT_NT) {
                const u32 i = i0 + threadIdx.x;
                const u64 dv = i < n ? unpack(i) : 0;
                u64 tot;
                const u64 incl = nat_scan(dv, wsum, tot);
                u64 v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = (carry + incl) & 0xFFFFFFFFULL;
                if (i < n) put8(i, 1, v);
                carry += tot;
                __syncthreads();
            }
        }
    }
}

// rows i0 .. i0 + cnt - 1 of v[] into a tw-wide column at o (8-byte stores when whole and aligned)
__device__ __forceinline__ void nat_store8(u8* o, u32 i0, u32 cnt, const u64 (&v)[8], u32 tw) {
    u8* d = o + (u64)i0 * tw;
    if (cnt == 8 && !((uintptr_t)d & 7)) {
        if (tw == 1) {
            u64 x = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) x |= (v[k] & 0xFF) << (8 * k);
            *(u64*)d = x;
        } else if (tw == 2) {
            u64 x0 = 0, x1 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x0 |= (v[k] & 0xFFFF) << (16 * k);
                x1 |= (v[k + 4] & 0xFFFF) << (16 * k);
            }
            ((u64*)d)[0] = x0;
            ((u64*)d)[1] = x1;
        } else if (tw == 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) ((u64*)d)[k] = (v[2 * k] & 0xFFFFFFFFULL) | (v[2 * k + 1] << 32);
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) ((u64*)d)[k] = v[k];
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if ((u32)k < cnt) nat_st(d + (u64)k * tw, v[k], tw);
}

// One workgroup per (page, slice): validity bytes, then the values — integers stored in the
// target width, a dictionary's indices resolved on the spot (the dictionary staged in LDS when
// it fits), Strings as (source address, length) for the offsets scan and the gather
__global__ void __launch_bounds__(NAT_NT) nat_decode_kernel(const NatPage* __restrict__ pages, NatBases B, u8* __restrict__ out,
                                                            u8* __restrict__ vbytes, u64* __restrict__ sptr, u64* __restrict__ lens,
                                                            u64* err) {
    __shared__ u64 sdict[NAT_LDS_DICT];
    const NatPage pg = pages[blockIdx.x];
    const bool whole = pg.blk.codec == NC_DBP;
    if (whole && blockIdx.y) return;
    const u32 per = whole ? pg.n : (((pg.n + gridDim.y - 1) / gridDim.y) + 127) & ~127u;
    const u32 lo = min(pg.n, blockIdx.y * per), hi = min(pg.n, lo + per);
    if (lo >= hi) return;
    if (vbytes) {  // 8 rows per lane: one bitmap byte -> 8 flag bytes
        const u8* vb = pg.valid == ~0ULL ? nullptr : B.at(pg.valid);
        for (u32 i0 = lo + 8 * threadIdx.x; i0 < hi; i0 += 8 * NAT_NT) {
            const u32 cnt = min(8u, hi - i0);
            const u32 bits = vb ? vb[i0 >> 3] : 0xFF;
            u8* d = vbytes + pg.row0 + i0;
            if (cnt == 8 && !((uintptr_t)d & 7)) {
                u64 x = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) x |= (u64)((bits >> k) & 1) << (8 * k);
                *(u64*)d = x;
            } else {
                for (u32 k = 0; k < cnt; ++k) d[k] = (bits >> k) & 1;
            }
        }
    }
    const u32 tw = pg.tw;
    if (pg.dict) {
        const u8* d = B.at(pg.dsrc);
        const u32 dn = pg.dn;
        u32 bad = 0;
        if (pg.kind == 0) {
            // Decimal128: the dictionary and the output in two 8-byte halves
            const u32 halves = tw == 16 ? 2 : 1, hw = tw == 16 ? 8 : tw;
            for (u32 hv = 0; hv < halves; ++hv) {
                const bool lds = dn <= NAT_LDS_DICT;
                if (lds) {
                    if (hv) __syncthreads();  // every lane is done with the previous half's entries
                    for (u32 k = threadIdx.x; k < dn; k += NAT_NT) sdict[k] = nat_ld(d + (u64)k * tw + 8 * hv, hw);
                    __syncthreads();
                }
                u8* o = out + pg.row0 * tw + 8 * hv;
                nat_block(pg.blk, pg.n, lo, hi, 4, B, err, [&](u32 i0, u32 cnt, const u64 (&ix)[8]) {
                    u64 v[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const u64 x = ix[k];
                        const bool in = x < dn;
                        bad |= (u32)k < cnt && !in;
                        v[k] = !in ? 0 : (lds ? sdict[x] : nat_ld(d + x * tw + 8 * hv, hw));
                    }
                    if (halves == 1) {
                        nat_store8(o, i0, cnt, v, tw);
                    } else {
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if ((u32)k < cnt) *(u64*)(o + (u64)(i0 + k) * 16) = v[k];
                    }
                });
            }
        } else {
            const u64* e = (const u64*)d;
            nat_block(pg.blk, pg.n, lo, hi, 4, B, err, [&](u32 i0, u32 cnt, const u64 (&ix)[8]) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if ((u32)k >= cnt) continue;
                    const u64 x = ix[k];
                    u64 a = (u64)B.at(0), l = 0;
                    if (x < dn) {
                        a = (u64)B.at(e[2 * x]);
                        l = e[2 * x + 1];
                    } else {
                        bad = 1;
                    }
                    sptr[pg.row0 + i0 + k] = a;
                    lens[pg.row0 + i0 + k] = l;
                }
            });
        }
        if (bad) atomicOr((unsigned long long*)err, (unsigned long long)NERR_RANGE);
        return;
    }
    if (pg.kind == 0 && tw == 16) {  // Decimal128: each 8-byte half in turn, at a 16-byte stride
        for (u32 hv = 0; hv < 2; ++hv) {
            u8* o = out + pg.row0 * 16 + 8 * hv;
            nat_block(pg.blk, pg.n, lo, hi, 8, B, err, [&](u32 i0, u32 cnt, const u64 (&v)[8]) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if ((u32)k < cnt) *(u64*)(o + (u64)(i0 + k) * 16) = v[k];
            }, 16, 8 * hv);
            __syncthreads();  // the Rle run tables in LDS are reused by the second half
        }
        return;
    }
    if (pg.kind == 0) {
        u8* o = out + pg.row0 * tw;
        nat_block(pg.blk, pg.n, lo, hi, tw, B, err, [&](u32 i0, u32 cnt, const u64 (&v)[8]) { nat_store8(o, i0, cnt, v, tw); });
        return;
    }
    if (pg.kind == 2) {  // Boolean: a byte per row (nonzero = true), bit-packed afterwards
        u8* o = out + pg.row0;
        nat_block(pg.blk, pg.n, lo, hi, 1, B, err, [&](u32 i0, u32 cnt, const u64 (&v)[8]) {
            u64 t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = v[k] != 0;
            nat_store8(o, i0, cnt, t, 1);
        });
        return;
    }
    if (pg.smode == 1) {
        const u64 a = (u64)B.at(pg.sdata);
        for (u32 i = lo + threadIdx.x; i < hi; i += NAT_NT) {
            sptr[pg.row0 + i] = a;
            lens[pg.row0 + i] = pg.stotal;
        }
        return;
    }
    const u8* offs = B.at(pg.soffs);
    const u64 a = (u64)B.at(pg.sdata);
    u32 bad = 0;
    for (u32 i = lo + threadIdx.x; i < hi; i += NAT_NT) {
        const u64 s0 = nat_ld(offs + 8ULL * i, 8), s1 = nat_ld(offs + 8ULL * (i + 1), 8);
        const bool ok = s0 <= s1 && s1 <= pg.stotal;
        bad |= !ok;
        sptr[pg.row0 + i] = ok ? a + s0 : a;
        lens[pg.row0 + i] = ok ? s1 - s0 : 0;
    }
    if (bad) atomicOr((unsigned long long*)err, (unsigned long long)NERR_MALFORMED);
}

__global__ void __launch_bounds__(256) nat_null_check_kernel(const u8* __restrict__ vb, u64 n, u64* err) {
    for (u64 i = blockIdx.x * 256ULL + threadIdx.x; i < n; i += (u64)gridDim.x * 256)
        if (!vb[i]) {
            atomicOr((unsigned long long*)err, (unsigned long long)NERR_NULL);
            return;
        }
}

// ---- host: page structure ----
struct NatParse {
    const u8* h;  // column bytes (host)
    std::vector<ScanPage> jobs[4];  // inflate jobs per basic codec (1 Lz4, 2 Zstd, 3 Snappy)
    u64 stage = 0;                  // staging bytes
    std::vector<u64> tab;           // host-built table (u64 words)
    std::string err;
    int vkind = 0;                  // the column's values: 0 integer, 1 Float32 / Float64, 2 Boolean
    u32 rd32(u64 p) const { u32 v; memcpy(&v, h + p, 4); return v; }
    u64 rd64(u64 p) const { u64 v; memcpy(&v, h + p, 8); return v; }
    bool fail(const std::string& m) {
        if (err.empty()) err = m;
        return false;
    }
    // a basic-codec section [payload, payload + comp) of `uncomp` bytes -> tagged address of its bytes
    bool basic(u32 codec, u64 payload, u32 comp, u32 uncomp, u64& addr) {
        if (codec == NC_NONE) {
            if (comp != uncomp) return fail("None section: compressed and uncompressed sizes differ");
            addr = NT_CHUNK | payload;
            return true;
        }
        ScanPage j;
        memset(&j, 0, sizeof(j));
        j.src = payload;
        j.dst = stage;
        j.comp = comp;
        j.uncomp = uncomp;
        j.compressed = 1;
        jobs[codec].push_back(j);
        addr = NT_STAGE | stage;
        stage += ((u64)uncomp + 15) & ~15ULL;
        return true;
    }
    // one integer block at p (inside [p, end)) of n values of width tw -> b; q = its end
    bool int_block(u64 p, u64 end, u32 n, u32 tw, bool allow_dict, NatBlock& b, NatPage* pg, u64& q) {
        if (p + 9 > end) return fail("integer block header past the page");
        const u32 codec = h[p], comp = rd32(p + 1), uncomp = rd32(p + 5);
        const u64 pl = p + 9;
        if (pl + comp > end) return fail("integer block past the page");
        q = pl + comp;
        memset(&b, 0, sizeof(b));
        const int vk = allow_dict ? vkind : 0;  // a Dict's nested index block holds integers
        // Float32 / Float64 (DoubleCompressor, compression/double/mod.rs): the integer layouts minus
        // the bit-packings; Boolean (compression/boolean/mod.rs): basic codecs hold the bitmap, its
        // uncompressed field the row count, plus Rle and OneValue of one byte
        if (vk == 1 && (codec == NC_BP || codec == NC_DBP)) return fail("Bitpacking in a Float column");
        if (vk == 2 && (codec == NC_BP || codec == NC_DBP || codec == NC_DICT)) return fail("codec " + std::to_string(codec) + " in a Boolean column");
        if (vk == 2 && codec <= NC_SNAPPY) {
            if (uncomp != n) return fail("Boolean block: uncompressed field != rows");
            b.codec = NC_BITMAP;
            return basic(codec, pl, comp, (u32)(((u64)n + 7) / 8), b.src);
        }
        switch (codec) {
            case NC_NONE: case NC_LZ4: case NC_ZSTD: case NC_SNAPPY:
                if ((u64)uncomp != (u64)n * tw) return fail("integer block: uncompressed size != rows x width");
                b.codec = NC_NONE;
                return basic(codec, pl, comp, uncomp, b.src);
            case NC_ONE:
                if (comp < tw && n) return fail("OneValue block too short");
                b.codec = NC_ONE;
                b.src = NT_CHUNK | pl;
                return true;
            case NC_RLE: {
                const u32 rs = 4 + tw;
                if (comp % rs) return fail("Rle block: not whole runs");
                b.codec = NC_RLE;
                b.src = NT_CHUNK | pl;
                b.nrec = comp / rs;
                u64 tot = 0;
                for (u32 r = 0; r < b.nrec; ++r) tot += rd32(pl + (u64)r * rs);
                if (tot < n) return fail("Rle runs cover fewer rows than the page");
                return true;
            }
            case NC_BP: case NC_DBP: {
                if (tw != 4) return fail("Bitpacking of a non-4-byte type");  // (Decimal128 included)
                b.codec = codec;
                b.src = NT_CHUNK | pl;
                b.nrec = (n + 127) / 128;
                b.tab = NT_TAB | (8 * (u64)tab.size());
                u64 x = pl;
                for (u32 k = 0; k < b.nrec; ++k) {
                    if (x + 1 > q) return fail("Bitpacking block header past the block");
                    const u32 bits = h[x];
                    if (bits > 32 || x + 1 + 16ULL * bits > q) return fail("Bitpacking block past the block");
                    tab.push_back(((x + 1) - pl) | ((u64)bits << 56));
                    x += 1 + 16ULL * bits;
                }
                return true;
            }
            case NC_DICT: {
                if (!allow_dict || !pg) return fail("Dict inside Dict");
                u64 r;
                NatBlock ib;
                if (!int_block(pl, q, n, 4, false, ib, nullptr, r)) return false;
                if (r + 4 > q) return fail("Dict entry count past the block");
                const u32 cnt = rd32(r);
                if (r + 4 + (u64)cnt * tw > q) return fail("Dict values past the block");
                pg->dict = 1;
                pg->dsrc = NT_CHUNK | (r + 4);
                pg->dn = cnt;
                b = ib;
                return true;
            }
            case NC_FREQ: err = "unsupported: Freq (roaring exceptions) is decoded on the CPU"; return false;
            default: err = "unsupported: native codec " + std::to_string(codec) + " is decoded on the CPU"; return false;
        }
    }
    bool str_block(u64 p, u64 end, u32 n, NatPage& pg, u64& q) {
        if (p + 9 > end) return fail("String block header past the page");
        const u32 codec = h[p], comp = rd32(p + 1), uncomp = rd32(p + 5);
        const u64 pl = p + 9;
        if (pl + comp > end) return fail("String block past the page");
        q = pl + comp;
        switch (codec) {
            case NC_NONE: case NC_LZ4: case NC_ZSTD: case NC_SNAPPY: {  // offsets block, then bytes block
                if ((u64)uncomp != 8ULL * (n + 1)) return fail("String offsets block: size != (rows + 1) x 8");
                pg.smode = 0;
                if (!basic(codec, pl, comp, uncomp, pg.soffs)) return false;
                const u64 p2 = q;
                if (p2 + 9 > end) return fail("String bytes header past the page");
                const u32 c2 = h[p2], comp2 = rd32(p2 + 1), uncomp2 = rd32(p2 + 5);
                if (c2 > NC_SNAPPY) return fail("String bytes block: not a basic codec");
                if (p2 + 9 + comp2 > end) return fail("String bytes block past the page");
                q = p2 + 9 + comp2;
                pg.stotal = uncomp2;
                return basic(c2, p2 + 9, comp2, uncomp2, pg.sdata);
            }
            case NC_ONE: {
                if (comp < 4) return fail("OneValue block too short");
                const u32 len = rd32(pl);
                if (4ULL + len > comp) return fail("OneValue value past the block");
                pg.smode = 1;
                pg.sdata = NT_CHUNK | (pl + 4);
                pg.stotal = len;
                return true;
            }
            case NC_DICT: {
                u64 r;
                NatBlock ib;
                if (!int_block(pl, q, n, 4, false, ib, nullptr, r)) return false;
                if (r + 4 > q) return fail("Dict entry count past the block");
                const u32 cnt = rd32(r);
                r += 4;
                pg.smode = 2;
                pg.dict = 1;
                pg.blk = ib;
                pg.dsrc = NT_TAB | (8 * (u64)tab.size());
                pg.dn = cnt;
                for (u32 k = 0; k < cnt; ++k) {
                    if (r + 8 > q) return fail("Dict entry past the block");
                    const u64 len = rd64(r);
                    if (len > q - r - 8) return fail("Dict entry bytes past the block");
                    tab.push_back(NT_CHUNK | (r + 8));
                    tab.push_back(len);
                    r += 8 + len;
                }
                return true;
            }
            case NC_FREQ: err = "unsupported: Freq (roaring exceptions) is decoded on the CPU"; return false;
            default: err = "unsupported: native String codec " + std::to_string(codec) + " is decoded on the CPU"; return false;
        }
    }
};

bool nat_int_target(int t, u32& w) {
    switch (t) {
        case DBG_BOOLEAN: w = 1; return true;
        case DBG_FLOAT32: w = 4; return true;
        case DBG_FLOAT64: w = 8; return true;
        case DBG_DECIMAL128: w = 16; return true;  // i128 pages (write/primitive.rs: compress_integer)
        case DBG_INT8: case DBG_UINT8: w = 1; return true;
        case DBG_INT16: case DBG_UINT16: w = 2; return true;
        case DBG_INT32: case DBG_UINT32: case DBG_DATE: w = 4; return true;
        case DBG_INT64: case DBG_UINT64: case DBG_TIMESTAMP: w = 8; return true;
        default: return false;
    }
}

}  // namespace

extern "C" {

int dbg_native_decode(dbg_scan_ctx* ctx, const dbg_native_column* col, dbg_datatype target, dbg_out_column* out, uint64_t max_rows,
                      uint64_t max_string_bytes, uint64_t* rows_out, uint64_t* string_bytes) {
    if (!ctx || !col || !col->host || !out || !rows_out || (col->n_pages && (!col->page_lengths || !col->page_rows)))
        return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: null argument");
    *rows_out = 0;
    if (string_bytes) *string_bytes = 0;
    const bool is_str = target.type == DBG_STRING;
    u32 tw = 0;
    if (!is_str && !nat_int_target(target.type, tw))
        return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_native: target type " + std::to_string(target.type) + " is decoded on the CPU");
    const bool is_bool = target.type == DBG_BOOLEAN;
    NatParse P;
    P.h = col->host;
    P.vkind = is_bool ? 2 : ((target.type == DBG_FLOAT32 || target.type == DBG_FLOAT64) ? 1 : 0);
    std::vector<NatPage> pages(col->n_pages);
    u64 pos = 0, row = 0;
    for (u32 k = 0; k < col->n_pages; ++k) {
        NatPage& pg = pages[k];
        memset(&pg, 0, sizeof(pg));
        const u64 len = col->page_lengths[k], n = col->page_rows[k];
        if (pos + len > col->len || n > 0xFFFFFFFFULL) return abi_fail(DBG_ERR_INVALID, "dbg_native: page " + std::to_string(k) + " past the column");
        const u64 end = pos + len;
        pg.row0 = row;
        pg.n = (u32)n;
        pg.kind = is_str ? 1 : (is_bool ? 2 : 0);
        pg.tw = tw;
        pg.valid = ~0ULL;
        u64 p = pos;
        if (col->nullable) {  // write_validity: u32 length + one bit-packed hybrid run
            if (p + 4 > end) return abi_fail(DBG_ERR_INVALID, "dbg_native: validity header past the page");
            const u32 vl = P.rd32(p);
            p += 4;
            if (vl) {
                if (p + vl > end) return abi_fail(DBG_ERR_INVALID, "dbg_native: validity past the page");
                u64 hdr = 0, q = p;
                for (u32 sh = 0;; sh += 7) {
                    if (q >= p + vl || sh > 35) return abi_fail(DBG_ERR_INVALID, "dbg_native: validity header");
                    const u32 c = col->host[q++];
                    hdr |= (u64)(c & 0x7F) << sh;
                    if (!(c & 0x80)) break;
                }
                if (!(hdr & 1)) return abi_fail(DBG_ERR_UNSUPPORTED, "dbg_native: RLE validity run (read_validity reads bit-packed runs only)");
                if ((hdr >> 1) * 8 < n || q + (n + 7) / 8 > p + vl) return abi_fail(DBG_ERR_INVALID, "dbg_native: validity shorter than the page");
                pg.valid = NT_CHUNK | q;
                p += vl;
            }
        }
        u64 q = 0;
        const bool ok = is_str ? P.str_block(p, end, (u32)n, pg, q) : P.int_block(p, end, (u32)n, tw, true, pg.blk, &pg, q);
        if (!ok) {
            const bool unsup = P.err.rfind("unsupported", 0) == 0;
            return abi_fail(unsup ? DBG_ERR_UNSUPPORTED : DBG_ERR_INVALID, "dbg_native: page " + std::to_string(k) + ": " + P.err);
        }
        row += n;
        pos = end;
    }
    *rows_out = row;
    if (row > max_rows) return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: " + std::to_string(row) + " rows exceed max_rows");
    if (!is_str && !out->data && row) return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: null data buffer");
    if (is_str && !out->offsets) return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: String output needs offsets");
    if (target.nullable && col->nullable && !out->validity && row) return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: null validity buffer");
    hipStream_t s = ctx->stream;
    const bool upload = col->device == nullptr;
    if (upload) {
        SCAN_RET(ensure(&ctx->chunk, &ctx->chunk_cap, col->len + 16));
        SCAN_HIP(hipMemcpyAsync(ctx->chunk, col->host, col->len, hipMemcpyHostToDevice, s));
    }
    SCAN_RET(ensure(&ctx->buf, &ctx->buf_cap, P.stage + 16));
    SCAN_RET(ensure(&ctx->ntab, &ctx->ntab_cap, P.tab.size() + 1));
    SCAN_RET(ensure(&ctx->npg, &ctx->npg_cap, pages.size() * sizeof(NatPage) + 16));
    SCAN_RET(ensure(&ctx->vbytes, &ctx->vbytes_cap, row + 1));
    u64 njobs = 0;
    for (int c = 1; c <= 3; ++c) njobs += P.jobs[c].size();
    SCAN_RET(ensure(&ctx->pages, &ctx->pages_cap, njobs + 1));
    if (is_str) SCAN_RET(ensure(&ctx->sptr, &ctx->sptr_cap, row + 1));
    if (is_bool) SCAN_RET(ensure(&ctx->bools, &ctx->bools_cap, row + 8));
    if (!P.jobs[NC_ZSTD].empty()) SCAN_RET(ensure(&ctx->zlit, &ctx->zlit_cap, (u64)P.jobs[NC_ZSTD].size() * ZS_MAX_BLOCK + 16));
    // the small tables are copied synchronously from pageable memory (staged by the runtime)
    if (!pages.empty()) SCAN_HIP(hipMemcpyAsync(ctx->npg, pages.data(), pages.size() * sizeof(NatPage), hipMemcpyHostToDevice, s));
    if (!P.tab.empty()) SCAN_HIP(hipMemcpyAsync(ctx->ntab, P.tab.data(), P.tab.size() * 8, hipMemcpyHostToDevice, s));
    SCAN_HIP(hipMemsetAsync(ctx->err, 0, 16, s));
    const u8* chunk = upload ? ctx->chunk : col->device;
    // basic-codec sections: the Parquet path's inflate kernels over a job list per codec
    {
        u64 off = 0;
        std::vector<ScanPage> all;
        for (int c = 1; c <= 3; ++c) all.insert(all.end(), P.jobs[c].begin(), P.jobs[c].end());
        if (!all.empty()) SCAN_HIP(hipMemcpyAsync(ctx->pages, all.data(), all.size() * sizeof(ScanPage), hipMemcpyHostToDevice, s));
        for (int c = 1; c <= 3; ++c) {
            const u64 nj = P.jobs[c].size();
            if (!nj) continue;
            ScanArgs a;
            memset(&a, 0, sizeof(a));
            a.chunk = chunk;
            a.buf = ctx->buf;
            a.pages = ctx->pages + off;
            a.n_pages = (u32)nj;
            a.err = ctx->err;
            void* ps = prof_scope_begin("nat_inflate", s);
            if (c == NC_LZ4) hipLaunchKernelGGL(pq_inflate_kernel<DBG_PQ_LZ4_RAW>, dim3((u32)nj), dim3(64), 0, s, a);
            else if (c == NC_SNAPPY) hipLaunchKernelGGL(pq_inflate_kernel<DBG_PQ_SNAPPY>, dim3((u32)nj), dim3(64), 0, s, a);
            else hipLaunchKernelGGL(pq_zstd_kernel, dim3((u32)nj), dim3(64), 0, s, a, ctx->zlit);
            prof_scope_end(ps);
            SCAN_HIP(hipGetLastError());
            off += nj;
        }
    }
    NatBases B;
    B.b[0] = chunk;
    B.b[1] = ctx->buf;
    B.b[2] = (const u8*)ctx->ntab;
    const bool want_vb = col->nullable != 0;
    if (!pages.empty()) {
        // slices per page: ≫ 256 workgroups over the chip, ≥ 1024 rows per slice
        u64 maxn = 0;
        for (const NatPage& pg : pages) maxn = std::max<u64>(maxn, pg.n);
        u32 split = (u32)std::max<u64>(1, std::min<u64>({16, (4096 + pages.size() - 1) / pages.size(), (maxn + 1023) / 1024}));
        void* ps = prof_scope_begin("nat_decode", s);
        hipLaunchKernelGGL(nat_decode_kernel, dim3((u32)pages.size(), split), dim3(NAT_NT), 0, s, (const NatPage*)ctx->npg, B,
                           is_bool ? ctx->bools : (u8*)out->data, want_vb ? ctx->vbytes : nullptr, ctx->sptr, out->offsets, ctx->err);
        prof_scope_end(ps);
        SCAN_HIP(hipGetLastError());
    }
    if (is_str) {  // lengths -> offsets, then the payload (the Parquet path's gather)
        if (row) launch_exclusive_scan(s, out->offsets, row, out->offsets + row);
        else SCAN_HIP(hipMemsetAsync(out->offsets, 0, 8, s));
        SCAN_HIP(hipMemcpyAsync(ctx->err + 1, out->offsets + row, 8, hipMemcpyDeviceToDevice, s));
        if (row && out->data)
            hipLaunchKernelGGL(pq_strings_kernel, dim3((u32)((row + 255) / 256)), dim3(256), 0, s, ctx->sptr, out->offsets, row,
                               (u8*)out->data, max_string_bytes);
        SCAN_HIP(hipGetLastError());
    }
    if (is_bool && row) launch_pack_bits(s, ctx->bools, row, (u8*)out->data);
    if (target.nullable && row && out->validity) {
        if (want_vb) launch_pack_bits(s, ctx->vbytes, row, out->validity);
        else SCAN_HIP(hipMemsetAsync(out->validity, 0xFF, (row + 7) / 8, s));
    }
    if (!target.nullable && want_vb && row) {
        hipLaunchKernelGGL(nat_null_check_kernel, dim3((u32)std::min<u64>(1024, (row + 255) / 256)), dim3(256), 0, s, ctx->vbytes, row,
                           ctx->err);
        SCAN_HIP(hipGetLastError());
    }
    SCAN_HIP(hipMemcpyAsync(ctx->herr, ctx->err, 16, hipMemcpyDeviceToHost, s));
    SCAN_HIP(hipStreamSynchronize(s));
    const u64 e = ctx->herr[0];
    if (e & (NERR_MALFORMED | SERR_COUNT)) return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: malformed page data");
    if (e & NERR_RANGE) return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: dictionary index out of range");
    if (is_str) {
        if (string_bytes) *string_bytes = ctx->herr[1];
        if (ctx->herr[1] > max_string_bytes)
            return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: String payload needs " + std::to_string(ctx->herr[1]) + " bytes");
    }
    if (e & NERR_NULL) return abi_fail(DBG_ERR_INVALID, "dbg_native_decode: NULL in a non-nullable column");
    return DBG_OK;
}

}  // extern "C"
