// zstd_dev.hpp — Zstandard frame decoder (RFC 8878) for Parquet ZSTD pages on gfx950.
//
// Fuse writes its blocks with TableCompression::Zstd by default
// (src/query/storages/common/table_meta/src/table/table_compression.rs:24-31), which the parquet
// writer maps to the ZSTD page codec; the reference decodes it through the `zstd` crate (libzstd).
// This is an independent restatement of the published format, written for one wave per page.
// Lane 0 parses the frame and entropy-decodes (Huffman tree, FSE tables, the sequence bitstream —
// inherently serial); the four Huffman literal streams decode on lanes 0-3 at once; sequences are
// decoded by lane 0 in batches of ZS_SEQ into LDS and executed by the whole wave: literal runs
// and matches are copied 64 bytes per step, a match's source bytes read from an LDS ring of the
// last ZS_RING output bytes (the global output only for longer offsets, after a fence) — an
// overlapping match is the periodic extension of the `off` bytes before it, so no byte of a match
// is read after the match writes it.  Every read is bounds-checked against the compressed page
// and every write against the page's uncompressed size: a malformed page sets `bad`, never
// faults.
//
// Tables, the ring and the sequence batch live in LDS (one set per page); the literals of the
// current block go to a per-page scratch of ZS_MAX_BLOCK bytes in global memory.
//
// The same source builds on the host (ZS_HOST: one "lane", plain loads) for the decoder's CPU
// test against libzstd-made frames (tests/test_zstd_host.py); the device build is the product.
#pragma once
#ifdef ZS_HOST
#include <cstdint>
typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
#define ZS_FN static inline
#define ZS_MFN inline
#define ZS_CONST static const
#define ZS_LD(p) (*(const u8*)(p))
#define ZS_LANES 1u
#define ZS_LANE_ID 0u
#define ZS_WAVE_SYNC()
#define ZS_CLZ(v) __builtin_clz(v)
#define ZS_LDS_SYNC()
#include <cstring>
static inline uint64_t zs_ld64(const u8* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
#else
#include "device.hpp"
#define ZS_FN __device__ __forceinline__
#define ZS_MFN __device__ __forceinline__
#define ZS_CONST __device__ __constant__ const
#define ZS_LD(p) gld<u8>(p)
#define ZS_LANES 64u
#define ZS_LANE_ID (threadIdx.x & 63)
#define ZS_WAVE_SYNC()                                   \
    do {                                                 \
        __builtin_amdgcn_wave_barrier();                 \
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); \
        __builtin_amdgcn_wave_barrier();                 \
    } while (0)
#define ZS_CLZ(v) __clz(v)
// LDS written by some lanes, then read by others of the same wave
#define ZS_LDS_SYNC()                                      \
    do {                                                   \
        __builtin_amdgcn_wave_barrier();                   \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
        __builtin_amdgcn_wave_barrier();                   \
    } while (0)
typedef u64 zs_u64u __attribute__((aligned(1)));
__device__ __forceinline__ u64 zs_ld64(const u8* p) {  // gfx950 global loads take byte addresses
    return *(const zs_u64u __attribute__((address_space(1)))*)p;
}
#endif

#define ZS_MAX_BLOCK (128 * 1024)
#define ZS_HUF_MAXBITS 11
#define ZS_LL_MAXLOG 9
#define ZS_ML_MAXLOG 9
#define ZS_OF_MAXLOG 8
#define ZS_RING 16384  // LDS history of the output (power of two)
#define ZS_SEQ 256     // sequences decoded per batch

struct ZsFse {  // one FSE decoding table entry
    u8 sym, nbits;
    u16 next;  // new-state baseline
};
struct ZsTables {
    ZsFse ll[1 << ZS_LL_MAXLOG], ml[1 << ZS_ML_MAXLOG], of[1 << ZS_OF_MAXLOG], hw[1 << 6];
    u16 huf[1 << ZS_HUF_MAXBITS];  // (symbol << 8) | nbits
    u32 ll_log, ml_log, of_log, huf_bits;
    u32 have_ll, have_ml, have_of, have_huf;  // a previous block's table may be repeated
    short norm[64];
    u8 weights[256];
};

// ---- predefined distributions and code tables (RFC 8878 §3.1.1.3.2.2) ----
ZS_CONST short zs_ll_def[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                                    2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
ZS_CONST short zs_ml_def[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
ZS_CONST short zs_of_def[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
ZS_CONST u32 zs_ll_base[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,    16,    18,
                                                   20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
ZS_CONST u8 zs_ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                                  1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
ZS_CONST u32 zs_ml_base[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,  16,   17,   18,   19,   20,
                                                   21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,  34,   35,   37,   39,   41,
                                                   43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
ZS_CONST u8 zs_ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                                  0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

ZS_FN u32 zs_highbit(u32 v) { return 31 - ZS_CLZ(v); }

struct ZsWork {  // per-page LDS beside the tables
    u8 ring[ZS_RING];
    u32 ll[ZS_SEQ], ml[ZS_SEQ], off[ZS_SEQ];
    u64 sh[16];  // lane 0 -> wave broadcast slots
};

// Forward little-endian bit reader over [p, p + n) (FSE table descriptions)
struct ZsFwd {
    const u8* p;
    u64 n;      // bytes
    u64 bit;    // next bit
    ZS_MFN u32 peek(u32 k) const {  // k <= 32; bytes past the end read as 0
        u64 v = 0;
        const u64 b0 = bit >> 3;
        for (u32 i = 0; i < 5; ++i)
            if (b0 + i < n) v |= (u64)ZS_LD(p + b0 + i) << (8 * i);
        return (u32)((v >> (bit & 7)) & ((1ULL << k) - 1));
    }
    ZS_MFN void skip(u32 k) { bit += k; }
};

// Backward bit reader (RFC 8878 §4.1): the stream is read from its end; the last byte's highest
// set bit is padding.  pos = bits left; reading past the start yields zeros (pos goes negative).
struct ZsBwd {
    const u8* p;
    u64 n;
    long long pos;
    ZS_MFN bool init(const u8* s, u64 len) {
        p = s;
        n = len;
        if (!len) return false;
        const u32 last = ZS_LD(s + len - 1);
        if (!last) return false;
        pos = (long long)(8 * (len - 1) + zs_highbit(last));
        return true;
    }
    ZS_MFN u64 window(long long at) const {  // 64 bits starting at bit `at` (may be < 0)
        u64 v = 0;
        const long long b0 = at >> 3;  // floor
        if (b0 >= 0 && (u64)b0 + 9 <= n) {  // inside the stream: one 8-byte load and one byte
            const u32 s = (u32)(at & 7);
            v = zs_ld64(p + b0) >> s;
            if (s) v |= (u64)ZS_LD(p + b0 + 8) << (64 - s);
            return v;
        }
        for (int i = 0; i < 9; ++i) {
            const long long b = b0 + i;
            if (b >= 0 && (u64)b < n) {
                const u64 byte = ZS_LD(p + b);
                const long long sh = (long long)8 * i - (at - 8 * b0);
                if (sh >= 0 && sh < 64) v |= byte << sh;
                else if (sh < 0 && sh > -8) v |= byte >> (-sh);
            }
        }
        return v;
    }
    ZS_MFN u64 read(u32 k) {  // k <= 56
        if (!k) return 0;
        pos -= k;
        return window(pos) & ((1ULL << k) - 1);
    }
    ZS_MFN u32 peek(u32 k) const { return (u32)(window(pos - k) & ((1ULL << k) - 1)); }
};

// FSE_readNCount: normalized counts of symbols 0..*max_sym; returns bytes consumed (0 = bad)
ZS_FN u64 zs_read_ncount(const u8* p, u64 n, short* norm, u32* max_sym, u32* log, u32 max_log) {
    ZsFwd r{p, n, 0};
    const u32 al = r.peek(4) + 5;
    r.skip(4);
    if (al > max_log) return 0;
    int remaining = (1 << al) + 1, threshold = 1 << al;
    u32 nbits = al + 1, sym = 0;
    bool prev0 = false;
    while (remaining > 1 && sym <= *max_sym) {
        if (sym >= 64) return 0;  // beyond every alphabet decoded here
        if (prev0) {
            u32 n0 = sym;
            while (r.peek(2) == 3) {
                n0 += 3;
                r.skip(2);
                if (r.bit > 8 * n) return 0;
            }
            n0 += r.peek(2);
            r.skip(2);
            if (n0 > *max_sym + 1 || n0 > 64) return 0;
            while (sym < n0) norm[sym++] = 0;
            if (sym > *max_sym) break;
        }
        const int mx = (2 * threshold - 1) - remaining;
        int count;
        const u32 v = r.peek(nbits);
        if ((int)(v & (threshold - 1)) < mx) {
            count = (int)(v & (threshold - 1));
            r.skip(nbits - 1);
        } else {
            count = (int)(v & (2 * threshold - 1));
            if (count >= threshold) count -= mx;
            r.skip(nbits);
        }
        count--;
        remaining -= count < 0 ? -count : count;
        if (sym >= 64) return 0;
        norm[sym++] = (short)count;
        prev0 = count == 0;
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
        if (r.bit > 8 * n) return 0;
    }
    if (remaining != 1) return 0;
    *max_sym = sym - 1;
    *log = al;
    return (r.bit + 7) >> 3;
}

// FSE_buildDTable
ZS_FN bool zs_build_fse(ZsFse* t, const short* norm, u32 max_sym, u32 log) {
    const u32 size = 1u << log;
    u32 high = size - 1;
    u16 next[64];
    for (u32 s = 0; s <= max_sym; ++s) {
        if (norm[s] == -1) {
            t[high--].sym = (u8)s;
            next[s] = 1;
        } else {
            next[s] = (u16)norm[s];
        }
    }
    const u32 step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    u32 pos = 0;
    for (u32 s = 0; s <= max_sym; ++s)
        for (int i = 0; i < norm[s]; ++i) {
            t[pos].sym = (u8)s;
            do pos = (pos + step) & mask;
            while (pos > high);
        }
    if (pos != 0) return false;
    for (u32 u = 0; u < size; ++u) {
        const u32 s = t[u].sym;
        const u32 ns = next[s]++;
        const u32 nb = log - zs_highbit(ns);
        t[u].nbits = (u8)nb;
        t[u].next = (u16)((ns << nb) - size);
    }
    return true;
}

ZS_FN void zs_rle_fse(ZsFse* t, u32 sym) {
    t[0].sym = (u8)sym;
    t[0].nbits = 0;
    t[0].next = 0;
}

// Huffman tree description (RFC 8878 §4.2.1) -> decoding table; returns bytes consumed (0 = bad)
ZS_FN u64 zs_read_huffman(const u8* p, u64 n, ZsTables& T) {
    if (!n) return 0;
    const u32 hb = ZS_LD(p);
    u32 nw = 0;
    u64 used;
    if (hb >= 128) {  // direct 4-bit weights
        nw = hb - 127;
        used = 1 + (nw + 1) / 2;
        if (used > n) return 0;
        for (u32 i = 0; i < nw; ++i) {
            const u32 b = ZS_LD(p + 1 + i / 2);
            T.weights[i] = (u8)((i & 1) ? (b & 15) : (b >> 4));
        }
    } else {  // FSE-compressed weights, two interleaved states
        used = 1 + hb;
        if (used > n || hb == 0) return 0;
        u32 ms = 255, log = 0;
        const u64 h = zs_read_ncount(p + 1, hb, T.norm, &ms, &log, 6);
        if (!h || ms > 63 || !zs_build_fse(T.hw, T.norm, ms, log)) return 0;
        ZsBwd b;
        if (!b.init(p + 1 + h, hb - h)) return 0;
        u32 s1 = (u32)b.read(log), s2 = (u32)b.read(log);
        while (true) {
            if (nw >= 255) return 0;
            T.weights[nw++] = T.hw[s1].sym;
            s1 = T.hw[s1].next + (u32)b.read(T.hw[s1].nbits);
            if (b.pos < 0) {
                if (nw >= 255) return 0;
                T.weights[nw++] = T.hw[s2].sym;
                break;
            }
            if (nw >= 255) return 0;
            T.weights[nw++] = T.hw[s2].sym;
            s2 = T.hw[s2].next + (u32)b.read(T.hw[s2].nbits);
            if (b.pos < 0) {
                if (nw >= 255) return 0;
                T.weights[nw++] = T.hw[s1].sym;
                break;
            }
        }
    }
    // the last weight is implied: the weights' 2^(w-1) must sum to a power of two
    u32 total = 0;
    for (u32 i = 0; i < nw; ++i) {
        if (T.weights[i] > ZS_HUF_MAXBITS) return 0;
        if (T.weights[i]) total += 1u << (T.weights[i] - 1);
    }
    if (!total) return 0;
    const u32 maxb = zs_highbit(total) + 1;
    if (maxb > ZS_HUF_MAXBITS) return 0;
    const u32 rest = (1u << maxb) - total;
    if (rest & (rest - 1)) return 0;
    T.weights[nw++] = (u8)(zs_highbit(rest) + 1);
    // canonical ranks: symbols of weight w fill 2^(w-1) consecutive table entries, by weight
    u32 rank[ZS_HUF_MAXBITS + 2];
    for (u32 w = 0; w <= ZS_HUF_MAXBITS + 1; ++w) rank[w] = 0;
    for (u32 i = 0; i < nw; ++i) rank[T.weights[i]]++;
    u32 start = 0;
    for (u32 w = 1; w <= maxb; ++w) {
        const u32 c = rank[w];
        rank[w] = start;
        start += c << (w - 1);
    }
    if (start != (1u << maxb)) return 0;
    for (u32 i = 0; i < nw; ++i) {
        const u32 w = T.weights[i];
        if (!w) continue;
        const u32 len = 1u << (w - 1);
        const u16 e = (u16)((i << 8) | (maxb + 1 - w));
        for (u32 u = rank[w]; u < rank[w] + len; ++u) T.huf[u] = e;
        rank[w] += len;
    }
    T.huf_bits = maxb;
    T.have_huf = 1;
    return used;
}

// one Huffman-coded literal stream of `count` bytes into out (lane 0)
ZS_FN bool zs_huf_stream(const u8* p, u64 n, u64 count, const ZsTables& T, u8* out) {
    ZsBwd b;
    if (!b.init(p, n)) return false;
    const u32 mb = T.huf_bits;
    for (u64 i = 0; i < count; ++i) {
        const u16 e = T.huf[b.peek(mb)];
        b.pos -= e & 0xff;
        out[i] = (u8)(e >> 8);
    }
    return b.pos == 0;
}

// Decode one zstd frame sequence occupying src[0, sn) into dst[0, dn) (exact size).  Called by
// all lanes of the wave (uniform control flow).
ZS_FN bool zs_decode(const u8* src, u64 sn, u8* dst, u64 dn, u8* lit, ZsTables& T, ZsWork& W) {
    const u32 lane = ZS_LANE_ID;
    u64 ip = 0, op = 0;
    bool bad = false;
    // sequence state: meaningful in lane 0 only
    u32 rep[3] = {1, 4, 8};
    ZsBwd bs;
    u32 sll = 0, sof = 0, sml = 0;
    auto wave_copy = [&](u8* d, const u8* s, u64 len) {
        for (u64 j = lane; j < len; j += ZS_LANES) {
            const u8 c = ZS_LD(s + j);
            d[j] = c;
            W.ring[(op + j) & (ZS_RING - 1)] = c;
        }
    };
    while (!bad && ip < sn) {
        // ---- frame header ----
        if (ip + 4 > sn) { bad = true; break; }
        const u32 magic = ZS_LD(src + ip) | (ZS_LD(src + ip + 1) << 8) | (ZS_LD(src + ip + 2) << 16) | ((u32)ZS_LD(src + ip + 3) << 24);
        ip += 4;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
            if (ip + 4 > sn) { bad = true; break; }
            const u32 sz = ZS_LD(src + ip) | (ZS_LD(src + ip + 1) << 8) | (ZS_LD(src + ip + 2) << 16) | ((u32)ZS_LD(src + ip + 3) << 24);
            ip += 4;
            if (sz > sn - ip) { bad = true; break; }
            ip += sz;
            continue;
        }
        if (magic != 0xFD2FB528u || ip >= sn) { bad = true; break; }
        const u32 fhd = ZS_LD(src + ip++);
        const u32 fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did = fhd & 3;
        if (fhd & 8) { bad = true; break; }  // reserved bit
        if (!single) ip += 1;                 // window descriptor
        ip += did == 0 ? 0 : (did == 1 ? 1 : (did == 2 ? 2 : 4));
        ip += fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : (fcs_flag == 2 ? 4 : 8));
        if (ip > sn) { bad = true; break; }
        T.have_ll = T.have_ml = T.have_of = T.have_huf = 0;
        rep[0] = 1;
        rep[1] = 4;
        rep[2] = 8;
        // ---- blocks ----
        bool last = false;
        while (!bad && !last) {
            if (ip + 3 > sn) { bad = true; break; }
            const u32 bh = ZS_LD(src + ip) | (ZS_LD(src + ip + 1) << 8) | (ZS_LD(src + ip + 2) << 16);
            ip += 3;
            last = bh & 1;
            const u32 btype = (bh >> 1) & 3, bsize = bh >> 3;
            if (btype == 0) {  // raw
                if (bsize > sn - ip || bsize > dn - op) { bad = true; break; }
                wave_copy(dst + op, src + ip, bsize);
                ZS_LDS_SYNC();
                ip += bsize;
                op += bsize;
            } else if (btype == 1) {  // RLE
                if (ip >= sn || bsize > dn - op) { bad = true; break; }
                const u8 v = ZS_LD(src + ip);
                for (u64 j = lane; j < bsize; j += ZS_LANES) {
                    dst[op + j] = v;
                    W.ring[(op + j) & (ZS_RING - 1)] = v;
                }
                ZS_LDS_SYNC();
                ip += 1;
                op += bsize;
            } else if (btype == 2) {  // compressed
                if (bsize > sn - ip || bsize > ZS_MAX_BLOCK) { bad = true; break; }
                const u8* b = src + ip;
                const u64 bn = bsize;
                ip += bsize;
                // (A) lane 0: literals header, Huffman tree, sequences header and FSE tables
                // sh: 0 ok, 1 lit mode (0 raw, 1 rle, 2 huffman), 2 regen, 3 raw offset / rle byte,
                //     4 streams, 5-8 stream offsets, 9-12 stream sizes, 13 nseq
                if (lane == 0) {
                    u64 q = 0;
                    bool ok = true;
                    const u32 b0 = bn ? ZS_LD(b) : 0;
                    const u32 lt = b0 & 3, sf = (b0 >> 2) & 3;
                    u64 regen = 0, csize = 0;
                    u32 streams = 1;
                    if (lt <= 1) {
                        if (sf == 0 || sf == 2) { regen = b0 >> 3; q = 1; }
                        else if (sf == 1) { regen = bn >= 2 ? (b0 >> 4) + ((u64)ZS_LD(b + 1) << 4) : 0; q = 2; }
                        else { regen = bn >= 3 ? (b0 >> 4) + ((u64)ZS_LD(b + 1) << 4) + ((u64)ZS_LD(b + 2) << 12) : 0; q = 3; }
                        if (q > bn) ok = false;
                    } else {
                        u64 h = 0;
                        const u32 hl = sf <= 1 ? 3 : (sf == 2 ? 4 : 5);
                        if (hl > bn) ok = false;
                        for (u32 i = 0; ok && i < hl; ++i) h |= (u64)ZS_LD(b + i) << (8 * i);
                        const u32 fb = sf <= 1 ? 10 : (sf == 2 ? 14 : 18);
                        regen = (h >> 4) & ((1ULL << fb) - 1);
                        csize = (h >> (4 + fb)) & ((1ULL << fb) - 1);
                        streams = sf == 0 ? 1 : 4;
                        q = hl;
                    }
                    if (regen > ZS_MAX_BLOCK) ok = false;
                    W.sh[1] = lt == 0 ? 0 : (lt == 1 ? 1 : 2);
                    W.sh[2] = regen;
                    W.sh[4] = 0;
                    if (ok && lt == 0) {  // raw literals: read in place
                        if (regen > bn - q) ok = false;
                        W.sh[3] = q;
                        q += regen;
                    } else if (ok && lt == 1) {  // RLE literals
                        if (q >= bn) ok = false;
                        else W.sh[3] = ZS_LD(b + q);
                        q += 1;
                    } else if (ok) {  // Huffman, with its tree (2) or the previous block's (3)
                        if (csize > bn - q) ok = false;
                        u64 tq = 0;
                        if (ok && lt == 2) {
                            tq = zs_read_huffman(b + q, csize, T);
                            if (!tq) ok = false;
                        } else if (ok && !T.have_huf) {
                            ok = false;
                        }
                        if (ok) {
                            const u64 s0 = q + tq, sl = csize - tq;
                            if (streams == 1) {
                                W.sh[4] = 1;
                                W.sh[5] = s0;
                                W.sh[9] = sl;
                            } else if (sl < 6) {
                                ok = false;
                            } else {
                                const u64 z1 = ZS_LD(b + s0) | (ZS_LD(b + s0 + 1) << 8), z2 = ZS_LD(b + s0 + 2) | (ZS_LD(b + s0 + 3) << 8),
                                          z3 = ZS_LD(b + s0 + 4) | (ZS_LD(b + s0 + 5) << 8);
                                const u64 per = (regen + 3) / 4;
                                if (6 + z1 + z2 + z3 > sl || 3 * per > regen) ok = false;
                                else {
                                    W.sh[4] = 4;
                                    W.sh[5] = s0 + 6;
                                    W.sh[6] = s0 + 6 + z1;
                                    W.sh[7] = s0 + 6 + z1 + z2;
                                    W.sh[8] = s0 + 6 + z1 + z2 + z3;
                                    W.sh[9] = z1;
                                    W.sh[10] = z2;
                                    W.sh[11] = z3;
                                    W.sh[12] = sl - 6 - z1 - z2 - z3;
                                }
                            }
                            q += csize;
                        }
                    }
                    // sequences header and tables
                    if (ok && q >= bn) ok = false;
                    u64 nseq = 0;
                    if (ok) {
                        const u32 c0 = ZS_LD(b + q);
                        if (c0 < 128) { nseq = c0; q += 1; }
                        else if (c0 < 255) { if (q + 2 > bn) ok = false; else { nseq = ((c0 - 128) << 8) + ZS_LD(b + q + 1); q += 2; } }
                        else { if (q + 3 > bn) ok = false; else { nseq = ZS_LD(b + q + 1) + ((u64)ZS_LD(b + q + 2) << 8) + 0x7F00; q += 3; } }
                    }
                    if (ok && nseq) {
                        if (q >= bn) ok = false;
                        const u32 modes = ok ? ZS_LD(b + q++) : 0;
                        if (modes & 3) ok = false;
                        // LL, OF, ML tables in that order
                        for (int k = 0; k < 3 && ok; ++k) {
                            const u32 m = (modes >> (6 - 2 * k)) & 3;
                            ZsFse* t = k == 0 ? T.ll : (k == 1 ? T.of : T.ml);
                            u32* lg = k == 0 ? &T.ll_log : (k == 1 ? &T.of_log : &T.ml_log);
                            u32* have = k == 0 ? &T.have_ll : (k == 1 ? &T.have_of : &T.have_ml);
                            const u32 maxlog = k == 0 ? ZS_LL_MAXLOG : (k == 1 ? ZS_OF_MAXLOG : ZS_ML_MAXLOG);
                            const u32 maxsym = k == 0 ? 35 : (k == 1 ? 31 : 52);
                            if (m == 0) {  // predefined
                                const short* d = k == 0 ? zs_ll_def : (k == 1 ? zs_of_def : zs_ml_def);
                                const u32 ms = k == 0 ? 35 : (k == 1 ? 28 : 52);
                                for (u32 s = 0; s <= ms; ++s) T.norm[s] = d[s];
                                *lg = k == 1 ? 5 : 6;
                                ok = zs_build_fse(t, T.norm, ms, *lg);
                                *have = 1;
                            } else if (m == 1) {  // RLE
                                if (q >= bn) { ok = false; break; }
                                const u32 sym = ZS_LD(b + q++);
                                if (sym > maxsym) { ok = false; break; }
                                zs_rle_fse(t, sym);
                                *lg = 0;
                                *have = 1;
                            } else if (m == 2) {  // FSE table description
                                u32 ms = maxsym, lgv = 0;
                                const u64 used = zs_read_ncount(b + q, bn - q, T.norm, &ms, &lgv, maxlog);
                                if (!used) { ok = false; break; }
                                q += used;
                                *lg = lgv;
                                ok = zs_build_fse(t, T.norm, ms, lgv);
                                *have = 1;
                            } else if (!*have) {  // repeat without a previous table
                                ok = false;
                            }
                        }
                        if (ok && !bs.init(b + q, bn - q)) ok = false;
                        if (ok) {
                            sll = (u32)bs.read(T.ll_log);
                            sof = (u32)bs.read(T.of_log);
                            sml = (u32)bs.read(T.ml_log);
                        }
                    }
                    W.sh[13] = nseq;
                    W.sh[0] = ok ? 1 : 0;
                }
                ZS_LDS_SYNC();
                if (!W.sh[0]) { bad = true; break; }
                const u32 lmode = (u32)W.sh[1];
                const u64 regen = W.sh[2], nseq = W.sh[13];
                const u8* litp = lmode == 0 ? b + W.sh[3] : lit;
                const u8 lrle = (u8)W.sh[3];
                // (B) Huffman streams: one lane each
                if (lmode == 2) {
                    const u32 ns = (u32)W.sh[4];
                    const u64 per = ns == 1 ? regen : (regen + 3) / 4;
                    bool hok = true;
                    for (u32 k = lane; k < ns; k += ZS_LANES) {
                        const u64 cnt = ns == 1 ? regen : (k < 3 ? per : regen - 3 * per);
                        hok = zs_huf_stream(b + W.sh[5 + k], W.sh[9 + k], cnt, T, lit + k * per) && hok;
                    }
#ifdef ZS_HOST
                    const bool all = hok;
#else
                    const bool all = __ballot(!hok) == 0;
#endif
                    ZS_WAVE_SYNC();  // the literals (global scratch) are visible to every lane
                    if (!all) { bad = true; break; }
                }
                auto lit_at = [&](u64 i) -> u8 { return lmode == 1 ? lrle : ZS_LD(litp + i); };
                // (C) sequences: lane 0 decodes a batch into LDS, the wave executes it
                u64 lp = 0;  // literals consumed
                for (u64 s0 = 0; s0 < nseq && !bad; s0 += ZS_SEQ) {
                    const u32 nb = (u32)(nseq - s0 < ZS_SEQ ? nseq - s0 : ZS_SEQ);
                    if (lane == 0) {
                        bool ok = true;
                        for (u32 i = 0; i < nb; ++i) {
                            const u32 llc = T.ll[sll].sym, ofc = T.of[sof].sym, mlc = T.ml[sml].sym;
                            if (llc > 35 || mlc > 52 || ofc > 31) { ok = false; break; }
                            // values: offset, match length, literal length (RFC order)
                            const u64 ofv = (1ULL << ofc) + bs.read(ofc);
                            const u64 ml = zs_ml_base[mlc] + bs.read(zs_ml_bits[mlc]);
                            const u64 ll = zs_ll_base[llc] + bs.read(zs_ll_bits[llc]);
                            u64 off;
                            if (ofv > 3) {
                                off = ofv - 3;
                                rep[2] = rep[1];
                                rep[1] = rep[0];
                                rep[0] = (u32)off;
                            } else {
                                const u64 idx = ofv + (ll == 0 ? 1 : 0);
                                if (idx == 1) off = rep[0];
                                else if (idx == 2) { off = rep[1]; rep[1] = rep[0]; rep[0] = (u32)off; }
                                else if (idx == 3) { off = rep[2]; rep[2] = rep[1]; rep[1] = rep[0]; rep[0] = (u32)off; }
                                else {
                                    off = rep[0] - 1;
                                    off += off == 0 ? 1 : 0;  // as libzstd: 0 is forced to 1
                                    rep[2] = rep[1]; rep[1] = rep[0]; rep[0] = (u32)off;
                                }
                            }
                            // state updates (not after the last sequence): LL, ML, OF
                            if (s0 + i + 1 < nseq) {
                                sll = T.ll[sll].next + (u32)bs.read(T.ll[sll].nbits);
                                sml = T.ml[sml].next + (u32)bs.read(T.ml[sml].nbits);
                                sof = T.of[sof].next + (u32)bs.read(T.of[sof].nbits);
                            }
                            if (off > 0xFFFFFFFFull) { ok = false; break; }
                            W.ll[i] = (u32)ll;
                            W.ml[i] = (u32)ml;
                            W.off[i] = (u32)off;
                        }
                        if (ok && s0 + nb == nseq && bs.pos != 0) ok = false;
                        W.sh[0] = ok ? 1 : 0;
                    }
                    ZS_LDS_SYNC();
                    if (!W.sh[0]) { bad = true; break; }
                    for (u32 i = 0; i < nb; ++i) {
                        const u64 ll = W.ll[i], ml = W.ml[i], off = W.off[i];
                        // literals
                        if (ll > regen - lp || ll > dn - op) { bad = true; break; }
                        for (u64 j = lane; j < ll; j += ZS_LANES) {
                            const u8 c = lit_at(lp + j);
                            dst[op + j] = c;
                            W.ring[(op + j) & (ZS_RING - 1)] = c;
                        }
                        op += ll;
                        lp += ll;
                        if (off == 0 || off > op || ml > dn - op) { bad = true; break; }
                        ZS_LDS_SYNC();
                        // out[op + j] = out[op - off + j % off]; j % off advanced incrementally
                        // (r: this lane's j % off, step: ZS_LANES % off)
                        const u32 o32 = (u32)off, step = ZS_LANES % o32;
                        if (off <= ZS_RING / 2) {
                            // from the ring; a segment of at most ZS_RING - off bytes overwrites no
                            // slot it still reads
                            u64 done = 0;
                            while (done < ml) {
                                const u64 seg = ml - done < ZS_RING - off ? ml - done : ZS_RING - off;
                                const u64 w = op + done;
                                u32 r = lane % o32;
                                for (u64 j = lane; j < seg; j += ZS_LANES) {
                                    const u8 c = W.ring[(w - off + r) & (ZS_RING - 1)];
                                    dst[w + j] = c;
                                    W.ring[(w + j) & (ZS_RING - 1)] = c;
                                    r += step;
                                    if (r >= o32) r -= o32;
                                }
                                ZS_LDS_SYNC();
                                done += seg;
                            }
                        } else {  // a long offset: its source bytes from the output, made visible first
                            ZS_WAVE_SYNC();
                            const u64 w = op;
                            u32 r = lane % o32;
                            for (u64 j = lane; j < ml; j += ZS_LANES) {
                                const u8 c = ZS_LD(dst + w - off + r);
                                dst[w + j] = c;
                                W.ring[(w + j) & (ZS_RING - 1)] = c;
                                r += step;
                                if (r >= o32) r -= o32;
                            }
                            ZS_LDS_SYNC();
                        }
                        op += ml;
                    }
                }
                if (bad) break;
                // (D) the remaining literals
                const u64 rest = regen - lp;
                if (rest > dn - op) { bad = true; break; }
                for (u64 j = lane; j < rest; j += ZS_LANES) {
                    const u8 c = lit_at(lp + j);
                    dst[op + j] = c;
                    W.ring[(op + j) & (ZS_RING - 1)] = c;
                }
                ZS_LDS_SYNC();
                op += rest;
            } else {
                bad = true;
            }
        }
        if (!bad && checksum) {
            if (ip + 4 > sn) bad = true;
            else ip += 4;  // xxh64 content checksum: not verified (Parquet's page CRC is the check)
        }
    }
    return !bad && op == dn;
}
