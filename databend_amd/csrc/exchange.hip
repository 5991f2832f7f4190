// exchange.hip — the multi-GPU exchange of the C ABI over RCCL (include/dbgpu_agg.h: dbg_comm_*,
// dbg_agg_exchange (before_merge), dbg_agg_exchange_payload(_chunk) (before_partial) and the
// payload counts / export / import primitives they are built from).
#include "abi_internal.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>  // types only: the entry points are resolved with dlsym

// ------------------------------------------------------------------------------------------
// multi-GPU exchange over RCCL (replaces the Flight shuffle of
// AGG/aggregate_exchange_injector.rs:154-354 for the final-merge stage)
// ------------------------------------------------------------------------------------------
namespace {
// RCCL is loaded on first use, so the library (and a host without RCCL) works for single-GPU
// aggregation.  DBG_RCCL_LIB overrides the library path.
struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*ErrorString)(ncclResult_t) = nullptr;
};

RcclApi& rccl_api() {
    static RcclApi A;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* env = getenv("DBG_RCCL_LIB");
        const char* names[] = {env, "librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
        void* so = nullptr;
        for (const char* n : names)
            if (n && (so = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!so) {
            A.err = std::string("cannot load RCCL: ") + dlerror();
            return;
        }
        auto sym = [&](const char* n) { return dlsym(so, n); };
        A.GetUniqueId = (decltype(A.GetUniqueId))sym("ncclGetUniqueId");
        A.CommInitRank = (decltype(A.CommInitRank))sym("ncclCommInitRank");
        A.CommDestroy = (decltype(A.CommDestroy))sym("ncclCommDestroy");
        A.AllGather = (decltype(A.AllGather))sym("ncclAllGather");
        A.Send = (decltype(A.Send))sym("ncclSend");
        A.Recv = (decltype(A.Recv))sym("ncclRecv");
        A.GroupStart = (decltype(A.GroupStart))sym("ncclGroupStart");
        A.GroupEnd = (decltype(A.GroupEnd))sym("ncclGroupEnd");
        A.ErrorString = (decltype(A.ErrorString))sym("ncclGetErrorString");
        A.ok = A.GetUniqueId && A.CommInitRank && A.CommDestroy && A.AllGather && A.Send && A.Recv && A.GroupStart &&
               A.GroupEnd && A.ErrorString;
        if (!A.ok) A.err = "RCCL library lacks an entry point";
    });
    return A;
}
}  // namespace

#define RCCLCHECK(x)                                                                              \
    do {                                                                                          \
        ncclResult_t r_ = (x);                                                                    \
        if (r_ != ncclSuccess) return fail(DBG_ERR_DEVICE, std::string("RCCL: ") + R.ErrorString(r_)); \
    } while (0)

struct dbg_comm {
    ncclComm_t comm = nullptr;
    int n = 0, rank = 0, device = 0;
    u64* dsizes = nullptr;  // device: [2n] own sizes, then [n][2n] gathered
    u64* hsizes = nullptr;  // pinned mirror of the gathered sizes
    u8* send_recs = nullptr;
    u8* send_strs = nullptr;
    u64 send_recs_cap = 0, send_strs_cap = 0;
    hipEvent_t sent = nullptr;  // the last exchange's sends: the next export into the buffers waits
    bool sent_valid = false;
    hipEvent_t merged = nullptr;  // the final table's stream after a merge: cached receive buffers are reused behind it
    // before-partial payload exchange: send and receive buffers kept between calls (grown only)
    u8* pay_send = nullptr;
    u8* pay_recv[2] = {nullptr, nullptr};
    u64 pay_send_cap = 0, pay_recv_cap[2] = {0, 0};
    u64* pay_dbuf = nullptr;  // counts all-gather: own row, then n rows
    u64 pay_dbuf_cap = 0;
    // chunked payload shuffle: transfers on a stream of their own (overlapping the next chunk's
    // level-1 work on the table's stream), two send buffers used in turn
    hipStream_t xs = nullptr;
    hipEvent_t xexp = nullptr;      // the table's stream after a chunk's export
    hipEvent_t xsent[2] = {nullptr, nullptr};
    bool xsent_valid[2] = {false, false};
    u8* xsend[2] = {nullptr, nullptr};
    u64 xsend_cap[2] = {0, 0};
    int xi = 0;
    // receive buffers per chunk slot (records, states), grown only; chunk i of every shuffle lands
    // in slot i.  Receives run on xs, so a slot's next use is stream-ordered behind its last one.
    struct XRecv {
        u8* p[2] = {nullptr, nullptr};
        u64 cap[2] = {0, 0};
    };
    std::vector<XRecv> xrecv;
};

extern "C" {

int dbg_comm_get_unique_id(uint8_t* id) {
    if (!id) return fail(DBG_ERR_INVALID, "null argument");
    RcclApi& R = rccl_api();
    if (!R.ok) return fail(DBG_ERR_UNSUPPORTED, R.err);
    ncclUniqueId u;
    RCCLCHECK(R.GetUniqueId(&u));
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return DBG_OK;
}

int dbg_comm_create(const uint8_t* id, int n_ranks, int rank, int device, dbg_comm** out) {
    if (!id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(DBG_ERR_INVALID, "bad communicator arguments");
    RcclApi& R = rccl_api();
    if (!R.ok) return fail(DBG_ERR_UNSUPPORTED, R.err);
    if (device < 0) HIPCHECK(hipGetDevice(&device));
    HIPCHECK(hipSetDevice(device));
    auto* c = new dbg_comm();
    c->n = n_ranks;
    c->rank = rank;
    c->device = device;
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclResult_t r = R.CommInitRank(&c->comm, n_ranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(DBG_ERR_DEVICE, std::string("ncclCommInitRank: ") + R.ErrorString(r));
    }
    const u64 words = (2ull * n_ranks + 1) * (n_ranks + 1);  // own [2n + 1] sizes + ok word, then n rows
    if (dev_alloc((void**)&c->dsizes, words * 8) != DBG_OK || hipHostMalloc((void**)&c->hsizes, words * 8, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&c->sent, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->merged, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->xexp, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->xsent[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->xsent[1], hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&c->xs, hipStreamNonBlocking) != hipSuccess) {
        dbg_comm_destroy(c);
        return fail(DBG_ERR_OOM, "communicator scratch");
    }
    *out = c;
    return DBG_OK;
}

void dbg_comm_destroy(dbg_comm* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->sent_valid) hipEventSynchronize(c->sent);
    if (c->xs) hipStreamSynchronize(c->xs);
    RcclApi& R = rccl_api();
    if (c->comm && R.ok) R.CommDestroy(c->comm);
    if (c->dsizes) hipFree(c->dsizes);
    if (c->send_recs) hipFree(c->send_recs);
    if (c->send_strs) hipFree(c->send_strs);
    if (c->pay_send) hipFree(c->pay_send);
    for (int k = 0; k < 2; ++k)
        if (c->pay_recv[k]) hipFree(c->pay_recv[k]);
    if (c->pay_dbuf) hipFree(c->pay_dbuf);
    if (c->hsizes) hipHostFree(c->hsizes);
    if (c->sent) hipEventDestroy(c->sent);
    if (c->merged) hipEventDestroy(c->merged);
    for (int i = 0; i < 2; ++i) {
        if (c->xsend[i]) hipFree(c->xsend[i]);
        if (c->xsent[i]) hipEventDestroy(c->xsent[i]);
    }
    for (auto& x : c->xrecv)
        for (int k = 0; k < 2; ++k)
            if (x.p[k]) hipFree(x.p[k]);
    if (c->xexp) hipEventDestroy(c->xexp);
    if (c->xs) hipStreamDestroy(c->xs);
    delete c;
}

// ---- before-partial shuffle of the partitioned payload (group_by_shuffle_mode = before_partial,
//      settings_default.rs:469-473): level-1 partition p (of 2^PP_L1_BITS) belongs to rank
//      p * n / 2^PP_L1_BITS, so every group's records meet on one rank and are aggregated once ----
static void payload_owned(u32 d, u32 n, u32& lo, u32& hi) {
    const u64 P = 1ull << PP_L1_BITS;
    lo = (u32)((d * P + n - 1) / n);
    hi = (u32)(((d + 1) * P + n - 1) / n);
}

static int payload_check(dbg_agg_handle* h) {
    if (!h->pp) return fail(DBG_ERR_UNSUPPORTED, "payload exchange: the handle is not in partitioned mode (dbg_agg_set_strategy)");
    if (h->spec.pp_str) return fail(DBG_ERR_UNSUPPORTED, "payload exchange: string keys (records may reference local rows)");
    return DBG_OK;
}

// level-1 segments [first[k], end) of each record kind: per-partition counts
static void payload_counts_range(const dbg_agg_handle* h, const u32 first[2], uint64_t* part_counts) {
    const u64 P = 1ull << PP_L1_BITS;
    for (int k = 0; k < 2; ++k) {
        for (u64 p = 0; p < P; ++p) part_counts[k * P + p] = 0;
        const auto& segs = h->ppk[k].segs;
        for (size_t i = first[k]; i < segs.size(); ++i)
            for (u64 p = 0; p < P; ++p) part_counts[k * P + p] += segs[i].off[p + 1] - segs[i].off[p];
    }
}

int dbg_agg_payload_counts(dbg_agg_handle* h, uint64_t* part_counts, uint32_t* widths) {
    const uint32_t first[2] = {0, 0};
    return dbg_agg_payload_counts_from(h, first, part_counts, widths, nullptr);
}

int dbg_agg_payload_counts_from(dbg_agg_handle* h, const uint32_t first_seg[2], uint64_t* part_counts, uint32_t* widths,
                                uint32_t* n_segs) {
    if (!h || !part_counts || !first_seg) return fail(DBG_ERR_INVALID, "null argument");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    RETURN_IF(payload_check(h));
    for (int k = 0; k < 2; ++k)
        if (first_seg[k] > h->ppk[k].segs.size()) return fail(DBG_ERR_INVALID, "dbg_agg_payload_counts_from: first_seg past the payload");
    payload_counts_range(h, first_seg, part_counts);
    if (widths) {
        widths[0] = h->spec.pp_rw_raw;
        widths[1] = h->spec.pp_rw_state;
    }
    if (n_segs) {
        n_segs[0] = (uint32_t)h->ppk[0].segs.size();
        n_segs[1] = (uint32_t)h->ppk[1].segs.size();
    }
    return DBG_OK;
}

// segments [first[k], end) packed destination-major (partition-major within a destination, segment
// order within a partition) into dev_buf, on the table's stream.  prepare: the copy ranges built
// and uploaded (the steps that can fail); launch: the copies
struct ExportPlan {
    const CopyRange* dr[2] = {nullptr, nullptr};
    u32 n[2] = {0, 0};
};
static int payload_export_prepare(dbg_agg_handle* h, u32 n_ranks, const u32 first[2], ExportPlan& X) {
    u64 dst = 0;
    for (int k = 0; k < 2; ++k) {
        const auto& K = h->ppk[k];
        const u64 rw = k ? h->spec.pp_rw_state : h->spec.pp_rw_raw;
        std::vector<CopyRange> rs;
        for (u32 d = 0; d < n_ranks; ++d) {
            u32 lo, hi;
            payload_owned(d, n_ranks, lo, hi);
            for (u32 p = lo; p < hi; ++p)
                for (size_t i = first[k]; i < K.segs.size(); ++i) {
                    const auto& sg = K.segs[i];
                    const u64 n = sg.off[p + 1] - sg.off[p];
                    if (!n) continue;
                    if (!rs.empty() && rs.back().src + rs.back().n == (sg.base + sg.off[p]) * rw && rs.back().dst + rs.back().n == dst)
                        rs.back().n += n * rw;  // contiguous with the previous range (one segment)
                    else
                        rs.push_back(CopyRange{(sg.base + sg.off[p]) * rw, dst, n * rw});
                    dst += n * rw;
                }
        }
        if (rs.empty()) continue;
        CopyRange* dr = nullptr;
        RETURN_IF(dev_alloc((void**)&dr, rs.size() * sizeof(CopyRange)));
        h->owned.push_back({dr, rs.size() * sizeof(CopyRange)});  // freed at the next reset
        HIPCHECK(hipMemcpy(dr, rs.data(), rs.size() * sizeof(CopyRange), hipMemcpyHostToDevice));
        X.dr[k] = dr;
        X.n[k] = (u32)rs.size();
    }
    return DBG_OK;
}

static int payload_export_launch(dbg_agg_handle* h, const ExportPlan& X, void* dev_buf) {
    for (int k = 0; k < 2; ++k) {
        if (!X.n[k]) continue;
        launch_copy_ranges(h->stream, h->ppk[k].l1, (u8*)dev_buf, X.dr[k], X.n[k]);
        HIPCHECK(hipGetLastError());
    }
    return DBG_OK;
}

static int payload_export_range(dbg_agg_handle* h, u32 n_ranks, const u32 first[2], void* dev_buf) {
    ExportPlan X;
    RETURN_IF(payload_export_prepare(h, n_ranks, first, X));
    return payload_export_launch(h, X, dev_buf);
}

int dbg_agg_payload_export(dbg_agg_handle* h, uint32_t n_ranks, void* dev_buf) {
    const uint32_t first[2] = {0, 0};
    return dbg_agg_payload_export_from(h, n_ranks, first, dev_buf);
}

int dbg_agg_payload_export_from(dbg_agg_handle* h, uint32_t n_ranks, const uint32_t first_seg[2], void* dev_buf) {
    if (!h || !dev_buf || !first_seg || n_ranks == 0 || n_ranks > (1u << PP_L1_BITS))
        return fail(DBG_ERR_INVALID, "dbg_agg_payload_export: bad argument");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    RETURN_IF(payload_check(h));
    for (int k = 0; k < 2; ++k)
        if (first_seg[k] > h->ppk[k].segs.size()) return fail(DBG_ERR_INVALID, "dbg_agg_payload_export_from: first_seg past the payload");
    RETURN_IF(payload_export_range(h, n_ranks, first_seg, dev_buf));
    HIPCHECK(hipStreamSynchronize(h->stream));  // dev_buf is complete when the call returns
    return DBG_OK;
}

// The received records of n_chunks shipments become this rank's level-1 payload: per kind, chunk c's
// buffer holds source-major (partition-major within a source) records of this rank's partitions;
// part_counts[c][s][k][P]; one level-1 segment per (chunk, source).
static int payload_import_chunks(dbg_agg_handle* h, u32 n_ranks, u32 rank, u32 n_chunks, const uint64_t* part_counts,
                                 const void* const* raw, const void* const* state) {
    const u64 P = 1ull << PP_L1_BITS;
    u32 lo, hi;
    payload_owned(rank, n_ranks, lo, hi);
    for (int k = 0; k < 2; ++k) {
        auto& K = h->ppk[k];
        const u64 rw = k ? h->spec.pp_rw_state : h->spec.pp_rw_raw;
        std::vector<dbg_agg_handle::Seg> segs;
        std::vector<u64> chunk_bytes(n_chunks, 0);
        u64 total = 0;
        for (u32 c = 0; c < n_chunks; ++c)
            for (u32 s = 0; s < n_ranks; ++s) {
                const uint64_t* cnt = part_counts + (((u64)c * n_ranks + s) * 2 + k) * P;
                dbg_agg_handle::Seg sg{total, 0, std::vector<u64>(P + 1, 0)};
                u64 run = 0;
                for (u64 p = 0; p < P; ++p) {
                    sg.off[p] = run;
                    if (p >= lo && p < hi) run += cnt[p];
                }
                sg.off[P] = run;
                sg.n = run;
                total += run;
                chunk_bytes[c] += run * rw;
                segs.push_back(std::move(sg));
            }
        for (u32 c = 0; c < n_chunks; ++c)
            if (chunk_bytes[c] && !(k ? state[c] : raw[c])) return fail(DBG_ERR_INVALID, "dbg_agg_payload_import: records missing");
        HIPCHECK(hipStreamSynchronize(h->stream));  // the export has read the old payload
        if (total > K.l1_cap) {
            if (K.l1) HIPCHECK(hipFree(K.l1));
            K.l1 = nullptr;
            K.l1_cap = 0;
            RETURN_IF(dev_alloc((void**)&K.l1, total * rw + 64));  // slack: the aggregation reads whole words
            K.l1_cap = total;
        }
        u64 at = 0;
        for (u32 c = 0; c < n_chunks; ++c) {
            if (chunk_bytes[c]) HIPCHECK(hipMemcpyAsync(K.l1 + at, k ? state[c] : raw[c], chunk_bytes[c], hipMemcpyDeviceToDevice, h->stream));
            at += chunk_bytes[c];
        }
        K.l1_n = total;
        K.dig_n = 0;  // imported records carry no digits
        K.segs = std::move(segs);
    }
    HIPCHECK(hipStreamSynchronize(h->stream));  // the caller may release the received buffers
    h->pp_grec_ready = false;
    h->finalized = false;
    h->xfirst[0] = h->xfirst[1] = 0;
    return DBG_OK;
}

int dbg_agg_payload_import(dbg_agg_handle* h, uint32_t n_ranks, uint32_t rank, const uint64_t* part_counts, const void* raw_records,
                           const void* state_records) {
    return dbg_agg_payload_import_chunks(h, n_ranks, rank, 1, part_counts, &raw_records, &state_records);
}

int dbg_agg_payload_import_chunks(dbg_agg_handle* h, uint32_t n_ranks, uint32_t rank, uint32_t n_chunks, const uint64_t* part_counts,
                                  const void* const* raw_records, const void* const* state_records) {
    if (!h || !part_counts || !raw_records || !state_records || n_chunks == 0 || n_ranks == 0 || rank >= n_ranks ||
        n_ranks > (1u << PP_L1_BITS))
        return fail(DBG_ERR_INVALID, "dbg_agg_payload_import: bad argument");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    RETURN_IF(payload_check(h));
    return payload_import_chunks(h, n_ranks, rank, n_chunks, part_counts, raw_records, state_records);
}

// Byte plan of the before-partial shuffle for one rank (host only): send_bytes[k * n + d] = this
// rank's kind-k records of the partitions rank d owns, recv_bytes[k * n + s] = source s's kind-k
// records of this rank's partitions; widths from the params' payload record formats.
static void payload_plan(u32 n, u32 me, const uint32_t widths[2], const uint64_t* all_counts, u64* send_bytes, u64* recv_bytes) {
    const u64 P = 1ull << PP_L1_BITS;
    u32 lo_me, hi_me;
    payload_owned(me, n, lo_me, hi_me);
    for (int k = 0; k < 2; ++k)
        for (u32 d = 0; d < n; ++d) {
            u32 lo, hi;
            payload_owned(d, n, lo, hi);
            u64 sb = 0, rb = 0;
            for (u32 p = lo; p < hi; ++p) sb += all_counts[((u64)me * 2 + k) * P + p];
            for (u32 p = lo_me; p < hi_me; ++p) rb += all_counts[((u64)d * 2 + k) * P + p];
            send_bytes[(u64)k * n + d] = sb * widths[k];
            recv_bytes[(u64)k * n + d] = rb * widths[k];
        }
}

int dbg_payload_exchange_plan(const dbg_agg_params* params, uint32_t n_ranks, uint32_t rank, const uint64_t* all_counts,
                              uint32_t* widths, uint64_t* send_bytes, uint64_t* recv_bytes) {
    if (!params || !all_counts || !send_bytes || !recv_bytes || n_ranks == 0 || rank >= n_ranks || n_ranks > (1u << PP_L1_BITS))
        return fail(DBG_ERR_INVALID, "dbg_payload_exchange_plan: bad argument");
    Spec S;
    std::vector<dbg_datatype> rt;
    RETURN_IF(build_spec(params, S, rt));
    const uint32_t w[2] = {S.pp_rw_raw, S.pp_rw_state};
    if (widths) {
        widths[0] = w[0];
        widths[1] = w[1];
    }
    payload_plan(n_ranks, rank, w, all_counts, send_bytes, recv_bytes);
    return DBG_OK;
}

static int grow_dev(u8** p, u64* cap, u64 need) {
    if (need <= *cap && *p) return DBG_OK;
    if (*p) HIPCHECK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    const u64 c = std::max<u64>(need, 1 << 20);
    RETURN_IF(dev_alloc((void**)p, c));
    *cap = c;
    return DBG_OK;
}

// One all-gather of a per-rank word (every rank calls it): true when every rank passed `ok`.
// A rank that failed locally after the counts all-gather still takes part in this one, so no peer
// is left waiting in a send / receive the failed rank never posts.
static int all_ok(dbg_comm* c, RcclApi& R, hipStream_t s, bool ok, int* bad_rank) {
    const u32 n = (u32)c->n;
    u64* d = c->dsizes;  // >= 2n (n + 1) words
    u64* hh = c->hsizes;
    hh[0] = ok ? 1 : 0;
    HIPCHECK(hipMemcpyAsync(d, hh, 8, hipMemcpyHostToDevice, s));
    RCCLCHECK(R.AllGather(d, d + 1, 1, ncclUint64, c->comm, s));
    HIPCHECK(hipMemcpyAsync(hh + 1, d + 1, 8ull * n, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    *bad_rank = -1;
    for (u32 r = 0; r < n; ++r)
        if (hh[1 + r] != 1) {
            *bad_rank = (int)r;
            break;
        }
    return DBG_OK;
}

int dbg_agg_exchange_payload(dbg_comm* c, dbg_agg_handle* h, dbg_exchange_stats* stats) {
    if (!c || !h) return fail(DBG_ERR_INVALID, "null argument");
    if (h->device != c->device) return fail(DBG_ERR_INVALID, "communicator and table are on different devices");
    RcclApi& R = rccl_api();
    if (!R.ok) return fail(DBG_ERR_UNSUPPORTED, R.err);
    HIPCHECK(hipSetDevice(c->device));
    const u32 n = (u32)c->n, me = (u32)c->rank;
    const u64 P = 1ull << PP_L1_BITS, W = 2 * P + 1;  // per rank: counts [2][P] + an eligibility flag
    std::vector<u64> mine(W, 0);
    uint32_t widths[2] = {0, 0};
    const int rc0 = dbg_agg_payload_counts(h, mine.data(), widths);
    mine[2 * P] = rc0 == DBG_OK ? 1 : 0;
    hipStream_t s = h->stream;
    // buffers of the last call are reused once its sends have left them
    if (c->sent_valid) HIPCHECK(hipEventSynchronize(c->sent));
    c->sent_valid = false;
    // 1. every rank's counts (and whether it can take part), one all-gather into a cached buffer
    if (c->pay_dbuf_cap < W * (n + 1)) {
        if (c->pay_dbuf) HIPCHECK(hipFree(c->pay_dbuf));
        c->pay_dbuf = nullptr;
        c->pay_dbuf_cap = 0;
        RETURN_IF(dev_alloc((void**)&c->pay_dbuf, 8 * W * (n + 1)));
        c->pay_dbuf_cap = W * (n + 1);
    }
    u64* dbuf = c->pay_dbuf;
    std::vector<u64> all(W * n);
    HIPCHECK(hipMemcpyAsync(dbuf, mine.data(), 8 * W, hipMemcpyHostToDevice, s));
    RCCLCHECK(R.AllGather(dbuf, dbuf + W, W, ncclUint64, c->comm, s));
    HIPCHECK(hipMemcpyAsync(all.data(), dbuf + W, 8 * W * n, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    for (u32 r = 0; r < n; ++r)
        if (all[(u64)r * W + 2 * P] != 1)  // every rank sees the same flags: all return here
            return rc0 != DBG_OK ? rc0 : fail(DBG_ERR_UNSUPPORTED, "payload exchange: rank " + std::to_string(r) + " cannot take part");
    // 2. the byte plan, the buffers and this rank's records packed destination-major.  A local
    //    failure here is made collective (all_ok) before any rank posts a send or receive.
    std::vector<u64> pc(2 * P * n);
    for (u32 r = 0; r < n; ++r)
        for (u64 x = 0; x < 2 * P; ++x) pc[(u64)r * 2 * P + x] = all[(u64)r * W + x];
    std::vector<u64> send_bytes(2 * n), recv_bytes(2 * n);
    payload_plan(n, me, widths, pc.data(), send_bytes.data(), recv_bytes.data());
    u64 kind_total[2] = {0, 0}, recv_total[2] = {0, 0};
    for (int k = 0; k < 2; ++k)
        for (u32 d = 0; d < n; ++d) {
            kind_total[k] += send_bytes[(u64)k * n + d];
            recv_total[k] += recv_bytes[(u64)k * n + d];
        }
    int rc = grow_dev(&c->pay_send, &c->pay_send_cap, kind_total[0] + kind_total[1]);
    for (int k = 0; k < 2 && rc == DBG_OK; ++k) rc = grow_dev(&c->pay_recv[k], &c->pay_recv_cap[k], recv_total[k]);
    if (rc == DBG_OK) rc = dbg_agg_payload_export(h, n, c->pay_send);
    const std::string local_err = rc == DBG_OK ? std::string() : std::string(dbg_last_error());
    int bad = -1;
    RETURN_IF(all_ok(c, R, s, rc == DBG_OK, &bad));
    if (bad >= 0) {
        if (rc != DBG_OK) return fail(rc, local_err);
        return fail(DBG_ERR_DEVICE, "payload exchange: rank " + std::to_string(bad) + " failed before the transfer");
    }
    // 3. grouped point-to-point over xGMI (self included)
    RCCLCHECK(R.GroupStart());
    for (int k = 0; k < 2; ++k) {
        u64 so = k ? kind_total[0] : 0, ro = 0;
        for (u32 p = 0; p < n; ++p) {
            const u64 sb = send_bytes[(u64)k * n + p], rb = recv_bytes[(u64)k * n + p];
            if (sb) RCCLCHECK(R.Send(c->pay_send + so, sb, ncclUint8, (int)p, c->comm, s));
            if (rb) RCCLCHECK(R.Recv(c->pay_recv[k] + ro, rb, ncclUint8, (int)p, c->comm, s));
            so += sb;
            ro += rb;
        }
    }
    RCCLCHECK(R.GroupEnd());
    // 4. the received records become this rank's level-1 payload (import copies them: the
    //    communicator's buffers are free again when it returns)
    rc = dbg_agg_payload_import(h, n, me, pc.data(), c->pay_recv[0], c->pay_recv[1]);
    HIPCHECK(hipEventRecord(c->sent, s));
    c->sent_valid = true;
    if (rc != DBG_OK) return rc;
    if (stats) {
        stats->sent_bytes = kind_total[0] + kind_total[1];
        stats->remote_bytes = stats->sent_bytes - send_bytes[me] - send_bytes[(u64)n + me];
        stats->received_records = 0;
        for (int k = 0; k < 2; ++k) stats->received_records += recv_total[k] / std::max<u32>(widths[k], 1);
        stats->received_string_bytes = 0;
    }
    return DBG_OK;
}

// Chunked before-partial shuffle: ships the level-1 segments appended since the previous call
// (one add_groups chunk, typically) while the caller goes on with the next chunk.  Per call: one
// all-gather of the chunk's counts (and every rank's ok) on the communicator's stream — it needs
// only the host-known segment counts, not the scatter's records; receive buffers for the chunk; a
// collective ok; the export on the table's stream (behind the chunk's scatter) into one of two
// send buffers; then the grouped send/recv on the communicator's stream behind that export — the
// call returns without waiting for it, and the next add_groups' kernels on the table's stream
// overlap the transfer.  The last call (last = 1) waits for every transfer and makes what arrived
// the payload (one level-1 segment per chunk and source), like dbg_agg_exchange_payload.
int dbg_agg_exchange_payload_chunk(dbg_comm* c, dbg_agg_handle* h, int last, dbg_exchange_stats* stats) {
    if (!c || !h) return fail(DBG_ERR_INVALID, "null argument");
    if (h->device != c->device) return fail(DBG_ERR_INVALID, "communicator and table are on different devices");
    RcclApi& R = rccl_api();
    if (!R.ok) return fail(DBG_ERR_UNSUPPORTED, R.err);
    HIPCHECK(hipSetDevice(c->device));
    const u32 n = (u32)c->n, me = (u32)c->rank;
    const u64 P = 1ull << PP_L1_BITS, W = 2 * P + 1;
    hipStream_t s = h->stream, xs = c->xs;
    std::vector<u64> mine(W, 0);
    uint32_t widths[2] = {0, 0}, nseg[2] = {0, 0};
    const int rc0 = dbg_agg_payload_counts_from(h, h->xfirst, mine.data(), widths, nseg);
    mine[2 * P] = rc0 == DBG_OK ? 1 : 0;
    // 1. the chunk's counts, every rank's, on the communicator's stream
    if (c->pay_dbuf_cap < W * (n + 1)) {
        HIPCHECK(hipStreamSynchronize(xs));
        if (c->pay_dbuf) HIPCHECK(hipFree(c->pay_dbuf));
        c->pay_dbuf = nullptr;
        c->pay_dbuf_cap = 0;
        RETURN_IF(dev_alloc((void**)&c->pay_dbuf, 8 * W * (n + 1)));
        c->pay_dbuf_cap = W * (n + 1);
    }
    u64* dbuf = c->pay_dbuf;
    std::vector<u64> all(W * n);
    HIPCHECK(hipMemcpyAsync(dbuf, mine.data(), 8 * W, hipMemcpyHostToDevice, xs));
    RCCLCHECK(R.AllGather(dbuf, dbuf + W, W, ncclUint64, c->comm, xs));
    HIPCHECK(hipMemcpyAsync(all.data(), dbuf + W, 8 * W * n, hipMemcpyDeviceToHost, xs));
    HIPCHECK(hipStreamSynchronize(xs));
    for (u32 r = 0; r < n; ++r)
        if (all[(u64)r * W + 2 * P] != 1)
            return rc0 != DBG_OK ? rc0 : fail(DBG_ERR_UNSUPPORTED, "payload exchange: rank " + std::to_string(r) + " cannot take part");
    // 2. plan, buffers (a collective ok before any transfer)
    dbg_agg_handle::XChunk X;
    X.pc.assign(2 * P * n, 0);
    for (u32 r = 0; r < n; ++r)
        for (u64 x = 0; x < 2 * P; ++x) X.pc[(u64)r * 2 * P + x] = all[(u64)r * W + x];
    std::vector<u64> send_bytes(2 * n), recv_bytes(2 * n);
    payload_plan(n, me, widths, X.pc.data(), send_bytes.data(), recv_bytes.data());
    u64 kind_total[2] = {0, 0}, recv_total[2] = {0, 0};
    for (int k = 0; k < 2; ++k)
        for (u32 d = 0; d < n; ++d) {
            kind_total[k] += send_bytes[(u64)k * n + d];
            recv_total[k] += recv_bytes[(u64)k * n + d];
        }
    const int xi = c->xi;
    int rc = DBG_OK;
    if (c->xsent_valid[xi]) {  // this send buffer's previous transfer has left it
        HIPCHECK(hipEventSynchronize(c->xsent[xi]));
        c->xsent_valid[xi] = false;
    }
    if (kind_total[0] + kind_total[1] > c->xsend_cap[xi]) rc = grow_dev(&c->xsend[xi], &c->xsend_cap[xi], kind_total[0] + kind_total[1]);
    // this chunk's receive slot: reused as is when large enough (the steady state); a slot that
    // must grow waits for the transfers still queued on xs (an abandoned shuffle's receives)
    const size_t slot = h->xchunks.size();
    if (c->xrecv.size() <= slot) c->xrecv.resize(slot + 1);
    auto& XR = c->xrecv[slot];
    for (int k = 0; k < 2 && rc == DBG_OK; ++k)
        if (recv_total[k]) {
            if (recv_total[k] > XR.cap[k]) {
                if (hipStreamSynchronize(xs) != hipSuccess) rc = fail(DBG_ERR_DEVICE, "hipStreamSynchronize");
                else rc = grow_dev(&XR.p[k], &XR.cap[k], recv_total[k]);
            }
            if (rc == DBG_OK) X.recv[k] = XR.p[k];
        }
    // the export's ranges (what can still fail) before the collective ok
    const u32 first[2] = {h->xfirst[0], h->xfirst[1]};
    ExportPlan EP;
    if (rc == DBG_OK) rc = payload_export_prepare(h, n, first, EP);
    const std::string local_err = rc == DBG_OK ? std::string() : std::string(dbg_last_error());
    int bad = -1;
    RETURN_IF(all_ok(c, R, xs, rc == DBG_OK, &bad));
    if (bad >= 0) {
        if (rc != DBG_OK) return fail(rc, local_err);
        return fail(DBG_ERR_DEVICE, "payload exchange: rank " + std::to_string(bad) + " failed before the transfer");
    }
    // 3. export behind the chunk's scatter, transfer behind the export
    RETURN_IF(payload_export_launch(h, EP, c->xsend[xi]));
    HIPCHECK(hipEventRecord(c->xexp, s));
    HIPCHECK(hipStreamWaitEvent(xs, c->xexp, 0));
    RCCLCHECK(R.GroupStart());
    for (int k = 0; k < 2; ++k) {
        u64 so = k ? kind_total[0] : 0, ro = 0;
        for (u32 p = 0; p < n; ++p) {
            const u64 sb = send_bytes[(u64)k * n + p], rb = recv_bytes[(u64)k * n + p];
            if (sb) RCCLCHECK(R.Send(c->xsend[xi] + so, sb, ncclUint8, (int)p, c->comm, xs));
            if (rb) RCCLCHECK(R.Recv((u8*)X.recv[k] + ro, rb, ncclUint8, (int)p, c->comm, xs));
            so += sb;
            ro += rb;
        }
    }
    RCCLCHECK(R.GroupEnd());
    HIPCHECK(hipEventRecord(c->xsent[xi], xs));
    c->xsent_valid[xi] = true;
    c->xi ^= 1;
    h->xfirst[0] = nseg[0];
    h->xfirst[1] = nseg[1];
    h->xchunks.push_back(std::move(X));
    if (stats) {
        stats->sent_bytes = kind_total[0] + kind_total[1];
        stats->remote_bytes = stats->sent_bytes - send_bytes[me] - send_bytes[(u64)n + me];
        stats->received_records = 0;
        for (int k = 0; k < 2; ++k) stats->received_records += recv_total[k] / std::max<u32>(widths[k], 1);
        stats->received_string_bytes = 0;
    }
    if (!last) return DBG_OK;
    // 4. the last chunk: every transfer done, the arrivals become the payload
    HIPCHECK(hipStreamSynchronize(xs));
    const u32 nc = (u32)h->xchunks.size();
    std::vector<u64> pcs;
    std::vector<const void*> raws(nc), states(nc);
    for (u32 i = 0; i < nc; ++i) {
        const auto& x = h->xchunks[i];
        pcs.insert(pcs.end(), x.pc.begin(), x.pc.end());
        raws[i] = x.recv[0];
        states[i] = x.recv[1];
    }
    rc = payload_import_chunks(h, n, me, nc, pcs.data(), raws.data(), states.data());  // copies, then synchronises
    h->xchunks.clear();
    return rc;
}

// Byte plan of the before_merge exchange for one rank (host only; Payload::scatter's routing,
// EAGG/payload.rs:356-391, shipped as AggregateExchangeInjector does per destination,
// AGG/aggregate_exchange_injector.rs:154-235).  all[s * 2n + 2d + {0, 1}] = the records / string
// bytes source s sends to rank d.  send_bytes[d] / send_bytes[n + d]: this rank's record / blob
// bytes for d in export (partition-major) order; recv_bytes[s] / recv_bytes[n + s] and
// recv_records[s]: what source s sends this rank, in merge (source-major) order.  The offsets are
// their prefix sums.  Self included.
static void merge_plan(u32 n, u32 me, u32 w, const u64* all, u64* send_bytes, u64* recv_bytes, u64* recv_records) {
    for (u32 d = 0; d < n; ++d) {
        send_bytes[d] = all[(u64)me * 2 * n + 2 * d] * w;
        send_bytes[n + d] = all[(u64)me * 2 * n + 2 * d + 1];
        recv_records[d] = all[(u64)d * 2 * n + 2 * me];
        recv_bytes[d] = recv_records[d] * w;
        recv_bytes[n + d] = all[(u64)d * 2 * n + 2 * me + 1];
    }
}

int dbg_merge_exchange_plan(const dbg_agg_params* params, uint32_t n_ranks, uint32_t rank, const uint64_t* all_sizes,
                            uint32_t* record_width, uint64_t* send_bytes, uint64_t* recv_bytes, uint64_t* recv_records) {
    if (!params || !all_sizes || !send_bytes || !recv_bytes || !recv_records || n_ranks == 0 || rank >= n_ranks)
        return fail(DBG_ERR_INVALID, "dbg_merge_exchange_plan: bad argument");
    Spec S;
    std::vector<dbg_datatype> rt;
    RETURN_IF(build_spec(params, S, rt));
    if (record_width) *record_width = S.rec_width;
    merge_plan(n_ranks, rank, S.rec_width, all_sizes, send_bytes, recv_bytes, recv_records);
    return DBG_OK;
}

// A receive buffer of the final table: its cached one when no group references it (grown only),
// otherwise a fresh allocation the table owns until its reset.
static int xrecv_buffer(dbg_agg_handle* fh, int k, u64 bytes, void** out) {
    bytes = std::max<u64>(bytes, 16);
    if (fh->xrecv_busy) {
        DevBuf b;
        b.bytes = bytes;
        RETURN_IF(dev_alloc(&b.p, bytes));
        fh->owned.push_back(b);
        *out = b.p;
        return DBG_OK;
    }
    DevBuf& b = fh->xrecv[k];
    if (b.bytes < bytes) {
        if (b.p) HIPCHECK(hipFree(b.p));
        b.p = nullptr;
        b.bytes = 0;
        RETURN_IF(dev_alloc(&b.p, bytes));
        b.bytes = bytes;
    }
    *out = b.p;
    return DBG_OK;
}

int dbg_agg_exchange(dbg_comm* c, dbg_agg_handle* partial, dbg_agg_handle* final_h, dbg_exchange_stats* stats) {
    if (!c || !partial || !final_h) return fail(DBG_ERR_INVALID, "null argument");
    if (partial->device != c->device || final_h->device != c->device)
        return fail(DBG_ERR_INVALID, "communicator and tables are on different devices");
    if (partial->spec.n_keys != final_h->spec.n_keys || partial->spec.n_aggs != final_h->spec.n_aggs ||
        partial->spec.stride_words != final_h->spec.stride_words)
        return fail(DBG_ERR_INVALID, "partial and final tables have different parameters");
    RcclApi& R = rccl_api();
    if (!R.ok) return fail(DBG_ERR_UNSUPPORTED, R.err);
    HIPCHECK(hipSetDevice(c->device));
    const u32 n = (u32)c->n, me = (u32)c->rank, W = 2 * n + 1;  // per rank: [records, bytes] per destination + ok
    std::vector<u64> counts(n, 0), sbytes(n, 0);
    // Payload::scatter's routing (EAGG/payload.rs:377-383): group -> rank hash % n.  A local
    // failure here still takes part in the sizes all-gather (ok word 0), so no peer is left
    // waiting in it; every rank then sees the same flags and all return together.
    int rc = dbg_agg_partition(partial, n, 0, counts.data(), sbytes.data());
    uint32_t w = 0;
    if (rc == DBG_OK) rc = dbg_agg_record_width(partial, &w);
    std::string local_err = rc == DBG_OK ? std::string() : std::string(dbg_last_error());
    if (rc != DBG_OK) std::fill(counts.begin(), counts.end(), 0), std::fill(sbytes.begin(), sbytes.end(), 0);
    hipStream_t s = partial->stream;
    // 1. sizes: every rank's [records, string bytes] per destination and its ok word, one all-gather
    u64* own = c->hsizes;
    for (u32 d = 0; d < n; ++d) {
        own[2 * d] = counts[d];
        own[2 * d + 1] = sbytes[d];
    }
    own[2 * n] = rc == DBG_OK ? 1 : 0;
    HIPCHECK(hipMemcpyAsync(c->dsizes, own, 8ull * W, hipMemcpyHostToDevice, s));
    RCCLCHECK(R.AllGather(c->dsizes, c->dsizes + W, W, ncclUint64, c->comm, s));
    HIPCHECK(hipMemcpyAsync(c->hsizes + W, c->dsizes + W, 8ull * W * n, hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
    std::vector<u64> all(2ull * n * n);
    for (u32 r = 0; r < n; ++r) {
        const u64* row = c->hsizes + W + (u64)r * W;
        if (row[2 * n] != 1) {
            if (rc != DBG_OK) return fail(rc, local_err);
            return fail(DBG_ERR_DEVICE, "exchange: rank " + std::to_string(r) + " failed before the size exchange");
        }
        std::copy(row, row + 2 * n, all.begin() + (u64)r * 2 * n);
    }
    // 2. the plan, records + blobs (partition-major) into the communicator's send buffers, the
    //    final table's receive buffers.  A local failure from here on is made collective (all_ok)
    //    before any rank posts a send or receive.
    std::vector<u64> send_b(2 * n), recv_b(2 * n), seg_r(n), seg_s(n);
    merge_plan(n, me, w, all.data(), send_b.data(), recv_b.data(), seg_r.data());
    u64 tot_r = 0, tot_s = 0, rr = 0, rs = 0;
    for (u32 d = 0; d < n; ++d) {
        tot_r += counts[d];
        tot_s += sbytes[d];
        seg_s[d] = recv_b[n + d];
        rr += seg_r[d];
        rs += seg_s[d];
    }
    if (c->sent_valid) HIPCHECK(hipEventSynchronize(c->sent));
    c->sent_valid = false;
    rc = grow_dev(&c->send_recs, &c->send_recs_cap, tot_r * w);
    if (rc == DBG_OK) rc = grow_dev(&c->send_strs, &c->send_strs_cap, tot_s);
    if (rc == DBG_OK) rc = dbg_agg_export_records(partial, c->send_recs, c->send_strs);
    if (rc == DBG_OK && (send_b[me] != counts[me] * w || seg_r[me] != counts[me] || seg_s[me] != sbytes[me]))
        rc = fail(DBG_ERR_INTERNAL, "exchange sizes disagree");
    void *rrec = nullptr, *rstr = nullptr;
    if (rc == DBG_OK) rc = xrecv_buffer(final_h, 0, rr * w, &rrec);
    if (rc == DBG_OK) rc = xrecv_buffer(final_h, 1, rs, &rstr);
    // the last merge into the cached buffers has read them before this exchange overwrites them
    if (rc == DBG_OK && final_h->stream != s) {
        if (hipEventRecord(c->merged, final_h->stream) != hipSuccess || hipStreamWaitEvent(s, c->merged, 0) != hipSuccess)
            rc = fail(DBG_ERR_DEVICE, "exchange: stream ordering");
    }
    local_err = rc == DBG_OK ? std::string() : std::string(dbg_last_error());
    int bad = -1;
    RETURN_IF(all_ok(c, R, s, rc == DBG_OK, &bad));
    if (bad >= 0) {
        if (rc != DBG_OK) return fail(rc, local_err);
        return fail(DBG_ERR_DEVICE, "exchange: rank " + std::to_string(bad) + " failed before the transfer");
    }
    // 3. grouped point-to-point over xGMI (records and blobs; self included)
    RCCLCHECK(R.GroupStart());
    u64 so_r = 0, so_s = 0, ro_r = 0, ro_s = 0;
    for (u32 p = 0; p < n; ++p) {
        if (send_b[p]) RCCLCHECK(R.Send(c->send_recs + so_r, send_b[p], ncclUint8, (int)p, c->comm, s));
        if (send_b[n + p]) RCCLCHECK(R.Send(c->send_strs + so_s, send_b[n + p], ncclUint8, (int)p, c->comm, s));
        if (recv_b[p]) RCCLCHECK(R.Recv((u8*)rrec + ro_r, recv_b[p], ncclUint8, (int)p, c->comm, s));
        if (recv_b[n + p]) RCCLCHECK(R.Recv((u8*)rstr + ro_s, recv_b[n + p], ncclUint8, (int)p, c->comm, s));
        so_r += send_b[p];
        so_s += send_b[n + p];
        ro_r += recv_b[p];
        ro_s += recv_b[n + p];
    }
    RCCLCHECK(R.GroupEnd());
    HIPCHECK(hipEventRecord(c->sent, s));
    c->sent_valid = true;
    if (final_h->stream != s) HIPCHECK(hipStreamWaitEvent(final_h->stream, c->sent, 0));
    // 4. merge_states of what arrived into this rank's final table; its entries may point into
    //    the receive buffers until its next reset
    final_h->xrecv_busy = true;
    RETURN_IF(dbg_agg_merge_records(final_h, rrec, rstr, (int32_t)n, seg_r.data(), seg_s.data()));
    if (stats) {
        stats->sent_bytes = tot_r * w + tot_s;
        stats->remote_bytes = stats->sent_bytes - counts[me] * w - sbytes[me];
        stats->received_records = rr;
        stats->received_string_bytes = rs;
    }
    return DBG_OK;
}

}  // extern "C"

