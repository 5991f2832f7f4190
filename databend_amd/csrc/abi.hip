// abi.hip — the C ABI of libdbgpu_agg.so (include/dbgpu_agg.h): handles, device memory, streams,
// deferred overflow handling, result extraction, records, profiling.  The multi-GPU exchange over
// RCCL is in exchange.hip; what both share is abi_internal.hpp.
//
// A handle is one AggregateHashTable (EAGG/aggregate_hashtable.rs:47) living in HBM.  It owns a
// HIP stream (or borrows the caller's) and its allocations; nothing here runs on the CPU except
// bookkeeping — there is no CPU fallback: a missing/unsupported case returns an error code.
#include "abi_internal.hpp"

// ------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;
static const char* const MINMAX_SPIN_MSG =
    "Decimal128 MIN/MAX: a state update gave up after 2^20 contended attempts (the result would be wrong)";

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
// the other translation units (scan.hip) report through the same last-error slot
int abi_fail(int code, const std::string& msg) { return fail(code, msg); }

// ------------------------------------------------------------------------------------------
// profiling: HIP events around every launch (dbg_prof_enable)
// ------------------------------------------------------------------------------------------
namespace prof {
struct Pending {
    std::string name;
    hipEvent_t a, b;
};
static std::mutex mu;
static bool enabled = false;
static std::vector<Pending> pending;
static std::vector<hipEvent_t> free_events;  // pooled: hipEventCreate is not free
static std::vector<std::pair<std::string, std::pair<double, uint64_t>>> totals;

static hipEvent_t get_event() {
    std::lock_guard<std::mutex> g(mu);
    if (!free_events.empty()) {
        hipEvent_t e = free_events.back();
        free_events.pop_back();
        return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
}

static void resolve_locked() {
    for (auto& p : pending) {
        float ms = 0;
        (void)hipEventSynchronize(p.b);
        (void)hipEventElapsedTime(&ms, p.a, p.b);
        free_events.push_back(p.a);
        free_events.push_back(p.b);
        bool found = false;
        for (auto& t : totals)
            if (t.first == p.name) {
                t.second.first += ms;
                t.second.second += 1;
                found = true;
                break;
            }
        if (!found) totals.push_back({p.name, {(double)ms, 1}});
    }
    pending.clear();
}

struct Scope;
static thread_local Scope* cur = nullptr;  // the innermost open scope of this thread
struct Scope {
    bool on;
    bool ext = false;  // a kernel launch stamped a / b itself (prof_ext_events)
    hipStream_t s;
    hipEvent_t a, b;
    const char* name;
    Scope* outer;
    Scope(const char* n, hipStream_t st) : on(enabled), s(st), name(n), outer(cur) {
        if (on) {
            a = get_event();
            b = get_event();
            (void)hipEventRecord(a, s);
            cur = this;
        }
    }
    ~Scope() {
        if (on) {
            cur = outer;
            if (!ext) (void)hipEventRecord(b, s);
            std::lock_guard<std::mutex> g(mu);
            pending.push_back({name, a, b});
        }
    }
};
}  // namespace prof

// A kernel that is the timed work of the innermost open scope: launched with
// hipExtLaunchKernelGGL and these two events, they are stamped at the kernel's own start and end
// (what rocprofv3 reports), not at the stream's event packets around it.  The scope then measures
// that kernel alone.
bool prof_ext_events(hipEvent_t* a, hipEvent_t* b) {
    prof::Scope* c = prof::cur;
    if (!c || !c->on || c->ext) return false;
    c->ext = true;
    *a = c->a;
    *b = c->b;
    return true;
}

// the same HIP-event scopes for the other translation units (scan.hip)
void* prof_scope_begin(const char* name, hipStream_t s) { return prof::enabled ? new prof::Scope(name, s) : nullptr; }
void prof_scope_end(void* p) { delete (prof::Scope*)p; }


int dev_alloc(void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return fail(DBG_ERR_OOM, std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
    return DBG_OK;
}

static int own_copy(dbg_agg_handle* h, const void* src, size_t bytes, const void** out) {
    DevBuf b;
    b.bytes = bytes;
    RETURN_IF(dev_alloc(&b.p, bytes));
    h->owned.push_back(b);
    if (bytes) HIPCHECK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, h->stream));
    *out = b.p;
    return DBG_OK;
}

// ------------------------------------------------------------------------------------------
// spec construction: AggregatorParams -> slot layout (+ result types, per the factory)
// ------------------------------------------------------------------------------------------
static bool is_signed_i(int t) { return t == DBG_INT8 || t == DBG_INT16 || t == DBG_INT32 || t == DBG_INT64; }
static bool is_unsigned_i(int t) { return t == DBG_UINT8 || t == DBG_UINT16 || t == DBG_UINT32 || t == DBG_UINT64; }
static bool is_float(int t) { return t == DBG_FLOAT32 || t == DBG_FLOAT64; }
static bool valid_type(int t) { return t >= DBG_INT8 && t <= DBG_BOOLEAN; }

// AggregateFunction::return_type() of the factory-built function.
static int result_type_of(const dbg_agg_spec& s, dbg_datatype* out) {
    int t = s.arg.type;
    dbg_datatype r{DBG_UINT64, 0, 0, 0, 0};
    if (s.kind == DBG_AGG_COUNT) {
        *out = r;  // AggregateCountFunction: UInt64, never nullable
        return DBG_OK;
    }
    if (t < 0 || !valid_type(t)) return fail(DBG_ERR_INVALID, "aggregate needs an argument type");
    switch (s.kind) {
        case DBG_AGG_SUM:  // ResultTypeOfUnary::Sum
            if (is_signed_i(t)) r.type = DBG_INT64;
            else if (is_unsigned_i(t)) r.type = DBG_UINT64;
            else if (is_float(t)) r.type = DBG_FLOAT64;
            else if (t == DBG_DECIMAL128) r = dbg_datatype{DBG_DECIMAL128, 38, s.arg.scale, 0, 0};
            else return fail(DBG_ERR_UNSUPPORTED, "sum: unsupported argument type");
            break;
        case DBG_AGG_AVG:
            if (is_signed_i(t) || is_unsigned_i(t) || is_float(t)) r.type = DBG_FLOAT64;
            else if (t == DBG_DECIMAL128) r = dbg_datatype{DBG_DECIMAL128, 38, (uint8_t)std::max<int>(s.arg.scale, 4), 0, 0};
            else return fail(DBG_ERR_UNSUPPORTED, "avg: unsupported argument type");
            break;
        case DBG_AGG_AVG_SQL:  // divide's result type (EXP/types/decimal.rs:1015-1037; numbers: Float64)
            if (is_signed_i(t) || is_unsigned_i(t) || is_float(t)) r.type = DBG_FLOAT64;
            else if (t == DBG_DECIMAL128)
                r = dbg_datatype{DBG_DECIMAL128, 38, (uint8_t)std::max<int>(s.arg.scale, std::min<int>(s.arg.scale + 6, 12)), 0, 0};
            else return fail(DBG_ERR_UNSUPPORTED, "avg: unsupported argument type");
            break;
        case DBG_AGG_MIN: case DBG_AGG_MAX:
            // Boolean: MinMaxAnyState<BooleanType> (false < true; the 0/1 value in an i64 state word,
            // one byte per row in results and borsh Option<bool>); String stays on the CPU path
            if (t == DBG_STRING) return fail(DBG_ERR_UNSUPPORTED, "min/max: String arguments stay on the CPU path");
            r = dbg_datatype{t, s.arg.precision, s.arg.scale, 0, 0};
            break;
        default: return fail(DBG_ERR_INVALID, "unknown aggregate kind");
    }
    r.nullable = (s.or_null || s.arg.nullable) ? 1 : 0;
    *out = r;
    return DBG_OK;
}

int build_spec(const dbg_agg_params* p, Spec& S, std::vector<dbg_datatype>& rtypes) {
    memset(&S, 0, sizeof(S));
    S.x_pp_cap = ~0u;  // no test hook (dbg_agg_create reads them)
    if (p->n_group_cols < 1 || p->n_group_cols > DBG_MAX_KEYS) return fail(DBG_ERR_UNSUPPORTED, "1..8 group columns supported");
    if (p->n_aggs < 0 || p->n_aggs > DBG_MAX_AGGS) return fail(DBG_ERR_UNSUPPORTED, "at most 32 aggregates");
    S.n_keys = p->n_group_cols;
    S.n_aggs = p->n_aggs;
    // inline packing: row format [validity bytes][values] (EAGG/payload.rs:100-129)
    int w = 0;
    bool fixed = true;
    for (int c = 0; c < S.n_keys; ++c) {
        dbg_datatype t = p->group_types[c];
        if (!valid_type(t.type)) return fail(DBG_ERR_INVALID, "bad group type");
        S.key_types[c] = t;
        if (t.type == DBG_STRING) S.has_strings = 1;
        if (t.type == DBG_STRING || t.type == DBG_DECIMAL128) fixed = false;
        if (t.nullable) S.voff[c] = (uint8_t)w++;
    }
    for (int c = 0; c < S.n_keys; ++c) {
        S.koff[c] = (uint8_t)w;
        w += type_width(S.key_types[c].type);
    }
    S.inline_keys = fixed && w <= 8;
    S.inline_width = w;
    // record layout: [hash][validity bytes][values, 8-aligned][state words]
    u32 off = 8;
    for (int c = 0; c < S.n_keys; ++c)
        if (S.key_types[c].nullable) S.rec_val_off[c] = off++;
    off = (off + 7) & ~7u;
    for (int c = 0; c < S.n_keys; ++c) {
        S.rec_key_off[c] = off;
        int t = S.key_types[c].type;
        off += (t == DBG_STRING || t == DBG_DECIMAL128) ? 16 : 8;
    }
    // state words
    int word = 1, flag_bits = 0;
    rtypes.clear();
    for (int a = 0; a < S.n_aggs; ++a) {
        const dbg_agg_spec& s = p->aggs[a];
        DAgg& A = S.aggs[a];
        dbg_datatype rt;
        RETURN_IF(result_type_of(s, &rt));
        rtypes.push_back(rt);
        const bool sql_avg = s.kind == DBG_AGG_AVG_SQL;
        A.kind = sql_avg ? DBG_AGG_AVG : s.kind;  // same state; only the result differs
        A.arg_type = s.kind == DBG_AGG_COUNT && s.arg.type < 0 ? -1 : s.arg.type;
        A.arg_nullable = A.arg_type >= 0 ? s.arg.nullable : 0;
        int t = A.arg_type;
        A.sumk = t == DBG_DECIMAL128 ? SUMK_I128 : (is_float(t) ? SUMK_F64 : SUMK_I64);
        A.mmk = is_unsigned_i(t) ? MMK_U64 : (is_float(t) ? MMK_F64 : MMK_I64);
        if (t == DBG_DECIMAL128 && s.arg.precision > 18) A.mmk = MMK_I128;
        A.w0 = word;
        switch (A.kind) {
            case DBG_AGG_COUNT: A.nwords = 1; break;
            case DBG_AGG_SUM: A.nwords = A.sumk == SUMK_I128 ? 2 : 1; break;
            case DBG_AGG_AVG: A.nwords = A.sumk == SUMK_I128 ? 3 : 2; break;
            default: A.nwords = A.mmk == MMK_I128 ? 3 : 1;
        }
        word += A.nwords;
        A.flag_bit = -1;
        if ((s.kind == DBG_AGG_SUM || s.kind == DBG_AGG_MIN || s.kind == DBG_AGG_MAX) && A.arg_nullable) A.flag_bit = flag_bits++;
        A.res_type = rt.type;
        A.res_precision = rt.precision;
        A.res_scale = rt.scale;
        A.res_nullable = rt.nullable;
        // SUM's range check (DecimalSumState<OVERFLOW>, p <= 18) also guards AVG_SQL's sum
        A.dec_check = ((s.kind == DBG_AGG_SUM || sql_avg) && t == DBG_DECIMAL128 && s.arg.precision <= 18) ? 1 : 0;
        A.scale_add = (A.kind == DBG_AGG_AVG && t == DBG_DECIMAL128) ? (int)rt.scale - (int)s.arg.scale : 0;
        A.avg_round = sql_avg && t == DBG_DECIMAL128;
        A.res_width = (int)type_width(rt.type);
        A.ser_flags = 0;
        if (s.kind != DBG_AGG_COUNT) {
            if (s.or_null) A.ser_flags |= SER_OR_NULL;
            if (A.arg_nullable) A.ser_flags |= SER_NULL_ADPT;
        }
    }
    if (flag_bits > 64) return fail(DBG_ERR_UNSUPPORTED, "too many nullable aggregates");
    S.flags_word = flag_bits ? word++ : -1;
    S.n_words = word - 1;
    if (word > DBG_MAX_WORDS) return fail(DBG_ERR_UNSUPPORTED, "aggregate states too wide");
    int sw = 1;
    while (sw < word && sw < 8) sw <<= 1;
    if (word > 8) sw = (word + 7) & ~7;
    S.stride_words = sw;
    // one non-null String key: the HBM slot also caches the key (agg_insert_str1_kernel), so a
    // probe compares in the slot's own line instead of reading the representative row
    S.tstride = sw;
    S.kc_word = 0;
    if (S.n_keys == 1 && S.key_types[0].type == DBG_STRING && !S.key_types[0].nullable) {
        const int need = word + 1 + KC_KEY_WORDS;  // entry + states (+ flags) + hdr + key words
        int ts = 1;
        while (ts < need && ts < 8) ts <<= 1;
        if (need > 8) ts = (need + 7) & ~7;
        if (ts <= DBG_MAX_WORDS) {
            S.tstride = ts;
            S.kc_word = word;
        }
    }
    for (int w = 0; w < DBG_MAX_WORDS; ++w) S.slot_init[w] = w == 0 ? SLOT_EMPTY : 0;
    for (int a = 0; a < S.n_aggs; ++a)
        if (S.aggs[a].kind == DBG_AGG_MIN || S.aggs[a].kind == DBG_AGG_MAX)
            for (int k = 0; k < S.aggs[a].nwords; ++k) S.slot_init[S.aggs[a].w0 + k] = state_init_word(S.aggs[a], k);
    S.rec_state_off = off;
    S.rec_width = off + 8 * (u32)S.n_words;
    // partitioned payload record formats (pp.hip): key part, then each argument value aligned to
    // its width, then one validity bit per nullable argument
    S.pp_str = S.has_strings;
    S.pp_kw = S.has_strings ? 48 : (u32)((S.inline_width + 7) & ~7);
    // raw records pack the arguments right after the key bytes (a 12-byte key + two Int16 = 16 B);
    // key words are compared / copied with the last one masked to the key bytes
    S.pp_klast_mask = (S.has_strings || (S.inline_width & 7) == 0) ? ~0ULL : ((1ULL << (8 * (S.inline_width & 7))) - 1);
    u32 po = S.has_strings ? S.pp_kw : (u32)S.inline_width;
    int vbits = 0;
    for (int a = 0; a < S.n_aggs; ++a) {
        const DAgg& A = S.aggs[a];
        S.pp_avbit[a] = -1;
        S.pp_aoff[a] = 0;
        if (A.arg_type < 0) continue;
        const u32 aw = A.arg_type == DBG_BOOLEAN ? 1 : type_width(A.arg_type);
        const u32 al = aw >= 8 ? 8 : aw;
        po = (po + al - 1) & ~(al - 1);
        S.pp_aoff[a] = (uint16_t)po;
        po += aw;
        if (A.arg_nullable) S.pp_avbit[a] = (int16_t)vbits++;
    }
    S.pp_avoff = po;
    po += (u32)(vbits + 7) / 8;
    S.pp_rw_raw = (po + 7) & ~7u;
    if (!vbits) S.pp_avoff = S.pp_rw_raw;
    S.pp_rw_state = S.pp_kw + 8 * (u32)S.n_words;
    S.pp_sw = 1 + S.pp_kw / 8 + (u32)S.n_words;
    S.pp_ok = S.pp_rw_raw <= 256 && S.pp_rw_state <= 256 && vbits <= 64 && S.pp_sw <= 64;
    return DBG_OK;
}

// ------------------------------------------------------------------------------------------
// table allocation / growth
// ------------------------------------------------------------------------------------------
static void table_init_now(dbg_agg_handle* h) {
    if (!h->init_pending) return;
    h->init_pending = false;
    prof::Scope ps("table_init", h->stream);
    launch_table_init(h->stream, h->dspec, h->spec, h->slots, h->cap, nullptr);
}

static int part_flush(dbg_agg_handle* h);

// The table as the kernels see it; a deferred initialisation, or a held-back partitioned table
// stage, is launched first (stream order).
static TableDesc table_desc(dbg_agg_handle* h) {
    if (h->def_part) (void)part_flush(h);  // launch errors surface from the stream's next check
    table_init_now(h);
    TableDesc t;
    t.slots = h->slots;
    t.cap = h->cap;
    t.stride_words = (u32)h->spec.tstride;
    t.probe_limit = (u32)std::min<u64>(h->cap, 512);
    t.counters = h->counters;
    t.ovf_rows = h->ovf_rows;
    t.ovf_rows_cap = h->ovf_rows_cap;
    t.ovf_recs = h->ovf_recs;
    t.ovf_recs_cap = h->ovf_recs_cap;
    t.scratch = h->scratch;
    t.scr_blocks = h->scr_blocks;

    return t;
}

static int flush_deferred(dbg_agg_handle* h) {
    if (h->def_part) RETURN_IF(part_flush(h));
    if (!h->def_on) return DBG_OK;
    h->def_on = false;
    {
        prof::Scope ps("agg_insert", h->stream);
        launch_insert(h->stream, h->dspec, h->spec, h->dbatches, h->def_bid, h->def_rows, false, table_desc(h), true, &h->def_hb);
    }
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

static u64 pow2_at_least(u64 x) {
    u64 p = 1;
    while (p < x) p <<= 1;
    return p;
}

static int alloc_table(dbg_agg_handle* h, u64 cap, u64** out) {
    size_t bytes = (size_t)(cap + 1) * h->spec.tstride * 8;
    RETURN_IF(dev_alloc((void**)out, bytes));
    prof::Scope ps("table_init", h->stream);
    launch_table_init(h->stream, h->dspec, h->spec, *out, cap);
    return DBG_OK;
}

static int grow_table(dbg_agg_handle* h, u64 new_cap) {
    table_init_now(h);  // the old table is rehashed below
    u64* ns = nullptr;
    RETURN_IF(alloc_table(h, new_cap, &ns));
    u64* old = h->slots;
    u64 old_cap = h->cap;
    h->slots = ns;
    h->cap = new_cap;
    {
        prof::Scope ps("agg_rehash", h->stream);
        launch_rehash(h->stream, h->dspec, h->spec, h->dbatches, old, old_cap, table_desc(h));
    }
    HIPCHECK(hipStreamSynchronize(h->stream));
    HIPCHECK(hipFree(old));
    return DBG_OK;
}

static int read_counters(dbg_agg_handle* h) {
    HIPCHECK(hipMemcpyAsync(h->hcounters, h->counters, CNT_WORDS * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    return DBG_OK;
}

// Resolve deferred overflow: grow so that every pending group fits at <= 50% load, re-insert.
static int resolve_overflow(dbg_agg_handle* h) {
    RETURN_IF(read_counters(h));
    bool grew = false;  // sized by overflowed rows this call: shrink to the groups once known
    for (int round = 0; round < 4; ++round) {
        u64 claims = h->hcounters[CNT_CLAIMS], orows = h->hcounters[CNT_OVF_ROWS], orecs = h->hcounters[CNT_OVF_RECS];
        if (h->hcounters[CNT_ERR] & ERR_OVF_LOST) return fail(DBG_ERR_INTERNAL, "overflow list exhausted");
        if (orows == 0 && orecs == 0) {
            h->pending_rows = h->pending_recs = 0;
            // keep the load factor sane for the next batch (the reference resizes at 1/1.5)
            const u64 fit = std::max<u64>(pow2_at_least((u64)(claims * 2.0) + 1), 1024);
            if ((double)claims * 1.5 > (double)h->cap) RETURN_IF(grow_table(h, fit));
            // overflow growth sizes by overflowed ROWS (an upper bound on the groups they hold):
            // once the groups are known, give back a table twice or more what they need at the
            // reference's load factor (get_capacity_for_count: next_pow2(1.5 x count),
            // EAGG/aggregate_hashtable.rs:567-569), so table_init, the finalize scans and
            // partitioned inserts touch what the groups need (C5: a first-step overflow left a
            // 2^25-slot, 2 GB table for 7e6 groups in every later step)
            else if (grew) {
                const u64 fit15 = std::max<u64>(pow2_at_least((u64)(claims * 1.5) + 1), 1024);
                if (h->cap >= 2 * fit15 && fit15 >= h->init_cap) RETURN_IF(grow_table(h, fit15));
            }
            return DBG_OK;
        }
        u64 need = pow2_at_least(2 * (claims + orows + orecs) + 1);
        if (need > h->cap) {
            RETURN_IF(grow_table(h, need));
            grew = true;
        }
        HIPCHECK(hipMemsetAsync(h->counters + CNT_OVF_ROWS, 0, 16, h->stream));
        {
            prof::Scope ps("agg_retry", h->stream);
            launch_retry(h->stream, h->dspec, h->spec, h->dbatches, table_desc(h), orows, orecs, h->ovf_rows, h->ovf_recs);
        }
        RETURN_IF(read_counters(h));
    }
    return fail(DBG_ERR_INTERNAL, "overflow did not converge");
}

// Make sure the deferred-overflow lists can hold everything the next launch may push.
static int ensure_ovf(dbg_agg_handle* h, u64 add_rows, u64 add_recs) {
    u64 need_rows = h->pending_rows + add_rows, need_recs = h->pending_recs + add_recs;
    if (need_rows <= h->ovf_rows_cap && need_recs <= h->ovf_recs_cap) {
        h->pending_rows = need_rows;
        h->pending_recs = need_recs;
        return DBG_OK;
    }
    // drain what is pending, then reallocate the lists at the new size
    RETURN_IF(resolve_overflow(h));
    need_rows = add_rows;
    need_recs = add_recs;
    if (need_rows > h->ovf_rows_cap) {
        if (h->ovf_rows) HIPCHECK(hipFree(h->ovf_rows));
        h->ovf_rows_cap = std::max<u64>(need_rows, 1024);
        RETURN_IF(dev_alloc((void**)&h->ovf_rows, h->ovf_rows_cap * 8));
    }
    if (need_recs > h->ovf_recs_cap) {
        if (h->ovf_recs) HIPCHECK(hipFree(h->ovf_recs));
        h->ovf_recs_cap = std::max<u64>(need_recs, 1024);
        RETURN_IF(dev_alloc((void**)&h->ovf_recs, h->ovf_recs_cap * h->spec.tstride * 8));
    }
    h->pending_rows = need_rows;
    h->pending_recs = need_recs;
    return DBG_OK;
}

// ------------------------------------------------------------------------------------------
// batches
// ------------------------------------------------------------------------------------------
static int new_batch(dbg_agg_handle* h, BatchDesc** staging, u32* bid) {
    if (h->n_batches >= 0xFFFE) return fail(DBG_ERR_UNSUPPORTED, "more than 65534 batches before reset");
    u32 id = h->n_batches + 1;
    if (id >= h->batch_cap) {
        u64 ncap = std::max<u64>(64, h->batch_cap * 2);
        BatchDesc* nb = nullptr;
        RETURN_IF(dev_alloc((void**)&nb, ncap * sizeof(BatchDesc)));
        if (h->dbatches) {
            HIPCHECK(hipMemcpyAsync(nb, h->dbatches, h->batch_cap * sizeof(BatchDesc), hipMemcpyDeviceToDevice, h->stream));
            HIPCHECK(hipStreamSynchronize(h->stream));
            HIPCHECK(hipFree(h->dbatches));
        }
        h->dbatches = nb;
        h->batch_cap = ncap;
    }
    // pinned staging descriptors are pooled: slot id is reused after dbg_agg_reset (which
    // synchronises the stream, so the previous upload from it has completed)
    while (h->pinned_descs.size() <= id) {
        BatchDesc* chunk = nullptr;
        HIPCHECK(hipHostMalloc((void**)&chunk, 64 * sizeof(BatchDesc), hipHostMallocDefault));
        h->pinned_chunks.push_back(chunk);
        for (int k = 0; k < 64; ++k) h->pinned_descs.push_back(chunk + k);
    }
    BatchDesc* st = h->pinned_descs[id];
    memset(st, 0, sizeof(BatchDesc));
    h->n_batches = id;
    *staging = st;
    *bid = id;
    return DBG_OK;
}

static u64 desc_hash(const BatchDesc& d) {
    const u64* w = (const u64*)&d;
    u64 hv = 0x9E3779B97F4A7C15ULL;
    for (size_t k = 0; k < sizeof(BatchDesc) / 8; ++k) hv = (hv ^ w[k]) * 0xff51afd7ed558ccdULL;
    return hv;
}

static int upload_batch(dbg_agg_handle* h, BatchDesc* st, u32 bid) {
    HIPCHECK(hipMemcpyAsync(h->dbatches + bid, st, sizeof(BatchDesc), hipMemcpyHostToDevice, h->stream));
    h->uploads_pending = true;
    return DBG_OK;
}

// Upload a filled batch descriptor, or reuse an identical cached one (device-resident inputs
// only: the descriptor is then pointers alone and immutable).  A cache hit needs no upload, so
// a steady stream of re-submitted device batches never forces dbg_agg_reset to synchronise.
static int submit_batch(dbg_agg_handle* h, BatchDesc** pst, u32* pbid, bool cacheable) {
    BatchDesc* st = *pst;
    u32 bid = *pbid;
    if (cacheable && bid == h->n_cached + 1 && h->desc_cache.size() < 64) {
        u64 hv = desc_hash(*st);
        u32 hit = 0;
        for (u32 k = 0; k < h->desc_cache.size() && !hit; ++k)
            if (h->desc_cache[k].first == hv && memcmp(&h->desc_cache[k].second, st, sizeof(BatchDesc)) == 0) hit = k + 1;
        if (hit) {
            h->n_batches = bid - 1;  // give the fresh id back
            *pbid = hit;
            *pst = &h->desc_cache[hit - 1].second;
            return DBG_OK;
        }
        RETURN_IF(upload_batch(h, st, bid));
        h->desc_cache.push_back({hv, *st});
        h->n_cached = bid;
        return DBG_OK;
    }
    return upload_batch(h, st, bid);
}

// dbg_column (host or device) -> DCol on device
static int to_dcol(dbg_agg_handle* h, const dbg_column& c, const dbg_datatype& want, bool check_type, int on_device, DCol& d) {
    memset(&d, 0, sizeof(d));
    if (!valid_type(c.dt.type)) return fail(DBG_ERR_INVALID, "bad column type");
    if (check_type && (c.dt.type != want.type || (c.dt.type == DBG_DECIMAL128 && c.dt.scale != want.scale)))
        return fail(DBG_ERR_INVALID, "column type does not match the declared type");
    if (check_type && c.dt.nullable && !want.nullable) return fail(DBG_ERR_INVALID, "nullable column for a non-nullable declared type");
    d.type = c.dt.type;
    d.precision = c.dt.precision;
    d.scale = c.dt.scale;
    d.nullable = check_type ? want.nullable : c.dt.nullable;
    d.layout = LAYOUT_ARROW;
    d.width = type_width(c.dt.type);
    d.stride = d.width;
    u64 n = c.len;
    if (on_device) {
        d.data = (const u8*)c.data;
        d.offsets = c.offsets;
        d.validity = c.dt.nullable ? c.validity : nullptr;
        d.validity_offset = c.validity_offset;
        d.data_offset = c.data_offset;
        return DBG_OK;
    }
    // host: copy what the rows need
    const void* p = nullptr;
    if (c.dt.type == DBG_STRING) {
        u64 lo = n ? c.offsets[0] : 0, hi = n ? c.offsets[n] : 0;
        // copy offsets rebased to 0 and the payload slice
        std::vector<uint64_t> offs(n + 1);
        for (u64 i = 0; i <= n; ++i) offs[i] = c.offsets[i] - lo;
        RETURN_IF(own_copy(h, offs.data(), (n + 1) * 8, &p));
        d.offsets = (const u64*)p;
        // the staging vector dies here: make the copy synchronous w.r.t. it
        HIPCHECK(hipStreamSynchronize(h->stream));
        RETURN_IF(own_copy(h, (const u8*)c.data + lo, hi - lo, &p));
        d.data = (const u8*)p;
    } else if (c.dt.type == DBG_BOOLEAN) {
        u64 bytes = (c.data_offset + n + 7) / 8;
        RETURN_IF(own_copy(h, c.data, bytes, &p));
        d.data = (const u8*)p;
        d.data_offset = c.data_offset;
    } else {
        RETURN_IF(own_copy(h, c.data, n * d.width, &p));
        d.data = (const u8*)p;
    }
    if (c.dt.nullable && c.validity) {
        u64 bytes = (c.validity_offset + n + 7) / 8;
        RETURN_IF(own_copy(h, c.validity, bytes, &p));
        d.validity = (const u8*)p;
        d.validity_offset = c.validity_offset;
    }
    return DBG_OK;
}

static int fill_filter(dbg_agg_handle* h, const dbg_filter* f, int on_device, DCol* cols, int* ncols, DNode* nodes, int* nnodes) {
    if (f->n_cols > DBG_MAX_FCOLS || f->n_nodes > DBG_MAX_NODES) return fail(DBG_ERR_UNSUPPORTED, "filter too large");
    int depth = 0;
    for (int k = 0; k < f->n_nodes; ++k) {
        const dbg_pred_node& n = f->nodes[k];
        DNode& d = nodes[k];
        memset(&d, 0, sizeof(d));
        d.op = n.op;
        d.cmp = n.cmp;
        d.col = n.col;
        d.col2 = n.col2;
        d.i64v = n.i64;
        d.f64v = n.f64;
        d.lo = n.i128_lo;
        d.hi = n.i128_hi;
        if (n.op == DBG_PRED_CMP_CONST || n.op == DBG_PRED_CMP_COLS || n.op == DBG_PRED_IS_NULL || n.op == DBG_PRED_IS_NOT_NULL) {
            if (n.col < 0 || n.col >= f->n_cols || (n.op == DBG_PRED_CMP_COLS && (n.col2 < 0 || n.col2 >= f->n_cols)))
                return fail(DBG_ERR_INVALID, "predicate column index out of range");
            depth++;
        } else if (n.op == DBG_PRED_TRUE) {
            depth++;
        } else if (n.op == DBG_PRED_AND || n.op == DBG_PRED_OR) {
            if (depth < 2) return fail(DBG_ERR_INVALID, "malformed predicate program");
            depth--;
        } else if (n.op == DBG_PRED_NOT) {
            if (depth < 1) return fail(DBG_ERR_INVALID, "malformed predicate program");
        } else {
            return fail(DBG_ERR_INVALID, "unknown predicate op");
        }
        if (depth > 15) return fail(DBG_ERR_UNSUPPORTED, "predicate too deep");
        if (n.op == DBG_PRED_CMP_CONST && f->cols[n.col].dt.type == DBG_STRING) {
            const void* p = nullptr;
            RETURN_IF(own_copy(h, n.str, n.str_len, &p));
            d.str = (const u8*)p;
            d.str_len = n.str_len;
        }
    }
    if (f->n_nodes && depth != 1) return fail(DBG_ERR_INVALID, "malformed predicate program");
    for (int c = 0; c < f->n_cols; ++c) RETURN_IF(to_dcol(h, f->cols[c], f->cols[c].dt, false, on_device, cols[c]));
    *ncols = f->n_cols;
    *nnodes = f->n_nodes;
    return DBG_OK;
}

// ------------------------------------------------------------------------------------------
// C API
// ------------------------------------------------------------------------------------------
extern "C" {

const char* dbg_version(void) { return "dbgpu_agg 0.1 (gfx950)"; }
const char* dbg_last_error(void) { return g_last_error.c_str(); }

int dbg_device_count(int* n) {
    HIPCHECK(hipGetDeviceCount(n));
    return DBG_OK;
}

int dbg_agg_result_type(const dbg_agg_spec* spec, dbg_datatype* out) {
    if (!spec || !out) return fail(DBG_ERR_INVALID, "null argument");
    return result_type_of(*spec, out);
}

int dbg_agg_create(const dbg_agg_params* params, dbg_agg_handle** out) {
    if (!params || !out) return fail(DBG_ERR_INVALID, "null argument");
    auto* h = new dbg_agg_handle();
    int rc = build_spec(params, h->spec, h->result_types);
    if (rc != DBG_OK) {
        delete h;
        return rc;
    }
    for (int a = 0; a < params->n_aggs; ++a) h->src_kinds.push_back(params->aggs[a].kind);
    h->partial = params->partial != 0;
    if (params->device >= 0) h->device = params->device;
    else {
        hipError_t e = hipGetDevice(&h->device);
        if (e != hipSuccess) {
            delete h;
            return fail(DBG_ERR_DEVICE, std::string("hipGetDevice: ") + hipGetErrorString(e));
        }
    }
    auto cleanup = [&](int code) {
        dbg_agg_destroy(h);
        return code;
    };
    if (hipSetDevice(h->device) != hipSuccess) return cleanup(fail(DBG_ERR_DEVICE, "hipSetDevice failed"));
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) return cleanup(fail(DBG_ERR_DEVICE, "hipStreamCreate failed"));
    h->stream = h->own_stream;
    if ((rc = dev_alloc((void**)&h->counters, CNT_WORDS * 8)) != DBG_OK) return cleanup(rc);
    if (hipMemset(h->counters, 0, CNT_WORDS * 8) != hipSuccess) return cleanup(fail(DBG_ERR_DEVICE, "memset"));
    h->spec.err = h->counters + CNT_ERR;  // error bits raised from inside state updates
    {
        const char* cx = getenv("DBG_X_PPSPEC_CAP");
        const char* fd = getenv("DBG_X_PPSPEC_DESC");
        h->spec.x_pp_cap = cx ? std::max<u32>(64, (u32)atoi(cx) & ~3u) : ~0u;
        h->spec.x_pp_desc = (fd && fd[0] == '1') ? 1 : 0;
    }
    if ((rc = dev_alloc((void**)&h->dspec, sizeof(Spec))) != DBG_OK) return cleanup(rc);
    if (hipMemcpy(h->dspec, &h->spec, sizeof(Spec), hipMemcpyHostToDevice) != hipSuccess) return cleanup(fail(DBG_ERR_DEVICE, "spec upload"));
    if (hipHostMalloc((void**)&h->hcounters, (CNT_WORDS + DBG_MAX_KEYS + 8) * 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return cleanup(fail(DBG_ERR_OOM, "pinned"));
    if (hipHostGetDevicePointer((void**)&h->hcounters_dev, h->hcounters, 0) != hipSuccess) h->hcounters_dev = nullptr;
    // initial capacity: 2x the hint, or 1024 slots (the CPU table starts at 32768 =
    // AggregateHashTable::initial_capacity(); on the GPU growth is a cheap rehash kernel and a
    // small table keeps init / finalize scans short for low-cardinality queries: 4096 -> 1024
    // slots took C2's fused finalize from 13.3 to 11.4 us and C1's from 58 to 50 us)
    h->hint_groups = params->capacity_hint;
    u64 hint = params->capacity_hint ? params->capacity_hint : 512;
    h->cap = pow2_at_least(std::max<u64>(hint * 2, 1024));
    h->init_cap = h->cap;
    if ((rc = alloc_table(h, h->cap, &h->slots)) != DBG_OK) return cleanup(rc);
    // parking rows for every workgroup of an insert launch (launch_insert caps its grid here)
    h->scr_blocks = DBG_INSERT_MAX_BLOCKS;
    if ((rc = dev_alloc((void**)&h->scratch, scr_words(h->scr_blocks, (u32)h->spec.stride_words) * 8)) != DBG_OK) return cleanup(rc);
    if (hipMemset(h->scratch, 0, (size_t)h->scr_blocks * 16) != hipSuccess) return cleanup(fail(DBG_ERR_DEVICE, "memset"));

    // the (empty) batch table
    BatchDesc* st;
    u32 bid;
    if ((rc = new_batch(h, &st, &bid)) != DBG_OK) return cleanup(rc);
    h->n_batches = 0;  // slot 0 reserved: ref entries always carry bid >= 1
    if (hipStreamSynchronize(h->stream) != hipSuccess) return cleanup(fail(DBG_ERR_DEVICE, "sync"));
    *out = h;
    return DBG_OK;
}

void dbg_agg_destroy(dbg_agg_handle* h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    for (auto& b : h->owned) hipFree(b.p);
    for (auto& b : h->xrecv)
        if (b.p) hipFree(b.p);
    for (auto* p : h->pinned_chunks) hipHostFree(p);
    void* bufs[] = {h->scratch, h->slots, h->counters, h->ovf_rows, h->ovf_recs, h->dbatches, h->dspec, h->d_pos, h->d_str_pos,
                    h->d_part_pos, h->d_part_str_pos, h->d_part_str_base, h->d_lpart, h->vbytes, h->part_sorted, h->part_bounds,
                    h->part_temp, h->ser_err, h->dense, h->part_status};
    for (void* p : bufs)
        if (p) hipFree(p);
    for (auto& K : h->ppk) {
        void* kb[] = {K.l1, K.a, K.b, K.part, K.dig};
        for (void* q : kb)
            if (q) hipFree(q);
    }
    void* pb[] = {h->pp_cnt, h->pp_off, h->pp_scan_tmp, h->pp_mid, h->pp_dchunks, h->pp_dc0, h->pp_tot, h->pp_set, h->pp_grec, h->pp_blk,
                  h->pp_spill};
    for (void* q : pb)
        if (q) hipFree(q);
    void* ph[] = {h->pp_hchunks, h->pp_hc0, h->pp_hpart, h->pp_htot};
    for (void* q : ph)
        if (q) hipHostFree(q);
    if (h->hcounters) hipHostFree(h->hcounters);
    if (h->switch_ev) hipEventDestroy(h->switch_ev);
    if (h->own_stream) hipStreamDestroy(h->own_stream);
    delete h;
}

int dbg_agg_set_stream(dbg_agg_handle* h, void* s) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_deferred(h));
    hipStream_t ns = s ? (hipStream_t)s : h->own_stream;
    if (ns != h->stream) {
        // device-side hand-off: work queued on the new stream waits for everything queued on the
        // old one (no host synchronisation, so a caller can alternate streams per launch)
        if (!h->switch_ev) HIPCHECK(hipEventCreateWithFlags(&h->switch_ev, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(h->switch_ev, h->stream));
        HIPCHECK(hipStreamWaitEvent(ns, h->switch_ev, 0));
        h->stream = ns;
    }
    return DBG_OK;
}

int dbg_agg_reset(dbg_agg_handle* h) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    HIPCHECK(hipSetDevice(h->device));
    h->def_on = false;  // the held-back insert is discarded with the groups
    h->def_part = false;
    h->stage.clear();   // and so are staged host rows
    // inputs copied by earlier batches, and the pinned batch descriptors reused below, may still
    // be read by queued work: wait if any were queued since the last synchronisation
    if (!h->owned.empty() || h->uploads_pending) {
        HIPCHECK(hipStreamSynchronize(h->stream));
        for (auto& b : h->owned) HIPCHECK(hipFree(b.p));
        h->owned.clear();
        h->uploads_pending = false;
    }
    h->n_batches = h->n_cached;  // cached descriptors stay valid (immutable)
    h->pending_rows = h->pending_recs = 0;
    h->finalized = false;
    h->table_rows = 0;
    h->remerged = 0;
    h->xrecv_busy = false;  // no group references the exchange's receive buffers any more
    h->xchunks.clear();  // an abandoned chunked shuffle (the last call never came): its buffers are the communicator's
    h->xfirst[0] = h->xfirst[1] = 0;
    for (auto& K : h->ppk) {  // partitioned payload: records dropped, buffers kept (the mode too)
        K.l1_n = 0;
        K.dig_n = 0;
        K.segs.clear();
    }
    h->pp_grec_ready = false;
    if (h->clean) return DBG_OK;  // the recycling finalize already re-initialised table + counters
    // the counters and the sentinel slot now; the slots when a kernel first touches the table
    // (table_desc), or never if a partitioned insert rewrites every slice first
    prof::Scope ps("table_init", h->stream);
    launch_table_init(h->stream, h->dspec, h->spec, h->slots + h->cap * (u64)h->spec.tstride, 0, h->counters);
    h->init_pending = true;
    h->clean = true;
    return DBG_OK;
}

static int ensure_buf(u64** p, u64* cap, u64 n);

// Radix-partitioned COUNT(*) insert of a high-cardinality batch (part.hip); buffers grow only.
static int part_insert(dbg_agg_handle* h, const BatchDesc* st, u32 bid, u64 rows, u32 sb, bool on_device_insert, bool was_clean) {
    (void)bid;
    const int width = (int)st->keys[0].width;
    size_t tb = part_temp_bytes(width, rows, sb, h->cap);
    if (!tb) return fail(DBG_ERR_INTERNAL, "rocprim radix_sort_keys sizing failed");
    if (tb > h->part_temp_cap) {
        if (h->part_temp) HIPCHECK(hipFree(h->part_temp));
        h->part_temp = nullptr;
        h->part_temp_cap = 0;
        RETURN_IF(dev_alloc(&h->part_temp, tb));
        h->part_temp_cap = tb;
    }
    RETURN_IF(ensure_buf(&h->part_sorted, &h->part_sorted_cap, rows));
    RETURN_IF(ensure_buf(&h->part_bounds, &h->part_bounds_cap, (h->cap >> sb) + 1));
    prof::Scope ps("agg_insert", h->stream);
    const char* step = "";
    // an empty table whose initialisation is still deferred: the slice kernel writes every slot
    const bool empty = h->init_pending;
    h->init_pending = false;
    hipError_t e = launch_part_sort(h->stream, *st, rows, h->cap, sb, h->part_temp, h->part_temp_cap, h->part_sorted, h->part_bounds,
                                    &step);
    // EXPERIMENT (EXP=1 build): DBG_X_PART_DIRECT=0 keeps the table stage in the insert
    static const bool direct_on = !(X_ENV("DBG_X_PART_DIRECT") && X_ENV("DBG_X_PART_DIRECT")[0] == '0');
    // (was_clean: no group since the last reset or recycling finalize, the slots EMPTY or their
    // initialisation pending — the slices may start from EMPTY either way)
    if (e == hipSuccess && (empty || was_clean) && h->recycle && on_device_insert && direct_on) {  // the table stage waits for the next call
        h->def_part = true;
        h->def_part_sb = sb;
        h->def_part_kw = width;
        return DBG_OK;
    }
    if (e == hipSuccess) e = launch_part_slices(h->stream, table_desc(h), sb, h->part_sorted, h->part_bounds, empty, &step);
    if (e != hipSuccess) return fail(DBG_ERR_DEVICE, std::string("partitioned insert (") + step + "): " + hipGetErrorString(e));
    return DBG_OK;
}

// The held-back table stage of a partitioned insert into an empty table: the regular slices.
static int part_flush(dbg_agg_handle* h) {
    if (!h->def_part) return DBG_OK;
    h->def_part = false;
    h->init_pending = false;  // part_slice<EMPTY> writes every slot
    prof::Scope ps("part_slice", h->stream);
    const char* step = "";
    hipError_t e = launch_part_slices(h->stream, table_desc(h), h->def_part_sb, h->part_sorted, h->part_bounds, true, &step);
    if (e != hipSuccess) return fail(DBG_ERR_DEVICE, std::string("partitioned insert (") + step + "): " + hipGetErrorString(e));
    return DBG_OK;
}

// ------------------------------------------------------------------------------------------
// partitioned payload (pp.hip), host side
// ------------------------------------------------------------------------------------------
}  // extern "C" (templates need C++ linkage)
template <typename T>
static int ensure_dev(T** p, u64* cap, u64 n) {
    if (n <= *cap && *p) return DBG_OK;
    if (*p) HIPCHECK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    const u64 c = std::max<u64>(n, 64);
    RETURN_IF(dev_alloc((void**)p, c * sizeof(T)));
    *cap = c;
    return DBG_OK;
}
template <typename T>
static int ensure_pinned(dbg_agg_handle* h, T** p, u64* cap, u64 n) {
    if (n <= *cap && *p) return DBG_OK;
    if (*p) {
        HIPCHECK(hipStreamSynchronize(h->stream));  // a queued copy may still read it
        HIPCHECK(hipHostFree(*p));
    }
    *p = nullptr;
    *cap = 0;
    const u64 c = std::max<u64>(n, 1024);
    HIPCHECK(hipHostMalloc((void**)p, c * sizeof(T), hipHostMallocDefault));
    *cap = c;
    return DBG_OK;
}

extern "C" {

#define PP_MIN_ROWS (1ULL << 22)
#define PP_MIN_GROUPS (1ULL << 20)
#define PP_SET_CAP (1ULL << 19)  // 2^18 samples at most: <= 50 % load

static void note_observed(dbg_agg_handle* h) {
    // compaction's re-merged group records are not input rows: leave them out of the ratio
    const u64 rows = h->table_rows > h->remerged ? h->table_rows - h->remerged : 0;
    if (h->pp || !rows) return;
    h->obs_rows = rows;
    h->obs_groups = h->n_groups;
}

// Cardinality probe of the first batch into an empty handle (AggregateHashTable decides its
// partial strategy by observed cardinality too: clear_ht / maybe_repartition,
// EAGG/aggregate_hashtable.rs:225-239, 453-503).  Distinct group hashes among 2^20 evenly spaced
// selected rows give the estimate: the larger of twice the uniform-frequency solution of
// D = G (1 - exp(-s / G)) and Haas's GEE sqrt(N / s) f1 + (D - f1), capped at the selected rows.
static int pp_maybe_switch(dbg_agg_handle* h, u32 bid, u64 rows) {
    const Spec& S = h->spec;
    h->est_groups = 0;  // set below only from this batch's probe or observation
    const int mode = h->strategy == DBG_STRATEGY_TABLE ? 0 : (h->strategy == DBG_STRATEGY_PARTITIONED ? 2 : 1);
    if (h->pp || !mode || !S.pp_ok || h->table_rows) return DBG_OK;
    if (mode == 1 && (rows < PP_MIN_ROWS || (!S.has_strings && S.inline_width <= 2))) return DBG_OK;
    if (mode == 1 && h->obs_rows >= PP_MIN_ROWS) {
        // the handle's last finalize saw this query's cardinality (groups per inserted row)
        const double ratio = std::min(1.0, (double)h->obs_groups / (double)h->obs_rows);
        h->pp_ratio = std::max(ratio, 1e-9);
        h->pp_probed = true;
        h->est_groups = ratio * (double)rows;
        if (ratio * (double)rows > (double)PP_MIN_GROUPS && ratio > 0.5) h->pp = true;
        return DBG_OK;
    }
    if (!h->pp_set) RETURN_IF(dev_alloc((void**)&h->pp_set, PP_SET_CAP * 16 + 64));
    u64* out = h->pp_set + 2 * PP_SET_CAP;
    // 1/64 of the rows, between 2^16 and 2^18 samples; the set sized for them (<= 50 % load)
    const u64 ns = std::min<u64>(rows, std::max<u64>(1ULL << 16, std::min<u64>(rows / 64, 1ULL << 18)));
    const u64 set_cap = std::min<u64>(PP_SET_CAP, pow2_at_least(2 * ns));
    {
        prof::Scope ps("pp_probe", h->stream);
        launch_pp_sample(h->stream, h->dspec, h->dbatches, bid, rows, ns, h->pp_set, set_cap, out);
    }
    HIPCHECK(hipGetLastError());
    RETURN_IF(ensure_pinned(h, &h->pp_hpart, &h->pp_hpart_cap, 1024));
    HIPCHECK(hipMemcpyAsync(h->pp_hpart, out, 32, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    const double sel = (double)h->pp_hpart[0], D = (double)h->pp_hpart[1], f1 = (double)h->pp_hpart[2];
    if (sel <= 0) return DBG_OK;
    const double nsel = (double)rows * sel / (double)ns;
    double gu = nsel;
    if (D < sel - 0.5) {  // bisection on G >= D of G (1 - exp(-sel / G)) = D (increasing in G)
        double lo = D, hi = 1e15;
        for (int it = 0; it < 200; ++it) {
            const double mid = 0.5 * (lo + hi);
            if (mid * -std::expm1(-sel / mid) < D) lo = mid;
            else hi = mid;
        }
        gu = lo;
    }
    const double gee = std::sqrt(nsel / sel) * f1 + (D - f1);
    const double g = std::min(nsel, std::max(1.25 * gu, gee));
    h->pp_ratio = std::min(1.0, std::max(g / nsel, 1e-9));
    h->pp_probed = true;
    h->est_groups = g;
    // the partitioned payload beats the HBM table when keys are mostly unique (ClickBench Q33:
    // 1e9 groups in 1e9 rows); moderate cardinality stays on the table
    if (mode == 2 || (g > (double)PP_MIN_GROUPS && h->pp_ratio > 0.5)) h->pp = true;
    return DBG_OK;
}

// The pinned chunk staging is rewritten only after the stream has drained its last upload.
static int pp_upload_chunks(dbg_agg_handle* h, const std::vector<PPChunk>& ch, const std::vector<u32>& c0) {
    HIPCHECK(hipStreamSynchronize(h->stream));
    RETURN_IF(ensure_pinned(h, &h->pp_hchunks, &h->pp_hchunks_cap, ch.size()));
    RETURN_IF(ensure_pinned(h, &h->pp_hc0, &h->pp_hc0_cap, c0.size()));
    RETURN_IF(ensure_dev(&h->pp_dchunks, &h->pp_dchunks_cap, ch.size()));
    RETURN_IF(ensure_dev(&h->pp_dc0, &h->pp_dc0_cap, c0.size()));
    memcpy(h->pp_hchunks, ch.data(), ch.size() * sizeof(PPChunk));
    memcpy(h->pp_hc0, c0.data(), c0.size() * sizeof(u32));
    HIPCHECK(hipMemcpyAsync(h->pp_dchunks, h->pp_hchunks, ch.size() * sizeof(PPChunk), hipMemcpyHostToDevice, h->stream));
    HIPCHECK(hipMemcpyAsync(h->pp_dc0, h->pp_hc0, c0.size() * sizeof(u32), hipMemcpyHostToDevice, h->stream));
    return DBG_OK;
}

// count + scan of one level: part_out receives G * K + 1 partition offsets
static const char* const PP_COUNT_NAME[4] = {"", "pp_count_l1", "pp_count_l2", "pp_count_l3"};
static const char* const PP_SCAN_NAME[4] = {"", "pp_scan_l1", "pp_scan_l2", "pp_scan_l3"};
static const char* const PP_SCATTER_NAME[4] = {"", "pp_scatter_l1", "pp_scatter_l2", "pp_scatter_l3"};

// The specialised level-1 form of a raw batch (pp.hip pp_l1_*), or kind 0 for the generic kernels.
static PPFast pp_fast_desc(const Spec& S, const BatchDesc& B, u32 bid, int kind) {
    PPFast F;
    memset(&F, 0, sizeof(F));
    if (kind != 0 || B.is_records || B.n_nodes > 1) return F;
    const DNode* nd = B.n_nodes ? &B.nodes[0] : nullptr;
    if (nd && nd->op != DBG_PRED_CMP_CONST) return F;
    const DCol* pc = nd ? &B.fcols[nd->col] : nullptr;
    if (pc && (pc->nullable || pc->layout != LAYOUT_ARROW)) return F;
    auto fixed_ok = [](int t) { return t != DBG_STRING && t != DBG_DECIMAL128 && t != DBG_BOOLEAN && type_width(t) > 0; };
    if (!S.has_strings) {
        if (S.pp_rw_raw > 64) return F;
        u32 n = 0;
        for (int c = 0; c < S.n_keys; ++c) {
            const dbg_datatype& t = S.key_types[c];
            const DCol& d = B.keys[c];
            if (t.nullable || !fixed_ok(t.type) || d.layout != LAYOUT_ARROW) return F;
            F.ptr[n] = d.data;
            F.width[n] = (u8)type_width(t.type);
            F.type[n] = (u8)t.type;
            F.off[n] = S.koff[c];
            ++n;
        }
        F.nk = n;
        for (int a = 0; a < S.n_aggs; ++a) {
            const DAgg& A = S.aggs[a];
            if (A.arg_type < 0) continue;
            const DCol& d = B.args[a];
            if (A.arg_nullable || !fixed_ok(A.arg_type) || d.layout != LAYOUT_ARROW || n >= 8) return F;
            F.ptr[n] = d.data;
            F.width[n] = (u8)type_width(A.arg_type);
            F.type[n] = (u8)A.arg_type;
            F.off[n] = S.pp_aoff[a];
            ++n;
        }
        F.ncol = n;
        if (pc) {
            const int t = pc->type;
            if (!fixed_ok(t) || t == DBG_FLOAT32 || t == DBG_FLOAT64) return F;
            F.has_pred = 1;
            F.pcmp = nd->cmp;
            F.ptype = t;
            F.pwidth = type_width(t);
            F.pptr = pc->data;
            F.pconst = nd->i64v;
        }
        F.wpr = S.pp_rw_raw / 8;
        F.kind = 1;
        return F;
    }
    if (S.n_keys != 1 || S.key_types[0].type != DBG_STRING || S.key_types[0].nullable || S.pp_rw_raw != 48) return F;
    for (int a = 0; a < S.n_aggs; ++a)
        if (S.aggs[a].arg_type >= 0) return F;
    const DCol& k = B.keys[0];
    if (k.layout != LAYOUT_ARROW) return F;
    if (pc) {
        if (pc->type != DBG_STRING || pc->data != k.data || pc->offsets != k.offsets) return F;
        F.has_pred = 1;
        F.pcmp = nd->cmp;
        F.pstr = nd->str;
        F.pstr_len = nd->str_len;
    }
    F.soffs = k.offsets;
    F.sdata = k.data;
    F.bid = bid;
    F.wpr = 6;
    F.kind = 2;
    return F;
}

// a result that is never NULL for a group: the aggregate's argument is never NULL (COUNT(*) or a
// non-nullable column), and SUM / AVG / MIN / MAX of one or more values is a value
static bool agg_always_valid(const DAgg& A) {
    return A.arg_type < 0 || !A.arg_nullable;
}

static int pp_count_scan(dbg_agg_handle* h, int level, int src, int kind, const u8* recs, const std::vector<PPChunk>& ch,
                         const std::vector<u32>& c0, u32 shift, u32 kbits, u64* part_out, const PPFast* F = nullptr,
                         bool counted = false, const u16* dig = nullptr) {
    const u64 K = 1ULL << kbits;
    RETURN_IF(pp_upload_chunks(h, ch, c0));
    if (counted && h->pp_cnt_cap < ch.size() * K) return fail(DBG_ERR_INTERNAL, "fused counts: buffer too small");
    RETURN_IF(ensure_dev(&h->pp_cnt, &h->pp_cnt_cap, ch.size() * K));
    RETURN_IF(ensure_dev(&h->pp_off, &h->pp_off_cap, ch.size() * K));
    if (!counted) {
        prof::Scope ps(PP_COUNT_NAME[level], h->stream);
        if (F && F->kind)
            launch_pp_l1_fast(h->stream, *F, 1, h->pp_dchunks, (u32)ch.size(), h->pp_cnt, nullptr, nullptr, nullptr);
        else if (dig)
            launch_pp_count_dig(h->stream, h->pp_dchunks, (u32)ch.size(), dig, kbits, h->pp_cnt);
        else
            launch_pp_count(h->stream, h->dspec, h->dbatches, src, kind, recs, h->pp_dchunks, (u32)ch.size(), shift, kbits, h->pp_cnt,
                            (kind ? h->spec.pp_rw_state : h->spec.pp_rw_raw) / 8);
    }
    RETURN_IF(ensure_dev(&h->pp_scan_tmp, &h->pp_scan_tmp_cap, pp_scan_scratch_words((u32)(c0.size() - 1), kbits)));
    {
        prof::Scope ps(PP_SCAN_NAME[level], h->stream);
        launch_pp_scan(h->stream, h->pp_cnt, (u32)ch.size(), kbits, h->pp_dc0, (u32)(c0.size() - 1), h->pp_off, part_out,
                       h->pp_scan_tmp);
    }
    h->pp_last_part = part_out;
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

static int pp_scatter(dbg_agg_handle* h, int level, int src, int kind, const u8* recs, u32 n_chunks, u32 shift, u32 kbits,
                      u8* dst, const PPFast* F = nullptr, u32* cnt_next = nullptr, u32 sh_next = 0, u32 kb_next = 0) {
    prof::Scope ps(PP_SCATTER_NAME[level], h->stream);
    if (F && F->kind) {
        launch_pp_l1_fast(h->stream, *F, 0, h->pp_dchunks, n_chunks, nullptr, h->pp_off, h->pp_last_part, dst);
        HIPCHECK(hipGetLastError());
        return DBG_OK;
    }
    launch_pp_scatter(h->stream, h->dspec, h->spec, h->dbatches, src, kind, recs, h->pp_dchunks, n_chunks, shift, kbits, h->pp_off,
                      h->pp_last_part, dst, cnt_next, sh_next, kb_next);
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

// Level 1 (TransformPartialAggregate::transform in partitioned mode): the batch's selected rows
// become records appended to the payload, grouped into 256 partitions (PartitionedPayload::
// append_rows, EAGG/partitioned_payload.rs:100-143).
// EXPERIMENT (DBG_X_PPDIG=0): level 2 counts from the records instead of the digit array
static bool kX_no_dig() {
    static const bool off = X_ENV("DBG_X_PPDIG") && X_ENV("DBG_X_PPDIG")[0] == '0';
    return off;
}

static int pp_add_batch(dbg_agg_handle* h, const BatchDesc* st, u32 bid, u64 rows, int kind) {
    const Spec& S = h->spec;
    auto& K = h->ppk[kind];
    PPFast F = pp_fast_desc(S, *st, bid, kind);
    F.dig = nullptr;
    const u32 rw = kind ? S.pp_rw_state : S.pp_rw_raw;
    std::vector<PPChunk> ch;
    for (u64 s = 0; s < rows; s += PP_CHUNK) ch.push_back(PPChunk{s, std::min<u64>(PP_CHUNK, rows - s), bid, 0});
    std::vector<u32> c0{0, (u32)ch.size()};
    RETURN_IF(ensure_dev(&h->pp_mid, &h->pp_mid_cap, 257));
    RETURN_IF(pp_count_scan(h, 1, 0, kind, nullptr, ch, c0, 64 - PP_L1_BITS, PP_L1_BITS, h->pp_mid, &F));
    RETURN_IF(ensure_pinned(h, &h->pp_hpart, &h->pp_hpart_cap, 1024));
    HIPCHECK(hipMemcpyAsync(h->pp_hpart, h->pp_mid, 257 * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    const u64 total = h->pp_hpart[256];
    if (!total) return DBG_OK;
    if (K.l1_n + total > K.l1_cap) {  // grow (x2), keeping the records already appended
        const u64 ncap = std::max<u64>(K.l1_n + total, K.l1_n ? 2 * K.l1_cap : 0);
        u8* nb = nullptr;
        RETURN_IF(dev_alloc((void**)&nb, ncap * rw + 64));  // slack: the aggregation reads whole words
        if (K.l1) {
            if (K.l1_n) HIPCHECK(hipMemcpyAsync(nb, K.l1, K.l1_n * rw, hipMemcpyDeviceToDevice, h->stream));
            HIPCHECK(hipStreamSynchronize(h->stream));
            HIPCHECK(hipFree(K.l1));
        }
        K.l1 = nb;
        K.l1_cap = ncap;
    }
    // the level-2 digits ride along while every record so far has them (fixed-shape raw batches)
    // (EXPERIMENT, DBG_X_PPDIG=0: no digits at all)
    const bool with_dig = F.kind == 1 && kind == 0 && K.dig_n == K.l1_n && !kX_no_dig();
    if (with_dig && K.l1_n + total > K.dig_cap) {
        const u64 ncap = std::max<u64>(K.l1_n + total, K.dig_n ? 2 * K.dig_cap : 0);
        u16* nd = nullptr;
        RETURN_IF(dev_alloc((void**)&nd, ncap * 2 + 64));
        if (K.dig) {
            if (K.dig_n) HIPCHECK(hipMemcpyAsync(nd, K.dig, K.dig_n * 2, hipMemcpyDeviceToDevice, h->stream));
            HIPCHECK(hipStreamSynchronize(h->stream));
            HIPCHECK(hipFree(K.dig));
        }
        K.dig = nd;
        K.dig_cap = ncap;
    }
    if (with_dig) F.dig = K.dig + K.l1_n;
    RETURN_IF(pp_scatter(h, 1, 0, kind, nullptr, (u32)ch.size(), 64 - PP_L1_BITS, PP_L1_BITS, K.l1 + K.l1_n * rw, &F));
    if (with_dig) K.dig_n = K.l1_n + total;
    K.segs.push_back(dbg_agg_handle::Seg{K.l1_n, total, std::vector<u64>(h->pp_hpart, h->pp_hpart + 257)});
    K.l1_n += total;
    h->pp_grec_ready = false;
    return DBG_OK;
}

// the specialised aggregation's table load per LDS round (linear probing in a 96-slot window;
// records whose window is full wait for a further mini-round).  0.7 halves C4's rounds (4 -> 2)
// but the longer probes cost more: pp_agg 32 -> 45 ms
#ifndef PS_LOAD
#define PS_LOAD 0.45
#endif


// Levels 2 and 3 (NewTransformPartitionBucket + the final bucket split): every level-1 partition
// of both record kinds is re-scattered by the next hash bits until the estimated groups of a
// final partition fit half a workgroup's LDS table.
static int pp_prepare(dbg_agg_handle* h, bool spec_ok) {
    const Spec& S = h->spec;
    const u64 nr = h->ppk[0].l1_n, nsr = h->ppk[1].l1_n;
    // estimated groups: the probe's, raised to the capacity hint (a hint below what the probe saw
    // would leave too few partition bits: many LDS overflow rounds); without a probe the hint, else
    // every record its own group
    const double probed = h->pp_ratio * (double)nr + (double)nsr;
    const double est = h->pp_probed ? std::max((double)h->hint_groups, probed)
                                    : (h->hint_groups ? (double)h->hint_groups : probed);
    const double g = std::min((double)(nr + nsr), est);
    // 45 % load: a wave's probe runs as long as its longest lane's (64 lanes in lockstep)
    const double target = std::max(64.0, 0.45 * (double)pp_agg_slots(S));
    const double need = std::max(1.0, std::ceil(g / target));
    u32 B = PP_L1_BITS + 1;
    while ((double)(1ULL << B) < need && B < PP_L1_BITS + 16) ++B;
    // level 2 takes up to 10 bits (one pass instead of a 1-2 bit third level), level 3 the rest
    u32 k2 = std::min<u32>(B - PP_L1_BITS <= 10 ? 10 : 8, B - PP_L1_BITS), k3 = B - PP_L1_BITS - k2;
    // Record-centric aggregation (raw records only): one workgroup per level-2 partition (sized
    // here for ~PP_RC_PART records on average), aggregated in 2^sub rounds of at most ~0.7 of one
    // LDS round's records — no level 3.
    h->pp_rc_sub = 0;
    // measured slower than the slot-table kernel on C4 (pp_agg 74 vs 58 ms): opt-in (DBG_X_PPRC=1)
    static const bool rc_on = X_ENV("DBG_X_PPRC") && X_ENV("DBG_X_PPRC")[0] == '1';
    if (rc_on && pp_rc_ok(S) && nsr == 0 && nr > 0) {
        const double per_part = (double)PP_RC_PART;
        u32 b2 = PP_L1_BITS + 1;
        while ((double)nr / (double)(1ULL << b2) > per_part && b2 < PP_L1_BITS + 10) ++b2;
        const double avg = (double)nr / (double)(1ULL << b2);
        const double round_cap = 0.7 * (double)pp_rc_records(S);
        u32 sub = 0;
        while (avg / (double)(1u << sub) > round_cap && sub < 5) ++sub;
        // (a capacity hint asking for fewer partitions than this sizing — e.g. one group — keeps
        // the slot-table kernel and its LDS overflow rounds)
        if (avg <= per_part && avg / (double)(1u << sub) <= round_cap && B >= b2) {
            B = b2;
            k2 = B - PP_L1_BITS;
            k3 = 0;
            h->pp_rc_sub = std::max<u32>(sub, 1);  // >= 1 round bit: the flag doubles as "record-centric"
        }
    }
    // Compile-time specialised aggregation (result columns, raw records of a supported shape): a
    // partition is loaded once and aggregated in 2^sub LDS rounds, so partitions hold up to the
    // kernel's register budget of records and level 2 alone (<= 10 bits) sizes them — no level 3.
    h->pp_spec = -1;
    static const bool spec_on = !(X_ENV("DBG_X_PPSPEC") && X_ENV("DBG_X_PPSPEC")[0] == '0');
    u32 scap = 0, smax = 0;
    const int shape = (spec_on && spec_ok && !h->pp_rc_sub && nsr == 0 && nr > 0) ? pp_spec_shape(S, &scap, &smax) : -1;
    if (shape >= 0) {
        const double fill = 0.75 * (double)smax;  // average records per partition (the max stays below smax)
        u32 b2 = PP_L1_BITS + 1;
        while ((double)nr / (double)(1ULL << b2) > fill && b2 < PP_L1_BITS + 10) ++b2;
        const double gp = g / (double)(1ULL << b2);
        u32 sub = 0;
        while (gp / (double)(1u << sub) > PS_LOAD * (double)scap && sub < 5) ++sub;
        if ((double)nr / (double)(1ULL << b2) <= fill && gp / (double)(1u << sub) <= PS_LOAD * (double)scap && B >= b2) {
            B = b2;
            k2 = B - PP_L1_BITS;
            k3 = 0;
            h->pp_spec = shape;
            h->pp_spec_sub = sub;
        }
    }
    h->pp_bits = B;
    for (int kind = 0; kind < 2; ++kind) {
        auto& K = h->ppk[kind];
        if (!K.l1_n) continue;
        const u32 rw = kind ? S.pp_rw_state : S.pp_rw_raw;
        if (K.ab_cap < K.l1_n) {
            if (K.a) HIPCHECK(hipFree(K.a));
            if (K.b) HIPCHECK(hipFree(K.b));
            K.a = K.b = nullptr;
            K.ab_cap = 0;
            RETURN_IF(dev_alloc((void**)&K.a, K.l1_n * rw + 64));
            RETURN_IF(dev_alloc((void**)&K.b, K.l1_n * rw + 64));
            K.ab_cap = K.l1_n;
        }
        RETURN_IF(ensure_dev(&K.part, &K.part_cap, (1ULL << B) + 1));
        // level 2: units never straddle a level-1 partition (group = partition index)
        std::vector<PPChunk> ch;
        std::vector<u32> c0;
        for (u32 g1 = 0; g1 < (1u << PP_L1_BITS); ++g1) {
            c0.push_back((u32)ch.size());
            for (const auto& sg : K.segs) {
                const u64 lo = sg.base + sg.off[g1], hi = sg.base + sg.off[g1 + 1];
                for (u64 x = lo; x < hi; x += PP_CHUNK) ch.push_back(PPChunk{x, std::min<u64>(PP_CHUNK, hi - x), 0, g1});
            }
            if (c0.back() == ch.size()) ch.push_back(PPChunk{0, 0, 0, g1});
        }
        c0.push_back((u32)ch.size());
        const u32 sh2 = 64 - PP_L1_BITS - k2;
        u64* p2 = k3 ? nullptr : K.part;
        if (k3) {
            RETURN_IF(ensure_dev(&h->pp_mid, &h->pp_mid_cap, (256ULL << k2) + 1));
            p2 = h->pp_mid;
        }
        // the level-2 count reads the digit array (2 bytes per record) when level 1 wrote one
        const bool use_dig = K.dig && K.dig_n == K.l1_n && k2 <= 16 && !kX_no_dig();
        RETURN_IF(pp_count_scan(h, 2, 1, kind, K.l1, ch, c0, sh2, k2, p2, nullptr, false, use_dig ? K.dig : nullptr));
        const u64 G2 = 256ULL << k2;
        const u32 sh3 = sh2 - k3;
        // Level 3's counts ride on the level-2 scatter when every level-2 partition is one level-3
        // unit (<= PP_CHUNK records): one fewer pass over the records.
        bool fused3 = false;
        if (k3) {
            RETURN_IF(ensure_pinned(h, &h->pp_hpart, &h->pp_hpart_cap, G2 + 1));
            HIPCHECK(hipMemcpyAsync(h->pp_hpart, p2, (G2 + 1) * 8, hipMemcpyDeviceToHost, h->stream));
            HIPCHECK(hipStreamSynchronize(h->stream));
            u64 mx = 0;
            for (u64 g2 = 0; g2 < G2; ++g2) mx = std::max<u64>(mx, h->pp_hpart[g2 + 1] - h->pp_hpart[g2]);
            fused3 = mx <= PP_CHUNK && ((1u << k2) << k3) <= PP_NEXT_HIST_MAX;
            if (fused3) {
                RETURN_IF(ensure_dev(&h->pp_cnt, &h->pp_cnt_cap, G2 << k3));
                HIPCHECK(hipMemsetAsync(h->pp_cnt, 0, (G2 << k3) * 4, h->stream));
            }
        }
        RETURN_IF(pp_scatter(h, 2, 1, kind, K.l1, (u32)ch.size(), sh2, k2, K.a, nullptr, fused3 ? h->pp_cnt : nullptr, sh3, k3));
        K.fin = K.a;
        K.alt = K.b;
        if (!k3) continue;
        // level 3: units inside level-2 partitions
        ch.clear();
        c0.clear();
        for (u64 g2 = 0; g2 < G2; ++g2) {
            c0.push_back((u32)ch.size());
            const u64 lo = h->pp_hpart[g2], hi = h->pp_hpart[g2 + 1];
            for (u64 x = lo; x < hi; x += PP_CHUNK) ch.push_back(PPChunk{x, std::min<u64>(PP_CHUNK, hi - x), 0, (u32)g2});
            if (c0.back() == ch.size()) ch.push_back(PPChunk{0, 0, 0, (u32)g2});
        }
        c0.push_back((u32)ch.size());
        if (fused3 && ch.size() != G2) return fail(DBG_ERR_INTERNAL, "fused level-3 counts: unit layout");
        RETURN_IF(pp_count_scan(h, 3, 1, kind, K.a, ch, c0, sh3, k3, K.part, nullptr, fused3));
        RETURN_IF(pp_scatter(h, 3, 1, kind, K.a, (u32)ch.size(), sh3, k3, K.b));
        K.fin = K.b;
        K.alt = K.a;
    }
    return DBG_OK;
}

static u64 pp_records(const dbg_agg_handle* h) { return h->ppk[0].l1_n + h->ppk[1].l1_n; }

// The LDS aggregation of every final partition: mode 0 writes the result columns of `od` (fixed-width
// keys), mode 1 the group records (state record format) into pp_grec.  Totals land in pp_tot.
static int pp_agg(dbg_agg_handle* h, int mode, const OutDesc* od) {
    const Spec& S = h->spec;
    if (!h->pp_tot) RETURN_IF(dev_alloc((void**)&h->pp_tot, PPT_WORDS * 8));
    HIPCHECK(hipMemsetAsync(h->pp_tot, 0, PPT_WORDS * 8, h->stream));
    const u64 N = pp_records(h);
    if (!N) return DBG_OK;
    RETURN_IF(pp_prepare(h, mode == 1 || (od && !od->ser)));
    PPAggOut o;
    memset(&o, 0, sizeof(o));
    o.tot = h->pp_tot;
    static u64* x_pptrace = nullptr;  // EXPERIMENT (DBG_X_PPTRACE)
    if (kPhaseTrace && X_ENV("DBG_X_PPTRACE")) {
        if (!x_pptrace) {
            RETURN_IF(dev_alloc((void**)&x_pptrace, 64));
            HIPCHECK(hipMemset(x_pptrace, 0, 64));
            atexit([] {
                u64 v[8];
                hipDeviceSynchronize();
                hipMemcpy(v, x_pptrace, 64, hipMemcpyDeviceToHost);
                const double n = v[5] ? (double)v[5] : 1.0;
                fprintf(stderr, "pptrace raw us/partition [0..4] %.2f %.2f %.2f %.2f %.2f (spec kernel: load+hash, stage, insert, "
                                "emit, barriers)\n", v[0] * 0.01 / n, v[1] * 0.01 / n, v[2] * 0.01 / n, v[3] * 0.01 / n, v[4] * 0.01 / n);
                fprintf(stderr, "pptrace partitions %llu groups/partition %.0f  per partition us: insert %.2f sync %.2f "
                                "atomic %.2f write %.2f tail %.2f\n", (unsigned long long)v[5], v[6] / n, v[0] * 0.01 / n,
                        v[1] * 0.01 / n, v[2] * 0.01 / n, v[3] * 0.01 / n, v[4] * 0.01 / n);
            });
        }
        o.trace = x_pptrace;
    }
    if (mode == 0) {
        o.cols = *od;
    } else {
        RETURN_IF(ensure_dev(&h->pp_grec, &h->pp_grec_cap, N * S.pp_rw_state));
        o.grec = h->pp_grec;
        o.grec_cap = N;
    }
    auto& R = h->ppk[0];
    auto& T = h->ppk[1];
    if (h->pp_spec >= 0) {
        // every final partition may spill (skewed keys): room for all their ids (<= 1 MB)
        const u32 SPILL_CAP = 1u << h->pp_bits;
        if (h->pp_spill_cap < SPILL_CAP) {
            if (h->pp_spill) HIPCHECK(hipFree(h->pp_spill));
            h->pp_spill = nullptr;
            h->pp_spill_cap = 0;
            RETURN_IF(dev_alloc((void**)&h->pp_spill, (1 + (size_t)SPILL_CAP) * 4));
            h->pp_spill_cap = SPILL_CAP;
        }
        HIPCHECK(hipMemsetAsync(h->pp_spill, 0, 4, h->stream));
        prof::Scope ps("pp_agg", h->stream);
        launch_pp_agg_spec(h->stream, S, h->pp_spec, mode, 1u << h->pp_bits, R.part, R.fin, h->pp_spec_sub, o, h->pp_spill, SPILL_CAP);
        // partitions larger than its register budget (skewed keys): the generic kernel, spilled ids only
        launch_pp_agg(h->stream, h->dspec, S, h->dbatches, mode, 1u << h->pp_bits, R.part, nullptr, R.fin, R.alt, nullptr, nullptr,
                      o, h->pp_spill, SPILL_CAP);
    } else if (h->pp_rc_sub) {
        // every final partition may spill (skewed keys): room for all their ids (<= 1 MB)
        const u32 SPILL_CAP = 1u << h->pp_bits;
        if (h->pp_spill_cap < SPILL_CAP) {
            if (h->pp_spill) HIPCHECK(hipFree(h->pp_spill));
            h->pp_spill = nullptr;
            h->pp_spill_cap = 0;
            RETURN_IF(dev_alloc((void**)&h->pp_spill, (1 + (size_t)SPILL_CAP) * 4));
            h->pp_spill_cap = SPILL_CAP;
        }
        HIPCHECK(hipMemsetAsync(h->pp_spill, 0, 4, h->stream));
        prof::Scope ps("pp_agg", h->stream);
        launch_pp_agg_rc(h->stream, h->dspec, S, h->dbatches, mode, 1u << h->pp_bits, R.part, R.fin, 64 - h->pp_bits - h->pp_rc_sub,
                         h->pp_rc_sub, o, h->pp_spill, SPILL_CAP);
        // partitions too large for it (skewed keys): the slot-table kernel, over the spilled ids only
        launch_pp_agg(h->stream, h->dspec, S, h->dbatches, mode, 1u << h->pp_bits, R.part, nullptr, R.fin, R.alt, nullptr, nullptr,
                      o, h->pp_spill, SPILL_CAP);
    } else {
        prof::Scope ps("pp_agg", h->stream);
        launch_pp_agg(h->stream, h->dspec, S, h->dbatches, mode, 1u << h->pp_bits, R.l1_n ? R.part : nullptr,
                      T.l1_n ? T.part : nullptr, R.fin, R.alt, T.fin, T.alt, o);
    }
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

// Group records + per-block string lengths (scanned; totals in pp_tot[PPT_STR + c]).  Async.
static int pp_grec_build(dbg_agg_handle* h) {
    const Spec& S = h->spec;
    RETURN_IF(pp_agg(h, 1, nullptr));
    const u64 N = std::max<u64>(pp_records(h), 1);
    h->pp_nb = pp_grec_blocks(N);
    RETURN_IF(ensure_dev(&h->pp_blk, &h->pp_blk_cap, (u64)S.n_keys * h->pp_nb + 8));
    if (S.has_strings && pp_records(h)) {
        launch_pp_grec_lengths(h->stream, h->dspec, h->pp_grec, h->pp_tot, h->pp_blk, h->pp_nb, h->dbatches);
        for (int c = 0; c < S.n_keys; ++c)
            if (S.key_types[c].type == DBG_STRING)
                launch_exclusive_scan(h->stream, h->pp_blk + (u64)c * h->pp_nb, h->pp_nb, h->pp_tot + PPT_STR + c);
    }
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

static int pp_read_tot(dbg_agg_handle* h) {
    if (!h->pp_htot) HIPCHECK(hipHostMalloc((void**)&h->pp_htot, PPT_WORDS * 8, hipHostMallocDefault));
    HIPCHECK(hipMemcpyAsync(h->pp_htot, h->pp_tot, PPT_WORDS * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    h->pp_stat_rounds = h->pp_htot[PPT_ROUNDS];
    if (h->pp_htot[PPT_ERR] & ERR_OVF_LOST) return fail(DBG_ERR_INTERNAL, "partitioned aggregate: spill list exhausted");
    return DBG_OK;
}

// dbg_agg_finalize in partitioned mode: group records built, sizes known.
// Decimal128 MIN/MAX (precision > 18) states are the only updates that can give up
// (at_minmax128); handles without them skip the read-back.
static int check_minmax_spin(dbg_agg_handle* h) {
    bool any = false;
    for (int a = 0; a < h->spec.n_aggs; ++a) any |= h->spec.aggs[a].mmk == MMK_I128 &&
                                                    (h->spec.aggs[a].kind == DBG_AGG_MIN || h->spec.aggs[a].kind == DBG_AGG_MAX);
    if (!any) return DBG_OK;
    u64 e = 0;
    HIPCHECK(hipMemcpyAsync(&e, h->counters + CNT_ERR, 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    if (e & ERR_MINMAX_SPIN) return fail(DBG_ERR_INTERNAL, MINMAX_SPIN_MSG);
    return DBG_OK;
}

static int pp_finalize(dbg_agg_handle* h, uint64_t* n_groups, uint64_t* string_bytes) {
    const Spec& S = h->spec;
    RETURN_IF(check_minmax_spin(h));
    if (!h->pp_grec_ready) {
        RETURN_IF(pp_grec_build(h));
        RETURN_IF(pp_read_tot(h));
        if (h->pp_htot[PPT_GROUPS] > pp_records(h)) return fail(DBG_ERR_INTERNAL, "partitioned aggregate: more groups than records");
        h->pp_grec_ready = true;
    }
    h->n_groups = h->pp_htot[PPT_GROUPS];
    h->string_bytes.assign(S.n_keys, 0);
    for (int c = 0; c < S.n_keys; ++c)
        h->string_bytes[c] = S.key_types[c].type == DBG_STRING ? h->pp_htot[PPT_STR + c] : 0;
    h->finalized = true;
    if (n_groups) *n_groups = h->n_groups;
    if (string_bytes)
        for (int c = 0; c < S.n_keys; ++c) string_bytes[c] = h->string_bytes[c];
    return DBG_OK;
}

static int add_groups_now(dbg_agg_handle* h, const dbg_column* group_cols, const dbg_column* arg_cols, const dbg_filter* filter,
                          uint64_t rows, int on_device) {
    if (rows >= 0xFFFFFFFFULL) return fail(DBG_ERR_UNSUPPORTED, "a batch holds fewer than 2^32 rows");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_deferred(h));
    h->finalized = false;
    if (rows == 0) return DBG_OK;
    const Spec& S = h->spec;
    BatchDesc* st;
    u32 bid;
    const size_t owned0 = h->owned.size();
    RETURN_IF(new_batch(h, &st, &bid));
    st->rows = rows;
    for (int c = 0; c < S.n_keys; ++c) {
        if (group_cols[c].len < rows) return fail(DBG_ERR_INVALID, "group column shorter than rows");
        RETURN_IF(to_dcol(h, group_cols[c], S.key_types[c], true, on_device, st->keys[c]));
    }
    for (int a = 0; a < S.n_aggs; ++a) {
        if (S.aggs[a].arg_type < 0) continue;
        if (!arg_cols) return fail(DBG_ERR_INVALID, "missing aggregate arguments");
        dbg_datatype want{S.aggs[a].arg_type, 0, arg_cols[a].dt.scale, (uint8_t)S.aggs[a].arg_nullable, 0};
        if (arg_cols[a].len < rows) return fail(DBG_ERR_INVALID, "argument column shorter than rows");
        RETURN_IF(to_dcol(h, arg_cols[a], want, true, on_device, st->args[a]));
    }
    if (filter && filter->n_nodes) RETURN_IF(fill_filter(h, filter, on_device, st->fcols, &st->n_fcols, st->nodes, &st->n_nodes));
    RETURN_IF(submit_batch(h, &st, &bid, on_device && h->owned.size() == owned0));
    // high cardinality: the radix-partitioned payload instead of the HBM table (pp.hip)
    if (!h->pp) RETURN_IF(pp_maybe_switch(h, bid, rows));
    if (h->pp) return pp_add_batch(h, st, bid, rows, 0);
    // A first batch the probe puts at many groups gets a table sized for them before its insert:
    // the partitioned insert needs a large table, and growing by overflow afterwards costs the
    // whole batch again (C3's first 1e9-row batch into the initial table: 1.5 s + a retry pass)
    // (AggregateHashTable::get_capacity_for_count: next_pow2(count * LOAD_FACTOR 1.5),
    // EAGG/aggregate_hashtable.rs:567-569, mod.rs:49 — 2x, the earlier rule, put C3's 1.34e8 groups
    // 0.06 % below 2^28 and any estimator overshoot doubled the table, a radix pass and both
    // finalize scans).  Best-effort: capped at half the free device memory, and a failed
    // allocation keeps the current table (overflow growth then sizes it by the rows it meets).
    if (h->table_rows == 0 && h->pp_probed && h->est_groups > 65536.0) {
        u64 target = pow2_at_least((u64)std::min(1.5 * h->est_groups + 1.0, (double)(1ULL << 31)));
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
            while (target > h->cap && (double)(target + 1) * h->spec.tstride * 8.0 > 0.5 * (double)free_b) target >>= 1;
        if (target > h->cap && grow_table(h, target) != DBG_OK) {
            (void)hipGetLastError();
            g_last_error.clear();
        }
    }
    h->table_rows += rows;
    const bool was_clean = h->clean;
    h->clean = false;
    // worst-case pushes of this launch: every row, and every LDS slot of every workgroup
    u64 blocks = std::min<u64>(2048, (rows + 4095) / 4096) + 1;
    if (part_slice_bits(S, *st, rows, h->cap)) {
        // radix-partitioned insert: every row may become an overflow record (probe left its
        // slice).  ensure_ovf may resolve pending overflow (and resize): shape after it.
        RETURN_IF(ensure_ovf(h, 0, rows));
    }
    if (u32 sb = part_slice_bits(S, *st, rows, h->cap)) {
        RETURN_IF(part_insert(h, st, bid, rows, sb, on_device != 0, was_clean));
        if (!on_device) RETURN_IF(resolve_overflow(h));
        return DBG_OK;
    }
    RETURN_IF(ensure_ovf(h, rows, 2 * blocks * 4096));
    if (on_device && h->recycle && h->hcounters_dev && insert_can_fuse(S, *st, h->cap)) {  // held back: see def_on
        h->def_on = true;
        h->def_clean = was_clean;
        h->def_bid = bid;
        h->def_rows = rows;
        h->def_hb = *st;
        return DBG_OK;
    }
    {
        prof::Scope ps("agg_insert", h->stream);
        launch_insert(h->stream, h->dspec, S, h->dbatches, bid, rows, false, table_desc(h), true, st);
    }
    HIPCHECK(hipGetLastError());
    if (!on_device) RETURN_IF(resolve_overflow(h));  // host path: synchronous like the reference processor
    return DBG_OK;
}

// Staged host blocks -> one batch (host_stage.hpp).  The host path is synchronous (it resolves
// overflow before returning), so the staging vectors are free again when this returns.
static int stage_flush(dbg_agg_handle* h) {
    if (h->stage.empty()) return DBG_OK;
    std::vector<dbg_column> k, a, fc;
    std::vector<dbg_pred_node> nd;
    dbg_filter flt;
    h->stage.views(k, a, fc, nd, flt);
    int rc = add_groups_now(h, k.data(), a.data(), flt.n_nodes ? &flt : nullptr, h->stage.rows, 0);
    if (rc == DBG_OK && hipStreamSynchronize(h->stream) != hipSuccess) rc = fail(DBG_ERR_DEVICE, "stream synchronize");
    h->stage.clear();
    return rc;
}

// Everything a caller queued (staged host rows, a held-back insert) reaches the table.
int flush_pending(dbg_agg_handle* h) {
    RETURN_IF(stage_flush(h));
    return flush_deferred(h);
}

int dbg_agg_add_groups(dbg_agg_handle* h, const dbg_column* group_cols, const dbg_column* arg_cols, const dbg_filter* filter,
                       uint64_t rows, int on_device) {
    if (!h || !group_cols) return fail(DBG_ERR_INVALID, "null argument");
    HIPCHECK(hipSetDevice(h->device));
    hstage::Stage& G = h->stage;
    if (on_device || !G.cap || rows >= G.cap) {
        RETURN_IF(stage_flush(h));
        return add_groups_now(h, group_cols, arg_cols, filter, rows, on_device);
    }
    const Spec& S = h->spec;
    // the checks add_groups_now would make, before the rows are accepted
    for (int c = 0; c < S.n_keys; ++c) {
        const dbg_column& g = group_cols[c];
        if (g.len < rows) return fail(DBG_ERR_INVALID, "group column shorter than rows");
        if (g.dt.type != S.key_types[c].type || (g.dt.type == DBG_DECIMAL128 && g.dt.scale != S.key_types[c].scale) ||
            (g.dt.nullable && !S.key_types[c].nullable))
            return fail(DBG_ERR_INVALID, "column type does not match the declared type");
    }
    for (int a = 0; a < S.n_aggs; ++a) {
        if (S.aggs[a].arg_type < 0) continue;
        if (!arg_cols) return fail(DBG_ERR_INVALID, "missing aggregate arguments");
        if (arg_cols[a].len < rows) return fail(DBG_ERR_INVALID, "argument column shorter than rows");
        if (arg_cols[a].dt.type != S.aggs[a].arg_type) return fail(DBG_ERR_INVALID, "column type does not match the declared type");
    }
    if (filter && filter->n_nodes)
        for (int c = 0; c < filter->n_cols; ++c)
            if (filter->cols[c].len < rows) return fail(DBG_ERR_INVALID, "filter column shorter than rows");
    if (!G.empty() && (G.rows + rows > G.cap || !G.same_filter(filter))) RETURN_IF(stage_flush(h));
    if (rows == 0) return DBG_OK;
    int32_t arg_types[DBG_MAX_AGGS];
    for (int a = 0; a < S.n_aggs; ++a) arg_types[a] = S.aggs[a].arg_type;
    G.append(S.n_keys, group_cols, S.n_aggs, arg_cols, arg_types, filter, rows);
    h->finalized = false;
    return DBG_OK;
}

int dbg_agg_set_host_staging(dbg_agg_handle* h, uint64_t rows) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(stage_flush(h));
    h->stage.cap = rows >= 0xFFFFFFFFULL ? 0xFFFFFFFEULL : rows;
    return DBG_OK;
}

static int ensure_buf(u64** p, u64* cap, u64 n) {
    if (n <= *cap) return DBG_OK;
    if (*p) HIPCHECK(hipFree(*p));
    *cap = std::max<u64>(n, 1024);
    return dev_alloc((void**)p, *cap * 8);
}

int dbg_agg_finalize(dbg_agg_handle* h, uint64_t* n_groups, uint64_t* string_bytes) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    if (h->pp) return pp_finalize(h, n_groups, string_bytes);
    const Spec& S = h->spec;
    // Optimistic single round trip: count + scan are enqueued behind the inserts and read back
    // together with the overflow counters; only when an insert overflowed does the table grow
    // (resolve_overflow) and the count run again.
    for (int round = 0; round < 3; ++round) {
        u64 nb = finalize_blocks(h->cap);
        RETURN_IF(ensure_buf(&h->d_pos, &h->pos_cap, nb + 16));
        RETURN_IF(ensure_buf(&h->d_str_pos, &h->str_pos_cap, (u64)S.n_keys * nb + 8));
        TableDesc t = table_desc(h);
        {
            prof::Scope ps("count_groups", h->stream);
            launch_count_groups(h->stream, h->dspec, S, h->dbatches, t, 1, 0, nullptr, h->d_pos, h->d_str_pos);
        }
        u64* totals = h->d_pos + nb;  // [0] groups, [1 + c] string bytes of key column c
        launch_exclusive_scan(h->stream, h->d_pos, nb, totals);
        if (S.has_strings && !S.inline_keys)
            for (int c = 0; c < S.n_keys; ++c)
                if (S.key_types[c].type == DBG_STRING) launch_exclusive_scan(h->stream, h->d_str_pos + (u64)c * nb, nb, totals + 1 + c);
        HIPCHECK(hipMemcpyAsync(h->hcounters, h->counters, CNT_WORDS * 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHECK(hipMemcpyAsync(h->hcounters + CNT_WORDS, totals, 8 * (S.n_keys + 1), hipMemcpyDeviceToHost, h->stream));
        HIPCHECK(hipStreamSynchronize(h->stream));
        if (h->hcounters[CNT_ERR] & ERR_OVF_LOST) return fail(DBG_ERR_INTERNAL, "overflow list exhausted");
        if (h->hcounters[CNT_ERR] & ERR_MINMAX_SPIN) return fail(DBG_ERR_INTERNAL, MINMAX_SPIN_MSG);
        if (h->hcounters[CNT_ERR] & ERR_FIXED_INCOMPLETE)
            return fail(DBG_ERR_INVALID, "fixed-capacity exchange incomplete (a partial held more groups than the "
                                         "buffer, or unresolved overflow): use dbg_agg_partition + export_records");
        if (h->hcounters[CNT_OVF_ROWS] || h->hcounters[CNT_OVF_RECS]) {
            RETURN_IF(resolve_overflow(h));
            continue;
        }
        h->pending_rows = h->pending_recs = 0;
        const u64* tot = h->hcounters + CNT_WORDS;
        h->n_groups = tot[0];
        note_observed(h);
        h->string_bytes.assign(S.n_keys, 0);
        for (int c = 0; c < S.n_keys; ++c)
            h->string_bytes[c] = (S.key_types[c].type == DBG_STRING && !S.inline_keys) ? tot[1 + c] : 0;
        if (h->n_groups != h->hcounters[CNT_CLAIMS])
            return fail(DBG_ERR_INTERNAL, "group count mismatch: " + std::to_string(h->n_groups) + " vs claims " +
                                              std::to_string(h->hcounters[CNT_CLAIMS]));
        // keep the load factor sane for the next batch (the reference resizes at 1/1.5)
        if ((double)h->n_groups * 1.5 > (double)h->cap) {
            RETURN_IF(grow_table(h, pow2_at_least((u64)(h->n_groups * 2.0) + 1)));
            continue;  // positions depend on the slot layout: count again
        }
        h->finalized = true;
        if (n_groups) *n_groups = h->n_groups;
        if (string_bytes)
            for (int c = 0; c < S.n_keys; ++c) string_bytes[c] = h->string_bytes[c];
        return DBG_OK;
    }
    return fail(DBG_ERR_INTERNAL, "finalize did not converge");
}

// Upper bound of one group's serialized state of aggregate a (agg_serialize).
static u32 ser_stride_of(const DAgg& A) {
    u32 n;
    switch (A.kind) {
        case DBG_AGG_COUNT: return 8;
        case DBG_AGG_SUM: n = A.sumk == SUMK_I128 ? 16 : 8; break;
        case DBG_AGG_AVG: n = A.sumk == SUMK_I128 ? 24 : 16; break;
        default: n = 1 + type_width(A.arg_type);
    }
    if (A.ser_flags & SER_NULL_ADPT) n++;
    if (A.ser_flags & SER_OR_NULL) n++;
    return n;
}

static int result_impl(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys, int on_device, bool ser);

int dbg_agg_result(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys, int on_device) {
    return result_impl(h, out_aggs, out_keys, on_device, false);
}

int dbg_agg_serialized_stride(dbg_agg_handle* h, uint32_t* stride) {
    if (!h || !stride) return fail(DBG_ERR_INVALID, "null argument");
    for (int a = 0; a < h->spec.n_aggs; ++a) {
        if (h->src_kinds[a] == DBG_AGG_AVG_SQL)
            return fail(DBG_ERR_UNSUPPORTED, "serialized states: SQL avg is sum and count in the reference plan");
        stride[a] = ser_stride_of(h->spec.aggs[a]);
    }
    return DBG_OK;
}

int dbg_agg_result_serialized(dbg_agg_handle* h, dbg_out_column* out_states, dbg_out_column* out_keys, int on_device) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    for (int a = 0; a < h->spec.n_aggs; ++a)
        if (h->src_kinds[a] == DBG_AGG_AVG_SQL)
            return fail(DBG_ERR_UNSUPPORTED, "serialized states: SQL avg is sum and count in the reference plan");
    return result_impl(h, out_states, out_keys, on_device, true);
}

static int result_impl(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys, int on_device, bool ser) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    if (!h->finalized) return fail(DBG_ERR_INVALID, "dbg_agg_finalize must precede dbg_agg_result");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    const Spec& S = h->spec;
    u64 n = h->n_groups;
    for (int a = 0; a < S.n_aggs; ++a) out_aggs[a].dt = ser ? dbg_datatype{DBG_STRING, 0, 0, 0, 0} : h->result_types[a];
    for (int c = 0; c < S.n_keys; ++c) out_keys[c].dt = S.key_types[c];
    if (n == 0) {
        for (int c = 0; c < S.n_keys; ++c)
            if (S.key_types[c].type == DBG_STRING && out_keys[c].offsets) {
                u64 z = 0;
                if (on_device) HIPCHECK(hipMemcpy(out_keys[c].offsets, &z, 8, hipMemcpyHostToDevice));
                else out_keys[c].offsets[0] = 0;
            }
        for (int a = 0; a < S.n_aggs && ser; ++a)
            if (out_aggs[a].offsets) {
                u64 z = 0;
                if (on_device) HIPCHECK(hipMemcpy(out_aggs[a].offsets, &z, 8, hipMemcpyHostToDevice));
                else out_aggs[a].offsets[0] = 0;
            }
        return DBG_OK;
    }
    std::vector<void*> temps;
    auto tmp = [&](size_t bytes, void** p) -> int {
        RETURN_IF(dev_alloc(p, bytes));
        temps.push_back(*p);
        return DBG_OK;
    };
    auto free_temps = [&]() {
        for (void* p : temps) hipFree(p);
    };
    OutDesc od;
    memset(&od, 0, sizeof(od));
    od.cap_groups = n;
    for (int c = 0; c < S.n_keys; ++c) od.cap_str[c] = h->string_bytes[c];
    int rc = DBG_OK;
    // device destinations
    for (int c = 0; c < S.n_keys && rc == DBG_OK; ++c) {
        const dbg_datatype& t = S.key_types[c];
        size_t bytes = t.type == DBG_STRING ? h->string_bytes[c] : n * type_width(t.type);
        if (on_device) od.key_data[c] = out_keys[c].data;
        else rc = tmp(bytes, &od.key_data[c]);
        if (rc == DBG_OK && t.type == DBG_STRING) {
            if (on_device) od.key_offsets[c] = out_keys[c].offsets;
            else rc = tmp((n + 1) * 8, (void**)&od.key_offsets[c]);
        }
        if (rc == DBG_OK && t.nullable) rc = tmp(n, (void**)&od.key_valid[c]);
    }
    for (int a = 0; a < S.n_aggs && rc == DBG_OK; ++a) {
        const dbg_datatype& t = h->result_types[a];
        if (ser) {  // fixed-stride rows + lengths, compacted into Binary columns below
            od.ser = 1;
            od.ser_stride[a] = ser_stride_of(S.aggs[a]);
            rc = tmp(n * od.ser_stride[a], &od.agg_data[a]);
            if (rc == DBG_OK) rc = tmp(n, (void**)&od.agg_valid[a]);
            continue;
        }
        if (on_device) od.agg_data[a] = out_aggs[a].data;
        else rc = tmp(n * type_width(t.type), &od.agg_data[a]);
        if (rc == DBG_OK && t.nullable) {
            if (agg_always_valid(S.aggs[a])) od.all_valid |= 1u << a;
            else rc = tmp(n, (void**)&od.agg_valid[a]);
        }
    }
    if (rc != DBG_OK) {
        free_temps();
        return rc;
    }
    if (h->pp) {
        prof::Scope ps("pp_write", h->stream);
        launch_pp_grec_write(h->stream, h->dspec, h->dbatches, h->pp_grec, h->pp_tot, h->pp_blk, h->pp_nb, od,
                             h->counters + CNT_ERR);
    } else {
        prof::Scope ps("write_results", h->stream);
        launch_write_results(h->stream, h->dspec, S, h->dbatches, table_desc(h), h->d_pos, h->d_str_pos, od);
    }
    // offsets[n] and bit-packed validity
    for (int c = 0; c < S.n_keys; ++c) {
        const dbg_datatype& t = S.key_types[c];
        if (t.type == DBG_STRING) {
            u64 tot = h->string_bytes[c];
            hipMemcpyAsync(od.key_offsets[c] + n, &h->string_bytes[c], 8, hipMemcpyHostToDevice, h->stream);
            (void)tot;
        }
        if (t.nullable) {
            u8* bits = nullptr;
            if (on_device) bits = out_keys[c].validity;
            else if (tmp((n + 7) / 8, (void**)&bits) != DBG_OK) {
                free_temps();
                return DBG_ERR_OOM;
            }
            if (bits) launch_pack_bits(h->stream, od.key_valid[c], n, bits);
            if (!on_device && out_keys[c].validity)
                hipMemcpyAsync(out_keys[c].validity, bits, (n + 7) / 8, hipMemcpyDeviceToHost, h->stream);
        }
    }
    std::vector<u64> ser_tot(S.n_aggs, 0);
    u64* dser_tot = nullptr;
    if (ser) {
        if (tmp(8ull * S.n_aggs, (void**)&dser_tot) != DBG_OK) {
            free_temps();
            return DBG_ERR_OOM;
        }
        for (int a = 0; a < S.n_aggs; ++a) {
            u64* offs = nullptr;
            u8* data = nullptr;
            if (on_device) {
                offs = out_aggs[a].offsets;
                data = (u8*)out_aggs[a].data;
            } else if (tmp((n + 1) * 8, (void**)&offs) != DBG_OK || tmp(n * od.ser_stride[a], (void**)&data) != DBG_OK) {
                free_temps();
                return DBG_ERR_OOM;
            }
            launch_ser_compact(h->stream, od.agg_valid[a], (const u8*)od.agg_data[a], od.ser_stride[a], n, offs, data, dser_tot + a);
            if (!on_device) {
                od.agg_data[a] = data;  // copied out below with the totals known
                if (out_aggs[a].offsets)
                    hipMemcpyAsync(out_aggs[a].offsets, offs, (n + 1) * 8, hipMemcpyDeviceToHost, h->stream);
            }
        }
        HIPCHECK(hipMemcpyAsync(ser_tot.data(), dser_tot, 8ull * S.n_aggs, hipMemcpyDeviceToHost, h->stream));
        HIPCHECK(hipStreamSynchronize(h->stream));
        if (!on_device)
            for (int a = 0; a < S.n_aggs; ++a)
                if (out_aggs[a].data && ser_tot[a])
                    hipMemcpyAsync(out_aggs[a].data, od.agg_data[a], ser_tot[a], hipMemcpyDeviceToHost, h->stream);
    }
    for (int a = 0; a < S.n_aggs && !ser; ++a) {
        const dbg_datatype& t = h->result_types[a];
        if (t.nullable) {
            u8* bits = nullptr;
            if (on_device) bits = out_aggs[a].validity;
            else if (tmp((n + 7) / 8, (void**)&bits) != DBG_OK) {
                free_temps();
                return DBG_ERR_OOM;
            }
            if (bits && od.agg_valid[a]) launch_pack_bits(h->stream, od.agg_valid[a], n, bits);
            else if (bits) launch_fill_valid(h->stream, n, bits);
            if (!on_device && out_aggs[a].validity)
                hipMemcpyAsync(out_aggs[a].validity, bits, (n + 7) / 8, hipMemcpyDeviceToHost, h->stream);
        }
    }
    if (!on_device) {
        for (int c = 0; c < S.n_keys; ++c) {
            const dbg_datatype& t = S.key_types[c];
            size_t bytes = t.type == DBG_STRING ? h->string_bytes[c] : n * type_width(t.type);
            if (out_keys[c].data && bytes) hipMemcpyAsync(out_keys[c].data, od.key_data[c], bytes, hipMemcpyDeviceToHost, h->stream);
            if (t.type == DBG_STRING && out_keys[c].offsets)
                hipMemcpyAsync(out_keys[c].offsets, od.key_offsets[c], (n + 1) * 8, hipMemcpyDeviceToHost, h->stream);
        }
        for (int a = 0; a < S.n_aggs && !ser; ++a)
            if (out_aggs[a].data)
                hipMemcpyAsync(out_aggs[a].data, od.agg_data[a], n * type_width(h->result_types[a].type), hipMemcpyDeviceToHost, h->stream);
    }
    HIPCHECK(hipMemcpyAsync(h->hcounters, h->counters, CNT_WORDS * 8, hipMemcpyDeviceToHost, h->stream));
    hipError_t e = hipStreamSynchronize(h->stream);
    free_temps();
    if (e != hipSuccess) return fail(DBG_ERR_DEVICE, std::string("result: ") + hipGetErrorString(e));
    if (h->hcounters[CNT_ERR] & ERR_DEC_OVERFLOW) {
        HIPCHECK(hipMemsetAsync(h->counters + CNT_ERR, 0, 8, h->stream));
        return fail(DBG_ERR_OVERFLOW, "Decimal overflow");
    }
    return DBG_OK;
}


int dbg_agg_set_strategy(dbg_agg_handle* h, int strategy) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    if (strategy < DBG_STRATEGY_AUTO || strategy > DBG_STRATEGY_PARTITIONED) return fail(DBG_ERR_INVALID, "unknown strategy");
    if (h->table_rows || h->ppk[0].l1_n || h->ppk[1].l1_n)
        return fail(DBG_ERR_INVALID, "dbg_agg_set_strategy: the handle holds groups (call it after create or reset)");
    // AUTO switches only for records of <= 256 bytes (build_spec: pp_ok); a forced partitioned
    // payload runs up to the scatter's limit: a tile needs one wave of 64 rows in its 32 KiB
    // scratch (pp_direct_t > 0, i.e. records of <= 512 bytes) and <= 64 state words per group
    const Spec& PS = h->spec;
    const bool pp_fits = pp_direct_t(PS.pp_rw_raw) > 0 && pp_direct_t(PS.pp_rw_state) > 0 && PS.pp_sw <= 64;
    if (strategy == DBG_STRATEGY_PARTITIONED && !pp_fits)
        return fail(DBG_ERR_UNSUPPORTED, "dbg_agg_set_strategy: records too wide for the partitioned payload");
    h->strategy = strategy;
    h->pp = strategy == DBG_STRATEGY_PARTITIONED;
    // a new strategy starts a new query on the handle: forget the cardinality the last finalize saw
    h->obs_rows = h->obs_groups = 0;
    return DBG_OK;
}

int dbg_agg_get_strategy(dbg_agg_handle* h, int* partitioned, uint64_t* extra_rounds) {
    if (!h || !partitioned) return fail(DBG_ERR_INVALID, "null argument");
    *partitioned = h->pp ? (h->pp_spec >= 0 ? 2 : 1) : 0;
    if (extra_rounds) *extra_rounds = h->pp_stat_rounds;
    return DBG_OK;
}

int dbg_agg_set_partition_keys(dbg_agg_handle* h, int n_keys) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    if (n_keys < 0 || n_keys > h->spec.n_keys) return fail(DBG_ERR_INVALID, "partition keys: 0..n_group_cols");
    h->part_keys = n_keys;
    return DBG_OK;
}

int dbg_agg_set_recycle(dbg_agg_handle* h, int on) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    h->recycle = on ? 1 : 0;
    return DBG_OK;
}

// Fused finalize in partitioned mode: the LDS aggregation writes the result columns directly
// (fixed-width keys) or through group records (string keys: offsets need the scanned lengths).
static int pp_fin_launch(dbg_agg_handle* h, const OutDesc& od) {
    const Spec& S = h->spec;
    if (!S.has_strings) {
        RETURN_IF(pp_agg(h, 0, &od));
    } else {
        RETURN_IF(pp_grec_build(h));
        if (pp_records(h)) {
            prof::Scope ps("pp_write", h->stream);
            launch_pp_grec_write(h->stream, h->dspec, h->dbatches, h->pp_grec, h->pp_tot, h->pp_blk, h->pp_nb, od,
                                 h->pp_tot + PPT_ERR);
        }
    }
    launch_finish_outputs(h->stream, od, h->pp_tot, S.n_keys, S.n_aggs);
    if (!h->pp_htot) HIPCHECK(hipHostMalloc((void**)&h->pp_htot, PPT_WORDS * 8, hipHostMallocDefault));
    HIPCHECK(hipMemcpyAsync(h->pp_htot, h->pp_tot, PPT_WORDS * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

static int pp_fin_complete(dbg_agg_handle* h, uint64_t* n_groups, uint64_t* string_bytes) {
    const Spec& S = h->spec;
    FinState& F = h->fin;
    HIPCHECK(hipStreamSynchronize(h->stream));
    h->uploads_pending = false;
    const u64* t = h->pp_htot;
    h->pp_stat_rounds = t[PPT_ROUNDS];
    h->n_groups = t[PPT_GROUPS];
    h->string_bytes.assign(S.n_keys, 0);
    bool short_buf = h->n_groups > F.max_groups;
    for (int c = 0; c < S.n_keys; ++c) {
        h->string_bytes[c] = S.key_types[c].type == DBG_STRING ? t[PPT_STR + c] : 0;
        if (S.key_types[c].type == DBG_STRING && h->string_bytes[c] > F.cap_str[c]) short_buf = true;
    }
    *n_groups = h->n_groups;
    if (string_bytes)
        for (int c = 0; c < S.n_keys; ++c) string_bytes[c] = h->string_bytes[c];
    h->pp_grec_ready = S.has_strings != 0;
    h->finalized = h->pp_grec_ready;
    if (t[PPT_ERR] & ERR_DEC_OVERFLOW) return fail(DBG_ERR_OVERFLOW, "Decimal overflow");
    if (t[PPT_ERR] & ERR_OVF_LOST) return fail(DBG_ERR_INTERNAL, "partitioned aggregate: spill list exhausted");
    RETURN_IF(check_minmax_spin(h));
    if (short_buf) return fail(DBG_ERR_INVALID, "output buffers too small: " + std::to_string(h->n_groups) + " groups");
    return DBG_OK;
}

// Fused finalize, split into launch and completion so a caller can overlap the device work with
// other launches (dbg_agg_finalize_into_async / dbg_agg_finalize_wait).
static int fin_launch(dbg_agg_handle* h) {
    FinState& F = h->fin;
    const Spec& S = h->spec;
    RETURN_IF(stage_flush(h));  // staged host rows first (this launches any held-back insert)
    u64 nb = finalize_blocks(h->cap);
    RETURN_IF(ensure_buf(&h->d_pos, &h->pos_cap, nb + 16));
    RETURN_IF(ensure_buf(&h->d_str_pos, &h->str_pos_cap, (u64)S.n_keys * nb + 8));
    // the held-back partitioned insert's table stage writes the result columns directly (one
    // non-nullable integer key, COUNT(*): what part_slice_bits admits; the table stays empty)
    const bool direct = h->def_part && !h->pp && S.n_keys == 1 && S.n_aggs == 1 && !S.key_types[0].nullable &&
                        !h->result_types[0].nullable && type_width(h->result_types[0].type) == 8 && F.keys[0].data && F.aggs[0].data &&
                        type_width(S.key_types[0].type) == (u32)h->def_part_kw;
    if (direct) {
        h->def_part = false;
        RETURN_IF(ensure_buf(&h->part_status, &h->part_status_cap, part_direct_status_words(h->cap, h->def_part_sb)));
    }
    TableDesc t = direct ? TableDesc{} : table_desc(h);
    const bool small = h->cap + 1 <= FIN_SMALL_SLOTS;
    const bool fuse = h->def_on && !h->pp && small && h->hcounters_dev && insert_can_fuse(S, h->def_hb, h->cap);
    if (!fuse) RETURN_IF(flush_deferred(h));
    u64* totals = h->d_pos + nb;
    F.direct = direct;
    if (!small && !h->pp && !direct) {
        prof::Scope ps("count_groups", h->stream);
        launch_count_groups(h->stream, h->dspec, S, h->dbatches, t, 1, 0, nullptr, h->d_pos, h->d_str_pos);
        launch_exclusive_scan(h->stream, h->d_pos, nb, totals);
        if (S.has_strings && !S.inline_keys)
            for (int c = 0; c < S.n_keys; ++c)
                if (S.key_types[c].type == DBG_STRING) launch_exclusive_scan(h->stream, h->d_str_pos + (u64)c * nb, nb, totals + 1 + c);
    }
    OutDesc od;
    memset(&od, 0, sizeof(od));
    od.cap_groups = F.max_groups;
    u8* vb = h->vbytes;
    for (int c = 0; c < S.n_keys; ++c) {
        od.key_data[c] = F.keys[c].data;
        od.key_offsets[c] = S.key_types[c].type == DBG_STRING ? F.keys[c].offsets : nullptr;
        od.cap_str[c] = (S.key_types[c].type == DBG_STRING && F.has_max_str) ? F.max_str[c] : 0;
        F.cap_str[c] = od.cap_str[c];
        if (S.key_types[c].nullable) {
            od.key_valid[c] = vb;
            od.key_bits[c] = F.keys[c].validity;
            vb += F.max_groups + 1;
        }
    }
    for (int a = 0; a < S.n_aggs; ++a) {
        od.agg_data[a] = F.aggs[a].data;
        if (h->result_types[a].nullable) {
            od.agg_bits[a] = F.aggs[a].validity;
            if (agg_always_valid(S.aggs[a])) {
                od.all_valid |= 1u << a;
            } else {
                od.agg_valid[a] = vb;
                vb += F.max_groups + 1;
            }
        }
    }
    if (h->pp) {
        F.zero_copy = false;
        F.seq = ++h->fin_seq;
        RETURN_IF(pp_fin_launch(h, od));
        F.active = true;
        return DBG_OK;
    }
    F.zero_copy = small && !direct && h->hcounters_dev != nullptr;
    F.seq = ++h->fin_seq;
    if (direct) {
        prof::Scope ps("part_direct", h->stream);
        TableDesc td{};
        td.slots = h->slots;
        td.cap = h->cap;
        hipError_t e = launch_part_direct(h->stream, td, h->def_part_sb, h->part_sorted, h->part_bounds, h->part_status,
                                          h->def_part_kw, od.key_data[0], (u64*)od.agg_data[0], od.cap_groups, totals);
        if (e != hipSuccess) return fail(DBG_ERR_DEVICE, std::string("partitioned insert (direct stage): ") + hipGetErrorString(e));
        launch_finish_outputs(h->stream, od, totals, S.n_keys, S.n_aggs);
    } else if (fuse) {  // the held-back insert and this finalize in one launch
        FusedFin ff;
        ff.out = od;
        ff.totals = totals;
        ff.host_mirror = h->hcounters_dev;
        ff.seq = F.seq;
        ff.recycle = h->recycle;
        ff.on = 1;
        ff.table_empty = h->def_clean ? 1 : 0;
        ff.trace = nullptr;
        ff.dense = nullptr;
        ff.dense_n = 0;
        {  // COUNT(*) over a <= 16-bit key into a recycled table: the direct-mapped hand-off
            // measured and not kept (C2 step 45.1 -> 138 us: 256 workgroups' device atomics on the
            // same ~33 addresses serialise at the memory side, profiles/r04/c2_dense_ab.json):
            // EXPERIMENT, DBG_X_DENSE=1
            static const bool dense_on = X_ENV("DBG_X_DENSE") && X_ENV("DBG_X_DENSE")[0] == '1';
            const int kt = S.key_types[0].type;
            const u32 kw = (kt == DBG_INT8 || kt == DBG_UINT8) ? 1 : ((kt == DBG_INT16 || kt == DBG_UINT16) ? 2 : 0);
            const bool co = S.n_aggs == 1 && S.aggs[0].kind == DBG_AGG_COUNT && S.aggs[0].arg_type < 0 && S.aggs[0].w0 == 1;
            if (dense_on && kw && co && h->def_clean && S.n_keys == 1) {
                if (!h->dense) {
                    RETURN_IF(dev_alloc((void**)&h->dense, (65536 + 1024) * 8));
                    HIPCHECK(hipMemsetAsync(h->dense, 0, (65536 + 1024) * 8, h->stream));
                }
                ff.dense = h->dense;
                ff.dense_n = kw == 1 ? 256u : 65536u;
            }
        }
        static u64* x_trace = nullptr;  // EXPERIMENT (DBG_X_TRACE): 8 words per launch, 4096 launches
        static std::vector<u64> x_init;
        if (kPhaseTrace && X_ENV("DBG_X_TRACE")) {
            if (!x_trace) {
                RETURN_IF(dev_alloc((void**)&x_trace, 4096 * 128));
                x_init.assign(16, 0);
                x_init[0] = x_init[1] = ~0ULL;
                atexit([] {
                    std::vector<u64> hb(4096 * 16);
                    hipDeviceSynchronize();
                    hipMemcpy(hb.data(), x_trace, hb.size() * 8, hipMemcpyDeviceToHost);
                    std::vector<std::vector<double>> d(14);
                    for (int k = 0; k < 4096; ++k) {
                        const u64* r = &hb[k * 16];
                        if (r[0] == 0 || r[0] == ~0ULL || r[6] == 0) continue;
                        for (int p = 1; p <= 14; ++p) d[p - 1].push_back((double)(r[p] - r[0]) * 0.01);
                    }
                    const char* nm[] = {"first WG stream end", "last WG stream end", "last block_flush end",
                                        "ticket (last WG)", "table copied", "finalize end", "fin: scanned",
                                        "fin: groups written", "fin: bits packed", "fin: counters read",
                                        "tail: view+counts", "tail: prefix", "tail: t0 loads", "tail: t0 merged"};
                    for (int p = 0; p < 14; ++p) {
                        if (d[p].empty()) continue;
                        std::sort(d[p].begin(), d[p].end());
                        fprintf(stderr, "trace %-22s median %7.2f us  (n=%zu)\n", nm[p], d[p][d[p].size() / 2], d[p].size());
                    }
                });
            }
            ff.trace = x_trace + (F.seq & 4095) * 16;
            HIPCHECK(hipMemcpyAsync(ff.trace, x_init.data(), 128, hipMemcpyHostToDevice, h->stream));
        }
        h->def_on = false;
        prof::Scope ps("agg_insert", h->stream);
        launch_insert(h->stream, h->dspec, S, h->dbatches, h->def_bid, h->def_rows, false, t, true, &h->def_hb, &ff);
    } else if (small) {
        prof::Scope ps("finalize_small", h->stream);
        launch_finalize_small(h->stream, h->dspec, h->dbatches, t, od, totals, F.zero_copy ? h->hcounters_dev : nullptr,
                              h->recycle && F.zero_copy, F.seq);
    } else {
        prof::Scope ps("write_results", h->stream);
        launch_write_results(h->stream, h->dspec, S, h->dbatches, t, h->d_pos, h->d_str_pos, od);
        launch_finish_outputs(h->stream, od, totals, S.n_keys, S.n_aggs);
    }
    if (!F.zero_copy) {
        HIPCHECK(hipMemcpyAsync(h->hcounters, h->counters, CNT_WORDS * 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHECK(hipMemcpyAsync(h->hcounters + CNT_WORDS, totals, 8 * (S.n_keys + 1), hipMemcpyDeviceToHost, h->stream));
    }
    F.active = true;
    return DBG_OK;
}

// Wait for the launched round; *retry = the inserts had overflowed (now resolved: launch again).
static int fin_complete(dbg_agg_handle* h, bool* retry, uint64_t* n_groups, uint64_t* string_bytes) {
    FinState& F = h->fin;
    const Spec& S = h->spec;
    *retry = false;
    F.active = false;
    if (h->pp) return pp_fin_complete(h, n_groups, string_bytes);
    bool recycled = false;
    const bool direct_done = F.direct;
    if (!F.zero_copy) {
        HIPCHECK(hipStreamSynchronize(h->stream));
    } else {
        // the kernel posts `seq` last (after its write-through mirror stores): spin on it
        // instead of a stream synchronisation (whose wake-up costs several microseconds); after
        // ~20 ms fall back to the blocking wait (long queued inserts)
        volatile u64* hseq = h->hcounters + CNT_WORDS + 2 + DBG_MAX_KEYS;
        volatile u64* hcomp = h->hcounters + MIRROR_COMPACT;
        bool seen = false, compact = false;
        auto t0 = std::chrono::steady_clock::now();
        for (u64 it = 0;; ++it) {
            if (__atomic_load_n(hseq, __ATOMIC_ACQUIRE) == F.seq) {
                seen = true;
                break;
            }
            // the count-only fused finalize posts one word [seq | recycled | groups] when its
            // counters are known (every group claimed in the launch, no overflow)
            const u64 cw = __atomic_load_n(hcomp, __ATOMIC_ACQUIRE);
            if ((cw >> 25) == (F.seq & ((1ULL << 39) - 1))) {
                for (int w = 0; w < CNT_WORDS; ++w) h->hcounters[w] = 0;
                h->hcounters[CNT_CLAIMS] = cw & 0xFFFFFF;
                h->hcounters[CNT_WORDS] = cw & 0xFFFFFF;
                for (int c = 0; c < DBG_MAX_KEYS; ++c) h->hcounters[CNT_WORDS + 1 + c] = 0;
                h->hcounters[CNT_WORDS + 1 + DBG_MAX_KEYS] = (cw >> 24) & 1;
                seen = compact = true;
                break;
            }
            if ((it & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
            __builtin_ia32_pause();
        }
        if (!seen) HIPCHECK(hipStreamSynchronize(h->stream));
        HIPCHECK(hipGetLastError());
        recycled = h->hcounters[CNT_WORDS + 1 + DBG_MAX_KEYS] != 0;
    }
    h->uploads_pending = false;
    if (F.direct) {
        F.direct = false;
        if (h->hcounters[CNT_WORDS] == ~0ULL) {
            // a slice held more keys than its slots, or the result columns are too short: the
            // regular table stage from the same sorted keys (the table was never written), then
            // the table finalize (which reports short buffers with the table intact)
            h->def_part = true;
            RETURN_IF(part_flush(h));
            *retry = true;
            return DBG_OK;
        }
        h->hcounters[CNT_CLAIMS] = h->hcounters[CNT_WORDS];  // the table's own counters were never touched
        recycled = true;
    }
    if (h->hcounters[CNT_ERR] & ERR_OVF_LOST) return fail(DBG_ERR_INTERNAL, "overflow list exhausted");
    if (h->hcounters[CNT_ERR] & ERR_MINMAX_SPIN) return fail(DBG_ERR_INTERNAL, MINMAX_SPIN_MSG);
    if (h->hcounters[CNT_ERR] & ERR_CHAIN_SPIN)
        return fail(DBG_ERR_INTERNAL, "fused finalize: a parked row was not posted in time (GPU hand-off stalled)");
    if (h->hcounters[CNT_ERR] & ERR_FIXED_INCOMPLETE)
        return fail(DBG_ERR_INVALID, "fixed-capacity exchange incomplete (a partial held more groups than the "
                                     "buffer, or unresolved overflow): use dbg_agg_partition + export_records");
    if (h->hcounters[CNT_OVF_ROWS] || h->hcounters[CNT_OVF_RECS]) {
        RETURN_IF(resolve_overflow(h));
        *retry = true;
        return DBG_OK;
    }
    h->pending_rows = h->pending_recs = 0;
    const u64* tot = h->hcounters + CNT_WORDS;
    h->n_groups = tot[0];
    note_observed(h);
    h->string_bytes.assign(S.n_keys, 0);
    bool short_buf = h->n_groups > F.max_groups;
    for (int c = 0; c < S.n_keys; ++c) {
        h->string_bytes[c] = (S.key_types[c].type == DBG_STRING && !S.inline_keys) ? tot[1 + c] : 0;
        if (S.key_types[c].type == DBG_STRING && h->string_bytes[c] > F.cap_str[c]) short_buf = true;
    }
    *n_groups = h->n_groups;
    if (string_bytes)
        for (int c = 0; c < S.n_keys; ++c) string_bytes[c] = h->string_bytes[c];
    if (h->n_groups != h->hcounters[CNT_CLAIMS])
        return fail(DBG_ERR_INTERNAL, "group count mismatch: " + std::to_string(h->n_groups) + " vs claims " +
                                          std::to_string(h->hcounters[CNT_CLAIMS]));
    h->finalized = true;
    if (recycled) {  // the table was re-initialised by the kernel (or never written): dbg_agg_reset state
        h->clean = true;
        h->init_pending = h->init_pending || direct_done;
        h->finalized = false;
        h->n_batches = h->n_cached;
        h->pending_rows = h->pending_recs = 0;
    }
    if (h->hcounters[CNT_ERR] & ERR_DEC_OVERFLOW) {
        if (!recycled) HIPCHECK(hipMemsetAsync(h->counters + CNT_ERR, 0, 8, h->stream));
        return fail(DBG_ERR_OVERFLOW, "Decimal overflow");
    }
    if (short_buf) return fail(DBG_ERR_INVALID, "output buffers too small: " + std::to_string(h->n_groups) + " groups");
    return DBG_OK;
}

static int fin_setup(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys, uint64_t max_groups,
                     const uint64_t* max_string_bytes) {
    const Spec& S = h->spec;
    FinState& F = h->fin;
    for (int a = 0; a < S.n_aggs; ++a) out_aggs[a].dt = h->result_types[a];
    for (int c = 0; c < S.n_keys; ++c) out_keys[c].dt = S.key_types[c];
    F.aggs.assign(out_aggs, out_aggs + S.n_aggs);
    F.keys.assign(out_keys, out_keys + S.n_keys);
    F.max_groups = max_groups;
    F.has_max_str = max_string_bytes != nullptr;
    F.max_str.assign(S.n_keys, 0);
    if (max_string_bytes)
        for (int c = 0; c < S.n_keys; ++c) F.max_str[c] = max_string_bytes[c];
    // validity bytes staging (bit-packed into the caller's buffers by finish_outputs)
    int n_nullable = 0;
    for (int c = 0; c < S.n_keys; ++c) n_nullable += S.key_types[c].nullable ? 1 : 0;
    for (int a = 0; a < S.n_aggs; ++a) n_nullable += h->result_types[a].nullable ? 1 : 0;
    u64 need = (u64)n_nullable * (max_groups + 1);
    if (need > h->vbytes_cap) {
        if (h->vbytes) HIPCHECK(hipFree(h->vbytes));
        h->vbytes_cap = std::max<u64>(need, 4096);
        RETURN_IF(dev_alloc((void**)&h->vbytes, h->vbytes_cap));
    }
    return DBG_OK;
}

int dbg_agg_finalize_into(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys, uint64_t max_groups,
                          const uint64_t* max_string_bytes, uint64_t* n_groups, uint64_t* string_bytes) {
    RETURN_IF(dbg_agg_finalize_into_async(h, out_aggs, out_keys, max_groups, max_string_bytes));
    return dbg_agg_finalize_wait(h, n_groups, string_bytes);
}

int dbg_agg_finalize_into_async(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys, uint64_t max_groups,
                                const uint64_t* max_string_bytes) {
    if (!h || !out_aggs || !out_keys) return fail(DBG_ERR_INVALID, "null argument");
    if (h->fin.active) return fail(DBG_ERR_INVALID, "a finalize is already in flight: dbg_agg_finalize_wait first");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(fin_setup(h, out_aggs, out_keys, max_groups, max_string_bytes));
    return fin_launch(h);
}

int dbg_agg_finalize_wait(dbg_agg_handle* h, uint64_t* n_groups, uint64_t* string_bytes) {
    if (!h || !n_groups) return fail(DBG_ERR_INVALID, "null argument");
    if (!h->fin.active) return fail(DBG_ERR_INVALID, "no finalize in flight");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    for (int round = 0; round < 3; ++round) {
        if (round) RETURN_IF(fin_launch(h));
        bool retry = false;
        int rc = fin_complete(h, &retry, n_groups, string_bytes);
        if (rc != DBG_OK || !retry) return rc;
    }
    return fail(DBG_ERR_INTERNAL, "finalize did not converge");
}

// ---- partial-state records ----
int dbg_agg_record_width(dbg_agg_handle* h, uint32_t* width) {
    if (!h || !width) return fail(DBG_ERR_INVALID, "null argument");
    *width = h->spec.rec_width;
    return DBG_OK;
}

int dbg_agg_record_layout(const dbg_agg_params* params, dbg_record_layout* out) {
    if (!params || !out) return fail(DBG_ERR_INVALID, "null argument");
    Spec S;
    std::vector<dbg_datatype> rt;
    RETURN_IF(build_spec(params, S, rt));
    memset(out, 0, sizeof(*out));
    out->width = S.rec_width;
    out->state_off = S.rec_state_off;
    for (int c = 0; c < S.n_keys; ++c) {
        out->key_off[c] = S.rec_key_off[c];
        out->validity_off[c] = S.key_types[c].nullable ? S.rec_val_off[c] : 0;
    }
    for (int a = 0; a < S.n_aggs; ++a) {
        out->agg_w0[a] = S.aggs[a].w0;
        out->agg_words[a] = S.aggs[a].nwords;
    }
    out->flags_word = S.flags_word;
    out->n_words = S.n_words;
    return DBG_OK;
}

static int legacy_method(const dbg_datatype* types, int n, int* kind, uint32_t* key_bytes);

// The group key's legacy layout (legacy_method's FixedKeys packing or SingleBinary) by key column.
static int legacy_layout(const Spec& S, u32 bits, LegacyLayout* L) {
    memset(L, 0, sizeof(*L));
    int kind = 0;
    uint32_t kb = 0;
    RETURN_IF(legacy_method(S.key_types, S.n_keys, &kind, &kb));
    L->bits = bits;
    if (kind == DBG_LEGACY_SERIALIZER) {  // FastHash of the serialized key bytes (SerCrc, legacy.hpp)
        L->serializer = 1;
        return DBG_OK;
    }
    if (kind == DBG_LEGACY_SINGLE_BINARY) {
        L->binary = 1;
        return DBG_OK;
    }
    L->words = kb <= 8 ? 1 : (kb <= 16 ? 2 : 4);
    // build_keys_vec: stable order by value width, widest first; null bytes after all values
    std::vector<int> order(S.n_keys);
    for (int j = 0; j < S.n_keys; ++j) order[j] = j;
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return type_width(S.key_types[a].type) > type_width(S.key_types[b].type); });
    u32 off = 0, noff = 0;
    for (int j = 0; j < S.n_keys; ++j) noff += type_width(S.key_types[j].type);
    for (int j = 0; j < S.n_keys; ++j) {
        const int c = order[j];
        L->off[c] = off;
        off += type_width(S.key_types[c].type);
        L->null_off[c] = S.key_types[c].nullable ? (int32_t)noff++ : -1;
    }
    return DBG_OK;
}

int dbg_agg_partition(dbg_agg_handle* h, uint32_t n_parts, int scheme, uint64_t* rec_counts, uint64_t* string_bytes) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    if (n_parts < 1 || n_parts > 256) return fail(DBG_ERR_UNSUPPORTED, "1..256 partitions");
    if (scheme < 0 || scheme > 2) return fail(DBG_ERR_INVALID, "scheme 0 (hash % n), 1 (radix bits) or 2 (legacy buckets)");
    if (scheme >= 1 && (n_parts & (n_parts - 1))) return fail(DBG_ERR_INVALID, "radix partitions must be a power of two");
    LegacyLayout L;
    if (scheme == 2) RETURN_IF(legacy_layout(h->spec, 31 - __builtin_clz(n_parts), &L));
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    if (h->pp) RETURN_IF(pp_finalize(h, nullptr, nullptr));
    else RETURN_IF(resolve_overflow(h));
    const Spec& S = h->spec;
    u64 nb = h->pp ? pp_grec_blocks(std::max<u64>(h->n_groups, 1)) : finalize_blocks(h->cap);
    const u32* lpart = nullptr;
    const bool prefix = scheme != 2 && h->part_keys > 0 && h->part_keys < S.n_keys;
    if (prefix && h->pp) return fail(DBG_ERR_UNSUPPORTED, "partition keys: table strategy only");
    if (prefix && n_parts > 1) {  // buckets of the first part_keys key columns' group hash, per slot
        RETURN_IF(ensure_buf(&h->d_lpart, &h->lpart_cap, (h->cap + 1) / 2 + 1));
        prof::Scope ps("prefix_bucket", h->stream);
        launch_prefix_slot_bucket(h->stream, h->dspec, h->dbatches, table_desc(h), h->part_keys, n_parts, scheme, (u32*)h->d_lpart);
        lpart = (const u32*)h->d_lpart;
        scheme = 2;  // count and export read lpart
    }
    if (scheme == 2 && n_parts > 1 && !prefix) {  // hash2bucket<bits, true> of each group's FastHash
        const u64 n = h->pp ? h->n_groups : h->cap + 1;
        RETURN_IF(ensure_buf(&h->d_lpart, &h->lpart_cap, n / 2 + 1));
        prof::Scope ps("legacy_bucket", h->stream);
        if (h->pp) launch_pp_grec_legacy_bucket(h->stream, h->dspec, h->dbatches, h->pp_grec, h->n_groups, L, (u32*)h->d_lpart);
        else launch_legacy_slot_bucket(h->stream, h->dspec, h->dbatches, table_desc(h), L, (u32*)h->d_lpart);
        lpart = (const u32*)h->d_lpart;
    }
    u64 nflat = (u64)n_parts * nb;
    RETURN_IF(ensure_buf(&h->d_part_pos, &h->part_cap, nflat + 8));
    RETURN_IF(ensure_buf(&h->d_part_str_pos, &h->part_str_cap, nflat * S.n_keys + 8));
    if (!h->d_part_str_base) RETURN_IF(dev_alloc((void**)&h->d_part_str_base, 257 * 8));
    HIPCHECK(hipMemsetAsync(h->d_part_str_pos, 0, (nflat * S.n_keys + 8) * 8, h->stream));
    {
        prof::Scope ps("count_groups", h->stream);
        if (h->pp)
            launch_pp_grec_count_parts(h->stream, h->dspec, h->dbatches, h->pp_grec, h->n_groups, n_parts, scheme, lpart,
                                       h->d_part_pos, h->d_part_str_pos, nb);
        else
            launch_count_groups(h->stream, h->dspec, S, h->dbatches, table_desc(h), n_parts, scheme, lpart, h->d_part_pos,
                                h->d_part_str_pos);
    }
    h->part_nb = nb;
    std::vector<u64> hist(nflat), shist(nflat * S.n_keys);
    HIPCHECK(hipMemcpyAsync(hist.data(), h->d_part_pos, nflat * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipMemcpyAsync(shist.data(), h->d_part_str_pos, nflat * S.n_keys * 8, hipMemcpyDeviceToHost, h->stream));
    launch_exclusive_scan(h->stream, h->d_part_pos, nflat, h->d_part_pos + nflat);
    launch_exclusive_scan(h->stream, h->d_part_str_pos, nflat * S.n_keys, h->d_part_str_pos + nflat * S.n_keys);
    HIPCHECK(hipStreamSynchronize(h->stream));
    h->part_counts.assign(n_parts, 0);
    h->part_strings.assign(n_parts, 0);
    for (u32 p = 0; p < n_parts; ++p) {
        for (u64 b = 0; b < nb; ++b) h->part_counts[p] += hist[(u64)p * nb + b];
        for (u64 k = 0; k < (u64)S.n_keys * nb; ++k) h->part_strings[p] += shist[(u64)p * S.n_keys * nb + k];
    }
    std::vector<u64> base(n_parts + 1, 0);
    for (u32 p = 0; p < n_parts; ++p) base[p + 1] = base[p] + h->part_strings[p];
    HIPCHECK(hipMemcpyAsync(h->d_part_str_base, base.data(), (n_parts + 1) * 8, hipMemcpyHostToDevice, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    h->part_n = n_parts;
    h->part_scheme = scheme;
    for (u32 p = 0; p < n_parts; ++p) {
        if (rec_counts) rec_counts[p] = h->part_counts[p];
        if (string_bytes) string_bytes[p] = h->part_strings[p];
    }
    return DBG_OK;
}

int dbg_agg_export_records(dbg_agg_handle* h, void* dev_records, void* dev_strings) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    if (!h->part_n) return fail(DBG_ERR_INVALID, "dbg_agg_partition must precede dbg_agg_export_records");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    prof::Scope ps("export_records", h->stream);
    if (h->pp)
        launch_pp_grec_export(h->stream, h->dspec, h->dbatches, h->pp_grec, h->n_groups, h->part_n, h->part_scheme,
                              (const u32*)h->d_lpart, h->d_part_pos, h->d_part_str_pos, h->part_nb, (u8*)dev_records,
                              (u8*)dev_strings, h->d_part_str_base);
    else
        launch_export(h->stream, h->dspec, h->spec, h->dbatches, table_desc(h), h->part_n, h->part_scheme, (const u32*)h->d_lpart,
                      h->d_part_pos, h->d_part_str_pos, (u8*)dev_records, (u8*)dev_strings, h->d_part_str_base);
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

int dbg_agg_capacity(dbg_agg_handle* h, uint64_t* slots) {
    if (!h || !slots) return fail(DBG_ERR_INVALID, "null argument");
    *slots = h->cap;
    return DBG_OK;
}

// ---- fixed-capacity exchange (replicas + gather, low cardinality) ----
int dbg_agg_export_fixed(dbg_agg_handle* h, void* dev_buf, uint64_t cap_records) {
    if (!h || !dev_buf) return fail(DBG_ERR_INVALID, "null argument");
    const Spec& S = h->spec;
    if (!S.inline_keys) return fail(DBG_ERR_UNSUPPORTED, "fixed export needs fixed-width (inline) group keys");
    if (h->cap + 1 > FIN_SMALL_SLOTS || h->pp) return fail(DBG_ERR_UNSUPPORTED, "fixed export is for small tables");
    if (S.rec_width < 16) return fail(DBG_ERR_INTERNAL, "record narrower than the fixed header");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    prof::Scope ps("export_fixed", h->stream);
    launch_export_fixed(h->stream, h->dspec, h->dbatches, table_desc(h), (u8*)dev_buf, cap_records, h->recycle);
    HIPCHECK(hipGetLastError());
    if (h->recycle) {  // the kernel re-initialised the table: dbg_agg_reset state
        h->clean = true;
        h->finalized = false;
        h->n_batches = h->n_cached;
        h->pending_rows = h->pending_recs = 0;
    }
    return DBG_OK;
}

int dbg_agg_merge_fixed(dbg_agg_handle* h, const void* dev_bufs, int32_t n_bufs, uint64_t cap_records) {
    if (!h || !dev_bufs || n_bufs < 1) return fail(DBG_ERR_INVALID, "bad argument");
    const Spec& S = h->spec;
    if (!S.inline_keys) return fail(DBG_ERR_UNSUPPORTED, "fixed merge needs fixed-width (inline) group keys");
    if (h->pp) return fail(DBG_ERR_UNSUPPORTED, "fixed merge: the handle runs partitioned (high cardinality)");
    const u64 n = (u64)n_bufs * (cap_records + 1);
    if (n >= 0xFFFFFFFFULL) return fail(DBG_ERR_UNSUPPORTED, "segment too large");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    h->finalized = false;
    h->clean = false;
    BatchDesc* st;
    u32 bid;
    RETURN_IF(new_batch(h, &st, &bid));
    h->table_rows += n;
    const u8* base = (const u8*)dev_bufs;
    st->rows = n;
    st->is_records = 1;
    st->rec_width = S.rec_width;
    st->rec_base = base;
    st->seg_records = cap_records + 1;
    for (int c = 0; c < S.n_keys; ++c) {
        DCol& d = st->keys[c];
        const dbg_datatype& t = S.key_types[c];
        d.type = t.type;
        d.precision = t.precision;
        d.scale = t.scale;
        d.nullable = t.nullable;
        d.layout = LAYOUT_RECORD;
        d.width = type_width(t.type);
        d.stride = S.rec_width;
        d.data = base + S.rec_key_off[c];
        d.validity = t.nullable ? base + S.rec_val_off[c] : nullptr;
    }
    RETURN_IF(submit_batch(h, &st, &bid, true));
    u64 blocks = std::min<u64>(2048, (n + 4095) / 4096) + 1;
    RETURN_IF(ensure_ovf(h, n, blocks * 4096));
    prof::Scope ps("agg_merge", h->stream);
    launch_insert(h->stream, h->dspec, S, h->dbatches, bid, n, true, table_desc(h), true);
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

// One segment of state records -> the table (combine_payload's merge_states).  strs[c]: the
// string bytes key column c's (offset, len) pairs point into.
static int merge_record_batch(dbg_agg_handle* h, const u8* base, u64 n, const u8* const* strs) {
    const Spec& S = h->spec;
    if (n == 0) return DBG_OK;
    if (n >= 0xFFFFFFFFULL) return fail(DBG_ERR_UNSUPPORTED, "segment too large");
    BatchDesc* st;
    u32 bid;
    RETURN_IF(new_batch(h, &st, &bid));
    st->rows = n;
    st->is_records = 1;
    st->rec_width = S.rec_width;
    st->rec_base = base;
    for (int c = 0; c < S.n_keys; ++c) {
        DCol& d = st->keys[c];
        const dbg_datatype& t = S.key_types[c];
        d.type = t.type;
        d.precision = t.precision;
        d.scale = t.scale;
        d.nullable = t.nullable;
        d.layout = LAYOUT_RECORD;
        d.width = type_width(t.type);
        d.stride = S.rec_width;
        d.data = base + S.rec_key_off[c];
        d.validity = t.nullable ? base + S.rec_val_off[c] : nullptr;
        d.strings = strs[c];
    }
    RETURN_IF(upload_batch(h, st, bid));
    if (!h->pp) RETURN_IF(pp_maybe_switch(h, bid, n));
    if (h->pp) return pp_add_batch(h, st, bid, n, 1);
    h->table_rows += n;
    u64 blocks = std::min<u64>(2048, (n + 4095) / 4096) + 1;
    RETURN_IF(ensure_ovf(h, n, blocks * 4096));
    prof::Scope ps("agg_merge", h->stream);
    launch_insert(h->stream, h->dspec, S, h->dbatches, bid, n, true, table_desc(h), true);
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

int dbg_agg_merge_records(dbg_agg_handle* h, const void* dev_records, const void* dev_strings, int32_t n_segments,
                          const uint64_t* seg_records, const uint64_t* seg_string_bytes) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    h->finalized = false;
    h->clean = false;
    const Spec& S = h->spec;
    u64 rec_off = 0, str_off = 0;
    for (int g = 0; g < n_segments; ++g) {
        u64 n = seg_records[g];
        const u8* base = (const u8*)dev_records + rec_off * S.rec_width;
        const u8* strs = (const u8*)dev_strings + str_off;
        rec_off += n;
        str_off += seg_string_bytes ? seg_string_bytes[g] : 0;
        const u8* per_col[DBG_MAX_KEYS];
        for (int c = 0; c < DBG_MAX_KEYS; ++c) per_col[c] = strs;
        RETURN_IF(merge_record_batch(h, base, n, per_col));
    }
    return DBG_OK;
}

// Key compaction (the reference copies only a new group's key into its payload arena,
// EAGG/payload_row.rs:111-130, so a partial's memory follows its groups, not the rows it saw):
// every group leaves as an exchange record (keys, string blob, states), the table restarts empty
// and merges the records back, so its ref-key entries point at one record batch of exactly the
// groups, and the inputs seen so far — the library's copies of host blocks and the caller's
// device columns — are no longer referenced.  O(groups); a no-op for inline keys (no references)
// and the partitioned payload (its records already hold the keys).
int dbg_agg_compact(dbg_agg_handle* h, int* compacted) {
    if (!h) return fail(DBG_ERR_INVALID, "null handle");
    if (compacted) *compacted = 0;
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    const Spec& S = h->spec;
    if (h->pp || S.inline_keys) return DBG_OK;
    u64 n = 0, sb = 0;
    RETURN_IF(dbg_agg_partition(h, 1, 0, &n, &sb));
    DevBuf rb, strb;
    rb.bytes = std::max<u64>(n * S.rec_width, 16);
    strb.bytes = std::max<u64>(sb, 16);
    RETURN_IF(dev_alloc(&rb.p, rb.bytes));
    int rc = dev_alloc(&strb.p, strb.bytes);
    if (rc == DBG_OK) rc = dbg_agg_export_records(h, rb.p, strb.p);
    if (rc == DBG_OK && hipStreamSynchronize(h->stream) != hipSuccess) rc = fail(DBG_ERR_DEVICE, "compact: export failed");
    // the handle keeps its strategy: the re-merged batch (one record per group) must not be
    // probed again — on an AUTO handle with many groups the probe would see ratio ~1 and switch
    // to the partitioned payload, after which compaction does nothing
    const u64 rows_before = h->table_rows, remerged_before = h->remerged;
    if (rc == DBG_OK) rc = dbg_agg_reset(h);  // frees the copies of earlier inputs
    h->table_rows = rows_before ? rows_before : 1;
    h->remerged = remerged_before + n;  // merge_record_batch below counts the n records as rows
    if (rc != DBG_OK) {
        hipFree(rb.p);
        if (strb.p) hipFree(strb.p);
        return rc;
    }
    h->owned.push_back(rb);
    h->owned.push_back(strb);
    h->finalized = false;
    h->clean = false;
    const u8* per_col[DBG_MAX_KEYS];
    for (int c = 0; c < DBG_MAX_KEYS; ++c) per_col[c] = (const u8*)strb.p;
    RETURN_IF(merge_record_batch(h, (const u8*)rb.p, n, per_col));
    if (compacted) *compacted = 1;
    return DBG_OK;
}

// Device bytes the handle keeps for the inputs its table references: copies of host blocks and
// received / compacted records (the caller's own device columns are not counted).
int dbg_agg_retained_bytes(dbg_agg_handle* h, uint64_t* bytes) {
    if (!h || !bytes) return fail(DBG_ERR_INVALID, "null argument");
    u64 t = 0;
    for (const auto& b : h->owned) t += b.bytes;
    *bytes = t;
    return DBG_OK;
}

// AggregateMeta::Serialized -> this table (SerializedPayload::convert_to_aggregate_table,
// AGG/aggregate_meta.rs:57-101; AggregateFunction::batch_merge, EAGG/aggregate_function.rs:96-103).
int dbg_agg_merge_serialized(dbg_agg_handle* h, const dbg_column* state_cols, const dbg_column* group_cols, uint64_t rows,
                             int on_device) {
    if (!h || (!state_cols && h->spec.n_aggs) || !group_cols) return fail(DBG_ERR_INVALID, "null argument");
    HIPCHECK(hipSetDevice(h->device));
    RETURN_IF(flush_pending(h));
    h->finalized = false;
    h->clean = false;
    const Spec& S = h->spec;
    for (int a = 0; a < S.n_aggs; ++a)
        if (h->src_kinds[a] == DBG_AGG_AVG_SQL)
            return fail(DBG_ERR_UNSUPPORTED, "serialized states: SQL avg is sum and count in the reference plan");
    if (rows == 0) return DBG_OK;
    if (rows >= 0xFFFFFFFFULL) return fail(DBG_ERR_UNSUPPORTED, "a block holds fewer than 2^32 rows");
    SerIngest in;
    memset(&in, 0, sizeof(in));
    for (int c = 0; c < S.n_keys; ++c) {
        if (group_cols[c].len < rows) return fail(DBG_ERR_INVALID, "group column shorter than rows");
        RETURN_IF(to_dcol(h, group_cols[c], S.key_types[c], true, on_device, in.keys[c]));
    }
    const dbg_datatype bin{DBG_STRING, 0, 0, 0, 0};
    for (int a = 0; a < S.n_aggs; ++a) {
        const dbg_column& sc = state_cols[a];
        if (sc.dt.type != DBG_STRING || sc.dt.nullable || !sc.offsets) return fail(DBG_ERR_INVALID, "a state column is a non-null Binary column");
        if (sc.len < rows) return fail(DBG_ERR_INVALID, "state column shorter than rows");
        DCol d;
        RETURN_IF(to_dcol(h, sc, bin, true, on_device, d));
        in.st_data[a] = d.data;
        in.st_offs[a] = d.offsets;
    }
    // records are retained (the table's ref-key entries point at them) until reset
    DevBuf rb;
    rb.bytes = rows * S.rec_width;
    RETURN_IF(dev_alloc(&rb.p, rows * S.rec_width));
    h->owned.push_back(rb);
    if (!h->ser_err) RETURN_IF(dev_alloc((void**)&h->ser_err, 8));
    HIPCHECK(hipMemsetAsync(h->ser_err, 0, 8, h->stream));
    {
        prof::Scope ps("ser_ingest", h->stream);
        launch_ser_ingest(h->stream, h->dspec, in, rows, (u8*)rb.p, h->ser_err);
    }
    HIPCHECK(hipGetLastError());
    u64 e = 0;
    HIPCHECK(hipMemcpyAsync(&e, h->ser_err, 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    if (e & ERR_SER_MALFORMED) return fail(DBG_ERR_INVALID, "serialized state bytes do not match the aggregate's state layout");
    if (e & ERR_SER_UNREP)
        return fail(DBG_ERR_UNSUPPORTED, "serialized state with a NULL result that the GPU state cannot carry "
                                         "(OrNull flag 0 or None without a nullable argument)");
    const u8* per_col[DBG_MAX_KEYS];
    for (int c = 0; c < DBG_MAX_KEYS; ++c) per_col[c] = c < S.n_keys ? in.keys[c].data : nullptr;
    return merge_record_batch(h, (const u8*)rb.p, rows, per_col);
}

// ---- standalone filter ----
int dbg_filter_select(const dbg_filter* filter, uint64_t rows, uint32_t* sel_out, uint64_t* n_sel, void* stream) {
    if (!filter || !sel_out || !n_sel) return fail(DBG_ERR_INVALID, "null argument");
    if (rows >= 0xFFFFFFFFULL) return fail(DBG_ERR_UNSUPPORTED, "selection indices are u32");
    hipStream_t s = (hipStream_t)stream;
    dbg_agg_handle tmp;  // for owned constant copies
    tmp.stream = s;
    FilterDesc fd;
    memset(&fd, 0, sizeof(fd));
    fd.rows = rows;
    RETURN_IF(fill_filter(&tmp, filter, 1, fd.cols, &fd.n_cols, fd.nodes, &fd.n_nodes));
    FilterDesc* dfd = nullptr;
    u64* scratch = nullptr;
    u64 nb = filter_blocks(rows);
    int rc = dev_alloc((void**)&dfd, sizeof(FilterDesc));
    if (rc == DBG_OK) rc = dev_alloc((void**)&scratch, (nb + 2) * 8);
    if (rc == DBG_OK) {
        hipMemcpyAsync(dfd, &fd, sizeof(fd), hipMemcpyHostToDevice, s);
        {
            prof::Scope ps("filter_select", s);
            launch_filter_select(s, dfd, rows, scratch, scratch + nb, sel_out);
        }
        u64 tot = 0;
        if (nb) hipMemcpyAsync(&tot, scratch + nb, 8, hipMemcpyDeviceToHost, s);
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = fail(DBG_ERR_DEVICE, std::string("filter: ") + hipGetErrorString(e));
        *n_sel = tot;
    }
    if (dfd) hipFree(dfd);
    if (scratch) hipFree(scratch);
    for (auto& b : tmp.owned) hipFree(b.p);
    tmp.owned.clear();
    tmp.stream = nullptr;
    return rc;
}

int dbg_take_fixed(const dbg_column* col, const uint32_t* sel, uint64_t n_sel, void* out_data, uint8_t* out_validity, void* stream) {
    if (!col || !sel || !out_data) return fail(DBG_ERR_INVALID, "null argument");
    if (col->dt.type == DBG_STRING) return fail(DBG_ERR_UNSUPPORTED, "dbg_take_fixed: fixed-width columns only");
    hipStream_t s = (hipStream_t)stream;
    DCol d;
    memset(&d, 0, sizeof(d));
    d.type = col->dt.type;
    d.nullable = col->dt.nullable;
    d.width = type_width(col->dt.type);
    d.stride = d.width;
    d.data = (const u8*)col->data;
    d.validity = col->validity;
    d.validity_offset = col->validity_offset;
    d.data_offset = col->data_offset;
    u8* vbytes = nullptr;
    if (out_validity && col->dt.nullable) RETURN_IF(dev_alloc((void**)&vbytes, n_sel + 1));
    launch_take_fixed(s, d, sel, n_sel, (u8*)out_data, vbytes);
    if (vbytes) launch_pack_bits(s, vbytes, n_sel, out_validity);
    HIPCHECK(hipStreamSynchronize(s));
    if (vbytes) hipFree(vbytes);
    return DBG_OK;
}

int dbg_take_string(const dbg_column* col, const uint32_t* sel, uint64_t n_sel, uint64_t* out_offsets, void* out_data,
                    uint64_t data_cap, uint8_t* out_validity, uint64_t* total_bytes, void* stream) {
    if (!col || !out_offsets || !total_bytes || (n_sel && !sel)) return fail(DBG_ERR_INVALID, "null argument");
    if (col->dt.type != DBG_STRING || !col->offsets) return fail(DBG_ERR_INVALID, "dbg_take_string: String columns only");
    hipStream_t s = (hipStream_t)stream;
    launch_take_string_offsets(s, col->offsets, sel, n_sel, out_offsets);
    // n_sel lengths + one zero -> exclusive scan -> n_sel + 1 offsets; the total lands in a pinned word
    HIPCHECK(hipMemsetAsync(out_offsets + n_sel, 0, 8, s));
    u64* dtot = nullptr;
    RETURN_IF(dev_alloc((void**)&dtot, 8));
    u64 total = 0;
    hipError_t e = hipMemsetAsync(dtot, 0, 8, s);
    if (e == hipSuccess && n_sel) launch_exclusive_scan(s, out_offsets, n_sel + 1, dtot);
    if (e == hipSuccess) e = hipMemcpyAsync(&total, dtot, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(dtot);
    if (e != hipSuccess) return fail(DBG_ERR_DEVICE, hipGetErrorString(e));
    *total_bytes = total;
    if (total > data_cap) return fail(DBG_ERR_INVALID, "dbg_take_string: data buffer too small (*total_bytes needed)");
    if (!n_sel) return DBG_OK;
    if (!out_data) return fail(DBG_ERR_INVALID, "null argument");
    DCol d;
    memset(&d, 0, sizeof(d));
    d.type = DBG_STRING;
    d.nullable = col->dt.nullable;
    d.data = (const u8*)col->data;
    d.offsets = col->offsets;
    d.validity = col->validity;
    d.validity_offset = col->validity_offset;
    u8* vbytes = nullptr;
    if (out_validity && col->dt.nullable) RETURN_IF(dev_alloc((void**)&vbytes, n_sel + 1));
    launch_take_string_bytes(s, d, sel, n_sel, out_offsets, (u8*)out_data, vbytes);
    if (vbytes) launch_pack_bits(s, vbytes, n_sel, out_validity);
    HIPCHECK(hipStreamSynchronize(s));
    if (vbytes) hipFree(vbytes);
    return DBG_OK;
}

// HashMethodKind::choose_hash_method_with_types (EXP/kernels/group_by.rs:48-97)
static int legacy_method(const dbg_datatype* types, int n, int* kind, uint32_t* key_bytes) {
    if (n < 1 || n > DBG_MAX_KEYS) return fail(DBG_ERR_UNSUPPORTED, "1..8 group columns");
    if (n == 1 && types[0].type == DBG_STRING && !types[0].nullable) {
        *kind = DBG_LEGACY_SINGLE_BINARY;
        *key_bytes = 0;
        return DBG_OK;
    }
    u32 len = 0;
    for (int j = 0; j < n; ++j) {
        const int t = types[j].type;
        if (t == DBG_STRING || t == DBG_BOOLEAN || !valid_type(t)) {
            *kind = DBG_LEGACY_SERIALIZER;
            *key_bytes = 0;
            return DBG_OK;
        }
        len += type_width(t) + (types[j].nullable ? 1 : 0);
    }
    *key_bytes = len;
    *kind = len == 1 ? DBG_LEGACY_KEYS_U8 : len == 2 ? DBG_LEGACY_KEYS_U16 : len <= 4 ? DBG_LEGACY_KEYS_U32
          : len <= 8 ? DBG_LEGACY_KEYS_U64 : len <= 16 ? DBG_LEGACY_KEYS_U128 : len <= 32 ? DBG_LEGACY_KEYS_U256
          : DBG_LEGACY_SERIALIZER;
    return DBG_OK;
}

int dbg_legacy_hash_method(const dbg_datatype* types, int n, int* kind, uint32_t* key_bytes) {
    if (!types || !kind || !key_bytes) return fail(DBG_ERR_INVALID, "null argument");
    return legacy_method(types, n, kind, key_bytes);
}

int dbg_legacy_group_hash(const dbg_column* cols, int n, uint64_t rows, uint64_t* out_hash, uint32_t* out_bucket,
                          int bucket_bits, void* stream) {
    if (!cols || !out_hash) return fail(DBG_ERR_INVALID, "null argument");
    if (out_bucket && (bucket_bits < 1 || bucket_bits > 31)) return fail(DBG_ERR_INVALID, "bucket bits 1..31");
    std::vector<dbg_datatype> types(n > 0 ? n : 1);
    for (int j = 0; j < n; ++j) types[j] = cols[j].dt;
    int kind = 0;
    uint32_t kb = 0;
    RETURN_IF(legacy_method(types.data(), n, &kind, &kb));
    for (int j = 0; j < n; ++j)
        if (cols[j].len < rows) return fail(DBG_ERR_INVALID, "column shorter than rows");
    hipStream_t s = (hipStream_t)stream;
    auto dcol = [&](const dbg_column& c) {
        DCol d;
        memset(&d, 0, sizeof(d));
        d.type = c.dt.type;
        d.nullable = c.dt.nullable;
        d.layout = LAYOUT_ARROW;
        d.width = type_width(c.dt.type);
        d.stride = d.width;
        d.data = (const u8*)c.data;
        d.offsets = c.offsets;
        d.validity = c.dt.nullable ? c.validity : nullptr;
        d.validity_offset = c.validity_offset;
        d.data_offset = c.data_offset;
        return d;
    };
    if (kind == DBG_LEGACY_SINGLE_BINARY) {
        launch_legacy_binary_hash(s, dcol(cols[0]), rows, out_hash, out_bucket, (u32)bucket_bits);
    } else if (kind == DBG_LEGACY_SERIALIZER) {
        LegacyKeyDesc d;
        memset(&d, 0, sizeof(d));
        d.n = n;
        for (int j = 0; j < n; ++j) d.cols[j] = dcol(cols[j]);  // key order: the serialized row
        launch_legacy_serializer_hash(s, d, rows, out_hash, out_bucket, (u32)bucket_bits);
    } else {
        LegacyKeyDesc d;
        memset(&d, 0, sizeof(d));
        d.n = n;
        const u32 width = kind == DBG_LEGACY_KEYS_U8 ? 1 : kind == DBG_LEGACY_KEYS_U16 ? 2 : kind == DBG_LEGACY_KEYS_U32 ? 4
                        : kind == DBG_LEGACY_KEYS_U64 ? 8 : kind == DBG_LEGACY_KEYS_U128 ? 16 : 32;
        d.words = width <= 8 ? 1 : width / 8;
        // build_keys_vec: stable sort by value width, widest first; null bytes after all values
        std::vector<int> order(n);
        for (int j = 0; j < n; ++j) order[j] = j;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return type_width(cols[a].dt.type) > type_width(cols[b].dt.type); });
        u32 off = 0, noff = 0;
        for (int j = 0; j < n; ++j) noff += type_width(cols[j].dt.type);
        for (int j = 0; j < n; ++j) {
            const dbg_column& c = cols[order[j]];
            d.cols[j] = dcol(c);
            d.off[j] = off;
            off += type_width(c.dt.type);
            if (c.dt.nullable) d.null_off[j] = noff++;
        }
        launch_legacy_fixed_hash(s, d, rows, out_hash, out_bucket, (u32)bucket_bits);
    }
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s));
    return DBG_OK;
}

int dbg_sort_limit_indices(const dbg_column* col, uint64_t rows, int asc, int nulls_first, uint64_t limit,
                           uint32_t* idx_out, uint64_t* n_out, void* stream) {
    if (!col || !n_out || (!idx_out && limit && rows)) return fail(DBG_ERR_INVALID, "null argument");
    const int t = col->dt.type;
    if (t == DBG_STRING || t == DBG_DECIMAL128 || type_width(t) == 0)
        return fail(DBG_ERR_UNSUPPORTED, "dbg_sort_limit_indices: fixed-width number columns only");
    DCol d;
    memset(&d, 0, sizeof(d));
    d.type = t;
    d.nullable = col->dt.nullable;
    d.width = type_width(t);
    d.stride = d.width;
    d.data = (const u8*)col->data;
    d.validity = col->validity;
    d.validity_offset = col->validity_offset;
    d.data_offset = col->data_offset;
    std::string err;
    int rc = sort_limit_run((hipStream_t)stream, d, rows, asc, nulls_first, limit, idx_out, n_out, err);
    return rc == DBG_OK ? rc : fail(rc, err);
}

int dbg_sort_limit_multi(const dbg_column* cols, int n_cols, const int* asc, const int* nulls_first, uint64_t rows,
                         uint64_t limit, uint32_t* idx_out, uint64_t* n_out, void* stream) {
    if (!cols || !asc || !nulls_first || !n_out || (!idx_out && limit && rows)) return fail(DBG_ERR_INVALID, "null argument");
    if (n_cols < 1 || n_cols > SORT_MAX_COLS) return fail(DBG_ERR_UNSUPPORTED, "dbg_sort_limit_multi: 1..8 sort columns");
    MKeyDesc K;
    memset(&K, 0, sizeof(K));
    K.n = n_cols;
    for (int c = 0; c < n_cols; ++c) {
        const dbg_column& col = cols[c];
        const int t = col.dt.type;
        if (!valid_type(t) || (t != DBG_STRING && type_width(t) == 0))
            return fail(DBG_ERR_UNSUPPORTED, "dbg_sort_limit_multi: number, Decimal128 and String columns");
        if (col.len < rows) return fail(DBG_ERR_INVALID, "column shorter than rows");
        if (t == DBG_STRING && !col.offsets) return fail(DBG_ERR_INVALID, "String column without offsets");
        DCol& d = K.cols[c];
        d.type = t;
        d.nullable = col.dt.nullable;
        d.layout = LAYOUT_ARROW;
        d.width = type_width(t);
        d.stride = d.width;
        d.data = (const u8*)col.data;
        d.offsets = col.offsets;
        d.validity = col.dt.nullable ? col.validity : nullptr;
        d.validity_offset = col.validity_offset;
        d.data_offset = col.data_offset;
        K.desc[c] = asc[c] ? 0 : 1;
        K.nulls_first[c] = nulls_first[c] ? 1 : 0;
    }
    std::string err;
    int rc = sort_multi_limit_run((hipStream_t)stream, K, rows, limit, idx_out, n_out, err);
    return rc == DBG_OK ? rc : fail(rc, err);
}

// ---- profiling ----
int dbg_prof_enable(int on) {
    std::lock_guard<std::mutex> g(prof::mu);
    prof::enabled = on != 0;
    return DBG_OK;
}
int dbg_prof_reset(void) {
    std::lock_guard<std::mutex> g(prof::mu);
    prof::resolve_locked();
    prof::totals.clear();
    return DBG_OK;
}
int dbg_prof_get(int i, const char** name, double* total_ms, uint64_t* launches) {
    std::lock_guard<std::mutex> g(prof::mu);
    prof::resolve_locked();
    if (i < 0 || (size_t)i >= prof::totals.size()) return DBG_ERR_INVALID;
    *name = prof::totals[i].first.c_str();
    *total_ms = prof::totals[i].second.first;
    *launches = prof::totals[i].second.second;
    return DBG_OK;
}

}  // extern "C"

__global__ void dbg_marker_kernel() {}

extern "C" {
int dbg_prof_marker(void* stream) {
    hipLaunchKernelGGL(dbg_marker_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream);
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

// ---- workload generator ----
int dbg_datagen(int cfg, uint64_t seed, uint64_t row_start, uint64_t rows, void** outs, int n_outs, const uint64_t* aux,
                void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (launch_datagen(s, cfg, seed, row_start, rows, outs, n_outs, aux) != 0) return fail(DBG_ERR_INVALID, "bad datagen config");
    HIPCHECK(hipGetLastError());
    return DBG_OK;
}

}  // extern "C"
