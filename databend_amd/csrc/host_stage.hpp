// host_stage.hpp — host-block staging for dbg_agg_add_groups (dbg_agg_set_host_staging).
//
// The reference feeds TransformPartialAggregate blocks of at most max_block_size = 65,536 rows
// (src/query/settings/src/settings_default.rs:131), one AggregateHashTable::add_groups per block
// (AGG/transform_aggregate_partial.rs:291-323).  On the GPU one launch per 65,536 rows leaves
// most of the chip idle and spends a host round trip per block, so host-resident blocks are
// appended here (columns concatenated: fixed-width values, string bytes with rebased offsets,
// validity and boolean bitmaps bit-appended) and handed to the device as one batch of up to
// `cap` rows.  A block whose filter program differs from the staged one, or any call that reads
// the table, flushes first; a block of >= cap rows passes straight through.
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dbgpu_agg.h"

namespace hstage {

inline int type_width(int t) {
    switch (t) {
        case DBG_INT8: case DBG_UINT8: case DBG_BOOLEAN: return 1;
        case DBG_INT16: case DBG_UINT16: return 2;
        case DBG_INT32: case DBG_UINT32: case DBG_FLOAT32: case DBG_DATE: return 4;
        case DBG_INT64: case DBG_UINT64: case DBG_FLOAT64: case DBG_TIMESTAMP: return 8;
        case DBG_DECIMAL128: return 16;
        default: return 0;
    }
}

// Append n bits of src (starting at bit src_off, LSB-first) after the first dst_bits bits of dst.
inline void append_bits(std::vector<uint8_t>& dst, uint64_t dst_bits, const uint8_t* src, uint64_t src_off, uint64_t n) {
    dst.resize((dst_bits + n + 7) / 8, 0);
    if ((dst_bits & 7) == 0 && (src_off & 7) == 0) {
        memcpy(dst.data() + dst_bits / 8, src + src_off / 8, (n + 7) / 8);
        if (n & 7) dst[(dst_bits + n) / 8] &= (uint8_t)((1u << (n & 7)) - 1);
        return;
    }
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t s = src_off + i, d = dst_bits + i;
        uint8_t bit = (src[s >> 3] >> (s & 7)) & 1;
        if (bit) dst[d >> 3] |= (uint8_t)(1u << (d & 7));
        else dst[d >> 3] &= (uint8_t)~(1u << (d & 7));
    }
}

inline void append_ones(std::vector<uint8_t>& dst, uint64_t dst_bits, uint64_t n) {
    dst.resize((dst_bits + n + 7) / 8, 0);
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t d = dst_bits + i;
        dst[d >> 3] |= (uint8_t)(1u << (d & 7));
    }
}

struct Column {
    dbg_datatype dt{};
    bool present = false;
    std::vector<uint8_t> data;
    std::vector<uint64_t> offsets;
    std::vector<uint8_t> validity;
    bool has_validity = false;
    uint64_t rows = 0;

    void clear() {
        present = false;
        has_validity = false;
        data.clear();
        offsets.clear();
        validity.clear();
        rows = 0;
    }

    void append(const dbg_column& c, uint64_t n) {
        if (!present) {
            dt = c.dt;
            present = true;
            if (dt.type == DBG_STRING) offsets.assign(1, 0);
        }
        if (c.dt.nullable) dt.nullable = 1;
        const int t = c.dt.type;
        if (t == DBG_STRING) {
            const uint64_t lo = n ? c.offsets[0] : 0, hi = n ? c.offsets[n] : 0;
            const uint64_t base = offsets.back();
            offsets.reserve(offsets.size() + n);
            for (uint64_t i = 1; i <= n; ++i) offsets.push_back(base + (c.offsets[i] - lo));
            data.insert(data.end(), (const uint8_t*)c.data + lo, (const uint8_t*)c.data + hi);
        } else if (t == DBG_BOOLEAN) {
            append_bits(data, rows, (const uint8_t*)c.data, c.data_offset, n);
        } else {
            const uint64_t w = (uint64_t)type_width(t);
            data.insert(data.end(), (const uint8_t*)c.data, (const uint8_t*)c.data + n * w);
        }
        const bool bitmap = c.dt.nullable && c.validity;
        if (bitmap && !has_validity) {  // earlier blocks were all valid
            append_ones(validity, 0, rows);
            has_validity = true;
        }
        if (bitmap) append_bits(validity, rows, c.validity, c.validity_offset, n);
        else if (has_validity) append_ones(validity, rows, n);
        rows += n;
    }

    dbg_column view() const {
        dbg_column c;
        memset(&c, 0, sizeof(c));
        c.dt = dt;
        c.data = data.empty() ? nullptr : data.data();
        c.offsets = dt.type == DBG_STRING ? offsets.data() : nullptr;
        c.validity = has_validity ? validity.data() : nullptr;
        c.len = rows;
        return c;
    }
};

struct Stage {
    uint64_t cap = 0;  // rows per launch; 0 = staging off
    uint64_t rows = 0;
    std::vector<Column> keys, args, fcols;
    std::vector<dbg_pred_node> nodes;  // str pointers rebound to strs on flush
    std::vector<std::string> strs;
    bool has_filter = false;

    bool empty() const { return rows == 0; }

    void clear() {
        rows = 0;
        for (auto& c : keys) c.clear();
        for (auto& c : args) c.clear();
        for (auto& c : fcols) c.clear();
        nodes.clear();
        strs.clear();
        has_filter = false;
    }

    // Does filter f evaluate exactly as the staged program?
    bool same_filter(const dbg_filter* f) const {
        const bool hf = f && f->n_nodes;
        if (hf != has_filter) return false;
        if (!hf) return true;
        if ((size_t)f->n_nodes != nodes.size() || (size_t)f->n_cols != fcols.size()) return false;
        for (int k = 0; k < f->n_nodes; ++k) {
            const dbg_pred_node &a = f->nodes[k], &b = nodes[k];
            if (a.op != b.op || a.cmp != b.cmp || a.col != b.col || a.col2 != b.col2 || a.i64 != b.i64 ||
                memcmp(&a.f64, &b.f64, 8) != 0 || a.i128_lo != b.i128_lo || a.i128_hi != b.i128_hi || a.str_len != b.str_len)
                return false;
            if (a.str_len && memcmp(a.str, strs[k].data(), a.str_len) != 0) return false;
        }
        for (int c = 0; c < f->n_cols; ++c)
            if (f->cols[c].dt.type != fcols[c].dt.type || f->cols[c].dt.scale != fcols[c].dt.scale) return false;
        return true;
    }

    // arg_types[c] < 0: aggregate c takes no argument (count(*)); its column is never read, as in
    // the unstaged add_groups (a zero-initialised dbg_column there has type 0 and no data)
    void append(int n_keys, const dbg_column* k, int n_aggs, const dbg_column* a, const int32_t* arg_types,
                const dbg_filter* f, uint64_t n) {
        keys.resize(n_keys);
        args.resize(n_aggs);
        for (int c = 0; c < n_keys; ++c) keys[c].append(k[c], n);
        for (int c = 0; c < n_aggs; ++c)
            if (a && arg_types[c] >= 0) args[c].append(a[c], n);
        if (f && f->n_nodes) {
            if (!has_filter) {
                has_filter = true;
                nodes.assign(f->nodes, f->nodes + f->n_nodes);
                strs.assign(f->n_nodes, std::string());
                for (int i = 0; i < f->n_nodes; ++i)
                    if (f->nodes[i].str_len) strs[i].assign((const char*)f->nodes[i].str, f->nodes[i].str_len);
                fcols.resize(f->n_cols);
            }
            for (int c = 0; c < f->n_cols; ++c) fcols[c].append(f->cols[c], n);
        }
        rows += n;
    }

    // Views for one add_groups call over everything staged.
    void views(std::vector<dbg_column>& k, std::vector<dbg_column>& a, std::vector<dbg_column>& fc,
               std::vector<dbg_pred_node>& nd, dbg_filter& flt) const {
        k.clear();
        a.clear();
        fc.clear();
        for (auto& c : keys) k.push_back(c.view());
        for (auto& c : args) {
            dbg_column v = c.view();
            if (!c.present) v.dt.type = -1;
            a.push_back(v);
        }
        for (auto& c : fcols) fc.push_back(c.view());
        nd = nodes;
        for (size_t i = 0; i < nd.size(); ++i) nd[i].str = nd[i].str_len ? (const uint8_t*)strs[i].data() : nullptr;
        flt.nodes = nd.data();
        flt.n_nodes = (int32_t)nd.size();
        flt.n_cols = (int32_t)fc.size();
        flt.cols = fc.data();
    }
};

}  // namespace hstage
