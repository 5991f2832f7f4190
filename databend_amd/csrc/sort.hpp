// sort.hpp — ORDER BY <one column> LIMIT k on device (sort.hip).
#pragma once
#include <string>

#include "device.hpp"

#define SORT_CAP 2048  // largest LIMIT served on device (one workgroup's LDS bitonic sort)

// ORDER BY several columns (numbers, Decimal128, String) LIMIT k: the columns in sort order with
// their directions (sort.hip sort_multi_limit_run).
#define SORT_MAX_COLS 8
struct MKeyDesc {
    int32_t n;
    uint8_t desc[SORT_MAX_COLS];
    uint8_t nulls_first[SORT_MAX_COLS];
    DCol cols[SORT_MAX_COLS];
};
int sort_multi_limit_run(hipStream_t s, const MKeyDesc& K, u64 rows, u64 limit, u32* idx_out, u64* n_out, std::string& err);

int sort_limit_run(hipStream_t s, const DCol& c, u64 rows, int asc, int nulls_first, u64 limit, u32* idx_out,
                   u64* n_out, std::string& err);
