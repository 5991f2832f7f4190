// sort.hpp — ORDER BY <one column> LIMIT k on device (sort.hip).
#pragma once
#include <string>

#include "device.hpp"

#define SORT_CAP 2048  // largest LIMIT served on device (one workgroup's LDS bitonic sort)

int sort_limit_run(hipStream_t s, const DCol& c, u64 rows, int asc, int nulls_first, u64 limit, u32* idx_out,
                   u64* n_out, std::string& err);
