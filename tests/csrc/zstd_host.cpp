// Host build of the device Zstandard decoder (databend_amd/csrc/zstd_dev.hpp, ZS_HOST) for
// tests/test_zstd_host.py: the decoder's logic checked on the CPU against libzstd-made frames.
#include <cstdlib>
#include <vector>
#define ZS_HOST 1
#include "zstd_dev.hpp"

extern "C" int zs_host_decode(const u8* src, u64 sn, u8* dst, u64 dn) {
    ZsTables* T = (ZsTables*)calloc(1, sizeof(ZsTables));
    ZsWork* W = (ZsWork*)calloc(1, sizeof(ZsWork));
    std::vector<u8> lit(ZS_MAX_BLOCK + 16);
    const bool ok = zs_decode(src, sn, dst, dn, lit.data(), *T, *W);
    free(W);
    free(T);
    return ok ? 0 : 1;
}
