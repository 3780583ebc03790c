// C++ harness: HipReductionScheme (include/hdrf_scheme.hpp, over libhdrf.so) against the CPU
// oracle (oracle/hdrf_oracle.c) on the same blocks, the way a DataNode drives the scheme:
// one reduce() per received block, in order.  Test infrastructure (links the oracle).
#include <cstdio>
#include <cstring>
#include <vector>

#include "hdrf_oracle.h"
#include "hdrf_scheme.hpp"

static std::vector<uint8_t> gen(uint64_t seed, size_t n)
{
    std::vector<uint8_t> v(n);
    for (size_t i = 0; i < n; i += 8) {
        uint64_t x = hdrf_oracle_mix64(seed * 0x9E3779B97F4A7C15ull + i / 8);
        std::memcpy(v.data() + i, &x, std::min<size_t>(8, n - i));
    }
    return v;
}

int main()
{
    hdrf_cfg cfg;
    hdrf_default_cfg(&cfg);
    cfg.max_block_bytes = 8 << 20;
    cfg.max_batch_blocks = 1;
    cfg.index_log2 = 18;
    cfg.container_max = 1 << 21;
    hdrf::HipReductionScheme scheme(&cfg);
    hdrf_oracle *ora = hdrf_oracle_new(0, 1, 1 << 21);
    std::vector<std::vector<uint8_t>> blocks;
    blocks.push_back(gen(1, 3 << 20));
    blocks.push_back(blocks[0]);                                   // whole-block duplicate
    std::vector<uint8_t> mix(blocks[0].begin(), blocks[0].begin() + (1 << 20));
    auto fresh = gen(2, 2 << 20);
    mix.insert(mix.end(), fresh.begin(), fresh.end());
    blocks.push_back(mix);
    blocks.push_back(std::vector<uint8_t>(1 << 20, 0));            // all-zero block
    blocks.push_back(gen(3, 777));
    int fails = 0;
    for (size_t i = 0; i < blocks.size(); i++) {
        const auto &b = blocks[i];
        auto g = scheme.reduce(b.data(), b.size(), 100 + i);
        const int64_t cap = (int64_t)b.size() / 700 + 2;
        std::vector<uint32_t> off(cap);
        std::vector<uint8_t> dig(cap * 20), nw(cap), val(cap * 11);
        int64_t ss = 0;
        int64_t n = hdrf_oracle_reduce(ora, b.data(), (int64_t)b.size(), 100 + i, cap, off.data(), dig.data(), nw.data(),
                                       val.data(), &ss);
        bool ok = n == (int64_t)g.offsets.size() && std::memcmp(off.data(), g.offsets.data(), n * 4) == 0 &&
                  std::memcmp(dig.data(), g.digests.data(), n * 20) == 0 &&
                  std::memcmp(nw.data(), g.is_new.data(), n) == 0 && ss == g.store_size &&
                  scheme.length(100 + i) == (int64_t)b.size();
        std::vector<uint8_t> orec(4 + n * 20);
        ok = ok && hdrf_oracle_recipe(ora, 100 + i, orec.data(), (int64_t)orec.size()) == (int64_t)orec.size() &&
             scheme.recipe(100 + i) == orec;
        uint8_t v1[11], v2[11];
        ok = ok && scheme.index_get(g.digests.data(), v1) && hdrf_oracle_index_get(ora, g.digests.data(), v2) &&
             std::memcmp(v1, v2, 11) == 0;
        std::printf("block %zu: n=%lld store=%lld %s\n", i, (long long)n, (long long)ss, ok ? "OK" : "MISMATCH");
        fails += !ok;
    }
    for (size_t i = 0; i < blocks.size(); i++) {                   // DataConstructor round trip
        const bool ok = scheme.reconstruct(100 + i) == blocks[i];
        std::printf("reconstruct %zu: %s\n", i, ok ? "OK" : "MISMATCH");
        fails += !ok;
    }
    try {
        scheme.reconstruct(999);
        fails++;
    } catch (const hdrf::Error &e) {
        std::printf("reconstruct unknown -> %s\n", e.what());
    }
    hdrf_oracle_free(ora);
    std::printf(fails ? "FAIL\n" : "PASS\n");
    return fails ? 1 : 0;
}
