// Host test of dm_copy::CopyPool (deoss_amd/csrc/copy_pool.hpp): many threads run copy jobs at
// once (ragged items, empty items, items larger than a piece, a pool of 0 helpers), every byte
// checked.  Built and run plain, with ASan/UBSan and with TSan by tests/test_copy_pool.py (no GPU).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "copy_pool.hpp"

static int fails = 0;
#define EXPECT(c)                                                         \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            fails++;                                                      \
        }                                                                 \
    } while (0)

static void one_thread(dm_copy::CopyPool& pool, unsigned seed, int rounds) {
    std::mt19937_64 rng(seed);
    for (int r = 0; r < rounds; r++) {
        const int n = 1 + (int)(rng() % 24);
        std::vector<std::vector<uint8_t>> src(n), dst(n);
        std::vector<dm_copy::CopyItem> items;
        for (int i = 0; i < n; i++) {
            const size_t len = (rng() % 5 == 0) ? 0 : (rng() % 3 == 0 ? dm_copy::kCopyPiece * 2 + rng() % 1000 : rng() % 70000);
            src[i].resize(len);
            for (size_t k = 0; k < len; k++) src[i][k] = (uint8_t)(k * 131 + i + seed);
            dst[i].assign(len + 16, 0xAB);   // guard bytes after the copy
            items.push_back({dst[i].data(), src[i].data(), len});
        }
        pool.run(items);
        for (int i = 0; i < n; i++) {
            const size_t len = src[i].size();
            EXPECT(std::equal(src[i].begin(), src[i].end(), dst[i].begin()));
            for (size_t k = len; k < len + 16; k++) EXPECT(dst[i][k] == 0xAB);
        }
    }
}

int main() {
    for (size_t helpers : {0, 1, 7}) {
        dm_copy::CopyPool pool(helpers);
        EXPECT(pool.threads() == helpers);
        pool.run({});                                  // nothing to copy
        std::vector<std::thread> th;
        for (unsigned t = 0; t < 8; t++) th.emplace_back(one_thread, std::ref(pool), 1000 * (unsigned)helpers + t, 4);
        for (auto& x : th) x.join();
    }
    if (fails) return 1;
    std::printf("copy pool: PASS\n");
    return 0;
}
