// Host test of the symmetric-heap arena (openshmem-async_amd/csrc/arena.cpp):
// random alloc/free sequences against a brute-force byte map (no overlap,
// alignment, in-bounds, full coalescing back to one free extent), the
// determinism two PEs rely on (same calls -> same offsets), and
// $SHMEM_SYMMETRIC_HEAP_SIZE parsing (utils/unitparse.c:102-135).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <vector>

#include "heap.h"

using shmx::heap::Arena;

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);    \
            ++fails;                                                    \
        }                                                               \
    } while (0)

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200000;
    const uint64_t cap = uint64_t(64) << 20;
    Arena a(cap), b(cap);          // two "PEs" fed the same calls
    std::vector<uint8_t> owner(cap / Arena::kGranule, 0);
    std::map<uint64_t, uint64_t> live;   // off -> bytes
    std::mt19937_64 rng(12345);
    for (int it = 0; it < iters && !fails; ++it) {
        if (live.empty() || rng() % 3) {
            const uint64_t bytes = 1 + rng() % (rng() % 8 ? 65536 : (4 << 20));
            const uint64_t align = uint64_t(1) << (rng() % 14);
            const uint64_t off = a.alloc(bytes, align);
            CHECK(b.alloc(bytes, align) == off);
            if (off == Arena::kNone) continue;
            CHECK(off % (align < Arena::kGranule ? Arena::kGranule : align) == 0);
            CHECK(off + bytes <= cap);
            for (uint64_t g = off / Arena::kGranule; g < (off + bytes + Arena::kGranule - 1) / Arena::kGranule; ++g) {
                CHECK(owner[g] == 0);
                owner[g] = 1;
            }
            CHECK(a.size_of(off) == bytes);
            live[off] = bytes;
        } else {
            auto itl = live.begin();
            std::advance(itl, rng() % live.size());
            const uint64_t off = itl->first, bytes = itl->second;
            CHECK(a.free(off));
            CHECK(b.free(off));
            for (uint64_t g = off / Arena::kGranule; g < (off + bytes + Arena::kGranule - 1) / Arena::kGranule; ++g)
                owner[g] = 0;
            live.erase(itl);
        }
        CHECK(a.live_blocks() == live.size());
    }
    CHECK(!a.free(12345));                 // not a block
    for (auto &kv : live) CHECK(a.free(kv.first));
    CHECK(a.free_bytes() == cap);
    CHECK(a.alloc(cap, 1) == 0);           // fully coalesced: one extent again
    CHECK(a.alloc(1, 1) == Arena::kNone);  // and now full
    CHECK(a.alloc(0, 1) == Arena::kNone);
    CHECK(a.alloc(16, 3) == Arena::kNone); // alignment not a power of two

    uint64_t v = 0;
    CHECK(shmx::heap::parse_size("1024", &v) && v == 1024);
    CHECK(shmx::heap::parse_size("32M", &v) && v == (uint64_t(32) << 20));
    CHECK(shmx::heap::parse_size("4g", &v) && v == (uint64_t(4) << 30));
    CHECK(shmx::heap::parse_size("2k", &v) && v == 2048);
    CHECK(shmx::heap::parse_size("1t", &v) && v == (uint64_t(1) << 40));
    CHECK(!shmx::heap::parse_size("", &v));
    CHECK(!shmx::heap::parse_size("12q", &v));
    CHECK(!shmx::heap::parse_size("12MB", &v));
    CHECK(!shmx::heap::parse_size("-5", &v));
    CHECK(!shmx::heap::parse_size("99999999999999999999", &v));
    CHECK(!shmx::heap::parse_size("99999999999e", &v));
    if (fails) return 1;
    std::printf("ok %d\n", iters);
    return 0;
}
