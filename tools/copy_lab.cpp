// Host copy lab (the pageable host-resident path): how fast
// can T threads move a 256 MiB pageable array through a 16 MiB bounce slot
// and back out, with glibc memcpy against 32-byte non-temporal stores?
//
//   copy_lab <threads> <MiB> <reps>
//
// Prints GB/s for: memcpy in (src -> slot, slot reused per chunk), NT in,
// memcpy out (slot -> dst), NT out.  CPU only; the GPU is not touched.
#include <immintrin.h>
#include <pthread.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

__attribute__((target("avx2"))) static void nt_copy(char *dst, const char *src, size_t n) {
    size_t i = 0;
    // head to 32-B alignment of the destination
    const size_t mis = (32 - ((uintptr_t)dst & 31)) & 31;
    if (mis) {
        const size_t h = std::min(mis, n);
        std::memcpy(dst, src, h);
        i = h;
    }
    for (; i + 128 <= n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i *)(src + i));
        __m256i b = _mm256_loadu_si256((const __m256i *)(src + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i *)(src + i + 64));
        __m256i d = _mm256_loadu_si256((const __m256i *)(src + i + 96));
        _mm256_stream_si256((__m256i *)(dst + i), a);
        _mm256_stream_si256((__m256i *)(dst + i + 32), b);
        _mm256_stream_si256((__m256i *)(dst + i + 64), c);
        _mm256_stream_si256((__m256i *)(dst + i + 96), d);
    }
    if (i < n) std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

static void par(int T, char *dst, const char *src, size_t n, bool nt) {
    std::vector<std::thread> th;
    const size_t per = (n / T + 63) & ~size_t(63);
    for (int t = 0; t < T; ++t) {
        const size_t lo = std::min(n, per * t), hi = std::min(n, per * (t + 1));
        th.emplace_back([=] {
            if (hi > lo) {
                if (nt) nt_copy(dst + lo, src + lo, hi - lo);
                else std::memcpy(dst + lo, src + lo, hi - lo);
            }
        });
    }
    for (auto &x : th) x.join();
}

int main(int argc, char **argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 8;
    const size_t bytes = (size_t)(argc > 2 ? std::atoi(argv[2]) : 256) << 20;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
    const size_t slot = size_t(16) << 20;
    char *src = (char *)std::malloc(bytes), *dst = (char *)std::malloc(bytes);
    char *ring = (char *)std::aligned_alloc(4096, 4 * slot);
    std::memset(src, 1, bytes);
    std::memset(dst, 2, bytes);
    std::memset(ring, 3, 4 * slot);
    for (int nt = 0; nt < 2; ++nt) {
        for (int dir = 0; dir < 2; ++dir) {
            double best = 1e30;
            for (int r = 0; r < reps; ++r) {
                const auto t0 = std::chrono::steady_clock::now();
                for (size_t off = 0, k = 0; off < bytes; off += slot, ++k) {
                    char *s = ring + (k % 4) * slot;
                    const size_t b = std::min(slot, bytes - off);
                    if (dir == 0) par(T, s, src + off, b, nt);
                    else par(T, dst + off, s, b, nt);
                }
                best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            }
            std::printf("%-3s %-4s threads %2d  %7.1f GB/s\n", nt ? "nt" : "mem", dir ? "out" : "in", T,
                        bytes / best / 1e9);
        }
    }
    return 0;
}
