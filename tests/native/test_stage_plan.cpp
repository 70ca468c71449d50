// CPU test of the host staging pipeline's chunk schedule (csrc/stage_plan.h):
// for many (n, chunk, element size, ramp) the chunks tile [0, n) in order,
// none exceeds a full chunk, every chunk but the last starts 16 B-aligned
// relative to the array, the ramp's quarter and half chunks sit at both ends
// when there are at least four chunks' worth, and uniform chunks otherwise.
//
//   test_stage_plan          prints "ok <schedules>"
#include <cstdio>
#include <vector>

#include "stage_plan.h"

int main() {
    long schedules = 0, fails = 0;
    const size_t sizes[] = {1, 2, 4, 8, 16};
    for (size_t sz : sizes) {
        const size_t g = sz >= 16 ? 1 : 16 / sz;
        for (size_t chunk_el : {g, 2 * g, 4 * g, 64 * g, 1000 * g, 4096 * g}) {
            for (size_t n : {size_t(1), g - 1 + 1, chunk_el - 1, chunk_el, chunk_el + 1, 3 * chunk_el + 7,
                             4 * chunk_el - 1, 4 * chunk_el, 4 * chunk_el + g + 3, 17 * chunk_el + 5,
                             64 * chunk_el + 2 * g - 1}) {
                if (n == 0) continue;
                for (bool ramp : {false, true}) {
                    std::vector<size_t> off, cnt;
                    shmx::stage_plan(n, chunk_el, g, ramp, off, cnt);
                    ++schedules;
                    bool ok = !cnt.empty() && off.size() == cnt.size() && off[0] == 0;
                    size_t end = 0;
                    for (size_t k = 0; ok && k < cnt.size(); ++k) {
                        ok = off[k] == end && cnt[k] > 0 && cnt[k] <= chunk_el + g;
                        if (k + 1 < cnt.size()) ok = ok && off[k] % g == 0 && cnt[k] <= chunk_el;
                        end += cnt[k];
                    }
                    ok = ok && end == n;
                    const bool ramped = ramp && n >= 4 * chunk_el && chunk_el >= g;
                    if (ok && ramped) {
                        const size_t q = (chunk_el / 4) / g * g > g ? (chunk_el / 4) / g * g : g;
                        const size_t h = (chunk_el / 2) / g * g > g ? (chunk_el / 2) / g * g : g;
                        ok = cnt.size() >= 4 && cnt[0] == q && cnt[1] == h && cnt[cnt.size() - 2] == h &&
                             cnt.back() >= q && cnt.back() < q + g;
                    } else if (ok) {
                        for (size_t k = 0; ok && k + 1 < cnt.size(); ++k) ok = cnt[k] == chunk_el;
                        ok = ok && cnt.size() == (n + chunk_el - 1) / chunk_el;
                    }
                    if (!ok) {
                        ++fails;
                        std::printf("FAIL sz %zu chunk %zu n %zu ramp %d (%zu chunks)\n", sz, chunk_el, n, (int)ramp,
                                    cnt.size());
                    }
                }
            }
        }
    }
    if (fails) return 1;
    std::printf("ok %ld\n", schedules);
    return 0;
}
