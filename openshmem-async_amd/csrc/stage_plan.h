// The host staging pipeline's chunk schedule (staging.cpp): which elements
// each chunk of a host-resident blocking call moves.  Header-only and
// host-only, so tests/native/test_stage_plan.cpp checks it on the CPU.
#pragma once

#include <algorithm>
#include <cstddef>
#include <vector>

namespace shmx {

// n elements in chunks of `chunk` (a multiple of g, the elements in 16 B),
// the last one partial; with ramp and at least four full chunks' worth, the
// first two and the last two are a quarter and a half chunk instead, so the
// pipeline's fill and drain, which nothing overlaps, are short.  Every chunk
// but the last starts a multiple of g elements in (the odd elements go
// last).  The same inputs give the same schedule on every PE.
inline void stage_plan(size_t n, size_t chunk, size_t g, bool ramp, std::vector<size_t> &off,
                       std::vector<size_t> &cnt) {
    off.clear();
    cnt.clear();
    std::vector<size_t> head, tail;
    if (ramp && chunk >= g && n >= 4 * chunk) {
        const size_t q = std::max(g, (chunk / 4) / g * g), h = std::max(g, (chunk / 2) / g * g);
        head = {q, h};
        tail = {h, q};
    }
    size_t mid = n;
    for (size_t x : head) mid -= x;
    for (size_t x : tail) mid -= x;
    if (!tail.empty()) {
        tail.back() += mid % g;
        mid -= mid % g;
    }
    auto add = [&](size_t c) {
        off.push_back(off.empty() ? 0 : off.back() + cnt.back());
        cnt.push_back(c);
    };
    for (size_t x : head) add(x);
    for (size_t done = 0; done < mid; done += chunk) add(std::min(chunk, mid - done));
    for (size_t x : tail) add(x);
}

}  // namespace shmx
