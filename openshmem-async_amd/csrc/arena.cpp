// First-fit allocator of the symmetric heap segment (heap.h).  Pure host
// code: the same call sequence gives the same offsets on every PE.
#include "heap.h"

#include <cctype>
#include <iterator>

namespace shmx {
namespace heap {

void Arena::reset(uint64_t capacity) {
    capacity_ = capacity / kGranule * kGranule;
    free_.clear();
    used_.clear();
    if (capacity_) free_[0] = capacity_;
}

uint64_t Arena::alloc(uint64_t bytes, uint64_t alignment) {
    if (bytes == 0 || (alignment & (alignment - 1))) return kNone;
    if (alignment < kGranule) alignment = kGranule;
    const uint64_t len = (bytes + kGranule - 1) / kGranule * kGranule;
    if (len < bytes) return kNone;   // overflow
    for (auto it = free_.begin(); it != free_.end(); ++it) {
        const uint64_t start = it->first, flen = it->second;
        const uint64_t user = (start + alignment - 1) & ~(alignment - 1);
        if (user < start || user - start > flen || flen - (user - start) < len) continue;
        free_.erase(it);
        if (user > start) free_[start] = user - start;       // leading gap stays free
        const uint64_t end = user + len, fend = start + flen;
        if (fend > end) free_[end] = fend - end;              // tail stays free
        used_[user] = Used{user, len, bytes};
        return user;
    }
    return kNone;
}

uint64_t Arena::size_of(uint64_t off) const {
    auto it = used_.find(off);
    return it == used_.end() ? 0 : it->second.bytes;
}

bool Arena::free(uint64_t off) {
    auto it = used_.find(off);
    if (it == used_.end()) return false;
    uint64_t start = it->second.start, len = it->second.len;
    used_.erase(it);
    // coalesce with the free neighbours on both sides
    auto next = free_.lower_bound(start);
    if (next != free_.end() && start + len == next->first) {
        len += next->second;
        next = free_.erase(next);
    }
    if (next != free_.begin()) {
        auto prev = std::prev(next);
        if (prev->first + prev->second == start) {
            start = prev->first;
            len += prev->second;
            free_.erase(prev);
        }
    }
    free_[start] = len;
    return true;
}

uint64_t Arena::free_bytes() const {
    uint64_t s = 0;
    for (const auto &f : free_) s += f.second;
    return s;
}

// utils/unitparse.c:102-135: digits, then an optional unit from "kmgtpe"
// (case-insensitive, powers of 1024).  Unlike the reference, an unknown unit
// or trailing characters are rejected rather than left unparsed.
bool parse_size(const char *s, uint64_t *bytes) {
    if (!s || !std::isdigit((unsigned char)*s)) return false;
    uint64_t v = 0;
    for (; std::isdigit((unsigned char)*s); ++s) {
        const uint64_t nv = v * 10 + (uint64_t)(*s - '0');
        if (nv / 10 != v) return false;
        v = nv;
    }
    if (*s) {
        static const char units[] = "kmgtpe";
        uint64_t mult = 1;
        const char u = (char)std::tolower((unsigned char)*s);
        bool found = false;
        for (const char *p = units; *p; ++p) {
            mult *= 1024;
            if (*p == u) {
                found = true;
                break;
            }
        }
        if (!found || s[1] != '\0') return false;
        if (v && mult > ~uint64_t(0) / v) return false;
        v *= mult;
    }
    *bytes = v;
    return true;
}

}  // namespace heap
}  // namespace shmx
