// Host check of the GPU's x87 soft-float (openshmem-async_amd/csrc/ld80.h)
// against the host's real x87 unit: add, mul, <, > over random and special
// 80-bit encodings.  Prints "ok <count>" or the first mismatch and exits 1.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "ld80.h"

using shmx::x87::ld80;

static ld80 from_ld(long double v) {
    ld80 r;
    std::memset(&r, 0, sizeof r);
    std::memcpy(&r, &v, 10);
    return r;
}
static long double to_ld(const ld80 &x) {
    long double v = 0;
    std::memcpy(&v, &x, 10);
    return v;
}
static bool same10(const ld80 &a, const ld80 &b) { return a.sig == b.sig && a.se == b.se; }

static std::mt19937_64 rng(20251015);

static ld80 enc(bool neg, unsigned e, uint64_t s) { return shmx::x87::make(neg, e, s); }

static ld80 random_value(int cls) {
    const uint64_t r = rng(), r2 = rng();
    const bool neg = r2 & 1;
    switch (cls) {
    case 0:  // normal, any exponent
        return enc(neg, 1 + (unsigned)(r2 >> 1) % 0x7FFE, r | (1ull << 63));
    case 1:  // normal, exponent near 16383 (cancellation / rounding)
        return enc(neg, 16383 - 3 + (unsigned)(r2 >> 1) % 7, r | (1ull << 63));
    case 2:  // denormal
        return enc(neg, 0, r >> (1 + (r2 >> 1) % 63));
    case 3:  // pseudo-denormal
        return enc(neg, 0, r | (1ull << 63));
    case 4:  // near underflow boundary
        return enc(neg, 1 + (unsigned)(r2 >> 1) % 70, r | (1ull << 63));
    case 5:  // near overflow boundary
        return enc(neg, 0x7FFE - (unsigned)(r2 >> 1) % 70, r | (1ull << 63));
    case 6: {  // specials
        switch ((r2 >> 1) % 9) {
        case 0: return enc(neg, 0, 0);                                   // zero
        case 1: return enc(neg, 0x7FFF, 1ull << 63);                     // inf
        case 2: return enc(neg, 0x7FFF, (3ull << 62) | (r >> 2));        // qnan
        case 3: return enc(neg, 0x7FFF, (1ull << 63) | ((r >> 2) | 1));  // snan
        case 4: return enc(neg, 0x7FFF, r >> 1);                         // pseudo-nan/inf
        case 5: return enc(neg, 1 + (unsigned)(r2 >> 8) % 0x7FFE, r >> 1); // unnormal
        case 6: return enc(neg, 0x7FFE, ~0ull);                          // max
        case 7: return enc(neg, 1, 1ull << 63);                          // min normal
        default: return enc(neg, 0, 1);                                  // min denormal
        }
    }
    default:  // any 80-bit pattern
        return enc(neg, (unsigned)(r2 >> 1) & 0x7FFF, r);
    }
}

int main(int argc, char **argv) {
    const long iters = argc > 1 ? std::atol(argv[1]) : 2000000;
    long checked = 0;
    for (long i = 0; i < iters; ++i) {
        const int ca = (int)(rng() % 8), cb = (i & 3) == 0 ? ca : (int)(rng() % 8);
        ld80 a = random_value(ca), b = random_value(cb);
        if (ca == 1 && cb == 1 && (i & 1)) b.se = (uint16_t)(a.se ^ 0x8000);  // near-cancel
        if (i % 7 == 3) {
            // both normal, exponents 0..70 apart: every alignment the fast
            // add takes (64-bit words, the d = 64/65 sticky cases, d >= 66)
            a = random_value(0);
            const int ea = a.se & 0x7FFF, d = (int)(rng() % 71);
            const int eb = ea - d >= 1 ? ea - d : ea + d;
            b = enc(rng() & 1, (unsigned)(eb > 0x7FFE ? 0x7FFE : eb), rng() | (1ull << 63));
            if (rng() & 1) b.sig = a.sig ^ (rng() & 7);   // nearly equal significands
        }
        volatile long double x = to_ld(a), y = to_ld(b);
        const long double s = x + y, p = x * y;
        const bool lt = x < y, gt = x > y;
        const ld80 hs = from_ld(s), hp = from_ld(p);
        const ld80 gs = shmx::x87::add(a, b), gp = shmx::x87::mul(a, b);
        const bool glt = shmx::x87::less(a, b), ggt = shmx::x87::greater(a, b);
        if (!same10(hs, gs) || !same10(hp, gp) || lt != glt || gt != ggt) {
            std::printf("MISMATCH a=%04x:%016llx b=%04x:%016llx\n", a.se, (unsigned long long)a.sig,
                        b.se, (unsigned long long)b.sig);
            std::printf(" add x87 %04x:%016llx soft %04x:%016llx\n", hs.se, (unsigned long long)hs.sig,
                        gs.se, (unsigned long long)gs.sig);
            std::printf(" mul x87 %04x:%016llx soft %04x:%016llx\n", hp.se, (unsigned long long)hp.sig,
                        gp.se, (unsigned long long)gp.sig);
            std::printf(" lt %d/%d gt %d/%d\n", lt, glt, gt, ggt);
            return 1;
        }
        ++checked;
    }
    std::printf("ok %ld\n", checked);
    return 0;
}
