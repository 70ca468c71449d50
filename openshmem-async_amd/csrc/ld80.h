// x87 80-bit extended precision ("long double" on x86-64 Linux) in software,
// for the GPU: the arithmetic of shmem_longdouble_{sum,prod,min,max}_to_all
// (reference reduce-op.c:91,150: a+b, a*b, a<b?a:b, a>b?a:b on x87).
//
// The GPU has no 80-bit format, so each op is computed exactly in 128-bit
// integer arithmetic and rounded once, reproducing what the host's x87 unit
// returns with the Linux default control word (64-bit precision, round to
// nearest even, all exceptions masked):
//   * IEEE-style rounding of the exact result to a 64-bit significand, with
//     gradual underflow to the x87 denormal format and overflow to +-inf;
//   * x87 NaN rules (Intel SDM vol. 1, "Rules for handling NaNs"): a NaN
//     operand is returned quieted; with two NaNs the quiet one wins over a
//     signalling one, otherwise the one with the larger significand (on a
//     tie the positive one, as measured on the host x87);
//   * invalid operations (inf - inf, 0 * inf) and unsupported encodings
//     (pseudo-NaN, pseudo-infinity, unnormal) give the "real indefinite" QNaN
//     (sign 1, exponent 0x7FFF, significand 0xC000000000000000);
//   * pseudo-denormals (exponent 0, integer bit 1) are read as exponent 1;
//   * a<b / a>b are the unordered-false comparisons gcc emits (fucomip), with
//     -0 == +0; unsupported encodings compare unordered.
// Storage is the host's 16-byte slot: 8 significand bytes, 2 sign/exponent
// bytes, 6 padding bytes (written as zero).
//
// Plain C++ with SHMX_HD on every function, so the same code is compiled for
// gfx950 and, in tests, for the host where it is checked against real x87.
#pragma once

#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#define SHMX_HD __host__ __device__ __forceinline__
#else
#define SHMX_HD inline
#endif

namespace shmx {
namespace x87 {

struct ld80 {
    uint64_t sig;   // explicit integer bit at 63
    uint16_t se;    // sign (bit 15) | biased exponent (bits 0-14)
    uint16_t pad[3];
};
static_assert(sizeof(ld80) == 16, "host long double slot is 16 bytes");

typedef unsigned __int128 u128;

constexpr int kBias = 16383;
constexpr int kEmin = 1 - kBias;       // exponent of the smallest normal
constexpr int kEmax = 0x7FFE - kBias;  // exponent of the largest finite
constexpr uint64_t kInt = 1ull << 63;  // integer bit
constexpr uint64_t kQuiet = 1ull << 62;

SHMX_HD ld80 make(bool neg, unsigned e, uint64_t s) {
    ld80 r;
    r.sig = s;
    r.se = (uint16_t)((neg ? 0x8000u : 0u) | (e & 0x7FFFu));
    r.pad[0] = r.pad[1] = r.pad[2] = 0;
    return r;
}
SHMX_HD bool sign_of(const ld80 &x) { return (x.se >> 15) != 0; }
SHMX_HD unsigned exp_of(const ld80 &x) { return x.se & 0x7FFFu; }
SHMX_HD ld80 indefinite() { return make(true, 0x7FFF, 0xC000000000000000ull); }

// unsupported encodings: pseudo-NaN/pseudo-inf (exp 0x7FFF, integer bit 0)
// and unnormals (0 < exp < 0x7FFF, integer bit 0)
SHMX_HD bool unsupported(const ld80 &x) {
    const unsigned e = exp_of(x);
    return e != 0 && (x.sig & kInt) == 0;
}
SHMX_HD bool is_nan(const ld80 &x) {
    return exp_of(x) == 0x7FFF && (x.sig & kInt) && (x.sig << 1) != 0;
}
SHMX_HD bool is_snan(const ld80 &x) { return is_nan(x) && !(x.sig & kQuiet); }
SHMX_HD bool is_inf(const ld80 &x) { return exp_of(x) == 0x7FFF && x.sig == kInt; }
SHMX_HD bool is_zero(const ld80 &x) { return exp_of(x) == 0 && x.sig == 0; }

SHMX_HD int clz64(uint64_t v) { return v ? __builtin_clzll(v) : 64; }
SHMX_HD int clz128(u128 v) {
    const uint64_t hi = (uint64_t)(v >> 64);
    return hi ? __builtin_clzll(hi) : 64 + clz64((uint64_t)v);
}

// The NaN an x87 add/mul returns when at least one operand is a NaN.
SHMX_HD ld80 nan_result(const ld80 &a, const ld80 &b) {
    const bool an = is_nan(a), bn = is_nan(b);
    ld80 r;
    if (an && bn) {
        const bool as = is_snan(a), bs = is_snan(b);
        if (as != bs) r = as ? b : a;                 // the quiet one
        else if (a.sig != b.sig) r = (b.sig > a.sig) ? b : a;  // larger significand
        else r = sign_of(a) ? b : a;                  // tie: the positive one (measured)
    } else {
        r = an ? a : b;
    }
    return make(sign_of(r), 0x7FFF, r.sig | kQuiet);
}

// Finite non-zero operand as value = m * 2^(E - 63), m with bit 63 set.
SHMX_HD void unpack(const ld80 &x, int &E, uint64_t &m) {
    const unsigned e = exp_of(x);
    E = (int)(e ? e : 1) - kBias;
    m = x.sig;
    const int lz = clz64(m);
    m <<= lz;
    E -= lz;
}

// Round value = m * 2^(E - 127) (bit 127 of m set, or m == 0 with sticky)
// plus a sticky remainder, to the x87 format, round to nearest even.
SHMX_HD ld80 round_pack(bool neg, int E, u128 m, bool sticky) {
    if (E < kEmin) {  // gradual underflow: denormalise before rounding
        const int sh = kEmin - E;
        if (sh >= 128) {
            sticky = sticky || m != 0;
            m = 0;
        } else {
            sticky = sticky || (m & ((((u128)1) << sh) - 1)) != 0;
            m >>= sh;
        }
        E = kEmin;
    }
    uint64_t sig = (uint64_t)(m >> 64);
    const uint64_t rest = (uint64_t)m;
    const bool rnd = (rest >> 63) != 0;
    const bool st = sticky || (rest << 1) != 0;
    if (rnd && (st || (sig & 1))) {
        ++sig;
        if (sig == 0) {  // carried out of the significand
            sig = kInt;
            ++E;
        }
    }
    if (E > kEmax) return make(neg, 0x7FFF, kInt);  // overflow -> inf
    if (sig & kInt) return make(neg, (unsigned)(E + kBias), sig);
    return make(neg, 0, sig);  // denormal or zero
}

// Fast path of add for the common case: both operands normal (exponent
// 1..0x7FFE, integer bit set) and a normal result.  64-bit words instead of
// the general path's 128-bit shifts: the significand of |b| aligned to |a|'s
// is split into the word beside a's (bh) and the word of bits shifted out
// below it (bl), plus one sticky bit (d == 65).  Returns false, without
// touching r, whenever the general path is needed (specials, denormals,
// over/underflow).
SHMX_HD bool add_fast(const ld80 &a, const ld80 &b, ld80 &r) {
    unsigned ea = exp_of(a), eb = exp_of(b);
    if (ea - 1u >= 0x7FFEu || eb - 1u >= 0x7FFEu || !(a.sig & b.sig & kInt)) return false;
    bool sa = sign_of(a), sb = sign_of(b);
    uint64_t ma = a.sig, mb = b.sig;
    if (ea < eb || (ea == eb && ma < mb)) {  // |a| >= |b| from here on
        const unsigned te = ea; ea = eb; eb = te;
        const uint64_t tm = ma; ma = mb; mb = tm;
        const bool ts = sa; sa = sb; sb = ts;
    }
    const unsigned d = ea - eb;
    if (d >= 66) {  // |b| < a quarter ulp of |a|: a itself, either sign
        r = make(sa, ea, ma);
        return true;
    }
    uint64_t bh, bl;
    bool st = false;
    if (d == 0) {
        bh = mb;
        bl = 0;
    } else if (d < 64) {
        bh = mb >> d;
        bl = mb << (64 - d);
    } else {
        bh = 0;
        bl = d == 64 ? mb : mb >> 1;
        st = d == 65 && (mb & 1);
    }
    uint64_t sig, rest;
    unsigned e = ea;
    if (sa == sb) {
        const uint64_t sum = ma + bh;
        if (sum < ma) {  // carry: one more bit above
            sig = (sum >> 1) | kInt;
            rest = (sum << 63) | (bl >> 1);
            st = st || (bl & 1);
            ++e;
        } else {
            sig = sum;
            rest = bl;
        }
    } else {
        // (ma:0) - (bh:bl) - sticky: the value lies in (r, r + 1) when sticky
        uint64_t lo = 0 - bl;
        uint64_t hi = ma - bh - (bl != 0 ? 1 : 0);
        if (st) {
            hi -= lo == 0 ? 1 : 0;
            lo -= 1;
        }
        if (hi == 0 && lo == 0 && !st) {  // exact cancellation: +0
            r = make(false, 0, 0);
            return true;
        }
        if (hi == 0) {  // only when d <= 1: exact, nothing below lo
            const int l = clz64(lo);
            if ((int)e - 64 - l < 1) return false;
            r = make(sa, e - 64 - (unsigned)l, lo << l);
            return true;
        }
        const int l = clz64(hi);
        if (l) {
            sig = (hi << l) | (lo >> (64 - l));
            rest = lo << l;
            if ((int)e - l < 1) return false;
            e -= (unsigned)l;
        } else {
            sig = hi;
            rest = lo;
        }
    }
    // round to nearest even on the guard bit (rest's top), sticky below it
    if ((rest >> 63) && (st || (rest << 1) != 0 || (sig & 1))) {
        if (++sig == 0) {
            sig = kInt;
            ++e;
        }
    }
    if (e > 0x7FFEu) return false;  // overflow: the general path returns inf
    r = make(sa, e, sig);
    return true;
}

SHMX_HD ld80 add(const ld80 &a, const ld80 &b) {
    ld80 fast;
    if (add_fast(a, b, fast)) return fast;
    if (unsupported(a) || unsupported(b)) return indefinite();
    if (is_nan(a) || is_nan(b)) return nan_result(a, b);
    const bool sa = sign_of(a), sb = sign_of(b);
    if (is_inf(a) || is_inf(b)) {
        if (is_inf(a) && is_inf(b)) return sa == sb ? a : indefinite();
        return is_inf(a) ? a : b;
    }
    const bool za = is_zero(a), zb = is_zero(b);
    if (za && zb) return make(sa && sb, 0, 0);
    if (za || zb) {  // x + 0: x, re-encoded (pseudo-denormals normalise)
        const ld80 &x = za ? b : a;
        int E;
        uint64_t m;
        unpack(x, E, m);
        return round_pack(sign_of(x), E, ((u128)m) << 64, false);
    }
    int Ea, Eb;
    uint64_t ma, mb;
    unpack(a, Ea, ma);
    unpack(b, Eb, mb);
    bool neg = sa;
    if (Ea < Eb || (Ea == Eb && ma < mb)) {  // |a| >= |b| from here on
        int te = Ea; Ea = Eb; Eb = te;
        uint64_t tm = ma; ma = mb; mb = tm;
        neg = sb;
    }
    const u128 ua = ((u128)ma) << 63;  // leading bit at 126 = 2^Ea
    u128 ub = ((u128)mb) << 63;
    const int d = Ea - Eb;
    bool sticky = false;
    if (d >= 127) {
        sticky = ub != 0;
        ub = 0;
    } else if (d > 0) {
        sticky = (ub & ((((u128)1) << d) - 1)) != 0;
        ub >>= d;
    }
    u128 r;
    if (sa == sb) {
        r = ua + ub;
    } else {
        r = ua - ub - (sticky ? 1 : 0);  // value in (r, r+1) when sticky
        if (r == 0 && !sticky) return make(false, 0, 0);  // exact cancel: +0
    }
    const int L = 127 - clz128(r);
    return round_pack(neg, Ea + (L - 126), r << (127 - L), sticky);
}

// Fast path of mul: both operands normal and a normal result (64x64 ->
// 128-bit product, one normalising shift, one rounding).
SHMX_HD bool mul_fast(const ld80 &a, const ld80 &b, ld80 &r) {
    const unsigned ea = exp_of(a), eb = exp_of(b);
    if (ea - 1u >= 0x7FFEu || eb - 1u >= 0x7FFEu || !(a.sig & b.sig & kInt)) return false;
    const u128 p = ((u128)a.sig) * b.sig;  // leading bit at 126 or 127
    uint64_t hi = (uint64_t)(p >> 64), lo = (uint64_t)p;
    int e = (int)ea + (int)eb - kBias + 1;
    if (!(hi >> 63)) {
        hi = (hi << 1) | (lo >> 63);
        lo <<= 1;
        --e;
    }
    if ((lo >> 63) && ((lo << 1) != 0 || (hi & 1))) {
        if (++hi == 0) {
            hi = kInt;
            ++e;
        }
    }
    if (e < 1 || e > 0x7FFE) return false;
    r = make(sign_of(a) != sign_of(b), (unsigned)e, hi);
    return true;
}

SHMX_HD ld80 mul(const ld80 &a, const ld80 &b) {
    ld80 fast;
    if (mul_fast(a, b, fast)) return fast;
    if (unsupported(a) || unsupported(b)) return indefinite();
    if (is_nan(a) || is_nan(b)) return nan_result(a, b);
    const bool neg = sign_of(a) != sign_of(b);
    const bool ia = is_inf(a), ib = is_inf(b), za = is_zero(a), zb = is_zero(b);
    if (ia || ib) {
        if (za || zb) return indefinite();
        return make(neg, 0x7FFF, kInt);
    }
    if (za || zb) return make(neg, 0, 0);
    int Ea, Eb;
    uint64_t ma, mb;
    unpack(a, Ea, ma);
    unpack(b, Eb, mb);
    const u128 p = ((u128)ma) * mb;  // leading bit at 126 or 127
    const int L = 127 - clz128(p);
    return round_pack(neg, Ea + Eb - 126 + L, p << (127 - L), false);
}

// Ordered comparison key: |x| as (E, significand) on one scale.
SHMX_HD bool less(const ld80 &a, const ld80 &b) {
    if (unsupported(a) || unsupported(b) || is_nan(a) || is_nan(b)) return false;
    const bool za = (a.sig == 0 && exp_of(a) == 0), zb = (b.sig == 0 && exp_of(b) == 0);
    if (za && zb) return false;  // -0 == +0
    const bool sa = sign_of(a) && !za, sb = sign_of(b) && !zb;
    if (sa != sb) return sa;     // negative < positive
    const unsigned ea = exp_of(a) ? exp_of(a) : 1, eb = exp_of(b) ? exp_of(b) : 1;
    const bool mag_less = (ea < eb) || (ea == eb && a.sig < b.sig);
    const bool mag_eq = ea == eb && a.sig == b.sig;
    if (mag_eq) return false;
    return sa ? !mag_less : mag_less;
}
SHMX_HD bool greater(const ld80 &a, const ld80 &b) { return less(b, a); }

}  // namespace x87
}  // namespace shmx
