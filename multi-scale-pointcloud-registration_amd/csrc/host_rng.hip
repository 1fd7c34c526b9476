// Host-side replay of the reference's multistart RNG draws, and the rigid-image
// check of the drop-in path (host code only).
//
// Aligner.initialize_rotation (reference Aligner/Aligner.py:125-162) draws,
// per attempt, three np.random.uniform(-deg, deg) angles and one
// np.random.randn(3) from numpy's global legacy RandomState (MT19937).  The
// reference never seeds inside the library (Q7), so the build must consume
// that stream exactly as numpy does: every multistart of an align() advances
// it by `attempts` draws, in order.  Drawing them through numpy's Python API
// costs ~4.6 us per attempt (two calls); the speculative compass draws up to
// 13 blocks of 64 attempts before its first device batch, ~4 ms of host time
// on every rank.  This restates numpy's legacy generator in C++:
//   * MT19937 (numpy/random/src/mt19937: genrand with the 624-word state
//     reloaded when pos reaches 624),
//   * legacy_double: (a >> 5, b >> 6) -> (a * 67108864.0 + b) / 2^53,
//   * uniform(low, high) = low + (high - low) * legacy_double,
//   * legacy_gauss: the polar method with one cached deviate (has_gauss),
//     rejection while r2 >= 1 or r2 == 0, f = sqrt(-2 log(r2) / r2), the
//     cached value f * x1, the returned f * x2.
// The state goes in and out in numpy's get_state() layout, so the caller
// resumes the global RandomState exactly where the reference would leave it.
// Bit-identity with numpy is tested (tests/test_host.py) over many seeds and
// block sizes, including odd attempt counts (a cached gaussian across blocks).
#include <cmath>
#include <cstdint>
#include <limits>

#include "orpcd_internal.h"

#pragma clang fp contract(off)  // numpy's C: no fused multiply-adds

namespace {

struct Mt {
    uint32_t* key;  // 624 words (the caller's buffer, updated in place)
    int pos;
    int has_gauss;
    double gauss;

    void reload() {
        constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrix = 0x9908b0dfu;
        int i = 0;
        for (; i < 624 - 397; ++i) {
            const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + 397] ^ (y >> 1) ^ (-(y & 1u) & kMatrix);
        }
        for (; i < 623; ++i) {
            const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + (397 - 624)] ^ (y >> 1) ^ (-(y & 1u) & kMatrix);
        }
        const uint32_t y = (key[623] & kUpper) | (key[0] & kLower);
        key[623] = key[396] ^ (y >> 1) ^ (-(y & 1u) & kMatrix);
        pos = 0;
    }
    uint32_t next32() {
        if (pos == 624) reload();
        uint32_t y = key[pos++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    double next_double() {
        const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }
    double next_gauss() {
        if (has_gauss) {
            const double t = gauss;
            has_gauss = 0;
            gauss = 0.0;
            return t;
        }
        double f, x1, x2, r2;
        do {
            x1 = 2.0 * next_double() - 1.0;
            x2 = 2.0 * next_double() - 1.0;
            r2 = x1 * x1 + x2 * x2;
        } while (r2 >= 1.0 || r2 == 0.0);
        f = std::sqrt(-2.0 * std::log(r2) / r2);
        gauss = f * x1;
        has_gauss = 1;
        return f * x2;
    }
};

}  // namespace

extern "C" int orpcd_rng_draw_attempts(uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss, int64_t n,
                                       double low, double high, double* theta, double* normal) {
    if (!key || !pos || !has_gauss || !gauss || n < 0 || (n > 0 && (!theta || !normal))) return ORPCD_EINVAL;
    if (*pos < 0 || *pos > 624) return ORPCD_EINVAL;
    Mt mt{key, *pos, *has_gauss, *gauss};
    const double range = high - low;  // as numpy's uniform: low + (high - low) * u
    for (int64_t k = 0; k < n; ++k) {
        for (int j = 0; j < 3; ++j) theta[3 * k + j] = low + range * mt.next_double();
        for (int j = 0; j < 3; ++j) normal[3 * k + j] = mt.next_gauss();
    }
    *pos = mt.pos;
    *has_gauss = mt.has_gauss;
    *gauss = mt.gauss;
    return ORPCD_OK;
}

// The drop-in path's rigid-image check (GeneralizedICP._rigid_image and its
// speculated attempts, generalizedICP.py): out[0] = max over points and axes
// of |src - (base R + t)| (row vectors, R row-major), out[1] = max |src|.  One
// pass without temporaries: numpy's expression made four 1.2 MB temporaries
// per call at C2 (~0.7-2 ms of page faults and passes against ~50 us here).
extern "C" int orpcd_rigid_residual(const double* base, const double* src, int64_t n, const double* R,
                                    const double* t, double* out) {
    if (!base || !src || !R || !t || !out || n < 0) return ORPCD_EINVAL;
    double res = 0.0, mag = 0.0;
    bool nan = false;
    const double R0 = R[0], R1 = R[1], R2 = R[2], R3 = R[3], R4 = R[4], R5 = R[5], R6 = R[6], R7 = R[7], R8 = R[8];
    for (int64_t i = 0; i < n; ++i) {  // plain compares (vectorisable; fmax's NaN rules are not)
        const double* b = base + 3 * i;
        const double* s = src + 3 * i;
        const double d0 = std::fabs(s[0] - (b[0] * R0 + b[1] * R3 + b[2] * R6 + t[0]));
        const double d1 = std::fabs(s[1] - (b[0] * R1 + b[1] * R4 + b[2] * R7 + t[1]));
        const double d2 = std::fabs(s[2] - (b[0] * R2 + b[1] * R5 + b[2] * R8 + t[2]));
        const double dm = d0 > d1 ? (d0 > d2 ? d0 : d2) : (d1 > d2 ? d1 : d2);
        const double a0 = std::fabs(s[0]), a1 = std::fabs(s[1]), a2 = std::fabs(s[2]);
        const double am = a0 > a1 ? (a0 > a2 ? a0 : a2) : (a1 > a2 ? a1 : a2);
        res = dm > res ? dm : res;
        mag = am > mag ? am : mag;
        nan |= (d0 != d0) | (d1 != d1) | (d2 != d2);
    }
    if (nan) res = std::numeric_limits<double>::infinity();  // not an image
    out[0] = res;
    out[1] = mag;
    return ORPCD_OK;
}
