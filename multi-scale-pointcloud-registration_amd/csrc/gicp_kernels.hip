// gicp_kernels.hip — the GICP inner loop on gfx950, batched over starts.
//
// One correspondence pass restates, for every running start at once,
//   O3D Registration.cpp GetRegistrationResultAndCorrespondences
//     (SearchHybrid(max_corr, 1): exact nearest target with d^2 < r^2)
// and
//   O3D GeneralizedICP.cpp TransformationEstimationForGeneralizedICP::
//     ComputeTransformation (JTJ / JTr with W = (Cs + Ct)^-1/2, L2 kernel).
// The solve kernel restates SolveJacobianSystemAndObtainExtrinsicMatrix and
// the RegistrationICP convergence test, per start, on device.
// Reference call site: generalizedICP.py:59-70, driven by Aligner.py:178-202.
//
// A pass is:
//  * nn_search_kernel (fp32, low VGPR, 8 waves/SIMD): every wave owns 128
//    Morton-consecutive queries (2 per lane) of one start.  Target tiles (64
//    Morton-consecutive points with an AABB) are culled first against the
//    wave's query AABB and worst bound (lane-parallel, 64 tiles per ballot),
//    then against each query's own bound; surviving tiles are staged into the
//    wave's LDS slot by one coalesced 1 KiB load (the next candidate's load is
//    in flight while the current tile is scanned) and scanned with packed fp32
//    math: per target and lane-pair of queries 6 v_pk ops for the two d^2, then
//    the key (d^2 bits with the low 6 bits replaced by the tile-local index)
//    enters a v_min3_u32 running minimum, so one integer min selects distance
//    AND index.  Candidates whose d^2 agree in the top 26 bits (2^-17 relative)
//    resolve to the lower Morton position; across tiles the earlier tile wins a
//    tie (exact duplicates keep the lowest input index: the Morton sort is
//    stable).  Each query's bound is seeded by the start's correspondence of
//    the previous pass, or on pass 0 by strided tile representatives (real
//    targets, so the bound is valid); the seed only bounds the scan.  When few
//    starts run, a query group's tiles are split over S waves whose results
//    merge by a 64-bit atomicMin on (d^2 bits, target index).
//  * gicp_accum_kernel (fp64): re-evaluates the chosen pair in fp64 (strict
//    radius test, d^2, Jacobian) and reduces the 29 normal-equation terms per
//    block in a fixed order.  Because W is symmetric, J^T J = A^T (Cs+Ct)^-1 A
//    and J^T r = A^T (Cs+Ct)^-1 d with A = [-[q]x | I]: no matrix square root
//    is needed.
//  * icp_solve_kernel: per start, fixed-order reduction, convergence test,
//    6x6 LDLT solve and pose update; then xform_queries_kernel writes the fp32
//    queries of the next pass (fp64 transform, one rounding).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "device_math.h"
#include "orpcd_internal.h"
#include "wave_ops.h"

// Issue priority of a search wave outside its tile scans (s_setprio): the
// culling chain (dependent box loads, ballots) outranks the VALU-heavy scans
// of the other waves on its SIMD.  3 measured: 8 starts 4.63 -> 4.50 ms, 64
// starts 24.45 -> 24.02 ms, 1 / 16 / 30 starts equal; bit-identical.  0: off.
#ifndef ORPCD_CULL_PRIO
#define ORPCD_CULL_PRIO 3
#endif

namespace orpcd {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// fp32 squared distance (seed evaluation)
__device__ __forceinline__ float d2f(float qx, float qy, float qz, float4 t) {
    const float dx = qx - t.x, dy = qy - t.y, dz = qz - t.z;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

__device__ __forceinline__ float box_d2(float x, float y, float z, float lx, float ly, float lz, float hx, float hy,
                                        float hz) {
    const float dx = fmaxf(0.0f, fmaxf(lx - x, x - hx));
    const float dy = fmaxf(0.0f, fmaxf(ly - y, y - hy));
    const float dz = fmaxf(0.0f, fmaxf(lz - z, z - hz));
    return dx * dx + dy * dy + dz * dz;
}

// box d^2 of a lane's two queries (packed: x = query 0, y = query 1) in the
// scan's own operation order, fma(dz, dz, fma(dy, dy, dx * dx)): each axis
// distance is <= |q - t| for every point t of the box and fp32 rounding and fma
// are monotone, so the result never exceeds the scan's d^2 of a point inside.
// The axis distance is q - med3(q, lo, hi): the clamp is exact and fp32
// subtraction is sign-symmetric, so it is the same value as max(lo - q,
// q - hi, 0) in 3 VALU per axis and query pair instead of 5 (bit-identical
// culling; an empty box is stored as the point (3e38, 3e38, 3e38), see
// tile_aabb_kernel, whose distance overflows to inf).
__device__ __forceinline__ f2 box_d2_2q(f2 qx, f2 qy, f2 qz, float lx, float ly, float lz, float hx, float hy,
                                        float hz) {
    const f2 cx = {__builtin_amdgcn_fmed3f(qx.x, lx, hx), __builtin_amdgcn_fmed3f(qx.y, lx, hx)};
    const f2 cy = {__builtin_amdgcn_fmed3f(qy.x, ly, hy), __builtin_amdgcn_fmed3f(qy.y, ly, hy)};
    const f2 cz = {__builtin_amdgcn_fmed3f(qz.x, lz, hz), __builtin_amdgcn_fmed3f(qz.y, lz, hz)};
    const f2 dx = qx - cx, dy = qy - cy, dz = qz - cz;
    f2 d = dx * dx;
    d = pk_fma(dy, dy, d);
    return pk_fma(dz, dz, d);
}

constexpr unsigned long long kNone = ~0ull;
constexpr int kNoSeed = -1;   // prevnn before the first pass (representative seed)
constexpr int kNoMatch = -2;  // no target within the search radius last pass
constexpr unsigned kKeyMask = 0xFFFFFFC0u;  // d^2 bits kept in a scan key (low 6 = tile-local index)
// quarter test: box d^2 < bound x (1 + 2^-19), i.e. box d^2 x (1 - 2^-20) <
// bound with the factor moved onto the bound (b (1 + 2^-19) rounded to fp32
// is >= b / (1 - 2^-20), so every quarter the round-3 form scanned is still
// scanned; a few more may be, which cannot change a result: their keys lie
// above the bound).  Exact mode widens the band once per improving tile
// instead of multiplying every box d^2.
constexpr float kQuarterWiden = 1.0f + 1.0f / 524288.0f;

// A load through a pointer the compiler cannot prove global (one read from a
// TargetDesc): as a global load, not a flat one -- flat loads count against
// both vmcnt and lgkmcnt, so every later wait drained all of them.
__device__ __forceinline__ double ldg_f64(const double* p) {
    return *(const __attribute__((address_space(1))) double*)p;
}
__device__ __forceinline__ float4 ldg_f4(const float4* p) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    const v4 v = *(const __attribute__((address_space(1))) v4*)p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float ldg_f32(const float* p) {
    return *(const __attribute__((address_space(1))) float*)p;
}

// ---------------------------------------------------------------------------
// Exact nearest neighbour (opt.exact_nn).  The fp32 search orders candidates
// by d32, which differs from the oracle's fp64 distance d64 (KD-tree, the
// lexicographic (d64^2, input index) minimum) by at most
//     |d32 - d64| <= delta = u (2A + 3.5 d) (1 + 3u),  u = 2^-24,
// A = |q32| (the query in the target's fp32 frame): the fp32 roundings of the
// query and target coordinates (u |q32| + u |t32|, |t32| <= A + d), the
// subtraction (u d) and the three roundings of the squared sum (1.5 u d).
// If the exact winner t* differs from the fp32 winner j, then d32(t*) <=
// d64(t*) + delta <= d64(j) + delta <= d32(j) + 2 delta: its key is at most
// band_hi(key(j)).  The search therefore finds every query's runner-up key
// (in-scan, and across the splits of a query group: the loser of every
// atomicMin merge); a query whose runner-up lies within the band of its
// winner is filed for an fp64 re-search (nn_exact_kernel), every other
// query's fp32 winner is provably the fp64 one.  band_hi adds 1% on delta,
// the key truncation (2^-17 relative on the winner's d^2) and 2^-19 for its
// own fp32 rounding.
// ---------------------------------------------------------------------------
// exact mode's search: 5 waves/SIMD with the pipelined scan (ORPCD_PIPE_EXACT:
// one pair read ahead, no deeper hoisting; 94 VGPRs).  C2 batches of 30 / 8
// starts: 19.79 / 8.70 ms at 4 waves/SIMD with the compiler's scan schedule
// (116 VGPRs; at 5 waves it spilled 17), 19.52 / 8.49 ms like this (hashes
// equal).  The fast search gains nothing from it (14.9 / 4.5 ms either way,
// also at 6 waves).
#ifndef ORPCD_SCAN_UNROLL_EXACT
#define ORPCD_SCAN_UNROLL_EXACT 8
#endif
#ifndef ORPCD_SCAN_UNROLL_FAST
#define ORPCD_SCAN_UNROLL_FAST 8
#endif
#ifndef ORPCD_EXACT_WAVES
#define ORPCD_EXACT_WAVES 5
#endif
#ifndef ORPCD_FAST_WAVES
#define ORPCD_FAST_WAVES 5
#endif
#ifndef ORPCD_PIPE_EXACT
#define ORPCD_PIPE_EXACT 1
#endif
#ifndef ORPCD_PIPE_FAST
#define ORPCD_PIPE_FAST 0
#endif
constexpr float kU = 5.9604645e-08f;  // 2^-24
__device__ __forceinline__ float exact_band_hi(float x, float A) {
#pragma clang fp contract(off)  // identical rounding in the query transform and the search
    // v_sqrt_f32 (1 ulp), not the correctly rounded expansion (~20 VALU): the
    // final 2^-19 margin covers this function's rounding (~7 ulp with it)
    const float d = __builtin_amdgcn_sqrtf(x * 1.0000080f);  // x (1 + 2^-17 + margin): the masked key's upper end
    const float dl = kU * (4.04f * A + 7.07f * d);      // 2 delta (+1%)
    const float r = d + dl;
    return r * r * 1.0000020f;  // (1 + 2^-19): this function's own fp32 rounding
}
__device__ __forceinline__ float qnorm(float x, float y, float z) {
#pragma clang fp contract(off)
    return __builtin_amdgcn_sqrtf(x * x + y * y + z * z) * 1.0000005f;  // 1-ulp sqrt inside the 8-ulp margin
}
// sentinel bound of a query in exact mode: strictly above band_hi of every
// key below the plain bound, so a runner-up can never be the sentinel
__device__ __forceinline__ float exact_sentinel(float bound, float A) {
#pragma clang fp contract(off)
    return exact_band_hi(bound, A) * 1.00003f + 1e-30f;  // > 2^-17: survives the key mask
}
__device__ __forceinline__ unsigned umed3(unsigned a, unsigned b, unsigned c) {
    return max(min(a, b), min(max(a, b), c));  // v_med3_u32
}
// v_min3_u32 (the compiler forms it from nested mins only sometimes)
__device__ __forceinline__ unsigned umin3(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
struct ExactArgs {
    unsigned* sec;                // B x N: runner-up key near the winner (0xFFFFFFFF: none; reset by the transform)
    unsigned long long* list;     // queries with a near runner-up: slot << 40 | target << 32 | query
    unsigned* cnt;                // entries of this pass's list (by pass parity)
    unsigned* cnt_next;           // the next pass's (zeroed by nn_exact_kernel)
    unsigned long long* total;    // queries re-searched (statistics)
};

// --------------------------------------------------------------------------
// Culled exact nearest search for the 2 queries of every lane of one wave,
// restricted to tiles t with t % S == s.  s0lo/s0hi: super-tile `lane`'s box
// (loaded early by the caller; any value when lane >= nsuper).  bound[] enters as the per-query
// bound on d^2 (<= 0: invalid query).  Returns quarters scanned; bj[] = Morton
// index of the chosen target or -1, bd[] its fp32 d^2 (key-truncated).
// --------------------------------------------------------------------------
// kExact: the bound is the exact-mode sentinel, candidates are culled against
// band_hi of the query's best key (see exact_band_hi), the in-scan minimum runs over the query's
// whole search (tie order among equal masked keys is then immaterial: such
// keys are within the band and re-searched in fp64), and sk[] returns the
// second-smallest key scanned (0xFFFFFFFF: none).
template <bool kGBox, bool kExact = false>
__device__ __forceinline__ int culled_search(float4* stage, const float4* __restrict__ p4,
                                             const float4* __restrict__ tlo, const float4* __restrict__ thi,
                                             const float4* __restrict__ qbox, int ntiles, const float4* __restrict__ slo,
                                             const float4* __restrict__ shi, int nsuper, int super_cull, int S, int s,
                                             const float qx[2], const float qy[2],
                                             const float qz[2], const float bound[2], float bd[2], int bj[2],
                                             float4 s0lo, float4 s0hi, const float4* gbox = nullptr,
                                             unsigned long long* phase_cull_out = nullptr,
                                             unsigned* sk = nullptr) {
    constexpr int kScanUnroll = kExact ? ORPCD_SCAN_UNROLL_EXACT : ORPCD_SCAN_UNROLL_FAST;
    // kPipe: the scan reads each target pair one iteration ahead and the
    // compiler may not hoist more (a scheduling barrier per iteration): left
    // to itself it issues a whole quarter's LDS reads up front, which holds
    // ~20 more VGPRs than the scan needs
    constexpr bool kPipe = kExact ? ORPCD_PIPE_EXACT : ORPCD_PIPE_FAST;
    const int lane = threadIdx.x & 63;
#if ORPCD_CULL_PRIO > 0
    __builtin_amdgcn_s_setprio(ORPCD_CULL_PRIO);  // culling at raised issue priority
#endif
    const bool v0 = bound[0] > 0.0f, v1 = bound[1] > 0.0f;
    unsigned k0 = v0 ? __float_as_uint(bound[0]) : 0u;  // best key (0: never improves)
    unsigned k1 = v1 ? __float_as_uint(bound[1]) : 0u;
    int t0 = -1, t1 = -1;                               // tile of the best key
    unsigned s0 = 0xFFFFFFFFu, s1 = 0xFFFFFFFFu;        // exact: second-smallest key
    bj[0] = bj[1] = -1;
    bd[0] = bd[1] = 0.0f;
    const float inf = 3.0e38f;
    // the wave's query box and worst bound: given by the query transform
    // (gbox: lo.xyz | max bound bits, hi.xyz), else reduced here
    unsigned Wk;
    float lox, loy, loz, hix, hiy, hiz;
    // exact: each query's culling bound, band_hi of its best key (the sentinel
    // before it has one): every candidate within the band is scanned
    float e0 = kExact && v0 ? bound[0] : 0.0f, e1 = kExact && v1 ? bound[1] : 0.0f;
    f2 ew = f2{e0, e1} * f2{kQuarterWiden, kQuarterWiden};  // exact: the quarter tests' bounds
    if constexpr (kGBox) {
        const float4 g0 = gbox[0], g1 = gbox[1];
        // wave-uniform: scalar registers (the record is one address for every lane)
        auto sc = [](float f) { return __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(f))); };
        Wk = __builtin_amdgcn_readfirstlane(__float_as_uint(g0.w)) & kKeyMask;
        lox = sc(g0.x), loy = sc(g0.y), loz = sc(g0.z), hix = sc(g1.x), hiy = sc(g1.y), hiz = sc(g1.z);
    } else {
        static_assert(kGBox || !kExact, "exact mode needs the transform's wave boxes");
        Wk = wave_umax((k0 > k1 ? k0 : k1) & kKeyMask);
        lox = wave_fmin(fminf(v0 ? qx[0] : inf, v1 ? qx[1] : inf));
        loy = wave_fmin(fminf(v0 ? qy[0] : inf, v1 ? qy[1] : inf));
        loz = wave_fmin(fminf(v0 ? qz[0] : inf, v1 ? qz[1] : inf));
        hix = wave_fmax(fmaxf(v0 ? qx[0] : -inf, v1 ? qx[1] : -inf));
        hiy = wave_fmax(fmaxf(v0 ? qy[0] : -inf, v1 ? qy[1] : -inf));
        hiz = wave_fmax(fmaxf(v0 ? qz[0] : -inf, v1 ? qz[1] : -inf));
    }
    if (Wk == 0u) return 0;  // no query of this wave can take anything
    float W = __uint_as_float(Wk);
    int visited = 0;

    // candidate cursor: rounds of 64 tiles, one tile per lane; wave-box test by
    // ballot, then the per-query test for each set bit.
    // Two levels: super-tiles (64 tiles each) are tested 64 at a time against
    // the wave box; the 64 tiles of each surviving super-tile form one round.
    int sb = -64;                  // super-tile round base
    unsigned long long smask = 0;  // surviving super-tiles of that round
    unsigned long long mask = 0;
    float lb = inf;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
#ifdef ORPCD_PHASES
    unsigned long long ph_cull = 0, ph_rounds = 0, ph_tests = 0, ph_impr = 0, ph_need = 0, ph_staged = 0;
#endif
    // the tile AABBs of the NEXT round are loaded while the current round is
    // tested and scanned (one round of load latency hidden).  A round holds
    // this split's tiles of up to P surviving super-tiles, packed over the
    // lanes: split s owns tiles s, s+S, ... of each super-tile (per of them),
    // so with S splits one round covers P = 64/per super-tiles instead of one
    // (S = 1: one super-tile, one tile per lane).  Lanes follow increasing
    // tile order, so candidates are visited in the same order as before.
    const int per = S == 1 ? kSuper : (kSuper - s + S - 1) / S;
    // k / per for k < 64 as (k * perM) >> 16, exact for per <= 64: scalar
    // integer ops per candidate instead of the VALU division expansion
    const unsigned perM = __builtin_amdgcn_readfirstlane((65536u + (unsigned)per - 1u) / (unsigned)per);
    const int P = kSuper / per;
    bool haven = false;  // a prefetched round exists
    // the prefetched round's super-tile base and surviving mask before it was
    // consumed (scalar): lanes recompute their tile from them at the switch
    // instead of holding it in a VGPR through the scan
    int nsb = 0;
    unsigned long long nmask = 0;
    auto lane_tile = [&](int base, unsigned long long m) -> int {
        const int lr = (int)(((unsigned)lane * perM) >> 16), lm = lane - lr * per;  // lane -> (super-tile of the round, tile of it)
        int su = -1;
        for (int r = 0; r < P && m; ++r) {  // the next P surviving super-tiles (scalar)
            const int st = base + __builtin_ctzll(m);
            m &= m - 1;
            if (lr == r) su = st;
        }
        const int tin = S == 1 ? lm : s + S * lm;  // tile within the super-tile
        const int t = su * kSuper + tin;
        return su >= 0 && tin < kSuper && t < ntiles ? t : -1;
    };
    float4 an = a, bn = b;
    auto prefetch_round = [&]() {
        while (smask == 0) {
            sb += 64;
            if (sb >= nsuper) {
                haven = false;
                return;
            }
            const int u = sb + lane;
            float sl = inf;
            if (u < nsuper && !super_cull) {
                sl = 0.0f;
            } else if (u < nsuper) {
                // the first round's super-tile boxes were loaded by the caller
                // together with its queries (no query dependence)
                const float4 c = sb == 0 ? s0lo : slo[u], d = sb == 0 ? s0hi : shi[u];
                const float dx = fmaxf(0.0f, fmaxf(c.x - hix, lox - d.x));
                const float dy = fmaxf(0.0f, fmaxf(c.y - hiy, loy - d.y));
                const float dz = fmaxf(0.0f, fmaxf(c.z - hiz, loz - d.z));
                sl = dx * dx + dy * dy + dz * dz;
            }
            smask = __ballot(sl < W);
        }
        haven = true;
        nsb = sb;
        nmask = smask;
        const int t = lane_tile(sb, smask);
        for (int r = 0; r < P && smask; ++r) smask &= smask - 1;  // those super-tiles are taken
        if (t >= 0) {
            an = tlo[t];
            bn = thi[t];
        } else {
            an = make_float4(inf, inf, inf, 0.f);  // empty box: never within the bound
            bn = make_float4(-inf, -inf, -inf, 0.f);
        }
    };
    prefetch_round();
    int csb = 0;                  // the current round's super-tile base and mask (scalar)
    unsigned long long cmask = 0;
    auto next_candidate_impl = [&](float& lbk) -> int {
        for (;;) {
            while (mask == 0) {
                if (!haven) return -1;
                csb = nsb;
                cmask = nmask;
                a = an;
                b = bn;
#ifdef ORPCD_PHASES
                ++ph_rounds;
#endif
                prefetch_round();
                {  // lanes without a tile hold the empty box: lb = inf
                    const float dx = fmaxf(0.0f, fmaxf(a.x - hix, lox - b.x));
                    const float dy = fmaxf(0.0f, fmaxf(a.y - hiy, loy - b.y));
                    const float dz = fmaxf(0.0f, fmaxf(a.z - hiz, loz - b.z));
                    lb = dx * dx + dy * dy + dz * dz;
                }
                mask = __ballot(lb < W);
            }
            const int k = __builtin_ctzll(mask);
            mask &= mask - 1;
            lbk = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(lb), k));
            if (!(lbk < W)) continue;  // the bound shrank since the ballot
#ifdef ORPCD_PHASES
            ++ph_tests;
#endif
            const float lx = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(a.x), k));
            const float ly = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(a.y), k));
            const float lz = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(a.z), k));
            const float hx = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(b.x), k));
            const float hy = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(b.y), k));
            const float hz = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(b.z), k));
            const f2 bd2 = box_d2_2q(f2{qx[0], qx[1]}, f2{qy[0], qy[1]}, f2{qz[0], qz[1]}, lx, ly, lz, hx, hy, hz);
            const bool need0 = bd2.x < (kExact ? e0 : __uint_as_float(k0 & kKeyMask));
            const bool need1 = bd2.y < (kExact ? e1 : __uint_as_float(k1 & kKeyMask));
#ifdef ORPCD_PHASES
            {
                const unsigned long long b0 = __ballot(need0), b1 = __ballot(need1);
                if (b0 | b1) ph_need += __builtin_popcountll(b0) + __builtin_popcountll(b1);
            }
#endif
            if (__any(need0 || need1)) {  // lane k's tile, from the round's scalar state
                const int r = (int)(((unsigned)k * perM) >> 16), m = k - r * per;
                unsigned long long cm = cmask;
                for (int i = 0; i < r; ++i) cm &= cm - 1;
                return (csb + __builtin_ctzll(cm)) * kSuper + (S == 1 ? m : s + S * m);
            }
        }
    };

    auto next_candidate = [&](float& lbk) -> int {
#ifdef ORPCD_PHASES
        const unsigned long long t0 = __builtin_readcyclecounter();
        const int r = next_candidate_impl(lbk);
        ph_cull += __builtin_readcyclecounter() - t0;
#else
        const int r = next_candidate_impl(lbk);
#endif
#ifdef ORPCD_BOUNDS_CHECK
        // the candidate's whole-tile loads (p4: npad = ntiles x 64 points, qbox)
        if (r >= ntiles) {
            if ((threadIdx.x & 63) == 0) printf("[chk] culled_search tile %d >= ntiles %d\n", r, ntiles);
            return -1;
        }
#endif
        return r;
    };
    // software pipeline: the next candidate's 1 KiB tile load is in flight
    // while the current tile is scanned out of LDS
    float lbn = inf;
    int nxt = next_candidate(lbn);
    float4 pre = make_float4(0.f, 0.f, 0.f, 0.f), preq = pre;
    if (nxt >= 0) {
        pre = p4[nxt * kTile + lane];
        if (lane < 2 * kNQ) preq = qbox[nxt * 2 * kNQ + lane];
    }
    while (nxt >= 0) {
        const int tile = __builtin_amdgcn_readfirstlane(nxt);
#ifdef ORPCD_PHASES
        ++ph_staged;
#endif
        // SoA stage: x[64] | y[64] | z[64] | quarter boxes (lo x4, hi x4); a
        // ds_read_b64 yields two targets' coordinate, already an aligned
        // register pair for v_pk_* math
        float* sx = reinterpret_cast<float*>(stage);
        sx[lane] = pre.x;
        sx[64 + lane] = pre.y;
        sx[128 + lane] = pre.z;
        if (lane < 2 * kNQ) reinterpret_cast<float4*>(sx + 192)[lane] = preq;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        nxt = next_candidate(lbn);
        if (nxt >= 0) {
            pre = p4[nxt * kTile + lane];
            if (lane < 2 * kNQ) preq = qbox[nxt * 2 * kNQ + lane];
        }
#if ORPCD_CULL_PRIO > 0
        __builtin_amdgcn_s_setprio(0);  // the scan yields issue slots to waves in their culling chain
#endif
        // exact: the running minimum of the whole search (from k0), else of this tile
        unsigned m0 = kExact ? k0 : 0xFFFFFFFFu, m1 = kExact ? k1 : 0xFFFFFFFFu;
        const f2 qx0 = {qx[0], qx[0]}, qy0 = {qy[0], qy[0]}, qz0 = {qz[0], qz[0]};
        const f2 qx1 = {qx[1], qx[1]}, qy1 = {qy[1], qy[1]}, qz1 = {qz[1], qz[1]};
        const float4* qb = reinterpret_cast<const float4*>(sx + 192);
#pragma unroll
        for (int qd = 0; qd < kTile / kQuarter; ++qd) {
            // a quarter is scanned only if some query's box distance to it is
            // below that query's bound (including this tile's earlier
            // quarters); the bound widened by 2^-19 (kQuarterWiden) keeps the
            // test conservative against the scan's own fp32 rounding
            const float4 lo = qb[qd], hi = qb[kNQ + qd];
            const f2 bw = kExact ? ew
                                 : f2{__uint_as_float((k0 < m0 ? k0 : m0) & kKeyMask),
                                      __uint_as_float((k1 < m1 ? k1 : m1) & kKeyMask)} *
                                       f2{kQuarterWiden, kQuarterWiden};
            const f2 qd2 = box_d2_2q(f2{qx[0], qx[1]}, f2{qy[0], qy[1]}, f2{qz[0], qz[1]}, lo.x, lo.y, lo.z, hi.x,
                                     hi.y, hi.z);
            const bool need = qd2.x < bw.x || qd2.y < bw.y;
            if (!__any(need)) continue;
            ++visited;
            f2 ntx, nty, ntz;
            unsigned p0 = 0xFFFFFFFFu, p1 = 0xFFFFFFFFu;  // exact: the pending pair's med3 (see below)
            if constexpr (kPipe) {
                ntx = *reinterpret_cast<const f2*>(sx + qd * kQuarter);
                nty = *reinterpret_cast<const f2*>(sx + 64 + qd * kQuarter);
                ntz = *reinterpret_cast<const f2*>(sx + 128 + qd * kQuarter);
            }
#pragma unroll kScanUnroll
            for (int kk = qd * kQuarter; kk < (qd + 1) * kQuarter; kk += 2) {
                f2 tx, ty, tz;
                if constexpr (kPipe) {  // this pair's coordinates were read one iteration ahead
                    tx = ntx, ty = nty, tz = ntz;
                    if (kk + 2 < (qd + 1) * kQuarter) {
                        ntx = *reinterpret_cast<const f2*>(sx + kk + 2);
                        nty = *reinterpret_cast<const f2*>(sx + 64 + kk + 2);
                        ntz = *reinterpret_cast<const f2*>(sx + 128 + kk + 2);
                    }
                } else {
                    tx = *reinterpret_cast<const f2*>(sx + kk);
                    ty = *reinterpret_cast<const f2*>(sx + 64 + kk);
                    tz = *reinterpret_cast<const f2*>(sx + 128 + kk);
                }
                f2 dx = qx0 - tx, dy = qy0 - ty, dz = qz0 - tz;  // query 0 vs targets kk, kk+1
                f2 d0 = dx * dx;
                d0 = pk_fma(dy, dy, d0);
                d0 = pk_fma(dz, dz, d0);
                dx = qx1 - tx;
                dy = qy1 - ty;
                dz = qz1 - tz;  // query 1
                f2 d1 = dx * dx;
                d1 = pk_fma(dy, dy, d1);
                d1 = pk_fma(dz, dz, d1);
                const unsigned a0 = (__float_as_uint(d0.x) & kKeyMask) | (unsigned)kk;
                const unsigned c0 = (__float_as_uint(d0.y) & kKeyMask) | (unsigned)(kk + 1);
                const unsigned a1 = (__float_as_uint(d1.x) & kKeyMask) | (unsigned)kk;
                const unsigned c1 = (__float_as_uint(d1.y) & kKeyMask) | (unsigned)(kk + 1);
                if constexpr (kExact) {
                    // (minimum, runner-up) of every key scanned: with m <= s, the
                    // second smallest of {m, s, a, c} is min(s, med3(m, a, c))
                    // (if s is among the two smallest, m is the smallest and
                    // a, c >= s; otherwise it is the second smallest of {m, a,
                    // c} <= s).  Two pairs share one update of s (a min3 of
                    // both med3s): 5 ops per query and two key pairs, not 6
                    // (a quarter's iteration count is even and unrolled)
                    static_assert(kQuarter % 4 == 0, "pairs of iterations per quarter");
                    if (((kk - qd * kQuarter) & 2) == 0) {
                        p0 = umed3(m0, a0, c0);
                        p1 = umed3(m1, a1, c1);
                    } else {
                        s0 = umin3(s0, p0, umed3(m0, a0, c0));
                        s1 = umin3(s1, p1, umed3(m1, a1, c1));
                    }
                    m0 = umin3(m0, a0, c0);
                    m1 = umin3(m1, a1, c1);
                } else {  // min(min(m, a), c): the compiler forms v_min3_u32 for this association (asm measured slower)
                    m0 = min(min(m0, a0), c0);
                    m1 = min(min(m1, a1), c1);
                }
                if constexpr (kPipe) __builtin_amdgcn_sched_barrier(0);
            }
        }
        asm volatile("" ::: "memory");  // all reads of this tile precede the next stage write
#if ORPCD_CULL_PRIO > 0
        __builtin_amdgcn_s_setprio(ORPCD_CULL_PRIO);
#endif
        // a tile improves a query only if its masked d^2 is strictly smaller
#ifdef ORPCD_PHASES
        ph_impr += __any((m0 & kKeyMask) < (k0 & kKeyMask) || (m1 & kKeyMask) < (k1 & kKeyMask)) ? 1 : 0;
#endif
        if constexpr (kExact) {  // the minimum moved into this tile: its band is the new bound
            if (m0 != k0) {
                k0 = m0;
                t0 = tile;
                e0 = exact_band_hi(__uint_as_float(k0 & kKeyMask), qnorm(qx[0], qy[0], qz[0]));
            }
            if (m1 != k1) {
                k1 = m1;
                t1 = tile;
                e1 = exact_band_hi(__uint_as_float(k1 & kKeyMask), qnorm(qx[1], qy[1], qz[1]));
            }
            ew = f2{e0, e1} * f2{kQuarterWiden, kQuarterWiden};
        } else {
            if ((m0 & kKeyMask) < (k0 & kKeyMask)) {
                k0 = m0;
                t0 = tile;
            }
            if ((m1 & kKeyMask) < (k1 & kKeyMask)) {
                k1 = m1;
                t1 = tile;
            }
        }
        if constexpr (kExact) {
            W = __uint_as_float(wave_umax(max(__float_as_uint(e0), __float_as_uint(e1))));
        } else {
            Wk = wave_umax((k0 > k1 ? k0 : k1) & kKeyMask);
            W = __uint_as_float(Wk);
        }
        // the prefetched candidate was chosen under the previous bound: re-test
        while (nxt >= 0 && !(lbn < W)) {
            nxt = next_candidate(lbn);
            if (nxt >= 0) {
                pre = p4[nxt * kTile + lane];
                if (lane < 2 * kNQ) preq = qbox[nxt * 2 * kNQ + lane];
            }
        }
    }
    if (t0 >= 0) {
        bj[0] = t0 * kTile + (int)(k0 & 63u);
        bd[0] = __uint_as_float(k0 & kKeyMask);
    }
    if (t1 >= 0) {
        bj[1] = t1 * kTile + (int)(k1 & 63u);
        bd[1] = __uint_as_float(k1 & kKeyMask);
    }
    if constexpr (kExact) {
        sk[0] = s0;
        sk[1] = s1;
    }
#ifdef ORPCD_PHASES
    if (phase_cull_out) {
        phase_cull_out[0] = ph_cull;
        phase_cull_out[1] = ph_rounds;
        phase_cull_out[2] = ph_tests;
        phase_cull_out[3] = ph_impr;
        phase_cull_out[4] = ph_need;
        phase_cull_out[5] = ph_staged;
    }
#endif
    return visited;
}

__device__ __forceinline__ void xform(const double Q[12], const double p[3], double q[3]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    q[0] = Q[0] * p[0] + Q[1] * p[1] + Q[2] * p[2] + Q[3];
    q[1] = Q[4] * p[0] + Q[5] * p[1] + Q[6] * p[2] + Q[7];
    q[2] = Q[8] * p[0] + Q[9] * p[1] + Q[10] * p[2] + Q[11];
}

// The target's fp32 frame origin (CloudLayout::org): an fp32 query is
// (float)(q - org), subtracted in fp64 before the one rounding.
struct Org3 {
    double x, y, z;
};
static inline Org3 org_of(const CloudLayout& L) { return Org3{L.org[0], L.org[1], L.org[2]}; }

// upper-triangle index of (a,b), a<=b, in a 6x6
__device__ __forceinline__ constexpr int ut(int a, int b) { return a * 6 - a * (a - 1) / 2 + (b - a); }

// fp32 search radius: enlarged so no pair with exact d^2 < r^2 is rejected by
// fp32 rounding or key truncation; the strict test is applied in fp64 later.
static inline float search_r2(double r2) { return (float)(r2 * (1.0 + 1e-5)) * 1.0001f; }

// seed slack: bound = d^2(seed) * (1 + 1e-4) so the seed target itself (and
// any closer one) is re-found by the scan (1e-4 >> the 2^-17 key truncation)
constexpr float kSeedSlack = 1.0001f;
__device__ __forceinline__ float seed_bound(float d2) {
#pragma clang fp contract(off)  // the same rounding in every transform kernel (a bound: answers never depend on it)
    return d2 * kSeedSlack + 1e-30f;
}


// ---------------------------------------------------------------------------
// Cost-ordered search dispatch (opt.sched).  The search of pass p measures
// each wave's duration (s_memrealtime, 10 ns ticks) and sums it per (start,
// 128-query group) into wcost[p & 1] and over the pass into wtot[p & 1].  The
// query transform of pass p + 1 (one thread per group) splits a group into
// S = ceil(cost / (pass total / sched_items)) waves (1..64; the uniform host
// split at pass 0, when no cost is known), files its S work items under the
// cost class of one split (log2 of cost / S, heaviest = class 0) and the
// search of pass p + 1 takes item k of the class-major list as wave k: the
// heaviest waves are dispatched first and no wave is much longer than the
// pass total / sched_items, so the launch no longer ends with a few long
// waves on an idle chip (measured per-wave timelines: the last 1% of a
// launch's waves held 15-35% of its span).  Splits and order never change
// an answer (every split returns the lexicographic (masked d^2, index)
// minimum over its tiles, merged by atomicMin).
// item: slot << 48 | target << 44 | group << 20 | split << 8 | S
__host__ __device__ __forceinline__ unsigned long long sched_item(int slot, int k, int wg, int split, int S) {
    return ((unsigned long long)slot << 48) | ((unsigned long long)k << 44) | ((unsigned long long)wg << 20) |
           ((unsigned long long)split << 8) | (unsigned long long)S;
}
// most splits of one 128-query group (item fields: 8 bits each for S and split)
#ifndef ORPCD_SCHED_SMAX
#define ORPCD_SCHED_SMAX 64
#endif
static_assert(ORPCD_SCHED_SMAX >= 1 && ORPCD_SCHED_SMAX <= 255, "split count must fit the item's 8-bit fields");
struct SchedX {                          // query transform side (pass p + 1)
    const unsigned* wcost_prev;          // the previous pass's per-group costs (B x NG)
    unsigned* wcost_cur;                 // this pass's: zeroed for the search
    const unsigned long long* wtot_prev; // the previous pass's total (kSchedTot words)
    unsigned* cnt;                       // this pass's items per class (zeroed by the previous search)
    unsigned long long* list;            // class-major items, cap per class
    int cap, NG, have_cost, S0;          // S0: the host's uniform split (no cost known)
    float inv_want;                      // 1 / sched_items
    float max_target;                    // cap on a split's planned cost (10 ns ticks; 0: none), opt.sched_cap_us
    float inv_max_items;                 // 1 / the item budget sched_capacity holds room for
};
struct SchedS {                          // search side (pass p)
    const unsigned* cnt;                 // this pass's items per class
    unsigned* cnt_next;                  // the next pass's: zeroed here (block 0)
    const unsigned long long* list;
    unsigned* wcost;                     // this pass's per-group costs
    unsigned long long* wtot;            // this pass's total
    unsigned long long* wtot_next;       // the next pass's: zeroed here (block 0; read by this
                                         // pass's transform, which ran before)
    int cap, NG, B;
    int xcd;                             // item order XCD-aware (option sched_xcd)
};

// The ordered dispatch's work items of start `slot` (one block per start,
// launched beside the query transform's blocks).
__device__ __forceinline__ void plan_start_items(const SchedX& sx, int slot, int tk) {
    const int lane = threadIdx.x & 63;
    // The items depend only on the previous pass's costs, so this block runs
    // beside the transform blocks (as the sequel of one of them it lengthened
    // the transform by 3-5 us).  Counts per class are aggregated in LDS first:
    // a pass takes kSchedClasses global atomics per start (one counter per
    // class bumped by every group serialised ~12k atomics on a few addresses).
    __shared__ float s_target;
    __shared__ unsigned lcnt[kSchedClasses], lbase[kSchedClasses];
    if (threadIdx.x < kSchedClasses) lcnt[threadIdx.x] = 0u;
    if (threadIdx.x < 64) {
        float t = 0.0f;
        if (sx.have_cost) {
            t = (float)sx.wtot_prev[lane];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
        }
        float tg = fmaxf(t * sx.inv_want, 1.0f);
        // early passes: the pass total / sched_items is long (~80 us at C2
        // pass 5) and a group's cost can double from one pass to the next, so
        // an unsplit group became the launch's critical wave (r05 wave dumps);
        // the cap splits heavy groups further there
        // the cap, within the list's room: at most ~1 / inv_max_items items
        if (sx.max_target > 0.0f) tg = fmaxf(fminf(tg, sx.max_target), fmaxf(t * sx.inv_max_items, 1.0f));
        if (lane == 0) s_target = tg;
    }
    __syncthreads();
    const int NG = sx.NG;
    const unsigned* cost = sx.wcost_prev + (size_t)slot * NG;
    auto plan = [&](int g, int& S, int& cls) {
        S = sx.S0;
        cls = kSchedClasses - 1;
        if (sx.have_cost) {
            const unsigned C = cost[g];
            S = min(ORPCD_SCHED_SMAX, max(1, (int)ceilf((float)C / s_target)));
            const unsigned per = C / (unsigned)S + 1u;
            cls = max(0, kSchedClasses - 1 - (31 - __builtin_clz(per)));  // log2 of a split's cost, heaviest first
        }
    };
    for (int g = threadIdx.x; g < NG; g += blockDim.x) {  // 1: items per class
        int S, cls;
        plan(g, S, cls);
        atomicAdd(lcnt + cls, (unsigned)S);
    }
    __syncthreads();
    if (threadIdx.x < kSchedClasses) {
        const unsigned n = lcnt[threadIdx.x];
        lbase[threadIdx.x] = n ? atomicAdd(sx.cnt + threadIdx.x, n) : 0u;
        lcnt[threadIdx.x] = 0u;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < NG; g += blockDim.x) {  // 2: the items
        int S, cls;
        plan(g, S, cls);
        const unsigned at = lbase[cls] + atomicAdd(lcnt + cls, (unsigned)S);
        sx.wcost_cur[(size_t)slot * NG + g] = 0u;
        unsigned long long* out = sx.list + (size_t)cls * sx.cap + at;
        for (int k = 0; k < S; ++k) out[k] = sched_item(slot, tk, g, k, S);
    }
}

// box and worst bound of each search wave's 128 queries (waves 0-1 and 2-3
// of this 256-query block bx): what the search would reduce, computed once
// by the query transform.  Every thread of the block calls it.
__device__ __forceinline__ void write_gbox(float x, float y, float z, float bound, bool valid, int slot, int bx, int N,
                                           float4* __restrict__ gbox) {
    const float inf = 3.0e38f;
    __shared__ float part[4][7];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float r[7] = {wave_fmin(x), wave_fmin(y), wave_fmin(z), wave_fmax(valid ? x : -inf),
                        wave_fmax(valid ? y : -inf), wave_fmax(valid ? z : -inf),
                        __uint_as_float(wave_umax(__float_as_uint(bound)))};
    if (lane < 7) part[w][lane] = r[lane];
    __syncthreads();
    if (threadIdx.x < 2 && (bx * 2 + threadIdx.x) * 128 < N) {
        const float* a = part[2 * threadIdx.x];
        const float* b = part[2 * threadIdx.x + 1];
        float4* g = gbox + ((size_t)slot * ((N + 127) / 128) + bx * 2 + threadIdx.x) * 2;
        g[0] = make_float4(fminf(a[0], b[0]), fminf(a[1], b[1]), fminf(a[2], b[2]),
                           __uint_as_float(max(__float_as_uint(a[6]), __float_as_uint(b[6]))));
        g[1] = make_float4(fmaxf(a[3], b[3]), fmaxf(a[4], b[4]), fmaxf(a[5], b[5]), 0.0f);
    }
}

// fp32 queries of every running start for the next pass: q = fp32(Q * p),
// and in q.w the query's search bound: d^2 to its previous correspondence
// (x 1 + 1e-4), or, without one, to the nearest of a strided set of tile
// representatives (real targets, so either bound is valid), capped at r2s.
__global__ __launch_bounds__(256) void xform_queries_kernel(const double* __restrict__ src, int N,
                                                            const int32_t* __restrict__ active,
                                                            const double* __restrict__ Qm,
                                                            const int32_t* __restrict__ done,
                                                            const TargetDesc* __restrict__ tdesc, TgtBounds tb,
                                                            const int32_t* __restrict__ prevnn,
                                                            float r2s, int reseed, float4* __restrict__ q32,
                                                            unsigned long long* __restrict__ best,
                                                            float4* __restrict__ gbox, SchedX sx, ExactArgs ex) {
    const int slot = active[blockIdx.y];
    if (done[slot]) return;
    const int tk = target_of_row(tb, blockIdx.y);
    if (sx.list && blockIdx.x == 0) {  // the extra block (dispatched first): the pass's work items of this start
        plan_start_items(sx, slot, tk);
        return;
    }
    const int bx = blockIdx.x - (sx.list ? 1 : 0);  // this block's 256 queries
    const TargetDesc& tg = tdesc[tk];
    const float4* __restrict__ p4 = tg.p4;
    const int i = bx * 256 + threadIdx.x;
    const bool valid = i < N;
    const float inf = 3.0e38f;
    float x = inf, y = inf, z = inf, bound = 0.0f;
    if (valid) {
        best[(size_t)slot * N + i] = kNone;  // split searches merge into it by atomicMin
        double Q[12];
#pragma unroll
        for (int t = 0; t < 12; ++t) Q[t] = Qm[12 * slot + t];
        const double p[3] = {src[3 * i], src[3 * i + 1], src[3 * i + 2]};
        double q[3];
        xform(Q, p, q);
        x = (float)(q[0] - tg.ox), y = (float)(q[1] - tg.oy), z = (float)(q[2] - tg.oz);
        bound = r2s;
        int jp = prevnn[(size_t)slot * N + i];
#ifdef ORPCD_BOUNDS_CHECK
        if (jp >= tg.npts) {
            printf("[chk] xform slot %d i %d prevnn %d npts %d\n", slot, i, jp, tg.npts);
            jp = kNoSeed;
        }
#endif
        if (jp >= 0) bound = fminf(bound, seed_bound(d2f(x, y, z, p4[jp])));
        if (tg.sgrid && tg.sg_on) {
            // the target nearest to the centre of the query's seed-grid cell
            // (clamped to the grid): early passes move the poses far, so the
            // previous correspondence alone is a loose bound (CPU study: a
            // median 1.8x the nearest distance in pass 1, 1.007x with this
            // seed beside it), and pass 0 needs no strided representatives
            const int cx = min(kSeedGrid - 1, max(0, (int)((x - tg.sg_lo[0]) * tg.sg_inv[0])));
            const int cy = min(kSeedGrid - 1, max(0, (int)((y - tg.sg_lo[1]) * tg.sg_inv[1])));
            const int cz = min(kSeedGrid - 1, max(0, (int)((z - tg.sg_lo[2]) * tg.sg_inv[2])));
            int g = tg.sgrid[(cx * kSeedGrid + cy) * kSeedGrid + cz];
#ifdef ORPCD_BOUNDS_CHECK
            if (g < 0 || g >= tg.npts) {
                printf("[chk] xform slot %d i %d seed cell %d,%d,%d -> %d npts %d\n", slot, i, cx, cy, cz, g, tg.npts);
                g = 0;
            }
#endif
            bound = fminf(bound, seed_bound(d2f(x, y, z, p4[g])));
        } else if (jp < 0 && (jp == kNoSeed || reseed)) {
            for (int t = 0; t < tg.ntiles; t += tg.seed_stride)
                bound = fminf(bound, seed_bound(d2f(x, y, z, p4[t * kTile])));
        }
        if (ex.sec) {  // exact mode: the sentinel bound; the split merge state of the pass
            bound = exact_sentinel(bound, qnorm(x, y, z));
            ex.sec[(size_t)slot * N + i] = 0xFFFFFFFFu;
        }
        q32[(size_t)slot * N + i] = make_float4(x, y, z, bound);
    }
    if (!gbox) return;
    write_gbox(x, y, z, bound, valid, slot, bx, N, gbox);
}

#ifdef ORPCD_WAVETIME
// per-wave timeline of nn_search_kernel launches (instrumented builds only):
// (entry, exit) in s_memrealtime ticks (100 MHz), and (start row, block, wave,
// quarters scanned)
constexpr unsigned kWtMax = 1u << 20;
__device__ unsigned long long g_wt[3 * kWtMax];
#endif

// --------------------------------------------------------------------------
// Search kernel: grid = (blocks per start * S, running starts), 4 waves/block.
// --------------------------------------------------------------------------
// first culling round's super-tile boxes: independent of the start and its
// queries, so their load overlaps the slot and query loads (xyz only, by raw
// buffer loads: lanes past nsuper read zeros, unguarded; a guarded 16 B load
// whose unused .w register was reused forced a wait for it before the query
// loads were issued)
// The search layout of one target, read once from its TargetDesc.
struct SearchTgt {
    const float4 *p4, *tlo, *thi, *qbox, *slo, *shi;
    int ntiles, nsuper;
};
__device__ __forceinline__ SearchTgt search_tgt(const TargetDesc& tg) {
    return SearchTgt{tg.p4, tg.tlo, tg.thi, tg.qbox, tg.slo, tg.shi, tg.ntiles, tg.nsuper};
}

__device__ __forceinline__ void load_super0(const SearchTgt& tg, float4& s0lo, float4& s0hi) {
    const int lane = threadIdx.x & 63;
    const int nb = tg.nsuper * (int)sizeof(float4);
    const auto lo = __builtin_amdgcn_raw_buffer_load_b96(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tg.slo), (short)0, nb, 0x00020000), lane * 16, 0, 0);
    const auto hi = __builtin_amdgcn_raw_buffer_load_b96(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tg.shi), (short)0, nb, 0x00020000), lane * 16, 0, 0);
    s0lo = make_float4(__uint_as_float(lo[0]), __uint_as_float(lo[1]), __uint_as_float(lo[2]), 0.f);
    s0hi = make_float4(__uint_as_float(hi[0]), __uint_as_float(hi[1]), __uint_as_float(hi[2]), 0.f);
}

// One wave's search: split `split` of S of the 128-query group wg of start
// `slot` (queries wg * 128 + lane + 64 k).  Returns quarters scanned.
template <bool kExact = false>
__device__ __forceinline__ int search_group(const float4* __restrict__ q32, int N, const SearchTgt tg,
                                            int super_cull, int S, int split, int slot, int wg,
                                            unsigned long long* __restrict__ best,
                                            unsigned long long* __restrict__ counters, unsigned cslot,
                                            float4* stage_w, const float4* __restrict__ gbox, float4 s0lo,
                                            float4 s0hi, ExactArgs ex = ExactArgs{}, int tk = 0) {
    const int lane = threadIdx.x & 63;
#ifdef ORPCD_PHASES
    const unsigned long long ph_t0 = __builtin_readcyclecounter();
#endif
    // wave-uniform by construction; readfirstlane keeps them (and the group's
    // box record address) in scalar registers
    slot = __builtin_amdgcn_readfirstlane(slot);
    wg = __builtin_amdgcn_readfirstlane(wg);
    S = __builtin_amdgcn_readfirstlane(S);
    split = __builtin_amdgcn_readfirstlane(split);
    const int i0 = wg * (64 * kCQPT) + lane;
    float qx[kCQPT], qy[kCQPT], qz[kCQPT], bound[kCQPT], bd[kCQPT];
    int bj[kCQPT];
    unsigned sk[kCQPT];
    const float4* qs = q32 + (size_t)slot * N;
    const float4* gb = gbox + ((size_t)slot * ((N + 127) / 128) + wg) * 2;
    // the queries by raw buffer loads: a lane past N reads zeros (bound 0: never
    // takes anything) without a guard.  Guarded global loads were each put in
    // a branch with its own wait, which serialised the two.
    const __amdgpu_buffer_rsrc_t qrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(qs), (short)0, N * (int)sizeof(float4), 0x00020000);
#pragma unroll
    for (int k = 0; k < kCQPT; ++k) {
        const int i = i0 + 64 * k;
        const auto q = __builtin_amdgcn_raw_buffer_load_b128(qrs, i * (int)sizeof(float4), 0, 0);
        qx[k] = __uint_as_float(q[0]);
        qy[k] = __uint_as_float(q[1]);
        qz[k] = __uint_as_float(q[2]);
        bound[k] = __uint_as_float(q[3]);
    }
#ifdef ORPCD_PHASES
    const float wq = __uint_as_float(wave_umax(__float_as_uint(qx[0] + qy[1])));  // the query loads have landed
    const unsigned long long ph_t1 = __builtin_readcyclecounter() + (wq == 1.2345f ? 1 : 0);
    unsigned long long ph_cull[6] = {0, 0, 0, 0, 0, 0};
    const int visited = culled_search<true>(stage_w, tg.p4, tg.tlo, tg.thi, tg.qbox, tg.ntiles, tg.slo, tg.shi,
                                            tg.nsuper, super_cull, S, split, qx, qy, qz, bound, bd, bj, s0lo, s0hi,
                                            gb, ph_cull);
#else
    const int visited = culled_search<true, kExact>(stage_w, tg.p4, tg.tlo, tg.thi, tg.qbox, tg.ntiles, tg.slo,
                                                    tg.shi, tg.nsuper, super_cull, S, split, qx, qy, qz, bound, bd,
                                                    bj, s0lo, s0hi, gb, nullptr, sk);
#endif
    if (lane == 0 && counters) {  // spread over kCounterSlots cache lines (one address serialises)
        unsigned long long* cs = counters + kCounterStride * (cslot % kCounterSlots);
        atomicAdd(cs, (unsigned long long)visited);
        atomicMax(cs + 1, (unsigned long long)visited);
#ifdef ORPCD_PHASES
        const unsigned long long ph_t2 = __builtin_readcyclecounter();
        atomicAdd(cs + 2, ph_t1 - ph_t0);   // query loads
        atomicAdd(cs + 3, ph_cull[0]);      // culling (next_candidate)
        atomicAdd(cs + 6, ph_cull[1]);      // tile-AABB rounds loaded
        atomicAdd(cs + 7, ph_cull[2]);      // per-query candidate tests
        atomicAdd(cs + 4, ph_t2 - ph_t1);   // search incl. culling
        atomicAdd(cs + 5, 1ull);            // waves
        atomicAdd(cs + 8, ph_cull[3]);      // scanned tiles that improved some query of the wave
        atomicAdd(cs + 9, ph_cull[4]);      // queries whose own box test wanted the candidate tile
        atomicAdd(cs + 10, ph_cull[5]);     // tiles staged (and their quarters tested)
#endif
    }
    unsigned long long* out = best + (size_t)slot * N;
    if constexpr (kExact) {
        // the query's runner-up over all splits is the minimum of every
        // split's runner-up and of every merge's loser; only keys within the
        // band of the key they lost to can matter (sec[], reset by the query
        // transform), so only those are published -- rarely.  The band test
        // against the final winner is nn_exact_kernel's.  Both merges are
        // issued before either result is used (one round trip per wave).
        unsigned long long v[kCQPT], old[kCQPT];
#pragma unroll
        for (int k = 0; k < kCQPT; ++k) {
            const int i = i0 + 64 * k;
            v[k] = bj[k] < 0 || i >= N ? kNone : ((unsigned long long)__float_as_uint(bd[k]) << 32) | (unsigned)bj[k];
            old[k] = kNone;
            if (v[k] == kNone) continue;
            if (S == 1)
                out[i] = v[k];
            else
                old[k] = atomicMin(out + i, v[k]);
        }
#pragma unroll
        for (int k = 0; k < kCQPT; ++k) {
            if (v[k] == kNone) continue;
            const int i = i0 + 64 * k;
            const float A = qnorm(qx[k], qy[k], qz[k]);
            unsigned s2 = __uint_as_float(sk[k] & kKeyMask) <= exact_band_hi(bd[k], A) ? sk[k] : 0xFFFFFFFFu;
            if (old[k] != kNone) {
                const unsigned long long lose = old[k] < v[k] ? v[k] : old[k], win = old[k] < v[k] ? old[k] : v[k];
                const unsigned lk = (unsigned)(lose >> 32);
                if (__uint_as_float(lk) <= exact_band_hi(__uint_as_float((unsigned)(win >> 32)), A)) s2 = min(s2, lk);
            }
            if (s2 == 0xFFFFFFFFu) continue;
            // the query's first publisher lists it for nn_exact_kernel
            const bool first = S == 1 || atomicMin(ex.sec + (size_t)slot * N + i, s2) == 0xFFFFFFFFu;
            if (S == 1) ex.sec[(size_t)slot * N + i] = s2;
            if (first) {
                const unsigned at = atomicAdd(ex.cnt, 1u);
                ex.list[at] = ((unsigned long long)slot << 40) | ((unsigned long long)tk << 32) | (unsigned)i;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < kCQPT; ++k) {
            const int i = i0 + 64 * k;
            if (i >= N) continue;
            const unsigned long long v =
                bj[k] < 0 ? kNone : ((unsigned long long)__float_as_uint(bd[k]) << 32) | (unsigned)bj[k];
            if (S == 1)
                out[i] = v;
            else if (v != kNone)
                atomicMin(out + i, v);
        }
    }
    return visited;
}

// Uniform-split dispatch: grid = (blocks per start * S, running starts), 4 waves/block.
template <bool kExact = false>
__device__ __forceinline__ void nn_search_body(
    const float4* __restrict__ q32, int N, const TargetDesc& tg, int super_cull, const int32_t* __restrict__ active,
    const int32_t* __restrict__ done, int S, unsigned long long* __restrict__ best,
    unsigned long long* __restrict__ counters, int by, int bx, int wid, float4* stage_w,
    const float4* __restrict__ gbox, ExactArgs ex = ExactArgs{}, int tk = 0) {
#ifdef ORPCD_WAVETIME
    const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
    const SearchTgt st = search_tgt(tg);
    float4 s0lo, s0hi;
    load_super0(st, s0lo, s0hi);
    const int slot = active[by];
    if (done[slot]) return;
    const int grp = bx / S, split = bx - grp * S;
    const int wg = grp * kCWaves + wid;
    if (wg * (64 * kCQPT) >= N) return;  // a wave past the last query group (no gbox entry)
    const int visited = search_group<kExact>(q32, N, st, super_cull, S, split, slot, wg, best, counters,
                                             (unsigned)(bx * kCWaves + wid + by), stage_w, gbox, s0lo, s0hi, ex, tk);
    (void)visited;
#ifdef ORPCD_WAVETIME
    if ((threadIdx.x & 63) == 0) {  // a fixed slot per wave: no shared counter to serialise on
        const unsigned k = ((unsigned)blockIdx.y * gridDim.x + blockIdx.x) * kCWaves + wid;
        if (k < kWtMax) {
            g_wt[3 * k] = wt0;
            g_wt[3 * k + 1] = __builtin_amdgcn_s_memrealtime();
            g_wt[3 * k + 2] = ((unsigned long long)by << 48) | ((unsigned long long)bx << 24) |
                              ((unsigned long long)wid << 20) | (unsigned long long)(visited & 0xFFFFF);
        }
    }
#endif
}

// Ordered dispatch (SchedS): wave k of the launch takes item k of the
// class-major list, heaviest class first; the wave's duration is added to its
// group's cost and to the pass total for the next pass's schedule.
// Waves per workgroup of the ordered dispatch (A/B macro ORPCD_SCHED_WAVES).
// One: a wave's slot is refilled as soon as it exits, without waiting for
// three sibling waves of different length (round 5, profiles/r05_sched_waves_ab.txt: C2 exact
// 30 starts 15.6 -> 15.2 ms, 64 starts 24.9 -> 24.1 ms, 2 waves per block in
// between; identical result hashes).
#ifndef ORPCD_SCHED_WAVES
#define ORPCD_SCHED_WAVES 1
#endif
constexpr int kSWaves = ORPCD_SCHED_WAVES;
template <bool kExact>
__global__ __launch_bounds__(64 * kSWaves) __attribute__((amdgpu_waves_per_eu(kExact ? ORPCD_EXACT_WAVES : ORPCD_FAST_WAVES, 8))) void nn_search_sched_kernel(
    const float4* __restrict__ q32, int N, const TargetDesc* __restrict__ tdesc, int super_cull,
    unsigned long long* __restrict__ best, unsigned long long* __restrict__ counters,
    const float4* __restrict__ gbox, SchedS sa, ExactArgs ex) {
    __shared__ float4 stage[kSWaves][kTile];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && wid == 0) {
        if (lane < kSchedClasses) sa.cnt_next[lane] = 0u;
        sa.wtot_next[lane] = 0ull;  // kSchedTot == 64
    }
    const unsigned w = __builtin_amdgcn_readfirstlane(blockIdx.x * kSWaves + wid);
    unsigned base = 0, off = 0, ncls = 0;
    int cls = -1;
#pragma unroll
    for (int c = 0; c < kSchedClasses; ++c) {
        const unsigned n = __builtin_amdgcn_readfirstlane(sa.cnt[c]);
        if (cls < 0 && w < base + n) {
            cls = c;
            off = w - base;
            ncls = n;
        }
        base += n;
    }
    if (cls < 0) return;  // past the pass's items
    if (sa.xcd) {
        // one-wave workgroups go to the XCDs round-robin (workgroup w on XCD
        // w % 8): waves w, w + 8, ... of a class take one contiguous chunk of
        // its items (adjacent query groups and their splits, which read the
        // same target tiles) instead of every 8th item, so each XCD's L2
        // holds one region's tiles (profiles/r06_pmc_waves.json: one-wave
        // workgroups raised the L2 misses 37%)
        const unsigned n8 = ncls >> 3;
        if (off < 8 * n8) off = (off & 7u) * n8 + (off >> 3);
    }
#ifdef ORPCD_SCHED_CHECK
    if (base > (unsigned)sa.cap || off >= (unsigned)sa.cap) {
        if (lane == 0 && w < 4) printf("[sched] counts %u exceed cap %d (w %u cls %d off %u)\n", base, sa.cap, w, cls, off);
        return;
    }
#endif
    const unsigned long long itv = sa.list[(size_t)cls * sa.cap + off];
    // wave-uniform: scalar registers (readfirstlane returns int: widen through
    // unsigned, or a low word with bit 31 set would sign-extend into the high one)
    const unsigned long long it =
        ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(itv >> 32)) << 32) |
        (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)itv);
    const int slot = (int)(it >> 48), tk = (int)((it >> 44) & 15u), wg = (int)((it >> 20) & 0xFFFFFFu);
    const int split = (int)((it >> 8) & 0xFFu), S = (int)(it & 0xFFu);
#ifdef ORPCD_SCHED_CHECK
    if (slot >= sa.B || wg >= sa.NG || tk >= kMaxTargets || S < 1 || S > ORPCD_SCHED_SMAX || split >= S || wg * 128 >= N) {
        if (lane == 0) printf("[sched] bad item w %u cls %d off %u: slot %d tk %d wg %d split %d S %d\n", w, cls, off, slot, tk, wg, split, S);
        return;
    }
#endif
    const SearchTgt st = search_tgt(tdesc[tk]);
    float4 s0lo, s0hi;
    load_super0(st, s0lo, s0hi);
    const int visited = search_group<kExact>(q32, N, st, super_cull, S, split, slot, wg, best, counters, w,
                                             stage[wid], gbox, s0lo, s0hi, ex, tk);
    (void)visited;
    if (lane == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned d = (unsigned)min(t1 - t0, 0xFFFFFFull);
        atomicAdd(sa.wcost + (size_t)slot * sa.NG + wg, d);
        atomicAdd(sa.wtot + (w & (kSchedTot - 1)), (unsigned long long)d);
#ifdef ORPCD_WAVETIME
        if (w < kWtMax) {
            g_wt[3 * w] = t0;
            g_wt[3 * w + 1] = t1;
            g_wt[3 * w + 2] = ((unsigned long long)slot << 48) | ((unsigned long long)wg << 24) |
                              ((unsigned long long)(S > 15 ? 15 : S) << 20) | (unsigned long long)(visited & 0xFFFFF);
        }
#endif
    }
}

// Uniform-split search: grid = (sblk * S, running starts), 4 waves/block;
// block (bx, by) is split bx % S of query block bx / S of launch row by.
template <bool kExact>
__global__ __launch_bounds__(kCBlock) __attribute__((amdgpu_waves_per_eu(kExact ? ORPCD_EXACT_WAVES : ORPCD_FAST_WAVES, 8))) void nn_search_kernel(
    const float4* __restrict__ q32, int N, const TargetDesc* __restrict__ tdesc, TgtBounds tb, int super_cull,
    const int32_t* __restrict__ active, const int32_t* __restrict__ done, int S, unsigned long long* __restrict__ best,
    unsigned long long* __restrict__ counters, const float4* __restrict__ gbox, ExactArgs ex) {
    __shared__ float4 stage[kCWaves][kTile];
    const int wid = threadIdx.x >> 6;
    const int by = blockIdx.y, bx = blockIdx.x;
    const int tk = target_of_row(tb, by);
    nn_search_body<kExact>(q32, N, tdesc[tk], super_cull, active, done, S, best, counters, by, bx, wid, stage[wid],
                           gbox, ex, tk);
}

// --------------------------------------------------------------------------
// Exact mode, second stage (after the search): a listed query whose published
// runner-up lies within the fp32 error band of its winner (exact_band_hi) is
// re-searched in fp64 by a whole wave: the surviving tiles are scanned in
// fp64 in the oracle's operation order ((dx^2 + dy^2) + dz^2, no contraction)
// and the lexicographic (d^2, input index) minimum replaces the winner in
// best[] -- KDTree::nn1 of oracle/orpcd_oracle.cpp:192-217.
//
// Candidates: every target t with d64(t) <= d64(j) (j: the fp32 winner) has
// d32(t) <= d32(j) + 2 delta, i.e. at most band_hi of j's key (exact_band_hi,
// the search's own certification bound), and a box d^2 never exceeds a member
// point's, so tiles are culled against band_hi(key(j)) (x 1.0001 against the
// box test's own rounding).  j itself is within it: the scan's minimum over
// the candidates is the oracle's answer without j's fp64 distance first.
//
// The kernel is a chain of dependent round trips, so it is laid out to be
// short: one list entry per wave (round 2 dealt 64 entries per wave and a
// wave re-searched its filed ones one after another), the entry read beside
// the entry count, then in one round everything that depends only on the
// entry (winner, fp32 query, runner-up, pose, source point, the first 64
// super-tile boxes), then the tile boxes, then the tile points.
// --------------------------------------------------------------------------
__device__ __forceinline__ double d2_oracle(const double q[3], const double* __restrict__ t) {
#pragma clang fp contract(off)
    const double dx = q[0] - t[0], dy = q[1] - t[1], dz = q[2] - t[2];
    return dx * dx + dy * dy + dz * dz;
}
__device__ __forceinline__ float box_d2_plain(float x, float y, float z, float4 lo, float4 hi) {
#pragma clang fp contract(off)
    return box_d2(x, y, z, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z);
}

constexpr int kExactList = 512;  // candidate tiles listed per wave before a scan

// fused mode: a listed query's winner in best[] carries this bit in its index
// word once its entry is done (Morton indices are < 2^27; kNone has it too)
constexpr unsigned long long kResolvedBit = 1ull << 31;

// One list entry (slot << 40 | target << 32 | query): the band test and, if
// filed, the re-search.  Every lane of the wave calls it with the same entry;
// returns the new winner's Morton index, or -1 when the fp32 winner stands.
// bv: the winner as read here (for the caller's store).
__device__ __forceinline__ int exact_entry(unsigned long long ent, const double* __restrict__ src, int N,
                                           const double* __restrict__ Qm, const TargetDesc* __restrict__ tdesc,
                                           const float4* __restrict__ q32, const ExactArgs& ex,
                                           const unsigned long long* __restrict__ best, int* __restrict__ tl,
                                           unsigned long long& bv, unsigned& filed) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int slot = (int)(ent >> 40), tk = (int)((ent >> 32) & 0xFFu), i = (int)(unsigned)ent;
#ifdef ORPCD_BOUNDS_CHECK
    if (slot >= 4096 || tk >= kMaxTargets || i >= N || i < 0) {
        if (lane == 0) printf("[chk] exact entry %llx: slot %d tk %d i %d N %d\n", ent, slot, tk, i, N);
        bv = kNone;
        return -1;
    }
#endif
    const size_t qi = (size_t)slot * N + i;
    const TargetDesc& tg = tdesc[tk];
    // the entry's independent loads, one round
    bv = best[qi];
    const float4 qq = q32[qi];
    const unsigned sk = ex.sec[qi];
    double Q[12];
#pragma unroll
    for (int t = 0; t < 12; ++t) Q[t] = Qm[12 * slot + t];
    const double p[3] = {src[3 * i], src[3 * i + 1], src[3 * i + 2]};
    const int nsuper = tg.nsuper;
    float4 s0lo, s0hi;
    load_super0(search_tgt(tg), s0lo, s0hi);
    double q[3];
    xform(Q, p, q);
    // one round trip for all of it: left alone, the compiler sinks the
    // pose, source and box loads past the band test (a second round trip)
    asm volatile("" ::"v"(bv), "v"(qq.x), "v"(qq.y), "v"(qq.z), "v"(sk), "v"(q[0]), "v"(q[1]), "v"(q[2]),
                 "v"(s0lo.x), "v"(s0lo.y), "v"(s0lo.z), "v"(s0hi.x), "v"(s0hi.y), "v"(s0hi.z));
    if (bv == kNone) return -1;
    // the band test against the final winner; its band is also the culling bound
    const float band = exact_band_hi(__uint_as_float((unsigned)(bv >> 32)), qnorm(qq.x, qq.y, qq.z));
    if (!(__uint_as_float(sk & kKeyMask) <= band)) return -1;
    ++filed;
    const float Tb = band * 1.0001f;
    const float x = qq.x, y = qq.y, z = qq.z;  // the search's fp32 query: (float)(Q p - origin)
    const double* __restrict__ t64 = tg.xyz64;
    double bD = 3.0e300;
    int bI = 0x7FFFFFFF, bM = (int)(unsigned)bv;
    int nt = 0;  // listed tiles (wave-uniform)
    auto scan_listed = [&]() {  // four tiles at a time: every lane's four loads in flight together
        for (int c = 0; c < nt; c += 4) {
            int kk[4], in[4];
            double tx[4], ty[4], tz[4];
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) {
                kk[u4] = c + u4 < nt ? tl[c + u4] * kTile + lane : -1;
#ifdef ORPCD_BOUNDS_CHECK
                if (kk[u4] >= tg.ntiles * kTile) {
                    printf("[chk] scan_listed tile %d >= ntiles %d\n", tl[c + u4], tg.ntiles);
                    kk[u4] = -1;
                }
#endif
                const int k = kk[u4] >= 0 ? kk[u4] : 0;
                in[u4] = __float_as_int(ldg_f32(&tg.p4[k].w));  // p4 holds the padded tiles: -1 past the points
                // the fp64 points stop at npts: a padding lane reads point 0
                // (and is skipped below).  Reading past them faulted whenever
                // the buffer's end met an unmapped page (round 5).
                const size_t kx = k < tg.npts ? (size_t)k : 0;
                tx[u4] = ldg_f64(t64 + 3 * kx);
                ty[u4] = ldg_f64(t64 + 3 * kx + 1);
                tz[u4] = ldg_f64(t64 + 3 * kx + 2);
            }
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) {
                if (kk[u4] < 0 || in[u4] < 0) continue;  // past the list / padding
                const double tp[3] = {tx[u4], ty[u4], tz[u4]};
                const double D = d2_oracle(q, tp);
                if (D < bD || (D == bD && in[u4] < bI)) {
                    bD = D;
                    bI = in[u4];
                    bM = kk[u4];
                }
            }
        }
        nt = 0;
    };
    // candidate tiles: their boxes are tested four surviving super-tiles
    // at a time and the survivors listed in LDS
    const unsigned long long sm0 = __ballot(lane < nsuper && box_d2_plain(x, y, z, s0lo, s0hi) <= Tb);
    for (int sb = 0; sb < nsuper; sb += 64) {
        const int u = sb + lane;
        unsigned long long sm = sm0;
        if (sb > 0) {
            const int uu = u < nsuper ? u : 0;
            sm = __ballot(u < nsuper && box_d2_plain(x, y, z, ldg_f4(tg.slo + uu), ldg_f4(tg.shi + uu)) <= Tb);
        }
        while (sm) {
            int su4[4];
            bool ok[4];
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) {
                su4[u4] = sm ? sb + __builtin_ctzll(sm) : -1;
                sm &= sm - 1;
                const int t = su4[u4] * kSuper + lane;
                ok[u4] = su4[u4] >= 0 && t < tg.ntiles;
                const int tt = ok[u4] ? t : 0;
                const float4 lo = ldg_f4(tg.tlo + tt), hi = ldg_f4(tg.thi + tt);
                ok[u4] = ok[u4] && box_d2_plain(x, y, z, lo, hi) <= Tb;
            }
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) {
                unsigned long long tm = __ballot(ok[u4]);
                const int cnt = __builtin_popcountll(tm);
                if (nt + cnt > kExactList) scan_listed();  // the list is full: scan it first
                const int pos = nt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(tm >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((unsigned)tm, 0));
                if (ok[u4]) tl[pos] = su4[u4] * kSuper + lane;
                nt += cnt;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    scan_listed();
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {  // lexicographic (d^2, input index) over the wave
        const double oD = __shfl_xor(bD, o);
        const int oI = __shfl_xor(bI, o), oM = __shfl_xor(bM, o);
        if (oD < bD || (oD == bD && oI < bI)) {
            bD = oD;
            bI = oI;
            bM = oM;
        }
    }
    return bM;
}

// The entries of this pass's list, one per wave at a time (entries gw, gw + nw,
// ...).  kMark: every entry's final winner is stored with kResolvedBit, one
// 64-bit agent-scope atomic store (no fence: the flag and the answer are one
// word), for the fused accumulation's waiting threads.
template <bool kMark>
__device__ __forceinline__ void exact_entries(unsigned gw, unsigned nw, const double* __restrict__ src, int N,
                                              const double* __restrict__ Qm, const TargetDesc* __restrict__ tdesc,
                                              const float4* __restrict__ q32, const ExactArgs& ex,
                                              unsigned long long* __restrict__ best, int* __restrict__ tl) {
    const int lane = threadIdx.x & 63;
    // the first entry is read beside the count (the list holds at least one
    // entry per wave of the grid; an entry past the count is ignored)
    unsigned long long ent0 = ex.list[gw];
    const unsigned n = __builtin_amdgcn_readfirstlane(*ex.cnt);
    if (gw == 0 && lane == 0) *ex.cnt_next = 0u;
    unsigned filed = 0;  // this wave's re-searched queries (statistics)
    for (unsigned e = gw; e < n; e += nw) {
        if (e != gw) ent0 = ex.list[e];
        const unsigned long long ent =
            ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(ent0 >> 32)) << 32) |
            (unsigned)__builtin_amdgcn_readfirstlane((unsigned)ent0);
        unsigned long long bv = kNone;
        const int m = exact_entry(ent, src, N, Qm, tdesc, q32, ex, best, tl, bv, filed);
        const size_t qi = (size_t)(ent >> 40) * N + (unsigned)ent;
        if (lane == 0) {
            const unsigned long long fin = m >= 0 ? (bv & 0xFFFFFFFF00000000ull) | (unsigned)m : bv;
            if constexpr (kMark)
                __hip_atomic_store(best + qi, fin | kResolvedBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (m >= 0)
                best[qi] = fin;
        }
        // the next entry's list writes follow this entry's reads of tl
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0 && filed) atomicAdd(ex.total, (unsigned long long)filed);
}

__global__ __launch_bounds__(256) void nn_exact_kernel(const double* __restrict__ src, int N,
                                                       const double* __restrict__ Qm,
                                                       const TargetDesc* __restrict__ tdesc,
                                                       const float4* __restrict__ q32, ExactArgs ex,
                                                       unsigned long long* __restrict__ best) {
    __shared__ int tlist[4][kExactList];  // a wave's listed candidate tiles
    const unsigned gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), nw = gridDim.x * (blockDim.x >> 6);
    exact_entries<false>(gw, nw, src, N, Qm, tdesc, q32, ex, best, tlist[threadIdx.x >> 6]);
}


// --------------------------------------------------------------------------
// Accumulation kernels: accum_qpt(N) queries per thread (grid = (blocks per start,
// running starts), 256 threads), each thread summing its queries' terms in
// registers; then a fixed-order block reduction (DPP within rows of 16 lanes,
// the four row sums, then the four waves) into one partial per block.  The
// chosen correspondence is written back as the next pass's seed.
// --------------------------------------------------------------------------
// queries per thread.  A function of N only, so the fixed-order reduction is
// the same for every batch composition.  Measured at C2: 1 (4x the blocks, 4x
// the partials for the solve) 18.5 ms per multistart, 2: 17.9, 4: 17.8.
// queries per accumulation thread; fixed (not per batch) so that a start's
// sums never depend on the batch it runs in.  C2 batches of 1/8/30/64 starts:
// 4: 0.54/4.72/15.07/24.36 ms, 2: 0.53/4.71/15.13/24.37, 1: 0.56/4.83/15.71/25.31
#ifndef ORPCD_ACCUM_QPT
#define ORPCD_ACCUM_QPT 4
#endif
constexpr __host__ __device__ __forceinline__ int accum_qpt(int64_t) { return ORPCD_ACCUM_QPT; }

template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, Ctrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), Ctrl, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// wave sum in a fixed order (identical in every lane): rows of 16 by DPP, then
// (row0 + row1) + (row2 + row3)
__device__ __forceinline__ double wave_sum_fixed(double v) {
    v += dpp_f64<0xb1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f64<0x4e>(v);   // quad_perm [2,3,0,1]
    v += dpp_f64<0x141>(v);  // row_half_mirror
    v += dpp_f64<0x140>(v);  // row_mirror
    auto rl = [&](int k) {
        const long long b = __double_as_longlong(v);
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, k);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), k);
        return __longlong_as_double(((long long)hi << 32) | lo);
    };
    return (rl(0) + rl(16)) + (rl(32) + rl(48));
}

// Block reduction of NV per-thread values into partial[slot, block][slot_of(v)].
template <int NV, typename SlotOf>
__device__ __forceinline__ void block_partial(const double* acc, double (*red)[NV], SlotOf slot_of,
                                              double* __restrict__ out) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double s = wave_sum_fixed(acc[v]);
        if (lane == 0) red[wid][v] = s;
    }
    __syncthreads();
    if (threadIdx.x < kNacc) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (slot_of(v) == (int)threadIdx.x) s = ((red[0][v] + red[1][v]) + red[2][v]) + red[3][v];
        out[threadIdx.x] = s;
    }
}

// Fixed-order reduction of one start's block partials (lane-strided, then
// the wave).
__device__ __forceinline__ void reduce_partials(const double* __restrict__ partial, int slot, int nblk,
                                                double s[kNacc]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int v = 0; v < kNacc; ++v) s[v] = 0.0;
    for (int b = lane; b < nblk; b += 64) {
        const double* pp = partial + ((size_t)slot * nblk + b) * kPartialStride;
        // every 16 B load of the partial issued before the first add: one
        // memory round trip (the partials were written on other XCDs and miss
        // this L2), not one per pair of terms
        static_assert(kPartialStride >= kNacc + 1 && kPartialStride % 2 == 0, "partial stride");
        double2 t[(kNacc + 1) / 2];
#pragma unroll
        for (int u = 0; u < (kNacc + 1) / 2; ++u) t[u] = reinterpret_cast<const double2*>(pp)[u];
#pragma unroll
        for (int v = 0; v < kNacc; ++v) s[v] += (v & 1) ? t[v >> 1].y : t[v >> 1].x;
    }
#pragma unroll
    for (int v = 0; v < kNacc; ++v) s[v] = wave_sum_fixed(s[v]);
}

struct SolveArgs {
    double* T;
    double* Q;
    double* R;
    const double* G;
    double* prev;
    int32_t* done;
    double* out_fit;
    double* out_rmse;
    int32_t* out_iters;
    int64_t* out_ncorr;
};

// --------------------------------------------------------------------------
// One start's convergence test (RegistrationICP), 6x6 solve (or Umeyama) and
// pose update from its 29 reduced sums.
// --------------------------------------------------------------------------
// Called by all 64 lanes of one wave with the same (uniform) sums; the 6x6
// system is solved wave-parallel (det6_wave / ldlt_solve6_wave, bit-identical
// to the single-lane det6 / ldlt_solve6); lane 0 stores.  Returns true when
// the start finished.
// A start's pose state as the solve reads it (previous fitness / rmse, T, G).
// One vector load per lane (lane 0-1 prev, 2-17 T, 18-29 G), issued by the
// caller before its reduction so that it overlaps it, then broadcast by
// readlanes (no scalar loads: their SGPR pressure serialised them).
struct PoseIn {
    double pf, pr, T[16], G[12];
};

__device__ __forceinline__ double pose_lane_load(int slot, const SolveArgs& a) {
    const int lane = threadIdx.x & 63;
    const double* p = lane < 2 ? a.prev + 2 * slot + lane
                      : lane < 18 ? a.T + 16 * slot + (lane - 2)
                      : lane < 30 ? a.G + 12 * slot + (lane - 18)
                                  : a.prev + 2 * slot;
    return *p;
}

// every lane of the wave (readlane)
__device__ __forceinline__ void pose_from_lanes(double v, PoseIn& p) {
    p.pf = rl64(v, 0);
    p.pr = rl64(v, 1);
#pragma unroll
    for (int t = 0; t < 16; ++t) p.T[t] = rl64(v, 2 + t);
#pragma unroll
    for (int t = 0; t < 12; ++t) p.G[t] = rl64(v, 18 + t);
}

// ldlt_x: null, or (two-wave solve: every caller's block is two waves holding
// the same sums) an LDS slot for x -- wave 1 runs the LDLT while wave 0
// evaluates the determinant check, joined through LDS (the two are
// independent: the LDLT's x is used only when the check passes).  Wave 0
// alone stores; the values are those of the one-wave solve bit for bit.
template <int kEst>  // kEst 0: GeneralizedICP, 1: PointToPoint
__device__ bool solve_start(int slot, const double s[kNacc], int64_t N, int pass, int max_iter, double rel_fit,
                            double rel_rmse, const SolveArgs& a, const PoseIn& pin, double* ldlt_x = nullptr) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    const int lane = threadIdx.x & 63;
    const bool store = ldlt_x == nullptr || (threadIdx.x >> 6) == 0;  // the storing wave
    const double cnt = s[28];
    const double fit = cnt > 0 ? cnt / (double)N : 0.0;
    const double rmse = cnt > 0 ? sqrt(s[27] / cnt) : 0.0;
    const double pf = pin.pf, pr = pin.pr;
    const bool converged = pass >= 1 && fabs(pf - fit) < rel_fit && fabs(pr - rmse) < rel_rmse;
    if (converged || pass >= max_iter) {
        if (lane == 0 && store) {
            a.out_fit[slot] = fit;
            a.out_rmse[slot] = rmse;
            a.out_iters[slot] = pass;
            a.out_ncorr[slot] = (int64_t)cnt;
            a.done[slot] = 1;
        }
        return true;
    }
    if (lane == 0 && store) {
        a.prev[2 * slot] = fit;
        a.prev[2 * slot + 1] = rmse;
    }

    double upd[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    if (cnt > 0 && kEst == 1) {
        umeyama_from_moments(s, cnt, upd);  // every lane, the same values
    } else if (cnt > 0 && ldlt_x) {
        double det = 0.0;
        if (!store) {  // wave 1: the LDLT (as below), x to LDS
            double JTJ[36], b[6], x[6];
            for (int r = 0; r < 6; ++r) b[r] = -s[21 + r];
            for (int i = 0, k = 0; i < 6; ++i)
                for (int j = i; j < 6; ++j, ++k) JTJ[6 * i + j] = JTJ[6 * j + i] = s[k];
            ldlt_solve6(JTJ, b, x);
            if (lane < 6) ldlt_x[lane] = x[lane];
        } else {       // wave 0: the determinant check
            double row[6];
            sym6_row(s, lane, row);
            det = det6_wave(row, lane);
        }
        __syncthreads();
        if (!store) return false;
        if (!(fabs(det) < 1e-6 || isnan(det) || isinf(det))) {
            double x[6];
            for (int r = 0; r < 6; ++r) x[r] = ldlt_x[r];
            vec6_to_m4_wave(x, upd, lane);
        }
    } else if (cnt > 0) {
        double row[6], b[6];
        sym6_row(s, lane, row);
        for (int r = 0; r < 6; ++r) b[r] = -s[21 + r];
        const double det = det6_wave(row, lane);
        if (!(fabs(det) < 1e-6 || isnan(det) || isinf(det))) {
            // LDLT as the single-lane routine on every lane (uniform values):
            // 6.5k cycles against 8.7k for ldlt_solve6_wave, whose readlane
            // chains outweigh the row parallelism (tools/solve_bench.hip);
            // det6_wave (2.2k vs 2.5k) and vec6_to_m4_wave (1.2k vs 3.1k) pay.
            // All are bit-identical to each other (test_wave_solve_bit_identical).
            double JTJ[36], x[6];
            for (int i = 0, k = 0; i < 6; ++i)
                for (int j = i; j < 6; ++j, ++k) JTJ[6 * i + j] = JTJ[6 * j + i] = s[k];
            ldlt_solve6(JTJ, b, x);
            vec6_to_m4_wave(x, upd, lane);
        }
    }
    double Tn[16];
    m4_mul(upd, pin.T, Tn);
    if (lane == 0)
        for (int t = 0; t < 16; ++t) a.T[16 * slot + t] = Tn[t];
    // Q = Tn * [G; 0 0 0 1]  (3x4), R = Tn[:3,:3]
    const double* G = pin.G;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 4; ++c) {
            double v = Tn[4 * r + 0] * G[c] + Tn[4 * r + 1] * G[4 + c] + Tn[4 * r + 2] * G[8 + c];
            if (c == 3) v += Tn[4 * r + 3];
            if (lane == 0) a.Q[12 * slot + 4 * r + c] = v;
        }
        if (lane == 0)
            for (int c = 0; c < 3; ++c) a.R[9 * slot + 3 * r + c] = Tn[4 * r + c];
    }
    return false;
}

// Test entry (orpcd_test_solve6): for each of n systems (21 upper JTJ + 6 JTr),
// det, x and the update matrix by the single-lane code (out_serial) and by the
// wave-parallel code (out_wave); 23 doubles each.
__global__ __launch_bounds__(64) void solve6_test_kernel(const double* __restrict__ sums, int n,
                                                         double* __restrict__ out_serial,
                                                         double* __restrict__ out_wave) {
    const int sys = blockIdx.x, lane = threadIdx.x;
    if (sys >= n) return;
    const double* s = sums + (size_t)27 * sys;
    double bb[6];
    for (int r = 0; r < 6; ++r) bb[r] = -s[21 + r];
    if (lane == 0) {
        double JTJ[36], x[6] = {0, 0, 0, 0, 0, 0};
        double upd[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 6; ++c) JTJ[6 * r + c] = r <= c ? s[ut(r, c)] : s[ut(c, r)];
        const double det = det6(JTJ);
        if (!(fabs(det) < 1e-6 || isnan(det) || isinf(det))) {
            ldlt_solve6(JTJ, bb, x);
            vec6_to_m4(x, upd);
        }
        double* o = out_serial + (size_t)23 * sys;
        o[0] = det;
        for (int i = 0; i < 6; ++i) o[1 + i] = x[i];
        for (int i = 0; i < 16; ++i) o[7 + i] = upd[i];
    }
    double row[6], x[6] = {0, 0, 0, 0, 0, 0};
    double upd[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    sym6_row(s, lane, row);
    const double det = det6_wave(row, lane);
    if (!(fabs(det) < 1e-6 || isnan(det) || isinf(det))) {
        ldlt_solve6_wave(row, bb, x, lane);
        vec6_to_m4_wave(x, upd, lane);
    }
    if (lane == 0) {
        double* o = out_wave + (size_t)23 * sys;
        o[0] = det;
        for (int i = 0; i < 6; ++i) o[1 + i] = x[i];
        for (int i = 0; i < 16; ++i) o[7 + i] = upd[i];
    }
}

hipError_t launch_solve6_test(const double* sums, int n, double* out_serial, double* out_wave, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    solve6_test_kernel<<<(unsigned)n, 64, 0, s>>>(sums, n, out_serial, out_wave);
    return hipGetLastError();
}

// The GICP normal-equation terms of accumulation block `ablk` of start
// `slot` (queries (ablk * qpt + k) * 256 + threadIdx.x): this thread's sums,
// in query order k.  Writes the next pass's seed (prevnn).  sec != null (the
// fused exact mode): a query listed for the re-search (sec[] set) waits until
// its entry is resolved and reads its final winner then.
__device__ __forceinline__ void gicp_block_terms(int slot, int ablk, const double* __restrict__ src,
                                                 const double* __restrict__ scov, int N,
                                                 const double* __restrict__ tgt64, const double* __restrict__ tcov,
                                                 const double* __restrict__ Qm, const double* __restrict__ Rm,
                                                 double r2, unsigned long long* __restrict__ best,
                                                 int32_t* __restrict__ prevnn, double acc[kNacc], double om,
                                                 unsigned* __restrict__ sec = nullptr,
                                                 unsigned long long* __restrict__ total = nullptr) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
#pragma unroll
    for (int v = 0; v < kNacc; ++v) acc[v] = 0.0;
    double Q[12], R[9];
#pragma unroll
    for (int t = 0; t < 12; ++t) Q[t] = Qm[12 * slot + t];
#pragma unroll
    for (int t = 0; t < 9; ++t) R[t] = Rm[9 * slot + t];
    // Loads in two rounds for all of the thread's queries (best, source point
    // and covariance; then the target point and covariance of each match),
    // not three dependent round trips per query; the terms are then added in
    // query order exactly as before.  Loads of a missing match read index 0.
    constexpr int kQ = accum_qpt(0);
    unsigned long long bv[kQ];
    unsigned sk[kQ];
    double p[kQ][3], cs[kQ][kCovW], t3[kQ][3], ct[kQ][kCovW];
#pragma unroll
    for (int k = 0; k < kQ; ++k) {
        const int i = (ablk * kQ + k) * 256 + threadIdx.x;
        const int ii = i < N ? i : 0;
        bv[k] = i < N ? best[(size_t)slot * N + i] : kNone;
        sk[k] = sec && i < N ? sec[(size_t)slot * N + i] : 0xFFFFFFFFu;
#pragma unroll
        for (int c = 0; c < 3; ++c) p[k][c] = src[3 * ii + c];
        const double* cs6 = scov + ((size_t)slot * N + ii) * kCovW;
#pragma unroll
        for (int c = 0; c < kCovW; ++c) cs[k][c] = cs6[c];
    }
    if (sec) {
#pragma unroll
        for (int k = 0; k < kQ; ++k) {
            if (sk[k] == 0xFFFFFFFFu) continue;  // not listed: the search's winner is final
            const size_t qi = (size_t)slot * N + (ablk * kQ + k) * 256 + threadIdx.x;
            // bounded: a wave never waits forever (2^22 polls); a time-out keeps
            // the search's winner and counts in stats (exact_filed >= 2^40)
            unsigned polls = 0;
            unsigned long long v = bv[k];
            while (!(v & kResolvedBit) && ++polls < (1u << 22)) {
                __builtin_amdgcn_s_sleep(1);
                v = __hip_atomic_load(best + qi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (!(v & kResolvedBit) && total) atomicAdd(total, 1ull << 40);
            bv[k] = v == kNone ? kNone : v & ~kResolvedBit;
        }
    }
#pragma unroll
    for (int k = 0; k < kQ; ++k) {
        const int i = (ablk * kQ + k) * 256 + threadIdx.x;
        int j = bv[k] == kNone ? -1 : (int)(unsigned)(bv[k] & 0xffffffffu);
#ifdef ORPCD_BOUNDS_CHECK
        if (j >= (1 << 26) || j < -1) {
            printf("[chk] accum slot %d i %d best %llx\n", slot, i, bv[k]);
            j = -1;
            bv[k] = kNone;
        }
#endif
        if (i < N) prevnn[(size_t)slot * N + i] = j >= 0 ? j : kNoMatch;
        const int jj = j >= 0 ? j : 0;
#pragma unroll
        for (int c = 0; c < 3; ++c) t3[k][c] = ldg_f64(tgt64 + 3 * jj + c);
#pragma unroll
        for (int c = 0; c < kCovW; ++c) ct[k][c] = ldg_f64(tcov + (size_t)jj * kCovW + c);
    }
#pragma unroll
    for (int k = 0; k < kQ; ++k) {
        if (bv[k] == kNone) continue;  // also every i >= N
        double q[3];
        xform(Q, p[k], q);
        const double d[3] = {q[0] - t3[k][0], q[1] - t3[k][1], q[2] - t3[k][2]};
        const double d2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        if (!(d2 < r2)) continue;
#if ORPCD_NORMAL_COV
        // Cs + Ct = 2 I - (1 - eps) (a a^T + b b^T), a = R e_s (the source's
        // effective normal in the current pose: R (I - (1-eps) e e^T) R^T), b = e_t
        const double* es = cs[k];
        const double* b = ct[k];
        const double a[3] = {R[0] * es[0] + R[1] * es[1] + R[2] * es[2], R[3] * es[0] + R[4] * es[1] + R[5] * es[2],
                             R[6] * es[0] + R[7] * es[1] + R[8] * es[2]};
        const Sym3 Mm{2.0 - om * (a[0] * a[0] + b[0] * b[0]), -om * (a[0] * a[1] + b[0] * b[1]),
                      -om * (a[0] * a[2] + b[0] * b[2]),      2.0 - om * (a[1] * a[1] + b[1] * b[1]),
                      -om * (a[1] * a[2] + b[1] * b[2]),      2.0 - om * (a[2] * a[2] + b[2] * b[2])};
#else
        (void)om;
        const double* cs6 = cs[k];
        const double* ct6 = ct[k];
        Sym3 Cs{cs6[0], cs6[1], cs6[2], cs6[3], cs6[4], cs6[5]};
        Cs = rotate_sym(R, Cs);
        const Sym3 Mm{Cs.xx + ct6[0], Cs.xy + ct6[1], Cs.xz + ct6[2], Cs.yy + ct6[3], Cs.yz + ct6[4],
                      Cs.zz + ct6[5]};
#endif
        const Sym3 P = sym3_inverse(Mm);
        const double Pm[3][3] = {{P.xx, P.xy, P.xz}, {P.xy, P.yy, P.yz}, {P.xz, P.yz, P.zz}};
        // g = P d ; JTr = [q x g ; g]
        const double g[3] = {P.xx * d[0] + P.xy * d[1] + P.xz * d[2], P.xy * d[0] + P.yy * d[1] + P.yz * d[2],
                             P.xz * d[0] + P.yz * d[1] + P.zz * d[2]};
        double qg[3];
        cross3(q, g, qg);
        acc[21] += qg[0];
        acc[22] += qg[1];
        acc[23] += qg[2];
        acc[24] += g[0];
        acc[25] += g[1];
        acc[26] += g[2];
        // SP = [q]x P (column b = q x P[:,b]);  TL row a = q x SP[a,:]
        double SP[3][3];
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const double col[3] = {Pm[0][b], Pm[1][b], Pm[2][b]};
            double c3[3];
            cross3(q, col, c3);
            SP[0][b] = c3[0];
            SP[1][b] = c3[1];
            SP[2][b] = c3[2];
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double tl[3];
            cross3(q, SP[a], tl);
#pragma unroll
            for (int b = a; b < 3; ++b) acc[ut(a, b)] += tl[b];
#pragma unroll
            for (int b = 0; b < 3; ++b) acc[ut(a, 3 + b)] += SP[a][b];
        }
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = a; b < 3; ++b) acc[ut(3 + a, 3 + b)] += Pm[a][b];
        acc[27] += d2;
        acc[28] += 1.0;
    }
}

// ORPCD_ACCUM_WAVES: a register budget for the accumulation (A/B builds); unset,
// the compiler's choice (214 VGPRs, 2 waves/SIMD)
#ifdef ORPCD_ACCUM_WAVES
#define ORPCD_ACCUM_ATTR __attribute__((amdgpu_waves_per_eu(ORPCD_ACCUM_WAVES, 8)))
#else
#define ORPCD_ACCUM_ATTR
#endif
__global__ __launch_bounds__(256) ORPCD_ACCUM_ATTR void gicp_accum_kernel(
    const double* __restrict__ src, const double* __restrict__ scov, int N, const TargetDesc* __restrict__ tdesc,
    TgtBounds tb, const int32_t* __restrict__ active, const double* __restrict__ Qm,
    const double* __restrict__ Rm, const int32_t* __restrict__ done, double r2,
    unsigned long long* __restrict__ best, int32_t* __restrict__ prevnn, double* __restrict__ partial,
    int nblk, double om) {
    const int slot = active[blockIdx.y];
    if (done[slot]) return;
    const TargetDesc& tg = tdesc[target_of_row(tb, blockIdx.y)];
    __shared__ double red[4][kNacc];
    double acc[kNacc];
    gicp_block_terms(slot, blockIdx.x, src, scov, N, tg.xyz64, tg.tcov, Qm, Rm, r2, best, prevnn, acc, om);
    block_partial<kNacc>(acc, red, [](int v) { return v; }, partial + ((size_t)slot * nblk + blockIdx.x) * kPartialStride);
}

// Exact mode, fused: the re-search of the listed queries and the
// accumulation in one launch (1-D grid).  Blocks [0, nexact) work the list one
// entry per wave and publish each entry's final winner (with kResolvedBit);
// the accumulation blocks after them ((row, block) = divmod(b -
// nexact, nblk)) wait only for their own listed queries (~0.2%), so the
// re-search's chain of round trips overlaps the accumulation instead of
// preceding it (round 2: a kernel of its own, 13-23 us per pass at C2).  No
// deadlock: a block waits only for blocks of lower index, which the
// dispatcher placed before it (each XCD dispatches its blocks in order), and
// those never wait.
__global__ __launch_bounds__(256) ORPCD_ACCUM_ATTR void gicp_accum_exact_kernel(
    const double* __restrict__ src, const double* __restrict__ scov, int N, const TargetDesc* __restrict__ tdesc,
    TgtBounds tb, const int32_t* __restrict__ active, const double* __restrict__ Qm,
    const double* __restrict__ Rm, const int32_t* __restrict__ done, double r2,
    unsigned long long* __restrict__ best, int32_t* __restrict__ prevnn, double* __restrict__ partial,
    int nblk, int nexact, const float4* __restrict__ q32, ExactArgs ex, double om) {
    __shared__ double red[4][kNacc];
    __shared__ int tlist[4][kExactList];
    if ((int)blockIdx.x < nexact) {
        exact_entries<true>(blockIdx.x * 4 + (threadIdx.x >> 6), (unsigned)nexact * 4, src, N, Qm, tdesc, q32, ex,
                            best, tlist[threadIdx.x >> 6]);
        return;
    }
    const int b = (int)blockIdx.x - nexact, row = b / nblk, bx = b - row * nblk;
    const int slot = active[row];
    if (done[slot]) return;
    const TargetDesc& tg = tdesc[target_of_row(tb, row)];
    double acc[kNacc];
    gicp_block_terms(slot, bx, src, scov, N, tg.xyz64, tg.tcov, Qm, Rm, r2, best, prevnn, acc, om, ex.sec, ex.total);
    block_partial<kNacc>(acc, red, [](int v) { return v; }, partial + ((size_t)slot * nblk + bx) * kPartialStride);
}

// PointToPoint accumulation (TransformationEstimationPointToPoint, Eigen::
// umeyama): per correspondence the fp64 re-check as above, then the first
// moments  sum src (0..2), sum dst (3..5), sum dst_a src_b (6..14), sum d^2
// (27), count (28) in the partial layout of the GICP terms.
constexpr int kP2PTerms = 17;
__device__ __forceinline__ int p2p_slot(int v) { return v < 15 ? v : 12 + v; }  // 15 -> 27, 16 -> 28

__device__ __forceinline__ void p2p_block_terms(int slot, int ablk, const double* __restrict__ src, int N,
                                                const double* __restrict__ tgt64, const double* __restrict__ Qm,
                                                double r2, unsigned long long* __restrict__ best,
                                                int32_t* __restrict__ prevnn, double acc[kP2PTerms]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
#pragma unroll
    for (int v = 0; v < kP2PTerms; ++v) acc[v] = 0.0;
    double Q[12];
#pragma unroll
    for (int t = 0; t < 12; ++t) Q[t] = Qm[12 * slot + t];
    const int qpt = accum_qpt(N);
    for (int k = 0; k < qpt; ++k) {
        const int i = (ablk * qpt + k) * 256 + threadIdx.x;
        if (i >= N) break;
        const unsigned long long v = best[(size_t)slot * N + i];
        const int j = v == kNone ? -1 : (int)(unsigned)(v & 0xffffffffu);
        prevnn[(size_t)slot * N + i] = j >= 0 ? j : kNoMatch;
        if (j < 0) continue;
        const double p[3] = {src[3 * i], src[3 * i + 1], src[3 * i + 2]};
        double q[3];
        xform(Q, p, q);
        const double t3[3] = {tgt64[3 * j], tgt64[3 * j + 1], tgt64[3 * j + 2]};
        const double d[3] = {q[0] - t3[0], q[1] - t3[1], q[2] - t3[2]};
        const double d2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        if (!(d2 < r2)) continue;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            acc[a] += q[a];
            acc[3 + a] += t3[a];
#pragma unroll
            for (int b = 0; b < 3; ++b) acc[6 + 3 * a + b] += t3[a] * q[b];
        }
        acc[15] += d2;
        acc[16] += 1.0;
    }
}

__global__ __launch_bounds__(256) void p2p_accum_kernel(const double* __restrict__ src, int N,
                                                        const TargetDesc* __restrict__ tdesc, TgtBounds tb,
                                                        const int32_t* __restrict__ active,
                                                        const double* __restrict__ Qm,
                                                        const int32_t* __restrict__ done, double r2,
                                                        unsigned long long* __restrict__ best,
                                                        int32_t* __restrict__ prevnn, double* __restrict__ partial,
                                                        int nblk) {
    const int slot = active[blockIdx.y];
    if (done[slot]) return;
    __shared__ double red[4][kP2PTerms];
    double acc[kP2PTerms];
    p2p_block_terms(slot, blockIdx.x, src, N, tdesc[target_of_row(tb, blockIdx.y)].xyz64, Qm, r2, best,
                           prevnn, acc);
    block_partial<kP2PTerms>(acc, red, p2p_slot, partial + ((size_t)slot * nblk + blockIdx.x) * kPartialStride);
}

// --------------------------------------------------------------------------
// Per-start reduction of the block partials, convergence test
// (RegistrationICP), and the 6x6 solve + pose update.  One wave per start.
// sums_in != null: the sums are given
// (row-sharded mode, already all-reduced over ranks) and the partials are
// not read.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(64) void reduce_partials_kernel(const double* __restrict__ partial, int slot, int nblk,
                                                             double* __restrict__ sums) {
    double s[kNacc];
    reduce_partials(partial, slot, nblk, s);
    if (threadIdx.x == 0)
        for (int v = 0; v < kNacc; ++v) sums[v] = s[v];
}

// kSolveWaves: one, or two for the GeneralizedICP solve (the determinant
// check and the LDLT in separate waves, solve_start; ORPCD_SOLVE_WAVES A/B).
#ifndef ORPCD_SOLVE_WAVES
#define ORPCD_SOLVE_WAVES 2
#endif
template <int kEst>
constexpr int solve_waves() { return kEst == 0 ? ORPCD_SOLVE_WAVES : 1; }
template <int kEst>  // 0: GeneralizedICP, 1: PointToPoint
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(1, 2))) void icp_solve_kernel(const int32_t* __restrict__ active,
                                                        const double* __restrict__ partial, int nblk,
                                                        const double* __restrict__ sums_in, int64_t N, int pass,
                                                        int max_iter, double rel_fit, double rel_rmse, SolveArgs a) {
    __shared__ double ldlt_x[8];
    const int slot = active[blockIdx.x];
    // the done flag, the partials and the pose are loaded together (one memory
    // round trip after active[]); a finished start only wasted the loads
    const int finished = a.done[slot];
    const double pose = pose_lane_load(slot, a);
    double s[kNacc];
    if (sums_in) {
#pragma unroll
        for (int v = 0; v < kNacc; ++v) s[v] = sums_in[v];
    } else {
        reduce_partials(partial, slot, nblk, s);
    }
    if (finished) return;
    PoseIn pin;
    pose_from_lanes(pose, pin);
    solve_start<kEst>(slot, s, N, pass, max_iter, rel_fit, rel_rmse, a, pin,
                      solve_waves<kEst>() == 2 ? ldlt_x : nullptr);
}

int seed_stride_for(int64_t ntiles, int reps = 512);

// The seed grid of a target (CloudLayout::sgrid): cell i of kSeedGrid^3 over
// the target's bounding box holds the Morton index of a target near its
// centre.  Only a bound seed: any real target would do (a bound never changes
// an answer, tests/test_gpu_seed.py), the nearest is the best.
//
// Built by jump flooding (round 5): every target point offers itself to its
// own cell (64-bit atomicMin on (fp32 d^2 to the centre, index)), then rounds
// with steps 32, 16, 8, 4, 2, 1, 1 let each cell take the best of the seeds of
// its 26 neighbours at that step (JFA+1: the nearest point to the centre for
// nearly every cell, a near one otherwise).  Rounds 1-4 searched every cell
// centre with the culled 1-NN search instead: exact, but its 110,592 centres
// in raster order make loose wave boxes, and cells far from the surface have
// large bounds -- 0.38 ms per 50k-point target, 6.3 ms per 1M-point target
// (C5's set-up, profiles/r05_c5_kernel_stats.csv); these ten launches are
// independent of the cloud size but for the scatter.
__device__ __forceinline__ int seed_axis(float x, float lo, float inv) {
    return min(kSeedGrid - 1, max(0, (int)((x - lo) * inv)));  // the query transform's clamp
}
__device__ __forceinline__ float seed_centre(float lo, float inv, int c) {
    return lo + ((float)c + 0.5f) * (1.0f / inv);
}
__device__ __forceinline__ unsigned long long seed_key(float d2, int j) {
    return ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)j;
}
__global__ __launch_bounds__(256) void seed_scatter_kernel(const TargetDesc* __restrict__ tdesc, int first) {
    const TargetDesc& tg = tdesc[first + blockIdx.y];
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= tg.npts) return;
    const float4 p = tg.p4[j];
    const int cx = seed_axis(p.x, tg.sg_lo[0], tg.sg_inv[0]), cy = seed_axis(p.y, tg.sg_lo[1], tg.sg_inv[1]),
              cz = seed_axis(p.z, tg.sg_lo[2], tg.sg_inv[2]);
    const float d2 = d2f(seed_centre(tg.sg_lo[0], tg.sg_inv[0], cx), seed_centre(tg.sg_lo[1], tg.sg_inv[1], cy),
                         seed_centre(tg.sg_lo[2], tg.sg_inv[2], cz), p);
    atomicMin(tg.sgk + (cx * kSeedGrid + cy) * kSeedGrid + cz, seed_key(d2, j));
}
// one flooding round: key_out[c] = the best of key_in over c and its 26
// neighbours at `step` (out = 0xFF.. fill when nothing reached c yet);
// last != 0: the grid's indices are written instead of the next keys
__global__ __launch_bounds__(256) void seed_jfa_kernel(const TargetDesc* __restrict__ tdesc, int first, int step,
                                                       int in_half, int last) {
    constexpr int G = kSeedGrid, G3 = G * G * G;
    const TargetDesc& tg = tdesc[first + blockIdx.y];
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= G3) return;
    const int cx = c / (G * G), cy = (c / G) % G, cz = c % G;
    const float qx = seed_centre(tg.sg_lo[0], tg.sg_inv[0], cx), qy = seed_centre(tg.sg_lo[1], tg.sg_inv[1], cy),
                qz = seed_centre(tg.sg_lo[2], tg.sg_inv[2], cz);
    const unsigned long long* in = tg.sgk + (size_t)in_half * G3;
    unsigned long long best = in[c];
    for (int dx = -1; dx <= 1; ++dx) {
        const int nx = cx + dx * step;
        if (nx < 0 || nx >= G) continue;
        for (int dy = -1; dy <= 1; ++dy) {
            const int ny = cy + dy * step;
            if (ny < 0 || ny >= G) continue;
            for (int dz = -1; dz <= 1; ++dz) {
                const int nz = cz + dz * step;
                if (nz < 0 || nz >= G || (dx | dy | dz) == 0) continue;
                const unsigned long long k = in[(nx * G + ny) * G + nz];
                if (k == ~0ull) continue;
                const int j = (int)(unsigned)k;
                const unsigned long long cand = seed_key(d2f(qx, qy, qz, tg.p4[j]), j);
                best = cand < best ? cand : best;
            }
        }
    }
    if (last)
        const_cast<int32_t*>(tg.sgrid)[c] = best == ~0ull ? 0 : (int)(unsigned)best;
    else
        tg.sgk[(size_t)(in_half ^ 1) * G3 + c] = best;
}

// The grid's buffer and frame (host side; the build is launch_seed_grids).
hipError_t prepare_seed_grid(CloudLayout& L) {
    constexpr int nq = kSeedGrid * kSeedGrid * kSeedGrid;
    hipError_t e = L.sgrid.ensure(nq);
    if (e != hipSuccess) return e;
    if ((e = L.sgk.ensure((size_t)2 * nq)) != hipSuccess) return e;
    for (int a = 0; a < 3; ++a) {
        // the grid in the fp32 frame, a hair larger than the box; a
        // degenerate axis gets a tiny cell (every query clamps into a cell)
        const double ext = std::max(L.hi[a] - L.lo[a], 1e-30);
        const double cell = ext * (1.0 + 1e-6) / kSeedGrid;
        L.sg_lo[a] = (float)(L.lo[a] - L.org[a] - 1e-7 * ext);
        L.sg_inv[a] = (float)std::min(1.0 / cell, 1e30);  // finite: (x - lo) * inv never meets 0 * inf
    }
    return hipSuccess;
}

// The grids of targets [first, first + count) (their descriptors uploaded).
hipError_t launch_seed_grids(const TargetDesc* tdesc, int first, int count, int max_points,
                             unsigned long long* const* sgk, hipStream_t s) {
    constexpr int nq = kSeedGrid * kSeedGrid * kSeedGrid;
    hipError_t e;
    for (int k = 0; k < count; ++k)  // every cell empty (0xFF.. keys) in the first half
        if ((e = hipMemsetAsync(sgk[k], 0xFF, (size_t)nq * 8, s)) != hipSuccess) return e;
    seed_scatter_kernel<<<dim3((unsigned)((max_points + 255) / 256), (unsigned)count), 256, 0, s>>>(tdesc, first);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int steps[] = {32, 16, 8, 4, 2, 1, 1};
    constexpr int nsteps = sizeof(steps) / sizeof(steps[0]);
    static_assert(kSeedGrid <= 64, "the first flooding step must reach across the grid");
    for (int r = 0; r < nsteps; ++r) {
        seed_jfa_kernel<<<dim3((unsigned)((nq + 255) / 256), (unsigned)count), 256, 0, s>>>(tdesc, first, steps[r],
                                                                                            r & 1, r == nsteps - 1);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

// Kernel-level 1-NN (orpcd_nn1_radius, FGR's EvaluateRegistration): the same
// culled search on Morton-ordered targets (representative seed, S = 1), fp64
// re-check, no accumulation.  order != null: query slot i serves input query
// order[i] (the batch's Morton order, so that a wave's queries share a small
// box and the culling works; results land at the input index).
__global__ __launch_bounds__(kCBlock) void nn1_kernel(const int32_t* __restrict__ order,
                                                      const double* __restrict__ q64, int nq,
                                                      const float4* __restrict__ p4, const float4* __restrict__ tlo,
                                                      const float4* __restrict__ thi, const float4* __restrict__ qbox, int ntiles,
                                                      const float4* __restrict__ slo, const float4* __restrict__ shi,
                                                      int nsuper, int seed_stride, const double* __restrict__ tgt64,
                                                      const int32_t* __restrict__ tperm, double r2, float r2s,
                                                      int32_t* __restrict__ idx, double* __restrict__ d2o, Org3 org) {
    __shared__ float4 stage[kCWaves][kTile];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int i0 = blockIdx.x * kCBlockQ + wid * (64 * kCQPT) + lane;
    float qx[kCQPT], qy[kCQPT], qz[kCQPT], bound[kCQPT], bd[kCQPT];
    int bj[kCQPT];
#pragma unroll
    for (int k = 0; k < kCQPT; ++k) {
        const int s = i0 + 64 * k;
        const bool valid = s < nq;
        const int i = valid && order ? order[s] : s;
        qx[k] = valid ? (float)(q64[3 * i] - org.x) : 0.f;
        qy[k] = valid ? (float)(q64[3 * i + 1] - org.y) : 0.f;
        qz[k] = valid ? (float)(q64[3 * i + 2] - org.z) : 0.f;
        float b = valid ? r2s : 0.0f;
        if (valid)
            for (int t = 0; t < ntiles; t += seed_stride)
                b = fminf(b, seed_bound(d2f(qx[k], qy[k], qz[k], p4[t * kTile])));
        bound[k] = b;
    }
    culled_search<false>(stage[wid], p4, tlo, thi, qbox, ntiles, slo, shi, nsuper, 1, 1, 0, qx, qy, qz, bound, bd, bj,
                  lane < nsuper ? slo[lane] : make_float4(0.f, 0.f, 0.f, 0.f),
                  lane < nsuper ? shi[lane] : make_float4(0.f, 0.f, 0.f, 0.f));
#pragma unroll
    for (int k = 0; k < kCQPT; ++k) {
        const int s = i0 + 64 * k;
        if (s >= nq) continue;
        const int i = order ? order[s] : s;
        int j = bj[k];
        double dd = 0.0;
        if (j >= 0) {
            const double dx = q64[3 * i] - tgt64[3 * j], dy = q64[3 * i + 1] - tgt64[3 * j + 1],
                         dz = q64[3 * i + 2] - tgt64[3 * j + 2];
            dd = dx * dx + dy * dy + dz * dz;
            if (!(dd < r2)) {
                j = -1;
                dd = 0.0;
            }
        }
        idx[i] = j >= 0 ? tperm[j] : -1;
        d2o[i] = dd;
    }
}

int seed_stride_for(int64_t ntiles, int reps) {  // at most ~reps representatives per query
    return (int)std::max<int64_t>(1, (ntiles + reps - 1) / reps);
}

int search_splits(int nact, int blocks_per_start, int want) {
    const int64_t waves = (int64_t)nact * blocks_per_start * kCWaves;
    return (int)std::min<int64_t>(64, std::max<int64_t>(1, (want + waves - 1) / waves));
}

int accum_blocks(int64_t N) { return (int)((N + 256 * accum_qpt(N) - 1) / (256 * accum_qpt(N))); }

// uniform splits of a launch over nact running starts (the pass-0 split of
// the ordered dispatch too)
static int uniform_splits(const orpcd_ctx* c, int nact) {
    const int sblk = (int)((c->src.n + kCBlockQ - 1) / kCBlockQ);
    const int want = nact <= c->opt.small_batch ? c->opt.search_waves / 2 : c->opt.search_waves;
    return search_splits(nact, sblk, want);
}

// the ordered dispatch serves batches of at least sched_min_starts starts:
// below that its planning
// (one block per start, beside the transform) and the wave's item lookup
// cost more than the order gains (C2: 1 start 0.53 -> 0.65 ms, 8 starts
// 4.53 -> 4.59 ms; 30 starts 16.6 -> 15.0 ms, 104 starts 43.7 -> 37.8 ms;
// C5 1 start 1478 -> 1304 iterations/s)
bool sched_wanted(const orpcd_ctx* c, int B) { return c->opt.sched && B >= c->opt.sched_min_starts; }

// items per class: every item of a pass may fall in one class.  Pass 0:
// S0 * groups <= search_waves + groups (search_splits rounds up); later
// passes: sum ceil(cost / target) <= total / target + groups with target >=
// total / sched_items, or >= total / sched_item_budget under sched_cap_us,
// doubled against float rounding of the per-group quotients.
static int64_t sched_item_budget(const orpcd_ctx* c) {
    return c->opt.sched_cap_us > 0 ? (int64_t)c->opt.sched_items * c->opt.sched_cap_mult : c->opt.sched_items;
}
int sched_capacity(const orpcd_ctx* c, int B) {
    const int64_t NG = (c->src.n + 127) / 128;
    return (int)(std::max<int64_t>(sched_item_budget(c), c->opt.search_waves) + 2 * (int64_t)B * NG + 64);
}

// the ordered dispatch's planner arguments for the queries of `pass` (none
// when the batch runs the uniform dispatch)
static SchedX sched_x(const orpcd_ctx* c, int nact, int pass) {
    SchedX sx{};
    if (!c->sched_live) return sx;
    const size_t B = (size_t)c->sched_B;
    const size_t NG = (size_t)(c->src.n + 127) / 128;
    const int par = pass & 1;
    sx.wcost_prev = c->wcost.p + (size_t)(par ^ 1) * B * NG;
    sx.wcost_cur = c->wcost.p + (size_t)par * B * NG;
    sx.wtot_prev = c->wtot.p + (size_t)(par ^ 1) * kSchedTot;
    sx.cnt = c->wcnt.p + (size_t)par * kSchedClasses;
    sx.list = c->wlist.p;
    sx.cap = c->sched_cap;
    sx.NG = (int)NG;
    sx.have_cost = pass > c->pass_base;  // costs exist from the batch's second pass on
    sx.S0 = uniform_splits(c, nact);
    sx.inv_want = 1.0f / (float)c->opt.sched_items;
    sx.max_target = (float)c->opt.sched_cap_us * 100.0f;  // us -> s_memrealtime ticks (10 ns)
    sx.inv_max_items = 1.0f / (float)sched_item_budget(c);
    return sx;
}

// exact mode: the runner-up array and the statistics counter
static ExactArgs exact_args(const orpcd_ctx* c, int pass) {
    ExactArgs ex{};
    if (!c->exact_live) return ex;
    ex.sec = c->xsec.p;
    ex.list = c->xlist.p;
    ex.cnt = c->xcnt.p + (pass & 1);
    ex.cnt_next = c->xcnt.p + ((pass + 1) & 1);
    ex.total = c->xtotal.p;
    return ex;
}

// ORPCD_SYNC_LAUNCH=1 (debugging only): drain the stream after every launch
// of the pass loop and name the kernel whose execution failed
static hipError_t launched(const char* name, hipStream_t s) {
    hipError_t e = hipGetLastError();
    static const bool sync = getenv("ORPCD_SYNC_LAUNCH") != nullptr;
    if (e == hipSuccess && sync) {
        e = hipStreamSynchronize(s);
        if (e != hipSuccess) fprintf(stderr, "[orpcd] %s failed: %s\n", name, hipGetErrorString(e));
    }
    return e;
}

hipError_t launch_xform(const orpcd_ctx* c, int nact, int pass, double r2, hipStream_t s, const TgtBounds& tb) {
    const int N = (int)c->src.n;
    const SchedX sx = sched_x(c, nact, pass);
    xform_queries_kernel<<<dim3((unsigned)((N + 255) / 256) + (sx.list ? 1u : 0u), (unsigned)nact), 256, 0, s>>>(
        c->src.xyz64.p, N, c->active.p, c->Q.p, c->done.p, c->tdesc.p, tb, c->prevnn.p, search_r2(r2),
        c->opt.reseed, c->q32.p, c->best.p, c->gbox.p, sx, exact_args(c, pass));
    return launched("xform_queries_kernel", s);
}

TgtBounds one_target() {
    TgtBounds tb{};
    tb.n = 1;
    return tb;
}

TgtBounds target_bounds(const orpcd_ctx* c, const int32_t* act, int nact) {
    TgtBounds tb{};
    tb.n = c->batch_ntgt;
    for (int k = 0; k < tb.n; ++k) {
        int r = 0;  // act is increasing: the rows whose slot precedes target k + 1's first
        while (r < nact && act[r] < c->batch_first[k + 1]) ++r;
        tb.row_end[k] = r;
    }
    return tb;
}

void write_target_desc(const CloudLayout& L, const double* tcov, int seed_reps, bool seed_grid, TargetDesc& d) {
    d.p4 = L.p4.p;
    d.tlo = L.tlo.p;
    d.thi = L.thi.p;
    d.qbox = L.qbox.p;
    d.slo = L.slo.p;
    d.shi = L.shi.p;
    d.xyz64 = L.xyz64.p;
    d.tcov = tcov;
    d.ntiles = (int)L.ntiles;
    d.nsuper = (int)L.nsuper;
    d.seed_stride = seed_stride_for(L.ntiles, seed_reps);
    d.sg_on = seed_grid ? 1 : 0;
    d.ox = L.org[0];
    d.oy = L.org[1];
    d.oz = L.org[2];
    d.sgrid = L.sgrid.n ? L.sgrid.p : nullptr;
    d.sgk = L.sgk.n ? L.sgk.p : nullptr;
    d.npts = (int)L.n;
    for (int a = 0; a < 3; ++a) {
        d.sg_lo[a] = L.sg_lo[a];
        d.sg_inv[a] = L.sg_inv[a];
    }
}

static SolveArgs solve_args(const orpcd_ctx* c) {
    return SolveArgs{c->T.p,    c->Q.p,       c->R.p,        c->G.p,         c->prev.p,
                     c->done.p, c->out_fit.p, c->out_rmse.p, c->out_iters.p, c->out_ncorr.p};
}

#ifdef ORPCD_WAVETIME
// append the records of the last search launch (n wave slots) to $ORPCD_WAVETIME
static hipError_t dump_wavetime(int pass, int nact, int S, unsigned n, hipStream_t s) {
    const char* path = getenv("ORPCD_WAVETIME");
    if (!path) return hipSuccess;
    hipError_t e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    n = std::min(n, kWtMax);
    std::vector<unsigned long long> h((size_t)3 * n), keep;
    void* dp = nullptr;
    if ((e = hipGetSymbolAddress(&dp, HIP_SYMBOL(g_wt))) != hipSuccess) return e;
    if ((e = d2h(h.data(), dp, h.size() * 8, s)) != hipSuccess) return e;
    if ((e = hipMemset(dp, 0, h.size() * 8)) != hipSuccess) return e;
    for (unsigned k = 0; k < n; ++k)  // waves that searched (others exited early)
        if (h[3 * k] != 0) keep.insert(keep.end(), h.begin() + 3 * k, h.begin() + 3 * k + 3);
    if (FILE* f = fopen(path, "ab")) {
        const int hdr[4] = {pass, nact, S, (int)(keep.size() / 3)};
        fwrite(hdr, 4, 4, f);
        fwrite(keep.data(), 8, keep.size(), f);
        fclose(f);
    }
    return hipSuccess;
}
#endif

hipError_t launch_gicp_pass(const orpcd_ctx* c, int nact, int pass, double r2, hipStream_t s, hipEvent_t mid,
                            const TgtBounds& tb) {
    const int N = (int)c->src.n;
    const int sblk = (N + kCBlockQ - 1) / kCBlockQ;
    hipError_t e;
    if (c->sched_live) {
        // ordered dispatch: the items were filed by this pass's query transform;
        // the grid covers their upper bound (surplus waves exit at once)
        const int64_t NG = (N + 127) / 128;
        const int64_t items = pass == c->pass_base ? (int64_t)uniform_splits(c, nact) * nact * NG
                                        : sched_item_budget(c) + 2 * (int64_t)nact * NG + 64;
        const int64_t B = c->sched_B;
        const int par = pass & 1;
        SchedS sa{};
        sa.cnt = c->wcnt.p + (size_t)par * kSchedClasses;
        sa.cnt_next = c->wcnt.p + (size_t)(par ^ 1) * kSchedClasses;
        sa.list = c->wlist.p;
        sa.wcost = c->wcost.p + (size_t)par * B * NG;
        sa.wtot = c->wtot.p + (size_t)par * kSchedTot;
        sa.wtot_next = c->wtot.p + (size_t)(par ^ 1) * kSchedTot;
        sa.cap = c->sched_cap;
        sa.NG = (int)NG;
        sa.B = (int)B;
        sa.xcd = kSWaves == 1 ? c->opt.sched_xcd : 0;
        const int64_t grid = (std::min<int64_t>(items, c->sched_cap) + kSWaves - 1) / kSWaves;
        auto kern = c->exact_live ? nn_search_sched_kernel<true> : nn_search_sched_kernel<false>;
        kern<<<dim3((unsigned)grid), 64 * kSWaves, 0, s>>>(c->q32.p, N, c->tdesc.p, c->opt.super_cull, c->best.p,
                                                      c->count_tiles ? c->counters.p : nullptr, c->gbox.p, sa,
                                                      exact_args(c, pass));
#ifdef ORPCD_WAVETIME
        if ((e = dump_wavetime(pass, nact, 0, (unsigned)(grid * kSWaves), s)) != hipSuccess) return e;
#endif
    } else {
        // few running starts: half the wave target (8 starts: 16k waves 8.16 ms
        // vs 32k 8.40 ms per batch; 30 starts keep 32k).  Splits never change
        // answers.  best[] was reset to kNone by xform_queries_kernel.
        const int S = uniform_splits(c, nact);
        auto kern = c->exact_live ? nn_search_kernel<true> : nn_search_kernel<false>;
        kern<<<dim3((unsigned)(sblk * S), (unsigned)nact), kCBlock, 0, s>>>(
            c->q32.p, N, c->tdesc.p, tb, c->opt.super_cull, c->active.p, c->done.p, S, c->best.p,
            c->count_tiles ? c->counters.p : nullptr, c->gbox.p, exact_args(c, pass));
#ifdef ORPCD_WAVETIME
        if ((e = dump_wavetime(pass, nact, S, (unsigned)(sblk * S) * (unsigned)nact * kCWaves, s)) != hipSuccess)
            return e;
#endif
    }
    if ((e = launched("nn_search(_sched)_kernel", s)) != hipSuccess) return e;
    const int ablk = accum_blocks(N);
    const bool fused = c->exact_live && c->est != kEstP2P && c->opt.exact_fused;
    if (c->exact_live && !fused) {  // fp64 re-search of the queries the search could not certify
        nn_exact_kernel<<<(unsigned)c->opt.exact_blocks, 256, 0, s>>>(c->src.xyz64.p, N, c->Q.p, c->tdesc.p, c->q32.p,
                                                     exact_args(c, pass), c->best.p);
        if ((e = launched("nn_exact_kernel", s)) != hipSuccess) return e;
    }
    if (mid && (e = hipEventRecord(mid, s)) != hipSuccess) return e;
    if (fused) {
        // re-search blocks: exact_fused per running start, at most exact_blocks
        const int nexact = std::max(8, std::min(c->opt.exact_blocks, c->opt.exact_fused * nact));
        gicp_accum_exact_kernel<<<(unsigned)(nexact + ablk * nact), 256, 0, s>>>(
            c->src.xyz64.p, c->scov.p, N, c->tdesc.p, tb, c->active.p, c->Q.p, c->R.p, c->done.p, r2, c->best.p,
            c->prevnn.p, c->partial.p, ablk, nexact, c->q32.p, exact_args(c, pass), 1.0 - c->batch_eps);
        return launched("gicp_accum_exact_kernel", s);
    }
    if (c->est == kEstP2P) {
        p2p_accum_kernel<<<dim3((unsigned)ablk, (unsigned)nact), 256, 0, s>>>(
            c->src.xyz64.p, N, c->tdesc.p, tb, c->active.p, c->Q.p, c->done.p, r2, c->best.p, c->prevnn.p,
            c->partial.p, ablk);
        return launched("p2p_accum_kernel", s);
    }
    gicp_accum_kernel<<<dim3((unsigned)ablk, (unsigned)nact), 256, 0, s>>>(
        c->src.xyz64.p, c->scov.p, N, c->tdesc.p, tb, c->active.p, c->Q.p, c->R.p, c->done.p, r2, c->best.p,
        c->prevnn.p, c->partial.p, ablk, 1.0 - c->batch_eps);
    return launched("gicp_accum_kernel", s);
}

hipError_t launch_gicp_solve(const orpcd_ctx* c, int nact, int pass, const orpcd_gicp_params& p, hipStream_t s,
                             const TgtBounds& tb) {
    const SolveArgs a = solve_args(c);
    auto solve = c->est == kEstP2P ? icp_solve_kernel<1> : icp_solve_kernel<0>;
    const int solve_threads = 64 * (c->est == kEstP2P ? solve_waves<1>() : solve_waves<0>());
    solve<<<(unsigned)nact, solve_threads, 0, s>>>(c->active.p, c->partial.p, accum_blocks(c->src.n), nullptr,
                                                    c->src.n, pass, p.max_iteration, p.relative_fitness,
                                                    p.relative_rmse, a);
    hipError_t e = launched("icp_solve_kernel", s);
    if (e != hipSuccess) return e;
    const double r2 = p.max_correspondence_distance * p.max_correspondence_distance;
    return launch_xform(c, nact, pass + 1, r2, s, tb);  // queries of the next pass (done starts skip)
}

hipError_t launch_reduce_partials(const orpcd_ctx* c, int slot, double* sums29, hipStream_t s) {
    reduce_partials_kernel<<<1, 64, 0, s>>>(c->partial.p, slot, accum_blocks(c->src.n), sums29);
    return hipGetLastError();
}

hipError_t launch_gicp_solve_sums(const orpcd_ctx* c, const double* sums29, int64_t n_total, int pass,
                                  const orpcd_gicp_params& p, hipStream_t s) {
    const SolveArgs a = solve_args(c);
    icp_solve_kernel<0><<<1, 64 * solve_waves<0>(), 0, s>>>(c->active.p, nullptr, 0, sums29, n_total, pass, p.max_iteration,
                                       p.relative_fitness, p.relative_rmse, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const double r2 = p.max_correspondence_distance * p.max_correspondence_distance;
    return launch_xform(c, 1, pass + 1, r2, s, one_target());
}

constexpr int64_t kNn1OrderMin = 4096;  // smaller batches search in input order

hipError_t launch_nn1(const double* q, int64_t nq, const CloudLayout& t, double r2, int32_t* idx, double* d2,
                      QueryOrder& qo, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((nq + kCBlockQ - 1) / kCBlockQ);
    // a batch in arbitrary order is first put in Morton order over the
    // target's box (30-bit codes, hipCUB radix sort): C3's evaluation, 100k
    // queries in input order, 1.44 ms unordered
    const int32_t* order = nullptr;
    if (nq >= kNn1OrderMin) {
        hipError_t e;
        if ((e = qo.codes.ensure((size_t)nq * 2)) != hipSuccess) return e;
        if ((e = qo.ids.ensure((size_t)nq)) != hipSuccess) return e;
        if ((e = qo.order.ensure((size_t)nq)) != hipSuccess) return e;
        double ext = 0.0;
        for (int a = 0; a < 3; ++a) ext = std::max(ext, t.hi[a] - t.lo[a]);
        const double scale = ext > 0 ? 1023.0 / ext : 0.0;
        if ((e = launch_morton(q, nq, t.lo, scale, qo.codes.p, qo.ids.p, s)) != hipSuccess) return e;
        size_t tmp = 0;
        if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, qo.codes.p, qo.codes.p + nq, qo.ids.p, qo.order.p,
                                                    (int)nq, 0, 30, s)) != hipSuccess)
            return e;
        if ((e = qo.tmp.ensure(tmp)) != hipSuccess) return e;
        if ((e = hipcub::DeviceRadixSort::SortPairs(qo.tmp.p, tmp, qo.codes.p, qo.codes.p + nq, qo.ids.p, qo.order.p,
                                                    (int)nq, 0, 30, s)) != hipSuccess)
            return e;
        order = qo.order.p;
    }
    nn1_kernel<<<grid, kCBlock, 0, s>>>(order, q, (int)nq, t.p4.p, t.tlo.p, t.thi.p, t.qbox.p, (int)t.ntiles, t.slo.p, t.shi.p,
                                        (int)t.nsuper, seed_stride_for(t.ntiles), t.xyz64.p, t.perm.p, r2,
                                        search_r2(r2), idx, d2, org_of(t));
    return hipGetLastError();
}

// this unit's code object loaded now (orpcd_ctx_create), not at its first launch
hipError_t preload_code_object_gicp() {
    hipFuncAttributes attr;
    return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&seed_scatter_kernel));
}

}  // namespace orpcd
