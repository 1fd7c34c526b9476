// knn_kernels.hip — per-point neighbourhood covariance and GICP covariance.
//
// Restates, for gfx950, Open3D 0.18 EstimatePerPointCovariances /
// EstimateNormals (KDTreeSearchParamKNN(20) inside registration_generalized_icp,
// generalizedICP.py:59-70; KDTreeSearchParamHybrid in fastGlobalOptimizer.py:118-127)
// and InitializePointCloudForGeneralizedICP.
//
// Design: exact K nearest in fp64 over the Morton-tiled cloud with two-level
// AABB culling (knn_tiles_kernel below).  The neighbour set is the K smallest
// by (d^2, input index) — identical to the oracle's KD-tree result — and the
// cumulants are summed in that order with contraction off, so the covariance
// and FastEigen3x3 normal match the CPU restatement operation for operation.
// This pass runs once per cloud (not per ICP iteration).
#include <cstdlib>

#include "device_math.h"
#include "orpcd_internal.h"
#include "wave_ops.h"

namespace orpcd {

// Normal (FastEigen3x3) and GICP covariance for `nslots` rotated copies of a
// cloud's raw covariances: slot b uses Sigma_b = Rc_b Sigma Rc_b^T
// (Rc_b = NULL -> identity).  Output index = b * n + i.
__global__ __launch_bounds__(256) void normals_cov_kernel(const double* __restrict__ rawcov6, int n,
                                                          const double* __restrict__ Rc9, int nslots, double eps,
                                                          double* __restrict__ normals3,
                                                          double* __restrict__ cov6,
                                                          double* __restrict__ enorm3) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)n * nslots) return;
    const int b = (int)(gid / n);
    const int i = (int)(gid - (int64_t)b * n);
    const double* r = rawcov6 + (size_t)i * 6;
    Sym3 S{r[0], r[1], r[2], r[3], r[4], r[5]};
    if (Rc9) {
        double Rb[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) Rb[t] = Rc9[9 * b + t];
        S = rotate_sym(Rb, S);
    }
    double nrm[3];
    fast_eigen3x3(S, nrm);
    if (nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2] == 0.0) {
        nrm[0] = 0.0;
        nrm[1] = 0.0;
        nrm[2] = 1.0;
    }
    if (normals3) {
        normals3[3 * gid] = nrm[0];
        normals3[3 * gid + 1] = nrm[1];
        normals3[3 * gid + 2] = nrm[2];
    }
    if (enorm3) {  // C = I - (1 - eps) e e^T: e = n, or e1 where GetRotationFromE1ToX takes R = I
        const bool quirk = nrm[0] < -0.99;
        enorm3[3 * gid] = quirk ? 1.0 : nrm[0];
        enorm3[3 * gid + 1] = quirk ? 0.0 : nrm[1];
        enorm3[3 * gid + 2] = quirk ? 0.0 : nrm[2];
    }
    if (cov6 && eps >= 0.0) {
        Sym3 C = gicp_cov_from_normal(nrm, eps);
        double* o = cov6 + (size_t)gid * 6;
        o[0] = C.xx;
        o[1] = C.xy;
        o[2] = C.xz;
        o[3] = C.yy;
        o[4] = C.yz;
        o[5] = C.zz;
    }
}

// ---------------------------------------------------------------------------
// Culled exact KNN over a Morton-tiled cloud (CloudLayout with tiles).
//
// One query per lane; a wave holds 64 Morton-consecutive queries (one tile),
// so its bounding box is tight.  The wave first scans its own tile (64
// candidates: enough to make every lane's K-th bound finite when K <= 63),
// then walks super-tiles / tiles whose boxes can still hold a closer point
// than some lane's K-th bound (ballot), staging each surviving tile in LDS as
// fp64 SoA.  Distances are fp64, insertion is by (d^2, input index), so the
// neighbour list — and the cumulant order of the covariance — is exactly the
// oracle's KD-tree answer regardless of traversal order.  Box tests are fp32
// on fp32-rounded boxes, made conservative by `margin` (an absolute bound on
// the fp32 rounding of any coordinate, per axis).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float gapf(float lo, float hi, float x, float margin) {
    return fmaxf(0.0f, fmaxf(lo - x, x - hi) - margin);
}

// the packed lane-per-query network (knn_tiles_kernel): on by default
#ifndef ORPCD_KNN_PACKED
#define ORPCD_KNN_PACKED 1
#endif
constexpr int kKnnSlack = 3;        // keys kept beyond K (a boundary run of equal buckets up to this long)
constexpr int kKnnPackedMaxK = 24;  // larger lists keep the exact network (their registers: 235-256 VGPRs)

// waves per SIMD asked of the lane-per-query kernel for K <= 24 (the GICP
// covariance lists): 3 (168 VGPRs; the packed network's state fits, the
// spills are in the exact fallback and the final resolution) measured faster
// than the compiler's 2 at C5; larger K keep the compiler's choice
#ifndef ORPCD_KNN_LANE_WAVES
#define ORPCD_KNN_LANE_WAVES 3
#endif
template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K <= 24 ? ORPCD_KNN_LANE_WAVES : 1, 8))) void knn_tiles_kernel(
    const double* __restrict__ xyz64, const int32_t* __restrict__ perm, int n, const float4* __restrict__ tlo,
    const float4* __restrict__ thi, int ntiles, const float4* __restrict__ slo, const float4* __restrict__ shi,
    int nsuper, const double* __restrict__ in64, double r2, float margin, double ox, double oy, double oz, int kout,
    int out_input_order, double* __restrict__ rawcov6, int32_t* __restrict__ nbr_idx, double* __restrict__ nbr_d2,
    int32_t* __restrict__ nbr_cnt, double* __restrict__ mean_dist, KnnTieOut ties, int t0, int t1) {
    __shared__ double sx[4][kTile], sy[4][kTile], sz[4][kTile];
    __shared__ int32_t sid[4][kTile];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int own = t0 + blockIdx.x * 4 + w;  // the wave's own tile (queries: tiles [t0, t1))
    if (own >= t1) return;                    // wave-uniform
    const int q = own * kTile + lane;
    const bool valid = q < n;
    const double qx = valid ? xyz64[3 * q] : 0.0, qy = valid ? xyz64[3 * q + 1] : 0.0,
                 qz = valid ? xyz64[3 * q + 2] : 0.0;
    double bd[K];
    int bi[K];
    const float inf = 3.0e38f;
    const float fx = (float)(qx - ox), fy = (float)(qy - oy), fz = (float)(qz - oz);  // the boxes' fp32 frame
    const float lox = wave_fmin(valid ? fx : inf), hix = wave_fmax(valid ? fx : -inf);
    const float loy = wave_fmin(valid ? fy : inf), hiy = wave_fmax(valid ? fy : -inf);
    const float loz = wave_fmin(valid ? fz : inf), hiz = wave_fmax(valid ? fz : -inf);
    // stage tile t in LDS as fp64 SoA (+ input indices)
    auto stage = [&](int t) {
        const int k = t * kTile + lane;
        const bool real = k < n;
        sx[w][lane] = real ? xyz64[3 * k] : 1e300;
        sy[w][lane] = real ? xyz64[3 * k + 1] : 1e300;
        sz[w][lane] = real ? xyz64[3 * k + 2] : 1e300;
        sid[w][lane] = real ? perm[k] : 0x7fffffff;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto dist = [&](int c) {
#pragma clang fp contract(off)
        const double dx = qx - sx[w][c], dy = qy - sy[w][c], dz = qz - sz[w][c];
        return dx * dx + dy * dy + dz * dz;
    };
    // The walk: own tile, then its Morton neighbours (a near-final bound
    // before the culled walk), then the super-tiles / tiles whose boxes can
    // still hold a point below some lane's bound.  visit(t) scans tile t;
    // bound() is the lane's fp32 culling bound.
    constexpr int kWin = 2;
    auto walk = [&](auto&& visit, auto&& bound) {
        visit(own);
        for (int dt = 1; dt <= kWin; ++dt) {
            if (own - dt >= 0) visit(own - dt);
            if (own + dt < ntiles) visit(own + dt);
        }
        for (int sb = 0; sb < nsuper; sb += 64) {
            float Wb = wave_fmax(bound());
            const int u = sb + lane;
            float sl = inf;
            if (u < nsuper) {
                const float4 c = slo[u], d = shi[u];
                const float dx = fmaxf(0.0f, fmaxf(c.x - hix, lox - d.x) - margin);
                const float dy = fmaxf(0.0f, fmaxf(c.y - hiy, loy - d.y) - margin);
                const float dz = fmaxf(0.0f, fmaxf(c.z - hiz, loz - d.z) - margin);
                sl = dx * dx + dy * dy + dz * dz;
            }
            unsigned long long smask = __ballot(sl < Wb);
            while (smask) {
                const int su = sb + __builtin_ctzll(smask);
                smask &= smask - 1;
                Wb = wave_fmax(bound());
                const int t = su * kSuper + lane;
                float lb = inf;
                float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
                if (t < ntiles && (t < own - kWin || t > own + kWin)) {
                    a = tlo[t];
                    b = thi[t];
                    const float dx = fmaxf(0.0f, fmaxf(a.x - hix, lox - b.x) - margin);
                    const float dy = fmaxf(0.0f, fmaxf(a.y - hiy, loy - b.y) - margin);
                    const float dz = fmaxf(0.0f, fmaxf(a.z - hiz, loz - b.z) - margin);
                    lb = dx * dx + dy * dy + dz * dz;
                }
                unsigned long long mask = __ballot(lb < Wb);
                while (mask) {
                    const int k = __builtin_ctzll(mask);
                    mask &= mask - 1;
                    const float ax = __shfl(a.x, k, 64), ay = __shfl(a.y, k, 64), az = __shfl(a.z, k, 64);
                    const float bx = __shfl(b.x, k, 64), by = __shfl(b.y, k, 64), bz = __shfl(b.z, k, 64);
                    const float gx = gapf(ax, bx, fx, margin), gy = gapf(ay, by, fy, margin),
                                gz = gapf(az, bz, fz, margin);
                    const bool need = valid && gx * gx + gy * gy + gz * gz < bound();
                    if (__ballot(need) == 0ull) continue;
                    visit(su * kSuper + k);
                }
            }
        }
    };
    auto to_bound = [&](double b) -> float {  // fp32 upper bound of a d^2 bound
        return b >= 3.0e38 ? inf : (float)b * 1.0000003f + 1e-37f;
    };
    // The exact network: the K best (d^2, input index) so far, sorted.  Two
    // phases per staged tile: (1) every lane marks the candidates that beat
    // its bound at tile start (the bound only shrinks, so this is a
    // superset); (2) each lane walks only its own marks.  The wave then pays
    // the insertion network max_lane(marks) times instead of once for every
    // candidate that ANY lane takes.
    auto exact_walk = [&]() {
#pragma unroll
        for (int s = 0; s < K; ++s) {
            bd[s] = r2;
            bi[s] = -1;
        }
        auto visit = [&](int t) {
            stage(t);
            const double b0 = bd[K - 1];
            unsigned long long marks = 0;
#pragma unroll 8
            for (int c = 0; c < kTile; ++c) marks |= (unsigned long long)(dist(c) <= b0) << c;
            if (!valid) marks = 0;
            while (marks) {
                const int c = __builtin_ctzll(marks);
                marks &= marks - 1;
                const double d = dist(c);
                const int id = sid[w][c];
                if (d < bd[K - 1] || (d == bd[K - 1] && bi[K - 1] >= 0 && id < bi[K - 1])) {
                    double cd = d;
                    int ci = id;
#pragma unroll
                    for (int s = 0; s < K; ++s) {
                        const bool sw = cd < bd[s] || (cd == bd[s] && (unsigned)ci < (unsigned)bi[s]);
                        const double td = bd[s];
                        const int ti = bi[s];
                        bd[s] = sw ? cd : td;
                        bi[s] = sw ? ci : ti;
                        cd = sw ? td : cd;
                        ci = sw ? ti : ci;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();  // the stage is rewritten by the next tile
        };
        walk(visit, [&]() -> float { return valid ? to_bound(bd[K - 1]) : 0.0f; });
    };
    if constexpr (ORPCD_KNN_PACKED && K <= kKnnPackedMaxK) {
    // The packed network (default for K <= kKnnPackedMaxK): one 64-bit key per kept candidate, the
    // fp64 d^2 bits truncated to their top 37 (a bucket of relative width
    // 2^-25) over the 27-bit input index (kMaxPoints = 2^27).  Keys are
    // unique, and their order is (bucket, index): a compare-exchange is one
    // 64-bit compare and four selects instead of the exact pair's three
    // compares and six selects.  The list keeps KL = K + kKnnSlack keys;
    // culling uses the upper end of the K-th key's bucket, so every point in a
    // bucket at most the K-th's is scanned.  At the end the keys whose bucket
    // is at most the K-th's are a superset of the exact K nearest (a point
    // outside it has a larger bucket, hence a larger d^2, than K kept ones)
    // whenever the list's last key lies in a larger bucket than the K-th;
    // their fp64 d^2 is recomputed (the same expression) and equal-bucket runs
    // are put in (d^2, index) order.  Otherwise a run of equal buckets may
    // continue past the list and the wave re-runs the exact network.
    constexpr int KL = K + kKnnSlack;
    constexpr unsigned long long kIdxMask = (1ull << 27) - 1ull, kBucketMask = ~kIdxMask, kEmpty = ~0ull;
    static_assert(kMaxPoints <= (int64_t)(1ull << 27), "the key's index field holds every input index");
    auto bucket_hi = [&](unsigned long long key) -> double {  // the largest d^2 of key's bucket (r2 if empty)
        return key == kEmpty ? r2 : fmin(r2, __longlong_as_double((long long)(key | kIdxMask)));
    };
    unsigned long long bk[KL];
#pragma unroll
    for (int s = 0; s < KL; ++s) bk[s] = kEmpty;
    auto visit = [&](int t) {
        stage(t);
        // marks: below r2 and in a bucket at most the K-th key's (at tile start).
        // A point left out -- unmarked, or marked when KL smaller keys were
        // already kept -- has a key above the final list's last one, so the
        // overflow test below sees any such point in the K-th key's bucket
        const double b0 = bucket_hi(bk[K - 1]);
        unsigned long long marks = 0;
#pragma unroll 8
        for (int c = 0; c < kTile; ++c) {
            const double d = dist(c);
            marks |= (unsigned long long)(d <= b0 && d < r2) << c;
        }
        if (!valid) marks = 0;
        while (marks) {
            const int c = __builtin_ctzll(marks);
            marks &= marks - 1;
            const unsigned long long key =
                ((unsigned long long)__double_as_longlong(dist(c)) & kBucketMask) | (unsigned long long)sid[w][c];
            if (key < bk[KL - 1]) {
                unsigned long long ck = key;
#pragma unroll
                for (int s = 0; s < KL; ++s) {
                    const bool sw = ck < bk[s];
                    const unsigned long long t2 = bk[s];
                    bk[s] = sw ? ck : t2;
                    ck = sw ? t2 : ck;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();  // the stage is rewritten by the next tile
    };
    walk(visit, [&]() -> float { return valid ? to_bound(bucket_hi(bk[K - 1])) : 0.0f; });
    const unsigned long long tK = bk[K - 1] & kBucketMask;
    const bool overflow = valid && bk[K - 1] != kEmpty && (bk[KL - 1] & kBucketMask) == tK;
    if (__ballot(overflow) != 0ull) {
        exact_walk();
    } else {
        double cd[KL];
        int ci[KL];
#pragma unroll
        for (int s = 0; s < KL; ++s) {
            const bool use = bk[s] != kEmpty && (bk[s] & kBucketMask) <= tK;
            ci[s] = use ? (int)(bk[s] & kIdxMask) : -1;
            double d = r2;
            if (use) {
#pragma clang fp contract(off)
                const int j = ci[s];
                const double dx = qx - in64[3 * j], dy = qy - in64[3 * j + 1], dz = qz - in64[3 * j + 2];
                d = dx * dx + dy * dy + dz * dz;
            }
            cd[s] = d;
        }
        // equal-bucket runs into (d^2, index) order: adjacent exchanges until
        // none is needed (keys already order different buckets correctly)
        for (;;) {
            bool moved = false;
#pragma unroll
            for (int s = 0; s + 1 < KL; ++s) {
                const bool sw = ci[s + 1] >= 0 && (cd[s + 1] < cd[s] || (cd[s + 1] == cd[s] && ci[s + 1] < ci[s]));
                const double td = cd[s];
                const int ti = ci[s];
                cd[s] = sw ? cd[s + 1] : td;
                ci[s] = sw ? ci[s + 1] : ti;
                cd[s + 1] = sw ? td : cd[s + 1];
                ci[s + 1] = sw ? ti : ci[s + 1];
                moved |= sw;
            }
            if (__ballot(moved) == 0ull) break;
        }
#pragma unroll
        for (int s = 0; s < K; ++s) {
            bd[s] = ci[s] >= 0 ? cd[s] : r2;
            bi[s] = ci[s];
        }
    }
    } else {
        exact_walk();
    }
    if (!valid) return;
    int c = 0;
#pragma unroll
    for (int s = 0; s < K; ++s) c += (s < kout && bi[s] >= 0) ? 1 : 0;
    const int o = out_input_order ? perm[q] : q;
    if (ties.cnt && kout < K) {
        // boundary tie (as knn_wave_kernel): the (kout+1)-th neighbour within
        // the band of the kout-th; the entry lists the kout + kTieExtra nearest
        const int Kt = kout + kTieExtra;
        double dk = r2, dk1 = r2;
#pragma unroll
        for (int s = 0; s < K; ++s) {
            if (s == kout) dk = bi[s] >= 0 ? bd[s] : r2;
            if (s == kout - 1) dk1 = bi[s] >= 0 ? bd[s] : r2;
        }
        if (dk < 3.0e38 && dk - dk1 <= ties.rel * dk + ties.abs_coef * sqrt(dk)) {
            const int e = atomicAdd(ties.cnt, 1);
            if (ties.detect) {
                if (e < ties.cap) ties.detect[e] = q;
            } else if (e < ties.cap) {
                int32_t* row = ties.rows + (size_t)e * (Kt + 2);
                row[0] = q;
                row[1] = perm[q];
#pragma unroll
                for (int s = 0; s < K; ++s)
                    if (s < Kt) {
                        row[2 + s] = bi[s];
                        ties.d2[(size_t)e * Kt + s] = bi[s] >= 0 ? bd[s] : __builtin_huge_val();
                    }
            }
        }
    }
    if (nbr_idx) {
#pragma unroll
        for (int s = 0; s < K; ++s)
            if (s < kout) nbr_idx[(size_t)o * kout + s] = s < c ? bi[s] : -1;
    }
    if (nbr_d2) {
#pragma unroll
        for (int s = 0; s < K; ++s)
            if (s < kout) nbr_d2[(size_t)o * kout + s] = s < c ? bd[s] : 0.0;
    }
    if (nbr_cnt) nbr_cnt[o] = c;
    if (mean_dist) {  // SOR: mean of sqrt(d^2) over the neighbours, ascending (-1: empty search)
        double m = -1.0;
        if (c > 0) {
            double sd = 0.0;
#pragma unroll
            for (int s = 0; s < K; ++s)
                if (s < c) sd += sqrt(bd[s]);
            m = sd / (double)c;
        }
        mean_dist[o] = m;
    }
    if (!rawcov6) return;
    Sym3 C;
    if (c >= 3) {
#pragma clang fp contract(off)
        double cu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < K; ++s) {
            if (s < c) {
                const int j = bi[s];
                const double px = in64[3 * j], py = in64[3 * j + 1], pz = in64[3 * j + 2];
                cu[0] += px;
                cu[1] += py;
                cu[2] += pz;
                cu[3] += px * px;
                cu[4] += px * py;
                cu[5] += px * pz;
                cu[6] += py * py;
                cu[7] += py * pz;
                cu[8] += pz * pz;
            }
        }
        const double cn = (double)c;
#pragma unroll
        for (int t = 0; t < 9; ++t) cu[t] /= cn;
        C.xx = cu[3] - cu[0] * cu[0];
        C.yy = cu[6] - cu[1] * cu[1];
        C.zz = cu[8] - cu[2] * cu[2];
        C.xy = cu[4] - cu[0] * cu[1];
        C.xz = cu[5] - cu[0] * cu[2];
        C.yz = cu[7] - cu[1] * cu[2];
    } else {
        C = Sym3{1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
    }
    double* out = rawcov6 + (size_t)o * 6;
    out[0] = C.xx;
    out[1] = C.xy;
    out[2] = C.xz;
    out[3] = C.yy;
    out[4] = C.yz;
    out[5] = C.zz;
}

// ---------------------------------------------------------------------------
// One wave per query (default KNN): the wave holds the query's K <= 64 best
// (d^2, input index) so far SORTED across its lanes (lane s = s-th nearest).
// Each candidate tile puts one point per lane: exact fp64 d^2 (contraction
// off, the oracle's expression), a bitonic sort of the 64 candidates across
// lanes, then the merge with the kept list (reverse, lane-wise min -> bitonic
// -> 6 merge steps).  A tile is skipped when no candidate beats the K-th kept
// pair, and whole tiles / super-tiles when their (conservative fp32) box is
// farther than the K-th distance.  The list -- and every sum made from it in
// list order (covariance cumulants, SOR's mean distance) -- is the oracle's
// KD-tree answer exactly.  Tiles: own, then +-1, +-2 (Morton neighbours), then
// the culled walk over super-tiles and tiles.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool pair_less(double d, int i, double e, int j) { return d < e || (d == e && i < j); }

__device__ __forceinline__ void xchg(double& d, int& i, int j_xor, bool keep_min) {
    const double pd = __shfl_xor(d, j_xor, 64);
    const int pi = __shfl_xor(i, j_xor, 64);
    const bool pl = pair_less(pd, pi, d, i);  // partner < self
    if (keep_min ? pl : pair_less(d, i, pd, pi)) {
        d = pd;
        i = pi;
    }
}

__device__ __forceinline__ void bitonic_sort64(double& d, int& i, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const bool up = (lane & k) == 0 || k == 64;
            const bool lower = (lane & j) == 0;
            xchg(d, i, j, lower == up);
        }
}

__global__ __launch_bounds__(256) void knn_wave_kernel(
    const double* __restrict__ xyz64, const int32_t* __restrict__ perm, int n, const float4* __restrict__ tlo,
    const float4* __restrict__ thi, int ntiles, const float4* __restrict__ slo, const float4* __restrict__ shi,
    int nsuper, const double* __restrict__ in64, double r2, float margin, double ox, double oy, double oz, int K,
    int out_input_order, double* __restrict__ rawcov6, int32_t* __restrict__ nbr_idx, double* __restrict__ nbr_d2,
    int32_t* __restrict__ nbr_cnt, double* __restrict__ mean_dist, int KC, KnnTieOut ties,
    const double* __restrict__ orgs = nullptr, const float* __restrict__ margins = nullptr,
    const int32_t* __restrict__ qlist = nullptr, int nq = 0, int q0 = 0, int q1 = 0x7fffffff) {
#pragma clang fp contract(off)
    if (orgs) {  // copy y of a BatchLayout: its frame, points, boxes and outputs
        const size_t y = blockIdx.y;
        ox = orgs[3 * y];
        oy = orgs[3 * y + 1];
        oz = orgs[3 * y + 2];
        margin = margins[y];
        xyz64 += y * 3 * n;
        in64 += y * 3 * n;
        tlo += y * ntiles;
        thi += y * ntiles;
        slo += y * nsuper;
        shi += y * nsuper;
        if (rawcov6) rawcov6 += y * 6 * n;
        if (nbr_idx) nbr_idx += y * (size_t)n * KC;
        if (nbr_d2) nbr_d2 += y * (size_t)n * KC;
        if (nbr_cnt) nbr_cnt += y * n;
    }
    const int lane = threadIdx.x & 63;
    int q = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (qlist) {  // only the listed Morton positions query (a row shard's points)
        if (q >= nq) return;  // wave-uniform
        q = __builtin_amdgcn_readfirstlane(qlist[q]);
    } else {      // Morton positions [q0, q1)
        q += q0;
        if (q >= q1) return;
    }
    if (q >= n) return;  // wave-uniform
    const double qx = xyz64[3 * q], qy = xyz64[3 * q + 1], qz = xyz64[3 * q + 2];
    const float fx = (float)(qx - ox), fy = (float)(qy - oy), fz = (float)(qz - oz);  // the boxes' fp32 frame
    const double INF = __builtin_huge_val();
    double Ld = INF;  // sorted kept list: lane s holds the s-th nearest so far
    int Li = 0x7fffffff;
    auto kth = [&]() {  // the K-th kept pair (uniform)
        const long long b = __double_as_longlong(Ld);
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, K - 1);
        const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), K - 1);
        return __longlong_as_double(((long long)hi << 32) | lo);
    };
    auto bound_f = [&]() -> float {  // fp32 upper bound of the K-th d^2 (and of the radius)
        const double b = fmin(kth(), r2);
        return b >= 3.0e38 ? 3.0e38f : (float)b * 1.0000003f + 1e-37f;
    };
    const int own = q / kTile;
    auto scan_tile = [&](int t) {
        const int k = t * kTile + lane;
        double d = INF;
        int id = 0x7fffffff;
        if (k < n) {
            const double dx = qx - xyz64[3 * k], dy = qy - xyz64[3 * k + 1], dz = qz - xyz64[3 * k + 2];
            const double dd = dx * dx + dy * dy + dz * dz;
            if (dd < r2) {
                d = dd;
                id = perm[k];
            }
        }
        const double kd = kth();
        const int ki = __builtin_amdgcn_readlane(Li, K - 1);
        if (!__any(pair_less(d, id, kd, ki))) return;
        bitonic_sort64(d, id, lane);
        // merge: the 64 smallest of (kept, new) are the lane-wise minima of the
        // kept list and the reversed new list (a bitonic sequence) ...
        const double rd = __shfl(d, 63 - lane, 64);
        const int ri = __shfl(id, 63 - lane, 64);
        if (pair_less(rd, ri, Ld, Li)) {
            Ld = rd;
            Li = ri;
        }
        // ... sorted ascending by the bitonic merge
#pragma unroll
        for (int j = 32; j > 0; j >>= 1) xchg(Ld, Li, j, (lane & j) == 0);
    };
    constexpr int kWin = 2;
    scan_tile(own);
    for (int dt = 1; dt <= kWin; ++dt) {
        if (own - dt >= 0) scan_tile(own - dt);
        if (own + dt < ntiles) scan_tile(own + dt);
    }
    auto gap = [&](float4 a, float4 b) {
        const float gx = fmaxf(0.0f, fmaxf(a.x - fx, fx - b.x) - margin);
        const float gy = fmaxf(0.0f, fmaxf(a.y - fy, fy - b.y) - margin);
        const float gz = fmaxf(0.0f, fmaxf(a.z - fz, fz - b.z) - margin);
        return gx * gx + gy * gy + gz * gz;
    };
    for (int sb = 0; sb < nsuper; sb += 64) {
        const int u = sb + lane;
        const float sl = u < nsuper ? gap(slo[u], shi[u]) : 3.0e38f;
        unsigned long long smask = __ballot(sl < bound_f());
        while (smask) {
            const int su = sb + __builtin_ctzll(smask);
            smask &= smask - 1;
            const int t = su * kSuper + lane;
            const float lb = (t < ntiles && (t < own - kWin || t > own + kWin)) ? gap(tlo[t], thi[t]) : 3.0e38f;
            unsigned long long tm = __ballot(lb < bound_f());
            while (tm) {
                const int k = __builtin_ctzll(tm);
                tm &= tm - 1;
                const float lbk = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(lb), k));
                if (!(lbk < bound_f())) continue;  // the K-th distance shrank meanwhile
                scan_tile(su * kSuper + k);
            }
        }
    }
    // outputs: the first KC (<= K) kept pairs (beyond the count they are
    // (INF, max) and written as -1 / 0)
    const int c = __popcll(__ballot(lane < KC && Ld < INF));
    const int o = out_input_order ? perm[q] : q;
    if (ties.cnt && KC < K) {
        // boundary tie: the (KC+1)-th neighbour within the band of the KC-th, so
        // a rigidly posed copy's rounding may swap them (a point the caller
        // re-decides per pose from the listed K nearest, runtime.hip SourceTies)
        const long long bk = __double_as_longlong(Ld);
        auto lane_d = [&](int l) {  // lane l's kept distance (both halves zero-extended)
            const unsigned hi = __builtin_amdgcn_readlane((unsigned)(bk >> 32), l);
            const unsigned lo = __builtin_amdgcn_readlane((unsigned)bk, l);
            return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
        };
        const double dk = lane_d(KC), dk1 = lane_d(KC - 1);
        if (ties.force || (dk < INF && dk - dk1 <= ties.rel * dk + ties.abs_coef * sqrt(dk))) {
            int e = 0;
            if (lane == 0) e = atomicAdd(ties.cnt, 1);
            e = __builtin_amdgcn_readfirstlane(e);
            if (ties.detect) {
                if (lane == 0 && e < ties.cap) ties.detect[e] = q;
            } else if (e < ties.cap) {
                int32_t* row = ties.rows + (size_t)e * (K + 2);
                if (lane == 0) {
                    row[0] = q;
                    row[1] = perm[q];
                }
                if (lane < K) {
                    row[2 + lane] = Ld < INF ? Li : -1;
                    ties.d2[(size_t)e * K + lane] = Ld;
                }
            }
        }
    }
    if (nbr_idx && lane < KC) nbr_idx[(size_t)o * KC + lane] = lane < c ? Li : -1;
    if (nbr_d2 && lane < KC) nbr_d2[(size_t)o * KC + lane] = lane < c ? Ld : 0.0;
    if (nbr_cnt && lane == 0) nbr_cnt[o] = c;
    if (mean_dist) {  // SOR: mean of sqrt(d^2) over the neighbours in list order (-1: empty search)
        const double sq = lane < c ? sqrt(Ld) : 0.0;
        double sd = 0.0;
        for (int s2 = 0; s2 < c; ++s2) {
            const long long b = __double_as_longlong(sq);
            const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, s2);
            const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), s2);
            sd += __longlong_as_double(((long long)hi << 32) | lo);
        }
        if (lane == 0) mean_dist[o] = c > 0 ? sd / (double)c : -1.0;
    }
    if (!rawcov6) return;
    Sym3 C;
    if (c >= 3) {  // O3D ComputeCovariance: one-pass cumulants in list order, 1/n
        double cu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int s2 = 0; s2 < c; ++s2) {
            const int j = __builtin_amdgcn_readlane(Li, s2);
            const double px = in64[3 * j], py = in64[3 * j + 1], pz = in64[3 * j + 2];
            cu[0] += px;
            cu[1] += py;
            cu[2] += pz;
            cu[3] += px * px;
            cu[4] += px * py;
            cu[5] += px * pz;
            cu[6] += py * py;
            cu[7] += py * pz;
            cu[8] += pz * pz;
        }
        const double cn = (double)c;
#pragma unroll
        for (int t = 0; t < 9; ++t) cu[t] /= cn;
        C.xx = cu[3] - cu[0] * cu[0];
        C.yy = cu[6] - cu[1] * cu[1];
        C.zz = cu[8] - cu[2] * cu[2];
        C.xy = cu[4] - cu[0] * cu[1];
        C.xz = cu[5] - cu[0] * cu[2];
        C.yz = cu[7] - cu[1] * cu[2];
    } else {
        C = Sym3{1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
    }
    if (lane == 0) {
        double* out = rawcov6 + (size_t)o * 6;
        out[0] = C.xx;
        out[1] = C.xy;
        out[2] = C.xz;
        out[3] = C.yy;
        out[4] = C.yz;
        out[5] = C.zz;
    }
}

// ---------------------------------------------------------------------------
// K > 64 (the reference accepts any positive neighbourhood size, e.g.
// FastGlobalOptimizer(fpfh_knn=100), fastGlobalOptimizer.py:86-105): one wave
// per query holds its K <= 64 P best (d^2, input index) SORTED over P chunks
// of 64 (chunk j, lane s = the (64 j + s)-th nearest).  A candidate tile is
// sorted across the lanes (bitonic), merged with the last chunk (its 64
// smallest, as in knn_wave_kernel), and the result cascades forward through
// the earlier chunks (each a sorted 64 + 64 merge: lane-wise min / max against
// the reversed carry, two half-cleaner sorts).  Every element of the chunks
// before the last ranks at most 64 (P - 1) + 64 among kept + new, so the K
// nearest are always kept.  Same exact fp64 distances, tie order, culling and
// outputs as knn_wave_kernel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void half_clean_sort(double& d, int& i, int lane) {  // bitonic 64 -> ascending
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) xchg(d, i, j, (lane & j) == 0);
}

__device__ __forceinline__ double lane_dbl(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

template <int P>
__global__ __launch_bounds__(256) void knn_wave_multi_kernel(
    const double* __restrict__ xyz64, const int32_t* __restrict__ perm, int n, const float4* __restrict__ tlo,
    const float4* __restrict__ thi, int ntiles, const float4* __restrict__ slo, const float4* __restrict__ shi,
    int nsuper, const double* __restrict__ in64, double r2, float margin, double ox, double oy, double oz, int K,
    int out_input_order, double* __restrict__ rawcov6, int32_t* __restrict__ nbr_idx, double* __restrict__ nbr_d2,
    int32_t* __restrict__ nbr_cnt, double* __restrict__ mean_dist) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (q >= n) return;  // wave-uniform
    const double qx = xyz64[3 * q], qy = xyz64[3 * q + 1], qz = xyz64[3 * q + 2];
    const float fx = (float)(qx - ox), fy = (float)(qy - oy), fz = (float)(qz - oz);
    const double INF = __builtin_huge_val();
    double Ld[P];
    int Li[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        Ld[j] = INF;
        Li[j] = 0x7fffffff;
    }
    const int kc = (K - 1) >> 6, kl = (K - 1) & 63;  // the K-th kept pair: chunk kc, lane kl (uniform)
    auto kth = [&](double& kd, int& ki) {
#pragma unroll
        for (int j = 0; j < P; ++j)
            if (j == kc) {
                kd = lane_dbl(Ld[j], kl);
                ki = __builtin_amdgcn_readlane(Li[j], kl);
            }
    };
    auto bound_f = [&]() -> float {
        double kd;
        int ki;
        kth(kd, ki);
        const double b = fmin(kd, r2);
        return b >= 3.0e38 ? 3.0e38f : (float)b * 1.0000003f + 1e-37f;
    };
    const int own = q / kTile;
    auto scan_tile = [&](int t) {
        const int k = t * kTile + lane;
        double d = INF;
        int id = 0x7fffffff;
        if (k < n) {
            const double dx = qx - xyz64[3 * k], dy = qy - xyz64[3 * k + 1], dz = qz - xyz64[3 * k + 2];
            const double dd = dx * dx + dy * dy + dz * dz;
            if (dd < r2) {
                d = dd;
                id = perm[k];
            }
        }
        double kd;
        int ki;
        kth(kd, ki);
        if (!__any(pair_less(d, id, kd, ki))) return;
        bitonic_sort64(d, id, lane);
        // the 64 smallest of (last chunk, new), sorted: the carry
        double cd = __shfl(d, 63 - lane, 64);
        int ci = __shfl(id, 63 - lane, 64);
        if (!pair_less(cd, ci, Ld[P - 1], Li[P - 1])) {
            cd = Ld[P - 1];
            ci = Li[P - 1];
        }
        half_clean_sort(cd, ci, lane);
        // cascade: chunk j and the carry -> chunk j = their 64 smallest, carry = the rest
#pragma unroll
        for (int j = 0; j < P - 1; ++j) {
            const double c0 = lane_dbl(cd, 0), lj = lane_dbl(Ld[j], 63);
            const int c0i = __builtin_amdgcn_readlane(ci, 0), lji = __builtin_amdgcn_readlane(Li[j], 63);
            if (!pair_less(c0, c0i, lj, lji)) continue;  // the carry lies wholly above chunk j (uniform)
            const double rd = __shfl(cd, 63 - lane, 64);
            const int ri = __shfl(ci, 63 - lane, 64);
            const bool take = pair_less(rd, ri, Ld[j], Li[j]);
            const double lo_d = take ? rd : Ld[j], hi_d = take ? Ld[j] : rd;
            const int lo_i = take ? ri : Li[j], hi_i = take ? Li[j] : ri;
            Ld[j] = lo_d;
            Li[j] = lo_i;
            cd = hi_d;
            ci = hi_i;
            half_clean_sort(Ld[j], Li[j], lane);
            half_clean_sort(cd, ci, lane);
        }
        Ld[P - 1] = cd;
        Li[P - 1] = ci;
    };
    constexpr int kWin = 2;
    scan_tile(own);
    for (int dt = 1; dt <= kWin; ++dt) {
        if (own - dt >= 0) scan_tile(own - dt);
        if (own + dt < ntiles) scan_tile(own + dt);
    }
    auto gap = [&](float4 a, float4 b) {
        const float gx = fmaxf(0.0f, fmaxf(a.x - fx, fx - b.x) - margin);
        const float gy = fmaxf(0.0f, fmaxf(a.y - fy, fy - b.y) - margin);
        const float gz = fmaxf(0.0f, fmaxf(a.z - fz, fz - b.z) - margin);
        return gx * gx + gy * gy + gz * gz;
    };
    for (int sb = 0; sb < nsuper; sb += 64) {
        const int u = sb + lane;
        const float sl = u < nsuper ? gap(slo[u], shi[u]) : 3.0e38f;
        unsigned long long smask = __ballot(sl < bound_f());
        while (smask) {
            const int su = sb + __builtin_ctzll(smask);
            smask &= smask - 1;
            const int t = su * kSuper + lane;
            const float lb = (t < ntiles && (t < own - kWin || t > own + kWin)) ? gap(tlo[t], thi[t]) : 3.0e38f;
            unsigned long long tm = __ballot(lb < bound_f());
            while (tm) {
                const int k = __builtin_ctzll(tm);
                tm &= tm - 1;
                const float lbk = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(lb), k));
                if (!(lbk < bound_f())) continue;
                scan_tile(su * kSuper + k);
            }
        }
    }
    // outputs: the first K kept pairs in list order
    int c = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) c += __popcll(__ballot(64 * j + lane < K && Ld[j] < INF));
    const int o = out_input_order ? perm[q] : q;
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int e = 64 * j + lane;
        if (e < K) {
            if (nbr_idx) nbr_idx[(size_t)o * K + e] = e < c ? Li[j] : -1;
            if (nbr_d2) nbr_d2[(size_t)o * K + e] = e < c ? Ld[j] : 0.0;
        }
    }
    if (nbr_cnt && lane == 0) nbr_cnt[o] = c;
    if (mean_dist) {  // SOR: mean of sqrt(d^2) over the neighbours in list order (-1: empty search)
        double sd = 0.0;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const double sq = Ld[j] < INF ? sqrt(Ld[j]) : 0.0;
            for (int s2 = 0; s2 < 64 && 64 * j + s2 < c; ++s2) sd += lane_dbl(sq, s2);
        }
        if (lane == 0) mean_dist[o] = c > 0 ? sd / (double)c : -1.0;
    }
    if (!rawcov6) return;
    Sym3 C;
    if (c >= 3) {  // O3D ComputeCovariance: one-pass cumulants in list order, 1/n
        double cu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < P; ++j)
            for (int s2 = 0; s2 < 64 && 64 * j + s2 < c; ++s2) {
                const int jj = __builtin_amdgcn_readlane(Li[j], s2);
                const double px = in64[3 * jj], py = in64[3 * jj + 1], pz = in64[3 * jj + 2];
                cu[0] += px;
                cu[1] += py;
                cu[2] += pz;
                cu[3] += px * px;
                cu[4] += px * py;
                cu[5] += px * pz;
                cu[6] += py * py;
                cu[7] += py * pz;
                cu[8] += pz * pz;
            }
        const double cn = (double)c;
#pragma unroll
        for (int t = 0; t < 9; ++t) cu[t] /= cn;
        C.xx = cu[3] - cu[0] * cu[0];
        C.yy = cu[6] - cu[1] * cu[1];
        C.zz = cu[8] - cu[2] * cu[2];
        C.xy = cu[4] - cu[0] * cu[1];
        C.xz = cu[5] - cu[0] * cu[2];
        C.yz = cu[7] - cu[1] * cu[2];
    } else {
        C = Sym3{1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
    }
    if (lane == 0) {
        double* out = rawcov6 + (size_t)o * 6;
        out[0] = C.xx;
        out[1] = C.xy;
        out[2] = C.xz;
        out[3] = C.yy;
        out[4] = C.yz;
        out[5] = C.zz;
    }
}

// lane-per-query (knn_tiles_kernel, K <= 64): kout neighbours kept in a
// register list of the template's K >= kout; ties as launch_knn_cov_ties
static hipError_t launch_knn_lanes(const CloudLayout& L, const double* in64, int K, int kout, double r2,
                                   double margin, bool out_input_order, double* rawcov6, int32_t* nbr_idx,
                                   double* nbr_d2, int32_t* nbr_cnt, double* mean_dist, const KnnTieOut& ties,
                                   hipStream_t s, int t0 = 0, int t1 = -1) {
    if (t1 < 0) t1 = (int)L.ntiles;
    if (t1 <= t0) return hipSuccess;
    const dim3 grid((unsigned)((t1 - t0 + 3) / 4));
#define ORPCD_KNN_LANES(KK)                                                                                       \
    knn_tiles_kernel<KK><<<grid, 256, 0, s>>>(L.xyz64.p, L.perm.p, (int)L.n, L.tlo.p, L.thi.p, (int)L.ntiles,    \
                                              L.slo.p, L.shi.p, (int)L.nsuper, in64, r2, (float)margin,          \
                                              L.org[0], L.org[1], L.org[2], kout, out_input_order ? 1 : 0, rawcov6, \
                                              nbr_idx, nbr_d2, nbr_cnt, mean_dist, ties, t0, t1)
    if (K <= 8)
        ORPCD_KNN_LANES(8);
    else if (K <= 20)
        ORPCD_KNN_LANES(20);
    else if (K <= 21)
        ORPCD_KNN_LANES(21);  // KNN-20 with its tie detection (the 21st neighbour)
    else if (K <= 24)
        ORPCD_KNN_LANES(24);
    else if (K <= 32)
        ORPCD_KNN_LANES(32);
    else if (K <= 64)
        ORPCD_KNN_LANES(64);
    else
        return hipErrorInvalidValue;
#undef ORPCD_KNN_LANES
    return hipGetLastError();
}

hipError_t launch_knn_tiles(const CloudLayout& L, const double* in64, int k, double radius, double margin,
                            bool out_input_order, double* rawcov6, int32_t* nbr_idx, double* nbr_d2,
                            int32_t* nbr_cnt, hipStream_t s, double* mean_dist, bool lane_per_query) {
    if (L.n <= 0) return hipSuccess;
    const double r2 = radius > 0 ? radius * radius : __builtin_huge_val();
    if (lane_per_query && k >= 1 && k <= 64)
        return launch_knn_lanes(L, in64, k, k, r2, margin, out_input_order, rawcov6, nbr_idx, nbr_d2, nbr_cnt,
                                mean_dist, KnnTieOut{}, s);
    if (k >= 1 && k <= 64) {
        knn_wave_kernel<<<(unsigned)((L.n + 3) / 4), 256, 0, s>>>(
            L.xyz64.p, L.perm.p, (int)L.n, L.tlo.p, L.thi.p, (int)L.ntiles, L.slo.p, L.shi.p, (int)L.nsuper, in64, r2,
            (float)margin, L.org[0], L.org[1], L.org[2], k, out_input_order ? 1 : 0, rawcov6, nbr_idx, nbr_d2, nbr_cnt,
            mean_dist, k, KnnTieOut{});
        return hipGetLastError();
    }
    if (k > 64) {  // chunked sorted lists (knn_wave_multi_kernel), K <= kMaxKnn
#define ORPCD_KNN_MULTI(PP)                                                                                       \
    knn_wave_multi_kernel<PP><<<(unsigned)((L.n + 3) / 4), 256, 0, s>>>(                                          \
        L.xyz64.p, L.perm.p, (int)L.n, L.tlo.p, L.thi.p, (int)L.ntiles, L.slo.p, L.shi.p, (int)L.nsuper, in64, r2, \
        (float)margin, L.org[0], L.org[1], L.org[2], k, out_input_order ? 1 : 0, rawcov6, nbr_idx, nbr_d2, nbr_cnt, \
        mean_dist)
        if (k <= 128)
            ORPCD_KNN_MULTI(2);
        else if (k <= 256)
            ORPCD_KNN_MULTI(4);
        else if (k <= 512)
            ORPCD_KNN_MULTI(8);
        else if (k <= kMaxKnn)
            ORPCD_KNN_MULTI(16);
        else
            return hipErrorInvalidValue;
#undef ORPCD_KNN_MULTI
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

hipError_t launch_knn_batch(const BatchLayout& L, const int32_t* perm, const double* in64, const double* orgs,
                            const float* margins, int k, double radius, double* rawcov6, int32_t* nbr_idx,
                            double* nbr_d2, int32_t* nbr_cnt, hipStream_t s) {
    if (L.n <= 0 || L.B <= 0) return hipSuccess;
    if (k < 1 || k > 64) return hipErrorInvalidValue;
    const double r2 = radius > 0 ? radius * radius : __builtin_huge_val();
    knn_wave_kernel<<<dim3((unsigned)((L.n + 3) / 4), (unsigned)L.B), 256, 0, s>>>(
        L.xyz64.p, perm, (int)L.n, L.tlo.p, L.thi.p, (int)L.ntiles, L.slo.p, L.shi.p, (int)L.nsuper, in64, r2, 0.0f,
        0.0, 0.0, 0.0, k, 1, rawcov6, nbr_idx, nbr_d2, nbr_cnt, nullptr, k, KnnTieOut{}, orgs, margins);
    return hipGetLastError();
}

hipError_t launch_knn_cov_ties(const CloudLayout& L, const double* in64, int kcov, double margin, bool out_input_order,
                               double* rawcov6, const KnnTieOut& ties, hipStream_t s, bool lane_per_query,
                               const int32_t* qlist, int64_t nq) {
    if (L.n <= 0) return hipSuccess;
    // detect-only: the kcov + 1 nearest decide a tie; the listed pass keeps kcov + kTieExtra
    const int K = ties.detect ? kcov + 1 : kcov + kTieExtra;
    if (kcov < 1 || K > 64) return hipErrorInvalidValue;
    if (qlist) {  // listed queries only: one wave each
        if (nq <= 0) return hipSuccess;
        knn_wave_kernel<<<(unsigned)((nq + 3) / 4), 256, 0, s>>>(
            L.xyz64.p, L.perm.p, (int)L.n, L.tlo.p, L.thi.p, (int)L.ntiles, L.slo.p, L.shi.p, (int)L.nsuper, in64,
            __builtin_huge_val(), (float)margin, L.org[0], L.org[1], L.org[2], K, out_input_order ? 1 : 0, rawcov6,
            nullptr, nullptr, nullptr, nullptr, kcov, ties, nullptr, nullptr, qlist, (int)nq);
        return hipGetLastError();
    }
    if (lane_per_query)
        return launch_knn_lanes(L, in64, K, kcov, __builtin_huge_val(), margin, out_input_order, rawcov6, nullptr,
                                nullptr, nullptr, nullptr, ties, s);
    knn_wave_kernel<<<(unsigned)((L.n + 3) / 4), 256, 0, s>>>(
        L.xyz64.p, L.perm.p, (int)L.n, L.tlo.p, L.thi.p, (int)L.ntiles, L.slo.p, L.shi.p, (int)L.nsuper, in64,
        __builtin_huge_val(), (float)margin, L.org[0], L.org[1], L.org[2], K, out_input_order ? 1 : 0, rawcov6, nullptr,
        nullptr, nullptr, nullptr, kcov, ties);
    return hipGetLastError();
}

hipError_t launch_knn_cov_range(const CloudLayout& L, const double* in64, int k, double margin, double* rawcov6,
                                int64_t lo, int64_t hi, bool lane_per_query, hipStream_t s) {
    hi = std::min<int64_t>(hi, L.n);
    if (hi <= lo) return hipSuccess;
    if (k < 1 || k > 64) return hipErrorInvalidValue;
    if (lane_per_query) {  // whole tiles of queries: lo on a tile boundary, hi too unless it is the end
        if (lo % kTile || (hi % kTile && hi != L.n)) return hipErrorInvalidValue;
        return launch_knn_lanes(L, in64, k, k, __builtin_huge_val(), margin, false, rawcov6, nullptr, nullptr,
                                nullptr, nullptr, KnnTieOut{}, s, (int)(lo / kTile), (int)((hi + kTile - 1) / kTile));
    }
    knn_wave_kernel<<<(unsigned)((hi - lo + 3) / 4), 256, 0, s>>>(
        L.xyz64.p, L.perm.p, (int)L.n, L.tlo.p, L.thi.p, (int)L.ntiles, L.slo.p, L.shi.p, (int)L.nsuper, in64,
        __builtin_huge_val(), (float)margin, L.org[0], L.org[1], L.org[2], k, 0, rawcov6, nullptr, nullptr, nullptr,
        nullptr, k, KnnTieOut{}, nullptr, nullptr, nullptr, 0, (int)lo, (int)hi);
    return hipGetLastError();
}

// qlist[k] = Morton position of input row row_begin + k (inv: the layout's perm inverted)
__global__ void rows_to_positions_kernel(const int32_t* __restrict__ perm, int n, int64_t row_begin, int64_t nrows,
                                         int32_t* __restrict__ qlist) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const int64_t r = (int64_t)perm[k] - row_begin;
    if (r >= 0 && r < nrows) qlist[r] = k;
}
hipError_t launch_rows_to_positions(const int32_t* perm, int64_t n, int64_t row_begin, int64_t nrows, int32_t* qlist,
                                    hipStream_t s) {
    if (n <= 0) return hipSuccess;
    rows_to_positions_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(perm, (int)n, row_begin, nrows, qlist);
    return hipGetLastError();
}

// Overrides of single (slot, point) source covariances: the raw neighbourhood
// covariance of a boundary-tie point as its posed copy decides it (host,
// runtime.hip SourceTies), already in the posed frame (no rotation).
__global__ __launch_bounds__(64) void cov_override_kernel(const double* __restrict__ ent, int count, int n,
                                                          double eps, double* __restrict__ cov6) {
    const int e = blockIdx.x * 64 + threadIdx.x;
    if (e >= count) return;
    const double* r = ent + (size_t)e * 8;  // slot, Morton position, raw covariance (6)
    const int64_t slot = (int64_t)r[0], pos = (int64_t)r[1];
    Sym3 S{r[2], r[3], r[4], r[5], r[6], r[7]};
    double nrm[3];
    fast_eigen3x3(S, nrm);
    if (nrm[0] * nrm[0] + nrm[1] * nrm[1] + nrm[2] * nrm[2] == 0.0) {
        nrm[0] = 0.0;
        nrm[1] = 0.0;
        nrm[2] = 1.0;
    }
#if ORPCD_NORMAL_COV
    (void)eps;
    const bool quirk = nrm[0] < -0.99;
    double* o = cov6 + ((size_t)slot * n + pos) * 3;
    o[0] = quirk ? 1.0 : nrm[0];
    o[1] = quirk ? 0.0 : nrm[1];
    o[2] = quirk ? 0.0 : nrm[2];
#else
    Sym3 C = gicp_cov_from_normal(nrm, eps);
    double* o = cov6 + ((size_t)slot * n + pos) * 6;
    o[0] = C.xx;
    o[1] = C.xy;
    o[2] = C.xz;
    o[3] = C.yy;
    o[4] = C.yz;
    o[5] = C.zz;
#endif
}

hipError_t launch_cov_override(const double* ent, int count, int64_t n, double eps, double* cov6, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    cov_override_kernel<<<(unsigned)((count + 63) / 64), 64, 0, s>>>(ent, count, (int)n, eps, cov6);
    return hipGetLastError();
}

hipError_t launch_normals_cov(const double* rawcov6, int64_t n, const double* Rc9, int nslots, double eps,
                              double* normals3, double* cov6, hipStream_t s, double* enorm3) {
    const int64_t total = n * (int64_t)nslots;
    if (total <= 0) return hipSuccess;
    normals_cov_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(rawcov6, (int)n, Rc9, nslots, eps,
                                                                       normals3, cov6, enorm3);
    return hipGetLastError();
}

// this unit's code object loaded now (orpcd_ctx_create), not at its first launch
hipError_t preload_code_object_knn() {
    hipFuncAttributes attr;
    return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&normals_cov_kernel));
}

}  // namespace orpcd
