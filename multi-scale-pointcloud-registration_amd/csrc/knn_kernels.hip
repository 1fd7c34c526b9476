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
                                                          double* __restrict__ cov6) {
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

template <int K>
__global__ __launch_bounds__(256) void knn_tiles_kernel(
    const double* __restrict__ xyz64, const int32_t* __restrict__ perm, int n, const float4* __restrict__ tlo,
    const float4* __restrict__ thi, int ntiles, const float4* __restrict__ slo, const float4* __restrict__ shi,
    int nsuper, const double* __restrict__ in64, double r2, float margin, int kout, int out_input_order,
    double* __restrict__ rawcov6, int32_t* __restrict__ nbr_idx, double* __restrict__ nbr_d2,
    int32_t* __restrict__ nbr_cnt, double* __restrict__ mean_dist) {
    __shared__ double sx[4][kTile], sy[4][kTile], sz[4][kTile];
    __shared__ int32_t sid[4][kTile];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int own = blockIdx.x * 4 + w;  // the wave's own tile
    if (own >= ntiles) return;           // wave-uniform
    const int q = own * kTile + lane;
    const bool valid = q < n;
    const double qx = valid ? xyz64[3 * q] : 0.0, qy = valid ? xyz64[3 * q + 1] : 0.0,
                 qz = valid ? xyz64[3 * q + 2] : 0.0;
    double bd[K];
    int bi[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
        bd[s] = r2;
        bi[s] = -1;
    }
    // Two phases per staged tile: (1) every lane marks the candidates that
    // beat its bound at tile start (the bound only shrinks, so this is a
    // superset); (2) each lane walks only its own marks.  The wave then pays
    // the insertion network max_lane(marks) times instead of once for every
    // candidate that ANY lane takes.
    auto scan_tile = [&](int t) {
        const int k = t * kTile + lane;
        const bool real = k < n;
        sx[w][lane] = real ? xyz64[3 * k] : 1e300;
        sy[w][lane] = real ? xyz64[3 * k + 1] : 1e300;
        sz[w][lane] = real ? xyz64[3 * k + 2] : 1e300;
        sid[w][lane] = real ? perm[k] : 0x7fffffff;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        auto dist = [&](int c) {
#pragma clang fp contract(off)
            const double dx = qx - sx[w][c], dy = qy - sy[w][c], dz = qz - sz[w][c];
            return dx * dx + dy * dy + dz * dz;
        };
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
    // own tile, then its Morton neighbours: a near-final bound before the walk
    constexpr int kWin = 2;
    scan_tile(own);
    for (int dt = 1; dt <= kWin; ++dt) {
        if (own - dt >= 0) scan_tile(own - dt);
        if (own + dt < ntiles) scan_tile(own + dt);
    }

    const float inf = 3.0e38f;
    const float fx = (float)qx, fy = (float)qy, fz = (float)qz;
    const float lox = wave_fmin(valid ? fx : inf), hix = wave_fmax(valid ? fx : -inf);
    const float loy = wave_fmin(valid ? fy : inf), hiy = wave_fmax(valid ? fy : -inf);
    const float loz = wave_fmin(valid ? fz : inf), hiz = wave_fmax(valid ? fz : -inf);
    auto lane_bound = [&]() -> float {  // fp32 upper bound of the lane's K-th distance
        if (!valid) return 0.0f;
        const double b = bd[K - 1];
        return b >= 3.0e38 ? inf : (float)b * 1.0000003f + 1e-37f;
    };
    for (int sb = 0; sb < nsuper; sb += 64) {
        float Wb = wave_fmax(lane_bound());
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
            Wb = wave_fmax(lane_bound());
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
                const float gx = gapf(ax, bx, fx, margin), gy = gapf(ay, by, fy, margin), gz = gapf(az, bz, fz, margin);
                const bool need = valid && gx * gx + gy * gy + gz * gz < lane_bound();
                if (__ballot(need) == 0ull) continue;
                scan_tile(su * kSuper + k);
            }
        }
    }
    if (!valid) return;
    int c = 0;
#pragma unroll
    for (int s = 0; s < K; ++s) c += (s < kout && bi[s] >= 0) ? 1 : 0;
    const int o = out_input_order ? perm[q] : q;
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

hipError_t launch_knn_tiles(const CloudLayout& L, const double* in64, int k, double radius, double margin,
                            bool out_input_order, double* rawcov6, int32_t* nbr_idx, double* nbr_d2,
                            int32_t* nbr_cnt, hipStream_t s, double* mean_dist) {
    if (L.n <= 0) return hipSuccess;
    const double r2 = radius > 0 ? radius * radius : __builtin_huge_val();
    const dim3 grid((unsigned)((L.ntiles + 3) / 4));
#define ORPCD_KNN_TILES(KK)                                                                                      \
    knn_tiles_kernel<KK><<<grid, 256, 0, s>>>(L.xyz64.p, L.perm.p, (int)L.n, L.tlo.p, L.thi.p, (int)L.ntiles,   \
                                              L.slo.p, L.shi.p, (int)L.nsuper, in64, r2, (float)margin, k,      \
                                              out_input_order ? 1 : 0, rawcov6, nbr_idx, nbr_d2, nbr_cnt, mean_dist)
    if (k <= 8)
        ORPCD_KNN_TILES(8);
    else if (k <= 20)
        ORPCD_KNN_TILES(20);
    else if (k <= 32)
        ORPCD_KNN_TILES(32);
    else if (k <= 64)
        ORPCD_KNN_TILES(64);
    else
        return hipErrorInvalidValue;
#undef ORPCD_KNN_TILES
    return hipGetLastError();
}

hipError_t launch_normals_cov(const double* rawcov6, int64_t n, const double* Rc9, int nslots, double eps,
                              double* normals3, double* cov6, hipStream_t s) {
    const int64_t total = n * (int64_t)nslots;
    if (total <= 0) return hipSuccess;
    normals_cov_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(rawcov6, (int)n, Rc9, nslots, eps,
                                                                       normals3, cov6);
    return hipGetLastError();
}

}  // namespace orpcd
