// knn_kernels.hip — per-point neighbourhood covariance and GICP covariance.
//
// Restates, for gfx950, Open3D 0.18 EstimatePerPointCovariances /
// EstimateNormals (KDTreeSearchParamKNN(20) inside registration_generalized_icp,
// generalizedICP.py:59-70; KDTreeSearchParamHybrid in fastGlobalOptimizer.py:118-127)
// and InitializePointCloudForGeneralizedICP.
//
// Design: exact brute-force K nearest in fp64 (one query per lane, cloud
// streamed through LDS in SoA tiles, broadcast reads).  The neighbour set is
// the K smallest by (d^2, index) — identical to the oracle's KD-tree result —
// and the cumulants are summed in that order with contraction off, so the
// covariance and FastEigen3x3 normal match the CPU restatement operation for
// operation.  This pass runs once per cloud (not per ICP iteration).
#include "device_math.h"
#include "orpcd_internal.h"

namespace orpcd {

constexpr int kKnnBlock = 256;
constexpr int kKnnTile = 1024;

template <int K>
__global__ __launch_bounds__(kKnnBlock) void knn_cov_kernel(const double* __restrict__ pts, int n, double r2,
                                                            double* __restrict__ rawcov6,
                                                            int32_t* __restrict__ nbr_idx, double* __restrict__ nbr_d2,
                                                            int32_t* __restrict__ nbr_cnt, int kout) {
    __shared__ double sx[kKnnTile], sy[kKnnTile], sz[kKnnTile];
    const int i = blockIdx.x * kKnnBlock + threadIdx.x;
    const bool valid = i < n;
    double qx = 0.0, qy = 0.0, qz = 0.0;
    if (valid) {
        qx = pts[3 * i];
        qy = pts[3 * i + 1];
        qz = pts[3 * i + 2];
    }
    double bd[K];
    int bi[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
        bd[s] = r2;
        bi[s] = -1;
    }
    for (int t0 = 0; t0 < n; t0 += kKnnTile) {
        const int cnt = min(kKnnTile, n - t0);
        __syncthreads();
        for (int k = threadIdx.x; k < cnt; k += kKnnBlock) {
            sx[k] = pts[3 * (t0 + k)];
            sy[k] = pts[3 * (t0 + k) + 1];
            sz[k] = pts[3 * (t0 + k) + 2];
        }
        __syncthreads();
        for (int k = 0; k < cnt; ++k) {
            double d;
            {
#pragma clang fp contract(off)
                double dx = qx - sx[k], dy = qy - sy[k], dz = qz - sz[k];
                d = dx * dx + dy * dy + dz * dz;
            }
            if (d < bd[K - 1]) {
                double cd = d;
                int ci = t0 + k;
#pragma unroll
                for (int s = 0; s < K; ++s) {
                    const bool sw = cd < bd[s];
                    const double td = bd[s];
                    const int ti = bi[s];
                    bd[s] = sw ? cd : td;
                    bi[s] = sw ? ci : ti;
                    cd = sw ? td : cd;
                    ci = sw ? ti : ci;
                }
            }
        }
    }
    if (!valid) return;
    int c = 0;
#pragma unroll
    for (int s = 0; s < K; ++s) c += (s < kout && bi[s] >= 0) ? 1 : 0;
    if (nbr_idx) {
#pragma unroll
        for (int s = 0; s < K; ++s)
            if (s < kout) nbr_idx[(size_t)i * kout + s] = s < c ? bi[s] : -1;
    }
    if (nbr_d2) {
#pragma unroll
        for (int s = 0; s < K; ++s)
            if (s < kout) nbr_d2[(size_t)i * kout + s] = s < c ? bd[s] : 0.0;
    }
    if (nbr_cnt) nbr_cnt[i] = c;
    if (!rawcov6) return;
    Sym3 C;
    if (c >= 3) {
#pragma clang fp contract(off)
        double cu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < K; ++s) {
            if (s < c) {
                const int j = bi[s];
                const double px = pts[3 * j], py = pts[3 * j + 1], pz = pts[3 * j + 2];
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
    double* o = rawcov6 + (size_t)i * 6;
    o[0] = C.xx;
    o[1] = C.xy;
    o[2] = C.xz;
    o[3] = C.yy;
    o[4] = C.yz;
    o[5] = C.zz;
}

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

hipError_t launch_knn_cov(const double* pts, int64_t n, int k, double radius, double* rawcov6, int32_t* nbr_idx,
                          double* nbr_d2, int32_t* nbr_cnt, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const double r2 = radius > 0 ? radius * radius : __builtin_huge_val();
    const dim3 grid((unsigned)((n + kKnnBlock - 1) / kKnnBlock));
    if (k <= 8)
        knn_cov_kernel<8><<<grid, kKnnBlock, 0, s>>>(pts, (int)n, r2, rawcov6, nbr_idx, nbr_d2, nbr_cnt, k);
    else if (k <= 20)
        knn_cov_kernel<20><<<grid, kKnnBlock, 0, s>>>(pts, (int)n, r2, rawcov6, nbr_idx, nbr_d2, nbr_cnt, k);
    else if (k <= 32)
        knn_cov_kernel<32><<<grid, kKnnBlock, 0, s>>>(pts, (int)n, r2, rawcov6, nbr_idx, nbr_d2, nbr_cnt, k);
    else if (k <= 64)
        knn_cov_kernel<64><<<grid, kKnnBlock, 0, s>>>(pts, (int)n, r2, rawcov6, nbr_idx, nbr_d2, nbr_cnt, k);
    else
        return hipErrorInvalidValue;
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
