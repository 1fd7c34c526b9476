// fgr_kernels.hip — FastGlobalOptimizer path on gfx950.
//
// Restates, for the reference's FastGlobalOptimizer (fastGlobalOptimizer.py:109-190):
//   * compute_fpfh_feature (O3D Feature.cpp ComputeSPFHFeature / ComputeFPFHFeature)
//     over Hybrid(r, k) neighbourhoods from knn_cov_kernel;
//   * InitialMatching of O3D FastGlobalRegistration.cpp: nearest neighbour in
//     the 33-D feature space in both directions.  This is the genuine dense
//     contraction of the path: d(q, t) = |q|^2 + |t|^2 - 2 q.t with q.t on the
//     fp64 matrix cores (v_mfma_f64_16x16x4_f64, K = 33 padded to 36, 9 MFMAs
//     per 16x16 tile).  fp64 keeps the mutual-match set identical to the
//     oracle's: FGR's tuple sampling indexes into that list, so one different
//     match would change every later tuple;
//   * OptimizePairwiseRegistration (GNC / Geman-McClure IRLS, 100 iterations)
//     in one workgroup, fixed-order reductions, fp64;
//   * the normalisation means / radius and EvaluateRegistration's reduction.
//   * AdvancedMatching's tuple test: 100 x ncorr trials of three draws of a
//     seeded mt19937 through uniform_int_distribution, kept in trial order up
//     to maximum_tuple_count.  The draws are sequential, the trials are not:
//     the raw word stream depends only on the seed (generated once on the
//     host and cached), uniform_int_distribution's mapping of a word only on
//     ncorr (Lemire's method: the rare rejected words are listed per start),
//     so every trial of every start is evaluated at once and the accepted
//     ones are compacted in order.
#include <cstdio>
#include <cstdlib>

#include <hipcub/hipcub.hpp>

#include "device_math.h"
#include "orpcd_internal.h"

namespace orpcd {

typedef double d4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------- FPFH
// Contraction off: the swap test below compares acos(|a1|) with acos(|a2|),
// which for nearly parallel normals is decided by the last bits of a1 and a2;
// unfused arithmetic keeps those bits equal to the CPU restatement's.
__device__ inline void pair_features(const double p1[3], const double n1[3], const double p2[3], const double n2[3],
                                     double out[4]) {
#pragma clang fp contract(off)
    double d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    out[3] = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    if (out[3] == 0.0) {
        out[0] = out[1] = out[2] = out[3] = 0.0;
        return;
    }
    double a[3] = {n1[0], n1[1], n1[2]}, b[3] = {n2[0], n2[1], n2[2]};
    const double angle1 = (a[0] * d[0] + a[1] * d[1] + a[2] * d[2]) / out[3];
    const double angle2 = (b[0] * d[0] + b[1] * d[1] + b[2] * d[2]) / out[3];
    if (acos(fabs(angle1)) > acos(fabs(angle2))) {
        for (int t = 0; t < 3; ++t) {
            const double tmp = a[t];
            a[t] = b[t];
            b[t] = tmp;
            d[t] = -d[t];
        }
        out[2] = -angle2;
    } else {
        out[2] = angle1;
    }
    double v[3];
    cross3(d, a, v);
    const double vn = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (vn == 0.0) {
        out[0] = out[1] = out[2] = out[3] = 0.0;
        return;
    }
    v[0] /= vn;
    v[1] /= vn;
    v[2] /= vn;
    double w[3];
    cross3(a, v, w);
    out[1] = v[0] * b[0] + v[1] * b[1] + v[2] * b[2];
    out[0] = atan2(w[0] * b[0] + w[1] * b[1] + w[2] * b[2], a[0] * b[0] + a[1] * b[1] + a[2] * b[2]);
}

__device__ __forceinline__ int fpfh_bin(double x) {
    int h = (int)floor(x);
    return h < 0 ? 0 : (h >= 11 ? 10 : h);
}

// SPFH: one thread per point, histogram in LDS (64 threads x 33 doubles).
// blockIdx.y: cloud y of a batch (every array at its per-cloud stride,
// neighbour indices within the cloud); one cloud: y = 0.
__global__ __launch_bounds__(64) void spfh_kernel(const double* __restrict__ pts, const double* __restrict__ nrm,
                                                  int n, const int32_t* __restrict__ nbr,
                                                  const int32_t* __restrict__ cnt, int k, double* __restrict__ spfh) {
    pts += (size_t)blockIdx.y * 3 * n;
    nrm += (size_t)blockIdx.y * 3 * n;
    nbr += (size_t)blockIdx.y * n * k;
    cnt += (size_t)blockIdx.y * n;
    spfh += (size_t)blockIdx.y * 33 * n;
    __shared__ double h[64][33];
    const int i = blockIdx.x * 64 + threadIdx.x;
    for (int j = 0; j < 33; ++j) h[threadIdx.x][j] = 0.0;
    if (i < n) {
        const int c = cnt[i];
        if (c > 1) {
            const double incr = 100.0 / (double)(c - 1);
            const double p1[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
            const double n1[3] = {nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2]};
            for (int s = 1; s < c; ++s) {
                const int j = nbr[(size_t)i * k + s];
                const double p2[3] = {pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]};
                const double n2[3] = {nrm[3 * j], nrm[3 * j + 1], nrm[3 * j + 2]};
                double pf[4];
                pair_features(p1, n1, p2, n2, pf);
                h[threadIdx.x][fpfh_bin(11 * (pf[0] + M_PI) / (2.0 * M_PI))] += incr;
                h[threadIdx.x][fpfh_bin(11 * (pf[1] + 1.0) * 0.5) + 11] += incr;
                h[threadIdx.x][fpfh_bin(11 * (pf[2] + 1.0) * 0.5) + 22] += incr;
            }
        }
        for (int j = 0; j < 33; ++j) spfh[(size_t)i * 33 + j] = h[threadIdx.x][j];
    }
}

// FPFH: weighted sum of the neighbours' SPFH (1/d^2), per-block renormalised
// to 100, plus the point's own SPFH.  Output padded to kFD columns (zeros).
constexpr int kFD = 36;
__global__ __launch_bounds__(256) void fpfh_kernel(const double* __restrict__ spfh, int n,
                                                   const int32_t* __restrict__ nbr, const double* __restrict__ d2,
                                                   const int32_t* __restrict__ cnt, int k, double* __restrict__ feat) {
#pragma clang fp contract(off)
    spfh += (size_t)blockIdx.y * 33 * n;  // cloud y of a batch
    nbr += (size_t)blockIdx.y * n * k;
    d2 += (size_t)blockIdx.y * n * k;
    cnt += (size_t)blockIdx.y * n;
    feat += (size_t)blockIdx.y * kFD * n;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double f[33];
#pragma unroll
    for (int j = 0; j < 33; ++j) f[j] = 0.0;
    const int c = cnt[i];
    if (c > 1) {
        double sum[3] = {0.0, 0.0, 0.0};
        for (int s = 1; s < c; ++s) {
            const double dist = d2[(size_t)i * k + s];
            if (dist == 0.0) continue;
            const double* sp = spfh + (size_t)nbr[(size_t)i * k + s] * 33;
#pragma unroll
            for (int j = 0; j < 33; ++j) {
                const double val = sp[j] / dist;
                sum[j / 11] += val;
                f[j] += val;
            }
        }
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (sum[j] != 0.0) sum[j] = 100.0 / sum[j];
#pragma unroll
        for (int j = 0; j < 33; ++j) f[j] = f[j] * sum[j / 11] + spfh[(size_t)i * 33 + j];
    }
#pragma unroll
    for (int j = 0; j < 33; ++j) feat[(size_t)i * kFD + j] = f[j];
#pragma unroll
    for (int j = 33; j < kFD; ++j) feat[(size_t)i * kFD + j] = 0.0;
}

// Pad caller-supplied n x 33 features to n x kFD.
__global__ void pad_features_kernel(const double* __restrict__ in, int n, double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int j = 0; j < 33; ++j) out[(size_t)i * kFD + j] = in[(size_t)i * 33 + j];
    for (int j = 33; j < kFD; ++j) out[(size_t)i * kFD + j] = 0.0;
}

__global__ void feat_norm_kernel(const double* __restrict__ F, int n, double* __restrict__ nrm2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int j = 0; j < kFD; ++j) s += F[(size_t)i * kFD + j] * F[(size_t)i * kFD + j];
    nrm2[i] = s;
}

// ------------------------------------------------ feature nearest neighbour
// Two passes over the targets on the fp64 matrix cores.
//
// Pass 1 (EXACT = false), every query: the target minimising the expansion
// |q|^2 + |t|^2 - 2 q.t (ties -> lowest index) and the runner-up distance.
// The expansion carries a rounding error of ~40 ulp of the norms, so it
// cannot order rows that are equal up to their last bits — FPFH produces many
// of those (neighbourhoods whose pair features all fall in the same bins).
// Queries whose best and runner-up lie within that bound are flagged.
//
// Pass 2 (EXACT = true), flagged queries only (compacted): the same products,
// and every target within the bound of the pass-1 best is re-measured with
// the oracle's distance (sum of squared differences in column order,
// unfused); the lexicographic (d, index) minimum of those wins.  Exact
// duplicate target rows are collapsed to their lowest index beforehand
// (dedup_rows): their exact distances are equal, so that is the answer the
// oracle gives, and the near-tie sets stay small.
//
// Tiling: one wave owns 64 queries as 4 column tiles of 16; the block stages
// 64 targets x 36 in LDS.  D[i][j] = C[i][j] + sum_k A[i][k] B[k][j] with
// A = 16 targets (lane l supplies A[l&15][l>>4]), B = -2 x 16 queries (lane l
// supplies B[l>>4][l&15]; the scaling is exact) and C = |q_j|^2, so the f64
// accumulator holds |q|^2 - 2 q.t at D[(l>>4) + 4r][l&15], r = 0..3, and a
// distance costs one add.  blockIdx.y splits the targets into parts
// (feat_nn_parts; merged by the merge kernels).  The accumulation order
// differs from |t|^2 + |q|^2 - 2 q.t by rounding only, inside the flag bound.
constexpr int kFT = 64;
constexpr int kMaxParts = 32;  // target parts per launch (feat_nn_parts)
// Padded target rows (past a part's end) carry this norm: their distances
// are huge but finite, so a key built from one is never a NaN.
constexpr double kPadNorm = 1e300;

// Pass-1 key: the distance with its low `bits` mantissa bits replaced by the
// target's index within the part (one v_bfi_b32).  Keys of distinct targets
// differ, order as their distances up to 2^(bits-52) relative, and the
// running best and runner-up become two minima and a maximum.
__host__ __device__ inline int feat_key_bits(int part_len) {
    int b = 1;
    while ((1 << b) < part_len) ++b;
    return b;
}
__device__ __forceinline__ double feat_key(double d, unsigned idx, unsigned mask) {
    const unsigned lo = (unsigned)__double2loint(d);
    return __hiloint2double(__double2hiint(d), (int)((lo & ~mask) | idx));
}
// v_min_f64 / v_max_f64 without the canonicalising moves the compiler adds for
// fmin/fmax of values it cannot prove canonical (keys are built bitwise; no
// operand is ever a NaN)
__device__ __forceinline__ double vmin_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmax_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// (d, i, s) <- merge with (od, oi, os): best distance, its lowest index, and
// the runner-up distance (a tie at the best counts as a runner-up).
__device__ __forceinline__ void merge_best(double& d, int& i, double& s, double od, int oi, double os) {
    if (oi < 0) return;
    if (i < 0 || od < d) {
        s = fmin(os, i < 0 ? __builtin_huge_val() : d);
        d = od;
        i = oi;
    } else if (od > d) {
        s = fmin(s, od);
    } else {
        s = od;
        i = min(i, oi);
    }
}

__device__ __forceinline__ void merge_lex(double& d, int& i, double od, int oi) {
    if (oi >= 0 && (i < 0 || od < d || (od == d && oi < i))) {
        d = od;
        i = oi;
    }
}

// EXACT: qidx / nsel / thr give the compacted flagged queries and their
// pass-1 thresholds; out_s is unused.  KB: MFMAs per 16x16 tile.  9 covers
// all 36 columns; 8 (dim <= 33, the FPFH case) covers columns 0..31 and adds
// column 32 with one VALU fma per element, skipping the zero padding's MFMA
// (an eighth of the matrix work).
template <bool EXACT, int KB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void feat_nn_kernel(const double* __restrict__ Fq, const double* __restrict__ nq2,
                                                      int nq, const int32_t* __restrict__ qidx,
                                                      const int32_t* __restrict__ nsel,
                                                      const double* __restrict__ thr, const double* __restrict__ Ft,
                                                      const double* __restrict__ nt2, int nt, int part_len, int dim,
                                                      double* __restrict__ out_d, double* __restrict__ out_s,
                                                      int32_t* __restrict__ out_i, const uint32_t* __restrict__ need,
                                                      int len1) {
    // double-buffered stage: the next 64 targets are loaded into registers
    // while the current ones are multiplied, then written to the other buffer
    // (one barrier per stage)
    __shared__ double sT2[2][kFT][kFD + 1];
    __shared__ double sN2[2][kFT];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nrow = EXACT ? *nsel : nq;  // queries (rows of the compact list in EXACT mode)
    if ((int)blockIdx.x * 256 >= nrow) return;  // block-uniform
    const int q0 = (blockIdx.x * 4 + wid) * 64;
    const int t_begin = blockIdx.y * part_len, t_end = min(nt, t_begin + part_len);
    static_assert(KB == 8 || KB == 9, "KB");
    if (EXACT && need) {
        // pass 2 over a sub-part: skipped (empty results) when no row of the
        // block can have a candidate in the pass-1 parts it overlaps
        uint32_t range = 0;
        if (t_begin < t_end) {
            const int p_lo = t_begin / len1, p_hi = (t_end - 1) / len1;
            range = (p_hi >= 31 ? 0xFFFFFFFFu : ((1u << (p_hi + 1)) - 1u)) & ~((1u << p_lo) - 1u);
        }
        const int j = (int)blockIdx.x * 256 + (int)threadIdx.x;
        if (!__syncthreads_or(j < nrow && (need[j] & range) != 0)) {
            if (j < nrow) {
                out_d[(size_t)blockIdx.y * nq + j] = __builtin_huge_val();
                out_i[(size_t)blockIdx.y * nq + j] = -1;
            }
            return;
        }
    }
    double b[4][9], qn[4], th[4], c32[4];
    const double* qrow[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
        const int j = q0 + 16 * qt + (lane & 15);
        const int q = j < nrow ? (EXACT ? qidx[j] : j) : -1;
        qn[qt] = q >= 0 ? nq2[q] : 0.0;
        th[qt] = (EXACT && q >= 0) ? thr[q] : -1.0;
        qrow[qt] = Fq + (size_t)(q >= 0 ? q : 0) * kFD;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) b[qt][kb] = q >= 0 ? -2.0 * qrow[qt][4 * kb + (lane >> 4)] : 0.0;
        c32[qt] = (KB == 8 && q >= 0) ? -2.0 * qrow[qt][32] : 0.0;
    }
    const double inf = __builtin_huge_val();
    double bd[4] = {inf, inf, inf, inf}, b2[4] = {inf, inf, inf, inf};
    int bi[4] = {-1, -1, -1, -1};
    constexpr int kPer = kFT * kFD / 256;  // staged doubles per thread
    static_assert(kFT * kFD % 256 == 0, "stage split");
    double pre[kPer], preN = kPadNorm;
    const unsigned kmask = (1u << feat_key_bits(part_len)) - 1u;
    auto load_stage = [&](int t0) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            // rows past the part's end re-read its last row (no branch per
            // load): their distances are inf through sN, whatever the row
            const int e = threadIdx.x + 256 * u, r = e / kFD, col = e - r * kFD;
            pre[u] = Ft[(size_t)min(t0 + r, t_end - 1) * kFD + col];
        }
        if (threadIdx.x < kFT) preN = (t0 + threadIdx.x < t_end) ? nt2[t0 + threadIdx.x] : kPadNorm;
    };
    auto store_stage = [&](int buf) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int e = threadIdx.x + 256 * u, r = e / kFD, col = e - r * kFD;
            sT2[buf][r][col] = pre[u];
        }
        if (threadIdx.x < kFT) sN2[buf][threadIdx.x] = preN;
    };
    if (t_begin < t_end) {
        load_stage(t_begin);
        store_stage(0);
    }
    __syncthreads();
    for (int t0 = t_begin, buf = 0; t0 < t_end; t0 += kFT, buf ^= 1) {
        const bool more = t0 + kFT < t_end;
        if (more) load_stage(t0 + kFT);
        double(*sT)[kFD + 1] = sT2[buf];
        const double* sN = sN2[buf];
#pragma unroll 1
        for (int sub = 0; sub < kFT / 16; ++sub) {
            d4 acc[4];
#pragma unroll
            for (int qt = 0; qt < 4; ++qt) acc[qt] = d4{qn[qt], qn[qt], qn[qt], qn[qt]};
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                const double a = sT[sub * 16 + (lane & 15)][4 * kb + (lane >> 4)];
#pragma unroll
                for (int qt = 0; qt < 4; ++qt) acc[qt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[qt][kb], acc[qt], 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = sub * 16 + (lane >> 4) + 4 * r;
                const double tn = sN[row];
                const double t32 = KB == 8 ? sT[row][32] : 0.0;
                const unsigned lidx = (unsigned)(t0 - t_begin + row);
#pragma unroll
                for (int qt = 0; qt < 4; ++qt) {
                    const double d = KB == 8 ? tn + fma(c32[qt], t32, acc[qt][r]) : tn + acc[qt][r];
                    if (!EXACT) {
                        // best and runner-up keys: five VALU per element, no
                        // compare or select (the compare/select form cost 11
                        // and held pass 1 at 9.3 ms against 8.2)
                        const double key = feat_key(d, lidx, kmask);
                        b2[qt] = vmin_f64(b2[qt], vmax_f64(bd[qt], key));
                        bd[qt] = vmin_f64(bd[qt], key);
                    } else if (d <= th[qt]) {
                        double ex = 0.0;
                        {
#pragma clang fp contract(off)
                            for (int k = 0; k < dim; ++k) {
                                const double df = qrow[qt][k] - sT[row][k];
                                ex += df * df;
                            }
                        }
                        if (ex < bd[qt]) {  // increasing rows per lane: strict keeps the lowest index
                            bd[qt] = ex;
                            bi[qt] = t0 + row;
                        }
                    }
                }
            }
        }
        // the other buffer was last read in the previous stage, before the
        // barrier that ended it
        if (more) store_stage(buf ^ 1);
        __syncthreads();
    }
    if (!EXACT) {
#pragma unroll
        for (int qt = 0; qt < 4; ++qt) {
            // a key's index is a row of this part; a padded row (past t_end)
            // can only win if every real distance was a NaN key, which the
            // entry points exclude (feature_rows_ok) -- dropped all the same
            const int cand = (int)((unsigned)__double2loint(bd[qt]) & kmask) + t_begin;
            bi[qt] = bd[qt] < inf && cand < t_end ? cand : -1;
        }
    }
    // merge the 4 lane groups (l>>4) holding the same query column
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
#pragma unroll
        for (int off = 16; off < 64; off <<= 1) {
            const double od = __shfl_xor(bd[qt], off, 64), os = __shfl_xor(b2[qt], off, 64);
            const int oi = __shfl_xor(bi[qt], off, 64);
            if (EXACT)
                merge_lex(bd[qt], bi[qt], od, oi);
            else
                merge_best(bd[qt], bi[qt], b2[qt], od, oi, os);
        }
        const int j = q0 + 16 * qt + lane;
        if (lane < 16 && j < nrow) {
            out_d[(size_t)blockIdx.y * nq + j] = bd[qt];
            if (!EXACT) out_s[(size_t)blockIdx.y * nq + j] = b2[qt];
            out_i[(size_t)blockIdx.y * nq + j] = bi[qt];
        }
    }
}

// Pass-1 merge over the target parts: answer, flag and pass-2 threshold.
// The expansion's error is ~40 ulp of the norms; 2e-13 relative leaves a
// wide margin (twice: the best's and the competitor's error).
__global__ void merge_parts_kernel(const double* __restrict__ pd, const double* __restrict__ ps,
                                   const int32_t* __restrict__ pi, int nq, int nparts, const double* __restrict__ nq2,
                                   const double* __restrict__ nt2, const int32_t* __restrict__ tmap,
                                   int32_t* __restrict__ out, int32_t* __restrict__ flag, double* __restrict__ thr,
                                   double key_slack, uint32_t* __restrict__ need) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    double bd = pd[q], bs = ps[q];
    int bi = pi[q];
    for (int p = 1; p < nparts; ++p)  // parts cover increasing target ranges
        merge_best(bd, bi, bs, pd[(size_t)p * nq + q], pi[(size_t)p * nq + q], ps[(size_t)p * nq + q]);
    out[q] = bi >= 0 && tmap ? tmap[bi] : bi;
    // + the keys' perturbation (key_slack = 2^(bits-51): twice 2^(bits-52))
    const double tol = 2e-13 * (nq2[q] + (bi >= 0 ? nt2[bi] : 0.0) + fabs(bd)) +
                       key_slack * (fabs(bd) + (bs < __builtin_huge_val() ? fabs(bs) : 0.0));
    flag[q] = (bi >= 0 && bs - bd <= tol) ? 1 : 0;
    const double th = bd + 2.0 * tol;
    thr[q] = th;
    // the parts that can hold a pass-2 candidate: every target of part p
    // has an expansion >= its best key - the key perturbation, and pass 2's
    // expansions differ from pass 1's by less than tol
    uint32_t m = 0;
    for (int p = 0; p < nparts; ++p) {
        const double kp = pd[(size_t)p * nq + q];
        if (pi[(size_t)p * nq + q] >= 0 && kp <= th + tol + key_slack * (fabs(kp) + fabs(th))) m |= 1u << p;
    }
    need[q] = m;
}

// need[j] = need_q[qidx[j]] for the compact list (sort keys of pass 2's order)
__global__ void gather_need_kernel(const int32_t* __restrict__ qidx, const int32_t* __restrict__ nsel,
                                   const uint32_t* __restrict__ need_q, uint32_t* __restrict__ key) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < *nsel) key[j] = need_q[qidx[j]];
}

// Pass-2 merge (lexicographic on the exact distance) into the answers.
__global__ void merge_exact_kernel(const double* __restrict__ pd, const int32_t* __restrict__ pi, int nq,
                                   int nparts, const int32_t* __restrict__ qidx, const int32_t* __restrict__ nsel,
                                   const int32_t* __restrict__ tmap, int32_t* __restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= *nsel) return;
    double bd = pd[j];
    int bi = pi[j];
    for (int p = 1; p < nparts; ++p) merge_lex(bd, bi, pd[(size_t)p * nq + j], pi[(size_t)p * nq + j]);
    if (bi >= 0) out[qidx[j]] = tmap ? tmap[bi] : bi;
}

// ------------------------------------------------ duplicate target rows
// hash -> stable sort -> run heads -> representative = lowest index of an
// equal row; compact list of representatives in increasing index order.
__global__ void row_hash_kernel(const double* __restrict__ F, int n, unsigned long long* __restrict__ key,
                                int32_t* __restrict__ val) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long h = 0x9E3779B97F4A7C15ull;
    for (int k = 0; k < kFD; ++k) {
        h ^= (unsigned long long)__double_as_longlong(F[(size_t)i * kFD + k]);
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 31;
    }
    key[i] = h;
    val[i] = i;
}

// seg: rows per segment (a batch's clouds sorted segment by segment; a run
// never crosses a segment); one cloud: seg = n
__global__ void run_start_kernel(const unsigned long long* __restrict__ ks, int n, int32_t* __restrict__ hv,
                                 int seg) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    hv[p] = (p % seg == 0 || ks[p] != ks[p - 1]) ? p : 0;
}

__global__ void representative_kernel(const double* __restrict__ F, const int32_t* __restrict__ vs,
                                      const int32_t* __restrict__ head, int n, unsigned char* __restrict__ uflag) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int i = vs[p], h = vs[head[p]];
    bool same = i != h;
    for (int k = 0; k < kFD && same; ++k) same = F[(size_t)i * kFD + k] == F[(size_t)h * kFD + k];
    uflag[i] = same ? 0 : 1;
}

__global__ void gather_rows_kernel(const double* __restrict__ F, const double* __restrict__ n2,
                                   const int32_t* __restrict__ idx, int nu, double* __restrict__ Fu,
                                   double* __restrict__ n2u) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nu * kFD) return;
    const int u = e / kFD, k = e - u * kFD;
    const int i = idx[u];
    Fu[e] = F[(size_t)i * kFD + k];
    if (k == 0) n2u[u] = n2[i];
}

// ------------------------------------------------------ IRLS (one block)
// O3D FastGlobalRegistration.cpp OptimizePairwiseRegistration over the tuple
// correspondences: p (normalised source) and q (normalised target, moved by
// every update in place).
// One correspondence's Geman-McClure weighted terms (21 JTJ + 6 JTr), with
// J = [[0, -z, y, -1, 0, 0], [z, 0, -x, 0, -1, 0], [-y, x, 0, 0, 0, -1]]
// written out: the terms J's zeros contribute are exact no-ops of the
// generic form (irls_terms), so only the nonzero ones are formed, in the
// same row order a = 0, 1, 2 — 27 accumulations instead of 63 products
// (the register-resident kernel runs on one CU, where its fp64 VALU work is
// the iteration's longest stage).
__device__ __forceinline__ void irls_terms_sparse(const double pc[3], const double qc[3], double par,
                                                  double acc[27]) {
    const double x = qc[0], y = qc[1], z = qc[2];
    const double r0 = pc[0] - x, r1 = pc[1] - y, r2 = pc[2] - z;
    const double temp = par / (r0 * r0 + r1 * r1 + r2 * r2 + par);
    const double s = temp * temp;
    const double my = -y, mz = -z, mx = -x;
    acc[0] += (z * z) * s;  // (0,0): a = 1, 2
    acc[0] += (my * my) * s;
    acc[1] += (my * x) * s;   // (0,1): a = 2
    acc[2] += (z * mx) * s;   // (0,2): a = 1
    acc[4] += (z * -1.0) * s;   // (0,4): a = 1
    acc[5] += (my * -1.0) * s;  // (0,5): a = 2
    acc[6] += (mz * mz) * s;  // (1,1): a = 0, 2
    acc[6] += (x * x) * s;
    acc[7] += (mz * y) * s;     // (1,2): a = 0
    acc[8] += (mz * -1.0) * s;  // (1,3): a = 0
    acc[10] += (x * -1.0) * s;  // (1,5): a = 2
    acc[11] += (y * y) * s;  // (2,2): a = 0, 1
    acc[11] += (mx * mx) * s;
    acc[12] += (y * -1.0) * s;   // (2,3): a = 0
    acc[13] += (mx * -1.0) * s;  // (2,4): a = 1
    acc[15] += s;  // (3,3): a = 0, (-1)(-1)
    acc[18] += s;  // (4,4): a = 1
    acc[20] += s;  // (5,5): a = 2
    acc[21] += (z * r1) * s;  // JTr: u = 0 (a = 1, 2)
    acc[21] += (my * r2) * s;
    acc[22] += (mz * r0) * s;  // u = 1 (a = 0, 2)
    acc[22] += (x * r2) * s;
    acc[23] += (y * r0) * s;  // u = 2 (a = 0, 1)
    acc[23] += (mx * r1) * s;
    acc[24] += (-1.0 * r0) * s;  // u = 3..5
    acc[25] += (-1.0 * r1) * s;
    acc[26] += (-1.0 * r2) * s;
}

// One correspondence's terms, the generic form (the memory-resident kernel).
__device__ __forceinline__ void irls_terms(const double pc[3], const double qc[3], double par, double acc[27]) {
    const double qx = qc[0], qy = qc[1], qz = qc[2];
    const double r[3] = {pc[0] - qx, pc[1] - qy, pc[2] - qz};
    const double temp = par / (r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + par);
    const double s = temp * temp;
    const double J[3][6] = {{0, -qz, qy, -1, 0, 0}, {qz, 0, -qx, 0, -1, 0}, {-qy, qx, 0, 0, 0, -1}};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        int e = 0;
#pragma unroll
        for (int u = 0; u < 6; ++u) {
#pragma unroll
            for (int v = u; v < 6; ++v) acc[e++] += J[a][u] * J[a][v] * s;
            acc[21 + u] += J[a][u] * r[a] * s;
        }
    }
}

// The register-resident form (K <= kIrlsThreads * kIrlsPer, the default
// maximum_tuple_count of 1000 gives K = 3000): 8 waves, each thread holding
// its correspondences (c = thread + 512 k) in registers for all iterations;
// per iteration the 16 distinct of the 27 sums reduced (DPP wave sums, then a
// fixed-order sum over the waves), and the 6x6 solve on wave 0 (det6_wave /
// ldlt_solve6 / vec6_to_m4_wave, bit-identical to the single-lane routines).
// The 256-thread form below re-reads q from memory and solves on one lane:
// 18 us per iteration at C3 against 8 here (-DORPCD_IRLS_TIME: accumulate
// 0.8, wave sums 1.3, cross-wave sums 1.3, solve 4.5, update 0.2 us).
constexpr int kIrlsThreads = 512, kIrlsPer = 6;

#ifndef ORPCD_IRLS_DPP
#define ORPCD_IRLS_DPP 1
#endif
// A double moved across lanes by one DPP pattern (both halves).
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, kCtrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), kCtrl, 0xF, 0xF, false);
    return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}
// Wave sum for lane 0 on the VALU's DPP paths: quad swaps (xor 1, xor 2),
// then the half-row and row mirrors (the other quad, the other half of the
// row: every row of 16 ends uniform), then the four row sums by readlane —
// instead of six ds_bpermute round trips per value (5.2 us of every IRLS
// iteration for 27 sums).  A different tree than wave_sum's xor butterfly.
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v += dpp_f64<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v += dpp_f64<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v += dpp_f64<0x141>(v);  // row_half_mirror
    v += dpp_f64<0x140>(v);  // row_mirror
    return (rl64(v, 0) + rl64(v, 16)) + (rl64(v, 32) + rl64(v, 48));
}
// meta (batched FGR, orpcd_fgr_optimize_batch): block b solves the problem
// meta[3b..3b+2] = {offset of its p rows (doubles), K, output slot}: p at
// p + offset, q right after it (3K doubles), T at T_out + 16 slot.  Each block
// runs the single problem's arithmetic unchanged, so a batched start's T is
// bit-identical to its own launch.
__device__ __forceinline__ void irls_problem(const int64_t* meta, const double*& p, double*& q, int& K,
                                             double*& T_out) {
    if (!meta) return;
    const int64_t* m = meta + 4 * blockIdx.x;
    K = (int)m[1];
    q = const_cast<double*>(p) + m[3];
    p = p + m[0];
    T_out = T_out + 16 * m[2];
}

__global__ __launch_bounds__(kIrlsThreads) void fgr_irls_reg_kernel(const double* __restrict__ p_,
                                                                    double* __restrict__ q_, int K_, double par0,
                                                                    int iters, double division_factor,
                                                                    double max_corr, int decrease_mu,
                                                                    double* __restrict__ T_out_,
                                                                    const int64_t* __restrict__ meta) {
    const double* p = p_;
    double* q = q_;
    int K = K_;
    double* T_out = T_out_;
    irls_problem(meta, p, q, K, T_out);
    constexpr int kW = kIrlsThreads / 64;
    // Of the 27 sums only 16 are distinct (irls_terms_sparse): (0,3), (1,4),
    // (2,5), (3,4), (3,5), (4,5) are never added to, (3,3) = (4,4) = (5,5),
    // and (1,3) = -(0,4), (2,3) = -(0,5), (2,4) = -(1,5) term by term, so
    // bit for bit.  Only those 16 are reduced.
    constexpr int kNd = 16;
    constexpr int kDist[kNd] = {0, 1, 2, 4, 5, 6, 7, 10, 11, 15, 21, 22, 23, 24, 25, 26};
    __shared__ double red[kW][kNd];
    __shared__ double sums[kNd];
    __shared__ double delta[16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double trans[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) trans[t] = (t % 5 == 0) ? 1.0 : 0.0;
    if (K < 10) {  // O3D: fewer than 10 correspondences -> identity
        if (threadIdx.x < 16) T_out[threadIdx.x] = trans[threadIdx.x];
        return;
    }
    double pl[kIrlsPer][3], ql[kIrlsPer][3];
#pragma unroll
    for (int k = 0; k < kIrlsPer; ++k) {
        const int c = threadIdx.x + kIrlsThreads * k;
        const int cc = c < K ? c : 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            pl[k][a] = p[3 * cc + a];
            ql[k][a] = q[3 * cc + a];
        }
    }
    double par = par0;
#ifdef ORPCD_IRLS_TIME  // phase times of wave 0 (s_memrealtime, 10 ns ticks), printed at the end
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tq = __builtin_amdgcn_s_memrealtime(), tc0 = __builtin_amdgcn_s_memtime();
#define IRLS_T(k)                                                  \
    do {                                                           \
        const unsigned long long tn_ = __builtin_amdgcn_s_memrealtime(); \
        ph[k] += tn_ - tq;                                         \
        tq = tn_;                                                  \
    } while (0)
#else
#define IRLS_T(k) (void)0
#endif
    for (int itr = 0; itr < iters; ++itr) {
        double acc[27];
#pragma unroll
        for (int v = 0; v < 27; ++v) acc[v] = 0.0;
#pragma unroll
        for (int k = 0; k < kIrlsPer; ++k)
            if ((int)threadIdx.x + kIrlsThreads * k < K) irls_terms_sparse(pl[k], ql[k], par, acc);
        IRLS_T(0);
#pragma unroll
        for (int v = 0; v < kNd; ++v) {
            const double sv = ORPCD_IRLS_DPP ? wave_sum_dpp(acc[kDist[v]]) : wave_sum(acc[kDist[v]]);
            if (lane == 0) red[wid][v] = sv;
        }
        IRLS_T(1);
        __syncthreads();
        if (threadIdx.x < kNd) {
            double t = red[0][threadIdx.x];
            for (int w = 1; w < kW; ++w) t += red[w][threadIdx.x];
            sums[threadIdx.x] = t;
        }
        __syncthreads();
        IRLS_T(2);
        if (wid == 0) {
            double s[27];
#pragma unroll
            for (int v = 0; v < 27; ++v) s[v] = 0.0;  // (0,3), (1,4), (2,5), (3,4), (3,5), (4,5)
#pragma unroll
            for (int v = 0; v < kNd; ++v) s[kDist[v]] = sums[v];
            s[18] = s[20] = s[15];
            s[8] = -s[4];
            s[12] = -s[5];
            s[13] = -s[10];
            double neg[21], row[6], A[36], bvec[6], x[6] = {0, 0, 0, 0, 0, 0}, dl[16];
#pragma unroll
            for (int v = 0; v < 21; ++v) neg[v] = -s[v];
            sym6_row(neg, lane, row);  // SolveLinearSystemPSD(-JTJ, JTr): check_det
            for (int u = 0, e = 0; u < 6; ++u)
                for (int v = u; v < 6; ++v, ++e) A[6 * u + v] = A[6 * v + u] = neg[e];
#pragma unroll
            for (int u = 0; u < 6; ++u) bvec[u] = s[21 + u];
            const double det = det6_wave(row, lane);
            if (!(fabs(det) < 1e-6 || isnan(det) || isinf(det))) ldlt_solve6(A, bvec, x);
            vec6_to_m4_wave(x, dl, lane);
            double tn[16];
            m4_mul(dl, trans, tn);
#pragma unroll
            for (int t = 0; t < 16; ++t) trans[t] = tn[t];
#pragma unroll
            for (int t = 0; t < 16; ++t)
                if (lane == t) delta[t] = dl[t];
        }
        IRLS_T(3);
        __syncthreads();
        IRLS_T(4);
        double dm[12];
#pragma unroll
        for (int t = 0; t < 12; ++t) dm[t] = delta[t];
#pragma unroll
        for (int k = 0; k < kIrlsPer; ++k) {
            const double x = ql[k][0], y = ql[k][1], z = ql[k][2];
            ql[k][0] = dm[0] * x + dm[1] * y + dm[2] * z + dm[3];
            ql[k][1] = dm[4] * x + dm[5] * y + dm[6] * z + dm[7];
            ql[k][2] = dm[8] * x + dm[9] * y + dm[10] * z + dm[11];
        }
        if (decrease_mu && itr % 4 == 0 && par > max_corr) par /= division_factor;
        // delta is rewritten only after the next iteration's first barrier
        IRLS_T(5);
    }
#ifdef ORPCD_IRLS_TIME
    if (threadIdx.x == 0)
        printf("[irls] %d iters, K %d: accumulate %.2f, wave sums %.2f, block sums %.2f, solve %.2f, barrier %.2f, "
               "update %.2f us total; shader cycles %llu\n", iters, K, ph[0] * 0.01, ph[1] * 0.01, ph[2] * 0.01,
               ph[3] * 0.01, ph[4] * 0.01, ph[5] * 0.01, __builtin_amdgcn_s_memtime() - tc0);
#endif
#undef IRLS_T
#pragma unroll
    for (int k = 0; k < kIrlsPer; ++k) {
        const int c = threadIdx.x + kIrlsThreads * k;
        if (c < K)
#pragma unroll
            for (int a = 0; a < 3; ++a) q[3 * c + a] = ql[k][a];
    }
    if (wid == 0 && lane < 16) {
#pragma unroll
        for (int t = 0; t < 16; ++t)
            if (lane == t) T_out[t] = trans[t];
    }
}

__global__ __launch_bounds__(256) void fgr_irls_kernel(const double* __restrict__ p_, double* __restrict__ q_, int K_,
                                                       double par0, int iters, double division_factor,
                                                       double max_corr, int decrease_mu, double* __restrict__ T_out_,
                                                       const int64_t* __restrict__ meta) {
    const double* p = p_;
    double* q = q_;
    int K = K_;
    double* T_out = T_out_;
    irls_problem(meta, p, q, K, T_out);
    __shared__ double red[4][27];
    __shared__ double delta[16];
    __shared__ double trans[16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x < 16) trans[threadIdx.x] = (threadIdx.x % 5 == 0) ? 1.0 : 0.0;
    double par = par0;
    __syncthreads();
    if (K < 10) {  // O3D: fewer than 10 correspondences -> identity
        if (threadIdx.x < 16) T_out[threadIdx.x] = trans[threadIdx.x];
        return;
    }
    for (int itr = 0; itr < iters; ++itr) {
        double acc[27];
#pragma unroll
        for (int v = 0; v < 27; ++v) acc[v] = 0.0;
        for (int c = threadIdx.x; c < K; c += 256) {
            const double pc[3] = {p[3 * c], p[3 * c + 1], p[3 * c + 2]};
            const double qc[3] = {q[3 * c], q[3 * c + 1], q[3 * c + 2]};
            irls_terms(pc, qc, par, acc);
        }
#pragma unroll
        for (int v = 0; v < 27; ++v) {
            const double sv = wave_sum(acc[v]);
            if (lane == 0) red[wid][v] = sv;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double s[27];
            for (int v = 0; v < 27; ++v) s[v] = ((red[0][v] + red[1][v]) + red[2][v]) + red[3][v];
            double A[36], bvec[6], x[6] = {0, 0, 0, 0, 0, 0};
            int e = 0;
            for (int u = 0; u < 6; ++u)
                for (int v = u; v < 6; ++v) {
                    A[6 * u + v] = -s[e];
                    A[6 * v + u] = -s[e];
                    ++e;
                }
            for (int u = 0; u < 6; ++u) bvec[u] = s[21 + u];
            const double det = det6(A);  // SolveLinearSystemPSD(-JTJ, JTr): check_det
            if (!(fabs(det) < 1e-6 || isnan(det) || isinf(det))) ldlt_solve6(A, bvec, x);
            vec6_to_m4(x, delta);
            double tn[16];
            m4_mul(delta, trans, tn);
            for (int t = 0; t < 16; ++t) trans[t] = tn[t];
        }
        __syncthreads();
        for (int c = threadIdx.x; c < K; c += 256) {
            const double x = q[3 * c], y = q[3 * c + 1], z = q[3 * c + 2];
            q[3 * c] = delta[0] * x + delta[1] * y + delta[2] * z + delta[3];
            q[3 * c + 1] = delta[4] * x + delta[5] * y + delta[6] * z + delta[7];
            q[3 * c + 2] = delta[8] * x + delta[9] * y + delta[10] * z + delta[11];
        }
        if (decrease_mu && itr % 4 == 0 && par > max_corr) par /= division_factor;
        __syncthreads();
    }
    if (threadIdx.x < 16) T_out[threadIdx.x] = trans[threadIdx.x];
}

// ---------------------------------------------------------- small helpers
// Each takes blockIdx.y as the cloud of a batch (orpcd_fgr_optimize_batch:
// cloud y at the given strides; a single cloud launches one row, strides 0):
// every cloud's blocks do the single-cloud arithmetic unchanged.
// Per-block fixed-order partial sums of x, y, z (normalisation means).
__global__ __launch_bounds__(256) void sum3_kernel(const double* __restrict__ xyz, int n, double* __restrict__ part,
                                                   int64_t xyz_stride, int64_t part_stride) {
    xyz += blockIdx.y * xyz_stride;
    part += blockIdx.y * part_stride;
    __shared__ double red[4][3];
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double v[3] = {0.0, 0.0, 0.0};
    if (i < n) {
        v[0] = xyz[3 * i];
        v[1] = xyz[3 * i + 1];
        v[2] = xyz[3 * i + 2];
    }
    for (int a = 0; a < 3; ++a) {
        const double s = wave_sum(v[a]);
        if (lane == 0) red[wid][a] = s;
    }
    __syncthreads();
    if (threadIdx.x < 3)
        part[3 * blockIdx.x + threadIdx.x] =
            ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// Per-block max of |p - mean|.
__global__ __launch_bounds__(256) void maxnorm_kernel(const double* __restrict__ xyz, int n, double mx, double my,
                                                      double mz, double* __restrict__ part,
                                                      const double* __restrict__ means, int64_t xyz_stride,
                                                      int64_t part_stride) {
    if (means) {  // batch: cloud y's mean
        mx = means[3 * blockIdx.y];
        my = means[3 * blockIdx.y + 1];
        mz = means[3 * blockIdx.y + 2];
    }
    xyz += blockIdx.y * xyz_stride;
    part += blockIdx.y * part_stride;
    __shared__ double red[4];
    const int i = blockIdx.x * 256 + threadIdx.x;
    double v = 0.0;
    if (i < n) {
        const double x = xyz[3 * i] - mx, y = xyz[3 * i + 1] - my, z = xyz[3 * i + 2] - mz;
        v = sqrt(x * x + y * y + z * z);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// q = T p (homogeneous, fp64) for EvaluateRegistration.
__global__ void transform_points_kernel(const double* __restrict__ in, int n, const double* __restrict__ T,
                                        double* __restrict__ out, int64_t stride) {
    in += blockIdx.y * stride;
    out += blockIdx.y * stride;
    T += 16 * blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = in[3 * i], y = in[3 * i + 1], z = in[3 * i + 2];
    out[3 * i] = T[0] * x + T[1] * y + T[2] * z + T[3];
    out[3 * i + 1] = T[4] * x + T[5] * y + T[6] * z + T[7];
    out[3 * i + 2] = T[8] * x + T[9] * y + T[10] * z + T[11];
}

// Per-block (count, sum d^2) of nn1 results (EvaluateRegistration).
__global__ __launch_bounds__(256) void corr_stats_kernel(const int32_t* __restrict__ idx,
                                                         const double* __restrict__ d2, int n,
                                                         double* __restrict__ part, int64_t stride,
                                                         int64_t part_stride) {
    idx += blockIdx.y * stride;
    d2 += blockIdx.y * stride;
    part += blockIdx.y * part_stride;
    __shared__ double red[4][2];
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double c = 0.0, s = 0.0;
    if (i < n && idx[i] >= 0) {
        c = 1.0;
        s = d2[i];
    }
    c = wave_sum(c);
    s = wave_sum(s);
    if (lane == 0) {
        red[wid][0] = c;
        red[wid][1] = s;
    }
    __syncthreads();
    if (threadIdx.x < 2)
        part[2 * blockIdx.x + threadIdx.x] =
            ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// ---------------------------------------------------------------- launchers
hipError_t launch_fpfh(const double* pts, const double* nrm, int64_t n, const int32_t* nbr, const double* d2,
                       const int32_t* cnt, int k, double* spfh, double* feat36, hipStream_t s, int clouds) {
    if (n <= 0) return hipSuccess;
    spfh_kernel<<<dim3((unsigned)((n + 63) / 64), (unsigned)clouds), 64, 0, s>>>(pts, nrm, (int)n, nbr, cnt, k, spfh);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    fpfh_kernel<<<dim3((unsigned)((n + 255) / 256), (unsigned)clouds), 256, 0, s>>>(spfh, (int)n, nbr, d2, cnt, k,
                                                                                   feat36);
    return hipGetLastError();
}

hipError_t launch_pad_features(const double* in33, int64_t n, double* out36, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    pad_features_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(in33, (int)n, out36);
    return hipGetLastError();
}

hipError_t launch_feat_norm(const double* F36, int64_t n, double* nrm2, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    feat_norm_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(F36, (int)n, nrm2);
    return hipGetLastError();
}

// Target parts for a launch of `blocks` query blocks per part, in [1, maxp]
// (at least 64 targets a part).  Every block of a launch runs the same number
// of 64-target stages, so the launch takes ceil(parts * blocks / slots)
// rounds of the device's resident block slots (2 four-wave blocks per CU at
// the kernels' ~250 VGPRs), each of ceil(nt / parts / 64) stages plus about
// two stages' worth of query loads and merges: the count minimising that
// product wins (100k queries x 67k targets: 9 parts, 7 full rounds, where a
// fixed 5 parts left the 4th of 4 rounds 18% idle).
int feat_nn_parts(int64_t blocks, int64_t nt, int maxp) {
    static const int slots = [] {  // thread-safe once-only initialisation
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return 2 * cus;
    }();
    const int64_t pmax = std::max<int64_t>(1, std::min<int64_t>(maxp, (nt + kFT - 1) / kFT));
    int best = 1;
    int64_t best_cost = INT64_MAX;
    for (int64_t p = 1; p <= pmax; ++p) {
        const int64_t rounds = (p * blocks + slots - 1) / slots;
        const int64_t stages = ((nt + p - 1) / p + kFT - 1) / kFT + 2;
        if (rounds * stages < best_cost) {
            best_cost = rounds * stages;
            best = (int)p;
        }
    }
    return best;
}

hipError_t launch_feat_nn(const double* Fq, const double* nq2, int64_t nq, const double* Ft, const double* nt2,
                          int64_t nt, const int32_t* tmap, int dim, FeatNNBufs& b, int32_t* out, hipStream_t s,
                          double* timing) {
    if (nq <= 0) return hipSuccess;
    hipError_t e;
    // timing (profiling): events around each pass; timing[0..4] += pass-1 ms,
    // pass-2 ms, pass-1 pairs, pass-2 pairs, calls
    if (timing)
        for (auto& ev : b.ev)
            if (!ev && (e = hipEventCreateWithFlags(&ev, hipEventDisableSystemFence)) != hipSuccess) return e;
    if (timing && (e = hipEventRecord(b.ev[0], s)) != hipSuccess) return e;
    const unsigned gq = (unsigned)((nq + 255) / 256);
    const int parts = feat_nn_parts(gq, nt, kMaxParts);
    if ((e = b.part_d.ensure((size_t)2 * kMaxParts * nq)) != hipSuccess) return e;
    if ((e = b.part_i.ensure((size_t)kMaxParts * nq)) != hipSuccess) return e;
    if ((e = b.flag.ensure((size_t)nq)) != hipSuccess) return e;
    if ((e = b.qidx.ensure((size_t)nq + 1)) != hipSuccess) return e;
    if ((e = b.thr.ensure((size_t)nq)) != hipSuccess) return e;
    if ((e = b.need.ensure((size_t)nq)) != hipSuccess) return e;
    if ((e = b.nkey.ensure((size_t)2 * nq)) != hipSuccess) return e;
    if ((e = b.qsort.ensure((size_t)nq)) != hipSuccess) return e;
    double* part_s = b.part_d.p + (size_t)kMaxParts * nq;
    int32_t* nsel = b.qidx.p + nq;
    const int len1 = (int)(((nt + parts - 1) / parts + kFT - 1) / kFT * kFT);
    auto pass1 = dim <= 33 ? feat_nn_kernel<false, 8> : feat_nn_kernel<false, 9>;
    pass1<<<dim3(gq, (unsigned)parts), 256, 0, s>>>(Fq, nq2, (int)nq, nullptr, nullptr, nullptr, Ft, nt2, (int)nt, len1,
                                                    dim, b.part_d.p, part_s, b.part_i.p, nullptr, len1);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (timing && (e = hipEventRecord(b.ev[1], s)) != hipSuccess) return e;
    merge_parts_kernel<<<gq, 256, 0, s>>>(b.part_d.p, part_s, b.part_i.p, (int)nq, parts, nq2, nt2, tmap, out,
                                          b.flag.p, b.thr.p, ldexp(1.0, feat_key_bits(len1) - 51), b.need.p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tmp = 0;
    if ((e = hipcub::DeviceSelect::Flagged(nullptr, tmp, hipcub::CountingInputIterator<int32_t>(0), b.flag.p,
                                           b.qidx.p, nsel, (int)nq, s)) != hipSuccess)
        return e;
    if ((e = b.tmp.ensure(tmp)) != hipSuccess) return e;
    if ((e = hipcub::DeviceSelect::Flagged(b.tmp.p, tmp, hipcub::CountingInputIterator<int32_t>(0), b.flag.p,
                                           b.qidx.p, nsel, (int)nq, s)) != hipSuccess)
        return e;
    // the flagged count sizes pass 2's grid and its parts (one 4-byte read;
    // the stream drains here anyway before the caller reads the answers)
    int32_t nflag = 0;
    if ((e = d2h(&nflag, nsel, 4, s)) != hipSuccess) return e;
    // Pass 2 runs over kMaxParts sub-parts, its flagged queries ordered by
    // their need masks (the pass-1 parts that can hold a candidate; most
    // near-tie clusters sit in one or two), and a block skips every sub-part
    // none of its rows needs.
    const unsigned g2 = (unsigned)((nflag + 255) / 256);
    const int parts2 = nflag > 0 ? (int)std::max<int64_t>(1, std::min<int64_t>(kMaxParts, (nt + kFT - 1) / kFT)) : 0;
    if (getenv("ORPCD_TRACE"))
        fprintf(stderr, "[orpcd] feat_nn: %lld queries, %lld targets, %d parts, %d flagged for the exact pass (%d parts)\n",
                (long long)nq, (long long)nt, parts, nflag, parts2);
    float ms1 = 0.f, ms2 = 0.f;
    if (timing && (e = hipEventElapsedTime(&ms1, b.ev[0], b.ev[1])) != hipSuccess) return e;  // drained by d2h
    if (timing) {
        timing[0] += ms1;
        timing[2] += (double)nq * (double)nt;
        timing[4] += 1;
    }
    if (nflag == 0) return hipSuccess;
    if (timing && (e = hipEventRecord(b.ev[2], s)) != hipSuccess) return e;
    gather_need_kernel<<<g2, 256, 0, s>>>(b.qidx.p, nsel, b.need.p, b.nkey.p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tmp2 = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp2, b.nkey.p, b.nkey.p + nq, b.qidx.p, b.qsort.p, nflag, 0,
                                                parts, s)) != hipSuccess)
        return e;
    if ((e = b.tmp.ensure(tmp2)) != hipSuccess) return e;
    if ((e = hipcub::DeviceRadixSort::SortPairs(b.tmp.p, tmp2, b.nkey.p, b.nkey.p + nq, b.qidx.p, b.qsort.p, nflag, 0,
                                                parts, s)) != hipSuccess)
        return e;
    const int len2 = (int)(((nt + parts2 - 1) / parts2 + kFT - 1) / kFT * kFT);
    auto pass2 = dim <= 33 ? feat_nn_kernel<true, 8> : feat_nn_kernel<true, 9>;
    pass2<<<dim3(g2, (unsigned)parts2), 256, 0, s>>>(Fq, nq2, (int)nq, b.qsort.p, nsel, b.thr.p, Ft, nt2, (int)nt, len2,
                                                     dim, b.part_d.p, nullptr, b.part_i.p, b.nkey.p + nq, len1);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (timing) {
        if ((e = hipEventRecord(b.ev[3], s)) != hipSuccess) return e;
        if ((e = hipEventSynchronize(b.ev[3])) != hipSuccess) return e;
        if ((e = hipEventElapsedTime(&ms2, b.ev[2], b.ev[3])) != hipSuccess) return e;
        timing[1] += ms2;
        // the pairs pass 2 evaluates: a block's real rows x its sub-part's
        // targets, for the (block, sub-part) tiles the need masks do not skip
        // (the kernel's own skip rule, over the sorted masks)
        std::vector<uint32_t> nk((size_t)nflag);
        if ((e = d2h(nk.data(), b.nkey.p + nq, (size_t)nflag * 4, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        double pairs2 = 0.0;
        for (int y = 0; y < parts2; ++y) {
            const int t_begin = y * len2, t_end = (int)std::min<int64_t>(nt, (int64_t)t_begin + len2);
            if (t_begin >= t_end) continue;
            const int p_lo = t_begin / len1, p_hi = (t_end - 1) / len1;
            const uint32_t range = (p_hi >= 31 ? 0xFFFFFFFFu : ((1u << (p_hi + 1)) - 1u)) & ~((1u << p_lo) - 1u);
            for (int r0 = 0; r0 < nflag; r0 += 256) {
                const int r1 = std::min(nflag, r0 + 256);
                bool run = false;
                for (int j = r0; j < r1 && !run; ++j) run = (nk[(size_t)j] & range) != 0;
                if (run) pairs2 += (double)(r1 - r0) * (double)(t_end - t_begin);
            }
        }
        timing[3] += pairs2;
    }
    merge_exact_kernel<<<g2, 256, 0, s>>>(b.part_d.p, b.part_i.p, (int)nq, parts2, b.qsort.p, nsel, tmap, out);
    return hipGetLastError();
}

// Answers of duplicate rows from their representatives' (dedup_rows' runs:
// sorted position p holds row vs[p]; a row that is not its own
// representative (uflag 0) equals the row at its run head): identical query
// rows have identical answers, so a search runs over the distinct rows only.
__global__ void unique_pos_kernel(const int32_t* __restrict__ uidx, int nu, int32_t* __restrict__ pos) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nu) pos[uidx[k]] = k;
}

__global__ void expand_dup_kernel(const int32_t* __restrict__ vs, const int32_t* __restrict__ head,
                                  const unsigned char* __restrict__ uflag, int n, const int32_t* __restrict__ pos,
                                  const int32_t* __restrict__ out_u, int32_t* __restrict__ out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int i = vs[p];
    const int r = uflag[i] ? i : vs[head[p]];
    out[i] = out_u[pos[r]];
}

hipError_t expand_dup_answers(const DedupBufs& b, int64_t n, int64_t nu, const int32_t* out_u, int32_t* pos,
                              int32_t* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    unique_pos_kernel<<<(unsigned)((nu + 255) / 256), 256, 0, s>>>(b.uidx.p, (int)nu, pos);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    expand_dup_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(b.val.p + n, b.head.p, b.uflag.p, (int)n, pos,
                                                                  out_u, out);
    return hipGetLastError();
}

// AdvancedMatching's cross check keeps (i, i_to_j[i]) only when
// j_to_i[i_to_j[i]] == i, so the second direction's search matters only for
// the rows i that some j chose: they are compacted here (needed_rows) and
// their answers scattered back (scatter_answers); every other i keeps -1,
// which the cross check rejects as it rejects a non-mutual match.
__global__ void need_flags_kernel(const int32_t* __restrict__ j_to_i, int nj, int ni, unsigned char* __restrict__ flag) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nj) return;
    const int i = j_to_i[j];
    if (i >= 0 && i < ni) flag[i] = 1;  // racing writers store the same byte
}

__global__ void scatter_answers_kernel(const int32_t* __restrict__ idx, int n, const int32_t* __restrict__ ans,
                                       int32_t* __restrict__ out) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) out[idx[k]] = ans[k];
}

hipError_t needed_rows(const int32_t* j_to_i, int64_t nj, const double* F, const double* n2, int64_t ni,
                       NeedBufs& b, int64_t* nq_out, hipStream_t s) {
    hipError_t e;
    *nq_out = 0;
    if (ni <= 0) return hipSuccess;
    if ((e = b.flag.ensure((size_t)ni)) != hipSuccess) return e;
    if ((e = b.idx.ensure((size_t)ni + 1)) != hipSuccess) return e;
    if ((e = b.out.ensure((size_t)ni)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(b.flag.p, 0, (size_t)ni, s)) != hipSuccess) return e;
    if (nj > 0) {
        need_flags_kernel<<<(unsigned)((nj + 255) / 256), 256, 0, s>>>(j_to_i, (int)nj, (int)ni, b.flag.p);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    int32_t* nsel = b.idx.p + ni;
    size_t tmp = 0;
    if ((e = hipcub::DeviceSelect::Flagged(nullptr, tmp, hipcub::CountingInputIterator<int32_t>(0), b.flag.p, b.idx.p,
                                           nsel, (int)ni, s)) != hipSuccess)
        return e;
    if ((e = b.tmp.ensure(tmp)) != hipSuccess) return e;
    if ((e = hipcub::DeviceSelect::Flagged(b.tmp.p, tmp, hipcub::CountingInputIterator<int32_t>(0), b.flag.p, b.idx.p,
                                           nsel, (int)ni, s)) != hipSuccess)
        return e;
    int32_t nq = 0;
    if ((e = d2h(&nq, nsel, 4, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if (nq > 0) {
        if ((e = b.F.ensure((size_t)nq * kFD)) != hipSuccess) return e;
        if ((e = b.n2.ensure((size_t)nq)) != hipSuccess) return e;
        gather_rows_kernel<<<(unsigned)(((int64_t)nq * kFD + 255) / 256), 256, 0, s>>>(F, n2, b.idx.p, nq, b.F.p,
                                                                                       b.n2.p);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    *nq_out = nq;
    return hipSuccess;
}

hipError_t scatter_answers(const int32_t* idx, int64_t n, const int32_t* ans, int32_t* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    scatter_answers_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(idx, (int)n, ans, out);
    return hipGetLastError();
}

hipError_t dedup_rows(const double* F, const double* n2, int64_t n, DedupBufs& b, int64_t* nu_out, hipStream_t s) {
    hipError_t e;
    if ((e = b.key.ensure((size_t)n * 2)) != hipSuccess) return e;
    if ((e = b.val.ensure((size_t)n * 2)) != hipSuccess) return e;
    if ((e = b.head.ensure((size_t)n + 1)) != hipSuccess) return e;
    if ((e = b.uflag.ensure((size_t)n)) != hipSuccess) return e;
    if ((e = b.uidx.ensure((size_t)n)) != hipSuccess) return e;
    if ((e = b.Fu.ensure((size_t)n * kFD)) != hipSuccess) return e;
    if ((e = b.n2u.ensure((size_t)n)) != hipSuccess) return e;
    const unsigned g = (unsigned)((n + 255) / 256);
    unsigned long long *k0 = b.key.p, *k1 = b.key.p + n;
    int32_t *v0 = b.val.p, *v1 = b.val.p + n, *nsel = b.head.p + n;
    row_hash_kernel<<<g, 256, 0, s>>>(F, (int)n, k0, v0);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t t1 = 0, t2 = 0, t3 = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, t1, k0, k1, v0, v1, (int)n, 0, 64, s)) != hipSuccess) return e;
    if ((e = hipcub::DeviceScan::InclusiveScan(nullptr, t2, v0, v0, hipcub::Max(), (int)n, s)) != hipSuccess) return e;
    if ((e = hipcub::DeviceSelect::Flagged(nullptr, t3, hipcub::CountingInputIterator<int32_t>(0), b.uflag.p,
                                           b.uidx.p, nsel, (int)n, s)) != hipSuccess)
        return e;
    if ((e = b.tmp.ensure(std::max(t1, std::max(t2, t3)))) != hipSuccess) return e;
    if ((e = hipcub::DeviceRadixSort::SortPairs(b.tmp.p, t1, k0, k1, v0, v1, (int)n, 0, 64, s)) != hipSuccess) return e;
    run_start_kernel<<<g, 256, 0, s>>>(k1, (int)n, v0, (int)n);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipcub::DeviceScan::InclusiveScan(b.tmp.p, t2, v0, b.head.p, hipcub::Max(), (int)n, s)) != hipSuccess)
        return e;
    representative_kernel<<<g, 256, 0, s>>>(F, v1, b.head.p, (int)n, b.uflag.p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipcub::DeviceSelect::Flagged(b.tmp.p, t3, hipcub::CountingInputIterator<int32_t>(0), b.uflag.p,
                                           b.uidx.p, nsel, (int)n, s)) != hipSuccess)
        return e;
    int32_t nu = 0;
    if ((e = d2h(&nu, nsel, 4, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    gather_rows_kernel<<<(unsigned)(((int64_t)nu * kFD + 255) / 256), 256, 0, s>>>(F, n2, b.uidx.p, nu, b.Fu.p,
                                                                                   b.n2u.p);
    *nu_out = nu;
    return hipGetLastError();
}

// dedup_rows' representative flags only (no count, no gather, no host
// sync), for `clouds` row sets of n rows each (F and uflag_out back to back):
// uflag_out[i] = 1 iff row i is the lowest index of the exact-equal rows of
// its set.  Several sets sort segment by segment (stable, as the single
// sort); scratch in b (reused in stream order by the next call).
__global__ void segment_offsets_kernel(int32_t* __restrict__ off, int nseg, int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k <= nseg) off[k] = k * n;
}
hipError_t dedup_flags(const double* F, int64_t n, DedupBufs& b, unsigned char* uflag_out, hipStream_t s,
                       int clouds) {
    hipError_t e;
    if (n <= 0) return hipSuccess;
    const int64_t N = n * clouds;
    if ((e = b.key.ensure((size_t)N * 2)) != hipSuccess) return e;
    if ((e = b.val.ensure((size_t)N * 2)) != hipSuccess) return e;
    if ((e = b.head.ensure((size_t)N + clouds + 2)) != hipSuccess) return e;
    const unsigned g = (unsigned)((N + 255) / 256);
    unsigned long long *k0 = b.key.p, *k1 = b.key.p + N;
    int32_t *v0 = b.val.p, *v1 = b.val.p + N, *off = b.head.p + N;
    row_hash_kernel<<<g, 256, 0, s>>>(F, (int)N, k0, v0);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t t1 = 0, t2 = 0;
    if (clouds > 1) {
        segment_offsets_kernel<<<(unsigned)((clouds + 256) / 256), 256, 0, s>>>(off, clouds, (int)n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, t1, k0, k1, v0, v1, (int)N, clouds, off,
                                                             off + 1, 0, 64, s)) != hipSuccess)
            return e;
    } else if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, t1, k0, k1, v0, v1, (int)n, 0, 64, s)) != hipSuccess) {
        return e;
    }
    if ((e = hipcub::DeviceScan::InclusiveScan(nullptr, t2, v0, v0, hipcub::Max(), (int)N, s)) != hipSuccess) return e;
    if ((e = b.tmp.ensure(std::max(t1, t2))) != hipSuccess) return e;
    if (clouds > 1) {
        if ((e = hipcub::DeviceSegmentedRadixSort::SortPairs(b.tmp.p, t1, k0, k1, v0, v1, (int)N, clouds, off,
                                                             off + 1, 0, 64, s)) != hipSuccess)
            return e;
    } else if ((e = hipcub::DeviceRadixSort::SortPairs(b.tmp.p, t1, k0, k1, v0, v1, (int)n, 0, 64, s)) != hipSuccess) {
        return e;
    }
    n = N;
    run_start_kernel<<<g, 256, 0, s>>>(k1, (int)n, v0, (int)(N / clouds));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipcub::DeviceScan::InclusiveScan(b.tmp.p, t2, v0, b.head.p, hipcub::Max(), (int)n, s)) != hipSuccess)
        return e;
    representative_kernel<<<g, 256, 0, s>>>(F, v1, b.head.p, (int)n, uflag_out);
    return hipGetLastError();
}

// ------------------------------------------------------------- tuple test
// O3D FastGlobalRegistration.cpp AdvancedMatching (tuple part), as restated
// sequentially by fgr_tuples (runtime.hip) and oracle/orpcd_oracle.cpp: trial t
// draws r0, r1, r2 = dis(gen) x 3 (dis = uniform_int_distribution<int>(0,
// ncorr - 1) over std::mt19937(seed)); the trial is accepted when the three
// side lengths of the fi-side triangle li and of the fj-side triangle lj
// satisfy li * s < lj < li / s; the accepted trials' pairs, in trial order,
// are the tuples, and the loop ends after maximum_tuple_count acceptances.
//
// libstdc++'s uniform_int_distribution (32-bit engine, range n) takes a word
// x, forms x * n in 64 bits, and rejects the word when the low half is below
// (2^32 - n) mod n; otherwise the draw is the high half.  Draw d of a window
// therefore reads word d + #{rejected words before it}: with the window's
// rejected positions r_j sorted, key_j = r_j - word0 - j is non-decreasing and
// the word is word0 + d + #{j : key_j <= d}.
//
// Arithmetic: no contraction; IEEE division and square root on both sides
// (the device's f64 sqrt and division are correctly rounded), so each length
// and each comparison is the host's, bit for bit.
__device__ __forceinline__ int64_t tuple_word(const TupleJob& J, const int64_t* __restrict__ keys, int64_t d) {
    int lo = 0, hi = J.nrej;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[J.rej + mid] <= d)
            lo = mid + 1;
        else
            hi = mid;
    }
    return J.word0 + d + lo;
}

__device__ __forceinline__ int tuple_draw(const TupleJob& J, const uint32_t* __restrict__ words,
                                          const int64_t* __restrict__ keys, int64_t d) {
    const uint64_t x = (uint64_t)words[tuple_word(J, keys, d)] * (uint64_t)(uint32_t)J.ncorr;
    return (int)(x >> 32);
}

__device__ __forceinline__ double tuple_side(const double* a, const double* b) {
#pragma clang fp contract(off)
    const double d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2];
    return sqrt(d0 * d0 + d1 * d1 + d2 * d2);
}

__global__ __launch_bounds__(256) void tuple_points_kernel(const TupleJob* __restrict__ jobs,
                                                           const int32_t* __restrict__ pairs, double* __restrict__ A,
                                                           double* __restrict__ Bv) {
    const TupleJob& J = jobs[blockIdx.y];
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= J.ncorr) return;
    const int64_t g = J.corr + k;
    const int i = pairs[2 * g], j = pairs[2 * g + 1];
    for (int a = 0; a < 3; ++a) {
        A[3 * g + a] = (J.xi[3 * (int64_t)i + a] - J.mi[a]) / J.scale;
        Bv[3 * g + a] = (J.xj[3 * (int64_t)j + a] - J.mj[a]) / J.scale;
    }
}

__global__ __launch_bounds__(256) void tuple_reject_kernel(const TupleJob* __restrict__ jobs,
                                                           const uint32_t* __restrict__ words,
                                                           int64_t* __restrict__ rej, int32_t* __restrict__ nrej,
                                                           int64_t rcap) {
    const TupleJob& J = jobs[blockIdx.y];
    if (J.tw == 0 || J.threshold == 0) return;
    const int64_t span = 3 * J.tw + rcap;
    const uint32_t n = (uint32_t)J.ncorr;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < span; k += (int64_t)gridDim.x * 256) {
        const int64_t w = J.word0 + k;
        const uint32_t low = (uint32_t)((uint64_t)words[w] * (uint64_t)n);
        if (low < J.threshold) {
            const int slot = atomicAdd(&nrej[blockIdx.y], 1);
            if (slot < rcap) rej[(int64_t)blockIdx.y * rcap + slot] = w;
        }
    }
}

constexpr int kTupleChunk = 4096;  // trials per eval workgroup: 4 waves x 16 rounds x 64 lanes

__global__ __launch_bounds__(256) void tuple_eval_kernel(const TupleJob* __restrict__ jobs,
                                                         const uint32_t* __restrict__ words,
                                                         const int64_t* __restrict__ keys,
                                                         const double* __restrict__ A, const double* __restrict__ Bv,
                                                         double sc, uint64_t* __restrict__ mask,
                                                         int32_t* __restrict__ chunk_cnt) {
#pragma clang fp contract(off)
    const int b = blockIdx.y;
    const TupleJob& J = jobs[b];
    const int64_t base = (int64_t)blockIdx.x * kTupleChunk;
    if (base >= J.tw) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ int part[4];
    int acc_count = 0;
    for (int it = 0; it < 16; ++it) {
        const int64_t t0 = base + (int64_t)(wid * 16 + it) * 64;
        if (t0 >= J.tw) break;  // wave-uniform
        const int64_t t = t0 + lane;
        bool acc = false;
        if (t < J.tw) {
            int r[3];
            for (int e = 0; e < 3; ++e) r[e] = tuple_draw(J, words, keys, 3 * t + e);
            double pi[3][3], pj[3][3];
            for (int e = 0; e < 3; ++e)
                for (int a = 0; a < 3; ++a) {
                    pi[e][a] = A[3 * (J.corr + r[e]) + a];
                    pj[e][a] = Bv[3 * (J.corr + r[e]) + a];
                }
            acc = true;
            for (int e = 0; e < 3; ++e) {
                const int f = (e + 1) % 3;
                const double li = tuple_side(pi[e], pi[f]), lj = tuple_side(pj[e], pj[f]);
                acc = acc && (li * sc < lj) && (lj < li / sc);
            }
        }
        const uint64_t m = __ballot(acc);
        if (lane == 0) mask[(int64_t)b * (kTupleWindow / 64) + t0 / 64] = m;
        acc_count += __popcll(m);
    }
    if (lane == 0) part[wid] = acc_count;
    __syncthreads();
    if (threadIdx.x == 0)
        chunk_cnt[(int64_t)b * (kTupleWindow / kTupleChunk) + blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// one workgroup per start; the first wave walks the window's chunks in order,
// lane k taking the chunk's k-th mask word, and writes each accepted trial's
// three pairs at its rank among all of the start's tuples
__global__ __launch_bounds__(64) void tuple_select_kernel(const TupleJob* __restrict__ jobs,
                                                          const uint32_t* __restrict__ words,
                                                          const int64_t* __restrict__ keys,
                                                          const uint64_t* __restrict__ mask,
                                                          const int32_t* __restrict__ chunk_cnt,
                                                          const double* __restrict__ A,
                                                          const double* __restrict__ Bv, int maxc,
                                                          int32_t* __restrict__ cnt, double* __restrict__ rows) {
    const int b = blockIdx.x;
    const TupleJob& J = jobs[b];
    if (J.tw == 0) return;
    const int lane = threadIdx.x;
    int have = cnt[b];
    const int64_t nch = (J.tw + kTupleChunk - 1) / kTupleChunk;
    const double* src = J.fi == 0 ? A : Bv;  // source rows: cloud 0
    const double* tgt = J.fi == 0 ? Bv : A;
    for (int64_t ch = 0; ch < nch && have < maxc; ++ch) {
        const int cc = chunk_cnt[(int64_t)b * (kTupleWindow / kTupleChunk) + ch];
        if (cc == 0) continue;
        const int64_t t0 = ch * kTupleChunk + (int64_t)lane * 64;
        uint64_t m = t0 < J.tw ? mask[(int64_t)b * (kTupleWindow / 64) + t0 / 64] : 0ull;
        // exclusive prefix of the lanes' popcounts
        const int pc = __popcll(m);
        int incl = pc;
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_up(incl, off, 64);
            if (lane >= off) incl += v;
        }
        int rank = have + incl - pc;
        while (m && rank < maxc) {
            const int bit = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const int64_t t = t0 + bit;
            for (int e = 0; e < 3; ++e) {
                const int64_t g = J.corr + tuple_draw(J, words, keys, 3 * t + e);
                const int64_t row = 3 * (int64_t)rank + e;
                for (int a = 0; a < 3; ++a) {
                    rows[J.out + 3 * row + a] = src[3 * g + a];
                    rows[J.out + 3 * J.cap + 3 * row + a] = tgt[3 * g + a];
                }
            }
            ++rank;
        }
        have = min(maxc, have + cc);
    }
    if (lane == 0) cnt[b] = have;
}

hipError_t launch_tuple_points(const TupleJob* jobs, int B, int max_ncorr, const int32_t* pairs, double* A,
                               double* Bv, hipStream_t s) {
    if (B <= 0 || max_ncorr <= 0) return hipSuccess;
    tuple_points_kernel<<<dim3((unsigned)((max_ncorr + 255) / 256), (unsigned)B), 256, 0, s>>>(jobs, pairs, A, Bv);
    return hipGetLastError();
}

hipError_t launch_tuple_reject(const TupleJob* jobs, int B, int64_t max_span, const uint32_t* words, int64_t* rej,
                               int32_t* nrej, int64_t rcap, hipStream_t s) {
    if (B <= 0 || max_span <= 0) return hipSuccess;
    // 16 words per thread: a window's span (<= 6.3M words) in <= 1536 blocks per start
    const int64_t blocks = std::min<int64_t>((max_span + 4095) / 4096, 1536);
    tuple_reject_kernel<<<dim3((unsigned)blocks, (unsigned)B), 256, 0, s>>>(jobs, words, rej, nrej, rcap);
    return hipGetLastError();
}

hipError_t launch_tuple_eval(const TupleJob* jobs, int B, int64_t max_tw, const uint32_t* words, const int64_t* keys,
                             const double* A, const double* Bv, double tuple_scale, uint64_t* mask,
                             int32_t* chunk_cnt, hipStream_t s) {
    if (B <= 0 || max_tw <= 0) return hipSuccess;
    const unsigned nch = (unsigned)((max_tw + kTupleChunk - 1) / kTupleChunk);
    tuple_eval_kernel<<<dim3(nch, (unsigned)B), 256, 0, s>>>(jobs, words, keys, A, Bv, tuple_scale, mask, chunk_cnt);
    return hipGetLastError();
}

hipError_t launch_tuple_select(const TupleJob* jobs, int B, const uint32_t* words, const int64_t* keys,
                               const uint64_t* mask, const int32_t* chunk_cnt, const double* A, const double* Bv,
                               int maxc, int32_t* cnt, double* rows, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    tuple_select_kernel<<<(unsigned)B, 64, 0, s>>>(jobs, words, keys, mask, chunk_cnt, A, Bv, maxc, cnt, rows);
    return hipGetLastError();
}


hipError_t launch_fgr_irls(const double* p, double* q, int K, double par0, int iters, double division_factor,
                           double max_corr, int decrease_mu, double* T_out, hipStream_t s) {
    if (K <= kIrlsThreads * kIrlsPer)
        fgr_irls_reg_kernel<<<1, kIrlsThreads, 0, s>>>(p, q, K, par0, iters, division_factor, max_corr, decrease_mu,
                                                       T_out, nullptr);
    else
        fgr_irls_kernel<<<1, 256, 0, s>>>(p, q, K, par0, iters, division_factor, max_corr, decrease_mu, T_out,
                                          nullptr);
    return hipGetLastError();
}

hipError_t launch_fgr_irls_batch(const double* pq, const int64_t* meta_reg, int nreg, const int64_t* meta_mem,
                                 int nmem, double par0, int iters, double division_factor, double max_corr,
                                 int decrease_mu, double* T_out, hipStream_t s) {
    // problems of <= 3072 correspondences: one register-resident 512-thread
    // workgroup each, all of them in one launch (one CU per start); larger
    // ones: the memory-resident form, likewise
    if (nreg > 0)
        fgr_irls_reg_kernel<<<(unsigned)nreg, kIrlsThreads, 0, s>>>(pq, nullptr, 0, par0, iters, division_factor,
                                                                    max_corr, decrease_mu, T_out, meta_reg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || nmem <= 0) return e;
    fgr_irls_kernel<<<(unsigned)nmem, 256, 0, s>>>(pq, nullptr, 0, par0, iters, division_factor, max_corr,
                                                   decrease_mu, T_out, meta_mem);
    return hipGetLastError();
}

hipError_t launch_sum3(const double* xyz, int64_t n, double* part, hipStream_t s, int clouds) {
    // partials: cloud y's ceil(n / 256) x 3 at part + 3 ceil(n / 256) y
    const int64_t nb = (n + 255) / 256;
    sum3_kernel<<<dim3((unsigned)nb, (unsigned)clouds), 256, 0, s>>>(xyz, (int)n, part, 3 * n, 3 * nb);
    return hipGetLastError();
}

hipError_t launch_maxnorm(const double* xyz, int64_t n, const double mean[3], double* part, hipStream_t s,
                          int clouds, const double* dev_means) {
    const int64_t nb = (n + 255) / 256;
    maxnorm_kernel<<<dim3((unsigned)nb, (unsigned)clouds), 256, 0, s>>>(
        xyz, (int)n, mean ? mean[0] : 0.0, mean ? mean[1] : 0.0, mean ? mean[2] : 0.0, part, dev_means, 3 * n, nb);
    return hipGetLastError();
}

hipError_t launch_transform_points(const double* in, int64_t n, const double* T, double* out, hipStream_t s,
                                   int clouds) {
    if (n <= 0) return hipSuccess;
    transform_points_kernel<<<dim3((unsigned)((n + 255) / 256), (unsigned)clouds), 256, 0, s>>>(in, (int)n, T, out,
                                                                                              3 * n);
    return hipGetLastError();
}

hipError_t launch_corr_stats(const int32_t* idx, const double* d2, int64_t n, double* part, hipStream_t s,
                             int clouds) {
    const int64_t nb = (n + 255) / 256;
    corr_stats_kernel<<<dim3((unsigned)nb, (unsigned)clouds), 256, 0, s>>>(idx, d2, (int)n, part, n, 2 * nb);
    return hipGetLastError();
}

}  // namespace orpcd
