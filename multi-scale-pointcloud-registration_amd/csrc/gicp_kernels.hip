// gicp_kernels.hip — the GICP inner loop on gfx950, batched over starts.
//
// One correspondence pass restates, for every running start at once,
//   O3D Registration.cpp GetRegistrationResultAndCorrespondences
//     (SearchHybrid(max_corr, 1): exact nearest target with d^2 < r^2)
// fused with
//   O3D GeneralizedICP.cpp TransformationEstimationForGeneralizedICP::
//     ComputeTransformation (JTJ / JTr with W = (Cs + Ct)^-1/2, L2 kernel).
// The solve kernel restates SolveJacobianSystemAndObtainExtrinsicMatrix and
// the RegistrationICP convergence test, per start, on device.
// Reference call site: generalizedICP.py:59-70, driven by Aligner.py:178-202.
//
// Numerics: the nearest-target search runs in fp32 over an LDS-staged target
// tile (packed v_pk_* math, one LDS broadcast per target per wave); the chosen
// pair is then re-evaluated in fp64 (radius test, d^2, Jacobian), so every
// accumulated quantity is fp64.  Because W is symmetric, J^T J = A^T (Cs+Ct)^-1 A
// and J^T r = A^T (Cs+Ct)^-1 d with A = [-[q]x | I]: no matrix square root is
// needed.  All reductions run in a fixed order (bitwise
// reproducible run to run).
#include "device_math.h"
#include "orpcd_internal.h"

namespace orpcd {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// --------------------------------------------------------------------------
// fp32 brute-force nearest search for kQPT queries per lane over all targets.
// Targets are padded to a multiple of kTargetTile with far points so the inner
// loop has no bounds check.  bd is initialised to the (slightly enlarged)
// squared radius; ties resolve to the lowest target index.
// --------------------------------------------------------------------------
__device__ __forceinline__ void nn_search_tiles(float4* tile, const float4* __restrict__ tgt4, int mpad, f2 qx01,
                                                f2 qy01, f2 qz01, f2 qx23, f2 qy23, f2 qz23, float bd[kQPT],
                                                int bj[kQPT]) {
    for (int t0 = 0; t0 < mpad; t0 += kTargetTile) {
        __syncthreads();
#pragma unroll
        for (int k = threadIdx.x; k < kTargetTile; k += kPassBlock) tile[k] = tgt4[t0 + k];
        __syncthreads();
#pragma unroll 8
        for (int k = 0; k < kTargetTile; ++k) {
            const float4 t = tile[k];
            const f2 tx = {t.x, t.x}, ty = {t.y, t.y}, tz = {t.z, t.z};
            f2 dx = qx01 - tx, dy = qy01 - ty, dz = qz01 - tz;
            f2 d01 = dx * dx;
            d01 = pk_fma(dy, dy, d01);
            d01 = pk_fma(dz, dz, d01);
            dx = qx23 - tx;
            dy = qy23 - ty;
            dz = qz23 - tz;
            f2 d23 = dx * dx;
            d23 = pk_fma(dy, dy, d23);
            d23 = pk_fma(dz, dz, d23);
            const int j = t0 + k;
            if (d01.x < bd[0]) {
                bd[0] = d01.x;
                bj[0] = j;
            }
            if (d01.y < bd[1]) {
                bd[1] = d01.y;
                bj[1] = j;
            }
            if (d23.x < bd[2]) {
                bd[2] = d23.x;
                bj[2] = j;
            }
            if (d23.y < bd[3]) {
                bd[3] = d23.y;
                bj[3] = j;
            }
        }
    }
}

__device__ __forceinline__ void xform(const double Q[12], const double p[3], double q[3]) {
    q[0] = Q[0] * p[0] + Q[1] * p[1] + Q[2] * p[2] + Q[3];
    q[1] = Q[4] * p[0] + Q[5] * p[1] + Q[6] * p[2] + Q[7];
    q[2] = Q[8] * p[0] + Q[9] * p[1] + Q[10] * p[2] + Q[11];
}

// upper-triangle index of (a,b), a<=b, in a 6x6
__device__ __forceinline__ constexpr int ut(int a, int b) { return a * 6 - a * (a - 1) / 2 + (b - a); }

// --------------------------------------------------------------------------
// Fused correspondence pass: grid = (blocks per start, running starts).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kPassBlock) void gicp_pass_kernel(
    const double* __restrict__ src, const double* __restrict__ scov, int N, const float4* __restrict__ tgt4,
    const double* __restrict__ tgt64, const double* __restrict__ tcov, int mpad,
    const int32_t* __restrict__ active, const double* __restrict__ Qm, const double* __restrict__ Rm,
    const int32_t* __restrict__ done, double r2, float r2s, double* __restrict__ partial, int nblk) {
    const int slot = active[blockIdx.y];
    if (done[slot]) return;
    __shared__ float4 tile[kTargetTile];
    __shared__ double red[kPassBlock / 64][kNacc];

    double Q[12], R[9];
#pragma unroll
    for (int t = 0; t < 12; ++t) Q[t] = Qm[12 * slot + t];
#pragma unroll
    for (int t = 0; t < 9; ++t) R[t] = Rm[9 * slot + t];

    const int qbase = blockIdx.x * kPassQueries + threadIdx.x;
    float qxs[kQPT], qys[kQPT], qzs[kQPT], bd[kQPT];
    int bj[kQPT];
#pragma unroll
    for (int k = 0; k < kQPT; ++k) {
        const int i = qbase + k * kPassBlock;
        bj[k] = -1;
        if (i < N) {
            const double p[3] = {src[3 * i], src[3 * i + 1], src[3 * i + 2]};
            double q[3];
            xform(Q, p, q);
            qxs[k] = (float)q[0];
            qys[k] = (float)q[1];
            qzs[k] = (float)q[2];
            bd[k] = r2s;
        } else {
            qxs[k] = qys[k] = qzs[k] = 0.0f;
            bd[k] = -1.0f;  // never improves
        }
    }
    nn_search_tiles(tile, tgt4, mpad, f2{qxs[0], qxs[1]}, f2{qys[0], qys[1]}, f2{qzs[0], qzs[1]},
                    f2{qxs[2], qxs[3]}, f2{qys[2], qys[3]}, f2{qzs[2], qzs[3]}, bd, bj);

    // ---------------- fp64 epilogue: exact radius test + GICP normal equations
    double acc[kNacc];
#pragma unroll
    for (int v = 0; v < kNacc; ++v) acc[v] = 0.0;
#pragma unroll
    for (int k = 0; k < kQPT; ++k) {
        const int i = qbase + k * kPassBlock;
        const int j = bj[k];
        if (i >= N || j < 0) continue;
        const double p[3] = {src[3 * i], src[3 * i + 1], src[3 * i + 2]};
        double q[3];
        xform(Q, p, q);
        const double d[3] = {q[0] - tgt64[3 * j], q[1] - tgt64[3 * j + 1], q[2] - tgt64[3 * j + 2]};
        const double d2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        if (!(d2 < r2)) continue;
        const double* cs6 = scov + ((size_t)slot * N + i) * 6;
        const double* ct6 = tcov + (size_t)j * 6;
        Sym3 Cs{cs6[0], cs6[1], cs6[2], cs6[3], cs6[4], cs6[5]};
        Cs = rotate_sym(R, Cs);
        const Sym3 Mm{Cs.xx + ct6[0], Cs.xy + ct6[1], Cs.xz + ct6[2], Cs.yy + ct6[3], Cs.yz + ct6[4],
                      Cs.zz + ct6[5]};
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

    // ---------------- fixed-order block reduction -> one partial per block
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < kNacc; ++v) {
        const double s = wave_sum(acc[v]);
        if (lane == 0) red[wid][v] = s;
    }
    __syncthreads();
    if (threadIdx.x < kNacc) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kPassBlock / 64; ++w) s += red[w][threadIdx.x];
        partial[((size_t)slot * nblk + blockIdx.x) * kPartialStride + threadIdx.x] = s;
    }
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
// Per-start reduction of the block partials, convergence test
// (RegistrationICP), and the 6x6 solve + pose update.  One wave per start.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(64) void gicp_solve_kernel(const int32_t* __restrict__ active,
                                                        const double* __restrict__ partial, int nblk, int N,
                                                        int pass, int max_iter, double rel_fit, double rel_rmse,
                                                        SolveArgs a) {
    const int slot = active[blockIdx.x];
    if (a.done[slot]) return;
    const int lane = threadIdx.x;
    double s[kNacc];
#pragma unroll
    for (int v = 0; v < kNacc; ++v) s[v] = 0.0;
    for (int b = lane; b < nblk; b += 64) {
        const double* pp = partial + ((size_t)slot * nblk + b) * kPartialStride;
#pragma unroll
        for (int v = 0; v < kNacc; ++v) s[v] += pp[v];
    }
#pragma unroll
    for (int v = 0; v < kNacc; ++v) s[v] = wave_sum(s[v]);
    if (lane != 0) return;

    const double cnt = s[28];
    const double fit = cnt > 0 ? cnt / (double)N : 0.0;
    const double rmse = cnt > 0 ? sqrt(s[27] / cnt) : 0.0;
    const double pf = a.prev[2 * slot], pr = a.prev[2 * slot + 1];
    const bool converged = pass >= 1 && fabs(pf - fit) < rel_fit && fabs(pr - rmse) < rel_rmse;
    if (converged || pass >= max_iter) {
        a.done[slot] = 1;
        a.out_fit[slot] = fit;
        a.out_rmse[slot] = rmse;
        a.out_iters[slot] = pass;
        a.out_ncorr[slot] = (int64_t)cnt;
        return;
    }
    a.prev[2 * slot] = fit;
    a.prev[2 * slot + 1] = rmse;

    double upd[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    if (cnt > 0) {
        double JTJ[36], b[6];
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 6; ++c) JTJ[6 * r + c] = r <= c ? s[ut(r, c)] : s[ut(c, r)];
        for (int r = 0; r < 6; ++r) b[r] = -s[21 + r];
        const double det = det6(JTJ);
        if (!(fabs(det) < 1e-6 || isnan(det) || isinf(det))) {
            double x[6];
            ldlt_solve6(JTJ, b, x);
            vec6_to_m4(x, upd);
        }
    }
    double Tcur[16], Tn[16];
    for (int t = 0; t < 16; ++t) Tcur[t] = a.T[16 * slot + t];
    m4_mul(upd, Tcur, Tn);
    for (int t = 0; t < 16; ++t) a.T[16 * slot + t] = Tn[t];
    // Q = Tn * [G; 0 0 0 1]  (3x4), R = Tn[:3,:3]
    const double* G = a.G + 12 * slot;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 4; ++c) {
            double v = Tn[4 * r + 0] * G[c] + Tn[4 * r + 1] * G[4 + c] + Tn[4 * r + 2] * G[8 + c];
            if (c == 3) v += Tn[4 * r + 3];
            a.Q[12 * slot + 4 * r + c] = v;
        }
        for (int c = 0; c < 3; ++c) a.R[9 * slot + 3 * r + c] = Tn[4 * r + c];
    }
}

__global__ void prep_targets_kernel(const double* __restrict__ t64, int m, int mpad, float4* __restrict__ t4) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= mpad) return;
    if (i < m)
        t4[i] = make_float4((float)t64[3 * i], (float)t64[3 * i + 1], (float)t64[3 * i + 2], 0.0f);
    else
        t4[i] = make_float4(kFarCoord, kFarCoord, kFarCoord, 0.0f);
}

// Kernel-level 1-NN (orpcd_nn1_radius): same search, fp64 re-check, no
// accumulation.
__global__ __launch_bounds__(kPassBlock) void nn1_kernel(const double* __restrict__ q64, int nq,
                                                         const float4* __restrict__ tgt4,
                                                         const double* __restrict__ tgt64, int mpad, double r2,
                                                         float r2s, int32_t* __restrict__ idx,
                                                         double* __restrict__ d2o) {
    __shared__ float4 tile[kTargetTile];
    const int qbase = blockIdx.x * kPassQueries + threadIdx.x;
    float qxs[kQPT], qys[kQPT], qzs[kQPT], bd[kQPT];
    int bj[kQPT];
#pragma unroll
    for (int k = 0; k < kQPT; ++k) {
        const int i = qbase + k * kPassBlock;
        bj[k] = -1;
        if (i < nq) {
            qxs[k] = (float)q64[3 * i];
            qys[k] = (float)q64[3 * i + 1];
            qzs[k] = (float)q64[3 * i + 2];
            bd[k] = r2s;
        } else {
            qxs[k] = qys[k] = qzs[k] = 0.0f;
            bd[k] = -1.0f;
        }
    }
    nn_search_tiles(tile, tgt4, mpad, f2{qxs[0], qxs[1]}, f2{qys[0], qys[1]}, f2{qzs[0], qzs[1]},
                    f2{qxs[2], qxs[3]}, f2{qys[2], qys[3]}, f2{qzs[2], qzs[3]}, bd, bj);
#pragma unroll
    for (int k = 0; k < kQPT; ++k) {
        const int i = qbase + k * kPassBlock;
        if (i >= nq) continue;
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
        idx[i] = j;
        d2o[i] = dd;
    }
}

// fp32 search radius: enlarged so no pair with exact d^2 < r^2 is rejected by
// fp32 rounding (coordinates |x| <~ 1e3 relative error < 1e-6).
static inline float search_r2(double r2) { return (float)(r2 * (1.0 + 1e-5)) * 1.0001f; }

hipError_t launch_prep_targets(const double* tgt64, int64_t m, int64_t mpad, float4* tgt4, hipStream_t s) {
    if (mpad <= 0) return hipSuccess;
    prep_targets_kernel<<<(unsigned)((mpad + 255) / 256), 256, 0, s>>>(tgt64, (int)m, (int)mpad, tgt4);
    return hipGetLastError();
}

hipError_t launch_gicp_pass(const orpcd_ctx* c, int nact, int nblk, double r2, hipStream_t s) {
    const dim3 grid((unsigned)nblk, (unsigned)nact);
    gicp_pass_kernel<<<grid, kPassBlock, 0, s>>>(c->src64.p, c->scov.p, (int)c->N, c->tgt4.p, c->tgt64.p,
                                                 c->tcov.p, (int)c->Mpad, c->active.p, c->Q.p, c->R.p,
                                                 c->done.p, r2, search_r2(r2), c->partial.p, nblk);
    return hipGetLastError();
}

hipError_t launch_gicp_solve(const orpcd_ctx* c, int nact, int nblk, int pass, const orpcd_gicp_params& p,
                             hipStream_t s) {
    SolveArgs a{c->T.p,    c->Q.p,       c->R.p,        c->G.p,         c->prev.p,
                c->done.p, c->out_fit.p, c->out_rmse.p, c->out_iters.p, c->out_ncorr.p};
    gicp_solve_kernel<<<(unsigned)nact, 64, 0, s>>>(c->active.p, c->partial.p, nblk, (int)c->N, pass,
                                                    p.max_iteration, p.relative_fitness, p.relative_rmse, a);
    return hipGetLastError();
}

hipError_t launch_nn1(const double* q, int64_t nq, const float4* tgt4, const double* tgt64, int64_t mpad,
                      double r2, int32_t* idx, double* d2, hipStream_t s) {
    if (nq <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((nq + kPassQueries - 1) / kPassQueries);
    nn1_kernel<<<grid, kPassBlock, 0, s>>>(q, (int)nq, tgt4, tgt64, (int)mpad, r2, search_r2(r2), idx, d2);
    return hipGetLastError();
}

}  // namespace orpcd
