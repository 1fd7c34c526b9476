// device_math.h — fp64 small-matrix routines used by the gfx950 kernels.
//
// Each routine restates the Open3D 0.18.0 algorithm the reference reaches
// through registration_generalized_icp (generalizedICP.py:59-70) /
// estimate_normals (fastGlobalOptimizer.py:118-127).  Floating-point
// contraction is disabled where the oracle (gcc, -ffp-contract=off) must be
// matched operation for operation (covariance cumulants, FastEigen3x3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orpcd {

struct Sym3 {  // symmetric 3x3: xx xy xz yy yz zz
    double xx, xy, xz, yy, yz, zz;
};

__device__ __forceinline__ void cross3(const double a[3], const double b[3], double r[3]) {
#pragma clang fp contract(off)
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
}

// O3D EstimateNormals.cpp ComputeEigenvector0 (division form of Eigen).
__device__ inline void eigvec0(const double A[3][3], double eval0, double out[3]) {
#pragma clang fp contract(off)
    double row0[3] = {A[0][0] - eval0, A[0][1], A[0][2]};
    double row1[3] = {A[0][1], A[1][1] - eval0, A[1][2]};
    double row2[3] = {A[0][2], A[1][2], A[2][2] - eval0};
    double r0xr1[3], r0xr2[3], r1xr2[3];
    cross3(row0, row1, r0xr1);
    cross3(row0, row2, r0xr2);
    cross3(row1, row2, r1xr2);
    double d0 = r0xr1[0] * r0xr1[0] + r0xr1[1] * r0xr1[1] + r0xr1[2] * r0xr1[2];
    double d1 = r0xr2[0] * r0xr2[0] + r0xr2[1] * r0xr2[1] + r0xr2[2] * r0xr2[2];
    double d2 = r1xr2[0] * r1xr2[0] + r1xr2[1] * r1xr2[1] + r1xr2[2] * r1xr2[2];
    double dmax = d0;
    int imax = 0;
    if (d1 > dmax) {
        dmax = d1;
        imax = 1;
    }
    if (d2 > dmax) imax = 2;
    if (imax == 0) {
        double s = sqrt(d0);
        out[0] = r0xr1[0] / s;
        out[1] = r0xr1[1] / s;
        out[2] = r0xr1[2] / s;
    } else if (imax == 1) {
        double s = sqrt(d1);
        out[0] = r0xr2[0] / s;
        out[1] = r0xr2[1] / s;
        out[2] = r0xr2[2] / s;
    } else {
        double s = sqrt(d2);
        out[0] = r1xr2[0] / s;
        out[1] = r1xr2[1] / s;
        out[2] = r1xr2[2] / s;
    }
}

// O3D EstimateNormals.cpp ComputeEigenvector1.
__device__ inline void eigvec1(const double A[3][3], const double e0[3], double eval1, double out[3]) {
#pragma clang fp contract(off)
    double U[3], V[3];
    if (fabs(e0[0]) > fabs(e0[1])) {
        double inv_length = 1.0 / sqrt(e0[0] * e0[0] + e0[2] * e0[2]);
        U[0] = -e0[2] * inv_length;
        U[1] = 0.0;
        U[2] = e0[0] * inv_length;
    } else {
        double inv_length = 1.0 / sqrt(e0[1] * e0[1] + e0[2] * e0[2]);
        U[0] = 0.0;
        U[1] = e0[2] * inv_length;
        U[2] = -e0[1] * inv_length;
    }
    cross3(e0, U, V);
    double AU[3] = {A[0][0] * U[0] + A[0][1] * U[1] + A[0][2] * U[2],
                    A[0][1] * U[0] + A[1][1] * U[1] + A[1][2] * U[2],
                    A[0][2] * U[0] + A[1][2] * U[1] + A[2][2] * U[2]};
    double AV[3] = {A[0][0] * V[0] + A[0][1] * V[1] + A[0][2] * V[2],
                    A[0][1] * V[0] + A[1][1] * V[1] + A[1][2] * V[2],
                    A[0][2] * V[0] + A[1][2] * V[1] + A[2][2] * V[2]};
    double m00 = U[0] * AU[0] + U[1] * AU[1] + U[2] * AU[2] - eval1;
    double m01 = U[0] * AV[0] + U[1] * AV[1] + U[2] * AV[2];
    double m11 = V[0] * AV[0] + V[1] * AV[1] + V[2] * AV[2] - eval1;
    double absM00 = fabs(m00), absM01 = fabs(m01), absM11 = fabs(m11);
    double a, b;  // result = a*U - b*V
    if (absM00 >= absM11) {
        double mx = fmax(absM00, absM01);
        if (mx > 0) {
            if (absM00 >= absM01) {
                m01 /= m00;
                m00 = 1.0 / sqrt(1.0 + m01 * m01);
                m01 *= m00;
            } else {
                m00 /= m01;
                m01 = 1.0 / sqrt(1.0 + m00 * m00);
                m00 *= m01;
            }
            a = m01;
            b = m00;
        } else {
            out[0] = U[0];
            out[1] = U[1];
            out[2] = U[2];
            return;
        }
    } else {
        double mx = fmax(absM11, absM01);
        if (mx > 0) {
            if (absM11 >= absM01) {
                m01 /= m11;
                m11 = 1.0 / sqrt(1.0 + m01 * m01);
                m01 *= m11;
            } else {
                m11 /= m01;
                m01 = 1.0 / sqrt(1.0 + m11 * m11);
                m11 *= m01;
            }
            a = m11;
            b = m01;
        } else {
            out[0] = U[0];
            out[1] = U[1];
            out[2] = U[2];
            return;
        }
    }
    out[0] = a * U[0] - b * V[0];
    out[1] = a * U[1] - b * V[1];
    out[2] = a * U[2] - b * V[2];
}

// O3D EstimateNormals.cpp FastEigen3x3: eigenvector of the smallest
// eigenvalue of a symmetric 3x3 (the surface normal).
__device__ inline void fast_eigen3x3(const Sym3& C, double n[3]) {
#pragma clang fp contract(off)
    double A[3][3] = {{C.xx, C.xy, C.xz}, {C.xy, C.yy, C.yz}, {C.xz, C.yz, C.zz}};
    double max_coeff = A[0][0];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) max_coeff = fmax(max_coeff, A[i][j]);
    if (max_coeff == 0) {
        n[0] = n[1] = n[2] = 0.0;
        return;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) A[i][j] /= max_coeff;
    double nrm = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
    if (nrm > 0) {
        double q = (A[0][0] + A[1][1] + A[2][2]) / 3.0;
        double b00 = A[0][0] - q, b11 = A[1][1] - q, b22 = A[2][2] - q;
        double p = sqrt((b00 * b00 + b11 * b11 + b22 * b22 + nrm * 2.0) / 6.0);
        double c00 = b11 * b22 - A[1][2] * A[1][2];
        double c01 = A[0][1] * b22 - A[1][2] * A[0][2];
        double c02 = A[0][1] * A[1][2] - b11 * A[0][2];
        double det = (b00 * c00 - A[0][1] * c01 + A[0][2] * c02) / (p * p * p);
        double half_det = det * 0.5;
        half_det = fmin(fmax(half_det, -1.0), 1.0);
        double angle = acos(half_det) / 3.0;
        const double two_thirds_pi = 2.09439510239319549;
        double beta2 = cos(angle) * 2.0;
        double beta0 = cos(angle + two_thirds_pi) * 2.0;
        double beta1 = -(beta0 + beta2);
        double eval0 = q + p * beta0, eval1 = q + p * beta1, eval2 = q + p * beta2;
        double ea[3], eb[3];
        if (half_det >= 0) {
            eigvec0(A, eval2, ea);
            if (eval2 < eval0 && eval2 < eval1) {
                n[0] = ea[0];
                n[1] = ea[1];
                n[2] = ea[2];
                return;
            }
            eigvec1(A, ea, eval1, eb);
            if (eval1 < eval0 && eval1 < eval2) {
                n[0] = eb[0];
                n[1] = eb[1];
                n[2] = eb[2];
                return;
            }
            cross3(eb, ea, n);  // evec1 x evec2
        } else {
            eigvec0(A, eval0, ea);
            if (eval0 < eval1 && eval0 < eval2) {
                n[0] = ea[0];
                n[1] = ea[1];
                n[2] = ea[2];
                return;
            }
            eigvec1(A, ea, eval1, eb);
            if (eval1 < eval0 && eval1 < eval2) {
                n[0] = eb[0];
                n[1] = eb[1];
                n[2] = eb[2];
                return;
            }
            cross3(ea, eb, n);  // evec0 x evec1
        }
    } else {
        n[0] = n[1] = n[2] = 0.0;
        if (A[0][0] < A[1][1] && A[0][0] < A[2][2])
            n[0] = 1.0;
        else if (A[1][1] < A[0][0] && A[1][1] < A[2][2])
            n[1] = 1.0;
        else
            n[2] = 1.0;
    }
}

// O3D GeneralizedICP.cpp GetRotationFromE1ToX + InitializePointCloudFor-
// GeneralizedICP: C = R diag(eps,1,1) R^T (R = I when n.e1 < -0.99).
__device__ inline Sym3 gicp_cov_from_normal(const double n[3], double eps) {
#pragma clang fp contract(off)
    double R[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
    double c = n[0];
    if (!(c < -0.99)) {
        // v = e1 x n = (0, -n2, n1);  sv = skew(v)
        double vx = 0.0, vy = -n[2], vz = n[1];
        double sv[3][3] = {{0.0, -vz, vy}, {vz, 0.0, -vx}, {-vy, vx, 0.0}};
        double factor = 1.0 / (1.0 + c);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                double s2 = sv[i][0] * sv[0][j] + sv[i][1] * sv[1][j] + sv[i][2] * sv[2][j];
                R[i][j] += sv[i][j] + s2 * factor;
            }
    }
    const double d[3] = {eps, 1.0, 1.0};
    double RC[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) RC[i][j] = R[i][0] * (j == 0 ? d[0] : 0.0) + R[i][1] * (j == 1 ? d[1] : 0.0) +
                                               R[i][2] * (j == 2 ? d[2] : 0.0);
    double O[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) O[i][j] = RC[i][0] * R[j][0] + RC[i][1] * R[j][1] + RC[i][2] * R[j][2];
    return Sym3{O[0][0], O[0][1], O[0][2], O[1][1], O[1][2], O[2][2]};
}

// Inverse of a symmetric positive-definite 3x3 (cofactors / det).
__device__ __forceinline__ Sym3 sym3_inverse(const Sym3& a) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    double c00 = a.yy * a.zz - a.yz * a.yz;
    double c01 = a.xz * a.yz - a.xy * a.zz;
    double c02 = a.xy * a.yz - a.xz * a.yy;
    double det = a.xx * c00 + a.xy * c01 + a.xz * c02;
    double id = 1.0 / det;
    Sym3 r;
    r.xx = c00 * id;
    r.xy = c01 * id;
    r.xz = c02 * id;
    r.yy = (a.xx * a.zz - a.xz * a.xz) * id;
    r.yz = (a.xy * a.xz - a.xx * a.yz) * id;
    r.zz = (a.xx * a.yy - a.xy * a.xy) * id;
    return r;
}

// R S R^T for symmetric S.
__device__ __forceinline__ Sym3 rotate_sym(const double R[9], const Sym3& S) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    double A[3][3] = {{S.xx, S.xy, S.xz}, {S.xy, S.yy, S.yz}, {S.xz, S.yz, S.zz}};
    double RA[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) RA[i][j] = R[3 * i] * A[0][j] + R[3 * i + 1] * A[1][j] + R[3 * i + 2] * A[2][j];
    double O[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) O[i][j] = RA[i][0] * R[3 * j] + RA[i][1] * R[3 * j + 1] + RA[i][2] * R[3 * j + 2];
    return Sym3{O[0][0], O[0][1], O[0][2], O[1][1], O[1][2], O[2][2]};
}

// ---------------------------------------------------------------- 6x6 solve
// O3D utility/Eigen.cpp SolveLinearSystemPSD with check_det=true:
// det by partial-pivot LU; |det| < 1e-6 -> failure; else Eigen LDLT.
// Row / column exchanges below index the 6x6 only at compile-time positions
// (never A[piv][j] with a runtime piv), so it stays in registers; the
// arithmetic and its order are those of the CPU restatement.  Every caller
// runs the solve in ONE lane (icp_solve_kernel / finish_pass / fgr_irls lane
// 0), so the pivot is made wave-uniform and each candidate exchange is a
// scalar branch that moves registers only when taken (written as selects
// over all candidates, the exchanges were ~half of the solve's 13k cycles,
// tools/solve_bench.hip).
__device__ __forceinline__ void swap_rows6(double A[6][6], int k, int p) {
    p = __builtin_amdgcn_readfirstlane(p);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        if (i <= k) continue;
        if (i == p) {
            asm volatile("" ::: "memory");  // keep the branch: no speculation into selects
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const double a = A[k][j];
                A[k][j] = A[i][j];
                A[i][j] = a;
            }
        }
    }
}
__device__ __forceinline__ void swap_cols6(double A[6][6], int k, int p) {
    p = __builtin_amdgcn_readfirstlane(p);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        if (i <= k) continue;
        if (i == p) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const double a = A[j][k];
                A[j][k] = A[j][i];
                A[j][i] = a;
            }
        }
    }
}

// Eigen PartialPivLU determinant (SolveLinearSystemPSD's check_det).
__device__ inline double det6(const double Ain[36]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    double A[6][6];
#pragma unroll
    for (int i = 0; i < 36; ++i) A[i / 6][i % 6] = Ain[i];
    double det = 1.0;
    bool zero = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int piv = k;
        double best = fabs(A[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i)
            if (fabs(A[i][k]) > best) {
                best = fabs(A[i][k]);
                piv = i;
            }
        if (piv != k) {
            swap_rows6(A, k, piv);
            det = -det;
        }
        zero = zero || A[k][k] == 0.0;
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double f = A[i][k] / A[k][k];
#pragma unroll
            for (int j = k + 1; j < 6; ++j) A[i][j] -= f * A[k][j];
        }
        det *= A[k][k];
    }
    return zero ? 0.0 : det;
}

// Eigen LDLT (diagonal pivoting) solve of A x = b.
__device__ inline void ldlt_solve6(const double Ain[36], const double b[6], double x[6]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    double A[6][6];
#pragma unroll
    for (int i = 0; i < 36; ++i) A[i / 6][i % 6] = Ain[i];
    int tr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int idx = k;
        double big = fabs(A[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; ++i)
            if (fabs(A[i][i]) > big) {
                big = fabs(A[i][i]);
                idx = i;
            }
        tr[k] = idx;
        if (idx != k) {
            swap_rows6(A, k, idx);
            swap_cols6(A, k, idx);
        }
        double tmp[6];
#pragma unroll
        for (int j = 0; j < k; ++j) tmp[j] = A[j][j] * A[k][j];
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < k; ++j) s += A[k][j] * tmp[j];
        A[k][k] -= s;
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < k; ++j) t += A[i][j] * tmp[j];
            A[i][k] -= t;
        }
        const double akk = A[k][k];
        if (fabs(akk) > 0.0) {
#pragma unroll
            for (int i = k + 1; i < 6; ++i) A[i][k] /= akk;
        }
    }
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) y[i] = b[i];
    auto swap_y = [&](int k, int p) {
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            if (m <= k) continue;
            const bool sw = m == p;
            const double a = y[k], c = y[m];
            y[k] = sw ? c : a;
            y[m] = sw ? a : c;
        }
    };
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (tr[k] != k) swap_y(k, tr[k]);
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < i; ++j) y[i] -= A[i][j] * y[j];
    const double tol = 2.2250738585072014e-308;
#pragma unroll
    for (int i = 0; i < 6; ++i) y[i] = fabs(A[i][i]) > tol ? y[i] / A[i][i] : 0.0;
#pragma unroll
    for (int i = 5; i >= 0; --i)
#pragma unroll
        for (int j = i + 1; j < 6; ++j) y[i] -= A[j][i] * y[j];
#pragma unroll
    for (int k = 5; k >= 0; --k)
        if (tr[k] != k) swap_y(k, tr[k]);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = y[i];
}

// O3D utility/Eigen.cpp TransformVector6dToMatrix4d (via Eigen quaternions).
__device__ inline void vec6_to_m4(const double x[6], double T[16]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    double zw = cos(x[2] * 0.5), zz = sin(x[2] * 0.5);
    double yw = cos(x[1] * 0.5), yy = sin(x[1] * 0.5);
    double xw = cos(x[0] * 0.5), xx = sin(x[0] * 0.5);
    // a = qz * qy   (qz = (zw,0,0,zz), qy = (yw,0,yy,0))
    double aw = zw * yw - 0.0 * 0.0 - 0.0 * yy - zz * 0.0;
    double ax = zw * 0.0 + 0.0 * yw + 0.0 * 0.0 - zz * yy;
    double ay = zw * yy + 0.0 * yw + zz * 0.0 - 0.0 * 0.0;
    double az = zw * 0.0 + zz * yw + 0.0 * yy - 0.0 * 0.0;
    // q = a * qx    (qx = (xw,xx,0,0))
    double qw = aw * xw - ax * xx - ay * 0.0 - az * 0.0;
    double qx = aw * xx + ax * xw + ay * 0.0 - az * 0.0;
    double qy = aw * 0.0 + ay * xw + az * xx - ax * 0.0;
    double qz = aw * 0.0 + az * xw + ax * 0.0 - ay * xx;
    double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    double twx = tx * qw, twy = ty * qw, twz = tz * qw;
    double txx = tx * qx, txy = ty * qx, txz = tz * qx;
    double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    T[0] = 1 - (tyy + tzz);
    T[1] = txy - twz;
    T[2] = txz + twy;
    T[3] = x[3];
    T[4] = txy + twz;
    T[5] = 1 - (txx + tzz);
    T[6] = tyz - twx;
    T[7] = x[4];
    T[8] = txz - twy;
    T[9] = tyz + twx;
    T[10] = 1 - (txx + tyy);
    T[11] = x[5];
    T[12] = 0.0;
    T[13] = 0.0;
    T[14] = 0.0;
    T[15] = 1.0;
}

__device__ __forceinline__ void m4_mul(const double A[16], const double B[16], double C[16]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += A[4 * i + k] * B[4 * k + j];
            C[4 * i + j] = s;
        }
}

// ------------------------------------------------ PointToPoint (Umeyama)
// 3x3 SVD A = U diag(s) V^T by one-sided (Hestenes) Jacobi in fp64, singular
// values descending; a vanished singular value's U column is completed
// orthonormally.  Single-lane code (the solve runs one lane per start).
__device__ inline void svd3_jacobi(const double A[3][3], double U[3][3], double s[3], double V[3][3]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    double a[3][3], v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) a[i][j] = A[i][j];
    for (int sweep = 0; sweep < 60; ++sweep) {
        bool rotated = false;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < 3; ++i) {
                    al += a[i][p] * a[i][p];
                    be += a[i][q] * a[i][q];
                    ga += a[i][p] * a[i][q];
                }
                if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
                rotated = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
                for (int i = 0; i < 3; ++i) {
                    const double x = a[i][p], y = a[i][q];
                    a[i][p] = c * x - sn * y;
                    a[i][q] = sn * x + c * y;
                    const double vx = v[i][p], vy = v[i][q];
                    v[i][p] = c * vx - sn * vy;
                    v[i][q] = sn * vx + c * vy;
                }
            }
        if (!rotated) break;
    }
    double nrm[3];
    for (int j = 0; j < 3; ++j) nrm[j] = sqrt(a[0][j] * a[0][j] + a[1][j] * a[1][j] + a[2][j] * a[2][j]);
    int ord[3] = {0, 1, 2};
    for (int x = 0; x < 2; ++x)  // stable descending sort of 3
        for (int y = 0; y < 2 - x; ++y)
            if (nrm[ord[y + 1]] > nrm[ord[y]]) {
                const int t = ord[y];
                ord[y] = ord[y + 1];
                ord[y + 1] = t;
            }
    for (int k = 0; k < 3; ++k) {
        const int j = ord[k];
        s[k] = nrm[j];
        for (int i = 0; i < 3; ++i) {
            V[i][k] = v[i][j];
            U[i][k] = nrm[j] > 1e-300 ? a[i][j] / nrm[j] : 0.0;
        }
    }
    if (!(s[0] > 1e-300)) {  // sigma == 0 (e.g. one pair): U = V = I as JacobiSVD leaves them
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) U[i][k] = V[i][k] = i == k ? 1.0 : 0.0;
    }
    else if (!(s[1] > 1e-300)) {
        const double c0[3] = {U[0][0], U[1][0], U[2][0]};
        const double e[3] = {fabs(c0[0]) < 0.9 ? 1.0 : 0.0, fabs(c0[0]) < 0.9 ? 0.0 : 1.0, 0.0};
        double c1[3];
        cross3(c0, e, c1);
        const double l = sqrt(c1[0] * c1[0] + c1[1] * c1[1] + c1[2] * c1[2]);
        for (int i = 0; i < 3; ++i) U[i][1] = c1[i] / l;
    }
    if (s[0] > 1e-300 && !(s[2] > 1e-300)) {
        const double c0[3] = {U[0][0], U[1][0], U[2][0]}, c1[3] = {U[0][1], U[1][1], U[2][1]};
        double c2[3];
        cross3(c0, c1, c2);
        for (int i = 0; i < 3; ++i) U[i][2] = c2[i];
    }
}

__device__ __forceinline__ double det3(const double a[3][3]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    return a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
           a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
}

// Eigen::umeyama(src, dst, with_scaling = false) from first moments:
// s = [sum src (3), sum dst (3), sum dst_a src_b (9, row-major)], n pairs.
// sigma = sum(dst src^T)/n - mean_dst mean_src^T; R = U diag(1,1,+-1) V^T;
// t = mean_dst - R mean_src.  T: 4x4 row-major, column convention.
__device__ inline void umeyama_from_moments(const double* s, double n, double T[16]) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    const double inv = 1.0 / n;
    const double ms[3] = {s[0] * inv, s[1] * inv, s[2] * inv};
    const double md[3] = {s[3] * inv, s[4] * inv, s[5] * inv};
    double sig[3][3], U[3][3], V[3][3], sv[3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) sig[a][b] = s[6 + 3 * a + b] * inv - md[a] * ms[b];
    svd3_jacobi(sig, U, sv, V);
    const double sgn = det3(U) * det3(V) < 0 ? -1.0 : 1.0;
    for (int a = 0; a < 3; ++a) {
        for (int b = 0; b < 3; ++b) T[4 * a + b] = U[a][0] * V[b][0] + U[a][1] * V[b][1] + sgn * U[a][2] * V[b][2];
        T[4 * a + 3] = md[a] - (T[4 * a] * ms[0] + T[4 * a + 1] * ms[1] + T[4 * a + 2] * ms[2]);
    }
    T[12] = T[13] = T[14] = 0.0;
    T[15] = 1.0;
}

// ------------------------------------------------- wave-parallel 6x6 solve
// det6 / ldlt_solve6 / vec6_to_m4 spread over one wave: lane r < 6 holds row
// r of the 6x6 system.  Every matrix element sees the same operations, in the
// same order, with the same operands as in the single-lane code above (pivot
// scans on the broadcast values, eliminations row-parallel, sums in index
// order), so the results are bit-identical (orpcd_test_solve6, tests/
// test_gpu_gicp.py::test_wave_solve_bit_identical); the transcendental half-
// angle terms run on six lanes at once.  All 64 lanes call these (uniform
// control flow); outputs are wave-uniform.
__device__ __forceinline__ double rl64(double v, int k) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, k);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), k);
    return __longlong_as_double(((long long)hi << 32) | lo);
}

// rows k and p (wave-uniform) exchange lanes
__device__ __forceinline__ void wave_swap_rows6(double a[6], int k, int p, int lane) {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const double ak = rl64(a[j], k), ap = rl64(a[j], p);
        a[j] = lane == k ? ap : (lane == p ? ak : a[j]);
    }
}

__device__ inline double det6_wave(const double row[6], int lane) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    double a[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) a[j] = row[j];
    double det = 1.0;
    bool zero = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int piv = k;
        double best = fabs(rl64(a[k], k));
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double v = fabs(rl64(a[k], i));
            if (v > best) {
                best = v;
                piv = i;
            }
        }
        piv = __builtin_amdgcn_readfirstlane(piv);
        if (piv != k) {
            wave_swap_rows6(a, k, piv, lane);
            det = -det;
        }
        const double akk = rl64(a[k], k);
        zero = zero || akk == 0.0;
        double rk[6];
#pragma unroll
        for (int j = k + 1; j < 6; ++j) rk[j] = rl64(a[j], k);
        if (lane > k && lane < 6) {
            const double f = a[k] / akk;
#pragma unroll
            for (int j = k + 1; j < 6; ++j) a[j] -= f * rk[j];
        }
        det *= akk;
    }
    return zero ? 0.0 : det;
}

__device__ inline void ldlt_solve6_wave(const double row[6], const double b[6], double x[6], int lane) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    double a[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) a[j] = row[j];
    int tr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int idx = k;
        double big = fabs(rl64(a[k], k));
#pragma unroll
        for (int i = k + 1; i < 6; ++i) {
            const double v = fabs(rl64(a[i], i));
            if (v > big) {
                big = v;
                idx = i;
            }
        }
        idx = __builtin_amdgcn_readfirstlane(idx);
        tr[k] = idx;
        if (idx != k) {
            wave_swap_rows6(a, k, idx, lane);
#pragma unroll
            for (int m = k + 1; m < 6; ++m) {  // the column exchange, inside every row
                if (idx == m) {
                    const double t = a[k];
                    a[k] = a[m];
                    a[m] = t;
                }
            }
        }
        double tmp[6];
#pragma unroll
        for (int j = 0; j < k; ++j) tmp[j] = rl64(a[j], j) * rl64(a[j], k);
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < k; ++j) s += rl64(a[j], k) * tmp[j];
        if (lane == k) a[k] -= s;
        if (lane > k && lane < 6) {
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < k; ++j) t += a[j] * tmp[j];
            a[k] -= t;
        }
        const double akk = rl64(a[k], k);
        if (fabs(akk) > 0.0 && lane > k && lane < 6) a[k] /= akk;
    }
    // substitutions (ldlt_solve6's order): y = P b, L y' = y, D, L^T, P^T
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) y[i] = b[i];
    auto swap_y = [&](int k, int p) {
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            if (m <= k) continue;
            const bool sw = m == p;
            const double u = y[k], c = y[m];
            y[k] = sw ? c : u;
            y[m] = sw ? u : c;
        }
    };
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (tr[k] != k) swap_y(k, tr[k]);
    // forward, column by column: y[i] -= A[i][j] y[j] in increasing j for every i
    double yl = 0.0;  // lane i: its y[i]
#pragma unroll
    for (int i = 0; i < 6; ++i)
        if (lane == i) yl = y[i];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const double yj = rl64(yl, j);
        if (lane > j && lane < 6) yl -= a[j] * yj;
    }
    double dl = a[0];  // lane i: A[i][i]
#pragma unroll
    for (int i = 1; i < 6; ++i)
        if (lane == i) dl = a[i];
    const double tol = 2.2250738585072014e-308;
    yl = fabs(dl) > tol ? yl / dl : 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) y[i] = rl64(yl, i);
    // backward: y[i] -= A[j][i] y[j] for j = i+1 .. 5 (uniform, sequential as ldlt_solve6)
#pragma unroll
    for (int i = 5; i >= 0; --i)
#pragma unroll
        for (int j = i + 1; j < 6; ++j) y[i] -= rl64(a[i], j) * y[j];
#pragma unroll
    for (int k = 5; k >= 0; --k)
        if (tr[k] != k) swap_y(k, tr[k]);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = y[i];
}

// vec6_to_m4 with its six half-angle cos / sin on lanes 0..5
__device__ inline void vec6_to_m4_wave(const double x[6], double T[16], int lane) {
#pragma clang fp contract(off)  // no fused multiply-add: the same rounding in every caller
    const double h = lane < 2 ? x[2] : (lane < 4 ? x[1] : x[0]);
    const double v = (lane & 1) ? sin(h * 0.5) : cos(h * 0.5);
    double zw = rl64(v, 0), zz = rl64(v, 1);
    double yw = rl64(v, 2), yy = rl64(v, 3);
    double xw = rl64(v, 4), xx = rl64(v, 5);
    double aw = zw * yw - 0.0 * 0.0 - 0.0 * yy - zz * 0.0;
    double ax = zw * 0.0 + 0.0 * yw + 0.0 * 0.0 - zz * yy;
    double ay = zw * yy + 0.0 * yw + zz * 0.0 - 0.0 * 0.0;
    double az = zw * 0.0 + zz * yw + 0.0 * yy - 0.0 * 0.0;
    double qw = aw * xw - ax * xx - ay * 0.0 - az * 0.0;
    double qx = aw * xx + ax * xw + ay * 0.0 - az * 0.0;
    double qy = aw * 0.0 + ay * xw + az * xx - ax * 0.0;
    double qz = aw * 0.0 + az * xw + ax * 0.0 - ay * xx;
    double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    double twx = tx * qw, twy = ty * qw, twz = tz * qw;
    double txx = tx * qx, txy = ty * qx, txz = tz * qx;
    double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    T[0] = 1 - (tyy + tzz);
    T[1] = txy - twz;
    T[2] = txz + twy;
    T[3] = x[3];
    T[4] = txy + twz;
    T[5] = 1 - (txx + tzz);
    T[6] = tyz - twx;
    T[7] = x[4];
    T[8] = txz - twy;
    T[9] = tyz + twx;
    T[10] = 1 - (txx + tyy);
    T[11] = x[5];
    T[12] = 0.0;
    T[13] = 0.0;
    T[14] = 0.0;
    T[15] = 1.0;
}

// lane r < 6: row r of the symmetric 6x6 whose upper triangle is
// s[ut(a, b)] (a <= b, ut = row-major upper-triangle index)
__device__ __forceinline__ void sym6_row(const double* s, int lane, double row[6]) {
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            const int a = r <= c ? r : c, b = r <= c ? c : r;
            if (lane == r) v = s[a * 6 - a * (a - 1) / 2 + (b - a)];
        }
        row[c] = v;
    }
}

// ------------------------------------------------------- wave reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace orpcd
