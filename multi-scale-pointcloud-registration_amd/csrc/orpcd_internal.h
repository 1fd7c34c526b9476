// orpcd_internal.h — host-side runtime structures shared by the .hip units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/orpcd.h"

namespace orpcd {

// ------------------------------------------------------------- geometry
constexpr int kPassBlock = 256;                     // threads per correspondence block
constexpr int kQPT = 4;                             // queries per thread (2 packed pairs)
constexpr int kPassQueries = kPassBlock * kQPT;     // queries per block (one start)
constexpr int kTargetTile = 1024;                   // fp32 targets staged per LDS tile
constexpr int kNacc = 29;                           // JTJ(21) + JTr(6) + sum d2 + count
constexpr int kPartialStride = 32;                  // doubles per block partial
constexpr float kFarCoord = 1.0e18f;                // padding target coordinate

// Device buffer that only grows (no hipMalloc inside steady-state loops).
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t count) {
        if (count <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, count * sizeof(T) + 256);
        if (e == hipSuccess) n = count;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

template <typename T>
struct HostBuf {  // pinned
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t count) {
        if (count <= n) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipHostMalloc(&p, count * sizeof(T) + 256, hipHostMallocDefault);
        if (e == hipSuccess) n = count;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

struct KernelStats {
    double launches = 0, ms = 0, pairs = 0, iterations = 0, passes = 0;
};

}  // namespace orpcd

struct orpcd_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // target (set per scale candidate)
    int64_t M = 0, Mpad = 0;
    orpcd::DevBuf<float4> tgt4;    // fp32 search copy (x,y,z,0), padded to Mpad
    orpcd::DevBuf<double> tgt64;   // M*3
    orpcd::DevBuf<double> tcov;    // M*6 GICP covariance
    double tgt_eps = -1.0;

    // source (set per align)
    int64_t N = 0;
    orpcd::DevBuf<double> src64;   // N*3
    orpcd::DevBuf<double> sraw;    // N*6 raw KNN-20 neighbourhood covariance

    // batch state (per start slot)
    orpcd::DevBuf<double> scov;    // B*N*6 posed-frame source covariance
    orpcd::DevBuf<double> G;       // B*12 base pose (3x4, column convention)
    orpcd::DevBuf<double> T;       // B*16 accumulated ICP transform
    orpcd::DevBuf<double> Q;       // B*12 T*G (3x4)
    orpcd::DevBuf<double> R;       // B*9 rotation of T
    orpcd::DevBuf<double> prev;    // B*2 previous (fitness, rmse)
    orpcd::DevBuf<double> partial; // B*nblk*32
    orpcd::DevBuf<int32_t> done;   // B
    orpcd::DevBuf<int32_t> active; // B
    orpcd::DevBuf<double> out_fit, out_rmse;
    orpcd::DevBuf<int32_t> out_iters;
    orpcd::DevBuf<int64_t> out_ncorr;

    // scratch for kernel-level entry points
    orpcd::DevBuf<double> scratch64a, scratch64b, scratch64c;
    orpcd::DevBuf<float4> scratch4;
    orpcd::DevBuf<int32_t> scratch32;

    orpcd::HostBuf<double> h64;
    orpcd::HostBuf<int32_t> h32;

    // profiling
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;
    orpcd::KernelStats stats;
};

namespace orpcd {

// launchers (knn_kernels.hip)
hipError_t launch_knn_cov(const double* pts, int64_t n, int k, double radius, double* rawcov6, int32_t* nbr_idx,
                          int32_t* nbr_cnt, hipStream_t s);
hipError_t launch_normals_cov(const double* rawcov6, int64_t n, const double* Rc9, int nslots, double eps,
                              double* normals3, double* cov6, hipStream_t s);

// launchers (gicp_kernels.hip)
hipError_t launch_prep_targets(const double* tgt64, int64_t m, int64_t mpad, float4* tgt4, hipStream_t s);
hipError_t launch_gicp_pass(const orpcd_ctx* c, int nact, int nblk, double r2, hipStream_t s);
hipError_t launch_gicp_solve(const orpcd_ctx* c, int nact, int nblk, int pass, const orpcd_gicp_params& p,
                             hipStream_t s);
hipError_t launch_nn1(const double* q, int64_t nq, const float4* tgt4, const double* tgt64, int64_t mpad,
                      double r2, int32_t* idx, double* d2, hipStream_t s);

}  // namespace orpcd
