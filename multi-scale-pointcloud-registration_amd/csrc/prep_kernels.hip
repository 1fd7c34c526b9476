// prep_kernels.hip — the steps either side of the hot path:
// statistical outlier removal, voxel downsampling and farthest-point
// sampling, on gfx950.
//
//  * SOR.process (sor.py:51-79) -> O3D PointCloud::RemoveStatisticalOutliers.
//    The KNN-k mean distances come from knn_tiles_kernel (knn_kernels.hip,
//    exact fp64 neighbour sets in (d^2, index) order); sor_stats_kernel then
//    folds them in index order exactly as std::accumulate / inner_product do
//    (one lane, fp64, the reference's order), so the threshold is bit-exact;
//    sor_flag_kernel marks 0 < mean < threshold and hipCUB compacts the kept
//    indices (increasing, as SelectByIndex keeps them).
//  * VoxelDownsampler (voxelDownsampler.py:77-126) -> O3D
//    PointCloud::VoxelDownSample.  voxel_key_kernel packs floor((p - min +
//    vs/2) / vs) per axis into a 63-bit lexicographic key; a stable radix sort
//    keeps each voxel's points in input order, run-length encoding gives the
//    voxels, and voxel_mean_kernel sums each run in that order and divides by
//    its count (Open3D's AccumulatedPoint), so every averaged point is
//    bit-exact.  Voxels come out in key order (Open3D: unordered_map order).
//  * FarthestDownsampler.process (farthestDownsampler.py:26-54).  One
//    cooperative launch runs all sample_size-1 steps: every thread keeps its
//    points and their running minimum distance in registers; per step each
//    block reduces (max distance, lowest index), publishes it, one grid
//    barrier (a step counter), then every block reduces the published values
//    itself (no second barrier).  Distances are the reference's cdist Euclidean: differences,
//    squares summed x, y, z in order, correctly rounded sqrt, contraction off.
#include <hipcub/hipcub.hpp>

#include "orpcd_internal.h"

namespace orpcd {

// ---------------------------------------------------------------- SOR
// stats[0] = cloud_mean, [1] = std_dev, [2] = threshold, [3] = valid count.
// The folds are sequential in index order (as std::accumulate and
// std::inner_product run them): the wave loads 64 values per step and the
// unrolled readlanes feed them, in lane order, to one dependent add chain.
__global__ __launch_bounds__(64) void sor_stats_kernel(const double* __restrict__ avg, int n, double std_ratio,
                                                       double* __restrict__ stats) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x;
    auto rl = [](double v, int k) {
        const unsigned long long b = __double_as_longlong(v);
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, k), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), k);
        return __longlong_as_double(((unsigned long long)hi << 32) | lo);
    };
    double cloud_mean = 0.0, sq_sum = 0.0;
    int valid = 0;
    // pass 1: accumulate(avg, 0.0, [](x, y) { return y > 0 ? x + y : x; }) and the
    // count of non-empty searches (mean != -1)
    for (int b = 0; b < n; b += 64) {
        const double v = b + lane < n ? avg[b + lane] : -1.0;
        valid += __popcll(__ballot(v != -1.0));
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            const double y = rl(v, k);
            cloud_mean = y > 0 ? cloud_mean + y : cloud_mean;
        }
    }
    if (valid == 0) {
        if (lane == 0) stats[0] = stats[1] = stats[2] = stats[3] = 0.0;
        return;
    }
    cloud_mean /= (double)valid;
    // pass 2: inner_product(..., plus, [](x, y) { return x > 0 ? (x-m)*(y-m) : 0; })
    for (int b = 0; b < n; b += 64) {
        const double v = b + lane < n ? avg[b + lane] : -1.0;
        const double t = v > 0 ? (v - cloud_mean) * (v - cloud_mean) : 0.0;  // per element, then folded in order
#pragma unroll
        for (int k = 0; k < 64; ++k) sq_sum = sq_sum + rl(t, k);
    }
    const double std_dev = sqrt(sq_sum / (double)(valid - 1));
    const double thr = cloud_mean + std_ratio * std_dev;
    if (lane == 0) {
        stats[0] = cloud_mean;
        stats[1] = std_dev;
        stats[2] = thr;
        stats[3] = (double)valid;
    }
}

__global__ void sor_flag_kernel(const double* __restrict__ avg, int n, const double* __restrict__ stats,
                                unsigned char* __restrict__ flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double a = avg[i];
    flag[i] = (stats[3] > 0.0 && a > 0 && a < stats[2]) ? 1 : 0;
}

hipError_t launch_sor_select(const double* avg, int64_t n, double std_ratio, double* stats, unsigned char* flag,
                             int32_t* kept, int32_t* nkept, DevBuf<unsigned char>& tmp, hipStream_t s) {
    sor_stats_kernel<<<1, 64, 0, s>>>(avg, (int)n, std_ratio, stats);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    sor_flag_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(avg, (int)n, stats, flag);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t bytes = 0;
    if ((e = hipcub::DeviceSelect::Flagged(nullptr, bytes, hipcub::CountingInputIterator<int32_t>(0), flag, kept,
                                           nkept, (int)n, s)) != hipSuccess)
        return e;
    if ((e = tmp.ensure(bytes)) != hipSuccess) return e;
    return hipcub::DeviceSelect::Flagged(tmp.p, bytes, hipcub::CountingInputIterator<int32_t>(0), flag, kept, nkept,
                                         (int)n, s);
}

// ---------------------------------------------------------------- voxel
constexpr int kVoxBits = 21;  // per axis: 2^21 cells

__global__ void voxel_key_kernel(const double* __restrict__ xyz, int n, double mx, double my, double mz, double vs,
                                 unsigned long long* __restrict__ key, int32_t* __restrict__ idx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // Eigen: ref_coord = (p - voxel_min_bound) / voxel_size, int(floor(.)) per axis
    const long long ix = (long long)floor((xyz[3 * i] - mx) / vs);
    const long long iy = (long long)floor((xyz[3 * i + 1] - my) / vs);
    const long long iz = (long long)floor((xyz[3 * i + 2] - mz) / vs);
    key[i] = ((unsigned long long)ix << (2 * kVoxBits)) | ((unsigned long long)iy << kVoxBits) |
             (unsigned long long)iz;
    idx[i] = i;
}

// one thread per voxel: sum of its points in input order / count
__global__ void voxel_mean_kernel(const double* __restrict__ xyz, const int32_t* __restrict__ sidx,
                                  const int32_t* __restrict__ start, const int32_t* __restrict__ count, int nvox,
                                  double* __restrict__ out) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nvox) return;
    const int b = start[v], c = count[v];
    double sx = 0.0, sy = 0.0, sz = 0.0;
    for (int k = 0; k < c; ++k) {
        const int i = sidx[b + k];
        sx = sx + xyz[3 * i];
        sy = sy + xyz[3 * i + 1];
        sz = sz + xyz[3 * i + 2];
    }
    const double dc = (double)c;
    out[3 * v] = sx / dc;
    out[3 * v + 1] = sy / dc;
    out[3 * v + 2] = sz / dc;
}

hipError_t launch_voxel_down_sample(const double* xyz, int64_t n, const double vmin[3], double vs, VoxelBufs& b,
                                    double* out, int64_t* nvox_out, hipStream_t s) {
    hipError_t e;
    const int N = (int)n;
    if ((e = b.key.ensure((size_t)2 * n)) != hipSuccess) return e;
    if ((e = b.idx.ensure((size_t)2 * n)) != hipSuccess) return e;
    if ((e = b.run.ensure((size_t)2 * n + 2)) != hipSuccess) return e;
    if ((e = b.ukey.ensure((size_t)n)) != hipSuccess) return e;
    unsigned long long *k0 = b.key.p, *k1 = b.key.p + n;
    int32_t *i0 = b.idx.p, *i1 = b.idx.p + n;
    int32_t *cnt = b.run.p, *start = b.run.p + n, *nrun = b.run.p + 2 * n;
    voxel_key_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(xyz, N, vmin[0], vmin[1], vmin[2], vs, k0, i0);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t t1 = 0, t2 = 0, t3 = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, t1, k0, k1, i0, i1, N, 0, 3 * kVoxBits, s)) != hipSuccess)
        return e;
    if ((e = hipcub::DeviceRunLengthEncode::Encode(nullptr, t2, k1, b.ukey.p, cnt, nrun, N, s)) != hipSuccess)
        return e;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, t3, cnt, start, N, s)) != hipSuccess) return e;
    if ((e = b.tmp.ensure(std::max(t1, std::max(t2, t3)))) != hipSuccess) return e;
    if ((e = hipcub::DeviceRadixSort::SortPairs(b.tmp.p, t1, k0, k1, i0, i1, N, 0, 3 * kVoxBits, s)) != hipSuccess)
        return e;
    if ((e = hipcub::DeviceRunLengthEncode::Encode(b.tmp.p, t2, k1, b.ukey.p, cnt, nrun, N, s)) != hipSuccess)
        return e;
    int32_t nv = 0;
    if ((e = d2h(&nv, nrun, 4, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    *nvox_out = nv;
    if (!out || nv == 0) return hipSuccess;
    if ((e = hipcub::DeviceScan::ExclusiveSum(b.tmp.p, t3, cnt, start, nv, s)) != hipSuccess) return e;
    voxel_mean_kernel<<<(unsigned)((nv + 255) / 256), 256, 0, s>>>(xyz, i1, start, cnt, nv, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------- FPS
constexpr int kFpsThreads = 1024;

struct FpsArgs {
    const double* xyz;                  // n x 3, input order
    int n, first, k, per_block;         // per_block = P * kFpsThreads
    int64_t* out;                       // k chosen indices
    double* bval;                       // 2 x gridDim.x published block maxima (by step parity)
    unsigned long long* btag;           // 2 x gridDim.x: index of the maximum
    unsigned* err;                      // [0] set when a wait exceeded its bound, [1] step counter
};

// (value, index) order of np.argmax: larger value, then lower index
__device__ __forceinline__ bool fps_better(double v, int i, double w, int j) { return v > w || (v == w && i < j); }

__device__ __forceinline__ void fps_wave_best(double& v, int& i) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double w = __shfl_xor(v, off, 64);
        const int j = __shfl_xor(i, off, 64);
        if (fps_better(w, j, v, i)) {
            v = w;
            i = j;
        }
    }
}

// block-wide best of (v, i); result valid in every thread
__device__ __forceinline__ void fps_block_best(double& v, int& i, double* sv, int* si) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    fps_wave_best(v, i);
    if (lane == 0) {
        sv[wid] = v;
        si[wid] = i;
    }
    __syncthreads();
    v = sv[0];
    i = si[0];
#pragma unroll
    for (int w = 1; w < kFpsThreads / 64; ++w)
        if (fps_better(sv[w], si[w], v, i)) {
            v = sv[w];
            i = si[w];
        }
    __syncthreads();
}

// Per step, block b publishes its maximum in slot (step & 1, b), then one
// agent-scope add on the step counter (release); thread 0 of every block
// waits for the counter to reach (step + 1) * G (acquire), and every block
// reduces the G published values itself.  Double buffering by step parity is
// safe: a block writes step s+2 only after every block has added for step
// s+1, i.e. finished reading step s.  Large blocks (1024 threads) keep G, the
// number of adders and of published values, small.  Waits are bounded.
template <int P>
__global__ __launch_bounds__(kFpsThreads) void fps_kernel(FpsArgs a) {
    __shared__ double sv[kFpsThreads / 64];
    __shared__ int si[kFpsThreads / 64];
    __shared__ int timed_out;
    const int G = gridDim.x;
    const int base = blockIdx.x * a.per_block + threadIdx.x;
    double px[P], py[P], pz[P], d[P];
#pragma unroll
    for (int s = 0; s < P; ++s) {
        const int i = base + s * kFpsThreads;
        const bool ok = i < a.n;
        px[s] = ok ? a.xyz[3 * i] : 0.0;
        py[s] = ok ? a.xyz[3 * i + 1] : 0.0;
        pz[s] = ok ? a.xyz[3 * i + 2] : 0.0;
        d[s] = ok ? 1e6 : -1.0;  // distances = np.ones((1, N)) * 1e6; padding never wins
    }
    if (threadIdx.x == 0) timed_out = 0;
    int cur = a.first;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.out[0] = cur;
    for (int step = 0; step + 1 < a.k; ++step) {
        const double cx = a.xyz[3 * cur], cy = a.xyz[3 * cur + 1], cz = a.xyz[3 * cur + 2];
        double bv = -2.0;
        int bi = 0x7fffffff;
#pragma unroll
        for (int s = 0; s < P; ++s) {
#pragma clang fp contract(off)
            const double dx = cx - px[s], dy = cy - py[s], dz = cz - pz[s];
            const double e = sqrt((dx * dx + dy * dy) + dz * dz);
            const int i = base + s * kFpsThreads;
            if (i < a.n) d[s] = e < d[s] ? e : d[s];
            if (fps_better(d[s], i, bv, bi)) {
                bv = d[s];
                bi = i;
            }
        }
        fps_block_best(bv, bi, sv, si);
        const int par = step & 1;
        if (threadIdx.x == 0) {
            __hip_atomic_store(&a.bval[par * G + blockIdx.x], bv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.btag[par * G + blockIdx.x], (unsigned long long)(unsigned)bi, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(a.err + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)(step + 1) * (unsigned)G;
            int spins = 0;
            while (__hip_atomic_load(a.err + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
                if (++spins > (1 << 22)) {  // a co-residency failure: give up loudly, never hang
                    timed_out = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        if (timed_out) {  // block-uniform (shared, after the barrier)
            if (threadIdx.x == 0) atomicExch(a.err, 1u);
            return;
        }
        bv = -2.0;
        bi = 0x7fffffff;
        for (int b = threadIdx.x; b < G; b += kFpsThreads) {
            const double w = __hip_atomic_load(&a.bval[par * G + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int j = (int)(unsigned)__hip_atomic_load(&a.btag[par * G + b], __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
            if (fps_better(w, j, bv, bi)) {
                bv = w;
                bi = j;
            }
        }
        fps_block_best(bv, bi, sv, si);
        cur = bi;
        if (blockIdx.x == 0 && threadIdx.x == 0) a.out[step + 1] = cur;
    }
}

int fps_points_per_thread(int64_t n, int max_blocks) {
    for (int P : {1, 2, 4, 8})
        if ((int64_t)P * kFpsThreads * max_blocks >= n) return P;
    return 0;
}

hipError_t launch_fps(const double* xyz, int64_t n, int first, int k, int max_blocks, int64_t* out, double* bval,
                      unsigned long long* btag, unsigned* err, hipStream_t s) {
    const int P = fps_points_per_thread(n, max_blocks);
    if (P == 0) return hipErrorInvalidValue;
    const int per_block = P * kFpsThreads;
    const int G = (int)((n + per_block - 1) / per_block);
    hipError_t e = hipMemsetAsync(err, 0, 2 * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    FpsArgs a{xyz, (int)n, first, k, per_block, out, bval, btag, err};
    void* args[] = {&a};
    const void* fn = nullptr;
    switch (P) {
        case 1: fn = (const void*)fps_kernel<1>; break;
        case 2: fn = (const void*)fps_kernel<2>; break;
        case 4: fn = (const void*)fps_kernel<4>; break;
        default: fn = (const void*)fps_kernel<8>; break;
    }
    return hipLaunchCooperativeKernel(fn, dim3((unsigned)G), dim3(kFpsThreads), args, 0, s);
}

int fps_max_blocks(int device) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fps_kernel<8>, kFpsThreads, 0) !=
        hipSuccess)
        return 0;
    return per_cu >= 1 ? cus : 0;  // one block per CU: every block co-resident
}

}  // namespace orpcd
