// Does fp64 VALU work overlap v_mfma_f64_16x16x4_f64 on gfx950?  (DESIGN.md §5,
// "Round 4: the FGR path".)  One wave per SIMD, every CU: per loop iteration a
// wave issues kM MFMAs on four independent accumulators, and/or kV fp64 VALU
// operations (v_add_f64 / v_max_f64 chains on registers the MFMAs do not touch).
//   mode 0: MFMAs only;  mode 1: VALU only;  mode 2: both, interleaved;
//   mode 3: two waves per SIMD, even blocks MFMAs only and odd blocks VALU only.
// If the fp64 VALU shares the MFMA's double-precision datapath, t(2) ~ t(0) + t(1);
// if it issues beside the matrix pipe, t(2) ~ max(t(0), t(1)).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_f64_overlap.hip -o tools/mfma_f64_overlap
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int kMode, int kV>
__global__ __launch_bounds__(64) void overlap_kernel(int iters, double seed, double* out) {
    const int lane = threadIdx.x;
    const int mode = kMode == 3 ? (blockIdx.x & 1) : kMode;  // mode 3: even blocks MFMA, odd VALU
    double a = seed + lane, b = seed * 0.5 + lane;
    d4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = seed * (k + 1) + lane;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            if (mode == 0 || mode == 2) {
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
            }
            if (mode == 1 || mode == 2) {
#pragma unroll
                for (int k = 0; k < kV; ++k) {
                    const int j = k & 7;
                    // alternate add / max so neither folds away; eight independent chains
                    if (k & 1)
                        asm volatile("v_max_f64 %0, %0, %1" : "+v"(v[j]) : "v"(a));
                    else
                        asm volatile("v_add_f64 %0, %0, %1" : "+v"(v[j]) : "v"(b));
                }
            }
        }
    }
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
    out[blockIdx.x * 64 + lane] = s;
}

template <int kMode, int kV>
float run(int blocks, int iters, double* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    overlap_kernel<kMode, kV><<<blocks, 64>>>(iters / 8, 1.0, out);  // warm-up
    (void)hipEventRecord(e0);
    overlap_kernel<kMode, kV><<<blocks, 64>>>(iters, 1.0, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms;
}

template <int kV>
void row(int blocks, int iters, double* out) {
    const float m = run<0, kV>(blocks, iters, out), v = run<1, kV>(blocks, iters, out), b = run<2, kV>(blocks, iters, out);
    const float two = run<3, kV>(2 * blocks, iters, out), m2 = run<0, kV>(2 * blocks, iters, out);
    printf("  two waves per SIMD: MFMA + MFMA %.3f ms, MFMA wave beside a VALU wave %.3f ms "
           "(-> / (mfma + valu) = %.2f, / max = %.2f)\n", m2, two, two / (m + v), two / (m > v ? m : v));
    const double mfmas = 8.0 * iters * blocks;  // per wave 8 MFMAs an iteration
    printf("VALU per 4 MFMAs %3d: mfma %.3f ms (%.1f cyc/MFMA at 2.4 GHz per SIMD), valu %.3f ms, both %.3f ms  "
           "-> both / (mfma + valu) = %.2f, both / max = %.2f\n",
           kV, m, m * 1e-3 * 2.4e9 / (mfmas / blocks), v, b, b / (m + v), b / (m > v ? m : v));
}

int main() {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = 4 * cus;  // one wave per SIMD
    double* out = nullptr;
    if (hipMalloc(&out, (size_t)blocks * 64 * sizeof(double)) != hipSuccess) return 1;
    const int iters = 20000;
    printf("%d CUs, %d one-wave blocks, %d iterations of 8 MFMAs\n", cus, blocks, iters);
    row<4>(blocks, iters, out);
    row<8>(blocks, iters, out);
    row<16>(blocks, iters, out);
    row<32>(blocks, iters, out);
    (void)hipFree(out);
    return 0;
}
