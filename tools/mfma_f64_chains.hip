#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int C>
__global__ __launch_bounds__(64) void k(int iters, double seed, double* out) {
    const int lane = threadIdx.x;
    double a = seed + lane, b = seed * 0.5 + lane;
    d4 acc[C];
#pragma unroll
    for (int q = 0; q < C; ++q) acc[q] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16 / C; ++r)
#pragma unroll
            for (int q = 0; q < C; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int q = 0; q < C; ++q) s += acc[q][0] + acc[q][3];
    out[blockIdx.x * 64 + lane] = s;
}
template <int C>
void run(int blocks, int iters, double* out, const char* what) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    k<C><<<blocks, 64>>>(iters / 8, 1.0, out);
    (void)hipEventRecord(e0); k<C><<<blocks, 64>>>(iters, 1.0, out); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
    const double per_simd = 16.0 * iters * blocks / 1024.0;  // MFMAs per SIMD
    printf("%s: %d chains per wave, %d waves: %.3f ms, %.1f cycles per MFMA per SIMD at 2.4 GHz\n", what, C, blocks, ms, ms * 1e-3 * 2.4e9 / per_simd);
}
int main() {
    double* out; if (hipMalloc(&out, 8192 * 64 * 8) != hipSuccess) return 1;
    const int it = 20000;
    run<1>(1024, it, out, "1/SIMD"); run<2>(1024, it, out, "1/SIMD"); run<4>(1024, it, out, "1/SIMD"); run<8>(1024, it, out, "1/SIMD"); run<16>(1024, it, out, "1/SIMD");
    run<4>(2048, it, out, "2/SIMD"); run<8>(2048, it, out, "2/SIMD"); run<4>(4096, it, out, "4/SIMD"); run<8>(4096, it, out, "4/SIMD");
    return 0;
}
