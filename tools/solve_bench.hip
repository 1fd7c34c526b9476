// solve_bench.hip — cycle breakdown of the per-start solve as icp_solve_kernel
// runs it: the 29 fixed-order wave reductions of the block partials, the
// single-lane det6 / LDLT / pose update, and their wave-parallel versions.
// A measurement tool, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -I multi-scale-pointcloud-registration_amd/csrc \
//         tools/solve_bench.hip -o tools/solve_bench && ./tools/solve_bench
#include <hip/hip_runtime.h>

#include <cstdio>

#include "device_math.h"

using namespace orpcd;

#define CLK(v) (__builtin_readcyclecounter() + ((v) == 1.2345 ? 1 : 0))

template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, Ctrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), Ctrl, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_fixed(double v) {  // as gicp_kernels.hip
    v += dpp_f64<0xb1>(v);
    v += dpp_f64<0x4e>(v);
    v += dpp_f64<0x141>(v);
    v += dpp_f64<0x140>(v);
    return (rl64(v, 0) + rl64(v, 16)) + (rl64(v, 32) + rl64(v, 48));
}

__global__ void solve_timing(const double* sums, double* out, unsigned long long* cyc) {
    const int lane = threadIdx.x;
    double s[29];
    for (int v = 0; v < 29; ++v) s[v] = sums[v] * (1.0 + lane * 1e-3);
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int v = 0; v < 29; ++v) s[v] = wave_sum_fixed(s[v]);
    const unsigned long long t1 = CLK(s[28] + s[0]);
    // single lane (lane 0 computes, as the round-1 kernel)
    double JTJ[36], b[6], x[6], upd[16], det = 0;
    unsigned long long c[8] = {};
    if (lane == 0) {
        for (int i = 0, k = 0; i < 6; ++i)
            for (int j = i; j < 6; ++j, ++k) JTJ[6 * i + j] = JTJ[6 * j + i] = s[k];
        for (int i = 0; i < 6; ++i) b[i] = -s[21 + i];
        const unsigned long long a0 = __builtin_readcyclecounter();
        det = det6(JTJ);
        const unsigned long long a1 = CLK(det);
        ldlt_solve6(JTJ, b, x);
        const unsigned long long a2 = CLK(x[0]);
        vec6_to_m4(x, upd);
        const unsigned long long a3 = CLK(upd[0]);
        c[0] = a1 - a0;
        c[1] = a2 - a1;
        c[2] = a3 - a2;
    }
    // wave
    double row[6], bw[6], xw[6], uw[16];
    const unsigned long long w0 = __builtin_readcyclecounter();
    sym6_row(s, lane, row);
    for (int r = 0; r < 6; ++r) bw[r] = -s[21 + r];
    const double dw = det6_wave(row, lane);
    const unsigned long long w1 = CLK(dw);
    ldlt_solve6_wave(row, bw, xw, lane);
    const unsigned long long w2 = CLK(xw[0]);
    vec6_to_m4_wave(xw, uw, lane);
    const unsigned long long w3 = CLK(uw[0]);
    if (lane == 0) {
        for (int i = 0; i < 16; ++i) out[i] = upd[i] - uw[i];
        out[16] = det - dw;
        cyc[0] = t1 - t0;
        cyc[1] = c[0];
        cyc[2] = c[1];
        cyc[3] = c[2];
        cyc[4] = w1 - w0;
        cyc[5] = w2 - w1;
        cyc[6] = w3 - w2;
    }
}

__global__ void empty_kernel() {}
__global__ void chain_kernel(const int* __restrict__ idx, const double* __restrict__ v, double* out, int hops) {
    int i = idx[blockIdx.x];  // dependent loads: the per-hop memory latency inside a kernel
    for (int h = 0; h < hops; ++h) i = idx[i & 1023];
    if (threadIdx.x == 0) out[blockIdx.x] = v[i & 1023];
}

int main() {
    double hs[29];
    double A[6][6], hb[6];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) A[i][j] = (i == j ? 10.0 + i : 0.0) + 0.1 * (i + j) / (1 + i * j);
    for (int i = 0, k = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j, ++k) hs[k] = A[i][j];
    for (int i = 0; i < 6; ++i) hs[21 + i] = 0.01 * (i + 1);
    hs[27] = 1.0;
    hs[28] = 100.0;
    double *ds, *dout;
    unsigned long long* dc;
    hipMalloc(&ds, sizeof(hs));
    hipMalloc(&dout, 17 * 8);
    hipMalloc(&dc, 7 * 8);
    hipMemcpy(ds, hs, sizeof(hs), hipMemcpyHostToDevice);
    unsigned long long c[7];
    double o[17];
    for (int rep = 0; rep < 3; ++rep) {
        solve_timing<<<1, 64>>>(ds, dout, dc);
        hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
        hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
        printf("29 wave sums %llu | lane: det6 %llu ldlt %llu vec6_to_m4 %llu | wave: row+det %llu ldlt %llu "
               "vec6_to_m4 %llu cycles (max |serial - wave| %g)\n",
               c[0], c[1], c[2], c[3], c[4], c[5], c[6], [&] {
                   double m = 0;
                   for (double v : o) m = m > __builtin_fabs(v) ? m : __builtin_fabs(v);
                   return m;
               }());
    }
    int* didx;
    double* dv;
    hipMalloc(&didx, 1024 * 4);
    hipMalloc(&dv, 1024 * 8);
    hipMemset(didx, 0, 1024 * 4);
    hipMemset(dv, 0, 1024 * 8);
    for (int r = 0; r < 200; ++r) empty_kernel<<<1, 64>>>();
    for (int r = 0; r < 200; ++r) chain_kernel<<<8, 64>>>(didx, dv, dout, 0);
    for (int r = 0; r < 200; ++r) chain_kernel<<<8, 64>>>(didx, dv, dout, 8);
    hipDeviceSynchronize();
    return 0;
}
