// solve_bench.hip — cycle breakdown of the per-start 6x6 solve (det6, LDLT,
// pose update) on one lane, as icp_solve_kernel runs it.  A measurement tool,
// not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -I multi-scale-pointcloud-registration_amd/csrc \
//         tools/solve_bench.hip -o tools/solve_bench && ./tools/solve_bench
#include <hip/hip_runtime.h>

#include <cstdio>

#include "device_math.h"

using namespace orpcd;

__global__ void solve_timing(const double* JTJin, const double* bin, double* out, unsigned long long* cyc) {
    if (threadIdx.x != 0) return;
    double JTJ[36], b[6], x[6], upd[16];
    for (int i = 0; i < 36; ++i) JTJ[i] = JTJin[i];
    for (int i = 0; i < 6; ++i) b[i] = bin[i];
    const unsigned long long t0 = __builtin_readcyclecounter();
    const double det = det6(JTJ);
    const unsigned long long t1 = __builtin_readcyclecounter() + (det == 1.2345 ? 1 : 0);
    ldlt_solve6(JTJ, b, x);
    const unsigned long long t2 = __builtin_readcyclecounter() + (x[0] == 1.2345 ? 1 : 0);
    vec6_to_m4(x, upd);
    const unsigned long long t3 = __builtin_readcyclecounter() + (upd[0] == 1.2345 ? 1 : 0);
    for (int i = 0; i < 16; ++i) out[i] = upd[i];
    out[16] = det;
    cyc[0] = t1 - t0;
    cyc[1] = t2 - t1;
    cyc[2] = t3 - t2;
}

int main() {
    double hA[36], hb[6];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) hA[6 * i + j] = (i == j ? 10.0 + i : 0.0) + 0.1 * (i + j) / (1 + i * j);
    for (int i = 0; i < 6; ++i) hb[i] = 0.01 * (i + 1);
    double *dA, *db, *dout;
    unsigned long long* dc;
    hipMalloc(&dA, sizeof(hA));
    hipMalloc(&db, sizeof(hb));
    hipMalloc(&dout, 17 * 8);
    hipMalloc(&dc, 3 * 8);
    hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
    unsigned long long c[3];
    for (int rep = 0; rep < 3; ++rep) {
        solve_timing<<<1, 64>>>(dA, db, dout, dc);
        hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
        printf("det6 %llu  ldlt %llu  vec6_to_m4 %llu cycles (s_memrealtime-free readcyclecounter)\n", c[0], c[1],
               c[2]);
    }
    return 0;
}
