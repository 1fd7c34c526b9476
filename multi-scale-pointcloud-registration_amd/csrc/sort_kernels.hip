// sort_kernels.hip — device-resident cloud layout: Morton order + 64-point tiles.
//
// Every cloud uploaded through the C-ABI is stored in Morton (Z-order) order
// so that (a) consecutive queries of a wave are spatially coherent under any
// rigid transform, and (b) each 64-point target tile has a tight AABB that the
// correspondence search can cull against.  The sort is a stable LSD radix
// sort (hipCUB), so points with identical coordinates keep their input order:
// scanning tiles in increasing order then still resolves exact ties to the
// lowest ORIGINAL index, the oracle's convention.
#include <hipcub/hipcub.hpp>

#include "orpcd_internal.h"

namespace orpcd {

__device__ __forceinline__ uint32_t spread10(uint32_t v) {
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ void morton_kernel(const double* __restrict__ xyz, int n, double lox, double loy, double loz,
                              double scale, uint32_t* __restrict__ code, int32_t* __restrict__ idx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    auto q = [scale](double v, double lo) {
        double s = (v - lo) * scale;
        s = s < 0.0 ? 0.0 : (s > 1023.0 ? 1023.0 : s);
        return (uint32_t)s;
    };
    const uint32_t x = q(xyz[3 * i], lox), y = q(xyz[3 * i + 1], loy), z = q(xyz[3 * i + 2], loz);
    code[i] = (spread10(x) << 2) | (spread10(y) << 1) | spread10(z);
    idx[i] = i;
}

// out64[k] = in64[perm[k]], out4[k] = (float (xyz - origin), orig index bits);
// padding far.
// blockIdx.y: cloud y of a batch of rigid copies sharing one Morton order
// (orgs: its origin; in64 / out64 at y 3n, out4 at y npad); one cloud: y = 0.
__global__ void gather_points_kernel(const double* __restrict__ in64, const int32_t* __restrict__ perm, int n,
                                     int npad, double ox, double oy, double oz, double* __restrict__ out64,
                                     float4* __restrict__ out4, const double* __restrict__ orgs) {
    if (orgs) {
        ox = orgs[3 * blockIdx.y];
        oy = orgs[3 * blockIdx.y + 1];
        oz = orgs[3 * blockIdx.y + 2];
    }
    in64 += (size_t)blockIdx.y * 3 * n;
    out64 += (size_t)blockIdx.y * 3 * n;
    if (out4) out4 += (size_t)blockIdx.y * npad;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= npad) return;
    if (k < n) {
        const int j = perm[k];
        const double x = in64[3 * j], y = in64[3 * j + 1], z = in64[3 * j + 2];
        out64[3 * k] = x;
        out64[3 * k + 1] = y;
        out64[3 * k + 2] = z;
        if (out4) out4[k] = make_float4((float)(x - ox), (float)(y - oy), (float)(z - oz), __int_as_float(j));
    } else if (out4) {
        out4[k] = make_float4(kFarCoord, kFarCoord, kFarCoord, __int_as_float(-1));
    }
}

// One thread per 64-point tile: fp32 AABB over the tile's real points, and
// the AABBs of its kNQ kQuarter-point quarters (qbox[2 kNQ t + k] = lo of quarter k,
// qbox[2 kNQ t + kNQ + k] = hi; a quarter without real points gets a point box at 3e38).
__global__ void tile_aabb_kernel(const float4* __restrict__ p4, int n, int ntiles, float4* __restrict__ lo,
                                 float4* __restrict__ hi, float4* __restrict__ qbox) {
    p4 += (size_t)blockIdx.y * ntiles * kTile;  // cloud y of a batch (npad = ntiles x 64)
    lo += (size_t)blockIdx.y * ntiles;
    hi += (size_t)blockIdx.y * ntiles;
    qbox += (size_t)blockIdx.y * ntiles * 2 * kNQ;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    float mnx = 3.0e38f, mny = 3.0e38f, mnz = 3.0e38f, mxx = -3.0e38f, mxy = -3.0e38f, mxz = -3.0e38f;
    for (int q = 0; q < kNQ; ++q) {
        float ax = 3.0e38f, ay = 3.0e38f, az = 3.0e38f, bx = -3.0e38f, by = -3.0e38f, bz = -3.0e38f;
        const int beg = t * kTile + q * kQuarter, end = min(n, beg + kQuarter);
        for (int k = beg; k < end; ++k) {
            const float4 p = p4[k];
            ax = fminf(ax, p.x);
            ay = fminf(ay, p.y);
            az = fminf(az, p.z);
            bx = fmaxf(bx, p.x);
            by = fmaxf(by, p.y);
            bz = fmaxf(bz, p.z);
        }
        // a quarter without points: the point box (3e38, 3e38, 3e38), whose
        // clamped distance (box_d2_2q) overflows to inf for any query
        const bool empty = end <= beg;
        qbox[2 * kNQ * (size_t)t + q] = empty ? make_float4(3.0e38f, 3.0e38f, 3.0e38f, 0.f) : make_float4(ax, ay, az, 0.f);
        qbox[2 * kNQ * (size_t)t + kNQ + q] = empty ? make_float4(3.0e38f, 3.0e38f, 3.0e38f, 0.f) : make_float4(bx, by, bz, 0.f);
        mnx = fminf(mnx, ax);
        mny = fminf(mny, ay);
        mnz = fminf(mnz, az);
        mxx = fmaxf(mxx, bx);
        mxy = fmaxf(mxy, by);
        mxz = fmaxf(mxz, bz);
    }
    lo[t] = make_float4(mnx, mny, mnz, 0.f);
    hi[t] = make_float4(mxx, mxy, mxz, 0.f);
}

// One thread per super-tile (64 tiles): AABB of the tile AABBs.
__global__ void super_aabb_kernel(const float4* __restrict__ tlo, const float4* __restrict__ thi, int ntiles,
                                  int nsuper, float4* __restrict__ slo, float4* __restrict__ shi) {
    tlo += (size_t)blockIdx.y * ntiles;  // cloud y of a batch
    thi += (size_t)blockIdx.y * ntiles;
    slo += (size_t)blockIdx.y * nsuper;
    shi += (size_t)blockIdx.y * nsuper;
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nsuper) return;
    float4 lo = make_float4(3.0e38f, 3.0e38f, 3.0e38f, 0.f), hi = make_float4(-3.0e38f, -3.0e38f, -3.0e38f, 0.f);
    const int end = min(ntiles, (u + 1) * kSuper);
    for (int t = u * kSuper; t < end; ++t) {
        const float4 a = tlo[t], b = thi[t];
        lo.x = fminf(lo.x, a.x);
        lo.y = fminf(lo.y, a.y);
        lo.z = fminf(lo.z, a.z);
        hi.x = fmaxf(hi.x, b.x);
        hi.y = fmaxf(hi.y, b.y);
        hi.z = fmaxf(hi.z, b.z);
    }
    slo[u] = lo;
    shi[u] = hi;
}

// out[k] = in[offset + idx[k]] (rows of w doubles)
__global__ void gather_rows_kernel(const double* __restrict__ in, const int32_t* __restrict__ idx, int64_t offset,
                                   int n, int w, double* __restrict__ out) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double* r = in + (size_t)(offset + idx[k]) * w;
    for (int c = 0; c < w; ++c) out[(size_t)k * w + c] = r[c];
}

hipError_t launch_gather_rows(const double* in, const int32_t* idx, int64_t offset, int64_t n, int w, double* out,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    gather_rows_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(in, idx, offset, (int)n, w, out);
    return hipGetLastError();
}

hipError_t launch_morton(const double* xyz, int64_t n, const double lo[3], double scale, uint32_t* code,
                         int32_t* idx, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    morton_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(xyz, (int)n, lo[0], lo[1], lo[2], scale, code, idx);
    return hipGetLastError();
}

// Every buffer a kernel loads whole tiles of holds the padded tiles (the
// round-5 fault was a whole-tile load past an n-point buffer): checked on the
// host after each layout build, always on (a few integer compares).
static hipError_t check_layout_sizes(const char* what, size_t copies, size_t n, size_t npad, size_t ntiles,
                                     size_t nsuper, size_t xyz64, size_t p4, size_t tlo, size_t thi, size_t qbox,
                                     size_t slo, size_t shi, bool xyz_padded) {
    const bool ok = npad == std::max<size_t>(kTile, ntiles * kTile) && npad >= n &&
                    xyz64 >= copies * 3 * (xyz_padded ? npad : n) && (p4 == 0 || (p4 >= copies * npad &&
                    tlo >= copies * ntiles && thi >= copies * ntiles && qbox >= copies * ntiles * 2 * kNQ &&
                    slo >= copies * nsuper && shi >= copies * nsuper));
    if (!ok) fprintf(stderr, "[orpcd] %s: layout buffers smaller than the padded tiles\n", what);
    return ok ? hipSuccess : hipErrorInvalidValue;
}

hipError_t build_layout(const double* dev_in64, int64_t n, const double bbox_lo[3], double bbox_ext,
                        const double origin[3], CloudLayout& L, bool with_tiles, hipStream_t s) {
    L.n = n;
    for (int a = 0; a < 3; ++a) L.org[a] = origin[a];
    L.npad = std::max<int64_t>(kTile, ((n + kTile - 1) / kTile) * kTile);
    L.ntiles = (n + kTile - 1) / kTile;
    hipError_t e;
    // xyz64 is sized to the padded tiles (its padding is never written nor
    // used): a kernel that loads a whole tile's fp64 points before testing
    // which lanes are real then stays inside the allocation
    if ((e = L.xyz64.ensure((size_t)L.npad * 3)) != hipSuccess) return e;
    if ((e = L.perm.ensure((size_t)n)) != hipSuccess) return e;
    if ((e = L.codes.ensure((size_t)n * 2)) != hipSuccess) return e;
    if ((e = L.ids.ensure((size_t)n)) != hipSuccess) return e;
    if (with_tiles) {
        if ((e = L.p4.ensure((size_t)L.npad)) != hipSuccess) return e;
        if ((e = L.tlo.ensure((size_t)L.ntiles)) != hipSuccess) return e;
        if ((e = L.thi.ensure((size_t)L.ntiles)) != hipSuccess) return e;
        if ((e = L.qbox.ensure((size_t)L.ntiles * 2 * kNQ)) != hipSuccess) return e;
        L.nsuper = (L.ntiles + kSuper - 1) / kSuper;
        if ((e = L.slo.ensure((size_t)L.nsuper)) != hipSuccess) return e;
        if ((e = L.shi.ensure((size_t)L.nsuper)) != hipSuccess) return e;
    }
    const double scale = bbox_ext > 0 ? 1023.0 / bbox_ext : 0.0;
    const unsigned g = (unsigned)((n + 255) / 256);
    morton_kernel<<<g, 256, 0, s>>>(dev_in64, (int)n, bbox_lo[0], bbox_lo[1], bbox_lo[2], scale, L.codes.p, L.ids.p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tmp = 0;
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, L.codes.p, L.codes.p + n, L.ids.p, L.perm.p, (int)n, 0, 30,
                                           s);
    if (e != hipSuccess) return e;
    if ((e = L.sort_tmp.ensure(tmp)) != hipSuccess) return e;
    e = hipcub::DeviceRadixSort::SortPairs(L.sort_tmp.p, tmp, L.codes.p, L.codes.p + n, L.ids.p, L.perm.p, (int)n, 0,
                                           30, s);
    if (e != hipSuccess) return e;
    const unsigned gp = (unsigned)((L.npad + 255) / 256);
    gather_points_kernel<<<gp, 256, 0, s>>>(dev_in64, L.perm.p, (int)n, (int)L.npad, origin[0], origin[1],
                                            origin[2], L.xyz64.p, with_tiles ? L.p4.p : nullptr, nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (with_tiles) {
        tile_aabb_kernel<<<(unsigned)((L.ntiles + 255) / 256), 256, 0, s>>>(L.p4.p, (int)n, (int)L.ntiles, L.tlo.p,
                                                                           L.thi.p, L.qbox.p);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        super_aabb_kernel<<<(unsigned)((L.nsuper + 255) / 256), 256, 0, s>>>(L.tlo.p, L.thi.p, (int)L.ntiles,
                                                                            (int)L.nsuper, L.slo.p, L.shi.p);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return check_layout_sizes("build_layout", 1, (size_t)n, (size_t)L.npad, (size_t)L.ntiles, (size_t)L.nsuper,
                              L.xyz64.n, with_tiles ? L.p4.n : 0, L.tlo.n, L.thi.n, L.qbox.n, L.slo.n, L.shi.n, true);
}

// B rigid copies (input order, B x n x 3 at in64) laid out in the Morton
// order `perm` of their common base cloud (BatchLayout): a rigid motion keeps
// Morton neighbours spatially coherent, and the culled searches' answers do
// not depend on the order, only their speed.  Per copy its own fp32 frame
// (orgs, B x 3 on the device), tiles and super-tiles.
hipError_t build_batch_layout(const double* in64, int64_t n, int B, const int32_t* perm, const double* orgs,
                              BatchLayout& L, hipStream_t s) {
    L.n = n;
    L.B = B;
    L.npad = std::max<int64_t>(kTile, ((n + kTile - 1) / kTile) * kTile);
    L.ntiles = (n + kTile - 1) / kTile;
    L.nsuper = (L.ntiles + kSuper - 1) / kSuper;
    hipError_t e;
    if ((e = L.xyz64.ensure((size_t)B * n * 3)) != hipSuccess) return e;
    if ((e = L.p4.ensure((size_t)B * L.npad)) != hipSuccess) return e;
    if ((e = L.tlo.ensure((size_t)B * L.ntiles)) != hipSuccess) return e;
    if ((e = L.thi.ensure((size_t)B * L.ntiles)) != hipSuccess) return e;
    if ((e = L.qbox.ensure((size_t)B * L.ntiles * 2 * kNQ)) != hipSuccess) return e;
    if ((e = L.slo.ensure((size_t)B * L.nsuper)) != hipSuccess) return e;
    if ((e = L.shi.ensure((size_t)B * L.nsuper)) != hipSuccess) return e;
    gather_points_kernel<<<dim3((unsigned)((L.npad + 255) / 256), (unsigned)B), 256, 0, s>>>(
        in64, perm, (int)n, (int)L.npad, 0.0, 0.0, 0.0, L.xyz64.p, L.p4.p, orgs);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tile_aabb_kernel<<<dim3((unsigned)((L.ntiles + 255) / 256), (unsigned)B), 256, 0, s>>>(
        L.p4.p, (int)n, (int)L.ntiles, L.tlo.p, L.thi.p, L.qbox.p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    super_aabb_kernel<<<dim3((unsigned)((L.nsuper + 255) / 256), (unsigned)B), 256, 0, s>>>(
        L.tlo.p, L.thi.p, (int)L.ntiles, (int)L.nsuper, L.slo.p, L.shi.p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the copies' fp64 points are n each (no whole-tile fp64 loads on them:
    // the batched KNN tests k < n before every load)
    return check_layout_sizes("build_batch_layout", (size_t)B, (size_t)n, (size_t)L.npad, (size_t)L.ntiles,
                              (size_t)L.nsuper, L.xyz64.n, L.p4.n, L.tlo.n, L.thi.n, L.qbox.n, L.slo.n, L.shi.n, false);
}

// this unit's code object loaded now (orpcd_ctx_create), not at its first launch
hipError_t preload_code_object_sort() {
    hipFuncAttributes attr;
    return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&morton_kernel));
}

}  // namespace orpcd
