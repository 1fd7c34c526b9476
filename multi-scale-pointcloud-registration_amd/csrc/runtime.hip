// runtime.hip — the C-ABI (include/orpcd.h): context, device-resident clouds
// and the batched GICP driver.  Host orchestration only; all arithmetic on
// the hot path runs in the kernels of knn_kernels.hip / gicp_kernels.hip.
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <random>
#include <utility>

#include <rccl/rccl.h>  // types only: librccl is loaded at run time (rccl_api)

#include "orpcd_internal.h"

using namespace orpcd;


#define CTX_CHECK(ctx, call)                                                                          \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess) {                                                                       \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);                           \
            return ORPCD_EDEVICE;                                                                     \
        }                                                                                             \
    } while (0)

#define CTX_REQUIRE(ctx, cond, msg)   \
    do {                              \
        if (!(cond)) {                \
            (ctx)->err = (msg);       \
            return ORPCD_EINVAL;      \
        }                             \
    } while (0)

namespace {

// Every coordinate finite, and the bounding box: one pass over the cloud,
// split over host threads for large clouds (C5's 1M points: 3.5 -> 0.6 ms).
struct CloudScan {
    bool finite = true;
    double lo[3] = {0.0, 0.0, 0.0}, hi[3] = {0.0, 0.0, 0.0};
};
CloudScan scan_cloud(const double* xyz, int64_t n) {
    CloudScan r;
    if (n <= 0) return r;
    constexpr int64_t kChunk = 1 << 16;
    const int nch = (int)((n + kChunk - 1) / kChunk);
    std::vector<CloudScan> part((size_t)nch);
    host_parallel(nch, [&](int ch) {
        CloudScan& p = part[(size_t)ch];
        const int64_t i0 = ch * kChunk, i1 = std::min(n, i0 + kChunk);
        bool fin = true;
        double lo[3] = {xyz[3 * i0], xyz[3 * i0 + 1], xyz[3 * i0 + 2]}, hi[3] = {lo[0], lo[1], lo[2]};
        for (int64_t i = i0; i < i1; ++i)
            for (int a = 0; a < 3; ++a) {
                const double v = xyz[3 * i + a];
                fin &= std::isfinite(v);
                lo[a] = std::min(lo[a], v);
                hi[a] = std::max(hi[a], v);
            }
        p.finite = fin;
        for (int a = 0; a < 3; ++a) {
            p.lo[a] = lo[a];
            p.hi[a] = hi[a];
        }
    });
    r = part[0];
    for (const CloudScan& p : part) {
        r.finite &= p.finite;
        for (int a = 0; a < 3; ++a) {
            r.lo[a] = std::min(r.lo[a], p.lo[a]);
            r.hi[a] = std::max(r.hi[a], p.hi[a]);
        }
    }
    return r;
}

bool finite_cloud(const double* xyz, int64_t n) { return scan_cloud(xyz, n).finite; }

// Feature rows the matrix-core search can order: finite entries and a squared
// norm <= 1e150, so every expansion |q|^2 + |t|^2 - 2 q.t stays finite and far
// below the padded rows' kPadNorm (1e300); a larger row would give an inf
// distance whose index-carrying key is a NaN (FPFH rows are histograms
// normalised to 100 per bin group: |f|^2 <= 3e4).
bool feature_rows_ok(const double* f, int64_t rows, int dim) {
    for (int64_t r = 0; r < rows; ++r) {
        double n2 = 0.0;
        for (int k = 0; k < dim; ++k) {
            const double v = f[r * dim + k];
            if (!std::isfinite(v)) return false;
            n2 += v * v;
        }
        if (!(n2 <= 1e150)) return false;
    }
    return true;
}

void host_bbox(const double* xyz, int64_t n, double lo[3], double hi[3], double* ext) {
    const CloudScan r = scan_cloud(xyz, n);  // min / max are exact: the same box in any order
    for (int a = 0; a < 3; ++a) {
        lo[a] = r.lo[a];
        hi[a] = r.hi[a];
    }
    *ext = std::max(hi[0] - lo[0], std::max(hi[1] - lo[1], hi[2] - lo[2]));
}

// Absolute bound (with 4x safety) on the fp32 rounding of any coordinate of
// the cloud in its fp32 frame (relative to `org`): the culled KNN widens its
// fp32 box tests by it.
double coord_margin(const double lo[3], const double hi[3], const double org[3]) {
    double m = 0.0;
    for (int a = 0; a < 3; ++a) m = std::max(m, std::max(std::fabs(lo[a] - org[a]), std::fabs(hi[a] - org[a])));
    return m * 0x1p-21;
}

// ORPCD_SETUP_TRACE=1: the set-up phases of set_target / set_source on
// stderr (each mark drains the stream first: the phases' own times)
struct SetupTrace {
    bool on = getenv("ORPCD_SETUP_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void mark(hipStream_t s, const char* what) {
        if (!on) return;
        (void)hipStreamSynchronize(s);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[orpcd setup] %-28s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    }
};
thread_local SetupTrace* g_setup_trace = nullptr;
static void setup_mark(hipStream_t s, const char* what) {
    if (g_setup_trace) g_setup_trace->mark(s, what);
}

// Lay out a device-resident (input-order) cloud in Morton order with tiles;
// its fp32 frame is centred on the bounding box (CloudLayout::org).
int layout_from_device(orpcd_ctx* c, const double* host_xyz, const double* dev_xyz, int64_t n, CloudLayout& L,
                       bool tiles, double* margin = nullptr) {
    double lo[3], hi[3], org[3], ext;
    host_bbox(host_xyz, n, lo, hi, &ext);
    setup_mark(c->stream, "upload + host bbox");
    for (int a = 0; a < 3; ++a) {
        org[a] = 0.5 * (lo[a] + hi[a]);
        L.lo[a] = lo[a];
        L.hi[a] = hi[a];
    }
    if (margin) *margin = coord_margin(lo, hi, org);
    CTX_CHECK(c, build_layout(dev_xyz, n, lo, ext, org, L, tiles, c->stream));
    setup_mark(c->stream, "Morton layout");
    return ORPCD_OK;
}

// Upload a cloud (input order, kept in scratch64a) and lay it out in Morton
// order on device.
int upload_layout(orpcd_ctx* c, const double* xyz, int64_t n, CloudLayout& L, bool tiles, double* margin = nullptr) {
    CTX_CHECK(c, c->scratch64a.ensure((size_t)n * 3));
    CTX_CHECK(c, h2d(c->scratch64a.p, xyz, (size_t)n * 24, c->stream));
    return layout_from_device(c, xyz, c->scratch64a.p, n, L, tiles, margin);
}

// The KNN kernel for a cloud of n points: lane-per-query (knn_tiles_kernel)
// from knn_lane_min points on, where its n / 256 workgroups fill the chip (C5
// target, 1M points: 8.0 -> 5.5 ms per set-up, profiles/r05_c5_jfa*.json);
// wave-per-query below.  Both return the same exact neighbour lists.
bool knn_lane(const orpcd_ctx* c, int64_t n) { return c->opt.knn_lane_min > 0 && n >= c->opt.knn_lane_min; }

// Target k: Morton layout + tiles + GICP covariances (KNN-20 normals), and
// its device descriptor (TargetDesc, read by the kernels of every batch).
int upload_target_k(orpcd_ctx* c, int k, const double* xyz, int64_t m, double eps) {
    double margin = 0.0;
    int rc = upload_layout(c, xyz, m, c->tgts[k], true, &margin);
    if (rc) return rc;
    CTX_CHECK(c, prepare_seed_grid(c->tgts[k]));  // built by launch_seed_grids once the descriptor is up
    CTX_CHECK(c, c->tcovs[k].ensure((size_t)m * kCovW));
    CTX_CHECK(c, c->scratch64b.ensure((size_t)m * 6));
    if (eps >= 0.0) {
        CTX_CHECK(c, launch_knn_tiles(c->tgts[k], c->scratch64a.p, 20, -1.0, margin, false, c->scratch64b.p, nullptr,
                                      nullptr, nullptr, c->stream, nullptr, knn_lane(c, m)));
        CTX_CHECK(c, launch_normals_cov(c->scratch64b.p, m, nullptr, 1, eps, nullptr,
                                        ORPCD_NORMAL_COV ? nullptr : c->tcovs[k].p, c->stream,
                                        ORPCD_NORMAL_COV ? c->tcovs[k].p : nullptr));
    }
    c->tgt_eps[k] = eps;
    // no host copy of the points: another epsilon rebuilds them from the
    // device layout (targets_for_epsilon); a 1M-point copy cost ~1 ms per set-up
    c->tgt_host[k].clear();
    setup_mark(c->stream, "KNN-20 covariances");
    CTX_CHECK(c, c->tdesc.ensure(kMaxTargets));
    write_target_desc(c->tgts[k], c->tcovs[k].p, c->opt.seed_reps, c->opt.seed_grid != 0, c->tdesc_h[k]);
    CTX_CHECK(c, h2d(c->tdesc.p + k, &c->tdesc_h[k], sizeof(TargetDesc), c->stream));
    return ORPCD_OK;
}

// the seed grids of targets [first, first + count) (descriptors uploaded)
hipError_t seed_grids(orpcd_ctx* c, int first, int count) {
    unsigned long long* sgk[kMaxTargets];
    int64_t mx = 0;
    for (int k = 0; k < count; ++k) {
        sgk[k] = c->tgts[first + k].sgk.p;
        mx = std::max(mx, c->tgts[first + k].n);
    }
    return launch_seed_grids(c->tdesc.p, first, count, (int)mx, sgk, c->stream);
}

int upload_target(orpcd_ctx* c, const double* xyz, int64_t m, double eps) {
    int rc = upload_target_k(c, 0, xyz, m, eps);
    if (rc) return rc;
    CTX_CHECK(c, seed_grids(c, 0, 1));
    return ORPCD_OK;
}

// every target of the batch with covariances for `eps` (they depend on it)
int targets_for_epsilon(orpcd_ctx* c, int ntgt, double eps) {
    for (int k = 0; k < ntgt; ++k) {
        if (c->tgt_eps[k] == eps) continue;
        if (c->tgt_host[k].empty()) {
            // the input-order points from the layout's Morton-order fp64
            // points and permutation (the set-up keeps no host copy)
            const CloudLayout& L = c->tgts[k];
            std::vector<double> mz((size_t)L.n * 3);
            std::vector<int32_t> perm((size_t)L.n);
            CTX_CHECK(c, d2h(mz.data(), L.xyz64.p, mz.size() * 8, c->stream));
            CTX_CHECK(c, d2h(perm.data(), L.perm.p, perm.size() * 4, c->stream));
            CTX_CHECK(c, hipStreamSynchronize(c->stream));
            c->tgt_host[k].resize(mz.size());
            for (int64_t i = 0; i < L.n; ++i)
                for (int a = 0; a < 3; ++a) c->tgt_host[k][3 * (size_t)perm[(size_t)i] + a] = mz[3 * (size_t)i + a];
        }
        const std::vector<double> host = std::move(c->tgt_host[k]);
        int rc = upload_target_k(c, k, host.data(), c->tgts[k].n, eps);
        if (rc) return rc;
        CTX_CHECK(c, seed_grids(c, k, 1));
    }
    return ORPCD_OK;
}

// sum / max of the spread profiling counters (device -> host, synchronous on s)
hipError_t read_counters(orpcd_ctx* c, unsigned long long& tiles, unsigned long long& maxw, bool reset_max) {
    std::vector<unsigned long long> h((size_t)kCounterSlots * kCounterStride);
    hipError_t e = d2h(h.data(), c->counters.p, h.size() * 8, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return e;
    tiles = 0;
    maxw = 0;
    for (int i = 0; i < kCounterSlots; ++i) {
        tiles += h[(size_t)i * kCounterStride];
        maxw = std::max(maxw, h[(size_t)i * kCounterStride + 1]);
        if (reset_max) h[(size_t)i * kCounterStride + 1] = 0;
    }
    if (reset_max) e = h2d(c->counters.p, h.data(), h.size() * 8, c->stream);
    return e;
}

int check_fgr_params(orpcd_ctx* c, const orpcd_fgr_params* p) {
    CTX_REQUIRE(c, p->division_factor > 0 && p->tuple_scale > 0 && p->maximum_correspondence_distance > 0,
                "fgr: division_factor, tuple_scale and maximum_correspondence_distance must be > 0");
    CTX_REQUIRE(c, p->iteration_number > 0 && p->maximum_tuple_count > 0,
                "fgr: iteration_number and maximum_tuple_count must be > 0");
    return ORPCD_OK;
}

// estimate_normals(Hybrid(normal_radius, normal_knn)) + compute_fpfh_feature(
// Hybrid(fpfh_radius, fpfh_knn)) of the input-order cloud in fgr.xyz[k]
// (fastGlobalOptimizer.py:114-142).  Normals -> fgr.nrm, features (n x 36,
// padded) -> fgr.feat[k].  Neighbour sets are exact (ties -> lower index) in
// input order, as the KD-tree of the oracle returns them.
int features_device(orpcd_ctx* c, const double* host_xyz, int k, int64_t n, double fpfh_radius, int fpfh_knn,
                    double margin);

int fpfh_buffers(orpcd_ctx* c, int k, int64_t n, int fpfh_knn) {
    auto& F = c->fgr;
    CTX_CHECK(c, F.raw.ensure((size_t)n * 6));
    CTX_CHECK(c, F.nrm.ensure((size_t)n * 3));
    CTX_CHECK(c, F.nbr.ensure((size_t)n * fpfh_knn));
    CTX_CHECK(c, F.nd2.ensure((size_t)n * fpfh_knn));
    CTX_CHECK(c, F.cnt.ensure((size_t)n));
    CTX_CHECK(c, F.spfh.ensure((size_t)n * 33));
    CTX_CHECK(c, F.feat[k].ensure((size_t)n * kFeatDim));
    return ORPCD_OK;
}

// Normals + FPFH of the device cloud `pts` (input order; host_xyz its host
// copy for the bounding box) into feat_out (n x 36), with c->aux as the
// layout and the fgr scratch buffers (sized by fpfh_buffers).  Stream-ordered
// throughout: no host synchronisation, so a batch can queue one cloud after
// another.
int fpfh_at(orpcd_ctx* c, const double* host_xyz, const double* pts, int64_t n, double normal_radius, int normal_knn,
            double fpfh_radius, int fpfh_knn, double* feat_out) {
    auto& F = c->fgr;
    double margin = 0.0;
    int rc = layout_from_device(c, host_xyz, pts, n, c->aux, true, &margin);
    if (rc) return rc;
    // the normals' and the features' neighbourhoods are the same search when
    // their (radius, knn) agree (the FGR defaults: 0.1, 20): one KNN pass
    // then writes the covariances and the neighbour lists together
    const bool shared = normal_knn == fpfh_knn && normal_radius == fpfh_radius;
    CTX_CHECK(c, launch_knn_tiles(c->aux, pts, normal_knn, normal_radius, margin, true, F.raw.p,
                                  shared ? F.nbr.p : nullptr, shared ? F.nd2.p : nullptr, shared ? F.cnt.p : nullptr,
                                  c->stream, nullptr, knn_lane(c, n)));
    CTX_CHECK(c, launch_normals_cov(F.raw.p, n, nullptr, 1, -1.0, F.nrm.p, nullptr, c->stream));
    if (!shared)  // compute_fpfh_feature's own neighbourhoods
        CTX_CHECK(c, launch_knn_tiles(c->aux, pts, fpfh_knn, fpfh_radius, margin, true, nullptr, F.nbr.p, F.nd2.p,
                                      F.cnt.p, c->stream, nullptr, knn_lane(c, n)));
    CTX_CHECK(c, launch_fpfh(pts, F.nrm.p, n, F.nbr.p, F.nd2.p, F.cnt.p, fpfh_knn, F.spfh.p, feat_out, c->stream));
    return ORPCD_OK;
}

int fpfh_device(orpcd_ctx* c, const double* host_xyz, int k, int64_t n, double normal_radius, int normal_knn,
                double fpfh_radius, int fpfh_knn) {
    CTX_REQUIRE(c, normal_knn > 0 && normal_knn <= kMaxKnn && fpfh_knn > 0 && fpfh_knn <= kMaxKnn,
                "fpfh: knn must be in [1, 1024]");
    CTX_REQUIRE(c, normal_radius > 0 && fpfh_radius > 0, "fpfh: radii must be > 0");
    int rc = fpfh_buffers(c, k, n, fpfh_knn);
    if (rc) return rc;
    auto& F = c->fgr;
    return fpfh_at(c, host_xyz, F.xyz[k].p, n, normal_radius, normal_knn, fpfh_radius, fpfh_knn, F.feat[k].p);
}

// compute_fpfh_feature of fgr.xyz[k] with the normals in fgr.nrm.  host_xyz
// (the same cloud on the host) == nullptr: c->aux already holds its layout
// and `margin` its box margin.
int features_device(orpcd_ctx* c, const double* host_xyz, int k, int64_t n, double fpfh_radius, int fpfh_knn,
                    double margin) {
    auto& F = c->fgr;
    const double* pts = F.xyz[k].p;
    if (host_xyz) {
        int rc = layout_from_device(c, host_xyz, pts, n, c->aux, true, &margin);
        if (rc) return rc;
    }
    CTX_CHECK(c, launch_knn_tiles(c->aux, pts, fpfh_knn, fpfh_radius, margin, true, nullptr, F.nbr.p, F.nd2.p,
                                  F.cnt.p, c->stream, nullptr, knn_lane(c, n)));
    CTX_CHECK(c, launch_fpfh(pts, F.nrm.p, n, F.nbr.p, F.nd2.p, F.cnt.p, fpfh_knn, F.spfh.p, F.feat[k].p, c->stream));
    return ORPCD_OK;
}

double norm3(const double* a) { return std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }

// O3D FastGlobalRegistration.cpp NormalizePointCloud's result for one cloud:
// (p - mean) / scale (scale: the larger of the two clouds' max |p - mean|).
struct FgrCloud {
    const double* xyz = nullptr;  // host, input order
    double mean[3] = {0.0, 0.0, 0.0};
    void at(int64_t i, double scale, double out[3]) const {
        for (int a = 0; a < 3; ++a) out[a] = (xyz[3 * i + a] - mean[a]) / scale;
    }
};

// AdvancedMatching's tuple test (Open3D's sequential mt19937 draws, seeded:
// DESIGN.md §2) over the cross-checked pairs `corres` (i in cloud fi, j in
// cloud fj), then the tuples as (source, target) rows, normalised: p[K x 3]
// followed by q[K x 3] in pq.  Returns K.
int fgr_tuples(const std::vector<std::pair<int, int>>& corres, const orpcd_fgr_params& p, const FgrCloud cl[2],
               double scale, int fi, int fj, std::vector<double>& pq) {
    const int ncorr = (int)corres.size();
    std::vector<std::pair<int, int>> tup;
    if (ncorr > 0) {
        std::mt19937 gen((std::mt19937::result_type)p.seed);
        std::uniform_int_distribution<int> dis(0, ncorr - 1);
        const int64_t trials = (int64_t)ncorr * 100;
        const double sc = p.tuple_scale;
        int cnt = 0;
        for (int64_t t = 0; t < trials; ++t) {
            const int r[3] = {dis(gen), dis(gen), dis(gen)};
            double pi[3][3], pj[3][3];
            for (int e = 0; e < 3; ++e) {
                cl[fi].at(corres[r[e]].first, scale, pi[e]);
                cl[fj].at(corres[r[e]].second, scale, pj[e]);
            }
            double li[3], lj[3];
            for (int e = 0; e < 3; ++e) {
                const int f = (e + 1) % 3;
                const double di[3] = {pi[e][0] - pi[f][0], pi[e][1] - pi[f][1], pi[e][2] - pi[f][2]};
                const double dj[3] = {pj[e][0] - pj[f][0], pj[e][1] - pj[f][1], pj[e][2] - pj[f][2]};
                li[e] = norm3(di);
                lj[e] = norm3(dj);
            }
            if ((li[0] * sc < lj[0]) && (lj[0] < li[0] / sc) && (li[1] * sc < lj[1]) && (lj[1] < li[1] / sc) &&
                (li[2] * sc < lj[2]) && (lj[2] < li[2] / sc)) {
                for (int e = 0; e < 3; ++e) tup.push_back(corres[r[e]]);
                ++cnt;
            }
            if (cnt >= p.maximum_tuple_count) break;
        }
    }
    // pairs back to (source, target)
    const int K = (int)tup.size();
    pq.assign((size_t)std::max(K, 1) * 6, 0.0);
    for (int e = 0; e < K; ++e) {
        const int si = fi == 0 ? tup[e].first : tup[e].second;
        const int ti = fi == 0 ? tup[e].second : tup[e].first;
        cl[0].at(si, scale, &pq[(size_t)3 * e]);
        cl[1].at(ti, scale, &pq[(size_t)3 * K + 3 * e]);
    }
    return K;
}

// One start of the device tuple test: its cross-checked pairs (i in cloud
// fi, j in cloud fj), the device points of both clouds in input order and the
// normalisation (means, common scale).
struct TupleStart {
    const std::vector<std::pair<int, int>>* corres = nullptr;
    const double* xi = nullptr;   // device
    const double* xj = nullptr;
    const double* hxi = nullptr;  // the same points on the host (ORPCD_FGR_HOST_TUPLES)
    const double* hxj = nullptr;
    double mi[3] = {0, 0, 0}, mj[3] = {0, 0, 0};
    double scale = 1.0;
    int fi = 0;
};

// the seed's mt19937 words [0, need) on the device (host copy extended on demand)
constexpr size_t kTupleCacheWords = size_t(16) << 20;  // 64 MB host + 64 MB device kept between calls
int tuple_stream(orpcd_ctx* c, uint32_t seed, size_t need) {
    auto& T = c->fgr.tup;
    if (!T.valid || T.seed != seed) {
        T.gen.seed(seed);
        T.host.clear();
        T.on_dev = 0;
        T.seed = seed;
        T.valid = true;
    }
    if (T.host.size() < need) {
        const size_t want = std::max(need, T.host.size() * 2);
        T.host.reserve(want);
        while (T.host.size() < want) T.host.push_back((uint32_t)T.gen());
    }
    if (T.on_dev < need) {
        if (T.words.n < T.host.size()) {
            CTX_CHECK(c, T.words.ensure(T.host.size()));
            T.on_dev = 0;
        }
        CTX_CHECK(c, h2d(T.words.p + T.on_dev, T.host.data() + T.on_dev, (T.host.size() - T.on_dev) * 4, c->stream));
        T.on_dev = T.host.size();
    }
    return ORPCD_OK;
}

// fgr_tuples for every start at once on the device (fgr_kernels.hip, "tuple
// test"); the same tuples, bit for bit.  Start b's K[b] rows are at
// c->fgr.tup.rows + out[b]: cap[b] source rows (x, y, z), then cap[b] target
// rows.  ORPCD_FGR_HOST_TUPLES=1 runs fgr_tuples on host threads instead and
// lays its rows out the same way (A/B and the parity test of this path).
int fgr_tuples_device(orpcd_ctx* c, const std::vector<TupleStart>& st, const orpcd_fgr_params& p,
                      std::vector<int>& K, std::vector<int64_t>& out, std::vector<int64_t>& cap) {
    auto& T = c->fgr.tup;
    hipStream_t s = c->stream;
    const int B = (int)st.size();
    const int maxc = p.maximum_tuple_count;
    K.assign((size_t)B, 0);
    out.assign((size_t)B, 0);
    cap.assign((size_t)B, 0);
    std::vector<TupleJob> jobs((size_t)B);
    int64_t npairs = 0, nrows = 0;
    int max_ncorr = 0;
    for (int b = 0; b < B; ++b) {
        TupleJob& J = jobs[b];
        J.ncorr = (int)st[b].corres->size();
        J.trials = (int64_t)J.ncorr * 100;
        J.cap = 3 * std::min<int64_t>(maxc, J.trials);
        J.corr = npairs;
        J.out = nrows;
        J.xi = st[b].xi;
        J.xj = st[b].xj;
        for (int a = 0; a < 3; ++a) {
            J.mi[a] = st[b].mi[a];
            J.mj[a] = st[b].mj[a];
        }
        J.scale = st[b].scale;
        J.fi = st[b].fi;
        J.threshold = J.ncorr > 0 ? (0u - (uint32_t)J.ncorr) % (uint32_t)J.ncorr : 0u;
        out[b] = nrows;
        cap[b] = J.cap;
        npairs += J.ncorr;
        nrows += 6 * std::max<int64_t>(J.cap, 1);
        max_ncorr = std::max(max_ncorr, J.ncorr);
    }
    CTX_CHECK(c, T.rows.ensure((size_t)std::max<int64_t>(nrows, 6)));
    if (getenv("ORPCD_FGR_HOST_TUPLES")) {
        std::vector<double> rows((size_t)nrows, 0.0);
        host_parallel(B, [&](int b) {
            const TupleStart& S = st[b];
            FgrCloud cl[2];
            cl[S.fi].xyz = S.hxi;
            cl[1 - S.fi].xyz = S.hxj;
            for (int a = 0; a < 3; ++a) {
                cl[S.fi].mean[a] = S.mi[a];
                cl[1 - S.fi].mean[a] = S.mj[a];
            }
            std::vector<double> pq;
            K[b] = fgr_tuples(*S.corres, p, cl, S.scale, S.fi, 1 - S.fi, pq);
            for (int64_t r = 0; r < K[b]; ++r)
                for (int a = 0; a < 3; ++a) {
                    rows[(size_t)(out[b] + 3 * r + a)] = pq[(size_t)(3 * r + a)];
                    rows[(size_t)(out[b] + 3 * cap[b] + 3 * r + a)] = pq[(size_t)(3 * K[b] + 3 * r + a)];
                }
        });
        CTX_CHECK(c, h2d(T.rows.p, rows.data(), rows.size() * 8, s));
        return ORPCD_OK;
    }
    if (npairs == 0) return ORPCD_OK;
    // pairs and their normalised points
    std::vector<int32_t> pairs((size_t)npairs * 2);
    for (int b = 0; b < B; ++b) {
        int64_t o = jobs[b].corr;
        for (const auto& pr : *st[b].corres) {
            pairs[(size_t)(2 * o)] = pr.first;
            pairs[(size_t)(2 * o + 1)] = pr.second;
            ++o;
        }
    }
    CTX_CHECK(c, T.pairs.ensure(pairs.size()));
    CTX_CHECK(c, T.A.ensure((size_t)npairs * 3));
    CTX_CHECK(c, T.Bv.ensure((size_t)npairs * 3));
    CTX_CHECK(c, T.jobs.ensure((size_t)B));
    CTX_CHECK(c, T.nrej.ensure((size_t)B));
    CTX_CHECK(c, T.cnt.ensure((size_t)B));
    CTX_CHECK(c, h2d(T.pairs.p, pairs.data(), pairs.size() * 4, s));
    CTX_CHECK(c, h2d(T.jobs.p, jobs.data(), jobs.size() * sizeof(TupleJob), s));
    CTX_CHECK(c, launch_tuple_points(T.jobs.p, B, max_ncorr, T.pairs.p, T.A.p, T.Bv.p, s));
    CTX_CHECK(c, hipMemsetAsync(T.cnt.p, 0, (size_t)B * 4, s));
    std::vector<int64_t> t0((size_t)B, 0);
    std::vector<int32_t> cnt((size_t)B, 0), nrej((size_t)B);
    std::vector<int64_t> lists;
    for (;;) {
        // --- this window's trials per start
        int64_t max_tw = 0, max_span = 0;
        double expect = 0.0;
        for (int b = 0; b < B; ++b) {
            TupleJob& J = jobs[b];
            // the first window is short when the tuple limit is small (most
            // calls reach it within a few hundred trials per tuple): fewer
            // words drawn, rejections scanned and trials evaluated for nothing
            const int64_t win = t0[b] == 0 ? std::min<int64_t>(kTupleWindow, std::max<int64_t>(65536, 256 * (int64_t)maxc))
                                           : kTupleWindow;
            J.tw = (cnt[b] >= maxc || t0[b] >= J.trials) ? 0 : std::min(win, J.trials - t0[b]);
            J.nrej = 0;
            max_tw = std::max(max_tw, J.tw);
            expect = std::max(expect, 3.0 * (double)J.tw * (double)J.threshold / 4294967296.0);
        }
        if (max_tw == 0) break;
        // --- the words uniform_int_distribution rejects (rcap per start;
        // a window with more is scanned again with room for all of them)
        int64_t rcap = (int64_t)(2.0 * expect) + 64;
        for (;;) {
            size_t need = 0;
            for (int b = 0; b < B; ++b)
                if (jobs[b].tw > 0) {
                    max_span = std::max(max_span, 3 * jobs[b].tw + rcap);
                    need = std::max(need, (size_t)(jobs[b].word0 + 3 * jobs[b].tw + rcap));
                }
            int rc = tuple_stream(c, (uint32_t)p.seed, need);
            if (rc) return rc;
            CTX_CHECK(c, T.rej.ensure((size_t)B * rcap));
            CTX_CHECK(c, h2d(T.jobs.p, jobs.data(), jobs.size() * sizeof(TupleJob), s));
            CTX_CHECK(c, hipMemsetAsync(T.nrej.p, 0, (size_t)B * 4, s));
            CTX_CHECK(c, launch_tuple_reject(T.jobs.p, B, max_span, T.words.p, T.rej.p, T.nrej.p, rcap, s));
            CTX_CHECK(c, d2h(nrej.data(), T.nrej.p, (size_t)B * 4, s));
            CTX_CHECK(c, hipStreamSynchronize(s));
            int32_t most = 0;
            for (int b = 0; b < B; ++b) most = std::max(most, nrej[b]);
            if (most <= rcap) break;
            rcap = (int64_t)most + 64;
        }
        // --- sorted rejection keys, window-relative: key_j = r_j - word0 - j
        bool any = false;
        for (int b = 0; b < B; ++b) any = any || nrej[b] > 0;
        if (any) {
            lists.resize((size_t)B * rcap);
            CTX_CHECK(c, d2h(lists.data(), T.rej.p, lists.size() * 8, s));
            CTX_CHECK(c, hipStreamSynchronize(s));
            for (int b = 0; b < B; ++b) {
                int64_t* L = &lists[(size_t)b * rcap];
                std::sort(L, L + nrej[b]);
                for (int j = 0; j < nrej[b]; ++j) L[j] = L[j] - jobs[b].word0 - j;
                jobs[b].nrej = nrej[b];
                jobs[b].rej = (int64_t)b * rcap;
            }
            CTX_CHECK(c, h2d(T.rej.p, lists.data(), lists.size() * 8, s));
            CTX_CHECK(c, h2d(T.jobs.p, jobs.data(), jobs.size() * sizeof(TupleJob), s));
        }
        // --- every trial of the window, then the accepted ones in order
        CTX_CHECK(c, T.mask.ensure((size_t)B * (kTupleWindow / 64)));
        CTX_CHECK(c, T.chunk.ensure((size_t)B * (kTupleWindow / 4096)));
        CTX_CHECK(c, launch_tuple_eval(T.jobs.p, B, max_tw, T.words.p, T.rej.p, T.A.p, T.Bv.p, p.tuple_scale,
                                       T.mask.p, T.chunk.p, s));
        CTX_CHECK(c, launch_tuple_select(T.jobs.p, B, T.words.p, T.rej.p, T.mask.p, T.chunk.p, T.A.p, T.Bv.p, maxc,
                                         T.cnt.p, T.rows.p, s));
        CTX_CHECK(c, d2h(cnt.data(), T.cnt.p, (size_t)B * 4, s));
        CTX_CHECK(c, hipStreamSynchronize(s));
        // --- the next window starts at the word after the last one read
        for (int b = 0; b < B; ++b) {
            TupleJob& J = jobs[b];
            if (J.tw == 0) continue;
            const int64_t* L = any ? &lists[(size_t)b * rcap] : nullptr;
            int64_t used = 0;
            for (int j = 0; j < J.nrej; ++j)
                if (L[j] <= 3 * J.tw - 1) ++used;
            J.word0 += 3 * J.tw + used;
            t0[b] += J.tw;
        }
    }
    for (int b = 0; b < B; ++b) K[b] = 3 * cnt[b];
    // the seed's word stream stays cached for the next call (the same seed
    // every call), up to kTupleCacheWords: a call that needed more (a very
    // long tuple test) releases it, host and device, and the next call
    // regenerates what it needs
    if (T.host.size() > kTupleCacheWords) {
        CTX_CHECK(c, hipStreamSynchronize(s));
        std::vector<uint32_t>().swap(T.host);
        T.words.release();
        T.on_dev = 0;
        T.valid = false;
    }
    return ORPCD_OK;
}

// GetInvTransformationOriginalScale: the normalised-frame Tn back to the
// clouds' own frames (Open3D's column convention).
void fgr_original_scale(const double Tn[16], const double mean_src[3], const double mean_tgt[3], double scale,
                        double T[16]) {
    double inner[3];
    for (int a = 0; a < 3; ++a) {
        const double mr = Tn[4 * a] * mean_tgt[0] + Tn[4 * a + 1] * mean_tgt[1] + Tn[4 * a + 2] * mean_tgt[2];
        inner[a] = -mr + Tn[4 * a + 3] * scale + mean_src[a];
    }
    for (int a = 0; a < 16; ++a) T[a] = 0.0;
    for (int a = 0; a < 3; ++a) {
        for (int b = 0; b < 3; ++b) T[4 * a + b] = Tn[4 * b + a];
        T[4 * a + 3] = -(Tn[a] * inner[0] + Tn[4 + a] * inner[1] + Tn[8 + a] * inner[2]);
    }
    T[15] = 1.0;
}

// ORPCD_FGR_TRACE=1: the FGR path's phases on stderr (each mark drains the
// stream first, so the phases' own times, not their overlap)
struct FgrTrace {
    bool on = getenv("ORPCD_FGR_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void mark(hipStream_t s, const char* what) {
        if (!on) return;
        (void)hipStreamSynchronize(s);
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[orpcd fgr] %-28s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    }
};
thread_local FgrTrace* g_fgr_trace = nullptr;
static void fgr_mark(hipStream_t s, const char* what) {
    if (g_fgr_trace) g_fgr_trace->mark(s, what);
}

// AdvancedMatching's initial matching and cross check over padded feature
// rows on the device (source n rows, target m rows): nearest rows both ways
// on the matrix cores (launch_feat_nn, exact), then (i, i_to_j[i]) with
// j_to_i[i_to_j[i]] == i in i order, i over the larger set (fi; Open3D
// swaps the roles when the target has more points).  same_features: the two
// sets are the same rows (Q4 on equal-size clouds, fastGlobalOptimizer.py:
// 137-142, or identical caller features).
int fgr_match(orpcd_ctx* c, const double* fsrc, int64_t n, const double* ftgt, int64_t m, bool same_features,
              std::vector<std::pair<int, int>>& corres) {
    auto& F = c->fgr;
    hipStream_t s = c->stream;
    const int64_t np[2] = {n, m};
    const double* feat[2] = {fsrc, ftgt};
    int fi = 0, fj = 1;
    if (np[1] > np[0]) std::swap(fi, fj);
    const int64_t nPti = np[fi], nPtj = np[fj];
    if (same_features) {
        // the two sets are the same rows (n == m): every row's nearest feature
        // row is the lowest index of its exact duplicates (distance 0; any
        // other row is strictly farther), in both directions, so the mutual
        // pairs are (i, i) for the rows that are their own representative --
        // the answer both exact searches would return (the batch path's Q4
        // rule, orpcd_fgr_optimize_batch).  No search runs.
        corres.clear();
        CTX_CHECK(c, F.dedup.uflag.ensure((size_t)nPti));
        CTX_CHECK(c, dedup_flags(feat[fi], nPti, F.dedup, F.dedup.uflag.p, s, 1));
        std::vector<unsigned char> fl((size_t)nPti);
        CTX_CHECK(c, d2h(fl.data(), F.dedup.uflag.p, fl.size(), s));
        CTX_CHECK(c, hipStreamSynchronize(s));
        for (int64_t i = 0; i < nPti; ++i)
            if (fl[(size_t)i]) corres.push_back({(int)i, (int)i});
        fgr_mark(s, "feature matching (same rows)");
        return ORPCD_OK;
    }
    for (int k = 0; k < 2; ++k) {
        CTX_CHECK(c, F.fn2[k].ensure((size_t)np[k]));
        CTX_CHECK(c, launch_feat_norm(feat[k], np[k], F.fn2[k].p, s));
    }
    CTX_CHECK(c, F.nn[0].ensure((size_t)nPtj));
    CTX_CHECK(c, F.nn[1].ensure((size_t)nPti));
    fgr_mark(s, "  feature norms");
    // the distinct rows of both sets: direction 1 searches the distinct j
    // rows against the distinct i rows (duplicates take their
    // representative's answer: identical rows, identical answers), direction
    // 2 the chosen i rows against the distinct j rows
    int64_t nu = 0, nuj = 0;
    CTX_CHECK(c, dedup_rows(feat[fi], F.fn2[fi].p, nPti, F.dedup, &nu, s));
    CTX_CHECK(c, dedup_rows(feat[fj], F.fn2[fj].p, nPtj, F.dedup2, &nuj, s));
    fgr_mark(s, "  dedup (both sets)");
    CTX_CHECK(c, F.need.out.ensure((size_t)std::max(nPti, nPtj)));
    CTX_CHECK(c, F.need.pos.ensure((size_t)nPtj));
    CTX_CHECK(c, launch_feat_nn(F.dedup2.Fu.p, F.dedup2.n2u.p, nuj, F.dedup.Fu.p, F.dedup.n2u.p, nu, F.dedup.uidx.p,
                                33, F.fnn, F.need.out.p, s, c->profiling ? c->stats.feat : nullptr));
    CTX_CHECK(c, expand_dup_answers(F.dedup2, nPtj, nuj, F.need.out.p, F.need.pos.p, F.nn[0].p, s));
    fgr_mark(s, "  search j -> i (distinct rows)");
    // the second direction for the rows i some j chose only: any other i
    // fails the cross check whatever its answer (needed_rows)
    int64_t nq = 0;
    CTX_CHECK(c, needed_rows(F.nn[0].p, nPtj, feat[fi], F.fn2[fi].p, nPti, F.need, &nq, s));
    CTX_CHECK(c, hipMemsetAsync(F.nn[1].p, 0xFF, (size_t)nPti * 4, s));
    if (nq > 0) {
        CTX_CHECK(c, launch_feat_nn(F.need.F.p, F.need.n2.p, nq, F.dedup2.Fu.p, F.dedup2.n2u.p, nuj, F.dedup2.uidx.p,
                                    33, F.fnn, F.need.out.p, s, c->profiling ? c->stats.feat : nullptr));
        CTX_CHECK(c, scatter_answers(F.need.idx.p, nq, F.need.out.p, F.nn[1].p, s));
    }
    fgr_mark(s, "  search i -> j (chosen rows)");
    fgr_mark(s, "feature matching");
    std::vector<int32_t> j_to_i((size_t)nPtj), i_to_j((size_t)nPti);
    CTX_CHECK(c, d2h(j_to_i.data(), F.nn[0].p, (size_t)nPtj * 4, s));
    CTX_CHECK(c, d2h(i_to_j.data(), F.nn[1].p, (size_t)nPti * 4, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    // cross check, in i order: (i, i_to_j[i]) with j_to_i[i_to_j[i]] == i
    corres.clear();
    for (int64_t i = 0; i < nPti; ++i) {
        const int j = i_to_j[i];
        if (j >= 0 && j < nPtj && j_to_i[j] == i) corres.push_back({(int)i, j});
    }
    return ORPCD_OK;
}

// O3D FastGlobalRegistration.cpp: NormalizePointCloud, AdvancedMatching,
// OptimizePairwiseRegistration, GetInvTransformationOriginalScale and
// EvaluateRegistration, with points and padded features already on device
// (fgr.xyz[0..1], fgr.feat[0..1]).  src / tgt are the host copies used by the
// sequential tuple test.
int fgr_device(orpcd_ctx* c, const double* src, int64_t n, const double* tgt, int64_t m, const orpcd_fgr_params& p,
               double* T_out, double* fitness_out, double* rmse_out, int64_t* ncorr_out, int64_t* n_mutual_out,
               bool same_features) {
    auto& F = c->fgr;
    hipStream_t s = c->stream;
    const int64_t np[2] = {n, m};
    const double* host[2] = {src, tgt};
    // --- normalisation: means and the global radius (fixed-order partials)
    const int64_t nb_max = (std::max(n, m) + 255) / 256;
    CTX_CHECK(c, F.red.ensure((size_t)nb_max * 3));
    double mean[2][3];
    double scale = 0.0;
    for (int k = 0; k < 2; ++k) {
        const int64_t nb = (np[k] + 255) / 256;
        std::vector<double> part((size_t)nb * 3);
        CTX_CHECK(c, launch_sum3(F.xyz[k].p, np[k], F.red.p, s));
        CTX_CHECK(c, d2h(part.data(), F.red.p, part.size() * 8, s));
        CTX_CHECK(c, hipStreamSynchronize(s));
        double sum[3] = {0.0, 0.0, 0.0};
        for (int64_t b = 0; b < nb; ++b)
            for (int a = 0; a < 3; ++a) sum[a] += part[(size_t)3 * b + a];
        for (int a = 0; a < 3; ++a) mean[k][a] = sum[a] / (double)np[k];
        CTX_CHECK(c, launch_maxnorm(F.xyz[k].p, np[k], mean[k], F.red.p, s));
        CTX_CHECK(c, d2h(part.data(), F.red.p, (size_t)nb * 8, s));
        CTX_CHECK(c, hipStreamSynchronize(s));
        double mx = 0.0;
        for (int64_t b = 0; b < nb; ++b) mx = std::max(mx, part[(size_t)b]);
        scale = std::max(scale, mx);
    }
    CTX_REQUIRE(c, scale > 0.0, "fgr: degenerate clouds (all points at their mean)");
    fgr_mark(s, "normalisation");
    // --- initial matching on the matrix cores, both directions
    int fi = 0, fj = 1;
    if (np[1] > np[0]) std::swap(fi, fj);
    std::vector<std::pair<int, int>> corres;
    int rc = fgr_match(c, F.feat[0].p, n, F.feat[1].p, m, same_features, corres);
    if (rc) return rc;
    // --- tuple test: Open3D's mt19937 draws, every trial at once (fgr_tuples_device)
    const int ncorr = (int)corres.size();
    std::vector<TupleStart> ts(1);
    ts[0].corres = &corres;
    ts[0].xi = F.xyz[fi].p;
    ts[0].xj = F.xyz[fj].p;
    ts[0].hxi = host[fi];
    ts[0].hxj = host[fj];
    for (int a = 0; a < 3; ++a) {
        ts[0].mi[a] = mean[fi][a];
        ts[0].mj[a] = mean[fj][a];
    }
    ts[0].scale = scale;
    ts[0].fi = fi;
    std::vector<int> Ks;
    std::vector<int64_t> outs, caps;
    rc = fgr_tuples_device(c, ts, p, Ks, outs, caps);
    if (rc) return rc;
    const int K = Ks[0];
    fgr_mark(s, "cross check + tuple test");
    // --- GNC / Geman-McClure IRLS in one workgroup (fp64)
    CTX_CHECK(c, F.Tn.ensure(16));
    double* rows = c->fgr.tup.rows.p + outs[0];
    CTX_CHECK(c, launch_fgr_irls(rows, rows + 3 * caps[0], K, 1.0, p.iteration_number, p.division_factor,
                                 p.maximum_correspondence_distance, p.decrease_mu ? 1 : 0, F.Tn.p, s));
    double Tn[16];
    CTX_CHECK(c, d2h(Tn, F.Tn.p, sizeof(Tn), s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    fgr_mark(s, "irls");
    // --- GetInvTransformationOriginalScale (4x4 algebra)
    double T[16];
    fgr_original_scale(Tn, mean[0], mean[1], scale, T);
    // --- EvaluateRegistration(source, target, max_corr, T); the target is
    // already on the device (F.xyz[1])
    rc = layout_from_device(c, tgt, F.xyz[1].p, m, c->aux, true);
    if (rc) return rc;
    CTX_CHECK(c, F.raw.ensure((size_t)n * 3 + 16));
    CTX_CHECK(c, c->scratch32.ensure((size_t)n));
    CTX_CHECK(c, c->scratch64c.ensure((size_t)n));
    double* dT = F.raw.p + (size_t)n * 3;
    CTX_CHECK(c, h2d(dT, T, sizeof(T), s));
    CTX_CHECK(c, launch_transform_points(F.xyz[0].p, n, dT, F.raw.p, s));
    const double r = p.maximum_correspondence_distance;
    CTX_CHECK(c, launch_nn1(F.raw.p, n, c->aux, r * r, c->scratch32.p, c->scratch64c.p, c->qorder, s));
    const int64_t nb = (n + 255) / 256;
    CTX_CHECK(c, F.red.ensure((size_t)nb * 2));
    CTX_CHECK(c, launch_corr_stats(c->scratch32.p, c->scratch64c.p, n, F.red.p, s));
    std::vector<double> part((size_t)nb * 2);
    CTX_CHECK(c, d2h(part.data(), F.red.p, part.size() * 8, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    double cnt = 0.0, err2 = 0.0;
    for (int64_t b = 0; b < nb; ++b) {
        cnt += part[(size_t)2 * b];
        err2 += part[(size_t)2 * b + 1];
    }
    fgr_mark(s, "evaluation");
    std::memcpy(T_out, T, sizeof(T));
    if (fitness_out) *fitness_out = cnt > 0 ? cnt / (double)n : 0.0;
    if (rmse_out) *rmse_out = cnt > 0 ? std::sqrt(err2 / cnt) : 0.0;
    if (ncorr_out) *ncorr_out = (int64_t)cnt;
    if (n_mutual_out) {
        n_mutual_out[0] = ncorr;
        n_mutual_out[1] = K;
    }
    return ORPCD_OK;
}

// ------------------------------------------------------------- SourceTies
// Open3D recomputes the source's KNN-20 covariances on every posed copy
// source_initialized = np.dot(source, R0) + t0 (Aligner.py:183-185; the
// PointCloud rebuilt in generalizedICP.py:54-70); the batch rotates the
// unposed cloud's covariances instead, which is the same up to rounding
// EXCEPT where a point's 20th and 21st neighbours are so close that the posed
// copy's rounding decides which one enters.  Those points are listed once per
// source (source_ties_detect) with every candidate that could enter, and
// re-decided per start from the posed coordinates numpy forms
// (source_ties_apply): the oracle's distance expression, (d2, index) order,
// ComputeCovariance's one-pass cumulants on the posed points.  Clouds without
// such ties (C2) pay one 24- instead of 20-neighbour search at set_source.
constexpr double kTieRel = 1e-8;     // tie band: relative part (posing rounding: ~1e-13 relative)
constexpr double kTieAbs = 1e-12;    // ... and abs_coef = kTieAbs * (1 + max |coordinate|) times |d|
constexpr int kTieCap = 4096;        // ties listed per cloud (the surplus keeps the rotated covariance)
constexpr double kTieBruteBudget = 4e8;  // host pairs for ties whose candidates overflow the K-list

// np.dot(p, R0) + t0 for one row as numpy computes it: OpenBLAS dgemm with
// k = 3 accumulates fma(a2, b2, fma(a1, b1, a0 * b0)), then the broadcast add
// (bit-identical to numpy: tests/test_host.py::test_posed_rows_match_numpy)
void pose_row(const double* p, const double* R, const double* t, double* out) {
#pragma clang fp contract(off)
    for (int k = 0; k < 3; ++k) out[k] = std::fma(p[2], R[6 + k], std::fma(p[1], R[3 + k], p[0] * R[k])) + t[k];
}

// the oracle's / Open3D's point distance (KDTree::pt_d2: s = 0; s += d * d)
double tie_d2(const double* a, const double* b) {
#pragma clang fp contract(off)
    double s = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double d = a[k] - b[k];
        s += d * d;
    }
    return s;
}

int source_ties_detect(orpcd_ctx* c, const CloudLayout& L, const double* dev_in64, const double* host_xyz, int64_t n,
                       double margin, bool input_order, double* rawcov6, const int32_t* qlist = nullptr,
                       int64_t nq = 0) {
    auto& T = c->ties;
    T.clear();
    const int kcov = T.kcov, K = kcov + kTieExtra;
    double A = 0.0;
    for (int a = 0; a < 3; ++a) A = std::max(A, std::max(std::fabs(L.lo[a]), std::fabs(L.hi[a])));
    const double abs_coef = kTieAbs * (1.0 + A);
    T.band_A = A;
    CTX_CHECK(c, c->tie_cnt.ensure(2));
    CTX_CHECK(c, c->tie_q.ensure((size_t)kTieCap));
    CTX_CHECK(c, c->tie_rows.ensure((size_t)kTieCap * (K + 2)));
    CTX_CHECK(c, c->tie_d2.ensure((size_t)kTieCap * K));
    CTX_CHECK(c, hipMemsetAsync(c->tie_cnt.p, 0, 8, c->stream));
    KnnTieOut to;
    to.cnt = c->tie_cnt.p;
    to.rows = c->tie_rows.p;
    to.d2 = c->tie_d2.p;
    to.cap = kTieCap;
    to.rel = kTieRel;
    to.abs_coef = abs_coef;
    // pass 1: the covariances from the kcov nearest and the tie DETECTION,
    // which needs only the (kcov + 1)-th (C5 source: 5.4 -> 3.2 ms with 21
    // instead of 24 kept neighbours); pass 2: the detected points alone keep
    // kcov + kTieExtra for their table rows (the same exact lists, so the same
    // decisions and rows as one pass with kcov + kTieExtra)
    KnnTieOut det = to;
    det.cnt = c->tie_cnt.p + 1;
    det.detect = c->tie_q.p;
    CTX_CHECK(c, launch_knn_cov_ties(L, dev_in64, kcov, margin, input_order, rawcov6, det, c->stream,
                                     knn_lane(c, L.n), qlist, nq));
    int ndet = 0;
    CTX_CHECK(c, d2h(&ndet, c->tie_cnt.p + 1, 4, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    if (ndet > 0) {
        KnnTieOut rows = to;
        rows.force = 1;  // detected already: every listed point writes its row
        CTX_CHECK(c, launch_knn_cov_ties(L, dev_in64, kcov, margin, input_order, nullptr, rows, c->stream, false,
                                         c->tie_q.p, std::min(ndet, kTieCap)));
    }
    int cnt = 0;
    CTX_CHECK(c, d2h(&cnt, c->tie_cnt.p, 4, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    if (ndet > kTieCap) cnt = ndet;  // the table overflowed (pass 2 listed its first kTieCap)
    setup_mark(c->stream, "KNN-20 covariances (ties listed)");
    T.on = true;
    if (cnt == 0) return ORPCD_OK;
    const int m = std::min(cnt, kTieCap);
    T.complete = cnt <= kTieCap;
    std::vector<int32_t> rows((size_t)m * (K + 2));
    std::vector<double> d2((size_t)m * K);
    CTX_CHECK(c, d2h(rows.data(), c->tie_rows.p, rows.size() * 4, c->stream));
    CTX_CHECK(c, d2h(d2.data(), c->tie_d2.p, d2.size() * 8, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    T.xyz.assign(host_xyz, host_xyz + 3 * n);
    // deterministic order (the atomic list order is not): by input index
    std::vector<int> order((size_t)m);
    for (int e = 0; e < m; ++e) order[e] = e;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return rows[(size_t)a * (K + 2) + 1] < rows[(size_t)b * (K + 2) + 1]; });
    double budget = kTieBruteBudget;
    std::vector<std::pair<double, int32_t>> bf;
    for (int e : order) {
        const int32_t* r = &rows[(size_t)e * (K + 2)];
        const double* d = &d2[(size_t)e * K];
        const double dk = d[kcov];  // the (kcov+1)-th neighbour
        const double thr = dk + kTieRel * dk + abs_coef * std::sqrt(dk);
        const size_t start = T.cand.size();
        if (r[2 + K - 1] >= 0 && d[K - 1] <= thr) {
            // more candidates than the list holds: all of them, by brute force
            if (budget < (double)n) {
                T.complete = false;
                continue;
            }
            budget -= (double)n;
            bf.clear();
            const double* q = &host_xyz[3 * (size_t)r[1]];
            for (int64_t j = 0; j < n; ++j) {
                const double dd = tie_d2(q, &host_xyz[3 * j]);
                if (dd <= thr) bf.push_back({dd, (int32_t)j});
            }
            std::sort(bf.begin(), bf.end());
            for (auto& x : bf) T.cand.push_back(x.second);
        } else {
            for (int s2 = 0; s2 < K; ++s2)
                if (r[2 + s2] >= 0 && d[s2] <= thr) T.cand.push_back(r[2 + s2]);
        }
        if ((int)(T.cand.size() - start) <= kcov) {  // nothing to decide (cannot happen for a listed tie)
            T.cand.resize(start);
            continue;
        }
        T.pt.push_back(r[1]);
        T.pos.push_back(input_order ? -1 : r[0]);
        T.off.push_back((int32_t)T.cand.size());
    }
    T.rows.assign(T.pt.begin(), T.pt.end());
    T.rows.insert(T.rows.end(), T.cand.begin(), T.cand.end());
    std::sort(T.rows.begin(), T.rows.end());
    T.rows.erase(std::unique(T.rows.begin(), T.rows.end()), T.rows.end());
    auto row_of = [&](int32_t i) { return (int32_t)(std::lower_bound(T.rows.begin(), T.rows.end(), i) - T.rows.begin()); };
    T.pt_row.resize(T.pt.size());
    for (size_t f = 0; f < T.pt.size(); ++f) T.pt_row[f] = row_of(T.pt[f]);
    T.cand_row.resize(T.cand.size());
    for (size_t k = 0; k < T.cand.size(); ++k) T.cand_row[k] = row_of(T.cand[k]);
    return ORPCD_OK;
}

// Tie f's kcov neighbours (input indices, (d2, index) order) among its
// candidates at posed rows P (rows x 3), and ComputeCovariance of them on the
// posed points (O3D utility/Eigen.cpp: one-pass cumulants, 1/n).
void tie_decide(const orpcd_ctx::SourceTies& T, size_t f, const double* P, int32_t* set_out, double cov6[6]) {
#pragma clang fp contract(off)
    const double* q = &P[3 * (size_t)T.pt_row[f]];
    std::pair<double, int32_t> cd[256];
    std::vector<std::pair<double, int32_t>> big;
    const int nc = T.off[f + 1] - T.off[f];
    std::pair<double, int32_t>* v = cd;
    if (nc > 256) {
        big.resize((size_t)nc);
        v = big.data();
    }
    for (int k = 0; k < nc; ++k) {
        const int32_t ck = T.off[f] + k;
        v[k] = {tie_d2(q, &P[3 * (size_t)T.cand_row[ck]]), T.cand[ck]};
    }
    const int kc = T.kcov;
    std::partial_sort(v, v + kc, v + nc);
    double cu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < kc; ++s) {
        set_out[s] = v[s].second;
        const int32_t row = (int32_t)(std::lower_bound(T.rows.begin(), T.rows.end(), v[s].second) - T.rows.begin());
        const double* p = &P[3 * (size_t)row];
        cu[0] += p[0];
        cu[1] += p[1];
        cu[2] += p[2];
        cu[3] += p[0] * p[0];
        cu[4] += p[0] * p[1];
        cu[5] += p[0] * p[2];
        cu[6] += p[1] * p[1];
        cu[7] += p[1] * p[2];
        cu[8] += p[2] * p[2];
    }
    for (double& x : cu) x /= (double)kc;
    cov6[0] = cu[3] - cu[0] * cu[0];
    cov6[1] = cu[4] - cu[0] * cu[1];
    cov6[2] = cu[5] - cu[0] * cu[2];
    cov6[3] = cu[6] - cu[1] * cu[1];
    cov6[4] = cu[7] - cu[1] * cu[2];
    cov6[5] = cu[8] - cu[2] * cu[2];
}

// posed rows of start b: the caller's (orpcd_set_posed_tie_rows), or numpy's
// np.dot(source, R0) + t0 of the source's own rows
void tie_posed_rows(const orpcd_ctx::SourceTies& T, int b, const double* R0, const double* t0, double* P) {
    const size_t nr = T.rows.size();
    if (!T.posed_slot.empty() && std::isfinite(T.posed_slot[(size_t)b * nr * 3])) {
        std::memcpy(P, &T.posed_slot[(size_t)b * nr * 3], nr * 3 * sizeof(double));
        return;
    }
    for (size_t r = 0; r < nr; ++r) pose_row(&T.xyz[3 * (size_t)T.rows[r]], R0 + 9 * b, t0 + 3 * b, &P[3 * r]);
}

// Slot-ordered starts (R0 row-major: source @ R0 + t0): every tie's
// covariance re-decided per start, written over the rotated one in c->scov.
int source_ties_apply(orpcd_ctx* c, const double* R0, const double* t0, int B, double eps, bool count_gaps) {
    auto& T = c->ties;
    T.last_sets.clear();
    if (T.on) {
        // starts whose ties may not all be re-decided (statistics, surfaced
        // as GeneralizedICP.spec_stats["tie_gaps"]): the table overflowed
        // (kTieCap / the brute-force budget), or the posed copy's coordinates
        // exceed what the band's absolute term assumes: posing rounds a
        // coordinate by ~u |x R0 + t0| <= u (sqrt(3) A + |t0|), and kTieAbs
        // (1 + A) holds ~2000x that for |x R0 + t0| <= 1000 (1 + A).  A start
        // is counted once: when it begins (pass 0), not again when a pass
        // window resumes it
        for (int b = 0; b < B && count_gaps; ++b) {
            double tb = 0.0;
            for (int k = 0; k < 3; ++k) tb = std::max(tb, std::fabs(t0[3 * b + k]));
            if (!T.complete || std::sqrt(3.0) * T.band_A + tb > 1000.0 * (1.0 + T.band_A)) c->stats.tie_gaps += 1;
        }
    }
    if (!T.on || T.pt.empty()) {
        T.posed_slot.clear();
        return ORPCD_OK;
    }
    const size_t nt = T.pt.size(), nr = T.rows.size();
    const int kc = T.kcov;
    std::vector<double> P(nr * 3);
    T.last_sets.assign((size_t)B * nt * kc, -1);
    std::vector<double> ent;
    ent.reserve((size_t)B * nt * 8);
    for (int b = 0; b < B; ++b) {
        tie_posed_rows(T, b, R0, t0, P.data());
        for (size_t f = 0; f < nt; ++f) {
            double cov[6];
            tie_decide(T, f, P.data(), &T.last_sets[((size_t)b * nt + f) * kc], cov);
            if (T.pos[f] < 0) continue;  // not on this rank's rows
            ent.push_back((double)b);
            ent.push_back((double)T.pos[f]);
            for (double x : cov) ent.push_back(x);
        }
    }
    T.posed_slot.clear();
    const int count = (int)(ent.size() / 8);
    if (count == 0) return ORPCD_OK;
    CTX_CHECK(c, c->tie_ent.ensure(ent.size()));
    CTX_CHECK(c, h2d(c->tie_ent.p, ent.data(), ent.size() * 8, c->stream));
    CTX_CHECK(c, launch_cov_override(c->tie_ent.p, count, c->src.n, eps, c->scov.p, c->stream));
    return ORPCD_OK;
}

// Device state of a batch of B starts (pose = source @ R0_b + t0_b) before
// pass 0: base poses, identity T, posed-frame source covariances, first
// queries.  Host staging in c->h64 / c->h32 (layout used by gicp_batch).
// init16 != null (PointToPoint refinement): base pose G_b = init16[b] (column
// convention, as registration_icp applies `init`), no covariances.
int batch_setup(orpcd_ctx* c, const double* R0, const double* t0, int B, const orpcd_gicp_params* p,
                const double* init16 = nullptr, const double* state_in = nullptr, int pass_begin = 0) {
    const int64_t N = c->src.n;
    const int nblk = accum_blocks(N);
    c->last_B = 0;  // set once the batch is set up
    c->last_slot.clear();
    static const bool gaps = getenv("ORPCD_GAPS") != nullptr;
    const auto t_setup = std::chrono::steady_clock::now();
    if (gaps) {
        if (!c->gaps_ev0) CTX_CHECK(c, hipEventCreateWithFlags(&c->gaps_ev0, hipEventDisableSystemFence));
        CTX_CHECK(c, hipEventRecord(c->gaps_ev0, c->stream));
    }
    if (!init16) CTX_CHECK(c, c->scov.ensure((size_t)B * N * kCovW));
    c->batch_eps = p->epsilon;
    CTX_CHECK(c, c->prevnn.ensure((size_t)B * N));
    CTX_CHECK(c, c->best.ensure((size_t)B * N));
    CTX_CHECK(c, c->q32.ensure((size_t)B * N));
    CTX_CHECK(c, c->gbox.ensure((size_t)B * ((N + 127) / 128) * 2));
    CTX_CHECK(c, c->G.ensure((size_t)B * 12));
    CTX_CHECK(c, c->T.ensure((size_t)B * 16));
    CTX_CHECK(c, c->Q.ensure((size_t)B * 12));
    CTX_CHECK(c, c->R.ensure((size_t)B * 9));
    CTX_CHECK(c, c->prev.ensure((size_t)B * 2));
    CTX_CHECK(c, c->partial.ensure((size_t)B * nblk * kPartialStride));
    c->sched_live = sched_wanted(c, B);
    c->exact_live = c->opt.exact_nn != 0;
    if (c->exact_live) {
        CTX_CHECK(c, c->xsec.ensure((size_t)B * N));
        CTX_CHECK(c, c->xtotal.ensure(1));
        // at least one entry per wave of the re-search grid (each wave reads its
        // first entry before the count)
        CTX_CHECK(c, c->xlist.ensure(std::max<size_t>((size_t)B * N, (size_t)4 * 65536)));
        CTX_CHECK(c, c->xcnt.ensure(2));
        CTX_CHECK(c, hipMemsetAsync(c->xcnt.p, 0, 8, c->stream));
        CTX_CHECK(c, hipMemsetAsync(c->xtotal.p, 0, 8, c->stream));
    }
    if (c->sched_live) {
        const size_t NG = (size_t)(N + 127) / 128;
        c->sched_cap = sched_capacity(c, B);
        c->sched_B = B;
        CTX_CHECK(c, c->wcost.ensure(2 * (size_t)B * NG));
        CTX_CHECK(c, c->wtot.ensure(2 * (size_t)kSchedTot));
        CTX_CHECK(c, c->wcnt.ensure(2 * (size_t)kSchedClasses));
        CTX_CHECK(c, c->wlist.ensure((size_t)kSchedClasses * c->sched_cap));
        CTX_CHECK(c, hipMemsetAsync(c->wcost.p, 0, 2 * (size_t)B * NG * 4, c->stream));
        CTX_CHECK(c, hipMemsetAsync(c->wtot.p, 0, 2 * (size_t)kSchedTot * 8, c->stream));
        CTX_CHECK(c, hipMemsetAsync(c->wcnt.p, 0, 2 * (size_t)kSchedClasses * 4, c->stream));
    }
    CTX_CHECK(c, c->done.ensure((size_t)B));
    CTX_CHECK(c, c->active.ensure((size_t)B));
    CTX_CHECK(c, c->out_fit.ensure((size_t)B));
    CTX_CHECK(c, c->out_rmse.ensure((size_t)B));
    CTX_CHECK(c, c->out_iters.ensure((size_t)B));
    CTX_CHECK(c, c->out_ncorr.ensure((size_t)B));
    CTX_CHECK(c, c->scratch64c.ensure((size_t)B * 9));
    CTX_CHECK(c, c->h64.ensure((size_t)B * 80));
    CTX_CHECK(c, c->h32.ensure((size_t)B * 4));

    // host: base pose G_b = [R0_b^T | t0_b] (source @ R0 + t0 in column form)
    double* hG = c->h64.p;
    double* hT = hG + (size_t)B * 12;
    double* hQ = hT + (size_t)B * 16;
    double* hR = hQ + (size_t)B * 12;
    double* hRc = hR + (size_t)B * 9;
    double* hPrev = hRc + (size_t)B * 9;
    double* hFit = hPrev + (size_t)B * 2;
    double* hRmse = hFit + B;
    for (int b = 0; b < B; ++b) {
        if (init16) {
            for (int t = 0; t < 12; ++t) hG[12 * b + t] = init16[16 * b + t];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) hRc[9 * b + 3 * i + j] = init16[16 * b + 4 * i + j];
        } else {
            const double* r = R0 + 9 * b;
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) {
                    hG[12 * b + 4 * i + j] = r[3 * j + i];
                    hRc[9 * b + 3 * i + j] = r[3 * j + i];
                }
                hG[12 * b + 4 * i + 3] = t0[3 * b + i];
            }
        }
        for (int t = 0; t < 16; ++t) hT[16 * b + t] = (t % 5 == 0) ? 1.0 : 0.0;
        for (int t = 0; t < 12; ++t) hQ[12 * b + t] = hG[12 * b + t];
        for (int t = 0; t < 9; ++t) hR[9 * b + t] = (t % 4 == 0) ? 1.0 : 0.0;
        hPrev[2 * b] = hPrev[2 * b + 1] = 0.0;
        if (state_in) {  // resumed at pass_begin: the pose and previous metrics the solve left there
#pragma clang fp contract(off)  // Q as icp_solve_kernel forms it (solve_start), bit for bit
            const double* S = state_in + (size_t)kStateW * b;
            const double* G = &hG[12 * b];
            for (int t = 0; t < 16; ++t) hT[16 * b + t] = S[t];
            for (int r = 0; r < 3; ++r) {
                for (int cc = 0; cc < 4; ++cc) {
                    double v = S[4 * r + 0] * G[cc] + S[4 * r + 1] * G[4 + cc] + S[4 * r + 2] * G[8 + cc];
                    if (cc == 3) v += S[4 * r + 3];
                    hQ[12 * b + 4 * r + cc] = v;
                }
                for (int cc = 0; cc < 3; ++cc) hR[9 * b + 3 * r + cc] = S[4 * r + cc];
            }
            hPrev[2 * b] = S[16];
            hPrev[2 * b + 1] = S[17];
        }
    }
    int32_t* hAct = c->h32.p;
    int32_t* hDone = hAct + B;
    int32_t* hIters = hDone + B;
    for (int b = 0; b < B; ++b) {
        hAct[b] = b;
        hDone[b] = 0;
    }
    hipStream_t s = c->stream;
    CTX_CHECK(c, hipMemcpyAsync(c->G.p, hG, (size_t)B * 12 * 8, hipMemcpyHostToDevice, s));
    CTX_CHECK(c, hipMemcpyAsync(c->T.p, hT, (size_t)B * 16 * 8, hipMemcpyHostToDevice, s));
    CTX_CHECK(c, hipMemcpyAsync(c->Q.p, hQ, (size_t)B * 12 * 8, hipMemcpyHostToDevice, s));
    CTX_CHECK(c, hipMemcpyAsync(c->R.p, hR, (size_t)B * 9 * 8, hipMemcpyHostToDevice, s));
    CTX_CHECK(c, hipMemcpyAsync(c->scratch64c.p, hRc, (size_t)B * 9 * 8, hipMemcpyHostToDevice, s));
    CTX_CHECK(c, hipMemcpyAsync(c->prev.p, hPrev, (size_t)B * 2 * 8, hipMemcpyHostToDevice, s));
    CTX_CHECK(c, hipMemcpyAsync(c->active.p, hAct, (size_t)B * 4, hipMemcpyHostToDevice, s));
    CTX_CHECK(c, hipMemcpyAsync(c->done.p, hDone, (size_t)B * 4, hipMemcpyHostToDevice, s));
    CTX_CHECK(c, hipMemsetAsync(c->prevnn.p, 0xff, (size_t)B * N * 4, s));

    c->last_B = B;
    // posed-frame source covariances for every start (rigid equivariance)
    c->est = init16 ? kEstP2P : kEstGICP;
    if (!init16) {
        CTX_CHECK(c, launch_normals_cov(c->sraw.p, N, c->scratch64c.p, B, p->epsilon, nullptr,
                                        ORPCD_NORMAL_COV ? nullptr : c->scov.p, s,
                                        ORPCD_NORMAL_COV ? c->scov.p : nullptr));
        int rc = source_ties_apply(c, R0, t0, B, p->epsilon, pass_begin == 0);  // boundary ties decided on the posed copies
        if (rc) return rc;
    }
    if (getenv("ORPCD_SYNC_LAUNCH")) {  // debugging: the set-up's kernels, apart from the pass loop's
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) fprintf(stderr, "[orpcd] batch set-up kernels failed: %s\n", hipGetErrorString(e));
        CTX_CHECK(c, e);
    }
    c->pass_base = pass_begin;
    CTX_CHECK(c, launch_xform(c, B, pass_begin, p->max_correspondence_distance * p->max_correspondence_distance, s,
                              target_bounds(c, hAct, B)));
    c->gaps_setup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_setup).count();
    return ORPCD_OK;
}

int run_passes(orpcd_ctx* c, int B, const orpcd_gicp_params* p, double* T_out, double* rmse_out,
               double* fitness_out, int32_t* iters_out, int64_t* ncorr_out, int pass_begin = 0,
               int pass_end = 0x7fffffff);
int read_outputs(orpcd_ctx* c, int B, unsigned long long tiles_before, double* T_out, double* rmse_out,
                 double* fitness_out, int32_t* iters_out, int64_t* ncorr_out);

// RCCL entry points, resolved from librccl.so at first use: the library
// itself links no collective library, so a host without RCCL still loads it
// (only orpcd_comm_* then fail, with ORPCD_EDEVICE).
struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};
const RcclApi& rccl_api() {
    static const RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            a.err = std::string("librccl.so not loadable: ") + (e ? e : "?");
            return a;
        }
        a.get_unique_id = (decltype(a.get_unique_id))dlsym(h, "ncclGetUniqueId");
        a.comm_init_rank = (decltype(a.comm_init_rank))dlsym(h, "ncclCommInitRank");
        a.all_reduce = (decltype(a.all_reduce))dlsym(h, "ncclAllReduce");
        a.all_gather = (decltype(a.all_gather))dlsym(h, "ncclAllGather");
        a.comm_destroy = (decltype(a.comm_destroy))dlsym(h, "ncclCommDestroy");
        a.error_string = (decltype(a.error_string))dlsym(h, "ncclGetErrorString");
        a.ok = a.get_unique_id && a.comm_init_rank && a.all_reduce && a.all_gather && a.comm_destroy && a.error_string;
        if (!a.ok) a.err = "librccl.so lacks an nccl* entry point";
        return a;
    }();
    return api;
}

}  // namespace

extern "C" {

int orpcd_abi_version(void) { return ORPCD_ABI_VERSION; }

int orpcd_device_count(int* count) {
    if (!count) return ORPCD_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return ORPCD_OK;
}

// Context creation runs the set-up path once on a synthetic cloud of
// kWarmPoints points (>= knn_lane_min: the kernels a large cloud takes), so
// that a fresh context's first set_target / set_source does not pay the
// process's one-time GPU runtime costs: code-object loads, the first launch
// of every kernel (rocprim's sort kernels alone cost ~13 ms at their first
// 1M-point sort), the blit kernels of the first copies.  Measured on MI355X
// (profiles/r06_c5_cold.md): allocations are not the cost (33 hipMalloc,
// 0.56 ms in all).  ORPCD_LAZY_CODE_OBJECTS=1 skips it.
constexpr int64_t kWarmPoints = 262144;
static int warm_setup(orpcd_ctx* c) {
    std::vector<double> pts((size_t)kWarmPoints * 3);
    uint64_t x = 0x9E3779B97F4A7C15ull;  // splitmix64: a fixed pseudo-random cube, no ties
    for (auto& v : pts) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        v = (double)((z ^ (z >> 31)) >> 11) * 0x1p-53;
    }
    int rc = upload_target(c, pts.data(), kWarmPoints, 1e-3);
    if (rc) return rc;
    double margin = 0.0;
    rc = upload_layout(c, pts.data(), kWarmPoints, c->src, true, &margin);
    if (rc) return rc;
    CTX_CHECK(c, c->sraw.ensure((size_t)kWarmPoints * 6));
    rc = source_ties_detect(c, c->src, c->scratch64a.p, pts.data(), kWarmPoints, margin, false, c->sraw.p);
    if (rc) return rc;
    std::vector<double> back(64);
    CTX_CHECK(c, d2h(back.data(), c->scratch64a.p, back.size() * 8, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    // nothing of the synthetic clouds stays usable
    c->ties.clear();
    c->tgt_host[0].clear();
    c->tgt_eps[0] = -1.0;
    c->ntgt = 0;
    c->src_cov = false;
    c->last_B = 0;
    c->tgts[0].n = 0;  // the buffers stay allocated (sized for the next cloud of this size)
    c->src.n = 0;
    return ORPCD_OK;
}

int orpcd_ctx_create(int device, orpcd_ctx** out) {
    if (!out) return ORPCD_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ORPCD_EDEVICE;
    if (device < 0 || device >= n) return ORPCD_EINVAL;
    orpcd_ctx* c = new (std::nothrow) orpcd_ctx();
    if (!c) return ORPCD_EDEVICE;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        c->counters.ensure(kCounterSlots * kCounterStride) != hipSuccess ||
        hipMemset(c->counters.p, 0, kCounterSlots * kCounterStride * 8) != hipSuccess ||
        (!getenv("ORPCD_LAZY_CODE_OBJECTS") &&
         (preload_code_object_sort() != hipSuccess || preload_code_object_knn() != hipSuccess ||
          preload_code_object_gicp() != hipSuccess ||
          // the creating thread's pinned staging buffer at its full size
          // (a 1M-point cloud's first upload would otherwise pin it: ~4 ms)
          staging_reserve(staging(), kStageChunk) != hipSuccess))) {
        if (c->stream) (void)hipStreamDestroy(c->stream);
        c->counters.release();
        delete c;
        return ORPCD_EDEVICE;
    }
    if (!getenv("ORPCD_LAZY_CODE_OBJECTS") && warm_setup(c) != ORPCD_OK) {
        orpcd_ctx_destroy(c);
        return ORPCD_EDEVICE;
    }
    *out = c;
    return ORPCD_OK;
}

int orpcd_ctx_destroy(orpcd_ctx* c) {
    if (!c) return ORPCD_EINVAL;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)orpcd_comm_destroy(c);
    for (int k = 0; k < kMaxTargets; ++k) {
        c->tgts[k].release();
        c->tcovs[k].release();
    }
    c->tdesc.release();
    c->src.release();
    c->aux.release();
    for (auto* b : {&c->sraw, &c->scov, &c->G, &c->T, &c->Q, &c->R, &c->prev, &c->partial, &c->out_fit,
                    &c->out_rmse, &c->scratch64a, &c->scratch64b, &c->scratch64c})
        b->release();
    c->prevnn.release();
    c->best.release();
    c->q32.release();
    c->gbox.release();
    c->done.release();
    c->active.release();
    for (auto* b : {&c->wcost, &c->wcnt}) b->release();
    c->wtot.release();
    c->wlist.release();
    c->xsec.release();
    c->xlist.release();
    c->xcnt.release();
    c->xtotal.release();
    c->out_iters.release();
    c->out_ncorr.release();
    c->scratch32.release();
    c->tie_ent.release();
    c->tie_rows.release();
    c->tie_d2.release();
    c->tie_cnt.release();
    c->tie_q.release();
    for (auto* b : {&c->qorder.ids, &c->qorder.order}) b->release();
    c->qorder.codes.release();
    c->qorder.tmp.release();
    c->counters.release();
    c->h64.release();
    c->h32.release();
    c->fgr.release();
    c->vox.release();
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return ORPCD_OK;
}

const char* orpcd_last_error(const orpcd_ctx* c) { return c ? c->err.c_str() : "null context"; }

int orpcd_set_target(orpcd_ctx* c, const double* xyz, int64_t m, double epsilon) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && m > 0, "set_target: empty target cloud");
    CTX_REQUIRE(c, m < kMaxPoints, "set_target: too many points");
    CTX_REQUIRE(c, finite_cloud(xyz, m), "set_target: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    c->ntgt = 0;
    c->last_B = 0;  // the last batch's correspondences refer to the old targets
    SetupTrace tr;
    g_setup_trace = &tr;
    struct Reset {
        ~Reset() { g_setup_trace = nullptr; }
    } reset;
    int rc = upload_target(c, xyz, m, epsilon);
    if (rc) return rc;
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    setup_mark(c->stream, "target: seed grid");
    c->ntgt = 1;
    return ORPCD_OK;
}

int orpcd_set_targets(orpcd_ctx* c, const double* xyz, const int64_t* m, int32_t ntargets, double epsilon) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && m, "set_targets: null argument");
    CTX_REQUIRE(c, ntargets >= 1 && ntargets <= kMaxTargets, "set_targets: 1 to 16 targets");
    int64_t off = 0;
    for (int k = 0; k < ntargets; ++k) {
        CTX_REQUIRE(c, m[k] > 0 && m[k] < kMaxPoints, "set_targets: empty target cloud or too many points");
        CTX_REQUIRE(c, finite_cloud(xyz + 3 * off, m[k]), "set_targets: non-finite coordinates");
        off += m[k];
    }
    CTX_CHECK(c, hipSetDevice(c->device));
    c->ntgt = 0;
    c->last_B = 0;
    off = 0;
    for (int k = 0; k < ntargets; ++k) {
        int rc = upload_target_k(c, k, xyz + 3 * off, m[k], epsilon);
        if (rc) return rc;
        off += m[k];
    }
    CTX_CHECK(c, seed_grids(c, 0, ntargets));  // every target's grid, one set of launches
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    c->ntgt = ntargets;
    return ORPCD_OK;
}

int orpcd_set_source(orpcd_ctx* c, const double* xyz, int64_t n) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && n > 0, "set_source: empty source cloud");
    CTX_REQUIRE(c, n < kMaxPoints, "set_source: too many points");
    CTX_REQUIRE(c, finite_cloud(xyz, n), "set_source: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    c->src_cov = false;
    c->last_B = 0;
    SetupTrace tr;
    g_setup_trace = &tr;
    struct Reset {
        ~Reset() { g_setup_trace = nullptr; }
    } reset;
    double margin = 0.0;
    int rc = upload_layout(c, xyz, n, c->src, true, &margin);
    if (rc) return rc;
    CTX_CHECK(c, c->sraw.ensure((size_t)n * 6));
    rc = source_ties_detect(c, c->src, c->scratch64a.p, xyz, n, margin, false, c->sraw.p);
    if (rc) return rc;
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    setup_mark(c->stream, "source: KNN-20 + ties");
    c->src_cov = true;
    return ORPCD_OK;
}

int orpcd_gicp_batch(orpcd_ctx* c, const double* R0, const double* t0, int32_t B, const orpcd_gicp_params* p,
                     double* T_out, double* rmse_out, double* fitness_out, int32_t* iters_out, int64_t* ncorr_out) {
    return orpcd_gicp_batch_targets(c, R0, t0, nullptr, B, p, T_out, rmse_out, fitness_out, iters_out, ncorr_out);
}

int orpcd_gicp_batch_window(orpcd_ctx* c, const double* R0, const double* t0, const int32_t* target_of_start,
                            int32_t B, const orpcd_gicp_params* p, int32_t pass_begin, int32_t pass_end,
                            const double* state_in, double* state_out, int32_t* done_out, double* T_out,
                            double* rmse_out, double* fitness_out, int32_t* iters_out, int64_t* ncorr_out);

int orpcd_gicp_batch_targets(orpcd_ctx* c, const double* R0, const double* t0, const int32_t* target_of_start,
                             int32_t B, const orpcd_gicp_params* p, double* T_out, double* rmse_out,
                             double* fitness_out, int32_t* iters_out, int64_t* ncorr_out) {
    return orpcd_gicp_batch_window(c, R0, t0, target_of_start, B, p, 0, 0x7fffffff, nullptr, nullptr, nullptr, T_out,
                                   rmse_out, fitness_out, iters_out, ncorr_out);
}

// The same batch run over passes [pass_begin, pass_end) only (DESIGN.md §7,
// the C4 re-deal): state_in (B x kStateW, caller order: T row-major 4x4, the
// previous pass's fitness and rmse) is where the starts stand at pass_begin
// (required when pass_begin > 0); after the window, done_out[b] tells which
// starts finished (their outputs are set) and state_out holds the others'
// state at pass_end.  Resuming a start from that state -- in any batch, on
// any context -- continues it bit for bit: a start's passes depend only on
// its pose, its covariances (from R0, t0) and the target.
int orpcd_gicp_batch_window(orpcd_ctx* c, const double* R0, const double* t0, const int32_t* target_of_start,
                            int32_t B, const orpcd_gicp_params* p, int32_t pass_begin, int32_t pass_end,
                            const double* state_in, double* state_out, int32_t* done_out, double* T_out,
                            double* rmse_out, double* fitness_out, int32_t* iters_out, int64_t* ncorr_out) {
    if (!c) return ORPCD_EINVAL;
    // the caller's posed tie rows (orpcd_set_posed_tie_rows) belong to this
    // call only: taken before any validation, so a rejected batch never
    // leaves them for the next one
    auto& TS = c->ties;
    std::vector<double> posed;
    posed.swap(TS.posed);
    const int posed_B = TS.posed_B;
    TS.posed_B = 0;
    TS.posed_slot.clear();
    CTX_REQUIRE(c, pass_begin >= 0 && pass_end > pass_begin && (pass_begin == 0 || state_in),
                "gicp_batch_window: bad pass window (pass_begin > 0 needs state_in)");
    CTX_REQUIRE(c, R0 && t0 && p && T_out && rmse_out, "gicp_batch: null argument");
    CTX_REQUIRE(c, B > 0, "gicp_batch: B must be > 0");
    CTX_REQUIRE(c, c->src.n > 0, "gicp_batch: no source (call orpcd_set_source)");
    CTX_REQUIRE(c, c->ntgt > 0 && c->tgt.n > 0, "gicp_batch: no target (call orpcd_set_target)");
    CTX_REQUIRE(c, p->max_correspondence_distance > 0, "gicp_batch: max_correspondence_distance must be > 0");
    CTX_REQUIRE(c, p->max_iteration >= 0, "gicp_batch: max_iteration must be >= 0");
    CTX_REQUIRE(c, p->epsilon >= 0, "gicp_batch: epsilon must be >= 0");
    CTX_REQUIRE(c, c->src_cov, "gicp_batch: the source has no covariances (set it with orpcd_set_source)");
    // slots ordered by target (stable): start b runs in slot pos[b]
    int first[kMaxTargets + 1] = {0};
    std::vector<int> pos((size_t)B);
    int ntg = 1;
    if (target_of_start) {
        for (int b = 0; b < B; ++b)
            CTX_REQUIRE(c, target_of_start[b] >= 0 && target_of_start[b] < c->ntgt,
                        "gicp_batch_targets: target index out of range (orpcd_set_targets)");
        ntg = c->ntgt;
        int cnt[kMaxTargets] = {0};
        for (int b = 0; b < B; ++b) ++cnt[target_of_start[b]];
        for (int k = 0; k < ntg; ++k) first[k + 1] = first[k] + cnt[k];
        int fill[kMaxTargets];
        for (int k = 0; k < ntg; ++k) fill[k] = first[k];
        for (int b = 0; b < B; ++b) pos[b] = fill[target_of_start[b]]++;
    } else {
        first[1] = B;
        for (int b = 0; b < B; ++b) pos[b] = b;
    }
    CTX_CHECK(c, hipSetDevice(c->device));
    if (posed_B) {  // caller order -> slot order
        CTX_REQUIRE(c, posed_B == B, "gicp_batch: posed tie rows were set for a different number of starts");
        const size_t w = TS.rows.size() * 3;
        TS.posed_slot.resize((size_t)B * w);
        for (int b = 0; b < B; ++b) std::memcpy(&TS.posed_slot[(size_t)pos[b] * w], &posed[(size_t)b * w], w * 8);
    }
    int rc = targets_for_epsilon(c, ntg, p->epsilon);  // target covariances depend on epsilon
    if (rc) return rc;
    c->batch_ntgt = ntg;
    for (int k = 0; k <= ntg; ++k) c->batch_first[k] = first[k];
    std::vector<double> sR((size_t)B * 9), st((size_t)B * 3), sS;
    for (int b = 0; b < B; ++b) {
        std::memcpy(&sR[(size_t)pos[b] * 9], R0 + 9 * b, 9 * sizeof(double));
        std::memcpy(&st[(size_t)pos[b] * 3], t0 + 3 * b, 3 * sizeof(double));
    }
    if (state_in) {
        sS.resize((size_t)B * kStateW);
        for (int b = 0; b < B; ++b)
            std::memcpy(&sS[(size_t)pos[b] * kStateW], state_in + (size_t)kStateW * b, kStateW * sizeof(double));
    }
    const auto t_batch = std::chrono::steady_clock::now();
    rc = batch_setup(c, sR.data(), st.data(), B, p, nullptr, state_in ? sS.data() : nullptr, pass_begin);
    if (rc) return rc;
    std::vector<double> oT((size_t)B * 16), orm((size_t)B), ofit((size_t)B);
    std::vector<int32_t> oit((size_t)B);
    std::vector<int64_t> onc((size_t)B);
    rc = run_passes(c, B, p, oT.data(), orm.data(), ofit.data(), oit.data(), onc.data(), pass_begin, pass_end);
    c->batch_ntgt = 1;
    c->batch_first[1] = 0;
    c->pass_base = 0;
    if (rc) return rc;
    if (done_out || state_out) {  // which starts finished in the window, and where the others stand
        std::vector<int32_t> dn((size_t)B);
        std::vector<double> hT((size_t)B * 16), hP((size_t)B * 2);
        CTX_CHECK(c, d2h(dn.data(), c->done.p, (size_t)B * 4, c->stream));
        CTX_CHECK(c, d2h(hT.data(), c->T.p, hT.size() * 8, c->stream));
        CTX_CHECK(c, d2h(hP.data(), c->prev.p, hP.size() * 8, c->stream));
        for (int b = 0; b < B; ++b) {
            const int q = pos[b];
            if (done_out) done_out[b] = dn[q] ? 1 : 0;
            if (state_out) {
                std::memcpy(state_out + (size_t)kStateW * b, &hT[(size_t)q * 16], 16 * sizeof(double));
                std::memcpy(state_out + (size_t)kStateW * b + 16, &hP[(size_t)q * 2], 2 * sizeof(double));
            }
        }
    }
    c->stats.host_batch_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_batch).count();
    c->stats.host_batches += 1;
    c->last_slot = pos;
    c->last_slot_tgt.assign((size_t)B, 0);
    for (int k = 0; k < ntg; ++k)
        for (int q = first[k]; q < first[k + 1]; ++q) c->last_slot_tgt[q] = k;
    for (int b = 0; b < B; ++b) {
        const int q = pos[b];
        std::memcpy(T_out + 16 * b, &oT[(size_t)q * 16], 16 * sizeof(double));
        rmse_out[b] = orm[q];
        if (fitness_out) fitness_out[b] = ofit[q];
        if (iters_out) iters_out[b] = oit[q];
        if (ncorr_out) ncorr_out[b] = onc[q];
    }
    return ORPCD_OK;
}

int orpcd_source_ties(orpcd_ctx* c, int64_t* n_ties, int64_t* n_rows, int32_t* complete, int64_t* rows_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, n_ties && n_rows, "source_ties: null argument");
    const auto& T = c->ties;
    *n_ties = (int64_t)T.pt.size();
    *n_rows = (int64_t)T.rows.size();
    if (complete) *complete = T.complete ? 1 : 0;
    if (rows_out)
        for (size_t r = 0; r < T.rows.size(); ++r) rows_out[r] = T.rows[r];
    return ORPCD_OK;
}

int orpcd_pose_rows(const double* xyz, const int64_t* idx, int64_t n, const double* R, const double* t, double* out) {
    if (!xyz || !R || !t || !out || n < 0) return ORPCD_EINVAL;
    for (int64_t i = 0; i < n; ++i) pose_row(xyz + 3 * (idx ? idx[i] : i), R, t, out + 3 * i);
    return ORPCD_OK;
}

int orpcd_set_posed_tie_rows(orpcd_ctx* c, int32_t B, const double* xyz) {
    if (!c) return ORPCD_EINVAL;
    auto& T = c->ties;
    if (B <= 0 || !xyz) {  // clear
        T.posed.clear();
        T.posed_B = 0;
        return ORPCD_OK;
    }
    T.posed.assign(xyz, xyz + (size_t)B * T.rows.size() * 3);
    T.posed_B = B;
    return ORPCD_OK;
}

int orpcd_tie_sets(orpcd_ctx* c, int32_t b, const double* posed_rows, int32_t* sets_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, sets_out, "tie_sets: null argument");
    const auto& T = c->ties;
    const size_t nt = T.pt.size(), kc = (size_t)T.kcov;
    if (nt == 0) return ORPCD_OK;
    if (posed_rows) {
        double cov[6];
        for (size_t f = 0; f < nt; ++f) tie_decide(T, f, posed_rows, sets_out + f * kc, cov);
        return ORPCD_OK;
    }
    CTX_REQUIRE(c, b >= 0 && b < (int32_t)c->last_slot.size() && !T.last_sets.empty(),
                "tie_sets: no such start in the last batch");
    std::memcpy(sets_out, &T.last_sets[(size_t)c->last_slot[b] * nt * kc], nt * kc * 4);
    return ORPCD_OK;
}

int orpcd_set_source_points(orpcd_ctx* c, const double* xyz, int64_t n) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && n > 0, "set_source_points: empty source cloud");
    CTX_REQUIRE(c, n < kMaxPoints, "set_source_points: too many points");
    CTX_REQUIRE(c, finite_cloud(xyz, n), "set_source_points: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    c->src_cov = false;
    c->last_B = 0;
    c->ties.clear();
    int rc = upload_layout(c, xyz, n, c->src, true);
    if (rc) return rc;
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    return ORPCD_OK;
}

int orpcd_icp_p2p_batch(orpcd_ctx* c, const double* init, int32_t B, const orpcd_gicp_params* p, double* T_out,
                        double* rmse_out, double* fitness_out, int32_t* iters_out, int64_t* ncorr_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, init && p && T_out && rmse_out, "icp_p2p_batch: null argument");
    CTX_REQUIRE(c, B > 0, "icp_p2p_batch: B must be > 0");
    CTX_REQUIRE(c, c->src.n > 0, "icp_p2p_batch: no source (call orpcd_set_source_points)");
    CTX_REQUIRE(c, c->tgt.n > 0, "icp_p2p_batch: no target (call orpcd_set_target)");
    CTX_REQUIRE(c, p->max_correspondence_distance > 0, "icp_p2p_batch: max_correspondence_distance must be > 0");
    CTX_REQUIRE(c, p->max_iteration >= 0, "icp_p2p_batch: max_iteration must be >= 0");
    for (int64_t t = 0; t < 16 * (int64_t)B; ++t) CTX_REQUIRE(c, std::isfinite(init[t]), "icp_p2p_batch: non-finite init");
    CTX_CHECK(c, hipSetDevice(c->device));
    int rc = batch_setup(c, nullptr, nullptr, B, p, init);
    if (rc) return rc;
    c->last_slot.resize((size_t)B);
    for (int b = 0; b < B; ++b) c->last_slot[b] = b;
    c->last_slot_tgt.assign((size_t)B, 0);
    return run_passes(c, B, p, T_out, rmse_out, fitness_out, iters_out, ncorr_out);
}

}  // extern "C"

namespace {

// Outputs of the batch (after the last pass): T (GICP: ICP transform of the
// posed source; PointToPoint: T * G), rmse, fitness, iterations, inliers.
int read_outputs(orpcd_ctx* c, int B, unsigned long long tiles_before, double* T_out, double* rmse_out,
                 double* fitness_out, int32_t* iters_out, int64_t* ncorr_out) {
    double* hT = c->h64.p + (size_t)B * 12;
    double* hFit = hT + (size_t)B * (16 + 12 + 9 + 9 + 2);
    double* hRmse = hFit + B;
    int32_t* hIters = c->h32.p + 2 * B;
    hipStream_t s = c->stream;
    unsigned long long unused = 0;
    if (c->est == kEstP2P) {
        double* hQ = hT + (size_t)B * 16;
        CTX_CHECK(c, hipMemcpyAsync(hQ, c->Q.p, (size_t)B * 12 * 8, hipMemcpyDeviceToHost, s));
        CTX_CHECK(c, hipStreamSynchronize(s));
        for (int b = 0; b < B; ++b) {
            for (int t = 0; t < 12; ++t) hT[16 * b + t] = hQ[12 * b + t];
            hT[16 * b + 12] = hT[16 * b + 13] = hT[16 * b + 14] = 0.0;
            hT[16 * b + 15] = 1.0;
        }
    } else {
        CTX_CHECK(c, hipMemcpyAsync(hT, c->T.p, (size_t)B * 16 * 8, hipMemcpyDeviceToHost, s));
    }
    CTX_CHECK(c, hipMemcpyAsync(hFit, c->out_fit.p, (size_t)B * 8, hipMemcpyDeviceToHost, s));
    CTX_CHECK(c, hipMemcpyAsync(hRmse, c->out_rmse.p, (size_t)B * 8, hipMemcpyDeviceToHost, s));
    CTX_CHECK(c, hipMemcpyAsync(hIters, c->out_iters.p, (size_t)B * 4, hipMemcpyDeviceToHost, s));
    std::vector<int64_t> nc((size_t)B);
    CTX_CHECK(c, d2h(nc.data(), c->out_ncorr.p, (size_t)B * 8, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    unsigned long long tiles_after = 0;
    if (c->count_tiles) CTX_CHECK(c, read_counters(c, tiles_after, unused, false));
    if (c->count_tiles) {
        const double t = (double)(tiles_after - tiles_before);
        c->stats.tiles += t;
        c->stats.pairs += t * kQuarter * (64.0 * kCQPT);  // pairs evaluated by the scan (t in quarters)
    }
    for (int b = 0; b < B; ++b) {
        std::memcpy(T_out + 16 * b, hT + 16 * b, 16 * sizeof(double));
        rmse_out[b] = hRmse[b];
        if (fitness_out) fitness_out[b] = hFit[b];
        if (iters_out) iters_out[b] = hIters[b];
        if (ncorr_out) ncorr_out[b] = nc[b];
        c->stats.iterations += hIters[b];
    }
    return ORPCD_OK;
}

// The ICP loop of every start of the batch set up by batch_setup (GICP or
// PointToPoint by c->est).  GICP outputs T (the ICP transform relative to the
// posed source); PointToPoint outputs T * G (registration_icp's result, init
// included).
int run_passes(orpcd_ctx* c, int B, const orpcd_gicp_params* p, double* T_out, double* rmse_out,
               double* fitness_out, int32_t* iters_out, int64_t* ncorr_out, int pass_begin, int pass_end) {
    const int64_t N = c->src.n;
    (void)N;
    double* hT = c->h64.p + (size_t)B * 12;
    double* hFit = hT + (size_t)B * (16 + 12 + 9 + 9 + 2);
    double* hRmse = hFit + B;
    int32_t* hAct = c->h32.p;
    int32_t* hDone = hAct + B;
    int32_t* hIters = hDone + B;
    hipStream_t s = c->stream;
    const double r2 = p->max_correspondence_distance * p->max_correspondence_distance;
    unsigned long long tiles_before = 0, unused = 0;
    if (c->profiling && c->opt.count_tiles) CTX_CHECK(c, read_counters(c, tiles_before, unused, false));
    int nact = B;
    static const bool trace = getenv("ORPCD_TRACE") != nullptr;
    const bool timed = c->profiling || trace;
    const int every = trace ? 1 : std::max(1, c->opt.sync_every);
    c->count_tiles = timed && c->opt.count_tiles;
    if (timed) {
        while ((int)c->ev_pool.size() < 3 * every) {
            hipEvent_t e;
            CTX_CHECK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));  // timing only: no cache writeback per record
            c->ev_pool.push_back(e);
        }
    }
    int pending = 0;  // timed passes since the last host sync
    // ORPCD_GAPS=1: GPU-side anatomy of every pass (events before the pass,
    // after the search, after the accumulation, after solve + next queries),
    // summed per batch and printed: where a batch's device time goes,
    // including idle gaps between kernels and around the host syncs
    static const bool gaps = getenv("ORPCD_GAPS") != nullptr;
    std::vector<hipEvent_t> gev;
    double g_search = 0, g_accum = 0, g_solve = 0, g_between = 0;
    hipEvent_t g_last = nullptr;
    if (gaps) {
        gev.resize((size_t)4 * (p->max_iteration + 2));
        for (auto& e : gev) CTX_CHECK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    }
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    const auto t_run = clk::now();
    const double sync_before = c->stats.host_sync_ms;
    int nsync = 0;
    double sync_max = 0.0;
    for (int pass = pass_begin; pass <= p->max_iteration && pass < pass_end && nact > 0; ++pass) {
        hipEvent_t* ev = timed ? &c->ev_pool[3 * pending] : nullptr;
        const auto tl = clk::now();
        hipEvent_t* ge = gaps ? &gev[(size_t)4 * pass] : nullptr;
        if (timed) CTX_CHECK(c, hipEventRecord(ev[0], s));
        if (gaps) CTX_CHECK(c, hipEventRecord(ge[0], s));
        const TgtBounds tb = target_bounds(c, hAct, nact);
        CTX_CHECK(c, launch_gicp_pass(c, nact, pass, r2, s, timed ? ev[1] : (gaps ? ge[1] : nullptr), tb));
        if (trace) CTX_CHECK(c, hipEventRecord(ev[2], s));  // accumulation time: traced runs only
        if (gaps) CTX_CHECK(c, hipEventRecord(ge[2], s));
        CTX_CHECK(c, launch_gicp_solve(c, nact, pass, *p, s, tb));
        if (gaps) CTX_CHECK(c, hipEventRecord(ge[3], s));
        c->stats.host_launch_ms += ms_since(tl);
        ++pending;
        c->stats.passes += nact;
        if (c->exact_live) c->stats.exact_queries += (double)nact * (double)c->src.n;
        // the host learns which starts finished only every few passes; a
        // finished start's blocks exit at once in the passes in between
        const bool sync = ((pass - pass_begin) % every) == every - 1 || pass == p->max_iteration || pass == pass_end - 1;
        if (!sync) continue;
        CTX_CHECK(c, hipMemcpyAsync(hDone, c->done.p, (size_t)B * 4, hipMemcpyDeviceToHost, s));
        unsigned long long tiles_now[2] = {0, 0};
        if (trace) CTX_CHECK(c, read_counters(c, tiles_now[0], tiles_now[1], true));
        const auto tw = clk::now();
        if (c->opt.sync_poll) {
            hipError_t e;
            while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
                if (ms_since(tw) > 120e3) {
                    c->err = "gicp: the device did not finish a pass interval within 120 s";
                    return ORPCD_EDEVICE;
                }
            }
            CTX_CHECK(c, e);
        } else {
            CTX_CHECK(c, hipStreamSynchronize(s));
        }
        const double waited = ms_since(tw);
        c->stats.host_sync_ms += waited;
        ++nsync;
        sync_max = std::max(sync_max, waited);
        if (gaps) {
            for (int q = pass - pending + 1; q <= pass; ++q) {
                hipEvent_t* g = &gev[(size_t)4 * q];
                float a = 0, b = 0, d = 0, e = 0;
                if (!timed) CTX_CHECK(c, hipEventElapsedTime(&a, g[0], g[1]));
                CTX_CHECK(c, hipEventElapsedTime(&b, g[1], g[2]));
                CTX_CHECK(c, hipEventElapsedTime(&d, g[2], g[3]));
                if (g_last) CTX_CHECK(c, hipEventElapsedTime(&e, g_last, g[0]));
                g_search += a;
                g_accum += b;
                g_solve += d;
                g_between += e;
                g_last = g[3];
            }
        }
        if (timed) {
            for (int q = 0; q < pending; ++q) {
                float ms = 0.f, ms2 = 0.f;
                CTX_CHECK(c, hipEventElapsedTime(&ms, c->ev_pool[3 * q], c->ev_pool[3 * q + 1]));
                if (trace) CTX_CHECK(c, hipEventElapsedTime(&ms2, c->ev_pool[3 * q + 1], c->ev_pool[3 * q + 2]));
                if (c->profiling) {
                    c->stats.launches += 1;
                    if (c->sched_live) c->stats.sched_launches += 1;
                    c->stats.ms += ms;
                    c->stats.accum_ms += ms2;
                }
                if (trace) {
                    static unsigned long long last = 0;
                    fprintf(stderr, "[orpcd] pass %3d nact %3d search %.3f ms accum %.3f ms quarters %llu max/wave %llu\n",
                            pass, nact, ms, ms2, tiles_now[0] - last, tiles_now[1]);
                    last = tiles_now[0];
                    if (getenv("ORPCD_PHASES")) {  // libraries built with -DORPCD_PHASES
                        std::vector<unsigned long long> h((size_t)kCounterSlots * kCounterStride);
                        CTX_CHECK(c, d2h(h.data(), c->counters.p, h.size() * 8, c->stream));
                        unsigned long long ph[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                        for (int q = 0; q < kCounterSlots; ++q)
                            for (int f = 0; f < 9; ++f) {
                                ph[f] += h[(size_t)q * kCounterStride + 2 + f];
                                h[(size_t)q * kCounterStride + 2 + f] = 0;
                            }
                        CTX_CHECK(c, h2d(c->counters.p, h.data(), h.size() * 8, c->stream));
                        const double w = ph[3] > 0 ? (double)ph[3] : 1.0;
                        fprintf(stderr, "[orpcd]   waves %llu cycles/wave: query load %.0f  search %.0f (culling %.0f)"
                                "  per wave: AABB rounds %.2f candidate tests %.2f improving tiles %.2f"
                                " queries wanting a returned candidate %.2f tiles staged %.2f\n",
                                ph[3], ph[0] / w, ph[2] / w, ph[1] / w, ph[4] / w, ph[5] / w, ph[6] / w, ph[7] / w,
                                ph[8] / w);
                    }
                }
            }
        }
        pending = 0;
        int k = 0;
        for (int b = 0; b < nact; ++b)
            if (!hDone[hAct[b]]) hAct[k++] = hAct[b];
        if (k != nact && k > 0) CTX_CHECK(c, hipMemcpyAsync(c->active.p, hAct, (size_t)k * 4, hipMemcpyHostToDevice, s));
        nact = k;
    }
    if (gaps) {
        float span = 0, pre = 0;
        if (g_last) CTX_CHECK(c, hipEventElapsedTime(&span, gev[0], g_last));
        if (c->gaps_ev0) CTX_CHECK(c, hipEventElapsedTime(&pre, c->gaps_ev0, gev[0]));
        fprintf(stderr, "[orpcd gaps] B %d: set-up host %.3f ms, device %.3f ms before pass 0; device span %.3f ms ="
                        " search %.3f + accumulation %.3f + solve/queries %.3f + between passes %.3f\n", B,
                c->gaps_setup_ms, pre, span, g_search, g_accum, g_solve, g_between);
        fprintf(stderr, "[orpcd gaps]   host: passes %.3f ms, %d device waits %.3f ms (longest %.3f)\n", ms_since(t_run),
                nsync, c->stats.host_sync_ms - sync_before, sync_max);
        for (auto e : gev) (void)hipEventDestroy(e);
    }
    if (c->exact_live) {  // entries re-searched over the batch (nn_exact_kernel adds each pass's count)
        unsigned long long tot = 0;
        CTX_CHECK(c, d2h(&tot, c->xtotal.p, 8, c->stream));
        if (tot >> 40) {  // a fused accumulation thread stopped waiting for its re-search (never expected)
            c->err = "exact_nn: a re-search result was not published in time";
            return ORPCD_EDEVICE;
        }
        c->stats.exact_filed += (double)tot;
    }
    return read_outputs(c, B, tiles_before, T_out, rmse_out, fitness_out, iters_out, ncorr_out);
}

}  // namespace

extern "C" {

int orpcd_sor(orpcd_ctx* c, const double* xyz, int64_t n, int32_t nb_neighbors, double std_ratio, int64_t* idx_out,
              int64_t* n_out, double* avg_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, n_out && (idx_out || n == 0), "sor: null argument");
    *n_out = 0;
    CTX_REQUIRE(c, nb_neighbors >= 1 && std_ratio > 0,
                "Illegal input parameters, the number of neighbors and standard deviation ratio must be positive.");
    CTX_REQUIRE(c, nb_neighbors <= kMaxKnn, "sor: nb_neighbors > 1024 is not supported by the device KNN");
    if (n == 0) return ORPCD_OK;
    CTX_REQUIRE(c, xyz && n > 0 && n < kMaxPoints, "sor: bad cloud size");
    CTX_REQUIRE(c, finite_cloud(xyz, n), "sor: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    double margin = 0.0;
    int rc = upload_layout(c, xyz, n, c->aux, true, &margin);
    if (rc) return rc;
    CTX_CHECK(c, c->scratch64b.ensure((size_t)n));
    CTX_CHECK(c, c->scratch64c.ensure(4));
    CTX_CHECK(c, c->scratch32.ensure((size_t)n + 1));
    CTX_CHECK(c, c->vox.flag.ensure((size_t)n));
    double* avg = c->scratch64b.p;
    CTX_CHECK(c, launch_knn_tiles(c->aux, c->scratch64a.p, nb_neighbors, -1.0, margin, true, nullptr, nullptr,
                                  nullptr, nullptr, s, avg, knn_lane(c, n)));
    CTX_CHECK(c, launch_sor_select(avg, n, std_ratio, c->scratch64c.p, c->vox.flag.p, c->scratch32.p,
                                   c->scratch32.p + n, c->vox.tmp, s));
    int32_t k = 0;
    CTX_CHECK(c, d2h(&k, c->scratch32.p + n, 4, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    std::vector<int32_t> kept((size_t)k);
    if (k > 0) CTX_CHECK(c, d2h(kept.data(), c->scratch32.p, (size_t)k * 4, s));
    if (avg_out) CTX_CHECK(c, d2h(avg_out, avg, (size_t)n * 8, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    for (int32_t i = 0; i < k; ++i) idx_out[i] = kept[i];
    *n_out = k;
    return ORPCD_OK;
}

int orpcd_voxel_down_sample(orpcd_ctx* c, const double* xyz, int64_t n, double voxel_size, double* out_xyz,
                            int64_t* n_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, n_out, "voxel_down_sample: null argument");
    *n_out = 0;
    CTX_REQUIRE(c, voxel_size > 0.0, "voxel_size <= 0.");
    if (n == 0) return ORPCD_OK;
    CTX_REQUIRE(c, xyz && n > 0 && n < kMaxPoints, "voxel_down_sample: bad cloud size");
    CTX_REQUIRE(c, finite_cloud(xyz, n), "voxel_down_sample: non-finite coordinates");
    double lo[3], hi[3], vmin[3];
    for (int a = 0; a < 3; ++a) lo[a] = hi[a] = xyz[a];
    for (int64_t i = 1; i < n; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], xyz[3 * i + a]);
            hi[a] = std::max(hi[a], xyz[3 * i + a]);
        }
    double ext = 0.0, cells = 0.0;
    for (int a = 0; a < 3; ++a) {
        vmin[a] = lo[a] - voxel_size * 0.5;
        ext = std::max(ext, (hi[a] + voxel_size * 0.5) - vmin[a]);
        cells = std::max(cells, std::floor((hi[a] - vmin[a]) / voxel_size) + 1.0);
    }
    CTX_REQUIRE(c, !(voxel_size * 2147483647.0 < ext), "voxel_size is too small.");
    CTX_REQUIRE(c, cells <= (double)(1 << 21), "voxel_down_sample: more than 2^21 voxels along an axis");
    CTX_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    CTX_CHECK(c, c->vox.xyz.ensure((size_t)n * 3));
    if (out_xyz) CTX_CHECK(c, c->vox.out.ensure((size_t)n * 3));
    CTX_CHECK(c, h2d(c->vox.xyz.p, xyz, (size_t)n * 24, s));
    int64_t nv = 0;
    CTX_CHECK(c, launch_voxel_down_sample(c->vox.xyz.p, n, vmin, voxel_size, c->vox, out_xyz ? c->vox.out.p : nullptr,
                                          &nv, s));
    if (out_xyz && nv > 0)
        CTX_CHECK(c, d2h(out_xyz, c->vox.out.p, (size_t)nv * 24, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    *n_out = nv;
    return ORPCD_OK;
}

int orpcd_farthest_downsample(orpcd_ctx* c, const double* xyz, int64_t n, int32_t sample_size, int64_t first,
                              int64_t* idx_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && idx_out, "farthest_downsample: null argument");
    CTX_REQUIRE(c, n > 0 && n < kMaxPoints, "farthest_downsample: empty cloud");
    CTX_REQUIRE(c, sample_size > 0, "farthest_downsample: sample_size must be > 0");
    CTX_REQUIRE(c, first >= 0 && first < n, "farthest_downsample: first index out of range");
    CTX_REQUIRE(c, finite_cloud(xyz, n), "farthest_downsample: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    if (c->fps_blocks == 0) c->fps_blocks = fps_max_blocks(c->device);
    CTX_REQUIRE(c, c->fps_blocks > 0 && fps_points_per_thread(n, c->fps_blocks) > 0,
                "farthest_downsample: cloud too large for one cooperative launch");
    hipStream_t s = c->stream;
    CTX_CHECK(c, c->vox.xyz.ensure((size_t)n * 3));
    CTX_CHECK(c, c->vox.idx64.ensure((size_t)sample_size));
    CTX_CHECK(c, c->scratch64c.ensure((size_t)2 * c->fps_blocks));
    CTX_CHECK(c, c->vox.tag.ensure((size_t)2 * c->fps_blocks));
    CTX_CHECK(c, c->scratch32.ensure(2));
    CTX_CHECK(c, h2d(c->vox.xyz.p, xyz, (size_t)n * 24, s));
    unsigned* err = reinterpret_cast<unsigned*>(c->scratch32.p);
    CTX_CHECK(c, launch_fps(c->vox.xyz.p, n, (int)first, sample_size, c->fps_blocks, c->vox.idx64.p,
                            c->scratch64c.p, c->vox.tag.p, err, s));
    unsigned herr = 0;
    CTX_CHECK(c, d2h(idx_out, c->vox.idx64.p, (size_t)sample_size * 8, s));
    CTX_CHECK(c, d2h(&herr, err, 4, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    if (herr) {
        c->err = "farthest_downsample: blocks of the cooperative launch were not co-resident";
        return ORPCD_EDEVICE;
    }
    return ORPCD_OK;
}

int orpcd_set_source_rows(orpcd_ctx* c, const double* xyz, int64_t n, int64_t row_begin, int64_t row_end) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && n > 0, "set_source_rows: empty source cloud");
    CTX_REQUIRE(c, n < kMaxPoints, "set_source_rows: too many points");
    CTX_REQUIRE(c, row_begin >= 0 && row_begin < row_end && row_end <= n, "set_source_rows: bad row range");
    CTX_REQUIRE(c, finite_cloud(xyz, n), "set_source_rows: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    // KNN-20 covariances of this shard's rows against the full cloud (input
    // order; the other rows' are not computed: each rank computes its own)
    double margin = 0.0;
    int rc = upload_layout(c, xyz, n, c->aux, true, &margin);
    if (rc) return rc;
    const int64_t nrows = row_end - row_begin;
    CTX_CHECK(c, c->scratch64b.ensure((size_t)n * 6));
    CTX_CHECK(c, c->scratch32.ensure((size_t)nrows));
    CTX_CHECK(c, launch_rows_to_positions(c->aux.perm.p, n, row_begin, nrows, c->scratch32.p, c->stream));
    rc = source_ties_detect(c, c->aux, c->scratch64a.p, xyz, n, margin, true, c->scratch64b.p, c->scratch32.p, nrows);
    if (rc) return rc;
    // the shard's rows in their own Morton layout, covariances gathered to it
    const int64_t ns = row_end - row_begin;
    rc = upload_layout(c, xyz + 3 * row_begin, ns, c->src, true);
    if (rc) return rc;
    CTX_CHECK(c, c->sraw.ensure((size_t)ns * 6));
    CTX_CHECK(c, launch_gather_rows(c->scratch64b.p, c->src.perm.p, row_begin, ns, 6, c->sraw.p, c->stream));
    if (!c->ties.pt.empty()) {  // the ties on this rank's rows: their Morton positions
        std::vector<int32_t> perm((size_t)ns), inv((size_t)ns);
        CTX_CHECK(c, d2h(perm.data(), c->src.perm.p, (size_t)ns * 4, c->stream));
        CTX_CHECK(c, hipStreamSynchronize(c->stream));
        for (int64_t k = 0; k < ns; ++k) inv[(size_t)perm[k]] = (int32_t)k;
        for (size_t f = 0; f < c->ties.pt.size(); ++f) {
            const int64_t i = c->ties.pt[f];
            c->ties.pos[f] = (i >= row_begin && i < row_end) ? inv[(size_t)(i - row_begin)] : -1;
        }
    }
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    c->src_cov = true;
    return ORPCD_OK;
}

int orpcd_gicp_shard_begin(orpcd_ctx* c, const double* R0, const double* t0, const orpcd_gicp_params* p,
                           int64_t n_total) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, R0 && t0 && p, "gicp_shard_begin: null argument");
    CTX_REQUIRE(c, c->src.n > 0 && c->tgt.n > 0, "gicp_shard_begin: set the target and the source rows first");
    CTX_REQUIRE(c, c->src_cov, "gicp_shard_begin: the source rows have no covariances (orpcd_set_source_rows)");
    CTX_REQUIRE(c, n_total >= c->src.n, "gicp_shard_begin: n_total smaller than this rank's rows");
    CTX_REQUIRE(c, p->max_correspondence_distance > 0 && p->max_iteration >= 0 && p->epsilon >= 0,
                "gicp_shard_begin: bad parameters");
    CTX_CHECK(c, hipSetDevice(c->device));
    int rc = targets_for_epsilon(c, 1, p->epsilon);
    if (rc) return rc;
    c->batch_ntgt = 1;
    rc = batch_setup(c, R0, t0, 1, p);
    if (rc) return rc;
    CTX_CHECK(c, c->scratch64c.ensure(kNacc));
    c->shard.begun = true;
    c->shard.pass = 0;
    c->shard.n_total = n_total;
    c->shard.p = *p;
    return ORPCD_OK;
}

int orpcd_gicp_shard_pass(orpcd_ctx* c, double* sums_out, int32_t* active) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, sums_out && active, "gicp_shard_pass: null argument");
    CTX_REQUIRE(c, c->shard.begun, "gicp_shard_pass: call orpcd_gicp_shard_begin first");
    int32_t done = 0;
    CTX_CHECK(c, d2h(&done, c->done.p, 4, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    *active = done ? 0 : 1;
    for (int v = 0; v < kNacc; ++v) sums_out[v] = 0.0;
    if (done) return ORPCD_OK;
    const double r2 = c->shard.p.max_correspondence_distance * c->shard.p.max_correspondence_distance;
    const bool timed = c->profiling;
    c->count_tiles = timed && c->opt.count_tiles;
    unsigned long long tiles0 = 0, tiles1 = 0, unused = 0;
    if (timed) {
        while (c->ev_pool.size() < 3) {
            hipEvent_t e;
            CTX_CHECK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));  // timing only: no cache writeback per record
            c->ev_pool.push_back(e);
        }
        CTX_CHECK(c, read_counters(c, tiles0, unused, false));
        CTX_CHECK(c, hipEventRecord(c->ev_pool[0], c->stream));
    }
    CTX_CHECK(c, launch_gicp_pass(c, 1, c->shard.pass, r2, c->stream, timed ? c->ev_pool[1] : nullptr,
                                  one_target()));
    if (timed) CTX_CHECK(c, hipEventRecord(c->ev_pool[2], c->stream));
    CTX_CHECK(c, launch_reduce_partials(c, 0, c->scratch64c.p, c->stream));
    CTX_CHECK(c, d2h(sums_out, c->scratch64c.p, kNacc * 8, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    if (timed) {
        float ms = 0.f, ms2 = 0.f;
        CTX_CHECK(c, hipEventElapsedTime(&ms, c->ev_pool[0], c->ev_pool[1]));
        CTX_CHECK(c, hipEventElapsedTime(&ms2, c->ev_pool[1], c->ev_pool[2]));
        CTX_CHECK(c, read_counters(c, tiles1, unused, false));
        c->stats.launches += 1;
        c->stats.ms += ms;
        c->stats.accum_ms += ms2;
        c->stats.tiles += (double)(tiles1 - tiles0);
        c->stats.pairs += (double)(tiles1 - tiles0) * kQuarter * (64.0 * kCQPT);
    }
    c->stats.passes += 1;
    return ORPCD_OK;
}

int orpcd_gicp_shard_update(orpcd_ctx* c, const double* sums_in, int32_t* done_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, sums_in && done_out, "gicp_shard_update: null argument");
    CTX_REQUIRE(c, c->shard.begun, "gicp_shard_update: call orpcd_gicp_shard_begin first");
    CTX_CHECK(c, h2d(c->scratch64c.p, sums_in, kNacc * 8, c->stream));
    CTX_CHECK(c, launch_gicp_solve_sums(c, c->scratch64c.p, c->shard.n_total, c->shard.pass, c->shard.p, c->stream));
    int32_t done = 0;
    CTX_CHECK(c, d2h(&done, c->done.p, 4, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    c->shard.pass += 1;
    *done_out = done;
    return ORPCD_OK;
}

int orpcd_gicp_shard_result(orpcd_ctx* c, double* T_out, double* rmse_out, double* fitness_out, int32_t* iters_out,
                            int64_t* ncorr_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, T_out && rmse_out, "gicp_shard_result: null argument");
    CTX_REQUIRE(c, c->shard.begun, "gicp_shard_result: call orpcd_gicp_shard_begin first");
    int32_t done = 0, iters = 0;
    double fit = 0.0;
    int64_t nc = 0;
    hipStream_t s = c->stream;
    CTX_CHECK(c, d2h(&done, c->done.p, 4, s));
    CTX_CHECK(c, d2h(T_out, c->T.p, 16 * 8, s));
    CTX_CHECK(c, d2h(rmse_out, c->out_rmse.p, 8, s));
    CTX_CHECK(c, d2h(&fit, c->out_fit.p, 8, s));
    CTX_CHECK(c, d2h(&iters, c->out_iters.p, 4, s));
    CTX_CHECK(c, d2h(&nc, c->out_ncorr.p, 8, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    CTX_REQUIRE(c, done, "gicp_shard_result: the start has not finished");
    if (fitness_out) *fitness_out = fit;
    if (iters_out) *iters_out = iters;
    if (ncorr_out) *ncorr_out = nc;
    c->stats.iterations += iters;
    return ORPCD_OK;
}

#define CTX_RCCL(ctx, call)                                                                         \
    do {                                                                                            \
        const ncclResult_t r_ = (call);                                                             \
        if (r_ != ncclSuccess) {                                                                    \
            (ctx)->err = std::string(#call) + ": " + rccl_api().error_string(r_);                   \
            return ORPCD_EDEVICE;                                                                   \
        }                                                                                           \
    } while (0)

int orpcd_comm_unique_id(uint8_t* id_out) {
    if (!id_out) return ORPCD_EINVAL;
    const RcclApi& api = rccl_api();
    if (!api.ok) return ORPCD_EDEVICE;
    ncclUniqueId id;
    if (api.get_unique_id(&id) != ncclSuccess) return ORPCD_EDEVICE;
    std::memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return ORPCD_OK;
}

int orpcd_comm_init(orpcd_ctx* c, int32_t nranks, int32_t rank, const uint8_t* id) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, id && nranks >= 1 && rank >= 0 && rank < nranks, "comm_init: bad arguments");
    const RcclApi& api = rccl_api();
    CTX_REQUIRE(c, api.ok, "comm_init: " + api.err);
    CTX_CHECK(c, hipSetDevice(c->device));
    (void)orpcd_comm_destroy(c);
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    CTX_RCCL(c, api.comm_init_rank(&comm, nranks, uid, rank));
    c->comm = comm;
    c->comm_ranks = nranks;
    c->comm_rank = rank;
    return ORPCD_OK;
}

int orpcd_comm_destroy(orpcd_ctx* c) {
    if (!c) return ORPCD_EINVAL;
    if (c->comm) {
        (void)hipStreamSynchronize(c->stream);
        (void)rccl_api().comm_destroy((ncclComm_t)c->comm);
    }
    c->comm = nullptr;
    c->comm_ranks = c->comm_rank = 0;
    return ORPCD_OK;
}

// The row-sharded start's pass loop with the collective on the device: per
// pass the local partials are reduced to the 29 sums (the same fixed-order
// kernel as orpcd_gicp_shard_pass), all-reduced by RCCL on the library's
// stream, and solved from the global sums (as orpcd_gicp_shard_update); the
// host reads the done flag only every sync_every passes.  Every rank computes
// the same global sums, hence the same done pass, so all ranks enqueue the
// same collectives; passes enqueued after the start finished are no-ops (every
// kernel skips a done start; their sums go unused).
// Target covariances split by Morton rows (SURVEY.md §8(e), C5's row split):
// every rank builds the whole target's layout and seed grid (the search needs
// them), but runs the KNN-20 covariance pass only over its slice of
// kTile-aligned Morton rows; one all-gather assembles the rest -- in place on
// the device through the context's RCCL communicator when it has one of
// nranks ranks, otherwise by the caller (orpcd_target_cov_rows on every rank,
// orpcd_set_target_cov with the concatenation: a host all-gather).
static int64_t target_slice(int64_t m, int nranks) {
    return ((m + nranks - 1) / nranks + kTile - 1) / kTile * kTile;
}

int orpcd_set_target_rows(orpcd_ctx* c, const double* xyz, int64_t m, double epsilon, int32_t rank, int32_t nranks,
                          int64_t* row_begin, int64_t* row_end) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && m > 0, "set_target_rows: empty target cloud");
    CTX_REQUIRE(c, m < kMaxPoints, "set_target_rows: too many points");
    CTX_REQUIRE(c, nranks >= 1 && nranks <= 65536 && rank >= 0 && rank < nranks, "set_target_rows: bad rank");
    CTX_REQUIRE(c, epsilon >= 0, "set_target_rows: epsilon must be >= 0");
    CTX_REQUIRE(c, finite_cloud(xyz, m), "set_target_rows: non-finite coordinates");
    const bool device_gather = nranks > 1 && c->comm;
    CTX_REQUIRE(c, !device_gather || (c->comm_ranks == nranks && c->comm_rank == rank),
                "set_target_rows: rank / nranks differ from the communicator's (orpcd_comm_init)");
    CTX_CHECK(c, hipSetDevice(c->device));
    c->ntgt = 0;
    c->last_B = 0;
    double margin = 0.0;
    int rc = upload_layout(c, xyz, m, c->tgts[0], true, &margin);
    if (rc) return rc;
    CTX_CHECK(c, prepare_seed_grid(c->tgts[0]));
    const int64_t slice = target_slice(m, nranks);
    const int64_t lo = std::min(m, (int64_t)rank * slice), hi = std::min(m, lo + slice);
    CTX_CHECK(c, c->tcovs[0].ensure((size_t)(slice * nranks) * kCovW));
    CTX_CHECK(c, c->scratch64b.ensure((size_t)m * 6));
    double* tcov = c->tcovs[0].p;
    if (hi > lo) {
        CTX_CHECK(c, launch_knn_cov_range(c->tgts[0], c->scratch64a.p, 20, margin, c->scratch64b.p, lo, hi,
                                          knn_lane(c, m), c->stream));
        CTX_CHECK(c, launch_normals_cov(c->scratch64b.p + lo * 6, hi - lo, nullptr, 1, epsilon, nullptr,
                                        ORPCD_NORMAL_COV ? nullptr : tcov + lo * kCovW, c->stream,
                                        ORPCD_NORMAL_COV ? tcov + lo * kCovW : nullptr));
    }
    if (device_gather) {
        const RcclApi& api = rccl_api();
        CTX_RCCL(c, api.all_gather(tcov + (size_t)rank * slice * kCovW, tcov, (size_t)slice * kCovW, ncclFloat64,
                                   (ncclComm_t)c->comm, c->stream));
    }
    c->tgt_eps[0] = epsilon;
    c->tgt_host[0].clear();  // rebuilt from the device layout if another epsilon is asked for
    CTX_CHECK(c, c->tdesc.ensure(kMaxTargets));
    write_target_desc(c->tgts[0], tcov, c->opt.seed_reps, c->opt.seed_grid != 0, c->tdesc_h[0]);
    CTX_CHECK(c, h2d(c->tdesc.p, &c->tdesc_h[0], sizeof(TargetDesc), c->stream));
    CTX_CHECK(c, seed_grids(c, 0, 1));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    c->tgt_rows[0] = lo;
    c->tgt_rows[1] = hi;
    if (row_begin) *row_begin = lo;
    if (row_end) *row_end = hi;
    // complete (usable by the GICP calls) once every row is there
    if (nranks == 1 || device_gather) c->ntgt = 1;
    return ORPCD_OK;
}

// ---------------------------------------------- target layouts as buffers
// One device buffer per target: a header, then the layout's arrays at
// 256-byte aligned offsets (orpcd_target_layout_bytes / get / set).
namespace {
constexpr uint64_t kLayoutMagic = 0x31304c4443505230ull;  // "0RPCDL01"
enum { kLayXyz, kLayPerm, kLayP4, kLayTlo, kLayThi, kLayQbox, kLaySlo, kLayShi, kLaySgrid, kLayTcov, kLaySections };
struct LayoutHeader {
    uint64_t magic;
    int64_t n, npad, ntiles, nsuper;
    double org[3], lo[3], hi[3], eps;
    float sg_lo[3], sg_inv[3];
    int32_t has_sgrid, cov_w;
    uint64_t off[kLaySections], len[kLaySections];  // bytes
    uint64_t total;
};
LayoutHeader layout_header(const CloudLayout& L, double eps) {
    LayoutHeader h{};
    h.magic = kLayoutMagic;
    h.n = L.n;
    h.npad = L.npad;
    h.ntiles = L.ntiles;
    h.nsuper = L.nsuper;
    for (int a = 0; a < 3; ++a) {
        h.org[a] = L.org[a];
        h.lo[a] = L.lo[a];
        h.hi[a] = L.hi[a];
        h.sg_lo[a] = L.sg_lo[a];
        h.sg_inv[a] = L.sg_inv[a];
    }
    h.eps = eps;
    h.has_sgrid = L.sgrid.n > 0;
    h.cov_w = kCovW;
    const uint64_t len[kLaySections] = {
        (uint64_t)L.npad * 3 * 8,  (uint64_t)L.n * 4,
        (uint64_t)L.npad * 16,     (uint64_t)L.ntiles * 16,
        (uint64_t)L.ntiles * 16,   (uint64_t)L.ntiles * 2 * kNQ * 16,
        (uint64_t)L.nsuper * 16,   (uint64_t)L.nsuper * 16,
        h.has_sgrid ? (uint64_t)kSeedGrid * kSeedGrid * kSeedGrid * 4 : 0,
        (uint64_t)L.n * kCovW * 8};
    uint64_t at = (sizeof(LayoutHeader) + 255) / 256 * 256;
    for (int i = 0; i < kLaySections; ++i) {
        h.off[i] = at;
        h.len[i] = len[i];
        at += (len[i] + 255) / 256 * 256;
    }
    h.total = at;
    return h;
}
}  // namespace

int64_t orpcd_target_layout_bytes(orpcd_ctx* c, int32_t k) {
    if (!c) return -1;
    if (k < 0 || k >= c->ntgt) {
        c->err = "target_layout_bytes: no such target";
        return -1;
    }
    return (int64_t)layout_header(c->tgts[k], c->tgt_eps[k]).total;
}

int orpcd_device_alloc(orpcd_ctx* c, int64_t bytes, void** dev_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, dev_out && bytes > 0, "device_alloc: bad arguments");
    *dev_out = nullptr;
    CTX_CHECK(c, hipSetDevice(c->device));
    CTX_CHECK(c, hipMalloc(dev_out, (size_t)bytes));  // hipMalloc: 256-byte aligned at least
    return ORPCD_OK;
}

int orpcd_device_free(orpcd_ctx* c, void* dev) {
    if (!c) return ORPCD_EINVAL;
    if (!dev) return ORPCD_OK;
    CTX_CHECK(c, hipSetDevice(c->device));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    CTX_CHECK(c, hipFree(dev));
    return ORPCD_OK;
}

int orpcd_get_target_layout(orpcd_ctx* c, int32_t k, void* dev_out, int64_t bytes) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, k >= 0 && k < c->ntgt, "get_target_layout: no such target");
    const CloudLayout& L = c->tgts[k];
    const LayoutHeader h = layout_header(L, c->tgt_eps[k]);
    CTX_REQUIRE(c, dev_out && bytes >= (int64_t)h.total && ((uintptr_t)dev_out & 255) == 0,
                "get_target_layout: the buffer is smaller than orpcd_target_layout_bytes or not 256-byte aligned");
    CTX_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    unsigned char* o = static_cast<unsigned char*>(dev_out);
    const void* src[kLaySections] = {L.xyz64.p, L.perm.p, L.p4.p, L.tlo.p, L.thi.p, L.qbox.p, L.slo.p, L.shi.p,
                                     L.sgrid.p, c->tcovs[k].p};
    CTX_CHECK(c, h2d(o, &h, sizeof(h), s));
    for (int i = 0; i < kLaySections; ++i)
        if (h.len[i]) CTX_CHECK(c, hipMemcpyAsync(o + h.off[i], src[i], h.len[i], hipMemcpyDeviceToDevice, s));
    CTX_CHECK(c, hipStreamSynchronize(s));
    return ORPCD_OK;
}

int orpcd_set_target_layouts(orpcd_ctx* c, const void* const* dev_in, int32_t ntargets) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, dev_in && ntargets >= 1 && ntargets <= kMaxTargets, "set_target_layouts: 1 to 16 layouts");
    CTX_CHECK(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    c->ntgt = 0;
    c->last_B = 0;  // the last batch's correspondences refer to the old targets
    for (int k = 0; k < ntargets; ++k) {
        CTX_REQUIRE(c, dev_in[k], "set_target_layouts: null buffer");
        LayoutHeader h;
        CTX_CHECK(c, d2h(&h, dev_in[k], sizeof(h), s));
        CTX_CHECK(c, hipStreamSynchronize(s));
        CTX_REQUIRE(c, h.magic == kLayoutMagic && h.cov_w == kCovW && h.n > 0 && h.n < kMaxPoints,
                    "set_target_layouts: not a target layout of this library (orpcd_get_target_layout)");
        CloudLayout& L = c->tgts[k];
        L.n = h.n;
        L.npad = h.npad;
        L.ntiles = h.ntiles;
        L.nsuper = h.nsuper;
        for (int a = 0; a < 3; ++a) {
            L.org[a] = h.org[a];
            L.lo[a] = h.lo[a];
            L.hi[a] = h.hi[a];
        }
        const LayoutHeader want = layout_header(L, h.eps);  // the sizes this layout implies
        for (int i = 0; i < kLaySections; ++i)
            CTX_REQUIRE(c, i == kLaySgrid ? (h.len[i] == 0 || h.len[i] == (uint64_t)kSeedGrid * kSeedGrid * kSeedGrid * 4)
                                          : h.len[i] == want.len[i],
                        "set_target_layouts: inconsistent layout header");
        CTX_CHECK(c, L.xyz64.ensure((size_t)L.npad * 3));
        CTX_CHECK(c, L.perm.ensure((size_t)L.n));
        CTX_CHECK(c, L.p4.ensure((size_t)L.npad));
        CTX_CHECK(c, L.tlo.ensure((size_t)L.ntiles));
        CTX_CHECK(c, L.thi.ensure((size_t)L.ntiles));
        CTX_CHECK(c, L.qbox.ensure((size_t)L.ntiles * 2 * kNQ));
        CTX_CHECK(c, L.slo.ensure((size_t)L.nsuper));
        CTX_CHECK(c, L.shi.ensure((size_t)L.nsuper));
        CTX_CHECK(c, prepare_seed_grid(L));  // sgrid / its scratch, sg_lo / sg_inv from the box
        for (int a = 0; a < 3; ++a) {
            L.sg_lo[a] = h.sg_lo[a];
            L.sg_inv[a] = h.sg_inv[a];
        }
        CTX_CHECK(c, c->tcovs[k].ensure((size_t)L.n * kCovW));
        void* dst[kLaySections] = {L.xyz64.p, L.perm.p, L.p4.p, L.tlo.p, L.thi.p, L.qbox.p, L.slo.p, L.shi.p,
                                   L.sgrid.p, c->tcovs[k].p};
        const unsigned char* in = static_cast<const unsigned char*>(dev_in[k]);
        for (int i = 0; i < kLaySections; ++i)
            if (h.len[i]) CTX_CHECK(c, hipMemcpyAsync(dst[i], in + h.off[i], h.len[i], hipMemcpyDeviceToDevice, s));
        c->tgt_eps[k] = h.eps;
        c->tgt_host[k].clear();  // rebuilt from the device layout if another epsilon is asked for
        CTX_CHECK(c, c->tdesc.ensure(kMaxTargets));
        write_target_desc(L, c->tcovs[k].p, c->opt.seed_reps, c->opt.seed_grid != 0, c->tdesc_h[k]);
        CTX_CHECK(c, h2d(c->tdesc.p + k, &c->tdesc_h[k], sizeof(TargetDesc), s));
        if (!h.has_sgrid) CTX_CHECK(c, seed_grids(c, k, 1));
    }
    CTX_CHECK(c, hipStreamSynchronize(s));
    c->ntgt = ntargets;
    return ORPCD_OK;
}

int32_t orpcd_target_cov_width(void) { return kCovW; }

int orpcd_target_cov_rows(orpcd_ctx* c, int64_t row_begin, int64_t row_end, double* out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, out && c->tgt.n > 0 && c->tcov.n >= (size_t)c->tgt.n * kCovW, "target_cov_rows: no target");
    const bool whole = c->ntgt > 0;
    CTX_REQUIRE(c, row_begin >= (whole ? 0 : c->tgt_rows[0]) && row_end <= (whole ? c->tgt.n : c->tgt_rows[1]) &&
                       row_begin <= row_end,
                "target_cov_rows: rows outside those computed here");
    CTX_CHECK(c, hipSetDevice(c->device));
    CTX_CHECK(c, d2h(out, c->tcov.p + row_begin * kCovW, (size_t)(row_end - row_begin) * kCovW * 8, c->stream));
    return ORPCD_OK;
}

int orpcd_set_target_cov(orpcd_ctx* c, const double* cov) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, cov && c->tgt.n > 0 && c->tcov.n >= (size_t)c->tgt.n * kCovW,
                "set_target_cov: no target layout (orpcd_set_target_rows)");
    CTX_CHECK(c, hipSetDevice(c->device));
    CTX_CHECK(c, h2d(c->tcov.p, cov, (size_t)c->tgt.n * kCovW * 8, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    c->ntgt = 1;
    return ORPCD_OK;
}

int orpcd_gicp_shard_run(orpcd_ctx* c, int32_t* passes_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, c->shard.begun, "gicp_shard_run: call orpcd_gicp_shard_begin first");
    CTX_REQUIRE(c, c->comm, "gicp_shard_run: no communicator (orpcd_comm_init)");
    CTX_CHECK(c, hipSetDevice(c->device));
    const RcclApi& api = rccl_api();
    const auto& p = c->shard.p;
    const double r2 = p.max_correspondence_distance * p.max_correspondence_distance;
    hipStream_t s = c->stream;
    c->count_tiles = false;
    const int every = std::max(1, c->opt.sync_every);
    int32_t done = 0;
    CTX_CHECK(c, d2h(&done, c->done.p, 4, s));
    while (!done) {
        for (int k = 0; k < every; ++k) {
            CTX_CHECK(c, launch_gicp_pass(c, 1, c->shard.pass, r2, s, nullptr, one_target()));
            CTX_CHECK(c, launch_reduce_partials(c, 0, c->scratch64c.p, s));
            CTX_RCCL(c, api.all_reduce(c->scratch64c.p, c->scratch64c.p, kNacc, ncclFloat64, ncclSum,
                                       (ncclComm_t)c->comm, s));
            CTX_CHECK(c, launch_gicp_solve_sums(c, c->scratch64c.p, c->shard.n_total, c->shard.pass, p, s));
            c->shard.pass += 1;
            c->stats.passes += 1;
        }
        CTX_CHECK(c, d2h(&done, c->done.p, 4, s));  // drains the stream
    }
    if (passes_out) *passes_out = c->shard.pass;
    return ORPCD_OK;
}

int orpcd_nn1_radius(orpcd_ctx* c, const double* q, int64_t nq, const double* t, int64_t m, double radius,
                     int32_t* idx_out, double* d2_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, q && t && idx_out && d2_out && nq >= 0 && m > 0, "nn1_radius: bad arguments");
    CTX_REQUIRE(c, radius > 0, "nn1_radius: radius must be > 0");
    CTX_REQUIRE(c, nq < kMaxPoints && m < kMaxPoints, "nn1_radius: too many points");
    CTX_REQUIRE(c, finite_cloud(t, m) && finite_cloud(q, nq), "nn1_radius: non-finite coordinates");
    if (nq == 0) return ORPCD_OK;
    CTX_CHECK(c, hipSetDevice(c->device));
    int rc = upload_layout(c, t, m, c->aux, true);
    if (rc) return rc;
    CTX_CHECK(c, c->scratch64b.ensure((size_t)nq * 3));
    CTX_CHECK(c, c->scratch64c.ensure((size_t)nq));
    CTX_CHECK(c, c->scratch32.ensure((size_t)nq));
    CTX_CHECK(c, h2d(c->scratch64b.p, q, (size_t)nq * 24, c->stream));
    CTX_CHECK(c, launch_nn1(c->scratch64b.p, nq, c->aux, radius * radius, c->scratch32.p, c->scratch64c.p, c->qorder,
                            c->stream));
    CTX_CHECK(c, d2h(idx_out, c->scratch32.p, (size_t)nq * 4, c->stream));
    CTX_CHECK(c, d2h(d2_out, c->scratch64c.p, (size_t)nq * 8, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    return ORPCD_OK;
}

int orpcd_estimate_normals(orpcd_ctx* c, const double* xyz, int64_t n, int32_t knn, double radius, double epsilon,
                           double* normals_out, double* rawcov_out, double* gicpcov_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && n > 0, "estimate_normals: empty cloud");
    CTX_REQUIRE(c, n < kMaxPoints, "estimate_normals: too many points");
    CTX_REQUIRE(c, knn > 0 && knn <= kMaxKnn, "estimate_normals: knn must be in [1, 1024]");
    CTX_REQUIRE(c, finite_cloud(xyz, n), "estimate_normals: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    double margin = 0.0;
    int rc = upload_layout(c, xyz, n, c->aux, true, &margin);
    if (rc) return rc;
    // input-order results in scratch64c: raw(6n) | normals(3n) | cov(6n)
    CTX_CHECK(c, c->scratch64c.ensure((size_t)n * 15));
    double* uraw = c->scratch64c.p;
    double* unrm = uraw + 6 * n;
    double* ucov = unrm + 3 * n;
    CTX_CHECK(c, launch_knn_tiles(c->aux, c->scratch64a.p, knn, radius, margin, true, uraw, nullptr, nullptr, nullptr,
                                  c->stream, nullptr, knn_lane(c, n)));
    CTX_CHECK(c, launch_normals_cov(uraw, n, nullptr, 1, epsilon, unrm, epsilon >= 0 ? ucov : nullptr, c->stream));
    std::vector<double> raw6((size_t)n * 6), cov6;
    CTX_CHECK(c, d2h(raw6.data(), uraw, (size_t)n * 48, c->stream));
    if (normals_out) CTX_CHECK(c, d2h(normals_out, unrm, (size_t)n * 24, c->stream));
    if (gicpcov_out && epsilon >= 0) {
        cov6.resize((size_t)n * 6);
        CTX_CHECK(c, d2h(cov6.data(), ucov, (size_t)n * 48, c->stream));
    }
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    auto expand = [n](const std::vector<double>& s6, double* o9) {
        for (int64_t i = 0; i < n; ++i) {
            const double* s = &s6[(size_t)6 * i];
            double* o = o9 + 9 * i;
            o[0] = s[0];
            o[1] = s[1];
            o[2] = s[2];
            o[3] = s[1];
            o[4] = s[3];
            o[5] = s[4];
            o[6] = s[2];
            o[7] = s[4];
            o[8] = s[5];
        }
    };
    if (rawcov_out) expand(raw6, rawcov_out);
    if (gicpcov_out && epsilon >= 0) expand(cov6, gicpcov_out);
    return ORPCD_OK;
}

int orpcd_fpfh(orpcd_ctx* c, const double* xyz, int64_t n, double normal_radius, int32_t normal_knn,
               double fpfh_radius, int32_t fpfh_knn, double* normals_out, double* feat_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && n > 0 && feat_out && n < kMaxPoints, "fpfh: bad arguments");
    CTX_REQUIRE(c, finite_cloud(xyz, n), "fpfh: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    CTX_CHECK(c, c->fgr.xyz[0].ensure((size_t)n * 3));
    CTX_CHECK(c, h2d(c->fgr.xyz[0].p, xyz, (size_t)n * 24, c->stream));
    int rc = fpfh_device(c, xyz, 0, n, normal_radius, normal_knn, fpfh_radius, fpfh_knn);
    if (rc) return rc;
    if (normals_out)
        CTX_CHECK(c, d2h(normals_out, c->fgr.nrm.p, (size_t)n * 24, c->stream));
    CTX_CHECK(c, d2h_2d(feat_out, 33 * sizeof(double), c->fgr.feat[0].p, kFeatDim * sizeof(double), 33 * sizeof(double), (size_t)n, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    return ORPCD_OK;
}

int orpcd_fpfh_from_normals(orpcd_ctx* c, const double* xyz, const double* normals, int64_t n,
                            double fpfh_radius, int32_t fpfh_knn, double* feat_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, xyz && normals && n > 0 && feat_out && n < kMaxPoints, "fpfh_from_normals: bad arguments");
    CTX_REQUIRE(c, fpfh_knn > 0 && fpfh_knn <= kMaxKnn, "fpfh: knn must be in [1, 1024]");
    CTX_REQUIRE(c, fpfh_radius > 0, "fpfh: radii must be > 0");
    CTX_REQUIRE(c, finite_cloud(xyz, n) && finite_cloud(normals, n), "fpfh_from_normals: non-finite values");
    CTX_CHECK(c, hipSetDevice(c->device));
    int rc = fpfh_buffers(c, 0, n, fpfh_knn);
    if (rc) return rc;
    CTX_CHECK(c, c->fgr.xyz[0].ensure((size_t)n * 3));
    CTX_CHECK(c, h2d(c->fgr.xyz[0].p, xyz, (size_t)n * 24, c->stream));
    CTX_CHECK(c, h2d(c->fgr.nrm.p, normals, (size_t)n * 24, c->stream));
    rc = features_device(c, xyz, 0, n, fpfh_radius, fpfh_knn, 0.0);
    if (rc) return rc;
    CTX_CHECK(c, d2h_2d(feat_out, 33 * sizeof(double), c->fgr.feat[0].p, kFeatDim * sizeof(double), 33 * sizeof(double), (size_t)n, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    return ORPCD_OK;
}

int orpcd_fgr(orpcd_ctx* c, const double* src, int64_t n, const double* tgt, int64_t m, const double* src_feat,
              const double* tgt_feat, const orpcd_fgr_params* p, double* T_out, double* fitness_out,
              double* rmse_out, int64_t* ncorr_out, int64_t* n_mutual_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, src && tgt && src_feat && tgt_feat && p && T_out && n > 0 && m > 0 && n < kMaxPoints &&
                       m < kMaxPoints,
                "fgr: bad arguments");
    int rc = check_fgr_params(c, p);
    if (rc) return rc;
    CTX_REQUIRE(c, finite_cloud(src, n) && finite_cloud(tgt, m), "fgr: non-finite coordinates");
    CTX_REQUIRE(c, feature_rows_ok(src_feat, n, 33) && feature_rows_ok(tgt_feat, m, 33),
                "fgr: non-finite feature, or a feature row with squared norm above 1e150");
    CTX_CHECK(c, hipSetDevice(c->device));
    const double* xyz[2] = {src, tgt};
    const double* feat[2] = {src_feat, tgt_feat};
    const int64_t np[2] = {n, m};
    CTX_CHECK(c, c->fgr.raw.ensure((size_t)std::max(n, m) * 33));
    for (int k = 0; k < 2; ++k) {
        CTX_CHECK(c, c->fgr.xyz[k].ensure((size_t)np[k] * 3));
        CTX_CHECK(c, c->fgr.feat[k].ensure((size_t)np[k] * kFeatDim));
        CTX_CHECK(c, h2d(c->fgr.xyz[k].p, xyz[k], (size_t)np[k] * 24, c->stream));
        CTX_CHECK(c, h2d(c->fgr.raw.p, feat[k], (size_t)np[k] * 33 * 8, c->stream));
        CTX_CHECK(c, launch_pad_features(c->fgr.raw.p, np[k], c->fgr.feat[k].p, c->stream));
    }
    const bool same = n == m && (src_feat == tgt_feat || std::memcmp(src_feat, tgt_feat, (size_t)n * 33 * 8) == 0);
    return fgr_device(c, src, n, tgt, m, *p, T_out, fitness_out, rmse_out, ncorr_out, n_mutual_out, same);
}

int orpcd_feature_nn(orpcd_ctx* c, const double* q, int64_t nq, const double* t, int64_t nt, int32_t dim,
                     int32_t* idx_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, q && t && idx_out && nq >= 0 && nt > 0, "feature_nn: bad arguments");
    CTX_REQUIRE(c, dim > 0 && dim <= kFeatDim, "feature_nn: dim must be in [1, 36]");
    CTX_REQUIRE(c, feature_rows_ok(q, nq, dim) && feature_rows_ok(t, nt, dim),
                "feature_nn: non-finite value, or a row with squared norm above 1e150");
    if (nq == 0) return ORPCD_OK;
    CTX_CHECK(c, hipSetDevice(c->device));
    auto& F = c->fgr;
    const double* in[2] = {q, t};
    const int64_t np[2] = {nq, nt};
    for (int k = 0; k < 2; ++k) {
        CTX_CHECK(c, F.feat[k].ensure((size_t)np[k] * kFeatDim));
        CTX_CHECK(c, F.fn2[k].ensure((size_t)np[k]));
        CTX_CHECK(c, hipMemsetAsync(F.feat[k].p, 0, (size_t)np[k] * kFeatDim * 8, c->stream));
        CTX_CHECK(c, h2d_2d(F.feat[k].p, kFeatDim * 8, in[k], (size_t)dim * 8, (size_t)dim * 8, (size_t)np[k], c->stream));
        CTX_CHECK(c, launch_feat_norm(F.feat[k].p, np[k], F.fn2[k].p, c->stream));
    }
    CTX_CHECK(c, F.nn[0].ensure((size_t)nq));
    int64_t nu = 0;
    CTX_CHECK(c, dedup_rows(F.feat[1].p, F.fn2[1].p, nt, F.dedup, &nu, c->stream));
    CTX_CHECK(c, launch_feat_nn(F.feat[0].p, F.fn2[0].p, nq, F.dedup.Fu.p, F.dedup.n2u.p, nu, F.dedup.uidx.p, dim,
                                F.fnn, F.nn[0].p, c->stream, c->profiling ? c->stats.feat : nullptr));
    CTX_CHECK(c, d2h(idx_out, F.nn[0].p, (size_t)nq * 4, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    return ORPCD_OK;
}

int orpcd_fgr_optimize(orpcd_ctx* c, const double* src, int64_t n, const double* tgt, int64_t m,
                       double normal_radius, int32_t normal_knn, double fpfh_radius, int32_t fpfh_knn,
                       int32_t target_features_from_source, const orpcd_fgr_params* p, double* T_out,
                       double* fitness_out, double* rmse_out, int64_t* ncorr_out, int64_t* n_mutual_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, src && tgt && p && T_out && n > 0 && m > 0 && n < kMaxPoints && m < kMaxPoints,
                "fgr_optimize: bad arguments");
    int rc = check_fgr_params(c, p);
    if (rc) return rc;
    CTX_REQUIRE(c, !target_features_from_source || m <= n,
                "fgr_optimize: target features taken from the source need m <= n "
                "(fastGlobalOptimizer.py:137-142 would index past the source's features)");
    CTX_REQUIRE(c, finite_cloud(src, n) && finite_cloud(tgt, m), "fgr_optimize: non-finite coordinates");
    CTX_CHECK(c, hipSetDevice(c->device));
    FgrTrace tr;
    g_fgr_trace = &tr;
    struct Reset {
        ~Reset() { g_fgr_trace = nullptr; }
    } reset;
    const double* xyz[2] = {src, tgt};
    const int64_t np[2] = {n, m};
    for (int k = 0; k < 2; ++k) {
        CTX_CHECK(c, c->fgr.xyz[k].ensure((size_t)np[k] * 3));
        CTX_CHECK(c, h2d(c->fgr.xyz[k].p, xyz[k], (size_t)np[k] * 24, c->stream));
    }
    fgr_mark(c->stream, "upload");
    rc = fpfh_device(c, src, 0, n, normal_radius, normal_knn, fpfh_radius, fpfh_knn);
    if (rc) return rc;
    fgr_mark(c->stream, "source normals + fpfh");
    CTX_CHECK(c, c->fgr.feat[1].ensure((size_t)m * kFeatDim));
    if (target_features_from_source) {
        CTX_CHECK(c, hipMemcpyAsync(c->fgr.feat[1].p, c->fgr.feat[0].p, (size_t)m * kFeatDim * 8,
                                    hipMemcpyDeviceToDevice, c->stream));
    } else {
        rc = fpfh_device(c, tgt, 1, m, normal_radius, normal_knn, fpfh_radius, fpfh_knn);
        if (rc) return rc;
    }
    fgr_mark(c->stream, "target normals + fpfh");
    return fgr_device(c, src, n, tgt, m, *p, T_out, fitness_out, rmse_out, ncorr_out, n_mutual_out,
                      target_features_from_source && m == n);
}

int orpcd_fgr_optimize_batch(orpcd_ctx* c, const double* src, int64_t n, const double* tgts, const int64_t* m,
                             int32_t ntgt, const double* R0, const double* t0, const int32_t* target_of_start,
                             int32_t B, double normal_radius, int32_t normal_knn, double fpfh_radius, int32_t fpfh_knn,
                             int32_t target_features_from_source, const orpcd_fgr_params* p, double* T_out,
                             double* fitness_out, double* rmse_out, int64_t* ncorr_out, int64_t* n_mutual_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, src && tgts && m && R0 && t0 && p && T_out && n > 0 && n < kMaxPoints && B > 0,
                "fgr_optimize_batch: bad arguments");
    CTX_REQUIRE(c, ntgt >= 1 && ntgt <= kMaxTargets, "fgr_optimize_batch: 1..16 targets");
    int rc = check_fgr_params(c, p);
    if (rc) return rc;
    CTX_REQUIRE(c, normal_knn > 0 && normal_knn <= kMaxKnn && fpfh_knn > 0 && fpfh_knn <= kMaxKnn,
                "fpfh: knn must be in [1, 1024]");
    CTX_REQUIRE(c, normal_radius > 0 && fpfh_radius > 0, "fpfh: radii must be > 0");
    const bool q4 = target_features_from_source != 0;
    std::vector<int64_t> toff((size_t)ntgt + 1, 0);
    for (int k = 0; k < ntgt; ++k) {
        CTX_REQUIRE(c, m[k] > 0 && m[k] < kMaxPoints, "fgr_optimize_batch: bad target size");
        CTX_REQUIRE(c, !q4 || m[k] <= n,
                    "fgr_optimize_batch: target features taken from the source need m <= n "
                    "(fastGlobalOptimizer.py:137-142 would index past the source's features)");
        toff[k + 1] = toff[k] + m[k];
    }
    std::vector<int> tk((size_t)B, 0);
    for (int b = 0; b < B; ++b) {
        tk[b] = target_of_start ? target_of_start[b] : 0;
        CTX_REQUIRE(c, tk[b] >= 0 && tk[b] < ntgt, "fgr_optimize_batch: target index out of range");
    }
    CTX_REQUIRE(c, finite_cloud(src, n) && finite_cloud(tgts, toff[ntgt]), "fgr_optimize_batch: non-finite coordinates");
    for (int64_t i = 0; i < 9 * (int64_t)B; ++i) CTX_REQUIRE(c, std::isfinite(R0[i]), "fgr_optimize_batch: non-finite R0");
    for (int64_t i = 0; i < 3 * (int64_t)B; ++i) CTX_REQUIRE(c, std::isfinite(t0[i]), "fgr_optimize_batch: non-finite t0");
    {
        // the per-start buffers (posed copy, padded features, SPFH, KNN
        // lists, normals; host copy) scale with B x n: a batch above the
        // budget (ORPCD_FGR_BATCH_BYTES, default 16 GiB) runs in chunks of
        // starts, each start's result being independent of its batch mates
        const int kk = std::max(normal_knn, fpfh_knn);
        const double per_start = (double)n * (3 * 8 + kFeatDim * 8 + 33 * 8 + 6 * 8 + 3 * 8 + 8.0 * kk + 4 + 3 * 8);
        const char* env = getenv("ORPCD_FGR_BATCH_BYTES");
        const double budget = env ? std::max(1.0, atof(env)) : 16.0 * (1ull << 30);
        const int32_t chunk = (int32_t)std::max(1.0, std::min((double)B, std::floor(budget / per_start)));
        if (chunk < B) {
            for (int32_t b0 = 0; b0 < B; b0 += chunk) {
                const int32_t nb = std::min(chunk, B - b0);
                rc = orpcd_fgr_optimize_batch(c, src, n, tgts, m, ntgt, R0 + 9 * (size_t)b0, t0 + 3 * (size_t)b0,
                                              target_of_start ? target_of_start + b0 : nullptr, nb, normal_radius,
                                              normal_knn, fpfh_radius, fpfh_knn, target_features_from_source, p,
                                              T_out + 16 * (size_t)b0, fitness_out ? fitness_out + b0 : nullptr,
                                              rmse_out ? rmse_out + b0 : nullptr, ncorr_out ? ncorr_out + b0 : nullptr,
                                              n_mutual_out ? n_mutual_out + 2 * (size_t)b0 : nullptr);
                if (rc) return rc;
            }
            return ORPCD_OK;
        }
    }
    CTX_CHECK(c, hipSetDevice(c->device));
    FgrTrace tr;  // ORPCD_FGR_TRACE=1: the batch's phases on stderr
    g_fgr_trace = &tr;
    struct Reset {
        ~Reset() { g_fgr_trace = nullptr; }
    } reset;
    auto& F = c->fgr;
    auto& bt = F.bt;
    hipStream_t s = c->stream;
    // --- targets, once each: points, normalisation (mean, max |p - mean|),
    // the evaluation's layout, and their own features unless Q4
    std::vector<double> tmean((size_t)ntgt * 3), tmax((size_t)ntgt);
    for (int k = 0; k < ntgt; ++k) {
        const double* tg = tgts + 3 * toff[k];
        const int64_t mk = m[k], nb = (mk + 255) / 256;
        CTX_CHECK(c, bt.txyz[k].ensure((size_t)mk * 3));
        CTX_CHECK(c, h2d(bt.txyz[k].p, tg, (size_t)mk * 24, s));
        CTX_CHECK(c, F.red.ensure((size_t)nb * 3));
        std::vector<double> part((size_t)nb * 3);
        CTX_CHECK(c, launch_sum3(bt.txyz[k].p, mk, F.red.p, s));
        CTX_CHECK(c, d2h(part.data(), F.red.p, part.size() * 8, s));
        double sum[3] = {0.0, 0.0, 0.0};
        for (int64_t q = 0; q < nb; ++q)
            for (int a = 0; a < 3; ++a) sum[a] += part[(size_t)3 * q + a];
        for (int a = 0; a < 3; ++a) tmean[3 * k + a] = sum[a] / (double)mk;
        CTX_CHECK(c, launch_maxnorm(bt.txyz[k].p, mk, &tmean[3 * k], F.red.p, s));
        CTX_CHECK(c, d2h(part.data(), F.red.p, (size_t)nb * 8, s));
        double mx = 0.0;
        for (int64_t q = 0; q < nb; ++q) mx = std::max(mx, part[(size_t)q]);
        tmax[k] = mx;
        if (!q4) {
            rc = fpfh_buffers(c, 1, mk, fpfh_knn);
            if (rc) return rc;
            CTX_CHECK(c, bt.tfeat[k].ensure((size_t)mk * kFeatDim));
            rc = fpfh_at(c, tg, bt.txyz[k].p, mk, normal_radius, normal_knn, fpfh_radius, fpfh_knn, bt.tfeat[k].p);
            if (rc) return rc;
        }
        rc = layout_from_device(c, tg, bt.txyz[k].p, mk, bt.tlay[k], true);
        if (rc) return rc;
    }
    fgr_mark(s, "batch: targets");
    // --- the posed sources source @ R0[b] + t0[b], rounded as numpy forms
    // them (pose_row), and their normals + FPFH, queued start after start
    std::vector<double> P((size_t)B * n * 3);
    host_parallel(B, [&](int b) {
        for (int64_t i = 0; i < n; ++i) pose_row(src + 3 * i, R0 + 9 * b, t0 + 3 * b, &P[((size_t)b * n + i) * 3]);
    });
    CTX_CHECK(c, bt.X.ensure((size_t)B * n * 3));
    CTX_CHECK(c, bt.FB.ensure((size_t)B * n * kFeatDim));
    CTX_CHECK(c, h2d(bt.X.p, P.data(), P.size() * 8, s));
    if (normal_knn <= 64 && fpfh_knn <= 64) {
        // every copy at once: the copies are rigid images of `src`, so they
        // share its Morton order (BatchLayout; each copy its own frame and
        // boxes, as its own layout would have them), and the exact KNN, the
        // normals and FPFH are those of a per-copy layout (the neighbour
        // lists do not depend on the order): one launch per stage
        CTX_CHECK(c, bt.src.ensure((size_t)n * 3));
        CTX_CHECK(c, h2d(bt.src.p, src, (size_t)n * 24, s));
        rc = layout_from_device(c, src, bt.src.p, n, bt.base, false);
        if (rc) return rc;
        std::vector<double> orgs((size_t)B * 3);
        std::vector<float> margins((size_t)B);
        host_parallel(B, [&](int b) {  // each copy's frame: its box centre, and the fp32 margin of that frame
            const CloudScan cs = scan_cloud(&P[(size_t)b * n * 3], n);
            double org[3];
            for (int a = 0; a < 3; ++a) org[a] = orgs[3 * b + a] = 0.5 * (cs.lo[a] + cs.hi[a]);
            margins[b] = (float)coord_margin(cs.lo, cs.hi, org);
        });
        CTX_CHECK(c, bt.orgs.ensure(orgs.size()));
        CTX_CHECK(c, bt.margins.ensure(margins.size()));
        CTX_CHECK(c, h2d(bt.orgs.p, orgs.data(), orgs.size() * 8, s));
        CTX_CHECK(c, h2d(bt.margins.p, margins.data(), margins.size() * 4, s));
        CTX_CHECK(c, build_batch_layout(bt.X.p, n, B, bt.base.perm.p, bt.orgs.p, bt.bl, s));
        const int kk = std::max(normal_knn, fpfh_knn);
        CTX_CHECK(c, bt.raw.ensure((size_t)B * n * 6));
        CTX_CHECK(c, bt.nrm.ensure((size_t)B * n * 3));
        CTX_CHECK(c, bt.nbr.ensure((size_t)B * n * kk));
        CTX_CHECK(c, bt.nd2.ensure((size_t)B * n * kk));
        CTX_CHECK(c, bt.cnt.ensure((size_t)B * n));
        CTX_CHECK(c, bt.spfh.ensure((size_t)B * n * 33));
        const bool shared = normal_knn == fpfh_knn && normal_radius == fpfh_radius;
        CTX_CHECK(c, launch_knn_batch(bt.bl, bt.base.perm.p, bt.X.p, bt.orgs.p, bt.margins.p, normal_knn,
                                      normal_radius, bt.raw.p, shared ? bt.nbr.p : nullptr,
                                      shared ? bt.nd2.p : nullptr, shared ? bt.cnt.p : nullptr, s));
        CTX_CHECK(c, launch_normals_cov(bt.raw.p, (int64_t)B * n, nullptr, 1, -1.0, bt.nrm.p, nullptr, s));
        if (!shared)
            CTX_CHECK(c, launch_knn_batch(bt.bl, bt.base.perm.p, bt.X.p, bt.orgs.p, bt.margins.p, fpfh_knn,
                                          fpfh_radius, nullptr, bt.nbr.p, bt.nd2.p, bt.cnt.p, s));
        CTX_CHECK(c, launch_fpfh(bt.X.p, bt.nrm.p, n, bt.nbr.p, bt.nd2.p, bt.cnt.p, fpfh_knn, bt.spfh.p, bt.FB.p, s,
                                 B));
    } else {  // neighbourhoods above 64 (chunked KNN lists): copy by copy
        rc = fpfh_buffers(c, 0, n, fpfh_knn);
        if (rc) return rc;
        for (int b = 0; b < B; ++b) {
            rc = fpfh_at(c, &P[(size_t)b * n * 3], bt.X.p + (size_t)b * n * 3, n, normal_radius, normal_knn,
                         fpfh_radius, fpfh_knn, bt.FB.p + (size_t)b * n * kFeatDim);
            if (rc) return rc;
        }
    }
    fgr_mark(s, "batch: pose + normals + fpfh");
    // --- normalisation of every posed source (fixed-order partials, one read-back per phase)
    const int64_t nb = (n + 255) / 256;
    CTX_CHECK(c, bt.part.ensure((size_t)B * nb * 3));
    std::vector<double> part((size_t)B * nb * 3), smean((size_t)B * 3), scale((size_t)B);
    CTX_CHECK(c, launch_sum3(bt.X.p, n, bt.part.p, s, B));  // every start's partials, one launch
    CTX_CHECK(c, d2h(part.data(), bt.part.p, part.size() * 8, s));
    for (int b = 0; b < B; ++b) {
        double sum[3] = {0.0, 0.0, 0.0};
        for (int64_t q = 0; q < nb; ++q)
            for (int a = 0; a < 3; ++a) sum[a] += part[((size_t)b * nb + q) * 3 + a];
        for (int a = 0; a < 3; ++a) smean[3 * b + a] = sum[a] / (double)n;
    }
    CTX_CHECK(c, bt.mean.ensure((size_t)B * 3));
    CTX_CHECK(c, h2d(bt.mean.p, smean.data(), smean.size() * 8, s));
    CTX_CHECK(c, launch_maxnorm(bt.X.p, n, nullptr, bt.part.p, s, B, bt.mean.p));
    CTX_CHECK(c, d2h(part.data(), bt.part.p, (size_t)B * nb * 8, s));
    for (int b = 0; b < B; ++b) {
        double mx = 0.0;
        for (int64_t q = 0; q < nb; ++q) mx = std::max(mx, part[(size_t)b * nb + q]);
        scale[b] = std::max(std::max(0.0, mx), tmax[tk[b]]);
        CTX_REQUIRE(c, scale[b] > 0.0, "fgr: degenerate clouds (all points at their mean)");
    }
    fgr_mark(s, "batch: normalisation");
    // --- initial matching + cross check per start
    std::vector<std::vector<std::pair<int, int>>> corres((size_t)B);
    if (q4) {
        // Q4 (the target's features are the posed source's own first m rows):
        // every row's nearest feature row is the lowest index of its exact
        // duplicates (distance 0; any other row is strictly farther), in both
        // directions, so the mutual pairs are (i, i) for the rows i < m that
        // are their own representative -- what the per-call path's exact
        // searches return (fgr_match; for i >= m the target-side answer
        // rep(j) <= j < m <= i can never point back).  No search is needed.
        CTX_CHECK(c, bt.uflag.ensure((size_t)B * n));
        CTX_CHECK(c, dedup_flags(bt.FB.p, n, F.dedup, bt.uflag.p, s, B));  // every start's rows, segment by segment
        std::vector<unsigned char> fl((size_t)B * n);
        CTX_CHECK(c, d2h(fl.data(), bt.uflag.p, fl.size(), s));
        for (int b = 0; b < B; ++b)
            for (int64_t i = 0; i < m[tk[b]]; ++i)
                if (fl[(size_t)b * n + i]) corres[b].push_back({(int)i, (int)i});
    } else {
        for (int b = 0; b < B; ++b) {
            rc = fgr_match(c, bt.FB.p + (size_t)b * n * kFeatDim, n, bt.tfeat[tk[b]].p, m[tk[b]], false, corres[b]);
            if (rc) return rc;
        }
    }
    fgr_mark(s, "batch: matching");
    // --- tuple tests: every trial of every start at once (fgr_tuples_device)
    std::vector<TupleStart> ts((size_t)B);
    for (int b = 0; b < B; ++b) {
        const int fi = m[tk[b]] > n ? 1 : 0;
        const double* dev[2] = {bt.X.p + (size_t)b * n * 3, bt.txyz[tk[b]].p};
        const double* hst[2] = {&P[(size_t)b * n * 3], tgts + 3 * toff[tk[b]]};
        const double* mn[2] = {&smean[3 * b], &tmean[3 * tk[b]]};
        TupleStart& S = ts[b];
        S.corres = &corres[b];
        S.xi = dev[fi];
        S.xj = dev[1 - fi];
        S.hxi = hst[fi];
        S.hxj = hst[1 - fi];
        for (int a = 0; a < 3; ++a) {
            S.mi[a] = mn[fi][a];
            S.mj[a] = mn[1 - fi][a];
        }
        S.scale = scale[b];
        S.fi = fi;
    }
    std::vector<int> K;
    std::vector<int64_t> outs, caps;
    rc = fgr_tuples_device(c, ts, *p, K, outs, caps);
    if (rc) return rc;
    fgr_mark(s, "batch: tuple tests");
    // --- IRLS: every start's problem in one launch (one workgroup each)
    std::vector<int64_t> meta_reg, meta_mem;
    for (int b = 0; b < B; ++b) {
        auto& mt = K[b] <= 512 * 6 ? meta_reg : meta_mem;  // kIrlsThreads x kIrlsPer: launch_fgr_irls's split
        mt.insert(mt.end(), {outs[b], (int64_t)K[b], (int64_t)b, outs[b] + 3 * caps[b]});
    }
    std::vector<int64_t> meta(meta_reg);
    meta.insert(meta.end(), meta_mem.begin(), meta_mem.end());
    CTX_CHECK(c, bt.meta.ensure(meta.size()));
    CTX_CHECK(c, bt.Tn.ensure((size_t)B * 16));
    CTX_CHECK(c, h2d(bt.meta.p, meta.data(), meta.size() * 8, s));
    const int nreg = (int)meta_reg.size() / 4, nmem = (int)meta_mem.size() / 4;
    CTX_CHECK(c, launch_fgr_irls_batch(c->fgr.tup.rows.p, bt.meta.p, nreg, bt.meta.p + 4 * (size_t)nreg, nmem, 1.0,
                                       p->iteration_number, p->division_factor, p->maximum_correspondence_distance,
                                       p->decrease_mu ? 1 : 0, bt.Tn.p, s));
    std::vector<double> Tn((size_t)B * 16), T((size_t)B * 16);
    CTX_CHECK(c, d2h(Tn.data(), bt.Tn.p, Tn.size() * 8, s));
    for (int b = 0; b < B; ++b)
        fgr_original_scale(&Tn[(size_t)b * 16], &smean[3 * b], &tmean[3 * tk[b]], scale[b], &T[(size_t)b * 16]);
    fgr_mark(s, "batch: irls");
    // --- EvaluateRegistration per start against its target's layout
    // every start's queries T_b x (one launch), one nn1 per run of starts on
    // the same target (a query's answer does not depend on its batch mates:
    // per-query bounds, tiles visited in one fixed order), the per-start
    // (count, sum d^2) partials in one launch
    CTX_CHECK(c, bt.T.ensure((size_t)B * 16));
    CTX_CHECK(c, bt.Q.ensure((size_t)B * n * 3));
    CTX_CHECK(c, h2d(bt.T.p, T.data(), T.size() * 8, s));
    CTX_CHECK(c, c->scratch32.ensure((size_t)B * n));
    CTX_CHECK(c, c->scratch64c.ensure((size_t)B * n));
    CTX_CHECK(c, launch_transform_points(bt.X.p, n, bt.T.p, bt.Q.p, s, B));
    const double r = p->maximum_correspondence_distance;
    for (int b0 = 0; b0 < B;) {
        int b1 = b0 + 1;
        while (b1 < B && tk[b1] == tk[b0]) ++b1;
        const size_t o = (size_t)b0 * n;
        CTX_CHECK(c, launch_nn1(bt.Q.p + 3 * o, (int64_t)(b1 - b0) * n, bt.tlay[tk[b0]], r * r, c->scratch32.p + o,
                                c->scratch64c.p + o, c->qorder, s));
        b0 = b1;
    }
    CTX_CHECK(c, launch_corr_stats(c->scratch32.p, c->scratch64c.p, n, bt.part.p, s, B));
    CTX_CHECK(c, d2h(part.data(), bt.part.p, (size_t)B * nb * 2 * 8, s));
    fgr_mark(s, "batch: evaluation");
    for (int b = 0; b < B; ++b) {
        double cnt = 0.0, err2 = 0.0;
        for (int64_t q = 0; q < nb; ++q) {
            cnt += part[((size_t)b * nb + q) * 2];
            err2 += part[((size_t)b * nb + q) * 2 + 1];
        }
        std::memcpy(T_out + 16 * (size_t)b, &T[(size_t)b * 16], 16 * sizeof(double));
        if (fitness_out) fitness_out[b] = cnt > 0 ? cnt / (double)n : 0.0;
        if (rmse_out) rmse_out[b] = cnt > 0 ? std::sqrt(err2 / cnt) : 0.0;
        if (ncorr_out) ncorr_out[b] = (int64_t)cnt;
        if (n_mutual_out) {
            n_mutual_out[2 * b] = (int64_t)corres[b].size();
            n_mutual_out[2 * b + 1] = K[b];
        }
    }
    return ORPCD_OK;
}

int orpcd_set_option(orpcd_ctx* c, const char* key, double value) {
    if (!c || !key) return ORPCD_EINVAL;
    const std::string k(key);
    const int v = (int)value;
    if (k == "search_waves" && v >= 1) c->opt.search_waves = v;
    else if (k == "sync_every" && v >= 1 && v <= 64) c->opt.sync_every = v;
    else if (k == "super_cull" && (v == 0 || v == 1)) c->opt.super_cull = v;
    else if (k == "small_batch" && v >= 0) c->opt.small_batch = v;
    else if (k == "reseed" && (v == 0 || v == 1)) c->opt.reseed = v;
    else if ((k == "seed_reps" && v >= 1) || (k == "seed_grid" && (v == 0 || v == 1))) {
        if (k == "seed_reps")
            c->opt.seed_reps = v;
        else
            c->opt.seed_grid = v;
        // both live in the targets' descriptors: rewrite them
        CTX_CHECK(c, hipSetDevice(c->device));
        for (int t = 0; t < c->ntgt; ++t) {
            write_target_desc(c->tgts[t], c->tcovs[t].p, c->opt.seed_reps, c->opt.seed_grid != 0, c->tdesc_h[t]);
            CTX_CHECK(c, h2d(c->tdesc.p + t, &c->tdesc_h[t], sizeof(TargetDesc), c->stream));
        }
        CTX_CHECK(c, hipStreamSynchronize(c->stream));
    }
    else if (k == "sched" && (v == 0 || v == 1)) c->opt.sched = v;
    else if (k == "sched_items" && v >= 64 && v <= (1 << 22)) c->opt.sched_items = v;
    else if (k == "sched_min_starts" && v >= 1) c->opt.sched_min_starts = v;
    else if (k == "sched_xcd" && (v == 0 || v == 1)) c->opt.sched_xcd = v;
    else if (k == "sched_cap_us" && v >= 0 && v <= 100000) c->opt.sched_cap_us = v;
    else if (k == "sched_cap_mult" && v >= 1 && v <= 16) c->opt.sched_cap_mult = v;
    else if (k == "knn_lane_min" && v >= 0) c->opt.knn_lane_min = v;
    else if (k == "exact_nn" && (v == 0 || v == 1)) c->opt.exact_nn = v;
    else if (k == "exact_blocks" && v >= 1 && v <= 65536) c->opt.exact_blocks = v;
    else if (k == "exact_fused" && v >= 0 && v <= 4096) c->opt.exact_fused = v;
    else if (k == "count_tiles" && (v == 0 || v == 1)) c->opt.count_tiles = v;
    else if (k == "sync_poll" && (v == 0 || v == 1)) c->opt.sync_poll = v;
    else {
        c->err = "set_option: unknown key or bad value: " + k;
        return ORPCD_EINVAL;
    }
    return ORPCD_OK;
}

int orpcd_gicp_correspondences(orpcd_ctx* c, int32_t B, int32_t* idx_out) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, idx_out && B > 0, "gicp_correspondences: bad arguments");
    const int64_t N = c->src.n;
    CTX_REQUIRE(c, N > 0 && B == c->last_B && c->prevnn.n >= (size_t)B * N && c->last_slot.size() == (size_t)B,
                "gicp_correspondences: B must be the last batch's number of starts (and no cloud set since)");
    CTX_CHECK(c, hipSetDevice(c->device));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    std::vector<int32_t> nn((size_t)B * N), sp((size_t)N);
    std::vector<std::vector<int32_t>> tp((size_t)kMaxTargets);
    CTX_CHECK(c, d2h(nn.data(), c->prevnn.p, nn.size() * 4, c->stream));
    CTX_CHECK(c, d2h(sp.data(), c->src.perm.p, sp.size() * 4, c->stream));
    for (int b = 0; b < B; ++b) {
        const int q = c->last_slot[b], k = c->last_slot_tgt[q];
        std::vector<int32_t>& perm = tp[k];
        const int64_t M = c->tgts[k].n;
        if (perm.empty()) {
            perm.resize((size_t)M);
            CTX_CHECK(c, d2h(perm.data(), c->tgts[k].perm.p, (size_t)M * 4, c->stream));
        }
        for (int64_t i = 0; i < N; ++i) {  // Morton query i is source point sp[i]
            const int32_t j = nn[(size_t)q * N + i];
            idx_out[(size_t)b * N + sp[i]] = j >= 0 && j < (int32_t)M ? perm[j] : -1;
        }
    }
    return ORPCD_OK;
}

int orpcd_test_solve6(orpcd_ctx* c, const double* sums27, int32_t n, double* out_serial, double* out_wave) {
    if (!c) return ORPCD_EINVAL;
    CTX_REQUIRE(c, sums27 && out_serial && out_wave && n >= 0, "test_solve6: bad arguments");
    if (n == 0) return ORPCD_OK;
    CTX_CHECK(c, hipSetDevice(c->device));
    CTX_CHECK(c, c->scratch64c.ensure((size_t)n * (27 + 46)));
    double* dsum = c->scratch64c.p;
    double* dser = dsum + (size_t)n * 27;
    double* dwav = dser + (size_t)n * 23;
    CTX_CHECK(c, h2d(dsum, sums27, (size_t)n * 27 * 8, c->stream));
    CTX_CHECK(c, launch_solve6_test(dsum, n, dser, dwav, c->stream));
    CTX_CHECK(c, d2h(out_serial, dser, (size_t)n * 23 * 8, c->stream));
    CTX_CHECK(c, d2h(out_wave, dwav, (size_t)n * 23 * 8, c->stream));
    CTX_CHECK(c, hipStreamSynchronize(c->stream));
    return ORPCD_OK;
}

int orpcd_profiling(orpcd_ctx* c, int32_t enable) {
    if (!c) return ORPCD_EINVAL;
    c->profiling = enable != 0;
    return ORPCD_OK;
}

int orpcd_stats(orpcd_ctx* c, double* out, int32_t n) {
    if (!c || !out) return ORPCD_EINVAL;
    const double v[20] = {c->stats.launches, c->stats.ms,       c->stats.pairs,          c->stats.iterations,
                          c->stats.passes,   c->stats.tiles,    c->stats.accum_ms,       c->stats.sched_launches,
                          c->stats.exact_filed, c->stats.exact_queries, c->stats.host_batch_ms,
                          c->stats.host_launch_ms, c->stats.host_sync_ms, c->stats.host_batches,
                          c->stats.feat[0], c->stats.feat[1], c->stats.feat[2], c->stats.feat[3], c->stats.feat[4],
                          c->stats.tie_gaps};
    for (int i = 0; i < n && i < 20; ++i) out[i] = v[i];
    return ORPCD_OK;
}

int orpcd_reset_stats(orpcd_ctx* c) {
    if (!c) return ORPCD_EINVAL;
    c->stats = KernelStats();
    return ORPCD_OK;
}

}  // extern "C"
