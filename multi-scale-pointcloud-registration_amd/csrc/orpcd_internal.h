// orpcd_internal.h — host-side runtime structures shared by the .hip units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <random>
#include <vector>

#include "../../include/orpcd.h"

namespace orpcd {

// ------------------------------------------------------------- geometry
constexpr int kTile = 64;                      // targets per culling tile (one wave-wide load)
constexpr int kSuper = 64;                     // tiles per super-tile (first culling level)
// 8-point in-tile boxes since round 4 (with the clamped box distance of
// box_d2_2q): C2 exact 30 starts 16.13 -> 15.88 ms, fp32 mode 13.38 -> 13.21,
// C5 search 0.216 ms either way with 23% fewer pairs scanned; identical
// results (profiles/r04_box_med3_ab.log).  16: round 3's boxes.
#ifndef ORPCD_QUARTER
#define ORPCD_QUARTER 8
#endif
constexpr int kQuarter = ORPCD_QUARTER;        // targets per tile quarter (per-query test inside a staged tile)
constexpr int kNQ = kTile / kQuarter;          // quarters per tile (their boxes: qbox[2 kNQ t + k] lo, [.. + kNQ + k] hi)
static_assert(kNQ * kQuarter == kTile && 2 * kNQ <= 16, "quarter boxes fit the stage after x|y|z (64 floats)");
constexpr int kCQPT = 2;                       // queries per lane in the culled search
constexpr int kCWaves = 4;                     // waves per block
constexpr int kCBlock = 64 * kCWaves;          // threads per block
constexpr int kCBlockQ = kCBlock * kCQPT;      // queries per block (one start)
constexpr int kNacc = 29;                      // JTJ(21) + JTr(6) + sum d2 + count
// GICP covariances stored as their effective normal e (C = I - (1 - eps) e e^T,
// 3 doubles per point; e = e1 where Open3D's GetRotationFromE1ToX takes R = I)
// instead of the 6 entries of C: half the accumulation's covariance loads.
// 0: the 6-entry form (A/B builds).
#ifndef ORPCD_NORMAL_COV
#define ORPCD_NORMAL_COV 1
#endif
constexpr int kCovW = ORPCD_NORMAL_COV ? 3 : 6;  // doubles per stored GICP covariance
constexpr int kEstGICP = 0, kEstP2P = 1;       // transformation estimation of a batch
constexpr int kPartialStride = 32;             // doubles per block partial
constexpr float kFarCoord = 1.0e18f;           // padding coordinate
constexpr int kSchedClasses = 16;              // cost classes of the ordered search dispatch (log2 of a wave's cost)
constexpr int kSchedTot = 64;                  // words the summed wave costs of a pass are spread over
constexpr int kCounterSlots = 256;             // profiling counters: {tiles, max tiles/wave} per slot
constexpr int kCounterStride = 16;             // u64 per slot (128 B: one cache line each)
// Largest cloud the ABI accepts: the raw buffer descriptors of the search
// (num_records = n * sizeof(float4), 32-bit) and its 32-bit byte offsets
// must not wrap.
constexpr int64_t kMaxPoints = (int64_t)1 << 27;

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

// f(b) for b in [0, n) on up to 16 host threads (the GPU box grants 16 cores;
// every b writes only its own outputs)
template <typename Fn>
void host_parallel(int n, Fn f) {
    const int nt = std::max(1, std::min({n, 16, (int)std::max(1u, std::thread::hardware_concurrency())}));
    if (nt <= 1) {
        for (int b = 0; b < n; ++b) f(b);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int b = t; b < n; b += nt) f(b);
        });
    for (auto& x : th) x.join();
}

// memcpy of a large block split over host threads (staging copies of 1M-point clouds)
inline void host_memcpy(void* dst, const void* src, size_t bytes) {
    constexpr size_t kPiece = (size_t)2 << 20;
    if (bytes <= 2 * kPiece) {
        std::memcpy(dst, src, bytes);
        return;
    }
    const int np = (int)((bytes + kPiece - 1) / kPiece);
    host_parallel(np, [&](int k) {
        const size_t o = (size_t)k * kPiece;
        std::memcpy(static_cast<unsigned char*>(dst) + o, static_cast<const unsigned char*>(src) + o,
                    std::min(kPiece, bytes - o));
    });
}

// ------------------------------------------------ host <-> device copies
// Every copy between the device and host memory the library does not own as
// pinned (the caller's arrays, std::vector buffers, stack scalars) goes
// through a pinned staging buffer of the calling thread, never through
// hipMemcpy* on pageable memory.  Measured on MI355X ("drop-in
// stalls"): HIP pins pageable host pages for its copies, and when the host
// later returns such pages to the kernel (glibc trimming its heap after the
// caller frees a large array) the driver stops every queue of the process
// until the mapping is restored -- 10-30 ms during which already enqueued
// passes do not start.  The reference-shaped drop-in loop (a 1.2 MB posed copy
// allocated and freed per attempt) hit it in most processes: a 30-start batch
// took 31-47 ms instead of 15.7 ms.  With staged copies no host page of the
// caller is ever known to the GPU.  A thread pins at most kStageChunk bytes;
// larger copies go through it in chunks.
struct Staging {
    HostBuf<unsigned char> buf;
    // recorded after the last staged host -> device copy, one event per device
    // (an event records only on streams of the device it was created on)
    std::vector<hipEvent_t> ev;
    int ev_dev = -1;        // device of the pending copy's event
    bool pending = false;   // that copy may still be reading buf
    ~Staging() {            // thread exit: the events and the pinned buffer go with the thread
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        buf.release();
    }
};
constexpr size_t kStageChunk = (size_t)32 << 20;  // pinned bytes per thread at most; larger copies go in chunks
inline Staging& staging() {
    thread_local Staging st;
    return st;
}
inline hipError_t staging_reserve(Staging& st, size_t bytes) {
    hipError_t e = hipSuccess;
    if (st.pending) {  // the previous host -> device copy still reads the buffer
        if ((e = hipEventSynchronize(st.ev[st.ev_dev])) != hipSuccess) return e;
        st.pending = false;
    }
    if (bytes > st.buf.n) e = st.buf.ensure(std::min(kStageChunk, std::max(bytes, 2 * st.buf.n)));  // few re-pins
    return e;
}
inline hipError_t staging_mark(Staging& st, hipStream_t s) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);  // the copy's stream belongs to the current device (callers set it)
    if (e != hipSuccess) return e;
    if ((int)st.ev.size() <= dev) st.ev.resize((size_t)dev + 1, nullptr);
    if (!st.ev[dev] && (e = hipEventCreateWithFlags(&st.ev[dev], hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipEventRecord(st.ev[dev], s)) != hipSuccess) return e;
    st.ev_dev = dev;
    st.pending = true;
    return hipSuccess;
}
// host -> device, asynchronous on s (src may be reused as soon as this returns)
inline hipError_t h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
    Staging& st = staging();
    for (size_t off = 0; off < bytes; off += kStageChunk) {
        const size_t n = std::min(kStageChunk, bytes - off);
        hipError_t e = staging_reserve(st, n);
        if (e != hipSuccess) return e;
        host_memcpy(st.buf.p, static_cast<const unsigned char*>(src) + off, n);
        if ((e = hipMemcpyAsync(static_cast<unsigned char*>(dst) + off, st.buf.p, n, hipMemcpyHostToDevice, s)) !=
            hipSuccess)
            return e;
        if ((e = staging_mark(st, s)) != hipSuccess) return e;
    }
    return hipSuccess;
}
// the same for a strided block: `rows` rows of `width` bytes, pitches in bytes
inline hipError_t h2d_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows,
                         hipStream_t s) {
    if (width == 0) return hipSuccess;
    Staging& st = staging();
    const size_t per = std::max<size_t>(1, kStageChunk / width);  // rows per chunk
    for (size_t r0 = 0; r0 < rows; r0 += per) {
        const size_t nr = std::min(per, rows - r0);
        hipError_t e = staging_reserve(st, width * nr);
        if (e != hipSuccess) return e;
        for (size_t r = 0; r < nr; ++r)
            std::memcpy(st.buf.p + r * width, static_cast<const unsigned char*>(src) + (r0 + r) * spitch, width);
        e = hipMemcpy2DAsync(static_cast<unsigned char*>(dst) + r0 * dpitch, dpitch, st.buf.p, width, width, nr,
                             hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
        if ((e = staging_mark(st, s)) != hipSuccess) return e;
    }
    return hipSuccess;
}
// device -> host after everything enqueued on s: returns with dst written
inline hipError_t d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
    Staging& st = staging();
    for (size_t off = 0; off < bytes; off += kStageChunk) {
        const size_t n = std::min(kStageChunk, bytes - off);
        hipError_t e = staging_reserve(st, n);
        if (e != hipSuccess) return e;
        if ((e = hipMemcpyAsync(st.buf.p, static_cast<const unsigned char*>(src) + off, n, hipMemcpyDeviceToHost,
                                s)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        host_memcpy(static_cast<unsigned char*>(dst) + off, st.buf.p, n);
    }
    return hipSuccess;
}
inline hipError_t d2h_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows,
                         hipStream_t s) {
    if (width == 0) return hipSuccess;
    Staging& st = staging();
    const size_t per = std::max<size_t>(1, kStageChunk / width);
    for (size_t r0 = 0; r0 < rows; r0 += per) {
        const size_t nr = std::min(per, rows - r0);
        hipError_t e = staging_reserve(st, width * nr);
        if (e != hipSuccess) return e;
        e = hipMemcpy2DAsync(st.buf.p, width, static_cast<const unsigned char*>(src) + r0 * spitch, spitch, width, nr,
                             hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        for (size_t r = 0; r < nr; ++r)
            std::memcpy(static_cast<unsigned char*>(dst) + (r0 + r) * dpitch, st.buf.p + r * width, width);
    }
    return hipSuccess;
}

// A cloud in device memory, in Morton order (sort_kernels.hip).
// Every fp32 copy (p4, tile / quarter / super-tile boxes) is relative to
// `org`, the cloud's bounding-box centre, subtracted in fp64 before the cast:
// fp32 resolution then follows the cloud's extent, not its distance from the
// coordinate origin.  Every fp32 query is formed the same way (q - org in
// fp64, then one rounding); xyz64 stays absolute.
struct CloudLayout {
    int64_t n = 0, npad = 0, ntiles = 0, nsuper = 0;
    double org[3] = {0.0, 0.0, 0.0};  // fp32 frame origin (bbox centre)
    DevBuf<double> xyz64;     // n*3, Morton order (absolute)
    DevBuf<int32_t> perm;     // Morton position -> input index
    DevBuf<float4> p4;        // npad fp32 (x,y,z relative to org, input index bits), padded far
    DevBuf<float4> tlo, thi;  // per 64-point tile AABB
    DevBuf<float4> qbox;      // per tile: its four 16-point quarters' AABBs (lo x4, hi x4)
    DevBuf<float4> slo, shi;  // per super-tile (64 tiles) AABB
    double lo[3] = {0.0, 0.0, 0.0}, hi[3] = {0.0, 0.0, 0.0};  // bounding box (absolute)
    // seed grid (targets): kSeedGrid^3 cells over the bounding box, per cell the
    // Morton index of the target nearest to its centre (a search bound seed)
    DevBuf<int32_t> sgrid;
    DevBuf<unsigned long long> sgk;  // its build's ping-pong cell keys (2 x kSeedGrid^3: d^2 bits << 32 | index)
    float sg_lo[3] = {0.f, 0.f, 0.f}, sg_inv[3] = {0.f, 0.f, 0.f};  // fp32 frame: cell = (x - lo) * inv
    DevBuf<uint32_t> codes;   // scratch (2n)
    DevBuf<int32_t> ids;      // scratch
    DevBuf<unsigned char> sort_tmp;
    void release() {
        xyz64.release();
        perm.release();
        p4.release();
        tlo.release();
        thi.release();
        qbox.release();
        slo.release();
        shi.release();
        sgrid.release();
        sgk.release();
        codes.release();
        ids.release();
        sort_tmp.release();
    }
};

// AdvancedMatching's tuple test on the device (fgr_kernels.hip, "tuple
// test"): one job per start, trials processed in windows of kTupleWindow.
constexpr int kStateW = 18;  // a running GICP start's state (orpcd_gicp_batch_window): T (16), prev fitness, rmse
constexpr int64_t kTupleWindow = (int64_t)1 << 21;  // trials per start and window
struct TupleJob {
    const double* xi = nullptr;  // cloud fi (the one with more points; the source on a tie), device, input order
    const double* xj = nullptr;  // cloud fj
    double mi[3] = {0, 0, 0}, mj[3] = {0, 0, 0};  // their means (NormalizePointCloud)
    double scale = 1.0;          // the common radius
    int64_t corr = 0;            // offset of the start's (i, j) pairs in the pair and point arrays
    int64_t rej = 0;             // offset of its rejection keys (window-relative, sorted)
    int64_t out = 0;             // offset of its tuple rows: cap source rows (x3), then cap target rows
    int64_t cap = 0;             // tuple rows reserved: 3 * min(maximum_tuple_count, trials)
    int64_t trials = 0;          // 100 * ncorr
    int64_t tw = 0;              // trials in this window (0: the start has finished)
    int64_t word0 = 0;           // stream index of the window's first draw
    int32_t ncorr = 0, fi = 0;
    uint32_t threshold = 0;      // (2^32 - ncorr) mod ncorr: the Lemire rejection bound of uniform_int_distribution
    int32_t nrej = 0;            // rejection keys of this window
};

// B rigid copies of one cloud in its Morton order (build_batch_layout): the
// copies' fp64 points, fp32 frames and tile / super-tile boxes, copy b at
// b x (3n | npad | ntiles | nsuper).
struct BatchLayout {
    int64_t n = 0, npad = 0, ntiles = 0, nsuper = 0;
    int B = 0;
    DevBuf<double> xyz64;
    DevBuf<float4> p4, tlo, thi, qbox, slo, shi;
    void release() {
        xyz64.release();
        for (auto* b : {&p4, &tlo, &thi, &qbox, &slo, &shi}) b->release();
    }
};

// Morton order of a query batch (launch_nn1): codes, identity ids, the
// sorted order and the sort's scratch.
struct QueryOrder {
    DevBuf<uint32_t> codes;
    DevBuf<int32_t> ids, order;
    DevBuf<unsigned char> tmp;
};

// The query rows the second direction of the mutual feature matching needs
// (needed_rows): flags, their indices, the gathered rows and norms, the
// search's answers for them.
struct NeedBufs {
    DevBuf<unsigned char> flag, tmp;
    DevBuf<int32_t> idx, out, pos;
    DevBuf<double> F, n2;
    void release() {
        flag.release();
        tmp.release();
        idx.release();
        out.release();
        pos.release();
        F.release();
        n2.release();
    }
};

struct DedupBufs {
    DevBuf<unsigned long long> key;
    DevBuf<int32_t> val, head, uidx;
    DevBuf<unsigned char> uflag, tmp;
    DevBuf<double> Fu, n2u;
    void release() {
        key.release();
        val.release();
        head.release();
        uidx.release();
        uflag.release();
        tmp.release();
        Fu.release();
        n2u.release();
    }
};

struct FeatNNBufs {
    DevBuf<double> part_d, thr;
    DevBuf<int32_t> part_i, flag, qidx, qsort;
    DevBuf<uint32_t> need, nkey;  // per-query pass-1 part masks; pass 2's sort keys (2 x)
    DevBuf<unsigned char> tmp;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // pass timing (created on first use)
    void release() {
        part_d.release();
        thr.release();
        part_i.release();
        flag.release();
        qidx.release();
        qsort.release();
        need.release();
        nkey.release();
        tmp.release();
        for (auto& e : ev) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
    }
};

struct VoxelBufs {  // preprocessing scratch (voxel, SOR, FPS)
    DevBuf<unsigned long long> key, ukey;
    DevBuf<int32_t> idx, run;
    DevBuf<unsigned char> tmp, flag;
    DevBuf<double> xyz, out;
    DevBuf<int64_t> idx64;
    DevBuf<unsigned long long> tag;
    void release() {
        tag.release();
        flag.release();
        idx64.release();
        key.release();
        ukey.release();
        idx.release();
        run.release();
        tmp.release();
        xyz.release();
        out.release();
    }
};

struct KernelStats {
    double launches = 0, ms = 0, pairs = 0, iterations = 0, passes = 0, tiles = 0, accum_ms = 0;
    double sched_launches = 0;  // timed launches of the ordered-dispatch search (nn_search_sched_kernel)
    double exact_filed = 0;     // exact_nn: queries re-searched in fp64 (nn_exact_kernel), every pass
    double exact_queries = 0;   // exact_nn: queries searched, every pass
    // host wall-clock of the batches (always on; steady_clock): the whole
    // gicp batch call, its launch calls, and its waits for the device
    double host_batch_ms = 0, host_launch_ms = 0, host_sync_ms = 0, host_batches = 0;
    // feature nearest neighbour (launch_feat_nn, while profiling): pass-1 ms,
    // pass-2 ms, pass-1 query-target pairs, pass-2 pairs, calls
    double feat[5] = {0, 0, 0, 0, 0};
    // starts whose source boundary ties may not all have been re-decided
    // (tie table overflowed, or posed coordinates beyond the band's assumption)
    double tie_gaps = 0;
};

// Boundary ties of a KNN covariance pass (launch_knn_cov_ties): points whose
// (kcov+1)-th neighbour lies within rel * d2 + abs_coef * sqrt(d2) of the
// kcov-th.  Entry e: rows[e * (K + 2)] = Morton position, [+1] = input index,
// [+2 ..] the K = kcov + kTieExtra nearest input indices, d2[e * K ..] their
// squared distances (ascending (d2, index)); cnt counts every tie (entries
// past cap are dropped: the caller sees cnt > cap).
struct KnnTieOut {
    int* cnt = nullptr;
    int32_t* rows = nullptr;
    double* d2 = nullptr;
    int cap = 0;
    double rel = 0.0, abs_coef = 0.0;
    // detect-only mode (non-null): a tie point appends its Morton position
    // here (at most cap) instead of its row, so the search needs only the
    // kout + 1 nearest; its rows come from a second, listed pass
    int32_t* detect = nullptr;
    // listed pass over detected points (knn_wave_kernel with a query list):
    // every listed point writes its row, without testing the band again
    int force = 0;
};

// ------------------------------------------------- several targets per batch
// A batch may hold starts against up to kMaxTargets targets (the six scale
// candidates of one speculative compass iteration, Aligner.py:263-298, run
// as ONE device batch).  The starts of a batch are ordered by target (slots
// [first[k], first[k+1]) use target k); since the running-start list keeps
// that order when it is compacted, a launch learns a block's target from the
// block's row `by` and per-launch row bounds passed by value (TgtBounds), with
// no memory load; the target's device pointers come from a TargetDesc array
// in device memory, static while the batch runs.
constexpr int kMaxTargets = 16;

struct TargetDesc {
    const float4 *p4, *tlo, *thi, *qbox, *slo, *shi;  // fp32 search layout (CloudLayout)
    const double *xyz64, *tcov;                        // fp64 points and GICP covariances (Morton order)
    int ntiles, nsuper, seed_stride, sg_on;            // sg_on: queries seeded by the seed grid (opt.seed_grid)
    double ox, oy, oz;                                 // fp32 frame origin (CloudLayout::org)
    const int32_t* sgrid;                              // seed grid (CloudLayout::sgrid; built with the target)
    unsigned long long* sgk;                           // its build's scratch (CloudLayout::sgk)
    int npts;                                          // real points (p4 holds ntiles x 64, padded far)
    float sg_lo[3], sg_inv[3];
};

struct TgtBounds {
    int row_end[kMaxTargets];  // launch rows [row_end[k-1], row_end[k]) run against target k
    int n;                     // targets in the batch (1: every row is target 0)
};

// target of launch row `by` (scalar compares over kernel-argument bounds)
__host__ __device__ __forceinline__ int target_of_row(const TgtBounds& tb, int by) {
    int k = 0;
#pragma unroll
    for (int i = 0; i < kMaxTargets - 1; ++i)
        if (i + 1 < tb.n && by >= tb.row_end[i]) k = i + 1;
    return k;
}

}  // namespace orpcd

struct orpcd_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // targets (set per scale candidate), Morton order; target 0 is `tgt`
    orpcd::CloudLayout tgts[orpcd::kMaxTargets];
    orpcd::DevBuf<double> tcovs[orpcd::kMaxTargets];  // M*kCovW GICP covariance (Morton order)
    double tgt_eps[orpcd::kMaxTargets] = {-1.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0,
                                          -1.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0, -1.0};
    std::vector<double> tgt_host[orpcd::kMaxTargets];  // input-order copies (epsilon re-derivation)
    int ntgt = 0;                                      // targets set (orpcd_set_target: 1)
    int64_t tgt_rows[2] = {0, 0};                      // orpcd_set_target_rows: the Morton rows computed here
    int pass_base = 0;                                 // the running batch's first pass (orpcd_gicp_batch_window)
    orpcd::CloudLayout& tgt = tgts[0];
    orpcd::DevBuf<double>& tcov = tcovs[0];
    orpcd::DevBuf<orpcd::TargetDesc> tdesc;  // kMaxTargets device descriptors of the targets
    orpcd::TargetDesc tdesc_h[orpcd::kMaxTargets] = {};  // their host copies (staging of the uploads)
    int batch_ntgt = 1;                      // targets of the running batch
    int batch_first[orpcd::kMaxTargets + 1] = {0};  // its slots [first[k], first[k+1]) use target k

    // source (set per align), Morton order
    orpcd::CloudLayout src;
    orpcd::DevBuf<double> sraw;     // N*6 raw KNN-20 neighbourhood covariance
    bool src_cov = false;           // sraw holds the source's covariances (orpcd_set_source)
    int est = orpcd::kEstGICP;      // estimation of the running batch (GICP / PointToPoint)

    // boundary ties of the source's KNN-20 neighbourhoods (SourceTies,
    // runtime.hip): points whose 20th and 21st neighbours are so close that a
    // posed copy's rounding decides which one enters the covariance.  Open3D
    // (inside the reference) recomputes the covariances on every posed copy
    // source @ R0 + t0 (Aligner.py:183-185, generalizedICP.py:54-70); the
    // batch re-decides these points per start from the posed coordinates.
    struct SourceTies {
        bool on = false;           // a table for the current source (set_source / set_source_rows)
        bool complete = true;      // every tie is in the table (false: the surplus keeps the rotated covariance)
        double band_A = 0.0;       // max |coordinate| of the cloud the band was sized for
        int kcov = 20;
        std::vector<double> xyz;   // the full source cloud, input order (posing)
        std::vector<int32_t> pt;   // per tie: input index
        std::vector<int32_t> pos;  // per tie: Morton position in the device source layout (-1: not on this rank)
        std::vector<int32_t> off;  // per tie: its candidates cand[off[f] .. off[f+1]) (unposed (d2, index) order)
        std::vector<int32_t> cand;
        std::vector<int32_t> rows;      // sorted input indices of every tie point and candidate (the posed rows)
        std::vector<int32_t> pt_row;    // per tie: its row in `rows`
        std::vector<int32_t> cand_row;  // per candidate: its row in `rows`
        std::vector<double> posed;      // caller-provided posed rows for the next batch (B x rows x 3, caller order)
        int posed_B = 0;
        std::vector<double> posed_slot;  // the same in slot order (batch_setup)
        std::vector<int32_t> last_sets;  // the last batch: per slot, per tie, its kcov neighbours
        void clear() {
            on = false;
            complete = true;
            pt.clear();
            pos.clear();
            off.assign(1, 0);
            cand.clear();
            rows.clear();
            pt_row.clear();
            cand_row.clear();
            posed.clear();
            posed_B = 0;
            posed_slot.clear();
            last_sets.clear();
        }
    } ties;
    orpcd::DevBuf<double> tie_ent;    // per batch: override entries {slot, position, raw covariance (6)}
    orpcd::DevBuf<int32_t> tie_rows;  // knn tie table (KnnTieOut)
    orpcd::DevBuf<double> tie_d2;
    orpcd::DevBuf<int> tie_cnt;       // [0] rows written, [1] tie points detected
    orpcd::DevBuf<int32_t> tie_q;     // the detected points (Morton positions)

    // batch state (per start slot)
    orpcd::DevBuf<double> scov;     // B*N*kCovW posed-frame source covariance
    double batch_eps = 1e-3;        // GICP epsilon of the running batch (the covariances' e e^T weight)
    hipEvent_t gaps_ev0 = nullptr;  // ORPCD_GAPS: recorded where a batch's set-up starts
    double gaps_setup_ms = 0;       // ORPCD_GAPS: host time of the last batch's set-up
    orpcd::DevBuf<int32_t> prevnn;  // B*N previous correspondence (Morton target index)
    orpcd::DevBuf<unsigned long long> best;  // B*N packed (d^2 bits, target) of the current pass
    orpcd::DevBuf<float4> q32;      // B*N fp32 queries of the current pass (x,y,z,0)
    orpcd::DevBuf<float4> gbox;     // B*ceil(N/128)*2: per search wave, its queries' box + worst bound
    orpcd::DevBuf<double> G;        // B*12 base pose (3x4, column convention)
    orpcd::DevBuf<double> T;        // B*16 accumulated ICP transform
    orpcd::DevBuf<double> Q;        // B*12 T*G (3x4)
    orpcd::DevBuf<double> R;        // B*9 rotation of T
    orpcd::DevBuf<double> prev;     // B*2 previous (fitness, rmse)
    orpcd::DevBuf<double> partial;  // B*nblk*32
    orpcd::DevBuf<int32_t> done;    // B
    orpcd::DevBuf<int32_t> active;  // B
    orpcd::DevBuf<double> out_fit, out_rmse;
    orpcd::DevBuf<int32_t> out_iters;
    orpcd::DevBuf<int64_t> out_ncorr;
    orpcd::DevBuf<unsigned long long> counters;  // kCounterSlots x {tiles visited, max per wave}
    // cost-ordered search dispatch (opt.sched; gicp_kernels.hip, SchedIn / SchedOut):
    // the search of pass p sums each wave's duration into wcost[p & 1] (per
    // start and 128-query group) and wtot[p & 1]; the query transform of pass
    // p + 1 turns them into per-group splits and cost classes and appends the
    // pass's work items to wlist (class-major, sched_cap per class)
    orpcd::DevBuf<unsigned> wcost;               // 2 x B x NG (10 ns ticks)
    orpcd::DevBuf<unsigned long long> wtot;      // 2 x kSchedTot
    orpcd::DevBuf<unsigned> wcnt;                // 2 x kSchedClasses: items per class
    orpcd::DevBuf<unsigned long long> wlist;     // kSchedClasses x sched_cap packed items
    int sched_cap = 0;
    int sched_B = 0;                             // starts of the batch (wcost parity stride B x NG)
    bool sched_live = false;                     // the running batch uses the ordered dispatch
    // exact nearest neighbours (opt.exact_nn): queries the fp32 search cannot
    // certify are filed and re-searched in fp64 (nn_exact_kernel)
    orpcd::DevBuf<unsigned> xsec;                // B x N: runner-up key near the winner (0xFFFFFFFF: none)
    orpcd::DevBuf<unsigned long long> xlist;     // B x N: queries with a published runner-up
    orpcd::DevBuf<unsigned> xcnt;                // 2: list entries, by pass parity
    orpcd::DevBuf<unsigned long long> xtotal;    // queries re-searched in fp64 (statistics)
    bool exact_live = false;                     // the running batch runs exact
    int last_B = 0;                              // starts of the last batch (orpcd_gicp_correspondences)
    std::vector<int> last_slot;                  // its start b -> slot (caller order -> target-ordered slots)
    std::vector<int> last_slot_tgt;              // its slot -> target index

    // kernel-level entry points
    orpcd::CloudLayout aux;
    orpcd::DevBuf<double> scratch64a, scratch64b, scratch64c;
    orpcd::DevBuf<int32_t> scratch32;
    orpcd::QueryOrder qorder;  // launch_nn1's Morton order of the queries

    orpcd::HostBuf<double> h64;
    orpcd::HostBuf<int32_t> h32;

    // FastGlobal path (fgr_kernels.hip); index 0 = source, 1 = target
    struct FgrBufs {
        orpcd::DevBuf<double> xyz[2];     // input-order points
        orpcd::DevBuf<double> feat[2];    // n x 36 padded features
        orpcd::DevBuf<double> fn2[2];     // |f|^2
        orpcd::DevBuf<double> nrm, raw, nd2, spfh, red, pq, Tn;
        orpcd::DevBuf<int32_t> nbr, cnt, nn[2];
        orpcd::DedupBufs dedup, dedup2;  // the two clouds' distinct feature rows (matching)
        orpcd::NeedBufs need;
        orpcd::FeatNNBufs fnn;
        // orpcd_fgr_optimize_batch: the batch's posed sources (B x n x 3) and
        // their features (B x n x 36), per-target points / features /
        // evaluation layouts, and the per-start reduction partials, tuples,
        // IRLS problem table and transforms
        struct Batch {
            orpcd::DevBuf<double> X, FB, part, pq, Tn, T, Q, mean, txyz[orpcd::kMaxTargets],
                tfeat[orpcd::kMaxTargets];
            orpcd::DevBuf<int64_t> meta;
            orpcd::DevBuf<unsigned char> uflag;
            orpcd::CloudLayout tlay[orpcd::kMaxTargets];
            // every start's features at once: the base's Morton order, the
            // copies' layouts and frames, their KNN / normals / SPFH scratch
            orpcd::CloudLayout base;
            orpcd::BatchLayout bl;
            orpcd::DevBuf<double> src, orgs, raw, nd2, nrm, spfh;
            orpcd::DevBuf<float> margins;
            orpcd::DevBuf<int32_t> nbr, cnt;
            void release() {
                for (auto* b : {&X, &FB, &part, &pq, &Tn, &T, &Q, &mean, &src, &orgs, &raw, &nd2, &nrm, &spfh})
                    b->release();
                base.release();
                bl.release();
                margins.release();
                nbr.release();
                cnt.release();
                for (int k = 0; k < orpcd::kMaxTargets; ++k) {
                    txyz[k].release();
                    tfeat[k].release();
                    tlay[k].release();
                }
                meta.release();
                uflag.release();
            }
        } bt;
        // the device tuple test (fgr_tuples_device): the seed's mt19937 word
        // stream (host copy extended on demand, mirrored on the device), jobs,
        // pairs, normalised pair points, rejection keys, accept bits, tuple rows
        struct Tuples {
            bool valid = false;
            uint32_t seed = 0;
            std::mt19937 gen;
            std::vector<uint32_t> host;
            size_t on_dev = 0;
            orpcd::DevBuf<uint32_t> words;
            orpcd::DevBuf<orpcd::TupleJob> jobs;
            orpcd::DevBuf<int32_t> pairs, nrej, chunk, cnt;
            orpcd::DevBuf<double> A, Bv, rows;
            orpcd::DevBuf<int64_t> rej;
            orpcd::DevBuf<uint64_t> mask;
            void release() {
                words.release();
                on_dev = 0;
                jobs.release();
                for (auto* b : {&pairs, &nrej, &chunk, &cnt}) b->release();
                for (auto* b : {&A, &Bv, &rows}) b->release();
                rej.release();
                mask.release();
            }
        } tup;
        void release() {
            bt.release();
            tup.release();
            for (int k = 0; k < 2; ++k) {
                xyz[k].release();
                feat[k].release();
                fn2[k].release();
                nn[k].release();
            }
            for (auto* b : {&nrm, &raw, &nd2, &spfh, &red, &pq, &Tn}) b->release();
            for (auto* b : {&nbr, &cnt}) b->release();
            dedup.release();
            dedup2.release();
            need.release();
            fnn.release();
        }
    } fgr;

    // preprocessing (SOR, voxel, FPS)
    orpcd::VoxelBufs vox;
    int fps_blocks = 0;  // co-resident blocks of the cooperative FPS launch (one per CU)

    // profiling
    bool profiling = false;
    bool count_tiles = false;  // tile counters live only while timing (profiling / ORPCD_TRACE)

    // tunables (orpcd_set_option): defaults are the measured best on MI355X
    struct Options {
        int search_waves = 32768;  // split a start's tiles until ~this many waves run (A/B: tools/ab_search.py)
        int small_batch = 8;      // at most this many running starts: half the search_waves target
        int sync_every = 16;      // passes between host checks of the done flags (round 5 sweep, C2 batches of
                                  // 1/8/30/64 starts, 8 -> 16: -2/+0.3/-1.2/-0.6 %; r05_sync_every_ab.txt)
        int super_cull = 1;       // first culling level over 64-tile super-tiles
        int reseed = 0;           // representative seeding also after pass 0
        int seed_reps = 64;       // pass-0 seed without a seed grid: nearest of ~this many tile representatives
        int seed_grid = 1;        // 1: every query also seeded by its seed-grid cell's target (CloudLayout::sgrid)
                                  // (C2 sweep 8..512: equal within noise; 64 keeps the transform cheap)
        int sched = 1;            // 1: search waves dispatched heaviest first, heavy query groups split
                                  // further (costs measured in the previous pass); 0: uniform splits
        int sched_items = 10240;  // ordered dispatch: split a group until its waves cost <= pass total / this
                                  // (C2 sweep 5120 / 10240 / 20480: 15.4 / 15.0 / 16.6 ms at 30 starts)
        int sched_min_starts = 16;  // ordered dispatch only for batches of at least this many starts
        int sched_xcd = 0;          // ordered dispatch: each XCD takes a contiguous chunk of a class's items
        int sched_cap_us = 30;    // ordered dispatch: a split's planned cost at most this many us (0: no cap;
                                  // C2 30 / 64 starts 15.50 -> 15.37 / 24.44 -> 24.23 ms, identical hashes,
                                  // profiles/r05_sched_cap_sweep*.log)
        int sched_cap_mult = 2;   // ... within an item budget of this many times sched_items
        int knn_lane_min = 65536;   // clouds of at least this many points: lane-per-query KNN (0: never)
        int exact_nn = 1;         // 1 (default): every correspondence is the fp64 nearest target (the
                                  // oracle's lexicographic (d^2, input index) minimum): fp32 search +
                                  // runner-up band test + fp64 re-search of the uncertified queries;
                                  // 0: the fp32 search's answer (ties within 2^-17 relative by position)
        int exact_blocks = 256;   // grid of the fp64 re-search (256-thread blocks, one listed query per wave
                                  // at a time)
        int count_tiles = 1;      // profiling: the search also counts the quarters it scans (stats "tiles",
                                  // "pairs"); 0: hipEvent timing only
        int sync_poll = 0;        // 1: the pass loop's device waits poll hipStreamQuery instead of blocking in
                                  // hipStreamSynchronize
        int exact_fused = 64;     // > 0: the re-search runs in the accumulation's launch (GICP), this many
                                  // blocks per running start (at most exact_blocks); 0: a launch of its own
    } opt;
    std::vector<hipEvent_t> ev_pool;
    orpcd::KernelStats stats;

    // row-sharded single start (orpcd_gicp_shard_*)
    struct Shard {
        bool begun = false;
        int pass = 0;
        int64_t n_total = 0;
        orpcd_gicp_params p{};
    } shard;
    // RCCL communicator of the row-sharded start (orpcd_comm_init; an
    // ncclComm_t, librccl loaded at run time)
    void* comm = nullptr;
    int comm_ranks = 0, comm_rank = 0;
};

namespace orpcd {

// sort_kernels.hip
hipError_t launch_gather_rows(const double* in, const int32_t* idx, int64_t offset, int64_t n, int w, double* out,
                              hipStream_t s);
// origin: the fp32 frame origin stored in L.org (the bbox centre)
// gicp_kernels.hip: the target's seed grid (CloudLayout::sgrid)
#ifndef ORPCD_SEED_GRID
#define ORPCD_SEED_GRID 48
#endif
constexpr int kSeedGrid = ORPCD_SEED_GRID;  // cells per axis
hipError_t prepare_seed_grid(CloudLayout& L);
// sgk[k]: target first + k's CloudLayout::sgk (host copy of the pointer); max_points: the largest of their n
hipError_t launch_seed_grids(const TargetDesc* tdesc, int first, int count, int max_points,
                             unsigned long long* const* sgk, hipStream_t s);
hipError_t launch_morton(const double* xyz, int64_t n, const double lo[3], double scale, uint32_t* code,
                         int32_t* idx, hipStream_t s);
hipError_t build_layout(const double* dev_in64, int64_t n, const double bbox_lo[3], double bbox_ext,
                        const double origin[3], CloudLayout& L, bool with_tiles, hipStream_t s);
hipError_t build_batch_layout(const double* in64, int64_t n, int B, const int32_t* perm, const double* orgs,
                              BatchLayout& L, hipStream_t s);

// knn_kernels.hip
constexpr int kMaxKnn = 1024;  // largest neighbourhood the device KNN keeps (16 sorted chunks of 64 per wave)
hipError_t launch_knn_tiles(const CloudLayout& L, const double* in64, int k, double radius, double margin,
                            bool out_input_order, double* rawcov6, int32_t* nbr_idx, double* nbr_d2,
                            int32_t* nbr_cnt, hipStream_t s, double* mean_dist = nullptr,
                            bool lane_per_query = false);
hipError_t launch_normals_cov(const double* rawcov6, int64_t n, const double* Rc9, int nslots, double eps,
                              double* normals3, double* cov6, hipStream_t s, double* enorm3 = nullptr);
// KNN-kcov covariances (pure KNN, as launch_knn_tiles) whose search also keeps
// kcov + kTieExtra neighbours and lists every boundary tie into `ties`
// (SourceTies in runtime.hip); cov_override: entries {slot, Morton position,
// raw covariance (6)} -> GICP covariance of that slot's point
constexpr int kTieExtra = 4;
hipError_t launch_knn_cov_ties(const CloudLayout& L, const double* in64, int kcov, double margin, bool out_input_order,
                               double* rawcov6, const KnnTieOut& ties, hipStream_t s, bool lane_per_query = false,
                               const int32_t* qlist = nullptr, int64_t nq = 0);
// KNN-k raw covariances of the queries at Morton positions [lo, hi) only
// (rawcov6 in Morton order; lane_per_query needs lo and hi on tile bounds)
hipError_t launch_knn_cov_range(const CloudLayout& L, const double* in64, int k, double margin, double* rawcov6,
                                int64_t lo, int64_t hi, bool lane_per_query, hipStream_t s);
// qlist[k] = the Morton position (perm inverted) of input row row_begin + k, k < nrows
hipError_t launch_rows_to_positions(const int32_t* perm, int64_t n, int64_t row_begin, int64_t nrows, int32_t* qlist,
                                    hipStream_t s);
// the same KNN (k <= 64) for every copy of a BatchLayout: perm its common
// Morton order, in64 the copies in input order (B x n x 3), orgs / margins
// per copy on the device; outputs at copy b x (6n | n k | n k | n), input order
hipError_t launch_knn_batch(const BatchLayout& L, const int32_t* perm, const double* in64, const double* orgs,
                            const float* margins, int k, double radius, double* rawcov6, int32_t* nbr_idx,
                            double* nbr_d2, int32_t* nbr_cnt, hipStream_t s);
hipError_t launch_cov_override(const double* ent, int count, int64_t n, double eps, double* cov6, hipStream_t s);

// prep_kernels.hip
hipError_t launch_sor_select(const double* avg, int64_t n, double std_ratio, double* stats, unsigned char* flag,
                             int32_t* kept, int32_t* nkept, DevBuf<unsigned char>& tmp, hipStream_t s);
hipError_t launch_voxel_down_sample(const double* xyz, int64_t n, const double vmin[3], double vs, VoxelBufs& b,
                                    double* out, int64_t* nvox_out, hipStream_t s);
int fps_max_blocks(int device);
int fps_points_per_thread(int64_t n, int max_blocks);
hipError_t launch_fps(const double* xyz, int64_t n, int first, int k, int max_blocks, int64_t* out, double* bval,
                      unsigned long long* btag, unsigned* err, hipStream_t s);

// gicp_kernels.hip
int accum_blocks(int64_t N);
hipError_t launch_xform(const orpcd_ctx* c, int nact, int pass, double r2, hipStream_t s, const TgtBounds& tb);
bool sched_wanted(const orpcd_ctx* c, int B);
int sched_capacity(const orpcd_ctx* c, int B);
TgtBounds one_target();
// bounds of the launch rows act[0..nact) (increasing slots) over the batch's targets
TgtBounds target_bounds(const orpcd_ctx* c, const int32_t* act, int nact);
void write_target_desc(const CloudLayout& L, const double* tcov, int seed_reps, bool seed_grid, TargetDesc& d);
hipError_t launch_gicp_pass(const orpcd_ctx* c, int nact, int pass, double r2, hipStream_t s, hipEvent_t mid,
                            const TgtBounds& tb);
hipError_t launch_gicp_solve(const orpcd_ctx* c, int nact, int pass, const orpcd_gicp_params& p, hipStream_t s,
                             const TgtBounds& tb);
hipError_t launch_reduce_partials(const orpcd_ctx* c, int slot, double* sums29, hipStream_t s);
hipError_t launch_gicp_solve_sums(const orpcd_ctx* c, const double* sums29, int64_t n_total, int pass,
                                  const orpcd_gicp_params& p, hipStream_t s);
hipError_t launch_nn1(const double* q, int64_t nq, const CloudLayout& t, double r2, int32_t* idx, double* d2,
                      QueryOrder& qo, hipStream_t s);
hipError_t launch_solve6_test(const double* sums, int n, double* out_serial, double* out_wave, hipStream_t s);

// fgr_kernels.hip
constexpr int kFeatDim = 36;  // 33 FPFH bins padded for the 16x16x4 f64 MFMA
// clouds > 1: that many clouds of n points back to back (every array at its
// per-cloud stride; neighbour indices within their cloud)
hipError_t launch_fpfh(const double* pts, const double* nrm, int64_t n, const int32_t* nbr, const double* d2,
                       const int32_t* cnt, int k, double* spfh, double* feat36, hipStream_t s, int clouds = 1);
hipError_t launch_pad_features(const double* in33, int64_t n, double* out36, hipStream_t s);
hipError_t launch_feat_norm(const double* F36, int64_t n, double* nrm2, hipStream_t s);
int feat_nn_parts(int64_t blocks, int64_t nt, int maxp);
// tmap (or null): target row -> reported index
hipError_t launch_feat_nn(const double* Fq, const double* nq2, int64_t nq, const double* Ft, const double* nt2,
                          int64_t nt, const int32_t* tmap, int dim, FeatNNBufs& b, int32_t* out, hipStream_t s,
                          double* timing = nullptr);
// Representatives (lowest index) of the distinct rows of F (n x 36): b.uidx
// (increasing), b.Fu / b.n2u their rows and norms; *nu_out their count.
hipError_t dedup_rows(const double* F, const double* n2, int64_t n, DedupBufs& b, int64_t* nu_out, hipStream_t s);
// the rows i of F (ni rows) that some j chose (j_to_i[j] == i, nj entries):
// their indices in b.idx, the rows and norms gathered into b.F / b.n2, their
// count in *nq_out (the stream drains once)
hipError_t needed_rows(const int32_t* j_to_i, int64_t nj, const double* F, const double* n2, int64_t ni,
                       NeedBufs& b, int64_t* nq_out, hipStream_t s);
// out[i] = out_u[position of row i's representative in b.uidx] for the n rows
// b was built from (pos: n ints of scratch)
hipError_t expand_dup_answers(const DedupBufs& b, int64_t n, int64_t nu, const int32_t* out_u, int32_t* pos,
                              int32_t* out, hipStream_t s);
// out[idx[k]] = ans[k], k < n
hipError_t scatter_answers(const int32_t* idx, int64_t n, const int32_t* ans, int32_t* out, hipStream_t s);
hipError_t launch_fgr_irls(const double* p, double* q, int K, double par0, int iters, double division_factor,
                           double max_corr, int decrease_mu, double* T_out, hipStream_t s);
// several IRLS problems in one launch each for the register- and the
// memory-resident form: meta = {offset of p in pq (doubles), K, output slot,
// offset of q in pq} per problem
hipError_t launch_fgr_irls_batch(const double* pq, const int64_t* meta_reg, int nreg, const int64_t* meta_mem,
                                 int nmem, double par0, int iters, double division_factor, double max_corr,
                                 int decrease_mu, double* T_out, hipStream_t s);
// the device tuple test (TupleJob)
// normalised points of every pair: A[k] = (xi[pair.x] - mi) / scale, Bv[k] likewise on cloud fj
hipError_t launch_tuple_points(const TupleJob* jobs, int B, int max_ncorr, const int32_t* pairs, double* A,
                               double* Bv, hipStream_t s);
// stream positions in [word0, word0 + 3 tw + rcap) whose draw uniform_int_distribution rejects (unordered)
hipError_t launch_tuple_reject(const TupleJob* jobs, int B, int64_t max_span, const uint32_t* words, int64_t* rej,
                               int32_t* nrej, int64_t rcap, hipStream_t s);
// every trial of the window: accept bits (mask, kTupleWindow / 64 words per
// start) and accepted trials per 4096 (chunk_cnt, kTupleWindow / 4096 per start)
hipError_t launch_tuple_eval(const TupleJob* jobs, int B, int64_t max_tw, const uint32_t* words, const int64_t* keys,
                             const double* A, const double* Bv, double tuple_scale, uint64_t* mask,
                             int32_t* chunk_cnt, hipStream_t s);
// the window's first accepted trials in order, up to maximum_tuple_count in
// all, as (source, target) rows; cnt[b] = tuples so far
hipError_t launch_tuple_select(const TupleJob* jobs, int B, const uint32_t* words, const int64_t* keys,
                               const uint64_t* mask, const int32_t* chunk_cnt, const double* A, const double* Bv,
                               int maxc, int32_t* cnt, double* rows, hipStream_t s);
// representative flags of dedup_rows (uflag_out[i] = row i is the lowest index of its equal rows)
// The GICP path's device code objects (one per translation unit: sort,
// KNN, GICP), loaded at context creation instead of at the first launch of
// each unit's kernels (hipFuncGetAttributes on one kernel loads the unit's
// code object): the one-time cost moves out of the first call.
hipError_t preload_code_object_sort();
hipError_t preload_code_object_knn();
hipError_t preload_code_object_gicp();
hipError_t dedup_flags(const double* F, int64_t n, DedupBufs& b, unsigned char* uflag_out, hipStream_t s,
                       int clouds = 1);
// clouds > 1: that many clouds of n points back to back (xyz, T, idx / d2 and
// partials at their natural strides; maxnorm's means from dev_means, 3 per cloud)
hipError_t launch_sum3(const double* xyz, int64_t n, double* part, hipStream_t s, int clouds = 1);
hipError_t launch_maxnorm(const double* xyz, int64_t n, const double mean[3], double* part, hipStream_t s,
                          int clouds = 1, const double* dev_means = nullptr);
hipError_t launch_transform_points(const double* in, int64_t n, const double* T, double* out, hipStream_t s,
                                   int clouds = 1);
hipError_t launch_corr_stats(const int32_t* idx, const double* d2, int64_t n, double* part, hipStream_t s,
                             int clouds = 1);

}  // namespace orpcd
