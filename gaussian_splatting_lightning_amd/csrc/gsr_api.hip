// gsr_api.hip -- the extern "C" boundary declared in include/gsrast.h.
//
// Mirrors the orchestration of the reference's CUDA entry points (rasterize_points.cu
// RasterizeGaussiansCUDA / RasterizeGaussiansBackwardCUDA / markVisible and
// rasterizer_impl.cu Rasterizer::forward/backward, SURVEY.md §2.1, [U]) with the MI355X stage list of
// preprocess -> depth sort -> instance scan -> one 8-byte readback -> expand -> tile sort ->
// ranges -> composite; backward: reverse composite -> big-Gaussian reduce -> preprocess backward.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>

#include <immintrin.h>
#include <chrono>
#include <string>
#include <vector>

#include "gsr_kernels.h"
#include "gsrast.h"

using namespace gsr;

namespace {

std::mutex g_tune_mu;
std::vector<std::pair<std::string, int>> g_tune;

}  // namespace

int gsr::tuning(const char *name, int default_value) {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    for (auto &kv : g_tune)
        if (kv.first == name) return kv.second;
    return default_value;
}

uint4 *gsr::stamp_buffer(int which) {
    static uint4 *buf[4] = {nullptr, nullptr, nullptr, nullptr};
    std::lock_guard<std::mutex> lk(g_tune_mu);
    if (which < 0 || which > 3) return nullptr;
    if (!buf[which] && hipMalloc(&buf[which], sizeof(uint4) * STAMP_SLOTS) == hipSuccess)
        (void)hipMemset(buf[which], 0, sizeof(uint4) * STAMP_SLOTS);
    return buf[which];
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define GSR_HIP(x)                                                                                  \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            (void)hipGetLastError(); /* do not leave a sticky error for the caller's runtime */     \
            return fail(GSR_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_));               \
        }                                                                                           \
    } while (0)

// ---- per-stage profiling --------------------------------------------------------------------------
enum Stage {
    ST_PREPROCESS = 0,
    ST_DEPTH_SORT,
    ST_SCAN,
    ST_READBACK,
    ST_EXPAND,
    ST_TILE_SORT,
    ST_RANGES,
    ST_RENDER_FWD,
    ST_RENDER_BWD,
    ST_BIG_REDUCE,
    ST_PREPROCESS_BWD,
    ST_SH_VIEWS,
    ST_BK_COUNT,
    ST_BK_SCATTER,
    ST_SEG_SORT,
    ST_ADAM_SH,
    ST_COUNT
};
const char *kStageNames[ST_COUNT] = {"preprocess", "depth_sort", "instance_scan", "readback",
                                     "expand",     "tile_sort",  "tile_ranges",   "render_fwd",
                                     "render_bwd", "big_reduce", "preprocess_bwd", "sh_views",
                                     "bucket_count", "bucket_scatter", "seg_sort", "adam_sh_views"};

struct Profiler {
    std::mutex mu;
    bool enabled = false;
    std::vector<hipEvent_t> pool;
    struct Pending {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    double total_ms[ST_COUNT] = {};
    int64_t calls[ST_COUNT] = {};

    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        return e;
    }
    void drain() {
        for (auto &p : pending) {
            float ms = 0.f;
            (void)hipEventSynchronize(p.b);
            if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
                total_ms[p.stage] += ms;
                calls[p.stage] += 1;
            }
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }
};
Profiler &prof() {
    static Profiler p;
    return p;
}

// Scoped stage: records an event pair when profiling, synchronises + checks when debugging.
struct StageScope {
    hipStream_t s;
    int stage;
    bool debug;
    hipEvent_t a = nullptr;
    StageScope(hipStream_t s_, int st, bool dbg) : s(s_), stage(st), debug(dbg) {
        Profiler &p = prof();
        // "prof_mask" (bit per Stage, default all): which stages get an event pair.  Every event adds a
        // marker to the stream, so bench.py times its steps with events around the dominant kernel only.
        if (p.enabled && ((tuning("prof_mask", -1) >> st) & 1)) {
            std::lock_guard<std::mutex> lk(p.mu);
            a = p.get();
            if (a) (void)hipEventRecord(a, s);
        }
    }
    int finish() {
        Profiler &p = prof();
        if (a) {
            std::lock_guard<std::mutex> lk(p.mu);
            hipEvent_t b = p.get();
            if (b) {
                (void)hipEventRecord(b, s);
                p.pending.push_back({stage, a, b});
            }
            if (p.pending.size() > 4096) p.drain();
        }
        hipError_t e = hipGetLastError();
        if (e == hipSuccess && debug) {
            e = hipStreamSynchronize(s);
            if (e == hipSuccess) e = hipGetLastError();
        }
        if (e != hipSuccess)
            return fail(GSR_ERR_HIP, std::string("stage ") + kStageNames[stage] + ": " + hipGetErrorString(e));
        return GSR_OK;
    }
};

#define GSR_STAGE(stage, dbg, ...)                      \
    do {                                                \
        StageScope sc_(stream, stage, dbg);             \
        __VA_ARGS__;                                    \
        int rc_ = sc_.finish();                         \
        if (rc_ != GSR_OK) return rc_;                  \
    } while (0)

// Every entry point runs with the device of its stream current (the caller's current device may differ, e.g. a
// thread rendering on cuda:1 after cuda:0), so scratch events, pinned words and launches all belong to the
// stream's device.  The null stream means the current device.
struct StreamDeviceGuard {
    int prev = -1, dev = -1;
    explicit StreamDeviceGuard(hipStream_t s) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        dev = prev;
        if (s && hipStreamGetDevice(s, &dev) != hipSuccess) dev = prev;
        if (dev != prev && dev >= 0) (void)hipSetDevice(dev);
        (void)hipGetLastError();
    }
    ~StreamDeviceGuard() {
        if (prev >= 0 && dev != prev) (void)hipSetDevice(prev);
    }
};

constexpr int kMaxDevices = 64;

// The readback event and pinned words are per thread AND per device: an event recorded on a stream of
// another device is an invalid handle.  One holder per thread owns them and releases them when the thread exits.
struct ReadbackSlots {
    hipEvent_t ev[64] = {};
    uint32_t *words[64] = {};
    ~ReadbackSlots() {
        for (int d = 0; d < 64; d++) {
            if (!ev[d] && !words[d]) continue;
            int prev = -1;
            if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(d) != hipSuccess) continue;
            if (ev[d]) (void)hipEventDestroy(ev[d]);
            if (words[d]) (void)hipHostFree(words[d]);
            if (prev >= 0) (void)hipSetDevice(prev);
        }
    }
};
ReadbackSlots &readback_slots() {
    thread_local ReadbackSlots s;
    return s;
}

hipEvent_t readback_event(int dev) {
    if (dev < 0 || dev >= kMaxDevices) return nullptr;
    hipEvent_t &e = readback_slots().ev[dev];
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    return e;
}

// Instance total of the last forward on this thread and device (the binning buffer's pre-wait size hint).
int64_t &readback_hint(int dev) {
    thread_local int64_t h[kMaxDevices] = {};
    static int64_t none = 0;
    if (dev < 0 || dev >= kMaxDevices) return none = 0;
    return h[dev];
}

// Sequence number of the next preprocess readback on this thread and device (never 0: the buffer starts zeroed).
uint32_t next_readback_seq(int dev) {
    thread_local uint32_t seq[kMaxDevices] = {};
    if (dev < 0 || dev >= kMaxDevices) return 1u;
    if (++seq[dev] == 0u) seq[dev] = 1u;
    return seq[dev];
}

// Spin until the preprocess's last workgroup has published {total lo, hi, big count, seq} at hw[CNT_WORDS] (one
// 16-B store, read here with one 16-B load: aligned 16-B SSE loads are single-copy atomic on AVX-capable x86).
// Once the wait has lasted a millisecond the stream is queried every millisecond, so a failed launch or a kernel
// fault returns an error instead of spinning forever.  Not sooner: a hipStreamQuery puts a marker on the stream,
// and the next kernel's dispatch waited ~6 us behind it (a gap before the bucket scatter on every forward).
int wait_readback(const uint32_t *hw, uint32_t seq, hipStream_t s, uint64_t *total, uint32_t *nbig, uint32_t *kmin,
                  uint32_t *kmax) {
    const __m128i *src = reinterpret_cast<const __m128i *>(hw + CNT_WORDS);
    auto next_query = std::chrono::steady_clock::now() + std::chrono::milliseconds(1);
    for (uint64_t it = 1;; it++) {
        // the compiler barrier forces a fresh load every iteration (the GPU writes this memory behind the
        // compiler's back); a matching sequence word is accepted only when a second 16-B load returns the same
        // bytes, so even a torn read of the 16-B store could not hand back a stale total
        asm volatile("" ::: "memory");
        const __m128i v = _mm_load_si128(src);
        alignas(16) uint32_t w[4];
        _mm_store_si128(reinterpret_cast<__m128i *>(w), v);
        if (w[3] == seq) {
            asm volatile("" ::: "memory");
            const __m128i v2 = _mm_load_si128(src);
            if (_mm_movemask_epi8(_mm_cmpeq_epi8(v, v2)) != 0xffff) continue;
            *total = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
            *nbig = w[2];
            // the depth range word, stored just before (the same thread's earlier store; checked anyway)
            const __m128i *src2 = src + 1;
            for (uint64_t it2 = 0;; it2++) {
                asm volatile("" ::: "memory");
                const __m128i r = _mm_load_si128(src2);
                alignas(16) uint32_t q[4];
                _mm_store_si128(reinterpret_cast<__m128i *>(q), r);
                asm volatile("" ::: "memory");
                const __m128i r2 = _mm_load_si128(src2);
                if (q[2] == seq && _mm_movemask_epi8(_mm_cmpeq_epi8(r, r2)) == 0xffff) {
                    *kmin = q[0];
                    *kmax = q[1];
                    return GSR_OK;
                }
                if (it2 > (1u << 24)) return fail(GSR_ERR_HIP, "preprocess published its total without its depth range");
                _mm_pause();
            }
        }
        if ((it & 255) == 0 && std::chrono::steady_clock::now() >= next_query) {
            const hipError_t e = hipStreamQuery(s);
            if (e != hipSuccess && e != hipErrorNotReady) return fail(GSR_ERR_HIP, hipGetErrorString(e));
            if (e == hipSuccess && __atomic_load_n(hw + CNT_WORDS + 3, __ATOMIC_ACQUIRE) != seq)
                return fail(GSR_ERR_HIP, "preprocess finished without publishing its counters");
            next_query = std::chrono::steady_clock::now() + std::chrono::milliseconds(1);
        }
        _mm_pause();
    }
}

uint32_t *pinned_words(int dev) {
    if (dev < 0 || dev >= kMaxDevices) return nullptr;
    uint32_t *&p = readback_slots().words[dev];
    if (!p) {
        // coherent (fine-grained) pinned memory: the preprocess writes the counters here directly
        if (hipHostMalloc((void **)&p, 4096, hipHostMallocCoherent) != hipSuccess) p = nullptr;
        else memset(p, 0, 4096);
    }
    return p;
}

// Armed while a preprocess that publishes into this thread's pinned words may still be in flight: an early error
// return then waits for the stream, so the late store of an abandoned sequence number can never land after the
// next forward's (possibly on another stream) and hide it.
struct InflightReadback {
    hipStream_t s = nullptr;
    bool armed = false;
    ~InflightReadback() {
        if (armed) (void)hipStreamSynchronize(s);
    }
};

// The decoupled look-backs (instance scan, bucket tile scan, onesweep sorts) never wait on a predecessor that is not
// running: after lb_patience polls they recompute its aggregate from their input (wave_lookback's decoupled
// fallback), so every forward completes with exact output whatever the scheduling; the flags they leave (bit 2 of
// the counters' overflow word, bit 2 of a onesweep error word) only record that a fallback ran.  What remains to
// check is the instance scan's overflow bit (bit 0), which the debug forward reads back (the readback total already
// bounds the count, so this is a second line).  Onesweep error words exist only for the sorts that ran onesweep.
// Debug mode: the instance scan's overflow flag, and whether a decoupled look-back had to recompute a stalled
// predecessor (bit 2 of the counters' flag word and of the radix sorts' error words: exact either way, but a sign of
// a scheduling problem; reported to stderr).  sort_err: the radix sorts' error words that this forward cleared (the
// depth and the tile sort), or null.
int check_lookback_flags(hipStream_t s, int dev, const uint32_t *counters, const uint32_t *depth_err,
                         const uint32_t *tile_err) {
    uint32_t *hw = pinned_words(dev);
    if (!hw) return fail(GSR_ERR_HIP, "pinned host buffer allocation failed");
    hw[1] = hw[2] = 0u;
    GSR_HIP(hipMemcpyAsync(hw, counters + CNT_OVERFLOW, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (depth_err) GSR_HIP(hipMemcpyAsync(hw + 1, depth_err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (tile_err) GSR_HIP(hipMemcpyAsync(hw + 2, tile_err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GSR_HIP(hipStreamSynchronize(s));
    if (hw[0] & 1u) return fail(GSR_ERR_OVERFLOW, "instance scan overflow");
    if ((hw[0] | hw[1] | hw[2]) & 4u)
        fprintf(stderr, "gsrast debug: a decoupled look-back recomputed a stalled predecessor\n");
    return GSR_OK;
}

int check_common(int P, int D, int M, int W, int H, const float *means3D, const float *opac,
                 const float *colors, const float *shs, const float *scales, const float *rots, const float *cov,
                 const float *view, const float *proj, const float *campos, const float *bg) {
    if (P < 0) return fail(GSR_ERR_ARG, "P must be >= 0");
    if (W <= 0 || H <= 0) return fail(GSR_ERR_ARG, "image_width and image_height must be positive");
    if ((int64_t)W * H > 0x7fffffffLL) return fail(GSR_ERR_ARG, "image too large");
    if ((uint64_t)P > (uint64_t)SCAN_TILE * SCAN_MAX_BLOCKS - 1)
        return fail(GSR_ERR_ARG, "too many Gaussians for the single-level scan");
    if (P == 0) return GSR_OK;
    if (!means3D || !opac) return fail(GSR_ERR_ARG, "means3D and opacities are required");
    if (!view || !proj || !bg) return fail(GSR_ERR_ARG, "viewmatrix, projmatrix and bg are required");
    if (!colors) {
        if (!shs || M <= 0) return fail(GSR_ERR_ARG, "Please provide exactly one of either SHs or precomputed colors!");
        if (D < 0 || D > 3) return fail(GSR_ERR_ARG, "sh_degree must be in [0, 3]");
        if ((D + 1) * (D + 1) > M) return fail(GSR_ERR_ARG, "sh_degree needs (deg+1)^2 coefficients per Gaussian");
        if (!campos) return fail(GSR_ERR_ARG, "campos is required with SHs");
    }
    if (!cov && (!scales || !rots))
        return fail(GSR_ERR_ARG, "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    return GSR_OK;
}

}  // namespace

extern "C" {

size_t gsr_geom_buffer_bytes(int P) {
    GeomState g;
    return carve_geom(nullptr, P, g);
}
size_t gsr_binning_buffer_bytes(int64_t R, int W, int H) {
    BinningState b;
    uint32_t T = (uint32_t)(((W + BLOCK_X - 1) / BLOCK_X) * ((H + BLOCK_Y - 1) / BLOCK_Y));
    return carve_binning(nullptr, R, T, b);
}
size_t gsr_image_buffer_bytes(int W, int H) {
    ImageState im;
    return carve_image(nullptr, W, H, im);
}
size_t gsr_bwd_scratch_bytes(int64_t R, int64_t num_big) { return bwd_scratch_bytes(R, num_big); }

void gsr_state_layout_query(int P, int64_t R, int W, int H, gsr_state_layout *caller) {
    if (!caller) return;
    // versioned: fill a full struct here, copy back only the caller's size (fields are only appended)
    const size_t want = caller->struct_size ? std::min(caller->struct_size, sizeof(gsr_state_layout))
                                            : sizeof(gsr_state_layout);
    gsr_state_layout full{};
    gsr_state_layout *out = &full;
    char *const base = reinterpret_cast<char *>(size_t(1) << 40);  // any aligned non-null base
    auto off = [&](const void *p) { return (size_t)(reinterpret_cast<const char *>(p) - base); };
    GeomState g;
    carve_geom(base, P, g);
    BinningState b;
    const uint32_t T = (uint32_t)(((W + BLOCK_X - 1) / BLOCK_X) * ((H + BLOCK_Y - 1) / BLOCK_Y));
    carve_binning(base, R, T, b);
    ImageState im;
    carve_image(base, W, H, im);
    out->geom_rec_a = off(&g.rec->a);
    out->geom_rec_b = off(&g.rec->b);
    out->geom_rec_c = off(&g.rec->c);
    out->geom_rec_stride = sizeof(GRec);
    out->geom_tiles = off(g.tiles);
    out->geom_order = off(g.order);
    out->geom_inst_off = off(g.inst_off);
    out->geom_inst_start = off(g.inst_start);
    out->geom_clamped = off(g.clamped);
    out->geom_expand_rec = off(g.exp_rec);
    out->geom_depth_key = off(g.depth_key);
    out->bin_point_list = off(b.point_list);
    out->bin_inv = off(b.inv);
    out->bin_keys_sorted = off(b.keys_sorted);
    out->bin_sorted_u = off(b.sorted_u);
    out->bin_inst_gid = off(b.inst_gid);
    out->img_tile_loaded = off(im.tile_loaded);
    out->bin_bk_keys = off(b.bk_keys);
    out->img_final_T = off(im.final_T);
    out->img_n_contrib = off(im.n_contrib);
    out->img_ranges = off(im.ranges);
    out->img_tile_last = off(im.tile_last);
    full.struct_size = want;
    memcpy(caller, &full, want);
}

int gsr_forward(gsr_forward_args *a, gsr_alloc_fn alloc, void *alloc_ctx, void *stream_ptr,
                int64_t *num_rendered) {
    if (!a || !alloc || !num_rendered) return fail(GSR_ERR_ARG, "null argument");
    int rc = check_common(a->P, a->D, a->M, a->W, a->H, a->means3D, a->opacities, a->colors_precomp, a->shs,
                          a->scales, a->rotations, a->cov3D_precomp, a->viewmatrix, a->projmatrix, a->campos,
                          a->background);
    if (rc) return rc;
    if (!a->out_color || (a->P > 0 && !a->radii)) return fail(GSR_ERR_ARG, "out_color and radii are required");
    hipStream_t stream = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(stream);
    const bool dbg = a->debug != 0;
    const int P = a->P, W = a->W, H = a->H;
    const int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    const uint32_t T = (uint32_t)(gx * gy);
    *num_rendered = 0;
    a->num_big_out = 0;
    if (P == 0) {
        // the reference returns its zero-initialised outputs untouched when P == 0
        GSR_HIP(hipMemsetAsync(a->out_color, 0, sizeof(float) * 3 * (size_t)W * H, stream));
        if (a->out_invdepth) GSR_HIP(hipMemsetAsync(a->out_invdepth, 0, sizeof(float) * (size_t)W * H, stream));
        return GSR_OK;
    }

    GeomState g;
    char *geom = alloc(alloc_ctx, GSR_BUF_GEOM, carve_geom(nullptr, P, g));
    if (!geom) return fail(GSR_ERR_ALLOC, "geometry buffer allocation failed");
    carve_geom(geom, P, g);
    ImageState im;
    char *img = alloc(alloc_ctx, GSR_BUF_IMAGE, carve_image(nullptr, W, H, im));
    if (!img) return fail(GSR_ERR_ALLOC, "image buffer allocation failed");
    carve_image(img, W, H, im);
    // counters + instance-scan and tile-scan look-back words; rounded up to the carver's 256-B alignment (the
    // next array starts there) so the memset is one aligned fill kernel, not an aligned fill plus a tail
    const size_t clear_bytes = align_up((size_t)(reinterpret_cast<char *>(g.tile_status + BK_MAX_TILES / 32 + 1) -
                                                 reinterpret_cast<char *>(g.counters)), 256);
    launch_zero16(stream, g.counters, clear_bytes);  // a plain kernel: the runtime's fill measured slower

    PreprocessParams pp;
    pp.P = P; pp.D = a->D; pp.M = a->M; pp.W = W; pp.H = H; pp.gx = gx; pp.gy = gy;
    pp.tan_fovx = a->tan_fovx; pp.tan_fovy = a->tan_fovy;
    pp.focal_x = W / (2.0f * a->tan_fovx);
    pp.focal_y = H / (2.0f * a->tan_fovy);
    pp.scale_modifier = a->scale_modifier;
    pp.antialiasing = a->antialiasing;
    pp.cull = tuning("cull", 1);
    pp.means3D = a->means3D; pp.opacities = a->opacities; pp.scales = a->scales; pp.rotations = a->rotations;
    pp.cov3D_precomp = a->cov3D_precomp; pp.colors_precomp = a->colors_precomp; pp.shs = a->shs;
    pp.view = a->viewmatrix; pp.proj = a->projmatrix; pp.campos = a->campos;
    pp.radii = a->radii;
    pp.g = g;
    // The bucket path's Gaussian-order instance scan is formed by its count pass from these block totals.
    pp.block_sums = g.block_sums;
    // The instance total only needs the per-Gaussian tile counts, so it is read back right after the
    // preprocess: its last workgroup writes the counters into pinned host memory and then a sequence word the
    // host polls ("rb_spin" 1, default; 0: a copy plus an event, one more kernel and a barrier on the stream).
    // The bucket path's count pass needs no total either: whenever the tile count admits that path it is queued
    // right behind the preprocess, so the GPU runs it while the host waits (its scratch is in the image buffer;
    // if the total then selects the radix path, its results are simply unused).
    uint32_t *hw = pinned_words(device_guard.dev);
    hipEvent_t rb_ev = readback_event(device_guard.dev);
    if (!hw || !rb_ev) return fail(GSR_ERR_HIP, "pinned host buffer / event allocation failed");
    const bool rb_spin = tuning("rb_spin", 1) != 0 && !dbg;
    const uint32_t seq = next_readback_seq(device_guard.dev);
    pp.host_words = rb_spin ? hw : nullptr;
    pp.stamps = tuning("stamp", 0) ? stamp_buffer(3) : nullptr;
    pp.seq = seq;
    InflightReadback inflight;  // armed before the launch: an error reported after it still waits for the kernel
    inflight.s = stream;
    inflight.armed = rb_spin;
    // the kept depth keys' range, for the radix path's relative depth sort: only where that sort can run (multi-kernel
    // depth sorts, P above the onesweep limit); else the range words stay empty and the sort takes its 32-bit keys
    const uint32_t os_max = (uint32_t)tuning("onesweep_max_n", 3 << 20);
    pp.depth_range = (tuning("depth_rel", 1) && (uint32_t)P > os_max) ? 1 : 0;
    GSR_STAGE(ST_PREPROCESS, dbg, launch_preprocess(stream, pp));
    if (!rb_spin) {
        GSR_HIP(hipMemcpyAsync(hw, g.counters, CNT_WORDS * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        GSR_HIP(hipEventRecord(rb_ev, stream));
    }
    const int bk = tuning("bucket", 1);
    const bool bk_possible = bk == 2 ? T <= BK_MAX_TILES : bk == 1 && T <= BK_MAX_TILES / 2;
    const int lpt = tuning("lpt", 1);
    BucketParams bp = {};
    if (bk_possible) {
        bp.P = (uint32_t)P; bp.T = T; bp.gx = gx; bp.nbig = g.counters + CNT_BIG;
        bp.nb = std::max(1u, std::min({(uint32_t)tuning("bk_blocks", 256), BK_MAX_BLOCKS, div_up(P, 1024)}));
        bp.gper = div_up(div_up(P, bp.nb), 256) * 256;  // whole preprocess blocks
        bp.nr = div_up(P, bp.gper);
        // extra walk blocks for the big rects (used only when the device's big-Gaussian count exceeds nr: bk_walk_blocks);
        // the block count is fixed here, before that count is read back.  2000 sparse-scene Gaussians at 1080p ran their
        // big rects on 2 blocks (count + scatter walks 220 + 310 us).  Only below half of that count of
        // range blocks: at cfg 3 (245 range blocks) 11 extra blocks measured +10 us of scatter (profiles/r4s_*)
        const uint32_t big_blocks = std::min((uint32_t)tuning("bk_big_blocks", 256), BK_MAX_BLOCKS);
        bp.nb = 2 * bp.nr < big_blocks ? big_blocks : bp.nr;
        bp.tiles = g.tiles; bp.inst_start = g.inst_start; bp.block_sums = g.block_sums; bp.depth_key = g.depth_key;
        bp.big_list = g.big_list; bp.exp_rec = g.exp_rec;
        bp.hist = im.bk_hist; bp.hist_pre = im.bk_hist_pre; bp.tile_next = im.bk_tile_next; bp.reg_start = im.bk_reg_start; bp.tile_start = im.bk_tile_start; bp.ranges = im.ranges;
        bp.tile_last = im.tile_last; bp.tile_loaded = im.tile_loaded;
        bp.lpt_bcnt = im.lpt_bcnt;
        bp.ticket = g.counters + CNT_COL_TICKET; bp.tile_status = g.tile_status; bp.err = g.counters + CNT_OVERFLOW;
        bp.long_list = im.bk_long_list; bp.long_cnt = g.counters + CNT_LONG;
        bp.lb_patience = (uint32_t)tuning("lb_patience", 1 << 16); bp.lb_force = tuning("lb_force", 0);
        bp.xcd_major = tuning("bk_xcd", 1);
        // every buffer the column pass clears must be wired (a null one would fault the GPU, not fail here)
        if (!bp.tile_last || !bp.tile_loaded || !bp.ranges || !bp.tile_start || !bp.hist_pre)
            return fail(GSR_ERR_ARG, "internal: bucket binning buffer not set");
        GSR_STAGE(ST_BK_COUNT, dbg, launch_bucket_count(stream, bp));
    }
    // The binning buffer's size depends on the instance total.  Requesting it through the caller's allocator
    // (a Python callback from rasterizer.py) after the readback put ~40 us of host work between the preprocess and
    // the next launch, longer than the queued count passes cover; so with a total from an earlier call on this
    // thread and device the buffer is requested before the wait, 25 % larger, and only re-requested when the
    // total exceeds it ("bin_prealloc" 0: always after the wait).
    BinningState b;
    char *bin = nullptr;
    int64_t bin_cap = -1;
    int64_t &r_hint = readback_hint(device_guard.dev);
    if (r_hint > 0 && tuning("bin_prealloc", 1)) {
        bin_cap = std::min<int64_t>(r_hint + r_hint / 4 + 4096, 0xffffffffLL);
        bin = alloc(alloc_ctx, GSR_BUF_BINNING, carve_binning(nullptr, bin_cap, T, b));
        if (!bin) return fail(GSR_ERR_ALLOC, "binning buffer allocation failed");
    }
    uint64_t total64 = 0;
    uint32_t nbig = 0, kmin = 0xffffffffu, kmax = 0;  // the kept depth keys' range (kmin > kmax: none kept)
    if (rb_spin) {
        GSR_STAGE(ST_READBACK, dbg, {
            const int rc = wait_readback(hw, seq, stream, &total64, &nbig, &kmin, &kmax);
            if (rc) return rc;
        });
        inflight.armed = false;
    } else {
        GSR_STAGE(ST_READBACK, dbg, GSR_HIP(hipEventSynchronize(rb_ev)));
        uint32_t cmax = 0;
        for (int k = 0; k < CNT_NPART; k++) {
            uint64_t part;
            memcpy(&part, hw + CNT_PARTIALS + 2 * k, sizeof(part));
            total64 += part;
            cmax = std::max(cmax, hw[CNT_DMIN + k]);
            kmax = std::max(kmax, hw[CNT_DMAX + k]);
        }
        kmin = ~cmax;
        nbig = hw[CNT_BIG];
    }
    if (total64 > 0xffffffffull) return fail(GSR_ERR_OVERFLOW, "more than 2^32-1 tile instances");
    const uint32_t R = (uint32_t)total64;
    *num_rendered = R;
    a->num_big_out = nbig;
    // Bucket binning (gsr_bin.hip) while the tile counters fit a workgroup's LDS with room for two per CU and
    // the tiles are short (per-tile sorts cost n log^2 n): at 1M Gaussians / 1080p (517 instances per tile) it
    // takes 0.20 ms against the radix path's 0.30; at 5M / 4K stress (1240 per tile) 4.4 ms against 1.4.
    // Otherwise the radix path: depth sort, depth-ordered expansion, stable tile sort.
    const bool bucket = bk_possible && (bk == 2 || (uint64_t)R <= (uint64_t)BK_MAX_MEAN * T);
    bool xcd_fwd = false;  // the forward composite runs the per-XCD LPT orders (set by the bucket scatter below)
    bool sorted_exp = false;
    bool depth_onesweep = false, tile_onesweep = false;  // which sorts ran on the onesweep path (diagnostics)
    if (bucket) gsr_set_tuning("stat_depth_passes", 0);
    if (!bucket) {
        // the depth sort's last pass also writes the tile counts in depth order, so the instance scan reads them
        // coalesced instead of gathering them through the order (the 16-B expansion records too measured slower: cfg 5
        // depth sort 0.232 -> 0.352 ms for expand 0.241 -> 0.221 ms, profiles/r6t_libab_sort_gather_cfg5.txt; the
        // expansion gathers them by rank)
        constexpr int sg = 1;
        SortGather ga;
        ga.src = g.tiles; ga.dst = g.tiles_sorted;
        bool sorted_recs = false;
        // Relative depth keys ("depth_rel" 1) where the sort takes the multi-kernel path: the kept keys span
        // kmax - kmin, so rs_rel_key maps them onto [0, span] and the culled ones onto span + 1, and the sort runs
        // ceil(bits / 9) passes instead of 4 (cfg 5: 26 bits, 3 passes of 9 bits)
        int rel_bits = 32;
        if (tuning("depth_rel", 1) && kmin <= kmax && (uint32_t)P > os_max && kmax - kmin < 0xfffffffeu) {
            const uint32_t cap = kmax - kmin + 1;
            rel_bits = 32 - __builtin_clz(cap);
        }
        gsr_set_tuning("stat_depth_passes", rel_bits <= 27 ? (rel_bits + 8) / 9 : 4);
        if (rel_bits <= 27) {
            GSR_STAGE(ST_DEPTH_SORT, dbg,
                      launch_depth_sort_rel(stream, g.sort, (uint32_t)P, g.depth_key, kmin, kmax - kmin + 1, rel_bits,
                                            sg ? &ga : nullptr));
            sorted_recs = sg != 0;
        } else {
            GSR_STAGE(ST_DEPTH_SORT, dbg,
                      sorted_recs = launch_radix_sort(stream, g.sort, (uint32_t)P, 32, false, g.depth_key,
                                                      sg ? &ga : nullptr, &depth_onesweep));
        }
        const bool sorted_tiles = sorted_recs && (sg & 1);
        sorted_exp = sorted_recs && (sg & 2);
        GSR_STAGE(ST_SCAN, dbg,
                  launch_exclusive_scan_lookback(stream, sorted_tiles ? g.tiles_sorted : g.tiles,
                                                 sorted_tiles ? nullptr : g.order, (uint32_t)P, g.inst_off,
                                                 g.scan_status, g.counters + CNT_SCAN_TICKET,
                                                 g.counters + CNT_OVERFLOW));
    }

    r_hint = R;
    if (!bin || (int64_t)R > bin_cap) {
        bin = alloc(alloc_ctx, GSR_BUF_BINNING, carve_binning(nullptr, R, T, b));
        if (!bin) return fail(GSR_ERR_ALLOC, "binning buffer allocation failed");
    }
    carve_binning(bin, R, T, b);  // offsets from R: a larger buffer only has unused space at the end
    if ((uint64_t)RS_BINS * div_up(R ? R : 1, RS_TILE) + 1 > (uint64_t)SCAN_TILE * SCAN_MAX_BLOCKS)
        return fail(GSR_ERR_OVERFLOW, "too many tile instances for the single-level scan");
    if (bucket) {
        if (R > 0) {
            bp.keys = b.bk_keys; bp.inst_gid = b.inst_gid; bp.inv = b.inv; bp.R = R;
            // region scatter: keys into 16-tile regions first (long runs per block), then a partition pass into the tile
            // buckets (gsr_bin.hip bk_partition_kernel) -- "bk_region" 1 (default) above 4096 tiles (short runs: cfg 3 has
            // ~2 keys per block and tile), 2 always, 0 never (at 800x800, 2500 tiles, the direct scatter's 12 us is
            // already below the partition pass alone)
            const int bkr = tuning("bk_region", 1);
            // (the tile-in-region rides in u's top bits: R <= 2^28; the automatic choice also wants >= 256 keys per region
            // on average, so that a partition chunk rarely spans more regions than its LDS bins cover)
            const uint32_t nreg = div_up(T, BK_REGION);
            bp.keys_reg = ((bkr == 2 || (bkr == 1 && T > 4096 && R >= 256u * nreg)) && R <= (1u << BK_REG_SHIFT))
                              ? b.bk_keys2 : nullptr;
            bp.order = lpt ? im.order_fwd : nullptr;
            // per-XCD LPT orders for the whole-tile composites ("xcd_lpt" 1, with the backward's bucket lists)
            xcd_fwd = lpt && lpt_append_range(T) && tuning("lpt_append", 1) && tuning("xcd_lpt", 1) &&
                      render_fwd_parts((int)T) == 1;
            bp.order_xcd = xcd_fwd ? im.order_xcd : nullptr;
            bp.lpt_shift = tuning("lpt_shift", 3);
            GSR_STAGE(ST_BK_SCATTER, dbg, launch_bucket_scatter(stream, bp));  // and the forward LPT order
            SegSortParams sp;
            // the long tiles lead the LPT order only while SEG_CAP + 1 is a multiple of the bucket width
            sp.T = T; sp.ranges = im.ranges;
            sp.tile_order = (lpt && (((SEG_CAP + 1) >> tuning("lpt_shift", 3)) << tuning("lpt_shift", 3)) == SEG_CAP + 1)
                                ? im.order_fwd : nullptr; sp.keys = b.bk_keys; sp.keys2 = b.bk_keys2;
            sp.sorted_u = b.sorted_u; sp.long_list = im.bk_long_list; sp.long_cnt = g.counters + CNT_LONG;
            // (Round 4's prefix binning -- radix-select each long bucket's 512 front-most keys, sort only those, and
            // let render_fwd extend a walk that outlives them -- measured slower at cfg 3, seg_sort 0.053 -> 0.060 ms
            // and render_fwd 0.171 -> 0.176 ms, and was removed in round 5: DESIGN.md appendix)
            GSR_STAGE(ST_SEG_SORT, dbg, launch_seg_sort(stream, sp));
        } else {
            GSR_HIP(hipMemsetAsync(im.ranges, 0, sizeof(uint2) * T, stream));
            if (lpt) launch_tile_order(stream, im.ranges, nullptr, 0, (int)T, im.order_fwd, im.lpt_hist);
        }
    } else {
        bool keys16 = false;
        if (R > 0) {
            ExpandParams ep;
            ep.P = (uint32_t)P; ep.R = R; ep.gx = gx; ep.gy = gy;
            ep.order = g.order; ep.inst_off = g.inst_off; ep.tiles = g.tiles; ep.exp_rec = g.exp_rec;
            ep.exp_sorted = sorted_exp ? g.exp_sorted : nullptr;
            ep.exp_owner = b.exp_owner;
            // 16-bit tile keys up to 65536 tiles ("tile_key16" 0: 32-bit): the tile sort, the expansion's key stores and
            // the range search move 2 bytes per key instead of 4
            const TileSortPlan plan = tile_sort_plan(T);
            const bool k16 = plan.k16;
            ep.keys_out = k16 ? nullptr : b.sort.k[0];
            ep.keys16_out = k16 ? reinterpret_cast<uint16_t *>(b.sort.k[0]) : nullptr;
            ep.inst_gid = b.inst_gid; ep.inst_start = g.inst_start; ep.inv_none = b.inv;
            GSR_STAGE(ST_EXPAND, dbg, launch_expand(stream, ep));
            if (k16)
                GSR_STAGE(ST_TILE_SORT, dbg, launch_radix_sort16(stream, b.sort, R, plan.digit_bits, plan.passes, tile_key_bits(T)));
            else
                GSR_STAGE(ST_TILE_SORT, dbg,
                          launch_radix_sort(stream, b.sort, R, tile_key_bits(T), false, nullptr, nullptr,
                                            &tile_onesweep));
            keys16 = k16;
        }
        GSR_STAGE(ST_RANGES, dbg, {
            GSR_HIP(hipMemsetAsync(im.ranges, 0, sizeof(uint2) * T, stream));
            if (keys16) launch_identify_ranges16(stream, reinterpret_cast<const uint16_t *>(b.keys_sorted), R, im.ranges);
            else launch_identify_ranges(stream, b.keys_sorted, R, im.ranges);
        });
        if (lpt) launch_tile_order(stream, im.ranges, nullptr, 0, (int)T, im.order_fwd, im.lpt_hist);
    }
    // split heavy tiles combine tile_last / tile_loaded with atomicMax: start from zero (adjacent arrays; the
    // bucket path's column pass clears them)
    if (!bucket || R == 0)
        GSR_HIP(hipMemsetAsync(im.tile_last, 0,
                               (size_t)(reinterpret_cast<char *>(im.lpt_bcnt + LPT_BCNT_WORDS) -
                                        reinterpret_cast<char *>(im.tile_last)),
                               stream));
    RenderFwdParams rp;
    rp.W = W; rp.H = H; rp.gx = gx; rp.gy = gy; rp.num_tiles = (int)T;
    rp.tile_order = lpt ? (xcd_fwd ? im.order_xcd : im.order_fwd) : nullptr;
    rp.xcd = xcd_fwd ? 1 : 0;
    rp.ranges = im.ranges; rp.sorted_u = b.sorted_u; rp.inst_gid = b.inst_gid;
    rp.point_list = b.point_list; rp.tile_loaded = im.tile_loaded;
    rp.inv = b.inv;
    rp.rec = g.rec;
    rp.bg = a->background;
    rp.out_color = a->out_color; rp.out_invdepth = a->out_invdepth; rp.final_T = im.final_T;
    rp.n_contrib = im.n_contrib; rp.tile_last = im.tile_last;
    // checkpoints for the segmented backward ("bwd_seg" 1, spacing "seg_k" instances: 32 or a multiple of 64) while the image
    // has few tiles; the forward records in ck_flag whether it wrote them, so the backward never reads stale ones
    rp.ck_flag = im.ck_flag;
    // the backward's LPT order from bucket lists the whole-tile waves append (no ordering launch in the backward)
    rp.lpt_valid = im.lpt_valid;
    rp.strip_mask = b.strip_mask; rp.smask_valid = im.smask_valid;
    if (lpt_append_range(T) && lpt && tuning("lpt_append", 1)) {
        rp.lpt_bcnt = im.lpt_bcnt; rp.lpt_blist = im.lpt_blist;
    }
    if (T <= SEG_MAX_TILES && tuning("bwd_seg", 1)) {
        rp.ckpt = b.ckpt; rp.ctot = im.ctot;
        const int k = tuning("seg_k", 64);  // cfg 2: 32 / 64 / 128 -> render_bwd 0.106 / 0.107 / 0.129 ms, render_fwd 0.070 / 0.065 / 0.062
        rp.ck_k = k <= 32 ? 32u : (uint32_t)(k / 64) * 64u;
    }
    if (R > 0 && (!rp.point_list || !rp.inst_gid || !rp.sorted_u))
        return fail(GSR_ERR_ARG, "internal: composite buffer not set");
    GSR_STAGE(ST_RENDER_FWD, dbg, launch_render_fwd(stream, rp));
    (void)depth_onesweep;
    (void)tile_onesweep;
    if (dbg)  // every radix sort clears its error word (onesweep: with its control block; multi-kernel: pass 0)
        return check_lookback_flags(stream, device_guard.dev, g.counters, bucket ? nullptr : g.sort.ctrl + RS_CTRL_ERR,
                                    bucket || R == 0 ? nullptr : b.sort.ctrl + RS_CTRL_ERR);
    return GSR_OK;
}

// The per-Gaussian outputs preprocess_bwd writes for Gaussians [g0, g1), as zero-fill segments of the composite backward
// (RenderBwdParams::zf_*): each output's 16-B aligned interior, its unaligned head / tail words listed.  At cfg 3,
// 78 % of the Gaussians have an identically zero gradient (culled, or no pixel took one; tools/zero_grad_census.py):
// their ~250 B of zeros are stored by the VALU-bound walk instead of the HBM-bound per-Gaussian pass.  False (no
// plan): a pointer not 4-B aligned, or too many segments / odd words.
static bool zero_fill_plan(const gsr_backward_args *a, int64_t g0, int64_t g1, RenderBwdParams &rp) {
    const size_t ng = (size_t)(g1 - g0);
    const bool sh_stage = !a->colors_precomp && a->shs && a->M > 0;  // preprocess_bwd writes the SH outputs
    struct Out { float *p; size_t w; };
    const Out outs[] = {{a->dL_dmeans2D, 3}, {a->dL_dcolors, 3}, {a->dL_dopacity, 1}, {a->dL_dmeans3D, 3},
                        {a->dL_dcov3D, 6}, {sh_stage ? a->dL_dsh : nullptr, (size_t)a->M * 3},
                        {sh_stage ? a->dL_dcolors_sh : nullptr, 3}, {a->dL_dscales, 3}, {a->dL_drotations, 4}};
    RenderBwdParams z = rp;
    z.zf_nseg = z.zf_nodd = 0;
    z.zf_total16 = 0;
    for (const Out &o : outs) {
        if (!o.p || ng == 0) continue;
        const uintptr_t b = reinterpret_cast<uintptr_t>(o.p), e = b + ng * o.w * sizeof(float);
        if (b & 3) return false;
        const uintptr_t ab = std::min((b + 15) & ~(uintptr_t)15, e), ae = std::max(e & ~(uintptr_t)15, ab);
        for (uintptr_t q = b; q < ab; q += 4) {
            if (z.zf_nodd >= (uint32_t)RenderBwdParams::ZF_ODD) return false;
            z.zf_odd[z.zf_nodd++] = reinterpret_cast<uint32_t *>(q);
        }
        for (uintptr_t q = ae; q < e; q += 4) {
            if (z.zf_nodd >= (uint32_t)RenderBwdParams::ZF_ODD) return false;
            z.zf_odd[z.zf_nodd++] = reinterpret_cast<uint32_t *>(q);
        }
        if (ae > ab) {
            if (z.zf_nseg >= (uint32_t)RenderBwdParams::ZF_SEGS) return false;
            z.zf_ptr[z.zf_nseg] = reinterpret_cast<uint4 *>(ab);
            z.zf_total16 += (ae - ab) / 16;
            z.zf_pre16[++z.zf_nseg] = z.zf_total16;
        }
    }
    rp = z;
    return true;
}

int gsr_backward(const gsr_backward_args *a, gsr_alloc_fn alloc, void *alloc_ctx, void *stream_ptr) {
    if (!a || !alloc) return fail(GSR_ERR_ARG, "null argument");
    int rc = check_common(a->P, a->D, a->M, a->W, a->H, a->means3D, a->opacities, a->colors_precomp, a->shs,
                          a->scales, a->rotations, a->cov3D_precomp, a->viewmatrix, a->projmatrix, a->campos,
                          a->background);
    if (rc) return rc;
    if (a->P == 0) return GSR_OK;
    if (!a->dL_dpix || !a->radii) return fail(GSR_ERR_ARG, "dL_dpix and radii are required");
    if (!a->geom_buffer || !a->image_buffer || (a->R > 0 && !a->binning_buffer))
        return fail(GSR_ERR_ARG, "forward buffers are required");
    if (a->stages != GSR_BWD_COMPOSITE && a->shs && a->M > 0 && !a->dL_dsh && !a->dL_dcolors_sh)
        return fail(GSR_ERR_ARG, "dL_dsh (or dL_dcolors_sh) is required when shs are given");
    if (a->R < 0 || a->R > 0xffffffffLL) return fail(GSR_ERR_ARG, "bad num_rendered");
    if (a->stages < GSR_BWD_ALL || a->stages > GSR_BWD_GAUSSIANS) return fail(GSR_ERR_ARG, "bad backward stages");
    if (a->campos_rows && (!a->campos || a->campos_nrows < 1 || a->campos_rank < 0 || a->campos_rank >= a->campos_nrows))
        return fail(GSR_ERR_ARG, "campos_rows needs campos and 0 <= campos_rank < campos_nrows");
    int64_t g0 = a->g_begin, g1 = a->g_end;
    if (g0 == 0 && g1 == 0) g1 = a->P;
    if (g0 < 0 || g1 < g0 || g1 > a->P) return fail(GSR_ERR_ARG, "bad Gaussian range [g_begin, g_end)");
    if (a->stages == GSR_BWD_GAUSSIANS && a->R > 0 && !a->bwd_scratch)
        return fail(GSR_ERR_ARG, "GSR_BWD_GAUSSIANS needs the bwd_scratch of the GSR_BWD_COMPOSITE call");
    hipStream_t stream = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(stream);
    const bool dbg = a->debug != 0;
    const int P = a->P, W = a->W, H = a->H;
    const int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    const uint32_t T = (uint32_t)(gx * gy);
    const uint32_t R = (uint32_t)a->R;

    GeomState g;
    carve_geom(a->geom_buffer, P, g);
    BinningState b;
    carve_binning(a->binning_buffer, R, T, b);
    ImageState im;
    carve_image(a->image_buffer, W, H, im);
    if (a->num_big > a->P) return fail(GSR_ERR_ARG, "bad num_big");
    // num_big < 0: not known on the host (the upstream backward signature has no such argument, gsr_torch_ext):
    // size the big-Gaussian sums for the most there can be (each has > BIG_GAUSSIAN_TILES instances) and let the
    // reduction read the count the preprocess left in the geometry buffer
    const bool nbig_on_device = a->num_big < 0;
    const uint32_t nbig = nbig_on_device ? R / (BIG_GAUSSIAN_TILES + 1) + 1 : (uint32_t)a->num_big;
    char *scratch = a->stages == GSR_BWD_GAUSSIANS ? a->bwd_scratch
                                                   : alloc(alloc_ctx, GSR_BUF_BWD_SCRATCH, bwd_scratch_bytes(R, nbig));
    if (!scratch && a->stages != GSR_BWD_GAUSSIANS) return fail(GSR_ERR_ALLOC, "backward scratch allocation failed");
    float *rows = reinterpret_cast<float *>(scratch);
    // Gaussian-major gradient rows: render_bwd scatters its 40-B rows to the instances' expansion indices so
    // the per-Gaussian gather in preprocess_bwd reads each Gaussian's rows contiguously.
    float *bigsum = bwd_bigsum_ptr(scratch, R);

    bool prezero = false;  // the composite zero-fills the per-Gaussian outputs (zero_fill_plan)
    if (R > 0 && a->stages != GSR_BWD_GAUSSIANS) {
        RenderBwdParams rp;
        rp.W = W; rp.H = H; rp.gx = gx; rp.gy = gy; rp.num_tiles = (int)T; rp.num_rendered = R;
        rp.ranges = im.ranges; rp.point_list = b.point_list; rp.n_contrib = im.n_contrib;
        const int lpt = tuning("lpt", 1);
        // the backward's own order (by tile_last; reusing the forward's range-length order measured slower)
        const bool own_order = lpt != 0;
        // in lpt_append_range the forward's whole-tile waves filled the bucket lists (render_bwd falls back to the
        // identity order if that forward did not, *lpt_valid = 0: the order never changes a result)
        const bool lists = own_order && lpt_append_range(T) && tuning("lpt_append", 1);
        if (own_order && !lists)
            launch_tile_order(stream, im.ranges, im.tile_last, 1, (int)T, im.order_bwd, im.lpt_hist);
        rp.tile_order = lpt ? (own_order ? (lists ? nullptr : im.order_bwd) : im.order_fwd) : nullptr;
        if (lists) {
            rp.lpt_bcnt = im.lpt_bcnt; rp.lpt_blist = im.lpt_blist; rp.lpt_valid = im.lpt_valid;
        }
        rp.tile_last = im.tile_last; rp.tile_loaded = im.tile_loaded;
        rp.rec = g.rec;
        rp.bg = a->background; rp.final_T = im.final_T; rp.dL_dpix = a->dL_dpix; rp.dL_dinvdepth = a->dL_dinvdepth;
        rp.rows = rows;
        rp.live = tuning("bwd_live", 1) ? g.live : nullptr;
        rp.live_valid = g.counters + CNT_LIVE_VALID;
        rp.sorted_u = b.sorted_u;
        rp.strip_mask = b.strip_mask; rp.smask_valid = im.smask_valid;
        if (T <= SEG_MAX_TILES && tuning("bwd_seg", 1)) {  // segmented walk (from the forward's checkpoints, if any)
            rp.ckpt = b.ckpt; rp.ctot = im.ctot; rp.ck_flag = im.ck_flag;
            rp.seg_list = b.seg_list; rp.seg_count = im.seg_count;
        }
        if (a->stages == GSR_BWD_ALL && tuning("bwd_prezero", 1)) prezero = zero_fill_plan(a, g0, g1, rp);
        GSR_STAGE(ST_RENDER_BWD, dbg, launch_render_bwd(stream, rp));
        BigReduceParams bp;
        bp.big_list = g.big_list; bp.inst_start = g.inst_start; bp.tiles = g.tiles;
        bp.inv = b.inv;
        bp.rows = rows; bp.bigsum = bigsum;
        bp.nbig_dev = nbig_on_device ? g.counters + CNT_BIG : nullptr;
        GSR_STAGE(ST_BIG_REDUCE, dbg, launch_big_reduce(stream, bp, nbig));
    }
    if (a->stages == GSR_BWD_COMPOSITE) return GSR_OK;
    // Chunk-relative outputs (a split backward) address Gaussian g0's row: shift them so the kernel indexes every
    // output by the absolute Gaussian index (integer arithmetic: the shifted address is never dereferenced)
    auto rel = [g0](auto *ptr, int64_t width) -> decltype(ptr) {
        if (!ptr || g0 == 0) return ptr;
        return reinterpret_cast<decltype(ptr)>(reinterpret_cast<uintptr_t>(ptr) - (uintptr_t)(g0 * width) * sizeof(*ptr));
    };
    PreprocessBwdParams pp;
    pp.P = P; pp.D = a->D; pp.M = a->M; pp.W = W; pp.H = H;
    pp.g0 = (int)g0; pp.g1 = (int)g1;
    pp.tan_fovx = a->tan_fovx; pp.tan_fovy = a->tan_fovy;
    pp.focal_x = W / (2.0f * a->tan_fovx);
    pp.focal_y = H / (2.0f * a->tan_fovy);
    pp.scale_modifier = a->scale_modifier;
    pp.antialiasing = a->antialiasing;
    pp.has_invdepth = a->dL_dinvdepth != nullptr;
    pp.means3D = a->means3D; pp.opacities = a->opacities; pp.scales = a->scales; pp.rotations = a->rotations;
    pp.cov3D_precomp = a->cov3D_precomp; pp.shs = (a->colors_precomp ? nullptr : a->shs);
    pp.view = a->viewmatrix; pp.proj = a->projmatrix; pp.campos = a->campos;
    pp.radii = a->radii; pp.tiles = g.tiles; pp.inst_start = g.inst_start; pp.clamped = g.clamped;
    pp.live = tuning("bwd_live", 1) ? g.live : nullptr;
    pp.live_valid = g.counters + CNT_LIVE_VALID;
    pp.inv = b.inv;
    pp.sh_jac = g.sh_jac;  // the forward's d rgb / d dir: the SH term of dL/dmeans3D reads no coefficient
    pp.big_slot = g.big_slot; pp.bigsum = bigsum;
    pp.rows = rows;
    pp.sh_vec16 = pp.shs && a->M == 16 && (((uintptr_t)pp.shs | (uintptr_t)a->dL_dsh) & 15) == 0;
    pp.dL_dmeans2D = rel(a->dL_dmeans2D, 3); pp.dL_dcolors = rel(a->dL_dcolors, 3);
    pp.dL_dopacity = rel(a->dL_dopacity, 1); pp.dL_dmeans3D = rel(a->dL_dmeans3D, 3);
    pp.dL_dcov3D = rel(a->dL_dcov3D, 6); pp.dL_dsh = rel(a->dL_dsh, (int64_t)a->M * 3);
    pp.dL_dcolors_sh = rel(a->dL_dcolors_sh, 3);
    pp.densify_stats = rel(a->densify_stats, 2);
    pp.densify_accumulate = a->densify_accumulate;
    pp.max_radii2D = rel(a->max_radii2D, 1);
    pp.dL_dscales = rel(a->dL_dscales, 3); pp.dL_drot = rel(a->dL_drotations, 4);
    pp.campos_rows = a->campos_rows; pp.campos_rank = a->campos_rank; pp.campos_nrows = a->campos_nrows;
    pp.prezeroed = prezero ? 1 : 0;
    const size_t ng = (size_t)(g1 - g0);
    if (pp.shs == nullptr && a->dL_dsh && a->M > 0)
        GSR_HIP(hipMemsetAsync(a->dL_dsh, 0, sizeof(float) * ng * a->M * 3, stream));
    if (pp.shs == nullptr && a->dL_dcolors_sh)
        GSR_HIP(hipMemsetAsync(a->dL_dcolors_sh, 0, sizeof(float) * ng * 3, stream));
    GSR_STAGE(ST_PREPROCESS_BWD, dbg, launch_preprocess_bwd(stream, pp));
    return GSR_OK;
}

int gsr_sh_backward_views_chunked(int P, int D, int M, int V, int64_t chunk_len, const float *means3D,
                                  const float *campos, const float *dL_dcolors_sh, float *dL_dsh, void *stream_ptr) {
    if (P < 0 || V < 0) return fail(GSR_ERR_ARG, "P and V must be >= 0");
    if (D < 0 || D > 3) return fail(GSR_ERR_ARG, "sh_degree must be in [0, 3]");
    if (M <= 0 || M > 16 || (D + 1) * (D + 1) > M)
        return fail(GSR_ERR_ARG, "M must hold (deg+1)^2 <= M <= 16 coefficients");
    if (chunk_len < 0) return fail(GSR_ERR_ARG, "chunk_len must be >= 0");
    if (P == 0) return GSR_OK;
    if (!means3D || !dL_dsh || (V > 0 && (!campos || !dL_dcolors_sh))) return fail(GSR_ERR_ARG, "null argument");
    hipStream_t stream = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(stream);
    const int L = (chunk_len == 0 || chunk_len >= P) ? P : (int)chunk_len;
    GSR_STAGE(ST_SH_VIEWS, 0, launch_sh_backward_views(stream, P, D, M, V, L, means3D, campos, dL_dcolors_sh, dL_dsh));
    return GSR_OK;
}

int gsr_sh_backward_views(int P, int D, int M, int V, const float *means3D, const float *campos,
                          const float *dL_dcolors_sh, float *dL_dsh, void *stream_ptr) {
    return gsr_sh_backward_views_chunked(P, D, M, V, 0, means3D, campos, dL_dcolors_sh, dL_dsh, stream_ptr);
}

int gsr_adam_sh_views_step(const gsr_adam_sh_views_args *a, double beta1, double beta2, double eps, void *stream_ptr) {
    if (!a) return fail(GSR_ERR_ARG, "adam sh views: null arguments");
    if (a->P < 0 || a->V < 0) return fail(GSR_ERR_ARG, "P and V must be >= 0");
    if (a->D < 0 || a->D > 3) return fail(GSR_ERR_ARG, "sh_degree must be in [0, 3]");
    if (a->M != 16) return fail(GSR_ERR_ARG, "adam sh views: M must be 16");
    if (a->chunk_len < 0) return fail(GSR_ERR_ARG, "chunk_len must be >= 0");
    if (a->dc_step < 1 || a->rest_step < 1) return fail(GSR_ERR_ARG, "adam: step must be >= 1");
    if (a->P == 0) return GSR_OK;
    if (!a->means3D || (a->V > 0 && (!a->campos || !a->dL_dcolors_sh)) || !a->dc_param || !a->dc_exp_avg ||
        !a->dc_exp_avg_sq || !a->rest_param || !a->rest_exp_avg || !a->rest_exp_avg_sq)
        return fail(GSR_ERR_ARG, "null argument");
    AdamShLaunch L{};
    L.P = a->P; L.V = a->V;
    L.L = (a->chunk_len == 0 || a->chunk_len >= a->P) ? a->P : (int)a->chunk_len;
    L.means3D = a->means3D; L.campos = a->campos; L.dc = a->dL_dcolors_sh;
    if ((a->param_row_stride != 0 && a->param_row_stride != 48) || (a->moment_row_stride != 0 && a->moment_row_stride != 48))
        return fail(GSR_ERR_ARG, "adam sh views: row strides must be 0 (packed) or 48 (one (P, 16, 3) tensor)");
    if (a->moment_row_stride == 48 && a->param_row_stride != 48)
        return fail(GSR_ERR_ARG, "adam sh views: joint moments need the joint parameter");
    if (a->param_row_stride == 48 && (a->rest_param != a->dc_param + 3 ||
                                      (a->moment_row_stride == 48 && (a->rest_exp_avg != a->dc_exp_avg + 3 ||
                                                                      a->rest_exp_avg_sq != a->dc_exp_avg_sq + 3))))
        return fail(GSR_ERR_ARG, "adam sh views: a joint tensor's rest block must start 3 floats after its dc block");
    auto group = [&](AdamShGroup &g, float *p, float *m, float *v, double lr, int64_t step, int64_t width) {
        const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
        g.param = p; g.exp_avg = m; g.exp_avg_sq = v;
        g.param_stride = a->param_row_stride ? a->param_row_stride : width;
        g.step_size = (float)(lr / bc1);  // as gsr_adam_step
        g.bc2_sqrt = (float)std::sqrt(bc2);
    };
    group(L.dc_group, a->dc_param, a->dc_exp_avg, a->dc_exp_avg_sq, a->dc_lr, a->dc_step, 3);
    group(L.rest_group, a->rest_param, a->rest_exp_avg, a->rest_exp_avg_sq, a->rest_lr, a->rest_step, 45);
    // float4 moments (and parameters when packed) need 16-B aligned bases
    const uintptr_t params = a->param_row_stride ? 0 : (((uintptr_t)a->dc_param) | ((uintptr_t)a->rest_param));
    L.vec4 = ((params | ((uintptr_t)a->dc_exp_avg) | ((uintptr_t)a->dc_exp_avg_sq) | ((uintptr_t)a->rest_exp_avg) |
               ((uintptr_t)a->rest_exp_avg_sq)) & 15) == 0;
    L.one_minus_beta1 = (float)(1.0 - beta1);
    L.beta2 = (float)beta2;
    L.one_minus_beta2 = (float)(1.0 - beta2);
    L.eps = (float)eps;
    L.joint = a->moment_row_stride == 48 &&
              ((((uintptr_t)a->dc_param) | ((uintptr_t)a->dc_exp_avg) | ((uintptr_t)a->dc_exp_avg_sq)) & 15) == 0;
    hipStream_t stream = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(stream);
    GSR_STAGE(ST_ADAM_SH, 0, launch_adam_sh_views(stream, L, a->D));
    return GSR_OK;
}

int gsr_adam_step(const gsr_adam_group *groups, int num_groups, double beta1, double beta2, double eps,
                  void *stream_ptr) {
    if (num_groups < 0 || num_groups > ADAM_MAX_GROUPS) return fail(GSR_ERR_ARG, "adam: 0..16 parameter groups");
    if (num_groups && !groups) return fail(GSR_ERR_ARG, "adam: null groups");
    AdamLaunch L{};
    int64_t slices = 0;
    int ng = 0;
    for (int i = 0; i < num_groups; i++) {
        const gsr_adam_group &g = groups[i];
        if (g.n < 0 || g.step < 1) return fail(GSR_ERR_ARG, "adam: n must be >= 0 and step >= 1");
        if (g.n == 0) continue;
        if (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq) return fail(GSR_ERR_ARG, "adam: null array");
        AdamGroupDev &d = L.g[ng];
        d.param = g.param; d.grad = g.grad; d.exp_avg = g.exp_avg; d.exp_avg_sq = g.exp_avg_sq; d.n = g.n;
        const double bc1 = 1.0 - std::pow(beta1, (double)g.step), bc2 = 1.0 - std::pow(beta2, (double)g.step);
        d.step_size = (float)(g.lr / bc1);
        d.bc2_sqrt = (float)std::sqrt(bc2);
        d.vec4 = ((((uintptr_t)g.param) | ((uintptr_t)g.grad) | ((uintptr_t)g.exp_avg) |
                   ((uintptr_t)g.exp_avg_sq)) & 15) == 0;
        L.slice_start[ng] = slices;
        slices += adam_slices(g.n);
        ng++;
    }
    if (slices > 0x7fffffffLL) return fail(GSR_ERR_ARG, "adam: too many elements");
    L.num_groups = ng;
    L.one_minus_beta1 = (float)(1.0 - beta1);
    L.beta2 = (float)beta2;
    L.one_minus_beta2 = (float)(1.0 - beta2);
    L.eps = (float)eps;
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_adam((hipStream_t)stream_ptr, L, slices);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

static bool aligned16(const void *p) { return (((uintptr_t)p) & 15) == 0; }

int gsr_activations_forward(int64_t N, const float *scaling, const float *opacity, const float *rotation,
                            float *scales, float *opacities, float *rotations, void *stream_ptr) {
    if (N < 0 || N > 0x7fffffffLL * 256) return fail(GSR_ERR_ARG, "activations: bad N");
    if (N == 0) return GSR_OK;
    if (!scaling || !opacity || !rotation || !scales || !opacities || !rotations)
        return fail(GSR_ERR_ARG, "activations: null array");
    if (!aligned16(rotation) || !aligned16(rotations)) return fail(GSR_ERR_ARG, "activations: rotation arrays must be 16-B aligned");
    ActivationArgs A{};
    A.N = N;
    A.scaling = scaling; A.opacity = opacity; A.rotation = rotation;
    A.scales = scales; A.opacities = opacities; A.rotations = rotations;
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_activations_forward((hipStream_t)stream_ptr, A);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

int gsr_activations_backward(int64_t N, const float *rotation, const float *scales, const float *opacities,
                             const float *rotations, const float *dL_dscales, const float *dL_dopacities,
                             const float *dL_drotations, float *dL_dscaling, float *dL_dopacity, float *dL_drotation,
                             void *stream_ptr) {
    if (N < 0 || N > 0x7fffffffLL * 256) return fail(GSR_ERR_ARG, "activations: bad N");
    if (N == 0) return GSR_OK;
    if (!rotation || !scales || !opacities || !rotations || !dL_dscales || !dL_dopacities || !dL_drotations ||
        !dL_dscaling || !dL_dopacity || !dL_drotation)
        return fail(GSR_ERR_ARG, "activations: null array");
    if (!aligned16(rotation) || !aligned16(rotations) || !aligned16(dL_drotations) || !aligned16(dL_drotation))
        return fail(GSR_ERR_ARG, "activations: rotation arrays must be 16-B aligned");
    ActivationArgs A{};
    A.N = N;
    A.rotation = rotation;
    A.scales = const_cast<float *>(scales); A.opacities = const_cast<float *>(opacities);
    A.rotations = const_cast<float *>(rotations);
    A.dL_dscales = dL_dscales; A.dL_dopacities = dL_dopacities; A.dL_drotations = dL_drotations;
    A.dL_dscaling = dL_dscaling; A.dL_dopacity = dL_dopacity; A.dL_drotation = dL_drotation;
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_activations_backward((hipStream_t)stream_ptr, A);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

int gsr_sparse_adam_step(const gsr_adam_group *groups, int num_groups, const uint8_t *visible, int64_t N,
                         double beta1, double beta2, double eps, void *stream_ptr) {
    if (num_groups < 0 || num_groups > ADAM_MAX_GROUPS) return fail(GSR_ERR_ARG, "sparse adam: 0..16 parameter groups");
    if (num_groups && !groups) return fail(GSR_ERR_ARG, "sparse adam: null groups");
    if (N <= 0) return fail(GSR_ERR_ARG, "sparse adam: N must be positive");
    if (!visible) return fail(GSR_ERR_ARG, "sparse adam: null visibility");
    AdamLaunch L{};
    int64_t slices = 0;
    int ng = 0;
    for (int i = 0; i < num_groups; i++) {
        const gsr_adam_group &g = groups[i];
        if (g.n < 0) return fail(GSR_ERR_ARG, "sparse adam: n must be >= 0");
        if (g.n == 0) continue;
        if (g.n % N != 0) return fail(GSR_ERR_ARG, "sparse adam: a group's element count is not a multiple of N");
        if (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq) return fail(GSR_ERR_ARG, "sparse adam: null array");
        AdamGroupDev &d = L.g[ng];
        d.param = g.param; d.grad = g.grad; d.exp_avg = g.exp_avg; d.exp_avg_sq = g.exp_avg_sq; d.n = g.n;
        d.M = g.n / N;
        d.lr = (float)g.lr;
        d.vec4 = ((((uintptr_t)g.param) | ((uintptr_t)g.grad) | ((uintptr_t)g.exp_avg) |
                   ((uintptr_t)g.exp_avg_sq)) & 15) == 0;
        L.slice_start[ng] = slices;
        slices += adam_slices(g.n);
        ng++;
    }
    if (slices > 0x7fffffffLL) return fail(GSR_ERR_ARG, "sparse adam: too many elements");
    L.num_groups = ng;
    L.beta1 = (float)beta1;
    L.one_minus_beta1 = 1.0f - (float)beta1;  // the upstream kernel forms 1 - b1 in float
    L.beta2 = (float)beta2;
    L.one_minus_beta2 = 1.0f - (float)beta2;
    L.eps = (float)eps;
    L.visible = visible;
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_sparse_adam((hipStream_t)stream_ptr, L, slices);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

// densify workspace: [dst_map 2N i32 | split_rank N i32 | block_counts 3*blocks i32 | row_class N u8]
static size_t densify_ws(int64_t N, size_t *o_rank, size_t *o_blk, size_t *o_cls) {
    const size_t nb = (size_t)densify_blocks(N);
    *o_rank = align_up((size_t)N * 8, 256);
    *o_blk = *o_rank + align_up((size_t)N * 4, 256);
    *o_cls = *o_blk + align_up(nb * 12, 256);
    return *o_cls + align_up((size_t)N, 256);
}

size_t gsr_densify_workspace_bytes(int64_t N) {
    size_t a, b, c;
    return N < 0 ? 0 : densify_ws(N, &a, &b, &c);
}

int gsr_densify_classify(const gsr_densify_args *args, void *workspace, int32_t *counts, int64_t *preserve_idx,
                         void *stream_ptr) {
    if (!args || args->N < 0 || args->N > 0x7fffffffLL) return fail(GSR_ERR_ARG, "densify: 0 <= N < 2^31");
    if (!counts) return fail(GSR_ERR_ARG, "densify: null counts");
    DensifyParams p{};
    p.N = args->N;
    if (p.N > 0 && (!args->opacity || !args->scaling || !args->xyz_grad_accum || !args->xyz_grad_count ||
                    !workspace || !preserve_idx || (args->apply_screensize && !args->max_radii2D)))
        return fail(GSR_ERR_ARG, "densify: null input");
    size_t o_rank, o_blk, o_cls;
    densify_ws(p.N, &o_rank, &o_blk, &o_cls);
    char *ws = (char *)workspace;
    p.opacity = args->opacity; p.scaling = args->scaling; p.max_radii2D = args->max_radii2D;
    p.grad_accum = args->xyz_grad_accum; p.grad_count = args->xyz_grad_count;
    p.opacity_threshold = args->opacity_threshold; p.screensize_threshold = args->screensize_threshold;
    p.size_threshold = args->size_threshold; p.grad_threshold = args->grad_threshold;
    p.clone_size_threshold = args->clone_size_threshold;
    p.apply_screensize = args->apply_screensize; p.apply_size = args->apply_size;
    p.dst_map = (int32_t *)ws;
    p.split_rank = (int32_t *)(ws + o_rank);
    p.block_counts = (int32_t *)(ws + o_blk);
    p.row_class = (uint8_t *)(ws + o_cls);
    p.counts = counts;
    p.preserve_idx = preserve_idx;
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_densify_classify((hipStream_t)stream_ptr, p);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

int gsr_densify_apply(int64_t N, const void *workspace, const float *rotation, const float *scaling, const float *z,
                      const gsr_densify_field *fields, int num_fields, void *stream_ptr) {
    if (N < 0 || N > 0x7fffffffLL) return fail(GSR_ERR_ARG, "densify: 0 <= N < 2^31");
    if (num_fields < 0 || num_fields > DENSIFY_MAX_FIELDS) return fail(GSR_ERR_ARG, "densify: 0..16 fields");
    if (N == 0 || num_fields == 0) return GSR_OK;
    if (!workspace || !fields || !rotation || !scaling) return fail(GSR_ERR_ARG, "densify: null input");
    size_t o_rank, o_blk, o_cls;
    densify_ws(N, &o_rank, &o_blk, &o_cls);
    DensifyApply A{};
    A.N = N;
    A.dst_map = (const int32_t *)workspace;
    A.split_rank = (const int32_t *)((const char *)workspace + o_rank);
    A.z = z; A.rotation = rotation; A.scaling = scaling;
    int64_t blocks = 0;
    for (int i = 0; i < num_fields; i++) {
        const gsr_densify_field &f = fields[i];
        if (f.width <= 0 || !f.src || !f.dst) return fail(GSR_ERR_ARG, "densify: field needs src, dst, width > 0");
        if (f.kind < GSR_FIELD_PLAIN || f.kind > GSR_FIELD_STAT) return fail(GSR_ERR_ARG, "densify: bad kind");
        if (f.kind == GSR_FIELD_XYZ && f.width != 3) return fail(GSR_ERR_ARG, "densify: xyz field width must be 3");
        if ((f.dst_exp_avg && !f.src_exp_avg) || (f.dst_exp_avg_sq && !f.src_exp_avg_sq))
            return fail(GSR_ERR_ARG, "densify: moment destination without source");
        DensifyFieldDev &d = A.f[i];
        d.src = f.src; d.dst = f.dst; d.src_exp_avg = f.src_exp_avg; d.src_exp_avg_sq = f.src_exp_avg_sq;
        d.dst_exp_avg = f.dst_exp_avg; d.dst_exp_avg_sq = f.dst_exp_avg_sq; d.width = f.width; d.kind = f.kind;
        A.block_start[i] = blocks;
        blocks += (N * f.width + 255) / 256;
    }
    if (blocks > 0x7fffffffLL) return fail(GSR_ERR_ARG, "densify: too many elements");
    A.num_fields = num_fields;
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_densify_apply((hipStream_t)stream_ptr, A, blocks);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

static int ply_setup(PlyLaunch &p, int64_t n, int record_bytes, int big_endian, const gsr_ply_column *columns,
                     int num_columns, const float *const *fields, const int *widths, int num_fields, bool pack) {
    if (n < 0 || record_bytes <= 0 || record_bytes > 48 * 1024) return fail(GSR_ERR_ARG, "ply: bad n or record size");
    if (num_columns < 0 || num_columns > PLY_MAX_COLS) return fail(GSR_ERR_ARG, "ply: at most 128 columns");
    if (num_fields < 0 || num_fields > PLY_MAX_FIELDS) return fail(GSR_ERR_ARG, "ply: at most 8 fields");
    if ((num_columns && !columns) || (num_fields && (!fields || !widths))) return fail(GSR_ERR_ARG, "ply: null table");
    int sum = 0;
    for (int f = 0; f < num_fields; f++) {
        if (widths[f] <= 0 || (n > 0 && !fields[f])) return fail(GSR_ERR_ARG, "ply: field needs width > 0 and data");
        p.field[f] = const_cast<float *>(fields[f]);
        p.width[f] = widths[f];
        sum += widths[f];
    }
    if (sum != num_columns) return fail(GSR_ERR_ARG, "ply: field widths must add up to the column count");
    static const int kSize[8] = {4, 8, 1, 1, 2, 2, 4, 4};
    for (int c = 0; c < num_columns; c++) {
        const gsr_ply_column &col = columns[c];
        if (col.type < GSR_PLY_FLOAT32 || col.type > GSR_PLY_INT32) return fail(GSR_ERR_ARG, "ply: bad column type");
        if (pack && col.type != GSR_PLY_FLOAT32) return fail(GSR_ERR_ARG, "ply: pack writes float32 columns only");
        if (col.offset < 0 || col.offset + kSize[col.type] > record_bytes)
            return fail(GSR_ERR_ARG, "ply: column outside the record");
        p.cols[c] = make_int2(col.offset, col.type);
    }
    p.n = n;
    p.record_bytes = record_bytes;
    p.rows_per_block = ply_rows_per_block(record_bytes);
    p.ncols = num_columns;
    p.nfields = num_fields;
    p.swap = big_endian ? 1 : 0;
    return GSR_OK;
}

int gsr_ply_unpack(const uint8_t *records, int64_t n, int record_bytes, int big_endian, const gsr_ply_column *columns,
                   int num_columns, float *const *fields, const int *widths, int num_fields, void *stream_ptr) {
    PlyLaunch p{};
    const int rc = ply_setup(p, n, record_bytes, big_endian, columns, num_columns, fields, widths, num_fields, false);
    if (rc != GSR_OK) return rc;
    if (n > 0 && !records) return fail(GSR_ERR_ARG, "ply: null records");
    p.records = records;
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_ply((hipStream_t)stream_ptr, p, false);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

int gsr_ply_pack(uint8_t *records, int64_t n, int record_bytes, int big_endian, const gsr_ply_column *columns,
                 int num_columns, const float *const *fields, const int *widths, int num_fields, void *stream_ptr) {
    PlyLaunch p{};
    const int rc = ply_setup(p, n, record_bytes, big_endian, columns, num_columns, fields, widths, num_fields, true);
    if (rc != GSR_OK) return rc;
    if (n > 0 && !records) return fail(GSR_ERR_ARG, "ply: null records");
    p.records_out = records;
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_ply((hipStream_t)stream_ptr, p, true);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

size_t gsr_knn_workspace_bytes(int64_t n) { return n < 0 ? 0 : knn_workspace(n, nullptr); }

int gsr_knn_mean_dist2(int64_t n, const float *points, float *out, void *workspace, void *stream_ptr) {
    if (n < 0 || n > (int64_t)RS_ONESWEEP_MAX_N) return fail(GSR_ERR_ARG, "knn: 0 <= n < 2^30");
    if (n == 0) return GSR_OK;
    if (!points || !out || !workspace) return fail(GSR_ERR_ARG, "knn: null pointer");
    KnnScratch k{};
    k.base = workspace;
    knn_workspace(n, &k);
    StreamDeviceGuard device_guard((hipStream_t)stream_ptr);
    launch_knn((hipStream_t)stream_ptr, k, points, n, out);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

size_t gsr_ssim_num_partials(int planes, int H, int W) {
    return (planes > 0 && H > 0 && W > 0) ? ssim_num_partials(planes, H, W) : 0;
}

int gsr_ssim_forward(int planes, int H, int W, const float *img1, const float *img2, int valid_padding,
                     float *partial_sums, float *dm_dmu1, float *dm_dsigma1_sq, float *dm_dsigma12, void *stream_ptr) {
    if (planes <= 0 || H <= 0 || W <= 0) return fail(GSR_ERR_ARG, "ssim: empty image");
    if ((int64_t)planes * H * W > 0x7fffffffLL) return fail(GSR_ERR_ARG, "ssim: image too large");
    if (planes > 65535) return fail(GSR_ERR_ARG, "ssim: too many planes");
    if (!img1 || !img2 || !partial_sums) return fail(GSR_ERR_ARG, "ssim: null argument");
    if ((dm_dmu1 == nullptr) != (dm_dsigma1_sq == nullptr) || (dm_dmu1 == nullptr) != (dm_dsigma12 == nullptr))
        return fail(GSR_ERR_ARG, "ssim: derivative maps must be all given or all NULL");
    hipStream_t s = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(s);
    launch_ssim_forward(s, planes, H, W, img1, img2, valid_padding, partial_sums, dm_dmu1, dm_dsigma1_sq, dm_dsigma12);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

int gsr_ssim_backward(int planes, int H, int W, const float *img1, const float *img2, int valid_padding,
                      const float *dL_dmean, const float *dm_dmu1, const float *dm_dsigma1_sq,
                      const float *dm_dsigma12, float *dL_dimg1, void *stream_ptr) {
    if (planes <= 0 || H <= 0 || W <= 0) return fail(GSR_ERR_ARG, "ssim: empty image");
    if (planes > 65535) return fail(GSR_ERR_ARG, "ssim: too many planes");
    if (!img1 || !img2 || !dL_dmean || !dm_dmu1 || !dm_dsigma1_sq || !dm_dsigma12 || !dL_dimg1)
        return fail(GSR_ERR_ARG, "ssim: null argument");
    const int64_t counted = (int64_t)planes * (valid_padding ? (int64_t)(H - 10) * (W - 10) : (int64_t)H * W);
    if (counted <= 0) return fail(GSR_ERR_ARG, "ssim: image smaller than the valid window");
    hipStream_t s = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(s);
    launch_ssim_backward(s, planes, H, W, img1, img2, valid_padding, dL_dmean, (float)(1.0 / (double)counted), dm_dmu1,
                         dm_dsigma1_sq, dm_dsigma12, dL_dimg1);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

int gsr_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix, uint8_t *present,
                     void *stream_ptr) {
    (void)projmatrix;
    if (P < 0) return fail(GSR_ERR_ARG, "P must be >= 0");
    if (P == 0) return GSR_OK;
    if (!means3D || !viewmatrix || !present) return fail(GSR_ERR_ARG, "null argument");
    hipStream_t s = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(s);
    launch_mark_visible(s, P, means3D, viewmatrix, present);
    GSR_HIP(hipGetLastError());
    return GSR_OK;
}

void gsr_set_tuning(const char *name, int value) {
    if (!name) return;
    std::lock_guard<std::mutex> lk(g_tune_mu);
    for (size_t k = 0; k < g_tune.size(); k++)
        if (g_tune[k].first == name) {
            if (value == GSR_TUNING_UNSET) g_tune.erase(g_tune.begin() + (long)k);  // back to the built-in default
            else g_tune[k].second = value;
            return;
        }
    if (value != GSR_TUNING_UNSET) g_tune.emplace_back(name, value);
}

int gsr_get_tuning(const char *name, int default_value) { return name ? tuning(name, default_value) : default_value; }

int gsr_debug_wave_stamps(int which, uint32_t *host_dst, int max_slots) {
    uint4 *b = stamp_buffer(which);
    if (!b || !host_dst) return fail(GSR_ERR_ARG, "no stamp buffer");
    const int n = max_slots < STAMP_SLOTS ? max_slots : STAMP_SLOTS;
    GSR_HIP(hipDeviceSynchronize());
    GSR_HIP(hipMemcpy(host_dst, b, sizeof(uint4) * (size_t)n, hipMemcpyDeviceToHost));
    return n;
}

void gsr_set_profiling(int enable) {
    Profiler &p = prof();
    std::lock_guard<std::mutex> lk(p.mu);
    p.enabled = enable != 0;
}
int gsr_num_stages(void) { return ST_COUNT; }
const char *gsr_stage_name(int stage) { return (stage >= 0 && stage < ST_COUNT) ? kStageNames[stage] : ""; }
int gsr_stage_times(double *total_ms, int64_t *calls, int max_stages) {
    Profiler &p = prof();
    std::lock_guard<std::mutex> lk(p.mu);
    p.drain();
    const int n = max_stages < ST_COUNT ? max_stages : ST_COUNT;
    for (int i = 0; i < n; i++) {
        if (total_ms) total_ms[i] = p.total_ms[i];
        if (calls) calls[i] = p.calls[i];
    }
    return n;
}
void gsr_reset_stage_times(void) {
    Profiler &p = prof();
    std::lock_guard<std::mutex> lk(p.mu);
    p.drain();
    for (int i = 0; i < ST_COUNT; i++) {
        p.total_ms[i] = 0;
        p.calls[i] = 0;
    }
}
const char *gsr_last_error(void) { return g_err.c_str(); }
int gsr_abi_version(void) { return GSR_ABI_VERSION; }

int gsr_stream_values_supported(void) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, dev) != hipSuccess) return 0;
    return v;
}

int gsr_stream_signal(void *stream_ptr, uint32_t *flag, uint32_t value) {
    if (!flag) return fail(GSR_ERR_ARG, "stream signal: null flag");
    hipStream_t stream = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(stream);
    GSR_HIP(hipStreamWriteValue32(stream, flag, value, 0));
    return GSR_OK;
}

int gsr_stream_wait(void *stream_ptr, uint32_t *flag, uint32_t value) {
    if (!flag) return fail(GSR_ERR_ARG, "stream wait: null flag");
    hipStream_t stream = (hipStream_t)stream_ptr;
    StreamDeviceGuard device_guard(stream);
    GSR_HIP(hipStreamWaitValue32(stream, flag, value, hipStreamWaitValueGte, 0xffffffffu));
    return GSR_OK;
}
const char *gsr_build_info(void) {
    return "gsrast: MI355X (gfx950) HIP rasterizer; wave64 tile compositing, LSD radix binning, "
           "deterministic gradient rows; built " __DATE__ " " __TIME__;
}

}  // extern "C"
