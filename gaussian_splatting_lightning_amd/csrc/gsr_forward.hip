// gsr_forward.hip -- forward kernels: preprocess, tile expansion, tile ranges, compositing, frustum test.
//
// Semantics follow the upstream CUDA rasterizer the reference calls ([U]) and are
// pinned against the reference's Python restatement through tests/golden (oracle/gsr_oracle.c):
//   preprocess   <-> gs_lightning/rasterize/rasterize.py:52-94, render_tools.py:13-131
//   binning      <-> rasterize.py:129-152, render_tools.py:134-139
//   compositing  <-> rasterize.py:210-261 with the CUDA termination rule
#include "gsr_kernels.h"
#include "gsr_sh.h"

namespace gsr {

// ------------------------------------------------------------------------------------------------
// preprocess: one thread per Gaussian.  Culls, projects, builds the conic and radius, evaluates SH,
// and emits the packed render records plus the depth-sort key and tile count.
// ------------------------------------------------------------------------------------------------
// Per-Gaussian state handed from the projection to the wave-cooperative tile culling.
struct CullIn {
    CullGauss cg;
    int rx, ry, rw;   // rect origin and width (tiles)
    uint32_t depth;   // float bits of the view depth
    bool need;        // cull the rect's tiles cooperatively
    bool vis;         // rendered (radius > 0): its colour is needed, even when culling leaves no tile
};

// Projection, conic, radius, SH colour and render records of one Gaussian.  Returns the area of its tile
// rect (0: not rendered); the tile culling, tile count and sort key are finished by preprocess_kernel.
// SHD >= 0: the SH degree at compile time (the common degree-3 launch).  With the runtime switch the compiler hoists the
// degree-0 term common to every case (the first coefficient's load and multiply) above the switch, so the other 45
// coefficients were only requested after that load had returned: one more memory round trip per wave.
template <int SHD = -1>
__device__ __forceinline__ uint32_t preprocess_gaussian(const PreprocessParams &p, const int i, CullIn &ci) {
    // uncontracted like the helpers it calls (gsr_common.h): radii, rects and render records bit-equal the oracle's
#pragma clang fp contract(off)
    const GeomState &g = p.g;
    // radii / clamped are stored once, below, for a rendered Gaussian; preprocess_kernel stores the zeros of the
    // others and the tile count and depth key of every Gaussian (one store per word, not a zero then the value)

    // Every per-Gaussian input except the SH block is loaded up front, before the frustum test, so a wave waits
    // for one memory round trip instead of one per dependent stage (the 27 % of loads for culled Gaussians at
    // cfg 3 cost ~12 MB).
    const Mat4 view = load_mat4(p.view);
    const float3 mean = load_f3(p.means3D, i);
    const float opacity_in = p.opacities[i];
    float4 q = make_float4(1.f, 0.f, 0.f, 0.f);
    float3 sc = make_float3(0.f, 0.f, 0.f);
    if (!p.cov3D_precomp) {
        q = make_float4(p.rotations[4 * i], p.rotations[4 * i + 1], p.rotations[4 * i + 2], p.rotations[4 * i + 3]);
        sc = load_f3(p.scales, i);
    }
    // the camera position too (it was loaded, and waited for, just before the coefficients)
    const float3 campos = p.campos ? make_float3(p.campos[0], p.campos[1], p.campos[2]) : make_float3(0.f, 0.f, 0.f);
    const float3 dir_raw = mean - campos;  // formed here: later the compiler re-loaded the mean (another round trip)
    const float3 pv = xform3(mean, view);
    if (!(pv.z > 0.2f)) return 0u;  // in_frustum (camera_tools.py:5-8)

    const Mat4 proj = load_mat4(p.proj);
    const float4 ph = xform4(mean, proj);
    const float pw = 1.0f / (ph.w + 0.0000001f);
    const float ndc_x = ph.x * pw, ndc_y = ph.y * pw;

    float c6[6];
    if (p.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; k++) c6[k] = p.cov3D_precomp[6 * i + k];
    } else {
        cov3d_from_scale_rot(sc, p.scale_modifier, q, c6);
    }
    const EwaT e = ewa_T(mean, view, p.focal_x, p.focal_y, p.tan_fovx, p.tan_fovy);
    float cxx = quad_form(e.t0, c6, e.t0);
    const float cxy = quad_form(e.t1, c6, e.t0);
    float cyy = quad_form(e.t1, c6, e.t1);
    constexpr float h_var = 0.3f;
    const float det_cov = cxx * cyy - cxy * cxy;
    cxx += h_var;
    cyy += h_var;
    const float det = cxx * cyy - cxy * cxy;
    float hscale = 1.0f;
    if (p.antialiasing) hscale = sqrtf(fmaxf(0.000025f, det_cov / det));
    if (det == 0.0f) return 0u;
    const float det_inv = 1.f / det;
    const float conic_x = cyy * det_inv, conic_y = -cxy * det_inv, conic_z = cxx * det_inv;
    const float mid = 0.5f * (cxx + cyy);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    const float2 pimg = make_float2(ndc2pix(ndc_x, p.W), ndc2pix(ndc_y, p.H));
    int2 rmin, rmax;
    get_rect(pimg, (int)radius, p.gx, p.gy, rmin, rmax);
    const uint32_t area = (uint32_t)((rmax.x - rmin.x) * (rmax.y - rmin.y));
    if (area == 0) return 0u;

    ci.vis = true;
    const float opacity = opacity_in * hscale;
    float3 rgb = make_float3(0.f, 0.f, 0.f);
    uint8_t clamp_bits = 0;
    if (p.colors_precomp) {
        rgb = load_f3(p.colors_precomp, i);
    } else {
        float3 dir = dir_raw;
        const float len = sqrtf(dot3(dir, dir));
        dir = make_float3(dir.x / len, dir.y / len, dir.z / len);
        if (SHD > 0 || (SHD < 0 && p.D > 0)) {  // the colour and its direction Jacobian for the backward (9 planes)
            float3 jx, jy, jz;
            if constexpr (SHD > 0) rgb = sh_eval_jac<SHD>(p.shs + (size_t)i * p.M * 3, dir, jx, jy, jz);
            else rgb = sh_eval_jac_dispatch(p.D, p.shs + (size_t)i * p.M * 3, dir, jx, jy, jz);
            const size_t n = (size_t)p.P;
            float *J = g.sh_jac + i;
            J[0] = jx.x; J[n] = jx.y; J[2 * n] = jx.z;
            J[3 * n] = jy.x; J[4 * n] = jy.y; J[5 * n] = jy.z;
            J[6 * n] = jz.x; J[7 * n] = jz.y; J[8 * n] = jz.z;
        } else {
            rgb = sh_dispatch(p.D, p.shs + (size_t)i * p.M * 3, dir);
        }
        rgb = sh_offset(rgb);
        clamp_bits = (rgb.x < 0.f ? 1 : 0) | (rgb.y < 0.f ? 2 : 0) | (rgb.z < 0.f ? 4 : 0);
        rgb = make_float3(fmaxf(rgb.x, 0.f), fmaxf(rgb.y, 0.f), fmaxf(rgb.z, 0.f));
    }
    g.rec[i].a = make_float4(pimg.x, pimg.y, conic_x, conic_y);
    g.rec[i].b = make_float4(conic_z, opacity, rgb.x, rgb.y);
    // the whole 48-B row (pad included), so the record array is written in full lines
    *reinterpret_cast<float4 *>(&g.rec[i].c) = make_float4(rgb.z, 1.f / pv.z, 0.f, 0.f);
    g.clamped[i] = clamp_bits;
    p.radii[i] = (int)radius;
    // culling (p.cull): the reference rect shrinks to the tight rect (cull_rect), whose tiles are then tested one by
    // one when there are at most CULL_MAX_AREA of them
    uint32_t tarea = area;
    ci.need = false;
    if (p.cull) {
        ci.cg = cull_setup(pimg.x, pimg.y, conic_x, conic_y, conic_z, opacity);
        cull_rect(ci.cg, rmin.x, rmin.y, rmax.x, rmax.y);
        tarea = (uint32_t)((rmax.x - rmin.x) * (rmax.y - rmin.y));
        ci.need = tarea > 0 && tarea <= (uint32_t)CULL_MAX_AREA;
    }
    ci.rx = rmin.x;
    ci.ry = rmin.y;
    ci.rw = rmax.x - rmin.x;
    ci.depth = __float_as_uint(pv.z);
    return tarea;
}

// Exact tile culling is balanced across the wave: the (Gaussian, tile) pairs of all 64 lanes' rects are
// enumerated jointly (prefix sum of the rect areas, each lane takes every 64th pair, owner found by marks and a
// max-scan), so a wave costs ceil(sum of areas / 64) tile tests instead of its largest rect.
//
// With p.block_sums (bucket binning) every block also stores its kept-tile total, from which the bucket count
// pass forms the Gaussian-order instance offsets.
#ifndef GSR_PRE_MINW
#define GSR_PRE_MINW 4  // 112 VGPRs, no spills: cfg3 0.106 -> 0.103 ms against 5 waves (96 VGPRs, 2 spilled); 6: 0.112
#endif
struct PreCullLds {
    CullGauss cg[64];
    int4 rect[64];  // rx, ry, rw, start of the lane's pairs
    unsigned long long mask[64];
    int own[64];    // lane whose rect's pair run starts at this pair of the step, else -1
};
__device__ __forceinline__ void publish_total(const PreprocessParams &p);

// The colour is evaluated inside preprocess_gaussian, each lane reading its own 192-B coefficient row.  (Rounds 4-5
// measured a split colour kernel behind the bucket count pass and a late, LDS-staged colour phase: both slower,
// DESIGN.md Appendix A.4; removed in round 6.)
template <int SHD = -1>
__global__ __launch_bounds__(256, GSR_PRE_MINW) void preprocess_kernel(PreprocessParams p) {
    __shared__ PreCullLds s_lds[4];
    __shared__ uint32_t s_w[4];
    const uint32_t bid = blockIdx.x;
    const int i = (int)bid * 256 + threadIdx.x;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    PreCullLds &L = s_lds[w];
    CullIn ci;
    ci.need = false;
    ci.vis = false;
    const uint32_t t_start = p.stamps ? stamp_now() : 0u;
    const uint32_t area = i < p.P ? preprocess_gaussian<SHD>(p, i, ci) : 0u;
    const uint32_t t_proj = p.stamps ? stamp_now() : 0u;
    const uint32_t need_area = ci.need ? area : 0u;
    const uint32_t incl = wave_inclusive_scan(need_area, lane);
    const uint32_t total = __shfl((int)incl, 63);
    if (ci.need) L.cg[lane] = ci.cg;
    // rw <= CULL_MAX_AREA and a pair's offset t < CULL_MAX_AREA = 64, so t / rw == (t * ceil(4096 / rw)) >> 12 exactly
    // (the rounding up adds t * (ceil - 4096 / rw) / 4096 < 64 / 4096 = 1/64 to a quotient whose fraction is at most
    // 63/64): two integer multiplies instead of the ~20-instruction unsigned division in the loop
    L.rect[lane] = make_int4(ci.rx, ci.ry, ci.rw | (ci.need ? (int)((4096u + ci.rw - 1) / ci.rw) << 16 : 0),
                             (int)(incl - need_area));
    L.mask[lane] = 0ull;
    // pair owners by marks and a max-scan (as the bucket walk): the lane whose pair run starts inside the step
    // marks its start, and every pair takes the largest marking lane at or before it (or the previous step's last
    // owner) -- one LDS round trip per step instead of a 6-deep dependent binary search over the starts (cfg 3
    // preprocess 0.1092 -> 0.1080 ms)
    L.own[lane] = -1;
    const uint32_t my_start = incl - need_area;
    int carry = -1;
    wave_lds_sync();
    for (uint32_t B = 0; B < total; B += 64) {
        const uint32_t j = B + (uint32_t)lane;
        const bool marks = need_area > 0 && my_start >= B && my_start < B + 64;
        if (marks) L.own[my_start - B] = lane;
        wave_lds_sync();
        const int o = max(wave_inclusive_max(L.own[lane]), carry);
        carry = __builtin_amdgcn_readlane(o, 63);
        wave_lds_sync();
        if (marks) L.own[my_start - B] = -1;
        if (j >= total) continue;
        const int4 r = L.rect[o];
        const uint32_t t = j - (uint32_t)r.w, rw = (uint32_t)r.z & 0xffffu;
        const uint32_t qy = (t * ((uint32_t)r.z >> 16)) >> 12;
        const int tx = r.x + (int)(t - qy * rw), ty = r.y + (int)qy;
        if (cull_keep(L.cg[o], tx, ty, p.W, p.H)) atomicOr(&L.mask[o], 1ull << t);
    }
    wave_lds_sync();
    const uint32_t t_cull = p.stamps ? stamp_now() : 0u;
    uint32_t kept = area;
    if (i < p.P) {
        const GeomState &g = p.g;
        if (area > 0) {
            const uint64_t mask = ci.need ? L.mask[lane] : 0ull;
            if (ci.need) kept = (uint32_t)__popcll(mask);
            g.exp_rec[i] = make_uint4((uint32_t)mask, (uint32_t)(mask >> 32), (uint32_t)ci.rx | ((uint32_t)ci.ry << 16),
                                      (uint32_t)ci.rw);
            if (kept > BIG_GAUSSIAN_TILES) {
                const uint32_t slot = atomicAdd(&g.counters[CNT_BIG], 1u);
                g.big_list[slot] = (uint32_t)i;
                g.big_slot[i] = slot;
            }
        } else if (!ci.vis) {  // not rendered: no radius, no clamp bits
            p.radii[i] = 0;
            g.clamped[i] = 0;
        }
        g.tiles[i] = kept;
        g.live[i] = 0;  // (set by the compositing backward for a Gaussian it stores a non-zero row of)
        // A Gaussian whose every tile is culled keeps its radius (reference output) but renders nothing; it
        // is sorted behind all rendered ones so the expansion never meets an empty rank.
        g.depth_key[i] = kept ? ci.depth : 0xffffffffu;
    }
    // instance total for the early host readback (gsr_forward): block sum, one 64-bit atomic per block into
    // one of CNT_NPART partial counters; likewise the range of the kept depth keys (the radix path's relative
    // depth sort), as the largest complemented key and the largest key
    // (only where the radix path's relative depth sort can use it: p.depth_range)
    uint32_t wmin = 0xffffffffu, wmax = 0u;
    if (p.depth_range) {
        const uint32_t my_dk = (i < p.P && area > 0 && kept > 0) ? ci.depth : 0xffffffffu;
        wmin = wave_min_u32(my_dk);
        wmax = wave_max_u32(my_dk == 0xffffffffu ? 0u : my_dk);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) kept += (uint32_t)__shfl_xor((int)kept, o);
    __shared__ uint32_t s_dmin[4], s_dmax[4];
    if (lane == 0) {
        s_w[w] = kept;
        s_dmin[w] = wmin;
        s_dmax[w] = wmax;
    }
    __syncthreads();
    __shared__ uint32_t s_last;
    if (threadIdx.x == 0) {
        const unsigned long long tot = (unsigned long long)s_w[0] + s_w[1] + s_w[2] + s_w[3];
        unsigned long long old = 0;
        if (tot) {
            const uint32_t bmin = min(min(s_dmin[0], s_dmin[1]), min(s_dmin[2], s_dmin[3]));
            const uint32_t bmax = max(max(s_dmax[0], s_dmax[1]), max(s_dmax[2], s_dmax[3]));
            if (p.depth_range) {
                atomicMax(p.g.counters + CNT_DMIN + (bid % CNT_NPART), ~bmin);
                atomicMax(p.g.counters + CNT_DMAX + (bid % CNT_NPART), bmax);
            }
            old = atomicAdd(reinterpret_cast<unsigned long long *>(p.g.counters + CNT_PARTIALS) + (bid % CNT_NPART), tot);
        }
        if (p.block_sums) p.block_sums[bid] = (uint32_t)tot;  // <= 256 * 2^16 tiles
        if (p.host_words) {
            // The workgroup's counter atomics have all returned before its ticket is taken (the big-slot ones before
            // the barrier, the partial sum here: its result is waited for), so the workgroup that draws the last
            // ticket sees every count.  No fence: an agent-scope release writes back the XCD's L2, ~60 ns per
            // workgroup, which over 3906 workgroups tripled the kernel.
            asm volatile("" ::"v"(old));
            s_last = atomicAdd(&p.g.counters[CNT_PRE_DONE], 1u) == gridDim.x - 1;
        }
    }
    if (p.host_words) {
        __syncthreads();
        if (s_last && threadIdx.x < 64) publish_total(p);
    }
    if (p.stamps && lane == 0 && (int)(bid * 4 + w) < STAMP_SLOTS / 2) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        p.stamps[2 * (bid * 4 + w)] = make_uint4(t_start, t_proj, t_cull, stamp_now());
        p.stamps[2 * (bid * 4 + w) + 1] = make_uint4(hw, xcc, 0u, 0u);
    }
}

// The last preprocess workgroup publishes {instance total lo, hi, big count, seq} to pinned host memory in ONE 16-B
// store (the host reads it with one 16-B load and trusts it when the sequence word matches), so no release fence is
// needed: a system-scope release writes back the L2 first and delayed the host's view by ~35 us.  Threads 0-63.
__device__ __forceinline__ void publish_total(const PreprocessParams &p) {
    const unsigned long long part = __hip_atomic_load(
        reinterpret_cast<unsigned long long *>(p.g.counters + CNT_PARTIALS) + threadIdx.x, __ATOMIC_RELAXED,
        __HIP_MEMORY_SCOPE_AGENT);  // CNT_NPART == 64: one partial per lane
    const uint32_t kmin = ~wave_max_u32(__hip_atomic_load(p.g.counters + CNT_DMIN + threadIdx.x, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t kmax = wave_max_u32(__hip_atomic_load(p.g.counters + CNT_DMAX + threadIdx.x, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT));
    const unsigned long long lo = (uint32_t)part, hi = part >> 32;
    unsigned long long slo = lo, shi = hi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        slo += (unsigned long long)__shfl_xor((long long)slo, o);
        shi += (unsigned long long)__shfl_xor((long long)shi, o);
    }
    if (threadIdx.x == 0) {
        const unsigned long long total = slo + (shi << 32);
        const uint32_t nbig = __hip_atomic_load(&p.g.counters[CNT_BIG], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 r = {kmin, kmax, p.seq, 0u};  // the depth range word first (the host reads it second)
        __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(p.host_words + CNT_WORDS + 4));
        const u32x4 v = {(uint32_t)total, (uint32_t)(total >> 32), nbig, p.seq};
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p.host_words + CNT_WORDS));
    }
}

void launch_preprocess(hipStream_t s, const PreprocessParams &p) {
    if (p.P <= 0) return;
    if (p.D == 3 && !p.colors_precomp) preprocess_kernel<3><<<div_up(p.P, 256), 256, 0, s>>>(p);
    else preprocess_kernel<><<<div_up(p.P, 256), 256, 0, s>>>(p);
}

// Zero fill of the forward's counter block (16-B aligned, a multiple of 16 B) by a plain kernel: the runtime's fill
// (hipMemsetAsync) ran 4.4 us at cfg 3 and the trace showed a ~6-us gap in front of it every step.
__global__ __launch_bounds__(256) void zero16_kernel(uint4 *__restrict__ p, uint32_t n16) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) p[i] = make_uint4(0u, 0u, 0u, 0u);
}
void launch_zero16(hipStream_t s, void *p, size_t bytes) {
    const uint32_t n16 = (uint32_t)(bytes / 16);
    if (n16 == 0) return;
    zero16_kernel<<<std::min(div_up(n16, 256u), 256u), 256, 0, s>>>(reinterpret_cast<uint4 *>(p), n16);
}

// ------------------------------------------------------------------------------------------------
// expand: instances are laid out in depth-rank order (Gaussian order[r] owns [inst_off[r], inst_off[r+1])).
// Each block owns a fixed slice of EXP_TILE instances (load balanced whatever the per-Gaussian tile
// counts are); its threads find their owning rank by a binary search over an LDS copy of the block's
// rank window and then walk EXP_PER consecutive instances, emitting the tile id (sort key) and the
// Gaussian id of each.
// ------------------------------------------------------------------------------------------------
constexpr int EXP_PER = 4;  // 1024 instances per block, 36 KB of LDS: 4 blocks/CU (cfg 5: 0.396 -> 0.380 ms; 2: 0.400)
constexpr int EXP_TILE = 256 * EXP_PER;

__global__ __launch_bounds__(256) void expand_kernel(ExpandParams p) {
    __shared__ uint32_t s_off[EXP_TILE + 2];
    __shared__ uint4 s_e[EXP_TILE + 1];     // expansion record: kept-tile mask lo, hi (0: all tiles), rmin, width
    __shared__ uint32_t s_gid[EXP_TILE + 1];
    static_assert(sizeof(uint4) == 16, "expansion record");
    __shared__ uint32_t s_lo, s_n;
    const uint32_t u0 = blockIdx.x * EXP_TILE;
    const uint32_t u1 = min(p.R, u0 + (uint32_t)EXP_TILE);
    if (threadIdx.x == 0) {  // owners of the block starts from expand_owner_kernel: one load instead of two searches
        const uint32_t lo = p.exp_owner[blockIdx.x];
        // the next block's first owner, or (last block) every remaining rank; ranks between two block starts
        // own >= 1 instance each, so at most EXP_TILE + 1 of them
        const uint32_t hi = blockIdx.x + 1 < gridDim.x ? p.exp_owner[blockIdx.x + 1] : p.P - 1;
        s_lo = lo;
        s_n = min(hi - lo + 1, (uint32_t)EXP_TILE + 1);
    }
    __syncthreads();
    const uint32_t r_lo = s_lo, nr = s_n;  // nr <= EXP_TILE + 1
    for (uint32_t k = threadIdx.x; k < nr + 1; k += 256) s_off[k] = p.inst_off[r_lo + k];
    for (uint32_t k = threadIdx.x; k < nr; k += 256) {
        const uint32_t gid = p.order[r_lo + k];
        // rect and kept-tile mask from the preprocess: in depth order already, or one 16-B gather
        s_e[k] = p.exp_sorted ? p.exp_sorted[r_lo + k] : p.exp_rec[gid];
        s_gid[k] = gid;
    }
    __syncthreads();
    // each thread expands EXP_PER consecutive instances and stores them as one 16-B vector per output array
    const uint32_t ub = u0 + threadIdx.x * EXP_PER;
    if (ub >= u1) return;
    // owner of ub within the window
    uint32_t lo = 0, hi = nr - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= ub) lo = mid; else hi = mid - 1;
    }
    uint32_t r = lo;
    uint32_t next = s_off[r + 1];
    uint4 e = s_e[r];
    uint32_t gid = s_gid[r];
    uint64_t m = (uint64_t)e.x | ((uint64_t)e.y << 32);
    uint32_t k = ub - s_off[r];
    if (m && k) m &= ~0ull << nth_set_bit(m, k);  // skip the kept tiles of earlier threads (k < popcount(m))
    float rw = __builtin_amdgcn_rcpf((float)e.w);
    uint32_t key[EXP_PER], gv[EXP_PER];
#pragma unroll
    for (int q = 0; q < EXP_PER; q++) {
        const uint32_t u = ub + q;
        key[q] = 0;
        gv[q] = 0;
        if (u < u1) {
            while (u >= next) {
                r++;
                next = s_off[r + 1];
                e = s_e[r];
                gid = s_gid[r];
                m = (uint64_t)e.x | ((uint64_t)e.y << 32);
                rw = __builtin_amdgcn_rcpf((float)e.w);
                k = 0;
            }
            uint32_t bit = k;
            if (m) {  // culled rect: the k-th kept tile is the lowest remaining mask bit
                bit = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
            }
            // bit / w through the reciprocal (bit < 2^24: off by at most one, corrected)
            const uint32_t w = e.w;
            uint32_t dy = (uint32_t)((float)bit * rw);
            int32_t dx = (int32_t)(bit - dy * w);
            if (dx < 0) { dy--; dx += (int32_t)w; }
            if (dx >= (int32_t)w) { dy++; dx -= (int32_t)w; }
            const uint32_t ty = (e.z >> 16) + dy, tx = (e.z & 0xffffu) + (uint32_t)dx;
            key[q] = ty * (uint32_t)p.gx + tx;
            gv[q] = gid;
            if (k == 0) p.inst_start[gid] = u;
            k++;
        }
    }
    if (ub + EXP_PER <= u1) {
        static_assert(EXP_PER == 4, "one uint4 store per thread");
        if (p.keys16_out)
            *reinterpret_cast<uint2 *>(p.keys16_out + ub) = make_uint2(key[0] | (key[1] << 16), key[2] | (key[3] << 16));
        else
            *reinterpret_cast<uint4 *>(p.keys_out + ub) = make_uint4(key[0], key[1], key[2], key[3]);
        *reinterpret_cast<uint4 *>(p.inst_gid + ub) = make_uint4(gv[0], gv[1], gv[2], gv[3]);
        if (p.inv_none) *reinterpret_cast<uint4 *>(p.inv_none + ub) = make_uint4(INV_NONE, INV_NONE, INV_NONE, INV_NONE);
    } else {
        for (uint32_t u = ub; u < u1; u++) {
            if (p.keys16_out) p.keys16_out[u] = (uint16_t)key[u - ub];
            else p.keys_out[u] = key[u - ub];
            p.inst_gid[u] = gv[u - ub];
            if (p.inv_none) p.inv_none[u] = INV_NONE;
        }
    }
}

// exp_owner[b] = the depth rank owning instance b * EXP_TILE (its inst_off range contains it): each rank writes
// the block starts inside its own range, so every entry b < div_up(R, EXP_TILE) is written exactly once.
__global__ __launch_bounds__(256) void expand_owner_kernel(const uint32_t *__restrict__ inst_off, uint32_t P,
                                                           uint32_t *__restrict__ exp_owner) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= P) return;
    const uint32_t a = inst_off[r], e = inst_off[r + 1];
    for (uint32_t b = (uint32_t)(((uint64_t)a + EXP_TILE - 1) / EXP_TILE); b * (uint64_t)EXP_TILE < e; b++) exp_owner[b] = r;
}

void launch_expand(hipStream_t s, const ExpandParams &p) {
    if (p.R == 0) return;
    expand_owner_kernel<<<div_up(p.P, 256u), 256, 0, s>>>(p.inst_off, p.P, p.exp_owner);
    expand_kernel<<<div_up(p.R, EXP_TILE), 256, 0, s>>>(p);
}

// ------------------------------------------------------------------------------------------------
// ranges: [start, end) of every tile's run in the sorted instance list
// ------------------------------------------------------------------------------------------------
// Tile boundaries of the sorted keys: 8 consecutive keys per thread (two 16-B loads) and the key before them.
constexpr uint32_t IR_PER = 8;
template <typename KT>
__global__ __launch_bounds__(256) void identify_ranges_kernel(const KT *__restrict__ keys, uint32_t R,
                                                              uint2 *__restrict__ ranges) {
    const uint32_t base = (blockIdx.x * 256 + threadIdx.x) * IR_PER;
    uint32_t k[IR_PER];
    if (base + IR_PER <= R) {
        if constexpr (sizeof(KT) == 2) {  // 8 keys in one 16-B load
            const uint4 a = *reinterpret_cast<const uint4 *>(keys + base);
            k[0] = a.x & 0xffffu; k[1] = a.x >> 16; k[2] = a.y & 0xffffu; k[3] = a.y >> 16;
            k[4] = a.z & 0xffffu; k[5] = a.z >> 16; k[6] = a.w & 0xffffu; k[7] = a.w >> 16;
        } else {
            const uint4 *k4 = reinterpret_cast<const uint4 *>(keys + base);
            const uint4 a = k4[0], b = k4[1];
            k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w; k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
        }
    } else {
#pragma unroll
        for (uint32_t q = 0; q < IR_PER; q++) k[q] = base + q < R ? keys[base + q] : 0u;
    }
    // the key before this thread's run: the previous lane's last key (one load per wave, not per thread); every
    // lane takes part in the shuffle, lanes past the end only lend their (unused) keys
    const int lane = threadIdx.x & 63;
    uint32_t prev = (uint32_t)__shfl_up((int)k[IR_PER - 1], 1);
    if (lane == 0) prev = (base > 0 && base <= R) ? keys[base - 1] : 0u;
    if (base == 0) ranges[k[0]].x = 0;
#pragma unroll
    for (uint32_t q = 0; q < IR_PER; q++) {
        const uint32_t i = base + q;
        if (i < R) {
            if (i > 0 && k[q] != prev) {
                ranges[prev].y = i;
                ranges[k[q]].x = i;
            }
            if (i == R - 1) ranges[k[q]].y = R;
            prev = k[q];
        }
    }
}

void launch_identify_ranges(hipStream_t s, const uint32_t *keys_sorted, uint32_t R, uint2 *ranges) {
    if (R == 0) return;
    identify_ranges_kernel<uint32_t><<<div_up(R, 256 * IR_PER), 256, 0, s>>>(keys_sorted, R, ranges);
}
void launch_identify_ranges16(hipStream_t s, const uint16_t *keys_sorted, uint32_t R, uint2 *ranges) {
    if (R == 0) return;
    identify_ranges_kernel<uint16_t><<<div_up(R, 256 * IR_PER), 256, 0, s>>>(keys_sorted, R, ranges);
}

// LPT (longest first) launch order for the composite kernels: tile costs vary ~2x around the image centre,
// and the GPU runs only ~8 tile waves per SIMD, so launching heavy tiles first keeps the tail short.  One
// workgroup: bucket histogram of the tile weights (2^shift instances per bucket, shift adapted to the heaviest
// tile), descending exclusive scan, scatter (lpt_order_block).  Order inside a bucket is arbitrary -- it only changes which tile runs when, never a result.
// (A 1024-bucket variant with ballot-ranked, tile-ordered buckets measured 4 % slower in render_fwd.)
__global__ __launch_bounds__(1024) void tile_order_kernel(const uint2 *__restrict__ ranges,
                                                             const uint32_t *__restrict__ tile_last, int use_last,
                                                             int T, int shift, uint32_t *__restrict__ order) {
    __shared__ uint32_t hist[LPT_HIST_WORDS];
    lpt_order_block(ranges, tile_last, use_last, T, shift, order, hist);
}

// More than 4096 tiles (1080p: 8160, 4K: 32400): the order by LPT_WG_TILES-tile workgroups in two launches, a per-workgroup histogram of
// scale-free buckets (lpt_log_bucket) and a scatter from the bucket bases every workgroup forms from all histograms
// (one 1024-thread workgroup over 32400 tiles took 40-47 us).
constexpr int LPT_WG_TILES = 4096;
__device__ __forceinline__ uint32_t lpt_weight(const uint2 *ranges, const uint32_t *tile_last, int use_last, int t) {
    return use_last ? tile_last[t] : ranges[t].y - ranges[t].x;
}
__global__ __launch_bounds__(1024) void lpt_hist_kernel(const uint2 *__restrict__ ranges,
                                                        const uint32_t *__restrict__ tile_last, int use_last, int T,
                                                        uint32_t *__restrict__ ghist) {
    __shared__ uint32_t hist[256];
    const int tid = threadIdx.x, lane = tid & 63;
    const uint64_t lt = lanemask_lt(lane);
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    constexpr int PER = LPT_WG_TILES / 1024;
    uint32_t b[PER];
    uint32_t wq[PER];  // weights loaded unconditionally (clamped tile): a load under `t < T` waited at its join
#pragma unroll
    for (int q = 0; q < PER; q++)
        wq[q] = lpt_weight(ranges, tile_last, use_last, min(blockIdx.x * LPT_WG_TILES + q * 1024 + tid, T - 1));
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int t = blockIdx.x * LPT_WG_TILES + q * 1024 + tid;
        b[q] = t < T ? lpt_log_bucket(wq[q]) : 0u;
    }
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int t = blockIdx.x * LPT_WG_TILES + q * 1024 + tid;
        lpt_item_b(t, b[q], t < T, hist, nullptr, lane, lt);
    }
    __syncthreads();
    if (tid < 256) ghist[blockIdx.x * 256 + tid] = hist[tid];
}
__global__ __launch_bounds__(1024) void lpt_scatter_kernel(const uint2 *__restrict__ ranges,
                                                           const uint32_t *__restrict__ tile_last, int use_last, int T,
                                                           const uint32_t *__restrict__ ghist,
                                                           uint32_t *__restrict__ order) {
    __shared__ uint32_t hist[256];
    const int tid = threadIdx.x, lane = tid & 63;
    const uint64_t lt = lanemask_lt(lane);
    constexpr int PER = LPT_WG_TILES / 1024;
    uint32_t b[PER];
    uint32_t wq[PER];  // weights loaded unconditionally (clamped tile): a load under `t < T` waited at its join
#pragma unroll
    for (int q = 0; q < PER; q++)
        wq[q] = lpt_weight(ranges, tile_last, use_last, min(blockIdx.x * LPT_WG_TILES + q * 1024 + tid, T - 1));
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int t = blockIdx.x * LPT_WG_TILES + q * 1024 + tid;
        b[q] = t < T ? lpt_log_bucket(wq[q]) : 0u;
    }
    if (tid < 64) {  // bucket bases: all workgroups' earlier buckets, plus this bucket in earlier workgroups
        // the workgroups' rows 8 at a time, one 16-B load each, all issued before any is used (a rolled loop waited
        // for every row in turn: one round trip per workgroup)
        uint32_t tot[4] = {0, 0, 0, 0}, pre[4] = {0, 0, 0, 0};
        const int G = (int)gridDim.x;
        for (int g0 = 0; g0 < G; g0 += 8) {
            uint4 v[8];
#pragma unroll
            for (int i = 0; i < 8; i++)
                v[i] = *reinterpret_cast<const uint4 *>(ghist + (size_t)min(g0 + i, G - 1) * 256 + 4 * tid);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int g = g0 + i;
                const uint32_t x[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t vv = g < G ? x[q] : 0u;
                    tot[q] += vv;
                    if (g < (int)blockIdx.x) pre[q] += vv;
                }
            }
        }
        const uint32_t sum = tot[0] + tot[1] + tot[2] + tot[3];
        uint32_t run = wave_inclusive_scan(sum, tid) - sum;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            hist[4 * tid + q] = run + pre[q];
            run += tot[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int t = blockIdx.x * LPT_WG_TILES + q * 1024 + tid;
        lpt_item_b(t, b[q], t < T, hist, order, lane, lt);
    }
}

void launch_tile_order(hipStream_t s, const uint2 *ranges, const uint32_t *tile_last, int use_last, int T,
                       uint32_t *order, uint32_t *scratch) {
    if (T <= 0) return;
    if (scratch && T > tuning("lpt_multi_tiles", 4096)) {  // cfg 3 (8160 tiles): step -12 us against one workgroup (14 us)
        const uint32_t g = div_up((uint32_t)T, (uint32_t)LPT_WG_TILES);
        lpt_hist_kernel<<<g, 1024, 0, s>>>(ranges, tile_last, use_last, T, scratch);
        lpt_scatter_kernel<<<g, 1024, 0, s>>>(ranges, tile_last, use_last, T, scratch, order);
        return;
    }
    tile_order_kernel<<<1, 1024, 0, s>>>(ranges, tile_last, use_last, T, tuning("lpt_shift", 3), order);
}

// ------------------------------------------------------------------------------------------------
// compositing (render_fwd_v6_kernel): one wave per 16x16 tile (or per row-strip part of one), NPIX pixels per
// lane (rows r, r+4, r+8, r+12 of the lane's column for whole tiles).  Each batch of 64 instances is gathered
// once per wave (one instance per lane) into the wave's LDS slice and then broadcast to all lanes.
// Front-to-back: alpha = min(0.99, o*exp(power)); skip alpha < 1/255; stop a pixel before the Gaussian that
// would take T below 1e-4.  No block barriers: the four waves of a block work on four independent tiles.
// The batch gather also materialises, for exactly the instances it loads, the sorted Gaussian id list
// (point_list) the backward walks and the inverse permutation inv[u] = s the backward's per-Gaussian gather reads
// (the binning filled it with INV_NONE: no row).  (Round 4 replaced inv by testing each row against a per-tile key of
// the last loaded instance in the backward: preprocess_bwd 0.094 -> 0.118 ms at cfg 3 for the row-tile search, for
// ~3 us of forward stores saved; measured and reverted, and round 5 removed the per-tile key.)
// Every piece of per-instance control is wave-uniform: the tile, its range and the contributor counter live
// in SGPRs, each batch's strip masks (cell_mask) are ballots (bit j = instance j can reach the strip), and the
// records of a batch sit in one LDS array of 48-byte entries read with immediate offsets.
// (Round 1-2 variants -- predicated v3, the composite_fwd split / part kernels and the negated-T v5 -- were
// bitwise identical and measured slower; DESIGN.md §4 keeps their numbers.)
// Pixel termination is kept off the per-pair path: a finished (or off-image) pixel gets a NaN row offset, so its
// exponent is NaN and the ordered `power2 <= 0` test already rejects it; the stop test's ballot guards a rare
// branch that retires the pixel and clears its lane from the strip's live mask (scalar), so a strip whose pixels
// have all finished is skipped like a dead cell, and the wave stops when no strip is live without any
// per-instance vector compare.
// CKPT (segmented backward, small images): at every ck_k-th instance of the tile the wave stores each pixel's T and
// colour / inverse-depth sums so far (checkpoint j before instance (j + 1) ck_k, at ckpt index ranges.x / ck_k + tile
// + j), and at the end the pixel's final sums (ctot); the backward walks each ck_k-instance segment from the
// checkpoint at its end.  A pixel still compositing at instance e is still walked when its wave reaches e, so every
// checkpoint the backward reads (e < the pixel's n_contrib) is written.
// SMASK (whole tiles): per batch, scalar masks cb[k] collect the instances some pixel of strip k took, and each loaded
// instance's 4-bit strip mask goes to strip_mask[s] -- the backward then walks exactly the strips that contributed
// instead of the conservative cell_mask (bitwise the same gradients: a skipped strip has no contributing pixel).
template <int NPIX, int MIN_WAVES, bool CKPT = false, bool GUARD = false, bool SMASK = false>
__global__ __launch_bounds__(256, MIN_WAVES) void render_fwd_v6_kernel(RenderFwdParams p) {
    constexpr int PARTS = 4 / NPIX;
    static_assert(!SMASK || PARTS == 1, "strip masks are recorded by whole-tile waves");
    __shared__ FwdRec s_rec[4][64];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int slot = blockIdx.x * 4 + w;
    if (p.ck_flag && slot == 0 && lane == 0) *p.ck_flag = CKPT ? p.ck_k : 0u;
    if (p.lpt_valid && slot == 0 && lane == 0)
        *p.lpt_valid = (PARTS == 1 && p.lpt_blist) ? (p.xcd ? LPT_LISTS_XCD : LPT_LISTS) : 0u;
    if (p.smask_valid && slot == 0 && lane == 0) *p.smask_valid = SMASK ? 1u : 0u;
    int tile;
    if (PARTS == 1 && p.xcd) {  // per-XCD LPT slot map (xcd_slots(T) slots)
        tile = __builtin_amdgcn_readfirstlane((int)p.tile_order[slot]);
        if (tile < 0) return;  // XCD_NONE
    } else {
        if (slot >= p.num_tiles * PARTS) return;
        tile = __builtin_amdgcn_readfirstlane(p.tile_order ? (int)p.tile_order[slot / PARTS] : slot / PARTS);
    }
    const int half = slot % PARTS;
    const uint32_t t_start = p.stamps ? stamp_now() : 0u;
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int px = tx * BLOCK_X + (lane & 15);
    const int py0 = ty * BLOCK_Y + (lane >> 4);
    const float pfx = (float)px, pfy0 = (float)py0;
    const float row0 = (float)(ty * BLOCK_Y), col0 = (float)(tx * BLOCK_X);
    const int kbase = NPIX * half;  // whole-tile pixel index of this wave's first pixel
    float T[NPIX], C0[NPIX], C1[NPIX], C2[NPIX], ID[NPIX], off[NPIX];
    uint32_t last[NPIX];
    uint64_t livek[NPIX];  // lanes whose pixel k still composites (wave-uniform)
#pragma unroll
    for (int k = 0; k < NPIX; k++) {
        const int py = py0 + 4 * (kbase + k);
        const bool inside = px < p.W && py < p.H;
        off[k] = inside ? (float)py : __builtin_nanf("");  // the pixel's row (exact); NaN retires the pixel
        livek[k] = __ballot(inside);
        T[k] = 1.0f;
        C0[k] = C1[k] = C2[k] = ID[k] = 0.f;
        last[k] = 0;
    }
    const uint2 rg = p.ranges[tile];
    const uint32_t r0 = __builtin_amdgcn_readfirstlane(rg.x), r1 = __builtin_amdgcn_readfirstlane(rg.y);
    uint32_t contributor = 0;
    uint32_t loaded_end = r0;
    FwdRec *sr = s_rec[w];
    // checkpoint before tile-relative instance e (a multiple of ck_k)
    auto store_ck = [&](uint32_t e) {
        float *ck = p.ckpt + (size_t)(r0 / p.ck_k + (uint32_t)tile + e / p.ck_k - 1) * CK_FLOATS;
#pragma unroll
        for (int k = 0; k < NPIX; k++) {
            const int i = lane + 64 * (kbase + k);  // pixel within the tile
            ck[i] = T[k];
            ck[256 + i] = C0[k];
            ck[512 + i] = C1[k];
            ck[768 + i] = C2[k];
            ck[1024 + i] = ID[k];
        }
    };
    for (uint32_t base = r0; base < r1; base += 64) {
        if (CKPT && base > r0 && (base - r0) % p.ck_k == 0) store_ck(base - r0);
        const uint32_t s = base + lane;
        uint32_t m = 0;
        if (s < r1) {
            const uint32_t u = p.sorted_u[s];
            const uint32_t gid = p.inst_gid[u];
            p.point_list[s] = gid;
            p.inv[u] = s;
            const float4 ga = p.rec[gid].a, gb = p.rec[gid].b;
            sr[lane].a = stage_rec_a(ga);
            sr[lane].b = stage_rec_b(gb);
            sr[lane].c = p.rec[gid].c;
            if (GUARD) sr[lane].pad.x = __uint_as_float(gid);  // the guard's slow path reloads the raw record
            m = cell_mask(p.strip_exact, ga, gb, row0, col0) >> kbase;
        }
        uint64_t sk[NPIX];
#pragma unroll
        for (int k = 0; k < NPIX; k++) sk[k] = livek[k] ? __ballot((m >> k) & 1u) : 0ull;  // finished strips: none
        loaded_end = min(r1, base + 64u);
        wave_lds_sync();
        // walk only the batch's instances that reach a live strip (in order): instances whose strips are all
        // unreachable or finished cost nothing
        uint64_t un = 0;
#pragma unroll
        for (int k = 0; k < NPIX; k++) un |= sk[k];
        const uint32_t cbase = contributor;
        uint64_t cb[NPIX];  // SMASK: bit j of cb[k] = some pixel of strip k took instance j
#pragma unroll
        for (int k = 0; k < NPIX; k++) cb[k] = 0;
        auto walk = [&](uint64_t &un) {
        while (un) {
            const uint32_t j = (uint32_t)__builtin_ctzll(un);
            const uint64_t bit = 1ull << j;
            un &= ~bit;  // one s_andn2_b64 with the bit the strip tests need anyway (un & (un - 1) costs three SALU)
            const float4 a = sr[j].a, b = sr[j].b;
            const float2 c = sr[j].c;
            contributor = cbase + j + 1;
            const float dx = a.x - pfx;
            const float P0 = (a.z * dx) * dx, L = a.w * dx;
#pragma unroll
            for (int k = 0; k < NPIX; k++) {
                if (!(sk[k] & bit)) continue;  // wave-uniform
                // dy = y - pixel row in one subtraction (the reference's own form): no per-instance row offset
                const float power2 = power2_at(b.x, a.y - off[k], P0, L);
                const float alpha = fminf(0.99f, b.y * __builtin_amdgcn_exp2f(power2));
                const float test_T = T[k] * (1 - alpha);
                // lane masks straight from the compares (scalar registers): ok = power2 <= 0 (ordered, so false
                // for a retired pixel's NaN exponent; power2 is never NaN otherwise) and !(alpha < 1/255)
                // GUARD: the alpha test at the band's lower edge, then the pairs inside the band re-decided (one
                // extra compare per pair: outside the band alpha >= A_LO <=> alpha >= 1/255)
                uint64_t ok = __builtin_amdgcn_fcmpf(power2, 0.0f, FCMP_OLE) &
                              __builtin_amdgcn_fcmpf(alpha, GUARD ? GUARD_A_LO : 1.0f / 255.0f, FCMP_UGE);
                const uint64_t low = __builtin_amdgcn_fcmpf(test_T, 0.0001f, FCMP_OLT);
                if constexpr (GUARD) {  // alpha decisions near 1/255 from the oracle's arithmetic (gsr_common.h)
                    const uint64_t near = ok & ~__builtin_amdgcn_fcmpf(alpha, GUARD_A_HI, FCMP_UGE);
                    if (__builtin_expect(near != 0, 0)) {  // rare
                        const uint32_t g = __float_as_uint(sr[j].pad.x);
                        const uint64_t okx = __ballot(
                            guard_alpha_pass(p.rec, g, pfx, pfy0 + (float)(4 * (kbase + k))));
                        ok = (ok & ~near) | (okx & near);
                    }
                }
                uint64_t take;
                if constexpr (SMASK) {  // cb[k] |= bit when take != 0: a select on the flag the s_andn2 forming take
                                        // sets (the compiler re-tests take and selects both halves: 4 SALU, not 2)
                    const uint64_t cbt = cb[k] | bit;
                    asm("s_andn2_b64 %0, %2, %3\n\ts_cselect_b64 %1, %4, %1"
                        : "=&s"(take), "+s"(cb[k]) : "s"(ok), "s"(low), "s"(cbt) : "scc");
                } else {
                    take = ok & ~low;
                }
                const uint64_t stop = ok & low;
                const float wgt = select_mask(take, alpha * T[k], 0.f);
                C0[k] = fmaf(b.z, wgt, C0[k]);
                C1[k] = fmaf(b.w, wgt, C1[k]);
                C2[k] = fmaf(c.x, wgt, C2[k]);
                ID[k] = fmaf(c.y, wgt, ID[k]);
                T[k] = select_mask(take, test_T, T[k]);
                last[k] = __float_as_uint(select_mask(take, __uint_as_float(contributor), __uint_as_float(last[k])));
                if (stop) {  // rare: some pixels of the strip reach T < 1e-4 and retire
                    off[k] = select_mask(stop, __builtin_nanf(""), off[k]);
                    livek[k] &= ~stop;
                    if (livek[k] == 0) {  // the whole strip finished: skip it for the rest of the batch
                        sk[k] = 0;
                        uint64_t live = 0;
#pragma unroll
                        for (int q = 0; q < NPIX; q++) live |= sk[q];
                        un &= live;  // every pixel of the wave finished: un = 0 ends the walk
                    }
                }
            }
        }
        };
        if (CKPT && p.ck_k == 32 && base + 32 < r1) {  // 32-instance checkpoints: one in the middle of the batch
            uint64_t lo = un & 0xffffffffull;
            walk(lo);
            store_ck(base + 32 - r0);
            uint64_t live = 0;
#pragma unroll
            for (int k = 0; k < NPIX; k++) live |= sk[k];
            uint64_t hi = un & live & ~0xffffffffull;
            walk(hi);
        } else {
            walk(un);
        }
        contributor = cbase + min(64u, r1 - base);
        if (SMASK && s < r1) {
            uint32_t mk = 0;
#pragma unroll
            for (int k = 0; k < NPIX; k++) mk |= (uint32_t)((cb[k] >> lane) & 1ull) << k;
            p.strip_mask[s] = (uint8_t)mk;
        }
        wave_lds_sync();
        uint64_t anylive = 0;
#pragma unroll
        for (int k = 0; k < NPIX; k++) anylive |= livek[k];
        if (anylive == 0) break;
    }
    const float bg0 = p.bg[0], bg1 = p.bg[1], bg2 = p.bg[2];
    const size_t HW = (size_t)p.W * p.H;
    uint32_t mx = 0;
    // the pixel column and row re-derived from the lane id (mbcnt, not threadIdx, so the compiler does not keep the
    // integer column live across the walk just to reuse it here: it re-materialised the float column from it instead,
    // one conversion per instance)
    const int lid = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const int pxe = tx * BLOCK_X + (lid & 15), py0e = ty * BLOCK_Y + (lid >> 4);
#pragma unroll
    for (int k = 0; k < NPIX; k++) {
        const int py = py0e + 4 * (kbase + k), px = pxe;
        if (px < p.W && py < p.H) {
            const size_t pid = (size_t)py * p.W + px;
            const float Tk = T[k];
            p.final_T[pid] = Tk;
            p.n_contrib[pid] = last[k];
            p.out_color[pid] = C0[k] + Tk * bg0;
            p.out_color[HW + pid] = C1[k] + Tk * bg1;
            p.out_color[2 * HW + pid] = C2[k] + Tk * bg2;
            if (p.out_invdepth) p.out_invdepth[pid] = ID[k];
            mx = max(mx, last[k]);
        }
        if (CKPT) {
            float *ct = p.ctot + (size_t)tile * 1024 + lane + 64 * (kbase + k);
            ct[0] = C0[k];
            ct[256] = C1[k];
            ct[512] = C2[k];
            ct[768] = ID[k];
        }
    }
    mx = wave_max_u32(mx);
    if (lane == 0) {
        atomicMax(&p.tile_last[tile], mx);
        atomicMax(&p.tile_loaded[tile], loaded_end - r0);
        if (PARTS == 1 && p.lpt_blist) {  // whole tile: mx is final; append it to its backward LPT bucket
            uint32_t b = lpt_log_bucket(mx), stride = (uint32_t)p.num_tiles;
            if (p.xcd) {  // the bucket of its XCD group (lpt_list_tile_xcd)
                b += 256u * xcd_group_of((uint32_t)tile, (uint32_t)p.gx, (uint32_t)p.gy);
                stride = xcd_slots((uint32_t)p.num_tiles) / LPT_XCD;
            }
            const uint32_t pos = atomicAdd(&p.lpt_bcnt[b], 1u);
            p.lpt_blist[(size_t)b * stride + pos] = (uint32_t)tile;
        }
    }
    stamp_store(p.stamps, slot, t_start, lane);
}

// "fwd_parts" 1, 2 or 4; 0 (default): 4 when that many part-waves still fit the GPU's ~8 resident waves per SIMD,
// twice over (small images, where one heavy tile's latency sets the kernel time), else whole tiles (measured at
// 1080p, 8160 tiles: whole tiles 0.175 ms against 0.196 in 2 parts; at 800x800, 2500 tiles: 4 parts 0.073, 2 parts
// 0.092, whole 0.126)
int render_fwd_parts(int num_tiles) {
    int parts = tuning("fwd_parts", 0);
    if (parts == 0) parts = num_tiles * 4 <= tuning("fwd_part_slots", 16384) ? 4 : 1;
    return (parts == 2 || parts == 4) ? parts : 1;
}

void launch_render_fwd(hipStream_t s, const RenderFwdParams &p0) {
    if (p0.num_tiles <= 0) return;
    RenderFwdParams p = p0;
    p.strip_exact = tuning("strip_exact", 1);
    p.stamps = tuning("stamp", 0) ? stamp_buffer(0) : nullptr;
    const int parts = render_fwd_parts(p.num_tiles);
    if (parts != 1) p.xcd = 0;
    const dim3 grid(div_up(p.xcd ? (uint64_t)xcd_slots((uint32_t)p.num_tiles) : (uint64_t)p.num_tiles * parts, 4)),
        block(256);
    // threshold guard band ("guard" 1; the default launch shapes only, and the backward must run with the same knob)
    // exact strip masks for the backward ("smask" 1): whole tiles only
    const bool sm = parts == 1 && p.strip_mask && tuning("smask", 1);
    if (!sm) p.strip_mask = nullptr;
    if (tuning("guard", 0)) {  // 6 waves per SIMD whole-tile: the guard's double exp needs the registers
        if (parts == 1 && sm) render_fwd_v6_kernel<4, 6, false, true, true><<<grid, block, 0, s>>>(p);
        else if (parts == 1) render_fwd_v6_kernel<4, 6, false, true><<<grid, block, 0, s>>>(p);
        else if (parts == 4 && p.ckpt && p.ctot && p.ck_k >= CK_MIN_K && p.ck_k % 32 == 0 &&
                 (p.ck_k == 32 || p.ck_k % 64 == 0))
            render_fwd_v6_kernel<1, 8, true, true><<<grid, block, 0, s>>>(p);
        else if (parts == 2) render_fwd_v6_kernel<2, 8, false, true><<<grid, block, 0, s>>>(p);
        else render_fwd_v6_kernel<1, 8, false, true><<<grid, block, 0, s>>>(p);
        return;
    }
    if (parts == 1) {
        // 8 waves per SIMD (64 VGPRs, one 8-byte spill outside the pair loop): cfg3 0.180 -> 0.172 ms, cfg5 0.517 ->
        // 0.478 ms against 6 waves (65 VGPRs, i.e. 7 resident)
        const int mw = tuning("fwd_whole_waves", 8);
        if (sm) render_fwd_v6_kernel<4, 8, false, false, true><<<grid, block, 0, s>>>(p);
        else if (mw >= 8) render_fwd_v6_kernel<4, 8><<<grid, block, 0, s>>>(p);
        else if (mw >= 6) render_fwd_v6_kernel<4, 6><<<grid, block, 0, s>>>(p);
        else render_fwd_v6_kernel<4, 4><<<grid, block, 0, s>>>(p);
        return;
    }
    const int mw = tuning("fwd_part_waves", 8);
    if (parts == 4 && p.ckpt && p.ctot && p.ck_k >= CK_MIN_K && p.ck_k % 32 == 0 && (p.ck_k == 32 || p.ck_k % 64 == 0))
        render_fwd_v6_kernel<1, 8, true><<<grid, block, 0, s>>>(p);
    else if (parts == 2 && mw >= 8) render_fwd_v6_kernel<2, 8><<<grid, block, 0, s>>>(p);
    else if (parts == 2) render_fwd_v6_kernel<2, 4><<<grid, block, 0, s>>>(p);
    else if (mw >= 8) render_fwd_v6_kernel<1, 8><<<grid, block, 0, s>>>(p);
    else render_fwd_v6_kernel<1, 4><<<grid, block, 0, s>>>(p);
}

// ------------------------------------------------------------------------------------------------
// markVisible (checkFrustum): z_view > 0.2
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mark_visible_kernel(int P, const float *__restrict__ means3D,
                                                           const float *__restrict__ view,
                                                           uint8_t *__restrict__ present) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const Mat4 v = load_mat4(view);
    present[i] = xform3(load_f3(means3D, i), v).z > 0.2f ? 1 : 0;
}

void launch_mark_visible(hipStream_t s, int P, const float *means3D, const float *view, uint8_t *present) {
    if (P <= 0) return;
    mark_visible_kernel<<<div_up(P, 256), 256, 0, s>>>(P, means3D, view, present);
}

}  // namespace gsr
