// gsr_backward.hip -- backward kernels: reverse-walk compositing gradient, per-Gaussian reduction,
// and the preprocess backward (2D conic -> cov2D -> cov3D -> scale/rotation, 2D mean -> 3D mean,
// SH -> colour).
//
// The upstream CUDA backward scatters every (pixel, Gaussian) contribution with ~10 global float
// atomics (SURVEY.md §2.1 BACKWARD::render).  Here one wave owns one tile: each lane walks 4 pixels
// in reverse, the wave sums the per-instance contributions with DPP reductions, and writes ONE 40-byte
// gradient row per (tile, Gaussian) instance, contiguously in sorted order.  The per-Gaussian kernel
// then gathers its rows through the inverse permutation.  No float atomics, so gradients are
// bitwise reproducible run to run.
#include "gsr_kernels.h"
#include "gsr_sh.h"

namespace gsr {

// ------------------------------------------------------------------------------------------------
// Moment accumulation + transposing reduction.
//   Per active (pixel, instance) pair a lane accumulates q = G * dL/dalpha and the moments q, q dx, q dy,
//   q dx^2, q dx dy, q dy^2 (plus the colour / inverse-depth weights).  Since dL/dG = o dL/dalpha and
//   dG/ddelta = -G (conic . delta), every conic / mean / opacity gradient term of the reference is a
//   uniform combination of these moments, applied once per instance after the reduction:
//     dopacity = S,  dconic = -o/2 (Sxx, Sxy, Syy),  dmean2D = -o (W/2, H/2) * (a Sx + b Sy, b Sx + c Sy).
//   The per-lane sums of two instances are reduced across the wave together by a transposing permlane/DPP
//   reduction (wave_reduce_pair_store) into LDS; after each batch of 32 instances lane j reads the 10 totals of
//   instance j, applies the uniform conversion and stores the gradient row.
//   One scalar "behind" accumulator per pixel carries the background: the reference keeps accum_rec (3 channels)
//   and accum_invdepth per pixel and adds -T_final / (1 - alpha) (bg . dL/dpix) to dL/dalpha.  Only the projection
//   onto the pixel's upstream gradient enters dL/dalpha, so one scalar D_k = (accum_rec_k + T_final / T_{k+1} bg)
//   . dL/dpix + accum_invdepth_k dL/dinvdepth carries all of it: at the last contributor D = bg . dL/dpix, it
//   follows the reference's recursion D <- D + alpha (c . dL/dpix - D), and dL/dalpha = T_k (c . dL/dpix - D).
//   (Round 1-2 variants -- per-channel accumulators v3, the branch / predication forms of v4 and the scalar-mask
//   v6 -- were bitwise identical or equal to rounding and measured slower; DESIGN.md §4 keeps their numbers.)
// ------------------------------------------------------------------------------------------------
// Zero fill of the per-Gaussian backward outputs (RenderBwdParams::zf_*), this workgroup's share of the virtual
// array, as non-temporal stores that drain while the other waves' VALU-bound walks run, so the HBM-bound preprocess
// backward after it stores only the Gaussians whose gradient is not identically zero ...
typedef unsigned int zf_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bwd_zero_fill(const RenderBwdParams &p) {
    if (p.zf_total16 == 0 && p.zf_nodd == 0) return;  // uniform
    const uint64_t nb = gridDim.x, b = blockIdx.x;
    const uint64_t per = (p.zf_total16 + nb - 1) / nb;
    const uint64_t lo = b * per, hi = min(p.zf_total16, lo + per);
    const zf_u4 z = {0u, 0u, 0u, 0u};
    for (uint32_t sg = 0; sg < p.zf_nseg; sg++) {
        const uint64_t s0 = p.zf_pre16[sg], s1 = p.zf_pre16[sg + 1];
        const uint64_t e = min(hi, s1);
        zf_u4 *base = reinterpret_cast<zf_u4 *>(p.zf_ptr[sg]) - s0;
        for (uint64_t k = max(lo, s0) + threadIdx.x; k < e; k += blockDim.x) __builtin_nontemporal_store(z, base + k);
    }
    if (b == 0 && threadIdx.x < p.zf_nodd) *p.zf_odd[threadIdx.x] = 0u;
}
// ... issued when the workgroup's walk is done (every return path): issued first, the walk's first load wait (vmcnt
// counts stores too) held each wave until its zero stores had landed
struct ZeroFillAtExit {
    const RenderBwdParams &p;
    __device__ ~ZeroFillAtExit() { bwd_zero_fill(p); }
};

constexpr int BWD_BATCH = 32;
constexpr int PART = 12;  // floats per instance in the LDS partial buffer (10 sums + 2 pad)

// x + y after v_permlane32_swap(x, y): lanes 0-31 hold x[l] + x[l+32], lanes 32-63 hold y[l-32] + y[l]
// (lane mapping measured on MI355X by tools/probes/permlane_probe.hip).
__device__ __forceinline__ float sum_swap32(float x, float y) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// x + y after v_permlane16_swap(x, y): even rows hold x summed over the row pair, odd rows hold y.
__device__ __forceinline__ float sum_swap16(float x, float y) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ constexpr float kZero8[8] = {0, 0, 0, 0, 0, 0, 0, 0};

// Two instances: the bit-5 exchange pairs each raw sum of instance 0 with the same sum of instance 1 (7 swaps, not
// the 10 of two moment sets), so every register then holds one quantity (instance b5's) and the moments are formed
// once for both instances, on sums already reduced over lane bit 5, with the lane's dx of its instance.  The
// remaining levels are wave_reduce20_store's: after the bit-4 swaps bb[k] holds value 2 k + b4, the bit-3 exchange
// makes value 4 m + 2 b3 + b4 (m = 0, 1) and 8 + b4; values are in gradient-row order
// (S, Sx, Sy, Sxx, Sxy, Syy, w0..w3) of instance b5 (the next PART-float row for instance 1).
// BOTH = false reduces instance 0 alone through the same operation tree (r1 all zero, only its row stored), so an
// instance's gradient bits do not depend on whether it was paired.
template <bool BOTH = true>
__device__ __forceinline__ void wave_reduce_pair_store(const float r0[8], const float r1[8], float *__restrict__ dst,
                                                       int lane, float *__restrict__ dst1 = nullptr) {
    const bool hi5 = (lane & 32) != 0;
    const float dx = hi5 ? r1[7] : r0[7];
    const float s0 = sum_swap32(r0[0], r1[0]), s1 = sum_swap32(r0[1], r1[1]), s2 = sum_swap32(r0[2], r1[2]);
    float R[10];
    R[0] = s0;
    R[1] = s0 * dx;
    R[2] = s1;
    R[3] = R[1] * dx;
    R[4] = s1 * dx;
    R[5] = s2;
#pragma unroll
    for (int i = 0; i < 4; i++) R[6 + i] = sum_swap32(r0[3 + i], r1[3 + i]);
    float bb[5];
#pragma unroll
    for (int k = 0; k < 5; k++) bb[k] = sum_swap16(R[2 * k], R[2 * k + 1]);
    const bool hi3 = (lane & 8) != 0;
    float c[3];
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const float keep = hi3 ? bb[2 * m + 1] : bb[2 * m], send = hi3 ? bb[2 * m] : bb[2 * m + 1];
        c[m] = dpp_xadd<0x128>(keep, send);
    }
    c[2] = dpp_add<0x128>(bb[4]);  // row_ror:8 (= lane ^ 8)
#pragma unroll
    for (int m = 0; m < 3; m++) {
        c[m] = dpp_add<0xB1>(c[m]);   // quad_perm [1,0,3,2]
        c[m] = dpp_add<0x4E>(c[m]);   // quad_perm [2,3,0,1]
        c[m] = dpp_add<0x141>(c[m]);  // row_half_mirror
        // materialise the sums in every lane: otherwise the last add sinks into the masked store blocks and the
        // row_half_mirror step costs a v_mov_b32_dpp plus a v_add instead of one v_add_f32_dpp
        asm volatile("" : "+v"(c[m]));
    }
    float *row = hi5 ? (dst1 ? dst1 : dst + PART) : dst;  // instance 1's row: dst1, or the next PART-float row
    const int low = ((lane >> 2) & 2) | ((lane >> 4) & 1);  // 2 b3 + b4
    if (!BOTH && hi5) return;
    if ((lane & 7) == 0) {
        row[low] = c[0];
        row[4 + low] = c[1];
    }
    if ((lane & 15) == 0) row[8 + (low & 1)] = c[2];
}

// Parts variant for small images: PARTS waves of one workgroup share one tile, wave w compositing the lane's
// pixels of row strips [w NP, w NP + NP) (NP = 4 / PARTS).  With few tiles (800x800: 2500 tiles for 1024
// SIMDs) one heavy tile's serial walk sets the kernel time; splitting its pixels shortens that walk.  Per batch
// of BWD_BATCH instances: wave 0 stages the records, every wave reduces its own per-instance sums into its
// s_part plane, and after a barrier wave 0 adds the planes in part order and writes the gradient row.  The
// per-instance reductions are repeated PARTS times, so it pays only where latency, not issue, is the limit.
template <bool HAS_INV, int PARTS>
__global__ __launch_bounds__(64 * PARTS) void render_bwd_parts_kernel(RenderBwdParams p) {
    constexpr int NP = PIX_PER_LANE / PARTS;
    __shared__ float4 s_a[BWD_BATCH];
    __shared__ float4 s_b[BWD_BATCH];
    __shared__ float2 s_c[BWD_BATCH];
    __shared__ uint32_t s_m[BWD_BATCH];
    __shared__ __attribute__((aligned(16))) float s_part[PARTS][BWD_BATCH][PART];
    const ZeroFillAtExit zero_fill_at_exit{p};
    if (p.live_valid && blockIdx.x == 0 && threadIdx.x == 0) *p.live_valid = p.live ? 1u : 0u;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int slot = blockIdx.x;
    const int tile = p.tile_order ? (int)p.tile_order[slot] : slot;
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int px = tx * BLOCK_X + (lane & 15);
    const int py0 = ty * BLOCK_Y + (lane >> 4);
    const float pfx = (float)px;
    const float row0 = (float)(ty * BLOCK_Y);
    const uint2 range = p.ranges[tile];
    const uint32_t tl = p.tile_last[tile];
    const uint32_t loaded = p.tile_loaded[tile];
    for (uint32_t s = range.x + tl + threadIdx.x; s < range.x + loaded; s += 64 * PARTS) {
        const float z[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        store_row(p.rows, p.sorted_u[s], z);
    }
    if (tl == 0) return;  // workgroup-uniform

    const int kbase = w * NP;
    const float bg0 = p.bg[0], bg1 = p.bg[1], bg2 = p.bg[2];
    const size_t HW = (size_t)p.W * p.H;
    float T[NP], dp0[NP], dp1[NP], dp2[NP], dinv[NP], D[NP], prow[NP];
    uint32_t lastc[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) prow[k] = (float)(py0 + 4 * (kbase + k));  // pixel rows (dy = y - row, as the forward)
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const int py = py0 + 4 * (kbase + k);
        const bool inside = px < p.W && py < p.H;
        const size_t pid = inside ? (size_t)py * p.W + px : 0;
        T[k] = inside ? p.final_T[pid] : 0.f;
        lastc[k] = inside ? p.n_contrib[pid] : 0u;
        dp0[k] = inside ? p.dL_dpix[pid] : 0.f;
        dp1[k] = inside ? p.dL_dpix[HW + pid] : 0.f;
        dp2[k] = inside ? p.dL_dpix[2 * HW + pid] : 0.f;
        dinv[k] = (HAS_INV && inside) ? p.dL_dinvdepth[pid] : 0.f;
        D[k] = fmaf(bg2, dp2[k], fmaf(bg1, dp1[k], bg0 * dp0[k]));
    }
    const float hW = 0.5f * p.W, hH = 0.5f * p.H;

    for (int bend = (int)tl; bend > 0; bend -= BWD_BATCH) {
        const int cnt = min(BWD_BATCH, bend);
        float4 my_a = make_float4(0, 0, 0, 0), my_b = my_a;
        uint32_t my_row = 0, my_gid = 0;
        if (w == 0 && lane < cnt) {
            const uint32_t s_me = range.x + (uint32_t)(bend - 1 - lane);
            my_row = p.sorted_u[s_me];
            const uint32_t gid = p.point_list[s_me];
            my_gid = gid;
            my_a = p.rec[gid].a;
            my_b = p.rec[gid].b;
            s_a[lane] = stage_rec_a(my_a);
            s_b[lane] = stage_rec_b(my_b);
            s_c[lane] = p.rec[gid].c;
            s_m[lane] = cell_mask(p.strip_exact, my_a, my_b, row0, (float)(tx * BLOCK_X));
        }
        __syncthreads();
        // strip k of instance j is live iff bit j of sk[k] (wave-uniform)
        const uint32_t mm = lane < cnt ? s_m[lane] : 0u;
        uint64_t sk[NP];
#pragma unroll
        for (int k = 0; k < NP; k++) sk[k] = __ballot((mm >> (kbase + k)) & 1u);
        auto pass = [&](const int j, float m[8]) -> bool {
            const uint32_t idx = (uint32_t)(bend - 1 - j);
            const float4 a = s_a[j], b = s_b[j];  // a: x, y, A, B; b: C, o, r, g
            const float2 c = s_c[j];              // b, 1/depth
            const float dx = a.x - pfx;
            const float P0 = (a.z * dx) * dx, L = a.w * dx;
            float Q0 = 0.f, Q1 = 0.f, Q2 = 0.f, w0 = 0.f, w1 = 0.f, w2 = 0.f, w3 = 0.f;
            bool any = false;
#pragma unroll
            for (int k = 0; k < NP; k++) {
                if (!((sk[k] >> j) & 1u)) continue;  // wave-uniform
                const float dy = a.y - prow[k];
                const float power2 = power2_at(b.x, dy, P0, L);
                const float G = __builtin_amdgcn_exp2f(power2);
                const float alpha = fminf(0.99f, b.y * G);
                if (!(idx < lastc[k] && !(power2 > 0.0f) && !(alpha < 1.0f / 255.0f))) continue;
                any = true;
                T[k] = T[k] * fast_rcp(1.f - alpha);
                const float wgt = alpha * T[k];
                float cd = fmaf(c.x, dp2[k], fmaf(b.w, dp1[k], b.z * dp0[k]));
                if (HAS_INV) cd = fmaf(c.y, dinv[k], cd);
                const float d = cd - D[k];
                D[k] = fmaf(alpha, d, D[k]);
                w0 = fmaf(wgt, dp0[k], w0);
                w1 = fmaf(wgt, dp1[k], w1);
                w2 = fmaf(wgt, dp2[k], w2);
                if (HAS_INV) w3 = fmaf(wgt, dinv[k], w3);
                const float q = G * (d * T[k]);
                const float qdy = q * dy;
                Q0 += q;
                Q1 += qdy;
                Q2 = fmaf(qdy, dy, Q2);
            }
            m[0] = Q0;
            m[1] = Q1;
            m[2] = Q2;
            m[3] = w0;
            m[4] = w1;
            m[5] = w2;
            m[6] = w3;
            m[7] = dx;
            return any;
        };
        for (int j = 0; j < cnt; j += 2) {
            float m0[8];
            const bool any0 = pass(j, m0);
            float *dst = s_part[w][j];
            if (j + 1 < cnt) {
                float m1[8];
                const bool any1 = pass(j + 1, m1);
                if (__ballot(any0 || any1)) {
                    wave_reduce_pair_store(m0, m1, dst, lane);
                } else if (lane < 10) {
                    dst[lane] = 0.f;
                    dst[PART + lane] = 0.f;
                }
            } else if (__ballot(any0)) {
                wave_reduce_pair_store<false>(m0, kZero8, dst, lane);
            } else if (lane < 10) {
                dst[lane] = 0.f;
            }
        }
        __syncthreads();
        if (w == 0 && lane < cnt) {
            float u[10];
#pragma unroll
            for (int v = 0; v < 10; v++) u[v] = s_part[0][lane][v];
#pragma unroll
            for (int q = 1; q < PARTS; q++)
#pragma unroll
                for (int v = 0; v < 10; v++) u[v] += s_part[q][lane][v];
            const float o = my_b.y, ca = my_a.z, cb = my_a.w, cc = my_b.x;
            float row[10];
            row[0] = -o * hW * (ca * u[1] + cb * u[2]);
            row[1] = -o * hH * (cb * u[1] + cc * u[2]);
            row[2] = -0.5f * o * u[3];
            row[3] = -0.5f * o * u[4];
            row[4] = -0.5f * o * u[5];
            row[5] = u[0];
            row[6] = u[6];
            row[7] = u[7];
            row[8] = u[8];
            row[9] = u[9];
            store_row(p.rows, my_row, row);
            if (p.live && row_nonzero(row)) p.live[my_gid] = 1;
        }
        __syncthreads();  // the next batch overwrites the staged records and the sums
    }
}

// render_bwd_v5_kernel: one wave per tile, the pair-reduced update with the per-instance control on the scalar unit.
//   render_bwd is VALU-issue-bound (SQ_INSTS_VALU x issue cost ~ 85 % of its cycles at cfg 3), so every saved
//   vector instruction counts: the strips an instance cannot reach are skipped by scalar bit tests (the forward's
//   exact strip masks), the contributing lanes come straight from compares as scalar masks, and the staged records
//   are one 48-byte FwdRec array.
#ifndef GSR_BWD_MINW
#define GSR_BWD_MINW 5
#endif
#ifndef GSR_BWD_SEG_MINW
#define GSR_BWD_SEG_MINW 6  // the segment walk's extra scalars took it to 83 VGPRs (5 waves / SIMD); 6 caps it at 80
#endif
// SEG (small images): the launch slot is a (tile, segment) work item of seg_list; with the forward's checkpoints
// (*ck_flag = K) segment s walks instances [s K, min((s + 1) K, tile_last)) back to front, starting each pixel from the
// checkpoint at the segment's end: T = T_e and D = (colour still to come . dL/dpix + T_final bg . dL/dpix) / T_e, the
// scalar accumulator's value there (D_k T_(k+1) = sum_(j > k) w_j c_j . dL/dpix + T_final bg . dL/dpix).  Without
// checkpoints every tile is one segment.  Rows agree with the one-walk backward to rounding.
template <bool HAS_INV, bool UNION = false, bool SEG = false, bool GUARD = false>
__global__ __launch_bounds__(64, GUARD ? 4 : SEG ? GSR_BWD_SEG_MINW : GSR_BWD_MINW) void render_bwd_v5_kernel(RenderBwdParams p) {
    __shared__ FwdRec s_rec[BWD_BATCH];
    __shared__ __attribute__((aligned(16))) float s_part[BWD_BATCH][PART];  // [instance][10 sums]
    // zeros the union walk's per-instance accumulators are loaded from (pass() below); one pair per batch slot, so the
    // loads are loop-variant and stay in the loop rather than being hoisted into registers copied per instance
    __shared__ float4 s_zero[UNION ? BWD_BATCH : 1][2];
    if constexpr (UNION) {
        if (threadIdx.x < 2 * BWD_BATCH) (&s_zero[0][0])[threadIdx.x] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const ZeroFillAtExit zero_fill_at_exit{p};
    if (p.live_valid && blockIdx.x == 0 && threadIdx.x == 0) *p.live_valid = p.live ? 1u : 0u;
    const int lane = threadIdx.x;
    const int slot = blockIdx.x;
    const uint32_t t_start = p.stamps ? stamp_now() : 0u;
    uint32_t seg = 0, ck_k = 0;
    int tile;
    if constexpr (SEG) {
        if ((uint32_t)slot >= __builtin_amdgcn_readfirstlane(*p.seg_count)) return;
        const uint2 item = p.seg_list[slot];
        tile = __builtin_amdgcn_readfirstlane((int)item.x);
        seg = __builtin_amdgcn_readfirstlane(item.y);
        ck_k = __builtin_amdgcn_readfirstlane(*p.ck_flag);
    } else {
        // the forward's bucket lists (per XCD group: xcd_slots(T) launch slots, lpt_list_tile_xcd), else the order
        const uint32_t lists = p.lpt_blist ? __builtin_amdgcn_readfirstlane(*p.lpt_valid) : 0u;
        if (lists == LPT_LISTS_XCD) {
            tile = lpt_list_tile_xcd(p.lpt_bcnt, p.lpt_blist, (uint32_t)p.num_tiles, (uint32_t)slot, lane);
        } else if (slot >= p.num_tiles) {
            tile = -1;
        } else if (lists == LPT_LISTS) {
            tile = lpt_list_tile(p.lpt_bcnt, p.lpt_blist, (uint32_t)p.num_tiles, (uint32_t)slot, lane, slot);
        } else {
            tile = __builtin_amdgcn_readfirstlane(p.tile_order ? (int)p.tile_order[slot] : slot);
        }
        if (tile < 0) return;  // a slot without a tile (uniform)
    }
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int px = tx * BLOCK_X + (lane & 15);
    const int py0 = ty * BLOCK_Y + (lane >> 4);
    const float pfx = (float)px, pfy0 = (float)py0;
    const float row0 = (float)(ty * BLOCK_Y), col0 = (float)(tx * BLOCK_X);
    const uint2 range = p.ranges[tile];
    const uint32_t r0 = __builtin_amdgcn_readfirstlane(range.x);
    const uint32_t tl = __builtin_amdgcn_readfirstlane(p.tile_last[tile]);
    const uint32_t loaded = __builtin_amdgcn_readfirstlane(p.tile_loaded[tile]);
    // this wave's instances [lo, hi) (tile-relative); the last segment also zeroes the rows of [tile_last, loaded)
    uint32_t lo = 0, hi = tl;
    bool last_seg = true;
    if (SEG && ck_k) {
        lo = seg * ck_k;
        hi = min(lo + ck_k, tl);
        last_seg = lo + ck_k >= tl;
    }
    if (last_seg)
        for (uint32_t s = r0 + tl + lane; s < r0 + loaded; s += 64) {
            const float z[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
            store_row(p.rows, p.sorted_u[s], z);
        }
    if (hi == 0) {
        stamp_store(p.stamps, slot, t_start, lane);
        return;
    }

    const float bg0 = p.bg[0], bg1 = p.bg[1], bg2 = p.bg[2];
    const size_t HW = (size_t)p.W * p.H;
    float T[PIX_PER_LANE], dp0[PIX_PER_LANE], dp1[PIX_PER_LANE], dp2[PIX_PER_LANE], dinv[PIX_PER_LANE];
    float D[PIX_PER_LANE], prow[PIX_PER_LANE];
    uint32_t lastc[PIX_PER_LANE];
#pragma unroll
    for (int k = 0; k < PIX_PER_LANE; k++) {
        const int py = py0 + 4 * k;
        const bool inside = px < p.W && py < p.H;
        const size_t pid = inside ? (size_t)py * p.W + px : 0;
        T[k] = inside ? p.final_T[pid] : 0.f;
        lastc[k] = inside ? p.n_contrib[pid] : 0u;
        dp0[k] = inside ? p.dL_dpix[pid] : 0.f;
        dp1[k] = inside ? p.dL_dpix[HW + pid] : 0.f;
        dp2[k] = inside ? p.dL_dpix[2 * HW + pid] : 0.f;
        dinv[k] = (HAS_INV && inside) ? p.dL_dinvdepth[pid] : 0.f;
        D[k] = fmaf(bg2, dp2[k], fmaf(bg1, dp1[k], bg0 * dp0[k]));
        prow[k] = (float)py;  // dy = y - pixel row in one subtraction, as the forward
    }
    if (SEG && !last_seg) {  // start from the checkpoint before instance hi
        const float *ck = p.ckpt + (size_t)(r0 / ck_k + (uint32_t)tile + seg) * CK_FLOATS;
        const float *ct = p.ctot + (size_t)tile * 1024;
#pragma unroll
        for (int k = 0; k < PIX_PER_LANE; k++) {
            const int i = lane + 64 * k;
            if (hi < lastc[k]) {
                const float Te = ck[i];
                const float c0 = ct[i] - ck[256 + i], c1 = ct[256 + i] - ck[512 + i], c2 = ct[512 + i] - ck[768 + i];
                float num = fmaf(c2, dp2[k], fmaf(c1, dp1[k], c0 * dp0[k]));
                if (HAS_INV) num = fmaf(ct[768 + i] - ck[1024 + i], dinv[k], num);
                D[k] = fmaf(T[k], D[k], num) / Te;
                T[k] = Te;
            }
        }
    }
    const float hW = 0.5f * p.W, hH = 0.5f * p.H;
    // the forward's exact strip masks (whole-tile forwards write them), else the conservative cell masks
    const bool smask = p.strip_mask && __builtin_amdgcn_readfirstlane(*p.smask_valid);

    for (int bend = (int)hi; bend > (int)lo; bend -= BWD_BATCH) {
        const int cnt = min(BWD_BATCH, bend - (int)lo);
        float4 my_a = make_float4(0, 0, 0, 0), my_b = my_a;
        uint32_t my_row = 0, my_m = 0, my_gid = 0;
        if (lane < cnt) {
            const uint32_t s_me = r0 + (uint32_t)(bend - 1 - lane);
            my_row = p.sorted_u[s_me];
            const uint32_t gid = p.point_list[s_me];
            my_gid = gid;
            if (GUARD) s_rec[lane].pad.x = __uint_as_float(gid);  // the guard's slow path reloads the raw record
            my_a = p.rec[gid].a;
            my_b = p.rec[gid].b;
            s_rec[lane].a = stage_rec_a(my_a);
            s_rec[lane].b = stage_rec_b(my_b);
            s_rec[lane].c = p.rec[gid].c;
            my_m = smask ? (uint32_t)p.strip_mask[s_me] : cell_mask(p.strip_exact, my_a, my_b, row0, col0);
        }
        // sk[k] bit j: strip k of instance j (idx = bend - 1 - j) may hold a contributing pixel.  (Strip liveness and
        // compare skipping from the strips' n_contrib bounds measured 2.5 % slower -- SALU -- and was removed.)
        uint64_t sk[PIX_PER_LANE];
#pragma unroll
        for (int k = 0; k < PIX_PER_LANE; k++) sk[k] = __ballot((my_m >> k) & 1u);
        wave_lds_sync();
        // one instance's pass over the lane's pixels: updates T / D, returns the lane's raw sums (Q0, Q1, Q2, w0..w3) and dx in m and the
        // ballot of the lanes that contributed
        auto pass = [&](const int j, float m[8]) -> uint64_t {
            const uint32_t idx = (uint32_t)(bend - 1 - j);
            const FwdRec &r = s_rec[j];
            const float4 a = r.a, b = r.b;  // a: x, y, A, B; b: C, o, r, g
            const float2 c = r.c;           // b, 1/depth
            const float dx = a.x - pfx;
            const float P0 = (a.z * dx) * dx, L = a.w * dx;
                        // The union walk (long tiles) loads the accumulators' zeros from LDS: two ds_read_b128 in place of seven
            // v_mov per instance (cfg 5 render_bwd 0.801 -> 0.779 ms; the plain walk of cfg 3 measured no gain, and
            // the segment walk, at its 80-VGPR cap, spilled: profiles/r6x_libab_lds_zero_cfg*.txt)
            float4 z0 = make_float4(0.f, 0.f, 0.f, 0.f), z1 = z0;
            if constexpr (UNION) {
                z0 = s_zero[j][0];
                z1 = s_zero[j][1];
            }
            float Q0 = z0.x, Q1 = z0.y, Q2 = z0.z, w0 = z0.w, w1 = z1.x, w2 = z1.y, w3 = z1.z;
            uint64_t any = 0;
#pragma unroll
            for (int k = 0; k < PIX_PER_LANE; k++) {
                if (!((sk[k] >> j) & 1u)) continue;  // wave-uniform
                const float dy = a.y - prow[k];
                const float power2 = power2_at(b.x, dy, P0, L);
                const float G = __builtin_amdgcn_exp2f(power2);
                const float alpha = fminf(0.99f, b.y * G);
                // the contributing lanes as a scalar mask straight from the compares: !(power2 > 0),
                // !(alpha < 1/255) and idx < n_contrib
                uint64_t ok = __builtin_amdgcn_fcmpf(power2, 0.0f, FCMP_ULE) &
                              __builtin_amdgcn_fcmpf(alpha, GUARD ? GUARD_A_LO : 1.0f / 255.0f, FCMP_UGE);
                if constexpr (GUARD) {  // the forward's guarded alpha decision, taken by the same test (gsr_common.h)
                    const uint64_t near = ok & ~__builtin_amdgcn_fcmpf(alpha, GUARD_A_HI, FCMP_UGE);
                    if (__builtin_expect(near != 0, 0)) {  // rare
                        const uint32_t g = __float_as_uint(r.pad.x);
                        const uint64_t okx = __ballot(guard_alpha_pass(p.rec, g, pfx, pfy0 + (float)(4 * k)));
                        ok = (ok & ~near) | (okx & near);
                    }
                }
                ok &= __builtin_amdgcn_uicmp(idx, lastc[k], ICMP_ULT);
                any |= ok;
                if (!__builtin_amdgcn_inverse_ballot_w64(ok)) continue;  // exec = ok
                T[k] = T[k] * fast_rcp(1.f - alpha);
                const float wgt = alpha * T[k];
                float cd = fmaf(c.x, dp2[k], fmaf(b.w, dp1[k], b.z * dp0[k]));
                if (HAS_INV) cd = fmaf(c.y, dinv[k], cd);
                const float d = cd - D[k];
                D[k] = fmaf(alpha, d, D[k]);
                w0 = fmaf(wgt, dp0[k], w0);
                w1 = fmaf(wgt, dp1[k], w1);
                w2 = fmaf(wgt, dp2[k], w2);
                if (HAS_INV) w3 = fmaf(wgt, dinv[k], w3);
                const float q = G * (d * T[k]);
                const float qdy = q * dy;
                Q0 += q;
                Q1 += qdy;
                Q2 = fmaf(qdy, dy, Q2);
            }
            m[0] = Q0;
            m[1] = Q1;
            m[2] = Q2;
            m[3] = w0;
            m[4] = w1;
            m[5] = w2;
            m[6] = w3;
            m[7] = dx;
            return any;
        };
        if constexpr (UNION) {
        // pair up only the instances that reach a live strip (lowest first); an instance's gradient bits do not
        // depend on its partner (wave_reduce_pair_store), and the others get zero sums from their own lane
        uint64_t un = 0;
#pragma unroll
        for (int k = 0; k < PIX_PER_LANE; k++) un |= sk[k];
        un &= cnt >= 64 ? ~0ull : (1ull << cnt) - 1ull;
        if (lane < cnt && !((un >> lane) & 1ull)) {
            float4 *z = reinterpret_cast<float4 *>(s_part[lane]);
            z[0] = make_float4(0.f, 0.f, 0.f, 0.f);
            z[1] = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float2 *>(s_part[lane] + 8) = make_float2(0.f, 0.f);
        }
        while (un) {
            const int j0 = (int)__builtin_ctzll(un);
            un &= ~(1ull << j0);  // s_andn2 with the strip tests' bit (un & (un - 1) costs three SALU)
            float m0[8];
            const uint64_t any0 = pass(j0, m0);
            float *dst = s_part[j0];
            if (un) {
                const int j1 = (int)__builtin_ctzll(un);
                un &= ~(1ull << j1);
                float m1[8];
                const uint64_t any1 = pass(j1, m1);
                float *dst1 = s_part[j1];
                if (any0 | any1) {
                    wave_reduce_pair_store(m0, m1, dst, lane, dst1);
                } else if (lane < 10) {
                    dst[lane] = 0.f;
                    dst1[lane] = 0.f;
                }
            } else if (any0) {
                wave_reduce_pair_store<false>(m0, kZero8, dst, lane);
            } else if (lane < 10) {
                dst[lane] = 0.f;
            }
        }
        } else {
        for (int j = 0; j < cnt; j += 2) {
            float m0[8];
            const uint64_t any0 = pass(j, m0);
            float *dst = s_part[j];
            if (j + 1 < cnt) {
                float m1[8];
                const uint64_t any1 = pass(j + 1, m1);
                if (any0 | any1) {
                    wave_reduce_pair_store(m0, m1, dst, lane);
                } else if (lane < 10) {
                    dst[lane] = 0.f;
                    dst[PART + lane] = 0.f;
                }
            } else if (any0) {
                wave_reduce_pair_store<false>(m0, kZero8, dst, lane);
            } else if (lane < 10) {
                dst[lane] = 0.f;
            }
        }
        }
        wave_lds_sync();
        if (lane < cnt) {
            const float4 *src = reinterpret_cast<const float4 *>(s_part[lane]);
            const float4 u0 = src[0], u1 = src[1];
            const float2 u2 = *reinterpret_cast<const float2 *>(s_part[lane] + 8);
            const float S = u0.x, Sx = u0.y, Sy = u0.z, Sxx = u0.w, Sxy = u1.x, Syy = u1.y;
            const float o = my_b.y, ca = my_a.z, cb = my_a.w, cc = my_b.x;
            float row[10];
            row[0] = -o * hW * (ca * Sx + cb * Sy);
            row[1] = -o * hH * (cb * Sx + cc * Sy);
            row[2] = -0.5f * o * Sxx;
            row[3] = -0.5f * o * Sxy;
            row[4] = -0.5f * o * Syy;
            row[5] = S;
            row[6] = u1.z;
            row[7] = u1.w;
            row[8] = u2.x;
            row[9] = u2.y;
            store_row(p.rows, my_row, row);
            if (p.live && row_nonzero(row)) p.live[my_gid] = 1;
        }
        wave_lds_sync();
    }
    stamp_store(p.stamps, slot, t_start, lane);
}

// (tile, segment) work list of the segmented backward, one workgroup: tiles in the backward's LPT order (heaviest
// first), each split into ceil(tile_last / K) segments (K = *ck_flag, the forward's checkpoint spacing; 0: one
// segment per tile); *seg_count = the number of items.  T <= SEG_MAX_TILES (4 tiles per thread).
__global__ __launch_bounds__(1024) void seg_list_kernel(const uint32_t *__restrict__ order,
                                                        const uint32_t *__restrict__ tile_last, int T,
                                                        const uint32_t *__restrict__ ck_flag, uint2 *__restrict__ list,
                                                        uint32_t *__restrict__ count) {
    __shared__ uint32_t s_wsum[16];
    constexpr int PER = (int)SEG_MAX_TILES / 1024;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t K = *ck_flag;
    uint32_t t[PER], n[PER], sum = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int i = tid * PER + q;
        t[q] = i < T ? (order ? order[i] : (uint32_t)i) : 0u;
        const uint32_t tl = i < T ? tile_last[t[q]] : 0u;
        n[q] = i < T ? (K ? max(1u, (tl + K - 1) / K) : 1u) : 0u;
        sum += n[q];
    }
    const uint32_t inc = wave_inclusive_scan(sum, lane);
    if (lane == 63) s_wsum[w] = inc;
    __syncthreads();
    uint32_t base = inc - sum, total = 0;
    for (int i = 0; i < 16; i++) {
        const uint32_t v = s_wsum[i];
        if (i < w) base += v;
        total += v;
    }
#pragma unroll
    for (int q = 0; q < PER; q++) {
        for (uint32_t s = 0; s < n[q]; s++) list[base + s] = make_uint2(t[q], s);
        base += n[q];
    }
    if (tid == 0) *count = total;
}

void launch_render_bwd(hipStream_t s, const RenderBwdParams &p) {
    if (p.num_tiles <= 0) return;
    RenderBwdParams q = p;
    q.strip_exact = tuning("strip_exact", 1);
    q.stamps = tuning("stamp", 0) ? stamp_buffer(1) : nullptr;
    // threshold guard band ("guard" 1, the forward's knob; the segmented and whole-tile walks, not the parts form)
    const bool gd = tuning("guard", 0) != 0;
    if (p.seg_list && p.ck_flag && p.ckpt && p.ctot && p.seg_count && p.num_tiles <= (int)SEG_MAX_TILES) {
        // segmented walk (800x800, 2500 tiles: one wave per 128-instance segment against 4 part-waves per tile)
        seg_list_kernel<<<1, 1024, 0, s>>>(p.tile_order, p.tile_last, p.num_tiles, p.ck_flag, q.seg_list, q.seg_count);
        const dim3 grid((uint32_t)seg_slots((int64_t)p.num_rendered, (uint32_t)p.num_tiles)), block(64);
        if (gd && p.dL_dinvdepth) render_bwd_v5_kernel<true, false, true, true><<<grid, block, 0, s>>>(q);
        else if (gd) render_bwd_v5_kernel<false, false, true, true><<<grid, block, 0, s>>>(q);
        else if (p.dL_dinvdepth) render_bwd_v5_kernel<true, false, true><<<grid, block, 0, s>>>(q);
        else render_bwd_v5_kernel<false, false, true><<<grid, block, 0, s>>>(q);
        return;
    }
    // "bwd_parts" 1, 2 or 4; 0 (default): 4 or 2 while that many part-waves fit within bwd_part_slots
    // (1024 SIMDs x 12: 800x800 (2500 tiles) takes 4 parts, 0.143 ms against 0.149 in 2 and 0.181 whole; 1080p
    // (8160 tiles) whole tiles)
    int parts = tuning("bwd_parts", 0);
    const int slots = tuning("bwd_part_slots", 12288);
    if (parts == 0) parts = p.num_tiles * 4 <= slots ? 4 : p.num_tiles * 2 <= slots ? 2 : 1;
    if (gd) parts = 1;
    if (parts == 2 || parts == 4) {
        const dim3 grid(p.num_tiles), block(64 * parts);
        if (p.dL_dinvdepth) {
            if (parts == 2) render_bwd_parts_kernel<true, 2><<<grid, block, 0, s>>>(q);
            else render_bwd_parts_kernel<true, 4><<<grid, block, 0, s>>>(q);
        } else {
            if (parts == 2) render_bwd_parts_kernel<false, 2><<<grid, block, 0, s>>>(q);
            else render_bwd_parts_kernel<false, 4><<<grid, block, 0, s>>>(q);
        }
        return;
    }
    // with the forward's bucket lists the slots run to xcd_slots(T) (per-XCD lists); the extra ones exit
    const dim3 grid(p.lpt_blist ? xcd_slots((uint32_t)p.num_tiles) : (uint32_t)p.num_tiles), block(64);
    // "bwd_union" -1 (auto): pair only the instances that reach a strip when tiles are long (mean above 1024
    // instances: cfg 5 render_bwd 0.93 -> 0.90 ms; at cfg 3's 517 the plain walk is faster, 0.305 vs 0.329 ms);
    // 0 / 1 force it
    const int un = tuning("bwd_union", -1);
    const bool u = un < 0 ? p.num_rendered > (uint64_t)1024 * (uint64_t)p.num_tiles : un != 0;
    if (gd) {
        if (p.dL_dinvdepth && u) render_bwd_v5_kernel<true, true, false, true><<<grid, block, 0, s>>>(q);
        else if (p.dL_dinvdepth) render_bwd_v5_kernel<true, false, false, true><<<grid, block, 0, s>>>(q);
        else if (u) render_bwd_v5_kernel<false, true, false, true><<<grid, block, 0, s>>>(q);
        else render_bwd_v5_kernel<false, false, false, true><<<grid, block, 0, s>>>(q);
        return;
    }
    if (p.dL_dinvdepth) {
        if (u) render_bwd_v5_kernel<true, true><<<grid, block, 0, s>>>(q);
        else render_bwd_v5_kernel<true><<<grid, block, 0, s>>>(q);
    } else {
        if (u) render_bwd_v5_kernel<false, true><<<grid, block, 0, s>>>(q);
        else render_bwd_v5_kernel<false><<<grid, block, 0, s>>>(q);
    }
}

// ------------------------------------------------------------------------------------------------
// Gaussians with many instances: one block sums all their rows (fixed stride order, deterministic)
// into bigsum[slot], which the preprocess backward then reads instead of walking the rows.
// ------------------------------------------------------------------------------------------------
template <bool PERSIST>
__global__ __launch_bounds__(256) void big_reduce_kernel(BigReduceParams p) {
    __shared__ float s_part[4][10];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // PERSIST: the big-Gaussian count is only known on the device, so the launch is sized by min(upper bound, 2048)
    // workgroups that loop to it, instead of one per possible big Gaussian; else one workgroup per big Gaussian (no loop:
    // the loop's live state took the kernel from 64 to 80 VGPRs, 8 to 6 waves, cfg 5 0.078 -> 0.12 ms)
    const uint32_t nb = PERSIST ? *p.nbig_dev : gridDim.x;
    for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {  // workgroup-uniform
        const uint32_t gidx = p.big_list[bi];
        const uint32_t start = p.inst_start[gidx], cnt = p.tiles[gidx];
        float acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        // rows by expansion index (every cell of a big Gaussian's rect is an instance): BR_UNROLL inv words per thread
        // (INV_NONE: the forward composite did not load the instance, no row) are loaded together, then the rows of
        // the loaded instances (most instances of a big Gaussian sit in saturated tiles and have none), summed in the
        // same k order as one at a time
        constexpr int BR_UNROLL = 4;
        for (uint32_t k0 = threadIdx.x; k0 < cnt; k0 += 256 * BR_UNROLL) {
            float r[BR_UNROLL][10];
            bool use[BR_UNROLL];
            // (guarded loads: unconditional clamped inv loads measured +10 us at cfg 5, where most of the 4 x 256 slots
            // of a big Gaussian lie past its count)
#pragma unroll
            for (int q = 0; q < BR_UNROLL; q++) {
                const uint32_t k = k0 + 256 * q;
                use[q] = k < cnt && p.inv[start + k] != INV_NONE;
            }
            // (rows stay under `if (use)`: loading row 0 for the unwritten ones instead measured slower at cfg 5)
#pragma unroll
            for (int q = 0; q < BR_UNROLL; q++)
                if (use[q]) load_row(p.rows, start + k0 + 256 * q, r[q]);
#pragma unroll
            for (int q = 0; q < BR_UNROLL; q++)
                if (use[q]) {
#pragma unroll
                    for (int v = 0; v < 10; v++) acc[v] += r[q][v];
                }
        }
#pragma unroll
        for (int v = 0; v < 10; v++) {
            const float sum = wave_sum(acc[v]);
            if (lane == 0) s_part[w][v] = sum;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            float tot[10];
#pragma unroll
            for (int v = 0; v < 10; v++) tot[v] = ((s_part[0][v] + s_part[1][v]) + s_part[2][v]) + s_part[3][v];
            store_row(p.bigsum, bi, tot);
        }
        if (!PERSIST) break;
        __syncthreads();  // s_part is rewritten by the next big Gaussian
    }
}

void launch_big_reduce(hipStream_t s, const BigReduceParams &p, uint32_t nbig) {
    if (nbig == 0) return;
    if (p.nbig_dev) big_reduce_kernel<true><<<std::min(nbig, 2048u), 256, 0, s>>>(p);
    else big_reduce_kernel<false><<<nbig, 256, 0, s>>>(p);
}

}  // namespace gsr
