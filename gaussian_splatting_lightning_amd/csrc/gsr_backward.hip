// gsr_backward.hip -- backward kernels: reverse-walk compositing gradient, per-Gaussian reduction,
// and the preprocess backward (2D conic -> cov2D -> cov3D -> scale/rotation, 2D mean -> 3D mean,
// SH -> colour).
//
// The upstream CUDA backward scatters every (pixel, Gaussian) contribution with ~10 global float
// atomics (SURVEY.md §2.1 BACKWARD::render).  Here one wave owns one tile: each lane walks 4 pixels
// in reverse, the wave sums the per-instance contributions with DPP reductions, and writes ONE 48-byte
// gradient row per (tile, Gaussian) instance, contiguously in sorted order.  The per-Gaussian kernel
// then gathers its rows through the inverse permutation.  No float atomics, so gradients are
// bitwise reproducible run to run.
#include "gsr_kernels.h"
#include "gsr_sh.h"

namespace gsr {

// Row layout: [0] dmean2D.x  [1] dmean2D.y  [2] dconic.x  [3] dconic.y  [4] dconic.w  [5] dopacity
//             [6..8] dcolor  [9] dinvdepth  [10..11] pad
__device__ __forceinline__ void store_row(float *__restrict__ rows, uint32_t s, const float r[10]) {
    float4 *dst = reinterpret_cast<float4 *>(rows + (size_t)s * GRAD_ROW);
    dst[0] = make_float4(r[0], r[1], r[2], r[3]);
    dst[1] = make_float4(r[4], r[5], r[6], r[7]);
    dst[2] = make_float4(r[8], r[9], 0.f, 0.f);
}

__device__ __forceinline__ void add_row(const float *__restrict__ rows, uint32_t s, float acc[10]) {
    const float4 *src = reinterpret_cast<const float4 *>(rows + (size_t)s * GRAD_ROW);
    const float4 a = src[0], b = src[1], c = src[2];
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
    acc[8] += c.x; acc[9] += c.y;
}

// ------------------------------------------------------------------------------------------------
// v3: moment accumulation + two-level reduction.
//   Per active (pixel, instance) pair a lane accumulates q = G * dL/dalpha and the moments q, q dx, q dy,
//   q dx^2, q dx dy, q dy^2 (plus the colour / inverse-depth weights).  Since dL/dG = o dL/dalpha and
//   dG/ddelta = -G (conic . delta), every conic / mean / opacity gradient term of the reference is a
//   uniform combination of these moments, applied once per instance after the reduction:
//     dopacity = S,  dconic = -o/2 (Sxx, Sxy, Syy),  dmean2D = -o (W/2, H/2) * (a Sx + b Sy, b Sx + c Sy).
//   The 10 per-lane sums are reduced across the wave by a transposing permlane/DPP reduction
//   (wave_reduce10_store) into LDS; after each batch of 32 instances lane j reads the 10 totals of instance j,
//   applies the uniform conversion and stores the gradient row.
// ------------------------------------------------------------------------------------------------
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

// Transposing reduction of 10 per-lane values over the wave: each exchange level halves the number of live
// registers by keeping one value of a pair on each side of the lane split (permlane32 / permlane16 swaps for
// lane bits 5 and 4, a DPP row_ror:8 exchange for bit 3), then bits 0-2 are summed with DPP.  ~30 VALU ops
// instead of 50 (5 DPP adds per value).  Lane l ends with the wave total of value 4 b3 + 2 b4 + b5 in c0 and
// of value 8 + b5 in c8 (b = bits of l); lanes with l % 8 == 0 store them.
__device__ __forceinline__ void wave_reduce10_store(const float m[10], float *__restrict__ dst, int lane) {
    const float a0 = sum_swap32(m[0], m[1]), a1 = sum_swap32(m[2], m[3]), a2 = sum_swap32(m[4], m[5]);
    const float a3 = sum_swap32(m[6], m[7]), a4 = sum_swap32(m[8], m[9]);  // a_i: value 2 i + b5
    const float b0 = sum_swap16(a0, a1);  // value 2 b4 + b5
    const float b1 = sum_swap16(a2, a3);  // value 4 + 2 b4 + b5
    float c8 = sum_swap16(a4, a4);        // value 8 + b5
    const bool hi3 = (lane & 8) != 0;
    const float keep = hi3 ? b1 : b0, send = hi3 ? b0 : b1;
    float c0 = keep + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0x128, 0xf, 0xf, false));
    c8 = dpp_add<0x128>(c8);  // row_ror:8 (= lane ^ 8)
    c0 = dpp_add<0xB1>(c0);   // quad_perm [1,0,3,2]
    c8 = dpp_add<0xB1>(c8);
    c0 = dpp_add<0x4E>(c0);   // quad_perm [2,3,0,1]
    c8 = dpp_add<0x4E>(c8);
    c0 = dpp_add<0x141>(c0);  // row_half_mirror: lanes {l, l^7} -> all 8 lanes of the half row
    c8 = dpp_add<0x141>(c8);
    if ((lane & 7) == 0) dst[((lane >> 1) & 4) | ((lane >> 3) & 2) | (lane >> 5)] = c0;
    if ((lane & 31) == 0) dst[8 + (lane >> 5)] = c8;
}

template <bool HAS_INV, int MIN_WAVES>
__global__ __launch_bounds__(256, MIN_WAVES) void render_bwd_v3_kernel(RenderBwdParams p) {
    __shared__ float4 s_a[4][BWD_BATCH];
    __shared__ float4 s_b[4][BWD_BATCH];
    __shared__ float2 s_c[4][BWD_BATCH];
    __shared__ __attribute__((aligned(16))) float s_part[4][BWD_BATCH][PART];  // [wave][instance][10 sums]
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + w;
    if (tile >= p.num_tiles) return;
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int px = tx * BLOCK_X + (lane & 15);
    const int py0 = ty * BLOCK_Y + (lane >> 4);
    const float pfx = (float)px;
    const uint2 range = p.ranges[tile];
    const uint32_t tl = p.tile_last[tile];

    // Loaded instances past every pixel's last contributor get exactly zero gradient; instances the
    // forward never loaded have inv = INV_NONE and are skipped by the per-Gaussian reduction.
    const uint32_t loaded = p.tile_loaded[tile];
    for (uint32_t s = range.x + tl + lane; s < range.x + loaded; s += 64) {
        const float z[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        store_row(p.rows, s, z);
    }
    if (tl == 0) return;

    const float bg0 = p.bg[0], bg1 = p.bg[1], bg2 = p.bg[2];
    const size_t HW = (size_t)p.W * p.H;
    float T[PIX_PER_LANE], nbg[PIX_PER_LANE], dp0[PIX_PER_LANE], dp1[PIX_PER_LANE], dp2[PIX_PER_LANE];
    float dinv[PIX_PER_LANE], ar0[PIX_PER_LANE], ar1[PIX_PER_LANE], ar2[PIX_PER_LANE], ainv[PIX_PER_LANE];
    float pfy[PIX_PER_LANE];
    uint32_t lastc[PIX_PER_LANE];
#pragma unroll
    for (int k = 0; k < PIX_PER_LANE; k++) {
        const int py = py0 + 4 * k;
        const bool inside = px < p.W && py < p.H;
        const size_t pid = inside ? (size_t)py * p.W + px : 0;
        const float Tf = inside ? p.final_T[pid] : 0.f;
        T[k] = Tf;
        pfy[k] = (float)py;
        lastc[k] = inside ? p.n_contrib[pid] : 0u;
        dp0[k] = inside ? p.dL_dpix[pid] : 0.f;
        dp1[k] = inside ? p.dL_dpix[HW + pid] : 0.f;
        dp2[k] = inside ? p.dL_dpix[2 * HW + pid] : 0.f;
        dinv[k] = (HAS_INV && inside) ? p.dL_dinvdepth[pid] : 0.f;
        nbg[k] = -Tf * (bg0 * dp0[k] + bg1 * dp1[k] + bg2 * dp2[k]);
        ar0[k] = ar1[k] = ar2[k] = ainv[k] = 0.f;
    }
    const float hW = 0.5f * p.W, hH = 0.5f * p.H;

    for (int bend = (int)tl; bend > 0; bend -= BWD_BATCH) {
        const int cnt = min(BWD_BATCH, bend);
        float4 my_a = make_float4(0, 0, 0, 0), my_b = my_a;
        if (lane < cnt) {
            const uint32_t gid = p.point_list[range.x + (uint32_t)(bend - 1 - lane)];
            my_a = p.rec_a[gid];
            my_b = p.rec_b[gid];
            s_a[w][lane] = stage_rec_a(my_a);
            s_b[w][lane] = stage_rec_b(my_b);
            s_c[w][lane] = p.rec_c[gid];
        }
        wave_lds_sync();
        for (int j = 0; j < cnt; j++) {
            const uint32_t idx = (uint32_t)(bend - 1 - j);
            const float4 a = s_a[w][j];  // x, y, A, B
            const float4 b = s_b[w][j];  // C, o, r, g
            const float2 c = s_c[w][j];  // b, 1/depth
            const float dx = a.x - pfx;
            const float P0 = (a.z * dx) * dx, L = a.w * dx;
            // per lane: Q0 = sum q, Q1 = sum q dy, Q2 = sum q dy^2 over its pixels (dx is shared), colour weights
            float Q0 = 0.f, Q1 = 0.f, Q2 = 0.f, w0 = 0.f, w1 = 0.f, w2 = 0.f, w3 = 0.f;
            bool any = false;
#pragma unroll
            for (int k = 0; k < PIX_PER_LANE; k++) {
                if (idx >= lastc[k]) continue;
                const float dy = a.y - pfy[k];
                const float power2 = power2_at(b.x, dy, P0, L);
                if (power2 > 0.0f) continue;
                const float G = __builtin_amdgcn_exp2f(power2);
                const float alpha = fminf(0.99f, b.y * G);
                if (alpha < 1.0f / 255.0f) continue;
                any = true;
                const float one_m = 1.f - alpha;
                const float r = fast_rcp(one_m);
                T[k] = T[k] * r;
                const float wgt = alpha * T[k];
                const float d0 = b.z - ar0[k], d1 = b.w - ar1[k], d2 = c.x - ar2[k];
                float dL_dalpha = d0 * dp0[k];
                dL_dalpha = fmaf(d1, dp1[k], dL_dalpha);
                dL_dalpha = fmaf(d2, dp2[k], dL_dalpha);
                w0 = fmaf(wgt, dp0[k], w0);
                w1 = fmaf(wgt, dp1[k], w1);
                w2 = fmaf(wgt, dp2[k], w2);
                ar0[k] = fmaf(alpha, d0, ar0[k]);  // alpha c + (1 - alpha) accum
                ar1[k] = fmaf(alpha, d1, ar1[k]);
                ar2[k] = fmaf(alpha, d2, ar2[k]);
                if (HAS_INV) {
                    const float di = c.y - ainv[k];
                    dL_dalpha = fmaf(di, dinv[k], dL_dalpha);
                    w3 = fmaf(wgt, dinv[k], w3);
                    ainv[k] = fmaf(alpha, di, ainv[k]);
                }
                dL_dalpha = fmaf(dL_dalpha, T[k], nbg[k] * r);
                const float q = G * dL_dalpha;
                const float qdy = q * dy;
                Q0 += q;
                Q1 += qdy;
                Q2 = fmaf(qdy, dy, Q2);
            }
            float *dst = s_part[w][j];
            if (__ballot(any)) {
                float m[10];
                m[0] = Q0;
                m[1] = Q0 * dx;
                m[2] = Q1;
                m[3] = m[1] * dx;
                m[4] = Q1 * dx;
                m[5] = Q2;
                m[6] = w0;
                m[7] = w1;
                m[8] = w2;
                m[9] = w3;
                wave_reduce10_store(m, dst, lane);
            } else if (lane < 10) {
                dst[lane] = 0.f;
            }
        }
        wave_lds_sync();
        if (lane < cnt) {
            const float4 *src = reinterpret_cast<const float4 *>(s_part[w][lane]);
            const float4 u0 = src[0], u1 = src[1];
            const float2 u2 = *reinterpret_cast<const float2 *>(s_part[w][lane] + 8);
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
            store_row(p.rows, range.x + (uint32_t)(bend - 1 - lane), row);
        }
        wave_lds_sync();
    }
}

void launch_render_bwd(hipStream_t s, const RenderBwdParams &p) {
    if (p.num_tiles <= 0) return;
    const dim3 grid(div_up(p.num_tiles, 4)), block(256);
    const int minw = tuning("bwd_minwaves", 4);
    if (p.dL_dinvdepth) {
        if (minw >= 4) render_bwd_v3_kernel<true, 4><<<grid, block, 0, s>>>(p);
        else render_bwd_v3_kernel<true, 1><<<grid, block, 0, s>>>(p);
    } else {
        if (minw >= 4) render_bwd_v3_kernel<false, 4><<<grid, block, 0, s>>>(p);
        else render_bwd_v3_kernel<false, 1><<<grid, block, 0, s>>>(p);
    }
}

// ------------------------------------------------------------------------------------------------
// Gaussians with many instances: one block sums all their rows (fixed stride order, deterministic)
// into bigsum[slot], which the preprocess backward then reads instead of walking the rows.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void big_reduce_kernel(BigReduceParams p) {
    __shared__ float s_part[4][10];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t bi = blockIdx.x;
    const uint32_t gidx = p.big_list[bi];
    const uint32_t start = p.inst_start[gidx], cnt = p.tiles[gidx];
    float acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t k = threadIdx.x; k < cnt; k += 256) {
        const uint32_t sidx = p.inv[start + k];
        if (sidx != INV_NONE) add_row(p.rows, sidx, acc);
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
}

void launch_big_reduce(hipStream_t s, const BigReduceParams &p, uint32_t nbig) {
    if (nbig == 0) return;
    big_reduce_kernel<<<nbig, 256, 0, s>>>(p);
}

// ------------------------------------------------------------------------------------------------
// preprocess backward: one thread per Gaussian
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void cov3d_backward(float3 scale, float mod, float4 rot, const float dc[6],
                                               float3 &dscale, float4 &drot) {
    const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
    const Mat3 R = quat_to_rot(rot);
    const float s[3] = {mod * scale.x, mod * scale.y, mod * scale.z};
    float M[3][3], dSig[3][3], dM[3][3], dMt[3][3];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++) M[c][rr] = s[rr] * R.m[c][rr];
    dSig[0][0] = dc[0]; dSig[0][1] = 0.5f * dc[1]; dSig[0][2] = 0.5f * dc[2];
    dSig[1][0] = 0.5f * dc[1]; dSig[1][1] = dc[3]; dSig[1][2] = 0.5f * dc[4];
    dSig[2][0] = 0.5f * dc[2]; dSig[2][1] = 0.5f * dc[4]; dSig[2][2] = dc[5];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++)
            dM[c][rr] = 2.0f * (M[0][rr] * dSig[c][0] + M[1][rr] * dSig[c][1] + M[2][rr] * dSig[c][2]);
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++) dMt[c][rr] = dM[rr][c];
    // dL/ds (w.r.t. the modified scale, as upstream; DESIGN.md notes the scale_modifier factor)
    dscale.x = R.m[0][0] * dMt[0][0] + R.m[1][0] * dMt[0][1] + R.m[2][0] * dMt[0][2];
    dscale.y = R.m[0][1] * dMt[1][0] + R.m[1][1] * dMt[1][1] + R.m[2][1] * dMt[1][2];
    dscale.z = R.m[0][2] * dMt[2][0] + R.m[1][2] * dMt[2][1] + R.m[2][2] * dMt[2][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        dMt[0][k] *= s[0];
        dMt[1][k] *= s[1];
        dMt[2][k] *= s[2];
    }
    drot.x = 2 * z * (dMt[0][1] - dMt[1][0]) + 2 * y * (dMt[2][0] - dMt[0][2]) + 2 * x * (dMt[1][2] - dMt[2][1]);
    drot.y = 2 * y * (dMt[1][0] + dMt[0][1]) + 2 * z * (dMt[2][0] + dMt[0][2]) + 2 * r * (dMt[1][2] - dMt[2][1]) -
             4 * x * (dMt[2][2] + dMt[1][1]);
    drot.z = 2 * x * (dMt[1][0] + dMt[0][1]) + 2 * r * (dMt[2][0] - dMt[0][2]) + 2 * z * (dMt[1][2] + dMt[2][1]) -
             4 * y * (dMt[2][2] + dMt[0][0]);
    drot.w = 2 * r * (dMt[0][1] - dMt[1][0]) + 2 * x * (dMt[2][0] + dMt[0][2]) + 2 * y * (dMt[1][2] + dMt[2][1]) -
             4 * z * (dMt[1][1] + dMt[0][0]);
}

__global__ __launch_bounds__(256) void preprocess_bwd_kernel(PreprocessBwdParams p) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= p.P) return;
    const bool vis = p.radii[i] > 0;
    float gs[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (vis) {
        const uint32_t start = p.inst_start[i], cnt = p.tiles[i];
        if (cnt > BIG_GAUSSIAN_TILES) {
            add_row(p.bigsum, p.big_slot[i], gs);
        } else {
            // issue the index loads, then all row loads of a group, before summing (memory-level parallelism)
            for (uint32_t k0 = 0; k0 < cnt; k0 += 4) {
                uint32_t sidx[4];
#pragma unroll
                for (int j = 0; j < 4; j++) sidx[j] = (k0 + j < cnt) ? p.inv[start + k0 + j] : INV_NONE;
                float4 ra[4], rb[4], rc[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (sidx[j] != INV_NONE) {
                        const float4 *src = reinterpret_cast<const float4 *>(p.rows + (size_t)sidx[j] * GRAD_ROW);
                        ra[j] = src[0];
                        rb[j] = src[1];
                        rc[j] = src[2];
                    } else {
                        ra[j] = rb[j] = rc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    gs[0] += ra[j].x; gs[1] += ra[j].y; gs[2] += ra[j].z; gs[3] += ra[j].w;
                    gs[4] += rb[j].x; gs[5] += rb[j].y; gs[6] += rb[j].z; gs[7] += rb[j].w;
                    gs[8] += rc[j].x; gs[9] += rc[j].y;
                }
            }
        }
    }
    if (p.dL_dmeans2D) {
        p.dL_dmeans2D[3 * i] = gs[0];
        p.dL_dmeans2D[3 * i + 1] = gs[1];
        p.dL_dmeans2D[3 * i + 2] = 0.f;
    }
    if (p.dL_dcolors) {
        p.dL_dcolors[3 * i] = gs[6];
        p.dL_dcolors[3 * i + 1] = gs[7];
        p.dL_dcolors[3 * i + 2] = gs[8];
    }
    const int ncoef = p.M * 3;
    if (!vis) {
        if (p.dL_dopacity) p.dL_dopacity[i] = 0.f;
        if (p.dL_dmeans3D) { p.dL_dmeans3D[3 * i] = 0.f; p.dL_dmeans3D[3 * i + 1] = 0.f; p.dL_dmeans3D[3 * i + 2] = 0.f; }
        if (p.dL_dcov3D)
            for (int k = 0; k < 6; k++) p.dL_dcov3D[6 * i + k] = 0.f;
        if (p.dL_dsh)
            for (int k = 0; k < ncoef; k++) p.dL_dsh[(size_t)i * ncoef + k] = 0.f;
        if (p.dL_dcolors_sh) { p.dL_dcolors_sh[3 * i] = 0.f; p.dL_dcolors_sh[3 * i + 1] = 0.f; p.dL_dcolors_sh[3 * i + 2] = 0.f; }
        if (p.dL_dscales) { p.dL_dscales[3 * i] = 0.f; p.dL_dscales[3 * i + 1] = 0.f; p.dL_dscales[3 * i + 2] = 0.f; }
        if (p.dL_drot)
            for (int k = 0; k < 4; k++) p.dL_drot[4 * i + k] = 0.f;
        return;
    }
    const Mat4 view = load_mat4(p.view);
    const float3 mean = load_f3(p.means3D, i);
    float c6[6];
    float3 scale = make_float3(0, 0, 0);
    float4 rot = make_float4(1, 0, 0, 0);
    if (p.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; k++) c6[k] = p.cov3D_precomp[6 * i + k];
    } else {
        scale = load_f3(p.scales, i);
        rot = make_float4(p.rotations[4 * i], p.rotations[4 * i + 1], p.rotations[4 * i + 2], p.rotations[4 * i + 3]);
        cov3d_from_scale_rot(scale, p.scale_modifier, rot, c6);
    }
    // ---- computeCov2D backward ----
    const EwaT e = ewa_T(mean, view, p.focal_x, p.focal_y, p.tan_fovx, p.tan_fovy);
    float c_xx = quad_form(e.t0, c6, e.t0), c_xy = quad_form(e.t1, c6, e.t0), c_yy = quad_form(e.t1, c6, e.t1);
    constexpr float h_var = 0.3f;
    float dopac = gs[5];
    float d_inside_root = 0.f;
    if (p.antialiasing) {
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_cov_plus = c_xx * c_yy - c_xy * c_xy;
        const float hs = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus));
        const float d_hs = dopac * p.opacities[i];
        dopac = dopac * hs;
        d_inside_root = (det_cov / det_cov_plus) <= 0.000025f ? 0.f : d_hs / (2 * hs);
    } else {
        c_xx += h_var;
        c_yy += h_var;
    }
    float dL_dc_xx = 0.f, dL_dc_xy = 0.f, dL_dc_yy = 0.f;
    if (p.antialiasing) {
        const float x = c_xx, y = c_yy, z = c_xy, wv = h_var;
        const float q = wv * wv + wv * (x + y) + x * y - z * z;
        const float denom_f = d_inside_root / (q * q);
        dL_dc_xx = wv * (wv * y + y * y + z * z) * denom_f;
        dL_dc_yy = wv * (wv * x + x * x + z * z) * denom_f;
        dL_dc_xy = -2.f * wv * z * (wv + x + y) * denom_f;
    }
    if (p.dL_dopacity) p.dL_dopacity[i] = dopac;
    const float dcx = gs[2], dcy = gs[3], dcz = gs[4];
    const float denom = c_xx * c_yy - c_xy * c_xy;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float dcov[6] = {0, 0, 0, 0, 0, 0};
    const float *t0 = e.t0, *t1 = e.t1;
    if (denom2inv != 0) {
        dL_dc_xx += denom2inv * (-c_yy * c_yy * dcx + 2 * c_xy * c_yy * dcy + (denom - c_xx * c_yy) * dcz);
        dL_dc_yy += denom2inv * (-c_xx * c_xx * dcz + 2 * c_xx * c_xy * dcy + (denom - c_xx * c_yy) * dcx);
        dL_dc_xy += denom2inv * 2 * (c_xy * c_yy * dcx - (denom + 2 * c_xy * c_xy) * dcy + c_xx * c_xy * dcz);
        dcov[0] = (t0[0] * t0[0] * dL_dc_xx + t0[0] * t1[0] * dL_dc_xy + t1[0] * t1[0] * dL_dc_yy);
        dcov[3] = (t0[1] * t0[1] * dL_dc_xx + t0[1] * t1[1] * dL_dc_xy + t1[1] * t1[1] * dL_dc_yy);
        dcov[5] = (t0[2] * t0[2] * dL_dc_xx + t0[2] * t1[2] * dL_dc_xy + t1[2] * t1[2] * dL_dc_yy);
        dcov[1] = 2 * t0[0] * t0[1] * dL_dc_xx + (t0[0] * t1[1] + t0[1] * t1[0]) * dL_dc_xy + 2 * t1[0] * t1[1] * dL_dc_yy;
        dcov[2] = 2 * t0[0] * t0[2] * dL_dc_xx + (t0[0] * t1[2] + t0[2] * t1[0]) * dL_dc_xy + 2 * t1[0] * t1[2] * dL_dc_yy;
        dcov[4] = 2 * t0[2] * t0[1] * dL_dc_xx + (t0[1] * t1[2] + t0[2] * t1[1]) * dL_dc_xy + 2 * t1[1] * t1[2] * dL_dc_yy;
    }
    if (p.dL_dcov3D)
        for (int k = 0; k < 6; k++) p.dL_dcov3D[6 * i + k] = dcov[k];
    float dT0[3], dT1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        // row k of the symmetric Vrk
        const float vk0 = k == 0 ? c6[0] : (k == 1 ? c6[1] : c6[2]);
        const float vk1 = k == 0 ? c6[1] : (k == 1 ? c6[3] : c6[4]);
        const float vk2 = k == 0 ? c6[2] : (k == 1 ? c6[4] : c6[5]);
        const float v0 = t0[0] * vk0 + t0[1] * vk1 + t0[2] * vk2;
        const float v1 = t1[0] * vk0 + t1[1] * vk1 + t1[2] * vk2;
        dT0[k] = 2 * v0 * dL_dc_xx + v1 * dL_dc_xy;
        dT1[k] = 2 * v1 * dL_dc_yy + v0 * dL_dc_xy;
    }
    const float *vm = view.m;
    const float dJ00 = vm[0] * dT0[0] + vm[4] * dT0[1] + vm[8] * dT0[2];
    const float dJ02 = vm[2] * dT0[0] + vm[6] * dT0[1] + vm[10] * dT0[2];
    const float dJ11 = vm[1] * dT1[0] + vm[5] * dT1[1] + vm[9] * dT1[2];
    const float dJ12 = vm[2] * dT1[0] + vm[6] * dT1[1] + vm[10] * dT1[2];
    const float3 t = e.t;
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float hx = p.focal_x, hy = p.focal_y;
    const float dtx = e.xmul * -hx * tz2 * dJ02;
    const float dty = e.ymul * -hy * tz2 * dJ12;
    float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * t.x) * tz3 * dJ02 + (2 * hy * t.y) * tz3 * dJ12;
    if (p.has_invdepth) dtz -= gs[9] / (t.z * t.z);
    float3 dm = make_float3(vm[0] * dtx + vm[1] * dty + vm[2] * dtz, vm[4] * dtx + vm[5] * dty + vm[6] * dtz,
                            vm[8] * dtx + vm[9] * dty + vm[10] * dtz);
    // ---- 2D mean -> 3D mean through the projection ----
    const Mat4 proj = load_mat4(p.proj);
    const float *pm = proj.m;
    const float4 mh = xform4(mean, proj);
    const float m_w = 1.0f / (mh.w + 0.0000001f);
    const float mul1 = (pm[0] * mean.x + pm[4] * mean.y + pm[8] * mean.z + pm[12]) * m_w * m_w;
    const float mul2 = (pm[1] * mean.x + pm[5] * mean.y + pm[9] * mean.z + pm[13]) * m_w * m_w;
    const float g2x = gs[0], g2y = gs[1];
    dm.x += (pm[0] * m_w - pm[3] * mul1) * g2x + (pm[1] * m_w - pm[3] * mul2) * g2y;
    dm.y += (pm[4] * m_w - pm[7] * mul1) * g2x + (pm[5] * m_w - pm[7] * mul2) * g2y;
    dm.z += (pm[8] * m_w - pm[11] * mul1) * g2x + (pm[9] * m_w - pm[11] * mul2) * g2y;
    // ---- SH backward ----
    if (p.shs && p.M > 0) {
        const uint8_t cl = p.clamped[i];
        const float3 dRGB = make_float3((cl & 1) ? 0.f : gs[6], (cl & 2) ? 0.f : gs[7], (cl & 4) ? 0.f : gs[8]);
        const float3 campos = make_float3(p.campos[0], p.campos[1], p.campos[2]);
        if (p.dL_dcolors_sh) {
            p.dL_dcolors_sh[3 * i] = dRGB.x;
            p.dL_dcolors_sh[3 * i + 1] = dRGB.y;
            p.dL_dcolors_sh[3 * i + 2] = dRGB.z;
        }
        float *dsh = p.dL_dsh ? p.dL_dsh + (size_t)i * ncoef : nullptr;  // null only with dL_dcolors_sh (API)
        const float *shp = p.shs + (size_t)i * ncoef;
        if (p.sh_vec16) {
            // 16 coefficients x 3 = 192 B per Gaussian: 12 float4 loads and stores per lane
            float shv[48], dshv[48];
            const float4 *s4 = reinterpret_cast<const float4 *>(shp);
#pragma unroll
            for (int k = 0; k < 12; k++) {
                const float4 q = s4[k];
                shv[4 * k] = q.x; shv[4 * k + 1] = q.y; shv[4 * k + 2] = q.z; shv[4 * k + 3] = q.w;
            }
#pragma unroll
            for (int k = 0; k < 48; k++) dshv[k] = 0.f;
            dm = dm + sh_backward_dispatch(p.D, shv, mean - campos, dRGB, dshv);
            if (dsh) {
                float4 *d4 = reinterpret_cast<float4 *>(dsh);
#pragma unroll
                for (int k = 0; k < 12; k++)
                    d4[k] = make_float4(dshv[4 * k], dshv[4 * k + 1], dshv[4 * k + 2], dshv[4 * k + 3]);
            }
        } else if (dsh) {
            dm = dm + sh_backward_dispatch(p.D, shp, mean - campos, dRGB, dsh);
            const int used = (p.D + 1) * (p.D + 1) * 3;
            for (int k = used; k < ncoef; k++) dsh[k] = 0.f;
        } else {
            float dtmp[48];  // dL/dsh discarded (compact multi-view mode); only the direction term is kept
            dm = dm + sh_backward_dispatch(p.D, shp, mean - campos, dRGB, dtmp);
        }
    }
    if (p.dL_dmeans3D) {
        p.dL_dmeans3D[3 * i] = dm.x;
        p.dL_dmeans3D[3 * i + 1] = dm.y;
        p.dL_dmeans3D[3 * i + 2] = dm.z;
    }
    // ---- cov3D backward ----
    if (!p.cov3D_precomp && (p.dL_dscales || p.dL_drot)) {
        float3 dsc;
        float4 dr;
        cov3d_backward(scale, p.scale_modifier, rot, dcov, dsc, dr);
        if (p.dL_dscales) { p.dL_dscales[3 * i] = dsc.x; p.dL_dscales[3 * i + 1] = dsc.y; p.dL_dscales[3 * i + 2] = dsc.z; }
        if (p.dL_drot) { p.dL_drot[4 * i] = dr.x; p.dL_drot[4 * i + 1] = dr.y; p.dL_drot[4 * i + 2] = dr.z; p.dL_drot[4 * i + 3] = dr.w; }
    } else {
        if (p.dL_dscales) { p.dL_dscales[3 * i] = 0.f; p.dL_dscales[3 * i + 1] = 0.f; p.dL_dscales[3 * i + 2] = 0.f; }
        if (p.dL_drot)
            for (int k = 0; k < 4; k++) p.dL_drot[4 * i + k] = 0.f;
    }
}

void launch_preprocess_bwd(hipStream_t s, const PreprocessBwdParams &p) {
    if (p.P <= 0) return;
    preprocess_bwd_kernel<<<div_up(p.P, 256), 256, 0, s>>>(p);
}

}  // namespace gsr
