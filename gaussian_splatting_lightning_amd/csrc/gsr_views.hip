// gsr_views.hip -- multi-view SH gradient from compact per-view colour-gradient factors.
//
// Data-parallel training renders one view per GPU.  The SH coefficient gradient of view v is rank one per
// Gaussian: dL/dsh_v[g] = basis(dir_v(g)) (x) dRGB_v[g] (computeColorFromSH backward of the CUDA submodule),
// so instead of all-reducing (P, 16, 3) floats, ranks all-gather the (P, 3) factors dRGB_v and every rank
// expands the sum over views here.  One thread per Gaussian; the per-view camera positions are wave-uniform
// (scalar loads); 48 accumulators stay in VGPRs; the 192-B output row is written with float4 stores.
#include "gsr_kernels.h"
#include "gsr_sh.h"

namespace gsr {

// M = 16 with a 16-B aligned output (STAGED): each half-wave's 32 rows are staged in LDS at a 52-float stride (as
// preprocess_bwd's dL/dsh) and the wave stores them as coalesced float4s, not 12 stores per lane 192 B apart.
constexpr int VIEWS_STRIDE = 52;
// The factors are laid out chunk-major (the multi-view exchange gathers them per Gaussian chunk): chunk c holds
// Gaussians [c L, min(P, (c+1) L)) as a (V, L_c, 3) block at offset c V L 3; L >= P is the plain (V, P, 3) array.
// Gaussian ii's expanded gradient row, in registers (shared by the expansion and the fused SH Adam, so the two
// produce the same bits).
template <int DEG>
__device__ __forceinline__ void views_accumulate(int ii, int P, int V, int L, const float *__restrict__ means3D,
                                                 const float *__restrict__ campos, const float *__restrict__ dc,
                                                 float (&acc)[3 * (DEG + 1) * (DEG + 1)]) {
#pragma clang fp contract(off)  // explicit FMAs only: the same bits wherever this is inlined
    constexpr int NB = (DEG + 1) * (DEG + 1);
    const float mx = means3D[3 * ii], my = means3D[3 * ii + 1], mz = means3D[3 * ii + 2];
    const int c = ii / L, g0 = c * L, Lc = min(L, P - g0);
    const float *dchunk = dc + (size_t)g0 * V * 3 + (size_t)(ii - g0) * 3;
#pragma unroll
    for (int k = 0; k < 3 * NB; k++) acc[k] = 0.f;
    for (int v = 0; v < V; v++) {
        const float *d = dchunk + (size_t)v * Lc * 3;
        const float r = d[0], g = d[1], b = d[2];
        if (r == 0.f && g == 0.f && b == 0.f) continue;  // not rendered (or fully clamped) in view v
        const float dx = mx - campos[3 * v], dy = my - campos[3 * v + 1], dz = mz - campos[3 * v + 2];
        const float len = sqrtf(dx * dx + dy * dy + dz * dz);
        float basis[16];
        sh_basis<DEG>(dx / len, dy / len, dz / len, basis);
#pragma unroll
        for (int k = 0; k < NB; k++) {
            acc[3 * k] = __fmaf_rn(basis[k], r, acc[3 * k]);
            acc[3 * k + 1] = __fmaf_rn(basis[k], g, acc[3 * k + 1]);
            acc[3 * k + 2] = __fmaf_rn(basis[k], b, acc[3 * k + 2]);
        }
    }
}

// One half-wave's 32 gradient rows (48 floats, zero beyond the active degree's coefficients) into LDS at a
// VIEWS_STRIDE-float stride.
template <int NB>
__device__ __forceinline__ void stage_rows(float *sw, int lane, int h, const float (&acc)[3 * NB]) {
    if ((lane >> 5) == h) {
        float *r = sw + (lane & 31) * VIEWS_STRIDE;
#pragma unroll
        for (int k = 0; k < 12; k++)
            *reinterpret_cast<float4 *>(r + 4 * k) =
                make_float4(4 * k < 3 * NB ? acc[4 * k < 3 * NB ? 4 * k : 0] : 0.f,
                            4 * k + 1 < 3 * NB ? acc[4 * k + 1 < 3 * NB ? 4 * k + 1 : 0] : 0.f,
                            4 * k + 2 < 3 * NB ? acc[4 * k + 2 < 3 * NB ? 4 * k + 2 : 0] : 0.f,
                            4 * k + 3 < 3 * NB ? acc[4 * k + 3 < 3 * NB ? 4 * k + 3 : 0] : 0.f);
    }
}

template <int DEG, bool STAGED>
__global__ __launch_bounds__(256) void sh_backward_views_kernel(int P, int M, int V, int L,
                                                                const float *__restrict__ means3D,
                                                                const float *__restrict__ campos,
                                                                const float *__restrict__ dc,
                                                                float *__restrict__ dsh) {
    constexpr int NB = (DEG + 1) * (DEG + 1);
    __shared__ __attribute__((aligned(16))) float s_row[STAGED ? 4 : 1][STAGED ? 32 * VIEWS_STRIDE : 1];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (!STAGED && i >= P) return;
    const bool live = i < P;
    const int ii = live ? i : P - 1;
    float acc[3 * NB];
    views_accumulate<DEG>(ii, P, V, L, means3D, campos, dc, acc);
    if constexpr (STAGED) {
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        float *sw = s_row[w];
        const size_t gbase = ((size_t)blockIdx.x * 256 + (size_t)w * 64) * 48, gend = (size_t)P * 48;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            wave_lds_sync();
            stage_rows<NB>(sw, lane, h, acc);
            wave_lds_sync();
#pragma unroll
            for (int c = 0; c < 6; c++) {  // 32 rows x 48 floats = 384 float4, 6 per lane
                const uint32_t f = c * 256 + lane * 4;
                const size_t go = gbase + (size_t)h * 1536 + f;
                if (go < gend)
                    *reinterpret_cast<float4 *>(dsh + go) =
                        *reinterpret_cast<const float4 *>(sw + (f / 48) * VIEWS_STRIDE + f % 48);
            }
        }
        return;
    }
    float *o = dsh + (size_t)i * M * 3;
    if (M == 16 && (((uintptr_t)dsh) & 15) == 0) {
        float row[48];
#pragma unroll
        for (int k = 0; k < 48; k++) row[k] = k < 3 * NB ? acc[k < 3 * NB ? k : 0] : 0.f;
        float4 *o4 = reinterpret_cast<float4 *>(o);
#pragma unroll
        for (int k = 0; k < 12; k++) o4[k] = make_float4(row[4 * k], row[4 * k + 1], row[4 * k + 2], row[4 * k + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < 3 * NB; k++) o[k] = acc[k];
        for (int k = 3 * NB; k < 3 * M; k++) o[k] = 0.f;
    }
}

// Fused Adam step of the two SH parameter groups whose gradient is the multi-view expansion above: features_dc
// (P, 1, 3) holds coefficient 0 of each row, features_rest (P, M - 1, 3) coefficients 1..15 (M = 16).  The row is
// formed in registers exactly as sh_backward_views_kernel forms it, staged in LDS, and every lane then updates
// consecutive float4s of the half-wave's 32-row block of each group (coalesced param / moment traffic) with
// adam_update's arithmetic (gsr_kernels.h), so the result is bitwise that of the expansion followed by adam_kernel --
// without the
// 192-B gradient row written and read back.
__device__ __forceinline__ void adam_elem(float &p, float g, float &m, float &v, const AdamShGroup &G,
                                          const AdamShLaunch &L) {
    adam_update(p, g, m, v, L.one_minus_beta1, L.beta2, L.one_minus_beta2, G.step_size, G.bc2_sqrt, L.eps);
}

// The group's elements of this half-wave block: element e of the block is row e / W, coefficient column e % W + C0 of
// the staged row (W = 3 for features_dc, 45 for features_rest).  The moments are contiguous (row r's elements at
// r W); the parameter either too (param_stride == W) or rows of a joint (P, 16, 3) SH tensor (param_stride == 48,
// the pointer at the group's first column): then the parameter is read and written per element.
template <int W, int C0, bool PACKED>
__device__ __forceinline__ void adam_block(const AdamShGroup &G, const AdamShLaunch &L, const float *sw, int lane,
                                           int64_t r0, int64_t rows_end, bool vec4) {
    constexpr int N = 32 * W;
    const int64_t e0 = r0 * W, e_end = rows_end * W;
    // the block's parameter base, then 32-bit offsets within it
    float *const pb = G.param + (PACKED ? e0 : r0 * G.param_stride);
    const int ps = (int)G.param_stride;
    auto pidx = [&](int e) { return PACKED ? e : (e / W) * ps + e % W; };
    if (vec4 && e0 + N <= e_end) {
        // a whole block: each lane's loads (parameter, both moments) for SUB float4s are issued together, then the
        // updates and stores -- a load-update-store loop waited for each iteration's loads in turn (the stores may
        // alias them)
        constexpr int NQ = (N / 4 + 63) / 64, SUB = 3;
#pragma unroll
        for (int i0 = 0; i0 < NQ; i0 += SUB) {
            float4 Pv[SUB], Mv[SUB], Vv[SUB];
#pragma unroll
            for (int i = 0; i < SUB && i0 + i < NQ; i++) {
                const int e = 4 * (lane + 64 * (i0 + i));
                if (e >= N) continue;
                Mv[i] = *reinterpret_cast<const float4 *>(G.exp_avg + e0 + e);
                Vv[i] = *reinterpret_cast<const float4 *>(G.exp_avg_sq + e0 + e);
                if (PACKED)
                    Pv[i] = *reinterpret_cast<const float4 *>(pb + e);
                else
                    Pv[i] = make_float4(pb[pidx(e)], pb[pidx(e + 1)], pb[pidx(e + 2)], pb[pidx(e + 3)]);
            }
#pragma unroll
            for (int i = 0; i < SUB && i0 + i < NQ; i++) {
                const int e = 4 * (lane + 64 * (i0 + i));
                if (e >= N) continue;
                adam_elem(Pv[i].x, sw[(e / W) * VIEWS_STRIDE + e % W + C0], Mv[i].x, Vv[i].x, G, L);
                adam_elem(Pv[i].y, sw[((e + 1) / W) * VIEWS_STRIDE + (e + 1) % W + C0], Mv[i].y, Vv[i].y, G, L);
                adam_elem(Pv[i].z, sw[((e + 2) / W) * VIEWS_STRIDE + (e + 2) % W + C0], Mv[i].z, Vv[i].z, G, L);
                adam_elem(Pv[i].w, sw[((e + 3) / W) * VIEWS_STRIDE + (e + 3) % W + C0], Mv[i].w, Vv[i].w, G, L);
                if (PACKED) {
                    *reinterpret_cast<float4 *>(pb + e) = Pv[i];
                } else {
                    pb[pidx(e)] = Pv[i].x;
                    pb[pidx(e + 1)] = Pv[i].y;
                    pb[pidx(e + 2)] = Pv[i].z;
                    pb[pidx(e + 3)] = Pv[i].w;
                }
                *reinterpret_cast<float4 *>(G.exp_avg + e0 + e) = Mv[i];
                *reinterpret_cast<float4 *>(G.exp_avg_sq + e0 + e) = Vv[i];
            }
        }
        return;
    }
    for (int q = lane; 4 * q < N; q += 64) {  // the last, partial block (or unaligned arrays): element by element
        const int e = 4 * q;
        const int64_t ge = e0 + e;
        if (ge >= e_end) break;
        for (int j = 0; j < 4 && ge + j < e_end; j++) {
            const int pi = pidx(e + j);
            float p = pb[pi], m = G.exp_avg[ge + j], v = G.exp_avg_sq[ge + j];
            adam_elem(p, sw[((e + j) / W) * VIEWS_STRIDE + (e + j) % W + C0], m, v, G, L);
            pb[pi] = p;
            G.exp_avg[ge + j] = m;
            G.exp_avg_sq[ge + j] = v;
        }
    }
}

// Fully joint layout: parameter and both moments are (P, 16, 3) tensors whose [:, :1] / [:, 1:] blocks are the two
// groups, so a half-wave's 32 rows are ONE contiguous 384-float4 run of each array, read and written as coalesced
// float4s; an element's group (its step size) is its column < 3.
__device__ __forceinline__ void adam_block_joint(const AdamShLaunch &L, const float *sw, int lane, int64_t r0,
                                                 int64_t rows_end) {
    constexpr int N = 32 * 48, SUB = 3;
    const int64_t e0 = r0 * 48, e_end = rows_end * 48;
    float *const pb = L.dc_group.param + e0, *const mb = L.dc_group.exp_avg + e0, *const vb = L.dc_group.exp_avg_sq + e0;
    const bool whole = e0 + N <= e_end;
#pragma unroll
    for (int i0 = 0; i0 < 6; i0 += SUB) {
        float4 Pv[SUB], Mv[SUB], Vv[SUB];
#pragma unroll
        for (int i = 0; i < SUB; i++) {
            const int e = 4 * (lane + 64 * (i0 + i));
            if (!whole && e0 + e >= e_end) continue;  // rows are whole float4s: 48 = 12 x 4
            Pv[i] = *reinterpret_cast<const float4 *>(pb + e);
            Mv[i] = *reinterpret_cast<const float4 *>(mb + e);
            Vv[i] = *reinterpret_cast<const float4 *>(vb + e);
        }
#pragma unroll
        for (int i = 0; i < SUB; i++) {
            const int e = 4 * (lane + 64 * (i0 + i));
            if (!whole && e0 + e >= e_end) continue;
            const int row = e / 48, col = e - 48 * row;  // col % 4 == 0: at most col 0's float4 mixes the groups
            const float *g = sw + row * VIEWS_STRIDE + col;
            const AdamShGroup &G0 = col == 0 ? L.dc_group : L.rest_group;
            adam_elem(Pv[i].x, g[0], Mv[i].x, Vv[i].x, G0, L);
            adam_elem(Pv[i].y, g[1], Mv[i].y, Vv[i].y, G0, L);
            adam_elem(Pv[i].z, g[2], Mv[i].z, Vv[i].z, G0, L);
            adam_elem(Pv[i].w, g[3], Mv[i].w, Vv[i].w, L.rest_group, L);
            *reinterpret_cast<float4 *>(pb + e) = Pv[i];
            *reinterpret_cast<float4 *>(mb + e) = Mv[i];
            *reinterpret_cast<float4 *>(vb + e) = Vv[i];
        }
    }
}

// LAYOUT 0: packed groups (tensors of their own); 1: the parameter is one (P, 16, 3) tensor, the moments packed;
// 2: parameter and moments each one (P, 16, 3) tensor (adam_block_joint).
template <int DEG, int LAYOUT>
__global__ __launch_bounds__(256) void adam_sh_views_kernel(AdamShLaunch L) {
    constexpr int NB = (DEG + 1) * (DEG + 1);
    // the wave's 64 gradient rows all staged first (two half-wave stores), so the 48 accumulators are dead before the
    // Adam phase's batched loads start
    __shared__ __attribute__((aligned(16))) float s_row[4][64 * VIEWS_STRIDE];
    const int P = L.P;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int ii = i < P ? i : P - 1;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    {
        float acc[3 * NB];
        views_accumulate<DEG>(ii, P, L.V, L.L, L.means3D, L.campos, L.dc, acc);
        stage_rows<NB>(s_row[w], lane, 0, acc);
        stage_rows<NB>(s_row[w] + 32 * VIEWS_STRIDE, lane, 1, acc);
    }
    wave_lds_sync();
    const int64_t row0 = (int64_t)blockIdx.x * 256 + (int64_t)w * 64;
#pragma unroll 1
    for (int h = 0; h < 2; h++) {
        const float *sw = s_row[w] + 32 * VIEWS_STRIDE * h;
        const int64_t r = row0 + 32 * h;
        if (r >= P) break;
        if constexpr (LAYOUT == 2) {
            adam_block_joint(L, sw, lane, r, P);
        } else {
            adam_block<3, 0, LAYOUT == 0>(L.dc_group, L, sw, lane, r, P, L.vec4);
            adam_block<45, 3, LAYOUT == 0>(L.rest_group, L, sw, lane, r, P, L.vec4);
        }
    }
}

void launch_adam_sh_views(hipStream_t s, const AdamShLaunch &L, int D) {
    if (L.P <= 0) return;
    const dim3 grid(div_up(L.P, 256)), block(256);
    const int layout = L.joint ? 2 : L.dc_group.param_stride == 3 ? 0 : 1;
#define GSR_ADAM_SH(D_) (layout == 2 ? adam_sh_views_kernel<D_, 2><<<grid, block, 0, s>>>(L) \
                         : layout == 0 ? adam_sh_views_kernel<D_, 0><<<grid, block, 0, s>>>(L) \
                                       : adam_sh_views_kernel<D_, 1><<<grid, block, 0, s>>>(L))
    switch (D) {
        case 0: GSR_ADAM_SH(0); break;
        case 1: GSR_ADAM_SH(1); break;
        case 2: GSR_ADAM_SH(2); break;
        default: GSR_ADAM_SH(3); break;
    }
#undef GSR_ADAM_SH
}

void launch_sh_backward_views(hipStream_t s, int P, int D, int M, int V, int chunk_len, const float *means3D,
                              const float *campos, const float *dcolors_sh, float *dsh) {
    if (P <= 0) return;
    const dim3 grid(div_up(P, 256)), block(256);
    const bool staged = M == 16 && (((uintptr_t)dsh) & 15) == 0;
    const int L = chunk_len <= 0 || chunk_len > P ? P : chunk_len;
#define GSR_VIEWS(D_, S_) sh_backward_views_kernel<D_, S_><<<grid, block, 0, s>>>(P, M, V, L, means3D, campos, dcolors_sh, dsh)
    switch (D) {
        case 0: if (staged) GSR_VIEWS(0, true); else GSR_VIEWS(0, false); break;
        case 1: if (staged) GSR_VIEWS(1, true); else GSR_VIEWS(1, false); break;
        case 2: if (staged) GSR_VIEWS(2, true); else GSR_VIEWS(2, false); break;
        default: if (staged) GSR_VIEWS(3, true); else GSR_VIEWS(3, false); break;
    }
#undef GSR_VIEWS
}

}  // namespace gsr
