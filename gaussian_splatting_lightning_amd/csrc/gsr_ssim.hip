// gsr_ssim.hip -- fused SSIM loss (forward + backward) for the training step.
//
// Replaces the `fused_ssim(img1, img2, padding="same", train=True)` CUDA extension the reference imports
// (gs_lightning_module.py:10, used as 1 - fused_ssim(render, gt) at :100,279; submodule
// rahul-goel/fused-ssim, empty in the snapshot -- SURVEY.md §8(f) "next" #1).  SSIM of Wang et al. 2004 with
// an 11x11 Gaussian window (sigma 1.5), C1 = 0.01^2, C2 = 0.03^2, zero-padded "same" convolution, mean over
// the map (or over the map cropped by 5 px for padding="valid").
//
// One workgroup computes a 64x16 output tile of one (image, channel) plane: the 74x26 input window of both
// images is staged in LDS, the five moment images (x, y, x^2, y^2, xy) are filtered horizontally into LDS and
// then vertically, each thread sliding an 8-wide (horizontal) or 4-tall (vertical) window of outputs through
// registers so every staged value is read from LDS about twice instead of 11 times (forward).  The forward writes the
// three per-pixel partial derivatives the backward needs and one partial sum of the SSIM map per workgroup
// (summed on the caller's stream by torch; no cross-XCD atomics).  The backward filters the three derivative maps (scaled by
// dL/dmean) the same way and combines them with x and y:
//     dL/dx = G*(g dm/dmu1) + 2 x G*(g dm/dsigma1^2) + y G*(g dm/dsigma12).
#include "gsr_kernels.h"

namespace gsr {

constexpr int SS_TW = 64, SS_TH = 16, SS_R = 5, SS_K = 11;
constexpr int SS_IW = SS_TW + 2 * SS_R, SS_IH = SS_TH + 2 * SS_R;  // 74 x 26 input window
constexpr int SS_HSEG = 8;                                          // horizontal outputs per thread
constexpr int SS_VSEG = 4;                                          // vertical outputs per thread
constexpr float SS_C1 = 0.01f * 0.01f, SS_C2 = 0.03f * 0.03f;

struct SsimWindow {
    float w[SS_K];
};

__device__ __forceinline__ bool ssim_counted(int x, int y, int W, int H, int valid) {
    return !valid || (x >= SS_R && x < W - SS_R && y >= SS_R && y < H - SS_R);
}

// Horizontal 11-tap filter of NQ quantities over SS_HSEG consecutive outputs per thread: the 18 inputs of a
// segment are read from LDS once and slid in registers (LDS reads per output ~2.25 instead of 11).
// Thread t < SS_IH * (SS_TW / SS_HSEG) handles row t / 8, outputs (t % 8) * 8 .. +7.
template <int NQ, typename F>
__device__ __forceinline__ void ssim_hpass(int tid, const SsimWindow &win, F load, float (*out)[SS_IH][SS_TW + 1]) {
    constexpr int SEGS = SS_TW / SS_HSEG;
    if (tid >= SS_IH * SEGS) return;
    const int r = tid / SEGS, c0 = (tid % SEGS) * SS_HSEG;
    float in[NQ][SS_HSEG + SS_K - 1];
#pragma unroll
    for (int j = 0; j < SS_HSEG + SS_K - 1; j++) load(r, c0 + j, in, j);
#pragma unroll
    for (int o = 0; o < SS_HSEG; o++) {
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < SS_K; k++) acc = fmaf(win.w[k], in[q][o + k], acc);
            out[q][r][c0 + o] = acc;
        }
    }
}

__global__ __launch_bounds__(256) void ssim_fwd_kernel(int H, int W, int tiles_x, const float *__restrict__ img1,
                                                       const float *__restrict__ img2, int valid, SsimWindow win,
                                                       float *__restrict__ partial, float *__restrict__ d_mu1,
                                                       float *__restrict__ d_s11, float *__restrict__ d_s12) {
    __shared__ float s_x[SS_IH][SS_IW + 1], s_y[SS_IH][SS_IW + 1];
    __shared__ float s_h[5][SS_IH][SS_TW + 1];
    __shared__ float s_red[4];
    const int plane = blockIdx.y;
    const int tx0 = (blockIdx.x % tiles_x) * SS_TW, ty0 = (blockIdx.x / tiles_x) * SS_TH;
    const size_t base = (size_t)plane * H * W;
    const int tid = threadIdx.x;
    for (int i = tid; i < SS_IH * SS_IW; i += 256) {
        const int r = i / SS_IW, c = i % SS_IW;
        const int gx = tx0 - SS_R + c, gy = ty0 - SS_R + r;
        const bool in = gx >= 0 && gx < W && gy >= 0 && gy < H;
        s_x[r][c] = in ? img1[base + (size_t)gy * W + gx] : 0.f;
        s_y[r][c] = in ? img2[base + (size_t)gy * W + gx] : 0.f;
    }
    __syncthreads();
    ssim_hpass<5>(tid, win,
                  [&](int r, int c, float (&in)[5][SS_HSEG + SS_K - 1], int j) {
                      const float x = s_x[r][c], y = s_y[r][c];
                      in[0][j] = x;
                      in[1][j] = y;
                      in[2][j] = x * x;
                      in[3][j] = y * y;
                      in[4][j] = x * y;
                  },
                  s_h);
    __syncthreads();
    // vertical: thread = (column, 4-row segment); 14 rows of 5 quantities slide through registers
    const int c = tid & (SS_TW - 1), r0 = (tid / SS_TW) * SS_VSEG;
    float acc = 0.f;
    float v[5][SS_VSEG + SS_K - 1];
#pragma unroll
    for (int j = 0; j < SS_VSEG + SS_K - 1; j++)
#pragma unroll
        for (int q = 0; q < 5; q++) v[q][j] = s_h[q][r0 + j][c];
#pragma unroll
    for (int o = 0; o < SS_VSEG; o++) {
        const int gx = tx0 + c, gy = ty0 + r0 + o;
        float m[5];
#pragma unroll
        for (int q = 0; q < 5; q++) {
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < SS_K; k++) a = fmaf(win.w[k], v[q][o + k], a);
            m[q] = a;
        }
        if (gx >= W || gy >= H) continue;
        const float m1 = m[0], m2 = m[1];
        const float s11 = m[2] - m1 * m1, s22 = m[3] - m2 * m2, s12 = m[4] - m1 * m2;
        const float A = 2.f * m1 * m2 + SS_C1, B = 2.f * s12 + SS_C2;
        const float Cc = m1 * m1 + m2 * m2 + SS_C1, D = s11 + s22 + SS_C2;
        const float inv_cd = 1.f / (Cc * D);
        const float map = A * B * inv_cd;
        if (ssim_counted(gx, gy, W, H, valid)) acc += map;
        if (d_mu1) {
            const size_t pid = base + (size_t)gy * W + gx;
            const float dm_ds12 = 2.f * A * inv_cd;
            const float dm_ds11 = -map / D;
            const float dm_dmu1_s = 2.f * m2 * B * inv_cd - 2.f * m1 * map / Cc;
            d_mu1[pid] = dm_dmu1_s - 2.f * m1 * dm_ds11 - m2 * dm_ds12;
            d_s11[pid] = dm_ds11;
            d_s12[pid] = dm_ds12;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((tid & 63) == 0) s_red[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0)
        partial[(size_t)plane * gridDim.x + blockIdx.x] = ((s_red[0] + s_red[1]) + s_red[2]) + s_red[3];
}

// Backward: 32x16 output tiles with per-output LDS reads (measured faster than the sliding windows here).
constexpr int SB_TW = 32, SB_IW = SB_TW + 2 * SS_R;
__global__ __launch_bounds__(256) void ssim_bwd_kernel(int H, int W, int tiles_x, const float *__restrict__ img1,
                                                       const float *__restrict__ img2, int valid, SsimWindow win,
                                                       const float *__restrict__ dL_dmean, float inv_n,
                                                       const float *__restrict__ d_mu1,
                                                       const float *__restrict__ d_s11,
                                                       const float *__restrict__ d_s12, float *__restrict__ dL_dimg1) {
    __shared__ float s_in[3][SS_IH][SB_IW + 1];
    __shared__ float s_h[3][SS_IH][SB_TW + 1];
    const int plane = blockIdx.y;
    const int tx0 = (blockIdx.x % tiles_x) * SB_TW, ty0 = (blockIdx.x / tiles_x) * SS_TH;
    const size_t base = (size_t)plane * H * W;
    const int tid = threadIdx.x;
    const float g = dL_dmean[0] * inv_n;  // dL/dmap at every counted pixel
    for (int i = tid; i < SS_IH * SB_IW; i += 256) {
        const int r = i / SB_IW, c = i % SB_IW;
        const int gx = tx0 - SS_R + c, gy = ty0 - SS_R + r;
        const bool in = gx >= 0 && gx < W && gy >= 0 && gy < H && ssim_counted(gx, gy, W, H, valid);
        const size_t pid = base + (size_t)gy * W + gx;
        s_in[0][r][c] = in ? g * d_mu1[pid] : 0.f;
        s_in[1][r][c] = in ? g * d_s11[pid] : 0.f;
        s_in[2][r][c] = in ? g * d_s12[pid] : 0.f;
    }
    __syncthreads();
    for (int i = tid; i < SS_IH * SB_TW; i += 256) {
        const int r = i / SB_TW, c = i % SB_TW;
        float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
        for (int k = 0; k < SS_K; k++) {
            const float wk = win.w[k];
            a = fmaf(wk, s_in[0][r][c + k], a);
            b = fmaf(wk, s_in[1][r][c + k], b);
            d = fmaf(wk, s_in[2][r][c + k], d);
        }
        s_h[0][r][c] = a;
        s_h[1][r][c] = b;
        s_h[2][r][c] = d;
    }
    __syncthreads();
    const int c = tid & 31;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int r = (tid >> 5) + 8 * h;
        const int gx = tx0 + c, gy = ty0 + r;
        float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
        for (int k = 0; k < SS_K; k++) {
            const float wk = win.w[k];
            a = fmaf(wk, s_h[0][r + k][c], a);
            b = fmaf(wk, s_h[1][r + k][c], b);
            d = fmaf(wk, s_h[2][r + k][c], d);
        }
        if (gx >= W || gy >= H) continue;
        const size_t pid = base + (size_t)gy * W + gx;
        dL_dimg1[pid] = a + 2.f * img1[pid] * b + img2[pid] * d;
    }
}

// ------------------------------------------------------------------------------------------------
// Streaming forward: one wave owns a 64-column strip of SX_CH output rows of one plane and walks its input rows
// (SX_CH + 10 of them) top to bottom once.  Each row is loaded with coalesced 64-lane loads (plus the 10 halo
// columns), staged in a 74-float LDS row, filtered horizontally per lane (11 taps, the same FMA order as the tiled
// kernels), and pushed into a 12-slot ring of horizontal results held in registers; once 11 rows are in, the lane
// filters its column vertically (11 taps, same order) and finishes the output row.  Loads run SX_PF rows ahead.
// No block barriers and a ~1 KB LDS footprint per wave, where the tiled kernels staged 26-row windows (62 % of the
// rows twice) in 49 KB per workgroup (3 per CU).  Outputs are bitwise those of the tiled kernels (same sums in the
// same order); the forward's partial sums are grouped per strip.
// ------------------------------------------------------------------------------------------------
constexpr int SX_CH = 32, SX_RING = 12, SX_PF = 4, SX_IW = 64 + 2 * SS_R;
static_assert(SX_RING % SX_PF == 0, "prefetch slots cycle with the ring unroll");

__device__ __forceinline__ float sx_load(const float *__restrict__ img, size_t base, int H, int W, int gy, int gx) {
    return (gy >= 0 && gy < H && gx >= 0 && gx < W) ? img[base + (size_t)gy * W + gx] : 0.f;
}

__global__ __launch_bounds__(64) void ssim_fwd_stream_kernel(int H, int W, const float *__restrict__ img1,
                                                             const float *__restrict__ img2, int valid,
                                                             SsimWindow win, float *__restrict__ partial,
                                                             float *__restrict__ d_mu1, float *__restrict__ d_s11,
                                                             float *__restrict__ d_s12) {
    __shared__ float s_x[SX_IW], s_y[SX_IW];
    const int lane = threadIdx.x;
    const int c0 = blockIdx.x * 64, r0 = blockIdx.y * SX_CH, plane = blockIdx.z;
    const size_t base = (size_t)plane * H * W;
    const int nrows = SX_CH + 2 * SS_R;
    const int gx0 = c0 - SS_R + lane, gx1 = c0 + 64 - SS_R + lane;  // lane's column and (lanes < 10) halo column
    float pf[SX_PF][4];
#pragma unroll
    for (int q = 0; q < SX_PF; q++) {
        const int gy = r0 - SS_R + q;
        pf[q][0] = sx_load(img1, base, H, W, gy, gx0);
        pf[q][1] = sx_load(img2, base, H, W, gy, gx0);
        pf[q][2] = lane < 2 * SS_R ? sx_load(img1, base, H, W, gy, gx1) : 0.f;
        pf[q][3] = lane < 2 * SS_R ? sx_load(img2, base, H, W, gy, gx1) : 0.f;
    }
    float ring[5][SX_RING];
    float acc = 0.f;
    const int gx = c0 + lane;
    for (int i0 = 0; i0 < nrows; i0 += SX_RING) {
#pragma unroll
        for (int u = 0; u < SX_RING; u++) {
            const int i = i0 + u;
            if (i >= nrows) break;  // uniform
            const int slot = u % SX_PF;
            s_x[lane] = pf[slot][0];
            s_y[lane] = pf[slot][1];
            if (lane < 2 * SS_R) {
                s_x[64 + lane] = pf[slot][2];
                s_y[64 + lane] = pf[slot][3];
            }
            if (i + SX_PF < nrows) {  // the row SX_PF ahead into the freed slot
                const int gy = r0 - SS_R + i + SX_PF;
                pf[slot][0] = sx_load(img1, base, H, W, gy, gx0);
                pf[slot][1] = sx_load(img2, base, H, W, gy, gx0);
                pf[slot][2] = lane < 2 * SS_R ? sx_load(img1, base, H, W, gy, gx1) : 0.f;
                pf[slot][3] = lane < 2 * SS_R ? sx_load(img2, base, H, W, gy, gx1) : 0.f;
            }
            wave_lds_sync();
            float h[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < SS_K; k++) {
                const float x = s_x[lane + k], y = s_y[lane + k];
                h[0] = fmaf(win.w[k], x, h[0]);
                h[1] = fmaf(win.w[k], y, h[1]);
                h[2] = fmaf(win.w[k], x * x, h[2]);
                h[3] = fmaf(win.w[k], y * y, h[3]);
                h[4] = fmaf(win.w[k], x * y, h[4]);
            }
            wave_lds_sync();  // every lane has read the row before the next one is staged
#pragma unroll
            for (int q = 0; q < 5; q++) ring[q][u] = h[q];
            if (i < 2 * SS_R) continue;
            const int gy = r0 + i - 2 * SS_R;  // output row: ring rows i - 10 .. i
            float m[5];
#pragma unroll
            for (int q = 0; q < 5; q++) {
                float a = 0.f;
#pragma unroll
                for (int k = 0; k < SS_K; k++) a = fmaf(win.w[k], ring[q][(u + SX_RING - 2 * SS_R + k) % SX_RING], a);
                m[q] = a;
            }
            if (gx >= W || gy >= H) continue;
            const float m1 = m[0], m2 = m[1];
            const float s11 = m[2] - m1 * m1, s22 = m[3] - m2 * m2, s12 = m[4] - m1 * m2;
            const float A = 2.f * m1 * m2 + SS_C1, B = 2.f * s12 + SS_C2;
            const float Cc = m1 * m1 + m2 * m2 + SS_C1, D = s11 + s22 + SS_C2;
            const float inv_cd = 1.f / (Cc * D);
            const float map = A * B * inv_cd;
            if (ssim_counted(gx, gy, W, H, valid)) acc += map;
            if (d_mu1) {
                const size_t pid = base + (size_t)gy * W + gx;
                const float dm_ds12 = 2.f * A * inv_cd;
                const float dm_ds11 = -map / D;
                const float dm_dmu1_s = 2.f * m2 * B * inv_cd - 2.f * m1 * map / Cc;
                d_mu1[pid] = dm_dmu1_s - 2.f * m1 * dm_ds11 - m2 * dm_ds12;
                d_s11[pid] = dm_ds11;
                d_s12[pid] = dm_ds12;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) partial[((size_t)plane * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = acc;
}

// "ssim_stream" 1 (default): the streaming forward (1080p x 3: 59-68 us against 86 for the tiled kernel).  A streaming
// backward of the same shape measured 92 us against the tiled backward's 72 (its per-row LDS round trips at 5 waves
// per SIMD cost more than the tiled kernel's halo re-reads) and was removed.
static bool ssim_stream_fwd() { return tuning("ssim_stream", 1) != 0; }

static SsimWindow ssim_window() {
    SsimWindow w;
    double g[SS_K], sum = 0.0;
    for (int k = 0; k < SS_K; k++) {
        const double d = k - SS_R;
        g[k] = exp(-d * d / (2.0 * 1.5 * 1.5));
        sum += g[k];
    }
    for (int k = 0; k < SS_K; k++) w.w[k] = (float)(g[k] / sum);
    return w;
}

size_t ssim_num_partials(int planes, int H, int W) {
    if (ssim_stream_fwd()) return (size_t)planes * div_up(W, 64) * div_up(H, SX_CH);
    return (size_t)planes * div_up(W, SS_TW) * div_up(H, SS_TH);
}

void launch_ssim_forward(hipStream_t s, int planes, int H, int W, const float *img1, const float *img2, int valid,
                         float *partial, float *d_mu1, float *d_s11, float *d_s12) {
    if (ssim_stream_fwd()) {
        const dim3 grid(div_up(W, 64), div_up(H, SX_CH), planes), block(64);
        ssim_fwd_stream_kernel<<<grid, block, 0, s>>>(H, W, img1, img2, valid, ssim_window(), partial, d_mu1, d_s11,
                                                      d_s12);
        return;
    }
    const int tiles_x = div_up(W, SS_TW), tiles = tiles_x * div_up(H, SS_TH);
    const dim3 grid(tiles, planes), block(256);
    ssim_fwd_kernel<<<grid, block, 0, s>>>(H, W, tiles_x, img1, img2, valid, ssim_window(), partial, d_mu1, d_s11,
                                           d_s12);
}

void launch_ssim_backward(hipStream_t s, int planes, int H, int W, const float *img1, const float *img2, int valid,
                          const float *dL_dmean, float inv_n, const float *d_mu1, const float *d_s11,
                          const float *d_s12, float *dL_dimg1) {
    const int tiles_x = div_up(W, SB_TW), tiles = tiles_x * div_up(H, SS_TH);
    const dim3 grid(tiles, planes), block(256);
    ssim_bwd_kernel<<<grid, block, 0, s>>>(H, W, tiles_x, img1, img2, valid, ssim_window(), dL_dmean, inv_n, d_mu1,
                                           d_s11, d_s12, dL_dimg1);
}

}  // namespace gsr
