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
    const float mx = means3D[3 * ii], my = means3D[3 * ii + 1], mz = means3D[3 * ii + 2];
    const int c = ii / L, g0 = c * L, Lc = min(L, P - g0);
    const float *dchunk = dc + (size_t)g0 * V * 3 + (size_t)(ii - g0) * 3;
    float acc[3 * NB];
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
            acc[3 * k] += basis[k] * r;
            acc[3 * k + 1] += basis[k] * g;
            acc[3 * k + 2] += basis[k] * b;
        }
    }
    if constexpr (STAGED) {
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        float *sw = s_row[w];
        const size_t gbase = ((size_t)blockIdx.x * 256 + (size_t)w * 64) * 48, gend = (size_t)P * 48;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            wave_lds_sync();
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

void launch_sh_backward_views(hipStream_t s, int P, int D, int M, int V, int chunk_len, const float *means3D,
                              const float *campos, const float *dcolors_sh, float *dsh) {
    if (P <= 0) return;
    const dim3 grid(div_up(P, 256)), block(256);
    const bool staged = M == 16 && (((uintptr_t)dsh) & 15) == 0 && tuning("views_staged", 1);
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
