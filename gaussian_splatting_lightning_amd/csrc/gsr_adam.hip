// gsr_adam.hip -- fused Adam step over all Gaussian parameter groups in one launch.
//
// The reference trains with torch.optim.Adam(eps=1e-15) over six parameter groups (xyz, features_dc,
// features_rest, opacity, scaling, rotation; gs_lightning_module.py:114-134, configs/train_gs.yaml:20-25);
// torch runs that as ~10 foreach kernels per group.  Here one launch updates every group: each workgroup
// owns a slice of one group (group boundaries are rounded to workgroup slices), each thread updates 4
// consecutive elements with float4 accesses when the group's arrays are 16-B aligned.  Per element the
// arithmetic follows torch's Adam (non-amsgrad, no weight decay):
//     m = lerp(m, g, 1 - b1);  v = v * b2 + (1 - b2) g^2;  p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps)
// with step_size = lr / bc1 and sqrt(bc2) formed on the host in double, as torch does with Python floats.
// HBM-bound: 16 B read + 12 B written per element (param, grad, two moments).
#include "gsr_kernels.h"

namespace gsr {

constexpr int ADAM_PER = 4;                   // elements per thread
constexpr int ADAM_SLICE = 256 * ADAM_PER;    // elements per workgroup

__device__ __forceinline__ void adam_one(float &p, float g, float &m, float &v, float b1c, float b2, float b2c,
                                         float step_size, float bc2_sqrt, float eps) {
    m = m + b1c * (g - m);            // exp_avg.lerp_(grad, 1 - beta1)   (weight < 0.5 branch of lerp)
    v = v * b2 + b2c * (g * g);       // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p + (-step_size) * (m / denom);  // param.addcdiv_(exp_avg, denom, value=-step_size)
}

__global__ __launch_bounds__(256) void adam_kernel(AdamLaunch L) {
    // group of this workgroup: slices are laid out group after group
    int gi = 0;
#pragma unroll 1
    while (gi + 1 < L.num_groups && (int64_t)blockIdx.x >= L.slice_start[gi + 1]) gi++;
    const AdamGroupDev &G = L.g[gi];
    const int64_t e0 = ((int64_t)blockIdx.x - L.slice_start[gi]) * ADAM_SLICE + (int64_t)threadIdx.x * ADAM_PER;
    if (e0 >= G.n) return;
    const float b1c = L.one_minus_beta1, b2 = L.beta2, b2c = L.one_minus_beta2, eps = L.eps;
    const float ss = G.step_size, bs = G.bc2_sqrt;
    if (G.vec4 && e0 + ADAM_PER <= G.n) {
        float4 p = *reinterpret_cast<const float4 *>(G.param + e0);
        const float4 g = *reinterpret_cast<const float4 *>(G.grad + e0);
        float4 m = *reinterpret_cast<const float4 *>(G.exp_avg + e0);
        float4 v = *reinterpret_cast<const float4 *>(G.exp_avg_sq + e0);
        adam_one(p.x, g.x, m.x, v.x, b1c, b2, b2c, ss, bs, eps);
        adam_one(p.y, g.y, m.y, v.y, b1c, b2, b2c, ss, bs, eps);
        adam_one(p.z, g.z, m.z, v.z, b1c, b2, b2c, ss, bs, eps);
        adam_one(p.w, g.w, m.w, v.w, b1c, b2, b2c, ss, bs, eps);
        *reinterpret_cast<float4 *>(G.param + e0) = p;
        *reinterpret_cast<float4 *>(G.exp_avg + e0) = m;
        *reinterpret_cast<float4 *>(G.exp_avg_sq + e0) = v;
    } else {
        for (int64_t e = e0; e < min(G.n, e0 + ADAM_PER); e++) {
            float p = G.param[e], m = G.exp_avg[e], v = G.exp_avg_sq[e];
            adam_one(p, G.grad[e], m, v, b1c, b2, b2c, ss, bs, eps);
            G.param[e] = p;
            G.exp_avg[e] = m;
            G.exp_avg_sq[e] = v;
        }
    }
}

int64_t adam_slices(int64_t n) { return (n + ADAM_SLICE - 1) / ADAM_SLICE; }

void launch_adam(hipStream_t s, const AdamLaunch &L, int64_t total_slices) {
    if (total_slices <= 0) return;
    adam_kernel<<<(unsigned)total_slices, 256, 0, s>>>(L);
}

}  // namespace gsr
