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
    adam_update(p, g, m, v, b1c, b2, b2c, step_size, bc2_sqrt, eps);  // gsr_kernels.h
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

// SparseGaussianAdam.step(visibility, N) of the upstream rasterizer package (the optimizer the reference's
// third_party GaussianModel takes with optimizer_type "sparse_adam", gaussian_model.py:26,194-196): only the
// elements of Gaussians with visibility set are updated, with the upstream kernel's arithmetic -- fixed betas, no
// bias correction, the step state never advanced:
//     m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;  p += -lr m / (sqrt(v) + eps)
// Same slice layout as adam_kernel; a thread's 4 elements may straddle Gaussians (M = 1, 3, 4, 45 ...), so each
// element takes its own visibility byte, and a thread whose 4 elements are all invisible loads nothing else.
__device__ __forceinline__ void sparse_adam_one(float &p, float g, float &m, float &v, float b1, float b1c, float b2,
                                                float b2c, float lr, float eps) {
    m = b1 * m + b1c * g;
    v = b2 * v + b2c * g * g;
    p += -lr * m / (sqrtf(v) + eps);
}

__global__ __launch_bounds__(256) void sparse_adam_kernel(AdamLaunch L) {
    int gi = 0;
#pragma unroll 1
    while (gi + 1 < L.num_groups && (int64_t)blockIdx.x >= L.slice_start[gi + 1]) gi++;
    const AdamGroupDev &G = L.g[gi];
    const int64_t e0 = ((int64_t)blockIdx.x - L.slice_start[gi]) * ADAM_SLICE + (int64_t)threadIdx.x * ADAM_PER;
    if (e0 >= G.n) return;
    const int64_t e1 = min(G.n, e0 + ADAM_PER);
    bool vis[ADAM_PER];
    bool any = false;
#pragma unroll
    for (int k = 0; k < ADAM_PER; k++) {
        vis[k] = e0 + k < e1 && L.visible[(e0 + k) / G.M] != 0;
        any |= vis[k];
    }
    if (!any) return;
    const float b1 = L.beta1, b1c = L.one_minus_beta1, b2 = L.beta2, b2c = L.one_minus_beta2, eps = L.eps, lr = G.lr;
    if (G.vec4 && e1 - e0 == ADAM_PER) {
        float4 p = *reinterpret_cast<const float4 *>(G.param + e0);
        const float4 g = *reinterpret_cast<const float4 *>(G.grad + e0);
        float4 m = *reinterpret_cast<const float4 *>(G.exp_avg + e0);
        float4 v = *reinterpret_cast<const float4 *>(G.exp_avg_sq + e0);
        float pa[4] = {p.x, p.y, p.z, p.w}, ga[4] = {g.x, g.y, g.z, g.w}, ma[4] = {m.x, m.y, m.z, m.w},
              va[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            float pk = pa[k], mk = ma[k], vk = va[k];
            sparse_adam_one(pk, ga[k], mk, vk, b1, b1c, b2, b2c, lr, eps);
            if (vis[k]) { pa[k] = pk; ma[k] = mk; va[k] = vk; }
        }
        *reinterpret_cast<float4 *>(G.param + e0) = make_float4(pa[0], pa[1], pa[2], pa[3]);
        *reinterpret_cast<float4 *>(G.exp_avg + e0) = make_float4(ma[0], ma[1], ma[2], ma[3]);
        *reinterpret_cast<float4 *>(G.exp_avg_sq + e0) = make_float4(va[0], va[1], va[2], va[3]);
    } else {
        for (int64_t e = e0; e < e1; e++) {
            if (!vis[e - e0]) continue;
            float p = G.param[e], m = G.exp_avg[e], v = G.exp_avg_sq[e];
            sparse_adam_one(p, G.grad[e], m, v, b1, b1c, b2, b2c, lr, eps);
            G.param[e] = p;
            G.exp_avg[e] = m;
            G.exp_avg_sq[e] = v;
        }
    }
}

void launch_sparse_adam(hipStream_t s, const AdamLaunch &L, int64_t total_slices) {
    if (total_slices <= 0) return;
    sparse_adam_kernel<<<(unsigned)total_slices, 256, 0, s>>>(L);
}

// Parameter activations of the reference's GaussianModel in front of the rasterizer (gaussian_model.py: get_scaling
// = exp, get_opacity = sigmoid, get_rotation = torch.nn.functional.normalize with eps 1e-12), forward and the chain
// rule back to the raw parameters, one thread per Gaussian.  torch runs these as ~15 elementwise kernels per step
// (forward + autograd); here two launches, HBM-bound: 64 B/Gaussian forward, 112 B/Gaussian backward.
constexpr float NORMALIZE_EPS = 1e-12f;

__global__ __launch_bounds__(256) void activations_forward_kernel(ActivationArgs A) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.N) return;
#pragma unroll
    for (int k = 0; k < 3; k++) A.scales[3 * i + k] = expf(A.scaling[3 * i + k]);
    A.opacities[i] = 1.0f / (1.0f + expf(-A.opacity[i]));
    const float4 q = *reinterpret_cast<const float4 *>(A.rotation + 4 * i);
    const float n = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), NORMALIZE_EPS);
    *reinterpret_cast<float4 *>(A.rotations + 4 * i) = make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
}

__global__ __launch_bounds__(256) void activations_backward_kernel(ActivationArgs A) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.N) return;
#pragma unroll
    for (int k = 0; k < 3; k++) A.dL_dscaling[3 * i + k] = A.dL_dscales[3 * i + k] * A.scales[3 * i + k];
    const float o = A.opacities[i];
    A.dL_dopacity[i] = A.dL_dopacities[i] * (1.0f - o) * o;  // torch's sigmoid_backward: g * (1 - y) * y
    const float4 q = *reinterpret_cast<const float4 *>(A.rotation + 4 * i);
    const float4 u = *reinterpret_cast<const float4 *>(A.rotations + 4 * i);
    const float4 g = *reinterpret_cast<const float4 *>(A.dL_drotations + 4 * i);
    const float nr = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    float4 d;
    if (nr > NORMALIZE_EPS) {  // d(q / |q|) = (g - u (u . g)) / |q|
        const float ug = u.x * g.x + u.y * g.y + u.z * g.z + u.w * g.w;
        d = make_float4((g.x - u.x * ug) / nr, (g.y - u.y * ug) / nr, (g.z - u.z * ug) / nr, (g.w - u.w * ug) / nr);
    } else {                   // clamped norm: q / eps is linear in q
        d = make_float4(g.x / NORMALIZE_EPS, g.y / NORMALIZE_EPS, g.z / NORMALIZE_EPS, g.w / NORMALIZE_EPS);
    }
    *reinterpret_cast<float4 *>(A.dL_drotation + 4 * i) = d;
}

void launch_activations_forward(hipStream_t s, const ActivationArgs &A) {
    if (A.N > 0) activations_forward_kernel<<<(unsigned)((A.N + 255) / 256), 256, 0, s>>>(A);
}

void launch_activations_backward(hipStream_t s, const ActivationArgs &A) {
    if (A.N > 0) activations_backward_kernel<<<(unsigned)((A.N + 255) / 256), 256, 0, s>>>(A);
}

int64_t adam_slices(int64_t n) { return (n + ADAM_SLICE - 1) / ADAM_SLICE; }

void launch_adam(hipStream_t s, const AdamLaunch &L, int64_t total_slices) {
    if (total_slices <= 0) return;
    adam_kernel<<<(unsigned)total_slices, 256, 0, s>>>(L);
}

}  // namespace gsr
