// gsr_densify.hip -- densify_and_prune as three small classification/scan launches plus one row-scatter launch.
//
// Follows gs_lightning/modules/gaussian_model.py:184-287 (densify_and_prune, _prune_gaussian, _clone_gaussian,
// _split_gaussian, _add_gaussian) together with the optimizer-state re-indexing of
// gs_lightning/lightning/gs_lightning_module.py:213-235 (update_optimizer_parameters):
//
//   keep   = sigmoid(opacity) > opacity_thr [&& max_radii2D < screensize_thr] [&& max(exp(scaling)) < size_thr]
//   grad   = xyz_grad_accum / xyz_grad_count (NaN -> 0);  bad = grad >= grad_thr
//   clone  = keep && bad && max(exp(scaling)) <  clone_thr     (appended as an exact copy)
//   split  = keep && bad && max(exp(scaling)) >= clone_thr     (moved by R(q) (z * exp(scaling)), scaling
//            becomes log(exp(scaling) / 1.6) in place, then appended as a copy of the moved row)
//
// Output rows: [kept rows in original order | clone copies in order | split copies in order].  Adam moments
// follow kept rows and are zero for appended rows; the densification statistics (kind STAT) follow kept rows
// and are zero for appended rows (_add_gaussian).  The host reads back the three counts between the
// classification and the scatter to size the outputs and to draw z ~ N(0, 1) with torch, so the split
// displacement is bit-identical to torch.normal(mean=0, std) (ATen draws normal_(0, 1) then mul_(std)).
#include "gsr_kernels.h"
#include "gsrast.h"

namespace gsr {

constexpr int DN_THREADS = 256;
constexpr int DN_PER = 4;                          // rows per thread
constexpr int DN_ROWS = DN_THREADS * DN_PER;       // rows per workgroup
constexpr int DN_SCAN_THREADS = 1024;
enum : uint8_t { DN_KEEP = 1, DN_CLONE = 2, DN_SPLIT = 4 };

// packed (keep, clone, split) counts: 21 bits each
__device__ __forceinline__ uint64_t dn_pack(uint32_t k, uint32_t c, uint32_t s) {
    return (uint64_t)k | ((uint64_t)c << 21) | ((uint64_t)s << 42);
}
__device__ __forceinline__ uint32_t dn_field(uint64_t v, int f) { return (uint32_t)(v >> (21 * f)) & 0x1fffffu; }

// exclusive scan of a packed u64 over the workgroup; returns the exclusive prefix, *total = workgroup sum
template <int NT>
__device__ __forceinline__ uint64_t block_exscan_u64(uint64_t v, uint64_t *s_wave, uint64_t *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint64_t off = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const uint64_t x = s_wave[w];
        if (w < wave) off += x;
        sum += x;
    }
    __syncthreads();
    *total = sum;
    return off + inc - v;
}

__device__ __forceinline__ uint8_t densify_class(const DensifyParams &p, int64_t i) {
    const float op = 1.f / (1.f + expf(-p.opacity[i]));
    const float s0 = expf(p.scaling[3 * i]), s1 = expf(p.scaling[3 * i + 1]), s2 = expf(p.scaling[3 * i + 2]);
    const float size = fmaxf(fmaxf(s0, s1), s2);
    bool keep = op > p.opacity_threshold;
    if (p.apply_screensize) keep = keep && (p.max_radii2D[i] < p.screensize_threshold);
    if (p.apply_size) keep = keep && (size < p.size_threshold);
    if (!keep) return 0;
    float g = p.grad_accum[i] / p.grad_count[i];
    if (g != g) g = 0.f;
    if (!(g >= p.grad_threshold)) return DN_KEEP;
    return DN_KEEP | (size < p.clone_size_threshold ? DN_CLONE : DN_SPLIT);
}

__global__ __launch_bounds__(DN_THREADS) void densify_classify_kernel(DensifyParams p) {
    __shared__ uint64_t s_wave[DN_THREADS / 64];
    const int64_t r0 = (int64_t)blockIdx.x * DN_ROWS + (int64_t)threadIdx.x * DN_PER;
    uint32_t k = 0, c = 0, s = 0;
#pragma unroll
    for (int j = 0; j < DN_PER; j++) {
        const int64_t i = r0 + j;
        if (i < p.N) {
            const uint8_t cl = densify_class(p, i);
            p.row_class[i] = cl;
            k += cl & DN_KEEP;
            c += (cl >> 1) & 1;
            s += (cl >> 2) & 1;
        }
    }
    uint64_t total;
    block_exscan_u64<DN_THREADS>(dn_pack(k, c, s), s_wave, &total);
    if (threadIdx.x == 0) {
        p.block_counts[3 * blockIdx.x] = (int32_t)dn_field(total, 0);
        p.block_counts[3 * blockIdx.x + 1] = (int32_t)dn_field(total, 1);
        p.block_counts[3 * blockIdx.x + 2] = (int32_t)dn_field(total, 2);
    }
}

// one workgroup: block_counts -> exclusive block offsets (in place), counts[0..2] = totals
__global__ __launch_bounds__(DN_SCAN_THREADS) void densify_scan_blocks_kernel(int32_t *block_counts, int nblocks,
                                                                              int32_t *counts) {
    __shared__ uint64_t s_wave[DN_SCAN_THREADS / 64];
    int64_t carry[3] = {0, 0, 0};
    for (int b0 = 0; b0 < nblocks; b0 += DN_SCAN_THREADS) {
        const int b = b0 + (int)threadIdx.x;
        uint32_t k = 0, c = 0, s = 0;
        if (b < nblocks) {
            k = (uint32_t)block_counts[3 * b];
            c = (uint32_t)block_counts[3 * b + 1];
            s = (uint32_t)block_counts[3 * b + 2];
        }
        uint64_t total;
        const uint64_t ex = block_exscan_u64<DN_SCAN_THREADS>(dn_pack(k, c, s), s_wave, &total);
        if (b < nblocks) {
            block_counts[3 * b] = (int32_t)(carry[0] + dn_field(ex, 0));
            block_counts[3 * b + 1] = (int32_t)(carry[1] + dn_field(ex, 1));
            block_counts[3 * b + 2] = (int32_t)(carry[2] + dn_field(ex, 2));
        }
        carry[0] += dn_field(total, 0);
        carry[1] += dn_field(total, 1);
        carry[2] += dn_field(total, 2);
    }
    if (threadIdx.x == 0) {
        counts[0] = (int32_t)carry[0];
        counts[1] = (int32_t)carry[1];
        counts[2] = (int32_t)carry[2];
    }
}

__global__ __launch_bounds__(DN_THREADS) void densify_map_kernel(DensifyParams p) {
    __shared__ uint64_t s_wave[DN_THREADS / 64];
    const int64_t r0 = (int64_t)blockIdx.x * DN_ROWS + (int64_t)threadIdx.x * DN_PER;
    uint8_t cl[DN_PER];
    uint32_t k = 0, c = 0, s = 0;
#pragma unroll
    for (int j = 0; j < DN_PER; j++) {
        cl[j] = (r0 + j < p.N) ? p.row_class[r0 + j] : 0;
        k += cl[j] & DN_KEEP;
        c += (cl[j] >> 1) & 1;
        s += (cl[j] >> 2) & 1;
    }
    uint64_t total;
    const uint64_t ex = block_exscan_u64<DN_THREADS>(dn_pack(k, c, s), s_wave, &total);
    const int32_t n_keep = p.counts[0], n_clone = p.counts[1];
    int32_t ok = p.block_counts[3 * blockIdx.x] + (int32_t)dn_field(ex, 0);
    int32_t oc = p.block_counts[3 * blockIdx.x + 1] + (int32_t)dn_field(ex, 1);
    int32_t os = p.block_counts[3 * blockIdx.x + 2] + (int32_t)dn_field(ex, 2);
#pragma unroll
    for (int j = 0; j < DN_PER; j++) {
        const int64_t i = r0 + j;
        if (i >= p.N) break;
        int32_t dk = -1, dc = -1, sr = -1;
        if (cl[j] & DN_KEEP) {
            dk = ok++;
            p.preserve_idx[dk] = i;
        }
        if (cl[j] & DN_CLONE) dc = n_keep + oc++;
        if (cl[j] & DN_SPLIT) {
            sr = os++;
            dc = n_keep + n_clone + sr;
        }
        p.dst_map[i] = dk;
        p.dst_map[p.N + i] = dc;
        p.split_rank[i] = sr;
    }
}

// R(q) row c of the normalised quaternion (w, x, y, z) -- kornia quaternion_to_rotation_matrix
__device__ __forceinline__ float split_offset(const float *q4, const float *s3, const float *z3, int c) {
    const float nq = fmaxf(sqrtf(q4[0] * q4[0] + q4[1] * q4[1] + q4[2] * q4[2] + q4[3] * q4[3]), 1e-12f);
    const float w = q4[0] / nq, x = q4[1] / nq, y = q4[2] / nq, z = q4[3] / nq;
    const float tx = 2.f * x, ty = 2.f * y, tz = 2.f * z;
    const float twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
    const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
    float r0, r1, r2;
    if (c == 0) {
        r0 = 1.f - (tyy + tzz); r1 = txy - twz; r2 = txz + twy;
    } else if (c == 1) {
        r0 = txy + twz; r1 = 1.f - (txx + tzz); r2 = tyz - twx;
    } else {
        r0 = txz - twy; r1 = tyz + twx; r2 = 1.f - (txx + tyy);
    }
    const float d0 = z3[0] * expf(s3[0]), d1 = z3[1] * expf(s3[1]), d2 = z3[2] * expf(s3[2]);
    return r0 * d0 + r1 * d1 + r2 * d2;
}

__global__ __launch_bounds__(256) void densify_apply_kernel(DensifyApply A) {
    int fi = 0;
#pragma unroll 1
    while (fi + 1 < A.num_fields && (int64_t)blockIdx.x >= A.block_start[fi + 1]) fi++;
    const DensifyFieldDev &F = A.f[fi];
    const int64_t e = ((int64_t)blockIdx.x - A.block_start[fi]) * 256 + threadIdx.x;
    const int64_t n_el = A.N * F.width;
    if (e >= n_el) return;
    const int64_t i = e / F.width;
    const int c = (int)(e - i * F.width);
    const int32_t dk = A.dst_map[i], dc = A.dst_map[A.N + i];
    if (dk < 0) return;  // pruned (a pruned row is never cloned or split)
    float v = F.src[e];
    if (dc >= 0 && A.split_rank[i] >= 0) {
        if (F.kind == GSR_FIELD_XYZ) v = v + split_offset(A.rotation + 4 * i, A.scaling + 3 * i, A.z + 3 * A.split_rank[i], c);
        else if (F.kind == GSR_FIELD_SCALING) v = logf(expf(v) / 1.6f);
    }
    const int64_t ok = (int64_t)dk * F.width + c;
    F.dst[ok] = v;
    if (F.dst_exp_avg) F.dst_exp_avg[ok] = F.src_exp_avg[e];
    if (F.dst_exp_avg_sq) F.dst_exp_avg_sq[ok] = F.src_exp_avg_sq[e];
    if (dc >= 0) {
        const int64_t oc = (int64_t)dc * F.width + c;
        F.dst[oc] = (F.kind == GSR_FIELD_STAT) ? 0.f : v;
        if (F.dst_exp_avg) F.dst_exp_avg[oc] = 0.f;
        if (F.dst_exp_avg_sq) F.dst_exp_avg_sq[oc] = 0.f;
    }
}

int64_t densify_blocks(int64_t N) { return (N + DN_ROWS - 1) / DN_ROWS; }

void launch_densify_classify(hipStream_t s, const DensifyParams &p) {
    const int64_t nb = densify_blocks(p.N);
    if (nb == 0) {
        (void)hipMemsetAsync(p.counts, 0, 3 * sizeof(int32_t), s);
        return;
    }
    densify_classify_kernel<<<(unsigned)nb, DN_THREADS, 0, s>>>(p);
    densify_scan_blocks_kernel<<<1, DN_SCAN_THREADS, 0, s>>>(p.block_counts, (int)nb, p.counts);
    densify_map_kernel<<<(unsigned)nb, DN_THREADS, 0, s>>>(p);
}

void launch_densify_apply(hipStream_t s, const DensifyApply &A, int64_t total_blocks) {
    if (total_blocks <= 0) return;
    densify_apply_kernel<<<(unsigned)total_blocks, 256, 0, s>>>(A);
}

}  // namespace gsr
