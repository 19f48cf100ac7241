// gsr_ply.hip -- PLY vertex records <-> per-Gaussian parameter tensors, on the GPU.
//
// A 3DGS checkpoint (gaussian_model.py:150-171 save_ply / third_party/.../gaussian_model.py:239-314) is one
// binary PLY "vertex" element: an array of fixed-size records (x y z nx ny nz f_dc_* f_rest_* opacity scale_*
// rot_*, 62 float32 = 248 B at SH degree 3).  The host maps the file and copies the record bytes to HBM in
// one transfer; these kernels then de-interleave (unpack) or interleave (pack) every column in one launch.
// Each workgroup stages a tile of whole records through LDS with contiguous global accesses, then reads or
// writes the output fields in their own contiguous row-major order -- the record-major <-> field-major
// transpose happens in LDS, never as strided HBM traffic.  The column table lists, in destination order
// (field after field, column after column), each column's byte offset inside the record and its PLY type;
// the channel-major f_rest layout of the file becomes a permutation of that table on the host.
#include "gsr_kernels.h"
#include "gsrast.h"

namespace gsr {

constexpr int PLY_THREADS = 256;

__device__ __forceinline__ uint32_t ld_bytes(const uint8_t *s, int n, bool swap) {
    uint32_t v = 0;
    for (int b = 0; b < n; b++) v |= (uint32_t)s[b] << (8 * (swap ? (n - 1 - b) : b));
    return v;
}

__device__ __forceinline__ float ply_value(const uint8_t *s, int type, bool swap) {
    switch (type) {
        case GSR_PLY_FLOAT32: return __uint_as_float(ld_bytes(s, 4, swap));
        case GSR_PLY_FLOAT64: {
            const uint64_t lo = ld_bytes(s + (swap ? 4 : 0), 4, swap), hi = ld_bytes(s + (swap ? 0 : 4), 4, swap);
            return (float)__longlong_as_double((long long)(lo | (hi << 32)));
        }
        case GSR_PLY_UINT8: return (float)s[0];
        case GSR_PLY_INT8: return (float)(int8_t)s[0];
        case GSR_PLY_UINT16: return (float)(uint16_t)ld_bytes(s, 2, swap);
        case GSR_PLY_INT16: return (float)(int16_t)ld_bytes(s, 2, swap);
        case GSR_PLY_UINT32: return (float)ld_bytes(s, 4, swap);
        default: return (float)(int32_t)ld_bytes(s, 4, swap);
    }
}

__device__ __forceinline__ void tile_load(uint8_t *s_rec, const uint8_t *g, int64_t bytes) {
    if ((((uintptr_t)g) & 3) == 0) {
        const int64_t nw = bytes >> 2;
        for (int64_t i = threadIdx.x; i < nw; i += PLY_THREADS)
            reinterpret_cast<uint32_t *>(s_rec)[i] = reinterpret_cast<const uint32_t *>(g)[i];
        for (int64_t i = (nw << 2) + threadIdx.x; i < bytes; i += PLY_THREADS) s_rec[i] = g[i];
    } else {
        for (int64_t i = threadIdx.x; i < bytes; i += PLY_THREADS) s_rec[i] = g[i];
    }
}

__device__ __forceinline__ void tile_store(uint8_t *g, const uint8_t *s_rec, int64_t bytes) {
    if ((((uintptr_t)g) & 3) == 0) {
        const int64_t nw = bytes >> 2;
        for (int64_t i = threadIdx.x; i < nw; i += PLY_THREADS)
            reinterpret_cast<uint32_t *>(g)[i] = reinterpret_cast<const uint32_t *>(s_rec)[i];
        for (int64_t i = (nw << 2) + threadIdx.x; i < bytes; i += PLY_THREADS) g[i] = s_rec[i];
    } else {
        for (int64_t i = threadIdx.x; i < bytes; i += PLY_THREADS) g[i] = s_rec[i];
    }
}

__global__ __launch_bounds__(PLY_THREADS) void ply_unpack_kernel(PlyLaunch p) {
    extern __shared__ uint8_t s_dyn[];
    int2 *s_col = reinterpret_cast<int2 *>(s_dyn);
    uint8_t *s_rec = s_dyn + align_up((size_t)p.ncols * sizeof(int2), 16);
    for (int i = threadIdx.x; i < p.ncols; i += PLY_THREADS) s_col[i] = p.cols[i];
    const int64_t row0 = (int64_t)blockIdx.x * p.rows_per_block;
    const int rows = (int)min((int64_t)p.rows_per_block, p.n - row0);
    tile_load(s_rec, p.records + row0 * p.record_bytes, (int64_t)rows * p.record_bytes);
    __syncthreads();
    int cb = 0;
    for (int f = 0; f < p.nfields; f++) {
        const int w = p.width[f];
        float *dst = p.field[f] + row0 * w;
        for (int e = threadIdx.x; e < rows * w; e += PLY_THREADS) {
            const int r = e / w, c = e - r * w;
            const int2 col = s_col[cb + c];
            dst[e] = ply_value(s_rec + (int64_t)r * p.record_bytes + col.x, col.y, p.swap);
        }
        cb += w;
    }
}

__global__ __launch_bounds__(PLY_THREADS) void ply_pack_kernel(PlyLaunch p) {
    extern __shared__ uint8_t s_dyn[];
    int2 *s_col = reinterpret_cast<int2 *>(s_dyn);
    uint8_t *s_rec = s_dyn + align_up((size_t)p.ncols * sizeof(int2), 16);
    for (int i = threadIdx.x; i < p.ncols; i += PLY_THREADS) s_col[i] = p.cols[i];
    const int64_t row0 = (int64_t)blockIdx.x * p.rows_per_block;
    const int rows = (int)min((int64_t)p.rows_per_block, p.n - row0);
    const int64_t bytes = (int64_t)rows * p.record_bytes;
    for (int64_t i = threadIdx.x; i < bytes; i += PLY_THREADS) s_rec[i] = 0;  // columns no field covers
    __syncthreads();
    int cb = 0;
    for (int f = 0; f < p.nfields; f++) {
        const int w = p.width[f];
        const float *src = p.field[f] + row0 * w;
        for (int e = threadIdx.x; e < rows * w; e += PLY_THREADS) {
            const int r = e / w, c = e - r * w;
            const uint32_t u = __float_as_uint(src[e]);
            uint8_t *d = s_rec + (int64_t)r * p.record_bytes + s_col[cb + c].x;
#pragma unroll
            for (int b = 0; b < 4; b++) d[b] = (uint8_t)(u >> (8 * (p.swap ? 3 - b : b)));
        }
        cb += w;
    }
    __syncthreads();
    tile_store(p.records_out + row0 * p.record_bytes, s_rec, bytes);
}

int ply_rows_per_block(int record_bytes) {
    const int r = (48 * 1024) / (record_bytes > 0 ? record_bytes : 1);
    return r < 1 ? 1 : (r > 128 ? 128 : r);
}

size_t ply_lds_bytes(const PlyLaunch &p) {
    return align_up((size_t)p.ncols * sizeof(int2), 16) + (size_t)p.rows_per_block * p.record_bytes;
}

void launch_ply(hipStream_t s, const PlyLaunch &p, bool pack) {
    const int64_t blocks = (p.n + p.rows_per_block - 1) / p.rows_per_block;
    if (blocks <= 0) return;
    const size_t lds = ply_lds_bytes(p);
    if (pack) ply_pack_kernel<<<(unsigned)blocks, PLY_THREADS, lds, s>>>(p);
    else ply_unpack_kernel<<<(unsigned)blocks, PLY_THREADS, lds, s>>>(p);
}

}  // namespace gsr
