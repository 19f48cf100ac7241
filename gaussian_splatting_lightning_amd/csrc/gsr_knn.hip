// gsr_knn.hip -- exact mean squared distance to the 3 nearest neighbours (scale initialisation).
//
// Replaces distCUDA2 of gs_lightning/utils/math.py:9-14 (scipy KDTree(points).query(points, k=4), the self
// match dropped, mean of the three squared distances), used by GaussianModel.initialize
// (gaussian_model.py:84-91) to size the initial Gaussians from the COLMAP points.  Exact, like the KDTree:
//
//   1. bounding cube (two-level min/max reduction);
//   2. 63-bit Morton code per point (21 bits per axis) and a stable LSD sort of the codes as two 32-bit
//      radix sorts (low word, then high word carrying the permutation) -- points become spatially ordered;
//   3. per point, an upper bound on the 3rd-neighbour distance R from the +-KNN_WINDOW neighbours in Morton
//      order; then the finest octree level L whose cells are at least R wide -- every point within R lies in
//      the 3x3x3 block of level-L cells around the query, and each such cell is one contiguous range of the
//      sorted codes (a Morton prefix), found by binary search.  A cell holding more than KNN_LEAF points is
//      descended depth-first through its octree children (their ranges split the parent's range), nearest
//      child first; any cell farther than the current 3rd distance is skipped -- an isolated outlier whose
//      window bound is loose therefore never scans whole clusters.  Candidates are ranked in fp32; the three winners' squared distances are recomputed in
//      fp64 (the KDTree works in fp64) and their mean is rounded to fp32.
//
// With fewer than four points the missing neighbours count as +inf, as KDTree.query reports them.
#include "gsr_kernels.h"

namespace gsr {

constexpr int KNN_THREADS = 256;
constexpr int KNN_WINDOW = 8;
constexpr int KNN_BITS = 21;
constexpr int KNN_BBOX_BLOCKS = 1024;

__device__ __forceinline__ uint64_t spread3(uint32_t v) {  // 21 bits -> every third bit of 63
    uint64_t x = v & 0x1fffffu;
    x = (x | (x << 32)) & 0x1f00000000ffffull;
    x = (x | (x << 16)) & 0x1f0000ff0000ffull;
    x = (x | (x << 8)) & 0x100f00f00f00f00full;
    x = (x | (x << 4)) & 0x10c30c30c30c30c3ull;
    x = (x | (x << 2)) & 0x1249249249249249ull;
    return x;
}

__device__ __forceinline__ uint64_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    return spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
}

__global__ __launch_bounds__(KNN_THREADS) void knn_bbox_partial_kernel(const float *pts, int64_t n, float *partial) {
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * KNN_THREADS) {
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const float v = pts[3 * i + a];
            mn[a] = fminf(mn[a], v);
            mx[a] = fmaxf(mx[a], v);
        }
    }
    __shared__ float s[6][KNN_THREADS / 64];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        for (int o = 32; o > 0; o >>= 1) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], o));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o));
        }
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
        for (int a = 0; a < 3; a++) {
            s[a][w] = mn[a];
            s[3 + a][w] = mx[a];
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        float r = s[threadIdx.x][0];
        for (int k = 1; k < KNN_THREADS / 64; k++)
            r = threadIdx.x < 3 ? fminf(r, s[threadIdx.x][k]) : fmaxf(r, s[threadIdx.x][k]);
        partial[6 * blockIdx.x + threadIdx.x] = r;
    }
}

// box[0..2] = min corner, box[3] = cube extent, box[4] = 2^21 / extent
__global__ __launch_bounds__(64) void knn_bbox_final_kernel(const float *partial, int nblocks, float *box) {
    if (threadIdx.x != 0) return;
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int b = 0; b < nblocks; b++)
        for (int a = 0; a < 3; a++) {
            mn[a] = fminf(mn[a], partial[6 * b + a]);
            mx[a] = fmaxf(mx[a], partial[6 * b + 3 + a]);
        }
    float ext = fmaxf(fmaxf(mx[0] - mn[0], mx[1] - mn[1]), mx[2] - mn[2]);
    if (!(ext > 0.f) || !isfinite(ext)) ext = 1.f;
    box[0] = mn[0];
    box[1] = mn[1];
    box[2] = mn[2];
    box[3] = ext;
    box[4] = (float)(1u << KNN_BITS) / ext;
}

__device__ __forceinline__ uint32_t knn_quant(float v, float lo, float scale) {
    const float q = floorf((v - lo) * scale);
    return q <= 0.f ? 0u : (q >= (float)((1u << KNN_BITS) - 1) ? (1u << KNN_BITS) - 1 : (uint32_t)q);
}

__global__ __launch_bounds__(KNN_THREADS) void knn_code_kernel(const float *pts, int64_t n, const float *box,
                                                              uint64_t *codes, uint32_t *key_lo) {
    const int64_t i = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x;
    if (i >= n) return;
    const float sc = box[4];
    const uint64_t c = morton3(knn_quant(pts[3 * i], box[0], sc), knn_quant(pts[3 * i + 1], box[1], sc),
                               knn_quant(pts[3 * i + 2], box[2], sc));
    codes[i] = c;
    key_lo[i] = (uint32_t)c;
}

__global__ __launch_bounds__(KNN_THREADS) void knn_hi_kernel(const uint64_t *codes, const uint32_t *perm, int64_t n,
                                                            uint32_t *key_hi) {
    const int64_t i = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x;
    if (i < n) key_hi[i] = (uint32_t)(codes[perm[i]] >> 32);
}

__global__ __launch_bounds__(KNN_THREADS) void knn_gather_kernel(const float *pts, const uint64_t *codes,
                                                                const uint32_t *order, int64_t n, uint64_t *scode,
                                                                float4 *spts) {
    const int64_t i = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x;
    if (i >= n) return;
    const uint32_t o = order[i];
    scode[i] = codes[o];
    spts[i] = make_float4(pts[3 * o], pts[3 * o + 1], pts[3 * o + 2], 0.f);
}

struct Best3 {
    float d[3];
    int j[3];
    __device__ __forceinline__ void init() {
        d[0] = d[1] = d[2] = INFINITY;
        j[0] = j[1] = j[2] = -1;
    }
    __device__ __forceinline__ void insert(float dd, int jj) {
        if (!(dd < d[2]) || jj == j[0] || jj == j[1] || jj == j[2]) return;
        if (dd < d[1]) {
            d[2] = d[1]; j[2] = j[1];
            if (dd < d[0]) {
                d[1] = d[0]; j[1] = j[0];
                d[0] = dd; j[0] = jj;
            } else {
                d[1] = dd; j[1] = jj;
            }
        } else {
            d[2] = dd; j[2] = jj;
        }
    }
};

__device__ __forceinline__ float d2f(float4 a, float4 b) {
    const float x = a.x - b.x, y = a.y - b.y, z = a.z - b.z;
    return x * x + y * y + z * z;
}

__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t *a, int64_t n, uint64_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// An octree cell of the Morton-ordered points: level-L integer coordinates and its range in sorted order.
struct KnnNode {
    uint32_t c[3];
    int L;
    int32_t r0, r1;
};
constexpr int KNN_LEAF = 24;            // scan ranges this small instead of subdividing
constexpr int KNN_STACK = 8 * KNN_BITS + 8;

struct KnnQuery {
    float4 p;
    float lo[3], ext;
    const float4 *spts;
    const uint64_t *scode;
    int64_t self;

    // squared distance from p to the cell's box
    __device__ __forceinline__ float gap2(const uint32_t c[3], int L) const {
        const float h = ext / (float)(1u << L);
        const float pc[3] = {p.x, p.y, p.z};
        float g2 = 0.f;
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const float b0 = lo[a] + (float)c[a] * h, b1 = b0 + h;
            const float g = fmaxf(fmaxf(b0 - pc[a], pc[a] - b1), 0.f);
            g2 += g * g;
        }
        return g2;
    }
    __device__ __forceinline__ bool prune(float g2, const Best3 &b) const { return g2 > b.d[2] * 1.0002f + 1e-30f; }

    __device__ __forceinline__ void scan(int32_t r0, int32_t r1, Best3 &b) const {
        for (int32_t j = r0; j < r1; j++)
            if (j != self) b.insert(d2f(p, spts[j]), j);
    }

    // depth-first descent from one cell, nearest child first, pruning cells beyond the current 3rd distance
    __device__ void visit(const KnnNode &start, Best3 &b) const {
        KnnNode st[KNN_STACK];
        int sp = 0;
        st[sp++] = start;
        while (sp > 0) {
            const KnnNode nd = st[--sp];
            if (prune(gap2(nd.c, nd.L), b)) continue;
            if (nd.r1 - nd.r0 <= KNN_LEAF || nd.L == KNN_BITS) {
                scan(nd.r0, nd.r1, b);
                continue;
            }
            const int cl = nd.L + 1, s3 = 3 * (KNN_BITS - cl);
            const uint64_t base = morton3(nd.c[0] * 2, nd.c[1] * 2, nd.c[2] * 2);
            int32_t bnd[9];
            bnd[0] = nd.r0;
            bnd[8] = nd.r1;
            for (int ch = 1; ch < 8; ch++) {
                const uint64_t key = (base | (uint64_t)ch) << s3;
                int32_t lo2 = bnd[ch - 1], hi2 = nd.r1;
                while (lo2 < hi2) {
                    const int32_t mid = (lo2 + hi2) >> 1;
                    if (scode[mid] < key) lo2 = mid + 1;
                    else hi2 = mid;
                }
                bnd[ch] = lo2;
            }
            // push non-empty children farthest first so the nearest is visited first
            float g[8];
            int idx[8], m = 0;
            for (int ch = 0; ch < 8; ch++) {
                if (bnd[ch + 1] <= bnd[ch]) continue;
                const uint32_t cc[3] = {nd.c[0] * 2 + (ch & 1), nd.c[1] * 2 + ((ch >> 1) & 1), nd.c[2] * 2 + (ch >> 2)};
                const float gg = gap2(cc, cl);
                if (prune(gg, b)) continue;
                int k = m++;
                while (k > 0 && g[k - 1] < gg) {  // descending by gap
                    g[k] = g[k - 1];
                    idx[k] = idx[k - 1];
                    k--;
                }
                g[k] = gg;
                idx[k] = ch;
            }
            for (int k = 0; k < m && sp < KNN_STACK; k++) {
                const int ch = idx[k];
                KnnNode c;
                c.c[0] = nd.c[0] * 2 + (ch & 1);
                c.c[1] = nd.c[1] * 2 + ((ch >> 1) & 1);
                c.c[2] = nd.c[2] * 2 + (ch >> 2);
                c.L = cl;
                c.r0 = bnd[ch];
                c.r1 = bnd[ch + 1];
                st[sp++] = c;
            }
        }
    }
};

__global__ __launch_bounds__(KNN_THREADS) void knn_query_kernel(const float4 *spts, const uint64_t *scode,
                                                               const uint32_t *order, int64_t n, const float *box,
                                                               float *out) {
    const int64_t i = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x;
    if (i >= n) return;
    KnnQuery q;
    q.p = spts[i];
    q.lo[0] = box[0];
    q.lo[1] = box[1];
    q.lo[2] = box[2];
    q.ext = box[3];
    q.spts = spts;
    q.scode = scode;
    q.self = i;
    const float sc = box[4];
    Best3 b;
    b.init();
    const int64_t w0 = i > KNN_WINDOW ? i - KNN_WINDOW : 0, w1 = min(n - 1, i + KNN_WINDOW);
    for (int64_t j = w0; j <= w1; j++)
        if (j != i) b.insert(d2f(q.p, spts[j]), (int)j);
    if (b.d[2] > 0.f) {
        // start from the 3x3x3 block of the finest level whose cells cover the window's 3rd distance
        const float R = sqrtf(b.d[2]) * 1.0001f;
        int L = KNN_BITS;
        while (L > 0 && q.ext / (float)(1u << L) < R) L--;
        const int sh = KNN_BITS - L;
        const uint32_t qc[3] = {knn_quant(q.p.x, q.lo[0], sc) >> sh, knn_quant(q.p.y, q.lo[1], sc) >> sh,
                                knn_quant(q.p.z, q.lo[2], sc) >> sh};
        const int64_t cmax = (int64_t)(1u << L) - 1;
        for (int dz = -1; dz <= 1; dz++)
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    const int64_t c[3] = {(int64_t)qc[0] + dx, (int64_t)qc[1] + dy, (int64_t)qc[2] + dz};
                    if (c[0] < 0 || c[1] < 0 || c[2] < 0 || c[0] > cmax || c[1] > cmax || c[2] > cmax) continue;
                    KnnNode nd;
                    nd.c[0] = (uint32_t)c[0];
                    nd.c[1] = (uint32_t)c[1];
                    nd.c[2] = (uint32_t)c[2];
                    nd.L = L;
                    if (q.prune(q.gap2(nd.c, L), b)) continue;
                    const uint64_t pre = morton3(nd.c[0], nd.c[1], nd.c[2]);
                    const int s3 = 3 * sh;
                    nd.r0 = (int32_t)lower_bound_u64(scode, n, pre << s3);
                    nd.r1 = (s3 >= 63) ? (int32_t)n : (int32_t)lower_bound_u64(scode, n, (pre + 1) << s3);
                    if (nd.r1 > nd.r0) q.visit(nd, b);
                }
    }
    float res;
    if (b.j[2] < 0) {
        res = INFINITY;
    } else {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float4 o = spts[b.j[k]];
            const double x = (double)q.p.x - (double)o.x, y = (double)q.p.y - (double)o.y,
                         z = (double)q.p.z - (double)o.z;
            acc += x * x + y * y + z * z;
        }
        res = (float)(acc / 3.0);
    }
    out[order[i]] = res;
}

size_t knn_workspace(int64_t n, KnnScratch *k) {
    Carver c(k ? reinterpret_cast<char *>(k->base) : nullptr);
    SortScratch sort{};
    carve_sort(c, sort, (uint32_t)(n ? n : 1), true);
    uint64_t *codes = c.take<uint64_t>(n ? n : 1);
    uint64_t *scode = c.take<uint64_t>(n ? n : 1);
    float4 *spts = c.take<float4>(n ? n : 1);
    float *partial = c.take<float>(6 * KNN_BBOX_BLOCKS);
    float *box = c.take<float>(8);
    if (k) {
        k->sort = sort;
        k->codes = codes;
        k->scode = scode;
        k->spts = spts;
        k->partial = partial;
        k->box = box;
    }
    return c.off + 256;
}

void launch_knn(hipStream_t s, KnnScratch &k, const float *pts, int64_t n, float *out) {
    if (n <= 0) return;
    const unsigned g = (unsigned)div_up((uint64_t)n, KNN_THREADS);
    const int bb = (int)(g < (unsigned)KNN_BBOX_BLOCKS ? g : (unsigned)KNN_BBOX_BLOCKS);
    knn_bbox_partial_kernel<<<bb, KNN_THREADS, 0, s>>>(pts, n, k.partial);
    knn_bbox_final_kernel<<<1, 64, 0, s>>>(k.partial, bb, k.box);
    knn_code_kernel<<<g, KNN_THREADS, 0, s>>>(pts, n, k.box, k.codes, k.sort.k[0]);
    launch_radix_sort(s, k.sort, (uint32_t)n, 32);                      // by low word: v[0] = permutation
    knn_hi_kernel<<<g, KNN_THREADS, 0, s>>>(k.codes, k.sort.v[0], n, k.sort.k[0]);
    launch_radix_sort(s, k.sort, (uint32_t)n, 32, true);               // by high word, stable, carrying v[0]
    knn_gather_kernel<<<g, KNN_THREADS, 0, s>>>(pts, k.codes, k.sort.v[0], n, k.scode, k.spts);
    knn_query_kernel<<<g, KNN_THREADS, 0, s>>>(k.spts, k.scode, k.sort.v[0], n, k.box, out);
}

}  // namespace gsr
