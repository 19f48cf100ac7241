// gsr_bin.hip -- bucket binning: the (tile, depth, index) instance order without a global sort.
//
// The reference duplicates every (Gaussian, tile) instance with a 64-bit key (tile << 32 | depth bits) and
// radix-sorts all of them (SURVEY.md §2.1 duplicateWithKeys + cub::DeviceRadixSort, [U]); the sort is stable
// and the instances are emitted in Gaussian order, so ties in depth fall back to the Gaussian index.  Here:
//   1. bk_count    each block walks a contiguous Gaussian range (plus a share of the big Gaussians) and
//                  histograms its instances per tile in LDS: one row of the (blocks x tiles) count matrix;
//   2. bk_columns  exclusive prefix of every tile column over the blocks, and the tile totals;
//   3. bk_tscan    exclusive scan of the tile totals -> tile ranges (one workgroup);
//   4. bk_scatter  the same walk again: each instance takes the next free slot of its tile's bucket
//                  (LDS counters seeded from the prefixes) and stores key = depth bits << 32 | u, where u is
//                  its Gaussian-major expansion index (u increases with the Gaussian index);
//   5. seg_sort    one wave per tile sorts the bucket by key in registers (bitonic network, 64-bit keys)
//                  and writes the expansion index of every sorted position.  Keys are unique inside a tile
//                  (one instance per Gaussian), so the order inside a bucket after step 4 does not matter
//                  and the result is exactly the reference's (tile, depth, index) order.  Tiles above
//                  SEG_CAP instances are sorted by a whole workgroup (seg_block: four waves' registers, the
//                  cross-wave stages through LDS); tiles above SEG_BLOCK_CAP in SEG_BLOCK_CAP-key chunks that
//                  seg_merge places by merge ranks (binary search of every key in the other chunks).
// Everything is integer work; nothing depends on scheduling, so the result is deterministic.
#include <algorithm>

#include "gsr_kernels.h"

namespace gsr {

// ------------------------------------------------------------------------------------------------
// steps 1 and 4: walk the instances of a block's Gaussians
// ------------------------------------------------------------------------------------------------
// A small Gaussian (<= BIG_GAUSSIAN_TILES instances) is enumerated by rect cells: its expansion record holds
// the kept-tile mask of its rect (0 = every cell kept), so cell c is an instance iff its mask bit is set, and
// its instance number is the count of kept cells before it.  The 64 lanes of a wave enumerate the cells of
// their 64 Gaussians jointly, 64 (Gaussian, cell) pairs per step whatever the mix of sizes: the lane whose
// cell run starts inside the step marks its start in LDS, and a DPP max-scan hands every pair its owner.
// Big Gaussians (every rect cell kept) are spread over the blocks round-robin; a whole block strides over
// each rect.  The next group's per-Gaussian records are loaded while the current group is walked.

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dpp_max_step(int v) {
    return max(v, __builtin_amdgcn_update_dpp(-1, v, CTRL, ROW_MASK, 0xf, false));
}
// inclusive max-scan over the wave for values >= -1
__device__ __forceinline__ int wave_inclusive_max(int v) {
    v = dpp_max_step<0x111, 0xf>(v);  // row_shr:1
    v = dpp_max_step<0x112, 0xf>(v);  // row_shr:2
    v = dpp_max_step<0x114, 0xf>(v);  // row_shr:4
    v = dpp_max_step<0x118, 0xf>(v);  // row_shr:8
    v = dpp_max_step<0x142, 0xa>(v);  // row_bcast:15
    v = dpp_max_step<0x143, 0xc>(v);  // row_bcast:31
    return v;
}

// (row, column) of cell c of a rect of width w: floor((c + 1/2) / w) in fp32 is exact here ((c + 1/2) / w is
// at least 1/(2w) from an integer and far below 2^20)
__device__ __forceinline__ uint32_t rect_tile(uint32_t c, uint32_t rx, uint32_t ry, uint32_t w, float inv_w,
                                              uint32_t gx) {
    const uint32_t cy = (uint32_t)(((float)c + 0.5f) * inv_w);
    return (ry + cy) * gx + rx + (c - cy * w);
}

template <bool SCATTER, int BKW>  // BKW: waves per workgroup
__global__ __launch_bounds__(64 * BKW) void bk_walk_kernel(BucketParams p) {
    extern __shared__ uint32_t s_tab[];   // T entries: tile counts (count) / next free bucket slot (scatter)
    __shared__ uint4 s_rec[BKW][64];      // expansion records: kept mask lo, hi, rect x | y << 16, rect width
    __shared__ uint4 s_aux[BKW][64];      // first cell pair, first expansion index, depth key, 1/width bits
    __shared__ int s_own[BKW][64];        // lane whose cell run starts at this pair of the step, else -1
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t b = blockIdx.x, T = p.T, gx = (uint32_t)p.gx;
    if (SCATTER) {
        const uint32_t *hrow = p.hist + (size_t)b * T;
        for (uint32_t t = tid; t < T; t += 64 * BKW) s_tab[t] = p.tile_start[t] + hrow[t];
    } else {
        for (uint32_t t = tid; t < T; t += 64 * BKW) s_tab[t] = 0u;
    }
    s_own[w][lane] = -1;
    __syncthreads();
    const uint32_t g_lo = b * p.gper, g_hi = min(p.P, g_lo + p.gper);
    uint32_t g = g_lo + (uint32_t)w * 64 + lane;
    uint32_t n_kept = 0, n_u = 0, n_dep = 0;
    uint4 n_e = make_uint4(0, 0, 0, 0);
    if (g < g_hi) {
        n_kept = p.tiles[g];
        n_e = p.exp_rec[g];
        if (SCATTER) {
            n_u = p.inst_start[g];
            n_dep = p.depth_key[g];
        }
    }
    for (uint32_t g0 = g_lo + (uint32_t)w * 64; g0 < g_hi; g0 += 64 * BKW) {  // uniform per wave
        const uint32_t kept = n_kept, u = n_u, dep = n_dep;
        const uint4 e = n_e;
        g = g0 + 64 * BKW + lane;
        n_kept = 0;
        if (g < g_hi) {
            n_kept = p.tiles[g];
            n_e = p.exp_rec[g];
            if (SCATTER) {
                n_u = p.inst_start[g];
                n_dep = p.depth_key[g];
            }
        }
        uint32_t len = 0;
        const uint64_t m = (uint64_t)e.x | ((uint64_t)e.y << 32);
        if (kept > 0 && kept <= BIG_GAUSSIAN_TILES) len = m ? 64u - (uint32_t)__builtin_clzll(m) : kept;
        const uint32_t incl = wave_inclusive_scan(len, lane);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t start = incl - len;
        s_rec[w][lane] = e;
        s_aux[w][lane] = make_uint4(start, u, dep, __float_as_uint(len ? 1.0f / (float)e.w : 0.f));
        int carry = -1;
        for (uint32_t B = 0; B < total; B += 64) {
            const bool marks = len > 0 && start >= B && start < B + 64;
            if (marks) s_own[w][start - B] = lane;
            wave_lds_sync();
            const int o = max(wave_inclusive_max(s_own[w][lane]), carry);
            carry = __builtin_amdgcn_readlane(o, 63);
            wave_lds_sync();
            if (marks) s_own[w][start - B] = -1;
            const uint32_t j = B + (uint32_t)lane;
            if (j < total) {
                const uint4 r = s_rec[w][o];
                const uint4 x = s_aux[w][o];
                const uint32_t c = j - x.x;
                const uint64_t mo = (uint64_t)r.x | ((uint64_t)r.y << 32);
                if (!mo || ((mo >> c) & 1ull)) {
                    const uint32_t tile = rect_tile(c, r.z & 0xffffu, r.z >> 16, r.w, __uint_as_float(x.w), gx);
                    if (!SCATTER) {
                        atomicAdd(&s_tab[tile], 1u);
                    } else {
                        const uint32_t ui = x.y + (mo ? (uint32_t)__popcll(mo & ((1ull << c) - 1ull)) : c);
                        const uint32_t slot = atomicAdd(&s_tab[tile], 1u);
                        p.keys[slot] = ((unsigned long long)x.z << 32) | ui;
                        p.inst_gid[ui] = g0 + (uint32_t)o;
                    }
                }
            }
        }
        wave_lds_sync();
    }
    for (uint32_t bi = b; bi < p.nbig; bi += p.nb) {
        const uint32_t gb = p.big_list[bi];
        const uint4 e = p.exp_rec[gb];
        const uint32_t area = p.tiles[gb];
        const float inv_w = 1.0f / (float)e.w;
        const uint32_t u0 = SCATTER ? p.inst_start[gb] : 0u;
        const unsigned long long dk = SCATTER ? ((unsigned long long)p.depth_key[gb] << 32) : 0ull;
        for (uint32_t c = tid; c < area; c += 64 * BKW) {
            const uint32_t tile = rect_tile(c, e.z & 0xffffu, e.z >> 16, e.w, inv_w, gx);
            if (!SCATTER) {
                atomicAdd(&s_tab[tile], 1u);
            } else {
                const uint32_t slot = atomicAdd(&s_tab[tile], 1u);
                p.keys[slot] = dk | (u0 + c);
                p.inst_gid[u0 + c] = gb;
            }
        }
    }
    if (!SCATTER) {
        __syncthreads();
        uint32_t *row = p.hist + (size_t)b * T;
        for (uint32_t t = tid; t < T; t += 64 * BKW) row[t] = s_tab[t];
    }
}

// ------------------------------------------------------------------------------------------------
// step 2: column prefixes of the count matrix.  A workgroup owns 64 tile columns (one per lane); its four
// waves own four contiguous quarters of the block rows.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bk_columns_kernel(uint32_t *__restrict__ hist, uint32_t nb, uint32_t T,
                                                         uint32_t *__restrict__ tile_cnt) {
    __shared__ uint32_t s_sum[4][64];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t t = blockIdx.x * 64 + lane;
    const uint32_t q = (nb + 3) / 4, r0 = min(nb, w * q), r1 = min(nb, r0 + q);
    uint32_t sum = 0;
    if (t < T) {
        uint32_t r = r0;
        for (; r + 8 <= r1; r += 8) {
            uint32_t v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) v[i] = hist[(size_t)(r + i) * T + t];
#pragma unroll
            for (int i = 0; i < 8; i++) sum += v[i];
        }
        for (; r < r1; r++) sum += hist[(size_t)r * T + t];
    }
    s_sum[w][lane] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (int i = 0; i < w; i++) run += s_sum[i][lane];
    if (t < T) {
        uint32_t r = r0;
        for (; r + 8 <= r1; r += 8) {
            uint32_t v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) v[i] = hist[(size_t)(r + i) * T + t];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                hist[(size_t)(r + i) * T + t] = run;
                run += v[i];
            }
        }
        for (; r < r1; r++) {
            const uint32_t v = hist[(size_t)r * T + t];
            hist[(size_t)r * T + t] = run;
            run += v;
        }
        if (w == 3) tile_cnt[t] = run;
    }
}

// ------------------------------------------------------------------------------------------------
// step 3: tile starts and ranges (one workgroup, T <= BK_MAX_TILES), and the lists of the long tiles that the
// per-wave sort leaves to seg_block: list 0 holds tiles of (SEG_CAP, SEG_BLOCK_CAP] instances, list 1 longer ones.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void bk_tscan_kernel(const uint32_t *__restrict__ tile_cnt, uint32_t T,
                                                        uint32_t *__restrict__ tile_start, uint2 *__restrict__ ranges,
                                                        uint32_t *__restrict__ long_list, uint32_t *__restrict__ long_cnt) {
    __shared__ uint32_t s_w[16], s_n[2];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid < 2) s_n[tid] = 0u;
    // wave w scans tiles [w * span, (w + 1) * span), 64 at a time (coalesced)
    const uint32_t span = (T + 16 * 64 - 1) / (16 * 64) * 64;
    const uint32_t t0 = (uint32_t)w * span, t1 = min(T, t0 + span);
    uint32_t sum = 0;
    for (uint32_t t = t0 + lane; t < t1; t += 64) sum += tile_cnt[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += (uint32_t)__shfl_xor((int)sum, o);
    if (lane == 0) s_w[w] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (int i = 0; i < w; i++) run += s_w[i];
    for (uint32_t tb = t0; tb < t1; tb += 64) {
        const uint32_t t = tb + lane;
        const uint32_t v = t < t1 ? tile_cnt[t] : 0u;
        const uint32_t inc = wave_inclusive_scan(v, lane);
        if (t < t1) {
            const uint32_t st = run + inc - v;
            tile_start[t] = st;
            ranges[t] = v ? make_uint2(st, st + v) : make_uint2(0, 0);  // empty: (0, 0), as the reference
            if (v > SEG_CAP) {
                const int which = v > SEG_BLOCK_CAP;
                long_list[which * (T + 1) + atomicAdd(&s_n[which], 1u)] = t;
            }
        }
        run += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    }
    if (w == 15 && lane == 0) tile_start[T] = run;
    __syncthreads();
    if (tid < 2) long_cnt[tid] = s_n[tid];
}

// ------------------------------------------------------------------------------------------------
// step 5: per-tile sort in registers.  The wave holds 64 * E keys, lane l the E consecutive keys
// [l E, l E + E); padding keys are all ones and sort last.  Bitonic network: compare distances below E are
// register pairs, distances of E and more are lane exchanges (ds_bpermute).
// ------------------------------------------------------------------------------------------------
// Merge levels with k < E are register-only networks (compile-time directions); from k = E on, the
// direction (i & k) == 0 depends only on the lane (i = l E + r, r < E <= k), so each stage is one lane mask.
// Output: sorted_u (the expansion index of every sorted position), or, with lds_out, the padded sorted keys
// [0, 64 E) into LDS.
template <int E>
__device__ __forceinline__ void seg_sort_wave_impl(const unsigned long long *__restrict__ keys, uint32_t start,
                                                   uint32_t n, uint32_t *__restrict__ sorted_u,
                                                   unsigned long long *__restrict__ lds_out, int lane) {
    constexpr int LOGE = (E >= 64) ? 6 : (E >= 32) ? 5 : (E >= 16) ? 4 : (E >= 8) ? 3 : (E >= 4) ? 2 : (E >= 2) ? 1 : 0;
    unsigned long long x[E];
    const uint32_t base = (uint32_t)lane * E;
#pragma unroll
    for (int r = 0; r < E; r++) x[r] = (base + r < n) ? keys[start + base + r] : ~0ull;
#pragma unroll
    for (int lk = 1; lk < LOGE; lk++) {
#pragma unroll
        for (int lj = lk - 1; lj >= 0; lj--) {
#pragma unroll
            for (int r = 0; r < E; r++) {
                if (r & (1 << lj)) continue;
                const bool asc = (r & (1 << lk)) == 0;
                const unsigned long long a = x[r], c = x[r | (1 << lj)];
                const bool sw = asc ? (a > c) : (a < c);
                x[r] = sw ? c : a;
                x[r | (1 << lj)] = sw ? a : c;
            }
        }
    }
    for (int lk = LOGE > 1 ? LOGE : 1; lk <= LOGE + 6; lk++) {
        const bool asc = (base & (1u << lk)) == 0;
        for (int lj = lk - 1; lj >= LOGE; lj--) {
            const int lm = 1 << (lj - LOGE);
            const bool take_min = asc == ((lane & lm) == 0);
            const int addr = (lane ^ lm) << 2;
            // the exchanges of a batch are issued back to back: one LDS round trip per batch, not per key
            constexpr int B = E < 16 ? E : 16;
#pragma unroll
            for (int r0 = 0; r0 < E; r0 += B) {
                uint32_t ylo[B], yhi[B];
#pragma unroll
                for (int r = 0; r < B; r++) {
                    ylo[r] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)x[r0 + r]);
                    yhi[r] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(x[r0 + r] >> 32));
                }
#pragma unroll
                for (int r = 0; r < B; r++) {
                    const unsigned long long y = ((unsigned long long)yhi[r] << 32) | ylo[r];
                    x[r0 + r] = (take_min == (x[r0 + r] < y)) ? x[r0 + r] : y;
                }
            }
        }
#pragma unroll
        for (int lj = LOGE - 1; lj >= 0; lj--) {
#pragma unroll
            for (int r = 0; r < E; r++) {
                if (r & (1 << lj)) continue;
                const unsigned long long a = x[r], c = x[r | (1 << lj)];
                const bool sw = (a > c) == asc;
                x[r] = sw ? c : a;
                x[r | (1 << lj)] = sw ? a : c;
            }
        }
    }
    if (lds_out) {
#pragma unroll
        for (int r = 0; r < E; r++) lds_out[base + r] = x[r];
    } else {
#pragma unroll
        for (int r = 0; r < E; r++)
            if (base + r < n) sorted_u[start + base + r] = (uint32_t)x[r];
    }
}

template <int E>
__device__ __forceinline__ void seg_sort_wave(const unsigned long long *keys, uint32_t start, uint32_t n,
                                              uint32_t *sorted_u, int lane) {
    seg_sort_wave_impl<E>(keys, start, n, sorted_u, nullptr, lane);
}
template <int E>
__device__ __forceinline__ void seg_sort_wave_to_lds(const unsigned long long *keys, uint32_t start, uint32_t n,
                                                     unsigned long long *lds_out, int lane) {
    seg_sort_wave_impl<E>(keys, start, n, nullptr, lds_out, lane);
}

// One wave per tile of at most SEG_CAP instances (longer ones are in the long lists).  Launch slots follow
// the LPT order, so the longest tiles start first.
__global__ __launch_bounds__(256) void seg_sort_kernel(SegSortParams p) {
    const int lane = threadIdx.x & 63;
    const uint32_t slot = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (slot >= p.T) return;
    const uint32_t tile = p.tile_order ? p.tile_order[slot] : slot;
    const uint2 rg = p.ranges[tile];
    const uint32_t n = rg.y - rg.x;
    if (n == 0 || n > SEG_CAP) return;
    if (n <= 64u) seg_sort_wave<1>(p.keys, rg.x, n, p.sorted_u, lane);
    else if (n <= 128u) seg_sort_wave<2>(p.keys, rg.x, n, p.sorted_u, lane);
    else if (n <= 256u) seg_sort_wave<4>(p.keys, rg.x, n, p.sorted_u, lane);
    else seg_sort_wave<8>(p.keys, rg.x, n, p.sorted_u, lane);
}

// Workgroup sort of up to SEG_BLOCK_CAP keys: wave w sorts keys [512 w, 512 w + 512) in registers (as
// seg_sort_wave<8>) into LDS, padded with all-ones keys; then every key's position is its index in its chunk
// plus its rank in each other chunk (branchless binary searches, 8 keys per thread interleaved).
constexpr uint32_t SB_CHUNK = 512;
__device__ __forceinline__ void seg_block_sort(const unsigned long long *__restrict__ keys, uint32_t start,
                                               uint32_t n, uint32_t *__restrict__ sorted_u,
                                               unsigned long long *__restrict__ keys_out,
                                               unsigned long long *__restrict__ s_x, int w, int lane) {
    const uint32_t nch = (n + SB_CHUNK - 1) / SB_CHUNK;
    if ((uint32_t)w < nch) {
        const uint32_t c0 = (uint32_t)w * SB_CHUNK;
        seg_sort_wave_to_lds<8>(keys, start + c0, min(SB_CHUNK, n - c0), s_x + c0, lane);
    }
    __syncthreads();
    constexpr int PER = SEG_BLOCK_CAP / 256;
    unsigned long long key[PER];
    uint32_t pos[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const uint32_t e = threadIdx.x + 256u * i;
        key[i] = e < n ? s_x[e] : ~0ull;
        pos[i] = e & (SB_CHUNK - 1);
    }
    for (uint32_t c2 = 0; c2 < nch; c2++) {
        const unsigned long long *ch = s_x + c2 * SB_CHUNK;
        uint32_t idx[PER];
#pragma unroll
        for (int i = 0; i < PER; i++) idx[i] = 0;
#pragma unroll
        for (uint32_t step = SB_CHUNK / 2; step; step >>= 1) {
#pragma unroll
            for (int i = 0; i < PER; i++)
                if (ch[idx[i] + step - 1] < key[i]) idx[i] += step;
        }
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint32_t e = threadIdx.x + 256u * i;
            // the last probe decides between idx and idx + 1 (lower bound over 512 entries)
            const uint32_t lb = idx[i] + (ch[idx[i]] < key[i] ? 1u : 0u);
            if ((e >> 9) != c2) pos[i] += lb;
        }
    }
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const uint32_t e = threadIdx.x + 256u * i;
        if (e >= n) continue;
        if (keys_out) keys_out[start + pos[i]] = key[i];
        else sorted_u[start + pos[i]] = (uint32_t)key[i];
    }
    __syncthreads();  // s_x is reused by the next chunk / tile
}

// Long tiles, one workgroup each (the workgroups loop over the device-side lists, so every wave reaches the
// exit): list 0 sorted whole, list 1 in SEG_BLOCK_CAP-key chunks for seg_merge (each chunk written back
// sorted, into a second key buffer).
__global__ __launch_bounds__(256) void seg_block_kernel(SegSortParams p) {
    __shared__ unsigned long long s_x[SEG_BLOCK_CAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t n0 = p.long_cnt[0], n1 = p.long_cnt[1];
    for (uint32_t i = blockIdx.x; i < n0 + n1; i += gridDim.x) {
        const bool chunked = i >= n0;
        const uint32_t tile = chunked ? p.long_list[p.T + 1 + (i - n0)] : p.long_list[i];
        const uint2 rg = p.ranges[tile];
        const uint32_t n = rg.y - rg.x;
        for (uint32_t c0 = 0; c0 < n; c0 += SEG_BLOCK_CAP)
            seg_block_sort(p.keys, rg.x + c0, min(SEG_BLOCK_CAP, n - c0), p.sorted_u,
                           chunked ? p.keys2 : nullptr, s_x, w, lane);
    }
}

// Merge ranks of the chunk-sorted tiles of list 1: an element's sorted position is its index in its chunk plus
// the number of smaller keys in every other chunk (keys are unique).  One workgroup per tile; the tile's keys
// are staged in LDS when they fit, else searched in global memory.
constexpr uint32_t MERGE_LDS_KEYS = 8192;
__global__ __launch_bounds__(256) void seg_merge_kernel(SegSortParams p) {
    constexpr uint32_t CAP = SEG_BLOCK_CAP;
    __shared__ unsigned long long s_k[MERGE_LDS_KEYS];
    const uint32_t nh = p.long_cnt[1];
    for (uint32_t h = blockIdx.x; h < nh; h += gridDim.x) {
        const uint2 rg = p.ranges[p.long_list[p.T + 1 + h]];
        const uint32_t n = rg.y - rg.x;
        const bool in_lds = n <= MERGE_LDS_KEYS;
        __syncthreads();  // the previous tile's readers are done with s_k
        if (in_lds)
            for (uint32_t e = threadIdx.x; e < n; e += 256) s_k[e] = p.keys2[rg.x + e];
        __syncthreads();
        const unsigned long long *kk = in_lds ? s_k : p.keys2 + rg.x;
        const uint32_t nch = (n + CAP - 1) / CAP;
        for (uint32_t e = threadIdx.x; e < n; e += 256) {
            const unsigned long long key = kk[e];
            const uint32_t c = e / CAP;
            uint32_t pos = e - c * CAP;
            for (uint32_t c2 = 0; c2 < nch; c2++) {
                if (c2 == c) continue;
                const unsigned long long *ch = kk + c2 * CAP;
                uint32_t lo = 0, hi = min(CAP, n - c2 * CAP);  // first index with ch[i] >= key
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (ch[mid] < key) lo = mid + 1; else hi = mid;
                }
                pos += lo;
            }
            p.sorted_u[rg.x + pos] = (uint32_t)key;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
// 16 waves per workgroup, or 8 when the tile counters leave too little LDS for 16 waves' staging.
template <bool SCATTER>
static void launch_walk(hipStream_t s, const BucketParams &p) {
    const size_t lds = sizeof(uint32_t) * p.T;
    if (lds + 40 * 1024 <= 160 * 1024) {
        if (lds > 65536)
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&bk_walk_kernel<SCATTER, 16>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        bk_walk_kernel<SCATTER, 16><<<p.nb, 64 * 16, lds, s>>>(p);
    } else {
        if (lds > 65536)
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&bk_walk_kernel<SCATTER, 8>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        bk_walk_kernel<SCATTER, 8><<<p.nb, 64 * 8, lds, s>>>(p);
    }
}

void launch_bucket_count(hipStream_t s, const BucketParams &p) {
    launch_walk<false>(s, p);
    bk_columns_kernel<<<div_up(p.T, 64), 256, 0, s>>>(p.hist, p.nb, p.T, p.tile_cnt);
    bk_tscan_kernel<<<1, 1024, 0, s>>>(p.tile_cnt, p.T, p.tile_start, p.ranges, p.long_list, p.long_cnt);
}

void launch_bucket_scatter(hipStream_t s, const BucketParams &p) { launch_walk<true>(s, p); }

void launch_seg_sort(hipStream_t s, const SegSortParams &p) {
    if (p.T == 0) return;
    seg_block_kernel<<<std::min(p.T, 1024u), 256, 0, s>>>(p);  // the longest tiles first
    seg_sort_kernel<<<div_up(p.T, 4), 256, 0, s>>>(p);
    seg_merge_kernel<<<256, 256, 0, s>>>(p);
}

}  // namespace gsr
