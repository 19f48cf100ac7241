// gsr_bin.hip -- bucket binning: the (tile, depth, index) instance order without a global sort.
//
// The reference duplicates every (Gaussian, tile) instance with a 64-bit key (tile << 32 | depth bits) and
// radix-sorts all of them (SURVEY.md §2.1 duplicateWithKeys + cub::DeviceRadixSort, [U]); the sort is stable
// and the instances are emitted in Gaussian order, so ties in depth fall back to the Gaussian index.  Here:
//   1. bk_count    each block walks a contiguous Gaussian range (plus a share of the big Gaussians) and
//                  histograms its instances per tile in LDS: one row of the (blocks x tiles) count matrix;
//   2. bk_columns  exclusive prefix of every tile column over the blocks, and the tile totals;
//   3.             step 2 also scans the tile totals (decoupled look-back) -> tile ranges;
//   4. bk_scatter  the same walk again: each instance takes the next free slot of its tile's bucket
//                  (LDS counters seeded from the prefixes) and stores key = depth bits << 32 | u, where u is
//                  its Gaussian-major expansion index (u increases with the Gaussian index);
//   5. seg_sort    one wave per tile sorts the bucket by key in registers (bitonic network on 32-bit proxy
//                  keys, ties repaired on the full keys) and writes the expansion index of every sorted
//                  position.  Keys are unique inside a tile (one instance per Gaussian), so the order inside
//                  a bucket after step 4 does not matter and the result is exactly the reference's (tile,
//                  depth, index) order.  Tiles above SEG_CAP instances are sorted by a whole workgroup (four
//                  waves sort 512-key chunks, then merge ranks through LDS); tiles above SEG_BLOCK_CAP by
//                  a workgroup in SEG_BLOCK_CAP-key chunks placed by merge ranks; ties of the 32-bit proxy
//                  keys are repaired on the full keys by odd-even passes run to convergence.
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


// Gaussian-order exclusive scan of the kept-tile counts over [g_lo, g_hi) (the instances' Gaussian-major
// expansion offsets u): the preprocess block totals before g_lo (a multiple of 256) give the base, then a
// workgroup scan of the range, 4 Gaussians per thread per round.  The workgroup holding the last Gaussian
// also writes the total.  s_tmp: >= BKW + 1 words of scratch LDS.
template <int BKW>
__device__ void bk_instance_offsets(const BucketParams &p, uint32_t g_lo, uint32_t g_hi, uint32_t *s_tmp) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    uint32_t acc = 0;
    for (uint32_t k = tid; k < g_lo / 256; k += 64 * BKW) acc += p.block_sums[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += (uint32_t)__shfl_xor((int)acc, o);
    if (lane == 0) s_tmp[w] = acc;
    __syncthreads();
    uint32_t base = 0;
    for (int k = 0; k < BKW; k++) base += s_tmp[k];
    __syncthreads();
    for (uint32_t r0 = g_lo; r0 < g_hi; r0 += 4 * 64 * BKW) {
        const uint32_t g = r0 + 4 * (uint32_t)tid;
        uint32_t v[4], loc = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = g + k < g_hi ? p.tiles[g + k] : 0u;
            loc += v[k];
        }
        const uint32_t inc = wave_inclusive_scan(loc, lane);
        if (lane == 63) s_tmp[w] = inc;
        __syncthreads();
        uint32_t run = base + inc - loc, all = 0;
        for (int k = 0; k < BKW; k++) {
            if (k < w) run += s_tmp[k];
            all += s_tmp[k];
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (g + k < g_hi) p.inst_start[g + k] = run;
            run += v[k];
        }
        base += all;
        __syncthreads();
    }
    if (g_hi == p.P && tid == 0) p.inst_start[p.P] = base;
}

// The walk blocks in use: the range blocks, plus extra blocks (launched up to p.nb) when there are more big Gaussians
// than range blocks, so a few Gaussians with large footprints are not walked by a handful of workgroups.  Read from
// the device count by all three passes, so they agree.
__device__ __forceinline__ uint32_t bk_walk_blocks(const BucketParams &p) {
    const uint32_t nbig = *p.nbig;
    return nbig > p.nr ? min(p.nb, nbig) : p.nr;
}

template <bool SCATTER, int BKW>  // BKW: waves per workgroup
__global__ __launch_bounds__(64 * BKW) void bk_walk_kernel(BucketParams p) {
    extern __shared__ uint32_t s_tab[];   // T entries: tile counts (count) / next free bucket slot (scatter)
    __shared__ uint4 s_rec[BKW][64];      // expansion records: kept mask lo, hi, rect x | y << 16, rect width
    __shared__ uint4 s_aux[BKW][64];      // first cell pair, first expansion index, depth key, 1/width bits
    __shared__ int s_own[BKW][64];        // lane whose cell run starts at this pair of the step, else -1
    static_assert(BKW * 64 >= LPT_HIST_WORDS, "the LPT workgroup's histogram lives in s_own");
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t b = blockIdx.x, T = p.T, gx = (uint32_t)p.gx;
    if (SCATTER && b == p.nb) {  // the extra workgroup: the forward LPT order (the column pass wrote the ranges)
        // (the per-XCD map needs the 1024-thread form, which every T of lpt_append_range takes: launch_walk)
        constexpr bool xok = 64 * BKW == 1024 && sizeof(s_rec) >= 4 * (LPT_BCNT_WORDS + LPT_XCD + 17);
        lpt_order_block(p.ranges, nullptr, 0, (int)T, p.lpt_shift, p.order, reinterpret_cast<uint32_t *>(&s_own[0][0]),
                        xok ? p.order_xcd : nullptr, reinterpret_cast<uint32_t *>(&s_rec[0][0]), p.gx,
                        (int)((T + gx - 1) / gx), 4);
        return;
    }
    const uint32_t nbw = bk_walk_blocks(p);
    if (b >= nbw) return;  // uniform: a block the big rects do not need (its count row is never read)
    const bool reg = SCATTER && p.keys_reg != nullptr;  // region scatter (uniform)
    if (SCATTER && reg) {
        // region r's next free slot for this block: the region's first tile start plus this block's column prefixes of
        // its tiles (the instances of the blocks before it in every tile of the region precede it)
        const uint32_t *hrow = p.hist_pre + (size_t)b * T;
        const uint32_t nr = (T + BK_REGION - 1) / BK_REGION;
        for (uint32_t r = tid; r < nr; r += 64 * BKW) {
            const uint32_t t0 = r * BK_REGION;
            uint32_t acc = p.tile_start[t0], v[BK_REGION];
            // the region's BK_REGION prefixes loaded together (clamped index, masked sum): a rolled loop waited for
            // each load before issuing the next, BK_REGION serial round trips per region
#pragma unroll
            for (int q = 0; q < BK_REGION; q++) v[q] = hrow[min(t0 + q, T - 1)];
#pragma unroll
            for (int q = 0; q < BK_REGION; q++) acc += t0 + q < T ? v[q] : 0u;
            s_tab[r] = acc;
        }
    } else if (SCATTER) {
        const uint32_t *hrow = p.hist_pre + (size_t)b * T;
        for (uint32_t t = tid; t < T; t += 64 * BKW) s_tab[t] = p.tile_start[t] + hrow[t];
    } else {
        for (uint32_t t = tid; t < T; t += 64 * BKW) s_tab[t] = 0u;
    }
    s_own[w][lane] = -1;
    const uint32_t g_lo = min(p.P, b * p.gper), g_hi = min(p.P, g_lo + p.gper);  // empty above the range blocks
    if (!SCATTER && b < p.nr) bk_instance_offsets<BKW>(p, g_lo, g_hi, reinterpret_cast<uint32_t *>(&s_aux[0][0]));
    __syncthreads();
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
                        const unsigned long long key = ((unsigned long long)x.z << 32) | ui;
                        if (reg) {
                            const uint32_t slot = atomicAdd(&s_tab[tile / BK_REGION], 1u);
                            p.keys_reg[slot] = key | ((unsigned long long)(tile % BK_REGION) << BK_REG_SHIFT);
                        } else {
                            p.keys[atomicAdd(&s_tab[tile], 1u)] = key;
                        }
                        p.inst_gid[ui] = g0 + (uint32_t)o;
                        p.inv[ui] = INV_NONE;
                    }
                }
            }
        }
        wave_lds_sync();
    }
    const uint32_t nbig = *p.nbig;
    for (uint32_t bi = b; bi < nbig; bi += nbw) {
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
                if (reg) {
                    const uint32_t slot = atomicAdd(&s_tab[tile / BK_REGION], 1u);
                    p.keys_reg[slot] = (dk | (u0 + c)) | ((unsigned long long)(tile % BK_REGION) << BK_REG_SHIFT);
                } else {
                    p.keys[atomicAdd(&s_tab[tile], 1u)] = dk | (u0 + c);
                }
                p.inst_gid[u0 + c] = gb;
                p.inv[u0 + c] = INV_NONE;
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
// steps 2 and 3: column prefixes of the count matrix (into hist_pre), tile totals, and the tile starts / ranges
// from a decoupled look-back over the workgroups in tile order (a column workgroup that has not published is
// recomputed from the counts, wave_lookback).  A workgroup owns 64 tile columns (one per lane); its
// four waves own four contiguous quarters of the block rows.  Workgroup ids come from an atomic ticket, so a
// workgroup only waits on workgroups that started before it.  The long tiles are appended to two lists for
// the workgroup sorts: list 0 holds tiles of (SEG_CAP, SEG_BLOCK_CAP] instances, list 1 longer ones.
// ------------------------------------------------------------------------------------------------
// CW waves per workgroup split the block rows into CW contiguous slices (16: 2048 waves at 1080p instead of 512, a
// quarter of the dependent load chain per wave).
//
// Bucket layout (p.xcd_major): a tile's bucket holds the runs of the walk blocks in the order the column prefix visits
// them, and the per-tile sort makes that order irrelevant to the result.  Visiting the blocks XCD-major -- all blocks
// b = x (mod 8) first, then x + 1, ... -- puts the runs that blocks sharing an XCD write (observed round-robin
// placement, MI355X_MICROARCH.md "Workgroup dispatch") next to each other, so a 128-B line of keys is filled by one
// XCD's L2 instead of partly by several (each writing back its own dirty part): runs are ~2 instances per (block,
// tile) at 1080p.  Position r of the visiting order -> block.
__device__ __forceinline__ uint32_t bk_row_block(uint32_t r, uint32_t nb, int xcd_major) {
    if (!xcd_major) return r;
    const uint32_t q = nb >> 3, rem = nb & 7u;  // XCD groups x < rem hold q + 1 blocks, the others q
    const uint32_t big = rem * (q + 1);
    uint32_t x, k;
    if (r < big) {
        x = r / (q + 1);
        k = r - x * (q + 1);
    } else {
        const uint32_t r2 = r - big;
        x = rem + r2 / q;
        k = r2 - (x - rem) * q;
    }
    return k * 8 + x;
}

// TW tiles per workgroup (64: one lane per tile; 32: the two lane halves of a wave split the wave's rows, so twice the
// workgroups (255 at 1080p instead of 128, i.e. every CU) walk half as long a dependent load chain each).
template <int CW, int TW = 64>
__global__ __launch_bounds__(64 * CW) void bk_columns_kernel(BucketParams p) {
    static_assert(TW == 64 || TW == 32, "tiles per workgroup");
    constexpr int NH = 64 / TW;  // row halves per wave
    __shared__ uint32_t s_sum[CW][64];
    __shared__ uint32_t s_bid;
    __shared__ unsigned long long s_excl;
    const uint32_t *__restrict__ hist = p.hist;
    uint32_t *__restrict__ hist_pre = p.hist_pre;
    const uint32_t nb = bk_walk_blocks(p), T = p.T;  // the count rows the walk wrote
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int sub = lane % TW, h = lane / TW;  // the lane's tile in the workgroup, its half of the wave's rows
    if (tid == 0) s_bid = atomicAdd(p.ticket, 1u);
    if (blockIdx.x == 0 && p.lpt_bcnt)
        for (uint32_t k = (uint32_t)tid; k < LPT_BCNT_WORDS; k += blockDim.x) p.lpt_bcnt[k] = 0u;
    __syncthreads();
    const uint32_t bid = s_bid;
    const uint32_t t = bid * TW + sub;
    const uint32_t q = (nb + CW - 1) / CW, r0w = min(nb, w * q), r1w = min(nb, r0w + q);
    const uint32_t qh = (q + NH - 1) / NH, r0 = min(r1w, r0w + h * qh), r1 = min(r1w, r0 + qh);
    uint32_t sum = 0;
    const int xm = p.xcd_major;
    if (t < T) {
        uint32_t r = r0;
        for (; r + 8 <= r1; r += 8) {
            uint32_t v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) v[i] = hist[(size_t)bk_row_block(r + i, nb, xm) * T + t];
#pragma unroll
            for (int i = 0; i < 8; i++) sum += v[i];
        }
        for (; r < r1; r++) sum += hist[(size_t)bk_row_block(r, nb, xm) * T + t];
    }
    uint32_t lowsum = 0;  // the wave's rows before this lane's half (the other half's sum, for the upper half)
    if constexpr (NH == 2) {
        const uint32_t other = (uint32_t)__shfl_xor((int)sum, 32);
        lowsum = h ? other : 0u;
        sum += other;  // both halves: the wave's column sum
    }
    if (h == 0) s_sum[w][sub] = sum;
    __syncthreads();
    uint32_t tot = 0;  // tile total
#pragma unroll
    for (int i = 0; i < CW; i++) tot += s_sum[i][sub];
    if (w == 0) {
        const uint32_t tv = h == 0 ? tot : 0u;  // lanes of the upper half repeat the tiles: they count nothing here
        const uint32_t inc = wave_inclusive_scan(tv, lane);
        // fallback aggregate of column workgroup q: its TW tiles' totals, summed from the (read-only) counts
        auto agg_of = [&](uint32_t qq) -> uint64_t {
            const uint32_t tq = qq * TW + sub;
            uint64_t v = 0;
            if (tq < T && h == 0)
                for (uint32_t r = 0; r < nb; r++) v += hist[(size_t)r * T + tq];
            return wave_sum_u64(v);
        };
        const uint64_t excl = wave_lookback(p.tile_status, bid, (uint64_t)__builtin_amdgcn_readlane((int)inc, 63),
                                            lane, p.err, p.lb_patience, p.lb_force != 0, agg_of);
        const bool mine = t < T && h == 0;
        if (mine) {
            const uint32_t st = (uint32_t)(excl + inc - tot);
            p.tile_start[t] = st;
            p.ranges[t] = tot ? make_uint2(st, st + tot) : make_uint2(0, 0);  // empty: (0, 0), as the reference
            p.tile_next[t] = st;
            if (t % BK_REGION == 0) p.reg_start[t / BK_REGION] = st;  // compact region starts (the region partition)
            p.tile_last[t] = 0u;
            p.tile_loaded[t] = 0u;
            if (t == T - 1) {
                p.tile_start[T] = st + tot;
                p.reg_start[(T + BK_REGION - 1) / BK_REGION] = st + tot;
            }
        }
        const bool l0 = mine && tot > SEG_CAP && tot <= SEG_BLOCK_CAP, l1 = mine && tot > SEG_BLOCK_CAP;
        const uint64_t m0 = __ballot(l0), m1 = __ballot(l1);
        uint32_t b0 = 0, b1 = 0;
        if (lane == 0) {
            if (m0) b0 = atomicAdd(&p.long_cnt[0], (uint32_t)__popcll(m0));
            if (m1) b1 = atomicAdd(&p.long_cnt[1], (uint32_t)__popcll(m1));
        }
        b0 = __builtin_amdgcn_readfirstlane(b0);
        b1 = __builtin_amdgcn_readfirstlane(b1);
        const uint64_t lt = lanemask_lt(lane);
        if (l0) p.long_list[b0 + __popcll(m0 & lt)] = t;
        if (l1) p.long_list[(T + 1) + b1 + __popcll(m1 & lt)] = t;
    }
    uint32_t run = lowsum;
    for (int i = 0; i < w; i++) run += s_sum[i][sub];
    if (t < T) {
        uint32_t r = r0;
        for (; r + 8 <= r1; r += 8) {
            uint32_t v[8];
            size_t row[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                row[i] = (size_t)bk_row_block(r + i, nb, xm) * T + t;
                v[i] = hist[row[i]];
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                hist_pre[row[i]] = run;
                run += v[i];
            }
        }
        for (; r < r1; r++) {
            const size_t row = (size_t)bk_row_block(r, nb, xm) * T + t;
            const uint32_t v = hist[row];
            hist_pre[row] = run;
            run += v;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Region scatter, second step (p.keys_reg): the region-grouped keys move into their tile buckets.  The direct scatter
// stores every key at a random slot of its tile's bucket, where a block's run is ~2 keys at 1080p (256 blocks, 8160
// tiles): 4.2 M partial-line stores (2.45x write amplification at cfg 3); into regions (BK_REGION consecutive tile ids)
// the runs are 16x longer.  Here every workgroup takes a fixed chunk of PART_CHUNK region-grouped keys (so a dense
// region is spread over many workgroups): a counting sort of the chunk by (region, tile) bin in LDS, one global atomic
// per non-empty bin for its slots in the tile's bucket (tile_next), then each bin's run stored contiguously.  A chunk
// over more than PART_MAXR regions (sparse ones) sends its keys one by one.  Bucket order is arbitrary (the per-tile
// sorts make it irrelevant).
#ifndef GSR_PART_THREADS  // chunk shape (overridable for library A/B builds, tools/build_variant.py)
#define GSR_PART_THREADS 256
#endif
#ifndef GSR_PART_ITEMS
#define GSR_PART_ITEMS 4
#endif
constexpr int PART_THREADS = GSR_PART_THREADS;
constexpr int PART_ITEMS = GSR_PART_ITEMS;
constexpr uint32_t PART_CHUNK = PART_THREADS * PART_ITEMS;
#ifndef GSR_PART_MAXR
#define GSR_PART_MAXR 4
#endif
constexpr uint32_t PART_MAXR = GSR_PART_MAXR;
constexpr uint32_t PART_BINS = PART_MAXR * BK_REGION;
static_assert(PART_BINS % 64 == 0 && PART_BINS >= 64, "the bin scan gives each lane of one wave PART_BINS / 64 bins");
// region of sorted position i: the last r < n with rs[r] <= i (rs non-decreasing, rs[0] <= i)
__device__ __forceinline__ uint32_t bk_region_of(const uint32_t *rs, uint32_t lo, uint32_t n, uint32_t i) {
    uint32_t hi = n - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (rs[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}
__global__ __launch_bounds__(PART_THREADS) void bk_partition_kernel(BucketParams p) {
    __shared__ unsigned long long s_keys[PART_CHUNK];
    __shared__ uint16_t s_bin[PART_CHUNK];
    __shared__ uint32_t s_cnt[PART_BINS], s_lstart[PART_BINS], s_gbase[PART_BINS];
    __shared__ uint32_t s_rstart[PART_MAXR + 1];
    __shared__ uint32_t s_nle[2];
    constexpr unsigned long long TB_MASK = (unsigned long long)(BK_REGION - 1) << BK_REG_SHIFT;
    const uint32_t T = p.T, nr = (T + BK_REGION - 1) / BK_REGION, R = p.tile_start[T];
    const uint32_t c0 = blockIdx.x * PART_CHUNK;
    if (c0 >= R) return;  // workgroup-uniform
    const uint32_t n = min(PART_CHUNK, R - c0);
    const int tid = threadIdx.x;
    unsigned long long k[PART_ITEMS];  // the chunk's keys, loaded first (they do not depend on the region search)
#pragma unroll
    for (int q = 0; q < PART_ITEMS; q++)  // unconditional loads (clamped index): issued together, one wait
        k[q] = p.keys_reg[c0 + min((uint32_t)(q * PART_THREADS + tid), n - 1)];
    if (tid < 64) {  // the chunk's first and last regions: 64-probe wave searches over the compact region starts
        const uint32_t rlo = wave_last_le(p.reg_start, nr - 1, c0, tid);
        const uint32_t rhi = wave_last_le(p.reg_start, nr - 1, c0 + n - 1, tid);
        if (tid == 0) {
            s_nle[0] = rlo;
            s_nle[1] = rhi;
        }
    }
    __syncthreads();
    const uint32_t rlo = s_nle[0], nreg = s_nle[1] - rlo + 1;  // regions rlo .. rlo + nreg - 1 hold the chunk
    if (nreg > PART_MAXR) {  // sparse regions: every key takes its slot alone
        for (uint32_t i = c0 + tid; i < c0 + n; i += PART_THREADS) {
            const unsigned long long k = p.keys_reg[i];
            const uint32_t t = bk_region_of(p.reg_start, rlo, rlo + nreg, i) * BK_REGION +
                               (uint32_t)((k & TB_MASK) >> BK_REG_SHIFT);
            p.keys[atomicAdd(&p.tile_next[t], 1u)] = k & ~TB_MASK;
        }
        return;
    }
    for (uint32_t j = tid; j <= nreg; j += PART_THREADS) s_rstart[j] = p.reg_start[rlo + j];
    for (uint32_t j = tid; j < nreg * BK_REGION; j += PART_THREADS) s_cnt[j] = 0u;
    __syncthreads();
    uint32_t bin[PART_ITEMS], rank[PART_ITEMS];
#pragma unroll
    for (int q = 0; q < PART_ITEMS; q++) {
        const uint32_t i = (uint32_t)(q * PART_THREADS + tid);
        rank[q] = 0xffffffffu;
        bin[q] = 0;
        if (i < n) {
            uint32_t j = 0;  // region of the key within the chunk's regions
#pragma unroll
            for (uint32_t step = PART_MAXR / 2; step; step >>= 1)
                if (j + step < nreg && s_rstart[j + step] <= c0 + i) j += step;
            bin[q] = j * BK_REGION + (uint32_t)((k[q] & TB_MASK) >> BK_REG_SHIFT);
            rank[q] = atomicAdd(&s_cnt[bin[q]], 1u);
        }
    }
    __syncthreads();
    const uint32_t nbins = nreg * BK_REGION;
    if (tid < 64) {  // chunk-local bin starts (one wave, PART_BINS / 64 bins per lane), then each bin's global slots
        constexpr int PER = PART_BINS / 64;
        uint32_t c[PER], sum = 0;
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const uint32_t b = (uint32_t)(tid * PER + q);
            c[q] = b < nbins ? s_cnt[b] : 0u;
            sum += c[q];
        }
        uint32_t run = wave_inclusive_scan(sum, tid) - sum;
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const uint32_t b = (uint32_t)(tid * PER + q);
            if (b < nbins) {
                s_lstart[b] = run;
                if (c[q]) s_gbase[b] = atomicAdd(&p.tile_next[(rlo + b / BK_REGION) * BK_REGION + b % BK_REGION], c[q]);
            }
            run += c[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PART_ITEMS; q++)
        if (rank[q] != 0xffffffffu) {
            const uint32_t pos = s_lstart[bin[q]] + rank[q];
            s_keys[pos] = k[q] & ~TB_MASK;
            s_bin[pos] = (uint16_t)bin[q];
        }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PART_ITEMS; q++) {  // bin by bin, contiguous: coalesced stores
        const uint32_t i = (uint32_t)(q * PART_THREADS + tid);
        if (i < n) {
            const uint32_t b = s_bin[i];
            p.keys[s_gbase[b] + (i - s_lstart[b])] = s_keys[i];
        }
    }
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
    // every lane loads (a clamped index past n): loads in a branch each wait for their data before the next
    // is issued, E serial memory round trips per sort
#pragma unroll
    for (int r = 0; r < E; r++) x[r] = keys[start + min(base + r, n - 1)];
#pragma unroll
    for (int r = 0; r < E; r++) x[r] = (base + r < n) ? x[r] : ~0ull;
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

// 32-bit form of the same network.  Within one sort the keys are ranked by a 32-bit proxy
//   k32 = ((depth bits - min depth bits) >> sh) << IDXB | index,   IDXB = log2(64 E),
// with sh chosen so the depth offsets fit 32 - IDXB bits: unique keys, compare-exchanges are v_min/v_max
// pairs and lane exchanges one ds_bpermute (about 2.5x fewer VALU ops than 64-bit keys).  The proxy orders
// exactly like (depth, u) unless two keys share a quantised depth (~8 % of 512-key sorts at cfg 3).  Such ties
// (a ballot over adjacent sorted keys) are put in order after the gather by odd-even transposition passes on
// the full keys: keys of different quantised depth are already ordered, so only the tie runs move, and a run of L
// keys settles within L pass pairs (odd-even transposition sorts any n keys in n phases; the loop stops at the first
// pass pair without a swap, and at n pass pairs at the latest).  Round 4 gave up after 8 pass pairs and re-sorted
// such tiles on the 64-bit keys in a second launch (seg_huge), whose ~5-us floor every step paid; a tie run of
// hundreds of keys (duplicated Gaussians) now costs its wave ~20 us once.  Descending merge halves run on
// complemented keys, so
// every stage of a merge level is an ascending min / max.  scratch: 64 E keys of LDS (the full keys, gathered
// back by index after the sort).
template <int E>
__device__ __forceinline__ void seg_sort_wave32(const unsigned long long *__restrict__ keys, uint32_t start, uint32_t n,
                                                unsigned long long *__restrict__ scratch, int lane,
                                                unsigned long long (&out)[E]) {
    constexpr int LOGE = (E >= 8) ? 3 : (E >= 4) ? 2 : (E >= 2) ? 1 : 0;
    constexpr int IDXB = LOGE + 6;
    const uint32_t base = (uint32_t)lane * E;
    unsigned long long x64[E];
    uint32_t dmin = 0xffffffffu, dmax = 0u;
#pragma unroll
    for (int r = 0; r < E; r++) x64[r] = keys[start + min(base + r, n - 1)];  // unconditional loads (as above)
#pragma unroll
    for (int r = 0; r < E; r++) {
        const bool valid = base + r < n;
        x64[r] = valid ? x64[r] : ~0ull;
        scratch[base + r] = x64[r];
        const uint32_t d = (uint32_t)(x64[r] >> 32);
        if (valid) {
            dmin = min(dmin, d);
            dmax = max(dmax, d);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        dmin = min(dmin, (uint32_t)__shfl_xor((int)dmin, o));
        dmax = max(dmax, (uint32_t)__shfl_xor((int)dmax, o));
    }
    const uint32_t range = dmax - dmin;
    const int bits = range ? 32 - __builtin_clz(range) : 0;
    const int sh = bits > 32 - IDXB ? bits - (32 - IDXB) : 0;
    uint32_t x[E];
#pragma unroll
    for (int r = 0; r < E; r++)
        x[r] = (base + r < n) ? ((((uint32_t)(x64[r] >> 32) - dmin) >> sh) << IDXB) | (base + r) : 0xffffffffu;
    // merge levels k < E: registers only, compile-time directions
#pragma unroll
    for (int lk = 1; lk < LOGE; lk++) {
#pragma unroll
        for (int lj = lk - 1; lj >= 0; lj--) {
#pragma unroll
            for (int r = 0; r < E; r++) {
                if (r & (1 << lj)) continue;
                const uint32_t a = x[r], c = x[r | (1 << lj)];
                const uint32_t lo = min(a, c), hi = max(a, c);
                const bool asc = (r & (1 << lk)) == 0;
                x[r] = asc ? lo : hi;
                x[r | (1 << lj)] = asc ? hi : lo;
            }
        }
    }
    for (int lk = LOGE > 1 ? LOGE : 1; lk <= LOGE + 6; lk++) {
        const uint32_t flip = (base & (1u << lk)) ? 0xffffffffu : 0u;  // descending half: complemented keys
#pragma unroll
        for (int r = 0; r < E; r++) x[r] ^= flip;
        for (int lj = lk - 1; lj >= LOGE; lj--) {
            const int lm = 1 << (lj - LOGE);
            const bool lower = (lane & lm) == 0;
            const int addr = (lane ^ lm) << 2;
            uint32_t y[E];
#pragma unroll
            for (int r = 0; r < E; r++) y[r] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)x[r]);
#pragma unroll
            for (int r = 0; r < E; r++) x[r] = lower ? min(x[r], y[r]) : max(x[r], y[r]);
        }
#pragma unroll
        for (int lj = LOGE - 1; lj >= 0; lj--) {
#pragma unroll
            for (int r = 0; r < E; r++) {
                if (r & (1 << lj)) continue;
                const uint32_t a = x[r], c = x[r | (1 << lj)];
                x[r] = min(a, c);
                x[r | (1 << lj)] = max(a, c);
            }
        }
#pragma unroll
        for (int r = 0; r < E; r++) x[r] ^= flip;
    }
    // ties of the quantised depth between adjacent sorted keys (both real)
    const uint32_t next0 = (uint32_t)__shfl_down((int)x[0], 1);
    bool tie = false;
#pragma unroll
    for (int r = 0; r < E; r++) {
        const uint32_t nx = r + 1 < E ? x[r + 1] : next0;
        const bool both = base + r + 1 < n && (r + 1 < E || lane < 63);
        tie |= both && (x[r] >> IDXB) == (nx >> IDXB);
    }
    const bool any_tie = __ballot(tie) != 0;
    wave_lds_sync();  // scratch written by every lane above
#pragma unroll
    for (int r = 0; r < E; r++) out[r] = scratch[x[r] & ((1u << IDXB) - 1u)];
    if (!any_tie) return;
    for (uint32_t it = 0; it < n; it++) {
        bool sw = false;
        auto ce = [&](unsigned long long &a, unsigned long long &b) {
            const bool s = b < a;
            const unsigned long long lo = s ? b : a, hi = s ? a : b;
            a = lo;
            b = hi;
            sw |= s;
        };
        // even phase: pairs (2m, 2m + 1)
        if (E == 1) {
            const unsigned long long y = __shfl_xor(out[0], 1);
            const bool lower = (lane & 1) == 0;
            const unsigned long long v = lower ? (y < out[0] ? y : out[0]) : (y > out[0] ? y : out[0]);
            sw |= v != out[0];
            out[0] = v;
        } else {
#pragma unroll
            for (int r = 0; r + 1 < E; r += 2) ce(out[r], out[r + 1]);
        }
        // odd phase: pairs (2m + 1, 2m + 2); the pair across lanes l, l + 1 is (l E + E - 1, (l + 1) E)
#pragma unroll
        for (int r = 1; r + 1 < E; r += 2) ce(out[r], out[r + 1]);
        const unsigned long long nx = __shfl_down(out[0], 1), pv = __shfl_up(out[E - 1], 1);
        // E == 1: lane l is one element, in the pair (l, l + 1) when l is odd, (l - 1, l) when even
        const bool low_end = E > 1 || (lane & 1), high_end = E > 1 || !(lane & 1);
        if (low_end && lane < 63 && nx < out[E - 1]) {
            out[E - 1] = nx;
            sw = true;
        }
        if (high_end && lane > 0 && out[0] < pv) {
            out[0] = pv;
            sw = true;
        }
        if (!__ballot(sw)) return;
    }
}

// Wrappers.  P32: the proxy-key sort; P32 = false: the 64-bit network (knob "seg32" 0, the A/B reference).
template <int E, bool P32>
__device__ __forceinline__ void seg_sort_wave(const unsigned long long *keys, uint32_t start, uint32_t n,
                                              uint32_t *sorted_u, int lane, unsigned long long *scratch) {
    if (!P32) {
        seg_sort_wave_impl<E>(keys, start, n, sorted_u, nullptr, lane);
        return;
    }
    unsigned long long y[E];
    seg_sort_wave32<E>(keys, start, n, scratch, lane, y);
    const uint32_t base = (uint32_t)lane * E;
#pragma unroll
    for (int r = 0; r < E; r++)
        if (base + r < n) sorted_u[start + base + r] = (uint32_t)y[r];
}
// sorted (padded) keys into lds_out, which is also the scratch
template <int E, bool P32>
__device__ __forceinline__ void seg_sort_wave_to_lds(const unsigned long long *keys, uint32_t start, uint32_t n,
                                                     unsigned long long *lds_out, int lane) {
    if (!P32) {
        seg_sort_wave_impl<E>(keys, start, n, nullptr, lds_out, lane);
        return;
    }
    unsigned long long y[E];
    seg_sort_wave32<E>(keys, start, n, lds_out, lane, y);
    wave_lds_sync();  // every lane's gathers done before the scratch is overwritten
    const uint32_t base = (uint32_t)lane * E;
#pragma unroll
    for (int r = 0; r < E; r++) lds_out[base + r] = y[r];
}

// Workgroup sort of up to 16 x 512 keys in LDS: the waves sort 512-key chunks in registers (as
// seg_sort_wave<8>) into LDS, padded with all-ones keys; then every key's position is its index in its chunk
// plus its lower bound in each other chunk (seg_merge_ranks).
constexpr uint32_t SB_CHUNK = 512;
constexpr uint32_t SB_WAVE_SCRATCH = SEG_BLOCK_CAP / 4;  // a wave's share of the workgroup's key LDS

// Merge ranks: branchless binary searches over the padded 512-key chunks, PER keys per thread interleaved.
// Key slot i of a thread lies in chunk e0 / 512 + i / 2, and visits the other chunks by rotation (own + d), so
// no search is spent on a key's own chunk; slots past n search harmlessly (chunk 0) and are not written.
template <int PER>
__device__ __forceinline__ void seg_merge_ranks(const unsigned long long *__restrict__ s_x, uint32_t n, uint32_t nch,
                                                uint32_t start, uint32_t *__restrict__ sorted_u,
                                                unsigned long long *__restrict__ keys_out) {
    const uint32_t span = nch * SB_CHUNK;
    for (uint32_t e0 = 0; e0 < n; e0 += 256 * PER) {
        unsigned long long key[PER];
        uint32_t pos[PER], own[PER];
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint32_t e = e0 + threadIdx.x + 256u * i;
            key[i] = e < n ? s_x[e] : ~0ull;
            pos[i] = e & (SB_CHUNK - 1);
            own[i] = e < n ? (e & ~(SB_CHUNK - 1)) : 0u;
        }
        for (uint32_t d = SB_CHUNK; d < span; d += SB_CHUNK) {
            uint32_t lo[PER], idx[PER];
#pragma unroll
            for (int i = 0; i < PER; i++) {
                lo[i] = own[i] + d;
                if (lo[i] >= span) lo[i] -= span;
                idx[i] = lo[i];
            }
#pragma unroll
            for (uint32_t step = SB_CHUNK / 2; step; step >>= 1) {
#pragma unroll
                for (int i = 0; i < PER; i++)
                    if (s_x[idx[i] + step - 1] < key[i]) idx[i] += step;
            }
#pragma unroll
            for (int i = 0; i < PER; i++)  // the last probe decides between idx and idx + 1
                pos[i] += idx[i] - lo[i] + (s_x[idx[i]] < key[i] ? 1u : 0u);
        }
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint32_t e = e0 + threadIdx.x + 256u * i;
            if (e >= n) continue;
            if (keys_out) keys_out[start + pos[i]] = key[i];
            else sorted_u[start + pos[i]] = (uint32_t)key[i];
        }
    }
}

template <bool P32>
__device__ __forceinline__ void seg_lds_sort(const unsigned long long *__restrict__ keys, uint32_t start, uint32_t n,
                                             uint32_t *__restrict__ sorted_u, unsigned long long *__restrict__ keys_out,
                                             unsigned long long *__restrict__ s_x, int w, int lane,
                                             uint32_t *t_mid = nullptr) {
    const uint32_t nch = (n + SB_CHUNK - 1) / SB_CHUNK;
    for (uint32_t c = (uint32_t)w; c < nch; c += 4) {
        const uint32_t c0 = c * SB_CHUNK;
        seg_sort_wave_to_lds<8, P32>(keys, start + c0, min(SB_CHUNK, n - c0), s_x + c0, lane);
    }
    __syncthreads();
    if (t_mid) *t_mid = stamp_now();
    if (n <= 256u * 4u) seg_merge_ranks<4>(s_x, n, nch, start, sorted_u, keys_out);
    else seg_merge_ranks<8>(s_x, n, nch, start, sorted_u, keys_out);
    __syncthreads();  // s_x is reused by the next chunk / tile
}

// A tile above SEG_BLOCK_CAP instances, by one workgroup: SEG_BLOCK_CAP-key chunks sorted in LDS and written to
// keys2, then every key placed by its rank in each other chunk (binary searches over the workgroup's own stores,
// ordered by a device-scope fence).
template <bool P32>
__device__ void seg_tile_chunked(const SegSortParams &p, uint2 rg, uint32_t n, unsigned long long *s_x, int w,
                                 int lane) {
    for (uint32_t c0 = 0; c0 < n; c0 += SEG_BLOCK_CAP)
        seg_lds_sort<P32>(p.keys, rg.x + c0, min(SEG_BLOCK_CAP, n - c0), nullptr, p.keys2, s_x, w, lane);
    __threadfence();
    __syncthreads();
    const unsigned long long *kk = p.keys2 + rg.x;
    const uint32_t nch = (n + SEG_BLOCK_CAP - 1) / SEG_BLOCK_CAP;
    for (uint32_t e = threadIdx.x; e < n; e += 256) {
        const unsigned long long key = kk[e];
        const uint32_t c = e / SEG_BLOCK_CAP;
        uint32_t pos = e - c * SEG_BLOCK_CAP;
        for (uint32_t c2 = 0; c2 < nch; c2++) {
            if (c2 == c) continue;
            const unsigned long long *ch = kk + c2 * SEG_BLOCK_CAP;
            uint32_t lo = 0, hi = min(SEG_BLOCK_CAP, n - c2 * SEG_BLOCK_CAP);  // first index with ch[i] >= key
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (ch[mid] < key) lo = mid + 1; else hi = mid;
            }
            pos += lo;
        }
        p.sorted_u[rg.x + pos] = (uint32_t)key;
    }
    __syncthreads();
}

// Every tile, in one persistent launch (the workgroups loop over the tiles, whose counts are only known on the
// device, so every wave reaches the exit), on 32-bit proxy keys (P32, else on the 64-bit keys: the A/B reference,
// knob "seg32"):
//   1. tiles above SEG_CAP instances, one workgroup each: up to SEG_BLOCK_CAP in LDS (seg_lds_sort), longer ones in
//      chunks (seg_tile_chunked).  With the LPT order they are exactly its first long_cnt[0] + long_cnt[1] slots
//      (SEG_CAP + 1 is a multiple of the LPT bucket width), taken longest first; without it, lists 0 and 1;
//   2. then the short tiles, one wave each (seg_sort_wave), again longest first.
// Proxy-key ties are repaired in place (seg_sort_wave32), so no second launch is needed (round 4 handed unresolved
// tie tiles, and the tiles above SEG_BLOCK_CAP, to a seg_huge launch whose ~5-us floor every step paid).
template <bool P32, int MIN_WAVES = 1>
__global__ __launch_bounds__(256, MIN_WAVES) void seg_sort_kernel(SegSortParams p) {
    __shared__ unsigned long long s_x[SEG_BLOCK_CAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t n0 = p.long_cnt[0], nlong = n0 + p.long_cnt[1];
    for (uint32_t i = blockIdx.x; i < nlong; i += gridDim.x) {
        const uint32_t tile = p.tile_order ? p.tile_order[i] : i < n0 ? p.long_list[i] : p.long_list[p.T + 1 + (i - n0)];
        const uint2 rg = p.ranges[tile];
        const uint32_t n = rg.y - rg.x;
        if (n <= SEG_CAP) continue;  // workgroup-uniform
        if (n > SEG_BLOCK_CAP) {
            seg_tile_chunked<P32>(p, rg, n, s_x, w, lane);
            continue;
        }
        const uint32_t t0 = p.stamps ? stamp_now() : 0u;
        uint32_t t1 = 0;
        seg_lds_sort<P32>(p.keys, rg.x, n, p.sorted_u, nullptr, s_x, w, lane, p.stamps ? &t1 : nullptr);
        if (p.stamps && threadIdx.x == 0 && i < (uint32_t)STAMP_SLOTS) p.stamps[i] = make_uint4(t0, t1, stamp_now(), n);
    }
    const uint32_t s0 = p.tile_order ? nlong : 0u;
    // waves in the order workgroups finished phase 1 would be better balanced, but a shared work counter
    // serialises ~10^4 device-scope atomics (measured 2x slower): a static round robin instead
    for (uint32_t j = s0 + blockIdx.x * 4 + (uint32_t)w; j < p.T; j += gridDim.x * 4) {
        const uint32_t tile = p.tile_order ? p.tile_order[j] : j;
        const uint2 rg = p.ranges[tile];
        const uint32_t n = rg.y - rg.x;
        if (n == 0 || n > SEG_CAP) continue;  // wave-uniform
        unsigned long long *scratch = s_x + w * SB_WAVE_SCRATCH;
        if (n <= 64u) seg_sort_wave<1, P32>(p.keys, rg.x, n, p.sorted_u, lane, scratch);
        else if (n <= 128u) seg_sort_wave<2, P32>(p.keys, rg.x, n, p.sorted_u, lane, scratch);
        else if (n <= 256u) seg_sort_wave<4, P32>(p.keys, rg.x, n, p.sorted_u, lane, scratch);
        else seg_sort_wave<8, P32>(p.keys, rg.x, n, p.sorted_u, lane, scratch);
    }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
// 16 waves per workgroup, or 8 when the tile counters leave too little LDS for 16 waves' staging.
template <bool SCATTER>
static void launch_walk(hipStream_t s, const BucketParams &p, uint32_t grid) {
    const size_t lds = sizeof(uint32_t) * p.T;
    if (lds + 40 * 1024 <= 160 * 1024) {
        if (lds > 65536)
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&bk_walk_kernel<SCATTER, 16>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        bk_walk_kernel<SCATTER, 16><<<grid, 64 * 16, lds, s>>>(p);
    } else {
        if (lds > 65536)
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&bk_walk_kernel<SCATTER, 8>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        bk_walk_kernel<SCATTER, 8><<<grid, 64 * 8, lds, s>>>(p);
    }
}

void launch_bucket_count(hipStream_t s, const BucketParams &p) {
    launch_walk<false>(s, p, p.nb);
    // "bk_colt" 32 (default): 32 tiles per column workgroup, the lane halves splitting the rows; 64: one lane per tile
    if (tuning("bk_colw", 16) >= 16 && tuning("bk_colt", 32) == 32) bk_columns_kernel<16, 32><<<div_up(p.T, 32), 1024, 0, s>>>(p);
    else if (tuning("bk_colw", 16) >= 16) bk_columns_kernel<16><<<div_up(p.T, 64), 1024, 0, s>>>(p);
    else bk_columns_kernel<4><<<div_up(p.T, 64), 256, 0, s>>>(p);
}

// plus one workgroup for the forward LPT order when p.order is set
void launch_bucket_scatter(hipStream_t s, const BucketParams &p) {
    // (order_xcd is set only within lpt_append_range, T <= 16384: launch_walk's 1024-thread form, which builds it)
    launch_walk<true>(s, p, p.nb + (p.order ? 1u : 0u));
    // one workgroup per PART_CHUNK keys of the upper bound on R the binning buffer was carved for (extra ones exit)
    if (p.keys_reg) bk_partition_kernel<<<div_up(p.R, PART_CHUNK), PART_THREADS, 0, s>>>(p);
}

void launch_seg_sort(hipStream_t s, const SegSortParams &p0) {
    if (p0.T == 0) return;
    SegSortParams p = p0;
    p.stamps = tuning("stamp", 0) ? stamp_buffer(2) : nullptr;
    // one wave per tile up to 16384 tiles (cfg 3, 8160 tiles: 2040 workgroups, seg_sort 0.0490 -> 0.0472 ms against a
    // 1536-workgroup cap, profiles/r6ai_ab_launch_knobs_cfg3.txt)
    const uint32_t grid = std::min(div_up(p.T, 4), (uint32_t)tuning("seg_grid", 4096));
    const int minw = tuning("seg_minw", 6);  // 80 VGPRs: 0.053 vs 0.060 ms at 4 waves/SIMD
    if (tuning("seg32", 1) && minw >= 7) seg_sort_kernel<true, 7><<<grid, 256, 0, s>>>(p);
    else if (tuning("seg32", 1) && minw == 6) seg_sort_kernel<true, 6><<<grid, 256, 0, s>>>(p);
    else if (tuning("seg32", 1) && minw == 5) seg_sort_kernel<true, 5><<<grid, 256, 0, s>>>(p);
    else if (tuning("seg32", 1)) seg_sort_kernel<true><<<grid, 256, 0, s>>>(p);
    else seg_sort_kernel<false><<<grid, 256, 0, s>>>(p);
}

}  // namespace gsr
