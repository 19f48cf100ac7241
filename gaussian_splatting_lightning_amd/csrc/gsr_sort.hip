// gsr_sort.hip -- device-wide exclusive scan and LSD radix sort for the binning stage.
//
// Replaces the reference's cub::DeviceScan::InclusiveSum over tiles_touched and
// cub::DeviceRadixSort::SortPairs over (tile << 32 | depth) keys.  The MI355X design
// splits that 45-bit sort in two cheaper ones (see DESIGN.md "Binning"):
//   * a 32-bit depth sort over the P Gaussians (4 passes over P, not over the ~6.5x larger instance list),
//   * a stable tile-id sort (ceil(log2 T) bits, 2 passes at 1080p) over the instances, which are
//     expanded in depth order, so the result equals the reference's stable (tile, depth, index) order.
// Each pass is histogram -> scan of the [block][digit] counts in (digit, block) order -> stable scatter.  The scatter ranks
// keys inside a wave with eight 64-lane ballots (wave64 multisplit), keeps per-wave digit counters in
// LDS, stages the block's output in LDS, and writes each digit's run contiguously.
#include "gsr_kernels.h"

namespace gsr {

// ------------------------------------------------------------------------------------------------
// exclusive scan
// ------------------------------------------------------------------------------------------------
template <bool GATHER>
__device__ __forceinline__ uint32_t scan_load(const uint32_t *__restrict__ in, const uint32_t *__restrict__ idx,
                                              uint32_t j) {
    return GATHER ? in[idx[j]] : in[j];
}

// Single-kernel exclusive scan with decoupled look-back (one launch instead of three).  Block ids come from an
// atomic ticket so a block only waits on blocks that started before it; its first wave inspects 64
// predecessors per round trip.  Status words: 2-bit flag | 62-bit inclusive/aggregate sum.

template <bool GATHER, int NT = 256, int PER = SCAN_TILE / 256>
__global__ __launch_bounds__(NT) void scan_lookback_kernel(const uint32_t *__restrict__ in,
                                                            const uint32_t *__restrict__ idx, uint32_t n,
                                                            uint32_t *__restrict__ out, uint64_t *__restrict__ status,
                                                            uint32_t *__restrict__ ticket,
                                                            uint32_t *__restrict__ flags, uint32_t patience,
                                                            int force) {
    // NT threads x PER items per workgroup (1024 x 16: a quarter of the workgroups, so the look-back chain is shorter)
    constexpr int TILE = NT * PER, NW = NT / 64;
    __shared__ uint32_t s_bid, s_w[NW];
    __shared__ unsigned long long s_excl;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_bid = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t bid = s_bid;
    const uint32_t base = bid * TILE + tid * PER;
    uint32_t v[PER];
    uint32_t local = 0;
    static_assert(PER % 4 == 0, "16-B loads");
    const bool full = !GATHER && base + PER <= n;  // 16-B loads and stores (base is a multiple of PER)
    if (full) {
#pragma unroll
        for (int q = 0; q < PER / 4; q++) {
            const uint4 x = reinterpret_cast<const uint4 *>(in + base)[q];
            v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const uint32_t j = base + k;
            v[k] = j < n ? scan_load<GATHER>(in, idx, j) : 0u;
        }
    }
#pragma unroll
    for (int k = 0; k < PER; k++) local += v[k];
    const uint32_t inc = wave_inclusive_scan(local, lane);
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    if (w == 0) {
        uint64_t agg = 0;
#pragma unroll
        for (int i = 0; i < NW; i++) agg += s_w[i];
        // fallback aggregate of block q: the sum of its TILE inputs (the input is never written here)
        auto agg_of = [&](uint32_t q) -> uint64_t {
            uint64_t a = 0;
            for (uint32_t j = q * TILE + lane; j < min(n, (q + 1) * TILE); j += 64)
                a += scan_load<GATHER>(in, idx, j);
            return wave_sum_u64(a);
        };
        const uint64_t excl = wave_lookback(status, bid, agg, lane, flags, patience, force != 0, agg_of);
        if (lane == 0) {
            s_excl = excl;
            if (n >= bid * TILE && n < bid * TILE + TILE) {  // the block holding element n writes the total
                const uint64_t tot = excl + agg;
                out[n] = (uint32_t)tot;
                if (tot > 0xffffffffull) atomicOr(flags, 1u);
            }
        }
    }
    __syncthreads();
    uint64_t run = s_excl + (uint64_t)(inc - local);
    for (int i = 0; i < w; i++) run += s_w[i];
    uint32_t o[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        o[k] = (uint32_t)run;
        run += v[k];
    }
    if (full) {
#pragma unroll
        for (int q = 0; q < PER / 4; q++)
            reinterpret_cast<uint4 *>(out + base)[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < PER; k++)
            if (base + k < n) out[base + k] = o[k];
    }
}

void launch_exclusive_scan_lookback(hipStream_t s, const uint32_t *in, const uint32_t *idx, uint32_t n, uint32_t *out,
                                    uint64_t *status, uint32_t *ticket, uint32_t *flags) {
    // status (div_up(n + 1, SCAN_TILE) words) and *ticket must be zero (cleared with the forward's counters)
    const uint32_t pat = (uint32_t)tuning("lb_patience", 1 << 16);
    const int force = tuning("lb_force", 0);
    const int snt = tuning("scan_nt", 2048);  // 256: 256 x 16 per workgroup
    if (snt == 2048) {  // 1024 threads x 32 items
        const uint32_t nb8 = div_up(n + 1, (uint32_t)(8 * SCAN_TILE));
        if (idx)
            scan_lookback_kernel<true, 1024, 32><<<nb8, 1024, 0, s>>>(in, idx, n, out, status, ticket, flags, pat, force);
        else
            scan_lookback_kernel<false, 1024, 32><<<nb8, 1024, 0, s>>>(in, nullptr, n, out, status, ticket, flags, pat, force);
        return;
    }
    if (snt == 1024) {  // status words: div_up(n + 1, 4 * SCAN_TILE) of the cleared ones
        const uint32_t nb4 = div_up(n + 1, (uint32_t)(4 * SCAN_TILE));
        if (idx)
            scan_lookback_kernel<true, 1024><<<nb4, 1024, 0, s>>>(in, idx, n, out, status, ticket, flags, pat, force);
        else
            scan_lookback_kernel<false, 1024><<<nb4, 1024, 0, s>>>(in, nullptr, n, out, status, ticket, flags, pat, force);
        return;
    }
    const uint32_t nb = div_up(n + 1, (uint32_t)SCAN_TILE);
    if (idx)
        scan_lookback_kernel<true><<<nb, 256, 0, s>>>(in, idx, n, out, status, ticket, flags, pat, force);
    else
        scan_lookback_kernel<false><<<nb, 256, 0, s>>>(in, nullptr, n, out, status, ticket, flags, pat, force);
}

// look-back status words of the radix passes: 2-bit flag | 30-bit count
constexpr uint32_t LB_AGG = 1u << 30, LB_INC = 2u << 30, LB_MASK = (1u << 30) - 1;

__device__ __forceinline__ uint32_t lb_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
// radix sort pass: histogram
// ------------------------------------------------------------------------------------------------
// With cs_status, the histogram also clears what the pass's one-launch count scan starts from: its look-back words
// (one RS_BINS row per chunk, cs_rows rows) and its ticket.
// Relative keys (kcap != 0, 32-bit keys, the depth sort's first pass): the key ranked is min(key - kbase, kcap), an
// order-preserving map of the kept depth keys onto [0, kcap) with every culled key (all ones) at kcap.
// REL (a template flag, so that no other sort carries the map: compiled in with a runtime kcap it slowed the 39.5 M-key
// cfg 5 tile-sort scatter passes from 0.19 to 0.30-0.35 ms each).
template <bool REL>
__device__ __forceinline__ uint32_t rs_rel_key(uint32_t k, uint32_t kbase, uint32_t kcap) {
    return REL ? min(k - kbase, kcap) : k;
}

template <int TILE, typename KT = uint32_t, int BINS = RS_BINS, bool REL = false>
__global__ __launch_bounds__(256) void rs_hist_kernel(const KT *__restrict__ keys, uint32_t n, int shift, uint32_t dmask,
                                                      uint32_t *__restrict__ counts, uint32_t nb,
                                                      uint32_t *__restrict__ cs_status, uint32_t cs_rows,
                                                      uint32_t *__restrict__ cs_ticket, uint32_t *__restrict__ cs_err,
                                                      uint32_t kbase = 0, uint32_t kcap = 0) {
    __shared__ uint32_t h[4][BINS];
    const int tid = threadIdx.x, w = tid >> 6;
    if (cs_status) {
        for (uint32_t r = blockIdx.x; r < cs_rows; r += gridDim.x)
            for (int d = tid; d < BINS; d += 256) cs_status[(size_t)r * BINS + d] = 0u;
        if (blockIdx.x == 0 && tid == 0) *cs_ticket = 0u;
    }
    if (cs_err && blockIdx.x == 0 && tid == 0) *cs_err = 0u;  // pass 0: the sort's look-back diagnostic word
    for (int i = tid; i < 4 * BINS; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * TILE;
    if (base + TILE <= n) {
        const uint4 *k4 = reinterpret_cast<const uint4 *>(keys + base);
        constexpr int PER16 = 16 / (int)sizeof(KT);  // keys per 16-B load
#pragma unroll
        for (int i = 0; i < TILE / PER16 / 256; i++) {
            const uint4 q = k4[i * 256 + tid];
            if constexpr (sizeof(KT) == 2) {
                const uint32_t wds[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    atomicAdd(&h[w][((wds[k] & 0xffffu) >> shift) & dmask], 1u);
                    atomicAdd(&h[w][((wds[k] >> 16) >> shift) & dmask], 1u);
                }
            } else {
                atomicAdd(&h[w][(rs_rel_key<REL>(q.x, kbase, kcap) >> shift) & dmask], 1u);
                atomicAdd(&h[w][(rs_rel_key<REL>(q.y, kbase, kcap) >> shift) & dmask], 1u);
                atomicAdd(&h[w][(rs_rel_key<REL>(q.z, kbase, kcap) >> shift) & dmask], 1u);
                atomicAdd(&h[w][(rs_rel_key<REL>(q.w, kbase, kcap) >> shift) & dmask], 1u);
            }
        }
    } else {
        for (int i = tid; i < TILE; i += 256) {
            const uint32_t j = base + i;
            if (j < n) atomicAdd(&h[w][(rs_rel_key<REL>((uint32_t)keys[j], kbase, kcap) >> shift) & dmask], 1u);
        }
    }
    __syncthreads();
    for (int d = tid; d < BINS; d += 256) counts[(size_t)blockIdx.x * BINS + d] = h[0][d] + h[1][d] + h[2][d] + h[3][d];
}

// ------------------------------------------------------------------------------------------------
// radix sort pass: global digit offsets of every (block, digit)
// ------------------------------------------------------------------------------------------------
// The count matrix is block-major -- [block][digit], one coalesced 1 KB row per histogram block, read back as one
// row by that block's scatter -- where a digit-major matrix scattered 4-B writes and reads over nb x 256 cache
// lines per pass (at 48M keys ~200 MB of partial-line traffic for 6 MB of counts).  The scan runs in (digit,
// block) order over it in three short launches: column sums of row chunks (launch_count_scan), one workgroup scanning the
// chunk sums per digit and the digit totals, then every chunk's rows.
__global__ __launch_bounds__(256) void rs_colsum_kernel(const uint32_t *__restrict__ counts, uint32_t nb,
                                                        uint32_t chunk, uint32_t *__restrict__ colsum) {
    const uint32_t c = blockIdx.x, d = threadIdx.x;
    const uint32_t b0 = c * chunk, b1 = min(nb, b0 + chunk);
    uint32_t s = 0;
    uint32_t b = b0;
    for (; b + 8 <= b1; b += 8) {
        uint32_t v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = counts[(size_t)(b + i) * RS_BINS + d];
#pragma unroll
        for (int i = 0; i < 8; i++) s += v[i];
    }
    for (; b < b1; b++) s += counts[(size_t)b * RS_BINS + d];
    colsum[(size_t)c * RS_BINS + d] = s;
}

// One workgroup, thread d = digit: the exclusive prefix of column d over the chunks (the chunk sums of 16 chunks are
// loaded together, so the chain costs one memory round trip per 16 chunks, not one per chunk), then the exclusive
// digit offsets into row nchunks (added by rs_colbase_kernel instead of a second pass over the chunks here).
__global__ __launch_bounds__(256) void rs_colscan_kernel(uint32_t *__restrict__ colsum, uint32_t nchunks) {
    __shared__ uint32_t s_w[4];
    const int d = threadIdx.x, lane = d & 63, w = d >> 6;
    constexpr uint32_t G = 16;
    uint32_t run = 0;
    for (uint32_t c0 = 0; c0 < nchunks; c0 += G) {
        uint32_t v[G];
#pragma unroll
        for (uint32_t i = 0; i < G; i++) v[i] = c0 + i < nchunks ? colsum[(size_t)(c0 + i) * RS_BINS + d] : 0u;
#pragma unroll
        for (uint32_t i = 0; i < G; i++) {
            if (c0 + i < nchunks) colsum[(size_t)(c0 + i) * RS_BINS + d] = run;
            run += v[i];
        }
    }
    const uint32_t inc = wave_inclusive_scan(run, lane);  // digit totals -> exclusive digit offsets
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t off = inc - run;
    for (int i = 0; i < w; i++) off += s_w[i];
    colsum[(size_t)nchunks * RS_BINS + d] = off;
}

__global__ __launch_bounds__(256) void rs_colbase_kernel(uint32_t *__restrict__ counts, uint32_t nb, uint32_t chunk,
                                                         const uint32_t *__restrict__ colsum) {
    const uint32_t c = blockIdx.x, d = threadIdx.x;
    const uint32_t b0 = c * chunk, b1 = min(nb, b0 + chunk);
    uint32_t run = colsum[(size_t)c * RS_BINS + d] + colsum[(size_t)gridDim.x * RS_BINS + d];
    uint32_t b = b0;
    for (; b + 8 <= b1; b += 8) {
        uint32_t v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = counts[(size_t)(b + i) * RS_BINS + d];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            counts[(size_t)(b + i) * RS_BINS + d] = run;
            run += v[i];
        }
    }
    for (; b < b1; b++) {
        const uint32_t v = counts[(size_t)b * RS_BINS + d];
        counts[(size_t)b * RS_BINS + d] = run;
        run += v;
    }
}

// One launch instead of rs_colsum / rs_colscan / rs_colbase (cfg 5 ran those three 6 times per step, ~16 us per pass).
// Workgroup = C consecutive block rows, thread = digit: the thread loads its column's C counts (C coalesced 1-KB
// rows), publishes their sum, and obtains the column prefix of the chunks before it by a decoupled look-back over
// their status words (flag | 30-bit count, as onesweep's; chunk ids from a ticket, so a workgroup only waits on
// workgroups that started before it; an unpublished predecessor is recounted from the counts, which this kernel never
// writes, after `patience` polls).  It writes the rows' exclusive prefixes to counts_pre and the last chunk writes
// the exclusive digit offsets behind them (row nb), which the scatter adds.  Counts < 2^30 (launch_radix_sort).
constexpr int CS_LBW = 16;  // predecessors' words loaded per look-back round trip
template <int C, int BINS = RS_BINS>
__global__ __launch_bounds__(BINS) void rs_countscan_kernel(const uint32_t *__restrict__ counts, uint32_t nb,
                                                            uint32_t *__restrict__ counts_pre,
                                                            uint32_t *__restrict__ status,
                                                            uint32_t *__restrict__ ticket, uint32_t *__restrict__ err,
                                                            uint32_t patience, int force) {
    constexpr int RS_BINS = BINS;  // one thread per digit; rows of BINS counts
    __shared__ uint32_t s_bid, s_w[BINS / 64];
    const int d = threadIdx.x, lane = d & 63, w = d >> 6;
    if (d == 0) s_bid = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t c = s_bid, nch = gridDim.x;
    const uint32_t b0 = c * C;
    uint32_t v[C];
    uint32_t agg = 0;
#pragma unroll
    for (int r = 0; r < C; r++) {
        v[r] = b0 + r < nb ? counts[(size_t)(b0 + r) * RS_BINS + d] : 0u;
        agg += v[r];
    }
    uint32_t *st = status + (size_t)c * RS_BINS + d;
    lb_store(st, (c == 0 ? LB_INC : LB_AGG) | agg);
    uint32_t excl = 0;
    if (c > 0) {
        int look = (int)c - 1;
        uint32_t spins = 0;
        while (true) {
            uint32_t sv[CS_LBW];
#pragma unroll
            for (int i = 0; i < CS_LBW; i++)
                sv[i] = (look - i >= 0) ? (force ? 0u : lb_load(status + (size_t)(look - i) * RS_BINS + d)) : LB_INC;
            const bool fb = force || spins >= patience;
            bool found = false, stalled = false;
            int used = 0;
#pragma unroll
            for (int i = 0; i < CS_LBW; i++) {
                if (!found && !stalled) {
                    uint32_t f = sv[i] & ~LB_MASK, val = sv[i] & LB_MASK;
                    if (f == 0 && fb) {  // recount chunk look - i of this column
                        const uint32_t q0 = (uint32_t)(look - i) * C, q1 = min(nb, q0 + C);
                        val = 0;
                        for (uint32_t b = q0; b < q1; b++) val += counts[(size_t)b * RS_BINS + d];
                        f = LB_AGG;
                        atomicOr(err, 4u);
                    }
                    if (f == 0) {
                        stalled = true;
                    } else {
                        excl += val;
                        used = i + 1;
                        found = f == LB_INC;
                    }
                }
            }
            if (found) break;
            look -= used;
            if (stalled) {
                ++spins;
                __builtin_amdgcn_s_sleep(1);
            }
        }
        lb_store(st, LB_INC | (excl + agg));
    }
    uint32_t run = excl;
#pragma unroll
    for (int r = 0; r < C; r++) {
        if (b0 + r < nb) counts_pre[(size_t)(b0 + r) * RS_BINS + d] = run;
        run += v[r];
    }
    if (c == nch - 1) {  // run = digit total: exclusive digit offsets into row nb
        const uint32_t inc = wave_inclusive_scan(run, lane);
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        uint32_t off = inc - run;
        for (int i = 0; i < w; i++) off += s_w[i];
        counts_pre[(size_t)nb * RS_BINS + d] = off;
    }
}

// Chunk rows per column workgroup: the column chains (chunk / 8 round trips in colsum and colbase) against the
// chunk-sum chain (nch / 16 in colscan).  cfg 5 (round 3): the 1221-row depth-sort matrices 0.280 -> 0.259 ms with 32
// rows (0.271 with 128), the 4822-row tile-sort matrices 0.531 -> 0.513 ms with 128 (0.520 with 32).
static void launch_count_scan(hipStream_t s, uint32_t *counts, uint32_t nb, uint32_t *colsum) {
    const uint32_t chunk = nb <= 2048u ? RS_COL_CHUNK : 4u * RS_COL_CHUNK;  // colsum is sized for RS_COL_CHUNK
    const uint32_t nch = div_up(nb, chunk);
    rs_colsum_kernel<<<nch, RS_BINS, 0, s>>>(counts, nb, chunk, colsum);
    rs_colscan_kernel<<<1, RS_BINS, 0, s>>>(colsum, nch);
    rs_colbase_kernel<<<nch, RS_BINS, 0, s>>>(counts, nb, chunk, colsum);
}

// ------------------------------------------------------------------------------------------------
// radix sort pass: stable scatter
// ------------------------------------------------------------------------------------------------
// digit_off (or null): exclusive digit offsets added to counts_scanned's column prefixes (rs_countscan_kernel)
template <bool IOTA_IN, int ITEMS, typename KT = uint32_t, int BINS = RS_BINS, bool REL = false>
__global__ __launch_bounds__(256) void rs_scatter_kernel(const KT *__restrict__ keys_in,
                                                         const uint32_t *__restrict__ vals_in, uint32_t n,
                                                         int shift, const uint32_t *__restrict__ counts_scanned,
                                                         const uint32_t *__restrict__ digit_off,
                                                         uint32_t nb, KT *__restrict__ keys_out,
                                                         uint32_t *__restrict__ vals_out, SortGather ga,
                                                         uint32_t dmask = 255u, uint32_t kbase = 0, uint32_t kcap = 0) {
    constexpr int DPT = BINS / 256;         // digits per thread in the base computation (consecutive digits)
    constexpr int DBITS = BINS == 512 ? 9 : 8;
    __shared__ uint32_t s_cnt[4][BINS];     // per-wave running digit counts, then per-wave bases
    __shared__ uint32_t s_dstart[BINS];     // block-local start of each digit's run
    __shared__ uint32_t s_gbase[BINS];      // global start of this block's run of each digit
    __shared__ uint32_t s_wsum[4];
    __shared__ KT s_keys[ITEMS * 256];
    __shared__ uint32_t s_vals[ITEMS * 256];

    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t blk = blockIdx.x * (ITEMS * 256);
    for (int i = tid; i < 4 * BINS; i += 256) (&s_cnt[0][0])[i] = 0;
    __syncthreads();

    // Each wave ranks a contiguous segment of 64 * ITEMS keys, 64 at a time, in input order (stable).
    uint32_t key[ITEMS], val[ITEMS], rank[ITEMS];
    const uint64_t lt = lanemask_lt(lane);
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {  // loads first (see rs_onesweep_kernel), unconditional: clamped index
        const uint32_t j = blk + w * ((ITEMS * 256) / 4) + it * 64 + lane, jc = min(j, n - 1);
        key[it] = (uint32_t)keys_in[jc];
        val[it] = IOTA_IN ? j : vals_in[jc];
    }
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {  // (a load in a branch waits for its data before the next is issued)
        const uint32_t j = blk + w * ((ITEMS * 256) / 4) + it * 64 + lane;
        key[it] = j < n ? rs_rel_key<REL>(key[it], kbase, kcap) : 0u;
        if (!IOTA_IN && j >= n) val[it] = 0u;
    }
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t j = blk + w * ((ITEMS * 256) / 4) + it * 64 + lane;
        const bool valid = j < n;
        const uint32_t k = key[it];
        const uint32_t d = (k >> shift) & dmask;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < DBITS; bit++) {
            if (!((dmask >> bit) & 1u)) break;  // digits of fewer bits (uniform)
            const bool set = (d >> bit) & 1u;
            const uint64_t m = __ballot(set);
            peers &= set ? m : ~m;
        }
        uint32_t r = 0;
        if (valid) {
            const uint32_t before = s_cnt[w][d];
            const uint64_t lower = peers & lt;
            r = before + (uint32_t)__popcll(lower);
            if (lower == 0) s_cnt[w][d] = before + (uint32_t)__popcll(peers);
        }
        rank[it] = r;
    }
    __syncthreads();
    {
        // thread tid owns digits [DPT tid, DPT tid + DPT)
        uint32_t tot[DPT], sum = 0;
#pragma unroll
        for (int q = 0; q < DPT; q++) {
            const int d = DPT * tid + q;
            const uint32_t c0 = s_cnt[0][d], c1 = s_cnt[1][d], c2 = s_cnt[2][d], c3 = s_cnt[3][d];
            s_cnt[0][d] = 0;
            s_cnt[1][d] = c0;
            s_cnt[2][d] = c0 + c1;
            s_cnt[3][d] = c0 + c1 + c2;
            tot[q] = c0 + c1 + c2 + c3;
            sum += tot[q];
        }
        const uint32_t inc = wave_inclusive_scan(sum, lane);
        if (lane == 63) s_wsum[w] = inc;
        __syncthreads();
        uint32_t woff = 0;
        for (int i = 0; i < w; i++) woff += s_wsum[i];
        uint32_t run = woff + inc - sum;
#pragma unroll
        for (int q = 0; q < DPT; q++) {
            const int d = DPT * tid + q;
            s_dstart[d] = run;
            run += tot[q];
            s_gbase[d] = counts_scanned[(size_t)blockIdx.x * BINS + d] + (digit_off ? digit_off[d] : 0u);
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t j = blk + w * ((ITEMS * 256) / 4) + it * 64 + lane;
        if (j < n) {
            const uint32_t d = (key[it] >> shift) & dmask;
            const uint32_t pos = s_dstart[d] + s_cnt[w][d] + rank[it];
            s_keys[pos] = (KT)key[it];
            s_vals[pos] = val[it];
        }
    }
    __syncthreads();
    const uint32_t cnt_blk = min((uint32_t)(ITEMS * 256), n - blk);
    if (ga.dst || ga.dst4) {  // final pass with a permuted gather (see rs_onesweep_kernel)
        for (uint32_t i0 = 0; i0 < cnt_blk; i0 += 256 * 8) {
            uint32_t g[8], gp[8];
            uint4 g4[8];
#pragma unroll
            for (int it = 0; it < 8; it++) {  // gathers unconditional (clamped slot) so they issue together
                const uint32_t i = i0 + tid + it * 256, ic = min(i, cnt_blk - 1);
                const uint32_t k = s_keys[ic], v = s_vals[ic];
                const uint32_t d = (k >> shift) & dmask;
                gp[it] = i < cnt_blk ? s_gbase[d] + (i - s_dstart[d]) : 0xffffffffu;
                if (ga.dst) g[it] = ga.src[v];
                if (ga.dst4) g4[it] = ga.src4[v];
                if (i < cnt_blk) {
                    keys_out[gp[it]] = (KT)k;
                    vals_out[gp[it]] = v;
                }
            }
#pragma unroll
            for (int it = 0; it < 8; it++)
                if (gp[it] != 0xffffffffu) {
                    if (ga.dst) ga.dst[gp[it]] = g[it];
                    if (ga.dst4) ga.dst4[gp[it]] = g4[it];
                }
        }
        return;
    }
    if (cnt_blk == (uint32_t)(ITEMS * 256)) {
        // full block: LDS reads and offsets of 8 elements first, then their 16 stores (one LDS round trip per 8
        // elements instead of per element)
#pragma unroll
        for (int i0 = 0; i0 < ITEMS; i0 += 8) {
            uint32_t k[8], v[8], g[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t i = (uint32_t)(i0 + q) * 256 + tid;
                k[q] = s_keys[i];
                v[q] = s_vals[i];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t i = (uint32_t)(i0 + q) * 256 + tid;
                const uint32_t d = (k[q] >> shift) & dmask;
                g[q] = s_gbase[d] + (i - s_dstart[d]);
            }
#pragma unroll
            for (int q = 0; q < 8; q++) {
                keys_out[g[q]] = (KT)k[q];
                vals_out[g[q]] = v[q];
            }
        }
        return;
    }
    for (uint32_t i = tid; i < cnt_blk; i += 256) {
        const uint32_t k = s_keys[i], v = s_vals[i];
        const uint32_t d = (k >> shift) & dmask;
        const uint32_t gpos = s_gbase[d] + (i - s_dstart[d]);
        keys_out[gpos] = (KT)k;
        vals_out[gpos] = v;
    }
}

// ------------------------------------------------------------------------------------------------
// onesweep radix sort: one histogram pass over the keys for every digit, then ONE kernel per digit pass
// whose blocks obtain their global digit offsets by decoupled look-back (each block publishes its digit
// counts, then its inclusive prefix; a block only waits on blocks that started before it, since block
// ids come from an atomic ticket).  3 + passes launches instead of 5 per pass.
// ------------------------------------------------------------------------------------------------

constexpr int MH_BATCH = 8;
// Digit histograms of every pass in one read of the keys.  Keys that share a digit inside a wave are
// aggregated by ballot (8 ballots per digit, one LDS add per distinct digit), so skewed digits -- the top
// byte of depth keys is nearly constant -- cause no atomic serialisation.
__global__ __launch_bounds__(256) void rs_multi_hist_kernel(const uint32_t *__restrict__ keys, uint32_t n,
                                                            int passes, uint32_t *__restrict__ ctrl, uint4 *stamps) {
    __shared__ uint32_t h[RS_MAX_PASSES][RS_BINS];
    const uint32_t t0 = stamps ? stamp_now() : 0u;
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < RS_MAX_PASSES * RS_BINS; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t lt = lanemask_lt(lane);
    const uint32_t stride = gridDim.x * 256;
    // keys are loaded MH_BATCH at a time before the ballot work (one load latency per batch, not per key)
    for (uint32_t base0 = blockIdx.x * 256; base0 < n; base0 += MH_BATCH * stride) {  // uniform per wave
        uint32_t kb[MH_BATCH];
#pragma unroll
        for (int b = 0; b < MH_BATCH; b++) {
            const uint32_t j = base0 + b * stride + tid;
            kb[b] = j < n ? keys[j] : 0u;
        }
#pragma unroll
        for (int b = 0; b < MH_BATCH; b++) {
        const uint32_t j = base0 + b * stride + tid;
        const bool valid = j < n;
        const uint32_t k = kb[b];
        for (int p = 0; p < passes; p++) {
            const uint32_t d = (k >> (8 * p)) & 255u;
            uint64_t peers = __ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 8; bit++) {
                const bool set = (d >> bit) & 1u;
                const uint64_t m = __ballot(set);
                peers &= set ? m : ~m;
            }
            if (valid && (peers & lt) == 0) atomicAdd(&h[p][d], (uint32_t)__popcll(peers));
        }
        }
    }
    __syncthreads();
    const uint32_t t1 = stamps ? stamp_now() : 0u;
    for (int p = 0; p < passes; p++) {
        const uint32_t c = h[p][tid];
        if (c) atomicAdd(&ctrl[RS_CTRL_HIST + p * RS_BINS + tid], c);
    }
    if (stamps) {
        __syncthreads();
        if (tid == 0 && blockIdx.x < (uint32_t)STAMP_SLOTS) stamps[blockIdx.x] = make_uint4(t0, t1, stamp_now(), 0u);
    }
}

// exclusive scan of every pass's 256 digit counts, in place
__global__ __launch_bounds__(256) void rs_hist_scan_kernel(uint32_t *__restrict__ ctrl, int passes) {
    __shared__ uint32_t s_w[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int p = 0; p < passes; p++) {
        uint32_t *h = ctrl + RS_CTRL_HIST + p * RS_BINS;
        const uint32_t v = h[tid];
        const uint32_t inc = wave_inclusive_scan(v, lane);
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        uint32_t off = 0;
        for (int i = 0; i < w; i++) off += s_w[i];
        h[tid] = off + inc - v;
        __syncthreads();
    }
}

// ga (final pass only, else empty): dst[sorted position] = src[value], i.e. arrays permuted into the sorted
// order while the values are written (the depth sort hands the instance scan and the expansion their per-Gaussian
// inputs in depth order this way, instead of each gathering them through the order with a dependent random load).
template <bool IOTA_IN, int ITEMS, int LBW>
__global__ __launch_bounds__(256) void rs_onesweep_kernel(const uint32_t *__restrict__ keys_in,
                                                          const uint32_t *__restrict__ vals_in, uint32_t n,
                                                          int pass, uint32_t *__restrict__ ctrl,
                                                          uint32_t *__restrict__ status,
                                                          uint32_t *__restrict__ keys_out,
                                                          uint32_t *__restrict__ vals_out, uint4 *stamps,
                                                          SortGather ga, uint32_t patience, int force) {
    __shared__ uint32_t s_cnt[4][RS_BINS];  // per-wave running digit counts, then per-wave bases
    __shared__ uint32_t s_dstart[RS_BINS];  // block-local start of each digit's run
    __shared__ uint32_t s_gbase[RS_BINS];   // global start of this block's run of each digit
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_bid;
    const uint32_t t0 = stamps ? stamp_now() : 0u;
    uint32_t t_rank = 0, t_lb = 0;
    __shared__ uint32_t s_keys[ITEMS * 256];
    __shared__ uint32_t s_vals[ITEMS * 256];

    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int shift = 8 * pass;
    if (tid == 0) s_bid = atomicAdd(&ctrl[RS_CTRL_COUNTER + pass], 1u);
    for (int i = tid; i < 4 * RS_BINS; i += 256) (&s_cnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t bid = s_bid;
    constexpr uint32_t TILE = ITEMS * 256;
    const uint32_t blk = bid * TILE;

    uint32_t key[ITEMS], val[ITEMS], rank[ITEMS];
    const uint64_t lt = lanemask_lt(lane);
    // all of the thread's loads are issued before the ranking: the ranking's LDS read-modify-write chain
    // would otherwise wait one global-load latency per item (measured ~0.6 us each)
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t j = blk + w * (TILE / 4) + it * 64 + lane;
        const bool valid = j < n;
        key[it] = valid ? keys_in[j] : 0u;
        val[it] = IOTA_IN ? j : (valid ? vals_in[j] : 0u);
    }
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t j = blk + w * (TILE / 4) + it * 64 + lane;
        const bool valid = j < n;
        const uint32_t k = key[it];
        const uint32_t d = (k >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const bool set = (d >> bit) & 1u;
            const uint64_t m = __ballot(set);
            peers &= set ? m : ~m;
        }
        uint32_t r = 0;
        if (valid) {
            const uint32_t before = s_cnt[w][d];
            const uint64_t lower = peers & lt;
            r = before + (uint32_t)__popcll(lower);
            if (lower == 0) s_cnt[w][d] = before + (uint32_t)__popcll(peers);
        }
        rank[it] = r;
    }
    __syncthreads();
    if (stamps) t_rank = stamp_now();
    {
        const int d = tid;
        const uint32_t c0 = s_cnt[0][d], c1 = s_cnt[1][d], c2 = s_cnt[2][d], c3 = s_cnt[3][d];
        const uint32_t tot = c0 + c1 + c2 + c3;
        uint32_t *st = status + (size_t)bid * RS_BINS + d;
        lb_store(st, (bid == 0 ? LB_INC : LB_AGG) | tot);  // publish early: successors can proceed
        s_cnt[0][d] = 0;
        s_cnt[1][d] = c0;
        s_cnt[2][d] = c0 + c1;
        s_cnt[3][d] = c0 + c1 + c2;
        const uint32_t inc = wave_inclusive_scan(tot, lane);
        if (lane == 63) s_wsum[w] = inc;
        uint32_t excl = 0;
        if (bid > 0) {
            // Windowed look-back: LBW predecessors' words are loaded at once (one round-trip latency per
            // window instead of per predecessor); published words are summed nearest first up to the first
            // inclusive prefix, and an unpublished one is re-polled.  Positions before block 0 read as an
            // inclusive prefix of 0.
            int look = (int)bid - 1;
            uint32_t spins = 0;
            while (true) {
                uint32_t v[LBW];
#pragma unroll
                for (int i = 0; i < LBW; i++)
                    v[i] = (look - i >= 0) ? (force ? 0u : lb_load(status + (size_t)(look - i) * RS_BINS + d)) : LB_INC;
                // decoupled fallback (wave_lookback): after `patience` polls (at once with force) an unpublished
                // predecessor's digit count is recounted from its keys, which this pass never writes
                const bool fb = force || spins >= patience;
                bool found = false, stalled = false;
                int used = 0;
#pragma unroll
                for (int i = 0; i < LBW; i++) {
                    if (!found && !stalled) {
                        uint32_t f = v[i] & ~LB_MASK, val = v[i] & LB_MASK;
                        if (f == 0 && fb) {
                            const uint32_t q = (uint32_t)(look - i), e = min(n, (q + 1) * TILE);
                            val = 0;
                            for (uint32_t j = q * TILE; j < e; j++) val += ((keys_in[j] >> shift) & 255u) == (uint32_t)d;
                            f = LB_AGG;
                            atomicOr(&ctrl[RS_CTRL_ERR], 4u);
                        }
                        if (f == 0) {
                            stalled = true;
                        } else {
                            excl += val;
                            used = i + 1;
                            found = f == LB_INC;
                        }
                    }
                }
                if (found) break;
                look -= used;
                if (stalled) {
                    ++spins;
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            lb_store(st, LB_INC | (excl + tot));
        }
        s_gbase[d] = ctrl[RS_CTRL_HIST + pass * RS_BINS + d] + excl;
        __syncthreads();
        if (stamps) t_lb = stamp_now();
        uint32_t woff = 0;
        for (int i = 0; i < w; i++) woff += s_wsum[i];
        s_dstart[d] = woff + inc - tot;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint32_t j = blk + w * (TILE / 4) + it * 64 + lane;
        if (j < n) {
            const uint32_t d = (key[it] >> shift) & 255u;
            const uint32_t pos = s_dstart[d] + s_cnt[w][d] + rank[it];
            s_keys[pos] = key[it];
            s_vals[pos] = val[it];
        }
    }
    __syncthreads();
    const uint32_t cnt_blk = min(TILE, n - blk);
    if (ga.dst || ga.dst4) {  // the gathers of a thread's elements are issued together, then stored
        uint32_t g[ITEMS], gp[ITEMS];
        uint4 g4[ITEMS];
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const uint32_t i = tid + it * 256;
            gp[it] = 0xffffffffu;
            if (i < cnt_blk) {
                const uint32_t k = s_keys[i], v = s_vals[i];
                const uint32_t d = (k >> shift) & 255u;
                gp[it] = s_gbase[d] + (i - s_dstart[d]);
                keys_out[gp[it]] = k;
                vals_out[gp[it]] = v;
                if (ga.dst) g[it] = ga.src[v];
                if (ga.dst4) g4[it] = ga.src4[v];
            }
        }
#pragma unroll
        for (int it = 0; it < ITEMS; it++)
            if (gp[it] != 0xffffffffu) {
                if (ga.dst) ga.dst[gp[it]] = g[it];
                if (ga.dst4) ga.dst4[gp[it]] = g4[it];
            }
    } else {
        for (uint32_t i = tid; i < cnt_blk; i += 256) {
            const uint32_t k = s_keys[i], v = s_vals[i];
            const uint32_t d = (k >> shift) & 255u;
            const uint32_t gpos = s_gbase[d] + (i - s_dstart[d]);
            keys_out[gpos] = k;
            vals_out[gpos] = v;
        }
    }
    if (stamps && tid == 0 && bid < (uint32_t)STAMP_SLOTS) stamps[bid] = make_uint4(t0, t_rank, t_lb, stamp_now());
}

template <int ITEMS, int LBW>
static void launch_radix_sort_onesweep(hipStream_t s, SortScratch &sc, uint32_t n, int passes, bool keyed,
                                       const uint32_t *keys0, const SortGather *gather) {
    const uint32_t nb = div_up(n, (uint32_t)ITEMS * 256u);
    (void)hipMemsetAsync(sc.ctrl, 0, sizeof(uint32_t) * (RS_CTRL_WORDS + (size_t)passes * nb * RS_BINS), s);
    const uint32_t hb = min(div_up(n, 256u * 8u), 2048u);
    uint4 *stamps = tuning("stamp", 0) ? stamp_buffer(2) : nullptr;
    const uint32_t pat = (uint32_t)tuning("lb_patience", 1 << 16);
    const int force = tuning("lb_force", 0);
    rs_multi_hist_kernel<<<max(hb, 1u), 256, 0, s>>>(keys0, n, passes, sc.ctrl,
                                                    stamps ? stamp_buffer(3) : nullptr);
    rs_hist_scan_kernel<<<1, 256, 0, s>>>(sc.ctrl, passes);
    for (int p = 0; p < passes; p++) {
        const int in = p & 1, out = (p + 1) & 1;
        uint32_t *st = sc.status + (size_t)p * nb * RS_BINS;
        const uint32_t *kin = p == 0 ? keys0 : sc.k[in];
        SortGather ga;
        if (p == passes - 1 && gather) ga = *gather;
        if (p == 0 && !keyed)
            rs_onesweep_kernel<true, ITEMS, LBW><<<nb, 256, 0, s>>>(kin, nullptr, n, p, sc.ctrl, st, sc.k[out],
                                                               sc.v[out], stamps, ga, pat, force);
        else
            rs_onesweep_kernel<false, ITEMS, LBW><<<nb, 256, 0, s>>>(kin, sc.v[in], n, p, sc.ctrl, st, sc.k[out],
                                                                sc.v[out], stamps, ga, pat, force);
    }
}

// multi-kernel path: per pass a block histogram, a scan of the (digit x block) counts, a stable scatter
// BINS = 512: digits of up to 9 bits (the relative depth sort); the count matrix rows are BINS wide, and the
// one-launch count scan (rs_cscan) is the only scan that takes them.  kcap != 0: pass 0 ranks relative keys
// (rs_rel_key).  flip: the passes write slot (p + 1 + 1) & 1, so an odd number of passes still ends in slot 0.
template <int ITEMS, typename KT = uint32_t, int BINS = RS_BINS>
static void launch_radix_sort_multi(hipStream_t s, SortScratch &sc, uint32_t n, int passes, bool keyed,
                                    const KT *keys0, const SortGather *gather, int dbits = 8, uint32_t kbase = 0,
                                    uint32_t kcap = 0, int flip = 0, int dbits0 = 0) {
    // dbits0 > 0: the first pass ranks the low dbits0 bits, the later ones dbits each above them
    const int d0 = dbits0 > 0 ? dbits0 : dbits;
    KT *k[2] = {reinterpret_cast<KT *>(sc.k[0]), reinterpret_cast<KT *>(sc.k[1])};
    const uint32_t nb = div_up(n, (uint32_t)ITEMS * 256u);  // <= the RS_TILE block count carve_sort sized
    // "rs_cscan" 1 (default): the one-launch count scan (look-back counts < 2^30); 0: the three-launch column scan
    const bool one = BINS != RS_BINS || (tuning("rs_cscan", 1) != 0 && n <= RS_ONESWEEP_MAX_N);
    // count-scan rows per workgroup: 64 for long 256-bin matrices ("rs_cs64"; the 16-bit tile sort at 16 keys per
    // thread has ~9.6 k rows at cfg 5), else 32
    const uint32_t CS_C = (BINS == RS_BINS && nb > 4096) ? 64u : 32u;
    const uint32_t nch = div_up(nb, CS_C);  // <= RS_MAX_PASSES * nb_os rows of sc.status per pass
    const uint32_t pat = (uint32_t)tuning("lb_patience", 1 << 16);
    const int force = tuning("lb_force", 0);
    for (int p = 0; p < passes; p++) {
        const int shift = p == 0 ? 0 : d0 + dbits * (p - 1), in = (p + flip) & 1, out = (p + 1 + flip) & 1;
        const uint32_t dmask = (1u << (p == 0 ? d0 : dbits)) - 1u;
        const KT *kin = p == 0 ? keys0 : k[in];
        const uint32_t cap = p == 0 ? kcap : 0u;
        uint32_t *cs_status = one ? sc.status + (size_t)p * nch * BINS : nullptr;
        if (cap)
            rs_hist_kernel<ITEMS * 256, KT, BINS, true><<<nb, 256, 0, s>>>(kin, n, shift, dmask, sc.counts, nb, cs_status,
                                                                          nch, sc.ctrl + RS_CTRL_COUNTER + p,
                                                                          sc.ctrl + RS_CTRL_ERR, kbase, cap);
        else
            rs_hist_kernel<ITEMS * 256, KT, BINS><<<nb, 256, 0, s>>>(kin, n, shift, dmask, sc.counts, nb, cs_status, nch,
                                                                    sc.ctrl + RS_CTRL_COUNTER + p,
                                                                    p == 0 ? sc.ctrl + RS_CTRL_ERR : nullptr);
        const uint32_t *scanned = sc.counts, *doff = nullptr;
        if (one) {
            if (CS_C == 64)
                rs_countscan_kernel<64, BINS><<<nch, BINS, 0, s>>>(sc.counts, nb, sc.counts_pre, cs_status,
                                                                  sc.ctrl + RS_CTRL_COUNTER + p, sc.ctrl + RS_CTRL_ERR,
                                                                  pat, force);
            else
                rs_countscan_kernel<32, BINS><<<nch, BINS, 0, s>>>(sc.counts, nb, sc.counts_pre, cs_status,
                                                                  sc.ctrl + RS_CTRL_COUNTER + p, sc.ctrl + RS_CTRL_ERR,
                                                                  pat, force);
            scanned = sc.counts_pre;
            doff = sc.counts_pre + (size_t)nb * BINS;
        } else {
            launch_count_scan(s, sc.counts, nb, sc.scan_tmp);
        }
        SortGather ga;
        if (p == passes - 1 && gather) ga = *gather;
        if (p == 0 && !keyed && cap)
            rs_scatter_kernel<true, ITEMS, KT, BINS, true><<<nb, 256, 0, s>>>(kin, nullptr, n, shift, scanned, doff, nb,
                                                                              k[out], sc.v[out], ga, dmask, kbase, cap);
        else if (p == 0 && !keyed)
            rs_scatter_kernel<true, ITEMS, KT, BINS><<<nb, 256, 0, s>>>(kin, nullptr, n, shift, scanned, doff, nb,
                                                                        k[out], sc.v[out], ga, dmask);
        else
            rs_scatter_kernel<false, ITEMS, KT, BINS><<<nb, 256, 0, s>>>(kin, sc.v[in], n, shift, scanned, doff, nb,
                                                                         k[out], sc.v[out], ga, dmask);
    }
}

bool launch_radix_sort(hipStream_t s, SortScratch &sc, uint32_t n, int nbits, bool keyed, const uint32_t *keys0,
                       const SortGather *gather, bool *onesweep_ran) {
    if (onesweep_ran) *onesweep_ran = false;
    if (n == 0) return gather != nullptr;
    if (!keys0) keys0 = sc.k[0];
    const int passes = radix_passes(nbits);
    // onesweep knob: bit 0 = depth-size sorts (nbits == 32), bit 1 = tile sorts
    const int os = tuning("onesweep", 1);
    // measured (depth sorts, with the permuted gather): onesweep 0.121 / 0.378 ms at 1 M / 5 M keys against
    // 0.183 / 0.329 for the multi-kernel path (32 keys per thread); linear fits cross near 3.2 M keys
    const uint32_t os_max = (uint32_t)tuning("onesweep_max_n", 3 << 20);
    if (n <= RS_ONESWEEP_MAX_N && n <= os_max && passes <= RS_MAX_PASSES && (os & (nbits == 32 ? 1 : 2))) {
        // 8-/32-key tiles measured slower
        const int lbw = tuning("lbw", 16);
        if (lbw >= 64) launch_radix_sort_onesweep<RS_ITEMS, 64>(s, sc, n, passes, keyed, keys0, gather);
        else if (lbw >= 32) launch_radix_sort_onesweep<RS_ITEMS, 32>(s, sc, n, passes, keyed, keys0, gather);
        else if (lbw >= 16) launch_radix_sort_onesweep<RS_ITEMS, 16>(s, sc, n, passes, keyed, keys0, gather);
        else launch_radix_sort_onesweep<RS_ITEMS, 1>(s, sc, n, passes, keyed, keys0, gather);
        if (onesweep_ran) *onesweep_ran = true;
        return gather != nullptr;
    }
    // "rs_items": keys per thread of the multi-kernel path, 16 or 32 (fewer blocks, longer digit runs per block);
    // 0 (default): 16 up to 8M keys, else 32 (cfg 5: the 5M-key depth sort 0.313 -> 0.275 ms with 16, the 48M-key
    // tile sort 0.667 -> 0.723 ms)
    int items = tuning("rs_items", 0);
    if (items == 0) items = n <= (8u << 20) ? 16 : 32;
    if (items >= 32) launch_radix_sort_multi<32>(s, sc, n, passes, keyed, keys0, gather);
    else launch_radix_sort_multi<RS_ITEMS>(s, sc, n, passes, keyed, keys0, gather);
    return gather != nullptr;
}

// The depth sort on relative keys (the multi-kernel path's sizes): the P depth keys mapped onto [0, kcap] by
// rs_rel_key (kcap = the kept keys' span + 1, the culled keys' slot), bits = bits of kcap, in ceil(bits / 9) passes
// of at most 9 bits -- 3 instead of 4 for spans up to 2^27 (depth ranges up to ~16x).  Same order as the 32-bit sort
// (stable, order-preserving map), values end in slot 0 (g.order) for any number of passes.
void launch_depth_sort_rel(hipStream_t s, SortScratch &sc, uint32_t n, const uint32_t *keys0, uint32_t kbase,
                           uint32_t kcap, int bits, const SortGather *gather) {
    if (n == 0) return;
    const int passes = (bits + 8) / 9;
    const int dbits = (bits + passes - 1) / passes;
    const int flip = passes & 1;
    int items = tuning("rs_items", 0);
    if (items == 0) items = n <= (8u << 20) ? 16 : 32;
    if (dbits > 8) {
        if (items >= 32) launch_radix_sort_multi<32, uint32_t, 512>(s, sc, n, passes, false, keys0, gather, dbits, kbase, kcap, flip);
        else launch_radix_sort_multi<RS_ITEMS, uint32_t, 512>(s, sc, n, passes, false, keys0, gather, dbits, kbase, kcap, flip);
    } else {
        if (items >= 32) launch_radix_sort_multi<32>(s, sc, n, passes, false, keys0, gather, dbits, kbase, kcap, flip);
        else launch_radix_sort_multi<RS_ITEMS>(s, sc, n, passes, false, keys0, gather, dbits, kbase, kcap, flip);
    }
}

void launch_radix_sort16(hipStream_t s, SortScratch &sc, uint32_t n, int dbits, int passes, int bits) {
    if (n == 0) return;
    const uint16_t *k0 = reinterpret_cast<const uint16_t *>(sc.k[0]);
    // 16 keys per thread at every size for the 16-bit tile keys (cfg 5, 39.5 M keys: 0.454 -> 0.427 ms against 32, whose
    // scatter holds 148 VGPRs, 3 waves per SIMD; profiles/r5ax_ab_rs_items_cfg5.txt)
    int items = tuning("rs_items", 0);
    if (items == 0) items = 16;
    // "tile_lo_short" 1: the first pass takes the short digit (15-bit keys: 7 + 8 bits instead of 8 + 7), so its 128
    // digit runs per block are twice as long as 256 would be
    const int d0 = (tuning("tile_lo_short", 1) && passes >= 2 && bits < dbits * passes) ? bits - dbits * (passes - 1) : 0;
    if (items >= 32) launch_radix_sort_multi<32, uint16_t>(s, sc, n, passes, false, k0, nullptr, dbits, 0, 0, 0, d0);
    else launch_radix_sort_multi<RS_ITEMS, uint16_t>(s, sc, n, passes, false, k0, nullptr, dbits, 0, 0, 0, d0);
}

}  // namespace gsr
