// gsr_common.h -- shared device/host definitions for the MI355X Gaussian rasterizer.
//
// Layout of the three caller-owned scratch buffers (SURVEY.md §8(b) "Ownership"; the reference keeps
// GeometryState/BinningState/ImageState in uint8 torch tensors, notes/rasterizer_note.h:27-40).  All
// per-Gaussian render attributes are packed into one 48-B record (GRec) so a tile batch gathers an instance with
// three 16/16/8-byte loads from the same cache line:
//   a = (x_pix, y_pix, conic.x, conic.y)   b = (conic.z, opacity, r, g)   c = (b, 1/depth)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

int tuning(const char *name, int default_value);  // gsr_api.hip: runtime knobs (gsr_set_tuning)

constexpr int BLOCK_X = 16;
constexpr int BLOCK_Y = 16;
constexpr int TILE_PIX = BLOCK_X * BLOCK_Y;
constexpr int WAVE = 64;
constexpr int PIX_PER_LANE = TILE_PIX / WAVE;  // one wave composites one 16x16 tile
constexpr uint32_t BIG_GAUSSIAN_TILES = 64;   // per-Gaussian gradient rows reduced by a whole block above this
constexpr int STAMP_SLOTS = 1 << 16;  // diagnostics: launch slots with a wave stamp (gsr_debug_wave_stamps)
constexpr int GRAD_ROW = 10;                   // floats per instance gradient row (40 B, 8-B aligned)

// counters block at the head of the geometry buffer (zeroed every forward)
// counters: [CNT_BIG] big-Gaussian count, [CNT_OVERFLOW] scan overflow flag, then CNT_NPART 64-bit partial
// sums of the instance total (spread over addresses so the per-block atomics do not serialise), then CNT_NPART
// partial maxima of the complemented kept depth keys (their minimum) and CNT_NPART of the kept depth keys
enum Counter : int { CNT_BIG = 0, CNT_OVERFLOW = 2, CNT_SCAN_TICKET = 3, CNT_COL_TICKET = 4, CNT_LONG = 6, CNT_PRE_DONE = 10, CNT_LIVE_VALID = 12, CNT_PARTIALS = 16, CNT_NPART = 64,
                     CNT_DMIN = 16 + 2 * 64, CNT_DMAX = CNT_DMIN + 64, CNT_WORDS = CNT_DMAX + 64 };

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) & ~(a - 1); }

struct Carver {
    char *base;
    size_t off;
    explicit Carver(char *b) : base(b), off(0) {}
    template <class T>
    T *take(size_t count, size_t alignment = 256) {
        off = align_up(off, alignment);
        T *p = base ? reinterpret_cast<T *>(base + off) : nullptr;
        off += count * sizeof(T);
        return p;
    }
};

// radix-sort / scan tiling
constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;  // 4096 keys per block
constexpr int RS_BINS = 256;
constexpr int RS_BINS_MAX = 512;  // the relative depth sort's 9-bit digits (count matrix rows)
constexpr int SCAN_TILE = 4096;
constexpr int SCAN_MAX_BLOCKS = 1024 * 16;  // single-block scan of block sums
constexpr uint32_t RS_COL_CHUNK = 32;  // smallest radix count-matrix row chunk per column-scan workgroup (sizes scan_tmp)

inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

constexpr int RS_MAX_PASSES = 4;
// onesweep control block: [0, 4) pass tile counters, [4] error flag, [8, 8 + 4 * 256) digit histograms of
// every pass; followed by the look-back status words (RS_MAX_PASSES x nblocks x RS_BINS).  One memset
// clears control + status before a sort.
constexpr int RS_CTRL_COUNTER = 0, RS_CTRL_ERR = 4, RS_CTRL_HIST = 8;
constexpr int RS_CTRL_WORDS = RS_CTRL_HIST + RS_MAX_PASSES * RS_BINS;
constexpr uint32_t RS_ONESWEEP_MAX_N = (1u << 30) - 1;  // 30-bit counts in the look-back words

struct SortScratch {
    uint32_t *k[2];
    uint32_t *v[2];
    uint32_t *counts;    // RS_BINS * nblocks (multi-kernel path)
    uint32_t *counts_pre;  // RS_BINS * nblocks column prefixes, then RS_BINS digit offsets (one-launch count scan)
    uint32_t *scan_tmp;  // column sums of the count matrix (RS_COL_CHUNK-row chunks x RS_BINS)
    uint32_t *ctrl;      // RS_CTRL_WORDS, then the look-back status words (onesweep path)
    uint32_t *status;
};

inline void carve_sort(Carver &c, SortScratch &s, uint32_t n, bool need_v0) {
    s.k[0] = c.take<uint32_t>(n ? n : 1);
    s.k[1] = c.take<uint32_t>(n ? n : 1);
    s.v[0] = need_v0 ? c.take<uint32_t>(n ? n : 1) : nullptr;
    s.v[1] = c.take<uint32_t>(n ? n : 1);
    uint32_t nb = div_up(n ? n : 1, RS_TILE);
    s.counts = c.take<uint32_t>((size_t)RS_BINS_MAX * nb + 1);
    s.counts_pre = c.take<uint32_t>((size_t)RS_BINS_MAX * (nb + 1));
    s.scan_tmp = c.take<uint32_t>(((size_t)div_up(nb, RS_COL_CHUNK) + 1) * RS_BINS);
    const uint32_t nb_os = div_up(n ? n : 1, RS_TILE / 2);  // onesweep tiles may be half a RS_TILE
    s.ctrl = c.take<uint32_t>(RS_CTRL_WORDS + (size_t)RS_MAX_PASSES * nb_os * RS_BINS);
    s.status = s.ctrl + RS_CTRL_WORDS;
}

// Bucket binning (gsr_bin.hip): used when the tile count fits the LDS histogram of one workgroup.
constexpr uint32_t BK_MAX_TILES = 32768;  // 128 KB of LDS counters (4K images: 32400 tiles)
constexpr uint32_t BK_MAX_BLOCKS = 512;   // rows of the count matrix (carved for the maximum)
constexpr uint32_t BK_MAX_MEAN = 1024;    // default path choice: mean instances per tile up to this
#ifndef GSR_BK_REGION_LOG2  // overridable for library A/B builds (tools/build_variant.py)
#define GSR_BK_REGION_LOG2 4
#endif
constexpr uint32_t BK_REGION = 1u << GSR_BK_REGION_LOG2;  // tiles per region of the region scatter (consecutive tile ids)
constexpr int BK_REG_SHIFT = 32 - GSR_BK_REGION_LOG2;    // the region scatter carries a key's tile-in-region in u's top bits
constexpr uint32_t SEG_CAP = 511;         // longest tile the per-wave register sort takes (8 keys per lane);
                                          // SEG_CAP + 1 is a multiple of the LPT bucket width (seg_block)
constexpr uint32_t SEG_BLOCK_CAP = 2048;  // longest tile one workgroup sorts (4 waves x 512 keys); longer: chunks

// One Gaussian's render record: interleaved rather than three arrays, so the composite passes' random gathers
// touch one or two cache lines per instance instead of three.
struct GRec {
    float4 a;  // x_pix, y_pix, conic.x, conic.y
    float4 b;  // conic.z, opacity, r, g
    float2 c;  // b, 1/depth
    float2 pad;
};
static_assert(sizeof(GRec) == 48, "render record");

struct GeomState {
    uint32_t *counters;    // CNT_WORDS
    GRec *rec;             // P
    uint32_t *depth_key;   // P: float bits of view depth, 0xffffffff if culled
    uint32_t *tiles;       // P: tiles touched
    uint8_t *clamped;      // P: bit c set if SH colour channel c was clamped at 0
    uint8_t *live;         // P: 0 from the preprocess; 1 once a compositing backward stored a non-zero row of it
    float *sh_jac;         // 9 x P: d rgb / d (unit view direction), planes [axis][channel] (SH degree > 0 only)
    uint4 *exp_rec;        // P: expansion record {kept-tile mask lo, hi, rmin.x | rmin.y << 16, rect width}; mask 0 =
                           //    all tiles of the rect (area > 64 or culling off).  One 16-B gather per Gaussian.
    uint32_t *inst_off;    // P+1: radix path: exclusive scan of tiles in depth order, [P] = total
    uint32_t *tiles_sorted;  // P: radix path: tiles in depth order (written by the depth sort's last pass)
    uint4 *exp_sorted;       // P: radix path: exp_rec in depth order (likewise)
    uint32_t *inst_start;  // P+1: first instance (expansion order) of each Gaussian (bucket path: the
                           //      exclusive scan of tiles in Gaussian order, [P] = total)
    uint32_t *block_sums;  // div_up(P, 256): kept-tile totals of the preprocess blocks (bucket path)
    uint32_t *big_list;    // P: Gaussians with > BIG_GAUSSIAN_TILES tiles
    uint32_t *big_slot;    // P: index of a big Gaussian in big_list (valid only for big ones)
    uint32_t *scan_tmp;    // block sums for the instance scan (multi-kernel path)
    uint64_t *scan_status; // look-back words of the single-kernel instance scan
    uint64_t *tile_status; // look-back words of the bucket path's tile scan
    SortScratch sort;      // depth sort (P keys); final order lands in sort.v[0]
    const uint32_t *order; // = sort.v[0] after the (even-pass) depth sort
};

inline size_t carve_geom(char *base, int P, GeomState &g) {
    Carver c(base);
    uint32_t n = (uint32_t)P;
    g.counters = c.take<uint32_t>(CNT_WORDS);
    g.scan_status = c.take<uint64_t>(div_up(n + 1, SCAN_TILE) + 1);  // cleared together with the counters
    g.tile_status = c.take<uint64_t>(BK_MAX_TILES / 32 + 1);         // cleared together with the counters (32-tile column groups)
    g.rec = c.take<GRec>(n);
    g.tiles = c.take<uint32_t>(n);
    g.clamped = c.take<uint8_t>(n);
    g.live = c.take<uint8_t>(n);
    g.sh_jac = c.take<float>((size_t)9 * n);
    g.exp_rec = c.take<uint4>(n);
    g.inst_off = c.take<uint32_t>((size_t)n + 1);
    g.tiles_sorted = c.take<uint32_t>(n);
    g.exp_sorted = c.take<uint4>(n);
    g.inst_start = c.take<uint32_t>((size_t)n + 1);
    g.depth_key = c.take<uint32_t>(n);
    g.block_sums = c.take<uint32_t>(div_up(n, 256) + 1);
    g.big_list = c.take<uint32_t>(n);
    g.big_slot = c.take<uint32_t>(n);
    g.scan_tmp = c.take<uint32_t>(div_up(n + 1, SCAN_TILE) + 1);
    carve_sort(c, g.sort, n, true);  // radix path: depth sort, keys read from depth_key
    g.order = g.sort.v[0];
    return c.off + 256;
}

inline int tile_key_bits(uint32_t num_tiles) {
    int b = 0;
    while (b < 32 && (uint64_t(1) << b) < num_tiles) b++;
    return b < 1 ? 1 : b;
}
inline int radix_passes(int bits) { return (bits + 7) / 8; }

// The radix binning's tile sort (gsr_api.hip): 16-bit keys up to 65536 tiles ("tile_key16"), sorted in digits of
// "tile_db" bits (default 8; 5 gives three passes over 15-bit tile ids at 4K instead of two, with 8x longer scatter
// runs per digit, but measured 1.03 ms against 0.75 for the two 8-bit passes at cfg 5).  The carving of the binning buffer (which ping-pong slot ends as sorted_u) follows the same plan.
struct TileSortPlan {
    bool k16;
    int digit_bits, passes;
};
inline TileSortPlan tile_sort_plan(uint32_t num_tiles) {
    TileSortPlan t;
    const int bits = tile_key_bits(num_tiles);
    t.k16 = num_tiles <= 65536u && tuning("tile_key16", 1) != 0;
    t.digit_bits = t.k16 ? tuning("tile_db", 8) : 8;  // cfg 5: 8-bit digits 0.75 ms, 5-bit 1.03 (r4d)
    if (t.digit_bits < 4 || t.digit_bits > 8) t.digit_bits = 8;
    t.passes = (bits + t.digit_bits - 1) / t.digit_bits;
    return t;
}

struct BinningState {
    uint32_t *exp_owner;   // div_up(R, 256) + 2: radix path: depth rank owning each expansion block's first instance
    uint32_t *inst_gid;    // R: Gaussian of each instance (expansion order)
    uint32_t *point_list;  // R: Gaussian ids sorted by (tile, depth, id); written by the forward composite
                           //    for the instances it loads (every instance any pixel can reach)
    uint32_t *sorted_u;    // R: expansion index of each sorted instance
    uint32_t *inv;         // R: sorted position of instance u (its gradient-row marker), INV_NONE where the forward
                           //    composite did not load it (filled by the binning, set by the composite)
    uint8_t *strip_mask;   // R: per sorted instance the 4-row strips of its tile where some pixel took it (bit k =
                           //    strip k), written by the whole-tile forward composite for every instance it loaded
    // scratch of the two binning paths (overlapping: only one runs per forward)
    uint32_t *keys_sorted; // radix path: R tile ids of the sorted instances
    SortScratch sort;      // radix path: tile sort (R keys); its final value buffer is sorted_u
    unsigned long long *bk_keys;  // bucket path: R keys (depth << 32 | u) bucketed by tile
    unsigned long long *bk_keys2; // bucket path: R, the region scatter's keys grouped by region, then the chunk-sorted
                                  //    keys of tiles longer than SEG_BLOCK_CAP (seg_sort's chunked path)
    // segmented backward (small images, num_tiles <= SEG_MAX_TILES; else null): the forward's per-pixel checkpoints
    // at every K-th instance of a tile (CK_FLOATS each: T, then the colour / inverse-depth sums so far), tile t's
    // checkpoint j (before instance (j + 1) K) at index ranges[t].x / K + t + j; and the backward's work list
    float *ckpt;           // (R / CK_MIN_K + T + 1) x CK_FLOATS
    uint2 *seg_list;       // R / CK_MIN_K + T + 1 entries (tile, segment)
};
constexpr uint32_t INV_NONE = 0xffffffffu;
// Segmented backward: tiles are split into K-instance segments walked by independent waves, each starting from the
// forward's checkpoint at its end (T and the colour still to come), while the image has few tiles.
constexpr uint32_t SEG_MAX_TILES = 4096;
constexpr uint32_t CK_MIN_K = 32;
constexpr uint32_t CK_FLOATS = 5 * 256;
inline uint64_t seg_slots(int64_t R, uint32_t num_tiles) { return (uint64_t)(R > 0 ? R : 0) / CK_MIN_K + num_tiles + 1; }

inline size_t carve_binning(char *base, int64_t R, uint32_t num_tiles, BinningState &b) {
    Carver c(base);
    uint32_t n = (uint32_t)R;
    b.inst_gid = c.take<uint32_t>(n ? n : 1);
    b.point_list = c.take<uint32_t>(n ? n : 1);
    b.sorted_u = c.take<uint32_t>(n ? n : 1);
    b.inv = c.take<uint32_t>(n ? n : 1);
    b.strip_mask = c.take<uint8_t>(n ? n : 1);
    Carver cr = c;  // radix view
    const int passes = tile_sort_plan(num_tiles).passes;
    carve_sort(cr, b.sort, n, passes >= 2);
    b.exp_owner = cr.take<uint32_t>(div_up(n, 256u) + 2);
    // keys and values end in slot (passes & 1); the last pass writes its values straight into sorted_u
    b.keys_sorted = b.sort.k[passes & 1];
    b.sort.v[passes & 1] = b.sorted_u;
    Carver cb = c;  // bucket view
    b.bk_keys = cb.take<unsigned long long>(n ? n : 1);
    b.bk_keys2 = cb.take<unsigned long long>(n ? n : 1);
    c.off = cr.off > cb.off ? cr.off : cb.off;
    b.ckpt = nullptr;
    b.seg_list = nullptr;
    if (num_tiles <= SEG_MAX_TILES) {
        const uint64_t ns = seg_slots(R, num_tiles);
        b.ckpt = c.take<float>((size_t)ns * CK_FLOATS);
        b.seg_list = c.take<uint2>((size_t)ns);
    }
    return c.off + 256;
}

struct ImageState {
    float *final_T;       // W*H
    uint32_t *n_contrib;  // W*H
    uint2 *ranges;        // T
    uint32_t *tile_last;  // T: max n_contrib over the tile's pixels
    uint32_t *tile_loaded; // T: instances of the tile the forward composite gathered (>= tile_last)
    uint32_t *lpt_bcnt;    // LPT_BCNT_WORDS: tiles per backward LPT bucket (per XCD group with the XCD lists), appended
                           //      by the forward's whole-tile waves (cleared with tile_last / tile_loaded)
    uint32_t *order_fwd;   // tiles in descending forward work (instances in range), LPT launch order
    uint32_t *order_xcd;   // xcd_slots(T): the forward's launch slot -> tile map of the per-XCD LPT orders (~0: none)
    uint32_t *order_bwd;   // tiles in descending backward work (tile_last)
    // bucket path count-pass scratch (gsr_bin.hip), here rather than in the binning buffer so that the pass
    // can run before the instance total (the binning buffer's size) reaches the host
    uint32_t *bk_hist;       // BK_MAX_BLOCKS x T count matrix (empty above BK_MAX_TILES)
    uint32_t *bk_hist_pre;   // its column prefixes (a separate array: the counts stay readable for the look-back's
                             // fallback while later column workgroups run)
    uint32_t *bk_tile_next;  // T: tile starts, advanced by the region partition's slot atomics
    uint32_t *bk_reg_start;  // T / BK_REGION + 2: region starts
    uint32_t *bk_tile_start; // T + 1
    uint32_t *bk_long_list;  // 2 x (T + 1): tiles of (SEG_CAP, SEG_BLOCK_CAP] instances, longer tiles
    // segmented backward (num_tiles <= SEG_MAX_TILES): each pixel's final colour / inverse-depth sums, tile-major
    // (tile t, plane c, pixel i at t * 1024 + c * 256 + i); the checkpoint spacing K the forward used (0: none);
    // the backward's segment count
    float *ctot;
    uint32_t *ck_flag;
    uint32_t *seg_count;
    uint32_t *lpt_hist;      // (T / 4096 + 1) x 256: per-workgroup bucket histograms of the multi-workgroup LPT order
    uint32_t *lpt_blist;     // 256 x (T + 128) in lpt_append_range (else 1): bucket b's tiles at [b T, b T + lpt_bcnt[b]),
                             // or with the XCD lists bucket b of XCD group x at [(256 x + b) C, + lpt_bcnt[256 x + b])
                             // (C = xcd_slots(T) / 8)
    uint32_t *lpt_valid;     // LPT_LISTS / LPT_LISTS_XCD when this forward appended every tile to the bucket lists, else 0
    uint32_t *smask_valid;   // 1 when this forward wrote every loaded instance's strip_mask (whole tiles), else 0
};
// Between these tile counts the forward's whole-tile waves append each finished tile to its backward LPT bucket, so
// the backward needs no ordering launch (1080p, 8160 tiles: step -13 us).  At 4K (32400 tiles of similar weight in a
// few buckets) the appends' atomics on the same counters cost render_fwd 27 us, more than the launch they save.
constexpr uint32_t LPT_APPEND_TILES = 4096, LPT_APPEND_MAX_TILES = 16384;
inline bool lpt_append_range(uint32_t T) { return T > LPT_APPEND_TILES && T <= LPT_APPEND_MAX_TILES; }

// Per-XCD LPT orders (bucket path, lpt_append_range).  Workgroups b and b + 8 share an XCD and its L2 (round-robin
// dispatch, MI355X_MICROARCH.md "Workgroup dispatch"); neighbouring tiles gather the same Gaussians' render records.
// So the tiles are dealt to 8 XCD groups in spatial runs -- a band order (column bands XCD_BAND tiles wide, row-major
// inside a band) cut into runs of XCD_GROUP tiles, run r to group r % 8 -- and each group runs its own LPT order on the slots
// of one XCD: launch slot s of a composite with `per` tiles per workgroup belongs to group (s / per) % 8, as its
// q-th tile with q = (s / (8 per)) per + s % per.  Slots run to xcd_slots(T); the extra ones hold no tile.
#ifndef GSR_XCD_GROUP  // overridable for library A/B builds (tools/build_variant.py)
#define GSR_XCD_GROUP 16
#endif
#ifndef GSR_XCD_BAND
#define GSR_XCD_BAND 8
#endif
constexpr uint32_t LPT_XCD = 8;
constexpr uint32_t XCD_GROUP = GSR_XCD_GROUP;
constexpr uint32_t XCD_BAND = GSR_XCD_BAND;  // band width (tiles) of the XCD groups' band order
constexpr uint32_t LPT_BCNT_WORDS = 256 * LPT_XCD;
constexpr uint32_t LPT_LISTS = 1, LPT_LISTS_XCD = 2;  // lpt_valid values
constexpr uint32_t XCD_NONE = 0xffffffffu;            // an order_xcd slot without a tile
__host__ __device__ inline uint32_t xcd_slots(uint32_t T) {
    return (T + LPT_XCD * XCD_GROUP - 1) / (LPT_XCD * XCD_GROUP) * (LPT_XCD * XCD_GROUP);
}
__host__ __device__ inline uint32_t xcd_group_of(uint32_t t, uint32_t gx, uint32_t gy) {
    const uint32_t tx = t % gx, ty = t / gx, band = tx / XCD_BAND, bw = min(XCD_BAND, gx - band * XCD_BAND);
    const uint32_t k = band * XCD_BAND * gy + ty * bw + (tx - band * XCD_BAND);
    return (k / XCD_GROUP) % LPT_XCD;
}
__host__ __device__ inline uint32_t xcd_slot(uint32_t x, uint32_t q, uint32_t per) {
    return ((q / per) * LPT_XCD + x) * per + q % per;
}

inline size_t carve_image(char *base, int W, int H, ImageState &im) {
    Carver c(base);
    size_t npix = (size_t)W * H;
    uint32_t gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    im.final_T = c.take<float>(npix ? npix : 1);
    im.n_contrib = c.take<uint32_t>(npix ? npix : 1);
    im.ranges = c.take<uint2>((size_t)gx * gy + 1);
    im.tile_last = c.take<uint32_t>((size_t)gx * gy + 1);
    im.tile_loaded = c.take<uint32_t>((size_t)gx * gy + 1);
    im.lpt_bcnt = c.take<uint32_t>(LPT_BCNT_WORDS);
    im.order_fwd = c.take<uint32_t>((size_t)gx * gy + 1);
    im.order_xcd = c.take<uint32_t>((size_t)xcd_slots(gx * gy) + 1);
    im.order_bwd = c.take<uint32_t>((size_t)gx * gy + 1);
    const size_t nt = (size_t)gx * gy;
    im.bk_hist = c.take<uint32_t>((nt <= BK_MAX_TILES ? (size_t)BK_MAX_BLOCKS * nt : 0) + 1);
    im.bk_hist_pre = c.take<uint32_t>((nt <= BK_MAX_TILES ? (size_t)BK_MAX_BLOCKS * nt : 0) + 1);
    im.bk_tile_next = c.take<uint32_t>(nt + 1);
    im.bk_reg_start = c.take<uint32_t>(nt / BK_REGION + 2);
    im.bk_tile_start = c.take<uint32_t>(nt + 1);
    im.bk_long_list = c.take<uint32_t>(2 * (nt + 1));
    im.ctot = c.take<float>(nt <= SEG_MAX_TILES ? nt * 1024 : 1);
    im.ck_flag = c.take<uint32_t>(1);
    im.seg_count = c.take<uint32_t>(1);
    im.lpt_hist = c.take<uint32_t>((nt / 4096 + 1) * 256);
    im.lpt_blist = c.take<uint32_t>(lpt_append_range((uint32_t)nt) ? 256 * (nt + 128) : 1);
    im.lpt_valid = c.take<uint32_t>(1);
    im.smask_valid = c.take<uint32_t>(1);
    return c.off + 256;
}

// backward scratch: one gradient row per instance, then one summed row per big Gaussian
inline size_t bwd_scratch_bytes(int64_t R, int64_t nbig) {
    return align_up((size_t)(R ? R : 1) * GRAD_ROW * sizeof(float), 256) +
           align_up((size_t)(nbig ? nbig : 1) * GRAD_ROW * sizeof(float), 256) + 256;
}
inline float *bwd_bigsum_ptr(char *scratch, int64_t R) {
    return reinterpret_cast<float *>(scratch + align_up((size_t)(R ? R : 1) * GRAD_ROW * sizeof(float), 256));
}

// ------------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------------
#ifdef __HIPCC__

// The geometry chain that produces the integer outputs (radii, tile rects, kept tiles, hence num_rendered and the
// sorted instance list) and the per-Gaussian render records is evaluated WITHOUT fp contraction: every a * b + c
// rounds twice, exactly as the oracle's C (gcc -std=c11 contracts nothing) and the reference's elementwise torch
// ops do, so those outputs are bit-identical to the oracle's (VERDICT r2 "Missing #1").  Division and sqrt are
// correctly rounded by default on gfx950 (v_div_scale/fmas/fixup, v_sqrt + correction), double arithmetic likewise.
// Explicit fmaf() calls (the compositing exponent) are unaffected.  Region ends after quad_form.
#pragma clang fp contract(off)

struct Mat4 {
    float m[16];
};

__device__ __forceinline__ Mat4 load_mat4(const float *__restrict__ p) {
    Mat4 r;
#pragma unroll
    for (int i = 0; i < 16; i++) r.m[i] = p[i];
    return r;
}

// [p,1] @ M with M stored row-major (torch) == transformPoint4x4 on the column-major view
__device__ __forceinline__ float4 xform4(const float3 p, const Mat4 &m) {
    return make_float4(m.m[0] * p.x + m.m[4] * p.y + m.m[8] * p.z + m.m[12],
                       m.m[1] * p.x + m.m[5] * p.y + m.m[9] * p.z + m.m[13],
                       m.m[2] * p.x + m.m[6] * p.y + m.m[10] * p.z + m.m[14],
                       m.m[3] * p.x + m.m[7] * p.y + m.m[11] * p.z + m.m[15]);
}
__device__ __forceinline__ float3 xform3(const float3 p, const Mat4 &m) {
    return make_float3(m.m[0] * p.x + m.m[4] * p.y + m.m[8] * p.z + m.m[12],
                       m.m[1] * p.x + m.m[5] * p.y + m.m[9] * p.z + m.m[13],
                       m.m[2] * p.x + m.m[6] * p.y + m.m[10] * p.z + m.m[14]);
}

__device__ __forceinline__ float3 load_f3(const float *__restrict__ p, int i) {
    return make_float3(p[3 * i], p[3 * i + 1], p[3 * i + 2]);
}

// ndc -> pixel; the upstream form evaluates in double ((v + 1.0) * S - 1.0) * 0.5
__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)(((v + 1.0) * S - 1.0) * 0.5); }

__device__ __forceinline__ void get_rect(float2 p, int radius, int gx, int gy, int2 &rmin, int2 &rmax) {
    rmin.x = min(gx, max(0, (int)((p.x - radius) / BLOCK_X)));
    rmin.y = min(gy, max(0, (int)((p.y - radius) / BLOCK_Y)));
    rmax.x = min(gx, max(0, (int)((p.x + radius + BLOCK_X - 1) / BLOCK_X)));
    rmax.y = min(gy, max(0, (int)((p.y + radius + BLOCK_Y - 1) / BLOCK_Y)));
}

// Exact tile culling.  A (Gaussian, tile) instance is dropped only when NO pixel centre of the tile can
// pass the compositing test `o * exp(power) >= 1/255` as the kernels evaluate it in fp32, so every output
// and gradient is bitwise unchanged (the skipped instances would all hit `alpha < 1/255`).  The per-Gaussian
// threshold on q (cull_setup, double) allows for the fp32 evaluation of q at any pixel being within eps*q of the
// exact value, eps = 1e-5 (|a|+|b|+|c|) / lambda_min (>= 25x the worst-case rounding of the prescaled 5-op power2
// expression), and v_exp_f32 within 1e-5 relative.  The per-tile minimum of q over the tile's pixel rectangle is then
// evaluated in fp32 (round 5; it was double, whose dependent chains left the preprocess's waves issue-stalled).  Two
// allowances raise the threshold before it is rounded up to fp32: the rounding of q itself, at most
// 8 u (|a| dx^2 + 2|b dx dy| + |c| dy^2) <= 8 u R q with R = (|a|+|b|+|c|)/lambda_min (factor 1 + 1e-6 R), and the
// rounding of each edge's minimiser, off by d <= 4 u (|coordinate| + tight-rect half-width + 16 + |b/c| (...)) pixels,
// which overestimates the edge minimum by at most c d^2 (vertical edges) or a d^2 (horizontal ones), added absolutely.
constexpr int CULL_MAX_AREA = 64;  // <= 64: the preprocess keeps the kept tiles in a 64-bit mask (and divides by rw with a multiply)
struct CullGauss {
    float x, y, a, b2, c, ba, bc, thr;  // b2 = 2 b, ba = b / a, bc = b / c, thr: fp32 threshold on q_min (rounded up)
    int mode;                           // 0: test each tile, 1: keep every tile, 2: drop every tile
    double ex, ey;                      // half-widths of the ellipse q <= thr's bounding box (cull_rect)
};
// Per-Gaussian part of the test (once per Gaussian): the error-adjusted threshold on q_min.
__host__ __device__ inline CullGauss cull_setup(double x, double y, double a, double b, double c, double o) {
    CullGauss g{(float)x, (float)y, (float)a, (float)(2.0 * b), (float)c, 0.f, 0.f, 0.f, 0, 0.0, 0.0};
    if (!(o * 255.0 * (1.0 + 1e-5) >= 1.0)) {  // o*G <= o < 1/255 everywhere
        g.mode = 2;
        return g;
    }
    const double tr = 0.5 * (a + c), df = 0.5 * (a - c);
    const double lmin = tr - sqrt(df * df + b * b);
    if (!(lmin > 0.0) || !(a > 0.0) || !(c > 0.0)) {
        g.mode = 1;
        return g;
    }
    const double R = (fabs(a) + fabs(b) + fabs(c)) / lmin;
    const double eps = 1e-5 * R;
    if (eps > 0.1) {
        g.mode = 1;
        return g;
    }
    // cull iff q_min (1 - eps) - 1e-6 > 2 ln(255 o (1 + 1e-5))
    const double thr = (2.0 * log(255.0 * o * (1.0 + 1e-5)) + 1e-6) / (1.0 - eps);
    const double det = a * c - b * b;  // > 0 (lambda_min > 0)
    g.ex = sqrt(thr * c / det) * (1.0 + 1e-9) + 1e-6;
    g.ey = sqrt(thr * a / det) * (1.0 + 1e-9) + 1e-6;
    const double ba = b / a, bc = b / c, u4 = 4.0 * 0x1p-24;
    const double dv = u4 * (fabs(y) + g.ey + 16.0 + fabs(bc) * (g.ex + 16.0));
    const double dh = u4 * (fabs(x) + g.ex + 16.0 + fabs(ba) * (g.ey + 16.0));
    g.ba = (float)ba;
    g.bc = (float)bc;
    g.thr = (float)((thr * (1.0 + 1e-6 * R) + c * dv * dv + a * dh * dh) * (1.0 + 1e-7));
    return g;
}
// Per-tile part: minimum of the quadratic form over the tile's pixel rectangle, in fp32.  The minimum of the convex q
// over a rectangle that does not hold the centre lies on an edge facing the centre: on the interior of an edge the
// gradient is normal to it, pointing out of the rectangle, and the line of conditional minima through that point runs
// to the centre, which therefore lies beyond that edge.  So at most one vertical edge (the one facing the centre, when
// x is outside [lx, hx]) and one horizontal edge are evaluated, each at its clamped stationary point; a corner minimum
// is the clamp of both.
__host__ __device__ inline bool cull_keep(const CullGauss &g, int tx, int ty, int W, int H) {
    const float lx = (float)(tx * BLOCK_X), ly = (float)(ty * BLOCK_Y);
    const float hx = (float)min(tx * BLOCK_X + BLOCK_X - 1, W - 1);
    const float hy = (float)min(ty * BLOCK_Y + BLOCK_Y - 1, H - 1);
    const bool in_x = g.x >= lx && g.x <= hx, in_y = g.y >= ly && g.y <= hy;
    // both edges are evaluated unconditionally and the one not facing the centre is replaced afterwards (branch-free:
    // the lanes of a wave test different tiles)
    float dx = g.x - (g.x < lx ? lx : hx);  // the vertical edge x = X facing the centre: minimise over y
    float dy = g.y - fminf(fmaxf(g.y + g.bc * dx, ly), hy);
    const float qv = g.a * dx * dx + g.b2 * dx * dy + g.c * dy * dy;
    dy = g.y - (g.y < ly ? ly : hy);  // the horizontal edge y = Y facing the centre: minimise over x
    dx = g.x - fminf(fmaxf(g.x + g.ba * dy, lx), hx);
    const float qh = g.a * dx * dx + g.b2 * dx * dy + g.c * dy * dy;
    const float qmin = fminf(in_x ? 3.0e38f : qv, in_y ? 3.0e38f : qh);
    // mode 1 keeps and mode 2 drops every tile (their conic fields are not set up)
    return g.mode == 1 || (g.mode == 0 && ((in_x && in_y) || !(qmin > g.thr)));
}

// Tight rect: the tiles of [x0, x1) x [y0, y1) (the reference rect on entry) that meet the bounding box of the ellipse
// q <= thr, outside which no pixel centre can pass the compositing test (cull_setup's error-adjusted threshold);
// tile tx is kept while 16 tx <= x + ex and 16 (tx + 1) > x - ex.  Mode 2 empties the rect, mode 1 keeps it.  Big
// Gaussians (tight rect > CULL_MAX_AREA tiles) keep their whole tight rect; smaller ones are culled tile by tile
// inside it.  At 4K with 1 % bloated Gaussians the 3-sigma rects of the big ones held 24 M of 48 M instances.
__host__ __device__ inline void cull_rect(const CullGauss &g, int &x0, int &y0, int &x1, int &y1) {
    if (g.mode == 2) {
        x1 = x0;
        y1 = y0;
        return;
    }
    if (g.mode == 1) return;
    const double ex = g.ex, ey = g.ey;
    const int tx0 = (int)floor((g.x - ex) / BLOCK_X), tx1 = (int)floor((g.x + ex) / BLOCK_X) + 1;
    const int ty0 = (int)floor((g.y - ey) / BLOCK_Y), ty1 = (int)floor((g.y + ey) / BLOCK_Y) + 1;
    x0 = x0 > tx0 ? x0 : tx0;
    x1 = x1 < tx1 ? x1 : tx1;
    y0 = y0 > ty0 ? y0 : ty0;
    y1 = y1 < ty1 ? y1 : ty1;
    if (x1 < x0) x1 = x0;
    if (y1 < y0) y1 = y0;
}

// SH basis constants (utils/sh.py:7-28 of the reference)
#define GSR_SH_C0 0.28209479177387814f
#define GSR_SH_C1 0.4886025119029199f
__constant__ const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                                     -1.0925484305920792f, 0.5462742152960396f};
__constant__ const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                                     0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                                     -0.5900435899266435f};

// Rotation (glm column-major R[c][r]) from an unnormalised (w,x,y,z) quaternion.
struct Mat3 {
    float m[3][3];
};
__device__ __forceinline__ Mat3 quat_to_rot(float4 q) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    Mat3 R;
    R.m[0][0] = 1.f - 2.f * (y * y + z * z); R.m[0][1] = 2.f * (x * y - r * z); R.m[0][2] = 2.f * (x * z + r * y);
    R.m[1][0] = 2.f * (x * y + r * z); R.m[1][1] = 1.f - 2.f * (x * x + z * z); R.m[1][2] = 2.f * (y * z - r * x);
    R.m[2][0] = 2.f * (x * z - r * y); R.m[2][1] = 2.f * (y * z + r * x); R.m[2][2] = 1.f - 2.f * (x * x + y * y);
    return R;
}

// Sigma = R S S^T R^T as 6 upper-triangle values (render_tools.py:56-70)
__device__ __forceinline__ void cov3d_from_scale_rot(float3 s, float mod, float4 q, float out[6]) {
    Mat3 R = quat_to_rot(q);
    const float sv[3] = {mod * s.x, mod * s.y, mod * s.z};
    float M[3][3];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++) M[c][r] = sv[r] * R.m[c][r];
    // Sigma[c][r] = sum_k M[r][k] * M[c][k]
    auto sig = [&](int c, int r) { return M[r][0] * M[c][0] + M[r][1] * M[c][1] + M[r][2] * M[c][2]; };
    out[0] = sig(0, 0); out[1] = sig(0, 1); out[2] = sig(0, 2);
    out[3] = sig(1, 1); out[4] = sig(1, 2); out[5] = sig(2, 2);
}

// EWA Jacobian rows times the view rotation (render_tools.py:13-52): t0 = J0 * Rv, t1 = J1 * Rv.
struct EwaT {
    float t0[3], t1[3];
    float3 t;  // view-space mean with clamped x, y
    float xmul, ymul;
};
__device__ __forceinline__ EwaT ewa_T(float3 mean, const Mat4 &view, float fx, float fy, float tanx, float tany) {
    EwaT e;
    float3 t = xform3(mean, view);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    e.xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    e.ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float j00 = fx / t.z, j02 = -(fx * t.x) / (t.z * t.z);
    const float j11 = fy / t.z, j12 = -(fy * t.y) / (t.z * t.z);
#pragma unroll
    for (int r = 0; r < 3; r++) {
        e.t0[r] = view.m[4 * r + 0] * j00 + view.m[4 * r + 2] * j02;
        e.t1[r] = view.m[4 * r + 1] * j11 + view.m[4 * r + 2] * j12;
    }
    e.t = t;
    return e;
}

__device__ __forceinline__ float quad_form(const float a[3], const float c6[6], const float b[3]) {
    // a^T V b with V the symmetric matrix of c6
    const float v0 = c6[0] * b[0] + c6[1] * b[1] + c6[2] * b[2];
    const float v1 = c6[1] * b[0] + c6[3] * b[1] + c6[4] * b[2];
    const float v2 = c6[2] * b[0] + c6[4] * b[1] + c6[5] * b[2];
    return a[0] * v0 + a[1] * v1 + a[2] * v2;
}
#pragma clang fp contract(fast)  // end of the uncontracted geometry region

// exp(x) as v_exp_f32(x * log2 e): 2 instructions instead of the 13 of the correctly rounded expf.
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// Compositing exponent, evaluated identically by the forward and the backward composite (so the backward's
// T recovery divides by exactly the (1 - alpha) the forward multiplied with).  In base 2 and with the conic
// prescaled when a batch is staged into LDS -- (A, B, C) = -log2(e) (a/2, b, c/2) -- the exponent is
//     power2 = log2(e) * power = A dx^2 + B dx dy + C dy^2,   G = v_exp_f32(power2).
// A lane's pixels share one column, so P0 = A dx^2 and L = B dx are formed once per instance and every pixel
// costs dy, fma, fma.  Relative error vs the reference's expf(power) ~1e-7 (DESIGN.md "Numerics").
constexpr float NEG_HALF_LOG2E = -0.72134752044448170f;
constexpr float NEG_LOG2E = -1.4426950408889634f;
__device__ __forceinline__ float4 stage_rec_a(float4 a) {  // (x, y, conic.x, conic.y) -> (x, y, A, B)
    return make_float4(a.x, a.y, a.z * NEG_HALF_LOG2E, a.w * NEG_LOG2E);
}
__device__ __forceinline__ float4 stage_rec_b(float4 b) {  // (conic.z, o, r, g) -> (C, o, r, g)
    return make_float4(b.x * NEG_HALF_LOG2E, b.y, b.z, b.w);
}
// Per-lane select by a wave lane mask held in scalar registers (e.g. from __builtin_amdgcn_fcmpf): one
// v_cndmask_b32 that reads the mask directly, where `cond ? a : b` on a bool rebuilt from a mask would first
// materialise it in a vector register.  Lanes outside exec are left undefined, as any VALU result.
__device__ __forceinline__ float select_mask(uint64_t mask, float a, float b) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(mask));
    return r;
}
// LLVM CmpInst predicates for __builtin_amdgcn_fcmpf / __builtin_amdgcn_uicmp
constexpr int FCMP_OLT = 4, FCMP_OLE = 5, FCMP_UGE = 11, FCMP_ULE = 13, ICMP_ULT = 36;

// One staged compositing record in LDS (48 B): both composite passes read a batch's instances from an array
// of these with immediate offsets from one address.
struct alignas(16) FwdRec {
    float4 a;  // x, y, A, B (stage_rec_a)
    float4 b;  // C, o, r, g (stage_rec_b)
    float2 c;  // b, 1/depth
    float2 pad;
};

__device__ __forceinline__ float power2_at(float C, float dy, float P0, float L) {
    return fmaf(dy, fmaf(C, dy, L), P0);
}

// Threshold guard band (knob "guard"; off by default).  The fast alpha above differs from the oracle's
// expf(power) by a few ulps of the exponent's term magnitudes, so a pair whose alpha lies within that error of 1/255,
// or whose T (1 - alpha) lies within it of 1e-4, may be decided differently from the oracle (a threshold flip).
// With the guard, such a pair's DECISIONS are re-taken from the oracle's own arithmetic: the exponent in its
// uncontracted order from the raw record, and exp in double rounded once to fp32 (the correctly rounded expf, which
// glibc's equals but for its rare 0.502-ulp misroundings).  The values (alpha in the colour and T updates) stay the
// fast ones, so the backward, which re-takes the alpha decision by the same test, stays consistent with the forward.
constexpr float GUARD_A_LO = (1.0f / 255.0f) * (1.0f - 2e-5f), GUARD_A_HI = (1.0f / 255.0f) * (1.0f + 2e-5f);
// oracle order (gsr_oracle.c render loop): -0.5 (a dx dx + c dy dy) - b dx dy, no contraction; ra = raw rec a
// (x, y, conic a, conic b), cz = conic c
__device__ __forceinline__ float guard_power(float4 ra, float cz, float pfx, float pfy) {
#pragma clang fp contract(off)
    const float dx = ra.x - pfx, dy = ra.y - pfy;
    return -0.5f * (ra.z * dx * dx + cz * dy * dy) - ra.w * dx * dy;
}
// exp(x) rounded once to fp32 (the correctly rounded expf but for double-rounding ties): Cody-Waite reduction by ln 2
// and a degree-11 Taylor polynomial in double (relative error ~1e-15), lighter in registers than the library's
// double exp.  For the guard's exponents (about -6 .. 0; anything below -87 underflows to 0 as expf does).
__device__ __forceinline__ float guard_expf(float x) {
    if (!(x > -87.5f)) return 0.0f;
    const double xd = (double)x;
    const double n = __builtin_rint(xd * 1.4426950408889634);
    const double r = __builtin_fma(n, -1.90821492927058770002e-10, __builtin_fma(n, -6.93147180369123816490e-01, xd));
    double p = 2.505210838544172e-08;  // 1/11!
    p = __builtin_fma(p, r, 2.755731922398589e-07);
    p = __builtin_fma(p, r, 2.755731922398589e-06);
    p = __builtin_fma(p, r, 2.48015873015873e-05);
    p = __builtin_fma(p, r, 1.984126984126984e-04);
    p = __builtin_fma(p, r, 1.388888888888889e-03);
    p = __builtin_fma(p, r, 8.333333333333333e-03);
    p = __builtin_fma(p, r, 4.166666666666666e-02);
    p = __builtin_fma(p, r, 1.666666666666667e-01);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    return (float)__builtin_ldexp(p, (int)n);
}
__device__ __forceinline__ float guard_alpha(float power, float o) {
    return fminf(0.99f, o * guard_expf(power));
}
// The oracle's alpha decision for Gaussian g at pixel (pfx, pfy): power <= 0 and alpha >= 1/255.  Inlined into a
// branch marked unlikely (an out-of-line call made the compositing loops save their scalar state around it and spill).
__device__ __forceinline__ bool guard_alpha_pass(const GRec *__restrict__ rec, uint32_t g, float pfx, float pfy) {
    const float4 ra = rec[g].a;
    const float2 rb = *reinterpret_cast<const float2 *>(&rec[g].b);
    const float pw = guard_power(ra, rb.x, pfx, pfy);
    return pw <= 0.0f && guard_alpha(pw, rb.y) >= 1.0f / 255.0f;
}

// Conservative 4-bit mask of the 4-row strips of a 16-row tile (first row row0) that hold a pixel where
// the Gaussian can pass the compositor's alpha >= 1/255 test.  a = raw rec_a (x, y, conic a, conic b),
// b = raw rec_b (conic c, opacity, ...).  alpha = min(0.99, o exp(power)) >= 1/255 needs
// d^T Q d <= tau = 2 ln(255 o) (Q = [[a, b], [b, c]]), whose row extent is |dy| <= sqrt(tau (Q^-1)_yy) =
// sqrt(tau a / (a c - b^2)).  1 % + 1 px of margin absorb the fp32 error of this bound; degenerate or
// non-finite conics keep every strip.
__device__ __forceinline__ uint32_t strip_mask(float4 a, float4 b, float row0) {
    const float o255 = 255.f * b.y;
    if (!(o255 >= 0.999f)) return o255 < 0.999f ? 0u : 0xfu;  // alpha <= o < 1/255 everywhere (NaN: keep all)
    const float det = a.z * b.x - a.w * a.w;
    const float tau = 2.f * __logf(fmaxf(o255, 1.f)) + 1e-3f;
    const float e = sqrtf(tau * a.z / det) * 1.01f + 1.f;
    if (!(det > 0.f) || !(e < 1e6f)) return 0xfu;
    const float lo = a.y - e - row0, hi = a.y + e - row0;  // band of rows, relative to the tile
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) m |= (hi >= 4.f * k && lo <= 4.f * k + 3.f) ? (1u << k) : 0u;
    return m;
}

// The same mask from the ellipse's row extent INSIDE the tile's column band [col0, col0 + 15] instead of its
// global row extent: cells of a Gaussian that only clips the tile's side drop out (at 1M Gaussians / 1080p the
// live strips fall from 0.82 to 0.69 of all, tools/cell_stats.py).  In offsets (u, v) = (px - x, py - y) the
// pass region is q = a u^2 + 2 b u v + c v^2 <= tau.  Its highest point (v = +V, V = sqrt(tau a / det)) lies at
// u = -b V / a; if that is outside the band, the highest point within the band is on the nearer band edge,
// where the vertical chord of the ellipse ends at v = (-b u + sqrt(c tau - det u^2)) / c; the lowest point is
// the mirror image.  The bound is conservative: tau carries the error allowance of the exact tile culling
// (cull_setup: fp32 evaluation of q within eps q, eps = 1e-5 (|a|+|b|+|c|) / lambda_min) plus 1e-3, and the
// row interval 1e-2 V + 1/16 px; elongated conics (eps >= 1e-2), degenerate or non-finite ones keep
// every strip.  A skipped strip therefore holds no pixel that passes, and outputs are bitwise unchanged.
__device__ __forceinline__ uint32_t strip_mask_exact(float4 a, float4 b, float row0, float col0) {
    const float A = a.z, B = a.w, C = b.x;
    const float o255 = 255.f * b.y;
    if (!(o255 >= 0.999f)) return o255 < 0.999f ? 0u : 0xfu;  // alpha <= o < 1/255 everywhere (NaN: keep all)
    const float det = A * C - B * B;
    const float hd = 0.5f * (A - C);
    const float lmin = 0.5f * (A + C) - sqrtf(hd * hd + B * B);
    if (!(det > 0.f) || !(lmin > 0.f)) return 0xfu;
    const float eps = 1e-5f * (fabsf(A) + fabsf(B) + fabsf(C)) / lmin;
    if (!(eps < 1e-2f)) return 0xfu;
    const float tau = (2.f * __logf(fmaxf(o255 * 1.00001f, 1.f)) + 1e-3f) / (1.f - eps);
    const float V = sqrtf(tau * A / det);
    if (!(V < 1e6f)) return 0xfu;
    const float uL = col0 - a.x, uR = uL + (float)(BLOCK_X - 1);
    const float ut = -B * V / A;  // u of the highest point; the lowest is at -ut
    const float ic = 1.f / C, ctau = C * tau;
    float vmax = V, vmin = -V;
    if (!(ut >= uL && ut <= uR)) {
        const float u = fminf(fmaxf(ut, uL), uR);
        vmax = (-B * u + sqrtf(fmaxf(ctau - det * u * u, 0.f))) * ic;
    }
    if (!(-ut >= uL && -ut <= uR)) {
        const float u = fminf(fmaxf(-ut, uL), uR);
        vmin = (-B * u - sqrtf(fmaxf(ctau - det * u * u, 0.f))) * ic;
    }
    // near-tangent chords amplify the rounding of c tau - det u^2 (det to ~6e-5 relative at eps < 1e-2): <= 1e-2 V
    const float mg = 1e-2f * V + 1e-3f * (fabsf(uL) + fabsf(uR)) + 0.0625f;
    const float lo = a.y + vmin - mg - row0, hi = a.y + vmax + mg - row0;  // band of rows, relative to the tile
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) m |= (hi >= 4.f * k && lo <= 4.f * k + 3.f) ? (1u << k) : 0u;
    return m;
}

__device__ __forceinline__ uint32_t cell_mask(bool exact, float4 a, float4 b, float row0, float col0) {
    return exact ? strip_mask_exact(a, b, row0, col0) : strip_mask(a, b, row0);
}

// --- per-instance gradient rows (render_bwd -> big_reduce / preprocess_bwd) -------------------------
// Row layout: [0] dmean2D.x  [1] dmean2D.y  [2] dconic.x  [3] dconic.y  [4] dconic.w  [5] dopacity
//             [6..8] dcolor  [9] dinvdepth; 40 B, accessed as five 8-B words (no pad: the rows are a third of the
//             backward's HBM traffic)
__device__ __forceinline__ void load_row(const float *__restrict__ rows, size_t s, float r[10]) {
    const float2 *src = reinterpret_cast<const float2 *>(rows + s * GRAD_ROW);
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const float2 v = src[k];
        r[2 * k] = v.x;
        r[2 * k + 1] = v.y;
    }
}

// a gradient row with a non-zero term: its Gaussian's per-Gaussian backward has work (GeomState::live)
__device__ __forceinline__ bool row_nonzero(const float r[10]) {
    bool nz = false;
#pragma unroll
    for (int k = 0; k < 10; k++) nz = nz || r[k] != 0.f;
    return nz;
}
__device__ __forceinline__ void store_row(float *__restrict__ rows, uint32_t s, const float r[10]) {
    float2 *dst = reinterpret_cast<float2 *>(rows + (size_t)s * GRAD_ROW);
#pragma unroll
    for (int k = 0; k < 5; k++) dst[k] = make_float2(r[2 * k], r[2 * k + 1]);
}

__device__ __forceinline__ void add_row(const float *__restrict__ rows, uint32_t s, float acc[10]) {
    float r[10];
    load_row(rows, s, r);
#pragma unroll
    for (int k = 0; k < 10; k++) acc[k] += r[k];
}

// --- wave64 primitives ---------------------------------------------------------------------------
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf, bool BOUND = false>
__device__ __forceinline__ float dpp_mov(float old, float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROW_MASK,
                                                      BANK_MASK, BOUND));
}

// keep + (v moved across lanes by DPP CTRL).  With full row/bank masks and a pattern that defines every lane
// (quad_perm, row_ror, row_mirror, row_half_mirror) bound_ctrl does not change the result, and it is what lets
// the compiler fold the move into the add (one v_add_f32_dpp instead of v_mov_b32_dpp + v_add_f32).  Partial
// masks keep the plain move: lanes outside ROW_MASK/BANK_MASK then receive an undefined value, so callers only
// read lanes the pattern fully defines.
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ float dpp_xadd(float keep, float v) {
    constexpr bool FULL = ROW_MASK == 0xf && BANK_MASK == 0xf;
    return keep + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, ROW_MASK, BANK_MASK, FULL));
}
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ float dpp_add(float v) {
    return dpp_xadd<CTRL, ROW_MASK, BANK_MASK>(v, v);
}

// Sum over the 64 lanes (every lane must be active); the result is returned wave-uniform.
__device__ __forceinline__ float wave_sum(float v) {
    v = dpp_add<0xB1>(v);        // quad_perm [1,0,3,2]
    v = dpp_add<0x4E>(v);        // quad_perm [2,3,0,1]
    v = dpp_add<0x141>(v);       // row_half_mirror
    v = dpp_add<0x140>(v);       // row_mirror -> row sums in every lane
    v = dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3 (lane 31 = r0 + r1)
    v = dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3 (lane 63 = total)
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

// inclusive prefix sum over the wave (lanes in order)
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = (uint32_t)__shfl_up((int)v, o);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (lane == 0) ? 0ull : (~0ull >> (64 - lane)); }

// Decoupled look-back by one whole wave, with decoupled fallback: publishes the block's aggregate, then sums
// predecessors' words 64 at a time (nearest first) up to the first inclusive prefix, and publishes its own
// inclusive prefix.  Returns the block's exclusive prefix (every lane).  Status words: 2-bit flag | 62-bit value,
// zero = not yet published.  Block ids follow start order (atomic ticket).
// A predecessor that has not published within `patience` polls -- a block that is not running, e.g. preempted --
// is not waited for: its aggregate is recomputed from the kernel's input by agg_of(q) (a wave-cooperative call
// returning the same value that block would publish; the inputs are never written by the kernel), so the chain
// always completes with the same result (the "decoupled fallback" of Smith, Levien & Owens).  With `force` every
// status word is ignored and every predecessor recomputed (the test of the fallback).  Bit 2 of *err records that
// a fallback ran (diagnostic only: the output is exact either way).
constexpr uint64_t SLB_AGG = 1ull << 62, SLB_INC = 2ull << 62, SLB_MASK = (1ull << 62) - 1;
template <class AggOf>
__device__ __forceinline__ uint64_t wave_lookback(uint64_t *status, uint32_t bid, uint64_t agg, int lane,
                                                  uint32_t *err, uint32_t patience, bool force, AggOf agg_of) {
    if (lane == 0)
        __hip_atomic_store(status + bid, (bid == 0 ? SLB_INC : SLB_AGG) | agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    int64_t look = (int64_t)bid - 1;
    uint32_t spins = 0;
    while (look >= 0) {
        const int64_t q = look - lane;
        uint64_t sv = q < 0 ? SLB_INC
                            : force ? 0ull : __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t inc_mask = __ballot((sv & ~SLB_MASK) == SLB_INC);
        const int first = inc_mask ? __builtin_ctzll(inc_mask) : 64;
        const uint64_t upto = first < 63 ? ((2ull << first) - 1) : ~0ull;
        uint64_t unpub = __ballot((sv & ~SLB_MASK) == 0) & upto;
        if (unpub) {  // a predecessor in the window has not published yet
            if (!force && ++spins <= patience) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            if (lane == 0) atomicOr(err, 4u);
            while (unpub) {  // recompute those aggregates, nearest first (wave-uniform loop)
                const int j = __builtin_ctzll(unpub);
                unpub &= unpub - 1;
                const uint64_t v = agg_of((uint32_t)(look - j));
                if (lane == j) sv = SLB_AGG | v;
            }
            spins = 0;
        }
        uint64_t part = (lane <= first) ? (sv & SLB_MASK) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
        excl += part;
        if (first < 64) break;
        look -= 64;
    }
    if (lane == 0 && bid > 0)
        __hip_atomic_store(status + bid, SLB_INC | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// wave-uniform 64-bit sum of one value per lane
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Wave timeline stamp (diagnostics): 100 MHz real-time clock at start / end, HW_ID and XCC_ID registers.
__device__ __forceinline__ uint32_t stamp_now() { return (uint32_t)__builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void stamp_store(uint4 *stamps, int slot, uint32_t t0, int lane) {
    if (!stamps || lane != 0 || slot >= STAMP_SLOTS) return;
    const uint32_t t1 = stamp_now();
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    stamps[slot] = make_uint4(t0, t1, hw, xcc);
}

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

// Tile of cell c of a rect at (rx, ry) of width w: the row floor((c + 1/2) / w) in fp32 is exact here ((c + 1/2) / w is
// at least 1/(2w) from an integer and far below 2^20).  Used by the bucket walks and the radix path's expansion.
// (row, column) of cell c of a rect of width w: floor((c + 1/2) / w) in fp32 is exact here ((c + 1/2) / w is
// at least 1/(2w) from an integer and far below 2^20)
__device__ __forceinline__ uint32_t rect_tile(uint32_t c, uint32_t rx, uint32_t ry, uint32_t w, float inv_w,
                                              uint32_t gx) {
    const uint32_t cy = (uint32_t)(((float)c + 0.5f) * inv_w);
    return (ry + cy) * gx + rx + (c - cy * w);
}

// Position of the j-th (from 0) set bit of m, j < popcount(m): a branch-free binary search on popcounts.
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t m, uint32_t j) {
    uint32_t c = 0, r = j;
#pragma unroll
    for (int wd = 32; wd >= 1; wd >>= 1) {
        const uint32_t cnt = (uint32_t)__popcll(m & ((1ull << wd) - 1ull));
        if (r >= cnt) {
            r -= cnt;
            m >>= wd;
            c += (uint32_t)wd;
        }
    }
    return c;
}
// Wave-cooperative search: last index r in [0, n] with off[r] <= u (off non-decreasing, off[0] <= u).
// 64 probes per step, so ~log64(n) dependent global loads instead of log2(n).
__device__ __forceinline__ uint32_t wave_last_le(const uint32_t *__restrict__ off, uint32_t n, uint32_t u,
                                                 int lane) {
    uint32_t lo = 0, hi = n;
    while (hi - lo >= 64) {
        const uint32_t step = (hi - lo) / 65;
        const uint32_t st = step ? step : 1;
        const uint32_t probe = lo + (uint32_t)(lane + 1) * st;
        const bool pred = probe <= hi && off[probe] <= u;
        const uint32_t c = (uint32_t)__popcll(__ballot(pred));
        const uint32_t nlo = lo + c * st;
        const uint32_t nhi = (c < 64) ? lo + (c + 1) * st - 1 : hi;
        lo = nlo;
        hi = nhi;
    }
    const uint32_t probe = lo + (uint32_t)lane;
    const bool pred = probe <= hi && off[probe] <= u;
    return lo + (uint32_t)__popcll(__ballot(pred)) - 1;
}

// Orders LDS writes before later LDS reads of other lanes of the SAME wave (no s_barrier).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LPT (longest-processing-time-first) tile order by one workgroup of any multiple of 64 threads: histogram of the
// tile weights (range length, or tile_last when use_last) in 2^shift-instance buckets, heaviest first, exclusive
// scan by one wave, scatter.  Order inside a bucket is arbitrary -- it only changes which tile runs when, never
// a result.  hist: 256 + 16 words of LDS (LPT_HIST_WORDS).  Run by tile_order_kernel and by the bucket scatter's extra workgroup.
// * shift adapts to the heaviest tile: max(shift0, bits(max weight) - 8), at most 9, so long-tile images (4K
//   stress: ~1500 instances per tile) spread over the buckets instead of piling into bucket 0 (the first slots
//   stay exactly the tiles above SEG_CAP while 512 is a multiple of the bucket width, which seg_sort relies on);
// * a thread's weights are loaded once, all together (up to KMAX per thread), not one dependent load per
//   histogram / scatter iteration (one workgroup over 32400 tiles took 25-30 us);
// * lanes of a wave with the same bucket share one LDS atomic (ballot-matched peers), so heavily shared buckets do
//   not serialise.
// Backward launch slot -> tile from the forward's bucket lists (heaviest bucket first): the wave forms the exclusive
// prefix of the 256 bucket counts (4 per lane) and picks the bucket holding the slot.  Uniform result.
// Launch slot -> tile from bucket lists: bcnt[0..255] the bucket sizes, bucket b's tiles at blist[b stride ..];
// returns `none` when slot is past the lists' total.
__device__ __forceinline__ int lpt_list_tile(const uint32_t *__restrict__ bcnt, const uint32_t *__restrict__ blist,
                                             uint32_t stride, uint32_t slot, int lane, int none) {
    const uint4 c = reinterpret_cast<const uint4 *>(bcnt)[lane];
    const uint32_t sum = c.x + c.y + c.z + c.w;
    const uint32_t pre = wave_inclusive_scan(sum, lane) - sum;
    const uint32_t p1 = pre + c.x, p2 = p1 + c.y, p3 = p2 + c.z, p4 = p3 + c.w;
    const bool mine = slot >= pre && slot < p4;
    const uint64_t m = __ballot(mine);
    int tile = none;
    if (m) {
        const int src = __builtin_ctzll(m);
        uint32_t b = 0, off = 0;
        if (mine) {
            b = 4u * (uint32_t)lane + (slot >= p1) + (slot >= p2) + (slot >= p3);
            off = slot - (slot >= p3 ? p3 : slot >= p2 ? p2 : slot >= p1 ? p1 : pre);
        }
        b = (uint32_t)__shfl((int)b, src);
        off = (uint32_t)__shfl((int)off, src);
        tile = (int)blist[(size_t)b * stride + off];
    }
    return __builtin_amdgcn_readfirstlane(tile);
}
// The same over the per-XCD lists (one tile per workgroup): slot s is the (s / 8)-th tile of XCD group s % 8; -1 when
// that group has fewer tiles.
__device__ __forceinline__ int lpt_list_tile_xcd(const uint32_t *__restrict__ bcnt, const uint32_t *__restrict__ blist,
                                                 uint32_t T, uint32_t slot, int lane) {
    const uint32_t x = slot % LPT_XCD, cap = xcd_slots(T) / LPT_XCD;
    return lpt_list_tile(bcnt + 256u * x, blist + (size_t)256u * x * cap, cap, slot / LPT_XCD, lane, -1);
}

constexpr int LPT_KMAX = 32;
constexpr int LPT_HIST_WORDS = 256 + 16;  // tile weights a thread keeps in registers (T <= 32 x the workgroup size)
// One histogram (order == null) or scatter pass over the tiles; item k of thread tid is tile tid + k nt.
// bucket b of tile t (ballot-matched peers share one LDS atomic): histogram (order == null) or scatter to order
__device__ __forceinline__ void lpt_item_b(int t, uint32_t b, bool valid, uint32_t *hist, uint32_t *order, int lane,
                                           uint64_t lt) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; bit++) {
        const bool set = (b >> bit) & 1u;
        const uint64_t m = __ballot(set);
        peers &= set ? m : ~m;
    }
    const uint64_t lower = peers & lt;
    uint32_t base = 0;
    if (valid && lower == 0) base = atomicAdd(&hist[b], (uint32_t)__popcll(peers));
    if (order) {
        const int leader = valid ? __builtin_ctzll(peers) : lane;
        base = (uint32_t)__shfl((int)base, leader);
        if (valid) order[base + (uint32_t)__popcll(lower)] = (uint32_t)t;
    }
}
__device__ __forceinline__ void lpt_item(int t, uint32_t wgt, bool valid, uint32_t shift, uint32_t *hist,
                                         uint32_t *order, int lane, uint64_t lt) {
    lpt_item_b(t, valid ? 255u - min(255u, wgt >> shift) : 0u, valid, hist, order, lane, lt);
}
// Scale-free LPT bucket for the multi-workgroup order (no max pass): heaviest first by the weight's exponent and
// its next 3 bits (buckets 1/8 of a binade wide); weight 0 last.
__device__ __forceinline__ uint32_t lpt_log_bucket(uint32_t w) {
    if (w == 0) return 255u;
    const uint32_t e = 31u - (uint32_t)__builtin_clz(w);
    const uint32_t m = e >= 3 ? (w >> (e - 3)) & 7u : (w << (3 - e)) & 7u;
    return 255u - (e * 8u + m);
}
template <class LoadW>
__device__ __forceinline__ void lpt_walk(int T, bool cached, const uint32_t (&wt)[LPT_KMAX], LoadW load_w,
                                         uint32_t shift, uint32_t *hist, uint32_t *order) {
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63;
    const uint64_t lt = lanemask_lt(lane);
    if (cached) {
#pragma unroll
        for (int k = 0; k < LPT_KMAX; k++) {
            if (k * nt >= T) break;  // uniform
            const int t = tid + k * nt;
            lpt_item(t, wt[k], t < T, shift, hist, order, lane, lt);
        }
    } else {
        for (int k0 = 0; k0 < T; k0 += nt) {  // uniform trip count
            const int t = tid + k0;
            lpt_item(t, t < T ? load_w(t) : 0u, t < T, shift, hist, order, lane, lt);
        }
    }
}
// xmap (optional, with xhist: LPT_BCNT_WORDS + LPT_XCD + 16 words of LDS): also the per-XCD LPT slot map of a composite
// with `per` tiles per workgroup (order_xcd; gx, gy the tile grid)
__device__ __forceinline__ void lpt_order_block(const uint2 *__restrict__ ranges, const uint32_t *__restrict__ tile_last,
                                                int use_last, int T, int shift0, uint32_t *__restrict__ order,
                                                uint32_t *hist, uint32_t *__restrict__ xmap = nullptr,
                                                uint32_t *xhist = nullptr, int gx = 0, int gy = 0, int per = 4) {
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, w = tid >> 6;
    auto load_w = [&](int t) -> uint32_t { return use_last ? tile_last[t] : ranges[t].y - ranges[t].x; };
    const bool cached = T <= nt * LPT_KMAX;
    uint32_t wt[LPT_KMAX];
    uint32_t mx = 0;
    if (cached) {
        // every load issued before any use, unconditional (clamped index): a load in a branch -- even a uniform one,
        // `k * nt < T ? load : 0` per round -- was waited for at the branch's join, one round trip per round in use
        // (rounds past T re-read the last tile: the same cache line)
#pragma unroll
        for (int k = 0; k < LPT_KMAX; k++) wt[k] = load_w(min(tid + k * nt, T - 1));
#pragma unroll
        for (int k = 0; k < LPT_KMAX; k++)
            if (tid + k * nt >= T) wt[k] = 0u;
    } else {
#pragma unroll
        for (int k = 0; k < LPT_KMAX; k++) wt[k] = 0u;
    }
#pragma unroll
    for (int k = 0; k < LPT_KMAX; k++) mx = max(mx, wt[k]);
    if (!cached)
        for (int t = tid; t < T; t += nt) mx = max(mx, load_w(t));
    for (int k = tid; k < 256; k += nt) hist[k] = 0;
    mx = wave_max_u32(mx);
    if (lane == 0) hist[256 + w] = mx;
    __syncthreads();
    uint32_t m = 0;
    for (int i = 0; i < (nt >> 6); i++) m = max(m, hist[256 + i]);
    const int bits = m ? 32 - __builtin_clz(m) : 0;
    const uint32_t shift = (uint32_t)max(shift0, min(9, bits - 8));
    lpt_walk(T, cached, wt, load_w, shift, hist, nullptr);
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the 256 buckets by one wave, 4 per lane
        const uint32_t a = hist[4 * tid], b = hist[4 * tid + 1], c = hist[4 * tid + 2], d = hist[4 * tid + 3];
        const uint32_t sum = a + b + c + d;
        const uint32_t excl = wave_inclusive_scan(sum, tid) - sum;
        hist[4 * tid] = excl;
        hist[4 * tid + 1] = excl + a;
        hist[4 * tid + 2] = excl + a + b;
        hist[4 * tid + 3] = excl + a + b + c;
    }
    __syncthreads();
    lpt_walk(T, cached, wt, load_w, shift, hist, order);
    if (!xmap) return;
    // per-XCD orders: the same buckets per XCD group, x-major; group x's tiles take its slots in bucket order
    uint32_t *xstart = xhist + LPT_BCNT_WORDS;  // LPT_XCD + 1 segment starts
    uint32_t *wsum = xstart + LPT_XCD + 1;      // per-wave sums of the scan (<= 16 waves)
    for (int k = tid; k < (int)LPT_BCNT_WORDS; k += nt) xhist[k] = 0;
    __syncthreads();
    auto xbucket = [&](int t, uint32_t wgt) -> uint32_t {
        return 256u * xcd_group_of((uint32_t)t, (uint32_t)gx, (uint32_t)gy) + (255u - min(255u, wgt >> shift));
    };
    // fn(t, bucket) over the tiles, the weights from registers when cached (a static index: no scratch)
    auto each_tile = [&](auto fn) {
        if (cached) {
#pragma unroll
            for (int k = 0; k < LPT_KMAX; k++) {
                if (k * nt >= T) break;  // uniform
                const int t = tid + k * nt;
                if (t < T) fn(t, xbucket(t, wt[k]));
            }
        } else {
            for (int t = tid; t < T; t += nt) fn(t, xbucket(t, load_w(t)));
        }
    };
    each_tile([&](int, uint32_t bb) { atomicAdd(&xhist[bb], 1u); });
    __syncthreads();
    // exclusive scan of the LPT_BCNT_WORDS counts, 2 per thread (the caller runs 1024 threads)
    constexpr int XPER = (int)LPT_BCNT_WORDS / 1024;
    uint32_t v[XPER], loc = 0;
#pragma unroll
    for (int j = 0; j < XPER; j++) {
        v[j] = tid < 1024 ? xhist[tid * XPER + j] : 0u;
        loc += v[j];
    }
    const uint32_t inc = wave_inclusive_scan(loc, lane);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t run = inc - loc;
    for (int i = 0; i < w; i++) run += wsum[i];
    __syncthreads();
    if (tid < 1024) {
#pragma unroll
        for (int j = 0; j < XPER; j++) {
            const int idx = tid * XPER + j;
            xhist[idx] = run;
            if (idx % 256 == 0) xstart[idx / 256] = run;
            run += v[j];
        }
        if (tid == 1023) xstart[LPT_XCD] = run;
    }
    __syncthreads();
    const uint32_t cap = xcd_slots((uint32_t)T) / LPT_XCD;
    for (uint32_t i = (uint32_t)tid; i < LPT_XCD * cap; i += (uint32_t)nt) {  // the slots no tile takes
        const uint32_t x = i / cap, q = i % cap;
        if (q >= xstart[x + 1] - xstart[x]) xmap[xcd_slot(x, q, (uint32_t)per)] = XCD_NONE;
    }
    each_tile([&](int t, uint32_t bb) {
        const uint32_t x = bb / 256u, q = atomicAdd(&xhist[bb], 1u) - xstart[x];
        xmap[xcd_slot(x, q, (uint32_t)per)] = (uint32_t)t;
    });
}

#endif  // __HIPCC__

}  // namespace gsr
