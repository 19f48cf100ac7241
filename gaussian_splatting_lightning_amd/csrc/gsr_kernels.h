// gsr_kernels.h -- host-side launchers of the HIP kernels (defined in gsr_*.hip).
#pragma once

#include "gsr_common.h"

namespace gsr {

// Internal tuning knobs (A/B experiments in one process; defaults are the shipped configuration).
int tuning(const char *name, int default_value);
// Diagnostics: per-wave (start, end, HW_ID, XCC_ID) stamps of the composite kernels, one uint4 per launch
// slot, written only when the "stamp" knob is set (buffer 0: render_fwd, 1: render_bwd; 2: the last onesweep
// sort pass, per block (start, ranked, looked back, end); 3: the multi-histogram, per block (start, loop done,
// end, 0)).
uint4 *stamp_buffer(int which);

// ---- scan / sort (gsr_sort.hip) ----
// Exclusive scan of n u32 values (optionally gathered through idx: v[i] = in[idx[i]]).
// out has n+1 entries; out[n] = total.  overflow_flag (device u32) is set if the total exceeds 2^32-1.
// Same result in one launch (decoupled look-back); status (div_up(n + 1, SCAN_TILE) words) and *ticket zeroed.
void launch_exclusive_scan_lookback(hipStream_t s, const uint32_t *in, const uint32_t *idx, uint32_t n, uint32_t *out,
                                    uint64_t *status, uint32_t *ticket, uint32_t *overflow_flag);

// LSD radix sort of n (key, value) pairs on bits [0, nbits).  Keys start in sc.k[0]; values are the
// implicit iota 0..n-1.  After ceil(nbits/8) passes the keys are in sc.k[passes & 1] and the values in
// sc.v[passes & 1].
// LSD radix sort of sc.k[0] (nbits significant bits); values are the iota permutation unless `keyed`, in which
// case sc.v[0] holds the input values.  The result lands in buffer index (passes & 1).
// keys0 (optional): read the first pass's keys from there instead of sc.k[0] (left unmodified).
// gather (optional): the last pass also writes dst[i] = src[sorted value i] for each non-null pair; returns
// whether it did (always, with a gather).
// onesweep_ran (optional): set to whether the onesweep path ran, i.e. whether sc.ctrl[RS_CTRL_ERR] was cleared and
// holds this sort's look-back error flag (the multi-kernel path never touches sc.ctrl).
struct SortGather {
    const uint32_t *src = nullptr;
    uint32_t *dst = nullptr;
    const uint4 *src4 = nullptr;
    uint4 *dst4 = nullptr;
};
bool launch_radix_sort(hipStream_t s, SortScratch &sc, uint32_t n, int nbits, bool keyed = false,
                       const uint32_t *keys0 = nullptr, const SortGather *gather = nullptr,
                       bool *onesweep_ran = nullptr);
// relative-key depth sort (multi-kernel path, up to 9-bit digits): see gsr_sort.hip
void launch_depth_sort_rel(hipStream_t s, SortScratch &sc, uint32_t n, const uint32_t *keys0, uint32_t kbase,
                           uint32_t kcap, int bits, const SortGather *gather);
// The same sort on 16-bit keys in `passes` digits of digit_bits bits (multi-kernel passes): sc.k[] hold uint16_t keys,
// values as above.  The radix binning's tile sort takes it up to 65536 tiles (tile_sort_plan).
void launch_radix_sort16(hipStream_t s, SortScratch &sc, uint32_t n, int digit_bits, int passes, int bits);  // bits: key bits in use

// ---- forward (gsr_forward.hip) ----
struct PreprocessParams {
    int P, D, M, W, H, gx, gy;
    float tan_fovx, tan_fovy, focal_x, focal_y, scale_modifier;
    int antialiasing;
    int cull;  // exact tile culling (see tile_has_contribution)
    const float *means3D, *opacities, *scales, *rotations, *cov3D_precomp, *colors_precomp, *shs;
    const float *view, *proj, *campos;
    int *radii;
    GeomState g;
    uint32_t *block_sums;  // optional: kept-tile total of every 256-Gaussian block
    // optional: pinned host words; the last preprocess workgroup writes {instance total lo, hi, big count, seq}
    // to host_words[CNT_WORDS .. +4) in one 16-B store (the forward's readback without a copy or an event)
    uint32_t *host_words;
    uint32_t seq;
    int depth_range = 0;  // publish the kept depth keys' range with the instance total (relative depth sort)
    uint4 *stamps = nullptr;  // diagnostics ("stamp" knob): per wave {start, projected, culled, end}, {HW_ID, XCC_ID}
};
void launch_preprocess(hipStream_t s, const PreprocessParams &p);
void launch_zero16(hipStream_t s, void *p, size_t bytes);  // bytes: a multiple of 16, p 16-B aligned

struct ExpandParams {
    uint32_t P, R;
    int gx, gy;
    const uint32_t *order, *inst_off, *tiles;
    const uint4 *exp_rec;
    const uint4 *exp_sorted;  // optional: exp_rec already in depth order (read by rank, no gather)
    uint32_t *exp_owner;      // owner ranks of the block starts (div_up(R, EXP_TILE) + 1 words)
    uint32_t *keys_out, *inst_gid, *inst_start;
    uint16_t *keys16_out;     // optional: 16-bit tile keys (launch_radix_sort16) instead of keys_out
    uint32_t *inv_none;       // optional: inv, set to INV_NONE for every instance here (no separate fill)
};
void launch_expand(hipStream_t s, const ExpandParams &p);

void launch_identify_ranges(hipStream_t s, const uint32_t *keys_sorted, uint32_t R, uint2 *ranges);
void launch_identify_ranges16(hipStream_t s, const uint16_t *keys_sorted, uint32_t R, uint2 *ranges);

// ---- bucket binning (gsr_bin.hip) ----
struct BucketParams {
    uint32_t P, T, nb, gper;  // Gaussians, tiles, walk blocks launched, Gaussians per block
    // walk blocks owning a Gaussian range (nr <= nb).  Blocks nr.. only walk big rects: bk_walk_blocks() is the count
    // the passes use, nr raised to min(nb, big-Gaussian count); the blocks above it exit and their rows are not read
    uint32_t nr;
    uint32_t R;               // instances (scatter; the region partition's grid)
    const uint32_t *nbig;     // big-Gaussian count (device word written by the preprocess)
    int gx;
    const uint32_t *tiles, *depth_key, *big_list;
    const uint32_t *block_sums;  // preprocess block totals (256 Gaussians each)
    uint32_t *inst_start;  // P + 1: written by the count pass (Gaussian-order exclusive scan of tiles)
    const uint4 *exp_rec;
    uint32_t *hist;        // nb x T counts (the count pass writes them; read-only for the column pass)
    uint32_t *hist_pre;    // nb x T column prefixes (column pass), seeding the scatter's bucket slots
    uint32_t *tile_next;   // T: the tiles' starts (column pass), then the region partition's next free slots (atomics)
    uint32_t *tile_start;  // T + 1
    uint2 *ranges;         // T
    uint32_t *long_list;   // 2 x (T + 1): tiles of (SEG_CAP, SEG_BLOCK_CAP] instances, longer tiles
    uint32_t *long_cnt;    // 2 counts (zeroed)
    uint32_t *ticket;      // zeroed: column-pass workgroup ticket
    uint64_t *tile_status; // zeroed: div_up(T, 32) look-back words of the column pass
    uint32_t *err;         // look-back flags (bit 2: a decoupled fallback ran; diagnostic)
    uint32_t lb_patience;  // look-back polls before recomputing an unpublished predecessor
    int lb_force;          // recompute every predecessor (tests the fallback)
    uint32_t *tile_last, *tile_loaded;  // T each: cleared by the column pass for the forward composite
    uint32_t *inv;         // R: reset to INV_NONE beside inst_gid (the forward composite fills it)
    uint32_t *lpt_bcnt;    // 256: cleared by the column pass (the forward's backward-LPT bucket counts)
    unsigned long long *keys;  // R: depth << 32 | u, bucketed by tile
    // region scatter (keys_reg != null; R <= 2^28): the scatter writes each key into its tile's REGION (BK_REGION
    // consecutive tile ids) with the tile's index in the region in bits 28-31 of u (BK_REG_SHIFT), and
    // bk_partition_kernel then moves the keys of each region into their tile buckets (keys), without those bits
    unsigned long long *keys_reg;  // R, or null
    uint32_t *reg_start;           // T / BK_REGION + 2: region starts (tile_start of each region's first tile), column pass
    uint32_t *inst_gid;    // R
    uint32_t *order;       // scatter: an extra workgroup writes the forward LPT order here (or null: none)
    uint32_t *order_xcd;   // and, when set, the per-XCD LPT slot map of the forward composite (xcd_slots(T) words)
    int lpt_shift;
    int xcd_major;         // bucket runs in XCD-major block order (bk_row_block)
};
void launch_bucket_count(hipStream_t s, const BucketParams &p);    // walk + column prefixes + tile ranges
void launch_bucket_scatter(hipStream_t s, const BucketParams &p);

struct SegSortParams {
    uint32_t T;
    const uint2 *ranges;
    const uint32_t *tile_order;  // or null
    unsigned long long *keys;   // R bucketed keys
    unsigned long long *keys2;  // R: chunk-sorted keys of the tiles longer than SEG_BLOCK_CAP
    uint32_t *sorted_u;
    const uint32_t *long_list, *long_cnt;
    uint4 *stamps;  // diagnostics (set by launch): per long-tile slot (start, chunks sorted, end, n), or null
};
void launch_seg_sort(hipStream_t s, const SegSortParams &p);

// Tiles ordered by descending work (range length, or tile_last when use_last) for an LPT launch order.
void launch_tile_order(hipStream_t s, const uint2 *ranges, const uint32_t *tile_last, int use_last, int T,
                       uint32_t *order, uint32_t *scratch = nullptr);  // scratch: ImageState::lpt_hist

struct RenderFwdParams {
    int W, H, gx, gy, num_tiles;
    int xcd;  // tile_order is the per-XCD slot map (order_xcd, XCD_NONE = no tile) and the appends go to the XCD lists
    const uint2 *ranges;
    const uint32_t *tile_order;  // launch slot -> tile (heaviest first), or null for identity
    const uint32_t *sorted_u, *inst_gid;
    uint32_t *point_list, *tile_loaded;
    uint32_t *inv;                        // R: inv[u] = sorted position of every instance the walk loads
    const GRec *rec;
    const float *bg;
    float *out_color, *out_invdepth, *final_T;
    uint32_t *n_contrib, *tile_last;
    uint4 *stamps; // diagnostics (set by launch), or null
    int strip_exact;  // strip skipping mask: 1 strip_mask_exact (column-band extent), 0 strip_mask (set by launch)
    // segmented-backward checkpoints (BinningState::ckpt, ImageState::ctot / ck_flag), or null: written every ck_k
    // instances when the launch runs tiles in 4 parts; *ck_flag = ck_k if it did, else 0
    float *ckpt = nullptr, *ctot = nullptr;
    uint32_t *ck_flag = nullptr;
    uint32_t ck_k = 0;
    // backward LPT bucket lists (ImageState::lpt_*), or null: whole-tile waves append their tile; *lpt_valid = 1 if
    // every tile was appended (whole tiles and lists given), else 0
    uint32_t *lpt_bcnt = nullptr, *lpt_blist = nullptr, *lpt_valid = nullptr;
    // exact per-instance strip masks for the backward (BinningState::strip_mask), or null: whole-tile waves record
    // which strips took each loaded instance; *smask_valid = 1 if this launch wrote them, else 0
    uint8_t *strip_mask = nullptr;
    uint32_t *smask_valid = nullptr;
};
void launch_render_fwd(hipStream_t s, const RenderFwdParams &p);
int render_fwd_parts(int num_tiles);  // row-strip parts per tile launch_render_fwd uses (1: whole tiles)

void launch_mark_visible(hipStream_t s, int P, const float *means3D, const float *view, uint8_t *present);

// ---- backward (gsr_backward.hip) ----
struct RenderBwdParams {
    int W, H, gx, gy, num_tiles;
    const uint2 *ranges;
    const uint32_t *tile_order;  // launch slot -> tile (heaviest first), or null for identity
    const uint32_t *point_list, *n_contrib, *tile_last, *tile_loaded;
    const uint32_t *sorted_u;  // sorted position -> expansion index u: an instance's gradient row is row u
    const GRec *rec;
    const float *bg, *final_T, *dL_dpix, *dL_dinvdepth;
    float *rows;    // R x GRAD_ROW
    uint8_t *live;  // P: set to 1 for the Gaussian of every non-zero row stored (GeomState::live), or null
    uint32_t *live_valid;  // 1 when this composite marked the live flags, 0 when it did not (read by preprocess_bwd)
    uint4 *stamps;  // diagnostics (set by launch), or null
    int strip_exact;  // as RenderFwdParams::strip_exact (set by launch)
    uint64_t num_rendered = 0;  // instances (the launch's walk-variant choice)
    // segmented walk (small images): the forward's checkpoints, or null for one wave (or workgroup) per tile
    const float *ckpt = nullptr, *ctot = nullptr;
    const uint32_t *ck_flag = nullptr;
    uint2 *seg_list = nullptr;
    uint32_t *seg_count = nullptr;
    uint32_t ck_k = 0;
    // launch order from the forward's LPT bucket lists when *lpt_valid (else tile_order / identity)
    const uint32_t *lpt_bcnt = nullptr, *lpt_blist = nullptr, *lpt_valid = nullptr;
    // the forward's exact strip masks when *smask_valid (else the conservative cell_mask of the record)
    const uint8_t *strip_mask = nullptr;
    const uint32_t *smask_valid = nullptr;
    // Zero fill of the per-Gaussian backward outputs, spread over the composite's workgroups (bwd_zero_fill): the
    // 16-B aligned interior of each output as segments of one virtual array of zf_total16 uint4, their unaligned
    // head / tail words listed one by one.  preprocess_bwd then stores only the Gaussians with a non-zero gradient.
    static constexpr int ZF_SEGS = 10, ZF_ODD = 60;
    uint32_t zf_nseg = 0, zf_nodd = 0;
    uint64_t zf_total16 = 0;
    uint4 *zf_ptr[ZF_SEGS] = {};
    uint64_t zf_pre16[ZF_SEGS + 1] = {};  // prefix sums of the segments' lengths
    uint32_t *zf_odd[ZF_ODD] = {};
};
void launch_render_bwd(hipStream_t s, const RenderBwdParams &p);

struct BigReduceParams {
    const uint32_t *big_list, *inst_start, *tiles;
    const uint32_t *inv;  // the forward's inverse permutation: INV_NONE where the composite loaded no instance (no row)
    const float *rows;
    float *bigsum;  // nbig x GRAD_ROW
    const uint32_t *nbig_dev;  // or null: the launch's nbig is exact; else an upper bound and this the count
};
void launch_big_reduce(hipStream_t s, const BigReduceParams &p, uint32_t nbig);

struct PreprocessBwdParams {
    int P, D, M, W, H;
    int g0, g1;  // Gaussians [g0, g1) (the whole [0, P) unless the backward is split into chunks); every output pointer
                 // is indexed by the absolute Gaussian index (the API pre-offsets chunk-relative ones)
    float tan_fovx, tan_fovy, focal_x, focal_y, scale_modifier;
    int antialiasing, has_invdepth;
    int sh_vec16;  // M == 16 and shs / dL_dsh 16-byte aligned: vectorised SH path
    const float *means3D, *opacities, *scales, *rotations, *cov3D_precomp, *shs;
    const float *view, *proj, *campos;
    const int *radii;
    const uint32_t *tiles, *inst_start, *big_slot;
    const uint32_t *inv;  // the forward's inverse permutation: INV_NONE where the composite loaded no instance (no row)
    const uint8_t *clamped;
    const uint8_t *live;  // P: 0 = no non-zero row (the gather is skipped: zero sums), or null = gather every Gaussian
    const uint32_t *live_valid;  // the flags are used only when the last composite marked them
    const float *sh_jac;  // 9 x P direction Jacobian of the colour, from the forward (SH degree > 0)
    const float *rows, *bigsum;
    float *dL_dmeans2D, *dL_dcolors, *dL_dopacity, *dL_dmeans3D, *dL_dcov3D, *dL_dsh, *dL_dscales, *dL_drot;
    float *dL_dcolors_sh;  // clamp-masked colour gradient (may be null)
    float *densify_stats;  // (P,2) |dL/dmeans2D[:2]|, radii > 0 (may be null)
    int densify_accumulate;  // densify_stats += instead of =
    int *max_radii2D;        // (P) max(max_radii2D, radii) (may be null)
    float *campos_rows;      // (campos_nrows, 3): campos in row campos_rank, zeros elsewhere (may be null)
    int campos_rank, campos_nrows;
    int prezeroed = 0;       // the outputs were zero-filled (RenderBwdParams::zf_*): store only non-zero gradients
};
void launch_preprocess_bwd(hipStream_t s, const PreprocessBwdParams &p);

// ---- multi-view SH gradient (gsr_views.hip) ----
void launch_sh_backward_views(hipStream_t s, int P, int D, int M, int V, int chunk_len, const float *means3D,
                              const float *campos, const float *dcolors_sh, float *dsh);

// One Adam element update (torch's Adam, non-amsgrad, no weight decay), shared by adam_kernel and the fused SH
// Adam so the two give the same bits: the contractions are explicit (the compiler's choice of FMA could differ between
// the kernels otherwise):
//     m = lerp(m, g, 1 - b1);  v = v b2 + (1 - b2) g^2;  p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps)
__device__ __forceinline__ void adam_update(float &p, float g, float &m, float &v, float b1c, float b2, float b2c,
                                            float step_size, float bc2_sqrt, float eps) {
#pragma clang fp contract(off)
    m = __fmaf_rn(b1c, __fsub_rn(g, m), m);                // exp_avg.lerp_(grad, 1 - beta1)
    v = __fmaf_rn(v, b2, __fmul_rn(b2c, __fmul_rn(g, g)));  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
    const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), bc2_sqrt), eps);
    p = __fmaf_rn(-step_size, __fdiv_rn(m, denom), p);     // param.addcdiv_(exp_avg, denom, value=-step_size)
}

// fused Adam of the SH groups on the multi-view expansion (gsr_views.hip; M = 16)
struct AdamShGroup {
    float *param, *exp_avg, *exp_avg_sq;
    float step_size, bc2_sqrt;
    int64_t param_stride;  // floats between the parameter's rows: 3 / 45 (own tensors) or 48 (one (P, 16, 3) tensor)
};
struct AdamShLaunch {
    int P, V, L;
    const float *means3D, *campos, *dc;
    AdamShGroup dc_group, rest_group;
    float one_minus_beta1, beta2, one_minus_beta2, eps;
    int vec4;
    int joint;  // parameter and moments each one 16-B aligned (P, 16, 3) tensor (dc_group's pointers: its base)
};
void launch_adam_sh_views(hipStream_t s, const AdamShLaunch &L, int D);

// ---- fused Adam (gsr_adam.hip) ----
constexpr int ADAM_MAX_GROUPS = 16;
struct AdamGroupDev {
    float *param;
    const float *grad;
    float *exp_avg, *exp_avg_sq;
    int64_t n;
    float step_size, bc2_sqrt;
    int vec4;
    int64_t M;   // sparse step: elements per Gaussian (element e belongs to Gaussian e / M)
    float lr;    // sparse step: the group's learning rate (no bias correction)
};
struct AdamLaunch {
    AdamGroupDev g[ADAM_MAX_GROUPS];
    int64_t slice_start[ADAM_MAX_GROUPS];
    int num_groups;
    float one_minus_beta1, beta2, one_minus_beta2, eps;
    float beta1;                 // sparse step
    const uint8_t *visible;      // sparse step: N bytes, nonzero = the Gaussian was rendered this step
};
int64_t adam_slices(int64_t n);
void launch_adam(hipStream_t s, const AdamLaunch &L, int64_t total_slices);
void launch_sparse_adam(hipStream_t s, const AdamLaunch &L, int64_t total_slices);

// ---- parameter activations (gsr_adam.hip) ----
struct ActivationArgs {
    int64_t N;
    const float *scaling, *opacity, *rotation;        // raw parameters (N,3) (N) (N,4)
    float *scales, *opacities, *rotations;            // forward outputs / backward inputs (activated)
    const float *dL_dscales, *dL_dopacities, *dL_drotations;
    float *dL_dscaling, *dL_dopacity, *dL_drotation;  // backward outputs
};
void launch_activations_forward(hipStream_t s, const ActivationArgs &A);
void launch_activations_backward(hipStream_t s, const ActivationArgs &A);

// ---- densify_and_prune (gsr_densify.hip) ----
struct DensifyParams {
    int64_t N;
    const float *opacity, *scaling, *max_radii2D, *grad_accum, *grad_count;
    float opacity_threshold, screensize_threshold, size_threshold, grad_threshold, clone_size_threshold;
    int apply_screensize, apply_size;
    uint8_t *row_class;      // (N)
    int32_t *block_counts;   // (3 * blocks)
    int32_t *counts;         // (3): kept, cloned, split
    int32_t *dst_map;        // (2N): kept row destination | appended copy destination (-1 = none)
    int32_t *split_rank;     // (N)
    int64_t *preserve_idx;   // (N): first counts[0] entries valid
};
constexpr int DENSIFY_MAX_FIELDS = 16;
struct DensifyFieldDev {
    const float *src, *src_exp_avg, *src_exp_avg_sq;
    float *dst, *dst_exp_avg, *dst_exp_avg_sq;
    int width, kind;
};
struct DensifyApply {
    DensifyFieldDev f[DENSIFY_MAX_FIELDS];
    int64_t block_start[DENSIFY_MAX_FIELDS];
    int num_fields;
    int64_t N;
    const int32_t *dst_map, *split_rank;
    const float *z, *rotation, *scaling;
};
int64_t densify_blocks(int64_t N);
void launch_densify_classify(hipStream_t s, const DensifyParams &p);
void launch_densify_apply(hipStream_t s, const DensifyApply &A, int64_t total_blocks);

// ---- PLY records <-> fields (gsr_ply.hip) ----
constexpr int PLY_MAX_COLS = 128, PLY_MAX_FIELDS = 8;
struct PlyLaunch {
    const uint8_t *records;   // unpack source
    uint8_t *records_out;     // pack destination
    int64_t n;
    int record_bytes, rows_per_block, ncols, nfields, swap;
    float *field[PLY_MAX_FIELDS];
    int width[PLY_MAX_FIELDS];
    int2 cols[PLY_MAX_COLS];  // (byte offset in the record, GSR_PLY_* type), destination order
};
int ply_rows_per_block(int record_bytes);
void launch_ply(hipStream_t s, const PlyLaunch &p, bool pack);

// ---- exact 3-NN mean squared distance (gsr_knn.hip) ----
struct KnnScratch {
    void *base;
    SortScratch sort;
    uint64_t *codes, *scode;
    float4 *spts;
    float *partial, *box;
};
size_t knn_workspace(int64_t n, KnnScratch *k);  // k == nullptr: size only; else carve from k->base
void launch_knn(hipStream_t s, KnnScratch &k, const float *pts, int64_t n, float *out);

// ---- fused SSIM loss (gsr_ssim.hip) ----
size_t ssim_num_partials(int planes, int H, int W);
void launch_ssim_forward(hipStream_t s, int planes, int H, int W, const float *img1, const float *img2, int valid,
                         float *partial, float *d_mu1, float *d_s11, float *d_s12);
void launch_ssim_backward(hipStream_t s, int planes, int H, int W, const float *img1, const float *img2, int valid,
                          const float *dL_dmean, float inv_n, const float *d_mu1, const float *d_s11,
                          const float *d_s12, float *dL_dimg1);

}  // namespace gsr
