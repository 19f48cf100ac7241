/*
 * gsrast.h -- C ABI of the MI355X-native differentiable Gaussian rasterizer.
 *
 * This is the drop-in boundary for the hot path that pomelyu/gaussian_splatting_lightning reaches
 * through `diff_gaussian_rasterization` (reference call sites:
 *   gs_lightning/lightning/gs_lightning_module.py:322-348   GaussianRasterizationSettings + GaussianRasterizer
 *   scripts/render_trained_image.py:98-124                  inference call, means2D=None
 *   tests/rasterizer_python/test_mark_visible.py:13-14      GaussianRasterizer(s).markVisible(points)).
 * The submodule that normally implements it (graphdeco-inria/diff-gaussian-rasterization@dr_aa,
 * .gitmodules:1-4) is not vendored; each entry point below replaces one of its pybind exports
 * (`_C.rasterize_gaussians`, `_C.rasterize_gaussians_backward`, `_C.mark_visible`, SURVEY.md §2.1 and
 * §8(b)).  Signatures are plain C: device pointers, sizes and a hipStream_t passed as void*.  No torch
 * types cross this boundary; the Python host layer (gaussian_splatting_lightning_amd/rasterizer.py)
 * binds it with ctypes.
 *
 * Conventions (identical to the reference's torch API):
 *   means3D (P,3), opacities (P,1), scales (P,3), rotations (P,4) as (w,x,y,z), shs (P,M,3),
 *   colors_precomp (P,3), cov3D_precomp (P,6) upper triangle, viewmatrix / projmatrix (4,4) row-major
 *   in the row-vector convention (p_view = [p,1] @ V), campos (3), background (3);
 *   out_color (3,H,W), out_invdepth (1,H,W), radii (P) int32.
 * All pointers are DEVICE pointers (fp32, contiguous) unless stated; every launch goes on `stream`.
 * Return value: 0 on success, nonzero error code; gsr_last_error() gives the message.
 */
#ifndef GSRAST_H
#define GSRAST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Scratch buffers are owned by the caller and grown through this callback, mirroring the
 * reference's resizeFunctional() lambdas over uint8 torch tensors (notes/rasterizer_note.h:27-40).
 * `which` is one of GSR_BUF_*; the callback returns a device pointer to >= nbytes bytes that stays
 * valid until the caller frees it (the forward's three buffers must survive until the backward). */
typedef char *(*gsr_alloc_fn)(void *ctx, int which, size_t nbytes);

enum { GSR_BUF_GEOM = 0, GSR_BUF_BINNING = 1, GSR_BUF_IMAGE = 2, GSR_BUF_BWD_SCRATCH = 3 };

enum {
    GSR_OK = 0,
    GSR_ERR_ARG = 1,      /* invalid shape/pointer/option (RuntimeError in Python) */
    GSR_ERR_HIP = 2,      /* HIP runtime error */
    GSR_ERR_ALLOC = 3,    /* allocation callback returned NULL */
    GSR_ERR_OVERFLOW = 4, /* more than 2^32-1 tile instances */
    GSR_ERR_UNSUPPORTED = 5
};

typedef struct gsr_forward_args {
    int P;                        /* number of Gaussians */
    int D;                        /* active SH degree (0..3) */
    int M;                        /* SH coefficients stored per Gaussian (shs.size(1)), 0 if none */
    int W, H;                     /* image size */
    const float *background;      /* (3) */
    const float *means3D;         /* (P,3) */
    const float *colors_precomp;  /* (P,3) or NULL (then shs is required) */
    const float *opacities;       /* (P) */
    const float *scales;          /* (P,3) or NULL (then cov3D_precomp is required) */
    float scale_modifier;
    const float *rotations;       /* (P,4) or NULL */
    const float *cov3D_precomp;   /* (P,6) or NULL */
    const float *viewmatrix;      /* (16) */
    const float *projmatrix;      /* (16) */
    const float *campos;          /* (3) */
    float tan_fovx, tan_fovy;
    const float *shs;             /* (P,M,3) or NULL */
    int prefiltered;              /* accepted; the frustum test is applied either way */
    int antialiasing;             /* EWA 2D filter opacity compensation (dr_aa) */
    int debug;                    /* synchronise + check after every stage */
    float *out_color;             /* (3,H,W) */
    float *out_invdepth;          /* (H,W) or NULL */
    int *radii;                   /* (P) */
    int64_t num_big_out;          /* OUTPUT: Gaussians with > 64 instances (pass to gsr_backward) */
} gsr_forward_args;

/* Replaces `_C.rasterize_gaussians` (rasterize_points.cu RasterizeGaussiansCUDA -> Rasterizer::forward).
 * Runs preprocess, depth sort, scan, one device->host read of the instance count, tile expansion,
 * tile sort, range identification and compositing.  *num_rendered receives the instance count. */
int gsr_forward(gsr_forward_args *args, gsr_alloc_fn alloc, void *alloc_ctx, void *stream,
                int64_t *num_rendered);

typedef struct gsr_backward_args {
    int P, D, M, W, H;
    int64_t R;                    /* num_rendered returned by gsr_forward */
    int64_t num_big;              /* num_big_out returned by gsr_forward, or < 0: read from geom_buffer on the device
                                     (the upstream backward signature does not carry it; gsr_torch_ext.cpp) */
    const float *background;
    const float *means3D;
    const float *colors_precomp;  /* or NULL */
    const float *opacities;
    const float *scales;          /* or NULL */
    float scale_modifier;
    const float *rotations;       /* or NULL */
    const float *cov3D_precomp;   /* or NULL */
    const float *viewmatrix, *projmatrix, *campos;
    float tan_fovx, tan_fovy;
    const float *dL_dpix;         /* (3,H,W) */
    const float *dL_dinvdepth;    /* (H,W) or NULL */
    const float *shs;             /* or NULL */
    const int *radii;             /* (P) from the forward */
    char *geom_buffer, *binning_buffer, *image_buffer; /* from the forward */
    int antialiasing, debug;
    /* outputs, each fully written (no pre-zeroing needed); any may be NULL to skip it */
    float *dL_dmeans2D;           /* (P,3), z = 0, NDC units (pixel grad * (W/2, H/2)) */
    float *dL_dcolors;            /* (P,3) */
    float *dL_dopacity;           /* (P) */
    float *dL_dmeans3D;           /* (P,3) */
    float *dL_dcov3D;             /* (P,6) */
    float *dL_dsh;                /* (P,M,3); may be NULL only when dL_dcolors_sh is given */
    float *dL_dscales;            /* (P,3) */
    float *dL_drotations;         /* (P,4) */
    /* (P,3) colour gradient with computeColorFromSH's clamp mask applied, i.e. the factor that multiplies
     * the SH basis in dL/dsh.  With dL_dsh == NULL this is the compact per-view SH gradient that
     * gsr_sh_backward_views expands (multi-view data parallelism); NULL to skip. */
    float *dL_dcolors_sh;
    /* (P,2) densification statistics of this view (gaussian_model.py:175-181): [i][0] = |dL/dmeans2D[i][:2]|,
     * [i][1] = 1 if radii[i] > 0 else 0; NULL to skip. */
    float *densify_stats;
    /* densify_accumulate != 0: densify_stats += this view's statistics instead of =, i.e. the reference's
     * add_densification_stats (xyz_gradient_accum += norm, denom += 1 for visible Gaussians) across views and
     * steps; max_radii2D (P) int32, if non-NULL, becomes max(max_radii2D, radii) (gaussian_model.py:175-176). */
    int densify_accumulate;
    int *max_radii2D;
    /* Split backward, so a gradient exchange can overlap the per-Gaussian stage (multiview.py; no counterpart in
     * the reference, whose batch is one view):
     *   stages = GSR_BWD_ALL (0): everything in one call;
     *   GSR_BWD_COMPOSITE: the compositing backward and the big-Gaussian reduction only -- the per-instance gradient
     *     rows land in the GSR_BUF_BWD_SCRATCH buffer, which the caller keeps for the next calls; no output written;
     *   GSR_BWD_GAUSSIANS: the per-Gaussian stage only, over Gaussians [g_begin, g_end), reading the rows from
     *     bwd_scratch (the GSR_BWD_COMPOSITE call's buffer).  Every output pointer then addresses Gaussian
     *     g_begin's row (a slice of a full array, or a chunk-sized buffer).
     * g_begin = g_end = 0 means the whole range [0, P) (any stage). */
    int stages;
    int64_t g_begin, g_end;
    char *bwd_scratch;
    /* Camera block of the multi-view exchange (multiview.py), written by the per-Gaussian stage so that no extra
     * launch is needed: campos_rows (campos_nrows, 3) gets campos in row campos_rank and zeros in the others (a
     * SUM all-reduce of the block then yields every rank's camera).  NULL to skip. */
    float *campos_rows;
    int campos_rank, campos_nrows;
} gsr_backward_args;

enum { GSR_BWD_ALL = 0, GSR_BWD_COMPOSITE = 1, GSR_BWD_GAUSSIANS = 2 };

/* Replaces `_C.rasterize_gaussians_backward` (RasterizeGaussiansBackwardCUDA -> Rasterizer::backward).
 * Deterministic: per-tile gradient rows are reduced in fixed order (no float atomics). */
int gsr_backward(const gsr_backward_args *args, gsr_alloc_fn alloc, void *alloc_ctx, void *stream);

/* Multi-view SH gradient from compact per-view factors (no counterpart in the reference, whose batch size is
 * one view: gs_lightning_module.py:139-141).  dL_dsh[g] = sum_v basis(normalize(means3D[g] - campos[v]))
 * (x) dL_dcolors_sh[v][g], i.e. the sum over views of gsr_backward's dL_dsh -- what an all-reduce of dL_dsh
 * computes, from 12 B per Gaussian per view instead of 12*M B.  campos (V,3), dL_dcolors_sh (V,P,3),
 * dL_dsh (P,M,3) fully written (coefficients above the active degree are zero).  Device pointers. */
int gsr_sh_backward_views(int P, int D, int M, int V, const float *means3D, const float *campos,
                          const float *dL_dcolors_sh, float *dL_dsh, void *stream);

/* The same expansion over factors gathered per Gaussian chunk (multiview.py's chunked exchange), in ONE launch:
 * dL_dcolors_sh is chunk-major -- chunk c covers Gaussians [c*chunk_len, min(P, (c+1)*chunk_len)) and is a
 * (V, L_c, 3) block at offset c*V*chunk_len*3.  chunk_len = 0 (or >= P) is gsr_sh_backward_views' (V,P,3). */
int gsr_sh_backward_views_chunked(int P, int D, int M, int V, int64_t chunk_len, const float *means3D,
                                  const float *campos, const float *dL_dcolors_sh, float *dL_dsh, void *stream);

/* Replaces `_C.mark_visible` (checkFrustum): present[i] = z_view(means3D[i]) > 0.2. */
int gsr_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *present, void *stream);

/* Fused SSIM loss -- replaces `fused_ssim(img1, img2, padding, train)` (rahul-goel/fused-ssim, imported at
 * gs_lightning_module.py:10 and used as 1 - fused_ssim(render, gt) at :100,279).  Images are (B,C,H,W)
 * contiguous fp32 device arrays; planes = B*C.  11x11 Gaussian window (sigma 1.5), C1 = 0.01^2, C2 = 0.03^2,
 * zero-padded "same" filtering; valid_padding = 1 averages only pixels >= 5 px from the border.
 * Forward: writes gsr_ssim_num_partials() partial sums of the SSIM map (mean = sum / counted pixels) and, when
 * the three derivative maps (planes*H*W each) are non-NULL, the per-pixel derivatives the backward needs.
 * Backward: dL_dimg1 from dL_dmean (device scalar: gradient of the mean SSIM) and the derivative maps. */
size_t gsr_ssim_num_partials(int planes, int H, int W);
int gsr_ssim_forward(int planes, int H, int W, const float *img1, const float *img2, int valid_padding,
                     float *partial_sums, float *dm_dmu1, float *dm_dsigma1_sq, float *dm_dsigma12, void *stream);
int gsr_ssim_backward(int planes, int H, int W, const float *img1, const float *img2, int valid_padding,
                      const float *dL_dmean, const float *dm_dmu1, const float *dm_dsigma1_sq,
                      const float *dm_dsigma12, float *dL_dimg1, void *stream);

/* Fused Adam step over up to 16 parameter groups in one launch -- replaces the torch.optim.Adam(eps=1e-15)
 * step of the reference's six Gaussian parameter groups (gs_lightning_module.py:114-134).  All arrays are
 * contiguous fp32 device arrays of n elements, updated in place; step is the 1-based step count of each
 * group (torch keeps it per parameter).  No weight decay, no amsgrad, as configured by the reference. */
typedef struct gsr_adam_group {
    float *param;
    const float *grad;
    float *exp_avg, *exp_avg_sq;
    int64_t n;
    double lr;
    int64_t step;
} gsr_adam_group;
int gsr_adam_step(const gsr_adam_group *groups, int num_groups, double beta1, double beta2, double eps, void *stream);

/* Fused Adam step of the two SH parameter groups of a multi-view (one view per GPU) step, on the gradient that
 * gsr_sh_backward_views_chunked would expand -- sum_v basis(dir_v) (x) dL_dcolors_sh_v -- formed inside the update, so
 * the (P, M, 3) gradient is never written: features_dc (P, 1, 3) and features_rest (P, M - 1, 3) with their Adam
 * moments, updated in place with gsr_adam_step's arithmetic (each group with its own lr and 1-based step).  The
 * result is bitwise that of the expansion followed by gsr_adam_step.  M must be 16; V, chunk_len, means3D, campos and
 * dL_dcolors_sh as for gsr_sh_backward_views_chunked. */
typedef struct gsr_adam_sh_views_args {
    int P, D, M, V;
    int64_t chunk_len;
    const float *means3D, *campos, *dL_dcolors_sh;
    float *dc_param, *dc_exp_avg, *dc_exp_avg_sq;
    double dc_lr;
    int64_t dc_step;
    float *rest_param, *rest_exp_avg, *rest_exp_avg_sq;
    double rest_lr;
    int64_t rest_step;
    /* floats between consecutive Gaussians' rows of each parameter: 0 = packed ((P, 1, 3) / (P, M - 1, 3) tensors);
     * 48 = the two groups are the column blocks of ONE (P, 16, 3) tensor (dc_param = its base, rest_param = base + 3),
     * which the forward reads as shs without a concatenation.  The moments are always packed. */
    int64_t param_row_stride;
    /* the same for the moments: 0 = packed, 48 = exp_avg / exp_avg_sq are each one (P, 16, 3) tensor too (dc_* the
     * base, rest_* = base + 3).  With both at 48 every array is streamed as one coalesced run per 32 rows. */
    int64_t moment_row_stride;
} gsr_adam_sh_views_args;
int gsr_adam_sh_views_step(const gsr_adam_sh_views_args *a, double beta1, double beta2, double eps, void *stream);

/* The parameter activations the reference's GaussianModel puts in front of the rasterizer
 * (gs_lightning/modules/gaussian_model.py: get_scaling = exp(_scaling), get_opacity = sigmoid(_opacity),
 * get_rotation = torch.nn.functional.normalize(_rotation), i.e. q / max(|q|, 1e-12)) and their chain rule, so a
 * training step that keeps the raw parameters (what the optimizer steps) needs two launches instead of torch's
 * elementwise autograd graph.  Shapes: scaling / scales (N,3), opacity / opacities (N) or (N,1), rotation / rotations
 * (N,4); fp32 device arrays, the (N,4) ones 16-B aligned.  The backward takes the raw rotation and the forward's
 * outputs and writes dL/d(raw) from dL/d(activated). */
int gsr_activations_forward(int64_t N, const float *scaling, const float *opacity, const float *rotation,
                            float *scales, float *opacities, float *rotations, void *stream);
int gsr_activations_backward(int64_t N, const float *rotation, const float *scales, const float *opacities,
                             const float *rotations, const float *dL_dscales, const float *dL_dopacities,
                             const float *dL_drotations, float *dL_dscaling, float *dL_dopacity, float *dL_drotation,
                             void *stream);

/* SparseGaussianAdam.step(visibility, N) of the upstream rasterizer package (diff_gaussian_rasterization, taken by
 * the reference's third_party GaussianModel with optimizer_type "sparse_adam": gaussian_model.py:26,194-196).  Each
 * group's n elements are N Gaussians of n / N elements; only the Gaussians with visible[g] != 0 are updated, as
 * m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2, p += -lr m / (sqrt(v) + eps) -- no bias correction, `step` is
 * ignored.  visible: N bytes on the device (a torch bool tensor). */
int gsr_sparse_adam_step(const gsr_adam_group *groups, int num_groups, const uint8_t *visible, int64_t N,
                         double beta1, double beta2, double eps, void *stream);

/* densify_and_prune of gs_lightning/modules/gaussian_model.py:184-287 with the optimizer-state re-indexing of
 * gs_lightning_module.py:213-235, in two calls:
 *   gsr_densify_classify  classifies every row (prune / keep / clone / split) and builds the row maps;
 *                         counts[0..2] (device) = rows kept, rows cloned, rows split.  The caller reads the
 *                         counts back, allocates outputs of N_new = kept + cloned + split rows and draws
 *                         z ~ N(0, 1) of shape (split, 3);
 *   gsr_densify_apply     scatters every field (parameters, Adam moments, statistics) into the new arrays.
 * Thresholds are absolute (the reference's *_threshold * spatial_scale already applied). */
typedef struct gsr_densify_args {
    int64_t N;
    const float *opacity;       /* (N) raw (pre-sigmoid) */
    const float *scaling;       /* (N,3) raw (log) */
    const float *max_radii2D;   /* (N) */
    const float *xyz_grad_accum, *xyz_grad_count;  /* (N) */
    float opacity_threshold;    /* prune unless sigmoid(opacity) > threshold */
    float screensize_threshold; /* with apply_screensize: prune unless max_radii2D < threshold */
    float size_threshold;       /* with apply_size: prune unless max(exp(scaling)) < threshold */
    float grad_threshold;       /* clone/split if accum / count >= threshold */
    float clone_size_threshold; /* clone if max(exp(scaling)) < threshold, split otherwise */
    int apply_screensize, apply_size;
} gsr_densify_args;
size_t gsr_densify_workspace_bytes(int64_t N);
/* preserve_idx (N int64): the first counts[0] entries are the kept row indices (the reference's return value). */
int gsr_densify_classify(const gsr_densify_args *args, void *workspace, int32_t *counts, int64_t *preserve_idx,
                         void *stream);

enum { GSR_FIELD_PLAIN = 0, GSR_FIELD_XYZ = 1, GSR_FIELD_SCALING = 2, GSR_FIELD_STAT = 3 };
typedef struct gsr_densify_field {
    const float *src; /* (N, width) */
    float *dst;       /* (N_new, width) */
    const float *src_exp_avg, *src_exp_avg_sq; /* NULL when the parameter has no optimizer state */
    float *dst_exp_avg, *dst_exp_avg_sq;
    int width;
    int kind; /* XYZ: split rows move by R(q)(z*exp(scaling)); SCALING: log(exp(s)/1.6); STAT: zero on copies */
} gsr_densify_field;
/* rotation (N,4) raw quaternions (w,x,y,z), scaling (N,3) raw, z (split,3): the rows the split moves */
int gsr_densify_apply(int64_t N, const void *workspace, const float *rotation, const float *scaling, const float *z,
                      const gsr_densify_field *fields, int num_fields, void *stream);

/* PLY vertex records <-> parameter fields (the 3DGS checkpoint of gaussian_model.py:112-171 and
 * third_party/.../gaussian_model.py:239-314).  `records` are n fixed-size records of record_bytes each, on the
 * device; `columns` (host array, destination order: field after field, column after column) give each
 * column's byte offset in the record and its PLY type; fields are row-major (n, widths[f]) fp32 device
 * arrays.  unpack converts any scalar PLY type to fp32; pack writes float32 and zero-fills record bytes no
 * column covers (the normals of save_ply).  big_endian selects binary_big_endian records. */
enum { GSR_PLY_FLOAT32 = 0, GSR_PLY_FLOAT64 = 1, GSR_PLY_UINT8 = 2, GSR_PLY_INT8 = 3, GSR_PLY_UINT16 = 4,
       GSR_PLY_INT16 = 5, GSR_PLY_UINT32 = 6, GSR_PLY_INT32 = 7 };
typedef struct gsr_ply_column {
    int32_t offset;
    int32_t type;
} gsr_ply_column;
int gsr_ply_unpack(const uint8_t *records, int64_t n, int record_bytes, int big_endian, const gsr_ply_column *columns,
                   int num_columns, float *const *fields, const int *widths, int num_fields, void *stream);
int gsr_ply_pack(uint8_t *records, int64_t n, int record_bytes, int big_endian, const gsr_ply_column *columns,
                 int num_columns, const float *const *fields, const int *widths, int num_fields, void *stream);

/* Mean squared distance of every point to its 3 nearest other points -- distCUDA2 of
 * gs_lightning/utils/math.py:9-14 (scipy KDTree query k=4, self dropped), used for the scale initialisation
 * of gaussian_model.py:84-91.  Exact (Morton-ordered octree search); points (n,3) fp32, out (n) fp32. */
size_t gsr_knn_workspace_bytes(int64_t n);
int gsr_knn_mean_dist2(int64_t n, const float *points, float *out, void *workspace, void *stream);

/* Buffer sizes the forward will request (host-only arithmetic; for planning and tests). */
size_t gsr_geom_buffer_bytes(int P);
size_t gsr_binning_buffer_bytes(int64_t R, int W, int H);
size_t gsr_image_buffer_bytes(int W, int H);
size_t gsr_bwd_scratch_bytes(int64_t R, int64_t num_big);

/* Byte offsets of the internal arrays inside the three forward buffers (host arithmetic only).  Used by
 * the parity tests to compare the integer binning state (sorted instance list, tile ranges,
 * per-pixel contributor counts) bit for bit against the oracle. */
typedef struct gsr_state_layout {
    /* in: sizeof(gsr_state_layout) as the caller was built (a caller built against an older header passes its
     * smaller size and gets only the fields it knows); out: the size the library filled (from GSR_ABI_VERSION 2
     * on, fields are only ever appended).  0 is taken as the library's own size.  Version-1 callers (before this
     * field existed) are NOT compatible: see gsr_abi_version(). */
    size_t struct_size;
    size_t geom_rec_a, geom_rec_b, geom_rec_c; /* float4, float4, float2 of Gaussian 0's record; Gaussian i's at
                                                  + i * geom_rec_stride */
    size_t geom_tiles, geom_order, geom_inst_off, geom_inst_start, geom_clamped; /* u32, u32, u32, u32, u8 */
    size_t geom_depth_key;    /* u32 float bits of each Gaussian's view depth (0xffffffff: not rendered) */
    size_t geom_expand_rec;   /* uint4 {kept-tile mask lo, hi, rmin.x | rmin.y << 16, rect width} (mask 0 = all) */
    size_t bin_point_list, bin_inv, bin_keys_sorted;                  /* u32 per instance (bin_inv: sorted position of
                                                                         each instance the composite loaded, else
                                                                         0xffffffff: the backward's row markers) */
    size_t bin_sorted_u, bin_inst_gid;                                /* u32 per instance */
    size_t img_final_T, img_n_contrib, img_ranges, img_tile_last;     /* f32/u32 per pixel, uint2/u32 per tile */
    size_t img_tile_loaded;                                           /* u32 per tile */
    size_t geom_rec_stride;                                           /* bytes per render record (48) */
    size_t bin_bk_keys;       /* u64 per instance: the bucket binning's keys (depth bits << 32 | u) grouped by tile */
} gsr_state_layout;
void gsr_state_layout_query(int P, int64_t R, int W, int H, gsr_state_layout *out);

/* Per-stage device timing (hipEvents on the launch stream).  When enabled, every forward/backward
 * records an event pair around each stage; gsr_stage_times() returns the accumulated milliseconds
 * and call counts since the last reset. */
void gsr_set_profiling(int enable);
int gsr_num_stages(void);
const char *gsr_stage_name(int stage);
int gsr_stage_times(double *total_ms, int64_t *calls, int max_stages);
void gsr_reset_stage_times(void);

/* Internal tuning knobs for A/B measurements (e.g. "bwd_occ4"); unknown names are ignored by kernels. */
void gsr_set_tuning(const char *name, int value);
/* gsr_set_tuning(name, GSR_TUNING_UNSET) forgets the knob: its built-in default applies again. */
#define GSR_TUNING_UNSET (-2147483647 - 1)
/* A knob's value (default_value if never set).  The forward also records diagnostics here under "stat_*" names
 * (e.g. "stat_depth_passes": the radix passes of the last depth sort, 0 on the bucket path). */
int gsr_get_tuning(const char *name, int default_value);

/* Diagnostics: with the "stamp" knob set, the composite kernels record one (start, end, HW_ID, XCC_ID)
 * uint32 quadruple per launch slot (start/end on the 100 MHz real-time clock).  which = 0: render_fwd,
 * 1: render_bwd, 2: radix-sort pass blocks (start, ranked, looked back, end), 3: radix histogram blocks.  Copies up to max_slots quadruples to host memory; returns the count or < 0. */
int gsr_debug_wave_stamps(int which, uint32_t *host_dst, int max_slots);

const char *gsr_last_error(void);
const char *gsr_build_info(void);

/* Stream-ordered hand-off between two streams without events (the multi-view exchange's chunk hand-offs between the
 * compute stream and the collective stream): gsr_stream_signal writes `value` to the 4-B device word `flag` once the
 * stream's earlier work is done (hipStreamWriteValue32); gsr_stream_wait holds the stream's later work until
 * *flag >= value (hipStreamWaitValue32).  gsr_stream_values_supported() is 0 where the device lacks stream wait
 * values (the caller then uses events). */
int gsr_stream_values_supported(void);
int gsr_stream_signal(void *stream, uint32_t *flag, uint32_t value);
int gsr_stream_wait(void *stream, uint32_t *flag, uint32_t value);

/* ABI version of this header.  2: gsr_state_layout gained struct_size at offset 0 and lost img_tile_sorted /
 * img_tile_lastkey (a one-time break: a caller built against a version-1 header reads shifted offsets, so it must
 * check gsr_abi_version() == GSR_ABI_VERSION before using the layout).  From version 2 on, fields of the versioned
 * structs are only appended, and callers built against this header or a later one interoperate. */
#define GSR_ABI_VERSION 2
int gsr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GSRAST_H */
