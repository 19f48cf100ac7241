// gsr_torch_ext.cpp -- the thin torch extension of the drop-in: the `_C` module of the diff_gaussian_rasterization
// package, with the pybind entry points the upstream package exports (graphdeco-inria/diff-gaussian-rasterization
// @dr_aa, ext.cpp / rasterize_points.h: rasterize_gaussians, rasterize_gaussians_backward, mark_visible, and adam.h's
// adamUpdate behind SparseGaussianAdam; SURVEY.md
// §8(b) "C-ABI / extension"), implemented over the C ABI of libgsrast.so (include/gsrast.h).  Tensors in, tensors
// out, on torch's current HIP stream; the scratch buffers are uint8 tensors grown through the ABI's allocation
// callback (the upstream resizeFunctional, notes/rasterizer_note.h:27-40).  The reference never calls _C itself
// (it goes through the Python API, gaussian_splatting_lightning_amd/rasterizer.py); this module is for code that
// imports `diff_gaussian_rasterization._C` directly, and tests/test_torch_ext.py checks it against the Python path.
#include <torch/extension.h>
// PyTorch-ROCm tags HIP devices as "cuda"; its own guard and stream accessors for them are the MasqueradingAsCUDA ones
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <algorithm>
#include <tuple>

#include "gsrast.h"

namespace {

struct Buffers {
    torch::Device device;
    torch::Tensor t[4];
};

char *alloc_cb(void *ctx, int which, size_t nbytes) {
    auto *b = static_cast<Buffers *>(ctx);
    if (which < 0 || which > 3) return nullptr;
    try {
        b->t[which] = torch::empty({(int64_t)std::max<size_t>(nbytes, 1)},
                                   torch::TensorOptions().dtype(torch::kUInt8).device(b->device));
    } catch (...) {
        return nullptr;  // GSR_ERR_ALLOC, reported below with the library's message
    }
    return reinterpret_cast<char *>(b->t[which].data_ptr());
}

void check(int rc, const char *what) { TORCH_CHECK(rc == 0, what, " failed (code ", rc, "): ", gsr_last_error()); }

const float *fptr(const torch::Tensor &t) { return t.defined() && t.numel() ? t.data_ptr<float>() : nullptr; }

torch::Tensor f32c(const torch::Tensor &t, const char *name) {
    if (!t.defined() || t.numel() == 0) return torch::Tensor();
    TORCH_CHECK(t.is_cuda(), name, " must be a HIP device tensor");
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
    return t.contiguous();
}

void *stream_of(const torch::Tensor &t) {
    return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

}  // namespace

// RasterizeGaussiansCUDA -> (num_rendered, color (3,H,W), radii (P), geomBuffer, binningBuffer, imgBuffer,
// invdepth (1,H,W))
std::tuple<int, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor>
rasterize_gaussians(const torch::Tensor &background, const torch::Tensor &means3D, const torch::Tensor &colors,
                    const torch::Tensor &opacity, const torch::Tensor &scales, const torch::Tensor &rotations,
                    const float scale_modifier, const torch::Tensor &cov3D_precomp, const torch::Tensor &viewmatrix,
                    const torch::Tensor &projmatrix, const float tan_fovx, const float tan_fovy, const int image_height,
                    const int image_width, const torch::Tensor &sh, const int degree, const torch::Tensor &campos,
                    const bool prefiltered, const bool antialiasing, const bool debug) {
    TORCH_CHECK(means3D.ndimension() == 2 && means3D.size(1) == 3, "means3D must have dimensions (num_points, 3)");
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(means3D.device());
    const int P = (int)means3D.size(0), H = image_height, W = image_width;
    auto m = f32c(means3D, "means3D"), bg = f32c(background, "background"), col = f32c(colors, "colors"),
         op = f32c(opacity, "opacity"), sc = f32c(scales, "scales"), rot = f32c(rotations, "rotations"),
         cov = f32c(cov3D_precomp, "cov3D_precomp"), vm = f32c(viewmatrix, "viewmatrix"),
         pm = f32c(projmatrix, "projmatrix"), shs = f32c(sh, "sh"), cp = f32c(campos, "campos");
    const int M = shs.defined() ? (int)(shs.ndimension() == 3 ? shs.size(1) : shs.size(1) / 3) : 0;
    auto fopt = torch::TensorOptions().dtype(torch::kFloat32).device(means3D.device());
    auto color = torch::empty({3, H, W}, fopt);
    auto invdepth = torch::empty({1, H, W}, fopt);
    auto radii = torch::empty({P}, fopt.dtype(torch::kInt32));
    Buffers bufs{means3D.device(), {}};
    gsr_forward_args a{};
    a.P = P; a.D = degree; a.M = M; a.W = W; a.H = H;
    a.background = fptr(bg); a.means3D = fptr(m); a.colors_precomp = fptr(col); a.opacities = fptr(op);
    a.scales = fptr(sc); a.scale_modifier = scale_modifier; a.rotations = fptr(rot); a.cov3D_precomp = fptr(cov);
    a.viewmatrix = fptr(vm); a.projmatrix = fptr(pm); a.campos = fptr(cp); a.tan_fovx = tan_fovx; a.tan_fovy = tan_fovy;
    a.shs = fptr(shs); a.prefiltered = prefiltered; a.antialiasing = antialiasing; a.debug = debug;
    a.out_color = color.data_ptr<float>(); a.out_invdepth = invdepth.data_ptr<float>();
    a.radii = P ? radii.data_ptr<int>() : nullptr;
    int64_t num_rendered = 0;
    check(gsr_forward(&a, alloc_cb, &bufs, stream_of(means3D), &num_rendered), "rasterize_gaussians");
    auto u8 = [&](int which) {
        return bufs.t[which].defined() ? bufs.t[which]
                                       : torch::empty({0}, torch::TensorOptions().dtype(torch::kUInt8).device(means3D.device()));
    };
    return {(int)num_rendered, color, radii, u8(GSR_BUF_GEOM), u8(GSR_BUF_BINNING), u8(GSR_BUF_IMAGE), invdepth};
}

// RasterizeGaussiansBackwardCUDA -> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh,
// dL_dscales, dL_drotations)
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
           torch::Tensor>
rasterize_gaussians_backward(const torch::Tensor &background, const torch::Tensor &means3D,
                             const torch::Tensor &radii, const torch::Tensor &colors, const torch::Tensor &opacities,
                             const torch::Tensor &scales, const torch::Tensor &rotations, const float scale_modifier,
                             const torch::Tensor &cov3D_precomp, const torch::Tensor &viewmatrix,
                             const torch::Tensor &projmatrix, const float tan_fovx, const float tan_fovy,
                             const torch::Tensor &dL_dout_color, const torch::Tensor &dL_dout_invdepth,
                             const torch::Tensor &sh, const int degree, const torch::Tensor &campos,
                             const torch::Tensor &geomBuffer, const int R, const torch::Tensor &binningBuffer,
                             const torch::Tensor &imageBuffer, const bool antialiasing, const bool debug) {
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(means3D.device());
    const int P = (int)means3D.size(0), H = (int)dL_dout_color.size(1), W = (int)dL_dout_color.size(2);
    auto m = f32c(means3D, "means3D"), bg = f32c(background, "background"), col = f32c(colors, "colors"),
         op = f32c(opacities, "opacities"), sc = f32c(scales, "scales"), rot = f32c(rotations, "rotations"),
         cov = f32c(cov3D_precomp, "cov3D_precomp"), vm = f32c(viewmatrix, "viewmatrix"),
         pm = f32c(projmatrix, "projmatrix"), shs = f32c(sh, "sh"), cp = f32c(campos, "campos"),
         dpix = f32c(dL_dout_color, "dL_dout_color"), dinv = f32c(dL_dout_invdepth, "dL_dout_invdepth");
    const int M = shs.defined() ? (int)(shs.ndimension() == 3 ? shs.size(1) : shs.size(1) / 3) : 0;
    auto fopt = torch::TensorOptions().dtype(torch::kFloat32).device(means3D.device());
    auto dmeans2D = torch::zeros({P, 3}, fopt), dcolors = torch::zeros({P, 3}, fopt),
         dopac = torch::zeros({P, 1}, fopt), dmeans3D = torch::zeros({P, 3}, fopt),
         dcov = torch::zeros({P, 6}, fopt), dsh = torch::zeros({P, M, 3}, fopt), dscales = torch::zeros({P, 3}, fopt),
         drot = torch::zeros({P, 4}, fopt);
    auto rad = radii.contiguous();
    TORCH_CHECK(rad.scalar_type() == torch::kInt32, "radii must be int32 (the forward's output)");
    Buffers bufs{means3D.device(), {}};
    gsr_backward_args a{};
    a.P = P; a.D = degree; a.M = M; a.W = W; a.H = H; a.R = R;
    a.num_big = -1;  // not part of the upstream signature: the library reads it from the geometry buffer
    a.background = fptr(bg); a.means3D = fptr(m); a.colors_precomp = fptr(col); a.opacities = fptr(op);
    a.scales = fptr(sc); a.scale_modifier = scale_modifier; a.rotations = fptr(rot); a.cov3D_precomp = fptr(cov);
    a.viewmatrix = fptr(vm); a.projmatrix = fptr(pm); a.campos = fptr(cp); a.tan_fovx = tan_fovx; a.tan_fovy = tan_fovy;
    a.dL_dpix = fptr(dpix); a.dL_dinvdepth = fptr(dinv); a.shs = fptr(shs);
    a.radii = P ? rad.data_ptr<int>() : nullptr;
    a.geom_buffer = reinterpret_cast<char *>(geomBuffer.data_ptr());
    a.binning_buffer = binningBuffer.numel() ? reinterpret_cast<char *>(binningBuffer.data_ptr()) : nullptr;
    a.image_buffer = reinterpret_cast<char *>(imageBuffer.data_ptr());
    a.antialiasing = antialiasing; a.debug = debug;
    a.dL_dmeans2D = dmeans2D.data_ptr<float>(); a.dL_dcolors = dcolors.data_ptr<float>();
    a.dL_dopacity = dopac.data_ptr<float>(); a.dL_dmeans3D = dmeans3D.data_ptr<float>();
    a.dL_dcov3D = dcov.data_ptr<float>(); a.dL_dsh = M ? dsh.data_ptr<float>() : nullptr;
    a.dL_dscales = dscales.data_ptr<float>(); a.dL_drotations = drot.data_ptr<float>();
    check(gsr_backward(&a, alloc_cb, &bufs, stream_of(means3D)), "rasterize_gaussians_backward");
    return {dmeans2D, dcolors, dopac, dmeans3D, dcov, dsh, dscales, drot};
}

// markVisible -> bool (P)
torch::Tensor mark_visible(const torch::Tensor &means3D, const torch::Tensor &viewmatrix,
                           const torch::Tensor &projmatrix) {
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(means3D.device());
    auto m = f32c(means3D, "means3D"), vm = f32c(viewmatrix, "viewmatrix"), pm = f32c(projmatrix, "projmatrix");
    const int P = (int)means3D.size(0);
    auto present = torch::zeros({P}, torch::TensorOptions().dtype(torch::kBool).device(means3D.device()));
    if (P)
        check(gsr_mark_visible(P, fptr(m), fptr(vm), fptr(pm), reinterpret_cast<uint8_t *>(present.data_ptr()),
                               stream_of(means3D)),
              "mark_visible");
    return present;
}

// adamUpdate (the upstream package's SparseGaussianAdam step, adam.h): param, exp_avg, exp_avg_sq updated in place
// for the Gaussians with visible set; N Gaussians of M elements each
void adamUpdate(torch::Tensor &param, torch::Tensor &param_grad, torch::Tensor &exp_avg, torch::Tensor &exp_avg_sq,
                torch::Tensor &visible, const float lr, const float b1, const float b2, const float eps, const uint32_t N,
                const uint32_t M) {
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(param.device());
    for (const torch::Tensor *t : {&param, &param_grad, &exp_avg, &exp_avg_sq}) {
        TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kFloat32 && t->is_contiguous(),
                    "adamUpdate: param, grad and moments must be contiguous float32 HIP tensors");
        TORCH_CHECK(t->numel() == (int64_t)N * M, "adamUpdate: tensors must hold N x M elements");
    }
    TORCH_CHECK(visible.is_cuda() && visible.numel() == (int64_t)N && visible.element_size() == 1 && visible.is_contiguous(),
                "adamUpdate: visible must be a contiguous (N,) bool HIP tensor");
    if ((int64_t)N * M == 0) return;
    gsr_adam_group g{param.data_ptr<float>(), param_grad.data_ptr<float>(), exp_avg.data_ptr<float>(),
                     exp_avg_sq.data_ptr<float>(), (int64_t)N * M, (double)lr, 0};
    check(gsr_sparse_adam_step(&g, 1, reinterpret_cast<const uint8_t *>(visible.data_ptr()), (int64_t)N, (double)b1,
                               (double)b2, (double)eps, stream_of(param)),
          "adamUpdate");
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.def("rasterize_gaussians", &rasterize_gaussians);
    m.def("rasterize_gaussians_backward", &rasterize_gaussians_backward);
    m.def("mark_visible", &mark_visible);
    m.def("adamUpdate", &adamUpdate);
}
