// gsr_preprocess_bwd.hip -- per-Gaussian backward: gathers the instance gradient rows of every Gaussian
// (deterministic fixed order, through the inverse permutation), then the preprocess backward of the CUDA
// submodule restated: 2D conic -> cov2D -> cov3D -> scale / rotation, 2D mean -> 3D mean, SH -> colour.
// Its own translation unit so it can be compiled without SLP packing (build.py FILE_FLAGS).
#include "gsr_kernels.h"
#include "gsr_sh.h"

namespace gsr {

// ------------------------------------------------------------------------------------------------
// preprocess backward: one thread per Gaussian
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void cov3d_backward(float3 scale, float mod, float4 rot, const float dc[6],
                                               float3 &dscale, float4 &drot) {
    const float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
    const Mat3 R = quat_to_rot(rot);
    const float s[3] = {mod * scale.x, mod * scale.y, mod * scale.z};
    float M[3][3], dSig[3][3], dM[3][3], dMt[3][3];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++) M[c][rr] = s[rr] * R.m[c][rr];
    dSig[0][0] = dc[0]; dSig[0][1] = 0.5f * dc[1]; dSig[0][2] = 0.5f * dc[2];
    dSig[1][0] = 0.5f * dc[1]; dSig[1][1] = dc[3]; dSig[1][2] = 0.5f * dc[4];
    dSig[2][0] = 0.5f * dc[2]; dSig[2][1] = 0.5f * dc[4]; dSig[2][2] = dc[5];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++)
            dM[c][rr] = 2.0f * (M[0][rr] * dSig[c][0] + M[1][rr] * dSig[c][1] + M[2][rr] * dSig[c][2]);
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++) dMt[c][rr] = dM[rr][c];
    // dL/ds (w.r.t. the modified scale, as upstream; DESIGN.md notes the scale_modifier factor)
    dscale.x = R.m[0][0] * dMt[0][0] + R.m[1][0] * dMt[0][1] + R.m[2][0] * dMt[0][2];
    dscale.y = R.m[0][1] * dMt[1][0] + R.m[1][1] * dMt[1][1] + R.m[2][1] * dMt[1][2];
    dscale.z = R.m[0][2] * dMt[2][0] + R.m[1][2] * dMt[2][1] + R.m[2][2] * dMt[2][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        dMt[0][k] *= s[0];
        dMt[1][k] *= s[1];
        dMt[2][k] *= s[2];
    }
    drot.x = 2 * z * (dMt[0][1] - dMt[1][0]) + 2 * y * (dMt[2][0] - dMt[0][2]) + 2 * x * (dMt[1][2] - dMt[2][1]);
    drot.y = 2 * y * (dMt[1][0] + dMt[0][1]) + 2 * z * (dMt[2][0] + dMt[0][2]) + 2 * r * (dMt[1][2] - dMt[2][1]) -
             4 * x * (dMt[2][2] + dMt[1][1]);
    drot.z = 2 * x * (dMt[1][0] + dMt[0][1]) + 2 * r * (dMt[2][0] - dMt[0][2]) + 2 * z * (dMt[1][2] + dMt[2][1]) -
             4 * y * (dMt[2][2] + dMt[0][0]);
    drot.w = 2 * r * (dMt[0][1] - dMt[1][0]) + 2 * x * (dMt[2][0] + dMt[0][2]) + 2 * y * (dMt[1][2] + dMt[2][1]) -
             4 * z * (dMt[1][1] + dMt[0][0]);
}

// One Gaussian.  In the LDS-staged path (LDS) dL/dsh is not written here: the Gaussian's clamp-masked colour
// gradient and view direction go to dRGB_out / dir_out (dRGB zero when not visible) for the kernel's staged
// coalesced store; otherwise dL/dsh is written directly.
// The camera, read at the kernel's start before any store, so the compiler proves nothing clobbers it and loads it
// through the scalar unit (SGPRs) instead of vector loads with their own round trips (view at the geometry, projection
// matrix and position after it)
struct PbwdCamera {
    Mat4 view, proj;
    float3 campos;
};
__device__ __forceinline__ PbwdCamera load_camera(const PreprocessBwdParams &p) {
    PbwdCamera c;
    c.view = load_mat4(p.view);
    c.proj = load_mat4(p.proj);
    c.campos = (p.shs && p.M > 0) ? make_float3(p.campos[0], p.campos[1], p.campos[2]) : make_float3(0, 0, 0);
    return c;
}
template <bool LDS>
__device__ __forceinline__ void preprocess_bwd_one(const PreprocessBwdParams &p, const PbwdCamera &cam, const int i,
                                                   const int radius, const uint32_t n_tiles, bool have_gs,
                                                   const float (&gs_in)[10], float3 &dRGB_out, float3 &dir_out,
                                                   bool &zeroed) {
    // radius and kept-tile count: the caller's loads (reloaded here they took a round trip of their own)
    const bool vis = radius > 0;
    // The densification statistics' read-modify-writes: the reads issued here, the writes at the end (put_stats).
    // Read and written in place they cost two memory round trips before the geometry's loads were issued.
    float2 st_old = make_float2(0.f, 0.f);
    int mr_old = 0;
    if (p.densify_stats && p.densify_accumulate) st_old = *reinterpret_cast<const float2 *>(p.densify_stats + 2 * i);
    if (p.max_radii2D) mr_old = p.max_radii2D[i];
    float gs[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    auto put_stats = [&]() {
        if (p.densify_stats) {  // torch.linalg.vector_norm(grad[:, :2]) and the visibility count of this view
            float2 st = make_float2(sqrtf(gs[0] * gs[0] + gs[1] * gs[1]), vis ? 1.f : 0.f);
            if (p.densify_accumulate) st = make_float2(st_old.x + st.x, st_old.y + st.y);
            *reinterpret_cast<float2 *>(p.densify_stats + 2 * i) = st;
        }
        if (p.max_radii2D) p.max_radii2D[i] = max(mr_old, radius);
    };
    if (vis && have_gs && n_tiles <= BIG_GAUSSIAN_TILES) {
#pragma unroll
        for (int k = 0; k < 10; k++) gs[k] = gs_in[k];
    } else if (vis && (!p.live || !*p.live_valid || p.live[i])) {  // (no non-zero row stored: zero sums)
        const uint32_t start = p.inst_start[i], cnt = n_tiles;
        if (cnt > BIG_GAUSSIAN_TILES) {
            add_row(p.bigsum, p.big_slot[i], gs);
        } else {
            // the inv words first (INV_NONE: not loaded by the forward composite, no row), then all row loads of a
            // group, before summing (memory-level parallelism)
            for (uint32_t k0 = 0; k0 < cnt; k0 += 4) {
                bool use[4];
                uint32_t iv[4];
#pragma unroll
                for (int j = 0; j < 4; j++) iv[j] = p.inv[start + min(k0 + j, cnt - 1)];  // unconditional (clamped)
#pragma unroll
                for (int j = 0; j < 4; j++) use[j] = k0 + j < cnt && iv[j] != INV_NONE;
                float rw[4][10];
#pragma unroll
                for (int j = 0; j < 4; j++) load_row(p.rows, use[j] ? (size_t)(start + k0 + j) : 0u, rw[j]);  // row 0: dropped
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int k = 0; k < 10; k++) gs[k] += use[j] ? rw[j][k] : 0.f;
            }
        }
    }
    dRGB_out = make_float3(0.f, 0.f, 0.f);
    dir_out = make_float3(1.f, 0.f, 0.f);
    // Outputs zero-filled by the composite backward (prezeroed): a culled Gaussian, or one no pixel took a gradient
    // from (all ten row sums zero -- 78 % of the Gaussians at cfg 3), has an identically zero gradient (every output is
    // a linear function of the sums): only its statistics are written, and none of its geometry is read.
    if (p.prezeroed) {
        bool z = true;
#pragma unroll
        for (int k = 0; k < 10; k++) z = z && gs[k] == 0.f;
        if (!vis || z) {
            zeroed = true;
            put_stats();
            return;
        }
    }
    if (p.dL_dmeans2D) {
        p.dL_dmeans2D[3 * i] = gs[0];
        p.dL_dmeans2D[3 * i + 1] = gs[1];
        p.dL_dmeans2D[3 * i + 2] = 0.f;
    }
    if (p.dL_dcolors) {
        p.dL_dcolors[3 * i] = gs[6];
        p.dL_dcolors[3 * i + 1] = gs[7];
        p.dL_dcolors[3 * i + 2] = gs[8];
    }
    const int ncoef = p.M * 3;
    if (!vis) {
        if (p.dL_dopacity) p.dL_dopacity[i] = 0.f;
        if (p.dL_dmeans3D) { p.dL_dmeans3D[3 * i] = 0.f; p.dL_dmeans3D[3 * i + 1] = 0.f; p.dL_dmeans3D[3 * i + 2] = 0.f; }
        if (p.dL_dcov3D)
            for (int k = 0; k < 6; k++) p.dL_dcov3D[6 * i + k] = 0.f;
        if (p.dL_dsh && !LDS)
            for (int k = 0; k < ncoef; k++) p.dL_dsh[(size_t)i * ncoef + k] = 0.f;
        if (p.dL_dcolors_sh) { p.dL_dcolors_sh[3 * i] = 0.f; p.dL_dcolors_sh[3 * i + 1] = 0.f; p.dL_dcolors_sh[3 * i + 2] = 0.f; }
        if (p.dL_dscales) { p.dL_dscales[3 * i] = 0.f; p.dL_dscales[3 * i + 1] = 0.f; p.dL_dscales[3 * i + 2] = 0.f; }
        if (p.dL_drot)
            for (int k = 0; k < 4; k++) p.dL_drot[4 * i + k] = 0.f;
        put_stats();
        return;
    }
    const Mat4 &view = cam.view;
    const float3 mean = load_f3(p.means3D, i);
    // The SH stage's inputs (clamp bits, camera, the forward's colour Jacobian) requested with the geometry's: issued
    // at the SH stage, the clamp byte's round trip came before the Jacobian's nine loads were issued, two more memory
    // round trips per wave after the geometry's (measured in round 5: Appendix A.4 of DESIGN.md)
    const bool sh_stage = p.shs && p.M > 0;  // uniform
    uint8_t cl = 0;
    const float3 campos = cam.campos;
    float3 jx = make_float3(0, 0, 0), jy = jx, jz = jx;
    if (sh_stage) {
        cl = p.clamped[i];
        if (p.D > 0) {
            const size_t n = (size_t)p.P;
            const float *J = p.sh_jac + i;
            jx = make_float3(J[0], J[n], J[2 * n]);
            jy = make_float3(J[3 * n], J[4 * n], J[5 * n]);
            jz = make_float3(J[6 * n], J[7 * n], J[8 * n]);
        }
    }
    float c6[6];
    float3 scale = make_float3(0, 0, 0);
    float4 rot = make_float4(1, 0, 0, 0);
    if (p.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; k++) c6[k] = p.cov3D_precomp[6 * i + k];
    } else {
        scale = load_f3(p.scales, i);
        rot = make_float4(p.rotations[4 * i], p.rotations[4 * i + 1], p.rotations[4 * i + 2], p.rotations[4 * i + 3]);
        cov3d_from_scale_rot(scale, p.scale_modifier, rot, c6);
    }
    // ---- computeCov2D backward ----
    const EwaT e = ewa_T(mean, view, p.focal_x, p.focal_y, p.tan_fovx, p.tan_fovy);
    float c_xx = quad_form(e.t0, c6, e.t0), c_xy = quad_form(e.t1, c6, e.t0), c_yy = quad_form(e.t1, c6, e.t1);
    constexpr float h_var = 0.3f;
    float dopac = gs[5];
    float d_inside_root = 0.f;
    if (p.antialiasing) {
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_cov_plus = c_xx * c_yy - c_xy * c_xy;
        const float hs = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus));
        const float d_hs = dopac * p.opacities[i];
        dopac = dopac * hs;
        d_inside_root = (det_cov / det_cov_plus) <= 0.000025f ? 0.f : d_hs / (2 * hs);
    } else {
        c_xx += h_var;
        c_yy += h_var;
    }
    float dL_dc_xx = 0.f, dL_dc_xy = 0.f, dL_dc_yy = 0.f;
    if (p.antialiasing) {
        const float x = c_xx, y = c_yy, z = c_xy, wv = h_var;
        const float q = wv * wv + wv * (x + y) + x * y - z * z;
        const float denom_f = d_inside_root / (q * q);
        dL_dc_xx = wv * (wv * y + y * y + z * z) * denom_f;
        dL_dc_yy = wv * (wv * x + x * x + z * z) * denom_f;
        dL_dc_xy = -2.f * wv * z * (wv + x + y) * denom_f;
    }
    if (p.dL_dopacity) p.dL_dopacity[i] = dopac;
    const float dcx = gs[2], dcy = gs[3], dcz = gs[4];
    const float denom = c_xx * c_yy - c_xy * c_xy;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float dcov[6] = {0, 0, 0, 0, 0, 0};
    const float *t0 = e.t0, *t1 = e.t1;
    if (denom2inv != 0) {
        dL_dc_xx += denom2inv * (-c_yy * c_yy * dcx + 2 * c_xy * c_yy * dcy + (denom - c_xx * c_yy) * dcz);
        dL_dc_yy += denom2inv * (-c_xx * c_xx * dcz + 2 * c_xx * c_xy * dcy + (denom - c_xx * c_yy) * dcx);
        dL_dc_xy += denom2inv * 2 * (c_xy * c_yy * dcx - (denom + 2 * c_xy * c_xy) * dcy + c_xx * c_xy * dcz);
        dcov[0] = (t0[0] * t0[0] * dL_dc_xx + t0[0] * t1[0] * dL_dc_xy + t1[0] * t1[0] * dL_dc_yy);
        dcov[3] = (t0[1] * t0[1] * dL_dc_xx + t0[1] * t1[1] * dL_dc_xy + t1[1] * t1[1] * dL_dc_yy);
        dcov[5] = (t0[2] * t0[2] * dL_dc_xx + t0[2] * t1[2] * dL_dc_xy + t1[2] * t1[2] * dL_dc_yy);
        dcov[1] = 2 * t0[0] * t0[1] * dL_dc_xx + (t0[0] * t1[1] + t0[1] * t1[0]) * dL_dc_xy + 2 * t1[0] * t1[1] * dL_dc_yy;
        dcov[2] = 2 * t0[0] * t0[2] * dL_dc_xx + (t0[0] * t1[2] + t0[2] * t1[0]) * dL_dc_xy + 2 * t1[0] * t1[2] * dL_dc_yy;
        dcov[4] = 2 * t0[2] * t0[1] * dL_dc_xx + (t0[1] * t1[2] + t0[2] * t1[1]) * dL_dc_xy + 2 * t1[1] * t1[2] * dL_dc_yy;
    }
    if (p.dL_dcov3D)
        for (int k = 0; k < 6; k++) p.dL_dcov3D[6 * i + k] = dcov[k];
    float dT0[3], dT1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        // row k of the symmetric Vrk
        const float vk0 = k == 0 ? c6[0] : (k == 1 ? c6[1] : c6[2]);
        const float vk1 = k == 0 ? c6[1] : (k == 1 ? c6[3] : c6[4]);
        const float vk2 = k == 0 ? c6[2] : (k == 1 ? c6[4] : c6[5]);
        const float v0 = t0[0] * vk0 + t0[1] * vk1 + t0[2] * vk2;
        const float v1 = t1[0] * vk0 + t1[1] * vk1 + t1[2] * vk2;
        dT0[k] = 2 * v0 * dL_dc_xx + v1 * dL_dc_xy;
        dT1[k] = 2 * v1 * dL_dc_yy + v0 * dL_dc_xy;
    }
    const float *vm = view.m;
    const float dJ00 = vm[0] * dT0[0] + vm[4] * dT0[1] + vm[8] * dT0[2];
    const float dJ02 = vm[2] * dT0[0] + vm[6] * dT0[1] + vm[10] * dT0[2];
    const float dJ11 = vm[1] * dT1[0] + vm[5] * dT1[1] + vm[9] * dT1[2];
    const float dJ12 = vm[2] * dT1[0] + vm[6] * dT1[1] + vm[10] * dT1[2];
    const float3 t = e.t;
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float hx = p.focal_x, hy = p.focal_y;
    const float dtx = e.xmul * -hx * tz2 * dJ02;
    const float dty = e.ymul * -hy * tz2 * dJ12;
    float dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * t.x) * tz3 * dJ02 + (2 * hy * t.y) * tz3 * dJ12;
    if (p.has_invdepth) dtz -= gs[9] / (t.z * t.z);
    float3 dm = make_float3(vm[0] * dtx + vm[1] * dty + vm[2] * dtz, vm[4] * dtx + vm[5] * dty + vm[6] * dtz,
                            vm[8] * dtx + vm[9] * dty + vm[10] * dtz);
    // ---- 2D mean -> 3D mean through the projection ----
    const Mat4 &proj = cam.proj;
    const float *pm = proj.m;
    const float4 mh = xform4(mean, proj);
    const float m_w = 1.0f / (mh.w + 0.0000001f);
    const float mul1 = (pm[0] * mean.x + pm[4] * mean.y + pm[8] * mean.z + pm[12]) * m_w * m_w;
    const float mul2 = (pm[1] * mean.x + pm[5] * mean.y + pm[9] * mean.z + pm[13]) * m_w * m_w;
    const float g2x = gs[0], g2y = gs[1];
    dm.x += (pm[0] * m_w - pm[3] * mul1) * g2x + (pm[1] * m_w - pm[3] * mul2) * g2y;
    dm.y += (pm[4] * m_w - pm[7] * mul1) * g2x + (pm[5] * m_w - pm[7] * mul2) * g2y;
    dm.z += (pm[8] * m_w - pm[11] * mul1) * g2x + (pm[9] * m_w - pm[11] * mul2) * g2y;
    // ---- SH backward ----
    // dL/dsh = basis(dir) (x) dRGB needs only the direction; the direction term of dL/dmeans3D uses the colour's
    // direction Jacobian the forward stored (sh_jac), so the 48 coefficients are not read here.  (The backward's
    // shs are the forward's, as in the autograd function and the upstream API.)
    if (sh_stage) {
        const float3 dRGB = make_float3((cl & 1) ? 0.f : gs[6], (cl & 2) ? 0.f : gs[7], (cl & 4) ? 0.f : gs[8]);
        if (p.dL_dcolors_sh) {
            p.dL_dcolors_sh[3 * i] = dRGB.x;
            p.dL_dcolors_sh[3 * i + 1] = dRGB.y;
            p.dL_dcolors_sh[3 * i + 2] = dRGB.z;
        }
        float *dsh = p.dL_dsh ? p.dL_dsh + (size_t)i * ncoef : nullptr;  // null only with dL_dcolors_sh (API)
        if (LDS) {
            // LDS-staged block (M = 16): the kernel writes dL/dsh = basis (x) dRGB through LDS
            dm = dm + sh_dir_grad(mean - campos, dRGB, jx, jy, jz);
            dRGB_out = dRGB;
            dir_out = mean - campos;
        } else {
            float dshv[48];
            dm = dm + sh_backward_jac_dispatch(p.D, mean - campos, dRGB, jx, jy, jz, dshv);
            if (dsh && p.sh_vec16) {
                float4 *d4 = reinterpret_cast<float4 *>(dsh);
#pragma unroll
                for (int k = 0; k < 12; k++)
                    d4[k] = make_float4(dshv[4 * k], dshv[4 * k + 1], dshv[4 * k + 2], dshv[4 * k + 3]);
            } else if (dsh) {
                for (int k = 0; k < ncoef; k++) dsh[k] = k < 48 ? dshv[k] : 0.f;
            }
        }
    }
    if (p.dL_dmeans3D) {
        p.dL_dmeans3D[3 * i] = dm.x;
        p.dL_dmeans3D[3 * i + 1] = dm.y;
        p.dL_dmeans3D[3 * i + 2] = dm.z;
    }
    // ---- cov3D backward ----
    if (!p.cov3D_precomp && (p.dL_dscales || p.dL_drot)) {
        float3 dsc;
        float4 dr;
        cov3d_backward(scale, p.scale_modifier, rot, dcov, dsc, dr);
        if (p.dL_dscales) { p.dL_dscales[3 * i] = dsc.x; p.dL_dscales[3 * i + 1] = dsc.y; p.dL_dscales[3 * i + 2] = dsc.z; }
        if (p.dL_drot) { p.dL_drot[4 * i] = dr.x; p.dL_drot[4 * i + 1] = dr.y; p.dL_drot[4 * i + 2] = dr.z; p.dL_drot[4 * i + 3] = dr.w; }
    } else {
        if (p.dL_dscales) { p.dL_dscales[3 * i] = 0.f; p.dL_dscales[3 * i + 1] = 0.f; p.dL_dscales[3 * i + 2] = 0.f; }
        if (p.dL_drot)
            for (int k = 0; k < 4; k++) p.dL_drot[4 * i + k] = 0.f;
    }
    put_stats();
}

// dL/dsh (192 B per Gaussian at M = 16) is written through LDS: each half of a wave's 64 Gaussians writes its
// products basis (x) dRGB into a 32-Gaussian staging area, then the wave stores that 6 KB block with coalesced
// float4 stores (instead of 12 float4 stores per lane strided by 192 B).  In LDS each Gaussian's 48 floats sit
// at a 52-float stride, so both the linear block copy (ds_read_b128 of consecutive lanes) and each lane's float4
// writes to its own Gaussian (52 = 4 x 13, 13 odd: 16 lanes of a b128 lane group hit 16 distinct 4-bank windows)
// are free of bank conflicts.  The coefficients themselves are not read (sh_jac).  A half-wave staging area
// (6.5 KB, shared with the row-gather chunks) keeps the block at 26 KB of LDS: six blocks, the VGPR limit, per CU.
// The next chunk's loaded tests (inverse-permutation words) are issued during this chunk's row loads: cfg3 0.104 ->
// 0.100 ms, cfg5 0.521 -> 0.507 against all of a chunk's inv words first (round 5).
constexpr int SH_STRIDE = 52;
constexpr int PBWD_STAGE = 32 * SH_STRIDE;  // floats of LDS per wave

// Outputs zero-filled by the composite (prezeroed): after the row gather, the workgroup's Gaussians with a non-zero
// gradient (22 % at cfg 3, 4 % at cfg 5) are compacted through LDS onto its first lanes, so the per-Gaussian
// projection / covariance / SH backward runs on ~a quarter of the waves instead of on every wave that holds one such
// Gaussian (most of them: without compaction the compute cost was that of every Gaussian).  The others write only
// their densification statistics.  dL/dsh rows are staged per half-wave as before and stored cooperatively, 12 float4
// per Gaussian at the entry's own index.  Every workgroup barrier is reached by all four waves.
__device__ __forceinline__ void zero_gaussian_stats(const PreprocessBwdParams &p, int i, int radius) {
    if (p.densify_stats) {
        float2 st = make_float2(0.f, radius > 0 ? 1.f : 0.f);
        if (p.densify_accumulate) {
            const float2 o = *reinterpret_cast<const float2 *>(p.densify_stats + 2 * i);
            st = make_float2(o.x + st.x, o.y + st.y);
        }
        *reinterpret_cast<float2 *>(p.densify_stats + 2 * i) = st;
    }
    if (p.max_radii2D) p.max_radii2D[i] = max(p.max_radii2D[i], radius);
}
__device__ __forceinline__ void compacted_tail(const PreprocessBwdParams &p, const PbwdCamera &cam, const int i,
                                               const int rad, const uint32_t cnt, const bool has_rows,
                                               const float (&gs)[10], float *sw, const int w, const int lane) {
    __shared__ uint32_t s_wcnt[4];
    __shared__ int s_gi[256];  // entry -> Gaussian index
    // every entry's words, [word][entry], over the four waves' staging areas (free between the gather and the staging)
    float *list = sw - w * PBWD_STAGE;
    constexpr int NW = 12;  // radius, tile count, 10 sums
    static_assert(NW * 256 <= 4 * PBWD_STAGE, "the entry list fits the staging areas");
    bool nz = false;
    if (i < p.g1 && rad > 0) {
        nz = cnt > BIG_GAUSSIAN_TILES && has_rows;  // its sum (big_reduce) is read by preprocess_bwd_one
#pragma unroll
        for (int k = 0; k < 10; k++) nz = nz || gs[k] != 0.f;
    }
    if (i < p.g1 && !nz) zero_gaussian_stats(p, i, rad);
    const uint64_t bal = __ballot(nz);
    if (lane == 0) s_wcnt[w] = (uint32_t)__popcll(bal);
    __syncthreads();  // every wave's gather is done (its staging area free) and its count published
    uint32_t off = 0, total = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t c = s_wcnt[q];
        off += q < w ? c : 0u;
        total += c;
    }
    if (nz) {
        const uint32_t e = off + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        s_gi[e] = i;
        list[e] = __int_as_float(rad);
        list[256 + e] = __uint_as_float(cnt);
#pragma unroll
        for (int k = 0; k < 10; k++) list[(2 + k) * 256 + e] = gs[k];
    }
    __syncthreads();
    const uint32_t e = (uint32_t)(w * 64 + lane);
    const bool has = e < total;
    int ge = 0, rade = 0;
    uint32_t cnte = 0;
    float gse[10];
    if (has) {
        ge = s_gi[e];
        rade = __float_as_int(list[e]);
        cnte = __float_as_uint(list[256 + e]);
    }
#pragma unroll
    for (int k = 0; k < 10; k++) gse[k] = has ? list[(2 + k) * 256 + e] : 0.f;
    __syncthreads();  // the list is consumed: the areas are the waves' staging areas again
    if ((uint32_t)(w * 64) >= total) return;  // wave-uniform: no entry for this wave
    float3 dRGB = make_float3(0.f, 0.f, 0.f), dir = make_float3(1.f, 0.f, 0.f);
    bool zg = false;
    if (has) preprocess_bwd_one<true>(p, cam, ge, rade, cnte, true, gse, dRGB, dir, zg);
    if (!p.dL_dsh) return;
    const uint64_t live = __ballot(has && !zg);  // (a big Gaussian whose sum is zero stays zero-filled)
#pragma unroll
    for (int h = 0; h < 2; h++) {
        if (((live >> (32 * h)) & 0xffffffffull) == 0ull) continue;  // wave-uniform
        wave_lds_sync();
        if ((lane >> 5) == h && has) sh_dsh_dispatch(p.D, dir, dRGB, sw + (lane & 31) * SH_STRIDE);
        wave_lds_sync();
#pragma unroll
        for (int c = 0; c < 6; c++) {  // 32 Gaussians x 12 float4, each Gaussian's 192 B by 12 consecutive lanes
            const uint32_t q = (uint32_t)(c * 64 + lane), gl = q / 12, part = q % 12;
            if ((live >> (32 * h + gl)) & 1ull) {
                const int gi = s_gi[w * 64 + 32 * h + (int)gl];
                *reinterpret_cast<float4 *>(p.dL_dsh + (size_t)gi * 48 + part * 4) =
                    *reinterpret_cast<const float4 *>(sw + gl * SH_STRIDE + part * 4);
            }
        }
    }
}
template <bool LDS_SH, bool COMPACT = false>  // COMPACT: p.prezeroed (compacted_tail)
__global__ __launch_bounds__(256) void preprocess_bwd_kernel(PreprocessBwdParams p) {
    const int i = p.g0 + blockIdx.x * 256 + threadIdx.x;
    const PbwdCamera cam = load_camera(p);  // before the first store (scalar loads)
    if (p.campos_rows && blockIdx.x == 0)  // the exchange's camera block (row campos_rank = campos, others zero)
        for (int t = threadIdx.x; t < 3 * p.campos_nrows; t += 256)
            p.campos_rows[t] = t / 3 == p.campos_rank ? p.campos[t % 3] : 0.f;
    if (!LDS_SH) {
        const float none[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        float3 d3, v3;
        if (i < p.g1) {
            const int rad = p.radii[i];
            bool zg = false;
            preprocess_bwd_one<false>(p, cam, i, rad, rad > 0 ? p.tiles[i] : 0u, false, none, d3, v3, zg);
        }
        return;
    }
    __shared__ __attribute__((aligned(16))) float s_sh[4][PBWD_STAGE];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t gbase = ((size_t)p.g0 + (size_t)blockIdx.x * 256 + (size_t)w * 64) * 48;  // the wave's first float
    const size_t gend = (size_t)p.g1 * 48;
    float *sw = s_sh[w];
    // Gradient rows of the wave's 64 Gaussians (each Gaussian's rows are contiguous), gathered
    // jointly: the (Gaussian, row) pairs of all lanes are enumerated in order, every lane loads the inv words of
    // pairs l, l + 64, ... of a chunk, then the rows the composite wrote (others read as zero) into the LDS that later
    // stages dL/dsh, then each lane sums its own Gaussian's rows in row order.  Divergent per-lane
    // loops of dependent loads cost ~40 % of the kernel otherwise.  Gaussians above BIG_GAUSSIAN_TILES rows
    // take their block-reduced sum in preprocess_bwd_one.
    float gs[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    int rad;
    uint32_t cnt;
    bool live;
    {
        // radius, kept-tile count and first expansion index loaded together (clamped index, selected after)
        const int ic = min(i, p.g1 - 1);
        const int rad_l = p.radii[ic];
        const uint32_t cnt_l = p.tiles[ic], ist_l = p.inst_start[ic];
        // no non-zero row stored (GeomState::live): the sums are zero, so its rows are not gathered
        live = !p.live || !__builtin_amdgcn_readfirstlane(*p.live_valid) || p.live[ic] != 0;
        rad = i < p.g1 ? rad_l : 0;
        const bool vis = rad > 0;
        cnt = vis ? cnt_l : 0u;
        const uint32_t len = (cnt <= BIG_GAUSSIAN_TILES && live) ? cnt : 0u;
        const uint32_t incl = wave_inclusive_scan(len, lane);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t pst = incl - len;
        constexpr uint32_t CH = 128, PER = CH / 64;  // pairs per chunk: 10 floats each fit the staging area
        // (first pair, first expansion index) of each lane's Gaussian, behind the chunk
        uint2 *s_meta = reinterpret_cast<uint2 *>(sw + CH * 10);
        static_assert(CH * 10 + 128 <= PBWD_STAGE, "row chunk + meta fit the staging area");
        s_meta[lane] = make_uint2(pst, len ? ist_l : 0u);
        wave_lds_sync();
        // the inv words of chunk c0 (expansion index uu, written-row marker sidx; pairs past the wave's total read
        // inv[0] and are dropped at use).  Every load is unconditional: a load (or a row load) under a branch made the
        // compiler wait for it before the next pair's test, one memory round trip per pair instead of per chunk.
        auto inv_chunk = [&](uint32_t c0, uint32_t (&uu)[PER], uint32_t (&sidx)[PER]) {
#pragma unroll
            for (uint32_t r = 0; r < PER; r++) {
                const uint32_t j = c0 + r * 64 + lane;
                int o = 0;
#pragma unroll
                for (int step = 32; step; step >>= 1)
                    if (s_meta[o + step].x <= j) o += step;
                const uint2 m = s_meta[o];
                uu[r] = j < total ? m.y + (j - m.x) : 0u;
                sidx[r] = p.inv[uu[r]];
            }
        };
        uint32_t uu_n[PER], sidx_n[PER];
        if (total) inv_chunk(0, uu_n, sidx_n);
        for (uint32_t c0 = 0; c0 < total; c0 += CH) {
            float rw[PER][10];
            uint32_t sidx[PER];
            uint32_t uu[PER];
#pragma unroll
            for (uint32_t r = 0; r < PER; r++) {  // this chunk's loaded tests, made during the previous chunk
                uu[r] = uu_n[r];
                sidx[r] = sidx_n[r];
            }
            bool use[PER];
#pragma unroll
            for (uint32_t r = 0; r < PER; r++) {  // the rows the composite wrote (others read row 0, dropped)
                use[r] = c0 + r * 64 + lane < total && sidx[r] != INV_NONE;
                load_row(p.rows, use[r] ? uu[r] : 0u, rw[r]);
            }
            if (c0 + CH < total) inv_chunk(c0 + CH, uu_n, sidx_n);  // the next chunk's inv words meanwhile
#pragma unroll
            for (uint32_t r = 0; r < PER; r++) {
                const uint32_t q = r * 64 + lane;  // pair within the chunk
                float *d = sw + q * 10;
#pragma unroll
                for (int k = 0; k < 10; k++) d[k] = use[r] ? rw[r][k] : 0.f;
            }
            wave_lds_sync();
            const uint32_t lo = max(pst, c0), hi = min(pst + len, c0 + CH);
            for (uint32_t j = lo; j < hi; j++) {
                const float *d = sw + (j - c0) * 10;
#pragma unroll
                for (int k = 0; k < 10; k++) gs[k] += d[k];
            }
            wave_lds_sync();
        }
    }
    float3 dRGB = make_float3(0.f, 0.f, 0.f), dir = make_float3(1.f, 0.f, 0.f);
    bool zg = false;
    if constexpr (COMPACT) {
        compacted_tail(p, cam, i, rad, cnt, live, gs, sw, w, lane);
        return;
    }
    if (i < p.g1) preprocess_bwd_one<true>(p, cam, i, rad, cnt, true, gs, dRGB, dir, zg);
    if (!p.dL_dsh) return;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        wave_lds_sync();  // the area's previous contents (row chunks or the other half) are consumed
        if ((lane >> 5) == h) sh_dsh_dispatch(p.D, dir, dRGB, sw + (lane & 31) * SH_STRIDE);
        wave_lds_sync();
#pragma unroll
        for (int c = 0; c < 6; c++) {  // 32 Gaussians x 48 floats = 384 float4, 6 per lane
            const uint32_t f = c * 256 + lane * 4;
            const size_t go = gbase + (size_t)h * 1536 + f;
            if (go < gend)
                *reinterpret_cast<float4 *>(p.dL_dsh + go) =
                    *reinterpret_cast<const float4 *>(sw + (f / 48) * SH_STRIDE + f % 48);
        }
    }
}

void launch_preprocess_bwd(hipStream_t s, const PreprocessBwdParams &p) {
    if (p.g1 <= p.g0) return;
    const uint32_t grid = div_up((uint32_t)(p.g1 - p.g0), 256);
    // the joint row gather and the LDS-staged dL/dsh stores; without dL/dsh (the compact multi-view exchange) only
    // the gather, which the per-lane path pays ~40 % of the kernel for
    if ((p.dL_dsh ? p.sh_vec16 : true) && tuning("pbwd_lds_sh", 1) && p.prezeroed)
        preprocess_bwd_kernel<true, true><<<grid, 256, 0, s>>>(p);
    else if ((p.dL_dsh ? p.sh_vec16 : true) && tuning("pbwd_lds_sh", 1))
        preprocess_bwd_kernel<true><<<grid, 256, 0, s>>>(p);
    else
        preprocess_bwd_kernel<false><<<grid, 256, 0, s>>>(p);
}

}  // namespace gsr
