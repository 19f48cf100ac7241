// gsr_sh.h -- spherical-harmonics colour (degree <= 3) and its backward, compile-time degree.
// Forward follows gs_lightning/utils/sh.py:41-98 + render_tools.py:118-131 of the reference
// (+0.5 offset, clamp at 0, record the clamp); backward is the CUDA rule (clamped channels get zero
// gradient, the view direction's normalisation is differentiated through dnormvdv).
#pragma once
#include "gsr_common.h"

namespace gsr {

__device__ __forceinline__ float3 f3(const float *p) { return make_float3(p[0], p[1], p[2]); }
__device__ __forceinline__ float3 operator*(float a, float3 b) { return make_float3(a * b.x, a * b.y, a * b.z); }
__device__ __forceinline__ float3 operator+(float3 a, float3 b) { return make_float3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ float3 operator-(float3 a, float3 b) { return make_float3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float dot3(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// The colour offset rgb + 0.5 (render_tools.py:129) as an add that is never contracted into the SH sum's last
// multiply: at degree 0 that sum IS a multiply (C0 * sh), and whether the backend fused the two into an fma depended on
// the block layout around the call (the fused preprocess's runtime degree switch vs the split kernel's template).
// The pragma strips the add's contract flag (HIP's __fadd_rn is a plain, contractable add).
__device__ __forceinline__ float3 sh_offset(float3 c) {
#pragma clang fp contract(off)
    return make_float3(c.x + 0.5f, c.y + 0.5f, c.z + 0.5f);
}

template <int DEG>
__device__ __forceinline__ float3 sh_eval(const float *__restrict__ sh, float3 dir) {
    float3 res = GSR_SH_C0 * f3(sh);
    if (DEG > 0) {
        const float x = dir.x, y = dir.y, z = dir.z;
        res = res - (GSR_SH_C1 * y) * f3(sh + 3) + (GSR_SH_C1 * z) * f3(sh + 6) - (GSR_SH_C1 * x) * f3(sh + 9);
        if (DEG > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            res = res + (SH_C2[0] * xy) * f3(sh + 12) + (SH_C2[1] * yz) * f3(sh + 15) +
                  (SH_C2[2] * (2.0f * zz - xx - yy)) * f3(sh + 18) + (SH_C2[3] * xz) * f3(sh + 21) +
                  (SH_C2[4] * (xx - yy)) * f3(sh + 24);
            if (DEG > 2) {
                res = res + (SH_C3[0] * y * (3.0f * xx - yy)) * f3(sh + 27) + (SH_C3[1] * xy * z) * f3(sh + 30) +
                      (SH_C3[2] * y * (4.0f * zz - xx - yy)) * f3(sh + 33) +
                      (SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy)) * f3(sh + 36) +
                      (SH_C3[4] * x * (4.0f * zz - xx - yy)) * f3(sh + 39) +
                      (SH_C3[5] * z * (xx - yy)) * f3(sh + 42) + (SH_C3[6] * x * (xx - 3.0f * yy)) * f3(sh + 45);
            }
        }
    }
    return res;
}

__device__ __forceinline__ float3 sh_dispatch(int deg, const float *__restrict__ sh, float3 dir) {
    switch (deg) {
        case 0: return sh_eval<0>(sh, dir);
        case 1: return sh_eval<1>(sh, dir);
        case 2: return sh_eval<2>(sh, dir);
        default: return sh_eval<3>(sh, dir);
    }
}

// Colour and its Jacobian with respect to the unit view direction, in one pass over the coefficients:
// jx = d rgb / d dir.x (one float3 over the colour channels), likewise jy, jz.  The forward stores the Jacobian
// (9 floats per Gaussian) so the backward forms dL/ddir = (jx . dRGB, jy . dRGB, jz . dRGB) without reading
// the 48 coefficients again; the expressions are sh_backward's, so the product is bitwise the same.
template <int DEG>
__device__ __forceinline__ float3 sh_eval_jac(const float *__restrict__ sh, float3 dir, float3 &jx, float3 &jy,
                                              float3 &jz) {
    const float3 res = sh_eval<DEG>(sh, dir);
    jx = jy = jz = make_float3(0, 0, 0);
    const float x = dir.x, y = dir.y, z = dir.z;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    if (DEG > 0) {
        jx = -GSR_SH_C1 * f3(sh + 9);
        jy = -GSR_SH_C1 * f3(sh + 3);
        jz = GSR_SH_C1 * f3(sh + 6);
        if (DEG > 1) {
            const float3 s4 = f3(sh + 12), s5 = f3(sh + 15), s6 = f3(sh + 18), s7 = f3(sh + 21), s8 = f3(sh + 24);
            jx = jx + (SH_C2[0] * y) * s4 + (SH_C2[2] * 2.f * -x) * s6 + (SH_C2[3] * z) * s7 + (SH_C2[4] * 2.f * x) * s8;
            jy = jy + (SH_C2[0] * x) * s4 + (SH_C2[1] * z) * s5 + (SH_C2[2] * 2.f * -y) * s6 + (SH_C2[4] * 2.f * -y) * s8;
            jz = jz + (SH_C2[1] * y) * s5 + (SH_C2[2] * 2.f * 2.f * z) * s6 + (SH_C2[3] * x) * s7;
            if (DEG > 2) {
                const float3 s9 = f3(sh + 27), s10 = f3(sh + 30), s11 = f3(sh + 33), s12 = f3(sh + 36),
                             s13 = f3(sh + 39), s14 = f3(sh + 42), s15 = f3(sh + 45);
                jx = jx + (SH_C3[0] * 3.f * 2.f * xy) * s9 + (SH_C3[1] * yz) * s10 + (SH_C3[2] * -2.f * xy) * s11 +
                     (SH_C3[3] * -3.f * 2.f * xz) * s12 + (SH_C3[4] * (-3.f * xx + 4.f * zz - yy)) * s13 +
                     (SH_C3[5] * 2.f * xz) * s14 + (SH_C3[6] * 3.f * (xx - yy)) * s15;
                jy = jy + (SH_C3[0] * 3.f * (xx - yy)) * s9 + (SH_C3[1] * xz) * s10 +
                     (SH_C3[2] * (-3.f * yy + 4.f * zz - xx)) * s11 + (SH_C3[3] * -3.f * 2.f * yz) * s12 +
                     (SH_C3[4] * -2.f * xy) * s13 + (SH_C3[5] * -2.f * yz) * s14 + (SH_C3[6] * -3.f * 2.f * xy) * s15;
                jz = jz + (SH_C3[1] * xy) * s10 + (SH_C3[2] * 4.f * 2.f * yz) * s11 +
                     (SH_C3[3] * 3.f * (2.f * zz - xx - yy)) * s12 + (SH_C3[4] * 4.f * 2.f * xz) * s13 +
                     (SH_C3[5] * (xx - yy)) * s14;
            }
        }
    }
    return res;
}

__device__ __forceinline__ float3 sh_eval_jac_dispatch(int deg, const float *__restrict__ sh, float3 dir, float3 &jx,
                                                       float3 &jy, float3 &jz) {
    switch (deg) {
        case 0: return sh_eval_jac<0>(sh, dir, jx, jy, jz);
        case 1: return sh_eval_jac<1>(sh, dir, jx, jy, jz);
        case 2: return sh_eval_jac<2>(sh, dir, jx, jy, jz);
        default: return sh_eval_jac<3>(sh, dir, jx, jy, jz);
    }
}

__device__ __forceinline__ float3 dnormvdv(float3 v, float3 dv) {
    const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    return make_float3(((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32,
                       (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32,
                       (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32);
}

__device__ __forceinline__ void st3(float *p, float3 v) {
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}

// Writes dL/dsh for coefficients [0, (DEG+1)^2) and returns dL/dmean through the view direction.
template <int DEG>
__device__ __forceinline__ float3 sh_backward(const float *__restrict__ sh, float3 dir_orig, float3 dRGB,
                                              float *__restrict__ dsh) {
    const float len = sqrtf(dot3(dir_orig, dir_orig));
    const float3 dir = make_float3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
    float3 dx = make_float3(0, 0, 0), dy = dx, dz = dx;
    const float x = dir.x, y = dir.y, z = dir.z;
    st3(dsh, GSR_SH_C0 * dRGB);
    if (DEG > 0) {
        st3(dsh + 3, (-GSR_SH_C1 * y) * dRGB);
        st3(dsh + 6, (GSR_SH_C1 * z) * dRGB);
        st3(dsh + 9, (-GSR_SH_C1 * x) * dRGB);
        dx = -GSR_SH_C1 * f3(sh + 9);
        dy = -GSR_SH_C1 * f3(sh + 3);
        dz = GSR_SH_C1 * f3(sh + 6);
        if (DEG > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            st3(dsh + 12, (SH_C2[0] * xy) * dRGB);
            st3(dsh + 15, (SH_C2[1] * yz) * dRGB);
            st3(dsh + 18, (SH_C2[2] * (2.f * zz - xx - yy)) * dRGB);
            st3(dsh + 21, (SH_C2[3] * xz) * dRGB);
            st3(dsh + 24, (SH_C2[4] * (xx - yy)) * dRGB);
            const float3 s4 = f3(sh + 12), s5 = f3(sh + 15), s6 = f3(sh + 18), s7 = f3(sh + 21), s8 = f3(sh + 24);
            dx = dx + (SH_C2[0] * y) * s4 + (SH_C2[2] * 2.f * -x) * s6 + (SH_C2[3] * z) * s7 + (SH_C2[4] * 2.f * x) * s8;
            dy = dy + (SH_C2[0] * x) * s4 + (SH_C2[1] * z) * s5 + (SH_C2[2] * 2.f * -y) * s6 + (SH_C2[4] * 2.f * -y) * s8;
            dz = dz + (SH_C2[1] * y) * s5 + (SH_C2[2] * 2.f * 2.f * z) * s6 + (SH_C2[3] * x) * s7;
            if (DEG > 2) {
                st3(dsh + 27, (SH_C3[0] * y * (3.f * xx - yy)) * dRGB);
                st3(dsh + 30, (SH_C3[1] * xy * z) * dRGB);
                st3(dsh + 33, (SH_C3[2] * y * (4.f * zz - xx - yy)) * dRGB);
                st3(dsh + 36, (SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy)) * dRGB);
                st3(dsh + 39, (SH_C3[4] * x * (4.f * zz - xx - yy)) * dRGB);
                st3(dsh + 42, (SH_C3[5] * z * (xx - yy)) * dRGB);
                st3(dsh + 45, (SH_C3[6] * x * (xx - 3.f * yy)) * dRGB);
                const float3 s9 = f3(sh + 27), s10 = f3(sh + 30), s11 = f3(sh + 33), s12 = f3(sh + 36),
                             s13 = f3(sh + 39), s14 = f3(sh + 42), s15 = f3(sh + 45);
                dx = dx + (SH_C3[0] * 3.f * 2.f * xy) * s9 + (SH_C3[1] * yz) * s10 + (SH_C3[2] * -2.f * xy) * s11 +
                     (SH_C3[3] * -3.f * 2.f * xz) * s12 + (SH_C3[4] * (-3.f * xx + 4.f * zz - yy)) * s13 +
                     (SH_C3[5] * 2.f * xz) * s14 + (SH_C3[6] * 3.f * (xx - yy)) * s15;
                dy = dy + (SH_C3[0] * 3.f * (xx - yy)) * s9 + (SH_C3[1] * xz) * s10 +
                     (SH_C3[2] * (-3.f * yy + 4.f * zz - xx)) * s11 + (SH_C3[3] * -3.f * 2.f * yz) * s12 +
                     (SH_C3[4] * -2.f * xy) * s13 + (SH_C3[5] * -2.f * yz) * s14 + (SH_C3[6] * -3.f * 2.f * xy) * s15;
                dz = dz + (SH_C3[1] * xy) * s10 + (SH_C3[2] * 4.f * 2.f * yz) * s11 +
                     (SH_C3[3] * 3.f * (2.f * zz - xx - yy)) * s12 + (SH_C3[4] * 4.f * 2.f * xz) * s13 +
                     (SH_C3[5] * (xx - yy)) * s14;
            }
        }
    }
    const float3 dL_ddir = make_float3(dot3(dx, dRGB), dot3(dy, dRGB), dot3(dz, dRGB));
    return dnormvdv(dir_orig, dL_ddir);
}

// sh_backward on one buffer: reads the coefficients, then overwrites them with dL/dsh (zeros above the degree,
// up to 16 coefficients).  For an LDS-staged block, so the coefficients never occupy registers all at once.
template <int DEG>
__device__ __forceinline__ float3 sh_backward_inplace(float *sh_io, float3 dir_orig, float3 dRGB) {
    const float len = sqrtf(dot3(dir_orig, dir_orig));
    const float3 dir = make_float3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
    float3 dx = make_float3(0, 0, 0), dy = dx, dz = dx;
    const float x = dir.x, y = dir.y, z = dir.z;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    const float *sh = sh_io;
    if (DEG > 0) {
        dx = -GSR_SH_C1 * f3(sh + 9);
        dy = -GSR_SH_C1 * f3(sh + 3);
        dz = GSR_SH_C1 * f3(sh + 6);
        if (DEG > 1) {
            const float3 s4 = f3(sh + 12), s5 = f3(sh + 15), s6 = f3(sh + 18), s7 = f3(sh + 21), s8 = f3(sh + 24);
            dx = dx + (SH_C2[0] * y) * s4 + (SH_C2[2] * 2.f * -x) * s6 + (SH_C2[3] * z) * s7 + (SH_C2[4] * 2.f * x) * s8;
            dy = dy + (SH_C2[0] * x) * s4 + (SH_C2[1] * z) * s5 + (SH_C2[2] * 2.f * -y) * s6 + (SH_C2[4] * 2.f * -y) * s8;
            dz = dz + (SH_C2[1] * y) * s5 + (SH_C2[2] * 2.f * 2.f * z) * s6 + (SH_C2[3] * x) * s7;
            if (DEG > 2) {
                const float3 s9 = f3(sh + 27), s10 = f3(sh + 30), s11 = f3(sh + 33), s12 = f3(sh + 36),
                             s13 = f3(sh + 39), s14 = f3(sh + 42), s15 = f3(sh + 45);
                dx = dx + (SH_C3[0] * 3.f * 2.f * xy) * s9 + (SH_C3[1] * yz) * s10 + (SH_C3[2] * -2.f * xy) * s11 +
                     (SH_C3[3] * -3.f * 2.f * xz) * s12 + (SH_C3[4] * (-3.f * xx + 4.f * zz - yy)) * s13 +
                     (SH_C3[5] * 2.f * xz) * s14 + (SH_C3[6] * 3.f * (xx - yy)) * s15;
                dy = dy + (SH_C3[0] * 3.f * (xx - yy)) * s9 + (SH_C3[1] * xz) * s10 +
                     (SH_C3[2] * (-3.f * yy + 4.f * zz - xx)) * s11 + (SH_C3[3] * -3.f * 2.f * yz) * s12 +
                     (SH_C3[4] * -2.f * xy) * s13 + (SH_C3[5] * -2.f * yz) * s14 + (SH_C3[6] * -3.f * 2.f * xy) * s15;
                dz = dz + (SH_C3[1] * xy) * s10 + (SH_C3[2] * 4.f * 2.f * yz) * s11 +
                     (SH_C3[3] * 3.f * (2.f * zz - xx - yy)) * s12 + (SH_C3[4] * 4.f * 2.f * xz) * s13 +
                     (SH_C3[5] * (xx - yy)) * s14;
            }
        }
    }
    // every read precedes the first write (the compiler cannot reorder them: same buffer)
    float *dsh = sh_io;
    const float3 zero = make_float3(0, 0, 0);
    st3(dsh, GSR_SH_C0 * dRGB);
    st3(dsh + 3, DEG > 0 ? (-GSR_SH_C1 * y) * dRGB : zero);
    st3(dsh + 6, DEG > 0 ? (GSR_SH_C1 * z) * dRGB : zero);
    st3(dsh + 9, DEG > 0 ? (-GSR_SH_C1 * x) * dRGB : zero);
    st3(dsh + 12, DEG > 1 ? (SH_C2[0] * xy) * dRGB : zero);
    st3(dsh + 15, DEG > 1 ? (SH_C2[1] * yz) * dRGB : zero);
    st3(dsh + 18, DEG > 1 ? (SH_C2[2] * (2.f * zz - xx - yy)) * dRGB : zero);
    st3(dsh + 21, DEG > 1 ? (SH_C2[3] * xz) * dRGB : zero);
    st3(dsh + 24, DEG > 1 ? (SH_C2[4] * (xx - yy)) * dRGB : zero);
    st3(dsh + 27, DEG > 2 ? (SH_C3[0] * y * (3.f * xx - yy)) * dRGB : zero);
    st3(dsh + 30, DEG > 2 ? (SH_C3[1] * xy * z) * dRGB : zero);
    st3(dsh + 33, DEG > 2 ? (SH_C3[2] * y * (4.f * zz - xx - yy)) * dRGB : zero);
    st3(dsh + 36, DEG > 2 ? (SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy)) * dRGB : zero);
    st3(dsh + 39, DEG > 2 ? (SH_C3[4] * x * (4.f * zz - xx - yy)) * dRGB : zero);
    st3(dsh + 42, DEG > 2 ? (SH_C3[5] * z * (xx - yy)) * dRGB : zero);
    st3(dsh + 45, DEG > 2 ? (SH_C3[6] * x * (xx - 3.f * yy)) * dRGB : zero);
    const float3 dL_ddir = make_float3(dot3(dx, dRGB), dot3(dy, dRGB), dot3(dz, dRGB));
    return dnormvdv(dir_orig, dL_ddir);
}
__device__ __forceinline__ float3 sh_backward_inplace_dispatch(int deg, float *sh_io, float3 dir_orig, float3 dRGB) {
    switch (deg) {
        case 0: return sh_backward_inplace<0>(sh_io, dir_orig, dRGB);
        case 1: return sh_backward_inplace<1>(sh_io, dir_orig, dRGB);
        case 2: return sh_backward_inplace<2>(sh_io, dir_orig, dRGB);
        default: return sh_backward_inplace<3>(sh_io, dir_orig, dRGB);
    }
}

// dL/dsh = basis(dir) (x) dRGB at the normalised direction of dir_orig: dsh[0..48), zeros above the degree (the
// same values as sh_backward_inplace writes).
template <int DEG>
__device__ __forceinline__ void sh_dsh(float3 dir_orig, float3 dRGB, float *__restrict__ dsh) {
    const float len = sqrtf(dot3(dir_orig, dir_orig));
    const float3 dir = make_float3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
    const float x = dir.x, y = dir.y, z = dir.z;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    const float3 zero = make_float3(0, 0, 0);
    st3(dsh, GSR_SH_C0 * dRGB);
    st3(dsh + 3, DEG > 0 ? (-GSR_SH_C1 * y) * dRGB : zero);
    st3(dsh + 6, DEG > 0 ? (GSR_SH_C1 * z) * dRGB : zero);
    st3(dsh + 9, DEG > 0 ? (-GSR_SH_C1 * x) * dRGB : zero);
    st3(dsh + 12, DEG > 1 ? (SH_C2[0] * xy) * dRGB : zero);
    st3(dsh + 15, DEG > 1 ? (SH_C2[1] * yz) * dRGB : zero);
    st3(dsh + 18, DEG > 1 ? (SH_C2[2] * (2.f * zz - xx - yy)) * dRGB : zero);
    st3(dsh + 21, DEG > 1 ? (SH_C2[3] * xz) * dRGB : zero);
    st3(dsh + 24, DEG > 1 ? (SH_C2[4] * (xx - yy)) * dRGB : zero);
    st3(dsh + 27, DEG > 2 ? (SH_C3[0] * y * (3.f * xx - yy)) * dRGB : zero);
    st3(dsh + 30, DEG > 2 ? (SH_C3[1] * xy * z) * dRGB : zero);
    st3(dsh + 33, DEG > 2 ? (SH_C3[2] * y * (4.f * zz - xx - yy)) * dRGB : zero);
    st3(dsh + 36, DEG > 2 ? (SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy)) * dRGB : zero);
    st3(dsh + 39, DEG > 2 ? (SH_C3[4] * x * (4.f * zz - xx - yy)) * dRGB : zero);
    st3(dsh + 42, DEG > 2 ? (SH_C3[5] * z * (xx - yy)) * dRGB : zero);
    st3(dsh + 45, DEG > 2 ? (SH_C3[6] * x * (xx - 3.f * yy)) * dRGB : zero);
}
__device__ __forceinline__ void sh_dsh_dispatch(int deg, float3 dir_orig, float3 dRGB, float *dsh) {
    switch (deg) {
        case 0: sh_dsh<0>(dir_orig, dRGB, dsh); break;
        case 1: sh_dsh<1>(dir_orig, dRGB, dsh); break;
        case 2: sh_dsh<2>(dir_orig, dRGB, dsh); break;
        default: sh_dsh<3>(dir_orig, dRGB, dsh); break;
    }
}

// The direction term of dL/dmean from the forward's colour Jacobian: dL/ddir = (jx . dRGB, jy . dRGB, jz . dRGB)
// through the normalisation (sh_backward's last two lines); no coefficient is read.
__device__ __forceinline__ float3 sh_dir_grad(float3 dir_orig, float3 dRGB, float3 jx, float3 jy, float3 jz) {
    const float3 dL_ddir = make_float3(dot3(jx, dRGB), dot3(jy, dRGB), dot3(jz, dRGB));
    return dnormvdv(dir_orig, dL_ddir);
}

// Both: the non-staged backward path (dL/dsh into registers or global memory).
template <int DEG>
__device__ __forceinline__ float3 sh_backward_jac(float3 dir_orig, float3 dRGB, float3 jx, float3 jy, float3 jz,
                                                  float *__restrict__ dsh) {
    sh_dsh<DEG>(dir_orig, dRGB, dsh);
    return sh_dir_grad(dir_orig, dRGB, jx, jy, jz);
}
__device__ __forceinline__ float3 sh_backward_jac_dispatch(int deg, float3 dir_orig, float3 dRGB, float3 jx, float3 jy,
                                                           float3 jz, float *dsh) {
    switch (deg) {
        case 0: return sh_backward_jac<0>(dir_orig, dRGB, jx, jy, jz, dsh);
        case 1: return sh_backward_jac<1>(dir_orig, dRGB, jx, jy, jz, dsh);
        case 2: return sh_backward_jac<2>(dir_orig, dRGB, jx, jy, jz, dsh);
        default: return sh_backward_jac<3>(dir_orig, dRGB, jx, jy, jz, dsh);
    }
}

// SH basis values b[0..(DEG+1)^2) at unit direction (x,y,z); b[k] * dRGB is sh_backward's dL/dsh[k].
template <int DEG>
__device__ __forceinline__ void sh_basis(float x, float y, float z, float *b) {
#pragma clang fp contract(off)  // the same bits in every kernel that inlines it (the expansion and the fused SH Adam)
    b[0] = GSR_SH_C0;
    if (DEG > 0) {
        b[1] = -GSR_SH_C1 * y;
        b[2] = GSR_SH_C1 * z;
        b[3] = -GSR_SH_C1 * x;
        if (DEG > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            b[4] = SH_C2[0] * xy;
            b[5] = SH_C2[1] * yz;
            b[6] = SH_C2[2] * (2.f * zz - xx - yy);
            b[7] = SH_C2[3] * xz;
            b[8] = SH_C2[4] * (xx - yy);
            if (DEG > 2) {
                b[9] = SH_C3[0] * y * (3.f * xx - yy);
                b[10] = SH_C3[1] * xy * z;
                b[11] = SH_C3[2] * y * (4.f * zz - xx - yy);
                b[12] = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                b[13] = SH_C3[4] * x * (4.f * zz - xx - yy);
                b[14] = SH_C3[5] * z * (xx - yy);
                b[15] = SH_C3[6] * x * (xx - 3.f * yy);
            }
        }
    }
}

__device__ __forceinline__ float3 sh_backward_dispatch(int deg, const float *__restrict__ sh, float3 dir_orig,
                                                       float3 dRGB, float *__restrict__ dsh) {
    switch (deg) {
        case 0: return sh_backward<0>(sh, dir_orig, dRGB, dsh);
        case 1: return sh_backward<1>(sh, dir_orig, dRGB, dsh);
        case 2: return sh_backward<2>(sh, dir_orig, dRGB, dsh);
        default: return sh_backward<3>(sh, dir_orig, dRGB, dsh);
    }
}

}  // namespace gsr
