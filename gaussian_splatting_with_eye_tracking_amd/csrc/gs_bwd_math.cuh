// gs_bwd_math.cuh -- the per-Gaussian backward's math (computeColorFromSH,
// computeCov2DCUDA, projection and computeCov3D backward of
// base/cr/backward.cu:20-396), shared by the single-view backward
// (backward.hip) and the multi-view backward (multiview.hip, compiled with
// contraction and reciprocal math: its gradients are held to a tolerance).
#pragma once

#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

// One thread per Gaussian (backward_gaussian_body).  With SH16 the 192-B SH
// gradient rows are staged in LDS (49-float rows: conflict-free per-thread
// writes) and the workgroup stores its contiguous 256 x 192 B with
// wave-contiguous 16-B stores: per-thread 192-B row stores measured ~3.5 TB/s
// against ~5.4 TB/s coalesced on MI355X (tools/membench.hip).
constexpr int kShRow = 49;

__device__ __forceinline__ void dnormvdv3(float vx, float vy, float vz, float dx, float dy, float dz, float& ox,
                                          float& oy, float& oz) {
    // base/cr/auxiliary.h:107-117
    const float sum2 = vx * vx + vy * vy + vz * vz;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    ox = ((+sum2 - vx * vx) * dx - vy * vx * dy - vz * vx * dz) * invsum32;
    oy = (-vx * vy * dx + (sum2 - vy * vy) * dy - vz * vy * dz) * invsum32;
    oz = (-vx * vz * dx - vy * vz * dy + (sum2 - vz * vz) * dz) * invsum32;
}

// SH rows of Gaussian idx into s[16][3] (zero past (D+1)^2 and M).
template <bool kSH16>
__device__ __forceinline__ void load_sh_rows(const BackwardGaussArgs& a, int idx, float (&s)[16][3],
                                             const float* lrow = nullptr) {
    const int ncoef = min((a.D + 1) * (a.D + 1), a.M);
    const float* sh = a.shs + (size_t)idx * a.M * 3;
    if (kSH16 && lrow) {  // row staged in LDS by the workgroup's coalesced load
#pragma unroll
        for (int k = 0; k < 16; k++)
#pragma unroll
            for (int c = 0; c < 3; c++) s[k][c] = (k < ncoef) ? lrow[3 * k + c] : 0.f;
    } else if (kSH16) {
        const float4* s4 = reinterpret_cast<const float4*>(sh);
        float buf[48];
#pragma unroll
        for (int i = 0; i < 12; i++) {
            const float4 v4 = (i * 4 < ncoef * 3) ? s4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            buf[4 * i + 0] = v4.x; buf[4 * i + 1] = v4.y; buf[4 * i + 2] = v4.z; buf[4 * i + 3] = v4.w;
        }
#pragma unroll
        for (int k = 0; k < 16; k++)
#pragma unroll
            for (int c = 0; c < 3; c++) s[k][c] = buf[3 * k + c];
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++)
#pragma unroll
            for (int c = 0; c < 3; c++) s[k][c] = (k < ncoef) ? sh[3 * k + c] : 0.f;
    }
}

// computeColorFromSH backward (backward.cu:20-139), shared part: the
// per-coefficient factors dsh_c[k] (dL_dsh[k][c] = dsh_c[k] * dRGB[c])
// and the view-direction term added to dmean (+=).
// (SH: float[16][3] in registers, or ShRowPtr, a row of 48 coefficients in LDS.)
struct ShRowPtr {
    const float* p;
    __device__ __forceinline__ const float* operator[](int k) const { return p + 3 * k; }
};

template <typename SH>
__device__ __forceinline__ void sh_backward_terms(int deg, const float* campos, float mx, float my, float mz,
                                                  const SH& s, uint8_t cb, const float* acc,
                                                  float (&dsh_c)[16], float (&dRGB)[3], float (&dmean)[3],
                                                  const float* drgb9 = nullptr) {
    const float dox = mx - campos[0], doy = my - campos[1], doz = mz - campos[2];
    const float len = sqrtf(dot3(dox, doy, doz, dox, doy, doz));
    const float x = dox / len, y = doy / len, z = doz / len;
#pragma unroll
    for (int c = 0; c < 3; c++) dRGB[c] = acc[c] * (((cb >> c) & 1) ? 0.0f : 1.0f);
    float dx3[3], dy3[3], dz3[3];
    sh_basis(deg, x, y, z, dsh_c);
    if (drgb9) {  // the forward's derivatives (sh_ddir on the same operands: the same bits)
#pragma unroll
        for (int c = 0; c < 3; c++) {
            dx3[c] = drgb9[c];
            dy3[c] = drgb9[3 + c];
            dz3[c] = drgb9[6 + c];
        }
    } else {
        sh_ddir(deg, s, x, y, z, dx3, dy3, dz3);
    }
    const float ddx = dot3(dx3[0], dx3[1], dx3[2], dRGB[0], dRGB[1], dRGB[2]);
    const float ddy = dot3(dy3[0], dy3[1], dy3[2], dRGB[0], dRGB[1], dRGB[2]);
    const float ddz = dot3(dz3[0], dz3[1], dz3[2], dRGB[0], dRGB[1], dRGB[2]);
    float ox, oy, oz;
    dnormvdv3(dox, doy, doz, ddx, ddy, ddz, ox, oy, oz);
    dmean[0] += ox;
    dmean[1] += oy;
    dmean[2] += oz;
}

// computeColorFromSH backward (backward.cu:20-139) for one Gaussian: writes
// its dL_dsh row and adds the view-direction term to dmean (+=, after the
// cov2D (=) and projection (+=) terms, the reference's order).
template <bool kSH16>
__device__ __forceinline__ void sh_backward(const BackwardGaussArgs& a, int idx, float mx, float my, float mz,
                                            const float (&s)[16][3], uint8_t cb, const float* acc,
                                            float (&dmean)[3], float* lrow = nullptr, const float* drgb9 = nullptr) {
    const int ncoef = min((a.D + 1) * (a.D + 1), a.M);
    float* dsh = a.dL_dsh + (size_t)idx * a.M * 3;
    float dsh_c[16], dRGB[3];
    sh_backward_terms(a.D, a.campos, mx, my, mz, s, cb, acc, dsh_c, dRGB, dmean, drgb9);
    if (kSH16) {
        float o[48];
#pragma unroll
        for (int k = 0; k < 16; k++)
#pragma unroll
            for (int c = 0; c < 3; c++) o[3 * k + c] = (k < ncoef) ? dsh_c[k] * dRGB[c] : 0.f;
#pragma unroll
        for (int i = 0; i < 12; i++)
            if (lrow) {  // staged in LDS; the workgroup stores its rows coalesced
#pragma unroll
                for (int e = 0; e < 4; e++) lrow[4 * i + e] = o[4 * i + e];
            } else {
                reinterpret_cast<float4*>(dsh)[i] = make_float4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
            }
    } else {
        for (int k = 0; k < a.M; k++)
#pragma unroll
            for (int c = 0; c < 3; c++) {
                float v = 0.f;
#pragma unroll
                for (int kk = 0; kk < 16; kk++) v = (kk == k && k < ncoef) ? dsh_c[kk] * dRGB[c] : v;
                dsh[3 * k + c] = v;
            }
    }
}

// computeCov2DCUDA backward (backward.cu:144-274) for one Gaussian and one
// view: dL_dconic (x, y, w) -> dmean (assigned, `=`) and dL_dcov3D.
__device__ __forceinline__ void cov2d_backward(float mx, float my, float mz, const float (&cov3D)[6],
                                               float dcx, float dcy, float dcz, const Mat4& V, float h_x, float h_y,
                                               float tan_fovx, float tan_fovy, float (&dmean)[3], float (&dcov)[6]) {
    float3 t = transform_point_4x3(mx, my, mz, V);
    const float limx = 1.3f * tan_fovx;
    const float limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
    const Mat3 J = mat3_cols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z,
                             -(h_y * t.y) / (t.z * t.z), 0, 0, 0);
    const float* v = V.m;
    const Mat3 Wm = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    const Mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4],
                               cov3D[5]);
    const Mat3 T = mat3_mul(Wm, J);
    Mat3 cov2D = mat3_mul(mat3_mul(mat3_transpose(T), mat3_transpose(Vrk)), T);
    const float aa = cov2D.m[0][0] += 0.3f;
    const float bb = cov2D.m[0][1];
    const float cc = cov2D.m[1][1] += 0.3f;
    const float denom = aa * cc - bb * bb;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const auto& Tm = T.m;
    const auto& Vm = Vrk.m;
    // (the reference's `if (denom2inv != 0)` as selects on the same
    // expressions -- the same values; as a branch, the compiler sank the two
    // paths' dcov stores into a pointer phi and kept dcov in scratch memory)
    const bool ok = denom2inv != 0;
    const float dL_da = ok ? denom2inv * (-cc * cc * dcx + 2 * bb * cc * dcy + (denom - aa * cc) * dcz) : 0.f;
    const float dL_dc = ok ? denom2inv * (-aa * aa * dcz + 2 * aa * bb * dcy + (denom - aa * cc) * dcx) : 0.f;
    const float dL_db = ok ? denom2inv * 2 * (bb * cc * dcx - (denom + 2 * bb * bb) * dcy + aa * bb * dcz) : 0.f;
    dcov[0] = ok ? (Tm[0][0] * Tm[0][0] * dL_da + Tm[0][0] * Tm[1][0] * dL_db + Tm[1][0] * Tm[1][0] * dL_dc) : 0.f;
    dcov[3] = ok ? (Tm[0][1] * Tm[0][1] * dL_da + Tm[0][1] * Tm[1][1] * dL_db + Tm[1][1] * Tm[1][1] * dL_dc) : 0.f;
    dcov[5] = ok ? (Tm[0][2] * Tm[0][2] * dL_da + Tm[0][2] * Tm[1][2] * dL_db + Tm[1][2] * Tm[1][2] * dL_dc) : 0.f;
    dcov[1] = ok ? 2 * Tm[0][0] * Tm[0][1] * dL_da + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_db +
                       2 * Tm[1][0] * Tm[1][1] * dL_dc
                 : 0.f;
    dcov[2] = ok ? 2 * Tm[0][0] * Tm[0][2] * dL_da + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_db +
                       2 * Tm[1][0] * Tm[1][2] * dL_dc
                 : 0.f;
    dcov[4] = ok ? 2 * Tm[0][2] * Tm[0][1] * dL_da + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_db +
                       2 * Tm[1][1] * Tm[1][2] * dL_dc
                 : 0.f;
    const float dL_dT00 = 2 * (Tm[0][0] * Vm[0][0] + Tm[0][1] * Vm[0][1] + Tm[0][2] * Vm[0][2]) * dL_da +
                          (Tm[1][0] * Vm[0][0] + Tm[1][1] * Vm[0][1] + Tm[1][2] * Vm[0][2]) * dL_db;
    const float dL_dT01 = 2 * (Tm[0][0] * Vm[1][0] + Tm[0][1] * Vm[1][1] + Tm[0][2] * Vm[1][2]) * dL_da +
                          (Tm[1][0] * Vm[1][0] + Tm[1][1] * Vm[1][1] + Tm[1][2] * Vm[1][2]) * dL_db;
    const float dL_dT02 = 2 * (Tm[0][0] * Vm[2][0] + Tm[0][1] * Vm[2][1] + Tm[0][2] * Vm[2][2]) * dL_da +
                          (Tm[1][0] * Vm[2][0] + Tm[1][1] * Vm[2][1] + Tm[1][2] * Vm[2][2]) * dL_db;
    const float dL_dT10 = 2 * (Tm[1][0] * Vm[0][0] + Tm[1][1] * Vm[0][1] + Tm[1][2] * Vm[0][2]) * dL_dc +
                          (Tm[0][0] * Vm[0][0] + Tm[0][1] * Vm[0][1] + Tm[0][2] * Vm[0][2]) * dL_db;
    const float dL_dT11 = 2 * (Tm[1][0] * Vm[1][0] + Tm[1][1] * Vm[1][1] + Tm[1][2] * Vm[1][2]) * dL_dc +
                          (Tm[0][0] * Vm[1][0] + Tm[0][1] * Vm[1][1] + Tm[0][2] * Vm[1][2]) * dL_db;
    const float dL_dT12 = 2 * (Tm[1][0] * Vm[2][0] + Tm[1][1] * Vm[2][1] + Tm[1][2] * Vm[2][2]) * dL_dc +
                          (Tm[0][0] * Vm[2][0] + Tm[0][1] * Vm[2][1] + Tm[0][2] * Vm[2][2]) * dL_db;
    const auto& Wq = Wm.m;
    const float dL_dJ00 = Wq[0][0] * dL_dT00 + Wq[0][1] * dL_dT01 + Wq[0][2] * dL_dT02;
    const float dL_dJ02 = Wq[2][0] * dL_dT00 + Wq[2][1] * dL_dT01 + Wq[2][2] * dL_dT02;
    const float dL_dJ11 = Wq[1][0] * dL_dT10 + Wq[1][1] * dL_dT11 + Wq[1][2] * dL_dT12;
    const float dL_dJ12 = Wq[2][0] * dL_dT10 + Wq[2][1] * dL_dT11 + Wq[2][2] * dL_dT12;
    const float tz = 1.f / t.z;
    const float tz2 = tz * tz;
    const float tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    const float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    const float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 +
                         (2 * h_y * t.y) * tz3 * dL_dJ12;
    // transformVec4x3Transpose (auxiliary.h:89-97): assign (=)
    dmean[0] = v[0] * dL_dtx + v[1] * dL_dty + v[2] * dL_dtz;
    dmean[1] = v[4] * dL_dtx + v[5] * dL_dty + v[6] * dL_dtz;
    dmean[2] = v[8] * dL_dtx + v[9] * dL_dty + v[10] * dL_dtz;
}

// preprocessCUDA backward, projection part (backward.cu:370-387): adds
// (+=) the mean2D gradient (gx, gy) pulled back through the projection.
__device__ __forceinline__ void proj_backward(float mx, float my, float mz, const Mat4& Pm, float gx, float gy,
                                              float (&dmean)[3]) {
    const float* proj = Pm.m;
    const float4 m_hom = transform_point_4x4(mx, my, mz, Pm);
    const float m_w = 1.0f / (m_hom.w + 0.0000001f);
    const float mul1 = (proj[0] * mx + proj[4] * my + proj[8] * mz + proj[12]) * m_w * m_w;
    const float mul2 = (proj[1] * mx + proj[5] * my + proj[9] * mz + proj[13]) * m_w * m_w;
    dmean[0] += (proj[0] * m_w - proj[3] * mul1) * gx + (proj[1] * m_w - proj[3] * mul2) * gy;
    dmean[1] += (proj[4] * m_w - proj[7] * mul1) * gx + (proj[5] * m_w - proj[7] * mul2) * gy;
    dmean[2] += (proj[8] * m_w - proj[11] * mul1) * gx + (proj[9] * m_w - proj[11] * mul2) * gy;
}

// computeCov3D backward (backward.cu:278-341): dL_dcov3D -> dL_dscale and
// dL_drot (w.r.t. the unnormalised quaternion, as the reference).
__device__ __forceinline__ void cov3d_backward(float4 qrot, const float (&scl)[3], float scale_modifier,
                                               const float (&dcov)[6], float (&dscale)[3], float4& dq) {
    const float r = qrot.x, x = qrot.y, y = qrot.z, z = qrot.w;
    const Mat3 R = quat_to_R(r, x, y, z);
    const float sx = scale_modifier * scl[0];
    const float sy = scale_modifier * scl[1];
    const float sz = scale_modifier * scl[2];
    Mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = sx; S.m[1][1] = sy; S.m[2][2] = sz;
    const Mat3 Mm = mat3_mul(S, R);
    const float* dc = dcov;
    const Mat3 dL_dSigma = mat3_cols(dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4],
                                     0.5f * dc[2], 0.5f * dc[4], dc[5]);
    Mat3 M2;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++) M2.m[c][rr] = 2.0f * Mm.m[c][rr];
    const Mat3 dL_dM = mat3_mul(M2, dL_dSigma);
    const Mat3 Rt = mat3_transpose(R);
    Mat3 D = mat3_transpose(dL_dM);
    dscale[0] = dot3(Rt.m[0][0], Rt.m[0][1], Rt.m[0][2], D.m[0][0], D.m[0][1], D.m[0][2]);
    dscale[1] = dot3(Rt.m[1][0], Rt.m[1][1], Rt.m[1][2], D.m[1][0], D.m[1][1], D.m[1][2]);
    dscale[2] = dot3(Rt.m[2][0], Rt.m[2][1], Rt.m[2][2], D.m[2][0], D.m[2][1], D.m[2][2]);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        D.m[0][k] *= sx;
        D.m[1][k] *= sy;
        D.m[2][k] *= sz;
    }
    const auto& Dm = D.m;
    dq.x = 2 * z * (Dm[0][1] - Dm[1][0]) + 2 * y * (Dm[2][0] - Dm[0][2]) + 2 * x * (Dm[1][2] - Dm[2][1]);
    dq.y = 2 * y * (Dm[1][0] + Dm[0][1]) + 2 * z * (Dm[2][0] + Dm[0][2]) + 2 * r * (Dm[1][2] - Dm[2][1]) -
           4 * x * (Dm[2][2] + Dm[1][1]);
    dq.z = 2 * x * (Dm[1][0] + Dm[0][1]) + 2 * r * (Dm[2][0] - Dm[0][2]) + 2 * z * (Dm[1][2] + Dm[2][1]) -
           4 * y * (Dm[2][2] + Dm[0][0]);
    dq.w = 2 * r * (Dm[0][1] - Dm[1][0]) + 2 * x * (Dm[2][0] + Dm[0][2]) + 2 * y * (Dm[1][2] + Dm[2][1]) -
           4 * z * (Dm[1][1] + Dm[0][0]);
}

// A 16-B store of an output nothing in this pass reads back; nt: with the
// non-temporal hint (the line is not kept in L2 for reuse).
__device__ __forceinline__ void store_out4(float4* p, float4 v, bool nt) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    if (nt) __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p));
    else *p = v;
}
__device__ __forceinline__ void store_out1(float* p, float v, bool nt) {
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

}  // namespace gsamd
