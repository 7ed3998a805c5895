// gs_device.cuh -- device-side helpers shared by the gfx950 kernels.
//
// Arithmetic contract (see DESIGN.md "Parity policy"): everything that feeds
// the tile keys (depth bits, means2D, radius) is evaluated in the exact
// operation order of the reference with FMA contraction OFF (the library is
// compiled with -ffp-contract=off; blend loops opt back in locally with
// `#pragma clang fp contract(fast)`).  Matrix products expand glm's
// column-major operator* (glm/detail/type_mat3x3.inl:486-520).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsamd {

constexpr int kChannels = 3;
constexpr int kWave = 64;

// Loads of per-Gaussian inputs a pass reads exactly once; kNt: with the
// non-temporal hint (the lines are not kept in L2 for reuse).
template <bool kNt>
__device__ __forceinline__ float ldg1(const float* p) {
    if constexpr (kNt) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool kNt>
__device__ __forceinline__ float4 ldg4(const float4* p) {
    if constexpr (kNt) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}

// base/cr/auxiliary.h:22-39
__device__ constexpr float SH_C0 = 0.28209479177387814f;
__device__ constexpr float SH_C1 = 0.4886025119029199f;
__device__ constexpr float SH_C2_0 = 1.0925484305920792f;
__device__ constexpr float SH_C2_1 = -1.0925484305920792f;
__device__ constexpr float SH_C2_2 = 0.31539156525252005f;
__device__ constexpr float SH_C2_3 = -1.0925484305920792f;
__device__ constexpr float SH_C2_4 = 0.5462742152960396f;
__device__ constexpr float SH_C3_0 = -0.5900435899266435f;
__device__ constexpr float SH_C3_1 = 2.890611442640554f;
__device__ constexpr float SH_C3_2 = -0.4570457994644658f;
__device__ constexpr float SH_C3_3 = 0.3731763325901154f;
__device__ constexpr float SH_C3_4 = -0.4570457994644658f;
__device__ constexpr float SH_C3_5 = 1.445305721320277f;
__device__ constexpr float SH_C3_6 = -0.5900435899266435f;

// computeColorFromSH backward (base/cr/backward.cu:20-139), split in two:
// sh_basis -- the per-coefficient factors (dL_dsh[k][c] = basis[k] dL_drgb[c]),
// a function of the view direction alone -- and sh_ddir -- d(rgb)/d(dir)
// (dx3, dy3, dz3 per channel), which needs the coefficients.  The forward's
// preprocess stores sh_ddir for the backward (GeomView::drgb), so the
// backward reads 36 B per visible Gaussian instead of the 192-B SH row.
__device__ __forceinline__ void sh_basis(int deg, float x, float y, float z, float (&dsh_c)[16]) {
#pragma unroll
    for (int k = 0; k < 16; k++) dsh_c[k] = 0.f;
    dsh_c[0] = SH_C0;
    if (deg > 0) {
        dsh_c[1] = -SH_C1 * y;
        dsh_c[2] = SH_C1 * z;
        dsh_c[3] = -SH_C1 * x;
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            dsh_c[4] = SH_C2_0 * xy;
            dsh_c[5] = SH_C2_1 * yz;
            dsh_c[6] = SH_C2_2 * (2.f * zz - xx - yy);
            dsh_c[7] = SH_C2_3 * xz;
            dsh_c[8] = SH_C2_4 * (xx - yy);
            if (deg > 2) {
                dsh_c[9] = SH_C3_0 * y * (3.f * xx - yy);
                dsh_c[10] = SH_C3_1 * xy * z;
                dsh_c[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
                dsh_c[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
                dsh_c[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
                dsh_c[14] = SH_C3_5 * z * (xx - yy);
                dsh_c[15] = SH_C3_6 * x * (xx - 3.f * yy);
            }
        }
    }
}

template <typename SH>
__device__ __forceinline__ void sh_ddir(int deg, const SH& s, float x, float y, float z, float (&dx3)[3],
                                        float (&dy3)[3], float (&dz3)[3]) {
#pragma unroll
    for (int c = 0; c < 3; c++) dx3[c] = dy3[c] = dz3[c] = 0.f;
    if (deg > 0) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            dx3[c] = -SH_C1 * s[3][c];
            dy3[c] = -SH_C1 * s[1][c];
            dz3[c] = SH_C1 * s[2][c];
        }
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                dx3[c] += SH_C2_0 * y * s[4][c] + SH_C2_2 * 2.f * -x * s[6][c] + SH_C2_3 * z * s[7][c] +
                          SH_C2_4 * 2.f * x * s[8][c];
                dy3[c] += SH_C2_0 * x * s[4][c] + SH_C2_1 * z * s[5][c] + SH_C2_2 * 2.f * -y * s[6][c] +
                          SH_C2_4 * 2.f * -y * s[8][c];
                dz3[c] += SH_C2_1 * y * s[5][c] + SH_C2_2 * 2.f * 2.f * z * s[6][c] + SH_C2_3 * x * s[7][c];
            }
            if (deg > 2) {
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    dx3[c] += (SH_C3_0 * s[9][c] * 3.f * 2.f * xy + SH_C3_1 * s[10][c] * yz +
                               SH_C3_2 * s[11][c] * -2.f * xy + SH_C3_3 * s[12][c] * -3.f * 2.f * xz +
                               SH_C3_4 * s[13][c] * (-3.f * xx + 4.f * zz - yy) + SH_C3_5 * s[14][c] * 2.f * xz +
                               SH_C3_6 * s[15][c] * 3.f * (xx - yy));
                    dy3[c] += (SH_C3_0 * s[9][c] * 3.f * (xx - yy) + SH_C3_1 * s[10][c] * xz +
                               SH_C3_2 * s[11][c] * (-3.f * yy + 4.f * zz - xx) +
                               SH_C3_3 * s[12][c] * -3.f * 2.f * yz + SH_C3_4 * s[13][c] * -2.f * xy +
                               SH_C3_5 * s[14][c] * -2.f * yz + SH_C3_6 * s[15][c] * -3.f * 2.f * xy);
                    dz3[c] += (SH_C3_1 * s[10][c] * xy + SH_C3_2 * s[11][c] * 4.f * 2.f * yz +
                               SH_C3_3 * s[12][c] * 3.f * (2.f * zz - xx - yy) + SH_C3_4 * s[13][c] * 4.f * 2.f * xz +
                               SH_C3_5 * s[14][c] * (xx - yy));
                }
            }
        }
    }
}

// Column-major 3x3 (glm convention: m[c][r]).
struct Mat3 {
    float m[3][3];
};

__device__ __forceinline__ Mat3 mat3_cols(float a0, float a1, float a2, float a3, float a4, float a5,
                                          float a6, float a7, float a8) {
    Mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}

__device__ __forceinline__ Mat3 mat3_mul(const Mat3& A, const Mat3& B) {
    Mat3 R;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++)
            R.m[c][r] = A.m[0][r] * B.m[c][0] + A.m[1][r] * B.m[c][1] + A.m[2][r] * B.m[c][2];
    return R;
}

__device__ __forceinline__ Mat3 mat3_transpose(const Mat3& A) {
    Mat3 R;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++) R.m[c][r] = A.m[r][c];
    return R;
}

__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    float t0 = a0 * b0, t1 = a1 * b1, t2 = a2 * b2;
    return t0 + t1 + t2;
}

// Quaternion (r,x,y,z) -> R, un-normalised as in base/cr/forward.cu:127-138.
__device__ __forceinline__ Mat3 quat_to_R(float r, float x, float y, float z) {
    return mat3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                     2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                     2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
}

// computeCov3D (base/cr/forward.cu:118-152): Sigma = (S R)^T (S R), upper
// triangle.  Shared by the forward preprocess and the multi-view backward so
// both see the same bits.
__device__ __forceinline__ void compute_cov3d(const float (&sc)[3], float4 q, float mod, float (&cov3D)[6]) {
    Mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * sc[0];
    S.m[1][1] = mod * sc[1];
    S.m[2][2] = mod * sc[2];
    const Mat3 R = quat_to_R(q.x, q.y, q.z, q.w);
    const Mat3 Mm = mat3_mul(S, R);
    const Mat3 Sigma = mat3_mul(mat3_transpose(Mm), Mm);
    cov3D[0] = Sigma.m[0][0]; cov3D[1] = Sigma.m[0][1]; cov3D[2] = Sigma.m[0][2];
    cov3D[3] = Sigma.m[1][1]; cov3D[4] = Sigma.m[1][2]; cov3D[5] = Sigma.m[2][2];
}

// 4x4 matrices as 16 floats, column-major like the reference (auxiliary.h:58-77).
struct Mat4 {
    float m[16];
};

__device__ __forceinline__ Mat4 load_mat4(const float* __restrict__ p) {
    Mat4 r;
#pragma unroll
    for (int i = 0; i < 16; i++) r.m[i] = p[i];
    return r;
}

__device__ __forceinline__ float3 transform_point_4x3(float x, float y, float z, const Mat4& M) {
    const float* m = M.m;
    return make_float3(m[0] * x + m[4] * y + m[8] * z + m[12], m[1] * x + m[5] * y + m[9] * z + m[13],
                       m[2] * x + m[6] * y + m[10] * z + m[14]);
}

__device__ __forceinline__ float4 transform_point_4x4(float x, float y, float z, const Mat4& M) {
    const float* m = M.m;
    return make_float4(m[0] * x + m[4] * y + m[8] * z + m[12], m[1] * x + m[5] * y + m[9] * z + m[13],
                       m[2] * x + m[6] * y + m[10] * z + m[14], m[3] * x + m[7] * y + m[11] * z + m[15]);
}

// base/cr/auxiliary.h:41-44: the double literals promote the whole expression.
__device__ __forceinline__ float ndc2pix(float v, int S) {
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

struct Rect {
    uint32_t x0, y0, x1, y1;
};

// base/cr/auxiliary.h:46-56 (tile size as template-free runtime args; the
// division by a power of two is exact in either form).
__device__ __forceinline__ Rect get_rect(float px, float py, int max_radius, int bx, int by, uint32_t gx,
                                         uint32_t gy) {
    const float fr = (float)max_radius;
    int a = (int)((px - fr) / (float)bx);
    int b = (int)((py - fr) / (float)by);
    int c = (int)(((px + fr) + (float)bx - 1.0f) / (float)bx);
    int d = (int)(((py + fr) + (float)by - 1.0f) / (float)by);
    a = max(a, 0); b = max(b, 0); c = max(c, 0); d = max(d, 0);
    Rect r;
    r.x0 = min(gx, (uint32_t)a);
    r.y0 = min(gy, (uint32_t)b);
    r.x1 = min(gx, (uint32_t)c);
    r.y1 = min(gy, (uint32_t)d);
    return r;
}

__device__ __forceinline__ uint32_t float_bits(float f) { return __float_as_uint(f); }

// ---------------------------------------------------------------- wave ops
// Sum across the 64 lanes of a wave; every lane gets the total.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

}  // namespace gsamd
