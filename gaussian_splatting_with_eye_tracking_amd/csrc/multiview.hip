// multiview.hip -- the data-parallel view exchange: view
// records (pack_view_grads) and the multi-view per-Gaussian backward.
// Compiled with -ffp-contract=fast -freciprocal-math (build.py
// FAST_MATH_SOURCES): 30 % fewer VALU instructions per view than the
// IEEE-exact expansion, gradients within the multi-view tolerance
// (tests/test_gpu_multiview.py).
#include <hip/hip_runtime.h>

#include "gs_bwd_math.cuh"
#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

// ------------------------------------------- data-parallel view exchange ---
// each rank back-propagates its own view.  The reference's
// per-Gaussian backward (computeCov2DCUDA / preprocessCUDA / SH / cov3D
// backward, backward.cu:20-396) is linear in the 9 screen-space sums the
// blend produces, given the view's camera, radius and SH clamp bits.  So the
// ranks exchange those (10 words per Gaussian per view, kViewRow) instead of
// the 59-float parameter gradients, and every rank rebuilds the sum over all
// views of the parameter gradients in one pass that reads the parameters
// once: (N-1) x 40 B per Gaussian received per rank instead of a ring
// all-reduce's 2 (N-1)/N x 236 B.
//
// Row layout: dL_dcolor[3], dL_dmean2D.xy[2], dL_dconic (x, y, w)[3],
// dL_dopacity, and word 9 = radius | clamped_bits << 24 (0 = not visible).
// A view record is the P rows followed by the view's camera (kCamWords:
// viewmatrix, projmatrix, campos, width, height, tan_fovx, tan_fovy, 0), so
// one all-gather moves everything the multi-view backward needs.
__global__ void __launch_bounds__(256) pack_view_grads_kernel(int P, const float* __restrict__ grad_accum,
                                                              const int* __restrict__ radii,
                                                              const uint8_t* __restrict__ clamped,
                                                              const float* __restrict__ viewmatrix,
                                                              const float* __restrict__ projmatrix,
                                                              const float* __restrict__ campos, float width,
                                                              float height, float tan_fovx, float tan_fovy,
                                                              float* __restrict__ out) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < kCamWords) {
        const int w = threadIdx.x;
        float c = 0.f;
        if (w < 16) c = viewmatrix[w];
        else if (w < 32) c = projmatrix[w - 16];
        else if (w < 35) c = campos[w - 32];
        else if (w == 35) c = width;
        else if (w == 36) c = height;
        else if (w == 37) c = tan_fovx;
        else if (w == 38) c = tan_fovy;
        out[(size_t)P * kViewRow + w] = c;
    }
    if (idx >= P) return;
    const int r = radii[idx];
    float v[kViewRow];
#pragma unroll
    for (int q = 0; q < kViewRow; q++) v[q] = 0.f;
    if (r > 0) {
        const float4* row = reinterpret_cast<const float4*>(grad_accum + (size_t)idx * kGradRow);
        const float4 r0 = row[0], r1 = row[1];
        v[0] = r0.x; v[1] = r0.y; v[2] = r0.z; v[3] = r0.w;
        v[4] = r1.x; v[5] = r1.y; v[6] = r1.z; v[7] = r1.w;
        v[8] = grad_accum[(size_t)idx * kGradRow + 8];
        const uint32_t cb = clamped ? clamped[idx] : 0u;
        v[9] = __uint_as_float((uint32_t)min(r, 0xFFFFFF) | (cb << 24));
    }
    float2* o = reinterpret_cast<float2*>(out + (size_t)idx * kViewRow);
#pragma unroll
    for (int q = 0; q < kViewRow / 2; q++) o[q] = make_float2(v[2 * q], v[2 * q + 1]);
}

void launch_pack_view_grads(int P, const GeomView& g, const int* radii, bool has_sh, const float* viewmatrix,
                            const float* projmatrix, const float* campos, int width, int height, float tan_fovx,
                            float tan_fovy, float* out, hipStream_t s) {
    hipLaunchKernelGGL(pack_view_grads_kernel, dim3((P + 255) / 256 > 0 ? (P + 255) / 256 : 1), dim3(256), 0, s,
                       P, g.grad_accum, radii, has_sh ? g.clamped : nullptr, viewmatrix, projmatrix, campos,
                       (float)width, (float)height, tan_fovx, tan_fovy, out);
}

// One thread per Gaussian: sum over the V views (in view order) of the
// reference's per-view parameter gradients.  Per view the terms are formed
// exactly as backward_gaussian_body does (cov2D `=`, projection `+=`, SH
// direction `+=`); dL_dcov3D is summed over views before the (linear) cov3D
// backward runs once.  Optional densification statistics (train.py:111-113)
// are accumulated view by view: accum += ||dL/dmean2D.xy||, denom += 1,
// max_radii = max(max_radii, radius) for every view that sees the Gaussian.
__device__ __forceinline__ const float* mv_row(const MultiViewArgs& a, int v) {
    return a.table ? a.table[v] : a.rows[v];
}
__device__ __forceinline__ const float* mv_cam(const MultiViewArgs& a, int v) {
    return a.table ? a.table[a.V + v] : a.cams[v];
}
// A wave-uniform pointer as a constant-address-space one: its loads become
// scalar (s_load), the view's camera lives in SGPRs instead of ~35 VGPRs.
typedef const __attribute__((address_space(4))) float* ConstF;
__device__ __forceinline__ ConstF uniform_const(const float* p) {
    const uint64_t u = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return reinterpret_cast<ConstF>(((uint64_t)hi << 32) | lo);
}

// computeColorFromSH backward (backward.cu:20-139) for the multi-view kernel:
// the basis factors dsh_c and the masked dL/drgb as sh_backward_terms, and the
// view-direction term through the contracted form -- w_k = sum_c dRGB_c s_kc
// first, then dL/ddir = sum_k w_k dB_k/ddir with the constant factors folded
// -- instead of the per-channel d(rgb)/d(dir) and three dot products (the
// same sum in another association: ~180 fewer VALU per view).
template <typename SH>
__device__ __forceinline__ void mv_sh_terms(int deg, const float (&campos)[3], float mx, float my, float mz,
                                            const SH& s, uint8_t cb, const float* acc, float (&dsh_c)[16],
                                            float (&dRGB)[3], float (&dmean)[3]) {
    const float dox = mx - campos[0], doy = my - campos[1], doz = mz - campos[2];
    const float len = sqrtf(dot3(dox, doy, doz, dox, doy, doz));
    const float x = dox / len, y = doy / len, z = doz / len;
#pragma unroll
    for (int c = 0; c < 3; c++) dRGB[c] = acc[c] * (((cb >> c) & 1) ? 0.0f : 1.0f);
    sh_basis(deg, x, y, z, dsh_c);
    float w[16];
#pragma unroll
    for (int k = 1; k < 16; k++) w[k] = s[k][0] * dRGB[0] + s[k][1] * dRGB[1] + s[k][2] * dRGB[2];
    float ddx = 0.f, ddy = 0.f, ddz = 0.f;
    if (deg > 0) {
        ddx = -SH_C1 * w[3];
        ddy = -SH_C1 * w[1];
        ddz = SH_C1 * w[2];
        if (deg > 1) {
            constexpr float k2_2 = 2.f * SH_C2_2, k2_4 = 2.f * SH_C2_4, k4_2 = 4.f * SH_C2_2;
            ddx += SH_C2_0 * y * w[4] - k2_2 * x * w[6] + SH_C2_3 * z * w[7] + k2_4 * x * w[8];
            ddy += SH_C2_0 * x * w[4] + SH_C2_1 * z * w[5] - k2_2 * y * w[6] - k2_4 * y * w[8];
            ddz += SH_C2_1 * y * w[5] + k4_2 * z * w[6] + SH_C2_3 * x * w[7];
            if (deg > 2) {
                const float xx = x * x, yy = y * y, zz = z * z;
                const float xy = x * y, yz = y * z, xz = x * z;
                constexpr float a0 = 6.f * SH_C3_0, a2 = -2.f * SH_C3_2, a3 = -6.f * SH_C3_3, a5 = 2.f * SH_C3_5,
                                a6 = 3.f * SH_C3_6;
                ddx += a0 * xy * w[9] + SH_C3_1 * yz * w[10] + a2 * xy * w[11] + a3 * xz * w[12] +
                       SH_C3_4 * (4.f * zz - 3.f * xx - yy) * w[13] + a5 * xz * w[14] + a6 * (xx - yy) * w[15];
                constexpr float b0 = 3.f * SH_C3_0, b3 = -6.f * SH_C3_3, b4 = -2.f * SH_C3_4, b5 = -2.f * SH_C3_5,
                                b6 = -6.f * SH_C3_6;
                ddy += b0 * (xx - yy) * w[9] + SH_C3_1 * xz * w[10] + SH_C3_2 * (4.f * zz - 3.f * yy - xx) * w[11] +
                       b3 * yz * w[12] + b4 * xy * w[13] + b5 * yz * w[14] + b6 * xy * w[15];
                constexpr float c2 = 8.f * SH_C3_2, c3 = 3.f * SH_C3_3, c4 = 8.f * SH_C3_4;
                ddz += SH_C3_1 * xy * w[10] + c2 * yz * w[11] + c3 * (2.f * zz - xx - yy) * w[12] + c4 * xz * w[13] +
                       SH_C3_5 * (xx - yy) * w[14];
            }
        }
    }
    float ox, oy, oz;
    dnormvdv3(dox, doy, doz, ddx, ddy, ddz, ox, oy, oz);
    dmean[0] += ox;
    dmean[1] += oy;
    dmean[2] += oz;
}

// One pass over the views with each view's rows staged through LDS: the
// workgroup's rows of view v (contiguous in the record) are read
// with 8-B loads by consecutive lanes -- five load instructions per thread per
// view instead of ten per-thread loads at a 40-B stride (each touching ~20
// cache lines per wave instruction) -- the next view's rows in flight in
// registers while this view's terms are formed.  (Round 4's two-pass form --
// an any-check pass, the geometry pass, the SH pass, each re-reading the rows
// per thread -- measured 0.3386 against 0.3360 ms per 8-view step at config
// 5, profiles/r05c_bench_cfg5_mv*.log, and is removed.)
// One wave per workgroup: the per-view staging needs no cross-wave barrier
// (with 4-wave workgroups the waves waited on each other twice per view).
constexpr int kMvT = 64;
constexpr int kMvRowF2 = kMvT * kViewRow / 2;          // float2 per view per workgroup (320)
constexpr int kMvRowPer = (kMvRowF2 + kMvT - 1) / kMvT;  // per thread (5)
template <bool kHasSH, bool kSH16>
__global__ void __launch_bounds__(kMvT) multiview_backward1_kernel(MultiViewArgs a) {
    constexpr bool kStage = kHasSH && kSH16;
    __shared__ float s_sh[kStage ? kMvT * kShRow : 1];
    __shared__ __attribute__((aligned(16))) float s_rows[kMvT * kViewRow];
    const int local0 = blockIdx.x * kMvT;
    const int nblk = min(kMvT, a.count - local0);
    if constexpr (kStage) {
        const float4* in = reinterpret_cast<const float4*>(a.shs) + (size_t)(a.g0 + local0) * 12;
        if (nblk == kMvT) {
            float4 v[12];
#pragma unroll
            for (int k = 0; k < 12; k++) v[k] = ldg4<true>(in + threadIdx.x + kMvT * k);
#pragma unroll
            for (int k = 0; k < 12; k++) {
                const int f = threadIdx.x + kMvT * k;
                float* r = s_sh + (f / 12) * kShRow + 4 * (f % 12);
                r[0] = v[k].x; r[1] = v[k].y; r[2] = v[k].z; r[3] = v[k].w;
            }
        } else {
            for (int f = threadIdx.x; f < nblk * 12; f += kMvT) {
                const float4 v = in[f];
                float* r = s_sh + (f / 12) * kShRow + 4 * (f % 12);
                r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
            }
        }
    }
    const int local = local0 + threadIdx.x;
    const bool live = local < a.count;
    const int idx = a.g0 + local;
    float* lrow = kStage ? s_sh + threadIdx.x * kShRow : nullptr;
    const int nf2 = nblk * (kViewRow / 2);  // this block's float2 per view
    // view v's rows of this block: a.rows[v] points at Gaussian g0's row
    auto load_rows = [&](int v, float2 (&r)[kMvRowPer]) {
        const float2* src = reinterpret_cast<const float2*>(mv_row(a, v) + (size_t)local0 * kViewRow);
#pragma unroll
        for (int i = 0; i < kMvRowPer; i++) {
            const int f = threadIdx.x + kMvT * i;
            if (f < nf2) {
                typedef float f2v __attribute__((ext_vector_type(2)));
                const f2v t = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(src + f));
                r[i] = make_float2(t.x, t.y);
            } else {
                r[i] = make_float2(0.f, 0.f);
            }
        }
    };
    float mx = 0.f, my = 0.f, mz = 0.f;
    float4 qrot = make_float4(0.f, 0.f, 0.f, 0.f);
    float scl[3] = {0.f, 0.f, 0.f}, cov3D[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float st_acc = 0.f, st_den = 0.f, st_max = 0.f;
    const bool stats = a.grad_norm_accum != nullptr;
    if (live) {
        mx = a.means3D[3 * idx];
        my = a.means3D[3 * idx + 1];
        mz = a.means3D[3 * idx + 2];
        qrot = reinterpret_cast<const float4*>(a.rotations)[idx];
        scl[0] = a.scales[3 * idx + 0];
        scl[1] = a.scales[3 * idx + 1];
        scl[2] = a.scales[3 * idx + 2];
        if (stats) {
            st_acc = a.grad_norm_accum[idx];
            st_den = a.denom[idx];
            st_max = a.max_radii[idx];
        }
    }
    compute_cov3d(scl, qrot, a.scale_modifier, cov3D);
    const int ncoef = min((a.D + 1) * (a.D + 1), a.M);
    float dmean_t[3] = {0.f, 0.f, 0.f}, ddir[3] = {0.f, 0.f, 0.f};
    float dcov_t[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, dop = 0.f;
    float dsh_t[kHasSH ? 48 : 1];
#pragma unroll
    for (int i = 0; i < (kHasSH ? 48 : 1); i++) dsh_t[i] = 0.f;
    float s_reg[kHasSH && !kStage ? 16 : 1][3];
    if constexpr (kHasSH && !kStage) {
        const float* sh = a.shs + (size_t)(live ? idx : a.g0) * a.M * 3;
#pragma unroll
        for (int k = 0; k < 16; k++)
#pragma unroll
            for (int c = 0; c < 3; c++) s_reg[k][c] = (live && k < ncoef) ? sh[3 * k + c] : 0.f;
    }
    bool any = false;
    float2 nxt[kMvRowPer];
    load_rows(0, nxt);
    for (int v = 0; v < a.V; v++) {
        __syncthreads();  // the previous view's rows are read (and, at v = 0, the SH rows staged)
        float2* srow = reinterpret_cast<float2*>(s_rows);
#pragma unroll
        for (int i = 0; i < kMvRowPer; i++) {
            const int f = threadIdx.x + kMvT * i;
            if (f < kMvRowF2) srow[f] = nxt[i];
        }
        __syncthreads();
        if (v + 1 < a.V) load_rows(v + 1, nxt);  // in flight while view v's terms are formed
        // (two views ahead measured the same: 0.2349 vs 0.2343 ms, profiles/r05r_bench_cfg5.log)
        const float* row = s_rows + threadIdx.x * kViewRow;
        const uint32_t w9 = __float_as_uint(row[9]);
        if (!live || w9 == 0u) continue;  // not visible in view v: no terms (the reference's radii > 0 filter)
        any = true;
        const float acc[3] = {row[0], row[1], row[2]};
        const float gx = row[3], gy = row[4], dcx = row[5], dcy = row[6], dcw = row[7], dop_v = row[8];
        const ConstF cam = uniform_const(mv_cam(a, v));
        Mat4 V, Pm;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            V.m[i] = cam[i];
            Pm.m[i] = cam[16 + i];
        }
        const float campos[3] = {cam[32], cam[33], cam[34]};
        const float tan_fovx = cam[37], tan_fovy = cam[38];
        // rasterizer_impl.cu:222-223 / gs_api.cpp: focal from the image size
        const float focal_x = cam[35] / (2.0f * tan_fovx);
        const float focal_y = cam[36] / (2.0f * tan_fovy);
        float dmean[3], dcov[6];
        cov2d_backward(mx, my, mz, cov3D, dcx, dcy, dcw, V, focal_x, focal_y, tan_fovx, tan_fovy, dmean, dcov);
        proj_backward(mx, my, mz, Pm, gx, gy, dmean);
#pragma unroll
        for (int i = 0; i < 3; i++) dmean_t[i] += dmean[i];
#pragma unroll
        for (int i = 0; i < 6; i++) dcov_t[i] += dcov[i];
        dop += dop_v;
        if (stats) {
            st_acc = st_acc + sqrtf(gx * gx + gy * gy);
            st_den = st_den + 1.f;
            st_max = fmaxf(st_max, (float)(w9 & 0xFFFFFFu));
        }
        if constexpr (kHasSH) {
            const uint8_t cb = (uint8_t)(w9 >> 24);
            float dsh_c[16], dRGB[3];
            if constexpr (kStage) {
                mv_sh_terms(a.D, campos, mx, my, mz, ShRowPtr{lrow}, cb, acc, dsh_c, dRGB, ddir);
            } else {
                mv_sh_terms(a.D, campos, mx, my, mz, s_reg, cb, acc, dsh_c, dRGB, ddir);
            }
            // (every coefficient: sh_basis leaves dsh_c[k >= ncoef] at 0, and
            // the stores below write 0 there -- no per-view selects)
#pragma unroll
            for (int k = 0; k < 16; k++)
#pragma unroll
                for (int c = 0; c < 3; c++) dsh_t[3 * k + c] += dsh_c[k] * dRGB[c];
        }
    }
    if (live) {
        // (a Gaussian no view sees: every output is zero, as the two-pass kernel writes)
        a.dL_dopacity[idx] = any ? dop : 0.f;
        float dscale[3] = {0.f, 0.f, 0.f};
        float4 dq = make_float4(0.f, 0.f, 0.f, 0.f);
        if (any) cov3d_backward(qrot, scl, a.scale_modifier, dcov_t, dscale, dq);
#pragma unroll
        for (int i = 0; i < 3; i++) a.dL_dscale[3 * idx + i] = dscale[i];
        reinterpret_cast<float4*>(a.dL_drot)[idx] = dq;
        if (stats && any) {
            a.grad_norm_accum[idx] = st_acc;
            a.denom[idx] = st_den;
            a.max_radii[idx] = st_max;
        }
#pragma unroll
        for (int i = 0; i < 3; i++) a.dL_dmean3D[3 * idx + i] = any ? dmean_t[i] + ddir[i] : 0.f;
    }
    if constexpr (kStage) {
        __syncthreads();  // every thread has read its SH row: the area takes the gradient rows
        if (live) {
#pragma unroll
            for (int i = 0; i < 48; i++) lrow[i] = (any && i < 3 * ncoef) ? dsh_t[i] : 0.f;
        }
        __syncthreads();
        float4* out = reinterpret_cast<float4*>(a.dL_dsh) + (size_t)(a.g0 + local0) * 12;
        for (int f = threadIdx.x; f < nblk * 12; f += kMvT) {
            const float* r = s_sh + (f / 12) * kShRow + 4 * (f % 12);
            store_out4(&out[f], make_float4(r[0], r[1], r[2], r[3]), a.nt != 0);
        }
    } else if constexpr (kHasSH) {
        if (live)
            for (int k = 0; k < a.M; k++)
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    float val = 0.f;
#pragma unroll
                    for (int kk = 0; kk < 16; kk++) val = (kk == k && any && k < ncoef) ? dsh_t[3 * kk + c] : val;
                    a.dL_dsh[(size_t)idx * a.M * 3 + 3 * k + c] = val;
                }
    }
}

void launch_multiview_backward(const MultiViewArgs& args, hipStream_t s) {
    if (args.count <= 0) return;
    MultiViewArgs a = args;
    a.nt = 1;  // the dL_dsh rows non-temporal (as backward_gaussians_kernel's)
    const dim3 grid((a.count + kMvT - 1) / kMvT);
    const bool sh = a.shs != nullptr;
    // (A role-split form -- 64 Gaussians per workgroup, wave 3 the geometry
    // terms, waves 0-2 one colour channel each, 128 VGPRs and 22 KB of LDS:
    // 4 waves per SIMD instead of 2 -- measured 0.4358 against 0.3360 ms per
    // 8-view step at config 5, profiles/r05d_bench_cfg5_roles.log: the
    // per-view barrier waits on the geometry wave and the channel waves redo
    // the direction and basis; removed.)
    if (sh && a.M == 16) hipLaunchKernelGGL((multiview_backward1_kernel<true, true>), grid, dim3(kMvT), 0, s, a);
    else if (sh) hipLaunchKernelGGL((multiview_backward1_kernel<true, false>), grid, dim3(kMvT), 0, s, a);
    else hipLaunchKernelGGL((multiview_backward1_kernel<false, false>), grid, dim3(kMvT), 0, s, a);
}

}  // namespace gsamd
