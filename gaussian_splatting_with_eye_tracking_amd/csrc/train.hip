// train.hip -- the per-iteration bookkeeping of train.py:67-125 around the
// rasterizer, as single-pass element-wise kernels on gfx950:
//   * adam_kernel: torch.optim.Adam over the flat parameter buffer (all six
//     param groups in one launch);
//   * densify_stats_kernel: the densification statistics of train.py:111-113
//     / scene/gaussian_model.py:405-407 (max screen radius, accumulated
//     ||dL/dmeans2D[:2]||, view count), one pass instead of torch's
//     gather / norm / scatter chain.
// Both are HBM-bound; they touch each byte once.
#include <algorithm>
#include <cmath>

#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

// ------------------------------------------------------------ fused Adam ---
// torch.optim.Adam (scene/gaussian_model.py:163: betas (0.9, 0.999), eps 1e-15,
// no weight decay) over one flat f32 parameter buffer split into segments,
// one per param group (:154-161), each with its own learning rate and step
// count (a group whose parameter was just replaced has no gradient and is
// skipped by torch, so counts can differ: step 0 = skip).  Per element in
// torch's order (torch/optim/adam.py, foreach path on the device):
//   m = lerp(m, g, 1 - b1)            (weight < 0.5: m + w * (g - m))
//   v = v * b2;  v = v + (1 - b2) * (g * g)              (mul_, addcmul_)
//   p = p + (-lr / bc1) * (m / (sqrt(v) / sqrt(bc2) + eps))   (addcdiv_)
// with the host-side scalars rounded to f32 and each "a + s * x" contracted
// to one fma, as torch's HIP-compiled element-wise kernels are (this library
// builds with -ffp-contract=off, so the fmas are written out).  One pass:
// 28 B per element of HBM traffic (p, g, m, v in; p, m, v out).
struct AdamSegments {
    int n;                 // number of segments (<= 8)
    long long end[8];      // exclusive end offset of each segment
    float neg_step[8];     // -lr / (1 - b1^t)
    float bc2_sqrt[8];     // sqrt(1 - b2^t)
    int active[8];
};

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long long N,
                                                   AdamSegments seg, float w1, float b2, float one_minus_b2,
                                                   float eps) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < N; i += (long long)gridDim.x * 256) {
        int s = 0;
        while (s + 1 < seg.n && i >= seg.end[s]) s++;
        if (!seg.active[s]) continue;
        const float gi = g[i];
        const float m0 = m[i];
        const float mi = fmaf(w1, gi - m0, m0);
        const float vi = fmaf(one_minus_b2, gi * gi, v[i] * b2);
        const float denom = sqrtf(vi) / seg.bc2_sqrt[s] + eps;
        p[i] = fmaf(seg.neg_step[s], mi / denom, p[i]);
        m[i] = mi;
        v[i] = vi;
    }
}

void launch_adam(float* p, const float* g, float* m, float* v, long long N, int nseg, const long long* seg_end,
                 const double* lr, const long long* step, double beta1, double beta2, double eps, hipStream_t s) {
    if (N <= 0) return;
    AdamSegments seg{};
    seg.n = nseg;
    for (int i = 0; i < nseg; i++) {
        seg.end[i] = seg_end[i];
        seg.active[i] = step[i] > 0;
        const double bc1 = 1.0 - std::pow(beta1, (double)step[i]);
        const double bc2 = 1.0 - std::pow(beta2, (double)step[i]);
        seg.neg_step[i] = step[i] > 0 ? (float)(-(lr[i] / bc1)) : 0.f;
        seg.bc2_sqrt[i] = step[i] > 0 ? (float)std::sqrt(bc2) : 1.f;
    }
    const int blocks = (int)std::min<long long>((N + 255) / 256, 256LL * 64);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, N, seg, (float)(1.0 - beta1),
                       (float)beta2, (float)(1.0 - beta2), (float)eps);
}

// ----------------------------------------------- densification statistics ---
// visible = radii > 0 (gaussian_renderer/__init__.py:97):
//   max_radii2D[v] = max(max_radii2D[v], radii[v])           (train.py:111)
//   xyz_gradient_accum[v] += ||grad_means2D[v, :2]||          (:406)
//   denom[v] += 1                                             (:407)
// 32 B per Gaussian (radii, the 2D gradient row, three f32 read and written).
__global__ void __launch_bounds__(256) densify_stats_kernel(int P, const int* __restrict__ radii,
                                                            const float* __restrict__ grad_means2D, int g_stride,
                                                            float* __restrict__ accum, float* __restrict__ denom,
                                                            float* __restrict__ max_radii) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    if (r <= 0) return;
    const float gx = grad_means2D[(size_t)i * g_stride];
    const float gy = grad_means2D[(size_t)i * g_stride + 1];
    accum[i] = accum[i] + sqrtf(gx * gx + gy * gy);
    denom[i] = denom[i] + 1.f;
    max_radii[i] = fmaxf(max_radii[i], (float)r);
}

void launch_densify_stats(int P, const int* radii, const float* grad_means2D, int g_stride, float* accum,
                          float* denom, float* max_radii, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(densify_stats_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, radii, grad_means2D,
                       g_stride, accum, denom, max_radii);
}

// -------------------------------------------------------- activations ---
// The getters of scene/gaussian_model.py:93-113 that feed the rasterizer
// (gaussian_renderer/__init__.py:55-78), evaluated from the raw parameter
// segments of the flat buffer into the rasterizer's input arrays:
//   scales = exp(_scaling), rotations = normalize(_rotation) (F.normalize,
//   eps 1e-12), opacities = sigmoid(_opacity), shs = cat(_features_dc,
//   _features_rest) -> [P, M, 3].
// SH elements are processed element-wise over the [P, M*3] output (reads of
// the dc / rest rows and the writes are both wave-contiguous); the
// per-Gaussian activations share the launch.  224 B read + 224 B written per
// Gaussian at M = 16.
__global__ void __launch_bounds__(256) activate_kernel(int P, int M, const float* __restrict__ dc,
                                                       const float* __restrict__ rest,
                                                       const float* __restrict__ opacity_raw,
                                                       const float* __restrict__ scaling_raw,
                                                       const float* __restrict__ rotation_raw,
                                                       float* __restrict__ shs, float* __restrict__ opacity,
                                                       float* __restrict__ scales, float* __restrict__ rotations) {
    const long long n_sh = (long long)P * M * 3;
    const int row = 3 * M, rrow = 3 * M - 3;
    const long long stride = (long long)gridDim.x * 256;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n_sh; e += stride) {
        const long long i = e / row;
        const int j = (int)(e - i * row);
        shs[e] = j < 3 ? dc[i * 3 + j] : rest[i * rrow + (j - 3)];
    }
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < P; i += stride) {
        opacity[i] = 1.0f / (1.0f + expf(-opacity_raw[i]));
#pragma unroll
        for (int k = 0; k < 3; k++) scales[3 * i + k] = expf(scaling_raw[3 * i + k]);
        const float4 r = reinterpret_cast<const float4*>(rotation_raw)[i];
        const float d = fmaxf(sqrtf(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w), 1e-12f);
        reinterpret_cast<float4*>(rotations)[i] = make_float4(r.x / d, r.y / d, r.z / d, r.w / d);
    }
}

void launch_activate(int P, int M, const float* dc, const float* rest, const float* opacity_raw,
                     const float* scaling_raw, const float* rotation_raw, float* shs, float* opacity, float* scales,
                     float* rotations, hipStream_t s) {
    if (P <= 0) return;
    const long long n = (long long)P * M * 3;
    const int blocks = (int)std::min<long long>((n + 255) / 256, 256LL * 32);
    hipLaunchKernelGGL(activate_kernel, dim3(blocks), dim3(256), 0, s, P, M, dc, rest, opacity_raw, scaling_raw,
                       rotation_raw, shs, opacity, scales, rotations);
}

// The backward of those activations (torch autograd's formulas):
//   d_scaling  = d_scales * exp(_scaling)                      (ExpBackward)
//   d_opacity  = d_opac * (1 - s) * s,  s = sigmoid(_opacity)  (sigmoid_backward)
//   d_rotation = g / d - r * (sum_j g_j r_j / d^2) / |r|       (div + clamp_min + norm backward,
//                                                               d = max(|r|, 1e-12); second term only if |r| >= 1e-12)
//   d_dc, d_rest = the two slices of d_shs                    (CatBackward)
//   d_xyz      = d_means3D
// written into the gradient segments of the flat buffer (accumulate: +=).
__global__ void __launch_bounds__(256) activation_backward_kernel(
    int P, int M, int accumulate, const float* __restrict__ d_shs, const float* __restrict__ d_opac,
    const float* __restrict__ d_scales, const float* __restrict__ d_rot, const float* __restrict__ d_means3D,
    const float* __restrict__ opacity_raw, const float* __restrict__ scaling_raw,
    const float* __restrict__ rotation_raw, float* __restrict__ g_xyz, float* __restrict__ g_dc,
    float* __restrict__ g_rest, float* __restrict__ g_opacity, float* __restrict__ g_scaling,
    float* __restrict__ g_rotation) {
    const long long n_sh = (long long)P * M * 3;
    const int row = 3 * M, rrow = 3 * M - 3;
    const long long stride = (long long)gridDim.x * 256;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n_sh; e += stride) {
        const long long i = e / row;
        const int j = (int)(e - i * row);
        float* dst = j < 3 ? &g_dc[i * 3 + j] : &g_rest[i * rrow + (j - 3)];
        *dst = accumulate ? *dst + d_shs[e] : d_shs[e];
    }
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < P; i += stride) {
        const float sg = 1.0f / (1.0f + expf(-opacity_raw[i]));
        const float go = d_opac[i] * (1.0f - sg) * sg;
        g_opacity[i] = accumulate ? g_opacity[i] + go : go;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float gs = d_scales[3 * i + k] * expf(scaling_raw[3 * i + k]);
            g_scaling[3 * i + k] = accumulate ? g_scaling[3 * i + k] + gs : gs;
            const float gx = d_means3D[3 * i + k];
            g_xyz[3 * i + k] = accumulate ? g_xyz[3 * i + k] + gx : gx;
        }
        const float4 r = reinterpret_cast<const float4*>(rotation_raw)[i];
        const float4 g = reinterpret_cast<const float4*>(d_rot)[i];
        const float nrm = sqrtf(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w);
        const float d = fmaxf(nrm, 1e-12f);
        float4 out = make_float4(g.x / d, g.y / d, g.z / d, g.w / d);
        if (nrm >= 1e-12f) {
            const float gd = -(g.x * r.x + g.y * r.y + g.z * r.z + g.w * r.w) / (d * d);  // dL/dd
            const float k = gd / nrm;                                                     // norm backward
            out = make_float4(out.x + k * r.x, out.y + k * r.y, out.z + k * r.z, out.w + k * r.w);
        }
        float4* gr = reinterpret_cast<float4*>(g_rotation) + i;
        if (accumulate) {
            const float4 o = *gr;
            out = make_float4(o.x + out.x, o.y + out.y, o.z + out.z, o.w + out.w);
        }
        *gr = out;
    }
}

void launch_activation_backward(int P, int M, int accumulate, const float* d_shs, const float* d_opac,
                                const float* d_scales, const float* d_rot, const float* d_means3D,
                                const float* opacity_raw, const float* scaling_raw, const float* rotation_raw,
                                float* g_xyz, float* g_dc, float* g_rest, float* g_opacity, float* g_scaling,
                                float* g_rotation, hipStream_t s) {
    if (P <= 0) return;
    const long long n = (long long)P * M * 3;
    const int blocks = (int)std::min<long long>((n + 255) / 256, 256LL * 32);
    hipLaunchKernelGGL(activation_backward_kernel, dim3(blocks), dim3(256), 0, s, P, M, accumulate, d_shs, d_opac,
                       d_scales, d_rot, d_means3D, opacity_raw, scaling_raw, rotation_raw, g_xyz, g_dc, g_rest,
                       g_opacity, g_scaling, g_rotation);
}

}  // namespace gsamd
