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

}  // namespace gsamd
