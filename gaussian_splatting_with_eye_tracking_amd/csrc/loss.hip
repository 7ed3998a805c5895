// loss.hip -- fused training loss of train.py:91-93 on gfx950:
//   loss = (1 - lambda) * l1_loss(x, y) + lambda * (1 - ssim(x, y))
// with utils/loss_utils.py:17-63 (11x11 Gaussian window, sigma 1.5, zero
// padding, per channel, mean over C*H*W), value AND gradient w.r.t. x in one
// pass over the image (oracle/loss_oracle.py has the derivation).
//
// One workgroup per 32x32 output tile of one channel.  The tile's input with
// a 10-px halo is staged in LDS once; the five separable 11-tap
// correlations (x, y, x^2, y^2, xy) are evaluated on the 42x42 region the
// adjoint needs, the SSIM map's three derivative maps are formed there
// (zero outside the image), and the three adjoint correlations give the
// gradient on the 32x32 tile.  HBM traffic: x and y read once (+ halo
// re-reads from L2), the gradient written once, 2 floats of partial sums per
// workgroup -- versus ~20 full-image intermediates for the reference's
// conv2d + elementwise autograd graph.
#include <cmath>

#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

namespace {
constexpr int kT = 32;             // output tile
constexpr int kR = 5;              // window radius
constexpr int kIn = kT + 4 * kR;   // 52: input region
constexpr int kMid = kT + 2 * kR;  // 42: region of the derivative maps
constexpr int kThreads = 256;
constexpr float kC1 = 0.01f * 0.01f;
constexpr float kC2 = 0.03f * 0.03f;

// utils/loss_utils.py:23-25 in float32: exp(-(x-5)^2 / 4.5) normalised
// (passed by value: lands in SGPRs / the kernel argument segment).
struct Window11 {
    float w[11];
};
}  // namespace

__global__ void __launch_bounds__(kThreads) l1_ssim_kernel(const float* __restrict__ img, const float* __restrict__ gt,
                                                           int H, int W, float lambda, float inv_n, Window11 win,
                                                           float* __restrict__ grad, float* __restrict__ partials) {
    const float* c_w = win.w;
    // LDS plan (floats): [in_x | in_y] (2 x 52 x 52) then h5 (5 x 52 x 42);
    // after the first vertical pass the derivative maps (3 x 42 x 42) reuse
    // the in_* space and the second horizontal pass (3 x 42 x 32) reuses h5.
    __shared__ float lds[2 * kIn * kIn + 5 * kIn * kMid];
    __shared__ float red[2][kThreads / 64];
    float* in_x = lds;
    float* in_y = lds + kIn * kIn;
    float* h5 = lds + 2 * kIn * kIn;
    float* g3 = lds;   // after pass 1
    float* gh = h5;    // after the derivative maps
    const int tid = threadIdx.x;
    const int ch = blockIdx.z;
    const int ox = blockIdx.x * kT, oy = blockIdx.y * kT;
    const size_t plane = (size_t)H * W;
    const float* X = img + ch * plane;
    const float* Y = gt + ch * plane;

    // 1. input with a 10-px halo, zero outside the image (the correlation's padding)
    for (int i = tid; i < kIn * kIn; i += kThreads) {
        const int r = i / kIn, c = i % kIn;
        const int gy = oy - 2 * kR + r, gx = ox - 2 * kR + c;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        in_x[i] = in ? X[(size_t)gy * W + gx] : 0.f;
        in_y[i] = in ? Y[(size_t)gy * W + gx] : 0.f;
    }
    __syncthreads();
    // 2. horizontal pass of x, y, x^2, y^2, xy: 52 rows x 42 columns
    for (int i = tid; i < kIn * kMid; i += kThreads) {
        const int r = i / kMid, c = i % kMid;
        const float* px = in_x + r * kIn + c;
        const float* py = in_y + r * kIn + c;
        float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
        for (int t = 0; t < 11; t++) {
            const float u = px[t], v = py[t], w = c_w[t];
            a += w * u;
            b += w * v;
            aa += w * (u * u);
            bb += w * (v * v);
            ab += w * (u * v);
        }
        h5[0 * kIn * kMid + i] = a;
        h5[1 * kIn * kMid + i] = b;
        h5[2 * kIn * kMid + i] = aa;
        h5[3 * kIn * kMid + i] = bb;
        h5[4 * kIn * kMid + i] = ab;
    }
    __syncthreads();
    // 3. vertical pass on 42 x 42, SSIM map and its derivative maps
    float ssim_sum = 0.f;
    for (int i = tid; i < kMid * kMid; i += kThreads) {
        const int r = i / kMid, c = i % kMid;
        const int gy = oy - kR + r, gx = ox - kR + c;
        float s[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 11; t++) {
            const float w = c_w[t];
#pragma unroll
            for (int q = 0; q < 5; q++) s[q] += w * h5[q * kIn * kMid + (r + t) * kMid + c];
        }
        float G1 = 0.f, G11 = 0.f, G12 = 0.f;
        if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
            const float mu1 = s[0], mu2 = s[1];
            const float s11 = s[2] - mu1 * mu1, s22 = s[3] - mu2 * mu2, s12 = s[4] - mu1 * mu2;
            const float A = 2.f * mu1 * mu2 + kC1, B = 2.f * s12 + kC2;
            const float Cd = mu1 * mu1 + mu2 * mu2 + kC1, D = s11 + s22 + kC2;
            const float inv = 1.f / (Cd * D);
            const float m = A * B * inv;
            if (r >= kR && r < kR + kT && c >= kR && c < kR + kT) ssim_sum += m;
            const float k = -lambda * inv_n;
            G1 = k * ((2.f * mu2 * B - 2.f * mu2 * A) * inv - m * (2.f * mu1 / Cd - 2.f * mu1 / D));
            G11 = k * (-m / D);
            G12 = k * (2.f * A * inv);
        }
        g3[0 * kMid * kMid + i] = G1;
        g3[1 * kMid * kMid + i] = G11;
        g3[2 * kMid * kMid + i] = G12;
    }
    __syncthreads();
    // 4. adjoint, horizontal: 42 rows x 32 columns
    for (int i = tid; i < kMid * kT; i += kThreads) {
        const int r = i / kT, c = i % kT;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const float* p = g3 + q * kMid * kMid + r * kMid + c;
            float a = 0.f;
#pragma unroll
            for (int t = 0; t < 11; t++) a += c_w[t] * p[t];
            gh[q * kMid * kT + i] = a;
        }
    }
    __syncthreads();
    // 5. adjoint, vertical, and the gradient on the 32 x 32 tile
    float l1_sum = 0.f;
    for (int i = tid; i < kT * kT; i += kThreads) {
        const int r = i / kT, c = i % kT;
        const int gy = oy + r, gx = ox + c;
        if (gy >= H || gx >= W) continue;
        float b[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 11; t++) {
            const float w = c_w[t];
#pragma unroll
            for (int q = 0; q < 3; q++) b[q] += w * gh[q * kMid * kT + (r + t) * kT + c];
        }
        const float x = X[(size_t)gy * W + gx], y = Y[(size_t)gy * W + gx];  // in_* space is reused
        const float d = x - y;
        l1_sum += fabsf(d);
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);  // torch abs backward
        grad[ch * plane + (size_t)gy * W + gx] =
            b[0] + 2.f * x * b[1] + y * b[2] + (1.f - lambda) * inv_n * sgn;
    }
    // 6. workgroup partial sums (fixed order: deterministic)
    ssim_sum = wave_sum(ssim_sum);
    l1_sum = wave_sum(l1_sum);
    if ((tid & 63) == 0) {
        red[0][tid >> 6] = ssim_sum;
        red[1][tid >> 6] = l1_sum;
    }
    __syncthreads();
    if (tid == 0) {
        float a = 0.f, b = 0.f;
        for (int w = 0; w < kThreads / 64; w++) {
            a += red[0][w];
            b += red[1][w];
        }
        const int blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partials[2 * blk + 0] = a;
        partials[2 * blk + 1] = b;
    }
}

// out[0] = loss, out[1] = l1, out[2] = ssim (means), summed in double in a
// fixed order by one workgroup.
__global__ void __launch_bounds__(256) l1_ssim_reduce_kernel(int nblk, const float* __restrict__ partials,
                                                             float lambda, double inv_n, float* __restrict__ out) {
    __shared__ double s[2][256];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nblk; i += 256) {
        a += partials[2 * i];
        b += partials[2 * i + 1];
    }
    s[0][threadIdx.x] = a;
    s[1][threadIdx.x] = b;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) {
            s[0][threadIdx.x] += s[0][threadIdx.x + off];
            s[1][threadIdx.x] += s[1][threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double ssim = s[0][0] * inv_n, l1 = s[1][0] * inv_n;
        out[0] = (float)((1.0 - lambda) * l1 + lambda * (1.0 - ssim));
        out[1] = (float)l1;
        out[2] = (float)ssim;
    }
}

size_t l1_ssim_workspace_bytes(int C, int H, int W) {
    const size_t nblk = (size_t)C * ((H + kT - 1) / kT) * ((W + kT - 1) / kT);
    return 2 * sizeof(float) * nblk;
}

void launch_l1_ssim(const float* img, const float* gt, int C, int H, int W, float lambda, float* grad, float* out3,
                    float* workspace, hipStream_t s) {
    Window11 win;
    {  // utils/loss_utils.py:23-25, float32 like torch.Tensor
        float sum = 0.f;
        for (int x = 0; x < 11; x++) {
            win.w[x] = (float)std::exp(-(double)((x - 5) * (x - 5)) / (2.0 * 1.5 * 1.5));
            sum += win.w[x];
        }
        for (int x = 0; x < 11; x++) win.w[x] = win.w[x] / sum;
    }
    if (C <= 0 || H <= 0 || W <= 0) return;
    const dim3 grid((W + kT - 1) / kT, (H + kT - 1) / kT, C);
    const double n = (double)C * H * W;
    hipLaunchKernelGGL(l1_ssim_kernel, grid, dim3(kThreads), 0, s, img, gt, H, W, lambda, (float)(1.0 / n), win,
                       grad, workspace);
    const int nblk = (int)(grid.x * grid.y * grid.z);
    hipLaunchKernelGGL(l1_ssim_reduce_kernel, dim3(1), dim3(256), 0, s, nblk, workspace, lambda, 1.0 / n, out3);
}

}  // namespace gsamd
