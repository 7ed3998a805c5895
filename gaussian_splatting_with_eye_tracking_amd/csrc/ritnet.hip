// ritnet.hip -- the eye-tracking front end on gfx950:
// RITnet's DenseNet2D segmentation (RITnet/densenet.py:17-144, the model
// track_render.py:50-97 runs on the eye image) and the pupil centroid that
// becomes the fovea centre.
//
// The network is 32 channels wide at every level (5 down blocks, 4 up
// blocks, 3x3 and 1x1 convolutions, LeakyReLU, eval-mode BatchNorm, 2x2
// average pooling, nearest 2x upsampling, channel concatenations).  Its
// activations are channel planes [C][H][W] in HBM and every concatenation is
// VIRTUAL: a convolution reads its input channels from up to three segments
// (the tensors being concatenated, one optionally read through the nearest
// 2x upsampling), so no cat / interpolate copies exist.
//
// conv_kernel: one thread per output pixel computes all 32 output channels
// (32 accumulators).  Weights are repacked on the host as [ci][tap][co], so
// the 32 weights of one (ci, tap) are wave-uniform and contiguous: the
// compiler reads them with scalar loads and every FMA takes its weight from
// an SGPR (one VALU op per multiply-add, no LDS traffic).  Inputs are read
// straight from HBM/L2 (the 3x3 neighbours of adjacent lanes share lines);
// the epilogue fuses bias, LeakyReLU (slope 0.01) and the BatchNorm affine.
// head_kernel: the final 1x1 convolution to 4 classes fused with the
// argmax (RITnet/utils.py:186-190, first maximum wins) into uint8 labels.
// avgpool2_kernel: nn.AvgPool2d(2) (sum of the 4 inputs in window order,
// then / 4).  label_moments_kernel: sum of x, y and count over label-3 pixels.
#include <cmath>

#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

namespace {
constexpr int kCo = 32;  // output channels of every RITnet convolution but the head
}

// 3 input segments = a virtual channel concatenation.  Segment s holds
// C[s] channel planes of size Hs x Ws; up[s] = 1 reads it through the
// nearest 2x upsampling (Hs = H / 2, Ws = W / 2).
struct ConvIn {
    const float* p[3];
    int C[3];
    int up[3];
};

__device__ __forceinline__ float read_in(const ConvIn& in, int ci, int y, int x, int H, int W) {
    // ci is wave-uniform: the segment choice is a scalar branch
    int s = 0;
    if (ci >= in.C[0]) {
        ci -= in.C[0];
        s = 1;
        if (ci >= in.C[1]) {
            ci -= in.C[1];
            s = 2;
        }
    }
    const int u = in.up[s];
    const int hs = H >> u, ws = W >> u;
    return in.p[s][((size_t)ci * hs + (y >> u)) * ws + (x >> u)];
}

template <int kK>
__global__ void __launch_bounds__(256) conv_kernel(ConvIn in, int Cin, int H, int W, const float* __restrict__ w,
                                                   const float* __restrict__ bias, int lrelu,
                                                   const float* __restrict__ bn_scale,
                                                   const float* __restrict__ bn_shift, float* __restrict__ out) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const bool live = x < W && y < H;
    float acc[kCo];
#pragma unroll
    for (int co = 0; co < kCo; co++) acc[co] = 0.f;
    for (int ci = 0; ci < Cin; ci++) {
        // one tap per iteration: its 32 weights fit in SGPRs (unrolling the
        // 9 taps made the compiler hoist 288 scalar loads and spill them)
#pragma unroll 1
        for (int t = 0; t < kK * kK; t++) {
            const int yy = y + t / kK - kK / 2, xx = x + t % kK - kK / 2;
            const bool in_img = live && yy >= 0 && yy < H && xx >= 0 && xx < W;  // zero padding
            const float v = in_img ? read_in(in, ci, yy, xx, H, W) : 0.f;
            const float* wt = w + ((size_t)ci * kK * kK + t) * kCo;  // uniform: scalar loads
#pragma unroll
            for (int co = 0; co < kCo; co++) acc[co] = __builtin_fmaf(wt[co], v, acc[co]);
        }
    }
    if (!live) return;
    const size_t plane = (size_t)H * W, pix = (size_t)y * W + x;
#pragma unroll
    for (int co = 0; co < kCo; co++) {
        float v = acc[co] + bias[co];
        if (lrelu) v = v > 0.f ? v : 0.01f * v;
        if (bn_scale) v = v * bn_scale[co] + bn_shift[co];
        out[co * plane + pix] = v;
    }
}

// Implicit-GEMM convolution on the f32 matrix cores
// (v_mfma_f32_32x32x2_f32: exact f32, a k-ordered fma chain per output).
// Per wave: D[co][px] (32 output channels x 32 pixels of one row) += W^T x
// im2col, two rows per wave, so a workgroup of 4 waves covers a 32 x 8
// pixel block.  Per chunk of kCK input channels the block's input tile (with
// the kK - 1 halo, zero padding, the virtual concatenation and the 2x
// upsampling resolved while staging) and the chunk's weights go to LDS; each
// MFMA then reads one A value (a weight: lane l -> co = l & 31, k = l >> 5)
// and one B value (an input: k = l >> 5, pixel l & 31) from LDS.  The
// accumulator layout (col = pixel = lane & 31, row = channel = (r & 3) +
// 8 (r >> 2) + 4 (lane >> 5)) makes every epilogue store a coalesced
// 128-B row segment of one output channel.
//
// Staging is software-pipelined: every thread issues all of its global loads
// for chunk c + 1 (a compile-time count, unrolled, so they are all in flight
// at once) into registers before the MFMAs of chunk c and writes them to LDS
// after them.  A thread owns fixed positions of the input tile and walks the
// chunk's channels: the channel is wave-uniform, so the segment choice of the
// virtual concatenation is scalar and each load is a scalar base + the
// lane's precomputed spatial offset (one for direct, one for upsampled
// segments; out-of-image positions load a safe address and are zeroed when
// written to LDS).  Weights are 16-B loads.  (A load-then-store loop
// serialises one memory latency per element: ~25 us per chunk at the small
// deep levels.)
template <int kK, int kR>
__global__ void __launch_bounds__(256) conv_mfma_kernel(ConvIn in, int Cin, int H, int W, const float* __restrict__ w,
                                                        const float* __restrict__ bias, int lrelu,
                                                        const float* __restrict__ bn_scale,
                                                        const float* __restrict__ bn_shift, float* __restrict__ out) {
    constexpr int kT = kK * kK;              // taps
    constexpr int kCK = kK == 3 ? 16 : 32;   // input channels per LDS chunk (kCK * kT is even)
    constexpr int kBW = 32, kBH = 4 * kR;    // output block: 32 x 4 kR pixels (kR rows per wave)
    constexpr int kIW = kBW + kK - 1, kIH = kBH + kK - 1;
    constexpr int kPos = kIH * kIW;          // input tile positions
    constexpr int kNP = (kPos + 255) / 256;  // positions per thread
    constexpr int kNW4 = kCK * kT * kCo / 4; // staged weight float4s per chunk
    constexpr int kRW = (kNW4 + 255) / 256;
    __shared__ float s_in[kCK * kPos];
    __shared__ float4 s_w4[kNW4];
    const float* s_w = reinterpret_cast<const float*>(s_w4);
    const float4* __restrict__ w4 = reinterpret_cast<const float4*>(w);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x0 = blockIdx.x * kBW, y0 = blockIdx.y * kBH;
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    f32x16 acc[kR];
#pragma unroll
    for (int t = 0; t < kR; t++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc[t][r] = 0.f;
    const int half = lane >> 5, col = lane & 31;
    // the lane's tile positions: validity and spatial offsets (direct / 2x upsampled)
    bool pv[kNP];
    int off0[kNP], off1[kNP];
#pragma unroll
    for (int q = 0; q < kNP; q++) {
        const int pos = tid + 256 * q;
        const int gy = y0 + pos / kIW - kK / 2, gx = x0 + pos % kIW - kK / 2;
        pv[q] = pos < kPos && gy >= 0 && gy < H && gx >= 0 && gx < W;
        off0[q] = pv[q] ? gy * W + gx : 0;
        off1[q] = pv[q] ? (gy >> 1) * (W >> 1) + (gx >> 1) : 0;
    }
    float rin[kCK][kNP];
    float4 rw[kRW];
    auto fetch = [&](int c0) {
#pragma unroll
        for (int cc = 0; cc < kCK; cc++) {
            int ci = c0 + cc;  // wave-uniform: scalar segment choice
            if (ci >= Cin) {
#pragma unroll
                for (int q = 0; q < kNP; q++) rin[cc][q] = 0.f;
                continue;
            }
            int sg = 0;
            if (ci >= in.C[0]) {
                ci -= in.C[0];
                sg = 1;
                if (ci >= in.C[1]) {
                    ci -= in.C[1];
                    sg = 2;
                }
            }
            const int u = sg == 0 ? in.up[0] : sg == 1 ? in.up[1] : in.up[2];
            const float* base = (sg == 0 ? in.p[0] : sg == 1 ? in.p[1] : in.p[2]) +
                                (size_t)ci * (size_t)(H >> u) * (size_t)(W >> u);
#pragma unroll
            for (int q = 0; q < kNP; q++) rin[cc][q] = base[u ? off1[q] : off0[q]];
        }
#pragma unroll
        for (int v = 0; v < kRW; v++) {
            const int i = tid + 256 * v;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            // kT * kCo is a multiple of 4: one float4 never spans two input channels
            if (i < kNW4 && c0 + (4 * i) / (kT * kCo) < Cin) x = w4[(size_t)c0 * (kT * kCo / 4) + i];
            rw[v] = x;
        }
    };
    fetch(0);
    for (int c0 = 0; c0 < Cin; c0 += kCK) {
        __syncthreads();  // the previous chunk's MFMAs are done with the LDS tiles
#pragma unroll
        for (int cc = 0; cc < kCK; cc++)
#pragma unroll
            for (int q = 0; q < kNP; q++)
                if (tid + 256 * q < kPos) s_in[cc * kPos + tid + 256 * q] = pv[q] ? rin[cc][q] : 0.f;
#pragma unroll
        for (int v = 0; v < kRW; v++)
            if (tid + 256 * v < kNW4) s_w4[tid + 256 * v] = rw[v];
        __syncthreads();
        if (c0 + kCK < Cin) fetch(c0 + kCK);  // in flight during this chunk's MFMAs
#pragma unroll 2
        for (int kp = 0; kp < kCK * kT / 2; kp++) {
            const int k = 2 * kp + half;
            const int cc = k / kT, tap = k % kT;
            const float a = s_w[k * kCo + col];
#pragma unroll
            for (int t = 0; t < kR; t++) {
                const int ry = kR * wave + t + tap / kK, rx = col + tap % kK;
                const float b = s_in[(cc * kIH + ry) * kIW + rx];
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
            }
        }
    }
    const size_t plane = (size_t)H * W;
    const int x = x0 + col;
#pragma unroll
    for (int t = 0; t < kR; t++) {
        const int y = y0 + kR * wave + t;
        if (x >= W || y >= H) continue;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int co = (r & 3) + 8 * (r >> 2) + 4 * half;
            float v = acc[t][r] + bias[co];
            if (lrelu) v = v > 0.f ? v : 0.01f * v;
            if (bn_scale) v = v * bn_scale[co] + bn_shift[co];
            out[co * plane + (size_t)y * W + x] = v;
        }
    }
}

__global__ void __launch_bounds__(256) avgpool2_kernel(const float* __restrict__ in, int C, int H, int W,
                                                       float* __restrict__ out) {
    const int Ho = H / 2, Wo = W / 2;
    const size_t n = (size_t)C * Ho * Wo;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int x = (int)(i % Wo), y = (int)((i / Wo) % Ho), c = (int)(i / ((size_t)Wo * Ho));
    const float* p = in + ((size_t)c * H + 2 * y) * W + 2 * x;
    float s = p[0];
    s = s + p[1];
    s = s + p[W];
    s = s + p[W + 1];
    out[i] = s / 4.0f;
}

// Final 1x1 convolution (32 -> 4 classes) + argmax (first maximum, as
// torch.max) into labels; the logits are written too when requested.
__global__ void __launch_bounds__(256) head_kernel(const float* __restrict__ in, int H, int W,
                                                   const float* __restrict__ w, const float* __restrict__ bias,
                                                   float* __restrict__ logits, uint8_t* __restrict__ labels) {
    const size_t plane = (size_t)H * W;
    const size_t pix = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (pix >= plane) return;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int ci = 0; ci < kCo; ci++) {
        const float v = in[ci * plane + pix];
#pragma unroll
        for (int co = 0; co < 4; co++) acc[co] = __builtin_fmaf(w[ci * 4 + co], v, acc[co]);
    }
    int best = 0;
    float bv = 0.f;
#pragma unroll
    for (int co = 0; co < 4; co++) {
        const float v = acc[co] + bias[co];
        if (logits) logits[co * plane + pix] = v;
        if (co == 0 || v > bv) {
            bv = v;
            best = co;
        }
    }
    labels[pix] = (uint8_t)best;
}

// Sums of x, y and the count of the pixels labelled `cls` (the pupil is 3),
// per workgroup, then one f64 atomic add per workgroup into out[3].
__global__ void __launch_bounds__(256) label_moments_kernel(const uint8_t* __restrict__ labels, int H, int W, int cls,
                                                            double* __restrict__ out) {
    const size_t n = (size_t)H * W;
    double sx = 0.0, sy = 0.0, c = 0.0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (labels[i] == cls) {
            sx += (double)(i % W);
            sy += (double)(i / W);
            c += 1.0;
        }
    }
    __shared__ double s[3][4];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        sx += __shfl_xor(sx, off, 64);
        sy += __shfl_xor(sy, off, 64);
        c += __shfl_xor(c, off, 64);
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s[0][wave] = sx;
        s[1][wave] = sy;
        s[2][wave] = c;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const double v = s[threadIdx.x][0] + s[threadIdx.x][1] + s[threadIdx.x][2] + s[threadIdx.x][3];
        atomicAdd(&out[threadIdx.x], v);
    }
}

int g_ritnet_mfma = 1;  // 1: conv_mfma_kernel (default), 0: the SGPR-weight FMA kernel
void set_ritnet_mfma(int v) { g_ritnet_mfma = v; }
constexpr int kRitnetSmallWgs = 512;  // below this many 32 x 8 blocks: 32 x 4 blocks (one row per wave)

void launch_ritnet_conv(int k, const float* const* in_ptr, const int* in_c, const int* in_up, int nseg, int H, int W,
                        const float* w, const float* bias, int lrelu, const float* bn_scale, const float* bn_shift,
                        float* out, hipStream_t s) {
    ConvIn in{};
    int Cin = 0;
    for (int i = 0; i < 3; i++) {
        in.p[i] = i < nseg ? in_ptr[i] : nullptr;
        in.C[i] = i < nseg ? in_c[i] : 0;
        in.up[i] = i < nseg ? in_up[i] : 0;
        Cin += in.C[i];
    }
    if (g_ritnet_mfma) {
        // small planes (the deep levels) are latency-bound: one row per wave
        // doubles the workgroups and halves each wave's MFMA chain
        const bool small = ((W + 31) / 32) * ((H + 7) / 8) < kRitnetSmallWgs;
        const dim3 grid((W + 31) / 32, small ? (H + 3) / 4 : (H + 7) / 8);
#define GS_CONV_MFMA(K, R) \
    hipLaunchKernelGGL((conv_mfma_kernel<K, R>), grid, dim3(256), 0, s, in, Cin, H, W, w, bias, lrelu, bn_scale, bn_shift, out)
        if (k == 3) {
            if (small) GS_CONV_MFMA(3, 1); else GS_CONV_MFMA(3, 2);
        } else {
            if (small) GS_CONV_MFMA(1, 1); else GS_CONV_MFMA(1, 2);
        }
#undef GS_CONV_MFMA
        return;
    }
    const dim3 grid((W + 63) / 64, (H + 3) / 4);
    if (k == 3)
        hipLaunchKernelGGL(conv_kernel<3>, grid, dim3(256), 0, s, in, Cin, H, W, w, bias, lrelu, bn_scale, bn_shift,
                           out);
    else
        hipLaunchKernelGGL(conv_kernel<1>, grid, dim3(256), 0, s, in, Cin, H, W, w, bias, lrelu, bn_scale, bn_shift,
                           out);
}

void launch_avgpool2(const float* in, int C, int H, int W, float* out, hipStream_t s) {
    const size_t n = (size_t)C * (H / 2) * (W / 2);
    if (n == 0) return;
    hipLaunchKernelGGL(avgpool2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, C, H, W, out);
}

void launch_ritnet_head(const float* in, int H, int W, const float* w, const float* bias, float* logits,
                        uint8_t* labels, hipStream_t s) {
    const size_t n = (size_t)H * W;
    if (n == 0) return;
    hipLaunchKernelGGL(head_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, H, W, w, bias, logits,
                       labels);
}

void launch_label_moments(const uint8_t* labels, int H, int W, int cls, double* out, hipStream_t s) {
    (void)hipMemsetAsync(out, 0, 3 * sizeof(double), s);
    const size_t n = (size_t)H * W;
    const unsigned blocks = (unsigned)std::min<size_t>(1024, (n + 255) / 256);
    if (blocks) hipLaunchKernelGGL(label_moments_kernel, dim3(blocks), dim3(256), 0, s, labels, H, W, cls, out);
}

}  // namespace gsamd
