// eye_preprocess.hip -- the eye-image preprocessing of the tracking front end
// (track_render.py:69-80) on gfx950, so a frame goes from the 8-bit camera
// image to RITnet's input without a host pass:
//
//   gamma 0.8 table, truncated to uint8 (track_render.py:72-73)
//   -> OpenCV 8-bit CLAHE, clip 1.5, 8x8 tiles (track_render.py:75-76)
//   -> ToTensor + Normalize([0.5], [0.5]) (RITnet/dataset.py:35-37)
//   -> the (0, 1, 3, 2) permute: the network sees the transposed image.
//
// Bit-exact with the host restatement eye_tracking.clahe (which reproduces
// the reference's saved segmentation): integer histograms, the clip limit
// int(clip * tile_area / 256) with batch + stepped-residual redistribution,
// LUT = rint(float(cdf) * (255.f / tile_area)) clamped to [0, 255], then the
// f32 bilinear blend of the four surrounding tile LUTs in OpenCV's operation
// order and rint again (the library is built with -ffp-contract=off, so every
// product and sum rounds as it does on the host).
//
// clahe_lut_kernel: one workgroup per tile -- LDS histogram (LDS atomics),
// clip + redistribution on 256 bins (one bin per thread), block inclusive
// scan, LUT to HBM as f32 [tiles][256] (integers 0..255, exact).
// clahe_apply_kernel: one workgroup per 64 x 64 pixel patch -- coalesced
// byte reads along x, the blended + normalised value through an LDS
// transposition, coalesced f32 stores along the output row (= source
// column).  Algorithmic bytes per 640 x 400 frame: 2 x 256 KB read (both
// kernels read the image) + 64 KB LUTs + 1 MB written.
#include <cmath>

#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

namespace {
constexpr int kBins = 256;
constexpr int kPatch = 64;
}

__global__ void __launch_bounds__(256) clahe_lut_kernel(const uint8_t* __restrict__ src, int W, int tiles_x,
                                                        int tile_w, int tile_h, const uint8_t* __restrict__ gamma,
                                                        int limit, float lut_scale, float* __restrict__ luts) {
    __shared__ uint32_t hist[kBins];
    __shared__ uint8_t s_gamma[kBins];
    __shared__ uint32_t wsum[4];
    const int tid = threadIdx.x;
    hist[tid] = 0;
    s_gamma[tid] = gamma[tid];
    __syncthreads();
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int area = tile_w * tile_h;
    const uint8_t* base = src + (size_t)ty * tile_h * W + (size_t)tx * tile_w;
    for (int i = tid; i < area; i += 256) {
        const int r = i / tile_w, c = i - r * tile_w;
        atomicAdd(&hist[s_gamma[base[(size_t)r * W + c]]], 1u);
    }
    __syncthreads();
    // clip (OpenCV CLAHE_CalcLut_Body): excess over the limit, redistributed
    // as a batch to every bin plus one to every step-th bin from 0
    uint32_t h = hist[tid];
    uint32_t over = 0;
    if (limit > 0) {
        over = h > (uint32_t)limit ? h - (uint32_t)limit : 0u;
        h -= over;
    }
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t w = over;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) w += __shfl_xor(w, off, 64);
    if (lane == 0) wsum[wave] = w;
    __syncthreads();
    const uint32_t clipped = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (limit > 0) {
        const uint32_t batch = clipped / kBins, residual = clipped - batch * kBins;
        h += batch;
        if (residual) {
            const uint32_t step = kBins / residual > 1 ? kBins / residual : 1u;
            if ((uint32_t)tid % step == 0 && (uint32_t)tid / step < residual) h += 1;
        }
    }
    // inclusive scan over the 256 bins: wave scans, then the wave totals
    uint32_t s = h;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(s, off, 64);
        if (lane >= off) s += t;
    }
    __syncthreads();
    if (lane == 63) wsum[wave] = s;
    __syncthreads();
    for (int k = 0; k < wave; k++) s += wsum[k];
    const float v = __builtin_rintf((float)s * lut_scale);  // saturate_cast<uchar>(float): nearest-even
    luts[(size_t)blockIdx.x * kBins + tid] = fminf(fmaxf(v, 0.f), 255.f);
}

// OpenCV CLAHE_Interpolation_Body: tile coordinate x / tile_w - 0.5, the
// lower / upper tile clamped to the grid, bilinear weights in f32.
__global__ void __launch_bounds__(256) clahe_apply_kernel(const uint8_t* __restrict__ src, int H, int W, int tiles_x,
                                                          int tiles_y, float inv_tw, float inv_th,
                                                          const uint8_t* __restrict__ gamma,
                                                          const float* __restrict__ luts, float* __restrict__ out) {
    __shared__ float tile[kPatch][kPatch + 1];
    __shared__ uint8_t s_gamma[kBins];
    const int tid = threadIdx.x;
    s_gamma[tid] = gamma[tid];
    __syncthreads();
    const int x0 = blockIdx.x * kPatch, y0 = blockIdx.y * kPatch;
    const int lx = tid & 63, ly0 = tid >> 6;
    const int x = x0 + lx;
    // per-column terms (x fixed for the lane)
    const float txf = (float)x * inv_tw - 0.5f;
    int tx1 = (int)floorf(txf);
    const float xa = txf - (float)tx1, xa1 = 1.0f - xa;
    int tx2 = tx1 + 1;
    tx1 = tx1 > 0 ? tx1 : 0;
    tx2 = tx2 < tiles_x - 1 ? tx2 : tiles_x - 1;
    for (int ly = ly0; ly < kPatch; ly += 4) {
        const int y = y0 + ly;
        if (x >= W || y >= H) continue;
        const float tyf = (float)y * inv_th - 0.5f;
        int ty1 = (int)floorf(tyf);
        const float ya = tyf - (float)ty1, ya1 = 1.0f - ya;
        int ty2 = ty1 + 1;
        ty1 = ty1 > 0 ? ty1 : 0;
        ty2 = ty2 < tiles_y - 1 ? ty2 : tiles_y - 1;
        const int v = s_gamma[src[(size_t)y * W + x]];
        const float* l1 = luts + (size_t)ty1 * tiles_x * kBins;
        const float* l2 = luts + (size_t)ty2 * tiles_x * kBins;
        const float a = l1[tx1 * kBins + v] * xa1 + l1[tx2 * kBins + v] * xa;
        const float b = l2[tx1 * kBins + v] * xa1 + l2[tx2 * kBins + v] * xa;
        const float res = a * ya1 + b * ya;
        const float q = fminf(fmaxf(__builtin_rintf(res), 0.f), 255.f);
        // ToTensor (/255 in f32) + Normalize(0.5, 0.5)
        tile[ly][lx] = (q / 255.0f - 0.5f) / 0.5f;
    }
    __syncthreads();
    // transposed store: out[x][y], lanes along y
    for (int lxx = ly0; lxx < kPatch; lxx += 4) {
        const int xo = x0 + lxx, yo = y0 + lx;
        if (xo < W && yo < H) out[(size_t)xo * H + yo] = tile[lx][lxx];
    }
}

void launch_eye_preprocess(const uint8_t* gray, int H, int W, const uint8_t* gamma, int tiles_x, int tiles_y,
                           int limit, float* luts, float* out, hipStream_t s) {
    const int tile_w = W / tiles_x, tile_h = H / tiles_y;
    const float lut_scale = (float)(kBins - 1) / (float)(tile_w * tile_h);  // OpenCV: float(255) / int area
    hipLaunchKernelGGL(clahe_lut_kernel, dim3(tiles_x * tiles_y), dim3(256), 0, s, gray, W, tiles_x, tile_w, tile_h,
                       gamma, limit, lut_scale, luts);
    const float inv_tw = 1.0f / (float)tile_w, inv_th = 1.0f / (float)tile_h;
    hipLaunchKernelGGL(clahe_apply_kernel, dim3((W + kPatch - 1) / kPatch, (H + kPatch - 1) / kPatch), dim3(256), 0,
                       s, gray, H, W, tiles_x, tiles_y, inv_tw, inv_th, gamma, luts, out);
}

}  // namespace gsamd
