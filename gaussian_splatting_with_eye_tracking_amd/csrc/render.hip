// render.hip -- front-to-back alpha blending on gfx950.
//
// Base: base/cr/forward.cu:261-374 (renderCUDA).  AMR: amr/cr/forward.cu:
// 261-518 (renderCUDA with per-tile level skip on the 2x2 sub-lattice) and
// :520-648 (interpolateCUDA).
//
// One 256-thread workgroup (4 wave64s) per 16x16 pixel block; wave w owns
// pixel rows 4w..4w+3 so a wave's 64 pixels are a compact 16x4 patch and its
// lanes tend to finish together.  Gaussians are staged in LDS 256 at a time
// (position, conic+opacity, colour -- the reference re-reads colour from
// global memory per pixel-Gaussian pair; here it is staged too).  The
// per-pixel semantics (contributor / last_contributor / done, the alpha<1/255
// and T<1e-4 tests) are the reference's; the forward additionally records the
// per-tile maximum n_contrib so the backward can skip the tail of a range no
// pixel of the tile consumed.
#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

constexpr int kBlk = 256;

struct BlendOut {
    float T;
    uint32_t last;
    float C[3];
};

// Blend `range` for pixel (pixf) -- the body shared by base and AMR kernels.
// All 256 threads must call it (it contains barriers); `done` marks lanes that
// do not blend (outside the image).
__device__ __forceinline__ BlendOut blend_range(uint2 range, float2 pixf, bool done,
                                                const uint32_t* __restrict__ point_list,
                                                const float2* __restrict__ means2D,
                                                const float* __restrict__ features,
                                                const float4* __restrict__ conic_opacity, float2* s_xy,
                                                float4* s_co, float4* s_rgb) {
#pragma clang fp contract(fast)
    const int tid = threadIdx.x;
    const int rounds = (int)((range.y - range.x + kBlk - 1) / kBlk);
    int toDo = (int)(range.y - range.x);
    BlendOut o;
    o.T = 1.0f;
    o.last = 0;
    o.C[0] = o.C[1] = o.C[2] = 0.f;
    uint32_t contributor = 0;
    for (int i = 0; i < rounds; i++, toDo -= kBlk) {
        if (__syncthreads_count(done) == kBlk) break;
        const uint32_t progress = (uint32_t)(i * kBlk + tid);
        if (range.x + progress < range.y) {
            const uint32_t id = point_list[range.x + progress];
            s_xy[tid] = means2D[id];
            s_co[tid] = conic_opacity[id];
            s_rgb[tid] = make_float4(features[3 * id], features[3 * id + 1], features[3 * id + 2], 0.f);
        }
        __syncthreads();
        const int cnt = min(kBlk, toDo);
        for (int j = 0; j < cnt && !done; j++) {
            contributor++;
            const float2 xy = s_xy[j];
            const float dx = xy.x - pixf.x, dy = xy.y - pixf.y;
            const float4 co = s_co[j];
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, co.w * __expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = o.T * (1 - alpha);
            if (test_T < 0.0001f) {
                done = true;
                continue;
            }
            const float4 f = s_rgb[j];
            const float w = alpha * o.T;
            o.C[0] += f.x * w;
            o.C[1] += f.y * w;
            o.C[2] += f.z * w;
            o.T = test_T;
            o.last = contributor;
        }
    }
    return o;
}

__device__ __forceinline__ void block_max_to(uint32_t v, uint32_t* smax, uint32_t* dst) {
    // wave max, then one LDS atomic per wave
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, kWave));
    if ((threadIdx.x & (kWave - 1)) == 0) atomicMax(smax, v);
    __syncthreads();
    if (threadIdx.x == 0) *dst = *smax;
}

__global__ void __launch_bounds__(kBlk) render_fwd_kernel(int W, int H, const uint32_t* __restrict__ ranges,
                                                          const uint32_t* __restrict__ point_list,
                                                          const float2* __restrict__ means2D,
                                                          const float* __restrict__ features,
                                                          const float4* __restrict__ conic_opacity,
                                                          float* __restrict__ final_T,
                                                          uint32_t* __restrict__ n_contrib,
                                                          uint32_t* __restrict__ max_contrib,
                                                          const float* __restrict__ bg, float* __restrict__ out_color) {
    __shared__ float2 s_xy[kBlk];
    __shared__ float4 s_co[kBlk];
    __shared__ float4 s_rgb[kBlk];
    __shared__ uint32_t s_max;
    const int tid = threadIdx.x;
    if (tid == 0) s_max = 0;
    const int tile = blockIdx.y * gridDim.x + blockIdx.x;
    const uint32_t px = blockIdx.x * 16 + (tid & 15);
    const uint32_t py = blockIdx.y * 16 + (tid >> 4);
    const bool inside = px < (uint32_t)W && py < (uint32_t)H;
    const uint2 range = reinterpret_cast<const uint2*>(ranges)[tile];
    const BlendOut o = blend_range(range, make_float2((float)px, (float)py), !inside, point_list, means2D, features,
                                   conic_opacity, s_xy, s_co, s_rgb);
    if (inside) {
        const uint32_t pid = (uint32_t)W * py + px;
        final_T[pid] = o.T;
        n_contrib[pid] = o.last;
        const size_t plane = (size_t)H * W;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) out_color[ch * plane + pid] = o.C[ch] + o.T * bg[ch];
    }
    block_max_to(inside ? o.last : 0u, &s_max, &max_contrib[tile]);
}

void launch_render_forward(int W, int H, const ImageView& img, const BinningView& b, const GeomView& g,
                           const float* features, const float* bg, float* out_color, hipStream_t s) {
    const int gx = (W + 15) / 16, gy = (H + 15) / 16;
    if (gx == 0 || gy == 0) return;
    hipLaunchKernelGGL(render_fwd_kernel, dim3(gx, gy), dim3(kBlk), 0, s, W, H, img.ranges, b.point_list,
                       reinterpret_cast<const float2*>(g.means2D), features,
                       reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib,
                       img.max_contrib, bg, out_color);
}

// ------------------------------------------------------------------- AMR ---
// amr/cr/forward.cu:313-339: sub-lattice offset -> AMR round
__device__ __forceinline__ uint32_t amr_round(uint32_t ox, uint32_t oy) {
    return ox == 0 ? (oy == 0 ? 1u : 4u) : (oy == 0 ? 3u : 2u);
}

// grid (2*tgx, 2*tgy) x 256: block -> (32-px tile, sub-lattice offset).
__global__ void __launch_bounds__(kBlk) amr_render_kernel(int W, int H, int tgx, const uint32_t* __restrict__ ranges,
                                                          const uint32_t* __restrict__ levels,
                                                          const uint32_t* __restrict__ levels_last,
                                                          const uint32_t* __restrict__ point_list,
                                                          const float2* __restrict__ means2D,
                                                          const float* __restrict__ features,
                                                          const float4* __restrict__ conic_opacity,
                                                          float* __restrict__ final_T,
                                                          uint32_t* __restrict__ n_contrib,
                                                          const float* __restrict__ bg, float* __restrict__ out_color,
                                                          int foveaStep) {
    __shared__ float2 s_xy[kBlk];
    __shared__ float4 s_co[kBlk];
    __shared__ float4 s_rgb[kBlk];
    const int tile = (blockIdx.y >> 1) * tgx + (blockIdx.x >> 1);
    const uint32_t L_last = levels_last[tile];
    uint32_t L = levels[tile];
    // Block-uniform early exits (amr/cr/forward.cu:287-367).
    if (L <= L_last) return;
    const uint32_t ox = blockIdx.x & 1, oy = blockIdx.y & 1;
    const uint32_t round = amr_round(ox, oy);
    if (L > 4) L = 4;
    if (foveaStep > 0 && round <= L_last) return;
    if (round > L) return;
    const int tid = threadIdx.x;
    const uint32_t px = (blockIdx.x >> 1) * 32 + 2 * (tid & 15) + ox;
    const uint32_t py = (blockIdx.y >> 1) * 32 + 2 * (tid >> 4) + oy;
    const bool inside = px < (uint32_t)W && py < (uint32_t)H;
    const uint2 range = reinterpret_cast<const uint2*>(ranges)[tile];
    const BlendOut o = blend_range(range, make_float2((float)px, (float)py), !inside, point_list, means2D, features,
                                   conic_opacity, s_xy, s_co, s_rgb);
    if (inside) {
        const uint32_t pid = (uint32_t)W * py + px;
        final_T[pid] = o.T;
        n_contrib[pid] = o.last;
        const size_t plane = (size_t)H * W;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) out_color[ch * plane + pid] = o.C[ch] + o.T * bg[ch];
    }
}

void launch_amr_render(int W, int H, const ImageView& img, const uint32_t* levels, const uint32_t* levels_last,
                       const BinningView& b, const GeomView& g, const float* features, const float* bg,
                       float* out_color, int foveaStep, hipStream_t s) {
    const int tgx = (W + 31) / 32, tgy = (H + 31) / 32;
    if (tgx == 0 || tgy == 0) return;
    hipLaunchKernelGGL(amr_render_kernel, dim3(2 * tgx, 2 * tgy), dim3(kBlk), 0, s, W, H, tgx, img.ranges, levels,
                       levels_last, b.point_list, reinterpret_cast<const float2*>(g.means2D), features,
                       reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib, bg,
                       out_color, foveaStep);
}

// amr/cr/forward.cu:520-648, per pixel.  pass 0 = the precomp copy of the
// foveaStep>0 branch, pass 1 = the neighbour copy.  The reference runs both
// in one launch (a race for foveaStep>0); they are two launches here.
__global__ void __launch_bounds__(256) amr_interpolate_kernel(int W, int H, int tgx, const uint32_t* __restrict__ levels,
                                                              const uint32_t* __restrict__ levels_last,
                                                              float* __restrict__ final_T,
                                                              uint32_t* __restrict__ n_contrib,
                                                              float* __restrict__ out_color, int foveaStep,
                                                              const float* __restrict__ precomp, int pass) {
    const int px = blockIdx.x * 16 + (threadIdx.x & 15);
    const int py = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (px >= W || py >= H) return;
    const int tile = (py / 32) * tgx + (px / 32);
    const uint32_t ox = px & 1, oy = py & 1;
    const uint32_t round = amr_round(ox, oy);
    uint32_t L = levels[tile];
    if (L > 4) L = 4;
    const size_t plane = (size_t)H * W;
    const size_t pid = (size_t)W * py + px;
    if (foveaStep > 0) {
        const int L_last = (int)levels_last[tile];
        if (pass == 0) {
            if (L <= (uint32_t)L_last || (int)round < L_last)
                for (int ch = 0; ch < 3; ch++) out_color[ch * plane + pid] = precomp[ch * plane + pid];
            return;
        }
        if ((int)round < L_last) return;
    }
    if (round <= L) return;
    const uint32_t olx = (L == 3 || L == 4) ? 1u : 0u;
    const int lx = px - (int)ox + (int)olx, ly = py - (int)oy + (int)olx;
    if (lx < W && ly < H) {
        const size_t lid = (size_t)W * ly + lx;
        final_T[pid] = final_T[lid];
        n_contrib[pid] = n_contrib[lid];
        for (int ch = 0; ch < 3; ch++) out_color[ch * plane + pid] = out_color[ch * plane + lid];
    }
}

void launch_amr_interpolate(int W, int H, const ImageView& img, const uint32_t* levels, const uint32_t* levels_last,
                            float* out_color, int foveaStep, const float* out_color_precomp, hipStream_t s) {
    const int tgx = (W + 31) / 32;
    const dim3 grid((W + 15) / 16, (H + 15) / 16);
    if (grid.x == 0 || grid.y == 0) return;
    if (foveaStep > 0)
        hipLaunchKernelGGL(amr_interpolate_kernel, grid, dim3(256), 0, s, W, H, tgx, levels, levels_last,
                           img.accum_alpha, img.n_contrib, out_color, foveaStep, out_color_precomp, 0);
    hipLaunchKernelGGL(amr_interpolate_kernel, grid, dim3(256), 0, s, W, H, tgx, levels, levels_last, img.accum_alpha,
                       img.n_contrib, out_color, foveaStep, out_color_precomp, 1);
}

}  // namespace gsamd
