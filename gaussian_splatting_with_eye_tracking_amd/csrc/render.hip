// render.hip -- front-to-back alpha blending on gfx950.
//
// Base: base/cr/forward.cu:261-374 (renderCUDA).  AMR: amr/cr/forward.cu:
// 261-518 (renderCUDA with per-tile level skip on the 2x2 sub-lattice) and
// :520-648 (interpolateCUDA).
//
// One wave64 per 16x16 pixel block, 4 pixels per lane (gs_blend.cuh).
// Gaussians are staged in LDS 64 at a time (position, conic+opacity, colour
// -- the reference re-reads colour from global memory per pixel-Gaussian
// pair; here it is staged too).  The
// per-pixel semantics (contributor / last_contributor / done, the alpha<1/255
// and T<1e-4 tests) are the reference's; the forward additionally records the
// per-tile maximum n_contrib so the backward can skip the tail of a range no
// pixel of the tile consumed.
#include "gs_blend.cuh"
#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, kWave));
    return v;
}

template <int kPPL>
__device__ __forceinline__ void write_pixels(const PixelSetT<kPPL>& px, const BlendStateT<kPPL>& st, int W, int H,
                                             float* __restrict__ final_T, uint32_t* __restrict__ n_contrib,
                                             const float* __restrict__ bg, float* __restrict__ out_color) {
    const size_t plane = (size_t)H * W;
    const float b0 = bg[0], b1 = bg[1], b2 = bg[2];
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
        if (!px.inside[k]) continue;
        const uint32_t pid = px.pid[k];
        final_T[pid] = st.T[k];
        n_contrib[pid] = st.last[k];
        out_color[pid] = st.C[k][0] + st.T[k] * b0;
        out_color[plane + pid] = st.C[k][1] + st.T[k] * b1;
        out_color[2 * plane + pid] = st.C[k][2] + st.T[k] * b2;
    }
}

// One 16x16 tile per workgroup of kWaves waves (kPPL pixels per lane).
template <int kPPL, int kWaves>
__global__ void __launch_bounds__(64 * kWaves) render_fwd_kernel(int W, int H, const uint32_t* __restrict__ ranges,
                                                                 const uint32_t* __restrict__ point_list,
                                                                 const float2* __restrict__ means2D,
                                                                 const float* __restrict__ features,
                                                                 const float4* __restrict__ conic_opacity,
                                                                 float* __restrict__ final_T,
                                                                 uint32_t* __restrict__ n_contrib,
                                                                 uint32_t* __restrict__ max_contrib,
                                                                 const float* __restrict__ bg,
                                                                 float* __restrict__ out_color, int cull,
                                                                 const uint32_t* __restrict__ order, int gx,
                                                                 int xcd) {
    __shared__ float2 s_xy[64 * kWaves];
    __shared__ float4 s_co[64 * kWaves];
    __shared__ float4 s_rgb[64 * kWaves];
    __shared__ uint64_t s_bal[4 * kWaves];
    __shared__ uint32_t s_max;
    if (kWaves > 1 && threadIdx.x == 0) s_max = 0;
    const int tile = order ? (int)order[blockIdx.x]
                           : xcd ? xcd_block_tile((int)blockIdx.x, gx, (int)(gridDim.x / gx)) : (int)blockIdx.x;
    const uint32_t ox = (uint32_t)(tile % gx) * 16, oy = (uint32_t)(tile / gx) * 16;
    const PixelSetT<kPPL> px = make_pixels_t<kPPL, kWaves>(W, H, ox, oy, 1);
    const uint2 range = reinterpret_cast<const uint2*>(ranges)[tile];
    const BlendStateT<kPPL> st =
        blend_tile_t<kPPL, kWaves>(range, px, (float)ox, (float)oy, 1.0f, point_list,
                                   means2D, features, conic_opacity, s_xy, s_co, s_rgb, s_bal, cull != 0);
    write_pixels(px, st, W, H, final_T, n_contrib, bg, out_color);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < kPPL; k++) m = max(m, px.inside[k] ? st.last[k] : 0u);
    m = wave_max_u32(m);
    if (kWaves == 1) {
        if (threadIdx.x == 0) max_contrib[tile] = m;
    } else {
        if ((threadIdx.x & 63) == 0) atomicMax(&s_max, m);
        __syncthreads();
        if (threadIdx.x == 0) max_contrib[tile] = s_max;
    }
}

int g_cull = 1;         // row-group cull on (gs_blend.cuh); 0 only for the exactness A/B test
void set_cull(int v) { g_cull = v; }

// XCD-aware tile placement (gs_blend.cuh): bit 0 the forward blend, bit 1 the
// backward blend.  Measured at config 2 (profiles/r01g_xcd_ab.log): it halves
// the blend kernels' L2 -> fabric fetches (forward 770 -> 395 MB, backward
// 1100 -> 602 MB per launch) at the same forward time; the backward keeps the
// global heaviest-first order, 1.7 % faster than per-XCD heaviest-first
// (its XCD regions carry unequal work).  Default: forward only.
int g_xcd_map = 1;
void set_xcd_map(int v) { g_xcd_map = v; }

int g_fwd_variant = 2;  // 0: 1 wave x 4 px/lane, 1: 2 waves x 2 px/lane, 2: 4 waves x 1 px/lane

void set_forward_variant(int v) { g_fwd_variant = v; }

void launch_render_forward(int W, int H, const ImageView& img, const BinningView& b, const GeomView& g,
                           const float* features, const float* bg, float* out_color, hipStream_t s) {
    const int gx = (W + 15) / 16, gy = (H + 15) / 16;
    if (gx == 0 || gy == 0) return;
    // Row-major launch: heaviest-first by range length measured slower here
    // (early termination makes the range a poor work estimate); the backward
    // orders by max_contrib instead (backward.hip).
    const uint32_t* order = nullptr;
#define GS_FWD_LAUNCH(PPL, WAVES)                                                                                \
    hipLaunchKernelGGL((render_fwd_kernel<PPL, WAVES>), dim3(gx * gy), dim3(64 * WAVES), 0, s, W, H, img.ranges, \
                       b.point_list, reinterpret_cast<const float2*>(g.means2D), features,                       \
                       reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib,         \
                       img.max_contrib, bg, out_color, g_cull, order, gx, g_xcd_map & 1)
    switch (g_fwd_variant) {
        case 0: GS_FWD_LAUNCH(4, 1); break;
        case 1: GS_FWD_LAUNCH(2, 2); break;
        default: GS_FWD_LAUNCH(1, 4); break;
    }
#undef GS_FWD_LAUNCH
}

// ------------------------------------------------------------------- AMR ---
// amr/cr/forward.cu:313-339: sub-lattice offset -> AMR round
__device__ __forceinline__ uint32_t amr_round(uint32_t ox, uint32_t oy) {
    return ox == 0 ? (oy == 0 ? 1u : 4u) : (oy == 0 ? 3u : 2u);
}

// grid (2*tgx, 2*tgy) x kWaves waves: block -> (32-px tile, sub-lattice
// offset); the block covers the tile's 16x16 sub-lattice with stride 2, in the
// gs_blend.cuh geometry (kPPL pixels per lane).
template <int kPPL, int kWaves>
__global__ void __launch_bounds__(64 * kWaves) amr_render_kernel(int W, int H, int tgx,
                                                                 const uint32_t* __restrict__ ranges,
                                                                 const uint32_t* __restrict__ levels,
                                                                 const uint32_t* __restrict__ levels_last,
                                                                 const uint32_t* __restrict__ point_list,
                                                                 const float2* __restrict__ means2D,
                                                                 const float* __restrict__ features,
                                                                 const float4* __restrict__ conic_opacity,
                                                                 float* __restrict__ final_T,
                                                                 uint32_t* __restrict__ n_contrib,
                                                                 const float* __restrict__ bg,
                                                                 float* __restrict__ out_color, int foveaStep,
                                                                 int cull) {
    __shared__ float2 s_xy[64 * kWaves];
    __shared__ float4 s_co[64 * kWaves];
    __shared__ float4 s_rgb[64 * kWaves];
    __shared__ uint64_t s_bal[4 * kWaves];
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
    const uint32_t bx = (blockIdx.x >> 1) * 32 + ox, by = (blockIdx.y >> 1) * 32 + oy;
    const PixelSetT<kPPL> px = make_pixels_t<kPPL, kWaves>(W, H, bx, by, 2);
    const uint2 range = reinterpret_cast<const uint2*>(ranges)[tile];
    const BlendStateT<kPPL> st =
        blend_tile_t<kPPL, kWaves>(range, px, (float)bx, (float)by, 2.0f, point_list, means2D, features,
                                   conic_opacity, s_xy, s_co, s_rgb, s_bal, cull != 0);
    write_pixels(px, st, W, H, final_T, n_contrib, bg, out_color);
}

int g_amr_variant = 2;  // same geometries as the forward: 0 = 1 x 4 px, 1 = 2 x 2, 2 = 4 x 1
void set_amr_variant(int v) { g_amr_variant = v; }

void launch_amr_render(int W, int H, const ImageView& img, const uint32_t* levels, const uint32_t* levels_last,
                       const BinningView& b, const GeomView& g, const float* features, const float* bg,
                       float* out_color, int foveaStep, hipStream_t s) {
    const int tgx = (W + 31) / 32, tgy = (H + 31) / 32;
    if (tgx == 0 || tgy == 0) return;
#define GS_AMR_LAUNCH(PPL, WAVES)                                                                                  \
    hipLaunchKernelGGL((amr_render_kernel<PPL, WAVES>), dim3(2 * tgx, 2 * tgy), dim3(64 * WAVES), 0, s, W, H, tgx, \
                       img.ranges, levels, levels_last, b.point_list, reinterpret_cast<const float2*>(g.means2D),  \
                       features, reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib, \
                       bg, out_color, foveaStep, g_cull)
    switch (g_amr_variant) {
        case 0: GS_AMR_LAUNCH(4, 1); break;
        case 1: GS_AMR_LAUNCH(2, 2); break;
        default: GS_AMR_LAUNCH(1, 4); break;
    }
#undef GS_AMR_LAUNCH
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
