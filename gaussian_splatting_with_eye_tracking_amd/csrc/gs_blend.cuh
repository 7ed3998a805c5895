// gs_blend.cuh -- the wave64 tile blend shared by the base and AMR renderers.
//
// Mapping (MI355X-specific, replaces the reference's 16x16-thread block per
// tile, base/cr/forward.cu:261-374): ONE wave64 renders one 16x16 pixel
// block, each lane owning kPix = 4 pixels of a column, (x, y0 + 4k).  All 64
// lanes walk the same Gaussian j in lockstep, so a Gaussian's position /
// conic / colour is read once per lane (an LDS broadcast) and used for 4
// pixels, and block-level barriers become wave-level ballots.  Per-pixel
// semantics are exactly the reference's: contributor counting,
// last_contributor, the power>0 / alpha<1/255 skips and the T<1e-4 stop.
#pragma once

#include "gs_device.cuh"

namespace gsamd {

constexpr int kPix = 4;      // pixels per lane of the single-wave (backward) geometry
constexpr int kBatch = 64;   // Gaussians staged per LDS batch in the single-wave geometry

// A 16x16 block is covered by kWaves wave64s with kPPL pixels per lane
// (kWaves * 64 * kPPL = 256): thread t owns (x, y) = (t & 15, (t >> 4) + 4*kWaves*k).
template <int kPPL>
struct PixelSetT {
    float x;  // shared by the lane's pixels
    float y[kPPL];
    uint32_t pid[kPPL];
    bool inside[kPPL];
};
using PixelSet = PixelSetT<kPix>;

// 16x16 block at (ox, oy) with pixel stride `st` (1 = base, 2 = AMR sub-lattice).
template <int kPPL, int kWaves>
__device__ __forceinline__ PixelSetT<kPPL> make_pixels_t(int W, int H, uint32_t ox, uint32_t oy, uint32_t st) {
    const uint32_t t = threadIdx.x;
    PixelSetT<kPPL> p;
    const uint32_t px = ox + st * (t & 15);
    p.x = (float)px;
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
        const uint32_t py = oy + st * ((t >> 4) + 4 * kWaves * k);
        p.y[k] = (float)py;
        p.inside[k] = px < (uint32_t)W && py < (uint32_t)H;
        p.pid[k] = p.inside[k] ? (uint32_t)W * py + px : 0u;
    }
    return p;
}

__device__ __forceinline__ PixelSet make_pixels(int W, int H, uint32_t ox, uint32_t oy, uint32_t st) {
    return make_pixels_t<kPix, 1>(W, H, ox, oy, st);
}

template <int kPPL>
struct BlendStateT {
    float T[kPPL];
    float C[kPPL][3];
    uint32_t last[kPPL];
};

// Front-to-back blend of `range` for the thread's kPPL pixels.  Called by the
// whole workgroup (kWaves waves); LDS batches hold 64*kWaves Gaussians.
template <int kPPL, int kWaves>
__device__ __forceinline__ BlendStateT<kPPL> blend_tile_t(uint2 range, const PixelSetT<kPPL>& px,
                                                          const uint32_t* __restrict__ point_list,
                                                          const float2* __restrict__ means2D,
                                                          const float* __restrict__ features,
                                                          const float4* __restrict__ conic_opacity, float2* s_xy,
                                                          float4* s_co, float4* s_rgb) {
#pragma clang fp contract(fast)
    constexpr uint32_t kB = 64 * kWaves;
    const uint32_t tid = threadIdx.x;
    BlendStateT<kPPL> st;
    bool done[kPPL];
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
        st.T[k] = 1.0f;
        st.C[k][0] = st.C[k][1] = st.C[k][2] = 0.f;
        st.last[k] = 0;
        done[k] = !px.inside[k];
    }
    const uint32_t n = range.y - range.x;
    for (uint32_t b0 = 0; b0 < n; b0 += kB) {
        bool any = false;
#pragma unroll
        for (int k = 0; k < kPPL; k++) any |= !done[k];
        if (kWaves == 1) {
            if (__ballot(any) == 0ull) break;  // the whole tile is saturated
            __syncthreads();                     // single-wave workgroup: LDS fence only
        } else {
            if (!__syncthreads_or(any)) break;
        }
        if (b0 + tid < n) {
            const uint32_t id = point_list[range.x + b0 + tid];
            s_xy[tid] = means2D[id];
            s_co[tid] = conic_opacity[id];
            s_rgb[tid] = make_float4(features[3 * id], features[3 * id + 1], features[3 * id + 2], 0.f);
        }
        __syncthreads();
        const int cnt = (int)min(kB, n - b0);
        if (__ballot(any) == 0ull) continue;  // this wave is done; keep joining the barriers
        for (int j = 0; j < cnt; j++) {
            const float2 xy = s_xy[j];
            const float4 co = s_co[j];
            const float dx = xy.x - px.x;
            const uint32_t contributor = b0 + (uint32_t)j + 1;
            bool alive = false;
#pragma unroll
            for (int k = 0; k < kPPL; k++) {
                if (done[k]) continue;
                alive = true;
                const float dy = xy.y - px.y[k];
                const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                if (power > 0.0f) continue;
                const float alpha = fminf(0.99f, co.w * __expf(power));
                if (alpha < 1.0f / 255.0f) continue;
                const float test_T = st.T[k] * (1 - alpha);
                if (test_T < 0.0001f) {
                    done[k] = true;
                    continue;
                }
                const float4 f = s_rgb[j];
                const float w = alpha * st.T[k];
                st.C[k][0] += f.x * w;
                st.C[k][1] += f.y * w;
                st.C[k][2] += f.z * w;
                st.T[k] = test_T;
                st.last[k] = contributor;
            }
            if (__ballot(alive) == 0ull) break;
        }
    }
    return st;
}

// ------------------------------------------------------------ DPP reduce
// Sum over the 64 lanes; the total lands in lane 63 (row_shr 1,2,4,8 within
// 16-lane rows, then row_bcast:15 and row_bcast:31 -- gfx9 DPP).
__device__ __forceinline__ float dpp_sum_lane63(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xa, 0xf, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0xc, 0xf, false));
    return v;
}

// The same reduction for 9 values at once, as fused v_add_f32_dpp (hipcc
// fuses only a few of the mov_dpp + add pairs above).  Each stage walks the
// 9 registers, so a DPP source was written >= 9 VALU ops earlier (the gfx9
// VALU-write -> DPP-read hazard needs 2); the leading s_nop covers the
// compiler's last writes.  Must run with all 64 lanes active.
__device__ __forceinline__ void dpp_sum9_lane63(float (&g)[9]) {
    asm volatile(
        "s_nop 1\n"
        "v_add_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %2, %2, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %3, %3, %3 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %4, %4, %4 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %5, %5, %5 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %6, %6, %6 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %7, %7, %7 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %8, %8, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %2, %2, %2 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %3, %3, %3 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %4, %4, %4 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %5, %5, %5 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %6, %6, %6 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %7, %7, %7 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %8, %8, %8 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %2, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %3, %3, %3 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %4, %4, %4 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %5, %5, %5 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %6, %6, %6 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %7, %7, %7 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %8, %8, %8 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %2, %2, %2 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %3, %3, %3 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %4, %4, %4 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %5, %5, %5 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %6, %6, %6 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %7, %7, %7 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %8, %8, %8 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %2, %2, %2 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %3, %3, %3 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %4, %4, %4 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %5, %5, %5 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %6, %6, %6 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %7, %7, %7 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %8, %8, %8 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_add_f32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_add_f32_dpp %2, %2, %2 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_add_f32_dpp %3, %3, %3 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_add_f32_dpp %4, %4, %4 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_add_f32_dpp %5, %5, %5 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_add_f32_dpp %6, %6, %6 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_add_f32_dpp %7, %7, %7 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_add_f32_dpp %8, %8, %8 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), "+v"(g[6]), "+v"(g[7]),
          "+v"(g[8]));
}

}  // namespace gsamd
