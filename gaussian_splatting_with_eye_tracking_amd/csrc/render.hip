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
template <int kPPL, int kWaves, int kMinWaves = 1, int kSel = 0>
__global__ void __launch_bounds__(64 * kWaves, kMinWaves) render_fwd_kernel(int W, int H, const uint32_t* __restrict__ ranges,
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
                                                                 int xcd, float4* __restrict__ zero4,
                                                                 int zero_n4, uint32_t* __restrict__ bucket_count,
                                                                 uint32_t* __restrict__ bucket_list,
                                                                 uint8_t* __restrict__ hit_codes,
                                                                 uint32_t* __restrict__ hdr, int zero_nt) {
    // The backward's per-Gaussian accumulator rows (grad_accum, idle in the
    // base forward) are zeroed here, behind the blend, instead of by a memset
    // on the backward's critical path: fire-and-forget stores in a kernel
    // bound by VALU / LDS, not HBM (gs_api.cpp: accum_clean).  zero_nt: with
    // the non-temporal hint (the rows are next touched by the backward).
    typedef float f4v __attribute__((ext_vector_type(4)));
    for (int i = (int)(blockIdx.x * blockDim.x + threadIdx.x); i < zero_n4; i += (int)(gridDim.x * blockDim.x)) {
        if (zero_nt) __builtin_nontemporal_store(f4v{0.f, 0.f, 0.f, 0.f}, reinterpret_cast<f4v*>(zero4 + i));
        else zero4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __shared__ float4 s_a[64 * kWaves];
    __shared__ float4 s_co[64 * kWaves];
    __shared__ __attribute__((aligned(16))) float s_b[64 * kWaves * (kSel ? 4 : 1)];  // (kSel: 16-B stride)
    __shared__ uint64_t s_bal[(kSel >= 2 ? 5 : 4) * kWaves];  // (kSel >= 2: + the safe-form masks)
    __shared__ uint64_t s_hit[kWaves * kWaves];
    __shared__ uint32_t s_max;
    if (kWaves > 1 && threadIdx.x == 0) s_max = 0;
    // whether this forward leaves exact row-group hit codes for the backward
    // (the select-form 4 x 1 geometry records them; every other leaves 0)
    constexpr bool kRec = kSel && kPPL == 1;
    if (hdr && blockIdx.x == 0 && threadIdx.x == 0) hdr[kHdrHitCodes] = (kRec && hit_codes) ? 1u : 0u;
    const int tile = order ? (int)order[blockIdx.x]
                           : xcd ? xcd_block_tile((int)blockIdx.x, gx, (int)(gridDim.x / gx)) : (int)blockIdx.x;
    const uint32_t ox = (uint32_t)(tile % gx) * 16, oy = (uint32_t)(tile / gx) * 16;
    const PixelSetT<kPPL> px = make_pixels_t<kPPL, kWaves>(W, H, ox, oy, 1);
    const uint2 range = reinterpret_cast<const uint2*>(ranges)[tile];
    const BlendStateT<kPPL> st =
        blend_tile_t<kPPL, kWaves, kSel>(range, px, (float)ox, (float)oy, 1.0f, point_list,
                                   means2D, features, conic_opacity, s_a, s_co, s_b, s_bal, cull != 0,
                                   kRec ? hit_codes : nullptr, s_hit);
    write_pixels(px, st, W, H, final_T, n_contrib, bg, out_color);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < kPPL; k++) m = max(m, px.inside[k] ? st.last[k] : 0u);
    m = wave_max_u32(m);
    if (kWaves > 1) {
        if ((threadIdx.x & 63) == 0) atomicMax(&s_max, m);
        __syncthreads();
        m = s_max;
    }
    if (threadIdx.x == 0) {
        max_contrib[tile] = m;
        // the backward's heaviest-first launch order: this tile joins its work
        // bucket's list (render_bwd_kernel finds its tile from the counts; no
        // sort kernel between the passes)
        if (bucket_count) {
            const uint32_t b = order_bucket64(min(range.y - range.x, m));
            bucket_list[(size_t)b * gridDim.x + atomicAdd(&bucket_count[b], 1u)] = (uint32_t)tile;
        }
    }
}

int g_cull = 1;         // row-group cull on (gs_blend.cuh); 0 only for the exactness A/B test
// set_tuning("zero_nt"): the forward's grad_accum zeroing with the
// non-temporal hint (default; fwd + bwd step equal at config 2, 2.552 ->
// 2.540 ms at config 4 in the A/B tool, profiles/r04z5_ab_znt*.log)
int g_zero_nt = 1;
void set_zero_nt(int v) { g_zero_nt = v; }
int g_hit_codes = 1;    // the forward records exact row-group hit codes for the backward (set_tuning("hit_codes"))
void set_hit_codes(int v) { g_hit_codes = v; }
void set_cull(int v) { g_cull = v; }

// XCD-aware tile placement (gs_blend.cuh): bit 0 the forward blend, bit 1 the
// backward blend.  Measured at config 2 (profiles/r01g_xcd_ab.log): it halves
// the blend kernels' L2 -> fabric fetches (forward 770 -> 395 MB, backward
// 1100 -> 602 MB per launch) at the same forward time; the backward keeps the
// global heaviest-first order, 1.7 % faster than per-XCD heaviest-first
// (its XCD regions carry unequal work).  Default: forward only.
int g_xcd_map = 1;
void set_xcd_map(int v) { g_xcd_map = v; }

// 0: 1 wave x 4 px/lane, 1: 2 waves x 2 px/lane, 2: 4 waves x 1 px/lane; 3: 2 at <= 64 VGPRs (8 waves
// per SIMD: 0.307 -> 0.299 ms at config 2, profiles/r03c_ab_fwd_variant_cfg2.log); 5: 3 with the
// select-form blend (gs_blend.cuh blend_one_sel: 0.305 -> 0.277 ms at config 2, 0.237 -> 0.223 ms at
// config 4, profiles/r03d_ab_fwd_select_cfg{2,4}.log); 6: 5 at the default occupancy
// (an earlier variant 8, variant 5 with each visited bit cleared by s_andn2
// on the hit bit, measured equal: 0.2540 vs 0.2555 ms at config 2, 0.2235 vs
// 0.2227 at config 4, profiles/r04h_ab_fwd*; removed)
// 8: 5 without the `power > 0` test in 64-slot chunks whose visited entries
// are all splat_form_safe: 0.2511 -> 0.2441 ms at config 2, 0.1872 -> 0.1824
// at config 4 (profiles/r04o_ab_fwd*.log)
// 9 (default since round 4): 8 with the wave's exit tested after every pair
// of entries instead of every 64-slot chunk: config 2 equal (0.2456 /
// 0.2458 ms), config 4 0.1819 -> 0.1755 (profiles/r04z3_ab_fwd*.log)
constexpr int kDefaultFwdVariant = 9;
int g_fwd_variant = kDefaultFwdVariant;

void set_forward_variant(int v) { g_fwd_variant = v < 0 ? kDefaultFwdVariant : v; }

bool launch_render_forward(int W, int H, const ImageView& img, const BinningView& b, const GeomView& g,
                           const float* features, const float* bg, float* out_color, hipStream_t s,
                           float* zero_rows, size_t zero_floats, uint8_t* hit_codes) {
    const int gx = (W + 15) / 16, gy = (H + 15) / 16;
    if (gx == 0 || gy == 0) return false;
    float4* const zero4 = reinterpret_cast<float4*>(zero_rows);
    const int zero_n4 = (zero_rows && zero_floats / 4 <= (size_t)INT32_MAX) ? (int)(zero_floats / 4) : 0;
    // Row-major launch: heaviest-first by range length measured slower here
    // (early termination makes the range a poor work estimate); the backward
    // orders by max_contrib instead (backward.hip).
    const uint32_t* order = nullptr;
#define GS_FWD_LAUNCH(PPL, WAVES, ...)                                                                           \
    hipLaunchKernelGGL((render_fwd_kernel<PPL, WAVES, ##__VA_ARGS__>), dim3(gx * gy), dim3(64 * WAVES), 0, s, W, H, \
                       img.ranges, \
                       b.point_list, reinterpret_cast<const float2*>(g.means2D), features,                       \
                       reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib,         \
                       img.max_contrib, bg, out_color, g_cull, order, gx, g_xcd_map & 1, zero4, zero_n4,     \
                       img.bucket_count, img.bucket_list, g_hit_codes ? hit_codes : nullptr, g.hdr, g_zero_nt)
    switch (g_fwd_variant) {
        case 0: GS_FWD_LAUNCH(4, 1); break;
        case 1: GS_FWD_LAUNCH(2, 2); break;
        case 2: GS_FWD_LAUNCH(1, 4); break;
        case 3: GS_FWD_LAUNCH(1, 4, 8); break;  // <= 64 VGPRs: 8 waves per SIMD
        case 4: GS_FWD_LAUNCH(1, 4, 6); break;
        case 6: GS_FWD_LAUNCH(1, 4, 1, 1); break;
        case 7: GS_FWD_LAUNCH(1, 4, 8, 2); break;  // 5 with SGPR-mask selects (gs_blend.cuh blend_one_msk)
        case 5: GS_FWD_LAUNCH(1, 4, 8, 1); break;  // 3 + the select-form blend
        case 8: GS_FWD_LAUNCH(1, 4, 8, 3); break;
        default: GS_FWD_LAUNCH(1, 4, 8, 4); break;  // 9
    }
#undef GS_FWD_LAUNCH
    return zero_n4 > 0;
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
    __shared__ float4 s_a[64 * kWaves];
    __shared__ float4 s_co[64 * kWaves];
    __shared__ float s_b[64 * kWaves];
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
                                   conic_opacity, s_a, s_co, s_b, s_bal, cull != 0);
    write_pixels(px, st, W, H, final_T, n_contrib, bg, out_color);
}

// ------------------------------------------------- AMR quadrant sub-lists ---
// A 32-px AMR tile renders its 1024 pixels as four interleaved sub-lattices
// (rounds), each spread over the whole tile, so a (tile, round) block walks
// the tile's whole list.  Splitting by space instead: each 16x16 quadrant of
// the tile keeps the positions of the tile's entries whose alpha >= 1/255
// ellipse can reach it (splat_rect_hit, exact and conservative like the
// row-group cull), in list order.  Every skipped (pixel, entry) pair is one
// the reference skips with its alpha < 1/255 `continue`
// (amr/cr/forward.cu:470-472) while still counting it as a contributor, so a
// pixel blending the sub-list with each entry's ORIGINAL position as its
// contributor index gets the reference's colour, final T and n_contrib.
// One 256-thread workgroup per tile; ordered compaction by ballots.
constexpr int kQlThreads = 256;
constexpr int kQlPer = 4;  // entries per thread per pass: 1024 per pass, loads issued together
__global__ void __launch_bounds__(kQlThreads) amr_quad_lists_kernel(int tgx, const uint32_t* __restrict__ ranges,
                                                                    const uint32_t* __restrict__ point_list,
                                                                    const float2* __restrict__ means2D,
                                                                    const float4* __restrict__ conic_opacity,
                                                                    uint32_t* __restrict__ lists,
                                                                    uint32_t* __restrict__ quad_count) {
    constexpr int kW = kQlThreads / 64;
    __shared__ uint32_t s_cnt[kQlPer][4][kW];  // [pass slot][quadrant][wave] hits
    __shared__ uint32_t s_base[4];             // entries written per quadrant so far
    const int tile = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t beg = ranges[2 * tile];
    const int n = (int)(ranges[2 * tile + 1] - beg);
    const float ox = (float)((tile % tgx) * 32), oy = (float)((tile / tgx) * 32);
    uint32_t* out = lists + 4 * (size_t)beg;
    if (tid < 4) s_base[tid] = 0;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int c0 = 0; c0 < n; c0 += kQlThreads * kQlPer) {
        // slot e of thread t: entry c0 + e * 256 + t (slot-major keeps the
        // list order = (slot, wave, lane) order)
        float2 xy[kQlPer];
        float4 co[kQlPer];
#pragma unroll
        for (int e = 0; e < kQlPer; e++) {
            const int i = c0 + e * kQlThreads + tid;
            const uint32_t id = i < n ? point_list[beg + i] : 0u;
            xy[e] = i < n ? means2D[id] : make_float2(0.f, 0.f);
            co[e] = i < n ? conic_opacity[id] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        uint32_t m[kQlPer];
        uint64_t bal[kQlPer][4];
#pragma unroll
        for (int e = 0; e < kQlPer; e++) {
            const int i = c0 + e * kQlThreads + tid;
            m[e] = 0;
            if (i < n) {
                const SplatBox b = splat_box(xy[e], co[e]);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float x0 = ox + 16.0f * (float)(q & 1), y0 = oy + 16.0f * (float)(q >> 1);
                    if (splat_rect_hit(b, x0, x0 + 15.0f, y0, y0 + 15.0f)) m[e] |= 1u << q;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                bal[e][q] = __ballot((m[e] >> q) & 1u);
                if (lane == 0) s_cnt[e][q][wave] = (uint32_t)__popcll(bal[e][q]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t off = s_base[q];
#pragma unroll
            for (int e = 0; e < kQlPer; e++) {
                uint32_t mine = off + (uint32_t)__popcll(bal[e][q] & below);
#pragma unroll
                for (int w = 0; w < kW; w++) {
                    const uint32_t c = s_cnt[e][q][w];
                    mine += w < wave ? c : 0u;
                    off += c;
                }
                if ((m[e] >> q) & 1u) out[(size_t)q * n + mine] = (uint32_t)(c0 + e * kQlThreads + tid);
            }
        }
        __syncthreads();
        if (tid < 4) {
            uint32_t add = 0;
#pragma unroll
            for (int e = 0; e < kQlPer; e++)
#pragma unroll
                for (int w = 0; w < kW; w++) add += s_cnt[e][tid][w];
            s_base[tid] += add;
        }
        __syncthreads();
    }
    if (tid < 4) quad_count[4 * tile + tid] = s_base[tid];
}

void launch_amr_quad_lists(int W, int H, const ImageView& img, const BinningView& b, const GeomView& g, int K,
                           hipStream_t s) {
    const int tgx = (W + 31) / 32, tgy = (H + 31) / 32;
    if (tgx == 0 || tgy == 0) return;
    if (K == 0) {  // no lists to build; the counts must still read 0
        (void)hipMemsetAsync(img.quad_count, 0, sizeof(uint32_t) * 4 * (size_t)tgx * tgy, s);  // checked by the caller's stage_check
        return;
    }
    hipLaunchKernelGGL(amr_quad_lists_kernel, dim3(tgx * tgy), dim3(kQlThreads), 0, s, tgx, img.ranges, b.point_list,
                       reinterpret_cast<const float2*>(g.means2D), reinterpret_cast<const float4*>(g.conic_opacity),
                       quad_lists(b), img.quad_count);
}

// One wave per (tile, quadrant) unit, units in the tile order of the step-0
// launch (heaviest tiles first).  The unit renders the rounds r with
// lo < r <= L of its quadrant: the 8x8 points of sub-lattice r, one pixel
// per lane (kRounds = 1, the progressive steps: one round each, blended two
// entries per iteration), or all rounds of the unit at once, one pixel per
// lane and round (kRounds = 4, render_once).  Per pixel the blend is
// amr/cr/forward.cu:440-495 (base/cr/forward.cu:300-373) with contributor =
// the entry's position in the tile list + 1.
template <int kRounds>
__global__ void __launch_bounds__(64) amr_quad_render_kernel(int W, int H, int tgx, const uint32_t* __restrict__ order,
                                                             const uint32_t* __restrict__ ranges,
                                                             const uint32_t* __restrict__ lists,
                                                             const uint32_t* __restrict__ quad_count,
                                                             const uint32_t* __restrict__ levels,
                                                             const uint32_t* __restrict__ levels_last,
                                                             const uint32_t* __restrict__ point_list,
                                                             const float2* __restrict__ means2D,
                                                             const float* __restrict__ features,
                                                             const float4* __restrict__ conic_opacity,
                                                             float* __restrict__ final_T,
                                                             uint32_t* __restrict__ n_contrib,
                                                             const float* __restrict__ bg,
                                                             float* __restrict__ out_color, int foveaStep) {
#pragma clang fp contract(fast)
    __shared__ float2 s_xy[64];
    __shared__ float4 s_co[64];
    __shared__ float4 s_rgb[64];
    __shared__ uint32_t s_pos[64];
    const int tile = (int)order[blockIdx.x >> 2];
    const int q = (int)(blockIdx.x & 3);
    const uint32_t L_last = levels_last[tile];
    uint32_t L = levels[tile];
    // Block-uniform early exits (amr/cr/forward.cu:287-367).
    if (L <= L_last) return;
    if (L > 4) L = 4;
    const uint32_t lo = foveaStep > 0 ? L_last : 0u;  // rounds (lo, L]
    const uint32_t cnt = quad_count[4 * tile + q];
    const uint32_t beg = ranges[2 * tile];
    const uint32_t n = ranges[2 * tile + 1] - beg;
    const uint32_t* list = lists + 4 * (size_t)beg + (size_t)q * n;
    const uint32_t lane = threadIdx.x;
    const uint32_t ax = (uint32_t)(tile % tgx) * 32 + 16 * (q & 1) + 2 * (lane & 7);
    const uint32_t ay = (uint32_t)(tile / tgx) * 32 + 16 * (q >> 1) + 2 * (lane >> 3);
    const size_t plane = (size_t)H * W;
    const float b0 = bg[0], b1 = bg[1], b2 = bg[2];
    constexpr int kSlots = kRounds;
    // the rounds this launch renders: kRounds = 4 -> slot k = round k + 1;
    // kRounds = 1 -> one round per pass, passes over (lo, L]
    for (uint32_t r1 = lo + 1; r1 <= L; r1 += kRounds) {
        float pxx[kSlots], pxy[kSlots], T[kSlots], C[kSlots][3];
        uint32_t last[kSlots], pid[kSlots];
        bool done[kSlots], active[kSlots];
#pragma unroll
        for (int k = 0; k < kSlots; k++) {
            const uint32_t r = kRounds == 1 ? r1 : (uint32_t)k + 1;
            active[k] = r > lo && r <= L;  // wave-uniform
            // round -> sub-lattice offset (amr/cr/forward.cu:313-339): 1 (0,0), 2 (1,1), 3 (1,0), 4 (0,1)
            const uint32_t sx = (r == 2 || r == 3) ? 1u : 0u, sy = (r == 2 || r == 4) ? 1u : 0u;
            const uint32_t x = ax + sx, y = ay + sy;
            pxx[k] = (float)x;
            pxy[k] = (float)y;
            const bool in = active[k] && x < (uint32_t)W && y < (uint32_t)H;
            pid[k] = in ? (uint32_t)W * y + x : 0u;
            done[k] = !in;
            T[k] = 1.0f;
            C[k][0] = C[k][1] = C[k][2] = 0.f;
            last[k] = 0;
        }
        for (uint32_t b0i = 0; b0i < cnt; b0i += 64) {
            bool any = false;
#pragma unroll
            for (int k = 0; k < kSlots; k++) any |= !done[k];
            if (__ballot(any) == 0ull) break;  // every pixel of the unit saturated
            __syncthreads();                     // single-wave workgroup: LDS fence only
            if (b0i + lane < cnt) {
                const uint32_t pos = list[b0i + lane];
                const uint32_t id = point_list[beg + pos];
                s_pos[lane] = pos;
                s_xy[lane] = means2D[id];
                s_co[lane] = splat_coef(conic_opacity[id]);
                s_rgb[lane] = make_float4(features[3 * id], features[3 * id + 1], features[3 * id + 2], 0.f);
            }
            __syncthreads();
            const uint32_t m = min(64u, cnt - b0i);
            if constexpr (kRounds == 1) {
                // two entries per iteration: their LDS reads share one wait and
                // their alpha chains interleave; the blend stays in list order
                for (uint32_t j = 0; j < m; j += 2) {
                    const bool two = j + 1 < m;  // wave-uniform
                    const uint32_t jB = two ? j + 1 : j;
                    const float2 xyA = s_xy[j], xyB = s_xy[jB];
                    const float4 coA = s_co[j], coB = s_co[jB];
                    const float4 fA = s_rgb[j], fB = s_rgb[jB];
                    const uint32_t cA = s_pos[j] + 1, cB = s_pos[jB] + 1;
                    const float pA = splat_p2(xyA.x - pxx[0], xyA.y - pxy[0], coA);
                    const float pB = splat_p2(xyB.x - pxx[0], xyB.y - pxy[0], coB);
                    const float aA = fminf(0.99f, coA.w * splat_exp(pA));
                    const float aB = fminf(0.99f, coB.w * splat_exp(pB));
                    {
                        const float test_T = T[0] * (1 - aA);
                        const bool hit = !done[0] && !(pA > 0.0f) && !(aA < 1.0f / 255.0f);
                        const bool stop = hit && test_T < 0.0001f;
                        done[0] = done[0] || stop;
                        if (hit && !stop) {
                            const float w = aA * T[0];
                            C[0][0] = __builtin_fmaf(fA.x, w, C[0][0]);
                            C[0][1] = __builtin_fmaf(fA.y, w, C[0][1]);
                            C[0][2] = __builtin_fmaf(fA.z, w, C[0][2]);
                            T[0] = test_T;
                            last[0] = cA;
                        }
                    }
                    if (two) {
                        const float test_T = T[0] * (1 - aB);
                        const bool hit = !done[0] && !(pB > 0.0f) && !(aB < 1.0f / 255.0f);
                        const bool stop = hit && test_T < 0.0001f;
                        done[0] = done[0] || stop;
                        if (hit && !stop) {
                            const float w = aB * T[0];
                            C[0][0] = __builtin_fmaf(fB.x, w, C[0][0]);
                            C[0][1] = __builtin_fmaf(fB.y, w, C[0][1]);
                            C[0][2] = __builtin_fmaf(fB.z, w, C[0][2]);
                            T[0] = test_T;
                            last[0] = cB;
                        }
                    }
                    if (__ballot(!done[0]) == 0ull) break;
                }
            } else {
                for (uint32_t j = 0; j < m; j++) {
                    const float2 xy = s_xy[j];
                    const float4 co = s_co[j];
                    const uint32_t contributor = s_pos[j] + 1;
                    bool alive = false;
#pragma unroll
                    for (int k = 0; k < kSlots; k++) {
                        alive |= !done[k];
                        if (!active[k]) continue;  // wave-uniform
                        const float p = splat_p2(xy.x - pxx[k], xy.y - pxy[k], co);
                        const float alpha = fminf(0.99f, co.w * splat_exp(p));
                        const float test_T = T[k] * (1 - alpha);
                        const bool hit = !done[k] && !(p > 0.0f) && !(alpha < 1.0f / 255.0f);
                        const bool stop = hit && test_T < 0.0001f;
                        done[k] = done[k] || stop;
                        if (!hit || stop) continue;
                        const float4 f = s_rgb[j];
                        const float w = alpha * T[k];
                        C[k][0] = __builtin_fmaf(f.x, w, C[k][0]);
                        C[k][1] = __builtin_fmaf(f.y, w, C[k][1]);
                        C[k][2] = __builtin_fmaf(f.z, w, C[k][2]);
                        T[k] = test_T;
                        last[k] = contributor;
                    }
                    if (__ballot(alive) == 0ull) break;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kSlots; k++) {
            const uint32_t x = (uint32_t)pxx[k], y = (uint32_t)pxy[k];
            if (!active[k] || x >= (uint32_t)W || y >= (uint32_t)H) continue;
            const uint32_t p = pid[k];
            final_T[p] = T[k];
            n_contrib[p] = last[k];
            out_color[p] = C[k][0] + T[k] * b0;
            out_color[plane + p] = C[k][1] + T[k] * b1;
            out_color[2 * plane + p] = C[k][2] + T[k] * b2;
        }
    }
}

// ------------------------------------------------- AMR 8x8 region lists ---
// Variant 4.  The progressive steps are bound by their longest unit: a wave
// walks its sub-list serially, one entry after the other for each of its
// pixels, and a step ends when the heaviest unit ends (step 4 renders a tenth
// of step 1's pixels in more than half its time).  So the unit's chain is
// shortened twice:
//   * finer lists: a (tile, quadrant) wave is four 16-lane groups, each the
//     16 pixels of one 8x8 region (at the round's stride-2 offset) walking the
//     region's own sub-list -- the entries whose alpha >= 1/255 ellipse can
//     reach the region (splat_rect_hit, exact and conservative) keep their
//     ORIGINAL tile-list positions, so contributor indices, n_contrib and
//     final T are the reference's (amr/cr/forward.cu:440-495);
//   * no pointer chase: foveaStep 0 writes each instance's blend record in
//     tile-list order (AmrBinningView), so a batch is one coalesced position
//     load and tile-local record loads, issued one batch ahead.
// One 256-thread workgroup per tile builds the records and the 16 lists
// (ordered compaction by ballots, 256 entries per round).
constexpr int kRlThreads = 256;
// entries per thread per pass (loads issued together): kRlPer * 256 entries a
// pass (A/B at config 3, profiles/r02n_ab_lists_per.log: 2 -> 0.077 ms,
// 4 -> 0.083, 8 -> 0.083: occupancy beats per-thread memory parallelism)
int g_amr_lists_per = 2;
void set_amr_lists_per(int v) { g_amr_lists_per = v; }
// 1: workgroup b builds the lists of tile_order[b] (the steps' heaviest-first
// order, computed before the K copy) instead of tile b -- the heavy tiles'
// serial passes no longer start last (0.0792 -> 0.0758 ms at config 3,
// profiles/r04q_ab_lorder.log); 2 (default): XCD-compact strips
// (gs_blend.cuh xcd_block_tile: neighbouring tiles, which gather the same
// Gaussians' rows, share an XCD's L2): 0.0789 (1) -> 0.0765 ms with 48-B
// rows, tile order 0.0818 (profiles/r04z2_ab_lorder.log)
int g_amr_lists_order = 2;
void set_amr_lists_order(int v) { g_amr_lists_order = v; }
// Region mask of one entry: the exact ellipse test (splat_rect_hit) on the
// four 16x16 quadrants, refined to the 8x8 regions by the alpha >= 1/255
// ellipse's bounding box (both conservative).  Bit g = 4 row + col.
__device__ __forceinline__ uint32_t region_mask(float2 xy, float4 co, float ox, float oy) {
    const SplatBox b = splat_box(xy, co);
    uint32_t qm = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const float x0 = ox + 16.0f * (float)(q & 1), y0 = oy + 16.0f * (float)(q >> 1);
        if (splat_rect_hit(b, x0, x0 + 15.0f, y0, y0 + 15.0f)) qm |= 1u << q;
    }
    // box columns / rows (comparisons false for NaN / inf widths -> kept)
    uint32_t cm = 0, rm = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const float x0 = ox + 8.0f * (float)c, y0 = oy + 8.0f * (float)c;
        if (!(xy.x + b.hx < x0 || xy.x - b.hx > x0 + 7.0f)) cm |= 1u << c;
        if (!(xy.y + b.hy < y0 || xy.y - b.hy > y0 + 7.0f)) rm |= 1u << c;
    }
    uint32_t m = 0;
#pragma unroll
    for (int g = 0; g < 16; g++) {
        const int col = g & 3, row = g >> 2;
        const bool in = ((cm >> col) & 1u) && ((rm >> row) & 1u) && ((qm >> (2 * (row >> 1) + (col >> 1))) & 1u);
        m |= in ? 1u << g : 0u;
    }
    return m;
}

// rows: the per-Gaussian 48-B blend rows the AMR preprocess wrote into
// grad_accum (preprocess.hip): (x, y, r, g), splat_coef, (b, raw conic).
template <int kRlPer>
__global__ void __launch_bounds__(kRlThreads) amr_region_lists_kernel(int tgx, const uint32_t* __restrict__ ranges,
                                                                      const uint32_t* __restrict__ point_list,
                                                                      const float4* __restrict__ rows,
                                                                      float4* __restrict__ rec_a,
                                                                      float4* __restrict__ rec_b,
                                                                      float* __restrict__ rec_c,
                                                                      uint32_t* __restrict__ lists,
                                                                      uint32_t* __restrict__ region_count,
                                                                      uint32_t* __restrict__ tile_done,
                                                                      const uint32_t* __restrict__ order, int xcd,
                                                                      int tgy) {
    constexpr int kW = kRlThreads / 64;
    // per pass: hits of (slot e, region g, wave w), then their exclusive
    // offsets in the pass's (e, w) order, per region
    __shared__ uint32_t s_cnt[16][kRlPer * kW];
    __shared__ uint32_t s_base[16];  // entries written per region by earlier passes
    const int tile = order ? (int)order[blockIdx.x] : xcd ? xcd_block_tile((int)blockIdx.x, tgx, tgy) : (int)blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t beg = ranges[2 * tile];
    const int n = (int)(ranges[2 * tile + 1] - beg);
    const float ox = (float)((tile % tgx) * 32), oy = (float)((tile / tgx) * 32);
    uint32_t* out = lists + 16 * (size_t)beg;
    if (tid < 16) s_base[tid] = 0;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int c0 = 0; c0 < n; c0 += kRlThreads * kRlPer) {
        // slot e of thread t: entry c0 + e * 256 + t (slot-major keeps the
        // list order = (slot, wave, lane) order)
        uint32_t m[kRlPer];
#pragma unroll
        for (int e = 0; e < kRlPer; e++) {
            const int i = c0 + e * kRlThreads + tid;
            m[e] = 0;
            if (i < n) {
                const uint32_t id = point_list[beg + i];
                const float4* rr = rows + (size_t)(kGradRow / 4) * id;
                const float4 ra = rr[0], rb = rr[1], rc = rr[2];
                rec_a[beg + i] = ra;
                rec_b[beg + i] = rb;
                rec_c[beg + i] = rc.x;
                m[e] = region_mask(make_float2(ra.x, ra.y), make_float4(rc.y, rc.z, rc.w, rb.w), ox, oy);
            }
#pragma unroll
            for (int g = 0; g < 16; g++) {
                const uint32_t c = (uint32_t)__popcll(__ballot((m[e] >> g) & 1u));
                if (lane == 0) s_cnt[g][e * kW + wave] = c;
            }
        }
        __syncthreads();
        if (tid < 16) {  // exclusive scan of region tid's 16 counts, in list order
            uint32_t acc = s_base[tid];
#pragma unroll
            for (int k = 0; k < kRlPer * kW; k++) {
                const uint32_t c = s_cnt[tid][k];
                s_cnt[tid][k] = acc;
                acc += c;
            }
            s_base[tid] = acc;
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kRlPer; e++) {
            const int i = c0 + e * kRlThreads + tid;
#pragma unroll
            for (int g = 0; g < 16; g++) {
                const uint64_t bal = __ballot((m[e] >> g) & 1u);
                if ((m[e] >> g) & 1u)
                    out[(size_t)g * n + s_cnt[g][e * kW + wave] + (uint32_t)__popcll(bal & below)] = (uint32_t)i;
            }
        }
        __syncthreads();  // s_cnt is rewritten by the next pass
    }
    if (tid < 16) region_count[16 * tile + tid] = s_base[tid];
    if (tid == 0) tile_done[tile] = 0;  // the steps' unit counters start at 0 mod 4
}

void launch_amr_region_lists(int W, int H, const ImageView& img, const BinningView& b, const AmrBinningView& ab,
                             const GeomView& g, const float* features, int K, hipStream_t s) {
    const int tgx = (W + 31) / 32, tgy = (H + 31) / 32;
    if (tgx == 0 || tgy == 0) return;
    if (K == 0) {  // no lists to build; the counts must still read 0
        // (checked by the caller's stage_check)
        (void)hipMemsetAsync(img.region_count, 0, sizeof(uint32_t) * 16 * (size_t)tgx * tgy, s);
        (void)hipMemsetAsync(img.tile_done, 0, sizeof(uint32_t) * (size_t)tgx * tgy, s);
        return;
    }
    (void)features;  // in the rows (the preprocess saw colors_precomp / the SH colours)
#define GS_RL_LAUNCH(PER)                                                                                       \
    hipLaunchKernelGGL(amr_region_lists_kernel<PER>, dim3(tgx * tgy), dim3(kRlThreads), 0, s, tgx, img.ranges,     \
                       b.point_list, reinterpret_cast<const float4*>(g.grad_accum), ab.rec_a, ab.rec_b, ab.rec_c,  \
                       ab.region_lists, img.region_count, img.tile_done,                                  \
                       g_amr_lists_order == 1 ? img.tile_order : nullptr, g_amr_lists_order == 2 ? 1 : 0, tgy)
    switch (g_amr_lists_per) {
        case 2: GS_RL_LAUNCH(2); break;
        case 5: GS_RL_LAUNCH(5); break;
        case 8: GS_RL_LAUNCH(8); break;
        default: GS_RL_LAUNCH(4); break;
    }
#undef GS_RL_LAUNCH
}

// One wave per (tile, quadrant): its four 16-lane groups are the quadrant's
// four 8x8 regions, lane (i, j) of a group the region pixel (2i, 2j) + the
// round's sub-lattice offset.  Waves b = 8 k + x (one XCD) take tile-order
// positions 8 (k / 4) + x, quadrant k % 4: the four waves of a tile share one
// XCD's L2 for its records, heaviest tiles first.  kRounds as in
// amr_quad_render_kernel (1: the progressive steps, one round per pass; 4:
// render_once, one pixel per lane and round).  feats_override (steps >= 1
// given colors_precomp): colours from it through point_list instead of the
// step-0 records.
// kPer: entries each lane stages per batch (a group stages 16 kPer)
template <int kRounds, int kPer, int kFold = 0, int kSelF = 0>
__global__ void __launch_bounds__(64) amr_region_render_kernel(
    int W, int H, int tgx, int T, const uint32_t* __restrict__ order, const uint32_t* __restrict__ ranges,
    const uint32_t* __restrict__ lists, const uint32_t* __restrict__ region_count,
    const uint32_t* __restrict__ levels, const uint32_t* __restrict__ levels_last, const float4* __restrict__ rec_a,
    const float4* __restrict__ rec_b, const float* __restrict__ rec_c, const uint32_t* __restrict__ point_list,
    const float* __restrict__ feats_override, float* __restrict__ final_T, uint32_t* __restrict__ n_contrib,
    const float* __restrict__ bg, float* __restrict__ out_color, int foveaStep, int scramble,
    uint32_t* __restrict__ lv_current, uint32_t* __restrict__ lv_last, uint32_t* __restrict__ tile_done, int P,
    int* __restrict__ zero_radii) {
#pragma clang fp contract(fast)
    constexpr int kRgBatch = 16 * kPer;
    __shared__ float4 s_a[4][kRgBatch];
    __shared__ float4 s_b[4][kRgBatch];
    __shared__ __attribute__((aligned(16))) float s_c[4][kRgBatch];  // (b128 reads of 4 entries)
    __shared__ __attribute__((aligned(16))) uint32_t s_pos[4][kRgBatch];
    const uint32_t bid = blockIdx.x, slot = bid >> 3;
    // the step's zero radii (the reference's torch::full(0) for steps >= 1)
    if (zero_radii)
        for (int i = (int)(bid * 64 + threadIdx.x); i < P; i += (int)(gridDim.x * 64)) zero_radii[i] = 0;
    const int p = (int)(8 * (slot >> 2) + (bid & 7));
    if (p >= T) return;
    // scramble (A/B): a fixed permutation of the tile order (1031 is prime,
    // so p -> 1031 p mod T is one whenever T is not a multiple of 1031)
    const int tile = (int)order[scramble && T % 1031 != 0 ? (int)((1031ull * (uint32_t)p) % (uint32_t)T) : p];
    const int q = (int)(slot & 3);
    const uint32_t lane = threadIdx.x, h = lane >> 4, l16 = lane & 15;
    const uint32_t gcol = 2 * (q & 1) + (h & 1), grow = 2 * (q >> 1) + (h >> 1);
    const uint32_t g = 4 * grow + gcol;
    const uint32_t ax = (uint32_t)(tile % tgx) * 32 + 8 * gcol + 2 * (l16 & 3);
    const uint32_t ay = (uint32_t)(tile / tgx) * 32 + 8 * grow + 2 * (l16 >> 2);
    const size_t plane = (size_t)H * W;
    // The call's image is zero wherever it renders nothing (the reference's
    // zero-filled out_color, amr/rasterize_points.cu), so the unit writes its
    // whole 16x16 quadrant: colours go to an LDS copy of the quadrant (zero
    // where this call renders nothing), stored at the end as 64-B row
    // segments (lane = row * 4 + 4-pixel chunk), so the caller needs no fill
    // and the image stores are coalesced.
    __shared__ float s_out[3][16][16];
    const uint32_t qx0 = (uint32_t)(tile % tgx) * 32 + 16 * (q & 1), qy0 = (uint32_t)(tile / tgx) * 32 + 16 * (q >> 1);
    const uint32_t orow = lane >> 2, ocol = 4 * (lane & 3);
    auto store_quadrant = [&](bool zero) {
        const uint32_t y = qy0 + orow, x = qx0 + ocol;
        if (y >= (uint32_t)H) return;
        const size_t pp = (size_t)W * y + x;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            const float4 v = zero ? make_float4(0.f, 0.f, 0.f, 0.f)
                                  : *reinterpret_cast<const float4*>(&s_out[ch][orow][ocol]);
            float* dst = out_color + ch * plane + pp;
            if ((W & 3) == 0 && x + 3 < (uint32_t)W) {
                *reinterpret_cast<float4*>(dst) = v;
            } else {
                if (x < (uint32_t)W) dst[0] = v.x;
                if (x + 1 < (uint32_t)W) dst[1] = v.y;
                if (x + 2 < (uint32_t)W) dst[2] = v.z;
                if (x + 3 < (uint32_t)W) dst[3] = v.w;
            }
        }
    };
    // Fused step levels (lv_current given, the progressive steps): the
    // reference's per-step level update (amr.hip fovea_levels_kernel,
    // amr/cr/rasterizer_impl.cu's tile_AMR_levels_last / _current) evaluated
    // by each of the tile's four units from the previous current level; the
    // last unit of the tile to finish stores it (tile_done counts units mod 4),
    // so every unit has read the previous value before it is replaced.
    uint32_t L_last, L;
    if (lv_current) {
        const uint32_t Lp = levels[tile], prev = lv_current[tile];
        if (foveaStep == 1) {
            L_last = 0;
            L = Lp >= 1u ? 1u : 0u;
        } else if (foveaStep <= 4) {
            L_last = prev;
            L = Lp >= (uint32_t)foveaStep ? (uint32_t)foveaStep : prev;
        } else {
            L_last = 0;
            L = Lp;
        }
    } else {
        L_last = levels_last[tile];
        L = levels[tile];
    }
    const uint32_t L_store = L;
    auto finish_unit = [&]() {
        if (lv_current && threadIdx.x == 0) {
            if ((atomicAdd(&tile_done[tile], 1u) & 3u) == 3u) {
                lv_last[tile] = L_last;
                lv_current[tile] = L_store;
            }
        }
    };
    // Block-uniform early exits (amr/cr/forward.cu:287-367).
    if (L <= L_last) {
        store_quadrant(true);
        finish_unit();
        return;
    }
    if (L > 4) L = 4;
    const uint32_t lo = foveaStep > 0 ? L_last : 0u;  // rounds (lo, L]
#pragma unroll
    for (int ch = 0; ch < 3; ch++)
        *reinterpret_cast<float4*>(&s_out[ch][orow][ocol]) = make_float4(0.f, 0.f, 0.f, 0.f);
    const uint32_t beg = ranges[2 * tile];
    const uint32_t n = ranges[2 * tile + 1] - beg;
    const uint32_t cnt = region_count[16 * tile + g];  // uniform per group
    // the wave's longest list (lanes 0, 16, 32, 48 hold the four counts)
    const uint32_t cmax = max(max((uint32_t)__builtin_amdgcn_readlane((int)cnt, 0),
                                  (uint32_t)__builtin_amdgcn_readlane((int)cnt, 16)),
                              max((uint32_t)__builtin_amdgcn_readlane((int)cnt, 32),
                                  (uint32_t)__builtin_amdgcn_readlane((int)cnt, 48)));
    const uint32_t* list = lists + 16 * (size_t)beg + (size_t)g * n;
    const float b0c = bg[0], b1c = bg[1], b2c = bg[2];
    constexpr int kSlots = kRounds;
    // staging: lane l16 of group h loads entries l16 + 16 u (u < kPer) of each batch
    auto load_pos = [&](uint32_t b0, uint32_t (&pos)[kPer]) {
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            const uint32_t i = b0 + l16 + 16 * u;
            pos[u] = i < cnt ? list[i] : 0xffffffffu;
        }
    };
    // kSelF 2: whether every staged entry of the wave's batch has a provably
    // negative-definite form (splat_form_safe: no power > 0 test needed)
    const float tox = (float)((tile % tgx) * 32), toy = (float)((tile / tgx) * 32);
    auto load_rec = [&](const uint32_t (&pos)[kPer], float4 (&a)[kPer], float4 (&bb)[kPer], float (&c)[kPer]) {
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            if (kSelF && pos[u] == 0xffffffffu) {
                // kSelF: past the group's list an all-zero record (p = 0,
                // alpha = 0 * exp2(0) = 0: rejected by the alpha test), so the
                // fold needs no per-entry bound test
                a[u] = bb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                c[u] = 0.f;
            }
            if (pos[u] != 0xffffffffu) {
                a[u] = rec_a[beg + pos[u]];
                bb[u] = rec_b[beg + pos[u]];
                c[u] = rec_c[beg + pos[u]];
                if (feats_override) {
                    const uint32_t id = point_list[beg + pos[u]];
                    a[u].z = feats_override[3 * id];
                    a[u].w = feats_override[3 * id + 1];
                    c[u] = feats_override[3 * id + 2];
                }
            }
        }
    };
    for (uint32_t r1 = lo + 1; r1 <= L; r1 += kRounds) {
        float pxx[kSlots], pxy[kSlots], T_[kSlots], C[kSlots][3];
        uint32_t last[kSlots], pid[kSlots];
        bool done[kSlots], active[kSlots];
#pragma unroll
        for (int k = 0; k < kSlots; k++) {
            const uint32_t r = kRounds == 1 ? r1 : (uint32_t)k + 1;
            active[k] = r > lo && r <= L;  // wave-uniform
            // round -> sub-lattice offset (amr/cr/forward.cu:313-339): 1 (0,0), 2 (1,1), 3 (1,0), 4 (0,1)
            const uint32_t sx = (r == 2 || r == 3) ? 1u : 0u, sy = (r == 2 || r == 4) ? 1u : 0u;
            const uint32_t x = ax + sx, y = ay + sy;
            pxx[k] = (float)x;
            pxy[k] = (float)y;
            const bool in = active[k] && x < (uint32_t)W && y < (uint32_t)H;
            pid[k] = in ? (uint32_t)W * y + x : 0u;
            done[k] = !in;
            T_[k] = (kSelF && !in) ? -1.0f : 1.0f;  // (kSelF: a finished pixel carries a negative T)
            C[k][0] = C[k][1] = C[k][2] = 0.f;
            last[k] = 0;
        }
        uint32_t pos[kPer], npos[kPer];
        float4 ra[kPer], rb[kPer];
        float rc[kPer];
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            ra[u] = rb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            rc[u] = 0.f;
        }
        load_pos(0, pos);
        load_rec(pos, ra, rb, rc);
        load_pos(kRgBatch, npos);
        for (uint32_t b0 = 0; b0 < cmax; b0 += kRgBatch) {
            bool any = false;
#pragma unroll
            for (int k = 0; k < kSlots; k++) any |= (kSelF ? T_[k] > 0.0f : !done[k]) && b0 < cnt;
            if (__ballot(any) == 0ull) break;  // every pixel saturated or its list exhausted
            __syncthreads();                     // single-wave workgroup: LDS fence only
#pragma unroll
            for (int u = 0; u < kPer; u++) {
                s_a[h][l16 + 16 * u] = ra[u];
                s_b[h][l16 + 16 * u] = rb[u];
                s_c[h][l16 + 16 * u] = rc[u];
                s_pos[h][l16 + 16 * u] = kSelF ? pos[u] + 1 : pos[u];  // (kSelF: the contributor index)
            }
            bool batch_safe = false;
            if constexpr (kSelF == 2) {
                bool unsafe = false;
#pragma unroll
                for (int u = 0; u < kPer; u++)  // (past-the-list zero records: p = 0, alpha 0 -- no test needed)
                    unsafe |= pos[u] != 0xffffffffu &&
                              !splat_form_safe(rb[u], fabsf(ra[u].x - tox), fabsf(ra[u].y - toy));
                batch_safe = __ballot(unsafe) == 0ull;
            }
            __syncthreads();
            // the next batch's records and the one after's positions, in flight
            // while this batch is blended
#pragma unroll
            for (int u = 0; u < kPer; u++) pos[u] = npos[u];
            load_rec(pos, ra, rb, rc);
            load_pos(b0 + 2 * kRgBatch, npos);
            // entries of this batch: [0, m) for the group, [0, mw) for the wave
            const int m = (int)min((uint32_t)kRgBatch, cnt > b0 ? cnt - b0 : 0u);
            const int mw = (int)min((uint32_t)kRgBatch, cmax - b0);
            if constexpr (kFold > 0 && kSelF == 2) {
                // kSelF 1 with every select on an SGPR-pair lane mask
                // (gs_blend.cuh gs_sel_*): phase 1 keeps each entry's accept mask
                // (alpha >= 1/255, and power <= 0 unless the batch is all
                // provably negative definite), phase 2 the stop mask; blended =
                // accept & !stop -- the lanes of kSelF 1's av != 0.
#pragma unroll
                for (int j0 = 0; j0 < kRgBatch; j0 += kFold) {
                    float al[kFold][kSlots];
                    uint64_t accm[kFold][kSlots];
                    float fr[kFold], fg[kFold], fb[kFold];
                    uint32_t fp[kFold];
#pragma unroll
                    for (int e4 = 0; e4 < kFold; e4 += 4) {
                        const float4 b4 = *reinterpret_cast<const float4*>(&s_c[h][j0 + e4]);
                        const uint4 p4 = *reinterpret_cast<const uint4*>(&s_pos[h][j0 + e4]);
                        fb[e4] = b4.x; fb[e4 + 1] = b4.y; fb[e4 + 2] = b4.z; fb[e4 + 3] = b4.w;
                        fp[e4] = p4.x; fp[e4 + 1] = p4.y; fp[e4 + 2] = p4.z; fp[e4 + 3] = p4.w;
                    }
#pragma unroll
                    for (int e = 0; e < kFold; e++) {
                        const int j = j0 + e;
                        const float4 a = s_a[h][j];
                        const float4 co = s_b[h][j];
                        fr[e] = a.z;
                        fg[e] = a.w;
#pragma unroll
                        for (int k = 0; k < kSlots; k++) {
                            if (kRounds > 1 && !active[k]) continue;  // wave-uniform (always on for one round)
                            const float pw = splat_p2(a.x - pxx[k], a.y - pxy[k], co);
                            const float av = fminf(0.99f, co.w * splat_exp(pw));
                            uint64_t am = __builtin_amdgcn_fcmpf(av, 1.0f / 255.0f, kFcmpUGE);
                            if (!batch_safe) am &= __builtin_amdgcn_fcmpf(pw, 0.0f, kFcmpULE);
                            accm[e][k] = am;
                            al[e][k] = gs_sel_v(am, av, 0.0f);
                        }
                    }
                    bool alive = false;
#pragma unroll
                    for (int e = 0; e < kFold; e++) {
#pragma unroll
                        for (int k = 0; k < kSlots; k++) {
                            if (kRounds > 1 && !active[k]) continue;
                            const float test_T = T_[k] * (1.0f - al[e][k]);
                            const uint64_t stop = __builtin_amdgcn_fcmpf(test_T, 0.0001f, kFcmpOLT);
                            const uint64_t blended = accm[e][k] & ~stop;
                            const float w = gs_sel_s(blended, al[e][k], 0.0f) * T_[k];
                            C[k][0] = __builtin_fmaf(fr[e], w, C[k][0]);
                            C[k][1] = __builtin_fmaf(fg[e], w, C[k][1]);
                            C[k][2] = __builtin_fmaf(fb[e], w, C[k][2]);
                            T_[k] = gs_sel_v_negabs(stop, T_[k], test_T);
                            last[k] = gs_sel_s_u32(blended, fp[e], last[k]);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < kSlots; k++) alive |= T_[k] > 0.0f && j0 + kFold < m;
                    if (j0 + kFold < kRgBatch && __ballot(alive) == 0ull) break;
                }
            } else if constexpr (kFold > 0 && kSelF) {
                // The fold of blend_one_sel2 (gs_blend.cuh): phase 1 turns each
                // staged entry's alpha into its select-form value (0 when the
                // reference skips the pair: power > 0 or alpha < 1/255; entries
                // past the group's list are zero records), phase 2 folds them
                // front to back with the finished state in T's sign -- no
                // per-entry exec masks or bound tests, the same bits for every
                // pixel still blending.  (Dropping the power > 0 select in
                // provably safe batches, the forward's variant 8 form, measured
                // equal here: 0.0583 ms either way, profiles/r04q_ab_sel.log.)
#pragma unroll
                for (int j0 = 0; j0 < kRgBatch; j0 += kFold) {
                    float al[kFold][kSlots];
                    float fr[kFold], fg[kFold], fb[kFold];
                    uint32_t fp[kFold];
#pragma unroll
                    for (int e4 = 0; e4 < kFold; e4 += 4) {
                        const float4 b4 = *reinterpret_cast<const float4*>(&s_c[h][j0 + e4]);
                        const uint4 p4 = *reinterpret_cast<const uint4*>(&s_pos[h][j0 + e4]);
                        fb[e4] = b4.x; fb[e4 + 1] = b4.y; fb[e4 + 2] = b4.z; fb[e4 + 3] = b4.w;
                        fp[e4] = p4.x; fp[e4 + 1] = p4.y; fp[e4 + 2] = p4.z; fp[e4 + 3] = p4.w;
                    }
#pragma unroll
                    for (int e = 0; e < kFold; e++) {
                        const int j = j0 + e;
                        const float4 a = s_a[h][j];
                        const float4 co = s_b[h][j];
                        fr[e] = a.z;
                        fg[e] = a.w;
#pragma unroll
                        for (int k = 0; k < kSlots; k++) {
                            if (kRounds > 1 && !active[k]) continue;  // wave-uniform (always on for one round)
                            const float pw = splat_p2(a.x - pxx[k], a.y - pxy[k], co);
                            float av = fminf(0.99f, co.w * splat_exp(pw));
                            av = (pw > 0.0f) ? 0.0f : av;
                            av = (av < 1.0f / 255.0f) ? 0.0f : av;
                            al[e][k] = av;
                        }
                    }
                    bool alive = false;
#pragma unroll
                    for (int e = 0; e < kFold; e++) {
#pragma unroll
                        for (int k = 0; k < kSlots; k++) {
                            if (kRounds > 1 && !active[k]) continue;
                            float av = al[e][k];
                            const float test_T = T_[k] * (1.0f - av);
                            const bool stop = test_T < 0.0001f;  // every finished pixel too (T < 0)
                            av = stop ? 0.0f : av;
                            const float w = av * T_[k];
                            C[k][0] = __builtin_fmaf(fr[e], w, C[k][0]);
                            C[k][1] = __builtin_fmaf(fg[e], w, C[k][1]);
                            C[k][2] = __builtin_fmaf(fb[e], w, C[k][2]);
                            T_[k] = stop ? -fabsf(T_[k]) : test_T;
                            // (as a bit-field insert under an all-ones mask: written
                            // as a select, the compiler sinks the move into an
                            // exec-masked branch, 3 SALU + 1 VALU per entry)
                            const uint32_t lm = av != 0.0f ? ~0u : 0u;
                            last[k] = (fp[e] & lm) | (last[k] & ~lm);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < kSlots; k++) alive |= T_[k] > 0.0f && j0 + kFold < m;
                    if (j0 + kFold < kRgBatch && __ballot(alive) == 0ull) break;
                }
            } else if constexpr (kFold > 0) {
                // Two phases per sub-batch of kFold entries.  The alpha of
                // every staged entry does not depend on T, so phase 1
                // evaluates them as independent chains (full issue rate even
                // with one wave per SIMD, the late steps' case); phase 2 is the
                // reference's front-to-back fold in list order, a few
                // dependent ops per entry.  Same operations on the same
                // operands as the one-entry loop: same bits.
#pragma unroll
                for (int j0 = 0; j0 < kRgBatch; j0 += kFold) {
                    float al[kFold][kSlots];
                    uint32_t okm[kSlots];  // entries j < m passing the alpha tests
                    // the fold's colour and position of each entry, read once
                    // here (the group's LDS reads are broadcasts, and at one
                    // entry per pixel per step the LDS array, not the VALU,
                    // is the busier unit): (r, g) from the record read the
                    // alpha needs, b and the position four entries per b128
                    float fr[kFold], fg[kFold], fb[kFold];
                    uint32_t fp[kFold];
#pragma unroll
                    for (int e4 = 0; e4 < kFold; e4 += 4) {
                        const float4 b4 = *reinterpret_cast<const float4*>(&s_c[h][j0 + e4]);
                        const uint4 p4 = *reinterpret_cast<const uint4*>(&s_pos[h][j0 + e4]);
                        fb[e4] = b4.x; fb[e4 + 1] = b4.y; fb[e4 + 2] = b4.z; fb[e4 + 3] = b4.w;
                        fp[e4] = p4.x; fp[e4 + 1] = p4.y; fp[e4 + 2] = p4.z; fp[e4 + 3] = p4.w;
                    }
#pragma unroll
                    for (int k = 0; k < kSlots; k++) okm[k] = 0;
#pragma unroll
                    for (int e = 0; e < kFold; e++) {
                        const int j = j0 + e;
                        const float4 a = s_a[h][j];
                        const float4 co = s_b[h][j];
                        fr[e] = a.z;
                        fg[e] = a.w;
#pragma unroll
                        for (int k = 0; k < kSlots; k++) {
                            if (!active[k]) continue;  // wave-uniform
                            const float pw = splat_p2(a.x - pxx[k], a.y - pxy[k], co);
                            al[e][k] = fminf(0.99f, co.w * splat_exp(pw));
                            okm[k] |= (j < m && !(pw > 0.0f) && !(al[e][k] < 1.0f / 255.0f)) ? 1u << e : 0u;
                        }
                    }
                    bool alive = false;
#pragma unroll
                    for (int e = 0; e < kFold; e++) {
#pragma unroll
                        for (int k = 0; k < kSlots; k++) {
                            if (!active[k]) continue;
                            const float test_T = T_[k] * (1 - al[e][k]);
                            const bool hit = ((okm[k] >> e) & 1u) && !done[k];
                            const bool stop = hit && test_T < 0.0001f;
                            done[k] = done[k] || stop;
                            if (hit && !stop) {
                                const float w = al[e][k] * T_[k];
                                C[k][0] = __builtin_fmaf(fr[e], w, C[k][0]);
                                C[k][1] = __builtin_fmaf(fg[e], w, C[k][1]);
                                C[k][2] = __builtin_fmaf(fb[e], w, C[k][2]);
                                T_[k] = test_T;
                                last[k] = fp[e] + 1;
                            }
                        }
                    }
#pragma unroll
                    for (int k = 0; k < kSlots; k++) alive |= !done[k] && j0 + kFold < m;
                    if (j0 + kFold < kRgBatch && __ballot(alive) == 0ull) break;
                }
            } else if constexpr (kRounds == 1) {
                // two entries per iteration: their LDS reads share one wait and
                // their alpha chains interleave; the blend stays in list order
                for (int j = 0; j < mw; j += 2) {
                    const int jB = j + 1 < mw ? j + 1 : j;
                    const bool okA = j < m, okB = j + 1 < m;
                    const float4 aA = s_a[h][j], aB = s_a[h][jB];
                    const float4 coA = s_b[h][j], coB = s_b[h][jB];
                    const float cA_ = s_c[h][j], cB_ = s_c[h][jB];
                    const uint32_t cA = s_pos[h][j] + 1, cB = s_pos[h][jB] + 1;
                    const float pA = splat_p2(aA.x - pxx[0], aA.y - pxy[0], coA);
                    const float pB = splat_p2(aB.x - pxx[0], aB.y - pxy[0], coB);
                    const float alA = fminf(0.99f, coA.w * splat_exp(pA));
                    const float alB = fminf(0.99f, coB.w * splat_exp(pB));
                    {
                        const float test_T = T_[0] * (1 - alA);
                        const bool hit = okA && !done[0] && !(pA > 0.0f) && !(alA < 1.0f / 255.0f);
                        const bool stop = hit && test_T < 0.0001f;
                        done[0] = done[0] || stop;
                        if (hit && !stop) {
                            const float w = alA * T_[0];
                            C[0][0] = __builtin_fmaf(aA.z, w, C[0][0]);
                            C[0][1] = __builtin_fmaf(aA.w, w, C[0][1]);
                            C[0][2] = __builtin_fmaf(cA_, w, C[0][2]);
                            T_[0] = test_T;
                            last[0] = cA;
                        }
                    }
                    {
                        const float test_T = T_[0] * (1 - alB);
                        const bool hit = okB && !done[0] && !(pB > 0.0f) && !(alB < 1.0f / 255.0f);
                        const bool stop = hit && test_T < 0.0001f;
                        done[0] = done[0] || stop;
                        if (hit && !stop) {
                            const float w = alB * T_[0];
                            C[0][0] = __builtin_fmaf(aB.z, w, C[0][0]);
                            C[0][1] = __builtin_fmaf(aB.w, w, C[0][1]);
                            C[0][2] = __builtin_fmaf(cB_, w, C[0][2]);
                            T_[0] = test_T;
                            last[0] = cB;
                        }
                    }
                    if (__ballot(!done[0] && j + 2 < m) == 0ull) break;
                }
            } else {
                for (int j = 0; j < mw; j++) {
                    const float4 a = s_a[h][j];
                    const float4 co = s_b[h][j];
                    const uint32_t contributor = s_pos[h][j] + 1;
                    const bool okj = j < m;
                    bool alive = false;
#pragma unroll
                    for (int k = 0; k < kSlots; k++) {
                        if (!active[k]) continue;  // wave-uniform
                        const float pw = splat_p2(a.x - pxx[k], a.y - pxy[k], co);
                        const float alpha = fminf(0.99f, co.w * splat_exp(pw));
                        const float test_T = T_[k] * (1 - alpha);
                        const bool hit = okj && !done[k] && !(pw > 0.0f) && !(alpha < 1.0f / 255.0f);
                        const bool stop = hit && test_T < 0.0001f;
                        done[k] = done[k] || stop;
                        alive |= !done[k] && j + 1 < m;
                        if (!hit || stop) continue;
                        const float w = alpha * T_[k];
                        C[k][0] = __builtin_fmaf(a.z, w, C[k][0]);
                        C[k][1] = __builtin_fmaf(a.w, w, C[k][1]);
                        C[k][2] = __builtin_fmaf(s_c[h][j], w, C[k][2]);
                        T_[k] = test_T;
                        last[k] = contributor;
                    }
                    if (__ballot(alive) == 0ull) break;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kSlots; k++) {
            const uint32_t x = (uint32_t)pxx[k], y = (uint32_t)pxy[k];
            if (!active[k] || x >= (uint32_t)W || y >= (uint32_t)H) continue;
            const uint32_t pp = pid[k];
            if (kSelF) T_[k] = fabsf(T_[k]);
            final_T[pp] = T_[k];
            n_contrib[pp] = last[k];
            const uint32_t lx = x - qx0, ly = y - qy0;
            s_out[0][ly][lx] = C[k][0] + T_[k] * b0c;
            s_out[1][ly][lx] = C[k][1] + T_[k] * b1c;
            s_out[2][ly][lx] = C[k][2] + T_[k] * b2c;
        }
    }
    __syncthreads();  // single-wave workgroup: LDS fence only
    store_quadrant(false);
    finish_unit();
}

int g_amr_variant = 4;  // 4: 8x8 region sub-lists + records (default); 3: quadrant sub-lists; 0 = 1 x 4 px, 1 = 2 x 2, 2 = 4 x 1 full-list blocks
void set_amr_variant(int v) { g_amr_variant = v; }
int g_amr_scramble = 0;  // variant 4: 1 = units in a scrambled (not heaviest-first) tile order
void set_amr_scramble(int v) { g_amr_scramble = v; }
int g_amr_batch = 1;  // variant 4: entries staged per lane and batch (1 or 2)
void set_amr_batch(int v) { g_amr_batch = v == 2 ? 2 : 1; }
// variant 4: bit k set = foveaStep k (bit 0: render_once) uses the
// alpha-phase + fold-phase sub-batches; bit 5 = 16-entry sub-batches for the
// steps (else 8)
// variant 4 + fold: bit k set = foveaStep k stages 32 entries per batch
// (two per lane: one batch of records in flight covers twice the blend work)
int g_amr_deep = 0;
void set_amr_deep(int v) { g_amr_deep = v; }
int g_amr_fold = 0x1e;
// the fold in the select form (amr_region_render_kernel kSelF): 1 compiler
// selects, 2 SGPR-mask selects (gs_blend.cuh gs_sel_*)
int g_amr_sel = 1;
void set_amr_sel(int v) { g_amr_sel = v; }
int g_amr_fold_n = 8;
void set_amr_fold(int v) {
    g_amr_fold = v & 0x1f;
    g_amr_fold_n = (v & 0x20) ? 16 : 8;
}

void launch_amr_render(int W, int H, const ImageView& img, const uint32_t* levels, const uint32_t* levels_last,
                       const BinningView& b, const AmrBinningView& ab, const GeomView& g, const float* features,
                       const float* bg, float* out_color, int foveaStep, hipStream_t s, bool fused, int P,
                       int* zero_radii) {
    const int tgx = (W + 31) / 32, tgy = (H + 31) / 32;
    if (tgx == 0 || tgy == 0) return;
    if (g_amr_variant == 4) {
        // lists, records and tile order from foveaStep 0 (or this render_once
        // call); colours from the records unless this step brought its own
        const int T = tgx * tgy;
        const float* ov = (foveaStep > 0 && features != g.rgb) ? features : nullptr;
        const int nb = 32 * ((T + 7) / 8);  // b = 8 (4 (p / 8) + q) + p % 8
#define GS_AMR_REGION(R, PER, FOLD, ...)                                                                          \
        hipLaunchKernelGGL((amr_region_render_kernel<R, PER, FOLD, ##__VA_ARGS__>), dim3(nb), dim3(64), 0, s, W, H, tgx, T,            \
                           img.tile_order,                                                                          \
                           img.ranges, ab.region_lists, img.region_count, levels, levels_last, ab.rec_a, ab.rec_b, \
                           ab.rec_c, b.point_list, ov, img.accum_alpha, img.n_contrib, bg, out_color, foveaStep,   \
                           g_amr_scramble, fused ? img.levels_current : nullptr, img.levels_last, img.tile_done, P,   \
                           fused ? zero_radii : nullptr)
        if (foveaStep > 0) {
            const bool fold = (g_amr_fold >> foveaStep) & 1;
            if (fold && g_amr_sel == 2 && g_amr_fold_n == 8 && !((g_amr_deep >> foveaStep) & 1)) GS_AMR_REGION(1, 1, 8, 2);
            else if (fold && g_amr_sel && ((g_amr_deep >> foveaStep) & 1)) GS_AMR_REGION(1, 2, 8, true);
            else if (fold && g_amr_sel && g_amr_fold_n == 16) GS_AMR_REGION(1, 1, 16, true);
            else if (fold && g_amr_sel) GS_AMR_REGION(1, 1, 8, true);
            else if (fold && ((g_amr_deep >> foveaStep) & 1)) GS_AMR_REGION(1, 2, 8);
            else if (fold && g_amr_fold_n == 16) GS_AMR_REGION(1, 1, 16);
            else if (fold) GS_AMR_REGION(1, 1, 8);
            else if (g_amr_batch == 2) GS_AMR_REGION(1, 2, 0);
            else GS_AMR_REGION(1, 1, 0);
        } else {
            if ((g_amr_fold & 1) && g_amr_sel == 2) GS_AMR_REGION(4, 1, 4, 2);
            else if ((g_amr_fold & 1) && g_amr_sel) GS_AMR_REGION(4, 1, 4, true);
            else if (g_amr_fold & 1) GS_AMR_REGION(4, 1, 4);
            else if (g_amr_batch == 2) GS_AMR_REGION(4, 2, 0);
            else GS_AMR_REGION(4, 1, 0);
        }
#undef GS_AMR_REGION
        return;
    }
    if (g_amr_variant == 3) {
        // the tile order and quadrant lists were built by foveaStep 0 (or this
        // render_once call) right after the binning (gs_api.cpp)
        const int T = tgx * tgy;
        if (foveaStep > 0)
            hipLaunchKernelGGL(amr_quad_render_kernel<1>, dim3(4 * T), dim3(64), 0, s, W, H, tgx, img.tile_order,
                               img.ranges, quad_lists(b), img.quad_count, levels, levels_last, b.point_list,
                               reinterpret_cast<const float2*>(g.means2D), features,
                               reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib, bg,
                               out_color, foveaStep);
        else
            hipLaunchKernelGGL(amr_quad_render_kernel<4>, dim3(4 * T), dim3(64), 0, s, W, H, tgx, img.tile_order,
                               img.ranges, quad_lists(b), img.quad_count, levels, levels_last, b.point_list,
                               reinterpret_cast<const float2*>(g.means2D), features,
                               reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib, bg,
                               out_color, foveaStep);
        return;
    }
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
