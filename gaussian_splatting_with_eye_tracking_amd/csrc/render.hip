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
#include <hip/hip_ext.h>

#include "gs_blend.cuh"
#include "gs_device.cuh"
#include "gs_kernels.h"
#include "gs_tilesort.cuh"

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
// (A form that sorted its own tile of <= 1024 instances before blending it,
// in LDS the batches reuse, measured 0.9978 -> 0.9948 ms per config-2 step
// and 2.4819 -> 2.4954 at config 4 -- the sort's latency hides behind the
// other workgroups' blending, but its LDS and registers cost the blend
// occupancy; profiles/r05g_ab_fuse*.log.  The AMR region-list pass keeps it,
// amr_region_lists_kernel.)
template <int kPPL, int kWaves, int kMinWaves = 1, bool kSel = false>
__global__ void __launch_bounds__(64 * kWaves, kMinWaves) render_fwd_kernel(int W, int H, const uint32_t* __restrict__ ranges,
                                                                 const uint32_t* __restrict__ point_list,
                                                                 const float2* __restrict__ means2D,
                                                                 const float* __restrict__ features,
                                                                 const float4* __restrict__ conic_opacity,
                                                                 float* __restrict__ final_T,
                                                                 uint32_t* __restrict__ n_contrib,
                                                                 uint32_t* __restrict__ max_contrib,
                                                                 const float* __restrict__ bg,
                                                                 float* __restrict__ out_color, int cull, int gx,
                                                                 float4* __restrict__ zero4, int zero_n4,
                                                                 uint32_t* __restrict__ bucket_count,
                                                                 uint32_t* __restrict__ bucket_list,
                                                                 uint8_t* __restrict__ hit_codes,
                                                                 uint32_t* __restrict__ hdr, uint32_t hit_word) {
    // The backward's per-Gaussian accumulator rows (grad_accum, idle in the
    // base forward) are zeroed here, behind the blend, instead of by a memset
    // on the backward's critical path: fire-and-forget stores in a kernel
    // bound by VALU / LDS, not HBM (gs_api.cpp: accum_clean), with the
    // non-temporal hint (the rows are next touched by the backward; step
    // 2.552 -> 2.540 ms at config 4, profiles/r04z5_ab_znt*.log).
    typedef float f4v __attribute__((ext_vector_type(4)));
    for (int i = (int)(blockIdx.x * blockDim.x + threadIdx.x); i < zero_n4; i += (int)(gridDim.x * blockDim.x))
        __builtin_nontemporal_store(f4v{0.f, 0.f, 0.f, 0.f}, reinterpret_cast<f4v*>(zero4 + i));
    __shared__ float4 s_a[64 * kWaves];
    __shared__ float4 s_co[64 * kWaves];
    __shared__ __attribute__((aligned(16))) float s_b[64 * kWaves * (kSel ? 4 : 1)];  // (kSel: 16-B stride)
    __shared__ uint64_t s_bal[(kSel ? 5 : 4) * kWaves];  // (kSel: + the safe-form masks)
    __shared__ uint64_t s_hit[kWaves * kWaves];
    __shared__ uint32_t s_max;
    if (kWaves > 1 && threadIdx.x == 0) s_max = 0;
    // whether this forward leaves exact row-group hit codes for the backward
    // (the select form records them; the fallback leaves 0)
    if (hdr && blockIdx.x == 0 && threadIdx.x == 0) hdr[kHdrHitCodes] = (kSel && hit_codes) ? hit_word : 0u;
    const int tile = xcd_block_tile((int)blockIdx.x, gx, (int)(gridDim.x / gx));
    const uint32_t ox = (uint32_t)(tile % gx) * 16, oy = (uint32_t)(tile / gx) * 16;
    const PixelSetT<kPPL> px = make_pixels_t<kPPL, kWaves>(W, H, ox, oy, 1);
    const uint2 range = reinterpret_cast<const uint2*>(ranges)[tile];
    const BlendStateT<kPPL> st =
        blend_tile_t<kPPL, kWaves, kSel>(range, px, (float)ox, (float)oy, 1.0f, point_list,
                                         means2D, features, conic_opacity, s_a, s_co, s_b, s_bal, cull != 0,
                                         kSel ? hit_codes : nullptr, s_hit);
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
void set_cull(int v) { g_cull = v; }

// Forward variants (set_tuning("fwd_variant")).  Default: 4 waves x 1 pixel
// per lane at <= 64 VGPRs (8 waves per SIMD) with the select-form blend
// (gs_blend.cuh blend_tile_t kSel), the power test dropped in provably safe
// chunks and the per-pair wave exit -- round 4's variant 9.  Fallback (0):
// one wave x 4 pixels per lane, the predicate form, no hit codes (the
// backward then culls by geometry).  Measured and removed (the A/B logs stay
// in profiles/): 2 waves x 2 px, 4 x 1 at the default occupancy or capped at
// 6 waves, the select form without safe chunks (r03d_ab_fwd_select*:
// 0.305 -> 0.277 ms at config 2 for the select form), with SGPR-mask selects
// (7 % slower, r04b_ab_*), with a per-chunk exit only (config 4 0.1819 ->
// 0.1755 ms for the per-pair exit, r04z3_ab_fwd*), quadrant waves (r04r).
// XCD-aware placement (gs_blend.cuh xcd_block_tile) in both: half the fetches
// at the same time (profiles/r01g_xcd_ab.log).
constexpr int kDefaultFwdVariant = 1;
int g_fwd_variant = kDefaultFwdVariant;

void set_forward_variant(int v) { g_fwd_variant = (v == 0) ? 0 : kDefaultFwdVariant; }

bool launch_render_forward(int W, int H, const ImageView& img, const BinningView& b, const GeomView& g,
                           const float* features, const float* bg, float* out_color, hipStream_t s,
                           float* zero_rows, size_t zero_floats, uint8_t* hit_codes) {
    const int gx = (W + 15) / 16, gy = (H + 15) / 16;
    if (gx == 0 || gy == 0) return false;
    float4* const zero4 = reinterpret_cast<float4*>(zero_rows);
    const int zero_n4 = (zero_rows && zero_floats / 4 <= (size_t)INT32_MAX) ? (int)(zero_floats / 4) : 0;
    // (Heaviest-first by range length measured slower here -- early
    // termination makes the range a poor work estimate; the backward orders
    // by max_contrib instead, backward.hip.)
    // (the profiler's stage events, if any, ride on the dispatch itself)
    const DispatchEvents ev = take_dispatch_events();
#define GS_FWD_LAUNCH(PPL, WAVES, ...)                                                                           \
    hipExtLaunchKernelGGL((render_fwd_kernel<PPL, WAVES, ##__VA_ARGS__>), dim3(gx * gy), dim3(64 * WAVES), 0, s,  \
                       ev.start, ev.stop, 0, W, H, img.ranges,                                                   \
                       b.point_list, reinterpret_cast<const float2*>(g.means2D), features,                       \
                       reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib,         \
                       img.max_contrib, bg, out_color, g_cull, gx, zero4, zero_n4,                               \
                       img.bucket_count, img.bucket_list, hit_codes, g.hdr, hit_codes_word(b.point_list, hit_codes))
    if (g_fwd_variant == 0) GS_FWD_LAUNCH(4, 1);
    else GS_FWD_LAUNCH(1, 4, 8, true);  // <= 64 VGPRs: 8 waves per SIMD
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
// 4 -> 0.083, 8 -> 0.083: occupancy beats per-thread memory parallelism).
// Tiles in XCD-compact strips (gs_blend.cuh xcd_block_tile: neighbouring
// tiles, which gather the same Gaussians' rows, share an XCD's L2): 0.0789
// (heaviest-first tile order) -> 0.0765 ms, row-major 0.0818
// (profiles/r04z2_ab_lorder.log).
constexpr int kRlPer = 2;
// Region mask of one entry: the exact ellipse test (splat_rect_hit) on the
// four 16x16 quadrants, refined to the 8x8 regions by the alpha >= 1/255
// ellipse's bounding box (both conservative).  Bit g = 4 row + col.
// (The per-Gaussian part -- splat_box's log, square roots and divisions --
// precomputed by the preprocess into the row's free words measured no
// faster, 0.0888 vs 0.0886 ms, with the preprocess 6 us slower,
// profiles/r05j_bench_cfg3.log; not kept.)
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

// rows: the per-Gaussian 64-B blend rows the AMR preprocess wrote
// (GeomView::amr_rows): (x, y, r, g), splat_coef, (b, raw conic), pad.
// kFuse (the default): a tile of 2..kAmrFusedSortMax instances arrives
// unsorted in pair_keys; the workgroup sorts it first (gs_tilesort.cuh bucket
// sort, 8 keys per thread), writes point_list and walks the sorted ids from
// LDS (no separate sort launches below 2048 instances, no point_list re-read).
template <bool kFuse>
__global__ void __launch_bounds__(kRlThreads) amr_region_lists_kernel(int tgx, const uint32_t* __restrict__ ranges,
                                                                      uint32_t* __restrict__ point_list,
                                                                      const float4* __restrict__ rows,
                                                                      float4* __restrict__ rec_a,
                                                                      float4* __restrict__ rec_b,
                                                                      float* __restrict__ rec_c,
                                                                      uint32_t* __restrict__ lists,
                                                                      uint32_t* __restrict__ region_count,
                                                                      uint32_t* __restrict__ tile_done, int tgy,
                                                                      const uint64_t* __restrict__ pair_keys) {
    constexpr int kW = kRlThreads / 64;
    static_assert(kRlThreads == 256, "the fused sort's workgroup");
    using SortL = TileSortLds<256, kAmrFusedSortMax / 256, 1>;
    __shared__ SortL s_sort[1];
    __shared__ uint32_t s_ids[kFuse ? kAmrFusedSortMax : 1];
    // per pass: hits of (slot e, region g, wave w), then their exclusive
    // offsets in the pass's (e, w) order, per region
    __shared__ uint32_t s_cnt[16][kRlPer * kW];
    __shared__ uint32_t s_base[16];  // entries written per region by earlier passes
    const int tile = xcd_block_tile((int)blockIdx.x, tgx, tgy);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t beg = ranges[2 * tile];
    const int n = (int)(ranges[2 * tile + 1] - beg);
    const float ox = (float)((tile % tgx) * 32), oy = (float)((tile / tgx) * 32);
    uint32_t* out = lists + 16 * (size_t)beg;
    const uint32_t* ids = point_list + beg;  // (kFuse and n <= kAmrFusedSortMax: the LDS copy below)
    if constexpr (kFuse) {
        if (n >= 2 && n <= kAmrFusedSortMax) {  // block-uniform
            tile_bucket_sort<256, kAmrFusedSortMax / 256, 1>(pair_keys + beg, n, point_list + beg, s_sort[0], s_ids);
            ids = s_ids;
        } else if (n == 1) {
            if (tid == 0) {
                const uint32_t v = (uint32_t)pair_keys[beg];
                point_list[beg] = v;
                s_ids[0] = v;
            }
            ids = s_ids;
        }
        __syncthreads();  // the LDS ids
    }
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
                const uint32_t id = ids[i];
                const float4* rr = rows + (size_t)4 * id;
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
                             const GeomView& g, const float* features, int K, hipStream_t s, bool fused_sort) {
    const int tgx = (W + 31) / 32, tgy = (H + 31) / 32;
    if (tgx == 0 || tgy == 0) return;
    if (K == 0) {  // no lists to build; the counts must still read 0
        // (checked by the caller's stage_check)
        (void)hipMemsetAsync(img.region_count, 0, sizeof(uint32_t) * 16 * (size_t)tgx * tgy, s);
        (void)hipMemsetAsync(img.tile_done, 0, sizeof(uint32_t) * (size_t)tgx * tgy, s);
        return;
    }
    (void)features;  // in the rows (the preprocess saw colors_precomp / the SH colours)
#define GS_RL_LAUNCH(F)                                                                                           \
    hipLaunchKernelGGL(amr_region_lists_kernel<F>, dim3(tgx * tgy), dim3(kRlThreads), 0, s, tgx, img.ranges,      \
                       b.point_list, reinterpret_cast<const float4*>(g.amr_rows), ab.rec_a, ab.rec_b, ab.rec_c,   \
                       ab.region_lists, img.region_count, img.tile_done, tgy, b.pair_keys)
    if (fused_sort) GS_RL_LAUNCH(true);
    else GS_RL_LAUNCH(false);
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
// kRounds 1 (the progressive steps): the select-form fold over 8-entry
// sub-batches (kFold, kSelF); 4 (render_once): the predicate loop over the
// four rounds.  One entry per lane per batch (a group stages 16).
template <int kRounds>
__global__ void __launch_bounds__(64) amr_region_render_kernel(
    int W, int H, int tgx, int T, const uint32_t* __restrict__ order, const uint32_t* __restrict__ ranges,
    const uint32_t* __restrict__ lists, const uint32_t* __restrict__ region_count,
    const uint32_t* __restrict__ levels, const uint32_t* __restrict__ levels_last, const float4* __restrict__ rec_a,
    const float4* __restrict__ rec_b, const float* __restrict__ rec_c, const uint32_t* __restrict__ point_list,
    const float* __restrict__ feats_override, float* __restrict__ final_T, uint32_t* __restrict__ n_contrib,
    const float* __restrict__ bg, float* __restrict__ out_color, int foveaStep,
    uint32_t* __restrict__ lv_current, uint32_t* __restrict__ lv_last, uint32_t* __restrict__ tile_done, int P,
    int* __restrict__ zero_radii, int accumulate) {
#pragma clang fp contract(fast)
    constexpr int kPer = 1;
    constexpr int kFold = kRounds == 1 ? 8 : 0;
    constexpr int kSelF = kRounds == 1 ? 1 : 0;
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
    const int tile = (int)order[p];
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
    // accumulate (the 5-step driver's fused image sum, gs_amr_accumulate_step):
    // out_color holds the frame's running sum; the unit adds its quadrant
    // (zeros where it renders nothing) to it -- the caller's
    // `out_color_precomp + rendered_image_k` (gaussian_renderer_amr/__init__.py:341)
    // on the same fp32 operands -- and a unit that renders nothing leaves it.
    __shared__ float s_out[3][16][16];
    const uint32_t qx0 = (uint32_t)(tile % tgx) * 32 + 16 * (q & 1), qy0 = (uint32_t)(tile / tgx) * 32 + 16 * (q >> 1);
    const uint32_t orow = lane >> 2, ocol = 4 * (lane & 3);
    // accumulate 2 (GSPLAT_AMD_AMR_STEPS_1_TO_4_SPLIT, the speculative step
    // images): out_color is four [3, H, W] images, image k - 1 the one
    // foveaStep k returns; each pixel's value goes to the image of its round
    // (amr/cr/forward.cu:313-339: (0,0) 1, (1,1) 2, (1,0) 3, (0,1) 4) and the
    // other three get its zeros -- every image fully written, as four calls
    // of one round each would write them.
    auto store_quadrant = [&](bool zero) {
        const uint32_t y = qy0 + orow, x = qx0 + ocol;
        if (y >= (uint32_t)H) return;
        const size_t pp = (size_t)W * y + x;
        if (accumulate == 2) {
            // the lane's 4 pixels start at an even x: rounds (re, ro, re, ro)
            const uint32_t re = (y & 1u) ? 4u : 1u, ro = (y & 1u) ? 2u : 3u;
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                const float4 v = zero ? make_float4(0.f, 0.f, 0.f, 0.f)
                                      : *reinterpret_cast<const float4*>(&s_out[ch][orow][ocol]);
#pragma unroll
                for (uint32_t r = 1; r <= 4; r++) {
                    const bool ke = r == re, ko = r == ro;
                    const float4 w = make_float4(ke ? v.x : 0.f, ko ? v.y : 0.f, ke ? v.z : 0.f, ko ? v.w : 0.f);
                    float* dst = out_color + (size_t)(r - 1) * 3 * plane + ch * plane + pp;
                    if ((W & 3) == 0 && x + 3 < (uint32_t)W) {
                        *reinterpret_cast<float4*>(dst) = w;
                    } else {
                        const float ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                        for (int j = 0; j < 4; j++)
                            if (x + j < (uint32_t)W) dst[j] = ww[j];
                    }
                }
            }
            return;
        }
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            const float4 v = zero ? make_float4(0.f, 0.f, 0.f, 0.f)
                                  : *reinterpret_cast<const float4*>(&s_out[ch][orow][ocol]);
            float* dst = out_color + ch * plane + pp;
            if ((W & 3) == 0 && x + 3 < (uint32_t)W) {
                if (accumulate) {
                    const float4 o = *reinterpret_cast<const float4*>(dst);
                    *reinterpret_cast<float4*>(dst) = make_float4(__fadd_rn(o.x, v.x), __fadd_rn(o.y, v.y),
                                                                  __fadd_rn(o.z, v.z), __fadd_rn(o.w, v.w));
                } else {
                    *reinterpret_cast<float4*>(dst) = v;
                }
            } else {
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (x + j < (uint32_t)W) dst[j] = accumulate ? __fadd_rn(dst[j], vv[j]) : vv[j];
            }
        }
    };
    // Fused step levels (lv_current given, the progressive steps): the
    // reference's per-step level update (amr.hip fovea_levels_kernel,
    // amr/cr/rasterizer_impl.cu's tile_AMR_levels_last / _current) evaluated
    // by each of the tile's four units from the previous current level; the
    // last unit of the tile to finish stores it (tile_done counts units mod 4),
    // so every unit has read the previous value before it is replaced.
    // (GSPLAT_AMD_AMR_STEPS_1_TO_4: steps 1..4 in one launch -- the unit
    // renders rounds 1..min(level, 4), the rounds steps 1..4 give it one by
    // one, and stores the level state step 4 leaves: current min(level, 4),
    // last min(level, 3))
    uint32_t L_last, L, L_last_store;
    if (lv_current) {
        const uint32_t Lp = levels[tile], prev = lv_current[tile];
        if (foveaStep == 1) {
            L_last = 0;
            L = Lp >= 1u ? 1u : 0u;
        } else if (foveaStep <= 4) {
            L_last = prev;
            L = Lp >= (uint32_t)foveaStep ? (uint32_t)foveaStep : prev;
        } else if (foveaStep == kAmrStepsAll) {
            L_last = 0;
            L = min(Lp, 4u);
        } else {
            L_last = 0;
            L = Lp;
        }
        L_last_store = foveaStep == kAmrStepsAll ? min(Lp, 3u) : L_last;
    } else {
        L_last = levels_last[tile];
        L = levels[tile];
        L_last_store = L_last;
    }
    const uint32_t L_store = L;
    auto finish_unit = [&]() {
        if (lv_current && threadIdx.x == 0) {
            if ((atomicAdd(&tile_done[tile], 1u) & 3u) == 3u) {
                lv_last[tile] = L_last_store;
                lv_current[tile] = L_store;
            }
        }
    };
    // Block-uniform early exits (amr/cr/forward.cu:287-367).
    if (L <= L_last) {
        if (accumulate != 1) store_quadrant(true);
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
            if constexpr (kFold > 0 && kSelF) {
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

// set_tuning("amr_variant"): 4 (default) the 8x8 region sub-lists + blend
// records built at foveaStep 0 (amr_region_lists_kernel) and the
// amr_region_render_kernel units; 0 (fallback) full-list blocks of one wave x
// 4 pixels per lane (amr_render_kernel, the gs_blend.cuh predicate form).
// Measured and removed (logs in profiles/): quadrant sub-lists (variant 3,
// r02c / r02g), 2 x 2 / 4 x 1 full-list geometries, scrambled unit order
// (r02f_ab_amr_scramble), two entries staged per lane (r02e_ab_amr_batch),
// 16-entry fold batches, the non-select fold and the SGPR-mask fold (amr_sel
// 2: 0.0582 -> 0.0645 ms, r04b_ab_*), the fold for render_once
// (r02l_ab_amr_fold_once).
int g_amr_variant = 4;
void set_amr_variant(int v) { g_amr_variant = v == 0 ? 0 : 4; }

void launch_amr_render(int W, int H, const ImageView& img, const uint32_t* levels, const uint32_t* levels_last,
                       const BinningView& b, const AmrBinningView& ab, const GeomView& g, const float* features,
                       const float* bg, float* out_color, int foveaStep, hipStream_t s, bool fused, int P,
                       int* zero_radii, int accumulate) {
    const int tgx = (W + 31) / 32, tgy = (H + 31) / 32;
    if (tgx == 0 || tgy == 0) return;
    if (g_amr_variant == 4) {
        // lists, records and tile order from foveaStep 0 (or this render_once
        // call); colours from the records unless this step brought its own
        const int T = tgx * tgy;
        const float* ov = (foveaStep > 0 && features != g.rgb) ? features : nullptr;
        const int nb = 32 * ((T + 7) / 8);  // b = 8 (4 (p / 8) + q) + p % 8
#define GS_AMR_REGION(R)                                                                                          \
        hipLaunchKernelGGL((amr_region_render_kernel<R>), dim3(nb), dim3(64), 0, s, W, H, tgx, T, img.tile_order, \
                           img.ranges, ab.region_lists, img.region_count, levels, levels_last, ab.rec_a, ab.rec_b, \
                           ab.rec_c, b.point_list, ov, img.accum_alpha, img.n_contrib, bg, out_color, foveaStep,   \
                           fused ? img.levels_current : nullptr, img.levels_last, img.tile_done, P,               \
                           fused ? zero_radii : nullptr, accumulate)
        if (foveaStep > 0) GS_AMR_REGION(1);
        else GS_AMR_REGION(4);
#undef GS_AMR_REGION
        return;
    }
    (void)accumulate;  // (variant 4 only: gs_amr_accumulate_step checks)
    hipLaunchKernelGGL((amr_render_kernel<4, 1>), dim3(2 * tgx, 2 * tgy), dim3(64), 0, s, W, H, tgx, img.ranges,
                       levels, levels_last, b.point_list, reinterpret_cast<const float2*>(g.means2D), features,
                       reinterpret_cast<const float4*>(g.conic_opacity), img.accum_alpha, img.n_contrib, bg,
                       out_color, foveaStep, g_cull);
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
