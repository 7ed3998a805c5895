// backward.hip -- gradients on gfx950.
//
// render_bwd_kernel follows base/cr/backward.cu:399-557 (renderCUDA
// backward): per pixel, back-to-front replay from n_contrib with the same
// T/accum_rec recurrences and the same nine per-(pixel, Gaussian) gradient
// terms.  What changes is where the sums go: the reference issues 9 global
// float atomics per contributing (pixel, Gaussian) pair -- on MI355X those
// are memory-side atomics at ~one 64-B request each, and 64 lanes hitting one
// address serialise.  Here one wave64 owns a whole 16x16 tile (4 pixels per
// lane, gs_blend.cuh) and, per Gaussian j of the LDS batch:
//   1. each lane sums its 4 pixels' terms as moments (the lane's pixels share
//      x), then the wave transposes the 64 lanes' values with permlane swaps
//      down to 16 column partials per value, parked in an LDS staging slot;
//   2. every 7 Gaussians, one 63-lane pass sums the staged partials (lane
//      9 s + q = value q of slot s), forms the reference's nine terms and adds
//      them into grad_accum[P][kGradRow] -- one atomic instruction per 7
//      (tile, Gaussian) pairs.
// (The fallback form sums by a full transposition into LDS rows and flushes
// one 64-B atomic row per (tile, Gaussian) at the end of each batch.)
// The backward also starts each tile at max(n_contrib) of its pixels
// (recorded by the forward) instead of the end of the range: entries past it
// are skipped by every pixel in the reference too.
//
// backward_gaussians_kernel fuses computeCov2DCUDA (base/cr/backward.cu:
// 144-274), preprocessCUDA (:346-396), computeColorFromSH (:20-139) and
// computeCov3D (:278-341) into one per-Gaussian pass that also emits the
// reference's dL_dmeans2D / dL_dconic / dL_dopacity / dL_dcolors layout from
// grad_accum, and writes every output element (zeros included).
#include <algorithm>
#include <type_traits>

#include <hip/hip_ext.h>

#include "gs_blend.cuh"
#include "gs_bwd_math.cuh"
#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

constexpr int kNG = 9;      // gradient terms per (pixel, Gaussian)
constexpr int kAccRow = 9;   // LDS accumulator row (floats; odd stride: 9 scalar stores per row)
constexpr int kPPL = 4;      // pixels per lane: one wave64 covers the 16x16 tile (gs_blend.cuh mapping)

// One 16x16 tile per single-wave workgroup, 4 pixels per lane (lane l: column
// l % 16 of the 4 row groups).  kSel (the default): the select-form visit
// with SGPR-mask selects and per-batch compare sets, staged transposed sums
// and the flush fused into the staging reduce (below).  !kSel (the fallback,
// and the AMR backward): the predicate form, full sums by transposition into
// LDS rows, one 64-B atomic row per (tile, Gaussian) at the end of each batch.
template <bool kSel, bool kAMR = false, bool kOpT = false>
__global__ void __launch_bounds__(64, 4) render_bwd_kernel(
    int W, int H, const uint32_t* __restrict__ ranges, const uint32_t* __restrict__ max_contrib,
    const uint32_t* __restrict__ point_list, const float2* __restrict__ means2D,
    const float4* __restrict__ conic_opacity, const float* __restrict__ colors, const float* __restrict__ final_Ts,
    const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpixels, const float* __restrict__ bg,
    float* __restrict__ grad_accum, int cull, int gx, int amr_mode, const uint32_t* __restrict__ levels,
    const uint32_t* __restrict__ bucket_count, const uint32_t* __restrict__ bucket_list,
    const uint32_t* __restrict__ hdr) {
#pragma clang fp contract(fast)
    static_assert(!(kSel && kAMR), "the AMR backward is the fallback form");
    constexpr int kB = 64;  // Gaussians per LDS batch
    __shared__ uint32_t s_id[2][kB];  // double-buffered: the next batch's ids land while this one flushes
    // (x, y, r, g) and the scaled conic / opacity as two b128 reads, b as one
    // b32 (LDS cycles per wave-read: b128 4, b96 8, b64 / b32 2)
    __shared__ float4 s_a[kB];
    __shared__ float4 s_co[kB];
    // (b at a 16-B stride: one LDS address serves all three record reads)
    __shared__ float4 s_b[kB];
    // !kSel: per-Gaussian sums, one row per batch slot, flushed per batch
    __shared__ float s_acc[kSel ? 1 : kB * kAccRow];
    __shared__ uint64_t s_bal[4];
    // kSel: the per-Gaussian sums are finished in groups of 7 Gaussians --
    // each visit parks its two transposed registers (16 column partials of
    // each of 8 values, swap_rows8_pk_t) in a staging slot, and one pass over
    // 7 slots sums them with 63 lanes at once (lane = 9 * slot + value)
    // instead of 14 DPP adds per Gaussian.  Layout: reduce lane l's 16
    // partials are 4 float4s at l * 4 + i * kStagePitch (i = 0..3), so each
    // b128 read is 64 consecutive dwords per 16 lanes; the pitch's 16-float pad
    // spreads the writers' 4 column groups over all 64 banks.
    constexpr int kStageSlots = 7;
    constexpr int kStagePitch = 272;
    __shared__ __attribute__((aligned(16))) float s_stage[kSel ? 3 * kStagePitch + 256 : 1];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // AMR mode (kAMR, amr_mode != 0; the foveated backward, an extension beyond
    // parity): block b = (32-px tile b / 4, sub-lattice (b & 1, (b >> 1) & 1)),
    // its 16 x 16 pixels at stride 2 -- the pixels amr_render_kernel blended
    // for that AMR round.  amr_mode = k > 0: foveaStep k's image (round k of
    // tiles with level >= k); < 0: render_once (rounds <= level).
    int tile;
    uint32_t ox, oy;
    // (a template parameter: run-time AMR branches cost the base kernel 12 %)
    constexpr uint32_t pstride = kAMR ? 2 : 1;
    if constexpr (kAMR) {
        tile = (int)(blockIdx.x >> 2);
        const uint32_t sx = blockIdx.x & 1u, sy = (blockIdx.x >> 1) & 1u;
        const uint32_t round = sx == 0 ? (sy == 0 ? 1u : 4u) : (sy == 0 ? 3u : 2u);  // amr/cr/forward.cu:313-339
        const uint32_t L = min(levels[tile], 4u);
        if (amr_mode > 0 ? (round != (uint32_t)amr_mode || L < round) : round > L) return;
        ox = (uint32_t)(tile % gx) * 32 + sx;
        oy = (uint32_t)(tile / gx) * 32 + sy;
    } else {
        tile = (int)blockIdx.x;
        if (bucket_count) {
            // rank blockIdx.x of the heaviest-first order: the bucket whose
            // inclusive count first exceeds it (256 buckets: 4 per lane)
            const uint4 c4 = reinterpret_cast<const uint4*>(bucket_count)[lane];
            const uint32_t c = c4.x + c4.y + c4.z + c4.w;
            uint32_t incl = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
                if (lane >= d) incl += y;
            }
            const uint32_t rank = blockIdx.x;
            const uint64_t past = __ballot(incl > rank);
            // counts that do not cover the grid exactly (an image buffer whose
            // base forward render did not fill the buckets, e.g. from another
            // caller or size): every block takes the identity order instead,
            // so each tile is still processed exactly once
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            if (total == gridDim.x && past != 0ull) {
                const int L = __builtin_ctzll(past);
                uint32_t r = rank - (uint32_t)__builtin_amdgcn_readlane((int)(incl - c), L);
                const uint32_t q0 = (uint32_t)__builtin_amdgcn_readlane((int)c4.x, L),
                               q1 = (uint32_t)__builtin_amdgcn_readlane((int)c4.y, L),
                               q2 = (uint32_t)__builtin_amdgcn_readlane((int)c4.z, L);
                int b = 4 * L;
                if (r >= q0) { r -= q0; b++;
                    if (r >= q1) { r -= q1; b++;
                        if (r >= q2) { r -= q2; b++; } } }
                tile = (int)bucket_list[(size_t)b * gridDim.x + r];
            }
        }
        ox = (uint32_t)(tile % gx) * 16;
        oy = (uint32_t)(tile / gx) * 16;
    }
    const uint2 range = reinterpret_cast<const uint2*>(ranges)[tile];
    const int n = (int)(range.y - range.x);
    int m = kAMR ? n : min(n, (int)max_contrib[tile]);
    if (m == 0) return;  // block-uniform

    const PixelSetT<kPPL> px = make_pixels_t<kPPL, 1>(W, H, ox, oy, pstride);
    const size_t plane = (size_t)H * W;
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
    // row group k's pixel y is py0 + 4 k stride: exact small-integer floats, the
    // same operand the forward subtracts (3 fewer live registers than px.y[])
    const float py0 = px.y[0];
    // accum_rec . dL_dpix is all the reference's accum_rec / last_color
    // recurrences (backward.cu:500-507) feed into dL_dalpha, so each pixel
    // carries that one scalar instead of 2 x 3.
    float T[kPPL], nbg[kPPL], dpx[kPPL][3], acc_dot[kPPL];
    uint32_t last[kPPL];
    uint32_t wave_last = 0;
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
        const uint32_t pid = px.pid[k];
        const float Tf = px.inside[k] ? final_Ts[pid] : 0.f;
        T[k] = Tf;
        last[k] = px.inside[k] ? n_contrib[pid] : 0u;
        wave_last = max(wave_last, last[k]);
#pragma unroll
        for (int c = 0; c < 3; c++) dpx[k][c] = px.inside[k] ? dL_dpixels[c * plane + pid] : 0.f;
        // (-T_final / (1 - alpha)) * bg.dL_dpix = nbg * 1/(1 - alpha)
        nbg[k] = -Tf * (bg0 * dpx[k][0] + bg1 * dpx[k][1] + bg2 * dpx[k][2]);
        // kSel: the background term folded into the recurrence -- with
        // B = T_final bg.dL_dpix / T (so the reference's bg term is -T_new B),
        // acc_dot + B obeys the same accum recurrence as acc_dot and starts at
        // bg.dL_dpix: dL_dalpha = T_new (c.dL_dpix - (acc_dot + B)).
        acc_dot[k] = kSel ? bg0 * dpx[k][0] + bg1 * dpx[k][1] + bg2 * dpx[k][2] : 0.f;
    }
    // entries at or past the wave's max n_contrib are skipped by all its pixels
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) wave_last = max(wave_last, (uint32_t)__shfl_xor((int)wave_last, off, 64));
    // per row group (the lane's k-th pixel): max n_contrib of its 64 pixels;
    // entries at or past it are skipped by every pixel of the group
    int group_last[kPPL];
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
        uint32_t g = last[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) g = max(g, (uint32_t)__shfl_xor((int)g, off, 64));
        group_last[k] = __builtin_amdgcn_readfirstlane((int)g);
    }
    // kSel: the smallest n_contrib of each row group's image pixels (pixels
    // outside the image count as started: their T and dL/dpix are 0, so any
    // finite alpha leaves their terms 0).  Entries with contributor below it
    // are taken by every pixel of the group: no per-pixel contributor test.
    uint32_t min_last = 0xffffffffu;
    if constexpr (kSel) {
#pragma unroll
        for (int k = 0; k < kPPL; k++) {
            uint32_t g = px.inside[k] ? last[k] : 0xffffffffu;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) g = min(g, (uint32_t)__shfl_xor((int)g, off, 64));
            min_last = min(min_last, g);
        }
        min_last = (uint32_t)__builtin_amdgcn_readfirstlane((int)min_last);
    }
    // = max_contrib[tile] for a whole base tile; AMR: no per-tile max_contrib
    // was recorded for the sub-lattice, the wave max is the block's
    m = min(kAMR ? n : m, __builtin_amdgcn_readfirstlane((int)wave_last));
    if (m == 0) return;
    // Row masks: the forward's exact hit codes when it left them (gs_blend.cuh
    // blend_tile_t: bit r = row group r has a pixel that blended the entry,
    // i.e. a pixel this backward takes it at), else the geometric cull.
    // (where the forward stored them: the header word, gs_layout.h hit_codes_of)
    const uint8_t* const codes = (!kAMR && hdr != nullptr) ? hit_codes_of(point_list, hdr[kHdrHitCodes]) : nullptr;
    const bool use_codes = codes != nullptr;
    const float ddelx_dx = (float)(0.5 * W);
    const float ddely_dy = (float)(0.5 * H);
    const int comp = lane & 15;
    // !kSel flush: the accumulator-row entry each output component starts from
    const int ia = comp < 3 ? comp : comp == 8 ? 3 : comp < 5 ? 4 : comp + 1;

    // Software pipeline over the batches (vector-memory counters retire in
    // issue order, so issue order decides what each wait covers): the next
    // batch's point_list ids are loaded while this batch is blended, its
    // Gaussian records are gathered before this batch's flush atomics are
    // issued, so neither the id round trip nor the atomics' completion is
    // waited for at the top of the next batch.
    // (the hit codes ride with the records: loaded a batch ahead with them, so
    // the batch's row masks wait for nothing the records did not -- loaded
    // at the top of the batch, they cost one more memory round trip per
    // batch, with the next batch's id load behind them in the same counter)
    uint32_t nid = 0, ncode = 0xfu;
    float2 nxy = make_float2(0.f, 0.f);
    float4 nco = make_float4(0.f, 0.f, 0.f, 0.f);
    float nrgb[3] = {0.f, 0.f, 0.f};
    if (tid < min(kB, m)) {
        nid = point_list[range.x + m - 1 - tid];
        if (use_codes) ncode = codes[range.x + m - 1 - tid];
        nxy = means2D[nid];
        nco = conic_opacity[nid];
        nrgb[0] = colors[3 * nid]; nrgb[1] = colors[3 * nid + 1]; nrgb[2] = colors[3 * nid + 2];
        s_id[0][tid] = nid;
    }
    // kSel staging reduce: lane (slot = lane / 9, value q = lane % 9) sums the
    // 16 column partials of value q parked by slot's Gaussian (za rows hold
    // values swap_sum_slot(r), zb rows 4 + swap_sum_slot(r); swap_sum_slot is
    // its own inverse) and adds the reference's term into grad_accum.
    const int st_slot = lane / 9, st_q = lane - 9 * (lane / 9);
    if constexpr (kSel) {
        for (int i = lane; i < 3 * kStagePitch + 256; i += 64) s_stage[i] = 0.f;
    }
    // writer lane: row r = lane / 16 of za / zb holds values swap_sum_slot(r) /
    // 4 + swap_sum_slot(r), column c = lane % 16 is element c of that sum.
    // zb's value v = 4 + swap_sum_slot(r) of (g4, s1, s2, g7) goes to output
    // q = v except s2 (v = 6) -> q = 8; g6 (q = 6) = dx x (g4's column
    // partial), formed after the transposition by lanes 0-15 (zb row 0 = g4),
    // the other lanes' product into their dummy word: no ninth-value DPP tree.
    const int st_dst = ((lane & 15) >> 2) * kStagePitch + 4 * swap_sum_slot(lane >> 4) + (lane & 3);
    const int st_dst_b = [&] {
        const int v = 4 + swap_sum_slot(lane >> 4);
        return ((lane & 15) >> 2) * kStagePitch + 4 * (v == 6 ? 8 : v) + (lane & 3);
    }();
    // (the idle lanes 16-63 store into the 16-word pads of pitch rows 0-2,
    // which the reduce never reads)
    const int st_g6 = lane < 16 ? ((lane & 15) >> 2) * kStagePitch + 4 * 6 + (lane & 3)
                                : ((lane - 16) >> 4) * kStagePitch + 256 + (lane & 15);
    int par = 0;
    for (int top = m; top > 0; top -= kB, par ^= 1) {  // entries [top-cnt, top), back to front
        const int cnt = min(kB, top);
        __syncthreads();
        uint32_t gm = 0;
        bool fastg = false;  // kSel: p2 <= 0 at every pixel of the tile, provably (below)
        if (tid < cnt) {
            const float2 xy = nxy;
            const float4 co = nco;
            float4 pc = splat_coef(co);
            // (+ 0: an add where the staged record takes the opacity, so the
            // compiler forms the b128 store's register tuple here, after the
            // wait for the gather, instead of with a copy right behind the
            // gather's issue at the end of the previous batch -- which made
            // every batch wait a full memory round trip there)
            pc.w = pc.w + 0.0f;
            s_a[tid] = make_float4(xy.x, xy.y, nrgb[0], nrgb[1]);
            s_co[tid] = pc;
            s_b[tid].x = nrgb[2];
            if constexpr (kSel)  // the reference's `power > 0` skip cannot fire (gs_blend.cuh)
                fastg = splat_form_safe(pc, fabsf(xy.x - (float)ox), fabsf(xy.y - (float)oy)) &&
                        (!kOpT || (pc.w <= 0.99f && pc.w > 0.0f));
            gm = use_codes ? ncode : cull ? splat_group_mask(xy, co, (float)ox, (float)oy, (float)pstride) : 0xfu;
        }
        const int ntop = top - kB;  // the next batch: entries [ntop - ncnt, ntop)
        const bool has_next = ntop > 0 && tid < min(kB, ntop);
        publish_group_masks<1>(gm, s_bal);
        const uint64_t fast_mask = kSel ? uniform_u64(__ballot(fastg)) : 0ull;
        if (has_next) {  // (after the masks: nothing below waits on this load until the batch ends)
            nid = point_list[range.x + ntop - 1 - tid];
            if (use_codes) ncode = codes[range.x + ntop - 1 - tid];
        }
        // every contributor of this batch (<= top - 1) below every row group's
        // smallest n_contrib: all pixels take its entries
        const bool bstarted = kSel && (uint32_t)(top - 1) < min_last;
        uint64_t written = 0;  // !kSel: batch slots whose sum rows were stored
        int nst = 0;           // kSel: staging slots in use (wave-uniform)
        uint64_t js = 0;       // kSel: batch slot j of staging slot s in bits [6 s, 6 s + 6)
        // kSel: the staging reduce finishes the reference's nine terms itself
        // (lane 9 s + q holds accumulator entry q of slot s's Gaussian; entries
        // 4 and 5 -- sum t dx, sum t dy -- fetched by two lane shuffles) and
        // adds them into grad_accum: no accumulator rows in LDS, no per-batch
        // flush pass, one atomic instruction per 7 Gaussians
        // kOpT runs of fast entries sum t' = alpha T dL_dalpha / G = o t (below):
        // the flush takes o out of the mean / conic factors and divides the
        // opacity sum by it
        auto stage_reduce = [&](const int nslot, auto kOT) {
            constexpr bool kOT_ = decltype(kOT)::value;
            if (nslot == kStageSlots || lane < 9 * nslot) {
                const float* src = &s_stage[4 * lane];
                const float4 a = *reinterpret_cast<const float4*>(src);
                const float4 b = *reinterpret_cast<const float4*>(src + kStagePitch);
                const float4 c = *reinterpret_cast<const float4*>(src + 2 * kStagePitch);
                const float4 d = *reinterpret_cast<const float4*>(src + 3 * kStagePitch);
                const gs_f2 x0 = gs_f2{a.x, a.y} + gs_f2{b.x, b.y}, x1 = gs_f2{a.z, a.w} + gs_f2{b.z, b.w};
                const gs_f2 x2 = gs_f2{c.x, c.y} + gs_f2{d.x, d.y}, x3 = gs_f2{c.z, c.w} + gs_f2{d.z, d.w};
                const gs_f2 y = (x0 + x1) + (x2 + x3);
                const uint32_t jj = (uint32_t)(js >> (6 * st_slot)) & 63u;
                // lane 9 s + q: output component fq of q (entries 0..2 colours,
                // 3 = sum t -> opacity (8), 4 = sum t dx -> mean x (3), 5 = sum t
                // dy -> mean y (4), 6..8 -> conic (5..7)); the flush's formula
                const float tot = y.x + y.y;
                const float g4 = __shfl(tot, 9 * st_slot + 4, 64), sy = __shfl(tot, 9 * st_slot + 5, 64);
                if (lane < 63) {
                    const int fq = st_q < 3 ? st_q : st_q == 3 ? 8 : st_q - 1;
                    const float qa = (fq == 3 || fq == 4) ? g4 : tot;
                    const float4 pc = s_co[jj];
                    const float o = kOT_ ? 1.0f : pc.w;
                    const float cx = pc.x * (-1.0f / kHalfLog2e), cy = pc.y * (-1.0f / kLog2e),
                                cz = pc.z * (-1.0f / kHalfLog2e);
                    const float ka = fq == 3 ? -o * cx * ddelx_dx
                                   : fq == 4 ? -o * cy * ddely_dy
                                   : (fq >= 5 && fq <= 7) ? -0.5f * o
                                   : (kOT_ && fq == 8) ? 1.0f / pc.w : 1.0f;
                    const float kb = fq == 3 ? -o * cy * ddelx_dx : fq == 4 ? -o * cz * ddely_dy : 0.0f;
                    const float v = ka * qa + kb * sy;
                    if (v != 0.f) atomicAdd(&grad_accum[(size_t)s_id[par][jj] * kGradRow + fq], v);
                }
            }
        };
        __syncthreads();
        // first batch slot this wave needs: contributor = top-1-j < wave_last
        // (readfirstlane: wave_last is uniform after the xor-shuffle max, but the
        // compiler cannot prove it; without this the bit-scan loop below is
        // compiled as a divergent VALU loop)
        const int j0 = __builtin_amdgcn_readfirstlane(max(0, top - (int)wave_last));
        uint64_t mk[kPPL];
        uint64_t todo = 0;
        const uint64_t lo_cut = j0 >= 64 ? 0ull : j0 > 0 ? ~0ull << j0 : ~0ull;
#pragma unroll
        for (int k = 0; k < kPPL; k++) {
            // slots j with contributor = top-1-j < group_last[k], i.e. j >= top - group_last[k]
            const int jk = top - group_last[k];
            const uint64_t gcut = jk <= 0 ? ~0ull : (jk >= 64 ? 0ull : ~0ull << jk);
            mk[k] = uniform_u64(s_bal[k]) & lo_cut & gcut;
            todo |= mk[k];
        }
        // One Gaussian (batch slot j, record staged in LDS) against the wave's
        // pixels.  (Reading the next set bit's record ahead, in two register
        // sets used in turn, measured no faster: the 4 waves per SIMD already
        // hide the LDS latency.)
        auto visit = [&](const int j, const float2 xy, const float4 pc, const float4 cf, auto kFastT, auto kStartedT,
                         auto kSlotT) {
            constexpr bool kFast = decltype(kFastT)::value, kStarted = decltype(kStartedT)::value;
            constexpr int kSlot = decltype(kSlotT)::value;  // kSel: this entry's staging slot
            const uint32_t contributor = (uint32_t)(top - 1 - j);
            const float dx = xy.x - px.x;
            const float pa = (pc.x * dx) * dx, pb = pc.y * dx;  // the lane's pixels share x
            // Per pixel with t = G dL_dalpha the reference adds (backward.cu:
            // 518-545) dL_dopacity += t; dL_dmean2D += -o t (C d) * (W/2, H/2);
            // dL_dconic += -o/2 t (dx^2, dx dy, dy^2).  A lane's pixels share dx,
            // so it sums s0 = sum t, s1 = sum t dy, s2 = sum t dy^2 and forms
            // the six moments (s0, dx s0, s1, dx^2 s0, dx s1, s2) once; the flush
            // applies o, the conic and the constants.
            // (-0: x + -0 == x for every x, so the first visited row group's
            // fma(a, b, -0) / -0 + t fold to a plain v_mul / move instead of a
            // 3-operand fma with an inline 0)
            float c0 = -0.f, c1 = -0.f, c2 = -0.f, s0 = -0.f, s1 = -0.f, s2 = -0.f;
            bool any = false;
            if constexpr (kSel) {
                // The select form: a rejected pixel takes alpha = G = 0, i.e.
                // rinv = 1 (T unchanged), dchannel = t = 0 and acc_dot += 0 --
                // the same bits as the predicate form for every accepted pixel,
                // no exec-mask bookkeeping: a visited Gaussian is always summed
                // (with the forward's hit codes a visited row group has a pixel
                // that blended; under the geometric cull an all-rejected visit
                // sums zeros, which the flush skips).  The selects take an
                // SGPR-pair mask (gs_sel2_zero_v) and only the compares the
                // entry needs: alpha >= 1/255 always; contributor < n_contrib
                // unless the batch is started for every pixel; power > 0 only
                // for Gaussians not provably negative definite (fast_mask).
#pragma unroll
                for (int k = 0; k < kPPL; k++) {
                    if (!((mk[k] >> j) & 1ull)) continue;  // wave-uniform
                    const float dy = xy.y - (py0 + (float)(4 * k * (int)pstride));
                    const float p2 = splat_p2(pa, pb, dy, pc);
                    const float Gr = splat_exp(p2);
                    const float ar = fminf(0.99f, pc.w * Gr);
                    uint64_t msk = __builtin_amdgcn_fcmpf(ar, 1.0f / 255.0f, kFcmpUGE);
                    if (!kFast || !kStarted) msk &= __builtin_amdgcn_uicmp(contributor, last[k], kIcmpULT);
                    if (!kFast) msk &= __builtin_amdgcn_fcmpf(p2, 0.0f, kFcmpULE);
                    // kOpT and a fast entry (o <= 0.99, p2 <= 0: alpha = o G
                    // unclamped, bit for bit the rounded product): t' = o t =
                    // alpha T (c - acc) = dchannel_dcolor diff -- no G select,
                    // one product fewer; the flush divides o back out
                    constexpr bool kOT = kOpT && kFast;
                    float G, alpha;
                    if constexpr (kOT) alpha = gs_sel_zero_v(msk, ar);
                    else gs_sel2_zero_v(msk, Gr, ar, G, alpha);
                    const float rinv = __builtin_amdgcn_rcpf(1.f - alpha);
                    T[k] = T[k] * rinv;
                    const float dchannel_dcolor = alpha * T[k];
                    // (c - accum_rec - B) . dL_dpix as one fma chain
                    const float diff = __builtin_fmaf(cf.z, dpx[k][2],
                                                      __builtin_fmaf(cf.y, dpx[k][1],
                                                                     __builtin_fmaf(cf.x, dpx[k][0], -acc_dot[k])));
                    acc_dot[k] = __builtin_fmaf(alpha, diff, acc_dot[k]);
                    c0 = __builtin_fmaf(dchannel_dcolor, dpx[k][0], c0);
                    c1 = __builtin_fmaf(dchannel_dcolor, dpx[k][1], c1);
                    c2 = __builtin_fmaf(dchannel_dcolor, dpx[k][2], c2);
                    const float t = kOT ? dchannel_dcolor * diff : G * (diff * T[k]);
                    const float tdy = t * dy;
                    s0 += t;
                    s1 += tdy;
                    s2 = __builtin_fmaf(tdy, dy, s2);
                }
                any = true;
            } else {
#pragma unroll
                for (int k = 0; k < kPPL; k++) {
                    if (!((mk[k] >> j) & 1ull)) continue;  // wave-uniform: culled for this row group
                    const float dy = xy.y - (py0 + (float)(4 * k * (int)pstride));
                    const float p2 = splat_p2(pa, pb, dy, pc);  // the forward's bits
                    const float G = splat_exp(p2);
                    const float alpha = fminf(0.99f, pc.w * G);
                    // The reference's three per-pixel `continue`s (backward.cu:466-482)
                    // as one predicate: only wave-uniform branches save SIMD time, and
                    // nested ones make the compiler re-zero g[] on every skip path.
                    // (contributor >= last also covers pixels outside the image.)
                    const bool ok = contributor < last[k] && !(p2 > 0.0f) && !(alpha < 1.0f / 255.0f);
                    if (!ok) continue;
                    any = true;
                    const float rinv = __builtin_amdgcn_rcpf(1.f - alpha);
                    T[k] = T[k] * rinv;
                    const float dchannel_dcolor = alpha * T[k];
                    // sum_ch (c - accum_rec) dL_dpix, with accum_rec . dL_dpix
                    // advanced by the reference's recurrence (backward.cu:500-507)
                    const float c_dot = cf.x * dpx[k][0] + cf.y * dpx[k][1] + cf.z * dpx[k][2];
                    // The reference advances accum_rec at the NEXT contributor from the
                    // stored (last_alpha, last_color); advancing it here with the same
                    // operands gives the same bits and needs no per-pixel "last" state.
                    const float diff = c_dot - acc_dot[k];
                    const float dL_dalpha = diff * T[k] + nbg[k] * rinv;
                    acc_dot[k] = __builtin_fmaf(alpha, diff, acc_dot[k]);
                    c0 = __builtin_fmaf(dchannel_dcolor, dpx[k][0], c0);
                    c1 = __builtin_fmaf(dchannel_dcolor, dpx[k][1], c1);
                    c2 = __builtin_fmaf(dchannel_dcolor, dpx[k][2], c2);
                    const float t = G * dL_dalpha;
                    const float tdy = t * dy;
                    s0 += t;
                    s1 += tdy;
                    s2 = __builtin_fmaf(tdy, dy, s2);
                }
            }
            float g[kNG];
            g[0] = c0;
            g[1] = c1;
            g[2] = c2;
            g[3] = s0;
            g[4] = dx * s0;
            g[5] = s1;
            g[6] = kSel ? s2 : dx * g[4];
            g[7] = dx * s1;
            g[8] = s2;
            if constexpr (kSel) {
                // s2 rides in the 8-value transposition (g6 = dx^2 s0 leaves it;
                // g6's column partials are dx x g4's, formed after it)
                float za, zb;
                swap_rows8_pk_t<false>(g, za, zb);
                const float w6 = dx * zb;
                s_stage[st_dst + 36 * kSlot] = za;
                s_stage[st_dst_b + 36 * kSlot] = zb;
                s_stage[st_g6 + (lane < 16 ? 36 * kSlot : 0)] = w6;
                js |= (uint64_t)j << (6 * kSlot);
            } else if (__ballot(any) != 0ull) {  // wave-uniform
                // full sums by transposition: 2 values per row leader + g8 in lane 63
                float za, zb;
                swap_sum9(g, za, zb);
                if ((lane & 15) == 15) {
                    float* row = &s_acc[j * kAccRow];
                    const int q = swap_sum_slot(lane >> 4);
                    row[q] = za;
                    row[4 + q] = zb;
                    if (lane == 63) row[8] = g[8];
                }
                written |= 1ull << j;
            }
        };
        using T1 = std::integral_constant<bool, true>;
        using T0 = std::integral_constant<bool, false>;
        using S0 = std::integral_constant<int, 0>;
        if constexpr (kSel) {
            // one copy of the loop per (all-safe, started) batch case, chosen
            // once per batch -- per-entry branches between the visit variants
            // made the register allocator shuffle the loop-carried pixel state
            // (8 v_mov per entry) at every join.  Rounds of 7 entries, one
            // unrolled copy of the visit per staging slot (slot offsets as
            // immediates, no per-entry slot counter or address VALU, the
            // visited bit cleared by one s_andn2)
            auto run = [&](auto kFastT, auto kStartedT) {
                auto one = [&](auto kSlotT) {
                    if (!todo) return;  // wave-uniform
                    const int j = __builtin_ctzll(todo);
                    todo &= ~(1ull << j);
                    const float4 a4 = s_a[j];
                    const float2 xy = make_float2(a4.x, a4.y);
                    const float4 pc = s_co[j], cf = make_float4(a4.z, a4.w, s_b[j].x, 0.f);
                    visit(j, xy, pc, cf, kFastT, kStartedT, kSlotT);
                    nst = decltype(kSlotT)::value + 1;
                };
                while (todo) {
                    one(S0{});
                    one(std::integral_constant<int, 1>{});
                    one(std::integral_constant<int, 2>{});
                    one(std::integral_constant<int, 3>{});
                    one(std::integral_constant<int, 4>{});
                    one(std::integral_constant<int, 5>{});
                    one(std::integral_constant<int, 6>{});
                    if (nst == kStageSlots) {
                        stage_reduce(kStageSlots, std::integral_constant<bool, kOpT && decltype(kFastT)::value>{});
                        nst = 0;
                        js = 0ull;
                    }
                }
                if (nst) stage_reduce(nst, std::integral_constant<bool, kOpT && decltype(kFastT)::value>{});
                nst = 0;
            };
            // every entry this wave visits has a provably negative-definite form
            const bool bsafe = (todo & ~fast_mask) == 0ull;
            if (bsafe && bstarted) run(T1{}, T1{});
            else if (bsafe) run(T1{}, T0{});
            else run(T0{}, T0{});
        } else {
            while (todo) {
                const int j = __builtin_ctzll(todo);
                todo &= todo - 1;
                const float4 a4 = s_a[j];
                const float2 xy = make_float2(a4.x, a4.y);
                const float4 pc = s_co[j], cf = make_float4(a4.z, a4.w, s_b[j].x, 0.f);
                visit(j, xy, pc, cf, T0{}, T0{}, S0{});
            }
        }
        __syncthreads();
        if (has_next) {  // gathers for the next batch, ahead of the flush atomics
            s_id[par ^ 1][tid] = nid;
            nxy = means2D[nid];
            nco = conic_opacity[nid];
            nrgb[0] = colors[3 * nid]; nrgb[1] = colors[3 * nid + 1]; nrgb[2] = colors[3 * nid + 2];
        }
        if constexpr (!kSel) {
            // Flush: 16 lanes per Gaussian row, 4 rows per wave instruction
            // (one 64-B memory-side atomic request per (tile, Gaussian)).  (A full
            // unroll lets the scheduler hoist all 64 LDS reads: 163 VGPRs.)
#pragma unroll 4
            for (int i = 0; i < kB / 4; i++) {
                const int r = (tid >> 4) + 4 * i;
                const bool live = r < cnt && comp < kNG && ((written >> (r & 63)) & 1ull);
                if (live) {
                    // row sums (c0, c1, c2, s0, sx, sy, sxx, sxy, syy) -> the
                    // reference's nine terms: v = ka * row[ia] + kb * sy, with o and
                    // the conic from the staged log2(e)-scaled record
                    const float* row0 = &s_acc[r * kAccRow];
                    const float qa = row0[ia], qb = row0[5];
                    const float4 pc = s_co[r];
                    const float o = pc.w;
                    const float cx = pc.x * (-1.0f / kHalfLog2e), cy = pc.y * (-1.0f / kLog2e),
                                cz = pc.z * (-1.0f / kHalfLog2e);
                    const float ka = comp == 3 ? -o * cx * ddelx_dx
                                   : comp == 4 ? -o * cy * ddely_dy
                                   : (comp >= 5 && comp <= 7) ? -0.5f * o : 1.0f;
                    const float kb = comp == 3 ? -o * cy * ddelx_dx : comp == 4 ? -o * cz * ddely_dy : 0.0f;
                    const float v = ka * qa + kb * qb;
                    if (v != 0.f) atomicAdd(&grad_accum[(size_t)s_id[par][r] * kGradRow + comp], v);
                }
            }
        }
    }
}

extern int g_cull;  // render.hip
// Backward variants (set_tuning("bwd_variant")).  Default: round 4's variant
// 11 -- the select form with SGPR-pair masks, per-batch compare sets, staged
// sums and the flush fused into the staging reduce: render_bwd 0.3707
// (variant 7) -> 0.3634 (masks) -> 0.3512 (s2 in the transposition) ->
// 0.3403 (unrolled slots) -> 0.3139 ms (fused flush) at config 2, 0.2887 ->
// 0.2433 at config 4 (profiles/r04b_ab_bwd*.log, r04e_ab_bwd*.log,
// r04l_ab_bwd*_m.log) -- plus, since round 5, the opacity-scaled sums
// (kOpT): in batches of provably negative-definite entries with o <= 0.99
// (alpha = o G unclamped, bit for bit the rounded product) the visit sums t'
// = alpha T (c - acc) . dL_dpix = o t, which needs no G select and one
// product less, and the flush takes o out of the mean / conic factors and
// divides the opacity sum by it (0.3116 -> 0.3063 ms at config 2, 0.2385 ->
// 0.2348 at config 4, profiles/r05d_ab_bwd_opt*.log).  Fallback (0): the
// predicate form with full sums in LDS rows (also the AMR backward's form).
// Measured and removed (logs in profiles/): 2 waves x 2 px and 4 x 1
// geometries, half-wave DPP-tree sums, a 5-wave occupancy cap (spills), the
// un-fused staged forms, the heavy-tile split (r01h / DESIGN.md §8e), an
// XCD-compact tile order (r04u_ab_xcd*), plain-store / no-flush timing
// diagnostics.
constexpr int kDefaultBwdVariant = 2;
int g_bwd_variant = kDefaultBwdVariant;
void set_backward_variant(int v) { g_bwd_variant = v == 0 ? 0 : kDefaultBwdVariant; }

void launch_render_backward(int W, int H, const ImageView& img, const BinningView& b, const GeomView& g,
                            const float* colors, const float* bg, const float* dL_dpix, hipStream_t s, int K) {
    (void)K;  // (the forward's hit codes are found through the header, gs_layout.h hit_codes_of)
    const int gx = (W + 15) / 16, gy = (H + 15) / 16;
    if (gx == 0 || gy == 0) return;
    // tiles heaviest first: the forward render filled this image buffer's 256
    // work buckets (the kernel falls back to the identity order otherwise)
    // (the profiler's stage events, if any, ride on the dispatch itself)
    const DispatchEvents ev = take_dispatch_events();
#define GS_BWD_LAUNCH(...)                                                                                         \
    hipExtLaunchKernelGGL((render_bwd_kernel<__VA_ARGS__>), dim3(gx * gy), dim3(64), 0, s, ev.start, ev.stop, 0, W, H,     \
                       img.ranges, img.max_contrib,                                                                \
                       b.point_list, reinterpret_cast<const float2*>(g.means2D),                                   \
                       reinterpret_cast<const float4*>(g.conic_opacity), colors, img.accum_alpha, img.n_contrib,    \
                       dL_dpix, bg, g.grad_accum, g_cull, gx, 0, nullptr, img.bucket_count, img.bucket_list,       \
                       g.hdr)
    if (g_bwd_variant == 0) GS_BWD_LAUNCH(false);
    else GS_BWD_LAUNCH(true, false, true);
#undef GS_BWD_LAUNCH
}

// The foveated (AMR) blend backward: 32-px tile ranges, one wave per
// (tile, sub-lattice) block of 16 x 16 pixels at stride 2, only the blocks
// whose round the forward rendered (mode: foveaStep k > 0, or < 0 for
// render_once).  The 1 wave x 4 px geometry (gs_blend.cuh) only.
void launch_amr_render_backward(int W, int H, int mode, const ImageView& img, const BinningView& b,
                                const GeomView& g, const float* colors, const float* bg, const float* dL_dpix,
                                hipStream_t s) {
    const int tgx = (W + 31) / 32, tgy = (H + 31) / 32;
    if (tgx == 0 || tgy == 0 || mode == 0) return;
    hipLaunchKernelGGL((render_bwd_kernel<false, true>), dim3(4 * tgx * tgy), dim3(64), 0, s, W, H, img.ranges,
                       img.max_contrib, b.point_list, reinterpret_cast<const float2*>(g.means2D),
                       reinterpret_cast<const float4*>(g.conic_opacity), colors, img.accum_alpha, img.n_contrib,
                       dL_dpix, bg, g.grad_accum, g_cull, tgx, mode, img.levels, nullptr, nullptr, nullptr);
}

// (the per-Gaussian backward math: gs_bwd_math.cuh)

// kSH16: SH with M = 16 coefficients (degree-3 models): compile-time loops,
// 16-B loads and stores of the 192-B SH rows.
// small: when given, the 3-float outputs (dL_dmeans2D, dL_dmeans3D,
// dL_dscales, dL_dcolors at 0, 3, 6, 9) are returned there for the caller's
// coalesced stores instead of stored per thread at a 12-B stride.
// kDrgb: the host knows the forward stored d(rgb)/d(dir) (no SH coefficient
// path compiled: 114 instead of 164 VGPRs); the SH basis and dL/drgb are
// returned in sh19 (16 + 3) for the caller's staged dL_dsh stores.
template <bool kHasSH, bool kHasScales, bool kSH16, bool kDrgb = false>
__device__ __forceinline__ void backward_gaussian_body(const BackwardGaussArgs& a,
                                                       const float* __restrict__ grad_accum,
                                                       const uint8_t* __restrict__ clamped_bits, int idx,
                                                       float* lrow, float (*small)[12] = nullptr,
                                                       float (*sh19)[19] = nullptr) {
    if (idx >= a.P) return;
    const bool vis = a.radii[idx] > 0;
    // Blend-stage gradients in the reference layout.
    float acc[kNG];
    if (vis) {
        const float4* row = reinterpret_cast<const float4*>(grad_accum + (size_t)idx * kGradRow);
        const float4 r0 = row[0], r1 = row[1];
        const float r2 = grad_accum[(size_t)idx * kGradRow + 8];
        acc[0] = r0.x; acc[1] = r0.y; acc[2] = r0.z; acc[3] = r0.w;
        acc[4] = r1.x; acc[5] = r1.y; acc[6] = r1.z; acc[7] = r1.w; acc[8] = r2;
    } else {
#pragma unroll
        for (int q = 0; q < kNG; q++) acc[q] = 0.f;
    }
    // (dL_dcolor, dL_dconic, dL_dcov3D: NULL = not wanted -- the autograd
    // wrapper discards them unless the matching precomputed input was given;
    // the uniform tests cost nothing, the skipped stores 52 B per Gaussian)
    if (small) {
        (*small)[9] = acc[0];
        (*small)[10] = acc[1];
        (*small)[11] = acc[2];
        (*small)[0] = acc[3];
        (*small)[1] = acc[4];
        (*small)[2] = 0.f;
    } else {
        if (a.dL_dcolor) {
            a.dL_dcolor[3 * idx + 0] = acc[0];
            a.dL_dcolor[3 * idx + 1] = acc[1];
            a.dL_dcolor[3 * idx + 2] = acc[2];
        }
        a.dL_dmean2D[3 * idx + 0] = acc[3];
        a.dL_dmean2D[3 * idx + 1] = acc[4];
        a.dL_dmean2D[3 * idx + 2] = 0.f;
    }
    if (a.dL_dconic) reinterpret_cast<float4*>(a.dL_dconic)[idx] = make_float4(acc[5], acc[6], 0.f, acc[7]);
    store_out1(&a.dL_dopacity[idx], acc[8], a.nt_out != 0);

    const int ncoef_out = a.M;  // dL_dsh is [P, M, 3]
    if (!vis) {
        if (small) {
#pragma unroll
            for (int i = 3; i < 9; i++) (*small)[i] = 0.f;
        } else {
#pragma unroll
            for (int i = 0; i < 3; i++) a.dL_dmean3D[3 * idx + i] = 0.f;
        }
        if (a.dL_dcov3D) {
#pragma unroll
            for (int i = 0; i < 6; i++) a.dL_dcov3D[6 * idx + i] = 0.f;
        }
        if (kDrgb) {
#pragma unroll
            for (int i = 0; i < 19; i++) (*sh19)[i] = 0.f;
        } else if (kHasSH && kSH16) {
#pragma unroll
            for (int i = 0; i < 48; i++) lrow[i] = 0.f;
        } else if (kHasSH) {
            for (int i = 0; i < ncoef_out * 3; i++) a.dL_dsh[(size_t)idx * ncoef_out * 3 + i] = 0.f;
        }
        if (!small)
            for (int i = 0; i < 3; i++) a.dL_dscale[3 * idx + i] = 0.f;
        for (int i = 0; i < 4; i++) a.dL_drot[4 * idx + i] = 0.f;
        return;
    }

    // All loads up front (one memory round trip per thread).
    const float mx = a.means3D[3 * idx], my = a.means3D[3 * idx + 1], mz = a.means3D[3 * idx + 2];
    float cov3D[6];
    float4 qrot = make_float4(0.f, 0.f, 0.f, 0.f);
    float scl[3] = {0.f, 0.f, 0.f};
    if (kHasScales) {
        qrot = reinterpret_cast<const float4*>(a.rotations)[idx];
        scl[0] = a.scales[3 * idx + 0];
        scl[1] = a.scales[3 * idx + 1];
        scl[2] = a.scales[3 * idx + 2];
    }
    if (kHasScales && !a.has_cov_precomp) {
        // the forward's cov3D recomputed from the scale / rotation this pass
        // reads anyway (same code, no contraction: the same bits) instead of
        // 24 more bytes per Gaussian from the geometry buffer
        compute_cov3d(scl, qrot, a.scale_modifier, cov3D);
    } else {
        // cov3D_precomp given (alone, or together with scales / rotations: the
        // forward rendered the precomputed covariance, backward.cu:160 reads
        // it, and the scales still receive the cov3D backward, :395-396)
#pragma unroll
        for (int i = 0; i < 6; i++) cov3D[i] = a.cov3D[6 * idx + i];
    }
    float s[16][3];
    uint8_t cb = 0;
    // the forward's d(rgb)/d(dir) when it stored them: no SH coefficients read
    // (the header word is checked in the drgb-known kernel too: the host picks
    // that kernel from a registry keyed by the rows' address, which cannot see
    // a geometry buffer no forward of this library wrote)
    const bool use_drgb = kHasSH && a.drgb && a.hdr[kHdrDrgb] == 1u;  // uniform
    float d9[9];
    if (kHasSH) {
        if (use_drgb) {
            const float4* row = reinterpret_cast<const float4*>(a.drgb) + 3 * (size_t)idx;
            const float4 r0 = row[0], r1 = row[1], r2 = row[2];
            d9[0] = r0.x; d9[1] = r0.y; d9[2] = r0.z; d9[3] = r0.w;
            d9[4] = r1.x; d9[5] = r1.y; d9[6] = r1.z; d9[7] = r1.w; d9[8] = r2.x;
        } else if constexpr (!kDrgb) {
            load_sh_rows<kSH16>(a, idx, s, lrow);
        } else {
            // drgb-known kernel, rows not written: the preprocess's derivatives
            // from the coefficients (same operands as sh_backward_terms: the
            // same bits), in a phase of their own before the body's peak
            float c[16][3];
            load_sh_rows<true>(a, idx, c);
            const float dox = mx - a.campos[0], doy = my - a.campos[1], doz = mz - a.campos[2];
            const float len = sqrtf(dot3(dox, doy, doz, dox, doy, doz));
            float dx3[3], dy3[3], dz3[3];
            sh_ddir(a.D, c, dox / len, doy / len, doz / len, dx3, dy3, dz3);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                d9[k] = dx3[k];
                d9[3 + k] = dy3[k];
                d9[6 + k] = dz3[k];
            }
        }
        cb = clamped_bits[idx];
    }
    const Mat4 V = load_mat4(a.viewmatrix);
    const Mat4 Pm = load_mat4(a.projmatrix);

    // ---- computeCov2DCUDA (backward.cu:144-274)
    float dmean[3];
    float dcov[6];
    cov2d_backward(mx, my, mz, cov3D, acc[5], acc[6], acc[7], V, a.focal_x, a.focal_y, a.tan_fovx, a.tan_fovy,
                   dmean, dcov);
    if (a.dL_dcov3D) {
#pragma unroll
        for (int i = 0; i < 6; i++) a.dL_dcov3D[6 * idx + i] = dcov[i];
    }

    // ---- preprocessCUDA backward (backward.cu:370-387): projection part (+=)
    proj_backward(mx, my, mz, Pm, acc[3], acc[4], dmean);

    // ---- computeColorFromSH backward (backward.cu:20-139)
    // (two calls with a constant pointer each: a run-time select of d9 or
    // nullptr made the compiler keep d9 in scratch memory)
    if constexpr (kDrgb) {
        float dsh_c[16], dRGB[3];
        sh_backward_terms(a.D, a.campos, mx, my, mz, s, cb, acc, dsh_c, dRGB, dmean, d9);
#pragma unroll
        for (int k = 0; k < 16; k++) (*sh19)[k] = dsh_c[k];
#pragma unroll
        for (int c = 0; c < 3; c++) (*sh19)[16 + c] = dRGB[c];
    } else if (kHasSH) {
        if (use_drgb) sh_backward<kSH16>(a, idx, mx, my, mz, s, cb, acc, dmean, kSH16 ? lrow : nullptr, d9);
        else sh_backward<kSH16>(a, idx, mx, my, mz, s, cb, acc, dmean, kSH16 ? lrow : nullptr, nullptr);
    }
#pragma unroll
    for (int i = 0; i < 3; i++) {
        if (small) (*small)[3 + i] = dmean[i];
        else a.dL_dmean3D[3 * idx + i] = dmean[i];
    }

    // ---- computeCov3D backward (backward.cu:278-341)
    if (kHasScales) {
        float dscale[3];
        float4 dq;
        cov3d_backward(qrot, scl, a.scale_modifier, dcov, dscale, dq);
        store_out4(reinterpret_cast<float4*>(a.dL_drot) + idx, dq, a.nt_out != 0);
        if (small) {
            (*small)[6] = dscale[0];
            (*small)[7] = dscale[1];
            (*small)[8] = dscale[2];
        } else {
            a.dL_dscale[3 * idx + 0] = dscale[0];
            a.dL_dscale[3 * idx + 1] = dscale[1];
            a.dL_dscale[3 * idx + 2] = dscale[2];
        }
    } else {
        if (small) {
            (*small)[6] = (*small)[7] = (*small)[8] = 0.f;
        } else {
            for (int i = 0; i < 3; i++) a.dL_dscale[3 * idx + i] = 0.f;
        }
        for (int i = 0; i < 4; i++) a.dL_drot[4 * idx + i] = 0.f;
    }
}

constexpr int kBgStageNt = 16;  // backward_gaussians_kernel stage flag: dL_dsh rows non-temporal


template <bool kHasSH, bool kHasScales, bool kSH16, bool kSmall = false>
__global__ void __launch_bounds__(256) backward_gaussians_kernel(BackwardGaussArgs a, const float* __restrict__ grad_accum,
                                                                 const uint8_t* __restrict__ clamped_bits, int stage) {
    constexpr bool kStage = kHasSH && kSH16;
    static_assert(!kSmall || kStage, "the small outputs are staged in the SH rows' LDS");
    __shared__ float s_dsh[kStage ? 256 * kShRow : 1];
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    // (not needed when the forward stored d(rgb)/d(dir): the SH coefficients
    // are then never read)
    if (kStage && !(a.drgb && a.hdr[kHdrDrgb] == 1u)) {  // the workgroup's 256 SH rows in, wave-contiguous
        const int g0 = blockIdx.x * blockDim.x;
        const int n = min(256, a.P - g0);
        const float4* in = reinterpret_cast<const float4*>(a.shs) + (size_t)g0 * 12;
        if (n == 256) {
            // a full workgroup: the 12 loads of each thread issued back to back
            // (one memory round trip; the loop below waits for each load before
            // its LDS write -- 12 round trips at 3 waves per SIMD)
            float4 v[12];
#pragma unroll
            for (int k = 0; k < 12; k++) v[k] = in[threadIdx.x + 256 * k];
#pragma unroll
            for (int k = 0; k < 12; k++) {
                const int f = threadIdx.x + 256 * k;
                float* r = s_dsh + (f / 12) * kShRow + 4 * (f % 12);
                r[0] = v[k].x; r[1] = v[k].y; r[2] = v[k].z; r[3] = v[k].w;
            }
        } else {
            for (int f = threadIdx.x; f < n * 12; f += 256) {
                const float4 v = in[f];
                float* r = s_dsh + (f / 12) * kShRow + 4 * (f % 12);
                r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
            }
        }
        __syncthreads();
    }
    // stage_small: the 3-float outputs too go out as the workgroup's
    // contiguous 3 x 256 floats per array (stores at a 12-B stride write one
    // 32-B granule per lane per instruction: ~+23 % write bytes at config 4,
    // profiles/r04d_cfg4_pmc_summary.json)
    float small[12];
    backward_gaussian_body<kHasSH, kHasScales, kSH16>(a, grad_accum, clamped_bits, idx,
                                                      kStage ? s_dsh + threadIdx.x * kShRow : nullptr,
                                                      kSmall ? &small : nullptr);
    if constexpr (kStage) {
        __syncthreads();
        const int g0 = blockIdx.x * blockDim.x;
        const int n = min(256, a.P - g0);
        float4* out = reinterpret_cast<float4*>(a.dL_dsh) + (size_t)g0 * 12;
        const bool nt = (stage & kBgStageNt) != 0;
        for (int f = threadIdx.x; f < n * 12; f += 256) {
            const float* r = s_dsh + (f / 12) * kShRow + 4 * (f % 12);
            store_out4(&out[f], make_float4(r[0], r[1], r[2], r[3]), nt);
        }
        if constexpr (kSmall) {
            __syncthreads();  // the SH rows are out: the LDS holds the small arrays now
            if (idx < a.P) {
#pragma unroll
                for (int i = 0; i < 12; i++) s_dsh[(i / 3) * 768 + 3 * threadIdx.x + i % 3] = small[i];
            }
            __syncthreads();
            const int nf = 3 * n;
            for (int f = threadIdx.x; f < 4 * 192; f += 256) {
                const int q = f / 192, i = f - 192 * q;
                float* d = q == 0 ? a.dL_dmean2D : q == 1 ? a.dL_dmean3D : q == 2 ? a.dL_dscale : a.dL_dcolor;
                if (!d || 4 * i >= nf) continue;
                const float* r = s_dsh + q * 768 + 4 * i;
                float* o = d + 3 * (size_t)g0 + 4 * i;
                if (4 * i + 4 <= nf) {
                    store_out4(reinterpret_cast<float4*>(o), make_float4(r[0], r[1], r[2], r[3]), a.nt_out != 0);
                } else {
                    for (int e = 0; e < 4 && 4 * i + e < nf; e++) o[e] = r[e];
                }
            }
        }
    }
}

// The drgb-known form (the training path: the forward stored d(rgb)/d(dir)):
// no SH-coefficient path (114 VGPRs: 4 waves per SIMD instead of 3) and the
// 192-B dL_dsh rows staged through a half-size LDS area in two rounds of 128
// Gaussians (25 KB, recomputed from the 16 basis values and dL/drgb each
// thread keeps), then the small outputs as in backward_gaussians_kernel.
__global__ void __launch_bounds__(256) backward_gaussians_drgb_kernel(BackwardGaussArgs a,
                                                                      const float* __restrict__ grad_accum,
                                                                      const uint8_t* __restrict__ clamped_bits,
                                                                      int nt) {
    __shared__ float s_half[128 * kShRow];
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    float small[12], sh19[19];
    backward_gaussian_body<true, true, true, true>(a, grad_accum, clamped_bits, idx, nullptr, &small, &sh19);
    const int g0 = blockIdx.x * blockDim.x;
    const int n = min(256, a.P - g0);
    const int ncoef = min((a.D + 1) * (a.D + 1), a.M);
#pragma unroll 1
    for (int h = 0; h < 2; h++) {
        const int gh = g0 + 128 * h, nh = min(128, n - 128 * h);
        if (nh <= 0) break;  // block-uniform
        if (h) __syncthreads();  // the previous round's stores have read the area
        if ((int)(threadIdx.x >> 7) == h && idx < a.P) {
            float* r = s_half + (threadIdx.x & 127) * kShRow;
#pragma unroll
            for (int k = 0; k < 16; k++)
#pragma unroll
                for (int c = 0; c < 3; c++) r[3 * k + c] = k < ncoef ? sh19[k] * sh19[16 + c] : 0.f;
        }
        __syncthreads();
        float4* out = reinterpret_cast<float4*>(a.dL_dsh) + (size_t)gh * 12;
        for (int f = threadIdx.x; f < nh * 12; f += 256) {
            const float* r = s_half + (f / 12) * kShRow + 4 * (f % 12);
            store_out4(&out[f], make_float4(r[0], r[1], r[2], r[3]), nt != 0);
        }
    }
    __syncthreads();  // the SH rows are out: the area holds the small arrays now
    if (idx < a.P) {
#pragma unroll
        for (int i = 0; i < 12; i++) s_half[(i / 3) * 768 + 3 * threadIdx.x + i % 3] = small[i];
    }
    __syncthreads();
    const int nf = 3 * n;
    for (int f = threadIdx.x; f < 4 * 192; f += 256) {
        const int q = f / 192, i = f - 192 * q;
        float* d = q == 0 ? a.dL_dmean2D : q == 1 ? a.dL_dmean3D : q == 2 ? a.dL_dscale : a.dL_dcolor;
        if (!d || 4 * i >= nf) continue;
        const float* r = s_half + q * 768 + 4 * i;
        float* o = d + 3 * (size_t)g0 + 4 * i;
        if (4 * i + 4 <= nf) {
            store_out4(reinterpret_cast<float4*>(o), make_float4(r[0], r[1], r[2], r[3]), a.nt_out != 0);
        } else {
            for (int e = 0; e < 4 && 4 * i + e < nf; e++) o[e] = r[e];
        }
    }
}

// The SH16 + scales kernel: the SH staging loads issued back to back and the
// 3-float outputs stored coalesced through LDS (stage_small: 0.0848 -> 0.0828
// ms at config 2, 0.529 -> 0.479 at config 4, profiles/r04j_ab_bg*.log); the
// drgb-known kernel when the host knows the forward stored d(rgb)/d(dir),
// below 4M Gaussians (config 2 0.0825 -> 0.0747 ms; at config 4 0.465 ->
// 0.486: 4 waves per SIMD help the latency-bound small scene, the two staging
// rounds cost the HBM-bound large one, profiles/r04n_ab_bg*.log, again with
// 48-B rows: 0.4617 vs 0.4703, r04y_ab_bg4.log).  The dL_dsh rows are stored
// with the non-temporal hint (0.0727 -> 0.0697 ms at config 2, 0.4582 ->
// 0.4393 at config 4, profiles/r04z4_ab_nt*.log); the other outputs and the
// input loads are not (+3 % / +9 %, r04z5_*, r04z7_*).  Measured and removed:
// the SH backward as its own kernel, per-thread SH staging loads, one-round
// drgb staging (r04z1_ab_bg*_stage4.log).
void launch_backward_gaussians(const BackwardGaussArgs& args, const GeomView& g, hipStream_t s) {
    if (args.P == 0) return;
    BackwardGaussArgs a = args;
    const dim3 grid((a.P + 255) / 256);
    const bool sh = a.shs != nullptr;
    const bool sh16 = sh && a.M == 16;
    const bool sc = a.scales != nullptr;
    a.nt_out = 0;
#define GS_BG_LAUNCH(A, B, C) \
    hipLaunchKernelGGL((backward_gaussians_kernel<A, B, C>), grid, dim3(256), 0, s, a, g.grad_accum, g.clamped, 0)
    if (sh16 && sc && a.drgb && a.drgb_known && a.P < 4000000)
        hipLaunchKernelGGL(backward_gaussians_drgb_kernel, grid, dim3(256), 0, s, a, g.grad_accum, g.clamped, 1);
    else if (sh16 && sc)
        hipLaunchKernelGGL((backward_gaussians_kernel<true, true, true, true>), grid, dim3(256), 0, s, a,
                           g.grad_accum, g.clamped, kBgStageNt);
    else if (sh16) GS_BG_LAUNCH(true, false, true);
    else if (sh && sc) GS_BG_LAUNCH(true, true, false);
    else if (sh) GS_BG_LAUNCH(true, false, false);
    else if (sc) GS_BG_LAUNCH(false, true, false);
    else GS_BG_LAUNCH(false, false, false);
#undef GS_BG_LAUNCH
}

}  // namespace gsamd

