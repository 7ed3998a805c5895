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

// A 16x16 block is covered by kWaves wave64s with kPPL pixels per lane
// (kWaves * 64 * kPPL = 256).  The block is 4 row groups of 16x4 pixels;
// wave w owns the contiguous groups r = w*kPPL + k (k < kPPL), lane l pixel
// (x, y) = (l & 15, 4r + (l >> 4)) of group r, so a wave's pixels form one
// 16 x 4*kPPL band (the cull below works per row group).
template <int kPPL>
struct PixelSetT {
    float x;  // shared by the lane's pixels
    float y[kPPL];
    uint32_t pid[kPPL];
    bool inside[kPPL];
};

// power = -0.5 (c.x dx^2 + c.z dy^2) - c.y dx dy (forward.cu:331-333,
// backward.cu:466-468), evaluated pre-scaled by log2(e) so exp(power) is one
// v_exp_f32 (exp2) and as a quadratic in dy: p2 = (hz dy + ny dx) dy + hx dx^2
// with (hx, ny, hz) = log2(e) (-c.x/2, -c.y, -c.z/2) computed once per
// Gaussian when it is staged (splat_coef).  For the backward's 4 pixels per
// lane (same x) hx dx^2 and ny dx are per-lane terms, so each pixel costs two
// fmas.  Every kernel evaluates the same expression with explicit fmas, so
// the backward's alpha carries the forward's bits.  sign(p2) = sign(power):
// the reference's `power > 0` skip is `p2 > 0`.
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kHalfLog2e = 0.5f * kLog2e;

__device__ __forceinline__ float4 splat_coef(float4 co) {
    return make_float4(-kHalfLog2e * co.x, -kLog2e * co.y, -kHalfLog2e * co.z, co.w);
}

// p2 from the per-lane terms a = (hx dx) dx and b = ny dx.
__device__ __forceinline__ float splat_p2(float a, float b, float dy, float4 pc) {
    return __builtin_fmaf(__builtin_fmaf(pc.z, dy, b), dy, a);
}

__device__ __forceinline__ float splat_p2(float dx, float dy, float4 pc) {
    return splat_p2((pc.x * dx) * dx, pc.y * dx, dy, pc);
}

// G = exp(power) = 2^p2 (the hardware exp2; the reference's expf within a
// few ulp).
__device__ __forceinline__ float splat_exp(float p2) { return __builtin_amdgcn_exp2f(p2); }

// ---------------------------------------------------- SGPR-mask selects
// The compiler's selects take their condition in VCC (VOP2 v_cndmask_b32);
// on gfx950 that form issues at ~15.5 cycles per wave instruction, the e64
// form with the lane mask in an SGPR pair at ~4.3 (tools/valu_rate.hip,
// profiles/r04a_valu_rate.log).  These helpers select on a 64-bit lane mask
// from __builtin_amdgcn_fcmpf / _uicmp (v_cmp_*_e64 into an SGPR pair).  The
// select starts with s_nop 1: a mask written by a VALU compare and read as a
// lane mask by a VALU needs 2 wait states on gfx950 (the compiler inserts them
// for its own selects, but cannot see into the asm).  (Used by the backward
// blend; in the forward and the AMR fold the mask form measured slower than
// the compiler's selects)
constexpr int kFcmpUGE = 11, kFcmpULE = 13, kIcmpULT = 36;

// m ? x : 0
__device__ __forceinline__ float gs_sel_zero_v(uint64_t m, float x) {
    float r;
    asm("s_nop 1\n\tv_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(x), "s"(m));
    return r;
}
// (m ? x : 0, m ? y : 0)
__device__ __forceinline__ void gs_sel2_zero_v(uint64_t m, float x, float y, float& rx, float& ry) {
    asm("s_nop 1\n\t"
        "v_cndmask_b32_e64 %0, 0, %2, %4\n\t"
        "v_cndmask_b32_e64 %1, 0, %3, %4"
        : "=&v"(rx), "=&v"(ry)
        : "v"(x), "v"(y), "s"(m));
}

// p2 <= 0 at every pixel, provably: the scaled form hx dx^2 + ny dx dy + hz
// dy^2 (pc = splat_coef) is negative definite when hx, hz < 0 and ny^2 <
// 0.998 * 4 hx hz; then its exact value is <= -(1 - 0.999) (|hx| dx^2 + |hz|
// dy^2) while the rounding of its evaluation (two fmas after two products)
// is < 1e-6 of that sum -- the computed p2 is never > 0, so the reference's
// `power > 0` skip cannot fire.  Coefficients and the offset to the block
// (ax, ay) bounded: every term < 1e19, nothing overflows.
__device__ __forceinline__ bool splat_form_safe(float4 pc, float ax, float ay) {
    return pc.x < 0.f && pc.z < 0.f && pc.y * pc.y < 0.998f * 4.0f * (pc.x * pc.z) && pc.x > -1e6f &&
           pc.z > -1e6f && fabsf(pc.y) < 1e6f && ax < 1e6f && ay < 1e6f;
}

// 16x16 block at (ox, oy) with pixel stride `st` (1 = base, 2 = AMR sub-lattice).
template <int kPPL, int kWaves>
__device__ __forceinline__ PixelSetT<kPPL> make_pixels_t(int W, int H, uint32_t ox, uint32_t oy, uint32_t st) {
    const uint32_t t = threadIdx.x;
    const uint32_t w = t >> 6, l = t & 63;
    PixelSetT<kPPL> p;
    const uint32_t px = ox + st * (l & 15);
    p.x = (float)px;
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
        const uint32_t py = oy + st * (4 * (w * kPPL + k) + (l >> 4));
        p.y[k] = (float)py;
        p.inside[k] = px < (uint32_t)W && py < (uint32_t)H;
        p.pid[k] = p.inside[k] ? (uint32_t)W * py + px : 0u;
    }
    return p;
}


// ------------------------------------------------------ XCD-aware placement
// Blocks b and b + 8 run on one XCD (round-robin dispatch; MI355X_MICROARCH.md
// §Workgroup dispatch -- observed, speed only), and each XCD has its own 4 MiB
// L2.  With row-major tiles, neighbouring tiles -- which share most of their
// Gaussians -- land on 8 different L2s and every gather of a shared record
// misses 8 times.  Instead the tiles are laid out in a 2-D-compact order
// (strips of kXcdStrip tile rows, walked column by column) and that order is
// cut into 8 contiguous chunks, chunk x going to the blocks b = 8 k + x: each
// XCD renders one compact region, in order.
constexpr int kXcdStrip = 4;

// position p of the strip order -> tile index
__host__ __device__ __forceinline__ int xcd_strip_tile_of_pos(int p, int gx, int gy) {
    const int s = p / (kXcdStrip * gx), q = p - s * kXcdStrip * gx;
    const int rows = min(kXcdStrip, gy - s * kXcdStrip);
    const int col = q / rows, r = q - col * rows;
    return (s * kXcdStrip + r) * gx + col;
}

// tile index -> position p of the strip order
__host__ __device__ __forceinline__ int xcd_strip_pos_of_tile(int t, int gx, int gy) {
    const int row = t / gx, col = t - row * gx;
    const int s = row / kXcdStrip, r = row - s * kXcdStrip;
    const int rows = min(kXcdStrip, gy - s * kXcdStrip);
    return s * kXcdStrip * gx + col * rows + r;
}

// chunk x of the NB positions: start(x) = x q + min(x, NB % 8), q = NB / 8
__host__ __device__ __forceinline__ int xcd_chunk_start(int x, int NB) { return x * (NB / 8) + min(x, NB % 8); }

__host__ __device__ __forceinline__ int xcd_chunk_of_pos(int p, int NB) {
    const int q = NB / 8, rem = NB % 8;
    if (p < rem * (q + 1)) return p / (q + 1);
    return rem + (p - rem * (q + 1)) / q;
}

// block b -> tile (b = 8 k + x takes position start(x) + k)
__device__ __forceinline__ int xcd_block_tile(int b, int gx, int gy) {
    const int NB = gx * gy;
    if (NB < 8) return b;
    return xcd_strip_tile_of_pos(xcd_chunk_start(b & 7, NB) + (b >> 3), gx, gy);
}

// ------------------------------------------------------------ row-group cull
// A (pixel, Gaussian) pair is blended only if alpha = min(0.99, o*exp(power))
// >= 1/255 with power = -Q/2, Q = d^T C d (C = conic, d = mean - pixel), i.e.
// only if Q <= 2 ln(255 o).  That set is an ellipse; its bounding box has
// half-widths sqrt(thr * C_yy / det C) and sqrt(thr * C_xx / det C).  A
// Gaussian whose box misses all pixels of a 16x4 row group is skipped by
// every pixel of the group in the reference too (the alpha < 1/255
// `continue`, base/cr/forward.cu:341-343, backward.cu:480-482), so skipping
// it is exact, provided the box is conservative w.r.t. the kernel's own
// float evaluation of Q, exp and the threshold:
//   * thr = 2.04 ln(255 o) + 2e-3 (2 % + absolute slack), box widths x1.001
//     + 0.02 px;
//   * the rounding of the kernel's Q is <= ~4 eps (1+rho)/(1-rho) Q, with
//     rho = |C_xy| / sqrt(C_xx C_yy); the cull is used only for rho^2 <
//     0.998 (error < 5e-4 Q, well inside the 2 % slack), otherwise and for
//     any non-finite value the Gaussian is kept ("hit");
//   * o*255 < 0.999 means alpha <= o < 1/255 for every pixel (exp(power) <= 1
//     once power <= 0, and power > 0 is skipped anyway): never blended.
// The same test on any pixel rectangle culls the AMR quadrant lists.
//
// The per-Gaussian part of the test: threshold, box half-widths and the
// edge-minimum slopes.  `never`: alpha < 1/255 at every pixel.
struct SplatBox {
    float2 xy;
    float4 co;
    float thr, hx, hy, kyx, kxy;
    bool ok, never;
};

__device__ __forceinline__ SplatBox splat_box(float2 xy, float4 co) {
    SplatBox b;
    b.xy = xy;
    b.co = co;
    const float o = co.w;
    b.never = o * 255.0f < 0.999f;  // false for NaN: kept
    const float lt = fmaxf(__logf(255.0f * o), 0.0f);
    b.thr = 2.04f * lt + 2e-3f;
    const float cxz = co.x * co.z;
    b.ok = co.x > 0.0f && co.z > 0.0f && co.y * co.y < 0.998f * cxz;
    const float det = cxz - co.y * co.y;
    b.hx = b.ok ? sqrtf(b.thr * co.z / det) * 1.001f + 0.02f : __builtin_inff();
    b.hy = b.ok ? sqrtf(b.thr * co.x / det) * 1.001f + 0.02f : __builtin_inff();
    b.kyx = -co.y / co.z;
    b.kxy = -co.y / co.x;
    return b;
}

// Does the Gaussian reach alpha >= 1/255 anywhere in the pixel-centre
// rectangle [x0, x1] x [y0, y1]?  (Conservative: false only when no pixel of
// the rectangle can pass the reference's alpha test.)  "misses" comparisons
// are false for NaN / inf widths -> kept.
__device__ __forceinline__ bool splat_rect_hit(const SplatBox& b, float x0, float x1, float y0, float y1) {
    if (b.never) return false;
    const float2 xy = b.xy;
    if (xy.x + b.hx < x0 || xy.x - b.hx > x1) return false;
    if (xy.y + b.hy < y0 || xy.y - b.hy > y1) return false;
    if (!b.ok) return true;  // ill-conditioned or non-finite: box test only
    // Exact second stage: the minimum of Q over the rectangle (grown by 0.02
    // px) against the same threshold; a box that only grazes the rectangle
    // with a corner the ellipse does not reach is culled too.  The minimum
    // lies inside (Q = 0) or on an edge, where Q is a 1-D quadratic minimised
    // at a clamped point; rounding of that point moves Q by O(c * (1e-4
    // px)^2), far inside the margins above.
    const float xa = x0 - 0.02f, xb = x1 + 0.02f, ya = y0 - 0.02f, yb = y1 + 0.02f;
    if (xy.x >= xa && xy.x <= xb && xy.y >= ya && xy.y <= yb) return true;
    const float4 co = b.co;
    float q = __builtin_inff();
#pragma unroll
    for (int e = 0; e < 2; e++) {  // vertical edges x = xa, xb
        const float dx = xy.x - (e ? xb : xa);
        const float dy = fminf(fmaxf(b.kyx * dx, xy.y - yb), xy.y - ya);
        q = fminf(q, co.x * dx * dx + 2.0f * co.y * dx * dy + co.z * dy * dy);
    }
#pragma unroll
    for (int e = 0; e < 2; e++) {  // horizontal edges y = ya, yb
        const float dy = xy.y - (e ? yb : ya);
        const float dx = fminf(fmaxf(b.kxy * dy, xy.x - xb), xy.x - xa);
        q = fminf(q, co.x * dx * dx + 2.0f * co.y * dx * dy + co.z * dy * dy);
    }
    return !(q > b.thr);  // NaN -> kept
}

// Bit r set when the Gaussian can reach row group r of the 16x16 block at
// (ox, oy) with pixel stride st (1 = base, 2 = AMR sub-lattice).
__device__ __forceinline__ uint32_t splat_group_mask(float2 xy, float4 co, float ox, float oy, float st) {
    const SplatBox b = splat_box(xy, co);
    const float x0 = ox, x1 = ox + 15.0f * st;
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const float y0 = oy + st * (4.0f * r), y1 = oy + st * (4.0f * r + 3.0f);
        if (splat_rect_hit(b, x0, x1, y0, y1)) m |= 1u << r;
    }
    return m;
}

// Backward launch order: the work bucket of a tile whose blend reads w
// entries, 0 = heaviest (16 log2(w + 1): steps of 2^(1/16), 256 buckets).
__device__ __forceinline__ uint32_t order_bucket64(uint32_t w) {
    return 255u - min((uint32_t)(16.0f * __log2f((float)w + 1.0f)), 255u);
}

// Scalar copy of a wave-uniform 64-bit value held in VGPRs.
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Per batch: s_bal[c * 4 + r] = 64-bit mask over batch slots 64c..64c+63 of
// the Gaussians meeting row group r.  Called by every thread after it has
// computed the mask of its own slot (0 for empty slots).
template <int kWaves>
__device__ __forceinline__ void publish_group_masks(uint32_t my_mask, uint64_t* s_bal) {
    const uint32_t c = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint64_t b = __ballot((my_mask >> r) & 1u);
        if ((threadIdx.x & 63) == 0) s_bal[c * 4 + r] = b;
    }
}

template <int kPPL>
struct BlendStateT {
    float T[kPPL];
    float C[kPPL][3];
    uint32_t last[kPPL];
};

// The select form of one (pixel, Gaussian) pair (forward.cu:333-352): the
// reference's per-pixel continues / early stop become values -- a rejected
// pair gets alpha 0, which leaves C (C + f * 0 * T) and T (T * (1 - 0))
// unchanged bit for bit.  A pixel that stops keeps T = -|T| (its final
// transmittance, negated), so T (1 - a) < 1e-4 holds for every later Gaussian
// and a = 0 follows from the stop test itself -- alpha is the plain
// min(0.99, o G), and the stop select writes -|T| through the VOP3 source
// modifiers.  The last contributor is tracked as the entry's LDS byte offset
// (lo, the VGPR the record reads already use) and converted once per 64
// entries.  No exec masks, no SALU bookkeeping.
template <bool kSafe = false>
__device__ __forceinline__ bool blend_one_sel2(float2 xy, float4 co, float4 f, float pxx, float pxy, uint32_t lo,
                                               float& T, float (&C)[3], uint32_t& last_lo) {
    const float dx = xy.x - pxx, dy = xy.y - pxy;
    const float p = splat_p2(dx, dy, co);
    float a = fminf(0.99f, co.w * splat_exp(p));
    // power > 0: skipped (kSafe: splat_form_safe -- the computed power is
    // never > 0 over the tile, so the test cannot fire)
    if (!kSafe) a = (p > 0.0f) ? 0.0f : a;
    a = (a < 1.0f / 255.0f) ? 0.0f : a;  // alpha < 1/255: skipped
    const float test_T = T * (1.0f - a);
    const bool stop = test_T < 0.0001f;  // false whenever a == 0 and T >= 1e-4; true for every finished pixel
    a = stop ? 0.0f : a;
    const float w = a * T;
    C[0] = __builtin_fmaf(f.x, w, C[0]);
    C[1] = __builtin_fmaf(f.y, w, C[1]);
    C[2] = __builtin_fmaf(f.z, w, C[2]);
    T = stop ? -fabsf(T) : test_T;
    const bool blended = a != 0.0f;
    last_lo = blended ? lo : last_lo;
    return blended;
}

// Front-to-back blend of `range` for the thread's kPPL pixels.  Called by the
// whole workgroup (kWaves waves); LDS batches hold 64*kWaves Gaussians.
// (ox, oy, st): the block origin and pixel stride, for the row-group cull.
// kSel (the base forward's default, 4 waves x 1 pixel per lane): the select
// form (blend_one_sel2), two Gaussians per iteration, the `power > 0` test
// dropped in 64-slot chunks whose visited entries are all provably negative
// definite over the tile (splat_form_safe; one loop copy per case), the
// wave's exit tested after every pair of entries, and the exact row-group
// hit codes recorded for the backward.  !kSel: the predicate form for any
// kPPL (the fallback geometry and the AMR full-list blocks).
template <int kPPL, int kWaves, bool kSel = false>
__device__ __forceinline__ BlendStateT<kPPL> blend_tile_t(uint2 range, const PixelSetT<kPPL>& px, float ox, float oy,
                                                          float st, const uint32_t* __restrict__ point_list,
                                                          const float2* __restrict__ means2D,
                                                          const float* __restrict__ features,
                                                          const float4* __restrict__ conic_opacity, float4* s_a,
                                                          float4* s_co, float* s_b, uint64_t* s_bal,
                                                          bool cull, uint8_t* __restrict__ hit_codes = nullptr,
                                                          uint64_t* s_hit = nullptr) {
#pragma clang fp contract(fast)
    static_assert(!kSel || kPPL == 1, "the select form is the 1-pixel-per-lane geometry");
    constexpr uint32_t kB = 64 * kWaves;
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6;
    // Exact row-group hit codes (kSel, hit_codes given): bit w of entry j's
    // code = some pixel of wave w's row group blended entry j -- precisely
    // the (row group, entry) pairs with a contributing pixel in the backward
    // (a pixel blends entry j iff j < n_contrib and the alpha tests pass,
    // backward.cu:466-482).  Wave w collects its 64-bit hit set per 64 batch
    // slots in s_hit[c kWaves + w]; the batch's codes are stored after the
    // next barrier.
    const bool rec = kSel && hit_codes != nullptr;
    auto flush_codes = [&](uint32_t fb0) {
        if (fb0 + tid < range.y - range.x) {
            const uint32_t c = tid >> 6, bit = tid & 63;
            uint32_t code = 0;
#pragma unroll
            for (int w = 0; w < kWaves; w++) code |= (uint32_t)((s_hit[c * kWaves + w] >> bit) & 1ull) << w;
            hit_codes[range.x + fb0 + tid] = (uint8_t)code;
        }
    };
    BlendStateT<kPPL> st_;
    bool done[kPPL];
#pragma unroll
    for (int k = 0; k < kPPL; k++) {
        st_.T[k] = (kSel && !px.inside[k]) ? -1.0f : 1.0f;  // (kSel: finished = negative T)
        st_.C[k][0] = st_.C[k][1] = st_.C[k][2] = 0.f;
        st_.last[k] = 0;
        done[k] = !px.inside[k];
    }
    const uint32_t n = range.y - range.x;
    uint32_t b0 = 0;
    for (; b0 < n; b0 += kB) {
        bool any = false;
#pragma unroll
        for (int k = 0; k < kPPL; k++) any |= !done[k];
        if (kWaves == 1) {
            if (__ballot(any) == 0ull) break;  // the whole tile is saturated
            __syncthreads();                     // single-wave workgroup: LDS fence only
        } else {
            if (!__syncthreads_or(any)) break;
        }
        if (rec && b0 > 0) flush_codes(b0 - kB);  // the previous batch's codes (s_hit rewritten after the next barrier)
        uint32_t gm = 0;
        bool safe = false;
        if (b0 + tid < n) {
            const uint32_t id = point_list[range.x + b0 + tid];
            const float2 xy = means2D[id];
            const float4 co = conic_opacity[id];
            // (x, y, r, g) + the scaled conic / opacity as two b128 reads, b as
            // one b32 (LDS cycles per wave-read: b128 4, b96 8, b64 / b32 2)
            s_a[tid] = make_float4(xy.x, xy.y, features[3 * id], features[3 * id + 1]);
            s_co[tid] = splat_coef(co);
            s_b[tid * (kSel ? 4 : 1)] = features[3 * id + 2];  // (kSel: at a 16-B stride, one address for all reads)
            gm = cull ? splat_group_mask(xy, co, ox, oy, st) : 0xfu;
            if (kSel) safe = splat_form_safe(splat_coef(co), fabsf(xy.x - ox), fabsf(xy.y - oy));
        }
        publish_group_masks<kWaves>(gm, s_bal);
        if (kSel) {
            const uint64_t sb = __ballot(safe);
            if ((tid & 63) == 0) s_bal[4 * kWaves + (tid >> 6)] = sb;
        }
        __syncthreads();
        if (rec && (tid & 63) == 0)
#pragma unroll
            for (int c = 0; c < kWaves; c++) s_hit[c * kWaves + wave] = 0ull;
        if (__ballot(any) == 0ull) continue;  // this wave is done; keep joining the barriers
        bool wave_alive = true;
#pragma unroll 1
        for (uint32_t c = 0; c < (uint32_t)kWaves && wave_alive; c++) {
            uint64_t mk[kPPL];
            uint64_t todo = 0;
#pragma unroll
            for (int k = 0; k < kPPL; k++) {
                mk[k] = uniform_u64(s_bal[c * 4 + wave * kPPL + k]);
                todo |= mk[k];
            }
            if constexpr (kSel) {
                const uint64_t safe_m = uniform_u64(s_bal[4 * kWaves + c]);
                uint64_t hits = 0;
                uint32_t last_lo = ~0u;
                const char* sa = reinterpret_cast<const char*>(s_a);
                const char* sco = reinterpret_cast<const char*>(s_co);
                const char* sb = reinterpret_cast<const char*>(s_b);
                auto loop = [&](auto kSafeT) {
                    constexpr bool kSafe = decltype(kSafeT)::value;
                    while (todo) {
                        const uint32_t bA = (uint32_t)__builtin_ctzll(todo);
                        todo &= todo - 1;
                        const bool two = todo != 0;  // wave-uniform
                        const uint32_t bB = two ? (uint32_t)__builtin_ctzll(todo) : bA;
                        if (two) todo &= todo - 1;
                        const uint32_t loA = (c * 64 + bA) * 16, loB = (c * 64 + bB) * 16;
                        const float4 sA = *reinterpret_cast<const float4*>(sa + loA);
                        const float4 sB = *reinterpret_cast<const float4*>(sa + loB);
                        const float4 coA = *reinterpret_cast<const float4*>(sco + loA);
                        const float4 coB = *reinterpret_cast<const float4*>(sco + loB);
                        const float bAc = *reinterpret_cast<const float*>(sb + loA);
                        const float bBc = *reinterpret_cast<const float*>(sb + loB);
                        const bool hA = blend_one_sel2<kSafe>(make_float2(sA.x, sA.y), coA,
                                                              make_float4(sA.z, sA.w, bAc, 0.f), px.x, px.y[0], loA,
                                                              st_.T[0], st_.C[0], last_lo);
                        hits |= __ballot(hA) != 0ull ? 1ull << bA : 0ull;
                        if (two) {
                            const bool hB = blend_one_sel2<kSafe>(make_float2(sB.x, sB.y), coB,
                                                                  make_float4(sB.z, sB.w, bBc, 0.f), px.x, px.y[0],
                                                                  loB, st_.T[0], st_.C[0], last_lo);
                            hits |= __ballot(hB) != 0ull ? 1ull << bB : 0ull;
                        }
                        // every pixel of the wave finished: the rest of the chunk
                        // holds entries no pixel can blend any more
                        if (__ballot(st_.T[0] > 0.0f) == 0ull) break;  // wave-uniform
                    }
                };
                if ((todo & ~safe_m) == 0ull) loop(std::integral_constant<bool, true>{});
                else loop(std::integral_constant<bool, false>{});
                // lo = 16 j, contributor = b0 + j + 1
                if (last_lo != ~0u) st_.last[0] = b0 + (last_lo >> 4) + 1;
                if (rec && (tid & 63) == 0) s_hit[c * kWaves + wave] = hits;
                done[0] = st_.T[0] < 0.0f;
                if (__ballot(!done[0]) == 0ull) wave_alive = false;
                continue;
            }
            while (todo) {
                const uint32_t bit = (uint32_t)__builtin_ctzll(todo);
                todo &= todo - 1;
                const uint32_t j = c * 64 + bit;
                const float4 a4 = s_a[j];
                const float2 xy = make_float2(a4.x, a4.y);
                const float4 co = s_co[j];
                const float dx = xy.x - px.x;
                const float pa = (co.x * dx) * dx, pb = co.y * dx;
                const uint32_t contributor = b0 + j + 1;
                bool alive = false;
#pragma unroll
                for (int k = 0; k < kPPL; k++) {
                    alive |= !done[k];
                    if (!((mk[k] >> bit) & 1ull)) continue;  // wave-uniform: culled for this row group
                    const float dy = xy.y - px.y[k];
                    const float power = splat_p2(pa, pb, dy, co);
                    const float alpha = fminf(0.99f, co.w * splat_exp(power));
                    const float test_T = st_.T[k] * (1 - alpha);
                    // forward.cu:333-352's per-pixel continues as predicates (only
                    // wave-uniform branches save SIMD time)
                    const bool hit = !done[k] && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
                    const bool stop = hit && test_T < 0.0001f;
                    done[k] = done[k] || stop;
                    if (!hit || stop) continue;
                    const float4 f = make_float4(a4.z, a4.w, s_b[j], 0.f);
                    const float w = alpha * st_.T[k];
                    st_.C[k][0] = __builtin_fmaf(f.x, w, st_.C[k][0]);
                    st_.C[k][1] = __builtin_fmaf(f.y, w, st_.C[k][1]);
                    st_.C[k][2] = __builtin_fmaf(f.z, w, st_.C[k][2]);
                    st_.T[k] = test_T;
                    st_.last[k] = contributor;
                }
                if (__ballot(alive) == 0ull) {
                    wave_alive = false;
                    break;
                }
            }
        }
    }
    if (rec) {  // the last processed batch (b0 - kB; every thread leaves the loop together)
        __syncthreads();
        if (b0 > 0) flush_codes(b0 - kB);
    }
    if constexpr (kSel) st_.T[0] = fabsf(st_.T[0]);  // (finished pixels: -T_final)
    return st_;
}

// ------------------------------------------------------- wave reductions
// Full 64-lane sums of 9 values by transposition (gfx950 v_permlane32_swap /
// v_permlane16_swap) instead of 9 independent DPP trees.  For a group of 4
// registers (a, b, c, d), rows = 16-lane quarters:
//   permlane32_swap(a, b); a + b  -> [a0+a2, a1+a3, b0+b2, b1+b3]   (same for c, d)
//   permlane16_swap(ab, cd); sum  -> [a, c, b, d] row partials in ONE register
//   row_shr 1, 2, 4, 8            -> lane 15 of row r holds the total of
//                                    value ((r & 1) << 1 | r >> 1) of the group.
// Two groups (g0..g3, g4..g7) cost 6 swaps + 6 adds + 8 DPP adds; g8 takes
// the plain tree (6 DPP adds, total in lane 63): 26 VALU ops instead of the
// 45 of dpp_sum9_halves, and one full sum per value (no half-wave partials).
// After it: lane 16r + 15 holds za = g[q(r)] and zb = g[4 + q(r)]; lane 63
// also holds g8.  Must run with all 64 lanes active.
__device__ __forceinline__ int swap_sum_slot(int row) { return ((row & 1) << 1) | (row >> 1); }

__device__ __forceinline__ float pl_add32(float a, float b) {
    // (the two halves go through named scalars: subscripting the returned
    // vector directly inside the expression miscompiles to r[0] + r[0] with
    // ROCm 7.2's clang)
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                                                    false, false);
    const uint32_t r0 = r[0], r1 = r[1];
    return __builtin_bit_cast(float, r0) + __builtin_bit_cast(float, r1);
}

__device__ __forceinline__ float pl_add16(float a, float b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                                                    false, false);
    const uint32_t r0 = r[0], r1 = r[1];
    return __builtin_bit_cast(float, r0) + __builtin_bit_cast(float, r1);
}

// Swaps returning both halves (for packed adds of the pairs).
typedef float gs_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ gs_f2 pl_swap32(float a, float b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                                                    false, false);
    const uint32_t r0 = r[0], r1 = r[1];
    return gs_f2{__builtin_bit_cast(float, r0), __builtin_bit_cast(float, r1)};
}
__device__ __forceinline__ gs_f2 pl_swap16(float a, float b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                                                    false, false);
    const uint32_t r0 = r[0], r1 = r[1];
    return gs_f2{__builtin_bit_cast(float, r0), __builtin_bit_cast(float, r1)};
}

// Transposition half of swap_sum9 with packed adds, for sums finished elsewhere: after it
// row r (lanes 16r..16r+15) of za holds the 16 column partials of value
// swap_sum_slot(r), zb those of 4 + swap_sum_slot(r); g[8] holds row r's sum
// in lane 16 r + 15.  9 swap / packed-add issues + 4 DPP adds.
template <int kCtrl, int kRowMask, bool kBound>
__device__ __forceinline__ float dpp_add(float e) {
    return e + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, e), kCtrl, kRowMask,
                                                                      0xf, kBound));
}
template <bool kG8>
__device__ __forceinline__ void swap_rows8_pk_t(float (&g)[9], float& za, float& zb) {
    const gs_f2 p0 = pl_swap32(g[0], g[1]), p4 = pl_swap32(g[4], g[5]);
    const gs_f2 p2 = pl_swap32(g[2], g[3]), p6 = pl_swap32(g[6], g[7]);
    const gs_f2 abef = gs_f2{p0.x, p4.x} + gs_f2{p0.y, p4.y};
    const gs_f2 cdgh = gs_f2{p2.x, p6.x} + gs_f2{p2.y, p6.y};
    const gs_f2 q0 = pl_swap16(abef.x, cdgh.x), q1 = pl_swap16(abef.y, cdgh.y);
    const gs_f2 z = gs_f2{q0.x, q1.x} + gs_f2{q0.y, q1.y};
    za = z.x;
    zb = z.y;
    if constexpr (kG8) {
        // g8: the DPP row tree (compiler-scheduled, so it interleaves with the
        // swaps above instead of waiting out its own hazards); lane 16 r + 15
        // ends with row r's sum
        float e = g[8];
        e = dpp_add<0x111, 0xf, true>(e);   // row_shr:1
        e = dpp_add<0x112, 0xf, true>(e);   // row_shr:2
        e = dpp_add<0x114, 0xf, true>(e);   // row_shr:4
        e = dpp_add<0x118, 0xf, true>(e);   // row_shr:8
        g[8] = e;
    }
}

__device__ __forceinline__ void swap_sum9(float (&g)[9], float& za, float& zb) {
    const float ab = pl_add32(g[0], g[1]), cd = pl_add32(g[2], g[3]);
    const float ef = pl_add32(g[4], g[5]), gh = pl_add32(g[6], g[7]);
    za = pl_add16(ab, cd);
    zb = pl_add16(ef, gh);
    float e = g[8];
    asm volatile(
        "s_nop 1\n"
        "v_add_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %2, %2, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %2, %2, %2 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %2, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_add_f32_dpp %2, %2, %2 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "s_nop 1\n"
        "v_add_f32_dpp %2, %2, %2 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "s_nop 1\n"
        "v_add_f32_dpp %2, %2, %2 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        : "+v"(za), "+v"(zb), "+v"(e));
    g[8] = e;
}

}  // namespace gsamd
