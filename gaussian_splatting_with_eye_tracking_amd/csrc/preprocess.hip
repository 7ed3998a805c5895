// preprocess.hip -- per-Gaussian forward preprocess for gfx950.
//
// Follows base/cr/forward.cu:155-256 (preprocessCUDA) and its helpers
// computeCov3D (:118-152), computeCov2D (:74-113), computeColorFromSH
// (:20-71), in_frustum (base/cr/auxiliary.h:139-164).  One thread per
// Gaussian; HBM-bound (≈236 B read per visible Gaussian at SH degree 3).
//
// MI355X-specific:
//   * the tile histogram the binning needs is fused here:
//     each visible Gaussian adds 1 to every tile of its rect with a no-return
//     global atomic, so the binning needs no P-wide scan;
//   * SH rows are read as float4 when M == 16 (192-B rows are 16-B aligned);
//   * no FMA contraction (file compiled with -ffp-contract=off): depth,
//     means2D and radius are bit-identical to the oracle, which makes the
//     tile keys bit-exact.
#include <algorithm>

#include "gs_blend.cuh"
#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

// Load this Gaussian's SH coefficients (zero past the active degree).
template <bool kSH16>
__device__ __forceinline__ void load_sh(int deg, int M, const float* __restrict__ sh, float (&c)[16][3]) {
    const int ncoef = min((deg + 1) * (deg + 1), M);
    if (kSH16) {
        const float4* s4 = reinterpret_cast<const float4*>(sh);
        float buf[48];
#pragma unroll
        for (int i = 0; i < 12; i++) {
            const float4 v = (i * 4 < ncoef * 3) ? s4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            buf[4 * i + 0] = v.x; buf[4 * i + 1] = v.y; buf[4 * i + 2] = v.z; buf[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int k = 0; k < 16; k++)
#pragma unroll
            for (int ch = 0; ch < 3; ch++) c[k][ch] = buf[3 * k + ch];
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++)
#pragma unroll
            for (int ch = 0; ch < 3; ch++) c[k][ch] = (k < ncoef) ? sh[3 * k + ch] : 0.f;
    }
}

// base/cr/forward.cu:20-71 on preloaded coefficients.
__device__ __forceinline__ float3 eval_sh_color(int deg, const float (&c)[16][3], float x, float y, float z,
                                                uint8_t& clamped_bits) {
    float res[3];
#pragma unroll
    for (int ch = 0; ch < 3; ch++) res[ch] = SH_C0 * c[0][ch];
    if (deg > 0) {
        const float k1 = SH_C1 * y, k2 = SH_C1 * z, k3 = SH_C1 * x;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) res[ch] = res[ch] - k1 * c[1][ch] + k2 * c[2][ch] - k3 * c[3][ch];
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            const float k4 = SH_C2_0 * xy;
            const float k5 = SH_C2_1 * yz;
            const float k6 = SH_C2_2 * (2.0f * zz - xx - yy);
            const float k7 = SH_C2_3 * xz;
            const float k8 = SH_C2_4 * (xx - yy);
#pragma unroll
            for (int ch = 0; ch < 3; ch++)
                res[ch] = res[ch] + k4 * c[4][ch] + k5 * c[5][ch] + k6 * c[6][ch] + k7 * c[7][ch] + k8 * c[8][ch];
            if (deg > 2) {
                const float k9 = SH_C3_0 * y * (3.0f * xx - yy);
                const float k10 = SH_C3_1 * xy * z;
                const float k11 = SH_C3_2 * y * (4.0f * zz - xx - yy);
                const float k12 = SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                const float k13 = SH_C3_4 * x * (4.0f * zz - xx - yy);
                const float k14 = SH_C3_5 * z * (xx - yy);
                const float k15 = SH_C3_6 * x * (xx - 3.0f * yy);
#pragma unroll
                for (int ch = 0; ch < 3; ch++)
                    res[ch] = res[ch] + k9 * c[9][ch] + k10 * c[10][ch] + k11 * c[11][ch] + k12 * c[12][ch] +
                              k13 * c[13][ch] + k14 * c[14][ch] + k15 * c[15][ch];
            }
        }
    }
    clamped_bits = 0;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        res[ch] += 0.5f;
        if (res[ch] < 0) clamped_bits |= (uint8_t)(1u << ch);
        res[ch] = fmaxf(res[ch], 0.0f);
    }
    return make_float3(res[0], res[1], res[2]);
}

// kDma (SH16): each wave copies its 64 Gaussians' 192-B SH rows (12 KB,
// contiguous) global -> LDS with 12 wave-contiguous global_load_lds_dwordx4
// (no VGPRs) at the top of the kernel, so the coalesced copy runs under the
// geometry math; each visible thread then reads its row from LDS.  Culled
// Gaussians' rows are copied too (~15 % more SH bytes at configs 2 / 4) --
// the price of whole-line requests instead of 12 scattered 16-B loads per
// thread.
constexpr int kPpThreads = 256;
// LDS row of one Gaussian: the 48 SH floats + one 16-B pad.  At 52 floats
// (13 pieces of 16 B) the 16 lanes of each b128 access hit 16 distinct
// 4-bank groups (52 l mod 64 = 4 (13 l mod 16)): no conflicts; at 48 every
// fourth lane repeated a group and the compiler's b32 reads hit 4 banks per
// wave (SQ_LDS_BANK_CONFLICT 28.6 cycles per LDS instruction at config 2,
// profiles/r06a_cfg2_sq_counters.json).  The LDS-DMA writes 16-B pieces to
// consecutive LDS addresses per lane, so the padding comes from the sources:
// piece p of a wave's area is row p / 13, piece p % 13, and piece 12 of
// every row is left unwritten.
constexpr int kShStride = 52;

// Everything after the loads of one Gaussian (forward.cu:155-256): the cull,
// cov2D, conic, radius / rect, SH colour (coefficients from load_shc, only for
// survivors), the records.  radii / tiles_touched were zeroed by the caller.
template <bool kHasSH, bool kCovPrecomp, typename ShFn>
__device__ __forceinline__ void pp_gaussian(const PreprocessArgs& a, const GeomView& g, int* __restrict__ radii,
                                            uint32_t* __restrict__ tile_count, int idx, bool radii_copy, float mx,
                                            float my, float mz, const float (&sc)[3], float4 q, float (&cov3D)[6],
                                            float opacity, const Mat4& V, const Mat4& Pm, ShFn&& load_shc,
                                            float* stage) {
    // in_frustum (auxiliary.h:139-164): near plane only.
    const float3 p_view = transform_point_4x3(mx, my, mz, V);
    if (p_view.z <= 0.2f) {
        if (a.prefiltered) g.hdr[kHdrError] = a.err_token;  // the reference __trap()s here
        return;
    }
    const float4 p_hom = transform_point_4x4(mx, my, mz, Pm);
    const float p_w = 1.0f / (p_hom.w + 0.0000001f);
    const float p_proj_x = p_hom.x * p_w;
    const float p_proj_y = p_hom.y * p_w;

    // computeCov3D (forward.cu:118-152)
    if (!kCovPrecomp) {
        compute_cov3d(sc, q, a.scale_modifier, cov3D);
        // the reference stores it for its backward; the backward here
        // recomputes it from the scale / rotation it reads anyway (bit-identical),
        // so the 24 B per Gaussian are written only on request (parity tests)
        if (a.store_cov3d) {
#pragma unroll
            for (int i = 0; i < 6; i++) g.cov3D[6 * idx + i] = cov3D[i];
        }
    }

    // computeCov2D (forward.cu:74-113)
    float3 t = transform_point_4x3(mx, my, mz, V);
    const float limx = 1.3f * a.tan_fovx;
    const float limy = 1.3f * a.tan_fovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const Mat3 J = mat3_cols(a.focal_x / t.z, 0.0f, -(a.focal_x * t.x) / (t.z * t.z), 0.0f, a.focal_y / t.z,
                             -(a.focal_y * t.y) / (t.z * t.z), 0, 0, 0);
    const float* v = V.m;
    const Mat3 Wm = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    const Mat3 T = mat3_mul(Wm, J);
    const Mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4],
                               cov3D[5]);
    Mat3 cov = mat3_mul(mat3_mul(mat3_transpose(T), mat3_transpose(Vrk)), T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    const float cx = cov.m[0][0], cy = cov.m[0][1], cz = cov.m[1][1];

    // EWA inverse + extent (forward.cu:219-237)
    const float det = (cx * cz - cy * cy);
    if (det == 0.0f) return;
    const float det_inv = 1.f / det;
    const float conic_x = cz * det_inv, conic_y = -cy * det_inv, conic_z = cx * det_inv;
    const float mid = 0.5f * (cx + cz);
    const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
    const float pix_x = ndc2pix(p_proj_x, a.W);
    const float pix_y = ndc2pix(p_proj_y, a.H);
    const uint32_t gx = (uint32_t)((a.W + a.block - 1) / a.block);
    const uint32_t gy = (uint32_t)((a.H + a.block - 1) / a.block);
    const int iradius = (int)my_radius;
    const Rect r = get_rect(pix_x, pix_y, iradius, a.block, a.block, gx, gy);
    const uint32_t area = (r.x1 - r.x0) * (r.y1 - r.y0);
    if (area == 0) return;

    float3 rgbv = make_float3(0.f, 0.f, 0.f);
    if (kHasSH) {
        // SH only for Gaussians that survive the cull (computeColorFromSH runs
        // after the rect test in the reference too, forward.cu:240-247)
        float shc[16][3];
        load_shc(shc);
        // computeColorFromSH: dir = normalize(mean - campos)
        float dx = mx - a.cam_pos[0], dy = my - a.cam_pos[1], dz = mz - a.cam_pos[2];
        const float len = sqrtf(dot3(dx, dy, dz, dx, dy, dz));
        dx = dx / len; dy = dy / len; dz = dz / len;
        uint8_t cbits;
        const float3 rgb = eval_sh_color(a.D, shc, dx, dy, dz, cbits);
        if (a.store_drgb) {  // the SH backward's d(rgb)/d(dir), from the coefficients already in registers
            float dx3[3], dy3[3], dz3[3];
            sh_ddir(a.D, shc, dx, dy, dz, dx3, dy3, dz3);
            // one 48-B row: three 16-B stores from one address (or into the
            // thread's LDS row, which its wave stores coalesced)
            float4* row = stage ? reinterpret_cast<float4*>(stage)
                                : reinterpret_cast<float4*>(g.drgb) + 3 * (size_t)idx;
            row[0] = make_float4(dx3[0], dx3[1], dx3[2], dy3[0]);
            row[1] = make_float4(dy3[1], dy3[2], dz3[0], dz3[1]);
            row[2] = make_float4(dz3[2], 0.f, 0.f, 0.f);
        }
        if (stage) {
            *reinterpret_cast<float4*>(stage + 12) = make_float4(rgb.x, rgb.y, rgb.z, 0.f);  // (one b128)
        } else {
            g.rgb[3 * idx + 0] = rgb.x;
            g.rgb[3 * idx + 1] = rgb.y;
            g.rgb[3 * idx + 2] = rgb.z;
        }
        rgbv = rgb;
        g.clamped[idx] = cbits;
    }
    g.depths[idx] = p_view.z;
    radii[idx] = iradius;
    if (radii_copy) g.radii[idx] = iradius;
    reinterpret_cast<float2*>(g.means2D)[idx] = make_float2(pix_x, pix_y);
    reinterpret_cast<float4*>(g.conic_opacity)[idx] = make_float4(conic_x, conic_y, conic_z, opacity);
    g.tiles_touched[idx] = area;
    if (a.block == 32) {
        // AMR: the blend record of this Gaussian as ONE 64-B row (GeomView::
        // amr_rows), so foveaStep 0's region-list pass (render.hip) gathers one
        // aligned sector per instance instead of three records: (x, y, r, g),
        // the log2(e)-scaled conic + opacity, (b, raw conic), zero pad.
        float r_, g_, b_;
        if (kHasSH) {
            r_ = rgbv.x; g_ = rgbv.y; b_ = rgbv.z;
        } else {
            r_ = a.colors_precomp[3 * idx]; g_ = a.colors_precomp[3 * idx + 1]; b_ = a.colors_precomp[3 * idx + 2];
        }
        float4* row = stage ? reinterpret_cast<float4*>(stage + 16)
                            : reinterpret_cast<float4*>(g.amr_rows + (size_t)16 * idx);
        const float4 co = make_float4(conic_x, conic_y, conic_z, opacity);
        row[0] = make_float4(pix_x, pix_y, r_, g_);
        row[1] = splat_coef(co);
        row[2] = make_float4(b_, conic_x, conic_y, conic_z);
        if (!stage) row[3] = make_float4(0.f, 0.f, 0.f, 0.f);
    }

    // Tile histogram with device atomics only when the tile grid is too large
    // for the LDS-privatised count_tiles kernel (binning.hip); wave-uniform.
    if (tile_count)
        for (uint32_t y = r.y0; y < r.y1; y++)
            for (uint32_t x = r.x0; x < r.x1; x++) atomicAdd(&tile_count[y * gx + x], 1u);
}

// One Gaussian: zero its counters, issue its loads, pp_gaussian.  stage: the
// thread's LDS row for the strided records (kStageOut) or nullptr.
template <bool kHasSH, bool kSH16, bool kCovPrecomp, bool kDma, bool kNtIn = false>
__device__ __forceinline__ void pp_thread(const PreprocessArgs& a, const GeomView& g, int* __restrict__ radii,
                                          uint32_t* __restrict__ tile_count, int idx, const float* sh_row,
                                          float* stage) {
    // AMR: the geometry buffer keeps its own copy of the radii (the progressive
    // steps return zero radii, their backward reads these); base: the caller's
    const bool radii_copy = a.block == 32 && radii != g.radii;
    radii[idx] = 0;
    if (radii_copy) g.radii[idx] = 0;
    g.tiles_touched[idx] = 0;

    // Every global load of this Gaussian is issued up front (one memory round
    // trip per thread); the math below then overlaps other waves' loads.
    // (kNtIn: non-temporal -- read once per pass, and the backward's re-read
    // comes after far more traffic than the caches hold)
    const float mx = ldg1<kNtIn>(a.means3D + 3 * idx + 0);
    const float my = ldg1<kNtIn>(a.means3D + 3 * idx + 1);
    const float mz = ldg1<kNtIn>(a.means3D + 3 * idx + 2);
    float sc[3] = {0.f, 0.f, 0.f};
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    float cov3D[6];
    if (kCovPrecomp) {
#pragma unroll
        for (int i = 0; i < 6; i++) cov3D[i] = a.cov3D_precomp[6 * idx + i];
    } else {
        sc[0] = ldg1<kNtIn>(a.scales + 3 * idx + 0);
        sc[1] = ldg1<kNtIn>(a.scales + 3 * idx + 1);
        sc[2] = ldg1<kNtIn>(a.scales + 3 * idx + 2);
        q = ldg4<kNtIn>(reinterpret_cast<const float4*>(a.rotations) + idx);
    }
    const float opacity = ldg1<kNtIn>(a.opacities + idx);
    const Mat4 V = load_mat4(a.viewmatrix);
    const Mat4 Pm = load_mat4(a.projmatrix);
    pp_gaussian<kHasSH, kCovPrecomp>(a, g, radii, tile_count, idx, radii_copy, mx, my, mz, sc, q, cov3D, opacity,
                                     V, Pm, [&](float (&shc)[16][3]) {
        if constexpr (kDma) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA rows have landed
            const int ncoef = min((a.D + 1) * (a.D + 1), a.M);
            // twelve b128 reads of the padded row (conflict-free, kShStride)
            // (the empty asm keeps each piece one 128-bit register tuple, so the
            // compiler does not split the reads into conflicting b32 / b64 ones)
            typedef float f4v __attribute__((ext_vector_type(4)));
            float v[48];
#pragma unroll
            for (int i = 0; i < 12; i++) {
                f4v t = reinterpret_cast<const f4v*>(sh_row)[i];
                asm volatile("" : "+v"(t));
                v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
            }
#pragma unroll
            for (int k = 0; k < 16; k++)
#pragma unroll
                for (int ch = 0; ch < 3; ch++) shc[k][ch] = k < ncoef ? v[3 * k + ch] : 0.f;
        } else {
            load_sh<kSH16>(a.D, a.M, a.shs + (size_t)idx * a.M * 3, shc);
        }
    }, stage);
}

// kDma (SH16, the default): the SH rows through LDS-DMA, and the strided
// records staged -- a visible Gaussian's d(rgb)/d(dir) row and rgb go into its
// thread's LDS row (free once its SH coefficients are in registers), and each
// wave then stores its 64 records as wave-contiguous 16-B pieces instead of
// per-thread stores at a 48-B / 12-B stride (one store instruction covers
// whole lines, not a third of each): config 4 0.503 -> 0.441 ms, config 3
// 0.084 -> 0.077, config 2 equal (profiles/r04f_ab_pp*.log).  Rows of culled
// Gaussians carry stale words, as their never-read records may.  Cache hints
// (non-temporal: read or written once per pass, and re-read only after more
// traffic than the caches hold): the SH rows' LDS-DMA loads (0.0645 -> 0.0578
// ms at config 2, 0.378 -> 0.356 at config 4, profiles/r04z6_ab_pp*.log), the
// drgb rows' stores (config-4 fwd + bwd step 2.544 -> 2.508 ms,
// r04z6_ab_ppstep4.log), the geometry loads (0.394 -> 0.380 ms at config 4,
// r04z7_ab_pp*.log).  Measured and removed: per-thread SH loads with LDS-DMA
// but unstaged records, a persistent pipelined form (0.537 vs 0.502 ms at
// config 4, profiles/r04e_ab_pp*.log).
template <bool kHasSH, bool kSH16, bool kCovPrecomp, bool kDma = false>
__global__ void __launch_bounds__(kPpThreads) preprocess_kernel(PreprocessArgs a, GeomView g, int* __restrict__ radii,
                                                                uint32_t* __restrict__ tile_count) {
    static_assert(!kDma || (kHasSH && kSH16), "LDS-DMA stages 16-coefficient SH rows");
    constexpr bool kStageOut = kDma, kNtIn = kDma;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    __shared__ __attribute__((aligned(16))) float s_sh[kDma ? kPpThreads * kShStride : 1];
    if constexpr (kDma) {
        // wave w: rows [64 w, 64 w + 64) of the block; lane l writes LDS piece
        // p = l + 64 i = (row p / 13, 16-B piece p % 13 of it)
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const size_t row0 = (size_t)blockIdx.x * kPpThreads + 64 * w;
        const float* src = a.shs + row0 * 48;
        float* dst = s_sh + 64 * kShStride * w;
        constexpr int kPieces = kShStride / 4;  // 13
#pragma unroll
        for (int i = 0; i < kPieces; i++) {
            const int p = 64 * i + lane, r = p / kPieces, j = p - kPieces * r;
            if (j < 12 && row0 + (size_t)r < (size_t)a.P)
                __builtin_amdgcn_global_load_lds(src + 48 * r + 4 * j, dst + 256 * i, 16, 0, 2);  // (nt)
        }
    }
    for (int i = idx; i < a.zero_n; i += (int)(gridDim.x * blockDim.x)) a.zero_words[i] = 0u;
    // whether the backward may take d(rgb)/d(dir) from g.drgb (every visible
    // Gaussian's row is written below)
    if (idx == 0) g.hdr[kHdrDrgb] = (kHasSH && a.store_drgb) ? 1u : 0u;
    float* row = s_sh + (kDma ? kShStride * threadIdx.x : 0);
    if constexpr (kStageOut) {
        // every lane of a wave takes part in its coalesced record stores below
        const int wrow0 = (int)(blockIdx.x * kPpThreads) + (int)(threadIdx.x & ~63u);
        if (wrow0 >= a.P) return;  // wave-uniform
        if (idx < a.P) pp_thread<kHasSH, kSH16, kCovPrecomp, kDma, kNtIn>(a, g, radii, tile_count, idx, row, row);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int lane = threadIdx.x & 63;
        const float* wl = s_sh + kShStride * (threadIdx.x & ~63u);
        const int nrow = min(64, a.P - wrow0);
        if (a.store_drgb) {  // 64 rows x three 16-B pieces
            float4* out = reinterpret_cast<float4*>(g.drgb) + 3 * (size_t)wrow0;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const int c = lane + 64 * i;
                if (c < 3 * nrow) {
                    const float4 v = *reinterpret_cast<const float4*>(wl + kShStride * (c / 3) + 4 * (c % 3));
                    typedef float f4v __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(out + c));
                }
            }
        }
        if (a.block == 32) {  // AMR blend rows: 64 x 64 B (three staged float4s + a zero pad each)
            float4* out = reinterpret_cast<float4*>(g.amr_rows + (size_t)16 * wrow0);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int c = lane + 64 * i;
                if (c < 4 * nrow)
                    out[c] = (c & 3) == 3 ? make_float4(0.f, 0.f, 0.f, 0.f)
                                          : *reinterpret_cast<const float4*>(wl + kShStride * (c >> 2) + 16 + 4 * (c & 3));
            }
        }
        // 64 x 3 rgb floats = 48 pieces of 4
        const int nf = 3 * nrow;
        if (4 * lane < nf) {
            float v4[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int f = min(4 * lane + e, nf - 1);
                v4[e] = wl[kShStride * (f / 3) + 12 + f % 3];
            }
            float* out = g.rgb + 3 * (size_t)wrow0 + 4 * lane;
            if (4 * lane + 4 <= nf) {
                *reinterpret_cast<float4*>(out) = make_float4(v4[0], v4[1], v4[2], v4[3]);
            } else {
#pragma unroll
                for (int e = 0; e < 3; e++)
                    if (4 * lane + e < nf) out[e] = v4[e];
            }
        }
        return;
    }
    if (idx >= a.P) return;
    pp_thread<kHasSH, kSH16, kCovPrecomp, kDma>(a, g, radii, tile_count, idx, row, nullptr);
}

template <bool A, bool B, bool C>
static void launch_pp(const PreprocessArgs& a, const GeomView& g, int* radii, uint32_t* tile_count, hipStream_t s) {
    const int blocks = (a.P + kPpThreads - 1) / kPpThreads;
    hipLaunchKernelGGL((preprocess_kernel<A, B, C, A && B>), dim3(blocks), dim3(kPpThreads), 0, s, a, g, radii,
                       tile_count);
}

void launch_preprocess(const PreprocessArgs& a, const GeomView& g, int* radii, uint32_t* tile_count,
                       hipStream_t s) {
    if (a.P == 0) return;
    const bool has_sh = a.colors_precomp == nullptr;
    const bool sh16 = has_sh && a.M == 16;
    const bool covp = a.cov3D_precomp != nullptr;
    if (has_sh) {
        if (sh16) {
            if (covp) launch_pp<true, true, true>(a, g, radii, tile_count, s);
            else launch_pp<true, true, false>(a, g, radii, tile_count, s);
        } else {
            if (covp) launch_pp<true, false, true>(a, g, radii, tile_count, s);
            else launch_pp<true, false, false>(a, g, radii, tile_count, s);
        }
    } else {
        if (covp) launch_pp<false, false, true>(a, g, radii, tile_count, s);
        else launch_pp<false, false, false>(a, g, radii, tile_count, s);
    }
}

// base/cr/rasterizer_impl.cu:54-66 (checkFrustum)
__global__ void __launch_bounds__(256) mark_visible_kernel(int P, const float* __restrict__ means3D,
                                                           const float* __restrict__ viewmatrix,
                                                           bool* __restrict__ present) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const Mat4 V = load_mat4(viewmatrix);
    const float3 pv = transform_point_4x3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2], V);
    present[idx] = !(pv.z <= 0.2f);
}

void launch_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                         bool* present, hipStream_t s) {
    (void)projmatrix;  // p_hom is computed but unused by the reference test
    if (P == 0) return;
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, viewmatrix,
                       present);
}

}  // namespace gsamd
