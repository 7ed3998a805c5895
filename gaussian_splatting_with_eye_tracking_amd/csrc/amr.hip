// amr.hip -- per-tile AMR level assignment on gfx950.
//
// Reference (amr/cr/rasterizer_impl.cu:590-656): calculateIntersections,
// cub::DeviceRadixSort::SortKeys of the T counts into a cudaMalloc'd temp,
// three blocking D2H copies of sorted[(int)(p*T)] for p in {0.25f,0.5f,0.9f},
// then setAMRLevelsKernel with a *host* array passed as a device pointer
// (amr/cr/rasterizer_impl.cu:610,644 -- only valid under HMM/ATS).
//
// Here one workgroup does all of it on device: the n_intersections are the
// tile counts the binning already holds (ranges[t].y - ranges[t].x ==
// tile_count[t]), each percentile is found by an MSD radix *select* over the
// four bytes of the counts (an order statistic needs no full sort), and the
// levels are written in the same launch.  No host synchronisation, no
// allocation, no host pointer on the device.
#include "gs_device.cuh"
#include "gs_kernels.h"

#include <algorithm>

namespace gsamd {

constexpr int kLvlThreads = 1024;
constexpr int kLvlSortMax = 2048;  // tile grids up to this size sort their counts in LDS
// Counts < 2^16 take the two-pass histogram select (select3_u16: 19.2 ->
// 13.5 us per frame at config 3, profiles/r04i_ab_lvl.log); a grid with a
// larger count sorts its counts in LDS (<= kLvlSortMax tiles) or runs the
// 4-pass radix select.

// k-th smallest (0-based) of v[0..n) -- MSD radix select, one workgroup.
// Counts are read straight from ranges (count = y - x) so no global value is
// read back after being written inside this launch.  Each 8-bit digit pass:
// LDS histogram of the candidates, then the 256 bins are scanned by the
// first four waves (wave prefix sums + a 4-entry carry) and the one bin whose
// [start, start + count) holds k names the digit -- no serial 256-step loop.
__device__ uint32_t block_select_kth(const uint32_t* __restrict__ ranges, int n, uint32_t k, uint32_t* hist,
                                     uint32_t* shared_word) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ uint32_t s_carry[4];
    uint32_t prefix = 0, mask = 0;
    for (int d = 3; d >= 0; d--) {
        for (int i = tid; i < 256; i += kLvlThreads) hist[i] = 0;
        __syncthreads();
        const int sh = 8 * d;
        for (int i = tid; i < n; i += kLvlThreads) {
            const uint32_t x = ranges[2 * i + 1] - ranges[2 * i];
            if ((x & mask) == prefix) atomicAdd(&hist[(x >> sh) & 0xFF], 1u);
        }
        __syncthreads();
        uint32_t h = 0, inc = 0;
        if (tid < 256) {
            h = hist[tid];
            inc = h;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t t = (uint32_t)__shfl_up((int)inc, off, 64);
                if (lane >= off) inc += t;
            }
            if (lane == 63) s_carry[wave] = inc;
        }
        __syncthreads();
        if (tid < 256) {
            uint32_t start = inc - h;
            for (int w = 0; w < wave; w++) start += s_carry[w];
            if (h > 0 && start <= k && k < start + h) {  // exactly one bin
                shared_word[0] = (uint32_t)tid;
                shared_word[1] = k - start;
            }
        }
        __syncthreads();
        const uint32_t dig = shared_word[0];
        k = shared_word[1];
        prefix |= dig << sh;
        mask |= 0xFFu << sh;
        __syncthreads();
    }
    return prefix;
}

// The three order statistics k[0..2] of the T counts when every count is
// below 65536: two 8-bit digit passes (high byte, then the low byte of the
// values in each statistic's high bin), all three statistics in the same
// passes -- ~8 barriers instead of the bitonic sort's 66.  hist: 768 words.
__device__ void select3_u16(const uint32_t* __restrict__ ranges, int T, const uint32_t (&k)[3], uint32_t* hist,
                            uint32_t* word, uint32_t (&out)[3]) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ uint32_t s_carry[12];
    for (int i = tid; i < 256; i += kLvlThreads) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < T; i += kLvlThreads) atomicAdd(&hist[(ranges[2 * i + 1] - ranges[2 * i]) >> 8], 1u);
    __syncthreads();
    uint32_t h = 0, inc = 0;
    if (tid < 256) {
        h = hist[tid];
        inc = h;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)inc, off, 64);
            if (lane >= off) inc += t;
        }
        if (lane == 63) s_carry[wave] = inc;
    }
    __syncthreads();
    if (tid < 256) {
        uint32_t start = inc - h;
        for (int w = 0; w < wave; w++) start += s_carry[w];
#pragma unroll
        for (int q = 0; q < 3; q++)
            if (h > 0 && start <= k[q] && k[q] < start + h) {  // exactly one bin per statistic
                word[2 * q] = (uint32_t)tid;
                word[2 * q + 1] = k[q] - start;
            }
    }
    __syncthreads();
    uint32_t b[3], r[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
        b[q] = word[2 * q];
        r[q] = word[2 * q + 1];
    }
    for (int i = tid; i < 768; i += kLvlThreads) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < T; i += kLvlThreads) {
        const uint32_t x = ranges[2 * i + 1] - ranges[2 * i];
#pragma unroll
        for (int q = 0; q < 3; q++)
            if ((x >> 8) == b[q]) atomicAdd(&hist[256 * q + (x & 255u)], 1u);
    }
    __syncthreads();
    h = 0;
    inc = 0;
    if (tid < 768) {
        h = hist[tid];
        inc = h;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)inc, off, 64);
            if (lane >= off) inc += t;
        }
        if (lane == 63) s_carry[wave] = inc;
    }
    __syncthreads();
    if (tid < 768) {
        const int q = tid >> 8;
        uint32_t start = inc - h;
        for (int w = 4 * q; w < wave; w++) start += s_carry[w];
        if (h > 0 && start <= r[q] && r[q] < start + h) word[q] = (b[q] << 8) | (uint32_t)(tid & 255);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; q++) out[q] = word[q];
}

__global__ void __launch_bounds__(kLvlThreads) amr_levels_kernel(int T, const uint32_t* __restrict__ ranges,
                                                                 uint32_t* __restrict__ n_inter,
                                                                 uint32_t* __restrict__ pv,
                                                                 uint32_t* __restrict__ levels,
                                                                 float4* __restrict__ zero4, int zero_n4) {
    // blocks >= 1 (if any): foveaStep 0's zero image, grid-stride float4
    // stores on the other CUs while block 0 -- one CU -- computes the levels
    // (one launch instead of the levels kernel and a separate fill)
    if (blockIdx.x > 0) {
        for (int i = (int)((blockIdx.x - 1) * kLvlThreads + threadIdx.x); i < zero_n4;
             i += (int)((gridDim.x - 1) * kLvlThreads))
            zero4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    __shared__ uint32_t hist[768];
    __shared__ uint32_t word[6];
    __shared__ uint32_t s_pv[3];
    const int tid = threadIdx.x;
    // calculateIntersections (amr/cr/rasterizer_impl.cu:181-188)
    bool big = false;
    for (int t = tid; t < T; t += kLvlThreads) {
        const uint32_t x = ranges[2 * t + 1] - ranges[2 * t];
        n_inter[t] = x;
        big |= x >= 65536u;
    }
    const float percentiles[3] = {0.25f, 0.5f, 0.9f};
    if (!__syncthreads_or(big)) {
        // every count < 2^16: two digit passes for all three statistics
        const uint32_t kq[3] = {(uint32_t)(int)(percentiles[0] * (float)T), (uint32_t)(int)(percentiles[1] * (float)T),
                                (uint32_t)(int)(percentiles[2] * (float)T)};  // float32 index, :630
        uint32_t v[3];
        select3_u16(ranges, T, kq, hist, word, v);
        if (tid < 3) s_pv[tid] = v[tid];
    } else if (T <= kLvlSortMax) {
        // small grids (1080p: 2040 tiles): one LDS bitonic sort of the counts
        // (padded with UINT32_MAX), then the three order statistics directly --
        // 66 barrier-separated stages instead of 12 radix-select passes
        __shared__ uint32_t s_sorted[kLvlSortMax];
        for (int i = tid; i < kLvlSortMax; i += kLvlThreads)
            s_sorted[i] = i < T ? ranges[2 * i + 1] - ranges[2 * i] : 0xFFFFFFFFu;
        __syncthreads();
        for (int kk = 2; kk <= kLvlSortMax; kk <<= 1) {
            for (int j = kk >> 1; j > 0; j >>= 1) {
                for (int p = tid; p < kLvlSortMax / 2; p += kLvlThreads) {
                    const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1));
                    const bool up = (i & kk) == 0;
                    const uint32_t a = s_sorted[i], b = s_sorted[i + j];
                    if ((a > b) == up) {
                        s_sorted[i] = b;
                        s_sorted[i + j] = a;
                    }
                }
                __syncthreads();
            }
        }
        if (tid < 3) s_pv[tid] = s_sorted[(int)(percentiles[tid] * (float)T)];  // float32 index, :630
    } else {
        for (int i = 0; i < 3; i++) {
            const uint32_t k = (uint32_t)(int)(percentiles[i] * (float)T);  // float32 index, :630
            const uint32_t val = block_select_kth(ranges, T, k, hist, word);
            if (tid == 0) s_pv[i] = val;
        }
    }
    __syncthreads();
    if (tid < 3) pv[tid] = s_pv[tid];
    const uint32_t p0 = s_pv[0], p1 = s_pv[1], p2 = s_pv[2];
    // setAMRLevelsKernel (amr/cr/rasterizer_impl.cu:190-205)
    for (int t = tid; t < T; t += kLvlThreads) {
        const uint32_t x = ranges[2 * t + 1] - ranges[2 * t];
        levels[t] = x <= p0 ? 1u : x <= p1 ? 2u : x <= p2 ? 3u : 4u;
    }
}

void launch_amr_levels(int T, const ImageView& img, hipStream_t s, float* zero_image, size_t zero_floats) {
    if (T == 0) return;
    const int n4 = (zero_image && zero_floats % 4 == 0 && zero_floats / 4 <= (size_t)INT32_MAX) ? (int)(zero_floats / 4) : 0;
    if (zero_image && n4 == 0 && zero_floats > 0)  // (an unaligned size: the plain fill)
        (void)hipMemsetAsync(zero_image, 0, sizeof(float) * zero_floats, s);
    const int zb = n4 > 0 ? std::min(512, (n4 + kLvlThreads * 8 - 1) / (kLvlThreads * 8)) : 0;
    hipLaunchKernelGGL(amr_levels_kernel, dim3(1 + zb), dim3(kLvlThreads), 0, s, T, img.ranges, img.tile_count, img.pv,
                       img.levels, reinterpret_cast<float4*>(zero_image), n4);
}

// amr/cr/rasterizer_impl.cu:208-243 (setFoveaAMRLevelsKernel)
// (+ the zero radii the progressive steps return, amr/rasterize_points.cu:
// the caller's radii need no separate fill: threads t < P write radii[t] = 0)
__global__ void __launch_bounds__(256) fovea_levels_kernel(int step, int T, uint32_t* __restrict__ last,
                                                           uint32_t* __restrict__ current,
                                                           const uint32_t* __restrict__ levels, int P,
                                                           int* __restrict__ zero_radii) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (zero_radii && t < P) zero_radii[t] = 0;
    if (t >= T) return;
    const uint32_t L = levels[t];
    switch (step) {
        case 0:
            break;
        case 1:
            last[t] = 0;
            current[t] = (L >= 1) ? 1u : 0u;
            break;
        case 2:
        case 3:
        case 4: {
            const uint32_t prev = current[t];
            last[t] = prev;
            current[t] = (L >= (uint32_t)step) ? (uint32_t)step : prev;
            break;
        }
        case kAmrStateAfter + 1:
        case kAmrStateAfter + 2:
        case kAmrStateAfter + 3:
        case kAmrStateAfter + 4: {
            // from the state steps 1..4 leave (current = min(L0, 4), L0 the
            // levels those steps saw) back to the one steps 1..j leave:
            // current = min(L0, j), last = min(L0, j - 1) (by induction over
            // the cases above) -- from current, not from `levels`, which a
            // fovea-level change may have rewritten since
            const uint32_t j = (uint32_t)(step - kAmrStateAfter), c4 = current[t];
            last[t] = min(c4, j - 1);
            current[t] = min(c4, j);
            break;
        }
        default:
            last[t] = 0;
            current[t] = L;
            break;
    }
}

void launch_fovea_levels(int step, int T, const ImageView& img, hipStream_t s, int P, int* zero_radii) {
    const int n = zero_radii ? std::max(T, P) : T;
    if (n <= 0) return;
    hipLaunchKernelGGL(fovea_levels_kernel, dim3((n + 255) / 256), dim3(256), 0, s, step, T, img.levels_last,
                       img.levels_current, img.levels, P, zero_radii);
}

// Backward of render_once's interpolation (amr/cr/forward.cu:520-648, the
// foveaStep < 0 branch): a pixel whose round exceeds its tile's level is a
// copy of its 2x2 cell's (0, 0) (levels 1, 2) or (1, 1) (level 3) pixel, so
// its cotangent is added to that source's.  One thread per cell, copies
// summed in round order; rendered pixels keep their own cotangent, copies
// get 0 (the blend backward reads only rendered pixels).
__global__ void __launch_bounds__(256) amr_interp_fold_kernel(int W, int H, int tgx, const uint32_t* __restrict__ levels,
                                                              const float* __restrict__ g_in,
                                                              float* __restrict__ g_out) {
    const int cw = (W + 1) / 2, ch = (H + 1) / 2;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= cw * ch) return;
    const int cx = c % cw, cy = c / cw;
    const int x0 = 2 * cx, y0 = 2 * cy;
    const uint32_t L = min(levels[(y0 / 32) * tgx + x0 / 32], 4u);
    const int o = (L == 3 || L == 4) ? 1 : 0;
    const int sxp = x0 + o, syp = y0 + o;
    const bool src_in = sxp < W && syp < H;
    const size_t plane = (size_t)W * H;
    // the cell's pixels in round order 1..4: (0,0), (1,1), (1,0), (0,1)
    const int dxs[4] = {0, 1, 1, 0}, dys[4] = {0, 1, 0, 1};
    for (int ch3 = 0; ch3 < 3; ch3++) {
        float fold = 0.f;
        for (int r = 0; r < 4; r++) {
            const int px = x0 + dxs[r], py = y0 + dys[r];
            if (px >= W || py >= H) continue;
            const size_t pid = (size_t)py * W + px;
            if ((uint32_t)(r + 1) <= L) {
                g_out[ch3 * plane + pid] = g_in[ch3 * plane + pid];
            } else {
                g_out[ch3 * plane + pid] = 0.f;
                if (src_in) fold += g_in[ch3 * plane + pid];
            }
        }
        if (src_in && L < 4) g_out[ch3 * plane + (size_t)syp * W + sxp] += fold;
    }
}

void launch_amr_interp_fold(int W, int H, const ImageView& img, const float* g_in, float* g_out, hipStream_t s) {
    const int cells = ((W + 1) / 2) * ((H + 1) / 2);
    if (cells == 0) return;
    hipLaunchKernelGGL(amr_interp_fold_kernel, dim3((cells + 255) / 256), dim3(256), 0, s, W, H, (W + 31) / 32,
                       img.levels, g_in, g_out);
}

// Fovea-driven levels (an extension beyond parity).
// The reference defines per-step fovea centres and radii
// (gaussian_renderer_amr/__init__.py:98-106: centre = image centre, radii
// W/2, W/4, W/8, W/16) but never passes them to the rasterizer, and leaves
// "if outside the current fovea, set to same as last step" as a TODO
// (:244).  This kernel implements that TODO on the step-0 levels: fovea k
// (k = 1..nf) is the disc (centre_k, radius_k); a tile is inside it when the
// disc meets the tile's pixel rectangle [x0, x1] x [y0, y1] (the squared
// distance from the centre to the rectangle <= radius^2).  F(t) = the
// largest k such that the tile is inside foveae 1..k (0 if not inside the
// first), floored at min_level; then
//   clamp   (replace = 0): L'(t) = min(L(t), max(F(t), min_level))
//   replace (replace = 1): L'(t) = max(F(t), min_level)
// so the steps k >= 1 that follow (setFoveaAMRLevelsKernel: current = L >= k
// ? k : last) keep a tile outside fovea k at its last round.  Integer
// output; float math only in the rectangle distance (no contraction).
struct FoveaDiscs {
    float cx[4], cy[4], r2[4];
};

__global__ void __launch_bounds__(256) fovea_override_kernel(int T, int grid_x, int W, int H, int tile, FoveaDiscs d,
                                                             int nf, uint32_t min_level, int replace,
                                                             uint32_t* __restrict__ levels) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const int tx = t % grid_x, ty = t / grid_x;
    const float x0 = (float)(tx * tile), y0 = (float)(ty * tile);
    const float x1 = (float)min(tx * tile + tile, W) - 1.0f, y1 = (float)min(ty * tile + tile, H) - 1.0f;
    uint32_t F = 0;
    for (int k = 0; k < nf; k++) {
        const float dx = fmaxf(fmaxf(x0 - d.cx[k], d.cx[k] - x1), 0.0f);
        const float dy = fmaxf(fmaxf(y0 - d.cy[k], d.cy[k] - y1), 0.0f);
        if (dx * dx + dy * dy > d.r2[k]) break;
        F = (uint32_t)(k + 1);
    }
    const uint32_t f = F > min_level ? F : min_level;
    const uint32_t L = levels[t];
    levels[t] = replace ? f : (L < f ? L : f);
}

void launch_fovea_override(int W, int H, const ImageView& img, int nf, const float* cx, const float* cy,
                           const float* radius, int min_level, int replace, hipStream_t s) {
    const int tile = 32, grid_x = (W + tile - 1) / tile, T = grid_x * ((H + tile - 1) / tile);
    if (T == 0) return;
    FoveaDiscs d{};
    for (int k = 0; k < nf; k++) {
        d.cx[k] = cx[k];
        d.cy[k] = cy[k];
        d.r2[k] = radius[k] * radius[k];
    }
    hipLaunchKernelGGL(fovea_override_kernel, dim3((T + 255) / 256), dim3(256), 0, s, T, grid_x, W, H, tile, d, nf,
                       (uint32_t)min_level, replace, img.levels);
}

}  // namespace gsamd
