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

namespace gsamd {

constexpr int kLvlThreads = 1024;

// k-th smallest (0-based) of v[0..n) -- MSD radix select, one workgroup.
// Counts are read straight from ranges (count = y - x) so no global value is
// read back after being written inside this launch.
__device__ uint32_t block_select_kth(const uint32_t* __restrict__ ranges, int n, uint32_t k, uint32_t* hist,
                                     uint32_t* shared_word) {
    const int tid = threadIdx.x;
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
        if (tid == 0) {
            uint32_t acc = 0, dig = 255;
            for (int b = 0; b < 256; b++) {
                if (acc + hist[b] > k) {
                    dig = (uint32_t)b;
                    break;
                }
                acc += hist[b];
            }
            k -= acc;
            shared_word[0] = dig;
            shared_word[1] = k;
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

__global__ void __launch_bounds__(kLvlThreads) amr_levels_kernel(int T, const uint32_t* __restrict__ ranges,
                                                                 uint32_t* __restrict__ n_inter,
                                                                 uint32_t* __restrict__ pv,
                                                                 uint32_t* __restrict__ levels) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t word[2];
    __shared__ uint32_t s_pv[3];
    const int tid = threadIdx.x;
    // calculateIntersections (amr/cr/rasterizer_impl.cu:181-188)
    for (int t = tid; t < T; t += kLvlThreads) n_inter[t] = ranges[2 * t + 1] - ranges[2 * t];
    const float percentiles[3] = {0.25f, 0.5f, 0.9f};
    for (int i = 0; i < 3; i++) {
        const uint32_t k = (uint32_t)(int)(percentiles[i] * (float)T);  // float32 index, :630
        const uint32_t val = T > 0 ? block_select_kth(ranges, T, k, hist, word) : 0u;
        if (tid == 0) s_pv[i] = val;
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

void launch_amr_levels(int T, const ImageView& img, hipStream_t s) {
    if (T == 0) return;
    hipLaunchKernelGGL(amr_levels_kernel, dim3(1), dim3(kLvlThreads), 0, s, T, img.ranges, img.tile_count, img.pv,
                       img.levels);
}

// amr/cr/rasterizer_impl.cu:208-243 (setFoveaAMRLevelsKernel)
__global__ void __launch_bounds__(256) fovea_levels_kernel(int step, int T, uint32_t* __restrict__ last,
                                                           uint32_t* __restrict__ current,
                                                           const uint32_t* __restrict__ levels) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
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
        default:
            last[t] = 0;
            current[t] = L;
            break;
    }
}

void launch_fovea_levels(int step, int T, const ImageView& img, hipStream_t s) {
    if (T == 0) return;
    hipLaunchKernelGGL(fovea_levels_kernel, dim3((T + 255) / 256), dim3(256), 0, s, step, T, img.levels_last,
                       img.levels_current, img.levels);
}

}  // namespace gsamd
