// knn.hip -- simple-knn (distCUDA2) on gfx950, plus the stable LSD radix sort
// it needs.
//
// Reference: knn/simple_knn.cu:185-221 (SimpleKNN::knn) and its kernels
// coord2Morton (:63-70), boxMinMax (:78-117), boxMeanDist (:147-183).  The
// reference does two cub::DeviceReduce passes with two blocking D2H copies of
// the bounding box, thrust vectors and a CUB radix sort.  Here the bounding
// box stays on device (the Morton kernel reads it from memory), so the whole
// call is one asynchronous chain on the stream.  The {0,0,0} initial value of
// both reductions (a reference quirk, :189) is kept: minn = min(0, .),
// maxx = max(0, .).  Results are bit-identical to the oracle: every float op
// is evaluated in the reference order without contraction.
#include <float.h>

#include "gs_device.cuh"
#include "gs_kernels.h"

namespace gsamd {

// ================================================================ radix sort
constexpr int kRsThreads = 256;
constexpr int kRsItems = 16;
constexpr int kRsTile = kRsThreads * kRsItems;  // 4096 items per block

__global__ void __launch_bounds__(kRsThreads) rs_hist_kernel(int n, const uint32_t* __restrict__ keys, int shift,
                                                             int nblocks, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x;
    h[tid] = 0;
    __syncthreads();
    const int base = blockIdx.x * kRsTile;
    for (int r = 0; r < kRsItems; r++) {
        const int i = base + r * kRsThreads + tid;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 0xFF], 1u);
    }
    __syncthreads();
    hist[tid * nblocks + blockIdx.x] = h[tid];  // digit-major
}

// Exclusive scan of m entries in one workgroup of 1024 threads.
__global__ void __launch_bounds__(1024) rs_scan_kernel(int m, uint32_t* __restrict__ data) {
    __shared__ uint32_t sums[1024];
    const int tid = threadIdx.x;
    const int per = (m + 1023) / 1024;
    const int beg = min(m, tid * per), end = min(m, beg + per);
    uint32_t s = 0;
    for (int i = beg; i < end; i++) s += data[i];
    sums[tid] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const uint32_t v = tid >= off ? sums[tid - off] : 0u;
        __syncthreads();
        sums[tid] += v;
        __syncthreads();
    }
    uint32_t run = sums[tid] - s;
    for (int i = beg; i < end; i++) {
        const uint32_t c = data[i];
        data[i] = run;
        run += c;
    }
}

// Stable scatter: items of a block are ranked in striped order
// (round r, wave w, lane l) == index order base + r*256 + tid.
__global__ void __launch_bounds__(kRsThreads) rs_scatter_kernel(int n, const uint32_t* __restrict__ keys_in,
                                                                const uint32_t* __restrict__ vals_in,
                                                                uint32_t* __restrict__ keys_out,
                                                                uint32_t* __restrict__ vals_out, int shift,
                                                                int nblocks, const uint32_t* __restrict__ offsets) {
    __shared__ uint32_t s_base[256];
    __shared__ uint32_t s_wcnt[4][256];
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    s_base[tid] = offsets[tid * nblocks + blockIdx.x];
    const int base = blockIdx.x * kRsTile;
    const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int r = 0; r < kRsItems; r++) {
        for (int w = 0; w < 4; w++) s_wcnt[w][tid] = 0;
        __syncthreads();
        const int i = base + r * kRsThreads + tid;
        const bool valid = i < n;
        const uint32_t key = valid ? keys_in[i] : 0u;
        const uint32_t dig = (key >> shift) & 0xFF;
        unsigned long long match = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const unsigned long long m = __ballot((dig >> b) & 1);
            match &= ((dig >> b) & 1) ? m : ~m;
        }
        const uint32_t rank_in_wave = (uint32_t)__popcll(match & lt_mask);
        if (valid && rank_in_wave == 0) s_wcnt[wave][dig] = (uint32_t)__popcll(match);
        __syncthreads();
        {  // per digit: exclusive prefix across the 4 waves, advance the running base
            const uint32_t c0 = s_wcnt[0][tid], c1 = s_wcnt[1][tid], c2 = s_wcnt[2][tid], c3 = s_wcnt[3][tid];
            const uint32_t b0 = s_base[tid];
            s_wcnt[0][tid] = b0;
            s_wcnt[1][tid] = b0 + c0;
            s_wcnt[2][tid] = b0 + c0 + c1;
            s_wcnt[3][tid] = b0 + c0 + c1 + c2;
            s_base[tid] = b0 + c0 + c1 + c2 + c3;
        }
        __syncthreads();
        if (valid) {
            const uint32_t pos = s_wcnt[wave][dig] + rank_in_wave;
            keys_out[pos] = key;
            vals_out[pos] = vals_in[i];
        }
        __syncthreads();
    }
}

size_t radix_sort_u32_workspace(int n) {
    const int nblocks = (n + kRsTile - 1) / kRsTile;
    return align_up(sizeof(uint32_t) * (size_t)n) * 2 + align_up(sizeof(uint32_t) * 256 * (size_t)max(nblocks, 1));
}

void radix_sort_pairs_u32(int n, const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in,
                          uint32_t* vals_out, int end_bit, char* workspace, hipStream_t s) {
    if (n <= 0) return;
    const int nblocks = (n + kRsTile - 1) / kRsTile;
    uint32_t* kalt = reinterpret_cast<uint32_t*>(workspace);
    uint32_t* valt = reinterpret_cast<uint32_t*>(workspace + align_up(sizeof(uint32_t) * (size_t)n));
    uint32_t* hist = reinterpret_cast<uint32_t*>(workspace + 2 * align_up(sizeof(uint32_t) * (size_t)n));
    const int passes = (end_bit + 7) / 8;
    // Ping-pong so that the last pass lands in *_out.
    const uint32_t* ks = keys_in;
    const uint32_t* vs = vals_in;
    for (int p = 0; p < passes; p++) {
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        uint32_t* kd = to_out ? keys_out : kalt;
        uint32_t* vd = to_out ? vals_out : valt;
        hipLaunchKernelGGL(rs_hist_kernel, dim3(nblocks), dim3(kRsThreads), 0, s, n, ks, 8 * p, nblocks, hist);
        hipLaunchKernelGGL(rs_scan_kernel, dim3(1), dim3(1024), 0, s, 256 * nblocks, hist);
        hipLaunchKernelGGL(rs_scatter_kernel, dim3(nblocks), dim3(kRsThreads), 0, s, n, ks, vs, kd, vd, 8 * p,
                           nblocks, hist);
        ks = kd;
        vs = vd;
    }
    if (passes == 0) {
        hipMemcpyAsync(keys_out, keys_in, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, s);
        hipMemcpyAsync(vals_out, vals_in, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, s);
    }
}

// ======================================================================= knn
constexpr int kBox = 1024;

// knn/simple_knn.cu:45-52
__device__ __forceinline__ uint32_t prep_morton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}

// float -> uint32 with cvt.rzi.u32.f32 semantics (NaN -> 0, saturating).
__device__ __forceinline__ uint32_t f2u_sat(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

// Bounding box: per-block partials, then one block finishes with init {0,0,0}.
__global__ void __launch_bounds__(256) knn_bbox_partial(int P, const float* __restrict__ pts, float* __restrict__ part) {
    __shared__ float s[6][256];
    const int tid = threadIdx.x;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * 256 + tid; i < P; i += gridDim.x * 256)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            mn[k] = fminf(mn[k], pts[3 * i + k]);
            mx[k] = fmaxf(mx[k], pts[3 * i + k]);
        }
#pragma unroll
    for (int k = 0; k < 3; k++) {
        s[k][tid] = mn[k];
        s[3 + k][tid] = mx[k];
    }
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off)
#pragma unroll
            for (int k = 0; k < 3; k++) {
                s[k][tid] = fminf(s[k][tid], s[k][tid + off]);
                s[3 + k][tid] = fmaxf(s[3 + k][tid], s[3 + k][tid + off]);
            }
        __syncthreads();
    }
    if (tid < 6) part[6 * blockIdx.x + tid] = s[tid][0];
}

__global__ void __launch_bounds__(256) knn_bbox_final(int nparts, const float* __restrict__ part, float* __restrict__ bbox) {
    if (threadIdx.x != 0) return;
    float mn[3] = {0.f, 0.f, 0.f}, mx[3] = {0.f, 0.f, 0.f};  // init {0,0,0} (simple_knn.cu:189)
    for (int b = 0; b < nparts; b++)
        for (int k = 0; k < 3; k++) {
            mn[k] = fminf(mn[k], part[6 * b + k]);
            mx[k] = fmaxf(mx[k], part[6 * b + 3 + k]);
        }
    for (int k = 0; k < 3; k++) {
        bbox[k] = mn[k];
        bbox[3 + k] = mx[k];
    }
}

// knn/simple_knn.cu:54-70
__global__ void __launch_bounds__(256) knn_morton_kernel(int P, const float* __restrict__ pts,
                                                         const float* __restrict__ bbox, uint32_t* __restrict__ codes,
                                                         uint32_t* __restrict__ iota) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    uint32_t c[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float mn = bbox[k], mx = bbox[3 + k];
        c[k] = prep_morton(f2u_sat(((pts[3 * i + k] - mn) / (mx - mn)) * (float)((1 << 10) - 1)));
    }
    codes[i] = c[0] | (c[1] << 1) | (c[2] << 2);
    iota[i] = (uint32_t)i;
}

// knn/simple_knn.cu:78-117
__global__ void __launch_bounds__(kBox) knn_box_minmax(int P, const float* __restrict__ pts,
                                                       const uint32_t* __restrict__ idx, float* __restrict__ boxes) {
    __shared__ float s[6][kBox];
    const int tid = threadIdx.x;
    const int i = blockIdx.x * kBox + tid;
    float mn[3], mx[3];
    if (i < P) {
        const uint32_t j = idx[i];
#pragma unroll
        for (int k = 0; k < 3; k++) mn[k] = mx[k] = pts[3 * j + k];
    } else {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            mn[k] = FLT_MAX;
            mx[k] = -FLT_MAX;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
        s[k][tid] = mn[k];
        s[3 + k][tid] = mx[k];
    }
    __syncthreads();
    for (int off = kBox / 2; off > 0; off >>= 1) {
        if (tid < off)
#pragma unroll
            for (int k = 0; k < 3; k++) {
                s[k][tid] = fminf(s[k][tid], s[k][tid + off]);
                s[3 + k][tid] = fmaxf(s[3 + k][tid], s[3 + k][tid + off]);
            }
        __syncthreads();
    }
    if (tid < 6) boxes[6 * blockIdx.x + tid] = s[tid][0];
}

__device__ __forceinline__ void update_kbest3(float rx, float ry, float rz, const float* __restrict__ p, float* knn) {
    const float dx = p[0] - rx, dy = p[1] - ry, dz = p[2] - rz;
    float dist = dx * dx + dy * dy + dz * dz;
#pragma unroll
    for (int j = 0; j < 3; j++)
        if (knn[j] > dist) {
            const float t = knn[j];
            knn[j] = dist;
            dist = t;
        }
}

// knn/simple_knn.cu:124-183 -- boxes are staged through LDS 1024 at a time.
__global__ void __launch_bounds__(kBox) knn_box_mean_dist(int P, const float* __restrict__ pts,
                                                          const uint32_t* __restrict__ idx,
                                                          const float* __restrict__ boxes, int nb,
                                                          float* __restrict__ dists) {
    __shared__ float sb[kBox * 6];
    const int i = blockIdx.x * kBox + threadIdx.x;
    const bool live = i < P;
    float px = 0, py = 0, pz = 0;
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    float reject = FLT_MAX;
    if (live) {
        const uint32_t me = idx[i];
        px = pts[3 * me];
        py = pts[3 * me + 1];
        pz = pts[3 * me + 2];
        for (int j = max(0, i - 3); j <= min(P - 1, i + 3); j++) {
            if (j == i) continue;
            update_kbest3(px, py, pz, pts + 3 * idx[j], best);
        }
        reject = best[2];
        best[0] = best[1] = best[2] = FLT_MAX;
    }
    for (int b0 = 0; b0 < nb; b0 += kBox) {
        const int cnt = min(kBox, nb - b0);
        __syncthreads();
        for (int t = threadIdx.x; t < cnt * 6; t += kBox) sb[t] = boxes[6 * b0 + t];
        __syncthreads();
        if (!live) continue;
        for (int bb = 0; bb < cnt; bb++) {
            const float* bx = sb + 6 * bb;
            float d[3] = {0.f, 0.f, 0.f};
            const float p[3] = {px, py, pz};
#pragma unroll
            for (int k = 0; k < 3; k++)
                if (p[k] < bx[k] || p[k] > bx[3 + k]) d[k] = fminf(fabsf(p[k] - bx[k]), fabsf(p[k] - bx[3 + k]));
            const float dist = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
            if (dist > reject || dist > best[2]) continue;
            const int b = b0 + bb;
            for (int j = b * kBox; j < min(P, (b + 1) * kBox); j++) {
                if (j == i) continue;
                update_kbest3(px, py, pz, pts + 3 * idx[j], best);
            }
        }
    }
    if (live) dists[idx[i]] = (best[0] + best[1] + best[2]) / 3.0f;
}

static size_t knn_offsets(int P, size_t* o_codes, size_t* o_iota, size_t* o_sc, size_t* o_si, size_t* o_boxes,
                          size_t* o_part, size_t* o_bbox, size_t* o_rs) {
    const int nb = (P + kBox - 1) / kBox;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        off = align_up(off);
        const size_t at = off;
        off += bytes;
        return at;
    };
    *o_codes = take(sizeof(uint32_t) * (size_t)P);
    *o_iota = take(sizeof(uint32_t) * (size_t)P);
    *o_sc = take(sizeof(uint32_t) * (size_t)P);
    *o_si = take(sizeof(uint32_t) * (size_t)P);
    *o_boxes = take(sizeof(float) * 6 * (size_t)max(nb, 1));
    *o_part = take(sizeof(float) * 6 * 1024);
    *o_bbox = take(sizeof(float) * 8);
    *o_rs = take(radix_sort_u32_workspace(P));
    return align_up(off);
}

size_t knn_workspace_bytes(int P) {
    size_t a, b, c, d, e, f, g, h;
    return knn_offsets(P, &a, &b, &c, &d, &e, &f, &g, &h);
}

void launch_knn(int P, const float* points, float* mean_dists, char* ws, hipStream_t s) {
    if (P <= 0) return;
    size_t o_codes, o_iota, o_sc, o_si, o_boxes, o_part, o_bbox, o_rs;
    knn_offsets(P, &o_codes, &o_iota, &o_sc, &o_si, &o_boxes, &o_part, &o_bbox, &o_rs);
    uint32_t* codes = reinterpret_cast<uint32_t*>(ws + o_codes);
    uint32_t* iota = reinterpret_cast<uint32_t*>(ws + o_iota);
    uint32_t* sc = reinterpret_cast<uint32_t*>(ws + o_sc);
    uint32_t* si = reinterpret_cast<uint32_t*>(ws + o_si);
    float* boxes = reinterpret_cast<float*>(ws + o_boxes);
    float* part = reinterpret_cast<float*>(ws + o_part);
    float* bbox = reinterpret_cast<float*>(ws + o_bbox);
    const int nparts = min(1024, (P + 255) / 256);
    hipLaunchKernelGGL(knn_bbox_partial, dim3(nparts), dim3(256), 0, s, P, points, part);
    hipLaunchKernelGGL(knn_bbox_final, dim3(1), dim3(64), 0, s, nparts, part, bbox);
    hipLaunchKernelGGL(knn_morton_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, points, bbox, codes, iota);
    radix_sort_pairs_u32(P, codes, sc, iota, si, 32, ws + o_rs, s);
    const int nb = (P + kBox - 1) / kBox;
    hipLaunchKernelGGL(knn_box_minmax, dim3(nb), dim3(kBox), 0, s, P, points, si, boxes);
    hipLaunchKernelGGL(knn_box_mean_dist, dim3(nb), dim3(kBox), 0, s, P, points, si, boxes, nb, mean_dists);
}

}  // namespace gsamd
