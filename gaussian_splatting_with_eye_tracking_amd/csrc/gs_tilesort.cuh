// gs_tilesort.cuh -- per-tile (depth, index) sort of one tile's keys by one
// workgroup, shared by binning.hip (sort_tiles_* kernels) and render.hip (the
// base forward sorts its own tile before blending it).  The sorted order is
// the reference's stable radix order (base/cr/rasterizer_impl.cu:300-308):
// keys are (depth bits << 32 | Gaussian index), unique, sorted ascending.
#pragma once

#include "gs_device.cuh"

namespace gsamd {

// Exclusive prefix sum of one value per thread over a workgroup of kThreads
// (<= 1024) threads: wave-level shuffle scans, one LDS exchange of the wave
// totals, two barriers.  Also returns the workgroup total.
template <int kThreads>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wave, uint32_t& total) {
    constexpr int kW = kThreads / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)inc, off, 64);
        if (lane >= off) inc += t;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        uint32_t w = lane < kW ? s_wave[lane] : 0u;
        uint32_t wi = w;
#pragma unroll
        for (int off = 1; off < kW; off <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)wi, off, 64);
            if (lane >= off) wi += t;
        }
        if (lane < kW) s_wave[lane] = wi - w;  // exclusive wave offsets
        if (lane == kW - 1) s_wave[kW] = wi;   // total
    }
    __syncthreads();
    total = s_wave[kW];
    return s_wave[wave] + inc - v;
}

// --------------------------------------------------------- tile sorting ---
// In-LDS bitonic sort of S (power of two) u64 keys by `nthreads` threads.
template <int kThreads>
__device__ __forceinline__ void bitonic_lds(uint64_t* s, int S) {
    const int tid = threadIdx.x;
    for (int k = 2; k <= S; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = tid; p < (S >> 1); p += kThreads) {
                const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1));  // j is a power of two
                const int ixj = i + j;
                const bool up = (i & k) == 0;
                const uint64_t a = s[i], b = s[ixj];
                if ((a > b) == up) {
                    s[i] = b;
                    s[ixj] = a;
                }
            }
            __syncthreads();
        }
    }
}

// ---- register-resident bitonic sort of one tile (S <= 256 * kEmax keys).
// Thread-major: thread t holds keys t*E .. t*E+E-1 (E = S/256, S = padded
// size).  A compare-exchange stage (k, j) pairs key i with i ^ j:
//   j < E          partner in the same thread's registers;
//   j < 64 E       partner in lane ^ (j/E) of the same wave (cross-lane shuffle);
//   j >= 64 E      partner in another wave: one LDS exchange + 2 barriers.
// Only log2(S/64E)... the last few stages of each merge touch LDS, so a
// 1024-key tile does 3 LDS stages instead of 55 LDS round trips.
// v of lane ^ M for M in {1, 2, 4, 8, 16, 32}, one cross-lane op each: DPP
// quad_perm (M = 1, 2: a VALU modifier), ds_swizzle bit mode (M = 4, 8: the
// LDS crossbar without an address VGPR), v_permlane16/32_swap (M = 16, 32:
// VALU) -- instead of ds_bpermute.
template <int M>
__device__ __forceinline__ uint32_t shfl_xor_c(uint32_t v) {
    static_assert(M == 1 || M == 2 || M == 4 || M == 8 || M == 16 || M == 32, "xor distance");
    if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // [1,0,3,2]
    if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
    if constexpr (M == 4) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F);              // and 0x1f, xor 4
    if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x201F);              // and 0x1f, xor 8
    if constexpr (M == 16) {
        // with vdst = vsrc = v: r0 = [row0, row0, row2, row2], r1 = [row1, row1, row3, row3]
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        const uint32_t r0 = r[0], r1 = r[1];
        return (__lane_id() & 16) ? r0 : r1;
    }
    if constexpr (M == 32) {
        // r0 = [lo, lo], r1 = [hi, hi] (32-lane halves)
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        const uint32_t r0 = r[0], r1 = r[1];
        return (__lane_id() & 32) ? r0 : r1;
    }
    return v;
}

// One cross-lane compare-exchange stage (k, j) with partner distance
// M = j / E lanes.
template <int M, int E>
__device__ __forceinline__ void bitonic_cross_stage(uint64_t (&v)[E], int k, int j) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int i = tid * E + e;
        const uint32_t lo = shfl_xor_c<M>((uint32_t)v[e]);
        const uint32_t hi = shfl_xor_c<M>((uint32_t)(v[e] >> 32));
        const uint64_t p = ((uint64_t)hi << 32) | lo;
        const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
        v[e] = keep_min ? (v[e] < p ? v[e] : p) : (v[e] < p ? p : v[e]);
    }
}

template <int E, int kWavesUsed>
__device__ __forceinline__ void bitonic_regs(uint64_t (&v)[E], uint64_t* lds) {
    constexpr int S = 64 * kWavesUsed * E;
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 2; k <= S; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j < E) {
#pragma unroll
                for (int e = 0; e < E; e++) {
                    if (e & j) continue;
                    const int i = tid * E + e;
                    const bool up = (i & k) == 0;
                    const uint64_t a = v[e], b = v[e | j];
                    const bool sw = (a > b) == up;
                    v[e] = sw ? b : a;
                    v[e | j] = sw ? a : b;
                }
            } else if (j < 64 * E) {
                if constexpr (E > 4) {
                    // E = 8, 16: the network is not fully unrolled; measured, a
                    // per-stage switch over the specialised moves ran 2.3x slower
                    // at config 4 than ds_bpermute (1.06 vs 0.46 ms)
#pragma unroll
                    for (int e = 0; e < E; e++) {
                        const int i = tid * E + e;
                        const int m = j / E;
                        const int lo = __shfl_xor((int)(uint32_t)v[e], m, 64);
                        const int hi = __shfl_xor((int)(uint32_t)(v[e] >> 32), m, 64);
                        const uint64_t p = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
                        const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
                        v[e] = keep_min ? (v[e] < p ? v[e] : p) : (v[e] < p ? p : v[e]);
                    }
                } else switch (j / E) {  // folded: the E <= 4 networks are fully unrolled
                    case 1: bitonic_cross_stage<1, E>(v, k, j); break;
                    case 2: bitonic_cross_stage<2, E>(v, k, j); break;
                    case 4: bitonic_cross_stage<4, E>(v, k, j); break;
                    case 8: bitonic_cross_stage<8, E>(v, k, j); break;
                    case 16: bitonic_cross_stage<16, E>(v, k, j); break;
                    default: bitonic_cross_stage<32, E>(v, k, j); break;
                }
            } else {
#pragma unroll
                for (int e = 0; e < E; e++) lds[tid * E + e] = v[e];
                __syncthreads();
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const int i = tid * E + e;
                    const uint64_t p = lds[i ^ j];
                    const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
                    v[e] = keep_min ? (v[e] < p ? v[e] : p) : (v[e] < p ? p : v[e]);
                }
                __syncthreads();
            }
        }
    }
}

// (ids: when given, an LDS copy of the sorted ids for the caller)
template <int E, int kWavesUsed>
__device__ __forceinline__ void sort_tile_regs(const uint64_t* __restrict__ keys, int n,
                                               uint32_t* __restrict__ out, uint64_t* lds, uint32_t* ids = nullptr) {
    const int tid = threadIdx.x;
    uint64_t v[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int i = tid * E + e;
        v[e] = i < n ? keys[i] : ~0ull;
    }
    bitonic_regs<E, kWavesUsed>(v, lds);
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int i = tid * E + e;
        if (i < n) {
            out[i] = (uint32_t)v[e];
            if (ids) ids[i] = (uint32_t)v[e];
        }
    }
}

// ---- bucket sort of one tile (n <= 256 kE keys).
// The bitonic networks above cost ~78 compare-exchange stages per key at
// n = 4096 (~20 ps per key at config 2 and config 4 alike).  Here the tile's
// keys go into nb ~ n / 2 buckets by their depth bits relative to the tile's
// min / max (a monotone map: bucket = (depth - min) >> sh), one LDS atomic
// count per key, one scan, one LDS atomic slot per key (arbitrary order inside
// a bucket); then each key's final position is its bucket's start plus the
// number of keys of its bucket that are smaller -- keys are (depth, idx),
// unique, so that is a total order, the same (depth, idx) order the bitonic
// networks and the reference's stable radix sort produce.  Per key: ~10
// VALU + the rank loop over its bucket (~2 keys on average, the wave's longest
// bucket bounds the loop).  A tile whose longest bucket exceeds kBucketMax
// (depths clustered far below the tile's range) takes the bitonic network
// instead, so no distribution is slower than before.
constexpr int kBucketMax = 64;
// kT threads, kE keys each (n <= kT kE); nb ~ n >> kBS buckets.
template <int kT, int kE, int kBS>
struct TileSortLds {
    static constexpr int kW = kT / 64;
    static constexpr int kN = kT * kE;      // keys per tile
    static constexpr int kNB = kN >> kBS;  // buckets at full capacity
    uint64_t tmp[kN];
    // bucket counts, then (scan) starts, then (fill) ends: after the fill,
    // bucket b spans [b ? fill[b - 1] : 0, fill[b])
    uint32_t fill[kNB];
    uint32_t red[2 * kW];
    uint32_t wave[kW + 1];
};

// One tile's n keys (2 <= n <= kT kE) sorted by the whole workgroup of kT
// threads into out (point_list + the tile's start) and, when ids is given,
// into that LDS array too.  Block-uniform n.
// kStageOut: the sorted ids are placed in LDS (over the keys, once every rank
// is known) and stored by consecutive threads, instead of each thread storing
// its keys' ids at their scattered final positions.
template <int kT, int kE, int kBS, bool kStageOut = false>
__device__ __forceinline__ void tile_bucket_sort(const uint64_t* __restrict__ keys, int n, uint32_t* __restrict__ out,
                                                 TileSortLds<kT, kE, kBS>& L, uint32_t* ids = nullptr) {
    constexpr int kW = kT / 64;
    uint64_t* s_tmp = L.tmp;
    uint32_t* s_fill = L.fill;
    uint32_t* s_red = L.red;
    uint32_t* s_wave = L.wave;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // buckets in use: a power of two >= n >> kBS, >= 64 (block-uniform)
    int lg = 6;
    while ((1 << lg) < ((n + (1 << kBS) - 1) >> kBS)) lg++;
    const int nb = 1 << lg;  // <= kNB
    uint64_t k[kE];
    uint32_t dmin = ~0u, dmax = 0u;
#pragma unroll
    for (int e = 0; e < kE; e++) {
        const int i = e * kT + tid;
        k[e] = i < n ? keys[i] : ~0ull;
        if (i < n) {
            const uint32_t d = (uint32_t)(k[e] >> 32);
            dmin = min(dmin, d);
            dmax = max(dmax, d);
        }
    }
    for (int b = tid; b < nb; b += kT) s_fill[b] = 0u;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        dmin = min(dmin, (uint32_t)__shfl_xor((int)dmin, off, 64));
        dmax = max(dmax, (uint32_t)__shfl_xor((int)dmax, off, 64));
    }
    if (lane == 0) {
        s_red[wave] = dmin;
        s_red[kW + wave] = dmax;
    }
    __syncthreads();
    dmin = s_red[0];
    dmax = s_red[kW];
#pragma unroll
    for (int w = 1; w < kW; w++) {
        dmin = min(dmin, s_red[w]);
        dmax = max(dmax, s_red[kW + w]);
    }
    const uint32_t range = dmax - dmin;
    const int bl = range ? 32 - __builtin_clz(range) : 0;
    const int sh = bl > lg ? bl - lg : 0;  // (range >> sh) < nb
    uint32_t bk[kE];
#pragma unroll
    for (int e = 0; e < kE; e++) {
        const int i = e * kT + tid;
        bk[e] = ((uint32_t)(k[e] >> 32) - dmin) >> sh;
        if (i < n) atomicAdd(&s_fill[bk[e]], 1u);
    }
    __syncthreads();
    // exclusive scan of the nb counts: thread t owns buckets [t per, (t + 1) per)
    const int per = nb >= kT ? nb / kT : 1;
    const int b0 = tid * per;
    uint32_t local = 0, cmax = 0;
    for (int q = 0; q < per; q++) {
        const uint32_t c = b0 + q < nb ? s_fill[b0 + q] : 0u;
        local += c;
        cmax = max(cmax, c);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor((int)cmax, off, 64));
    if (lane == 0) s_red[wave] = cmax;  // (s_red's min half was read before the barrier above)
    uint32_t total;
    uint32_t run = block_exclusive_scan<kT>(local, s_wave, total);  // (its barriers publish s_red too)
    for (int q = 0; q < per; q++) {
        if (b0 + q < nb) {
            const uint32_t c = s_fill[b0 + q];
            s_fill[b0 + q] = run;  // start = the fill pointer
            run += c;
        }
    }
    uint32_t bmax = s_red[0];
#pragma unroll
    for (int w = 1; w < kW; w++) bmax = max(bmax, s_red[w]);
    __syncthreads();
    if (bmax > (uint32_t)kBucketMax) {  // block-uniform: clustered depths
        sort_tile_regs<kE, kW>(keys, n, out, s_tmp, ids);
        return;
    }
#pragma unroll
    for (int e = 0; e < kE; e++) {
        const int i = e * kT + tid;
        if (i < n) s_tmp[atomicAdd(&s_fill[bk[e]], 1u)] = k[e];
    }
    __syncthreads();
    uint32_t pos[kE];
#pragma unroll
    for (int e = 0; e < kE; e++) {
        const int i = e * kT + tid;
        pos[e] = ~0u;
        if (i < n) {
            const uint32_t b = bk[e];
            const uint32_t bs = b ? s_fill[b - 1] : 0u, be = s_fill[b];
            uint32_t r = 0;
            for (uint32_t j = bs; j < be; j++) r += s_tmp[j] < k[e] ? 1u : 0u;
            pos[e] = bs + r;
            if constexpr (!kStageOut) {
                out[bs + r] = (uint32_t)k[e];
                if (ids) ids[bs + r] = (uint32_t)k[e];
            }
        }
    }
    if constexpr (kStageOut) {
        uint32_t* s_out = reinterpret_cast<uint32_t*>(s_tmp);
        __syncthreads();  // every rank loop has read the keys
#pragma unroll
        for (int e = 0; e < kE; e++)
            if (pos[e] != ~0u) s_out[pos[e]] = (uint32_t)k[e];
        __syncthreads();
        for (int i = tid; i < n; i += kT) {
            const uint32_t v = s_out[i];
            out[i] = v;
            if (ids) ids[i] = v;
        }
    }
}

}  // namespace gsamd
