// binning.hip -- tile binning for gfx950.
//
// Reference (base/cr/rasterizer_impl.cu:277-318): inclusive scan of
// tiles_touched, duplicateWithKeys (key = tile<<32 | depth bits, value =
// Gaussian idx, emitted in idx order), a STABLE 64-bit LSD radix sort on
// [0, 32+bit(T)), and identifyTileRanges.  Stability + idx-ordered emission
// means the sorted list is exactly "by tile, then by depth bits, then by
// Gaussian idx".
//
// This build produces the same point_list and ranges (bit-exact) with far
// less HBM traffic:
//   1. the preprocess kernel already built a per-tile histogram;
//   2. tile_scan (one workgroup) turns it into ranges/cursors and K;
//   3. duplicate scatters each (depth_bits<<32 | idx) into its tile's bucket
//      with a returning atomic on the tile cursor (order inside a bucket is
//      arbitrary);
//   4. sort_tiles sorts every bucket by the 64-bit (depth, idx) key -- a total
//      order, so the result is deterministic and equals the reference's
//      stable order.  Buckets <= kSmallCap sort in LDS with a bitonic network;
//      larger ones use an LDS chunk sort + in-block merge-path passes.
// Per instance this moves ~20 B instead of the ~200 B of a 6-pass 64-bit
// radix sort.
#include <algorithm>
#include <atomic>
#include <stdexcept>

#include "gs_blend.cuh"
#include "gs_device.cuh"
#include "gs_kernels.h"
#include "gs_tilesort.cuh"

namespace gsamd {

constexpr int kScanThreads = 1024;
constexpr int kSmallCap = 4096;  // LDS bitonic capacity (u64) = 32 KiB
constexpr int kSortThreads = 256;
constexpr int kLargeThreads = 1024;
constexpr int kChunk = 4096;

// ------------------------------------------------------------ tile scan ---
// Tile i's count is the sum of its kBinSlots sub-bucket counts (slot-major
// [kBinSlots][T]: every load is wave-contiguous).
__device__ __forceinline__ uint32_t slot_total(const uint32_t* __restrict__ count, int T, int i, int nslots) {
    uint32_t c = count[i];
#pragma unroll
    for (int s = 1; s < kBinSlots; s++)
        if (s < nslots) c += count[(size_t)s * T + i];
    return c;
}

// Sub-bucket cursors of tile i (slots back to back from the tile's start),
// and the tile's total in place of slot 0's count (tile_count[0..T) = totals
// after the scan: AMR n_intersections, parse_buffers).
__device__ __forceinline__ void slot_cursors(uint32_t* __restrict__ count, uint32_t* __restrict__ cursor, int T,
                                             int i, uint32_t start, uint32_t total, int nslots) {
    cursor[i] = start;
    if (nslots > 1) {
        uint32_t run = start + count[i];
#pragma unroll
        for (int s = 1; s < kBinSlots; s++) {
            if (s >= nslots) break;
            cursor[(size_t)s * T + i] = run;
            run += count[(size_t)s * T + i];
        }
        count[i] = total;
    }
}

// The host's copy of the first four header words, stored straight into
// mapped, coherent host memory (vector stores over the fabric) by the scan:
// the forward's read-back then needs no copy kernel, only an event after the
// scan.
// token != 0 (the polled read-back): after the words, a system-scope fence and
// the call's token in word 4 -- the host spins on the token instead of
// waiting for an event after the scan, so the stream carries no marker packet
// between the scan and the work behind it.
// seqlock: the slot's token is invalidated before the words change, so a
// reader that saw a token, copied the words and sees the same token again read
// words no later scan had started to rewrite (gs_api.cpp finish_header_read).
// The invalidation (and its fence) is issued by the scan's first thread at the
// top of the kernel, under the count loads, instead of in the tail after the
// scan: one system-scope round trip fewer on the scan's critical path.
__device__ __forceinline__ void mirror_invalidate(uint32_t* m, uint32_t token) {
    if (m && token) {
        __hip_atomic_store(m + 4, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
    }
}
__device__ __forceinline__ void mirror_header(uint32_t* m, uint32_t K, uint32_t err, uint32_t maxc, uint32_t nlarge,
                                              uint32_t token) {
    *reinterpret_cast<uint4*>(m) = make_uint4(K, err, maxc, nlarge);  // kHdrNumRendered, kHdrError, kHdrMaxTileCount, kHdrNumLargeTiles
    if (token) {
        __threadfence_system();
        __hip_atomic_store(m + 4, token, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}


// The speculative duplicate publishes the read-back instead of the scan: the
// header words are final once the scan has ended, and its first workgroup's
// first thread copies them to the mapped host slot while the rest of the
// duplicate runs -- the system-scope stores and fences leave the scan's tail
// (the critical path of every forward) for a thread whose wave is one of
// hundreds.  Before the capacity test, so a refused launch still publishes K.
__device__ __forceinline__ void publish_header(const uint32_t* __restrict__ hdr, uint32_t* m, uint32_t token) {
    if (!m || !token || blockIdx.x != 0 || threadIdx.x != 0) return;
    const uint4 w = make_uint4(hdr[kHdrNumRendered], hdr[kHdrError], hdr[kHdrMaxTileCount], hdr[kHdrNumLargeTiles]);
    mirror_invalidate(m, token);
    mirror_header(m, w.x, w.y, w.z, w.w, token);
}

// Row-banded duplicate (below): a tile row's tiles are consecutive, so its
// instances are one contiguous range of the sorted layout, starting at the
// exclusive prefix of its first tile.  The scan stores that start (and the
// staging cursor) per row.
struct BandScan {
    uint32_t* start;  // nullptr: direct duplicate
    uint32_t* cursor;
    uint32_t gx;
    uint32_t mirror_token;  // the polled header read-back's token (0: none; see mirror_header)
    __device__ __forceinline__ void emit(int i, uint32_t ex) const {
        if (!start || (uint32_t)i % gx) return;
        const uint32_t row = (uint32_t)i / gx;
        start[row] = ex;
        cursor[row] = ex;
    }
};

// kPer > 0: T <= 1024 kPer, each thread's kPer counts loaded by an unrolled
// loop (all loads in flight at once, no serial load-add chain: 16 -> 5 us at
// 8160 tiles); kPer = 0: any T, run-time loop.
template <int kPer>
__global__ void __launch_bounds__(kScanThreads) tile_scan_kernel(int T, uint32_t* __restrict__ count,
                                                                 uint32_t* __restrict__ ranges,
                                                                 uint32_t* __restrict__ cursor,
                                                                 uint32_t* __restrict__ large_tiles,
                                                                 uint32_t* __restrict__ hdr,
                                                                 uint32_t* __restrict__ bucket_count,
                                                                 uint32_t* __restrict__ hdr_mirror, int nslots,
                                                                 BandScan band) {
    __shared__ uint32_t s_wave[kScanThreads / 64 + 1];
    __shared__ uint32_t s_max[kScanThreads / 64];
    __shared__ uint32_t nlarge;
    const int tid = threadIdx.x;
    if (bucket_count && tid < kOrderBuckets64) bucket_count[tid] = 0;  // the forward render appends to the buckets
    const int per = kPer > 0 ? kPer : (T + kScanThreads - 1) / kScanThreads;
    const int beg = min(T, tid * per), end = min(T, beg + per);
    uint32_t sum = 0, mx = 0;
    uint32_t cv[kPer > 0 ? kPer : 1];
    // (the preprocess's error word, read while the counts load; this kernel
    // does not write it)
    const uint32_t err = (tid == 0 && hdr_mirror) ? hdr[kHdrError] : 0u;
    if constexpr (kPer > 0) {
#pragma unroll
        for (int k = 0; k < kPer; k++) cv[k] = beg + k < end ? slot_total(count, T, beg + k, nslots) : 0u;
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            sum += cv[k];
            mx = max(mx, cv[k]);
        }
    } else {
        for (int i = beg; i < end; i++) {
            const uint32_t c = slot_total(count, T, i, nslots);
            sum += c;
            mx = max(mx, c);
        }
    }
    if (tid == 0) {
        nlarge = 0;
        mirror_invalidate(hdr_mirror, band.mirror_token);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    if ((tid & 63) == 0) s_max[tid >> 6] = mx;
    uint32_t total;
    uint32_t run = block_exclusive_scan<kScanThreads>(sum, s_wave, total);
    auto emit = [&](int i, uint32_t c) {
        // identifyTileRanges leaves empty tiles at (0,0) (rasterizer_impl.cu:310).
        reinterpret_cast<uint2*>(ranges)[i] = make_uint2(c ? run : 0u, c ? run + c : 0u);
        slot_cursors(count, cursor, T, i, run, c, nslots);
        band.emit(i, run);
        if (c > (uint32_t)kSmallCap) {
            const uint32_t slot = atomicAdd(&nlarge, 1u);
            large_tiles[slot] = (uint32_t)i;
        }
        run += c;
    };
    if constexpr (kPer > 0) {
#pragma unroll
        for (int k = 0; k < kPer; k++)
            if (beg + k < end) emit(beg + k, cv[k]);
    } else {
        for (int i = beg; i < end; i++) emit(i, slot_total(count, T, i, nslots));
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t m = 0;
        for (int w = 0; w < kScanThreads / 64; w++) m = max(m, s_max[w]);
        hdr[kHdrNumRendered] = total;
        hdr[kHdrMaxTileCount] = m;
        hdr[kHdrNumLargeTiles] = nlarge;
        hdr[kHdrT] = (uint32_t)T;
        if (hdr_mirror) mirror_header(hdr_mirror, total, err, m, nlarge, band.mirror_token);
    }
}

// The same scan with tile i = k * kScanThreads + tid (slice k of the thread):
// every count load and every range / cursor store is wave-contiguous (the
// thread-contiguous layout above issues each store as 64 scattered sector
// writes from the one CU).  The kS slices are scanned together: a 64-lane
// shuffle scan per slice, the per-(wave, slice) totals through LDS, one
// barrier; slice k's base is the total of slices < k.  Same sums, same order of
// the integer adds' results: bit-identical ranges, cursors, K.
template <int kS>
__global__ void __launch_bounds__(kScanThreads) tile_scan_slices_kernel(int T, uint32_t* __restrict__ count,
                                                                        uint32_t* __restrict__ ranges,
                                                                        uint32_t* __restrict__ cursor,
                                                                        uint32_t* __restrict__ large_tiles,
                                                                        uint32_t* __restrict__ hdr,
                                                                        uint32_t* __restrict__ bucket_count,
                                                                        uint32_t* __restrict__ hdr_mirror,
                                                                        int nslots, BandScan band) {
    constexpr int kW = kScanThreads / 64;
    if (bucket_count && threadIdx.x < kOrderBuckets64) bucket_count[threadIdx.x] = 0;  // the forward render appends
    __shared__ uint32_t s_tot[kW][kS];
    __shared__ uint32_t s_base[kW][kS];
    __shared__ uint32_t s_total;
    __shared__ uint32_t s_max[kW];
    __shared__ uint32_t nlarge;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t c[kS], incl[kS];
    uint32_t mx = 0;
    const uint32_t err = (tid == 0 && hdr_mirror) ? hdr[kHdrError] : 0u;  // (as tile_scan_kernel)
#pragma unroll
    for (int k = 0; k < kS; k++) {
        const int i = k * kScanThreads + tid;
        c[k] = i < T ? slot_total(count, T, i, nslots) : 0u;
        incl[k] = c[k];
        mx = max(mx, c[k]);
    }
    if (tid == 0) {
        nlarge = 0;
        mirror_invalidate(hdr_mirror, band.mirror_token);
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
        for (int k = 0; k < kS; k++) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl[k], d, 64);
            if (lane >= d) incl[k] += y;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    if (lane == 63) {
#pragma unroll
        for (int k = 0; k < kS; k++) s_tot[wave][k] = incl[k];
        s_max[wave] = mx;
    }
    __syncthreads();
    // wave 0: exclusive prefix of the kS x kW (slice, wave) totals in (slice,
    // wave) order -- each thread then reads its one base per slice instead of
    // all kW totals of every slice (128 broadcast LDS reads per thread: 0.0139
    // -> 0.0110 ms at config 2, profiles/r04za_ab_scan*.log)
    static_assert(kS * kW <= 128, "two (slice, wave) totals per lane");
    if (wave == 0) {
        const int q0 = 2 * lane, q1 = 2 * lane + 1;  // flattened k * kW + w
        const uint32_t v0 = q0 < kS * kW ? s_tot[q0 % kW][q0 / kW] : 0u;
        const uint32_t v1 = q1 < kS * kW ? s_tot[q1 % kW][q1 / kW] : 0u;
        uint32_t inc = v0 + v1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= d) inc += y;
        }
        const uint32_t ex0 = inc - v0 - v1;
        if (q0 < kS * kW) s_base[q0 % kW][q0 / kW] = ex0;
        if (q1 < kS * kW) s_base[q1 % kW][q1 / kW] = ex0 + v0;
        if (lane == 63) s_total = inc;
    }
    __syncthreads();
    const uint32_t run = s_total;  // K
#pragma unroll
    for (int k = 0; k < kS; k++) {
        const int i = k * kScanThreads + tid;
        if (i < T) {
            const uint32_t ex = s_base[wave][k] + incl[k] - c[k];
            // identifyTileRanges leaves empty tiles at (0,0) (rasterizer_impl.cu:310)
            reinterpret_cast<uint2*>(ranges)[i] = make_uint2(c[k] ? ex : 0u, c[k] ? ex + c[k] : 0u);
            slot_cursors(count, cursor, T, i, ex, c[k], nslots);
            band.emit(i, ex);
            if (c[k] > (uint32_t)kSmallCap) large_tiles[atomicAdd(&nlarge, 1u)] = (uint32_t)i;
        }
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t m = 0;
        for (int w = 0; w < kW; w++) m = max(m, s_max[w]);
        hdr[kHdrNumRendered] = run;
        hdr[kHdrMaxTileCount] = m;
        hdr[kHdrNumLargeTiles] = nlarge;
        hdr[kHdrT] = (uint32_t)T;
        if (hdr_mirror) mirror_header(hdr_mirror, run, err, m, nlarge, band.mirror_token);
    }
}

void launch_tile_scan(int T, const ImageView& img, uint32_t* hdr, hipStream_t s, uint32_t* hdr_mirror, int nslots,
                      int gx, bool banded, uint32_t mirror_token) {
    BandScan band{nullptr, nullptr, (uint32_t)std::max(gx, 1), mirror_token};
    if (banded) {
        band.start = img.band_start;
        band.cursor = img.band_cursor;
    }
    {  // T <= 8192 (1080p at 16 px: 8160): the wave-contiguous slices; larger grids below
        const int slices = (T + kScanThreads - 1) / kScanThreads;
#define GS_SLICE_LAUNCH(S)                                                                                        \
    hipLaunchKernelGGL(tile_scan_slices_kernel<S>, dim3(1), dim3(kScanThreads), 0, s, T, img.tile_count,         \
                       img.ranges, img.tile_cursor, img.large_tiles, hdr, img.bucket_count, hdr_mirror, nslots, band)
        if (slices <= 1) { GS_SLICE_LAUNCH(1); return; }
        if (slices <= 2) { GS_SLICE_LAUNCH(2); return; }
        if (slices <= 4) { GS_SLICE_LAUNCH(4); return; }
        if (slices <= 8) { GS_SLICE_LAUNCH(8); return; }
#undef GS_SLICE_LAUNCH
    }
#define GS_SCAN_LAUNCH(PER)                                                                                      \
    hipLaunchKernelGGL(tile_scan_kernel<PER>, dim3(1), dim3(kScanThreads), 0, s, T, img.tile_count, img.ranges, \
                       img.tile_cursor, img.large_tiles, hdr, img.bucket_count, hdr_mirror, nslots, band)
    const int per = (T + kScanThreads - 1) / kScanThreads;
    if (per <= 2) GS_SCAN_LAUNCH(2);
    else if (per <= 4) GS_SCAN_LAUNCH(4);
    else if (per <= 8) GS_SCAN_LAUNCH(8);
    else if (per <= 16) GS_SCAN_LAUNCH(16);
    else GS_SCAN_LAUNCH(0);
#undef GS_SCAN_LAUNCH
}

// ------------------------------------------------------------- duplicate ---
__global__ void __launch_bounds__(256) duplicate_kernel(int P, const float* __restrict__ means2D,
                                                        const float* __restrict__ depths,
                                                        const int* __restrict__ radii, int block, uint32_t gx,
                                                        uint32_t gy, uint32_t* __restrict__ cursor,
                                                        uint64_t* __restrict__ pair_keys,
                                                        const uint32_t* __restrict__ hdr, uint32_t cap,
                                                        uint32_t* mirror, uint32_t mirror_token) {
    publish_header(hdr, mirror, mirror_token);
    if (hdr && hdr[kHdrNumRendered] > cap) return;  // speculative launch, K > cap (duplicate_lds_kernel)
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const int rad = radii[idx];
    if (rad <= 0) return;
    const float2 xy = reinterpret_cast<const float2*>(means2D)[idx];
    const Rect r = get_rect(xy.x, xy.y, rad, block, block, gx, gy);
    const uint64_t key = ((uint64_t)float_bits(depths[idx]) << 32) | (uint32_t)idx;
    // Walk the rect row-major with kInFlight returning atomics outstanding
    // (one round trip per kInFlight tiles instead of per tile).
    constexpr int kInFlight = 8;
    const uint32_t w = r.x1 - r.x0;
    const uint32_t area = w * (r.y1 - r.y0);
    uint32_t x = r.x0, y = r.y0;
    for (uint32_t i0 = 0; i0 < area; i0 += kInFlight) {
        uint32_t pos[kInFlight];
#pragma unroll
        for (int u = 0; u < kInFlight; u++) {
            if (i0 + u < area) {
                pos[u] = atomicAdd(&cursor[y * gx + x], 1u);
                if (++x == r.x1) {
                    x = r.x0;
                    ++y;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kInFlight; u++)
            if (i0 + u < area) pair_keys[pos[u]] = key;
    }
}

// ------------------------------------------- LDS-privatised binning ---
// Device-scope atomics execute at the memory side, one 64-B request each
// when scattered (MI355X_MICROARCH.md "Global float atomics"): 4.4M per-pair
// histogram increments plus 4.4M returning cursor bumps at config 2 cost
// ~0.2 ms apiece.  Instead a workgroup of kBinThreads threads takes a chunk
// of bin_chunk_for(P) consecutive Gaussians and counts its (Gaussian, tile) pairs
// in an LDS histogram over all T tiles, then
//   count_tiles: adds the histogram to tile_count with consecutive-tile
//                (coalesced, no-return) atomics, one per non-empty tile;
//   duplicate:   reserves each non-empty tile's run with ONE coalesced
//                returning atomic on the tile cursor, then hands out slots
//                inside the run with LDS atomics and writes the keys.
// Slot order inside a bucket stays arbitrary; sort_tiles makes it exact.
constexpr int kBinThreads = 1024;
// Gaussians per binning workgroup (count_tiles and duplicate_lds must agree:
// the chunk -> sub-bucket slot map): 8192 from 4M Gaussians (config 4
// count_tiles 57.0 -> 52.4 us), else 4096 (config 2: 22.1 us vs 29.9 at
// 8192; 2048 / 1024: 27.4 / 42.4 us), profiles/r04l_ab_chunk*.log,
// r04zh_chunk_*.log
int bin_chunk_for(int P) { return P >= 4000000 ? 8192 : 4096; }
// The banded duplicate's workgroup shape: 1024 threads x 1 source below 2M
// Gaussians (config 2: 77.6 us, direct duplicate 87.3), 512 x 2 sources per
// thread above (config 4: 282 us, direct 318; profiles/r03h_ab_threads_cfg*.json,
// the other shapes removed).
constexpr int kBandBins = 1024;  // bins of one coalesced append round (rows, or the tiles of a row)
// Banded only on the base 16-px grid: on the AMR 32-px grid (34 tile rows
// at 1080p, ~2.2 instances per Gaussian) the direct duplicate is cheaper
// (46 vs 56 us at config 3, profiles/r03h_ab_amr_band.json).
bool band_lds_fits();  // (below: the banded kernels' dynamic LDS fits the current device)
bool dup_banded(int gx, int gy, int block) {
    if (gx * gy > kLdsTiles || gx > kBandBins || gy > kBandBins) return false;
    return block == 16 && band_lds_fits();
}
// sub-bucket slots the LDS binning spreads its chunks over (1..kBinSlots; the
// scan sums all kBinSlots, unused ones stay zero).  Measured
// (profiles/r03b_ab_bin_slots*): the sub-buckets save ~30 us of the direct
// duplicate at config 4 (6.1M Gaussians) and ~4 us at config 2, where the
// scan's 8x count loads cost more (+6 us): slots only for large scenes.
int bin_slots_for(int P, int gx, int gy, int block) {
    if (dup_banded(gx, gy, block)) return 1;  // the banded duplicate reserves per-tile runs itself
    return P >= 2000000 ? kBinSlots : 1;
}

__device__ __forceinline__ bool gaussian_rect(int idx, const float* __restrict__ means2D,
                                              const int* __restrict__ radii, int block, uint32_t gx, uint32_t gy,
                                              Rect& r) {
    const int rad = radii[idx];
    if (rad <= 0) return false;
    const float2 xy = reinterpret_cast<const float2*>(means2D)[idx];
    r = get_rect(xy.x, xy.y, rad, block, block, gx, gy);
    return true;
}

// The rect of a Gaussian whose radius and mean are already loaded (the
// binning loops request every Gaussian's loads up front: a loop over
// gaussian_rect waited for the radius, then -- behind its branch -- for the
// mean, twice per Gaussian).
__device__ __forceinline__ bool rect_of(int rad, float2 xy, int block, uint32_t gx, uint32_t gy, Rect& r) {
    if (rad <= 0) return false;
    r = get_rect(xy.x, xy.y, rad, block, block, gx, gy);
    return true;
}
constexpr int kBinPerMax = 8;  // Gaussians per thread per binning chunk (bin_chunk_for / kBinThreads)

__global__ void __launch_bounds__(kBinThreads) count_tiles_kernel(int P, int chunk, const float* __restrict__ means2D,
                                                                  const int* __restrict__ radii, int block,
                                                                  uint32_t gx, uint32_t gy,
                                                                  uint32_t* __restrict__ tile_count, uint32_t nslots) {
    extern __shared__ uint32_t hist[];
    const int T = (int)(gx * gy);
    const int beg = blockIdx.x * chunk, end = min(P, beg + chunk);
    int rad[kBinPerMax];
    float2 xy[kBinPerMax];
#pragma unroll
    for (int u = 0; u < kBinPerMax; u++) {
        const int idx = beg + threadIdx.x + u * kBinThreads;
        const bool in = u * kBinThreads < chunk && idx < end;
        rad[u] = in ? radii[idx] : 0;
        xy[u] = in ? reinterpret_cast<const float2*>(means2D)[idx] : make_float2(0.f, 0.f);
    }
    for (int i = threadIdx.x; i < T; i += kBinThreads) hist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kBinPerMax; u++) {
        Rect r;
        if (!rect_of(rad[u], xy[u], block, gx, gy, r)) continue;
        for (uint32_t y = r.y0; y < r.y1; y++)
            for (uint32_t x = r.x0; x < r.x1; x++) atomicAdd(&hist[y * gx + x], 1u);
    }
    __syncthreads();
    uint32_t* cnt = tile_count + (size_t)(blockIdx.x % nslots) * T;  // this chunk's sub-bucket slot
    for (int i = threadIdx.x; i < T; i += kBinThreads) {
        const uint32_t c = hist[i];
        if (c) atomicAdd(&cnt[i], c);
    }
}

__global__ void __launch_bounds__(kBinThreads) duplicate_lds_kernel(int P, int chunk,
                                                                    const float* __restrict__ means2D,
                                                                    const float* __restrict__ depths,
                                                                    const int* __restrict__ radii, int block,
                                                                    uint32_t gx, uint32_t gy,
                                                                    uint32_t* __restrict__ cursor,
                                                                    uint64_t* __restrict__ pair_keys,
                                                                    const uint32_t* __restrict__ hdr, uint32_t cap,
                                                                    uint32_t nslots, uint32_t* mirror,
                                                                    uint32_t mirror_token) {
    publish_header(hdr, mirror, mirror_token);
    // speculative launch (hdr given): the keys fit the buffer only if K <= cap;
    // otherwise nothing is touched (no cursor moved) and the host relaunches
    if (hdr && hdr[kHdrNumRendered] > cap) return;
    extern __shared__ uint32_t slot[];
    const int T = (int)(gx * gy);
    const int beg = blockIdx.x * chunk, end = min(P, beg + chunk);
    // the chunk's radii, means and depths, requested up front and kept for
    // both passes
    int rad[kBinPerMax];
    float2 xy[kBinPerMax];
    float dep[kBinPerMax];
#pragma unroll
    for (int u = 0; u < kBinPerMax; u++) {
        const int idx = beg + threadIdx.x + u * kBinThreads;
        const bool in = u * kBinThreads < chunk && idx < end;
        rad[u] = in ? radii[idx] : 0;
        xy[u] = in ? reinterpret_cast<const float2*>(means2D)[idx] : make_float2(0.f, 0.f);
        dep[u] = in ? depths[idx] : 0.f;
    }
    for (int i = threadIdx.x; i < T; i += kBinThreads) slot[i] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kBinPerMax; u++) {
        Rect r;
        if (!rect_of(rad[u], xy[u], block, gx, gy, r)) continue;
        for (uint32_t y = r.y0; y < r.y1; y++)
            for (uint32_t x = r.x0; x < r.x1; x++) atomicAdd(&slot[y * gx + x], 1u);
    }
    __syncthreads();
    // one returning atomic per non-empty tile: the chunk's run in the bucket
    uint32_t* cur = cursor + (size_t)(blockIdx.x % nslots) * T;  // the slot count_tiles counted this chunk in
    for (int i = threadIdx.x; i < T; i += kBinThreads) {
        const uint32_t c = slot[i];
        if (c) slot[i] = atomicAdd(&cur[i], c);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kBinPerMax; u++) {
        Rect r;
        if (!rect_of(rad[u], xy[u], block, gx, gy, r)) continue;
        const int idx = beg + threadIdx.x + u * kBinThreads;
        const uint64_t key = ((uint64_t)float_bits(dep[u]) << 32) | (uint32_t)idx;
        for (uint32_t y = r.y0; y < r.y1; y++)
            for (uint32_t x = r.x0; x < r.x1; x++) {
                const uint32_t sl = atomicAdd(&slot[y * gx + x], 1u);
                pair_keys[sl] = key;
            }
    }
}

void launch_count_tiles(int P, const GeomView& g, const int* radii, int W, int H, int block, const ImageView& img,
                        hipStream_t s) {
    const uint32_t gx = (uint32_t)((W + block - 1) / block), gy = (uint32_t)((H + block - 1) / block);
    if (P == 0 || gx * gy == 0) return;
    const int chunk = bin_chunk_for(P);
    hipLaunchKernelGGL(count_tiles_kernel, dim3((P + chunk - 1) / chunk), dim3(kBinThreads),
                       sizeof(uint32_t) * gx * gy, s, P, chunk, g.means2D, radii, block, gx, gy, img.tile_count,
                       (uint32_t)bin_slots_for(P, (int)gx, (int)gy, block));
}

// ------------------------------------------------- banded duplicate ---
// Measured: the direct duplicate's cost follows its scattered store
// REQUESTS, not its bytes -- at config 4 ~22M lane-scattered 8-B stores
// take ~240 of its ~310 us, and staging half as many entries with the same
// scatter pattern costs the same (profiles/r03h_band*).  A wave's store is
// only cheap when its 64 lanes hit a few contiguous segments.  So both
// passes below append through a workgroup-level LDS reorder
// (coalesced_append): each round, every thread emits up to kRound items
// (bin, payload); an LDS histogram + workgroup scan gives each bin a local
// range, ONE returning atomic per non-empty bin reserves its global run, the
// items are placed bin-major in LDS and written out by consecutive threads
// -- consecutive addresses within each run.  With bins = the tile ROWS
// (gy <= 1024) the runs per round are ~64 items long:
//   stage: one entry per (Gaussian, tile row it touches) -- the key in
//          scratch, its column span x0 | x1 << 16 in point_list (both dead
//          until the sort) -- appended into the row's range of the sorted
//          layout (capacity = the row's instances >= its entries);
//   split: workgroups per row read its entries coalesced and append each
//          (entry, tile) key into the tile's range, bins = the row's tiles.
// Per tile the multiset of keys is the direct duplicate's; the sort makes
// the order exact (bit-identical point_list).
// Gaussians per stage workgroup (runs reserved once per row per chunk): 2048
// -- twice the workgroups of 4096, two or four Gaussians per thread -- against
// 4096: duplicate 0.0678 -> 0.0663 ms at config 2, 0.2464 -> 0.2409 at config
// 4 (1024: 0.0702; profiles/r05at_ab_stage_chunk_*.log)
constexpr int kStageChunk = 2048;

// kNT threads per workgroup; each owns kBandBins / kNT consecutive bins in
// the per-bin steps.
template <int kNT, int kRound>  // items per thread per round
struct AppendLds {
    uint32_t cnt[kBandBins];  // round counts -> local offsets
    uint32_t dst[kBandBins];  // global slot - local offset, this round
    uint32_t run[kBandBins];  // the workgroup's next global slot per bin (runs reserved up front)
    uint32_t wave[kNT / 64 + 1];
    uint64_t key[kNT * kRound];
    uint32_t aux[kNT * kRound];
    uint32_t to[kNT * kRound];
    uint16_t src[kNT * kRound];  // expand_sources: the source of each pair of the round
};

// The workgroup's whole histogram (accumulated in L.run by the caller) ->
// its runs: ONE returning device atomic per non-empty bin per workgroup.
template <int kNT, int kRound>
__device__ __forceinline__ void reserve_runs(AppendLds<kNT, kRound>& L, uint32_t* __restrict__ cursor,
                                             uint32_t nbins) {
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += kNT) {
        const uint32_t c = L.run[b];
        if (c) L.run[b] = atomicAdd(&cursor[b], c);
    }
    __syncthreads();
}

// One round: items (bin[r], key[r], aux[r]) for r < n (per thread) are
// placed bin-major in LDS and written out by consecutive threads at the
// workgroup's runs -- consecutive addresses inside each run.  LDS only (the
// runs are reserved); must be called by the whole workgroup.
template <bool kAux, int kNT, int kRound>
__device__ __forceinline__ void coalesced_append(AppendLds<kNT, kRound>& L, int n, const uint32_t* bin,
                                                 const uint64_t* key, const uint32_t* aux,
                                                 uint64_t* __restrict__ out_key, uint32_t* __restrict__ out_aux,
                                                 uint32_t limit) {
    constexpr int kBPT = kBandBins / kNT;
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < kBPT; q++) L.cnt[tid * kBPT + q] = 0;
    __syncthreads();
    uint32_t rank[kRound];
#pragma unroll
    for (int r = 0; r < kRound; r++)
        if (r < n) rank[r] = atomicAdd(&L.cnt[bin[r]], 1u);
    __syncthreads();
    uint32_t c[kBPT], sum = 0;
#pragma unroll
    for (int q = 0; q < kBPT; q++) {
        c[q] = L.cnt[tid * kBPT + q];
        sum += c[q];
    }
    uint32_t total;
    uint32_t lo = block_exclusive_scan<kNT>(sum, L.wave, total);
#pragma unroll
    for (int q = 0; q < kBPT; q++) {
        const int bq = tid * kBPT + q;
        if (c[q]) {
            const uint32_t base = L.run[bq];
            L.dst[bq] = base - lo;
            L.run[bq] = base + c[q];
        }
        L.cnt[bq] = lo;
        lo += c[q];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRound; r++) {
        if (r < n) {
            const uint32_t i = L.cnt[bin[r]] + rank[r];
            L.key[i] = key[r];
            if constexpr (kAux) L.aux[i] = aux[r];
            L.to[i] = L.dst[bin[r]] + i;
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < total; i += kNT) {
        const uint32_t t = L.to[i];
        if (t >= limit) continue;  // never past the buffer (the runs are exact; this only bounds a bug)
        out_key[t] = L.key[i];
        if constexpr (kAux) out_aux[t] = L.aux[i];
    }
}

// Sources (kSPT per thread: Gaussians, or staged entries) expand to count
// consecutive bins from first; the workgroup's expansion is handed out in
// blocks of kRound consecutive pairs per thread, kRound x kNT pairs per append
// round.  Each round the sources overlapping its window write their index
// into the window's pair slots (L.src) and every pair reads its source from
// there (one LDS read instead of a binary search over the scanned counts).
template <int kNS>
struct SourceLds {
    uint64_t key[kNS];
    uint32_t aux[kNS];
    uint32_t first[kNS];
    uint32_t pref[kNS];  // exclusive prefix of the counts
    uint32_t wave[kNS / 64 + 1];
};

template <bool kAux, int kNT, int kRound, int kSPT>
__device__ __forceinline__ void expand_sources(SourceLds<kNT * kSPT>& S, AppendLds<kNT, kRound>& L,
                                               const uint32_t* cnt, const uint64_t* key, const uint32_t* aux,
                                               const uint32_t* first, uint64_t* __restrict__ out_key,
                                               uint32_t* __restrict__ out_aux, uint32_t limit) {
    constexpr int kNS = kNT * kSPT;
    const int tid = threadIdx.x;
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < kSPT; q++) sum += cnt[q];
    static_assert(kNS <= 65536, "16-bit source indices");
    constexpr uint32_t kW = kNT * kRound;  // pairs per round
    uint32_t np;
    uint32_t pre = block_exclusive_scan<kNT>(sum, S.wave, np);
    uint32_t pr[kSPT];
#pragma unroll
    for (int q = 0; q < kSPT; q++) {
        const int i = tid * kSPT + q;
        S.key[i] = key[q];
        if constexpr (kAux) S.aux[i] = aux[q];
        S.first[i] = first[q];
        S.pref[i] = pre;
        pr[q] = pre;
        pre += cnt[q];
    }
    for (uint32_t j0 = 0; j0 < np; j0 += kW) {
        // the window's pairs -> their sources
#pragma unroll
        for (int q = 0; q < kSPT; q++) {
            const uint32_t lo = max(pr[q], j0), hi = min(pr[q] + cnt[q], j0 + kW);
            for (uint32_t k = lo; k < hi; k++) L.src[k - j0] = (uint16_t)(tid * kSPT + q);
        }
        __syncthreads();  // (also: the sources' LDS rows, at the first round)
        uint32_t bin[kRound], ax[kRound];
        uint64_t ky[kRound];
        int n = 0;
        uint32_t j = j0 + (uint32_t)(tid * kRound);
#pragma unroll
        for (int r = 0; r < kRound; r++, j++) {
            if (j < np) {
                const int s = L.src[j - j0];
                bin[n] = S.first[s] + (j - S.pref[s]);
                ky[n] = S.key[s];
                if constexpr (kAux) ax[n] = S.aux[s];
                n++;
            }
        }
        coalesced_append<kAux, kNT, kRound>(L, n, bin, ky, ax, out_key, out_aux, limit);
        __syncthreads();
    }
}

template <int kNT, int kRound, int kSPT>
struct BandLds {
    AppendLds<kNT, kRound> a;
    SourceLds<kNT * kSPT> src;
};

// The banded kernels need more than 64 KiB of dynamic LDS (65.6 KB for
// <1024, 2, 1>): fine on gfx950's 160 KB, not on 64-KiB parts.  Checked per
// device, once; a device where it does not fit keeps the direct duplicate
// (dup_banded false, so the bin-slot policy follows too).
constexpr size_t kBandLdsMax = std::max(sizeof(BandLds<1024, 2, 1>), sizeof(BandLds<512, 2, 2>));
constexpr int kMaxDevices = 64;
std::atomic<int> g_band_fits[kMaxDevices];  // 0 unknown, 1 fits, 2 does not
bool band_lds_fits() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return false;
    int v = g_band_fits[dev].load(std::memory_order_relaxed);
    if (v == 0) {
        // the opt-in maximum (what hipFuncSetAttribute may grant), not the
        // 64-KiB default per-block figure
        int cap = 0;
        if (hipDeviceGetAttribute(&cap, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || cap <= 0)
            cap = 0;
        const bool ok = (size_t)cap >= kBandLdsMax;
        v = ok ? 1 : 2;
        g_band_fits[dev].store(v, std::memory_order_relaxed);
    }
    return v == 1;
}

template <int kNT, int kRound, int kSPT>
__global__ void __launch_bounds__(kNT) band_stage_kernel(int P, const float* __restrict__ means2D,
                                                         const float* __restrict__ depths,
                                                         const int* __restrict__ radii, int block, uint32_t gx,
                                                         uint32_t gy, uint32_t* __restrict__ row_cursor,
                                                         uint64_t* __restrict__ stage_keys,
                                                         uint32_t* __restrict__ stage_cols,
                                                         const uint32_t* __restrict__ hdr, uint32_t cap,
                                                         uint32_t limit, uint32_t* mirror, uint32_t mirror_token) {
    publish_header(hdr, mirror, mirror_token);
    if (hdr && hdr[kHdrNumRendered] > cap) return;  // speculative launch, K > cap (duplicate_lds_kernel)
    constexpr int kStageG = kStageChunk / kNT;
    static_assert(kStageG % kSPT == 0, "whole source groups");
    extern __shared__ __align__(16) unsigned char lds_raw[];
    BandLds<kNT, kRound, kSPT>& B = *reinterpret_cast<BandLds<kNT, kRound, kSPT>*>(lds_raw);
    // the thread's Gaussians: kSPT consecutive indices per group
    uint32_t cnt[kStageG], cols[kStageG], y0[kStageG];
    uint64_t key[kStageG];
    int rad[kStageG];
    float2 xy[kStageG];
    float dep[kStageG];
#pragma unroll
    for (int g = 0; g < kStageG; g++) {  // every Gaussian's loads requested up front
        const int idx = blockIdx.x * kStageChunk + ((g / kSPT) * kNT + threadIdx.x) * kSPT + g % kSPT;
        rad[g] = idx < P ? radii[idx] : 0;
        xy[g] = idx < P ? reinterpret_cast<const float2*>(means2D)[idx] : make_float2(0.f, 0.f);
        dep[g] = idx < P ? depths[idx] : 0.f;
    }
#pragma unroll
    for (int g = 0; g < kStageG; g++) {
        const int idx = blockIdx.x * kStageChunk + ((g / kSPT) * kNT + threadIdx.x) * kSPT + g % kSPT;
        cnt[g] = cols[g] = y0[g] = 0;
        key[g] = 0;
        Rect rc;
        if (rect_of(rad[g], xy[g], block, gx, gy, rc) && rc.x1 > rc.x0) {
            cnt[g] = rc.y1 - rc.y0;  // one entry per tile row
            y0[g] = rc.y0;
            cols[g] = rc.x0 | (rc.x1 << 16);
            key[g] = ((uint64_t)float_bits(dep[g]) << 32) | (uint32_t)idx;
        }
    }
    for (int b = threadIdx.x; b < kBandBins; b += kNT) B.a.run[b] = 0;
    __syncthreads();
#pragma unroll
    for (int g = 0; g < kStageG; g++)
        for (uint32_t y = y0[g]; y < y0[g] + cnt[g]; y++) atomicAdd(&B.a.run[y], 1u);
    reserve_runs(B.a, row_cursor, gy);
#pragma unroll
    for (int g = 0; g < kStageG; g += kSPT)
        expand_sources<true, kNT, kRound, kSPT>(B.src, B.a, cnt + g, key + g, cols + g, y0 + g, stage_keys,
                                                stage_cols, limit);
}

template <int kNT, int kRound, int kSPT>
__global__ void __launch_bounds__(kNT) band_split_kernel(uint32_t gx, int split, const uint32_t* __restrict__ row_start,
                                                         const uint32_t* __restrict__ row_cursor,
                                                         const uint64_t* __restrict__ stage_keys,
                                                         const uint32_t* __restrict__ stage_cols,
                                                         uint32_t* __restrict__ tile_cursor,
                                                         uint64_t* __restrict__ pair_keys,
                                                         const uint32_t* __restrict__ hdr, uint32_t cap,
                                                         uint32_t limit) {
    if (hdr && hdr[kHdrNumRendered] > cap) return;
    constexpr uint32_t kCh = kNT * kSPT;  // entries per chunk
    extern __shared__ __align__(16) unsigned char lds_raw[];
    BandLds<kNT, kRound, kSPT>& B = *reinterpret_cast<BandLds<kNT, kRound, kSPT>*>(lds_raw);
    const uint32_t row = blockIdx.x / (uint32_t)split, part = blockIdx.x % (uint32_t)split;
    const uint32_t beg = row_start[row], n_ent = row_cursor[row] - beg;
    const uint32_t stride = (uint32_t)split * kCh;
    // the workgroup's entries: chunks of kCh at part, part + split, ...;
    // thread tid holds entries c0 + tid kSPT + q
    for (int b = threadIdx.x; b < kBandBins; b += kNT) B.a.run[b] = 0;
    __syncthreads();
    constexpr int kU = 8 / kSPT;  // histogram pass: kU x kSPT loads in flight per thread
    for (uint32_t c0 = part * kCh; c0 < n_ent; c0 += kU * stride) {
        uint32_t c[kU * kSPT];
#pragma unroll
        for (int u = 0; u < kU; u++)
#pragma unroll
            for (int q = 0; q < kSPT; q++) {
                const uint32_t e = c0 + (uint32_t)u * stride + threadIdx.x * kSPT + q;
                c[u * kSPT + q] = e < n_ent ? stage_cols[beg + e] : 0u;
            }
#pragma unroll
        for (int u = 0; u < kU * kSPT; u++)
            for (uint32_t x = c[u] & 0xffffu; x < (c[u] >> 16); x++) atomicAdd(&B.a.run[x], 1u);
    }
    // the entries of the chunk after the one being expanded are in flight
    // (the first chunk's behind the run reservation's device atomics)
    uint32_t col[kSPT];
    uint64_t key[kSPT];
    auto load_chunk = [&](uint32_t c0) {
#pragma unroll
        for (int q = 0; q < kSPT; q++) {
            const uint32_t e = c0 + threadIdx.x * kSPT + q;
            col[q] = e < n_ent ? stage_cols[beg + e] : 0u;
            key[q] = e < n_ent ? stage_keys[beg + e] : 0ull;
        }
    };
    load_chunk(part * kCh);
    reserve_runs(B.a, tile_cursor + row * gx, gx);
    for (uint32_t c0 = part * kCh; c0 < n_ent; c0 += stride) {
        uint32_t cnt[kSPT], x0[kSPT];
        uint64_t k[kSPT];
#pragma unroll
        for (int q = 0; q < kSPT; q++) {
            x0[q] = col[q] & 0xffffu;
            cnt[q] = (col[q] >> 16) - x0[q];
            k[q] = key[q];
        }
        if (c0 + stride < n_ent) load_chunk(c0 + stride);
        expand_sources<false, kNT, kRound, kSPT>(B.src, B.a, cnt, k, x0, x0, pair_keys, nullptr, limit);
    }
}

template <int kNT, int kR, int kSPT>
void launch_banded(int P, const GeomView& g, const int* radii, int block, uint32_t gx, uint32_t gy, int split,
                   const ImageView& img, const BinningView& b, hipStream_t s, uint32_t n_keys,
                   const uint32_t* spec_hdr, uint32_t spec_cap, uint32_t* mirror, uint32_t mirror_token) {
    using Lds = BandLds<kNT, kR, kSPT>;
    // > 64 KiB of dynamic LDS: the attribute once per device (and variant)
    static std::atomic<int> attr[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices)
        throw std::runtime_error("launch_banded: no current device");
    if (attr[dev].load(std::memory_order_acquire) == 0) {
        if (hipFuncSetAttribute((const void*)band_stage_kernel<kNT, kR, kSPT>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(Lds)) != hipSuccess ||
            hipFuncSetAttribute((const void*)band_split_kernel<kNT, kR, kSPT>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(Lds)) != hipSuccess)
            throw std::runtime_error("launch_banded: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
        attr[dev].store(1, std::memory_order_release);
    }
    hipLaunchKernelGGL((band_stage_kernel<kNT, kR, kSPT>), dim3((P + kStageChunk - 1) / kStageChunk), dim3(kNT),
                       sizeof(Lds), s, P, g.means2D, g.depths, radii, block, gx, gy, img.band_cursor, b.scratch,
                       b.point_list, spec_hdr, spec_cap, n_keys, mirror, mirror_token);
    hipLaunchKernelGGL((band_split_kernel<kNT, kR, kSPT>), dim3(gy * split), dim3(kNT), sizeof(Lds), s, gx, split,
                       img.band_start, img.band_cursor, b.scratch, b.point_list, img.tile_cursor, b.pair_keys,
                       spec_hdr, spec_cap, n_keys);
}

void launch_duplicate(int P, const GeomView& g, const int* radii, int W, int H, int block, const ImageView& img,
                      const BinningView& b, hipStream_t s, uint32_t n_keys, const uint32_t* spec_hdr,
                      uint32_t spec_cap, uint32_t* mirror, uint32_t mirror_token) {
    if (P == 0) return;
    const uint32_t gx = (uint32_t)((W + block - 1) / block), gy = (uint32_t)((H + block - 1) / block);
    if (dup_banded((int)gx, (int)gy, block)) {
        // ~4 split workgroups per CU over the rows
        // ~4096 split workgroups in all over the rows (per tile row at config 4:
        // 62; 16 / 32 / 128 / 256 measured slower, profiles/r03p_ab_band_*.json)
        const int want = 4096;
        const int split = std::max(1, std::min(256, (want + (int)gy - 1) / (int)gy));
        if (P >= 2000000)
            launch_banded<512, 2, 2>(P, g, radii, block, gx, gy, split, img, b, s, n_keys, spec_hdr, spec_cap, mirror,
                                     mirror_token);
        else
            launch_banded<1024, 2, 1>(P, g, radii, block, gx, gy, split, img, b, s, n_keys, spec_hdr, spec_cap, mirror,
                                      mirror_token);
        return;
    }
    if (gx * gy <= (uint32_t)kLdsTiles) {
        const int chunk = bin_chunk_for(P);
        hipLaunchKernelGGL(duplicate_lds_kernel, dim3((P + chunk - 1) / chunk), dim3(kBinThreads),
                           sizeof(uint32_t) * gx * gy, s, P, chunk, g.means2D, g.depths, radii, block, gx, gy,
                           img.tile_cursor, b.pair_keys, spec_hdr, spec_cap,
                           (uint32_t)bin_slots_for(P, (int)gx, (int)gy, block), mirror, mirror_token);
        return;
    }
    hipLaunchKernelGGL(duplicate_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, g.means2D, g.depths, radii,
                       block, gx, gy, img.tile_cursor, b.pair_keys, spec_hdr, spec_cap, mirror, mirror_token);
}

// ------------------------------------------------------- launch order ---
// One workgroup: counting sort of the tiles by descending work (1024 log
// buckets, order inside a bucket arbitrary -- it only steers scheduling).
// The AMR units' heaviest-first order (the base backward takes its order from
// the forward render's work buckets instead, backward.hip).
constexpr int kOrderThreads = 1024;
constexpr int kOrderBuckets = 1024;  // one per thread: bucket b = 64 log2(work + 1), heaviest first

__global__ void __launch_bounds__(kOrderThreads) order_tiles_kernel(int T, const uint32_t* __restrict__ ranges,
                                                                    const uint32_t* __restrict__ max_contrib,
                                                                    uint32_t* __restrict__ order) {
    __shared__ uint32_t hist[kOrderBuckets];
    __shared__ uint32_t s_wave[kOrderThreads / 64 + 1];
    const int tid = threadIdx.x;
    hist[tid] = 0;
    __syncthreads();
    auto bucket = [&](int t) -> uint32_t {
        uint32_t w = ranges[2 * t + 1] - ranges[2 * t];
        if (max_contrib) w = min(w, max_contrib[t]);
        const uint32_t b = min((uint32_t)(64.0f * __log2f((float)w + 1.0f)), (uint32_t)(kOrderBuckets - 1));
        return (uint32_t)(kOrderBuckets - 1) - b;  // heaviest first
    };
    for (int t = tid; t < T; t += kOrderThreads) atomicAdd(&hist[bucket(t)], 1u);
    __syncthreads();
    uint32_t total;
    const uint32_t base = block_exclusive_scan<kOrderThreads>(hist[tid], s_wave, total);
    __syncthreads();
    hist[tid] = base;
    __syncthreads();
    for (int t = tid; t < T; t += kOrderThreads) order[atomicAdd(&hist[bucket(t)], 1u)] = (uint32_t)t;
}

void launch_order_tiles(int T, const ImageView& img, bool use_max_contrib, hipStream_t s) {
    if (T <= 0) return;
    hipLaunchKernelGGL(order_tiles_kernel, dim3(1), dim3(kOrderThreads), 0, s, T, img.ranges,
                       use_max_contrib ? img.max_contrib : nullptr, img.tile_order);
}

// (tile sorting helpers: gs_tilesort.cuh)
// Tiles with lo < n <= hi (hi <= 256 * kEmax), one 256-thread workgroup each.
template <int kEmax>
__global__ void __launch_bounds__(kSortThreads) sort_tiles_small_kernel(int lo, int hi,
                                                                         const uint32_t* __restrict__ ranges,
                                                                         const uint64_t* __restrict__ pair_keys,
                                                                         uint32_t* __restrict__ point_list) {
    __shared__ uint64_t lds[256 * kEmax];
    const int tile = blockIdx.x;
    const uint32_t beg = ranges[2 * tile], end = ranges[2 * tile + 1];
    const int n = (int)(end - beg);
    if (n <= lo || n > hi) return;
    const uint64_t* keys = pair_keys + beg;
    uint32_t* out = point_list + beg;
    if (n == 1) {
        if (threadIdx.x == 0) out[0] = (uint32_t)keys[0];
        return;
    }
    if (n <= 64) {  // one wave, shuffles only
        if (threadIdx.x < 64) sort_tile_regs<1, 1>(keys, n, out, lds);
        return;
    }
    if (kEmax == 4) {
        if (n <= 256) sort_tile_regs<1, 4>(keys, n, out, lds);
        else if (n <= 512) sort_tile_regs<2, 4>(keys, n, out, lds);
        else sort_tile_regs<4, 4>(keys, n, out, lds);
    } else {
        if (n <= 2048) sort_tile_regs<8, 4>(keys, n, out, lds);
        else sort_tile_regs<16, 4>(keys, n, out, lds);
    }
}

// Tiles with lo < n <= hi as ONE E = 4 register network over kThreads / 64
// waves (n <= 4 kThreads): the fully unrolled E <= 4 networks move partners
// with DPP / ds_swizzle / permlane swaps instead of the ds_bpermute of the
// E = 8 / 16 networks, at the price of log2(kThreads / 64) more LDS stages
// per merge.  n in (1024, 2048] -> 512 threads, (2048, 4096] -> 1024.
template <int kThreads>
__global__ void __launch_bounds__(kThreads) sort_tiles_wide_kernel(int lo, int hi, const uint32_t* __restrict__ ranges,
                                                                   const uint64_t* __restrict__ pair_keys,
                                                                   uint32_t* __restrict__ point_list) {
    __shared__ uint64_t lds[4 * kThreads];
    const int tile = blockIdx.x;
    const uint32_t beg = ranges[2 * tile], end = ranges[2 * tile + 1];
    const int n = (int)(end - beg);
    if (n <= lo || n > hi) return;
    sort_tile_regs<4, kThreads / 64>(pair_keys + beg, n, point_list + beg, lds);
}

// set_tuning("sort_algo"): 1 (default) the bucket sort (gs_tilesort.cuh), 0
// (fallback) the bitonic register networks alone (which the bucket sort also
// takes for a tile with clustered depths)
int g_sort_algo = 1;
void set_sort_algo(int v) { g_sort_algo = v; }

// kT threads, kE keys each (n <= kT kE); nb ~ n >> kBS buckets.
template <int kT, int kE, int kBS, bool kStageOut = false>
__global__ void __launch_bounds__(kT) sort_tiles_bucket_kernel(int lo, int hi, const uint32_t* __restrict__ ranges,
                                                                const uint64_t* __restrict__ pair_keys,
                                                                uint32_t* __restrict__ point_list) {
    __shared__ TileSortLds<kT, kE, kBS> L;
    const int tile = blockIdx.x;
    const uint32_t beg = ranges[2 * tile], end = ranges[2 * tile + 1];
    const int n = (int)(end - beg);
    if (n <= lo || n > hi) return;
    const uint64_t* keys = pair_keys + beg;
    uint32_t* out = point_list + beg;
    if (n == 1) {
        if (threadIdx.x == 0) out[0] = (uint32_t)keys[0];
        return;
    }
    tile_bucket_sort<kT, kE, kBS, kStageOut>(keys, n, out, L);
}

// All three bucket-sort classes in one launch of 512-thread workgroups
// (tiles of <= 2048 keys on the <512, 4, 1> path, (2048, 4096] on <512, 8, 2>
// through LDS), for grids whose tiles span the classes: one grid of T
// workgroups instead of three grids of mostly early-exiting ones (the same
// LDS and 59 vs 58 VGPRs as the largest class alone): config-4 sort_tiles
// 0.1222 -> 0.1089 ms (profiles/r05bb_ab_sort_mixed_cfg4.log).
__global__ void __launch_bounds__(512) sort_tiles_mixed_kernel(const uint32_t* __restrict__ ranges,
                                                               const uint64_t* __restrict__ pair_keys,
                                                               uint32_t* __restrict__ point_list) {
    __shared__ union {
        TileSortLds<512, 4, 1> a;
        TileSortLds<512, 8, 2> b;
    } L;
    const int tile = blockIdx.x;
    const uint32_t beg = ranges[2 * tile], end = ranges[2 * tile + 1];
    const int n = (int)(end - beg);
    if (n == 0 || n > kSmallCap) return;
    const uint64_t* keys = pair_keys + beg;
    uint32_t* out = point_list + beg;
    if (n == 1) {
        if (threadIdx.x == 0) out[0] = (uint32_t)keys[0];
        return;
    }
    if (n <= 2048) tile_bucket_sort<512, 4, 1, false>(keys, n, out, L.a);
    else tile_bucket_sort<512, 8, 2, true>(keys, n, out, L.b);
}

// Merge-path split: number of elements taken from A for the first `diag`
// outputs of merge(A[0..na), B[0..nb)); keys are unique.
__device__ __forceinline__ int merge_path(const uint64_t* A, int na, const uint64_t* B, int nb, int diag) {
    int lo = max(0, diag - nb), hi = min(diag, na);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (A[mid] < B[diag - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kLargeThreads) sort_tiles_large_kernel(const uint32_t* __restrict__ large_tiles,
                                                                          const uint32_t* __restrict__ ranges,
                                                                          uint64_t* __restrict__ pair_keys,
                                                                          uint64_t* __restrict__ scratch,
                                                                          uint32_t* __restrict__ point_list) {
    __shared__ uint64_t s[kChunk];
    const int tile = (int)large_tiles[blockIdx.x];
    const uint32_t beg = ranges[2 * tile], end = ranges[2 * tile + 1];
    const int n = (int)(end - beg);
    const int tid = threadIdx.x;
    uint64_t* src = pair_keys + beg;
    uint64_t* dst = scratch + beg;
    // 1. chunk sort in LDS, in place in src.
    for (int c0 = 0; c0 < n; c0 += kChunk) {
        const int m = min(kChunk, n - c0);
        int S = 2;
        while (S < m) S <<= 1;
        for (int i = tid; i < S; i += kLargeThreads) s[i] = i < m ? src[c0 + i] : ~0ull;
        __syncthreads();
        bitonic_lds<kLargeThreads>(s, S);
        for (int i = tid; i < m; i += kLargeThreads) src[c0 + i] = s[i];
        __syncthreads();
    }
    // 2. merge passes (src -> dst, swap).
    for (int w = kChunk; w < n; w <<= 1) {
        for (int r0 = 0; r0 < n; r0 += 2 * w) {
            const int na = min(w, n - r0);
            const int nb = max(0, min(w, n - r0 - w));
            const uint64_t* A = src + r0;
            const uint64_t* B = A + na;
            const int tot = na + nb;
            const int per = (tot + kLargeThreads - 1) / kLargeThreads;
            const int d0 = min(tot, tid * per), d1 = min(tot, d0 + per);
            if (d0 < d1) {
                int i = merge_path(A, na, B, nb, d0);
                int j = d0 - i;
                for (int d = d0; d < d1; d++) {
                    const bool takeA = (j >= nb) || (i < na && A[i] < B[j]);
                    dst[r0 + d] = takeA ? A[i++] : B[j++];
                }
            }
        }
        __syncthreads();
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    for (int i = tid; i < n; i += kLargeThreads) point_list[beg + i] = (uint32_t)src[i];
}

// The AMR region-list pass sorts its tiles of <= kAmrFusedSortMax keys
// itself (render.hip amr_region_lists_kernel kFuse) with the bucket sort
// below; with the bitonic fallback (sort_algo 0) every tile is sorted here.
bool fused_sort_on() { return g_sort_algo == 1; }

void launch_sort_tiles(int T, const ImageView& img, const BinningView& b, int max_count_host, int num_large_host,
                       hipStream_t s, int fused_max) {
    if (T == 0) return;
    if (g_sort_algo == 1) {
#define GS_BK(TH, E, BS, LO, HI, OUT)                                                                 \
    hipLaunchKernelGGL((sort_tiles_bucket_kernel<TH, E, BS, OUT>), dim3(T), dim3(TH), 0, s, LO, HI, img.ranges, \
                       b.pair_keys, b.point_list)
        // size classes (measured best at configs 2, 3 and 4 among 6 geometries,
        // profiles/r03c_ab_sort_variant_*); the (2048, 4096] class stores its
        // sorted ids through LDS, wave-contiguous (0.1616 -> 0.1225 ms at config 4;
        // the small class measured 0.0293 -> 0.0303 ms at config 2 that way and
        // keeps the direct stores, profiles/r05k_ab_sortout*.log)
        if (fused_max == 0 && max_count_host > 2048) {
            hipLaunchKernelGGL(sort_tiles_mixed_kernel, dim3(T), dim3(512), 0, s, img.ranges, b.pair_keys,
                               b.point_list);
        } else {
            if (fused_max < 1024) GS_BK(256, 4, 1, 0, 1024, false);
            if (max_count_host > 1024 && fused_max < 2048) GS_BK(512, 4, 1, 1024, 2048, false);
            if (max_count_host > 2048) GS_BK(512, 8, 2, 2048, kSmallCap, true);
        }
#undef GS_BK
        if (num_large_host > 0)
            hipLaunchKernelGGL(sort_tiles_large_kernel, dim3(num_large_host), dim3(kLargeThreads), 0, s,
                               img.large_tiles, img.ranges, b.pair_keys, b.scratch, b.point_list);
        return;
    }
    // n <= 1024 with 8 KiB of LDS; 1024 < n <= 4096 with 32 KiB (launched
    // only if such a tile exists: the forward read back the maximum count)
    hipLaunchKernelGGL(sort_tiles_small_kernel<4>, dim3(T), dim3(kSortThreads), 0, s, 0, 1024, img.ranges,
                       b.pair_keys, b.point_list);
    // (1024, 2048]: the E = 4 network over 8 waves (AMR tiles: 0.078 -> 0.073 ms
    // at config 3); (2048, 4096] stays on E = 16 over 4 waves (the 16-wave E = 4
    // network measured 0.453 -> 0.467 ms at config 4; profiles/r02f_ab_sort*)
    if (max_count_host > 1024) {
        hipLaunchKernelGGL(sort_tiles_wide_kernel<512>, dim3(T), dim3(512), 0, s, 1024, 2048, img.ranges,
                           b.pair_keys, b.point_list);
        if (max_count_host > 2048)
            hipLaunchKernelGGL(sort_tiles_small_kernel<16>, dim3(T), dim3(kSortThreads), 0, s, 2048, kSmallCap,
                               img.ranges, b.pair_keys, b.point_list);
    }
    if (num_large_host > 0)
        hipLaunchKernelGGL(sort_tiles_large_kernel, dim3(num_large_host), dim3(kLargeThreads), 0, s,
                           img.large_tiles, img.ranges, b.pair_keys, b.scratch, b.point_list);
}

// (tile << 32 | depth bits) for every sorted instance: the reference's
// binningState.point_list_keys, rebuilt for the parity accessor only.
__global__ void __launch_bounds__(256) reconstruct_keys_kernel(const uint32_t* __restrict__ ranges,
                                                               const uint32_t* __restrict__ point_list,
                                                               const float* __restrict__ depths,
                                                               uint64_t* __restrict__ keys) {
    const int tile = blockIdx.x;
    const uint32_t beg = ranges[2 * tile], end = ranges[2 * tile + 1];
    for (uint32_t i = beg + threadIdx.x; i < end; i += blockDim.x)
        keys[i] = ((uint64_t)tile << 32) | float_bits(depths[point_list[i]]);
}

void launch_reconstruct_keys(int T, const ImageView& img, const BinningView& b, const GeomView& g, uint64_t* keys,
                             hipStream_t s) {
    if (T == 0) return;
    hipLaunchKernelGGL(reconstruct_keys_kernel, dim3(T), dim3(256), 0, s, img.ranges, b.point_list, g.depths, keys);
}

}  // namespace gsamd
