// gs_layout.h -- how the three opaque byte buffers of the rasterizer are carved.
//
// The reference hands three uint8 tensors (geomBuffer / binningBuffer /
// imgBuffer) between forward, backward and AMR steps and carves them with
// GeometryState/ImageState/BinningState::fromChunk
// (base/cr/rasterizer_impl.cu:155-194, amr/cr/rasterizer_impl.cu:245-292).
// The contract is "opaque, round-trips unchanged" (SURVEY §8(a) A13), so this
// build chooses its own MI355X layout: structure-of-arrays, every array
// 256-B aligned (a wave's 64 x 4 B access is one 256-B segment), and
//   * geom   (per Gaussian, P):  depths, radii, means2D (float2), conic_opacity
//     (float4), rgb[3], cov3D[6], clamped (1 B bitmask), tiles_touched, and a
//     64-B-row gradient accumulator grad_accum[P][16] for the backward blend
//     (one 64-B memory-side atomic request per (tile, Gaussian) pair);
//   * image  (per pixel N and per tile T): accum_alpha (final T), n_contrib,
//     ranges (uint2), tile_count, tile_cursor, max_contrib, AMR levels;
//   * binning (per instance K): point_list, the (depth|idx) sort keys, and a
//     scratch copy for the large-tile merge sort.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>  // float4
#include "gsplat_amd.h"  // GSPLAT_AMD_GRAD_ROW

namespace gsamd {

constexpr size_t kAlign = 256;
// floats per grad_accum row: the blend's 9 sums, or the AMR forward's blend
// record (three float4s); 48 B keeps every row 16-B aligned for float4 access
// (64-B rows cost the forward's zeroing and the Gaussian backward's read 33 %
// more bytes: 390 MB each per launch at config 4)
constexpr int kGradRow = 12;
static_assert(kGradRow == GSPLAT_AMD_GRAD_ROW, "the public layout constant");

// Header words (geom buffer, device side).
enum HdrWord : int {
    kHdrNumRendered = 0,  // K
    kHdrError = 1,        // nonzero: a kernel raised (e.g. prefiltered violation)
    kHdrMaxTileCount = 2,
    kHdrNumLargeTiles = 3,
    kHdrP = 4,
    kHdrT = 5,
    kHdrHitCodes = 6,     // != 0: where the base forward render stored exact row-group hit codes (hit_codes_of)
    kHdrDrgb = 7,         // 1: the preprocess stored d(rgb)/d(view dir) of every visible Gaussian (GeomView::drgb)
    kHdrWords = 64,
};

inline size_t align_up(size_t x, size_t a = kAlign) { return (x + a - 1) & ~(a - 1); }

template <typename T>
inline T* carve(char* base, size_t& off, size_t count) {
    off = align_up(off);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += sizeof(T) * count;
    return p;
}

struct GeomView {
    uint32_t* hdr;
    float* depths;
    int* radii;
    float* means2D;        // [P][2]
    float* conic_opacity;  // [P][4]
    float* rgb;            // [P][3]
    float* cov3D;          // [P][6]
    uint8_t* clamped;      // [P] bit c = channel c clamped
    float* drgb;           // [P][12] d(rgb)/d(dir): (x, y, z) x (r, g, b) + 3 pad, SH colours, visible Gaussians
    uint32_t* tiles_touched;
    float* grad_accum;  // [P][kGradRow]
    float* amr_rows;    // [P][16] AMR buffers only: the AMR forward's per-Gaussian blend row (below)
};

// base is 256-B aligned by the caller (torch allocations are).
// The optional tail -- d(rgb)/d(dir) rows (written when the forward stores
// them for an SH backward, header flag kHdrDrgb) and cov3D (written only on
// request, set_tuning("store_cov3d")) -- comes last: a forward that writes
// neither sizes its buffer without it (tail = false: 72 B per Gaussian less,
// ~440 MB at 6.1M Gaussians); the pointers are carved either way and read
// only when the header / the request says they were written.
// AMR buffers (amr: 32-px tiles) always carry the tail and then amr_rows: one
// 64-B row per Gaussian -- (x, y, r, g), the log2(e)-scaled conic + opacity,
// (b, raw conic) and a zero pad -- which the AMR preprocess writes and
// foveaStep 0's region-list pass gathers, one aligned 64-B sector per
// instance (48-B rows straddled two sectors in most rows: 286 MB of traffic
// per launch for ~106 MB of rows at config 3, profiles/r04zf_cfg3_pmc_summary.json).
inline size_t carve_geom(char* base, size_t P, GeomView* v, bool tail = true, bool amr = false) {
    size_t off = 0;
    GeomView g;
    g.hdr = carve<uint32_t>(base, off, kHdrWords);
    g.depths = carve<float>(base, off, P);
    g.radii = carve<int>(base, off, P);
    g.means2D = carve<float>(base, off, 2 * P);
    g.conic_opacity = carve<float>(base, off, 4 * P);
    g.rgb = carve<float>(base, off, 3 * P);
    g.clamped = carve<uint8_t>(base, off, P);
    g.tiles_touched = carve<uint32_t>(base, off, P);
    g.grad_accum = carve<float>(base, off, (size_t)kGradRow * P);
    const size_t head = align_up(off);
    g.drgb = carve<float>(base, off, 12 * P);
    g.cov3D = carve<float>(base, off, 6 * P);
    const size_t full = align_up(off);
    g.amr_rows = carve<float>(base, off, 16 * P);
    if (v) *v = g;
    return amr ? align_up(off) : tail ? full : head;
}

struct ImageView {
    float* accum_alpha;   // [N]
    uint32_t* n_contrib;  // [N]
    uint32_t* ranges;     // [T][2]
    uint32_t* tile_count;  // [kBinSlots][T] per-slot counts; after the tile scan [0..T) holds the totals
                           // (= n_intersections for AMR)
    uint32_t* tile_cursor; // [kBinSlots][T] sub-bucket cursors
    uint32_t* max_contrib;
    uint32_t* levels;          // tile_AMR_levels
    uint32_t* levels_last;     // tile_AMR_levels_last
    uint32_t* levels_current;  // tile_AMR_levels_current
    uint32_t* pv;              // [4] percentile values (AMR)
    uint32_t* large_tiles;     // [T] list of tiles needing the large sort
    uint32_t* tile_order;      // [4T] tiles (or backward units: tile | row-group set << 28) by descending
                               // blend work (launch order)
    uint32_t* quad_count;      // [T][4] AMR: entries of each 16x16 quadrant's sub-list
    uint32_t* region_count;    // [T][16] AMR: entries of each 8x8 region's sub-list
    uint32_t* tile_done;       // [T] AMR steps: finished (tile, quadrant) units, mod 4
    uint32_t* bucket_count;    // [kOrderBuckets64 = 256] tiles per work bucket (base forward render appends)
    uint32_t* bucket_list;     // [kOrderBuckets64][T] the tiles of each bucket, in append order
    uint32_t* band_start;      // [<= T] banded duplicate: first instance of each band's tile range
    uint32_t* band_cursor;     // [<= T] banded duplicate: staging cursor of each band
};
constexpr int kOrderBuckets64 = 256;  // (name kept: the bucket count of the backward order)
// Each tile's bucket is split into kBinSlots sub-buckets, one per
// binning-workgroup slot (blockIdx % kBinSlots = the XCD the round-robin
// dispatch puts the workgroup on): the runs that concurrently running chunks
// of one XCD append to a tile are then adjacent in memory, and that XCD's L2
// merges their scattered 8-B key stores into whole lines before write-back
// (instead of one 32-B write granule per key).  The per-tile sort makes the
// order inside a tile exact either way.
constexpr int kBinSlots = 8;

// tile: 16 (base) or 32 (AMR); the backward's work buckets (256 x T words,
// filled by the base forward render) are carved for the base layout only.
inline size_t carve_image(char* base, size_t N, size_t T, ImageView* v, int tile) {
    size_t off = 0;
    ImageView g;
    g.accum_alpha = carve<float>(base, off, N);
    g.n_contrib = carve<uint32_t>(base, off, N);
    g.ranges = carve<uint32_t>(base, off, 2 * T);
    g.tile_count = carve<uint32_t>(base, off, (size_t)kBinSlots * T);
    g.tile_cursor = carve<uint32_t>(base, off, (size_t)kBinSlots * T);
    g.max_contrib = carve<uint32_t>(base, off, T);
    g.levels = carve<uint32_t>(base, off, T);
    g.levels_last = carve<uint32_t>(base, off, T);
    g.levels_current = carve<uint32_t>(base, off, T);
    g.pv = carve<uint32_t>(base, off, 4);
    g.large_tiles = carve<uint32_t>(base, off, T);
    g.tile_order = carve<uint32_t>(base, off, 4 * T);
    g.quad_count = carve<uint32_t>(base, off, 4 * T);
    g.region_count = carve<uint32_t>(base, off, 16 * T);
    g.tile_done = carve<uint32_t>(base, off, T);
    g.band_start = carve<uint32_t>(base, off, T);
    g.band_cursor = carve<uint32_t>(base, off, T);
    g.bucket_count = nullptr;
    g.bucket_list = nullptr;
    if (tile != 32) {
        g.bucket_count = carve<uint32_t>(base, off, kOrderBuckets64);
        g.bucket_list = carve<uint32_t>(base, off, (size_t)kOrderBuckets64 * T);
    }
    if (v) *v = g;
    return align_up(off);
}

struct BinningView {
    uint32_t* point_list;  // [K]
    uint64_t* pair_keys;   // [K]  (depth_bits << 32 | gaussian idx), grouped by tile
    uint64_t* scratch;     // [K]  merge-sort ping-pong
};

// Base forward: the render's exact row-group hit code of every sorted
// instance (1 B; bit r: row group r of the tile has a pixel that blended it),
// which the backward uses as its row masks, lives in the forward's binning
// scratch: the merge-sort ping-pong, dead once the duplicate and the
// large-tile merges are done, and nothing after the sort reads it.  (Only the
// AMR region-list pass sorts tiles during a render, from pair_keys,
// render.hip amr_region_lists_kernel kFuse; the base render writes codes
// alone.)  The header word kHdrHitCodes says
// where: 0 = no codes, else 1 + (byte offset from point_list) / kAlign.  The
// offset cannot come from K: a speculative forward carves the buffer for a
// capacity >= K (its scratch further out), the backward carves it for K; both
// leave point_list at 0.
inline uint32_t hit_codes_word(const uint32_t* point_list, const uint8_t* codes) {
    return codes ? 1u + (uint32_t)((size_t)(codes - reinterpret_cast<const uint8_t*>(point_list)) / kAlign) : 0u;
}
__host__ __device__ inline const uint8_t* hit_codes_of(const uint32_t* point_list, uint32_t word) {
    return word ? reinterpret_cast<const uint8_t*>(point_list) + (size_t)(word - 1u) * kAlign : nullptr;
}

// AMR (32-px tiles): once the tile lists are sorted, pair_keys and scratch
// (>= 16 K bytes, contiguous up to alignment) are dead; they hold the
// quadrant sub-lists instead: tile t with range [beg, beg + n) keeps the
// list of its quadrant q (16x16 pixels) at quad_lists(b) + 4 beg + q n --
// positions i in [0, n) of the tile's entries that can reach the quadrant,
// ascending (render.hip amr_quad_lists_kernel).
inline uint32_t* quad_lists(const BinningView& b) { return reinterpret_cast<uint32_t*>(b.pair_keys); }

// AMR binning extension (32-px tiles only; appended after the base arrays,
// whose offsets it leaves unchanged).  Filled once per frame by foveaStep 0
// (render.hip amr_region_lists_kernel), read by every progressive step:
//   * the blend record of every instance in sorted tile-list order, so a
//     step's loads are tile-local and coalesced instead of three random
//     per-Gaussian gathers behind a point_list gather: rec_a = (mean x,
//     mean y, r, g), rec_b = the log2(e)-scaled conic and opacity
//     (gs_blend.cuh splat_coef), rec_c = b;
//   * region lists: tile t with range [beg, beg + n) keeps, for each of its
//     16 regions of 8x8 pixels (g = 4 row + col), the positions i in [0, n)
//     of the entries that can reach the region, ascending, at
//     region_lists + 16 beg + g n.
struct AmrBinningView {
    float4* rec_a;
    float4* rec_b;
    float* rec_c;
    uint32_t* region_lists;
};

inline size_t carve_binning(char* base, size_t K, BinningView* v, AmrBinningView* amr = nullptr,
                            bool with_amr = false) {
    size_t off = 0;
    BinningView g;
    g.point_list = carve<uint32_t>(base, off, K);
    g.pair_keys = carve<uint64_t>(base, off, K);
    g.scratch = carve<uint64_t>(base, off, K);
    if (v) *v = g;
    if (amr || with_amr) {
        AmrBinningView a;
        a.rec_a = carve<float4>(base, off, K);
        a.rec_b = carve<float4>(base, off, K);
        a.rec_c = carve<float>(base, off, K);
        a.region_lists = carve<uint32_t>(base, off, 16 * K);
        if (amr) *amr = a;
    }
    // Unpadded end: strictly increasing in K (>= 8 B per instance), so the
    // caller can recover K from the buffer size (gs_binning_count_of_bytes,
    // gs_amr_binning_count_of_bytes) without a device read-back.
    return off;
}

}  // namespace gsamd
