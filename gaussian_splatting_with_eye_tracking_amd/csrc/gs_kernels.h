// gs_kernels.h -- host-side launchers of the gfx950 kernels (one per stage).
// Every launcher enqueues on `stream` and never synchronises; the C-ABI
// orchestrators (gs_api.cpp) own the single K read-back.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_layout.h"

namespace gsamd {

// Stage-timing events a single-kernel launcher attaches to its dispatch
// (hipExtLaunchKernelGGL) when the profiler times that stage (gs_api.cpp
// StageTimer on_dispatch); {nullptr, nullptr} otherwise.  Taking them clears
// the thread's pending pair.
struct DispatchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
DispatchEvents take_dispatch_events();

struct PreprocessArgs {
    int P, D, M;
    const float* means3D;
    const float* scales;
    float scale_modifier;
    const float* rotations;
    const float* opacities;
    const float* shs;
    const float* cov3D_precomp;
    const float* colors_precomp;
    const float* viewmatrix;
    const float* projmatrix;
    const float* cam_pos;
    int W, H;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    int block;  // tile edge in pixels (16 base, 32 AMR)
    int prefiltered;
    int store_cov3d;  // write the geometry buffer's cov3D (nothing in the path reads it back)
    int store_drgb;   // write d(rgb)/d(dir) of the SH colours for the backward (GeomView::drgb)
    // Words the launch zeroes before anything reads them (the binning's tile
    // histogram: no separate memset launch), and the value a prefiltered
    // violation stores in the header's error word (a per-call token, so that
    // word needs no zeroing either).
    uint32_t* zero_words;
    int zero_n;
    uint32_t err_token;
};

// base/cr/forward.cu:155-256 (+ the tile histogram the binning needs).
void launch_preprocess(const PreprocessArgs& a, const GeomView& g, int* radii, uint32_t* tile_count,
                       hipStream_t s);
// base/cr/rasterizer_impl.cu:54-66
void launch_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                         bool* present, hipStream_t s);

// Binning (replaces scan + duplicateWithKeys + radix sort + identifyTileRanges,
// base/cr/rasterizer_impl.cu:277-318, with identical outputs).
// hdr_mirror: device address of 16 mapped host bytes that receive header
// words 0..3 (K, error, max tile count, large tiles) when the scan finishes.
void launch_tile_scan(int T, const ImageView& img, uint32_t* hdr, hipStream_t s, uint32_t* hdr_mirror, int nslots,
                      int gx, bool banded, uint32_t mirror_token = 0);
// spec_hdr: a speculative launch into a buffer of spec_cap keys, enqueued
// before the host knows K; it does nothing when the header's K > spec_cap.
// n_keys: the instance capacity the binning buffer was carved for (K, or the
// speculative capacity); the banded duplicate never writes past it.
// mirror / mirror_token (the speculative launch): the header read-back is
// published by the duplicate's first thread instead of the tile scan.
void launch_duplicate(int P, const GeomView& g, const int* radii, int W, int H, int block, const ImageView& img,
                      const BinningView& b, hipStream_t s, uint32_t n_keys, const uint32_t* spec_hdr = nullptr,
                      uint32_t spec_cap = 0, uint32_t* mirror = nullptr, uint32_t mirror_token = 0);
// Tile grids up to kLdsTiles are binned with workgroup-private LDS histograms
// (count_tiles + chunked duplicate); larger grids use device atomics.
constexpr int kLdsTiles = 16384;
void launch_count_tiles(int P, const GeomView& g, const int* radii, int W, int H, int block, const ImageView& img,
                        hipStream_t s);
void set_sort_algo(int v);  // 0 = bitonic networks, 1 = bucket sort (default)
int bin_slots_for(int P, int gx, int gy, int block);  // sub-bucket slots of the LDS binning (P-Gaussian forward)
bool dup_banded(int gx, int gy, int block);           // the row-banded duplicate runs for this tile grid
// img.tile_order = tiles sorted by descending work (heaviest first) so the
// long tiles of a blend launch start early instead of forming its tail.
// Work = range length, or min(range length, max_contrib) if use_max_contrib.
// (The AMR units' order; the base backward takes its order from the forward
// render's work buckets.)
void launch_order_tiles(int T, const ImageView& img, bool use_max_contrib, hipStream_t s);
// fused_max: tiles of <= fused_max instances (0 or kAmrFusedSortMax) are
// left to the kernel that consumes them first -- the AMR region-list pass
// (amr_region_lists_kernel kFuse) -- which sorts its own tile.
void launch_sort_tiles(int T, const ImageView& img, const BinningView& b, int max_count_host, int num_large_host,
                       hipStream_t s, int fused_max = 0);
constexpr int kAmrFusedSortMax = 2048;
constexpr int kAmrStepsAll = GSPLAT_AMD_AMR_STEPS_1_TO_4;  // foveaStep: steps 1..4 in one launch (gs_amr_accumulate_step)
constexpr int kAmrStepsAllFill = GSPLAT_AMD_AMR_STEPS_1_TO_4_FILL;  // ... storing every pixel instead of adding
constexpr int kAmrStepsAllSplit = GSPLAT_AMD_AMR_STEPS_1_TO_4_SPLIT;  // ... into the four steps' own images
constexpr int kAmrStateAfter = 100;  // launch_fovea_levels step kAmrStateAfter + j: the level state foveaStep j leaves
bool fused_sort_on();  // the AMR region-list pass sorts its tiles of <= kAmrFusedSortMax instances itself
// (tile << 32 | depth) reconstruction of the reference's point_list_keys.
void launch_reconstruct_keys(int T, const ImageView& img, const BinningView& b, const GeomView& g, uint64_t* keys,
                             hipStream_t s);

// Blend (base/cr/forward.cu:261-374).  zero_rows: zeroed (zero_floats,
// a multiple of 4, 16-B aligned) by the same launch; returns whether it was.
// hit_codes: where the render stores its row-group hit codes (the binning
// scratch, gs_layout.h hit_codes_of; null: none).
bool launch_render_forward(int W, int H, const ImageView& img, const BinningView& b, const GeomView& g,
                           const float* features, const float* bg, float* out_color, hipStream_t s,
                           float* zero_rows = nullptr, size_t zero_floats = 0, uint8_t* hit_codes = nullptr);
// Tuning knobs (gs_set_tuning): the default or one fallback each.
void set_forward_variant(int v);
void set_backward_variant(int v);
void set_amr_variant(int v);
void set_cull(int v);  // row-group cull in the blend kernels (default on)
void set_ritnet_mfma(int v);
// Blend backward (base/cr/backward.cu:399-557) into g.grad_accum.
void launch_render_backward(int W, int H, const ImageView& img, const BinningView& b, const GeomView& g,
                            const float* colors, const float* bg, const float* dL_dpix, hipStream_t s, int K);

struct BackwardGaussArgs {
    int P, D, M;
    const float* means3D;
    const int* radii;
    const float* shs;
    const float* scales;
    const float* rotations;
    float scale_modifier;
    const float* cov3D;  // precomp or geom
    const float* viewmatrix;
    const float* projmatrix;
    const float* campos;
    float focal_x, focal_y, tan_fovx, tan_fovy;
    int has_cov_precomp;
    const float* drgb;      // the forward's d(rgb)/d(dir) [9][P] (nullptr: from the SH coefficients)
    const uint32_t* hdr;    // the geometry header (kHdrDrgb says whether drgb was written)
    int drgb_known;         // the host knows this geometry buffer's forward wrote drgb (gs_api registry)
    int nt_out = 0;         // the outputs other than dL_dsh stored with the non-temporal hint (off: +3 %)
    // outputs (every element written; no memsets needed)
    float* dL_dmean2D;
    float* dL_dconic;
    float* dL_dopacity;
    float* dL_dcolor;
    float* dL_dmean3D;
    float* dL_dcov3D;
    float* dL_dsh;
    float* dL_dscale;
    float* dL_drot;
};
// base/cr/backward.cu:144-396 fused into one per-Gaussian pass.
void launch_backward_gaussians(const BackwardGaussArgs& a, const GeomView& g, hipStream_t s);

// Data-parallel view exchange (backward.hip): per-view screen-space rows and
// the multi-view per-Gaussian backward.
constexpr int kViewRow = 10;   // words per Gaussian per view
constexpr int kCamWords = 40;  // view 16, proj 16, campos 3, W, H, tan_fovx, tan_fovy, pad
constexpr int kMaxViews = 64;  // views summed by one multi-view launch
struct MultiViewArgs {
    int P, D, M, V;
    int g0, count;                  // this launch: Gaussians [g0, g0 + count)
    const float* rows[kMaxViews];   // view v's row of Gaussian g0 ([kViewRow] words per Gaussian), summed in v order
    const float* cams[kMaxViews];   // view v's camera ([kCamWords])
    // V > kMaxViews: the same two pointer arrays in device memory (rows at
    // [0, V), cams at [V, 2V)); null otherwise
    const float* const* table;
    const float* means3D;
    const float* shs;  // nullable (colors precomputed: no SH gradient)
    const float* scales;
    const float* rotations;
    float scale_modifier;
    float* dL_dmean3D;
    float* dL_dsh;
    float* dL_dopacity;
    float* dL_dscale;
    float* dL_drot;
    float* grad_norm_accum;  // nullable: densification statistics, accumulated
    float* denom;
    float* max_radii;
    int nt = 0;  // the dL_dsh rows stored with the non-temporal hint (launcher: on, as bwd_gauss's)
};
void launch_pack_view_grads(int P, const GeomView& g, const int* radii, bool has_sh, const float* viewmatrix,
                            const float* projmatrix, const float* campos, int width, int height, float tan_fovx,
                            float tan_fovy, float* out, hipStream_t s);
void launch_multiview_backward(const MultiViewArgs& a, hipStream_t s);

// Eye-tracking front end (ritnet.hip): RITnet DenseNet2D building blocks.
void launch_ritnet_conv(int k, const float* const* in_ptr, const int* in_c, const int* in_up, int nseg, int H, int W,
                        const float* w, const float* bias, int lrelu, const float* bn_scale, const float* bn_shift,
                        float* out, hipStream_t s);
void launch_avgpool2(const float* in, int C, int H, int W, float* out, hipStream_t s);
void launch_ritnet_head(const float* in, int H, int W, const float* w, const float* bias, float* logits,
                        uint8_t* labels, hipStream_t s);
void launch_label_moments(const uint8_t* labels, int H, int W, int cls, double* out, hipStream_t s);
// AMR backward (extension): blend backward over the rendered sub-lattices,
// and the backward of render_once's interpolation.
void launch_amr_render_backward(int W, int H, int mode, const ImageView& img, const BinningView& b,
                                const GeomView& g, const float* colors, const float* bg, const float* dL_dpix,
                                hipStream_t s);
void launch_amr_interp_fold(int W, int H, const ImageView& img, const float* g_in, float* g_out, hipStream_t s);
// Fovea-driven AMR levels (amr.hip), applied to the step-0 levels in place.
void launch_fovea_override(int W, int H, const ImageView& img, int nf, const float* cx, const float* cy,
                           const float* radius, int min_level, int replace, hipStream_t s);
// Eye-image preprocessing (eye_preprocess.hip): gamma table, CLAHE, normalise, transpose.
void launch_eye_preprocess(const uint8_t* gray, int H, int W, const uint8_t* gamma, int tiles_x, int tiles_y,
                           int limit, float* luts, float* out, hipStream_t s);

// AMR (amr/cr/rasterizer_impl.cu:181-243, amr/cr/forward.cu:261-648).
// zero_image (optional): foveaStep 0's zero image, written by the same launch
void launch_amr_levels(int T, const ImageView& img, hipStream_t s, float* zero_image = nullptr, size_t zero_floats = 0);
// The 8x8-region sub-lists and per-instance blend records (variant 4).
// fused_sort: tiles of <= kAmrFusedSortMax instances arrive unsorted
// (launch_sort_tiles fused_max) and are sorted by the launch itself.
void launch_amr_region_lists(int W, int H, const ImageView& img, const BinningView& b, const AmrBinningView& ab,
                             const GeomView& g, const float* features, int K, hipStream_t s, bool fused_sort = false);
extern int g_amr_variant;
// the other gs_set_tuning choices (read by gs_get_tuning)
extern int g_fwd_variant, g_bwd_variant, g_sort_algo, g_cull, g_ritnet_mfma;
void launch_fovea_levels(int step, int T, const ImageView& img, hipStream_t s, int P = 0, int* zero_radii = nullptr);
void launch_amr_render(int W, int H, const ImageView& img, const uint32_t* levels, const uint32_t* levels_last,
                       const BinningView& b, const AmrBinningView& ab, const GeomView& g, const float* features,
                       const float* bg, float* out_color, int foveaStep, hipStream_t s, bool fused = false, int P = 0,
                       int* zero_radii = nullptr, int accumulate = 0);  // 1 add, 2 split (render.hip)
void launch_amr_interpolate(int W, int H, const ImageView& img, const uint32_t* levels, const uint32_t* levels_last,
                            float* out_color, int foveaStep, const float* out_color_precomp, hipStream_t s);

// simple-knn (knn/simple_knn.cu).
size_t knn_workspace_bytes(int P);
void launch_knn(int P, const float* points, float* mean_dists, char* workspace, hipStream_t s);

// Generic stable LSD radix sort of (u32 key, u32 value) pairs.
size_t radix_sort_u32_workspace(int n);
void radix_sort_pairs_u32(int n, const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in,
                          uint32_t* vals_out, int end_bit, char* workspace, hipStream_t s);

// Training loss of train.py:91-93 (loss.hip): grad <- dloss/dimg, out3 <- {loss, l1, ssim}.
size_t l1_ssim_workspace_bytes(int C, int H, int W);
void launch_l1_ssim(const float* img, const float* gt, int C, int H, int W, float lambda, float* grad, float* out3,
                    float* workspace, hipStream_t s);
// torch.optim.Adam step over a flat buffer with per-segment learning rates.
void launch_adam(float* p, const float* g, float* m, float* v, long long N, int nseg, const long long* seg_end,
                 const double* lr, const long long* step, double beta1, double beta2, double eps, hipStream_t s);
// train.py:111-113 densification statistics for the visible Gaussians.
void launch_densify_stats(int P, const int* radii, const float* grad_means2D, int g_stride, float* accum,
                          float* denom, float* max_radii, hipStream_t s);
// scene/gaussian_model.py:93-113 activations from raw segments, and their backward.
void launch_activate(int P, int M, const float* dc, const float* rest, const float* opacity_raw,
                     const float* scaling_raw, const float* rotation_raw, float* shs, float* opacity, float* scales,
                     float* rotations, hipStream_t s);
void launch_activation_backward(int P, int M, int accumulate, const float* d_shs, const float* d_opac,
                                const float* d_scales, const float* d_rot, const float* d_means3D,
                                const float* opacity_raw, const float* scaling_raw, const float* rotation_raw,
                                float* g_xyz, float* g_dc, float* g_rest, float* g_opacity, float* g_scaling,
                                float* g_rotation, hipStream_t s);

}  // namespace gsamd
