/*
 * gsplat_amd.h -- C ABI of the MI355X (gfx950) Gaussian rasterizer.
 *
 * Plain pointers and sizes only (no torch types).  Every pointer argument
 * that refers to per-Gaussian / per-pixel data is a DEVICE pointer (HBM);
 * scalars are host values.  `stream` is a hipStream_t (NULL = legacy
 * default stream).  Every call is asynchronous on `stream` except where a
 * comment says it reads the instance count K back to the host (the
 * reference performs that same blocking read, base/cr/rasterizer_impl.cu:281).
 *
 * Return value: >= 0 on success (the forward calls return num_rendered = K),
 * negative on error; gs_last_error() then returns a message (thread-local).
 *
 * Buffer contract (SURVEY §8(b) "Ownership"): the three opaque byte buffers
 * (geometry / binning / image) are allocated by the CALLER through
 * gs_resize_fn callbacks, exactly like the reference's resizeFunctional
 * (base/rasterize_points.cu:27-33), and must be handed back unchanged to the
 * backward call or to the next AMR step.  Their internal layout is this
 * library's own (see DESIGN.md "Data layout in HBM").
 */
#ifndef GSPLAT_AMD_H
#define GSPLAT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSPLAT_AMD_ABI_VERSION 7  /* 4: drgb / cov3D moved to an optional tail of the geometry buffer;
                                     5: grad_accum rows of GSPLAT_AMD_GRAD_ROW = 12 floats (were 16);
                                     6: AMR geometry buffers end with 64-B blend rows (amr_rows);
                                     7: the base forward's hit codes in the binning scratch, located by
                                        header word 6 (1 + byte offset from point_list / 256) */
/* floats per grad_accum row of the geometry buffer (gs_geom_view.grad_accum) */
#define GSPLAT_AMD_GRAD_ROW 12

/* Resize the caller-owned byte buffer `ctx` to `nbytes` and return its
 * (device, >=256-B aligned) base pointer, or NULL on failure.
 * Mirrors std::function<char*(size_t)> resizeFunctional
 * (base/rasterize_points.cu:27-33). */
typedef char* (*gs_resize_fn)(void* ctx, size_t nbytes);

typedef struct {
    gs_resize_fn resize;
    void* ctx;
} gs_buffer;

int gs_abi_version(void);
/* Digest of the sources + compiler flags this library was built from
 * (build.py source_digest(); not part of any reference interface: the
 * benchmark and smoke test refuse a library whose digest differs from the
 * tree's). */
const char* gs_build_digest(void);
const char* gs_last_error(void);

/* Replaces CudaRasterizer::Rasterizer::forward
 * (base/cr/rasterizer.h:35-59, base/cr/rasterizer_impl.cu:198-336).
 * Reads K back to the host once.  The binning buffer may be sized for more
 * than K entries: the duplicate is launched before K reaches the host into a
 * buffer sized from the previous call's K (+1/8), re-sized for K only when K
 * exceeds that; only its first 4K bytes (point_list) are read afterwards, by
 * gs_rasterizer_backward with R = the returned K.  Its size is therefore not
 * gs_binning_bytes(K) in general (gs_binning_count_of_bytes gives the
 * capacity, not K). */
int gs_rasterizer_forward(gs_buffer geometry, gs_buffer binning, gs_buffer image, int P, int D, int M,
                          const float* background, int width, int height, const float* means3D, const float* shs,
                          const float* colors_precomp, const float* opacities, const float* scales,
                          float scale_modifier, const float* rotations, const float* cov3D_precomp,
                          const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                          float tan_fovy, int prefiltered, float* out_color, int* radii, int debug, void* stream);

/* Replaces CudaRasterizer::Rasterizer::backward
 * (base/cr/rasterizer.h:61-84, base/cr/rasterizer_impl.cu:340-434).
 * Unlike the reference, every output element is written (the reference
 * relies on 9 zero-filled tensors, base/rasterize_points.cu:151-159), so
 * the outputs may be uninitialised memory.  dL_dconic is [P][4] (a 2x2). */
int gs_rasterizer_backward(int P, int D, int M, int R, const float* background, int width, int height,
                           const float* means3D, const float* shs, const float* colors_precomp, const float* scales,
                           float scale_modifier, const float* rotations, const float* cov3D_precomp,
                           const float* viewmatrix, const float* projmatrix, const float* campos, float tan_fovx,
                           float tan_fovy, const int* radii, char* geom_buffer, char* binning_buffer,
                           char* img_buffer, const float* dL_dpix, float* dL_dmean2D, float* dL_dconic,
                           float* dL_dopacity, float* dL_dcolor, float* dL_dmean3D, float* dL_dcov3D,
                           float* dL_dsh, float* dL_dscale, float* dL_drot, int debug, void* stream);

/* Data-parallel training (no reference counterpart: the
 * reference trains one view per step on one GPU, train.py:67-125).
 *
 * Stage 1 of the backward of one view: the blend backward only
 * (base/cr/backward.cu:399-557), written as a VIEW RECORD of P * 10 + 40
 * floats: per Gaussian dL_dcolor[3], dL_dmean2D.xy[2], dL_dconic (x, y,
 * w)[3], dL_dopacity, and word 9 = radius | clamped_bits << 24 (bit
 * pattern; 0 = not visible in this view); then the camera: viewmatrix[16],
 * projmatrix[16], campos[3], width, height, tan_fovx, tan_fovy, 0.  The
 * ranks exchange (all-gather) these records instead of parameter
 * gradients. */
int gs_rasterizer_backward_view_grads(int P, int R, const float* background, int width, int height,
                                      const float* colors_precomp, const float* viewmatrix, const float* projmatrix,
                                      const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                                      char* geom_buffer, char* binning_buffer, char* img_buffer,
                                      const float* dL_dpix, float* out_record, int debug, void* stream);

/* Stage 2: the per-Gaussian backward (base/cr/backward.cu:20-396) of V views
 * at once, summed over the views in view order; views = V stage-1 records
 * back to back (device).  Writes every element of dL_dmeans3D[P][3],
 * dL_dsh[P][M][3] (if shs), dL_dopacity[P], dL_dscales[P][3],
 * dL_drotations[P][4].  If grad_norm_accum is non-null, the densification
 * statistics of every view (train.py:111-113) are accumulated into
 * grad_norm_accum[P], denom[P], max_radii[P] (float), view by view. */
int gs_backward_gaussians_multiview(int P, int D, int M, int V, const float* views, const float* means3D,
                                    const float* shs, const float* scales, const float* rotations,
                                    float scale_modifier, float* dL_dmeans3D, float* dL_dsh, float* dL_dopacity,
                                    float* dL_dscales, float* dL_drotations, float* grad_norm_accum, float* denom,
                                    float* max_radii, void* stream);

/* The same for Gaussians [g0, g0 + count) with the rows and cameras of the V
 * views anywhere in device memory: view v's row of Gaussian g0 + i at
 * rows + v * row_view_stride + 10 i, its camera at cams + v * cam_stride.
 * Lets the exchange run chunk by chunk (the all-gather of chunk c + 1
 * overlapping the backward of chunk c). Outputs and statistics are indexed
 * by the global Gaussian index. */
int gs_backward_gaussians_multiview_range(int P, int g0, int count, int D, int M, int V, const float* rows,
                                          size_t row_view_stride, const float* cams, size_t cam_stride,
                                          const float* means3D, const float* shs, const float* scales,
                                          const float* rotations, float scale_modifier, float* dL_dmeans3D,
                                          float* dL_dsh, float* dL_dopacity, float* dL_dscales,
                                          float* dL_drotations, float* grad_norm_accum, float* denom,
                                          float* max_radii, void* stream);

/* The same over V views whose rows need not share a stride: rows[v]
 * (host array of device pointers) is view v's row of Gaussian g0, cams[v]
 * its 40-word camera; views are summed in v order.  Lets every all-gathered
 * piece stay in its own contiguous [world, n] buffer (no flatten copies).
 * Any V >= 1: up to 64 views the pointers travel as kernel arguments, beyond
 * that in a stream-ordered device table (one host synchronisation for its
 * upload); the sums are the same either way. */
int gs_backward_gaussians_multiview_views(int P, int g0, int count, int D, int M, int V, const float* const* rows,
                                          const float* const* cams, const float* means3D, const float* shs,
                                          const float* scales, const float* rotations, float scale_modifier,
                                          float* dL_dmeans3D, float* dL_dsh, float* dL_dopacity, float* dL_dscales,
                                          float* dL_drotations, float* grad_norm_accum, float* denom,
                                          float* max_radii, void* stream);

/* Eye-tracking front end (RITnet/densenet.py:17-144,
 * track_render.py:50-97).  Activations are [C][H][W] float32 planes.
 *
 * One RITnet convolution (3x3 padding 1, or 1x1) to 32 output channels over a
 * virtual channel concatenation of nseg <= 3 inputs: in[i] holds
 * in_channels[i] planes, read through nearest 2x upsampling when
 * in_upsample[i] (then it is height/2 x width/2).  weight is [Cin][k*k][32]
 * (the torch [32][Cin][k][k] tensor repacked), bias [32]; epilogue:
 * LeakyReLU(0.01) if leaky_relu, then y * bn_scale + bn_shift if given
 * (eval BatchNorm). Replaces nn.Conv2d / torch.cat / F.interpolate /
 * nn.LeakyReLU / nn.BatchNorm2d of DenseNet2D_down_block and _up_block. */
int gs_ritnet_conv(int ksize, int nseg, const float* const* in, const int* in_channels, const int* in_upsample,
                   int height, int width, const float* weight, const float* bias, int leaky_relu, const float* bn_scale,
                   const float* bn_shift, float* out, void* stream);
/* nn.AvgPool2d(2) (densenet.py:26) over [channels][height][width]. */
int gs_avgpool2(const float* in, int channels, int height, int width, float* out, void* stream);
/* out_conv1 (32 -> 4, 1x1; weight [32][4]) + get_predictions' argmax
 * (RITnet/utils.py:186-190): labels [H][W] uint8, logits [4][H][W] if non-null. */
int gs_ritnet_head(const float* in, int height, int width, const float* weight, const float* bias, float* logits,
                   uint8_t* labels, void* stream);
/* out3 (device, f64) = {sum x, sum y, count} over the pixels labelled `label`
 * (the pupil centroid of the segmentation). */
int gs_label_moments(const uint8_t* labels, int height, int width, int label, double* out3, void* stream);
/* Eye-image preprocessing (track_render.py:69-80): gray [height][width]
 * uint8 -> gamma_lut (256 bytes: uint8(255 * (i/255)^0.8), track_render.py:72)
 * -> OpenCV 8-bit CLAHE (clip_limit, tiles_x x tiles_y grid;
 * cv2.createCLAHE(1.5, (8, 8)).apply, track_render.py:75-76) -> ToTensor +
 * Normalize([0.5], [0.5]) (RITnet/dataset.py:35-37) -> out [width][height]
 * float32, the transposed image RITnet is fed (track_render.py:80).
 * luts: scratch of tiles_x * tiles_y * 256 floats.  height and width must be
 * multiples of the grid (error otherwise). */
int gs_eye_preprocess(const uint8_t* gray, int height, int width, const uint8_t* gamma_lut, double clip_limit,
                      int tiles_x, int tiles_y, float* luts, float* out, void* stream);

/* Replaces CudaRasterizer::Rasterizer::markVisible
 * (base/cr/rasterizer.h:24-29, base/cr/rasterizer_impl.cu:141-153). */
int gs_rasterizer_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                               uint8_t* present, void* stream);

/* Replaces the AMR CudaRasterizer::Rasterizer::forward
 * (amr/cr/rasterizer.h:35-73, amr/cr/rasterizer_impl.cu:296-694).
 * foveaStep 0: preprocess + binning + levels, no render (blank image);
 * 1..4: progressive step on the *_precomp buffers (image buffer mutated in
 * place), the geometry/binning/image callbacks are not called;
 * <0: one-shot render of every level (render_once).
 * Every pixel of out_color is written (0 where the call renders nothing, as
 * the reference's zero-filled output), and steps 1..4 write radii = 0 (the
 * reference's zero radii), so neither need be initialised.
 * Reads K back to the host once (both branches, as the reference does). */
int gs_amr_rasterizer_forward(gs_buffer geometry, gs_buffer binning, gs_buffer image, int P, int D, int M,
                              const float* background, int width, int height, const float* means3D,
                              const float* shs, const float* colors_precomp, const float* opacities,
                              const float* scales, float scale_modifier, const float* rotations,
                              const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                              const float* cam_pos, float tan_fovx, float tan_fovy, int prefiltered, int foveaStep,
                              const float* out_color_precomp, char* geom_buffer_precomp,
                              char* binning_buffer_precomp, char* image_buffer_precomp, float* out_color, int* radii,
                              int interpolate_image, int debug, void* stream);

/* gs_amr_rasterizer_forward with num_rendered_hint: for foveaStep >= 1, a
 * hint >= 0 is taken as K (the caller recovered it from the binning buffer's
 * size with gs_amr_binning_count_of_bytes) and the device read-back of K is
 * skipped, so the progressive steps run without host synchronisation; -1
 * reads it back like the reference. */
int gs_amr_rasterizer_forward_ex(gs_buffer geometry, gs_buffer binning, gs_buffer image, int P, int D, int M,
                                 const float* background, int width, int height, const float* means3D,
                                 const float* shs, const float* colors_precomp, const float* opacities,
                                 const float* scales, float scale_modifier, const float* rotations,
                                 const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                                 const float* cam_pos, float tan_fovx, float tan_fovy, int prefiltered,
                                 int foveaStep, const float* out_color_precomp, char* geom_buffer_precomp,
                                 char* binning_buffer_precomp, char* image_buffer_precomp, float* out_color,
                                 int* radii, int interpolate_image, int debug, int num_rendered_hint, void* stream);

/* The 5-step driver's progressive step fused with its image sum: the
 * caller's `rendered_image_k = rasterize(foveaStep k, ...)` followed by
 * `out_color_precomp = out_color_precomp + rendered_image_k`
 * (gaussian_renderer_amr/__init__.py:295-341, 384-427, 470-510, 553-594;
 * interpolate_image false).  `accum` (3 x height x width floats, the running
 * sum, step 0's zero image at first) is updated in place: every pixel this
 * step renders gets accum + (C + T bg), the same fp32 add, and the rest keep
 * their value (+ 0 in the reference) -- bit-identical to the reference's sum.
 * Buffers, radii (zeros written), num_rendered_hint and return value as
 * gs_amr_rasterizer_forward_ex at foveaStep >= 1.  Needs the default AMR
 * variant (gs_set_tuning("amr_variant") 4).
 * foveaStep = GSPLAT_AMD_AMR_STEPS_1_TO_4: steps 1, 2, 3 and 4 in order in ONE
 * launch -- each (tile, quadrant) unit renders the rounds 1..min(level, 4)
 * those four calls would give it, one after another, and leaves accum, final
 * T, n_contrib, radii and the buffers' level state exactly as the four calls
 * do (each pixel belongs to one round, so every rendered pixel gets one
 * accum + (C + T bg) either way).
 * foveaStep = GSPLAT_AMD_AMR_STEPS_1_TO_4_FILL: the same launch for a frame
 * that is step 0's image left unfilled (gs_set_thread_option
 * "amr_step0_unfilled" before that step-0 call): every pixel of accum is
 * stored -- C + T bg where a round renders, 0 elsewhere: the bits of 0 + the
 * four steps' images -- instead of added to. */
#define GSPLAT_AMD_AMR_STEPS_1_TO_4 14
#define GSPLAT_AMD_AMR_STEPS_1_TO_4_FILL 15
/* foveaStep = GSPLAT_AMD_AMR_STEPS_1_TO_4_SPLIT: the same one launch writing
 * the four steps' OWN images -- accum is 4 x 3 x height x width floats, image
 * k - 1 the one foveaStep k alone returns (its round's pixels, zeros
 * elsewhere), every element written -- and radii 4 x P zeros (each step's
 * zero radii).  Final T, n_contrib and the level state are left as after
 * step 4.  The torch binding uses it to serve the reference's literal
 * step-by-step sequence (torch_ext.cpp, speculative steps). */
#define GSPLAT_AMD_AMR_STEPS_1_TO_4_SPLIT 16
int gs_amr_accumulate_step(int P, const float* background, int width, int height, const float* colors_precomp,
                           int foveaStep, char* geom_buffer_precomp, char* binning_buffer_precomp,
                           char* image_buffer_precomp, float* accum, int* radii, int debug, int num_rendered_hint,
                           void* stream);

/* Takes the level state (tile_AMR_levels_last / _current,
 * amr/cr/rasterizer_impl.cu:208-243) of an AMR image buffer from the one
 * foveaStep 1..4 leave (as GSPLAT_AMD_AMR_STEPS_1_TO_4* leave it) back to the
 * one foveaStep 1..`step` leave (step in 1..4): with c = current, last =
 * min(c, step - 1), current = min(c, step).  Lets a caller that ran steps
 * 1..4 at once go back to the literal sequence at step + 1. */
int gs_amr_set_step_state(char* image_buffer, size_t image_buffer_bytes, int width, int height, int step,
                          void* stream);

/* Replaces SimpleKNN::knn (knn/simple_knn.h:16-19, knn/simple_knn.cu:185-221)
 * behind simple_knn._C.distCUDA2.  `scratch` is resized to the workspace
 * size; no host synchronisation. */
/* The AMR (foveated) backward -- an extension: the reference's
 * amr/cr/rasterizer.h:69-98 / rasterizer_impl.cu:698-796 is unreachable
 * (SURVEY §8(a) B-AMR bwd).
 * Gradients of the image one AMR forward call produced, on the buffers it
 * returned: foveaStep k in 1..4 -> round k of the tiles whose level >= k;
 * foveaStep < 0 -> render_once (rounds <= level), through the interpolation
 * when interpolate_image (then dL_dpix_scratch: 3 * width * height floats).
 * Outputs and their layout as gs_rasterizer_backward (all written). */
int gs_amr_rasterizer_backward(int P, int D, int M, int R, const float* background, int width, int height,
                               const float* means3D, const float* shs, const float* colors_precomp,
                               const float* scales, float scale_modifier, const float* rotations,
                               const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                               const float* campos, float tan_fovx, float tan_fovy, const int* radii,
                               char* geom_buffer, char* binning_buffer, char* img_buffer, int foveaStep,
                               int interpolate_image, const float* dL_dpix, float* dL_dpix_scratch,
                               float* dL_dmean2D, float* dL_dconic, float* dL_dopacity, float* dL_dcolor,
                               float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale, float* dL_drot,
                               int debug, void* stream);

/* Fovea-driven AMR levels -- an extension beyond parity.
 * The reference builds foveaCenters [4][2] / foveaRadii [4]
 * (gaussian_renderer_amr/__init__.py:98-106) but never passes them on, and
 * leaves "if outside the current fovea, set to same as last step" as a TODO
 * (:244).  Called between foveaStep 0 and the steps 1..4 on the image
 * buffer foveaStep 0 returned (levels mutated in place): F(t) = the largest
 * k <= nfovea such that tile t's pixel rectangle meets the discs
 * (centres_xy[2j], centres_xy[2j+1], radii[j]) for all j < k;
 * replace = 0: level = min(level, max(F, min_level)); replace = 1: level =
 * max(F, min_level).  centres_xy / radii are host arrays; image_buffer_bytes
 * is checked against the layout of width x height. */
int gs_amr_fovea_levels(char* image_buffer, size_t image_buffer_bytes, int width, int height, int nfovea, const float* centres_xy,
                        const float* radii, int min_level, int replace, void* stream);
int gs_simple_knn(int P, const float* points, float* mean_dists, gs_buffer scratch, void* stream);

/* Training loss of the reference (train.py:91-93, utils/loss_utils.py:17-63):
 *   loss = (1 - lambda_dssim) * mean|image - gt| + lambda_dssim * (1 - SSIM(image, gt))
 * image, gt: [C][H][W] float32 (device).  Writes grad = dloss/dimage
 * ([C][H][W]) and out3 = {loss, l1, ssim} (device); one fused pass plus a
 * fixed-order reduction (deterministic); no host synchronisation. */
int gs_l1_ssim_loss(const float* image, const float* gt, int C, int H, int W, float lambda_dssim, float* grad,
                    float* out3, gs_buffer workspace, void* stream);

/* One torch.optim.Adam step (scene/gaussian_model.py:154-163: per-group
 * learning rates, betas (0.9, 0.999), eps 1e-15) over a flat f32 buffer of n
 * parameters split into nseg <= 8 segments [seg_end[i-1], seg_end[i]) with
 * learning rate lr[i] and 1-based step count step[i] after this update
 * (0 = the segment has no gradient this iteration and is left untouched, as
 * torch skips a parameter whose .grad is None).  Element-wise in torch's
 * operation order; one pass over p, g, m, v. */
int gs_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, long long n, int nseg,
                 const long long* seg_end, const double* lr, const long long* step, double beta1, double beta2, double eps,
                 void* stream);

/* Densification statistics of train.py:111-113 and
 * scene/gaussian_model.py:405-407 for the Gaussians with radii > 0:
 * max_radii2D = max(max_radii2D, radii), xyz_gradient_accum +=
 * ||grad_means2D[:2]|| (rows of grad_stride floats), denom += 1. */
int gs_densify_stats(int P, const int* radii, const float* grad_means2D, int grad_stride, float* xyz_gradient_accum,
                     float* denom, float* max_radii2D, void* stream);

/* The rasterizer inputs from the raw parameters (scene/gaussian_model.py:
 * 93-113): shs [P][M][3] = cat(features_dc [P][1][3], features_rest
 * [P][M-1][3]), opacities = sigmoid(opacity_raw), scales = exp(scaling_raw),
 * rotations = rotation_raw / max(|rotation_raw|, 1e-12). */
int gs_activate_gaussians(int P, int M, const float* features_dc, const float* features_rest, const float* opacity_raw,
                          const float* scaling_raw, const float* rotation_raw, float* shs, float* opacities,
                          float* scales, float* rotations, void* stream);
/* Backward of gs_activate_gaussians (the gradients torch autograd would give
 * the raw parameters) plus dL/dxyz = dL/dmeans3D, stored into (accumulate =
 * 0) or added to (accumulate = 1) the raw-parameter gradient arrays. */
int gs_activation_backward(int P, int M, int accumulate, const float* dL_dshs, const float* dL_dopacities,
                           const float* dL_dscales, const float* dL_drotations, const float* dL_dmeans3D,
                           const float* opacity_raw, const float* scaling_raw, const float* rotation_raw,
                           float* grad_xyz, float* grad_features_dc, float* grad_features_rest, float* grad_opacity,
                           float* grad_scaling, float* grad_rotation, void* stream);

/* ------------------------------------------------ parity / debug accessors
 * The reference exposes its internal buffers only in the AMR-debug variant
 * (ParseBuffers, amr-debug/rasterize_points.cu:37-61).  These views let the
 * tests compare every intermediate with the oracle. */
typedef struct {
    uint32_t* hdr; /* [64]: [0]=K, [1]=error flag, [2]=max tile count, [3]=#large tiles */
    float* depths;
    int* radii;
    float* means2D;       /* [P][2] */
    float* conic_opacity; /* [P][4] */
    float* rgb;           /* [P][3] */
    float* cov3D;         /* [P][6], in the optional tail (written on request only) -- ABI 4 */
    uint8_t* clamped;     /* [P] bit c = channel c clamped */
    float* drgb;          /* [P][12] d(rgb)/d(view dir) of the SH colours, (x, y, z) x (r, g, b) + 3 pad (hdr[7] = 1: written), in the optional tail -- ABI 3 / 4 */
    uint32_t* tiles_touched;
    float* grad_accum; /* [P][GSPLAT_AMD_GRAD_ROW] */
    float* amr_rows;   /* [P][16] AMR blend rows after the tail (AMR geometry buffers only) -- ABI 6 */
} gs_geom_view;

typedef struct {
    float* accum_alpha; /* final T, [N] */
    uint32_t* n_contrib;
    uint32_t* ranges; /* [T][2] */
    uint32_t* tile_count;
    uint32_t* tile_cursor;
    uint32_t* max_contrib;
    uint32_t* levels;
    uint32_t* levels_last;
    uint32_t* levels_current;
    uint32_t* pv; /* [4] */
    uint32_t* large_tiles;
    uint32_t* tile_order; /* [4T] blend launch order (descending work; backward units) */
    uint32_t* quad_count; /* [T][4] AMR quadrant sub-list lengths */
    uint32_t* region_count; /* [T][16] AMR 8x8-region sub-list lengths */
    uint32_t* tile_done; /* [T] AMR steps: finished units per tile, mod 4 */
    uint32_t* bucket_count; /* [256] base forward: tiles per work bucket (heaviest first); NULL for tile 32 */
    uint32_t* bucket_list;  /* [256][T] base forward: the tiles of each bucket; NULL for tile 32 */
    uint32_t* band_start;   /* [<= T] banded duplicate: first instance of each band (row of 2^k tiles) */
    uint32_t* band_cursor;  /* [<= T] banded duplicate: staging cursor of each band */
} gs_image_view;

typedef struct {
    uint32_t* point_list;
    uint64_t* pair_keys;
    uint64_t* scratch;
} gs_binning_view;

/* Upper bound: the geometry buffer with its optional tail (d(rgb)/d(dir)
 * rows and cov3D, csrc/gs_layout.h); a forward that writes neither asks its
 * resize callback for 72 B per Gaussian less, and gs_geom_view_of's drgb /
 * cov3D pointers are then past the end of that buffer (read them only when
 * header word kHdrDrgb / the store_cov3d request says they were written). */
size_t gs_geom_bytes(int P);
/* An AMR (32-px) forward's geometry buffer: the tail always, then the 64-B
 * AMR blend rows (gs_geom_view.amr_rows) -- ABI 6. */
size_t gs_amr_geom_bytes(int P);
size_t gs_image_bytes(int width, int height, int tile);
size_t gs_binning_bytes(int K);
/* Inverse of gs_binning_bytes (exact; -1 if nbytes is not a binning size). */
int gs_binning_count_of_bytes(size_t nbytes);
/* The AMR (32-px tile) binning buffer: the base arrays at the same offsets,
 * followed by the per-instance blend records and the 8x8-region sub-lists
 * foveaStep 0 builds for the progressive steps (csrc/gs_layout.h). */
size_t gs_amr_binning_bytes(int K);
int gs_amr_binning_count_of_bytes(size_t nbytes);
size_t gs_knn_workspace_bytes(int P);
int gs_geom_view_of(char* base, int P, gs_geom_view* out);
int gs_image_view_of(char* base, int width, int height, int tile, gs_image_view* out);
int gs_binning_view_of(char* base, int K, gs_binning_view* out);

/* The reference's binningState.point_list_keys (tile << 32 | depth bits),
 * rebuilt from point_list + ranges + depths into keys_out[K] (device). */
int gs_reconstruct_keys(char* geom_buffer, char* binning_buffer, char* img_buffer, int P, int K, int width,
                        int height, int tile, uint64_t* keys_out, void* stream);

/* ---------------------------------------------------- per-stage timing
 * When enabled, every stage records a pair of hipEvents on its launch stream;
 * gs_profile_read() waits for them and returns the accumulated milliseconds
 * and launch counts per stage (names from gs_profile_stage_name).  Used by
 * bench.py for the live per-kernel roofline (cross-checked with rocprofv3). */
void gs_profile_enable(int on);
/* Restrict the timing to the stages whose bit (1 << stage index) is set
 * (default: all).  Each timed stage adds two event records per launch, so
 * the headline timing records only the kernel its roofline is quoted on. */
void gs_profile_set_mask(unsigned mask);
/* Process-wide performance choices for A/B measurements, each the default
 * or one fallback (every pair gives the same results): "fwd_variant" (0 = one
 * wave x 4 px/lane predicate form; else the default 4 waves x 1 px/lane select
 * form), "bwd_variant" (0 = predicate form with LDS-row sums; else the
 * default select form with staged sums), "amr_variant" (0 = full-list AMR
 * blocks; else the default 8x8 region sub-lists), "sort_algo" (0 = bitonic
 * networks only; 1 = per-tile bucket sort, the default), "cull" (1 = skip
 * Gaussians whose alpha >= 1/255 ellipse misses a 16x4 row group, the
 * default; 0 only to verify that the cull is exact), "hdr_mirror" (2 = the
 * polled K read-back, the default; 0 = copy + event), "spec_dup" (1 = the
 * speculative duplicate before the K read-back, the default), "ritnet_mfma"
 * (1 = matrix-core convolutions, the default; 0 = SGPR-weight FMA kernel).
 * Returns 0, or -1 for an unknown key. */
int gs_set_tuning(const char* key, int value);
/* The current value of a gs_set_tuning key into *value (0 = the fallback
 * variant); -1 for an unknown key. */
int gs_get_tuning(const char* key, int* value);
/* Per-call options of the calling thread's forwards (thread-local): "fwd_zero"
 * (1 = the forward render zeroes the backward's accumulator rows, default),
 * "sh_drgb" (1 = the preprocess stores d(rgb)/d(view dir) for the SH
 * backward, default), "store_cov3d" (1 = the forward also writes the geometry
 * buffer's cov3D, which nothing in the path reads back -- for buffer-level
 * parity checks; default 0), "fwd_no_grad" (one-shot: the next forward on this
 * thread needs no backward), "amr_step0_unfilled" (one-shot: the next AMR
 * forward, if at foveaStep 0, leaves its image unwritten for a
 * GSPLAT_AMD_AMR_STEPS_1_TO_4_FILL launch to fill).  Returns 0, or -1 for an
 * unknown key. */
int gs_set_thread_option(const char* key, int value);
int gs_profile_stage_count(void);
const char* gs_profile_stage_name(int i);
void gs_profile_read(double* total_ms, long* counts, int reset);

#ifdef __cplusplus
}
#endif

#endif /* GSPLAT_AMD_H */
