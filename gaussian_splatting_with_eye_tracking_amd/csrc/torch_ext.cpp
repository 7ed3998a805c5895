// torch_ext.cpp -- PyTorch binding (`_C`) over the C ABI in include/gsplat_amd.h.
//
// Mirrors the reference bindings one for one:
//   base/rasterize_points.cu:35-217 + base/ext.cpp:15-19
//     rasterize_gaussians / rasterize_gaussians_backward / mark_visible
//   amr/rasterize_points.cu:65-202 + amr/ext.cpp
//     amr_rasterize_gaussians (exported to diff_gaussian_rasterization_amr._C
//     as rasterize_gaussians)
//   knn/spatial.cu:14-24 + knn/ext.cpp
//     distCUDA2
// Same argument order, same return tuples, same "empty tensor == nullptr"
// convention (SURVEY §8(b) "Ownership"), same AT_ERROR on a bad means3D.
// Differences: work is enqueued on torch's *current* HIP stream of the
// input's device (the reference uses the legacy default stream and the
// current device), and the library writes every output element, so outputs
// are allocated with torch::empty instead of zero-filled.
#include <torch/extension.h>

#include <c10/hip/HIPStream.h>

#include <string>
#include <tuple>
#include <vector>

#include "gsplat_amd.h"

namespace {

using torch::Tensor;

char* resize_tensor(void* ctx, size_t n) {
    auto* t = static_cast<Tensor*>(ctx);
    t->resize_({(int64_t)n});
    return reinterpret_cast<char*>(t->data_ptr());
}

gs_buffer buf_of(Tensor& t) { return gs_buffer{&resize_tensor, &t}; }

void* stream_of(const Tensor& t) {
    return static_cast<void*>(c10::hip::getCurrentHIPStream(t.device().index()).stream());
}

void check(int rc, const char* what) {
    if (rc < 0) TORCH_CHECK(false, what, ": ", gs_last_error());
}

void require_device(const Tensor& t, const char* name) {
    if (t.numel() == 0) return;
    TORCH_CHECK(t.is_cuda(), name, " must be a HIP device tensor (the MI355X rasterizer has no CPU path)");
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
}

// A non-empty operand must live on `ref`'s device with the given dtype and
// hold `numel` elements (numel < 0: any): a host or other-GPU pointer, or a
// short array, would otherwise reach a kernel as a raw pointer and fault the
// GPU instead of raising here.
void require_like(const Tensor& t, const Tensor& ref, const char* name, int64_t numel = -1,
                  torch::ScalarType dt = torch::kFloat32) {
    if (t.numel() == 0) return;
    TORCH_CHECK(t.is_cuda() && t.device() == ref.device(), name, " must be on ", ref.device(),
                " (the MI355X rasterizer has no CPU path)");
    TORCH_CHECK(t.scalar_type() == dt, name, " must be ", c10::toString(dt));
    TORCH_CHECK(numel < 0 || t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
}

// The per-Gaussian and camera operands of a forward / backward call.
void check_operands(const Tensor& means3D, int P, const Tensor& bg, const Tensor& colors, const Tensor& opacity,
                    const Tensor& scales, const Tensor& rotations, const Tensor& cov3D_precomp,
                    const Tensor& viewmatrix, const Tensor& projmatrix, const Tensor& sh, const Tensor& campos) {
    require_like(bg, means3D, "bg", 3);
    require_like(colors, means3D, "colors_precomp", 3LL * P);
    require_like(opacity, means3D, "opacities", P);
    require_like(scales, means3D, "scales", 3LL * P);
    require_like(rotations, means3D, "rotations", 4LL * P);
    require_like(cov3D_precomp, means3D, "cov3D_precomp", 6LL * P);
    require_like(viewmatrix, means3D, "viewmatrix", 16);
    require_like(projmatrix, means3D, "projmatrix", 16);
    require_like(campos, means3D, "campos", 3);
    if (sh.numel()) {
        TORCH_CHECK(sh.dim() == 3 && sh.size(0) == P && sh.size(2) == 3 && sh.size(1) >= 1 && sh.size(1) <= 16,
                    "sh must be [P, M, 3] with 1 <= M <= 16");
        require_like(sh, means3D, "sh");
    }
}

// Empty tensor -> nullptr (rasterize_points.cu: `.contiguous().data<float>()` of an empty tensor).
const float* fptr(const Tensor& t) { return t.numel() ? t.data_ptr<float>() : nullptr; }
float* fptr_mut(Tensor& t) { return t.numel() ? t.data_ptr<float>() : nullptr; }

// Speculative AMR steps.  The reference's foveated caller
// (gaussian_renderer_amr/__init__.py:183-594) calls foveaStep 1, 2, 3, 4 one
// after another on step 0's buffers, each call returning its own full image
// that the caller adds up in torch.  Step k's image depends only on those
// buffers (levels, lists, records), the background and colors_precomp -- not
// on anything the caller does in between -- so step 1 renders the rounds of
// all four steps in ONE launch (GSPLAT_AMD_AMR_STEPS_1_TO_4_SPLIT) into four
// images and returns the first; steps 2..4 return the others without a
// launch.  Four launches' tails become one.  A step is served from the
// speculation only if it is the next step on the same buffers, none of
// whose torch version counters moved (apply_fovea_levels bumps the image
// buffer's), with the same background / colours tensors and versions, size,
// stream and no interpolation or debug; anything else is a miss: the image
// buffer's level state (left as after step 4 by the one launch) is set back
// to the state after the last step served (gs_amr_set_step_state) and the
// step runs as usual.  Final T and n_contrib are those of every round from
// step 1 on (each pixel belongs to one round; the rounds' values are the
// same either way).  _C.set_amr_speculation(False) turns it off.
struct SpecSteps {
    const void* g = nullptr;
    const void* b = nullptr;
    const void* im = nullptr;
    int64_t vg = 0, vb = 0, vim = 0, vbg = 0, vcol = 0;
    const void* bg = nullptr;
    const void* col = nullptr;
    int W = 0, H = 0, P = 0, K = 0, next = 0;  // next: the step served next (2..4); 0 = nothing cached
    size_t im_bytes = 0;
    void* stream = nullptr;
    Tensor images, radii;  // [4, 3, H, W], [4, P]
    void clear() {
        next = 0;
        images = Tensor();
        radii = Tensor();
        g = b = im = bg = col = nullptr;
    }
};
thread_local SpecSteps t_spec;
thread_local bool t_spec_on = true;

int64_t version_of(const Tensor& t) { return t.defined() && t.numel() ? (int64_t)t._version() : -1; }

std::tuple<int, Tensor, Tensor, Tensor, Tensor, Tensor> rasterize_impl(
    bool amr, const Tensor& background, const Tensor& means3D_in, const Tensor& colors_in, const Tensor& opacity_in,
    const Tensor& scales_in, const Tensor& rotations_in, float scale_modifier, const Tensor& cov3D_precomp_in,
    const Tensor& viewmatrix_in, const Tensor& projmatrix_in, float tan_fovx, float tan_fovy, int image_height,
    int image_width, const Tensor& sh_in, int degree, const Tensor& campos_in, bool prefiltered, int foveaStep,
    const Tensor& out_color_precomp_in, const Tensor& geom_pre, const Tensor& bin_pre, const Tensor& img_pre,
    bool interpolate_image, bool debug) {
    if (means3D_in.ndimension() != 2 || means3D_in.size(1) != 3) {
        AT_ERROR("means3D must have dimensions (num_points, 3)");
    }
    const int P = (int)means3D_in.size(0);
    const int H = image_height;
    const int W = image_width;
    const at::OptionalDeviceGuard guard(device_of(means3D_in));
    require_device(means3D_in, "means3D");
    auto float_opts = means3D_in.options().dtype(torch::kFloat32);
    // both forwards write every pixel (the AMR one zeros where it renders nothing)
    Tensor out_color = P == 0 ? torch::zeros({3, H, W}, float_opts) : torch::empty({3, H, W}, float_opts);
    // (the AMR steps >= 1 write their zero radii in the fovea-levels launch)
    Tensor radii = P == 0 ? torch::zeros({P}, means3D_in.options().dtype(torch::kInt32))
                          : torch::empty({P}, means3D_in.options().dtype(torch::kInt32));
    auto byte_opts = means3D_in.options().dtype(torch::kByte);
    Tensor geomBuffer = torch::empty({0}, byte_opts);
    Tensor binningBuffer = torch::empty({0}, byte_opts);
    Tensor imgBuffer = torch::empty({0}, byte_opts);
    int rendered = 0;
    if (P != 0) {
        const Tensor bg = background.contiguous(), means3D = means3D_in.contiguous(), colors = colors_in.contiguous(),
                     opacity = opacity_in.contiguous(), scales = scales_in.contiguous(),
                     rotations = rotations_in.contiguous(), cov3D_precomp = cov3D_precomp_in.contiguous(),
                     viewmatrix = viewmatrix_in.contiguous(), projmatrix = projmatrix_in.contiguous(),
                     sh = sh_in.contiguous(), campos = campos_in.contiguous();
        check_operands(means3D, P, bg, colors, opacity, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, sh,
                       campos);
        const int M = sh.size(0) != 0 ? (int)sh.size(1) : 0;
        void* stream = stream_of(means3D);
        if (!amr) {
            rendered = gs_rasterizer_forward(buf_of(geomBuffer), buf_of(binningBuffer), buf_of(imgBuffer), P, degree, M,
                                             fptr(bg), W, H, fptr(means3D), fptr(sh), fptr(colors), fptr(opacity),
                                             fptr(scales), scale_modifier, fptr(rotations), fptr(cov3D_precomp),
                                             fptr(viewmatrix), fptr(projmatrix), fptr(campos), tan_fovx, tan_fovy,
                                             prefiltered, out_color.data_ptr<float>(), radii.data_ptr<int>(), debug,
                                             stream);
            check(rendered, "rasterize_gaussians");
        } else {
            const Tensor pre = out_color_precomp_in.contiguous();
            require_like(pre, means3D, "out_color_precomp", 3LL * H * W);
            for (const Tensor* bt : {&geom_pre, &bin_pre, &img_pre}) require_like(*bt, means3D, "precomp buffer", -1, torch::kByte);
            Tensor g = geom_pre, b = bin_pre, im = img_pre;
            // K of the precomputed buffers from the binning buffer's size (no sync)
            const int hint = foveaStep >= 1 ? gs_amr_binning_count_of_bytes((size_t)b.numel()) : -1;
            SpecSteps& sp = t_spec;
            const bool same_bufs = sp.next != 0 && g.numel() && im.numel() && sp.g == g.data_ptr() &&
                                   sp.im == im.data_ptr() && sp.b == (b.numel() ? b.data_ptr() : nullptr);
            if (foveaStep >= 2 && foveaStep <= 4 && same_bufs) {
                if (sp.next == foveaStep && !interpolate_image && !debug && sp.vg == version_of(g) &&
                    sp.vb == version_of(b) && sp.vim == version_of(im) && sp.bg == bg.data_ptr() &&
                    sp.vbg == version_of(background) && sp.col == (colors.numel() ? colors.data_ptr() : nullptr) &&
                    sp.vcol == version_of(colors_in) && sp.W == W && sp.H == H && sp.P == P && sp.stream == stream) {
                    Tensor img_k = sp.images[foveaStep - 1], rad_k = sp.radii[foveaStep - 1];
                    const int K = sp.K;
                    if (foveaStep == 4) sp.clear();
                    else sp.next = foveaStep + 1;
                    return std::make_tuple(K, img_k, rad_k, geom_pre, bin_pre, img_pre);
                }
                // a miss on the speculated buffers: back to the state after the last step served
                check(gs_amr_set_step_state(reinterpret_cast<char*>(im.data_ptr()), (size_t)im.numel(), W, H,
                                            sp.next - 1, stream),
                      "amr speculation (level state)");
                sp.clear();
            } else if (foveaStep <= 1) {
                sp.clear();  // a new frame (or a new step 1): nothing cached survives it
            }
            int amr_variant = 0;
            check(gs_get_tuning("amr_variant", &amr_variant), "get_tuning");
            if (foveaStep == 1 && t_spec_on && !interpolate_image && !debug && amr_variant == 4 && g.numel() &&
                im.numel()) {
                Tensor imgs = torch::empty({4, 3, H, W}, float_opts);
                Tensor rads = torch::empty({4, P}, means3D_in.options().dtype(torch::kInt32));
                rendered = gs_amr_accumulate_step(P, fptr(bg), W, H, fptr(colors), GSPLAT_AMD_AMR_STEPS_1_TO_4_SPLIT,
                                                  reinterpret_cast<char*>(g.data_ptr()),
                                                  b.numel() ? reinterpret_cast<char*>(b.data_ptr()) : nullptr,
                                                  reinterpret_cast<char*>(im.data_ptr()), imgs.data_ptr<float>(),
                                                  rads.data_ptr<int>(), 0, hint, stream);
                check(rendered, "rasterize_gaussians (AMR, speculative steps 1..4)");
                sp.g = g.data_ptr();
                sp.b = b.numel() ? b.data_ptr() : nullptr;
                sp.im = im.data_ptr();
                sp.vg = version_of(g);
                sp.vb = version_of(b);
                sp.vim = version_of(im);
                sp.bg = bg.data_ptr();
                sp.vbg = version_of(background);
                sp.col = colors.numel() ? colors.data_ptr() : nullptr;
                sp.vcol = version_of(colors_in);
                sp.W = W;
                sp.H = H;
                sp.P = P;
                sp.K = rendered;
                sp.stream = stream;
                sp.images = imgs;
                sp.radii = rads;
                sp.next = 2;
                return std::make_tuple(rendered, imgs[0], rads[0], geom_pre, bin_pre, img_pre);
            }
            rendered = gs_amr_rasterizer_forward_ex(
                buf_of(geomBuffer), buf_of(binningBuffer), buf_of(imgBuffer), P, degree, M, fptr(bg), W, H,
                fptr(means3D), fptr(sh), fptr(colors), fptr(opacity), fptr(scales), scale_modifier, fptr(rotations),
                fptr(cov3D_precomp), fptr(viewmatrix), fptr(projmatrix), fptr(campos), tan_fovx, tan_fovy, prefiltered,
                foveaStep, fptr(pre), g.numel() ? reinterpret_cast<char*>(g.data_ptr()) : nullptr,
                b.numel() ? reinterpret_cast<char*>(b.data_ptr()) : nullptr,
                im.numel() ? reinterpret_cast<char*>(im.data_ptr()) : nullptr, out_color.data_ptr<float>(),
                radii.data_ptr<int>(), interpolate_image, debug, hint, stream);
            check(rendered, "rasterize_gaussians (AMR)");
        }
    }
    if (amr && foveaStep > 0)  // amr/rasterize_points.cu:182-190: hand the precomputed buffers back
        return std::make_tuple(rendered, out_color, radii, geom_pre, bin_pre, img_pre);
    return std::make_tuple(rendered, out_color, radii, geomBuffer, binningBuffer, imgBuffer);
}

// base/rasterize_points.cu:35-115
std::tuple<int, Tensor, Tensor, Tensor, Tensor, Tensor> RasterizeGaussians(
    const Tensor& background, const Tensor& means3D, const Tensor& colors, const Tensor& opacity,
    const Tensor& scales, const Tensor& rotations, const float scale_modifier, const Tensor& cov3D_precomp,
    const Tensor& viewmatrix, const Tensor& projmatrix, const float tan_fovx, const float tan_fovy,
    const int image_height, const int image_width, const Tensor& sh, const int degree, const Tensor& campos,
    const bool prefiltered, const bool debug) {
    Tensor none;
    auto e = torch::empty({0});
    return rasterize_impl(false, background, means3D, colors, opacity, scales, rotations, scale_modifier,
                          cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh,
                          degree, campos, prefiltered, -1, e, e, e, e, false, debug);
}

// amr/rasterize_points.cu:65-202
std::tuple<int, Tensor, Tensor, Tensor, Tensor, Tensor> AMRRasterizeGaussians(
    const Tensor& background, const Tensor& means3D, const Tensor& colors, const Tensor& opacity,
    const Tensor& scales, const Tensor& rotations, const float scale_modifier, const Tensor& cov3D_precomp,
    const Tensor& viewmatrix, const Tensor& projmatrix, const float tan_fovx, const float tan_fovy,
    const int image_height, const int image_width, const Tensor& sh, const int degree, const Tensor& campos,
    const bool prefiltered, const int foveaStep, const Tensor& out_color_precomp, const Tensor& geomBuffer_precomp,
    const Tensor& binningBuffer_precomp, const Tensor& imageBuffer_precomp, const bool interpolate_image,
    const bool debug) {
    return rasterize_impl(true, background, means3D, colors, opacity, scales, rotations, scale_modifier,
                          cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh,
                          degree, campos, prefiltered, foveaStep, out_color_precomp, geomBuffer_precomp,
                          binningBuffer_precomp, imageBuffer_precomp, interpolate_image, debug);
}

// The 5-step driver's step k with its image sum fused (gs_amr_accumulate_step):
// accum += rendered_image_k in place; returns the step's zero radii.
Tensor AmrAccumulateStep(const Tensor& background, const Tensor& colors_in, int image_height, int image_width,
                         int P, int foveaStep, Tensor& accum, const Tensor& geom, const Tensor& bin,
                         const Tensor& img, bool debug) {
    TORCH_CHECK(accum.is_cuda() && accum.scalar_type() == torch::kFloat32 && accum.is_contiguous() &&
                    accum.numel() == 3LL * image_height * image_width,
                "accum must be a contiguous float32 [3, H, W] device tensor");
    const at::OptionalDeviceGuard guard(device_of(accum));
    const Tensor bg = background.contiguous(), colors = colors_in.contiguous();
    require_like(bg, accum, "bg", 3);
    require_like(colors, accum, "colors_precomp", 3LL * P);
    for (const Tensor* bt : {&geom, &bin, &img}) require_like(*bt, accum, "precomp buffer", -1, torch::kByte);
    TORCH_CHECK(geom.numel() && img.numel(), "amr_accumulate_step needs the buffers returned by foveaStep 0");
    Tensor radii = torch::empty({P}, accum.options().dtype(torch::kInt32));
    if (P == 0) return radii;
    const int hint = gs_amr_binning_count_of_bytes((size_t)bin.numel());
    check(gs_amr_accumulate_step(P, fptr(bg), image_width, image_height, fptr(colors), foveaStep,
                                 reinterpret_cast<char*>(geom.data_ptr()),
                                 bin.numel() ? reinterpret_cast<char*>(bin.data_ptr()) : nullptr,
                                 reinterpret_cast<char*>(img.data_ptr()), accum.data_ptr<float>(), radii.data_ptr<int>(),
                                 debug ? 1 : 0, hint, stream_of(accum)),
          "amr_accumulate_step");
    return radii;
}

// base/rasterize_points.cu:117-196
using Grads8 = std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor>;

// amr_step 0: the base backward; != 0: the AMR (foveated) backward of
// foveaStep amr_step (< 0: render_once, with `interpolate`).
Grads8 BackwardImpl(int amr_step, bool interpolate, const Tensor& background, const Tensor& means3D_in,
                    const Tensor& radii_in, const Tensor& colors_in, const Tensor& scales_in,
                    const Tensor& rotations_in, const float scale_modifier, const Tensor& cov3D_precomp_in,
                    const Tensor& viewmatrix_in, const Tensor& projmatrix_in, const float tan_fovx,
                    const float tan_fovy, const Tensor& dL_dout_color_in, const Tensor& sh_in, const int degree,
                    const Tensor& campos_in, const Tensor& geomBuffer, const int R, const Tensor& binningBuffer,
                    const Tensor& imageBuffer, const bool debug, const bool lean) {
    const int P = (int)means3D_in.size(0);
    const int H = (int)dL_dout_color_in.size(1);
    const int W = (int)dL_dout_color_in.size(2);
    const int M = sh_in.size(0) != 0 ? (int)sh_in.size(1) : 0;
    const at::OptionalDeviceGuard guard(device_of(means3D_in));
    auto opts = means3D_in.options();
    // dL_dconic is never returned (base/rasterize_points.cu:185-196): not
    // computed into memory at all.  lean (the autograd wrappers): the colour /
    // covariance gradients only when their precomputed input was given --
    // otherwise autograd drops them -- as empty tensors.
    const bool want_colors = !lean || colors_in.numel() != 0;
    const bool want_cov3D = !lean || cov3D_precomp_in.numel() != 0;
    Tensor dL_dmeans3D = torch::empty({P, 3}, opts);
    Tensor dL_dmeans2D = torch::empty({P, 3}, opts);
    Tensor dL_dcolors = want_colors ? torch::empty({P, 3}, opts) : torch::empty({0}, opts);
    Tensor dL_dopacity = torch::empty({P, 1}, opts);
    Tensor dL_dcov3D = want_cov3D ? torch::empty({P, 6}, opts) : torch::empty({0}, opts);
    Tensor dL_dsh = torch::empty({P, M, 3}, opts);
    Tensor dL_dscales = torch::empty({P, 3}, opts);
    Tensor dL_drotations = torch::empty({P, 4}, opts);
    if (P != 0) {
        const Tensor bg = background.contiguous(), means3D = means3D_in.contiguous(), radii = radii_in.contiguous(),
                     colors = colors_in.contiguous(), scales = scales_in.contiguous(),
                     rotations = rotations_in.contiguous(), cov3D_precomp = cov3D_precomp_in.contiguous(),
                     viewmatrix = viewmatrix_in.contiguous(), projmatrix = projmatrix_in.contiguous(),
                     dL_dout = dL_dout_color_in.contiguous(), sh = sh_in.contiguous(), campos = campos_in.contiguous();
        require_device(means3D, "means3D");
        require_like(dL_dout, means3D, "dL_dout_color", 3LL * H * W);
        TORCH_CHECK(dL_dout.dim() == 3 && dL_dout.size(0) == 3, "dL_dout_color must be [3, H, W]");
        // (AMR steps >= 1 pass no radii: the geometry buffer keeps step 0's)
        TORCH_CHECK(radii.numel() == P || (amr_step != 0 && radii.numel() == 0), "radii must have P elements");
        require_like(radii, means3D, "radii", P, torch::kInt32);
        const Tensor no_opacity = torch::empty({0}, opts);
        check_operands(means3D, P, bg, colors, no_opacity, scales, rotations, cov3D_precomp, viewmatrix,
                       projmatrix, sh, campos);
        for (const Tensor* bt : {&geomBuffer, &binningBuffer, &imageBuffer})
            require_like(*bt, means3D, "geometry / binning / image buffer", -1, torch::kByte);
        int rc;
        if (amr_step == 0) {
            rc = gs_rasterizer_backward(
                P, degree, M, R, fptr(bg), W, H, fptr(means3D), fptr(sh), fptr(colors), fptr(scales), scale_modifier,
                fptr(rotations), fptr(cov3D_precomp), fptr(viewmatrix), fptr(projmatrix), fptr(campos), tan_fovx,
                tan_fovy, radii.data_ptr<int>(), reinterpret_cast<char*>(geomBuffer.data_ptr()),
                reinterpret_cast<char*>(binningBuffer.data_ptr()), reinterpret_cast<char*>(imageBuffer.data_ptr()),
                fptr(dL_dout), fptr_mut(dL_dmeans2D), nullptr, fptr_mut(dL_dopacity),
                want_colors ? fptr_mut(dL_dcolors) : nullptr, fptr_mut(dL_dmeans3D),
                want_cov3D ? fptr_mut(dL_dcov3D) : nullptr, fptr_mut(dL_dsh),
                fptr_mut(dL_dscales), fptr_mut(dL_drotations), debug, stream_of(means3D));
        } else {
            TORCH_CHECK(imageBuffer.numel() > 0, "the AMR backward needs the image buffer of the forward");
            Tensor scratch = interpolate ? torch::empty_like(dL_dout) : torch::empty({0}, opts);
            rc = gs_amr_rasterizer_backward(
                P, degree, M, R, fptr(bg), W, H, fptr(means3D), fptr(sh), fptr(colors), fptr(scales), scale_modifier,
                fptr(rotations), fptr(cov3D_precomp), fptr(viewmatrix), fptr(projmatrix), fptr(campos), tan_fovx,
                tan_fovy, radii.data_ptr<int>(), reinterpret_cast<char*>(geomBuffer.data_ptr()),
                reinterpret_cast<char*>(binningBuffer.data_ptr()), reinterpret_cast<char*>(imageBuffer.data_ptr()),
                amr_step, interpolate ? 1 : 0, fptr(dL_dout), interpolate ? fptr_mut(scratch) : nullptr,
                fptr_mut(dL_dmeans2D), nullptr, fptr_mut(dL_dopacity), want_colors ? fptr_mut(dL_dcolors) : nullptr,
                fptr_mut(dL_dmeans3D), want_cov3D ? fptr_mut(dL_dcov3D) : nullptr, fptr_mut(dL_dsh), fptr_mut(dL_dscales),
                fptr_mut(dL_drotations), debug, stream_of(means3D));
        }
        check(rc, amr_step ? "amr_rasterize_gaussians_backward" : "rasterize_gaussians_backward");
    }
    return std::make_tuple(dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                           dL_drotations);
}

// base/rasterize_points.cu:117-196
Grads8 RasterizeGaussiansBackward(const Tensor& background, const Tensor& means3D, const Tensor& radii,
                                  const Tensor& colors, const Tensor& scales, const Tensor& rotations,
                                  const float scale_modifier, const Tensor& cov3D_precomp, const Tensor& viewmatrix,
                                  const Tensor& projmatrix, const float tan_fovx, const float tan_fovy,
                                  const Tensor& dL_dout_color, const Tensor& sh, const int degree,
                                  const Tensor& campos, const Tensor& geomBuffer, const int R,
                                  const Tensor& binningBuffer, const Tensor& imageBuffer, const bool debug) {
    return BackwardImpl(0, false, background, means3D, radii, colors, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree, campos,
                        geomBuffer, R, binningBuffer, imageBuffer, debug, false);
}

// The same, for the autograd wrappers: grad_colors_precomp / grad_cov3Ds_precomp
// come back empty (not computed into memory) when those inputs were empty.
Grads8 RasterizeGaussiansBackwardLean(const Tensor& background, const Tensor& means3D, const Tensor& radii,
                                      const Tensor& colors, const Tensor& scales, const Tensor& rotations,
                                      const float scale_modifier, const Tensor& cov3D_precomp,
                                      const Tensor& viewmatrix, const Tensor& projmatrix, const float tan_fovx,
                                      const float tan_fovy, const Tensor& dL_dout_color, const Tensor& sh,
                                      const int degree, const Tensor& campos, const Tensor& geomBuffer, const int R,
                                      const Tensor& binningBuffer, const Tensor& imageBuffer, const bool debug) {
    return BackwardImpl(0, false, background, means3D, radii, colors, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree, campos,
                        geomBuffer, R, binningBuffer, imageBuffer, debug, true);
}

// The AMR backward (an extension: the reference's is unreachable): the
// image of foveaStep k (1..4) or of render_once (foveaStep < 0, optionally
// interpolated) -> the same 8 gradients as the base backward.
Grads8 AmrRasterizeGaussiansBackward(const Tensor& background, const Tensor& means3D, const Tensor& radii,
                                     const Tensor& colors, const Tensor& scales, const Tensor& rotations,
                                     const float scale_modifier, const Tensor& cov3D_precomp,
                                     const Tensor& viewmatrix, const Tensor& projmatrix, const float tan_fovx,
                                     const float tan_fovy, const Tensor& dL_dout_color, const Tensor& sh,
                                     const int degree, const Tensor& campos, const Tensor& geomBuffer, const int R,
                                     const Tensor& binningBuffer, const Tensor& imageBuffer, const int foveaStep,
                                     const bool interpolate_image, const bool debug) {
    TORCH_CHECK(foveaStep != 0, "foveaStep 0 renders nothing: its gradient is zero");
    return BackwardImpl(foveaStep, interpolate_image, background, means3D, radii, colors, scales, rotations,
                        scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh,
                        degree, campos, geomBuffer, R, binningBuffer, imageBuffer, debug, true);
}

// Data-parallel stage 1 (gsplat_amd.h): blend backward of one view -> its
// view record, [P * 10 + 40] floats (the record the ranks all-gather).
Tensor RasterizeGaussiansBackwardViewGrads(const Tensor& background, const Tensor& radii_in,
                                           const Tensor& colors_in, const Tensor& viewmatrix_in,
                                           const Tensor& projmatrix_in, const float tan_fovx, const float tan_fovy,
                                           const Tensor& campos_in, const Tensor& dL_dout_color_in,
                                           const Tensor& geomBuffer, const int R, const Tensor& binningBuffer,
                                           const Tensor& imageBuffer, const bool debug) {
    const int P = (int)radii_in.size(0);
    const int H = (int)dL_dout_color_in.size(1);
    const int W = (int)dL_dout_color_in.size(2);
    const at::OptionalDeviceGuard guard(device_of(dL_dout_color_in));
    Tensor rec = torch::empty({(int64_t)P * 10 + 40}, dL_dout_color_in.options());
    const Tensor bg = background.contiguous(), radii = radii_in.contiguous(), colors = colors_in.contiguous(),
                 dL_dout = dL_dout_color_in.contiguous(), viewmatrix = viewmatrix_in.contiguous(),
                 projmatrix = projmatrix_in.contiguous(), campos = campos_in.contiguous();
    require_device(dL_dout, "dL_dout_color");
    require_device(viewmatrix, "viewmatrix");
    TORCH_CHECK(dL_dout.dim() == 3 && dL_dout.size(0) == 3, "dL_dout_color must be [3, H, W]");
    require_like(viewmatrix, dL_dout, "viewmatrix", 16);
    require_like(projmatrix, dL_dout, "projmatrix", 16);
    require_like(campos, dL_dout, "campos", 3);
    require_like(bg, dL_dout, "bg", 3);
    require_like(colors, dL_dout, "colors_precomp", 3LL * P);
    for (const Tensor* bt : {&geomBuffer, &binningBuffer, &imageBuffer})
        require_like(*bt, dL_dout, "geometry / binning / image buffer", -1, torch::kByte);
    TORCH_CHECK(radii.is_cuda() && radii.scalar_type() == torch::kInt32, "radii must be an int32 device tensor");
    require_like(radii, dL_dout, "radii", P, torch::kInt32);
    check(gs_rasterizer_backward_view_grads(
              P, R, fptr(bg), W, H, fptr(colors), fptr(viewmatrix), fptr(projmatrix), fptr(campos), tan_fovx,
              tan_fovy, radii.data_ptr<int>(), reinterpret_cast<char*>(geomBuffer.data_ptr()),
              reinterpret_cast<char*>(binningBuffer.data_ptr()), reinterpret_cast<char*>(imageBuffer.data_ptr()),
              fptr(dL_dout), rec.data_ptr<float>(), debug, stream_of(dL_dout)),
          "rasterize_gaussians_backward_view_grads");
    return rec;
}

// Data-parallel stage 2: the per-Gaussian backward of V views at once (views
// = [V, P * 10 + 40] records), summed over views; returns (dL_dmeans3D,
// dL_dsh, dL_dopacity, dL_dscales, dL_drotations); densification statistics
// accumulated in place when given (non-empty).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> BackwardGaussiansMultiview(
    const Tensor& views_in, const Tensor& means3D_in, const Tensor& sh_in, const int degree, const Tensor& scales_in,
    const Tensor& rotations_in, const float scale_modifier, Tensor grad_norm_accum, Tensor denom,
    Tensor max_radii) {
    const int P = (int)means3D_in.size(0);
    TORCH_CHECK(views_in.dim() == 2 && views_in.size(1) == (int64_t)P * 10 + 40,
                "views must be [V, P * 10 + 40] view records");
    const int V = (int)views_in.size(0);
    const int M = sh_in.numel() != 0 ? (int)sh_in.size(1) : 0;
    const at::OptionalDeviceGuard guard(device_of(means3D_in));
    auto opts = means3D_in.options();
    Tensor dL_dmeans3D = torch::empty({P, 3}, opts);
    Tensor dL_dsh = torch::empty({P, M, 3}, opts);
    Tensor dL_dopacity = torch::empty({P, 1}, opts);
    Tensor dL_dscales = torch::empty({P, 3}, opts);
    Tensor dL_drotations = torch::empty({P, 4}, opts);
    const bool stats = grad_norm_accum.numel() != 0;
    if (stats) {
        for (const Tensor* t : {&grad_norm_accum, &denom, &max_radii}) {
            TORCH_CHECK(t->numel() == P && t->is_contiguous() && t->is_cuda() && t->scalar_type() == torch::kFloat32,
                        "statistics tensors must be contiguous float32 device tensors with P elements");
        }
    }
    if (P != 0) {
        const Tensor views = views_in.contiguous(), means3D = means3D_in.contiguous(), sh = sh_in.contiguous(),
                     scales = scales_in.contiguous(), rotations = rotations_in.contiguous();
        require_device(means3D, "means3D");
        require_like(views, means3D, "views");
        require_like(scales, means3D, "scales", 3LL * P);
        require_like(rotations, means3D, "rotations", 4LL * P);
        require_like(sh, means3D, "sh", (int64_t)P * M * 3);
        check(gs_backward_gaussians_multiview(
                  P, degree, M, V, fptr(views), fptr(means3D), fptr(sh), fptr(scales), fptr(rotations),
                  scale_modifier, fptr_mut(dL_dmeans3D), fptr_mut(dL_dsh), fptr_mut(dL_dopacity), fptr_mut(dL_dscales),
                  fptr_mut(dL_drotations), stats ? grad_norm_accum.data_ptr<float>() : nullptr,
                  stats ? denom.data_ptr<float>() : nullptr, stats ? max_radii.data_ptr<float>() : nullptr,
                  stream_of(means3D)),
              "backward_gaussians_multiview");
    }
    return std::make_tuple(dL_dmeans3D, dL_dsh, dL_dopacity, dL_dscales, dL_drotations);
}

// Chunked stage 2: rows [V, count * 10] (view v's rows of Gaussians [g0,
// g0 + count)), cams [V, 40]; writes that range of the caller's full-size
// output tensors (and statistics, when non-empty).
void BackwardGaussiansMultiviewRange(const Tensor& rows_in, const Tensor& cams_in, const int g0,
                                     const Tensor& means3D_in, const Tensor& sh_in, const int degree,
                                     const Tensor& scales_in, const Tensor& rotations_in, const float scale_modifier,
                                     Tensor dL_dmeans3D, Tensor dL_dsh, Tensor dL_dopacity, Tensor dL_dscales,
                                     Tensor dL_drotations, Tensor grad_norm_accum, Tensor denom, Tensor max_radii) {
    const int P = (int)means3D_in.size(0);
    TORCH_CHECK(rows_in.dim() == 2 && rows_in.size(1) % 10 == 0, "rows must be [V, count * 10]");
    const int V = (int)rows_in.size(0);
    const int count = (int)(rows_in.size(1) / 10);
    TORCH_CHECK(cams_in.dim() == 2 && cams_in.size(0) == V && cams_in.size(1) == 40, "cams must be [V, 40]");
    TORCH_CHECK(g0 >= 0 && g0 + count <= P, "Gaussian range out of bounds");
    const int M = sh_in.numel() != 0 ? (int)sh_in.size(1) : 0;
    for (const Tensor* t : {&dL_dmeans3D, &dL_dopacity, &dL_dscales, &dL_drotations})
        TORCH_CHECK(t->is_contiguous() && t->size(0) == P && t->scalar_type() == torch::kFloat32,
                    "outputs must be contiguous float32 [P, ...] tensors");
    TORCH_CHECK(M == 0 || (dL_dsh.is_contiguous() && dL_dsh.numel() == (int64_t)P * M * 3), "dL_dsh must be [P, M, 3]");
    const bool stats = grad_norm_accum.numel() != 0;
    if (stats) {
        for (const Tensor* t : {&grad_norm_accum, &denom, &max_radii}) {
            TORCH_CHECK(t->numel() == P && t->is_contiguous() && t->is_cuda() && t->scalar_type() == torch::kFloat32,
                        "statistics tensors must be contiguous float32 device tensors with P elements");
        }
    }
    const at::OptionalDeviceGuard guard(device_of(means3D_in));
    TORCH_CHECK(rows_in.stride(1) == 1 && cams_in.stride(1) == 1, "rows / cams rows must be contiguous");
    const Tensor means3D = means3D_in.contiguous(), sh = sh_in.contiguous(), scales = scales_in.contiguous(),
                 rotations = rotations_in.contiguous();
    require_device(means3D, "means3D");
    require_like(rows_in, means3D, "rows");
    require_like(cams_in, means3D, "cams");
    require_like(scales, means3D, "scales", 3LL * P);
    require_like(rotations, means3D, "rotations", 4LL * P);
    require_like(sh, means3D, "sh", (int64_t)P * M * 3);
    check(gs_backward_gaussians_multiview_range(
              P, g0, count, degree, M, V, rows_in.data_ptr<float>(), (size_t)rows_in.stride(0), cams_in.data_ptr<float>(),
              (size_t)cams_in.stride(0), fptr(means3D), fptr(sh), fptr(scales), fptr(rotations), scale_modifier,
              fptr_mut(dL_dmeans3D), M ? fptr_mut(dL_dsh) : nullptr, fptr_mut(dL_dopacity), fptr_mut(dL_dscales),
              fptr_mut(dL_drotations), stats ? grad_norm_accum.data_ptr<float>() : nullptr,
              stats ? denom.data_ptr<float>() : nullptr, stats ? max_radii.data_ptr<float>() : nullptr,
              stream_of(means3D)),
          "backward_gaussians_multiview_range");
}

// Stage 2 over separately stored views: rows[v] = view v's rows of Gaussians
// [g0, g0 + count) (a contiguous [count * 10] slice), cams[v] = its camera
// ([40]); views summed in list order.  Each all-gathered piece can stay in its
// own [world, n] buffer.
void BackwardGaussiansMultiviewViews(const std::vector<Tensor>& rows, const std::vector<Tensor>& cams, const int g0,
                                     const Tensor& means3D_in, const Tensor& sh_in, const int degree,
                                     const Tensor& scales_in, const Tensor& rotations_in, const float scale_modifier,
                                     Tensor dL_dmeans3D, Tensor dL_dsh, Tensor dL_dopacity, Tensor dL_dscales,
                                     Tensor dL_drotations, Tensor grad_norm_accum, Tensor denom, Tensor max_radii) {
    const int P = (int)means3D_in.size(0);
    const int V = (int)rows.size();
    TORCH_CHECK(V >= 1 && (int)cams.size() == V, "at least one view, one camera each");
    TORCH_CHECK(rows[0].dim() == 1 && rows[0].numel() % 10 == 0, "rows[v] must be a 1-D [count * 10] slice");
    const int count = (int)(rows[0].numel() / 10);
    TORCH_CHECK(g0 >= 0 && g0 + count <= P, "Gaussian range out of bounds");
    const int M = sh_in.numel() != 0 ? (int)sh_in.size(1) : 0;
    for (const Tensor* t : {&dL_dmeans3D, &dL_dopacity, &dL_dscales, &dL_drotations})
        TORCH_CHECK(t->is_contiguous() && t->size(0) == P && t->scalar_type() == torch::kFloat32,
                    "outputs must be contiguous float32 [P, ...] tensors");
    TORCH_CHECK(M == 0 || (dL_dsh.is_contiguous() && dL_dsh.numel() == (int64_t)P * M * 3), "dL_dsh must be [P, M, 3]");
    const bool stats = grad_norm_accum.numel() != 0;
    if (stats) {
        for (const Tensor* t : {&grad_norm_accum, &denom, &max_radii}) {
            TORCH_CHECK(t->numel() == P && t->is_contiguous() && t->is_cuda() && t->scalar_type() == torch::kFloat32,
                        "statistics tensors must be contiguous float32 device tensors with P elements");
        }
    }
    const at::OptionalDeviceGuard guard(device_of(means3D_in));
    const Tensor means3D = means3D_in.contiguous(), sh = sh_in.contiguous(), scales = scales_in.contiguous(),
                 rotations = rotations_in.contiguous();
    require_device(means3D, "means3D");
    std::vector<const float*> rp(V), cp(V);
    for (int v = 0; v < V; v++) {
        TORCH_CHECK(rows[v].dim() == 1 && rows[v].numel() == (int64_t)count * 10 && rows[v].is_contiguous(),
                    "rows[v] must be contiguous [count * 10] slices of equal length");
        TORCH_CHECK(cams[v].dim() == 1 && cams[v].numel() == 40 && cams[v].is_contiguous(), "cams[v] must be [40]");
        require_like(rows[v], means3D, "rows");
        require_like(cams[v], means3D, "cams");
        rp[v] = rows[v].data_ptr<float>();
        cp[v] = cams[v].data_ptr<float>();
    }
    require_like(scales, means3D, "scales", 3LL * P);
    require_like(rotations, means3D, "rotations", 4LL * P);
    require_like(sh, means3D, "sh", (int64_t)P * M * 3);
    check(gs_backward_gaussians_multiview_views(
              P, g0, count, degree, M, V, rp.data(), cp.data(), fptr(means3D), fptr(sh), fptr(scales),
              fptr(rotations), scale_modifier, fptr_mut(dL_dmeans3D), M ? fptr_mut(dL_dsh) : nullptr,
              fptr_mut(dL_dopacity), fptr_mut(dL_dscales), fptr_mut(dL_drotations),
              stats ? grad_norm_accum.data_ptr<float>() : nullptr, stats ? denom.data_ptr<float>() : nullptr,
              stats ? max_radii.data_ptr<float>() : nullptr, stream_of(means3D)),
          "backward_gaussians_multiview_views");
}

// ---- eye-tracking front end (ritnet.hip) ----
// out [32, H, W] = conv over the virtual concatenation of `ins` (each
// [C, h, w]; up[i] = 1: read through nearest 2x upsampling).
void RitnetConv(int ksize, const std::vector<Tensor>& ins, const std::vector<int>& up, const Tensor& weight,
                const Tensor& bias, bool leaky_relu, const Tensor& bn_scale, const Tensor& bn_shift, Tensor out) {
    TORCH_CHECK(!ins.empty() && ins.size() <= 3 && up.size() == ins.size(), "1 to 3 inputs, one up flag each");
    TORCH_CHECK(out.dim() == 3 && out.size(0) == 32 && out.is_contiguous(), "out must be a contiguous [32, H, W]");
    const int H = (int)out.size(1), W = (int)out.size(2);
    const float* p[3];
    int c[3], u[3];
    int Cin = 0;
    for (size_t i = 0; i < ins.size(); i++) {
        const Tensor& t = ins[i];
        require_device(t, "input");
        TORCH_CHECK(t.dim() == 3 && t.is_contiguous(), "inputs must be contiguous [C, h, w]");
        TORCH_CHECK(t.size(1) == (up[i] ? H / 2 : H) && t.size(2) == (up[i] ? W / 2 : W), "input size mismatch");
        p[i] = t.data_ptr<float>();
        c[i] = (int)t.size(0);
        u[i] = up[i];
        Cin += c[i];
    }
    TORCH_CHECK(weight.numel() == (int64_t)Cin * ksize * ksize * 32 && weight.is_contiguous(),
                "weight must be [Cin, k*k, 32]");
    TORCH_CHECK(bias.numel() == 32, "bias must have 32 elements");
    const at::OptionalDeviceGuard guard(device_of(out));
    check(gs_ritnet_conv(ksize, (int)ins.size(), p, c, u, H, W, weight.data_ptr<float>(), bias.data_ptr<float>(),
                         leaky_relu ? 1 : 0, bn_scale.numel() ? bn_scale.data_ptr<float>() : nullptr,
                         bn_shift.numel() ? bn_shift.data_ptr<float>() : nullptr, out.data_ptr<float>(),
                         stream_of(out)),
          "ritnet_conv");
}

Tensor AvgPool2(const Tensor& in) {
    require_device(in, "input");
    TORCH_CHECK(in.dim() == 3 && in.is_contiguous(), "input must be a contiguous [C, H, W]");
    const at::OptionalDeviceGuard guard(device_of(in));
    Tensor out = torch::empty({in.size(0), in.size(1) / 2, in.size(2) / 2}, in.options());
    check(gs_avgpool2(in.data_ptr<float>(), (int)in.size(0), (int)in.size(1), (int)in.size(2), out.data_ptr<float>(),
                      stream_of(in)),
          "avgpool2");
    return out;
}

std::tuple<Tensor, Tensor> RitnetHead(const Tensor& in, const Tensor& weight, const Tensor& bias, bool want_logits) {
    require_device(in, "input");
    TORCH_CHECK(in.dim() == 3 && in.size(0) == 32 && in.is_contiguous(), "input must be a contiguous [32, H, W]");
    TORCH_CHECK(weight.numel() == 128 && bias.numel() == 4, "head weight [32, 4], bias [4]");
    const int H = (int)in.size(1), W = (int)in.size(2);
    const at::OptionalDeviceGuard guard(device_of(in));
    Tensor labels = torch::empty({H, W}, in.options().dtype(torch::kUInt8));
    Tensor logits = want_logits ? torch::empty({4, H, W}, in.options()) : torch::empty({0}, in.options());
    check(gs_ritnet_head(in.data_ptr<float>(), H, W, weight.data_ptr<float>(), bias.data_ptr<float>(),
                         want_logits ? logits.data_ptr<float>() : nullptr, labels.data_ptr<uint8_t>(), stream_of(in)),
          "ritnet_head");
    return std::make_tuple(logits, labels);
}

Tensor LabelMoments(const Tensor& labels, int label) {
    TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == torch::kUInt8 && labels.dim() == 2 && labels.is_contiguous(),
                "labels must be a contiguous uint8 [H, W] device tensor");
    const at::OptionalDeviceGuard guard(device_of(labels));
    Tensor out = torch::empty({3}, labels.options().dtype(torch::kFloat64));
    check(gs_label_moments(labels.data_ptr<uint8_t>(), (int)labels.size(0), (int)labels.size(1), label,
                           out.data_ptr<double>(), stream_of(labels)),
          "label_moments");
    return out;
}

// Fovea-driven AMR levels on the image buffer of foveaStep 0 (in place).
void AmrFoveaLevels(Tensor imageBuffer, int width, int height, const std::vector<double>& centres_xy,
                    const std::vector<double>& radii, int min_level, bool replace) {
    TORCH_CHECK(imageBuffer.is_cuda() && imageBuffer.scalar_type() == torch::kUInt8 && imageBuffer.numel() > 0,
                "imageBuffer must be the uint8 device buffer returned by foveaStep 0");
    TORCH_CHECK(centres_xy.size() == 2 * radii.size() && radii.size() <= 4, "up to 4 foveae: centres [n][2], radii [n]");
    float c[8], r[4];
    for (size_t i = 0; i < radii.size(); i++) {
        c[2 * i] = (float)centres_xy[2 * i];
        c[2 * i + 1] = (float)centres_xy[2 * i + 1];
        r[i] = (float)radii[i];
    }
    const at::OptionalDeviceGuard guard(device_of(imageBuffer));
    check(gs_amr_fovea_levels(reinterpret_cast<char*>(imageBuffer.data_ptr<uint8_t>()), (size_t)imageBuffer.numel(),
                              width, height,
                              (int)radii.size(), c, r, min_level, replace ? 1 : 0, stream_of(imageBuffer)),
          "amr_fovea_levels");
}

// gray [H, W] uint8 -> RITnet input [W, H] float32 (gamma, CLAHE, normalise, transpose).
Tensor EyePreprocess(const Tensor& gray, const Tensor& gamma_lut, double clip_limit, int tiles_x, int tiles_y) {
    TORCH_CHECK(gray.is_cuda() && gray.scalar_type() == torch::kUInt8 && gray.dim() == 2 && gray.is_contiguous(),
                "gray must be a contiguous uint8 [H, W] device tensor");
    TORCH_CHECK(gamma_lut.is_cuda() && gamma_lut.scalar_type() == torch::kUInt8 && gamma_lut.numel() == 256,
                "gamma_lut must be 256 uint8 on the device");
    const at::OptionalDeviceGuard guard(device_of(gray));
    const int H = (int)gray.size(0), W = (int)gray.size(1);
    Tensor out = torch::empty({W, H}, gray.options().dtype(torch::kFloat32));
    Tensor luts = torch::empty({(int64_t)tiles_x * tiles_y * 256}, gray.options().dtype(torch::kFloat32));
    check(gs_eye_preprocess(gray.data_ptr<uint8_t>(), H, W, gamma_lut.data_ptr<uint8_t>(), clip_limit, tiles_x,
                            tiles_y, luts.data_ptr<float>(), out.data_ptr<float>(), stream_of(gray)),
          "eye_preprocess");
    return out;
}

// base/rasterize_points.cu:198-217
Tensor MarkVisible(Tensor& means3D_in, Tensor& viewmatrix_in, Tensor& projmatrix_in) {
    const int P = (int)means3D_in.size(0);
    const at::OptionalDeviceGuard guard(device_of(means3D_in));
    Tensor present = torch::zeros({P}, means3D_in.options().dtype(at::kBool));
    if (P != 0) {
        const Tensor means3D = means3D_in.contiguous(), viewmatrix = viewmatrix_in.contiguous(),
                     projmatrix = projmatrix_in.contiguous();
        require_device(means3D, "means3D");
        check(gs_rasterizer_mark_visible(P, fptr(means3D), fptr(viewmatrix), fptr(projmatrix),
                                         reinterpret_cast<uint8_t*>(present.data_ptr<bool>()), stream_of(means3D)),
              "mark_visible");
    }
    return present;
}

// knn/spatial.cu:14-24
Tensor DistCUDA2(const Tensor& points_in) {
    const int P = (int)points_in.size(0);
    const at::OptionalDeviceGuard guard(device_of(points_in));
    Tensor means = torch::empty({P}, points_in.options().dtype(torch::kFloat32));
    if (P != 0) {
        const Tensor points = points_in.contiguous();
        require_device(points, "points");
        Tensor scratch = torch::empty({0}, points.options().dtype(torch::kByte));
        check(gs_simple_knn(P, fptr(points), means.data_ptr<float>(), buf_of(scratch), stream_of(points)),
              "distCUDA2");
    }
    return means;
}

// Parity accessor (the idea of amr-debug's ParseBuffers,
// amr-debug/rasterize_points.cu:37-61): copies of every internal buffer.
py::dict ParseBuffers(const Tensor& geomBuffer, const Tensor& binningBuffer, const Tensor& imgBuffer, int P, int K,
                      int width, int height, int tile) {
    const at::OptionalDeviceGuard guard(device_of(geomBuffer));
    auto o = geomBuffer.options();
    auto f32 = o.dtype(torch::kFloat32);
    auto i32 = o.dtype(torch::kInt32);
    gs_geom_view g;
    gs_image_view im;
    gs_binning_view b;
    gs_geom_view_of(reinterpret_cast<char*>(geomBuffer.data_ptr()), P, &g);
    gs_image_view_of(reinterpret_cast<char*>(imgBuffer.data_ptr()), width, height, tile, &im);
    gs_binning_view_of(binningBuffer.numel() ? reinterpret_cast<char*>(binningBuffer.data_ptr()) : nullptr, K, &b);
    const int64_t T = (int64_t)((width + tile - 1) / tile) * ((height + tile - 1) / tile);
    const int64_t N = (int64_t)width * height;
    auto view = [&](void* p, std::vector<int64_t> shape, c10::TensorOptions opt) {
        return torch::from_blob(p, shape, opt).clone();
    };
    py::dict d;
    d["hdr"] = view(g.hdr, {64}, i32);
    d["depths"] = view(g.depths, {P}, f32);
    d["radii"] = view(g.radii, {P}, i32);
    d["means2D"] = view(g.means2D, {P, 2}, f32);
    d["conic_opacity"] = view(g.conic_opacity, {P, 4}, f32);
    d["rgb"] = view(g.rgb, {P, 3}, f32);
    if ((size_t)geomBuffer.numel() >= gs_geom_bytes((int)P))  // (the optional tail: a forward that wrote it)
        d["cov3D"] = view(g.cov3D, {P, 6}, f32);
    d["clamped_bits"] = view(g.clamped, {P}, o.dtype(torch::kUInt8));
    d["tiles_touched"] = view(g.tiles_touched, {P}, i32);
    d["grad_accum"] = view(g.grad_accum, {P, GSPLAT_AMD_GRAD_ROW}, f32);
    d["accum_alpha"] = view(im.accum_alpha, {N}, f32);
    d["n_contrib"] = view(im.n_contrib, {N}, i32);
    d["ranges"] = view(im.ranges, {T, 2}, i32);
    d["tile_count"] = view(im.tile_count, {T}, i32);
    d["max_contrib"] = view(im.max_contrib, {T}, i32);
    d["levels"] = view(im.levels, {T}, i32);
    d["levels_last"] = view(im.levels_last, {T}, i32);
    d["levels_current"] = view(im.levels_current, {T}, i32);
    d["pv"] = view(im.pv, {4}, i32);
    if (tile == 32) {
        d["tile_order"] = view(im.tile_order, {T}, i32);
        d["region_count"] = view(im.region_count, {T, 16}, i32);
    }
    if (K > 0) {
        d["point_list"] = view(b.point_list, {K}, i32);
        // the forward's per-instance row-group hit codes (base grid), where
        // the header word says they are (gs_layout.h hit_codes_of: 0 = none,
        // else 1 + byte offset from point_list / 256)
        if (tile == 16) {
            uint32_t w = 0;
            TORCH_CHECK(hipMemcpy(&w, g.hdr + 6, sizeof(uint32_t), hipMemcpyDeviceToHost) == hipSuccess,
                        "parse_buffers: header read-back failed");
            const size_t off = w ? (size_t)(w - 1u) * 256u : 0u;
            if (w && off + (size_t)K <= (size_t)binningBuffer.numel())
                d["hit_codes"] = view(reinterpret_cast<uint8_t*>(b.point_list) + off, {K}, o.dtype(torch::kUInt8));
        }
        Tensor keys = torch::empty({K}, o.dtype(torch::kInt64));
        check(gs_reconstruct_keys(reinterpret_cast<char*>(geomBuffer.data_ptr()),
                                  reinterpret_cast<char*>(binningBuffer.data_ptr()),
                                  reinterpret_cast<char*>(imgBuffer.data_ptr()), P, K, width, height, tile,
                                  reinterpret_cast<uint64_t*>(keys.data_ptr<int64_t>()), stream_of(geomBuffer)),
              "reconstruct_keys");
        d["point_list_keys"] = keys;
    }
    return d;
}

py::dict ProfileRead(bool reset) {
    const int n = gs_profile_stage_count();
    std::vector<double> ms(n);
    std::vector<long> cnt(n);
    gs_profile_read(ms.data(), cnt.data(), reset ? 1 : 0);
    py::dict d;
    for (int i = 0; i < n; i++) d[py::str(gs_profile_stage_name(i))] = py::make_tuple(ms[i], cnt[i]);
    return d;
}

}  // namespace

// Fused L1 + D-SSIM training loss (loss.hip): returns (out3 = [loss, l1, ssim], grad).
std::tuple<Tensor, Tensor> L1SsimLoss(const Tensor& image, const Tensor& gt, double lambda_dssim) {
    TORCH_CHECK(image.sizes() == gt.sizes() && image.dim() == 3, "image and gt must both be [C, H, W]");
    require_device(image, "image");
    require_device(gt, "gt");
    const at::OptionalDeviceGuard guard(device_of(image));
    const Tensor x = image.contiguous(), y = gt.contiguous();
    Tensor grad = torch::empty_like(x);
    Tensor out3 = torch::empty({3}, x.options());
    Tensor ws = torch::empty({0}, x.options().dtype(torch::kByte));
    check(gs_l1_ssim_loss(x.data_ptr<float>(), y.data_ptr<float>(), (int)x.size(0), (int)x.size(1), (int)x.size(2),
                          (float)lambda_dssim, grad.data_ptr<float>(), out3.data_ptr<float>(), buf_of(ws),
                          stream_of(x)),
          "l1_ssim_loss");
    return std::make_tuple(out3, grad);
}

// Fused Adam over flat buffers: seg_end / lr per segment (host lists).
void AdamStep(Tensor& params, const Tensor& grads, Tensor& exp_avg, Tensor& exp_avg_sq,
              const std::vector<int64_t>& seg_end, const std::vector<double>& lr, const std::vector<int64_t>& step, double beta1,
              double beta2, double eps) {
    for (const Tensor* t : std::initializer_list<const Tensor*>{&params, &grads, &exp_avg, &exp_avg_sq}) {
        require_device(*t, "adam buffer");
        TORCH_CHECK(t->is_contiguous() && t->numel() == params.numel(), "adam buffers: contiguous, same size");
    }
    TORCH_CHECK(seg_end.size() == lr.size() && step.size() == lr.size() && !seg_end.empty() && seg_end.back() == params.numel(),
                "adam segments must cover the buffer");
    const at::OptionalDeviceGuard guard(device_of(params));
    std::vector<long long> ends(seg_end.begin(), seg_end.end()), steps(step.begin(), step.end());
    check(gs_adam_step(params.data_ptr<float>(), grads.data_ptr<float>(), exp_avg.data_ptr<float>(),
                       exp_avg_sq.data_ptr<float>(), params.numel(), (int)ends.size(), ends.data(), lr.data(), steps.data(),
                       beta1, beta2, eps, stream_of(params)),
          "adam_step");
}

// train.py:111-113: in-place statistics update (accum / denom [P, 1], max_radii [P]).
void DensifyStats(const Tensor& radii, const Tensor& grad_means2D, Tensor& accum, Tensor& denom, Tensor& max_radii) {
    const int64_t P = radii.size(0);
    TORCH_CHECK(radii.is_cuda() && radii.scalar_type() == torch::kInt32 && radii.is_contiguous(),
                "radii: int32 contiguous HIP device tensor");
    require_device(grad_means2D, "grad_means2D");
    TORCH_CHECK(grad_means2D.dim() == 2 && grad_means2D.size(0) == P && grad_means2D.size(1) >= 2 &&
                    grad_means2D.stride(1) == 1 && grad_means2D.scalar_type() == torch::kFloat32,
                "grad_means2D: [P, >=2] f32 rows");
    for (const Tensor* t : std::initializer_list<const Tensor*>{&accum, &denom, &max_radii}) {
        require_device(*t, "densification statistic");
        TORCH_CHECK(t->numel() == P && t->is_contiguous() && t->scalar_type() == torch::kFloat32,
                    "densification statistics: P contiguous f32");
    }
    const at::OptionalDeviceGuard guard(device_of(radii));
    check(gs_densify_stats((int)P, radii.data_ptr<int>(), grad_means2D.data_ptr<float>(), (int)grad_means2D.stride(0),
                           accum.data_ptr<float>(), denom.data_ptr<float>(), max_radii.data_ptr<float>(),
                           stream_of(radii)),
          "densify_stats");
}

void check_f32_rows(const Tensor& t, int64_t P, int64_t n, const char* name) {
    require_device(t, name);
    TORCH_CHECK(t.is_contiguous() && t.numel() == P * n, name, ": contiguous, ", n, " floats per Gaussian");
}

// scene/gaussian_model.py:93-113: raw groups -> rasterizer inputs (outputs preallocated).
void Activate(const Tensor& dc, const Tensor& rest, const Tensor& opacity_raw, const Tensor& scaling_raw,
              const Tensor& rotation_raw, Tensor& shs, Tensor& opacities, Tensor& scales, Tensor& rotations) {
    const int64_t P = dc.size(0);
    const int64_t M = rest.numel() / std::max<int64_t>(P, 1) / 3 + 1;
    check_f32_rows(dc, P, 3, "features_dc");
    check_f32_rows(rest, P, 3 * (M - 1), "features_rest");
    check_f32_rows(opacity_raw, P, 1, "opacity");
    check_f32_rows(scaling_raw, P, 3, "scaling");
    check_f32_rows(rotation_raw, P, 4, "rotation");
    check_f32_rows(shs, P, 3 * M, "shs");
    check_f32_rows(opacities, P, 1, "opacities");
    check_f32_rows(scales, P, 3, "scales");
    check_f32_rows(rotations, P, 4, "rotations");
    const at::OptionalDeviceGuard guard(device_of(dc));
    check(gs_activate_gaussians((int)P, (int)M, fptr(dc), fptr(rest), fptr(opacity_raw), fptr(scaling_raw),
                                fptr(rotation_raw), fptr_mut(shs), fptr_mut(opacities), fptr_mut(scales),
                                fptr_mut(rotations), stream_of(dc)),
          "activate");
}

void ActivationBackward(const Tensor& d_shs, const Tensor& d_opac, const Tensor& d_scales, const Tensor& d_rot,
                        const Tensor& d_means3D, const Tensor& opacity_raw, const Tensor& scaling_raw,
                        const Tensor& rotation_raw, Tensor& g_xyz, Tensor& g_dc, Tensor& g_rest, Tensor& g_opacity,
                        Tensor& g_scaling, Tensor& g_rotation, bool accumulate) {
    const int64_t P = d_means3D.size(0);
    const int64_t M = d_shs.numel() / std::max<int64_t>(P, 1) / 3;
    check_f32_rows(d_shs, P, 3 * M, "dL_dshs");
    check_f32_rows(d_opac, P, 1, "dL_dopacities");
    check_f32_rows(d_scales, P, 3, "dL_dscales");
    check_f32_rows(d_rot, P, 4, "dL_drotations");
    check_f32_rows(d_means3D, P, 3, "dL_dmeans3D");
    check_f32_rows(opacity_raw, P, 1, "opacity");
    check_f32_rows(scaling_raw, P, 3, "scaling");
    check_f32_rows(rotation_raw, P, 4, "rotation");
    check_f32_rows(g_xyz, P, 3, "grad xyz");
    check_f32_rows(g_dc, P, 3, "grad features_dc");
    check_f32_rows(g_rest, P, 3 * (M - 1), "grad features_rest");
    check_f32_rows(g_opacity, P, 1, "grad opacity");
    check_f32_rows(g_scaling, P, 3, "grad scaling");
    check_f32_rows(g_rotation, P, 4, "grad rotation");
    const at::OptionalDeviceGuard guard(device_of(d_shs));
    check(gs_activation_backward((int)P, (int)M, accumulate ? 1 : 0, fptr(d_shs), fptr(d_opac), fptr(d_scales),
                                 fptr(d_rot), fptr(d_means3D), fptr(opacity_raw), fptr(scaling_raw),
                                 fptr(rotation_raw), fptr_mut(g_xyz), fptr_mut(g_dc), fptr_mut(g_rest),
                                 fptr_mut(g_opacity), fptr_mut(g_scaling), fptr_mut(g_rotation), stream_of(d_shs)),
          "activation_backward");
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "MI355X (gfx950) Gaussian rasterizer -- PyTorch binding over include/gsplat_amd.h";
    m.def("rasterize_gaussians", &RasterizeGaussians);
    m.def("rasterize_gaussians_backward", &RasterizeGaussiansBackward);
    m.def("rasterize_gaussians_backward_lean", &RasterizeGaussiansBackwardLean);
    m.def("amr_rasterize_gaussians_backward", &AmrRasterizeGaussiansBackward);
    m.def("mark_visible", &MarkVisible);
    m.def("rasterize_gaussians_backward_view_grads", &RasterizeGaussiansBackwardViewGrads);
    m.def("backward_gaussians_multiview", &BackwardGaussiansMultiview);
    m.def("backward_gaussians_multiview_range", &BackwardGaussiansMultiviewRange);
    m.def("backward_gaussians_multiview_views", &BackwardGaussiansMultiviewViews);
    m.def("ritnet_conv", &RitnetConv);
    m.def("avgpool2", &AvgPool2);
    m.def("ritnet_head", &RitnetHead);
    m.def("label_moments", &LabelMoments);
    m.def("eye_preprocess", &EyePreprocess);
    m.def("amr_fovea_levels", &AmrFoveaLevels);
    m.def("amr_rasterize_gaussians", &AMRRasterizeGaussians);
    m.def("amr_accumulate_step", &AmrAccumulateStep);
    m.def("distCUDA2", &DistCUDA2);
    m.def("parse_buffers", &ParseBuffers);
    m.def("l1_ssim_loss", &L1SsimLoss);
    m.def("adam_step", &AdamStep);
    m.def("densify_stats", &DensifyStats);
    m.def("activate", &Activate);
    m.def("activation_backward", &ActivationBackward);
    m.def("abi_version", []() { return gs_abi_version(); });
    m.def("amr_geom_bytes", [](int P) { return gs_amr_geom_bytes(P); },
          "bytes of an AMR forward's geometry buffer (the tail, then the 64-B AMR blend rows)");
    m.def("geom_bytes", [](int P) { return gs_geom_bytes(P); },
          "geometry-buffer bytes with the optional tail (the upper bound a forward asks for)");
    m.def("profile_enable", [](bool on) { gs_profile_enable(on ? 1 : 0); });
    m.def("profile_stages", [](const std::vector<std::string>& names) {
        // [] = all stages
        unsigned mask = names.empty() ? ~0u : 0u;
        for (const auto& n : names) {
            int i = 0;
            for (; i < gs_profile_stage_count(); i++)
                if (n == gs_profile_stage_name(i)) break;
            if (i == gs_profile_stage_count()) throw std::invalid_argument("unknown stage " + n);
            mask |= 1u << i;
        }
        gs_profile_set_mask(mask);
    });
    m.def("profile_read", &ProfileRead, py::arg("reset") = true);
    m.def("set_tuning", [](const std::string& k, int v) { check(gs_set_tuning(k.c_str(), v), "set_tuning"); });
    m.def("set_amr_speculation", [](bool on) {
        t_spec_on = on;
        if (!on) t_spec.clear();
    }, "speculative AMR steps (this thread): step 1 renders steps 1..4 at once, steps 2..4 return its images");
    m.def("get_tuning", [](const std::string& k) {
        int v = 0;
        check(gs_get_tuning(k.c_str(), &v), "get_tuning");
        return v;
    });
    m.def("set_thread_option",
          [](const std::string& k, int v) { check(gs_set_thread_option(k.c_str(), v), "set_thread_option"); });
}
