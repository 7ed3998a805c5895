/*
 * gs_oracle.c -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference hot path of
 * XinShuo-ph/gaussian_splatting_with_eye_tracking:
 *   submodules/diff-gaussian-rasterization      (base/)
 *   submodules/diff-gaussian-rasterization-amr  (amr/)
 *   submodules/simple-knn                       (knn/)
 * Every function cites the reference file:line it follows.  Nothing in the
 * product path links, loads or calls this file: only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() use it, as the checker.
 *
 * Arithmetic policy (shared with the HIP kernels, see DESIGN.md "parity"):
 *   - compiled with -ffp-contract=off: every a*b+c is two rounded ops, in the
 *     left-to-right order of the reference source (glm column-major products
 *     expanded exactly like glm/detail/type_mat3x3.inl:486-520);
 *   - correctly rounded '/', sqrtf; ndc2Pix in double (base/cr/auxiliary.h:41-44);
 *   - exp uses libm expf (the GPU uses the hardware exp; blend outputs are
 *     therefore compared within tolerance, binning buffers bit-exactly).
 *   - gradient accumulation (the reference's float atomics) is done in double
 *     here, i.e. the oracle returns the exact sum the atomics approximate.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NUM_CHANNELS 3

/* Host threads for the per-Gaussian and per-pixel loops (OpenMP).  1 (the
 * default) runs every loop serially, in the order the frozen golden fixtures
 * were made with; n > 1 parallelises the loops whose iterations are
 * independent, and the blend backward sums its per-Gaussian terms per band
 * of tile rows, in band order (deterministic for a given n; differs from the
 * serial sum only in double-precision rounding). */
static int g_threads = 1;
void orc_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
int orc_get_threads(void) { return g_threads; }

/* ---------------------------------------------------------------- constants */
/* base/cr/auxiliary.h:22-39 */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

/* ------------------------------------------------------------- glm mat3 ops */
/* m[c][r]: column c, row r (glm convention). */
typedef struct { float m[3][3]; } mat3;

static mat3 mat3_cols(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                      float a7, float a8) {
    mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}

/* glm/detail/type_mat3x3.inl:486-520 */
static mat3 mat3_mul(const mat3* A, const mat3* B) {
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++)
            R.m[c][r] = A->m[0][r] * B->m[c][0] + A->m[1][r] * B->m[c][1] + A->m[2][r] * B->m[c][2];
    return R;
}

static mat3 mat3_transpose(const mat3* A) {
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) R.m[c][r] = A->m[r][c];
    return R;
}

static mat3 mat3_scale(float s, const mat3* A) {
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) R.m[c][r] = s * A->m[c][r];
    return R;
}

/* glm dot (func_geometric.inl): tmp = a*b; tmp.x + tmp.y + tmp.z */
static float dot3(const float* a, const float* b) {
    float t0 = a[0] * b[0], t1 = a[1] * b[1], t2 = a[2] * b[2];
    return t0 + t1 + t2;
}

/* ---------------------------------------------------------------- auxiliary */
/* base/cr/auxiliary.h:41-44 (evaluated in double, as the `1.0` literals force) */
static float ndc2Pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

/* base/cr/auxiliary.h:46-56 (BLOCK_X/BLOCK_Y passed explicitly: 16 base, 32 AMR) */
static void getRect(float px, float py, int max_radius, int bx, int by, unsigned gx, unsigned gy,
                    unsigned* rmin, unsigned* rmax) {
    float fr = (float)max_radius;
    int a = (int)((px - fr) / (float)bx);
    int b = (int)((py - fr) / (float)by);
    int c = (int)(((px + fr) + (float)bx - 1.0f) / (float)bx);
    int d = (int)(((py + fr) + (float)by - 1.0f) / (float)by);
    a = a > 0 ? a : 0; b = b > 0 ? b : 0; c = c > 0 ? c : 0; d = d > 0 ? d : 0;
    rmin[0] = (unsigned)a < gx ? (unsigned)a : gx;
    rmin[1] = (unsigned)b < gy ? (unsigned)b : gy;
    rmax[0] = (unsigned)c < gx ? (unsigned)c : gx;
    rmax[1] = (unsigned)d < gy ? (unsigned)d : gy;
}

/* base/cr/auxiliary.h:58-66 */
static void transformPoint4x3(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}

/* base/cr/auxiliary.h:68-77 */
static void transformPoint4x4(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}

/* base/cr/auxiliary.h:89-97 */
static void transformVec4x3Transpose(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[1] * p[1] + m[2] * p[2];
    o[1] = m[4] * p[0] + m[5] * p[1] + m[6] * p[2];
    o[2] = m[8] * p[0] + m[9] * p[1] + m[10] * p[2];
}

/* base/cr/auxiliary.h:107-117 */
static void dnormvdv3(const float* v, const float* dv, float* o) {
    float sum2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    o[0] = ((+sum2 - v[0] * v[0]) * dv[0] - v[1] * v[0] * dv[1] - v[2] * v[0] * dv[2]) * invsum32;
    o[1] = (-v[0] * v[1] * dv[0] + (sum2 - v[1] * v[1]) * dv[1] - v[2] * v[1] * dv[2]) * invsum32;
    o[2] = (-v[0] * v[2] * dv[0] - v[1] * v[2] * dv[1] + (sum2 - v[2] * v[2]) * dv[2]) * invsum32;
}

/* base/cr/auxiliary.h:139-164 ; returns 1 if in frustum (near plane only). */
static int in_frustum(const float* p_orig, const float* viewmatrix, const float* projmatrix,
                      float* p_view) {
    float p_hom[4];
    transformPoint4x4(p_orig, projmatrix, p_hom); /* computed but unused, as in the reference */
    (void)p_hom;
    transformPoint4x3(p_orig, viewmatrix, p_view);
    return !(p_view[2] <= 0.2f);
}

/* base/rasterize_points.cu / rasterizer_impl.cu:141-153 + checkFrustum :54-66 */
void orc_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                      uint8_t* present) {
    for (int i = 0; i < P; i++) {
        float pv[3];
        present[i] = (uint8_t)in_frustum(means3D + 3 * i, viewmatrix, projmatrix, pv);
    }
}

/* rasterizer_impl.cu:35-50 */
uint32_t orc_get_higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

/* ------------------------------------------------------------ forward math */
/* base/cr/forward.cu:20-71 ; shs is [P, max_coeffs, 3] */
static void computeColorFromSH(int idx, int deg, int max_coeffs, const float* means,
                               const float* campos, const float* shs, uint8_t* clamped,
                               float* out) {
    const float* pos = means + 3 * idx;
    float dir[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    float len = sqrtf(dot3(dir, dir));
    dir[0] = dir[0] / len; dir[1] = dir[1] / len; dir[2] = dir[2] / len;
    const float* sh = shs + (size_t)idx * max_coeffs * 3;
    float res[3];
    for (int c = 0; c < 3; c++) res[c] = SH_C0 * sh[0 * 3 + c];
    if (deg > 0) {
        float x = dir[0], y = dir[1], z = dir[2];
        float k1 = SH_C1 * y, k2 = SH_C1 * z, k3 = SH_C1 * x;
        for (int c = 0; c < 3; c++)
            res[c] = res[c] - k1 * sh[1 * 3 + c] + k2 * sh[2 * 3 + c] - k3 * sh[3 * 3 + c];
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            float k4 = SH_C2[0] * xy;
            float k5 = SH_C2[1] * yz;
            float k6 = SH_C2[2] * (2.0f * zz - xx - yy);
            float k7 = SH_C2[3] * xz;
            float k8 = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; c++)
                res[c] = res[c] + k4 * sh[4 * 3 + c] + k5 * sh[5 * 3 + c] + k6 * sh[6 * 3 + c] +
                         k7 * sh[7 * 3 + c] + k8 * sh[8 * 3 + c];
            if (deg > 2) {
                float k9 = SH_C3[0] * y * (3.0f * xx - yy);
                float k10 = SH_C3[1] * xy * z;
                float k11 = SH_C3[2] * y * (4.0f * zz - xx - yy);
                float k12 = SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                float k13 = SH_C3[4] * x * (4.0f * zz - xx - yy);
                float k14 = SH_C3[5] * z * (xx - yy);
                float k15 = SH_C3[6] * x * (xx - 3.0f * yy);
                for (int c = 0; c < 3; c++)
                    res[c] = res[c] + k9 * sh[9 * 3 + c] + k10 * sh[10 * 3 + c] +
                             k11 * sh[11 * 3 + c] + k12 * sh[12 * 3 + c] + k13 * sh[13 * 3 + c] +
                             k14 * sh[14 * 3 + c] + k15 * sh[15 * 3 + c];
            }
        }
    }
    for (int c = 0; c < 3; c++) {
        res[c] += 0.5f;
        clamped[3 * idx + c] = (uint8_t)(res[c] < 0);
        out[c] = fmaxf(res[c], 0.0f);
    }
}

/* Test hook: the SH polynomial of computeColorFromSH (forward.cu:30-62) for a
 * given unit direction, before the +0.5 and the clamp.  sh is [max_coeffs][3]. */
void orc_eval_sh(int deg, const float* dir, const float* sh, float* out) {
    float x = dir[0], y = dir[1], z = dir[2];
    float res[3];
    for (int c = 0; c < 3; c++) res[c] = SH_C0 * sh[0 * 3 + c];
    if (deg > 0) {
        float k1 = SH_C1 * y, k2 = SH_C1 * z, k3 = SH_C1 * x;
        for (int c = 0; c < 3; c++) res[c] = res[c] - k1 * sh[1 * 3 + c] + k2 * sh[2 * 3 + c] - k3 * sh[3 * 3 + c];
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            float k4 = SH_C2[0] * xy, k5 = SH_C2[1] * yz, k6 = SH_C2[2] * (2.0f * zz - xx - yy);
            float k7 = SH_C2[3] * xz, k8 = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; c++)
                res[c] = res[c] + k4 * sh[4 * 3 + c] + k5 * sh[5 * 3 + c] + k6 * sh[6 * 3 + c] +
                         k7 * sh[7 * 3 + c] + k8 * sh[8 * 3 + c];
            if (deg > 2) {
                float k9 = SH_C3[0] * y * (3.0f * xx - yy), k10 = SH_C3[1] * xy * z;
                float k11 = SH_C3[2] * y * (4.0f * zz - xx - yy);
                float k12 = SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                float k13 = SH_C3[4] * x * (4.0f * zz - xx - yy), k14 = SH_C3[5] * z * (xx - yy);
                float k15 = SH_C3[6] * x * (xx - 3.0f * yy);
                for (int c = 0; c < 3; c++)
                    res[c] = res[c] + k9 * sh[9 * 3 + c] + k10 * sh[10 * 3 + c] + k11 * sh[11 * 3 + c] +
                             k12 * sh[12 * 3 + c] + k13 * sh[13 * 3 + c] + k14 * sh[14 * 3 + c] +
                             k15 * sh[15 * 3 + c];
            }
        }
    }
    out[0] = res[0]; out[1] = res[1]; out[2] = res[2];
}

/* base/cr/forward.cu:74-113 */
static void computeCov2D(const float* mean, float focal_x, float focal_y, float tan_fovx,
                         float tan_fovy, const float* cov3D, const float* viewmatrix, float* out) {
    float t[3];
    transformPoint4x3(mean, viewmatrix, t);
    const float limx = 1.3f * tan_fovx;
    const float limy = 1.3f * tan_fovy;
    const float txtz = t[0] / t[2];
    const float tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
    mat3 J = mat3_cols(focal_x / t[2], 0.0f, -(focal_x * t[0]) / (t[2] * t[2]), 0.0f,
                       focal_y / t[2], -(focal_y * t[1]) / (t[2] * t[2]), 0, 0, 0);
    const float* v = viewmatrix;
    mat3 W = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    mat3 T = mat3_mul(&W, &J);
    mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2],
                         cov3D[4], cov3D[5]);
    mat3 Tt = mat3_transpose(&T), Vt = mat3_transpose(&Vrk);
    mat3 tmp = mat3_mul(&Tt, &Vt);
    mat3 cov = mat3_mul(&tmp, &T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    out[0] = cov.m[0][0]; out[1] = cov.m[0][1]; out[2] = cov.m[1][1];
}

static mat3 quat_to_R(float r, float x, float y, float z) {
    return mat3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                     2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                     2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
}

/* base/cr/forward.cu:118-152 */
static void computeCov3D(const float* scale, float mod, const float* rot, float* cov3D) {
    mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale[0];
    S.m[1][1] = mod * scale[1];
    S.m[2][2] = mod * scale[2];
    mat3 R = quat_to_R(rot[0], rot[1], rot[2], rot[3]);
    mat3 M = mat3_mul(&S, &R);
    mat3 Mt = mat3_transpose(&M);
    mat3 Sigma = mat3_mul(&Mt, &M);
    cov3D[0] = Sigma.m[0][0]; cov3D[1] = Sigma.m[0][1]; cov3D[2] = Sigma.m[0][2];
    cov3D[3] = Sigma.m[1][1]; cov3D[4] = Sigma.m[1][2]; cov3D[5] = Sigma.m[2][2];
}

/* base/cr/forward.cu:155-256 (preprocessCUDA<3>); block_x/block_y = tile size. */
void orc_preprocess(int P, int D, int M, const float* orig_points, const float* scales,
                    float scale_modifier, const float* rotations, const float* opacities,
                    const float* shs, uint8_t* clamped, const float* cov3D_precomp,
                    const float* colors_precomp, const float* viewmatrix, const float* projmatrix,
                    const float* cam_pos, int W, int H, float tan_fovx, float tan_fovy,
                    float focal_x, float focal_y, int block_x, int block_y, int* radii,
                    float* points_xy_image, float* depths, float* cov3Ds, float* rgb,
                    float* conic_opacity, uint32_t* tiles_touched, int prefiltered) {
    (void)prefiltered;
    const unsigned gx = (unsigned)((W + block_x - 1) / block_x);
    const unsigned gy = (unsigned)((H + block_y - 1) / block_y);
#pragma omp parallel for schedule(static, 4096) num_threads(g_threads) if (g_threads > 1)
    for (int idx = 0; idx < P; idx++) {
        radii[idx] = 0;
        tiles_touched[idx] = 0;
        const float* p_orig = orig_points + 3 * idx;
        float p_view[3];
        if (!in_frustum(p_orig, viewmatrix, projmatrix, p_view)) continue;
        float p_hom[4];
        transformPoint4x4(p_orig, projmatrix, p_hom);
        float p_w = 1.0f / (p_hom[3] + 0.0000001f);
        float p_proj[3] = {p_hom[0] * p_w, p_hom[1] * p_w, p_hom[2] * p_w};
        const float* cov3D;
        if (cov3D_precomp != NULL) {
            cov3D = cov3D_precomp + 6 * idx;
        } else {
            computeCov3D(scales + 3 * idx, scale_modifier, rotations + 4 * idx, cov3Ds + 6 * idx);
            cov3D = cov3Ds + 6 * idx;
        }
        float cov[3];
        computeCov2D(p_orig, focal_x, focal_y, tan_fovx, tan_fovy, cov3D, viewmatrix, cov);
        float det = (cov[0] * cov[2] - cov[1] * cov[1]);
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
        float mid = 0.5f * (cov[0] + cov[2]);
        float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
        float pix[2] = {ndc2Pix(p_proj[0], W), ndc2Pix(p_proj[1], H)};
        unsigned rmin[2], rmax[2];
        getRect(pix[0], pix[1], (int)my_radius, block_x, block_y, gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        if (colors_precomp == NULL) {
            float res[3];
            computeColorFromSH(idx, D, M, orig_points, cam_pos, shs, clamped, res);
            rgb[idx * 3 + 0] = res[0];
            rgb[idx * 3 + 1] = res[1];
            rgb[idx * 3 + 2] = res[2];
        }
        depths[idx] = p_view[2];
        radii[idx] = (int)my_radius;
        points_xy_image[2 * idx + 0] = pix[0];
        points_xy_image[2 * idx + 1] = pix[1];
        conic_opacity[4 * idx + 0] = conic[0];
        conic_opacity[4 * idx + 1] = conic[1];
        conic_opacity[4 * idx + 2] = conic[2];
        conic_opacity[4 * idx + 3] = opacities[idx];
        tiles_touched[idx] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
    }
}

/* rasterizer_impl.cu:277 cub::DeviceScan::InclusiveSum */
void orc_inclusive_scan_u32(int n, const uint32_t* in, uint32_t* out) {
    uint32_t acc = 0;
    for (int i = 0; i < n; i++) { acc += in[i]; out[i] = acc; }
}

/* rasterizer_impl.cu:70-111 */
void orc_duplicate_with_keys(int P, const float* points_xy, const float* depths,
                             const uint32_t* offsets, const int* radii, int W, int H, int block_x,
                             int block_y, uint64_t* keys, uint32_t* values) {
    const unsigned gx = (unsigned)((W + block_x - 1) / block_x);
    const unsigned gy = (unsigned)((H + block_y - 1) / block_y);
#pragma omp parallel for schedule(dynamic, 4096) num_threads(g_threads) if (g_threads > 1)
    for (int idx = 0; idx < P; idx++) {
        if (radii[idx] > 0) {
            uint32_t off = (idx == 0) ? 0 : offsets[idx - 1];
            unsigned rmin[2], rmax[2];
            getRect(points_xy[2 * idx], points_xy[2 * idx + 1], radii[idx], block_x, block_y, gx,
                    gy, rmin, rmax);
            uint32_t dbits;
            memcpy(&dbits, &depths[idx], 4);
            for (unsigned y = rmin[1]; y < rmax[1]; y++)
                for (unsigned x = rmin[0]; x < rmax[0]; x++) {
                    uint64_t key = (uint64_t)(y * gx + x);
                    key <<= 32;
                    key |= dbits;
                    keys[off] = key;
                    values[off] = (uint32_t)idx;
                    off++;
                }
        }
    }
}

/* rasterizer_impl.cu:303-308 cub::DeviceRadixSort::SortPairs(begin_bit 0, end_bit):
 * a STABLE LSD radix sort on bits [0, end_bit).  In-place on (keys, values). */
void orc_sort_pairs_u64(int n, uint64_t* keys, uint32_t* values, int end_bit) {
    if (n <= 1) return;
    uint64_t* k2 = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
    uint32_t* v2 = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
    uint64_t *ks = keys, *kd = k2;
    uint32_t *vs = values, *vd = v2;
    for (int shift = 0; shift < end_bit; shift += 8) {
        size_t cnt[257];
        memset(cnt, 0, sizeof(cnt));
        uint64_t mask = (end_bit - shift >= 8) ? 0xFFull : ((1ull << (end_bit - shift)) - 1);
        for (int i = 0; i < n; i++) cnt[((ks[i] >> shift) & mask) + 1]++;
        for (int b = 0; b < 256; b++) cnt[b + 1] += cnt[b];
        for (int i = 0; i < n; i++) {
            size_t d = cnt[(ks[i] >> shift) & mask]++;
            kd[d] = ks[i];
            vd[d] = vs[i];
        }
        uint64_t* tk = ks; ks = kd; kd = tk;
        uint32_t* tv = vs; vs = vd; vd = tv;
    }
    if (ks != keys) {
        memcpy(keys, ks, sizeof(uint64_t) * (size_t)n);
        memcpy(values, vs, sizeof(uint32_t) * (size_t)n);
    }
    free(k2);
    free(v2);
}

/* rasterizer_impl.cu:116-138 (+ memset :310).  ranges is uint2[T] (x,y interleaved). */
void orc_identify_tile_ranges(int L, const uint64_t* keys, int T, uint32_t* ranges) {
    memset(ranges, 0, sizeof(uint32_t) * 2 * (size_t)T);
    for (int idx = 0; idx < L; idx++) {
        uint32_t currtile = (uint32_t)(keys[idx] >> 32);
        if (idx == 0) ranges[2 * currtile + 0] = 0;
        else {
            uint32_t prevtile = (uint32_t)(keys[idx - 1] >> 32);
            if (currtile != prevtile) {
                ranges[2 * prevtile + 1] = (uint32_t)idx;
                ranges[2 * currtile + 0] = (uint32_t)idx;
            }
        }
        if (idx == L - 1) ranges[2 * currtile + 1] = (uint32_t)L;
    }
}

/* Per-pixel front-to-back blend of one range: base/cr/forward.cu:300-373
 * (block-level __syncthreads_count exit does not change any per-pixel result). */
static void blend_pixel(uint32_t rx, uint32_t ry, const uint32_t* point_list, float pixx,
                        float pixy, const float* points_xy, const float* features,
                        const float* conic_opacity, float* T_out, uint32_t* ncontrib_out,
                        float* C) {
    float T = 1.0f;
    uint32_t contributor = 0, last_contributor = 0;
    C[0] = C[1] = C[2] = 0.0f;
    for (uint32_t p = rx; p < ry; p++) {
        contributor++;
        uint32_t id = point_list[p];
        float dx = points_xy[2 * id] - pixx, dy = points_xy[2 * id + 1] - pixy;
        const float* co = conic_opacity + 4 * id;
        float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        if (power > 0.0f) continue;
        float alpha = fminf(0.99f, co[3] * expf(power));
        if (alpha < 1.0f / 255.0f) continue;
        float test_T = T * (1 - alpha);
        if (test_T < 0.0001f) break; /* done = true */
        for (int ch = 0; ch < NUM_CHANNELS; ch++) C[ch] += features[id * 3 + ch] * alpha * T;
        T = test_T;
        last_contributor = contributor;
    }
    *T_out = T;
    *ncontrib_out = last_contributor;
}

/* base/cr/forward.cu:261-374 (renderCUDA<3>), tile size block_x x block_y */
void orc_render_forward(int W, int H, int block_x, int block_y, const uint32_t* ranges,
                        const uint32_t* point_list, const float* points_xy, const float* features,
                        const float* conic_opacity, float* final_T, uint32_t* n_contrib,
                        const float* bg_color, float* out_color) {
    const int gx = (W + block_x - 1) / block_x;
#pragma omp parallel for schedule(dynamic, 1) num_threads(g_threads) if (g_threads > 1)
    for (int py = 0; py < H; py++)
        for (int px = 0; px < W; px++) {
            int tile = (py / block_y) * gx + (px / block_x);
            float T, C[3];
            uint32_t nc;
            blend_pixel(ranges[2 * tile], ranges[2 * tile + 1], point_list, (float)px, (float)py,
                        points_xy, features, conic_opacity, &T, &nc, C);
            size_t pid = (size_t)W * py + px;
            final_T[pid] = T;
            n_contrib[pid] = nc;
            for (int ch = 0; ch < 3; ch++)
                out_color[(size_t)ch * H * W + pid] = C[ch] + T * bg_color[ch];
        }
}

/* ---- Conditioning of the blend's discrete decisions (TEST SUPPORT, not the
 * reference's algorithm).  A pixel's blend takes three discrete decisions
 * per list entry (base/cr/forward.cu:337-350): the `power > 0` skip, the
 * `alpha < 1/255` skip and the `test_T < 1e-4` stop.  Where one is taken
 * within the rounding error any float32 evaluation of the same formulas
 * carries, a last-bit difference in an operand (another exp implementation,
 * another operation order) switches it, and the gradient of every Gaussian
 * on that pixel's chain jumps: the gradient is discontinuous there.  The
 * margins:
 *   power:  |power| <= kTieRel * S, S = |cx dx^2| / 2 + |cz dy^2| / 2 + |cy dx dy|
 *           (the terms it is summed from);
 *   alpha:  |ln(255 alpha)| <= kTieRel * (1 + S) (exp of an argument known to
 *           kTieRel * S; alpha clamped at 0.99 is exact);
 *   T:      |test_T - 1e-4| <= 1e-4 * eT, eT the running relative error bound of
 *           T (kTieRel per blend plus the alpha error times alpha / (1 - alpha)),
 * with kTieRel = 32 * 2^-24 (a few ulps of each operand).
 * orc_render_tie_allowance replays every such decision the other way, one
 * at a time, and adds |terms(flipped) - terms(as taken)| of every chain entry
 * to allowance[gid][0..8] (the nine blend-backward terms of bwd_pixel): the
 * exact jump each near-tie decision can make.  The element-wise gradient
 * tests (tests/gs_helpers.py) add it to their bound. */
#define kTieRel (32.0f / 16777216.0f)
#define TIE_POWER 1
#define TIE_ALPHA 2
#define TIE_T 4

/* Forward replay of one pixel (blend_pixel's decisions) with the decision of
 * kind `fkind` at entry `fp` inverted (fkind 0: none).  Returns the final T
 * and last contributor; with ties != NULL records up to max_ties near-tie
 * decisions (entry, kind) of the unforced replay. */
static void tie_forward(uint32_t rx, uint32_t ry, const uint32_t* point_list, float pixx, float pixy,
                        const float* points_xy, const float* conic_opacity, uint32_t fp, int fkind,
                        float* T_out, uint32_t* nc_out, uint32_t* ties, int* nties, int max_ties) {
    float T = 1.0f, eT = 0.0f;
    uint32_t contributor = 0, last_contributor = 0;
    for (uint32_t p = rx; p < ry; p++) {
        contributor++;
        const uint32_t id = point_list[p];
        const float dx = points_xy[2 * id] - pixx, dy = points_xy[2 * id + 1] - pixy;
        const float* co = conic_opacity + 4 * id;
        const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        const float S = 0.5f * fabsf(co[0] * dx * dx) + 0.5f * fabsf(co[2] * dy * dy) + fabsf(co[1] * dx * dy);
        int near = 0;
        if (S > 0.0f && fabsf(power) <= kTieRel * S) near |= TIE_POWER;
        int skip = power > 0.0f;
        if (p == fp && fkind == TIE_POWER) skip = !skip;
        float alpha = 0.0f, ea = 0.0f;
        if (!skip) {
            alpha = fminf(0.99f, co[3] * expf(power));
            ea = alpha < 0.99f ? kTieRel * (1.0f + S) : 0.0f;
            if (fabsf(logf(255.0f * alpha)) <= ea) near |= TIE_ALPHA;
            int askip = alpha < 1.0f / 255.0f;
            if (p == fp && fkind == TIE_ALPHA) askip = !askip;
            skip = askip;
        }
        if (!skip) {
            const float test_T = T * (1 - alpha);
            eT += kTieRel + ea * alpha / (1.0f - alpha);
            if (fabsf(test_T - 0.0001f) <= 0.0001f * eT) near |= TIE_T;
            int stop = test_T < 0.0001f;
            if (p == fp && fkind == TIE_T) stop = !stop;
            if (ties)
                for (int k = 1; k <= 4; k <<= 1)
                    if ((near & k) && *nties < max_ties) { ties[2 * *nties] = p; ties[2 * *nties + 1] = (uint32_t)k; (*nties)++; }
            if (stop) break;
            T = test_T;
            last_contributor = contributor;
        } else if (ties) {
            for (int k = 1; k <= 2; k <<= 1)
                if ((near & k) && *nties < max_ties) { ties[2 * *nties] = p; ties[2 * *nties + 1] = (uint32_t)k; (*nties)++; }
        }
    }
    *T_out = T;
    *nc_out = last_contributor;
}

/* bwd_pixel's nine terms of every chain entry into terms[(p - rx) * 9 + q]
 * (zeroed first), with the forced decision as in tie_forward. */
static void tie_terms(int W, int H, int px, int py, uint32_t rx, uint32_t ry, const uint32_t* point_list,
                      const float* bg_color, const float* points_xy, const float* conic_opacity,
                      const float* colors, float T_final, uint32_t last_contributor, const float* dL_dpixel,
                      uint32_t fp, int fkind, float* terms) {
    const float ddelx_dx = (float)(0.5 * W);
    const float ddely_dy = (float)(0.5 * H);
    memset(terms, 0, sizeof(float) * 9 * (size_t)(ry - rx));
    float T = T_final;
    uint32_t contributor = ry - rx;
    float accum_rec[3] = {0, 0, 0}, last_color[3] = {0, 0, 0};
    float last_alpha = 0;
    const float pixx = (float)px, pixy = (float)py;
    for (uint32_t q = ry; q > rx; q--) {
        const uint32_t p = q - 1;
        contributor--;
        if (contributor >= last_contributor) continue;
        const uint32_t gid = point_list[p];
        const float dx = points_xy[2 * gid] - pixx, dy = points_xy[2 * gid + 1] - pixy;
        const float* co = conic_opacity + 4 * gid;
        const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        int skip = power > 0.0f;
        if (p == fp && fkind == TIE_POWER) skip = !skip;
        if (skip) continue;
        const float G = expf(power);
        const float alpha = fminf(0.99f, co[3] * G);
        int askip = alpha < 1.0f / 255.0f;
        if (p == fp && fkind == TIE_ALPHA) askip = !askip;
        if (askip) continue;
        float* a = terms + 9 * (size_t)(p - rx);
        T = T / (1.f - alpha);
        const float dchannel_dcolor = alpha * T;
        float dL_dalpha = 0.0f;
        for (int ch = 0; ch < 3; ch++) {
            const float c = colors[gid * 3 + ch];
            accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
            last_color[ch] = c;
            dL_dalpha += (c - accum_rec[ch]) * dL_dpixel[ch];
            a[ch] = dchannel_dcolor * dL_dpixel[ch];
        }
        dL_dalpha *= T;
        last_alpha = alpha;
        float bg_dot_dpixel = 0;
        for (int i = 0; i < 3; i++) bg_dot_dpixel += bg_color[i] * dL_dpixel[i];
        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
        const float dL_dG = co[3] * dL_dalpha;
        const float gdx = G * dx, gdy = G * dy;
        const float dG_ddelx = -gdx * co[0] - gdy * co[1];
        const float dG_ddely = -gdy * co[2] - gdx * co[1];
        a[3] = dL_dG * dG_ddelx * ddelx_dx;
        a[4] = dL_dG * dG_ddely * ddely_dy;
        a[5] = -0.5f * gdx * dx * dL_dG;
        a[6] = -0.5f * gdx * dy * dL_dG;
        a[7] = -0.5f * gdy * dy * dL_dG;
        a[8] = G * dL_dalpha;
    }
}

/* allowance [P, 9] (double, accumulated); counts[0] = pixels with a
 * near-tie decision, counts[1..3] = decisions of kind power / alpha / T. */
void orc_render_tie_allowance(int W, int H, int block_x, int block_y, const uint32_t* ranges,
                              const uint32_t* point_list, const float* bg_color, const float* points_xy,
                              const float* conic_opacity, const float* colors, const float* dL_dpixels, int P,
                              double* allowance, long* counts) {
    const int gx = (W + block_x - 1) / block_x;
    long npix = 0, nk[3] = {0, 0, 0};
    enum { kMaxTies = 64 };
#pragma omp parallel num_threads(g_threads) if (g_threads > 1) reduction(+ : npix, nk[:3])
    {
        float* t0 = NULL;
        float* t1 = NULL;
        size_t cap = 0;
        uint32_t ties[2 * kMaxTies];
#pragma omp for schedule(dynamic, 1)
        for (int py = 0; py < H; py++)
            for (int px = 0; px < W; px++) {
                const int tile = (py / block_y) * gx + (px / block_x);
                const uint32_t rx = ranges[2 * tile], ry = ranges[2 * tile + 1];
                float T;
                uint32_t nc;
                int nt = 0;
                tie_forward(rx, ry, point_list, (float)px, (float)py, points_xy, conic_opacity, 0xffffffffu, 0, &T,
                            &nc, ties, &nt, kMaxTies);
                if (nt == 0) continue;
                npix++;
                if (cap < (size_t)(ry - rx)) {
                    cap = (size_t)(ry - rx);
                    t0 = (float*)realloc(t0, sizeof(float) * 9 * cap);
                    t1 = (float*)realloc(t1, sizeof(float) * 9 * cap);
                }
                const size_t pid = (size_t)W * py + px;
                const float dpx[3] = {dL_dpixels[pid], dL_dpixels[(size_t)H * W + pid], dL_dpixels[2 * (size_t)H * W + pid]};
                tie_terms(W, H, px, py, rx, ry, point_list, bg_color, points_xy, conic_opacity, colors, T, nc, dpx,
                          0xffffffffu, 0, t0);
                for (int k = 0; k < nt; k++) {
                    const uint32_t fp = ties[2 * k];
                    const int kind = (int)ties[2 * k + 1];
                    nk[kind == TIE_POWER ? 0 : kind == TIE_ALPHA ? 1 : 2]++;
                    float Tf;
                    uint32_t ncf;
                    tie_forward(rx, ry, point_list, (float)px, (float)py, points_xy, conic_opacity, fp, kind, &Tf, &ncf,
                                NULL, NULL, 0);
                    tie_terms(W, H, px, py, rx, ry, point_list, bg_color, points_xy, conic_opacity, colors, Tf, ncf,
                              dpx, fp, kind, t1);
                    for (uint32_t p = rx; p < ry; p++) {
                        const float* u = t0 + 9 * (size_t)(p - rx);
                        const float* v = t1 + 9 * (size_t)(p - rx);
                        double* al = allowance + 9 * (size_t)point_list[p];
                        for (int q = 0; q < 9; q++) {
                            const double d = fabs((double)v[q] - (double)u[q]);
                            if (d != 0.0) {
#pragma omp atomic
                                al[q] += d;
                            }
                        }
                    }
                }
            }
        free(t0);
        free(t1);
    }
    counts[0] = npix;
    counts[1] = nk[0];
    counts[2] = nk[1];
    counts[3] = nk[2];
}

/* base/cr/backward.cu:399-557 (renderCUDA<3> backward), one pixel: adds its
 * nine per-Gaussian terms to acc[gid * stride + 0..8] in double (the exact
 * sum of the reference's float atomics). */
static void bwd_pixel(int W, int H, int px, int py, uint32_t rx, uint32_t ry,
                      const uint32_t* point_list, const float* bg_color, const float* points_xy,
                      const float* conic_opacity, const float* colors, const float* final_Ts,
                      const uint32_t* n_contrib, const float* dL_dpixels, double* acc, int stride,
                      int absolute) {
/* absolute: accumulate |term| instead (orc_render_backward_abs) */
#define ACC(i, v) (a[i] += absolute ? fabs((double)(v)) : (double)(v))
    const float ddelx_dx = (float)(0.5 * W);
    const float ddely_dy = (float)(0.5 * H);
    size_t pid = (size_t)W * py + px;
    const float T_final = final_Ts[pid];
    float T = T_final;
    uint32_t contributor = ry - rx;
    const uint32_t last_contributor = n_contrib[pid];
    float accum_rec[3] = {0, 0, 0}, dL_dpixel[3], last_color[3] = {0, 0, 0};
    float last_alpha = 0;
    for (int i = 0; i < 3; i++) dL_dpixel[i] = dL_dpixels[(size_t)i * H * W + pid];
    const float pixx = (float)px, pixy = (float)py;
    for (uint32_t q = ry; q > rx; q--) {
        uint32_t p = q - 1;
        contributor--;
        if (contributor >= last_contributor) continue;
        uint32_t gid = point_list[p];
        double* a = acc + (size_t)gid * stride;
        float dx = points_xy[2 * gid] - pixx, dy = points_xy[2 * gid + 1] - pixy;
        const float* co = conic_opacity + 4 * gid;
        float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        if (power > 0.0f) continue;
        const float G = expf(power);
        const float alpha = fminf(0.99f, co[3] * G);
        if (alpha < 1.0f / 255.0f) continue;
        T = T / (1.f - alpha);
        const float dchannel_dcolor = alpha * T;
        float dL_dalpha = 0.0f;
        for (int ch = 0; ch < 3; ch++) {
            const float c = colors[gid * 3 + ch];
            accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
            last_color[ch] = c;
            const float dL_dchannel = dL_dpixel[ch];
            dL_dalpha += (c - accum_rec[ch]) * dL_dchannel;
            ACC(0 + ch, dchannel_dcolor * dL_dchannel);
        }
        dL_dalpha *= T;
        last_alpha = alpha;
        float bg_dot_dpixel = 0;
        for (int i = 0; i < 3; i++) bg_dot_dpixel += bg_color[i] * dL_dpixel[i];
        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
        const float dL_dG = co[3] * dL_dalpha;
        const float gdx = G * dx;
        const float gdy = G * dy;
        const float dG_ddelx = -gdx * co[0] - gdy * co[1];
        const float dG_ddely = -gdy * co[2] - gdx * co[1];
        ACC(3, dL_dG * dG_ddelx * ddelx_dx);
        ACC(4, dL_dG * dG_ddely * ddely_dy);
        ACC(5, -0.5f * gdx * dx * dL_dG);
        ACC(6, -0.5f * gdx * dy * dL_dG);
        ACC(7, -0.5f * gdy * dy * dL_dG);
        ACC(8, G * dL_dalpha);
    }
}
#undef ACC

/* base/cr/backward.cu:399-557 (renderCUDA<3> backward).  Accumulates in double
 * (the exact sum of the reference's float atomics). dL_dconic is [P,4] (2x2).
 * With g_threads > 1 the image is cut into g_threads bands of tile rows, each
 * summed into its own accumulator (pixel order within a band as the serial
 * loop), and the bands are added in band order. */
void orc_render_backward(int W, int H, int block_x, int block_y, const uint32_t* ranges,
                         const uint32_t* point_list, const float* bg_color, const float* points_xy,
                         const float* conic_opacity, const float* colors, const float* final_Ts,
                         const uint32_t* n_contrib, const float* dL_dpixels, int P,
                         float* dL_dmean2D, float* dL_dconic2D, float* dL_dopacity,
                         float* dL_dcolors) {
    const int gx = (W + block_x - 1) / block_x;
    const int gy = (H + block_y - 1) / block_y;
    const int nb = g_threads > 1 ? (g_threads < gy ? g_threads : (gy > 0 ? gy : 1)) : 1;
    const int stride = 9;
    double* acc = (double*)calloc((size_t)P * stride * (size_t)nb, sizeof(double));
#pragma omp parallel for schedule(dynamic, 1) num_threads(nb) if (nb > 1)
    for (int b = 0; b < nb; b++) {
        const int ty0 = (int)((long)gy * b / nb), ty1 = (int)((long)gy * (b + 1) / nb);
        const int py0 = ty0 * block_y, py1 = ty1 * block_y < H ? ty1 * block_y : H;
        double* a = acc + (size_t)P * stride * (size_t)b;
        for (int py = py0; py < py1; py++)
            for (int px = 0; px < W; px++) {
                int tile = (py / block_y) * gx + (px / block_x);
                bwd_pixel(W, H, px, py, ranges[2 * tile], ranges[2 * tile + 1], point_list, bg_color,
                          points_xy, conic_opacity, colors, final_Ts, n_contrib, dL_dpixels, a, stride, 0);
            }
    }
#pragma omp parallel for schedule(static, 4096) num_threads(g_threads) if (g_threads > 1)
    for (int g = 0; g < P; g++) {
        double s[9];
        for (int q = 0; q < 9; q++) s[q] = acc[(size_t)g * stride + q];
        for (int b = 1; b < nb; b++)
            for (int q = 0; q < 9; q++) s[q] += acc[((size_t)P * b + g) * stride + q];
        dL_dcolors[3 * g + 0] = (float)s[0];
        dL_dcolors[3 * g + 1] = (float)s[1];
        dL_dcolors[3 * g + 2] = (float)s[2];
        dL_dmean2D[3 * g + 0] = (float)s[3];
        dL_dmean2D[3 * g + 1] = (float)s[4];
        dL_dmean2D[3 * g + 2] = 0.0f;
        dL_dconic2D[4 * g + 0] = (float)s[5];
        dL_dconic2D[4 * g + 1] = (float)s[6];
        dL_dconic2D[4 * g + 2] = 0.0f;
        dL_dconic2D[4 * g + 3] = (float)s[7];
        dL_dopacity[g] = (float)s[8];
    }
    free(acc);
}

/* Test support: per Gaussian the sums of |term| of the nine blend-backward
 * terms (orc_render_backward's sums with every term's magnitude), S[P][9]
 * in double.  Any float32 summation order of those terms (the GPU's
 * float atomics) is within a small multiple of 2^-24 S of the exact sum;
 * the element-wise gradient tests derive their accumulation allowance from
 * it (oracle.py grad_allowance). */
void orc_render_backward_abs(int W, int H, int block_x, int block_y, const uint32_t* ranges,
                             const uint32_t* point_list, const float* bg_color, const float* points_xy,
                             const float* conic_opacity, const float* colors, const float* final_Ts,
                             const uint32_t* n_contrib, const float* dL_dpixels, int P, double* S) {
    const int gx = (W + block_x - 1) / block_x;
    const int gy = (H + block_y - 1) / block_y;
    const int nb = g_threads > 1 ? (g_threads < gy ? g_threads : (gy > 0 ? gy : 1)) : 1;
    const int stride = 9;
    double* acc = nb > 1 ? (double*)calloc((size_t)P * stride * (size_t)(nb - 1), sizeof(double)) : NULL;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nb) if (nb > 1)
    for (int b = 0; b < nb; b++) {
        const int ty0 = (int)((long)gy * b / nb), ty1 = (int)((long)gy * (b + 1) / nb);
        const int py0 = ty0 * block_y, py1 = ty1 * block_y < H ? ty1 * block_y : H;
        double* a = b == 0 ? S : acc + (size_t)P * stride * (size_t)(b - 1);
        for (int py = py0; py < py1; py++)
            for (int px = 0; px < W; px++) {
                int tile = (py / block_y) * gx + (px / block_x);
                bwd_pixel(W, H, px, py, ranges[2 * tile], ranges[2 * tile + 1], point_list, bg_color,
                          points_xy, conic_opacity, colors, final_Ts, n_contrib, dL_dpixels, a, stride, 1);
            }
    }
    if (acc) {
#pragma omp parallel for schedule(static, 4096) num_threads(g_threads) if (g_threads > 1)
        for (int g = 0; g < P; g++)
            for (int b = 1; b < nb; b++)
                for (int q = 0; q < 9; q++) S[(size_t)g * stride + q] += acc[((size_t)P * (b - 1) + g) * stride + q];
        free(acc);
    }
}

/* base/cr/backward.cu:144-274 (computeCov2DCUDA) */
void orc_cov2d_backward(int P, const float* means, const int* radii, const float* cov3Ds,
                        float h_x, float h_y, float tan_fovx, float tan_fovy,
                        const float* view_matrix, const float* dL_dconics, float* dL_dmeans,
                        float* dL_dcov) {
#pragma omp parallel for schedule(static, 4096) num_threads(g_threads) if (g_threads > 1)
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        const float* cov3D = cov3Ds + 6 * idx;
        const float* mean = means + 3 * idx;
        float dL_dconic[3] = {dL_dconics[4 * idx], dL_dconics[4 * idx + 1], dL_dconics[4 * idx + 3]};
        float t[3];
        transformPoint4x3(mean, view_matrix, t);
        const float limx = 1.3f * tan_fovx;
        const float limy = 1.3f * tan_fovy;
        const float txtz = t[0] / t[2];
        const float tytz = t[1] / t[2];
        t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
        t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
        const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
        const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
        mat3 J = mat3_cols(h_x / t[2], 0.0f, -(h_x * t[0]) / (t[2] * t[2]), 0.0f, h_y / t[2],
                           -(h_y * t[1]) / (t[2] * t[2]), 0, 0, 0);
        const float* v = view_matrix;
        mat3 W = mat3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
        mat3 Vrk = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2],
                             cov3D[4], cov3D[5]);
        mat3 T = mat3_mul(&W, &J);
        mat3 Tt = mat3_transpose(&T), Vt = mat3_transpose(&Vrk);
        mat3 tmp = mat3_mul(&Tt, &Vt);
        mat3 cov2D = mat3_mul(&tmp, &T);
        float a = cov2D.m[0][0] += 0.3f;
        float b = cov2D.m[0][1];
        float c = cov2D.m[1][1] += 0.3f;
        float denom = a * c - b * b;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float* dc = dL_dcov + 6 * idx;
        const float (*Tm)[3] = (const float (*)[3])T.m;
        const float (*Vm)[3] = (const float (*)[3])Vrk.m;
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c * c * dL_dconic[0] + 2 * b * c * dL_dconic[1] +
                                 (denom - a * c) * dL_dconic[2]);
            dL_dc = denom2inv * (-a * a * dL_dconic[2] + 2 * a * b * dL_dconic[1] +
                                 (denom - a * c) * dL_dconic[0]);
            dL_db = denom2inv * 2 *
                    (b * c * dL_dconic[0] - (denom + 2 * b * b) * dL_dconic[1] + a * b * dL_dconic[2]);
            dc[0] = (Tm[0][0] * Tm[0][0] * dL_da + Tm[0][0] * Tm[1][0] * dL_db + Tm[1][0] * Tm[1][0] * dL_dc);
            dc[3] = (Tm[0][1] * Tm[0][1] * dL_da + Tm[0][1] * Tm[1][1] * dL_db + Tm[1][1] * Tm[1][1] * dL_dc);
            dc[5] = (Tm[0][2] * Tm[0][2] * dL_da + Tm[0][2] * Tm[1][2] * dL_db + Tm[1][2] * Tm[1][2] * dL_dc);
            dc[1] = 2 * Tm[0][0] * Tm[0][1] * dL_da + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_db + 2 * Tm[1][0] * Tm[1][1] * dL_dc;
            dc[2] = 2 * Tm[0][0] * Tm[0][2] * dL_da + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_db + 2 * Tm[1][0] * Tm[1][2] * dL_dc;
            dc[4] = 2 * Tm[0][2] * Tm[0][1] * dL_da + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_db + 2 * Tm[1][1] * Tm[1][2] * dL_dc;
        } else {
            for (int i = 0; i < 6; i++) dc[i] = 0;
        }
        float dL_dT00 = 2 * (Tm[0][0] * Vm[0][0] + Tm[0][1] * Vm[0][1] + Tm[0][2] * Vm[0][2]) * dL_da +
                        (Tm[1][0] * Vm[0][0] + Tm[1][1] * Vm[0][1] + Tm[1][2] * Vm[0][2]) * dL_db;
        float dL_dT01 = 2 * (Tm[0][0] * Vm[1][0] + Tm[0][1] * Vm[1][1] + Tm[0][2] * Vm[1][2]) * dL_da +
                        (Tm[1][0] * Vm[1][0] + Tm[1][1] * Vm[1][1] + Tm[1][2] * Vm[1][2]) * dL_db;
        float dL_dT02 = 2 * (Tm[0][0] * Vm[2][0] + Tm[0][1] * Vm[2][1] + Tm[0][2] * Vm[2][2]) * dL_da +
                        (Tm[1][0] * Vm[2][0] + Tm[1][1] * Vm[2][1] + Tm[1][2] * Vm[2][2]) * dL_db;
        float dL_dT10 = 2 * (Tm[1][0] * Vm[0][0] + Tm[1][1] * Vm[0][1] + Tm[1][2] * Vm[0][2]) * dL_dc +
                        (Tm[0][0] * Vm[0][0] + Tm[0][1] * Vm[0][1] + Tm[0][2] * Vm[0][2]) * dL_db;
        float dL_dT11 = 2 * (Tm[1][0] * Vm[1][0] + Tm[1][1] * Vm[1][1] + Tm[1][2] * Vm[1][2]) * dL_dc +
                        (Tm[0][0] * Vm[1][0] + Tm[0][1] * Vm[1][1] + Tm[0][2] * Vm[1][2]) * dL_db;
        float dL_dT12 = 2 * (Tm[1][0] * Vm[2][0] + Tm[1][1] * Vm[2][1] + Tm[1][2] * Vm[2][2]) * dL_dc +
                        (Tm[0][0] * Vm[2][0] + Tm[0][1] * Vm[2][1] + Tm[0][2] * Vm[2][2]) * dL_db;
        const float (*Wm)[3] = (const float (*)[3])W.m;
        float dL_dJ00 = Wm[0][0] * dL_dT00 + Wm[0][1] * dL_dT01 + Wm[0][2] * dL_dT02;
        float dL_dJ02 = Wm[2][0] * dL_dT00 + Wm[2][1] * dL_dT01 + Wm[2][2] * dL_dT02;
        float dL_dJ11 = Wm[1][0] * dL_dT10 + Wm[1][1] * dL_dT11 + Wm[1][2] * dL_dT12;
        float dL_dJ12 = Wm[2][0] * dL_dT10 + Wm[2][1] * dL_dT11 + Wm[2][2] * dL_dT12;
        float tz = 1.f / t[2];
        float tz2 = tz * tz;
        float tz3 = tz2 * tz;
        float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
        float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
        float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t[0]) * tz3 * dL_dJ02 +
                       (2 * h_y * t[1]) * tz3 * dL_dJ12;
        float dt[3] = {dL_dtx, dL_dty, dL_dtz};
        transformVec4x3Transpose(dt, view_matrix, dL_dmeans + 3 * idx); /* assign (=) */
    }
}

/* base/cr/backward.cu:20-139 (computeColorFromSH backward) */
static void computeColorFromSH_bwd(int idx, int deg, int max_coeffs, const float* means,
                                   const float* campos, const float* shs, const uint8_t* clamped,
                                   const float* dL_dcolor, float* dL_dmeans, float* dL_dshs) {
    const float* pos = means + 3 * idx;
    float dir_orig[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    float len = sqrtf(dot3(dir_orig, dir_orig));
    float dir[3] = {dir_orig[0] / len, dir_orig[1] / len, dir_orig[2] / len};
    const float* sh = shs + (size_t)idx * max_coeffs * 3;
    float dL_dRGB[3];
    for (int c = 0; c < 3; c++)
        dL_dRGB[c] = dL_dcolor[3 * idx + c] * (clamped[3 * idx + c] ? 0.0f : 1.0f);
    float dRGBdx[3] = {0, 0, 0}, dRGBdy[3] = {0, 0, 0}, dRGBdz[3] = {0, 0, 0};
    float x = dir[0], y = dir[1], z = dir[2];
    float* dsh = dL_dshs + (size_t)idx * max_coeffs * 3;
#define SH(k, c) sh[(k) * 3 + (c)]
#define DSH(k, c) dsh[(k) * 3 + (c)]
    float dRGBdsh0 = SH_C0;
    for (int c = 0; c < 3; c++) DSH(0, c) = dRGBdsh0 * dL_dRGB[c];
    if (deg > 0) {
        float d1 = -SH_C1 * y, d2 = SH_C1 * z, d3 = -SH_C1 * x;
        for (int c = 0; c < 3; c++) {
            DSH(1, c) = d1 * dL_dRGB[c];
            DSH(2, c) = d2 * dL_dRGB[c];
            DSH(3, c) = d3 * dL_dRGB[c];
            dRGBdx[c] = -SH_C1 * SH(3, c);
            dRGBdy[c] = -SH_C1 * SH(1, c);
            dRGBdz[c] = SH_C1 * SH(2, c);
        }
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            float d4 = SH_C2[0] * xy, d5 = SH_C2[1] * yz, d6 = SH_C2[2] * (2.f * zz - xx - yy);
            float d7 = SH_C2[3] * xz, d8 = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; c++) {
                DSH(4, c) = d4 * dL_dRGB[c];
                DSH(5, c) = d5 * dL_dRGB[c];
                DSH(6, c) = d6 * dL_dRGB[c];
                DSH(7, c) = d7 * dL_dRGB[c];
                DSH(8, c) = d8 * dL_dRGB[c];
                dRGBdx[c] += SH_C2[0] * y * SH(4, c) + SH_C2[2] * 2.f * -x * SH(6, c) +
                             SH_C2[3] * z * SH(7, c) + SH_C2[4] * 2.f * x * SH(8, c);
                dRGBdy[c] += SH_C2[0] * x * SH(4, c) + SH_C2[1] * z * SH(5, c) +
                             SH_C2[2] * 2.f * -y * SH(6, c) + SH_C2[4] * 2.f * -y * SH(8, c);
                dRGBdz[c] += SH_C2[1] * y * SH(5, c) + SH_C2[2] * 2.f * 2.f * z * SH(6, c) +
                             SH_C2[3] * x * SH(7, c);
            }
            if (deg > 2) {
                float d9 = SH_C3[0] * y * (3.f * xx - yy);
                float d10 = SH_C3[1] * xy * z;
                float d11 = SH_C3[2] * y * (4.f * zz - xx - yy);
                float d12 = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                float d13 = SH_C3[4] * x * (4.f * zz - xx - yy);
                float d14 = SH_C3[5] * z * (xx - yy);
                float d15 = SH_C3[6] * x * (xx - 3.f * yy);
                for (int c = 0; c < 3; c++) {
                    DSH(9, c) = d9 * dL_dRGB[c];
                    DSH(10, c) = d10 * dL_dRGB[c];
                    DSH(11, c) = d11 * dL_dRGB[c];
                    DSH(12, c) = d12 * dL_dRGB[c];
                    DSH(13, c) = d13 * dL_dRGB[c];
                    DSH(14, c) = d14 * dL_dRGB[c];
                    DSH(15, c) = d15 * dL_dRGB[c];
                    dRGBdx[c] += (SH_C3[0] * SH(9, c) * 3.f * 2.f * xy + SH_C3[1] * SH(10, c) * yz +
                                  SH_C3[2] * SH(11, c) * -2.f * xy + SH_C3[3] * SH(12, c) * -3.f * 2.f * xz +
                                  SH_C3[4] * SH(13, c) * (-3.f * xx + 4.f * zz - yy) +
                                  SH_C3[5] * SH(14, c) * 2.f * xz + SH_C3[6] * SH(15, c) * 3.f * (xx - yy));
                    dRGBdy[c] += (SH_C3[0] * SH(9, c) * 3.f * (xx - yy) + SH_C3[1] * SH(10, c) * xz +
                                  SH_C3[2] * SH(11, c) * (-3.f * yy + 4.f * zz - xx) +
                                  SH_C3[3] * SH(12, c) * -3.f * 2.f * yz + SH_C3[4] * SH(13, c) * -2.f * xy +
                                  SH_C3[5] * SH(14, c) * -2.f * yz + SH_C3[6] * SH(15, c) * -3.f * 2.f * xy);
                    dRGBdz[c] += (SH_C3[1] * SH(10, c) * xy + SH_C3[2] * SH(11, c) * 4.f * 2.f * yz +
                                  SH_C3[3] * SH(12, c) * 3.f * (2.f * zz - xx - yy) +
                                  SH_C3[4] * SH(13, c) * 4.f * 2.f * xz + SH_C3[5] * SH(14, c) * (xx - yy));
                }
            }
        }
    }
#undef SH
#undef DSH
    float dL_ddir[3] = {dot3(dRGBdx, dL_dRGB), dot3(dRGBdy, dL_dRGB), dot3(dRGBdz, dL_dRGB)};
    float dL_dmean[3];
    dnormvdv3(dir_orig, dL_ddir, dL_dmean);
    dL_dmeans[3 * idx + 0] += dL_dmean[0];
    dL_dmeans[3 * idx + 1] += dL_dmean[1];
    dL_dmeans[3 * idx + 2] += dL_dmean[2];
}

/* base/cr/backward.cu:278-341 (computeCov3D backward) */
static void computeCov3D_bwd(int idx, const float* scale, float mod, const float* rot,
                             const float* dL_dcov3Ds, float* dL_dscales, float* dL_drots) {
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    mat3 R = quat_to_R(r, x, y, z);
    mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2];
    mat3 M = mat3_mul(&S, &R);
    const float* dc = dL_dcov3Ds + 6 * idx;
    mat3 dL_dSigma = mat3_cols(dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4],
                               0.5f * dc[2], 0.5f * dc[4], dc[5]);
    mat3 M2 = mat3_scale(2.0f, &M);
    mat3 dL_dM = mat3_mul(&M2, &dL_dSigma);
    mat3 Rt = mat3_transpose(&R);
    mat3 dL_dMt = mat3_transpose(&dL_dM);
    float* ds = dL_dscales + 3 * idx;
    ds[0] = dot3(Rt.m[0], dL_dMt.m[0]);
    ds[1] = dot3(Rt.m[1], dL_dMt.m[1]);
    ds[2] = dot3(Rt.m[2], dL_dMt.m[2]);
    for (int k = 0; k < 3; k++) {
        dL_dMt.m[0][k] *= s[0];
        dL_dMt.m[1][k] *= s[1];
        dL_dMt.m[2][k] *= s[2];
    }
    const float (*Dm)[3] = (const float (*)[3])dL_dMt.m;
    float* dq = dL_drots + 4 * idx;
    dq[0] = 2 * z * (Dm[0][1] - Dm[1][0]) + 2 * y * (Dm[2][0] - Dm[0][2]) + 2 * x * (Dm[1][2] - Dm[2][1]);
    dq[1] = 2 * y * (Dm[1][0] + Dm[0][1]) + 2 * z * (Dm[2][0] + Dm[0][2]) + 2 * r * (Dm[1][2] - Dm[2][1]) - 4 * x * (Dm[2][2] + Dm[1][1]);
    dq[2] = 2 * x * (Dm[1][0] + Dm[0][1]) + 2 * r * (Dm[2][0] - Dm[0][2]) + 2 * z * (Dm[1][2] + Dm[2][1]) - 4 * y * (Dm[2][2] + Dm[0][0]);
    dq[3] = 2 * r * (Dm[0][1] - Dm[1][0]) + 2 * x * (Dm[2][0] + Dm[0][2]) + 2 * y * (Dm[1][2] + Dm[2][1]) - 4 * z * (Dm[1][1] + Dm[0][0]);
}

/* base/cr/backward.cu:346-396 (preprocessCUDA<3> backward) */
void orc_preprocess_backward(int P, int D, int M, const float* means, const int* radii,
                             const float* shs, const uint8_t* clamped, const float* scales,
                             const float* rotations, float scale_modifier, const float* proj,
                             const float* campos, const float* dL_dmean2D, float* dL_dmeans,
                             const float* dL_dcolor, const float* dL_dcov3D, float* dL_dsh,
                             float* dL_dscale, float* dL_drot) {
#pragma omp parallel for schedule(static, 4096) num_threads(g_threads) if (g_threads > 1)
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        const float* m = means + 3 * idx;
        float m_hom[4];
        transformPoint4x4(m, proj, m_hom);
        float m_w = 1.0f / (m_hom[3] + 0.0000001f);
        float mul1 = (proj[0] * m[0] + proj[4] * m[1] + proj[8] * m[2] + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m[0] + proj[5] * m[1] + proj[9] * m[2] + proj[13]) * m_w * m_w;
        const float* g2 = dL_dmean2D + 3 * idx;
        float dmx = (proj[0] * m_w - proj[3] * mul1) * g2[0] + (proj[1] * m_w - proj[3] * mul2) * g2[1];
        float dmy = (proj[4] * m_w - proj[7] * mul1) * g2[0] + (proj[5] * m_w - proj[7] * mul2) * g2[1];
        float dmz = (proj[8] * m_w - proj[11] * mul1) * g2[0] + (proj[9] * m_w - proj[11] * mul2) * g2[1];
        dL_dmeans[3 * idx + 0] += dmx;
        dL_dmeans[3 * idx + 1] += dmy;
        dL_dmeans[3 * idx + 2] += dmz;
        if (shs)
            computeColorFromSH_bwd(idx, D, M, means, campos, shs, clamped, dL_dcolor, dL_dmeans, dL_dsh);
        if (scales)
            computeCov3D_bwd(idx, scales + 3 * idx, scale_modifier, rotations + 4 * idx, dL_dcov3D,
                             dL_dscale, dL_drot);
    }
}

/* ======================================================================= AMR */
/* amr/cr/rasterizer_impl.cu:181-188 + :607-648 + :190-205.
 * n_intersections[T], sorted[T] (ascending), pv[3], levels[T]. */
void orc_amr_levels(int T, const uint32_t* ranges, uint32_t* n_inter, uint32_t* sorted,
                    uint32_t* pv, uint32_t* levels) {
    for (int t = 0; t < T; t++) n_inter[t] = ranges[2 * t + 1] - ranges[2 * t];
    memcpy(sorted, n_inter, sizeof(uint32_t) * (size_t)T);
    /* counting-free insertion of a small array: a plain ascending sort */
    for (int i = 1; i < T; i++) {
        uint32_t v = sorted[i];
        int j = i - 1;
        while (j >= 0 && sorted[j] > v) { sorted[j + 1] = sorted[j]; j--; }
        sorted[j + 1] = v;
    }
    const float percentiles[3] = {0.25f, 0.5f, 0.9f};
    for (int i = 0; i < 3; i++) {
        int pidx = (int)(percentiles[i] * (float)T);
        pv[i] = (T > 0) ? sorted[pidx] : 0;
    }
    for (int t = 0; t < T; t++) {
        uint32_t v = n_inter[t];
        levels[t] = v <= pv[0] ? 1u : v <= pv[1] ? 2u : v <= pv[2] ? 3u : 4u;
    }
}

/* amr/cr/rasterizer_impl.cu:208-243 (setFoveaAMRLevelsKernel) */
void orc_amr_fovea_levels(int step, int T, uint32_t* last, uint32_t* current,
                          const uint32_t* levels) {
    for (int t = 0; t < T; t++) {
        uint32_t L = levels[t];
        switch (step) {
            case 0: break;
            case 1: last[t] = 0; current[t] = (L >= 1) ? 1 : last[t]; break;
            case 2: case 3: case 4:
                last[t] = current[t];
                current[t] = (L >= (uint32_t)step) ? (uint32_t)step : last[t];
                break;
            default: last[t] = 0; current[t] = L; break;
        }
    }
}

static uint32_t amr_round_of(uint32_t ox, uint32_t oy) {
    /* amr/cr/forward.cu:313-339: (0,0)->1, (0,1)->4, (1,0)->3, (1,1)->2 */
    if (ox == 0) return oy == 0 ? 1u : 4u;
    return oy == 0 ? 3u : 2u;
}

/* amr/cr/forward.cu:261-518 (renderCUDA, AMR).  32-px tiles rendered on the
 * 2x2 sub-lattice; `levels` is the tile_AMR_levels argument, `levels_last`
 * tile_AMR_levels_last. */
void orc_amr_render(int W, int H, const uint32_t* ranges, const uint32_t* levels,
                    const uint32_t* levels_last, const uint32_t* point_list,
                    const float* points_xy, const float* features, const float* conic_opacity,
                    float* final_T, uint32_t* n_contrib, const float* bg_color, float* out_color,
                    int foveaStep) {
    const int BX = 32, R = 2;
    const int tgx = (W + BX - 1) / BX, tgy = (H + BX - 1) / BX;
#pragma omp parallel for schedule(dynamic, 1) num_threads(g_threads) if (g_threads > 1)
    for (int gy = 0; gy < tgy * R; gy++)
        for (int gx = 0; gx < tgx * R; gx++) {
            int tile = (gy / R) * tgx + (gx / R);
            uint32_t L_last = levels_last[tile];
            uint32_t L = levels[tile];
            if (L <= L_last) continue;
            uint32_t ox = (uint32_t)(gx % R), oy = (uint32_t)(gy % R);
            uint32_t round = amr_round_of(ox, oy);
            if (L > 4) L = 4;
            if (foveaStep > 0 && round <= L_last) continue;
            if (round > L) continue;
            uint32_t rx = ranges[2 * tile], ry = ranges[2 * tile + 1];
            for (int ty = 0; ty < 16; ty++)
                for (int tx = 0; tx < 16; tx++) {
                    int px = (gx / R) * BX + tx * R + (int)ox;
                    int py = (gy / R) * BX + ty * R + (int)oy;
                    if (!(px < W && py < H)) continue;
                    float T, C[3];
                    uint32_t nc;
                    blend_pixel(rx, ry, point_list, (float)px, (float)py, points_xy, features,
                                conic_opacity, &T, &nc, C);
                    size_t pid = (size_t)W * py + px;
                    final_T[pid] = T;
                    n_contrib[pid] = nc;
                    for (int ch = 0; ch < 3; ch++)
                        out_color[(size_t)ch * H * W + pid] = C[ch] + T * bg_color[ch];
                }
        }
}

/* amr/cr/forward.cu:520-648 (interpolateCUDA).  The reference runs the
 * precomp copy and the neighbour copy in one launch (a read/write race for
 * foveaStep>0); this restatement runs the precomp copy first (the order the
 * HIP path also fixes).  foveaStep<=0 (render_once) has no race. */
void orc_amr_interpolate(int W, int H, const uint32_t* levels, const uint32_t* levels_last,
                         float* final_T, uint32_t* n_contrib, float* out_color, int foveaStep,
                         const float* out_color_precomp) {
    const int BX = 32, R = 2;
    const int tgx = (W + BX - 1) / BX;
    const size_t N = (size_t)W * H;
    for (int pass = 0; pass < 2; pass++)
        for (int py = 0; py < H; py++)
            for (int px = 0; px < W; px++) {
                int tile = (py / BX) * tgx + (px / BX);
                uint32_t ox = (uint32_t)(px % R), oy = (uint32_t)(py % R);
                uint32_t round = amr_round_of(ox, oy);
                uint32_t L = levels[tile];
                if (L > 4) L = 4;
                size_t pid = (size_t)W * py + px;
                if (foveaStep > 0) {
                    int L_last = (int)levels_last[tile];
                    int copy = ((int)L <= L_last) || ((int)round < L_last);
                    if (pass == 0) {
                        if (copy)
                            for (int ch = 0; ch < 3; ch++)
                                out_color[ch * N + pid] = out_color_precomp[ch * N + pid];
                        continue;
                    }
                    if ((int)round < L_last) continue;
                } else if (pass == 0) {
                    continue;
                }
                if (round <= L) continue;
                uint32_t olx = 0, oly = 0;
                if (L == 3 || L == 4) { olx = 1; oly = 1; }
                int lx = px - (int)ox + (int)olx, ly = py - (int)oy + (int)oly;
                if (lx < W && ly < H) {
                    size_t lid = (size_t)W * ly + lx;
                    final_T[pid] = final_T[lid];
                    n_contrib[pid] = n_contrib[lid];
                    for (int ch = 0; ch < 3; ch++) out_color[ch * N + pid] = out_color[ch * N + lid];
                }
            }
}

/* ================================================================ simple-knn */
/* knn/simple_knn.cu:45-52 */
static uint32_t prepMorton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}

/* float -> uint32 with the CUDA cvt.rzi.u32.f32 semantics (NaN->0, saturate) */
static uint32_t f2u_sat(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

/* knn/simple_knn.cu:54-61 */
static uint32_t coord2Morton(const float* c, const float* mn, const float* mx) {
    uint32_t x = prepMorton(f2u_sat(((c[0] - mn[0]) / (mx[0] - mn[0])) * (float)((1 << 10) - 1)));
    uint32_t y = prepMorton(f2u_sat(((c[1] - mn[1]) / (mx[1] - mn[1])) * (float)((1 << 10) - 1)));
    uint32_t z = prepMorton(f2u_sat(((c[2] - mn[2]) / (mx[2] - mn[2])) * (float)((1 << 10) - 1)));
    return x | (y << 1) | (z << 2);
}

/* knn/simple_knn.cu:124-146 */
static float distBoxPoint(const float* bmin, const float* bmax, const float* p) {
    float diff[3] = {0, 0, 0};
    for (int k = 0; k < 3; k++)
        if (p[k] < bmin[k] || p[k] > bmax[k])
            diff[k] = fminf(fabsf(p[k] - bmin[k]), fabsf(p[k] - bmax[k]));
    return diff[0] * diff[0] + diff[1] * diff[1] + diff[2] * diff[2];
}

static void updateKBest3(const float* ref, const float* pt, float* knn) {
    float d[3] = {pt[0] - ref[0], pt[1] - ref[1], pt[2] - ref[2]};
    float dist = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    for (int j = 0; j < 3; j++)
        if (knn[j] > dist) { float t = knn[j]; knn[j] = dist; dist = t; }
}

/* knn/simple_knn.cu:185-221 (SimpleKNN::knn) with kernels :63-183.
 * Also returns the intermediates morton_sorted[P], indices_sorted[P] and
 * boxes[nb*6] when the pointers are non-NULL. */
void orc_knn(int P, const float* points, float* meanDists, uint32_t* morton_sorted_out,
             uint32_t* indices_sorted_out, float* boxes_out) {
    const int BOX = 1024;
    float minn[3] = {0, 0, 0}, maxx[3] = {0, 0, 0}; /* init {0,0,0} quirk, :189 */
    for (int i = 0; i < P; i++)
        for (int k = 0; k < 3; k++) {
            minn[k] = fminf(minn[k], points[3 * i + k]);
            maxx[k] = fmaxf(maxx[k], points[3 * i + k]);
        }
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(P > 0 ? P : 1));
    uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(P > 0 ? P : 1));
    for (int i = 0; i < P; i++) {
        keys[i] = coord2Morton(points + 3 * i, minn, maxx);
        idx[i] = (uint32_t)i;
    }
    orc_sort_pairs_u64(P, keys, idx, 32);
    int nb = (P + BOX - 1) / BOX;
    float* boxes = (float*)malloc(sizeof(float) * 6 * (size_t)(nb > 0 ? nb : 1));
    for (int b = 0; b < nb; b++) {
        float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int i = b * BOX; i < P && i < (b + 1) * BOX; i++)
            for (int k = 0; k < 3; k++) {
                mn[k] = fminf(mn[k], points[3 * idx[i] + k]);
                mx[k] = fmaxf(mx[k], points[3 * idx[i] + k]);
            }
        for (int k = 0; k < 3; k++) { boxes[6 * b + k] = mn[k]; boxes[6 * b + 3 + k] = mx[k]; }
    }
    for (int i = 0; i < P; i++) {
        const float* point = points + 3 * idx[i];
        float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
        int lo = i - 3 > 0 ? i - 3 : 0, hi = i + 3 < P - 1 ? i + 3 : P - 1;
        for (int j = lo; j <= hi; j++) {
            if (j == i) continue;
            updateKBest3(point, points + 3 * idx[j], best);
        }
        float reject = best[2];
        best[0] = best[1] = best[2] = FLT_MAX;
        for (int b = 0; b < nb; b++) {
            float dist = distBoxPoint(boxes + 6 * b, boxes + 6 * b + 3, point);
            if (dist > reject || dist > best[2]) continue;
            for (int j = b * BOX; j < P && j < (b + 1) * BOX; j++) {
                if (j == i) continue;
                updateKBest3(point, points + 3 * idx[j], best);
            }
        }
        meanDists[idx[i]] = (best[0] + best[1] + best[2]) / 3.0f;
    }
    if (morton_sorted_out)
        for (int i = 0; i < P; i++) morton_sorted_out[i] = (uint32_t)keys[i];
    if (indices_sorted_out) memcpy(indices_sorted_out, idx, sizeof(uint32_t) * (size_t)P);
    if (boxes_out) memcpy(boxes_out, boxes, sizeof(float) * 6 * (size_t)nb);
    free(keys);
    free(idx);
    free(boxes);
}
