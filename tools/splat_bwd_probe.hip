// Cost probe (tools only) for a splat-parallel blend backward -- the
// structure the round-4 review proposed for render_bwd: a lane owns one
// Gaussian of a 64-entry batch and walks the pixels; per pixel the lanes need
// the transmittance in front of their entry (an exclusive prefix product of
// (1 - alpha) over the batch, seeded by a forward checkpoint) and the colour
// accumulated behind it (an affine suffix scan over the batch, seeded by the
// pixel's carried accum_rec).  This probe runs exactly that loop on synthetic
// lists with config 2's statistics -- the row-group form (the cheaper one: a
// wave per (16x16 tile, 4-row group), lists of the entries that reach the
// row group, 1.36 of 4 row groups per entry as measured by tools/cull_stats.py),
// batches back to front, per (pixel, batch): the checkpoint load, the alpha
// evaluation, both scans (DPP), the dL/dalpha terms, nine per-lane gradient
// accumulators, and one atomic row add per entry per batch.  Omitted (so the
// probe is a LOWER bound on the kernel): the T > 1e-4 / n_contrib tests, the
// dL/dconic and dL/dmean terms beyond one shared factor, the checkpoint
// writes in the forward.
//
// usage: splat_bwd_probe [tiles=8160] [mean_entries=544]   (config 2: 8160 tiles, 4.44M instances)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// x combined with the value dpp_ctrl moves into this lane (identity `id` where
// no lane moves in)
template <int kCtrl, int kRowMask = 0xf, int kBankMask = 0xf>
__device__ __forceinline__ float dpp(float x, float id) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, id), __builtin_bit_cast(int, x),
                                                                 kCtrl, kRowMask, kBankMask, false));
}

// inclusive prefix product over the 64 lanes (row_shr 1/2/4/8, row_bcast 15/31)
__device__ __forceinline__ float scan_mul(float x) {
    x *= dpp<0x111>(x, 1.f);
    x *= dpp<0x112>(x, 1.f);
    x *= dpp<0x114>(x, 1.f);
    x *= dpp<0x118>(x, 1.f);
    x *= dpp<0x142, 0xa>(x, 1.f);
    x *= dpp<0x143, 0xc>(x, 1.f);
    return x;
}

// inclusive affine scan: (a, b) o (a', b') = (a a', a' b + b') per lane, three
// b channels sharing a
__device__ __forceinline__ void scan_affine(float& a, float (&b)[3]) {
#define GS_STEP(CTRL, RM)                                       \
    {                                                           \
        const float pa = dpp<CTRL, RM>(a, 1.f);                 \
        float pb[3];                                            \
        for (int c = 0; c < 3; c++) pb[c] = dpp<CTRL, RM>(b[c], 0.f); \
        for (int c = 0; c < 3; c++) b[c] = __builtin_fmaf(a, pb[c], b[c]); \
        a *= pa;                                                \
    }
    GS_STEP(0x111, 0xf)
    GS_STEP(0x112, 0xf)
    GS_STEP(0x114, 0xf)
    GS_STEP(0x118, 0xf)
    GS_STEP(0x142, 0xa)
    GS_STEP(0x143, 0xc)
#undef GS_STEP
}

__global__ void __launch_bounds__(64) splat_probe(int nrg, int gx, const uint32_t* __restrict__ rg_start,
                                                  const uint32_t* __restrict__ rg_count,
                                                  const uint32_t* __restrict__ ids, const float4* __restrict__ g0,
                                                  const float4* __restrict__ g1, const float* __restrict__ ckpt,
                                                  const float* __restrict__ dldp, float* __restrict__ grad) {
    const int rg = blockIdx.x;
    if (rg >= nrg) return;
    const int lane = threadIdx.x;
    const int tile = rg >> 2, q = rg & 3;
    const float rx0 = 16.f * (float)(tile % gx), ry0 = 16.f * (float)(tile / gx) + 4.f * (float)q;
    const uint32_t beg = rg_start[rg], n = rg_count[rg];
    const int nb = (int)((n + 63) / 64);
    // the lane's own pixel (lane = 16 row + col): carried accum_rec, dL/dpix
    float acc_own[3] = {0.f, 0.f, 0.f}, dl_own[3];
    for (int c = 0; c < 3; c++) dl_own[c] = dldp[(size_t)rg * 192 + 64 * c + lane];
    for (int b = nb - 1; b >= 0; b--) {
        const uint32_t e = (uint32_t)b * 64u + (uint32_t)lane;
        const bool ok = e < n;
        const uint32_t id = ok ? ids[beg + e] : 0u;
        const float4 A = g0[id];  // x, y, conic.x, conic.y
        const float4 B = g1[id];  // conic.z, opacity, r, g
        const float cb = B.w * 0.5f + A.w;
        float gacc[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const float* ck = ckpt + ((size_t)rg * 64 + (size_t)b) * 64;  // T at the batch's front, per pixel
        for (int p = 0; p < 64; p++) {
            const float px = rx0 + (float)(p & 15), py = ry0 + (float)(p >> 4);
            const float T0 = ck[p];
            float accp[3];
            for (int c = 0; c < 3; c++)
                accp[c] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, acc_own[c]), p));
            float dl[3];
            for (int c = 0; c < 3; c++)
                dl[c] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, dl_own[c]), p));
            const float dx = A.x - px, dy = A.y - py;
            const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
            float alpha = fminf(0.99f, B.y * __expf(power));
            alpha = (ok && power <= 0.f && alpha >= 1.f / 255.f) ? alpha : 0.f;
            const float om = 1.f - alpha;
            // transmittance in front of each entry: T0 x exclusive prefix of (1 - alpha)
            const float incl = scan_mul(om);
            const float T = T0 * incl / om;
            // colour behind each entry: affine scan from the back (lanes reversed by index)
            float a = om;
            float bch[3] = {alpha * A.z, alpha * B.z, alpha * cb};
            scan_affine(a, bch);
            float acc[3];
            for (int c = 0; c < 3; c++)
                acc[c] = __builtin_fmaf(a, accp[c], bch[c]);
            // dL/dalpha and the per-entry accumulators (colour, opacity, one shared
            // geometry factor spread over the six conic / mean terms)
            const float dLda = T * ((A.z - acc[0]) * dl[0] + (B.z - acc[1]) * dl[1] + (cb - acc[2]) * dl[2]);
            const float w = alpha * T;
            gacc[0] = __builtin_fmaf(w, dl[0], gacc[0]);
            gacc[1] = __builtin_fmaf(w, dl[1], gacc[1]);
            gacc[2] = __builtin_fmaf(w, dl[2], gacc[2]);
            const float g = dLda * alpha;
            gacc[3] = __builtin_fmaf(g, dx, gacc[3]);
            gacc[4] = __builtin_fmaf(g, dy, gacc[4]);
            gacc[5] = __builtin_fmaf(g, dx * dx, gacc[5]);
            gacc[6] = __builtin_fmaf(g, dx * dy, gacc[6]);
            gacc[7] = __builtin_fmaf(g, dy * dy, gacc[7]);
            gacc[8] = __builtin_fmaf(dLda, alpha / B.y, gacc[8]);
            // the pixel's accum_rec in front of the batch (lane 0's inclusive value)
            const float front = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, acc[0]), 0));
            if (lane == p) acc_own[0] = front, acc_own[1] = acc[1], acc_own[2] = acc[2];
        }
        if (ok)
            for (int k = 0; k < 9; k++) atomicAdd(&grad[(size_t)id * 9 + k], gacc[k]);
    }
}

int main(int argc, char** argv) {
    const int tiles = argc > 1 ? atoi(argv[1]) : 8160;
    const int mean = argc > 2 ? atoi(argv[2]) : 544;
    const int gx = 120;
    const int P = 1000000;
    const int nrg = 4 * tiles;
    // per row group: ~1.36 / 4 of the tile's entries, tile sizes spread +-50 %
    std::vector<uint32_t> start(nrg), count(nrg);
    srand(1);
    uint64_t tot = 0;
    for (int t = 0; t < tiles; t++) {
        const int n = mean / 2 + rand() % (mean + 1);
        for (int q = 0; q < 4; q++) {
            const uint32_t c = (uint32_t)((double)n * 1.36 / 4.0 * (0.5 + (rand() % 1001) / 1000.0));
            start[4 * t + q] = (uint32_t)tot;
            count[4 * t + q] = c;
            tot += c;
        }
    }
    std::vector<uint32_t> ids(tot);
    for (auto& v : ids) v = (uint32_t)(rand() % P);
    std::vector<float4> h0(P), h1(P);
    for (int i = 0; i < P; i++) {
        const float x = (float)(rand() % 1920), y = (float)(rand() % 1080);
        h0[i] = make_float4(x, y, 0.02f, 0.001f);
        h1[i] = make_float4(0.02f, 0.6f, 0.5f, 0.4f);
    }
    int maxb = 0;
    for (int r = 0; r < nrg; r++) maxb = std::max(maxb, (int)((count[r] + 63) / 64));
    uint32_t *d_start, *d_count, *d_ids;
    float4 *d0, *d1;
    float *d_ck, *d_dl, *d_g;
    CK(hipMalloc(&d_start, nrg * 4));
    CK(hipMalloc(&d_count, nrg * 4));
    CK(hipMalloc(&d_ids, tot * 4));
    CK(hipMalloc(&d0, (size_t)P * 16));
    CK(hipMalloc(&d1, (size_t)P * 16));
    CK(hipMalloc(&d_ck, (size_t)nrg * 64 * 64 * 4));
    CK(hipMalloc(&d_dl, (size_t)nrg * 192 * 4));
    CK(hipMalloc(&d_g, (size_t)P * 9 * 4));
    CK(hipMemcpy(d_start, start.data(), nrg * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_count, count.data(), nrg * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ids, ids.data(), tot * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d0, h0.data(), (size_t)P * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(d1, h1.data(), (size_t)P * 16, hipMemcpyHostToDevice));
    CK(hipMemset(d_ck, 0, (size_t)nrg * 64 * 64 * 4));
    CK(hipMemset(d_dl, 0, (size_t)nrg * 192 * 4));
    CK(hipMemset(d_g, 0, (size_t)P * 9 * 4));
    if (maxb > 64) {
        fprintf(stderr, "list too long for the checkpoint buffer\n");
        return 1;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; w++)
        hipLaunchKernelGGL(splat_probe, dim3(nrg), dim3(64), 0, 0, nrg, gx, d_start, d_count, d_ids, d0, d1, d_ck, d_dl, d_g);
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL(splat_probe, dim3(nrg), dim3(64), 0, 0, nrg, gx, d_start, d_count, d_ids, d0, d1, d_ck, d_dl, d_g);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"probe\": \"splat-parallel blend backward skeleton (row-group lists)\", \"tiles\": %d, "
           "\"row_group_entries\": %llu, \"tile_instances_equiv\": %.0f, \"ms\": %.4f}\n",
           tiles, (unsigned long long)tot, (double)tot / 1.36, ms / reps);
    return 0;
}
