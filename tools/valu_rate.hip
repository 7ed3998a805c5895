// VALU issue-rate probe (tools only): wave-instructions per second per SIMD for
// independent v_fma_f32 chains vs v_pk_fma_f32 (two f32 FMAs per lane per
// instruction), many waves per SIMD.  Tells whether the blend kernels' VALU
// roofline is 2 or 4 cycles per wave64 instruction and whether packed f32
// doubles the FMA rate.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float float2_t __attribute__((ext_vector_type(2)));

template <int kChains>
__global__ void __launch_bounds__(256) fma_kernel(float* out, int iters, float a, float b, unsigned long long* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    float v[kChains];
#pragma unroll
    for (int c = 0; c < kChains; c++) v[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < kChains; c++) v[c] = __builtin_fmaf(v[c], a, b);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kChains; c++) s += v[c];
    if (s == 12345.678f) out[threadIdx.x] = s;
    if (clk && threadIdx.x == 0 && blockIdx.x == 0) clk[0] = __builtin_amdgcn_s_memtime() - t0;  // one wave's cycles
}

template <int kChains>
__global__ void __launch_bounds__(256) pkfma_kernel(float* out, int iters, float a, float b, unsigned long long*) {
    float2_t v[kChains];
#pragma unroll
    for (int c = 0; c < kChains; c++) v[c] = float2_t{threadIdx.x * 1e-3f + c, c * 0.5f};
    const float2_t A = {a, a}, B = {b, b};
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < kChains; c++) v[c] = __builtin_elementwise_fma(v[c], A, B);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kChains; c++) s += v[c].x + v[c].y;
    if (s == 12345.678f) out[threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) exp_kernel(float* out, int iters, float a, float b, unsigned long long*) {
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = threadIdx.x * 1e-6f + c * 1e-3f;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) v[c] = __builtin_amdgcn_exp2f(v[c]) * a;
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; c++) s += v[c];
    if (s == 12345.678f) out[threadIdx.x] = s;
}

// v_cndmask_b32 chains (the select-form blends are full of them)
__global__ void __launch_bounds__(256) cnd_kernel(float* out, int iters, float a, float b, unsigned long long*) {
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = threadIdx.x * 1e-3f + c;
    const bool m = (threadIdx.x & 1) != 0;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            v[c] = m ? v[c] : a;
            asm volatile("" : "+v"(v[c]));
        }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; c++) s += v[c];
    if (s == 12345.678f) out[threadIdx.x] = s;
}

// v_add_u32 chains (integer ALU)
__global__ void __launch_bounds__(256) iadd_kernel(float* out, int iters, float a, float b, unsigned long long*) {
    unsigned v[8];
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = threadIdx.x + c;
    const unsigned k = (unsigned)iters * 7u + 3u;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) v[c] = v[c] + k;
    }
    unsigned s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s += v[c];
    if (s == 12345u) out[threadIdx.x] = (float)s;
}

// v_cmp + v_cndmask pairs (a select on a compare)
__global__ void __launch_bounds__(256) cmpsel_kernel(float* out, int iters, float a, float b, unsigned long long*) {
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            v[c] = v[c] > a ? v[c] : b;
            asm volatile("" : "+v"(v[c]));
        }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; c++) s += v[c];
    if (s == 12345.678f) out[threadIdx.x] = s;
}

int main() {
    float* out;
    hipMalloc(&out, 1024 * sizeof(float));
    const int blocks = 256 * 32, iters = 4096;  // 8 waves per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    unsigned long long* clk;
    hipMalloc(&clk, sizeof(unsigned long long));
    // shader clock: one wave alone on the chip, s_memtime ticks vs wall time
    {
        hipLaunchKernelGGL(fma_kernel<8>, dim3(1), dim3(64), 0, 0, out, 16, 0.999f, 1e-3f, clk);
        hipEventRecord(e0);
        hipLaunchKernelGGL(fma_kernel<8>, dim3(1), dim3(64), 0, 0, out, 1 << 20, 0.999f, 1e-3f, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c = 0;
        hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
        printf("{\"probe\": \"one wave, 8 fma chains\", \"ms\": %.3f, \"memtime_ticks\": %llu, \"ticks_per_us\": %.1f, "
               "\"ticks_per_fma_instr\": %.3f}\n", ms, c, c / (ms * 1e3), (double)c / (8.0 * (1 << 20)));
    }
    auto run = [&](const char* name, auto kern, double instr_per_iter) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 16, 0.999f, 1e-3f, nullptr);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 1e-3f, nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double waves = blocks * 4.0;
        const double winstr = waves * iters * instr_per_iter;
        const double per_simd_cycle = winstr / (ms * 1e-3) / (1024.0 * 2.4e9);
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"wave_instr_per_simd_per_cycle\": %.4f, \"cycles_per_wave_instr\": %.3f}\n",
               name, ms, per_simd_cycle, 1.0 / per_simd_cycle);
    };
    run("v_fma_f32 x8 chains", fma_kernel<8>, 8);
    run("v_fma_f32 x16 chains", fma_kernel<16>, 16);
    run("v_pk_fma_f32 x8 chains", pkfma_kernel<8>, 8);
    run("v_exp_f32 + v_mul x8 chains", exp_kernel, 16);
    run("v_cndmask_b32 x8 chains", cnd_kernel, 8);
    run("v_add_u32 x8 chains", iadd_kernel, 8);
    run("v_cmp + v_cndmask x8 chains (per pair)", cmpsel_kernel, 16);
    return 0;
}
