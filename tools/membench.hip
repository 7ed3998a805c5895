// membench.hip -- access-pattern probe for the per-Gaussian kernels
// (preprocess / bwd_gauss read and write 192-B SH rows, one row per thread).
// Compares, over the same buffers (P rows of 192 B):
//   aos_copy : thread i copies row i with 12 float4 loads / stores (AoS)
//   coal_copy: the same bytes, float4 index = t + k * stride (wave-contiguous)
//   aos_write / coal_write: stores only (zeros)
// Build: hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ void aos_copy(const float4* __restrict__ in, float4* __restrict__ out, int P) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    float4 v[12];
#pragma unroll
    for (int k = 0; k < 12; k++) v[k] = in[(size_t)i * 12 + k];
#pragma unroll
    for (int k = 0; k < 12; k++) out[(size_t)i * 12 + k] = v[k];
}

__global__ void coal_copy(const float4* __restrict__ in, float4* __restrict__ out, int P) {
    // each workgroup owns 256 rows = 3072 float4, thread t moves t + 256 k
    const size_t base = (size_t)blockIdx.x * 256 * 12;
    const size_t n = (size_t)P * 12;
    float4 v[12];
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const size_t f = base + threadIdx.x + 256 * k;
        v[k] = f < n ? in[f] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const size_t f = base + threadIdx.x + 256 * k;
        if (f < n) out[f] = v[k];
    }
}

__global__ void aos_write(float4* __restrict__ out, int P) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
#pragma unroll
    for (int k = 0; k < 12; k++) out[(size_t)i * 12 + k] = make_float4(0, 0, 0, 0);
}

__global__ void coal_write(float4* __restrict__ out, int P) {
    const size_t base = (size_t)blockIdx.x * 256 * 12;
    const size_t n = (size_t)P * 12;
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const size_t f = base + threadIdx.x + 256 * k;
        if (f < n) out[f] = make_float4(0, 0, 0, 0);
    }
}

template <typename F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int P = argc > 1 ? std::atoi(argv[1]) : 6100000;
    const size_t bytes = (size_t)P * 192;
    float4 *in, *out;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    CK(hipMemset(in, 1, bytes));
    const dim3 grid((P + 255) / 256);
    const int reps = 20;
    const float t1 = time_ms([&] { hipLaunchKernelGGL(aos_copy, grid, dim3(256), 0, 0, in, out, P); }, reps);
    const float t2 = time_ms([&] { hipLaunchKernelGGL(coal_copy, grid, dim3(256), 0, 0, in, out, P); }, reps);
    const float t3 = time_ms([&] { hipLaunchKernelGGL(aos_write, grid, dim3(256), 0, 0, out, P); }, reps);
    const float t4 = time_ms([&] { hipLaunchKernelGGL(coal_write, grid, dim3(256), 0, 0, out, P); }, reps);
    CK(hipDeviceSynchronize());
    std::printf("{\"P\": %d, \"bytes\": %zu, \"aos_copy_ms\": %.4f, \"aos_copy_TBps\": %.3f, \"coal_copy_ms\": %.4f, "
                "\"coal_copy_TBps\": %.3f, \"aos_write_ms\": %.4f, \"aos_write_TBps\": %.3f, \"coal_write_ms\": %.4f, "
                "\"coal_write_TBps\": %.3f}\n",
                P, bytes, t1, 2.0 * bytes / t1 / 1e9, t2, 2.0 * bytes / t2 / 1e9, t3, bytes / t3 / 1e9, t4,
                bytes / t4 / 1e9);
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
