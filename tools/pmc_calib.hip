// pmc_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950
// for the access patterns of this repository's kernels
// (MI355X_MICROARCH.md §HBM: "FETCH_SIZE reports exactly 1/2 of the bytes of
// a wide coalesced streaming read ... Other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").
//
// Every pattern runs over a 1 GiB buffer (4x the 256 MiB Infinity Cache, so
// nothing is re-served on-die) and touches each 128-B line at most once, so the
// lines it touches (`lines`) and the bytes its lanes ask for (`bytes`) are
// known exactly.  Random line order: line = (i * odd) mod 2^k, a bijection.
//   stream16   float4 per lane, wave-contiguous        (preprocess / bwd_gauss SH rows, image planes)
//   stream4    float per lane, wave-contiguous         (point_list, final_T, n_contrib, dL_dpix)
//   gather8    one float2 per lane at a random line    (means2D gathers)
//   gather16   one float4 per lane at a random line    (conic_opacity gathers)
//   halves     low then high 64 B of one random line per lane (line vs sector requests)
//   row64      one 64-B row (4 lanes x float4) at a random 64-B row  (AMR blend rows)
//   wstream16  float4 stores, wave-contiguous
//   scatter8   one 8-B store per lane at a random line (duplicate's key stores)
//   atomrow64  16 lanes atomicAdd a 64-B row at a random row (render_bwd's flush)
// Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` and, separately,
// `--pmc WRITE_SIZE`; tools/pmc_calib.py turns the CSVs into factors.
// Build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

constexpr size_t kBytes = size_t(1) << 30;
constexpr uint32_t kLines = uint32_t(kBytes / 128);  // 2^23
constexpr uint32_t kRows = uint32_t(kBytes / 64);    // 2^24
constexpr uint32_t kOdd = 2654435761u;

__device__ __forceinline__ uint32_t perm(uint32_t i, uint32_t n) { return (i * kOdd) & (n - 1); }

__global__ void stream16(const float4* __restrict__ in, float* __restrict__ sink, size_t n) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[0] = acc;  // never true for the zero buffer: keeps the loads
}

__global__ void stream4(const float* __restrict__ in, float* __restrict__ sink, size_t n) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += in[i];
    if (acc == 12345.f) sink[0] = acc;
}

__global__ void gather8(const float2* __restrict__ in, float* __restrict__ sink, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 v = in[(size_t)perm(i, kLines) * 16];  // 16 float2 per 128-B line
    if (v.x + v.y == 12345.f) sink[0] = v.x;
}

// Line or sector?  Each lane reads the low 64 B of a random line, then -- after
// that load has returned (the address depends on its value) -- the high 64 B.
// FETCH per line: 64 if the first miss brought the whole 128-B line (tallied
// at 64, like a stream's line) and the second read hit L2; 128 if each half is
// its own 64-B request.
__global__ void halves(const float2* __restrict__ in, float* __restrict__ sink, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const size_t base = (size_t)perm(i, kLines) * 16;
    const float2 lo = in[base];
    const float2 hi = in[base + 8 + (lo.x != 0.f ? 1 : 0)];
    if (lo.y + hi.x + hi.y == 12345.f) sink[0] = lo.x;
}

__global__ void gather16(const float4* __restrict__ in, float* __restrict__ sink, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = in[(size_t)perm(i, kLines) * 8];
    if (v.x + v.y + v.z + v.w == 12345.f) sink[0] = v.x;
}

__global__ void row64(const float4* __restrict__ in, float* __restrict__ sink, uint32_t n) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = t >> 2;  // 4 lanes per row
    if (i >= n) return;
    const float4 v = in[(size_t)perm(i, kRows) * 4 + (t & 3)];
    if (v.x + v.y + v.z + v.w == 12345.f) sink[0] = v.x;
}

__global__ void wstream16(float4* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

__global__ void scatter8(uint64_t* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[(size_t)perm(i, kLines) * 16] = 0x0102030405060708ull + i;
}

__global__ void atomrow64(float* __restrict__ out, uint32_t n) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = t >> 4;  // 16 lanes per row
    if (i >= n) return;
    atomicAdd(&out[(size_t)perm(i, kRows) * 16 + (t & 15)], 1.0f);
}

int main() {
    char* buf;
    float* sink;
    CK(hipMalloc(&buf, kBytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, kBytes));
    CK(hipDeviceSynchronize());
    const uint32_t nl = kLines / 4;  // a quarter of the lines / rows: 256 MiB of lines touched
    const uint32_t nr = kRows / 4;
    std::printf("{\"buffer_bytes\": %zu, \"patterns\": {\n", kBytes);
    hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink, kBytes / 16);
    std::printf(" \"stream16\": {\"kernel\": \"stream16\", \"bytes\": %zu, \"lines\": %u},\n", kBytes, kLines);
    hipLaunchKernelGGL(stream4, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float*>(buf), sink, kBytes / 4);
    std::printf(" \"stream4\": {\"kernel\": \"stream4\", \"bytes\": %zu, \"lines\": %u},\n", kBytes, kLines);
    hipLaunchKernelGGL(gather8, dim3(nl / 256), dim3(256), 0, 0, reinterpret_cast<const float2*>(buf), sink, nl);
    std::printf(" \"gather8\": {\"kernel\": \"gather8\", \"bytes\": %zu, \"lines\": %u},\n", (size_t)nl * 8, nl);
    hipLaunchKernelGGL(halves, dim3(nl / 256), dim3(256), 0, 0, reinterpret_cast<const float2*>(buf), sink, nl);
    std::printf(" \"halves\": {\"kernel\": \"halves\", \"bytes\": %zu, \"lines\": %u},\n", (size_t)nl * 16, nl);
    hipLaunchKernelGGL(gather16, dim3(nl / 256), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink, nl);
    std::printf(" \"gather16\": {\"kernel\": \"gather16\", \"bytes\": %zu, \"lines\": %u},\n", (size_t)nl * 16, nl);
    hipLaunchKernelGGL(row64, dim3(nr * 4 / 256), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink, nr);
    std::printf(" \"row64\": {\"kernel\": \"row64\", \"bytes\": %zu, \"rows\": %u},\n", (size_t)nr * 64, nr);
    hipLaunchKernelGGL(wstream16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<float4*>(buf), kBytes / 16);
    std::printf(" \"wstream16\": {\"kernel\": \"wstream16\", \"bytes\": %zu, \"lines\": %u},\n", kBytes, kLines);
    hipLaunchKernelGGL(scatter8, dim3(nl / 256), dim3(256), 0, 0, reinterpret_cast<uint64_t*>(buf), nl);
    std::printf(" \"scatter8\": {\"kernel\": \"scatter8\", \"bytes\": %zu, \"lines\": %u},\n", (size_t)nl * 8, nl);
    hipLaunchKernelGGL(atomrow64, dim3(nr * 16 / 256), dim3(256), 0, 0, reinterpret_cast<float*>(buf), nr);
    std::printf(" \"atomrow64\": {\"kernel\": \"atomrow64\", \"bytes\": %zu, \"rows\": %u}\n", (size_t)nr * 64, nr);
    std::printf("}}\n");
    CK(hipDeviceSynchronize());
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
