// VALU / SALU issue-rate probe (tools only).  Every loop body is inline asm,
// so the instruction stream is exactly what the row names (the first version
// of this probe let clang's SLP pass turn its "v_fma_f32" chains into
// v_pk_fma_f32, which halved the instruction count it divided by).
//
// For each body and for 1, 2, 4, 8 waves per SIMD (256-thread workgroups, one
// wave per SIMD each, 256 x w workgroups) it prints the chip-wide issue rate:
// cycles per wave-instruction per SIMD at 2.4 GHz, and, from s_memtime, the
// cycles one wave spent per instruction of its own stream.
//
// usage: valu_rate            (all bodies, all occupancies)
//        valu_rate <body> <w> (one launch, for rocprofv3 --pmc passes)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

// 16 independent accumulators per lane, a loop of kRep repetitions of the body
#define BODY_KERNEL(NAME, ASM, PER)                                                                      \
    __global__ void __launch_bounds__(256) NAME(float* out, int iters, unsigned long long* clk) {       \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                     \
        float v0 = threadIdx.x * 1e-3f, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, \
              v6 = v0 + 6, v7 = v0 + 7, v8 = v0 + 8, v9 = v0 + 9, v10 = v0 + 10, v11 = v0 + 11,           \
              v12 = v0 + 12, v13 = v0 + 13, v14 = v0 + 14, v15 = v0 + 15;                               \
        float k = 0.999f;                                                                               \
        for (int i = 0; i < iters; i++) {                                                               \
            asm volatile(ASM                                                                            \
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7), \
                           "+v"(v8), "+v"(v9), "+v"(v10), "+v"(v11), "+v"(v12), "+v"(v13), "+v"(v14),     \
                           "+v"(v15)                                                                    \
                         : "v"(k)                                                                       \
                         : "vcc", "scc", "s40", "s41", "s42", "s43", "s44", "v40", "v41");                                          \
        }                                                                                               \
        const float s = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + v8 + v9 + v10 + v11 + v12 + v13 + v14 + v15; \
        if (s == 12345.678f) out[threadIdx.x] = s;                                                      \
        if (clk && (threadIdx.x & 63) == 0 && blockIdx.x == 0)                                          \
            clk[threadIdx.x >> 6] = __builtin_amdgcn_s_memtime() - t0;                                  \
    }

// 16 x op on v0..v15 (the %0..%15 operands), %16 = k
#define OP_FMA(i) "v_fma_f32 %" #i ", %" #i ", %16, %16\n"
#define OP_FMA3(i) "v_fma_f32 %" #i ", %" #i ", %16, v40\n"
#define OP_FMAS(i) "v_fma_f32 %" #i ", %" #i ", s44, %16\n"
#define OP_FMAI(i) "v_fma_f32 %" #i ", %" #i ", %16, 1.0\n"
#define OP_FMAC(i) "v_fmac_f32 %" #i ", %16, v40\n"
#define OP_MUL(i) "v_mul_f32 %" #i ", %" #i ", %16\n"
#define OP_MUL3(i) "v_mul_f32_e64 %" #i ", -%" #i ", %16\n"
#define OP_ADD(i) "v_add_f32 %" #i ", %" #i ", %16\n"
#define OP_MIN(i) "v_min_f32 %" #i ", %" #i ", %16\n"
#define OP_MOV(i) "v_mov_b32 %" #i ", %16\n"
#define OP_ADDU(i) "v_add_u32 %" #i ", %" #i ", %16\n"
#define OP_EXP(i) "v_exp_f32 %" #i ", %" #i "\n"
#define OP_RCP(i) "v_rcp_f32 %" #i ", %" #i "\n"
#define OP_EXPMUL(i) "v_exp_f32 %" #i ", %" #i "\nv_mul_f32 v41, v41, %16\n"
#define OP_CND(i) "v_cndmask_b32 %" #i ", %" #i ", %16, vcc\n"
#define OP_CNDS(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %16, s[40:41]\n"
#define OP_CMP(i) "v_cmp_lt_f32 vcc, %" #i ", %16\n"
#define OP_CMPS(i) "v_cmp_lt_f32 s[40:41], %" #i ", %16\n"
#define OP_DPP(i) "v_add_f32_dpp %" #i ", %" #i ", %" #i " row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define OP_FMA_SALU(i) "v_fma_f32 %" #i ", %" #i ", %16, %16\ns_add_u32 s42, s42, 1\n"
#define OP_MUL_SALU(i) "v_mul_f32 %" #i ", %" #i ", %16\ns_add_u32 s42, s42, 1\n"
#define OP_MUL_2SALU(i) "v_mul_f32 %" #i ", %" #i ", %16\ns_add_u32 s42, s42, 1\ns_and_b64 s[40:41], s[40:41], vcc\n"

#define OP_CNDE(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %16, vcc\n"
#define OP_MINK(i) "v_min_f32 %" #i ", 0x3f7d70a4, %" #i "\n"
#define OP_MAX(i) "v_max_f32 %" #i ", %" #i ", %16\n"
#define OP_SUBR(i) "v_sub_f32 %" #i ", 1.0, %" #i "\n"
// the kernels' pattern: one compare feeding two selects
#define OP_CMP_CND2(i) "v_cmp_lt_f32 vcc, %" #i ", %16\nv_cndmask_b32 %" #i ", 0, %" #i ", vcc\nv_cndmask_b32 v41, 0, %" #i ", vcc\n"
#define OP_CMP_CND2S(i) "v_cmp_lt_f32_e64 s[40:41], %" #i ", %16\nv_cndmask_b32_e64 %" #i ", 0, %" #i ", s[40:41]\nv_cndmask_b32_e64 v41, 0, %" #i ", s[40:41]\n"
#define PRE "v_mov_b32 v40, 1.0\nv_mov_b32 v41, 1.0\ns_mov_b32 s44, 0.5\n"
// (each body twice per iteration: 32 instructions against the loop's 3 SALU)
#define TWICE(OP) PRE R16(OP) R16(OP)
BODY_KERNEL(k_fma, TWICE(OP_FMA), 32)
BODY_KERNEL(k_fma3, TWICE(OP_FMA3), 32)
BODY_KERNEL(k_fmas, TWICE(OP_FMAS), 32)
BODY_KERNEL(k_fmai, TWICE(OP_FMAI), 32)
BODY_KERNEL(k_fmac, TWICE(OP_FMAC), 32)
BODY_KERNEL(k_mul, TWICE(OP_MUL), 32)
BODY_KERNEL(k_mul3, TWICE(OP_MUL3), 32)
BODY_KERNEL(k_add, TWICE(OP_ADD), 32)
BODY_KERNEL(k_min, TWICE(OP_MIN), 32)
BODY_KERNEL(k_mov, TWICE(OP_MOV), 32)
BODY_KERNEL(k_addu, TWICE(OP_ADDU), 32)
BODY_KERNEL(k_exp, TWICE(OP_EXP), 32)
BODY_KERNEL(k_rcp, TWICE(OP_RCP), 32)
BODY_KERNEL(k_expmul, TWICE(OP_EXPMUL), 64)
BODY_KERNEL(k_cnd, PRE "v_cmp_lt_f32 vcc, %16, v40\n" R16(OP_CND) R16(OP_CND), 32)
BODY_KERNEL(k_cnds, PRE "v_cmp_lt_f32 s[40:41], %16, v40\n" R16(OP_CNDS) R16(OP_CNDS), 32)
BODY_KERNEL(k_cnd_salu, PRE "s_mov_b64 vcc, -1\n" R16(OP_CND) R16(OP_CND), 32)
BODY_KERNEL(k_cmp, TWICE(OP_CMP), 32)
BODY_KERNEL(k_cmps, TWICE(OP_CMPS), 32)
BODY_KERNEL(k_dpp, TWICE(OP_DPP), 32)
BODY_KERNEL(k_cnde, PRE "v_cmp_lt_f32 vcc, %16, v40\n" R16(OP_CNDE) R16(OP_CNDE), 32)
BODY_KERNEL(k_mink, TWICE(OP_MINK), 32)
BODY_KERNEL(k_max, TWICE(OP_MAX), 32)
BODY_KERNEL(k_subr, TWICE(OP_SUBR), 32)
BODY_KERNEL(k_cmpcnd2, PRE R16(OP_CMP_CND2), 48)
BODY_KERNEL(k_cmpcnd2s, PRE R16(OP_CMP_CND2S), 48)
BODY_KERNEL(k_fma_salu, TWICE(OP_FMA_SALU), 32)
BODY_KERNEL(k_mul_salu, TWICE(OP_MUL_SALU), 32)
BODY_KERNEL(k_mul_2salu, PRE "s_mov_b64 vcc, -1\n" R16(OP_MUL_2SALU) R16(OP_MUL_2SALU), 32)

// packed: 8 register pairs (v0,v1) .. (v14,v15) -- the pairs must be adjacent
// VGPRs, so these bodies use float2 vectors
typedef float f2 __attribute__((ext_vector_type(2)));
#define OP_PK(i) "v_pk_fma_f32 %" #i ", %" #i ", %8, %8\n"
#define OP_PKM(i) "v_pk_mul_f32 %" #i ", %" #i ", %8\n"
#define OP_PKA(i) "v_pk_add_f32 %" #i ", %" #i ", %8\n"
#define R8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
#define PK_KERNEL(NAME, ASM)                                                                                   \
    __global__ void __launch_bounds__(256) NAME(float* out, int iters, unsigned long long* clk) {            \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                          \
        f2 v0 = {threadIdx.x * 1e-3f, 1}, v1 = v0 + 2, v2 = v0 + 4, v3 = v0 + 6, v4 = v0 + 8, v5 = v0 + 10,  \
           v6 = v0 + 12, v7 = v0 + 14;                                                                       \
        f2 k = {0.999f, 0.999f};                                                                             \
        for (int i = 0; i < iters; i++) {                                                                    \
            asm volatile(ASM : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7) \
                         : "v"(k));                                                                          \
        }                                                                                                    \
        const f2 s = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;                                                  \
        if (s.x + s.y == 12345.678f) out[threadIdx.x] = s.x;                                                 \
        if (clk && (threadIdx.x & 63) == 0 && blockIdx.x == 0)                                               \
            clk[threadIdx.x >> 6] = __builtin_amdgcn_s_memtime() - t0;                                       \
    }
PK_KERNEL(k_pkfma, R8(OP_PK) R8(OP_PK) R8(OP_PK) R8(OP_PK))
PK_KERNEL(k_pkmul, R8(OP_PKM) R8(OP_PKM) R8(OP_PKM) R8(OP_PKM))
PK_KERNEL(k_pkadd, R8(OP_PKA) R8(OP_PKA) R8(OP_PKA) R8(OP_PKA))

struct Body {
    const char* name;
    void (*fn)(float*, int, unsigned long long*);
    double instr_per_iter;  // VALU instructions per loop iteration (the body's 32 + the 2 v_mov of PRE)
};

static const Body kBodies[] = {
    {"v_fma_f32 v,v,k,k", k_fma, 34},     {"v_fma_f32 v,v,k,v40", k_fma3, 34}, {"v_fma_f32 v,v,s,k", k_fmas, 34},
    {"v_fma_f32 v,v,k,1.0", k_fmai, 34},  {"v_fmac_f32", k_fmac, 34},          {"v_mul_f32", k_mul, 34},
    {"v_mul_f32_e64 neg", k_mul3, 34},    {"v_add_f32", k_add, 34},            {"v_min_f32", k_min, 34},
    {"v_mov_b32", k_mov, 34},             {"v_add_u32", k_addu, 34},           {"v_exp_f32", k_exp, 34},
    {"v_rcp_f32", k_rcp, 34},             {"v_exp_f32 + v_mul_f32", k_expmul, 66},
    {"v_cndmask_b32 (vcc from v_cmp)", k_cnd, 34}, {"v_cndmask_b32_e64 (sgpr from v_cmp)", k_cnds, 34},
    {"v_cndmask_b32 (vcc from s_mov)", k_cnd_salu, 34}, {"v_cmp_lt_f32 (vcc)", k_cmp, 34},
    {"v_cmp_lt_f32 (sgpr)", k_cmps, 34},  {"v_add_f32_dpp row_shr", k_dpp, 34},
    {"v_cndmask_b32_e64 (vcc from v_cmp)", k_cnde, 34}, {"v_min_f32 literal", k_mink, 34},
    {"v_max_f32", k_max, 34},             {"v_sub_f32 1.0 - v", k_subr, 34},
    {"v_cmp (vcc) + 2 v_cndmask_b32 (vcc)", k_cmpcnd2, 50}, {"v_cmp (sgpr) + 2 v_cndmask_b32_e64 (sgpr)", k_cmpcnd2s, 50},
    {"v_pk_fma_f32", k_pkfma, 32},        {"v_pk_mul_f32", k_pkmul, 32},       {"v_pk_add_f32", k_pkadd, 32},
    {"v_fma_f32 + s_add (1:1)", k_fma_salu, 34}, {"v_mul_f32 + s_add (1:1)", k_mul_salu, 34},
    {"v_mul_f32 + 2 SALU (1:2)", k_mul_2salu, 34},
};

int main(int argc, char** argv) {
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, 1024 * sizeof(float));
    hipMalloc(&clk, 4 * sizeof(unsigned long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 4096;
    const double clock_hz = 2.4e9;
    auto run = [&](const Body& b, int w, bool print) {
        const int blocks = cus * w;
        hipLaunchKernelGGL(b.fn, dim3(blocks), dim3(256), 0, 0, out, 8, nullptr);
        hipEventRecord(e0);
        hipLaunchKernelGGL(b.fn, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c[4] = {0, 0, 0, 0};
        hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
        const double winstr_per_simd = (double)w * iters * b.instr_per_iter;
        const double cyc = ms * 1e-3 * clock_hz / winstr_per_simd;
        const double wave_cyc = (double)c[0] / (iters * b.instr_per_iter);
        if (print)
            printf("{\"body\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_wave_instr\": %.3f, "
                   "\"one_wave_cycles_per_own_instr\": %.3f}\n",
                   b.name, w, ms, cyc, wave_cyc);
    };
    if (argc >= 3) {  // one body at one occupancy (for counter passes)
        for (const Body& b : kBodies)
            if (!strcmp(b.name, argv[1])) run(b, atoi(argv[2]), true);
        return 0;
    }
    for (const Body& b : kBodies) {
        for (int w : {1, 2, 4, 8}) run(b, w, true);
        fflush(stdout);
    }
    return 0;
}
