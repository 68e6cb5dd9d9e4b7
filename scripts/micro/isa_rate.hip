// Microbenchmark (diagnostic, not product): issue cost of single VALU instructions on
// gfx950, every SIMD full (8 waves of 256-thread workgroups per CU), 8 independent
// dependency chains per lane so latency is hidden.  Prints cycles per wave-instruction
// per SIMD (the "(pair)" rows: cycles per PAIR of instructions; a pair costing no more than
// one of its halves means the two issue side by side).
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/isa_rate scripts/micro/isa_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void kop(uint32_t* out, int iters, uint64_t* clk_out)
{
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a0 = t, a1 = t * 3, a2 = t * 5, a3 = t * 7, a4 = t * 11, a5 = t * 13, a6 = t * 17, a7 = t * 19;
    uint32_t b0 = t ^ 1, b1 = t ^ 2, b2 = t ^ 3, b3 = t ^ 4, b4 = t ^ 5, b5 = t ^ 6, b6 = t ^ 7, b7 = t ^ 8;
    uint32_t sb0 = 1, sb1 = 2, sb2 = 3, sb3 = 4, sb4 = 5, sb5 = 6, sb6 = 7, sb7 = 8;
    uint64_t d0 = t, d1 = t + 1, d2 = t + 2, d3 = t + 3, d4 = t + 4, d5 = t + 5, d6 = t + 6, d7 = t + 7;
    const uint32_t k = 0xD2511F53u;
    const uint64_t msk = 0x5555555555555555ull;
    const uint64_t dx = (uint64_t)t * 0x100000001ull, dy = dx ^ 0x3F8000003F800000ull;
    uint64_t mk0, mk1, mk2, mk3, mk4, mk5, mk6, mk7;
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < iters; ++i) {
#define STEP(j)                                                                                                 \
        if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a##j) : "v"(k));                  \
        if constexpr (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(d##j) : "v"(d0));             \
        if constexpr (OP == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(d##j) : "v"(a##j), "s"(k) : "vcc"); \
        if constexpr (OP == 3) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a##j) : "s"(k));                  \
        if constexpr (OP == 4) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##j) : "s"(k));                  \
        if constexpr (OP == 5) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d##j) : "v"(d0));                \
        if constexpr (OP == 6) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d##j) : "v"(d0));                    \
        if constexpr (OP == 7) asm volatile("v_log_f32 %0, %0" : "+v"(a##j));                                   \
        if constexpr (OP == 8) asm volatile("v_exp_f32 %0, %0" : "+v"(a##j));                                   \
        if constexpr (OP == 9) asm volatile("v_rcp_f32 %0, %0" : "+v"(a##j));                                   \
        if constexpr (OP == 10) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a##j) : "v"(k)); \
        if constexpr (OP == 11) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##j) : "v"(k));           \
        if constexpr (OP == 12) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a##j));                              \
        if constexpr (OP == 13) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d##j) : "v"(d0));                   \
        if constexpr (OP == 14) asm volatile("v_rcp_f64 %0, %0" : "+v"(d##j));                                  \
        if constexpr (OP == 15) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a##j));                                 \
        if constexpr (OP == 16) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a##j) : "v"(k), "s"(msk));   \
        if constexpr (OP == 17) asm volatile("v_cmp_lt_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1" : "+v"(a##j), "=s"(mk##j) : "v"(k)); \
        if constexpr (OP == 18) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a##j) : "v"(k));                   \
        if constexpr (OP == 19) asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(a##j) : "v"(k));               \
        if constexpr (OP == 20) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##j) : "v"(k));                    \
        if constexpr (OP == 21) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a##j)); \
        if constexpr (OP == 22) asm volatile("v_cmp_lt_u32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a##j) : "v"(k) : "vcc"); \
        if constexpr (OP == 23) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a##j) : "v"(t), "v"(k)); \
        if constexpr (OP == 24) asm volatile("v_fma_f32 %0, %0, %2, %2\n\tv_exp_f32 %1, %1" : "+v"(a##j), "+v"(b##j) : "v"(k)); \
        if constexpr (OP == 25) asm volatile("v_fma_f32 %0, %0, %2, %2\n\tv_add_u32 %1, %1, %2" : "+v"(a##j), "+v"(b##j) : "v"(k)); \
        if constexpr (OP == 26) asm volatile("v_fma_f32 %0, %0, %2, %2\n\ts_add_u32 %1, %1, %3" : "+v"(a##j), "+s"(sb##j) : "v"(k), "s"(k)); \
        if constexpr (OP == 27) asm volatile("v_fma_f32 %0, %0, %2, %2\n\tv_pk_fma_f32 %1, %1, %3, %3" : "+v"(a##j), "+v"(d##j) : "v"(k), "v"(d0)); \
        if constexpr (OP == 28) asm volatile("v_fma_f32 %0, %0, %2, %2\n\tv_fma_f32 %1, %1, %2, %2" : "+v"(a##j), "+v"(b##j) : "v"(k)); \
        if constexpr (OP == 29) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(d##j) : "v"(dx), "v"(dy)); \
        if constexpr (OP == 30) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d##j) : "v"(dx), "v"(dy)); \
        if constexpr (OP == 31) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a##j) : "v"(t)); \
        if constexpr (OP == 32) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a##j) : "v"(t)); \
        if constexpr (OP == 33) asm volatile("v_fma_f32 %0, %2, %3, %0\n\tv_fma_f32 %1, %2, %3, %1" : "+v"(a##j), "+v"(b##j) : "v"(t), "v"(k)); \
        if constexpr (OP == 34) asm volatile("v_fma_f32 %0, %2, %3, %0\n\tv_pk_fma_f32 %1, %4, %5, %1" : "+v"(a##j), "+v"(d##j) : "v"(t), "v"(k), "v"(dx), "v"(dy)); \
        if constexpr (OP == 35) asm volatile("v_fma_f32 %0, %2, %3, %0\n\tv_exp_f32 %1, %1" : "+v"(a##j), "+v"(b##j) : "v"(t), "v"(k)); \
        if constexpr (OP == 36) asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a##j) : "v"(t), "s"(msk)); \
        if constexpr (OP == 37) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(d##j) : "v"(a##j), "v"(t) : "vcc"); \
        if constexpr (OP == 38) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(a##j) : "v"(t)); \
        if constexpr (OP == 39) asm volatile("v_cndmask_b32_e32 %0, %1, %0, vcc" : "+v"(a##j) : "v"(t)); \
        if constexpr (OP == 40) asm volatile("v_max_f32 %0, %1, %0" : "+v"(a##j) : "v"(t)); \
        if constexpr (OP == 41) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(a##j) : "v"(t), "v"(k)); \
        if constexpr (OP == 42) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(d##j) : "v"(dx)); \
        if constexpr (OP == 43) asm volatile("v_fmaak_f32 %0, %1, %0, 0x3f800000" : "+v"(a##j) : "v"(t)); \
        if constexpr (OP == 44) asm volatile("v_cmp_lt_f32_e32 vcc, %0, %1" : : "v"(a##j), "v"(t) : "vcc"); \
        if constexpr (OP == 45) asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(a##j) : "v"(b##j)); \
        if constexpr (OP == 46) asm volatile("v_add_f64 %0, %1, %0" : "+v"(d##j) : "v"(dx)); \
        if constexpr (OP == 47) asm volatile("v_med3_f32 %0, %1, %2, %0" : "+v"(a##j) : "v"(t), "v"(k)); \
        if constexpr (OP == 48) asm volatile("v_mov_b32 %0, %1" : "=v"(a##j) : "v"(b##j));
        REP8(STEP)
#undef STEP
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        clk_out[0] = t1 - t0;
        clk_out[1] = r1 - r0;
    }
    out[t] ^= b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7 ^ sb0 ^ sb1 ^ sb2 ^ sb3 ^ sb4 ^ sb5 ^ sb6 ^ sb7;
    out[t] += a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(d0 ^ d1 ^ d2 ^ d3 ^ d4 ^ d5 ^ d6 ^ d7);
}

int main()
{
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8 * 4, threads = 256, iters = 4096;   // 8 waves per SIMD, 4 rounds
    uint32_t* o;
    uint64_t* ck;
    hipMalloc(&o, (size_t)blocks * threads * 4);
    hipMalloc(&ck, 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_mad_u64_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_fma_f64",
                           "v_add_f64", "v_log_f32", "v_exp_f32", "v_rcp_f32", "v_bitop3_b32", "v_cndmask_b32",
                           "v_cvt_f32_u32", "v_mul_f64", "v_rcp_f64", "v_sqrt_f32", "v_cndmask_e64 s[]",
                           "v_cmp+v_cndmask", "v_max_f32", "v_med3_f32", "v_add_u32", "v_mov_b32_dpp",
                           "v_cmp_e32+cndmask_e32", "v_fma_f32 distinct",
                           "fma+exp (pair)", "fma+add_u32 (pair)", "fma+s_add (pair)", "fma+pk_fma (pair)",
                           "fma+fma (pair)", "v_pk_fma_f32 distinct", "v_fma_f64 distinct", "v_add_u32 distinct",
                           "v_mul_f32 distinct", "fma+fma distinct (pair)", "fma+pk_fma distinct (pair)",
                           "fma+exp distinct (pair)", "v_cndmask_e64 distinct", "v_mad_u64_u32 distinct",
                           "v_mul_hi_u32 distinct", "v_cndmask_e32 vcc distinct", "v_max_f32 distinct",
                           "v_bitop3 distinct", "v_pk_mul_f32 distinct", "v_fmaak_f32 literal", "v_cmp_lt_f32_e32",
                           "v_cvt_f32_u32 distinct", "v_add_f64 distinct", "v_med3_f32 distinct", "v_mov_b32"};
    auto run = [&](int op, auto launch) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double wave_instr = (double)blocks * threads / 64 * iters * 8;
        const double clk = p.clockRate * 1e3;   // kHz -> Hz
        const double cyc = ms * 1e-3 * clk * cus * 4 / wave_instr;
        uint64_t cc[2];
        hipMemcpy(cc, ck, 16, hipMemcpyDeviceToHost);
        const double mhz = (double)cc[0] / ((double)cc[1] / 100.0);   // s_memrealtime: 100 MHz
        printf("%-20s %8.3f ms  %6.2f cycles/wave-instr/SIMD at nominal %.0f MHz; wave 0 saw %.0f MHz -> %.2f cycles\n",
               names[op], ms, cyc, clk / 1e6, mhz, cyc * mhz / (clk / 1e6));
    };
#define RUN(op) run(op, [&] { kop<op><<<blocks, threads>>>(o, iters, ck); });
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9) RUN(10) RUN(11) RUN(12) RUN(13) RUN(14) RUN(15)
    RUN(16) RUN(17) RUN(18) RUN(19) RUN(20) RUN(21) RUN(22) RUN(23) RUN(24) RUN(25) RUN(26) RUN(27) RUN(28) RUN(29) RUN(30) RUN(31) RUN(32) RUN(33) RUN(34) RUN(35) RUN(36) RUN(37) RUN(38) RUN(39) RUN(40) RUN(41) RUN(42) RUN(43) RUN(44) RUN(45) RUN(46) RUN(47) RUN(48)
    return 0;
}
