// Diagnostic kernel for scripts/contend.py: one wave per SIMD (256-thread workgroups,
// one per CU) holding ~NV*2 VGPRs for a given time, either sleeping (mode 0) or
// running independent fp64 FMA chains (mode 1).  Measures what
// a resident walk wave costs the expansion beside it: registers alone, or issue.
#include <hip/hip_runtime.h>
#include <cstdint>
#ifndef NV
#define NV 68
#endif
#ifndef NVG
#define NVG 144
#endif
extern "C" __global__ __launch_bounds__(256, 1) void occupy(int mode, int iters, double* out)
{
    double v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = threadIdx.x * 1e-3 + i;
    for (int it = 0; it < iters; ++it) {
        if (mode == 0) {
            __builtin_amdgcn_s_sleep(100);
#pragma unroll
            for (int i = 0; i < NV; ++i) asm volatile("" : "+v"(v[i]));
        } else {
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = fma(v[i], 0.999999, 1e-9);
        }
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += v[i];
    if (s == 12345.678) out[threadIdx.x] = s;
}
extern "C" int launch_occupy(int mode, int iters, int blocks, void* stream, double* out)
{
    hipLaunchKernelGGL(occupy, dim3(blocks), dim3(256), 0, (hipStream_t)stream, mode, iters, out);
    return (int)hipGetLastError();
}
