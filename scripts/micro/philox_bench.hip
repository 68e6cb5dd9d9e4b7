// Microbenchmark (diagnostic, not product): Philox4x32-10 formulations and fp32
// inverse-normal variants, throughput per lane on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox_mulhi(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    return U4{c0, c1, c2, c3};
}

__device__ __forceinline__ U4 philox_mad64(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    return U4{c0, c1, c2, c3};
}

template <int V>
__global__ void kphilox(uint32_t* out, int iters, uint32_t seed)
{
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        U4 u = V == 0 ? philox_mulhi(i, 0x10000000u, c, 0, seed, 0) : philox_mad64(i, 0x10000000u, c, 0, seed, 0);
        acc ^= u.x + u.y + u.z + u.w;
    }
    out[c] = acc;
}

template <int V>
__global__ void kndtri(float* out, int iters)
{
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0;
    for (int i = 0; i < iters; ++i) {
        float u = ((c * 2654435761u + i * 40503u) >> 8) * 0x1p-24f + 0x1p-25f;
        if (V == 0) acc += normcdfinvf(u);
        else acc += logf(u);
    }
    out[c] = acc;
}

__global__ void kpow(double* out, int iters)
{
    uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0;
    for (int i = 0; i < iters; ++i) {
        double u = ((c * 2654435761u + i * 40503u) >> 8) * 0x1p-24 + 0x1p-25;
        acc += pow(1.0e-4 + 0.05 * u, -1.5151515151515154);
    }
    out[c] = acc;
}

int main()
{
    const int blocks = 256 * 32, threads = 256, iters = 256;
    const double n = (double)blocks * threads * iters;
    uint32_t* o; float* of; double* od;
    hipMalloc(&o, blocks * threads * 4); hipMalloc(&of, blocks * threads * 4); hipMalloc(&od, blocks * threads * 8);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float ms;
    auto run = [&](const char* name, auto launch) {
        launch(); hipDeviceSynchronize();
        hipEventRecord(a); for (int r = 0; r < 5; ++r) launch(); hipEventRecord(b); hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("%-22s %8.3f ms  %7.2f G/s  %.2f ns/lane-op-equiv\n", name, ms / 5, n / (ms / 5 * 1e6), ms / 5 * 1e6 / n * 256 * 4 * 32 * 2.4);
    };
    run("philox mul_lo+mul_hi", [&] { kphilox<0><<<blocks, threads>>>(o, iters, 7); });
    run("philox mad_u64_u32", [&] { kphilox<1><<<blocks, threads>>>(o, iters, 7); });
    run("normcdfinvf", [&] { kndtri<0><<<blocks, threads>>>(of, iters); });
    run("logf", [&] { kndtri<1><<<blocks, threads>>>(of, iters); });
    run("pow f64", [&] { kpow<<<blocks, threads>>>(od, iters); });
    return 0;
}
