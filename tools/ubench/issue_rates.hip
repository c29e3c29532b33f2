// Issue-cost microbenchmark of the VALU operations on the render path (gfx950).
// Each kernel runs 8 independent dependency chains per lane (enough to cover
// latency at full occupancy) for ITERS iterations; time per op relative to
// v_add_f32 gives the issue cost.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
#define CHAINS 8

template <int OP>
__global__ __launch_bounds__(256) void bench(uint32_t *out, uint32_t seed)
{
    uint32_t u[CHAINS];
    uint64_t q[CHAINS];
    float f[CHAINS];
    double g[CHAINS];
    for (int c = 0; c < CHAINS; ++c) {
        u[c] = seed + threadIdx.x * 7 + c;
        q[c] = ((uint64_t)u[c] << 32) | (u[c] * 3u);
        f[c] = 1.0f + (float)u[c] * 1e-9f;
        g[c] = 1.0 + (double)u[c] * 1e-12;
    }
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (OP == 0) f[c] = f[c] + 1.0000001f;                                     // v_add_f32
            if (OP == 1) u[c] = u[c] * 0x9E3779B9u + 1u;                               // v_mul_lo_u32 + add
            if (OP == 2) u[c] = __umulhi(u[c], 0x9E3779B9u) ^ u[c];                    // v_mul_hi_u32 + xor
            if (OP == 3) q[c] = q[c] * 0xBF58476D1CE4E5B9ull;                          // 64-bit mul
            if (OP == 4) f[c] = __builtin_sqrtf(f[c] + 1.0f);                          // IEEE sqrt sequence
            if (OP == 5) f[c] = 1.0000001f / f[c];                                     // IEEE div sequence
            if (OP == 6) g[c] = g[c] * 1.0000000001 + 1e-12;                           // f64 mul + add
            if (OP == 7) f[c] = __builtin_amdgcn_sqrtf(f[c] + 1.0f);                   // v_sqrt_f32 + add
            if (OP == 8) u[c] = __mul24(u[c], 0x3779B9u) + 1u;                         // v_mul_u32_u24 + add
            if (OP == 9) q[c] = (q[c] ^ (q[c] >> 30)) * 0xBF58476D1CE4E5B9ull;         // splitmix step
        }
    }
    uint32_t acc = 0;
    for (int c = 0; c < CHAINS; ++c)
        acc ^= u[c] ^ (uint32_t)q[c] ^ (uint32_t)(q[c] >> 32) ^ __float_as_uint(f[c]) ^ (uint32_t)__double_as_longlong(g[c]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
float run(uint32_t *out, int blocks)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(a);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 3;
}

int main()
{
    int cu = 0;
    hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cu * 8;  // 8 waves per SIMD
    uint32_t *out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    const char *names[] = {"v_add_f32", "mul_lo_u32+add", "mul_hi_u32+xor", "u64 mul", "sqrtf (IEEE)",
                           "div (IEEE)", "f64 mul+add", "v_sqrt_f32+add", "mul_u32_u24+add", "splitmix step"};
    float t[10];
    t[0] = run<0>(out, blocks);
    t[1] = run<1>(out, blocks);
    t[2] = run<2>(out, blocks);
    t[3] = run<3>(out, blocks);
    t[4] = run<4>(out, blocks);
    t[5] = run<5>(out, blocks);
    t[6] = run<6>(out, blocks);
    t[7] = run<7>(out, blocks);
    t[8] = run<8>(out, blocks);
    t[9] = run<9>(out, blocks);
    const double ops = (double)blocks * 256 / 64 * ITERS * CHAINS;  // wave-ops per kernel
    for (int i = 0; i < 10; ++i)
        printf("%-18s %8.3f ms  %6.2f x v_add_f32  (%.2f ns per wave-op per CU)\n", names[i], t[i], t[i] / t[0],
               t[i] * 1e6 / ops * cu);
    hipFree(out);
    return 0;
}
