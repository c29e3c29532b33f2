// spt_testhooks.hip -- test-only kernels for the render-service liveness tests
// (tests/test_gpu_service.py); built into simplepathtracer_amd/lib/libspt_testhooks.so,
// never linked into libspt_hip.so.
//
// spt_test_blocker: `blocks` blocks of 512 threads, each wave holding 256 VGPRs (half a
// SIMD's register file), spinning for `us` microseconds.  Like RCCL's collective kernels
// for gfx950 (248-256 VGPRs, up to 512 threads per block: DESIGN.md §5), such a block
// needs a CU with no render-service wave on it, so while a session is resident it cannot
// start: work queued behind it on a stream (a fold) waits for the session to end.
#include <hip/hip_runtime.h>

#include <stdint.h>

__global__ __launch_bounds__(512) void blocker_kernel(uint32_t us, uint32_t *ran)
{
    // the clobber makes the kernel allocate all 256 VGPRs a wave of a 512-thread block may
    // have; no register is actually used
    asm volatile("" ::: "v255");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(32);
    if (ran && threadIdx.x == 0) atomicAdd(ran, 1u);
}

extern "C" __attribute__((visibility("default"))) int spt_test_blocker(void *stream, uint32_t us, uint32_t blocks,
                                                                       uint32_t *d_ran)
{
    hipLaunchKernelGGL(blocker_kernel, dim3(blocks ? blocks : 1u), dim3(512), 0, (hipStream_t)stream, us, d_ran);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

// VGPRs per wave of blocker_kernel (from the code object), for the test's own check
extern "C" __attribute__((visibility("default"))) int spt_test_blocker_vgprs(int *vgprs)
{
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, (const void *)blocker_kernel) != hipSuccess) return 3;
    *vgprs = fa.numRegs;
    return 0;
}

// Placement probes for the reserved-CU tests (tests/test_gpu_reserve.py, tools/cu_mask_probe.py):
// each block's first thread records HW_ID (gfx9: wave[3:0] simd[5:4] cu[11:8] sh[12]
// se[15:13]), XCC_ID and its start time (100 MHz ticks), then the block spins `us`.
__device__ inline void record_where(uint32_t *where, unsigned long long t0)
{
    if (where && threadIdx.x == 0) {
        where[4 * blockIdx.x + 0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
        where[4 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        where[4 * blockIdx.x + 2] = (uint32_t)t0;
        where[4 * blockIdx.x + 3] = (uint32_t)(t0 >> 32);
    }
}

__global__ __launch_bounds__(512) void blocker_where_kernel(uint32_t us, uint32_t *where)
{
    asm volatile("" ::: "v255");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    record_where(where, t0);
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(32);
}

__global__ __launch_bounds__(64) void where_kernel(uint32_t us, uint32_t *where)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    record_where(where, t0);
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(32);
}

// big != 0: the blocker's shape (512 threads, 256 VGPRs); else 64-thread blocks.
// where: 4 words per block
extern "C" __attribute__((visibility("default"))) int spt_test_where(void *stream, uint32_t us, uint32_t blocks,
                                                                     int big, uint32_t *where)
{
    if (big)
        hipLaunchKernelGGL(blocker_where_kernel, dim3(blocks ? blocks : 1u), dim3(512), 0, (hipStream_t)stream, us, where);
    else
        hipLaunchKernelGGL(where_kernel, dim3(blocks ? blocks : 1u), dim3(64), 0, (hipStream_t)stream, us, where);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

// One thread stores s_memrealtime (100 MHz ticks) to *out: queued on a stream after a
// render, its value is a time at which the render had ended (tests/test_gpu_reserve.py)
__global__ void stamp_kernel(unsigned long long *out) { *out = __builtin_amdgcn_s_memrealtime(); }

extern "C" __attribute__((visibility("default"))) int spt_test_stamp(void *stream, unsigned long long *out)
{
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, out);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

// A stream whose CU mask holds the low `keep` of `total` bits (the layout spt_ctx.cpp's
// masked_for uses); *out receives the hipStream_t.
extern "C" __attribute__((visibility("default"))) int spt_test_masked_stream(uint32_t keep, uint32_t total, void **out)
{
    uint32_t mask[64] = {};
    if (total == 0 || total > 64 * 32 || keep > total) return 1;
    for (uint32_t i = 0; i < keep; ++i) mask[i / 32] |= 1u << (i % 32);
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (total + 31) / 32, mask) != hipSuccess) return 3;
    *out = (void *)s;
    return 0;
}

extern "C" __attribute__((visibility("default"))) int spt_test_stream_destroy(void *s)
{
    return hipStreamDestroy((hipStream_t)s) == hipSuccess ? 0 : 3;
}

// WRITE_SIZE calibration for 4-byte sample words (tools/write_calib.sh):
// `words` u32 words written once each, by 64-lane waves over 256-word (1 KiB) chunks.
// pattern 0: four coalesced stores per wave (64 lanes x 4 B each, the whole chunk);
// pattern 1: the chunk's 256 words one lane at a time, 256 stores per wave, in a
// scrambled order (stride 97 mod 256): the lines are assembled in L2 from single words,
// the way lanes finishing their paths at different times write their slots.
__global__ __launch_bounds__(256) void write_calib_kernel(uint32_t *out, uint32_t words, int pattern)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t chunk = (blockIdx.x * 256u + threadIdx.x) >> 6;
    const uint32_t base = chunk * 256u;
    if (base >= words) return;
    if (pattern == 0) {
        for (uint32_t r = 0; r < 4u; ++r) out[base + r * 64u + lane] = base + r * 64u + lane;
    } else {
        for (uint32_t r = 0; r < 256u; ++r) {
            const uint32_t w = (r * 97u) & 255u;
            if ((w & 63u) == lane) out[base + w] = base + w;
        }
    }
}

extern "C" __attribute__((visibility("default"))) int spt_test_write_calib(void *stream, uint32_t *out, uint32_t words,
                                                                           int pattern)
{
    if (words % 256u) return 1;
    const uint32_t waves = words / 256u;
    hipLaunchKernelGGL(write_calib_kernel, dim3((waves + 3u) / 4u), dim3(256), 0, (hipStream_t)stream, out, words, pattern);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
