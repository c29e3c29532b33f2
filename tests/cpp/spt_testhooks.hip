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
