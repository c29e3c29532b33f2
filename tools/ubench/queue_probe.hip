// queue_probe.hip -- measures the primitives a resident render service relies on
// ("Render service"):
//   T1/T2  hipStreamWaitValue32 on a counter a RUNNING kernel on another stream
//          increments (plain hipMalloc word / hipMallocSignalMemory word): does the
//          gated kernel wait, and how long after the increment does it start?
//   T3     hipStreamWriteValue32 into a word a running kernel polls: is it seen?
//   T4     a one-thread "publish" kernel storing the word instead.
//   T5     host cost of one job's stream operations (publish kernel + wait value +
//          gated kernel + event) over 1000 jobs.
//   T6-T9  which streams share a hardware queue with a long-running kernel (priorities).
//   T10    a running kernel polling a word of coherent pinned host memory the host stores.
// Every spin is bounded (s_memrealtime, 100 MHz): a missed signal ends in a timeout
// code, never a hang.  Build: hipcc --offload-arch=gfx950 -O2 queue_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

__device__ __forceinline__ unsigned long long now_rt() { return __builtin_amdgcn_s_memrealtime(); }

// producer: waits `delay_us`, then records the time and adds 1 to *ctr (release, agent)
__global__ void producer(unsigned *ctr, unsigned long long *t_out, unsigned delay_us)
{
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = now_rt();
    while (now_rt() - t0 < (unsigned long long)delay_us * 100ull) __builtin_amdgcn_s_sleep(2);
    t_out[0] = now_rt();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// consumer: records its start time and the counter value it sees
__global__ void consumer(const unsigned *ctr, unsigned long long *t_out, unsigned *seen)
{
    if (threadIdx.x != 0) return;
    t_out[1] = now_rt();
    seen[0] = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// poller: spins (bounded: timeout_us) until *w >= want; records the time seen or ~0
__global__ void poller(const unsigned *w, unsigned want, unsigned long long *t_out, unsigned timeout_us)
{
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = now_rt();
    t_out[0] = t0;
    for (;;) {
        const unsigned v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t = now_rt();
        if (v >= want) {
            t_out[1] = t;
            return;
        }
        if (t - t0 > (unsigned long long)timeout_us * 100ull) {
            t_out[1] = ~0ull;
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

__global__ void publish(unsigned *w, unsigned v, unsigned long long *t_out)
{
    if (threadIdx.x != 0) return;
    t_out[2] = now_rt();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void noop(unsigned *p)
{
    if (threadIdx.x == 0 && p) p[1] = p[0];
}

static int wait_test(const char *name, unsigned *ctr, unsigned long long *d_t, unsigned *d_seen)
{
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(ctr, 0, 4));
        CK(hipMemset(d_t, 0, 32));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(producer, dim3(1), dim3(64), 0, a, ctr, d_t, 2000u);
        const hipError_t ew = hipStreamWaitValue32(b, ctr, 1u, hipStreamWaitValueGte, 0xFFFFFFFFu);
        hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, b, ctr, d_t, d_seen);
        // bounded wait for both streams
        const auto t0 = std::chrono::steady_clock::now();
        bool done = false;
        while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5)) {
            if (hipStreamQuery(a) == hipSuccess && hipStreamQuery(b) == hipSuccess) {
                done = true;
                break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        if (!done) {
            printf("%s rep %d: streams not done after 5 s (wait api rc %d)\n", name, rep, (int)ew);
            unsigned one = 1;
            CK(hipMemcpy(ctr, &one, 4, hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            continue;
        }
        unsigned long long t[2];
        unsigned seen = 0;
        CK(hipMemcpy(t, d_t, 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&seen, d_seen, 4, hipMemcpyDeviceToHost));
        printf("%s rep %d: wait rc %d, consumer start - increment = %.2f us, consumer saw %u\n", name, rep, (int)ew,
               ((double)(long long)(t[1] - t[0])) / 100.0, seen);
    }
    CK(hipStreamDestroy(a));
    CK(hipStreamDestroy(b));
    return 0;
}

int main()
{
    int dev = 0;
    CK(hipSetDevice(dev));
    int can = -1;
    (void)hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, dev);
    printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can);
    unsigned *ctr = nullptr, *sig = nullptr, *seen = nullptr;
    unsigned long long *d_t = nullptr;
    CK(hipMalloc(&ctr, 256));
    CK(hipMalloc(&seen, 256));
    CK(hipMalloc(&d_t, 256));
    if (wait_test("T1 hipMalloc word", ctr, d_t, seen)) return 1;
    const hipError_t es = hipExtMallocWithFlags((void **)&sig, 8, hipMallocSignalMemory);
    printf("hipMallocSignalMemory alloc rc %d\n", (int)es);
    if (es == hipSuccess && wait_test("T2 signal word", sig, d_t, seen)) return 1;

    // T3: hipStreamWriteValue32 seen by a running poller
    {
        hipStream_t a, c;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemset(ctr, 0, 4));
            CK(hipMemset(d_t, 0, 32));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(poller, dim3(1), dim3(64), 0, a, ctr, 1u, d_t, 200000u);
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            const auto h0 = std::chrono::steady_clock::now();
            const hipError_t ew = hipStreamWriteValue32(c, ctr, 1u, 0);
            const double api_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
            CK(hipStreamSynchronize(c));
            const double done_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
            CK(hipStreamSynchronize(a));
            const double seen_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
            unsigned long long t[2];
            CK(hipMemcpy(t, d_t, 16, hipMemcpyDeviceToHost));
            printf("T3 writeValue rep %d: rc %d api %.1f us, write stream done %.1f us, poller %s (%.1f us after its "
                   "start), host saw poller end at %.1f us\n",
                   rep, (int)ew, api_us, done_us, t[1] == ~0ull ? "TIMED OUT" : "saw it", (double)(t[1] - t[0]) / 100.0,
                   seen_us);
        }
        // T4: a publish kernel instead
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemset(ctr, 0, 4));
            CK(hipMemset(d_t, 0, 32));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(poller, dim3(1), dim3(64), 0, a, ctr, 1u, d_t, 200000u);
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            hipLaunchKernelGGL(publish, dim3(1), dim3(64), 0, c, ctr, 1u, d_t);
            CK(hipStreamSynchronize(c));
            CK(hipStreamSynchronize(a));
            unsigned long long t[3];
            CK(hipMemcpy(t, d_t, 24, hipMemcpyDeviceToHost));
            printf("T4 publish kernel rep %d: poller %s, seen %.2f us after the publish kernel's store\n", rep,
                   t[1] == ~0ull ? "TIMED OUT" : "saw it", ((double)(long long)(t[1] - t[2])) / 100.0);
        }
        // T5: host cost of one job's stream operations
        {
            const int jobs = 1000;
            CK(hipMemset(ctr, 0, 4));
            CK(hipDeviceSynchronize());
            hipEvent_t ev;
            CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            const auto h0 = std::chrono::steady_clock::now();
            for (int j = 0; j < jobs; ++j) {
                hipLaunchKernelGGL(publish, dim3(1), dim3(64), 0, c, ctr, (unsigned)(j + 1), d_t);
                CK(hipStreamWaitValue32(a, ctr, (unsigned)(j + 1), hipStreamWaitValueGte, 0xFFFFFFFFu));
                hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, a, seen);
                CK(hipEventRecord(ev, a));
            }
            const double enq = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
            CK(hipStreamSynchronize(a));
            const double all = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
            printf("T5 %d jobs: enqueue %.2f us per job, all done %.2f us per job\n", jobs, enq / jobs, all / jobs);
            CK(hipEventDestroy(ev));
        }
        CK(hipStreamDestroy(a));
        CK(hipStreamDestroy(c));
    }
    // T6: a long kernel on one stream, short kernels on 7 other streams: which of them run
    // while it runs (streams sharing a hardware queue with it would wait for it)
    {
        const int ns = 8;
        hipStream_t st[ns];
        for (int i = 0; i < ns; ++i) CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
        unsigned long long *d_ts = nullptr;
        CK(hipMalloc(&d_ts, 64 * sizeof(unsigned long long)));
        CK(hipMemset(d_ts, 0, 64 * sizeof(unsigned long long)));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(producer, dim3(1), dim3(64), 0, st[0], ctr, d_ts, 30000u);  // 30 ms
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        for (int i = 1; i < ns; ++i) hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, st[i], ctr, d_ts + 2 * i, seen);
        CK(hipDeviceSynchronize());
        unsigned long long t[64];
        CK(hipMemcpy(t, d_ts, sizeof t, hipMemcpyDeviceToHost));
        const char *env = getenv("GPU_MAX_HW_QUEUES");
        printf("T6 GPU_MAX_HW_QUEUES=%s: long kernel ends at t=0; short kernels start at", env ? env : "(unset)");
        for (int i = 1; i < ns; ++i) printf(" %+.1f", ((double)(long long)(t[2 * i + 1] - t[0])) / 100.0);
        printf(" us\n");
        for (int i = 0; i < ns; ++i) CK(hipStreamDestroy(st[i]));
        // T7: the same with the long kernel on a high-priority stream, 12 short streams
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        hipStream_t hs;
        CK(hipStreamCreateWithPriority(&hs, hipStreamNonBlocking, hi));
        const int nl = 12;
        hipStream_t ls[nl];
        for (int i = 0; i < nl; ++i) CK(hipStreamCreateWithFlags(&ls[i], hipStreamNonBlocking));
        CK(hipMemset(d_ts, 0, 64 * sizeof(unsigned long long)));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(producer, dim3(1), dim3(64), 0, hs, ctr, d_ts, 30000u);
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        for (int i = 0; i < nl; ++i) hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, ls[i], ctr, d_ts + 2 * (i + 1), seen);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(t, d_ts, sizeof t, hipMemcpyDeviceToHost));
        printf("T7 priority range [%d, %d], long kernel on priority %d: short kernels (12 streams) start at", lo, hi, hi);
        for (int i = 0; i < nl; ++i) printf(" %+.1f", ((double)(long long)(t[2 * (i + 1) + 1] - t[0])) / 100.0);
        printf(" us\n");
        CK(hipStreamDestroy(hs));
        for (int i = 0; i < nl; ++i) CK(hipStreamDestroy(ls[i]));
        // T8 / T9: the long kernel on a high-priority stream, short kernels on 7 other
        // streams of the same (high) or the lowest priority
        for (int variant = 0; variant < 2; ++variant) {
            const int prio = variant == 0 ? hi : lo;
            hipStream_t h0, os[7];
            CK(hipStreamCreateWithPriority(&h0, hipStreamNonBlocking, hi));
            for (int i = 0; i < 7; ++i) CK(hipStreamCreateWithPriority(&os[i], hipStreamNonBlocking, prio));
            CK(hipMemset(d_ts, 0, 64 * sizeof(unsigned long long)));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(producer, dim3(1), dim3(64), 0, h0, ctr, d_ts, 30000u);
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            for (int i = 0; i < 7; ++i) hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, os[i], ctr, d_ts + 2 * (i + 1), seen);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(t, d_ts, sizeof t, hipMemcpyDeviceToHost));
            printf("T%d long kernel on priority %d, short kernels on 7 streams of priority %d start at", 8 + variant, hi,
                   prio);
            for (int i = 0; i < 7; ++i) printf(" %+.1f", ((double)(long long)(t[2 * (i + 1) + 1] - t[0])) / 100.0);
            printf(" us\n");
            CK(hipStreamDestroy(h0));
            for (int i = 0; i < 7; ++i) CK(hipStreamDestroy(os[i]));
        }
    }
    // T10: a running kernel polls a word in coherent pinned host memory that the host
    // stores (no stream operation): host store -> the kernel's end seen by the host
    {
        unsigned *hw = nullptr;
        CK(hipHostMalloc((void **)&hw, 64, hipHostMallocCoherent));
        hipStream_t a;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        for (int rep = 0; rep < 3; ++rep) {
            __atomic_store_n(hw, 0u, __ATOMIC_RELEASE);
            CK(hipMemset(d_t, 0, 32));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(poller, dim3(1), dim3(64), 0, a, hw, 1u, d_t, 200000u);
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            const auto h0 = std::chrono::steady_clock::now();
            __atomic_store_n(hw, 1u, __ATOMIC_RELEASE);
            while (hipStreamQuery(a) == hipErrorNotReady) {
            }
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
            unsigned long long t2[2];
            CK(hipMemcpy(t2, d_t, 16, hipMemcpyDeviceToHost));
            printf("T10 host store rep %d: poller %s, host saw the kernel end %.1f us after its store\n", rep,
                   t2[1] == ~0ull ? "TIMED OUT" : "saw it", us);
        }
        CK(hipStreamDestroy(a));
        CK(hipHostFree(hw));
    }
    printf("done\n");
    return 0;
}
