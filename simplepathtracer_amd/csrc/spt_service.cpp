// spt_service.cpp -- the render service's host half: sessions of the resident kernel, job
// publication, flow control and bounded waits (spt_host.h).
#include "spt_host.h"

namespace spt_api {

// ---- render service (DESIGN.md §4.7 "Render service") ----------------------------------
// Liveness rests on two rules (DESIGN.md §4.7 "Liveness"):
//  * a publication never waits for anything but its session's start: when one would
//    have to wait for an unfinished fold (its ring words or its completion counter still
//    in use), the session is ended first and the new session's kernel itself waits for
//    those folds -- so no publish is ever held behind work that waits for the session;
//  * a wave leaves an idle session only through the closing handshake (spt_internal.h
//    kSvcIdleTicks): the host commits every job before publishing it and ends a session
//    whose closing flag it finds raised, so no job is published to a session that left.
// Every host wait on a session is bounded (SPT_SVC_TIMEOUT_MS, svc_wait).

hipEvent_t svc_event(spt_ctx *ctx)
{
    Service &v = ctx->svc;
    if (!v.ev_pool.empty()) {
        hipEvent_t e = v.ev_pool.back();
        v.ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    return e;
}

// The slowest rate a session's published work is assumed to render at, samples per ms
// (100 M samples/s: config 5, the slowest config, renders 7.5 G/s): a session may take
// its timeout plus its published samples at this rate to end.  A whole 16 GiB ring of
// sample words queued on a slow scene is real work, not a hang.
constexpr double kSvcMinRate = 1e5;

// Wait for event e at most the service's timeout plus the time the running session's
// published work may take (kSvcMinRate): SPT_OK, or SPT_ERR_TIMEOUT.  Spins (yielding)
// for the first 2 ms, then polls every 50 us.
int svc_wait(spt_ctx *ctx, hipEvent_t e, const char *what)
{
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = ctx->svc.timeout_ms + (double)ctx->svc.session_items / kSvcMinRate;
    for (;;) {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return SPT_OK;
        if (q != hipErrorNotReady) return fail(ctx, SPT_ERR_HIP, "%s: %s", what, hipGetErrorString(q));
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms > limit) {
            const Service &v = ctx->svc;
            const uint32_t closing = __atomic_load_n(v.h_host + spt::kSvcHostClosing, __ATOMIC_SEQ_CST);
            return fail(ctx, SPT_ERR_TIMEOUT,
                        "render service: %s did not finish within %.0f ms (session %llu: %u jobs published, "
                        "%llu claims, %llu samples; closing flag %u)",
                        what, limit, (unsigned long long)v.sessions, v.n_jobs, (unsigned long long)v.claims,
                        (unsigned long long)v.session_items, closing);
        }
        if (ms < 2.0)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// End the session: the stop flag after every publication (host memory: the forwarder
// passes it on after the last record), then wait (bounded) for the kernel to drain the
// jobs and leave.  No-op without a session.
int svc_end(spt_ctx *ctx)
{
    Service &v = ctx->svc;
    if (v.draining) {
        // an earlier end timed out: the session is over only once its kernel has left
        if (int rc = svc_wait(ctx, v.ev_end, "ending the session (after an earlier timeout)")) return rc;
    } else {
        if (!v.running) return SPT_OK;
        v.running = false;
        v.draining = true;
        SVC_DBG(ctx, "end session %llu (%u jobs): stop", (unsigned long long)v.sessions, v.n_jobs);
        __atomic_store_n(v.h_host + spt::kSvcHostStop, 1u, __ATOMIC_SEQ_CST);
        if (int rc = svc_wait(ctx, v.ev_end, "ending the session")) return rc;
    }
    v.draining = false;
    SVC_DBG(ctx, "end session %llu: kernel done", (unsigned long long)v.sessions);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, v.ev_start, v.ev_end) == hipSuccess) v.kernel_ms += ms;
    // read from host memory: no device call here (a synchronous copy would queue behind
    // whatever else the device is running)
    const uint32_t wd = __atomic_load_n(v.h_host + spt::kSvcHostWatchdog, __ATOMIC_SEQ_CST);
    if (wd) v.watchdog_exits++;
    SVC_DBG(ctx, "end session %llu: watchdog %u", (unsigned long long)v.sessions, wd);
    if (v.d_trace) {
        // per counter used this session: first / last claim taken, last count, in us
        // from the session's first claim (s_memrealtime: 100 MHz)
        std::vector<unsigned long long> tr((size_t)v.done_cap * 4 + spt::kSvcTraceClaims);
        HIP_TRY(ctx, hipMemcpy(tr.data(), v.d_trace, tr.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (uint32_t i = 0; i < v.done_cap; ++i) t0 = std::min(t0, tr[4 * i]);
        for (uint32_t i = 0; i < v.done_cap; ++i)
            if (tr[4 * i] != ~0ull)
                std::fprintf(stderr, "svc trace idx %u: claims %.1f .. %.1f us, last count %.1f us\n", i,
                             (tr[4 * i] - t0) / 100.0, (tr[4 * i + 1] - t0) / 100.0, (tr[4 * i + 2] - t0) / 100.0);
        if (const char *path = env_var("SPT_SVC_TRACE_FILE")) {
            // the per-claim take times (block << 40 | 40-bit time), raw
            if (FILE *f = std::fopen(path, "wb")) {
                std::fwrite(&t0, sizeof t0, 1, f);
                std::fwrite(tr.data() + (size_t)v.done_cap * 4, sizeof(unsigned long long), spt::kSvcTraceClaims, f);
                std::fclose(f);
            }
        }
    }
    return SPT_OK;
}

// Page-locked, fine-grained (coherent) host memory: the host's stores and the device's
// system-scope accesses reach the same bytes.  Host and device views.
template <class T>
int host_shared(spt_ctx *ctx, size_t count, T **host, T **dev)
{
    void *p = nullptr, *d = nullptr;
    HIP_TRY(ctx, hipHostMalloc(&p, count * sizeof(T), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(p, 0, count * sizeof(T));
    HIP_TRY(ctx, hipHostGetDevicePointer(&d, p, 0));
    *host = (T *)p;
    *dev = (T *)d;
    return SPT_OK;
}

// Start a session for `mode` (the session's kernel arguments hold the scene, camera,
// frame and mode of the context as they are now; the setters end the session).  The
// session's kernel waits for `waits` (folds whose ring words or counters its first
// publication reuses); reset_idx (or -1): a completion counter zeroed before it, with
// the caller's stream s ordered after that.
int svc_begin(spt_ctx *ctx, int mode, const std::vector<hipEvent_t> &waits, int64_t reset_idx, hipStream_t s)
{
    Service &v = ctx->svc;
    if (!v.h_host) {
        int rc = host_shared(ctx, spt::kSvcHostWords, &v.h_host, &v.d_host);
        if (!rc) rc = host_shared(ctx, v.job_cap, &v.h_jobs, &v.dh_jobs);
        if (!rc) rc = host_shared(ctx, v.job_cap, &v.h_job_claim, &v.dh_job_claim);
        if (rc) return rc;
    }
    if (!v.stream) {
        // The resident kernel never ends while the session runs, so nothing may queue
        // behind it: HIP maps a process's streams of one priority round-robin onto
        // GPU_MAX_HW_QUEUES hardware queues (4 on the box), and a stream sharing the
        // kernel's queue would wait for the session's end.  A stream of another priority
        // gets a queue of its own (tools/ubench/queue_probe T6/T7,
        // profiles/queue_probe_r04.txt); SPT_SVC_PRIO picks it (default: the greatest).
        int lo = 0, hi = 0;
        HIP_TRY(ctx, hipDeviceGetStreamPriorityRange(&lo, &hi));
        int prio = hi;
        if (const char *e = env_var("SPT_SVC_PRIO")) prio = std::atoi(e);
        HIP_TRY(ctx, hipStreamCreateWithPriority(&v.stream, hipStreamNonBlocking, prio));
        HIP_TRY(ctx, hipEventCreate(&v.ev_start));
        HIP_TRY(ctx, hipEventCreate(&v.ev_end));
        HIP_TRY(ctx, hipEventCreateWithFlags(&v.ev_ctl, hipEventDisableTiming));
        if (!v.ring_set) {
            // default ring: 1/16 of the device's memory within [4, 16] GiB (MI355X: 16 GiB = 44
            // config-2 frames of sample words).  A publication that would overwrite words whose
            // fold has not run ends the session (flow control above), so the ring bounds how
            // far a caller may run ahead without a restart: 4 GiB held 10 such frames, and a
            // 20-frame bench restarted its session once (14.0 vs 10.7 ms to the 11th frame)
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot > 0)
                v.ring_bytes = std::min<uint64_t>(16ull << 30, std::max<uint64_t>(4ull << 30, (uint64_t)tot / 16 >> 20 << 20));
        }
        v.ring_words = v.ring_bytes / sizeof(uint32_t) / 2 * 2;
        const bool ok = hipMalloc((void **)&v.d_ctl, spt::kSvcCtlWords * sizeof(uint32_t)) == hipSuccess &&
                        hipMalloc((void **)&v.d_jobs, (size_t)v.job_cap * sizeof(spt::SvcJob)) == hipSuccess &&
                        hipMalloc((void **)&v.d_job_claim, (size_t)v.job_cap * sizeof(uint32_t)) == hipSuccess &&
                        hipMalloc((void **)&v.d_done, (size_t)v.done_cap * sizeof(uint32_t)) == hipSuccess &&
                        hipMalloc((void **)&v.d_ring, (size_t)v.ring_words * sizeof(uint32_t)) == hipSuccess;
        if (!ok) return fail(ctx, SPT_ERR_NOMEM, "render service buffers (%llu MiB ring) allocation failed",
                             (unsigned long long)(v.ring_bytes >> 20));
        HIP_TRY(ctx, hipMemsetAsync(v.d_done, 0, (size_t)v.done_cap * sizeof(uint32_t), v.stream));
    }
    const uint32_t grid = svc_session_grid(ctx);
    spt::RenderArgs ra{};
    ra.scene = device_scene(ctx);
    ra.prim = ctx->prim;
    ra.cam = ctx->cam;
    ra.width = ctx->W;
    ra.height = ctx->H;
    ra.bounces = ctx->bounces;
    ra.mode = (uint32_t)mode;
    ra.seed_key = fmix64(ctx->seed);
    ra.samples = v.d_ring;
    ra.slot_words = mode == SPT_MODE_SEGMENT ? 1u : 2u;
    ra.claim = v.claim;
    ra.n_queues = v.queues;
    ra.counters = ctx->d_counters;
    ra.svc_ctl = v.d_ctl;
    ra.svc_jobs = v.d_jobs;
    ra.svc_job_claim = v.d_job_claim;
    ra.svc_done = v.d_done;
    ra.svc_host = v.d_host;
    ra.svc_host_jobs = v.dh_jobs;
    ra.svc_host_job_claim = v.dh_job_claim;
    if (env_var("SPT_SVC_TRACE")) {
        const size_t n = (size_t)v.done_cap * 4 + spt::kSvcTraceClaims;
        if (!v.d_trace) HIP_TRY(ctx, hipMalloc((void **)&v.d_trace, n * sizeof(unsigned long long)));
        std::vector<unsigned long long> init(n, 0ull);
        for (size_t i = 0; i < (size_t)v.done_cap * 4; i += 4) init[i] = ~0ull;
        HIP_TRY(ctx, hipMemcpy(v.d_trace, init.data(), n * sizeof(unsigned long long), hipMemcpyHostToDevice));
        ra.svc_trace = v.d_trace;
    }
    // the previous session's kernel has ended (svc_end), so no wave reads the host words
    // while they are reset; the kernel launch below orders these stores before it
    __atomic_store_n(v.h_host + spt::kSvcHostCommitted, 0u, __ATOMIC_SEQ_CST);
    __atomic_store_n(v.h_host + spt::kSvcHostClosing, 0u, __ATOMIC_SEQ_CST);
    __atomic_store_n((uint64_t *)(v.h_host + spt::kSvcHostPub), (uint64_t)0, __ATOMIC_SEQ_CST);
    __atomic_store_n(v.h_host + spt::kSvcHostStop, 0u, __ATOMIC_SEQ_CST);
    __atomic_store_n(v.h_host + spt::kSvcHostWatchdog, 0u, __ATOMIC_SEQ_CST);
    for (hipEvent_t e : waits) HIP_TRY(ctx, hipStreamWaitEvent(v.stream, e, 0));
    // control words zeroed, the render-wave count set (every wave but the forwarder), before
    // the kernel
    HIP_TRY(ctx, hipMemsetAsync(v.d_ctl, 0, spt::kSvcCtlWords * sizeof(uint32_t), v.stream));
    const uint32_t bw = spt::svc_block(ctx->accel) / 64u;  // waves per block of the session kernel
    const uint32_t render_waves = grid * bw - 1u;
    HIP_TRY(ctx, hipMemsetD32Async((hipDeviceptr_t)(v.d_ctl + spt::kSvcLive), (int)render_waves, 1, v.stream));
    if (reset_idx >= 0) {
        // a completion counter whose running total restarts: zeroed after the folds that
        // waited on it (waits), and the caller's stream ordered after the zeroing
        HIP_TRY(ctx, hipMemsetAsync(v.d_done + reset_idx, 0, sizeof(uint32_t), v.stream));
        HIP_TRY(ctx, hipEventRecord(v.ev_ctl, v.stream));
        HIP_TRY(ctx, hipStreamWaitEvent(s, v.ev_ctl, 0));
    }
    HIP_TRY(ctx, hipEventRecord(v.ev_start, v.stream));
    HIP_TRY(ctx, spt::launch_render_svc(ra, grid, v.stream));
    HIP_TRY(ctx, hipEventRecord(v.ev_end, v.stream));
    v.running = true;
    v.mode = mode;
    v.n_jobs = 0;
    v.claims = 0;
    v.session_items = 0;
    v.sessions++;
    SVC_DBG(ctx, "begin session %llu, grid %u, %zu waits", (unsigned long long)v.sessions, grid, waits.size());
    return SPT_OK;
}

// Blocks of a session over the context's scene: the wave-walk kernel's svc_grid, or the
// LDS-tree kernel's (1 024-thread blocks: every slot with SPT_SVC_FULL_GRID, else one per
// CU fewer, so that folds and other kernels find room), divided by SPT_SVC_GRID_DIV
uint32_t svc_session_grid(const spt_ctx *ctx)
{
    const uint32_t g = spt::svc_lds(ctx->accel) ? spt::svc_lds_grid(ctx->svc_full) : ctx->svc_grid;
    return std::max<uint32_t>(1u, g / ctx->svc.grid_div);
}

// Can render_impl hand a launch of `words` sample words to the service?
bool svc_eligible(const spt_ctx *ctx, uint64_t words, bool keep_samples)
{
    const Service &v = ctx->svc;
    return v.enabled && !keep_samples && ctx->engine == SPT_ENGINE_MEGAKERNEL && spt::svc_supported(ctx->accel) &&
           (v.lds || !spt::svc_lds(ctx->accel)) && words <= v.ring_bytes / sizeof(uint32_t) / 2;
}

// Publish jobs sharing one completion counter (a render_impl batch: one job; a batched
// drop-in launch: one job per call) whose slots take total_slots consecutive ring slots,
// and make stream s wait for all their samples.  Out: the ring word of the publication's
// first slot and its counter (svc_retire after the folds).
int svc_submit_jobs(spt_ctx *ctx, int mode, const SvcJobSpec *jobs, size_t n, uint64_t total_slots, hipStream_t s,
                    uint64_t *w0_out, uint32_t *idx_out)
{
    Service &v = ctx->svc;
    const uint32_t slot_words = mode == SPT_MODE_SEGMENT ? 1u : 2u;
    uint64_t items = 0, nclaims = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t it = (uint64_t)spt::rows_owned(jobs[i].map) * jobs[i].map.width * jobs[i].spp_batch;
        items += it;
        nclaims += (it + v.claim - 1) / v.claim;
    }
    if (items > 0xFFFFFFFFull) return fail(ctx, SPT_ERR_ARG, "render service: %llu samples in one publication",
                                           (unsigned long long)items);
    if (n > v.job_cap) return fail(ctx, SPT_ERR_ARG, "render service: %zu jobs in one publication", n);
    const uint64_t words = total_slots * slot_words;
    // the publication's ring words and completion counter
    const uint64_t w0 = v.ring_head + words > v.ring_words ? 0 : v.ring_head, w1 = w0 + words;
    const uint32_t idx = v.next_done;
    if (v.done_cum.empty()) v.done_cum.assign(v.done_cap, 0);  // counters zeroed with their allocation
    uint64_t target = v.done_cum[idx] + items;
    const bool reset = target > 0xFFFFFFFFull;
    // Flow control: earlier jobs whose folds still read these ring words or still wait on
    // this counter (or the oldest, with 1024 jobs in flight) must be folded first.  Folds
    // found finished are retired; an unfinished one is never waited for inside the running
    // session -- a fold can sit behind work that itself waits for the session to end (an
    // RCCL gather cannot become resident beside it) -- so the session is ended
    // and the next one's kernel waits for those folds instead.
    std::vector<hipEvent_t> waits;
    for (size_t i = 0; i < v.inflight.size();) {
        SvcInflight &e = v.inflight[i];
        const bool busy = (e.w0 < w1 && w0 < e.w1) || e.done_idx == idx || (i == 0 && v.inflight.size() >= 1024);
        if (!busy) {
            ++i;
            continue;
        }
        const hipError_t q = hipEventQuery(e.ev);
        if (q != hipSuccess && q != hipErrorNotReady) return fail(ctx, SPT_ERR_HIP, "fold event: %s", hipGetErrorString(q));
        if (q == hipErrorNotReady) waits.push_back(e.ev);
        else v.ev_pool.push_back(e.ev);
        v.inflight.erase(v.inflight.begin() + (std::ptrdiff_t)i);
    }
    // a new session: none yet, another mode, a kernel that left already, the session's job
    // table / claim range full, folds to wait for, or a counter to zero
    bool fresh = !v.running || v.mode != mode || hipEventQuery(v.ev_end) != hipErrorNotReady ||
                 v.n_jobs + n > v.job_cap || (v.claims + nclaims) * v.claim > 0x7FFFFFFFull || !waits.empty() || reset;
    if (!fresh) {
        // commit the jobs to the running session, then look for a raised closing flag
        // (store, full fence, load: the host half of the handshake)
        __atomic_store_n(v.h_host + spt::kSvcHostCommitted, v.n_jobs + (uint32_t)n, __ATOMIC_SEQ_CST);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        if (__atomic_load_n(v.h_host + spt::kSvcHostClosing, __ATOMIC_SEQ_CST) != 0u) {
            fresh = true;
            v.closing_restarts++;
        }
    } else if (!waits.empty() && v.running) {
        v.flow_restarts++;
    }
    SVC_DBG(ctx, "submit %zu job(s), words [%llu, %llu), counter %u: %zu waits, fresh %d", n, (unsigned long long)w0,
            (unsigned long long)w1, idx, waits.size(), (int)fresh);
    if (fresh) {
        int rc = svc_end(ctx);
        if (!rc) rc = svc_begin(ctx, mode, waits, reset ? (int64_t)idx : -1, s);
        for (hipEvent_t e : waits) v.ev_pool.push_back(e);  // the waits are enqueued (or abandoned)
        if (rc) return rc;
        __atomic_store_n(v.h_host + spt::kSvcHostCommitted, (uint32_t)n, __ATOMIC_SEQ_CST);
    }
    v.ring_head = w1;
    v.session_items += items;
    v.next_done = (v.next_done + 1u) % v.done_cap;
    if (reset) target = items;
    v.done_cum[idx] = target;
    // SPT_SVC_TEST_PUB_DELAY_US (fault injection): committed, not yet published
    if (v.pub_delay_us) std::this_thread::sleep_for(std::chrono::microseconds(v.pub_delay_us));
    // the records and first claims (host tables, the forwarder copies them), then the pair
    for (size_t k = 0; k < n; ++k) {
        const SvcJobSpec &js = jobs[k];
        const uint64_t it = (uint64_t)spt::rows_owned(js.map) * js.map.width * js.spp_batch;
        const uint64_t nc = (it + v.claim - 1) / v.claim;
        spt::SvcJob j{};
        j.item_off = (uint32_t)(v.claims * v.claim);
        j.item_end = (uint32_t)(j.item_off + it);
        j.slot_off = (uint32_t)(w0 / slot_words + js.slot_local);
        j.done_idx = idx;
        j.rows = js.rows;
        j.spp_batch = js.spp_batch;
        j.s0 = js.s0;
        j.claim_end = (uint32_t)(v.claims + nc);
        j.map = js.map;
        j.div_band = js.div_band;
        j.div_tile = js.div_tile;
        j.div_strip = js.div_strip;
        j.claim_first = (uint32_t)v.claims;
        std::memcpy(&v.h_jobs[v.n_jobs], &j, sizeof j);
        v.h_job_claim[v.n_jobs] = j.claim_first;
        v.claims += nc;
        v.n_jobs++;
        v.jobs++;
    }
    // x86 keeps stores in order: the device sees the pair only after the records it covers
    __atomic_store_n((uint64_t *)(v.h_host + spt::kSvcHostPub), (uint64_t)(uint32_t)v.claims | ((uint64_t)v.n_jobs << 32),
                     __ATOMIC_RELEASE);
    // the caller's stream waits for the job's samples
    HIP_TRY(ctx, hipStreamWaitValue32(s, v.d_done + idx, (uint32_t)target, hipStreamWaitValueGte, 0xFFFFFFFFu));
    SVC_DBG(ctx, "submitted, %u jobs in session", v.n_jobs);
    *w0_out = w0;
    *idx_out = idx;
    return SPT_OK;
}

// One render_impl launch (`ra`: map, npix, spp_batch, s0, divisors) as one job.
int svc_submit(spt_ctx *ctx, const spt::RenderArgs &ra, int mode, hipStream_t s, uint64_t *w0_out, uint32_t *idx_out)
{
    SvcJobSpec js{ra.map, ra.npix / ra.map.width, ra.spp_batch, ra.s0, ra.div_band, ra.div_tile, ra.div_strip, 0};
    return svc_submit_jobs(ctx, mode, &js, 1, (uint64_t)ra.n_items, s, w0_out, idx_out);
}

// After the job's fold was enqueued on s: its ring words and counter are free once the
// fold has run.
int svc_retire(spt_ctx *ctx, hipStream_t s, uint64_t w0, uint64_t words, uint32_t idx)
{
    hipEvent_t e = svc_event(ctx);
    if (!e) return fail(ctx, SPT_ERR_HIP, "event creation failed");
    HIP_TRY(ctx, hipEventRecord(e, s));
    ctx->svc.inflight.push_back(SvcInflight{w0, w0 + words, idx, e});
    return SPT_OK;
}

}  // namespace spt_api

extern "C" {

int spt_service_start(spt_ctx *ctx)
{
    return for_members(ctx, [](spt_ctx *c) {
        std::lock_guard<std::mutex> lk(c->mu);
        c->svc.enabled = true;
        return SPT_OK;
    });
}

int spt_service_set_full_grid(spt_ctx *ctx, uint32_t full)
{
    return for_members(ctx, [full](spt_ctx *c) -> int {
        std::lock_guard<std::mutex> lk(c->mu);
        if (c->svc.running || c->svc.draining)
            return fail(c, SPT_ERR_STATE, "a render-service session is running (spt_service_stop first)");
        c->svc_full = full != 0;
        c->svc_grid = (uint32_t)((full ? c->svc_per_cu : std::max(1, c->svc_per_cu - 1)) * c->num_cu);
        return SPT_OK;
    });
}

int spt_service_stop(spt_ctx *ctx)
{
    return for_members(ctx, [](spt_ctx *c) {
        std::lock_guard<std::mutex> lk(c->mu);
        HIP_TRY(c, hipSetDevice(c->device));
        c->svc.enabled = false;
        return svc_end(c);
    });
}

}  // extern "C"
