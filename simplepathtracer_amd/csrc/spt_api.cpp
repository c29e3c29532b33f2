// spt_api.cpp -- C ABI (include/spt_hip.h) over the gfx950 render kernels.
//
// Owns the device copy of the reference's global state (scene SoA, camera,
// config: Globals.hpp:8-37), the per-sample workspace and the launch geometry
// of the persistent render kernel, and rebuilds the two reference entry points
// RenderSegment (SingleThreadPathTracer.hpp:114-137) and RenderSegmentTask
// (TaskBasedPathTracer.hpp:54-206) as render + fold launches.
#include "spt_hip.h"
#include "spt_accel.h"
#include "spt_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <string>
#include <utility>
#include <vector>

namespace {
// An environment variable's value, or null when unset or empty (a variable set to ""
// reads as unset: SPT_BLOCKS_PER_CU= would otherwise mean a 1-block grid)
const char *env_var(const char *name)
{
    const char *e = std::getenv(name);
    return e && *e ? e : nullptr;
}
}  // namespace

namespace {

thread_local std::string g_thread_error;
// the context whose progress callback is running on this thread (spt_render_progressive)
thread_local const spt_ctx *t_in_callback = nullptr;

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
};

}  // namespace

namespace {
// caller streams (spt_render_rows_async) + the host-call slots below
constexpr size_t kMaxCallerStreams = 4;
constexpr size_t kCounters = 4 + SPT_DIAG_WORDS;  // device counters: casts, samples, dropped, -, diag[]
constexpr size_t kMaxHostSlots = 8;
constexpr uint32_t kMaxBatchSets = 8;  // batches of host calls in flight (BatchSet below)
// + one companion stream per caller stream / host slot for double-buffered sample
// batches (render_impl)
constexpr size_t kMaxCompanions = kMaxCallerStreams + kMaxHostSlots;
constexpr size_t kMaxWorkspaces = kMaxCallerStreams + kMaxHostSlots + kMaxBatchSets + 1 + kMaxCompanions + 4;  // + read-ahead parts (SpecFrame::kParts)
// One in-flight unbatched host call (spt_render_progressive, or any call with
// SPT_BATCH=0 or too large for one batch): its own stream (hence its own workspace) and
// output staging, so such calls run on the GPU together instead of one after another.
struct HostSlot {
    hipStream_t stream = nullptr;
    float4 *d_stage = nullptr;  // region-local float4 output
    size_t stage_cap = 0;
    bool busy = false;
};
// Batched host calls: concurrent spt_render_segment[_task] calls are rendered together,
// one render + one fold launch per batch over a table of rectangles (BatchRect), so
// the reference's RenderJob threads (Renderer.hpp:242-302) -- 16 tiles a frame at the
// shipped g_maxThreads = 4, 1 024 at tc = 2 * 16 cores -- do not each pay a launch,
// its fold, its tail and its own synchronisation.  Two batch sets by default
// (SPT_BATCH_SETS): while one batch renders, the calls arriving meanwhile form the next.
struct BatchSet {
    hipStream_t stream = nullptr;
    spt::BatchRect *d_rects = nullptr, *h_rects = nullptr;  // device table, pinned host copy
    size_t rects_cap = 0, h_rects_cap = 0;
    float4 *d_stage = nullptr;  // float4 outputs of the batch's rectangles, concatenated
    size_t stage_cap = 0;
    bool busy = false;
};
struct BatchReq {
    int mode;
    uint32_t yB, yE, xB, xE;
    float *rgba;
    uint8_t *g_data;
    int rc;
    bool launched, done;
};
// Read-ahead of the reference's tiling (render_segment_host, DESIGN.md §5 "Drop-in
// read-ahead"): RenderImageParallelMain (Renderer.hpp:257-302) calls RenderSegment on the
// tc x tc tiles of MakeRenderSegmentData, at most tc at a time, from detached threads (so
// in no fixed order).  Once a caller has called every tile of such a tiling (the tiling is
// "armed": a caller rendering one tile alone never arms it), the first call of a tile of it
// renders every tile of the frame at once in `parts` batched launches of consecutive tile
// rows (SPT_READAHEAD_PARTS, default 4) into a device copy of g_data; each tile's call then
// waits for its part and copies its own rows to the caller's g_data.  Every tile is still
// rendered once per frame; nothing is written to the caller's buffer before its call.
struct SpecFrame {
    bool active = false;
    int mode = 0;
    uint32_t tc = 0, sw = 0, sh = 0;
    uint64_t gen = 0;            // spt_ctx::gen when launched
    std::vector<uint8_t> served; // per tile (row-major over tile rows j, columns i)
    static constexpr int kParts = 4;
    uint32_t parts = 4, rows_per_part = 1;  // tile rows per launch
    hipEvent_t ev[kParts] = {};
    bool launched[kParts] = {};
    BatchSet bs[kParts];
    uint8_t *d8 = nullptr;  // the frame's RGB8 bytes (g_data layout), device
    size_t d8_cap = 0;
    // serves copying out of d8 with the context unlocked: the next read-ahead neither
    // rewrites nor reallocates d8 before they are done (readers_cv, ctx->mu)
    uint32_t readers = 0;
    std::condition_variable readers_cv;
    // arming: the tiles of one tiling (mode, tc, frame size) called so far by plain calls
    int arm_mode = -1;
    uint32_t arm_tc = 0, arm_w = 0, arm_h = 0, arm_count = 0;
    std::vector<uint8_t> arm_seen;
    bool armed = false;
};

struct Workspace {
    hipStream_t stream = nullptr;  // key
    uint32_t *d_samples = nullptr; // per-sample slots of the current batch (sample words)
    size_t samples_cap = 0;
    float4 *d_acc = nullptr;       // ordered partial sums when a frame is batched
    size_t acc_cap = 0;
    uint32_t *d_head = nullptr;    // claim counter
    bool head_clean = false;       // d_head zeroed by the last batched fold (launch_batch)
    spt::WavefrontBuffers wf{};    // queues of the wavefront engine (allocated on first use)
};

// The render service: one resident launch of render_kernel_svc per session
// renders the jobs published to it -- every render of render_impl while the service is on
// (frames, rank shares, sample batches, host-slot calls) -- so consecutive jobs follow each
// other without a launch ramp and tail between them.  A job's sample words live in a ring
// in HBM; its fold waits (hipStreamWaitValue32) on its completion counter.
struct SvcInflight {
    uint64_t w0, w1;    // ring words of its slots
    uint32_t done_idx;  // its completion counter
    hipEvent_t ev;      // recorded after its fold
};
struct Service {
    bool enabled = false;  // spt_service_start: renders go through the service
    bool running = false;  // a session's kernel is resident
    hipStream_t stream = nullptr;  // the session kernel
    uint32_t *d_ctl = nullptr;
    spt::SvcJob *d_jobs = nullptr;
    uint32_t *d_job_claim = nullptr, *d_done = nullptr, *d_ring = nullptr;
    uint64_t ring_words = 0;
    uint64_t ring_bytes = 4ull << 30;  // SPT_SVC_RING_MB, else sized at the first session (svc_start)
    bool ring_set = false;             // SPT_SVC_RING_MB given
    uint32_t job_cap = 1u << 16, done_cap = 4096;
    uint32_t claim = 448, queues = spt::kMaxQueues;  // SPT_SVC_CLAIM, SPT_SVC_QUEUES
    // session
    int mode = 0;
    uint32_t n_jobs = 0;
    uint64_t claims = 0;  // published
    uint64_t ring_head = 0;
    uint32_t next_done = 0;
    // completion counters only grow (zeroed once at allocation): a job waits for its
    // counter to reach the host's running total of the counter's samples, so no wait can
    // see a count left over from an earlier job (a zeroing launch on the publish stream
    // is not ordered before the caller's wait); a total that would pass 2^32 restarts at
    // zero, with the caller's stream ordered after that publish
    std::vector<uint64_t> done_cum;
    std::vector<SvcInflight> inflight;
    std::vector<hipEvent_t> ev_pool;
    hipEvent_t ev_start = nullptr, ev_end = nullptr, ev_ctl = nullptr;
    // the session's closing-handshake words (spt_internal.h kSvcIdleTicks), page-locked
    // host memory: host view and device view
    uint32_t *h_host = nullptr, *d_host = nullptr;
    // the host job tables the forwarder copies from (same memory kind): host / device views
    spt::SvcJob *h_jobs = nullptr, *dh_jobs = nullptr;
    uint32_t *h_job_claim = nullptr, *dh_job_claim = nullptr;
    uint32_t grid_div = 1;       // SPT_SVC_GRID_DIV: the session takes 1/div of its grid
    uint32_t pub_delay_us = 0;   // SPT_SVC_TEST_PUB_DELAY_US: fault injection before every publish
    // SPT_SVC_TIMEOUT_MS: the longest wait for a session to end beyond the time its
    // published work may take at kSvcMinRate (svc_wait)
    double timeout_ms = 30000;
    uint64_t session_items = 0;  // samples published to the running session
    // a session whose end timed out: its kernel may still be resident, so no new session
    // starts (and no host word is reset) until its end event completes (svc_end)
    bool draining = false;
    bool debug = false;          // SPT_SVC_DEBUG: a line on stderr per session event
    uint64_t sessions = 0, jobs = 0, watchdog_exits = 0;
    // sessions ended early: a publication would have waited for an unfinished fold (flow
    // control), or a wave of the session had raised the closing flag
    uint64_t flow_restarts = 0, closing_restarts = 0;
    double kernel_ms = 0;  // summed session spans
    unsigned long long *d_trace = nullptr;  // SPT_SVC_TRACE: printed by svc_end
};
}  // namespace

struct spt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::string err;
    int num_cu = 0;
    uint32_t grid = 0, block = spt::kRenderBlock, claim = 0;  // 0 = per launch (claim_size)
    uint32_t claims_per_wave = 2;                              // render_grid (config 1: 2 > 1, 4)
    uint32_t queues = spt::kMaxQueues;                         // claim counters (RenderArgs::n_queues)
    uint32_t grid_overlap = 0;  // grid while frames are in flight on several streams
    uint32_t grid_small = 0;    // grid_overlap for small launches (render_grid), 0 = none
    // the render service's grid: the occupancy's blocks per CU minus one, always (its
    // folds, publish launches and other streams' kernels need the free slot)
    uint32_t svc_grid = 0;
    uint32_t last_grid = 0, last_block = 0;  // shape of the most recent render launch

    // scene (Globals.hpp:31-37)
    float4 *d_shade = nullptr, *d_slots = nullptr;
    spt::AccelNode *d_nodes = nullptr;
    uint32_t *d_mat = nullptr, *d_orig = nullptr;
    float *d_kpre = nullptr;
    size_t shade_cap = 0, mat_cap = 0, slots_cap = 0, orig_cap = 0, nodes_cap = 0, kpre_cap = 0;
    spt::AccelTables tables;
    uint32_t n = 0;
    // primary-ray candidate lists (spt_internal.h PrimLists), rebuilt by the setters once
    // scene, camera and frame are set; SPT_PRIM_LISTS=0 turns them off, SPT_PRIM_MAX caps a
    // block's list (longer ones walk the tree)
    bool prim_enabled = true;
    uint32_t prim_max = 24;
    spt::PrimLists prim{};
    uint2 *d_prim_b8 = nullptr, *d_prim_b4 = nullptr;
    uint32_t *d_prim_slots = nullptr;
    size_t prim_b8_cap = 0, prim_b4_cap = 0, prim_slots_cap = 0;
    double prim_build_s = 0;  // host time of the last build
    uint64_t prim_builds = 0;
    double accel_build_s = 0;  // host time of the last rebuild_accel (build, check, upload)
    // what the lists were built for (rebuild_prim skips a rebuild when nothing the lists
    // depend on changed: spp, depth and seed setters do not touch them)
    struct PrimKey {
        float view[12], eye[3];
        uint32_t W, H, prim_max;
        uint64_t accel_gen;
        bool valid;
        bool same(const PrimKey &o) const
        {
            return valid && o.valid && std::memcmp(view, o.view, sizeof view) == 0 &&
                   std::memcmp(eye, o.eye, sizeof eye) == 0 && W == o.W && H == o.H && prim_max == o.prim_max &&
                   accel_gen == o.accel_gen;
        }
    } prim_key{};
    uint64_t accel_gen = 0;  // rebuild_accel count
    uint32_t prim_blocks = 0, prim_entries = 0;  // 8x8 blocks with a list, list entries
    // diffuse sample codes (spt_internal.h diffuse_code): the slot count, and the halvings
    // after which every finite albedo of the scene is 0 (j saturates at min(bounces - 1, jz))
    uint32_t code_stride = 1, code_jz = 0;
    bool scene_set = false;
    // host copy of the hit geometry, to rebuild the traversal tables
    std::vector<float> h_centers, h_radii;
    std::vector<float4> h_shade;  // {r, g, b, fuzz} per sphere
    std::vector<uint32_t> h_mat;
    uint32_t cluster_k = SPT_CLUSTER_AUTO;  // members per culling cluster; 0 = brute force
    uint32_t tree_branching = SPT_TREE_AUTO;  // children per inner node; 0 = flat cluster list
    int engine = SPT_ENGINE_MEGAKERNEL;
    uint32_t wf_cap = 1u << 24;  // rays in the wavefront engine's block queues (at most)
    uint32_t wf_queue = 4096;    // rays per block queue (a multiple of 256)
    spt::AccelView accel{};
    // camera (Globals.hpp:21-29)
    spt::Camera cam{};
    bool cam_set = false;
    // config (Globals.hpp:12-15)
    uint32_t W = 0, H = 0, spp = 0, bounces = 0;
    uint64_t seed = 0;
    bool params_set = false;

    // workspace
    uint64_t ws_bytes = 16ull << 30;  // of 288 GB HBM: config 5 in one launch, config 3 in 6
    // one workspace per stream, so renders on different streams can be in flight
    // together (the next frame's blocks fill the GPU while the last paths of the
    // previous one drain)
    std::vector<Workspace> ws;  // reserved to kMaxWorkspaces: pointers into it stay valid
    // frames of several sample batches: batch j renders on the caller's stream (j even)
    // or its companion (j odd), each with its own workspace, so one batch renders while
    // the other's samples are folded (render_impl); SPT_BATCH_DBUF=0 turns it off
    bool batch_dbuf = true;
    std::vector<std::pair<hipStream_t, hipStream_t>> companions;  // (caller stream, companion)
    // spt_set_reserved_cus: launched renders run on CU-masked streams of the context
    // (masked_for), one per caller stream, with the two events that order them
    uint32_t reserve_cus = 0;
    struct Masked {
        hipStream_t caller, stream;
        hipEvent_t go, done;
    };
    std::vector<Masked> masked;
    hipEvent_t dbuf_start = nullptr, dbuf_fold = nullptr;
    unsigned long long *d_counters = nullptr;
    uint8_t *d_frame8 = nullptr;
    size_t frame8_cap = 0;

    // host buffers registered by spt_pin_host, with their device-side addresses
    struct Pinned {
        void *ptr;
        size_t bytes;
        uint8_t *dev;  // the buffer as this member's device sees it
        bool owner;    // registered by this context (member 0 of a multi-device context)
    };
    std::vector<Pinned> pinned;
    // serialises spt_pin_host / spt_unpin_host as a whole: they drop ctx->mu while they
    // visit the member devices, and a concurrent pair must not both find and erase an entry
    std::mutex pin_mu;

    // host-call slots (render_segment_host), created on demand up to host_slots
    std::vector<HostSlot *> slots;
    std::condition_variable slot_cv;
    uint32_t host_slots = kMaxHostSlots;
    uint32_t host_grid_div = 0;  // 0: half the slots in use (SPT_HOST_GRID_DIV overrides)
    std::atomic<int> inflight{0};  // host calls in progress on this device
    // batched host calls (render_batched); SPT_BATCH=0 renders every call on its own
    bool batching = true;
    std::vector<BatchReq *> batch_pending;
    bool batch_leader = false;  // a caller is assembling the next batch
    BatchSet bsets[kMaxBatchSets];
    uint32_t batch_sets = 2;  // batches in flight at once (SPT_BATCH_SETS)
    // tiling read-ahead (SpecFrame; SPT_READAHEAD=0 turns it off); gen counts the setters
    bool readahead = true;
    SpecFrame spec;
    uint64_t gen = 0;
    // each batch launch takes 1/div of the grid (SPT_BATCH_GRID_DIV): two batches in flight
    // then run side by side and each one's tail drains beside the other's blocks (config 2
    // through the C++ shim at tc = 4: 7.93 -> 7.64 ms per frame, its folds 2x shorter)
    uint32_t batch_grid_div = 2;
    std::condition_variable batch_cv;
    uint64_t batches = 0, batched_calls = 0;

    // multi-device context (spt_ctx_create_multi): member contexts of the other devices,
    // each with its own scene copy; this context is member 0
    std::vector<spt_ctx *> peers;
    float4 *d_tile = nullptr;  // spt_render_frame: this member's strips (member 0: all members' strips)
    size_t tile_cap = 0;
    float4 *d_fullframe = nullptr;  // spt_render_frame: assembled float4 frame (member 0)
    size_t fullframe_cap = 0;
    hipEvent_t frame_ev = nullptr;

    // timing
    std::vector<EventPair> pending_render, pending_fold, pool;
    double render_ms = 0, fold_ms = 0, last_render_ms = 0;
    // render-launch intervals relative to ref_ev (recorded before the first launch
    // after a stats reset), for the union of overlapping launches (render_busy_ms)
    hipEvent_t ref_ev = nullptr;
    bool ref_recorded = false;
    std::vector<std::pair<double, double>> spans;
    uint64_t launches = 0;

    Service svc;
};

namespace {

int fail(spt_ctx *ctx, int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    g_thread_error = buf;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                          \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail((ctx), SPT_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));        \
    } while (0)

int svc_end(spt_ctx *ctx);

template <class T>
int ensure(spt_ctx *ctx, T **p, size_t *cap, size_t count)
{
    if (*cap >= count && *p) return SPT_OK;
    if (*p) {
        // a resident service session would hold the device synchronisation until it idles out
        if (int rc = svc_end(ctx)) return rc;
        HIP_TRY(ctx, hipDeviceSynchronize());  // launches on caller streams may still read it
        HIP_TRY(ctx, hipFree(*p));
        *p = nullptr;
        *cap = 0;
    }
    size_t want = std::max<size_t>(count, 1);
    hipError_t e = hipMalloc((void **)p, want * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        return fail(ctx, SPT_ERR_NOMEM, "hipMalloc(%zu bytes) failed: %s", want * sizeof(T), hipGetErrorString(e));
    }
    *cap = want;
    return SPT_OK;
}

// A device buffer of ctx must live on ctx->device (multi-device contexts switch the
// current device between members).
int check_on_device(spt_ctx *ctx, const void *p, const char *what)
{
    hipPointerAttribute_t at{};
    HIP_TRY(ctx, hipPointerGetAttributes(&at, p));
    if (at.device != ctx->device)
        return fail(ctx, SPT_ERR_STATE, "%s is on device %d, not on member 0's device %d", what, at.device, ctx->device);
    return SPT_OK;
}

EventPair get_pair(spt_ctx *ctx)
{
    if (!ctx->pool.empty()) {
        EventPair p = ctx->pool.back();
        ctx->pool.pop_back();
        return p;
    }
    EventPair p;
    (void)hipEventCreate(&p.a);
    (void)hipEventCreate(&p.b);
    return p;
}

// Harvest launch timings: all of them (wait: blocking on their stop events), or only
// those whose launches have finished (a host call must not wait for other callers').
int collect_timings(spt_ctx *ctx, bool wait = true)
{
    for (auto *vec : {&ctx->pending_render, &ctx->pending_fold}) {
        std::vector<EventPair> keep;
        for (EventPair &p : *vec) {
            if (!wait) {
                const hipError_t q = hipEventQuery(p.b);
                if (q == hipErrorNotReady) {
                    keep.push_back(p);
                    continue;
                }
                HIP_TRY(ctx, q);
            }
            HIP_TRY(ctx, hipEventSynchronize(p.b));
            float ms = 0.f;
            HIP_TRY(ctx, hipEventElapsedTime(&ms, p.a, p.b));
            if (vec == &ctx->pending_render) {
                ctx->render_ms += ms;
                ctx->last_render_ms = ms;
                float ta = 0.f;
                HIP_TRY(ctx, hipEventElapsedTime(&ta, ctx->ref_ev, p.a));
                ctx->spans.emplace_back((double)ta, (double)ta + ms);
            } else {
                ctx->fold_ms += ms;
            }
            ctx->pool.push_back(p);
        }
        vec->swap(keep);
    }
    return SPT_OK;
}

// Length of the union of the recorded render-launch intervals.
double busy_ms(const spt_ctx *ctx)
{
    std::vector<std::pair<double, double>> v = ctx->spans;
    std::sort(v.begin(), v.end());
    double total = 0, cs = 0, ce = -1e300;
    for (const auto &iv : v) {
        if (iv.first > ce) {
            if (ce > cs) total += ce - cs;
            cs = iv.first;
            ce = iv.second;
        } else {
            ce = std::max(ce, iv.second);
        }
    }
    if (ce > cs) total += ce - cs;
    return total;
}

// Halvings after which every finite albedo component a of the scene, as the diffuse code
// rebuilds it (a * 0.5f, then * 0.5f per further bounce: spt_kernels.hip halve_n), is 0;
// at most kCodeSat.  Saturating j there changes no colour (diffuse_code).
uint32_t halvings_to_zero(const std::vector<float4> &shade)
{
    uint32_t jz = 0;
    for (const float4 &s : shade)
        for (float a : {s.x, s.y, s.z}) {
            if (!std::isfinite(a)) continue;  // inf and NaN stay themselves
            volatile float x = a * 0.5f;
            uint32_t j = 0;
            while (x != 0.f && j < spt::kCodeSat) {
                x = x * 0.5f;
                ++j;
            }
            jz = std::max(jz, j);
        }
    return jz;
}

// j's saturation of the diffuse codes at the context's depth: j <= bounces - 1 always
uint32_t code_jmax(const spt_ctx *ctx)
{
    return std::min(ctx->bounces > 0 ? ctx->bounces - 1u : 0u, ctx->code_jz);
}

spt::DeviceScene device_scene(const spt_ctx *ctx)
{
    return spt::DeviceScene{ctx->d_shade, ctx->d_mat, ctx->n, ctx->code_stride, code_jmax(ctx), ctx->accel};
}

int check_ready(spt_ctx *ctx)
{
    if (!ctx->scene_set) return fail(ctx, SPT_ERR_STATE, "scene not set (spt_set_scene)");
    if (!ctx->cam_set) return fail(ctx, SPT_ERR_STATE, "camera not set (spt_set_camera)");
    if (!ctx->params_set) return fail(ctx, SPT_ERR_STATE, "params not set (spt_set_params)");
    if (!spt::code_layout_fits(ctx->code_stride, code_jmax(ctx)))
        return fail(ctx, SPT_ERR_ARG,
                    "%u sphere slots at depth %u exceed the sample code space ((jmax + 1) * slots + 1 <= %u, jmax = %u)",
                    ctx->code_stride, ctx->bounces, spt::kCodeMax, code_jmax(ctx));
    return SPT_OK;
}

uint64_t fmix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Persistent grid of the context: once the caller renders on more than one stream
// (frames in flight), one block slot per CU is left free so the next frame's
// blocks start while this frame's tail drains: config 2 two-stream frame 8.57 ->
// 8.41 ms; single-stream launches keep the full grid (1-3% faster there).
// items per wave below which a launch with frames in flight takes grid_small
constexpr uint64_t kSmallGridItems = 3072;

// masked: the launch runs on a CU-masked stream (spt_set_reserved_cus, masked_for)
uint32_t full_grid(const spt_ctx *ctx, bool masked = false)
{
    const uint32_t g = ctx->ws.size() > 1 ? ctx->grid_overlap : ctx->grid;
    // reserved CUs: the persistent grid of the CUs the masked launch may use
    if (masked && ctx->reserve_cus && ctx->num_cu > 0)
        return std::max<uint32_t>(1u, (uint32_t)((uint64_t)g * (uint32_t)(ctx->num_cu - (int)ctx->reserve_cus) / (uint32_t)ctx->num_cu));
    return g;
}

// The CU-masked stream a launched render of caller stream s runs on (spt_set_reserved_cus;
// created on first use: every CU but the device's last reserve_cus) in *out.  A stream
// that cannot be created is an error (the render would otherwise keep no CU free).
int masked_for(spt_ctx *ctx, hipStream_t s, spt_ctx::Masked **out)
{
    *out = nullptr;
    for (spt_ctx::Masked &m : ctx->masked)
        if (m.caller == s) {
            *out = &m;
            return SPT_OK;
        }
    if (ctx->masked.size() >= kMaxCompanions)
        return fail(ctx, SPT_ERR_STATE, "reserved CUs: more than %zu caller streams", kMaxCompanions);
    const uint32_t n = (uint32_t)ctx->num_cu, keep = n - ctx->reserve_cus;
    std::vector<uint32_t> mask((n + 31) / 32, 0u);
    for (uint32_t i = 0; i < keep; ++i) mask[i / 32] |= 1u << (i % 32);
    spt_ctx::Masked m{s, nullptr, nullptr, nullptr};
    HIP_TRY(ctx, hipExtStreamCreateWithCUMask(&m.stream, (uint32_t)mask.size(), mask.data()));
    if (hipEventCreateWithFlags(&m.go, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m.done, hipEventDisableTiming) != hipSuccess) {
        (void)hipStreamDestroy(m.stream);
        return fail(ctx, SPT_ERR_HIP, "reserved CUs: event creation failed");
    }
    ctx->masked.reserve(kMaxCompanions);  // pointers handed out stay valid
    ctx->masked.push_back(m);
    *out = &ctx->masked.back();
    return SPT_OK;
}

// Items per claim: 256, or 512 for launches of at least 64 Ki items per wave (config 3's
// sample batches: 424.4 vs 429.0 ms per frame), 192 below 4 Ki items per wave (config 2's
// 1/8 rank share: 0.78 vs 0.82 ms), fewer only when the launch has under 4 claims per
// wave.  Every claim is one device-scope atomic, and atomics on one address
// serialise: with a single counter config 2 at 128 / 256 / 512 items per claim ran
// 8.66 / 6.04 / 5.29 ms per frame.  Claims now come from one counter per XCD
// (RenderArgs::n_queues), where small claims cost little and even out the tail: config 2
// at 128 / 192 / 256 / 384 / 512 items 5.43 / 5.32 / 5.29 / 5.28 / 5.32 ms, its 1/8
// rank share 0.78 / 0.78 / 0.80 / 0.91 / 1.03 ms (tools/scaling_probe.py), config 5
// (lane walk) 89.1 / 88.8 / 89.3 / - / 91.8 ms.  With primary
// batches and the max-ILP build, launches of 12-64 Ki items per wave (config 2's full
// frame) prefer 448: bench 20 533-20 561 (256) / 20 677-20 697 (384) / 20 727-20 731 (448)
// / 20 699-20 707 (512) Msamples/s, while its rank shares still prefer 256 (384: the 1/2
// share 2.414 -> 2.447 ms); trees walked lane by lane keep 256.
constexpr uint32_t kSmallClaim = 192, kClaim = 256, kMidClaim = 448, kBigClaim = 512;
uint32_t claim_size(const spt_ctx *ctx, uint64_t items, bool masked = false)
{
    if (ctx->claim) return ctx->claim;
    const uint64_t waves = std::max<uint64_t>((uint64_t)full_grid(ctx, masked) * (ctx->block / 64), 1);
    const uint64_t fair = items / (waves * 4);
    const uint64_t per_wave = items / waves;
    const bool lane = spt::lane_walk_tree(ctx->accel);
    const uint32_t cap = per_wave < 4096u ? kSmallClaim
                       : lane ? kClaim
                       : per_wave >= 65536u ? kBigClaim
                       : per_wave >= 12288u ? kMidClaim : kClaim;
    return (uint32_t)std::min<uint64_t>(cap, std::max<uint64_t>(64, fair / 64 * 64));
}

// Blocks of one render launch: the persistent grid, or fewer when the launch has
// fewer claims than that grid has waves.  A wave without a claim only starts,
// finds the counter exhausted and exits, and on config 1 (1250 claims, 8192
// waves) those waves tripled the launch time.
// div: host calls sharing the GPU side by side (each gets 1/div of the grid).
uint32_t render_grid(const spt_ctx *ctx, uint64_t items, uint32_t claim, uint32_t div, bool masked = false)
{
    const uint64_t claims = (items + claim - 1) / claim;
    const uint64_t per_block = (uint64_t)(ctx->block / 64) * ctx->claims_per_wave;
    uint64_t full = (full_grid(ctx, masked) + div - 1) / div;
    // frames in flight, a launch of under 3 Ki items per wave (config 2's 1/8 rank share):
    // one more block slot per CU left free, so fewer of the launch's paths are still in
    // flight when its claims run out and the other stream's launch takes the CUs sooner
    // (the 1/8 share 0.755-0.762 -> 0.725 ms per frame; the 1/4 share, 3.9 Ki items per
    // wave, would lose 0.5%: tools/scaling_probe.py)
    if (div == 1 && ctx->ws.size() > 1 && ctx->grid_small &&
        items < (uint64_t)full_grid(ctx, masked) * (ctx->block / 64) * kSmallGridItems)
        full = ctx->grid_small;
    return (uint32_t)std::min<uint64_t>(full, std::max<uint64_t>(1, (claims + per_block - 1) / per_block));
}

// The workspace of stream s (created on first use, at most kMaxWorkspaces).
Workspace *workspace_for(spt_ctx *ctx, hipStream_t s)
{
    for (Workspace &w : ctx->ws)
        if (w.stream == s) return &w;
    if (ctx->ws.size() >= kMaxWorkspaces) {
        fail(ctx, SPT_ERR_STATE, "more than %zu streams in use on one context", kMaxWorkspaces);
        return nullptr;
    }
    Workspace w;
    w.stream = s;
    if (hipMalloc((void **)&w.d_head, sizeof(uint32_t) * spt::kMaxQueues * spt::kQueueStride) != hipSuccess) {
        fail(ctx, SPT_ERR_NOMEM, "workspace allocation failed");
        return nullptr;
    }
    ctx->ws.push_back(w);
    return &ctx->ws.back();
}

// The companion stream of caller stream s (created on first use), or nullptr.
hipStream_t companion_for(spt_ctx *ctx, hipStream_t s)
{
    for (const auto &c : ctx->companions)
        if (c.first == s) return c.second;
    if (ctx->companions.size() >= kMaxCompanions) return nullptr;
    if (!ctx->dbuf_start && (hipEventCreateWithFlags(&ctx->dbuf_start, hipEventDisableTiming) != hipSuccess ||
                             hipEventCreateWithFlags(&ctx->dbuf_fold, hipEventDisableTiming) != hipSuccess))
        return nullptr;
    hipStream_t c = nullptr;
    if (hipStreamCreateWithFlags(&c, hipStreamNonBlocking) != hipSuccess) return nullptr;
    ctx->companions.emplace_back(s, c);
    return c;
}

// Queues of the wavefront engine in workspace w: `cap` rays in block queues of qcap.
int ensure_wavefront(spt_ctx *ctx, Workspace *w, uint32_t cap, uint32_t qcap)
{
    spt::WavefrontBuffers &b = w->wf;
    cap = std::max(cap / qcap, 1u) * qcap;
    if (b.cap >= cap && b.qcap == qcap && b.state) return SPT_OK;
    HIP_TRY(ctx, hipDeviceSynchronize());
    for (void *p : {(void *)b.o, (void *)b.d, (void *)b.m, (void *)b.state})
        if (p) (void)hipFree(p);
    b = spt::WavefrontBuffers{};
    bool ok = hipMalloc((void **)&b.o, (size_t)cap * sizeof(float4)) == hipSuccess;
    ok = ok && hipMalloc((void **)&b.d, (size_t)cap * sizeof(float4)) == hipSuccess;
    ok = ok && hipMalloc((void **)&b.m, (size_t)cap * sizeof(uint4)) == hipSuccess;
    ok = ok && hipMalloc((void **)&b.state, spt::kWfStateWords * sizeof(uint32_t)) == hipSuccess;
    if (!ok) return fail(ctx, SPT_ERR_NOMEM, "wavefront queues for %u rays: allocation failed", cap);
    b.cap = cap;
    b.qcap = qcap;
    return SPT_OK;
}

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

#define SVC_DBG(ctx, ...)                                                                              \
    do {                                                                                               \
        if ((ctx)->svc.debug) {                                                                        \
            std::fprintf(stderr, "[svc %.3f] ", std::chrono::duration<double, std::milli>(               \
                                                     std::chrono::steady_clock::now().time_since_epoch()) \
                                                     .count());                                        \
            std::fprintf(stderr, __VA_ARGS__);                                                         \
            std::fputc('\n', stderr);                                                                  \
        }                                                                                              \
    } while (0)

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
    const uint32_t grid = std::max<uint32_t>(1u, ctx->svc_grid / v.grid_div);
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
    // control words zeroed, the render-wave count set, before the kernel
    HIP_TRY(ctx, hipMemsetAsync(v.d_ctl, 0, spt::kSvcCtlWords * sizeof(uint32_t), v.stream));
    HIP_TRY(ctx, hipMemsetD32Async((hipDeviceptr_t)(v.d_ctl + spt::kSvcLive), (int)(grid * (spt::kRenderBlock / 64u) - 1u),
                                   1, v.stream));
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

// Can render_impl hand a launch of `words` sample words to the service?
bool svc_eligible(const spt_ctx *ctx, uint64_t words, bool keep_samples)
{
    const Service &v = ctx->svc;
    return v.enabled && !keep_samples && ctx->engine == SPT_ENGINE_MEGAKERNEL && spt::svc_supported(ctx->accel) &&
           words <= v.ring_bytes / sizeof(uint32_t) / 2;
}

// One job of a publication: a region (rows or interleaved strips, columns) at spp_batch
// samples from sample s0, its slots at slot_local of the publication's ring region.
struct SvcJobSpec {
    spt::RowMap map;
    uint32_t rows, spp_batch, s0;
    spt::FastDiv div_band, div_tile, div_strip;
    uint64_t slot_local;
};

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

// Fold arguments shared by every fold of ctx: the slots and the decode tables of the
// sample words (shading table, sky colour, code stride).
spt::FoldArgs fold_args(const spt_ctx *ctx, const uint32_t *samples, uint32_t slot_words)
{
    spt::FoldArgs fa{};
    fa.samples = samples;
    fa.slot_words = slot_words;
    fa.shade = ctx->d_shade;
    for (int j = 0; j < 3; ++j) fa.sky[j] = ctx->cam.sky[j];
    fa.code_div = spt::make_fastdiv(ctx->code_stride);
    return fa;
}

// Render the rows of `map` and fold them into d_rgba (local pixel order) and/or
// d_rgb8 (full frame).  keep_samples: leave the per-sample colours of a single
// batch in d_samples (debug path).
// Progressive rendering: batches of at most pass_spp samples, outputs written after
// every batch and after_pass(samples done) called (nonzero return: stop early).
struct Progress {
    uint32_t pass_spp;
    std::function<int(uint32_t)> after_pass;
};

// A range of RenderSegmentTask's colorIndex (spt_render_frame's split of a non-square
// frame): outputs [i0, i0 + n) of a call of map.width x alias_h pixels, folded from the
// rows the launch renders (FoldArgs::range_alias); d_rgba then holds n outputs.
struct AliasRange {
    uint32_t i0, n, alias_h;
};

// grid_div: concurrent host calls on this context share the GPU (render_grid)
int render_impl(spt_ctx *ctx, int mode, const spt::RowMap &map, float4 *d_rgba, uint8_t *d_rgb8, hipStream_t s,
                bool keep_samples, const Progress *pg = nullptr, uint32_t grid_div = 1, const AliasRange *ar = nullptr)
{
    const uint32_t rows = spt::rows_owned(map);
    const uint64_t npix64 = (uint64_t)rows * map.width;
    if (npix64 == 0 && ar && ar->n) {
        // a colorIndex range no pixel maps into: its outputs are 0 * (1.f / 0) = NaN
        // (TaskBasedPathTracer.hpp:196-205); the fold writes them without sources
        spt::FoldArgs fa = fold_args(ctx, nullptr, 2u);
        fa.out_rgba = d_rgba;
        fa.map = map;
        fa.width = ctx->W;
        fa.height = ctx->H;
        fa.npix = ar->n;
        fa.spp_batch = fa.spp_total = fa.s_done = ctx->spp;
        fa.first = fa.last = 1;
        fa.mode = mode;
        fa.range_alias = 1;
        fa.out_i0 = ar->i0;
        fa.alias_h = ar->alias_h;
        fa.src_rows = 0;
        HIP_TRY(ctx, spt::launch_fold(fa, s));
        return SPT_OK;
    }
    if (npix64 == 0) return SPT_OK;
    if (npix64 > 0x7FFFFFFFull) return fail(ctx, SPT_ERR_ARG, "region too large (%llu pixels)", (unsigned long long)npix64);
    const uint32_t npix = (uint32_t)npix64;
    const uint32_t slot_words = mode == SPT_MODE_SEGMENT ? 1u : 2u;  // task mode keeps the path's order key
    uint64_t budget = std::max<uint64_t>(ctx->ws_bytes / (slot_words * sizeof(uint32_t)), 1);
    budget = std::min<uint64_t>(budget, 0x7FFFFFFFull);
    uint64_t per = std::max<uint64_t>(1, budget / npix);
    uint32_t spp_batch = (uint32_t)std::min<uint64_t>(ctx->spp, per);
    if (pg) spp_batch = std::min(spp_batch, std::max(pg->pass_spp, 1u));
    if (keep_samples && spp_batch != ctx->spp)
        return fail(ctx, SPT_ERR_ARG, "region * spp exceeds the workspace for spt_render_samples");
    const uint64_t items_max = (uint64_t)npix * spp_batch;
    // the resident render service takes the launch when it is on and can (svc_eligible);
    // a launch it cannot take ends the session first, so that launch has the whole GPU
    const bool use_svc = svc_eligible(ctx, items_max * slot_words, keep_samples);
    int rc = SPT_OK;
    if (!use_svc && (rc = svc_end(ctx))) return rc;
    Workspace *w = workspace_for(ctx, s);
    if (!w) return SPT_ERR_STATE;
    if (!use_svc && (rc = ensure(ctx, &w->d_samples, &w->samples_cap, items_max * slot_words))) return rc;
    if (spp_batch < ctx->spp) {
        rc = ensure(ctx, &w->d_acc, &w->acc_cap, ar ? std::max(npix, ar->n) : npix);
        if (rc) return rc;
    }
    // several batches: odd batches render on the companion stream into its own
    // workspace, so batch j+1 renders while batch j is folded and the GPU never waits
    // for a batch's last paths (config 3: 6 batches per frame).  The folds stay in
    // batch order (each waits for the previous one): the sums are unchanged.
    hipStream_t s2 = nullptr;
    Workspace *w2 = nullptr;
    if (!use_svc && spp_batch < ctx->spp && !pg && !keep_samples && ctx->batch_dbuf && ctx->engine == SPT_ENGINE_MEGAKERNEL &&
        (s2 = companion_for(ctx, s)) != nullptr && (w2 = workspace_for(ctx, s2)) != nullptr) {
        if ((rc = ensure(ctx, &w2->d_samples, &w2->samples_cap, items_max * slot_words))) return rc;
        // the companion starts after the work already queued on the caller's stream
        HIP_TRY(ctx, hipEventRecord(ctx->dbuf_start, s));
        HIP_TRY(ctx, hipStreamWaitEvent(s2, ctx->dbuf_start, 0));
    } else {
        s2 = nullptr;
        w2 = nullptr;
    }
    const hipStream_t s_caller = s;
    Workspace *const w_caller = w;
    // reserved CUs: the launches of this call on the caller stream's CU-masked stream,
    // ordered after the caller's queued work (and the caller after them, below)
    // (renders through the service, double-buffered batches and progressive passes run on
    // every CU with the whole grid)
    spt_ctx::Masked *mk_ = nullptr;
    if (ctx->reserve_cus && !use_svc && !s2 && !pg && (rc = masked_for(ctx, s, &mk_))) return rc;
    if (mk_) {
        HIP_TRY(ctx, hipEventRecord(mk_->go, s));
        HIP_TRY(ctx, hipStreamWaitEvent(mk_->stream, mk_->go, 0));
        s = mk_->stream;
    }

    spt::RenderArgs ra{};
    ra.scene = device_scene(ctx);
    ra.prim = ctx->prim;
    ra.cam = ctx->cam;
    ra.width = ctx->W;
    ra.height = ctx->H;
    ra.bounces = ctx->bounces;
    ra.mode = (uint32_t)mode;
    ra.seed_key = fmix64(ctx->seed);
    ra.map = map;
    ra.div_strip = spt::make_fastdiv(std::max<uint32_t>(map.strip, 1u));
    ra.npix = npix;
    ra.claim = claim_size(ctx, (uint64_t)npix * spp_batch, mk_ != nullptr);
    ra.samples = w->d_samples;
    ra.slot_words = slot_words;
    ra.head = w->d_head;
    ra.counters = ctx->d_counters;

    spt::FoldArgs fa = fold_args(ctx, w->d_samples, slot_words);
    fa.acc = w->d_acc;
    fa.out_rgba = d_rgba;
    fa.out_rgb8 = d_rgb8;
    fa.map = map;
    fa.width = ctx->W;
    fa.height = ctx->H;
    fa.npix = npix;
    fa.spp_total = ctx->spp;
    fa.mode = mode;
    fa.preview = pg ? 1 : 0;
    // one rectangle in task mode = one RenderSegmentTask call: its colorIndex aliasing
    fa.alias = mode == SPT_MODE_TASK && map.parts == 1u && rows != map.width ? 1 : 0;
    if (ar) {
        fa.range_alias = 1;
        fa.alias = 0;
        fa.npix = ar->n;
        fa.out_i0 = ar->i0;
        fa.alias_h = ar->alias_h;
        fa.src_rows = rows;
        fa.out_rgb8 = nullptr;
    }

    uint32_t j = 0;
    for (uint32_t s0 = 0; s0 < ctx->spp; s0 += spp_batch, ++j) {
        const uint32_t b = std::min(spp_batch, ctx->spp - s0);
        if (s2) {
            s = (j & 1u) ? s2 : s_caller;
            w = (j & 1u) ? w2 : w_caller;
            ra.samples = w->d_samples;
            fa.samples = w->d_samples;
            ra.head = w->d_head;
        }
        ra.spp_batch = b;
        ra.s0 = s0;
        ra.n_items = npix * b;
        ra.n_queues = ctx->queues;
        {
            const uint32_t per = (ra.n_items + ra.n_queues - 1u) / ra.n_queues;
            ra.queue_items = (per + ra.claim - 1u) / ra.claim * ra.claim;
        }
        ra.div_band = spt::make_fastdiv(rows >= 8 ? 8u * map.width * b : 1u);
        ra.div_tile = spt::make_fastdiv(64u * b);
        EventPair ev = get_pair(ctx);
        uint64_t svc_w0 = 0;
        uint32_t svc_idx = 0;
        if (use_svc) {
            // published to the service; the stream waits for the job's completion counter
            // (the events bracket that wait: the job's span as the stream sees it)
            if (!ctx->ref_recorded) {
                HIP_TRY(ctx, hipEventRecord(ctx->ref_ev, s));
                ctx->ref_recorded = true;
            }
            HIP_TRY(ctx, hipEventRecord(ev.a, s));
            if ((rc = svc_submit(ctx, ra, mode, s, &svc_w0, &svc_idx))) return rc;
            HIP_TRY(ctx, hipEventRecord(ev.b, s));
            fa.samples = ctx->svc.d_ring + svc_w0;
        } else if (ctx->engine == SPT_ENGINE_WAVEFRONT) {
            // every pass of the batch in one launch of block queue workers; queue
            // lengths stay on the device
            // (queues for the resident blocks only: a block past them would start late)
            const uint64_t blocks = spt::wavefront_blocks(ctx->accel, ctx->device);
            if (blocks == 0) return fail(ctx, SPT_ERR_HIP, "wavefront engine: no resident blocks");
            const uint32_t cap = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(ctx->wf_cap, blocks * ctx->wf_queue),
                                                               std::max<uint32_t>(ra.n_items, 1024u));
            if ((rc = ensure_wavefront(ctx, w, cap, ctx->wf_queue))) return rc;
            HIP_TRY(ctx, hipEventRecord(ev.a, s));
            if (!ctx->ref_recorded) {
                HIP_TRY(ctx, hipEventRecord(ctx->ref_ev, s));
                ctx->ref_recorded = true;
            }
            HIP_TRY(ctx, spt::launch_wavefront(w->wf, ra, s));
            HIP_TRY(ctx, hipEventRecord(ev.b, s));
        } else {
            HIP_TRY(ctx, hipMemsetAsync(w->d_head, 0, sizeof(uint32_t) * spt::kQueueStride * ra.n_queues, s));
            if (!ctx->ref_recorded) {
                HIP_TRY(ctx, hipEventRecord(ctx->ref_ev, s));
                ctx->ref_recorded = true;
            }
            HIP_TRY(ctx, hipEventRecord(ev.a, s));
            spt::LaunchShape sh{render_grid(ctx, ra.n_items, ra.claim, grid_div, mk_ != nullptr), ctx->block, grid_div, 0, 0};
            HIP_TRY(ctx, spt::launch_render(ra, sh, s));
            ctx->last_grid = sh.ran_grid;
            ctx->last_block = sh.ran_block;
            HIP_TRY(ctx, hipEventRecord(ev.b, s));
        }
        ctx->pending_render.push_back(ev);
        ctx->launches++;
        if (keep_samples) continue;
        fa.spp_batch = b;
        fa.first = s0 == 0;
        fa.last = s0 + b >= ctx->spp;
        fa.s_done = s0 + b;
        EventPair ef = get_pair(ctx);
        // double-buffered: fold j after fold j-1 (the other stream; shared accumulator)
        if (s2 && j > 0) HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->dbuf_fold, 0));
        fa.prio = use_svc ? 0 : 1;
        HIP_TRY(ctx, hipEventRecord(ef.a, s));
        HIP_TRY(ctx, spt::launch_fold(fa, s));
        HIP_TRY(ctx, hipEventRecord(ef.b, s));
        if (s2) HIP_TRY(ctx, hipEventRecord(ctx->dbuf_fold, s));
        ctx->pending_fold.push_back(ef);
        if (use_svc && (rc = svc_retire(ctx, s, svc_w0, (uint64_t)npix * b * slot_words, svc_idx))) return rc;
        if (pg && pg->after_pass) {
            const int r = pg->after_pass(s0 + b);
            if (r < 0) return r;
            if (r > 0) break;  // the caller stopped the render
        }
    }
    // the caller's stream continues after the last fold (and with it every batch)
    if (s2 && s != s_caller) HIP_TRY(ctx, hipStreamWaitEvent(s_caller, ctx->dbuf_fold, 0));
    if (mk_) {
        HIP_TRY(ctx, hipEventRecord(mk_->done, mk_->stream));
        HIP_TRY(ctx, hipStreamWaitEvent(s_caller, mk_->done, 0));
    }
    if (ctx->pending_render.size() > 256) return collect_timings(ctx);
    return SPT_OK;
}

template <class T>
int upload(spt_ctx *ctx, T **p, size_t *cap, const std::vector<T> &v)
{
    int rc = ensure(ctx, p, cap, v.size());
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return SPT_OK;
}

// Traversal shape for the current scene: a 4-ary (3-ary above 512 spheres) tree of
// boxes over 8-sphere clusters (config 2: 14 650 Msamples/s against 13 950 for round 1's flat list of
// 4-sphere clusters under bounding spheres); the flat list remains
// selectable (spt_set_cluster_tree(ctx, 0)).  Scenes of <= 32 spheres are tested
// brute force (build_accel).
struct Shape {
    uint32_t k, branching, leaf_slots;
};
Shape resolve_shape(const spt_ctx *ctx)
{
    const bool tree = ctx->tree_branching == SPT_TREE_AUTO ? true : ctx->tree_branching >= 2;
    Shape sh;
    sh.k = ctx->cluster_k != SPT_CLUSTER_AUTO ? ctx->cluster_k : tree ? spt::kClusterSlots : spt::kFlatLeafSlots;
    // auto: 4 children per node; 3 for large scenes, whose trees the LDS kernel walks
    // lane by lane (config 5: 107 ms per frame against 110 for 4)
    sh.branching = tree ? (ctx->tree_branching == SPT_TREE_AUTO ? (ctx->n > 512 ? 3u : 4u) : ctx->tree_branching) : 0u;
    sh.leaf_slots = !tree && sh.k <= spt::kFlatLeafSlots ? spt::kFlatLeafSlots : spt::kClusterSlots;
    return sh;
}

// Build and upload the hot-loop traversal tables (spt_accel.cpp) for the current scene.
int rebuild_accel(spt_ctx *ctx)
{
    const auto t_start = std::chrono::steady_clock::now();
    const uint32_t g = spt::render_group_size();
    const Shape sh = resolve_shape(ctx);
    spt::AccelTables t = spt::build_accel(ctx->h_centers.data(), ctx->h_radii.data(), ctx->n, sh.k, g, sh.branching,
                                          sh.leaf_slots);
    const std::string bad = spt::validate_accel(t, ctx->h_centers.data(), ctx->h_radii.data(), ctx->n);
    if (!bad.empty()) return fail(ctx, SPT_ERR_STATE, "traversal tables invalid: %s", bad.c_str());
    // a diffuse sample's code is 2 + j * slots + slot (diffuse_code); check_ready checks
    // that the scene's codes fit at the frame's depth
    const uint32_t jz = halvings_to_zero(ctx->h_shade);
    if (!spt::code_layout_fits(t.slots.size(), 0))
        return fail(ctx, SPT_ERR_ARG, "%zu sphere slots exceed the sample code space", t.slots.size());
    // shading tables in slot order: the kernel keeps the winner's slot, not its index
    std::vector<float4> shade(t.slots.size(), make_float4(0.f, 0.f, 0.f, 0.f));
    std::vector<uint32_t> mat(t.slots.size(), SPT_SKYBOX);
    for (size_t j = 0; j < t.slots.size(); ++j)
        if (t.orig[j] != 0xFFFFFFFFu) {
            shade[j] = ctx->h_shade[t.orig[j]];
            mat[j] = ctx->h_mat[t.orig[j]];
        }
    // every stream: host calls and caller-stream renders may still read the tables
    HIP_TRY(ctx, hipDeviceSynchronize());
    int rc = upload(ctx, &ctx->d_slots, &ctx->slots_cap, t.slots);
    if (!rc) rc = upload(ctx, &ctx->d_shade, &ctx->shade_cap, shade);
    if (!rc) rc = upload(ctx, &ctx->d_mat, &ctx->mat_cap, mat);
    if (!rc) rc = upload(ctx, &ctx->d_orig, &ctx->orig_cap, t.orig);
    if (!rc) rc = upload(ctx, &ctx->d_nodes, &ctx->nodes_cap, t.nodes);
    if (!rc) rc = upload(ctx, &ctx->d_kpre, &ctx->kpre_cap, t.kpre);
    if (rc) return rc;
    ctx->accel = spt::AccelView{ctx->d_slots, ctx->d_orig, ctx->d_nodes, t.always_groups, t.n_nodes,
                                t.n_nodes > t.leaves ? 1u : 0u, t.leaf_slots, ctx->d_kpre, t.pre_cm};
    ctx->code_stride = (uint32_t)std::max<size_t>(t.slots.size(), 1);
    ctx->code_jz = jz;
    ctx->tables = std::move(t);
    ctx->accel_gen++;
    ctx->accel_build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    return SPT_OK;
}

// Wait for every render launch this context has enqueued (on any stream) -- not for the
// device: unrelated work of the process (torch kernels, RCCL) keeps running.
int wait_own_renders(spt_ctx *ctx)
{
    for (const EventPair &p : ctx->pending_render) HIP_TRY(ctx, hipEventSynchronize(p.b));
    return SPT_OK;
}

// Build and upload the primary-ray candidate lists for the current scene, camera and frame
// size (none for trees walked lane by lane, which have no primary batches: casting their
// freshly started paths against the lists cut config 5's node visits per ray 17.1 -> 12.7
// but not its walk iterations or time).
int rebuild_prim(spt_ctx *ctx)
{
    const bool want = ctx->prim_enabled && ctx->scene_set && ctx->cam_set && ctx->params_set &&
                      !spt::lane_walk_tree(ctx->accel);
    spt_ctx::PrimKey key{};
    for (int i = 0; i < 12; ++i) key.view[i] = ctx->cam.view[i];
    for (int i = 0; i < 3; ++i) key.eye[i] = ctx->cam.eye[i];
    key.W = ctx->W;
    key.H = ctx->H;
    key.prim_max = ctx->prim_max;
    key.accel_gen = ctx->accel_gen;
    key.valid = true;
    // the lists depend on the accel tables, the camera and the frame size only
    if (want && key.same(ctx->prim_key)) return SPT_OK;
    ctx->prim = spt::PrimLists{};
    ctx->prim_blocks = ctx->prim_entries = 0;
    ctx->prim_key = spt_ctx::PrimKey{};
    if (!want) return SPT_OK;
    spt::PrimListTables pl = spt::build_prim_lists(ctx->tables, ctx->cam, ctx->W, ctx->H, ctx->prim_max);
    ctx->prim_build_s = pl.seconds;
    ctx->prim_builds++;
    ctx->prim_key = key;
    if (!pl.on) return SPT_OK;
    // this context's renders in flight may still read the previous lists
    if (int rc = wait_own_renders(ctx)) return rc;
    int rc = upload(ctx, &ctx->d_prim_b8, &ctx->prim_b8_cap, pl.b8);
    if (!rc) rc = upload(ctx, &ctx->d_prim_b4, &ctx->prim_b4_cap, pl.b4);
    if (!rc) rc = upload(ctx, &ctx->d_prim_slots, &ctx->prim_slots_cap, pl.slots);
    if (rc) return rc;
    ctx->prim = spt::PrimLists{ctx->d_prim_b8, ctx->d_prim_b4, ctx->d_prim_slots, pl.bw, 1u};
    for (const uint2 &b : pl.b8) ctx->prim_blocks += b.y != spt::kPrimWalk ? 1u : 0u;
    ctx->prim_entries = (uint32_t)pl.slots.size();
    return SPT_OK;
}

int check_region(spt_ctx *ctx, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE)
{
    if (yE > ctx->H || xE > ctx->W)
        return fail(ctx, SPT_ERR_ARG, "region [%u,%u)x[%u,%u) outside %ux%u frame", yB, yE, xB, xE, ctx->W, ctx->H);
    return SPT_OK;
}

// A free host-call slot of ctx (created on demand, at most ctx->host_slots; waits for
// one to free up beyond that).  Called with ctx->mu held through lk.
HostSlot *acquire_slot(spt_ctx *ctx, std::unique_lock<std::mutex> &lk)
{
    for (;;) {
        for (HostSlot *h : ctx->slots)
            if (!h->busy) {
                h->busy = true;
                return h;
            }
        if (ctx->slots.size() < ctx->host_slots) {
            HostSlot *h = new HostSlot();
            if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
                delete h;
                fail(ctx, SPT_ERR_HIP, "stream creation failed");
                return nullptr;
            }
            h->busy = true;
            ctx->slots.push_back(h);
            return h;
        }
        ctx->slot_cv.wait(lk);
    }
}

void release_slot(spt_ctx *ctx, HostSlot *h)
{
    h->busy = false;
    ctx->slot_cv.notify_one();
}

// The member of a multi-device context with the fewest host calls in flight.
spt_ctx *pick_member(spt_ctx *ctx)
{
    spt_ctx *best = ctx;
    for (spt_ctx *p : ctx->peers)
        if (p->inflight.load() < best->inflight.load()) best = p;
    return best;
}

// Bytes of per-sample slots a rectangle needs in one batch (all spp samples at once).
uint64_t batch_slot_bytes(const spt_ctx *ctx, int mode, uint64_t npix)
{
    return npix * ctx->spp * (mode == SPT_MODE_SEGMENT ? 1u : 2u) * sizeof(uint32_t);
}

// Enqueue one batch on bs->stream: rectangle table, render, fold, the copy-back of
// every request's outputs.  Called with ctx->mu held.
int launch_batch(spt_ctx *ctx, BatchSet *bs, const std::vector<BatchReq *> &batch, uint8_t *spec_d8 = nullptr)
{
    const int mode = batch[0]->mode;
    const uint32_t slot_words = mode == SPT_MODE_SEGMENT ? 1u : 2u;
    const uint32_t spp = ctx->spp, W = ctx->W, H = ctx->H;
    uint64_t items = 0, pix = 0;
    bool any_rgba = false, any_g = false;
    for (const BatchReq *r : batch) {
        const uint64_t np = (uint64_t)(r->xE - r->xB) * (r->yE - r->yB);
        items += np * spp;
        pix += np;
        any_rgba |= r->rgba != nullptr;
        any_g |= r->g_data != nullptr;
    }
    const uint32_t claim = claim_size(ctx, items);
    // rectangles' items start at claim multiples (a claim never spans two)
    const size_t n = batch.size();
    int rc = SPT_OK;
    if (bs->h_rects_cap < n) {
        // hipHostFree synchronises the device, which a resident service kernel would hold
        // until its waves idle out (0.5 s): end the session first; grow geometrically
        if ((rc = svc_end(ctx))) return rc;
        const size_t cap = std::max<size_t>({n, 2 * bs->h_rects_cap, 64});
        if (bs->h_rects) HIP_TRY(ctx, hipHostFree(bs->h_rects));
        bs->h_rects = nullptr;
        bs->h_rects_cap = 0;
        HIP_TRY(ctx, hipHostMalloc((void **)&bs->h_rects, cap * sizeof(spt::BatchRect)));
        bs->h_rects_cap = cap;
    }
    if ((rc = ensure(ctx, &bs->d_rects, &bs->rects_cap, n))) return rc;
    if (any_g && !spec_d8 && (rc = ensure(ctx, &ctx->d_frame8, &ctx->frame8_cap, (size_t)W * H * 3))) return rc;
    uint64_t item = 0, slot = 0, px = 0;
    for (size_t i = 0; i < n; ++i) {
        const BatchReq *r = batch[i];
        spt::BatchRect &b = bs->h_rects[i];
        const uint32_t w = r->xE - r->xB, rows = r->yE - r->yB, np = w * rows;
        item = (item + claim - 1) / claim * claim;
        b.item_off = (uint32_t)item;
        b.item_end = (uint32_t)(item + (uint64_t)np * spp);
        b.slot_off = (uint32_t)slot;
        b.pix_off = (uint32_t)px;
        b.x0 = r->xB;
        b.y0 = r->yB;
        b.w = w;
        b.rows = rows;
        b.npix = np;
        b.alias = mode == SPT_MODE_TASK && rows != w ? 1u : 0u;
        // g_data inside a page-locked buffer (spt_pin_host; the C++ shim pins it): the
        // fold writes the bytes in place, no copy-back
        b.rgb8 = nullptr;
        if (r->g_data && spec_d8) {
            b.rgb8 = spec_d8;  // read-ahead: the frame's device copy, no copy-back here
        } else if (r->g_data) {
            b.rgb8 = ctx->d_frame8;
            const size_t fb = (size_t)W * H * 3;
            for (const spt_ctx::Pinned &p : ctx->pinned) {
                const uint8_t *base = (const uint8_t *)p.ptr;
                if (p.dev && r->g_data >= base && r->g_data + fb <= base + p.bytes) {
                    b.rgb8 = p.dev + (r->g_data - base);
                    break;
                }
            }
        }
        b.div_band = spt::make_fastdiv(rows >= 8 ? 8u * w * spp : 1u);
        b.div_tile = spt::make_fastdiv(64u * spp);
        item = b.item_end;
        slot += (uint64_t)np * spp;
        px += np;
    }
    // the render service takes the batch when it is on: one job per call, one counter
    const bool use_svc = svc_eligible(ctx, slot * slot_words, false);
    if (!use_svc && (rc = svc_end(ctx))) return rc;
    Workspace *w = workspace_for(ctx, bs->stream);
    if (!w) return SPT_ERR_STATE;
    if (!use_svc && (rc = ensure(ctx, &w->d_samples, &w->samples_cap, (size_t)slot * slot_words))) return rc;
    if (any_rgba && (rc = ensure(ctx, &bs->d_stage, &bs->stage_cap, (size_t)pix))) return rc;
    const hipStream_t s = bs->stream;
    uint64_t svc_w0 = 0;
    uint32_t svc_idx = 0;
    EventPair ev = get_pair(ctx);
    if (use_svc) {
        std::vector<SvcJobSpec> specs(n);
        for (size_t i = 0; i < n; ++i) {
            const spt::BatchRect &b = bs->h_rects[i];
            specs[i] = SvcJobSpec{spt::RowMap{b.y0, b.y0 + b.rows, 1u, 1u, 0u, b.x0, b.w}, b.rows, spp, 0u, b.div_band,
                                  b.div_tile, spt::make_fastdiv(1u), b.slot_off};
        }
        if (!ctx->ref_recorded) {
            HIP_TRY(ctx, hipEventRecord(ctx->ref_ev, s));
            ctx->ref_recorded = true;
        }
        HIP_TRY(ctx, hipEventRecord(ev.a, s));
        if ((rc = svc_submit_jobs(ctx, mode, specs.data(), n, slot, s, &svc_w0, &svc_idx))) return rc;
        HIP_TRY(ctx, hipEventRecord(ev.b, s));
        // the fold reads each call's slots in the ring
        for (size_t i = 0; i < n; ++i) bs->h_rects[i].slot_off += (uint32_t)(svc_w0 / slot_words);
        ctx->pending_render.push_back(ev);
        ctx->launches++;
    }
    // up to kInlineRects rectangles travel in the kernel arguments; more in the table
    const bool inl = n <= spt::kInlineRects;
    if (!inl)
        HIP_TRY(ctx, hipMemcpyAsync(bs->d_rects, bs->h_rects, n * sizeof(spt::BatchRect), hipMemcpyHostToDevice, s));

    spt::RenderArgs ra{};
    ra.scene = device_scene(ctx);
    ra.prim = ctx->prim;
    ra.cam = ctx->cam;
    ra.width = W;
    ra.height = H;
    ra.bounces = ctx->bounces;
    ra.mode = (uint32_t)mode;
    ra.seed_key = fmix64(ctx->seed);
    ra.map = spt::RowMap{0u, 1u, 1u, 1u, 0u, 0u, 1u};  // per rectangle (BatchRect)
    ra.div_strip = spt::make_fastdiv(1u);
    ra.npix = (uint32_t)pix;
    ra.spp_batch = spp;
    ra.s0 = 0;
    ra.n_items = (uint32_t)item;
    ra.claim = claim;
    // queues of claim multiples: a claim still never spans two rectangles
    ra.n_queues = ctx->queues;
    {
        const uint32_t per = (ra.n_items + ra.n_queues - 1u) / ra.n_queues;
        ra.queue_items = (per + claim - 1u) / claim * claim;
    }
    ra.div_band = ra.div_tile = spt::make_fastdiv(1u);
    ra.samples = w->d_samples;
    ra.slot_words = slot_words;
    ra.head = w->d_head;
    ra.counters = ctx->d_counters;
    ra.rects = bs->d_rects;
    ra.n_rects = (uint32_t)n;
    ra.inline_rects = inl ? 1u : 0u;
    if (inl)
        for (size_t i = 0; i < n; ++i) ra.rects_inline[i] = bs->h_rects[i];

    // the claim counters are zeroed by the previous batch's fold on this workspace
    // (FoldArgs::head_reset), or here when that fold did not run
    if (!use_svc) {
        if (!w->head_clean)
            HIP_TRY(ctx, hipMemsetAsync(w->d_head, 0, sizeof(uint32_t) * spt::kQueueStride * ra.n_queues, s));
        w->head_clean = false;
        if (!ctx->ref_recorded) {
            HIP_TRY(ctx, hipEventRecord(ctx->ref_ev, s));
            ctx->ref_recorded = true;
        }
        HIP_TRY(ctx, hipEventRecord(ev.a, s));
        // read-ahead parts take the whole grid: the second part's blocks fill the CUs as the
        // first part's drain, so the first half of the tiles is served at half the frame
        const uint32_t gdiv = spec_d8 ? 1u : ctx->batch_grid_div;
        spt::LaunchShape sh{render_grid(ctx, ra.n_items, claim, gdiv), ctx->block, gdiv,
                            0, 0};
        HIP_TRY(ctx, spt::launch_render(ra, sh, s));
        ctx->last_grid = sh.ran_grid;
        ctx->last_block = sh.ran_block;
        HIP_TRY(ctx, hipEventRecord(ev.b, s));
        ctx->pending_render.push_back(ev);
        ctx->launches++;
    }

    spt::FoldArgs fa = fold_args(ctx, use_svc ? ctx->svc.d_ring : w->d_samples, slot_words);
    fa.out_rgba = any_rgba ? bs->d_stage : nullptr;
    fa.out_rgb8 = any_g ? (spec_d8 ? spec_d8 : ctx->d_frame8) : nullptr;
    fa.width = W;
    fa.height = H;
    fa.npix = (uint32_t)pix;
    fa.spp_batch = spp;
    fa.spp_total = spp;
    fa.s_done = spp;
    fa.first = fa.last = 1;
    fa.mode = mode;
    fa.rects = bs->d_rects;
    fa.n_rects = (uint32_t)n;
    fa.inline_rects = inl ? 1u : 0u;
    if (inl)
        for (size_t i = 0; i < n; ++i) fa.rects_inline[i] = bs->h_rects[i];
    fa.head_reset = !use_svc ? w->d_head : nullptr;
    fa.head_queues = ra.n_queues;
    fa.prio = use_svc ? 0 : 1;
    EventPair ef = get_pair(ctx);
    HIP_TRY(ctx, hipEventRecord(ef.a, s));
    HIP_TRY(ctx, spt::launch_fold(fa, s));
    w->head_clean = !use_svc;
    HIP_TRY(ctx, hipEventRecord(ef.b, s));
    ctx->pending_fold.push_back(ef);

    for (size_t i = 0; i < n; ++i) {
        const BatchReq *r = batch[i];
        const spt::BatchRect &b = bs->h_rects[i];
        if (r->rgba)
            HIP_TRY(ctx, hipMemcpyAsync(r->rgba, bs->d_stage + b.pix_off, (size_t)b.npix * sizeof(float4),
                                        hipMemcpyDeviceToHost, s));
        if (r->g_data && !spec_d8 && b.rgb8 == ctx->d_frame8) {
            // rows y in [yB, yE) live at g_data rows H-1-y: one band, xB.. per row
            const size_t pitch = (size_t)W * 3;
            const size_t off = (size_t)(H - r->yE) * pitch + (size_t)r->xB * 3;
            HIP_TRY(ctx, hipMemcpy2DAsync(r->g_data + off, pitch, ctx->d_frame8 + off, pitch, (size_t)b.w * 3, b.rows,
                                          hipMemcpyDeviceToHost, s));
        }
    }
    if (use_svc && (rc = svc_retire(ctx, s, svc_w0, slot * slot_words, svc_idx))) return rc;
    return SPT_OK;
}

// One RenderSegment / RenderSegmentTask call through the batcher: the call joins the
// pending list; a caller that finds no batch being assembled becomes the leader,
// waits for a free batch set, takes every pending call of the first one's mode (up
// to the workspace), launches them as one batch and waits for it unlocked, then
// marks them done.  Called with ctx->mu held through lk.
int render_batched(spt_ctx *ctx, std::unique_lock<std::mutex> &lk, int mode, uint32_t yB, uint32_t yE, uint32_t xB,
                   uint32_t xE, float *rgba, uint8_t *g_data)
{
    BatchReq req{mode, yB, yE, xB, xE, rgba, g_data, SPT_OK, false, false};
    ctx->batch_pending.push_back(&req);
    while (!req.done) {
        if (ctx->batch_leader || req.launched) {
            ctx->batch_cv.wait(lk);
            continue;
        }
        ctx->batch_leader = true;
        BatchSet *bs = nullptr;
        for (;;) {
            for (uint32_t q = 0; q < ctx->batch_sets; ++q)
                if (!ctx->bsets[q].busy) {
                    bs = &ctx->bsets[q];
                    break;
                }
            if (bs) break;
            ctx->batch_cv.wait(lk);
        }
        // FIFO, the first pending call's mode, within the workspace and 2^31 items
        std::vector<BatchReq *> batch, rest;
        uint64_t bytes = 0, items = 0;
        const int bmode = ctx->batch_pending.empty() ? req.mode : ctx->batch_pending.front()->mode;
        for (BatchReq *r : ctx->batch_pending) {
            const uint64_t np = (uint64_t)(r->xE - r->xB) * (r->yE - r->yB);
            if (r->yE > ctx->H || r->xE > ctx->W || np * ctx->spp >= 0x7FFF0000ull) {
                // the frame shrank or spp grew (spt_set_params) after the call was checked
                r->rc = fail(ctx, SPT_ERR_ARG, "region [%u,%u)x[%u,%u) no longer fits the %ux%u frame at %u spp",
                             r->yB, r->yE, r->xB, r->xE, ctx->W, ctx->H, ctx->spp);
                r->launched = r->done = true;
                continue;
            }
            const uint64_t b = batch_slot_bytes(ctx, bmode, np), it = np * ctx->spp + 1024;
            const bool fits = batch.empty() || (bytes + b <= ctx->ws_bytes && items + it < 0x7FFFFFFFull);
            if (r->mode != bmode || !fits) {
                rest.push_back(r);
                continue;
            }
            batch.push_back(r);
            bytes += b;
            items += it;
        }
        ctx->batch_pending.swap(rest);
        if (batch.empty()) {  // every pending call failed the checks above
            ctx->batch_leader = false;
            ctx->batch_cv.notify_all();
            continue;
        }
        for (BatchReq *r : batch) r->launched = true;
        bs->busy = true;
        ctx->batch_leader = false;
        ctx->batch_cv.notify_all();  // the next caller may assemble the next batch
        if (!bs->stream && hipStreamCreateWithFlags(&bs->stream, hipStreamNonBlocking) != hipSuccess) bs->stream = nullptr;
        int rc = bs->stream ? launch_batch(ctx, bs, batch) : fail(ctx, SPT_ERR_HIP, "stream creation failed");
        if (rc == SPT_OK) {
            lk.unlock();
            const hipError_t e = hipStreamSynchronize(bs->stream);
            lk.lock();
            if (e != hipSuccess) rc = fail(ctx, SPT_ERR_HIP, "hipStreamSynchronize failed: %s", hipGetErrorString(e));
        } else if (bs->stream) {
            (void)hipStreamSynchronize(bs->stream);  // whatever was enqueued before the failure
        }
        ctx->batches++;
        ctx->batched_calls += batch.size();
        for (BatchReq *r : batch) {
            r->rc = rc;
            r->done = true;
        }
        bs->busy = false;
        if (rc == SPT_OK) rc = collect_timings(ctx, false);
        ctx->batch_cv.notify_all();
    }
    return req.rc;
}

// ---- tiling read-ahead (SpecFrame) ------------------------------------------------------
constexpr uint32_t kSpecMaxTiles = 64 * 64;
constexpr int kSpecMiss = 1;  // spec_serve: not a read-ahead tile (render it as usual)

// Wait for a read-ahead frame's launched parts (before its buffers are reused).
int spec_drain(spt_ctx *ctx)
{
    SpecFrame &sp = ctx->spec;
    for (int p = 0; p < SpecFrame::kParts; ++p)
        if (sp.launched[p]) {
            HIP_TRY(ctx, hipEventSynchronize(sp.ev[p]));
            sp.launched[p] = false;
        }
    sp.active = false;
    return SPT_OK;
}

// The stream of read-ahead part p (created on first use).  The parts' streams take the
// least priority (SPT_READAHEAD_PRIO overrides): a priority the callers' streams do not
// use gives the parts hardware queues of their own, so a part's render does not queue
// behind another part's fold (tc = 4: 5.75-6.04 -> 5.48-5.60 ms per frame in segment mode).
int spec_stream(spt_ctx *ctx, int p)
{
    SpecFrame &sp = ctx->spec;
    BatchSet *bs = &sp.bs[p];
    if (!bs->stream) {
        int lo = 0, hi = 0;
        HIP_TRY(ctx, hipDeviceGetStreamPriorityRange(&lo, &hi));
        int prio = lo;
        if (const char *e = env_var("SPT_READAHEAD_PRIO")) prio = std::atoi(e);
        HIP_TRY(ctx, hipStreamCreateWithPriority(&bs->stream, hipStreamNonBlocking, prio));
    }
    if (!sp.ev[p]) HIP_TRY(ctx, hipEventCreateWithFlags(&sp.ev[p], hipEventDisableTiming));
    return SPT_OK;
}

// The buffers the read-ahead of a tc x tc tiling will use (its parts' streams, rectangle
// tables and sample-word workspaces, the frame's device bytes), allocated when the tiling
// arms: allocated by the first read-ahead itself, each part's first allocations held its
// launch until the previous part's render had ended (the four parts of the first read-ahead
// frame ran one after another, 15 ms apart, profiles/r05_dropin_trace.md).
// Called with lk (ctx->mu) held; waits (unlocked) for serves still copying out of d8, which
// ensure() may free when this tiling's frame is larger.
int spec_prepare(spt_ctx *ctx, std::unique_lock<std::mutex> &lk, int mode, uint32_t tc)
{
    SpecFrame &sp = ctx->spec;
    sp.readers_cv.wait(lk, [&] { return sp.readers == 0; });
    const uint32_t W = ctx->W, H = ctx->H, sw = W / tc, sh = H / tc;
    const uint32_t slot_words = mode == SPT_MODE_SEGMENT ? 1u : 2u;
    int rc = ensure(ctx, &sp.d8, &sp.d8_cap, (size_t)W * H * 3);
    if (rc) return rc;
    const uint32_t np = std::min(sp.parts, tc), rpp = (tc + np - 1) / np;
    for (uint32_t p = 0; p * rpp < tc; ++p) {
        if ((rc = spec_stream(ctx, (int)p))) return rc;
        BatchSet *bs = &sp.bs[p];
        const size_t tiles = (size_t)(std::min(tc, (p + 1) * rpp) - p * rpp) * tc;
        if (bs->h_rects_cap < tiles) {
            if ((rc = svc_end(ctx))) return rc;
            const size_t cap = std::max<size_t>(tiles, 64);
            if (bs->h_rects) HIP_TRY(ctx, hipHostFree(bs->h_rects));
            bs->h_rects = nullptr;
            bs->h_rects_cap = 0;
            HIP_TRY(ctx, hipHostMalloc((void **)&bs->h_rects, cap * sizeof(spt::BatchRect)));
            bs->h_rects_cap = cap;
        }
        if ((rc = ensure(ctx, &bs->d_rects, &bs->rects_cap, tiles))) return rc;
        Workspace *w = workspace_for(ctx, bs->stream);
        if (!w) return SPT_ERR_STATE;
        if ((rc = ensure(ctx, &w->d_samples, &w->samples_cap, tiles * sw * sh * ctx->spp * slot_words))) return rc;
    }
    return SPT_OK;
}

// Render every tile of the tc x tc tiling of `mode` (MakeRenderSegmentData order) into the
// read-ahead frame, in sp.parts batched launches.  Called with lk (ctx->mu) held; waits
// (unlocked) for the previous frame's serves still copying out of d8.
int spec_launch(spt_ctx *ctx, std::unique_lock<std::mutex> &lk, int mode, uint32_t tc)
{
    SpecFrame &sp = ctx->spec;
    sp.readers_cv.wait(lk, [&] { return sp.readers == 0; });
    int rc = spec_drain(ctx);
    if (rc) return rc;
    const uint32_t W = ctx->W, H = ctx->H, sw = W / tc, sh = H / tc;
    if ((rc = ensure(ctx, &sp.d8, &sp.d8_cap, (size_t)W * H * 3))) return rc;
    std::vector<BatchReq> reqs((size_t)tc * tc);
    for (uint32_t j = 0; j < tc; ++j)
        for (uint32_t i = 0; i < tc; ++i)
            reqs[(size_t)j * tc + i] = BatchReq{mode,    sh * j,    std::min(sh * j + sh, H), sw * i, std::min(sw * i + sw, W),
                                                nullptr, sp.d8,    SPT_OK,                   true,   false};
    const uint32_t np = std::min(sp.parts, tc), rpp = (tc + np - 1) / np;  // launches, tile rows each
    sp.rows_per_part = rpp;
    for (uint32_t p = 0; p * rpp < tc; ++p) {
        std::vector<BatchReq *> part;
        for (uint32_t j = p * rpp; j < std::min(tc, (p + 1) * rpp); ++j)
            for (uint32_t i = 0; i < tc; ++i) part.push_back(&reqs[(size_t)j * tc + i]);
        BatchSet *bs = &sp.bs[p];
        if ((rc = spec_stream(ctx, (int)p))) return rc;
        if ((rc = launch_batch(ctx, bs, part, sp.d8))) return rc;
        HIP_TRY(ctx, hipEventRecord(sp.ev[p], bs->stream));
        sp.launched[p] = true;
        ctx->batches++;
        ctx->batched_calls += part.size();
    }
    sp.active = true;
    sp.mode = mode;
    sp.tc = tc;
    sp.sw = sw;
    sp.sh = sh;
    sp.gen = ctx->gen;
    sp.served.assign((size_t)tc * tc, 0);
    return SPT_OK;
}

// A RenderSegment call with only g_data: served from the read-ahead frame when it is one
// of its tiles not yet served (starting a read-ahead at any tile of an armed tiling: the
// reference's detached RenderJob threads call the tiles in no fixed order), else
// kSpecMiss.  Called with lk (ctx->mu) held; waits unlocked.
int spec_serve(spt_ctx *ctx, std::unique_lock<std::mutex> &lk, int mode, uint32_t yB, uint32_t yE, uint32_t xB,
               uint32_t xE, uint8_t *g_data)
{
    SpecFrame &sp = ctx->spec;
    const uint32_t W = ctx->W, H = ctx->H;
    auto tile_of = [&]() -> int64_t {
        if (!sp.active || sp.mode != mode || sp.gen != ctx->gen) return -1;
        if (xB % sp.sw || yB % sp.sh || xE != xB + sp.sw || yE != yB + sp.sh) return -1;
        const uint32_t i = xB / sp.sw, j = yB / sp.sh;
        if (i >= sp.tc || j >= sp.tc) return -1;
        const size_t k = (size_t)j * sp.tc + i;
        return sp.served[k] ? -1 : (int64_t)k;
    };
    int64_t k = tile_of();
    if (k < 0) {
        // a tile of a tiling (Renderer.hpp:264-273: W / tc x H / tc tiles, tc even)?
        const uint32_t w = xE - xB, h = yE - yB, tc = W / w;
        if (!(tc >= 2 && tc % 2 == 0 && (uint64_t)tc * tc <= kSpecMaxTiles && W / tc == w && H / tc == h &&
              xB % w == 0 && yB % h == 0 && xB / w < tc && yB / h < tc &&
              batch_slot_bytes(ctx, mode, (uint64_t)w * h * tc * tc) <= ctx->ws_bytes &&
              (uint64_t)w * h * (tc * tc + tc) * ctx->spp < 0x7FFF0000ull))
            return kSpecMiss;
        if (!(sp.armed && sp.arm_mode == mode && sp.arm_tc == tc && sp.arm_w == W && sp.arm_h == H)) {
            // not armed: note the tile; the tiling arms once all its tiles have been called
            if (sp.arm_mode != mode || sp.arm_tc != tc || sp.arm_w != W || sp.arm_h != H) {
                sp.arm_mode = mode;
                sp.arm_tc = tc;
                sp.arm_w = W;
                sp.arm_h = H;
                sp.arm_seen.assign((size_t)tc * tc, 0);
                sp.arm_count = 0;
                sp.armed = false;
            }
            uint8_t &seen = sp.arm_seen[(size_t)(yB / h) * tc + xB / w];
            if (!seen) {
                seen = 1;
                sp.armed = ++sp.arm_count == tc * tc;
                // the read-ahead's buffers now, while this frame's tiles render as usual
                if (sp.armed) {
                    const int rc = spec_prepare(ctx, lk, mode, tc);
                    if (rc) return rc;
                }
            }
            return kSpecMiss;
        }
        int rc = spec_launch(ctx, lk, mode, tc);
        if (rc) return rc;
        k = tile_of();
        if (k < 0) return kSpecMiss;
    }
    sp.served[(size_t)k] = 1;
    const uint32_t part = (uint32_t)k / sp.tc / sp.rows_per_part;
    const hipEvent_t ev = sp.ev[part];
    uint8_t *const src = sp.d8;
    sp.readers++;
    lk.unlock();
    // rows y in [yB, yE) live at g_data rows H-1-y: one band, xB.. per row
    const size_t pitch = (size_t)W * 3, off = (size_t)(H - yE) * pitch + (size_t)xB * 3;
    hipError_t e = hipEventSynchronize(ev);
    if (e == hipSuccess)
        e = hipMemcpy2D(g_data + off, pitch, src + off, pitch, (size_t)(xE - xB) * 3, yE - yB, hipMemcpyDeviceToHost);
    lk.lock();
    if (--sp.readers == 0) sp.readers_cv.notify_all();
    if (e != hipSuccess) return fail(ctx, SPT_ERR_HIP, "read-ahead tile copy failed: %s", hipGetErrorString(e));
    return SPT_OK;
}

// RenderSegment / RenderSegmentTask with host outputs; with pass_spp > 0 progressively,
// copying the outputs back and calling cb after every pass.  The context lock is held
// only while launches are enqueued: each call renders on its own slot (stream,
// workspace, staging), waits for its stream unlocked, so concurrent callers -- the
// reference's RenderJob threads -- overlap on the GPU; cb runs unlocked too.
// spread: a multi-device context sends the call to its least busy member (else member 0).
int render_segment_host(spt_ctx *ctx, int mode, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *rgba,
                        uint8_t *g_data, uint32_t pass_spp = 0, spt_progress_fn cb = nullptr, void *user = nullptr,
                        bool spread = true)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    const bool single = ctx->peers.empty();
    if (spread && !ctx->peers.empty()) ctx = pick_member(ctx);  // tiles go to the least busy device
    std::unique_lock<std::mutex> lk(ctx->mu);
    int rc = check_ready(ctx);
    if (rc) return rc;
    if ((rc = check_region(ctx, yB, yE, xB, xE))) return rc;
    if (yB >= yE || xB >= xE) return SPT_OK;  // the reference's loops do nothing
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    // the reference's tiling, g_data only: from the read-ahead frame (SpecFrame)
    if (pass_spp == 0 && single && ctx->readahead && ctx->batching && !rgba && g_data &&
        ctx->engine == SPT_ENGINE_MEGAKERNEL) {
        ctx->inflight.fetch_add(1);
        rc = spec_serve(ctx, lk, mode, yB, yE, xB, xE, g_data);
        ctx->inflight.fetch_sub(1);
        if (rc != kSpecMiss) return rc;
    }
    // one-shot calls join a batch unless one call's samples exceed the workspace (then
    // it renders alone, in sample batches)
    if (pass_spp == 0 && ctx->batching && ctx->engine == SPT_ENGINE_MEGAKERNEL &&
        batch_slot_bytes(ctx, mode, (uint64_t)(xE - xB) * (yE - yB)) <= ctx->ws_bytes &&
        (uint64_t)(xE - xB) * (yE - yB) * ctx->spp < 0x7FFF0000ull) {
        ctx->inflight.fetch_add(1);
        rc = render_batched(ctx, lk, mode, yB, yE, xB, xE, rgba, g_data);
        ctx->inflight.fetch_sub(1);
        return rc;
    }
    HostSlot *hs = acquire_slot(ctx, lk);
    if (!hs) return SPT_ERR_HIP;
    ctx->inflight.fetch_add(1);
    struct Release {
        spt_ctx *c;
        HostSlot *h;
        ~Release()
        {
            c->inflight.fetch_sub(1);
            release_slot(c, h);
        }
    } release{ctx, hs};  // runs with lk held (declared after it)
    const uint32_t w = xE - xB, h = yE - yB;
    const size_t npix = (size_t)w * h;
    if ((rc = ensure(ctx, &hs->d_stage, &hs->stage_cap, npix))) return rc;
    uint8_t *d8 = nullptr;
    if (g_data) {
        if ((rc = ensure(ctx, &ctx->d_frame8, &ctx->frame8_cap, (size_t)ctx->W * ctx->H * 3))) return rc;
        d8 = ctx->d_frame8;
    }
    const uint32_t W = ctx->W, H = ctx->H;
    spt::RowMap map{yB, yE, 1u, 1u, 0u, xB, w};
    // enqueue the copy-back of the outputs, then wait for the slot's stream unlocked
    auto copy_out_and_wait = [&]() -> int {
        if (rgba)
            HIP_TRY(ctx, hipMemcpyAsync(rgba, hs->d_stage, npix * sizeof(float4), hipMemcpyDeviceToHost, hs->stream));
        if (g_data) {
            // rows y in [yB, yE) live at g_data rows H-1-y: one contiguous band, xB.. per row
            const size_t pitch = (size_t)W * 3;
            const size_t off = (size_t)(H - yE) * pitch + (size_t)xB * 3;
            HIP_TRY(ctx, hipMemcpy2DAsync(g_data + off, pitch, d8 + off, pitch, (size_t)w * 3, h,
                                          hipMemcpyDeviceToHost, hs->stream));
        }
        lk.unlock();
        const hipError_t e = hipStreamSynchronize(hs->stream);
        lk.lock();
        if (e != hipSuccess) return fail(ctx, SPT_ERR_HIP, "hipStreamSynchronize failed: %s", hipGetErrorString(e));
        return SPT_OK;
    };
    // concurrent callers (RenderJob threads) share the GPU side by side: with k slots in
    // use each launch gets 2/k of the grid, so launches overlap and no single launch's
    // tail idles the device (config 2 through the C++ shim, Msamples/s, grid divisor
    // 1 / k/2 / k: tc = 4: 7 923 / 8 715 / 7 417; tc = 8: 4 117 / 6 303 / 5 769)
    const uint32_t div = ctx->host_grid_div ? ctx->host_grid_div : std::max<uint32_t>(1u, (uint32_t)ctx->slots.size() / 2u);
    if (pass_spp == 0) {
        if ((rc = render_impl(ctx, mode, map, hs->d_stage, d8, hs->stream, false, nullptr, div))) return rc;
    } else {
        Progress pg{pass_spp, [&](uint32_t done) -> int {
                        const int r = copy_out_and_wait();
                        if (r) return -r;
                        if (!cb) return 0;
                        lk.unlock();
                        t_in_callback = ctx;
                        const int stop = cb(user, done);
                        t_in_callback = nullptr;
                        lk.lock();
                        return stop != 0 ? 1 : 0;
                    }};
        rc = render_impl(ctx, mode, map, hs->d_stage, d8, hs->stream, false, &pg, div);
        if (rc) return rc < 0 ? -rc : rc;
    }
    if ((rc = copy_out_and_wait())) return rc;
    return collect_timings(ctx, false);
}

// Setters must not run from a progress callback of the same context (the render in
// progress reads the state they change).
int check_not_in_callback(spt_ctx *ctx)
{
    if (t_in_callback == ctx) return fail(ctx, SPT_ERR_STATE, "called from a progress callback of this context");
    return SPT_OK;
}

// Rows per strip of the multi-device frame split: the largest of 8, 4, 2, 1 that deals
// the frame's strips evenly over the members, else 8 (simplepathtracer_amd/distributed.py
// even_strip, the same rule as the one-process-per-GPU path).
uint32_t even_strip(uint32_t height, uint32_t parts)
{
    for (uint32_t s : {8u, 4u, 2u, 1u})
        if (height % s == 0 && (height / s) % parts == 0) return s;
    return 8u;
}

// Apply a setter to the context and every member device of a multi-device context.
template <class F>
int for_members(spt_ctx *ctx, F &&f)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    int rc = check_not_in_callback(ctx);
    if (rc) return rc;
    if ((rc = f(ctx))) return rc;
    for (spt_ctx *p : ctx->peers)
        if ((rc = f(p))) return fail(ctx, rc, "member device %d: %s", p->device, p->err.c_str());
    return SPT_OK;
}

// Setters of one context; the exported setters apply them to every member device.
int spt_set_scene_one(spt_ctx *ctx, const float *centers4, const float *radii, const float *colors4,
                  const uint8_t *materials, const float *fuzz, uint32_t n)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (int rc_ = svc_end(ctx)) return rc_;  // the session holds the state this setter changes
    ctx->gen++;                              // a read-ahead frame of the old state is stale
    if (n > 0 && (!centers4 || !radii || !colors4 || !materials || !fuzz))
        return fail(ctx, SPT_ERR_ARG, "null scene array");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    std::vector<float4> shade(n);
    std::vector<uint32_t> mat(n);
    for (uint32_t i = 0; i < n; ++i) {
        shade[i] = make_float4(colors4[4 * i], colors4[4 * i + 1], colors4[4 * i + 2], fuzz[i]);
        mat[i] = materials[i];
    }
    ctx->h_shade = std::move(shade);
    ctx->h_mat = std::move(mat);
    ctx->h_centers.assign(centers4, centers4 + 4 * (size_t)n);
    ctx->h_radii.assign(radii, radii + n);
    ctx->n = n;
    int rc = rebuild_accel(ctx);
    if (rc) return rc;
    ctx->scene_set = true;
    return rebuild_prim(ctx);
}

int spt_set_camera_one(spt_ctx *ctx, const float view[16], const float eye[4], const float sky[4])
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (int rc_ = svc_end(ctx)) return rc_;  // the session holds the state this setter changes
    ctx->gen++;                              // a read-ahead frame of the old state is stale
    if (!view || !eye || !sky) return fail(ctx, SPT_ERR_ARG, "null camera array");
    for (int j = 12; j < 16; ++j)
        if (view[j] != 0.0f)
            return fail(ctx, SPT_ERR_ARG, "viewMatrix row 3 must be zero (CreateCameraBasisMatrix, Math.hpp:204-208)");
    for (int j = 0; j < 12; ++j) ctx->cam.view[j] = view[j];
    for (int j = 0; j < 3; ++j) {
        ctx->cam.eye[j] = eye[j];
        ctx->cam.sky[j] = sky[j];
    }
    ctx->cam_set = true;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return rebuild_prim(ctx);
}

int spt_set_params_one(spt_ctx *ctx, uint32_t width, uint32_t height, uint32_t spp, uint32_t bounces, uint64_t seed)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (int rc_ = svc_end(ctx)) return rc_;  // the session holds the state this setter changes
    ctx->gen++;                              // a read-ahead frame of the old state is stale
    if (width == 0 || height == 0) return fail(ctx, SPT_ERR_ARG, "empty frame %ux%u", width, height);
    if ((uint64_t)width * height * 3 > 0xFFFFFFFFull)
        return fail(ctx, SPT_ERR_ARG, "frame %ux%u overflows the reference's uint32 g_size", width, height);
    if (spp == 0) return fail(ctx, SPT_ERR_ARG, "spp must be >= 1 (1.f/0 samples)");
    if (bounces == 0) return fail(ctx, SPT_ERR_ARG, "bounces must be >= 1 (--bounceCount never reaches 0)");
    ctx->W = width;
    ctx->H = height;
    ctx->spp = spp;
    ctx->bounces = bounces;
    ctx->seed = seed;
    ctx->params_set = true;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return rebuild_prim(ctx);
}

int spt_set_cluster_size_one(spt_ctx *ctx, uint32_t k)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (int rc_ = svc_end(ctx)) return rc_;  // the session holds the state this setter changes
    ctx->gen++;                              // a read-ahead frame of the old state is stale
    if (k > spt::kClusterSlots && k != SPT_CLUSTER_AUTO)
        return fail(ctx, SPT_ERR_ARG, "cluster size %u > %u", k, spt::kClusterSlots);
    ctx->cluster_k = k;
    if (!ctx->scene_set) return SPT_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int rc = rebuild_accel(ctx);
    return rc ? rc : rebuild_prim(ctx);
}

int spt_set_cluster_tree_one(spt_ctx *ctx, uint32_t branching)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (int rc_ = svc_end(ctx)) return rc_;  // the session holds the state this setter changes
    ctx->gen++;                              // a read-ahead frame of the old state is stale
    if (branching == 1 || (branching > 64 && branching != SPT_TREE_AUTO))
        return fail(ctx, SPT_ERR_ARG, "tree branching %u not in {0, 2..64, SPT_TREE_AUTO}", branching);
    ctx->tree_branching = branching;
    if (!ctx->scene_set) return SPT_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int rc = rebuild_accel(ctx);
    return rc ? rc : rebuild_prim(ctx);
}

int spt_set_engine_one(spt_ctx *ctx, int engine)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (int rc_ = svc_end(ctx)) return rc_;  // the session holds the state this setter changes
    ctx->gen++;                              // a read-ahead frame of the old state is stale
    if (engine != SPT_ENGINE_MEGAKERNEL && engine != SPT_ENGINE_WAVEFRONT)
        return fail(ctx, SPT_ERR_ARG, "unknown engine %d", engine);
    ctx->engine = engine;
    return SPT_OK;
}

int spt_set_workspace_one(spt_ctx *ctx, uint64_t bytes)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (int rc_ = svc_end(ctx)) return rc_;  // the session holds the state this setter changes
    ctx->gen++;                              // a read-ahead frame of the old state is stale
    if (bytes < sizeof(float4)) return fail(ctx, SPT_ERR_ARG, "workspace too small");
    ctx->ws_bytes = bytes;
    return SPT_OK;
}

}  // namespace

extern "C" {

int spt_abi_version(void) { return SPT_ABI_VERSION; }

int spt_device_count(int *count)
{
    if (!count) return fail(nullptr, SPT_ERR_ARG, "null count");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *count = c;
    return SPT_OK;
}

int spt_ctx_create(int device, spt_ctx **out)
{
    if (!out) return fail(nullptr, SPT_ERR_ARG, "null out");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(nullptr, SPT_ERR_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= count) return fail(nullptr, SPT_ERR_NODEVICE, "device %d out of range (%d)", device, count);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return fail(nullptr, SPT_ERR_NODEVICE, "hipGetDeviceProperties(%d) failed", device);
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, SPT_ERR_NODEVICE, "device %d is %s, this build targets gfx950", device, prop.gcnArchName);
    spt_ctx *ctx = new spt_ctx();
    ctx->ws.reserve(kMaxWorkspaces);
    ctx->masked.reserve(kMaxCompanions);  // masked_for hands out pointers into it
    ctx->block = spt::render_block_size();
    ctx->device = device;
    ctx->num_cu = prop.multiProcessorCount;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return fail(nullptr, SPT_ERR_HIP, "stream creation failed on device %d", device);
    }
    int per_cu = 0;
    if (spt::render_occupancy(ctx->block, &per_cu) != hipSuccess || per_cu <= 0) per_cu = 1;
    ctx->svc_grid = (uint32_t)(std::max(1, per_cu - 1) * ctx->num_cu);
    // SPT_SVC_FULL_GRID=1: the session takes every block slot (folds and other streams'
    // kernels then wait for the session's end; for pipelines that end their sessions
    // themselves, like bench.py's timed regions: DESIGN.md §5)
    if (const char *e = env_var("SPT_SVC_FULL_GRID"))
        if (std::atoi(e) != 0) ctx->svc_grid = (uint32_t)(per_cu * ctx->num_cu);
    // launch_bounds / occupancy API may over-report by one block per CU for SGPR-heavy
    // kernels (MI355X_MICROARCH.md, Residency): the kernel needs no co-residency, so
    // extra blocks only queue.  SPT_BLOCKS_PER_CU overrides for tuning.
    if (const char *e = env_var("SPT_BLOCKS_PER_CU")) per_cu = std::max(1, std::atoi(e));
    if (const char *e = env_var("SPT_CLAIM")) ctx->claim = (uint32_t)std::max(0, std::atoi(e));  // 0 = per launch
    if (const char *e = env_var("SPT_CLUSTER_K")) ctx->cluster_k = (uint32_t)std::max(0, std::atoi(e));
    if (const char *e = env_var("SPT_TREE_B")) ctx->tree_branching = (uint32_t)std::max(0, std::atoi(e));
    if (const char *e = env_var("SPT_CLAIMS_PER_WAVE")) ctx->claims_per_wave = (uint32_t)std::max(1, std::atoi(e));
    if (const char *e = env_var("SPT_QUEUES"))
        ctx->queues = (uint32_t)std::min<int>((int)spt::kMaxQueues, std::max(1, std::atoi(e)));
    if (const char *e = env_var("SPT_WF_CAP")) ctx->wf_cap = (uint32_t)std::max(1024, std::atoi(e));
    if (const char *e = env_var("SPT_WF_QUEUE")) ctx->wf_queue = (uint32_t)std::min(8192, std::max(1, std::atoi(e) / 256)) * 256u;
    if (const char *e = env_var("SPT_HOST_GRID_DIV")) ctx->host_grid_div = (uint32_t)std::max(0, std::atoi(e));
    if (const char *e = env_var("SPT_BATCH")) ctx->batching = std::atoi(e) != 0;
    if (const char *e = env_var("SPT_READAHEAD")) ctx->readahead = std::atoi(e) != 0;
    if (const char *e = env_var("SPT_READAHEAD_PARTS"))
        ctx->spec.parts = (uint32_t)std::min(SpecFrame::kParts, std::max(1, std::atoi(e)));
    if (const char *e = env_var("SPT_BATCH_DBUF")) ctx->batch_dbuf = std::atoi(e) != 0;
    if (const char *e = env_var("SPT_BATCH_GRID_DIV")) ctx->batch_grid_div = (uint32_t)std::max(1, std::atoi(e));
    if (const char *e = env_var("SPT_BATCH_SETS"))
        ctx->batch_sets = (uint32_t)std::min<int>((int)kMaxBatchSets, std::max(1, std::atoi(e)));
    if (const char *e = env_var("SPT_HOST_SLOTS"))
        ctx->host_slots = (uint32_t)std::min<int>((int)kMaxHostSlots, std::max(1, std::atoi(e)));
    // SPT_SERVICE=1: the context starts with the render service on (spt_service_start)
    if (const char *e = env_var("SPT_SERVICE")) ctx->svc.enabled = std::atoi(e) != 0;
    if (const char *e = env_var("SPT_SVC_CLAIM")) ctx->svc.claim = (uint32_t)std::max(64, std::atoi(e) / 64 * 64);
    if (const char *e = env_var("SPT_SVC_QUEUES"))
        ctx->svc.queues = (uint32_t)std::min<int>((int)spt::kMaxQueues, std::max(1, std::atoi(e)));
    if (const char *e = env_var("SPT_SVC_RING_MB")) {
        ctx->svc.ring_bytes = (uint64_t)std::max(64, std::atoi(e)) << 20;
        ctx->svc.ring_set = true;
    }
    // CUs kept free of launched renders (spt_set_reserved_cus)
    if (const char *e = env_var("SPT_RESERVE_CUS"))
        ctx->reserve_cus = (uint32_t)std::min(std::max(0, std::atoi(e)), std::max(0, ctx->num_cu - 1));
    // a fraction of the session grid (rehearsing several ranks' sessions on one GPU), the
    // bound on waiting for a session to end, and the publish-delay fault injection of the
    // liveness tests (tests/test_gpu_service.py)
    if (const char *e = env_var("SPT_PRIM_LISTS")) ctx->prim_enabled = std::atoi(e) != 0;
    if (const char *e = env_var("SPT_PRIM_MAX")) ctx->prim_max = (uint32_t)std::max(0, std::atoi(e));
    if (const char *e = env_var("SPT_SVC_GRID_DIV")) ctx->svc.grid_div = (uint32_t)std::max(1, std::atoi(e));
    if (const char *e = env_var("SPT_SVC_TIMEOUT_MS")) ctx->svc.timeout_ms = std::max(1.0, std::atof(e));
    if (const char *e = env_var("SPT_SVC_DEBUG")) ctx->svc.debug = std::atoi(e) != 0;
    if (const char *e = env_var("SPT_SVC_TEST_PUB_DELAY_US"))
        ctx->svc.pub_delay_us = (uint32_t)std::min(5000000, std::max(0, std::atoi(e)));
    ctx->grid = (uint32_t)(per_cu * ctx->num_cu);
    ctx->grid_overlap = env_var("SPT_BLOCKS_PER_CU") || per_cu < 2 ? ctx->grid : (uint32_t)((per_cu - 1) * ctx->num_cu);
    ctx->grid_small = env_var("SPT_BLOCKS_PER_CU") || per_cu < 3 ? 0u : (uint32_t)((per_cu - 2) * ctx->num_cu);
    if (const char *e = env_var("SPT_SMALL_GRID")) ctx->grid_small = std::atoi(e) != 0 ? ctx->grid_small : 0u;
    if (hipEventCreate(&ctx->ref_ev) != hipSuccess || hipEventCreateWithFlags(&ctx->frame_ev, hipEventDisableTiming) != hipSuccess ||
        hipMalloc((void **)&ctx->d_counters, kCounters * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(ctx->d_counters, 0, kCounters * sizeof(unsigned long long)) != hipSuccess) {
        spt_ctx_destroy(ctx);
        return fail(nullptr, SPT_ERR_NOMEM, "workspace allocation failed");
    }
    *out = ctx;
    return SPT_OK;
}

int spt_ctx_create_multi(const int *devices, uint32_t n, spt_ctx **out)
{
    if (!out) return fail(nullptr, SPT_ERR_ARG, "null out");
    *out = nullptr;
    if (!devices || n == 0) return fail(nullptr, SPT_ERR_ARG, "empty device list");
    spt_ctx *ctx = nullptr;
    int rc = spt_ctx_create(devices[0], &ctx);
    if (rc) return rc;
    for (uint32_t i = 1; i < n; ++i) {
        spt_ctx *p = nullptr;
        if ((rc = spt_ctx_create(devices[i], &p))) {
            const std::string why = g_thread_error;
            spt_ctx_destroy(ctx);
            return fail(nullptr, rc, "member %u (device %d): %s", i, devices[i], why.c_str());
        }
        ctx->peers.push_back(p);
        // member 0 pulls the members' strips over xGMI (hipMemcpyPeerAsync)
        if (devices[i] != devices[0]) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devices[0], devices[i]) == hipSuccess && can) {
                (void)hipSetDevice(devices[0]);
                const hipError_t e = hipDeviceEnablePeerAccess(devices[i], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                    spt_ctx_destroy(ctx);
                    return fail(nullptr, SPT_ERR_HIP, "peer access %d -> %d: %s", devices[0], devices[i],
                                hipGetErrorString(e));
                }
                (void)hipGetLastError();
            }
        }
    }
    *out = ctx;
    return SPT_OK;
}

int spt_ctx_devices(spt_ctx *ctx, uint32_t *n, int *devices)
{
    if (!ctx || !n) return fail(ctx, SPT_ERR_ARG, "null argument");
    const uint32_t cap = *n;
    *n = 1u + (uint32_t)ctx->peers.size();
    if (devices) {
        if (cap >= 1) devices[0] = ctx->device;
        for (uint32_t i = 1; i < *n && i < cap; ++i) devices[i] = ctx->peers[i - 1]->device;
    }
    return SPT_OK;
}

void spt_ctx_destroy(spt_ctx *ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)svc_end(ctx);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto *vec : {&ctx->pending_render, &ctx->pending_fold, &ctx->pool})
        for (EventPair &p : *vec) {
            (void)hipEventDestroy(p.a);
            (void)hipEventDestroy(p.b);
        }
    (void)hipDeviceSynchronize();  // async renders on caller streams
    for (const spt_ctx::Pinned &p : ctx->pinned)
        if (p.owner) (void)hipHostUnregister(p.ptr);
    if (ctx->ref_ev) (void)hipEventDestroy(ctx->ref_ev);
    void *bufs[] = {ctx->d_shade, ctx->d_mat, ctx->d_slots, ctx->d_orig, ctx->d_nodes,
                    ctx->d_kpre, ctx->d_counters, ctx->d_frame8, ctx->d_prim_b8, ctx->d_prim_b4,
                    ctx->d_prim_slots};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (Workspace &w : ctx->ws) {
        const spt::WavefrontBuffers &q = w.wf;
        for (void *b : {(void *)w.d_samples, (void *)w.d_acc, (void *)w.d_head, (void *)q.o, (void *)q.d, (void *)q.m,
                        (void *)q.state})
            if (b) (void)hipFree(b);
    }
    for (HostSlot *h : ctx->slots) {
        if (h->d_stage) (void)hipFree(h->d_stage);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        delete h;
    }
    for (BatchSet &b : ctx->spec.bs) {
        if (b.d_rects) (void)hipFree(b.d_rects);
        if (b.h_rects) (void)hipHostFree(b.h_rects);
        if (b.d_stage) (void)hipFree(b.d_stage);
        if (b.stream) (void)hipStreamDestroy(b.stream);
    }
    for (hipEvent_t e : ctx->spec.ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->spec.d8) (void)hipFree(ctx->spec.d8);
    for (BatchSet &b : ctx->bsets) {
        if (b.d_rects) (void)hipFree(b.d_rects);
        if (b.h_rects) (void)hipHostFree(b.h_rects);
        if (b.d_stage) (void)hipFree(b.d_stage);
        if (b.stream) (void)hipStreamDestroy(b.stream);
    }
    for (void *b : {(void *)ctx->d_tile, (void *)ctx->d_fullframe})
        if (b) (void)hipFree(b);
    if (ctx->frame_ev) (void)hipEventDestroy(ctx->frame_ev);
    for (const auto &c : ctx->companions) (void)hipStreamDestroy(c.second);
    for (const spt_ctx::Masked &m : ctx->masked) {
        (void)hipStreamDestroy(m.stream);
        (void)hipEventDestroy(m.go);
        (void)hipEventDestroy(m.done);
    }
    for (hipEvent_t e : {ctx->dbuf_start, ctx->dbuf_fold})
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    {
        Service &v = ctx->svc;
        for (void *b : {(void *)v.d_ctl, (void *)v.d_jobs, (void *)v.d_job_claim, (void *)v.d_done, (void *)v.d_ring})
            if (b) (void)hipFree(b);
        for (const SvcInflight &e : v.inflight) (void)hipEventDestroy(e.ev);
        for (hipEvent_t e : v.ev_pool) (void)hipEventDestroy(e);
        for (hipEvent_t e : {v.ev_start, v.ev_end, v.ev_ctl})
            if (e) (void)hipEventDestroy(e);
        if (v.stream) (void)hipStreamDestroy(v.stream);
        for (void *h : {(void *)v.h_host, (void *)v.h_jobs, (void *)v.h_job_claim})
            if (h) (void)hipHostFree(h);
    }
    for (spt_ctx *p : ctx->peers) spt_ctx_destroy(p);
    delete ctx;
}

const char *spt_last_error(const spt_ctx *ctx)
{
    if (ctx) return ctx->err.c_str();
    return g_thread_error.c_str();
}

int spt_set_scene(spt_ctx *ctx, const float *centers4, const float *radii, const float *colors4,
                  const uint8_t *materials, const float *fuzz, uint32_t n)
{
    return for_members(ctx, [&](spt_ctx *c) { return spt_set_scene_one(c, centers4, radii, colors4, materials, fuzz, n); });
}

int spt_set_camera(spt_ctx *ctx, const float view[16], const float eye[4], const float sky[4])
{
    return for_members(ctx, [&](spt_ctx *c) { return spt_set_camera_one(c, view, eye, sky); });
}

int spt_set_params(spt_ctx *ctx, uint32_t width, uint32_t height, uint32_t spp, uint32_t bounces, uint64_t seed)
{
    return for_members(ctx, [&](spt_ctx *c) { return spt_set_params_one(c, width, height, spp, bounces, seed); });
}

int spt_set_cluster_size(spt_ctx *ctx, uint32_t k)
{
    return for_members(ctx, [&](spt_ctx *c) { return spt_set_cluster_size_one(c, k); });
}

int spt_set_cluster_tree(spt_ctx *ctx, uint32_t branching)
{
    return for_members(ctx, [&](spt_ctx *c) { return spt_set_cluster_tree_one(c, branching); });
}

int spt_set_reserved_cus(spt_ctx *ctx, uint32_t n)
{
    return for_members(ctx, [&](spt_ctx *c) -> int {
        std::lock_guard<std::mutex> lk(c->mu);
        if (c->num_cu > 0 && n >= (uint32_t)c->num_cu)
            return fail(c, SPT_ERR_ARG, "%u reserved CUs of %d", n, c->num_cu);
        if (n != c->reserve_cus) {
            // streams masked for the old count: retired once their work is done
            if (int rc = svc_end(c)) return rc;
            HIP_TRY(c, hipDeviceSynchronize());
            for (const spt_ctx::Masked &m : c->masked) {
                (void)hipStreamDestroy(m.stream);
                (void)hipEventDestroy(m.go);
                (void)hipEventDestroy(m.done);
            }
            c->masked.clear();
        }
        c->reserve_cus = n;
        return SPT_OK;
    });
}

int spt_accel_check(const float *centers4, const float *radii, uint32_t n, uint32_t cluster_k, uint32_t branching,
                    uint32_t *out_nodes)
{
    if (n > 0 && (!centers4 || !radii)) return fail(nullptr, SPT_ERR_ARG, "null scene array");
    if (cluster_k > spt::kClusterSlots) return fail(nullptr, SPT_ERR_ARG, "cluster size %u > %u", cluster_k, spt::kClusterSlots);
    if (branching == 1) return fail(nullptr, SPT_ERR_ARG, "tree branching 1");
    const uint32_t k = cluster_k == 0 ? 0u : cluster_k;
    const uint32_t leaf = branching == 0 && k <= spt::kFlatLeafSlots ? spt::kFlatLeafSlots : spt::kClusterSlots;
    const spt::AccelTables t = spt::build_accel(centers4, radii, n, k, spt::render_group_size(), branching, leaf);
    const std::string bad = spt::validate_accel(t, centers4, radii, n);
    if (!bad.empty()) return fail(nullptr, SPT_ERR_STATE, "traversal tables invalid: %s", bad.c_str());
    if (out_nodes) *out_nodes = t.n_nodes;
    return SPT_OK;
}

int spt_prim_lists_check(const float *centers4, const float *radii, uint32_t n, const float view[16], const float eye[4],
                         uint32_t width, uint32_t height, uint32_t max_count, uint32_t *blocks8, uint32_t *blocks4,
                         uint32_t *slot_ids, uint32_t *slot_orig, uint32_t cap, uint32_t *counts)
{
    if (n > 0 && (!centers4 || !radii)) return fail(nullptr, SPT_ERR_ARG, "null scene array");
    if (!view || !eye || !counts || width == 0 || height == 0) return fail(nullptr, SPT_ERR_ARG, "bad arguments");
    // the default traversal shape (resolve_shape with both settings on auto)
    const uint32_t branching = n > 512 ? 3u : 4u;
    const spt::AccelTables t =
        spt::build_accel(centers4, radii, n, spt::kClusterSlots, spt::render_group_size(), branching, spt::kClusterSlots);
    spt::Camera cam{};
    for (int j = 0; j < 12; ++j) cam.view[j] = view[j];
    for (int j = 0; j < 3; ++j) cam.eye[j] = eye[j];
    const spt::PrimListTables pl = spt::build_prim_lists(t, cam, width, height, max_count);
    counts[0] = (uint32_t)pl.slots.size();
    counts[1] = (uint32_t)t.slots.size();
    counts[2] = pl.bw;
    counts[3] = pl.on ? 1u : 0u;
    if ((slot_ids && cap < pl.slots.size()) || (slot_orig && cap < t.slots.size()))
        return fail(nullptr, SPT_ERR_ARG, "capacity %u < %zu list entries / %zu slots", cap, pl.slots.size(), t.slots.size());
    for (size_t i = 0; blocks8 && i < pl.b8.size(); ++i) {
        blocks8[2 * i] = pl.b8[i].x;
        blocks8[2 * i + 1] = pl.b8[i].y;
    }
    for (size_t i = 0; blocks4 && i < pl.b4.size(); ++i) {
        blocks4[2 * i] = pl.b4[i].x;
        blocks4[2 * i + 1] = pl.b4[i].y;
    }
    if (slot_ids) std::copy(pl.slots.begin(), pl.slots.end(), slot_ids);
    if (slot_orig) std::copy(t.orig.begin(), t.orig.end(), slot_orig);
    return SPT_OK;
}

int spt_set_engine(spt_ctx *ctx, int engine)
{
    return for_members(ctx, [&](spt_ctx *c) { return spt_set_engine_one(c, engine); });
}

int spt_set_workspace(spt_ctx *ctx, uint64_t bytes)
{
    return for_members(ctx, [&](spt_ctx *c) { return spt_set_workspace_one(c, bytes); });
}

int spt_render_segment(spt_ctx *ctx, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *rgba, uint8_t *g_data)
{
    return render_segment_host(ctx, SPT_MODE_SEGMENT, yB, yE, xB, xE, rgba, g_data);
}

int spt_render_segment_task(spt_ctx *ctx, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *rgba,
                            uint8_t *g_data)
{
    return render_segment_host(ctx, SPT_MODE_TASK, yB, yE, xB, xE, rgba, g_data);
}

int spt_pin_host(spt_ctx *ctx, void *ptr, size_t bytes)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    if (!ptr || bytes == 0) return fail(ctx, SPT_ERR_ARG, "null or empty host buffer");
    std::lock_guard<std::mutex> plk(ctx->pin_mu);
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        for (const spt_ctx::Pinned &p : ctx->pinned)
            if (p.ptr == ptr) return SPT_OK;
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        // portable: every member device of a multi-device context writes its tiles' bytes
        // into the buffer in place (none copies them back over the others' writes)
        HIP_TRY(ctx, hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
        void *dev = nullptr;
        if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess) dev = nullptr;
        ctx->pinned.push_back(spt_ctx::Pinned{ptr, bytes, (uint8_t *)dev, true});
    }
    for (spt_ctx *m : ctx->peers) {
        std::lock_guard<std::mutex> lk(m->mu);
        HIP_TRY(ctx, hipSetDevice(m->device));
        void *dev = nullptr;
        if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess) dev = nullptr;
        m->pinned.push_back(spt_ctx::Pinned{ptr, bytes, (uint8_t *)dev, false});
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return SPT_OK;
}

int spt_unpin_host(spt_ctx *ctx, void *ptr)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    auto find = [&](spt_ctx *c) {
        return std::find_if(c->pinned.begin(), c->pinned.end(), [&](const spt_ctx::Pinned &p) { return p.ptr == ptr; });
    };
    std::lock_guard<std::mutex> plk(ctx->pin_mu);
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (find(ctx) == ctx->pinned.end() || !find(ctx)->owner)
            return fail(ctx, SPT_ERR_ARG, "buffer %p was not pinned", ptr);
    }
    // batched calls of any member may be writing into it directly
    for (spt_ctx *m : ctx->peers) {
        std::lock_guard<std::mutex> lk(m->mu);
        HIP_TRY(ctx, hipSetDevice(m->device));
        if (svc_end(m)) return fail(ctx, SPT_ERR_HIP, "member device %d: %s", m->device, m->err.c_str());
        HIP_TRY(ctx, hipDeviceSynchronize());
        auto it = find(m);
        if (it != m->pinned.end()) m->pinned.erase(it);
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (int rc = svc_end(ctx)) return rc;
    HIP_TRY(ctx, hipDeviceSynchronize());
    const auto it = find(ctx);
    if (it == ctx->pinned.end() || !it->owner) return fail(ctx, SPT_ERR_ARG, "buffer %p was not pinned", ptr);
    HIP_TRY(ctx, hipHostUnregister(ptr));
    ctx->pinned.erase(it);
    return SPT_OK;
}

int spt_render_progressive(spt_ctx *ctx, int mode, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE,
                           uint32_t pass_spp, float *rgba, uint8_t *g_data, spt_progress_fn cb, void *user)
{
    if (mode != SPT_MODE_SEGMENT && mode != SPT_MODE_TASK) return fail(ctx, SPT_ERR_ARG, "bad mode %d", mode);
    if (pass_spp == 0) return fail(ctx, SPT_ERR_ARG, "pass_spp must be >= 1");
    return render_segment_host(ctx, mode, yB, yE, xB, xE, rgba, g_data, pass_spp, cb, user);
}

int spt_render_frame(spt_ctx *ctx, int mode, float *rgba_out, uint8_t *g_data)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    if (mode != SPT_MODE_SEGMENT && mode != SPT_MODE_TASK) return fail(ctx, SPT_ERR_ARG, "bad mode %d", mode);
    {
        std::unique_lock<std::mutex> lk(ctx->mu);
        int rc = check_ready(ctx);
        if (rc) return rc;
        const uint32_t W = ctx->W, H = ctx->H;
        if (ctx->peers.empty()) {
            lk.unlock();
            return render_segment_host(ctx, mode, 0, H, 0, W, rgba_out, g_data, 0, nullptr, nullptr, false);
        }
    }
    // every member renders its interleaved row strips into a compact tile; member 0
    // pulls the tiles over xGMI (peer copies ordered after each member's render by an
    // event), scatters them into the frame (assemble_kernel) and copies the frame back.
    // RenderImage's RenderSegmentTask({0, H, 0, W}) on a non-square frame aliases pixels
    // across rows (colorIndex = dx + dy * H, TaskBasedPathTracer.hpp:103,186,196-205), so
    // a strip split cannot resolve it locally: there member r owns a colorIndex range
    // [i0_r, i1_r), renders the rows holding its sources (every row whose pixels map into
    // the range: about (i1_r - i0_r) / H + W / H rows) and folds the range; the ranges are
    // the frame's pixels in row-major order, so member 0 places them end to end.  Only
    // outputs up to p_max = (W - 1) + (H - 1) H have sources (the rest resolve to NaN
    // without any render), so the source-holding outputs are dealt evenly and the
    // last member also takes the source-less tail: every member renders about the same
    // number of rows (an even split of all W H outputs left members idle: 2 of 8 on a
    // 1200 x 800 frame, all but member 0 when W is about 10 H).
    std::vector<spt_ctx *> m{ctx};
    m.insert(m.end(), ctx->peers.begin(), ctx->peers.end());
    const uint32_t parts = (uint32_t)m.size();
    std::vector<std::unique_lock<std::mutex>> locks;
    for (spt_ctx *c : m) {
        locks.emplace_back(c->mu);
        int rc = check_ready(c);
        if (rc) return c == ctx ? rc : fail(ctx, rc, "member device %d: %s", c->device, c->err.c_str());
        if (c->W != ctx->W || c->H != ctx->H) return fail(ctx, SPT_ERR_STATE, "members disagree on the frame size");
    }
    const uint32_t W = ctx->W, H = ctx->H;
    const uint32_t strip = even_strip(H, parts);
    const bool alias = mode == SPT_MODE_TASK && W != H;
    const uint64_t total = (uint64_t)W * H;
    // alias: outputs [0, n_src) have sources (p_max + 1 = W + (H - 1) H, at most W H)
    const uint64_t n_src = std::min<uint64_t>(total, (uint64_t)W + (uint64_t)(H - 1u) * H);
    const uint64_t L = (n_src + parts - 1) / parts;  // source-holding outputs per member (alias)
    uint32_t max_rows = 0;
    for (uint32_t r = 0; r < parts; ++r) max_rows = std::max(max_rows, spt::rows_owned(spt::RowMap{0, H, strip, parts, r, 0, W}));
    auto range_of = [&](uint32_t r) {
        const uint64_t i0 = std::min<uint64_t>((uint64_t)r * L, n_src);
        const uint64_t i1 = r + 1 == parts ? total : std::min<uint64_t>(i0 + L, n_src);
        return std::make_pair((uint32_t)i0, (uint32_t)i1);
    };
    // a member's tile: its strips, or its colorIndex range (the largest: the last member's,
    // with the source-less tail); member 0 stacks the tiles (alias: the whole frame)
    size_t tile = (size_t)max_rows * W;
    if (alias) {
        tile = 0;
        for (uint32_t r = 0; r < parts; ++r) tile = std::max<size_t>(tile, range_of(r).second - range_of(r).first);
    }
    const size_t stack = alias ? (size_t)total : tile * parts;
    // member 0's buffers live on member 0's device: the setters (for_members) and the
    // previous frame leave another member's device current
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int rc = ensure(ctx, &ctx->d_tile, &ctx->tile_cap, std::max(stack, tile));  // member 0: the gathered stack
    if (rc) return rc;
    if ((rc = check_on_device(ctx, ctx->d_tile, "the gathered tile stack"))) return rc;
    for (uint32_t r = 0; r < parts; ++r) {
        spt_ctx *c = m[r];
        HIP_TRY(ctx, hipSetDevice(c->device));
        if (r > 0 && (rc = ensure(c, &c->d_tile, &c->tile_cap, tile)))
            return fail(ctx, rc, "member device %d: %s", c->device, c->err.c_str());
        float4 *dst = r == 0 ? ctx->d_tile : c->d_tile;
        if (alias) {
            const auto [i0, i1] = range_of(r);
            if (i1 > i0) {
                // the rows holding the range's sources: dx + dy H in [i0, i1), 0 <= dx < W
                // (none when i0 >= (W - 1) + (H - 1) H + 1: an empty map, NaN outputs)
                const uint32_t dy_lo = i0 >= W ? (i0 - W + H) / H : 0u, dy_hi = std::min(H - 1u, (i1 - 1u) / H);
                const spt::RowMap map{std::min(dy_lo, H), std::max(std::min(dy_lo, H), dy_hi + 1u), 1u, 1u, 0u, 0u, W};
                const AliasRange ar{i0, i1 - i0, H};
                if ((rc = render_impl(c, mode, map, dst, nullptr, c->stream, false, nullptr, 1, &ar)))
                    return r == 0 ? rc : fail(ctx, rc, "member device %d: %s", c->device, c->err.c_str());
            }
        } else {
            spt::RowMap map{0, H, strip, parts, r, 0, W};
            if ((rc = render_impl(c, mode, map, dst, nullptr, c->stream, false)))
                return r == 0 ? rc : fail(ctx, rc, "member device %d: %s", c->device, c->err.c_str());
        }
        if (r > 0) HIP_TRY(ctx, hipEventRecord(c->frame_ev, c->stream));
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (uint32_t r = 1; r < parts; ++r) {
        spt_ctx *c = m[r];
        const size_t n_r = alias ? (size_t)(range_of(r).second - range_of(r).first)
                                 : (size_t)spt::rows_owned(spt::RowMap{0, H, strip, parts, r, 0, W}) * W;
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, c->frame_ev, 0));
        // alias: member r's range lands at its first output, so the stack is the frame
        const size_t at = alias ? (size_t)range_of(r).first : (size_t)r * tile;
        if (n_r)
            HIP_TRY(ctx, hipMemcpyPeerAsync(ctx->d_tile + at, ctx->device, c->d_tile, c->device,
                                            n_r * sizeof(float4), ctx->stream));
    }
    float4 *dframe = nullptr;
    if (rgba_out) {
        if ((rc = ensure(ctx, &ctx->d_fullframe, &ctx->fullframe_cap, (size_t)W * H))) return rc;
        if ((rc = check_on_device(ctx, ctx->d_fullframe, "the assembled frame"))) return rc;
        dframe = ctx->d_fullframe;
    }
    uint8_t *d8 = nullptr;
    if (g_data) {
        if ((rc = ensure(ctx, &ctx->d_frame8, &ctx->frame8_cap, (size_t)W * H * 3))) return rc;
        if ((rc = check_on_device(ctx, ctx->d_frame8, "g_data's device copy"))) return rc;
        d8 = ctx->d_frame8;
    }
    // alias: the stack is the frame in row-major order (one part of H rows)
    if (alias)
        HIP_TRY(ctx, spt::launch_assemble(ctx->d_tile, H, spt::RowMap{0, H, 1u, 1u, 0u, 0, W}, W, H, dframe, d8,
                                          ctx->stream));
    else
        HIP_TRY(ctx, spt::launch_assemble(ctx->d_tile, max_rows, spt::RowMap{0, H, strip, parts, 0u, 0, W}, W, H,
                                          dframe, d8, ctx->stream));
    if (rgba_out)
        HIP_TRY(ctx, hipMemcpyAsync(rgba_out, dframe, (size_t)W * H * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
    if (g_data) HIP_TRY(ctx, hipMemcpyAsync(g_data, d8, (size_t)W * H * 3, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    for (spt_ctx *c : m) {
        HIP_TRY(ctx, hipSetDevice(c->device));
        if ((rc = collect_timings(c, false))) return rc;
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return SPT_OK;
}

int spt_service_start(spt_ctx *ctx)
{
    return for_members(ctx, [](spt_ctx *c) {
        std::lock_guard<std::mutex> lk(c->mu);
        c->svc.enabled = true;
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

int spt_rows_count(uint32_t yB, uint32_t yE, uint32_t strip, uint32_t parts, uint32_t part, uint32_t *rows)
{
    if (!rows || strip == 0 || parts == 0 || part >= parts) return fail(nullptr, SPT_ERR_ARG, "bad row map");
    spt::RowMap m{yB, yE, strip, parts, part, 0u, 0u};
    *rows = spt::rows_owned(m);
    return SPT_OK;
}

int spt_render_rows_async(spt_ctx *ctx, int mode, uint32_t yB, uint32_t yE, uint32_t strip, uint32_t parts,
                          uint32_t part, uint32_t xB, uint32_t xE, void *d_rgba, void *d_rgb8, void *stream)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (mode != SPT_MODE_SEGMENT && mode != SPT_MODE_TASK) return fail(ctx, SPT_ERR_ARG, "bad mode %d", mode);
    if (strip == 0 || parts == 0 || part >= parts) return fail(ctx, SPT_ERR_ARG, "bad row map");
    if ((rc = check_region(ctx, yB, yE, xB, xE))) return rc;
    if (yB >= yE || xB >= xE) return SPT_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    spt::RowMap map{yB, yE, strip, parts, part, xB, xE - xB};
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP default stream
    return render_impl(ctx, mode, map, (float4 *)d_rgba, (uint8_t *)d_rgb8, s, false);
}

int spt_assemble_rows_async(spt_ctx *ctx, const void *d_tiles, uint32_t max_rows, uint32_t yB, uint32_t yE,
                            uint32_t strip, uint32_t parts, uint32_t xB, uint32_t xE, void *d_frame_rgba, void *d_rgb8,
                            void *stream)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!d_tiles || strip == 0 || parts == 0 || yE > ctx->H || xE > ctx->W || yB > yE || xB > xE)
        return fail(ctx, SPT_ERR_ARG, "bad assemble arguments");
    if (!ctx->params_set) return fail(ctx, SPT_ERR_STATE, "params not set");
    for (uint32_t p = 0; p < parts; ++p) {
        spt::RowMap m{yB, yE, strip, parts, p, xB, xE - xB};
        if (spt::rows_owned(m) > max_rows) return fail(ctx, SPT_ERR_ARG, "max_rows smaller than part %u's rows", p);
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    spt::RowMap base{yB, yE, strip, parts, 0u, xB, xE - xB};
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP default stream
    HIP_TRY(ctx, spt::launch_assemble((const float4 *)d_tiles, max_rows, base, ctx->W, ctx->H, (float4 *)d_frame_rgba,
                                      (uint8_t *)d_rgb8, s));
    return SPT_OK;
}

int spt_synchronize(spt_ctx *ctx)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    // a resident service session ends first (its kernel would keep the device busy until it
    // idles out); the next render starts a new one
    for (spt_ctx *c : ctx->peers) {
        std::lock_guard<std::mutex> lk(c->mu);
        HIP_TRY(ctx, hipSetDevice(c->device));
        if (svc_end(c)) return fail(ctx, SPT_ERR_HIP, "member device %d: %s", c->device, c->err.c_str());
        HIP_TRY(ctx, hipDeviceSynchronize());
        if (collect_timings(c)) return fail(ctx, SPT_ERR_HIP, "member device %d: %s", c->device, c->err.c_str());
    }
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (int rc = svc_end(ctx)) return rc;
    HIP_TRY(ctx, hipDeviceSynchronize());
    return collect_timings(ctx);
}

int spt_render_samples(spt_ctx *ctx, int mode, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *out)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (!out) return fail(ctx, SPT_ERR_ARG, "null out");
    if ((rc = check_region(ctx, yB, yE, xB, xE))) return rc;
    if (yB >= yE || xB >= xE) return SPT_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    spt::RowMap map{yB, yE, 1u, 1u, 0u, xB, xE - xB};
    // the sample words are decoded on the device, out[p * spp + s] = {r, g, b, counted},
    // in chunks of pixels through one staging buffer of at most 256 MiB, allocated before
    // the render (a failed allocation leaves nothing rendered)
    const size_t npix = (size_t)(xE - xB) * (yE - yB);
    const size_t per_px = (size_t)ctx->spp * sizeof(float4);
    const size_t chunk = std::max<size_t>(1, std::min(npix, ((size_t)256 << 20) / per_px));
    float4 *d_out = nullptr;
    if (hipMalloc((void **)&d_out, chunk * per_px) != hipSuccess)
        return fail(ctx, SPT_ERR_NOMEM, "spt_render_samples: %zu bytes of staging", chunk * per_px);
    if ((rc = render_impl(ctx, mode, map, nullptr, nullptr, ctx->stream, true))) {
        (void)hipFree(d_out);
        return rc;
    }
    spt::FoldArgs fa = fold_args(ctx, workspace_for(ctx, ctx->stream)->d_samples, mode == SPT_MODE_SEGMENT ? 1u : 2u);
    fa.map = map;
    fa.npix = (uint32_t)npix;
    fa.spp_batch = ctx->spp;
    hipError_t e = hipSuccess;
    for (size_t p0 = 0; p0 < npix && e == hipSuccess; p0 += chunk) {
        const size_t n = std::min(chunk, npix - p0);
        e = spt::launch_expand(fa, d_out, (uint32_t)p0, (uint32_t)n, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(out + p0 * ctx->spp * 4, d_out, n * per_px, hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    }
    (void)hipFree(d_out);
    if (e != hipSuccess) return fail(ctx, SPT_ERR_HIP, "spt_render_samples: %s", hipGetErrorString(e));
    return collect_timings(ctx);
}

namespace {
int stats_one(spt_ctx *ctx, spt_stats *out)
{
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int rc = collect_timings(ctx);
    if (rc) return rc;
    unsigned long long c[kCounters] = {0};
    HIP_TRY(ctx, hipMemcpy(c, ctx->d_counters, sizeof c, hipMemcpyDeviceToHost));
    out->casts = c[0];
    out->samples = c[1];
    out->dropped = c[2];
    for (int i = 0; i < SPT_DIAG_WORDS; ++i) out->diag[i] = c[4 + i];
    out->launches = ctx->launches;
    out->render_ms = ctx->render_ms;
    out->fold_ms = ctx->fold_ms;
    out->last_render_ms = ctx->last_render_ms;
    out->render_busy_ms = busy_ms(ctx);
    out->grid_blocks = ctx->last_grid ? ctx->last_grid : ctx->grid;
    out->block_threads = ctx->last_block ? ctx->last_block : ctx->block;
    out->batches = ctx->batches;
    out->batched_calls = ctx->batched_calls;
    out->svc_sessions = ctx->svc.sessions;
    out->svc_jobs = ctx->svc.jobs;
    out->svc_watchdog_exits = ctx->svc.watchdog_exits;
    out->svc_kernel_ms = ctx->svc.kernel_ms;
    out->svc_running = ctx->svc.running ? 1u : 0u;
    out->svc_grid_blocks = std::max<uint32_t>(1u, ctx->svc_grid / ctx->svc.grid_div);
    out->svc_flow_restarts = ctx->svc.flow_restarts;
    out->svc_closing_restarts = ctx->svc.closing_restarts;
    out->prim_list_blocks = ctx->prim_blocks;
    out->prim_list_entries = ctx->prim_entries;
    out->prim_list_build_ms = ctx->prim_build_s * 1e3;
    out->prim_list_builds = ctx->prim_builds;
    out->accel_build_ms = ctx->accel_build_s * 1e3;
    return SPT_OK;
}

int reset_one(spt_ctx *ctx)
{
    std::lock_guard<std::mutex> lk(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int rc = svc_end(ctx);  // its waves add their counts when they leave
    if (!rc) rc = collect_timings(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemset(ctx->d_counters, 0, kCounters * sizeof(unsigned long long)));
    ctx->render_ms = ctx->fold_ms = ctx->last_render_ms = 0;
    ctx->launches = 0;
    ctx->batches = ctx->batched_calls = 0;
    ctx->svc.sessions = ctx->svc.jobs = ctx->svc.watchdog_exits = 0;
    ctx->svc.flow_restarts = ctx->svc.closing_restarts = 0;
    ctx->svc.kernel_ms = 0;
    ctx->spans.clear();
    ctx->ref_recorded = false;
    return SPT_OK;
}
}  // namespace

int spt_get_stats(spt_ctx *ctx, spt_stats *out)
{
    if (!ctx || !out) return fail(ctx, SPT_ERR_ARG, "null argument");
    int rc = stats_one(ctx, out);
    // a multi-device context sums the members' counters and device times; busy time is
    // the longest member's (the devices run concurrently)
    for (spt_ctx *p : ctx->peers) {
        spt_stats q{};
        if ((rc = stats_one(p, &q))) return fail(ctx, rc, "member device %d: %s", p->device, p->err.c_str());
        out->casts += q.casts;
        out->samples += q.samples;
        out->dropped += q.dropped;
        for (int i = 0; i < SPT_DIAG_WORDS; ++i) out->diag[i] += q.diag[i];
        out->launches += q.launches;
        out->batches += q.batches;
        out->batched_calls += q.batched_calls;
        out->render_ms += q.render_ms;
        out->fold_ms += q.fold_ms;
        out->render_busy_ms = std::max(out->render_busy_ms, q.render_busy_ms);
    }
    return rc;
}

int spt_reset_stats(spt_ctx *ctx)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    int rc = reset_one(ctx);
    for (spt_ctx *p : ctx->peers)
        if (!rc && (rc = reset_one(p))) return fail(ctx, rc, "member device %d: %s", p->device, p->err.c_str());
    return rc;
}

int spt_selftest_numerics(spt_ctx *ctx, const float *a, const float *b, const uint32_t *bits, uint32_t n, float *out)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!a || !b || !bits || !out) return fail(ctx, SPT_ERR_ARG, "null argument");
    if (n == 0) return SPT_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    uint32_t *dbits = nullptr;
    HIP_TRY(ctx, hipMalloc((void **)&da, n * sizeof(float)));
    HIP_TRY(ctx, hipMalloc((void **)&db, n * sizeof(float)));
    HIP_TRY(ctx, hipMalloc((void **)&dbits, n * sizeof(uint32_t)));
    HIP_TRY(ctx, hipMalloc((void **)&dout, (size_t)n * SPT_SELFTEST_COLS * sizeof(float)));
    HIP_TRY(ctx, hipMemcpy(da, a, n * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(db, b, n * sizeof(float), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(dbits, bits, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(ctx, spt::launch_selftest(da, db, dbits, n, dout, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipMemcpy(out, dout, (size_t)n * SPT_SELFTEST_COLS * sizeof(float), hipMemcpyDeviceToHost));
    (void)hipFree(da);
    (void)hipFree(db);
    (void)hipFree(dbits);
    (void)hipFree(dout);
    return SPT_OK;
}

}  // extern "C"
