// spt_host.h -- the host side of the C ABI (include/spt_hip.h), shared by its translation
// units (round 6: spt_api.cpp split along its sections, no behaviour change):
//   spt_ctx.cpp      context, setters, scene / accel / primary-list uploads, stats
//   spt_render.cpp   render_impl (render + fold launches), host calls, rows / samples entry points
//   spt_batch.cpp    batched host calls and the tiling read-ahead (SpecFrame)
//   spt_service.cpp  the render service's host half (sessions, publication, flow control)
//   spt_multi.cpp    multi-device frames (spt_render_frame) and page-locked g_data
// The context owns the device copy of the reference's global state (scene SoA, camera,
// config: Globals.hpp:8-37), the per-sample workspaces and the launch geometry of the
// persistent render kernel, and rebuilds the two reference entry points RenderSegment
// (SingleThreadPathTracer.hpp:114-137) and RenderSegmentTask (TaskBasedPathTracer.hpp:54-206)
// as render + fold launches.
#pragma once
#include "spt_hip.h"
#include "spt_accel.h"
#include "spt_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace spt_api {

// An environment variable's value, or null when unset or empty (a variable set to ""
// reads as unset: SPT_BLOCKS_PER_CU= would otherwise mean a 1-block grid)
inline const char *env_var(const char *name)
{
    const char *e = std::getenv(name);
    return e && *e ? e : nullptr;
}

extern thread_local std::string g_thread_error;
// the context whose progress callback is running on this thread (spt_render_progressive)
extern thread_local const spt_ctx *t_in_callback;

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
};

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
// "armed": a caller rendering one tile alone never arms it; with arm_first, the drop-in's
// setting, its first call arms it), the first call of a tile of it
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
    // per tile, calls still owed by an earlier frame of this tiling: tiles that frame had
    // not served when the next one began -- a RenderJob thread that starts only after its
    // frame's final wait ended (Renderer.hpp:242-255, 282-292) -- served from the current
    // frame (same state, the same bytes) instead of starting another one
    std::vector<uint8_t> owed;
    static constexpr int kParts = 4;
    uint32_t parts = 4, rows_per_part = 1;  // tile rows per launch
    hipEvent_t ev[kParts] = {};
    bool launched[kParts] = {};
    bool finished[kParts] = {};  // a serve saw the part's event complete (later serves skip the sync)
    BatchSet bs[kParts];
    // the frame's RGB8 bytes (g_data layout) in page-locked host memory: the parts' folds
    // write them through its device view, each serve copies its tile's rows on the host
    // (a hipMemcpy2D per tile cost ~10 us of runtime time each: 1 024 per frame at tc = 32)
    uint8_t *h8 = nullptr, *h8_dev = nullptr;
    size_t h8_cap = 0;
    // serves copying out of h8 with the context unlocked: the next read-ahead neither
    // rewrites nor reallocates h8 before they are done (readers_cv, ctx->mu)
    uint32_t readers = 0;
    std::condition_variable readers_cv;
    // arming: the tiles of one tiling (mode, tc, frame size) called so far by plain calls
    int arm_mode = -1;
    uint32_t arm_tc = 0, arm_w = 0, arm_h = 0, arm_count = 0;
    std::vector<uint8_t> arm_seen;
    bool armed = false;
    // arm at a tiling's first call instead of after a whole tiling (the drop-in,
    // spt_prepare_dropin: its caller is RenderImageParallelMain, which renders every tile
    // of every frame -- and MainLoop only one frame per process)
    bool arm_first = false;
};

constexpr int kSpecMiss = 1;  // spec_serve: not a read-ahead tile (render it as usual)

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
    // SPT_SVC_LDS=1: scenes whose tree takes the LDS lane walk run LDS-tree sessions
    // (render_kernel_svc_lds); off by default: measured slower than launches (§4.7)
    bool lds = false;
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
// One job of a publication: a region (rows or interleaved strips, columns) at spp_batch
// samples from sample s0, its slots at slot_local of the publication's ring region.
struct SvcJobSpec {
    spt::RowMap map;
    uint32_t rows, spp_batch, s0;
    spt::FastDiv div_band, div_tile, div_strip;
    uint64_t slot_local;
};
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

}  // namespace spt_api

using namespace spt_api;

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
    bool svc_full = false;  // SPT_SVC_FULL_GRID: sessions take every block slot (LDS-tree sessions too)
    int svc_per_cu = 1;     // the occupancy's blocks per CU the session grids derive from
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

    // Stream warm-up for the drop-in (spt_prepare_dropin, spt_ctx.cpp): the second batch
    // set's stream (s[0]) and the read-ahead parts' streams (s[1 + p]), created up front
    // and taken by the first call that needs each (warm_take)
    struct Warm {
        hipStream_t s[1 + SpecFrame::kParts] = {};
        bool started = false;
    } warm;
};

namespace spt_api {

#define HIP_TRY(ctx, expr)                                                                          \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail((ctx), SPT_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));        \
    } while (0)

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

int spt_set_workspace_one(spt_ctx *ctx, uint64_t bytes);
int spt_set_engine_one(spt_ctx *ctx, int engine);
int spt_set_cluster_tree_one(spt_ctx *ctx, uint32_t branching);
int spt_set_cluster_size_one(spt_ctx *ctx, uint32_t k);
int spt_set_params_one(spt_ctx *ctx, uint32_t width, uint32_t height, uint32_t spp, uint32_t bounces, uint64_t seed);
int spt_set_camera_one(spt_ctx *ctx, const float view[16], const float eye[4], const float sky[4]);
int spt_set_scene_one(spt_ctx *ctx, const float *centers4, const float *radii, const float *colors4, const uint8_t *materials, const float *fuzz, uint32_t n);
uint32_t even_strip(uint32_t height, uint32_t parts);
int check_not_in_callback(spt_ctx *ctx);
int rebuild_prim(spt_ctx *ctx);
int wait_own_renders(spt_ctx *ctx);
int rebuild_accel(spt_ctx *ctx);
int ensure_wavefront(spt_ctx *ctx, Workspace *w, uint32_t cap, uint32_t qcap);
hipStream_t companion_for(spt_ctx *ctx, hipStream_t s);
Workspace * workspace_for(spt_ctx *ctx, hipStream_t s);
uint32_t render_grid(const spt_ctx *ctx, uint64_t items, uint32_t claim, uint32_t div, bool masked = false);
uint32_t claim_size(const spt_ctx *ctx, uint64_t items, bool masked = false);
int masked_for(spt_ctx *ctx, hipStream_t s, spt_ctx::Masked **out);
uint32_t full_grid(const spt_ctx *ctx, bool masked = false);
uint64_t fmix64(uint64_t z);
int check_ready(spt_ctx *ctx);
spt::DeviceScene device_scene(const spt_ctx *ctx);
uint32_t code_jmax(const spt_ctx *ctx);
uint32_t halvings_to_zero(const std::vector<float4> &shade);
double busy_ms(const spt_ctx *ctx);
int collect_timings(spt_ctx *ctx, bool wait = true);
EventPair get_pair(spt_ctx *ctx);
int check_on_device(spt_ctx *ctx, const void *p, const char *what);
int fail(spt_ctx *ctx, int code, const char *fmt, ...);
int svc_retire(spt_ctx *ctx, hipStream_t s, uint64_t w0, uint64_t words, uint32_t idx);
int svc_submit(spt_ctx *ctx, const spt::RenderArgs &ra, int mode, hipStream_t s, uint64_t *w0_out, uint32_t *idx_out);
int svc_submit_jobs(spt_ctx *ctx, int mode, const SvcJobSpec *jobs, size_t n, uint64_t total_slots, hipStream_t s, uint64_t *w0_out, uint32_t *idx_out);
bool svc_eligible(const spt_ctx *ctx, uint64_t words, bool keep_samples);
// SPT_HOST_TRACE=1: a line on stderr with the ms since the process's first trace point
// (where host time goes in a cold frame: allocations, stream creation, first launches)
void host_trace(const char *what, const void *arg = nullptr);
void warm_start(spt_ctx *ctx);
hipStream_t warm_take(spt_ctx *ctx, int i);
void warm_join(spt_ctx *ctx);
uint32_t svc_session_grid(const spt_ctx *ctx);
int svc_begin(spt_ctx *ctx, int mode, const std::vector<hipEvent_t> &waits, int64_t reset_idx, hipStream_t s);
int svc_end(spt_ctx *ctx);
int svc_wait(spt_ctx *ctx, hipEvent_t e, const char *what);
hipEvent_t svc_event(spt_ctx *ctx);
int render_segment_host(spt_ctx *ctx, int mode, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *rgba, uint8_t *g_data, uint32_t pass_spp = 0, spt_progress_fn cb = nullptr, void *user = nullptr, bool spread = true);
spt_ctx * pick_member(spt_ctx *ctx);
void release_slot(spt_ctx *ctx, HostSlot *h);
HostSlot * acquire_slot(spt_ctx *ctx, std::unique_lock<std::mutex> &lk);
int check_region(spt_ctx *ctx, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE);
int render_impl(spt_ctx *ctx, int mode, const spt::RowMap &map, float4 *d_rgba, uint8_t *d_rgb8, hipStream_t s, bool keep_samples, const Progress *pg = nullptr, uint32_t grid_div = 1, const AliasRange *ar = nullptr);
int render_task_range(spt_ctx *ctx, uint32_t i0, uint32_t i1, float4 *d_out, hipStream_t s);
spt::FoldArgs fold_args(const spt_ctx *ctx, const uint32_t *samples, uint32_t slot_words);
int spec_serve(spt_ctx *ctx, std::unique_lock<std::mutex> &lk, int mode, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, uint8_t *g_data);
int spec_frame_bytes(spt_ctx *ctx, size_t bytes);
int spec_launch(spt_ctx *ctx, std::unique_lock<std::mutex> &lk, int mode, uint32_t tc);
int spec_prepare(spt_ctx *ctx, std::unique_lock<std::mutex> &lk, int mode, uint32_t tc);
int spec_stream(spt_ctx *ctx, int p);
int spec_drain(spt_ctx *ctx);
int render_batched(spt_ctx *ctx, std::unique_lock<std::mutex> &lk, int mode, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *rgba, uint8_t *g_data);
int launch_batch(spt_ctx *ctx, BatchSet *bs, const std::vector<BatchReq *> &batch, uint8_t *spec_d8 = nullptr);
uint64_t batch_slot_bytes(const spt_ctx *ctx, int mode, uint64_t npix);
int reset_one(spt_ctx *ctx);
int stats_one(spt_ctx *ctx, spt_stats *out);

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
template <class T>
int upload(spt_ctx *ctx, T **p, size_t *cap, const std::vector<T> &v)
{
    int rc = ensure(ctx, p, cap, v.size());
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return SPT_OK;
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

}  // namespace spt_api
