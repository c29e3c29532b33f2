// spt_ctx.cpp -- context lifetime, setters (scene, camera, params, traversal shape), the scene's
// device tables and primary-ray lists, stats (spt_host.h).
#include "spt_host.h"

namespace spt_api {

thread_local std::string g_thread_error;
thread_local const spt_ctx *t_in_callback = nullptr;

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

void host_trace(const char *what, const void *arg)
{
    static const bool on = env_var("SPT_HOST_TRACE") && std::atoi(env_var("SPT_HOST_TRACE")) != 0;
    if (!on) return;
    static const auto t0 = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::fprintf(stderr, "[spt %9.3f ms] %s %p\n", ms, what, arg);
}

// ---- stream warm-up (spt_prepare_dropin) ----------------------------------------------
// Creates the second batch set's stream and the read-ahead parts' streams now, in the
// caller, so that no frame pays for them.  Creating a stream adds a hardware queue, and
// on the box that stalls every queue of the device for ~9.5 ms (the scheduler's queue
// map is rewritten): done while the first frame renders (a helper thread, measured
// round 6) it stretched that frame by the same ~45 ms it took off it
void warm_start(spt_ctx *ctx)
{
    spt_ctx::Warm &w = ctx->warm;
    if (w.started) return;
    w.started = true;
    // the member's own device (a multi-device context's members: the caller's current
    // device is another member's)
    if (hipSetDevice(ctx->device) != hipSuccess) return;  // no warm streams: created on first use
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    int prio = lo;  // the read-ahead parts' priority (spec_stream)
    if (const char *e = env_var("SPT_READAHEAD_PRIO")) prio = std::atoi(e);
    for (int i = 0; i < 1 + SpecFrame::kParts; ++i) {
        hipStream_t s = nullptr;
        const hipError_t e = i == 0 ? hipStreamCreateWithFlags(&s, hipStreamNonBlocking)
                                    : hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio);
        w.s[i] = e == hipSuccess ? s : nullptr;  // null: the taker creates its own
    }
    // the process's first device-to-host hipMemcpy2D waits ~8.6 ms for the runtime's copy
    // setup (round 6 API trace of the cold frame, gpurun r06bo: its first four tile copies
    // out of the read-ahead frame took 8.6 ms each, the later ones 0.1-0.3 ms; the read-ahead
    // now serves from page-locked memory, batches copy back unpinned g_data so), and so does
    // its first host-to-device copy on a copy engine (the primary lists' upload, 8.5 ms for
    // 120 KB; the smaller scene tables go through blit kernels): one small 2D copy into
    // page-locked (registered and allocated) memory and one 256 KiB upload now
    uint8_t *d = nullptr;
    if (hipMalloc((void **)&d, 256 << 10) != hipSuccess) return;
    {
        std::vector<uint8_t> up((size_t)256 << 10, 0);
        (void)hipMemcpy(d, up.data(), up.size(), hipMemcpyHostToDevice);
    }
    static thread_local uint8_t pageable[8192];
    uint8_t *reg = (uint8_t *)(((uintptr_t)pageable + 4095) & ~(uintptr_t)4095);
    const bool registered = hipHostRegister(reg, 4096, hipHostRegisterDefault) == hipSuccess;
    uint8_t *pinned = nullptr;
    if (hipHostMalloc((void **)&pinned, 4096) != hipSuccess) pinned = nullptr;
    for (uint8_t *h : {reg, pinned})
        if (h) (void)hipMemcpy2D(h, 64, d, 64, 48, 16, hipMemcpyDeviceToHost);
    if (registered) (void)hipHostUnregister(reg);
    if (pinned) (void)hipHostFree(pinned);
    (void)hipFree(d);
}

// Warm stream i, or nullptr without a warm-up (or once taken)
hipStream_t warm_take(spt_ctx *ctx, int i)
{
    hipStream_t s = ctx->warm.s[i];
    ctx->warm.s[i] = nullptr;
    return s;
}

void warm_join(spt_ctx *ctx)
{
    for (hipStream_t &s : ctx->warm.s)
        if (s) {
            (void)hipStreamDestroy(s);
            s = nullptr;
        }
}

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
int collect_timings(spt_ctx *ctx, bool wait)
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
uint32_t full_grid(const spt_ctx *ctx, bool masked)
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
uint32_t claim_size(const spt_ctx *ctx, uint64_t items, bool masked)
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
uint32_t render_grid(const spt_ctx *ctx, uint64_t items, uint32_t claim, uint32_t div, bool masked)
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

// Setters must not run from a progress callback of the same context (the render in
// progress reads the state they change).
int check_not_in_callback(spt_ctx *ctx)
{
    if (t_in_callback == ctx) return fail(ctx, SPT_ERR_STATE, "called from a progress callback of this context");
    return SPT_OK;
}

// Rows per strip of the multi-device frame split (simplepathtracer_amd/distributed.py
// even_strip, the same rule as the one-process-per-GPU path).
uint32_t even_strip(uint32_t height, uint32_t parts)
{
    // the tallest strip (8, 4, 2, 1 rows) whose deal gives no part more than 6% over an
    // even share: 8-row strips keep the 8x8 pixel blocks of the primary batches and
    // candidate lists whole (round 6, tools/scaling_probe.py at N = 8: config 3 42.85 /
    // 46.26 / 51.05 ms per share at 8 / 4 / 2 rows, config 2 5.9 / 6.2 / 6.9 us per row);
    // distributed.even_strip is the same rule
    if (parts <= 1) return 8u;
    for (uint32_t s : {8u, 4u, 2u}) {
        const uint64_t strips = (height + s - 1) / s;
        const uint64_t rows = std::min<uint64_t>(height, (strips + parts - 1) / parts * s);
        if ((double)rows <= 1.06 * (double)height / parts) return s;
    }
    return 1u;
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
    // the drop-in (spt_prepare_dropin) renders its first frame through the tiling read-ahead:
    // its page-locked frame now, with the setup, not in that frame
    if (ctx->spec.arm_first && ctx->readahead)
        (void)spec_frame_bytes(ctx, (size_t)width * height * 3);  // best effort: else at arming
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
    out->svc_grid_blocks = svc_session_grid(ctx);
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

}  // namespace spt_api

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
    ctx->svc_per_cu = per_cu;
    ctx->svc_grid = (uint32_t)(std::max(1, per_cu - 1) * ctx->num_cu);
    // SPT_SVC_FULL_GRID=1: the session takes every block slot (folds and other streams'
    // kernels then wait for the session's end; for pipelines that end their sessions
    // themselves, like bench.py's timed regions: DESIGN.md §5)
    if (const char *e = env_var("SPT_SVC_FULL_GRID"))
        if (std::atoi(e) != 0) {
            ctx->svc_grid = (uint32_t)(per_cu * ctx->num_cu);
            ctx->svc_full = true;
        }
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
    if (const char *e = env_var("SPT_SVC_LDS")) ctx->svc.lds = std::atoi(e) != 0;
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
    warm_join(ctx);
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
    if (ctx->spec.h8) (void)hipHostFree(ctx->spec.h8);
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

int spt_prepare_dropin(spt_ctx *ctx)
{
    // the drop-in's caller renders whole tilings: the read-ahead may arm at a tiling's
    // first tile (SPT_READAHEAD_FIRST=0: only after a whole tiling, as for other callers)
    const char *e = env_var("SPT_READAHEAD_FIRST");
    const bool first = !e || std::atoi(e) != 0;
    return for_members(ctx, [&](spt_ctx *c) {
        std::lock_guard<std::mutex> lk(c->mu);
        warm_start(c);
        c->spec.arm_first = first;
        return SPT_OK;
    });
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
