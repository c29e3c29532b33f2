// spt_render.cpp -- render + fold launches (render_impl), host-output calls and their slots,
// the rows / assemble / samples entry points (spt_host.h).
#include "spt_host.h"

namespace spt_api {

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

// grid_div: concurrent host calls on this context share the GPU (render_grid)
int render_impl(spt_ctx *ctx, int mode, const spt::RowMap &map, float4 *d_rgba, uint8_t *d_rgb8, hipStream_t s,
                bool keep_samples, const Progress *pg, uint32_t grid_div, const AliasRange *ar)
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

// RenderSegment / RenderSegmentTask with host outputs; with pass_spp > 0 progressively,
// copying the outputs back and calling cb after every pass.  The context lock is held
// only while launches are enqueued: each call renders on its own slot (stream,
// workspace, staging), waits for its stream unlocked, so concurrent callers -- the
// reference's RenderJob threads -- overlap on the GPU; cb runs unlocked too.
// spread: a multi-device context sends the call to its least busy member (else member 0).
int render_segment_host(spt_ctx *ctx, int mode, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *rgba,
                        uint8_t *g_data, uint32_t pass_spp, spt_progress_fn cb, void *user,
                        bool spread)
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

}  // namespace spt_api

extern "C" {

int spt_render_segment(spt_ctx *ctx, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *rgba, uint8_t *g_data)
{
    return render_segment_host(ctx, SPT_MODE_SEGMENT, yB, yE, xB, xE, rgba, g_data);
}

int spt_render_segment_task(spt_ctx *ctx, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE, float *rgba,
                            uint8_t *g_data)
{
    return render_segment_host(ctx, SPT_MODE_TASK, yB, yE, xB, xE, rgba, g_data);
}

int spt_render_progressive(spt_ctx *ctx, int mode, uint32_t yB, uint32_t yE, uint32_t xB, uint32_t xE,
                           uint32_t pass_spp, float *rgba, uint8_t *g_data, spt_progress_fn cb, void *user)
{
    if (mode != SPT_MODE_SEGMENT && mode != SPT_MODE_TASK) return fail(ctx, SPT_ERR_ARG, "bad mode %d", mode);
    if (pass_spp == 0) return fail(ctx, SPT_ERR_ARG, "pass_spp must be >= 1");
    return render_segment_host(ctx, mode, yB, yE, xB, xE, rgba, g_data, pass_spp, cb, user);
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

}  // extern "C"
