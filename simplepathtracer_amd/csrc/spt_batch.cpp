// spt_batch.cpp -- batched host calls (concurrent RenderJob tiles in shared launches) and the
// read-ahead of the reference's tiling (spt_host.h).
#include "spt_host.h"

namespace spt_api {

// Bytes of per-sample slots a rectangle needs in one batch (all spp samples at once).
uint64_t batch_slot_bytes(const spt_ctx *ctx, int mode, uint64_t npix)
{
    return npix * ctx->spp * (mode == SPT_MODE_SEGMENT ? 1u : 2u) * sizeof(uint32_t);
}

// Enqueue one batch on bs->stream: rectangle table, render, fold, the copy-back of
// every request's outputs.  Called with ctx->mu held.
int launch_batch(spt_ctx *ctx, BatchSet *bs, const std::vector<BatchReq *> &batch, uint8_t *spec_d8)
{
    host_trace("launch_batch begin", bs);
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
        host_trace("launch_batch render launch", bs);
        HIP_TRY(ctx, spt::launch_render(ra, sh, s));
        host_trace("launch_batch render launched", bs);
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
    host_trace("launch_batch end", bs);
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
        if (!bs->stream && bs == &ctx->bsets[1]) bs->stream = warm_take(ctx, 0);  // created while set 0 rendered
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
    if (!bs->stream) bs->stream = warm_take(ctx, 1 + p);
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

// The read-ahead frame's page-locked bytes (SpecFrame::h8), at least `bytes` of them.
int spec_frame_bytes(spt_ctx *ctx, size_t bytes)
{
    SpecFrame &sp = ctx->spec;
    if (sp.h8_cap >= bytes) return SPT_OK;
    // hipHostFree synchronises the device, which a resident service session would hold
    if (int rc = svc_end(ctx)) return rc;
    if (sp.h8) HIP_TRY(ctx, hipHostFree(sp.h8));
    sp.h8 = sp.h8_dev = nullptr;
    sp.h8_cap = 0;
    HIP_TRY(ctx, hipHostMalloc((void **)&sp.h8, bytes));
    void *dp = nullptr;
    HIP_TRY(ctx, hipHostGetDevicePointer(&dp, sp.h8, 0));
    sp.h8_dev = (uint8_t *)dp;
    sp.h8_cap = bytes;
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
    host_trace("spec_prepare begin");
    (void)mode;
    const uint32_t W = ctx->W, H = ctx->H;
    int rc = spec_frame_bytes(ctx, (size_t)W * H * 3);
    host_trace("spec_prepare frame bytes");
    if (rc) return rc;
    const uint32_t np = std::min(sp.parts, tc), rpp = (tc + np - 1) / np;
    // the parts' streams and sample workspaces come with the first read-ahead (spec_launch):
    // a one-frame caller (the reference's MainLoop renders one frame per process) never
    // pays for them
    for (uint32_t p = 0; p * rpp < tc; ++p) {
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
        host_trace("spec_prepare host rects", (void *)(uintptr_t)p);
        if ((rc = ensure(ctx, &bs->d_rects, &bs->rects_cap, tiles))) return rc;
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
    // the frame being replaced (before spec_drain retires it): its unserved tiles are owed to
    // late callers (at most 4 per tile, so a caller that never asks for a tile does not
    // accumulate them)
    const size_t ntiles = (size_t)tc * tc;
    const bool replaces = sp.active && sp.mode == mode && sp.tc == tc && sp.gen == ctx->gen &&
                          sp.owed.size() == ntiles && sp.served.size() == ntiles;
    int rc = spec_drain(ctx);
    if (rc) return rc;
    const uint32_t W = ctx->W, H = ctx->H, sw = W / tc, sh = H / tc;
    if ((rc = spec_frame_bytes(ctx, (size_t)W * H * 3))) return rc;
    if (replaces) {
        for (size_t k = 0; k < ntiles; ++k)
            if (!sp.served[k] && sp.owed[k] < 4) sp.owed[k]++;
    } else {
        sp.owed.assign(ntiles, 0);
    }
    std::vector<BatchReq> reqs((size_t)tc * tc);
    for (uint32_t j = 0; j < tc; ++j)
        for (uint32_t i = 0; i < tc; ++i)
            reqs[(size_t)j * tc + i] = BatchReq{mode,    sh * j,    std::min(sh * j + sh, H), sw * i, std::min(sw * i + sw, W),
                                                nullptr, sp.h8,    SPT_OK,                   true,   false};
    const uint32_t np = std::min(sp.parts, tc), rpp = (tc + np - 1) / np;  // launches, tile rows each
    sp.rows_per_part = rpp;
    for (uint32_t p = 0; p * rpp < tc; ++p) {
        std::vector<BatchReq *> part;
        for (uint32_t j = p * rpp; j < std::min(tc, (p + 1) * rpp); ++j)
            for (uint32_t i = 0; i < tc; ++i) part.push_back(&reqs[(size_t)j * tc + i]);
        BatchSet *bs = &sp.bs[p];
        if ((rc = spec_stream(ctx, (int)p))) return rc;
        if ((rc = launch_batch(ctx, bs, part, sp.h8_dev))) return rc;
        HIP_TRY(ctx, hipEventRecord(sp.ev[p], bs->stream));
        sp.launched[p] = true;
        sp.finished[p] = false;
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
        if (!sp.served[k]) return (int64_t)k;
        if (k < sp.owed.size() && sp.owed[k] > 0) {
            // a call an earlier frame still owed (late RenderJob thread): same bytes
            --sp.owed[k];
            return (int64_t)k;
        }
        return -1;
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
        // the read-ahead frame's page-locked bytes (grown only once no serve copies out of the
        // old ones): without them the call renders as usual
        if (sp.h8_cap < (size_t)W * H * 3) {
            sp.readers_cv.wait(lk, [&] { return sp.readers == 0; });
            if (spec_frame_bytes(ctx, (size_t)W * H * 3) != SPT_OK) return kSpecMiss;
        }
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
            // arm_first: the first call of a tiling (RenderImageParallelMain's detached
            // threads reach the library in no fixed order) arms it and starts the read-ahead at
            // once -- the one frame of the reference's MainLoop is then rendered whole
            // 
            const bool now = !seen && sp.arm_first && sp.arm_count == 0;
            if (!seen) {
                seen = 1;
                sp.armed = ++sp.arm_count == tc * tc || now;
                // the read-ahead's buffers now, while this frame's tiles render as usual
                if (sp.armed) {
                    const int rc = spec_prepare(ctx, lk, mode, tc);
                    if (rc) return rc;
                }
            }
            if (!now) {
                host_trace("spec_serve miss (not armed), tile", (void *)(uintptr_t)((yB / h) * tc + xB / w));
                return kSpecMiss;
            }
        }
        host_trace("spec_serve launch for tile", (void *)(uintptr_t)((yB / h) * tc + xB / w));
        int rc = spec_launch(ctx, lk, mode, tc);
        if (rc) return rc;
        k = tile_of();
        if (k < 0) return kSpecMiss;
    }
    sp.served[(size_t)k] = 1;
    const uint32_t part = (uint32_t)k / sp.tc / sp.rows_per_part;
    const hipEvent_t ev = sp.ev[part];
    const bool finished = sp.finished[part];
    const uint8_t *const src = sp.h8;
    sp.readers++;
    lk.unlock();
    // rows y in [yB, yE) live at g_data rows H-1-y: one band, xB.. per row; the part's fold
    // wrote them into the page-locked frame (its event completes after the kernel's writes;
    // once one serve has seen it complete, the part's other serves skip the sync: 1 024
    // serves per frame at tc = 32)
    const size_t pitch = (size_t)W * 3, off = (size_t)(H - yE) * pitch + (size_t)xB * 3;
    const hipError_t e = finished ? hipSuccess : hipEventSynchronize(ev);
    if (e == hipSuccess)
        for (uint32_t r = 0; r < yE - yB; ++r)
            std::memcpy(g_data + off + r * pitch, src + off + r * pitch, (size_t)(xE - xB) * 3);
    lk.lock();
    if (e == hipSuccess && sp.ev[part] == ev && sp.launched[part]) sp.finished[part] = true;
    if (--sp.readers == 0) sp.readers_cv.notify_all();
    if (e != hipSuccess) return fail(ctx, SPT_ERR_HIP, "read-ahead tile copy failed: %s", hipGetErrorString(e));
    return SPT_OK;
}

}  // namespace spt_api
