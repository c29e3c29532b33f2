// spt_multi.cpp -- multi-device frames (spt_render_frame: strips per member, peer copies,
// assemble) and page-locked g_data (spt_pin_host; spt_host.h).
#include "spt_host.h"

// Outputs [i0, i1) of RenderSegmentTask({0, H, 0, W}) on a non-square frame (the
// context's frame; RenderImage's aliasing, TaskBasedPathTracer.hpp:103,186,196-205) into
// d_out[0, i1 - i0) on stream s: the rows holding the range's sources (dx + dy H in
// [i0, i1), 0 <= dx < W; none when i0 >= (W - 1) + (H - 1) H + 1: NaN outputs) rendered,
// the range folded.  Called with ctx->mu held.
namespace spt_api {

int render_task_range(spt_ctx *ctx, uint32_t i0, uint32_t i1, float4 *d_out, hipStream_t s)
{
    const uint32_t W = ctx->W, H = ctx->H;
    if (i1 <= i0) return SPT_OK;
    const uint32_t dy_lo = i0 >= W ? (i0 - W + H) / H : 0u, dy_hi = std::min(H - 1u, (i1 - 1u) / H);
    const spt::RowMap map{std::min(dy_lo, H), std::max(std::min(dy_lo, H), dy_hi + 1u), 1u, 1u, 0u, 0u, W};
    const AliasRange ar{i0, i1 - i0, H};
    return render_impl(ctx, SPT_MODE_TASK, map, d_out, nullptr, s, false, nullptr, 1, &ar);
}

}  // namespace spt_api


extern "C" {

int spt_task_range(uint32_t width, uint32_t height, uint32_t parts, uint32_t part, uint32_t *i0, uint32_t *i1)
{
    if (!i0 || !i1 || width == 0 || height == 0 || parts == 0 || part >= parts)
        return fail(nullptr, SPT_ERR_ARG, "bad task range arguments");
    // outputs [0, n_src) have sources (p_max + 1 = W + (H - 1) H, at most W H): dealt evenly,
    // the last part also takes the source-less tail (every part renders about the same rows)
    const uint64_t total = (uint64_t)width * height;
    const uint64_t n_src = std::min<uint64_t>(total, (uint64_t)width + (uint64_t)(height - 1u) * height);
    const uint64_t L = (n_src + parts - 1) / parts;
    const uint64_t a = std::min<uint64_t>((uint64_t)part * L, n_src);
    const uint64_t b = part + 1 == parts ? total : std::min<uint64_t>(a + L, n_src);
    if (total > 0xFFFFFFFFull) return fail(nullptr, SPT_ERR_ARG, "frame too large");
    *i0 = (uint32_t)a;
    *i1 = (uint32_t)b;
    return SPT_OK;
}

int spt_render_task_range_async(spt_ctx *ctx, uint32_t i0, uint32_t i1, void *d_rgba, void *stream)
{
    if (!ctx) return fail(nullptr, SPT_ERR_ARG, "null context");
    std::lock_guard<std::mutex> lk(ctx->mu);
    int rc = check_ready(ctx);
    if (rc) return rc;
    if (i0 > i1 || (uint64_t)i1 > (uint64_t)ctx->W * ctx->H || (i1 > i0 && !d_rgba))
        return fail(ctx, SPT_ERR_ARG, "bad task range [%u, %u) of a %ux%u frame", i0, i1, ctx->W, ctx->H);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return render_task_range(ctx, i0, i1, (float4 *)d_rgba, (hipStream_t)stream);
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
    uint32_t max_rows = 0;
    for (uint32_t r = 0; r < parts; ++r) max_rows = std::max(max_rows, spt::rows_owned(spt::RowMap{0, H, strip, parts, r, 0, W}));
    auto range_of = [&](uint32_t r) {
        uint32_t i0 = 0, i1 = 0;
        (void)spt_task_range(W, H, parts, r, &i0, &i1);
        return std::make_pair(i0, i1);
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
            if ((rc = render_task_range(c, i0, i1, dst, c->stream)))
                return r == 0 ? rc : fail(ctx, rc, "member device %d: %s", c->device, c->err.c_str());
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

}  // extern "C"
