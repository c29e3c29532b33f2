// spt_wavefront.hip -- queue-based (wavefront) variant of the render loop.
//
// the design of RenderSegmentTask's material queues
// (TaskBasedPathTracer.hpp:54-193) as separate HIP kernels with ballot/prefix
// compaction, to compare against the persistent megakernel.  The reference keeps
// per-material task vectors and runs one material at a time per pass; here a
// ray queue in HBM is topped up with primary rays, then per pass
//
//   wf_extend   one FindClosestIntersectionSphere per queued ray; the ray's
//               category (sky/miss, diffuse first hit, mirror, glass,
//               diffuse-loop step) and per-wave category counts (ballots);
//   scan        exclusive scan of the [category][wave] counts (hipCUB
//               DeviceScan, decoupled look-back): the offset of every wave's
//               rays in one category-major list;
//   wf_split    that list, by mbcnt rank + the wave offsets (order preserving);
//   wf_shade    one shading step for every ray of one category (homogeneous
//               work per launch, like the reference's per-material loops), in
//               place; finished paths write their sample slot;
//   wf_count / scan / wf_compact   the surviving rays, in queue order, into
//               the next queue; new primaries are appended after them.
//
// Order-preserving compaction keeps the queue in the megakernel's tile order, so a
// wave's 64 rays stay spatially coherent and cull together.  Nothing in the pass
// kernels synchronises a block or hits one global address: statistics come from
// the scans (rays cast = queue length, finished = length - survivors).  Per-lane
// counter atomics on one address made the first version 2.4x slower.
//
// Per-path arithmetic is the megakernel's own (spt_path.h: start_path,
// find_closest, shade_step), so every (pixel, sample) gets bit-identical results
// and the same fold kernel resolves the frame.
#include "spt_path.h"

#include <hipcub/hipcub.hpp>

namespace spt {

namespace {

// Ray queue entry (SoA of 16-byte records, coalesced): o + first diffuse slot, d,
// {-, item, bounce, phase | spec << 2}, RNG state.
struct WfRay {
    float4 *o, *d, *m;
    uint2 *st;
};

struct WfArgs {
    RenderArgs ra;
    WfRay cur, next;
    float4 *hit;         // {p.x, p.y, p.z, slot} of the current queue's rays
    uint32_t *cat_idx;   // category-major list of ray indices
    uint8_t *tag;        // per ray: category after the cast, alive flag after shading
    uint32_t *bcount;    // [kWfCats][nw] per-wave category counts, then [nw] survivor counts
    uint32_t *boff;      // exclusive scan of bcount (same layout)
    uint32_t *totals;    // [kWfCats] next queue length (host readback)
};

__device__ __forceinline__ Path load_ray(const WfRay &q, uint32_t i)
{
    const float4 o = q.o[i], d = q.d[i], m = q.m[i];
    const uint2 st = q.st[i];
    Path ps;
    ps.o = mk(o.x, o.y, o.z);
    ps.d = mk(d.x, d.y, d.z);
    ps.slot = __float_as_uint(o.w);
    ps.item = __float_as_uint(m.y);
    ps.bounce = __float_as_uint(m.z);
    const uint32_t ps_bits = __float_as_uint(m.w);
    ps.phase = ps_bits & 3u;
    ps.spec = ps_bits >> 2;
    ps.st = (uint64_t)st.x | ((uint64_t)st.y << 32);
    return ps;
}

__device__ __forceinline__ void store_ray(const WfRay &q, uint32_t i, const Path &ps)
{
    q.o[i] = make_float4(ps.o.x, ps.o.y, ps.o.z, __uint_as_float(ps.slot));
    q.d[i] = make_float4(ps.d.x, ps.d.y, ps.d.z, 0.f);
    q.m[i] = make_float4(0.f, __uint_as_float(ps.item), __uint_as_float(ps.bounce),
                         __uint_as_float(ps.phase | (ps.spec << 2)));
    q.st[i] = make_uint2((uint32_t)ps.st, (uint32_t)(ps.st >> 32));
}

__global__ __launch_bounds__(256) void wf_generate(WfArgs w, uint32_t base_item, uint32_t n_new, uint32_t dst0)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_new) return;
    const RenderArgs &a = w.ra;
    const uint32_t rows = a.npix / a.map.width;
    const Recip rw = recip((float)a.width), rh = recip((float)a.height);
    Path ps;
    ps.slot = 0;
    start_path(a, base_item + i, rows, rw, rh, mk(a.cam.eye[0], a.cam.eye[1], a.cam.eye[2]), ps);
    store_ray(w.cur, dst0 + i, ps);
}

// Global wave index (64-lane waves of the 1-D grid).
__device__ __forceinline__ uint32_t wave_id() { return (blockIdx.x * blockDim.x + threadIdx.x) >> 6; }

template <bool TREE, int LEAF>
__global__ __launch_bounds__(256) void wf_extend(WfArgs w, uint32_t n, uint32_t nw)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t wv = wave_id();
    if (wv >= nw) return;  // whole wave past the queue (wave-uniform); no block barriers below
    const bool act = i < n;  // every lane of a live wave takes part in the traversal
    const uint32_t ii = act ? i : 0u;
    const float4 o4 = w.cur.o[ii], d4 = w.cur.d[ii], m4 = w.cur.m[ii];
    const f3 o = mk(o4.x, o4.y, o4.z), d = mk(d4.x, d4.y, d4.z);
    CastDiag dg;
    const Hit h = find_closest<TREE, LEAF>(w.ra.scene.accel, o, d, act, dg);
    uint32_t cat = kWfCats;  // none
    if (act) {
        w.hit[i] = make_float4(h.t, 0.f, 0.f, __uint_as_float(h.idx));
        // category of the next shading step: the material switch of
        // TraceAndSampleColor (SingleThreadPathTracer.hpp:98-111) or the diffuse loop
        cat = 0;  // sky / miss / unknown material
        if ((__float_as_uint(m4.w) & 3u) == PH_DLOOP) {
            cat = 4;
        } else if (h.idx != kMiss) {
            const uint32_t mt = w.ra.scene.mat[h.idx];
            cat = mt == SPT_DIFFUSE_ID ? 1u : mt == SPT_REFLECTIVE_ID ? 2u : mt == SPT_REFRACTIVE_ID ? 3u : 0u;
        }
        w.tag[i] = (uint8_t)cat;
    }
#pragma unroll
    for (uint32_t c = 0; c < kWfCats; ++c) {
        const uint32_t k = (uint32_t)__popcll(__ballot(cat == c));
        if (__lane_id() == 0) w.bcount[(size_t)c * nw + wv] = k;
    }
}

// Category lists in queue order (per-wave offsets from the scan + mbcnt rank).
__global__ __launch_bounds__(256) void wf_split(WfArgs w, uint32_t n, uint32_t nw)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t wv = wave_id();
    if (wv >= nw) return;
    const uint32_t cat = i < n ? w.tag[i] : kWfCats;
#pragma unroll
    for (uint32_t c = 0; c < kWfCats; ++c) {
        const unsigned long long m = __ballot(cat == c);
        if (cat == c) w.cat_idx[w.boff[(size_t)c * nw + wv] + lane_rank(m)] = i;
    }
}

__global__ __launch_bounds__(256) void wf_shade(WfArgs w, uint32_t cat, uint32_t n_all, uint32_t nw)
{
    __shared__ uint32_t s_lds[256];  // wave-private scratch of the cooperative sampler
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t start = w.boff[(size_t)cat * nw];
    const uint32_t n = (cat + 1 < kWfCats ? w.boff[(size_t)(cat + 1) * nw] : n_all) - start;  // this category's rays
    if (j - __lane_id() >= n) return;  // whole wave past the list (wave-uniform)
    const bool act = j < n;
    const uint32_t i = act ? w.cat_idx[start + j] : 0u;
    Path ps = load_ray(w.cur, i);
    if (!act) ps.phase = PH_IDLE;
    const float4 h4 = w.hit[i];
    Hit h;
    h.idx = __float_as_uint(h4.w);
    h.best = 0.f;
    h.t = h4.x;
    unsigned long long done = 0, dropped = 0;
    shade_step(w.ra, ps, h, act, done, dropped, s_lds + (threadIdx.x & ~63u));
    if (act) {
        const bool alive = ps.phase != PH_IDLE;
        if (alive) store_ray(w.cur, i, ps);  // in place; compacted in queue order below
        w.tag[i] = alive ? 1u : 0u;
    }
    if (dropped) atomicAdd(&w.ra.counters[2], dropped);  // task mode only, rare
}

__global__ __launch_bounds__(256) void wf_count(WfArgs w, uint32_t n, uint32_t nw)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t wv = wave_id();
    if (wv >= nw) return;
    const uint32_t k = (uint32_t)__popcll(__ballot(i < n && w.tag[i] != 0u));
    if (__lane_id() == 0) w.bcount[(size_t)kWfCats * nw + wv] = k;
}

// Next queue length (host readback) and the pass statistics: rays cast = n,
// paths finished = n - survivors.
__global__ void wf_totals(WfArgs w, uint32_t n, uint32_t nw)
{
    const size_t last = (size_t)kWfCats * nw + nw - 1;
    const uint32_t alive = w.boff[last] + w.bcount[last];
    w.totals[0] = alive;
    atomicAdd(&w.ra.counters[0], (unsigned long long)n);
    atomicAdd(&w.ra.counters[1], (unsigned long long)(n - alive));
}

__global__ __launch_bounds__(256) void wf_compact(WfArgs w, uint32_t n, uint32_t nw)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t wv = wave_id();
    if (wv >= nw) return;
    const bool alive = i < n && w.tag[i] != 0u;
    const unsigned long long m = __ballot(alive);
    if (!alive) return;
    const uint32_t at = w.boff[(size_t)kWfCats * nw + wv] + lane_rank(m);
    w.next.o[at] = w.cur.o[i];
    w.next.d[at] = w.cur.d[i];
    w.next.m[at] = w.cur.m[i];
    w.next.st[at] = w.cur.st[i];
}

}  // namespace

size_t wavefront_scan_bytes(uint32_t cap)
{
    size_t bytes = 0;
    const uint32_t items = (kWfCats + 1) * (cap / 64 + 1);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (uint32_t *)nullptr, (uint32_t *)nullptr, items);
    return bytes;
}

hipError_t launch_wavefront_pass(const WavefrontBuffers &b, const RenderArgs &a, uint32_t cur, uint32_t n_cur,
                                 uint32_t gen_base, uint32_t gen_n, hipStream_t s)
{
    WfArgs w;
    w.ra = a;
    const uint32_t nxt = cur ^ 1u;
    w.cur = WfRay{b.o[cur], b.d[cur], b.m[cur], b.st[cur]};
    w.next = WfRay{b.o[nxt], b.d[nxt], b.m[nxt], b.st[nxt]};
    w.hit = b.hit;
    w.cat_idx = b.cat_idx;
    w.tag = b.tag;
    w.bcount = b.bcount;
    w.boff = b.boff;
    w.totals = b.counts;
    if (gen_n) hipLaunchKernelGGL(wf_generate, dim3((gen_n + 255) / 256), dim3(256), 0, s, w, gen_base, gen_n, n_cur);
    const uint32_t n = n_cur + gen_n;
    if (n == 0) return hipMemsetAsync(b.counts, 0, sizeof(uint32_t), s);
    const uint32_t nw = (n + 63) / 64;  // waves
    const dim3 grid((n + 255) / 256);
    size_t tmp = b.scan_bytes;
    if (a.scene.accel.tree)
        hipLaunchKernelGGL((wf_extend<true, (int)kClusterSlots>), grid, dim3(256), 0, s, w, n, nw);
    else if (a.scene.accel.leaf_slots == kFlatLeafSlots)
        hipLaunchKernelGGL((wf_extend<false, (int)kFlatLeafSlots>), grid, dim3(256), 0, s, w, n, nw);
    else
        hipLaunchKernelGGL((wf_extend<false, (int)kClusterSlots>), grid, dim3(256), 0, s, w, n, nw);
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.bcount, b.boff, kWfCats * nw, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(wf_split, grid, dim3(256), 0, s, w, n, nw);
    for (uint32_t c = 0; c < kWfCats; ++c) hipLaunchKernelGGL(wf_shade, grid, dim3(256), 0, s, w, c, n, nw);
    hipLaunchKernelGGL(wf_count, grid, dim3(256), 0, s, w, n, nw);
    tmp = b.scan_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, tmp, b.bcount + (size_t)kWfCats * nw,
                                         b.boff + (size_t)kWfCats * nw, nw, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(wf_totals, dim3(1), dim3(1), 0, s, w, n, nw);
    hipLaunchKernelGGL(wf_compact, grid, dim3(256), 0, s, w, n, nw);
    return hipGetLastError();
}

}  // namespace spt
