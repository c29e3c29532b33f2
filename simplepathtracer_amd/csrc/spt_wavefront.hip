// spt_wavefront.hip -- queue-based (wavefront) variant of the render loop.
//
// the design of RenderSegmentTask's material queues
// (TaskBasedPathTracer.hpp:54-193) on the GPU, to compare against the persistent
// megakernel.  The reference keeps per-material task vectors and runs one material
// at a time per pass.  Here every block of one launch per sample batch owns a ray
// queue in HBM (qcap rays) and runs passes over it with no host round trip:
//
//   top-up      new paths for the free positions, from one claim on the batch's
//               item counter (the only global atomic, one per block and pass);
//   per 256-ray chunk of the queue
//     cast      one FindClosestIntersectionSphere per ray; the ray's category
//               (sky/miss, diffuse first hit, mirror, glass, diffuse-loop step);
//     split     a counting sort of the chunk by category in LDS (wave ballots,
//               per-wave counts, block prefix), so each wave shades rays of one
//               material, like the reference's per-material loops;
//     shade     one shading step; finished paths write their sample word;
//     compact   the survivors (wave ballot ranks + the block's prefix) to the front
//               of the queue, in order.
//
// Queue lengths never leave the block, so nothing is read back and no block waits
// for another (an earlier version ran global passes with grid barriers in one
// cooperative launch: 7x the megakernel's frame time, one atomic per chunk on the
// pass's length).  Every path's arithmetic is the megakernel's own (spt_path.h:
// start_path, find_closest, shade_step) and its sample word sits at its item's slot,
// so frames are bit-identical to the megakernel's.
#include "spt_path.h"

#include <algorithm>
#include <mutex>

namespace spt {

namespace {

constexpr uint32_t kWfBlock = 256;
constexpr uint32_t kWfWaves = kWfBlock / 64;

struct WfQueue {
    float4 *o, *d;  // {o, first diffuse slot}, {d, item}
    uint4 *m;       // {RNG state lo, hi, bounce, phase | spec << 2}
};

struct WfArgs {
    RenderArgs ra;
    WfQueue q;        // the blocks' queues, qcap rays each
    uint32_t *state;  // [0] next batch item to start (claimed by the blocks)
    uint32_t qcap;    // rays per block queue (a multiple of kWfBlock)
};

__device__ __forceinline__ void load_ray(const WfQueue &q, uint32_t i, Path &ps)
{
    const float4 o = q.o[i], d = q.d[i];
    const uint4 m = q.m[i];
    ps.o = mk(o.x, o.y, o.z);
    ps.slot = __float_as_uint(o.w);
    ps.d = mk(d.x, d.y, d.z);
    ps.item = __float_as_uint(d.w);
    ps.st = (uint64_t)m.x | ((uint64_t)m.y << 32);
    ps.bounce = m.z;
    ps.phase = m.w & 3u;
    ps.spec = m.w >> 2;
}

__device__ __forceinline__ void store_ray(const WfQueue &q, uint32_t i, const Path &ps)
{
    q.o[i] = make_float4(ps.o.x, ps.o.y, ps.o.z, __uint_as_float(ps.slot));
    q.d[i] = make_float4(ps.d.x, ps.d.y, ps.d.z, __uint_as_float(ps.item));
    q.m[i] = make_uint4((uint32_t)ps.st, (uint32_t)(ps.st >> 32), ps.bounce, ps.phase | (ps.spec << 2));
}

// One block = one queue worker.  Per pass: top the block's queue up to qcap rays with
// new paths (one claim on the batch's item counter), then for each 256-ray chunk of
// the queue cast, sort by category in LDS, shade, and compact the survivors in queue
// order to the front of the same queue (in place: a chunk's survivors land at or
// before its own positions, all loaded before the first store).  A block leaves when
// its queue is empty and the items are exhausted.
template <bool TREE, int LEAF, bool GLANE>
__global__ __launch_bounds__(kWfBlock) void wf_render(WfArgs w)
{
    __shared__ float4 s_o[kWfBlock], s_d[kWfBlock];
    __shared__ uint4 s_m[kWfBlock];
    __shared__ float2 s_h[kWfBlock];                   // the cast's {t, slot} of the sorted rays
    __shared__ uint32_t s_lds[kWfBlock];               // wave-private scratch of the cooperative sampler
    __shared__ uint32_t s_cnt[kWfWaves][kWfCats + 1];  // per wave: category counts, survivors
    __shared__ uint32_t s_claim;

    typedef __attribute__((address_space(1))) uint32_t gu32;
    const RenderArgs &a = w.ra;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = __lane_id();
    const uint32_t rows = a.npix / a.map.width;
    const Recip rw = recip((float)a.width), rh = recip((float)a.height);
    const f3 eye = mk(a.cam.eye[0], a.cam.eye[1], a.cam.eye[2]);
    const size_t q0 = (size_t)blockIdx.x * w.qcap;
    const WfQueue q{w.q.o + q0, w.q.d + q0, w.q.m + q0};
    uint32_t len = 0;  // rays queued (block-uniform)
    unsigned long long cast = 0, finished = 0, done = 0, dropped = 0;
    for (;;) {
        // top-up: claim qcap - len items (the counter may run past n_items)
        if (tid == 0) s_claim = __hip_atomic_fetch_add((gu32 *)w.state, w.qcap - len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const uint32_t first = s_claim;
        const uint32_t got = first < a.n_items ? min(w.qcap - len, a.n_items - first) : 0u;
        const uint32_t n = len + got;
        if (n == 0u) break;
        uint32_t wp = 0;  // the next survivor's position (block-uniform)
        for (uint32_t base = 0; base < n; base += kWfBlock) {
            const uint32_t i = base + tid;
            const uint32_t live = min(n - base, kWfBlock);
            const bool act = i < n;
            Path ps;
            ps.phase = PH_IDLE;
            ps.item = ps.bounce = ps.spec = ps.slot = 0;
            ps.st = 0;
            ps.o = ps.d = mk(0.f, 0.f, 0.f);
            if (act) {
                if (i < len) {
                    load_ray(q, i, ps);
                } else {
                    start_path(a, first + (i - len), rows, rw, rh, eye, ps);
                    ps.slot = 0;
                }
            }
            CastDiag dg;
            // GLANE (trees the megakernel walks lane by lane, lane_walk_tree): each lane
            // walks layout 0 from global memory; otherwise the wave walk
            const Hit h = GLANE ? find_closest_lane<LEAF>(a.scene.accel, ps.o, ps.d, act, dg, (const uint32_t *)a.scene.accel.nodes)
                                : find_closest<TREE, LEAF>(a.scene.accel, ps.o, ps.d, act, dg);
            // category of the next shading step: the material switch of
            // TraceAndSampleColor (SingleThreadPathTracer.hpp:98-111) or the diffuse loop
            uint32_t cat = kWfCats;
            if (act) {
                cat = 0u;  // sky / miss / unknown material
                if (ps.phase == PH_DLOOP) {
                    cat = 4u;
                } else if (h.idx != kMiss) {
                    const uint32_t mt = a.scene.mat[h.idx];
                    cat = mt == SPT_DIFFUSE_ID ? 1u : mt == SPT_REFLECTIVE_ID ? 2u : mt == SPT_REFRACTIVE_ID ? 3u : 0u;
                }
            }
            // counting sort of the chunk by category: wave ballots, then the block prefix
            uint32_t rank = 0;
#pragma unroll
            for (uint32_t c = 0; c < kWfCats; ++c) {
                const unsigned long long m = __ballot(cat == c);
                if (lane == 0) s_cnt[wave][c] = (uint32_t)__popcll(m);
                if (cat == c) rank = lane_rank(m);
            }
            __syncthreads();
            if (act) {
                uint32_t pos = rank;
#pragma unroll
                for (uint32_t c = 0; c < kWfCats; ++c)
#pragma unroll
                    for (uint32_t v = 0; v < kWfWaves; ++v)
                        if (c < cat || (c == cat && v < wave)) pos += s_cnt[v][c];
                s_o[pos] = make_float4(ps.o.x, ps.o.y, ps.o.z, __uint_as_float(ps.slot));
                s_d[pos] = make_float4(ps.d.x, ps.d.y, ps.d.z, __uint_as_float(ps.item));
                s_m[pos] = make_uint4((uint32_t)ps.st, (uint32_t)(ps.st >> 32), ps.bounce, ps.phase | (ps.spec << 2));
                s_h[pos] = make_float2(h.t, __uint_as_float(h.idx));
            }
            __syncthreads();
            // shade the sorted chunk: lanes [0, live) hold rays, category by category
            const bool act2 = tid < live;
            Hit hh;
            hh.best = 0.f;
            hh.t = 0.f;
            hh.idx = kMiss;
            if (act2) {
                const float4 o = s_o[tid], d = s_d[tid];
                const uint4 m = s_m[tid];
                const float2 t = s_h[tid];
                ps.o = mk(o.x, o.y, o.z);
                ps.slot = __float_as_uint(o.w);
                ps.d = mk(d.x, d.y, d.z);
                ps.item = __float_as_uint(d.w);
                ps.st = (uint64_t)m.x | ((uint64_t)m.y << 32);
                ps.bounce = m.z;
                ps.phase = m.w & 3u;
                ps.spec = m.w >> 2;
                hh.t = t.x;
                hh.idx = __float_as_uint(t.y);
            } else {
                ps.phase = PH_IDLE;
            }
            shade_step(a, ps, hh, act2, done, dropped, s_lds + wave * 64u);
            // compaction: the survivors, in order, to the front of the queue
            const bool alive = act2 && ps.phase != PH_IDLE;
            const unsigned long long am = __ballot(alive);
            if (lane == 0) s_cnt[wave][kWfCats] = (uint32_t)__popcll(am);
            __syncthreads();
            uint32_t at = wp + lane_rank(am), tot = 0;
#pragma unroll
            for (uint32_t v = 0; v < kWfWaves; ++v) {
                const uint32_t k = s_cnt[v][kWfCats];
                if (v < wave) at += k;
                tot += k;
            }
            if (alive) store_ray(q, at, ps);
            wp += tot;
            __syncthreads();  // the chunk's LDS is reused by the next one; its stores precede the next loads
        }
        cast += n;
        finished += n - wp;
        len = wp;
    }
    (void)done;
    if (tid == 0) {
        atomicAdd(&a.counters[0], cast);
        atomicAdd(&a.counters[1], finished);
    }
    if (dropped) atomicAdd(&a.counters[2], dropped);  // task mode only, rare
}

template <bool TREE, int LEAF, bool GLANE>
uint32_t resident_blocks(int dev)
{
    // blocks per CU at this kernel's register / LDS footprint, per device (cached)
    static std::mutex mu;
    static int cached[64];
    std::lock_guard<std::mutex> lk(mu);
    if (dev < 0 || dev >= 64) return 0;
    if (cached[dev] == 0) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wf_render<TREE, LEAF, GLANE>, kWfBlock, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 0;
        cached[dev] = std::max(per_cu, 0) * std::max(cus, 0);
        if (cached[dev] == 0) cached[dev] = -1;
    }
    return cached[dev] > 0 ? (uint32_t)cached[dev] : 0u;
}

template <bool TREE, int LEAF, bool GLANE>
hipError_t launch(const WavefrontBuffers &b, const RenderArgs &a, hipStream_t s)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint32_t resident = resident_blocks<TREE, LEAF, GLANE>(dev);
    if (resident == 0) return hipErrorInvalidConfiguration;
    // one block per queue: as many as are resident at once (a block that waits for a
    // CU only starts later; no block waits for another)
    const uint32_t grid = std::max(1u, std::min(resident, b.cap / b.qcap));
    WfArgs w;
    w.ra = a;
    w.q = WfQueue{b.o, b.d, b.m};
    w.state = b.state;
    w.qcap = b.qcap;
    e = hipMemsetAsync(b.state, 0, kWfStateWords * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((wf_render<TREE, LEAF, GLANE>), dim3(grid), dim3(kWfBlock), 0, s, w);
    return hipGetLastError();
}

}  // namespace

uint32_t wavefront_blocks(const AccelView &ac, int dev)
{
    if (lane_walk_tree(ac)) return resident_blocks<true, (int)kClusterSlots, true>(dev);
    if (ac.tree) return resident_blocks<true, (int)kClusterSlots, false>(dev);
    if (ac.leaf_slots == kFlatLeafSlots) return resident_blocks<false, (int)kFlatLeafSlots, false>(dev);
    return resident_blocks<false, (int)kClusterSlots, false>(dev);
}

hipError_t launch_wavefront(const WavefrontBuffers &b, const RenderArgs &a, hipStream_t s)
{
    if (a.n_items == 0) return hipSuccess;
    if (lane_walk_tree(a.scene.accel)) return launch<true, (int)kClusterSlots, true>(b, a, s);
    if (a.scene.accel.tree) return launch<true, (int)kClusterSlots, false>(b, a, s);
    if (a.scene.accel.leaf_slots == kFlatLeafSlots) return launch<false, (int)kFlatLeafSlots, false>(b, a, s);
    return launch<false, (int)kClusterSlots, false>(b, a, s);
}

}  // namespace spt
