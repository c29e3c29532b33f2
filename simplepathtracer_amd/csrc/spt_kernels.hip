// spt_kernels.hip -- MI355X (gfx950) kernels of the SimplePathTracer render loop.
//
// render_kernel: persistent wavefront megakernel.  Each lane owns one
// (pixel, sample) path at a time and runs the reference's recursion
// (TraceAndSampleColor -> SampleColor{Diffuse,Reflective,Refractive,Skybox},
// SingleThreadPathTracer.hpp:11-112) as an iterative state machine: one
// FindClosestIntersectionSphere cast (Collision.hpp:87-109) followed by one
// shading step per loop iteration.  When a path ends its colour goes to a
// per-sample slot and the lane takes the next (pixel, sample) item; items are
// handed out by a wave-level ballot/mbcnt prefix over a block claimed from one
// global counter, so lanes never wait for the slowest path of their wave.
//
// Sphere data is read with wave-uniform scalar loads (s_load) -- the sphere
// index of the hot loop is the same for all lanes.  Small spheres sit in 8-slot
// clusters under a tree of expanded boxes walked by the whole wave without a
// stack (preorder + skip links); a subtree is skipped when no lane can pass any
// member's test or beat its current winner (spt_accel.cpp).
// render_kernel_lds walks large trees from a per-block LDS copy of the node table;
// the *_batch kernels render several host calls' rectangles in one launch
// (spt_batch.cpp render_batched).
//
// fold_kernel: RenderSegment's `pixelColor += sample` in sample order followed by
// `*= 1/g_samples` (SingleThreadPathTracer.hpp:121-134) or RenderSegmentTask's
// count-weighted resolve (TaskBasedPathTracer.hpp:196-205), plus WritePixel.
// Sums are formed in sample order, so results are bit-identical to the
// sequential reference loop whatever order the paths finished in.
#include "spt_path.h"

#include <algorithm>
#include <mutex>

namespace spt {


#ifndef SPT_WAVES_PER_EU
#define SPT_WAVES_PER_EU 0
#endif
// SGPR cap of the render kernels (with SPT_KERNARG_RELOAD); 0 = no cap.  80 lets 8
// waves per SIMD be resident, 81-96 seven, the uncapped 106 six; since the member
// pretest 96 (7 waves, fewer SGPR spills) measures faster than 80
#ifndef SPT_NUM_SGPR
#define SPT_NUM_SGPR 96
#endif
#if SPT_WAVES_PER_EU
#define SPT_RENDER_ATTR __attribute__((amdgpu_waves_per_eu(SPT_WAVES_PER_EU, SPT_WAVES_PER_EU)))
#elif SPT_NUM_SGPR
// the SGPR cap's wave count also bounds the VGPRs (7 waves: 72) so that registers
// never become the tighter limit
#define SPT_CAP_WAVES (800 / (((SPT_NUM_SGPR - 2 + 15) / 16) * 16 + 16) > 8 ? 8 : 800 / (((SPT_NUM_SGPR - 2 + 15) / 16) * 16 + 16))
#define SPT_RENDER_ATTR __attribute__((amdgpu_num_sgpr(SPT_NUM_SGPR), amdgpu_waves_per_eu(SPT_CAP_WAVES)))
#else
#define SPT_RENDER_ATTR
#endif

// LDS tree variant (SPT_LDS_TREE): blocks of kLdsBlock threads copy node layout 0
// into LDS once and walk it with broadcast LDS reads; two blocks per CU.
#ifndef SPT_LDS_BLOCK
#define SPT_LDS_BLOCK 1024
#endif
constexpr uint32_t kLdsBlock = SPT_LDS_BLOCK;
// 32-byte node records (pad included) per block: 2432 = 76 KiB, with the sampler's
// 4 KiB exactly half of the CU's 160 KiB
#ifndef SPT_LDS_NODES
#define SPT_LDS_NODES 2432
#endif
constexpr uint32_t kLdsNodeRecords = SPT_LDS_NODES;
// the LDS-tree session kernel (render_kernel_svc_lds) also holds its waves' job records
// (16 x kSvcRecWords words = 80 records' worth): its table is that much shorter, so that
// two blocks still fit a CU (at 81 920 B the compiler keeps 64 VGPRs, 8 waves per SIMD)
constexpr uint32_t kLdsSvcNodeRecords = kLdsNodeRecords - 80u;
// smallest tree walked from LDS: below it the 8 octant layouts (64 nodes: 16 KiB) fit
// the scalar cache
#ifndef SPT_LDS_MIN_NODES
#define SPT_LDS_MIN_NODES 64
#endif
constexpr uint32_t kLdsMinNodes = SPT_LDS_MIN_NODES;
// largest tree walked lane by lane from global memory; larger ones take the wave walk
// (stress scenes at 16 spp, lane / wave walk: 20 000 spheres, 4 083 nodes, 12.7 / 18.6
// ms; 30 000, 6 104: 15.6 / 20.1; 40 000, 8 115: 17.7 / 20.2; 50 000, 10 053: 23.8 /
// 21.2 -- the per-lane node reads outgrow the caches)
#ifndef SPT_GLANE_MAX_NODES
#define SPT_GLANE_MAX_NODES 9000
#endif
constexpr uint32_t kGlaneMaxNodes = SPT_GLANE_MAX_NODES;
#ifndef SPT_LANE_BUDGET
#define SPT_LANE_BUDGET 7
#endif
#ifndef SPT_REFILL_MIN
#define SPT_REFILL_MIN 16
#endif
// 1: the LDS tree is walked lane by lane (find_closest_lane; 0: the whole wave walks
// the union of its lanes' paths, find_closest)
#ifndef SPT_LANE_WALK
#define SPT_LANE_WALK 1
#endif
// 1: the wave-walk kernels start paths in primary batches (render_body, PRIM): 64 new
// paths at a time, all 64 lanes, cast and shaded once together, the survivors parked
// in a per-wave LDS queue that refills idle lanes
#ifndef SPT_PRIM
#define SPT_PRIM 1
#endif
// idle lanes needed before a refill from the primary queue (the queue's pops are cheap;
// SPT_REFILL_MIN rules the kernels without it)
#ifndef SPT_PRIM_REFILL_MIN
#define SPT_PRIM_REFILL_MIN 8
#endif

// A path parked in LDS (the primary queue of render_body): 12 words, structure of arrays
// over the wave's 64 rows (conflict-free b32 accesses).  Fields: item, st (2), o (3), d (3),
// slot, bounce, phase | spec << 2; the render service adds its job's counter (word 12).
constexpr uint32_t kParkWords = 12;
template <bool JOB = false>
__device__ __forceinline__ void park_path(uint32_t *q, uint32_t row, const Path &ps)
{
    if (JOB) q[12 * 64 + row] = ps.job;
    q[0 * 64 + row] = ps.item;
    q[1 * 64 + row] = (uint32_t)ps.st;
    q[2 * 64 + row] = (uint32_t)(ps.st >> 32);
    q[3 * 64 + row] = __float_as_uint(ps.o.x);
    q[4 * 64 + row] = __float_as_uint(ps.o.y);
    q[5 * 64 + row] = __float_as_uint(ps.o.z);
    q[6 * 64 + row] = __float_as_uint(ps.d.x);
    q[7 * 64 + row] = __float_as_uint(ps.d.y);
    q[8 * 64 + row] = __float_as_uint(ps.d.z);
    q[9 * 64 + row] = ps.slot;
    q[10 * 64 + row] = ps.bounce;
    q[11 * 64 + row] = ps.phase | (ps.spec << 2);
}
template <bool JOB = false>
__device__ __forceinline__ void unpark_path(const uint32_t *q, uint32_t row, Path &ps)
{
    if (JOB) ps.job = q[12 * 64 + row];
    ps.item = q[0 * 64 + row];
    ps.st = (uint64_t)q[1 * 64 + row] | ((uint64_t)q[2 * 64 + row] << 32);
    ps.o = mk(__uint_as_float(q[3 * 64 + row]), __uint_as_float(q[4 * 64 + row]), __uint_as_float(q[5 * 64 + row]));
    ps.d = mk(__uint_as_float(q[6 * 64 + row]), __uint_as_float(q[7 * 64 + row]), __uint_as_float(q[8 * 64 + row]));
    ps.slot = q[9 * 64 + row];
    ps.bounce = q[10 * 64 + row];
    const uint32_t w = q[11 * 64 + row];
    ps.phase = w & 3u;
    ps.spec = w >> 2;
}

// One kernel per traversal shape (flat list of 4- or 8-slot leaves, tree of
// 8-slot leaves), each with its own register allocation; launch_render picks.
// BATCH: the launch renders a.n_rects rectangles (a.rects, concurrent host calls
// batched by spt_batch.cpp); each refill then serves lanes from one claim only, and a
// claim's rectangle is looked up once per claim.
// The next claim of a launch (lane 0).  Items come from a.n_queues counters,
// one per XCD: queue k hands out [k * queue_items, (k + 1) * queue_items), so the
// device-scope atomics of the grid spread over 8 addresses instead of serialising on
// one.  A wave starts on queue `home` (blockIdx % n_queues: its XCD under round-robin
// dispatch) and moves on to the next queue when one is dry; n_items when all are.
__device__ __forceinline__ uint32_t claim_next(const RenderArgs &a, uint32_t home, uint32_t &qi)
{
    while (qi < a.n_queues) {
        uint32_t k = home + qi;
        if (k >= a.n_queues) k -= a.n_queues;
        const uint32_t lo = k * a.queue_items;
        const uint32_t len = lo < a.n_items ? min(a.queue_items, a.n_items - lo) : 0u;
        if (len != 0u) {
            const uint32_t c = atomicAdd(a.head + k * kQueueStride, a.claim);
            if (c < len) return lo + c;
        }
        ++qi;
    }
    return a.n_items;
}

// ---- render service (SVC): claims, publication, jobs, completion ----------------------
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// Reserve queue q's next claim: lane 0 issues the add and keeps its result (the claim
// is value * n_queues + q, published or not yet) in flight until the claim is taken.
// The address is formed in uniform code (scalar loads of the kernel arguments).
__device__ __forceinline__ uint32_t svc_reserve(uint32_t q, uint32_t lane, uint32_t old)
{
    kargs_t &k = *kernarg_args();
    uint32_t *const h = k.svc_ctl + q * kQueueStride;
    return lane == 0 ? atomicAdd(h, 1u) : old;
}
// the wave's LDS words after its job record: published claims and jobs as last seen, the
// current job and the first claim after it, the fold-ring entries it is done taking from
constexpr uint32_t kSvcSt = 28;
constexpr uint32_t kSvcRecWords = 40;  // LDS words per wave: job record (32) + state

// The published pair {claims, jobs} (one 64-bit sc1 load: the forwarder stores it after
// its records, sc1, with its stores drained -- MI355X_MICROARCH.md, hand-off table)
__device__ __forceinline__ unsigned long long svc_pub()
{
    kargs_t &k = *kernarg_args();
    return __hip_atomic_load((gu64 *)(k.svc_ctl + kSvcPub), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool svc_stopped()
{
    kargs_t &k = *kernarg_args();
    return __hip_atomic_load((gu32 *)(k.svc_ctl + kSvcStop), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// The forwarder (wave 0 of block 0 of a session; it renders nothing and takes no claim):
// polls the host's published pair and stop flag (system-scope loads of page-locked host
// memory), copies each newly published record and first claim into the device tables
// (sc1 stores, drained), then stores the device pair -- or, after the stop flag, the pair
// covering every publication and then the device stop flag -- and leaves on the stop or
// once no render wave is left (all left through the closing handshake).  Host publication
// thus needs no GPU queue: nothing a dispatch stuck behind the session's CU residency can
// hold back (spt_internal.h).
__device__ __forceinline__ void svc_forward(uint32_t lane)
{
    kargs_t &k = *kernarg_args();
    const gu32 *hw = (const gu32 *)k.svc_host;
    uint32_t fwd = 0;  // records forwarded
    for (uint32_t idle = 0;; ++idle) {
        const uint32_t st = lane == 0 ? __hip_atomic_load(hw + kSvcHostStop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
        const bool stop = __builtin_amdgcn_readfirstlane(st) != 0u;
        // after the stop flag, the pair is read after it (the host stores the pair first)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long pv =
            lane == 0 ? __hip_atomic_load((const gu64 *)(hw + kSvcHostPub), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                      : 0ull;
        const uint32_t plo = __builtin_amdgcn_readfirstlane((uint32_t)pv);
        const uint32_t phi = __builtin_amdgcn_readfirstlane((uint32_t)(pv >> 32));
        if (phi > fwd) {
            // records [fwd, phi): lanes 0-31 one record's words, lane 32 its first claim,
            // stored before the pair that publishes them
            const gu32 *hj = (const gu32 *)k.svc_host_jobs;
            const gu32 *hc = (const gu32 *)k.svc_host_job_claim;
            for (uint32_t j = fwd; j < phi; ++j) {
                if (lane < kSvcJobWords) {
                    const uint32_t w = __hip_atomic_load(hj + (size_t)j * kSvcJobWords + lane, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store((gu32 *)(k.svc_jobs + j) + lane, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else if (lane == kSvcJobWords) {
                    const uint32_t c = __hip_atomic_load(hc + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store((gu32 *)(k.svc_job_claim + j), c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0)
                __hip_atomic_store((gu64 *)(k.svc_ctl + kSvcPub), (unsigned long long)plo | ((unsigned long long)phi << 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fwd = phi;
            idle = 0;
        }
        if (stop) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_store((gu32 *)(k.svc_ctl + kSvcStop), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        const uint32_t live = lane == 0 ? __hip_atomic_load((gu32 *)(k.svc_ctl + kSvcLive), __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT)
                                        : 1u;
        if (__builtin_amdgcn_readfirstlane(live) == 0u) return;
        // ~0.1 us between polls while publications arrive, ~3 us once idle for a while
        if (idle < 256u)
            __builtin_amdgcn_s_sleep(2);
        else
            __builtin_amdgcn_s_sleep(127);
    }
}

// The job holding published claim nb, searched forward from job `cur` (a wave's claims
// only grow) over the first claims of the njobs published jobs, 64 per step (ballot of
// job_claim <= nb: a prefix, job_claim is increasing); its record is copied into the
// wave's LDS record `rec`, one word per lane.  Wave-uniform.
__device__ __forceinline__ uint32_t svc_find_job(uint32_t nb, uint32_t cur, uint32_t njobs, uint32_t *rec,
                                                 uint32_t lane)
{
    kargs_t &k = *kernarg_args();
    const gu32 *jc = (const gu32 *)k.svc_job_claim;
    for (;;) {
        const uint32_t j = cur + lane;
        const uint32_t v = j < njobs ? __hip_atomic_load(jc + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0xFFFFFFFFu;
        const unsigned long long le = __ballot(v <= nb);
        if (le != ~0ull || cur + 64u >= njobs) {
            if (le != 0ull) cur += 63u - (uint32_t)__builtin_clzll(le);  // (never 0: job_claim[cur] <= nb)
            break;
        }
        cur += 64u;
    }
    // words 0-23 (the fields start_path_svc reads); kSvcSt.. hold the wave's claim state
    const gu32 *src = (const gu32 *)(k.svc_jobs + cur);
    const uint32_t w = lane < 24u ? __hip_atomic_load(src + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    if (lane < 24u) rec[lane] = w;
    return __builtin_amdgcn_readfirstlane(cur);
}

// The colour of a sample word (code_word, spt_internal.h), with the render kernel's own
// operations: the sky as SampleColorSkybox computes it (SingleThreadPathTracer.hpp:11-14),
// a diffuse sample as the albedo * 0.5 (line 24) halved once more per further bounce
// (line 31), bit for bit.  Halving is exact while the value stays normal, so j halvings
// are one multiply by 2^-j when the result is normal (or 0 / inf / NaN); otherwise (a
// denormal result: each halving may round) they are done one at a time.
__device__ __forceinline__ float halve_n(float x, uint32_t j)
{
    if (j <= 126u) {
        const float r = x * __uint_as_float((127u - j) << 23);
        if (__builtin_fabsf(r) >= 0x1p-126f || x == 0.f || !__builtin_isfinite(x)) return r;
    }
    for (uint32_t i = 0; i < j; ++i) x = x * 0.5f;
    return x;
}
__device__ __forceinline__ f3 decode_sample(const FoldArgs &a, uint32_t w)
{
    const uint32_t c = word_code(w);
    if (c == 0u) {
        const float k = __uint_as_float(w);
        return mul(mk(a.sky[0] * k, a.sky[1] * k, a.sky[2] * k), 0.5f);
    }
    if (c == 1u) return mk(0.f, 0.f, 0.f);
    uint32_t j, slot;
    diffuse_decode(c, a.code_div, j, slot);
    const float4 sh = a.shade[slot];
    return mk(halve_n(sh.x * 0.5f, j), halve_n(sh.y * 0.5f, j), halve_n(sh.z * 0.5f, j));
}

// decode_sample for a run of words without branches around the loads: the shading-table
// reads of all N words are issued together (slot 0 stands in for sky and zero words), the
// colours selected afterwards; only denormal halvings (halve_n's slow path) branch.
template <int N>
__device__ __forceinline__ void decode_run(const FoldArgs &a, const uint32_t (&w)[N], f3 (&col)[N])
{
    uint32_t c[N], j[N];
    float4 sh[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        c[i] = word_code(w[i]);
        uint32_t slot;
        diffuse_decode(c[i] >= 2u ? c[i] : 2u, a.code_div, j[i], slot);
        sh[i] = a.shade[slot];
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float k = __uint_as_float(w[i]);
        const f3 s = mul(mk(a.sky[0] * k, a.sky[1] * k, a.sky[2] * k), 0.5f);
        const f3 d = mk(halve_n(sh[i].x * 0.5f, j[i]), halve_n(sh[i].y * 0.5f, j[i]), halve_n(sh[i].z * 0.5f, j[i]));
        col[i] = c[i] == 0u ? s : c[i] == 1u ? mk(0.f, 0.f, 0.f) : d;
    }
}

// words loaded ahead per thread in the fold (a multiple of 8): small folds (the drop-in's
// batches of one or two tiles) have few threads, and each is bound by its loads' latency
#ifndef SPT_FOLD_RUN
#define SPT_FOLD_RUN 8
#endif
// words decoded together (their shading-table reads in flight at once)
constexpr int kFoldDecode = SPT_FOLD_RUN < 8 ? SPT_FOLD_RUN : 8;
static_assert(SPT_FOLD_RUN % kFoldDecode == 0, "fold runs are decoded kFoldDecode words at a time");

// RenderSegmentTask's colorIndex aliasing (TaskBasedPathTracer.hpp:103,186,196-205) for
// output index p of a W x H call: colors[p] collects every pixel (dx, dy) of the call with
// dx + dy * H == p, and the resolve writes colors[p] to pixel (p % W, p / W).  Within a
// sample the sources reach colors[p] in the order of their (key, pixel) (finish_step), so
// each sample's sources are added in that order.  No source: 0 samples, and 0 * (1.f / 0)
// is NaN, as in the reference.  The sources' slots are those of rows [row0, row0 + rows)
// of the launch (the call's own rows, or a range of them: spt_render_frame).
__device__ __forceinline__ void alias_accumulate(const FoldArgs &a, const uint32_t *samples, uint32_t p, uint32_t W,
                                                 uint32_t H, uint32_t row0, uint32_t rows, uint32_t S, float4 &acc)
{
    const uint32_t dy_lo = p >= W ? (p - W + H) / H : 0u;
    const uint32_t dy_hi = min(H - 1u, p / H);
    const uint32_t ns = dy_hi + 1u - dy_lo;  // sources: pixels (p - dy H, dy)
    const uint2 *s2 = (const uint2 *)samples;
    auto add = [&](uint32_t w) {
        const f3 c = decode_sample(a, w);
        acc.x = acc.x + c.x;
        acc.y = acc.y + c.y;
        acc.z = acc.z + c.z;
        acc.w = acc.w + 1.f;
    };
    constexpr uint32_t kSrc = 4;  // sources kept in registers (config 2's tiles: <= 2)
    if (ns <= kSrc) {
        // the sources' slot bases once; per sample their keys, added in (key, pixel)
        // order (pixel order = dy order when W > H, reversed when W < H)
        uint32_t sq[kSrc], sst[kSrc];
#pragma unroll
        for (uint32_t j = 0; j < kSrc; ++j) {
            const uint32_t dy = j < ns ? dy_lo + j : dy_lo;
            ts_slot_base(dy - row0, p - dy * H, W, rows, S, sq[j], sst[j]);
        }
        const bool rev = W < H;
        for (uint32_t k = 0; k < S; ++k) {
            uint2 v[kSrc];
#pragma unroll
            for (uint32_t j = 0; j < kSrc; ++j) v[j] = j < ns ? s2[sq[j] + k * sst[j]] : make_uint2(0u, 0u);
            uint32_t done = 0;  // sources already added (bit j)
            for (uint32_t t = 0; t < ns; ++t) {
                uint32_t bj = kSrc, bk = 0, bw = 0;  // the next source: index, key, word
#pragma unroll
                for (uint32_t j = 0; j < kSrc; ++j) {
                    const bool cand = j < ns && v[j].y != 0u && !((done >> j) & 1u);
                    const bool before = bj == kSrc || v[j].y < bk || (v[j].y == bk && rev);
                    if (cand && before) {
                        bj = j;
                        bk = v[j].y;
                        bw = v[j].x;
                    }
                }
                if (bj == kSrc) break;
                done |= 1u << bj;
                add(bw);
            }
        }
    } else {
        for (uint32_t k = 0; k < S; ++k) {
            uint64_t prev = 0;  // (key << 32 | pixel) of the last source added
            for (uint32_t t = dy_lo; t <= dy_hi; ++t) {
                uint64_t best = ~0ull;
                uint32_t best_slot = 0;
                for (uint32_t dy = dy_lo; dy <= dy_hi; ++dy) {
                    const uint32_t dx = p - dy * H;  // source pixel (dx, dy)
                    uint32_t sq0, sst;
                    ts_slot_base(dy - row0, dx, W, rows, S, sq0, sst);
                    const uint32_t q = sq0 + k * sst;
                    const uint32_t key = s2[q].y;
                    const uint64_t kp = ((uint64_t)key << 32) | (dy * W + dx);
                    if (key != 0u && kp > prev && kp < best) {
                        best = kp;
                        best_slot = q;
                    }
                }
                if (best == ~0ull) break;
                add(s2[best_slot].x);
                prev = best;
            }
        }
    }
}

// RenderSegment's / RenderSegmentTask's resolve of local pixel (lr, col) of a region
// (map, `rows` rows, alias: task mode on a non-square tile) whose slots start at
// `samples` (item order of a batch of a.spp_batch samples: ts_slot_base); local float4
// output at out_rgba[lr * width + col].
__device__ __forceinline__ void fold_pixel(const FoldArgs &a, const uint32_t *samples, const RowMap &map,
                                           uint32_t rows, int alias, uint32_t lr, uint32_t col, float4 *out_rgba,
                                           uint8_t *out_rgb8)
{
    const uint32_t W = map.width, S = a.spp_batch;
    const uint32_t p = lr * W + col;
    float4 acc = a.first ? make_float4(0.f, 0.f, 0.f, 0.f) : a.acc[p];
    uint32_t q0, step;
    ts_slot_base(lr, col, W, rows, S, q0, step);
    if (a.mode == 0) {
        // RenderSegment: one word per slot, every sample counts.  Runs of kFoldRun words
        // are loaded before any is decoded (the loads of a run are in flight together),
        // then decoded kFoldDecode (8) at a time
        constexpr int kFoldRun = SPT_FOLD_RUN;
        uint32_t k = 0;
        for (; k + kFoldRun <= S; k += kFoldRun) {
            uint32_t w[kFoldRun];
#pragma unroll
            for (int i = 0; i < kFoldRun; ++i) w[i] = samples[q0 + (k + i) * step];
#pragma unroll
            for (int g = 0; g < kFoldRun; g += kFoldDecode) {
                uint32_t w8[kFoldDecode];
#pragma unroll
                for (int i = 0; i < kFoldDecode; ++i) w8[i] = w[g + i];
                f3 c[kFoldDecode];
                decode_run<kFoldDecode>(a, w8, c);
#pragma unroll
                for (int i = 0; i < kFoldDecode; ++i) {
                    acc.x = acc.x + c[i].x;
                    acc.y = acc.y + c[i].y;
                    acc.z = acc.z + c[i].z;
                    acc.w = acc.w + 1.f;
                }
            }
        }
        for (; k < S; ++k) {
            const f3 c = decode_sample(a, samples[q0 + k * step]);
            acc.x = acc.x + c.x;
            acc.y = acc.y + c.y;
            acc.z = acc.z + c.z;
            acc.w = acc.w + 1.f;
        }
    } else if (!alias) {
        // RenderSegmentTask on a square tile: pixel p is colors[p]; key 0 marks a dropped path
        const uint2 *s2 = (const uint2 *)samples;
        for (uint32_t k = 0; k < S; ++k) {
            const uint2 v = s2[q0 + k * step];
            if (v.y != 0u) {
                const f3 c = decode_sample(a, v.x);
                acc.x = acc.x + c.x;
                acc.y = acc.y + c.y;
                acc.z = acc.z + c.z;
                acc.w = acc.w + 1.f;
            }
        }
    } else {
        alias_accumulate(a, samples, p, W, rows, 0u, rows, S, acc);
    }
    if (!a.last) {
        a.acc[p] = acc;
        if (!a.preview) return;
    }
    // RenderSegment: *= (1.f / g_samples) (line 133); RenderSegmentTask: *= 1.f / samples[i]
    // (line 198).  s_done == g_samples after the last batch; a progressive preview after
    // s_done samples is the render at g_samples = s_done, bit for bit (keyed samples).
    const float scale = a.mode == 0 ? 1.f / (float)a.s_done : 1.f / acc.w;
    const float r = acc.x * scale, g = acc.y * scale, b = acc.z * scale;
    if (out_rgba) out_rgba[p] = make_float4(r, g, b, 0.f);
    if (out_rgb8) {
        const uint32_t x = map.x0 + col;
        const uint32_t y = row_of(map, lr);
        const size_t gi = (size_t)3 * ((size_t)(a.height - 1u - y) * a.width + x);
        out_rgb8[gi + 0] = gamma_byte(r);
        out_rgb8[gi + 1] = gamma_byte(g);
        out_rgb8[gi + 2] = gamma_byte(b);
    }
}

// 1 (default): the service stores sample words write-through (sc1), and a completion
// count needs only the wave's own drain; 0: plain stores and an agent release (buffer_wbl2,
// a write-back of the XCD's whole L2) before every count
#ifndef SPT_SVC_WT
#define SPT_SVC_WT 1
#endif

// Publish `cnt` finished samples of completion counter `idx`: every sample word the wave
// stored is drained (write-through stores: in memory once drained; else written back by
// an agent release: the fold runs on any XCD) before the add (MI355X_MICROARCH.md
// hand-off table, each storing wave signalling for itself; Compiler hazard: the asm wait
// after the fence).
__device__ __forceinline__ void svc_flush(uint32_t idx, uint32_t cnt, uint32_t lane)
{
    if (cnt == 0u) return;
    kargs_t &k = *kernarg_args();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!SPT_SVC_WT) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (lane == 0) __hip_atomic_fetch_add((gu32 *)(k.svc_done + idx), cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k.svc_trace && lane == 0) atomicMax(k.svc_trace + 4u * idx + 2u, __builtin_amdgcn_s_memrealtime());
}

template <bool TREE, int LEAF, bool LDSN, uint32_t BLOCK, bool BATCH = false, bool GLANE = false, bool SVC = false>
__device__ __forceinline__ void render_body(const RenderArgs &a)
{
    static_assert(!SVC || (!GLANE && !BATCH && (LDSN || SPT_PRIM)),
                  "the render service runs the wave-walk kernel or the LDS lane walk");
    const uint32_t lane = __lane_id();
    const uint32_t rows = SVC ? 0u : a.npix / a.map.width;  // region rows (uniform; SVC: per job)

    __shared__ uint32_t s_lds[BLOCK];  // wave-private scratch of the cooperative sampler
    __shared__ uint4 s_nodes[LDSN ? 2 * (SVC ? kLdsSvcNodeRecords : kLdsNodeRecords) : 1];
    // the LDS copy holds byte-offset skip links when only lane_cast walks it
    constexpr bool LDS_BYTES = LDSN && SPT_LANE_WALK && SPT_LANE_BUDGET > 0;
    // Primary batches (SPT_PRIM; the wave-walk kernels): when idle lanes want
    // more paths than the wave's queue holds, every lane parks its own path in the queue
    // rows, takes a NEW item (64 consecutive items: one sample of one 8x8 tile) and the
    // wave runs one ordinary iteration -- cast + shading step -- over those 64 primary
    // rays; then each lane takes its own path back and the survivors (paths not finished
    // by their first shading step) fill the queue, from which idle lanes are refilled.
    // The primary cast is one coherent bundle from the eye (the wave walk's union of
    // leaves is about a single ray's), and every path enters the main loop one cast in.
    // Per path the arithmetic and its order are unchanged: bit-identical frames.
    constexpr bool PRIM = SPT_PRIM && !LDSN && !GLANE;
    constexpr uint32_t PW = kParkWords + (SVC ? 1u : 0u);  // parked words per path
    __shared__ uint32_t s_park[PRIM ? (BLOCK / 64u) * PW * 64u : 1];
    uint32_t *const park = s_park + (PRIM ? (threadIdx.x >> 6) * PW * 64u : 0u);
    // SVC: the wave's copy of its current job's record (svc_find_job, words 0-23) and its
    // claim state (words kSvcSt..31: kept in LDS, not SGPRs, since only claims read them)
    __shared__ uint32_t s_rec[SVC ? (BLOCK / 64u) * kSvcRecWords : 1];
    uint32_t *const rec = s_rec + (SVC ? (threadIdx.x >> 6) * kSvcRecWords : 0u);
    if (SVC && lane < kSvcRecWords - kSvcSt) rec[kSvcSt + lane] = 0u;
    // the session's forwarder: wave 0 of block 0 (before any claim is reserved).  The
    // LDS-tree session's forwarder first joins its block's node-table copy (its barrier)
    if (SVC && !LDSN && blockIdx.x == 0u && (threadIdx.x >> 6) == 0u) {
        svc_forward(lane);
        return;
    }
    uint32_t q_n = 0, q_pos = 0;  // the wave's queue: rows [q_pos, q_n) hold parked paths
    if (LDSN) {
        // the host launches this variant only when n_nodes + 1 <= kLdsNodeRecords
        const uint4 *src = (const uint4 *)a.scene.accel.nodes;
        const uint32_t n4 = 2u * (a.scene.accel.n_nodes + 1u);
        for (uint32_t k = threadIdx.x; k < n4; k += BLOCK) {
            uint4 v = src[k];
            // the lane walk's copy: skip links as byte offsets (lane_cast BYTES)
            if (LDS_BYTES && (k & 1u)) v.x <<= 5;
            s_nodes[k] = v;
        }
        __syncthreads();
        if (SVC && blockIdx.x == 0u && (threadIdx.x >> 6) == 0u) {
            svc_forward(lane);
            return;
        }
    }
    Path ps;
    ps.phase = PH_IDLE;
    ps.item = ps.bounce = ps.spec = 0;
    ps.st = 0;
    ps.o = ps.d = mk(0.f, 0.f, 0.f);
    ps.slot = 0;
    ps.job = 0;

    // Items are handed out in claims of a.claim from one global counter; each wave
    // keeps the next claim in flight (lane 0) so the atomic's latency is hidden.
    uint32_t blk_cur = 0, blk_end = 0;
    uint32_t pend = 0;
    uint32_t rect = 0;  // BATCH: rectangle of the current claim
    const uint32_t home = blockIdx.x % a.n_queues;
    uint32_t qi = 0;  // queues tried after the home queue ran dry (lane 0)
    if (SVC)
        pend = svc_reserve(home, lane, 0u);
    else if (lane == 0)
        pend = claim_next(a, home, qi);
    bool exhausted = false;  // SVC: no published claim right now (the reservation waits)
    // SVC: the wave's finished samples not yet added to completion counter acc_idx
    uint32_t acc_idx = 0, acc_cnt = 0;
    unsigned long long casts = 0, done = 0, dropped = 0;
    struct {
        unsigned long long iters = 0, cast = 0, shade = 0, refill = 0;  // SPT_DIAG counts and s_memtime split
        // the primary batches' share: iterations, nodes, spheres, update branches, cast cycles
        unsigned long long p_iters = 0, p_nodes = 0, p_spheres = 0, p_branches = 0, p_cast = 0;
        unsigned long long s_rounds[3] = {0, 0, 0};  // sampler calls, cooperative rounds after round 0, cycles
        unsigned long long t_iters = 0, t_live = 0;  // iterations after the items ran out, their live lanes
    } dc;
    CastDiag dg;
    // resumable lane walk (SPT_LANE_BUDGET): the cast state of lanes whose walk ran
    // out of its iteration budget, continued on the next iteration
    Hit hres;
    hres.idx = kMiss;
    hres.best = FLT_MAX;
    hres.t = 0.f;
    uint32_t li = 0, lleaf = kNoSlot, lleaf2 = kNoSlot;
    bool fresh = true;
#if SPT_DIAG
    unsigned long long d_t0 = __builtin_amdgcn_s_memtime();
#define SPT_STAMP(acc)                                              \
    do {                                                            \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        acc += t_ - d_t0;                                           \
        d_t0 = t_;                                                  \
    } while (0)
#else
#define SPT_STAMP(acc) \
    do {               \
    } while (0)
#endif

    // items of the launch for the lanes of `need` (ballot + prefix rank over the current
    // claim, then the claim in flight); 0xFFFFFFFF for lanes that get none
    auto take_items = [&](unsigned long long need) -> uint32_t {
        const uint32_t cnt = (uint32_t)__popcll(need);
        const uint32_t rank = lane_rank(need);
        const uint32_t avail = blk_end - blk_cur;
        uint32_t mine = 0xFFFFFFFFu;
        if (rank < avail) mine = blk_cur + rank;
        if (avail >= cnt) {
            blk_cur += cnt;
        } else {
            // switch to the claim in flight and put the next one in flight
            const uint32_t nb = __builtin_amdgcn_readfirstlane(pend);
            if (nb < a.n_items && lane == 0) pend = claim_next(a, home, qi);
            if (nb >= a.n_items) {
                exhausted = true;
                blk_cur = blk_end = 0;
            } else {
                const uint32_t ne = min(nb + a.claim, a.n_items);
                const uint32_t r2 = rank - avail;
                if (rank >= avail && r2 < ne - nb) mine = nb + r2;
                blk_cur = nb + min(cnt - avail, ne - nb);
                blk_end = ne;
            }
        }
        return __builtin_amdgcn_inverse_ballot_w64(need) ? mine : 0xFFFFFFFFu;
    };

    // BATCH: the claim in flight becomes current (with its rectangle), the next one goes
    // in flight
    auto next_claim = [&]() {
        const uint32_t nb = __builtin_amdgcn_readfirstlane(pend);
        if (nb < a.n_items && lane == 0) pend = claim_next(a, home, qi);
        if (nb >= a.n_items) {
            exhausted = true;
        } else {
            blk_cur = nb;
            blk_end = min(nb + a.claim, a.n_items);
            rect = find_rect(nb);
        }
    };

    // SVC: the reserved claim becomes current once published (re-reading the published
    // pair when it is beyond the last one seen), the next one is reserved, and the job
    // record of a claim past the current job is looked up; else exhausted (waiting)
    auto next_claim_svc = [&]() {
        uint32_t *const st = rec + kSvcSt;
        const uint32_t nb = __builtin_amdgcn_readfirstlane(pend) * a.n_queues + home;
        uint32_t pc = __builtin_amdgcn_readfirstlane(st[0]);
        if (nb >= pc) {
            const unsigned long long p = svc_pub();
            pc = __builtin_amdgcn_readfirstlane((uint32_t)p);
            const uint32_t pj = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
            if (lane == 0) {
                st[0] = pc;
                st[1] = pj;
            }
        }
        exhausted = nb >= pc;
        if (exhausted) return;
        pend = svc_reserve(home, lane, pend);
        if (nb >= __builtin_amdgcn_readfirstlane(st[3])) {
            const uint32_t cur = svc_find_job(nb, __builtin_amdgcn_readfirstlane(st[2]),
                                              __builtin_amdgcn_readfirstlane(st[1]), rec, lane);
            const uint32_t ce = __builtin_amdgcn_readfirstlane(rec[7]);
            if (lane == 0) {
                st[2] = cur;
                st[3] = ce;
            }
        }
        blk_cur = nb * a.claim;
        blk_end = min(blk_cur + a.claim, __builtin_amdgcn_readfirstlane(rec[1]));
        kargs_t &kt = *kernarg_args();
        if (kt.svc_trace && lane == 0) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            unsigned long long *tr = kt.svc_trace + 4u * rec[3];
            atomicMin(tr, t);
            atomicMax(tr + 1, t);
            // per claim (SPT_SVC_TRACE_FILE): its take time, the taking block in the top bits
            if (nb < kSvcTraceClaims)
                kt.svc_trace[4u * 4096u + nb] = (t & 0xFFFFFFFFFFull) | ((unsigned long long)blockIdx.x << 40);
        }
    };

    for (;;) {
        // ---- refill: hand out (pixel, sample) items to idle lanes (ballot + prefix)
        // idle lanes wait until SPT_REFILL_MIN of them (or the whole wave) can be
        // refilled together: the refill's primary-ray code then runs a quarter as
        // often for ~4 more idle lanes per iteration (config 2 -2%, config 5 -1.5%)
        unsigned long long need = __ballot(ps.phase == PH_IDLE);
        if (__popcll(need) < (PRIM ? SPT_PRIM_REFILL_MIN : SPT_REFILL_MIN) && need != ~0ull) need = 0ull;
        bool prim_iter = false;  // PRIM: this iteration runs a primary batch
        uint32_t pxy = 0;        // PRIM: the lane's pixel in the batch (y << 16 | x)
        if (PRIM) {
            if (need != 0ull) {
                const uint32_t cnt = (uint32_t)__popcll(need);
                const uint32_t rank = lane_rank(need);
                const uint32_t take = min(cnt, q_n - q_pos);
                if (ps.phase == PH_IDLE && rank < take) unpark_path<SVC>(park, q_pos + rank, ps);
                q_pos += take;
                bool more = !exhausted;
                if (SVC && cnt > take) {
                    if (blk_cur == blk_end) next_claim_svc();
                    more = blk_cur < blk_end;
                }
                if (cnt > take && more) {
                    // the queue is empty: park every lane's own path in its own row and
                    // start 64 new paths (wave-uniform)
                    park_path<SVC>(park, lane, ps);
                    // the own path lives in LDS across the batch, not in registers
                    asm volatile("" ::: "memory");
                    ps.phase = PH_IDLE;
                    if (SVC) {
                        // claims are multiples of 64 items and never span two jobs: a batch
                        // is 64 items of one claim (fewer at a job's end)
                        const uint32_t n = min(64u, blk_end - blk_cur);
                        const uint32_t mine = blk_cur + lane;
                        blk_cur += n;
                        if (lane < n) start_path_svc(mine, rec, ps, &pxy);
                    } else if (BATCH) {
                        // claims are multiples of 64 items and never span two rectangles:
                        // a batch is 64 items of one claim (fewer at the launch's end)
                        if (blk_cur == blk_end) next_claim();
                        if (!exhausted) {
                            const uint32_t n = min(64u, blk_end - blk_cur);
                            const uint32_t mine = blk_cur + lane;
                            blk_cur += n;
                            if (lane < n) start_path_rect(mine, rect, ps, &pxy);
                        }
                    } else {
                        const uint32_t mine = take_items(~0ull);
                        if (mine != 0xFFFFFFFFu) start_path_kernarg(mine, rows, ps, &pxy);
                        if ((SPT_DUP & 4) && mine != 0xFFFFFFFFu) {
                            Path p2;
                            uint32_t pxy2 = 0;
                            start_path_kernarg(opaque_v(mine), rows, p2, &pxy2);
                            sink_v(p2.d.x);
                            sink_v(p2.d.y);
                            sink_v(p2.d.z);
                            sink_v(p2.st);
                            sink_v(pxy2);
                        }
                    }
                    prim_iter = true;
                }
            }
        } else if (SVC && !PRIM && need != 0ull) {
            // the LDS-tree session: idle lanes take items of the current claim, then of the
            // next published one (a claim never spans two jobs: each lane starts from the
            // job record current when it takes its item)
            // (one claim per refill: lanes left over take the next claim next iteration)
            if (blk_cur == blk_end) next_claim_svc();
            if (blk_cur < blk_end) {
                const uint32_t take = min((uint32_t)__popcll(need), blk_end - blk_cur);
                const uint32_t rank = lane_rank(need);
                if (__builtin_amdgcn_inverse_ballot_w64(need) && rank < take) start_path_svc(blk_cur + rank, rec, ps);
                blk_cur += take;
            }
        } else if (BATCH && need != 0ull && !exhausted) {
            if (blk_cur == blk_end) next_claim();
            if (!exhausted) {
                const uint32_t take = min((uint32_t)__popcll(need), blk_end - blk_cur);
                const uint32_t rank = lane_rank(need);
                const uint32_t mine = blk_cur + rank;
                blk_cur += take;
                if (ps.phase == PH_IDLE && rank < take) {
                    start_path_rect(mine, rect, ps);
                }
            }
        } else if (!BATCH && need != 0ull && !exhausted) {
            const uint32_t mine = take_items(need);
            if (mine != 0xFFFFFFFFu) start_path_kernarg(mine, rows, ps);
        }
        const unsigned long long live = __ballot(ps.phase != PH_IDLE);
        if (live == 0ull) {
            if (PRIM && prim_iter) {
                // no item was left for the batch: the lanes' own paths back
                unpark_path<SVC>(park, lane, ps);
                q_n = q_pos = 0;
                continue;
            }
            if (SVC && q_pos == q_n) {
                // no path and no published claim: publish the finished samples, then wait
                // for a publication or the stop flag (read before the last look at the
                // published pair: jobs are published before the stop).  After kSvcIdleTicks
                // without work the wave may leave through the closing handshake with the
                // host (spt_internal.h kSvcIdleTicks), then the watchdog word tells the host.
                svc_flush(acc_idx, acc_cnt, lane);
                acc_cnt = 0;
                unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                bool leave = false;
                bool closing = false;  // this wave has raised the closing flag
                uint32_t committed = 0;
                for (;;) {
                    // the stop flag is stored after every publication: once it is seen, the
                    // published pair must be read after it (the two loads would otherwise be
                    // in flight together, and the pair's could return a value older than the
                    // flag's, leaving a published reservation behind)
                    const bool stop = svc_stopped();
                    if (stop) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    }
                    if (closing) {
                        // the jobs the host has committed to this session, read after the
                        // closing store reached host memory; the published pair is read
                        // after this (next_claim_svc re-reads it: the wave is exhausted)
                        kargs_t &k = *kernarg_args();
                        const uint32_t c = lane == 0 ? __hip_atomic_load((gu32 *)(k.svc_host + kSvcHostCommitted),
                                                                         __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM)
                                                     : 0u;
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        committed = __builtin_amdgcn_readfirstlane(c);
                    }
                    next_claim_svc();
                    if (!exhausted) break;
                    if (stop) {
                        leave = true;
                        break;
                    }
                    if (closing) {
                        // every committed job published and none holds the wave's reserved
                        // claim: the host publishes nothing more to this session (it saw the
                        // flag, or the wave saw its commit), so the wave may leave
                        if (__builtin_amdgcn_readfirstlane(rec[kSvcSt + 1]) >= committed) {
                            kargs_t &k = *kernarg_args();
                            if (lane == 0)
                                __hip_atomic_store((gu32 *)(k.svc_host + kSvcHostWatchdog), 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_SYSTEM);
                            leave = true;
                            break;
                        }
                        // a committed job is not published yet (its publish launch is still
                        // queued): keep waiting for it
                        closing = false;
                        t0 = __builtin_amdgcn_s_memrealtime();
                    } else if (__builtin_amdgcn_s_memrealtime() - t0 > kSvcIdleTicks) {
                        // raise the closing flag: a system-scope store to host memory, drained
                        // before the committed count is read
                        kargs_t &k = *kernarg_args();
                        if (lane == 0)
                            __hip_atomic_store((gu32 *)(k.svc_host + kSvcHostClosing), 1u, __ATOMIC_SEQ_CST,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
                        closing = true;
                        continue;
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
                if (leave) break;
                continue;
            }
            if (exhausted && q_pos == q_n) break;
            continue;
        }
        SPT_STAMP(dc.refill);
#if SPT_DIAG
        const unsigned long long d_n0 = dg.nodes, d_s0 = dg.spheres, d_b0 = dg.branches, d_c0 = dc.cast;
#endif
        // the lane walks are resumable: a lane still walking after SPT_LANE_BUDGET walk
        // iterations and leaf passes keeps its cast state (winner, node, parked leaves)
        // and continues it next iteration while the other lanes shade and refill, so a
        // few long walks (grazing rays) do not hold the wave (config 5: 97.5 -> 90 ms)
        constexpr bool RES = SPT_LANE_BUDGET > 0 && (LDSN || GLANE);
        if (!RES) casts += (unsigned long long)__popcll(live);
        ++dc.iters;
        if (SPT_DIAG && exhausted) {
            dc.t_iters += 1;
            dc.t_live += (unsigned long long)__popcll(live);
        }
        // ---- one cast + one shading step ----
        const bool act = ps.phase != PH_IDLE;
        // GLANE: the lane walk over layout 0 in global memory (trees too large for LDS)
        bool cdone = true;
        Hit h;
        if constexpr (RES) {
            if (SPT_DUP & 512) {
                Hit h2 = hres;
                h2.best = opaque_v(h2.best);
                uint32_t li2 = opaque_v(li), ll2 = lleaf, ll22 = lleaf2;
                const bool c2 = lane_cast<LEAF, LDS_BYTES>(a.scene.accel, opaque_v3(ps.o), opaque_v3(ps.d), act, dg,
                                    LDSN ? (const uint32_t *)s_nodes : (const uint32_t *)a.scene.accel.nodes, fresh,
                                    (uint32_t)SPT_LANE_BUDGET, h2, li2, ll2, ll22);
                sink_v(h2.idx);
                sink_v(h2.best);
                sink_v(li2);
                sink_v(c2 ? 1u : 0u);
            }
            cdone = lane_cast<LEAF, LDS_BYTES>(a.scene.accel, ps.o, ps.d, act, dg,
                                    LDSN ? (const uint32_t *)s_nodes : (const uint32_t *)a.scene.accel.nodes, fresh,
                                    (uint32_t)SPT_LANE_BUDGET, hres, li, lleaf, lleaf2);
            h = hres;
            casts += (unsigned long long)__popcll(__ballot(act && cdone));
        } else if constexpr (PRIM) {
            // a primary batch casts against its block's candidate list when there is one
            // (prim_list_cast); every other cast walks the tree
            bool listed = false;
            if (prim_iter && kernarg_args()->prim.on) {
                if (SPT_DUP & 64) {
                    Hit h2;
                    prim_list_cast(a.scene.accel, opaque_v3(ps.o), opaque_v3(ps.d), act, pxy, h2, dg);
                    sink_v(h2.idx);
                    sink_v(h2.best);
                    sink_v(h2.t);
                }
                listed = prim_list_cast(a.scene.accel, ps.o, ps.d, act, pxy, h, dg);
            }
            if (!listed)
                h = find_closest<TREE, LEAF, LDSN>(a.scene.accel, ps.o, ps.d, act, dg, (const uint32_t *)s_nodes,
                                                   s_lds + (threadIdx.x & ~63u));
            if (SPT_DUP & 1) {
                const f3 o2 = opaque_v3(ps.o), d2 = opaque_v3(ps.d);
                Hit h2;
                bool l2 = false;
                if (prim_iter && kernarg_args()->prim.on) l2 = prim_list_cast(a.scene.accel, o2, d2, act, pxy, h2, dg);
                if (!l2) h2 = find_closest<TREE, LEAF, LDSN>(a.scene.accel, o2, d2, act, dg, (const uint32_t *)s_nodes);
                sink_v(h2.idx);
                sink_v(h2.best);
                sink_v(h2.t);
            }
        } else {
            h = (LDSN && SPT_LANE_WALK)
                    ? find_closest_lane<LEAF>(a.scene.accel, ps.o, ps.d, act, dg, (const uint32_t *)s_nodes)
                : GLANE
                    ? find_closest_lane<LEAF>(a.scene.accel, ps.o, ps.d, act, dg, (const uint32_t *)a.scene.accel.nodes)
                    : find_closest<TREE, LEAF, LDSN>(a.scene.accel, ps.o, ps.d, act, dg, (const uint32_t *)s_nodes);
        }
        SPT_STAMP(dc.cast);
#if SPT_DIAG
        if (prim_iter) {
            dc.p_iters += 1;
            dc.p_nodes += dg.nodes - d_n0;
            dc.p_spheres += dg.spheres - d_s0;
            dc.p_branches += dg.branches - d_b0;
            dc.p_cast += dc.cast - d_c0;
        }
#endif
        shade_step<true, SVC && SPT_SVC_WT>(a, ps, h, act && cdone, done, dropped, s_lds + (threadIdx.x & ~63u),
                                            SPT_DIAG ? dc.s_rounds : nullptr);
        fresh = cdone;
        if (SVC) {
            // finished samples per completion counter, summed in the wave (acc) and added
            // to the counter when the wave moves on to another one (svc_flush)
            const bool fin = act && ps.phase == PH_IDLE;
            unsigned long long fm = __ballot(fin);
            while (fm != 0ull) {
                const uint32_t j = __builtin_amdgcn_readlane(ps.job, (int)__builtin_ctzll(fm));
                const unsigned long long m = __ballot(fin && ps.job == j);
                if (j != acc_idx) {
                    svc_flush(acc_idx, acc_cnt, lane);
                    acc_idx = j;
                    acc_cnt = 0;
                }
                acc_cnt += (uint32_t)__popcll(m);
                fm &= ~m;
            }
        }
        if (PRIM && prim_iter) {
            // the lane's own path back from its row, then the batch's survivors into
            // rows [0, n) of the queue (a lane writes row rank <= lane, after the whole
            // wave has read its own row: LDS operations of a wave complete in order)
            Path own;
            unpark_path<SVC>(park, lane, own);
            __builtin_amdgcn_wave_barrier();
            const unsigned long long lv = __ballot(ps.phase != PH_IDLE);
            if (ps.phase != PH_IDLE) park_path<SVC>(park, lane_rank(lv), ps);
            ps = own;
            q_n = (uint32_t)__popcll(lv);
            q_pos = 0;
        }
        SPT_STAMP(dc.shade);
    }

    if (SVC) {
        svc_flush(acc_idx, acc_cnt, lane);
        // one render wave fewer (the forwarder leaves when none is left)
        kargs_t &k = *kernarg_args();
        if (lane == 0) __hip_atomic_fetch_add((gu32 *)(k.svc_ctl + kSvcLive), 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // per-lane done/dropped -> wave sums (butterfly), one atomic per counter and wave
    // (same-address atomics from every lane cost a launch ~10%; see render_grid)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        done += __shfl_xor(done, o);
        dropped += __shfl_xor(dropped, o);
    }
    if (lane == 0) {
        if (casts) atomicAdd(&a.counters[0], casts);
        if (done) atomicAdd(&a.counters[1], done);
        if (dropped) atomicAdd(&a.counters[2], dropped);
    }
#if SPT_DIAG
    if (lane == 0) {
        atomicAdd(&a.counters[4], dc.iters);
        atomicAdd(&a.counters[5], dg.leaves);
        atomicAdd(&a.counters[6], dg.nodes);
        atomicAdd(&a.counters[7], dc.cast);
        atomicAdd(&a.counters[8], dc.shade);
        atomicAdd(&a.counters[9], dc.refill);
        atomicAdd(&a.counters[10], dg.pairs);
        atomicAdd(&a.counters[11], dg.live);
        atomicAdd(&a.counters[12], dg.spheres);
        atomicAdd(&a.counters[13], dg.branches);
        atomicAdd(&a.counters[14], dg.passing);
        atomicAdd(&a.counters[15], dg.improving);
        atomicAdd(&a.counters[16], dg.lane_tests);
        atomicAdd(&a.counters[17], dg.lane_pretests);
        atomicAdd(&a.counters[18], dc.p_iters);
        atomicAdd(&a.counters[19], dc.p_nodes);
        atomicAdd(&a.counters[20], dc.p_spheres);
        atomicAdd(&a.counters[21], dc.p_branches);
        atomicAdd(&a.counters[22], dc.p_cast);
        atomicAdd(&a.counters[23], dc.s_rounds[0]);
        atomicAdd(&a.counters[24], dc.s_rounds[1]);
        atomicAdd(&a.counters[25], dg.leaves8);
        atomicAdd(&a.counters[26], dg.leaves16);
        atomicAdd(&a.counters[27], dc.s_rounds[2]);
        atomicAdd(&a.counters[28], dc.t_iters);
        atomicAdd(&a.counters[29], dc.t_live);
    }
#endif
#undef SPT_STAMP
}

template <bool TREE, int LEAF>
__global__ __launch_bounds__(kRenderBlock) SPT_RENDER_ATTR void render_kernel(RenderArgs a)
{
    render_body<TREE, LEAF, false, kRenderBlock>(a);
}

// batched launches (RenderArgs::rects): concurrent RenderSegment calls in one launch
template <bool TREE, int LEAF>
__global__ __launch_bounds__(kRenderBlock) SPT_RENDER_ATTR void render_kernel_batch(RenderArgs a)
{
    render_body<TREE, LEAF, false, kRenderBlock, true>(a);
}

// the render service: one resident launch over a stream of published jobs (RenderArgs
// svc_*)
template <bool TREE, int LEAF>
__global__ __launch_bounds__(kRenderBlock) SPT_RENDER_ATTR void render_kernel_svc(RenderArgs a)
{
    render_body<TREE, LEAF, false, kRenderBlock, false, false, true>(a);
}

// trees of kLdsNodeRecords to kGlaneMaxNodes nodes: the lane walk reading layout 0 from
// global memory (L1/L2), in the 256-thread kernel's shape
__global__ __launch_bounds__(kRenderBlock) SPT_RENDER_ATTR void render_kernel_glane(RenderArgs a)
{
    render_body<true, (int)kClusterSlots, false, kRenderBlock, false, true>(a);
}
__global__ __launch_bounds__(kRenderBlock) SPT_RENDER_ATTR void render_kernel_glane_batch(RenderArgs a)
{
    render_body<true, (int)kClusterSlots, false, kRenderBlock, true, true>(a);
}

// its own register budget: 1024-thread blocks, two per CU, need 8 waves per SIMD
#ifndef SPT_LDS_NUM_SGPR
#define SPT_LDS_NUM_SGPR 80
#endif
__global__ __launch_bounds__(kLdsBlock)
    __attribute__((amdgpu_num_sgpr(SPT_LDS_NUM_SGPR), amdgpu_waves_per_eu(2 * kLdsBlock / 256))) void render_kernel_lds(RenderArgs a)
{
    render_body<true, (int)kClusterSlots, true, kLdsBlock>(a);
}
__global__ __launch_bounds__(kLdsBlock)
    __attribute__((amdgpu_num_sgpr(SPT_LDS_NUM_SGPR), amdgpu_waves_per_eu(2 * kLdsBlock / 256))) void render_kernel_lds_batch(RenderArgs a)
{
    render_body<true, (int)kClusterSlots, true, kLdsBlock, true>(a);
}

// the render service over the LDS lane walk (config 5's trees): one resident launch of
// render_kernel_lds's shape over the published jobs (DESIGN.md §4.7 "LDS-tree sessions")
__global__ __launch_bounds__(kLdsBlock)
    __attribute__((amdgpu_num_sgpr(SPT_LDS_NUM_SGPR), amdgpu_waves_per_eu(2 * kLdsBlock / 256))) void render_kernel_svc_lds(RenderArgs a)
{
    render_body<true, (int)kClusterSlots, true, kLdsBlock, false, false, true>(a);
}

// Threads take the region's pixels in 8x8-tile order (tile_pixel), so the 64 lanes of
// a wave read 64 consecutive slots per sample.
// the launched fold's wave priority (s_setprio) when FoldArgs::prio is set
#ifndef SPT_FOLD_PRIO
#define SPT_FOLD_PRIO 3
#endif
// threads per fold block (its blocks run beside the next frame's render)
#ifndef SPT_FOLD_BLOCK
#define SPT_FOLD_BLOCK 256
#endif
__global__ __launch_bounds__(SPT_FOLD_BLOCK) void fold_kernel(FoldArgs a)
{
    // a launched render's fold runs beside the next frame's persistent render launch, whose
    // waves are older and win the SIMDs' issue arbitration: at the default priority the
    // fold's waves stalled for 2.8 ms (config 2) and the caller's next render waited on them;
    // at priority 3 the fold takes 0.6 ms and the bench gains 0.8%.  Beside
    // the render service nothing waits to start after a fold, and the raised priority only
    // took issue cycles from the service's waves (-1.5%): FoldArgs::prio is 0 there.
    if (a.prio) __builtin_amdgcn_s_setprio(SPT_FOLD_PRIO);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.npix) return;
    const uint32_t rows = a.npix / a.map.width;
    uint32_t lr, col;
    tile_pixel(i, a.map.width, rows, lr, col);
    fold_pixel(a, a.samples, a.map, rows, a.alias, lr, col, a.out_rgba, a.out_rgb8);
}

// Range alias fold (FoldArgs::range_alias): output t is alias index out_i0 + t, local
// float4 output at out_rgba[t] (g_data is written by the assemble step).
__global__ __launch_bounds__(256) void fold_alias_range_kernel(FoldArgs a)
{
    if (a.prio) __builtin_amdgcn_s_setprio(3);  // as fold_kernel
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.npix) return;
    float4 acc = a.first ? make_float4(0.f, 0.f, 0.f, 0.f) : a.acc[t];
    alias_accumulate(a, a.samples, a.out_i0 + t, a.map.width, a.alias_h, a.map.y0, a.src_rows, a.spp_batch, acc);
    if (!a.last) {
        a.acc[t] = acc;
        if (!a.preview) return;
    }
    const float scale = 1.f / acc.w;
    if (a.out_rgba) a.out_rgba[t] = make_float4(acc.x * scale, acc.y * scale, acc.z * scale, 0.f);
}

// The rectangle of pixel i of a batched fold (FoldArgs::rects).
typedef __attribute__((address_space(4))) const BatchRect crect_k;
__device__ __forceinline__ uint32_t fold_rect(crect_k *rs, uint32_t n, uint32_t i)
{
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rs[mid].pix_off <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// Batched fold (FoldArgs::rects): pixel i of the batch's concatenated rectangles.  Block
// 0 also zeroes the render's claim counters for the workspace's next batch.
__global__ __launch_bounds__(256) void fold_kernel_batch(FoldArgs a)
{
#ifndef SPT_FOLD_PRIO_BATCH
#define SPT_FOLD_PRIO_BATCH 1
#endif
    if (SPT_FOLD_PRIO_BATCH && a.prio) __builtin_amdgcn_s_setprio(3);  // as fold_kernel
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && a.head_reset && threadIdx.x < a.head_queues) a.head_reset[threadIdx.x * kQueueStride] = 0u;
    if (i >= a.npix) return;
    // the rectangles from the kernel arguments (this kernel's first argument is `a`)
    typedef __attribute__((address_space(4))) const FoldArgs cfold_t;
    typedef __attribute__((address_space(4))) const char kchar;
    cfold_t *ka = (cfold_t *)(kchar *)__builtin_amdgcn_kernarg_segment_ptr();
    crect_k *rs = a.inline_rects ? (crect_k *)ka->rects_inline : (crect_k *)a.rects;
    crect_k &r = rs[fold_rect(rs, a.n_rects, i)];
    const RowMap map{r.y0, r.y0 + r.rows, 1u, 1u, 0u, r.x0, r.w};
    uint32_t lr, col;
    tile_pixel(i - r.pix_off, r.w, r.rows, lr, col);
    fold_pixel(a, a.samples + (size_t)a.slot_words * r.slot_off, map, r.rows, (int)r.alias, lr, col,
               a.out_rgba ? a.out_rgba + r.pix_off : nullptr, r.rgb8);
}

// Per-sample colours of a single-batch region (spt_render_samples, a debug path):
// out[p * spp + s] = {r, g, b, counted}, p the local row-major pixel.
__global__ __launch_bounds__(256) void expand_kernel(FoldArgs a, float4 *out, uint32_t p0, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = p0 + i;
    const uint32_t W = a.map.width, rows = a.npix / W, lr = p / W, col = p - lr * W;
    uint32_t q0, step;
    ts_slot_base(lr, col, W, rows, a.spp_batch, q0, step);
    for (uint32_t k = 0; k < a.spp_batch; ++k) {
        const uint32_t q = q0 + k * step;
        const uint32_t w = a.slot_words == 1u ? a.samples[q] : a.samples[2u * q];
        const bool counted = a.slot_words == 1u || a.samples[2u * q + 1u] != 0u;
        const f3 c = decode_sample(a, w);
        out[(size_t)i * a.spp_batch + k] = make_float4(c.x, c.y, c.z, counted ? 1.f : 0.f);
    }
}

__global__ __launch_bounds__(256) void assemble_kernel(const float4 *tiles, uint32_t max_rows, RowMap base,
                                                       uint32_t width, uint32_t height, float4 *frame, uint8_t *rgb8)
{
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t k = blockIdx.y;
    const uint32_t r = blockIdx.z;
    if (x >= base.width) return;
    RowMap m = base;
    m.part = r;
    if (k >= rows_owned(m)) return;
    const uint32_t y = row_of(m, k);
    const float4 c = tiles[((size_t)r * max_rows + k) * base.width + x];
    if (frame) frame[(size_t)(y - base.y0) * base.width + x] = c;
    if (rgb8) {
        const uint32_t gx = base.x0 + x;
        const size_t gi = (size_t)3 * ((size_t)(height - 1u - y) * width + gx);
        rgb8[gi + 0] = gamma_byte(c.x);
        rgb8[gi + 1] = gamma_byte(c.y);
        rgb8[gi + 2] = gamma_byte(c.z);
    }
}

__global__ void selftest_kernel(const float *a, const float *b, const uint32_t *bits, uint32_t n, float *out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = a[i], y = b[i], c = __uint_as_float(bits[i]);
    float *o = out + (size_t)i * SPT_SELFTEST_COLS;
    o[0] = div_rn(x, y);
    o[1] = __builtin_sqrtf(x);
    o[2] = pow5f(x);                    // glibc powf(x, 5.f) restated
    o[3] = pow5f(c);                    // ... over any bit pattern
    o[4] = spt_glibc_powf(x, 2.f);      // the rSq form, powf(x, 2.f)
    o[5] = no_tir(kAirToGlass, x) ? refract_k(kAirToGlass, x) : -1e30f;
    o[6] = uniform_bits(bits[i], -1.f, 1.f);
    o[7] = (float)f2u8(x);
    const f3 nv = normalize(mk(x, y, c));  // c: any bit pattern (NaN, inf, denormal, huge)
    o[8] = nv.x;
    o[9] = nv.y;
    o[10] = nv.z;
    o[11] = div_rn(c, x);
    o[12] = uniform_bits(bits[i], -0.5f, 0.5f);
    o[13] = uniform_bits(bits[i], 0.f, 1.f);
    const uint32_t j = ((bits[i] * 2654435761u) >> 23) % 301u;  // halvings of a diffuse sample word
    o[14] = halve_n(c, j);
    o[15] = halve_n(x, j);
}

// Blocks per CU of the LDS tree variant and CUs of a device, queried once per device
// (thread-safe: RenderJob threads launch concurrently).  per_cu = 0 disables the variant.
static void lds_tree_shape(int *per_cu, int *num_cu)
{
    constexpr int kMaxDevices = 64;
    static std::mutex mu;
    static int pc[kMaxDevices], nc[kMaxDevices];
    static bool known[kMaxDevices];
    int dev = 0;
    *per_cu = *num_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return;
    std::lock_guard<std::mutex> lk(mu);
    if (!known[dev]) {
        if (hipDeviceGetAttribute(&nc[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc[dev], render_kernel_lds, (int)kLdsBlock, 0) != hipSuccess)
            pc[dev] = 0;
        known[dev] = true;
    }
    *per_cu = pc[dev];
    *num_cu = nc[dev];
}

uint32_t svc_lds_grid(bool full)
{
    int per_cu = 0, num_cu = 0;
    lds_tree_shape(&per_cu, &num_cu);
    if (per_cu <= 0 || num_cu <= 0) return 0u;
    return (uint32_t)((full ? per_cu : std::max(1, per_cu - 1)) * num_cu);
}

hipError_t launch_render(const RenderArgs &a, LaunchShape &sh, hipStream_t s)
{
    const uint32_t div = sh.div ? sh.div : 1u;
    const bool batch = a.rects != nullptr;
    // trees of >= kLdsMinNodes nodes walk an LDS copy of the node table (config 5);
    // smaller ones stay in the scalar cache (all 8 octant layouts: config 2's 26-node
    // tree is 6.7 KB), where the 256-thread kernel overlaps frames in flight better
    if (a.scene.accel.tree && a.scene.accel.n_nodes >= kLdsMinNodes && a.scene.accel.n_nodes + 1u <= kLdsNodeRecords) {
        // all resident blocks (divided among the host calls in flight), or fewer when the
        // launch has under 2 claims per wave (render_grid's rule)
        int per_cu = 0, num_cu = 0;
        lds_tree_shape(&per_cu, &num_cu);
        if (per_cu > 0) {
            const uint64_t claims = ((uint64_t)a.n_items + a.claim - 1) / a.claim;
            const uint64_t per_block = 2 * (kLdsBlock / 64);
            const uint64_t full = ((uint64_t)per_cu * num_cu + div - 1) / div;
            uint64_t g = (claims + per_block - 1) / per_block;
            g = g < full ? g : full;
            sh.ran_grid = (uint32_t)g;
            sh.ran_block = kLdsBlock;
            if (batch)
                hipLaunchKernelGGL(render_kernel_lds_batch, dim3(sh.ran_grid), dim3(kLdsBlock), 0, s, a);
            else
                hipLaunchKernelGGL(render_kernel_lds, dim3(sh.ran_grid), dim3(kLdsBlock), 0, s, a);
            return hipGetLastError();
        }
    }
    sh.ran_grid = sh.grid;
    sh.ran_block = sh.block;
    if (a.scene.accel.tree && a.scene.accel.n_nodes >= kLdsMinNodes && a.scene.accel.n_nodes <= kGlaneMaxNodes) {
        if (batch)
            hipLaunchKernelGGL(render_kernel_glane_batch, dim3(sh.grid), dim3(sh.block), 0, s, a);
        else
            hipLaunchKernelGGL(render_kernel_glane, dim3(sh.grid), dim3(sh.block), 0, s, a);
        return hipGetLastError();
    }
    if (batch) {
        if (a.scene.accel.tree)
            hipLaunchKernelGGL((render_kernel_batch<true, (int)kClusterSlots>), dim3(sh.grid), dim3(sh.block), 0, s, a);
        else if (a.scene.accel.leaf_slots == kFlatLeafSlots)
            hipLaunchKernelGGL((render_kernel_batch<false, (int)kFlatLeafSlots>), dim3(sh.grid), dim3(sh.block), 0, s, a);
        else
            hipLaunchKernelGGL((render_kernel_batch<false, (int)kClusterSlots>), dim3(sh.grid), dim3(sh.block), 0, s, a);
    } else if (a.scene.accel.tree)
        hipLaunchKernelGGL((render_kernel<true, (int)kClusterSlots>), dim3(sh.grid), dim3(sh.block), 0, s, a);
    else if (a.scene.accel.leaf_slots == kFlatLeafSlots)
        hipLaunchKernelGGL((render_kernel<false, (int)kFlatLeafSlots>), dim3(sh.grid), dim3(sh.block), 0, s, a);
    else
        hipLaunchKernelGGL((render_kernel<false, (int)kClusterSlots>), dim3(sh.grid), dim3(sh.block), 0, s, a);
    return hipGetLastError();
}

bool svc_lds(const AccelView &ac)
{
    return ac.tree && ac.n_nodes >= kLdsMinNodes && ac.n_nodes + 1u <= kLdsSvcNodeRecords;
}

bool svc_supported(const AccelView &ac)
{
    return !(ac.tree && ac.n_nodes >= kLdsMinNodes && ac.n_nodes <= kGlaneMaxNodes) || svc_lds(ac);
}

uint32_t svc_block(const AccelView &ac) { return svc_lds(ac) ? kLdsBlock : kRenderBlock; }

hipError_t launch_render_svc(const RenderArgs &a, uint32_t grid, hipStream_t s)
{
    if (!svc_supported(a.scene.accel) || !a.svc_host) return hipErrorInvalidValue;
    if (svc_lds(a.scene.accel)) {
        hipLaunchKernelGGL(render_kernel_svc_lds, dim3(grid), dim3(kLdsBlock), 0, s, a);
        return hipGetLastError();
    }
    if (a.scene.accel.tree)
        hipLaunchKernelGGL((render_kernel_svc<true, (int)kClusterSlots>), dim3(grid), dim3(kRenderBlock), 0, s, a);
    else if (a.scene.accel.leaf_slots == kFlatLeafSlots)
        hipLaunchKernelGGL((render_kernel_svc<false, (int)kFlatLeafSlots>), dim3(grid), dim3(kRenderBlock), 0, s, a);
    else
        hipLaunchKernelGGL((render_kernel_svc<false, (int)kClusterSlots>), dim3(grid), dim3(kRenderBlock), 0, s, a);
    return hipGetLastError();
}


hipError_t launch_fold(const FoldArgs &a, hipStream_t s)
{
    if (a.npix == 0) return hipSuccess;
    if (a.range_alias)
        hipLaunchKernelGGL(fold_alias_range_kernel, dim3((a.npix + 255) / 256), dim3(256), 0, s, a);
    else if (a.rects)
        hipLaunchKernelGGL(fold_kernel_batch, dim3((a.npix + 255) / 256), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(fold_kernel, dim3((a.npix + SPT_FOLD_BLOCK - 1) / SPT_FOLD_BLOCK), dim3(SPT_FOLD_BLOCK), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_expand(const FoldArgs &a, float4 *out, uint32_t p0, uint32_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(expand_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, out, p0, n);
    return hipGetLastError();
}

hipError_t launch_assemble(const float4 *tiles, uint32_t max_rows, RowMap base, uint32_t width, uint32_t height,
                           float4 *frame, uint8_t *rgb8, hipStream_t s)
{
    if (max_rows == 0 || base.width == 0) return hipSuccess;
    dim3 grid((base.width + 255) / 256, max_rows, base.parts);
    hipLaunchKernelGGL(assemble_kernel, grid, dim3(256), 0, s, tiles, max_rows, base, width, height, frame, rgb8);
    return hipGetLastError();
}

hipError_t launch_selftest(const float *a, const float *b, const uint32_t *bits, uint32_t n, float *out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, b, bits, n, out);
    return hipGetLastError();
}

uint32_t render_group_size() { return SPT_GROUP; }
uint32_t render_block_size() { return kRenderBlock; }
bool lane_walk_tree(const AccelView &ac)
{
    return ac.tree && ac.n_nodes >= kLdsMinNodes && (ac.n_nodes + 1u <= kLdsNodeRecords || ac.n_nodes <= kGlaneMaxNodes);
}

hipError_t render_occupancy(uint32_t block, int *blocks_per_cu)
{
    // the smallest occupancy of the four shapes sizes the persistent grid.  All four
    // compile to the same register budget (SPT_RENDER_ATTR: 94 SGPRs, 72 VGPRs at the
    // 96-SGPR cap, `make asm`), so the minimum equals each kernel's own occupancy and the
    // global-memory lane walk does not shrink the grid of the other shapes
    int a = 0, b = 0, c = 0, g = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, render_kernel<true, (int)kClusterSlots>, (int)block, 0);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, render_kernel<false, (int)kFlatLeafSlots>, (int)block, 0);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&c, render_kernel<false, (int)kClusterSlots>, (int)block, 0);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&g, render_kernel_glane, (int)block, 0);
    *blocks_per_cu = std::min(std::min(a, b), std::min(c, g));
    // the occupancy API reports one block per CU too many at 81-96 and 97-112 SGPRs
    // (MI355X_MICROARCH.md, Correctness boundaries): waves per SIMD are bounded by
    // 800 / (ceil(sgpr / 16) * 16 + 16) SGPRs; a block of w waves takes w/4 wave slots per SIMD
    if (SPT_NUM_SGPR > 0) {
        // .sgpr_count = the cap minus the 2 VCC registers
        const int cap = 800 / (((SPT_NUM_SGPR - 2 + 15) / 16) * 16 + 16);  // waves per SIMD
        const int cap_blocks = cap * 4 / (int)(block / 64u);                 // 4 SIMDs per CU
        if (*blocks_per_cu > cap_blocks) *blocks_per_cu = cap_blocks;
    }
    return e;
}

}  // namespace spt
