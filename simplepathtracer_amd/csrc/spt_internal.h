// spt_internal.h -- kernel launch interface shared by spt_kernels.hip and the host side (spt_host.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spt_hip.h"

namespace spt {

// Row map of a launch: rows y in [y0, y1) with ((y - y0) / strip) % parts == part.
struct RowMap {
    uint32_t y0, y1, strip, parts, part;
    uint32_t x0, width;  // columns [x0, x0 + width)
};

__host__ __device__ inline uint32_t row_of(const RowMap &m, uint32_t lr)
{
    uint32_t blk = lr / m.strip;
    return m.y0 + (blk * m.parts + m.part) * m.strip + (lr - blk * m.strip);
}

__host__ __device__ inline uint32_t rows_owned(const RowMap &m)
{
    if (m.y1 <= m.y0) return 0;
    uint32_t h = m.y1 - m.y0;
    uint32_t period = m.strip * m.parts;
    uint32_t full = h / period, rem = h % period;
    uint32_t r = full * m.strip;
    uint32_t start = m.part * m.strip;
    if (rem > start) r += (rem - start < m.strip) ? rem - start : m.strip;
    return r;
}

// Pixel of the q-th item of one sample in a region of `rows` x `width` pixels
// whose items run through 8x8 tiles (row-major tiles, row-major inside a tile;
// ragged tiles at the right and bottom edges).  A wave's consecutive items then
// cover a compact patch instead of a 64-pixel row strip, so its rays start close
// together and cull together.  Bijective on [0, rows*width).
__host__ __device__ inline void tile_pixel(uint32_t q, uint32_t width, uint32_t rows, uint32_t &lr, uint32_t &col)
{
    const uint32_t band = (q / width) >> 3;
    const uint32_t h = rows - (band << 3) < 8u ? rows - (band << 3) : 8u;
    const uint32_t qb = q - band * 8u * width;
    const uint32_t ft = width >> 3, wr = width & 7u;
    uint32_t row, c;
    if (h == 8u) {
        const uint32_t t = qb >> 6;
        if (t < ft) {
            row = (qb >> 3) & 7u;
            c = (t << 3) | (qb & 7u);
        } else {
            const uint32_t e = qb - (ft << 6);
            row = e / wr;
            c = (ft << 3) + (e - row * wr);
        }
    } else {
        const uint32_t th = h << 3;
        const uint32_t t = qb / th;
        if (t < ft) {
            const uint32_t e = qb - t * th;
            row = e >> 3;
            c = (t << 3) | (e & 7u);
        } else {
            const uint32_t e = qb - ft * th;
            row = e / wr;
            c = (ft << 3) + (e - row * wr);
        }
    }
    lr = (band << 3) + row;
    col = c;
}

// Division of x < 2^31 by a divisor d >= 1 fixed for a launch (Granlund-Montgomery,
// N = 31 bits): l = ceil(log2 d), m = floor(2^(31+l) / d) + 1 < 2^32, and
// x / d == mulhi(x, m) >> (l - 1) for every x < 2^31; d == 1 passes x through.
struct FastDiv {
    uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d)
{
    FastDiv f{d, 0u, 0u};
    if (d <= 1u) return f;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.m = (uint32_t)(((1ull << (31 + l)) / d) + 1ull);
    f.s = l - 1u;
    return f;
}
__host__ __device__ inline uint32_t fast_div(uint32_t x, const FastDiv &f)
{
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t hi = __umulhi(x, f.m);
#else
    const uint32_t hi = (uint32_t)(((uint64_t)x * f.m) >> 32);
#endif
    return f.d <= 1u ? x : hi >> f.s;
}

// row_of with the strip division by multiply-shift (div_strip = FastDiv(m.strip))
__host__ __device__ inline uint32_t row_of_fast(const RowMap &m, uint32_t lr, const FastDiv &div_strip)
{
    const uint32_t blk = fast_div(lr, div_strip);
    return m.y0 + (blk * m.parts + m.part) * m.strip + (lr - blk * m.strip);
}

// (sample, pixel) of the q-th item of a batch of S samples over a region of
// `rows` x `width` pixels, items ordered [8-row band][8-column tile][sample]
// [pixel in tile] (ragged tiles at the right and bottom edges).  A claim of
// consecutive items then stays inside one 8x8 tile across several samples, so a
// wave's rays start close together whatever the claim size.  Full tiles use
// shifts; only edge tiles divide.  Bijective on [0, rows*width*S) (host test).
// div_band = FastDiv(8*width*S) (unused when rows < 8), div_tile = FastDiv(64*S).
__host__ __device__ inline void ts_item(uint32_t q, uint32_t width, uint32_t rows, uint32_t S, const FastDiv &div_band,
                                        const FastDiv &div_tile, uint32_t &sl, uint32_t &lr, uint32_t &col)
{
    // 8*width*S <= rows*width*S < 2^31 whenever rows >= 8; a single band otherwise
    const uint32_t band = rows >= 8u ? fast_div(q, div_band) : 0u;
    const uint32_t h = rows - (band << 3) < 8u ? rows - (band << 3) : 8u;
    const uint32_t qb = q - band * 8u * width * S;
    const uint32_t ft = width >> 3, wr = width & 7u;
    const uint32_t ti = h * 8u * S;  // items of a full-width tile of this band
    uint32_t e, wt, c0;
    if (h == 8u) {
        const uint32_t t = fast_div(qb, div_tile);
        if (t < ft) {
            e = qb - t * 64u * S;
            sl = e >> 6;
            const uint32_t pix = e & 63u;
            lr = (band << 3) + (pix >> 3);
            col = (t << 3) + (pix & 7u);
            return;
        }
        e = qb - ft * ti;
        wt = wr;
        c0 = ft << 3;
    } else {
        const uint32_t t = qb / ti;
        wt = t < ft ? 8u : wr;
        e = qb - (t < ft ? t : ft) * ti;
        c0 = (t < ft ? t : ft) << 3;
    }
    sl = e / (h * wt);
    const uint32_t pix = e - sl * h * wt;
    const uint32_t row = pix / wt;
    lr = (band << 3) + row;
    col = c0 + (pix - row * wt);
}

// Inverse of ts_item for one pixel: the item index (= slot) of sample 0 of local pixel
// (lr, col) and the step between its consecutive samples.  Slots are stored in item
// order, so a claim's paths write one contiguous run of slots; the fold reads sample s
// of a pixel at q0 + s * step (64 consecutive slots for the 64 pixels of a full 8x8 tile).
__host__ __device__ inline void ts_slot_base(uint32_t lr, uint32_t col, uint32_t width, uint32_t rows, uint32_t S,
                                             uint32_t &q0, uint32_t &step)
{
    const uint32_t band = lr >> 3;
    const uint32_t h = rows - (band << 3) < 8u ? rows - (band << 3) : 8u;
    const uint32_t ft = width >> 3, wr = width & 7u;
    const uint32_t t = col >> 3;
    const uint32_t tc = t < ft ? t : ft;  // full-width tile, or the ragged right one
    const uint32_t wt = t < ft ? 8u : wr;
    q0 = band * 8u * width * S + tc * h * 8u * S + (lr - (band << 3)) * wt + (col - (tc << 3));
    step = h * wt;
}

// Sample codes: one 32-bit word per sample instead of its colour.  A
// sample's colour is one of
//   * the sky, initColor * k * 0.5 with k = d.y + 1.f of the final ray
//     (SampleColorSkybox, SingleThreadPathTracer.hpp:11-14): the word is k's bits;
//   * a diffuse albedo halved 1 + j times (SampleColorDiffuse, lines 21-37: the first
//     diffuse hit's colour * 0.5, then * 0.5 per further bounce): a code naming the
//     first hit's slot and j;
//   * 0 (the specular-event cap; RenderSegmentTask's dropped paths).
// A finite k is 0 or at least 2^-24 in magnitude (fl(y + 1) for float y: only y = -1
// lies within 2^-24 of -1), so the words whose magnitude as a float is below 2^-24 and
// nonzero never hold a k: they carry the codes c in [1, kCodeMax], positive words
// first, then the same magnitudes with the sign bit.  c = 1 is the colour 0,
// c = 2 + j * stride + slot a diffuse sample (stride = the scene's slot count).  j is
// saturated at jmax = min(bounces - 1, jz): j <= bounces - 1 always, and after jz
// halvings every finite albedo of the scene is 0 (inf / NaN stay themselves; jz <=
// kCodeSat, since 2^-280 * FLT_MAX rounds to 0), so saturating there changes no colour.
// A scene fits when (jmax + 1) * stride + 1 <= kCodeMax: ~34 M slots at depth 50, ~11 M
// for deep paths over albedos up to 255 (jz = 157).  The fold rebuilds the colour with
// the render kernel's own operations: bit-identical.
constexpr uint32_t kCodeSmall = 0x33800000u;        // bits of 2^-24
constexpr uint32_t kCodeMax = 2u * (kCodeSmall - 1u);  // the largest code
constexpr uint32_t kCodeSat = 280;                  // 2^-280 * FLT_MAX rounds to 0
__host__ __device__ inline bool code_layout_fits(uint64_t stride, uint32_t jmax)
{
    return (jmax + 1ull) * stride + 1ull <= kCodeMax;
}
// diffuse code of (j, slot) and back (div = FastDiv(stride), defined below)
__host__ __device__ inline uint32_t diffuse_code(uint32_t j, uint32_t slot, uint32_t stride)
{
    return 2u + j * stride + slot;
}
__host__ __device__ inline void diffuse_decode(uint32_t c, const FastDiv &div, uint32_t &j, uint32_t &slot)
{
    const uint32_t v = c - 2u;  // < kCodeMax < 2^31 (fast_div's range)
    j = fast_div(v, div);
    slot = v - j * div.d;
}
__host__ __device__ inline uint32_t code_word(uint32_t c)
{
    return c < kCodeSmall ? c : 0x80000000u | (c - kCodeSmall + 1u);
}
// the code of a word, 0 for a sky word
__host__ __device__ inline uint32_t word_code(uint32_t w)
{
    const uint32_t a = w & 0x7FFFFFFFu;
    if (a == 0u || a >= kCodeSmall) return 0u;
    return (w >> 31) ? a + kCodeSmall - 1u : a;
}
constexpr uint32_t kZeroWord = 1u;  // code_word(1): the colour 0

constexpr uint32_t kMaxGroup = 16;     // sphere-table padding granule (>= SPT_GROUP)
constexpr uint32_t kClusterSlots = 8;  // max members per cluster = slots of a tree leaf
constexpr uint32_t kFlatLeafSlots = 4; // slots of a flat-list leaf holding <= 4 members
// Flat-list line test (spt_path.h find_closest): the 1e-4 |Cb-o|^2 margin is folded
// in by scaling the expanded |Cb-o|^2 by kFlatScale = 1 - 1e-4; nodes store
// kFlatScale |Cb|^2.
constexpr double kFlatScale = 1.0 - 1e-4;
// Tree nodes are boxes expanded by kBoxS (|o| + Bm) on every side (Bm >= max |C| + r
// over the node's members): a ray whose member test passes comes within
// sqrt(r^2 + 2.6e-6 X^2) <= r + 1.6125e-3 X of the member's centre, X = |C - o|
// <= |o| + Bm; the rest of the margin covers the slab arithmetic.
// The node stores kBoxS Bm in its box, the lane adds kBoxS |o|.
constexpr double kBoxS = 1.63e-3;
// Reciprocal of a direction component: |d_i| is raised to at least 2^-20 first (no
// inf/NaN in the slab arithmetic; sound by the margin argument of DESIGN.md §4.4).
constexpr float kBoxMinDir = 0x1p-20f;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;  // AccelNode::slot of inner nodes
constexpr uint32_t kMiss = 0xFFFFFFFFu;    // Hit::idx when no sphere was hit

// Hot-loop traversal tables (spt_accel.cpp).
struct AccelView {
    const float4 *slots;    // {cx, cy, cz, r*r} in traversal order (always groups, then clusters)
    const uint32_t *orig;   // original sphere index per slot
    const void *nodes;      // AccelNode[8][n_nodes + 1]: per-octant preorder layouts (spt_accel.h)
    uint32_t always_groups, n_nodes;
    uint32_t tree;        // 0: flat cluster list (every node a leaf), 1: tree with inner nodes
    uint32_t leaf_slots;  // slots per leaf: kFlatLeafSlots or kClusterSlots
    const float *kpre;    // member pretest constant K' per slot (spt_accel.h)
    float pre_cm;         // >= max |C| + r over the cluster members
};

// Primary-ray candidate lists (round 5): for every 8x8 and 8x4
// pixel block of the frame, the slots a primary ray of the block -- from the eye, through
// any pixel of the block with any jitter -- can pass RaySphereIntersection for (a
// conservative cone test with the member test's fp reach, spt_accel.cpp
// build_prim_lists).  The closest hit of such a ray is in its block's list, so a
// primary batch (64 rays of one 8x8 tile) tests that list instead of walking the tree,
// with the same (distance, original index) winner.
struct PrimLists {
    const uint2 *b8, *b4;       // {first entry, count} per block, row-major; count kPrimWalk: walk
    const uint32_t *slots;      // candidate slots (each block's run ascending)
    uint32_t bw;                // blocks per row: ceil(width / 8)
    uint32_t on;                // lists built for this scene, camera and frame size
};
constexpr uint32_t kPrimWalk = 0xFFFFFFFFu;

struct DeviceScene {
    const float4 *shade;    // {red, green, blue, fuzz} per slot (hit geometry: accel.slots)
    const uint32_t *mat;    // material id per slot
    uint32_t n;
    uint32_t code_stride, code_jmax;  // diffuse sample codes (diffuse_code)
    AccelView accel;
};

struct Camera {
    float view[12];  // rows 0..2 of viewMatrix (row 3 is zero)
    float eye[3];
    float sky[3];
};

// One rectangle of a batched launch (several concurrent RenderSegment calls rendered
// by one render + one fold launch, spt_batch.cpp render_batched).  Its items are
// [item_off, item_end) of the launch, in the order of a single-rectangle launch
// (ts_item over w x rows pixels and all spp samples); item_off is a multiple of the
// launch's claim size, so a claim never spans two rectangles, and items in
// [item_end, next item_off) are padding (no path).  Its per-sample slots are
// [slot_off, slot_off + npix * spp), in its own item order; its fold output sits at
// pixels [pix_off, pix_off + npix) of the batch's staging.
struct BatchRect {
    uint32_t item_off, item_end, slot_off, pix_off;
    uint32_t x0, y0, w, rows;
    uint32_t npix, alias;  // alias: task mode on a non-square tile (fold_kernel)
    uint8_t *rgb8;         // the call's g_data as the device sees it (its page-locked host buffer,
                           // written in place, or the context's device frame), or null
    FastDiv div_band, div_tile;  // ts_item divisors 8*w*spp and 64*spp
};
static_assert(sizeof(BatchRect) == 72, "BatchRect layout");
constexpr uint32_t kInlineRects = 4;  // rectangles carried in the kernel arguments

struct RenderArgs {
    DeviceScene scene;
    Camera cam;
    uint32_t width, height, bounces, mode;
    uint64_t seed_key;  // fmix64(seed)
    RowMap map;
    uint32_t npix;       // pixels of the launch (rows_owned * width)
    uint32_t spp_batch;  // samples per pixel in this batch
    uint32_t s0;         // first sample index of the batch
    uint32_t n_items;    // npix * spp_batch
    uint32_t claim;      // items per queue claim
    FastDiv div_band, div_tile;  // ts_item divisors 8*width*spp_batch and 64*spp_batch
    FastDiv div_strip;           // row_of_fast divisor map.strip
    uint32_t *samples;   // [n_items] per-sample slots in item order: the sample word (segment mode) or
                         // {word, key} (task mode; key 0 = dropped path)
    uint32_t slot_words;  // 1 or 2
    uint32_t *head;      // queue head (zeroed before launch)
    unsigned long long *counters;  // [0] casts, [1] samples, [2] dropped
    const BatchRect *rects;  // batched launch: n_rects rectangles (map/npix/div_* unused); else null
    uint32_t n_rects;
    // claims come from n_queues counters head[k * kQueueStride], queue k
    // handing out items [k * queue_items, (k + 1) * queue_items) (claim multiples)
    uint32_t n_queues, queue_items;
    // batched launches of at most kInlineRects rectangles may carry them here, in the
    // kernel arguments (inline_rects = 1: no table upload before the launch)
    uint32_t inline_rects;
    BatchRect rects_inline[kInlineRects];
    // render service (render_kernel_svc): the session's device control words
    // (SvcCtl), its job table and first claim of every job (device copies, written by the
    // forwarder wave) and completion counters; the fields above then hold the session's constants only (scene,
    // camera, frame, mode, ring of sample slots in `samples`, claim size, n_queues)
    uint32_t *svc_ctl;
    const struct SvcJob *svc_jobs;
    const uint32_t *svc_job_claim;
    uint32_t *svc_done;
    // SPT_SVC_TRACE (diagnostics, null otherwise): per completion counter, the
    // s_memrealtime of the first and last claim taken and of the last count added
    unsigned long long *svc_trace;
    // the session's SvcHost words and host job tables in page-locked host memory (committed
    // jobs, closing flag, published pair, stop flag; records and first claims the forwarder
    // copies into svc_jobs / svc_job_claim), as the device sees them
    uint32_t *svc_host;
    const struct SvcJob *svc_host_jobs;
    const uint32_t *svc_host_job_claim;
    // primary-ray candidate lists (PrimLists; on = 0: every primary batch walks the tree)
    PrimLists prim;
};

// claim counters: at most one per XCD, 256 bytes apart (separate cache lines)
constexpr uint32_t kMaxQueues = 8, kQueueStride = 64;

// ---- render service (DESIGN.md §4.7 "Render service") --------------------------------
// One resident launch of render_kernel_svc renders a stream of jobs (a frame, a rank's
// strips, a sample batch, a drop-in tile), published while it runs.  A session's claims
// form one sequence: job j owns claims [job_claim[j], job_claim[j] + n) of `claim` items,
// its items [item_off, item_end) (item_off = its first claim * claim, the rest of its last
// claim is padding).  Queue q of n_queues reserves claims q, q + n_queues, ... from its
// counter; a wave keeps one reserved claim and takes it once the host has published it.
// Finished samples are counted per completion counter (several jobs may share one);
// hipStreamWaitValue32 on the counter gates the job's fold.
//
// Publication needs no GPU queue: the host writes the job records, their first claims and
// the published pair {claims, jobs} into fine-grained page-locked host memory (the SvcHost
// block and tables); one wave of the session kernel -- the forwarder, wave 0 of block 0,
// which renders nothing -- polls that pair with system-scope loads and copies new records
// into the device job table, then stores the device pair the render waves poll (the R1
// hand-off of MI355X_MICROARCH.md, as round 4's publish kernel did).  Round 4 published from
// a one-wave kernel on a stream of its own; a dispatch waiting for CU resources the session
// holds (an RCCL gather, the liveness test's blocker) held that kernel back, and with it
// the session (tests/test_gpu_service.py).
struct SvcJob {
    uint32_t item_off, item_end;  // session items of the job
    uint32_t slot_off;            // slot of its item 0 in the ring (samples, item order)
    uint32_t done_idx;            // its completion counter
    uint32_t rows, spp_batch, s0; // region rows; samples of the batch and the first one
    uint32_t claim_end;           // first claim after the job
    RowMap map;                   // region (rows or interleaved strips, columns)
    FastDiv div_band, div_tile, div_strip;  // ts_item / row_of_fast divisors
    uint32_t claim_first;         // its first claim (item_off / claim)
    uint32_t pad[7];
};
static_assert(sizeof(SvcJob) == 128, "SvcJob: 32 words, one per lane of the loading wave");
constexpr uint32_t kSvcJobWords = 32;
static_assert(offsetof(SvcJob, claim_first) == 24 * 4 && offsetof(SvcJob, map) == 8 * 4 &&
                  offsetof(SvcJob, div_strip) == 21 * 4,
              "SvcJob word offsets (the service kernel reads the record by word)");
// SvcCtl words (device memory, svc_ctl): claim counters head[q * kQueueStride]
// (q < kMaxQueues), then on lines of their own the device copy of the published pair
// {claims, jobs} (one 64-bit word, stored and loaded as one), the stop flag, and the
// render waves still in the session (the forwarder leaves at 0).
constexpr uint32_t kSvcPub = kMaxQueues * kQueueStride;  // uint64_t: claims | jobs << 32
constexpr uint32_t kSvcStop = kSvcPub + 64;
constexpr uint32_t kSvcLive = kSvcStop + 64;
constexpr uint32_t kSvcCtlWords = kSvcLive + 64;
// A wave with no work for 0.5 s (s_memrealtime, 100 MHz) may leave, but only through the
// closing handshake with the host (SvcHost words):
//   wave:  closing = 1; fence; c = committed; read the published pair; leave iff every one
//          of the c committed jobs is published and its reserved claim is not among them
//   host:  committed = jobs of the session after this publication; fence; if closing is
//          set, end the session and publish to a new one instead
// Store-then-load on both sides (system scope on the device, seq_cst on the host): at
// least one side sees the other's store, so a wave never leaves a session that is still
// owed a publication.  "Published" is the device pair (forwarded).
constexpr unsigned long long kSvcIdleTicks = 50000000ull;
// SvcHost words (page-locked host memory), each on a 128-byte line of its own: the
// committed job count, the closing flag, the host's published pair (uint64: claims |
// jobs << 32), the stop flag (stored after the session's last publication) and the
// watchdog flag (a wave left the session through the closing handshake)
constexpr uint32_t kSvcHostCommitted = 0, kSvcHostClosing = 32, kSvcHostPub = 64, kSvcHostStop = 96,
                   kSvcHostWatchdog = 128, kSvcHostWords = 160;
constexpr uint32_t kSvcTraceClaims = 1u << 21;  // SPT_SVC_TRACE: claims with a take time
// grid: blocks of the session kernel's shape (svc_grid: 256-thread blocks, or the LDS-tree
// kernel's 1 024-thread blocks when the scene's tree takes the LDS lane walk)
hipError_t launch_render_svc(const RenderArgs &a, uint32_t grid, hipStream_t s);
// the service covers the wave-walk kernels (render_kernel's shapes) and the LDS lane walk
// (render_kernel_lds's shape, round 6); trees walked from global memory keep their launches
bool svc_supported(const AccelView &ac);
// does the scene's session run the LDS-tree kernel (1 024-thread blocks)?
bool svc_lds(const AccelView &ac);
// the LDS-tree session's grid: every block slot (full) or one per CU fewer, at least one
// per CU; 0 when the LDS-tree kernel cannot run on this device
uint32_t svc_lds_grid(bool full);
// threads per block of the session kernel for this scene
uint32_t svc_block(const AccelView &ac);

struct FoldArgs {
    const uint32_t *samples;  // slot_words per slot, in item order (ts_slot_base)
    uint32_t slot_words;
    const float4 *shade;      // the scene's shading table (diffuse codes name its slots)
    float sky[3];             // initColor (sky words)
    FastDiv code_div;         // FastDiv(code stride): diffuse_decode
    float4 *acc;         // persistent accumulator (w = sample count)
    float4 *out_rgba;    // nullable, local pixel order
    uint8_t *out_rgb8;   // nullable, full frame (g_data layout)
    RowMap map;
    uint32_t width, height, npix, spp_batch, spp_total;
    uint32_t s_done;     // samples folded after this batch (s0 + spp_batch)
    int first, last, mode;
    int preview;         // write the outputs after every batch (progressive rendering)
    int prio;            // fold_kernel raises its waves' priority (launched renders; not beside the service)
    int alias;           // task mode, one non-square rectangle: RenderSegmentTask's colorIndex
                         // (dx + dy * segmentHeight, TaskBasedPathTracer.hpp:103,186) aliases pixels
    const BatchRect *rects;  // batched fold: n_rects rectangles over npix = their total pixels
    uint32_t n_rects;        // (map and alias per rectangle; spp_batch = spp_total, first = last = 1)
    // range alias fold (spt_render_frame: RenderSegmentTask over a non-square frame split
    // over several devices by ranges of its colorIndex): the npix outputs are the alias
    // indices [out_i0, out_i0 + npix) of a call of map.width x alias_h pixels, whose source
    // pixels' slots are those of the launch's rows (map: rows [map.y0, map.y0 + src_rows))
    uint32_t range_alias, out_i0, alias_h, src_rows;
    // batched fold: the render's claim counters (head[k * kQueueStride], k < head_queues),
    // zeroed for the workspace's next launch (no memset before it); null = leave them
    uint32_t *head_reset;
    uint32_t head_queues;
    uint32_t inline_rects;                 // as RenderArgs::inline_rects / rects_inline
    BatchRect rects_inline[kInlineRects];
};

// Launch geometry of one render launch: the context's persistent grid for the
// 256-thread kernels (`grid`, `block`), a divisor of every kernel's full grid (several
// host calls in flight share the GPU side by side), and on return the grid and block
// the chosen kernel ran with (the LDS tree kernel sizes its own: 1024-thread blocks).
struct LaunchShape {
    uint32_t grid, block, div;
    uint32_t ran_grid, ran_block;
};
hipError_t launch_render(const RenderArgs &a, LaunchShape &sh, hipStream_t s);

// Wavefront variant (spt_wavefront.hip): per-block ray queues of qcap rays (three
// 16-byte records per ray; cap = blocks x qcap) and the batch's item counter.
constexpr uint32_t kWfCats = 5;  // sky/miss, diffuse first hit, mirror, glass, diffuse-loop step
constexpr uint32_t kWfStateWords = 4;
struct WavefrontBuffers {
    float4 *o, *d;
    uint4 *m;
    uint32_t *state;  // [kWfStateWords]
    uint32_t cap, qcap;
};
// Every pass of a sample batch's paths through the ray queues, in one launch: the
// host issues it and waits for nothing (queue lengths stay on the device).
hipError_t launch_wavefront(const WavefrontBuffers &b, const RenderArgs &a, hipStream_t s);
// Blocks of the engine resident at once on device dev (its launch's grid), 0 on error.
uint32_t wavefront_blocks(const AccelView &ac, int dev);
hipError_t launch_fold(const FoldArgs &a, hipStream_t s);
// spt_render_samples: pixels [p0, p0 + n) of the region, out[(p - p0) * spp + s]
hipError_t launch_expand(const FoldArgs &a, float4 *out, uint32_t p0, uint32_t n, hipStream_t s);
hipError_t launch_assemble(const float4 *tiles, uint32_t max_rows, RowMap base, uint32_t width, uint32_t height,
                           float4 *frame, uint8_t *rgb8, hipStream_t s);
hipError_t launch_selftest(const float *a, const float *b, const uint32_t *bits, uint32_t n, float *out,
                           hipStream_t s);
hipError_t render_occupancy(uint32_t block, int *blocks_per_cu);
uint32_t render_group_size();  // spheres per group of the hot loop (SPT_GROUP)

constexpr uint32_t kSpecularCap = 1024;  // see spt_oracle.h SPO_SPECULAR_CAP
constexpr uint32_t kTaskPasses = 10;     // TaskBasedPathTracer.hpp:81
// threads per block of the 256-thread render kernels (the LDS tree kernel has its own)
#ifndef SPT_RENDER_BLOCK
#define SPT_RENDER_BLOCK 256
#endif
constexpr uint32_t kRenderBlock = SPT_RENDER_BLOCK;
uint32_t render_block_size();  // kRenderBlock of the kernel object (the launch uses it)
// true when launch_render walks this tree lane by lane (LDS or global-memory lane walk)
bool lane_walk_tree(const AccelView &ac);

}  // namespace spt
