/*
 * spt_hip.h -- C ABI of the MI355X (gfx950) render loop of SimplePathTracer.
 *
 * This is the drop-in boundary.  The reference's hot path is reached through
 * two void free functions that read mutable globals and write bytes into the
 * caller-owned framebuffer g_data:
 *
 *   void RenderSegment(RenderSegmentData)       SingleThreadPathTracer.hpp:114-137
 *   void RenderSegmentTask(RenderSegmentData)   TaskBasedPathTracer.hpp:54-206
 *
 * called from RenderJob (Renderer.hpp:242-255) on up to threadCount concurrent
 * threads and from RenderImage (Renderer.hpp:304-308).  Their implicit inputs
 * are the globals of Globals.hpp:8-37 (scene SoA, viewMatrix, eyePos,
 * initColor, g_width/g_height/g_samples/g_bounces).  The functions below make
 * each of those inputs explicit; include/spt/RenderSegmentShim.hpp rebuilds the
 * two reference entry points on top of them so Renderer.hpp / Main.cpp and the
 * GL preview keep compiling unchanged.
 *
 * Plain C types only.  Every function returns an spt_status; on failure
 * spt_last_error() describes why.  A context is safe to use from several host
 * threads: its state is guarded by a lock, and concurrent render calls (the
 * reference's RenderJob threads) are rendered together: the calls that arrive while
 * one batch renders form the next (one render + one fold launch over their tiles).
 */
#ifndef SPT_HIP_H
#define SPT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPT_ABI_VERSION 11

/* Only the functions below are exported from libspt_hip.so (built with
 * -fvisibility=hidden), so several builds can be loaded side by side. */
#if defined(__GNUC__)
#define SPT_API __attribute__((visibility("default")))
#else
#define SPT_API
#endif

typedef enum spt_status {
    SPT_OK = 0,
    SPT_ERR_ARG = 1,      /* invalid argument (null pointer, bad range, ...) */
    SPT_ERR_STATE = 2,    /* scene / camera / params not set */
    SPT_ERR_HIP = 3,      /* HIP runtime error */
    SPT_ERR_NOMEM = 4,    /* allocation failed */
    SPT_ERR_NODEVICE = 5, /* no gfx950 device / bad ordinal */
    SPT_ERR_TIMEOUT = 6   /* a render-service session did not end within SPT_SVC_TIMEOUT_MS
                             (default 30 s); the message counts its unpublished jobs */
} spt_status;

/* Material ids, Definitions.hpp:7-13 (enum class Material : uint8_t). */
enum { SPT_SKYBOX = 0, SPT_REFLECTIVE = 1, SPT_REFRACTIVE = 2, SPT_DIFFUSE = 3 };

/* Render modes: which reference entry point's semantics a launch follows. */
enum {
    SPT_MODE_SEGMENT = 0,  /* RenderSegment: every sample counts, acc *= 1/spp  */
    SPT_MODE_TASK = 1      /* RenderSegmentTask: paths needing > 10 passes are
                              dropped (TaskBasedPathTracer.hpp:81) and the pixel
                              is averaged over the samples that finished (196-205) */
};

typedef struct spt_ctx spt_ctx;

#define SPT_DIAG_WORDS 26

typedef struct spt_stats {
    uint64_t samples;      /* (pixel, sample) paths completed */
    uint64_t casts;        /* FindClosestIntersectionSphere calls (rays) */
    uint64_t dropped;      /* task mode: samples dropped by the pass cap */
    uint64_t launches;     /* render-kernel launches */
    double render_ms;      /* summed device time of render-kernel launches */
    double fold_ms;        /* summed device time of resolve (fold) launches */
    double last_render_ms; /* device time of the most recent render launch */
    uint32_t grid_blocks;  /* grid of the most recent render launch (the persistent grid
                              before any launch) */
    uint32_t block_threads; /* its block size (256; 1024 for the LDS tree kernel) */
    double render_busy_ms; /* length of the union of the render launches' intervals: with
                              frames in flight on several streams launches overlap, and
                              this is the device time during which some render launch ran */
    uint64_t diag[SPT_DIAG_WORDS]; /* diagnostic build only (-DSPT_DIAG=1): wave iterations,
                              clusters entered, tree nodes tested, s_memtime cycles in
                              cast / shading / refill, (lane, cluster) pairs that may
                              pass, live lanes of entered clusters, spheres tested per
                              wave, their update branches taken (some lane passes),
                              lanes passing in those branches, branches that
                              improve some lane's winner, RaySphereIntersection
                              evaluations for live lanes (lane-tests), member pretests
                              for live lanes (lane-pretests); then, of the primary
                              batches (64 new paths of one 8x8 tile cast together):
                              iterations, tree nodes tested, spheres tested, update
                              branches taken, s_memtime cycles of their casts; the
                              cube-minus-ball sampler's calls and its cooperative rounds
                              after round 0; tree leaves entered by at most 8 and at
                              most 16 lanes; s_memtime cycles in the sampler; wave
                              iterations after the launch's items ran out (the drain)
                              and their live lanes */
    uint64_t batches;       /* batched launches of concurrent spt_render_segment[_task] calls */
    uint64_t batched_calls; /* calls rendered in them */
    /* render service (spt_service_start); the device counters above include a session's
       waves once the session has ended (spt_service_stop, spt_synchronize) */
    uint64_t svc_sessions;       /* service sessions (resident launches) started */
    uint64_t svc_jobs;           /* jobs published to them */
    uint64_t svc_watchdog_exits; /* sessions whose waves left after 0.5 s without work */
    double svc_kernel_ms;        /* summed device time of the ended sessions' launches */
    uint32_t svc_running;        /* a session is resident now */
    uint32_t svc_grid_blocks;    /* the service's grid (one block slot per CU left free) */
    uint64_t svc_flow_restarts;  /* sessions ended because a publication would have waited for
                                    an unfinished fold (ring words or counter still in use) */
    uint64_t svc_closing_restarts; /* sessions ended because a wave had raised its closing flag */
    uint32_t prim_list_blocks;   /* 8x8 pixel blocks with a primary-ray candidate list (0: lists off) */
    uint32_t prim_list_entries;  /* candidate slots over all blocks' lists (8x8 and 8x4) */
    double prim_list_build_ms;   /* host time of their last build */
    uint64_t prim_list_builds;   /* builds so far (a setter rebuilds the lists only when the
                                    accel tables, the camera or the frame size changed) */
    double accel_build_ms;       /* host time of the last traversal-table build + upload
                                    (spt_set_scene / cluster setters) */
} spt_stats;

SPT_API int spt_abi_version(void);
/* Number of visible HIP devices. */
SPT_API int spt_device_count(int *count);

/* Context on one device.  Replaces nothing in the reference (its state is global);
 * it owns the device copies of Globals.hpp's scene/camera and a workspace. */
SPT_API int spt_ctx_create(int device, spt_ctx **out);
/* Context over several devices (one process driving the node's
 * GPUs).  devices[0] is member 0; a device may be listed more than once (members on
 * one device render concurrently on their own streams).  Every setter applies to all
 * members (each keeps its own copy of the scene); spt_render_frame splits the frame
 * over the members; spt_render_segment[_task] / spt_render_progressive send each
 * call (a RenderJob tile) to the member with the fewest calls in flight; the other
 * entry points (rows/assemble/samples/selftest) use member 0. */
SPT_API int spt_ctx_create_multi(const int *devices, uint32_t n, spt_ctx **out);
/* Members of ctx: on entry *n = capacity of devices (nullable), on return *n = count. */
SPT_API int spt_ctx_devices(spt_ctx *ctx, uint32_t *n, int *devices);
SPT_API void spt_ctx_destroy(spt_ctx *ctx);
/* Last error of ctx, or of the calling thread when ctx is NULL. Never NULL. */
SPT_API const char *spt_last_error(const spt_ctx *ctx);

/* Scene SoA, Globals.hpp:31-37: g_spheres (float4 per sphere, w ignored),
 * g_radii, g_colors (float4, w ignored), g_materials, g_diffuses (fuzz),
 * g_sphereNumber.  Data is copied.  The reference's uint8_t sphere index
 * (Collision.hpp:87-92) limits it to n <= 255; this build uses a 32-bit index,
 * identical for n <= 255, and accepts larger scenes as an extension. */
SPT_API int spt_set_scene(spt_ctx *ctx, const float *centers4, const float *radii, const float *colors4,
                  const uint8_t *materials, const float *fuzz, uint32_t n);
/* viewMatrix (row-major, already transposed, Renderer.hpp:321; its fourth row
 * must be zero as CreateCameraBasisMatrix makes it), eyePos and initColor
 * (Globals.hpp:21-29).  w lanes of eye/sky are ignored (0 in the reference). */
SPT_API int spt_set_camera(spt_ctx *ctx, const float view[16], const float eye[4], const float sky[4]);
/* g_width, g_height, g_samples, g_bounces (Globals.hpp:12-15) + RNG seed.
 * bounces == 0 is rejected: `while (--bounceCount && ...)` would never count
 * down (SingleThreadPathTracer.hpp:28). */
SPT_API int spt_set_params(spt_ctx *ctx, uint32_t width, uint32_t height, uint32_t spp, uint32_t bounces, uint64_t seed);
/* Hot-loop culling: small spheres are grouped into clusters of k <= 8
 * (SPT_CLUSTER_AUTO, the default: 4 for a flat cluster list, 8 for a tree)
 * whose conservative bounding test skips them exactly when no ray of a wave can
 * pass RaySphereIntersection for any member; k = 0 tests every sphere for every
 * ray (the reference's brute force).  Results are identical either way. */
#define SPT_CLUSTER_AUTO 0xFFFFFFFFu
SPT_API int spt_set_cluster_size(spt_ctx *ctx, uint32_t k);
/* Clusters are the leaves of a tree of expanded boxes (built top down by the
 * surface-area heuristic); `branching` children per inner node at most, 0 = flat list
 * of clusters under bounding spheres, SPT_TREE_AUTO (default) = a tree with 4 (scenes
 * of <= 512 spheres) or 3 children.  Trees of 64..2431 nodes are walked lane by lane
 * from LDS, up to 9000 nodes lane by lane from global memory, others by the whole
 * wave.  Results are identical for any value. */
#define SPT_TREE_AUTO 0xFFFFFFFFu
SPT_API int spt_set_cluster_tree(spt_ctx *ctx, uint32_t branching);
/* Keep `n` CUs free of render launches (0, the default: none).  A launched render then
 * runs on a stream of ctx's own whose CU mask leaves out the mask's last n bits
 * (hipExtStreamCreateWithCUMask; the driver deals mask bits out XCC first, then shader
 * engine, so n = 8 is one CU per XCC and n = 32 one per shader engine on MI355X), ordered
 * after the caller's stream and before its later work, with a persistent grid sized to
 * the CUs it may use.  For co-scheduling other work beside a render: a block that needs
 * a whole CU (RCCL's gfx950 collective kernels: 248-256 VGPRs per wave) waits for room in
 * the shader engine it is dispatched to, so it starts at once only with one free CU per
 * engine (DESIGN.md §5 "Reserved CUs": 3.1 ms vs 18.5 ms into a 19 ms render at n = 32;
 * not bench.py's default -- the multi-rank bench is faster with the render service).
 * Results are identical for any n; the render service ignores it.  n < the CU count. */
/* The drop-in's warm-up (the C++ shim calls it once, right after creating its
 * context): creates the streams of the second batch set and of the tiling read-ahead
 * now, so that the first frame does not pay for them (a HIP stream costs ~9.5 ms to
 * create on MI355X and stalls the device's other queues meanwhile), runs one small
 * device-to-host 2D copy and one host-to-device upload (the process's first of each waits
 * ~8.5 ms for the runtime's copy setup: the first frame's tile copies, the setup's list
 * upload), and lets the tiling
 * read-ahead arm at a tiling's first call (RenderImageParallelMain's first tile to arrive)
 * rather than after one whole tiling, so that the reference app's one frame per process
 * (Renderer.hpp:335-344) is rendered whole at its first tile (SPT_READAHEAD_FIRST=0: not).
 * Results unchanged; optional. */
SPT_API int spt_prepare_dropin(spt_ctx *ctx);
SPT_API int spt_set_reserved_cus(spt_ctx *ctx, uint32_t n);
/* Host-only check (no device needed): build the traversal tables for a scene and
 * verify the properties exactness rests on (every sphere once, preorder/skip
 * structure of all 8 octant layouts, each node's bounding sphere contains every
 * member below it).  *out_nodes (nullable) = tree nodes per layout. */
SPT_API int spt_accel_check(const float *centers4, const float *radii, uint32_t n, uint32_t cluster_k,
                            uint32_t branching, uint32_t *out_nodes);
/* Host-only check (no device needed): the primary-ray candidate lists (DESIGN.md §4.2
 * item 6) a context builds for this scene (default traversal shape), camera (view as
 * spt_set_camera) and frame size.  counts[4] = {list entries, slots, blocks per row,
 * lists on}.  blocks8 (2 * ceil(width/8) * ceil(height/8) words) and blocks4
 * (2 * ceil(width/8) * ceil(height/4)) receive {first entry, count} per block (count
 * 0xFFFFFFFF: the block walks the tree), slot_ids the entries and slot_orig the sphere
 * index of every slot (0xFFFFFFFF: dummy); each nullable, the last two of capacity cap.
 * max_count: longer lists walk (the contexts use 24, SPT_PRIM_MAX). */
SPT_API int spt_prim_lists_check(const float *centers4, const float *radii, uint32_t n, const float view[16],
                                 const float eye[4], uint32_t width, uint32_t height, uint32_t max_count,
                                 uint32_t *blocks8, uint32_t *blocks4, uint32_t *slot_ids, uint32_t *slot_orig,
                                 uint32_t cap, uint32_t *counts);
/* Engine of the render loop (results are bit-identical either way):
 * SPT_ENGINE_MEGAKERNEL (default) -- one persistent kernel, per-lane state machines;
 * SPT_ENGINE_WAVEFRONT -- RenderSegmentTask's material-queue design
 *   (TaskBasedPathTracer.hpp:54-193): one launch per sample batch whose blocks are
 *   queue workers -- each block casts its ray queue, sorts the rays by material in LDS
 *   (ballot/prefix), shades them and compacts the survivors in place, pass after pass.
 *   Queue lengths never leave the device: the host issues the launch and reads nothing
 *   back. */
enum { SPT_ENGINE_MEGAKERNEL = 0, SPT_ENGINE_WAVEFRONT = 1 };
SPT_API int spt_set_engine(spt_ctx *ctx, int engine);
/* Upper bound of the per-sample workspace (default 16 GiB).  Larger frames are
 * rendered in sample batches folded in order. */
SPT_API int spt_set_workspace(spt_ctx *ctx, uint64_t bytes);

/* ---- drop-in entry points (host memory, blocking) ----------------------------
 * Render pixels [yBegin,yEnd) x [xBegin,xEnd).  Concurrent calls on one context run
 * on the GPU together (up to 8 in flight per device; SPT_HOST_SLOTS lowers it).
 * rgba_out (nullable): region-local row-major float4 per pixel = the reference's
 *   pixelColor after `*= 1/g_samples` (the value WritePixel receives).
 * g_data (nullable): full-frame width*height*3 bytes; the region's pixels are
 *   written at g_size - ((g_width - x)*3 + y*g_width*3) exactly as
 *   io::WritePixel does (IOHelpers.hpp:17-22), other bytes untouched. */
SPT_API int spt_render_segment(spt_ctx *ctx, uint32_t yBegin, uint32_t yEnd, uint32_t xBegin, uint32_t xEnd,
                       float *rgba_out, uint8_t *g_data);
/* The whole frame (RenderImage, Renderer.hpp:304-308, over every device of the
 * context): member r of n renders the interleaved row strips r, r+n, ... (strip =
 * the largest of 8/4/2/1 rows that deals the strips evenly) into a compact tile;
 * member 0 pulls the tiles over xGMI (peer copies), scatters them into the frame and
 * writes rgba_out (nullable, width*height float4, row-major) and g_data (nullable,
 * the reference layout).  Pixels are keyed per (pixel, sample), so the frame is
 * bit-identical for any member count.  In task mode a non-square frame
 * (RenderImage's RenderSegmentTask({0, H, 0, W}) aliases pixels across rows,
 * TaskBasedPathTracer.hpp:103,186) is split by ranges of its colorIndex instead: member
 * r folds outputs [r L, (r + 1) L) from the rows holding their sources.  Blocking. */
SPT_API int spt_render_frame(spt_ctx *ctx, int mode, float *rgba_out, uint8_t *g_data);
/* Progressive RenderSegment / RenderSegmentTask (the preview of RenderImageParallelMain,
 * Renderer.hpp:257-302): the region is rendered in passes of pass_spp samples; after
 * each pass rgba_out / g_data (either nullable) hold the render at the samples done so
 * far -- bit-identical to a render with g_samples = samples_done, since samples are
 * keyed per (pixel, sample) -- and cb(user, samples_done) runs on the calling thread
 * (nullable; a nonzero return stops the render there).  The last pass is the full
 * render.  cb runs with the context unlocked: it may read stats, pin buffers or render
 * elsewhere, but setters of the same context called from it fail with SPT_ERR_STATE. */
/* Page-lock a caller-owned host buffer -- typically g_data (Globals.hpp:19, malloc'd)
 * -- so the per-call device-to-host copy of the render is a direct DMA and the GL
 * thread's UpdateTexture (Renderer.hpp:157-164) reads the same pinned bytes.
 * Idempotent per pointer; spt_unpin_host releases it (spt_ctx_destroy releases all). */
SPT_API int spt_pin_host(spt_ctx *ctx, void *ptr, size_t bytes);
SPT_API int spt_unpin_host(spt_ctx *ctx, void *ptr);
typedef int (*spt_progress_fn)(void *user, uint32_t samples_done);
SPT_API int spt_render_progressive(spt_ctx *ctx, int mode, uint32_t yBegin, uint32_t yEnd, uint32_t xBegin,
                                   uint32_t xEnd, uint32_t pass_spp, float *rgba_out, uint8_t *g_data,
                                   spt_progress_fn cb, void *user);
SPT_API int spt_render_segment_task(spt_ctx *ctx, uint32_t yBegin, uint32_t yEnd, uint32_t xBegin, uint32_t xEnd,
                            float *rgba_out, uint8_t *g_data);

/* ---- device-resident entry point (asynchronous) -------------------------------
 * Rows y in [yBegin,yEnd) with ((y - yBegin) / strip) % parts == part, columns
 * [xBegin,xEnd) -- the interleaved row-strip tiling used to split a frame over
 * GPUs (parts = world size, part = rank; parts = 1 for a plain rectangle).
 * d_rgba (nullable): device float4 per local pixel, local order (row k of the
 *   owned rows, then x).  d_rgb8 (nullable): device full frame in g_data layout.
 * stream: a hipStream_t; NULL is HIP's default (null) stream, as for any HIP
 * call.  Launches are ordered on that stream only.  Returns after enqueueing;
 * pair with spt_synchronize or the caller's stream sync.  Each distinct stream
 * (up to 4 per context) gets its own workspace, so renders enqueued on different
 * streams may be in flight together: the next frame's blocks then fill the GPU
 * while the previous frame's last paths drain. */
SPT_API int spt_render_rows_async(spt_ctx *ctx, int mode, uint32_t yBegin, uint32_t yEnd, uint32_t strip, uint32_t parts,
                          uint32_t part, uint32_t xBegin, uint32_t xEnd, void *d_rgba, void *d_rgb8, void *stream);
/* ---- render service ----------------------------------------------------------------
 * spt_service_start: from now on the renders of spt_render_rows_async, spt_render_frame
 * and the unbatched host calls are jobs of a resident render service instead of launches
 * of their own.  One launch of the service kernel (a "session") stays on the device and
 * renders the jobs in the order they are published: claims of the next job fill the CUs
 * while the last paths of the previous one drain, so consecutive frames, rank shares and
 * sample batches pay no launch ramp and tail each.  A job's fold waits for its completion
 * counter on the caller's stream (hipStreamWaitValue32); results are bit-identical to the
 * launched renders.  Sessions start on the first job and end on spt_service_stop,
 * spt_synchronize, a setter, a render the service does not take (lane-walk trees,
 * spt_render_samples, the wavefront engine, jobs over half the slot ring: 1/16 of device
 * memory within [4, 16] GiB), when a
 * publication would have to wait for an unfinished fold (the ring wrapped onto words a
 * fold still reads; the next session's launch waits for it instead), or when its waves
 * have gone idle: a session's waves may leave after 0.5 s without work -- only through
 * a handshake with the host, so no job is ever published to a session that left -- and a
 * device-wide synchronisation (hipDeviceSynchronize, torch.cuda.synchronize) therefore
 * waits at most that long.  spt_service_stop drains and ends the session and turns the
 * service off.  Every host wait for a session is bounded (SPT_SVC_TIMEOUT_MS, default
 * 30 s: SPT_ERR_TIMEOUT). */
SPT_API int spt_service_start(spt_ctx *ctx);
/* full != 0: sessions take every block slot (SPT_SVC_FULL_GRID's setting, for callers that
 * end their sessions themselves and need no kernel of their own beside one); 0: one slot
 * per CU left free (the default).  SPT_ERR_STATE while a session runs. */
SPT_API int spt_service_set_full_grid(spt_ctx *ctx, uint32_t full);
SPT_API int spt_service_stop(spt_ctx *ctx);

/* Number of rows the (yBegin, yEnd, strip, parts, part) map owns. */
SPT_API int spt_rows_count(uint32_t yBegin, uint32_t yEnd, uint32_t strip, uint32_t parts, uint32_t part, uint32_t *rows);
/* Scatter a gathered, rank-major stack of local float4 tiles (parts tiles of
 * max_rows*(xEnd-xBegin) pixels each, on device) into a full-frame float4
 * buffer and/or a g_data RGB8 frame.  Used by rank 0 after the RCCL gather. */
SPT_API int spt_assemble_rows_async(spt_ctx *ctx, const void *d_tiles, uint32_t max_rows, uint32_t yBegin, uint32_t yEnd,
                            uint32_t strip, uint32_t parts, uint32_t xBegin, uint32_t xEnd, void *d_frame_rgba,
                            void *d_rgb8, void *stream);
SPT_API int spt_synchronize(spt_ctx *ctx);
/* The rank-share form of RenderImage's RenderSegmentTask({0, H, 0, W}) on a NON-SQUARE
 * frame (mode TASK, W != H).  There the reference strides its colour accumulator by the
 * tile height (TaskBasedPathTracer.hpp:103,186,196-205), so pixels alias across rows and a
 * row-strip split cannot resolve them locally; the frame is split by output index instead.
 * spt_task_range: part `part` of `parts`'s outputs [i0, i1) of the frame's row-major order
 * (outputs with sources dealt evenly; the last part also takes the source-less tail,
 * which resolves to NaN / bytes 0).  spt_render_task_range_async: renders the rows
 * holding those outputs' sources and writes outputs [i0, i1) to d_rgba[0, i1 - i0)
 * (float4, device) on `stream`.  The parts' outputs end to end are the frame, which
 * spt_assemble_rows_async turns into RGBA / g_data with max_rows = H, strip 1, parts 1.
 * (spt_render_frame does the same over a multi-device context.) */
SPT_API int spt_task_range(uint32_t width, uint32_t height, uint32_t parts, uint32_t part, uint32_t *i0, uint32_t *i1);
SPT_API int spt_render_task_range_async(spt_ctx *ctx, uint32_t i0, uint32_t i1, void *d_rgba, void *stream);

/* ---- copy-engine tile transport (one process per GPU, ranks of one node) -------------
 * The alternative to distributed.py's RCCL gather of the rank tiles (Renderer.hpp:257-302's
 * tile split; DESIGN.md §5 "Round 6"): rank 0 holds nbuf gathered buffers of world tiles
 * (tile_bytes each, rank-major, the layout spt_assemble_rows_async reads) in one device
 * allocation it exports by IPC handle; rank r > 0 copies its tile into slot r of the
 * frame's buffer with an asynchronous device-to-device copy on its own stream (peer
 * memory over xGMI) and then raises its ready word; rank 0's stream waits for every ready
 * word before its assemble and raises the buffer's consumed word after it, which a
 * rank's copy into the same buffer nbuf frames later waits for.  The words live in a
 * POSIX shared-memory segment (/dev/shm) page-locked in every process: stream
 * wait/write-value packets, no host thread and no collective kernel on the path.
 * Frames are numbered 0, 1, ... identically on every rank; frame f uses buffer f % nbuf.
 * Setup: rank 0 calls spt_tiles_create(name) first; after a barrier every other rank
 * calls it with the same name, then spt_tiles_attach with rank 0's spt_tiles_handle;
 * after another barrier rank 0 may spt_tiles_unlink the name (the mappings stay).
 * Rank 0 renders its own tile into slot 0 of spt_tiles_buffer(frame) on a stream ordered
 * after its spt_tiles_release_async(frame - nbuf).  spt_tiles_destroy synchronizes the
 * device (stop the render service first: a resident session would hold it up to its idle
 * exit).  Errors: SPT_ERR_ARG (bad sizes, a segment name in use), SPT_ERR_STATE (a call for
 * the other side), SPT_ERR_HIP. */
typedef struct spt_tiles spt_tiles;
SPT_API int spt_tiles_create(spt_ctx *ctx, const char *name, uint32_t rank, uint32_t world, uint64_t tile_bytes,
                             uint32_t nbuf, spt_tiles **out);
SPT_API int spt_tiles_handle(spt_tiles *t, uint8_t handle[64]);
SPT_API int spt_tiles_attach(spt_tiles *t, const uint8_t handle[64]);
SPT_API int spt_tiles_unlink(spt_tiles *t);
SPT_API int spt_tiles_buffer(spt_tiles *t, uint64_t frame, void **d_buffer);
SPT_API int spt_tiles_send_async(spt_tiles *t, uint64_t frame, const void *d_tile, void *stream);
/* The same for `bytes` at byte `offset` of the frame's buffer instead of slot `rank` (the
 * task-range split, spt_task_range: each part's outputs at their place in the frame) */
SPT_API int spt_tiles_send_range_async(spt_tiles *t, uint64_t frame, const void *d_src, uint64_t offset,
                                       uint64_t bytes, void *stream);
SPT_API int spt_tiles_recv_async(spt_tiles *t, uint64_t frame, void *stream);
SPT_API int spt_tiles_release_async(spt_tiles *t, uint64_t frame, void *stream);
/* Give the transport up: every ready / consumed word of the shared segment set to the
 * largest value from the host, so that no rank's stream stays blocked on a wait packet
 * (then destroy it).  Used when the setup check (distributed.TileTransport.verify) fails. */
SPT_API int spt_tiles_abort(spt_tiles *t);
SPT_API void spt_tiles_destroy(spt_tiles *t);

/* Per-(pixel, sample) colors of a rectangle, host memory: out[(p*spp + s)*4 + c]
 * with p the region-local pixel.  w = 1 if the sample counts, 0 if dropped
 * (task mode).  Debug/parity aid; same kernel as the render path. */
SPT_API int spt_render_samples(spt_ctx *ctx, int mode, uint32_t yBegin, uint32_t yEnd, uint32_t xBegin, uint32_t xEnd,
                       float *out);

SPT_API int spt_get_stats(spt_ctx *ctx, spt_stats *out);
SPT_API int spt_reset_stats(spt_ctx *ctx);

/* ---- input producers (SceneGenerators.hpp, Math.hpp) -------------------------
 * GenerateSpheres (SceneGenerators.hpp:6-66) and InitSpheres (68-133) driven by
 * splitmix(seed) (Random.hpp:19) instead of the clock; capacity in spheres. */
SPT_API int spt_scene_generate_random(uint32_t seed, uint32_t capacity, float *centers4, float *radii, float *colors4,
                              uint8_t *materials, float *fuzz, uint32_t *n_out);
/* GenerateSpheres with its row loop (SceneGenerators.hpp:32) run to z < z_end instead of
 * 20 (z_end = 20 is spt_scene_generate_random): BASELINE.json's "~500-sphere" RTIOW scene
 * with the reference's placement rule and draw order (z_end 37.5: 488 spheres, seed 1). */
SPT_API int spt_scene_generate_random_rows(uint32_t seed, float z_end, uint32_t capacity, float *centers4, float *radii,
                                           float *colors4, uint8_t *materials, float *fuzz, uint32_t *n_out);
SPT_API int spt_scene_init_reference(uint32_t seed, float *centers4, float *radii, float *colors4, uint8_t *materials,
                             float *fuzz, uint32_t *n_out);
/* Stress scene for the >255-sphere extension (BASELINE config 5): the four big
 * spheres of GenerateSpheres plus n-4 small spheres on a jittered grid. */
SPT_API int spt_scene_generate_stress(uint32_t seed, uint32_t n, float *centers4, float *radii, float *colors4,
                              uint8_t *materials, float *fuzz);
/* Transpose(CreateCameraBasisMatrix(eye, lookAt, up)), Math.hpp:198-231. */
SPT_API int spt_camera_basis(const float eye[4], const float look_at[4], const float up[4], float view_out[16]);

/* io::SaveImage (IOHelpers.hpp:24-27) without stb: writes g_data (width x height,
 * comp = g_stride = 3 bytes per pixel, row 0 first) as the 24-bit BMP that
 * stbi_write_bmp(path, width, height, 3, g_data) writes: 54-byte header, rows
 * from the last to the first, BGR, each row zero-padded to 4 bytes. */
SPT_API int spt_save_bmp(const char *path, uint32_t width, uint32_t height, uint32_t comp, const uint8_t *data);

/* ---- numerics self-test ------------------------------------------------------
 * Runs the device primitives the render path relies on over n inputs and
 * writes SPT_SELFTEST_COLS floats per input: a/b, sqrtf(a),
 * glibc's powf(a, 5) and powf(c, 5) restated, powf(a, 2), the refraction scalar
 * r*a - sqrt(1 - r*r*(1 - a*a)) (r = 1/1.5; -1e30 under total reflection), uniform(-1,1)
 * of bits, u8 of a, Normalize({a, b, c}) (3 floats), c/a, uniform(-0.5,0.5) and
 * uniform(0,1) of bits, with c the float whose bit pattern is bits; then c and a
 * halved j times as the fold rebuilds a diffuse sample (j = (bits * 2654435761) >> 23
 * mod 301; spt_kernels.hip halve_n). */
#define SPT_SELFTEST_COLS 16
SPT_API int spt_selftest_numerics(spt_ctx *ctx, const float *a, const float *b, const uint32_t *bits, uint32_t n,
                          float *out);

#ifdef __cplusplus
}
#endif
#endif
