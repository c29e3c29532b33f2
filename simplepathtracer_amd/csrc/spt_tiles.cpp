// Copy-engine tile transport between the ranks of one node (spt_tiles_*, include/spt_hip.h;
// DESIGN.md §5 "Round 6"): the rank tiles of a frame reach rank 0 by asynchronous
// device-to-device copies into a buffer rank 0 exported by IPC handle, ordered by
// stream wait/write-value packets on words in a small shared host segment -- no kernel,
// no host thread, no collective on the path.  The alternative to the RCCL gather of
// distributed.py (Renderer.hpp:257-302's tile split).
#include "spt_host.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <string>

// Word layout of the shared segment (one 64-byte line per word, so no two writers share
// a line): ready[r][b] at line r * nbuf + b (r >= 1), consumed[b] at line b (r = 0).
struct spt_tiles {
    spt_ctx *ctx = nullptr;
    uint32_t rank = 0, world = 0, nbuf = 0;
    uint64_t tile_bytes = 0;
    std::string name;    // "/spt_tiles_<name>"
    bool owner = false;  // rank 0: created the segment and the buffers
    void *host = nullptr;  // the segment, mapped
    size_t host_bytes = 0;
    uint8_t *words = nullptr;  // its device address (page-locked, mapped)
    bool registered = false;
    uint8_t *buf = nullptr;  // nbuf x world tiles: rank 0's allocation, or the IPC mapping of it
    bool opened = false;     // buf is an IPC mapping
};

namespace {

constexpr size_t kLine = 64;

uint32_t *word(spt_tiles *t, uint32_t r, uint32_t b)
{
    return (uint32_t *)(t->words + ((size_t)r * t->nbuf + b) * kLine);
}

// frame f uses buffer f % nbuf for the (f / nbuf + 1)-th time: the value its words take
uint32_t generation(const spt_tiles *t, uint64_t frame) { return (uint32_t)(frame / t->nbuf + 1u); }

int tiles_fail(spt_tiles *t, int code, const char *what)
{
    return fail(t ? t->ctx : nullptr, code, "%s", what);
}

void release(spt_tiles *t)
{
    if (t->buf) {
        if (t->opened)
            (void)hipIpcCloseMemHandle(t->buf);
        else
            (void)hipFree(t->buf);
        t->buf = nullptr;
    }
    if (t->registered) (void)hipHostUnregister(t->host);
    t->registered = false;
    if (t->host) munmap(t->host, t->host_bytes);
    t->host = nullptr;
    if (t->owner && !t->name.empty()) shm_unlink(t->name.c_str());  // no-op once unlinked
}

}  // namespace

extern "C" {

int spt_tiles_create(spt_ctx *ctx, const char *name, uint32_t rank, uint32_t world, uint64_t tile_bytes,
                     uint32_t nbuf, spt_tiles **out)
{
    if (!ctx || !out || !name || !*name) return fail(ctx, SPT_ERR_ARG, "null context, name or output");
    *out = nullptr;
    if (world < 2 || rank >= world || nbuf == 0 || nbuf > 16 || tile_bytes == 0 || tile_bytes % 16u)
        return fail(ctx, SPT_ERR_ARG, "tiles: rank %u of %u, %u buffers, %llu-byte tiles", rank, world, nbuf,
                    (unsigned long long)tile_bytes);
    for (const char *c = name; *c; ++c)
        if (*c == '/') return fail(ctx, SPT_ERR_ARG, "tiles: '/' in the segment name");
    spt_tiles *t = new spt_tiles;
    t->ctx = ctx;
    t->rank = rank;
    t->world = world;
    t->nbuf = nbuf;
    t->tile_bytes = tile_bytes;
    t->name = std::string("/spt_tiles_") + name;
    t->owner = rank == 0;
    const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    t->host_bytes = ((size_t)world * nbuf * kLine + page - 1) / page * page;
    // rank 0 creates the segment (zero-filled: every word starts at generation 0); the
    // others open it after rank 0's create (the caller's barrier)
    const int fd = t->owner ? shm_open(t->name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600)
                            : shm_open(t->name.c_str(), O_RDWR, 0600);
    if (fd < 0) {
        const int e = fail(ctx, SPT_ERR_ARG, "tiles: shm_open(%s): %s", t->name.c_str(), std::strerror(errno));
        t->owner = false;  // not ours to unlink
        delete t;
        return e;
    }
    if (t->owner && ftruncate(fd, (off_t)t->host_bytes) != 0) {
        close(fd);
        release(t);
        delete t;
        return fail(ctx, SPT_ERR_NOMEM, "tiles: ftruncate of the shared segment");
    }
    t->host = mmap(nullptr, t->host_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (t->host == MAP_FAILED) {
        t->host = nullptr;
        release(t);
        delete t;
        return fail(ctx, SPT_ERR_NOMEM, "tiles: mmap of the shared segment");
    }
    auto hip_fail = [&](hipError_t e, const char *what) {
        release(t);
        delete t;
        return fail(ctx, SPT_ERR_HIP, "tiles: %s: %s", what, hipGetErrorString(e));
    };
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    e = hipHostRegister(t->host, t->host_bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) return hip_fail(e, "hipHostRegister of the shared segment");
    t->registered = true;
    e = hipHostGetDevicePointer((void **)&t->words, t->host, 0);
    if (e != hipSuccess) return hip_fail(e, "hipHostGetDevicePointer");
    if (t->owner) {
        // uncached device memory: the other ranks' copy engines write it over xGMI, which no
        // L2 of this device observes, and the assemble reads each buffer again nbuf frames
        // later -- an uncached line cannot be stale.  (The assemble reads it once per frame:
        // 1/8 frame x 8 ranks of float4, no reuse to lose.)  Plain hipMalloc if refused.
        const size_t bytes = (size_t)nbuf * world * tile_bytes;
        e = hipExtMallocWithFlags((void **)&t->buf, bytes, hipDeviceMallocUncached);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            t->buf = nullptr;
            e = hipMalloc((void **)&t->buf, bytes);
        }
        if (e != hipSuccess) return hip_fail(e, "hipMalloc of the gathered buffers");
    }
    *out = t;
    return SPT_OK;
}

int spt_tiles_handle(spt_tiles *t, uint8_t handle[64])
{
    if (!t || !handle) return tiles_fail(t, SPT_ERR_ARG, "null tiles or handle");
    if (!t->owner) return tiles_fail(t, SPT_ERR_STATE, "tiles: only rank 0 exports the gathered buffers");
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, t->buf);
    if (e != hipSuccess) return fail(t->ctx, SPT_ERR_HIP, "tiles: hipIpcGetMemHandle: %s", hipGetErrorString(e));
    std::memcpy(handle, &h, 64);
    return SPT_OK;
}

int spt_tiles_attach(spt_tiles *t, const uint8_t handle[64])
{
    if (!t || !handle) return tiles_fail(t, SPT_ERR_ARG, "null tiles or handle");
    if (t->owner) return SPT_OK;
    if (t->buf) return tiles_fail(t, SPT_ERR_STATE, "tiles: already attached");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, 64);
    hipError_t e = hipSetDevice(t->ctx->device);
    if (e == hipSuccess) e = hipIpcOpenMemHandle((void **)&t->buf, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        t->buf = nullptr;
        return fail(t->ctx, SPT_ERR_HIP, "tiles: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
    }
    t->opened = true;
    return SPT_OK;
}

int spt_tiles_unlink(spt_tiles *t)
{
    if (!t) return tiles_fail(t, SPT_ERR_ARG, "null tiles");
    if (t->owner && !t->name.empty()) {
        shm_unlink(t->name.c_str());
        t->name.clear();
    }
    return SPT_OK;
}

int spt_tiles_buffer(spt_tiles *t, uint64_t frame, void **d_buffer)
{
    if (!t || !d_buffer) return tiles_fail(t, SPT_ERR_ARG, "null tiles or output");
    if (!t->owner) return tiles_fail(t, SPT_ERR_STATE, "tiles: the gathered buffers are rank 0's");
    *d_buffer = t->buf + (size_t)(frame % t->nbuf) * t->world * t->tile_bytes;
    return SPT_OK;
}

int spt_tiles_send_range_async(spt_tiles *t, uint64_t frame, const void *d_src, uint64_t offset, uint64_t bytes,
                               void *stream)
{
    if (!t || (!d_src && bytes)) return tiles_fail(t, SPT_ERR_ARG, "null tiles or source");
    if (t->owner) return tiles_fail(t, SPT_ERR_STATE, "tiles: rank 0 renders into its slot (spt_tiles_buffer)");
    if (!t->buf) return tiles_fail(t, SPT_ERR_STATE, "tiles: not attached");
    const uint64_t cap = (uint64_t)t->world * t->tile_bytes;
    if (offset > cap || bytes > cap - offset) return tiles_fail(t, SPT_ERR_ARG, "tiles: range outside the buffer");
    spt_ctx *ctx = t->ctx;
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t b = (uint32_t)(frame % t->nbuf), gen = generation(t, frame);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    // the buffer's previous use (frame - nbuf) must be assembled before this copy lands
    if (gen > 1u) HIP_TRY(ctx, hipStreamWaitValue32(s, word(t, 0, b), gen - 1u, hipStreamWaitValueGte, 0xFFFFFFFFu));
    if (bytes) {
        uint8_t *dst = t->buf + (size_t)b * cap + offset;
        HIP_TRY(ctx, hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToDevice, s));
    }
    HIP_TRY(ctx, hipStreamWriteValue32(s, word(t, t->rank, b), gen, 0));
    return SPT_OK;
}

int spt_tiles_send_async(spt_tiles *t, uint64_t frame, const void *d_tile, void *stream)
{
    if (!t || !d_tile) return tiles_fail(t, SPT_ERR_ARG, "null tiles or tile");
    return spt_tiles_send_range_async(t, frame, d_tile, (uint64_t)t->rank * t->tile_bytes, t->tile_bytes, stream);
}

int spt_tiles_recv_async(spt_tiles *t, uint64_t frame, void *stream)
{
    if (!t) return tiles_fail(t, SPT_ERR_ARG, "null tiles");
    if (!t->owner) return tiles_fail(t, SPT_ERR_STATE, "tiles: rank 0 receives");
    spt_ctx *ctx = t->ctx;
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t b = (uint32_t)(frame % t->nbuf), gen = generation(t, frame);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (uint32_t r = 1; r < t->world; ++r)
        HIP_TRY(ctx, hipStreamWaitValue32(s, word(t, r, b), gen, hipStreamWaitValueGte, 0xFFFFFFFFu));
    return SPT_OK;
}

int spt_tiles_release_async(spt_tiles *t, uint64_t frame, void *stream)
{
    if (!t) return tiles_fail(t, SPT_ERR_ARG, "null tiles");
    if (!t->owner) return tiles_fail(t, SPT_ERR_STATE, "tiles: rank 0 releases");
    spt_ctx *ctx = t->ctx;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipStreamWriteValue32((hipStream_t)stream, word(t, 0, (uint32_t)(frame % t->nbuf)),
                                       generation(t, frame), 0));
    return SPT_OK;
}

int spt_tiles_abort(spt_tiles *t)
{
    if (!t) return tiles_fail(t, SPT_ERR_ARG, "null tiles");
    // every word to the largest generation, from the host: every wait packet of every rank
    // on this segment is satisfied, so no stream stays blocked on a transport given up
    if (t->host)
        for (size_t w = 0; w < t->host_bytes / kLine; ++w)
            __atomic_store_n((uint32_t *)((uint8_t *)t->host + w * kLine), 0xFFFFFFFFu, __ATOMIC_SEQ_CST);
    return SPT_OK;
}

void spt_tiles_destroy(spt_tiles *t)
{
    if (!t) return;
    if (t->ctx) (void)hipSetDevice(t->ctx->device);
    (void)hipDeviceSynchronize();  // no copy or wait packet may still use the words or buffers
    release(t);
    delete t;
}

}  // extern "C"
