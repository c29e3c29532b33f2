// RenderSegmentShim.hpp -- the reference's two render entry points rebuilt on the
// MI355X C ABI (spt_hip.h).  Include it in the reference's translation unit in
// place of SingleThreadPathTracer.hpp / TaskBasedPathTracer.hpp (or put
// include/dropin first on the include path, which does exactly that) and link
// libspt_hip.so.  Renderer.hpp, Main.cpp and the GL preview compile unchanged.
//
// Replaces:
//   void RenderSegment(RenderSegmentData)       SingleThreadPathTracer.hpp:114-137
//   void RenderSegmentTask(RenderSegmentData)   TaskBasedPathTracer.hpp:54-206
// Reads the same globals (Globals.hpp:12-37: g_width, g_height, g_samples,
// g_bounces, viewMatrix, eyePos, initColor, g_spheres, g_radii, g_colors,
// g_materials, g_diffuses, g_sphereNumber) and writes the same g_data bytes
// (IOHelpers.hpp:17-22).  The reference has no error channel, so a failure is
// reported on stderr and aborts.  Sampling uses the keyed per-(pixel, sample)
// stream seeded with spt_shim::seed (default 1; SPT_SEED overrides) instead of
// the clock-seeded thread_local splitmix (Random.hpp:86-93).  Concurrent RenderJob
// threads are rendered together (the library batches their tiles into shared
// launches, and writes into the page-locked g_data in place);
// SPT_DEVICES=0,1,... spreads them over several devices.
#pragma once

#include <spt_hip.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace spt_shim {

inline uint64_t seed = std::getenv("SPT_SEED") ? std::strtoull(std::getenv("SPT_SEED"), nullptr, 0) : 1ull;

inline void check(spt_ctx *ctx, int rc, const char *what)
{
    if (rc != SPT_OK) {
        std::fprintf(stderr, "spt: %s failed: %s\n", what, spt_last_error(ctx));
        std::abort();
    }
}

inline spt_ctx *context()
{
    // SPT_DEVICES=0,1,...: a multi-device context (each RenderJob tile goes to the
    // least busy device); else SPT_DEVICE (default 0)
    static spt_ctx *ctx = [] {
        spt_ctx *c = nullptr;
        if (const char *list = std::getenv("SPT_DEVICES")) {
            // a comma-separated list of ordinals; anything else aborts (a typo must not
            // turn into extra members on device 0)
            std::vector<int> devs;
            for (const char *p = list;;) {
                char *end = nullptr;
                const long d = std::strtol(p, &end, 10);
                if (end == p || (*end != ',' && *end != '\0') || d < 0) {
                    std::fprintf(stderr, "spt: malformed SPT_DEVICES=\"%s\" (want e.g. 0,1,2)\n", list);
                    std::abort();
                }
                devs.push_back((int)d);
                if (*end == '\0') break;
                p = end + 1;
            }
            check(nullptr, spt_ctx_create_multi(devs.data(), (uint32_t)devs.size(), &c), "spt_ctx_create_multi");
        } else {
            const char *dev = std::getenv("SPT_DEVICE");
            check(nullptr, spt_ctx_create(dev ? std::atoi(dev) : 0, &c), "spt_ctx_create");
        }
        // SPT_SERVICE=1: RenderJob tiles are jobs of the resident render service (else one
        // launch per batch of tiles); its session idles out by itself between frames
        const char *svc = std::getenv("SPT_SERVICE");
        if (svc && std::atoi(svc) != 0) check(c, spt_service_start(c), "spt_service_start");
        // the batch and read-ahead streams, created with the context so that the first
        // frame does not pay for them
        check(c, spt_prepare_dropin(c), "spt_prepare_dropin");
        return c;
    }();
    return ctx;
}

// Push the reference globals to the device when they changed since the last call.  Every
// RenderSegment call checks (1 024 calls per frame at tc = 32, each on a thread of its
// own): the globals are flattened into one thread-local key outside the lock and compared
// with the last pushed one under it.
inline void sync_globals()
{
    static std::mutex mu;
    static std::vector<float> last;
    thread_local std::vector<float> key;
    const uint32_t n = g_sphereNumber;
    key.clear();
    key.reserve(11 * (size_t)n + 29);
    for (uint32_t i = 0; i < n; ++i) key.insert(key.end(), g_spheres[i].xyzw, g_spheres[i].xyzw + 4);
    for (uint32_t i = 0; i < n; ++i) key.insert(key.end(), g_colors[i].xyzw, g_colors[i].xyzw + 4);
    for (uint32_t i = 0; i < n; ++i) key.push_back(g_radii[i]);
    for (uint32_t i = 0; i < n; ++i) key.push_back(g_diffuses[i]);
    for (uint32_t i = 0; i < n; ++i) key.push_back((float)static_cast<uint8_t>(g_materials[i]));
    key.insert(key.end(), viewMatrix.array, viewMatrix.array + 16);
    key.insert(key.end(), eyePos.xyzw, eyePos.xyzw + 4);
    key.insert(key.end(), initColor.xyzw, initColor.xyzw + 4);
    key.push_back((float)g_width);
    key.push_back((float)g_height);
    key.push_back((float)g_samples);
    key.push_back((float)g_bounces);
    key.push_back((float)(seed & 0xFFFFFF));
    std::lock_guard<std::mutex> lk(mu);
    if (key.size() == last.size() && std::memcmp(key.data(), last.data(), key.size() * sizeof(float)) == 0) return;
    const float *k = key.data();
    std::vector<float> centers(k, k + 4 * (size_t)n), colors(k + 4 * (size_t)n, k + 8 * (size_t)n),
        radii(k + 8 * (size_t)n, k + 9 * (size_t)n), fuzz(k + 9 * (size_t)n, k + 10 * (size_t)n);
    std::vector<uint8_t> mats(n);
    for (uint32_t i = 0; i < n; ++i) mats[i] = static_cast<uint8_t>(g_materials[i]);
    const float *view = k + 11 * (size_t)n, *eye = view + 16, *sky = eye + 4;
    spt_ctx *ctx = context();
    check(ctx, spt_set_scene(ctx, centers.data(), radii.data(), colors.data(), mats.data(), fuzz.data(), n),
          "spt_set_scene");
    check(ctx, spt_set_camera(ctx, view, eye, sky), "spt_set_camera");
    check(ctx, spt_set_params(ctx, g_width, g_height, g_samples, g_bounces, seed), "spt_set_params");
    last = key;
    // page-lock g_data once (best effort; SPT_PIN=0 leaves it pageable): batched calls
    // then write their tiles' bytes into it in place (no copy-back)
    static const void *pinned = nullptr;
    static const bool pin = !std::getenv("SPT_PIN") || std::atoi(std::getenv("SPT_PIN")) != 0;
    if (pin && g_data && pinned != g_data && spt_pin_host(ctx, g_data, (size_t)g_width * g_height * 3) == SPT_OK)
        pinned = g_data;
}

}  // namespace spt_shim

// SingleThreadPathTracer.hpp:114-137
inline void RenderSegment(RenderSegmentData segment)
{
    spt_shim::sync_globals();
    spt_ctx *ctx = spt_shim::context();
    spt_shim::check(ctx,
                    spt_render_segment(ctx, segment.yBegin, segment.yEnd, segment.xBegin, segment.xEnd, nullptr, g_data),
                    "spt_render_segment");
}

// TaskBasedPathTracer.hpp:54-206 (non-square tiles alias pixels as the reference does)
inline void RenderSegmentTask(RenderSegmentData segment)
{
    spt_shim::sync_globals();
    spt_ctx *ctx = spt_shim::context();
    spt_shim::check(ctx,
                    spt_render_segment_task(ctx, segment.yBegin, segment.yEnd, segment.xBegin, segment.xEnd, nullptr,
                                            g_data),
                    "spt_render_segment_task");
}
