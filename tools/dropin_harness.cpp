// Harness of the C++ drop-in (include/spt/RenderSegmentShim.hpp), for the parity
// tests and for `bench.py --dropin`.  It declares globals with the names and types of
// the reference's Globals.hpp / Definitions.hpp / Math.hpp (as the reference's own
// translation unit would), includes the shim, and drives RenderSegment /
// RenderSegmentTask from concurrent threads the way RenderImageParallelMain does
// (Renderer.hpp:257-302: tc x tc tiles, at most tc RenderJob threads in flight).
// Writes g_data to argv[1].
// Usage: dropin_harness out.bin width height spp bounces threads task(0|1) [frames]
//   frames > 0: render one untimed frame, then `frames` timed frames, and print
//   "frames=K seconds=T" (wall clock of the K frames).  SPT_DEVICES=0,1,.. (shim)
//   renders on a multi-device context.
//   SPT_HARNESS_COLD=1: the reference app's own pattern -- MainLoop renders exactly one
//   frame per process (Renderer.hpp:335-344) -- timed in its parts and printed as
//   "cold ctx_ms=.. setup_ms=.. frame_ms=..": context creation (HIP runtime and device
//   init, the library's buffers), the globals' upload (scene, traversal tables, primary-ray
//   lists, g_data page-locking), and the first RenderImageParallelMain frame itself.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace math {
struct Vec4 { float xyzw[4]; };
struct Mat4 { float array[16]; };
}  // namespace math
enum class Material : uint8_t { SKYBOX, REFLECTIVE, REFRACTIVE, DIFFUSE };
struct RenderSegmentData { uint32_t yBegin = 0, yEnd = 0, xBegin = 0, xEnd = 0; };

uint32_t g_width, g_height, g_samples, g_bounces;
uint8_t *g_data;
math::Mat4 viewMatrix;
math::Vec4 eyePos = {{0, 1, -3, 0}}, lookAt = {{0, 1, 0, 0}}, upDir = {{0, 1, 0, 0}}, initColor = {{137, 207, 240, 0}};
std::vector<math::Vec4> g_colors, g_spheres;
std::vector<float> g_radii, g_diffuses;
std::vector<Material> g_materials;
uint32_t g_sphereNumber = 10;

#include <spt/RenderSegmentShim.hpp>

int main(int argc, char **argv)
{
    if (argc < 8) return 2;
    g_width = atoi(argv[2]);
    g_height = atoi(argv[3]);
    g_samples = atoi(argv[4]);
    g_bounces = atoi(argv[5]);
    const uint32_t tc = atoi(argv[6]);
    const bool task = atoi(argv[7]) != 0;
    std::vector<uint8_t> frame((size_t)g_width * g_height * 3, 0);
    g_data = frame.data();
    // GenerateSpheres (SceneGenerators.hpp:6-66) through the library's producer
    std::vector<float> c(4 * 4096), r(4096), col(4 * 4096), fz(4096);
    std::vector<uint8_t> m(4096);
    uint32_t n = 0;
    if (spt_scene_generate_random(1, 4096, c.data(), r.data(), col.data(), m.data(), fz.data(), &n)) return 3;
    g_sphereNumber = n;
    for (uint32_t i = 0; i < n; ++i) {
        g_spheres.push_back({{c[4 * i], c[4 * i + 1], c[4 * i + 2], 0}});
        g_colors.push_back({{col[4 * i], col[4 * i + 1], col[4 * i + 2], 0}});
        g_radii.push_back(r[i]);
        g_diffuses.push_back(fz[i]);
        g_materials.push_back(static_cast<Material>(m[i]));
    }
    if (spt_camera_basis(eyePos.xyzw, lookAt.xyzw, upDir.xyzw, viewMatrix.array)) return 4;
    // SPT_HARNESS_NOOP=1: the same threads and tiles with RenderJob doing nothing -- the
    // calling pattern's own cost (thread spawn, condition variable, join) per frame, the
    // ceiling any RenderSegment implementation can reach under it
    const bool noop = std::getenv("SPT_HARNESS_NOOP") && std::atoi(std::getenv("SPT_HARNESS_NOOP")) != 0;
    // RenderImageParallelMain (Renderer.hpp:257-302) as written: per tile a thread running
    // RenderJob (242-255: it takes a free slot when it starts and returns it when its tile
    // is done, then notifies) is spawned and detached, and the main thread waits for a free
    // slot before the next; at the end it waits until all tc slots are free.  Two changes
    // keep the harness itself defined: the count, condition variable and mutex of a frame
    // outlive it (the reference's are locals while detached threads may still notify them:
    // here each frame's live in a block its threads share), and the slot is returned under
    // the mutex (the reference's unlocked fetch_add + notify can be lost and leave the final
    // wait asleep).  As in the reference, a thread takes its slot only when it starts, so the
    // final wait can end while a spawned thread has not started yet: that thread then works
    // on its own frame's count (one count shared by all frames and reset per frame drifted
    // when such a thread straddled the reset, and a later frame's final wait never ended).
    // `alive` lets main return only after every detached thread has finished.
    // SPT_HARNESS_COLD=2 also prints every tile's RenderJob span (ms from the frame's start)
    struct FrameSync {
        std::atomic<int> free_threads{0};
        std::condition_variable cv;
        std::mutex mu;
    };
    static std::vector<std::pair<double, double>> spans((size_t)tc * tc);
    static std::chrono::steady_clock::time_point frame_t0;
    static std::atomic<int> alive{0};
    static std::mutex spans_mu;
    auto frame_once = [&]() {
        const uint32_t sw = g_width / tc, sh = g_height / tc;
        auto fs = std::make_shared<FrameSync>();
        fs->free_threads = (int)tc;
        frame_t0 = std::chrono::steady_clock::now();
        std::unique_lock<std::mutex> lk(fs->mu);
        for (uint32_t j = 0; j < tc; ++j)
            for (uint32_t i = 0; i < tc; ++i) {
                RenderSegmentData seg{sh * j, sh * j + sh > g_height ? g_height : sh * j + sh, sw * i,
                                      sw * i + sw > g_width ? g_width : sw * i + sw};
                alive.fetch_add(1);
                const size_t k = (size_t)j * tc + i;
                const auto t_frame = frame_t0;
                std::thread thread([seg, task, noop, k, fs, t_frame] {
                    fs->free_threads.fetch_sub(1);
                    const auto ts = std::chrono::steady_clock::now();
                    if (noop) {
                    } else if (task) {
                        RenderSegmentTask(seg);
                    } else {
                        RenderSegment(seg);
                    }
                    {
                        std::lock_guard<std::mutex> g(fs->mu);
                        const auto te = std::chrono::steady_clock::now();
                        {
                            std::lock_guard<std::mutex> gs(spans_mu);
                            spans[k] = {std::chrono::duration<double, std::milli>(ts - t_frame).count(),
                                        std::chrono::duration<double, std::milli>(te - t_frame).count()};
                        }
                        fs->free_threads.fetch_add(1);
                    }
                    fs->cv.notify_one();
                    alive.fetch_sub(1);
                });
                thread.detach();
                fs->cv.wait(lk, [&] { return fs->free_threads.load() > 0; });
            }
        fs->cv.wait(lk, [&] { return fs->free_threads.load() == (int)tc; });
    };
    const bool cold = std::getenv("SPT_HARNESS_COLD") && std::atoi(std::getenv("SPT_HARNESS_COLD")) != 0;
    if (cold && !noop) {
        using clk = std::chrono::steady_clock;
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        const auto t0 = clk::now();
        spt_shim::context();
        const auto t1 = clk::now();
        spt_shim::sync_globals();
        const auto t2 = clk::now();
        frame_once();
        const auto t3 = clk::now();
        spt_stats st{};
        spt_get_stats(spt_shim::context(), &st);
        if (std::atoi(std::getenv("SPT_HARNESS_COLD")) == 2)
            for (size_t k = 0; k < spans.size(); ++k) printf("tile %zu: %.3f .. %.3f ms\n", k, spans[k].first, spans[k].second);
        printf("cold ctx_ms=%.3f setup_ms=%.3f frame_ms=%.3f accel_ms=%.3f prim_ms=%.3f batches=%llu calls=%llu\n",
               ms(t0, t1), ms(t1, t2), ms(t2, t3), st.accel_build_ms, st.prim_list_build_ms,
               (unsigned long long)st.batches, (unsigned long long)st.batched_calls);
    } else {
        frame_once();
    }
    const int frames = argc > 8 ? atoi(argv[8]) : 0;
    if (frames > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < frames; ++k) frame_once();
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        spt_stats st{};
        if (!noop) spt_get_stats(spt_shim::context(), &st);  // since the context's creation (no reset)
        printf("frames=%d seconds=%.6f calls=%llu batches=%llu render_ms=%.3f busy_ms=%.3f fold_ms=%.3f "
               "svc_sessions=%llu svc_jobs=%llu svc_watchdog_exits=%llu svc_kernel_ms=%.3f\n",
               frames, sec, (unsigned long long)st.batched_calls, (unsigned long long)st.batches, st.render_ms,
               st.render_busy_ms, st.fold_ms, (unsigned long long)st.svc_sessions, (unsigned long long)st.svc_jobs,
               (unsigned long long)st.svc_watchdog_exits, st.svc_kernel_ms);
    }
    while (alive.load() != 0) std::this_thread::yield();
    FILE *f = fopen(argv[1], "wb");
    if (!f) return 5;
    fwrite(frame.data(), 1, frame.size(), f);
    fclose(f);
    return 0;
}
