/*
 * spt_oracle.h -- CPU restatement of SimplePathTracer's per-pixel render loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (simplepathtracer_amd/,
 * include/spt_hip.h) includes, links or calls this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, as the
 * checker / CPU timing baseline.
 *
 * PARITY STATUS: the reference (/root/reference, header-only MSVC C++) cannot be
 * built in this image without stand-ins for headers it lacks (<intrin.h>,
 * glbinding/GLFW via Gl.hpp, stb via IOHelpers.hpp), so it is "unbuildable here"
 * and there is no oracle/_ref.  The reference ships no tests or golden vectors.
 * End-to-end pixel values are therefore PARITY UNPINNED against the reference
 * itself.  What IS pinned (tests/test_oracle_kat.py, oracle/kat_*.c*):
 *   - uniform draws vs the real libstdc++ std::uniform_real_distribution<float>
 *     driven by the reference's splitmix mixer (Random.hpp:30-36, 86-93);
 *   - Vec4 arithmetic (Dot/LengthSquared/Normalize/Reflect/Mat4*Vec4) vs the real
 *     SSE4.1 intrinsics the reference uses (Math.hpp:107-187);
 *   - glibc pow/sqrt in double precision as used by SampleColorRefractive.
 * Semantics follow SURVEY.md §8(a): fp32 everywhere, no FMA contraction, IEEE
 * division and sqrt, libstdc++/glibc double promotion of pow()/sqrt() in the
 * refraction branch.  Build with -ffp-contract=off and without -ffast-math.
 *
 * RNG seam (SURVEY.md §8c seam (b)): the reference draws from a time-seeded
 * thread_local splitmix (Random.hpp:86-93).  Here every (pixel, sample) owns a
 * keyed splitmix stream: state0 = fmix64(fmix64(seed) ^ (pixel << 32 | sample)),
 * pixel = y * width + x.  Draw n mixes state0 + (n+1)*0x9E3779B97F4A7C15 with the
 * reference mixer, so results are independent of tiling and thread scheduling.
 */
#ifndef SPT_ORACLE_H
#define SPT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Material enum, Definitions.hpp:7-13 */
enum { SPO_SKYBOX = 0, SPO_REFLECTIVE = 1, SPO_REFRACTIVE = 2, SPO_DIFFUSE = 3 };

/* Paths with more specular events than this are cut (color 0).  The reference
 * recurses without bound (SingleThreadPathTracer.hpp:45,63-91) and would overflow
 * its stack long before; the GPU path uses the same cap. */
#define SPO_SPECULAR_CAP 1024u
/* RenderSegmentTask's pass cap, TaskBasedPathTracer.hpp:81 (pass < 10). */
#define SPO_TASK_PASSES 10u

/* Scene SoA, Globals.hpp:31-37 (g_spheres, g_radii, g_colors, g_materials,
 * g_diffuses, g_sphereNumber).  centers/colors are float4 per sphere; the w lane
 * is treated as 0 as in the reference's Vec4{x,y,z} initialisers. */
typedef struct spo_scene {
    uint32_t n;
    const float *centers;
    const float *radii;
    const float *colors;
    const uint8_t *materials;
    const float *fuzz;
} spo_scene;

/* Camera + compile-time config, Globals.hpp:8-29. view is viewMatrix (row-major,
 * already transposed as in Renderer.hpp:321). */
typedef struct spo_frame {
    float view[16];
    float eye[4];
    float sky[4];
    uint32_t width, height, spp, bounces;
    uint64_t seed;
} spo_frame;

/* ---- RNG (Random.hpp) ---- */
uint32_t spo_next_u32(uint64_t *state);
float spo_uniform(uint64_t *state, float a, float b);
float spo_uniform_u32(uint32_t bits, float a, float b);
uint64_t spo_sample_key(uint64_t seed, uint32_t pixel, uint32_t sample);
uint64_t spo_scene_state(uint32_t seed);
void spo_ball_vector(uint64_t *state, float out[4]);
void spo_unit_vector(uint64_t *state, float out[4]);

/* ---- math / geometry (Math.hpp, Collision.hpp) ---- */
float spo_dot(const float a[4], const float b[4]);
float spo_length_squared(const float a[4]);
void spo_normalize(const float a[4], float out[4]);
void spo_reflect(const float v[4], const float n[4], float out[4]);
void spo_matvec(const float m[16], const float v[4], float out[4]);
void spo_camera_basis(const float eye[4], const float look_at[4], const float up[4], float view_out[16]);
uint32_t spo_find_closest(const spo_scene *sc, const float d[4], const float o[4]);
void spo_write_pixel(const float c[4], uint8_t out[3]);

/* ---- render loop (SingleThreadPathTracer.hpp, TaskBasedPathTracer.hpp) ---- */
/* One (pixel, sample) path of RenderSegment: out[0..3] = color, returns number
 * of FindClosest calls.  task_mode: apply RenderSegmentTask's pass cap; out[3]
 * becomes 1.0 if the sample is counted, 0.0 if dropped. */
void spo_primary_winners(const spo_scene *sc, const spo_frame *fr, const uint32_t *xys, uint32_t n, uint32_t *winner);
uint32_t spo_trace_sample(const spo_scene *sc, const spo_frame *fr, uint32_t x, uint32_t y,
                          uint32_t s, int task_mode, float out[4]);
/* RenderSegment over [yB,yE)x[xB,xE).  rgba: region-local float4 per pixel
 * (row-major), rgb8: full-frame g_data in the reference index layout.  Either may
 * be NULL. Returns total FindClosest calls. */
uint64_t spo_render_segment(const spo_scene *sc, const spo_frame *fr, uint32_t yB, uint32_t yE,
                            uint32_t xB, uint32_t xE, float *rgba, uint8_t *rgb8);
/* RenderSegmentTask, faithful breadth-first restatement including its material
 * queues, its 10-pass cap and its colorIndex stride (correct for square tiles). */
uint64_t spo_render_segment_task(const spo_scene *sc, const spo_frame *fr, uint32_t yB, uint32_t yE,
                                 uint32_t xB, uint32_t xE, float *rgba, uint8_t *rgb8);
/* RenderImageParallelMain tiling (Renderer.hpp:257-302) with thread_count tiles
 * per side and at most thread_count tiles in flight.  mode 0 = RenderSegment,
 * 1 = RenderSegmentTask.  rgba is a full-frame float4 buffer (may be NULL). */
int spo_render_image_parallel(const spo_scene *sc, const spo_frame *fr, uint32_t thread_count,
                              int mode, float *rgba, uint8_t *rgb8);

/* ---- scene generators (SceneGenerators.hpp), sequential splitmix(seed) ---- */
uint32_t spo_generate_spheres(uint32_t seed, uint32_t cap, float *centers, float *radii,
                              float *colors, uint8_t *materials, float *fuzz);
uint32_t spo_init_spheres(uint32_t seed, float *centers, float *radii, float *colors,
                          uint8_t *materials, float *fuzz);

#ifdef __cplusplus
}
#endif
#endif
