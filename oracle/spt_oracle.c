/*
 * spt_oracle.c -- CPU restatement of SimplePathTracer's render loop.
 *
 * TEST INFRASTRUCTURE ONLY (see spt_oracle.h for the parity status and the
 * rules on who may load this).  Every function cites the reference file:line it
 * restates; line numbers are into /root/reference/include/.
 *
 * Vec4 is kept as four IEEE fp32 lanes with the exact SSE4.1 semantics of
 * Math.hpp: _mm_dp_ps(...,0xF1) sums (x*x'+y*y')+(z*z'+w*w'); two _mm_hadd_ps
 * give the same order; _mm_sqrt_ps/_mm_div_ps are correctly rounded.
 * Build: -O2 -ffp-contract=off (no FMA contraction), no -ffast-math.
 */
#include "spt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct v4 { float x, y, z, w; } v4;

static inline v4 V3(float x, float y, float z) { v4 r = {x, y, z, 0.0f}; return r; }
static inline v4 ld4(const float *p) { v4 r = {p[0], p[1], p[2], 0.0f}; return r; }
static inline void st4(float *p, v4 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; p[3] = a.w; }

/* Math.hpp:33-48 (operator+, _mm_add_ps; IEEE add is commutative bitwise) */
static inline v4 vadd(v4 a, v4 b) { v4 r = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; return r; }
/* Math.hpp:16-31 (operator-, a - b) */
static inline v4 vsub(v4 a, v4 b) { v4 r = {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; return r; }
/* Math.hpp:50-64 (operator*(float)) */
static inline v4 vmul(v4 a, float s) { v4 r = {a.x * s, a.y * s, a.z * s, a.w * s}; return r; }
/* Math.hpp:66-80 (unary minus: xor with -0.0 == IEEE negation) */
static inline v4 vneg(v4 a) { v4 r = {-a.x, -a.y, -a.z, -a.w}; return r; }
/* Math.hpp:107-111: _mm_dp_ps(a, b, 0xF1) */
static inline float vdot(v4 a, v4 b) { return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w); }
/* Math.hpp:122-133: mul, hadd, hadd */
static inline float vlensq(v4 a) { return (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w); }
/* Math.hpp:135-138 */
static inline float vlen(v4 a) { return sqrtf(vlensq(a)); }
/* Math.hpp:140-154: lane-wise v / sqrt(hadd(hadd(v*v))) */
static inline v4 vnorm(v4 a)
{
    float l = sqrtf(vlensq(a));
    v4 r = {a.x / l, a.y / l, a.z / l, a.w / l};
    return r;
}
/* Math.hpp:156-159: vec - normal * Dot(vec, normal) * 2.f */
static inline v4 vreflect(v4 v, v4 n) { return vsub(v, vmul(vmul(n, vdot(v, n)), 2.0f)); }
/* Math.hpp:113-120, including the z-component bug of the reference */
static inline v4 vcross(v4 a, v4 b)
{
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.x - a.y * b.x);
}
/* Math.hpp:178-186: four dpps, one per row */
static inline v4 vmatvec(const float *m, v4 v)
{
    v4 r;
    r.x = (m[0] * v.x + m[1] * v.y) + (m[2] * v.z + m[3] * v.w);
    r.y = (m[4] * v.x + m[5] * v.y) + (m[6] * v.z + m[7] * v.w);
    r.z = (m[8] * v.x + m[9] * v.y) + (m[10] * v.z + m[11] * v.w);
    r.w = (m[12] * v.x + m[13] * v.y) + (m[14] * v.z + m[15] * v.w);
    return r;
}

/* ------------------------------------------------------------------------- */
/* RNG                                                                        */
/* ------------------------------------------------------------------------- */
#define SPO_GAMMA 0x9E3779B97F4A7C15ULL

/* Random.hpp:30-36, splitmix::operator() */
uint32_t spo_next_u32(uint64_t *state)
{
    uint64_t z = (*state += SPO_GAMMA);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return (uint32_t)((z ^ (z >> 31)) >> 31);
}

/* Random.hpp:86-93 -> std::uniform_real_distribution<float>::operator()
 * (libstdc++ bits/random.h:1870) -> generate_canonical<float,24>
 * (bits/random.tcc:3348-3380): one 32-bit draw, float(u)/2^32, clamp >=1 to
 * nextafter(1,0); then u*(b-a)+a. */
float spo_uniform_u32(uint32_t bits, float a, float b)
{
    float u = (float)bits / 4294967296.0f;
    if (u >= 1.0f) u = nextafterf(1.0f, 0.0f);
    return u * (b - a) + a;
}

float spo_uniform(uint64_t *state, float a, float b) { return spo_uniform_u32(spo_next_u32(state), a, b); }

static uint64_t fmix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* Keyed per-(pixel, sample) stream, SURVEY.md §8c item 5. */
uint64_t spo_sample_key(uint64_t seed, uint32_t pixel, uint32_t sample)
{
    return fmix64(fmix64(seed) ^ (((uint64_t)pixel << 32) | (uint64_t)sample));
}

/* Random.hpp:19 splitmix(uint64_t seed): m_seed(seed << 31 | seed); the reference
 * feeds static_cast<unsigned int>(clock) (Random.hpp:88-89). */
uint64_t spo_scene_state(uint32_t seed)
{
    uint64_t s = (uint64_t)seed;
    return (s << 31) | s;
}

/* Random.hpp:115-127 GenerateUniformDistInsideSphereVector(0.5f) (identical to
 * GenerateNormalDistInsideSphereVector, 129-141): x, y, z drawn in that order,
 * repeated while Length < radius -> samples the cube minus the ball. */
static v4 ball_vector(uint64_t *st)
{
    const float radius = 0.5f;
    v4 r;
    do {
        float x = spo_uniform(st, -radius, radius);
        float y = spo_uniform(st, -radius, radius);
        float z = spo_uniform(st, -radius, radius);
        r = V3(x, y, z);
    } while (vlen(r) < radius);
    return r;
}

void spo_ball_vector(uint64_t *state, float out[4]) { st4(out, ball_vector(state)); }

/* Random.hpp:95-113 GenerateUnitVector<3>: x, y, z from U(-1,1), Normalize. */
static v4 unit_vector(uint64_t *st)
{
    float x = spo_uniform(st, -1.0f, 1.0f);
    float y = spo_uniform(st, -1.0f, 1.0f);
    float z = spo_uniform(st, -1.0f, 1.0f);
    return vnorm(V3(x, y, z));
}

void spo_unit_vector(uint64_t *state, float out[4]) { st4(out, unit_vector(state)); }

/* ------------------------------------------------------------------------- */
/* Math wrappers for the KAT tests                                            */
/* ------------------------------------------------------------------------- */
static v4 ld4w(const float *p) { v4 r = {p[0], p[1], p[2], p[3]}; return r; }
float spo_dot(const float a[4], const float b[4]) { return vdot(ld4w(a), ld4w(b)); }
float spo_length_squared(const float a[4]) { return vlensq(ld4w(a)); }
void spo_normalize(const float a[4], float out[4]) { st4(out, vnorm(ld4w(a))); }
void spo_reflect(const float v[4], const float n[4], float out[4]) { st4(out, vreflect(ld4w(v), ld4w(n))); }
void spo_matvec(const float m[16], const float v[4], float out[4]) { st4(out, vmatvec(m, ld4w(v))); }

/* Math.hpp:198-209 CreateCameraBasisMatrix + Math.hpp:211-231 Transpose
 * (Renderer.hpp:321). Rows of the basis: right, up, viewDir, 0. */
void spo_camera_basis(const float eye[4], const float look_at[4], const float up[4], float view_out[16])
{
    v4 e = ld4(eye), l = ld4(look_at), u = ld4(up);
    v4 view = vnorm(vsub(l, e));
    v4 right = vnorm(vcross(u, view));
    v4 up2 = vcross(view, right);
    float b[16] = {right.x, right.y, right.z, right.w, up2.x, up2.y, up2.z, up2.w,
                   view.x,  view.y,  view.z,  view.w,  0.0f,  0.0f,  0.0f,  0.0f};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) view_out[i * 4 + j] = b[j * 4 + i];
}

/* ------------------------------------------------------------------------- */
/* Collision.hpp                                                              */
/* ------------------------------------------------------------------------- */
static inline v4 center(const spo_scene *sc, uint32_t i) { return ld4(sc->centers + 4 * (size_t)i); }

/* Collision.hpp:9-17 RaySphereIntersection, threshold 1e-3f */
static inline int ray_sphere(v4 c, float r, v4 d, v4 o)
{
    c = vsub(c, o);
    float tc = vdot(c, d);
    float d2 = vdot(c, c) - tc * tc;
    return (tc > 1e-3f) && (r * r - d2 > 1e-3f);
}

/* Collision.hpp:19-27 / 29-37 */
static inline float min_factor(v4 rs, float r, v4 d)
{
    float tc = vdot(rs, d);
    float d2 = vdot(rs, rs) - tc * tc;
    float td = sqrtf(r * r - d2);
    return tc - td;
}
static inline float max_factor(v4 rs, float r, v4 d)
{
    float tc = vdot(rs, d);
    float d2 = vdot(rs, rs) - tc * tc;
    float td = sqrtf(r * r - d2);
    return tc + td;
}
/* Collision.hpp:49-56 / 58-65: rayOrigin + rayDirection * t */
static inline v4 closest_contact(v4 c, float r, v4 o, v4 d) { return vadd(o, vmul(d, min_factor(vsub(c, o), r, d))); }
static inline v4 farthest_contact(v4 c, float r, v4 o, v4 d) { return vadd(o, vmul(d, max_factor(vsub(c, o), r, d))); }
/* Collision.hpp:67-71 */
static inline v4 contact_normal(v4 p, v4 c) { return vnorm(vsub(p, c)); }

/* Collision.hpp:87-109 FindClosestIntersectionSphere.  The reference index is
 * uint8_t (hangs for n > 255); this restatement uses uint32 and is identical for
 * n <= 255.  Strict '>' update: the lowest index wins ties. */
static uint32_t find_closest(const spo_scene *sc, v4 d, v4 o)
{
    uint32_t min_index = sc->n;
    float min_d = FLT_MAX;
    for (uint32_t i = 0; i < sc->n; ++i) {
        v4 c = center(sc, i);
        float r = sc->radii[i];
        if (ray_sphere(c, r, d, o)) {
            v4 p = closest_contact(c, r, o, d);
            if (vdot(o, d) < vdot(p, d)) {
                float ds = vlensq(vsub(o, p));
                min_index = min_d > ds ? i : min_index;
                min_d = min_d > ds ? ds : min_d;
            }
        }
    }
    return min_index;
}

uint32_t spo_find_closest(const spo_scene *sc, const float d[4], const float o[4])
{
    return find_closest(sc, ld4w(d), ld4w(o));
}

/* IOHelpers.hpp:17-22 WritePixel: uint8(round(sqrt(c/255)*255)) per channel, no
 * clamp.  static_cast<uint8_t>(float) is emitted by gcc/clang on x86-64 as
 * cvttss2si (int32, INT_MIN for NaN/out of range) then the low byte. */
static inline uint8_t f2u8(float v)
{
    if (!(v > -2147483648.0f && v < 2147483648.0f)) return 0;
    return (uint8_t)(int32_t)v;
}
static inline void write_pixel(uint8_t *g, v4 c)
{
    g[0] = f2u8(roundf(sqrtf(c.x / 255.f) * 255.f));
    g[1] = f2u8(roundf(sqrtf(c.y / 255.f) * 255.f));
    g[2] = f2u8(roundf(sqrtf(c.z / 255.f) * 255.f));
}
void spo_write_pixel(const float c[4], uint8_t out[3]) { write_pixel(out, ld4w(c)); }

/* ------------------------------------------------------------------------- */
/* SingleThreadPathTracer.hpp (recursive)                                     */
/* ------------------------------------------------------------------------- */
typedef struct tctx {
    const spo_scene *sc;
    const spo_frame *fr;
    uint64_t st;
    uint32_t casts;
    uint32_t spec;
    int task_mode;
    int dropped;
} tctx;

static v4 trace(tctx *t, v4 d, v4 o, uint32_t bounce);

/* SingleThreadPathTracer.hpp:11-19 */
static inline v4 sky(const tctx *t, v4 d) { return vmul(vmul(ld4(t->fr->sky), d.y + 1.f), 0.5f); }

static inline uint32_t cast(tctx *t, v4 d, v4 o)
{
    t->casts++;
    return find_closest(t->sc, d, o);
}

/* SingleThreadPathTracer.hpp:21-37 */
static v4 sample_diffuse(tctx *t, v4 d, v4 o, uint32_t bounce, uint32_t idx)
{
    const spo_scene *sc = t->sc;
    v4 color = vmul(ld4(sc->colors + 4 * (size_t)idx), 0.5f);
    o = closest_contact(center(sc, idx), sc->radii[idx], o, d);
    d = vnorm(vadd(contact_normal(o, center(sc, idx)), ball_vector(&t->st)));
    idx = cast(t, d, o);
    while (--bounce && idx < sc->n) {
        color = vmul(color, 0.5f);
        o = closest_contact(center(sc, idx), sc->radii[idx], o, d);
        v4 n = contact_normal(o, center(sc, idx));
        d = vnorm(vadd(vadd(o, n), ball_vector(&t->st)));
        idx = cast(t, d, o);
    }
    return color;
}

/* returns nonzero if the path must stop (pass cap or specular cap) */
static int specular_event(tctx *t)
{
    t->spec++;
    if (t->task_mode && t->spec >= SPO_TASK_PASSES) { t->dropped = 1; return 1; }
    if (t->spec > SPO_SPECULAR_CAP) return 1;
    return 0;
}

/* SingleThreadPathTracer.hpp:39-46 */
static v4 sample_reflective(tctx *t, v4 d, v4 o, uint32_t bounce, uint32_t idx)
{
    const spo_scene *sc = t->sc;
    o = closest_contact(center(sc, idx), sc->radii[idx], o, d);
    v4 n = contact_normal(o, center(sc, idx));
    d = vnorm(vadd(vreflect(d, n), vmul(ball_vector(&t->st), sc->fuzz[idx])));
    if (specular_event(t)) return V3(0.f, 0.f, 0.f);
    return trace(t, d, o, bounce);
}

/* SingleThreadPathTracer.hpp:48-92.  pow()/sqrt() on float arguments bind to
 * std::pow(float,float) / std::sqrt(float) in the reference's translation unit:
 * IOHelpers.hpp:5-9 includes the stb implementations, whose <math.h>/<stdlib.h>
 * are libstdc++'s `using std::pow; using std::sqrt; using std::abs;` wrappers,
 * before Renderer.hpp:6-8 includes the tracers and the scene generator
 * (oracle/probe_overloads.cpp).  So Schlick, the total-internal-reflection test
 * and the Snell scalar are all float: glibc's powf (called here, as the
 * reference's __builtin_powf does) and the correctly rounded sqrtf. */
static inline float schlick_of(float rsq, float c)
{
    return rsq + (1.f - rsq) * powf(1.f - c, 5.f);
}
static inline int no_tir(float r, float c)
{
    return r * sqrtf(1.f - c * c) < 1.f;
}
static inline v4 refract_dir(v4 d, v4 n, float r, float c)
{
    float k = r * c - sqrtf(1.f - r * r * (1.f - c * c));
    return vnorm(vadd(vmul(d, r), vmul(n, k)));
}

static v4 sample_refractive(tctx *t, v4 d, v4 o, uint32_t bounce, uint32_t idx)
{
    const spo_scene *sc = t->sc;
    const float nAir = 1.0f, nGlass = 1.5f;
    v4 c0 = center(sc, idx);
    float rad = sc->radii[idx];

    o = closest_contact(c0, rad, o, d);
    v4 n = contact_normal(o, c0);
    float c = vdot(vneg(n), d);
    float r = nAir / nGlass;
    float rsq = powf((nAir - nGlass) / (nAir + nGlass), 2.f);
    float schlick = schlick_of(rsq, c);
    v4 nd;

    if (spo_uniform(&t->st, 0.f, 1.f) < schlick) {
        nd = vreflect(d, n);
    } else if (no_tir(r, c)) {
        d = refract_dir(d, n, r, c);
        o = farthest_contact(c0, rad, o, d);
        n = vneg(contact_normal(o, c0));
        c = vdot(vneg(n), d);
        r = nGlass / nAir;
        rsq = powf((nGlass - nAir) / (nGlass + nAir), 2.f);
        schlick = schlick_of(rsq, c);
        if (spo_uniform(&t->st, 0.f, 1.f) < schlick)
            nd = vreflect(d, n);
        else if (no_tir(r, c))
            nd = refract_dir(d, n, r, c);
        else
            nd = vreflect(d, n);
    } else {
        nd = vreflect(d, n);
    }
    if (specular_event(t)) return V3(0.f, 0.f, 0.f);
    return trace(t, nd, o, bounce);
}

/* SingleThreadPathTracer.hpp:94-112 */
static v4 trace(tctx *t, v4 d, v4 o, uint32_t bounce)
{
    uint32_t idx = cast(t, d, o);
    if (idx < t->sc->n) {
        switch (t->sc->materials[idx]) {
        case SPO_DIFFUSE: return sample_diffuse(t, d, o, bounce, idx);
        case SPO_REFLECTIVE: return sample_reflective(t, d, o, bounce, idx);
        case SPO_REFRACTIVE: return sample_refractive(t, d, o, bounce, idx);
        default: break;
        }
    }
    return sky(t, d);
}

/* SingleThreadPathTracer.hpp:125-128: primary ray of sample s of pixel (x, y).
 * Note the reference divides y by width and x by height. */
static inline v4 primary_dir(const spo_frame *fr, uint64_t *st, uint32_t x, uint32_t y)
{
    float u = ((float)y + spo_uniform(st, -1.f, 1.f)) / (float)fr->width;
    float v = ((float)x + spo_uniform(st, -1.f, 1.f)) / (float)fr->height;
    return vnorm(vmatvec(fr->view, V3(-1.f + 2.f * v, -1.f + 2.f * u, 1.f)));
}

/* The primary ray of sample s of pixel (x, y) (SingleThreadPathTracer.hpp:123-130) and its
 * closest sphere (Collision.hpp:87-109; sc->n = none), for n (x, y, s) triples: the
 * checker of the GPU's primary-ray candidate lists (tests/test_prim_lists.py). */
void spo_primary_winners(const spo_scene *sc, const spo_frame *fr, const uint32_t *xys, uint32_t n, uint32_t *winner)
{
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t x = xys[3 * i], y = xys[3 * i + 1], s = xys[3 * i + 2];
        uint64_t st = spo_sample_key(fr->seed, y * fr->width + x, s);
        v4 d = primary_dir(fr, &st, x, y);
        winner[i] = find_closest(sc, d, ld4(fr->eye));
    }
}

uint32_t spo_trace_sample(const spo_scene *sc, const spo_frame *fr, uint32_t x, uint32_t y, uint32_t s,
                          int task_mode, float out[4])
{
    tctx t = {sc, fr, spo_sample_key(fr->seed, y * fr->width + x, s), 0, 0, task_mode, 0};
    v4 d = primary_dir(fr, &t.st, x, y);
    v4 c = trace(&t, d, ld4(fr->eye), fr->bounces);
    if (task_mode) c.w = t.dropped ? 0.0f : 1.0f;
    st4(out, c);
    return t.casts;
}

/* Globals.hpp:14-18 / SingleThreadPathTracer.hpp:120: byte index of (x, y) */
static inline size_t g_index(const spo_frame *fr, uint32_t x, uint32_t y)
{
    uint32_t g_size = fr->width * fr->height * 3u;
    return (size_t)(g_size - ((fr->width - x) * 3u + y * fr->width * 3u));
}

/* SingleThreadPathTracer.hpp:114-137 RenderSegment */
uint64_t spo_render_segment(const spo_scene *sc, const spo_frame *fr, uint32_t yB, uint32_t yE, uint32_t xB,
                            uint32_t xE, float *rgba, uint8_t *rgb8)
{
    uint64_t casts = 0;
    v4 eye = ld4(fr->eye);
    for (uint32_t y = yB; y < yE; ++y) {
        for (uint32_t x = xB; x < xE; ++x) {
            v4 acc = {0.f, 0.f, 0.f, 0.f};
            for (uint32_t s = 0; s < fr->spp; ++s) {
                tctx t = {sc, fr, spo_sample_key(fr->seed, y * fr->width + x, s), 0, 0, 0, 0};
                v4 d = primary_dir(fr, &t.st, x, y);
                acc = vadd(acc, trace(&t, d, eye, fr->bounces));
                casts += t.casts;
            }
            acc = vmul(acc, 1.f / (float)fr->spp);
            if (rgba) st4(rgba + 4 * ((size_t)(y - yB) * (xE - xB) + (x - xB)), acc);
            if (rgb8) write_pixel(rgb8 + g_index(fr, x, y), acc);
        }
    }
    return casts;
}

/* ------------------------------------------------------------------------- */
/* TaskBasedPathTracer.hpp (breadth-first material queues)                    */
/* ------------------------------------------------------------------------- */
typedef struct task_t { /* Definitions.hpp:23-31 + the keyed stream state */
    v4 origin, direction;
    uint32_t sphere_index, bounce_count, x, y;
    uint64_t st;
} task_t;

typedef struct tqueue { task_t *v; size_t n, cap; } tqueue;
typedef struct tasks_t { tqueue diffuse, reflective, refractive, skybox; } tasks_t;

static void q_push(tqueue *q, task_t t)
{
    if (q->n == q->cap) {
        q->cap = q->cap ? q->cap * 2 : 256;
        q->v = (task_t *)realloc(q->v, q->cap * sizeof(task_t));
    }
    q->v[q->n++] = t;
}
/* TaskBasedPathTracer.hpp:40-46 / 32-38 / 48-52 */
static void clear_tasks(tasks_t *t) { t->diffuse.n = t->reflective.n = t->refractive.n = t->skybox.n = 0; }
static void swap_tasks(tasks_t *a, tasks_t *b) { tasks_t tmp = *a; *a = *b; *b = tmp; }
static size_t tasks_size(const tasks_t *t) { return t->diffuse.n + t->reflective.n + t->refractive.n + t->skybox.n; }
static void free_tasks(tasks_t *t) { free(t->diffuse.v); free(t->reflective.v); free(t->refractive.v); free(t->skybox.v); }

/* TaskBasedPathTracer.hpp:9-30 */
static void trace_task(const spo_scene *sc, task_t task, tasks_t *tasks, uint64_t *casts)
{
    (*casts)++;
    task.sphere_index = find_closest(sc, task.direction, task.origin);
    if (task.sphere_index < sc->n) {
        switch (sc->materials[task.sphere_index]) {
        case SPO_DIFFUSE: q_push(&tasks->diffuse, task); return;
        case SPO_REFLECTIVE: q_push(&tasks->reflective, task); return;
        case SPO_REFRACTIVE: q_push(&tasks->refractive, task); return;
        default: break;
        }
    }
    q_push(&tasks->skybox, task);
}

/* TaskBasedPathTracer.hpp:54-206 RenderSegmentTask. */
uint64_t spo_render_segment_task(const spo_scene *sc, const spo_frame *fr, uint32_t yB, uint32_t yE, uint32_t xB,
                                 uint32_t xE, float *rgba, uint8_t *rgb8)
{
    const uint32_t segW = xE - xB, segH = yE - yB;
    /* colorIndex (lines 103, 186) strides rows by segmentHeight; size the arrays so
     * that the aliasing of non-square tiles stays in bounds here. */
    size_t slots = (size_t)segW * segH;
    size_t need = (size_t)(segW ? segW - 1 : 0) + (size_t)(segH ? segH - 1 : 0) * segH + 1;
    size_t alloc = slots > need ? slots : need;
    v4 *colors = (v4 *)calloc(alloc ? alloc : 1, sizeof(v4));
    float *samples = (float *)calloc(alloc ? alloc : 1, sizeof(float));
    tasks_t tasks = {0}, next = {0};
    uint64_t casts = 0;
    v4 eye = ld4(fr->eye);
    const float nAir = 1.0f, nGlass = 1.5f;

    for (uint32_t s = 0; s < fr->spp; ++s) {
        clear_tasks(&tasks);
        clear_tasks(&tasks);
        /* primary pass, lines 68-79 */
        for (uint32_t y = yB; y < yE; ++y)
            for (uint32_t x = xB; x < xE; ++x) {
                task_t tk;
                tk.st = spo_sample_key(fr->seed, y * fr->width + x, s);
                tk.origin = eye;
                tk.direction = primary_dir(fr, &tk.st, x, y);
                tk.sphere_index = sc->n;
                tk.bounce_count = fr->bounces;
                tk.x = x;
                tk.y = y;
                trace_task(sc, tk, &tasks, &casts);
            }

        for (uint32_t pass = 0; pass < SPO_TASK_PASSES && tasks_size(&tasks) > 0; ++pass) {
            /* diffuse, lines 83-106 */
            for (size_t i = 0; i < tasks.diffuse.n; ++i) {
                task_t *tk = &tasks.diffuse.v[i];
                uint32_t idx = tk->sphere_index;
                v4 color = vmul(ld4(sc->colors + 4 * (size_t)idx), 0.5f);
                tk->origin = closest_contact(center(sc, idx), sc->radii[idx], tk->origin, tk->direction);
                tk->direction = vnorm(vadd(contact_normal(tk->origin, center(sc, idx)), ball_vector(&tk->st)));
                casts++;
                idx = find_closest(sc, tk->direction, tk->origin);
                while (--tk->bounce_count && idx < sc->n) {
                    color = vmul(color, 0.5f);
                    tk->origin = closest_contact(center(sc, idx), sc->radii[idx], tk->origin, tk->direction);
                    v4 n = contact_normal(tk->origin, center(sc, idx));
                    tk->direction = vnorm(vadd(vadd(tk->origin, n), ball_vector(&tk->st)));
                    casts++;
                    idx = find_closest(sc, tk->direction, tk->origin);
                }
                tk->sphere_index = idx;
                size_t ci = (size_t)(tk->x - xB) + (size_t)(tk->y - yB) * segH;
                colors[ci] = vadd(colors[ci], color);
                samples[ci] += 1.f;
            }
            /* reflective, lines 108-122 */
            for (size_t i = 0; i < tasks.reflective.n; ++i) {
                task_t *tk = &tasks.reflective.v[i];
                uint32_t idx = tk->sphere_index;
                tk->origin = closest_contact(center(sc, idx), sc->radii[idx], tk->origin, tk->direction);
                v4 n = contact_normal(tk->origin, center(sc, idx));
                tk->direction = vnorm(vadd(vreflect(tk->direction, n), vmul(ball_vector(&tk->st), sc->fuzz[idx])));
                casts++;
                idx = find_closest(sc, tk->direction, tk->origin);
                task_t nt = *tk;
                nt.sphere_index = idx;
                nt.bounce_count = fr->bounces;
                trace_task(sc, nt, &next, &casts);
            }
            /* refractive, lines 124-180 */
            for (size_t i = 0; i < tasks.refractive.n; ++i) {
                task_t *tk = &tasks.refractive.v[i];
                uint32_t idx = tk->sphere_index;
                v4 c0 = center(sc, idx);
                float rad = sc->radii[idx];
                tk->origin = closest_contact(c0, rad, tk->origin, tk->direction);
                v4 n = contact_normal(tk->origin, c0);
                float c = vdot(vneg(n), tk->direction);
                float r = nAir / nGlass;
                float rsq = powf((nAir - nGlass) / (nAir + nGlass), 2.f);
                float schlick = schlick_of(rsq, c);
                if (spo_uniform(&tk->st, 0.f, 1.f) < schlick) {
                    tk->direction = vreflect(tk->direction, n);
                } else if (no_tir(r, c)) {
                    tk->direction = refract_dir(tk->direction, n, r, c);
                    tk->origin = farthest_contact(c0, rad, tk->origin, tk->direction);
                    n = vneg(contact_normal(tk->origin, c0));
                    c = vdot(vneg(n), tk->direction);
                    r = nGlass / nAir;
                    rsq = powf((nGlass - nAir) / (nGlass + nAir), 2.f);
                    schlick = schlick_of(rsq, c);
                    if (spo_uniform(&tk->st, 0.f, 1.f) < schlick)
                        tk->direction = vreflect(tk->direction, n);
                    else if (no_tir(r, c))
                        tk->direction = refract_dir(tk->direction, n, r, c);
                    else
                        tk->direction = vreflect(tk->direction, n);
                } else {
                    tk->direction = vreflect(tk->direction, n);
                }
                casts++;
                idx = find_closest(sc, tk->direction, tk->origin);
                task_t nt = *tk;
                nt.sphere_index = idx;
                nt.bounce_count = fr->bounces;
                trace_task(sc, nt, &next, &casts);
            }
            /* skybox, lines 182-189 */
            for (size_t i = 0; i < tasks.skybox.n; ++i) {
                task_t *tk = &tasks.skybox.v[i];
                v4 color = vmul(vmul(ld4(fr->sky), tk->direction.y + 1.f), 0.5f);
                size_t ci = (size_t)(tk->x - xB) + (size_t)(tk->y - yB) * segH;
                colors[ci] = vadd(colors[ci], color);
                samples[ci] += 1.f;
            }
            swap_tasks(&tasks, &next);
            clear_tasks(&next);
        }
    }

    /* resolve, lines 196-205 */
    for (size_t i = 0; i < slots; ++i) {
        colors[i] = vmul(colors[i], 1.f / samples[i]);
        uint32_t x = (uint32_t)(i % segW) + xB;
        uint32_t y = (uint32_t)(i / segW) + yB;
        if (rgba) st4(rgba + 4 * ((size_t)(y - yB) * segW + (x - xB)), colors[i]);
        if (rgb8) write_pixel(rgb8 + g_index(fr, x, y), colors[i]);
    }
    free_tasks(&tasks);
    free_tasks(&next);
    free(colors);
    free(samples);
    return casts;
}

/* ------------------------------------------------------------------------- */
/* Renderer.hpp:232-302 dispatch: tc x tc tiles, at most tc in flight         */
/* ------------------------------------------------------------------------- */
typedef struct par_job {
    const spo_scene *sc;
    const spo_frame *fr;
    int mode;
    float *rgba;
    uint8_t *rgb8;
    uint32_t tc, seg_w, seg_h, ntiles;
    uint32_t next;
    pthread_mutex_t mu;
} par_job;

static void *par_worker(void *arg)
{
    par_job *j = (par_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t k = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (k >= j->ntiles) break;
        uint32_t i = k % j->tc, jj = k / j->tc;
        /* Renderer.hpp:232-240 MakeRenderSegmentData */
        uint32_t yB = j->seg_h * jj;
        uint32_t yE = yB + j->seg_h > j->fr->height ? j->fr->height : yB + j->seg_h;
        uint32_t xB = j->seg_w * i;
        uint32_t xE = xB + j->seg_w > j->fr->width ? j->fr->width : xB + j->seg_w;
        uint32_t w = xE - xB;
        float *tile = j->rgba ? (float *)malloc(sizeof(float) * 4 * (size_t)w * (yE - yB) + 16) : NULL;
        if (j->mode == 0)
            spo_render_segment(j->sc, j->fr, yB, yE, xB, xE, tile, j->rgb8);
        else
            spo_render_segment_task(j->sc, j->fr, yB, yE, xB, xE, tile, j->rgb8);
        if (tile) {
            for (uint32_t y = yB; y < yE; ++y)
                memcpy(j->rgba + 4 * ((size_t)y * j->fr->width + xB), tile + 4 * (size_t)(y - yB) * w,
                       sizeof(float) * 4 * w);
            free(tile);
        }
    }
    return NULL;
}

int spo_render_image_parallel(const spo_scene *sc, const spo_frame *fr, uint32_t thread_count, int mode, float *rgba,
                              uint8_t *rgb8)
{
    if (thread_count == 0) return -1;
    par_job j;
    j.sc = sc;
    j.fr = fr;
    j.mode = mode;
    j.rgba = rgba;
    j.rgb8 = rgb8;
    j.tc = thread_count;
    j.seg_w = fr->width / thread_count;
    j.seg_h = fr->height / thread_count;
    j.ntiles = thread_count * thread_count;
    j.next = 0;
    pthread_mutex_init(&j.mu, NULL);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * thread_count);
    for (uint32_t t = 0; t < thread_count; ++t) pthread_create(&th[t], NULL, par_worker, &j);
    for (uint32_t t = 0; t < thread_count; ++t) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&j.mu);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* SceneGenerators.hpp                                                        */
/* ------------------------------------------------------------------------- */
static void put_sphere(float *centers, float *radii, float *colors, uint8_t *materials, uint32_t i, v4 c, float r,
                       v4 col, uint8_t m)
{
    st4(centers + 4 * (size_t)i, c);
    radii[i] = r;
    st4(colors + 4 * (size_t)i, col);
    materials[i] = m;
}

/* SceneGenerators.hpp:6-66 GenerateSpheres.  `abs(z)` (line 34) binds to
 * std::abs(float) (the stb headers' <stdlib.h>, see schlick_of), i.e. fabsf.  Draws that feed
 * the dead g_attenuations (lines 56-59) are consumed to keep the stream. */
uint32_t spo_generate_spheres(uint32_t seed, uint32_t cap, float *centers, float *radii, float *colors,
                              uint8_t *materials, float *fuzz)
{
    uint64_t st = spo_scene_state(seed);
    uint32_t n = 0;
    if (cap < 4) return 0;
    put_sphere(centers, radii, colors, materials, n++, V3(0, -1e6f, 0), 1e6f, V3(30, 144, 255), SPO_DIFFUSE);
    put_sphere(centers, radii, colors, materials, n++, V3(0, 3, 10), 3, V3(0, 0, 0), SPO_REFRACTIVE);
    put_sphere(centers, radii, colors, materials, n++, V3(5, 3, 5), 3, V3(0, 0, 0), SPO_REFLECTIVE);
    put_sphere(centers, radii, colors, materials, n++, V3(-7, 3, 14), 3, V3(223, 55, 132), SPO_DIFFUSE);

    const float minR = 0.3f, maxR = 0.5f;
    v4 s1 = ld4(centers + 4), s2 = ld4(centers + 8), s3 = ld4(centers + 12);
    for (float z = 0; z < 20; z += 1.25f) {
        const float bound = fabsf(z) * 0.85f;
        for (float x = -5 - bound; x < 6 + bound; x += 1.25f) {
            if (spo_uniform(&st, 0, 1.f) > 0.5f) {
                float r = spo_uniform(&st, minR, maxR);
                float cx = x + spo_uniform(&st, 0, minR);
                float cz = z + spo_uniform(&st, 0, minR);
                v4 c = V3(cx, r, cz);
                if ((vlen(vsub(c, s1)) - r - radii[1] < 0.5f) || (vlen(vsub(c, s2)) - r - radii[2] < 0.5f) ||
                    (vlen(vsub(c, s3)) - r - radii[3] < 0.5f))
                    continue;
                float cr = spo_uniform(&st, 0, 255);
                float cg = spo_uniform(&st, 0, 255);
                float cb = spo_uniform(&st, 0, 255);
                float mf = roundf(spo_uniform(&st, 0.5f, 6.0f));
                uint8_t m = (uint8_t)(mf < 3.0f ? mf : 3.0f);
                if (n >= cap) return 0;
                put_sphere(centers, radii, colors, materials, n++, c, r, V3(cr, cg, cb), m);
            }
        }
    }
    for (uint32_t i = 0; i < n; ++i)
        if (spo_uniform(&st, 0, 1) > 0.2f) (void)unit_vector(&st);
    for (uint32_t i = 0; i < n; ++i) {
        fuzz[i] = 0.0f;
        if (spo_uniform(&st, 0, 1) > 0.2f) fuzz[i] = spo_uniform(&st, 0, 1);
    }
    fuzz[2] = 0.01f;
    return n;
}

/* SceneGenerators.hpp:68-133 InitSpheres (g_sphereNumber = 10, Globals.hpp:37) */
uint32_t spo_init_spheres(uint32_t seed, float *centers, float *radii, float *colors, uint8_t *materials, float *fuzz)
{
    static const float col[10][3] = {{30, 144, 255}, {10, 255, 110}, {110, 10, 255}, {255, 100, 230}, {200, 255, 110},
                                     {210, 10, 255}, {255, 100, 150}, {50, 255, 200}, {10, 210, 255}, {255, 100, 220}};
    static const float cen[10][3] = {{0, -1e3f - 0.5f, 0}, {-1, 0, 0}, {0, 0, 0}, {1, 0, 0}, {-1, 1, 0},
                                     {0, 1, 0},            {1, 1, 0},  {-1, 2, 0}, {0, 2, 0}, {1, 2, 0}};
    static const uint8_t mat[10] = {SPO_DIFFUSE, SPO_DIFFUSE,    SPO_REFLECTIVE, SPO_DIFFUSE,    SPO_DIFFUSE,
                                    SPO_REFRACTIVE, SPO_DIFFUSE, SPO_DIFFUSE,    SPO_REFLECTIVE, SPO_DIFFUSE};
    uint64_t st = spo_scene_state(seed);
    for (uint32_t i = 0; i < 10; ++i)
        put_sphere(centers, radii, colors, materials, i, V3(cen[i][0], cen[i][1], cen[i][2]), i == 0 ? 1e3f : 0.5f,
                   V3(col[i][0], col[i][1], col[i][2]), mat[i]);
    for (uint32_t i = 0; i < 10; ++i)
        if (spo_uniform(&st, 0, 1) > 0.3f) (void)unit_vector(&st);
    for (uint32_t i = 0; i < 10; ++i) {
        fuzz[i] = 0.01f;
        if (spo_uniform(&st, 0, 1) > 0.3f) fuzz[i] = spo_uniform(&st, 0, 1);
    }
    fuzz[2] = 0.0f;
    return 10;
}
