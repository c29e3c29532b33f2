// spt_kernels.hip -- MI355X (gfx950) kernels of the SimplePathTracer render loop.
//
// render_kernel: persistent wavefront megakernel.  Each lane owns one
// (pixel, sample) path at a time and runs the reference's recursion
// (TraceAndSampleColor -> SampleColor{Diffuse,Reflective,Refractive,Skybox},
// SingleThreadPathTracer.hpp:11-112) as an iterative state machine: every loop
// iteration is exactly one FindClosestIntersectionSphere cast
// (Collision.hpp:87-109) for every live lane, followed by one shading step.
// When a path ends its colour goes to a per-sample slot and the lane takes the
// next (pixel, sample) item; items are handed out by a wave-level ballot/mbcnt
// prefix over a block claimed from one global counter, so lanes never wait for
// the slowest path of their wave.  Sphere data is read with wave-uniform scalar
// loads (s_load) -- the sphere index of the hot loop is the same for all lanes.
//
// fold_kernel: RenderSegment's `pixelColor += sample` in sample order followed by
// `*= 1/g_samples` (SingleThreadPathTracer.hpp:121-134) or RenderSegmentTask's
// count-weighted resolve (TaskBasedPathTracer.hpp:196-205), plus WritePixel.
// Sums are formed in sample order, so results are bit-identical to the
// sequential reference loop whatever order the paths finished in.
#include "spt_device.h"
#include "spt_internal.h"

#include <float.h>

#pragma clang fp contract(off)

namespace spt {

namespace {

constexpr uint32_t PH_IDLE = 0, PH_TRACE = 1, PH_DLOOP = 2;

// rSq of SampleColorRefractive (lines 58 and 75): float(pow(double(-0.2f), 2)).
// The exact square of a float is representable in double, so pow returns it.
constexpr float kRsq = (float)((double)((1.0f - 1.5f) / (1.0f + 1.5f)) * (double)((1.0f - 1.5f) / (1.0f + 1.5f)));
constexpr float kAirToGlass = 1.0f / 1.5f;
constexpr float kGlassToAir = 1.5f / 1.0f;

__device__ __forceinline__ uint32_t lane_rank(unsigned long long mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

}  // namespace

__global__ __launch_bounds__(kRenderBlock) void render_kernel(RenderArgs a)
{
    const uint32_t lane = __lane_id();
    const uint32_t n = a.scene.n;
    const float4 *__restrict__ hit = a.scene.hit;
    const float4 *__restrict__ shade = a.scene.shade;
    const uint32_t *__restrict__ mat = a.scene.mat;

    uint32_t phase = PH_IDLE, item = 0, bounce = 0, spec = 0;
    uint64_t st = 0;
    f3 o = mk(0.f, 0.f, 0.f), d = mk(0.f, 0.f, 0.f), c = mk(0.f, 0.f, 0.f);

    uint32_t blk_cur = 0, blk_end = 0;
    bool exhausted = false;
    unsigned long long casts = 0, done = 0, dropped = 0;

    for (;;) {
        // ---- hand out (pixel, sample) items to idle lanes: ballot + prefix ----
        const unsigned long long need = __ballot(phase == PH_IDLE);
        if (need != 0ull && !exhausted) {
            const uint32_t cnt = (uint32_t)__popcll(need);
            const uint32_t rank = lane_rank(need);
            const uint32_t avail = blk_end - blk_cur;
            uint32_t mine = 0xFFFFFFFFu;
            if (rank < avail) mine = blk_cur + rank;
            if (avail >= cnt) {
                blk_cur += cnt;
            } else {
                uint32_t nb = 0;
                if (lane == 0) nb = atomicAdd(a.head, a.claim);
                nb = __builtin_amdgcn_readfirstlane(nb);
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
            if (phase == PH_IDLE && mine != 0xFFFFFFFFu) {
                // primary ray, SingleThreadPathTracer.hpp:123-130
                item = mine;
                const uint32_t pl = item / a.spp_batch;
                const uint32_t s = a.s0 + (item - pl * a.spp_batch);
                const uint32_t lr = pl / a.map.width;
                const uint32_t x = a.map.x0 + (pl - lr * a.map.width);
                const uint32_t y = row_of(a.map, lr);
                st = fmix64(a.seed_key ^ (((uint64_t)(y * a.width + x) << 32) | (uint64_t)s));
                const float u = ((float)y + uniform(st, -1.f, 1.f)) / (float)a.width;
                const float v = ((float)x + uniform(st, -1.f, 1.f)) / (float)a.height;
                const float vx = -1.f + 2.f * v, vy = -1.f + 2.f * u;
                const float *m = a.cam.view;
                d = normalize(mk((m[0] * vx + m[1] * vy) + (m[2] * 1.f + m[3] * 0.f),
                                 (m[4] * vx + m[5] * vy) + (m[6] * 1.f + m[7] * 0.f),
                                 (m[8] * vx + m[9] * vy) + (m[10] * 1.f + m[11] * 0.f)));
                o = mk(a.cam.eye[0], a.cam.eye[1], a.cam.eye[2]);
                phase = PH_TRACE;
                bounce = a.bounces;
                spec = 0;
            }
        }
        const unsigned long long live = __ballot(phase != PH_IDLE);
        if (live == 0ull) break;
        casts += (unsigned long long)__popcll(live);

        // ---- FindClosestIntersectionSphere, Collision.hpp:87-109 ----
        uint32_t idx = n;
        float best = FLT_MAX;
        f3 bp = o;
        const float dod = dot(o, d);
#pragma unroll 2
        for (uint32_t i = 0; i < n; ++i) {
            const float4 sp = hit[i];
            // RaySphereIntersection, Collision.hpp:9-17
            const float ocx = sp.x - o.x, ocy = sp.y - o.y, ocz = sp.z - o.z;
            const float tc = (ocx * d.x + ocy * d.y) + ocz * d.z;
            const float d2 = ((ocx * ocx + ocy * ocy) + ocz * ocz) - tc * tc;
            const float h = sp.w - d2;
            if (tc > 1e-3f && h > 1e-3f) {
                // CalculateRaySphereClosestContactPoint, Collision.hpp:19-27,49-56
                const float t = tc - __builtin_sqrtf(h);
                const f3 p = mk(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t);
                if (dod < dot(p, d)) {
                    const float ds = lensq(sub(o, p));
                    if (best > ds) {
                        best = ds;
                        idx = i;
                        bp = p;
                    }
                }
            }
        }

        // ---- one shading step ----
        if (phase != PH_IDLE) {
            bool fin = false;
            float counted = 1.f;
            f3 col = mk(0.f, 0.f, 0.f);
            const bool dl = phase == PH_DLOOP;
            uint32_t m = SPT_SKYBOX_ID;
            if (idx < n) m = mat[idx];
            bool scatter, refr;
            if (dl) {
                // while (--bounceCount && sphereIndex < N), SingleThreadPathTracer.hpp:28
                --bounce;
                const bool end = bounce == 0u || idx >= n;
                if (end) {
                    col = c;
                    fin = true;
                }
                scatter = !end;
                refr = false;
            } else {
                // TraceAndSampleColor material switch, SingleThreadPathTracer.hpp:98-111
                scatter = m == SPT_DIFFUSE_ID || m == SPT_REFLECTIVE_ID;
                refr = m == SPT_REFRACTIVE_ID;
                if (!scatter && !refr) {
                    // SampleColorSkybox, lines 11-14
                    const float k = d.y + 1.f;
                    col = mul(mk(a.cam.sky[0] * k, a.cam.sky[1] * k, a.cam.sky[2] * k), 0.5f);
                    fin = true;
                }
            }
            bool spec_event = false;
            if (scatter) {
                // contact point + normal + cube-minus-ball vector, shared by the diffuse
                // first hit (lines 23-26), the diffuse loop (30-33) and the mirror (41-43)
                const float4 cs = hit[idx];
                const f3 C = mk(cs.x, cs.y, cs.z);
                o = bp;
                const f3 nrm = normalize(sub(o, C));
                f3 rv = ball_vector(st);
                f3 base;
                if (dl) {
                    c = mul(c, 0.5f);
                    base = add(o, nrm);  // origin + normal (+ rv), line 32
                } else if (m == SPT_DIFFUSE_ID) {
                    const float4 sh = shade[idx];
                    c = mk(sh.x * 0.5f, sh.y * 0.5f, sh.z * 0.5f);
                    base = nrm;
                    phase = PH_DLOOP;
                } else {
                    base = reflect(d, nrm);
                    rv = mul(rv, shade[idx].w);
                    spec_event = true;
                }
                d = normalize(add(base, rv));
            }
            if (refr) {
                // SampleColorRefractive, lines 48-92
                const float4 cs = hit[idx];
                const f3 C = mk(cs.x, cs.y, cs.z);
                o = bp;
                const f3 nrm = normalize(sub(o, C));
                const float cc = dot(neg(nrm), d);
                f3 nd;
                if (uniform(st, 0.f, 1.f) < schlick(kRsq, cc)) {
                    nd = reflect(d, nrm);
                } else if (no_tir(kAirToGlass, cc)) {
                    const f3 d2 = refract_dir(d, nrm, kAirToGlass, cc);
                    // CalculateRaySphereFarthestContactPoint, Collision.hpp:29-37,58-65
                    const f3 rs = sub(C, o);
                    const float tc = dot(rs, d2);
                    const float dd = lensq(rs) - tc * tc;
                    const float t = tc + __builtin_sqrtf(cs.w - dd);
                    o = mk(o.x + d2.x * t, o.y + d2.y * t, o.z + d2.z * t);
                    const f3 n2 = neg(normalize(sub(o, C)));
                    const float c2 = dot(neg(n2), d2);
                    if (uniform(st, 0.f, 1.f) < schlick(kRsq, c2))
                        nd = reflect(d2, n2);
                    else if (no_tir(kGlassToAir, c2))
                        nd = refract_dir(d2, n2, kGlassToAir, c2);
                    else
                        nd = reflect(d2, n2);
                } else {
                    nd = reflect(d, nrm);
                }
                d = nd;
                spec_event = true;
            }
            if (spec_event) {
                ++spec;
                if (a.mode == 1u && spec >= kTaskPasses) {
                    // the path would be processed in pass 10, which never runs
                    fin = true;
                    counted = 0.f;
                    col = mk(0.f, 0.f, 0.f);
                    ++dropped;
                } else if (spec > kSpecularCap) {
                    fin = true;
                    col = mk(0.f, 0.f, 0.f);
                }
            }
            if (fin) {
                a.samples[item] = make_float4(col.x, col.y, col.z, counted);
                phase = PH_IDLE;
                d = mk(0.f, 0.f, 0.f);
                ++done;
            }
        }
    }

    // per-lane done/dropped -> wave sums via atomics from every lane that has any
    if (done) atomicAdd(&a.counters[1], done);
    if (dropped) atomicAdd(&a.counters[2], dropped);
    if (lane == 0) atomicAdd(&a.counters[0], casts);
}

__global__ __launch_bounds__(256) void fold_kernel(FoldArgs a)
{
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.npix) return;
    float4 acc = a.first ? make_float4(0.f, 0.f, 0.f, 0.f) : a.acc[p];
    const float4 *s = a.samples + (size_t)p * a.spp_batch;
    for (uint32_t k = 0; k < a.spp_batch; ++k) {
        const float4 c = s[k];
        if (a.mode == 0 || c.w != 0.f) {
            acc.x = acc.x + c.x;
            acc.y = acc.y + c.y;
            acc.z = acc.z + c.z;
            acc.w = acc.w + 1.f;
        }
    }
    if (!a.last) {
        a.acc[p] = acc;
        return;
    }
    // RenderSegment: *= (1.f / g_samples) (line 133); RenderSegmentTask: *= 1.f / samples[i] (line 198)
    const float scale = a.mode == 0 ? 1.f / (float)a.spp_total : 1.f / acc.w;
    const float r = acc.x * scale, g = acc.y * scale, b = acc.z * scale;
    if (a.out_rgba) a.out_rgba[p] = make_float4(r, g, b, 0.f);
    if (a.out_rgb8) {
        const uint32_t lr = p / a.map.width;
        const uint32_t x = a.map.x0 + (p - lr * a.map.width);
        const uint32_t y = row_of(a.map, lr);
        const size_t gi = (size_t)3 * ((size_t)(a.height - 1u - y) * a.width + x);
        a.out_rgb8[gi + 0] = gamma_byte(r);
        a.out_rgb8[gi + 1] = gamma_byte(g);
        a.out_rgb8[gi + 2] = gamma_byte(b);
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
    const float x = a[i], y = b[i];
    float *o = out + (size_t)i * 8;
    o[0] = x / y;
    o[1] = __builtin_sqrtf(x);
    const double sq = __builtin_sqrt((double)x);
    const double p5 = pow5((double)x);
    const uint64_t sqb = __builtin_bit_cast(uint64_t, sq), p5b = __builtin_bit_cast(uint64_t, p5);
    o[2] = __builtin_bit_cast(float, (uint32_t)sqb);
    o[3] = __builtin_bit_cast(float, (uint32_t)(sqb >> 32));
    o[4] = __builtin_bit_cast(float, (uint32_t)p5b);
    o[5] = __builtin_bit_cast(float, (uint32_t)(p5b >> 32));
    o[6] = canon_u32(bits[i]) * (1.f - (-1.f)) + (-1.f);
    o[7] = (float)f2u8(x);
}

hipError_t launch_render(const RenderArgs &a, uint32_t grid, uint32_t block, hipStream_t s)
{
    hipLaunchKernelGGL(render_kernel, dim3(grid), dim3(block), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fold(const FoldArgs &a, hipStream_t s)
{
    if (a.npix == 0) return hipSuccess;
    hipLaunchKernelGGL(fold_kernel, dim3((a.npix + 255) / 256), dim3(256), 0, s, a);
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

hipError_t render_occupancy(uint32_t block, int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, render_kernel, (int)block, 0);
}

}  // namespace spt
