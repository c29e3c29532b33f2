// spt_scene.cpp -- input producers of the render loop (product side).
//
// GenerateSpheres / InitSpheres (SceneGenerators.hpp:6-133) and the camera basis
// (Math.hpp:198-231), restated with the reference's splitmix seeded from a
// caller-supplied seed instead of steady_clock (Random.hpp:86-93).  Compiled
// with -ffp-contract=off so the fp32 arithmetic matches the reference bit for bit.
#include "spt_hip.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#pragma clang fp contract(off)

namespace {

struct V {
    float x, y, z, w;
};
inline V v3(float x, float y, float z) { return V{x, y, z, 0.0f}; }
inline V vsub(V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
inline float vlensq(V a) { return (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w); }
inline float vlen(V a) { return std::sqrt(vlensq(a)); }
inline V vnorm(V a)
{
    float l = std::sqrt(vlensq(a));
    return V{a.x / l, a.y / l, a.z / l, a.w / l};
}
// Math.hpp:113-120, z-component bug included
inline V vcross(V a, V b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.x - a.y * b.x); }

// Random.hpp:11-46 splitmix; seeded as splitmix(uint64_t seed): seed << 31 | seed.
struct SplitMix {
    uint64_t s;
    explicit SplitMix(uint32_t seed) : s(((uint64_t)seed << 31) | (uint64_t)seed) {}
    uint32_t operator()()
    {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return (uint32_t)((z ^ (z >> 31)) >> 31);
    }
    // std::uniform_real_distribution<float>(a, b) over this engine (libstdc++):
    // generate_canonical<float,24> = float(u)/2^32 clamped below 1, then u*(b-a)+a.
    float uniform(float a, float b)
    {
        float u = (float)(*this)() / 4294967296.0f;
        if (u >= 1.0f) u = std::nextafter(1.0f, 0.0f);
        return u * (b - a) + a;
    }
    // Random.hpp:95-113 GenerateUnitVector<3> (only its draws matter here)
    void unit_vector()
    {
        float x = uniform(-1.f, 1.f), y = uniform(-1.f, 1.f), z = uniform(-1.f, 1.f);
        (void)vnorm(v3(x, y, z));
    }
};

struct Out {
    float *c, *r, *col, *f;
    uint8_t *m;
    void put(uint32_t i, V center, float radius, V color, uint8_t mat)
    {
        c[4 * i + 0] = center.x;
        c[4 * i + 1] = center.y;
        c[4 * i + 2] = center.z;
        c[4 * i + 3] = 0.0f;
        r[i] = radius;
        col[4 * i + 0] = color.x;
        col[4 * i + 1] = color.y;
        col[4 * i + 2] = color.z;
        col[4 * i + 3] = 0.0f;
        m[i] = mat;
    }
    V center(uint32_t i) const { return v3(c[4 * i], c[4 * i + 1], c[4 * i + 2]); }
};

}  // namespace

extern "C" int spt_scene_generate_random(uint32_t seed, uint32_t capacity, float *centers4, float *radii,
                                         float *colors4, uint8_t *materials, float *fuzz, uint32_t *n_out)
{
    return spt_scene_generate_random_rows(seed, 20.0f, capacity, centers4, radii, colors4, materials, fuzz, n_out);
}

// GenerateSpheres with its row loop run to z < z_end (the reference: 20).  Wider z ranges
// give BASELINE.json's "~500-sphere" RTIOW scene (z_end 37.5: 488 spheres for seed 1)
// with the reference's own placement rule, draw order and materials; only the row count
// changes.  More than 255 spheres need the 32-bit index.
extern "C" int spt_scene_generate_random_rows(uint32_t seed, float z_end, uint32_t capacity, float *centers4,
                                              float *radii, float *colors4, uint8_t *materials, float *fuzz,
                                              uint32_t *n_out)
{
    if (!centers4 || !radii || !colors4 || !materials || !fuzz || !n_out || capacity < 4) return SPT_ERR_ARG;
    if (!(z_end >= 0.0f && z_end <= 1000.0f)) return SPT_ERR_ARG;
    SplitMix rng(seed);
    Out o{centers4, radii, colors4, fuzz, materials};
    uint32_t n = 0;
    // SceneGenerators.hpp:8-26: ground + three big spheres
    o.put(n++, v3(0, -1e6f, 0), 1e6f, v3(30, 144, 255), SPT_DIFFUSE);
    o.put(n++, v3(0, 3, 10), 3, v3(0, 0, 0), SPT_REFRACTIVE);
    o.put(n++, v3(5, 3, 5), 3, v3(0, 0, 0), SPT_REFLECTIVE);
    o.put(n++, v3(-7, 3, 14), 3, v3(223, 55, 132), SPT_DIFFUSE);
    const float minR = 0.3f, maxR = 0.5f;
    const V s1 = o.center(1), s2 = o.center(2), s3 = o.center(3);
    // SceneGenerators.hpp:32-53.  abs(z) binds std::abs(float) in the reference's TU
    // (oracle/probe_overloads.cpp).
    for (float z = 0; z < z_end; z += 1.25f) {
        const float bound = std::fabs(z) * 0.85f;
        for (float x = -5 - bound; x < 6 + bound; x += 1.25f) {
            if (rng.uniform(0, 1.f) > 0.5f) {
                const float r = rng.uniform(minR, maxR);
                const float cx = x + rng.uniform(0, minR);
                const float cz = z + rng.uniform(0, minR);
                const V c = v3(cx, r, cz);
                if ((vlen(vsub(c, s1)) - r - radii[1] < 0.5f) || (vlen(vsub(c, s2)) - r - radii[2] < 0.5f) ||
                    (vlen(vsub(c, s3)) - r - radii[3] < 0.5f))
                    continue;
                const float red = rng.uniform(0, 255), green = rng.uniform(0, 255), blue = rng.uniform(0, 255);
                const float mf = std::round(rng.uniform(0.5f, 6.0f));
                if (n >= capacity) return SPT_ERR_ARG;
                o.put(n++, c, r, v3(red, green, blue), (uint8_t)(mf < 3.0f ? mf : 3.0f));
            }
        }
    }
    // SceneGenerators.hpp:56-65: dead attenuations still consume draws; fuzz
    for (uint32_t i = 0; i < n; ++i)
        if (rng.uniform(0, 1) > 0.2f) rng.unit_vector();
    for (uint32_t i = 0; i < n; ++i) {
        fuzz[i] = 0.0f;
        if (rng.uniform(0, 1) > 0.2f) fuzz[i] = rng.uniform(0, 1);
    }
    fuzz[2] = 0.01f;
    *n_out = n;
    return SPT_OK;
}

extern "C" int spt_scene_init_reference(uint32_t seed, float *centers4, float *radii, float *colors4,
                                        uint8_t *materials, float *fuzz, uint32_t *n_out)
{
    if (!centers4 || !radii || !colors4 || !materials || !fuzz || !n_out) return SPT_ERR_ARG;
    // SceneGenerators.hpp:70-120
    static const float kColor[10][3] = {{30, 144, 255}, {10, 255, 110}, {110, 10, 255}, {255, 100, 230},
                                        {200, 255, 110}, {210, 10, 255}, {255, 100, 150}, {50, 255, 200},
                                        {10, 210, 255},  {255, 100, 220}};
    static const float kCenter[10][3] = {{0, -1e3f - 0.5f, 0}, {-1, 0, 0}, {0, 0, 0}, {1, 0, 0}, {-1, 1, 0},
                                         {0, 1, 0},            {1, 1, 0},  {-1, 2, 0}, {0, 2, 0}, {1, 2, 0}};
    static const uint8_t kMat[10] = {SPT_DIFFUSE, SPT_DIFFUSE,    SPT_REFLECTIVE, SPT_DIFFUSE,    SPT_DIFFUSE,
                                     SPT_REFRACTIVE, SPT_DIFFUSE, SPT_DIFFUSE,    SPT_REFLECTIVE, SPT_DIFFUSE};
    Out o{centers4, radii, colors4, fuzz, materials};
    for (uint32_t i = 0; i < 10; ++i)
        o.put(i, v3(kCenter[i][0], kCenter[i][1], kCenter[i][2]), i == 0 ? 1e3f : 0.5f,
              v3(kColor[i][0], kColor[i][1], kColor[i][2]), kMat[i]);
    // SceneGenerators.hpp:122-132 (g_sphereNumber = 10, Globals.hpp:37)
    SplitMix rng(seed);
    for (uint32_t i = 0; i < 10; ++i)
        if (rng.uniform(0, 1) > 0.3f) rng.unit_vector();
    for (uint32_t i = 0; i < 10; ++i) {
        fuzz[i] = 0.01f;
        if (rng.uniform(0, 1) > 0.3f) fuzz[i] = rng.uniform(0, 1);
    }
    fuzz[2] = 0.0f;
    *n_out = 10;
    return SPT_OK;
}

// Build-side stress scene (BASELINE config 5, > 255 spheres): the four big spheres
// of GenerateSpheres, then small spheres on a jittered square grid in front of the
// camera, material drawn like SceneGenerators.hpp:50, fuzz like lines 61-64.
extern "C" int spt_scene_generate_stress(uint32_t seed, uint32_t n, float *centers4, float *radii, float *colors4,
                                         uint8_t *materials, float *fuzz)
{
    if (!centers4 || !radii || !colors4 || !materials || !fuzz || n < 4) return SPT_ERR_ARG;
    SplitMix rng(seed);
    Out o{centers4, radii, colors4, fuzz, materials};
    o.put(0, v3(0, -1e6f, 0), 1e6f, v3(30, 144, 255), SPT_DIFFUSE);
    o.put(1, v3(0, 3, 10), 3, v3(0, 0, 0), SPT_REFRACTIVE);
    o.put(2, v3(5, 3, 5), 3, v3(0, 0, 0), SPT_REFLECTIVE);
    o.put(3, v3(-7, 3, 14), 3, v3(223, 55, 132), SPT_DIFFUSE);
    const uint32_t m = n - 4;
    uint32_t side = 1;
    while (side * side < m) ++side;
    const float pitch = 0.55f;
    for (uint32_t k = 0; k < m; ++k) {
        const uint32_t gi = k % side, gj = k / side;
        const float r = rng.uniform(0.1f, 0.25f);
        const float cx = ((float)gi - 0.5f * (float)side) * pitch + rng.uniform(0, 0.2f);
        const float cz = (float)gj * pitch + rng.uniform(0, 0.2f) - 1.0f;
        const float red = rng.uniform(0, 255), green = rng.uniform(0, 255), blue = rng.uniform(0, 255);
        const float mf = std::round(rng.uniform(0.5f, 6.0f));
        o.put(4 + k, v3(cx, r, cz), r, v3(red, green, blue), (uint8_t)(mf < 3.0f ? mf : 3.0f));
    }
    for (uint32_t i = 0; i < n; ++i) {
        fuzz[i] = 0.0f;
        if (rng.uniform(0, 1) > 0.2f) fuzz[i] = rng.uniform(0, 1);
    }
    fuzz[2] = 0.01f;
    return SPT_OK;
}

// stbi_write_bmp's 24-bit layout (stb_image_write.h stbi_write_bmp_core for comp 3:
// file header "BM", size, 0, 0, 54; BITMAPINFOHEADER 40, w, h, 1 plane, 24 bpp, six
// zero words; pixels bottom-up, BGR, rows padded to 4 bytes), IOHelpers.hpp:24-27.
extern "C" int spt_save_bmp(const char *path, uint32_t width, uint32_t height, uint32_t comp, const uint8_t *data)
{
    if (!path || (!data && width && height) || comp != 3 || width > 0x7FFFFFFFu / 4 || height > 0x7FFFFFFFu)
        return SPT_ERR_ARG;
    const uint32_t pad = (0u - width * 3u) & 3u, row = width * 3u + pad;
    if ((uint64_t)row * height > 0xFFFFFFFFull - 54) return SPT_ERR_ARG;
    std::vector<uint8_t> out(54 + (size_t)row * height, 0);
    auto put4 = [&](size_t at, uint32_t v) {
        for (int k = 0; k < 4; ++k) out[at + k] = (uint8_t)(v >> (8 * k));
    };
    out[0] = 'B';
    out[1] = 'M';
    put4(2, (uint32_t)(54 + (uint64_t)row * height));
    put4(10, 54);
    put4(14, 40);
    put4(18, width);
    put4(22, height);
    out[26] = 1;   // planes
    out[28] = 24;  // bits per pixel
    for (uint32_t r = 0; r < height; ++r) {
        const uint8_t *src = data + (size_t)(height - 1 - r) * width * 3;
        uint8_t *dst = out.data() + 54 + (size_t)r * row;
        for (uint32_t x = 0; x < width; ++x) {
            dst[3 * x + 0] = src[3 * x + 2];
            dst[3 * x + 1] = src[3 * x + 1];
            dst[3 * x + 2] = src[3 * x + 0];
        }
    }
    FILE *f = std::fopen(path, "wb");
    if (!f) return SPT_ERR_ARG;
    const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    return (std::fclose(f) == 0 && ok) ? SPT_OK : SPT_ERR_ARG;
}

extern "C" int spt_camera_basis(const float eye[4], const float look_at[4], const float up[4], float view_out[16])
{
    if (!eye || !look_at || !up || !view_out) return SPT_ERR_ARG;
    const V e = v3(eye[0], eye[1], eye[2]), l = v3(look_at[0], look_at[1], look_at[2]), u = v3(up[0], up[1], up[2]);
    const V view = vnorm(vsub(l, e));
    const V right = vnorm(vcross(u, view));
    const V up2 = vcross(view, right);
    const float basis[16] = {right.x, right.y, right.z, right.w, up2.x, up2.y, up2.z, up2.w,
                             view.x,  view.y,  view.z,  view.w,  0.0f,  0.0f,  0.0f,  0.0f};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) view_out[i * 4 + j] = basis[j * 4 + i];  // Transpose, Math.hpp:211-231
    return SPT_OK;
}
