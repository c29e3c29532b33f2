// Known-answer test: pins spo_uniform / spo_uniform_u32 (oracle restatement of
// Random.hpp:86-93) against the real libstdc++ std::uniform_real_distribution<float>
// of this image, driven by a restated splitmix engine (Random.hpp:11-46).
// TEST INFRASTRUCTURE ONLY.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include "spt_oracle.h"

struct splitmix_engine {  // same mixer and state update as Random.hpp:30-36
    using result_type = uint32_t;
    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return UINT32_MAX; }
    uint64_t s;
    result_type operator()() {
        uint64_t z = (s += UINT64_C(0x9E3779B97F4A7C15));
        z = (z ^ (z >> 30)) * UINT64_C(0xBF58476D1CE4E5B9);
        z = (z ^ (z >> 27)) * UINT64_C(0x94D049BB133111EB);
        return result_type((z ^ (z >> 31)) >> 31);
    }
};

struct fixed_engine {  // replays chosen 32-bit outputs (edge cases of generate_canonical)
    using result_type = uint32_t;
    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return UINT32_MAX; }
    uint32_t v;
    result_type operator()() { return v; }
};

static uint32_t bits(float f) { uint32_t b; std::memcpy(&b, &f, 4); return b; }

int main() {
    const float ranges[][2] = {{-1.f, 1.f}, {-0.5f, 0.5f}, {0.f, 1.f}, {0.3f, 0.5f}, {0.f, 0.3f},
                               {0.f, 255.f}, {0.5f, 6.0f}};
    long checked = 0, bad = 0;
    for (uint32_t seed = 1; seed <= 64; ++seed) {
        for (auto &rg : ranges) {
            splitmix_engine e{spo_scene_state(seed)};
            uint64_t st = spo_scene_state(seed);
            std::uniform_real_distribution<float> u(rg[0], rg[1]);
            for (int i = 0; i < 20000; ++i) {
                float ref = u(e);
                float got = spo_uniform(&st, rg[0], rg[1]);
                ++checked;
                if (bits(ref) != bits(got)) ++bad;
            }
        }
    }
    // edge values: top of range (canonical >= 1 -> nextafter), powers of two, rounding ties
    const uint32_t edges[] = {0u, 1u, 2u, 127u, 128u, 129u, 255u, 256u, 257u, 0x00FFFFFFu, 0x01000000u,
                              0x01000001u, 0x7FFFFFFFu, 0x80000000u, 0x80000001u, 0xFFFFFF7Fu, 0xFFFFFF80u,
                              0xFFFFFF81u, 0xFFFFFFFEu, 0xFFFFFFFFu};
    for (uint32_t v : edges) {
        for (auto &rg : ranges) {
            fixed_engine e{v};
            std::uniform_real_distribution<float> u(rg[0], rg[1]);
            float ref = u(e);
            float got = spo_uniform_u32(v, rg[0], rg[1]);
            ++checked;
            if (bits(ref) != bits(got)) { ++bad; std::printf("edge mismatch u32=%08x\n", v); }
        }
    }
    std::printf("kat_libstdcxx checked=%ld mismatches=%ld\n", checked, bad);
    return bad ? 1 : 0;
}
