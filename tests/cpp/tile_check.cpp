// Host check of the kernel's item orders (spt_internal.h): spt::tile_pixel
// ([sample][tile][pixel]) and spt::ts_item ([band][tile][sample][pixel]) are
// bijections onto the region (x samples) for every shape in a range plus the
// config sizes, full 8x8 tiles are contiguous runs of 64 items, and
// spt::ts_slot_base inverts ts_item (the fold's slot of (pixel, sample)).  The
// sample codes: code_word / word_code round trip, and no sky word k = fl(y + 1.f)
// (any float y) falls in the code range.  Exit 0 = pass.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "spt_internal.h"

int main()
{
    for (uint32_t rows = 1; rows <= 41; ++rows)
        for (uint32_t width = 1; width <= 70; ++width) {
            std::vector<int> seen(rows * width, 0);
            for (uint32_t q = 0; q < rows * width; ++q) {
                uint32_t lr, col;
                spt::tile_pixel(q, width, rows, lr, col);
                if (lr >= rows || col >= width || seen[lr * width + col]++) {
                    std::printf("FAIL rows=%u width=%u q=%u -> (%u, %u)\n", rows, width, q, lr, col);
                    return 1;
                }
                if (rows % 8 == 0 && width % 8 == 0) {
                    uint32_t l0, c0;
                    spt::tile_pixel(q & ~63u, width, rows, l0, c0);
                    if (lr / 8 != l0 / 8 || col / 8 != c0 / 8) {
                        std::printf("FAIL tile run rows=%u width=%u q=%u\n", rows, width, q);
                        return 1;
                    }
                }
            }
        }
    // config-sized shapes
    const uint32_t shapes[][2] = {{800, 1200}, {2160, 3840}, {1080, 1920}, {100, 200}, {101, 1201}};
    for (auto &sh : shapes) {
        const uint32_t rows = sh[0], width = sh[1];
        std::vector<unsigned char> seen((size_t)rows * width, 0);
        for (uint32_t q = 0; q < rows * width; ++q) {
            uint32_t lr, col;
            spt::tile_pixel(q, width, rows, lr, col);
            if (lr >= rows || col >= width || seen[(size_t)lr * width + col]++) {
                std::printf("FAIL rows=%u width=%u q=%u\n", rows, width, q);
                return 1;
            }
        }
    }
    // ts_item: [band][tile][sample][pixel] over rows x width x S is a bijection
    for (uint32_t S = 1; S <= 5; S += 2)
        for (uint32_t rows = 1; rows <= 27; ++rows)
            for (uint32_t width = 1; width <= 35; ++width) {
                const spt::FastDiv fb = spt::make_fastdiv(rows >= 8 ? 8 * width * S : 1), ft = spt::make_fastdiv(64 * S);
                std::vector<int> seen((size_t)rows * width * S, 0);
                for (uint32_t q = 0; q < rows * width * S; ++q) {
                    uint32_t sl, lr, col;
                    spt::ts_item(q, width, rows, S, fb, ft, sl, lr, col);
                    if (sl >= S || lr >= rows || col >= width || seen[((size_t)sl * rows + lr) * width + col]++) {
                        std::printf("FAIL ts rows=%u width=%u S=%u q=%u -> (%u, %u, %u)\n", rows, width, S, q, sl, lr, col);
                        return 1;
                    }
                    uint32_t q0, step;
                    spt::ts_slot_base(lr, col, width, rows, S, q0, step);
                    if (q0 + sl * step != q) {
                        std::printf("FAIL slot rows=%u width=%u S=%u q=%u -> %u + %u * %u\n", rows, width, S, q, q0, sl, step);
                        return 1;
                    }
                    // full tiles: 64 consecutive items are the 64 pixels of one tile and sample
                    if (rows % 8 == 0 && width % 8 == 0) {
                        uint32_t s0, l0, c0;
                        spt::ts_item(q & ~63u, width, rows, S, fb, ft, s0, l0, c0);
                        if (s0 != sl || lr / 8 != l0 / 8 || col / 8 != c0 / 8) {
                            std::printf("FAIL ts run rows=%u width=%u S=%u q=%u\n", rows, width, S, q);
                            return 1;
                        }
                    }
                }
            }
    {
        const uint32_t shapes[][3] = {{800, 1200, 4}, {101, 1201, 3}, {1080, 1920, 2}, {7, 1200, 9}};
        for (auto &sh : shapes) {
            const uint32_t rows = sh[0], width = sh[1], S = sh[2];
            const spt::FastDiv fb = spt::make_fastdiv(rows >= 8 ? 8 * width * S : 1), ft = spt::make_fastdiv(64 * S);
            std::vector<unsigned char> seen((size_t)rows * width * S, 0);
            for (uint32_t q = 0; q < rows * width * S; ++q) {
                uint32_t sl, lr, col;
                spt::ts_item(q, width, rows, S, fb, ft, sl, lr, col);
                if (sl >= S || lr >= rows || col >= width || seen[((size_t)sl * rows + lr) * width + col]++) {
                    std::printf("FAIL ts rows=%u width=%u S=%u q=%u\n", rows, width, S, q);
                    return 1;
                }
                uint32_t q0, step;
                spt::ts_slot_base(lr, col, width, rows, S, q0, step);
                if (q0 + sl * step != q) {
                    std::printf("FAIL slot rows=%u width=%u S=%u q=%u\n", rows, width, S, q);
                    return 1;
                }
            }
        }
    }
    // FastDiv == plain division for x < 2^31 (edges, powers of two, random)
    {
        uint64_t z = 0x9E3779B97F4A7C15ull;
        auto rnd = [&]() { z ^= z << 13; z ^= z >> 7; z ^= z << 17; return z; };
        const uint32_t ds[] = {1, 2, 3, 5, 7, 63, 64, 65, 100, 640, 6400, 76800, 76801, 65536, 0x7FFFFFFF, 0x40000000, 12345677};
        for (uint32_t d : ds) {
            const spt::FastDiv f = spt::make_fastdiv(d);
            for (uint32_t k = 0; k < 200000; ++k) {
                uint32_t x = (uint32_t)(rnd() & 0x7FFFFFFF);
                if (k < 64) x = k < 32 ? k : 0x7FFFFFFFu - (k - 32);
                if (k >= 64 && k < 128) x = (uint32_t)std::min<uint64_t>(0x7FFFFFFFu, (uint64_t)d * (k - 64) + (k & 1 ? d - 1 : 0));
                if (spt::fast_div(x, f) != x / d) {
                    std::printf("FAIL fast_div %u / %u\n", x, d);
                    return 1;
                }
            }
        }
        for (uint32_t k = 0; k < 2000000; ++k) {
            const uint32_t d = (uint32_t)(rnd() % 0x7FFFFFFF) + 1, x = (uint32_t)(rnd() & 0x7FFFFFFF);
            if (spt::fast_div(x, spt::make_fastdiv(d)) != x / d) {
                std::printf("FAIL fast_div %u / %u\n", x, d);
                return 1;
            }
        }
    }
    // sample codes: every code round-trips (edges + a stride), the colour-0 word, and
    // no k = fl(y + 1.f) of any float y is a code word (so sky words and codes never mix)
    {
        const uint32_t cmax = spt::kCodeMax;
        // diffuse codes 2 + j * stride + slot: every (j, slot) of a fitting layout stays in
        // [2, cmax] and decodes back (edges of j and slot, strides up to the largest that fits)
        const uint32_t strides[] = {1, 2, 3, 149, 164, 10007, 1u << 22, 34500000u, 0x66FFFFFCu};
        const uint32_t jmaxes[] = {0, 1, 49, 157, 280};
        for (uint32_t S : strides)
            for (uint32_t J : jmaxes) {
                if (!spt::code_layout_fits(S, J)) continue;
                const spt::FastDiv div = spt::make_fastdiv(S);
                const uint32_t js[] = {0, 1, J / 2, J > 0 ? J - 1 : 0, J};
                const uint32_t ss[] = {0, 1, S / 2, S - 1};
                for (uint32_t j : js)
                    for (uint32_t sl : ss) {
                        if (j > J || sl >= S) continue;
                        const uint32_t c = spt::diffuse_code(j, sl, S);
                        uint32_t j2, s2;
                        spt::diffuse_decode(c, div, j2, s2);
                        if (c < 2 || c > cmax || j2 != j || s2 != sl) {
                            std::printf("FAIL diffuse code S=%u J=%u j=%u slot=%u -> %u -> (%u, %u)\n", S, J, j, sl, c,
                                        j2, s2);
                            return 1;
                        }
                    }
            }
        if (spt::code_layout_fits(0x66FFFFFEu, 0) || !spt::code_layout_fits(34500000u, 49) ||
            spt::code_layout_fits(34600000u, 49)) {
            std::printf("FAIL code capacity bounds\n");
            return 1;
        }
        for (uint64_t c = 1; c <= cmax; c += (c < 64 || cmax - c < 64 || (c > spt::kCodeSmall - 64 && c < spt::kCodeSmall + 64)) ? 1 : 9973) {
            const uint32_t w = spt::code_word((uint32_t)c);
            if (spt::word_code(w) != c) {
                std::printf("FAIL code %llu -> %08x -> %u\n", (unsigned long long)c, w, spt::word_code(w));
                return 1;
            }
        }
        if (spt::code_word(1) != spt::kZeroWord || spt::word_code(spt::kZeroWord) != 1) {
            std::printf("FAIL zero word\n");
            return 1;
        }
        volatile float one = 1.0f;
        uint32_t bits = 0;
        do {
            float y, k;
            std::memcpy(&y, &bits, 4);
            k = y + one;
            uint32_t kw;
            std::memcpy(&kw, &k, 4);
            if (spt::word_code(kw) != 0) {
                std::printf("FAIL sky word y=%08x k=%08x is a code\n", bits, kw);
                return 1;
            }
        } while (++bits != 0);
    }
    std::printf("ok\n");
    return 0;
}
