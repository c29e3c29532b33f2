// Host check of spt::tile_pixel (spt_internal.h): for every region shape in a
// range, the item -> (row, col) map is a bijection onto the region, and full
// 8x8 tiles are contiguous runs of 64 items.  Exit status 0 = pass.
#include <cstdio>
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
    std::printf("ok\n");
    return 0;
}
