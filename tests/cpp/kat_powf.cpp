// Exhaustive known-answer test of spt_glibc_powf (simplepathtracer_amd/csrc/spt_powf.h,
// the restatement the GPU kernel uses) against this host's glibc powf.
//   kat_powf [y]   -- every non-NaN float x, y = 5 by default
// Prints "n=<count> bad=<mismatches>" and the first mismatches; exit 0 iff bad == 0.
#include "spt_powf.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <thread>
#include <vector>

int main(int argc, char **argv)
{
    const float y = argc > 1 ? strtof(argv[1], nullptr) : 5.f;
    const unsigned nt = std::max(1u, std::thread::hardware_concurrency());
    std::atomic<long> bad{0}, n{0};
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            long b = 0, c = 0;
            for (uint64_t u = t; u <= 0xffffffffull; u += nt) {
                const float x = spt_powf_detail::u2f((uint32_t)u);
                if (x != x) continue;
                const float want = powf(x, y), got = spt_glibc_powf(x, y);
                ++c;
                if (spt_powf_detail::f2u(want) != spt_powf_detail::f2u(got)) {
                    if (b++ < 4) printf("x=%a y=%a glibc=%a restated=%a\n", x, y, want, got);
                }
            }
            bad += b;
            n += c;
        });
    for (auto &x : th) x.join();
    // the refraction's constant exponent-2 calls (rSq), both signs
    for (float x : {-0.2f, 0.2f, (1.0f - 1.5f) / (1.0f + 1.5f), (1.5f - 1.0f) / (1.5f + 1.0f)}) {
        const float want = powf(x, 2.f), got = spt_glibc_powf(x, 2.f);
        if (spt_powf_detail::f2u(want) != spt_powf_detail::f2u(got)) {
            printf("x=%a y=2 glibc=%a restated=%a\n", x, want, got);
            ++bad;
        }
    }
    printf("n=%ld bad=%ld\n", n.load(), bad.load());
    return bad.load() == 0 ? 0 : 1;
}
