// spt_accel.cpp -- traversal tables of the hot loop (host side).
//
// FindClosestIntersectionSphere (Collision.hpp:87-109) tests every sphere.  The
// GPU keeps that result exactly but skips spheres that provably cannot pass
// RaySphereIntersection (Collision.hpp:9-17) for any lane of a wave:
//
//  * "always" spheres (large radius: the ground r = 1e6, the three r = 3 balls of
//    GenerateSpheres) are tested for every ray;
//  * the small spheres are sorted along a Morton curve and cut into clusters of
//    K slots, each with a bounding sphere (Cb, Rb >= |Cm - Cb| + r_m).
//
// Cull condition, derived in DESIGN.md §4.1 (fp32 error analysis of both the
// member test and the cluster test for a ray whose fp32 direction has
// | |d|^2 - 1 | <= 1e-6; other lanes never cull): a member can pass only if the
// cluster's computed value
//     d2b = |Cb-o|^2 - ((Cb-o).d)^2  <=  K1 + K2 * |Cb-o|^2,
// K1 = 1.15 Rb^2 + 1e-5, K2 = 1e-4  (each about 2x the derived worst case).
// The kernel evaluates exactly that; clusters failing it for every lane are
// skipped.  Tests run in traversal order, so the closest hit is selected by the
// lexicographic (distance, original index) minimum, which equals the
// reference's strict-'>' first-index-wins scan.
#include "spt_accel.h"
#include "spt_internal.h"

#pragma clang fp contract(off)

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

namespace spt {

namespace {

uint32_t spread10(uint32_t v)
{
    v &= 0x3FF;
    v = (v | (v << 16)) & 0x030000FF;
    v = (v | (v << 8)) & 0x0300F00F;
    v = (v | (v << 4)) & 0x030C30C3;
    v = (v | (v << 2)) & 0x09249249;
    return v;
}

float round_up(double x)
{
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
}

const float4 kDummy = make_float4(0.f, 0.f, 0.f, -INFINITY);  // r*r = -inf: never passes

}  // namespace

AccelTables build_accel(const float *centers4, const float *radii, uint32_t n, uint32_t cluster_k, uint32_t group)
{
    AccelTables t;
    t.group = group;
    std::vector<uint32_t> always, small;
    if (cluster_k == 0 || n <= 32) {
        always.resize(n);
        std::iota(always.begin(), always.end(), 0u);
    } else {
        std::vector<float> r(radii, radii + n);
        std::nth_element(r.begin(), r.begin() + n / 2, r.end());
        const float med = r[n / 2];
        for (uint32_t i = 0; i < n; ++i) {
            const bool finite = std::isfinite(radii[i]) && std::isfinite(centers4[4 * i]) &&
                                std::isfinite(centers4[4 * i + 1]) && std::isfinite(centers4[4 * i + 2]);
            (radii[i] > 4.0f * med || !finite ? always : small).push_back(i);
        }
    }
    // always-list, padded to whole groups
    auto push_slot = [&](uint32_t i) {
        const float rr = radii[i] * radii[i];
        t.slots.push_back(make_float4(centers4[4 * i], centers4[4 * i + 1], centers4[4 * i + 2], rr));
        t.orig.push_back(i);
    };
    auto pad_to = [&](size_t mult, size_t base) {  // pad (size - base) to a multiple of mult
        while ((t.slots.size() - base) % mult) {
            t.slots.push_back(kDummy);
            t.orig.push_back(0xFFFFFFFFu);
        }
    };
    for (uint32_t i : always) push_slot(i);
    pad_to(group, 0);
    t.always_groups = (uint32_t)(t.slots.size() / group);
    if (!small.empty()) {
        const uint32_t k = std::min(cluster_k, kClusterSlots);  // members per cluster
        t.cluster_k = kClusterSlots;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i : small)
            for (int c = 0; c < 3; ++c) {
                lo[c] = std::min(lo[c], (double)centers4[4 * i + c]);
                hi[c] = std::max(hi[c], (double)centers4[4 * i + c]);
            }
        std::vector<std::pair<uint32_t, uint32_t>> keyed;
        for (uint32_t i : small) {
            uint32_t q[3];
            for (int c = 0; c < 3; ++c) {
                const double span = hi[c] - lo[c];
                q[c] = span > 0 ? (uint32_t)std::min(1023.0, (centers4[4 * i + c] - lo[c]) / span * 1023.0) : 0u;
            }
            keyed.push_back({spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2), i});
        }
        std::sort(keyed.begin(), keyed.end());
        for (size_t b = 0; b < keyed.size(); b += k) {
            const size_t e = std::min(keyed.size(), b + k);
            double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (size_t j = b; j < e; ++j)
                for (int c = 0; c < 3; ++c) {
                    clo[c] = std::min(clo[c], (double)centers4[4 * keyed[j].second + c]);
                    chi[c] = std::max(chi[c], (double)centers4[4 * keyed[j].second + c]);
                }
            const double cb[3] = {(clo[0] + chi[0]) / 2, (clo[1] + chi[1]) / 2, (clo[2] + chi[2]) / 2};
            const float cbf[3] = {(float)cb[0], (float)cb[1], (float)cb[2]};
            double rb = 0;
            for (size_t j = b; j < e; ++j) {
                const uint32_t i = keyed[j].second;
                double d2 = 0;
                for (int c = 0; c < 3; ++c) {
                    const double dd = (double)centers4[4 * i + c] - (double)cbf[c];
                    d2 += dd * dd;
                }
                rb = std::max(rb, std::sqrt(d2) + std::fabs((double)radii[i]));
                push_slot(i);
            }
            pad_to(kClusterSlots, (size_t)t.always_groups * group);
            rb *= 1.0 + 1e-6;
            t.bounds.push_back(make_float4(cbf[0], cbf[1], cbf[2], round_up(1.15 * rb * rb + 1e-5)));
        }
        t.clusters = (uint32_t)t.bounds.size();
    }
    // the kernel prefetches up to two groups past the last slot it tests
    for (uint32_t j = 0; j < 2 * group; ++j) {
        t.slots.push_back(kDummy);
        t.orig.push_back(0xFFFFFFFFu);
    }
    t.bounds.push_back(make_float4(0.f, 0.f, 0.f, -INFINITY));  // prefetch pad
    return t;
}

std::vector<float4> eye_relative(const std::vector<float4> &points, const float eye[3])
{
    std::vector<float4> out(points.size());
    for (size_t i = 0; i < points.size(); ++i) {
        const float x = points[i].x - eye[0], y = points[i].y - eye[1], z = points[i].z - eye[2];
        out[i] = make_float4(x, y, z, (x * x + y * y) + z * z);  // lensq order, Math.hpp:122-133
    }
    return out;
}

}  // namespace spt
