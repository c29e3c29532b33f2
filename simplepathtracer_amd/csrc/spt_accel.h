// spt_accel.h -- traversal tables of the hot loop (see spt_accel.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace spt {

struct AccelTables {
    std::vector<float4> slots;     // {cx, cy, cz, r*r} in traversal order, dummy = r*r -inf
    std::vector<uint32_t> orig;    // original sphere index per slot (0xFFFFFFFF = dummy)
    std::vector<float4> bounds;    // per cluster {Cb.x, Cb.y, Cb.z, K1} (+1 pad)
    uint32_t group = 4;            // spheres per test group (SPT_GROUP)
    uint32_t always_groups = 0;    // groups of always-tested spheres at the front
    uint32_t clusters = 0;         // clusters following them
    uint32_t cluster_k = 0;        // slots per cluster (multiple of group)
};

// Eye-relative copies for the primary-ray pass: {P - eye, |P - eye|^2} with the
// kernel's own fp32 operation order (bit-identical to computing them in-kernel).
std::vector<float4> eye_relative(const std::vector<float4> &points, const float eye[3]);

// cluster_k == 0 (or n <= 32): every sphere is "always" tested (brute force).
AccelTables build_accel(const float *centers4, const float *radii, uint32_t n, uint32_t cluster_k, uint32_t group);

}  // namespace spt
