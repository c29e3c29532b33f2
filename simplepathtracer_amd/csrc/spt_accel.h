// spt_accel.h -- traversal tables of the hot loop (see spt_accel.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "spt_internal.h"

namespace spt {

// One node of the cluster tree, 32 B (one s_load_dwordx8 or two ds_read_b128).
// Nodes are stored in depth-first preorder: the first child of an inner node is the
// next record, and `skip` is the index just past the node's subtree.  Leaves are
// clusters.  Flat-list nodes (no inner nodes) carry a bounding sphere; tree nodes an
// axis-aligned box.  skip/slot sit at dwords 4-5 in both forms.
struct AccelNode {
    union {
        struct {
            float cx, cy, cz;  // flat list: bounding-sphere centre Cb
            float k1;          // flat list: cull constant K1 = 1.15 Rb^2 + 1e-5 (rounded up)
        };
        struct {
            float lox, loy, loz;  // tree: box lo = min (C - r) - kBoxS Bm (rounded down)
            float hix;            // tree: box hi.x = max (C + r) + kBoxS Bm (rounded up)
        };
    };
    uint32_t skip;  // next node when this one is culled (or is a leaf)
    uint32_t slot;  // leaf: first of its leaf_slots slots; inner: kNoSlot
    union {
        struct {
            float rb;   // flat list: K1'' = K1 + 4e-6 |Cb|^2 - cb2 (rounded up), the expanded-form
                        // margin less the node's c |Cb|^2 term
            float cb2;  // flat list: c |Cb|^2 (the expanded line test)
        };
        struct {
            float hiy, hiz;  // tree: box hi.y, hi.z
        };
    };
};
static_assert(sizeof(AccelNode) == 32, "one 32-byte record per node");

struct AccelTables {
    std::vector<float4> slots;      // {cx, cy, cz, r*r} in traversal order, dummy = r*r -inf
    std::vector<uint32_t> orig;     // original sphere index per slot (0xFFFFFFFF = dummy)
    std::vector<AccelNode> nodes;   // 8 octant layouts of the tree in preorder, each
                                    // n_nodes + 1 pad records (one pad if no tree)
    uint32_t group = 4;             // spheres per always-list test group (SPT_GROUP)
    uint32_t always_groups = 0;     // groups of always-tested spheres at the front
    uint32_t n_nodes = 0;           // tree nodes (without the pad)
    uint32_t leaves = 0;            // clusters
    uint32_t depth = 0;             // levels of the tree (1 = flat cluster list)
    uint32_t leaf_slots = kClusterSlots;  // slots per leaf (members <= leaf_slots)
    // member pretest (spt_path.h test_group_pre): per slot
    // K' = c |C|^2 - r^2 (1 + 1e-6) - 4e-6 |C|^2 rounded down (c = kFlatScale; +inf
    // for dummies, 0 in the always-list), and pre_cm >= max |C| + r over the
    // cluster members (rounded up)
    std::vector<float> kpre;
    float pre_cm = 0.f;
};

// cluster_k: members per cluster (0, or n <= 32: every sphere is "always" tested).
// branching: children per inner node; 0 = flat list of clusters (no inner nodes).
// leaf_slots: kFlatLeafSlots (flat lists only, cluster_k <= 4) or kClusterSlots.
AccelTables build_accel(const float *centers4, const float *radii, uint32_t n, uint32_t cluster_k, uint32_t group,
                        uint32_t branching, uint32_t leaf_slots);

// Structural and containment checks of the tables the kernel relies on for
// exactness and in-bounds loads; empty string = valid, else the first problem.
std::string validate_accel(const AccelTables &t, const float *centers4, const float *radii, uint32_t n);

// Primary-ray candidate lists (PrimLists, spt_internal.h) of a scene's traversal tables
// for a camera and frame size: host copies of the device arrays.  `on` is false (every
// block walks) when the camera or the scene makes the cone test unsound (non-finite or
// huge values, a degenerate view).  Blocks with more than max_count candidates walk.
struct PrimListTables {
    std::vector<uint2> b8, b4;
    std::vector<uint32_t> slots;
    uint32_t bw = 0;
    bool on = false;
    double seconds = 0;  // build time (host)
};
PrimListTables build_prim_lists(const AccelTables &t, const Camera &cam, uint32_t width, uint32_t height,
                                uint32_t max_count);

}  // namespace spt
