// spt_accel.cpp -- traversal tables of the hot loop (host side).
//
// FindClosestIntersectionSphere (Collision.hpp:87-109) tests every sphere.  The
// GPU keeps that result exactly but skips spheres that provably cannot pass
// RaySphereIntersection (Collision.hpp:9-17) for any lane of a wave:
//
//  * "always" spheres (large radius: the ground r = 1e6, the three r = 3 balls of
//    GenerateSpheres) are tested for every ray;
//  * the small spheres are sorted along a Morton curve and cut into clusters of
//    k <= 8 members (8 slots each, dummies pad).  Up to 64 clusters form a flat list
//    whose nodes carry a bounding sphere of their members (Cb, Rb >= |Cm - Cb| + r_m);
//    beyond that the clusters are the leaves of a tree built top down by the
//    surface-area heuristic (up to `branching` children per node, spheres regrouped
//    into the leaves it chooses), every tree node carrying an axis-aligned box of all
//    member spheres below it, expanded by kBoxS Bm (Bm = max |C| + r over those
//    members).  The tree is stored in preorder with skip links, so the traversal
//    needs no stack: enter a node (next record) if the ray (wave walk: any lane) may
//    pass, else jump to `skip`.
//
// Cull conditions, derived in DESIGN.md §4.4 from an fp32 error analysis of the
// member test and of the node test for a ray whose computed |d|^2 is within 1e-6
// of 1 (other lanes never cull):
//   flat line: keep iff d2b = |Cb-o|^2 - ((Cb-o).d)^2 <= K1 + 1e-4 |Cb-o|^2,
//          K1 = 1.15 Rb^2 + 1e-5 (rounded up);  derived need 1.0835 Rb^2 + 3.6e-5 |Cb-o|^2
//   tree box: keep iff the ray's line crosses the box grown by kBoxS |o| more (a
//          passing member's centre lies within r + 1.6125e-3 |C - o| of the line),
//          at a parameter >= -1e-6 (|o| + Bs) (a member may lie ahead) and entering it
//          at most sqrt(best) (1 + 1e-5) + 1e-5 (|o| + Bs) along the ray (a member's
//          contact point may beat the lane's winner), Bs = pre_cm >= every Bm
// They use only the containment of the members, so they hold for inner nodes as
// for clusters; nodes failing them for every lane of a wave are skipped with their
// subtree.  Tests run in traversal order, so the closest hit is selected by the
// lexicographic (distance, original index) minimum, which equals the reference's
// strict-'>' first-index-wins scan.  Eight preorder layouts, one per direction
// octant, differ only in sibling order.
#include "spt_accel.h"
#include "spt_internal.h"

#pragma clang fp contract(off)

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <numeric>
#include <thread>
#include <string>

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

float round_down(double x)
{
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
}

// K' of one cluster slot (AccelTables::kpre): c |C|^2 - r^2 (1 + 1e-6) - 4e-6 |C|^2,
// rounded down, with r^2 the slot's float r*r
float pretest_k(const float4 &s)
{
    const double cc = (double)s.x * s.x + (double)s.y * s.y + (double)s.z * s.z;
    return round_down(kFlatScale * cc - (double)s.w * (1.0 + 1e-6) - 4e-6 * cc);
}

const float4 kDummy = make_float4(0.f, 0.f, 0.f, -INFINITY);  // r*r = -inf: never passes

// |C| + |r| of sphere i: Bm of a tree node is the largest over its members
double member_reach(const float *centers4, const float *radii, uint32_t i)
{
    const double x = centers4[4 * i], y = centers4[4 * i + 1], z = centers4[4 * i + 2];
    return std::sqrt(x * x + y * y + z * z) + std::fabs((double)radii[i]);
}

// Bm of the members idx[0..m) (0 when empty)
double node_reach(const float *centers4, const float *radii, const uint32_t *idx, size_t m)
{
    double bm = 0;
    for (size_t j = 0; j < m; ++j) bm = std::max(bm, member_reach(centers4, radii, idx[j]));
    return bm;
}

// Tree node box of the members idx[0..m): lo = min (C - |r|) - kBoxS Bm
// rounded down, hi = max (C + |r|) + kBoxS Bm rounded up.  Members beyond 1e15 from the
// origin: the box is everything (the node never culls).
AccelNode box_node(const float *centers4, const float *radii, const uint32_t *idx, size_t m)
{
    AccelNode nd{};
    const double bm = node_reach(centers4, radii, idx, m);
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t j = 0; j < m; ++j)
        for (int c = 0; c < 3; ++c) {
            const double cc = centers4[4 * idx[j] + c], r = std::fabs((double)radii[idx[j]]);
            lo[c] = std::min(lo[c], cc - r);
            hi[c] = std::max(hi[c], cc + r);
        }
    float flo[3], fhi[3];
    for (int c = 0; c < 3; ++c) {
        const bool off = !(bm <= 1e15);
        flo[c] = off ? -INFINITY : round_down(lo[c] - kBoxS * bm);
        fhi[c] = off ? INFINITY : round_up(hi[c] + kBoxS * bm);
    }
    nd.lox = flo[0];
    nd.loy = flo[1];
    nd.loz = flo[2];
    nd.hix = fhi[0];
    nd.hiy = fhi[1];
    nd.hiz = fhi[2];
    return nd;
}

// the record one past a layout's last node (the kernels prefetch it; never tested)
AccelNode pad_node(uint32_t skip)
{
    AccelNode nd{};
    nd.cx = nd.cy = nd.cz = 0.f;
    nd.k1 = -INFINITY;
    nd.skip = skip;
    nd.slot = kNoSlot;
    nd.rb = -INFINITY;
    nd.cb2 = 0.f;
    return nd;
}

}  // namespace

AccelTables build_accel(const float *centers4, const float *radii, uint32_t n, uint32_t cluster_k, uint32_t group,
                        uint32_t branching, uint32_t leaf_slots)
{
    AccelTables t;
    t.group = group;
    t.leaf_slots = leaf_slots;
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
    // always-list, padded to whole groups
    for (uint32_t i : always) push_slot(i);
    pad_to(group, 0);
    t.always_groups = (uint32_t)(t.slots.size() / group);
    const size_t cbase = t.slots.size();

    if (!small.empty()) {
        const uint32_t k = std::min(cluster_k, leaf_slots);  // members per cluster
        // Morton order of the small spheres' centres
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i : small)
            for (int c = 0; c < 3; ++c) {
                lo[c] = std::min(lo[c], (double)centers4[4 * i + c]);
                hi[c] = std::max(hi[c], (double)centers4[4 * i + c]);
            }
        // one scale for all axes (a cube), so a thin axis does not split clusters
        const double span = std::max({hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]});
        std::vector<std::pair<uint32_t, uint32_t>> keyed;
        for (uint32_t i : small) {
            uint32_t q[3];
            for (int c = 0; c < 3; ++c)
                q[c] = span > 0 ? (uint32_t)std::min(1023.0, (centers4[4 * i + c] - lo[c]) / span * 1023.0) : 0u;
            keyed.push_back({spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2), i});
        }
        std::sort(keyed.begin(), keyed.end());
        std::vector<uint32_t> sorted(keyed.size());
        for (size_t j = 0; j < keyed.size(); ++j) sorted[j] = keyed[j].second;

        // Tree over leaves of k consecutive spheres of `sorted`: node = a contiguous run
        // of leaves [c0, c1) and its children.  Flat lists (branching 0, or at most
        // `branching` leaves): the Morton leaves in slot order.  Trees: built top down,
        // each node's run split into up to `branching` parts by repeated halving of the
        // part with the most leaves (halve: SAH over leaf-aligned cuts; the spheres of a
        // part are reordered so that both halves stay contiguous and leaf boundaries stay
        // at multiples of k).  Config 5: 118 ms per frame against 170 for the bottom-up
        // grouping of consecutive Morton leaves, 114 for median splits.
        const uint32_t leaves = (uint32_t)((sorted.size() + k - 1) / k);
        t.leaves = leaves;
        struct TNode {
            uint32_t c0, c1;
            std::vector<uint32_t> kids;
        };
        std::vector<TNode> tn;
        const bool tree = branching >= 2 && leaves > branching;
        auto sph_end = [&](uint32_t c) { return std::min(sorted.size(), (size_t)c * k); };
        std::vector<uint32_t> top;  // children of the implicit root
        if (!tree) {
            for (uint32_t c = 0; c < leaves; ++c) {
                top.push_back((uint32_t)tn.size());
                tn.push_back({c, c + 1, {}});
            }
        } else {
            // split point (a leaf index) of leaves [c0, c1): the surface-area heuristic
            // over leaf-aligned cuts along each axis (spheres sorted by that centre
            // coordinate): min of area(left) leaves(left) + area(right) leaves(right),
            // areas of the members' boxes; the spheres end up in the chosen axis' order
            auto halve = [&](uint32_t c0, uint32_t c1) {
                const size_t j0 = (size_t)c0 * k, j1 = sph_end(c1);
                {
                    double best = INFINITY;
                    int bax = 0;
                    uint32_t bcut = c0 + (c1 - c0 + 1) / 2;
                    auto area = [](const double *lo, const double *hi) {
                        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
                        return dx * dy + dy * dz + dz * dx;
                    };
                    for (int ax = 0; ax < 3; ++ax) {
                        std::stable_sort(sorted.begin() + j0, sorted.begin() + j1, [&](uint32_t a, uint32_t b) {
                            return centers4[4 * a + ax] < centers4[4 * b + ax];
                        });
                        const uint32_t nl = c1 - c0;
                        std::vector<double> left(nl + 1);  // area of leaves [c0, c0 + q)
                        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                        auto grow = [&](size_t j) {
                            const uint32_t i = sorted[j];
                            const double r = std::fabs((double)radii[i]);
                            for (int c = 0; c < 3; ++c) {
                                lo[c] = std::min(lo[c], (double)centers4[4 * i + c] - r);
                                hi[c] = std::max(hi[c], (double)centers4[4 * i + c] + r);
                            }
                        };
                        for (uint32_t q = 1; q <= nl; ++q) {
                            for (size_t j = (size_t)(c0 + q - 1) * k; j < sph_end(c0 + q); ++j) grow(j);
                            left[q] = area(lo, hi);
                        }
                        std::fill(lo, lo + 3, INFINITY);
                        std::fill(hi, hi + 3, -INFINITY);
                        for (uint32_t q = nl - 1; q >= 1; --q) {
                            for (size_t j = (size_t)(c0 + q) * k; j < sph_end(c0 + q + 1); ++j) grow(j);
                            const double cost = left[q] * q + area(lo, hi) * (nl - q);
                            if (cost < best) {
                                best = cost;
                                bax = ax;
                                bcut = c0 + q;
                            }
                        }
                    }
                    std::stable_sort(sorted.begin() + j0, sorted.begin() + j1, [&](uint32_t a, uint32_t b) {
                        return centers4[4 * a + bax] < centers4[4 * b + bax];
                    });
                    return bcut;
                }
            };
            auto build = [&](auto &&self, uint32_t c0, uint32_t c1) -> uint32_t {
                const uint32_t me = (uint32_t)tn.size();
                tn.push_back({c0, c1, {}});
                if (c1 - c0 <= 1) return me;
                std::vector<std::pair<uint32_t, uint32_t>> parts{{c0, c1}};
                while (parts.size() < branching) {
                    size_t p = 0;
                    for (size_t q = 1; q < parts.size(); ++q)
                        if (parts[q].second - parts[q].first > parts[p].second - parts[p].first) p = q;
                    const auto [a0, a1] = parts[p];
                    if (a1 - a0 <= 1) break;
                    const uint32_t m = halve(a0, a1);
                    parts[p] = {a0, m};
                    parts.insert(parts.begin() + p + 1, {m, a1});
                }
                for (const auto &pr : parts) {
                    const uint32_t kid = self(self, pr.first, pr.second);
                    tn[me].kids.push_back(kid);
                }
                return me;
            };
            const uint32_t root = build(build, 0, leaves);
            top = tn[root].kids;
        }
        // leaves in slot order: k spheres each, leaf_slots slots each
        for (uint32_t c = 0; c < leaves; ++c) {
            for (size_t j = (size_t)c * k; j < sph_end(c + 1); ++j) push_slot(sorted[j]);
            pad_to(leaf_slots, cbase);
        }
        auto depth_of = [&](auto &&self, uint32_t q) -> uint32_t {
            uint32_t dd = 0;
            for (uint32_t kq : tn[q].kids) dd = std::max(dd, self(self, kq));
            return dd + 1;
        };
        t.depth = 0;
        for (uint32_t q : top) t.depth = std::max(t.depth, depth_of(depth_of, q));

        // bounding sphere (flat lists) or expanded box (trees) of the member spheres of
        // leaves [c0, c1); `ctr` = centre of the members' centres (sibling order)
        auto bound = [&](const TNode &sp, AccelNode &nd, double *ctr) {
            const size_t j0 = (size_t)sp.c0 * k, j1 = sph_end(sp.c1);
            double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (size_t j = j0; j < j1; ++j)
                for (int c = 0; c < 3; ++c) {
                    clo[c] = std::min(clo[c], (double)centers4[4 * sorted[j] + c]);
                    chi[c] = std::max(chi[c], (double)centers4[4 * sorted[j] + c]);
                }
            for (int c = 0; c < 3; ++c) ctr[c] = (clo[c] + chi[c]) / 2;
            if (tree) {
                nd = box_node(centers4, radii, sorted.data() + j0, j1 - j0);
                return;
            }
            const float cbf[3] = {(float)ctr[0], (float)ctr[1], (float)ctr[2]};
            double rb = 0;
            for (size_t j = j0; j < j1; ++j) {
                const uint32_t i = sorted[j];
                double d2 = 0;
                for (int c = 0; c < 3; ++c) {
                    const double dd = (double)centers4[4 * i + c] - (double)cbf[c];
                    d2 += dd * dd;
                }
                rb = std::max(rb, std::sqrt(d2) + std::fabs((double)radii[i]));
            }
            rb *= 1.0 + 1e-6;
            nd.cx = cbf[0];
            nd.cy = cbf[1];
            nd.cz = cbf[2];
            const float rbf = round_up(rb);
            nd.k1 = round_up(1.15 * (double)rbf * (double)rbf + 1e-5);
            // expanded line test (spt_path.h find_closest): K1'' = K1 +
            // 4e-6 |Cb|^2 - c |Cb|^2 -- the kernel leaves c |Cb|^2 out of the per-lane sum
            // and compares against K1'' instead (one add fewer)
            const double cbb = (double)nd.cx * nd.cx + (double)nd.cy * nd.cy + (double)nd.cz * nd.cz;
            nd.cb2 = (float)(kFlatScale * cbb);
            nd.rb = round_up((double)nd.k1 + 4e-6 * cbb - (double)nd.cb2);
        };
        // Preorder emission, once per direction octant: siblings are ordered front to
        // back along the octant's diagonal, so a wave walking the layout of its
        // majority octant finds near hits first and the distance test culls more.
        // The top level sits under an implicit root (never tested).
        std::vector<AccelNode> bounds(tn.size());
        std::vector<std::array<double, 3>> ctrs(tn.size());
        for (size_t q = 0; q < tn.size(); ++q) bound(tn[q], bounds[q], ctrs[q].data());
        for (uint32_t oct = 0; oct < 8; ++oct) {
            const double sx = (oct & 1) ? -1.0 : 1.0, sy = (oct & 2) ? -1.0 : 1.0, sz = (oct & 4) ? -1.0 : 1.0;
            const size_t base = t.nodes.size();
            auto ordered = [&](const std::vector<uint32_t> &kids) {
                std::vector<uint32_t> ix = kids;
                if (!tree) return ix;  // flat list: slot order (the kernel relies on it)
                std::stable_sort(ix.begin(), ix.end(), [&](uint32_t a, uint32_t b) {
                    const std::array<double, 3> &ca = ctrs[a], &cb = ctrs[b];
                    return sx * ca[0] + sy * ca[1] + sz * ca[2] < sx * cb[0] + sy * cb[1] + sz * cb[2];
                });
                return ix;
            };
            auto emit = [&](auto &&self, uint32_t q) -> void {
                const size_t me = t.nodes.size();
                t.nodes.push_back(bounds[q]);
                if (tn[q].kids.empty()) {
                    t.nodes[me].slot = (uint32_t)(cbase + (size_t)tn[q].c0 * leaf_slots);
                } else {
                    t.nodes[me].slot = kNoSlot;
                    for (uint32_t kq : ordered(tn[q].kids)) self(self, kq);
                }
                t.nodes[me].skip = (uint32_t)(t.nodes.size() - base);
            };
            for (uint32_t q : ordered(top)) emit(emit, q);
            if (oct == 0) t.n_nodes = (uint32_t)t.nodes.size();
            // pad node (the kernel prefetches one node past the layout)
            t.nodes.push_back(pad_node(t.n_nodes + 1));
        }
    }
    // the kernel prefetches one always-group past the list and one node past the tree
    for (uint32_t j = 0; j < 2 * group; ++j) {
        t.slots.push_back(kDummy);
        t.orig.push_back(0xFFFFFFFFu);
    }
    if (t.nodes.empty())  // no tree: one pad record per octant layout (n_nodes = 0)
        for (int oct = 0; oct < 8; ++oct) t.nodes.push_back(pad_node(1));
    // member pretest constants of the cluster slots (dummies: K' = +inf never passes)
    t.kpre.assign(t.slots.size(), 0.f);
    double cm = 0;
    for (size_t j = cbase; j < t.slots.size(); ++j) {
        if (t.orig[j] == 0xFFFFFFFFu) {
            t.kpre[j] = INFINITY;
            continue;
        }
        const float4 &q = t.slots[j];
        t.kpre[j] = pretest_k(q);
        // over the slot's r*r (the pretest) and the sphere's |r| (tree boxes' Bm)
        cm = std::max({cm,
                       std::sqrt((double)q.x * q.x + (double)q.y * q.y + (double)q.z * q.z) + std::sqrt((double)q.w),
                       member_reach(centers4, radii, t.orig[j])});
    }
    t.pre_cm = round_up(cm * (1.0 + 1e-9));
    if (!(cm <= 1e15)) {
        // squares near the float range: the pretest passes every lane (K' = -inf)
        t.pre_cm = INFINITY;
        for (size_t j = cbase; j < t.slots.size(); ++j)
            if (t.orig[j] != 0xFFFFFFFFu) t.kpre[j] = -INFINITY;
    }
    return t;
}

std::string validate_accel(const AccelTables &t, const float *centers4, const float *radii, uint32_t n)
{
    char buf[256];
    auto bad = [&](const char *fmt, auto... a) {
        if constexpr (sizeof...(a) == 0)
            std::snprintf(buf, sizeof buf, "%s", fmt);
        else
            std::snprintf(buf, sizeof buf, fmt, a...);
        return std::string(buf);
    };
    const size_t g = t.group, cbase = (size_t)t.always_groups * g;
    if (t.slots.size() != t.orig.size()) return bad("slots/orig size mismatch");
    if (t.leaf_slots != kClusterSlots && !(t.leaf_slots == kFlatLeafSlots && t.n_nodes == t.leaves))
        return bad("leaf width %u needs a flat list", t.leaf_slots);
    if (t.slots.size() < cbase + 2 * g) return bad("slot table lacks the prefetch pad");
    if (t.nodes.size() != 8 * ((size_t)t.n_nodes + 1)) return bad("node table is not 8 layouts of %u + 1", t.n_nodes);
    // every sphere exactly once
    std::vector<int> seen(n, 0);
    for (size_t j = 0; j < t.slots.size(); ++j) {
        const uint32_t o = t.orig[j];
        if (o == 0xFFFFFFFFu) {
            if (!(t.slots[j].w == -INFINITY)) return bad("dummy slot %zu can pass", j);
            continue;
        }
        if (o >= n || seen[o]++) return bad("slot %zu: sphere %u out of range or repeated", j, o);
    }
    for (uint32_t i = 0; i < n; ++i)
        if (!seen[i]) return bad("sphere %u missing from the slot table", i);
    // member pretest constants (cluster slots)
    if (t.kpre.size() != t.slots.size()) return bad("pretest table size mismatch");
    for (size_t j = cbase; j < t.slots.size(); ++j) {
        const float4 &q = t.slots[j];
        if (t.orig[j] == 0xFFFFFFFFu) {
            if (!(t.kpre[j] == INFINITY)) return bad("dummy slot %zu: pretest can pass", j);
            continue;
        }
        if (t.pre_cm == INFINITY) {
            if (!(t.kpre[j] == -INFINITY)) return bad("slot %zu: pretest not disabled", j);
            continue;
        }
        if (!(t.kpre[j] == pretest_k(q))) return bad("slot %zu: pretest K' wrong", j);
        const double cl = std::sqrt((double)q.x * q.x + (double)q.y * q.y + (double)q.z * q.z);
        if (!((double)t.pre_cm >= cl + std::sqrt((double)q.w))) return bad("slot %zu: outside the pretest bound", j);
    }
    for (uint32_t oct = 0; oct < 8; ++oct) {
        const AccelNode *L = t.nodes.data() + (size_t)oct * (t.n_nodes + 1);
        if (!(L[t.n_nodes].k1 == -INFINITY) || L[t.n_nodes].slot != kNoSlot) return bad("layout %u: bad pad", oct);
        size_t leaves = 0;
        for (uint32_t i = 0; i < t.n_nodes; ++i) {
            const AccelNode &nd = L[i];
            const bool leaf = nd.slot != kNoSlot;
            if (nd.skip <= i || nd.skip > t.n_nodes || (leaf && nd.skip != i + 1) || (!leaf && nd.skip == i + 1))
                return bad("layout %u node %u: skip %u breaks preorder", oct, i, nd.skip);
            if (leaf) {
                ++leaves;
                if (nd.slot < cbase || (nd.slot - cbase) % t.leaf_slots || nd.slot + t.leaf_slots > t.slots.size())
                    return bad("layout %u node %u: leaf slot %u out of range", oct, i, nd.slot);
            }
            // containment of every member below.  Flat lists (Rb = max |Cm - Cb| + r over the
            // members): Rb <= sqrt((K1 - 1e-5) / 1.15), K1'' >= K1 + 4e-6 |Cb|^2 - cb2 and
            // cb2 = c |Cb|^2.  Trees: lo <= C - |r| - kBoxS Bm and hi >= C + |r| + kBoxS Bm on
            // every axis, Bm = max |C| + |r| over the members (box_node's arithmetic)
            const bool flat = t.n_nodes == t.leaves;
            std::vector<uint32_t> below;
            for (uint32_t q = i; q < nd.skip; ++q) {
                if (L[q].slot == kNoSlot) continue;
                for (uint32_t k = 0; k < t.leaf_slots; ++k)
                    if (t.orig[L[q].slot + k] != 0xFFFFFFFFu) below.push_back(t.orig[L[q].slot + k]);
            }
            if (!flat) {
                const double bm = node_reach(centers4, radii, below.data(), below.size());
                const bool off = !(bm <= 1e15);
                const float blo[3] = {nd.lox, nd.loy, nd.loz}, bhi[3] = {nd.hix, nd.hiy, nd.hiz};
                for (uint32_t o : below)
                    for (int c = 0; c < 3; ++c) {
                        const double cc = centers4[4 * o + c], r = std::fabs((double)radii[o]);
                        const bool in = off ? (blo[c] == -INFINITY && bhi[c] == INFINITY)
                                            : ((double)blo[c] <= (cc - r) - kBoxS * bm &&
                                               (double)bhi[c] >= (cc + r) + kBoxS * bm);
                        if (!in) return bad("layout %u node %u: sphere %u outside the expanded box", oct, i, o);
                    }
                if (!(t.pre_cm >= bm || t.pre_cm == INFINITY))
                    return bad("layout %u node %u: Bm above the scene bound", oct, i);
                continue;
            }
            const double cbb = (double)nd.cx * nd.cx + (double)nd.cy * nd.cy + (double)nd.cz * nd.cz;
            if (!(std::fabs((double)nd.cb2 - kFlatScale * cbb) <= 2e-7 * cbb &&
                  (double)nd.rb >= (double)nd.k1 + 4e-6 * cbb - (double)nd.cb2))
                return bad("layout %u node %u: flat-list |Cb|^2 or K1' wrong", oct, i);
            double rbm = 0;
            for (uint32_t o : below) {
                double d2 = 0;
                const double cb[3] = {nd.cx, nd.cy, nd.cz};
                for (int c = 0; c < 3; ++c) {
                    const double dd = (double)centers4[4 * o + c] - cb[c];
                    d2 += dd * dd;
                }
                rbm = std::max(rbm, std::sqrt(d2) + std::fabs((double)radii[o]));
            }
            if (!((double)nd.k1 >= 1.15 * rbm * rbm + 1e-5))
                return bad("layout %u node %u: a member lies outside the K1 bound", oct, i);
        }
        if (leaves != t.leaves) return bad("layout %u: %zu leaves, expected %u", oct, leaves, t.leaves);
        if (t.n_nodes == t.leaves)  // flat list: node i is leaf i, in slot order
            for (uint32_t i = 0; i < t.n_nodes; ++i)
                if (L[i].slot != cbase + (size_t)i * t.leaf_slots) return bad("flat layout %u not in slot order", oct);
    }
    return std::string();
}

// ---- primary-ray candidate lists (PrimLists) ---------------------
//
// A primary ray of pixel (x, y) (start_path, SingleThreadPathTracer.hpp:123-130) leaves the
// eye along d = normalize(M (vx, vy, 1, 0)), vx = -1 + 2 (x + U) / H, vy = -1 + 2 (y + U') / W
// with jitters U, U' in [-1, 1) (the reference divides the row coordinate by g_width and
// the column coordinate by g_height; the kernel follows).  Over a pixel block the exact
// (vx, vy) fill a rectangle, so the exact directions fill the cone over a quadrilateral:
// with `a` the direction of the rectangle's centre, every direction of the block lies
// within theta = max over the four corners of angle(a, corner) of a (the angle from a is
// a monotone function of the distance from a's point in the gnomonic projection onto the
// plane normal to a, where the quadrilateral stays convex: its maximum is at a vertex).
// The kernel's fp direction deviates from the exact one by at most delta (its rounding
// of the rectangle coordinates is inside the rectangle's slack; the matrix product and
// the normalisation add <= 8u |M| / |Md| + 6u, u = 2^-24).
//
// The member test of sphere (C, r) passes only if the computed d2 < r^2 - 1e-3 and tc >
// 1e-3; d2 is at least p^2 - eps X^2 with p the exact distance of C from the line through
// the eye along the computed d, X = |C - eye| and eps = 2.6e-6 (for
// | |d| - 1 | <= 6e-7, true of a normalised primary direction), and tc > 1e-3 puts C
// within 90 deg + 3e-7 rad of d.  So a passing member has angle(d, C - eye) < asin(R / X),
// R = sqrt(r^2 + eps X^2), and the sphere can be dropped from the block's list when
//     angle(a, C - eye) > theta + asin(R / X) + delta
// (triangle inequality on the sphere of directions).  R gets 0.1% + 1e-4 and the angles
// 1e-6 rad of extra slack; spheres with X <= R (the eye at or inside their reach),
// non-finite values, and every block of a camera that is not finite (or whose block
// cones exceed 0.5 rad) keep the tree walk.  The closest hit of a primary ray is then in
// its block's list, and the list cast's (distance, original index) minimum over the list
// is the reference's winner over all spheres.  tests/test_abi.py checks every winner of
// 4 096 sampled primary rays per scene against the lists (oracle rays, CPU);
// tests/test_gpu_parity.py renders with and without the lists, bit for bit.
namespace {

struct PrimCone {
    double a[3];
    double theta, delta;
    bool ok;
};

constexpr double kU = 1.0 / 16777216.0;  // 2^-24

double norm3(const double v[3]) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// angle between unit a and v (any length), robust near 0 and pi
double angle_to(const double a[3], const double v[3])
{
    const double cx = a[1] * v[2] - a[2] * v[1], cy = a[2] * v[0] - a[0] * v[2], cz = a[0] * v[1] - a[1] * v[0];
    const double s = std::sqrt(cx * cx + cy * cy + cz * cz), c = a[0] * v[0] + a[1] * v[1] + a[2] * v[2];
    return std::atan2(s, c);
}

// Cone of the primary rays of pixel columns [x0, x1), rows [y0, y1).
PrimCone prim_cone(const Camera &cam, uint32_t W, uint32_t H, uint32_t x0, uint32_t x1, uint32_t y0, uint32_t y1)
{
    PrimCone pc{};
    // jittered row / column coordinates un = y + U, vn = x + U' (U in [-1, 1)), widened by
    // their fp rounding, then u = un / W, v = vn / H (correctly rounded), vy = -1 + 2u,
    // vx = -1 + 2v, each widened by its rounding
    auto widen = [](double lo, double hi, double rel, double abs_) {
        const double m = std::max(std::fabs(lo), std::fabs(hi));
        return std::pair<double, double>(lo - m * rel - abs_, hi + m * rel + abs_);
    };
    auto un = widen((double)y0 - 1.0, (double)y1, 4 * kU, 1e-6);
    auto vn = widen((double)x0 - 1.0, (double)x1, 4 * kU, 1e-6);
    auto u = widen(un.first / (double)W, un.second / (double)W, 4 * kU, 1e-12);
    auto v = widen(vn.first / (double)H, vn.second / (double)H, 4 * kU, 1e-12);
    auto vy = widen(-1.0 + 2.0 * u.first, -1.0 + 2.0 * u.second, 4 * kU, 1e-7);
    auto vx = widen(-1.0 + 2.0 * v.first, -1.0 + 2.0 * v.second, 4 * kU, 1e-7);
    const float *m = cam.view;
    auto dir = [&](double px, double py, double out[3], double &mag) {
        mag = 0;
        for (int r = 0; r < 3; ++r) {
            const double t0 = (double)m[4 * r] * px, t1 = (double)m[4 * r + 1] * py, t2 = (double)m[4 * r + 2];
            out[r] = t0 + t1 + t2;
            mag += std::fabs(t0) + std::fabs(t1) + std::fabs(t2);
        }
    };
    double c[3], cm;
    dir(0.5 * (vx.first + vx.second), 0.5 * (vy.first + vy.second), c, cm);
    const double cl = norm3(c);
    if (!(cl > 0) || !std::isfinite(cl)) return pc;
    for (int k = 0; k < 3; ++k) pc.a[k] = c[k] / cl;
    double theta = 0, smax = cm, amin = 1e300;
    for (int k = 0; k < 4; ++k) {
        double d[3], dm;
        dir(k & 1 ? vx.second : vx.first, k & 2 ? vy.second : vy.first, d, dm);
        const double along = pc.a[0] * d[0] + pc.a[1] * d[1] + pc.a[2] * d[2];
        if (!(along > 0) || !std::isfinite(along)) return pc;
        theta = std::max(theta, angle_to(pc.a, d));
        smax = std::max(smax, dm);
        amin = std::min(amin, along);
    }
    if (!(theta < 0.5)) return pc;
    pc.theta = theta;
    pc.delta = 8 * kU * smax / amin + 6 * kU + 1e-6;
    pc.ok = std::isfinite(pc.delta) && pc.delta < 1e-3;
    return pc;
}

// Can a primary ray of cone pc pass the member test of slot s (eye e)?
bool prim_candidate(const PrimCone &pc, const float4 &sl, const double e[3])
{
    if (sl.w == -INFINITY) return false;  // dummy slot: never passes
    const double c[3] = {(double)sl.x - e[0], (double)sl.y - e[1], (double)sl.z - e[2]};
    const double L = norm3(c), r2 = (double)sl.w;
    if (!std::isfinite(L) || !std::isfinite(r2)) return true;
    const double R = std::sqrt(std::max(r2 + 2.6e-6 * L * L, 0.0)) * 1.001 + 1e-4;
    if (!(L > R * 1.01 + 1e-3)) return true;
    const double alpha = std::asin(std::min(1.0, R / L));
    return angle_to(pc.a, c) <= pc.theta + alpha + pc.delta + 1e-6;
}

}  // namespace

PrimListTables build_prim_lists(const AccelTables &t, const Camera &cam, uint32_t W, uint32_t H, uint32_t max_count)
{
    const auto t_start = std::chrono::steady_clock::now();
    PrimListTables out;
    // the device packs a batch lane's pixel as (y << 16 | x) (spt_path.h prim_list_cast):
    // frames of 65 536 or more columns or rows walk the tree
    if (W == 0 || H == 0 || W > 0xFFFFu || H > 0xFFFFu) return out;
    out.bw = (W + 7) / 8;
    const uint32_t bh8 = (H + 7) / 8, bh4 = (H + 3) / 4;
    out.b8.assign((size_t)out.bw * bh8, make_uint2(0, kPrimWalk));
    out.b4.assign((size_t)out.bw * bh4, make_uint2(0, kPrimWalk));
    bool finite = true;
    for (int i = 0; i < 12; ++i) finite = finite && std::isfinite(cam.view[i]);
    double e[3];
    for (int i = 0; i < 3; ++i) {
        e[i] = cam.eye[i];
        finite = finite && std::isfinite(cam.eye[i]) && std::fabs(cam.eye[i]) < 1e15;
    }
    if (!finite || t.slots.empty()) {
        out.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
        return out;
    }
    // a dummy slot (r*r = -inf) to pad the runs with; the tables end with pad slots
    uint32_t pad = kPrimWalk;
    for (size_t s = t.slots.size(); s-- > 0;)
        if (t.slots[s].w == -INFINITY) {
            pad = (uint32_t)s;
            break;
        }
    if (pad == kPrimWalk) return out;
    std::vector<uint32_t> all(t.slots.size());
    std::iota(all.begin(), all.end(), 0u);
    // super-blocks of 64 x 64 pixels first: a slot culled for a super-block's cone is
    // culled for every block inside it (its rectangle holds theirs).  Super-blocks are
    // independent: host threads build their lists, concatenated in super-block order (the
    // tables are the same as one thread's)
    struct Sup {
        uint32_t sx, sy;
        std::vector<std::pair<uint32_t, uint2>> runs;  // (level << 31 | block, {offset in slots, count})
        std::vector<uint32_t> slots;
    };
    std::vector<Sup> sups;
    for (uint32_t sy = 0; sy < H; sy += 64)
        for (uint32_t sx = 0; sx < W; sx += 64) sups.push_back(Sup{sx, sy, {}, {}});
    auto work = [&](size_t first, size_t step) {
        std::vector<uint32_t> sup, cand;
        for (size_t q = first; q < sups.size(); q += step) {
            Sup &S = sups[q];
            const uint32_t sx = S.sx, sy = S.sy;
            const PrimCone sc = prim_cone(cam, W, H, sx, std::min(W, sx + 64), sy, std::min(H, sy + 64));
            sup.clear();
            for (uint32_t s : all)
                if (!sc.ok || prim_candidate(sc, t.slots[s], e)) sup.push_back(s);
            for (uint32_t level = 0; level < 2; ++level) {
                const uint32_t bhgt = level == 0 ? 8u : 4u;
                for (uint32_t y = sy; y < std::min(H, sy + 64); y += bhgt)
                    for (uint32_t x = sx; x < std::min(W, sx + 64); x += 8) {
                        const PrimCone pc = prim_cone(cam, W, H, x, std::min(W, x + 8), y, std::min(H, y + bhgt));
                        if (!pc.ok) continue;  // walk
                        cand.clear();
                        for (uint32_t s : sup)
                            if (prim_candidate(pc, t.slots[s], e)) cand.push_back(s);
                        if (cand.size() > max_count) continue;  // walk
                        // runs of whole groups of 4 (the kernel loads 4 entries at a time),
                        // padded with a dummy slot (never passes)
                        while (cand.size() % 4) cand.push_back(pad);
                        const uint32_t blk = (y / bhgt) * out.bw + x / 8;
                        S.runs.push_back({level << 31 | blk, make_uint2((uint32_t)S.slots.size(), (uint32_t)cand.size())});
                        S.slots.insert(S.slots.end(), cand.begin(), cand.end());
                    }
            }
        }
    };
    const size_t work_units = sups.size() * t.slots.size();
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    // config 2 (247 super-blocks x 160 slots) took 7.5 ms on one thread: threads from 2^14
    // work units (a thread's start costs ~50 us)
    size_t nth = work_units < (1u << 14) ? 1 : std::min<size_t>({(size_t)hw, (size_t)16, sups.size()});
    if (const char *ev = std::getenv("SPT_PRIM_THREADS"))  // tests: one thread vs many give the same tables
        if (*ev) nth = std::max(1, std::atoi(ev));
    if (nth <= 1) {
        work(0, 1);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 0; k < nth; ++k) th.emplace_back(work, k, nth);
        for (std::thread &x : th) x.join();
    }
    for (const Sup &S : sups) {
        const uint32_t base = (uint32_t)out.slots.size();
        for (const auto &r : S.runs) {
            std::vector<uint2> &dst = (r.first >> 31) == 0 ? out.b8 : out.b4;
            dst[r.first & 0x7FFFFFFFu] = make_uint2(base + r.second.x, r.second.y);
        }
        out.slots.insert(out.slots.end(), S.slots.begin(), S.slots.end());
    }
    if (out.slots.empty()) out.slots.assign(4, pad);  // a valid pointer for the device copy
    out.on = true;
    out.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    return out;
}

}  // namespace spt
