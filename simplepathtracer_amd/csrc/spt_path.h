// spt_path.h -- per-path device code shared by the render kernels: the cast
// (FindClosestIntersectionSphere with exact culling), the
// shading step of the flattened recursion, the cooperative cube-minus-ball
// sampler and the primary-ray generator.  Included by spt_kernels.hip (the
// persistent megakernel) and spt_wavefront.hip (the queue-based variant), so
// both compute every path with the same instructions.
#pragma once
#include "spt_device.h"
#include "spt_internal.h"

#include <float.h>

#ifndef SPT_GROUP
#define SPT_GROUP 4
#endif

#ifndef SPT_DIAG
#define SPT_DIAG 0
#endif
#ifndef SPT_LEAF_SPLIT
#define SPT_LEAF_SPLIT 1
#endif
// Attribution builds only (tools/attrib.sh, never the product library): SPT_DUP runs one
// phase a second time on opaque copies of its inputs and discards the result, so the
// difference in SQ_INSTS_VALU per launch against the product build is that phase's
// instruction count.  Bits: 1 the whole cast, 2 the cooperative sampler, 4 the primary
// ray (start_path), 8 the tree node test, 16 the member tests + updates of entered leaves,
// 32 the always-tested group, 64 the primary batches' candidate-list casts, 128 the
// shading step less the sampler, 256 the refraction event, 512 the lane walk (lane_cast).
#ifndef SPT_DUP
#define SPT_DUP 0
#endif
// the cube-minus-ball sampler skips its one-trial-per-lane round 0 when at most 32 lanes
// need a vector (coop_ball_vector)
#ifndef SPT_SAMPLER_SKIP0
#define SPT_SAMPLER_SKIP0 1
#endif
// wave walk: leaves entered by at most 8 lanes are tested as dealt (lane, member) pairs
// (test_leaf_pairs); 2: also those entered by 9-16 lanes, two members per lane
#ifndef SPT_LEAF_PAIRS
#define SPT_LEAF_PAIRS 2
#endif

// Item order of a batch: [band][8x8 tile][sample][pixel] (ts_item, spt_internal.h)

#pragma clang fp contract(off)

namespace spt {
namespace {

constexpr uint32_t PH_IDLE = 0, PH_TRACE = 1, PH_DLOOP = 2;

// rSq of SampleColorRefractive (lines 58 and 75): powf(-0.2f, 2.f) = powf(0.2f, 2.f)
// = 0x1.47ae16p-5, the correctly rounded square (glibc's powf agrees:
// tests/cpp/kat_powf.cpp; selftest column 4 checks spt_glibc_powf on the device).
constexpr float kRsq = ((1.0f - 1.5f) / (1.0f + 1.5f)) * ((1.0f - 1.5f) / (1.0f + 1.5f));
static_assert(kRsq == 0x1.47ae16p-5f, "rSq");
constexpr float kAirToGlass = 1.0f / 1.5f;
constexpr float kGlassToAir = 1.5f / 1.0f;

// Tables as constant-address-space data: wave-uniform indices become scalar
// (s_load) reads even though the kernel also stores to global memory.
typedef __attribute__((address_space(4))) const float cfloat;
typedef __attribute__((address_space(4))) const uint32_t cuint;

__device__ __forceinline__ float4 ld_uniform(cfloat *p, uint32_t i)
{
    return make_float4(p[4 * i + 0], p[4 * i + 1], p[4 * i + 2], p[4 * i + 3]);
}

// v_min/max(3)_f32 without the compiler's IEEE-mode canonicalisation of operands it
// cannot prove canonical (loop-carried or negated values: one v_max_f32 x, x each per
// use).  No operand here is a signalling NaN, so the raw instructions give the same
// result as fminf/fmaxf.
__device__ __forceinline__ float max_raw(float a, float b)
{
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float min_raw(float a, float b)
{
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float max3_raw(float a, float b, float c)
{
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float min3_raw(float a, float b, float c)
{
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ uint32_t lane_rank(unsigned long long mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <class T>
__device__ __forceinline__ T opaque_v(T x)
{
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ f3 opaque_v3(f3 a) { return mk(opaque_v(a.x), opaque_v(a.y), opaque_v(a.z)); }
template <class T>
__device__ __forceinline__ void sink_v(T x)
{
    asm volatile("" ::"v"(x));
}

// Closest-hit state of one FindClosestIntersectionSphere call.
struct Hit {
    uint32_t idx;        // slot of the winner (traversal order), kMiss = none
    float best;          // its squared distance
    float t;             // its contact parameter: contact point o + d t (contact())
};

// CalculateRaySphereClosestContactPoint's point o + d t (Collision.hpp:49-56), in the
// reference's operation order; recomputed after the cast from the winner's t (two
// VGPRs fewer in the traversal than carrying the point), bit-identical
__device__ __forceinline__ f3 contact(const f3 &o, const f3 &d, float t)
{
    return mk(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t);
}

// Wave-diagnostic counters of the SPT_DIAG build.
struct CastDiag {
    unsigned long long nodes = 0, leaves = 0, pairs = 0, live = 0;
    unsigned long long spheres = 0, branches = 0, passing = 0, improving = 0;
    // lane-level work: RaySphereIntersection evaluations (17 FLOP each) and
    // member pretests (10 VALU each) for the wave's live lanes
    unsigned long long lane_tests = 0, lane_pretests = 0;
    unsigned long long leaves8 = 0, leaves16 = 0;  // tree leaves entered by <= 8 / <= 16 lanes
    uint32_t live_now = 0;  // live lanes of the current cast
};

// The closest-contact / distance update of one member (Collision.hpp:19-27,49-56,
// 87-109) for the lanes that pass RaySphereIntersection (wave mask `pm`, with their tc and
// hh); called in wave-uniform control flow when some lane passes.  Slots are
// visited in traversal order, so the winner is the lexicographic minimum of
// (distance, original index): identical to the reference's strict-'>' scan in
// index order (first index wins ties; NaN and FLT_MAX distances never win).
__device__ __forceinline__ void update_member(unsigned long long pm, float tc, float hh,
                                              const uint32_t *__restrict__ orig, uint32_t s, const f3 &o, const f3 &d,
                                              float dod, Hit &h, CastDiag &dg)
{
    // CalculateRaySphereClosestContactPoint, Collision.hpp:19-27,49-56
    const float t = tc - sqrt_pos_normal(hh);
    const f3 p = contact(o, d, t);
    const float ds = lensq(sub(o, p));
    // wave masks (ballots of the compares themselves; a bool kept across the tie
    // branch would round-trip through a VGPR): `pm` = the lanes that pass
    // RaySphereIntersection, ok = those whose contact point lies ahead
    const unsigned long long ok = pm & __ballot(dod < dot(p, d));
    unsigned long long bm = ok & __ballot(ds < h.best);
    // exact tie (rare): the first original index wins.  Scalar loads only (one per
    // distinct current winner): a vector load here made every cast wait on vmcnt(0),
    // i.e. on the previous shading step's sample stores.
    unsigned long long tm = ok & __ballot(ds == h.best) & __ballot(h.idx != kMiss);
    if (__builtin_expect(tm != 0ull, 0)) {
        const uint32_t mo = ((cuint *)orig)[s];
        while (tm != 0ull) {
            const uint32_t wi = __builtin_amdgcn_readlane(h.idx, (int)__builtin_ctzll(tm));
            const uint32_t wo = ((cuint *)orig)[wi];
            const unsigned long long same = tm & __ballot(h.idx == wi);
            if (mo < wo) bm |= same;
            tm &= ~same;
        }
    }
    if (SPT_DIAG) dg.improving += bm != 0ull ? 1 : 0;
    const bool better = __builtin_amdgcn_inverse_ballot_w64(bm);
    h.best = better ? ds : h.best;
    h.idx = better ? s : h.idx;
    h.t = better ? t : h.t;
}

// RaySphereIntersection, Collision.hpp:9-17, in the reference's operation order:
// tc and hh = r*r - d2; the lane passes iff tc > 1e-3 && hh > 1e-3.
__device__ __forceinline__ bool ray_sphere(const float4 &sp, const f3 &o, const f3 &d, float &tc, float &hh)
{
    const float ocx = sp.x - o.x, ocy = sp.y - o.y, ocz = sp.z - o.z;
    tc = (ocx * d.x + ocy * d.y) + ocz * d.z;
    const float d2 = ((ocx * ocx + ocy * ocy) + ocz * ocz) - tc * tc;
    hh = sp.w - d2;
    // tc > 1e-3 && hh > 1e-3 as one compare (VALU, not a scalar AND of two masks).
    // A NaN operand can make it true where the pair is false; such a lane's
    // contact point is NaN and the dot test of update_member rejects it.
    return __builtin_fminf(tc, hh) > 1e-3f;
}

// One group of G slots {C, r*r}: RaySphereIntersection for all of them, then the
// rare update behind one wave-uniform branch per member (the scalar unit is
// shared by the CU's four SIMDs).
template <int G>
__device__ __forceinline__ void test_group(const float4 (&sp)[G], const uint32_t *__restrict__ orig, uint32_t slot,
                                           const f3 &o, const f3 &d, float dod, Hit &h, CastDiag &dg)
{
    float tcv[G], hv[G];
    bool pass[G];
#pragma unroll
    for (int k = 0; k < G; ++k) pass[k] = ray_sphere(sp[k], o, d, tcv[k], hv[k]);
    if (SPT_DIAG) dg.lane_tests += (unsigned long long)G * dg.live_now;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        if (SPT_DIAG) {
            dg.spheres += 1;
            dg.branches += __ballot(pass[k]) != 0ull ? 1 : 0;
            dg.passing += (unsigned long long)__popcll(__ballot(pass[k]));
        }
        // the update takes the pass mask (a bool kept across the branch would be rebuilt
        // from a VGPR copy: 2 VALU per update)
        const unsigned long long pmk = __ballot(pass[k]);
        if (pmk != 0ull)
            update_member(pmk, tcv[k], hv[k], orig, slot + k, o, d, dod, h, dg);
    }
}

// Per-lane terms of the member pretest (test_group_pre), formed once per cast.
struct PreLane {
    float osx, osy, osz;  // -2c o (c = kFlatScale, as the flat node test)
    float qoe;            // (c - 4.1e-6) |o|^2; +inf for inactive lanes, -inf for lanes that must not cull
    float tinit;          // mt - o.d, mt = 2e-6 (pre_cm + |o|) + 1e-6; -inf inactive, +inf must not cull
};

// A group of cluster members behind a cheaper conservative pretest (10 VALU per
// member instead of 18): with tcs = C.d - o.d + mt and
//   w = c |C|^2 - r^2 (1 + 1e-6) - 4e-6 |C|^2 - 2c C.o + (c - 4.1e-6) |o|^2
// (K' = the first three terms, stored per slot), a lane may pass the member only
// if min(tcs, tcs^2 - w) > 1e-3 (every lane that passes the
// reference test passes this one).  The exact test runs only behind the member's
// wave-uniform branch.  Flat lists only: on tree leaves (config 5) it measured 10%
// slower -- the tree walk, not the member tests, bounds that kernel.
template <int G>
__device__ __forceinline__ void test_group_pre(const float4 (&sp)[G], const float (&kp)[G],
                                               const uint32_t *__restrict__ orig, uint32_t slot, const f3 &o,
                                               const f3 &d, float dod, const PreLane &pl, Hit &h, CastDiag &dg)
{
    bool pre[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const float tcs = __builtin_fmaf(sp[k].x, d.x, __builtin_fmaf(sp[k].y, d.y, __builtin_fmaf(sp[k].z, d.z, pl.tinit)));
        const float w =
            __builtin_fmaf(sp[k].x, pl.osx, __builtin_fmaf(sp[k].y, pl.osy, __builtin_fmaf(sp[k].z, pl.osz, pl.qoe))) + kp[k];
        pre[k] = __builtin_fminf(tcs, __builtin_fmaf(tcs, tcs, -w)) > 1e-3f;
    }
    // all G pretests before the first branch (independent chains in flight
    // together), and one branch past the group when no lane passes any member
    unsigned long long pm[G], any = 0ull;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        pm[k] = __ballot(pre[k]);
        any |= pm[k];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (SPT_DIAG) dg.lane_pretests += (unsigned long long)G * dg.live_now;
    if (any == 0ull) {
        if (SPT_DIAG) dg.spheres += G;
        return;
    }
#pragma unroll
    for (int k = 0; k < G; ++k) {
        if (SPT_DIAG) {
            dg.spheres += 1;
            dg.branches += __ballot(pre[k]) != 0ull ? 1 : 0;
            dg.passing += (unsigned long long)__popcll(__ballot(pre[k]));
        }
        if (pm[k] != 0ull) {
            float tc, hh;
            const bool pass = ray_sphere(sp[k], o, d, tc, hh);
            if (SPT_DIAG) dg.lane_tests += dg.live_now;
            const unsigned long long pmk = __ballot(pass);
            if (pmk != 0ull)
                update_member(pmk, tc, hh, orig, slot + k, o, d, dod, h, dg);
        }
    }
}

// Leaf test: the cluster's S slots (S = 8: two s_load_dwordx16, S = 4: one) off one
// base pointer.
template <int S>
__device__ __forceinline__ void test_leaf(cfloat *slots, const uint32_t *__restrict__ orig, uint32_t leaf_slot,
                                          const f3 &o, const f3 &d, float dod, Hit &h, CastDiag &dg)
{
    cfloat *cs = slots + 4 * leaf_slot;
#if SPT_LEAF_SPLIT
    // SPT_LEAF_SPLIT: the members in groups of four (16 SGPRs at a time instead of 32;
    // SGPR spills 22 -> 13; config 2 5.61 -> 5.57 ms, a config-3 sample 7.20 -> 7.05 ms)
#pragma unroll
    for (int g = 0; g < S; g += 4) {
        float4 ms[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) ms[k] = ld_uniform(cs, g + k);
        test_group<4>(ms, orig, leaf_slot + g, o, d, dod, h, dg);
    }
#else
    float4 ms[S];
#pragma unroll
    for (int k = 0; k < S; ++k) ms[k] = ld_uniform(cs, k);
    test_group<S>(ms, orig, leaf_slot, o, d, dod, h, dg);
#endif
}

// Leaf test for a leaf that few lanes need (the wave walk's `mm`, at most 64 / LEAF lanes;
// config 2: 60% of the leaves entered): the (lane, member) pairs are dealt one per lane --
// lane L tests member L % LEAF for the (L / LEAF)-th lane of mm, on that lane's ray (six
// ds_bpermute) and the member's record (vector loads, cache-resident) -- instead of every
// lane testing every member.  Each pair forms update_member's candidate (contact distance,
// original index, slot, t), never-winning ones (the member test fails, the contact lies
// behind, NaN) as +inf; the lexicographic minimum over a lane's LEAF pairs (three DPP
// butterflies inside each group of 8 lanes) goes back to the lane and is merged into its
// winner by update_member's rule.  The winner is the (distance, original index) minimum
// over every member tested, whatever the order, and lanes outside mm cannot improve on
// this leaf (the box test's proof): the result is test_leaf's.
// scratch: 64 words of wave-private LDS.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_fl(float x)
{
    return __uint_as_float(dpp_u<CTRL>(__float_as_uint(x)));
}
// one butterfly step of test_leaf_pairs' minimum: the partner lane's candidate via DPP
template <int CTRL>
__device__ __forceinline__ void pair_min_step(float &cds, uint32_t &cor, uint32_t &csl, float &ct)
{
    const float pds = dpp_fl<CTRL>(cds), pt = dpp_fl<CTRL>(ct);
    const uint32_t por = dpp_u<CTRL>(cor), psl = dpp_u<CTRL>(csl);
    const bool take = pds < cds || (pds == cds && por < cor);
    cds = take ? pds : cds;
    cor = take ? por : cor;
    csl = take ? psl : csl;
    ct = take ? pt : ct;
}
// PER members per lane (1: groups of 8 lanes per owner, at most 8 owners; 2: groups of 4
// lanes, at most 16 owners, each lane testing members m and m + 4 and keeping the lesser
// candidate before the two butterflies).
template <int LEAF, int PER>
__device__ __forceinline__ void test_leaf_pairs(const AccelView &ac, uint32_t leaf_slot, unsigned long long mm,
                                                const f3 &o, const f3 &d, Hit &h, uint32_t *scratch, CastDiag &dg)
{
    static_assert(LEAF == 8 && (PER == 1 || PER == 2), "pairs are dealt in groups of 8 / PER lanes");
    constexpr uint32_t G = 8 / PER, LG = PER == 1 ? 3 : 2;
    const uint32_t lane = __lane_id();
    const uint32_t rank = lane_rank(mm);
    const bool owner = __builtin_amdgcn_inverse_ballot_w64(mm);
    if (owner) scratch[rank] = lane;
    const uint32_t q = lane >> LG, s0 = leaf_slot + (lane & (G - 1u));
    const bool valid = q < (uint32_t)__popcll(mm);
    // the members' records and original indices (vector loads, issued before the shuffles)
    float4 sp[PER];
    uint32_t so[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        sp[j] = ac.slots[s0 + j * G];
        so[j] = ac.orig[s0 + j * G];
    }
    const uint32_t src = scratch[valid ? q : 0u];
    const f3 po = mk(__shfl(o.x, (int)src), __shfl(o.y, (int)src), __shfl(o.z, (int)src));
    const f3 pd = mk(__shfl(d.x, (int)src), __shfl(d.y, (int)src), __shfl(d.z, (int)src));
    if (SPT_DIAG) {
        dg.spheres += LEAF;
        dg.lane_tests += (unsigned long long)LEAF * __popcll(mm);
    }
    float tc[PER], hh[PER];
    bool pass[PER];
    unsigned long long anyp = 0ull;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        pass[j] = valid && ray_sphere(sp[j], po, pd, tc[j], hh[j]);
        anyp |= __ballot(pass[j]);
    }
    if (anyp == 0ull) return;
    if (SPT_DIAG) dg.branches += 1;
    // update_member's arithmetic for each pair (Collision.hpp:19-27,49-56); the lane keeps
    // its lexicographic (distance, original index) minimum
    const float pdod = dot(po, pd);
    float cds = INFINITY, ct = 0.f;
    uint32_t cor = 0xFFFFFFFFu, csl = 0u;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const float t = tc[j] - sqrt_pos_normal(hh[j]);
        const f3 p = contact(po, pd, t);
        const bool ok = pass[j] && pdod < dot(p, pd);
        const float dv = lensq(sub(po, p));
        const float jds = ok && dv == dv ? dv : INFINITY;
        if (j == 0) {
            cds = jds;
            cor = so[0];
            csl = s0;
            ct = t;
        } else {
            const bool take = jds < cds || (jds == cds && so[j] < cor);
            cds = take ? jds : cds;
            cor = take ? so[j] : cor;
            csl = take ? s0 + j * G : csl;
            ct = take ? t : ct;
        }
    }
    // the minimum within each group of G lanes: quad_perm [1,0,3,2], quad_perm [2,3,0,1],
    // and for groups of 8 row_half_mirror
    pair_min_step<0xB1>(cds, cor, csl, ct);
    pair_min_step<0x4E>(cds, cor, csl, ct);
    if (G == 8) pair_min_step<0x141>(cds, cor, csl, ct);
    // each owner takes its group's minimum and merges it like update_member
    const int from = (int)(rank << LG);
    const float gds = __shfl(cds, from), gt = __shfl(ct, from);
    const uint32_t gor = (uint32_t)__shfl((int)cor, from), gsl = (uint32_t)__shfl((int)csl, from);
    unsigned long long bm = mm & __ballot(gds < h.best);
    unsigned long long tm = mm & __ballot(gds == h.best) & __ballot(h.idx != kMiss);
    if (__builtin_expect(tm != 0ull, 0)) {
        // exact tie with the current winner (rare): the lower original index wins
        while (tm != 0ull) {
            const int l = (int)__builtin_ctzll(tm);
            const uint32_t wo = ((cuint *)ac.orig)[__builtin_amdgcn_readlane(h.idx, l)];
            const uint32_t go = __builtin_amdgcn_readlane(gor, l);
            if (go < wo) bm |= 1ull << l;
            tm &= tm - 1ull;
        }
    }
    if (SPT_DIAG) dg.improving += bm != 0ull ? 1 : 0;
    const bool better = __builtin_amdgcn_inverse_ballot_w64(bm);
    h.best = better ? gds : h.best;
    h.idx = better ? gsl : h.idx;
    h.t = better ? gt : h.t;
}

// Leaf test behind the member pretest: the S slots plus their S pretest constants.
template <int S>
__device__ __forceinline__ void test_leaf_pre(cfloat *slots, cfloat *kpre, const uint32_t *__restrict__ orig,
                                              uint32_t leaf_slot, const f3 &o, const f3 &d, float dod,
                                              const PreLane &pl, Hit &h, CastDiag &dg)
{
    // 32-bit byte offsets off the table bases: the loads take them as SGPR offsets
    // (no 64-bit address arithmetic on the scalar unit)
    typedef __attribute__((address_space(4))) const char cchar;
    cfloat *cs = (cfloat *)((cchar *)slots + (leaf_slot << 4));
    cfloat *kb = (cfloat *)((cchar *)kpre + (leaf_slot << 2));
    float4 ms[S];
    float kp[S];
#pragma unroll
    for (int k = 0; k < S; ++k) ms[k] = ld_uniform(cs, k);
#pragma unroll
    for (int k = 0; k < S; ++k) kp[k] = kb[k];
    test_group_pre<S>(ms, kp, orig, leaf_slot, o, d, dod, pl, h, dg);
}

// FindClosestIntersectionSphere for every lane of the wave (Collision.hpp:87-109).
// `active`: lanes whose result matters (others never open a node).
// TREE = false: the clusters form a flat list (small scenes) and a node is
// entered when the ray's line may pass one of its members (the "line" test of
// DESIGN.md §4.4).  TREE = true: preorder walk of the cluster tree in the layout
// of the wave's majority direction octant with the line, front and near tests.
// LDSN (tree only): the node records are read from the block's LDS copy of layout 0
// (`lnodes`, render_kernel's prologue) instead of scalar loads of the octant layouts.
template <bool TREE, int LEAF, bool LDSN = false>
__device__ __forceinline__ Hit find_closest(const AccelView &ac, const f3 &o, const f3 &d, bool active,
                                            CastDiag &dg, const uint32_t *lnodes = nullptr, uint32_t *scratch = nullptr)
{
    Hit h;
    h.idx = kMiss;
    h.best = FLT_MAX;
    h.t = 0.f;
    const float dod = dot(o, d);
    cfloat *slots = (cfloat *)ac.slots;
    // Lanes whose direction is not unit length within 1e-6 (the glass branch
    // reflects without renormalising) never cull.
    const float ddev = lensq(d) - 1.0f;
    const bool no_cull = active && !(ddev <= 1e-6f && ddev >= -1e-6f);
    // per-lane terms of the expanded node tests (flat and tree):
    // c |Cb-o|^2 - 4.1e-6 |o|^2 = c |Cb|^2 + (-2c o).Cb + (c - 4.1e-6) |o|^2, c = kFlatScale
    const float oo = lensq(o);
    const float qo = (float)(kFlatScale - 4.1e-6) * oo;
    const float m2c = (float)(-2.0 * kFlatScale);
    const float osx = m2c * o.x, osy = m2c * o.y, osz = m2c * o.z;
    if (SPT_DIAG) dg.live_now = (uint32_t)__popcll(__ballot(active));
    // always-tested spheres (ground, large balls; every sphere when culling is off)
    {
        for (uint32_t g = 0; g < ac.always_groups; ++g) {
            float4 g4[SPT_GROUP];
#pragma unroll
            for (int k = 0; k < SPT_GROUP; ++k) g4[k] = ld_uniform(slots, g * SPT_GROUP + k);
            if (SPT_DUP & 32) {
                Hit h2 = h;
                h2.best = opaque_v(h2.best);
                test_group<SPT_GROUP>(g4, ac.orig, g * SPT_GROUP, opaque_v3(o), opaque_v3(d), dod, h2, dg);
                sink_v(h2.idx);
                sink_v(h2.best);
                sink_v(h2.t);
            }
            test_group<SPT_GROUP>(g4, ac.orig, g * SPT_GROUP, o, d, dod, h, dg);
        }
    }
    const unsigned long long live_mask = __ballot(active);
    cuint *nodes = (cuint *)ac.nodes;
    if (!TREE) {
        // flat list: node i is leaf i.  The line test in expanded form, with FMAs
        // (a conservative test need not follow the reference's operation order;
        // DESIGN.md §4.4): keep iff
        //   d2b <= K1 + 1e-4 |Cb-o|^2 + 4e-6 |Cb|^2 + 4.1e-6 |o|^2,   d2b = |Cb-o|^2 - tcb^2,
        // evaluated as  -2c Cb.o + (c - 4.1e-6) |o|^2 - tcb^2 <= K1''  with
        // c = kFlatScale = 1 - 1e-4, tcb = Cb.d - o.d and K1'' = K1 + 4e-6 |Cb|^2 - c |Cb|^2
        // (rounded up).  The absolute terms cover the expansion's rounding
        // (<= 2.7e-6 (|Cb|^2 + |o|^2)).  Per node: 3 FMA (tcb), 3 FMA (the scaled
        // |Cb-o|^2 less c |Cb|^2), 1 FMA, 1 compare = 8 VALU.
        auto diag_node = [&](unsigned long long mm) {
            if (SPT_DIAG) {
                dg.nodes += 1;
                dg.leaves += mm != 0ull ? 1 : 0;
                dg.pairs += (unsigned long long)__popcll(mm);
                dg.live += mm != 0ull ? (unsigned long long)__popcll(live_mask) : 0ull;
            }
        };
        // flat list: node i is leaf i.  Records are read two at a time into
        // alternating buffers (the next pair loads while this pair is tested), off one
        // pointer with immediate offsets; reading one pair past the layout stays inside
        // the node table (the eight layouts follow each other).  Inactive lanes carry
        // qo = +inf (never pass) and lanes that must not cull carry -inf (always
        // pass), so the ballot of the compare is the node mask: about 5 SALU per node
        // instead of 17.
        const float qoe = !active ? INFINITY : (no_cull ? -INFINITY : qo);
        // member pretest terms: the node test's -2c o and qoe, plus the tc slack
        // mt = 2e-6 (pre_cm + |o|) + 1e-6 folded into -o.d
        const float olen = __builtin_amdgcn_sqrtf(oo) * 1.000001f;
        PreLane pl;
        pl.osx = osx;
        pl.osy = osy;
        pl.osz = osz;
        pl.qoe = qoe;
        pl.tinit = !active ? -INFINITY : (no_cull ? INFINITY : __builtin_fmaf(2e-6f, ac.pre_cm + olen, 1e-6f) - dod);
        // c |Cb|^2 is left out of the sum: the node's threshold is K1'' = K1' - c |Cb|^2
        // (one rounding fewer)
        auto node_x = [&](const uint32_t *r) {
            const float bx = __uint_as_float(r[0]), by = __uint_as_float(r[1]), bz = __uint_as_float(r[2]);
            const float tcb = __builtin_fmaf(bx, d.x, __builtin_fmaf(by, d.y, __builtin_fmaf(bz, d.z, -dod)));
            const float w = __builtin_fmaf(bx, osx, __builtin_fmaf(by, osy, __builtin_fmaf(bz, osz, qoe)));
            return __builtin_fmaf(-tcb, tcb, w);
        };
        // the node's mask (vs K1'') and leaf test; `x` from node_x(r)
        auto finish = [&](const uint32_t *r, float x) {
            const unsigned long long mm = __ballot(x <= __uint_as_float(r[6]));
            diag_node(mm);
            if (mm != 0ull) test_leaf_pre<LEAF>(slots, (cfloat *)ac.kpre, ac.orig, r[5], o, d, dod, pl, h, dg);
        };
        // The next record's load is issued only after this record's first use: a
        // scalar-load wait is lgkmcnt(0), so an earlier issue would be waited for here.
        cuint *p = nodes;
        uint32_t ra[8], rb[8];
        // the whole record in one s_load_dwordx8 (the compiler would load only the six
        // dwords the flat test uses, as four loads); the empty asm keeps all eight
        typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
        typedef __attribute__((address_space(4))) const u32x8 cu32x8;
        auto load_rec = [&](cuint *q, uint32_t(&r)[8]) {
            u32x8 v = *(cu32x8 *)q;
            asm volatile("" : "+s"(v));
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = v[i];
        };
        load_rec(p, ra);
        uint32_t left = ac.n_nodes;
        while (left >= 2u) {
            const float xa = node_x(ra);
            __builtin_amdgcn_sched_barrier(0);
            load_rec(p + 8, rb);
            finish(ra, xa);
            const float xb = node_x(rb);
            __builtin_amdgcn_sched_barrier(0);
            load_rec(p + 16, ra);
            finish(rb, xb);
            p += 16;
            left -= 2u;
        }
        if (left != 0u) finish(ra, node_x(ra));
        return h;
    }
    // |o| (rounded up), for the box margin and the front and near slack
    const float olen = __builtin_amdgcn_sqrtf(oo) * 1.000001f;
    if (TREE) {
        // the layout of the wave's majority direction octant (siblings front to back)
        const uint32_t nlive = (uint32_t)__popcll(live_mask);
        // ballots of the compares themselves, masked with the live lanes (a ballot of
        // `active && ...` goes through a VGPR bool per term)
        const uint32_t oct = (2u * (uint32_t)__popcll(__ballot(d.x < 0.f) & live_mask) > nlive ? 1u : 0u) |
                             (2u * (uint32_t)__popcll(__ballot(d.y < 0.f) & live_mask) > nlive ? 2u : 0u) |
                             (2u * (uint32_t)__popcll(__ballot(d.z < 0.f) & live_mask) > nlive ? 4u : 0u);
        if (!LDSN) nodes += (size_t)8 * (ac.n_nodes + 1) * oct;
    }
    // Tree nodes are boxes [lo, hi] already expanded by kBoxS Bm.  Per
    // lane: the margin el = kBoxS |o| + 1e-6, the reciprocals ir of d (|d_i| raised to
    // kBoxMinDir) and ql = -(o + el) ir, qh = (el - o) ir, so the entry and exit
    // parameters of slab i along d are min / max of  fma(lo_i, ir_i, ql_i)  and
    // fma(hi_i, ir_i, qh_i).  A lane may need the node iff
    //   max(t_near, -eta) <= min(t_far, sbl)
    // i.e. the slabs overlap (line), t_far >= -eta (front: a member may lie ahead) and
    // t_near <= sbl (near: a member's contact point may be closer than the lane's
    // winner), with eta = 1e-6 (|o| + Bs) + 1e-6 and
    // sbl = sqrt(best) (1 + 1e-5) + 1e-5 (|o| + Bs) + 1e-6, Bs = pre_cm >= every Bm.
    // 17 VALU per node.  Lanes with |o| > 1e15 never cull.
        const float el = __builtin_fmaf((float)kBoxS, olen, 1e-6f);
    auto rcp_dir = [](float x) {
        const float m = __builtin_fmaxf(__builtin_fabsf(x), kBoxMinDir);
        return __builtin_amdgcn_rcpf(__builtin_copysignf(m, x));
    };
    const float irx = rcp_dir(d.x), iry = rcp_dir(d.y), irz = rcp_dir(d.z);
    const float qlx = (-o.x - el) * irx, qly = (-o.y - el) * iry, qlz = (-o.z - el) * irz;
    const float qhx = (el - o.x) * irx, qhy = (el - o.y) * iry, qhz = (el - o.z) * irz;
    const float obs = olen + ac.pre_cm;
    const float neta = -__builtin_fmaf(1e-6f, obs, 1e-6f);
    // -inf for inactive lanes: their sbl stays -inf and they never pass a node
    const float kn = active ? __builtin_fmaf(1e-5f, obs, 1e-6f) : -INFINITY;
    // tree node masks are (ballot(test) & live) | nocull: the ballot of a compare is
    // the compare's own lane mask, with no VALU round trip
    const unsigned long long tree_nocull =
        (__ballot(!(ddev <= 1e-6f && ddev >= -1e-6f)) | __ballot(!(oo <= 1e30f))) & live_mask;
    // near bound of the lane's current winner, refreshed after every leaf test;
    // ~1.8e19 while there is none (best = FLT_MAX: never culls)
    auto near_bound = [&](float best) {
        return __builtin_fmaf(__builtin_amdgcn_sqrtf(best), 1.00001f, kn);
    };
    float sbl = near_bound(h.best);
    // node record q of node j: a scalar load, or a broadcast LDS read
    // (scalar loads off a 32-bit byte offset: one SGPR-offset s_load_dwordx8, no
    // 64-bit address arithmetic per node)
    typedef __attribute__((address_space(4))) const char cchar;
    auto ldn = [&](uint32_t j, int q) -> uint32_t {
        return LDSN ? lnodes[8 * j + q] : *(cuint *)((cchar *)nodes + (j << 5) + 4 * q);
    };
    uint32_t i = 0;
    uint32_t nb[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) nb[q] = ldn(0, q);
    while (i < ac.n_nodes) {
        const float lx = __uint_as_float(nb[0]), ly = __uint_as_float(nb[1]), lz = __uint_as_float(nb[2]);
        const float hx = __uint_as_float(nb[3]), hy = __uint_as_float(nb[6]), hz = __uint_as_float(nb[7]);
        const uint32_t skip = LDSN ? __builtin_amdgcn_readfirstlane(nb[4]) : nb[4];
        const uint32_t leaf_slot = LDSN ? __builtin_amdgcn_readfirstlane(nb[5]) : nb[5];
        // LDS walk: this node's scalars before the successor's reads are issued (a
        // readfirstlane after them would wait for them: LDS waits are lgkmcnt(0))
        if (LDSN) asm volatile("" ::"s"(skip), "s"(leaf_slot));
        // speculative prefetch of the preorder successor (prefetching the skip
        // target as well measured 4% slower on config 5)
#pragma unroll
        for (int q = 0; q < 8; ++q) nb[q] = ldn(i + 1, q);
        // LDS walk: keep the successor's ds_reads ahead of this node's tests
        if (LDSN) __builtin_amdgcn_sched_barrier(0);
        const float ax = __builtin_fmaf(lx, irx, qlx), bx = __builtin_fmaf(hx, irx, qhx);
        const float ay = __builtin_fmaf(ly, iry, qly), by = __builtin_fmaf(hy, iry, qhy);
        const float az = __builtin_fmaf(lz, irz, qlz), bz = __builtin_fmaf(hz, irz, qhz);
        const float tn = max3_raw(__builtin_fminf(ax, bx), __builtin_fminf(ay, by),
                                  max_raw(__builtin_fminf(az, bz), neta));
        const float tf = min3_raw(__builtin_fmaxf(ax, bx), __builtin_fmaxf(ay, by),
                                  min_raw(__builtin_fmaxf(az, bz), sbl));
        // inactive lanes have sbl = -inf, so t_f < t_n: no AND with the live mask
        const unsigned long long mm = __ballot(tn <= tf) | tree_nocull;
        if (SPT_DUP & 8) {
            const float jx = opaque_v(irx), jy = opaque_v(iry), jz = opaque_v(irz);
            const float ax2 = __builtin_fmaf(lx, jx, qlx), bx2 = __builtin_fmaf(hx, jx, qhx);
            const float ay2 = __builtin_fmaf(ly, jy, qly), by2 = __builtin_fmaf(hy, jy, qhy);
            const float az2 = __builtin_fmaf(lz, jz, qlz), bz2 = __builtin_fmaf(hz, jz, qhz);
            const float tn2 = max3_raw(__builtin_fminf(ax2, bx2), __builtin_fminf(ay2, by2),
                                       max_raw(__builtin_fminf(az2, bz2), neta));
            const float tf2 = min3_raw(__builtin_fmaxf(ax2, bx2), __builtin_fmaxf(ay2, by2),
                                       min_raw(__builtin_fmaxf(az2, bz2), sbl));
            const unsigned long long mm2 = __ballot(tn2 <= tf2);
            asm volatile("" ::"s"(mm2));
        }
        const bool leaf = leaf_slot != kNoSlot;
        if (SPT_DIAG) {
            dg.nodes += 1;
            dg.leaves += (mm != 0ull && leaf) ? 1 : 0;
            if (leaf) {
                dg.pairs += (unsigned long long)__popcll(mm);
                dg.leaves8 += (mm != 0ull && __popcll(mm) <= 8) ? 1 : 0;
                dg.leaves16 += (mm != 0ull && __popcll(mm) <= 16) ? 1 : 0;
                dg.live += mm != 0ull ? (unsigned long long)__popcll(live_mask) : 0ull;
            }
        }
        // (one branch per outcome -- culled inner node / entered leaf / else -- measured
        // 2% slower on config 2 and 8% on config 5 than this form)
        if (mm != 0ull && leaf) {
            // few lanes need the leaf: deal its (lane, member) pairs (SPT_LEAF_PAIRS)
            auto leaf_test = [&](const f3 &lo, const f3 &ld, Hit &lh) {
                bool paired = false;
                if constexpr (SPT_LEAF_PAIRS && LEAF == 8 && !LDSN) {
                    const uint32_t nm = (uint32_t)__popcll(mm);
                    if (scratch && nm <= 8u) {
                        test_leaf_pairs<LEAF, 1>(ac, leaf_slot, mm, lo, ld, lh, scratch, dg);
                        paired = true;
                    } else if (SPT_LEAF_PAIRS >= 2 && scratch && nm <= 16u) {
                        test_leaf_pairs<LEAF, 2>(ac, leaf_slot, mm, lo, ld, lh, scratch, dg);
                        paired = true;
                    }
                }
                if (!paired) test_leaf<LEAF>(slots, ac.orig, leaf_slot, lo, ld, dot(lo, ld), lh, dg);
            };
            if (SPT_DUP & 16) {
                Hit h2 = h;
                h2.best = opaque_v(h2.best);
                leaf_test(opaque_v3(o), opaque_v3(d), h2);
                sink_v(h2.idx);
                sink_v(h2.best);
                sink_v(h2.t);
            }
            leaf_test(o, d, h);
            sbl = near_bound(h.best);
        }
        const uint32_t next = (mm != 0ull && !leaf) ? i + 1 : skip;
        if (next != i + 1) {
#pragma unroll
            for (int q = 0; q < 8; ++q) nb[q] = ldn(next, q);
        }
        i = next;
    }
    return h;
}

// The closest-contact / distance update of one member for one lane (update_member
// for lane-divergent walks): the lane passed RaySphereIntersection with tc, hh.
// Exact ties go to the lower original index (vector loads, behind a divergent branch).
__device__ __forceinline__ void update_member_lane(float tc, float hh, const uint32_t *__restrict__ orig,
                                                   uint32_t s, const f3 &o, const f3 &d, float dod, Hit &h)
{
    const float t = tc - sqrt_pos_normal(hh);
    const f3 p = contact(o, d, t);
    const bool front = dod < dot(p, d);
    const float ds = lensq(sub(o, p));
    bool better = front && ds < h.best;
    if (__builtin_expect(front && ds == h.best && h.idx != kMiss, 0)) better = orig[s] < orig[h.idx];
    h.best = better ? ds : h.best;
    h.idx = better ? s : h.idx;
    h.t = better ? t : h.t;
}

// Lane-divergent walk of the LDS box tree (SPT_LANE_WALK, render_kernel_lds): every
// lane follows its own preorder/skip path through the node records (two ds_read_b128
// per lane and node) and tests only the leaves its own ray may need, their member
// records read by vector loads.  A lane parks the leaves it meets (two at most; it
// stops walking at the second) and the wave tests the parked leaves -- each lane its
// newest one -- once SPT_LANE_LEAF_T lanes hold one or no lane can walk on (Aila &
// Laine's postponed leaves, while-while).  The wave walk (find_closest) pays for the union of its lanes'
// leaves -- on config 5 a lane needs ~10% of the members the wave tests.  Node test,
// margins and near bound are find_closest's, per lane; leaves are
// tested in a lane-dependent order, and the winner is still the lexicographic minimum
// of (distance, original index), which does not depend on the order.
// SPT_DIAG counters here: nodes = lane node visits, live = walk iterations, leaves =
// leaf passes, pairs = (lane, leaf) tests.
#ifndef SPT_LANE_LEAF_T
#define SPT_LANE_LEAF_T 24
#endif
#ifndef SPT_LANE_GROUP
#define SPT_LANE_GROUP 2
#endif
#ifndef SPT_LANE_STEPS
#define SPT_LANE_STEPS 8
#endif
// The lane walk as a resumable cast: `fresh` lanes start (winner none, node 0); the
// others continue from their saved node, parked leaves and winner.  The always-list is
// re-tested for every lane (idempotent: a sphere tested twice cannot replace itself --
// equal distance and index).  Runs at most `budget` walk iterations and leaf passes;
// returns whether the lane's cast is complete (inactive lanes: true).
// BYTES: node positions (i, the records' skip links) are byte offsets into `lnodes` (the
// LDS copy of render_kernel_lds stores them so: no shift per node step); else indices.
// Parked leaves form a two-entry shift register: a leaf reached goes to `leaf`, the one
// there moves to `leaf2` (2 VALU per step fewer than filling the first free entry; the
// pass tests both, in any order: the winner does not depend on it).
template <int LEAF, bool BYTES = false>
__device__ __forceinline__ bool lane_cast(const AccelView &ac, const f3 &o, const f3 &d, bool active, CastDiag &dg,
                                          const uint32_t *lnodes, bool fresh, uint32_t budget, Hit &h, uint32_t &i,
                                          uint32_t &leaf, uint32_t &leaf2)
{
    if (fresh) {
        h.idx = kMiss;
        h.best = FLT_MAX;
        h.t = 0.f;
        i = active ? 0u : (BYTES ? ac.n_nodes << 5 : ac.n_nodes);
        leaf = leaf2 = kNoSlot;
    }
    const float dod = dot(o, d);
    cfloat *slots = (cfloat *)ac.slots;
    const float ddev = lensq(d) - 1.0f;
    const bool no_cull = active && !(ddev <= 1e-6f && ddev >= -1e-6f);
    const float oo = lensq(o);
    if (SPT_DIAG) dg.live_now = (uint32_t)__popcll(__ballot(active));
    for (uint32_t g = 0; g < ac.always_groups; ++g) {
        float4 g4[SPT_GROUP];
#pragma unroll
        for (int k = 0; k < SPT_GROUP; ++k) g4[k] = ld_uniform(slots, g * SPT_GROUP + k);
        test_group<SPT_GROUP>(g4, ac.orig, g * SPT_GROUP, o, d, dod, h, dg);
    }
    auto rcp_dir = [](float x) {
        const float m = __builtin_fmaxf(__builtin_fabsf(x), kBoxMinDir);
        return __builtin_amdgcn_rcpf(__builtin_copysignf(m, x));
    };
    const bool nocull = no_cull || (active && !(oo <= 1e30f));
    // the node test's per-lane terms (slabs, front slack, near bound), formed from o, d and
    // the winner
    float irx, iry, irz, qlx, qly, qlz, qhx, qhy, qhz, neta, kn, sbl;
    auto near_bound = [&](float best) { return __builtin_fmaf(__builtin_amdgcn_sqrtf(best), 1.00001f, kn); };
    auto walk_terms = [&]() {
        const float olen = __builtin_amdgcn_sqrtf(lensq(o)) * 1.000001f;
        const float el = __builtin_fmaf((float)kBoxS, olen, 1e-6f);
        irx = rcp_dir(d.x);
        iry = rcp_dir(d.y);
        irz = rcp_dir(d.z);
        qlx = (-o.x - el) * irx;
        qly = (-o.y - el) * iry;
        qlz = (-o.z - el) * irz;
        qhx = (el - o.x) * irx;
        qhy = (el - o.y) * iry;
        qhz = (el - o.z) * irz;
        const float obs = olen + ac.pre_cm;
        neta = -__builtin_fmaf(1e-6f, obs, 1e-6f);
        kn = __builtin_fmaf(1e-5f, obs, 1e-6f);
        sbl = near_bound(h.best);
    };
    walk_terms();
    const uint4 *ln = (const uint4 *)lnodes;
    const float4 *__restrict__ gs = ac.slots;
    const uint32_t n = BYTES ? ac.n_nodes << 5 : ac.n_nodes;  // end of the walk
    // parked leaves (first slots), kNoSlot = none: a lane keeps walking while one
    // leaf is parked and stops at the second
    uint32_t it = 0;
    for (;;) {
        if (++it > budget) break;
        const bool tr = i < n && leaf2 == kNoSlot;
        const unsigned long long mt = __ballot(tr);
        const unsigned long long mp = __ballot(leaf != kNoSlot);
        if ((mt | mp) == 0ull) break;
        if (mp != 0ull && (mt == 0ull || __popcll(mp) >= SPT_LANE_LEAF_T)) {
            if (SPT_DIAG) {
                const unsigned long long nl = (unsigned long long)__popcll(mp);
                dg.leaves += 1;
                dg.pairs += nl;
                dg.lane_tests += (unsigned long long)LEAF * nl;
            }
            if (leaf != kNoSlot) {
                // the lane's newest parked leaf, its members SPT_LANE_GROUP at a time (8
                // waves/SIMD: 64 VGPRs; loading a whole leaf at once spills).  A second
                // leaf stays parked for a later pass and the lane walks on, so a pass is
                // LEAF member tests (testing both kept the whole wave at 2 LEAF whenever
                // one lane held two: config 5 71.8 -> 70.8 ms)
#pragma unroll 1
                for (int k0 = 0; k0 < LEAF; k0 += SPT_LANE_GROUP) {
                    float4 m[SPT_LANE_GROUP];
#pragma unroll
                    for (int k = 0; k < SPT_LANE_GROUP; ++k) m[k] = gs[leaf + k0 + k];
#pragma unroll
                    for (int k = 0; k < SPT_LANE_GROUP; ++k) {
                        float tc, hh;
                        if (ray_sphere(m[k], o, d, tc, hh))
                            update_member_lane(tc, hh, ac.orig, leaf + k0 + k, o, d, dod, h);
                    }
                }
                sbl = near_bound(h.best);
                leaf = leaf2;
                leaf2 = kNoSlot;
            }
            continue;
        }
        if (SPT_DIAG) dg.live += 1;
        // one node step of the lane's own walk (lanes with a second parked leaf wait)
        auto visit = [&]() {
            const uint4 *rec = BYTES ? (const uint4 *)((const char *)lnodes + i) : ln + 2 * i;
            const uint4 ra = rec[0], rb = rec[1];
            const uint32_t nskip = rb.x, nslot = rb.y;
            const float ax = __builtin_fmaf(__uint_as_float(ra.x), irx, qlx);
            const float bx = __builtin_fmaf(__uint_as_float(ra.w), irx, qhx);
            const float ay = __builtin_fmaf(__uint_as_float(ra.y), iry, qly);
            const float by = __builtin_fmaf(__uint_as_float(rb.z), iry, qhy);
            const float az = __builtin_fmaf(__uint_as_float(ra.z), irz, qlz);
            const float bz = __builtin_fmaf(__uint_as_float(rb.w), irz, qhz);
            const float tn = max3_raw(__builtin_fminf(ax, bx), __builtin_fminf(ay, by),
                                      max_raw(__builtin_fminf(az, bz), neta));
            const float tf = min3_raw(__builtin_fmaxf(ax, bx), __builtin_fmaxf(ay, by),
                                      min_raw(__builtin_fmaxf(az, bz), sbl));
            const bool hit = (tn <= tf) | nocull;
            const bool is_leaf = nslot != kNoSlot;
            if (hit && is_leaf) {
                leaf2 = leaf;
                leaf = nslot;
            }
            i = (hit && !is_leaf) ? i + (BYTES ? 32u : 1u) : nskip;
        };
        // SPT_LANE_STEPS node steps per walk iteration: the iteration's ballots, budget
        // check and leaf-pass test are paid once per that many steps (config 5: 1 / 3 / 4 /
        // 6 steps at budgets 40 / 16 / 12 / 8 iterations: 90.4 / 80.5 / 79.5 / 78.2 ms; with
        // leaf passes at 24 lanes, steps x budget 6x8 / 7x7 / 7x6 / 8x6 / 8x5 / 6x6 / 5x8:
        // 77.1 / 75.5 / 75.6 / 75.3 / 75.8 / 78.4 / 77.0 ms)
#pragma unroll
        for (int k = 0; k < SPT_LANE_STEPS; ++k) {
            const bool w = i < n && leaf2 == kNoSlot;
            if (SPT_DIAG) dg.nodes += (unsigned long long)__popcll(__ballot(w));
            if (w) visit();
        }
    }
    return !(i < n || leaf != kNoSlot);
}

// One-shot lane walk (the whole cast in one call).
template <int LEAF>
__device__ __forceinline__ Hit find_closest_lane(const AccelView &ac, const f3 &o, const f3 &d, bool active,
                                                 CastDiag &dg, const uint32_t *lnodes)
{
    Hit h;
    uint32_t i, leaf, leaf2;
    (void)lane_cast<LEAF>(ac, o, d, active, dg, lnodes, true, 0xFFFFFFFFu, h, i, leaf, leaf2);
    return h;
}

// Per-lane path state of the flattened recursion.  The diffuse loop's colour is not
// carried: it is the first diffuse hit's albedo halved once per bounce, so the path
// keeps that hit's slot and the sample code records it with the bounce count (the fold
// rebuilds the colour, code_word in spt_internal.h).
struct Path {
    uint32_t phase, item, bounce, spec;
    uint64_t st;  // keyed splitmix stream of this (pixel, sample)
    f3 o, d;
    uint32_t slot;  // slot of the first diffuse hit (PH_DLOOP)
    uint32_t job;   // render service: the completion counter of the path's job (else unused)
};

// GenerateUniformDistInsideSphereVector (Random.hpp:115-127) for every lane with
// `need`, all 64 lanes cooperating.  The stream is counter-based (draw n of a lane
// is mix(st0 + (n+1) gamma)), so trial j = draws 3j..3j+2 can be evaluated by any
// lane.  Round 0: every lane runs its own trial 0.  Later rounds: each still
// pending lane gets H helper lanes (H = the largest power of two <= 64 / pending,
// at most 16) that evaluate its trials jb .. jb+H-1 at once; it takes the lowest
// accepted one.  The result and the advanced state st0 + 3 (j* + 1) gamma equal
// the sequential loop's.  Must be called in wave-uniform control flow.
// `lds`: 64 words of wave-private LDS.
__device__ __forceinline__ f3 coop_ball_vector(uint64_t &st, bool need, uint32_t *lds, unsigned long long *rounds = nullptr)
{
    const uint32_t lane = __lane_id();
    const uint64_t st0 = st;
    f3 r;
    uint32_t jacc = 0;
    unsigned long long pend;
    uint32_t jb;
    const unsigned long long needm = __ballot(need);
    if (SPT_SAMPLER_SKIP0 && __popcll(needm) <= 32) {
        // at most 32 lanes need a vector: every one gets two or more helpers from trial 0 on
        // (round 0 would run one trial per lane for all 64, half of them for nothing)
        r = mk(0.f, 0.f, 0.f);
        pend = needm;
        jb = 0;
    } else {
        uint64_t t = st0;
        r.x = uniform(t, -0.5f, 0.5f);
        r.y = uniform(t, -0.5f, 0.5f);
        r.z = uniform(t, -0.5f, 0.5f);
        pend = __ballot(need && lensq(r) < 0.25f);
        jb = 1;
    }
    const uint32_t s_lo = (uint32_t)st0, s_hi = (uint32_t)(st0 >> 32);
    if (SPT_DIAG && rounds) rounds[0] += 1;  // calls (round 0 for every lane)
#if SPT_DIAG
    const unsigned long long t_in = __builtin_amdgcn_s_memtime();
#endif
    while (pend != 0ull) {
        if (SPT_DIAG && rounds) rounds[1] += 1;  // cooperative rounds after round 0
        const uint32_t np = (uint32_t)__popcll(pend);
        // lg = min(floor(log2(64 / np)), 4) = min(6 - ceil(log2 np), 4) on the scalar unit
        // (64 / np compiled to a float reciprocal sequence on the vector unit)
        uint32_t lg = np <= 4u ? 4u : (uint32_t)__builtin_clz(np - 1u) - 26u;
        lg = lg > 4u ? 4u : lg;
        // the lane's bit of a wave mask as a lane predicate without vector instructions
        const bool is_p = __builtin_amdgcn_inverse_ballot_w64(pend);
        const uint32_t rank = lane_rank(pend);
        if (is_p) lds[rank] = lane;
        const uint32_t pidx = lane >> lg, tt = lane & ((1u << lg) - 1u);
        const bool valid = pidx < np;
        const uint32_t src = lds[valid ? pidx : 0u];
        const uint32_t h_lo = (uint32_t)__shfl((int)s_lo, (int)src), h_hi = (uint32_t)__shfl((int)s_hi, (int)src);
        uint64_t b = (((uint64_t)h_hi << 32) | h_lo) + (uint64_t)(3u * (jb + tt)) * kGamma;
        f3 c;
        c.x = uniform(b, -0.5f, 0.5f);
        c.y = uniform(b, -0.5f, 0.5f);
        c.z = uniform(b, -0.5f, 0.5f);
        const unsigned long long acc = __ballot(valid && !(lensq(c) < 0.25f));
        const uint32_t seg = is_p ? (uint32_t)(acc >> (rank << lg)) & ((1u << (1u << lg)) - 1u) : 0u;
        const bool found = seg != 0u;
        const uint32_t tstar = found ? (uint32_t)__builtin_ctz(seg) : 0u;
        const uint32_t from = found ? (rank << lg) + tstar : lane;
        const float rx = __shfl(c.x, (int)from), ry = __shfl(c.y, (int)from), rz = __shfl(c.z, (int)from);
        if (found) {
            r = mk(rx, ry, rz);
            jacc = jb + tstar;
        }
        pend = __ballot(is_p && !found);
        jb += 1u << lg;
    }
    if (need) st = st0 + (uint64_t)(3u * (jacc + 1u)) * kGamma;
#if SPT_DIAG
    if (rounds) rounds[2] += __builtin_amdgcn_s_memtime() - t_in;  // sampler cycles
#endif
    return r;
}

// The kernel's RenderArgs in the kernarg segment, behind an opaque zero offset: the
// refill-only fields read through it are loaded (scalar cache) where they are used
// instead of being hoisted into SGPRs for the kernel's lifetime.  Only valid in a
// kernel whose first argument is a RenderArgs (render_kernel: start_path<true>).
typedef __attribute__((address_space(4))) const RenderArgs kargs_t;
__device__ __forceinline__ kargs_t *kernarg_args()
{
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    typedef __attribute__((address_space(4))) const char kchar;
    return (kargs_t *)((kchar *)__builtin_amdgcn_kernarg_segment_ptr() + z);
}

// FindClosestIntersectionSphere for a primary batch from its block's candidate list
// (PrimLists, spt_internal.h): every lane's closest hit is in the
// list of its pixel's block, so the (distance, original index) minimum over the list --
// the winner update_member keeps, independent of the order members are tested in -- is
// the reference's.  pxy: the lane's pixel (y << 16 | x).  The lanes' common 8x8 block's
// list, or when they span several blocks (ragged edge tiles, interleaved rank strips)
// the union of their 8x4 blocks' lists (a member tested twice cannot replace itself).
// Returns false, with h undefined, when the wave must walk the tree instead: a block
// without a list, or a lane that may not cull (direction off unit length, |o| > 1e15).
__device__ __forceinline__ bool prim_list_cast(const AccelView &ac, const f3 &o, const f3 &d, bool active, uint32_t pxy,
                                               Hit &h, CastDiag &dg)
{
    kargs_t &k = *kernarg_args();
    const float ddev = lensq(d) - 1.0f;
    if (__ballot(active && !(ddev <= 1e-6f && ddev >= -1e-6f && lensq(o) <= 1e30f)) != 0ull) return false;
    h.idx = kMiss;
    h.best = FLT_MAX;
    h.t = 0.f;
    const unsigned long long live = __ballot(active);
    if (live == 0ull) return true;
    const uint32_t bw = k.prim.bw;
    const uint32_t x = pxy & 0xFFFFu, y = pxy >> 16;
    const float dod = dot(o, d);
    cfloat *slots = (cfloat *)ac.slots;
    cuint *ids = (cuint *)k.prim.slots;
    if (SPT_DIAG) dg.live_now = (uint32_t)__popcll(live);
    // one run of candidate slots, 4 at a time (runs are padded with a dummy slot)
    auto test_run = [&](uint2 e) {
        for (uint32_t i = e.x; i < e.x + e.y; i += 4u) {
            uint32_t s[4];
            float4 sp[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q] = ids[i + q];
#pragma unroll
            for (int q = 0; q < 4; ++q) sp[q] = ld_uniform(slots, s[q]);
            float tcv[4], hv[4];
            bool pass[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) pass[q] = ray_sphere(sp[q], o, d, tcv[q], hv[q]);
            if (SPT_DIAG) dg.lane_tests += 4ull * dg.live_now;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const unsigned long long pm = __ballot(pass[q]);
                if (SPT_DIAG) {
                    dg.spheres += 1;
                    dg.branches += pm != 0ull ? 1 : 0;
                }
                if (pm != 0ull) update_member(pm, tcv[q], hv[q], ac.orig, s[q], o, d, dod, h, dg);
            }
        }
    };
    const uint32_t b8 = (y >> 3) * bw + (x >> 3);
    const uint32_t lead = __builtin_amdgcn_readlane(b8, (int)__builtin_ctzll(live));
    if (__ballot(active && b8 != lead) == 0ull) {
        cuint *blk = (cuint *)k.prim.b8 + 2u * lead;
        const uint2 e = make_uint2(blk[0], blk[1]);
        if (e.y == kPrimWalk) return false;
        test_run(e);
        return true;
    }
    const uint32_t b4 = (y >> 2) * bw + (x >> 3);
    unsigned long long todo = live;
    while (todo != 0ull) {
        const uint32_t b = __builtin_amdgcn_readlane(b4, (int)__builtin_ctzll(todo));
        cuint *blk = (cuint *)k.prim.b4 + 2u * b;
        const uint2 e = make_uint2(blk[0], blk[1]);
        if (e.y == kPrimWalk) return false;
        test_run(e);
        todo &= ~__ballot(active && b4 == b);
    }
    return true;
}

// SampleColorRefractive (SingleThreadPathTracer.hpp:48-92) for a lane whose ray hit
// the glass slot idx at the contact point ps.o: new ps.o (exit point) and ps.d.
__device__ __forceinline__ void refract_event(const float4 *__restrict__ slots, Path &ps, uint32_t idx)
{
    const float4 cs = slots[idx];
    const f3 C = mk(cs.x, cs.y, cs.z);
    const f3 nrm = normalize(sub(ps.o, C));
    const f3 d = ps.d;
    const float cc = dot(neg(nrm), d);
    f3 nd;
    if (uniform(ps.st, 0.f, 1.f) < schlick(kRsq, cc)) {
        nd = reflect(d, nrm);
    } else if (no_tir(kAirToGlass, cc)) {
        const f3 d2 = refract_dir(d, nrm, kAirToGlass, cc);
        // CalculateRaySphereFarthestContactPoint, Collision.hpp:29-37,58-65
        const f3 rs = sub(C, ps.o);
        const float tc = dot(rs, d2);
        const float dd = lensq(rs) - tc * tc;
        const float t = tc + __builtin_sqrtf(cs.w - dd);
        ps.o = mk(ps.o.x + d2.x * t, ps.o.y + d2.y * t, ps.o.z + d2.z * t);
        const f3 n2 = neg(normalize(sub(ps.o, C)));
        const float c2 = dot(neg(n2), d2);
        if (uniform(ps.st, 0.f, 1.f) < schlick(kRsq, c2))
            nd = reflect(d2, n2);
        else if (no_tir(kGlassToAir, c2))
            nd = refract_dir(d2, n2, kGlassToAir, c2);
        else
            nd = reflect(d2, n2);
    } else {
        nd = reflect(d, nrm);
    }
    ps.d = nd;
}

// The tail of a shading step: the specular-event cap (RenderSegmentTask's pass limit,
// the safety cap) and, for finishing paths, the sample slot write.
//
// ps.spec: bits 0-15 count the path's specular events (= the RenderSegmentTask pass
// it is in); in task mode bits 16-25 record which queue each of its first ten
// events came from (bit 16 + k: 1 = refractive queue of pass k, 0 = reflective).
// A task-mode slot's w is the path's position key inside its sample
// (TaskBasedPathTracer.hpp:81-193): 1 + (pass << 11 | sky << 10 | queue bits), 0 for
// a dropped path.  Within one sample RenderSegmentTask adds colours pass by pass,
// the diffuse queue before the skybox queue, and a queue holds the tasks pushed by
// the previous pass's reflective loop before those of its refractive loop, each in
// its own queue order; so two paths of a sample reach `colors` in the order of
// (key, pixel) -- which only matters where colorIndex aliases pixels (non-square
// tiles, lines 103 and 186; fold_kernel).
// WT (the render service): the sample word is stored write-through (sc1: it leaves the
// XCD's L2 at once), so the completion count that follows needs only the wave's own
// s_waitcnt, not an L2 write-back (spt_kernels.hip svc_flush).
template <bool WT = false>
__device__ __forceinline__ void finish_step(uint32_t mode, uint32_t *samples, Path &ps, bool fin, bool spec_event,
                                            bool refr_event, bool sky, uint32_t word, unsigned long long &done,
                                            unsigned long long &dropped)
{
    bool counted = true;
    if (spec_event) {
        const uint32_t k = ps.spec & 0xFFFFu;
        if (mode == 1u && k < kTaskPasses && refr_event) ps.spec |= 1u << (16u + k);
        ++ps.spec;
        if (mode == 1u && k + 1u >= kTaskPasses) {
            // RenderSegmentTask: this path would be processed in pass 10, which never runs
            fin = true;
            counted = false;
            word = kZeroWord;
            ++dropped;
        } else if (k + 1u > kSpecularCap) {
            fin = true;
            word = kZeroWord;
        }
    }
    if (fin) {
        typedef __attribute__((address_space(1))) uint32_t gu32_t;
        typedef __attribute__((address_space(1))) unsigned long long gu64_t;
        if (mode == 0u) {
            // RenderSegment counts every sample: one word per slot
            if (WT)
                __hip_atomic_store((gu32_t *)(samples + ps.item), word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                samples[ps.item] = word;
        } else {
            const uint32_t key =
                counted ? 1u + (((ps.spec & 0xFFFFu) << 11) | (sky ? 1u << 10 : 0u) | ((ps.spec >> 16) & 0x3FFu)) : 0u;
            if (WT)
                __hip_atomic_store((gu64_t *)(samples + (size_t)2 * ps.item), (unsigned long long)word | ((unsigned long long)key << 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                *(uint2 *)(samples + (size_t)2 * ps.item) = make_uint2(word, key);
        }
        ps.phase = PH_IDLE;
        ps.d = mk(0.f, 0.f, 0.f);
        ++done;
    }
}

// One shading step after a cast: the material switch of TraceAndSampleColor
// (SingleThreadPathTracer.hpp:94-112) in PH_TRACE, or one turn of the diffuse
// bounce loop (21-37) in PH_DLOOP.  Finishing paths write their sample slot.
// Called by every lane of the wave (`act` = the lane holds a path), so the
// cooperative cube-minus-ball sampler runs in uniform control flow.
template <bool KARG, bool WT, bool SAMPLER>
__device__ __forceinline__ void shade_step_body(const RenderArgs &a, Path &ps, const Hit &h, bool act,
                                                unsigned long long &done, unsigned long long &dropped, uint32_t *lds,
                                                unsigned long long *diag_rounds)
{
    // hit, shade and material tables are in slot order (spt_accel.cpp)
    const float4 *__restrict__ hit = a.scene.accel.slots;
    const float4 *__restrict__ shade = a.scene.shade;
    const uint32_t *__restrict__ mat = a.scene.mat;
    uint32_t *samples = a.samples;
    uint32_t mode = a.mode;
    uint32_t bounces = a.bounces, code_stride = a.scene.code_stride, code_jmax = a.scene.code_jmax;
    if constexpr (KARG) {
        // render kernels: read at the point of use from the kernarg segment (scalar
        // loads) instead of holding them in SGPRs across the loop
        kargs_t &k = *kernarg_args();
        hit = k.scene.accel.slots;
        shade = k.scene.shade;
        mat = k.scene.mat;
        samples = k.samples;
        mode = k.mode;
        bounces = k.bounces;
        code_stride = k.scene.code_stride;
        code_jmax = k.scene.code_jmax;
    }
    const uint32_t idx = h.idx;
    bool fin = false;
    uint32_t word = kZeroWord;  // the sample's code (spt_internal.h code_word)
    const bool dl = ps.phase == PH_DLOOP;
    uint32_t m = SPT_SKYBOX_ID;
    if (act && idx != kMiss) m = mat[idx];
    bool scatter = false, refr = false;
    if (!act) {
    } else if (dl) {
        // while (--bounceCount && sphereIndex < N), SingleThreadPathTracer.hpp:28
        --ps.bounce;
        const bool end = ps.bounce == 0u || idx == kMiss;
        if (end) {
            // the albedo of the first diffuse hit halved 1 + j times: once at that hit
            // (line 24) and once per further bounce (line 31), j = bounces - bounce - 1
            // (saturated where every albedo of the scene is 0: diffuse_code)
            const uint32_t j = min(bounces - ps.bounce - 1u, code_jmax);
            word = code_word(diffuse_code(j, ps.slot, code_stride));
            fin = true;
        }
        scatter = !end;
        refr = false;
    } else {
        // TraceAndSampleColor material switch, SingleThreadPathTracer.hpp:98-111
        scatter = m == SPT_DIFFUSE_ID || m == SPT_REFLECTIVE_ID;
        refr = m == SPT_REFRACTIVE_ID;
        if (!scatter && !refr) {
            // SampleColorSkybox, lines 11-14: initColor * (d.y + 1) * 0.5, rebuilt by the
            // fold from k = d.y + 1
            word = __float_as_uint(ps.d.y + 1.f);
            fin = true;
        }
    }
    bool spec_event = false;
    // (SAMPLER = false: SPT_DUP attribution's copy of the step, without the sampler)
    const f3 rv_coop = SAMPLER ? coop_ball_vector(ps.st, scatter, lds, diag_rounds) : opaque_v3(mk(0.1f, 0.2f, 0.3f));
    if ((SPT_DUP & 2) && SAMPLER) {
        uint64_t st2 = opaque_v(ps.st);
        const f3 r2 = coop_ball_vector(st2, opaque_v(scatter ? 1u : 0u) != 0u, lds);
        sink_v(r2.x);
        sink_v(r2.y);
        sink_v(r2.z);
        sink_v(st2);
    }
    if (scatter) {
        // contact point + normal + cube-minus-ball vector, shared by the diffuse
        // first hit (lines 23-26), the diffuse loop (30-33) and the mirror (41-43)
        const float4 cs = hit[idx];
        const f3 C = mk(cs.x, cs.y, cs.z);
        ps.o = contact(ps.o, ps.d, h.t);
        const f3 nrm = normalize(sub(ps.o, C));
        f3 rv = rv_coop;
        f3 base;
        if (dl) {
            base = add(ps.o, nrm);  // origin + normal (+ rv), line 32; colour *= 0.5 (line 31) in the code
        } else if (m == SPT_DIFFUSE_ID) {
            ps.slot = idx;  // colour = albedo * 0.5 (line 24), in the code
            base = nrm;
            ps.phase = PH_DLOOP;
        } else {
            base = reflect(ps.d, nrm);
            rv = mul(rv, shade[idx].w);
            spec_event = true;
        }
        ps.d = normalize(add(base, rv));
    }
    if (refr) {
        ps.o = contact(ps.o, ps.d, h.t);
        if (SPT_DUP & 256) {
            Path p2 = ps;
            p2.o = opaque_v3(p2.o);
            refract_event(hit, p2, idx);
            sink_v(p2.d.x);
            sink_v(p2.o.x);
            sink_v(p2.st);
        }
        refract_event(hit, ps, idx);
        spec_event = true;
    }
    finish_step<WT>(mode, samples, ps, fin, spec_event, refr, !dl, word, done, dropped);
}
template <bool KARG = false, bool WT = false>
__device__ __forceinline__ void shade_step(const RenderArgs &a, Path &ps, const Hit &h, bool act,
                                           unsigned long long &done, unsigned long long &dropped, uint32_t *lds,
                                           unsigned long long *diag_rounds = nullptr)
{
    if (SPT_DUP & 128) {
        // attribution: the shading step less the sampler, a second time on a copy of the path
        // (its sample stores go to an opaque null-offset copy of the same words: same values)
        Path p2 = ps;
        p2.o = opaque_v3(p2.o);
        p2.d = opaque_v3(p2.d);
        Hit h2 = h;
        h2.t = opaque_v(h2.t);
        unsigned long long d2 = 0, x2 = 0;
        shade_step_body<KARG, WT, false>(a, p2, h2, act, d2, x2, lds, nullptr);
        sink_v(p2.o.x);
        sink_v(p2.d.x);
        sink_v(p2.st);
    }
    shade_step_body<KARG, WT, true>(a, ps, h, act, done, dropped, lds, diag_rounds);
}


// Start the path of batch item `mine`: its (pixel, sample), keyed RNG stream and
// primary ray (SingleThreadPathTracer.hpp:123-130).  rw, rh: shared reciprocals
// of g_width, g_height (div_core); `rows` = rows of the region.

__device__ __forceinline__ void start_path(const RenderArgs &a, uint32_t mine, uint32_t rows, const Recip &rw,
                                           const Recip &rh, const f3 &eye, Path &ps, uint32_t *pxy = nullptr)
{
    // primary ray, SingleThreadPathTracer.hpp:123-130.  A claim of
    // consecutive items stays inside one 8x8 tile (ts_item).
    uint32_t sl, lr, cx;
    ts_item(mine, a.map.width, rows, a.spp_batch, a.div_band, a.div_tile, sl, lr, cx);
    const uint32_t s = a.s0 + sl;
    ps.item = mine;  // slots in item order (ts_slot_base)
    const uint32_t x = a.map.x0 + cx;
    const uint32_t y = a.map.parts == 1u ? a.map.y0 + lr : row_of_fast(a.map, lr, a.div_strip);
    if (pxy) *pxy = (y << 16) | x;  // the primary batch's candidate-list lookup (prim_list_cast)
    ps.st = fmix64(a.seed_key ^ (((uint64_t)(y * a.width + x) << 32) | (uint64_t)s));
    const float un = (float)y + uniform(ps.st, -1.f, 1.f);
    const float vn = (float)x + uniform(ps.st, -1.f, 1.f);
    float u = div_core(un, rw), v = div_core(vn, rh);  // / g_width, / g_height
    if (__builtin_expect(!(div_operand_ok(un) && div_operand_ok(vn)), 0)) {
        u = un / (float)a.width;
        v = vn / (float)a.height;
    }
    const float vx = -1.f + 2.f * v, vy = -1.f + 2.f * u;
    const float *m = a.cam.view;
    ps.d = normalize(mk((m[0] * vx + m[1] * vy) + (m[2] * 1.f + m[3] * 0.f),
                        (m[4] * vx + m[5] * vy) + (m[6] * 1.f + m[7] * 0.f),
                        (m[8] * vx + m[9] * vy) + (m[10] * 1.f + m[11] * 0.f)));
    ps.o = eye;
    ps.phase = PH_TRACE;
    ps.bounce = a.bounces;
    ps.spec = 0;
}

// start_path with the refill parameters copied out of the kernarg segment at the
// point of use (scalar loads); render_kernel only.
__device__ __forceinline__ void start_path_kernarg(uint32_t mine, uint32_t rows, Path &ps, uint32_t *pxy = nullptr)
{
    kargs_t &k = *kernarg_args();
    RenderArgs a;
    a.map = RowMap{k.map.y0, k.map.y1, k.map.strip, k.map.parts, k.map.part, k.map.x0, k.map.width};
    a.width = k.width;
    a.height = k.height;
    a.bounces = k.bounces;
    a.npix = k.npix;
    a.n_items = k.n_items;
    a.spp_batch = k.spp_batch;
    a.s0 = k.s0;
    a.seed_key = k.seed_key;
    a.div_band = FastDiv{k.div_band.d, k.div_band.m, k.div_band.s};
    a.div_tile = FastDiv{k.div_tile.d, k.div_tile.m, k.div_tile.s};
    a.div_strip = FastDiv{k.div_strip.d, k.div_strip.m, k.div_strip.s};
#pragma unroll
    for (int q = 0; q < 12; ++q) a.cam.view[q] = k.cam.view[q];
    start_path(a, mine, rows, recip((float)a.width), recip((float)a.height),
               mk(k.cam.eye[0], k.cam.eye[1], k.cam.eye[2]), ps, pxy);
}

// Batched launches (RenderArgs::rects): the rectangle holding item `nb` (the first
// item of a claim; claims never span two rectangles), by binary search over the
// rectangles' item_off with scalar loads (nb is wave-uniform).
typedef __attribute__((address_space(4))) const BatchRect crect_t;
__device__ __forceinline__ uint32_t find_rect(uint32_t nb)
{
    kargs_t &k = *kernarg_args();
    crect_t *r = k.inline_rects ? (crect_t *)k.rects_inline : (crect_t *)k.rects;
    uint32_t lo = 0, hi = k.n_rects;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (r[mid].item_off <= nb) lo = mid; else hi = mid;
    }
    return lo;
}

// start_path for item `mine` of a batched launch, in rectangle `ri` (wave-uniform):
// the rectangle's own region, item order and slot range.  Items past its item_end
// (claim padding) start nothing: the lane stays idle.
__device__ __forceinline__ void start_path_rect(uint32_t mine, uint32_t ri, Path &ps, uint32_t *pxy = nullptr)
{
    kargs_t &k = *kernarg_args();
    crect_t &r = (k.inline_rects ? (crect_t *)k.rects_inline : (crect_t *)k.rects)[ri];
    if (mine >= r.item_end) return;
    RenderArgs a;
    a.map = RowMap{r.y0, r.y0 + r.rows, 1u, 1u, 0u, r.x0, r.w};
    a.width = k.width;
    a.height = k.height;
    a.bounces = k.bounces;
    a.npix = r.npix;
    a.spp_batch = k.spp_batch;
    a.s0 = k.s0;
    a.seed_key = k.seed_key;
    a.div_band = FastDiv{r.div_band.d, r.div_band.m, r.div_band.s};
    a.div_tile = FastDiv{r.div_tile.d, r.div_tile.m, r.div_tile.s};
    a.div_strip = FastDiv{1u, 0u, 0u};
#pragma unroll
    for (int q = 0; q < 12; ++q) a.cam.view[q] = k.cam.view[q];
    start_path(a, mine - r.item_off, r.rows, recip((float)a.width), recip((float)a.height),
               mk(k.cam.eye[0], k.cam.eye[1], k.cam.eye[2]), ps, pxy);
    ps.item += r.slot_off;
}

// start_path for session item `mine` of the render service: the job's fields from the
// wave's LDS copy of its record (SvcJob words, wave-uniform), the session's constants
// from the kernel arguments.  Items past the job's item_end (claim padding) start nothing.
__device__ __forceinline__ void start_path_svc(uint32_t mine, const uint32_t *rec, Path &ps, uint32_t *pxy = nullptr)
{
    auto f = [&](int i) -> uint32_t { return (uint32_t)__builtin_amdgcn_readfirstlane(rec[i]); };
    if (mine >= f(1)) return;
    kargs_t &k = *kernarg_args();
    RenderArgs a;
    a.map = RowMap{f(8), f(9), f(10), f(11), f(12), f(13), f(14)};
    a.width = k.width;
    a.height = k.height;
    a.bounces = k.bounces;
    a.spp_batch = f(5);
    a.s0 = f(6);
    a.seed_key = k.seed_key;
    a.div_band = FastDiv{f(15), f(16), f(17)};
    a.div_tile = FastDiv{f(18), f(19), f(20)};
    a.div_strip = FastDiv{f(21), f(22), f(23)};
#pragma unroll
    for (int q = 0; q < 12; ++q) a.cam.view[q] = k.cam.view[q];
    start_path(a, mine - f(0), f(4), recip((float)a.width), recip((float)a.height),
               mk(k.cam.eye[0], k.cam.eye[1], k.cam.eye[2]), ps, pxy);
    ps.item += f(2);
    ps.job = f(3);
}

}  // namespace
}  // namespace spt
