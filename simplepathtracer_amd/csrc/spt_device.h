// spt_device.h -- device-side arithmetic of the render loop (gfx950).
//
// Every helper restates one reference function with its exact fp32 operation
// order.  The whole translation unit is compiled with
// -ffp-contract=off (and the pragma below): no FMA contraction, IEEE division
// and sqrt (hipcc's default correctly-rounded f32 div/sqrt), denormals kept.
//
// Vec4 lanes: the reference's w lane is always +-0 (Vec4{x,y,z} initialisers,
// viewMatrix row 3 = 0), so dpps' (x*x'+y*y')+(z*z'+w*w') reduces to
// (x*x'+y*y')+z*z' up to the sign of an all-zero result, which no comparison or
// colour depends on.  The oracle keeps all four lanes; parity tests check both.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spt_powf.h"

#pragma clang fp contract(off)

namespace spt {

// Material ids, Definitions.hpp:7-13
constexpr uint32_t SPT_SKYBOX_ID = 0, SPT_REFLECTIVE_ID = 1, SPT_REFRACTIVE_ID = 2, SPT_DIFFUSE_ID = 3;

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
// Math.hpp:16-48
__device__ __forceinline__ f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
// Math.hpp:50-64
__device__ __forceinline__ f3 mul(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 neg(f3 a) { return f3{-a.x, -a.y, -a.z}; }
// Math.hpp:107-111 (_mm_dp_ps 0xF1)
__device__ __forceinline__ float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
// Math.hpp:122-133 (mul + 2x hadd)
__device__ __forceinline__ float lensq(f3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }
// Correctly rounded sqrt for arguments known to be normal and positive (the
// hit test only takes the root of r*r - d2 > 1e-3): v_sqrt_f32 (<= 1 ulp) plus
// the residual correction hipcc emits for sqrtf, without its denormal scaling
// (which applies below 2^-96 only) and its +-0/+inf pass-through.
__device__ __forceinline__ float sqrt_pos_normal(float h)
{
    float s = __builtin_amdgcn_sqrtf(h);
    const float dn = __builtin_bit_cast(float, __builtin_bit_cast(int, s) - 1);
    const float up = __builtin_bit_cast(float, __builtin_bit_cast(int, s) + 1);
    const float rdn = __builtin_fmaf(-dn, s, h);
    const float rup = __builtin_fmaf(-up, s, h);
    s = rdn <= 0.0f ? dn : s;
    s = rup > 0.0f ? up : s;
    return s;
}

// IEEE f32 division without div_scale / div_fixup.  hipcc lowers `a / b` to
//   div_scale(b), rcp, e = fma(-b, rc, 1), rc = fma(e, rc, rc), q = a * rc,
//   r = fma(-b, q, a), q = fma(r, rc, q), r = fma(-b, q, a),
//   div_fmas(r, rc, q), div_fixup.
// For |a| in [2^-40, 2^40] and |b| in [2^-40, 2^42] (both normal, exponent gap
// < 96, quotient normal, no overflow) div_scale returns its operand with VCC = 0,
// div_fmas is then a plain fma and div_fixup returns the quotient unchanged
// (CDNA ISA, V_DIV_SCALE/FMAS/FIXUP_F32), so the core below is bit-identical.
// The reciprocal refinement depends on b only and is shared by equal divisors.
struct Recip {
    float b, rc;
};
__device__ __forceinline__ Recip recip(float b)
{
    float rc = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, rc, 1.0f);
    rc = __builtin_fmaf(e, rc, rc);
    return Recip{b, rc};
}
__device__ __forceinline__ float div_core(float a, Recip r)
{
    float q = a * r.rc;
    float e = __builtin_fmaf(-r.b, q, a);
    q = __builtin_fmaf(e, r.rc, q);
    e = __builtin_fmaf(-r.b, q, a);
    return __builtin_fmaf(e, r.rc, q);
}
__device__ __forceinline__ bool div_operand_ok(float x)
{
    const float ax = __builtin_fabsf(x);
    return ax >= 0x1p-40f && ax <= 0x1p40f;  // false for 0, inf, NaN
}
// a / b (IEEE): the core when both operands are in range (b <= 2^40 here), the
// full sequence on the lanes that are not.
__device__ __forceinline__ float div_rn(float a, float b)
{
    float q = div_core(a, recip(b));
    if (__builtin_expect(!(div_operand_ok(a) && div_operand_ok(b)), 0)) q = a / b;
    return q;
}

// Math.hpp:140-154: v / sqrt(|v|^2), lane-wise IEEE division.  Components in
// [2^-40, 2^40] give |v|^2 in [2^-80, 2^82) (unscaled sqrt path) and a divisor in
// [2^-40, 2^41], inside div_core's range; other lanes take the full sequences.
__device__ __forceinline__ f3 normalize(f3 a)
{
    const float L = lensq(a);
    const Recip r = recip(sqrt_pos_normal(L));
    f3 out = f3{div_core(a.x, r), div_core(a.y, r), div_core(a.z, r)};
    if (__builtin_expect(!(div_operand_ok(a.x) && div_operand_ok(a.y) && div_operand_ok(a.z)), 0)) {
        const float l = __builtin_sqrtf(L);
        out = f3{a.x / l, a.y / l, a.z / l};
    }
    return out;
}
// Math.hpp:156-159: vec - normal * Dot(vec, normal) * 2.f
__device__ __forceinline__ f3 reflect(f3 v, f3 n) { return sub(v, mul(mul(n, dot(v, n)), 2.0f)); }

// ---------------------------------------------------------------------------
// RNG: Random.hpp:30-36 splitmix mixer on a keyed counter stream.
// ---------------------------------------------------------------------------
constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t fmix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t next_u32(uint64_t &st)
{
    st += kGamma;
    uint64_t z = st;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((z ^ (z >> 31)) >> 31);
}

// libstdc++ generate_canonical<float,24> + uniform_real_distribution (Random.hpp:86-93):
// float(u)/2^32 (exact scaling), clamp >= 1 to nextafter(1,0), then u*(b-a)+a.
__device__ __forceinline__ float canon_u32(uint32_t bits)
{
    float u = (float)bits * 2.3283064365386963e-10f;  // * 2^-32, exact
    return u >= 1.0f ? 0x1.fffffep-1f : u;  // nextafterf(1, 0)
}
// uniform(a, b) from the raw draw.  Every call site has a power-of-two width b - a (1
// or 2), so canon * (b - a) is exact and the reference's two roundings (the product
// is exact, the add rounds once) are one FMA: fl(canon * w + a) == fma(f, 2^-32 w, a)
// with f = float(bits).  The clamp moves onto f: f == 2^32 exactly when canon == 1.
__device__ __forceinline__ float uniform_bits(uint32_t bits, float a, float b)
{
    const float f = __builtin_fminf((float)bits, 0x1.fffffep+31f);
    return __builtin_fmaf(f, 0x1p-32f * (b - a), a);
}
__device__ __forceinline__ float uniform(uint64_t &st, float a, float b) { return uniform_bits(next_u32(st), a, b); }

// Random.hpp:115-127 (== 129-141), x, y, z ~ U(-0.5,0.5) while Length < 0.5, is
// coop_ball_vector (spt_path.h).  sqrt_rn is monotone and sqrt_rn(0.25) == 0.5,
// sqrt_rn(prev(0.25)) < 0.5, so `sqrtf(L) < 0.5f` <=> `L < 0.25f` (checked in tests).

// ---------------------------------------------------------------------------
// Refraction helpers (SingleThreadPathTracer.hpp:48-92).  In the reference's
// translation unit pow(float, float) and sqrt(float) bind to the float overloads
// (the stb implementations included by IOHelpers.hpp:5-9 bring libstdc++'s
// <math.h> wrapper; oracle/probe_overloads.cpp), so everything here is float:
// glibc's powf restated bit for bit (spt_powf.h, exhaustively pinned) and the
// correctly rounded sqrtf.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float pow5f(float x) { return spt_glibc_powf(x, 5.f); }

// rSq + (1 - rSq) * pow(1 - c, 5)  (lines 58-59, 75-76)
__device__ __forceinline__ float schlick(float rsq, float c) { return rsq + (1.f - rsq) * pow5f(1.f - c); }

// direction * r + n * (r*c - sqrt(1 - r*r*(1 - c*c)))  (lines 68, 84)
__device__ __forceinline__ float refract_k(float r, float c) { return r * c - __builtin_sqrtf(1.f - r * r * (1.f - c * c)); }
__device__ __forceinline__ f3 refract_dir(f3 d, f3 n, float r, float c)
{
    return normalize(add(mul(d, r), mul(n, refract_k(r, c))));
}

// r * sqrt(1 - c*c) < 1  (lines 66, 82)
__device__ __forceinline__ bool no_tir(float r, float c) { return r * __builtin_sqrtf(1.f - c * c) < 1.f; }

// IOHelpers.hpp:17-22 + x86 cvttss2si semantics of static_cast<uint8_t>(float)
__device__ __forceinline__ uint8_t f2u8(float v)
{
    if (!(v > -2147483648.0f && v < 2147483648.0f)) return 0;
    return (uint8_t)(int32_t)v;
}
__device__ __forceinline__ uint8_t gamma_byte(float c)
{
    return f2u8(__builtin_roundf(__builtin_sqrtf(c / 255.f) * 255.f));
}

}  // namespace spt
