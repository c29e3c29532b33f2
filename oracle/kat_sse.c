/* Known-answer test: pins the oracle's Vec4 arithmetic (Math.hpp:107-187) against
 * the SSE4.1 intrinsics the reference itself uses: _mm_dp_ps(...,0xF1),
 * 2x _mm_hadd_ps, _mm_sqrt_ps, _mm_div_ps.  TEST INFRASTRUCTURE ONLY. */
#include <smmintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "spt_oracle.h"

static uint64_t rs = 0x1234567ULL;
static uint32_t rnd32(void) { rs = rs * 6364136223846793005ULL + 1442695040888963407ULL; return (uint32_t)(rs >> 32); }
static float rndf(int mode)
{
    uint32_t u = rnd32();
    float f;
    switch (mode) {
    case 0: f = ((float)(u >> 8) / 16777216.0f) * 2.0f - 1.0f; break;          /* [-1,1) */
    case 1: f = ((float)(u >> 8) / 16777216.0f) * 2000.0f - 1000.0f; break;    /* wide */
    case 2: memcpy(&f, &u, 4); if (f != f || f - f != 0) f = 0.5f; break;    /* any finite bits */
    default: f = (u & 1) ? -0.0f : 0.0f; break;                                 /* signed zeros */
    }
    return f;
}
static int same(const float *a, const float *b, int n) { return memcmp(a, b, sizeof(float) * n) == 0; }

static float sse_dot(__m128 a, __m128 b) { float r[4]; _mm_storeu_ps(r, _mm_dp_ps(a, b, 0xF1)); return r[0]; }
static float sse_lensq(__m128 v) { v = _mm_mul_ps(v, v); v = _mm_hadd_ps(v, v); v = _mm_hadd_ps(v, v); return _mm_cvtss_f32(v); }
static __m128 sse_norm(__m128 v)
{
    __m128 l = _mm_mul_ps(v, v); l = _mm_hadd_ps(l, l); l = _mm_hadd_ps(l, l); l = _mm_sqrt_ps(l);
    return _mm_div_ps(v, l);
}

int main(void)
{
    long checked = 0, bad = 0;
    for (int it = 0; it < 400000; ++it) {
        int mode = it % 4 == 3 ? (it % 8 == 7 ? 3 : 0) : it % 3;
        float a[4], b[4], m[16], o1[4], o2[4];
        for (int i = 0; i < 4; ++i) { a[i] = rndf(mode); b[i] = rndf(mode == 3 ? 0 : mode); }
        if (it & 1) { a[3] = 0.0f; b[3] = 0.0f; }  /* the reference's w lanes are 0 */
        for (int i = 0; i < 16; ++i) m[i] = rndf(mode == 2 ? 1 : mode);
        __m128 va = _mm_loadu_ps(a), vb = _mm_loadu_ps(b);
        float d1 = spo_dot(a, b), d2 = sse_dot(va, vb);
        float l1 = spo_length_squared(a), l2 = sse_lensq(va);
        checked += 2; bad += !same(&d1, &d2, 1); bad += !same(&l1, &l2, 1);
        spo_normalize(a, o1); _mm_storeu_ps(o2, sse_norm(va)); checked++; bad += !same(o1, o2, 4);
        /* Reflect: vec - normal * Dot(vec, normal) * 2.f  (Math.hpp:156-159) */
        spo_reflect(a, b, o1);
        {
            __m128 t = _mm_mul_ps(_mm_mul_ps(vb, _mm_set1_ps(sse_dot(va, vb))), _mm_set1_ps(2.f));
            _mm_storeu_ps(o2, _mm_sub_ps(va, t));
        }
        checked++; bad += !same(o1, o2, 4);
        /* Mat4 * Vec4: four dpps (Math.hpp:178-186) */
        spo_matvec(m, a, o1);
        for (int r = 0; r < 4; ++r) o2[r] = sse_dot(_mm_loadu_ps(m + 4 * r), va);
        checked++; bad += !same(o1, o2, 4);
    }
    printf("kat_sse checked=%ld mismatches=%ld\n", checked, bad);
    return bad ? 1 : 0;
}
