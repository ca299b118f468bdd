// Exactness checks of the decode prologue's fast arithmetic (wf_device.h div_rn / act_scale_f /
// quant8) against the IEEE sequences they replace, on the host (fmaf = correctly rounded fma):
//   gcc -O2 -mfma -o check_fast_arith tools/check_fast_arith.c -lm && ./check_fast_arith [scale]
// scale (default 1.0) multiplies the random sample counts (tests/test_fast_arith_cpu.py uses 0.02).
// Prints the mismatch counts; exit status 1 on any mismatch.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t rs = 88172645463325252ull;
static uint64_t xr(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
static float markstein(float a, float b, float yb) {  // RN(a/b), yb = RN(1/b)
    float q = a * yb;
    float r = fmaf(-q, b, a);
    return fmaf(r, yb, q);
}
static float act_scale_ref(float m) { double md = m; if (md < 1e-6) md = 1.0; return (float)(md / 127.0); }
static float act_scale_new(float m) {
    const float lim = 9.99999997e-07f;  // float(1e-6) < 1e-6: m <= lim <=> double(m) < 1e-6
    if (m <= lim) return u2f(f2u((float)(1.0 / 127.0)));
    return markstein(m, 127.0f, 1.0f / 127.0f);
}
static int8_t q_ref(float x, float sf) { float v = rintf(x / sf); v = fminf(fmaxf(v, -128.f), 127.f); return (int8_t)(int)v; }
// fast code + exact check (branch-free form used on the slow path)
static int8_t q_exact(float x, float sf, float inv) {
    float v = rintf(markstein(x, sf, inv));
    v = fminf(fmaxf(v, -128.f), 127.f);
    return (int8_t)(int)v;
}
int main(int argc, char** argv) {
    const double scale = argc > 1 ? atof(argv[1]) : 1.0;
    const long n_div = (long)(20000000 * scale), n_q = (long)(200000000 * scale);
    // 1) a / K by Markstein for K in the model's sizes, random a (sums of squares: positive)
    int Ks[] = {512, 640, 768, 2560, 6912, 128, 1024, 4096};
    long bad = 0, n = 0;
    for (int ki = 0; ki < 8; ++ki) {
        float K = (float)Ks[ki], y = 1.0f / K;
        for (long i = 0; i < n_div; ++i) {
            uint32_t u = (uint32_t)(xr() & 0x7fffffffu);
            float a = u2f(u);
            if (!isfinite(a) || a < 1e-30f || a > 1e30f) continue;
            ++n;
            if (f2u(markstein(a, K, y)) != f2u(a / K)) { if (bad < 5) printf("div K=%g a=%a\n", K, a); ++bad; }
        }
    }
    printf("markstein a/K: %ld mismatches of %ld\n", bad, n);
    long total = bad;
    // 2) act scale: every positive bf16 m
    bad = 0;
    for (uint32_t h = 0; h < 0x7f80; ++h) {
        float m = u2f(h << 16);
        if (f2u(act_scale_new(m)) != f2u(act_scale_ref(m))) { if (bad < 5) printf("scale m=%a\n", m); ++bad; }
    }
    // all floats near 1e-6 too
    for (uint32_t u = f2u(9.9e-7f); u < f2u(1.01e-6f); ++u) {
        float m = u2f(u);
        if (f2u(act_scale_new(m)) != f2u(act_scale_ref(m))) { if (bad < 10) printf("scale m=%a\n", m); ++bad; }
    }
    printf("act scale: %ld mismatches\n", bad);
    total += bad;
    // 3) quantizer: random bf16 x with s from a random bf16 max, plus constructed near-ties
    bad = 0; n = 0; long bad2 = 0;
    for (long i = 0; i < n_q; ++i) {
        float m = u2f((uint32_t)((0x3000u + (xr() % 0x1800u)) << 16));  // ~2^-31 .. 2^17
        float sf = act_scale_ref(m);
        float inv = 1.0f / sf;
        float x;
        if (i & 1) { x = u2f((uint32_t)(f2u(m) & 0xffff0000u) - (uint32_t)((xr() % 0x800u) << 16)); if (xr() & 1) x = -x; }
        else { // near a half-integer: (k + 0.5) * sf rounded to bf16 +- a few ulps
            float k = (float)((int)(xr() % 255) - 127);
            float t = (k + 0.5f) * sf;
            x = u2f((f2u(t) & 0xffff0000u) + ((uint32_t)((int)(xr() % 5) - 2) << 16));
            if (!(fabsf(x) <= m)) continue;
        }
        ++n;
        if (q_exact(x, sf, inv) != q_ref(x, sf)) { if (bad < 5) printf("q x=%a sf=%a\n", x, sf); ++bad; }
        float invp = u2f(f2u(inv) + 1), invm = u2f(f2u(inv) - 1);
        if (q_exact(x, sf, invp) != q_ref(x, sf)) { if (bad2 < 5) printf("q+ x=%a sf=%a\n", x, sf); ++bad2; }
        if (q_exact(x, sf, invm) != q_ref(x, sf)) { if (bad2 < 5) printf("q- x=%a sf=%a\n", x, sf); ++bad2; }
    }
    printf("quantizer: %ld mismatches of %ld (inv +-1 ulp: %ld)\n", bad, n, bad2);
    total += bad + bad2;
    // 4) exhaustive over x: EVERY bf16 x with |x| <= m, for a sweep of bf16 maxima m (every
    //    1/scale-th one of 2^-31 .. 2^17), with the reciprocal RN(1/sf) and +-1 ulp -- the prologue
    //    forms 1/sf as v_rcp_f32 + one Newton step, within 1 ulp of RN(1/sf) (wf_device.h rcp_1ulp)
    long bad3 = 0, n3 = 0;
    const uint32_t mstep = scale >= 1.0 ? 1u : (uint32_t)(1.0 / scale);
    for (uint32_t hm = 0x3000u; hm < 0x4800u; hm += mstep) {
        const float m = u2f(hm << 16), sf = act_scale_ref(m), inv = 1.0f / sf;
        const float invs[3] = {inv, u2f(f2u(inv) + 1), u2f(f2u(inv) - 1)};
        for (uint32_t hx = 0; hx <= hm; ++hx)
            for (uint32_t sg = 0; sg <= 0x8000u; sg += 0x8000u) {
                const float x = u2f((hx | sg) << 16);
                const int8_t r = q_ref(x, sf);
                for (int j = 0; j < 3; ++j)
                    if (q_exact(x, sf, invs[j]) != r) { if (bad3 < 5) printf("qx x=%a sf=%a j=%d\n", x, sf, j); ++bad3; }
                ++n3;
            }
    }
    printf("quantizer, every bf16 x: %ld mismatches of %ld x 3 reciprocals\n", bad3, n3);
    total += bad3;
    return total ? 1 : 0;
}
