/*
 * Julia Base's Float64 elementary functions as the reference evaluates them — one
 * implementation compiled into both the product (HIP device code, gfx950) and the CPU oracle
 * (plain C), so the exact evaluator and the oracle compute the same bits per sample.
 *
 * The reference calls, per sample and per χ² evaluation (FerreolS/GPPupilDemodulation.jl):
 *   sin(ω t + ϕ)                                    src/Modulation.jl:137 → jl_sin
 *   exp(ȷ b sin(…)) = exp(Complex(±0, β)) → sincos(β)                 :137 → jl_sincos
 *   exp.(im .* angle.(FC)), angle(z) = atan(imag z, real z)           :388 → jl_atan2 + jl_sincos
 *   angle(a) in getphase and the output pass               :66-69, 419-421 → jl_atan2
 *   abs(::Complex) = hypot in mean(abs, …), var(abs, …)  src/Faint.jl:95-97 → jl_hypot
 * and OptimPackNextGen's NEWUOA (pure Julia) takes cos/sin of its trial angles → jl_cos, jl_sin.
 *
 * Restated from Julia Base (base/special/trig.jl, base/special/rem_pio2.jl, base/math.jl: the
 * msun/FreeBSD-derived implementations of Julia 1.6-1.11; the reference pins no Julia version):
 * Cody–Waite reduction by π/2 with two constants (|x| ≲ 9π/4) or three (|x| < 2^20·π/2), the
 * Payne–Hanek reduction with 1/(2π) in 64-bit words beyond (MJD-scale timestamps: ω t ≈ 3.3e10),
 * msun's sin/cos kernel polynomials on the double-double remainder, msun's atan/atan2 and Julia's
 * fma-corrected hypot.  Julia's `muladd` and `@horner` contract to an FMA on x86-64 hosts with
 * FMA (every CPU the reference runs on today); they are explicit fma() here, everything else is
 * unfused (build with -ffp-contract=off).  sin/cos of ±Inf throw DomainError in Julia; here they
 * return NaN (the fit's NaN status then marks the series).
 *
 * Parity of this restatement with Julia itself is UNPINNED (no Julia in the build container);
 * tests/test_jlmath.py checks it against correctly rounded values and glibc on the CPU, and on
 * the GPU that device and host evaluations agree bit for bit.
 */
#ifndef GPD_JLMATH_H
#define GPD_JLMATH_H

#include <stdint.h>

#if defined(__HIP__)
#define JLM_FN static __host__ __device__ inline __attribute__((always_inline))
#else
#define JLM_FN static inline
#endif

typedef unsigned __int128 jlm_u128;
typedef __int128 jlm_i128;

JLM_FN uint64_t jlm_bits(double x) {
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    return u;
}
JLM_FN double jlm_from_bits(uint64_t u) {
    double x;
    __builtin_memcpy(&x, &u, 8);
    return x;
}
JLM_FN uint32_t jlm_highword(double x) { return (uint32_t)(jlm_bits(x) >> 32); }
JLM_FN uint32_t jlm_poshighword(double x) { return jlm_highword(x) & 0x7fffffffu; }
JLM_FN double jlm_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

/* ---- argument reduction (base/special/rem_pio2.jl) -------------------------------------- */

/* 1/(2π) in 64-bit words, most significant first: 1/(2π) = Σ_i W_i 2^(-64(i+1)), i = 0..18
 * (oracle/tools/inv2pi.py derives them from an exact integer expansion of π).  An indexed table
 * (device: constant memory) — a switch compiled to ~200 compare-and-branch instructions per
 * Payne–Hanek reduction on the device. */
#define JLM_INV2PI_WORDS                                                                      \
    {0x28be60db9391054aull, 0x7f09d5f47d4d3770ull, 0x36d8a5664f10e410ull,                    \
     0x7f9458eaf7aef158ull, 0x6dc91b8e909374b8ull, 0x01924bba82746487ull,                    \
     0x3f877ac72c4a69cfull, 0xba208d7d4baed121ull, 0x3a671c09ad17df90ull,                    \
     0x4e64758e60d4ce7dull, 0x272117e2ef7e4a0eull, 0xc7fe25fff7816603ull,                    \
     0xfbcbc462d6829b47ull, 0xdb4d9fb3c9f2c26dull, 0xd3d18fd9a797fa8bull,                    \
     0x5d49eeb1faf97c5eull, 0xcf41ce7de294a4baull, 0x9afed7ec47e35742ull,                    \
     0x1580cc11bf1edaeaull}
#if defined(__HIP__)
__device__ __constant__ static const uint64_t jlm_inv2pi_dev[19] = JLM_INV2PI_WORDS;
#endif
static const uint64_t jlm_inv2pi_host[19] = JLM_INV2PI_WORDS;
JLM_FN uint64_t jlm_inv2pi(int i) {
    if (i < 0 || i > 18) return 0;
#if defined(__HIP_DEVICE_COMPILE__)
    return jlm_inv2pi_dev[i];
#else
    return jlm_inv2pi_host[i];
#endif
}

/* Julia's shifts: a negative count shifts the other way, a count ≥ the width gives 0 */
JLM_FN jlm_u128 jlm_shr128(jlm_u128 x, int n) {
    if (n >= 0) return n >= 128 ? (jlm_u128)0 : x >> n;
    return -n >= 128 ? (jlm_u128)0 : x << (-n);
}
JLM_FN jlm_u128 jlm_shl128(jlm_u128 x, int n) { return jlm_shr128(x, -n); }
JLM_FN int jlm_clz128(jlm_u128 x) {
    const uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;
    if (hi) return __builtin_clzll(hi);
    if (lo) return 64 + __builtin_clzll(lo);
    return 128;
}

/* fromfraction(f::Int128): (z1, z2) with z1 + z2 ≈ f / 2^128, z1 cut to 26 significant bits */
JLM_FN void jlm_fromfraction(jlm_i128 f, double *z1, double *z2) {
    if (f == 0) {
        *z1 = 0.0;
        *z2 = 0.0;
        return;
    }
    const uint64_t s = (uint64_t)(f < 0) << 63;
    const jlm_u128 x = f < 0 ? (jlm_u128)0 - (jlm_u128)f : (jlm_u128)f; /* abs(f) % UInt128 */
    const int n1 = 128 - jlm_clz128(x);
    const uint64_t m1 = (uint64_t)jlm_shr128(x, n1 - 26) << 27;
    const uint64_t d1 = (uint64_t)(int64_t)(n1 - 128 + 1021) << 52;
    *z1 = jlm_from_bits(s | (d1 + m1));
    const jlm_u128 x2 = x - jlm_shl128((jlm_u128)m1, n1 - 53);
    if (x2 == 0) {
        *z2 = 0.0;
        return;
    }
    const int n2 = 128 - jlm_clz128(x2);
    const uint64_t m2 = (uint64_t)jlm_shr128(x2, n2 - 53);
    const uint64_t d2 = (uint64_t)(int64_t)(n2 - 128 + 1021) << 52;
    *z2 = jlm_from_bits(s | (d2 + m2));
}

/* paynehanek(x): |x| ≥ 2^20·π/2 */
JLM_FN int jlm_paynehanek(double x, double *yhi, double *ylo) {
    const uint64_t u = jlm_bits(x);
    const uint64_t X = (u & 0x000fffffffffffffull) | (1ull << 52);
    const int k = (int)((u & 0x7ff0000000000000ull) >> 52) - 1023 - 52;
    const int idx = k >> 6; /* floor division (arithmetic shift) */
    const int shift = k - idx * 64;
    uint64_t a1, a2, a3;
    if (shift == 0) {
        a1 = jlm_inv2pi(idx);
        a2 = jlm_inv2pi(idx + 1);
        a3 = jlm_inv2pi(idx + 2);
    } else {
        a1 = (idx < 0 ? 0ull : jlm_inv2pi(idx) << shift) | (jlm_inv2pi(idx + 1) >> (64 - shift));
        a2 = (jlm_inv2pi(idx + 1) << shift) | (jlm_inv2pi(idx + 2) >> (64 - shift));
        a3 = (jlm_inv2pi(idx + 2) << shift) | (jlm_inv2pi(idx + 3) >> (64 - shift));
    }
    const jlm_u128 w1 = (jlm_u128)(X * a1) << 64; /* overflow becomes the integer part */
    const jlm_u128 w2 = (jlm_u128)X * a2;
    const jlm_u128 w3 = ((jlm_u128)X * a3) >> 64;
    jlm_u128 w = w1 + w2 + w3; /* fraction of x / 2π */
    if (__builtin_signbit(x)) w = (jlm_u128)0 - w; /* flipsign(w, x) */
    const int q = (int)(((int64_t)(uint64_t)(w >> 125) + 1) >> 1); /* nearest quadrant */
    const jlm_i128 f = (jlm_i128)(w << 2);                         /* fraction of the quadrant */
    double zhi, zlo;
    jlm_fromfraction(f, &zhi, &zlo);
    const double pio2 = 1.5707963267948966, pio2_hi = 1.5707963407039642,
                 pio2_lo = -1.3909067614167116e-8;
    const double yh = (zhi + zlo) * pio2;
    *yhi = yh;
    *ylo = (((zhi * pio2_hi - yh) + zhi * pio2_lo) + zlo * pio2_hi) + zlo * pio2_lo;
    return q;
}

#define JLM_PIO2_1 1.57079632673412561417e+00
#define JLM_PIO2_1T 6.07710050650619224932e-11
#define JLM_PIO2_2 6.07710050630396597660e-11
#define JLM_PIO2_2T 2.02226624879595063154e-21
#define JLM_PIO2_3 2.02226624871116645580e-21
#define JLM_PIO2_3T 8.47842766036889956997e-32

/* cody_waite_2c_pio2(x, fn, n) */
JLM_FN int jlm_cw2c(double x, double fn, double *yhi, double *ylo) {
    const double z = jlm_fma(-fn, JLM_PIO2_1, x);
    const double y1 = jlm_fma(-fn, JLM_PIO2_1T, z);
    *yhi = y1;
    *ylo = jlm_fma(-fn, JLM_PIO2_1T, z - y1);
    return (int)fn;
}

/* cody_waite_ext_pio2(x, xhp) */
JLM_FN int jlm_cwext(double x, uint32_t xhp, double *yhi, double *ylo) {
    const double fn = __builtin_rint(x * 0x1.45f306dc9c883p-1); /* round(x * (2/π)) */
    double r = jlm_fma(-fn, JLM_PIO2_1, x);
    double w = fn * JLM_PIO2_1T;
    const uint32_t j = xhp >> 20;
    double y1 = r - w;
    uint32_t i = j - ((jlm_highword(y1) >> 20) & 0x7ffu);
    if (i > 16u) { /* 2nd iteration, good to 118 bits */
        double t = r;
        w = fn * JLM_PIO2_2;
        r = t - w;
        w = jlm_fma(fn, JLM_PIO2_2T, -((t - r) - w));
        y1 = r - w;
        i = j - ((jlm_highword(y1) >> 20) & 0x7ffu);
        if (i > 49u) { /* 3rd iteration, 151 bits */
            t = r;
            w = fn * JLM_PIO2_3;
            r = t - w;
            w = jlm_fma(fn, JLM_PIO2_3T, -((t - r) - w));
            y1 = r - w;
        }
    }
    *yhi = y1;
    *ylo = (r - y1) - w;
    return (int)fn; /* unsafe_trunc(Int, fn) */
}

/* rem_pio2_kernel(x) for |x| ≥ π/4: x = n·π/2 + (yhi + ylo) */
JLM_FN int jl_rem_pio2(double x, double *yhi, double *ylo) {
    const uint32_t xhp = jlm_poshighword(x);
    if (xhp <= 0x401c463bu) { /* |x| ≲ 9π/4 */
        /* |x| ≈ π/2 or π (same low 20 high-word bits as π/2), 3π/2, 2π: the precise scheme */
        const int ext = xhp <= 0x400f6a7au ? (xhp & 0xfffffu) == 0x921fbu
                                           : (xhp == 0x4012d97cu || xhp == 0x401921fbu);
        if (!ext) { /* two-constant Cody–Waite with n = ±1..±4 */
            double fn = xhp <= 0x4002d97cu ? 1.0
                        : xhp <= 0x400f6a7au ? 2.0
                        : xhp <= 0x4015fdbcu ? 3.0
                                             : 4.0;
            if (!(x > 0.0)) fn = -fn;
            return jlm_cw2c(x, fn, yhi, ylo);
        }
        return jlm_cwext(x, xhp, yhi, ylo);
    }
    if (xhp < 0x413921fbu) return jlm_cwext(x, xhp, yhi, ylo); /* |x| < 2^20·π/2 */
    return jlm_paynehanek(x, yhi, ylo);
}

/* ---- sin / cos kernels (base/special/trig.jl, msun k_sin.c / k_cos.c) -------------------- */
#define JLM_DS1 -1.66666666666666324348e-01
#define JLM_DS2 8.33333333332248946124e-03
#define JLM_DS3 -1.98412698298579493134e-04
#define JLM_DS4 2.75573137070700676789e-06
#define JLM_DS5 -2.50507602534068634195e-08
#define JLM_DS6 1.58969099521155010221e-10
#define JLM_DC1 4.16666666666666019037e-02
#define JLM_DC2 -1.38888888888741095749e-03
#define JLM_DC3 2.48015872894767294178e-05
#define JLM_DC4 -2.75573143513906633035e-07
#define JLM_DC5 2.08757232129817482790e-09
#define JLM_DC6 -1.13596475577881948265e-11

/* sin_kernel(y::Float64) when `plain` (|x| < π/4, no reduction), sin_kernel(y::DoubleFloat64)
 * otherwise */
JLM_FN double jlm_sin_kernel(double hi, double lo, int plain) {
    const double y2 = hi * hi, y4 = y2 * y2;
    const double r = jlm_fma(y2, jlm_fma(y2, JLM_DS4, JLM_DS3), JLM_DS2) +
                     y2 * y4 * jlm_fma(y2, JLM_DS6, JLM_DS5);
    const double y3 = y2 * hi;
    if (plain) return hi + y3 * (JLM_DS1 + y2 * r);
    return hi - ((y2 * (0.5 * lo - y3 * r) - lo) - y3 * JLM_DS1);
}

/* cos_kernel (the Float64 method is the DoubleFloat64 one at lo = 0) */
JLM_FN double jlm_cos_kernel(double hi, double lo) {
    const double y2 = hi * hi, y4 = y2 * y2;
    const double r = y2 * jlm_fma(y2, jlm_fma(y2, JLM_DC3, JLM_DC2), JLM_DC1) +
                     y4 * y4 * jlm_fma(y2, jlm_fma(y2, JLM_DC6, JLM_DC5), JLM_DC4);
    const double half_y2 = 0.5 * y2;
    const double w = 1.0 - half_y2;
    return w + (((1.0 - w) - half_y2) + (y2 * r - hi * lo));
}

#define JLM_PI_4 0x1.921fb54442d18p-1 /* Float64(π)/4 */

JLM_FN double jl_sin(double x) {
    const double ax = __builtin_fabs(x);
    if (ax < JLM_PI_4) {
        if (ax < 0x1p-26) return x; /* sqrt(eps(Float64)) */
        return jlm_sin_kernel(x, 0.0, 1);
    }
    if (__builtin_isnan(x) || __builtin_isinf(x)) return x - x;
    double hi, lo;
    const int n = jl_rem_pio2(x, &hi, &lo) & 3;
    if (n == 0) return jlm_sin_kernel(hi, lo, 0);
    if (n == 1) return jlm_cos_kernel(hi, lo);
    if (n == 2) return -jlm_sin_kernel(hi, lo, 0);
    return -jlm_cos_kernel(hi, lo);
}

JLM_FN double jl_cos(double x) {
    const double ax = __builtin_fabs(x);
    if (ax < JLM_PI_4) {
        if (ax < 0x1.6a09e667f3bcdp-27) return 1.0; /* sqrt(eps(Float64)/2) */
        return jlm_cos_kernel(x, 0.0);
    }
    if (__builtin_isnan(x) || __builtin_isinf(x)) return x - x;
    double hi, lo;
    const int n = jl_rem_pio2(x, &hi, &lo) & 3;
    if (n == 0) return jlm_cos_kernel(hi, lo);
    if (n == 1) return -jlm_sin_kernel(hi, lo, 0);
    if (n == 2) return -jlm_cos_kernel(hi, lo);
    return jlm_sin_kernel(hi, lo, 0);
}

/* sincos(x): both kernels at one reduced argument.  They are evaluated once on (hi, lo, plain)
 * after the reduction — the values Julia's branches give — so the device does not run
 * divergent copies of the polynomials. */
JLM_FN void jl_sincos(double x, double *s, double *c) {
    const double ax = __builtin_fabs(x);
    double hi, lo;
    int n, plain;
    if (ax < JLM_PI_4) {
        if (x == 0.0) {
            *s = x;
            *c = 1.0;
            return;
        }
        hi = x;
        lo = 0.0;
        n = 0;
        plain = 1;
    } else if (__builtin_isnan(x) || __builtin_isinf(x)) {
        *s = x - x;
        *c = x - x;
        return;
    } else {
        n = jl_rem_pio2(x, &hi, &lo) & 3;
        plain = 0;
    }
    const double si = jlm_sin_kernel(hi, lo, plain), co = jlm_cos_kernel(hi, lo);
    if (n == 0) {
        *s = si;
        *c = co;
    } else if (n == 1) {
        *s = co;
        *c = -si;
    } else if (n == 2) {
        *s = -si;
        *c = -co;
    } else {
        *s = -co;
        *c = si;
    }
}

/* ---- branch-free forms, one argument regime each ----------------------------------------
 * The same operations as jl_sin / jl_sincos above, with every branch of the regime evaluated and
 * the result selected (no control flow), so that a batch of independent arguments compiles to
 * one basic block the scheduler can interleave (the exact evaluator's per-sample model at one
 * wave per SIMD).  The caller tests the regime (jlm_*_in) and otherwise calls the general
 * function; inside its regime each form gives that function's bits. */
JLM_FN uint64_t jlm_inv2pi_nb(int i) {
    const int j = i < 0 ? 0 : (i > 18 ? 18 : i);
#if defined(__HIP_DEVICE_COMPILE__)
    const uint64_t v = jlm_inv2pi_dev[j];
#else
    const uint64_t v = jlm_inv2pi_host[j];
#endif
    return (i < 0 || i > 18) ? 0ull : v;
}
JLM_FN int jlm_clz128_nb(jlm_u128 x) {
    const uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;
    const int ch = __builtin_clzll(hi | 1ull), cl = __builtin_clzll(lo | 1ull);
    return hi ? ch : (lo ? 64 + cl : 128);
}
/* 128-bit left shift by 0 ≤ c < 128 */
JLM_FN jlm_u128 jlm_shl128_nb(jlm_u128 x, int c) { return x << (c & 127); }
/* jlm_fromfraction through normalised forms: y = |f| << clz(|f|) puts the leading bit at 127, so
 * z1's 26 bits are y's top 26 (= |f| >> (n1 - 26)) and the remainder x2 = |f| - (those bits) is
 * y's lower 102 bits >> clz(|f|) — no bit is lost in either shift, so x2's leading 53 bits (z2's
 * truncated mantissa; zero-padded when x2 has fewer) are those of y2 = y mod 2^102 normalised. */
JLM_FN void jlm_fromfraction_nb(jlm_i128 f, double *z1, double *z2) {
    const uint64_t s = (uint64_t)(f < 0) << 63;
    const jlm_u128 x = f < 0 ? (jlm_u128)0 - (jlm_u128)f : (jlm_u128)f;
    const int c = jlm_clz128_nb(x | 1); /* f = 0: any shape, the result is selected */
    const jlm_u128 y = jlm_shl128_nb(x, c);
    const int n1 = 128 - c;
    const uint64_t m1 = (uint64_t)(y >> 102) << 27;
    const uint64_t d1 = (uint64_t)(int64_t)(n1 - 128 + 1021) << 52;
    const jlm_u128 y2 = y & (((jlm_u128)1 << 102) - 1);
    const int c2 = jlm_clz128_nb(y2 | 1);
    const int n2 = 128 - c - c2; /* 128 - clz(x2): clz(x2) = clz(y2) + c */
    const uint64_t m2 = (uint64_t)(jlm_shl128_nb(y2, c2) >> 75);
    const uint64_t d2 = (uint64_t)(int64_t)(n2 - 128 + 1021) << 52;
    *z1 = f == 0 ? 0.0 : jlm_from_bits(s | (d1 + m1));
    *z2 = (f == 0 || y2 == 0) ? 0.0 : jlm_from_bits(s | (d2 + m2));
}
/* Payne–Hanek's three words of 2/π for the binade of biased exponent e (k = e - 1075; shift 0
 * takes the words unshifted) */
JLM_FN void jlm_ph_words(int e, uint64_t *a1, uint64_t *a2, uint64_t *a3) {
    const int k = e - 1023 - 52;
    const int idx = k >> 6;
    const int shift = k - idx * 64;
    const uint64_t v0 = jlm_inv2pi_nb(idx), v1 = jlm_inv2pi_nb(idx + 1),
                   v2 = jlm_inv2pi_nb(idx + 2), v3 = jlm_inv2pi_nb(idx + 3);
    *a1 = (v0 << shift) | ((v1 >> 1) >> (63 - shift));
    *a2 = (v1 << shift) | ((v2 >> 1) >> (63 - shift));
    *a3 = (v2 << shift) | ((v3 >> 1) >> (63 - shift));
}
JLM_FN int jlm_biased_exponent(double x) { return (int)((jlm_bits(x) >> 52) & 0x7ffu); }
/* jlm_paynehanek on x's binade words; regime |x| ≥ 2^20·π/2, finite */
/* Payne–Hanek after the product: wp = the 128-bit fraction of |x|·(2/π)/4 (mod 1), neg = x < 0 */
JLM_FN int jlm_ph_tail(jlm_u128 wp, int neg, double *yhi, double *ylo) {
    const jlm_u128 w = neg ? (jlm_u128)0 - wp : wp;
    const int q = (int)(((int64_t)(uint64_t)(w >> 125) + 1) >> 1);
    const jlm_i128 f = (jlm_i128)(w << 2);
    double zhi, zlo;
    jlm_fromfraction_nb(f, &zhi, &zlo);
    const double pio2 = 1.5707963267948966, pio2_hi = 1.5707963407039642,
                 pio2_lo = -1.3909067614167116e-8;
    const double yh = (zhi + zlo) * pio2;
    *yhi = yh;
    *ylo = (((zhi * pio2_hi - yh) + zhi * pio2_lo) + zlo * pio2_hi) + zlo * pio2_lo;
    return q;
}
JLM_FN int jlm_paynehanek_w(double x, uint64_t a1, uint64_t a2, uint64_t a3, double *yhi,
                            double *ylo) {
    const uint64_t X = (jlm_bits(x) & 0x000fffffffffffffull) | (1ull << 52);
    const jlm_u128 w1 = (jlm_u128)(X * a1) << 64;
    const jlm_u128 w2 = (jlm_u128)X * a2;
    const jlm_u128 w3 = ((jlm_u128)X * a3) >> 64;
    return jlm_ph_tail(w1 + w2 + w3, __builtin_signbit(x), yhi, ylo);
}
JLM_FN int jlm_paynehanek_nb(double x, double *yhi, double *ylo) {
    uint64_t a1, a2, a3;
    jlm_ph_words(jlm_biased_exponent(x), &a1, &a2, &a3);
    return jlm_paynehanek_w(x, a1, a2, a3, yhi, ylo);
}
/* jlm_cwext; regime 9π/4 ≲ |x| < 2^20·π/2 (every iteration evaluated, the needed one kept) */
JLM_FN int jlm_cwext_nb(double x, uint32_t xhp, double *yhi, double *ylo) {
    const double fn = __builtin_rint(x * 0x1.45f306dc9c883p-1);
    const double r1 = jlm_fma(-fn, JLM_PIO2_1, x);
    const double w1 = fn * JLM_PIO2_1T;
    const uint32_t j = xhp >> 20;
    const double y11 = r1 - w1;
    const uint32_t i1 = j - ((jlm_highword(y11) >> 20) & 0x7ffu);
    const double w2a = fn * JLM_PIO2_2;
    const double r2 = r1 - w2a;
    const double w2 = jlm_fma(fn, JLM_PIO2_2T, -((r1 - r2) - w2a));
    const double y12 = r2 - w2;
    const uint32_t i2 = j - ((jlm_highword(y12) >> 20) & 0x7ffu);
    const double w3a = fn * JLM_PIO2_3;
    const double r3 = r2 - w3a;
    const double w3 = jlm_fma(fn, JLM_PIO2_3T, -((r2 - r3) - w3a));
    const double y13 = r3 - w3;
    const int it = i1 > 16u ? (i2 > 49u ? 3 : 2) : 1;
    const double r = it == 1 ? r1 : (it == 2 ? r2 : r3);
    const double w = it == 1 ? w1 : (it == 2 ? w2 : w3);
    const double y1 = it == 1 ? y11 : (it == 2 ? y12 : y13);
    *yhi = y1;
    *ylo = (r - y1) - w;
    return (int)fn;
}
/* jlm_sin_kernel with `plain` a value: both forms evaluated */
JLM_FN double jlm_sin_kernel_sel(double hi, double lo, int plain) {
    const double y2 = hi * hi, y4 = y2 * y2;
    const double r = jlm_fma(y2, jlm_fma(y2, JLM_DS4, JLM_DS3), JLM_DS2) +
                     y2 * y4 * jlm_fma(y2, JLM_DS6, JLM_DS5);
    const double y3 = y2 * hi;
    const double p = hi + y3 * (JLM_DS1 + y2 * r);
    const double d = hi - ((y2 * (0.5 * lo - y3 * r) - lo) - y3 * JLM_DS1);
    return plain ? p : d;
}
JLM_FN double jlm_sin_quadrant(int n, double hi, double lo) {
    const double si = jlm_sin_kernel(hi, lo, 0), co = jlm_cos_kernel(hi, lo);
    n &= 3;
    return n == 0 ? si : (n == 1 ? co : (n == 2 ? -si : -co));
}
/* regimes of jl_sin for |x| ≥ π/4: Payne–Hanek (MJD-scale ωt) and Cody–Waite extended */
JLM_FN int jlm_sin_ph_in(double x) {
    const uint32_t xhp = jlm_poshighword(x);
    return xhp >= 0x413921fbu && xhp < 0x7ff00000u;
}
JLM_FN int jlm_sin_cwx_in(double x) {
    const uint32_t xhp = jlm_poshighword(x);
    return xhp > 0x401c463bu && xhp < 0x413921fbu;
}
JLM_FN double jl_sin_ph_nb(double x) {
    double hi, lo;
    const int n = jlm_paynehanek_nb(x, &hi, &lo);
    return jlm_sin_quadrant(n, hi, lo);
}
/* the same with the binade's words given (arguments sharing one exponent) */
JLM_FN double jl_sin_ph_w(double x, uint64_t a1, uint64_t a2, uint64_t a3) {
    double hi, lo;
    const int n = jlm_paynehanek_w(x, a1, a2, a3, &hi, &lo);
    return jlm_sin_quadrant(n, hi, lo);
}
/* ---- Payne–Hanek of θ = fl(x + ϕ) from a per-sample precomputation of x (r6) -------------
 * The exact evaluator's sin(θ) for MJD-scale phases: x = fl(ω t) is fixed per sample and every
 * evaluation adds one ϕ.  When every x lies in one binade e (mantissa X ∈ [2^52, 2^53), ulp
 * u = 2^(e−1075)) and r = ϕ/u is not a half-integer, θ = x + δ·u with δ = rint(r) for every x
 * (fl(x + ϕ) is the multiple of u nearest x + ϕ) as long as X + δ stays inside the binade — so θ's
 * mantissa is X + δ and Payne–Hanek's products are linear in it:
 *   (X+δ)·a1 mod 2^64 = X·a1 + δ·a1,   (X+δ)·a2 = X·a2 + δ·a2,
 *   ⌊(X+δ)·a3 / 2^64⌋ = ⌊X·a3 / 2^64⌋ + ⌊δ·a3 / 2^64⌋ + carry(X·a3 mod 2^64 + δ·a3 mod 2^64)
 * (all mod 2^128; ⌊·⌋ of the signed δ·a3 is an arithmetic shift).  The table holds per sample
 * W = (X·a1 mod 2^64)·2^64 + X·a2 + ⌊X·a3 / 2^64⌋ and A3 = X·a3 mod 2^64; an evaluation forms
 * K = δ·a1·2^64 + δ·a2 + ⌊δ·a3 / 2^64⌋ and D3 = δ·a3 mod 2^64 once; then per sample
 *   w(θ) = W + K + [A3 + D3 ≥ 2^64]   — the 128-bit word jlm_paynehanek_w computes for θ,
 * bit for bit, with two 64-bit adds in place of three 64×64-bit products. */
JLM_FN void jlm_ph_table_entry(double x, uint64_t *wlo, uint64_t *whi, uint64_t *a3lo) {
    uint64_t a1, a2, a3;
    jlm_ph_words(jlm_biased_exponent(x), &a1, &a2, &a3);
    const uint64_t X = (jlm_bits(x) & 0x000fffffffffffffull) | (1ull << 52);
    const jlm_u128 p3 = (jlm_u128)X * a3;
    const jlm_u128 W = ((jlm_u128)(X * a1) << 64) + (jlm_u128)X * a2 + (p3 >> 64);
    *wlo = (uint64_t)W;
    *whi = (uint64_t)(W >> 64);
    *a3lo = (uint64_t)p3;
}
/* the per-evaluation shift for xmin ≤ every x ≤ xmax (one binade, Payne–Hanek regime, positive):
 * 1 and (K, D3) when the table applies to θ = fl(x + ϕ), else 0 */
JLM_FN int jlm_ph_shift(double xmin, double xmax, double phi, uint64_t *klo, uint64_t *khi,
                        uint64_t *d3lo) {
    const int e0 = jlm_biased_exponent(xmin);
    if (!(xmin > 0.0) || !(xmax >= xmin) || jlm_biased_exponent(xmax) != e0 || e0 == 0x7ff ||
        e0 - 1023 < 21) /* θ ≥ 2^21 > 2^20·π/2: the Payne–Hanek regime of jl_sin */
        return 0;
    const double r = __builtin_ldexp(phi, 1075 - e0); /* ϕ / u, exact */
    if (!(__builtin_fabs(r) < 0x1p40)) return 0;       /* NaN, huge */
    const double d0 = __builtin_rint(r);
    if (__builtin_fabs(r - d0) == 0.5) return 0; /* a tie: fl(x + ϕ) depends on X's parity */
    const int64_t dl = (int64_t)d0;
    const int64_t Xmin = (int64_t)((jlm_bits(xmin) & 0x000fffffffffffffull) | (1ull << 52));
    const int64_t Xmax = (int64_t)((jlm_bits(xmax) & 0x000fffffffffffffull) | (1ull << 52));
    if (Xmin + dl - 1 < (int64_t)(1ull << 52) || Xmax + dl + 1 > (int64_t)((1ull << 53) - 1))
        return 0; /* some θ could leave the binade (or round across its edge) */
    uint64_t a1, a2, a3;
    jlm_ph_words(e0, &a1, &a2, &a3);
    const uint64_t D1 = (uint64_t)dl * a1;
    const jlm_i128 D2 = (jlm_i128)dl * (jlm_i128)(jlm_u128)a2;
    const jlm_i128 D3 = (jlm_i128)dl * (jlm_i128)(jlm_u128)a3;
    const jlm_u128 K = ((jlm_u128)D1 << 64) + (jlm_u128)D2 + (jlm_u128)(D3 >> 64);
    *klo = (uint64_t)K;
    *khi = (uint64_t)(K >> 64);
    *d3lo = (uint64_t)D3;
    return 1;
}
/* jl_sin(θ) from the sample's table entry and the evaluation's shift (θ > 0, regime above) */
JLM_FN double jl_sin_ph_shifted(uint64_t wlo, uint64_t whi, uint64_t a3lo, uint64_t klo,
                                uint64_t khi, uint64_t d3lo) {
    const uint64_t c = (uint64_t)(a3lo + d3lo < a3lo);
    const jlm_u128 w = ((((jlm_u128)whi << 64) | wlo) + (((jlm_u128)khi << 64) | klo)) + c;
    double hi, lo;
    const int n = jlm_ph_tail(w, 0, &hi, &lo);
    return jlm_sin_quadrant(n, hi, lo);
}

JLM_FN double jl_sin_cwx_nb(double x) {
    double hi, lo;
    const int n = jlm_cwext_nb(x, jlm_poshighword(x), &hi, &lo);
    return jlm_sin_quadrant(n, hi, lo);
}
/* jl_sincos for |x| ≲ 9π/4 outside the extended-precision points (|x| ≈ π/2, π, 3π/2, 2π) */
JLM_FN int jlm_sincos_small_in(double x) {
    const uint32_t xhp = jlm_poshighword(x);
    const int ext = xhp <= 0x400f6a7au ? (xhp & 0xfffffu) == 0x921fbu
                                       : (xhp == 0x4012d97cu || xhp == 0x401921fbu);
    return xhp <= 0x401c463bu && !(__builtin_fabs(x) >= JLM_PI_4 && ext);
}
JLM_FN void jl_sincos_small_nb(double x, double *s, double *c) {
    const uint32_t xhp = jlm_poshighword(x);
    const int plain = __builtin_fabs(x) < JLM_PI_4;
    const double fm = xhp <= 0x4002d97cu ? 1.0
                      : xhp <= 0x400f6a7au ? 2.0
                      : xhp <= 0x4015fdbcu ? 3.0
                                           : 4.0;
    const double fn = x > 0.0 ? fm : -fm;
    const double z = jlm_fma(-fn, JLM_PIO2_1, x);
    const double y1 = jlm_fma(-fn, JLM_PIO2_1T, z);
    const double l1 = jlm_fma(-fn, JLM_PIO2_1T, z - y1);
    const double hi = plain ? x : y1, lo = plain ? 0.0 : l1;
    const int n = plain ? 0 : ((int)fn & 3);
    const double si = jlm_sin_kernel_sel(hi, lo, plain), co = jlm_cos_kernel(hi, lo);
    const double ss = n == 0 ? si : (n == 1 ? co : (n == 2 ? -si : -co));
    const double cc = n == 0 ? co : (n == 1 ? -si : (n == 2 ? -co : si));
    *s = x == 0.0 ? x : ss;
    *c = x == 0.0 ? 1.0 : cc;
}
/* per-argument dispatch onto the forms above (the tests' view of them: = jl_sin, jl_sincos) */
JLM_FN double jl_sin_sel(double x) {
    if (jlm_sin_ph_in(x)) return jl_sin_ph_nb(x);
    if (jlm_sin_cwx_in(x)) return jl_sin_cwx_nb(x);
    return jl_sin(x);
}
JLM_FN void jl_sincos_sel(double x, double *s, double *c) {
    if (jlm_sincos_small_in(x)) {
        jl_sincos_small_nb(x, s, c);
        return;
    }
    jl_sincos(x, s, c);
}

/* ---- atan, atan(y, x) (base/special/trig.jl, msun s_atan.c / e_atan2.c) ----------------- */
JLM_FN double jlm_atan_hi(int id) {
    return id == 0   ? 4.63647609000806093515e-01
           : id == 1 ? 7.85398163397448278999e-01
           : id == 2 ? 9.82793723247329054082e-01
                     : 1.57079632679489655800e+00;
}
JLM_FN double jlm_atan_lo(int id) {
    return id == 0   ? 2.26987774529616870924e-17
           : id == 1 ? 3.06161699786838301793e-17
           : id == 2 ? 1.39033110312309984516e-17
                     : 6.12323399573676603587e-17;
}

JLM_FN double jl_atan(double x) {
    if (__builtin_isnan(x)) return x;
    const double xa = __builtin_fabs(x);
    if (xa >= 0x1p66) return __builtin_copysign(1.5707963267948966, x);
    int id;
    double xr;
    if (xa < 0.4375) {
        if (xa < 0x1p-27) return x;
        id = -1;
        xr = x;
    } else if (xa < 1.1875) {
        if (xa < 0.6875) {
            id = 0;
            xr = (2.0 * xa - 1.0) / (2.0 + xa);
        } else {
            id = 1;
            xr = (xa - 1.0) / (xa + 1.0);
        }
    } else if (xa < 2.4375) {
        id = 2;
        xr = (xa - 1.5) / (1.0 + 1.5 * xa);
    } else {
        id = 3;
        xr = -1.0 / xa;
    }
    const double z = xr * xr, w = z * z;
    /* odd and even halves of Σ aT[i] z^(i+1), Horner by muladd */
    const double s1 =
        z * jlm_fma(w,
                    jlm_fma(w,
                            jlm_fma(w,
                                    jlm_fma(w,
                                            jlm_fma(w, 1.62858201153657823623e-02,
                                                    4.97687799461593236017e-02),
                                            6.66107313738753120669e-02),
                                    9.09088713343650656196e-02),
                            1.42857142725034663711e-01),
                    3.33333333333329318027e-01);
    const double s2 =
        w * jlm_fma(w,
                    jlm_fma(w,
                            jlm_fma(w,
                                    jlm_fma(w, -3.65315727442169155270e-02,
                                            -5.83357013379057348645e-02),
                                    -7.69187620504482999495e-02),
                            -1.11111104054623557880e-01),
                    -1.99999999998764832476e-01);
    if (id < 0) return xr - xr * (s1 + s2);
    const double zz = jlm_atan_hi(id) - ((xr * (s1 + s2) - jlm_atan_lo(id)) - xr);
    return __builtin_copysign(zz, x);
}

#define JLM_PI 3.141592653589793
#define JLM_PI_LO 1.2246467991473531772e-16

/* atan(y, x) = angle(Complex(x, y)) */
JLM_FN double jl_atan2(double y, double x) {
    if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_isnan(x) ? x : y;
    if (x == 1.0) return jl_atan(y);
    int m = 2 * (__builtin_signbit(x) != 0) + (__builtin_signbit(y) != 0);
    if (y == 0.0) {
        if (m == 0 || m == 1) return y;
        return m == 2 ? JLM_PI : -JLM_PI;
    } else if (x == 0.0) {
        return __builtin_signbit(y) ? -(JLM_PI / 2) : JLM_PI / 2; /* flipsign(π/2, y) */
    }
    if (__builtin_isinf(x)) {
        if (__builtin_isinf(y)) {
            if (m == 0) return JLM_PI / 4;
            if (m == 1) return -JLM_PI / 4;
            if (m == 2) return 3 * JLM_PI / 4;
            return -3 * JLM_PI / 4;
        }
        if (m == 0) return 0.0;
        if (m == 1) return -0.0;
        if (m == 2) return JLM_PI;
        return -JLM_PI;
    }
    if (__builtin_isinf(y)) return __builtin_copysign(JLM_PI / 2, y);
    const uint32_t ypw = jlm_poshighword(y), xpw = jlm_poshighword(x);
    const int32_t k = (int32_t)(ypw - xpw) >> 20;
    double z;
    if (k > 60) { /* |y/x| > 2^60 */
        z = JLM_PI / 2 + 0.5 * JLM_PI_LO;
        m &= 1;
    } else if (x < 0 && k < -60) { /* 0 > |y|/x > -2^-60 */
        z = 0.0;
    } else {
        z = jl_atan(__builtin_fabs(y / x));
    }
    if (m == 0) return z;
    if (m == 1) return -z;
    if (m == 2) return JLM_PI - (z - JLM_PI_LO);
    return (z - JLM_PI_LO) - JLM_PI;
}

/* ---- hypot (base/math.jl; the branch taken with hardware fma, correctly rounded) ---------- */
JLM_FN double jl_hypot(double x, double y) {
    double ax = __builtin_fabs(x), ay = __builtin_fabs(y);
    if (__builtin_isinf(ax) || __builtin_isinf(ay)) return __builtin_inf();
    if (ay > ax) {
        const double t = ax;
        ax = ay;
        ay = t;
    }
    if (ay <= ax * 0x1.6a09e667f3bcdp-27) return ax; /* sqrt(eps/2); also ay == 0 */
    double scale = 0x1p-563;                         /* eps·sqrt(floatmin) */
    if (ax > 0x1.6a09e667f3bccp+511) {               /* sqrt(floatmax/2) */
        ax = ax * scale;
        ay = ay * scale;
        scale = 0x1p+563;
    } else if (ay < 0x1p-511) { /* sqrt(floatmin) */
        ax = ax / scale;
        ay = ay / scale;
    } else {
        scale = 1.0;
    }
    double h = __builtin_sqrt(jlm_fma(ax, ax, ay * ay));
    const double hsquared = h * h, axsquared = ax * ax;
    h = h - ((jlm_fma(-ay, ay, hsquared - axsquared) + jlm_fma(h, h, -hsquared)) -
             jlm_fma(ax, ax, -axsquared)) /
                (2 * h);
    return h * scale;
}

/* jl_hypot without branches: every path of jl_hypot is evaluated and the result selected, so
 * that many independent evaluations interleave (the faint statistics evaluate 16 per thread at
 * a time).  The same operations on the same operands as the taken path of jl_hypot — the same
 * bits for every input (tests/test_jlmath.py: special values, scaling ranges, random pairs). */
JLM_FN double jl_hypot_nb(double x, double y) {
    const double fx = __builtin_fabs(x), fy = __builtin_fabs(y);
    const int inf = __builtin_isinf(fx) | __builtin_isinf(fy);
    const int sw = fy > fx;
    const double ax = sw ? fy : fx, ay = sw ? fx : fy;
    const int early = ay <= ax * 0x1.6a09e667f3bcdp-27;
    const int big = ax > 0x1.6a09e667f3bccp+511;
    const int small = !big && (ay < 0x1p-511);
    /* x / 2^-563 == x * 2^563 exactly (a power-of-two reciprocal): the scaled operands of both
     * scaling branches are products */
    const double f = big ? 0x1p-563 : (small ? 0x1p+563 : 1.0);
    const double scale = big ? 0x1p+563 : (small ? 0x1p-563 : 1.0);
    const double bx = ax * f, by = ay * f;
    double h = __builtin_sqrt(jlm_fma(bx, bx, by * by));
    const double hsquared = h * h, axsquared = bx * bx;
    h = h - ((jlm_fma(-by, by, hsquared - axsquared) + jlm_fma(h, h, -hsquared)) -
             jlm_fma(bx, bx, -axsquared)) /
                (2 * h);
    const double r = h * scale;
    return inf ? __builtin_inf() : (early ? ax : r);
}

#endif /* GPD_JLMATH_H */
