// Device building blocks for the demodulation engine (gfx950).
//
//  * Julia Complex{Float64} arithmetic (Base.:*, Base.:/ robust division, exp(im·x)) so the
//    exact evaluator reproduces the reference's per-sample rounding
//    (src/Modulation.jl:137,143-146,189-192).  Built with -ffp-contract=off.
//  * Bessel J_n(b), n = 0..K+1, by Miller's backward recurrence — the coefficients of the
//    Jacobi–Anger expansion e^{-j b sin θ} = Σ_n J_n(b) e^{-j n θ} used by the harmonic path.
//  * Deterministic workgroup reductions (xor-butterfly inside a wave, fixed-order across waves):
//    every lane ends with bit-identical totals, so optimizer control flow stays uniform.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "gpd_jlmath.h"  // Julia Base's sin/cos/sincos/atan/hypot, shared with the oracle

namespace gpd {

struct c64 {
    double re, im;
};

// Julia ComplexF32 — FITS VOLT precision.  Series stored this way are widened to Float64 on
// load (exact), so every evaluation sees the same values as Float64.(data).
struct c32 {
    float re, im;
};

__device__ __forceinline__ c64 widen(c32 z) { return {(double)z.re, (double)z.im}; }
__device__ __forceinline__ c64 widen(c64 z) { return z; }

__device__ __forceinline__ c64 cmul(c64 x, c64 y) {  // Base.:*(::ComplexF64, ::ComplexF64)
    return {x.re * y.re - x.im * y.im, x.re * y.im + x.im * y.re};
}

__device__ __forceinline__ double robust_cdiv2(double a, double b, double c, double d, double r,
                                               double t) {
    if (r != 0) {
        const double br = b * r;
        return (br != 0 ? (a + br) * t : a * t + (b * t) * r);
    }
    return (a + d * (b / c)) * t;
}

// Base.:/(::ComplexF64, ::ComplexF64): Baudin–Smith robust complex division.
__device__ __forceinline__ c64 cdiv(c64 z, c64 w) {
    double a = z.re, b = z.im, c = w.re, d = w.im;
    const double absa = fabs(a), absb = fabs(b), ab = absa >= absb ? absa : absb;
    const double absc = fabs(c), absd = fabs(d), cd = absc >= absd ? absc : absd;
    const double halfov = 0.5 * 1.7976931348623157e308;
    const double twouneps = 2.2250738585072014e-308 * 2.0 / 2.220446049250313e-16;
    const double bs = 2.0 / (2.220446049250313e-16 * 2.220446049250313e-16);
    double s = 1.0, p, q;
    if (ab >= halfov) { a = 0.5 * a; b = 0.5 * b; s = 2.0; }
    if (cd >= halfov) { c = 0.5 * c; d = 0.5 * d; s *= 0.5; }
    if (ab <= twouneps) { a *= bs; b *= bs; s /= bs; }
    if (cd <= twouneps) { c *= bs; d *= bs; s *= bs; }
    if (absd <= absc) {
        const double r = d / c, t = 1.0 / (c + d * r);
        p = robust_cdiv2(a, b, c, d, r, t);
        q = robust_cdiv2(b, -a, c, d, r, t);
    } else {
        const double r = c / d, t = 1.0 / (d + c * r);
        p = robust_cdiv2(b, a, d, c, r, t);
        q = -robust_cdiv2(a, -b, d, c, r, t);
    }
    return {p * s, q * s};
}

// exp(Complex(±0, x)) as Julia evaluates it: (cos x, sin x) from sincos(x), or (1, x) when
// x == 0 (base/complex.jl exp; the sincos is Julia Base's, gpd_jlmath.h).
__device__ __forceinline__ c64 cisj(double x) {
    if (x == 0.0) return {1.0, x};
    double s, c;
    jl_sincos(x, &s, &c);
    return {c, s};
}

// ---------------------------------------------------------------------------------------
// Bessel functions of the first kind J_0..J_{KP} at b (any sign), the coefficients of the
// Jacobi–Anger expansion.  |b| ≥ 0.05: Miller's backward recurrence J_{n-1} = (2n/b) J_n − J_{n+1}
// (one fma per step)
// from the fixed, fully unrolled start order KP + 32 (compile-time indices: no select chains),
// normalised with J_0 + 2 Σ_k J_{2k} = 1; relative accuracy ~1e-16 for |b| ≤ 0.45·KP (callers
// reject larger |b|).  |b| < 0.05: ascending series J_n = Σ_k (−b²/4)^k (b/2)^n / (k! (n+k)!).
template <int KP>
__host__ __device__ __forceinline__ void bessel_j(double b, double (&J)[KP + 1]) {
    const double ab = fabs(b);
    if (ab < 0.05) {
        const double h = 0.5 * ab, h2 = -h * h;
        double pw = 1.0;  // (b/2)^n / n!
#pragma unroll
        for (int n = 0; n <= KP; ++n) {
            // Σ_{k=0..4} h2^k / (k! (n+1)…(n+k)): |h2|^5 ≤ 4e-18 relative
            const double c1 = h2 / (n + 1), c2 = c1 * h2 / (2.0 * (n + 2)),
                         c3 = c2 * h2 / (3.0 * (n + 3)), c4 = c3 * h2 / (4.0 * (n + 4));
            J[n] = pw * (1.0 + (c1 + (c2 + (c3 + c4))));
            pw = pw * h / (n + 1);
        }
    } else {
        constexpr int M = KP + 32;  // even start order
        const double inv = 2.0 / ab;
        double jp1 = 0.0, jn = 1.0e-280, norm = 0.0;
#pragma unroll
        for (int n = M; n >= 1; --n) {
            // J_{n-1}: one fma on the recurrence's dependent chain (n·inv is off it; r5 —
            // the separate multiply and subtract made the chain twice as long, ~1 k of the
            // objective's ~3 k cycles)
            const double jm1 = fma((double)n * inv, jn, -jp1);
            jp1 = jn;
            jn = jm1;
            if (n <= KP) J[n] = jp1;
            if ((n & 1) == 0) norm += 2.0 * jp1;
        }
        J[0] = jn;
        norm += jn;
        const double sc = 1.0 / norm;
#pragma unroll
        for (int n = 0; n <= KP; ++n) J[n] *= sc;
    }
    if (b < 0.0) {
#pragma unroll
        for (int n = 1; n <= KP; n += 2) J[n] = -J[n];
    }
}

// ---------------------------------------------------------------------------------------
// Deterministic sum over a workgroup of WG threads (WG multiple of 64) of NV doubles.
// lds must hold (WG/64)*NV doubles.  On return every thread holds the same totals.
// PT: double* or an LDS-qualified pointer (out-of-line callers pass the latter so that the
// partials go through ds_ instructions, not flat ones)
// The value of lane (this lane xor OFF) — exactly __shfl_xor(v, OFF, 64), through the cheapest
// cross-lane path: DPP quad permutes for 1 and 2, ds_swizzle's xor mode within 32-lane halves
// for 4, 8 and 16, ds_bpermute for 32.  GPD_BS_DPP=0 (A/B builds) keeps __shfl_xor throughout.
#ifndef GPD_BS_DPP
#define GPD_BS_DPP 1
#endif
template <int OFF>
__device__ __forceinline__ double lane_xor(double v) {
#if GPD_BS_DPP
    if constexpr (OFF <= 16) {
        const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
        int lo = (int)(unsigned)u, hi = (int)(unsigned)(u >> 32);
        if constexpr (OFF == 1) {  // quad_perm [1,0,3,2]
            lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);
            hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
        } else if constexpr (OFF == 2) {  // quad_perm [2,3,0,1]
            lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false);
            hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false);
        } else {  // bit mode: and_mask 0x1F, xor_mask OFF
            lo = __builtin_amdgcn_ds_swizzle(lo, 0x1F | (OFF << 10));
            hi = __builtin_amdgcn_ds_swizzle(hi, 0x1F | (OFF << 10));
        }
        return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
    }
#endif
    return __shfl_xor(v, OFF, 64);
}

// The wave stage of block_sum: xor butterfly over the 64 lanes, partners 32, 16, …, 1 (each
// step adds the partner's value); every lane ends with the same total.
template <int NV>
__device__ __forceinline__ void wave_sum(double (&v)[NV]) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = v[k] + lane_xor<32>(v[k]);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = v[k] + lane_xor<16>(v[k]);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = v[k] + lane_xor<8>(v[k]);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = v[k] + lane_xor<4>(v[k]);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = v[k] + lane_xor<2>(v[k]);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = v[k] + lane_xor<1>(v[k]);
}

template <int WG, int NV, class PT = double *>
__device__ __forceinline__ void block_sum(double (&v)[NV], PT lds) {
    constexpr int NW = WG / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    wave_sum<NV>(v);
    if (NW == 1) return;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) lds[wave * NV + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = lds[k];
#pragma unroll
        for (int w = 1; w < NW; ++w) s = s + lds[w * NV + k];
        v[k] = s;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------------------
// Counter-based RNG (splitmix64), identical to tests/synth.py.
__device__ __host__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double rng_uniform(uint64_t seed, uint64_t stream, uint64_t idx) {
    const uint64_t key = splitmix64((seed * 0x100000001B3ull) ^ stream);
    return (double)(splitmix64(idx ^ key) >> 11) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ double rng_normal(uint64_t seed, uint64_t stream, uint64_t idx) {
    const double u1 = rng_uniform(seed, 2 * stream, idx);
    const double u2 = rng_uniform(seed, 2 * stream + 1, idx);
    return sqrt(-2.0 * log1p(-u1)) * cos(6.283185307179586 * u2);
}

}  // namespace gpd
