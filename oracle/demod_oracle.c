/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into or called by the product library.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it, as the checker.
 *
 * Plain-C restatement of the reference hot path (FerreolS/GPPupilDemodulation.jl @ 2024-10-16):
 *   - updatemodulation! (weighted, 8-arg)        src/Modulation.jl:122-148
 *   - linearregression (weighted, offsets)       src/Modulation.jl:174-195
 *   - weighted_norm2 / Chi2CostFunction functor  src/Modulation.jl:299-326
 *   - minimize! → newuoa(…, 1, 1e-3)             src/Modulation.jl:332-342 (newuoa_oracle.c)
 *   - demodulateall per-diode body               src/Modulation.jl:360-432
 *   - getphase / Modulation functor              src/Modulation.jl:57-69
 *   - buildstates, compute_mean_var_power        src/Faint.jl:21-73, 89-100
 * Arithmetic follows Julia's Complex{Float64} formulas (no FMA contraction: build with
 * -ffp-contract=off).  Sums are sequential (the reference's @simd/BLAS order is not
 * reproducible anyway).  Non-faint semantics (broken in the reference at this snapshot,
 * SURVEY §0.3) are defined as w ≡ 1, p = FC phasor.
 * PARITY UNPINNED (no Julia in this container; the reference has no tests or fixtures).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include "oracle.h"
/* Julia Base's sin / sincos / atan(y,x) / hypot, restated once and shared with the device so the
 * exact evaluator and this oracle compute the same per-sample bits (src/Modulation.jl:137,388,
 * 419-421; src/Faint.jl:95-97) */
#include "../gppupildemodulation.jl_amd/csrc/gpd_jlmath.h"
#ifdef _OPENMP
#include <omp.h>
#endif

#define PI_F64 3.141592653589793115997963468544185161590576171875

enum { ST_TRANSIENT = -1, ST_OFF = 0, ST_LOW = 1, ST_NORMAL = 2, ST_HIGH = 3 };

void oracle_phi_grid(double *out8) {
    /* Bit-exact Julia range(-π, π, 8) (derived by oracle/tools/phi_grid.py). */
    static const double g[8] = {-0x1.921fb54442d18p+1, -0x1.1f3b3855544c8p+1,
                                -0x1.58ad76cccb8f0p+0, -0x1.cb91f3bbba140p-2,
                                0x1.cb91f3bbba140p-2,  0x1.58ad76cccb8f0p+0,
                                0x1.1f3b3855544c8p+1,  0x1.921fb54442d18p+1};
    memcpy(out8, g, sizeof g);
}

/* ---- Julia Complex{Float64} primitives ------------------------------------------- */
typedef struct { double re, im; } cplx;

static inline cplx cmul(cplx x, cplx y) { /* Base.:*(::Complex, ::Complex) */
    cplx r = {x.re * y.re - x.im * y.im, x.re * y.im + x.im * y.re};
    return r;
}

static inline double robust_cdiv2(double a, double b, double c, double d, double r, double t) {
    if (r != 0) {
        double br = b * r;
        return (br != 0 ? (a + br) * t : a * t + (b * t) * r);
    }
    return (a + d * (b / c)) * t;
}

static inline void robust_cdiv1(double a, double b, double c, double d, double *p, double *q) {
    double r = d / c;
    double t = 1.0 / (c + d * r);
    *p = robust_cdiv2(a, b, c, d, r, t);
    *q = robust_cdiv2(b, -a, c, d, r, t);
}

/* Base.:/(::ComplexF64, ::ComplexF64) — Baudin & Smith robust division. */
static cplx cdiv(cplx z, cplx w) {
    double a = z.re, b = z.im, c = w.re, d = w.im;
    double absa = fabs(a), absb = fabs(b), ab = absa >= absb ? absa : absb;
    double absc = fabs(c), absd = fabs(d), cd = absc >= absd ? absc : absd;
    const double halfov = 0.5 * DBL_MAX, twouneps = DBL_MIN * 2.0 / DBL_EPSILON,
                 bs = 2.0 / (DBL_EPSILON * DBL_EPSILON);
    double s = 1.0, p, q;
    if (ab >= halfov) { a = 0.5 * a; b = 0.5 * b; s = 2.0; }
    if (cd >= halfov) { c = 0.5 * c; d = 0.5 * d; s *= 0.5; }
    if (ab <= twouneps) { a *= bs; b *= bs; s /= bs; }
    if (cd <= twouneps) { c *= bs; d *= bs; s *= bs; }
    if (absd <= absc) {
        robust_cdiv1(a, b, c, d, &p, &q);
    } else {
        robust_cdiv1(b, a, d, c, &p, &q);
        q = -q;
    }
    cplx r = {p * s, q * s};
    return r;
}

/* exp(im*x) as Julia evaluates exp(Complex(±0, x)): (cos x, sin x); x == 0 → (1, x). */
static inline cplx cisj(double x) {
    cplx r;
    if (x == 0) {
        r.re = 1.0;
        r.im = x;
    } else {
        jl_sincos(x, &r.im, &r.re); /* exp(Complex(0, x)): s, c = sincos(x) */
    }
    return r;
}

/* ---- deterministic reduction order -------------------------------------------------
 * Julia's @simd loops, mapreduce's pairwise blocks and BLAS zdotc fix no summation order, so any
 * order is a faithful evaluation of the reference sums.  The oracle and the product use ONE
 * canonical order ("CR8"): sample i of a series (index counted from the series' first sample)
 * adds into slot i mod 2048, slots accumulate in increasing i; the slots form 8 blocks of 256,
 * each block is 4 groups of 64 combined by the xor butterfly (off = 32..1) with the 4 group
 * totals added left to right, and the 8 block totals are added left to right.  The device runs
 * a block per 256-thread workgroup pass (one workgroup sweeping the 8 blocks in turn, or up to 8
 * workgroups per series exchanging block totals), so every split gives the same bits. */
#define GSUM_W 2048
#define GSUM_BLOCK 256
#define GSUM_NV 16
typedef struct {
    int nv;
    double v[GSUM_NV][GSUM_W]; /* [quantity][slot] */
} gsum_t;

static void gsum_zero(gsum_t *g, int nv) {
    g->nv = nv;
    memset(g->v, 0, sizeof(double) * GSUM_W * (size_t)nv);
}

#define GSLOT(g, i, q) ((g)->v[q][(i) % GSUM_W])

static void gsum_total(const gsum_t *g, double *out) {
    double lane[64];
    for (int q = 0; q < g->nv; ++q) {
        double total = 0.0;
        for (int blk = 0; blk < GSUM_W / GSUM_BLOCK; ++blk) {
            double s = 0.0;
            for (int w = 0; w < GSUM_BLOCK / 64; ++w) {
                for (int l = 0; l < 64; ++l) lane[l] = g->v[q][blk * GSUM_BLOCK + w * 64 + l];
                for (int off = 32; off >= 1; off >>= 1) {
                    double nxt[64];
                    for (int l = 0; l < 64; ++l) nxt[l] = lane[l] + lane[l ^ off];
                    memcpy(lane, nxt, sizeof lane);
                }
                s = (w == 0) ? lane[0] : s + lane[0];
            }
            total = (blk == 0) ? s : total + s;
        }
        out[q] = total;
    }
}

/* ---- Chi2CostFunction ---------------------------------------------------------------- */
typedef struct {
    int64_t n;
    const double *t;   /* [n]            */
    const cplx *d;     /* [n]            */
    const double *w;   /* [n] or NULL ≡ 1 */
    const cplx *p;     /* [n]            */
    double omega;
    int offsets;
    cplx *model;       /* scratch [n]    */
    const int64_t *orig; /* original sample index of each valid sample (reduction lane) */
    gsum_t *gs;        /* reduction scratch */
    oracle_param *mod; /* mutated by every evaluation, like lkl.mod */
    int nfev;
    uint64_t perturb;  /* 0, or a seed: χ² *= 1 + u per evaluation (tie-sensitivity probe) */
    double perturb_ulps; /* |u| = 2^-52 (≤ 1), or uniform in [0, perturb_ulps·2^-52] */
    int order;         /* summation order of the cost's sums: 0 = CR8 (the product's), else an
                          alternative order the reference's own loops may take (red_slot) */
} chi2_ctx;

/* Alternative summation orders (the reference-ceiling probe, bench.py cpu_baseline): Julia's
 * `@simd` loops (src/Modulation.jl:181,301) and BLAS zdotc (:143-144) leave the order to the
 * compiler / BLAS kernel, so the reference's own χ² differs by ulps from one CPU to another.
 * order 1: strictly sequential (a loop without @simd); order L > 1: what a vectorised loop with
 * L accumulators does — sample i (counted over the valid samples, as the reference's
 * data[valid] vectors are) adds into accumulator i mod L for i < n - n mod L, the remainder into
 * a scalar tail; at the end the unrolled vectors (width V = 4 for L = 16: AVX2 × 4 unroll; V = 8
 * for L = 32: AVX-512 × 4) are added one after the other, the vector lanes by a halving tree,
 * then the tail.  Test infrastructure only; the product keeps CR8. */
static inline int64_t red_slot(const chi2_ctx *c, int64_t i) {
    if (c->order == 0) return c->orig[i];
    if (c->order == 1) return 0;
    const int64_t L = c->order;
    return i < c->n - c->n % L ? i % L : L;
}

static void red_total(const chi2_ctx *c, const gsum_t *g, double *out) {
    if (c->order == 0) {
        gsum_total(g, out);
        return;
    }
    for (int q = 0; q < g->nv; ++q) {
        if (c->order == 1) {
            out[q] = g->v[q][0];
            continue;
        }
        const int L = c->order, V = L >= 32 ? 8 : 4, U = L / V;
        double acc[8];
        for (int l = 0; l < V; ++l) acc[l] = g->v[q][l];
        for (int u = 1; u < U; ++u)
            for (int l = 0; l < V; ++l) acc[l] = g->v[q][u * V + l] + acc[l];
        for (int h = V / 2; h >= 1; h >>= 1)
            for (int l = 0; l < h; ++l) acc[l] = acc[l] + acc[l + h];
        out[q] = acc[0] + g->v[q][L];
    }
}

static uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static double chi2_eval(chi2_ctx *c, double b, double phi) {
    const int64_t n = c->n;
    oracle_param *mod = c->mod;
    cplx *model = c->model;
    mod->b = b;
    mod->phi = phi;
    c->nfev++;
    /* @. model = power * exp(ȷ * b * sin(ω * timestamp + ϕ))      (src/Modulation.jl:137) */
    for (int64_t i = 0; i < n; ++i) {
        double th = c->omega * c->t[i];
        th = th + phi;
        double beta = b * jl_sin(th);
        model[i] = cmul(c->p[i], cisj(beta));
    }
    if (c->offsets) {
        /* linearregression(model, data, weight)                (src/Modulation.jl:174-195) */
        gsum_t *g = c->gs;
        double tot[8];
        gsum_zero(g, 8);
        for (int64_t i = 0; i < n; ++i) {
            double wi = c->w ? c->w[i] : 1.0;
            cplx m = model[i], dd = c->d[i];
            const int64_t o = red_slot(c, i);
            GSLOT(g, o, 0) += wi;
            GSLOT(g, o, 1) += wi * m.re;
            GSLOT(g, o, 2) += wi * m.im;
            GSLOT(g, o, 3) += wi * (m.re * m.re + m.im * m.im);
            GSLOT(g, o, 4) += wi * dd.re;
            GSLOT(g, o, 5) += wi * dd.im;
            cplx wm = {wi * m.re, wi * (-m.im)}; /* weight[i]*conj(model[i]) */
            cplx pr = cmul(wm, dd);
            GSLOT(g, o, 6) += pr.re;
            GSLOT(g, o, 7) += pr.im;
        }
        red_total(c, g, tot);
        double a11 = tot[0], a22 = tot[3];
        cplx a12 = {tot[1], tot[2]}, b1 = {tot[4], tot[5]}, b2 = {tot[6], tot[7]};
        /* SMatrix{2,2}([a11 a12; conj(a12) a22]) \ [b1, b2]  — StaticArrays 2×2 Cramer */
        cplx A11 = {a11, 0.0}, A12 = a12, A21 = {a12.re, -a12.im}, A22 = {a22, 0.0};
        cplx t1 = cmul(A11, A22), t2 = cmul(A12, A21);
        cplx det = {t1.re - t2.re, t1.im - t2.im};
        cplx u1 = cmul(A22, b1), u2 = cmul(A12, b2);
        cplx cn = {u1.re - u2.re, u1.im - u2.im};
        cplx v1 = cmul(A11, b2), v2 = cmul(A21, b1);
        cplx an = {v1.re - v2.re, v1.im - v2.im};
        cplx cc = cdiv(cn, det), aa = cdiv(an, det);
        mod->c_re = cc.re;
        mod->c_im = cc.im;
        mod->a_re = aa.re;
        mod->a_im = aa.im;
        for (int64_t i = 0; i < n; ++i) { /* @. model = c + a * model */
            cplx am = cmul(aa, model[i]);
            model[i].re = cc.re + am.re;
            model[i].im = cc.im + am.im;
        }
    } else {
        /* mw = model .* weight; a = (mw ⋅ data) / (mw ⋅ model)   (src/Modulation.jl:143-145) */
        gsum_t *g = c->gs;
        double tot[4];
        gsum_zero(g, 4);
        for (int64_t i = 0; i < n; ++i) {
            double wi = c->w ? c->w[i] : 1.0;
            cplx mw = {model[i].re * wi, model[i].im * wi};
            cplx mwc = {mw.re, -mw.im};
            cplx x = cmul(mwc, c->d[i]);
            cplx y = cmul(mwc, model[i]);
            const int64_t o = red_slot(c, i);
            GSLOT(g, o, 0) += x.re;
            GSLOT(g, o, 1) += x.im;
            GSLOT(g, o, 2) += y.re;
            GSLOT(g, o, 3) += y.im;
        }
        red_total(c, g, tot);
        cplx num = {tot[0], tot[1]}, den = {tot[2], tot[3]};
        cplx aa = cdiv(num, den);
        mod->c_re = 0;
        mod->c_im = 0;
        mod->a_re = aa.re;
        mod->a_im = aa.im;
        for (int64_t i = 0; i < n; ++i) model[i] = cmul(aa, model[i]);
    }
    /* weighted_norm2(model .- data, weight) / N             (src/Modulation.jl:299-305,325) */
    double s;
    {
        gsum_t *g = c->gs;
        gsum_zero(g, 1);
        for (int64_t i = 0; i < n; ++i) {
            double rr = model[i].re - c->d[i].re, ri = model[i].im - c->d[i].im;
            double a2 = rr * rr + ri * ri;
            GSLOT(g, red_slot(c, i), 0) += (c->w ? c->w[i] : 1.0) * a2;
        }
        red_total(c, g, &s);
    }
    if (c->perturb) {
        const uint64_t r = mix64(c->perturb ^ ((uint64_t)c->nfev << 20));
        double u = (r & 1) ? 0x1p-52 : -0x1p-52;
        if (c->perturb_ulps > 1.0) u *= c->perturb_ulps * (double)(r >> 11) * 0x1p-53;
        return (s / (double)n) * (1.0 + u);
    }
    return s / (double)n;
}

static double chi2_objfun(void *ctx, int n, const double *x) {
    (void)n;
    return chi2_eval((chi2_ctx *)ctx, x[0], x[1]);
}

double oracle_chi2(int64_t n, const double *t, const double *d, const double *w,
                   const double *p, double omega, int offsets, double b, double phi,
                   oracle_param *mod) {
    chi2_ctx c;
    c.n = n;
    c.t = t;
    c.d = (const cplx *)d;
    c.w = w;
    c.p = (const cplx *)p;
    c.omega = omega;
    c.offsets = offsets;
    c.model = (cplx *)malloc(sizeof(cplx) * (size_t)(n > 0 ? n : 1));
    int64_t *orig = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) orig[i] = i;
    c.orig = orig;
    c.gs = (gsum_t *)malloc(sizeof(gsum_t));
    c.mod = mod;
    c.nfev = 0;
    c.perturb = 0;
    c.order = 0;
    double r = chi2_eval(&c, b, phi);
    free(c.model);
    free(orig);
    free(c.gs);
    return r;
}

/* compute_mean_var_power(states, data)                       (src/Faint.jl:89-100)
 * mean(abs, x) = Σ|x|/n and var(|x|; mean=m) = Σ(|x|-m)²/(n-1); sums in the reduction order
 * above (lane = original sample index mod 256).  A 1-sample state gives 0/0 = NaN weights. */
static void mean_var_power_idx(int64_t n, const int8_t *states, const cplx *d, const int64_t *orig,
                               double *m, double *w, gsum_t *g, double *m5o, double *w5o) {
    double tot[10], m5[5], w5[5], ss[5];
    gsum_zero(g, 10);
    for (int64_t i = 0; i < n; ++i) {
        int q = states[i] + 1; /* TRANSIENT=-1 → 0 ... HIGH=3 → 4 */
        GSLOT(g, orig[i], q) += 1.0;
        GSLOT(g, orig[i], 5 + q) += jl_hypot(d[i].re, d[i].im); /* abs(::Complex) = hypot */
    }
    gsum_total(g, tot);
    for (int q = 0; q < 5; ++q) m5[q] = tot[5 + q] / tot[q];
    gsum_zero(g, 5);
    for (int64_t i = 0; i < n; ++i) {
        int q = states[i] + 1;
        double dv = jl_hypot(d[i].re, d[i].im) - m5[q];
        GSLOT(g, orig[i], q) += dv * dv;
    }
    gsum_total(g, ss);
    for (int q = 0; q < 5; ++q) w5[q] = 1.0 / (ss[q] / (tot[q] - 1.0));
    for (int64_t i = 0; i < n; ++i) {
        m[i] = m5[states[i] + 1];
        w[i] = w5[states[i] + 1];
    }
    if (m5o)
        for (int q = 0; q < 5; ++q) m5o[q] = m5[q];
    if (w5o)
        for (int q = 0; q < 5; ++q) w5o[q] = w5[q];
}

void oracle_mean_var_power(int64_t n, const int8_t *states, const double *d_, double *m,
                           double *w) {
    int64_t *orig = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    gsum_t *g = (gsum_t *)malloc(sizeof(gsum_t));
    for (int64_t i = 0; i < n; ++i) orig[i] = i;
    mean_var_power_idx(n, states, (const cplx *)d_, orig, m, w, g, NULL, NULL);
    free(orig);
    free(g);
}

/* The fused faint statistics of the state-split moment pass (r4; gpd_kernels.hpp k_moments_ws
 * <FAINT> producers + k_faint_fused_fin): compute_mean_var_power (src/Faint.jl:89-100) in ONE
 * pass over the valid samples as shifted sums, K_s = abs(d) at the first valid sample of state s,
 *   S1 = Σ (|d| − K_s),  S2 = Σ (|d| − K_s)²,  m = K_s + S1/n,  w = 1 / ((S2 − S1·(S1/n)) / (n − 1)).
 * The algorithm the device runs, restated in sample order with Julia's hypot for |d| (the device
 * forms |q| = |p̄ d| through a hardware rsq and sums in its tile order, so its bits differ by a
 * few ulps; the stated tolerance against the two-pass restatement above is 1e-13 relative on w).
 * Checker only (tests/test_oracle.py, tests/test_gpu_faint_stats.py). */
void oracle_mean_var_power_fused(int64_t n, const int8_t *states, const double *d_, uint32_t flags,
                                 double *m5, double *w5) {
    const cplx *d = (const cplx *)d_;
    double K[5] = {0, 0, 0, 0, 0}, cnt[5] = {0, 0, 0, 0, 0}, s1[5] = {0, 0, 0, 0, 0},
           s2[5] = {0, 0, 0, 0, 0};
    for (int64_t i = 0; i < n; ++i) {
        int ok = 1;
        if (flags & ORACLE_ONLY_HIGH) ok = (states[i] == ST_HIGH) || (states[i] == ST_NORMAL);
        if (states[i] == ST_TRANSIENT) ok = 0;
        if (!ok) continue;
        const int q = states[i] + 1;
        const double x = jl_hypot(d[i].re, d[i].im);
        if (cnt[q] == 0.0) K[q] = x;
        const double y = x - K[q];
        cnt[q] += 1.0;
        s1[q] += y;
        s2[q] = fma(y, y, s2[q]);
    }
    for (int q = 0; q < 5; ++q) {
        if (cnt[q] == 0.0) {
            m5[q] = w5[q] = NAN;
            continue;
        }
        m5[q] = K[q] + s1[q] / cnt[q];
        w5[q] = 1.0 / ((s2[q] - s1[q] * (s1[q] / cnt[q])) / (cnt[q] - 1.0));
    }
}

void oracle_mean_var_power_series(int64_t n, const int8_t *states, const double *d_, uint32_t flags,
                                  double *m5, double *w5) {
    const cplx *d = (const cplx *)d_;
    int64_t *orig = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int8_t *sv = (int8_t *)malloc((size_t)(n > 0 ? n : 1));
    cplx *dv = (cplx *)malloc(sizeof(cplx) * (size_t)(n > 0 ? n : 1));
    double *m = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double *w = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    gsum_t *g = (gsum_t *)malloc(sizeof(gsum_t));
    int64_t nv = 0;
    for (int64_t i = 0; i < n; ++i) { /* valid mask, src/Modulation.jl:373-382 */
        int ok = 1;
        if (flags & ORACLE_ONLY_HIGH) ok = (states[i] == ST_HIGH) || (states[i] == ST_NORMAL);
        if (states[i] == ST_TRANSIENT) ok = 0;
        if (!ok) continue;
        orig[nv] = i;
        sv[nv] = states[i];
        dv[nv] = d[i];
        nv++;
    }
    mean_var_power_idx(nv, sv, dv, orig, m, w, g, m5, w5);
    free(orig);
    free(sv);
    free(dv);
    free(m);
    free(w);
    free(g);
}

/* buildstates(faintstates, timestamp; lag, preswitchdelay, postwitchdelay)   (src/Faint.jl:21-73) */
int oracle_buildstates(int64_t n, const double *t, int64_t n1, const double *timer1, int64_t n2,
                       const double *timer2, int8_t state1, int8_t state2, double preswitchdelay,
                       double postwitchdelay, int8_t *states) {
    if (n < 2 || n1 < 1 || n2 < 1) return -1;
    double timestep = t[1] - t[0];
    int64_t premax = (int64_t)ceil(preswitchdelay / timestep);
    int64_t postmax = (int64_t)ceil(postwitchdelay / timestep);
    int8_t current = ST_NORMAL;
    int64_t i1 = 0, i2 = 0;
    double first1 = timer1[i1++], first2 = timer2[i2++];
    double tlast = t[n - 1];
    int64_t forget = 0;
    for (int64_t k = 0; k < n; ++k) {
        double time = t[k];
        if (time >= first1) {
            current = state1;
            forget = premax;
            if (i1 >= n1) {
                first1 = tlast;
                if (first2 == tlast) current = ST_NORMAL;
            } else {
                first1 = timer1[i1++];
            }
        }
        if (time >= first2) {
            current = state2;
            forget = postmax;
            if (i2 >= n2) {
                first2 = tlast;
                if (first1 == tlast) current = ST_NORMAL;
            } else {
                first2 = timer2[i2++];
            }
        }
        if (forget > 0) {
            states[k] = ST_TRANSIENT;
            forget -= 1;
        } else {
            states[k] = current;
        }
    }
    return 0;
}

/* ---- per-pixel demodulate (body of the diode loop, src/Modulation.jl:390-431) ------- */
typedef struct {
    double *t, *w;
    cplx *d, *p, *model;
    int64_t *orig;
    gsum_t *gs;
} scratch_t;

static int julia_argmin(const double *v, int n) { /* findmin: first NaN, else first minimum */
    int best = 0;
    for (int k = 1; k < n; ++k) {
        if (isnan(v[best])) break;
        if (isnan(v[k]) || v[best] > v[k]) best = k;
    }
    return best;
}

static void fit_pixel(int64_t n, const double *t, const cplx *dcol, const cplx *fccol,
                      const int8_t *state, double omega, const double *xinit, uint32_t flags,
                      int maxfun, oracle_param *par, cplx *outcol, scratch_t *s,
                      uint64_t perturb, double perturb_ulps) {
    const int offsets = (flags & ORACLE_FIT_OFFSETS) != 0;
    const int faint = state != NULL;
    int64_t nv = 0;
    memset(par, 0, sizeof *par);
    /* valid mask (src/Modulation.jl:373-382) and FC phasor (src/Modulation.jl:388) */
    for (int64_t i = 0; i < n; ++i) {
        int ok = 1;
        if (faint) {
            if (flags & ORACLE_ONLY_HIGH) ok = (state[i] == ST_HIGH) || (state[i] == ST_NORMAL);
            if (state[i] == ST_TRANSIENT) ok = 0;
        }
        if (!ok) continue;
        s->t[nv] = t[i];
        s->orig[nv] = i;
        s->d[nv] = dcol[i];
        s->p[nv] = cisj(jl_atan2(fccol[i].im, fccol[i].re));
        nv++;
    }
    if (faint) {
        int8_t *sv = (int8_t *)malloc((size_t)(nv > 0 ? nv : 1));
        double *m = (double *)malloc(sizeof(double) * (size_t)(nv > 0 ? nv : 1));
        int64_t k = 0;
        for (int64_t i = 0; i < n; ++i) {
            int ok = 1;
            if (flags & ORACLE_ONLY_HIGH) ok = (state[i] == ST_HIGH) || (state[i] == ST_NORMAL);
            if (state[i] == ST_TRANSIENT) ok = 0;
            if (ok) sv[k++] = state[i];
        }
        mean_var_power_idx(nv, sv, s->d, s->orig, m, s->w, s->gs, NULL, NULL);
        for (int64_t i = 0; i < nv; ++i) { /* p = power .* FCphasor[valid] */
            s->p[i].re = m[i] * s->p[i].re;
            s->p[i].im = m[i] * s->p[i].im;
        }
        free(sv);
        free(m);
    }
    chi2_ctx c;
    c.n = nv;
    c.t = s->t;
    c.d = s->d;
    c.w = faint ? s->w : NULL;
    c.p = s->p;
    c.omega = omega;
    c.offsets = offsets;
    c.model = s->model;
    c.orig = s->orig;
    c.gs = s->gs;
    c.mod = par;
    c.nfev = 0;
    c.perturb = perturb;
    c.perturb_ulps = perturb_ulps;
    c.order = (int)((flags >> ORACLE_ORDER_SHIFT) & 0xffu);

    double x[2];
    if (xinit) {
        x[0] = xinit[0];
        x[1] = xinit[1];
    } else { /* 8-point ϕ grid at binit = 0.1 (src/Modulation.jl:402-405) */
        double grid[8], f[8];
        oracle_phi_grid(grid);
        for (int k = 0; k < 8; ++k) f[k] = chi2_eval(&c, 0.1, grid[k]);
        x[0] = 0.1;
        x[1] = grid[julia_argmin(f, 8)];
    }
    int status = 0;
    double fx;
    int nf = oracle_newuoa(2, 5, x, 1.0, 1e-3, maxfun, chi2_objfun, &c, &fx);
    if (nf >= maxfun) status |= 2;
    double lklval = chi2_eval(&c, x[0], x[1]);
    double phipi = x[1] + (x[1] < 0 ? PI_F64 : -PI_F64);
    if (lklval > chi2_eval(&c, x[0], phipi)) { /* "bad minima" re-fit (src/Modulation.jl:411-414) */
        status |= 1;
        x[1] = phipi;
        nf = oracle_newuoa(2, 5, x, 1.0, 1e-3, maxfun, chi2_objfun, &c, &fx);
        if (nf >= maxfun) status |= 2;
    }
    par->chi2 = chi2_eval(&c, x[0], x[1]); /* likelihood[idx] = lkl(x) sets mod to x */
    if (isnan(par->chi2)) status |= 4;

    if (outcol) { /* output column over ALL samples (src/Modulation.jl:417-425) */
        double b = par->b, phi = par->phi;
        cplx aa = {par->a_re, par->a_im}, cc = {par->c_re, par->c_im};
        double arga = jl_atan2(aa.im, aa.re);
        for (int64_t i = 0; i < n; ++i) {
            double th = omega * t[i];
            th = th + phi;
            cplx dd = dcol[i];
            if (flags & ORACLE_RECENTER) {
                double ph = b * jl_sin(th); /* getphase: b .* sin.(ω .* t .+ ϕ) .+ angle(a) */
                ph = ph + arga;
                double psi = ph - arga;
                cplx e = cisj(-psi);
                if (offsets) { dd.re = dd.re - cc.re; dd.im = dd.im - cc.im; }
                outcol[i] = cmul(dd, e);
            } else { /* data * exp(-im*angle(mod(t))) */
                cplx mv = cmul(aa, cisj(b * jl_sin(th)));
                if (offsets) { mv.re = cc.re + mv.re; mv.im = cc.im + mv.im; }
                outcol[i] = cmul(dd, cisj(-jl_atan2(mv.im, mv.re)));
            }
        }
    }
    if (par->b < 0) { /* sign normalisation (src/Modulation.jl:427-430) */
        par->b *= -1;
        par->phi += (par->phi < 0 ? PI_F64 : -PI_F64);
    }
    par->nfev = c.nfev;
    par->status = status;
}

int oracle_fit_batch(int64_t n_samples, int64_t n_pixels, const double *t, const double *d,
                     int64_t ldd, const double *fc, int64_t ldfc, const int32_t *fc_of_pixel,
                     const int8_t *state, double omega, const double *xinit, uint32_t flags,
                     int maxfun, oracle_param *params, double *out, int64_t ldo, int nthreads,
                     uint64_t perturb_seed, double perturb_ulps) {
    (void)ldfc;
    const int64_t n = n_samples;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        scratch_t s;
        s.t = (double *)malloc(sizeof(double) * (size_t)n);
        s.w = (double *)malloc(sizeof(double) * (size_t)n);
        s.d = (cplx *)malloc(sizeof(cplx) * (size_t)n);
        s.p = (cplx *)malloc(sizeof(cplx) * (size_t)n);
        s.model = (cplx *)malloc(sizeof(cplx) * (size_t)n);
        s.orig = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
        s.gs = (gsum_t *)malloc(sizeof(gsum_t));
#pragma omp for schedule(dynamic, 1)
        for (int64_t k = 0; k < n_pixels; ++k) {
            const cplx *dcol = (const cplx *)d + (size_t)k * (size_t)ldd;
            const cplx *fcol = (const cplx *)fc + (size_t)fc_of_pixel[k] * (size_t)ldfc;
            cplx *ocol = out ? (cplx *)out + (size_t)k * (size_t)ldo : NULL;
            const uint64_t pk = perturb_seed ? mix64(perturb_seed * 0x100000001B3ull + (uint64_t)k) | 1u : 0;
            fit_pixel(n, t, dcol, fcol, state, omega, xinit, flags, maxfun, &params[k], ocol, &s, pk, perturb_ulps);
        }
        free(s.t);
        free(s.w);
        free(s.d);
        free(s.p);
        free(s.model);
        free(s.orig);
        free(s.gs);
    }
    return 0;
}

/* Elementwise evaluation of the shared Julia-libm restatement (tests/test_jlmath.py).
 * fn: 0 sin, 1 cos, 2 sincos → (s, c) pairs in out[2i..2i+1], 3 atan, 4 atan(x[i], y[i]),
 *     5 hypot(x[i], y[i]), 6 rem_pio2 → (n, hi, lo) triples in out[3i..3i+2], 7 hypot_nb,
 *     8 sin through the branch-free regime forms, 9 sincos likewise (pairs), 10 sin(fl(x[i] + y[0]))
 *     through the Payne–Hanek table of x and the shift of ϕ = y[0] (NaN where it does not apply) */
int oracle_jl_eval(int fn, int64_t n, const double *x, const double *y, double *out) {
    if ((fn == 4 || fn == 5 || fn == 7 || fn == 10) && n > 0 && !y) return -1;
    for (int64_t i = 0; i < n; ++i) {
        switch (fn) {
        case 0: out[i] = jl_sin(x[i]); break;
        case 1: out[i] = jl_cos(x[i]); break;
        case 2: jl_sincos(x[i], &out[2 * i], &out[2 * i + 1]); break;
        case 3: out[i] = jl_atan(x[i]); break;
        case 4: out[i] = jl_atan2(x[i], y[i]); break;
        case 5: out[i] = jl_hypot(x[i], y[i]); break;
        case 7: out[i] = jl_hypot_nb(x[i], y[i]); break;
        case 8: out[i] = jl_sin_sel(x[i]); break;
        case 9: jl_sincos_sel(x[i], &out[2 * i], &out[2 * i + 1]); break;
        case 10: { /* jl_sin(fl(x[i] + y[0])) through the Payne–Hanek table and shift (NaN when
                    * the shift does not apply to this x range and ϕ; the exact path then takes
                    * the general forms) */
            if (i == 0) {
                double xmin = x[0], xmax = x[0];
                for (int64_t k = 1; k < n; ++k) {
                    xmin = x[k] < xmin ? x[k] : xmin;
                    xmax = x[k] > xmax ? x[k] : xmax;
                }
                uint64_t klo, khi, d3;
                const int on = jlm_ph_shift(xmin, xmax, y[0], &klo, &khi, &d3);
                for (int64_t k = 0; k < n; ++k) {
                    uint64_t wlo, whi, a3;
                    jlm_ph_table_entry(x[k], &wlo, &whi, &a3);
                    out[k] = on ? jl_sin_ph_shifted(wlo, whi, a3, klo, khi, d3) : __builtin_nan("");
                }
            }
            break;
        }
        case 6: {
            double hi, lo;
            const int q = jl_rem_pio2(x[i], &hi, &lo);
            out[3 * i] = (double)q;
            out[3 * i + 1] = hi;
            out[3 * i + 2] = lo;
            break;
        }
        default: return -1;
        }
    }
    return 0;
}
