// Device-side Powell NEWUOA for the per-series (b, ϕ) fit.
//
// Replaces OptimPackNextGen.Powell.Newuoa.newuoa as called by minimize!
// (src/Modulation.jl:332-342: newuoa(f, xinit, 1, 1e-3; check=false), npt = 2n+1 = 5,
// maxfun = 30n = 60 by default).  Algorithm: M.J.D. Powell, "The NEWUOA software for
// unconstrained optimization without derivatives" (DAMTP 2004/NA05) — NEWUOB, TRSAPP,
// BIGLAG, BIGDEN, UPDATE.  This is a structured re-implementation for GPU threads: fixed
// N/NPT known at compile time so every array lives in registers, runtime interpolation-point
// indices go through branch-free select helpers, and the objective is a device functor so the
// same code serves the wave-cooperative exact evaluator and the lane-per-series harmonic one.
// Every floating-point expression keeps the operation order of the published algorithm
// (compile with -ffp-contract=off) so trajectories agree with the CPU oracle to rounding.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#include <type_traits>

#include "gpd_jlmath.h"  // OptimPackNextGen is pure Julia: Julia Base cos/sin

namespace gpd {

#define GPD_HD __host__ __device__ __forceinline__
#define GPD_HDN __host__ __device__
// the large NEWUOA subroutines stay out of line: inlined into one body their temporaries
// exceed the register file (512 VGPR+AGPR and ~1.4 KB of spills per lane)
#define GPD_HDX __host__ __device__

// ---------------------------------------------------------------- select helpers ------
template <int L>
GPD_HD double rd(const double (&a)[L], int k) {  // a[k], k runtime (0-based)
    double v = a[0];
#pragma unroll
    for (int j = 1; j < L; ++j) v = (k == j) ? a[j] : v;
    return v;
}
template <int L>
GPD_HD void wr(double (&a)[L], int k, double v) {
#pragma unroll
    for (int j = 0; j < L; ++j)
        if (k == j) a[j] = v;
}
template <int R, int C>
GPD_HD double rd2(const double (&a)[R][C], int r, int c) {  // a[r][c], r runtime, c static
    double v = a[0][c];
#pragma unroll
    for (int j = 1; j < R; ++j) v = (r == j) ? a[j][c] : v;
    return v;
}
template <int R, int C>
GPD_HD void wr2(double (&a)[R][C], int r, int c, double v) {
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (r == j) a[j][c] = v;
}
// column c runtime, row static
template <int R, int C>
GPD_HD double rdc(const double (&a)[R][C], int r, int c) {
    double v = a[r][0];
#pragma unroll
    for (int j = 1; j < C; ++j) v = (c == j) ? a[r][j] : v;
    return v;
}
template <int R, int C>
GPD_HD void wrc(double (&a)[R][C], int r, int c, double v) {
#pragma unroll
    for (int j = 0; j < C; ++j)
        if (c == j) a[r][j] = v;
}

// has_multi<F>: the objective F can evaluate NP independent points at once
// (f.template multi<NP>(pts, vals), every lane of the fit getting every value) — the harmonic
// fit's lane groups evaluate them in parallel, each point by one lane with the canonical
// objective's single-lane form (the same bits as one at a time)
template <class F, class = void>
struct has_multi : std::false_type {};
template <class F>
struct has_multi<F, std::void_t<decltype(F::kMulti)>> : std::integral_constant<bool, F::kMulti> {};

constexpr double kTwoPi = 6.283185307179586476925286766559;  // 8·atan(1)
// cos/sin of the fixed trial angles i·dang, dang = kTwoPi/50, of the three angle searches
// (TRSAPP, BIGLAG, BIGDEN: 49 angles each), exactly as Julia Base's cos/sin give them
// (gpd_jlmath.h, the oracle's too; oracle/tools/angle_table.py).  Read by uniform index (scalar loads) instead of 98 fp64
// sin/cos evaluations per search — the bulk of the device NEWUOA's vector instructions.
constexpr double kAngCos[50] = {
    0x1.0000000000000p+0, 0x1.fbf675480d903p-1, 0x1.efea21d101ee0p-1, 0x1.dc0ba9def5ae5p-1,
    0x1.c0ab44e81c059p-1, 0x1.9e3779b97f4a8p-1, 0x1.753b603d2b816p-1, 0x1.465c6feb501bbp-1,
    0x1.1257e3c182b50p-1, 0x1.b3ff7c925819cp-2, 0x1.3c6ef372fe950p-2, 0x1.7fc1c65037a75p-3,
    0x1.0130a1be09374p-4, -0x1.0130a1be0937bp-4, -0x1.7fc1c65037a80p-3, -0x1.3c6ef372fe952p-2,
    -0x1.b3ff7c925819dp-2, -0x1.1257e3c182b53p-1, -0x1.465c6feb501bcp-1, -0x1.753b603d2b817p-1,
    -0x1.9e3779b97f4a7p-1, -0x1.c0ab44e81c059p-1, -0x1.dc0ba9def5ae5p-1, -0x1.efea21d101ee0p-1,
    -0x1.fbf675480d903p-1, -0x1.0000000000000p+0, -0x1.fbf675480d903p-1, -0x1.efea21d101ee0p-1,
    -0x1.dc0ba9def5ae3p-1, -0x1.c0ab44e81c059p-1, -0x1.9e3779b97f4a6p-1, -0x1.753b603d2b816p-1,
    -0x1.465c6feb501bap-1, -0x1.1257e3c182b4ep-1, -0x1.b3ff7c9258193p-2, -0x1.3c6ef372fe952p-2,
    -0x1.7fc1c65037a79p-3, -0x1.0130a1be0936dp-4, 0x1.0130a1be09392p-4, 0x1.7fc1c65037a8bp-3,
    0x1.3c6ef372fe94cp-2, 0x1.b3ff7c925819bp-2, 0x1.1257e3c182b52p-1, 0x1.465c6feb501bep-1,
    0x1.753b603d2b819p-1, 0x1.9e3779b97f4abp-1, 0x1.c0ab44e81c059p-1, 0x1.dc0ba9def5ae5p-1,
    0x1.efea21d101ee1p-1, 0x1.fbf675480d903p-1,
};
constexpr double kAngSin[50] = {
    0x0.0p+0, 0x1.00aeb5da15be0p-3, 0x1.fd511fa1c0796p-3, 0x1.78f5a48a8a919p-2,
    0x1.ed50d5cbfa952p-2, 0x1.2cf2304755a5ep-1, 0x1.5e7cf55112014p-1, 0x1.8a80b635b6beap-1,
    0x1.b04bbff642e86p-1, 0x1.cf457dcdc158cp-1, 0x1.e6f0e134454ffp-1, 0x1.f6ee5ac2509ffp-1,
    0x1.fefd5bfe443fep-1, 0x1.fefd5bfe443fep-1, 0x1.f6ee5ac2509fep-1, 0x1.e6f0e134454ffp-1,
    0x1.cf457dcdc158bp-1, 0x1.b04bbff642e85p-1, 0x1.8a80b635b6beap-1, 0x1.5e7cf55112012p-1,
    0x1.2cf2304755a5fp-1, 0x1.ed50d5cbfa950p-2, 0x1.78f5a48a8a915p-2, 0x1.fd511fa1c0797p-3,
    0x1.00aeb5da15bdap-3, -0x1.72cece675d1fdp-52, -0x1.00aeb5da15be1p-3, -0x1.fd511fa1c079ep-3,
    -0x1.78f5a48a8a91fp-2, -0x1.ed50d5cbfa953p-2, -0x1.2cf2304755a60p-1, -0x1.5e7cf55112014p-1,
    -0x1.8a80b635b6bebp-1, -0x1.b04bbff642e88p-1, -0x1.cf457dcdc158ep-1, -0x1.e6f0e134454ffp-1,
    -0x1.f6ee5ac2509ffp-1, -0x1.fefd5bfe443fep-1, -0x1.fefd5bfe443fep-1, -0x1.f6ee5ac2509fep-1,
    -0x1.e6f0e13445500p-1, -0x1.cf457dcdc158cp-1, -0x1.b04bbff642e85p-1, -0x1.8a80b635b6be8p-1,
    -0x1.5e7cf55112010p-1, -0x1.2cf2304755a59p-1, -0x1.ed50d5cbfa952p-2, -0x1.78f5a48a8a917p-2,
    -0x1.fd511fa1c078bp-3, -0x1.00aeb5da15bcfp-3,
};

// DIRECT = true: the object lives in LDS (one per lane, k_fit_harmonic), so runtime indices
// address it directly; false: per-thread objects held in registers, runtime indices become
// select chains (no scratch).
// Diagnostics build (build.py --diag, GPD_FIT_PROF=1): cycles of NEWUOA's phases per lane
// (TRSAPP, BIGLAG, BIGDEN, UPDATE), summed over the fit's lanes by k_fit_harmonic.
#if defined(GPD_DIAG) && defined(__HIP_DEVICE_COMPILE__)
#define GPD_NW_T0(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
// lane-level cycles in prof_[slot], wave-level (counted by the first active lane of each
// execution of the phase) in prof_[8 + slot]
#define GPD_NW_T1(v, slot)                                                            \
    do {                                                                             \
        const unsigned long long dt_ = __builtin_amdgcn_s_memtime() - (v);           \
        prof_[slot] += dt_;                                                          \
        if ((int)threadIdx.x == __builtin_amdgcn_readfirstlane((int)threadIdx.x))     \
            prof_[8 + (slot)] += dt_;                                                \
    } while (0)
#else
#define GPD_NW_T0(v)
#define GPD_NW_T1(v, slot)
#endif

// LPS: lanes per fit (k_fit_harmonic<LPS>: a group of LPS consecutive lanes runs one NEWUOA,
// replicated — every lane of the group holds the same values and takes the same branches — and
// splits the 49-angle searches of TRSAPP, BIGLAG and BIGDEN across its lanes, angle_search).
template <int N, int NPT, bool DIRECT = false, int LPS = 1>
struct Newuoa {
#ifdef GPD_DIAG
    unsigned long long prof_[16];
#endif
    template <int L>
    GPD_HD static double rd_(const double (&a)[L], int k) {
        if constexpr (DIRECT) return a[k];
        else return rd(a, k);
    }
    template <int L>
    GPD_HD static void wr_(double (&a)[L], int k, double v) {
        if constexpr (DIRECT) a[k] = v;
        else wr(a, k, v);
    }
    template <int R, int C>
    GPD_HD static double rd2_(const double (&a)[R][C], int r, int c) {
        if constexpr (DIRECT) return a[r][c];
        else return rd2(a, r, c);
    }
    template <int R, int C>
    GPD_HD static void wr2_(double (&a)[R][C], int r, int c, double v) {
        if constexpr (DIRECT) a[r][c] = v;
        else wr2(a, r, c, v);
    }
    template <int R, int C>
    GPD_HD static double rdc_(const double (&a)[R][C], int r, int c) {
        if constexpr (DIRECT) return a[r][c];
        else return rdc(a, r, c);
    }
    template <int R, int C>
    GPD_HD static void wrc_(double (&a)[R][C], int r, int c, double v) {
        if constexpr (DIRECT) a[r][c] = v;
        else wrc(a, r, c, v);
    }

    static constexpr int NDIM = NPT + N;
    static constexpr int NPTM = NPT - N - 1;
    static constexpr int NH = N * (N + 1) / 2;

    // persistent state (NEWUOB)
    double xbase[N], xopt[N], xnew[N], xpt[NPT][N], fval[NPT], gq[N], hq[NH], pq[NPT];
    double bmat[NDIM][N], zmat[NPT][NPTM], d[N], vlag[NDIM], w[NDIM];


    // Powell's search over the trial angles i·2π/50 (TRSAPP's boundary iterations, BIGLAG,
    // BIGDEN): f(0) = fbeg, f(i) = val(i) for i = 1..49.  The published loop walks i in order
    // keeping the first strictly better value (better(a, b); NaN is never better) and the values
    // around it: fbest = f(isave), tempa = f(isave − 1) (f(−1) = f(49)), tempb = f(isave + 1)
    // (f(50) = fbeg).  isave is therefore the first index of the best key among the non-NaN
    // values, index 0 winning ties (none of f(1..49) strictly better than fbeg, or fbeg NaN).
    // LPS > 1 (device): lane r of the group takes i = r + 1, r + 1 + LPS, … in order and keeps
    // its first best, the group combines (value, index) pairs by a butterfly whose rule — a
    // valid value strictly better wins, between equals the smaller index — picks that same
    // index on every lane; fbest, tempa, tempb are then val() at isave and its neighbours,
    // recomputed with the same operations: the same bits as the sequential loop.
    template <class V, class B>
    GPD_HD static void angle_search(double fbeg, V &&val, B &&better, int &isave, double &fbest,
                                    double &tempa, double &tempb) {
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (LPS > 1) {
            const int r = (int)threadIdx.x & (LPS - 1);
            int bi = 0;
            double bv = __builtin_nan("");
            for (int i = r + 1; i <= 49; i += LPS) {
                const double v = val(i);
                if (v == v && (bv != bv || better(v, bv))) {
                    bv = v;
                    bi = i;
                }
            }
            auto merge = [&](double pv, int pi) {
                if (pv == pv && (bv != bv || better(pv, bv) || (!better(bv, pv) && pi < bi))) {
                    bv = pv;
                    bi = pi;
                }
            };
            if constexpr (LPS >= 8) merge(lane_xor<4>(bv), __shfl_xor(bi, 4, 64));
            if constexpr (LPS >= 4) merge(lane_xor<2>(bv), __shfl_xor(bi, 2, 64));
            merge(lane_xor<1>(bv), __shfl_xor(bi, 1, 64));
            isave = better(bv, fbeg) ? bi : 0;
            fbest = isave == 0 ? fbeg : val(isave);
            tempa = isave == 0 ? val(49) : isave == 1 ? fbeg : val(isave - 1);
            tempb = isave == 49 ? fbeg : val(isave + 1);
            return;
        }
#endif
        double fsav = fbeg, fnew = fbeg;
        fbest = fbeg;
        tempa = 0.0;
        tempb = 0.0;
        isave = 0;
#pragma unroll 7  // 49 = 7·7 trial angles: independent values, ILP across 7
        for (int i = 1; i <= 49; ++i) {
            fnew = val(i);
            if (better(fnew, fbest)) {
                fbest = fnew;
                isave = i;
                tempa = fsav;
            } else if (i == isave + 1) {
                tempb = fnew;
            }
            fsav = fnew;
        }
        if (isave == 0) tempa = fnew;
        if (isave == 49) tempb = fbeg;
    }

    // ---------------------------------------------------- hd = ∇²Q · v (TRSAPP label 170)
    GPD_HD void hess_mul(const double (&v)[N], double (&hd)[N]) const {
#pragma unroll
        for (int i = 0; i < N; ++i) hd[i] = 0.0;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            double temp = 0.0;
#pragma unroll
            for (int j = 0; j < N; ++j) temp = temp + xpt[k][j] * v[j];
            temp = temp * pq[k];
#pragma unroll
            for (int i = 0; i < N; ++i) hd[i] = hd[i] + temp * xpt[k][i];
        }
        int ih = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
#pragma unroll
            for (int i = 0; i <= j; ++i) {
                if (i < j) hd[j] = hd[j] + hq[ih] * v[i];
                hd[i] = hd[i] + hq[ih] * v[j];
                ++ih;
            }
        }
    }

    // ------------------------------------------------------------------------- TRSAPP
    // Truncated CG + 2-D boundary search for the trust-region step.  Writes step, crvmin.
    GPD_HDX void trsapp(double delta, double (&step)[N], double &crvmin) const {
        double dv[N], g[N], hd[N], hs[N];
        const double delsq = delta * delta;
        int iterc = 0;
        const int itermax = N;
        double dd, ds, ss, gg, ggbeg, qred, bstep, alpha, dhd, temp;
        double sg = 0, shs = 0;
        hess_mul(xopt, hd);
        qred = 0.0;
        dd = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            step[i] = 0.0;
            hs[i] = 0.0;
            g[i] = gq[i] + hd[i];
            dv[i] = -g[i];
            dd = dd + dv[i] * dv[i];
        }
        crvmin = 0.0;
        if (dd == 0.0) return;
        ds = 0.0;
        ss = 0.0;
        gg = dd;
        ggbeg = gg;
        // ---- conjugate-gradient phase
        for (;;) {
            ++iterc;
            temp = delsq - ss;
            bstep = temp / (ds + sqrt(ds * ds + dd * temp));
            hess_mul(dv, hd);
            dhd = 0.0;
#pragma unroll
            for (int j = 0; j < N; ++j) dhd = dhd + dv[j] * hd[j];
            alpha = bstep;
            if (dhd > 0.0) {
                temp = dhd / dd;
                if (iterc == 1) crvmin = temp;
                crvmin = fmin(crvmin, temp);
                alpha = fmin(alpha, gg / dhd);
            }
            const double qadd = alpha * (gg - 0.5 * alpha * dhd);
            qred = qred + qadd;
            const double ggsav = gg;
            gg = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                step[i] = step[i] + alpha * dv[i];
                hs[i] = hs[i] + alpha * hd[i];
                gg = gg + (g[i] + hs[i]) * (g[i] + hs[i]);
            }
            if (!(alpha < bstep)) break;  // reached the boundary
            if (qadd <= 0.01 * qred) return;
            if (gg <= 1.0e-4 * ggbeg) return;
            if (iterc == itermax) return;
            temp = gg / ggsav;
            dd = 0.0;
            ds = 0.0;
            ss = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                dv[i] = temp * dv[i] - g[i] - hs[i];
                dd = dd + dv[i] * dv[i];
                ds = ds + dv[i] * step[i];
                ss = ss + step[i] * step[i];
            }
            if (ds <= 0.0) return;
            if (!(ss < delsq)) break;
        }
        crvmin = 0.0;
        // ---- alternative iterations on the boundary
        for (;;) {
            if (gg <= 1.0e-4 * ggbeg) return;
            sg = 0.0;
            shs = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                sg = sg + step[i] * g[i];
                shs = shs + step[i] * hs[i];
            }
            const double sgk = sg + shs;
            const double angtest = sgk / sqrt(gg * delsq);
            if (angtest <= -0.99) return;
            ++iterc;
            temp = sqrt(delsq * gg - sgk * sgk);
            const double ta = delsq / temp, tb = sgk / temp;
#pragma unroll
            for (int i = 0; i < N; ++i) dv[i] = ta * (g[i] + hs[i]) - tb * step[i];
            hess_mul(dv, hd);
            double dg = 0.0, dhs = 0.0;
            dhd = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                dg = dg + dv[i] * g[i];
                dhd = dhd + hd[i] * dv[i];
                dhs = dhs + hd[i] * step[i];
            }
            const double cf = 0.5 * (shs - dhd);
            const double qbeg = sg + cf;
            double qmin, tempa, tempb;
            int isave;
            const int iu = 49;
            const double dang = kTwoPi / (double)(iu + 1);
            angle_search(
                qbeg,
                [&](int i) {
                    const double cth = kAngCos[i], sth = kAngSin[i];
                    return (sg + cf * cth) * cth + (dg + dhs * cth) * sth;
                },
                [](double a, double b) { return a < b; }, isave, qmin, tempa, tempb);
            double ang = 0.0;
            if (tempa != tempb) {
                tempa = tempa - qmin;
                tempb = tempb - qmin;
                ang = 0.5 * (tempa - tempb) / (tempa + tempb);
            }
            ang = dang * ((double)isave + ang);
            double cth, sth;  // = jl_cos(ang), jl_sin(ang): one reduction (the same bits, r4)
            jl_sincos(ang, &sth, &cth);
            const double reduc = qbeg - (sg + cf * cth) * cth - (dg + dhs * cth) * sth;
            gg = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                step[i] = cth * step[i] + sth * dv[i];
                hs[i] = cth * hs[i] + sth * hd[i];
                gg = gg + (g[i] + hs[i]) * (g[i] + hs[i]);
            }
            qred = qred + reduc;
            const double ratio = reduc / qred;
            if (!(iterc < itermax && ratio > 0.01)) return;
        }
    }

    // H column of point knew (1-based): hcol[k] = Σ_j ±zmat[knew][j] zmat[k][j]
    GPD_HD void h_column(int knew, int idz, double (&hcol)[NPT]) const {
#pragma unroll
        for (int k = 0; k < NPT; ++k) hcol[k] = 0.0;
#pragma unroll
        for (int j = 0; j < NPTM; ++j) {
            double temp = rd2_(zmat, knew - 1, j);
            if (j + 1 < idz) temp = -temp;
#pragma unroll
            for (int k = 0; k < NPT; ++k) hcol[k] = hcol[k] + temp * zmat[k][j];
        }
    }

    // ------------------------------------------------------------------------- BIGLAG
    // Step that (approximately) maximises |Lagrange function knew| within radius delta.
    GPD_HDX void biglag(int idz, int knew, double delta, double &alpha) {
        double hcol[NPT], gc[N], gd[N], s[N], wv[N];
        const double delsq = delta * delta;
        h_column(knew, idz, hcol);
        alpha = rd_(hcol, knew - 1);
        double dd = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            d[i] = rd2_(xpt, knew - 1, i) - xopt[i];
            gc[i] = rd2_(bmat, knew - 1, i);
            gd[i] = 0.0;
            dd = dd + d[i] * d[i];
        }
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            double temp = 0.0, sum = 0.0;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                temp = temp + xpt[k][j] * xopt[j];
                sum = sum + xpt[k][j] * d[j];
            }
            temp = hcol[k] * temp;
            sum = hcol[k] * sum;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                gc[i] = gc[i] + temp * xpt[k][i];
                gd[i] = gd[i] + sum * xpt[k][i];
            }
        }
        double gg = 0.0, sp = 0.0, dhd = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            gg = gg + gc[i] * gc[i];
            sp = sp + d[i] * gc[i];
            dhd = dhd + d[i] * gd[i];
        }
        double scale = delta / sqrt(dd);
        if (sp * dhd < 0.0) scale = -scale;
        double temp = 0.0;
        if (sp * sp > 0.99 * dd * gg) temp = 1.0;
        double tau = scale * (fabs(sp) + 0.5 * scale * fabs(dhd));
        if (gg * delsq < 0.01 * tau * tau) temp = 1.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            d[i] = scale * d[i];
            gd[i] = scale * gd[i];
            s[i] = gc[i] + temp * gd[i];
        }
        for (int iterc = 1;; ++iterc) {
            double ss = 0.0;
            dd = 0.0;
            sp = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                dd = dd + d[i] * d[i];
                sp = sp + d[i] * s[i];
                ss = ss + s[i] * s[i];
            }
            temp = dd * ss - sp * sp;
            if (temp <= 1.0e-8 * dd * ss) return;
            const double denom = sqrt(temp);
#pragma unroll
            for (int i = 0; i < N; ++i) {
                s[i] = (dd * s[i] - sp * d[i]) / denom;
                wv[i] = 0.0;
            }
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                double sum = 0.0;
#pragma unroll
                for (int j = 0; j < N; ++j) sum = sum + xpt[k][j] * s[j];
                sum = hcol[k] * sum;
#pragma unroll
                for (int i = 0; i < N; ++i) wv[i] = wv[i] + sum * xpt[k][i];
            }
            double cf1 = 0.0, cf2 = 0.0, cf3 = 0.0, cf4 = 0.0, cf5 = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                cf1 = cf1 + s[i] * wv[i];
                cf2 = cf2 + d[i] * gc[i];
                cf3 = cf3 + s[i] * gc[i];
                cf4 = cf4 + d[i] * gd[i];
                cf5 = cf5 + s[i] * gd[i];
            }
            cf1 = 0.5 * cf1;
            cf4 = 0.5 * cf4 - cf1;
            const double taubeg = cf1 + cf2 + cf4;
            double taumax, tempa, tempb;
            int isave;
            const int iu = 49;
            const double dang = kTwoPi / (double)(iu + 1);
            angle_search(
                taubeg,
                [&](int i) {
                    const double cth = kAngCos[i], sth = kAngSin[i];
                    return cf1 + (cf2 + cf4 * cth) * cth + (cf3 + cf5 * cth) * sth;
                },
                [](double a, double b) { return fabs(a) > fabs(b); }, isave, taumax, tempa, tempb);
            double stp = 0.0;
            if (tempa != tempb) {
                tempa = tempa - taumax;
                tempb = tempb - taumax;
                stp = 0.5 * (tempa - tempb) / (tempa + tempb);
            }
            const double ang = dang * ((double)isave + stp);
            double cth, sth;  // = jl_cos(ang), jl_sin(ang): one reduction (the same bits, r4)
            jl_sincos(ang, &sth, &cth);
            tau = cf1 + (cf2 + cf4 * cth) * cth + (cf3 + cf5 * cth) * sth;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                d[i] = cth * d[i] + sth * s[i];
                gd[i] = cth * gd[i] + sth * wv[i];
                s[i] = gc[i] + gd[i];
            }
            if (fabs(tau) <= 1.1 * fabs(taubeg)) return;
            if (!(iterc < N)) return;
        }
    }

    // ------------------------------------------------------------------------- BIGDEN
    // Alternative step maximising |denominator| of the update; sets w (Wcheck), vlag, beta.
    GPD_HDX void bigden(int idz, int kopt, int knew, double &beta) {
        double hw[N + NPT];                    // W(1..N+NPT) of the published routine
        double s[N], den[9], denex[9], par[9];
        double wvec[NDIM][5], prod[NDIM][5];
#pragma unroll
        for (int k = 0; k < NPT; ++k) hw[N + k] = 0.0;
#pragma unroll
        for (int j = 0; j < NPTM; ++j) {
            double temp = rd2_(zmat, knew - 1, j);
            if (j + 1 < idz) temp = -temp;
#pragma unroll
            for (int k = 0; k < NPT; ++k) hw[N + k] = hw[N + k] + temp * zmat[k][j];
        }
        double alpha = hw[N];
#pragma unroll
        for (int k = 1; k < NPT; ++k) alpha = (knew - 1 == k) ? hw[N + k] : alpha;

        double dd = 0.0, ds = 0.0, ss = 0.0, xoptsq = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            dd = dd + d[i] * d[i];
            s[i] = rd2_(xpt, knew - 1, i) - xopt[i];
            ds = ds + d[i] * s[i];
            ss = ss + s[i] * s[i];
            xoptsq = xoptsq + xopt[i] * xopt[i];
        }
        if (ds * ds > 0.99 * dd * ss) {
            int ksav = knew;
            double dtest = ds * ds / ss;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                if (k + 1 != kopt) {
                    double dstemp = 0.0, sstemp = 0.0;
#pragma unroll
                    for (int i = 0; i < N; ++i) {
                        const double diff = xpt[k][i] - xopt[i];
                        dstemp = dstemp + d[i] * diff;
                        sstemp = sstemp + diff * diff;
                    }
                    if (dstemp * dstemp / sstemp < dtest) {
                        ksav = k + 1;
                        dtest = dstemp * dstemp / sstemp;
                        ds = dstemp;
                        ss = sstemp;
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < N; ++i) s[i] = rd2_(xpt, ksav - 1, i) - xopt[i];
        }
        double ssden = dd * ss - ds * ds;
        double densav = 0.0;
        double tau = 0.0, tempa = 0.0, tempb = 0.0, tempc, sum, denold = 0.0, denmax = 0.0;
        for (int iterc = 1;; ++iterc) {
            double temp = 1.0 / sqrt(ssden);
            double xoptd = 0.0, xopts = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                s[i] = temp * (dd * s[i] - ds * d[i]);
                xoptd = xoptd + xopt[i] * d[i];
                xopts = xopts + xopt[i] * s[i];
            }
            tempa = 0.5 * xoptd * xoptd;
            tempb = 0.5 * xopts * xopts;
            den[0] = dd * (xoptsq + 0.5 * dd) + tempa + tempb;
            den[1] = 2.0 * xoptd * dd;
            den[2] = 2.0 * xopts * dd;
            den[3] = tempa - tempb;
            den[4] = xoptd * xopts;
#pragma unroll
            for (int i = 5; i < 9; ++i) den[i] = 0.0;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                double ta = 0.0, tb = 0.0, tc = 0.0;
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    ta = ta + xpt[k][i] * d[i];
                    tb = tb + xpt[k][i] * s[i];
                    tc = tc + xpt[k][i] * xopt[i];
                }
                wvec[k][0] = 0.25 * (ta * ta + tb * tb);
                wvec[k][1] = ta * tc;
                wvec[k][2] = tb * tc;
                wvec[k][3] = 0.25 * (ta * ta - tb * tb);
                wvec[k][4] = 0.5 * ta * tb;
            }
#pragma unroll
            for (int i = 0; i < N; ++i) {
                wvec[NPT + i][0] = 0.0;
                wvec[NPT + i][1] = d[i];
                wvec[NPT + i][2] = s[i];
                wvec[NPT + i][3] = 0.0;
                wvec[NPT + i][4] = 0.0;
            }
#pragma unroll
            for (int jc = 0; jc < 5; ++jc) {
                const bool full = (jc == 1 || jc == 2);
#pragma unroll
                for (int k = 0; k < NPT; ++k) prod[k][jc] = 0.0;
#pragma unroll
                for (int j = 0; j < NPTM; ++j) {
                    sum = 0.0;
#pragma unroll
                    for (int k = 0; k < NPT; ++k) sum = sum + zmat[k][j] * wvec[k][jc];
                    if (j + 1 < idz) sum = -sum;
#pragma unroll
                    for (int k = 0; k < NPT; ++k) prod[k][jc] = prod[k][jc] + sum * zmat[k][j];
                }
                if (full) {
#pragma unroll
                    for (int k = 0; k < NPT; ++k) {
                        sum = 0.0;
#pragma unroll
                        for (int j = 0; j < N; ++j) sum = sum + bmat[k][j] * wvec[NPT + j][jc];
                        prod[k][jc] = prod[k][jc] + sum;
                    }
                }
#pragma unroll
                for (int j = 0; j < N; ++j) {
                    sum = 0.0;
                    const int nw = full ? NDIM : NPT;
#pragma unroll
                    for (int i = 0; i < NDIM; ++i)
                        if (i < nw) sum = sum + bmat[i][j] * wvec[i][jc];
                    prod[NPT + j][jc] = sum;
                }
            }
#pragma unroll
            for (int k = 0; k < NDIM; ++k) {
                sum = 0.0;
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    par[i] = 0.5 * prod[k][i] * wvec[k][i];
                    sum = sum + par[i];
                }
                den[0] = den[0] - par[0] - sum;
                tempa = prod[k][0] * wvec[k][1] + prod[k][1] * wvec[k][0];
                tempb = prod[k][1] * wvec[k][3] + prod[k][3] * wvec[k][1];
                tempc = prod[k][2] * wvec[k][4] + prod[k][4] * wvec[k][2];
                den[1] = den[1] - tempa - 0.5 * (tempb + tempc);
                den[5] = den[5] - 0.5 * (tempb - tempc);
                tempa = prod[k][0] * wvec[k][2] + prod[k][2] * wvec[k][0];
                tempb = prod[k][1] * wvec[k][4] + prod[k][4] * wvec[k][1];
                tempc = prod[k][2] * wvec[k][3] + prod[k][3] * wvec[k][2];
                den[2] = den[2] - tempa - 0.5 * (tempb - tempc);
                den[6] = den[6] - 0.5 * (tempb + tempc);
                tempa = prod[k][0] * wvec[k][3] + prod[k][3] * wvec[k][0];
                den[3] = den[3] - tempa - par[1] + par[2];
                tempa = prod[k][0] * wvec[k][4] + prod[k][4] * wvec[k][0];
                tempb = prod[k][1] * wvec[k][2] + prod[k][2] * wvec[k][1];
                den[4] = den[4] - tempa - 0.5 * tempb;
                den[7] = den[7] - par[3] + par[4];
                tempa = prod[k][3] * wvec[k][4] + prod[k][4] * wvec[k][3];
                den[8] = den[8] - 0.5 * tempa;
            }
            double pk[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) pk[i] = rd2_(prod, knew - 1, i);
            sum = 0.0;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                par[i] = 0.5 * pk[i] * pk[i];
                sum = sum + par[i];
            }
            denex[0] = alpha * den[0] + par[0] + sum;
            tempa = 2.0 * pk[0] * pk[1];
            tempb = pk[1] * pk[3];
            tempc = pk[2] * pk[4];
            denex[1] = alpha * den[1] + tempa + tempb + tempc;
            denex[5] = alpha * den[5] + tempb - tempc;
            tempa = 2.0 * pk[0] * pk[2];
            tempb = pk[1] * pk[4];
            tempc = pk[2] * pk[3];
            denex[2] = alpha * den[2] + tempa + tempb - tempc;
            denex[6] = alpha * den[6] + tempb + tempc;
            tempa = 2.0 * pk[0] * pk[3];
            denex[3] = alpha * den[3] + tempa + par[1] - par[2];
            tempa = 2.0 * pk[0] * pk[4];
            denex[4] = alpha * den[4] + tempa + pk[1] * pk[2];
            denex[7] = alpha * den[7] + par[3] - par[4];
            denex[8] = alpha * den[8] + pk[3] * pk[4];

            sum = denex[0] + denex[1] + denex[3] + denex[5] + denex[7];
            denold = sum;
            int isave = 0;
            const int iu = 49;
            const double dang = kTwoPi / (double)(iu + 1);
            par[0] = 1.0;
            // the published loop over i = 1..49 (first strictly larger |Σ denex·par|) as
            // angle_search: the same index and values (split across the group for LPS > 1)
            angle_search(
                denold,
                [&](int i) {
                    double pw[9];
                    pw[0] = 1.0;
                    pw[1] = kAngCos[i];
                    pw[2] = kAngSin[i];
#pragma unroll
                    for (int j = 3; j <= 7; j += 2) {
                        pw[j] = pw[1] * pw[j - 2] - pw[2] * pw[j - 1];
                        pw[j + 1] = pw[1] * pw[j - 1] + pw[2] * pw[j - 2];
                    }
                    double sm = 0.0;
#pragma unroll
                    for (int j = 0; j < 9; ++j) sm = sm + denex[j] * pw[j];
                    return sm;
                },
                [](double a, double b) { return fabs(a) > fabs(b); }, isave, denmax, tempa, tempb);
            double stp = 0.0;
            if (tempa != tempb) {
                tempa = tempa - denmax;
                tempb = tempb - denmax;
                stp = 0.5 * (tempa - tempb) / (tempa + tempb);
            }
            const double ang = dang * ((double)isave + stp);
            jl_sincos(ang, &par[2], &par[1]);  // = jl_cos(ang), jl_sin(ang) (the same bits)
#pragma unroll
            for (int j = 3; j <= 7; j += 2) {
                par[j] = par[1] * par[j - 2] - par[2] * par[j - 1];
                par[j + 1] = par[1] * par[j - 1] + par[2] * par[j - 2];
            }
            beta = 0.0;
            denmax = 0.0;
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                beta = beta + den[j] * par[j];
                denmax = denmax + denex[j] * par[j];
            }
#pragma unroll
            for (int k = 0; k < NDIM; ++k) {
                vlag[k] = 0.0;
#pragma unroll
                for (int j = 0; j < 5; ++j) vlag[k] = vlag[k] + prod[k][j] * par[j];
            }
            tau = rd_(vlag, knew - 1);
            dd = 0.0;
            tempa = 0.0;
            tempb = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                d[i] = par[1] * d[i] + par[2] * s[i];
                hw[i] = xopt[i] + d[i];
                dd = dd + d[i] * d[i];
                tempa = tempa + d[i] * hw[i];
                tempb = tempb + hw[i] * hw[i];
            }
            if (iterc >= N) break;
            if (iterc > 1) densav = fmax(densav, denold);
            if (fabs(denmax) <= 1.1 * fabs(densav)) break;
            densav = denmax;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                temp = tempa * xopt[i] + tempb * d[i] - vlag[NPT + i];
                s[i] = tau * rd2_(bmat, knew - 1, i) + alpha * temp;
            }
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                sum = 0.0;
#pragma unroll
                for (int j = 0; j < N; ++j) sum = sum + xpt[k][j] * hw[j];
                temp = (tau * hw[N + k] - alpha * vlag[k]) * sum;
#pragma unroll
                for (int i = 0; i < N; ++i) s[i] = s[i] + temp * xpt[k][i];
            }
            ss = 0.0;
            ds = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                ss = ss + s[i] * s[i];
                ds = ds + d[i] * s[i];
            }
            ssden = dd * ss - ds * ds;
            if (!(ssden >= 1.0e-8 * dd * ss)) break;
        }
#pragma unroll
        for (int k = 0; k < NDIM; ++k) {
            w[k] = 0.0;
#pragma unroll
            for (int j = 0; j < 5; ++j) w[k] = w[k] + wvec[k][j] * par[j];
        }
        wr_(vlag, kopt - 1, rd_(vlag, kopt - 1) + 1.0);
    }

    // ------------------------------------------------------------------------- UPDATE
    // Shift interpolation point knew: update BMAT, ZMAT, IDZ (vlag, beta from the step).
    GPD_HDX void update(int &idz, double beta, int knew) {
        double wk[NDIM];
        int jl = 1;  // 1-based column index into zmat
#pragma unroll
        for (int j = 2; j <= NPTM; ++j) {
            if (j == idz) {
                jl = idz;
            } else if (rd2_(zmat, knew - 1, j - 1) != 0.0) {
                const double zl = rdc_(zmat, knew - 1, jl - 1);  // zmat[knew][jl]
                const double zj = rd2_(zmat, knew - 1, j - 1);
                double temp = sqrt(zl * zl + zj * zj);
                const double ta = zl / temp, tb = zj / temp;
#pragma unroll
                for (int i = 0; i < NPT; ++i) {
                    const double zil = rdc_(zmat, i, jl - 1);
                    temp = ta * zil + tb * zmat[i][j - 1];
                    zmat[i][j - 1] = ta * zmat[i][j - 1] - tb * zil;
                    wrc_(zmat, i, jl - 1, temp);
                }
                wr2_(zmat, knew - 1, j - 1, 0.0);
            }
        }
        double tempa = rd2_(zmat, knew - 1, 0);
        if (idz >= 2) tempa = -tempa;
        double tempb = 0.0;
        if (jl > 1) tempb = rdc_(zmat, knew - 1, jl - 1);
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            wk[i] = tempa * zmat[i][0];
            if (jl > 1) wk[i] = wk[i] + tempb * rdc_(zmat, i, jl - 1);
        }
        const double alpha = rd_(wk, knew - 1);  // only wk[0..NPT) are set; knew <= NPT
        const double tau = rd_(vlag, knew - 1);
        const double tausq = tau * tau;
        const double denom = alpha * beta + tausq;
        wr_(vlag, knew - 1, tau - 1.0);
        int iflag = 0;
        if (jl == 1) {
            const double temp = sqrt(fabs(denom));
            tempb = tempa / temp;
            tempa = tau / temp;
#pragma unroll
            for (int i = 0; i < NPT; ++i) zmat[i][0] = tempa * zmat[i][0] - tempb * vlag[i];
            if (idz == 1 && temp < 0.0) idz = 2;
            if (idz >= 2 && temp >= 0.0) iflag = 1;
        } else {
            int ja = 1;
            if (beta >= 0.0) ja = jl;
            const int jb = jl + 1 - ja;
            double temp = rdc_(zmat, knew - 1, jb - 1) / denom;
            tempa = temp * beta;
            tempb = temp * tau;
            temp = rdc_(zmat, knew - 1, ja - 1);
            const double scala = 1.0 / sqrt(fabs(beta) * temp * temp + tausq);
            const double scalb = scala * sqrt(fabs(denom));
#pragma unroll
            for (int i = 0; i < NPT; ++i) {
                const double za = rdc_(zmat, i, ja - 1), zb = rdc_(zmat, i, jb - 1);
                wrc_(zmat, i, ja - 1, scala * (tau * za - temp * vlag[i]));
                wrc_(zmat, i, jb - 1, scalb * (zb - tempa * wk[i] - tempb * vlag[i]));
            }
            if (denom <= 0.0) {
                if (beta < 0.0) idz = idz + 1;
                if (beta >= 0.0) iflag = 1;
            }
        }
        if (iflag == 1) {
            idz = idz - 1;
#pragma unroll
            for (int i = 0; i < NPT; ++i) {
                const double temp = zmat[i][0];
                zmat[i][0] = rdc_(zmat, i, idz - 1);
                wrc_(zmat, i, idz - 1, temp);
            }
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const int jp = NPT + j;  // 0-based row of BMAT / entry of VLAG, W
            wk[jp] = rd2_(bmat, knew - 1, j);
            const double ta = (alpha * vlag[jp] - tau * wk[jp]) / denom;
            const double tb = (-beta * wk[jp] - tau * vlag[jp]) / denom;
#pragma unroll
            for (int i = 0; i <= jp; ++i) {
                bmat[i][j] = bmat[i][j] + ta * vlag[i] + tb * wk[i];
                if (i >= NPT) bmat[jp][i - NPT] = bmat[i][j];
            }
        }
    }

    // ------------------------------------------------------------------------- NEWUOB
    // Minimise f from x (in/out).  Returns the number of evaluations; *fx = f(x).
    template <class F>
    GPD_HDN int run(double (&x)[N], double rhobeg, double rhoend, int maxfun, F &fun,
                   double &fx) {
        GPD_NW_T0(tinit_);
        const int nftest = maxfun > 1 ? maxfun : 1;
        const int np = N + 1;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            xbase[j] = x[j];
#pragma unroll
            for (int k = 0; k < NPT; ++k) xpt[k][j] = 0.0;
#pragma unroll
            for (int i = 0; i < NDIM; ++i) bmat[i][j] = 0.0;
        }
#pragma unroll
        for (int ih = 0; ih < NH; ++ih) hq[ih] = 0.0;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            pq[k] = 0.0;
#pragma unroll
            for (int j = 0; j < NPTM; ++j) zmat[k][j] = 0.0;
        }
        double rhosq = rhobeg * rhobeg;
        const double recip = 1.0 / rhosq;
        const double reciq = sqrt(0.5) / rhosq;
        double f = 0.0, fbeg = 0.0, fopt = 0.0;
        int kopt = 1;
        // NPT ≤ 2N + 1: the initial points x_nf = xbase ± rhobeg·e_j depend on no f value, so an
        // objective with has_multi evaluates all NPT of them at once (the same points, each
        // x_j = xpt_j + xbase_j as the loop below forms it, the same values)
        double fpre[NPT];
        bool pre = false;
        if constexpr (has_multi<F>::value && NPT <= 2 * N + 1) {
            if (nftest >= NPT) {
                double pts[NPT][2];
#pragma unroll
                for (int nf = 1; nf <= NPT; ++nf) {
                    const int nfm = nf - 1;
#pragma unroll
                    for (int j = 0; j < N; ++j) {
                        double v = 0.0;
                        if (nfm >= 1 && nfm <= N && j == nfm - 1) v = rhobeg;
                        if (nfm > N && j == nfm - N - 1) v = -rhobeg;
                        pts[nf - 1][j] = v + xbase[j];
                    }
                }
                fun.template multi<NPT>(pts, fpre);
                pre = true;
            }
        }

        // ---------------------------------------- initial interpolation set (NPT points)
        for (int nf = 1; nf <= NPT; ++nf) {
            const int nfm = nf - 1, nfmm = nf - 1 - N;
            int ipt = 0, jpt = 0;
            double xipt = 0.0, xjpt = 0.0;
            if (nfm <= 2 * N) {
                if (nfm >= 1 && nfm <= N) {
                    wr2_(xpt, nf - 1, nfm - 1, rhobeg);
                } else if (nfm > N) {
#pragma unroll
                    for (int j = 0; j < N; ++j)
                        if (j == nfmm - 1) wr2_(xpt, nf - 1, j, -rhobeg);
                }
            } else {
                int itemp = (nfmm - 1) / N;
                jpt = nfm - itemp * N - N;
                ipt = jpt + itemp;
                if (ipt > N) {
                    itemp = jpt;
                    jpt = ipt - N;
                    ipt = itemp;
                }
                xipt = rhobeg;
                if (rd_(fval, ipt + np - 1) < rd_(fval, ipt)) xipt = -xipt;
                xjpt = rhobeg;
                if (rd_(fval, jpt + np - 1) < rd_(fval, jpt)) xjpt = -xjpt;
#pragma unroll
                for (int j = 0; j < N; ++j) {
                    if (j == ipt - 1) wr2_(xpt, nf - 1, j, xipt);
                    if (j == jpt - 1) wr2_(xpt, nf - 1, j, xjpt);
                }
            }
            double xe[N];
#pragma unroll
            for (int j = 0; j < N; ++j) xe[j] = rd2_(xpt, nf - 1, j) + xbase[j];
#pragma unroll
            for (int j = 0; j < N; ++j) x[j] = xe[j];
            if (nf > nftest) {  // maxfun < NPT: stop during initialisation
                fx = f;
                finish(x, fopt, f);
                fx = f;
                return nf - 1;
            }
            f = pre ? fpre[nf - 1] : fun(x);
            wr_(fval, nf - 1, f);
            if (nf == 1) {
                fbeg = f;
                fopt = f;
                kopt = 1;
            } else if (f < fopt) {
                fopt = f;
                kopt = nf;
            }
            if (nfm <= 2 * N) {
                if (nfm >= 1 && nfm <= N) {
                    wr_(gq, nfm - 1, (f - fbeg) / rhobeg);
                    if (NPT < nf + N) {
#pragma unroll
                        for (int j = 0; j < N; ++j)
                            if (j == nfm - 1) {
                                bmat[0][j] = -1.0 / rhobeg;
                                wr2_(bmat, nf - 1, j, 1.0 / rhobeg);
                                wr2_(bmat, NPT + nfm - 1, j, -0.5 * rhosq);
                            }
                    }
                } else if (nfm > N) {
#pragma unroll
                    for (int j = 0; j < N; ++j) {
                        if (j == nfmm - 1) {
                            wr2_(bmat, nf - N - 1, j, 0.5 / rhobeg);
                            wr2_(bmat, nf - 1, j, -0.5 / rhobeg);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < NPTM; ++j) {
                        if (j == nfmm - 1) {
                            zmat[0][j] = -reciq - reciq;
                            wr2_(zmat, nf - N - 1, j, reciq);
                            wr2_(zmat, nf - 1, j, reciq);
                        }
                    }
                    const int ih = (nfmm * (nfmm + 1)) / 2;
                    const double temp = (fbeg - f) / rhobeg;
                    const double g = rd_(gq, nfmm - 1);
                    wr_(hq, ih - 1, (g - temp) / rhobeg);
                    wr_(gq, nfmm - 1, 0.5 * (g + temp));
                }
            } else {
                const int ih = (ipt * (ipt - 1)) / 2 + jpt;
                if (xipt < 0.0) ipt = ipt + N;
                if (xjpt < 0.0) jpt = jpt + N;
#pragma unroll
                for (int j = 0; j < NPTM; ++j) {
                    if (j == nfmm - 1) {
                        zmat[0][j] = recip;
                        wr2_(zmat, nf - 1, j, recip);
                        wr2_(zmat, ipt, j, -recip);
                        wr2_(zmat, jpt, j, -recip);
                    }
                }
                wr_(hq, ih - 1, (fbeg - rd_(fval, ipt) - rd_(fval, jpt) + f) / (xipt * xjpt));
            }
        }
        int nf = NPT;
        GPD_NW_T1(tinit_, 4);

        // ---------------------------------------- iterations
        // NEWUOB's labels as explicit states, walked so that a wave's fits meet at the objective:
        // each trip of the outer loop is one evaluation (L290) for every fit still running.
        // Within a trip a fit first walks L460 / L490 / L100 (trust-region step, geometry point,
        // ρ reduction — in that order within one pass of the inner loop, so the common paths
        // take one pass) until it stands at L120 (a step to evaluate), at L290 (L490's final
        // evaluation) or is done; then the L120 block (VLAG, BETA, BIGLAG/BIGDEN) and the
        // evaluation run once for all of them together.  The same operations in the same order
        // as the published goto structure — only the points where diverged fits wait for each
        // other change (before r5 the fits of a wave reached the objective in different passes
        // of the compiler's structurised loop, ~3 objective executions per evaluation).
        double rho = rhobeg, delta = rho;
        int idz = 1;
        double diffa = 0.0, diffb = 0.0, diffc = 0.0, ratio = 0.0, crvmin = 0.0;
        double dnorm = 0.0, dsq = 0.0, dstep = 0.0, alpha = 0.0, beta = 0.0, vquad = 0.0;
        double diff = 0.0;
        int itest = 0, knew = 0, nfsav;
        double xoptsq = 0.0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            xopt[i] = rd2_(xpt, kopt - 1, i);
            xoptsq = xoptsq + xopt[i] * xopt[i];
        }
        enum { S100, S120, S290, S460, S490, SDONE };
        int st = S100;
        nfsav = nf;  // L90
        for (;;) {
            while (st == S460 || st == S490 || st == S100) {
                if (st == S460) {  // L460: the point farthest from xopt, if far enough
                    double distsq = 4.0 * delta * delta;
#pragma unroll
                    for (int k = 0; k < NPT; ++k) {
                        double sum = 0.0;
#pragma unroll
                        for (int j = 0; j < N; ++j) sum = sum + (xpt[k][j] - xopt[j]) * (xpt[k][j] - xopt[j]);
                        if (sum > distsq) {
                            knew = k + 1;
                            distsq = sum;
                        }
                    }
                    if (knew > 0) {
                        dstep = fmax(fmin(0.1 * sqrt(distsq), 0.5 * delta), rho);
                        dsq = dstep * dstep;
                        st = S120;
                    } else if (ratio > 0.0) {
                        st = S100;
                    } else if (fmax(delta, dnorm) > rho) {
                        st = S100;
                    } else {
                        st = S490;
                    }
                }
                if (st == S490) {  // L490: reduce ρ, or stop
                    if (rho > rhoend) {
                        delta = 0.5 * rho;
                        ratio = rho / rhoend;
                        if (ratio <= 16.0) {
                            rho = rhoend;
                        } else if (ratio <= 250.0) {
                            rho = sqrt(ratio) * rhoend;
                        } else {
                            rho = 0.1 * rho;
                        }
                        delta = fmax(delta, rho);
                        nfsav = nf;  // L90
                        st = S100;
                    } else {
                        st = knew == -1 ? S290 : SDONE;
                    }
                }
                if (st == S100) {  // L100: trust-region step
                    knew = 0;
                    {
                        GPD_NW_T0(tt_);
                        trsapp(delta, d, crvmin);
                        GPD_NW_T1(tt_, 0);
                    }
                    dsq = 0.0;
#pragma unroll
                    for (int i = 0; i < N; ++i) dsq = dsq + d[i] * d[i];
                    dnorm = fmin(delta, sqrt(dsq));
                    if (dnorm < 0.5 * rho) {
                        knew = -1;
                        delta = 0.1 * delta;
                        ratio = -1.0;
                        if (delta <= 1.5 * rho) delta = rho;
                        if (nf <= nfsav + 2) {
                            st = S460;
                        } else {
                            const double temp = 0.125 * crvmin * rho * rho;
                            st = temp <= fmax(fmax(diffa, diffb), diffc) ? S460 : S490;
                        }
                    } else {
                        st = S120;
                    }
                }
            }
            if (st == SDONE) break;
            if (st == S120) {  // L120
                if (dsq <= 1.0e-3 * xoptsq) shift_base(xoptsq, idz);
                if (knew > 0) {
                    GPD_NW_T0(tt_);
                    biglag(idz, knew, dstep, alpha);
                    GPD_NW_T1(tt_, 1);
                }
                // VLAG and BETA for the current D; W(1..NPT) = Wcheck
                {
                    GPD_NW_T0(tvl_);
#pragma unroll
                    for (int k = 0; k < NPT; ++k) {
                        double suma = 0.0, sumb = 0.0, sum = 0.0;
#pragma unroll
                        for (int j = 0; j < N; ++j) {
                            suma = suma + xpt[k][j] * d[j];
                            sumb = sumb + xpt[k][j] * xopt[j];
                            sum = sum + bmat[k][j] * d[j];
                        }
                        w[k] = suma * (0.5 * suma + sumb);
                        vlag[k] = sum;
                    }
                    beta = 0.0;
#pragma unroll
                    for (int k = 0; k < NPTM; ++k) {
                        double sum = 0.0;
#pragma unroll
                        for (int i = 0; i < NPT; ++i) sum = sum + zmat[i][k] * w[i];
                        if (k + 1 < idz) {
                            beta = beta + sum * sum;
                            sum = -sum;
                        } else {
                            beta = beta - sum * sum;
                        }
#pragma unroll
                        for (int i = 0; i < NPT; ++i) vlag[i] = vlag[i] + sum * zmat[i][k];
                    }
                    double bsum = 0.0, dx = 0.0;
#pragma unroll
                    for (int j = 0; j < N; ++j) {
                        double sum = 0.0;
#pragma unroll
                        for (int i = 0; i < NPT; ++i) sum = sum + w[i] * bmat[i][j];
                        bsum = bsum + sum * d[j];
                        const int jp = NPT + j;
#pragma unroll
                        for (int k = 0; k < N; ++k) sum = sum + bmat[jp][k] * d[k];
                        vlag[jp] = sum;
                        bsum = bsum + sum * d[j];
                        dx = dx + d[j] * xopt[j];
                    }
                    beta = dx * dx + dsq * (xoptsq + dx + dx + 0.5 * dsq) + beta - bsum;
                    wr_(vlag, kopt - 1, rd_(vlag, kopt - 1) + 1.0);
                    GPD_NW_T1(tvl_, 5);
                }
                if (knew > 0) {
                    const double vk = rd_(vlag, knew - 1);
                    const double temp = 1.0 + alpha * beta / (vk * vk);
                    if (fabs(temp) <= 0.8) {
                        GPD_NW_T0(tt_);
                        bigden(idz, kopt, knew, beta);
                        GPD_NW_T1(tt_, 2);
                    }
                }
            }
            // L290: evaluate
#pragma unroll
            for (int i = 0; i < N; ++i) {
                xnew[i] = xopt[i] + d[i];
                x[i] = xbase[i] + xnew[i];
            }
            nf = nf + 1;
            if (nf > nftest) {
                nf = nf - 1;
                break;  // L530
            }
            f = fun(x);
            if (knew == -1) break;  // L530
            {
                vquad = 0.0;
                int ih = 0;
#pragma unroll
                for (int j = 0; j < N; ++j) {
                    vquad = vquad + d[j] * gq[j];
#pragma unroll
                    for (int i = 0; i <= j; ++i) {
                        double temp = d[i] * xnew[j] + d[j] * xopt[i];
                        if (i == j) temp = 0.5 * temp;
                        vquad = vquad + temp * hq[ih];
                        ++ih;
                    }
                }
#pragma unroll
                for (int k = 0; k < NPT; ++k) vquad = vquad + pq[k] * w[k];
            }
            diff = f - fopt - vquad;
            diffc = diffb;
            diffb = diffa;
            diffa = fabs(diff);
            if (dnorm > rho) nfsav = nf;
            {
                const double fsave = fopt;
                if (f < fopt) {
                    fopt = f;
                    xoptsq = 0.0;
#pragma unroll
                    for (int i = 0; i < N; ++i) {
                        xopt[i] = xnew[i];
                        xoptsq = xoptsq + xopt[i] * xopt[i];
                    }
                }
                const int ksave = knew;
                if (knew <= 0) {
                    if (vquad >= 0.0) break;  // L530: trust-region step failed to reduce Q
                    ratio = (f - fsave) / vquad;
                    if (ratio <= 0.1) {
                        delta = 0.5 * dnorm;
                    } else if (ratio <= 0.7) {
                        delta = fmax(0.5 * delta, dnorm);
                    } else {
                        delta = fmax(0.5 * delta, dnorm + dnorm);
                    }
                    if (delta <= 1.5 * rho) delta = rho;
                    // point to drop
                    double rs = fmax(0.1 * delta, rho);
                    rs = rs * rs;
                    int ktemp = 0;
                    double detrat = 0.0;
                    if (f >= fsave) {
                        ktemp = kopt;
                        detrat = 1.0;
                    }
#pragma unroll
                    for (int k = 0; k < NPT; ++k) {
                        double hdiag = 0.0;
#pragma unroll
                        for (int j = 0; j < NPTM; ++j) {
                            double temp = 1.0;
                            if (j + 1 < idz) temp = -1.0;
                            hdiag = hdiag + temp * zmat[k][j] * zmat[k][j];
                        }
                        double temp = fabs(beta * hdiag + vlag[k] * vlag[k]);
                        double distsq = 0.0;
#pragma unroll
                        for (int j = 0; j < N; ++j)
                            distsq = distsq + (xpt[k][j] - xopt[j]) * (xpt[k][j] - xopt[j]);
                        if (distsq > rs) {
                            const double r = distsq / rs;
                            temp = temp * (r * r * r);
                        }
                        if (temp > detrat && k + 1 != ktemp) {
                            detrat = temp;
                            knew = k + 1;
                        }
                    }
                    if (knew == 0) {  // L460 with knew = 0
                        st = S460;
                        continue;
                    }
                }
                // L410: move point knew to xnew and update the model
                {
                    GPD_NW_T0(tt_);
                    update(idz, beta, knew);
                    GPD_NW_T1(tt_, 3);
                }
                wr_(fval, knew - 1, f);
                {
                    GPD_NW_T0(tmu_);
                    const double pqk = rd_(pq, knew - 1);
                    int ih = 0;
#pragma unroll
                    for (int i = 0; i < N; ++i) {
                        const double temp = pqk * rd2_(xpt, knew - 1, i);
#pragma unroll
                        for (int j = 0; j <= i; ++j) {
                            hq[ih] = hq[ih] + temp * rd2_(xpt, knew - 1, j);
                            ++ih;
                        }
                    }
                    wr_(pq, knew - 1, 0.0);
#pragma unroll
                    for (int j = 0; j < NPTM; ++j) {
                        double temp = diff * rd2_(zmat, knew - 1, j);
                        if (j + 1 < idz) temp = -temp;
#pragma unroll
                        for (int k = 0; k < NPT; ++k) pq[k] = pq[k] + temp * zmat[k][j];
                    }
                    double gqsq = 0.0;
#pragma unroll
                    for (int i = 0; i < N; ++i) {
                        gq[i] = gq[i] + diff * rd2_(bmat, knew - 1, i);
                        gqsq = gqsq + gq[i] * gq[i];
                        wr2_(xpt, knew - 1, i, xnew[i]);
                    }
                    if (ksave == 0 && delta == rho) {
                        if (fabs(ratio) > 1.0e-2) {
                            itest = 0;
                        } else {
                            const double fk = rd_(fval, kopt - 1);
#pragma unroll
                            for (int k = 0; k < NPT; ++k) vlag[k] = fval[k] - fk;
                            double gisq = 0.0;
#pragma unroll
                            for (int i = 0; i < N; ++i) {
                                double sum = 0.0;
#pragma unroll
                                for (int k = 0; k < NPT; ++k) sum = sum + bmat[k][i] * vlag[k];
                                gisq = gisq + sum * sum;
                                w[i] = sum;
                            }
                            itest = itest + 1;
                            if (gqsq < 1.0e2 * gisq) itest = 0;
                            if (itest >= 3) {
#pragma unroll
                                for (int i = 0; i < N; ++i) gq[i] = w[i];
#pragma unroll
                                for (int ih2 = 0; ih2 < NH; ++ih2) hq[ih2] = 0.0;
                                double wz[NPTM];
#pragma unroll
                                for (int j = 0; j < NPTM; ++j) {
                                    wz[j] = 0.0;
#pragma unroll
                                    for (int k = 0; k < NPT; ++k) wz[j] = wz[j] + vlag[k] * zmat[k][j];
                                    if (j + 1 < idz) wz[j] = -wz[j];
                                }
#pragma unroll
                                for (int j = 0; j < NPTM; ++j) w[j] = wz[j];
#pragma unroll
                                for (int k = 0; k < NPT; ++k) {
                                    pq[k] = 0.0;
#pragma unroll
                                    for (int j = 0; j < NPTM; ++j) pq[k] = pq[k] + zmat[k][j] * w[j];
                                }
                                itest = 0;
                            }
                        }
                    }
                    GPD_NW_T1(tmu_, 6);
                }
                if (f < fsave) kopt = knew;
                if (f <= fsave + 0.1 * vquad) {
                    st = S100;
                    continue;
                }
                if (ksave > 0) {
                    st = S100;
                    continue;
                }
            }
            knew = 0;
            st = S460;
        }
        // L530
        finish(x, fopt, f);
        fx = f;
        return nf;
    }

    GPD_HD void finish(double (&x)[N], double fopt, double &f) const {
        if (fopt <= f) {
#pragma unroll
            for (int i = 0; i < N; ++i) x[i] = xbase[i] + xopt[i];
            f = fopt;
        }
    }

    // Move XBASE to XBASE+XOPT (NEWUOB label 120 block).
    GPD_HDX void shift_base(double &xoptsq, int idz) {
        const double tempq = 0.25 * xoptsq;
        double wt[NPT], v[N], wi[N];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            double sum = 0.0;
#pragma unroll
            for (int i = 0; i < N; ++i) sum = sum + xpt[k][i] * xopt[i];
            const double temp = pq[k] * sum;
            sum = sum - 0.5 * xoptsq;
            wt[k] = sum;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                gq[i] = gq[i] + temp * xpt[k][i];
                xpt[k][i] = xpt[k][i] - 0.5 * xopt[i];
                v[i] = bmat[k][i];
                wi[i] = sum * xpt[k][i] + tempq * xopt[i];
                const int ip = NPT + i;
#pragma unroll
                for (int j = 0; j <= i; ++j) bmat[ip][j] = bmat[ip][j] + v[i] * wi[j] + wi[i] * v[j];
            }
        }
#pragma unroll
        for (int k = 0; k < NPTM; ++k) {
            double sumz = 0.0, wz[NPT];
#pragma unroll
            for (int i = 0; i < NPT; ++i) {
                sumz = sumz + zmat[i][k];
                wz[i] = wt[i] * zmat[i][k];
            }
#pragma unroll
            for (int j = 0; j < N; ++j) {
                double sum = tempq * sumz * xopt[j];
#pragma unroll
                for (int i = 0; i < NPT; ++i) sum = sum + wz[i] * xpt[i][j];
                v[j] = sum;
                if (k + 1 < idz) sum = -sum;
#pragma unroll
                for (int i = 0; i < NPT; ++i) bmat[i][j] = bmat[i][j] + sum * zmat[i][k];
            }
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int ip = i + NPT;
                double temp = v[i];
                if (k + 1 < idz) temp = -temp;
#pragma unroll
                for (int j = 0; j <= i; ++j) bmat[ip][j] = bmat[ip][j] + temp * v[j];
            }
        }
        int ih = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            wi[j] = 0.0;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                wi[j] = wi[j] + pq[k] * xpt[k][j];
                xpt[k][j] = xpt[k][j] - 0.5 * xopt[j];
            }
#pragma unroll
            for (int i = 0; i <= j; ++i) {
                if (i < j) gq[j] = gq[j] + hq[ih] * xopt[i];
                gq[i] = gq[i] + hq[ih] * xopt[j];
                hq[ih] = hq[ih] + wi[i] * xopt[j] + xopt[i] * wi[j];
                bmat[NPT + i][j] = bmat[NPT + j][i];
                ++ih;
            }
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            xbase[j] = xbase[j] + xopt[j];
            xopt[j] = 0.0;
        }
        xoptsq = 0.0;
    }
};

}  // namespace gpd
