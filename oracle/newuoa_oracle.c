/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, called by, or shipped with the
 * product library (gppupildemodulation.jl_amd/).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * Restatement of M.J.D. Powell's NEWUOA (DAMTP 2004/NA05, "The NEWUOA software for
 * unconstrained optimization without derivatives"): subroutines NEWUOB, TRSAPP, BIGLAG,
 * BIGDEN and UPDATE, written from the published algorithm with Fortran's 1-based indexing
 * and goto structure kept so that the arithmetic order matches the published code.
 *
 * Reference call site: src/Modulation.jl:335
 *     (status, x, χ2) = newuoa(x -> self(scratch,x), xinit, 1, 1e-3; check=false)
 * i.e. OptimPackNextGen.Powell.Newuoa.newuoa (third-party, src/Modulation.jl:2,
 * Project.toml:12, version UNPINNED: no [compat], no Manifest).  Defaults assumed:
 * npt = 2n+1, maxfun = 30n, status ignored (check=false).  PARITY UNPINNED: the Julia
 * package is absent from this container and the reference ships no fixtures.
 */
#include <math.h>
#include <stddef.h>
#include "oracle.h"
/* cos/sin of the trial angles as OptimPackNextGen (pure Julia) evaluates them: Julia Base's
 * msun-derived functions, restated once for the oracle and the device */
#include "../gppupildemodulation.jl_amd/csrc/gpd_jlmath.h"

#define ZERO 0.0
#define HALF 0.5
#define ONE 1.0
#define TENTH 0.1

/* 1-based accessors, column-major like the Fortran. */
#define XPT(k, j) xpt[((k)-1) + ((j)-1) * npt]
#define BMAT(i, j) bmat[((i)-1) + ((j)-1) * ndim]
#define ZMAT(k, j) zmat[((k)-1) + ((j)-1) * npt]
#define WVEC(k, j) wvec[((k)-1) + ((j)-1) * ndim]
#define PROD(k, j) prod[((k)-1) + ((j)-1) * ndim]

static const double TWOPI = 6.283185307179586476925286766559; /* = 8*atan(1) exactly */

/* ---------------------------------------------------------------- TRSAPP ---- */
static void trsapp(int n, int npt, const double *xopt_, const double *xpt, const double *gq_,
                   const double *hq_, const double *pq_, double delta, double *step_,
                   double *d_, double *g_, double *hd_, double *hs_, double *crvmin) {
    const double *XOPT = xopt_ - 1, *GQ = gq_ - 1, *HQ = hq_ - 1, *PQ = pq_ - 1;
    double *STEP = step_ - 1, *D = d_ - 1, *G = g_ - 1, *HD = hd_ - 1, *HS = hs_ - 1;
    int i, j, k, ih, iterc, itermax, itersw, isave, iu;
    double delsq, qred = 0, dd = 0, ds = 0, ss = 0, gg = 0, ggbeg = 0, temp, bstep = 0, dhd,
           alpha, qadd, ggsav, sg = 0, shs = 0, sgk, angtest, tempa = 0, tempb = 0, dg, dhs,
           cf, qbeg, qsav, qmin, qnew, angle, cth, sth, reduc, ratio;

    delsq = delta * delta;
    iterc = 0;
    itermax = n;
    itersw = itermax;
    for (i = 1; i <= n; ++i) D[i] = XOPT[i];
    goto L170;

L20:
    qred = ZERO;
    dd = ZERO;
    for (i = 1; i <= n; ++i) {
        STEP[i] = ZERO;
        HS[i] = ZERO;
        G[i] = GQ[i] + HD[i];
        D[i] = -G[i];
        dd = dd + D[i] * D[i];
    }
    *crvmin = ZERO;
    if (dd == ZERO) goto L160;
    ds = ZERO;
    ss = ZERO;
    gg = dd;
    ggbeg = gg;

L40:
    iterc = iterc + 1;
    temp = delsq - ss;
    bstep = temp / (ds + sqrt(ds * ds + dd * temp));
    goto L170;

L50:
    dhd = ZERO;
    for (j = 1; j <= n; ++j) dhd = dhd + D[j] * HD[j];
    alpha = bstep;
    if (dhd > ZERO) {
        temp = dhd / dd;
        if (iterc == 1) *crvmin = temp;
        *crvmin = fmin(*crvmin, temp);
        alpha = fmin(alpha, gg / dhd);
    }
    qadd = alpha * (gg - HALF * alpha * dhd);
    qred = qred + qadd;
    ggsav = gg;
    gg = ZERO;
    for (i = 1; i <= n; ++i) {
        STEP[i] = STEP[i] + alpha * D[i];
        HS[i] = HS[i] + alpha * HD[i];
        gg = gg + (G[i] + HS[i]) * (G[i] + HS[i]);
    }
    if (alpha < bstep) {
        if (qadd <= 0.01 * qred) goto L160;
        if (gg <= 1.0e-4 * ggbeg) goto L160;
        if (iterc == itermax) goto L160;
        temp = gg / ggsav;
        dd = ZERO;
        ds = ZERO;
        ss = ZERO;
        for (i = 1; i <= n; ++i) {
            D[i] = temp * D[i] - G[i] - HS[i];
            dd = dd + D[i] * D[i];
            ds = ds + D[i] * STEP[i];
            ss = ss + STEP[i] * STEP[i];
        }
        if (ds <= ZERO) goto L160;
        if (ss < delsq) goto L40;
    }
    *crvmin = ZERO;
    itersw = iterc;

L90:
    if (gg <= 1.0e-4 * ggbeg) goto L160;
    sg = ZERO;
    shs = ZERO;
    for (i = 1; i <= n; ++i) {
        sg = sg + STEP[i] * G[i];
        shs = shs + STEP[i] * HS[i];
    }
    sgk = sg + shs;
    angtest = sgk / sqrt(gg * delsq);
    if (angtest <= -0.99) goto L160;
    iterc = iterc + 1;
    temp = sqrt(delsq * gg - sgk * sgk);
    tempa = delsq / temp;
    tempb = sgk / temp;
    for (i = 1; i <= n; ++i) D[i] = tempa * (G[i] + HS[i]) - tempb * STEP[i];
    goto L170;

L120:
    dg = ZERO;
    dhd = ZERO;
    dhs = ZERO;
    for (i = 1; i <= n; ++i) {
        dg = dg + D[i] * G[i];
        dhd = dhd + HD[i] * D[i];
        dhs = dhs + HD[i] * STEP[i];
    }
    cf = HALF * (shs - dhd);
    qbeg = sg + cf;
    qsav = qbeg;
    qmin = qbeg;
    isave = 0;
    iu = 49;
    temp = TWOPI / (double)(iu + 1);
    qnew = qbeg;
    for (i = 1; i <= iu; ++i) {
        angle = (double)i * temp;
        cth = jl_cos(angle);
        sth = jl_sin(angle);
        qnew = (sg + cf * cth) * cth + (dg + dhs * cth) * sth;
        if (qnew < qmin) {
            qmin = qnew;
            isave = i;
            tempa = qsav;
        } else if (i == isave + 1) {
            tempb = qnew;
        }
        qsav = qnew;
    }
    if (isave == 0) tempa = qnew;
    if (isave == iu) tempb = qbeg;
    angle = ZERO;
    if (tempa != tempb) {
        tempa = tempa - qmin;
        tempb = tempb - qmin;
        angle = HALF * (tempa - tempb) / (tempa + tempb);
    }
    angle = temp * ((double)isave + angle);
    cth = jl_cos(angle);
    sth = jl_sin(angle);
    reduc = qbeg - (sg + cf * cth) * cth - (dg + dhs * cth) * sth;
    gg = ZERO;
    for (i = 1; i <= n; ++i) {
        STEP[i] = cth * STEP[i] + sth * D[i];
        HS[i] = cth * HS[i] + sth * HD[i];
        gg = gg + (G[i] + HS[i]) * (G[i] + HS[i]);
    }
    qred = qred + reduc;
    ratio = reduc / qred;
    if (iterc < itermax && ratio > 0.01) goto L90;
L160:
    return;

L170: /* HD = (second-derivative matrix of Q) * D */
    for (i = 1; i <= n; ++i) HD[i] = ZERO;
    for (k = 1; k <= npt; ++k) {
        temp = ZERO;
        for (j = 1; j <= n; ++j) temp = temp + XPT(k, j) * D[j];
        temp = temp * PQ[k];
        for (i = 1; i <= n; ++i) HD[i] = HD[i] + temp * XPT(k, i);
    }
    ih = 0;
    for (j = 1; j <= n; ++j) {
        for (i = 1; i <= j; ++i) {
            ih = ih + 1;
            if (i < j) HD[j] = HD[j] + HQ[ih] * D[i];
            HD[i] = HD[i] + HQ[ih] * D[j];
        }
    }
    if (iterc == 0) goto L20;
    if (iterc <= itersw) goto L50;
    goto L120;
}

/* ---------------------------------------------------------------- BIGLAG ---- */
static void biglag(int n, int npt, const double *xopt_, const double *xpt, const double *bmat,
                   const double *zmat, int idz, int ndim, int knew, double delta, double *d_,
                   double *alpha, double *hcol_, double *gc_, double *gd_, double *s_,
                   double *w_) {
    const double *XOPT = xopt_ - 1;
    double *D = d_ - 1, *HCOL = hcol_ - 1, *GC = gc_ - 1, *GD = gd_ - 1, *S = s_ - 1,
           *W = w_ - 1;
    int i, j, k, iterc, nptm, isave, iu;
    double delsq, temp, sum, dd, gg, sp, dhd, scale, tau, ss, denom, cf1, cf2, cf3, cf4, cf5,
        taubeg, taumax, tauold, tempa = 0, tempb = 0, angle, cth, sth, step;

    delsq = delta * delta;
    nptm = npt - n - 1;
    iterc = 0;
    for (k = 1; k <= npt; ++k) HCOL[k] = ZERO;
    for (j = 1; j <= nptm; ++j) {
        temp = ZMAT(knew, j);
        if (j < idz) temp = -temp;
        for (k = 1; k <= npt; ++k) HCOL[k] = HCOL[k] + temp * ZMAT(k, j);
    }
    *alpha = HCOL[knew];
    dd = ZERO;
    for (i = 1; i <= n; ++i) {
        D[i] = XPT(knew, i) - XOPT[i];
        GC[i] = BMAT(knew, i);
        GD[i] = ZERO;
        dd = dd + D[i] * D[i];
    }
    for (k = 1; k <= npt; ++k) {
        temp = ZERO;
        sum = ZERO;
        for (j = 1; j <= n; ++j) {
            temp = temp + XPT(k, j) * XOPT[j];
            sum = sum + XPT(k, j) * D[j];
        }
        temp = HCOL[k] * temp;
        sum = HCOL[k] * sum;
        for (i = 1; i <= n; ++i) {
            GC[i] = GC[i] + temp * XPT(k, i);
            GD[i] = GD[i] + sum * XPT(k, i);
        }
    }
    gg = ZERO;
    sp = ZERO;
    dhd = ZERO;
    for (i = 1; i <= n; ++i) {
        gg = gg + GC[i] * GC[i];
        sp = sp + D[i] * GC[i];
        dhd = dhd + D[i] * GD[i];
    }
    scale = delta / sqrt(dd);
    if (sp * dhd < ZERO) scale = -scale;
    temp = ZERO;
    if (sp * sp > 0.99 * dd * gg) temp = ONE;
    tau = scale * (fabs(sp) + HALF * scale * fabs(dhd));
    if (gg * delsq < 0.01 * tau * tau) temp = ONE;
    for (i = 1; i <= n; ++i) {
        D[i] = scale * D[i];
        GD[i] = scale * GD[i];
        S[i] = GC[i] + temp * GD[i];
    }

L80:
    iterc = iterc + 1;
    dd = ZERO;
    sp = ZERO;
    ss = ZERO;
    for (i = 1; i <= n; ++i) {
        dd = dd + D[i] * D[i];
        sp = sp + D[i] * S[i];
        ss = ss + S[i] * S[i];
    }
    temp = dd * ss - sp * sp;
    if (temp <= 1.0e-8 * dd * ss) return;
    denom = sqrt(temp);
    for (i = 1; i <= n; ++i) {
        S[i] = (dd * S[i] - sp * D[i]) / denom;
        W[i] = ZERO;
    }
    for (k = 1; k <= npt; ++k) {
        sum = ZERO;
        for (j = 1; j <= n; ++j) sum = sum + XPT(k, j) * S[j];
        sum = HCOL[k] * sum;
        for (i = 1; i <= n; ++i) W[i] = W[i] + sum * XPT(k, i);
    }
    cf1 = ZERO;
    cf2 = ZERO;
    cf3 = ZERO;
    cf4 = ZERO;
    cf5 = ZERO;
    for (i = 1; i <= n; ++i) {
        cf1 = cf1 + S[i] * W[i];
        cf2 = cf2 + D[i] * GC[i];
        cf3 = cf3 + S[i] * GC[i];
        cf4 = cf4 + D[i] * GD[i];
        cf5 = cf5 + S[i] * GD[i];
    }
    cf1 = HALF * cf1;
    cf4 = HALF * cf4 - cf1;
    taubeg = cf1 + cf2 + cf4;
    taumax = taubeg;
    tauold = taubeg;
    isave = 0;
    iu = 49;
    temp = TWOPI / (double)(iu + 1);
    tau = taubeg;
    for (i = 1; i <= iu; ++i) {
        angle = (double)i * temp;
        cth = jl_cos(angle);
        sth = jl_sin(angle);
        tau = cf1 + (cf2 + cf4 * cth) * cth + (cf3 + cf5 * cth) * sth;
        if (fabs(tau) > fabs(taumax)) {
            taumax = tau;
            isave = i;
            tempa = tauold;
        } else if (i == isave + 1) {
            tempb = tau;
        }
        tauold = tau;
    }
    if (isave == 0) tempa = tau;
    if (isave == iu) tempb = taubeg;
    step = ZERO;
    if (tempa != tempb) {
        tempa = tempa - taumax;
        tempb = tempb - taumax;
        step = HALF * (tempa - tempb) / (tempa + tempb);
    }
    angle = temp * ((double)isave + step);
    cth = jl_cos(angle);
    sth = jl_sin(angle);
    tau = cf1 + (cf2 + cf4 * cth) * cth + (cf3 + cf5 * cth) * sth;
    for (i = 1; i <= n; ++i) {
        D[i] = cth * D[i] + sth * S[i];
        GD[i] = cth * GD[i] + sth * W[i];
        S[i] = GC[i] + GD[i];
    }
    if (fabs(tau) <= 1.1 * fabs(taubeg)) return;
    if (iterc < n) goto L80;
}

/* ---------------------------------------------------------------- BIGDEN ---- */
static void bigden(int n, int npt, const double *xopt_, const double *xpt, const double *bmat,
                   const double *zmat, int idz, int ndim, int kopt, int knew, double *d_,
                   double *w_, double *vlag_, double *beta, double *s_, double *wvec,
                   double *prod) {
    const double *XOPT = xopt_ - 1;
    double *D = d_ - 1, *W = w_ - 1, *VLAG = vlag_ - 1, *S = s_ - 1;
    double den[10], denex[10], par[10]; /* 1-based */
    int i, j, k, jc, nw, ksav, iterc, nptm, isave, iu;
    double temp, alpha, dd, ds, ss, xoptsq, dtest, dstemp, sstemp, diff, ssden, densav, xoptd,
        xopts, tempa = 0, tempb = 0, tempc, sum, sumold, denold, denmax, angle, step, tau;
    const double QUART = 0.25, TWO = 2.0;

    nptm = npt - n - 1;
    for (k = 1; k <= npt; ++k) W[n + k] = ZERO;
    for (j = 1; j <= nptm; ++j) {
        temp = ZMAT(knew, j);
        if (j < idz) temp = -temp;
        for (k = 1; k <= npt; ++k) W[n + k] = W[n + k] + temp * ZMAT(k, j);
    }
    alpha = W[n + knew];

    dd = ZERO;
    ds = ZERO;
    ss = ZERO;
    xoptsq = ZERO;
    for (i = 1; i <= n; ++i) {
        dd = dd + D[i] * D[i];
        S[i] = XPT(knew, i) - XOPT[i];
        ds = ds + D[i] * S[i];
        ss = ss + S[i] * S[i];
        xoptsq = xoptsq + XOPT[i] * XOPT[i];
    }
    if (ds * ds > 0.99 * dd * ss) {
        ksav = knew;
        dtest = ds * ds / ss;
        for (k = 1; k <= npt; ++k) {
            if (k != kopt) {
                dstemp = ZERO;
                sstemp = ZERO;
                for (i = 1; i <= n; ++i) {
                    diff = XPT(k, i) - XOPT[i];
                    dstemp = dstemp + D[i] * diff;
                    sstemp = sstemp + diff * diff;
                }
                if (dstemp * dstemp / sstemp < dtest) {
                    ksav = k;
                    dtest = dstemp * dstemp / sstemp;
                    ds = dstemp;
                    ss = sstemp;
                }
            }
        }
        for (i = 1; i <= n; ++i) S[i] = XPT(ksav, i) - XOPT[i];
    }
    ssden = dd * ss - ds * ds;
    iterc = 0;
    densav = ZERO;

L70:
    iterc = iterc + 1;
    temp = ONE / sqrt(ssden);
    xoptd = ZERO;
    xopts = ZERO;
    for (i = 1; i <= n; ++i) {
        S[i] = temp * (dd * S[i] - ds * D[i]);
        xoptd = xoptd + XOPT[i] * D[i];
        xopts = xopts + XOPT[i] * S[i];
    }
    tempa = HALF * xoptd * xoptd;
    tempb = HALF * xopts * xopts;
    den[1] = dd * (xoptsq + HALF * dd) + tempa + tempb;
    den[2] = TWO * xoptd * dd;
    den[3] = TWO * xopts * dd;
    den[4] = tempa - tempb;
    den[5] = xoptd * xopts;
    for (i = 6; i <= 9; ++i) den[i] = ZERO;

    for (k = 1; k <= npt; ++k) {
        tempa = ZERO;
        tempb = ZERO;
        tempc = ZERO;
        for (i = 1; i <= n; ++i) {
            tempa = tempa + XPT(k, i) * D[i];
            tempb = tempb + XPT(k, i) * S[i];
            tempc = tempc + XPT(k, i) * XOPT[i];
        }
        WVEC(k, 1) = QUART * (tempa * tempa + tempb * tempb);
        WVEC(k, 2) = tempa * tempc;
        WVEC(k, 3) = tempb * tempc;
        WVEC(k, 4) = QUART * (tempa * tempa - tempb * tempb);
        WVEC(k, 5) = HALF * tempa * tempb;
    }
    for (i = 1; i <= n; ++i) {
        int ip = i + npt;
        WVEC(ip, 1) = ZERO;
        WVEC(ip, 2) = D[i];
        WVEC(ip, 3) = S[i];
        WVEC(ip, 4) = ZERO;
        WVEC(ip, 5) = ZERO;
    }

    for (jc = 1; jc <= 5; ++jc) {
        nw = npt;
        if (jc == 2 || jc == 3) nw = ndim;
        for (k = 1; k <= npt; ++k) PROD(k, jc) = ZERO;
        for (j = 1; j <= nptm; ++j) {
            sum = ZERO;
            for (k = 1; k <= npt; ++k) sum = sum + ZMAT(k, j) * WVEC(k, jc);
            if (j < idz) sum = -sum;
            for (k = 1; k <= npt; ++k) PROD(k, jc) = PROD(k, jc) + sum * ZMAT(k, j);
        }
        if (nw == ndim) {
            for (k = 1; k <= npt; ++k) {
                sum = ZERO;
                for (j = 1; j <= n; ++j) sum = sum + BMAT(k, j) * WVEC(npt + j, jc);
                PROD(k, jc) = PROD(k, jc) + sum;
            }
        }
        for (j = 1; j <= n; ++j) {
            sum = ZERO;
            for (i = 1; i <= nw; ++i) sum = sum + BMAT(i, j) * WVEC(i, jc);
            PROD(npt + j, jc) = sum;
        }
    }

    for (k = 1; k <= ndim; ++k) {
        sum = ZERO;
        for (i = 1; i <= 5; ++i) {
            par[i] = HALF * PROD(k, i) * WVEC(k, i);
            sum = sum + par[i];
        }
        den[1] = den[1] - par[1] - sum;
        tempa = PROD(k, 1) * WVEC(k, 2) + PROD(k, 2) * WVEC(k, 1);
        tempb = PROD(k, 2) * WVEC(k, 4) + PROD(k, 4) * WVEC(k, 2);
        tempc = PROD(k, 3) * WVEC(k, 5) + PROD(k, 5) * WVEC(k, 3);
        den[2] = den[2] - tempa - HALF * (tempb + tempc);
        den[6] = den[6] - HALF * (tempb - tempc);
        tempa = PROD(k, 1) * WVEC(k, 3) + PROD(k, 3) * WVEC(k, 1);
        tempb = PROD(k, 2) * WVEC(k, 5) + PROD(k, 5) * WVEC(k, 2);
        tempc = PROD(k, 3) * WVEC(k, 4) + PROD(k, 4) * WVEC(k, 3);
        den[3] = den[3] - tempa - HALF * (tempb - tempc);
        den[7] = den[7] - HALF * (tempb + tempc);
        tempa = PROD(k, 1) * WVEC(k, 4) + PROD(k, 4) * WVEC(k, 1);
        den[4] = den[4] - tempa - par[2] + par[3];
        tempa = PROD(k, 1) * WVEC(k, 5) + PROD(k, 5) * WVEC(k, 1);
        tempb = PROD(k, 2) * WVEC(k, 3) + PROD(k, 3) * WVEC(k, 2);
        den[5] = den[5] - tempa - HALF * tempb;
        den[8] = den[8] - par[4] + par[5];
        tempa = PROD(k, 4) * WVEC(k, 5) + PROD(k, 5) * WVEC(k, 4);
        den[9] = den[9] - HALF * tempa;
    }

    sum = ZERO;
    for (i = 1; i <= 5; ++i) {
        par[i] = HALF * PROD(knew, i) * PROD(knew, i);
        sum = sum + par[i];
    }
    denex[1] = alpha * den[1] + par[1] + sum;
    tempa = TWO * PROD(knew, 1) * PROD(knew, 2);
    tempb = PROD(knew, 2) * PROD(knew, 4);
    tempc = PROD(knew, 3) * PROD(knew, 5);
    denex[2] = alpha * den[2] + tempa + tempb + tempc;
    denex[6] = alpha * den[6] + tempb - tempc;
    tempa = TWO * PROD(knew, 1) * PROD(knew, 3);
    tempb = PROD(knew, 2) * PROD(knew, 5);
    tempc = PROD(knew, 3) * PROD(knew, 4);
    denex[3] = alpha * den[3] + tempa + tempb - tempc;
    denex[7] = alpha * den[7] + tempb + tempc;
    tempa = TWO * PROD(knew, 1) * PROD(knew, 4);
    denex[4] = alpha * den[4] + tempa + par[2] - par[3];
    tempa = TWO * PROD(knew, 1) * PROD(knew, 5);
    denex[5] = alpha * den[5] + tempa + PROD(knew, 2) * PROD(knew, 3);
    denex[8] = alpha * den[8] + par[4] - par[5];
    denex[9] = alpha * den[9] + PROD(knew, 4) * PROD(knew, 5);

    sum = denex[1] + denex[2] + denex[4] + denex[6] + denex[8];
    denold = sum;
    denmax = sum;
    isave = 0;
    iu = 49;
    temp = TWOPI / (double)(iu + 1);
    par[1] = ONE;
    for (i = 1; i <= iu; ++i) {
        angle = (double)i * temp;
        par[2] = jl_cos(angle);
        par[3] = jl_sin(angle);
        for (j = 4; j <= 8; j += 2) {
            par[j] = par[2] * par[j - 2] - par[3] * par[j - 1];
            par[j + 1] = par[2] * par[j - 1] + par[3] * par[j - 2];
        }
        sumold = sum;
        sum = ZERO;
        for (j = 1; j <= 9; ++j) sum = sum + denex[j] * par[j];
        if (fabs(sum) > fabs(denmax)) {
            denmax = sum;
            isave = i;
            tempa = sumold;
        } else if (i == isave + 1) {
            tempb = sum;
        }
    }
    if (isave == 0) tempa = sum;
    if (isave == iu) tempb = denold;
    step = ZERO;
    if (tempa != tempb) {
        tempa = tempa - denmax;
        tempb = tempb - denmax;
        step = HALF * (tempa - tempb) / (tempa + tempb);
    }
    angle = temp * ((double)isave + step);

    par[2] = jl_cos(angle);
    par[3] = jl_sin(angle);
    for (j = 4; j <= 8; j += 2) {
        par[j] = par[2] * par[j - 2] - par[3] * par[j - 1];
        par[j + 1] = par[2] * par[j - 1] + par[3] * par[j - 2];
    }
    *beta = ZERO;
    denmax = ZERO;
    for (j = 1; j <= 9; ++j) {
        *beta = *beta + den[j] * par[j];
        denmax = denmax + denex[j] * par[j];
    }
    for (k = 1; k <= ndim; ++k) {
        VLAG[k] = ZERO;
        for (j = 1; j <= 5; ++j) VLAG[k] = VLAG[k] + PROD(k, j) * par[j];
    }
    tau = VLAG[knew];
    dd = ZERO;
    tempa = ZERO;
    tempb = ZERO;
    for (i = 1; i <= n; ++i) {
        D[i] = par[2] * D[i] + par[3] * S[i];
        W[i] = XOPT[i] + D[i];
        dd = dd + D[i] * D[i];
        tempa = tempa + D[i] * W[i];
        tempb = tempb + W[i] * W[i];
    }
    if (iterc >= n) goto L340;
    if (iterc > 1) densav = fmax(densav, denold);
    if (fabs(denmax) <= 1.1 * fabs(densav)) goto L340;
    densav = denmax;

    for (i = 1; i <= n; ++i) {
        temp = tempa * XOPT[i] + tempb * D[i] - VLAG[npt + i];
        S[i] = tau * BMAT(knew, i) + alpha * temp;
    }
    for (k = 1; k <= npt; ++k) {
        sum = ZERO;
        for (j = 1; j <= n; ++j) sum = sum + XPT(k, j) * W[j];
        temp = (tau * W[n + k] - alpha * VLAG[k]) * sum;
        for (i = 1; i <= n; ++i) S[i] = S[i] + temp * XPT(k, i);
    }
    ss = ZERO;
    ds = ZERO;
    for (i = 1; i <= n; ++i) {
        ss = ss + S[i] * S[i];
        ds = ds + D[i] * S[i];
    }
    ssden = dd * ss - ds * ds;
    if (ssden >= 1.0e-8 * dd * ss) goto L70;

L340:
    for (k = 1; k <= ndim; ++k) {
        W[k] = ZERO;
        for (j = 1; j <= 5; ++j) W[k] = W[k] + WVEC(k, j) * par[j];
    }
    VLAG[kopt] = VLAG[kopt] + ONE;
}

/* ---------------------------------------------------------------- UPDATE ---- */
static void update(int n, int npt, double *bmat, double *zmat, int *idz, int ndim,
                   double *vlag_, double beta, int knew, double *w_) {
    double *VLAG = vlag_ - 1, *W = w_ - 1;
    int i, j, jl, ja, jb, jp, iflag, nptm;
    double temp, tempa, tempb = 0, alpha, tau, tausq, denom, scala, scalb;

    nptm = npt - n - 1;
    jl = 1;
    for (j = 2; j <= nptm; ++j) {
        if (j == *idz) {
            jl = *idz;
        } else if (ZMAT(knew, j) != ZERO) {
            temp = sqrt(ZMAT(knew, jl) * ZMAT(knew, jl) + ZMAT(knew, j) * ZMAT(knew, j));
            tempa = ZMAT(knew, jl) / temp;
            tempb = ZMAT(knew, j) / temp;
            for (i = 1; i <= npt; ++i) {
                temp = tempa * ZMAT(i, jl) + tempb * ZMAT(i, j);
                ZMAT(i, j) = tempa * ZMAT(i, j) - tempb * ZMAT(i, jl);
                ZMAT(i, jl) = temp;
            }
            ZMAT(knew, j) = ZERO;
        }
    }
    tempa = ZMAT(knew, 1);
    if (*idz >= 2) tempa = -tempa;
    if (jl > 1) tempb = ZMAT(knew, jl);
    for (i = 1; i <= npt; ++i) {
        W[i] = tempa * ZMAT(i, 1);
        if (jl > 1) W[i] = W[i] + tempb * ZMAT(i, jl);
    }
    alpha = W[knew];
    tau = VLAG[knew];
    tausq = tau * tau;
    denom = alpha * beta + tausq;
    VLAG[knew] = VLAG[knew] - ONE;

    iflag = 0;
    if (jl == 1) {
        temp = sqrt(fabs(denom));
        tempb = tempa / temp;
        tempa = tau / temp;
        for (i = 1; i <= npt; ++i) ZMAT(i, 1) = tempa * ZMAT(i, 1) - tempb * VLAG[i];
        if (*idz == 1 && temp < ZERO) *idz = 2;
        if (*idz >= 2 && temp >= ZERO) iflag = 1;
    } else {
        ja = 1;
        if (beta >= ZERO) ja = jl;
        jb = jl + 1 - ja;
        temp = ZMAT(knew, jb) / denom;
        tempa = temp * beta;
        tempb = temp * tau;
        temp = ZMAT(knew, ja);
        scala = ONE / sqrt(fabs(beta) * temp * temp + tausq);
        scalb = scala * sqrt(fabs(denom));
        for (i = 1; i <= npt; ++i) {
            ZMAT(i, ja) = scala * (tau * ZMAT(i, ja) - temp * VLAG[i]);
            ZMAT(i, jb) = scalb * (ZMAT(i, jb) - tempa * W[i] - tempb * VLAG[i]);
        }
        if (denom <= ZERO) {
            if (beta < ZERO) *idz = *idz + 1;
            if (beta >= ZERO) iflag = 1;
        }
    }
    if (iflag == 1) {
        *idz = *idz - 1;
        for (i = 1; i <= npt; ++i) {
            temp = ZMAT(i, 1);
            ZMAT(i, 1) = ZMAT(i, *idz);
            ZMAT(i, *idz) = temp;
        }
    }
    for (j = 1; j <= n; ++j) {
        jp = npt + j;
        W[jp] = BMAT(knew, j);
        tempa = (alpha * VLAG[jp] - tau * W[jp]) / denom;
        tempb = (-beta * W[jp] - tau * VLAG[jp]) / denom;
        for (i = 1; i <= jp; ++i) {
            BMAT(i, j) = BMAT(i, j) + tempa * VLAG[i] + tempb * W[i];
            if (i > npt) BMAT(jp, i - npt) = BMAT(i, j);
        }
    }
}

/* ---------------------------------------------------------------- NEWUOB ---- */
/* Returns the number of function evaluations; x is overwritten with the solution and
 * *fx with its function value. */
int oracle_newuoa(int n, int npt, double *x_, double rhobeg, double rhoend, int maxfun,
                  oracle_objfun f_eval, void *ctx, double *fx) {
    enum { NMAX = ORACLE_NEWUOA_NMAX, NPTMAX = 2 * ORACLE_NEWUOA_NMAX + 1 };
    double xbase_[NMAX], xopt_[NMAX], xnew_[NMAX], xpt[NPTMAX * NMAX], fval_[NPTMAX],
        gq_[NMAX], hq_[NMAX * (NMAX + 1) / 2], pq_[NPTMAX], bmat[(NPTMAX + NMAX) * NMAX],
        zmat[NPTMAX * NPTMAX], d_[NMAX], vlag_[NPTMAX + NMAX],
        w_[(NPTMAX + 13) * (NPTMAX + NMAX) + 3 * NMAX * (NMAX + 3) / 2];
    double *X = x_ - 1, *XBASE = xbase_ - 1, *XOPT = xopt_ - 1, *XNEW = xnew_ - 1,
           *FVAL = fval_ - 1, *GQ = gq_ - 1, *HQ = hq_ - 1, *PQ = pq_ - 1, *D = d_ - 1,
           *VLAG = vlag_ - 1, *W = w_ - 1;
    int np, nh, nptm, nftest, ndim, i, j, k, ih, nf, nfm, nfmm, itemp, ipt = 0, jpt = 0, kopt = 1,
        idz, itest, nfsav, knew, ksave, ktemp, ip, jp;
    double rhosq, recip, reciq, f = 0, fbeg = 0, fopt = 0, xipt = 0, xjpt = 0, temp, rho, delta,
        diffa, diffb, diffc = 0, xoptsq, dsq, dnorm, ratio = 0, crvmin = 0, tempq, sum, sumz,
        suma, sumb, bsum, dx, beta = 0, alpha = 0, vquad, diff = 0, fsave, detrat, hdiag,
        distsq, gqsq, gisq, dstep = 0;

    if (n < 1 || n > NMAX || npt < n + 2 || npt > ((n + 2) * (n + 1)) / 2 || npt > NPTMAX)
        return -1;
    np = n + 1;
    nh = (n * np) / 2;
    nptm = npt - np;
    nftest = maxfun > 1 ? maxfun : 1;
    ndim = npt + n;

    for (j = 1; j <= n; ++j) {
        XBASE[j] = X[j];
        for (k = 1; k <= npt; ++k) XPT(k, j) = ZERO;
        for (i = 1; i <= ndim; ++i) BMAT(i, j) = ZERO;
    }
    for (ih = 1; ih <= nh; ++ih) HQ[ih] = ZERO;
    for (k = 1; k <= npt; ++k) {
        PQ[k] = ZERO;
        for (j = 1; j <= nptm; ++j) ZMAT(k, j) = ZERO;
    }

    rhosq = rhobeg * rhobeg;
    recip = ONE / rhosq;
    reciq = sqrt(HALF) / rhosq;
    nf = 0;

L50:
    nfm = nf;
    nfmm = nf - n;
    nf = nf + 1;
    if (nfm <= 2 * n) {
        if (nfm >= 1 && nfm <= n) {
            XPT(nf, nfm) = rhobeg;
        } else if (nfm > n) {
            XPT(nf, nfmm) = -rhobeg;
        }
    } else {
        itemp = (nfmm - 1) / n;
        jpt = nfm - itemp * n - n;
        ipt = jpt + itemp;
        if (ipt > n) {
            itemp = jpt;
            jpt = ipt - n;
            ipt = itemp;
        }
        xipt = rhobeg;
        if (FVAL[ipt + np] < FVAL[ipt + 1]) xipt = -xipt;
        xjpt = rhobeg;
        if (FVAL[jpt + np] < FVAL[jpt + 1]) xjpt = -xjpt;
        XPT(nf, ipt) = xipt;
        XPT(nf, jpt) = xjpt;
    }
    for (j = 1; j <= n; ++j) X[j] = XPT(nf, j) + XBASE[j];
    goto L310;

L70:
    FVAL[nf] = f;
    if (nf == 1) {
        fbeg = f;
        fopt = f;
        kopt = 1;
    } else if (f < fopt) {
        fopt = f;
        kopt = nf;
    }
    if (nfm <= 2 * n) {
        if (nfm >= 1 && nfm <= n) {
            GQ[nfm] = (f - fbeg) / rhobeg;
            if (npt < nf + n) {
                BMAT(1, nfm) = -ONE / rhobeg;
                BMAT(nf, nfm) = ONE / rhobeg;
                BMAT(npt + nfm, nfm) = -HALF * rhosq;
            }
        } else if (nfm > n) {
            BMAT(nf - n, nfmm) = HALF / rhobeg;
            BMAT(nf, nfmm) = -HALF / rhobeg;
            ZMAT(1, nfmm) = -reciq - reciq;
            ZMAT(nf - n, nfmm) = reciq;
            ZMAT(nf, nfmm) = reciq;
            ih = (nfmm * (nfmm + 1)) / 2;
            temp = (fbeg - f) / rhobeg;
            HQ[ih] = (GQ[nfmm] - temp) / rhobeg;
            GQ[nfmm] = HALF * (GQ[nfmm] + temp);
        }
    } else {
        ih = (ipt * (ipt - 1)) / 2 + jpt;
        if (xipt < ZERO) ipt = ipt + n;
        if (xjpt < ZERO) jpt = jpt + n;
        ZMAT(1, nfmm) = recip;
        ZMAT(nf, nfmm) = recip;
        ZMAT(ipt + 1, nfmm) = -recip;
        ZMAT(jpt + 1, nfmm) = -recip;
        HQ[ih] = (fbeg - FVAL[ipt + 1] - FVAL[jpt + 1] + f) / (xipt * xjpt);
    }
    if (nf < npt) goto L50;

    rho = rhobeg;
    delta = rho;
    idz = 1;
    diffa = ZERO;
    diffb = ZERO;
    itest = 0;
    xoptsq = ZERO;
    for (i = 1; i <= n; ++i) {
        XOPT[i] = XPT(kopt, i);
        xoptsq = xoptsq + XOPT[i] * XOPT[i];
    }
L90:
    nfsav = nf;

L100:
    knew = 0;
    trsapp(n, npt, xopt_, xpt, gq_, hq_, pq_, delta, d_, &W[1], &W[np], &W[np + n],
           &W[np + 2 * n], &crvmin);
    dsq = ZERO;
    for (i = 1; i <= n; ++i) dsq = dsq + D[i] * D[i];
    dnorm = fmin(delta, sqrt(dsq));
    if (dnorm < HALF * rho) {
        knew = -1;
        delta = TENTH * delta;
        ratio = -1.0;
        if (delta <= 1.5 * rho) delta = rho;
        if (nf <= nfsav + 2) goto L460;
        temp = 0.125 * crvmin * rho * rho;
        if (temp <= fmax(fmax(diffa, diffb), diffc)) goto L460;
        goto L490;
    }

L120:
    if (dsq <= 1.0e-3 * xoptsq) {
        tempq = 0.25 * xoptsq;
        for (k = 1; k <= npt; ++k) {
            sum = ZERO;
            for (i = 1; i <= n; ++i) sum = sum + XPT(k, i) * XOPT[i];
            temp = PQ[k] * sum;
            sum = sum - HALF * xoptsq;
            W[npt + k] = sum;
            for (i = 1; i <= n; ++i) {
                GQ[i] = GQ[i] + temp * XPT(k, i);
                XPT(k, i) = XPT(k, i) - HALF * XOPT[i];
                VLAG[i] = BMAT(k, i);
                W[i] = sum * XPT(k, i) + tempq * XOPT[i];
                ip = npt + i;
                for (j = 1; j <= i; ++j) BMAT(ip, j) = BMAT(ip, j) + VLAG[i] * W[j] + W[i] * VLAG[j];
            }
        }
        for (k = 1; k <= nptm; ++k) {
            sumz = ZERO;
            for (i = 1; i <= npt; ++i) {
                sumz = sumz + ZMAT(i, k);
                W[i] = W[npt + i] * ZMAT(i, k);
            }
            for (j = 1; j <= n; ++j) {
                sum = tempq * sumz * XOPT[j];
                for (i = 1; i <= npt; ++i) sum = sum + W[i] * XPT(i, j);
                VLAG[j] = sum;
                if (k < idz) sum = -sum;
                for (i = 1; i <= npt; ++i) BMAT(i, j) = BMAT(i, j) + sum * ZMAT(i, k);
            }
            for (i = 1; i <= n; ++i) {
                ip = i + npt;
                temp = VLAG[i];
                if (k < idz) temp = -temp;
                for (j = 1; j <= i; ++j) BMAT(ip, j) = BMAT(ip, j) + temp * VLAG[j];
            }
        }
        ih = 0;
        for (j = 1; j <= n; ++j) {
            W[j] = ZERO;
            for (k = 1; k <= npt; ++k) {
                W[j] = W[j] + PQ[k] * XPT(k, j);
                XPT(k, j) = XPT(k, j) - HALF * XOPT[j];
            }
            for (i = 1; i <= j; ++i) {
                ih = ih + 1;
                if (i < j) GQ[j] = GQ[j] + HQ[ih] * XOPT[i];
                GQ[i] = GQ[i] + HQ[ih] * XOPT[j];
                HQ[ih] = HQ[ih] + W[i] * XOPT[j] + XOPT[i] * W[j];
                BMAT(npt + i, j) = BMAT(npt + j, i);
            }
        }
        for (j = 1; j <= n; ++j) {
            XBASE[j] = XBASE[j] + XOPT[j];
            XOPT[j] = ZERO;
        }
        xoptsq = ZERO;
    }

    if (knew > 0) {
        biglag(n, npt, xopt_, xpt, bmat, zmat, idz, ndim, knew, dstep, d_, &alpha, &VLAG[1],
               &VLAG[npt + 1], &W[1], &W[np], &W[np + n]);
    }

    for (k = 1; k <= npt; ++k) {
        suma = ZERO;
        sumb = ZERO;
        sum = ZERO;
        for (j = 1; j <= n; ++j) {
            suma = suma + XPT(k, j) * D[j];
            sumb = sumb + XPT(k, j) * XOPT[j];
            sum = sum + BMAT(k, j) * D[j];
        }
        W[k] = suma * (HALF * suma + sumb);
        VLAG[k] = sum;
    }
    beta = ZERO;
    for (k = 1; k <= nptm; ++k) {
        sum = ZERO;
        for (i = 1; i <= npt; ++i) sum = sum + ZMAT(i, k) * W[i];
        if (k < idz) {
            beta = beta + sum * sum;
            sum = -sum;
        } else {
            beta = beta - sum * sum;
        }
        for (i = 1; i <= npt; ++i) VLAG[i] = VLAG[i] + sum * ZMAT(i, k);
    }
    bsum = ZERO;
    dx = ZERO;
    for (j = 1; j <= n; ++j) {
        sum = ZERO;
        for (i = 1; i <= npt; ++i) sum = sum + W[i] * BMAT(i, j);
        bsum = bsum + sum * D[j];
        jp = npt + j;
        for (k = 1; k <= n; ++k) sum = sum + BMAT(jp, k) * D[k];
        VLAG[jp] = sum;
        bsum = bsum + sum * D[j];
        dx = dx + D[j] * XOPT[j];
    }
    beta = dx * dx + dsq * (xoptsq + dx + dx + HALF * dsq) + beta - bsum;
    VLAG[kopt] = VLAG[kopt] + ONE;

    if (knew > 0) {
        temp = ONE + alpha * beta / (VLAG[knew] * VLAG[knew]);
        if (fabs(temp) <= 0.8) {
            bigden(n, npt, xopt_, xpt, bmat, zmat, idz, ndim, kopt, knew, d_, &W[1], &VLAG[1],
                   &beta, xnew_, &W[ndim + 1], &W[6 * ndim + 1]);
        }
    }

L290:
    for (i = 1; i <= n; ++i) {
        XNEW[i] = XOPT[i] + D[i];
        X[i] = XBASE[i] + XNEW[i];
    }
    nf = nf + 1;
L310:
    if (nf > nftest) {
        nf = nf - 1;
        goto L530;
    }
    f = f_eval(ctx, n, x_);
    if (nf <= npt) goto L70;
    if (knew == -1) goto L530;

    vquad = ZERO;
    ih = 0;
    for (j = 1; j <= n; ++j) {
        vquad = vquad + D[j] * GQ[j];
        for (i = 1; i <= j; ++i) {
            ih = ih + 1;
            temp = D[i] * XNEW[j] + D[j] * XOPT[i];
            if (i == j) temp = HALF * temp;
            vquad = vquad + temp * HQ[ih];
        }
    }
    for (k = 1; k <= npt; ++k) vquad = vquad + PQ[k] * W[k];
    diff = f - fopt - vquad;
    diffc = diffb;
    diffb = diffa;
    diffa = fabs(diff);
    if (dnorm > rho) nfsav = nf;

    fsave = fopt;
    if (f < fopt) {
        fopt = f;
        xoptsq = ZERO;
        for (i = 1; i <= n; ++i) {
            XOPT[i] = XNEW[i];
            xoptsq = xoptsq + XOPT[i] * XOPT[i];
        }
    }
    ksave = knew;
    if (knew > 0) goto L410;

    if (vquad >= ZERO) goto L530;
    ratio = (f - fsave) / vquad;
    if (ratio <= TENTH) {
        delta = HALF * dnorm;
    } else if (ratio <= 0.7) {
        delta = fmax(HALF * delta, dnorm);
    } else {
        delta = fmax(HALF * delta, dnorm + dnorm);
    }
    if (delta <= 1.5 * rho) delta = rho;

    rhosq = fmax(TENTH * delta, rho);
    rhosq = rhosq * rhosq;
    ktemp = 0;
    detrat = ZERO;
    if (f >= fsave) {
        ktemp = kopt;
        detrat = ONE;
    }
    for (k = 1; k <= npt; ++k) {
        hdiag = ZERO;
        for (j = 1; j <= nptm; ++j) {
            temp = ONE;
            if (j < idz) temp = -ONE;
            hdiag = hdiag + temp * ZMAT(k, j) * ZMAT(k, j);
        }
        temp = fabs(beta * hdiag + VLAG[k] * VLAG[k]);
        distsq = ZERO;
        for (j = 1; j <= n; ++j) distsq = distsq + (XPT(k, j) - XOPT[j]) * (XPT(k, j) - XOPT[j]);
        if (distsq > rhosq) {
            double r = distsq / rhosq;
            temp = temp * (r * r * r);
        }
        if (temp > detrat && k != ktemp) {
            detrat = temp;
            knew = k;
        }
    }
    if (knew == 0) goto L460;

L410:
    update(n, npt, bmat, zmat, &idz, ndim, &VLAG[1], beta, knew, &W[1]);
    FVAL[knew] = f;
    ih = 0;
    for (i = 1; i <= n; ++i) {
        temp = PQ[knew] * XPT(knew, i);
        for (j = 1; j <= i; ++j) {
            ih = ih + 1;
            HQ[ih] = HQ[ih] + temp * XPT(knew, j);
        }
    }
    PQ[knew] = ZERO;
    for (j = 1; j <= nptm; ++j) {
        temp = diff * ZMAT(knew, j);
        if (j < idz) temp = -temp;
        for (k = 1; k <= npt; ++k) PQ[k] = PQ[k] + temp * ZMAT(k, j);
    }
    gqsq = ZERO;
    for (i = 1; i <= n; ++i) {
        GQ[i] = GQ[i] + diff * BMAT(knew, i);
        gqsq = gqsq + GQ[i] * GQ[i];
        XPT(knew, i) = XNEW[i];
    }
    if (ksave == 0 && delta == rho) {
        if (fabs(ratio) > 1.0e-2) {
            itest = 0;
        } else {
            for (k = 1; k <= npt; ++k) VLAG[k] = FVAL[k] - FVAL[kopt];
            gisq = ZERO;
            for (i = 1; i <= n; ++i) {
                sum = ZERO;
                for (k = 1; k <= npt; ++k) sum = sum + BMAT(k, i) * VLAG[k];
                gisq = gisq + sum * sum;
                W[i] = sum;
            }
            itest = itest + 1;
            if (gqsq < 1.0e2 * gisq) itest = 0;
            if (itest >= 3) {
                for (i = 1; i <= n; ++i) GQ[i] = W[i];
                for (ih = 1; ih <= nh; ++ih) HQ[ih] = ZERO;
                for (j = 1; j <= nptm; ++j) {
                    W[j] = ZERO;
                    for (k = 1; k <= npt; ++k) W[j] = W[j] + VLAG[k] * ZMAT(k, j);
                    if (j < idz) W[j] = -W[j];
                }
                for (k = 1; k <= npt; ++k) {
                    PQ[k] = ZERO;
                    for (j = 1; j <= nptm; ++j) PQ[k] = PQ[k] + ZMAT(k, j) * W[j];
                }
                itest = 0;
            }
        }
    }
    if (f < fsave) kopt = knew;

    if (f <= fsave + TENTH * vquad) goto L100;
    if (ksave > 0) goto L100;

    knew = 0;
L460:
    distsq = 4.0 * delta * delta;
    for (k = 1; k <= npt; ++k) {
        sum = ZERO;
        for (j = 1; j <= n; ++j) sum = sum + (XPT(k, j) - XOPT[j]) * (XPT(k, j) - XOPT[j]);
        if (sum > distsq) {
            knew = k;
            distsq = sum;
        }
    }
    if (knew > 0) {
        dstep = fmax(fmin(TENTH * sqrt(distsq), HALF * delta), rho);
        dsq = dstep * dstep;
        goto L120;
    }
    if (ratio > ZERO) goto L100;
    if (fmax(delta, dnorm) > rho) goto L100;

L490:
    if (rho > rhoend) {
        delta = HALF * rho;
        ratio = rho / rhoend;
        if (ratio <= 16.0) {
            rho = rhoend;
        } else if (ratio <= 250.0) {
            rho = sqrt(ratio) * rhoend;
        } else {
            rho = TENTH * rho;
        }
        delta = fmax(delta, rho);
        goto L90;
    }
    if (knew == -1) goto L290;
L530:
    if (fopt <= f) {
        for (i = 1; i <= n; ++i) X[i] = XBASE[i] + XOPT[i];
        f = fopt;
    }
    *fx = f;
    return nf;
}
