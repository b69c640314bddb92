/*
 * Plain C host of the drop-in boundary: one GRAVITY-like exposure (32 diodes + 8 fibre-coupler
 * columns in idx() order, Julia's column-major Matrix{ComplexF64} layout) through ONE
 * gpd_demodulateall call — demodulateall (src/Modulation.jl:344-435) as the Julia wrapper of
 * INTEGRATION.md calls it through `ccall`: the exposure in, the 32 records and the N×40 output
 * (demodulated diodes, FC columns as given) back.
 *
 * The synthetic series follow the reference's model d = p·a·exp(j·b·sin(ωt + ϕ)) + noise
 * (src/Modulation.jl:57-64, 122-148) with ω = M_2PI = 6.283185 (src/Modulation.jl:11) and 500 Hz
 * timestamps.  Prints one line per diode and exits non-zero if a fitted b strays from the truth
 * by more than the noise allows, or on any library error.
 *
 *   gcc -O2 -Iinclude examples/demod_exposure.c -Lgppupildemodulation.jl_amd -lgpdemod \
 *       -Wl,-rpath,$PWD/gppupildemodulation.jl_amd -lm -o examples/demod_exposure
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "gpdemod.h"

enum { NDIODE = 32, NFC = 8, NCOL = NDIODE + NFC };

static uint64_t rng_state = 0x243f6a8885a308d3ull;
static double urand(void) { /* splitmix64 → U[0,1) */
    uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}
static double nrand(void) { return sqrt(-2.0 * log1p(-urand())) * cos(6.283185307179586 * urand()); }

int main(int argc, char **argv) {
    const int64_t N = argc > 1 ? atoll(argv[1]) : 100000;
    const double omega = 6.283185, dt = 0.002, sigma = 0.1;
    if (gpd_version() != GPD_ABI_VERSION) {
        fprintf(stderr, "ABI version mismatch\n");
        return 2;
    }
    if (gpd_device_count() < 1) {
        fprintf(stderr, "no HIP device\n");
        return 3;
    }
    double *t = malloc(N * sizeof *t);
    gpd_c64 *data = malloc((size_t)N * NCOL * sizeof *data); /* column k at data + k·N */
    gpd_c64 *out = malloc((size_t)N * NCOL * sizeof *out); /* output, N×40 like data */
    double bt[NDIODE], pt[NDIODE];
    gpd_param par[NDIODE];
    if (!t || !data || !out) return 4;
    for (int64_t i = 0; i < N; ++i) t[i] = (double)i * dt;
    for (int g = 0; g < NFC; ++g) { /* FC column: a slow random-walk phase, |fc| = 1.3 */
        double ph = 6.283185307179586 * urand();
        for (int64_t i = 0; i < N; ++i) {
            ph += 1e-3 * nrand();
            data[(int64_t)(NDIODE + g) * N + i] = (gpd_c64){1.3 * cos(ph), 1.3 * sin(ph)};
        }
    }
    for (int k = 0; k < NDIODE; ++k) {
        const int g = k / 4; /* the 4 diodes of one (telescope, side) share its FC column:
                                idx(side, telescope, FC) − 1 = 32 + k ÷ 4 */
        bt[k] = 0.3 + 2.2 * urand();
        pt[k] = -3.141592653589793 + 6.283185307179586 * urand();
        const double amp = 0.5 + urand(), arg = 6.283185307179586 * urand();
        for (int64_t i = 0; i < N; ++i) {
            const gpd_c64 f = data[(int64_t)(NDIODE + g) * N + i];
            const double r = hypot(f.re, f.im), pr = f.re / r, pi = f.im / r;
            const double beta = bt[k] * sin(omega * t[i] + pt[k]) + arg;
            const double mr = amp * cos(beta), mi = amp * sin(beta);
            data[(int64_t)k * N + i] = (gpd_c64){pr * mr - pi * mi + sigma * nrand() / sqrt(2.0),
                                                 pr * mi + pi * mr + sigma * nrand() / sqrt(2.0)};
        }
    }
    char err[512];
    /* (output, param, likelihood) = demodulateall(t, data; recenter=true) */
    const int rc = gpd_demodulateall(N, t, data, N, NULL, NULL, GPD_RECENTER, 60, par, out, N, 1,
                                     err, sizeof err);
    if (rc != GPD_OK) {
        fprintf(stderr, "gpd_demodulateall: %s: %s\n", gpd_strerror(rc), err);
        return 5;
    }
    int bad = 0;
    for (int64_t i = 0; i < (int64_t)NFC * N; ++i) { /* the FC columns pass through */
        const gpd_c64 a = out[(int64_t)NDIODE * N + i], b = data[(int64_t)NDIODE * N + i];
        if (a.re != b.re || a.im != b.im) {
            fprintf(stderr, "FC column sample %lld differs in the output\n", (long long)i);
            return 6;
        }
    }
    for (int k = 0; k < NDIODE; ++k) {
        const double db = fabs(par[k].b - bt[k]);
        printf("diode %2d  b %.6f (truth %.6f)  phi %+.6f  |a| %.6f  chi2 %.6e  nfev %d  status 0x%x\n",
               k + 1, par[k].b, bt[k], par[k].phi, hypot(par[k].a.re, par[k].a.im), par[k].chi2,
               par[k].nfev, par[k].status);
        if (!(db < 1e-2)) ++bad;
    }
    free(t);
    free(data);
    free(out);
    gpd_release(0);
    printf("%s: %d/%d diodes recover b within 1e-2\n", bad ? "FAIL" : "ok", NDIODE - bad, NDIODE);
    return bad ? 1 : 0;
}
