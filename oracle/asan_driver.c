/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  A command-line driver of the oracle's C entry points for the
 * AddressSanitizer + UndefinedBehaviorSanitizer build (`make -C oracle asan`, SURVEY.md §5
 * "optional ASan on the host oracle"): the oracle sources (and the product's libm restatement
 * gpd_jlmath.h they include) are compiled with -fsanitize=address,undefined and
 * -fno-sanitize-recover=all, so any out-of-bounds access, use after free, leak, signed overflow,
 * misaligned load or invalid shift aborts the process with a report.  A Python test cannot load a
 * sanitized .so without preloading the sanitizer runtime into the interpreter, so the test
 * (tests/test_oracle_asan.py) writes the inputs of its cases to this driver's stdin and compares
 * the results it prints with the ordinary liboracle.so's, bit for bit.
 *
 * stdin: a sequence of jobs, each an int32 job code followed by its arguments (little-endian,
 * arrays as raw element bytes); stdout: each job's results in order.  Job codes:
 *   1 fit_batch    i64 N, P, nfc; u32 flags; i32 maxfun, nthreads, has_state, has_xinit,
 *                  want_out; u64 perturb_seed; f64 omega, perturb_ulps; f64 t[N]; f64 d[2PN];
 *                  f64 fc[2 nfc N]; i32 fop[P]; [i8 state[N]]; [f64 xinit[2]]
 *                  → i32 rc, oracle_param[P] (64 B each), [f64 out[2PN]]
 *   2 chi2         i64 N; i32 offsets, has_w; f64 omega, b, phi; f64 t[N], d[2N], p[2N], [w[N]]
 *                  → f64 chi2, oracle_param
 *   3 buildstates  i64 n, n1, n2; i8 s1, s2; f64 pre, post; f64 t[n], timer1[n1], timer2[n2]
 *                  → i32 rc, i8 states[n]
 *   4 mean_var     i64 n; u32 flags; i32 fused; i8 states[n]; f64 d[2n] → f64 m5[5], w5[5]
 *   5 jl_eval      i32 fn, has_y; i64 n; f64 x[n], [y[n]] → i32 rc, f64 out[n·width]
 *   6 newuoa       i32 n, npt, maxfun; f64 rhobeg, rhoend, x0[n]  (chained Rosenbrock)
 *                  → i32 nfev, f64 x[n], f64 fx
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static void *take(size_t bytes) {
    void *p = malloc(bytes ? bytes : 1);
    if (!p) {
        fprintf(stderr, "asan_driver: out of memory\n");
        exit(3);
    }
    if (bytes && fread(p, 1, bytes, stdin) != bytes) {
        fprintf(stderr, "asan_driver: short input\n");
        exit(2);
    }
    return p;
}

#define READ(T, v)                                                   \
    T v;                                                             \
    if (fread(&v, sizeof v, 1, stdin) != 1) {                        \
        fprintf(stderr, "asan_driver: short input (" #v ")\n");      \
        exit(2);                                                     \
    }

static void put(const void *p, size_t bytes) {
    if (bytes && fwrite(p, 1, bytes, stdout) != bytes) exit(4);
}

static double rosen(void *ctx, int n, const double *x) {
    (void)ctx;
    double f = 0.0;
    for (int i = 0; i + 1 < n; ++i) {
        const double a = x[i + 1] - x[i] * x[i], b = 1.0 - x[i];
        f += 100.0 * a * a + b * b;
    }
    return f;
}

int main(void) {
    int32_t job;
    while (fread(&job, sizeof job, 1, stdin) == 1) {
        if (job == 1) {
            READ(int64_t, N);
            READ(int64_t, P);
            READ(int64_t, nfc);
            READ(uint32_t, flags);
            READ(int32_t, maxfun);
            READ(int32_t, nthreads);
            READ(int32_t, has_state);
            READ(int32_t, has_xinit);
            READ(int32_t, want_out);
            READ(uint64_t, seed);
            READ(double, omega);
            READ(double, ulps);
            double *t = take((size_t)N * 8), *d = take((size_t)2 * P * N * 8),
                   *fc = take((size_t)2 * nfc * N * 8);
            int32_t *fop = take((size_t)P * 4);
            int8_t *st = has_state ? take((size_t)N) : NULL;
            double *xi = has_xinit ? take(16) : NULL;
            oracle_param *par = calloc((size_t)P, sizeof *par);
            double *out = want_out ? calloc((size_t)2 * P * N, 8) : NULL;
            const int32_t rc = oracle_fit_batch(N, P, t, d, N, fc, N, fop, st, omega, xi, flags,
                                                maxfun, par, out, N, nthreads, seed, ulps);
            put(&rc, 4);
            put(par, (size_t)P * sizeof *par);
            if (out) put(out, (size_t)2 * P * N * 8);
            free(t), free(d), free(fc), free(fop), free(st), free(xi), free(par), free(out);
        } else if (job == 2) {
            READ(int64_t, N);
            READ(int32_t, offsets);
            READ(int32_t, has_w);
            READ(double, omega);
            READ(double, b);
            READ(double, phi);
            double *t = take((size_t)N * 8), *d = take((size_t)2 * N * 8),
                   *p = take((size_t)2 * N * 8), *w = has_w ? take((size_t)N * 8) : NULL;
            oracle_param rec;
            memset(&rec, 0, sizeof rec);
            const double v = oracle_chi2(N, t, d, w, p, omega, offsets, b, phi, &rec);
            put(&v, 8);
            put(&rec, sizeof rec);
            free(t), free(d), free(p), free(w);
        } else if (job == 3) {
            READ(int64_t, n);
            READ(int64_t, n1);
            READ(int64_t, n2);
            READ(int8_t, s1);
            READ(int8_t, s2);
            READ(double, pre);
            READ(double, post);
            double *t = take((size_t)n * 8), *t1 = take((size_t)n1 * 8), *t2 = take((size_t)n2 * 8);
            int8_t *st = calloc((size_t)(n > 0 ? n : 1), 1);
            const int32_t rc = oracle_buildstates(n, t, n1, t1, n2, t2, s1, s2, pre, post, st);
            put(&rc, 4);
            put(st, (size_t)n);
            free(t), free(t1), free(t2), free(st);
        } else if (job == 4) {
            READ(int64_t, n);
            READ(uint32_t, flags);
            READ(int32_t, fused);
            int8_t *st = take((size_t)n);
            double *d = take((size_t)2 * n * 8);
            double m5[5], w5[5];
            if (fused)
                oracle_mean_var_power_fused(n, st, d, flags, m5, w5);
            else
                oracle_mean_var_power_series(n, st, d, flags, m5, w5);
            put(m5, sizeof m5);
            put(w5, sizeof w5);
            free(st), free(d);
        } else if (job == 5) {
            READ(int32_t, fn);
            READ(int32_t, has_y);
            READ(int64_t, n);
            double *x = take((size_t)n * 8), *y = has_y ? take((size_t)n * 8) : NULL;
            const int width = fn == 2 || fn == 9 ? 2 : (fn == 6 ? 3 : 1);
            double *out = calloc((size_t)(n > 0 ? n : 1) * width, 8);
            const int32_t rc = oracle_jl_eval(fn, n, x, y, out);
            put(&rc, 4);
            put(out, (size_t)n * width * 8);
            free(x), free(y), free(out);
        } else if (job == 6) {
            READ(int32_t, n);
            READ(int32_t, npt);
            READ(int32_t, maxfun);
            READ(double, rhobeg);
            READ(double, rhoend);
            double *x = take((size_t)n * 8);
            double fx = 0.0;
            const int32_t nf = oracle_newuoa(n, npt, x, rhobeg, rhoend, maxfun, rosen, NULL, &fx);
            put(&nf, 4);
            put(x, (size_t)n * 8);
            put(&fx, 8);
            free(x);
        } else {
            fprintf(stderr, "asan_driver: unknown job %d\n", job);
            return 2;
        }
    }
    return 0;
}
