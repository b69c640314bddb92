/*
 * gpdemod — MI355X (gfx950) per-pixel complex demodulation engine, C ABI.
 *
 * Drop-in boundary for FerreolS/GPPupilDemodulation.jl @ 2024-10-16:
 *   demodulateall(timestamp, data; init, recenter, faintparam, onlyhigh, fitoffsets,
 *                 preswitchdelay, postwitchdelay) -> (output, param, likelihood)
 *   (src/Modulation.jl:344-435).  The Julia side keeps that signature and replaces the
 *   `Threads.@threads` diode loop (src/Modulation.jl:387-433) by ONE call of
 *   gpd_fit_batch covering all 32 diodes (or all windows); see INTEGRATION.md for the
 *   `ccall` stub.  The calling convention mirrors the reference's only native call,
 *   `ccall((:ffcrimll, libcfitsio), Cint, …)` + `fits_assert_ok` (src/FitsUtils.jl:40-59):
 *   integer status return, 0 = ok, message in a caller-owned buffer.
 *
 * Plain C types only (no torch / HIP types in signatures).  All entry points are reentrant;
 * per-device contexts (streams, workspaces) are created lazily under a mutex.
 */
#ifndef GPDEMOD_H
#define GPDEMOD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPD_ABI_VERSION 1

/* Julia ComplexF64 / Complex{Float64}: interleaved (re, im), 16 bytes. */
typedef struct {
    double re, im;
} gpd_c64;

/* Julia ComplexF32: interleaved (re, im), 8 bytes — the precision of the FITS VOLT column. */
typedef struct {
    float re, im;
} gpd_c32;

/* One fitted series = the reference's Modulation record (src/Modulation.jl:24-39:
 * ModulationWithOffsets{c,a,b,ϕ,ω} / ModulationNoOffsets{a,b,ϕ,ω}) plus the likelihood
 * (src/Modulation.jl:359,416) and bookkeeping.  64 bytes.  c == 0 without GPD_FIT_OFFSETS.
 * b, phi are sign-normalised (b >= 0) exactly as src/Modulation.jl:427-430. */
typedef struct {
    gpd_c64 c;
    gpd_c64 a;
    double b;
    double phi;
    double chi2;    /* likelihood = χ²(b,ϕ) = Σ w|r|² / N_valid (src/Modulation.jl:320,416) */
    int32_t nfev;   /* χ² evaluations spent on this series (grid + NEWUOA + checks)          */
    int32_t status; /* GPD_ST_* bits                                                         */
} gpd_param;

/* flags — demodulateall keywords (src/Modulation.jl:345-351) */
#define GPD_FIT_OFFSETS 0x1u      /* fitoffsets=true → ModulationWithOffsets               */
#define GPD_RECENTER 0x2u         /* recenter=true (default in the reference)              */
#define GPD_ONLY_HIGH 0x4u        /* onlyhigh=true (faint mode only)                        */
#define GPD_METHOD_EXACT 0x10u    /* force the per-sample (reference-arithmetic) evaluator  */
#define GPD_METHOD_HARMONIC 0x20u /* force the one-pass harmonic-moment evaluator           */
#define GPD_FP32 0x40u            /* Float32 per-sample arithmetic (BASELINE config 5's fp32
                                     half, the build's own experiment): the exact evaluator
                                     with θ, sin, sincos, phasor, model, products and
                                     residual in Float32 on phases reduced modulo 2π once per
                                     call in Float64; sums and NEWUOA stay Float64.  Not with
                                     FIT_OFFSETS or METHOD_HARMONIC.                          */
/* neither METHOD bit: automatic (harmonic when the timestamps allow it, else exact)          */

/* per-series status bits (the reference ignores NEWUOA's status: check=false) */
#define GPD_ST_REFIT 0x1    /* "bad minima" π-flip re-fit ran (src/Modulation.jl:411-414)    */
#define GPD_ST_MAXFUN 0x2   /* a NEWUOA call stopped at maxfun                               */
#define GPD_ST_NAN 0x4      /* final χ² is NaN (e.g. a 1-sample faint state, src/Faint.jl:97)*/
#define GPD_ST_EXACT 0x8    /* fitted with the exact per-sample evaluator                    */
#define GPD_ST_FALLBACK 0x10 /* harmonic evaluator left its safe |b| range → exact re-fit     */
#define GPD_ST_SYNC 0x20    /* multi-workgroup exact fit: a per-series barrier gave up (a part
                               not resident after ~1 s; never observed) — every part stopped,
                               the record is NaN (with GPD_ST_NAN)                            */

/* error codes (negative) */
#define GPD_OK 0
#define GPD_E_ARG -1
#define GPD_E_HIP -2
#define GPD_E_NODEV -3
#define GPD_E_OOM -4
#define GPD_E_UNSAFE -5 /* GPD_METHOD_HARMONIC requested on timestamps it cannot represent */

/* MetState codes (src/Faint.jl:1) for the `state` arrays. */
#define GPD_STATE_TRANSIENT (-1)
#define GPD_STATE_OFF 0
#define GPD_STATE_LOW 1
#define GPD_STATE_NORMAL 2
#define GPD_STATE_HIGH 3

int gpd_version(void);                /* = GPD_ABI_VERSION                            */
const char *gpd_build_id(void);       /* id of the sources the library was built from */
const char *gpd_strerror(int code);   /* static string                                */
int gpd_device_count(void);           /* visible HIP devices (0 if none)              */
/* Free the library's cached device memory on `device` (fit workspace and the arena holding
 * device copies of host-buffer calls; both grow to the largest call and are reused).  Waits
 * for that device's pending library work.  0 = ok, GPD_E_ARG for a bad device.  No reference
 * counterpart (Julia frees through its GC); call it after a one-off very large batch. */
int gpd_release(int device);

/* Test and diagnostics controls (no reference counterpart: demodulateall has no such knobs,
 * src/Modulation.jl:344-351).  The library reads no environment variable; these process-wide
 * options default to the production path and are set only by tests and A/B tools, through this
 * call.  Names and defaults (INTEGRATION.md lists them): mix 1, faint_stats 0, faint_side 0,
 * fake_gpus 0, exact_g 0, exact_waves 0, exact_wgt 0, exact_fast 1, exact_mcache 1,
 * xspin_test 0, units 0, upw 0, fit_lanes 0, fit_lps 0, fit_wpb 0, cohorts 1, harm_min_span 256, fs_cohort_mb 4096,
 * moments 0, fit_prof 0, sync_debug 0, host_prof 0, fit_mcache 1, stage_pinned 1, h2d_parts 0
 * (0 = automatic where a count is meant).
 * gpd_set_option / gpd_get_option: GPD_OK, or GPD_E_ARG for an unknown name.
 * gpd_option_name(i): the i-th option's name, NULL past the last. */
int gpd_set_option(const char *name, int64_t value);
int gpd_get_option(const char *name, int64_t *value);
void gpd_reset_options(void);
const char *gpd_option_name(int index);

/*
 * demodulateall itself (src/Modulation.jl:344-435) on the library's side of the boundary: the
 * exposure as the reference takes it and returns it.
 *   data, ldd        the N×40 column-major matrix in idx() order (src/Modulation.jl:17-22):
 *                    columns 0..31 the diodes, 32..39 the fibre couplers; ldd ≥ n_samples
 *   t, state, xinit, flags, maxfun   as gpd_fit_batch (ω = M_2PI = 6.283185, src/Modulation.jl:11,399)
 *   params[32]       the 32 diodes' records in idx() order (param, likelihood)
 *   output, ldo      a second N×40 matrix (ldo ≥ n_samples) that receives what
 *                    `output = copy(data)` and the diode loop leave in it (:353, :417-425):
 *                    columns 0..31 the demodulated diodes, 32..39 the FC columns as given.
 *                    The caller allocates it (Julia `similar(data)`) and need not touch it:
 *                    the library fills every column — the demodulated ones through a bounded
 *                    staging ring (4 × 16 MB per device, pinned; pageable if pinning fails) and
 *                    parallel host copies, the FC ones copied while the device computes — so no
 *                    `copy(data)` of the exposure runs on the caller's side and the first touch
 *                    of the fresh pages is spread over threads.  output must not overlap data
 *                    (GPD_E_ARG): it is a fresh array, as `copy(data)` is.
 *   n_gpus           devices (as gpd_fit_batch; one exposure runs on one)
 * _c32: ComplexF32 data and output (the FITS VOLT precision; Float64 arithmetic, the
 * demodulated columns rounded to Float32 as Complex{Float32}.(…) does).
 */
int gpd_demodulateall(int64_t n_samples, const double *t, const gpd_c64 *data, int64_t ldd,
                      const int8_t *state, const double *xinit, uint32_t flags, int32_t maxfun,
                      gpd_param *params, gpd_c64 *output, int64_t ldo, int32_t n_gpus,
                      char *errbuf, size_t errlen);
int gpd_demodulateall_c32(int64_t n_samples, const double *t, const gpd_c32 *data, int64_t ldd,
                          const int8_t *state, const double *xinit, uint32_t flags,
                          int32_t maxfun, gpd_param *params, gpd_c32 *output, int64_t ldo,
                          int32_t n_gpus, char *errbuf, size_t errlen);

/*
 * Fit (and optionally demodulate) a batch of series.  Replaces the diode loop of
 * demodulateall (src/Modulation.jl:387-433): per series, the FC phasor
 * exp(im·angle(fc)) (:388), faint power/weight (:391-396, src/Faint.jl:89-100), the 8-point
 * ϕ grid at b = 0.1 (:402-405), NEWUOA(rhobeg 1, rhoend 1e-3) (:407, :332-342), the π-flip
 * check and re-fit (:408-414), the final χ² (:416), the output column (:417-425) and the sign
 * normalisation (:426-431).
 *
 *   n_samples, t[n_samples]     timestamps (s), shared by every series (Float64)
 *   d, ldd                      series, column-major complex, column k = series k
 *                               (Julia Matrix{ComplexF64} column, idx() order)
 *   fc, n_fc, ldfc              raw fibre-coupler columns (complex); the phasor is formed here
 *   fc_of_pixel[n_pixels]       FC column index (0-based) used by series k
 *   state[n_samples]            MetState per sample (faint mode), or NULL (non-faint: w≡1, p=phasor)
 *   omega                       modulation pulsation (reference: M_2PI = 6.283185)
 *   xinit                       NULL → init=:auto grid; else {b, ϕ} start for every series
 *   flags                       GPD_* above
 *   maxfun                      NEWUOA evaluation cap per call (<=0 → 60 = 30·n)
 *   out_params[n_pixels]        fitted records
 *   out_demod, ldo              NULL → fit only; else demodulated columns (all n_samples)
 *   n_gpus                      <=0 → 1; series are sharded over that many devices
 *   errbuf, errlen              optional message buffer
 * Host pointers; synchronous.  Returns GPD_OK or a negative GPD_E_*.
 */
int gpd_fit_batch(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c64 *d,
                  int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                  const int32_t *fc_of_pixel, const int8_t *state, double omega,
                  const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                  gpd_c64 *out_demod, int64_t ldo, int32_t n_gpus, char *errbuf, size_t errlen);

/*
 * Same computation on device-resident buffers of device `device` (all pointers are device
 * pointers, params included), enqueued on `stream` (hipStream_t, NULL = default stream).
 * Asynchronous: returns once enqueued.  Workspace is owned by the library (per device,
 * grown on demand, reused across calls); concurrent calls on one device serialise on it.
 */
int gpd_fit_batch_dev(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c64 *d,
                      int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                      const int32_t *fc_of_pixel, const int8_t *state, double omega,
                      const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                      gpd_c64 *out_demod, int64_t ldo, int device, void *stream, char *errbuf,
                      size_t errlen);

/*
 * χ²(b_k, ϕ_k) of every series at a caller-given point, no optimisation: the Chi2CostFunction
 * functor lkl(b, ϕ) (src/Modulation.jl:318-330) as a batch.  bphi[2k], bphi[2k+1] = (b, ϕ) of
 * series k.  out_params[k] receives chi2 and the closed-form a (and c) at that point; b, phi echo
 * the input.  Same data arguments and flags as gpd_fit_batch (METHOD bits select the evaluator).
 */
int gpd_chi2_batch(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c64 *d,
                   int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                   const int32_t *fc_of_pixel, const int8_t *state, double omega,
                   const double *bphi, uint32_t flags, gpd_param *out_params, int32_t n_gpus,
                   char *errbuf, size_t errlen);

int gpd_chi2_batch_dev(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c64 *d,
                       int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                       const int32_t *fc_of_pixel, const int8_t *state, double omega,
                       const double *bphi, uint32_t flags, gpd_param *out_params, int device,
                       void *stream, char *errbuf, size_t errlen);

/*
 * Windowed demodulation (processmetrology with `window`, src/GPPupilDemodulation.jl:191-205):
 * the samples are partitioned into consecutive windows of `window` samples (the last one
 * shorter, Iterators.partition) and every window is fitted as its own demodulateall call —
 * one call here covers all windows × columns.  d/fc/t/state/out_demod are the whole-exposure
 * arrays (as gpd_fit_batch, n_cols series columns); out_params has ceil(n_samples/window) ×
 * n_cols records, window-major (record w·n_cols + k = column k of window w); out_demod rows of
 * window w are demodulated with that window's parameters.  Per-window state statistics
 * (compute_mean_var_power on state[I]) and valid-sample counts follow the reference.  By
 * default the windows are fitted from per-window harmonic moments (one workgroup per window ×
 * column); with FIT_OFFSETS, or METHOD_EXACT, by the exact evaluator (METHOD_HARMONIC with
 * FIT_OFFSETS is rejected here).  n_gpus > 1 splits the windows across devices.
 */
int gpd_fit_windows(int64_t n_samples, int64_t window, int64_t n_cols, const double *t,
                    const gpd_c64 *d, int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                    const int32_t *fc_of_col, const int8_t *state, double omega,
                    const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                    gpd_c64 *out_demod, int64_t ldo, int32_t n_gpus, char *errbuf, size_t errlen);

int gpd_fit_windows_dev(int64_t n_samples, int64_t window, int64_t n_cols, const double *t,
                        const gpd_c64 *d, int64_t ldd, const gpd_c64 *fc, int64_t n_fc,
                        int64_t ldfc, const int32_t *fc_of_col, const int8_t *state, double omega,
                        const double *xinit, uint32_t flags, int32_t maxfun,
                        gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo, int device,
                        void *stream, char *errbuf, size_t errlen);

/*
 * processmetrology's numeric core (src/GPPupilDemodulation.jl:147-171 and, with window > 0,
 * 191-207) on one device, straight from the FITS VOLT column: volt = n_samples Float32 rows
 * of 80 values [re1 im1 … re40 im40] (row pitch ldv floats, the FITS/Julia layout), centres =
 * the 40 column centres subtracted first (`offsets` vector; NULL = none, e.g. fitoffsets), then
 * demodulateall over the 32 diode columns (window = 0) or every window of `window` samples.
 * out_params: 32 records (window = 0) or ceil(n_samples/window)×32, window-major.
 * out_volt (optional, pitch ldov ≥ 80 floats): the demodulated rows in the same Float32 layout,
 * FC columns carrying the centred input (volt[1:2:end,:] .= real(output)', Float32.(volt)).
 */
int gpd_process_volt(int64_t n_samples, const double *t, const float *volt, int64_t ldv,
                     const gpd_c64 *centres, const int8_t *state, double omega,
                     const double *xinit, uint32_t flags, int32_t maxfun, int64_t window,
                     gpd_param *out_params, float *out_volt, int64_t ldov, int device,
                     char *errbuf, size_t errlen);

/*
 * Float32-storage variants (BASELINE config 5; the VOLT column is Float32 on disk,
 * src/GPPupilDemodulation.jl:147): d and fc are ComplexF32 columns (ldd, ldfc in elements),
 * widened to Float64 as they are loaded, so every χ² evaluation and the fit run in Float64 on
 * exactly the values Float64.(data) would hold — results equal gpd_fit_batch / gpd_fit_windows
 * on the widened arrays, with half the HBM traffic of the series pass.  Same arguments,
 * flags, outputs (complex128 out_demod) and errors as the Float64 entry points.
 * The reference's demodulateall(::Vector{T}, ::Matrix{Complex{T}}) is generic in T
 * (src/Modulation.jl:344); with T = Float32 it would also compute in Float32 — this engine keeps
 * Float64 arithmetic (the reference's own Float32 path cannot run: binit is Float64, :403).
 */
int gpd_fit_batch_c32(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c32 *d,
                      int64_t ldd, const gpd_c32 *fc, int64_t n_fc, int64_t ldfc,
                      const int32_t *fc_of_pixel, const int8_t *state, double omega,
                      const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                      gpd_c64 *out_demod, int64_t ldo, int32_t n_gpus, char *errbuf, size_t errlen);

int gpd_fit_batch_c32_dev(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c32 *d,
                          int64_t ldd, const gpd_c32 *fc, int64_t n_fc, int64_t ldfc,
                          const int32_t *fc_of_pixel, const int8_t *state, double omega,
                          const double *xinit, uint32_t flags, int32_t maxfun,
                          gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo, int device,
                          void *stream, char *errbuf, size_t errlen);

int gpd_fit_windows_c32(int64_t n_samples, int64_t window, int64_t n_cols, const double *t,
                        const gpd_c32 *d, int64_t ldd, const gpd_c32 *fc, int64_t n_fc,
                        int64_t ldfc, const int32_t *fc_of_col, const int8_t *state, double omega,
                        const double *xinit, uint32_t flags, int32_t maxfun,
                        gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo, int32_t n_gpus,
                        char *errbuf, size_t errlen);

int gpd_fit_windows_c32_dev(int64_t n_samples, int64_t window, int64_t n_cols, const double *t,
                            const gpd_c32 *d, int64_t ldd, const gpd_c32 *fc, int64_t n_fc,
                            int64_t ldfc, const int32_t *fc_of_col, const int8_t *state,
                            double omega, const double *xinit, uint32_t flags, int32_t maxfun,
                            gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo, int device,
                            void *stream, char *errbuf, size_t errlen);

/*
 * buildstates (src/Faint.jl:21-73): two-timer faint state machine on the host.
 * timer1 = HIGH switch times, timer2 = LOW switch times (FaintStates already orders them by
 * voltage, src/Faint.jl:12-19), both already shifted by lag·timestep.  Writes MetState codes.
 */
int gpd_buildstates(int64_t n_samples, const double *t, int64_t n1, const double *timer1,
                    int64_t n2, const double *timer2, double preswitchdelay,
                    double postwitchdelay, int8_t *states);

/*
 * buildstates on device (same semantics, src/Faint.jl:21-73): t [n_samples] and states
 * [n_samples] are device arrays of device `device`, timer1 [n1] / timer2 [n2] host arrays of the
 * unshifted switch times (buildfaintparameters, src/GPPupilDemodulation.jl:64-81), shifted on
 * device by lag·(t[1] − t[0]) as src/Faint.jl:25-26.  Enqueued on `stream`; the timer lists may
 * be released when the call returns.  n1, n2 ≤ 4096.  Non-decreasing timestamps: firing samples
 * by binary search and a parallel fill; otherwise the reference loop on one lane.
 */
int gpd_buildstates_dev(int64_t n_samples, const double *t, int64_t n1, const double *timer1,
                        int64_t n2, const double *timer2, int64_t lag, double preswitchdelay,
                        double postwitchdelay, int8_t *states, int device, void *stream);

/*
 * compute_mean_var_power (src/Faint.jl:89-100) as demodulateall applies it to whole series
 * (src/Modulation.jl:373-396): per series k (column k of d, host buffers) and MetState, over the
 * valid samples (TRANSIENT dropped; GPD_ONLY_HIGH in flags keeps HIGH ∪ NORMAL),
 *   m = mean(abs, d[state .== s]),   w = 1 / var(abs.(d[state .== s]); mean = m)
 * — computed by the kernels of the exact evaluator (method EXACT, and the harmonic path with
 * option faint_stats = 1|2), bit for bit the oracle's two-pass restatement.  The default
 * whole-exposure harmonic path forms these statistics inside its moment pass (one pass,
 * shifted sums per state: m within 1e-14, w within 1e-13 relative of these values) for the
 * harmonic fit; the series it hands to the exact evaluator (GPD_ST_FALLBACK) get these two-pass
 * statistics first, so every exact record — method EXACT and fallback — is the oracle's bit for
 * bit (tests/test_gpu_parity.py::test_faint_large_b_fallback_statistics).
 * out[10k + c] = m and out[10k + 5 + c] = w of MetState code c − 1 (c = 0 TRANSIENT … 4 HIGH;
 * NaN for a state without samples, w NaN for a 1-sample state, as Julia's 0/0).  Synchronous.
 */
int gpd_mean_var_power(int64_t n_samples, int64_t n_series, const gpd_c64 *d, int64_t ldd,
                       const int8_t *state, uint32_t flags, double *out, int device, char *errbuf,
                       size_t errlen);

/*
 * Synthetic GRAVITY-like metrology batch generated ON DEVICE (benchmarks):
 * d[k][i] = p_i(c_k + a_k exp(j b_k sin(ω t_i + ϕ_k))) + σ CN(0,1), FC column g = 1.3 exp(jΦ_g),
 * Φ a random walk (σ 1e-3 rad/step), 4 series per FC column, counter-based RNG keyed by
 * (seed, global series index, sample) so that shards generate identical data.
 * t[i] = t0 + i·dt.  truth (optional, device) receives {c, a, b, ϕ} per series as gpd_param.
 */
int gpd_synth_fill_dev(int64_t n_samples, int64_t n_pixels, int64_t pixel_offset, uint64_t seed,
                       double t0, double dt, double sigma, int with_offsets, double omega,
                       double *t, gpd_c64 *d, int64_t ldd, gpd_c64 *fc, int64_t ldfc,
                       int32_t *fc_of_pixel, gpd_param *truth, int device, void *stream);

/*
 * Julia Base's Float64 elementary functions exactly as the device evaluates them (gpd_jlmath.h:
 * the restatement the exact evaluator applies per sample, src/Modulation.jl:137,388,419-421,
 * src/Faint.jl:95-97), for host-vs-device bit-for-bit checks.  fn: 0 sin, 1 cos, 2 sincos (out
 * holds n (s, c) pairs), 3 atan, 4 atan(x[i], y[i]), 5 hypot(x[i], y[i]), 6 rem_pio2 (n triples
 * (quadrant, hi, lo)), 7 hypot(x[i], y[i]) in its branch-free form (the faint statistics'),
 * 8 sin and 9 sincos (pairs) through the branch-free per-regime forms the exact evaluator
 * batches (= fn 0 and 2), 10 sin(fl(x[i] + y[0])) through the exact evaluator's Payne–Hanek
 * table of x and shift of ϕ = y[0] (= fn 0 of the sum; NaN where the shift does not apply).  Host arrays (y may be NULL for the one-argument functions),
 * synchronous.
 */
int gpd_libm_eval(int fn, int64_t n, const double *x, const double *y, double *out, int device);

/* Per-kernel timing of the last gpd_fit_batch_dev call on `device` (ms, HIP events on the
 * launch stream).  names/ms arrays of length cap; returns the number of entries. */
int gpd_last_timings(int device, const char **names, double *ms, int cap);

/* Faint statistics of the last fit call on `device` (test hook): the first n_series records of
 * 16 doubles each — m of MetState code c − 1 at [16k + c] (c = 0 TRANSIENT … 4 HIGH), w at
 * [16k + 5 + c], then Σw|d|², Σw m² n, Σ(w m)²|d|² at [16k + 10 … 12] — as the fit used them
 * (the fused statistics of the state-split moment pass for whole-exposure harmonic fits — the
 * two-pass ones for the series re-fitted by the exact fallback —, the separate kernels
 * otherwise).  Waits for that call.  GPD_E_ARG if it had no faint series. */
int gpd_last_faint_stats(int device, double *out, int64_t n_series);

#ifdef __cplusplus
}
#endif
#endif /* GPDEMOD_H */
