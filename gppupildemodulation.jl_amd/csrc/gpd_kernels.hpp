// gfx950 kernels of the demodulation engine.  See DESIGN.md for the data layout and rooflines.
//
// Reference hot path (FerreolS/GPPupilDemodulation.jl @ 2024-10-16): the per-diode body of
// demodulateall (src/Modulation.jl:388-432) — χ²(b,ϕ) (Chi2CostFunction, :245-330) minimised by
// NEWUOA (:332-342) from an 8-point ϕ grid, π-flip check, final χ², output column, sign
// normalisation — plus the faint-mode weights (src/Faint.jl:89-100).
//
// Two evaluators of χ²(b,ϕ), both feeding the same device NEWUOA (gpd_newuoa.hpp):
//   exact     one workgroup per series, every χ² evaluation is a full pass over the samples
//             with the reference's arithmetic (model → a (or c,a) → residual norm);
//   harmonic  one HBM pass computes Jacobi–Anger moments F_n = Σ_i q_i e^{-j n x_i}
//             (q = w p̄ d, x = fl(ω t)); afterwards χ² costs O(K) per evaluation:
//             S(b,ϕ) = Σ_n J_n(b) e^{-j n ϕ} F_n,  N χ² = Σ w|d|² − |S|²/Σ w|p|².
#pragma once

#include "gpd_device.hpp"
#include "gpd_newuoa.hpp"

// Split build: build.py compiles the kernels in several translation units (gpd_engine.hip =
// unit 0 with the host code and the light kernels, gpd_part*.hip) in parallel.  GPD_PART is
// the unit being compiled; a kernel body is compiled only in the units of its GPD_OWNS mask,
// the other units see its declaration and launch it through the host stub the owning unit
// defines (each unit instantiates the template kernels it owns, gpd_part*.hip).  Without
// GPD_PART every kernel is defined (single-unit build).
#ifdef GPD_PART
#define GPD_OWNS(mask) ((((mask) >> GPD_PART) & 1) != 0)
#else
#define GPD_OWNS(mask) 1
#endif
#define GPD_U_ENGINE 0x1  // unit 0: gpd_engine.hip
#define GPD_U_FITH 0x2    // unit 1: k_fit_harmonic, k_chi2_harmonic
#define GPD_U_MOM 0x44    // units 2, 6: k_moments_ws (Float64 / Float32 storage)
#define GPD_U_EXACT 0xF198  // units 3, 4, 7, 8 / 12-15: k_fit_exact (faint × offsets, MINB 1 / 2)
#define GPD_U_EXACT64 0xF0000  // units 16-19: k_fit_exact one wave per series (faint × offsets)
#define GPD_U_CHI2X 0xE20  // units 5, 9, 10, 11: k_chi2_exact, k_refine_exact

namespace gpd {

constexpr int KH = 24;               // harmonics kept (|b| ≤ ~4.3 at 1e-16 tail)
constexpr int NMOM = 3 + 4 * KH;     // F0r, F0i, W2, then (A,B,C,D)_n for n = 1..K
// shortest window fitted from harmonic moments: below it NEWUOA's landing point drifts by
// ~1e-10 under the expansion's χ² rounding and the exact evaluator is cheap
constexpr long long HARM_MIN_SPAN = 256;
constexpr int MOM_TS = 8;            // samples per LDS tile in the moment kernel
constexpr int EXACT_WG = 256;        // threads per series in the exact evaluator
constexpr double PI_F64 = 3.141592653589793;

// ϕrange = range(-π, π, 8) (src/Modulation.jl:360), bit-exact Float64 values.
static __device__ __constant__ const double c_phi_grid[8] = {
    -0x1.921fb54442d18p+1, -0x1.1f3b3855544c8p+1, -0x1.58ad76cccb8f0p+0, -0x1.cb91f3bbba140p-2,
    0x1.cb91f3bbba140p-2,  0x1.58ad76cccb8f0p+0,  0x1.1f3b3855544c8p+1,  0x1.921fb54442d18p+1};

// status bits (mirror include/gpdemod.h)
constexpr int ST_REFIT = 0x1, ST_MAXFUN = 0x2, ST_NAN = 0x4, ST_EXACT = 0x8, ST_FALLBACK = 0x10,
              ST_SYNC = 0x20;
constexpr uint32_t F_OFFSETS = 0x1u, F_RECENTER = 0x2u, F_ONLY_HIGH = 0x4u, F_FP32 = 0x40u;
constexpr uint32_t F_PROF = 0x80000000u;  // internal: k_fit_harmonic cycle split (GPD_FIT_PROF)
// internal (tests, GPD_XSPIN_TEST=1): the multi-workgroup exact fit's barrier gives up at once
// instead of after ~1 s, so the give-up path (poisoned series, GPD_ST_SYNC) runs on demand
constexpr uint32_t F_XSPIN_TEST = 0x40000000u;
// internal (A/B, tests): the exact evaluator's general load path even where FAST applies
constexpr uint32_t F_NOFAST = 0x20000000u;
// Diagnostic cycle counters (options fit_prof, moments = 7: ws_prof) live in the workspace, reached
// through Problem::prof: [0..3] fit split (objective, whole fit, evals, exact exchange),
// [8..15] moment-kernel roles, [16..31] NEWUOA phases (diagnostics build: lane- and wave-level);
// diagnostics build also [PROF_WV + 4 w ..]: harmonic-fit wave w's start and end (s_memrealtime,
// 100 MHz), its lanes' largest evaluation count and its hardware id (HW_ID | XCC_ID << 32)
#ifdef GPD_DIAG
constexpr int PROF_FIT = 0, PROF_WS = 8, PROF_NW = 16, PROF_WV = 40, PROF_WV_MAX = 4096,
              PROF_LEN = PROF_WV + 4 * PROF_WV_MAX;
#else
constexpr int PROF_FIT = 0, PROF_WS = 8, PROF_NW = 16, PROF_LEN = 40;
#endif

struct Param {  // == gpd_param
    double c_re, c_im, a_re, a_im, b, phi, chi2;
    int32_t nfev, status;
};

// Per-launch facts computed on device (k_prepare).
struct Info {
    long long nvalid;  // valid samples (shared by every series)
    int mode;          // 0: harmonic, plain ϕ; 1: harmonic, ϕ quantised to the ulp of fl(ωt); 2: exact only
    int xpos;          // 1: every valid fl(ωt) is > 0 (none negative, zero or NaN): the exact
                       // evaluator's Payne–Hanek table may apply (jlm_ph_shift, xmin/xmax below)
    double qbase;      // mode 1: a multiple of that ulp inside the binade of fl(ωt)
    double xmin, xmax; // range of |fl(ω t)| over valid samples
    double phimax;     // mode 1: |ϕ| up to which fl(x+ϕ) stays in the binade of every x
};
// ϕ margin of the quantised mode: NEWUOA starts at |ϕ| ≤ π with rhobeg 1 and after a π-flip
// re-fit may step past ±π by its trust radius, so the binade test covers |ϕ| ≤ 2π + 2; an
// evaluation beyond it sends the series to the exact evaluator (HarmChi2::eval).
constexpr double PHI_MARGIN = 2.0 * 3.141592653589793 + 2.0;

struct Problem {
    long long N, P;
    const double *__restrict__ t;
    // series and FC columns: Float64 complex (d, fc) or Float32 complex as stored in the FITS
    // VOLT column (d32, fc32; the other pointer is null); ldd / ldfc count elements
    const c64 *__restrict__ d;
    const c32 *__restrict__ d32;
    long long ldd;
    const c64 *__restrict__ fc;
    const c32 *__restrict__ fc32;
    long long ldfc, n_fc;
    const int32_t *__restrict__ fcop;
    const int8_t *__restrict__ state;  // nullptr: non-faint
    double omega;
    uint32_t flags;
    int maxfun;
    int has_xinit;
    double x0, x1;
    // windowed batches (src/GPPupilDemodulation.jl:191-205): win > 0 splits the samples into
    // consecutive windows of win samples (the last one shorter); series k is column k % ncol
    // of window k / ncol.  win = 0: series k is column k over all N samples.
    long long win, ncol;
    // windows shorter than this many samples are fitted by the exact evaluator (HARM_MIN_SPAN;
    // GPD_HARM_MIN_SPAN overrides it for the window-length sweep, tools/window_sweep.py)
    long long harm_min;
    unsigned long long *prof;  // PROF_LEN diagnostic counters (workspace), or nullptr
    int fit_lanes;             // series per k_fit_harmonic wave (0 = GPD_FIT_WAVE_LANES)
    const float *xr32;         // F_FP32: rem(fl(ω t_i), 2π) per sample (k_phase32), or nullptr
    // exact path: Payne–Hanek table of x_i = fl(ω t_i) (k_ph_table; W lo/hi pairs [2N], then A3
    // [N]; gpd_jlmath.h jlm_ph_table_entry), or nullptr
    const uint64_t *pht;
};

// Column and sample range [s0, s1) of series k.
struct Span {
    long long col, s0, s1;
};
__device__ __forceinline__ Span span_of(const Problem &pb, long long k) {
    if (pb.win <= 0) return {k, 0, pb.N};
    const long long w = k / pb.ncol;
    const long long s0 = w * pb.win;
    return {k - w * pb.ncol, s0, s0 + pb.win < pb.N ? s0 + pb.win : pb.N};
}

// Loads through the global address space.  The Problem's pointers arrive inside a by-value
// struct, where the compiler only sees generic pointers: plain indexing emits flat loads, whose
// waits drain every outstanding memory operation (flat counts on vmcnt and lgkmcnt).  Every
// Problem array is device (global) memory.
__device__ __forceinline__ c64 gld(const c64 *p) {
    const __attribute__((address_space(1))) c64 *g = (const __attribute__((address_space(1))) c64 *)p;
    return c64{g->re, g->im};
}
__device__ __forceinline__ c32 gld(const c32 *p) {
    const __attribute__((address_space(1))) c32 *g = (const __attribute__((address_space(1))) c32 *)p;
    return c32{g->re, g->im};
}
template <class T>
__device__ __forceinline__ T gld(const T *p) {
    return *(const __attribute__((address_space(1))) T *)p;
}

// Element `off` of the series / FC storage, widened to Float64 (uniform branch on the type).
__device__ __forceinline__ c64 d_at(const Problem &pb, long long off) {
    return pb.d32 ? widen(gld(pb.d32 + off)) : gld(pb.d + off);
}
__device__ __forceinline__ c64 fc_at(const Problem &pb, long long off) {
    return pb.fc32 ? widen(gld(pb.fc32 + off)) : gld(pb.fc + off);
}
// Typed base pointers for the kernels instantiated per storage type TS (c64 or c32).
template <class TS>
__device__ __forceinline__ const TS *d_base(const Problem &pb) {
    if constexpr (sizeof(TS) == 8) return pb.d32;
    else return pb.d;
}
template <class TS>
__device__ __forceinline__ const TS *fc_base(const Problem &pb) {
    if constexpr (sizeof(TS) == 8) return pb.fc32;
    else return pb.fc;
}

__device__ __forceinline__ bool sample_valid(const Problem &pb, long long i, int &st) {
    if (pb.state == nullptr) {
        st = 0;
        return true;
    }
    st = gld(pb.state + i);
    if (st == -1) return false;  // TRANSIENT always dropped (src/Modulation.jl:380-382)
    if (pb.flags & F_ONLY_HIGH) return st == 3 || st == 2;  // HIGH ∪ NORMAL (:375-376)
    return true;
}

// FC phasor exp(im·angle(fc)) (src/Modulation.jl:388), Julia arithmetic.
__device__ __forceinline__ c64 fc_phasor(c64 z) { return cisj(jl_atan2(z.im, z.re)); }

// ---------------------------------------------------------------------------------------
// Driver shared by both evaluators (src/Modulation.jl:402-416).  F: double operator()(double(&)[2])
template <class F, class NW>
__device__ __forceinline__ void drive_fit(F &f, const Problem &pb, double (&x)[2], int &status,
                                          NW &nw) {
    if (pb.has_xinit) {
        x[0] = pb.x0;
        x[1] = pb.x1;
    } else {
        double fg[8];
        if constexpr (has_multi<F>::value) {  // the 8 grid points at once (same values)
            double pts[8][2];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                pts[k][0] = 0.1;
                pts[k][1] = c_phi_grid[k];
            }
            f.template multi<8>(pts, fg);
        } else {
            for (int k = 0; k < 8; ++k) {
                double xx[2] = {0.1, c_phi_grid[k]};
                fg[k] = f(xx);
            }
        }
        int best = 0;  // findmin: first NaN wins, else first minimum
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            const bool keep = (fg[best] != fg[best]);  // best is NaN → stays
            if (!keep && ((fg[k] != fg[k]) || fg[best] > fg[k])) best = k;
        }
        double g = c_phi_grid[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) g = (best == k) ? c_phi_grid[k] : g;
        x[0] = 0.1;
        x[1] = g;
    }
    double fx;
    // NEWUOB, then the π-flip check and at most one re-fit from ϕ ∓ π (src/Modulation.jl:407-414)
    // — one call site of run() in a two-pass loop, so the inlined NEWUOA exists once in the
    // kernel's code (r4: the harmonic fit kernel 19.5 k → ~10 k instructions, against a 64 KB
    // instruction cache shared by two CUs), the same operations in the same order
    for (int pass = 0;; ++pass) {
        const int nf = nw.run(x, 1.0, 1e-3, pb.maxfun, f, fx);
        if (nf >= pb.maxfun) status |= ST_MAXFUN;
        if (pass > 0) break;
        const double php = x[1] + (x[1] < 0 ? PI_F64 : -PI_F64);
        double lklval, lflip;
        if constexpr (has_multi<F>::value) {  // lkl(x) and lkl(x[1], ϕπ) at once
            double pts[2][2] = {{x[0], x[1]}, {x[0], php}}, v[2];
            f.template multi<2>(pts, v);
            lklval = v[0];
            lflip = v[1];
        } else {
            lklval = f(x);
            double xf[2] = {x[0], php};
            lflip = f(xf);
        }
        if (!(lklval > lflip)) break;  // "bad minima" (src/Modulation.jl:411-414)
        status |= ST_REFIT;
        x[1] = php;
    }
}

template <class F>
__device__ __forceinline__ void drive_fit(F &f, const Problem &pb, double (&x)[2], int &status) {
    Newuoa<2, 5> nw;  // per-thread state (exact path: replicated in every thread)
    drive_fit(f, pb, x, status, nw);
}

__device__ __forceinline__ void store_param(Param *out, double *raw, long long k, double c_re,
                                            double c_im, double a_re, double a_im, double b,
                                            double phi, double chi2, int nfev, int status) {
    raw[2 * k] = b;  // pre-normalisation (b, ϕ) feed the output pass (src/Modulation.jl:417-425)
    raw[2 * k + 1] = phi;
    if (b < 0) {  // src/Modulation.jl:427-430
        b *= -1;
        phi += (phi < 0 ? PI_F64 : -PI_F64);
    }
    if (chi2 != chi2) status |= ST_NAN;
    Param p;
    p.c_re = c_re;
    p.c_im = c_im;
    p.a_re = a_re;
    p.a_im = a_im;
    p.b = b;
    p.phi = phi;
    p.chi2 = chi2;
    p.nfev = nfev;
    p.status = status;
    out[k] = p;
}

// ---------------------------------------------------------------------------------------
// k_prepare: counts valid samples and classifies fl(ωt) for the harmonic path.  Many
// workgroups (k_prepare_part: PREP_PER samples per workgroup, loads issued before use) write
// partial (count, min, max) triples; k_prepare_fin combines them.  The count is an exact integer
// and min/max are order-free, so the result does not depend on the split (r4; it was one
// latency-bound 1024-thread workgroup, 53-73 µs per call).
constexpr int PREP_PER = 4096;  // samples per k_prepare_part workgroup (256 threads × 16)
__global__ __launch_bounds__(256) void k_prepare_part(Problem pb, double *__restrict__ part)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ double red[4 * 4];
    double cnt = 0.0, xmn = 1.0e308, xmx = 0.0, bad = 0.0;
    const long long base = (long long)blockIdx.x * PREP_PER + threadIdx.x;
    constexpr int U = PREP_PER / 256;
    double tv[U];
    int sv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long long i = base + 256LL * u;
        const long long ic = i < pb.N ? i : pb.N - 1;
        tv[u] = gld(pb.t + ic);
        sv[u] = pb.state ? (int)gld(pb.state + ic) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long long i = base + 256LL * u;
        const int st = sv[u];
        bool ok = i < pb.N;
        if (pb.state) ok = ok && st != -1 && (!(pb.flags & F_ONLY_HIGH) || st == 3 || st == 2);
        const double xs = pb.omega * tv[u], x = fabs(xs);
        cnt += ok ? 1.0 : 0.0;
        bad += (ok && !(xs > 0.0)) ? 1.0 : 0.0;  // negative, zero or NaN fl(ωt)
        xmn = ok ? fmin(xmn, x) : xmn;
        xmx = ok ? fmax(xmx, x) : xmx;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        cnt += __shfl_xor(cnt, off, 64);
        bad += __shfl_xor(bad, off, 64);
        xmn = fmin(xmn, __shfl_xor(xmn, off, 64));
        xmx = fmax(xmx, __shfl_xor(xmx, off, 64));
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[wave * 4] = cnt;
        red[wave * 4 + 1] = xmn;
        red[wave * 4 + 2] = xmx;
        red[wave * 4 + 3] = bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            cnt += red[w * 4];
            xmn = fmin(xmn, red[w * 4 + 1]);
            xmx = fmax(xmx, red[w * 4 + 2]);
            bad += red[w * 4 + 3];
        }
        part[4 * blockIdx.x] = cnt;
        part[4 * blockIdx.x + 1] = xmn;
        part[4 * blockIdx.x + 2] = xmx;
        part[4 * blockIdx.x + 3] = bad;
    }
}
#else
;
#endif

__global__ __launch_bounds__(256) void k_prepare_fin(const double *__restrict__ part, int nparts,
                                                     Info *info)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ double red[4 * 4];
    double cnt = 0.0, xmn = 1.0e308, xmx = 0.0, bad = 0.0;
    for (int b = threadIdx.x; b < nparts; b += 256) {
        cnt += part[4 * b];
        xmn = fmin(xmn, part[4 * b + 1]);
        xmx = fmax(xmx, part[4 * b + 2]);
        bad += part[4 * b + 3];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        cnt += __shfl_xor(cnt, off, 64);
        bad += __shfl_xor(bad, off, 64);
        xmn = fmin(xmn, __shfl_xor(xmn, off, 64));
        xmx = fmax(xmx, __shfl_xor(xmx, off, 64));
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[wave * 4] = cnt;
        red[wave * 4 + 1] = xmn;
        red[wave * 4 + 2] = xmx;
        red[wave * 4 + 3] = bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            cnt += red[w * 4];
            xmn = fmin(xmn, red[w * 4 + 1]);
            xmx = fmax(xmx, red[w * 4 + 2]);
            bad += red[w * 4 + 3];
        }
        Info in;
        in.nvalid = (long long)cnt;
        in.xmin = xmn;
        in.xmax = xmx;
        in.xpos = bad == 0.0 ? 1 : 0;
        in.qbase = 0.0;
        // Rounding of θ = fl(fl(ωt) + ϕ) (src/Modulation.jl:137).  While every |fl(ωt)| ± π sits
        // in one binade [2^e, 2^(e+1)), fl(x+ϕ) = x + round(ϕ to a multiple of ulp 2^(e-52)):
        // the harmonic path reproduces it by quantising ϕ.  Small |x| (< 2^16): the per-sample
        // rounding noise is below 2e-11 rad and uncorrelated, harmonic without quantisation.
        const double lo = xmn - PHI_MARGIN, hi = xmx + PHI_MARGIN;
        in.phimax = PHI_MARGIN;
        int elo, ehi;
        frexp(lo > 0 ? lo : 0.0, &elo);
        frexp(hi, &ehi);
        if (hi < 65536.0) {
            in.mode = 0;
        } else if (lo > 64.0 && elo == ehi) {
            in.mode = 1;
            in.qbase = ldexp(0.75, ehi);  // 1.5·2^(e) — a multiple of the ulp in that binade
        } else {
            in.mode = 2;
        }
        if (in.nvalid == 0) in.mode = 2;
        *info = in;
    }
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// k_table: c_n(i) = cos(n x_i), s_n(i) = sin(n x_i), n = 1..K, x_i = fl(ω t_i), by the
// angle-addition recurrence from sincos(x_i) (exact range reduction of x_i; error ~n·eps).
__global__ __launch_bounds__(256) void k_table(const double *__restrict__ t, long long N,
                                               double omega, double *__restrict__ tab)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const double x = omega * t[i];
    double s1, c1;
    jl_sincos(x, &s1, &c1);
    double cn = c1, sn = s1;
    double *row = tab + i * (2 * KH);
#pragma unroll
    for (int n = 1; n <= KH; ++n) {
        row[2 * (n - 1)] = cn;
        row[2 * (n - 1) + 1] = sn;
        const double cn1 = cn * c1 - sn * s1;
        const double sn1 = sn * c1 + cn * s1;
        cn = cn1;
        sn = sn1;
    }
}
#else
;
#endif


// k_table_mix: the table of the mixed-precision moment kernel (k_moments_ws<…, MIX = true>).
// Same 48-double rows per sample, tiles of MM_TS = 32 samples:
//   doubles [0, 32) of row s: cos/sin n x_s for n = 1..16 (fp64, read by the f64 MFMAs);
//   doubles [32, 48) of rows 0..15 of a tile (16 × 128 B = 2 KB): the bf16 B fragments of the
//   harmonics 17..24 (16 columns c = 2(n−17) + {0 cos, 1 sin}), as v_mfma_f32_16x16x32_bf16
//   lane l = 16·fk + c reads them: element j ↔ sample fk + 4j of the tile (the order in which
//   the consumer wave's f64 A fragments arrive, K-step j), split T = hi + lo (bf16 each, RNE).
//   Lane l's 32 bytes (hi 16 B, lo 16 B) sit in row l >> 2 at byte 256 + 32 (l & 3).
// Rows ≥ N (up to the tile boundary) are zero.  Launch over ceil(N/32)·32 threads.
__device__ __forceinline__ unsigned short bf16_rne(float f) {
    unsigned u = __builtin_bit_cast(unsigned, f);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}
__global__ __launch_bounds__(256) void k_table_mix(const double *__restrict__ t, long long N,
                                                   double omega, double *__restrict__ tab)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long npad = (N + 31) / 32 * 32;
    if (i >= npad) return;
    double cs[2 * KH];
    if (i < N) {
        const double x = omega * t[i];
        double s1, c1;
        jl_sincos(x, &s1, &c1);
        double cn = c1, sn = s1;
#pragma unroll
        for (int n = 1; n <= KH; ++n) {  // the recurrence of k_table, bit for bit
            cs[2 * (n - 1)] = cn;
            cs[2 * (n - 1) + 1] = sn;
            const double cn1 = cn * c1 - sn * s1;
            const double sn1 = sn * c1 + cn * s1;
            cn = cn1;
            sn = sn1;
        }
    } else {
#pragma unroll
        for (int c = 0; c < 2 * KH; ++c) cs[c] = 0.0;
    }
    double *row = tab + i * (2 * KH);
#pragma unroll
    for (int c = 0; c < 32; ++c) row[c] = cs[c];
    const int s = (int)(i & 31), fk = s & 3, j = s >> 2;
    unsigned char *tile = (unsigned char *)(tab + (i - s) * (2 * KH));
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const float f = (float)cs[32 + c];
        const unsigned short hb = bf16_rne(f);
        const float hf = __builtin_bit_cast(float, (unsigned)hb << 16);
        const unsigned short lb = bf16_rne(f - hf);
        const int l = 16 * fk + c;
        unsigned char *frag = tile + (l >> 2) * (2 * KH * 8) + 256 + 32 * (l & 3);
        ((unsigned short *)frag)[j] = hb;
        ((unsigned short *)(frag + 16))[j] = lb;
    }
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// k_faint_stats: per series and MetState, m = mean(|d|), w = 1/var(|d|; mean=m) (two passes,
// src/Faint.jl:89-100) over the valid samples, plus Σ|d|² per state.  One workgroup per series;
// sums in the canonical order CR8 (8 block sweeps of 256 strided slots, the oracle's gsum), so m
// and w are the oracle's bits.  out[k*16 + ...]: m[5] | w[5] | W2 | DEN | Q2 (state = code + 1).
__device__ __forceinline__ void faint_stats_one(const Problem &pb, long long k,
                                                double *__restrict__ out, double *lds);

__global__ __launch_bounds__(256) void k_faint_stats(Problem pb, double *__restrict__ out)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ double lds[4 * 15];
    faint_stats_one(pb, blockIdx.x, out, lds);
}
#else
;
#endif

// k_faint_stats over the harmonic fit's fallback list (series list[0 .. *count)): the faint
// series the exact evaluator re-fits get compute_mean_var_power's two-pass statistics — the
// oracle's bits — in place of the moment pass's fused ones (m ≤ 1e-14, w ≤ 1e-13 off), so a
// GPD_ST_FALLBACK record is the oracle's bit for bit like any exact record.  The list is read
// on the device (no host round trip); with no fallback the launch only reads the count.
__global__ __launch_bounds__(256) void k_faint_stats_list(Problem pb, const int *__restrict__ list,
                                                          const int *__restrict__ count,
                                                          double *__restrict__ out)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ double lds[4 * 15];
    const long long total = *count;
    for (long long j = blockIdx.x; j < total; j += gridDim.x) {
        faint_stats_one(pb, list[j], out, lds);
        __syncthreads();  // lds is reused by the next listed series
    }
}
#else
;
#endif

__device__ __forceinline__ void faint_stats_one(const Problem &pb, long long k,
                                                double *__restrict__ out, double *lds)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const Span sp = span_of(pb, k);  // per window: compute_mean_var_power on state[I] (:205)
    const long long doff = sp.col * pb.ldd;
    // the loads of U consecutive samples of a slot (2048 apart) are issued together
    constexpr int U = 4;
    auto fetch = [&](long long i0, c64 (&z)[U], int (&st)[U], bool (&ok)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = i0 + 2048LL * u;
            ok[u] = i < sp.s1;
            const long long ic = ok[u] ? i : sp.s0;
            z[u] = d_at(pb, doff + ic);
            ok[u] = ok[u] && sample_valid(pb, ic, st[u]);
        }
    };
    double v[15];
    for (int blk = 0; blk < 8; ++blk) {
        double a[15];
#pragma unroll
        for (int q = 0; q < 15; ++q) a[q] = 0.0;
        for (long long i0 = sp.s0 + 256 * blk + threadIdx.x; i0 < sp.s1; i0 += 2048LL * U) {
            c64 z[U];
            int st[U];
            bool ok[U];
            fetch(i0, z, st, ok);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!ok[u]) continue;
                const double ad = jl_hypot(z[u].re, z[u].im);
                const double d2 = z[u].re * z[u].re + z[u].im * z[u].im;
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    if (st[u] + 1 == q) {
                        a[q] += 1.0;
                        a[5 + q] += ad;
                        a[10 + q] += d2;
                    }
            }
        }
        block_sum<256, 15>(a, lds);
#pragma unroll
        for (int q = 0; q < 15; ++q) v[q] = blk == 0 ? a[q] : v[q] + a[q];
    }
    double m[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) m[q] = v[5 + q] / v[q];
    double s[5];
    for (int blk = 0; blk < 8; ++blk) {
        double a[5] = {0, 0, 0, 0, 0};
        for (long long i0 = sp.s0 + 256 * blk + threadIdx.x; i0 < sp.s1; i0 += 2048LL * U) {
            c64 z[U];
            int st[U];
            bool ok[U];
            fetch(i0, z, st, ok);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!ok[u]) continue;
                const double ad = jl_hypot(z[u].re, z[u].im);
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    if (st[u] + 1 == q) {
                        const double dv = ad - m[q];
                        a[q] += dv * dv;
                    }
            }
        }
        block_sum<256, 5>(a, lds);
#pragma unroll
        for (int q = 0; q < 5; ++q) s[q] = blk == 0 ? a[q] : s[q] + a[q];
    }
    if (threadIdx.x == 0) {
        double *o = out + k * 16;
        double W2 = 0.0, DEN = 0.0, Q2 = 0.0;
        for (int q = 0; q < 5; ++q) {
            const double w = 1.0 / (s[q] / (v[q] - 1.0));
            o[q] = m[q];
            o[5 + q] = w;
            if (v[q] > 0) {
                W2 += w * v[10 + q];
                DEN += w * m[q] * m[q] * v[q];
                Q2 += (w * m[q]) * (w * m[q]) * v[10 + q];
            }
        }
        o[10] = W2;
        o[11] = DEN;
        o[12] = Q2;
    }
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// Faint statistics in one pass over the series and one hypot per sample (k_faint_stats re-reads
// every series for the variance and evaluates Julia's hypot twice per sample: VALU-bound).  The
// same chains as k_faint_stats, so the same bits: a series is split into its FS_G = 8 canonical
// blocks (part g owns the samples i ≡ 256g + t (mod 2048), t = thread, M = ⌈N/2048⌉ per thread).
//   k_faint_p1  per (series, part): loads each sample once (non-temporal, two register batches
//               of FS_U loads in flight), |d| = hypot (branch-free form, FS_U evaluations
//               interleaved), count / Σ|d| / Σ|d|² per state along the slot chain → the part's
//               block totals; |d| is written to a scratch buffer;
//   k_faint_p2  per (series, part): m = the 8 block totals added in block order, then
//               Σ (|d| − m)² along the same chain from the scratch;
//   k_faint_fin per series: adds the block totals in order, writes m, w, W2, DEN, Q2.
// Series are processed in cohorts of ≤ 4 GB of scratch (8 B per sample; streamed, non-temporal).
// No LDS beyond block_sum's,
// no cross-workgroup waits: full occupancy hides the latencies (a persistent one-workgroup-per-CU
// version holding |d| in LDS ran at one wave per SIMD and spent 4.7 ms on C5, latency-bound).
// Whole-exposure series; windows take k_faint_stats (per-window spans).
constexpr int FS_G = 8;  // = CR_BLOCKS, the canonical order's blocks
#ifndef GPD_FS_U
#define GPD_FS_U 2  // A/B builds: -DGPD_FS_U=n (C5 statistics: 4 +4 %, 8 +18 %, 16 +95 %)
#endif
constexpr int FS_U = GPD_FS_U;
#ifndef GPD_FS_U2
#define GPD_FS_U2 4  // k_faint_p2 scratch loads per batch (A/B -DGPD_FS_U2=n; 8: +7 %, 16: +24 % on C5)
#endif
constexpr int FS_U2 = GPD_FS_U2;
constexpr int FS_NV = 16;  // payload doubles per block total (15 used)

// Add (1, a, b) to the sums of state q (no state: q < 0) — the chains of k_faint_stats.  A
// wave's 64 lanes hold 64 consecutive samples (128 ms at 2 ms), almost always of one state:
// then one wave-uniform branch updates that state's three sums; otherwise every state's sums
// take the sample or keep their value (branch-free).
__device__ __forceinline__ void fs_accum3(int q, double a, double b, int (&cnt)[5],
                                          double (&sa)[5], double (&sb)[5]) {
    const int q0 = __builtin_amdgcn_readfirstlane(q);
    if (__builtin_amdgcn_ballot_w64(q != q0) == 0) {
        switch (q0) {
#define GPD_FS_CASE(S)   \
    case S:              \
        cnt[S] += 1;     \
        sa[S] += a;      \
        sb[S] += b;      \
        break;
            GPD_FS_CASE(0) GPD_FS_CASE(1) GPD_FS_CASE(2) GPD_FS_CASE(3) GPD_FS_CASE(4)
#undef GPD_FS_CASE
        default: break;
        }
        return;
    }
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const bool h = q == s;
        cnt[s] += h;
        const double xa = sa[s] + a, xb = sb[s] + b;
        sa[s] = h ? xa : sa[s];
        sb[s] = h ? xb : sb[s];
    }
}

#ifndef GPD_FS_MINW
#define GPD_FS_MINW 1  // A/B builds: minimum waves per SIMD the register allocation must allow
#endif
template <class TS>
__global__ __launch_bounds__(256, GPD_FS_MINW) void k_faint_p1(Problem pb, long long k0, int Mmax,
                                                  double *__restrict__ scr,
                                                  double *__restrict__ xt)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ double lds[4 * 16];
    typedef double nv2d __attribute__((ext_vector_type(2)));
    typedef float nv2f __attribute__((ext_vector_type(2)));
    // samples stay in their storage type until processed (a widening at the load would wait
    // for it there)
    typedef typename std::conditional<sizeof(TS) == 16, nv2d, nv2f>::type VT;
    typedef const __attribute__((address_space(1))) VT gVT;
    typedef __attribute__((address_space(1))) double gd;
    const long long j = blockIdx.x / FS_G, k = k0 + j;
    const int g = (int)(blockIdx.x % FS_G), t = threadIdx.x;
    const long long N = pb.N, i0 = 256LL * g + t;
    const int M = i0 < N ? (int)((N - 1 - i0) / 2048 + 1) : 0;
    const bool only_high = (pb.flags & F_ONLY_HIGH) != 0;
    gVT *dp = (gVT *)d_base<TS>(pb) + k * pb.ldd + i0;
    gd *sp = (gd *)scr + (long long)blockIdx.x * Mmax * 256 + t;
    struct Batch {
        VT z[FS_U];
        int st[FS_U];
    };
    auto issue = [&](Batch &B, int m0) {
#pragma unroll
        for (int u = 0; u < FS_U; ++u) {
            const int m = m0 + u < M ? m0 + u : M - 1;  // clamped (branch-free loads)
            B.z[u] = __builtin_nontemporal_load(dp + 2048LL * m);
            B.st[u] = gld(pb.state + i0 + 2048LL * m);
        }
    };
    int cnt[5] = {0, 0, 0, 0, 0};
    double sa[5] = {0, 0, 0, 0, 0}, s2[5] = {0, 0, 0, 0, 0};
    auto process = [&](const Batch &Bt, int m0) {
        double a[FS_U], d2[FS_U];
#pragma unroll
        for (int u = 0; u < FS_U; ++u) {
            const double zr = (double)Bt.z[u].x, zi = (double)Bt.z[u].y;
            a[u] = jl_hypot_nb(zr, zi);
            d2[u] = zr * zr + zi * zi;
        }
#pragma unroll
        for (int u = 0; u < FS_U; ++u) {
            const int m = m0 + u;
            if (m >= M) break;
            const int c = Bt.st[u];
            const bool ok = c != -1 && (!only_high || c == 3 || c == 2);
            const int q = ok ? c + 1 : -1;
            __builtin_nontemporal_store(a[u], &sp[(long long)m * 256]);
            fs_accum3(q, a[u], d2[u], cnt, sa, s2);
        }
    };
    if (M > 0) {
        Batch A, B;
        issue(A, 0);
        int m0 = 0;
        for (; m0 + FS_U < M; m0 += 2 * FS_U) {
            issue(B, m0 + FS_U);
            process(A, m0);
            if (m0 + 2 * FS_U < M) issue(A, m0 + 2 * FS_U);
            process(B, m0 + FS_U);
        }
        if (m0 < M) process(A, m0);
    }
    double v[15];
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        v[s] = (double)cnt[s];  // counts are exact in Float64: the bits of adding 1.0
        v[5 + s] = sa[s];
        v[10 + s] = s2[s];
    }
    block_sum<256, 15>(v, lds);
    if (t < 15) {
        double x = v[0];
#pragma unroll
        for (int q = 1; q < 15; ++q) x = (t == q) ? v[q] : x;
        xt[(long long)blockIdx.x * FS_NV + t] = x;
    }
}
#else
;
#endif


// the 8 block totals of series j (cohort-local) added in block order
__device__ __forceinline__ void fs_totals(const double *__restrict__ xt, long long j, double (&tv)[15]) {
#pragma unroll
    for (int b = 0; b < FS_G; ++b)
#pragma unroll
        for (int q = 0; q < 15; ++q) {
            const double x = xt[(j * FS_G + b) * FS_NV + q];
            tv[q] = (b == 0) ? x : tv[q] + x;
        }
}

__global__ __launch_bounds__(256) void k_faint_p2(Problem pb, int Mmax,
                                                  const double *__restrict__ scr,
                                                  const double *__restrict__ xt,
                                                  double *__restrict__ x2)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ double lds[4 * 8];
    __shared__ double mus[5];
    typedef const __attribute__((address_space(1))) double gd;
    const long long j = blockIdx.x / FS_G;
    const int g = (int)(blockIdx.x % FS_G), t = threadIdx.x;
    const long long N = pb.N, i0 = 256LL * g + t;
    const int M = i0 < N ? (int)((N - 1 - i0) / 2048 + 1) : 0;
    const bool only_high = (pb.flags & F_ONLY_HIGH) != 0;
    if (t == 0) {
        double tv[15];
        fs_totals(xt, j, tv);
        for (int s = 0; s < 5; ++s) mus[s] = tv[5 + s] / tv[s];
    }
    __syncthreads();
    double mu[5];
#pragma unroll
    for (int s = 0; s < 5; ++s) mu[s] = mus[s];
    gd *sp = (gd *)scr + (long long)blockIdx.x * Mmax * 256 + t;
    double sv[5] = {0, 0, 0, 0, 0};
    for (int mb = 0; mb < M; mb += FS_U2) {
        int qq[FS_U2];
        double aa[FS_U2];
#pragma unroll
        for (int u = 0; u < FS_U2; ++u) {
            const int m = mb + u < M ? mb + u : M - 1;
            const int c = gld(pb.state + i0 + 2048LL * m);
            const bool ok = c != -1 && (!only_high || c == 3 || c == 2);
            qq[u] = (ok && mb + u < M) ? c + 1 : -1;
            aa[u] = __builtin_nontemporal_load(&sp[(long long)m * 256]);
        }
#pragma unroll
        for (int u = 0; u < FS_U2; ++u) {
            const int q = qq[u];
            const int q0 = __builtin_amdgcn_readfirstlane(q);
            if (__builtin_amdgcn_ballot_w64(q != q0) == 0) {  // one state across the wave
                switch (q0) {
#define GPD_FS_CASE(S)                        \
    case S: {                                 \
        const double dv = aa[u] - mu[S];      \
        sv[S] += dv * dv;                     \
    } break;
                    GPD_FS_CASE(0) GPD_FS_CASE(1) GPD_FS_CASE(2) GPD_FS_CASE(3) GPD_FS_CASE(4)
#undef GPD_FS_CASE
                default: break;
                }
                continue;
            }
            double mq = mu[0];
#pragma unroll
            for (int s = 1; s < 5; ++s) mq = q == s ? mu[s] : mq;
            const double dv = aa[u] - mq;
            const double d2v = dv * dv;
#pragma unroll
            for (int s = 0; s < 5; ++s) {
                const double x = sv[s] + d2v;
                sv[s] = q == s ? x : sv[s];
            }
        }
    }
    block_sum<256, 5>(sv, lds);
    if (t < 5) {
        double x = sv[0];
#pragma unroll
        for (int q = 1; q < 5; ++q) x = (t == q) ? sv[q] : x;
        x2[(long long)blockIdx.x * 8 + t] = x;
    }
}
#else
;
#endif


__global__ __launch_bounds__(64) void k_faint_fin(long long k0, const double *__restrict__ xt,
                                                  const double *__restrict__ x2,
                                                  double *__restrict__ out)
#if GPD_OWNS(GPD_U_ENGINE)
{
    // one wave per series: the lanes fetch the 8 × (15 + 5) block totals, lane 0 adds them in
    // block order and writes the record
    __shared__ double v[FS_G * 20];
    const long long j = blockIdx.x;
    for (int e = threadIdx.x; e < FS_G * 20; e += 64) {
        const int b = e / 20, q = e - 20 * b;
        v[e] = q < 15 ? xt[(j * FS_G + b) * FS_NV + q] : x2[(j * FS_G + b) * 8 + (q - 15)];
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double tv[15], ss[5];
    for (int b = 0; b < FS_G; ++b) {
        for (int q = 0; q < 15; ++q) tv[q] = (b == 0) ? v[b * 20 + q] : tv[q] + v[b * 20 + q];
        for (int q = 0; q < 5; ++q) ss[q] = (b == 0) ? v[b * 20 + 15 + q] : ss[q] + v[b * 20 + 15 + q];
    }
    double *o = out + (k0 + j) * 16;
    double W2 = 0.0, DEN = 0.0, Q2 = 0.0;
    for (int q = 0; q < 5; ++q) {
        const double m = tv[5 + q] / tv[q];
        const double w = 1.0 / (ss[q] / (tv[q] - 1.0));
        o[q] = m;
        o[5 + q] = w;
        if (tv[q] > 0) {
            W2 += w * tv[10 + q];
            DEN += w * m * m * tv[q];
            Q2 += (w * m) * (w * m) * tv[10 + q];
        }
    }
    o[10] = W2;
    o[11] = DEN;
    o[12] = Q2;
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// k_phasor: FC phasor buffer for the exact evaluator (only when it fits the workspace).
// F_FP32 phase table: x_i = fl(ω t_i) (the reference's product, src/Modulation.jl:137) reduced
// modulo 2π in Float64 (Cody–Waite with fma: 2π = P1 + P2), rounded to Float32 — the Float32
// evaluator's θ = x_i + ϕ then stays within a few radians, where Float32 sin keeps ~1e-7.
__global__ __launch_bounds__(256) void k_phase32(const double *__restrict__ t, long long N,
                                                 double omega, float *__restrict__ xr)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const double x = omega * t[i];
    const double k = rint(x * 0.15915494309189535);  // 1/(2π)
    double r = fma(-k, 6.283185307179586, x);
    r = fma(-k, 2.4492935982947064e-16, r);
    xr[i] = (float)r;
}
#else
;
#endif

__global__ __launch_bounds__(256) void k_phasor(Problem pb, c64 *__restrict__ ph)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long g = blockIdx.y, N = pb.N;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < N; i += (long long)gridDim.x * 256)
        ph[g * N + i] = fc_phasor(fc_at(pb, g * pb.ldfc + i));
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// HARMONIC PATH — k_moments: the HBM-streaming pass (roofline kernel).
// One wave per workgroup; lane = series (64 series per workgroup); blockIdx.y = sample chunk.
// Series tiles of MOM_TS samples are staged through LDS transposed ([sample][series]) from
// coalesced 128-B row loads; the cos/sin table row of each sample is wave-uniform (SMEM).
// Writes partial moments part[chunk][m][P].
template <bool FAINT>
__global__ __launch_bounds__(64) void k_moments(Problem pb, const double *__restrict__ tab,
                                                const double *__restrict__ fstat,
                                                long long chunk_len, double *__restrict__ part)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ c64 dtile[MOM_TS][65];
    __shared__ c64 ptile[MOM_TS][65];
    const int lane = threadIdx.x;
    const long long p0 = (long long)blockIdx.x * 64;
    const long long pix = p0 + lane;
    const long long s_begin = (long long)blockIdx.y * chunk_len;
    long long s_end = s_begin + chunk_len;
    if (s_end > pb.N) s_end = pb.N;

    double wm[5];  // faint: w_s · m_s for this series
    if (FAINT) {
#pragma unroll
        for (int q = 0; q < 5; ++q) wm[q] = pix < pb.P ? fstat[pix * 16 + 5 + q] * fstat[pix * 16 + q] : 0.0;
    }
    double acc[NMOM];
#pragma unroll
    for (int q = 0; q < NMOM; ++q) acc[q] = 0.0;

    const int ls = lane & (MOM_TS - 1);   // sample within tile this lane stages
    const int lp = lane / MOM_TS;          // series sub-row this lane stages
    for (long long s0 = s_begin; s0 < s_end; s0 += MOM_TS) {
        const long long ss = s0 + ls;
#pragma unroll
        for (int r = 0; r < 64 / MOM_TS; ++r) {
            const long long pp = p0 + lp + r * (64 / MOM_TS) * 1;
            const int prow = lp + r * (64 / MOM_TS);
            c64 dv = {0.0, 0.0}, pv = {0.0, 0.0};
            if (pp < pb.P && ss < s_end) {
                dv = d_at(pb, pp * pb.ldd + ss);
                const c64 z = fc_at(pb, (long long)gld(pb.fcop + pp) * pb.ldfc + ss);
                const double r2 = z.re * z.re + z.im * z.im;
                if (r2 == 0.0) {
                    pv = {1.0, 0.0};  // angle(0) = 0 (a NaN sample stays NaN)
                } else {
                    const double inv = 1.0 / sqrt(r2);
                    pv = {z.re * inv, z.im * inv};
                }
            }
            dtile[ls][prow] = dv;
            ptile[ls][prow] = pv;
        }
        __syncthreads();
        const int nts = (int)((s_end - s0) < MOM_TS ? (s_end - s0) : MOM_TS);
        for (int s = 0; s < nts; ++s) {
            const long long i = s0 + s;
            int st = 0;
            if (FAINT) {
                if (!sample_valid(pb, i, st)) continue;  // wave-uniform
            }
            const c64 dv = dtile[s][lane];
            const c64 pv = ptile[s][lane];
            double qr = fma(pv.re, dv.re, pv.im * dv.im);   // q = p̄ d  (× w m in faint mode)
            double qi = fma(pv.re, dv.im, -(pv.im * dv.re));
            if (FAINT) {
                double f = wm[0];
#pragma unroll
                for (int q = 1; q < 5; ++q) f = (st + 1 == q) ? wm[q] : f;
                qr *= f;
                qi *= f;
            } else {
                acc[2] = fma(dv.re, dv.re, fma(dv.im, dv.im, acc[2]));
            }
            acc[0] += qr;
            acc[1] += qi;
            const double *row = tab + i * (2 * KH);
#pragma unroll
            for (int n = 0; n < KH; ++n) {
                const double c = row[2 * n], sn = row[2 * n + 1];
                acc[3 + 4 * n + 0] = fma(qr, c, acc[3 + 4 * n + 0]);
                acc[3 + 4 * n + 1] = fma(qi, sn, acc[3 + 4 * n + 1]);
                acc[3 + 4 * n + 2] = fma(qi, c, acc[3 + 4 * n + 2]);
                acc[3 + 4 * n + 3] = fma(qr, sn, acc[3 + 4 * n + 3]);
            }
        }
        __syncthreads();
    }
    if (pix < pb.P) {
        double *o = part + (long long)blockIdx.y * NMOM * pb.P + pix;
#pragma unroll
        for (int q = 0; q < NMOM; ++q) o[(long long)q * pb.P] = acc[q];
    }
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// MFMA moment pass (k_moments_ws below): the moments as a dense fp64 contraction on the matrix
//   cores.  Out[row][col] = Σ_s A[row][s] · B[s][col],  row = (series, re/im of q), col =
//   (harmonic n, cos/sin), s = sample.  v_mfma_f64_16x16x4_f64: A = 16 rows (8 series) × 4
//   samples, B = 4 samples × 16 cols (8 harmonics).
// Fragment maps (gfx950, cdna_hip_programming.md §3): A lane l ↔ A[l&15][l>>4];
// B lane l ↔ B[l>>4][l&15]; D lane l, reg r ↔ D[(l>>4)+4r][l&15].
typedef double v4d __attribute__((ext_vector_type(4)));

// z/|z| for the harmonic moments (angle(0) = 0 → 1): v_rsq_f64 + one Newton step, ~1 ulp
// — the harmonic path's tolerance is set by its truncation test, not by correct rounding.
// Only z = 0 maps to 1: a NaN sample keeps a NaN phasor, as exp(im·angle(NaN)) does in the
// reference (src/Modulation.jl:388), so its series end with a NaN χ² (status NAN).
__device__ __forceinline__ c64 unit_phasor(c64 z) {
    const double r2 = fma(z.re, z.re, z.im * z.im);
    double y = __builtin_amdgcn_rsq(r2);
    y = y * fma(-0.5 * r2, y * y, 1.5);
    c64 ph = {z.re * y, z.im * y};
    if (r2 == 0.0) ph = {1.0, 0.0};
    return ph;
}

// A pointer made provably wave-uniform for a buffer descriptor (T8).  readfirstlane returns
// int: each half is taken back to unsigned before widening, or a low word with bit 31 set
// would sign-extend over the high word.
__device__ __forceinline__ void *uniform_ptr(const void *p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    return (void *)(((unsigned long long)hi << 32) | lo);
}
constexpr int MM_TS = 32;          // samples per tile (8 MFMA K-steps)
constexpr int MM_PIX = 128;        // series per workgroup
constexpr int MM_ROW = MM_PIX + 1; // padded LDS row (16-B elements)
constexpr int MM_GRP = MM_PIX / 4; // FC groups per workgroup

__device__ __forceinline__ int mm_phys(int p, int s) { return s * MM_ROW + (p ^ ((s & 1) << 3)); }

// State-split faint moments: one partial slot per valid MetState code (OFF, LOW, NORMAL, HIGH =
// 0..3, src/Faint.jl:1); TRANSIENT (-1) and onlyhigh's excluded states contribute nothing.
constexpr int FST_SLOTS = 4;
__device__ __forceinline__ bool fst_valid(unsigned flags, int st) {
    return st >= 0 && st < FST_SLOTS && (!(flags & F_ONLY_HIGH) || st == 3 || st == 2);
}
// |q| of the fused faint statistics (x = abs(d) through q = p̄ d, |p| = 1): sqrt of the
// fma-formed |q|² by v_rsq_f64 and one Goldschmidt correction (≤ 1 ulp; no rescaling — |q|²
// stays far from the subnormal and overflow ranges for metrology voltages; 0 → 0, Inf → NaN).
// The statistics are a restatement with a stated tolerance (oracle: faint_stats_fused in
// demod_oracle.c forms the same sums from Julia's hypot), not a bit-for-bit one.  r5: 0 → 0
// through rsq of max(|q|², DBL_MIN) (g = 0·y stays 0 through the corrections) instead of a
// compare and two selects — the same bits for every |q|² ≥ DBL_MIN (the hardware v_sqrt_f64
// would be cheaper still but is ~2^-25 relative: tools/probes/sqrt_ulp.hip).
__device__ __forceinline__ double fs_abs(double re, double im) {
    const double r2 = fma(re, re, im * im);
#ifdef GPD_FS_RSQ32  // A/B: the seed from the single-precision rsq (r2 within float's range)
    const double y = (double)__builtin_amdgcn_rsqf((float)fmax(r2, 0x1p-126));
#else
    const double y = __builtin_amdgcn_rsq(fmax(r2, 0x1p-1022));
#endif
    double g = r2 * y, h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    g = fma(fma(-g, g, r2), h, g);
    return g;
}

// One complex element of storage type TS (c64: 16 B, c32: 8 B) through a buffer descriptor;
// kept in its storage type until staged (widening at the load would wait on it there).
// POL: cache policy bits of the load (0 default, 2 = nt: streamed once, no MALL allocation).
template <class TS, int POL = 0>
__device__ __forceinline__ TS buf_ld(__amdgpu_buffer_rsrc_t rs, int voff) {
    if constexpr (sizeof(TS) == 16)
        return __builtin_bit_cast(TS, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, POL));
    else
        return __builtin_bit_cast(TS, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 0, POL));
}

// k_moments_ws: the MFMA contraction with producer/consumer wave roles (every whole-exposure
// series; faint ones weighted per state).
//   Workgroup = 8 waves, one workgroup per CU (LDS 157 KB): waves 0-3 (consumers) only run the
//   MFMA phase — f64 fragments (maps above) for harmonics 1..16 (8 accumulators per
//   wave) and, with MIX, split-bf16 MFMAs for harmonics 17..24 (4 f32 accumulators); waves 4-7
//   (producers) stream d / FC / cos-sin rows two tiles ahead in registers, form q = p̄ d and
//   write the next tile into the other half of a double-buffered LDS tile.  One barrier per
//   tile: consumers on buffer i&1 while producers fill buffer (i+1)&1, so each SIMD hosts one
//   consumer that keeps its matrix core busy and one producer whose loads and VALU work overlap
//   it (a single-role kernel serialises staging and MFMA behind two barriers per tile: 61.5 vs
//   52.6 ms on C3).
// DBG == 6 (diagnostics only): per-role cycle split, summed over waves
//   [0] producer stage, [1] producer issue, [2] producer barrier, [3] consumer MFMA phase,
//   [4] consumer barrier

template <bool B>
struct BoolTag {
    static constexpr bool value = B;
};

template <class TS>
struct WsRegs {
    TS d[4][4], f[4];
    int st;  // FAINT: MetState code of the lane's sample
};

// DBG (timing experiments only, results invalid): 1 = consumers skip the MFMA phase,
// 7 = consumers skip the F0/Σ|q|² VALU, 8 = producers stage d without forming q = p̄ d,
// 2 = producers skip the global loads, 5 = producers only keep the barrier cadence;
// FAINT: 9 = no fused statistics, 10 = no masking of the staged q.
// UNIT: the series are FC columns and d ≡ 1, i.e. the moments G_n = Σ p̄ e^{-jnx} of the
// unit phasors (harmonic fitoffsets: Σ w m = conj(Σ_n J_n(b) e^{-jnϕ} G_n)).
// MIX (production): harmonics 1..16 on the f64 MFMAs (2 column tiles), harmonics 17..24 on
// v_mfma_f32_16x16x32_bf16 with both operands split hi + lo (A_hi·B_hi + A_hi·B_lo + A_lo·B_hi,
// ~2^-17 relative per product, f32 accumulation over the chunk).  Those moments enter χ² only
// through J_n(b) ≤ J_17(3.9) ≈ 2e-10 at the largest b NEWUOA probes, so their
// ~1e-3·|q| absolute error moves S by < 1e-12·|q| — below the f64 evaluation's own rounding at
// the χ² tolerance.  It replaces 32 of the 96 f64 MFMAs per tile (64 cycles each) by 12 bf16
// MFMAs (16 cycles each).  Needs the k_table_mix layout.  MIX = false: all 24 harmonics in f64
// (k_table layout).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
// (f0, f1) → packed bf16 hi and lo dwords (element 0 in the low half), RNE
__device__ __forceinline__ void split_bf16x2(float f0, float f1, unsigned &h, unsigned &l) {
    const v2f f = {f0, f1};
    const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(f, bf16x2));
    const v2f hf = {__builtin_bit_cast(float, hu << 16), __builtin_bit_cast(float, hu & 0xffff0000u)};
    const v2f r = f - hf;
    h = hu;
    l = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));
}

// FAINT (state-split moments, r3): the weighted moments Σ w_s m_s p̄ d e^{-jnx} of a faint
// series (compute_mean_var_power's per-state weight w and power m, src/Faint.jl:89-100;
// src/Modulation.jl:392-396) are linear in the per-state constant w_s·m_s, so the kernel sums
// the unweighted q = p̄ d per (unit, state) and k_reduce_moments applies w_s·m_s — the moment
// pass does not wait for the faint statistics, which run beside it on a second stream.  Each
// 32-sample tile is given one state: that of its first valid sample (samples outside the valid
// mask — TRANSIENT, or not HIGH/NORMAL with onlyhigh, src/Modulation.jl:373-382 — contribute
// 0); the accumulators are flushed into part[unit][state] whenever the tile state changes and
// at the unit end (adding to the slot when a state recurs within a unit), smask[unit] records
// the slots written.  A valid sample whose state differs from its tile's (two valid states
// within 32 samples, which buildstates' TRANSIENT margins never produce) is left to
// k_moments_fix.  Tiles with no valid sample skip the MFMAs.
// Sample units: the samples are cut into fixed units of unit_len samples (a function of N only,
// plan() in gpd_engine.hip) and the consumers write one set of partial moments per unit,
// part[unit][moment][series], restarting their accumulators at each unit boundary; a workgroup
// streams chunk_len = (units per workgroup) × unit_len samples.  The units per workgroup follow
// the grid fill (a function of P), but every moment is the same sum in the same order for any
// of them — a series' moments, and so its fit, do not depend on the batch or shard it is in.
template <int DBG = 0, bool UNIT = false, class TS = c64, int POL = 0, bool MIX = true,
          bool FAINT = false>
__global__ __launch_bounds__(512, 1) void k_moments_ws(Problem pb, const double *__restrict__ tab,
                                                       long long chunk_len, long long unit_len,
                                                       double *__restrict__ part,
                                                       unsigned *__restrict__ smask = nullptr,
                                                       double *__restrict__ fsp = nullptr,
                                                       int *__restrict__ fcnt = nullptr,
                                                       const int *__restrict__ dhdr = nullptr)
#if GPD_OWNS(GPD_U_MOM)
{
    __shared__ c64 qs[2][MM_TS * MM_ROW];
    __shared__ __attribute__((aligned(16))) double ts[2][MM_TS * 2 * KH];
    __shared__ int fcl[MM_PIX];
    __shared__ int tds[2];       // FAINT: the state of the staged tile (-1: no valid sample)
    __shared__ unsigned tmk[2];  // FAINT: the staged tile's samples of that state (bit = sample)
    // FAINT: the producer threads' statistics (K, S1, S2) — in the LDS left over (6 KB), not in
    // registers: the faint producers are at the 256-VGPR limit of two waves per SIMD
    __shared__ double fsl[FAINT ? 3 : 1][FAINT ? 256 : 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long p0 = (long long)blockIdx.x * MM_PIX;
    const long long s_begin = (long long)blockIdx.y * chunk_len;
    long long s_end = s_begin + chunk_len;
    if (s_end > pb.N) s_end = pb.N;
    const int ntiles = s_end > s_begin ? (int)((s_end - s_begin + MM_TS - 1) / MM_TS) : 0;
    const int tpu = (int)(unit_len / MM_TS);  // tiles per unit (units are whole tiles)
    const long long u_first = s_begin / unit_len;
    if (tid < MM_PIX) {
        const long long p = p0 + tid;
        fcl[tid] = p < pb.P ? pb.fcop[p] : 0;
    }
    __syncthreads();
    // general layout: some series of the workgroup does not use its 4-group's FC column
    // (uniform: every thread scans the same 128 LDS words)
    const int nrow = (int)((pb.P - p0) < MM_PIX ? (pb.P - p0) : MM_PIX);
    bool general = false;
    for (int k = 0; k < nrow; ++k) general |= fcl[k] != fcl[k & ~3];

    if (wave >= 4) {
        // ================================ producer ================================
        // Branch-free loads (clamped indices; d through a buffer descriptor whose range check
        // zero-fills rows beyond P), so the in-order vmcnt waits of stage() only ever wait for
        // the register set being staged, never for the set two tiles ahead.
        const int ptid = tid - 256;
        const int ss = ptid & 31, gq = ptid >> 5;
        const long long ldd = pb.ldd, ldfc = pb.ldfc, Nm1 = pb.N - 1;
        const long long nrows = (pb.P - p0) < MM_PIX ? (pb.P - p0) : MM_PIX;
        constexpr int ES = (int)sizeof(TS);
        const unsigned dbytes = __builtin_amdgcn_readfirstlane((unsigned)(nrows * ldd * ES));
        const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
            uniform_ptr(d_base<TS>(pb) + p0 * ldd), (short)0, (int)dbytes, 0x00020000);
        const int dvoff = (int)((4 * gq * ldd + ss) * ES);
        const int ldd16 = __builtin_amdgcn_readfirstlane((int)(ldd * ES));
        const TS *fcb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) fcb[r] = fc_base<TS>(pb) + (long long)fcl[4 * (gq + 8 * r)] * ldfc;
        // cos/sin tile: MM_TS rows × KH double2; this thread's slots e = ptid + 256 u, read
        // through a buffer descriptor (rows ≥ N read as 0; keeps the loads where they are issued
        // — plain loads of the read-only table would be sunk to their use past the barrier)
        // (MIX: the table is padded to whole tiles — the bf16 fragments live in rows 0..15)
        const long long trows = MIX ? (pb.N + MM_TS - 1) / MM_TS * MM_TS : pb.N;
        const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(
            uniform_ptr(tab), (short)0, __builtin_amdgcn_readfirstlane((int)(trows * KH * 16)),
            0x00020000);
        const int tvoff = ptid * 16;  // slot e = ptid + 256 u of a tile starting at row s0

        auto issue = [&](WsRegs<TS> &R, int it) __attribute__((always_inline)) {
            if constexpr (DBG == 2 || DBG == 5) {
                for (int r = 0; r < 4; ++r) {
                    R.f[r] = TS{1.0f + it, 0};
                    for (int j = 0; j < 4; ++j) R.d[r][j] = TS{0.5f * it, 1};
                }
                return;
            }
            it = it < ntiles ? it : ntiles - 1;
            const long long s0 = s_begin + (long long)it * MM_TS;
            const long long sl = (s0 + ss) < Nm1 ? (s0 + ss) : Nm1;
            const int s016 = (int)(s0 * ES);
            if constexpr (FAINT) R.st = gld(pb.state + sl);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if constexpr (POL == 2) {  // FC columns are read once per launch too
                    typedef double nv2d __attribute__((ext_vector_type(2)));
                    typedef float nv2f __attribute__((ext_vector_type(2)));
                    if constexpr (sizeof(TS) == 16)
                        R.f[r] = __builtin_bit_cast(TS, __builtin_nontemporal_load((const nv2d *)&fcb[r][sl]));
                    else
                        R.f[r] = __builtin_bit_cast(TS, __builtin_nontemporal_load((const nv2f *)&fcb[r][sl]));
                } else {
                    R.f[r] = gld(fcb[r] + sl);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if constexpr (UNIT) continue;
                    // all offset parts in voffset (the range check ignores soffset): rows
                    // beyond P and samples beyond the last row read as 0
                    R.d[r][j] = buf_ld<TS, POL>(drs, dvoff + (32 * r + j) * ldd16 + s016);
                }
            }
        };
        // cos/sin rows (L2-resident table) one tile ahead in a single register set
        double2 T0, T1, T2;
        auto issue_t = [&](int it) __attribute__((always_inline)) {
            if constexpr (DBG == 2 || DBG == 5) {
                T0 = T1 = T2 = double2{0.25 * it, 1.0};
                return;
            }
            it = it < ntiles ? it : ntiles - 1;
            const int vo = tvoff + (int)((s_begin + (long long)it * MM_TS) * KH * 16);
            T0 = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(trs, vo, 0, 0));
            T1 = __builtin_bit_cast(double2,
                                    __builtin_amdgcn_raw_buffer_load_b128(trs, vo + 4096, 0, 0));
            T2 = __builtin_bit_cast(double2,
                                    __builtin_amdgcn_raw_buffer_load_b128(trs, vo + 8192, 0, 0));
        };
        // masked: zero the q of samples outside the tile's state (FAINT) or past the chunk end
        auto stage_q = [&](const WsRegs<TS> &R, int it, auto gen, auto masked, bool sok) __attribute__((always_inline)) {
            const long long s = s_begin + (long long)it * MM_TS + ss;
            const long long sl = s < Nm1 ? s : Nm1;
            // mm_phys(4(gq + 8r) + j, ss) = q_base + 32r + j: the swizzle (bit 3 of the series)
            // only touches 4·gq's bits, so the 16 stores share one address and immediate offsets
            // (written per (r, j), the compiler kept an address register each — the faint variant
            // spilled them, and every spill reload waited for the tile prefetch: vmcnt(0))
            c64 *q_out = qs[it & 1] + (ss * MM_ROW + ((4 * gq) ^ ((ss & 1) << 3)));
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const c64 ph = unit_phasor(widen(R.f[r]));
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int pl = 4 * (gq + 8 * r) + j;
                    c64 pj = ph;
                    if (decltype(gen)::value)  // general layout: the series' own FC column
                        pj = unit_phasor(fc_at(pb, (long long)fcl[pl] * ldfc + sl));
                    const c64 dv = UNIT ? c64{1.0, 0.0} : widen(R.d[r][j]);
                    c64 q;
                    if constexpr (DBG == 8) {
                        q = dv;
                    } else {
                        q.re = fma(pj.re, dv.re, pj.im * dv.im);
                        q.im = fma(pj.re, dv.im, -(pj.im * dv.re));
                    }
                    if (decltype(masked)::value) {  // rows beyond P read as 0 already
                        q.re = sok ? q.re : 0.0;
                        q.im = sok ? q.im : 0.0;
                    }
                    q_out[32 * r + j] = q;
                }
            }
        };
        auto stage = [&](const WsRegs<TS> &R, int it, auto gen) __attribute__((always_inline)) {
            if (it >= ntiles) return;
            if constexpr (DBG == 5) return;
            const long long s = s_begin + (long long)it * MM_TS + ss;
            bool sok = s < s_end;
            // only a chunk's last tile can be partial (chunks are whole tiles, N may not be)
            bool whole = s_begin + (long long)(it + 1) * MM_TS <= s_end;  // uniform
            if constexpr (FAINT) {
                const int st = R.st;
                const bool v = sok && fst_valid(pb.flags, st);
                // lanes l and l + 32 hold the same sample: bits 0..31 are the tile's samples
                const unsigned b32 = (unsigned)__builtin_amdgcn_ballot_w64(v);
                const int ds = b32 ? __builtin_amdgcn_readlane(st, __builtin_ctz(b32)) : -1;
                sok = v && st == ds;
                const unsigned okm = (unsigned)__builtin_amdgcn_ballot_w64(sok);
                if (ptid == 0) {
                    tds[it & 1] = ds;
                    tmk[it & 1] = okm;
                }
                // every sample of the tile valid and of one state (most tiles of a faint
                // series: states change only at the few shutter switches) — nothing to mask
                whole = okm == 0xffffffffu;
            }
            if (whole || DBG == 10)  // (DBG 10: timing only, masks dropped)
                stage_q(R, it, gen, BoolTag<false>{}, sok);
            else
                stage_q(R, it, gen, BoolTag<true>{}, sok);
            double2 *tsb = (double2 *)ts[it & 1] + ptid;
            tsb[0] = T0;
            tsb[256] = T1;
            tsb[512] = T2;
        };

        // FAINT: compute_mean_var_power's statistics (src/Faint.jl:89-100) fused into this
        // pass.  While the consumers run tile i, the producers read tile i back from LDS with
        // one series per thread (series fs_p, sample half fs_h: waves 4-5 samples 0..15, waves
        // 6-7 samples 16..31; 16-B rows, conflict-free) and add x = |q| = |p̄ d| (= abs(d), |p| =
        // 1) of the tile's state-ds samples as shifted sums S1 = Σ(x − K), S2 = Σ(x − K)², K =
        // abs(d) at the first valid sample of that state (dhdr[2 + s], k_faint_defer) — the
        // same K for every partial of the series, so the partials add and the variance
        // M2 = S2 − S1²/n loses only ~(1 + (m − K)²/σ²) ulps (a raw Σx² − (Σx)²/n would lose
        // m²/σ²).  Flushed per (unit, state) exactly where the consumers flush their moments:
        // fsp[(slot·4 + 2·fs_h + {0, 1})·P + series], the counts (series-independent) by the
        // first series group: fcnt[slot].  k_faint_fused_fin merges them in unit order.
        const int fs_p = ptid & (MM_PIX - 1), fs_h = ptid >> 7;
        const long long fs_k = p0 + fs_p;
        if constexpr (FAINT) fsl[0][ptid] = fsl[1][ptid] = fsl[2][ptid] = 0.0;  // K, S1, S2
        int fs_cs = -1, fs_n = 0;
        unsigned fs_um = 0;
        auto fs_flush = [&](long long slot, bool add) __attribute__((always_inline)) {
            if (fs_k < pb.P) {
                double *o = fsp + (slot * 4 + 2 * fs_h) * pb.P + fs_k;
                const double s1 = fsl[1][ptid], s2 = fsl[2][ptid];
                o[0] = add ? o[0] + s1 : s1;
                o[pb.P] = add ? o[pb.P] + s2 : s2;
            }
            if (blockIdx.x == 0 && ptid == 0) fcnt[slot] = add ? fcnt[slot] + fs_n : fs_n;
            fsl[1][ptid] = fsl[2][ptid] = 0.0;
            fs_n = 0;
        };
        auto fs_tile = [&](int i) __attribute__((always_inline)) {
            if constexpr (FAINT && (DBG == 0 || DBG == 10)) {
                const int ds = __builtin_amdgcn_readfirstlane(tds[i & 1]);
                const unsigned mk = (unsigned)__builtin_amdgcn_readfirstlane((int)tmk[i & 1]);
                if (ds >= 0 && ds != fs_cs) {  // uniform
                    if (fs_cs >= 0) {
                        fs_flush((u_first + i / tpu) * FST_SLOTS + fs_cs, (fs_um >> fs_cs) & 1u);
                        fs_um |= 1u << fs_cs;
                    }
                    fs_cs = ds;
                    double K = 0.0;
                    if (fs_k < pb.P) {
                        const c64 z = d_at(pb, fs_k * pb.ldd + dhdr[2 + ds]);
                        K = jl_hypot(z.re, z.im);
                    }
                    fsl[0][ptid] = K;
                }
                if (ds >= 0) {
                    const double fsK = fsl[0][ptid];
                    double fsS1 = fsl[1][ptid], fsS2 = fsl[2][ptid];
                    fs_n += __builtin_popcount(mk);
                    const unsigned hm = (mk >> (16 * fs_h)) & 0xffffu;  // wave-uniform
                    const double2 *qt = (const double2 *)qs[i & 1];
                    if (hm == 0xffffu) {
#pragma unroll 1
                        for (int s4 = 0; s4 < 16; s4 += 4) {
                            double2 qv[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) qv[u] = qt[mm_phys(fs_p, 16 * fs_h + s4 + u)];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const double y = fs_abs(qv[u].x, qv[u].y) - fsK;
                                fsS1 += y;
                                fsS2 = fma(y, y, fsS2);
                            }
                        }
                    } else {
                        for (int s = 0; s < 16; ++s) {
                            if (!((hm >> s) & 1u)) continue;  // uniform
                            const double2 qv = qt[mm_phys(fs_p, 16 * fs_h + s)];
                            const double y = fs_abs(qv.x, qv.y) - fsK;
                            fsS1 += y;
                            fsS2 = fma(y, y, fsS2);
                        }
                    }
                    fsl[1][ptid] = fsS1;
                    fsl[2][ptid] = fsS2;
                }
                if ((i + 1) % tpu == 0 || i + 1 == ntiles) {  // unit end (uniform)
                    if (fs_cs >= 0) fs_flush((u_first + i / tpu) * FST_SLOTS + fs_cs, (fs_um >> fs_cs) & 1u);
                    fs_cs = -1;
                    fs_um = 0;
                }
            }
        };

        // loader waves first: their few VALU ops and the next loads must not queue behind the
        // MFMA stream of the consumer wave on the same SIMD (fp64 MFMA and VALU share it)
        __builtin_amdgcn_s_setprio(2);
        unsigned long long pst = 0, pis = 0, pbar = 0, tq = 0;
        auto tick = [&]() -> unsigned long long {
            if constexpr (DBG == 6) return __builtin_amdgcn_s_memtime();
            return 0;
        };
        auto run = [&](auto gen) __attribute__((always_inline)) {
            WsRegs<TS> R0, R1;
            issue(R0, 0);
            issue_t(0);
            issue(R1, 1);
            stage(R0, 0, gen);
            issue_t(1);
            issue(R0, 2);
            __syncthreads();
            // iteration i: stage tile i+1 (registers loaded two iterations ago), reload them
            // with tile i+3; unrolled by two so each register set is a fixed set of VGPRs, with
            // the odd last iteration peeled so the loop body has no conditional loads
            int i = 0;
            // (FAINT: between the barriers that publish tiles i and i+1 the consumers only read
            // buffer i&1, so the producers' statistics read it too — fs_tile(i))
            for (; i + 1 < ntiles; i += 2) {
                tq = tick();
                stage(R1, i + 1, gen);
                if constexpr (DBG == 6) { const auto t1 = tick(); pst += t1 - tq; tq = t1; }
                issue_t(i + 2);
                fs_tile(i);  // (R1's registers are free until their reload)
                issue(R1, i + 3);
                if constexpr (DBG == 6) { const auto t1 = tick(); pis += t1 - tq; tq = t1; }
                __syncthreads();
                if constexpr (DBG == 6) { const auto t1 = tick(); pbar += t1 - tq; tq = t1; }
                stage(R0, i + 2, gen);
                if constexpr (DBG == 6) { const auto t1 = tick(); pst += t1 - tq; tq = t1; }
                issue_t(i + 3);
                fs_tile(i + 1);
                issue(R0, i + 4);
                if constexpr (DBG == 6) { const auto t1 = tick(); pis += t1 - tq; tq = t1; }
                __syncthreads();
                if constexpr (DBG == 6) { const auto t1 = tick(); pbar += t1 - tq; tq = t1; }
            }
            if (i < ntiles) {
                stage(R1, i + 1, gen);
                fs_tile(i);
                __syncthreads();
            }
        };
        if (general)
            run(BoolTag<true>{});
        else
            run(BoolTag<false>{});
        if constexpr (DBG == 6) {
            if (lane == 0) {
                atomicAdd(&pb.prof[PROF_WS + 0], pst);
                atomicAdd(&pb.prof[PROF_WS + 1], pis);
                atomicAdd(&pb.prof[PROF_WS + 2], pbar);
            }
        }
        // the last iterations re-read the final tile; let those loads land before the wave
        // ends rather than leave them in flight past s_endpgm
        __builtin_amdgcn_s_waitcnt(0);
        return;
    }

    // ================================ consumer ================================
    const int fi = lane & 15, fk = lane >> 4, comp = fi & 1, ppair = fi >> 1;
    constexpr int NC = MIX ? 2 : 3;  // f64 column tiles (8 harmonics each)
    v4d acc[4][NC];
    v4f acc32[4];  // MIX: harmonics 17..24 (bf16 C/D layout: row 4·fk + r)
    double f0[4] = {0, 0, 0, 0}, q2[4] = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int n = 0; n < NC; ++n) acc[m][n] = (v4d){0.0, 0.0, 0.0, 0.0};
        acc32[m] = (v4f){0.0f, 0.0f, 0.0f, 0.0f};
    }
    // partial moments of one sample unit: write part[u], restart the accumulators
    auto put = [&](double *base, int m, int n, int row, int col, double v) {
        // moment index of output element (row, col) of column tile n: series row >> 1, re/im
        // of q row & 1, harmonic 8n + (col >> 1) + 1, cos/sin col & 1 → (A, B, C, D) code
        const long long pix = p0 + wave * 32 + m * 8 + (row >> 1);
        const int cq = row & 1, trig = col & 1;
        const int h = n * 8 + (col >> 1);
        const int code = cq == 0 ? (trig == 0 ? 0 : 3) : (trig == 1 ? 1 : 2);
        if (pix < pb.P) base[(long long)(3 + 4 * h + code) * pb.P + pix] = v;
    };
    // slot: the unit (FAINT: unit · FST_SLOTS + state); add: the slot already holds a partial
    // of this unit (FAINT, a state recurring within the unit) — same thread, same element
    auto flush = [&](long long slot, bool add) {
        double *base = part + slot * NMOM * pb.P;
        auto putv = [&](int m, int n, int row, int col, double v) {
            if (add) {
                const long long pix = p0 + wave * 32 + m * 8 + (row >> 1);
                const int cq = row & 1, trig = col & 1, h = n * 8 + (col >> 1);
                const int code = cq == 0 ? (trig == 0 ? 0 : 3) : (trig == 1 ? 1 : 2);
                if (pix < pb.P) v += base[(long long)(3 + 4 * h + code) * pb.P + pix];
            }
            put(base, m, n, row, col, v);
        };
#pragma unroll
        for (int m = 0; m < 4; ++m) {
#pragma unroll
            for (int n = 0; n < NC; ++n)
#pragma unroll
                for (int r = 0; r < 4; ++r) putv(m, n, fk + 4 * r, fi, acc[m][n][r]);  // f64 D map
            if constexpr (MIX) {
#pragma unroll
                for (int r = 0; r < 4; ++r) putv(m, 2, 4 * fk + r, fi, (double)acc32[m][r]);  // bf16 D map
            }
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            double f = f0[m], q = q2[m];
            f += __shfl_xor(f, 16, 64);
            f += __shfl_xor(f, 32, 64);
            q += __shfl_xor(q, 16, 64);
            q += __shfl_xor(q, 32, 64);
            const double qo = __shfl_xor(q, 1, 64);
            const long long pix = p0 + wave * 32 + m * 8 + ppair;
            if (fk == 0 && pix < pb.P) {
                double *bf = base + (long long)comp * pb.P + pix;
                *bf = add ? *bf + f : f;
                if (comp == 0) base[2 * pb.P + pix] = add ? base[2 * pb.P + pix] + (q + qo) : q + qo;
            }
            f0[m] = q2[m] = 0.0;
#pragma unroll
            for (int n = 0; n < NC; ++n) acc[m][n] = (v4d){0.0, 0.0, 0.0, 0.0};
            acc32[m] = (v4f){0.0f, 0.0f, 0.0f, 0.0f};
        }
    };
    __syncthreads();  // tile 0 staged
    unsigned long long cmf = 0, cbar = 0;  // DBG == 6 only
    int cs = -1;      // FAINT: state of the accumulators (-1: empty)
    unsigned um = 0;  // FAINT: state slots of the current unit written so far
    // fragments of K-step ks+1 are read from LDS while the MFMAs of K-step ks run
    // (register double buffer; only the first read of each tile waits on LDS latency)
    for (int i = 0; i < ntiles; ++i) {
        const double *qd = (const double *)qs[i & 1];
        const double *tb = ts[i & 1];
        bool live = true;  // FAINT: the tile holds a valid sample
        if constexpr (FAINT) {
            const int ds = __builtin_amdgcn_readfirstlane(tds[i & 1]);
            live = ds >= 0;
            if (live && ds != cs) {
                if (cs >= 0) {
                    flush((u_first + i / tpu) * FST_SLOTS + cs, (um >> cs) & 1u);
                    um |= 1u << cs;
                }
                cs = ds;
            }
        }
        auto ldfrag = [&](int ks, double (&a)[4], double (&b)[NC]) {
            const int k = ks * 4 + fk;
#pragma unroll
            for (int m = 0; m < 4; ++m) a[m] = qd[2 * mm_phys(wave * 32 + m * 8 + ppair, k) + comp];
#pragma unroll
            for (int n = 0; n < NC; ++n) b[n] = tb[k * 2 * KH + n * 16 + fi];
        };
        auto step = [&](const double (&a)[4], const double (&b)[NC]) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int n = 0; n < NC; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[n], acc[m][n], 0, 0, 0);
            if constexpr (DBG != 7) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    f0[m] += a[m];
                    q2[m] = fma(a[m], a[m], q2[m]);
                }
            }
        };
        unsigned long long c0 = 0;
        if constexpr (DBG == 6) c0 = __builtin_amdgcn_s_memtime();
        if (DBG != 1 && live) {
            // MIX: the bf16 B fragments of this tile (hi, lo), and the A fragments gathered
            // over the 8 K-steps — element j of lane l is sample fk + 4j, as in the table
            v4u bh, bl, ah[4], al[4];
            if constexpr (MIX) {
                const v4u *bf = (const v4u *)(tb + (lane >> 2) * (2 * KH) + 32 + 4 * (lane & 3));
                bh = bf[0];
                bl = bf[1];
            }
            float fe[4];
            double a0[4], b0[NC], a1[4], b1[NC];
            ldfrag(0, a0, b0);
#pragma unroll
            for (int ks = 0; ks < MM_TS / 4; ks += 2) {
                ldfrag(ks + 1, a1, b1);
                step(a0, b0);
                if constexpr (MIX) {
#pragma unroll
                    for (int m = 0; m < 4; ++m) fe[m] = (float)a0[m];
                }
                if (ks + 2 < MM_TS / 4) ldfrag(ks + 2, a0, b0);
                step(a1, b1);
                if constexpr (MIX) {
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        unsigned h, l;
                        split_bf16x2(fe[m], (float)a1[m], h, l);
                        ah[m][ks >> 1] = h;
                        al[m][ks >> 1] = l;
                    }
                }
            }
            if constexpr (MIX) {
                const bf16x8 Bh = __builtin_bit_cast(bf16x8, bh), Bl = __builtin_bit_cast(bf16x8, bl);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const bf16x8 Ah = __builtin_bit_cast(bf16x8, ah[m]);
                    acc32[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah, Bh, acc32[m], 0, 0, 0);
                    acc32[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah, Bl, acc32[m], 0, 0, 0);
                    acc32[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, al[m]), Bh, acc32[m], 0, 0, 0);
                }
            }
        }
        unsigned long long c1 = 0;
        if constexpr (DBG == 6) {
            // the MFMA results are consumed at the end; count issue time of the phase
            c1 = __builtin_amdgcn_s_memtime();
            cmf += c1 - c0;
        }
        __syncthreads();
        if constexpr (DBG == 6) cbar += __builtin_amdgcn_s_memtime() - c1;
        if ((i + 1) % tpu == 0 || i + 1 == ntiles) {  // uniform
            const long long u = u_first + i / tpu;
            if constexpr (FAINT) {
                if (cs >= 0) {
                    flush(u * FST_SLOTS + cs, (um >> cs) & 1u);
                    um |= 1u << cs;
                }
                if (tid == 0) smask[u] = um;  // the same value from every series group
                cs = -1;
                um = 0;
            } else {
                flush(u, false);
            }
        }
    }
    if constexpr (DBG == 6) {
        if (lane == 0) {
            atomicAdd(&pb.prof[PROF_WS + 3], cmf);
            atomicAdd(&pb.prof[PROF_WS + 4], cbar);
        }
    }
}
#else
;
#endif


// k_reduce_moments: mom[m][k] = Σ_chunk part[chunk][m][k] (fixed order), plus per-series
// aux[k] = {W2, DEN, Q2, 0}.  faint = 2 (state-split moments of k_moments_ws<FAINT>): the
// partial of unit c and state s is part[c·FST_SLOTS + s] (written where smask[c] has bit s),
// weighted here by f_s = w_s·m_s of compute_mean_var_power (f_s² for Σ|q|², row 2), units in
// order, states in order, then k_moments_fix's slots of the deferred samples (fixp, when dhdr
// counts any; dhdr[1] = their states).  faint = 1: the partials are weighted already.
__global__ __launch_bounds__(256) void k_reduce_moments(const double *__restrict__ part, int nch,
                                                        long long P, const Info *__restrict__ info,
                                                        const double *__restrict__ fstat, int faint,
                                                        double *__restrict__ mom,
                                                        double *__restrict__ aux,
                                                        const unsigned *__restrict__ smask = nullptr,
                                                        const double *__restrict__ fixp = nullptr,
                                                        const int *__restrict__ dhdr = nullptr)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
    const int m = blockIdx.y;
    if (k >= P) return;
    double s = 0.0;
    if (faint == 2) {
        double f[FST_SLOTS];
#pragma unroll
        for (int q = 0; q < FST_SLOTS; ++q) {
            f[q] = fstat[k * 16 + 6 + q] * fstat[k * 16 + 1 + q];  // w·m of state code q
            if (m == 2) f[q] *= f[q];
        }
        for (int c = 0; c < nch; ++c) {
            const unsigned um = smask[c];
#pragma unroll
            for (int q = 0; q < FST_SLOTS; ++q)
                if ((um >> q) & 1u) s += f[q] * part[(((long long)c * FST_SLOTS + q) * NMOM + m) * P + k];
        }
        if (dhdr[0] > 0) {
            const unsigned dm = (unsigned)dhdr[1];
#pragma unroll
            for (int q = 0; q < FST_SLOTS; ++q)
                if ((dm >> q) & 1u) s += f[q] * fixp[((long long)q * NMOM + m) * P + k];
        }
    } else {
        // 8 partials in flight per thread, then summed in chunk order (the same additions as
        // one load at a time, which waited out a full HBM round trip per chunk: 0.43 ms on C3)
        const double *pk = part + (long long)m * P + k;
        const long long cs = (long long)NMOM * P;
        int c = 0;
        for (; c + 8 <= nch; c += 8) {
            double v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = __builtin_nontemporal_load(pk + (c + j) * cs);
#pragma unroll
            for (int j = 0; j < 8; ++j) s += v[j];
        }
        for (; c < nch; ++c) s += __builtin_nontemporal_load(pk + c * cs);
    }
    mom[(long long)m * P + k] = s;
    if (m == 2) {
        if (faint) {
            aux[4 * k + 0] = fstat[k * 16 + 10];
            aux[4 * k + 1] = fstat[k * 16 + 11];
            aux[4 * k + 2] = fstat[k * 16 + 12];
        } else {
            aux[4 * k + 0] = s;                    // Σ|d|²
            aux[4 * k + 1] = (double)info->nvalid;  // Σ|p|² (|p| = 1)
            aux[4 * k + 2] = s;                    // Σ|q|² = Σ|d|²
        }
        aux[4 * k + 3] = (double)info->nvalid;  // N of the χ² (per series: windows)
    }
}
#else
;
#endif


// k_faint_fused_fin: compute_mean_var_power (src/Faint.jl:89-100) of every faint series from the
// moment pass's fused statistics — per state code s, in unit order, the counts fcnt and shifted
// sums fsp (S1, S2 of both sample halves) of the units whose slot s was written (smask), then
// the deferred samples' sums (fixs, k_moments_fix; when dhdr lists any of state s):
//   m = K + S1/n,   var = (S2 − S1·(S1/n)) / (n − 1),   w = 1/var,   K = abs(d) at dhdr[2 + s],
// and W2 = Σ_s w_s Σ|q|²_s, DEN = Σ_s w_s m_s² n_s, Q2 = Σ_s (w_s m_s)² Σ|q|²_s from the moment
// partials' row 2 (Σ|q|² = Σ|d|² per state) — the record k_faint_p1/p2/fin write (fstat[16k …]:
// m then w of TRANSIENT, OFF … HIGH; the TRANSIENT slot and states without samples NaN).
// One thread per series.
__global__ __launch_bounds__(256) void k_faint_fused_fin(Problem pb, int units,
                                                         const double *__restrict__ fsp,
                                                         const int *__restrict__ fcnt,
                                                         const unsigned *__restrict__ smask,
                                                         const double *__restrict__ part,
                                                         const double *__restrict__ fixs,
                                                         const double *__restrict__ fixp,
                                                         const int *__restrict__ dhdr,
                                                         double *__restrict__ fstat)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
    if (k >= pb.P) return;
    const long long P = pb.P;
    const int ndef = dhdr[0];
    const unsigned dm = (unsigned)dhdr[1];
    double *o = fstat + k * 16;
    const double nan = __builtin_nan("");
    o[0] = nan;  // TRANSIENT: never valid
    o[5] = nan;
    double W2 = 0.0, DEN = 0.0, Q2 = 0.0;
    for (int s = 0; s < FST_SLOTS; ++s) {
        double n = 0.0, S1 = 0.0, S2 = 0.0, D2 = 0.0;
        for (int u = 0; u < units; ++u) {
            if (!((smask[u] >> s) & 1u)) continue;
            const long long slot = (long long)u * FST_SLOTS + s;
            n += (double)fcnt[slot];
            S1 += fsp[(slot * 4 + 0) * P + k] + fsp[(slot * 4 + 2) * P + k];
            S2 += fsp[(slot * 4 + 1) * P + k] + fsp[(slot * 4 + 3) * P + k];
            D2 += part[(slot * NMOM + 2) * P + k];
        }
        if (ndef > 0 && ((dm >> s) & 1u)) {
            n += fixs[(long long)(3 * s + 0) * P + k];
            S1 += fixs[(long long)(3 * s + 1) * P + k];
            S2 += fixs[(long long)(3 * s + 2) * P + k];
            D2 += fixp[((long long)s * NMOM + 2) * P + k];
        }
        double m = nan, w = nan;
        if (n > 0) {
            const c64 z = d_at(pb, k * pb.ldd + dhdr[2 + s]);
            const double K = jl_hypot(z.re, z.im);
            m = K + S1 / n;
            w = 1.0 / ((S2 - S1 * (S1 / n)) / (n - 1.0));
            W2 += w * D2;
            DEN += w * m * m * n;
            Q2 += (w * m) * (w * m) * D2;
        }
        o[1 + s] = m;
        o[6 + s] = w;
    }
    o[10] = W2;
    o[11] = DEN;
    o[12] = Q2;
}
#else
;
#endif


// k_faint_defer: the samples the state-split moment pass leaves out — valid samples whose state
// differs from their 32-sample tile's (the state of its first valid sample) — as a list of
// (tile, sample bits) pairs in tile order: dlist[2e], dlist[2e + 1], e < dhdr[0]; dhdr[1] = the
// OR of 1 << state over them.  States depend on the sample only, so the list serves every series
// (and every shard: the order is that of the tiles).  dhdr[2 + s]: the first valid sample of
// state s (the shift of the fused faint statistics, k_moments_ws<FAINT>; 0 when the state has
// none).  Two launches over blocks of DEFER_TILES tiles, one sample per thread (r6; r4 had a
// thread walk each tile's 32 samples, blocks of 1024 tiles: 36 µs for C5's 3125 tiles):
// k_faint_defer_count writes each block's count / state mask / first samples into bsum[6b …],
// k_faint_defer_list writes the entries at the block's offset (the sum of the counts before it,
// summed by the block in parallel) in tile order, and its block 0 the header.
constexpr int DEFER_TILES = 8;  // 32-sample tiles per 256-thread block
static_assert(MM_TS == 32, "k_faint_defer: a tile is a half-wave of 32 lanes");
struct DeferLane {
    unsigned dm;    // this tile's deferred-sample bits (same on the tile's 32 lanes)
    unsigned sm;    // OR of 1 << state over them
    int first[FST_SLOTS];  // the tile's first valid sample of each state (INT_MAX if none)
};
// The per-tile masks of the 32-lane half-wave holding tile j = sample i >> 5 (lane s = i & 31).
__device__ __forceinline__ DeferLane defer_lane(const Problem &pb, long long i) {
    const int lane = (int)threadIdx.x & 63, sh = lane & 32;
    int st = -1;
    if (i < pb.N) st = (int)(signed char)pb.state[i];
    const bool v = i < pb.N && fst_valid(pb.flags, st);
    const unsigned hv = (unsigned)(__ballot(v) >> sh);
    const int f = hv ? __builtin_ctz(hv) : 0;
    const int ds = __shfl(st, sh + f, 64);
    const bool diff = v && st != ds;
    DeferLane r;
    r.dm = (unsigned)(__ballot(diff) >> sh);
    r.sm = 0;
    const long long j0 = (i >> 5) << 5;
#pragma unroll
    for (int q = 0; q < FST_SLOTS; ++q) {
        const unsigned mq = (unsigned)(__ballot(v && st == q) >> sh);
        r.first[q] = mq ? (int)(j0 + __builtin_ctz(mq)) : 0x7fffffff;
        if ((unsigned)(__ballot(diff && st == q) >> sh)) r.sm |= 1u << q;
    }
    return r;
}

__global__ __launch_bounds__(256) void k_faint_defer_count(Problem pb, int *__restrict__ bsum)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ int tcnt[DEFER_TILES];
    __shared__ unsigned tsm[DEFER_TILES];
    __shared__ int tfirst[DEFER_TILES][FST_SLOTS];
    const int tid = threadIdx.x, t = tid >> 5;
    const DeferLane r = defer_lane(pb, (long long)blockIdx.x * 256 + tid);
    if ((tid & 31) == 0) {
        tcnt[t] = r.dm != 0;
        tsm[t] = r.sm;
        for (int q = 0; q < FST_SLOTS; ++q) tfirst[t][q] = r.first[q];
    }
    __syncthreads();
    if (tid == 0) {
        int c = 0;
        unsigned sm = 0;
        int first[FST_SLOTS] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
        for (int u = 0; u < DEFER_TILES; ++u) {
            c += tcnt[u];
            sm |= tsm[u];
            for (int q = 0; q < FST_SLOTS; ++q) first[q] = min(first[q], tfirst[u][q]);
        }
        int *o = bsum + 6 * blockIdx.x;
        o[0] = c;
        o[1] = (int)sm;
        for (int q = 0; q < FST_SLOTS; ++q) o[2 + q] = first[q];
    }
}
#else
;
#endif

__global__ __launch_bounds__(256) void k_faint_defer_list(Problem pb, const int *__restrict__ bsum,
                                                          int *__restrict__ dlist,
                                                          int *__restrict__ dhdr)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ int wsum[4];
    __shared__ unsigned tdm[DEFER_TILES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, t = tid >> 5;
    const long long i = (long long)blockIdx.x * 256 + tid;
    // the block's offset: the counts of the blocks before it, summed by the whole block
    int part = 0;
    for (unsigned q = tid; q < blockIdx.x; q += 256) part += bsum[6 * q];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o, 64);
    if (lane == 0) wsum[wave] = part;
    if (blockIdx.x == 0) {  // the header: totals over every block
        int tot = 0;
        unsigned sm = 0;
        int first[FST_SLOTS] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
        for (unsigned q = tid; q < gridDim.x; q += 256) {
            tot += bsum[6 * q];
            sm |= (unsigned)bsum[6 * q + 1];
            for (int s = 0; s < FST_SLOTS; ++s) first[s] = min(first[s], bsum[6 * q + 2 + s]);
        }
        __shared__ int htot[4];
        __shared__ unsigned hsm[4];
        __shared__ int hfirst[4][FST_SLOTS];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            tot += __shfl_xor(tot, o, 64);
            sm |= (unsigned)__shfl_xor((int)sm, o, 64);
            for (int s = 0; s < FST_SLOTS; ++s) first[s] = min(first[s], __shfl_xor(first[s], o, 64));
        }
        if (lane == 0) {
            htot[wave] = tot;
            hsm[wave] = sm;
            for (int s = 0; s < FST_SLOTS; ++s) hfirst[wave][s] = first[s];
        }
        __syncthreads();
        if (tid == 0) {
            int T = 0;
            unsigned M = 0;
            int F[FST_SLOTS] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
            for (int w = 0; w < 4; ++w) {
                T += htot[w];
                M |= hsm[w];
                for (int s = 0; s < FST_SLOTS; ++s) F[s] = min(F[s], hfirst[w][s]);
            }
            dhdr[0] = T;
            dhdr[1] = (int)M;
            for (int s = 0; s < FST_SLOTS; ++s) dhdr[2 + s] = F[s] == 0x7fffffff ? 0 : F[s];
        }
    }
    const DeferLane r = defer_lane(pb, i);
    if ((tid & 31) == 0) tdm[t] = r.dm;
    __syncthreads();
    if ((tid & 31) == 0 && r.dm) {
        int off = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        for (int u = 0; u < t; ++u) off += tdm[u] != 0;
        dlist[2 * off] = (int)(i >> 5);
        dlist[2 * off + 1] = (int)r.dm;
    }
}
#else
;
#endif


// k_fix_table: cos/sin n x (n = 1..KH, k_table's recurrence) of every sample k_faint_defer
// lists, once for all series: ftab[(e·32 + sl)·2KH + …] for entry e, sample bit sl.  Launched over
// every possible entry (⌈N/32⌉·32 threads); threads beyond the list return.
__global__ __launch_bounds__(256) void k_fix_table(Problem pb, const int *__restrict__ dlist,
                                                   const int *__restrict__ dhdr,
                                                   double *__restrict__ ftab)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long e = g / MM_TS;
    const int sl = (int)(g % MM_TS);
    if (e >= dhdr[0]) return;
    if (!(((unsigned)dlist[2 * e + 1] >> sl) & 1u)) return;
    const long long i = (long long)dlist[2 * e] * MM_TS + sl;
    double s1, c1;
    jl_sincos(pb.omega * gld(pb.t + i), &s1, &c1);
    double cn = c1, sn = s1;
    double *row = ftab + g * (2 * KH);
    for (int n = 1; n <= KH; ++n) {
        row[2 * (n - 1)] = cn;
        row[2 * (n - 1) + 1] = sn;
        const double cn1 = cn * c1 - sn * s1;
        const double sn1 = sn * c1 + cn * s1;
        cn = cn1;
        sn = sn1;
    }
}
#else
;
#endif


// k_moments_fix: the unweighted moments q = p̄ d of the samples k_faint_defer lists, per state:
// fixp[(q·NMOM + row)·P + k], the rows of k_moments_ws (Σq, Σ|q|², then A, B, C, D per
// harmonic; every state of dhdr[1] written, nothing when the list is empty).  One workgroup
// per (series, state) (grid P × FST_SLOTS; with an empty list or a state without deferred
// samples they return at once); thread = (harmonic group hg of 3 harmonics, sample lane sl of 32); lane sl takes
// sample sl of each listed tile in list order (cos/sin n x from k_fix_table; entries in batches
// of 4), the lanes are reduced by a fixed xor tree.
__global__ __launch_bounds__(256) void k_moments_fix(Problem pb, const int *__restrict__ dlist,
                                                     const int *__restrict__ dhdr,
                                                     const double *__restrict__ ftab,
                                                     double *__restrict__ fixp,
                                                     double *__restrict__ fixs = nullptr)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const int cnt = dhdr[0];
    if (cnt == 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hg = wave * 2 + (lane >> 5), sl = lane & 31;
    const unsigned smk = (unsigned)dhdr[1];
    const long long k = blockIdx.x;  // one workgroup per (series, state)
    const int q = blockIdx.y;
    if (!((smk >> q) & 1u)) return;
    {
        const long long doff = k * pb.ldd, foff = (long long)pb.fcop[k] * pb.ldfc;
        double acc[12], f0r = 0.0, f0i = 0.0, w2 = 0.0;
        double sn = 0.0, s1 = 0.0, s2 = 0.0, K = 0.0;  // fixs: the fused statistics' sums
        if (fixs) {
            const c64 z = d_at(pb, doff + dhdr[2 + q]);
            K = jl_hypot(z.re, z.im);
        }
#pragma unroll
        for (int c = 0; c < 12; ++c) acc[c] = 0.0;
        // entries in batches of 4 with every load issued up front (a list walk one entry at a
        // time is a chain of dependent loads per entry); the same order of the sums
        constexpr int EB = 4;
        for (int e0 = 0; e0 < cnt; e0 += EB) {
            long long ii[EB];
            bool ok[EB];
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                const int e = e0 + u;
                const unsigned dm = e < cnt ? (unsigned)dlist[2 * e + 1] : 0u;
                ok[u] = (dm >> sl) & 1u;
                ii[u] = ok[u] ? (long long)dlist[2 * e] * MM_TS + sl : 0;
            }
            c64 fv[EB], dvv[EB];
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                ok[u] = ok[u] && gld(pb.state + ii[u]) == q;
                fv[u] = fc_at(pb, foff + ii[u]);
                dvv[u] = d_at(pb, doff + ii[u]);
            }
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                if (!ok[u]) continue;
                const c64 ph = unit_phasor(fv[u]);
                const c64 dv = dvv[u];
                const double qr = fma(ph.re, dv.re, ph.im * dv.im);
                const double qi = fma(ph.re, dv.im, -(ph.im * dv.re));
                const double *row = ftab + ((long long)(e0 + u) * MM_TS + sl) * (2 * KH) + 6 * hg;
#pragma unroll
                for (int h = 0; h < 3; ++h) {
                    const double cn = row[2 * h], sn = row[2 * h + 1];
                    acc[4 * h + 0] = fma(qr, cn, acc[4 * h + 0]);
                    acc[4 * h + 1] = fma(qi, sn, acc[4 * h + 1]);
                    acc[4 * h + 2] = fma(qi, cn, acc[4 * h + 2]);
                    acc[4 * h + 3] = fma(qr, sn, acc[4 * h + 3]);
                }
                f0r += qr;
                f0i += qi;
                w2 = fma(qr, qr, fma(qi, qi, w2));
                const double y = fs_abs(qr, qi) - K;
                sn += 1.0;
                s1 += y;
                s2 = fma(y, y, s2);
            }
        }
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) {
#pragma unroll
            for (int c = 0; c < 12; ++c) acc[c] += __shfl_xor(acc[c], off, 64);
            f0r += __shfl_xor(f0r, off, 64);
            f0i += __shfl_xor(f0i, off, 64);
            w2 += __shfl_xor(w2, off, 64);
            if (fixs && hg == 0) {
                sn += __shfl_xor(sn, off, 64);
                s1 += __shfl_xor(s1, off, 64);
                s2 += __shfl_xor(s2, off, 64);
            }
        }
        if (fixs && hg == 0 && sl == 0) {
            double *o = fixs + (long long)q * 3 * pb.P + k;
            o[0] = sn;
            o[pb.P] = s1;
            o[2 * pb.P] = s2;
        }
        if (sl == 0) {
            double *o = fixp + (long long)q * NMOM * pb.P + k;
#pragma unroll
            for (int h = 0; h < 3; ++h)
#pragma unroll
                for (int c = 0; c < 4; ++c) o[(long long)(3 + 4 * (3 * hg + h) + c) * pb.P] = acc[4 * h + c];
            if (hg == 0) {
                o[0] = f0r;
                o[pb.P] = f0i;
                o[2 * pb.P] = w2;
            }
        }
    }
}
#else
;
#endif


// Harmonic moments of windowed series (short spans, ≤ ~10k samples): one 256-thread workgroup
// per (window, column) series; thread = (harmonic group hg of 3 harmonics, sample lane sl of
// 32), samples sl, sl+32, … of the span; lanes reduced by a fixed xor tree, groups write
// their own rows.  Writes mom[m][k] and aux[k] = {Σw|d|², Σw|p|², Σ|q|², N_valid} directly.
template <bool FAINT>
__global__ __launch_bounds__(256) void k_moments_win(Problem pb, const double *__restrict__ tab,
                                                     const double *__restrict__ fstat,
                                                     double *__restrict__ mom,
                                                     double *__restrict__ aux)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long k = blockIdx.x;
    const Span sp = span_of(pb, k);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hg = wave * 2 + (lane >> 5), sl = lane & 31;  // hg 0..7 → harmonics 3hg+1..3hg+3
    const long long doff = sp.col * pb.ldd, foff = (long long)pb.fcop[sp.col] * pb.ldfc;
    double wm[5] = {0, 0, 0, 0, 0};
    if (FAINT) {
#pragma unroll
        for (int q = 0; q < 5; ++q) wm[q] = fstat[k * 16 + 5 + q] * fstat[k * 16 + q];
    }
    double acc[12], f0r = 0.0, f0i = 0.0, w2 = 0.0, cnt = 0.0;
#pragma unroll
    for (int q = 0; q < 12; ++q) acc[q] = 0.0;
    for (long long i = sp.s0 + sl; i < sp.s1; i += 32) {
        int st = 0;
        if (FAINT && !sample_valid(pb, i, st)) continue;
        const c64 ph = unit_phasor(fc_at(pb, foff + i));
        const c64 dv = d_at(pb, doff + i);
        double qr = fma(ph.re, dv.re, ph.im * dv.im);  // q = w m p̄ d
        double qi = fma(ph.re, dv.im, -(ph.im * dv.re));
        if (FAINT) {
            double f = wm[0];
#pragma unroll
            for (int q = 1; q < 5; ++q) f = (st + 1 == q) ? wm[q] : f;
            qr *= f;
            qi *= f;
        }
        const double *row = tab + i * (2 * KH) + 6 * hg;
#pragma unroll
        for (int h = 0; h < 3; ++h) {
            const double c = row[2 * h], sn = row[2 * h + 1];
            acc[4 * h + 0] = fma(qr, c, acc[4 * h + 0]);
            acc[4 * h + 1] = fma(qi, sn, acc[4 * h + 1]);
            acc[4 * h + 2] = fma(qi, c, acc[4 * h + 2]);
            acc[4 * h + 3] = fma(qr, sn, acc[4 * h + 3]);
        }
        if (hg == 0) {
            f0r += qr;
            f0i += qi;
            w2 = fma(dv.re, dv.re, fma(dv.im, dv.im, w2));
            cnt += 1.0;
        }
    }
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) {
#pragma unroll
        for (int q = 0; q < 12; ++q) acc[q] += __shfl_xor(acc[q], off, 64);
        f0r += __shfl_xor(f0r, off, 64);
        f0i += __shfl_xor(f0i, off, 64);
        w2 += __shfl_xor(w2, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
    }
    if (sl == 0) {
#pragma unroll
        for (int h = 0; h < 3; ++h)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                mom[(long long)(3 + 4 * (3 * hg + h) + c) * pb.P + k] = acc[4 * h + c];
        if (hg == 0) {
            mom[0 * pb.P + k] = f0r;
            mom[1 * pb.P + k] = f0i;
            mom[2 * pb.P + k] = FAINT ? 0.0 : w2;
            if (FAINT) {
                aux[4 * k + 0] = fstat[k * 16 + 10];
                aux[4 * k + 1] = fstat[k * 16 + 11];
                aux[4 * k + 2] = fstat[k * 16 + 12];
            } else {
                aux[4 * k + 0] = w2;
                aux[4 * k + 1] = cnt;
                aux[4 * k + 2] = w2;
            }
            aux[4 * k + 3] = cnt;
        }
    }
}
#else
;
#endif


// Where the moments of the series are read (r5).  HarmG: the moment array in global memory,
// row q of column col at p[q·ld + col] (through a global-address-space pointer: a generic one
// makes every wait drain all outstanding loads).  HarmL: the series' 99 rows copied once into
// LDS by the fit (k_fit_harmonic<LPS, true>), row q at p[q] — an evaluation then waits ~100
// cycles per batch of reads instead of an L2 round trip (the global form's loads arrive in 5
// dependent batches per evaluation, 3-5 k cycles of the objective's time).
struct HarmG {
    typedef const __attribute__((address_space(1))) double gdouble;
    const double *p;
    long long ld, col;
    __device__ __forceinline__ double operator[](int q) const {
        return ((gdouble *)p)[(long long)q * ld + col];
    }
};
struct HarmL {
    const __attribute__((address_space(3))) double *p;
    __device__ __forceinline__ double operator[](int q) const { return p[q]; }
};
constexpr int HARM_ROWS = 3 + 4 * KH;  // rows of a series' moments (F0 re/im, Q2, (A,B,C,D)_n)

// Σ_n J_n(b) e^{-jnϕ} M_n for moments M in the layout of k_moments (F0 re/im at rows 0-1,
// (A,B,C,D)_n at rows 3+4(n-1)..), canonical order (above), by the L lanes of a group (L = 1:
// one lane alone; r: the lane's index in its group)
template <int L, class M>
__device__ __forceinline__ void harm_combine(const M &m, int r, const double (&J)[KH + 2],
                                             double cph, double sph, double &Sr, double &Si) {
    constexpr int NS = 8 / L;
    double c[9], s[9];
    c[1] = cph;
    s[1] = sph;
#pragma unroll
    for (int q = 2; q <= 8; ++q) {
        c[q] = c[q - 1] * cph - s[q - 1] * sph;
        s[q] = s[q - 1] * cph + c[q - 1] * sph;
    }
    const double c8 = c[8], s8 = s[8];
    double vr[NS], vi[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        // slot j's angle components and Bessel factors: compile-time for L = 1; for L > 1
        // the slot depends on the lane — captured by compare-and-select against every
        // candidate (no register array indexed at run time, which would go through scratch)
        int mi;
        double cn, sn, jq[3];
        if constexpr (L == 1) {
            mi = j + 1;
            cn = c[mi];
            sn = s[mi];
#pragma unroll
            for (int q = 0; q < 3; ++q) jq[q] = J[mi + 8 * q];
        } else {
            mi = r + L * j + 1;
            cn = c[1];
            sn = s[1];
#pragma unroll
            for (int q = 0; q < 3; ++q) jq[q] = J[1 + 8 * q];
#pragma unroll
            for (int mm = 2; mm <= 8; ++mm) {
                const bool hit = mi == mm;
                cn = hit ? c[mm] : cn;
                sn = hit ? s[mm] : sn;
#pragma unroll
                for (int q = 0; q < 3; ++q) jq[q] = hit ? J[mm + 8 * q] : jq[q];
            }
        }
        // odd n: the even form with (A', B', C', D') = (B, A, −D, −C) gives fma(B, cn, C sn)
        // and −fma(D, cn, A sn), bit for bit (negation and ×(±1) are exact)
        const bool odd = (mi & 1) != 0;
        const int oA = odd ? 1 : 0, oB = odd ? 0 : 1, oC = odd ? 3 : 2, oD = odd ? 2 : 3;
        const double sg = odd ? -1.0 : 1.0;
        double pr = 0.0, pi = 0.0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int n = mi + 8 * q;
            if (q > 0) {
                const double c2 = cn * c8 - sn * s8;
                const double s2 = sn * c8 + cn * s8;
                cn = c2;
                sn = s2;
            }
            const int rw = 3 + 4 * (n - 1);
            const double A = m[rw + oA], B = m[rw + oB];
            const double C = sg * m[rw + oC], D = sg * m[rw + oD];
            const double tr = fma(A, cn, -(D * sn));
            const double ti = fma(C, cn, -(B * sn));
            const double j2 = 2.0 * jq[q];
            if (q == 0) {
                pr = j2 * tr;
                pi = j2 * ti;
            } else {
                pr = fma(j2, tr, pr);
                pi = fma(j2, ti, pi);
            }
        }
        vr[j] = pr;
        vi[j] = pi;
    }
    // the butterfly over the 8 slots: distance 4, 2, 1 (in-lane while the distance spans
    // this lane's slots, then across the group's lanes)
    if constexpr (L <= 4) {
#pragma unroll
        for (int j = 0; j < 4 / L; ++j) {
            vr[j] = vr[j] + vr[j + 4 / L];
            vi[j] = vi[j] + vi[j + 4 / L];
        }
    } else {
        vr[0] = vr[0] + lane_xor<4>(vr[0]);
        vi[0] = vi[0] + lane_xor<4>(vi[0]);
    }
    if constexpr (L <= 2) {
#pragma unroll
        for (int j = 0; j < 2 / L; ++j) {
            vr[j] = vr[j] + vr[j + 2 / L];
            vi[j] = vi[j] + vi[j + 2 / L];
        }
    } else {
        vr[0] = vr[0] + lane_xor<2>(vr[0]);
        vi[0] = vi[0] + lane_xor<2>(vi[0]);
    }
    if constexpr (L == 1) {
        vr[0] = vr[0] + vr[1];
        vi[0] = vi[0] + vi[1];
    } else {
        vr[0] = vr[0] + lane_xor<1>(vr[0]);
        vi[0] = vi[0] + lane_xor<1>(vi[0]);
    }
    Sr = J[0] * m[0] + vr[0];
    Si = J[0] * m[1] + vi[0];
}

// The objective's heavy part, out of line (one copy per (L, source) whatever NEWUOA's call sites)
// with everything it reads passed by value: the Bessel factors, the safe-range checks, sin/cos
// of the phase and the sums S = Σ w m̄ d (and G = Σ w m̄ for fitoffsets).  bad: the truncated
// expansion is not exact at this point (→ exact evaluator).
struct HarmS {
    double Sr, Si, Gr, Gi;
    int bad;
};
// (OFFS a template parameter: the second combine in the same body raises the one-lane form's
// registers past 256 — spills in every evaluation of C3's fit)
template <int L, class M, bool OFFS>
__device__ __attribute__((noinline)) HarmS harm_core(double b, double phi, M m, M mg, int r,
                                                     double tailref, double qbase, double phimax) {
    HarmS o;
    o.Sr = o.Si = o.Gr = o.Gi = 0.0;
    o.bad = 0;
    double J[KH + 2];
    bessel_j<KH + 1>(b, J);
    if (!(fabs(b) < 0.45 * KH) || fabs(J[KH + 1]) > tailref) {
        o.bad = 1;
        return o;
    }
    if (qbase != 0.0) {
        if (!(fabs(phi) <= phimax)) {  // fl(x + ϕ) may leave the binade: exact evaluator
            o.bad = 1;
            return o;
        }
        phi = (qbase + phi) - qbase;  // θ = fl(x + ϕ) = x + ϕ_q (one binade)
    }
    double sph, cph;
    jl_sincos(phi, &sph, &cph);
    harm_combine<L>(m, r, J, cph, sph, o.Sr, o.Si);
    if constexpr (OFFS) harm_combine<L>(mg, r, J, cph, sph, o.Gr, o.Gi);  // Gm = Σ w m̄ = Σ w p̄ e^{-jβ}
    else (void)mg;
    return o;
}

// χ²(b,ϕ) from the moments of one series, evaluated by a group of LPS consecutive lanes of a
// wave (LPS ∈ {1, 2, 4, 8}; sub-lane r = lane mod LPS).  The arithmetic is canonical — the
// same operations in the same order whatever LPS is (r5), so that the records do not depend on
// how many lanes a series gets (the engine picks LPS from the batch size):
//   S(b,ϕ) = J_0·F_0 + T,  T = Σ_{n=1..24} 2J_n·t_n(ϕ) summed as 8 slot partials — slot s holds
//   n = s+1, s+9, s+17 (in that order, the first product then two fmas) — combined by the xor
//   butterfly over the slots at distances 4, 2, 1 (each level: lower slot + upper slot, so both
//   partners hold the same bits); e^{-jnϕ}'s components by angle addition: (c_m, s_m) for
//   m = 1..8 from (cos ϕ, sin ϕ), then n = m + 8q by q rotations through (c_8, s_8).
// Lane r of the group holds slots r, r + LPS, …: with LPS = 8 every level of the butterfly is a
// cross-lane exchange, with LPS = 1 every level is in-lane.  (Before r5: one lane per series, the
// 24 harmonics in one sequential recurrence and fma chain — a different rounding of the same
// sum, within the harmonic evaluator's stated χ² error.)
// M: where the moments are read (HarmG / HarmL above); the functor itself is inlined into the
// fit, so its fields stay in registers.
template <int LPS, class M = HarmG>
struct HarmChi2 {
    static_assert(LPS == 1 || LPS == 2 || LPS == 4 || LPS == 8, "lanes per series");
    static constexpr bool kMulti = LPS > 1;  // independent points in parallel (has_multi)
    M src, srcG;  // the series' moments; fitoffsets: those of its FC phasor (momG)
    double nvalid, W2, DEN, tailref, qbase, phimax;
    double a_re, a_im;
    int nfev;
    int r;  // sub-lane of the group (0 for LPS = 1)
    bool fallback;
    // fitoffsets (ModulationWithOffsets, src/Modulation.jl:174-192): Σw and Σw d
    bool offs;
    double W0, D0r, D0i, c_re, c_im;

    unsigned long long prof_cycles, prof_wave;  // lane-level / wave-level (first active lane)
    bool prof;

    __device__ __forceinline__ double operator()(const double (&x)[2]) {
        // the cycle split brackets the evaluation
        const unsigned long long t0 = prof ? __builtin_amdgcn_s_memtime() : 0;
        const double v = eval<LPS>(x);
        if (prof) {
            const unsigned long long dt = __builtin_amdgcn_s_memtime() - t0;
            prof_cycles += dt;
            if ((int)threadIdx.x == __builtin_amdgcn_readfirstlane((int)threadIdx.x)) prof_wave += dt;
        }
        return v;
    }
    // the same χ² evaluated by this lane alone (LPS = 1 form of the canonical arithmetic)
    __device__ __forceinline__ double single(const double (&x)[2]) { return eval<1>(x); }
    // NP independent points: lane r of the group evaluates points r, r + LPS, … alone; every
    // lane then holds every value (shuffled from its owner), nfev counts NP evaluations and a
    // fallback anywhere in the group is the group's
    template <int NP>
    __device__ __forceinline__ void multi(const double (&pts)[NP][2], double (&vals)[NP]) {
        constexpr int R = (NP + LPS - 1) / LPS;
        const int nf0 = nfev;
        double mine[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int pi = q * LPS + r;
            mine[q] = 0.0;
            if (pi < NP) {
                double xx[2] = {pts[q * LPS][0], pts[q * LPS][1]};
#pragma unroll
                for (int u = 1; u < LPS; ++u) {
                    if (q * LPS + u < NP) {
                        const bool hit = r == u;
                        xx[0] = hit ? pts[q * LPS + u][0] : xx[0];
                        xx[1] = hit ? pts[q * LPS + u][1] : xx[1];
                    }
                }
                mine[q] = single(xx);
            }
        }
        const int base = ((int)threadIdx.x & 63) & ~(LPS - 1);
#pragma unroll
        for (int p = 0; p < NP; ++p) vals[p] = __shfl(mine[p / LPS], base + p % LPS, 64);
        const unsigned long long bal = __ballot(fallback);
        fallback = ((bal >> base) & ((1ull << LPS) - 1)) != 0;
        nfev = nf0 + NP;
    }
    template <int LPS_ = LPS>
    __device__ __forceinline__ double eval(const double (&x)[2]) {
        ++nfev;
        if (fallback) return 0.0;
        const HarmS h = offs ? harm_core<LPS_, M, true>(x[0], x[1], src, srcG, r, tailref, qbase, phimax)
                             : harm_core<LPS_, M, false>(x[0], x[1], src, srcG, r, tailref, qbase, phimax);
        if (h.bad) {
            fallback = true;  // truncated expansion not exact here → exact evaluator
            return 0.0;
        }
        const double Sr = h.Sr, Si = h.Si;  // S = Σ w m̄ d
        if (offs) {
            // [Σw  Σw m; Σw m̄  Σw|m|²] [c; a] = [Σw d; Σw m̄ d], StaticArrays 2×2 solve as in the
            // exact evaluator; Nχ² = Σw|d|² − Re(c̄ Σw d + ā S) at the solution
            const double Gr = h.Gr, Gi = h.Gi;
            const c64 A11 = {W0, 0.0}, A12 = {Gr, -Gi}, A21 = {Gr, Gi}, A22 = {DEN, 0.0};
            const c64 b1 = {D0r, D0i}, b2 = {Sr, Si};
            const c64 t1 = cmul(A11, A22), t2 = cmul(A12, A21);
            const c64 det = {t1.re - t2.re, t1.im - t2.im};
            const c64 u1 = cmul(A22, b1), u2 = cmul(A12, b2);
            const c64 v1 = cmul(A11, b2), v2 = cmul(A21, b1);
            const c64 cc = cdiv(c64{u1.re - u2.re, u1.im - u2.im}, det);
            const c64 aa = cdiv(c64{v1.re - v2.re, v1.im - v2.im}, det);
            c_re = cc.re;
            c_im = cc.im;
            a_re = aa.re;
            a_im = aa.im;
            const double proj = (cc.re * D0r + cc.im * D0i) + (aa.re * Sr + aa.im * Si);
            return (W2 - proj) / nvalid;
        }
        a_re = Sr / DEN;  // a = Σ w m̄ d / Σ w|m|²  (src/Modulation.jl:144)
        a_im = Si / DEN;
        const double chi2n = W2 - (Sr * Sr + Si * Si) / DEN;
        return chi2n / nvalid;
    }
};

// k_fit_harmonic: lane = series.  Series whose NEWUOA probes leave the expansion's safe
// range are appended to `list` for the exact evaluator.
// Offsets fields of the objective (fitoffsets, non-faint): Σw and Σ d of the series (the G
// moments of its FC column are the caller's srcG).
template <class F>
__device__ __forceinline__ void harm_offsets(F &f, const Problem &pb, long long k,
                                             const double *__restrict__ d0) {
    f.offs = (pb.flags & F_OFFSETS) != 0;
    f.c_re = f.c_im = 0.0;
    if (!f.offs) return;
    f.W0 = f.nvalid;  // Σ w (w ≡ 1)
    f.D0r = d0[2 * k];
    f.D0i = d0[2 * k + 1];
}

// k_fit_harmonic<LPS, MC>: a group of LPS lanes per series (the canonical objective above and
// NEWUOA's trial-angle searches split across the group; NEWUOA itself runs replicated on the
// group's lanes, its state shared in LDS), pb.fit_lanes series per wave, blockDim.x / 64 waves
// per workgroup (a workgroup's waves are placed on different SIMDs of one CU).  Dynamic LDS:
// one NEWUOA state (71 doubles, odd 8-byte stride) per series of the workgroup, then with MC the
// series' moments (HARM_ROWS doubles per series, odd stride; fitoffsets: then those of their FC
// columns), copied in by the group's lanes before the fit — the objective reads them there
// (HarmL).  Series whose NEWUOA probes leave the expansion's safe range are appended to `list`
// for the exact evaluator.
#ifndef GPD_FIT_MINW
#define GPD_FIT_MINW 1  // A/B builds: -DGPD_FIT_MINW=2 (two fit waves per SIMD, 256 registers)
#endif
template <int LPS, bool MC>
__global__ __launch_bounds__(256, GPD_FIT_MINW) void k_fit_harmonic(Problem pb, const Info *__restrict__ info,
                                                         const double *__restrict__ mom,
                                                         const double *__restrict__ aux,
                                                         const double *__restrict__ momG, long long PG,
                                                         const double *__restrict__ d0,
                                                         Param *__restrict__ out, double *__restrict__ raw,
                                                         int *__restrict__ list, int *__restrict__ count)
#if GPD_OWNS(GPD_U_FITH)
{
    typedef Newuoa<2, 5, true, LPS> NW;
    typedef __attribute__((address_space(3))) double ldouble;
    typedef typename std::conditional<MC, HarmL, HarmG>::type Src;
    extern __shared__ __attribute__((aligned(16))) double fit_lds[];
    const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
    const int gpw = pb.fit_lanes > 0 ? pb.fit_lanes : 64 / LPS;  // series per wave
    const int grp = lane / LPS, r = lane & (LPS - 1);
    if (grp >= gpw) return;
    const long long k = ((long long)blockIdx.x * (blockDim.x >> 6) + wv) * gpw + grp;
    if (k >= pb.P) return;
    const int slot = wv * gpw + grp;
    NW &nw = ((NW *)fit_lds)[slot];
    const Info in = *info;
    const Span sp = span_of(pb, k);
    // harmonic path unusable for these timestamps, or a short (last) window: exact fit
    if (in.mode == 2 || sp.s1 - sp.s0 < pb.harm_min) {
        if (r == 0) list[atomicAdd(count, 1)] = (int)k;
        return;
    }
    HarmChi2<LPS, Src> f;
    f.r = r;
    f.nvalid = aux[4 * k + 3];
    f.W2 = aux[4 * k + 0];
    f.DEN = aux[4 * k + 1];
    const double Q2 = aux[4 * k + 2];
    // tail bound: |Σ_{|n|>K} J_n e^{-jnϕ} F_n| ≤ 2|J_{K+1}| sqrt(N Σ|q|²) ≤ 1e-16 sqrt(W2·DEN)
    f.tailref = 0.5e-16 * sqrt(f.W2 * f.DEN) / sqrt(f.nvalid * Q2);
    f.qbase = in.mode == 1 ? in.qbase : 0.0;
    f.phimax = in.phimax;
    f.a_re = f.a_im = 0.0;
    f.nfev = 0;
    f.fallback = false;
    harm_offsets(f, pb, k, d0);
    const long long g = f.offs ? (long long)pb.fcop[k] : 0;
    if constexpr (MC) {
        const int nsl = (int)(blockDim.x >> 6) * gpw;  // series slots of the workgroup
        ldouble *cache = (ldouble *)((char *)fit_lds + (size_t)nsl * sizeof(NW));
        ldouble *cs = cache + (size_t)slot * HARM_ROWS;
        for (int q = r; q < HARM_ROWS; q += LPS) cs[q] = mom[(long long)q * pb.P + k];
        f.src.p = cs;
        f.srcG.p = cs;
        if (f.offs) {
            ldouble *cg = cache + (size_t)(nsl + slot) * HARM_ROWS;
            for (int q = r; q < HARM_ROWS; q += LPS) cg[q] = momG[(long long)q * PG + g];
            f.srcG.p = cg;
        }
        // the group's lanes read each other's rows: one wave, LDS in issue order
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        f.src = HarmG{mom, pb.P, k};
        f.srcG = f.offs ? HarmG{momG, PG, g} : f.src;
    }
    f.prof = (pb.flags & F_PROF) != 0;
    f.prof_cycles = f.prof_wave = 0;
    const unsigned long long tfit = f.prof ? __builtin_amdgcn_s_memtime() : 0;
    double x[2];
    int status = 0;
#ifdef GPD_DIAG
    const unsigned long long rt0 = f.prof ? __builtin_amdgcn_s_memrealtime() : 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) nw.prof_[q] = 0;
#endif
    drive_fit(f, pb, x, status, nw);
#ifdef GPD_DIAG
    if (f.prof) {  // the wave's fit time (its lanes meet again here): mean and max over waves
        const unsigned long long tw = __builtin_amdgcn_s_memtime() - tfit;
        const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
        const long long wid = (long long)blockIdx.x * (blockDim.x >> 6) + wv;
        unsigned long long *wrec = pb.prof + PROF_WV + 4 * wid;
        if ((int)threadIdx.x == __builtin_amdgcn_readfirstlane((int)threadIdx.x)) {
            atomicAdd(&pb.prof[PROF_FIT + 5], tw);
            atomicMax(&pb.prof[PROF_FIT + 6], tw);
            atomicAdd(&pb.prof[PROF_FIT + 7], 1ull);
            if (wid < PROF_WV_MAX) {  // the wave's timeline record (vector atomics)
                atomicMax(&wrec[0], rt0);
                atomicMax(&wrec[1], rt1);
                const unsigned long long hw = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
                const unsigned long long xcc = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));
                atomicMax(&wrec[3], hw | (xcc << 32));
            }
        }
        if (r == 0 && wid < PROF_WV_MAX) atomicMax(&wrec[2], (unsigned long long)f.nfev);
    }
#endif
    const double chi2 = f(x);  // likelihood[idx] = lkl(x) (src/Modulation.jl:416)
    if (f.prof && r == 0) {
        atomicAdd(&pb.prof[PROF_FIT + 0], f.prof_cycles);
        atomicAdd(&pb.prof[PROF_FIT + 1], __builtin_amdgcn_s_memtime() - tfit);
        atomicAdd(&pb.prof[PROF_FIT + 2], (unsigned long long)f.nfev);
#ifdef GPD_DIAG
#pragma unroll
        for (int q = 0; q < 16; ++q) atomicAdd(&pb.prof[PROF_NW + q], nw.prof_[q]);
        atomicAdd(&pb.prof[PROF_FIT + 4], f.prof_wave);
#endif
    }
    if (r != 0) return;
    if (f.fallback) {
        list[atomicAdd(count, 1)] = (int)k;
        return;
    }
    store_param(out, raw, k, f.c_re, f.c_im, f.a_re, f.a_im, x[0], x[1], chi2, f.nfev, status);
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// EXACT PATH — a series is fitted by G ∈ {1, 2, 4, 8} workgroups of EXACT_WG threads; NEWUOA
// runs replicated on every thread of every one of them (uniform control flow: every thread
// obtains bit-identical χ² totals), χ² is a cooperative pass with the reference arithmetic.
//
// Canonical reduction order CR8 (the oracle's gsum, oracle/demod_oracle.c): sample i of the
// series (counted from its first sample) adds into slot i mod 2048; slot s = 256·blk + t is
// thread t's accumulator during block blk's sweep (samples s0 + 256·blk + t + 2048·m in order);
// a block total is block_sum's fixed tree (xor butterfly per wave, 4 wave totals left to right);
// the 8 block totals are added left to right.  One workgroup (G = 1) sweeps the 8 blocks in
// turn; with G > 1 workgroup g sweeps blocks [g·8/G, (g+1)·8/G), publishes its block totals and
// every workgroup of the series adds all 8 after a per-series barrier — the same bits for every
// G, so small batches (one exposure: 32 series) can spread over the chip.
constexpr int CR_BLOCKS = 8;
static_assert(FS_G == CR_BLOCKS, "the one-pass faint statistics split a series along the CR8 blocks");
constexpr int CR_SLOTS = CR_BLOCKS * EXACT_WG;  // 2048
constexpr int CR_NV = 8;                        // values per block total (offsets: 8)
#ifndef GPD_CR_U
#define GPD_CR_U 4  // A/B builds: -DGPD_CR_U=n
#endif
constexpr int CR_U = GPD_CR_U;                  // cr_sum2: samples per prefetched batch
#ifndef GPD_CR_UR
#define GPD_CR_UR 4
#endif
constexpr int CR_UR = GPD_CR_UR;                // the same for the residual pass (loads only)
constexpr int CR_FLAG = (EXACT_WG / 64) * 8;    // LDS word after block_sum's partials
constexpr int EXACT_LDS = CR_FLAG + 1;          // doubles of LDS per exact-path workgroup

// Per-series exchange of block totals between the G workgroups of a multi-workgroup fit:
// tot[2 slots][CR_BLOCKS][CR_NV] doubles per series, one arrival counter per series (zeroed
// before the launch).  Barrier k (k = 1, 2, …) uses slot k & 1 and completes when the counter
// reaches k·G.  Payload stores are write-through (sc1) and drained before the arrival add,
// consumers poll the counter relaxed, take one agent acquire, and read the payload with sc1
// loads (cdna_hip_programming.md Guideline 16, R1; MI355X_MICROARCH.md § visibility).
struct Xchg {
    double *tot;
    unsigned *cnt;
};
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// UR: samples per prefetched batch of the residual pass (the model cache and the series);
// 8 at two waves per SIMD (C5 exact 339 → 315-320 ms), 4 at one (r2: 2/6/8/16 no better there).
// WGT: threads per series — EXACT_WG (256: thread t owns slot t of each canonical block), or 64
// for short spans (k_fit_exact with WGT = 64: lane l owns the block's slots l, l+64, l+128,
// l+192 and reduces them as block_sum's four waves would — the same sums, one wave per series).
// r4: an evaluation reads the functor's fields once (View), streams the per-series arrays
// non-temporally (ld_s) and, for ComplexF64 storage and Float64 arithmetic, takes the FAST form
// whose per-sample loads are unconditional (eval<true>): C5 exact 316 → 254 ms, same bits.
#ifndef GPD_EXACT_NT
#define GPD_EXACT_NT 1
#endif
// A sample's Payne–Hanek table entry (PHT instances; gpd_jlmath.h jlm_ph_table_entry) and an
// evaluation's shift of it (jlm_ph_shift)
template <bool ON> struct PhRaw {
    uint64_t w0, w1, a3;
};
template <> struct PhRaw<false> {};
struct PhShift {
    bool on;
    uint64_t klo, khi, d3;
};
// PHT (r6, the one-wave-per-SIMD instances: one exposure at G workgroups per series): with MJD-scale
// phases, the first pass reads each sample's Payne–Hanek table entry in place of t and forms
// sin(θ) from it and the evaluation's shift — the bits of jl_sin(fl(fl(ωt) + ϕ)) with two 64-bit
// adds per sample in place of Payne–Hanek's three 64×64-bit products (gpd_jlmath.h).
template <bool FAINT, bool OFFS, bool PHBUF, int UR = CR_UR, int WGT = EXACT_WG, bool PHT = false>
struct ExactChi2 {
    static constexpr bool kOffs = OFFS;
    const Problem *pb;
    long long doff, foff;         // series column / raw FC column offsets (setup_exact)
    const c64 *__restrict__ src;  // PHBUF: phasor column
    double *lds;
    double m5[5], w5[5];
    double nvalid;
    double a_re, a_im, c_re, c_im;
    long long s0, s1;  // sample range (the series' window)
    int nfev;
    // model cache (nullptr: none): the final pass of each evaluation reads the model the first
    // pass computed (same values, so the same sums) instead of re-evaluating sin/sincos and the
    // FC phasor; element i − s0 of the series' slot
    c64 *mc;
    // multi-workgroup split: G workgroups per series, this one is g; x: the series' exchange
    int G, g;
    Xchg x;
    unsigned nbar;  // barriers passed
    bool sync_fail; // the series' barrier was poisoned (never observed; NaN, GPD_ST_SYNC)
    bool fp32;      // F_FP32: Float32 per-sample arithmetic (non-offsets only)
    // GPD_FIT_PROF (diagnostics): cycles of the first pass, the residual pass, the G > 1
    // exchange (barrier) and the whole fit, per workgroup
    bool prof;
    unsigned long long pc[3];
    // PHT: the range of fl(ωt) over the valid samples (Info xmin / xmax when every one is > 0;
    // 0 otherwise: the table is never used)
    double phx0, phx1;

    // Global-address-space views of the problem's arrays, taken once per evaluation: this
    // functor runs out of line, where plain pointers are generic and every flat load's wait
    // drains all outstanding loads.
    typedef const __attribute__((address_space(1))) double gdouble;
    typedef const __attribute__((address_space(1))) c64 gc64;
    typedef const __attribute__((address_space(1))) c32 gc32;
    typedef const __attribute__((address_space(1))) int8_t gi8;
    typedef __attribute__((address_space(3))) double ldouble;
    struct View {
        gdouble *t;
        gc64 *d, *fc, *src;
        gc32 *d32, *fc32;
        gi8 *state;
        const __attribute__((address_space(1))) float *xr;  // F_FP32 phase table
        double omega;
        bool only_high;
        // the model cache, read once per evaluation (members of an out-of-line functor are
        // read through its pointer, again after every store that may alias it)
        __attribute__((address_space(1))) c64 *mc;
        long long s0;
        long long doff, foff;   // series column / raw FC column offsets
        const double *m5, *w5;  // faint power and weight per state (the functor's)
        const __attribute__((address_space(1))) uint64_t *pht;  // PHT: the Payne–Hanek table
        long long N;
    };
    __device__ __forceinline__ View view() const {
        View v;
        v.t = (gdouble *)pb->t;
        v.d = (gc64 *)pb->d;
        v.d32 = (gc32 *)pb->d32;
        v.fc = (gc64 *)pb->fc;
        v.fc32 = (gc32 *)pb->fc32;
        v.src = (gc64 *)src;
        v.state = (gi8 *)pb->state;
        v.omega = pb->omega;
        v.only_high = (pb->flags & F_ONLY_HIGH) != 0;
        v.xr = (const __attribute__((address_space(1))) float *)(fp32 ? pb->xr32 : nullptr);
        v.mc = (__attribute__((address_space(1))) c64 *)mc;
        v.s0 = s0;
        v.doff = doff;
        v.foff = foff;
        v.m5 = m5;
        v.w5 = w5;
        v.pht = (const __attribute__((address_space(1))) uint64_t *)(PHT ? pb->pht : nullptr);
        v.N = pb->N;
        return v;
    }
    typedef __attribute__((address_space(1))) c64 gmc64;
    static __device__ __forceinline__ c64 ld(gc64 *p) { return c64{p->re, p->im}; }
    // the streamed per-series arrays (series, phasor column, model cache): non-temporal, so
    // that the shared phases and states keep their L2 lines (r4: C5 exact 302-306 → 287-288 ms;
    // -DGPD_EXACT_NT=0 for plain loads and stores)
    typedef double nv2d __attribute__((ext_vector_type(2)));
    static __device__ __forceinline__ c64 ld_s(gc64 *p) {
#if GPD_EXACT_NT
        const nv2d v = __builtin_nontemporal_load((const __attribute__((address_space(1))) nv2d *)p);
        return c64{v.x, v.y};
#else
        return c64{p->re, p->im};
#endif
    }
    // weight of a valid sample (FAINT: w of its state; the power m is inside the cached model)
    static __device__ __forceinline__ double weight_of(const View &v, int st) {
        if (!FAINT) return 1.0;
        double ww = v.w5[0];
#pragma unroll
        for (int q = 1; q < 5; ++q) ww = (st + 1 == q) ? v.w5[q] : ww;
        return ww;
    }
    static __device__ __forceinline__ c64 ld(gc32 *p) { return c64{(double)p->re, (double)p->im}; }
    __device__ __forceinline__ c64 d_of(const View &v, long long off) const {
        return v.d32 ? ld(v.d32 + off) : ld_s(v.d + off);
    }
    // sample_valid (TRANSIENT dropped, onlyhigh keeps HIGH ∪ NORMAL), src/Modulation.jl:373-382
    __device__ __forceinline__ bool valid(const View &v, long long i, int &st) const {
        if (v.state == nullptr) {
            st = 0;
            return true;
        }
        st = v.state[i];
        if (st == -1) return false;
        if (v.only_high) return st == 3 || st == 2;
        return true;
    }
    __device__ __forceinline__ bool load(const View &v, long long i, c64 &p, double &w) const {
        int st;
        if (!valid(v, i, st)) return false;
        const c64 ph = PHBUF ? ld(v.src + i)
                             : fc_phasor(v.fc32 ? ld(v.fc32 + v.foff + i) : ld(v.fc + v.foff + i));
        if (FAINT) {
            double m = v.m5[0], ww = v.w5[0];
#pragma unroll
            for (int q = 1; q < 5; ++q) {
                m = (st + 1 == q) ? v.m5[q] : m;
                ww = (st + 1 == q) ? v.w5[q] : ww;
            }
            p = {m * ph.re, m * ph.im};  // power .* FCphasor (src/Modulation.jl:396)
            w = ww;
        } else {
            p = ph;
            w = 1.0;
        }
        return true;
    }
    // A sample's inputs, loaded ahead of their use (cr_sum2): the state, ωt's t, the phasor
    // (PHBUF) or the raw FC sample, the series sample — or, for the residual pass, the cached
    // model in place of t and the phasor.
    struct Raw {
        c64 f, d;
        double t;
        int st;
        PhRaw<PHT> ph;  // PHT: the table entry (loaded in place of t when the shift applies)
    };
    // FAST (r4): ComplexF64 storage, Float64 arithmetic, and the state
    // array present exactly when FAINT — every load of a sample unconditional, so that the
    // compiler counts the prefetched batch's loads exactly and waits only for the batch in use
    // (with the runtime storage / fp32 / state selects it fell back to waiting for all
    // outstanding loads on every path that might skip one).
    // D32 (FAST only, r6): ComplexF32 storage read as 8-B elements (the widened values, as the
    // general form's d_of gives them)
    template <bool FAST = false, bool D32 = false>
    __device__ __forceinline__ void load_raw(const View &v, long long i, Raw &r) const {
        if constexpr (FAST) {
            r.st = FAINT ? (int)v.state[i] : 0;
            r.t = v.t[i];
            if constexpr (D32) {
                r.f = PHBUF ? ld_s(v.src + i) : ld(v.fc32 + v.foff + i);
                r.d = ld(v.d32 + v.doff + i);
            } else {
                r.f = PHBUF ? ld_s(v.src + i) : ld_s(v.fc + v.foff + i);
                r.d = ld_s(v.d + v.doff + i);
            }
            return;
        }
        r.st = v.state ? (int)v.state[i] : 0;
        r.t = v.xr ? (double)v.xr[i] : v.t[i];  // F_FP32: the reduced phase instead of t
        r.f = PHBUF ? ld_s(v.src + i) : (v.fc32 ? ld(v.fc32 + v.foff + i) : ld_s(v.fc + v.foff + i));
        r.d = d_of(v, v.doff + i);
    }
    // PHT: the FAST loads with the sample's table entry in place of t
    __device__ __forceinline__ void load_raw_ph(const View &v, long long i, Raw &r) const {
        if constexpr (PHT) {
            typedef uint64_t u2v __attribute__((ext_vector_type(2)));
            r.st = FAINT ? (int)v.state[i] : 0;
            const u2v w = *(const __attribute__((address_space(1))) u2v *)(v.pht + 2 * i);
            r.ph.w0 = w.x;
            r.ph.w1 = w.y;
            r.ph.a3 = v.pht[2 * v.N + i];
            r.f = PHBUF ? ld_s(v.src + i) : ld_s(v.fc + v.foff + i);
            r.d = ld_s(v.d + v.doff + i);
        }
    }
    template <bool FAST = false, bool D32 = false>
    __device__ __forceinline__ void load_res(const View &v, long long i, Raw &r) const {
        if constexpr (FAST) {
            r.st = FAINT ? (int)v.state[i] : 0;
            r.f = ld_s(v.mc + (i - v.s0));
            if constexpr (D32)
                r.d = ld(v.d32 + v.doff + i);
            else
                r.d = ld_s(v.d + v.doff + i);
            return;
        }
        r.st = v.state ? (int)v.state[i] : 0;
        r.f = ld_s(v.mc + (i - v.s0));
        r.d = d_of(v, v.doff + i);
    }
    // the first pass's store of sample i's model into the workgroup's model-cache slot
    template <bool FAST = false>
    __device__ __forceinline__ static void mc_put(const View &v, long long i, const c64 &m) {
        const long long e = i - v.s0;
#if GPD_EXACT_NT
        __builtin_nontemporal_store(nv2d{m.re, m.im}, (__attribute__((address_space(1))) nv2d *)(v.mc + e));
#else
        v.mc[e].re = m.re;
        v.mc[e].im = m.im;
#endif
    }
    // sample_valid on a loaded state (TRANSIENT dropped, onlyhigh keeps HIGH ∪ NORMAL)
    template <bool FAST = false>
    __device__ __forceinline__ bool valid_st(const View &v, int st) const {
        if (FAST ? !FAINT : v.state == nullptr) return true;
        if (st == -1) return false;
        if (v.only_high) return st == 3 || st == 2;
        return true;
    }
    // load() on a loaded sample: power·phasor and weight
    static __device__ __forceinline__ void pw_of(const View &v, const Raw &r, c64 &p, double &w) {
        const c64 ph = PHBUF ? r.f : fc_phasor(r.f);
        if (FAINT) {
            double m = v.m5[0], ww = v.w5[0];
#pragma unroll
            for (int q = 1; q < 5; ++q) {
                m = (r.st + 1 == q) ? v.m5[q] : m;
                ww = (r.st + 1 == q) ? v.w5[q] : ww;
            }
            p = {m * ph.re, m * ph.im};  // power .* FCphasor (src/Modulation.jl:396)
            w = ww;
        } else {
            p = ph;
            w = 1.0;
        }
    }
    // model() of U loaded samples at once: when every lane's U arguments lie in one regime of
    // jl_sin (MJD-scale Payne–Hanek, Cody–Waite extended) and of jl_sincos (|β| ≲ 9π/4), the
    // regime's branch-free form runs for all U in one basic block; otherwise the general
    // functions.  Either way each sample's model has model()'s bits (gpd_jlmath.h).
    template <int U>
    __device__ __forceinline__ void model_batch(const View &v, const Raw (&X)[U], double b,
                                                double phi, c64 (&m)[U]) const {
        double th[U], s[U];
        int ph = 1, cw = 1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            th[u] = v.omega * X[u].t;
            th[u] = th[u] + phi;
            ph &= jlm_sin_ph_in(th[u]);
            cw &= jlm_sin_cwx_in(th[u]);
        }
        if (__all(ph)) {
            // one binade for the whole wave (MJD-scale ωt spans one or two): its three words of
            // 2/π fetched once, wave-uniform, instead of per lane and sample
            const int e0 = __builtin_amdgcn_readfirstlane(jlm_biased_exponent(th[0]));
            int one = 1;
#pragma unroll
            for (int u = 0; u < U; ++u) one &= jlm_biased_exponent(th[u]) == e0;
            if (__all(one)) {
                uint64_t a1, a2, a3;
                jlm_ph_words(e0, &a1, &a2, &a3);
#pragma unroll
                for (int u = 0; u < U; ++u) s[u] = jl_sin_ph_w(th[u], a1, a2, a3);
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) s[u] = jl_sin_ph_nb(th[u]);
            }
        } else if (__all(cw)) {
#pragma unroll
            for (int u = 0; u < U; ++u) s[u] = jl_sin_cwx_nb(th[u]);
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) s[u] = jl_sin(th[u]);
        }
        model_tail<U>(v, X, b, s, m);
    }
    // model_batch from the samples' Payne–Hanek table entries and the evaluation's shift (PHT,
    // sh.on): sin(θ) = jl_sin_ph_shifted — jl_sin(fl(fl(ωt) + ϕ))'s bits
    template <int U>
    __device__ __forceinline__ void model_batch_ph(const View &v, const Raw (&X)[U], double b,
                                                   const PhShift &sh, c64 (&m)[U]) const {
        double s[U];
        if constexpr (PHT) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                s[u] = jl_sin_ph_shifted(X[u].ph.w0, X[u].ph.w1, X[u].ph.a3, sh.klo, sh.khi, sh.d3);
        }
        model_tail<U>(v, X, b, s, m);
    }
    // β = b·sin θ, exp(ȷβ) and the model of U samples from their sin θ
    template <int U>
    __device__ __forceinline__ void model_tail(const View &v, const Raw (&X)[U], double b,
                                               const double (&s)[U], c64 (&m)[U]) const {
        double be[U];
        int sm = 1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            be[u] = b * s[u];
            sm &= jlm_sincos_small_in(be[u]);
        }
        c64 e[U];
        if (__all(sm)) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                double ss, cc;
                jl_sincos_small_nb(be[u], &ss, &cc);
                e[u] = c64{cc, ss};  // cisj: exp(ȷβ), β = 0 → (1, β)
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) e[u] = cisj(be[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            c64 p;
            double w;
            pw_of(v, X[u], p, w);
            m[u] = cmul(p, e[u]);  // power * exp(ȷ b sin(ωt+ϕ)) (src/Modulation.jl:137)
        }
    }
    __device__ __forceinline__ c64 model(const View &v, long long i, const c64 &p, double b,
                                         double phi) const {
        double th = v.omega * v.t[i];
        th = th + phi;
        const double beta = b * jl_sin(th);
        return cmul(p, cisj(beta));  // power * exp(ȷ b sin(ωt+ϕ)) (src/Modulation.jl:137)
    }

    // ---- Float32 per-sample arithmetic (F_FP32; BASELINE config 5's fp32 half, the build's own
    // experiment — the reference's Float32 path cannot run).  θ = x_i + ϕ with x_i =
    // fl(ω t_i) reduced modulo 2π once per call in Float64 (k_phase32, shared by all series);
    // sin, sincos, the FC phasor z/|z|, the model, the products and the residual in Float32;
    // the sums (canonical order) and NEWUOA in Float64.
    struct f2 {
        float re, im;
    };
    static __device__ __forceinline__ f2 fmul2(f2 a, f2 b) {
        return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
    }
    static __device__ __forceinline__ float weight32(const View &v, int st) {
        return (float)weight_of(v, st);
    }
    static __device__ __forceinline__ f2 power_phasor32(const View &v, const Raw &r) {
        const float fr = (float)r.f.re, fi = (float)r.f.im;
        f2 ph;
        if (PHBUF) {  // the phasor buffer holds the Float64 phasor
            ph = {fr, fi};
        } else {
            const float inv = rsqrtf(fr * fr + fi * fi);
            ph = {fr * inv, fi * inv};
        }
        if (FAINT) {
            double m = v.m5[0];
#pragma unroll
            for (int q = 1; q < 5; ++q) m = (r.st + 1 == q) ? v.m5[q] : m;
            const float mf = (float)m;
            ph = {mf * ph.re, mf * ph.im};
        }
        return ph;
    }
    // Float32 sin and cos for the small arguments of this evaluator (|θ| ≲ 2π + |ϕ|, |β| ≤ |b|):
    // Cody–Waite reduction by π/2 in three Float32 parts with fma, the classic minimax
    // polynomials on [−π/4, π/4] (Cephes sinf/cosf coefficients), quadrant selected branch-free
    static __device__ __forceinline__ void sincos32(float x, float &s, float &c) {
        const float k = rintf(x * 0.636619772f);
        float r = fmaf(-k, 1.57079637050628662109375f, x);
        r = fmaf(-k, -4.37113882867379e-8f, r);
        r = fmaf(-k, -1.7151245e-15f, r);
        const float r2 = r * r;
        float sp = fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
        sp = fmaf(r2, sp, -1.6666654611e-1f);
        sp = fmaf(r2 * r, sp, r);
        float cp = fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
        cp = fmaf(r2, cp, 4.166664568298827e-2f);
        cp = fmaf(r2 * r2, cp, fmaf(-0.5f, r2, 1.0f));
        const int q = (int)k & 3;
        s = (q == 0) ? sp : (q == 1) ? cp : (q == 2) ? -sp : -cp;
        c = (q == 0) ? cp : (q == 1) ? -sp : (q == 2) ? -cp : sp;
    }
    __device__ __forceinline__ f2 model32(float x, const f2 &p, float b, float phi) const {
        const float th = x + phi;
        float st, ct, sn, cs;
        sincos32(th, st, ct);
        sincos32(b * st, sn, cs);
        return fmul2(p, f2{cs, sn});
    }
    template <int U>
    __device__ __forceinline__ void model_batch32(const View &v, const Raw (&X)[U], double b,
                                                  double phi, c64 (&m)[U]) const {
        const float bf = (float)b, pf = (float)phi;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const f2 mm = model32((float)X[u].t, power_phasor32(v, X[u]), bf, pf);
            m[u] = c64{(double)mm.re, (double)mm.im};
        }
    }

    // Per-series barrier of the G workgroups (G > 1); the caller has issued its payload stores.
    // A part that waits too long (~1 s: a sibling is not resident — never observed) poisons the
    // series' arrival counter with XPOISON by compare-and-swap, unless the last sibling arrived
    // meanwhile.  Every part of the series reads the poison at this same barrier (its own add or
    // its wait returns the poisoned count), so all G parts set sync_fail together, skip every
    // later pass and barrier (NaN totals), and the record carries GPD_ST_SYNC | GPD_ST_NAN.
    static constexpr unsigned XPOISON = 0x80000000u;
    __device__ __forceinline__ void xbarrier() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
        __syncthreads();
        ++nbar;
        if (threadIdx.x == 0) {
            const unsigned target = nbar * (unsigned)G;
            const unsigned spin_max = (pb->flags & F_XSPIN_TEST) ? 0u : (1u << 24);
            unsigned c = __hip_atomic_fetch_add((gu32 *)x.cnt, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) + 1u;
            unsigned spins = 0;
            while (!(c & XPOISON) && c < target) {
                if (++spins > spin_max) {
                    // give up, unless the count moved on (c is refreshed by a failed CAS)
                    if (__hip_atomic_compare_exchange_strong((gu32 *)x.cnt, &c, c | XPOISON,
                                                             __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT)) {
                        c |= XPOISON;
                        break;
                    }
                    continue;
                }
                __builtin_amdgcn_s_sleep(2);
                c = __hip_atomic_load((gu32 *)x.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            ((ldouble *)lds)[CR_FLAG] = (c & XPOISON) ? 1.0 : 0.0;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        sync_fail = ((ldouble *)lds)[CR_FLAG] != 0.0;  // every thread takes the same branches
    }

    // Σ over the series' samples of accum(i, acc) in the canonical order CR8; every thread of
    // every workgroup of the series returns the same NV totals.
    template <int NV, class A>
    __device__ __forceinline__ void cr_sum(A &&accum, double (&tot)[NV]) {
        cr_sum_blocks<NV>(
            [&](long long i0, double (&acc)[NV]) {
                for (long long i = i0; i < s1; i += CR_SLOTS) accum(i, acc);
            },
            tot);
    }
    // chain(i0, acc): add the chain of samples i0, i0 + 2048, … < s1 into acc, in order
    template <int NV, class C>
    __device__ __forceinline__ void cr_sum_blocks(C &&chain, double (&tot)[NV]) {
        ldouble *lp = (ldouble *)lds;
        if (sync_fail) {  // the series' barrier was poisoned: every part stops passing samples
#pragma unroll
            for (int k = 0; k < NV; ++k) tot[k] = __builtin_nan("");
            return;
        }
        if constexpr (WGT == 64) {
            // one wave per series (G = 1): block blk's 256 slots in four quarters of 64 lanes,
            // each quarter butterflied as block_sum's wave stage, the quarter totals added left
            // to right as its LDS stage — block_sum<256>'s tree, bit for bit
            const int lane = (int)threadIdx.x;
            for (int blk = 0; blk < CR_BLOCKS; ++blk) {
                if (blk > 0 && s0 + (long long)blk * EXACT_WG >= s1) {  // empty blocks: as below
#pragma unroll
                    for (int k = 0; k < NV; ++k) tot[k] = tot[k] + 0.0;
                    break;
                }
                double part[NV];
#pragma unroll
                for (int q = 0; q < EXACT_WG / 64; ++q) {
                    double acc[NV];
#pragma unroll
                    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
                    chain(s0 + blk * EXACT_WG + q * 64 + lane, acc);
                    wave_sum<NV>(acc);
#pragma unroll
                    for (int k = 0; k < NV; ++k) part[k] = (q == 0) ? acc[k] : part[k] + acc[k];
                }
#pragma unroll
                for (int k = 0; k < NV; ++k) tot[k] = (blk == 0) ? part[k] : tot[k] + part[k];
            }
            return;
        }
        const int nb = CR_BLOCKS / G, b0 = g * nb;
        for (int blk = b0; blk < b0 + nb; ++blk) {
            if (G == 1 && blk > 0 && s0 + (long long)blk * EXACT_WG >= s1) {
                // a span of at most blk·256 samples: this block and every later one hold no
                // sample, so their totals are +0.0; adding +0.0 once does what adding all of
                // them would (x + 0.0 == x, except −0.0 → +0.0) — the same bits, without the
                // block reductions of empty blocks (short windows)
#pragma unroll
                for (int k = 0; k < NV; ++k) tot[k] = tot[k] + 0.0;
                break;
            }
            double acc[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) acc[k] = 0.0;
            chain(s0 + blk * EXACT_WG + threadIdx.x, acc);
            block_sum<EXACT_WG, NV>(acc, lp);
            if (G == 1) {
#pragma unroll
                for (int k = 0; k < NV; ++k) tot[k] = (blk == 0) ? acc[k] : tot[k] + acc[k];
            } else {
                xpublish<NV>(blk, acc);
            }
        }
        if (G == 1) return;
        xfinish<NV>(tot);
    }
    // G > 1: block blk's totals into the series' exchange slot of the next barrier
    template <int NV>
    __device__ __forceinline__ void xpublish(int blk, const double (&acc)[NV]) {
        if (threadIdx.x < NV) {
            double v = acc[0];
#pragma unroll
            for (int k = 1; k < NV; ++k) v = ((int)threadIdx.x == k) ? acc[k] : v;
            gu64 *slot = (gu64 *)(x.tot + ((nbar + 1) & 1) * (CR_BLOCKS * CR_NV) +
                                  blk * CR_NV + threadIdx.x);
            __hip_atomic_store(slot, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // G > 1: the series' barrier, then the 8 block totals added in block order
    template <int NV>
    __device__ __forceinline__ void xfinish(double (&tot)[NV]) {
        const unsigned long long tb = prof ? __builtin_amdgcn_s_memtime() : 0;
        xbarrier();
        if (prof) pc[2] += __builtin_amdgcn_s_memtime() - tb;
        const double *base = x.tot + (nbar & 1) * (CR_BLOCKS * CR_NV);
#pragma unroll
        for (int blk = 0; blk < CR_BLOCKS; ++blk) {
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                const double v = __builtin_bit_cast(
                    double, __hip_atomic_load((gu64 *)(base + blk * CR_NV + k), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT));
                tot[k] = (blk == 0) ? v : tot[k] + v;
            }
        }
        if (sync_fail) {
#pragma unroll
            for (int k = 0; k < NV; ++k) tot[k] = __builtin_nan("");
        }
    }

    // cr_sum with the loads of each chain issued CR_U samples ahead: load(i, Raw&) fetches a
    // sample's inputs, accum(i, const Raw&, acc) computes and adds in chain order — the same
    // sums as cr_sum (one wave per SIMD: nothing else hides the memory latency of a chain).
    template <int NV, int U = CR_U, class L, class A>
    __device__ __forceinline__ void cr_sum2(L &&load, A &&accum, double (&tot)[NV]) {
        cr_sum2m<NV, U>(
            load, [](const Raw (&)[U], c64 (&)[U]) {},
            [&](long long i, const Raw &r, const c64 &, double (&a)[NV]) { accum(i, r, a); }, tot);
    }
    // cr_sum2 with a batch step: batch(X, m) computes the U samples' models together (one basic
    // block, independent chains for the scheduler) before accum(i, X[u], m[u], acc) adds them
    // in chain order.
    template <int NV, int U = CR_U, class L, class B, class A>
    __device__ __forceinline__ void cr_sum2m(L &&load, B &&batch, A &&accum, double (&tot)[NV]) {
        cr_sum_blocks<NV>(
            [&](long long i0, double (&acc)[NV]) {
                const int M = i0 < s1 ? (int)((s1 - 1 - i0) / CR_SLOTS + 1) : 0;
                if (M == 0) return;
                Raw A_[U], B_[U];
                auto issue = [&](Raw (&X)[U], int m0) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int m = m0 + u < M ? m0 + u : M - 1;
                        load(i0 + (long long)m * CR_SLOTS, X[u]);
                    }
                };
                auto run = [&](const Raw (&X)[U], int m0) {
                    c64 mb[U];
                    batch(X, mb);
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (m0 + u >= M) break;
                        accum(i0 + (long long)(m0 + u) * CR_SLOTS, X[u], mb[u], acc);
                    }
                };
                issue(A_, 0);
                int m0 = 0;
                for (; m0 + U < M; m0 += 2 * U) {
                    issue(B_, m0 + U);
                    run(A_, m0);
                    if (m0 + 2 * U < M) issue(A_, m0 + 2 * U);
                    run(B_, m0 + U);
                }
                if (m0 < M) run(A_, m0);
            },
            tot);
    }
    // The first pass of an evaluation (the model, its sums, the model cache): from the samples'
    // Payne–Hanek table entries when the evaluation's shift applies (PHT, FAST), else from t
    template <int NV, bool FAST, bool D32, class A>
    __device__ __forceinline__ void first_pass(const View &V, double b, double phi,
                                               const PhShift &sh, A &&accum, double (&v)[NV]) {
        if constexpr (PHT && FAST && !D32) {
            if (sh.on) {  // uniform
                cr_sum2m<NV>(
                    [&](long long i, Raw &r) { load_raw_ph(V, i, r); },
                    [&](const Raw (&X)[CR_U], c64 (&mb)[CR_U]) { model_batch_ph(V, X, b, sh, mb); },
                    accum, v);
                return;
            }
        }
        cr_sum2m<NV>(
            [&](long long i, Raw &r) { load_raw<FAST, D32>(V, i, r); },
            [&](const Raw (&X)[CR_U], c64 (&mb)[CR_U]) { model_batch(V, X, b, phi, mb); },
            accum, v);
    }
    __device__ double operator()(const double (&xx)[2]) {
        ++nfev;
        const View V = view();
        const bool nofast = (pb->flags & F_NOFAST) != 0;
        if constexpr (!OFFS && !PHBUF) {
            // F_FP32 with unconditional loads and a Float32 model cache (r6): ComplexF32 or
            // ComplexF64 storage, the state array present exactly when FAINT, a model cache
            if (fp32 && !nofast && V.mc != nullptr && (FAINT == (V.state != nullptr)) &&
                (V.d32 != nullptr) == (V.fc32 != nullptr))
                return V.d32 ? eval32f<true>(V, xx[0], xx[1]) : eval32f<false>(V, xx[0], xx[1]);
        }
        const bool fast_base = !fp32 && (FAINT == (V.state != nullptr)) && !nofast;
        if (fast_base && V.d32 == nullptr && V.fc32 == nullptr) return eval<true>(V, xx[0], xx[1]);
        // ComplexF32 storage, Float64 arithmetic (r6): the FAST form on 8-B elements
        if (fast_base && V.d32 != nullptr && (PHBUF || V.fc32 != nullptr))
            return eval<true, true>(V, xx[0], xx[1]);
        return eval<false>(V, xx[0], xx[1]);
    }
    // ---- F_FP32, FAST form (r6).  The general form (eval<false>) selects per sample between
    // the storage types, the phase table and the optional state, so the compiler waits for every
    // outstanding load at each of those branches, and its model cache holds Float64 copies of the
    // Float32 model.  Here every load is unconditional (the storage type C32 a template
    // argument), the model cache holds the Float32 model itself (8 B per sample instead of 16:
    // the residual pass widens the same Float32 values, so the same sums), and the stored
    // ComplexF32 series (C32) are read as 8-B elements — the same records bit for bit as the
    // general form (tests/test_gpu_fp32.py).
    template <bool C32>
    __device__ __forceinline__ void load_raw32f(const View &v, long long i, Raw &r) const {
        r.st = FAINT ? (int)v.state[i] : 0;
        r.t = (double)v.xr[i];
        if constexpr (C32) {
            r.f = ld(v.fc32 + v.foff + i);
            r.d = ld(v.d32 + v.doff + i);
        } else {
            r.f = ld_s(v.fc + v.foff + i);
            r.d = ld_s(v.d + v.doff + i);
        }
    }
    typedef float nv2f __attribute__((ext_vector_type(2)));
    template <bool C32>
    __device__ __forceinline__ void load_res32f(const View &v, long long i, Raw &r) const {
        r.st = FAINT ? (int)v.state[i] : 0;
#if GPD_EXACT_NT
        const nv2f m = __builtin_nontemporal_load(
            (const __attribute__((address_space(1))) nv2f *)v.mc + (i - v.s0));
#else
        const nv2f m = ((const __attribute__((address_space(1))) nv2f *)v.mc)[i - v.s0];
#endif
        r.f = c64{(double)m.x, (double)m.y};
        if constexpr (C32)
            r.d = ld(v.d32 + v.doff + i);
        else
            r.d = ld_s(v.d + v.doff + i);
    }
    static __device__ __forceinline__ void mc_put32(const View &v, long long i, const c64 &m) {
        const nv2f x = {(float)m.re, (float)m.im};  // the Float32 model (exact: m holds floats)
        __attribute__((address_space(1))) nv2f *p = (__attribute__((address_space(1))) nv2f *)v.mc + (i - v.s0);
#if GPD_EXACT_NT
        __builtin_nontemporal_store(x, p);
#else
        *p = x;
#endif
    }
    template <bool C32>
    __device__ __forceinline__ double eval32f(const View &V, const double b, const double phi) {
        double v[4];  // num(2), den(2): Float32 products, Float64 sums
        cr_sum2m<4>(
            [&](long long i, Raw &r) { load_raw32f<C32>(V, i, r); },
            [&](const Raw (&X)[CR_U], c64 (&mb)[CR_U]) { model_batch32(V, X, b, phi, mb); },
            [&](long long i, const Raw &r, const c64 &m, double (&a)[4]) {
                if (!valid_st<true>(V, r.st)) return;
                mc_put32(V, i, m);
                const float w = weight32(V, r.st);
                const f2 m2 = {(float)m.re, (float)m.im}, d2 = {(float)r.d.re, (float)r.d.im};
                const f2 mwc = {m2.re * w, -(m2.im * w)};
                const f2 xv = fmul2(mwc, d2), yv = fmul2(mwc, m2);
                a[0] += (double)xv.re;
                a[1] += (double)xv.im;
                a[2] += (double)yv.re;
                a[3] += (double)yv.im;
            },
            v);
        const c64 aa = cdiv(c64{v[0], v[1]}, c64{v[2], v[3]});
        c_re = c_im = 0.0;
        a_re = aa.re;
        a_im = aa.im;
        double s[1];
        const f2 a2 = {(float)a_re, (float)a_im};
        cr_sum2<1, UR>([&](long long i, Raw &r) { load_res32f<C32>(V, i, r); },
                       [&](long long i, const Raw &r, double (&a)[1]) {
                           if (!valid_st<true>(V, r.st)) return;
                           const f2 mm = fmul2(a2, f2{(float)r.f.re, (float)r.f.im});
                           const float rr = mm.re - (float)r.d.re, ri = mm.im - (float)r.d.im;
                           a[0] += (double)(weight32(V, r.st) * (rr * rr + ri * ri));
                       },
                       s);
        return s[0] / nvalid;
    }
    template <bool FAST, bool D32 = false>
    __device__ __forceinline__ double eval(const View &V, const double b, const double phi) {
        const bool mcg = mc != nullptr;  // a model cache
        const unsigned long long tp0 = prof ? __builtin_amdgcn_s_memtime() : 0;
        PhShift sh{};
        if constexpr (PHT && FAST)
            sh.on = V.pht != nullptr && jlm_ph_shift(phx0, phx1, phi, &sh.klo, &sh.khi, &sh.d3);
        if (OFFS) {
            double v[8];  // a11, a12(2), a22, b1(2), b2(2)
            first_pass<8, FAST, D32>(
                V, b, phi, sh,
                [&](long long i, const Raw &r, const c64 &m, double (&a)[8]) {
                    if (!valid_st<FAST>(V, r.st)) return;
                    c64 p;
                    double w;
                    pw_of(V, r, p, w);
                    if (mcg) mc_put<FAST>(V, i, m);
                    const c64 dd = r.d;
                    a[0] += w;
                    a[1] += w * m.re;
                    a[2] += w * m.im;
                    a[3] += w * (m.re * m.re + m.im * m.im);
                    a[4] += w * dd.re;
                    a[5] += w * dd.im;
                    const c64 pr = cmul(c64{w * m.re, w * (-m.im)}, dd);
                    a[6] += pr.re;
                    a[7] += pr.im;
                },
                v);
            // StaticArrays 2×2 Cramer solve (src/Modulation.jl:189-192)
            const c64 A11 = {v[0], 0.0}, A12 = {v[1], v[2]}, A21 = {v[1], -v[2]}, A22 = {v[3], 0.0};
            const c64 b1 = {v[4], v[5]}, b2 = {v[6], v[7]};
            const c64 t1 = cmul(A11, A22), t2 = cmul(A12, A21);
            const c64 det = {t1.re - t2.re, t1.im - t2.im};
            const c64 u1 = cmul(A22, b1), u2 = cmul(A12, b2);
            const c64 v1 = cmul(A11, b2), v2 = cmul(A21, b1);
            const c64 cc = cdiv(c64{u1.re - u2.re, u1.im - u2.im}, det);
            const c64 aa = cdiv(c64{v1.re - v2.re, v1.im - v2.im}, det);
            c_re = cc.re;
            c_im = cc.im;
            a_re = aa.re;
            a_im = aa.im;
        } else if (!FAST && fp32) {
            double v[4];  // num(2), den(2): Float32 products, Float64 sums
            cr_sum2m<4>(
                [&](long long i, Raw &r) { load_raw<FAST, D32>(V, i, r); },
                [&](const Raw (&X)[CR_U], c64 (&mb)[CR_U]) { model_batch32(V, X, b, phi, mb); },
                [&](long long i, const Raw &r, const c64 &m, double (&a)[4]) {
                    if (!valid_st<FAST>(V, r.st)) return;
                    if (mcg) mc_put<FAST>(V, i, m);
                    const float w = weight32(V, r.st);
                    const f2 m2 = {(float)m.re, (float)m.im}, d2 = {(float)r.d.re, (float)r.d.im};
                    const f2 mwc = {m2.re * w, -(m2.im * w)};
                    const f2 xv = fmul2(mwc, d2), yv = fmul2(mwc, m2);
                    a[0] += (double)xv.re;
                    a[1] += (double)xv.im;
                    a[2] += (double)yv.re;
                    a[3] += (double)yv.im;
                },
                v);
            const c64 aa = cdiv(c64{v[0], v[1]}, c64{v[2], v[3]});
            c_re = c_im = 0.0;
            a_re = aa.re;
            a_im = aa.im;
        } else {
            double v[4];  // num(2), den(2)
            first_pass<4, FAST, D32>(
                V, b, phi, sh,
                [&](long long i, const Raw &r, const c64 &m, double (&a)[4]) {
                    if (!valid_st<FAST>(V, r.st)) return;
                    c64 p;
                    double w;
                    pw_of(V, r, p, w);
                    if (mcg) mc_put<FAST>(V, i, m);
                    const c64 mwc = {m.re * w, -(m.im * w)};  // conj(model .* weight)
                    const c64 xv = cmul(mwc, r.d);
                    const c64 yv = cmul(mwc, m);
                    a[0] += xv.re;
                    a[1] += xv.im;
                    a[2] += yv.re;
                    a[3] += yv.im;
                },
                v);
            const c64 aa = cdiv(c64{v[0], v[1]}, c64{v[2], v[3]});  // (src/Modulation.jl:144)
            c_re = c_im = 0.0;
            a_re = aa.re;
            a_im = aa.im;
        }
        const unsigned long long tp1 = prof ? __builtin_amdgcn_s_memtime() : 0;
        if (prof) pc[0] += tp1 - tp0;
        // weighted_norm2(model .- data, weight) / N  (src/Modulation.jl:299-305, 325)
        double s[1];
        const c64 aa = {a_re, a_im};
        auto resid = [&](const c64 &m, const c64 &dd, double w, double (&a)[1]) {
            c64 mm = cmul(aa, m);
            if (OFFS) {
                mm.re = c_re + mm.re;
                mm.im = c_im + mm.im;
            }
            const double rr = mm.re - dd.re, ri = mm.im - dd.im;
            a[0] += w * (rr * rr + ri * ri);
        };
        if (!FAST && fp32) {  // Float32 residual, Float64 sum
            const f2 a2 = {(float)a_re, (float)a_im};
            auto resid32 = [&](const f2 &m2, const c64 &dd, float w, double (&a)[1]) {
                const f2 mm = fmul2(a2, m2);
                const float rr = mm.re - (float)dd.re, ri = mm.im - (float)dd.im;
                a[0] += (double)(w * (rr * rr + ri * ri));
            };
            if (mcg) {
                cr_sum2<1, UR>([&](long long i, Raw &r) { load_res<FAST, D32>(V, i, r); },
                                  [&](long long i, const Raw &r, double (&a)[1]) {
                                      if (!valid_st<FAST>(V, r.st)) return;
                                      resid32(f2{(float)r.f.re, (float)r.f.im}, r.d,
                                              weight32(V, r.st), a);
                                  },
                                  s);
            } else {
                cr_sum2<1, UR>([&](long long i, Raw &r) { load_raw<FAST, D32>(V, i, r); },
                                  [&](long long i, const Raw &r, double (&a)[1]) {
                                      if (!valid_st<FAST>(V, r.st)) return;
                                      const f2 m2 = model32((float)r.t, power_phasor32(V, r),
                                                            (float)b, (float)phi);
                                      resid32(m2, r.d, weight32(V, r.st), a);
                                  },
                                  s);
            }
        } else if (mcg) {  // the model the same thread wrote for element i in the first pass
            cr_sum2<1, UR>([&](long long i, Raw &r) { load_res<FAST, D32>(V, i, r); },
                       [&](long long i, const Raw &r, double (&a)[1]) {
                           if (!valid_st<FAST>(V, r.st)) return;
                           resid(r.f, r.d, weight_of(V, r.st), a);
                       },
                       s);
        } else if (FAST) {
            // no model cache (GPD option exact_mcache = 0, or a batch whose cache would exceed
            // 8 GB): the residual pass evaluates the first pass's batched model again — the same
            // values, so the same sums (r5: 82 → 66 B per sample-evaluation, twice the model's
            // VALU work)
            cr_sum2m<1>([&](long long i, Raw &r) { load_raw<FAST, D32>(V, i, r); },
                        [&](const Raw (&X)[CR_U], c64 (&mb)[CR_U]) { model_batch(V, X, b, phi, mb); },
                        [&](long long i, const Raw &r, const c64 &m, double (&a)[1]) {
                            if (!valid_st<FAST>(V, r.st)) return;
                            resid(m, r.d, weight_of(V, r.st), a);
                        },
                        s);
        } else {
            cr_sum<1>(
                [&](long long i, double (&a)[1]) {
                    c64 p;
                    double w;
                    if (!load(V, i, p, w)) return;
                    resid(model(V, i, p, b, phi), d_of(V, V.doff + i), w, a);
                },
                s);
        }
        if (prof) pc[1] += __builtin_amdgcn_s_memtime() - tp1;
        return s[0] / nvalid;
    }
};

// Series k's column, FC source and sample range; a windowed series counts its own valid
// samples (N of demodulateall on that window's state[I]).
template <class F>
__device__ __forceinline__ void setup_exact(F &f, const Problem &pb, long long k,
                                            const c64 *__restrict__ phbuf, double *lds,
                                            double nvalid_all, int G = 1, int g = 0,
                                            Xchg x = Xchg{nullptr, nullptr}) {
    const Span sp = span_of(pb, k);
    f.pb = &pb;
    f.doff = sp.col * pb.ldd;
    const long long fcol = pb.fcop[sp.col];
    f.foff = fcol * pb.ldfc;
    f.src = phbuf ? phbuf + fcol * pb.N : nullptr;
    f.lds = lds;
    f.mc = nullptr;
    f.s0 = sp.s0;
    f.s1 = sp.s1;
    f.G = G;
    f.g = g;
    f.x = x;
    f.nbar = 0;
    f.sync_fail = false;
    f.fp32 = !F::kOffs && (pb.flags & F_FP32) != 0;
    f.prof = (pb.flags & F_PROF) != 0;
    f.pc[0] = f.pc[1] = f.pc[2] = 0;
    if (pb.win > 0) {
        double c[1];
        f.cr_sum([&](long long i, double (&a)[1]) {
            int st;
            if (sample_valid(pb, i, st)) a[0] += 1.0;
        }, c);
        f.nvalid = c[0];
    } else {
        f.nvalid = nvalid_all;
    }
}

// Multi-workgroup layout: workgroup b serves series xser(b) as part xpart(b) of G.  Blocks b and
// b + 8 share an XCD (round-robin dispatch), so the G parts of one series are dealt to one XCD
// (their exchange stays in its L2) — placement is a speed hint only, never correctness.
__device__ __forceinline__ long long xser(long long b, int G) { return ((b >> 3) / G) * 8 + (b & 7); }
__device__ __forceinline__ int xpart(long long b, int G) { return (int)((b >> 3) % G); }

// MINB: minimum workgroups per CU the register allocation must allow.  1 (512 registers, one
// wave per SIMD) for small grids — one exposure, G workgroups per series, a single round of
// waves, where spills would only cost; 2 (256 registers, two waves per SIMD, spills to scratch)
// for batches of several rounds, where the second wave hides the first one's latency (C5 exact:
// 491 → 330 ms; C2 at G = 8: 3.40 → 3.71 ms, profiles/r3/ab_exact).
// WGT = 64 (units 16-19): one wave per series for short spans (windows of < 256 samples, where a
// 256-thread workgroup leaves most threads without a sample): four times the series in flight,
// NEWUOA run once per series instead of once per wave; the same records (ExactChi2 WGT).
template <bool FAINT, bool OFFS, bool PHBUF, int MINB = 1, int WGT = EXACT_WG>
__global__ __launch_bounds__(WGT, MINB) void k_fit_exact(Problem pb, const Info *__restrict__ info,
                                                        const c64 *__restrict__ phbuf,
                                                        const double *__restrict__ fstat,
                                                        const int *__restrict__ list,
                                                        const int *__restrict__ count,
                                                        Param *__restrict__ out,
                                                        double *__restrict__ raw, int extra_status,
                                                        c64 *__restrict__ mcache = nullptr,
                                                        long long mstride = 0, int G = 1,
                                                        double *__restrict__ xtot = nullptr,
                                                        unsigned *__restrict__ xcnt = nullptr)
#if GPD_OWNS(GPD_U_EXACT | GPD_U_EXACT64)
{
    __shared__ double lds[EXACT_LDS];
    // NEWUOA state: one copy per wave in LDS (all lanes of a wave run the same iteration and
    // read/write the same addresses), instead of replicated in every thread's registers
    __shared__ Newuoa<2, 5, true> nwx[WGT / 64];
    const double nvalid = (double)info->nvalid;
    // the Payne–Hanek table path in the one-wave-per-SIMD instances (registers to spare for the
    // wider prefetched samples); its range of fl(ωt) when every valid one is > 0
    constexpr bool kPHT = MINB == 1 && WGT == EXACT_WG;
    const double phx0 = info->xpos ? info->xmin : 0.0, phx1 = info->xpos ? info->xmax : 0.0;
    if (WGT == EXACT_WG && G > 1) {  // one series per G workgroups
      // one round of gridDim.x / G series (gridDim.x = G·⌈P/8⌉·8: a series' G parts are resident
      // together); written as a loop over rounds of per_round series, model-cache slot k mod
      // per_round
      const long long per_round = gridDim.x / G;
      for (long long bb = blockIdx.x;; bb += gridDim.x) {
        const long long k = xser(bb, G);
        if (k >= pb.P) return;  // uniform per series: all its parts leave together
        const int g = xpart(bb, G);
        ExactChi2<FAINT, OFFS, PHBUF, (MINB == 2 ? 8 : CR_UR), WGT, kPHT> f;
        setup_exact(f, pb, k, PHBUF ? phbuf : nullptr, lds, nvalid, G, g,
                    Xchg{xtot + k * (2 * CR_BLOCKS * CR_NV), xcnt + k});
        f.phx0 = phx0;
        f.phx1 = phx1;
        if (mcache) f.mc = mcache + (k % per_round) * mstride;
        if (FAINT) {
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                f.m5[q] = fstat[k * 16 + q];
                f.w5[q] = fstat[k * 16 + 5 + q];
            }
        }
        f.a_re = f.a_im = f.c_re = f.c_im = 0.0;
        f.nfev = 0;
        double x[2];
        int status = ST_EXACT | extra_status;
        const unsigned long long tf = f.prof ? __builtin_amdgcn_s_memtime() : 0;
        drive_fit(f, pb, x, status, nwx[threadIdx.x >> 6]);
        const double chi2 = f(x);
        if (f.sync_fail) status |= ST_SYNC;
        if (g == 0 && threadIdx.x == 0)
            store_param(out, raw, k, f.c_re, f.c_im, f.a_re, f.a_im, x[0], x[1], chi2, f.nfev, status);
        if (f.prof && threadIdx.x == 0) {
            atomicAdd(&pb.prof[PROF_FIT + 0], f.pc[0]);
            atomicAdd(&pb.prof[PROF_FIT + 1], f.pc[1]);
            atomicAdd(&pb.prof[PROF_FIT + 2], f.pc[2]);
            atomicAdd(&pb.prof[PROF_FIT + 3], __builtin_amdgcn_s_memtime() - tf);
        }
        __syncthreads();  // lds and the NEWUOA state are reused by the next round's series
      }
    }
    const long long total = list ? (long long)(*count) : pb.P;
    for (long long idx = blockIdx.x; idx < total; idx += gridDim.x) {
        const long long k = list ? (long long)list[idx] : idx;
        ExactChi2<FAINT, OFFS, PHBUF, (MINB == 2 ? 8 : CR_UR), WGT, kPHT> f;
        setup_exact(f, pb, k, PHBUF ? phbuf : nullptr, lds, nvalid);
        f.phx0 = phx0;
        f.phx1 = phx1;
        if (mcache) f.mc = mcache + (long long)blockIdx.x * mstride;
        if (FAINT) {
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                f.m5[q] = fstat[k * 16 + q];
                f.w5[q] = fstat[k * 16 + 5 + q];
            }
        }
        f.a_re = f.a_im = f.c_re = f.c_im = 0.0;
        f.nfev = 0;
        double x[2];
        int status = ST_EXACT | extra_status;
        drive_fit(f, pb, x, status, nwx[threadIdx.x >> 6]);
        const double chi2 = f(x);
        if (threadIdx.x == 0)
            store_param(out, raw, k, f.c_re, f.c_im, f.a_re, f.a_im, x[0], x[1], chi2, f.nfev, status);
        __syncthreads();
    }
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// χ²(b_k, ϕ_k) for every series at a given point: the Chi2CostFunction functor
// (src/Modulation.jl:318-330) as a batch operation (one evaluation, no optimisation).
// Final evaluation by the exact evaluator at the fitted (pre-normalisation) point: the harmonic
// fitoffsets path re-derives (c, a, χ²) with the reference arithmetic (src/Modulation.jl:416),
// since its 2×2 system is ill-conditioned for small b and would amplify the expansion's
// ~1e-14 rounding into the 1e-11…1e-10 range.  Series already fitted exactly are skipped.
template <bool PHBUF>
__global__ __launch_bounds__(EXACT_WG) void k_refine_exact(Problem pb, const Info *__restrict__ info,
                                                           const c64 *__restrict__ phbuf,
                                                           const double *__restrict__ raw,
                                                           Param *__restrict__ out)
#if GPD_OWNS(GPD_U_CHI2X)
{
    __shared__ double lds[EXACT_LDS];
    for (long long k = blockIdx.x; k < pb.P; k += gridDim.x) {
        if (out[k].status & ST_EXACT) continue;  // uniform per workgroup
        ExactChi2<false, true, PHBUF> f;
        setup_exact(f, pb, k, PHBUF ? phbuf : nullptr, lds, (double)info->nvalid);
        f.nfev = 0;
        double x[2] = {raw[2 * k], raw[2 * k + 1]};
        const double chi2 = f(x);
        if (threadIdx.x == 0) {
            out[k].c_re = f.c_re;
            out[k].c_im = f.c_im;
            out[k].a_re = f.a_re;
            out[k].a_im = f.a_im;
            out[k].chi2 = chi2;
            if (chi2 != chi2) out[k].status |= ST_NAN;
        }
        __syncthreads();
    }
}
#else
;
#endif


template <bool FAINT, bool OFFS, bool PHBUF>
__global__ __launch_bounds__(EXACT_WG) void k_chi2_exact(Problem pb, const Info *__restrict__ info,
                                                         const c64 *__restrict__ phbuf,
                                                         const double *__restrict__ fstat,
                                                         const double *__restrict__ bphi,
                                                         Param *__restrict__ out)
#if GPD_OWNS(GPD_U_CHI2X)
{
    __shared__ double lds[EXACT_LDS];
    const long long k = blockIdx.x;
    ExactChi2<FAINT, OFFS, PHBUF> f;
    setup_exact(f, pb, k, PHBUF ? phbuf : nullptr, lds, (double)info->nvalid);
    if (FAINT) {
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            f.m5[q] = fstat[k * 16 + q];
            f.w5[q] = fstat[k * 16 + 5 + q];
        }
    }
    f.nfev = 0;
    double x[2] = {bphi[2 * k], bphi[2 * k + 1]};
    const double chi2 = f(x);
    if (threadIdx.x == 0) {
        Param p;
        p.c_re = f.c_re;
        p.c_im = f.c_im;
        p.a_re = f.a_re;
        p.a_im = f.a_im;
        p.b = x[0];
        p.phi = x[1];
        p.chi2 = chi2;
        p.nfev = 1;
        p.status = ST_EXACT;
        out[k] = p;
    }
}
#else
;
#endif


__global__ __launch_bounds__(64) void k_chi2_harmonic(Problem pb, const Info *__restrict__ info,
                                                      const double *__restrict__ mom,
                                                      const double *__restrict__ aux,
                                                      const double *__restrict__ momG, long long PG,
                                                      const double *__restrict__ d0,
                                                      const double *__restrict__ bphi,
                                                      Param *__restrict__ out)
#if GPD_OWNS(GPD_U_FITH)
{
    const long long k = (long long)blockIdx.x * 64 + threadIdx.x;
    if (k >= pb.P) return;
    const Info in = *info;
    HarmChi2<1> f;
    f.r = 0;
    f.nvalid = aux[4 * k + 3];
    f.W2 = aux[4 * k + 0];
    f.DEN = aux[4 * k + 1];
    f.tailref = 0.5e-16 * sqrt(f.W2 * f.DEN) / sqrt(f.nvalid * aux[4 * k + 2]);
    f.qbase = in.mode == 1 ? in.qbase : 0.0;
    f.phimax = in.phimax;
    f.a_re = f.a_im = 0.0;
    f.nfev = 0;
    f.fallback = in.mode == 2;
    f.prof = false;
    harm_offsets(f, pb, k, d0);
    f.src = HarmG{mom, pb.P, k};
    f.srcG = f.offs ? HarmG{momG, PG, (long long)pb.fcop[k]} : f.src;
    double x[2] = {bphi[2 * k], bphi[2 * k + 1]};
    const double chi2 = f(x);
    Param p;
    p.c_re = f.c_re;
    p.c_im = f.c_im;
    p.a_re = f.a_re;
    p.a_im = f.a_im;
    p.b = x[0];
    p.phi = x[1];
    p.chi2 = f.fallback ? __builtin_nan("") : chi2;
    p.nfev = 1;
    p.status = f.fallback ? ST_FALLBACK : 0;
    out[k] = p;
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// k_output: demodulated column over ALL samples (src/Modulation.jl:417-425).
__global__ void k_iota(int32_t *__restrict__ a, long long n)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = (int32_t)i;
}
#else
;
#endif


// Σ d over the valid samples of series k (non-faint fitoffsets: b1 = Σ w d, w ≡ 1).
__global__ __launch_bounds__(256) void k_series_sum(Problem pb, double *__restrict__ d0)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ double lds[4 * 2];
    const long long k = blockIdx.x;
    const Span sp = span_of(pb, k);
    const long long doff = sp.col * pb.ldd;
    double v[2] = {0.0, 0.0};
    for (long long i = sp.s0 + threadIdx.x; i < sp.s1; i += 256) {
        int st;
        if (!sample_valid(pb, i, st)) continue;
        const c64 z = d_at(pb, doff + i);
        v[0] += z.re;
        v[1] += z.im;
    }
    block_sum<256, 2>(v, lds);
    if (threadIdx.x == 0) {
        d0[2 * k] = v[0];
        d0[2 * k + 1] = v[1];
    }
}
#else
;
#endif


__global__ __launch_bounds__(256) void k_output(Problem pb, const Param *__restrict__ par,
                                                const double *__restrict__ raw,
                                                c64 *__restrict__ outd, long long ldo)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long k = blockIdx.y;
    const Span sp = span_of(pb, k);
    const Param pk = par[k];
    const double b = raw[2 * k], phi = raw[2 * k + 1];
    const double arga = jl_atan2(pk.a_im, pk.a_re);
    const c64 aa = {pk.a_re, pk.a_im};
    const bool offs = (pb.flags & F_OFFSETS) != 0;
    const long long doff = sp.col * pb.ldd;
    c64 *o = outd + sp.col * ldo;
    for (long long i = sp.s0 + (long long)blockIdx.x * 256 + threadIdx.x; i < sp.s1;
         i += (long long)gridDim.x * 256) {
        double th = pb.omega * gld(pb.t + i);
        th = th + phi;
        c64 dd = d_at(pb, doff + i);
        if (pb.flags & F_RECENTER) {
            double ph = b * jl_sin(th);  // getphase (src/Modulation.jl:66-69)
            ph = ph + arga;
            const double psi = ph - arga;
            if (offs) {
                dd.re = dd.re - pk.c_re;
                dd.im = dd.im - pk.c_im;
            }
            o[i] = cmul(dd, cisj(-psi));
        } else {
            c64 mv = cmul(aa, cisj(b * jl_sin(th)));
            if (offs) {
                mv.re = pk.c_re + mv.re;
                mv.im = pk.c_im + mv.im;
            }
            o[i] = cmul(dd, cisj(-jl_atan2(mv.im, mv.re)));
        }
    }
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// k_ph_table: the exact evaluator's Payne–Hanek table (gpd_jlmath.h jlm_ph_table_entry) of
// x_i = fl(ω t_i), once per call for all series: pht[2i], pht[2i+1] = W (lo, hi), pht[2N+i] = A3.
// Used by the first pass when every x lies in one binade of the Payne–Hanek regime (MJD-scale
// timestamps) and the evaluation's ϕ shifts them all by one whole number of ulps (jlm_ph_shift);
// the values of samples outside that binade are never used.
__global__ __launch_bounds__(256) void k_ph_table(const double *__restrict__ t, long long N,
                                                  double omega, uint64_t *__restrict__ pht)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const double x = omega * t[i];
    uint64_t wlo = 0, whi = 0, a3 = 0;
    if (x > 0.0 && jlm_biased_exponent(x) < 0x7ff) jlm_ph_table_entry(x, &wlo, &whi, &a3);
    pht[2 * i] = wlo;
    pht[2 * i + 1] = whi;
    pht[2 * N + i] = a3;
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// gpd_libm_eval: the shared Julia-libm restatement evaluated on the device (bitwise tests).
__global__ __launch_bounds__(256) void k_libm(int fn, long long n, const double *__restrict__ x,
                                              const double *__restrict__ y, double *__restrict__ out)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    switch (fn) {
    case 0: out[i] = jl_sin(x[i]); break;
    case 1: out[i] = jl_cos(x[i]); break;
    case 2: {
        double s, c;
        jl_sincos(x[i], &s, &c);
        out[2 * i] = s;
        out[2 * i + 1] = c;
        break;
    }
    case 3: out[i] = jl_atan(x[i]); break;
    case 4: out[i] = jl_atan2(x[i], y[i]); break;
    case 5: out[i] = jl_hypot(x[i], y[i]); break;
    case 7: out[i] = jl_hypot_nb(x[i], y[i]); break;
    case 8: out[i] = jl_sin_sel(x[i]); break;
    case 9: {
        double s, c;
        jl_sincos_sel(x[i], &s, &c);
        out[2 * i] = s;
        out[2 * i + 1] = c;
        break;
    }
    case 10: {  // the Payne–Hanek table entry of x[i] and the shift (y: klo, khi, d3, on)
        const uint64_t *ky = (const uint64_t *)y;
        uint64_t wlo, whi, a3;
        jlm_ph_table_entry(x[i], &wlo, &whi, &a3);
        out[i] = ky[3] ? jl_sin_ph_shifted(wlo, whi, a3, ky[0], ky[1], ky[2]) : __builtin_nan("");
        break;
    }
    default: {
        double hi, lo;
        const int q = jl_rem_pio2(x[i], &hi, &lo);
        out[3 * i] = (double)q;
        out[3 * i + 1] = hi;
        out[3 * i + 2] = lo;
    }
    }
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// Synthetic data (benchmarks).  Same counter-based RNG streams as tests/synth.py.
__global__ __launch_bounds__(256) void k_synth_truth(long long P, long long pixel_offset,
                                                     uint64_t seed, int with_offsets, Param *truth)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
    if (k >= P) return;
    const uint64_t gk = (uint64_t)(pixel_offset + k);
    Param p;
    p.b = 0.3 + 2.2 * rng_uniform(seed, 1, gk);
    p.phi = -PI_F64 + 2 * PI_F64 * rng_uniform(seed, 2, gk);
    const double amp = 0.5 + rng_uniform(seed, 3, gk);
    const double arga = -PI_F64 + 2 * PI_F64 * rng_uniform(seed, 4, gk);
    double s, c;
    sincos(arga, &s, &c);
    p.a_re = amp * c;
    p.a_im = amp * s;
    if (with_offsets) {
        p.c_re = 0.1 * rng_normal(seed, 5, gk) / sqrt(2.0);
        p.c_im = 0.1 * rng_normal(seed, 6, gk) / sqrt(2.0);
    } else {
        p.c_re = p.c_im = 0.0;
    }
    p.chi2 = 0.0;
    p.nfev = 0;
    p.status = 0;
    truth[k] = p;
}
#else
;
#endif


__global__ __launch_bounds__(64) void k_synth_fc(long long N, long long n_fc, long long fc_offset,
                                                 uint64_t seed, c64 *fc, long long ldfc)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long g = (long long)blockIdx.x * 64 + threadIdx.x;
    if (g >= n_fc) return;
    const uint64_t gg = (uint64_t)(fc_offset + g);
    double Phi = 2 * PI_F64 * rng_uniform(seed, 7, gg);
    c64 *col = fc + g * ldfc;
    for (long long i = 0; i < N; ++i) {
        Phi += 1e-3 * rng_normal(seed, 100 + gg, (uint64_t)i);
        double s, c;
        sincos(Phi, &s, &c);
        col[i] = {1.3 * c, 1.3 * s};
    }
}
#else
;
#endif


__global__ __launch_bounds__(256) void k_synth_d(long long N, long long P, long long pixel_offset,
                                                 uint64_t seed, double t0, double dt, double sigma,
                                                 double omega, const Param *__restrict__ truth,
                                                 const c64 *__restrict__ fc, long long ldfc,
                                                 c64 *__restrict__ d, long long ldd,
                                                 int32_t *__restrict__ fcop)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long k = blockIdx.y;
    const Param tr = truth[k];
    const uint64_t gk = (uint64_t)(pixel_offset + k);
    const long long g = k / 4;
    if (blockIdx.x == 0 && threadIdx.x == 0) fcop[k] = (int32_t)g;
    const c64 *fcol = fc + g * ldfc;
    c64 *col = d + k * ldd;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < N; i += (long long)gridDim.x * 256) {
        const double t = t0 + (double)i * dt;
        const c64 z = fcol[i];
        const double r = sqrt(z.re * z.re + z.im * z.im);
        const c64 p = {z.re / r, z.im / r};
        const c64 e = cisj(tr.b * sin(omega * t + tr.phi));
        const c64 ae = cmul(c64{tr.a_re, tr.a_im}, e);
        const c64 mdl = {tr.c_re + ae.re, tr.c_im + ae.im};
        const c64 pm = cmul(p, mdl);
        const double n1 = rng_normal(seed, 1000 + 2 * gk, (uint64_t)i);
        const double n2 = rng_normal(seed, 1001 + 2 * gk, (uint64_t)i);
        col[i] = {pm.re + sigma * n1 / sqrt(2.0), pm.im + sigma * n2 / sqrt(2.0)};
    }
}
#else
;
#endif


__global__ __launch_bounds__(256) void k_synth_t(long long N, double t0, double dt, double *t)
#if GPD_OWNS(GPD_U_ENGINE)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < N) t[i] = t0 + (double)i * dt;
}
#else
;
#endif


// ---------------------------------------------------------------------------------------
// VOLT ingest / egress (processmetrology, src/GPPupilDemodulation.jl:147-157, 164-171): the FITS
// table rows are Float32 [re1 im1 … re40 im40]; the fit wants complex128 columns (Julia
// Matrix{ComplexF64} N×40) with the centre of each column subtracted.  64-row tiles through LDS:
// row-major coalesced reads, column-major coalesced writes (and the reverse for egress).
constexpr int VT_ROWS = 64;

__global__ __launch_bounds__(256) void k_volt_ingest(long long N, const float *__restrict__ volt,
                                                     long long ldv, const c64 *__restrict__ centers,
                                                     c64 *__restrict__ out, long long ldo)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ float tile[VT_ROWS][81];
    const long long r0 = (long long)blockIdx.x * VT_ROWS;
    const int nr = (int)((N - r0) < VT_ROWS ? (N - r0) : VT_ROWS);
    for (int e = threadIdx.x; e < VT_ROWS * 80; e += 256) {
        const int r = e / 80, c = e - r * 80;
        tile[r][c] = r < nr ? volt[(r0 + r) * ldv + c] : 0.f;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 40 * VT_ROWS; e += 256) {
        const int k = e / VT_ROWS, r = e - k * VT_ROWS;
        if (r >= nr) continue;
        c64 z = {(double)tile[r][2 * k], (double)tile[r][2 * k + 1]};  // Float64.(VOLT)
        if (centers) {  // cmplxV .-= reshape(offsets, 1, 40)
            z.re = z.re - centers[k].re;
            z.im = z.im - centers[k].im;
        }
        out[k * ldo + r0 + r] = z;
    }
}
#else
;
#endif


// Demodulated columns 0..31 (dem, ld) + the (centred) FC columns 32..39 (src, ld) → Float32 rows.
__global__ __launch_bounds__(256) void k_volt_egress(long long N, const c64 *__restrict__ dem,
                                                     const c64 *__restrict__ src, long long ld,
                                                     float *__restrict__ outv, long long ldov)
#if GPD_OWNS(GPD_U_ENGINE)
{
    __shared__ float tile[VT_ROWS][81];
    const long long r0 = (long long)blockIdx.x * VT_ROWS;
    const int nr = (int)((N - r0) < VT_ROWS ? (N - r0) : VT_ROWS);
    for (int e = threadIdx.x; e < 40 * VT_ROWS; e += 256) {
        const int k = e / VT_ROWS, r = e - k * VT_ROWS;
        if (r >= nr) continue;
        const c64 z = k < 32 ? dem[k * ld + r0 + r] : src[k * ld + r0 + r];
        tile[r][2 * k] = (float)z.re;  // Float32.(volt) after volt[1:2:end,:] .= real(output)'
        tile[r][2 * k + 1] = (float)z.im;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < VT_ROWS * 80; e += 256) {
        const int r = e / 80, c = e - r * 80;
        if (r < nr) outv[(r0 + r) * ldov + c] = tile[r][c];
    }
}
#else
;
#endif


}  // namespace gpd
