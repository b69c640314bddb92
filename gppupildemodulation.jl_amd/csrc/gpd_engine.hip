// C-ABI implementation of include/gpdemod.h on top of the gfx950 kernels (gpd_kernels.hpp).
//
// Host runtime: per-device context (workspace arena, ordering event, kernel timing events)
// created lazily under a mutex; gpd_fit_batch shards series over devices with one host thread
// per device; gpd_fit_batch_dev enqueues the whole pipeline on the caller's stream without a
// host round trip (the harmonic → exact fallback list is consumed on device).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <functional>
#include <cstdarg>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define GPD_PART 0  // split build: unit 0 (gpd_kernels.hpp GPD_OWNS)
#include "../../include/gpdemod.h"
#include "gpd_kernels.hpp"
#include "gpd_states.hpp"

using namespace gpd;

static_assert(sizeof(Param) == sizeof(gpd_param), "gpd_param layout");
static_assert(sizeof(c64) == sizeof(gpd_c64), "gpd_c64 layout");
static_assert(sizeof(c32) == sizeof(gpd_c32), "gpd_c32 layout");

namespace {

void set_err(char *buf, size_t len, const char *fmt, ...) {
    if (!buf || len == 0) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, len, fmt, ap);
    va_end(ap);
}

// Test and diagnostics controls (gpd_set_option, include/gpdemod.h).  The library reads no
// environment variable: a process inheriting one cannot change the product path or the bits of
// its records.  Every option defaults to the production behaviour; tests and the A/B tools set
// them explicitly through the C-ABI and reset them afterwards.
enum OptId {
    O_MIX,           // 1: harmonics 17..24 on split-bf16 MFMAs; 0: all on f64 MFMAs (A/B)
    O_FAINT_STATS,   // 0: faint statistics fused into the moment pass; 1: one-pass kernels; 2: two-pass
    O_FAINT_SIDE,    // 1: separate faint statistics on the side stream (measured: no gain)
    O_FAKE_GPUS,     // 1: keep n_gpus shards on fewer devices (shard g on device g mod ndev)
    O_EXACT_G,       // 0: automatic workgroups per exact series; 1|2|4|8 forced
    O_EXACT_WAVES,   // 0: automatic; 1|2 waves per SIMD of the exact fit
    O_EXACT_WGT,     // 0: automatic; 64|256 threads per exact series
    O_EXACT_FAST,    // 1: unconditional-load evaluator where it applies; 0: general form
    O_EXACT_MCACHE,  // 1: model cache of the exact evaluator; 0: residual pass re-evaluates it
    O_XSPIN_TEST,    // 1: the multi-workgroup barrier gives up at once (poison path, tests)
    O_UNITS,         // 0: automatic sample units of the moment pass; n forced
    O_UPW,           // 0: automatic units per moment workgroup; n forced
    O_FIT_LANES,     // 0: automatic series per harmonic-fit wave; n forced
    O_FIT_LPS,       // 0: automatic lanes per series of the harmonic fit; 1|2|4|8 forced
    O_FIT_WPB,       // 0: automatic waves per harmonic-fit workgroup; 1..4 forced
    O_COHORTS,       // 1: one series cohort; n > 1: pipelined harmonic cohorts
    O_HARM_MIN_SPAN, // shortest window fitted from harmonic moments (samples)
    O_FS_COHORT_MB,  // |d| scratch per cohort of the one-pass faint statistics (MB)
    O_MOMENTS,       // 0: automatic moment kernel; 1: VALU kernel; 2..7 diagnostics variants
    O_FIT_PROF,      // 1: cycle split of the fit kernels on stderr (diagnostics)
    O_SYNC_DEBUG,    // 1: synchronise after every stage and name the stage that faulted
    O_HOST_PROF,     // 1: wall-clock split of the host-buffer calls on stderr (diagnostics)
    O_FIT_MCACHE,    // 1: harmonic fit reads the series' moments from LDS where they fit; 0: L2
    O_STAGE_PINNED,  // 1: demodulated columns staged through a pinned ring; 0: pageable ring (tests)
    O_H2D_PARTS,     // 0: automatic (2 parts for pinned host data, else 1); n: host-buffer harmonic
                     // calls cut into n parts, H2D / compute / D2H pipelined
    O_MOM_CUS,       // 0: the moment pass on the caller's stream; n: on a stream masked to n CUs (A/B)
    O_FIT_CUS,       // 0: off; r > 0: pipelined cohorts (option cohorts) keep r CUs per XCD for
                     // the fits of all but the last cohort, the moment pass on the others
    O_COUNT
};
struct OptDef {
    const char *name;
    long long def;
};
constexpr OptDef kOpt[O_COUNT] = {
    {"mix", 1},          {"faint_stats", 0},   {"faint_side", 0},    {"fake_gpus", 0},
    {"exact_g", 0},      {"exact_waves", 0},   {"exact_wgt", 0},     {"exact_fast", 1},
    {"exact_mcache", 1}, {"xspin_test", 0},    {"units", 0},         {"upw", 0},
    {"fit_lanes", 0},    {"fit_lps", 0},       {"fit_wpb", 0},       {"cohorts", 1},       {"harm_min_span", 256}, {"fs_cohort_mb", 4096},
    {"moments", 0},      {"fit_prof", 0},      {"sync_debug", 0},    {"host_prof", 0},
    {"fit_mcache", 1},   {"stage_pinned", 1},  {"h2d_parts", 0},   {"mom_cus", 0},
    {"fit_cus", 0}};
std::atomic<long long> g_opt[O_COUNT] = {{1}, {0}, {0},   {0},    {0}, {0}, {0}, {1}, {1}, {0}, {0},
                                          {0}, {0}, {0},   {0},    {1}, {256}, {4096}, {0}, {0}, {0},
                                          {0}, {1}, {1}, {0}, {0}, {0}};
inline long long opt(OptId o) { return g_opt[o].load(std::memory_order_relaxed); }
int opt_find(const char *name) {
    if (!name) return -1;
    for (int i = 0; i < O_COUNT; ++i)
        if (std::strcmp(kOpt[i].name, name) == 0) return i;
    return -1;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            set_err(errbuf, errlen, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                    __FILE__, __LINE__);                                                 \
            return GPD_E_HIP;                                                            \
        }                                                                                \
    } while (0)

constexpr int kMaxCohorts = 16;  // series cohorts of the pipelined harmonic path
// timing events / named intervals of the last call (both streams): ≤ 7 per cohort plus the
// per-call stages, so the pipelined path never runs out (advisor r3)
constexpr int kMaxEv = 8 * kMaxCohorts + 16;
constexpr int kMaxTimers = 8 * kMaxCohorts + 16;
// exact fits of short spans take one wave per series once the series outnumber two 256-thread
// workgroups per CU (one round of those); below, the 256-thread workgroup's lower latency per
// evaluation wins (r3: 32 series 0.98 vs 1.56 ms; 16 000 windows 41.6 vs 17.0 ms)
constexpr long long kOneWaveMinSeriesPerCU = 2;
constexpr int kMaxParts = 8;  // parts of a pipelined host-buffer call (option h2d_parts)

struct DevCtx {
    int dev = -1;
    std::mutex mu;
    char *ws = nullptr;
    size_t ws_cap = 0;
    hipEvent_t done = nullptr;  // orders successive calls that share the workspace
    hipEvent_t ev[kMaxEv] = {};
    const char *tname[kMaxTimers] = {};
    int tbeg[kMaxTimers] = {}, tend[kMaxTimers] = {};  // event indices of each interval
    int ntimers = 0;
    // pipelined harmonic path: the fits of cohort c run on `side` while the moment pass of
    // cohort c+1 runs on the caller's stream (high priority: the latency-bound fit waves take
    // CUs as soon as they free up)
    hipStream_t side = nullptr;
    hipEvent_t fork[kMaxCohorts] = {}, join = nullptr;
    // CU-masked streams (options mom_cus / fit_cus): `mstream` on the low mbits bits of the CU
    // mask, `fstream` on the bits above them (gfx950: bit i of the mask is a CU of XCD i mod 8,
    // so the top 8r bits are r CUs of every XCD — tools/probes/cumask.hip)
    hipStream_t mstream = nullptr, fstream = nullptr;
    int mbits = 0;
    hipEvent_t mev[4] = {};
    bool have_timers = false;
    int n_cu = 0;  // compute units (wave-quantisation of the moment grid)
    // gpd_buildstates_dev: pinned staging of the timer lists, reused once its copy has run
    double *bs_pinned = nullptr;
    hipEvent_t bs_done = nullptr;
    // host-buffer entry points (gpd_fit_batch & co.): device copies of the caller's arrays in
    // one grow-only arena and one stream, reused across calls (no hipMalloc/hipFree per
    // exposure); hmu serialises host calls on this device for the duration of a call
    std::mutex hmu;
    char *harena = nullptr;
    size_t harena_cap = 0;
    hipStream_t hstream = nullptr;
    // gpd_demodulateall: staging ring of the demodulated columns — kStageSlots slots of
    // kStageSlotBytes, pinned (hipHostMalloc) or, if that fails or option stage_pinned = 0,
    // pageable (malloc); a bounded allocation whatever the exposure's length
    char *hpin = nullptr;
    bool hpin_pinned = false, hpin_nopin = false;
    hipEvent_t hpin_ev[4] = {};  // each slot's chunk has arrived (host copy pipelined)
    // H2D pipelining of host-buffer harmonic calls (option h2d_parts): part k's columns go up on
    // cstream (event up[k]) while part k−1 computes on hstream (event fin[k−1]); the staged
    // demodulated columns come back on ostream, which waits for fin[k]
    hipStream_t cstream = nullptr, ostream = nullptr;
    hipEvent_t up[kMaxParts] = {}, fin[kMaxParts] = {};
    // the last fit call's faint statistics in the workspace (gpd_last_faint_stats; tests)
    const double *last_fstat = nullptr;
    long long last_fstat_P = 0;
};

std::mutex g_mu;
std::vector<DevCtx *> g_ctx;

DevCtx *ctx_for(int dev) {
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1, nullptr);
    if (!g_ctx[dev]) {
        g_ctx[dev] = new DevCtx();
        g_ctx[dev]->dev = dev;
    }
    return g_ctx[dev];
}

size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

struct Layout {
    size_t info, prof, tab, part, mom, aux, fstat, raw, list, phbuf, partG, momG, auxG, fcid, d0,
        mcache, xtot, xcnt, fsx, fsc, xr32, total;
    long long mstride;  // model-cache elements per exact-path workgroup (0: no cache)
    int nch;            // sample chunks of the moment grid (grid.y)
    long long chunk;    // samples per chunk (a whole number of units)
    int units;          // sample units = partial-moment sets
    long long unit_len; // samples per unit
    size_t smask, dlist, fixp, ftab;  // faint state-split moments (k_moments_ws<FAINT>)
    size_t fsp, fcnt, fixs;           // fused faint statistics (k_moments_ws<FAINT> producers)
    size_t prep;                      // k_prepare_part's partial (count, min, max, bad) per workgroup
    size_t pht;                       // exact path: Payne–Hanek table of fl(ω t) (k_ph_table)
    bool fs1;           // faint statistics in one pass (k_faint_p1/p2/fin), cohorts of fs_pc
    long long fs_pc;    // series per cohort
    int fs_mmax;        // samples per thread and part: ⌈N/2048⌉
};

// Moment-pass grid: (series groups) × (sample chunks).  The samples are cut into U ≤ 26 fixed
// units (whole 32-sample tiles, a function of N only) and every unit gets its own set of partial
// moments, reduced in unit order — so a series' moments do not depend on P, i.e. on the batch,
// the shard or the cohort it is in (a sharded run gives the 1-GPU records bit for bit).  A
// workgroup of the producer/consumer kernel (one per CU) streams `upw` consecutive units; upw is
// chosen to fill the last wave of workgroups: the smallest number of unit-times
// ceil(npg·ceil(U/upw) / n_cu)·upw, ties to the larger upw (fewer, longer workgroups).
// C3 (782 series groups, 256 CUs, U = 26): upw 1 or 2 → 79.4 / 39.7 waves; 12 500 series per GPU
// (C4 on 8 GPUs, 98 groups): upw 1 → 2548 workgroups = 9.95 waves (with 32 units: 12.25 waves,
// a 0.75-wave tail).
// Shape of the harmonic fit (k_fit_harmonic<lps>): lps lanes per series, gpw series per wave,
// wpb waves per workgroup.  A wave lasts as long as its slowest series' NEWUOA (lanes diverging
// through NEWUOA's branches serialise its phases), and one series' own path is a
// long latency-bound chain; so a small batch gets several lanes per series (the objective's
// harmonics and the 49-angle searches split across them), a large one one lane per series.
// lps: the most lanes (≤ 8) that keep the fit within one wave per SIMD; gpw: the series spread
// over every SIMD; wpb: below.  The canonical
// objective makes the records the same bits for every shape.  Options fit_lps, fit_lanes,
// fit_wpb override (A/B).
struct FitShape {
    int lps, gpw, wpb;
    bool mc;  // the series' moments cached in LDS (k_fit_harmonic<lps, true>)
    unsigned grid;
    size_t lds;
};
// offs: fitoffsets (the FC columns' moments are cached too)
FitShape fit_shape(long long P, int n_cu, bool offs) {
    const long long simds = 4LL * std::max(1, n_cu);
    FitShape f{};
    f.lps = 1;
    for (int l = 8; l >= 2; l >>= 1)
        if ((P + 64 / l - 1) / (64 / l) <= simds) {
            f.lps = l;
            break;
        }
    if (opt(O_FIT_LPS) > 0) f.lps = (int)opt(O_FIT_LPS);
    const long long cap = 64 / f.lps;
    long long gpw = (P + simds - 1) / simds;
    gpw = std::max<long long>(1, std::min<long long>(cap, gpw));
    if (opt(O_FIT_LANES) > 0) gpw = std::min<long long>(cap, opt(O_FIT_LANES));
    f.gpw = (int)gpw;
    const long long waves = (P + gpw - 1) / gpw;
    // 4 waves per workgroup once the waves outnumber the CUs with several lanes per series
    // (C4 rank: 0.90 → 0.86 ms); otherwise 1 — waves sharing a CU slow each other (r5 sweep:
    // 32 series 0.31 vs 0.52 ms, C3 2.60 vs 2.81 ms)
    f.wpb = (f.lps > 1 && waves > n_cu) ? 4 : 1;
    if (opt(O_FIT_WPB) > 0) f.wpb = (int)std::min(4LL, opt(O_FIT_WPB));
    f.wpb = (int)std::max(1LL, std::min<long long>(f.wpb, waves));
    f.grid = (unsigned)((waves + f.wpb - 1) / f.wpb);
    const size_t slots = (size_t)f.wpb * (size_t)f.gpw;
    f.lds = slots * sizeof(Newuoa<2, 5, true, 1>);
    // the moments in LDS (several lanes per series only: at one lane per series — C3 — the
    // 64 series of a wave would take 50 KB more per wave, fewer waves per CU); within 128 KB
    const size_t mlds = slots * (size_t)HARM_ROWS * sizeof(double) * (offs ? 2 : 1);
    f.mc = f.lps > 1 && opt(O_FIT_MCACHE) != 0 && f.lds + mlds <= 128 * 1024;
    if (f.mc) f.lds += mlds;
    return f;
}

hipError_t launch_fit(const FitShape &fs, Problem pb, const Info *info, const double *mom,
                      const double *aux, const double *momG, long long PG, const double *d0,
                      Param *out, double *raw, int *list, int *count, hipStream_t s) {
    pb.fit_lanes = fs.gpw;
    const dim3 g(fs.grid), b(64 * fs.wpb);
    hipError_t e = hipSuccess;
    auto go = [&](auto kern) {
        if (fs.lds > 48 * 1024) {  // beyond the default dynamic-LDS limit (C3: 4 × 64 states)
            e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)fs.lds);
            if (e != hipSuccess) return;
        }
        kern<<<g, b, fs.lds, s>>>(pb, info, mom, aux, momG, PG, d0, out, raw, list, count);
        e = hipGetLastError();
    };
    switch (fs.lps * 2 + (fs.mc ? 1 : 0)) {
        case 17: go(k_fit_harmonic<8, true>); break;
        case 16: go(k_fit_harmonic<8, false>); break;
        case 9: go(k_fit_harmonic<4, true>); break;
        case 8: go(k_fit_harmonic<4, false>); break;
        case 5: go(k_fit_harmonic<2, true>); break;
        case 4: go(k_fit_harmonic<2, false>); break;
        default: go(k_fit_harmonic<1, false>); break;
    }
    return e;
}

void moment_grid(long long N, long long P, int n_cu, bool harmonic, bool mfma, int &units,
                 long long &unit_len, long long &chunk, int &nch, bool faint = false) {
    const long long per = mfma ? MM_PIX : 64;
    const long long npg = (P + per - 1) / per;
    // at most 26 units: 26 (not 32) makes both the C3 batch (782 groups: 79.4 waves) and its
    // 8-way shard of 12 500 series (98 groups: 9.95 waves) fill their last wave of workgroups.
    // Faint series (state-split partials, their own records): 32 units, which fill the C5 batch
    // (32 groups: 4 waves; with 26, 3.25 → a quarter-filled last wave: moments 2.1 → 1.65 ms,
    // GPD_UNITS A/B, r3) and a faint 1e5 batch (97.75 waves).
    long long umax = faint ? 32 : 26;
    if (opt(O_UNITS) > 0) umax = opt(O_UNITS);  // A/B only
    long long U = std::min<long long>(umax, std::max<long long>(1, (N + 255) / 256));
    long long ulen = (N + U - 1) / U;
    ulen = (ulen + MM_TS - 1) / MM_TS * MM_TS;
    U = (N + ulen - 1) / ulen;
    long long upw = 1;
    if (harmonic && mfma && n_cu > 0) {
        long long best = LLONG_MAX;
        for (long long w = 1; w <= U; ++w) {
            const long long wg = npg * ((U + w - 1) / w);
            const long long cost = (wg + n_cu - 1) / n_cu * w;
            if (cost <= best) {
                best = cost;
                upw = w;
            }
        }
    }
    if (opt(O_UPW) > 0) upw = std::min(U, opt(O_UPW));  // A/B only
    units = (int)U;
    unit_len = ulen;
    chunk = mfma ? upw * ulen : ulen;
    nch = (int)((U + (chunk / ulen) - 1) / (chunk / ulen));
}

Layout plan(long long N, long long P, long long n_fc, bool faint, bool harmonic, bool phbuf,
            bool mfma, int n_cu, bool harm_offs, bool windowed = false, int exact_g = 1,
            bool fp32 = false, bool mcache = true) {
    Layout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off += align_up(bytes);
        return o;
    };
    moment_grid(N, P, n_cu, harmonic, mfma, L.units, L.unit_len, L.chunk, L.nch, faint);
    const long long U = L.units;
    const long long nch = U;  // partial-moment sets (units)
    L.info = take(sizeof(Info));
    L.prof = take(PROF_LEN * sizeof(unsigned long long));  // diagnostic counters
    L.prep = take((size_t)((N + PREP_PER - 1) / PREP_PER) * 4 * sizeof(double));  // k_prepare_part
    // cos/sin table, padded to whole MM_TS-sample tiles (k_table_mix fills the padding)
    L.tab = take(harmonic ? (size_t)((N + MM_TS - 1) / MM_TS * MM_TS) * 2 * KH * sizeof(double) : 0);
    // windowed series: k_moments_win writes mom directly (no partial moments)
    // (faint: one slot per unit and state, FST_SLOTS; state masks of the units; the deferred
    // samples' list and their per-state moments, k_faint_defer / k_moments_fix)
    const bool fsplit = harmonic && !windowed && faint;
    L.part = take(harmonic && !windowed
                      ? (size_t)nch * (fsplit ? FST_SLOTS : 1) * NMOM * P * sizeof(double) : 0);
    L.smask = take(fsplit ? (size_t)U * sizeof(unsigned) : 0);
    // (+ the header, + k_faint_defer_count's 6 ints per block of 1024 tiles)
    L.dlist = take(fsplit ? (size_t)(2 * ((N + MM_TS - 1) / MM_TS) + 6 +
                             6 * ((N + MM_TS - 1) / MM_TS / DEFER_TILES + 1)) * sizeof(int) : 0);
    L.fixp = take(fsplit ? (size_t)FST_SLOTS * NMOM * P * sizeof(double) : 0);
    L.ftab = take(fsplit ? (size_t)((N + MM_TS - 1) / MM_TS) * MM_TS * 2 * KH * sizeof(double) : 0);
    // fused faint statistics: per (unit, state) slot, S1/S2 of the two sample halves per series,
    // the counts per slot, the deferred samples' (n, S1, S2) per state
    L.fsp = take(fsplit ? (size_t)nch * FST_SLOTS * 4 * P * sizeof(double) : 0);
    L.fcnt = take(fsplit ? (size_t)nch * FST_SLOTS * sizeof(int) : 0);
    L.fixs = take(fsplit ? (size_t)FST_SLOTS * 3 * P * sizeof(double) : 0);
    L.mom = take(harmonic ? (size_t)NMOM * P * sizeof(double) : 0);
    L.aux = take((size_t)P * 4 * sizeof(double));
    L.fstat = take(faint ? (size_t)P * 16 * sizeof(double) : 0);
    L.raw = take((size_t)P * 2 * sizeof(double));
    L.list = take((size_t)(P + 64 + kMaxCohorts) * sizeof(int));  // + per-cohort counters
    L.phbuf = take(phbuf ? (size_t)n_fc * N * sizeof(c64) : 0);
    // harmonic fitoffsets: G moments of the FC columns (same chunking), Σ d per series
    L.partG = take(harm_offs ? (size_t)nch * NMOM * n_fc * sizeof(double) : 0);
    L.momG = take(harm_offs ? (size_t)NMOM * n_fc * sizeof(double) : 0);
    L.auxG = take(harm_offs ? (size_t)4 * n_fc * sizeof(double) : 0);
    L.fcid = take(harm_offs ? (size_t)n_fc * sizeof(int32_t) : 0);
    L.d0 = take(harm_offs ? (size_t)2 * P * sizeof(double) : 0);
    // exact evaluator: one model-cache slot of N complex per workgroup of the fit grid
    // (min(P, 1024) workgroups), or per series with the multi-workgroup split, when that stays
    // below 8 GB; mcache = false (option exact_mcache = 0, A/B): none, the residual pass
    // evaluates the model again
    const long long mc_slots = exact_g > 1 ? P : std::min<long long>(P, 1024);
    const size_t mc_bytes = (size_t)mc_slots * (size_t)N * sizeof(c64);
    L.mstride = (!harmonic && mcache && mc_bytes <= (size_t(8) << 30)) ? N : 0;
    L.mcache = take(L.mstride ? mc_bytes : 0);
    // multi-workgroup exact fit: per-series block totals (2 slots × 8 blocks × 8 values) and
    // arrival counters (zeroed per launch)
    L.xtot = take(exact_g > 1 ? (size_t)P * 2 * CR_BLOCKS * CR_NV * sizeof(double) : 0);
    L.xcnt = take(exact_g > 1 ? (size_t)(P + 3) / 4 * 16 : 0);
    // one-pass faint statistics: |d| scratch for a cohort of series (≤ 4 GB; MALL-sized cohorts
    // of ~192 MB measured no faster: 3.54 vs 3.34 ms on C5), block totals of the cohort
    L.fs_mmax = (int)((N + 2047) / 2048);
    L.fs1 = faint && !windowed;
    const long long fs_mb = std::max(1LL, opt(O_FS_COHORT_MB));
    L.fs_pc = std::max<long long>(1, std::min<long long>(
        P, (fs_mb << 20) / ((long long)FS_G * L.fs_mmax * 256 * 8)));
    L.fs_pc = std::min<long long>(L.fs_pc, (1LL << 31) / FS_G - 1);
    L.fsx = take(L.fs1 ? (size_t)L.fs_pc * FS_G * L.fs_mmax * 256 * sizeof(double) : 0);
    L.fsc = take(L.fs1 ? (size_t)L.fs_pc * FS_G * (FS_NV + 8) * sizeof(double) : 0);
    L.xr32 = take(fp32 ? (size_t)N * sizeof(float) : 0);  // F_FP32 phase table
    L.pht = take(!harmonic && !fp32 ? (size_t)N * 3 * sizeof(uint64_t) : 0);
    L.total = off;
    return L;
}

// One-pass faint statistics over P series in cohorts of pc (k_faint_p1 → k_faint_p2 →
// k_faint_fin; the cohort's |d| scratch stays in the MALL between the first two).
hipError_t run_faint_onepass(const Problem &pb, double *fstat, double *scr, double *xt,
                             long long pc, int mmax, bool is_c32, hipStream_t stream) {
    double *x2 = xt + (size_t)pc * FS_G * FS_NV;
    for (long long k0 = 0; k0 < pb.P; k0 += pc) {
        const long long np = std::min<long long>(pc, pb.P - k0);
        const unsigned grid = (unsigned)(np * FS_G);
        if (is_c32)
            k_faint_p1<c32><<<grid, 256, 0, stream>>>(pb, k0, mmax, scr, xt);
        else
            k_faint_p1<c64><<<grid, 256, 0, stream>>>(pb, k0, mmax, scr, xt);
        k_faint_p2<<<grid, 256, 0, stream>>>(pb, mmax, scr, xt, x2);
        k_faint_fin<<<(unsigned)np, 64, 0, stream>>>(k0, xt, x2, fstat);
    }
    return hipGetLastError();
}

// Host copy workers (gpd_demodulateall): a persistent pool that spreads host copies — and the
// first touch of the caller's fresh output pages, which dominates them — over threads.  At most
// 16 threads (the CPU share of one GPU on the MI355X boxes), fewer if the process may run on
// fewer CPUs.  run(n, fn) calls fn(0..n-1) on the pool's threads and the caller's, returns when
// all are done; one job at a time.  Leaked on purpose (no join during static destruction).
class HostPool {
  public:
    static HostPool &get() {
        static HostPool *p = new HostPool();
        return *p;
    }
    int size() const { return n_; }
    void run(int n, const std::function<void(int)> &fn) {
        std::lock_guard<std::mutex> one(run_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &fn;
            njob_ = n;
            next_.store(0);
            acked_ = 0;
            ++gen_;
        }
        cv_.notify_all();
        work(fn, n);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return acked_ == n_ - 1; });  // every worker is done with this job
    }

  private:
    HostPool() {
        int ncpu = 8;
        cpu_set_t cs;
        if (sched_getaffinity(0, sizeof cs, &cs) == 0) ncpu = CPU_COUNT(&cs);
        n_ = std::max(1, std::min(16, ncpu));
        for (int i = 1; i < n_; ++i) th_.emplace_back([this] { loop(); });
    }
    void work(const std::function<void(int)> &fn, int n) {
        for (int i; (i = next_.fetch_add(1)) < n;) fn(i);
    }
    void loop() {
        unsigned long seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            const std::function<void(int)> *fn = job_;
            const int n = njob_;
            lk.unlock();
            work(*fn, n);
            lk.lock();
            if (++acked_ == n_ - 1) done_.notify_all();
        }
    }
    int n_ = 1;
    std::vector<std::thread> th_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int njob_ = 0, acked_ = 0;
    unsigned long gen_ = 0;
    std::atomic<int> next_{0};
};

// Copy ncols columns of rows elements (src: element size ses, leading dimension sld; dst: des,
// dld) with the host pool, in pieces of about 1 MB; ses == des copies, ses = 16 → des = 8
// rounds ComplexF64 to ComplexF32 (Complex{Float32}.(…): each part rounded to nearest).
void pool_copy_cols(char *dst, size_t des, int64_t dld, const char *src, size_t ses, int64_t sld,
                    int64_t rows, int64_t ncols) {
    const int64_t per = std::max<int64_t>(1, (int64_t)(1 << 20) / (int64_t)ses);  // rows per piece
    const int64_t pieces_per_col = (rows + per - 1) / per;
    const int64_t npieces = pieces_per_col * ncols;
    HostPool::get().run((int)npieces, [&](int i) {
        const int64_t c = i / pieces_per_col, r0 = (i % pieces_per_col) * per;
        const int64_t nr = std::min(per, rows - r0);
        const char *s = src + ((size_t)c * sld + r0) * ses;
        char *d = dst + ((size_t)c * dld + r0) * des;
        if (ses == des) {
            std::memcpy(d, s, (size_t)nr * ses);
        } else {
            const double *sv = (const double *)s;
            float *dv = (float *)d;
            for (int64_t k = 0; k < 2 * nr; ++k) dv[k] = (float)sv[k];
        }
    });
}

// One store per page of ncols columns of rows elements (element size es, leading dimension ld),
// inside each column's bytes only: the page faults of a fresh destination taken up front, in
// parallel, rather than inside the copy that follows (which overwrites every byte stored here).
void pool_touch_cols(char *dst, size_t es, int64_t ld, int64_t rows, int64_t ncols) {
    constexpr int64_t kPage = 4096;
    const int64_t per = std::max<int64_t>(1, (int64_t)(1 << 20) / (int64_t)es);
    const int64_t pieces_per_col = (rows + per - 1) / per;
    HostPool::get().run((int)(pieces_per_col * ncols), [&](int i) {
        const int64_t c = i / pieces_per_col, r0 = (i % pieces_per_col) * per;
        const int64_t nr = std::min(per, rows - r0);
        volatile char *b = dst + ((size_t)c * ld + r0) * es, *e = b + nr * es;
        for (volatile char *q = b; q < e;
             q = (volatile char *)(((uintptr_t)q + kPage) & ~(uintptr_t)(kPage - 1)))
            *q = 0;
    });
}

// Copy the elements [e0, e1) of a P×N ComplexF64 matrix with contiguous columns (ld N), held
// contiguously at src, into the caller's columns (dst: element size des, leading dimension dld;
// des = 8 rounds to ComplexF32 as pool_copy_cols), in pieces of about 1 MB within columns.
void pool_copy_range(char *dst, size_t des, int64_t dld, const char *src, int64_t N, int64_t e0,
                     int64_t e1) {
    constexpr size_t ses = 16;
    const int64_t per = (int64_t)(1 << 20) / (int64_t)ses;
    struct Piece {
        int64_t col, r0, nr, off;  // off: element offset in src
    };
    std::vector<Piece> pcs;
    for (int64_t c = e0 / N; c * N < e1; ++c) {
        const int64_t r0 = std::max<int64_t>(0, e0 - c * N), r1 = std::min<int64_t>(N, e1 - c * N);
        for (int64_t r = r0; r < r1; r += per)
            pcs.push_back({c, r, std::min(per, r1 - r), c * N + r - e0});
    }
    HostPool::get().run((int)pcs.size(), [&](int i) {
        const Piece &q = pcs[i];
        const char *sp = src + (size_t)q.off * ses;
        char *d = dst + ((size_t)q.col * dld + q.r0) * des;
        if (des == ses) {
            std::memcpy(d, sp, (size_t)q.nr * ses);
        } else {
            const double *sv = (const double *)sp;
            float *dv = (float *)d;
            for (int64_t k = 0; k < 2 * q.nr; ++k) dv[k] = (float)sv[k];
        }
    });
}

// The output staging ring of a device (host_batch, out_kind 1/2): kStageSlots × kStageSlotBytes
// (64 MB) whatever the exposure's length (advisor r5: the whole P×N×16 B used to be pinned,
// grow-only).  Pinned (hipHostMalloc) by default; if that fails — or with option stage_pinned = 0
// — pageable memory (hipMemcpyAsync into it returns once the bytes are staged: the same bytes,
// less overlap), and a failed pinned allocation is not retried on every call.
constexpr int kStageSlots = 4;
constexpr size_t kStageSlotBytes = (size_t)16 << 20;

void free_stage(DevCtx *cx) {
    if (cx->hpin) {
        if (cx->hpin_pinned)
            (void)hipHostFree(cx->hpin);
        else
            std::free(cx->hpin);
    }
    cx->hpin = nullptr;
    cx->hpin_pinned = false;
}

bool ensure_stage(DevCtx *cx) {
    const bool want_pin = opt(O_STAGE_PINNED) != 0 && !cx->hpin_nopin;
    if (cx->hpin && cx->hpin_pinned == want_pin) return true;
    free_stage(cx);
    const size_t bytes = (size_t)kStageSlots * kStageSlotBytes;
    if (want_pin) {
        if (hipHostMalloc((void **)&cx->hpin, bytes, hipHostMallocDefault) == hipSuccess) {
            cx->hpin_pinned = true;
            return true;
        }
        (void)hipGetLastError();
        cx->hpin = nullptr;
        cx->hpin_nopin = true;
    }
    cx->hpin = (char *)std::malloc(bytes);
    return cx->hpin != nullptr;
}

const char *kErrStr[] = {"ok", "invalid argument", "HIP runtime error", "no HIP device",
                         "out of device memory", "harmonic method unsafe for these timestamps"};

}  // namespace

extern "C" {

int gpd_version(void) { return GPD_ABI_VERSION; }

// build provenance: the tree id build.py computes over the sources and flags (build.tree_id),
// also kept as a marker string that build.py reads from the library's bytes
#ifndef GPD_BUILD_ID
#define GPD_BUILD_ID "unknown"
#endif
__attribute__((used)) static const char kBuildIdMarker[] = "GPD_BUILD_ID=" GPD_BUILD_ID;
const char *gpd_build_id(void) { return kBuildIdMarker + 13; }

const char *gpd_strerror(int code) {
    if (code > 0 || code < -5) return "unknown error";
    return kErrStr[-code];
}

int gpd_set_option(const char *name, int64_t value) {
    const int i = opt_find(name);
    if (i < 0) return GPD_E_ARG;
    g_opt[i].store(value, std::memory_order_relaxed);
    return GPD_OK;
}

int gpd_get_option(const char *name, int64_t *value) {
    const int i = opt_find(name);
    if (i < 0 || !value) return GPD_E_ARG;
    *value = opt((OptId)i);
    return GPD_OK;
}

void gpd_reset_options(void) {
    for (int i = 0; i < O_COUNT; ++i) g_opt[i].store(kOpt[i].def, std::memory_order_relaxed);
}

const char *gpd_option_name(int index) {
    return index >= 0 && index < O_COUNT ? kOpt[index].name : nullptr;
}

int gpd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int gpd_release(int device) {
    if (device < 0 || device >= gpd_device_count()) return GPD_E_ARG;
    DevCtx *cx = ctx_for(device);
    std::lock_guard<std::mutex> hlk(cx->hmu);
    std::lock_guard<std::mutex> lk(cx->mu);
    if (hipSetDevice(device) != hipSuccess) return GPD_E_HIP;
    if (cx->hstream) (void)hipStreamSynchronize(cx->hstream);
    if (cx->cstream) (void)hipStreamSynchronize(cx->cstream);
    if (cx->ostream) (void)hipStreamSynchronize(cx->ostream);
    if (cx->done) (void)hipEventSynchronize(cx->done);
    (void)hipFree(cx->ws);
    (void)hipFree(cx->harena);
    free_stage(cx);
    cx->ws = cx->harena = nullptr;
    cx->ws_cap = cx->harena_cap = 0;
    cx->last_fstat = nullptr;  // pointed into the freed workspace (advisor r4)
    cx->last_fstat_P = 0;
    return GPD_OK;
}

}  // extern "C"

// Whole device pipeline.  bphi == nullptr: fit (gpd_fit_batch_dev); else evaluate χ² at
// (bphi[2k], bphi[2k+1]) for every series (gpd_chi2_batch_dev).
// is_c32: d and fc hold ComplexF32 elements (gpd_c32), widened to Float64 on load.
static int pipeline_dev(int64_t n_samples, int64_t n_pixels, const double *t, const void *d,
                        int64_t ldd, const void *fc, int64_t n_fc, int64_t ldfc,
                        const int32_t *fc_of_pixel, const int8_t *state, double omega,
                        const double *xinit, uint32_t flags, int32_t maxfun,
                        gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo,
                        const double *bphi, int device, void *stream_, char *errbuf,
                        size_t errlen, int64_t window = 0, bool is_c32 = false) {
    if (window < 0 || (window > 0 && bphi)) {
        set_err(errbuf, errlen, "gpd_fit_windows: window must be >= 0 (and fits only)");
        return GPD_E_ARG;
    }
    if (n_samples < (window > 0 ? 1 : 2) || n_pixels < 1 || !t || !d || !fc || !fc_of_pixel ||
        !out_params || ldd < n_samples || ldfc < n_samples || n_fc < 1 ||
        (out_demod && ldo < n_samples)) {
        set_err(errbuf, errlen, "gpd_fit_batch_dev: invalid shapes/pointers (N=%lld P=%lld)",
                (long long)n_samples, (long long)n_pixels);
        return GPD_E_ARG;
    }
    if (n_pixels * (window > 0 ? (n_samples + window - 1) / window : 1) > (int64_t)0x7fffff00) {
        set_err(errbuf, errlen, "gpd_fit_batch_dev: too many series");
        return GPD_E_ARG;
    }
    if ((flags & GPD_METHOD_EXACT) && (flags & GPD_METHOD_HARMONIC)) {
        set_err(errbuf, errlen, "gpd_fit_batch_dev: both METHOD bits set");
        return GPD_E_ARG;
    }
    const bool fp32 = (flags & GPD_FP32) != 0;
    if (fp32 && (flags & (GPD_FIT_OFFSETS | GPD_METHOD_HARMONIC))) {
        set_err(errbuf, errlen, "gpd_fit_batch_dev: GPD_FP32 is the exact evaluator without "
                                "fitoffsets (not with FIT_OFFSETS or METHOD_HARMONIC)");
        return GPD_E_ARG;
    }
    int ndev = gpd_device_count();
    if (ndev <= 0) {
        set_err(errbuf, errlen, "gpd_fit_batch_dev: no HIP device visible");
        return GPD_E_NODEV;
    }
    if (device < 0 || device >= ndev) {
        set_err(errbuf, errlen, "gpd_fit_batch_dev: device %d out of range", device);
        return GPD_E_ARG;
    }
    HIP_TRY(hipSetDevice(device));
    hipStream_t stream = (hipStream_t)stream_;
    const bool faint = state != nullptr;
    const bool offs = (flags & GPD_FIT_OFFSETS) != 0;
    // fp64 MFMA moment pass (producer/consumer kernel, non-temporal series loads); the VALU
    // kernel when a series row or the cos/sin table exceeds the buffer descriptors' 32-bit
    // offsets (N ≳ 1e6 samples) — option moments = 1 forces it (tests of that fallback);
    // moments = 2..7: the diagnostics build's timing variants
    const long long mk = opt(O_MOMENTS);
    // buffer descriptors of the MFMA kernels address 128 series rows / the cos-sin table
    // with 32-bit offsets
    const double esz = is_c32 ? 8.0 : 16.0;  // bytes per stored complex element
    const bool use_mfma = mk != 1 &&
                          (double)MM_PIX * (double)ldd * esz < 2147483648.0 &&
                          (double)(n_samples + MM_TS) * KH * 16.0 < 2147483648.0;
    // mixed-precision moment kernel (harmonics 17..24 on split-bf16 MFMAs);
    // option mix = 0 keeps all harmonics on the f64 MFMAs (A/B runs and precision checks; read
    // per call so a test can switch it)
    const bool mix = opt(O_MIX) != 0;
    // Harmonic fitoffsets (non-faint, on request): the χ² of the 2×2 system needs the moments
    // G_n of the FC phasors (producer/consumer kernel in UNIT mode over the FC columns) and Σ d
    // per series.  METHOD_EXACT uses the exact evaluator; so do windows with fitoffsets.
    const bool harm_offs_ok =
        !faint && use_mfma && (double)MM_PIX * (double)ldfc * esz < 2147483648.0;
    // Offsets default to the exact evaluator: the 2×2 system is ill-conditioned for small b and
    // the flat landscape turns the expansion's ~1e-14 χ² rounding into ~1e-10 moves of NEWUOA's
    // iterate; METHOD_HARMONIC asks for the fast path anyway (parity ~1e-9).
    // Windows of ≥ HARM_MIN_SPAN samples: harmonic moments from k_moments_win (a shorter last
    // window is re-fitted exactly); shorter windows: the exact evaluator.
    const long long harm_min = std::max(1LL, opt(O_HARM_MIN_SPAN));  // HARM_MIN_SPAN; sweeps only
    const bool want_exact =
        fp32 || (flags & GPD_METHOD_EXACT) || (window > 0 && window < harm_min) ||
        (offs && !(harm_offs_ok && window == 0 && (flags & GPD_METHOD_HARMONIC)));
    if ((flags & GPD_METHOD_HARMONIC) && want_exact) {
        set_err(errbuf, errlen, "gpd_fit_batch_dev: harmonic method unavailable here "
                                "(fitoffsets with faint states or windows, short windows)");
        return GPD_E_ARG;
    }
    const bool harmonic = !want_exact;
    const bool harm_offs = harmonic && offs;
    const long long N = n_samples, ncol = n_pixels;
    const long long nwin = window > 0 ? (N + window - 1) / window : 1;
    const long long P = ncol * nwin;  // series
    // (F_FP32 forms its Float32 phasor z/|z| from the raw FC columns: no phasor buffer)
    const bool phbuf = want_exact && !fp32 && (size_t)n_fc * N * sizeof(c64) <= (size_t(4) << 30);

    DevCtx *cx = ctx_for(device);
    std::lock_guard<std::mutex> lk(cx->mu);
    if (cx->n_cu == 0) HIP_TRY(hipDeviceGetAttribute(&cx->n_cu, hipDeviceAttributeMultiprocessorCount, device));
    // Small whole-exposure exact fits (one exposure: 32 series) spread each series over G
    // workgroups, one per CU (all resident: the per-series barrier needs its G parts on chip);
    // the canonical reduction order makes the records identical for every G.  Option exact_g
    // forces G (tests of that identity).
    int exact_g = 1;
    if (want_exact && !bphi && window == 0) {
        const long long p8 = (P + 7) / 8 * 8;
        // no more parts than canonical blocks that hold samples (N ≤ 1792 leaves some empty)
        const long long filled = std::min<long long>(8, (N + 255) / 256);
        for (int gg = 8; gg >= 2 && exact_g == 1; gg >>= 1)
            if (p8 * gg <= cx->n_cu && gg <= filled) exact_g = gg;
        if (const long long f = opt(O_EXACT_G)) {
            if ((f == 1 || f == 2 || f == 4 || f == 8) && p8 * f <= (long long)cx->n_cu) exact_g = (int)f;
        }
    }
    // (r5: the measured-slower exact forms of r4 — the cohort form, the LDS model cache and the
    // split form, DESIGN.md §12 — are gone from the library; git history keeps them)
    const Layout L = plan(N, P, n_fc, faint, harmonic, phbuf, use_mfma, cx->n_cu, harm_offs,
                          window > 0, exact_g, fp32, opt(O_EXACT_MCACHE) != 0);
    if (cx->ws_cap < L.total) {
        if (cx->ws) {
            cx->last_fstat = nullptr;  // points into the workspace being freed (advisor r4)
            cx->last_fstat_P = 0;
            HIP_TRY(hipDeviceSynchronize());
            HIP_TRY(hipFree(cx->ws));
            cx->ws = nullptr;
            cx->ws_cap = 0;
        }
        hipError_t e = hipMalloc(&cx->ws, L.total);
        if (e != hipSuccess) {
            set_err(errbuf, errlen, "gpd_fit_batch_dev: workspace of %zu bytes: %s", L.total,
                    hipGetErrorString(e));
            (void)hipGetLastError();
            return GPD_E_OOM;
        }
        cx->ws_cap = L.total;
    }
    if (!cx->done) {
        HIP_TRY(hipEventCreateWithFlags(&cx->done, hipEventDisableTiming));
        for (int i = 0; i < kMaxEv; ++i) HIP_TRY(hipEventCreate(&cx->ev[i]));
    } else {
        HIP_TRY(hipStreamWaitEvent(stream, cx->done, 0));
    }
    char *ws = cx->ws;
    Info *info = (Info *)(ws + L.info);
    double *tab = (double *)(ws + L.tab);
    double *part = (double *)(ws + L.part);
    double *mom = (double *)(ws + L.mom);
    double *aux = (double *)(ws + L.aux);
    double *fstat = (double *)(ws + L.fstat);
    cx->last_fstat = faint ? fstat : nullptr;
    cx->last_fstat_P = faint ? P : 0;
    double *raw = (double *)(ws + L.raw);
    int *list = (int *)(ws + L.list);
    int *count = list + P;
    c64 *ph = (c64 *)(ws + L.phbuf);

    Problem pb;
    pb.N = N;
    pb.P = P;
    pb.t = t;
    pb.d = is_c32 ? nullptr : (const c64 *)d;
    pb.d32 = is_c32 ? (const c32 *)d : nullptr;
    pb.ldd = ldd;
    pb.fc = is_c32 ? nullptr : (const c64 *)fc;
    pb.fc32 = is_c32 ? (const c32 *)fc : nullptr;
    pb.ldfc = ldfc;
    pb.n_fc = n_fc;
    pb.fcop = fc_of_pixel;
    pb.state = state;
    pb.omega = omega;
    pb.flags = flags;
    pb.maxfun = maxfun <= 0 ? 60 : std::max(maxfun, 6);
    pb.has_xinit = xinit != nullptr;
    pb.x0 = xinit ? xinit[0] : 0.0;
    pb.x1 = xinit ? xinit[1] : 0.0;
    pb.win = window;
    pb.ncol = ncol;
    pb.harm_min = harm_min;
    pb.prof = (unsigned long long *)(ws + L.prof);
    pb.fit_lanes = 0;
    pb.xr32 = fp32 ? (const float *)(ws + L.xr32) : nullptr;
    pb.pht = nullptr;
    Param *outp = (Param *)out_params;

    int nt = 0, ne = 0;
    // GPD_SYNC_DEBUG=1: synchronise after every stage and name the stage that faulted
    const bool sync_debug = opt(O_SYNC_DEBUG) != 0;
    auto rec = [&](hipStream_t s) -> int {  // a timing event on stream s (index, or -1)
        if (ne >= kMaxEv) {
            static bool warned = false;
            if (!warned) fprintf(stderr, "gpdemod: timing events exhausted; timings truncated\n");
            warned = true;
            return -1;
        }
        (void)hipEventRecord(cx->ev[ne], s);
        return ne++;
    };
    // interval [beg, new event on s] named `name`; returns the new event's index
    auto mark_on = [&](hipStream_t s, int beg, const char *name) -> int {
        if (sync_debug) {
            const hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) fprintf(stderr, "gpdemod: stage %s: %s\n", name, hipGetErrorString(e));
        }
        const int e = rec(s);
        if (e >= 0 && beg >= 0 && nt < kMaxTimers) {
            cx->tname[nt] = name;
            cx->tbeg[nt] = beg;
            cx->tend[nt] = e;
            ++nt;
        }
        return e;
    };
    int lastA = rec(stream);  // consecutive intervals on the caller's stream
    auto mark = [&](const char *name) { lastA = mark_on(stream, lastA, name); };
    // diagnostic counters (options fit_prof, moments = 7): zeroed, read back after the kernel
    unsigned long long prof_h[PROF_LEN] = {};
    auto prof_reset = [&]() { return hipMemsetAsync(pb.prof, 0, sizeof prof_h, stream); };
    auto prof_read = [&]() {
        hipError_t e = hipMemcpyAsync(prof_h, pb.prof, sizeof prof_h, hipMemcpyDeviceToHost, stream);
        return e == hipSuccess ? hipStreamSynchronize(stream) : e;
    };

    {
        const unsigned np = (unsigned)((N + PREP_PER - 1) / PREP_PER);
        double *pp = (double *)(ws + L.prep);
        k_prepare_part<<<np, 256, 0, stream>>>(pb, pp);
        k_prepare_fin<<<1, 256, 0, stream>>>(pp, (int)np, info);
    }
    HIP_TRY(hipMemsetAsync(count, 0, sizeof(int), stream));
    mark("prepare");
    // Pipelined harmonic path (whole-exposure series, fits only, without fitoffsets): the
    // series are cut into cohorts; cohort c's statistics, moment pass and reduction run on the
    // caller's stream while cohort c−1's fit (latency-bound NEWUOA lanes, a few CUs) runs on the
    // side stream.  Per-series results do not depend on the cohort (fixed sample units, §7 of
    // DESIGN.md), so the records equal the one-cohort run's bit for bit.  Off by default
    // (option cohorts = n opts in): the last cohort's fit is one round of waves whose latency
    // (~1.1-1.4 ms) is exposed whatever the cohort size, so C3, C4 and C5 gained nothing
    // (profiles/r3/cohorts.txt).
    const bool fit_prof = opt(O_FIT_PROF) != 0;  // diagnostics only
    int cohorts = 1;
    if (harmonic && use_mfma && window == 0 && !bphi && !harm_offs && !fit_prof && mk < 2) {
        // measured: no gain by default; option cohorts = n opts in
        cohorts = (int)std::max(1LL, std::min<long long>(kMaxCohorts, opt(O_COHORTS)));
        cohorts = (int)std::min<long long>(cohorts, std::max<long long>(1, P / (2 * MM_PIX)));
    }
    auto ensure_side = [&]() -> hipError_t {  // the high-priority side stream and its events
        if (cx->side) return hipSuccess;
        int lo = 0, hi = 0;
        hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&cx->side, hipStreamNonBlocking, hi);
        for (int c = 0; c < kMaxCohorts && e == hipSuccess; ++c)
            e = hipEventCreateWithFlags(&cx->fork[c], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&cx->join, hipEventDisableTiming);
        return e;
    };
    // CU-masked streams: mstream on mask bits [0, mb), fstream on [mb, n_cu) (created once per
    // device context, re-created when mb changes; A/B options mom_cus and fit_cus)
    auto ensure_masked = [&](int mb) -> hipError_t {
        if (cx->mstream && cx->mbits == mb) return hipSuccess;
        hipError_t e = hipSuccess;
        if (cx->mstream) {
            e = hipStreamSynchronize(cx->mstream);
            if (e == hipSuccess && cx->fstream) e = hipStreamSynchronize(cx->fstream);
            if (e != hipSuccess) return e;
            (void)hipStreamDestroy(cx->mstream);
            if (cx->fstream) (void)hipStreamDestroy(cx->fstream);
            cx->mstream = cx->fstream = nullptr;
        }
        const int words = (cx->n_cu + 31) / 32;
        std::vector<uint32_t> lo(words, 0), hi(words, 0);
        for (int i = 0; i < cx->n_cu; ++i) (i < mb ? lo : hi)[i / 32] |= 1u << (i % 32);
        e = hipExtStreamCreateWithCUMask(&cx->mstream, (uint32_t)words, lo.data());
        if (e == hipSuccess && mb < cx->n_cu)
            e = hipExtStreamCreateWithCUMask(&cx->fstream, (uint32_t)words, hi.data());
        for (int i = 0; i < 4 && e == hipSuccess; ++i)
            if (!cx->mev[i]) e = hipEventCreateWithFlags(&cx->mev[i], hipEventDisableTiming);
        if (e == hipSuccess) cx->mbits = mb;
        return e;
    };
    // faint whole-exposure series on the MFMA kernel: state-split moments (k_moments_ws<FAINT>,
    // weighted in k_reduce_moments).  GPD_FAINT_SIDE=1 runs the statistics beside the moment
    // pass on the side stream — measured on C5 (r3): no gain, both passes stream HBM (statistics
    // 2.57 → 4.5 ms, moments 1.8 → 3.5 ms when overlapped); off by default.
    const bool fsplit_on = faint && harmonic && use_mfma && window == 0;
    const bool faint_side = opt(O_FAINT_SIDE) == 1;
    // the state-split moment pass also forms compute_mean_var_power's sums (k_moments_ws<FAINT>
    // producers, k_faint_fused_fin): one HBM pass for the faint series (r4).  Option
    // faint_stats = 1 (one-pass kernels k_faint_p1/p2/fin) or 2 (two-pass kernel) computes the
    // statistics separately instead — the exact evaluator's statistics, bit for bit the
    // oracle's (A/B and tests).
    const long long fse = opt(O_FAINT_STATS);
    const bool fused = fsplit_on && !(fse == 1 || fse == 2);
    double *fsp = (double *)(ws + L.fsp), *fixs = (double *)(ws + L.fixs);
    int *fcnt = (int *)(ws + L.fcnt);
    unsigned *smask = (unsigned *)(ws + L.smask);
    int *dlist = (int *)(ws + L.dlist);
    int *dhdr = dlist + 2 * ((N + MM_TS - 1) / MM_TS);
    int *dbsum = dhdr + 6;
    const unsigned defer_blocks = (unsigned)(((N + MM_TS - 1) / MM_TS + DEFER_TILES - 1) / DEFER_TILES);
    auto faint_defer = [&]() {
        k_faint_defer_count<<<defer_blocks, 256, 0, stream>>>(pb, dbsum);
        k_faint_defer_list<<<defer_blocks, 256, 0, stream>>>(pb, dbsum, dlist, dhdr);
    };
    double *fixp = (double *)(ws + L.fixp), *ftab = (double *)(ws + L.ftab);
    const unsigned ftab_grid = (unsigned)((N + MM_TS - 1) / MM_TS * MM_TS / 256 + 1);
    if (cohorts > 1) {
        HIP_TRY(ensure_side());
        hipStream_t side = cx->side;
        const bool tm = mix;  // the producer/consumer kernel reads the k_table_mix layout
        if (tm)
            k_table_mix<<<(unsigned)((N + MM_TS - 1) / MM_TS * MM_TS / 256 + 1), 256, 0, stream>>>(
                t, N, omega, tab);
        else
            k_table<<<(unsigned)((N + 255) / 256), 256, 0, stream>>>(t, N, omega, tab);
        mark("table");
        int *ccount = list + P + 64;  // one fallback counter per cohort
        HIP_TRY(hipMemsetAsync(ccount, 0, kMaxCohorts * sizeof(int), stream));
        // option fit_cus = r (A/B, non-faint): r CUs of every XCD run the fits of all but the
        // last cohort on a CU-masked stream, the moment passes run on the other CUs (a masked
        // stream of their own); the last cohort's fit on the side stream, every CU
        const int resv = faint ? 0 : (int)std::min<long long>(cx->n_cu / 2, 8 * opt(O_FIT_CUS));
        hipStream_t ms = stream, fs = side;
        int mcu = cx->n_cu;
        if (resv > 0) {
            HIP_TRY(ensure_masked(cx->n_cu - resv));
            HIP_TRY(hipEventRecord(cx->mev[0], stream));
            HIP_TRY(hipStreamWaitEvent(cx->mstream, cx->mev[0], 0));
            ms = cx->mstream;
            fs = cx->fstream;
            mcu = cx->n_cu - resv;
        }
        const bool fs1 = L.fs1 && fse != 2;
        const long long step = ((P + cohorts - 1) / cohorts + MM_PIX - 1) / MM_PIX * MM_PIX;
        int c = 0;
        for (long long k0 = 0; k0 < P; k0 += step, ++c) {
            const long long n = std::min(step, P - k0);
            Problem sp = pb;  // the cohort's series k0 .. k0 + n
            sp.P = n;
            sp.ncol = n;
            if (is_c32)
                sp.d32 = pb.d32 + k0 * ldd;
            else
                sp.d = pb.d + k0 * ldd;
            sp.fcop = pb.fcop + k0;
            double *fs_c = fstat + 16 * k0,
                   *part_c = part + (size_t)L.units * (faint ? FST_SLOTS : 1) * NMOM * k0,
                   *fix_c = fixp + (size_t)FST_SLOTS * NMOM * k0,
                   *fsp_c = fsp + (size_t)L.units * FST_SLOTS * 4 * k0,
                   *fixs_c = fixs + (size_t)FST_SLOTS * 3 * k0,
                   *mom_c = mom + (size_t)NMOM * k0, *aux_c = aux + 4 * k0, *raw_c = raw + 2 * k0;
            int *list_c = list + k0, *count_c = ccount + c;
            Param *out_c = outp + k0;
            if (faint && !fused) {
                if (fs1)
                    HIP_TRY(run_faint_onepass(sp, fs_c, (double *)(ws + L.fsx),
                                              (double *)(ws + L.fsc), L.fs_pc, L.fs_mmax, is_c32,
                                              stream));
                else
                    k_faint_stats<<<(unsigned)n, 256, 0, stream>>>(sp, fs_c);
                mark("faint_stats");
            }
            int units, nch;
            long long ulen, chunk;
            moment_grid(N, n, mcu, true, true, units, ulen, chunk, nch, faint);
            dim3 g((unsigned)((n + MM_PIX - 1) / MM_PIX), (unsigned)nch);
            if (faint && c == 0) {
                faint_defer();
                k_fix_table<<<ftab_grid, 256, 0, stream>>>(pb, dlist, dhdr, ftab);
                mark("faint_defer");
            }
            if (faint) k_moments_fix<<<dim3((unsigned)n, FST_SLOTS), 256, 0, stream>>>(sp, dlist, dhdr, ftab, fix_c, fixs_c);
            if (faint && is_c32 && tm)
                k_moments_ws<0, false, c32, 2, true, true><<<g, 512, 0, stream>>>(sp, tab, chunk, ulen, part_c, smask, fsp_c, fcnt, dhdr);
            else if (faint && tm)
                k_moments_ws<0, false, c64, 2, true, true><<<g, 512, 0, stream>>>(sp, tab, chunk, ulen, part_c, smask, fsp_c, fcnt, dhdr);
            else if (faint && is_c32)
                k_moments_ws<0, false, c32, 2, false, true><<<g, 512, 0, stream>>>(sp, tab, chunk, ulen, part_c, smask, fsp_c, fcnt, dhdr);
            else if (faint)
                k_moments_ws<0, false, c64, 2, false, true><<<g, 512, 0, stream>>>(sp, tab, chunk, ulen, part_c, smask, fsp_c, fcnt, dhdr);
            else if (!tm && is_c32)
                k_moments_ws<0, false, c32, 2, false><<<g, 512, 0, ms>>>(sp, tab, chunk, ulen, part_c);
            else if (!tm)
                k_moments_ws<0, false, c64, 2, false><<<g, 512, 0, ms>>>(sp, tab, chunk, ulen, part_c);
            else if (is_c32)
                k_moments_ws<0, false, c32, 2><<<g, 512, 0, ms>>>(sp, tab, chunk, ulen, part_c);
            else
                k_moments_ws<0, false, c64, 2><<<g, 512, 0, ms>>>(sp, tab, chunk, ulen, part_c);
            if (ms == stream) mark("moments");
            if (fused) {
                k_faint_fused_fin<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(
                    sp, units, fsp_c, fcnt, smask, part_c, fixs_c, fix_c, dhdr, fs_c);
                mark("faint_stats");
            }
            dim3 gr((unsigned)((n + 255) / 256), (unsigned)NMOM);
            k_reduce_moments<<<gr, 256, 0, ms>>>(part_c, units, n, info, fs_c, faint ? 2 : 0,
                                                 mom_c, aux_c, smask, fix_c, dhdr);
            if (ms == stream) mark("reduce");
            // the cohort's fit on the side stream (fit_cus: all but the last on the reserved
            // CUs), after its moments
            const bool on_resv = resv > 0 && k0 + step < P;
            hipStream_t fst = on_resv ? fs : side;
            HIP_TRY(hipEventRecord(cx->fork[c], ms));
            HIP_TRY(hipStreamWaitEvent(fst, cx->fork[c], 0));
            const int b0 = rec(fst);
            HIP_TRY(launch_fit(fit_shape(n, on_resv ? resv : cx->n_cu, (sp.flags & F_OFFSETS) != 0), sp, info, mom_c, aux_c, nullptr, n_fc,
                               nullptr, out_c, raw_c, list_c, count_c, fst));
            const int b1 = mark_on(fst, b0, "fit_harmonic");
            const unsigned xg = (unsigned)std::min<long long>(n, on_resv ? resv : 1024);
            if (fused)  // the fallback series' two-pass statistics (as above, one cohort)
                k_faint_stats_list<<<xg, 256, 0, fst>>>(sp, list_c, count_c, fs_c);
            if (faint)
                k_fit_exact<true, false, false><<<xg, EXACT_WG, 0, fst>>>(
                    sp, info, nullptr, fs_c, list_c, count_c, out_c, raw_c, ST_FALLBACK);
            else
                k_fit_exact<false, false, false><<<xg, EXACT_WG, 0, fst>>>(
                    sp, info, nullptr, fs_c, list_c, count_c, out_c, raw_c, ST_FALLBACK);
            mark_on(fst, b1, "fit_fallback");
        }
        HIP_TRY(hipEventRecord(cx->join, side));
        HIP_TRY(hipStreamWaitEvent(stream, cx->join, 0));
        if (resv > 0) {  // the reserved CUs' fits and the masked moment stream join too
            HIP_TRY(hipEventRecord(cx->mev[2], fs));
            HIP_TRY(hipStreamWaitEvent(stream, cx->mev[2], 0));
            HIP_TRY(hipEventRecord(cx->mev[3], ms));
            HIP_TRY(hipStreamWaitEvent(stream, cx->mev[3], 0));
        }
        mark("fit_tail");  // the last cohort's fit, exposed
    } else if (faint && !fused) {
        // whole-exposure series: one pass over the series, one hypot per sample (k_faint_p1/p2/
        // fin); windows: the two-pass kernel over each window's span (same bits);
        // option faint_stats = 2 forces the two-pass kernel (tests of that identity)
        const bool fs1 = L.fs1 && fse != 2;
        auto run_stats = [&](hipStream_t s) -> hipError_t {
            if (fs1)
                return run_faint_onepass(pb, fstat, (double *)(ws + L.fsx),
                                         (double *)(ws + L.fsc), L.fs_pc, L.fs_mmax, is_c32, s);
            k_faint_stats<<<(unsigned)P, 256, 0, s>>>(pb, fstat);
            return hipGetLastError();
        };
        if (fsplit_on && faint_side) {
            // the state-split moment pass does not read the statistics: they run beside it
            // on the side stream and join before the reduction
            HIP_TRY(ensure_side());
            HIP_TRY(hipEventRecord(cx->fork[0], stream));
            HIP_TRY(hipStreamWaitEvent(cx->side, cx->fork[0], 0));
            const int b0 = rec(cx->side);
            HIP_TRY(run_stats(cx->side));
            mark_on(cx->side, b0, "faint_stats");
            HIP_TRY(hipEventRecord(cx->join, cx->side));
        } else {
            HIP_TRY(run_stats(stream));
            mark("faint_stats");
        }
    }
    const unsigned exact_grid = (unsigned)std::min<long long>(P, 1024);
    bool tmix = false;  // the table holds the k_table_mix layout
    if (harmonic && cohorts > 1) {
        // fitted by the pipelined cohorts above
    } else if (harmonic) {
        // the producer/consumer kernel (non-faint whole-exposure series, also the UNIT pass
        // of harmonic fitoffsets) reads the k_table_mix layout when mixing; every other
        // moment kernel the plain rows
        const bool ws_kernel = use_mfma && window == 0;
        tmix = mix && ws_kernel;
        if (tmix)
            k_table_mix<<<(unsigned)((N + MM_TS - 1) / MM_TS * MM_TS / 256 + 1), 256, 0, stream>>>(
                t, N, omega, tab);
        else
            k_table<<<(unsigned)((N + 255) / 256), 256, 0, stream>>>(t, N, omega, tab);
        mark("table");
        if (window > 0) {
            if (faint)
                k_moments_win<true><<<(unsigned)P, 256, 0, stream>>>(pb, tab, fstat, mom, aux);
            else
                k_moments_win<false><<<(unsigned)P, 256, 0, stream>>>(pb, tab, fstat, mom, aux);
            mark("moments_win");
        } else if (use_mfma) {
            dim3 g((unsigned)((P + MM_PIX - 1) / MM_PIX), (unsigned)L.nch);
            // option mom_cus (A/B): the non-faint moment pass on a stream masked to that many CUs
            hipStream_t mst = stream;
            const long long mcus = opt(O_MOM_CUS);
            if (!faint && mcus > 0 && mcus < cx->n_cu) {
                HIP_TRY(ensure_masked((int)mcus));
                HIP_TRY(hipEventRecord(cx->mev[0], stream));
                HIP_TRY(hipStreamWaitEvent(cx->mstream, cx->mev[0], 0));
                mst = cx->mstream;
            }
            if (faint) {  // the deferred samples of the state-split pass (usually none)
                faint_defer();
                k_fix_table<<<ftab_grid, 256, 0, stream>>>(pb, dlist, dhdr, ftab);
                k_moments_fix<<<dim3((unsigned)P, FST_SLOTS), 256, 0, stream>>>(pb, dlist, dhdr, ftab, fixp, fixs);
                mark("faint_defer");
            }
            if (faint && is_c32 && tmix)  // faint series: the producer/consumer kernel, state-split
                k_moments_ws<0, false, c32, 2, true, true><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part, smask, fsp, fcnt, dhdr);
#ifdef GPD_DIAG
            // timing variants of the faint kernel (results invalid), diagnostics build only
            else if (faint && tmix && mk == 9)
                k_moments_ws<9, false, c64, 2, true, true><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part, smask, fsp, fcnt, dhdr);
            else if (faint && tmix && mk == 10)
                k_moments_ws<10, false, c64, 2, true, true><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part, smask, fsp, fcnt, dhdr);
#endif
            else if (faint && tmix)
                k_moments_ws<0, false, c64, 2, true, true><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part, smask, fsp, fcnt, dhdr);
            else if (faint && is_c32)
                k_moments_ws<0, false, c32, 2, false, true><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part, smask, fsp, fcnt, dhdr);
            else if (faint)
                k_moments_ws<0, false, c64, 2, false, true><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part, smask, fsp, fcnt, dhdr);
            else if (!tmix && is_c32)  // all-f64 MFMA variants (option mix = 0)
                k_moments_ws<0, false, c32, 2, false><<<g, 512, 0, mst>>>(pb, tab, L.chunk, L.unit_len, part);
            else if (!tmix)
                k_moments_ws<0, false, c64, 2, false><<<g, 512, 0, mst>>>(pb, tab, L.chunk, L.unit_len, part);
            else if (is_c32)  // Float32 storage: the producer/consumer kernel on 8-B elements
                k_moments_ws<0, false, c32, 2><<<g, 512, 0, mst>>>(pb, tab, L.chunk, L.unit_len, part);
#ifdef GPD_DIAG
            // timing variants (results invalid), diagnostics build only (build.py --diag)
            else if (mk == 2)  // ws_nomfma
                k_moments_ws<1><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part);
            else if (mk == 3)  // ws_noload
                k_moments_ws<2><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part);
            else if (mk == 4)  // ws_nof0
                k_moments_ws<7><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part);
            else if (mk == 5)  // ws_noq
                k_moments_ws<8><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part);
            else if (mk == 6)  // ws_mfmaonly
                k_moments_ws<5><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part);
            else if (mk == 7) {  // ws_prof: cycle split per role (stderr)
                HIP_TRY(prof_reset());
                k_moments_ws<6><<<g, 512, 0, stream>>>(pb, tab, L.chunk, L.unit_len, part);
                HIP_TRY(prof_read());
                const unsigned long long *z = prof_h + PROF_WS;
                const double pw = 4.0 * g.x * g.y, cw = pw;  // waves per role
                fprintf(stderr,
                        "ws_prof cycles/wave: producer stage %.3g issue %.3g barrier %.3g | "
                        "consumer mfma %.3g barrier %.3g\n",
                        z[0] / pw, z[1] / pw, z[2] / pw, z[3] / cw, z[4] / cw);
            }
#endif
            else  // the production kernel
                k_moments_ws<0, false, c64, 2><<<g, 512, 0, mst>>>(pb, tab, L.chunk, L.unit_len, part);
            if (mst != stream) {
                HIP_TRY(hipEventRecord(cx->mev[1], mst));
                HIP_TRY(hipStreamWaitEvent(stream, cx->mev[1], 0));
            }
        } else {
            dim3 g((unsigned)((P + 63) / 64), (unsigned)L.units);
            if (faint)
                k_moments<true><<<g, 64, 0, stream>>>(pb, tab, fstat, L.unit_len, part);
            else
                k_moments<false><<<g, 64, 0, stream>>>(pb, tab, fstat, L.unit_len, part);
        }
        if (window == 0) {
            mark("moments");
            if (fused) {
                k_faint_fused_fin<<<(unsigned)((P + 255) / 256), 256, 0, stream>>>(
                    pb, L.units, fsp, fcnt, smask, part, fixs, fixp, dhdr, fstat);
                mark("faint_stats");
            }
            if (fsplit_on && faint_side && !fused) HIP_TRY(hipStreamWaitEvent(stream, cx->join, 0));  // statistics
            dim3 gr((unsigned)((P + 255) / 256), (unsigned)NMOM);
            k_reduce_moments<<<gr, 256, 0, stream>>>(part, L.units, P, info, fstat,
                                                     fsplit_on ? 2 : (faint ? 1 : 0), mom, aux,
                                                     smask, fixp, dhdr);
            mark("reduce");
        }
        double *momG = (double *)(ws + L.momG), *d0 = (double *)(ws + L.d0);
        if (harm_offs) {
            // G_n of every FC column: the producer/consumer kernel in UNIT mode with the FC
            // columns as its series (identity fc_of_pixel → per-series FC path)
            int32_t *fcid = (int32_t *)(ws + L.fcid);
            k_iota<<<(unsigned)((n_fc + 255) / 256), 256, 0, stream>>>(fcid, n_fc);
            Problem pg = pb;
            pg.P = n_fc;
            pg.d = pb.fc;
            pg.d32 = pb.fc32;
            pg.ldd = ldfc;
            pg.fcop = fcid;
            pg.win = 0;
            pg.ncol = n_fc;
            double *partG = (double *)(ws + L.partG), *auxG = (double *)(ws + L.auxG);
            dim3 gG((unsigned)((n_fc + MM_PIX - 1) / MM_PIX), (unsigned)L.nch);
            if (is_c32 && tmix)
                k_moments_ws<0, true, c32><<<gG, 512, 0, stream>>>(pg, tab, L.chunk, L.unit_len, partG);
            else if (tmix)
                k_moments_ws<0, true><<<gG, 512, 0, stream>>>(pg, tab, L.chunk, L.unit_len, partG);
            else if (is_c32)
                k_moments_ws<0, true, c32, 0, false><<<gG, 512, 0, stream>>>(pg, tab, L.chunk, L.unit_len, partG);
            else
                k_moments_ws<0, true, c64, 0, false><<<gG, 512, 0, stream>>>(pg, tab, L.chunk, L.unit_len, partG);
            dim3 grG((unsigned)((n_fc + 255) / 256), (unsigned)NMOM);
            k_reduce_moments<<<grG, 256, 0, stream>>>(partG, L.units, n_fc, info, nullptr, 0, momG, auxG);
            k_series_sum<<<(unsigned)P, 256, 0, stream>>>(pb, d0);
            mark("offsets_moments");
        }
        if (bphi) {
            k_chi2_harmonic<<<(unsigned)((P + 63) / 64), 64, 0, stream>>>(pb, info, mom, aux, momG,
                                                                        n_fc, d0, bphi, outp);
            mark("chi2_harmonic");
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipEventRecord(cx->done, stream));
            cx->ntimers = nt;
            cx->have_timers = true;
            return GPD_OK;
        }
        if (fit_prof) {
            HIP_TRY(prof_reset());
            Problem pp = pb;
            pp.flags |= F_PROF;
            const FitShape fsh = fit_shape(P, cx->n_cu, (pb.flags & F_OFFSETS) != 0);
            HIP_TRY(launch_fit(fsh, pp, info, mom, aux, momG, n_fc, d0, outp, raw, list, count,
                               stream));
            HIP_TRY(prof_read());
            const unsigned long long *z = prof_h + PROF_FIT;
            fprintf(stderr, "fit_prof per series: objective %.3g cycles, whole fit %.3g, evals %.3g\n",
                    (double)z[0] / P, (double)z[1] / P, (double)z[2] / P);
#ifdef GPD_DIAG
            const unsigned long long *zn = prof_h + PROF_NW;
            fprintf(stderr, "fit_prof newuoa per series: trsapp %.3g biglag %.3g bigden %.3g "
                    "update %.3g init %.3g vlag/beta %.3g model-update %.3g cycles (lps %d, "
                    "series per wave %d, waves per workgroup %d, moments in LDS %d)\n",
                    (double)zn[0] / P, (double)zn[1] / P, (double)zn[2] / P, (double)zn[3] / P,
                    (double)zn[4] / P, (double)zn[5] / P, (double)zn[6] / P, fsh.lps, fsh.gpw,
                    fsh.wpb, (int)fsh.mc);
            const double nw = (double)((P + fsh.gpw - 1) / fsh.gpw);  // waves
            fprintf(stderr, "fit_prof per wave: objective %.3g trsapp %.3g biglag %.3g update %.3g "
                    "init %.3g vlag/beta %.3g model-update %.3g cycles; whole fit mean %.3g max %.3g "
                    "cycles over %llu waves\n", (double)z[4] / nw, (double)zn[8] / nw,
                    (double)zn[9] / nw, (double)zn[11] / nw, (double)zn[12] / nw,
                    (double)zn[13] / nw, (double)zn[14] / nw, (double)z[5] / (double)(z[7] ? z[7] : 1),
                    (double)z[6], (unsigned long long)z[7]);
            // the waves' timeline: start, end (100 MHz), largest evaluation count, hardware id
            const long long nwr = std::min<long long>(PROF_WV_MAX, (long long)nw);
            for (long long w = 0; w < nwr; ++w) {
                const unsigned long long *q = prof_h + PROF_WV + 4 * w;
                fprintf(stderr, "fitwave %lld %llu %llu %llu %llx\n", w, q[0], q[1], q[2], q[3]);
            }
#endif
        } else {
            HIP_TRY(launch_fit(fit_shape(P, cx->n_cu, (pb.flags & F_OFFSETS) != 0), pb, info, mom, aux, momG, n_fc, d0, outp,
                               raw, list, count, stream));
        }
        mark("fit_harmonic");
        // fallback: series whose fit left the expansion's safe range, re-fitted exactly — faint
        // ones with the two-pass statistics of the listed series (the oracle's bits), not the
        // fused ones the harmonic fit used
        // (one workgroup per CU walks the list — one round of the exact fit's one-workgroup-
        // per-CU occupancy; an empty list costs the launch of n_cu workgroups, not of 1024)
        const unsigned fb_grid = (unsigned)std::min<long long>(P, std::max(1, cx->n_cu));
        if (fused) {
            k_faint_stats_list<<<fb_grid, 256, 0, stream>>>(pb, list, count, fstat);
            mark("fallback_stats");
        }
        if (faint)
            k_fit_exact<true, false, false><<<fb_grid, EXACT_WG, 0, stream>>>(
                pb, info, nullptr, fstat, list, count, outp, raw, ST_FALLBACK);
        else if (harm_offs)
            k_fit_exact<false, true, false><<<fb_grid, EXACT_WG, 0, stream>>>(
                pb, info, nullptr, fstat, list, count, outp, raw, ST_FALLBACK);
        else
            k_fit_exact<false, false, false><<<fb_grid, EXACT_WG, 0, stream>>>(
                pb, info, nullptr, fstat, list, count, outp, raw, ST_FALLBACK);
        mark("fit_fallback");
        if (harm_offs) {
            k_refine_exact<false><<<exact_grid, EXACT_WG, 0, stream>>>(pb, info, nullptr, raw, outp);
            mark("refine_exact");
        }
    } else {
        if (fp32) {
            k_phase32<<<(unsigned)((N + 255) / 256), 256, 0, stream>>>(t, N, omega, (float *)pb.xr32);
            mark("phase32");
        } else {
            // the Payne–Hanek table of fl(ω t) (r6): the one-wave-per-SIMD fits read it in place
            // of t when every phase lies in one binade of the Payne–Hanek regime (MJD-scale
            // timestamps; ExactChi2 PHT) — built for every exact call, 24 B per sample
            uint64_t *pht = (uint64_t *)(ws + L.pht);
            k_ph_table<<<(unsigned)((N + 255) / 256), 256, 0, stream>>>(t, N, omega, pht);
            pb.pht = pht;
            mark("ph_table");
        }
        if (phbuf) {
            dim3 g((unsigned)std::min<long long>((N + 255) / 256, 256), (unsigned)n_fc);
            k_phasor<<<g, 256, 0, stream>>>(pb, ph);
            mark("phasor");
        }
        if (exact_g > 1) {
            HIP_TRY(hipMemsetAsync(ws + L.xcnt, 0, (size_t)(P + 3) / 4 * 16, stream));
            // option xspin_test (tests): the per-series barrier gives up at once (poison path)
            if (opt(O_XSPIN_TEST) > 0) pb.flags |= F_XSPIN_TEST;
        }
        // option exact_fast = 0 (A/B, tests): the evaluator's general load path everywhere
        if (opt(O_EXACT_FAST) == 0) pb.flags |= F_NOFAST;
        // option fit_prof (diagnostics): per-phase cycles of the multi-workgroup exact fit
        if (fit_prof && exact_g > 1 && !bphi) {
            pb.flags |= F_PROF;
            HIP_TRY(prof_reset());
        }
        const unsigned fit_grid =
            exact_g > 1 ? (unsigned)((P + 7) / 8 * 8 * exact_g) : exact_grid;
        // two waves per SIMD (k_fit_exact MINB = 2) when the grid needs more than one round of
        // one-wave-per-SIMD workgroups; option exact_waves = 1|2 forces it (A/B and tests)
        bool two_waves = exact_g == 1 && (long long)fit_grid * (EXACT_WG / 64) > 4LL * cx->n_cu;
        if (opt(O_EXACT_WAVES) > 0) two_waves = opt(O_EXACT_WAVES) == 2 && exact_g == 1;
        // short spans (every series or window ≤ 2048 samples = one sample per canonical slot,
        // e.g. windows of ≤ 4 s at 500 Hz): one wave per series (k_fit_exact WGT = 64; the same
        // records), no model cache, a persistent grid of two waves per SIMD — measured faster
        // from 100- to 2000-sample windows, slower on 5000 and on whole 1e5-sample series
        // (DESIGN.md §9).  Option exact_wgt = 64|256 forces it (A/B, tests).
        const long long span = window > 0 ? std::min<long long>(window, N) : N;
        bool one_wave = exact_g == 1 && span <= CR_SLOTS &&
                        P > kOneWaveMinSeriesPerCU * std::max(1, cx->n_cu);
        if (opt(O_EXACT_WGT) > 0) one_wave = exact_g == 1 && opt(O_EXACT_WGT) == 64;
        const unsigned grid64 = (unsigned)std::min<long long>(P, 8LL * std::max(1, cx->n_cu));
#define GPD_LAUNCH_EXACT(FA, OF, PH)                                                                 \
    do {                                                                                        \
        if (bphi)                                                                               \
            k_chi2_exact<FA, OF, PH><<<(unsigned)P, EXACT_WG, 0, stream>>>(pb, info, ph, fstat, \
                                                                           bphi, outp);         \
        else if (one_wave)                                                                      \
            k_fit_exact<FA, OF, PH, 2, 64><<<grid64, 64, 0, stream>>>(                         \
                pb, info, ph, fstat, nullptr, nullptr, outp, raw, 0, nullptr, 0, 1, nullptr,    \
                nullptr);                                                                       \
        else if (two_waves)                                                                   \
            k_fit_exact<FA, OF, PH, 2><<<fit_grid, EXACT_WG, 0, stream>>>(                    \
                pb, info, ph, fstat, nullptr, nullptr, outp, raw, 0,                            \
                L.mstride ? (c64 *)(ws + L.mcache) : nullptr, L.mstride, exact_g,               \
                (double *)(ws + L.xtot), (unsigned *)(ws + L.xcnt));                            \
        else {                                                                                  \
            k_fit_exact<FA, OF, PH><<<fit_grid, EXACT_WG, 0, stream>>>(                       \
                pb, info, ph, fstat, nullptr, nullptr, outp, raw, 0,                            \
                L.mstride ? (c64 *)(ws + L.mcache) : nullptr, L.mstride, exact_g,               \
                (double *)(ws + L.xtot), (unsigned *)(ws + L.xcnt));                            \
        }                                                                                       \
    } while (0)
        if (faint) {
            if (offs) { if (phbuf) GPD_LAUNCH_EXACT(true, true, true); else GPD_LAUNCH_EXACT(true, true, false); }
            else { if (phbuf) GPD_LAUNCH_EXACT(true, false, true); else GPD_LAUNCH_EXACT(true, false, false); }
        } else {
            if (offs) { if (phbuf) GPD_LAUNCH_EXACT(false, true, true); else GPD_LAUNCH_EXACT(false, true, false); }
            else { if (phbuf) GPD_LAUNCH_EXACT(false, false, true); else GPD_LAUNCH_EXACT(false, false, false); }
        }
#undef GPD_LAUNCH_EXACT
        mark(bphi ? "chi2_exact" : "fit_exact");
        if (pb.flags & F_PROF) {
            pb.flags &= ~F_PROF;
            HIP_TRY(prof_read());
            const unsigned long long *zx = prof_h + PROF_FIT;
            const double nwg = (double)P * exact_g;
            fprintf(stderr, "exact fit_prof cycles per workgroup: pass1 %.4g residual %.4g "
                    "exchange %.4g whole %.4g\n", zx[0] / nwg, zx[1] / nwg, zx[2] / nwg,
                    zx[3] / nwg);
        }
    }
    if (out_demod && !bphi) {
        const long long span = window > 0 ? std::min<long long>(window, N) : N;
        dim3 g((unsigned)std::min<long long>((span + 255) / 256, 64), (unsigned)P);
        k_output<<<g, 256, 0, stream>>>(pb, outp, raw, (c64 *)out_demod, ldo);
        mark("output");
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(cx->done, stream));
    cx->ntimers = nt;
    cx->have_timers = true;
    return GPD_OK;
}

extern "C" {

int gpd_fit_batch_dev(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c64 *d,
                      int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                      const int32_t *fc_of_pixel, const int8_t *state, double omega,
                      const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                      gpd_c64 *out_demod, int64_t ldo, int device, void *stream, char *errbuf,
                      size_t errlen) {
    return pipeline_dev(n_samples, n_pixels, t, d, ldd, fc, n_fc, ldfc, fc_of_pixel, state, omega,
                        xinit, flags, maxfun, out_params, out_demod, ldo, nullptr, device, stream,
                        errbuf, errlen);
}

int gpd_chi2_batch_dev(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c64 *d,
                       int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                       const int32_t *fc_of_pixel, const int8_t *state, double omega,
                       const double *bphi, uint32_t flags, gpd_param *out_params, int device,
                       void *stream, char *errbuf, size_t errlen) {
    if (!bphi) {
        set_err(errbuf, errlen, "gpd_chi2_batch_dev: bphi is NULL");
        return GPD_E_ARG;
    }
    return pipeline_dev(n_samples, n_pixels, t, d, ldd, fc, n_fc, ldfc, fc_of_pixel, state, omega,
                        nullptr, flags, 0, out_params, nullptr, n_samples, bphi, device, stream,
                        errbuf, errlen);
}

int gpd_fit_windows_dev(int64_t n_samples, int64_t window, int64_t n_cols, const double *t,
                        const gpd_c64 *d, int64_t ldd, const gpd_c64 *fc, int64_t n_fc,
                        int64_t ldfc, const int32_t *fc_of_col, const int8_t *state, double omega,
                        const double *xinit, uint32_t flags, int32_t maxfun,
                        gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo, int device,
                        void *stream, char *errbuf, size_t errlen) {
    if (window < 1) {
        set_err(errbuf, errlen, "gpd_fit_windows_dev: window must be >= 1");
        return GPD_E_ARG;
    }
    return pipeline_dev(n_samples, n_cols, t, d, ldd, fc, n_fc, ldfc, fc_of_col, state, omega,
                        xinit, flags, maxfun, out_params, out_demod, ldo, nullptr, device, stream,
                        errbuf, errlen, window);
}

int gpd_fit_batch_c32_dev(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c32 *d,
                          int64_t ldd, const gpd_c32 *fc, int64_t n_fc, int64_t ldfc,
                          const int32_t *fc_of_pixel, const int8_t *state, double omega,
                          const double *xinit, uint32_t flags, int32_t maxfun,
                          gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo, int device,
                          void *stream, char *errbuf, size_t errlen) {
    return pipeline_dev(n_samples, n_pixels, t, d, ldd, fc, n_fc, ldfc, fc_of_pixel, state, omega,
                        xinit, flags, maxfun, out_params, out_demod, ldo, nullptr, device, stream,
                        errbuf, errlen, 0, true);
}

int gpd_fit_windows_c32_dev(int64_t n_samples, int64_t window, int64_t n_cols, const double *t,
                            const gpd_c32 *d, int64_t ldd, const gpd_c32 *fc, int64_t n_fc,
                            int64_t ldfc, const int32_t *fc_of_col, const int8_t *state,
                            double omega, const double *xinit, uint32_t flags, int32_t maxfun,
                            gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo, int device,
                            void *stream, char *errbuf, size_t errlen) {
    if (window < 1) {
        set_err(errbuf, errlen, "gpd_fit_windows_c32_dev: window must be >= 1");
        return GPD_E_ARG;
    }
    return pipeline_dev(n_samples, n_cols, t, d, ldd, fc, n_fc, ldfc, fc_of_col, state, omega,
                        xinit, flags, maxfun, out_params, out_demod, ldo, nullptr, device, stream,
                        errbuf, errlen, window, true);
}

int gpd_last_timings(int device, const char **names, double *ms, int cap) {
    if (device < 0 || device >= gpd_device_count()) return 0;
    DevCtx *cx = ctx_for(device);
    std::lock_guard<std::mutex> lk(cx->mu);
    if (!cx->have_timers) return 0;
    if (hipSetDevice(device) != hipSuccess) return 0;
    int n = std::min(cap, cx->ntimers);
    for (int i = 0; i < n; ++i)
        if (hipEventSynchronize(cx->ev[cx->tend[i]]) != hipSuccess) return 0;
    for (int i = 0; i < n; ++i) {
        float f = 0.f;
        (void)hipEventElapsedTime(&f, cx->ev[cx->tbeg[i]], cx->ev[cx->tend[i]]);
        if (names) names[i] = cx->tname[i];
        if (ms) ms[i] = (double)f;
    }
    return n;
}

int gpd_last_faint_stats(int device, double *out, int64_t n_series) {
    if (device < 0 || device >= gpd_device_count() || !out || n_series < 1) return GPD_E_ARG;
    DevCtx *cx = ctx_for(device);
    std::lock_guard<std::mutex> lk(cx->mu);
    if (!cx->last_fstat || n_series > cx->last_fstat_P) return GPD_E_ARG;
    if (hipSetDevice(device) != hipSuccess || hipEventSynchronize(cx->done) != hipSuccess ||
        hipMemcpy(out, cx->last_fstat, (size_t)n_series * 16 * sizeof(double),
                  hipMemcpyDeviceToHost) != hipSuccess)
        return GPD_E_HIP;
    return GPD_OK;
}

}  // extern "C"

// Host-pointer driver: shard series over devices (one host thread per device), copy in, run the
// device pipeline, copy out.  bphi (host, 2 per series) selects χ²-evaluation mode.
static int host_batch(int64_t n_samples, int64_t n_pixels, const double *t, const void *d_,
                      int64_t ldd, const void *fc_, int64_t n_fc, int64_t ldfc,
                      const int32_t *fc_of_pixel, const int8_t *state, double omega,
                      const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                      gpd_c64 *out_demod, int64_t ldo, const double *bphi, int32_t n_gpus,
                      char *errbuf, size_t errlen, int64_t window = 0, bool is_c32 = false,
                      int out_kind = 0) {
    // out_kind: 0 — out_demod receives ComplexF64 columns straight from the device (pageable
    // copy); 1 — through the device's pinned staging buffer and the host pool (ComplexF64);
    // 2 — the same, rounded to ComplexF32 (out_demod then points to gpd_c32 columns)
    const size_t esz = is_c32 ? sizeof(gpd_c32) : sizeof(gpd_c64);  // stored element bytes
    const char *d = (const char *)d_, *fc = (const char *)fc_;
    if (n_samples < 2 || n_pixels < 1 || !t || !d || !fc || !fc_of_pixel || !out_params ||
        ldd < n_samples || ldfc < n_samples || n_fc < 1 || (out_demod && ldo < n_samples) ||
        window < 0) {
        set_err(errbuf, errlen, "gpd_batch: invalid shapes/pointers");
        return GPD_E_ARG;
    }
    for (int64_t k = 0; k < n_pixels; ++k) {
        if (fc_of_pixel[k] < 0 || fc_of_pixel[k] >= n_fc) {
            set_err(errbuf, errlen, "gpd_batch: fc_of_pixel[%lld]=%d outside [0,%lld)",
                    (long long)k, fc_of_pixel[k], (long long)n_fc);
            return GPD_E_ARG;
        }
    }
    const int ndev = gpd_device_count();
    if (ndev <= 0) {
        set_err(errbuf, errlen, "gpd_batch: no HIP device visible");
        return GPD_E_NODEV;
    }
    // option fake_gpus = 1 (tests): keep n_gpus shards even beyond the visible devices, shard g on
    // device g % ndev — the multi-device split (series / window ranges, FC column subsets,
    // record offsets) then runs on a one-GPU box exactly as on an 8-GPU node
    const bool fake = opt(O_FAKE_GPUS) > 0;
    int G = n_gpus <= 0 ? 1 : (fake ? std::min<int>(n_gpus, 64) : std::min<int>(n_gpus, ndev));
    const int64_t nwin = window > 0 ? (n_samples + window - 1) / window : 0;
    G = (int)std::min<int64_t>(G, window > 0 ? nwin : n_pixels);
    const int64_t Nall = n_samples;
    std::vector<int> rc(G, GPD_OK);
    std::vector<std::string> msg(G);

    auto worker = [&](int g) {
        char eb[512] = {0};
        const size_t errlen_l = sizeof eb;
        char *errbuf_l = eb;
        auto fail = [&](int code) {
            rc[g] = code;
            msg[g] = eb;
        };
        // series mode: device g owns series [p0, p1) over all samples; window mode: it owns
        // windows [w0, w1), i.e. samples [s0, s0 + N) of every column
        int64_t p0 = n_pixels * g / G, p1 = n_pixels * (g + 1) / G, s0 = 0, N = Nall, o0 = p0;
        if (window > 0) {
            const int64_t w0 = nwin * g / G, w1 = nwin * (g + 1) / G;
            p0 = 0;
            p1 = n_pixels;
            s0 = w0 * window;
            N = std::min<int64_t>(Nall, w1 * window) - s0;
            o0 = w0 * n_pixels;  // first output record (window-major)
        }
        const int64_t P = p1 - p0;
        const int64_t nrec = window > 0 ? P * ((N + window - 1) / window) : P;
        const int dev = g % ndev;
        if (hipSetDevice(dev) != hipSuccess) {
            set_err(errbuf_l, errlen_l, "hipSetDevice(%d) failed", dev);
            return fail(GPD_E_HIP);
        }
        auto chk = [&](hipError_t e, const char *what) {
            if (e != hipSuccess) {
                set_err(errbuf_l, errlen_l, "%s: %s", what, hipGetErrorString(e));
                return false;
            }
            return true;
        };
        auto cleanup = [&]() {};
        // only the FC columns this shard references travel (e.g. 8 of the 40 columns of an
        // exposure matrix passed whole as `fc`)
        int32_t cmin = INT32_MAX, cmax = 0;
        for (int64_t k = p0; k < p1; ++k) {
            cmin = std::min(cmin, fc_of_pixel[k]);
            cmax = std::max(cmax, fc_of_pixel[k]);
        }
        const int64_t nfc = (int64_t)cmax - cmin + 1;
        std::vector<int32_t> fcop_l(fc_of_pixel + p0, fc_of_pixel + p1);
        for (auto &c : fcop_l) c -= cmin;
        // H2D pipelining (option h2d_parts, r6): a harmonic fit call in series mode is cut into
        // K parts at multiples of 4 series.  Part k's diode columns — and the FC columns it is the
        // first to reference — go up on the copy stream while part k−1 computes on s, and the
        // staged demodulated columns of part k−1 come back on the output stream meanwhile (PCIe is
        // full duplex).  The records do not depend on the cut (fixed sample units, whole-series
        // fits: the shard tests), so K changes the time only.  Exact-evaluator calls stay whole
        // (their fit spreads each series over up to 8 CUs; parts would serialise those fits).
        // Automatic (0): 2 parts when the caller's data is pinned (page-locked: the copies are
        // DMA'd asynchronously), 1 for pageable data — a pageable H2D is staged by the runtime
        // and did not overlap the previous part's kernels (measured, r6: C2 3.3 → 4.0 ms at K = 2)
        const bool harm_call = window == 0 && !bphi && !(flags & (GPD_METHOD_EXACT | GPD_FP32)) &&
                               (!(flags & GPD_FIT_OFFSETS) || (flags & GPD_METHOD_HARMONIC));
        long long kopt = opt(O_H2D_PARTS);
        if (kopt <= 0) {
            hipPointerAttribute_t pa;
            const bool pinned = hipPointerGetAttributes(&pa, d) == hipSuccess && pa.type == hipMemoryTypeHost;
            (void)hipGetLastError();  // unregistered host memory reports an error: not pinned
            kopt = pinned ? 2 : 1;
        }
        int K = harm_call ? (int)std::min<long long>(kMaxParts, kopt) : 1;
        K = (int)std::min<int64_t>(K, (P + 3) / 4);
        std::vector<int64_t> q(K + 1);  // part k: the shard's series [q[k], q[k + 1])
        for (int k = 0; k <= K; ++k) q[k] = std::min<int64_t>(P, (P * k / K + 3) / 4 * 4);
        DevCtx *cx = ctx_for(dev);
        std::lock_guard<std::mutex> hlk(cx->hmu);  // shards sharing a device run in turn
        size_t off = 0;
        auto take = [&](size_t bytes) {
            const size_t o = off;
            off += align_up(bytes);
            return o;
        };
        const size_t o_t = take(N * sizeof(double)), o_d = take((size_t)P * N * esz),
                     o_fc = take((size_t)nfc * N * esz), o_fcop = take(P * sizeof(int32_t)),
                     o_par = take(nrec * sizeof(Param)), o_st = take(state ? N : 0),
                     o_bphi = take(bphi ? 2 * P * sizeof(double) : 0),
                     o_out = take(out_demod ? (size_t)P * N * sizeof(c64) : 0),
                     o_fst = take(state && K > 1 ? (size_t)P * 16 * sizeof(double) : 0);
        if (!cx->hstream && !chk(hipStreamCreateWithFlags(&cx->hstream, hipStreamNonBlocking),
                                 "hipStreamCreate"))
            return fail(GPD_E_HIP);
        hipStream_t s = cx->hstream;
        if (cx->harena_cap < off) {
            if (cx->harena) {
                {  // gpd_last_faint_stats must not read the arena being freed
                    std::lock_guard<std::mutex> lk(cx->mu);
                    if (cx->last_fstat && (const char *)cx->last_fstat >= cx->harena &&
                        (const char *)cx->last_fstat < cx->harena + cx->harena_cap) {
                        cx->last_fstat = nullptr;
                        cx->last_fstat_P = 0;
                    }
                }
                (void)hipStreamSynchronize(s);
                (void)hipFree(cx->harena);
                cx->harena = nullptr;
                cx->harena_cap = 0;
            }
            if (hipMalloc(&cx->harena, off) != hipSuccess) {
                (void)hipGetLastError();
                set_err(errbuf_l, errlen_l, "device arena of %zu bytes: out of device memory", off);
                return fail(GPD_E_OOM);
            }
            cx->harena_cap = off;
        }
        char *A = cx->harena;
        double *dt = (double *)(A + o_t);
        char *dd = A + o_d, *dfc = A + o_fc;
        int32_t *dfcop = (int32_t *)(A + o_fcop);
        Param *dpar = (Param *)(A + o_par);
        const auto hs = std::chrono::steady_clock::now();
        int8_t *dst = state ? (int8_t *)(A + o_st) : nullptr;
        double *dbphi = bphi ? (double *)(A + o_bphi) : nullptr;
        c64 *dout = out_demod ? (c64 *)(A + o_out) : nullptr;
        bool ok = true;
        if (K > 1) {
            ok = (cx->cstream || chk(hipStreamCreateWithFlags(&cx->cstream, hipStreamNonBlocking), "hipStreamCreate")) &&
                 (cx->ostream || chk(hipStreamCreateWithFlags(&cx->ostream, hipStreamNonBlocking), "hipStreamCreate"));
            for (int k = 0; ok && k < kMaxParts; ++k)
                ok = (cx->up[k] || chk(hipEventCreateWithFlags(&cx->up[k], hipEventDisableTiming), "hipEventCreate")) &&
                     (cx->fin[k] || chk(hipEventCreateWithFlags(&cx->fin[k], hipEventDisableTiming), "hipEventCreate"));
            if (!ok) return fail(GPD_E_HIP);
        }
        hipStream_t cs = K > 1 ? cx->cstream : s, os = K > 1 ? cx->ostream : s;
        ok = chk(hipMemcpyAsync(dt, t + s0, N * sizeof(double), hipMemcpyHostToDevice, s), "H2D t") &&
             chk(hipMemcpyAsync(dfcop, fcop_l.data(), P * sizeof(int32_t), hipMemcpyHostToDevice, s),
                 "H2D fcop") &&
             (!state || chk(hipMemcpyAsync(dst, state + s0, N, hipMemcpyHostToDevice, s), "H2D state")) &&
             (!bphi || chk(hipMemcpyAsync(dbphi, bphi + 2 * p0, 2 * P * sizeof(double),
                                          hipMemcpyHostToDevice, s), "H2D bphi"));
        std::vector<char> fc_up(nfc, 0);  // FC column already sent
        auto h2d_part = [&](int k) {
            const int64_t a = q[k], b = q[k + 1];
            bool r = chk(hipMemcpy2DAsync(dd + (size_t)a * N * esz, N * esz, d + ((p0 + a) * ldd + s0) * esz,
                                          ldd * esz, N * esz, b - a, hipMemcpyHostToDevice, cs), "H2D d");
            std::vector<char> need(nfc, 0);
            for (int64_t i = a; i < b; ++i) need[fcop_l[i]] = !fc_up[fcop_l[i]];
            for (int64_t c = 0; r && c < nfc;) {  // runs of consecutive columns
                if (!need[c]) {
                    ++c;
                    continue;
                }
                int64_t e = c;
                while (e < nfc && need[e]) fc_up[e++] = 1;
                r = chk(hipMemcpy2DAsync(dfc + (size_t)c * N * esz, N * esz, fc + ((cmin + c) * ldfc + s0) * esz,
                                         ldfc * esz, N * esz, e - c, hipMemcpyHostToDevice, cs), "H2D fc");
                c = e;
            }
            return r && (K == 1 || chk(hipEventRecord(cx->up[k], cs), "hipEventRecord"));
        };
        const bool hprof = opt(O_HOST_PROF) != 0;
        auto hnow = [] { return std::chrono::steady_clock::now(); };
        // the staged output (out_kind 1/2): the P×N demodulated columns (contiguous on the device)
        // come back in chunks through the device's staging ring — chunk c into slot
        // c mod kStageSlots, an event after each; the host pool copies chunk c into the caller's
        // columns (ldo; rounded to ComplexF32 for kind 2) while chunks c + 1 … are in flight, then
        // the slot takes chunk c + kStageSlots.  Each part's columns in ≥ ⌈4 / K⌉ chunks (C2: 4 ×
        // 12.8 MB), at most one slot each; a chunk is issued on the output stream after its part's
        // compute, as soon as its slot is free.
        const bool staged = out_demod && out_kind != 0;
        struct Chunk {
            int64_t e0, e1;
            int part;
        };
        std::vector<Chunk> chunks;
        if (staged) {
            const int64_t per_slot = (int64_t)(kStageSlotBytes / sizeof(c64));
            for (int k = 0; k < K; ++k) {
                const int64_t f0 = q[k] * N, f1 = q[k + 1] * N, tot = f1 - f0;
                if (tot <= 0) continue;
                const int64_t n = std::max<int64_t>(std::min<int64_t>((kStageSlots + K - 1) / K, tot),
                                                    (tot + per_slot - 1) / per_slot);
                for (int64_t c = 0; c < n; ++c) chunks.push_back({f0 + tot * c / n, f0 + tot * (c + 1) / n, k});
            }
            ok = ok && ensure_stage(cx);
            if (!ok) set_err(errbuf_l, errlen_l, "output staging ring: out of host memory");
            for (int c = 0; ok && c < kStageSlots; ++c)
                if (!cx->hpin_ev[c])
                    ok = chk(hipEventCreateWithFlags(&cx->hpin_ev[c], hipEventDisableTiming), "hipEventCreate");
        }
        const int64_t nch = (int64_t)chunks.size();
        int64_t issued = 0;
        auto issue = [&](int64_t c) {
            const Chunk &h = chunks[c];
            const int sl = (int)(c % kStageSlots);
            return (K == 1 || chk(hipStreamWaitEvent(os, cx->fin[h.part], 0), "hipStreamWaitEvent")) &&
                   chk(hipMemcpyAsync(cx->hpin + (size_t)sl * kStageSlotBytes, dout + h.e0,
                                      (size_t)(h.e1 - h.e0) * sizeof(c64), hipMemcpyDeviceToHost, os),
                       "D2H out (staged)") &&
                   chk(hipEventRecord(cx->hpin_ev[sl], os), "hipEventRecord");
        };
        // the first touch of the caller's destination columns (a fresh output's page faults — the
        // kernel zeroing each page — are most of an unpipelined host copy), on the host pool from
        // a helper thread while this thread issues the (pageable, host-blocking) H2D copies; one
        // store per page inside the columns only (never the ldo gaps), joined before the chunk
        // copies overwrite those pages
        const size_t des = out_kind == 2 ? sizeof(gpd_c32) : sizeof(gpd_c64);
        char *dst0 = staged ? (char *)out_demod + ((size_t)p0 * ldo + s0) * des : nullptr;
        struct Joiner {
            std::thread t;
            ~Joiner() {
                if (t.joinable()) t.join();
            }
        } toucher;
        std::chrono::steady_clock::time_point ht0, ht1;
        if (ok && staged)
            toucher.t = std::thread([&] {
                ht0 = hnow();
                pool_touch_cols(dst0, des, ldo, N, P);
                ht1 = hnow();
            });
        const auto h0 = hnow();
        std::vector<double> hpart;  // host_prof: ms at each part's H2D issued, compute launched
        auto ms_since = [&](std::chrono::steady_clock::time_point a) {
            return std::chrono::duration<double, std::milli>(hnow() - a).count();
        };
        for (int k = 0; ok && k < K; ++k) {
            const int64_t a = q[k], b = q[k + 1];
            if (b <= a) continue;
            ok = h2d_part(k) && (K == 1 || chk(hipStreamWaitEvent(s, cx->up[k], 0), "hipStreamWaitEvent"));
            if (hprof) hpart.push_back(ms_since(h0));
            if (!ok) break;
            const int r = pipeline_dev(N, K == 1 ? P : b - a, dt, dd + (size_t)a * N * esz, N, dfc, nfc, N,
                                       dfcop + a, dst, omega, xinit, flags, maxfun,
                                       (gpd_param *)(dpar + a), dout ? (gpd_c64 *)(dout + a * N) : nullptr,
                                       N, dbphi, dev, s, errbuf_l, errlen_l, window, is_c32);
            if (r != GPD_OK) {
                cleanup();
                return fail(r);
            }
            if (K > 1 && state) {  // the part's faint statistics, kept for gpd_last_faint_stats
                std::lock_guard<std::mutex> lk(cx->mu);
                ok = cx->last_fstat &&
                     chk(hipMemcpyAsync(A + o_fst + (size_t)a * 16 * sizeof(double), cx->last_fstat,
                                        (size_t)(b - a) * 16 * sizeof(double), hipMemcpyDeviceToDevice, s),
                         "D2D faint statistics");
                if (ok && b == P) {
                    cx->last_fstat = (const double *)(A + o_fst);
                    cx->last_fstat_P = P;
                }
            }
            if (K > 1) ok = ok && chk(hipEventRecord(cx->fin[k], s), "hipEventRecord");
            while (ok && issued < std::min<int64_t>(nch, kStageSlots) && chunks[issued].part <= k)
                ok = issue(issued++);
            if (hprof) hpart.push_back(ms_since(h0));
        }
        if (!ok) {
            cleanup();
            return fail(GPD_E_HIP);
        }
        // the records (and the unstaged output) into the caller's pageable memory: a host-blocking
        // copy that waits for the last part's fit — after the staged chunks' host copies, which
        // overlap the device's work
        auto d2h_tail = [&] {
            return chk(hipMemcpyAsync(out_params + o0, dpar, nrec * sizeof(Param), hipMemcpyDeviceToHost, s),
                       "D2H params") &&
                   (!out_demod || out_kind != 0 ||
                    chk(hipMemcpy2DAsync(out_demod + p0 * ldo + s0, ldo * sizeof(gpd_c64), dout,
                                         N * sizeof(c64), N * sizeof(c64), P,
                                         hipMemcpyDeviceToHost, s), "D2H out"));
        };
        if (!staged) ok = d2h_tail();
        const auto h1 = hnow();
        if (hprof && !staged) (void)hipStreamSynchronize(s);
        const auto h2 = hnow();
        auto h3 = h2, h4 = h2;
        if (ok && staged) {
            toucher.t.join();
            h3 = hnow();
            for (int64_t c = 0; ok && c < nch; ++c) {
                const int sl = (int)(c % kStageSlots);
                ok = chk(hipEventSynchronize(cx->hpin_ev[sl]), "hipEventSynchronize");
                if (ok)
                    pool_copy_range(dst0, des, ldo, cx->hpin + (size_t)sl * kStageSlotBytes, N,
                                    chunks[c].e0, chunks[c].e1);
                if (ok && c + kStageSlots < nch) ok = issue(c + kStageSlots);
            }
            ok = ok && d2h_tail();
            h4 = hnow();
        }
        if (hprof) {
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            fprintf(stderr, "host_prof dev %d: setup %.3f ms, H2D + launches issued %.3f ms (%d parts), "
                    "device wait %.3f ms, output touch %.3f ms, D2H + host copy %.3f ms (pool %d "
                    "threads)\n", dev, ms(hs, h0), ms(h0, h1), K, ms(h1, h2), ms(h2, h3), ms(h3, h4),
                    HostPool::get().size());
            for (size_t i = 0; i + 1 < hpart.size(); i += 2)
                fprintf(stderr, "host_prof   part %zu: H2D issued at %.3f ms, compute launched at %.3f ms\n",
                        i / 2, hpart[i], hpart[i + 1]);
            if (staged)
                fprintf(stderr, "host_prof   output touch (helper thread) %.3f .. %.3f ms\n", ms(h0, ht0), ms(h0, ht1));
        }
        ok = ok && chk(hipStreamSynchronize(s), "hipStreamSynchronize");
        if (K > 1) {  // nothing of this call may still write the arena or the ring (error paths)
            (void)hipStreamSynchronize(cs);
            (void)hipStreamSynchronize(os);
        }
        cleanup();
        if (!ok) return fail(GPD_E_HIP);
    };
    if (G == 1) {
        worker(0);
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < G; ++g) th.emplace_back(worker, g);
        for (auto &x : th) x.join();
    }
    for (int g = 0; g < G; ++g) {
        if (rc[g] != GPD_OK) {
            set_err(errbuf, errlen, "device %d: %s", g, msg[g].c_str());
            return rc[g];
        }
    }
    return GPD_OK;
}

// demodulateall over the N×40 idx()-ordered exposure (gpd_demodulateall): the 32 diodes fitted
// by host_batch with the FC columns 32..39 of the same matrix, their demodulated columns staged
// into `output`, and the FC columns copied into `output` by the host pool while the device
// computes (what `output = copy(data)` leaves there, src/Modulation.jl:353).
static int host_demodulateall(int64_t N, const double *t, const void *data, int64_t ldd,
                              bool c32, const int8_t *state, const double *xinit, uint32_t flags,
                              int32_t maxfun, gpd_param *params, void *output, int64_t ldo,
                              int32_t n_gpus, char *errbuf, size_t errlen) {
    if (N < 2 || !t || !data || !params || !output || ldd < N || ldo < N) {
        set_err(errbuf, errlen, "gpd_demodulateall: invalid shapes/pointers (N=%lld)",
                (long long)N);
        return GPD_E_ARG;
    }
    const size_t esz = c32 ? sizeof(gpd_c32) : sizeof(gpd_c64);
    // output must not overlap data (advisor r5): the FC columns are copied from data into output
    // and the diode columns read by the H2D copies while output's pages are touched and written
    {
        const uintptr_t d0 = (uintptr_t)data, d1 = d0 + ((size_t)39 * ldd + N) * esz;
        const uintptr_t o0 = (uintptr_t)output, o1 = o0 + ((size_t)39 * ldo + N) * esz;
        if (d0 < o1 && o0 < d1) {
            set_err(errbuf, errlen, "gpd_demodulateall: output overlaps data (output = copy(data) "
                    "is a fresh array)");
            return GPD_E_ARG;
        }
    }
    // 0-based FC column of diode c among the 8 FC columns: idx(side, telescope, FC) − 33 with
    // side FT for c < 16, SC otherwise, telescope = (c mod 16) ÷ 4 + 1 (src/Modulation.jl:17-22,388)
    int32_t fcop[32];
    for (int c = 0; c < 32; ++c) fcop[c] = (c < 16 ? 0 : 4) + (c % 16) / 4;
    const char *fc = (const char *)data + (size_t)32 * ldd * esz;
    const auto tcall = std::chrono::steady_clock::now();
    std::thread fcopy([&] {
        const auto t0 = std::chrono::steady_clock::now();
        pool_copy_cols((char *)output + (size_t)32 * ldo * esz, esz, ldo, fc, esz, ldd, N, 8);
        if (opt(O_HOST_PROF))
            fprintf(stderr, "host_prof FC columns copy %.3f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    });
    const int r = host_batch(N, 32, t, data, ldd, fc, 8, ldd, fcop, state, 6.283185, xinit, flags,
                             maxfun, params, (gpd_c64 *)output, ldo, nullptr, n_gpus, errbuf,
                             errlen, 0, c32, c32 ? 2 : 1);
    fcopy.join();
    if (opt(O_HOST_PROF))
        fprintf(stderr, "host_prof demodulateall total %.3f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tcall).count());
    return r;
}

extern "C" {

int gpd_demodulateall(int64_t n_samples, const double *t, const gpd_c64 *data, int64_t ldd,
                      const int8_t *state, const double *xinit, uint32_t flags, int32_t maxfun,
                      gpd_param *params, gpd_c64 *output, int64_t ldo, int32_t n_gpus,
                      char *errbuf, size_t errlen) {
    return host_demodulateall(n_samples, t, data, ldd, false, state, xinit, flags, maxfun, params,
                              output, ldo, n_gpus, errbuf, errlen);
}

int gpd_demodulateall_c32(int64_t n_samples, const double *t, const gpd_c32 *data, int64_t ldd,
                          const int8_t *state, const double *xinit, uint32_t flags,
                          int32_t maxfun, gpd_param *params, gpd_c32 *output, int64_t ldo,
                          int32_t n_gpus, char *errbuf, size_t errlen) {
    return host_demodulateall(n_samples, t, data, ldd, true, state, xinit, flags, maxfun, params,
                              output, ldo, n_gpus, errbuf, errlen);
}

int gpd_fit_batch(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c64 *d,
                  int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                  const int32_t *fc_of_pixel, const int8_t *state, double omega,
                  const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                  gpd_c64 *out_demod, int64_t ldo, int32_t n_gpus, char *errbuf, size_t errlen) {
    return host_batch(n_samples, n_pixels, t, d, ldd, fc, n_fc, ldfc, fc_of_pixel, state, omega,
                      xinit, flags, maxfun, out_params, out_demod, ldo, nullptr, n_gpus, errbuf,
                      errlen);
}

int gpd_chi2_batch(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c64 *d,
                   int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                   const int32_t *fc_of_pixel, const int8_t *state, double omega,
                   const double *bphi, uint32_t flags, gpd_param *out_params, int32_t n_gpus,
                   char *errbuf, size_t errlen) {
    if (!bphi) {
        set_err(errbuf, errlen, "gpd_chi2_batch: bphi is NULL");
        return GPD_E_ARG;
    }
    return host_batch(n_samples, n_pixels, t, d, ldd, fc, n_fc, ldfc, fc_of_pixel, state, omega,
                      nullptr, flags, 0, out_params, nullptr, n_samples, bphi, n_gpus, errbuf,
                      errlen);
}

int gpd_fit_windows(int64_t n_samples, int64_t window, int64_t n_cols, const double *t,
                    const gpd_c64 *d, int64_t ldd, const gpd_c64 *fc, int64_t n_fc, int64_t ldfc,
                    const int32_t *fc_of_col, const int8_t *state, double omega,
                    const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                    gpd_c64 *out_demod, int64_t ldo, int32_t n_gpus, char *errbuf, size_t errlen) {
    if (window < 1) {
        set_err(errbuf, errlen, "gpd_fit_windows: window must be >= 1");
        return GPD_E_ARG;
    }
    return host_batch(n_samples, n_cols, t, d, ldd, fc, n_fc, ldfc, fc_of_col, state, omega,
                      xinit, flags, maxfun, out_params, out_demod, ldo, nullptr, n_gpus, errbuf,
                      errlen, window);
}

int gpd_fit_batch_c32(int64_t n_samples, int64_t n_pixels, const double *t, const gpd_c32 *d,
                      int64_t ldd, const gpd_c32 *fc, int64_t n_fc, int64_t ldfc,
                      const int32_t *fc_of_pixel, const int8_t *state, double omega,
                      const double *xinit, uint32_t flags, int32_t maxfun, gpd_param *out_params,
                      gpd_c64 *out_demod, int64_t ldo, int32_t n_gpus, char *errbuf,
                      size_t errlen) {
    return host_batch(n_samples, n_pixels, t, d, ldd, fc, n_fc, ldfc, fc_of_pixel, state, omega,
                      xinit, flags, maxfun, out_params, out_demod, ldo, nullptr, n_gpus, errbuf,
                      errlen, 0, true);
}

int gpd_fit_windows_c32(int64_t n_samples, int64_t window, int64_t n_cols, const double *t,
                        const gpd_c32 *d, int64_t ldd, const gpd_c32 *fc, int64_t n_fc,
                        int64_t ldfc, const int32_t *fc_of_col, const int8_t *state, double omega,
                        const double *xinit, uint32_t flags, int32_t maxfun,
                        gpd_param *out_params, gpd_c64 *out_demod, int64_t ldo, int32_t n_gpus,
                        char *errbuf, size_t errlen) {
    if (window < 1) {
        set_err(errbuf, errlen, "gpd_fit_windows_c32: window must be >= 1");
        return GPD_E_ARG;
    }
    return host_batch(n_samples, n_cols, t, d, ldd, fc, n_fc, ldfc, fc_of_col, state, omega,
                      xinit, flags, maxfun, out_params, out_demod, ldo, nullptr, n_gpus, errbuf,
                      errlen, window, true);
}

int gpd_process_volt(int64_t n_samples, const double *t, const float *volt, int64_t ldv,
                     const gpd_c64 *centers, const int8_t *state, double omega,
                     const double *xinit, uint32_t flags, int32_t maxfun, int64_t window,
                     gpd_param *out_params, float *out_volt, int64_t ldov, int device,
                     char *errbuf, size_t errlen) {
    // processmetrology's numeric core (src/GPPupilDemodulation.jl:147-171, 191-207) on one
    // device: Float32 VOLT rows → centred complex128 columns → demodulateall (or every window)
    // → demodulated Float32 VOLT rows.  Column c < 32 uses FC column 32 + c/4 (idx(), :388).
    const int64_t N = n_samples;
    if (N < 2 || !t || !volt || ldv < 80 || !out_params || (out_volt && ldov < 80) || window < 0) {
        set_err(errbuf, errlen, "gpd_process_volt: invalid shapes/pointers");
        return GPD_E_ARG;
    }
    const int ndev = gpd_device_count();
    if (ndev <= 0) {
        set_err(errbuf, errlen, "gpd_process_volt: no HIP device visible");
        return GPD_E_NODEV;
    }
    if (device < 0 || device >= ndev) {
        set_err(errbuf, errlen, "gpd_process_volt: device %d out of range", device);
        return GPD_E_ARG;
    }
    HIP_TRY(hipSetDevice(device));
    const int64_t nrec = 32 * (window > 0 ? (N + window - 1) / window : 1);
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess) {
            set_err(errbuf, errlen, "gpd_process_volt: %s: %s", what, hipGetErrorString(e));
            return false;
        }
        return true;
    };
    int32_t fcop[32];
    for (int c = 0; c < 32; ++c) fcop[c] = c / 4;  // idx(side, tel, FC) - 33 for diode column c
    // the device's grow-only arena and stream of the host-buffer entry points (no hipMalloc /
    // hipFree / stream creation per exposure); hmu serialises host calls on this device
    DevCtx *cx = ctx_for(device);
    std::lock_guard<std::mutex> hlk(cx->hmu);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(bytes);
        return o;
    };
    const size_t o_t = take(N * sizeof(double)), o_v = take((size_t)N * 80 * sizeof(float)),
                 o_cplx = take((size_t)40 * N * sizeof(c64)), o_fcop = take(32 * sizeof(int32_t)),
                 o_par = take(nrec * sizeof(Param)), o_cen = take(centers ? 40 * sizeof(c64) : 0),
                 o_st = take(state ? N : 0),
                 o_out = take(out_volt ? (size_t)32 * N * sizeof(c64) : 0),
                 o_ov = take(out_volt ? (size_t)N * 80 * sizeof(float) : 0);
    if (!cx->hstream && !chk(hipStreamCreateWithFlags(&cx->hstream, hipStreamNonBlocking), "stream"))
        return GPD_E_HIP;
    hipStream_t s = cx->hstream;
    if (cx->harena_cap < off) {
        if (cx->harena) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(cx->harena);
            cx->harena = nullptr;
            cx->harena_cap = 0;
        }
        if (hipMalloc(&cx->harena, off) != hipSuccess) {
            (void)hipGetLastError();
            set_err(errbuf, errlen, "gpd_process_volt: device arena of %zu bytes: out of device memory", off);
            return GPD_E_OOM;
        }
        cx->harena_cap = off;
    }
    char *A = cx->harena;
    double *dt = (double *)(A + o_t);
    float *dv = (float *)(A + o_v), *dov = out_volt ? (float *)(A + o_ov) : nullptr;
    c64 *dcplx = (c64 *)(A + o_cplx), *dcen = centers ? (c64 *)(A + o_cen) : nullptr;
    c64 *dout = out_volt ? (c64 *)(A + o_out) : nullptr;
    int32_t *dfcop = (int32_t *)(A + o_fcop);
    Param *dpar = (Param *)(A + o_par);
    int8_t *dst = state ? (int8_t *)(A + o_st) : nullptr;
    // rows of 80 Float32: one linear copy when the caller's rows are contiguous
    auto copy_rows = [&](void *dst_, size_t dpitch, const void *src, size_t spitch, hipMemcpyKind k) {
        if (dpitch == spitch)
            return hipMemcpyAsync(dst_, src, (size_t)N * dpitch, k, s);
        return hipMemcpy2DAsync(dst_, dpitch, src, spitch, 80 * sizeof(float), N, k, s);
    };
    bool ok = chk(hipMemcpyAsync(dt, t, N * sizeof(double), hipMemcpyHostToDevice, s), "H2D t") &&
              chk(copy_rows(dv, 80 * sizeof(float), volt, ldv * sizeof(float), hipMemcpyHostToDevice),
                  "H2D volt") &&
              chk(hipMemcpyAsync(dfcop, fcop, sizeof fcop, hipMemcpyHostToDevice, s), "H2D fcop") &&
              (!centers || chk(hipMemcpyAsync(dcen, centers, 40 * sizeof(c64), hipMemcpyHostToDevice, s),
                               "H2D centres")) &&
              (!state || chk(hipMemcpyAsync(dst, state, N, hipMemcpyHostToDevice, s), "H2D state"));
    if (!ok) return GPD_E_HIP;
    const unsigned tiles = (unsigned)((N + VT_ROWS - 1) / VT_ROWS);
    k_volt_ingest<<<tiles, 256, 0, s>>>(N, dv, 80, dcen, dcplx, N);
    int r = pipeline_dev(N, 32, dt, (const gpd_c64 *)dcplx, N, (const gpd_c64 *)(dcplx + 32 * N), 8,
                         N, dfcop, dst, omega, xinit, flags, maxfun, (gpd_param *)dpar,
                         (gpd_c64 *)dout, N, nullptr, device, s, errbuf, errlen, window);
    if (r != GPD_OK) {
        (void)hipStreamSynchronize(s);
        return r;
    }
    if (out_volt) k_volt_egress<<<tiles, 256, 0, s>>>(N, dout, dcplx, N, dov, 80);
    ok = chk(hipGetLastError(), "launch") &&
         chk(hipMemcpyAsync(out_params, dpar, nrec * sizeof(Param), hipMemcpyDeviceToHost, s),
             "D2H params") &&
         (!out_volt || chk(copy_rows(out_volt, ldov * sizeof(float), dov, 80 * sizeof(float),
                                     hipMemcpyDeviceToHost),
                           "D2H volt")) &&
         chk(hipStreamSynchronize(s), "synchronize");
    return ok ? GPD_OK : GPD_E_HIP;
}

int gpd_libm_eval(int fn, int64_t n, const double *x, const double *y, double *out, int device) {
    char *errbuf = nullptr;
    size_t errlen = 0;
    if (fn < 0 || fn > 10 || n < 0 || (n > 0 && (!x || !out)) ||
        ((fn == 4 || fn == 5 || fn == 7 || fn == 10) && n > 0 && !y))
        return GPD_E_ARG;
    // fn 10: jl_sin(fl(x[i] + y[0])) through the Payne–Hanek table and shift; the shift of the
    // whole x range is formed here on the host (the same jlm_ph_shift) and handed to the device
    uint64_t shift[4] = {0, 0, 0, 0};
    if (fn == 10 && n > 0) {
        double xmin = x[0], xmax = x[0];
        for (int64_t i = 1; i < n; ++i) {
            xmin = std::min(xmin, x[i]);
            xmax = std::max(xmax, x[i]);
        }
        shift[3] = (uint64_t)jlm_ph_shift(xmin, xmax, y[0], &shift[0], &shift[1], &shift[2]);
    }
    const int ndev = gpd_device_count();
    if (ndev <= 0) return GPD_E_NODEV;
    if (device < 0 || device >= ndev) return GPD_E_ARG;
    if (n == 0) return GPD_OK;
    HIP_TRY(hipSetDevice(device));
    const int width = (fn == 2 || fn == 9) ? 2 : fn == 6 ? 3 : 1;
    double *dx = nullptr, *dy = nullptr, *dout = nullptr;
    auto release = [&]() {
        (void)hipFree(dx);
        (void)hipFree(dy);
        (void)hipFree(dout);
    };
    if (hipMalloc(&dx, n * sizeof(double)) != hipSuccess ||
        hipMalloc(&dy, std::max<int64_t>(n, 4) * sizeof(double)) != hipSuccess ||
        hipMalloc(&dout, n * width * sizeof(double)) != hipSuccess) {
        release();
        (void)hipGetLastError();
        return GPD_E_OOM;
    }
    hipError_t e = hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess && fn == 10)
        e = hipMemcpy(dy, shift, sizeof shift, hipMemcpyHostToDevice);  // dy holds ≥ 4 words
    else if (e == hipSuccess)
        e = hipMemcpy(dy, y ? y : x, n * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        k_libm<<<(unsigned)((n + 255) / 256), 256>>>(fn, n, dx, dy, dout);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, n * width * sizeof(double), hipMemcpyDeviceToHost);
    release();
    return e == hipSuccess ? GPD_OK : GPD_E_HIP;
}

int gpd_mean_var_power(int64_t n_samples, int64_t n_series, const gpd_c64 *d, int64_t ldd,
                       const int8_t *state, uint32_t flags, double *out, int device, char *errbuf,
                       size_t errlen) {
    // compute_mean_var_power (src/Faint.jl:89-100) of whole series with demodulateall's valid
    // mask — the statistics the fit uses (the one-pass kernels; option faint_stats = 2: the two-pass
    // kernel the windows use)
    if (n_samples < 1 || n_series < 1 || !d || !state || !out || ldd < n_samples) {
        set_err(errbuf, errlen, "gpd_mean_var_power: invalid shapes/pointers");
        return GPD_E_ARG;
    }
    const int ndev = gpd_device_count();
    if (ndev <= 0) {
        set_err(errbuf, errlen, "gpd_mean_var_power: no HIP device visible");
        return GPD_E_NODEV;
    }
    if (device < 0 || device >= ndev) {
        set_err(errbuf, errlen, "gpd_mean_var_power: device %d out of range", device);
        return GPD_E_ARG;
    }
    HIP_TRY(hipSetDevice(device));
    const long long N = n_samples, P = n_series;
    const bool fs1 =
        opt(O_FAINT_STATS) != 2;
    const Layout L = plan(N, P, 1, true, false, false, false, 0, false);  // fs_pc, fs_mmax
    c64 *dd = nullptr;
    int8_t *dst = nullptr;
    double *fst = nullptr, *fx = nullptr, *fxt = nullptr;
    auto release = [&]() {
        (void)hipFree(dd);
        (void)hipFree(dst);
        (void)hipFree(fst);
        (void)hipFree(fx);
        (void)hipFree(fxt);
    };
    if (hipMalloc(&dd, (size_t)P * N * sizeof(c64)) != hipSuccess ||
        hipMalloc(&dst, (size_t)N) != hipSuccess ||
        hipMalloc(&fst, (size_t)P * 16 * sizeof(double)) != hipSuccess ||
        (fs1 && (hipMalloc(&fx, L.fsc - L.fsx) != hipSuccess ||
                 hipMalloc(&fxt, L.total - L.fsc) != hipSuccess))) {
        release();
        (void)hipGetLastError();
        set_err(errbuf, errlen, "gpd_mean_var_power: out of device memory");
        return GPD_E_OOM;
    }
    Problem pb{};
    pb.N = N;
    pb.P = P;
    pb.d = dd;
    pb.ldd = N;
    pb.state = dst;
    pb.flags = flags & GPD_ONLY_HIGH;
    pb.ncol = P;
    hipError_t e = hipMemcpy2D(dd, N * sizeof(c64), d, ldd * sizeof(gpd_c64), N * sizeof(c64), P,
                               hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dst, state, (size_t)N, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        if (fs1) {
            e = run_faint_onepass(pb, fst, fx, fxt, L.fs_pc, L.fs_mmax, false, nullptr);
        } else {
            k_faint_stats<<<(unsigned)P, 256>>>(pb, fst);
            e = hipGetLastError();
        }
    }
    std::vector<double> h((size_t)P * 16);
    if (e == hipSuccess) e = hipMemcpy(h.data(), fst, h.size() * sizeof(double), hipMemcpyDeviceToHost);
    release();
    if (e != hipSuccess) {
        set_err(errbuf, errlen, "gpd_mean_var_power: %s", hipGetErrorString(e));
        return GPD_E_HIP;
    }
    for (long long k = 0; k < P; ++k)
        for (int q = 0; q < 10; ++q) out[k * 10 + q] = h[k * 16 + q];
    return GPD_OK;
}

int gpd_synth_fill_dev(int64_t n_samples, int64_t n_pixels, int64_t pixel_offset, uint64_t seed,
                       double t0, double dt, double sigma, int with_offsets, double omega,
                       double *t, gpd_c64 *d, int64_t ldd, gpd_c64 *fc, int64_t ldfc,
                       int32_t *fc_of_pixel, gpd_param *truth, int device, void *stream_) {
    char *errbuf = nullptr;
    size_t errlen = 0;
    if (n_samples < 1 || n_pixels < 1 || pixel_offset % 4 != 0 || !t || !d || !fc ||
        !fc_of_pixel || ldd < n_samples || ldfc < n_samples)
        return GPD_E_ARG;
    HIP_TRY(hipSetDevice(device));
    hipStream_t s = (hipStream_t)stream_;
    const long long N = n_samples, P = n_pixels, nfc = (P + 3) / 4;
    Param *tr = (Param *)truth;
    Param *tmp = nullptr;
    if (!tr) {
        HIP_TRY(hipMallocAsync((void **)&tmp, P * sizeof(Param), s));
        tr = tmp;
    }
    k_synth_t<<<(unsigned)((N + 255) / 256), 256, 0, s>>>(N, t0, dt, t);
    k_synth_truth<<<(unsigned)((P + 255) / 256), 256, 0, s>>>(P, pixel_offset, seed, with_offsets, tr);
    k_synth_fc<<<(unsigned)((nfc + 63) / 64), 64, 0, s>>>(N, nfc, pixel_offset / 4, seed, (c64 *)fc, ldfc);
    dim3 g((unsigned)std::min<long long>((N + 255) / 256, 64), (unsigned)P);
    k_synth_d<<<g, 256, 0, s>>>(N, P, pixel_offset, seed, t0, dt, sigma, omega, tr, (const c64 *)fc,
                               ldfc, (c64 *)d, ldd, fc_of_pixel);
    HIP_TRY(hipGetLastError());
    if (tmp) HIP_TRY(hipFreeAsync(tmp, s));
    return GPD_OK;
}

int gpd_buildstates_dev(int64_t n, const double *t, int64_t n1, const double *timer1, int64_t n2,
                        const double *timer2, int64_t lag, double preswitchdelay,
                        double postwitchdelay, int8_t *states, int device, void *stream_) {
    // src/Faint.jl:21-73 on device (gpd_states.hpp): t and states are device arrays, the timer
    // lists (FITS header values, buildfaintparameters) host arrays, shifted here by lag·Δt.
    char *errbuf = nullptr;
    size_t errlen = 0;
    if (n < 2 || n1 < 1 || n2 < 1 || n1 > BS_MAX_TIMER || n2 > BS_MAX_TIMER || !t || !timer1 ||
        !timer2 || !states)
        return GPD_E_ARG;
    const int ndev = gpd_device_count();
    if (ndev <= 0) return GPD_E_NODEV;
    if (device < 0 || device >= ndev) return GPD_E_ARG;
    HIP_TRY(hipSetDevice(device));
    hipStream_t s = (hipStream_t)stream_;
    const long long nt = n1 + n2, cap = nt + n + 1;
    DevCtx *cx = ctx_for(device);
    std::lock_guard<std::mutex> lk(cx->mu);
    if (!cx->bs_pinned) {
        HIP_TRY(hipHostMalloc((void **)&cx->bs_pinned, 2 * BS_MAX_TIMER * sizeof(double),
                              hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&cx->bs_done, hipEventDisableTiming));
    } else {
        HIP_TRY(hipEventSynchronize(cx->bs_done));  // the previous call's copy has consumed it
    }
    std::memcpy(cx->bs_pinned, timer1, n1 * sizeof(double));
    std::memcpy(cx->bs_pinned + n1, timer2, n2 * sizeof(double));
    const size_t o_lb = align_up(nt * sizeof(double)), o_ctl = o_lb + align_up(nt * sizeof(long long)),
                 o_evk = o_ctl + align_up(sizeof(BsCtl)), o_evf = o_evk + align_up(cap * sizeof(long long)),
                 o_evs = o_evf + align_up(cap * sizeof(long long)), total = o_evs + align_up(cap);
    char *w = nullptr;
    HIP_TRY(hipMallocAsync((void **)&w, total, s));
    double *tim = (double *)w;
    long long *lb = (long long *)(w + o_lb), *evk = (long long *)(w + o_evk),
              *evf = (long long *)(w + o_evf);
    BsCtl *ctl = (BsCtl *)(w + o_ctl);
    int8_t *evs = (int8_t *)(w + o_evs);
    HIP_TRY(hipMemcpyAsync(tim, cx->bs_pinned, nt * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(cx->bs_done, s));
    HIP_TRY(hipMemsetAsync(ctl, 0, sizeof(BsCtl), s));
    const long long np = std::max<long long>(n - 1, nt);
    k_bs_prep<<<(unsigned)((np + 255) / 256), 256, 0, s>>>(t, n, tim, n1, n2, lag, preswitchdelay,
                                                         postwitchdelay, lb, ctl);
    k_bs_events<<<1, 256, 0, s>>>(t, n, tim, n1, n2, lb, ctl, evk, evs, evf);
    k_bs_fill<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(n, ctl, evk, evs, evf, states);
    k_bs_serial<<<1, 64, 0, s>>>(t, n, tim, n1, n2, ctl, states);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipFreeAsync(w, s));
    return GPD_OK;
}

int gpd_buildstates(int64_t n, const double *t, int64_t n1, const double *timer1, int64_t n2,
                    const double *timer2, double preswitchdelay, double postwitchdelay,
                    int8_t *states) {
    // src/Faint.jl:21-73, sequential state machine (host; O(N) once per exposure).
    if (n < 2 || n1 < 1 || n2 < 1 || !t || !timer1 || !timer2 || !states) return GPD_E_ARG;
    const double timestep = t[1] - t[0];
    const long long premax = (long long)std::ceil(preswitchdelay / timestep);
    const long long postmax = (long long)std::ceil(postwitchdelay / timestep);
    const int8_t HIGH = GPD_STATE_HIGH, LOW = GPD_STATE_LOW, NORMAL = GPD_STATE_NORMAL;
    int8_t current = NORMAL;
    int64_t i1 = 0, i2 = 0;
    double first1 = timer1[i1++], first2 = timer2[i2++];
    const double tlast = t[n - 1];
    long long forget = 0;
    for (int64_t k = 0; k < n; ++k) {
        const double time = t[k];
        if (time >= first1) {  // HIGH switch
            current = HIGH;
            forget = premax;
            if (i1 >= n1) {
                first1 = tlast;
                if (first2 == tlast) current = NORMAL;
            } else {
                first1 = timer1[i1++];
            }
        }
        if (time >= first2) {  // LOW switch
            current = LOW;
            forget = postmax;
            if (i2 >= n2) {
                first2 = tlast;
                if (first1 == tlast) current = NORMAL;
            } else {
                first2 = timer2[i2++];
            }
        }
        if (forget > 0) {
            states[k] = GPD_STATE_TRANSIENT;
            forget -= 1;
        } else {
            states[k] = current;
        }
    }
    return GPD_OK;
}

}  // extern "C"
