// Faint-mode state sequence on device: buildstates (src/Faint.jl:21-73) without the sequential
// per-sample loop.
//
// The reference walks the samples once with two pending timer values (first1: next HIGH switch,
// first2: next LOW switch).  A timer entry fires at the first sample after the previous firing of
// the same timer whose time is ≥ the entry (one pop per sample); the firing sets the current state
// and restarts the TRANSIENT countdown (premax / postmax samples); the LOW branch runs after the
// HIGH branch on the same sample.  An exhausted timer keeps last(timestamp) as pending value, so
// it fires again on every sample with t ≥ t[N-1], and a firing that exhausts a timer while the
// other one pends at last(timestamp) yields NORMAL.
//
// With non-decreasing timestamps the firing sample of entry j is max(previous + 1, lb(x_j)),
// lb = first sample with t ≥ x_j, so the state machine reduces to:
//   k_bs_prep    (one wave per timer entry block) lb of every entry, lb(t[N-1]), Δt, monotonicity
//   k_bs_events  (one thread, entries staged in LDS) the ordered list of firing samples with the
//                state and countdown each leaves behind — O(n1 + n2) steps instead of O(N)
//   k_bs_fill    (grid over samples) each sample binary-searches the last firing ≤ it:
//                TRANSIENT while k − k_e < countdown_e, else state_e (NORMAL before any firing)
// Non-monotone timestamps take k_bs_serial, the reference loop on one lane (exact, slow).
#pragma once

#include "gpd_device.hpp"

namespace gpd {

constexpr int BS_MAX_TIMER = 4096;  // entries per timer staged in LDS by k_bs_events
constexpr int8_t ST_HIGH = 3, ST_LOW = 1, ST_NORMAL = 2, ST_TRANSIENT = -1;

struct BsCtl {
    int nonmono;     // set by k_bs_prep when some t[i+1] < t[i] (zeroed by the host)
    int nev;         // firing samples written by k_bs_events
    long long lbT;   // first sample with t ≥ t[N-1]
    long long premax, postmax;
};

__device__ __forceinline__ long long lower_bound_t(const double *__restrict__ t, long long n,
                                                   double x) {
    long long lo = 0, hi = n;  // first index with t[i] >= x (n if none)
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if (t[mid] >= x)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

// timers (device copies, unshifted) → shifted entries x_j = timer_j + lag·Δt (Julia: timer .+
// lag*timestep, src/Faint.jl:25-26), lb of each; thread 0 also the countdown lengths.
__global__ __launch_bounds__(256) void k_bs_prep(const double *__restrict__ t, long long n,
                                                 double *__restrict__ tim, long long n1,
                                                 long long n2, long long lag, double pre,
                                                 double post, long long *__restrict__ lb,
                                                 BsCtl *__restrict__ ctl) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const double step = t[1] - t[0];
    if (i < n - 1 && t[i + 1] < t[i]) ctl->nonmono = 1;  // any writer writes 1 (benign race)
    if (i < n1 + n2) {
        const double x = tim[i] + (double)lag * step;
        tim[i] = x;
        lb[i] = lower_bound_t(t, n, x);
    }
    if (i == 0) {
        ctl->lbT = lower_bound_t(t, n, t[n - 1]);
        ctl->premax = (long long)ceil(pre / step);  // ceil(Int, preswitchdelay / timestep)
        ctl->postmax = (long long)ceil(post / step);
    }
}

// One thread walks the firings in sample order.  ev_k: firing sample, ev_s: state after both
// branches of that sample, ev_f: countdown after them.  Capacity: n1 + n2 + (N − lbT) + 1.
__global__ __launch_bounds__(256) void k_bs_events(const double *__restrict__ t, long long n,
                                                   const double *__restrict__ tim, long long n1,
                                                   long long n2, const long long *__restrict__ lb,
                                                   BsCtl *__restrict__ ctl,
                                                   long long *__restrict__ ev_k,
                                                   int8_t *__restrict__ ev_s,
                                                   long long *__restrict__ ev_f) {
    __shared__ long long slb[2 * BS_MAX_TIMER];
    __shared__ unsigned char slast[2 * BS_MAX_TIMER];  // entry == last(timestamp)
    if (ctl->nonmono) return;
    const double tlast = t[n - 1];
    for (long long j = threadIdx.x; j < n1 + n2; j += 256) {
        slb[j] = lb[j];
        slast[j] = tim[j] == tlast;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    const long long lbT = ctl->lbT, premax = ctl->premax, postmax = ctl->postmax;
    long long c1 = 0, c2 = 0;        // pending entry (c1 == n1 / c2 == n2: exhausted, pends tlast)
    long long last1 = -1, last2 = -1; // sample of each timer's previous firing
    int8_t cur = ST_NORMAL;
    long long nev = 0;
    const long long NEVER = n;
    // next firing sample of a timer: pending real entry → max(prev + 1, lb); exhausted → every
    // sample from max(prev + 1, lbT)
    auto next1 = [&]() -> long long {
        const long long l = c1 < n1 ? slb[c1] : lbT;
        const long long k = last1 + 1 > l ? last1 + 1 : l;
        return k < n ? k : NEVER;
    };
    auto next2 = [&]() -> long long {
        const long long l = c2 < n2 ? slb[n1 + c2] : lbT;
        const long long k = last2 + 1 > l ? last2 + 1 : l;
        return k < n ? k : NEVER;
    };
    while (true) {
        const long long k1 = next1(), k2 = next2();
        const long long k = k1 < k2 ? k1 : k2;
        if (k >= NEVER) break;
        long long fg = 0;
        if (k1 == k) {  // HIGH branch (src/Faint.jl:41-52)
            cur = ST_HIGH;
            fg = premax;
            if (c1 >= n1 - 1) {  // isempty(t1): first1 = last(timestamp)
                c1 = n1;
                const bool first2_is_last = c2 >= n2 || slast[n1 + c2];
                if (first2_is_last) cur = ST_NORMAL;
            } else {
                ++c1;
            }
            last1 = k;
        }
        if (k2 == k) {  // LOW branch (:54-65), after HIGH on the same sample
            cur = ST_LOW;
            fg = postmax;
            if (c2 >= n2 - 1) {
                c2 = n2;
                const bool first1_is_last = c1 >= n1 || slast[c1];
                if (first1_is_last) cur = ST_NORMAL;
            } else {
                ++c2;
            }
            last2 = k;
        }
        ev_k[nev] = k;
        ev_s[nev] = cur;
        ev_f[nev] = fg;
        ++nev;
    }
    ctl->nev = (int)nev;
}

__global__ __launch_bounds__(256) void k_bs_fill(long long n, const BsCtl *__restrict__ ctl,
                                                 const long long *__restrict__ ev_k,
                                                 const int8_t *__restrict__ ev_s,
                                                 const long long *__restrict__ ev_f,
                                                 int8_t *__restrict__ states) {
    if (ctl->nonmono) return;
    const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const int nev = ctl->nev;
    int lo = 0, hi = nev;  // number of firings at samples ≤ k
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (ev_k[mid] <= k)
            lo = mid + 1;
        else
            hi = mid;
    }
    int8_t s = ST_NORMAL;
    if (lo > 0) {
        const int e = lo - 1;
        s = (k - ev_k[e] < ev_f[e]) ? ST_TRANSIENT : ev_s[e];
    }
    states[k] = s;
}

// The reference loop itself, one lane (non-monotone timestamps only).
__global__ void k_bs_serial(const double *__restrict__ t, long long n,
                            const double *__restrict__ tim, long long n1, long long n2,
                            const BsCtl *__restrict__ ctl, int8_t *__restrict__ states) {
    if (!ctl->nonmono || threadIdx.x != 0 || blockIdx.x != 0) return;
    const double tlast = t[n - 1];
    long long i1 = 0, i2 = 0, forget = 0;
    double first1 = tim[i1++], first2 = tim[n1 + i2++];
    int8_t cur = ST_NORMAL;
    for (long long k = 0; k < n; ++k) {
        const double time = t[k];
        if (time >= first1) {
            cur = ST_HIGH;
            forget = ctl->premax;
            if (i1 >= n1) {
                first1 = tlast;
                if (first2 == tlast) cur = ST_NORMAL;
            } else {
                first1 = tim[i1++];
            }
        }
        if (time >= first2) {
            cur = ST_LOW;
            forget = ctl->postmax;
            if (i2 >= n2) {
                first2 = tlast;
                if (first1 == tlast) cur = ST_NORMAL;
            } else {
                first2 = tim[n1 + i2++];
            }
        }
        if (forget > 0) {
            states[k] = ST_TRANSIENT;
            forget -= 1;
        } else {
            states[k] = cur;
        }
    }
}

}  // namespace gpd
