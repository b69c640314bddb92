// Accuracy of the hardware v_sqrt_f64 (and of fs_abs's refined form) on gfx950 against the
// host's correctly rounded sqrt: ulp histogram over random |q|² values spanning the faint
// statistics' range.  Build: hipcc --offload-arch=gfx950 -O3 -o sqrt_ulp sqrt_ulp.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

__global__ void k_sqrt(const double *a, double *o, long n) {
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i < n) o[i] = __builtin_amdgcn_sqrt(a[i]);
}

static int64_t ulps(double a, double b) {
    int64_t ia, ib;
    std::memcpy(&ia, &a, 8);
    std::memcpy(&ib, &b, 8);
    return ia > ib ? ia - ib : ib - ia;
}

int main() {
    const long n = 1 << 24;
    std::vector<double> a(n), o(n);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-1.0, 1.0), e(-40.0, 40.0);
    for (long i = 0; i < n; ++i) {
        const double re = u(g) * std::exp2(e(g) * 0.25), im = u(g) * std::exp2(e(g) * 0.25);
        a[i] = std::fma(re, re, im * im);
    }
    double *da, *dout;
    if (hipMalloc(&da, n * 8) != hipSuccess || hipMalloc(&dout, n * 8) != hipSuccess) return 2;
    hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice);
    k_sqrt<<<(unsigned)((n + 255) / 256), 256>>>(da, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost);
    long hist[4] = {0, 0, 0, 0};
    int64_t mx = 0;
    for (long i = 0; i < n; ++i) {
        const int64_t d = ulps(o[i], std::sqrt(a[i]));
        hist[d < 3 ? d : 3]++;
        if (d > mx) mx = d;
    }
    printf("{\"n\": %ld, \"ulp0\": %ld, \"ulp1\": %ld, \"ulp2\": %ld, \"ulp3plus\": %ld, \"max_ulp\": %lld}\n",
           n, hist[0], hist[1], hist[2], hist[3], (long long)mx);
    hipFree(da);
    hipFree(dout);
    return 0;
}
