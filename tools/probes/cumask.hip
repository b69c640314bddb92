// Which CUs a stream's CU mask selects on gfx950 (8 XCDs): every workgroup of a wide launch on a
// masked stream records its XCC id and HW_ID (SE / SH / CU fields); the host prints the distinct
// (XCC, SE, CU) triples per mask.  Masks tried: all CUs, the low 240 bits, every bit i with
// i mod 32 < 30 (two CUs per 32-bit word cleared), and every bit whose i / 8 ... — enough to tell
// a contiguous per-XCD layout of the mask from an interleaved one.
// Build: hipcc --offload-arch=gfx950 -O2 -o cumask cumask.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void k_where(unsigned *out) {
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
    // keep the workgroup resident a little so the launch spreads over every allowed CU
    for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(1);
}

static void run(const char *name, const std::vector<unsigned> &mask, int ncu) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (unsigned)mask.size(), mask.data()) != hipSuccess) {
        printf("%s: stream creation failed\n", name);
        return;
    }
    const int nb = 8192;
    unsigned *d;
    hipMalloc(&d, nb * 2 * sizeof(unsigned));
    k_where<<<nb, 64, 0, s>>>(d);
    hipStreamSynchronize(s);
    std::vector<unsigned> h(nb * 2);
    hipMemcpy(h.data(), d, nb * 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> cus;
    std::set<unsigned> xccs;
    for (int b = 0; b < nb; ++b) {
        const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
        const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        cus.insert({xcc, se, sh, cu});
        xccs.insert(xcc);
    }
    int per[16] = {0};
    for (auto &t : cus) per[std::get<0>(t)]++;
    printf("%s: mask bits set %d of %d, distinct CUs %zu, per XCC:", name,
           [&] { int c = 0; for (unsigned w : mask) c += __builtin_popcount(w); return c; }(), ncu,
           cus.size());
    for (int x = 0; x < 8; ++x) printf(" %d", per[x]);
    printf("\n");
    hipFree(d);
    hipStreamDestroy(s);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    const int words = (ncu + 31) / 32;
    printf("device %s, %d CUs\n", p.gcnArchName, ncu);
    std::vector<unsigned> all(words, 0xffffffffu);
    run("all", all, ncu);
    std::vector<unsigned> low(words, 0);
    for (int i = 0; i < ncu - 16; ++i) low[i / 32] |= 1u << (i % 32);
    run("low ncu-16 bits", low, ncu);
    std::vector<unsigned> wd(words, 0);
    for (int i = 0; i < ncu; ++i)
        if (i % 32 < 30) wd[i / 32] |= 1u << (i % 32);
    run("bits i%32<30", wd, ncu);
    std::vector<unsigned> il(words, 0);
    for (int i = 0; i < ncu; ++i)
        if (i < ncu - 16) il[i / 32] |= 1u << (i % 32);
    std::vector<unsigned> one(words, 0);
    for (int i = 0; i < ncu; ++i)
        if (i % 8 == 0) one[i / 32] |= 1u << (i % 32);
    run("bits i%8==0", one, ncu);
    std::vector<unsigned> first(words, 0);
    for (int i = 0; i < 32; ++i) first[0] |= 1u << i;
    run("bits 0..31", first, ncu);
    return 0;
}
