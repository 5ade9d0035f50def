// A/B harness for Winograd kernel variants on random data (the DVFS clock depends on the operands: zero-filled
// inputs run faster, MI355X_MICROARCH.md 'DVFS give-back').  Compiles csrc/wino.hip into this translation unit and
// times two wino_kernel variants <TC, SM, PERSIST, PROBE> on the
// synthesis conv1 shapes (FFHQ-1024, batch 4), interleaved, and checks that the outputs are bit-identical.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/probes/wino_ab.hip stylemc_amd/csrc/errors.hip \
//         -o tools/probes/wino_ab && tools/probes/wino_ab
#include "../../stylemc_amd/csrc/wino.hip"

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__global__ void fill_kernel(float* p, size_t n, unsigned seed, float scale, float offset) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        p[i] = ((h & 0xffffff) / 16777216.f - 0.5f) * scale + offset;
    }
}

template <int SM_, int PERSIST_, int PROBE_ = 0>
struct V {
    static constexpr int SM = SM_, PERSIST = PERSIST_, PROBE = PROBE_;
};

template <int TC, int SM, int PERSIST, int PROBE>
void launch_i(const WinoParams& p, int r, int n, int c) {
    WinoParams q = p;
    q.gx = (r / 2) / TC;
    q.gy = (r / 2) / (WBT / TC);
    q.ntn = c / WBO;
    const int items = n * q.gx * q.gy * q.ntn;
    if (PERSIST) {
        launch_wino<TC, SM, 0>(q, items, 0);
    } else {
        auto kern = &wino_kernel<TC, SM, 0, 0, PROBE>;
        hipLaunchKernelGGL(kern, dim3(items), dim3(256), 0, 0, q);
    }
}

template <int TC, class VV>
void launch(const WinoParams& p, int r, int n, int c) {
    launch_i<TC, VV::SM, VV::PERSIST, VV::PROBE>(p, r, n, c);
}

template <int TC, class VV>
float time_kernel(const WinoParams& p, int r, int n, int c, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch<TC, VV>(p, r, n, c);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return 1e3f * ms / reps;
}

template <class VV>
void name(char* buf) {
    std::snprintf(buf, 64, "SM%d,PERSIST%d,PROBE%d", VV::SM, VV::PERSIST, VV::PROBE);
}

// variant A vs variant B at shape r (with_s: the style-scaled forward; else the data gradient's plain conv)
template <int TC, class VA, class VB>
int run(int r, bool with_s, double* tot) {
    const int n = 4, c = std::min(32768 / r, 512);
    const size_t xe = (size_t)n * c * r * r, ue = (size_t)16 * c * c;
    float *x, *y0, *y1, *uw, *s;
    CK(hipMalloc(&x, xe * 4));
    CK(hipMalloc(&y0, xe * 4));
    CK(hipMalloc(&y1, xe * 4));
    CK(hipMalloc(&uw, ue * 4));
    CK(hipMalloc(&s, (size_t)n * c * 4));
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, x, xe, 1u, 2.f, 0.f);
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, uw, ue, 2u, 0.2f, 0.f);
    hipLaunchKernelGGL(fill_kernel, dim3(16), dim3(256), 0, 0, s, (size_t)n * c, 3u, 1.f, 1.f);
    WinoParams p{};
    p.x = x; p.n = n; p.cin = c; p.h = r; p.w = r; p.cout = c; p.uw = uw; p.s = with_s ? s : nullptr;
    p.mode = SMC_EPI_STORE; p.act = SMC_ACT_LINEAR; p.gain = 1.f; p.clamp = -1.f; p.nsplit = 1;
    p.ext.rs = 1;
    const double flops = 2.0 * n * c * c * (r / 2) * (r / 2) * 16;
    p.y = y0;
    launch<TC, VA>(p, r, n, c);
    p.y = y1;
    launch<TC, VB>(p, r, n, c);
    CK(hipDeviceSynchronize());
    std::vector<float> h0(xe), h1(xe);
    CK(hipMemcpy(h0.data(), y0, xe * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), y1, xe * 4, hipMemcpyDeviceToHost));
    const bool same = std::memcmp(h0.data(), h1.data(), xe * 4) == 0;
    float t[2] = {0.f, 0.f};
    const int reps = 10, rounds = 3;
    for (int k = 0; k < rounds; ++k) {  // interleaved
        p.y = y0;
        t[0] += time_kernel<TC, VA>(p, r, n, c, reps);
        p.y = y1;
        t[1] += time_kernel<TC, VB>(p, r, n, c, reps);
    }
    for (int v = 0; v < 2; ++v) {
        t[v] /= rounds;
        tot[v] += t[v];
    }
    char na[64], nb[64];
    name<VA>(na);
    name<VB>(nb);
    std::printf("r=%5d c=%4d TC=%2d %s  A(%s) %7.1f us (frac %.3f)  B(%s) %7.1f us (frac %.3f)  %+.1f%%  outputs %s\n",
                r, c, TC, with_s ? "fwd" : "bwd", na, t[0], flops / (t[0] * 1e-6) / 157.3e12, nb, t[1],
                flops / (t[1] * 1e-6) / 157.3e12, 100.0 * (t[0] / t[1] - 1.0), same ? "bit-identical" : "DIFFER");
    CK(hipFree(x)); CK(hipFree(y0)); CK(hipFree(y1)); CK(hipFree(uw)); CK(hipFree(s));
    return same ? 0 : 2;
}

int main() {
    double tot[2] = {0, 0};
    int rc = 0;
    rc |= run<16, V<1, 0>, V<1, 1>>(32, true, tot);
    rc |= run<32, V<1, 0>, V<1, 1>>(64, true, tot);
    rc |= run<64, V<1, 0>, V<1, 1>>(128, true, tot);
    rc |= run<64, V<1, 0>, V<1, 1>>(256, true, tot);
    rc |= run<64, V<1, 0>, V<1, 1>>(512, true, tot);
    rc |= run<64, V<1, 0>, V<1, 1>>(1024, true, tot);
    rc |= run<64, V<2, 0>, V<2, 1>>(512, false, tot);
    rc |= run<64, V<2, 0>, V<2, 1>>(1024, false, tot);
    std::printf("total A %.1f us  B %.1f us  (%+.1f%%)\n", tot[0], tot[1], 100.0 * (tot[0] / tot[1] - 1.0));
    return rc;
}
