// Timing probe for the Winograd conv kernel: which part of a K step costs what.  Compiles csrc/wino.hip into this
// translation unit and times wino_kernel<TC, PROBE> variants (PROBE bits in wino.hip: 1 no U DMA after step 0,
// 2 no patch DMA after step 0, 4 no per-step wait + barrier, 8 no epilogue, 16 no input transform).  The variants
// compute garbage; only their durations matter.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/probes/wino_probe.hip stylemc_amd/csrc/errors.hip \
//         -o tools/probes/wino_probe
//   tools/probes/wino_probe
#include "../../stylemc_amd/csrc/wino.hip"

#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

template <int TC, int OBW, int PROBE>
float time_variant(const WinoParams& p, int wgs, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((wino_kernel<TC, OBW, PROBE>), dim3(wgs), dim3(64 * 8 / OBW), 0, 0, p);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((wino_kernel<TC, OBW, PROBE>), dim3(wgs), dim3(64 * 8 / OBW), 0, 0, p);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return 1e3f * ms / reps;
}

template <int TC, int OBW>
int run(int r) {
    const int n = 4, c = std::min(32768 / r, 512);
    const size_t xe = (size_t)n * c * r * r, ue = (size_t)16 * c * c;
    float *x, *y, *uw, *s;
    CK(hipMalloc(&x, xe * 4));
    CK(hipMalloc(&y, xe * 4));
    CK(hipMalloc(&uw, ue * 4));
    CK(hipMalloc(&s, (size_t)n * c * 4));
    CK(hipMemset(x, 0, xe * 4));
    CK(hipMemset(uw, 0, ue * 4));
    CK(hipMemset(s, 0, (size_t)n * c * 4));
    WinoParams p{};
    p.x = x; p.n = n; p.cin = c; p.h = r; p.w = r; p.y = y; p.cout = c; p.uw = uw; p.s = s;
    p.mode = SMC_EPI_STORE; p.act = SMC_ACT_LINEAR; p.gain = 1.f; p.clamp = -1.f;
    p.ext.rs = 1;
    p.gx = (r / 2) / TC;
    p.gy = (r / 2) / (WBT / TC);
    p.ntn = c / WBO;
    const int wgs = n * p.gx * p.gy * p.ntn;
    const double flops = 2.0 * n * c * c * (r / 2) * (r / 2) * 16;
    const int reps = 10;
    struct V { const char* name; float us; };
    std::vector<V> v = {
        {"full", time_variant<TC, OBW, 0>(p, wgs, reps)},
        {"no U DMA", time_variant<TC, OBW, 1>(p, wgs, reps)},
        {"no patch DMA", time_variant<TC, OBW, 2>(p, wgs, reps)},
        {"no DMA", time_variant<TC, OBW, 3>(p, wgs, reps)},
        {"no wait+barrier", time_variant<TC, OBW, 4>(p, wgs, reps)},
        {"no epilogue", time_variant<TC, OBW, 8>(p, wgs, reps)},
        {"no transform", time_variant<TC, OBW, 16>(p, wgs, reps)},
        {"no DMA/barrier/epi", time_variant<TC, OBW, 15>(p, wgs, reps)},
        {"MFMA + LDS reads only", time_variant<TC, OBW, 31>(p, wgs, reps)},
        {"MFMA only", time_variant<TC, OBW, 63>(p, wgs, reps)},
    };
    for (auto& e : v)
        std::printf("OBW=%d r=%4d c=%3d %-22s %8.1f us  MFMA frac %.3f\n", OBW, r, c, e.name, e.us, flops / (e.us * 1e-6) / 157.3e12);
    CK(hipFree(x));
    CK(hipFree(y));
    CK(hipFree(uw));
    CK(hipFree(s));
    return 0;
}

int main() {
    if (run<64, 2>(256) || run<64, 2>(1024) || run<32, 2>(64)) return 1;
    return 0;
}
