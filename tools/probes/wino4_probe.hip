// Where does the F(4x4) Winograd kernel's time go?  Compiles csrc/wino4.hip into this translation unit and times
// wino4_kernel with pieces removed (PROBE bits: 1 U DMAs after step 0, 2 patch DMAs after step 1, 4 the transform
// after step 0) on the synthesis conv1 shapes (batch 4), random data, interleaved repetitions.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -I include tools/probes/wino4_probe.hip \
//         stylemc_amd/csrc/errors.hip -o tools/probes/wino4_probe && tools/probes/wino4_probe
#include "../../stylemc_amd/csrc/wino4.hip"

#include <cstdio>

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

template <int SM, int PROBE>
void launch_p(const Wino4Params& p, int64_t items) {
    hipLaunchKernelGGL((wino4_kernel<SM, 0, PROBE>), dim3((unsigned)items), dim3(W4_THREADS), 0, 0, p);
}

template <int SM>
void launch_probe(int probe, const Wino4Params& p, int64_t items) {
    switch (probe) {
        case 0: launch_p<SM, 0>(p, items); break;
        case 1: launch_p<SM, 1>(p, items); break;
        case 2: launch_p<SM, 2>(p, items); break;
        case 3: launch_p<SM, 3>(p, items); break;
        case 4: launch_p<SM, 4>(p, items); break;
        case 7: launch_p<SM, 7>(p, items); break;
    }
}

int main() {
    const int n = 4;
    const int rs[] = {64, 128, 256};
    const int probes[] = {0, 1, 2, 3, 4, 7};
    const char* names[] = {"full", "-U dma", "-P dma", "-U-P dma", "-transform", "-dma-transform"};
    constexpr int NP = 6;
    for (int r : rs) {
        const int c = std::min(32768 / r, 512);
        const size_t nx = (size_t)n * c * r * r;
        float *x, *y, *uw, *s;
        CK(hipMalloc(&x, nx * 4));
        CK(hipMalloc(&y, nx * 4));
        CK(hipMalloc(&uw, (size_t)36 * c * c * 4));
        CK(hipMalloc(&s, (size_t)n * c * 4));
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, x, nx, 1u, 2.f, 0.f);
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, uw, (size_t)36 * c * c, 2u, 0.1f, 0.f);
        hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, 0, s, (size_t)n * c, 3u, 0.5f, 1.f);
        CK(hipDeviceSynchronize());
        Wino4Params p{};
        p.x = x; p.n = n; p.cin = c; p.h = r; p.w = r; p.y = y; p.cout = c; p.uw = uw; p.s = s;
        p.mode = SMC_EPI_STORE; p.act = SMC_ACT_LINEAR; p.gain = 1.f; p.clamp = -1.f;
        p.gx = r / 64;
        p.gy = r / 8;
        p.ntn = c / 64;
        const int64_t items = (int64_t)n * p.gx * p.gy * p.ntn;
        const double flops = 2.0 * n * c * c * (r / 4) * (r / 4) * 36;
        float ms[NP] = {0};
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int rep = 0; rep < 6; ++rep)
            for (int i = 0; i < NP; ++i) {
                CK(hipEventRecord(e0));
                for (int k = 0; k < 5; ++k) launch_probe<1>(probes[i], p, items);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (rep > 0) ms[i] += t / 5 / 5;
            }
        for (int i = 0; i < NP; ++i)
            std::printf("r=%4d c=%3d %-16s %7.1f us  MFMA frac %.3f\n", r, c, names[i], ms[i] * 1e3,
                        flops / (ms[i] * 1e-3) / 157.3e12);
        CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(uw)); CK(hipFree(s));
    }
    return 0;
}
