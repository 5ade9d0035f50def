// Sustained fp32 MFMA FLOP/s on MI355X: v_mfma_f32_32x32x2_f32 vs v_mfma_f32_16x16x4_f32, operands in
// registers (random, non-zero), 4 independent accumulators per wave, WAVES waves per SIMD.  Answers
// whether the 16x16 shape holds a higher clock under load (MI355X_MICROARCH.md DVFS item 7) for f32.
// Measured (r01): 148.5 / 155.2 / 154.6 TF/s (32x32x2) and 155.6 / 155.6 / 155.0 (16x16x4) at 1 / 2 / 4
// waves per SIMD: no shape-dependent clock for f32 -- the f32 peak holds.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/mfma_f32_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ float rnd(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return (float)(x & 0xffff) / 65536.f - 0.5f;
}

__global__ __launch_bounds__(256) void k32(float* out, int iters) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    float a0 = rnd(t), a1 = rnd(t + 7), b0 = rnd(t + 13), b1 = rnd(t + 29);
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, c3, 0, 0, 0);
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
    out[t] = s;
}

__global__ __launch_bounds__(256) void k16(float* out, int iters) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    float a0 = rnd(t), a1 = rnd(t + 7), b0 = rnd(t + 13), b1 = rnd(t + 29);
    f32x4 c[16] = {};
    for (int i = 0; i < iters; ++i) {
        // 16 x (16x16x4) = 2x the FLOPs of 4 x (32x32x2): counted as such in main()
#pragma unroll
        for (int j = 0; j < 16; ++j)
            c[j] = __builtin_amdgcn_mfma_f32_16x16x4f32((j & 1) ? a1 : a0, (j & 2) ? b1 : b0, c[j], 0, 0, 0);
    }
    float s = 0.f;
    for (int j = 0; j < 16; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    out[t] = s;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 20000;
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int blocks = cus * wps;  // 4 waves per block -> wps waves per SIMD
        float* out;
        hipMalloc(&out, (size_t)blocks * 256 * 4);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int shape = 0; shape < 2; ++shape) {
            for (int rep = 0; rep < 3; ++rep) {  // warm the clock
                if (shape == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, out, iters);
                else hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, out, iters);
            }
            hipEventRecord(e0);
            const int reps = 5;
            for (int rep = 0; rep < reps; ++rep) {
                if (shape == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, out, iters);
                else hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, out, iters);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            const double per_iter = shape == 0 ? 4 * (2.0 * 32 * 32 * 2) : 16 * (2.0 * 16 * 16 * 4);
            const double flops = (double)reps * blocks * 4 /*waves*/ * iters * per_iter;
            printf("waves/SIMD %d  %s  %.1f TF/s\n", wps, shape == 0 ? "32x32x2 f32" : "16x16x4 f32",
                   flops / (ms * 1e-3) / 1e12);
        }
        hipFree(out);
    }
    return 0;
}
