// Throughput probe: fp32 products on the exact-fp32 MFMA (v_mfma_f32_32x32x2_f32) against the same products as
// three-term bf16 splits on the bf16 MFMA (v_mfma_f32_32x32x16_bf16, six products a_i b_j with i + j <= 2: every
// term of a * b above 2^-23 |a b|; the splits a = a0 + a1 + a2 are exact, by truncation).
//
// One LDS-resident GEMM tile loop per workgroup (256 threads = 2 x 2 waves, each wave 64 x 64 outputs = 2 x 2 blocks
// of 32 x 32), the conv GEMM's orientation: A = weights [o][k] (frozen: pre-split once into three bf16 planes),
// B = input [k][m] fp32 (split in registers after the LDS read, as a conv's gathered input would be).
//   mode 0: fp32 MFMA, both operands fp32 from LDS (the shipped kernels' inner loop)
//   mode 1: bf16 x 6, A planes from LDS, B fp32 from LDS split in registers
//   mode 2: bf16 x 6, both operands pre-split in LDS (upper bound: no split VALU)
// Prints TF/s (fp32-equivalent: 2 MACs counted once per fp32 product) and the max error of each mode's result
// against an fp64 host reference.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/probes/bx6_probe tools/probes/bx6_probe.hip && tools/probes/bx6_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BO = 128, BM = 128, KC = 16, NCH = 2;  // LDS: NCH chunks of K = 16

__device__ __forceinline__ unsigned perm_hi(unsigned lo_word, unsigned hi_word) {
    // (hi16 of lo_word) | (hi16 of hi_word) << 16
    return __builtin_amdgcn_perm(hi_word, lo_word, 0x07060302u);
}

// 8 fp32 -> three bf16x8 planes: x = p0 + p1 + p2 exactly (truncating splits)
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
    unsigned u0[8], u1[8], u2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const unsigned u = __float_as_uint(x[j]);
        const float r1 = x[j] - __uint_as_float(u & 0xffff0000u);
        const unsigned v = __float_as_uint(r1);
        const float r2 = r1 - __uint_as_float(v & 0xffff0000u);
        u0[j] = u;
        u1[j] = v;
        u2[j] = __float_as_uint(r2);
    }
    unsigned w0[4], w1[4], w2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        w0[j] = perm_hi(u0[2 * j], u0[2 * j + 1]);
        w1[j] = perm_hi(u1[2 * j], u1[2 * j + 1]);
        w2[j] = perm_hi(u2[2 * j], u2[2 * j + 1]);
    }
    memcpy(&p0, w0, 16);
    memcpy(&p1, w1, 16);
    memcpy(&p2, w2, 16);
}

template <int MODE>
__global__ __launch_bounds__(256, 2) void probe(const float* wsrc, const float* xsrc, const short* wsplit,
                                                const short* xsplit, float* out, int iters) {
    // LDS: W fp32 [NCH][KC][BO] | X fp32 [NCH][KC][BM] | W planes [3][NCH][BO][KC] bf16 | X planes [3][NCH][BM][KC]
    __shared__ __attribute__((aligned(16))) float wf[NCH * KC * BO];
    __shared__ __attribute__((aligned(16))) float xf[NCH * KC * BM];
    __shared__ __attribute__((aligned(16))) short wp[3 * NCH * BO * KC];
    __shared__ __attribute__((aligned(16))) short xp[3 * NCH * BM * KC];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < NCH * KC * BO; i += 256) wf[i] = wsrc[i];
    for (int i = tid; i < NCH * KC * BM; i += 256) xf[i] = xsrc[i];
    for (int i = tid; i < 3 * NCH * BO * KC; i += 256) wp[i] = wsplit[i];
    for (int i = tid; i < 3 * NCH * BM * KC; i += 256) xp[i] = xsplit[i];
    __syncthreads();
    const int wo = wave >> 1, wm = wave & 1;
    const int r = lane & 31, h = lane >> 5;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
    for (int it = 0; it < iters; ++it) {
        const int c = it & (NCH - 1);
        if constexpr (MODE == 0) {
#pragma unroll
            for (int kk = 0; kk < KC / 2; ++kk) {
                float a[2], b[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) a[i] = wf[(c * KC + 2 * kk + h) * BO + wo * 64 + i * 32 + r];
#pragma unroll
                for (int j = 0; j < 2; ++j) b[j] = xf[(c * KC + 2 * kk + h) * BM + wm * 64 + j * 32 + r];
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
            }
        } else {
            bf16x8 a[2][3], b[2][3];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int s = 0; s < 3; ++s)
                    a[i][s] = *reinterpret_cast<const bf16x8*>(&wp[((s * NCH + c) * BO + wo * 64 + i * 32 + r) * KC + 8 * h]);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if constexpr (MODE == 1) {
                    float x[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) x[e] = xf[(c * KC + 8 * h + e) * BM + wm * 64 + j * 32 + r];
                    split8(x, b[j][0], b[j][1], b[j][2]);
                } else {
#pragma unroll
                    for (int s = 0; s < 3; ++s)
                        b[j][s] = *reinterpret_cast<const bf16x8*>(
                            &xp[((s * NCH + c) * BM + wm * 64 + j * 32 + r) * KC + 8 * h]);
                }
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    // small terms first
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[j][0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][2], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[j][0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[j][0], acc[i][j], 0, 0, 0);
                }
        }
    }
    // C[o][m]: block (i, j), register q -> o = 32 i + (q & 3) + 8 (q >> 2) + 4 h, m = 32 j + r
    float* dst = out + (size_t)blockIdx.x * BO * BM;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int o = wo * 64 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                const int m = wm * 64 + j * 32 + r;
                dst[o * BM + m] = acc[i][j][q];
            }
}

static void split_host(float x, short (&p)[3]) {
    unsigned u;
    memcpy(&u, &x, 4);
    unsigned hi = u & 0xffff0000u;
    float fh;
    memcpy(&fh, &hi, 4);
    float r1 = x - fh;
    unsigned v;
    memcpy(&v, &r1, 4);
    unsigned mid = v & 0xffff0000u;
    float fm;
    memcpy(&fm, &mid, 4);
    float r2 = r1 - fm;
    unsigned w;
    memcpy(&w, &r2, 4);
    p[0] = (short)(u >> 16);
    p[1] = (short)(v >> 16);
    p[2] = (short)(w >> 16);
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

int main(int argc, char** argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 1024;
    const int iters = argc > 2 ? atoi(argv[2]) : 4000;
    std::vector<float> w(NCH * KC * BO), x(NCH * KC * BM);
    srand(7);
    for (auto& v : w) v = (float)rand() / (float)RAND_MAX * 2.f - 1.f;
    for (auto& v : x) v = ((float)rand() / (float)RAND_MAX * 2.f - 1.f) * 3.f;
    std::vector<short> wsp(3 * NCH * BO * KC), xsp(3 * NCH * BM * KC);
    for (int c = 0; c < NCH; ++c)
        for (int k = 0; k < KC; ++k) {
            for (int o = 0; o < BO; ++o) {
                short p[3];
                split_host(w[(c * KC + k) * BO + o], p);
                for (int s = 0; s < 3; ++s) wsp[((s * NCH + c) * BO + o) * KC + k] = p[s];
            }
            for (int m = 0; m < BM; ++m) {
                short p[3];
                split_host(x[(c * KC + k) * BM + m], p);
                for (int s = 0; s < 3; ++s) xsp[((s * NCH + c) * BM + m) * KC + k] = p[s];
            }
        }
    float *dw, *dx, *dout;
    short *dws, *dxs;
    CK(hipMalloc(&dw, w.size() * 4));
    CK(hipMalloc(&dx, x.size() * 4));
    CK(hipMalloc(&dws, wsp.size() * 2));
    CK(hipMalloc(&dxs, xsp.size() * 2));
    CK(hipMalloc(&dout, (size_t)grid * BO * BM * 4));
    CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dws, wsp.data(), wsp.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxs, xsp.data(), xsp.size() * 2, hipMemcpyHostToDevice));
    // fp64 reference for a short run (iters_chk) of workgroup 0
    const int iters_chk = 4;
    std::vector<double> ref(BO * BM, 0.0);
    for (int it = 0; it < iters_chk; ++it) {
        const int c = it & (NCH - 1);
        for (int o = 0; o < BO; ++o)
            for (int m = 0; m < BM; ++m) {
                double s = 0;
                for (int k = 0; k < KC; ++k) s += (double)w[(c * KC + k) * BO + o] * x[(c * KC + k) * BM + m];
                ref[o * BM + m] += s;
            }
    }
    double refmax = 0, sumabs = 0;
    for (double v : ref) refmax = fmax(refmax, fabs(v));
    for (int o = 0; o < BO; ++o)
        for (int k = 0; k < KC; ++k) sumabs = fmax(sumabs, fabs(w[k * BO + o]));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> got(BO * BM);
    for (int mode = 0; mode < 3; ++mode) {
        auto launch = [&](int g, int n) {
            if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(g), dim3(256), 0, 0, dw, dx, dws, dxs, dout, n);
            else if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(g), dim3(256), 0, 0, dw, dx, dws, dxs, dout, n);
            else hipLaunchKernelGGL(probe<2>, dim3(g), dim3(256), 0, 0, dw, dx, dws, dxs, dout, n);
        };
        launch(1, iters_chk);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), dout, BO * BM * 4, hipMemcpyDeviceToHost));
        double err = 0;
        for (int i = 0; i < BO * BM; ++i) err = fmax(err, fabs(got[i] - ref[i]));
        for (int rep = 0; rep < 2; ++rep) launch(grid, iters);  // warm-up (clocks)
        CK(hipEventRecord(e0));
        const int reps = 5;
        for (int rep = 0; rep < reps; ++rep) launch(grid, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double flop = 2.0 * BO * BM * KC * (double)iters * grid * reps;
        printf("mode %d (%s): %.3f ms/launch  %.1f TF/s fp32-equivalent   max err vs fp64 %.3e (max |ref| %.3e)\n",
               mode, mode == 0 ? "fp32 MFMA" : mode == 1 ? "bf16x6, B split in registers" : "bf16x6, pre-split",
               ms / reps, flop / (ms * 1e-3) / 1e12, err, refmax);
    }
    return 0;
}
