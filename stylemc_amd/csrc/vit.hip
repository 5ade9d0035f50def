// CLIP ViT image tower on gfx950: fp32 MFMA GEMMs with fused epilogues, LayerNorm, softmax attention,
// patch embedding, and a native forward / data-gradient executor over a packed weight buffer.
//
// Replaces the third-party openai/CLIP ``VisionTransformer`` the reference calls at clip_loss.py:21,25-26
// (encode_image of the edited and the original image; gradients flow to the edited image only, the
// weights are frozen -- so the backward is the data gradient alone, no weight gradients).
//
// Token stream: X[M = B*L][D] row-major fp32 (L = grid^2 + 1 tokens, CLS first), the layout the GEMMs
// stream through: every projection is C[M][N] = A[M][K] . Bw[K][N] with Bw the frozen weight stored
// K-major once at pack time (nn.Linear's W^T for the forward, W itself for the data gradient).
//
// GEMM on the matrix core (v_mfma_f32_32x32x2_f32, exact fp32): a 256-thread workgroup owns a
// 32-row x 128-column tile, each wave one 32x32 block whose lane index runs over columns, so every
// accumulator register stores 32 consecutive floats of one output row (128-B coalesced).  The token
// counts are small (M = 200 for 4 images), so the K loop is split across workgroups when the tile
// grid alone cannot fill the 256 CUs; partial tiles go to a workspace that the epilogue kernel sums.
// Epilogues (bias, QuickGELU with the pre-activation saved, QuickGELU' for the backward, residual add)
// are fused into whichever kernel writes the final value.
#include <cmath>
#include <cstdlib>

#include "common.hpp"

// Zero a buffer on the stream: a kernel (smc::zero_async), or hipMemsetAsync in the SMC_HIP_MEMSET=1 A/B build.
#ifndef SMC_HIP_MEMSET
#define SMC_HIP_MEMSET 0
#endif
#define SMC_TRY_MEMSET(ptr, bytes, st, what)                                                       \
    do {                                                                                           \
        if (SMC_HIP_MEMSET) {                                                                      \
            if (hipMemsetAsync((ptr), 0, (bytes), (st)) != hipSuccess) {                           \
                smc::set_error("%s failed", what);                                                 \
                return SMC_ERR_LAUNCH;                                                             \
            }                                                                                      \
        } else {                                                                                   \
            const int rz_ = smc::zero_async((ptr), (bytes), (st), what);                            \
            if (rz_ != SMC_OK) return rz_;                                                         \
        }                                                                                          \
    } while (0)

namespace {

constexpr int LBM = 32, LBN = 128, LBK = 32, LNT = 256;
constexpr int LAP = LBM + 1;  // A tile row (k-major) pitch: conflict-free transposed writes
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct LinParams {
    const float* a;
    int lda;
    const float* b;
    int ldb;
    float* c;
    int ldc;
    int M, N, K;
    smc_linear_epilogue e;
    int nsplit;
    float* ws;       // [nsplit][M][N] when nsplit > 1
    int* counters;   // zeroed, one per output tile: the last split to finish a tile reduces it (may be NULL)
};

__device__ __forceinline__ float qgelu_sigmoid(float x) { return 1.f / (1.f + expf(-1.702f * x)); }

// v = epi(acc) for output element (m, n).
__device__ __forceinline__ float lin_epi(float v, int m, int n, const smc_linear_epilogue& e) {
    if (e.bias) v += e.bias[n];
    if (e.dact_pre) {  // backward of QuickGELU: v *= d/dx [x * sigmoid(1.702 x)] at the saved pre-activation
        const float x = e.dact_pre[(int64_t)m * e.ld_dact + n];
        const float s = qgelu_sigmoid(x);
        v *= s + 1.702f * x * s * (1.f - s);
    }
    if (e.act == SMC_LIN_ACT_QUICKGELU) {
        if (e.pre_save) e.pre_save[(int64_t)m * e.ld_pre + n] = v;
        v = v * qgelu_sigmoid(v);
    }
    if (e.residual) v += e.residual[(int64_t)m * e.ld_res + n];
    return v;
}

__global__ __launch_bounds__(LNT, 2) void lin_gemm_kernel(LinParams p) {
    // one LDS object (a second __shared__ object, e.g. a reducer flag, can make hipcc drain vmcnt in
    // the k-loop): [stage][ Bs[LBK][LBN] | As[LBK][LAP] ]
    __shared__ __attribute__((aligned(16))) float smem[2 * LBK * (LBN + LAP)];
    auto As = [&](int st, int k, int r) -> float& { return smem[st * LBK * (LBN + LAP) + LBK * LBN + k * LAP + r]; };
    auto Bs = [&](int st, int k, int c) -> float* { return &smem[st * LBK * (LBN + LAP) + k * LBN + c]; };

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kh = lane >> 5, l32 = lane & 31;
    const int m0 = blockIdx.x * LBM, n0 = blockIdx.y * LBN, split = blockIdx.z;
    const int nks = p.K / LBK;
    const int ks0 = (int)((int64_t)nks * split / p.nsplit);
    const int ks1 = (int)((int64_t)nks * (split + 1) / p.nsplit);

    // A: one float4 per thread (row tid/8, k 4*(tid%8)); rows past M re-read row M-1 (results dropped)
    const int ar = tid >> 3, ak = (tid & 7) * 4;
    const int arow = min(m0 + ar, p.M - 1);
    const float* aptr = p.a + (int64_t)arow * p.lda + ak;
    // B: four float4 per thread (row v/32, column 4*(v%32)); columns past N re-read a valid vector
    float4 ra, rb[4];
    auto load = [&](int ks) {
        const int k0 = ks * LBK;
        ra = *reinterpret_cast<const float4*>(aptr + k0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int v = tid + q * LNT;
            const int r = v >> 5, cc = (v & 31) * 4;
            const int n = min(n0 + cc, p.N - 4);
            rb[q] = *reinterpret_cast<const float4*>(p.b + (int64_t)(k0 + r) * p.ldb + n);
        }
    };
    auto store = [&](int st) {
        As(st, ak + 0, ar) = ra.x;
        As(st, ak + 1, ar) = ra.y;
        As(st, ak + 2, ar) = ra.z;
        As(st, ak + 3, ar) = ra.w;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int v = tid + q * LNT;
            const int r = v >> 5, cc = (v & 31) * 4;
            *reinterpret_cast<float4*>(Bs(st, r, cc)) = rb[q];
        }
    };

    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;

    int st = 0;
    if (ks0 < ks1) {
        load(ks0);
        store(0);
    }
    __syncthreads();
    for (int ks = ks0; ks < ks1; ++ks) {
        const bool more = ks + 1 < ks1;
        if (more) load(ks + 1);
        float af[LBK / 2], bf[LBK / 2];
#pragma unroll
        for (int q = 0; q < LBK / 2; ++q) {
            af[q] = As(st, 2 * q + kh, l32);
            bf[q] = *Bs(st, 2 * q + kh, wave * 32 + l32);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < LBK / 2; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q], bf[q], acc, 0, 0, 0);
        if (more) store(st ^ 1);
        __syncthreads();
        st ^= 1;
    }

    const int n = n0 + wave * 32 + l32;
    const bool nok = n < p.N;
    if (p.nsplit == 1) {
        if (!nok) return;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
            if (m < p.M) p.c[(int64_t)m * p.ldc + n] = lin_epi(acc[r], m, n, p.e);
        }
        return;
    }
    if (nok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
            if (m < p.M) p.ws[((int64_t)split * p.M + m) * p.N + n] = acc[r];
        }
    }
    if (!p.counters) return;  // a separate kernel reduces the partial tiles
    // Split-K hand-off without a second launch (cdna_hip_programming.md section 6 Guideline 16, counter
    // form): every wave drains its partial-tile stores, one lane releases them at agent scope (one L2
    // write-back per workgroup, not a __threadfence per thread) and takes a ticket; the workgroup that
    // draws the last ticket acquires and sums the partials in split order (the order of the separate
    // epilogue kernel: deterministic whichever split finishes last).
    int* flag = reinterpret_cast<int*>(smem);  // the k-loop is over: the LDS array is free
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int prev = __hip_atomic_fetch_add(p.counters + blockIdx.y * gridDim.x + blockIdx.x, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == p.nsplit - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    if (!*flag || !nok) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
        if (m >= p.M) continue;
        float v = 0.f;
        for (int k = 0; k < p.nsplit; ++k) v += p.ws[((int64_t)k * p.M + m) * p.N + n];
        p.c[(int64_t)m * p.ldc + n] = lin_epi(v, m, n, p.e);
    }
}

// Sum the split-K partial tiles and apply the epilogue (float4 along n; N % 4 == 0).
__global__ void lin_splitk_epilogue_kernel(const float* ws, int nsplit, float* c, int ldc, int M, int N,
                                           smc_linear_epilogue e) {
    const int64_t nv = (int64_t)M * (N / 4);
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(v / (N / 4));
        const int n = (int)(v - (int64_t)m * (N / 4)) * 4;
        float4 s = *reinterpret_cast<const float4*>(ws + (int64_t)m * N + n);
        for (int k = 1; k < nsplit; ++k) {
            const float4 t = *reinterpret_cast<const float4*>(ws + ((int64_t)k * M + m) * N + n);
            s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
        }
        float* dst = c + (int64_t)m * ldc + n;
        dst[0] = lin_epi(s.x, m, n + 0, e);
        dst[1] = lin_epi(s.y, m, n + 1, e);
        dst[2] = lin_epi(s.z, m, n + 2, e);
        dst[3] = lin_epi(s.w, m, n + 3, e);
    }
}

// Split-K factor from a wave-quantised cost model: a CU runs ceil(tiles*s / CUs) workgroups one after
// another (their MFMAs share the SIMDs), each costing its K steps plus ~2 steps of prologue/epilogue,
// plus one step for the partial-tile reduction when s > 1.  (M = 200: the 2304-wide QKV product picks
// s = 2 -> 252 workgroups, the 768-wide projections s = 6 -> 252, the 3072-wide MLP product s = 3.)
int lin_nsplit(int M, int N, int K) {
    const int64_t tiles = smc::ceil_div(smc::plan_rows(M), LBM) * smc::ceil_div(N, LBN);
    const int nks = K / LBK;
    const int64_t cus = smc::device_cu_count();
    int best = 1;
    int64_t best_cost = -1;
    for (int s = 1; s <= 16 && s <= nks; ++s) {
        const int64_t cost = smc::ceil_div(tiles * s, cus) * (smc::ceil_div(nks, s) + 2) + (s > 1 ? 1 : 0);
        if (best_cost < 0 || cost < best_cost) {
            best_cost = cost;
            best = s;
        }
    }
    return best;
}

// output tiles of a call (the in-launch split-K counters): the v2 kernel's 32 x 64 tiles, >= the v1 kernel's 32 x 128
int64_t lin_tiles(int M, int N) { return smc::ceil_div(M, 32) * smc::ceil_div(N, 64); }

int64_t lin_ws_floats(int M, int N, int K);  // defined after the v2 kernel (same plan as lin_launch)

int lin_validate(const float* a, int lda, const float* b, int ldb, const float* c, int ldc, int M, int N, int K) {
    SMC_CHECK(a && b && c, "smc_linear_f32: null pointer");
    SMC_CHECK(M >= 1 && N >= 1 && K >= 1, "smc_linear_f32: bad shape M=%d N=%d K=%d", M, N, K);
    if (K % LBK != 0 || N % 4 != 0) {
        smc::set_error("smc_linear_f32: needs K %% %d == 0 and N %% 4 == 0 (M=%d N=%d K=%d)", LBK, M, N, K);
        return SMC_ERR_UNSUPPORTED;
    }
    SMC_CHECK(lda >= K && lda % 4 == 0 && ldb >= N && ldb % 4 == 0 && ldc >= N,
              "smc_linear_f32: bad leading dimensions lda=%d ldb=%d ldc=%d", lda, ldb, ldc);
    SMC_CHECK((reinterpret_cast<uintptr_t>(a) & 15) == 0 && (reinterpret_cast<uintptr_t>(b) & 15) == 0,
              "smc_linear_f32: A and B must be 16-byte aligned");
    return SMC_OK;
}

// ------------------------------------------------------------------------------------------ GEMM v2
// The default for K % 64 == 0, N % 64 == 0 (every ViT projection): a 32 x 64 output tile per 256-thread
// workgroup, waves 2 x 2, each 16 rows x 32 columns = two v_mfma_f32_16x16x4_f32 accumulators (independent,
// so they issue back to back despite the 40-cycle dependent latency).  Both operand tiles go global -> LDS
// by global_load_lds_dwordx4 (no VGPR staging) into a 2-stage ring, BK = 64:
//   A [32 rows][64 k]  row-major, float4 column c of row i stored at slot c ^ (i & 15): one ds_read_b128
//                      gives a lane 4 consecutive k of its row, conflict-free over the 16 rows of a group;
//   B [64 k][64 n]     row-major, float4 column c of row k stored at c ^ (((k >> 2) & 1) << 2): the two
//                      k-rows a 32-lane ds_read_b32 group touches land 16 banks apart.
// K order inside a 16-deep chunk is permuted consistently for A and B (lane group g = lane / 16 owns k
// = 4g + s at MFMA step s), which is what lets A come from one 16-B read.  Tiles are laid out XCD-aware:
// consecutive tiles share an N column block and go to the same XCD, so each weight tile is streamed into
// one L2.
constexpr int L2M = 32, L2N = 64, L2K = 64;

// The hand-off's partial-tile loads as sc1 (L1-bypassing) agent loads (diagnostic knob)
#ifndef SMC_LIN_SC1LOAD
#define SMC_LIN_SC1LOAD 0
#endif
#ifndef SMC_LIN_NST
#define SMC_LIN_NST 2
#endif
#ifndef SMC_LIN_KW
#define SMC_LIN_KW 2
#endif
// KW = 2: two wave quads per workgroup split each staged K step between them (k 0..31 / 32..63) and add their
// accumulators through LDS at the end -- twice the waves per SIMD for the same tile grid and global traffic.
// Measured (profiles/r04/lin_ab/, tools/bench_linear.py): the eight B = 4 projections 144.0 -> 134.8 us, B = 8
// unchanged; NST = 3 (two steps in flight) 2-3 % slower at both batches.
// BT: B given transposed, bt [N][K] row-major (ldb = its row pitch): the B tile is staged like the A tile (k fastest,
// XOR-swizzled float4 columns) and a B fragment (4 consecutive k of one column) is one ds_read_b128 instead of four
// ds_read_b32.  Every ViT projection has both orientations in the packed buffer (W^T for the forward, W for the
// data gradient), so the executor hands each call the other one.
template <int NST, int KW, bool BT>
__global__ __launch_bounds__(256 * KW, 2) void lin_gemm2_kernel(LinParams p, int mt, int ntl) {
    constexpr int ATILE = L2M * L2K, BTILE = L2K * L2N, STAGE = ATILE + BTILE;
    constexpr int AJ = 2 / KW, BJ = 4 / KW, DW = AJ + BJ;  // DMAs per wave: A, B, per step
    __shared__ __attribute__((aligned(16))) float smem[NST * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wq = wave & 3, kg = wave >> 2;
    const int wm = wq >> 1, wn = wq & 1;
    // XCD-aware tile order (bijective for any grid size)
    const int nb = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
    const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int m_tile = lin % mt;
    const int rest = lin / mt;
    const int n_tile = rest % ntl;
    const int split = rest / ntl;
    const int m0 = m_tile * L2M, n0 = n_tile * L2N;
    const int nks = p.K / L2K;
    const int ks0 = (int)((int64_t)nks * split / p.nsplit);
    const int ks1 = (int)((int64_t)nks * (split + 1) / p.nsplit);

    auto issue = [&](int ks, int slot) {
        float* As = smem + slot * STAGE;
        float* Bs = As + ATILE;
        const int k0 = ks * L2K;
        // A: 512 float4 slots = 8 DMAs, AJ per wave; slot v -> row v/16, physical column v%16
#pragma unroll
        for (int j = 0; j < AJ; ++j) {
            const int base = (wave * AJ + j) * 256;          // float offset of this DMA in the tile
            const int v = base / 4 + lane;
            const int row = v >> 4, cphys = v & 15;
            const int c = cphys ^ (row & 15);
            const int grow = min(m0 + row, p.M - 1);
            __builtin_amdgcn_global_load_lds((const void*)(p.a + (int64_t)grow * p.lda + k0 + 4 * c),
                                             (__attribute__((address_space(3))) void*)(As + base), 16, 0, 0);
        }
        // B: 1024 float4 slots = 16 DMAs, BJ per wave; slot v -> k-row v/16, physical column v%16
        // (BT: n-row v/16 of bt, physical k-column v%16, swizzled as A)
#pragma unroll
        for (int j = 0; j < BJ; ++j) {
            const int base = (wave * BJ + j) * 256;
            const int v = base / 4 + lane;
            const int row = v >> 4, cphys = v & 15;
            const float* src;
            if constexpr (BT) {
                src = p.b + (int64_t)(n0 + row) * p.ldb + k0 + 4 * (cphys ^ (row & 15));
            } else {
                src = p.b + (int64_t)(k0 + row) * p.ldb + n0 + 4 * (cphys ^ (((row >> 2) & 1) << 2));
            }
            __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(Bs + base),
                                             16, 0, 0);
        }
    };

    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int i = lane & 15, g = lane >> 4;  // A row / B column within the block, k group
    const int arow = wm * 16 + i;
    // NST-stage ring: NST - 1 steps in flight ahead of the one being multiplied (DW DMAs per wave per step)
#pragma unroll
    for (int j = 0; j < NST - 1; ++j)
        if (ks0 + j < ks1) issue(ks0 + j, j);
    for (int ks = ks0; ks < ks1; ++ks) {
        const int ahead = min(NST - 2, ks1 - 1 - ks);  // later steps that may stay in flight
        if (NST >= 4 && ahead >= 2)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DW) : "memory");
        else if (NST >= 3 && ahead >= 1)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DW) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (ks + NST - 1 < ks1) issue(ks + NST - 1, (ks + NST - 1 - ks0) % NST);
        const float* As = smem + ((ks - ks0) % NST) * STAGE;
        const float* Bs = As + ATILE;
#pragma unroll
        for (int kc = kg * (L2K / KW); kc < (kg + 1) * (L2K / KW); kc += 16) {
            // A: row arow, k = kc + 4g .. +3 -> logical float4 column (kc/4 + g)
            const int ca = (kc / 4 + g) ^ (arow & 15);
            const f32x4 av = *reinterpret_cast<const f32x4*>(As + arow * L2K + 4 * ca);
            float bv[2][4];
            if constexpr (BT) {
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    const int n = wn * 32 + blk * 16 + i;
                    const f32x4 b4 = *reinterpret_cast<const f32x4*>(Bs + n * L2K + 4 * ((kc / 4 + g) ^ (n & 15)));
#pragma unroll
                    for (int s2 = 0; s2 < 4; ++s2) bv[blk][s2] = b4[s2];
                }
            } else {
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    const int krow = kc + 4 * g + s2;
                    const int sw = ((krow >> 2) & 1) << 2;
#pragma unroll
                    for (int blk = 0; blk < 2; ++blk) {
                        const int n = wn * 32 + blk * 16 + i;
                        bv[blk][s2] = Bs[krow * L2N + 4 * ((n >> 2) ^ sw) + (n & 3)];
                    }
                }
            }
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
                for (int blk = 0; blk < 2; ++blk)
                    acc[blk] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s2], bv[blk][s2], acc[blk], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (KW == 2) {  // the second quad's partial sums through LDS (every wave is past its last LDS read)
        __syncthreads();
        float* red = smem + wq * 512 + lane;
        if (kg == 1) {
#pragma unroll
            for (int blk = 0; blk < 2; ++blk)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) red[(blk * 4 + rr) * 64] = acc[blk][rr];
        }
        __syncthreads();
        if (kg == 0) {
#pragma unroll
            for (int blk = 0; blk < 2; ++blk)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) acc[blk][rr] += red[(blk * 4 + rr) * 64];
        }
    }
    const bool writer = kg == 0;
    // epilogue: block blk, register rr -> row 4g + rr, column i
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
        const int n = n0 + wn * 32 + blk * 16 + i;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int m = m0 + wm * 16 + 4 * g + rr;
            if (m >= p.M || !writer) continue;
            if (p.nsplit == 1)
                p.c[(int64_t)m * p.ldc + n] = lin_epi(acc[blk][rr], m, n, p.e);
            else if (p.counters)  // write-through (sc1): the hand-off below needs no release fence
                __hip_atomic_store(p.ws + ((int64_t)split * p.M + m) * p.N + n, acc[blk][rr], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            else
                p.ws[((int64_t)split * p.M + m) * p.N + n] = acc[blk][rr];
        }
    }
    if (p.nsplit == 1 || !p.counters) return;
    // In-launch split-K hand-off (cdna_hip_programming.md section 6 Guideline 16, R1 counter form): every wave drains
    // its write-through partial stores, one lane takes a ticket, the last split's workgroup acquires and sums the
    // partials in split order (the separate epilogue kernel's order).  Measured (profiles/r02_splitk_inlaunch_ab):
    // ViT-B/32 B = 8 fwd + bwd 4.7-5.0 -> 3.7 ms, no-grad fwd 1.60 -> 1.70 ms; the same hand-off in the synthesis /
    // IR-SE50 conv GEMM lost (layer set 10.75 -> 11.7 ms), so that one keeps its reduction kernel.
    int* flag = reinterpret_cast<int*>(smem);  // the k-loop is over: the LDS array is free
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int prev = __hip_atomic_fetch_add(p.counters + n_tile * mt + m_tile, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == p.nsplit - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    if (!*flag || !writer) return;
    // split-major sums: all 8 loads of one split in flight before the adds; rows past M re-read row M - 1
    float v[2][4];
    for (int k = 0; k < p.nsplit; ++k) {
        const float* part = p.ws + (int64_t)k * p.M * p.N;
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int m = min(m0 + wm * 16 + 4 * g + rr, p.M - 1);
                const float* src = part + (int64_t)m * p.N + n0 + wn * 32 + blk * 16 + i;
                const float t = SMC_LIN_SC1LOAD ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *src;
                v[blk][rr] = k == 0 ? t : v[blk][rr] + t;
            }
    }
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
        const int n = n0 + wn * 32 + blk * 16 + i;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int m = m0 + wm * 16 + 4 * g + rr;
            if (m < p.M) p.c[(int64_t)m * p.ldc + n] = lin_epi(v[blk][rr], m, n, p.e);
        }
    }
}

// ------------------------------------------------------------------------------------------ GEMM, split-bf16
// lin_gemm2_kernel with the fp32 products as three-term bf16 splits on v_mfma_f32_16x16x32_bf16 (the scheme of
// conv_gemm.hip's conv_gemm_x3_kernel: a = a0 + a1 + a2 exactly, six products a_i b_j with i + j <= 2, error per
// product <= 2^-23 |a b|).  Same 32 x 64 tiles, 2-stage DMA ring, XCD order, split-K hand-off and epilogue; the
// frozen B operand comes pre-split as planes [K/32][3][4][N][8] bf16 (lin_x3_planes_kernel), so a B fragment (8
// consecutive k of one column) is one conflict-free ds_read_b128 per term; the A tile stays fp32 (its XOR-swizzled
// image of lin_gemm2_kernel) and each wave splits its A fragment (8 consecutive k of one row) in registers, once for
// the wave's two column blocks.
typedef short bf16x8v __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void lin_split8(const float (&x)[8], bf16x8v (&t)[3]) {
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
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 w0, w1, w2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        w0[j] = __builtin_amdgcn_perm(u0[2 * j + 1], u0[2 * j], 0x07060302u);
        w1[j] = __builtin_amdgcn_perm(u1[2 * j + 1], u1[2 * j], 0x07060302u);
        w2[j] = __builtin_amdgcn_perm(u2[2 * j + 1], u2[2 * j], 0x07060302u);
    }
    t[0] = __builtin_bit_cast(bf16x8v, w0);
    t[1] = __builtin_bit_cast(bf16x8v, w1);
    t[2] = __builtin_bit_cast(bf16x8v, w2);
}

// planes of a row-major [K][N] fp32 matrix (ldb floats per row): term s of b[k][n] at
// ((((k / 32) * 3 + s) * 4 + (k % 32) / 8) * N + n) * 8 + k % 8
__global__ __launch_bounds__(256) void lin_x3_planes_kernel(const float* b, int ldb, int K, int N, short* out) {
    const int64_t total = (int64_t)K * N;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int ke = (int)(e & 7);
        int64_t r = e >> 3;
        const int n = (int)(r % N);
        r /= N;
        const int g = (int)(r & 3);
        const int kb = (int)(r >> 2);
        const int k = kb * 32 + g * 8 + ke;
        const float v = b[(int64_t)k * ldb + n];
        const unsigned u = __float_as_uint(v);
        const float r1 = v - __uint_as_float(u & 0xffff0000u);
        const unsigned w = __float_as_uint(r1);
        const float r2 = r1 - __uint_as_float(w & 0xffff0000u);
        const unsigned term[3] = {u >> 16, w >> 16, __float_as_uint(r2) >> 16};
#pragma unroll
        for (int s = 0; s < 3; ++s)
            out[((((int64_t)kb * 3 + s) * 4 + g) * N + n) * 8 + ke] = (short)term[s];
    }
}

__global__ __launch_bounds__(256, 2) void lin_gemm2_x3_kernel(LinParams p, const short* bx3, int mt, int ntl) {
    constexpr int ABYTES = L2M * L2K * 4;               // A tile [32][64] fp32
    constexpr int BBYTES = (L2K / 32) * 12 * L2N * 16;  // B planes [2][3][4][64][8] bf16
    constexpr int STAGE = ABYTES + BBYTES;
    constexpr int BDMA = BBYTES / 1024;                 // 24 1-KB DMAs, 6 per wave
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int nb = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
    const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int m_tile = lin % mt;
    const int rest = lin / mt;
    const int n_tile = rest % ntl;
    const int split = rest / ntl;
    const int m0 = m_tile * L2M, n0 = n_tile * L2N;
    const int nks = p.K / L2K;
    const int ks0 = (int)((int64_t)nks * split / p.nsplit);
    const int ks1 = (int)((int64_t)nks * (split + 1) / p.nsplit);

    auto issue = [&](int ks, int slot) {
        char* st = smem + slot * STAGE;
        float* As = reinterpret_cast<float*>(st);
        const int k0 = ks * L2K;
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // A: as lin_gemm2_kernel
            const int base = (wave * 2 + j) * 256;
            const int v = base / 4 + lane;
            const int row = v >> 4, cphys = v & 15;
            const int c = cphys ^ (row & 15);
            const int grow = min(m0 + row, p.M - 1);
            __builtin_amdgcn_global_load_lds((const void*)(p.a + (int64_t)grow * p.lda + k0 + 4 * c),
                                             (__attribute__((address_space(3))) void*)(As + base), 16, 0, 0);
        }
        // B planes: lane L of the step's 1536 16-B lanes -> (chunk kc, run = term * 4 + octet, column n)
#pragma unroll
        for (int j = 0; j < BDMA / 4; ++j) {
            const int jj = wave * (BDMA / 4) + j;
            const int L = jj * 64 + lane;
            const int kc = L / (12 * L2N), rem = L - kc * (12 * L2N);
            const int run = rem / L2N, n = rem - run * L2N;
            const short* src = bx3 + ((((int64_t)(k0 / 32 + kc) * 12 + run) * p.N) + n0 + n) * 8;
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(st + ABYTES + jj * 1024), 16, 0, 0);
        }
    };

    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int i = lane & 15, g = lane >> 4;
    const int arow = wm * 16 + i;
    if (ks0 < ks1) issue(ks0, 0);
    for (int ks = ks0; ks < ks1; ++ks) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (ks + 1 < ks1) issue(ks + 1, (ks + 1 - ks0) & 1);
        const char* st = smem + ((ks - ks0) & 1) * STAGE;
        const float* As = reinterpret_cast<const float*>(st);
        const short* Bs = reinterpret_cast<const short*>(st + ABYTES);
#pragma unroll
        for (int kc = 0; kc < L2K / 32; ++kc) {
            const int c0 = kc * 8 + 2 * g;  // float4 columns of k = 32 kc + 8 g .. + 7
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(As + arow * L2K + 4 * (c0 ^ (arow & 15)));
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(As + arow * L2K + 4 * ((c0 + 1) ^ (arow & 15)));
            const float xv[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
            bf16x8v at[3], bt[2][3];
            lin_split8(xv, at);
#pragma unroll
            for (int blk = 0; blk < 2; ++blk)
#pragma unroll
                for (int s = 0; s < 3; ++s)
                    bt[blk][s] = *reinterpret_cast<const bf16x8v*>(
                        Bs + (((kc * 3 + s) * 4 + g) * L2N + wn * 32 + blk * 16 + i) * 8);
#pragma unroll
            for (int blk = 0; blk < 2; ++blk) {
                acc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[2], bt[blk][0], acc[blk], 0, 0, 0);
                acc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[1], bt[blk][1], acc[blk], 0, 0, 0);
                acc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[0], bt[blk][2], acc[blk], 0, 0, 0);
                acc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[1], bt[blk][0], acc[blk], 0, 0, 0);
                acc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[0], bt[blk][1], acc[blk], 0, 0, 0);
                acc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[0], bt[blk][0], acc[blk], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // epilogue and split-K hand-off: as lin_gemm2_kernel (the 16x16x32 C layout is the 16x16x4 one)
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
        const int n = n0 + wn * 32 + blk * 16 + i;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int m = m0 + wm * 16 + 4 * g + rr;
            if (m >= p.M) continue;
            if (p.nsplit == 1)
                p.c[(int64_t)m * p.ldc + n] = lin_epi(acc[blk][rr], m, n, p.e);
            else if (p.counters)
                __hip_atomic_store(p.ws + ((int64_t)split * p.M + m) * p.N + n, acc[blk][rr], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            else
                p.ws[((int64_t)split * p.M + m) * p.N + n] = acc[blk][rr];
        }
    }
    if (p.nsplit == 1 || !p.counters) return;
    int* flag = reinterpret_cast<int*>(smem);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int prev = __hip_atomic_fetch_add(p.counters + n_tile * mt + m_tile, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == p.nsplit - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    float v[2][4];
    for (int k = 0; k < p.nsplit; ++k) {
        const float* part = p.ws + (int64_t)k * p.M * p.N;
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int m = min(m0 + wm * 16 + 4 * g + rr, p.M - 1);
                const float* src = part + (int64_t)m * p.N + n0 + wn * 32 + blk * 16 + i;
                const float t = SMC_LIN_SC1LOAD ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *src;
                v[blk][rr] = k == 0 ? t : v[blk][rr] + t;
            }
    }
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
        const int n = n0 + wn * 32 + blk * 16 + i;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int m = m0 + wm * 16 + 4 * g + rr;
            if (m < p.M) p.c[(int64_t)m * p.ldc + n] = lin_epi(v[blk][rr], m, n, p.e);
        }
    }
}

bool lin_v2_ok(int N, int K, int lda, int ldb) {
    return K % L2K == 0 && N % L2N == 0 && lda % 4 == 0 && ldb % 4 == 0;
}

// In-launch split-K hand-off in the executor's GEMMs (0: the separate reduction kernel; diagnostic knob)
#ifndef SMC_LIN_INLAUNCH
#define SMC_LIN_INLAUNCH 1
#endif
// Split-K planned for 1 / SMC_LIN_CU_DIV of the CUs: in the step CLIP runs beside IR-SE50 (and the prefetched
// synthesis), and fewer, longer splits leave CUs to the other chain.  Measured (profiles/r05/loss_split/, interleaved):
// 1 -> 2: 469.1 -> 471.0 images/s over three rounds (459.3 / 463.9 -> 466.8 / 467.0 in the first A/B); 4: 471.1.
#ifndef SMC_LIN_CU_DIV
#define SMC_LIN_CU_DIV 2
#endif
int lin_nsplit2(int M, int N, int K) {
    const int64_t tiles = smc::ceil_div(smc::plan_rows(M), L2M) * (N / L2N);
    const int nks = K / L2K;
    const int64_t cus = std::max<int64_t>(1, smc::device_cu_count() / SMC_LIN_CU_DIV);
    int best = 1;
    int64_t best_cost = -1;
    for (int s = 1; s <= 16 && s <= nks; ++s) {
        const int64_t cost = smc::ceil_div(tiles * s, cus) * (smc::ceil_div(nks, s) + 2) + (s > 1 ? 1 : 0);
        if (best_cost < 0 || cost < best_cost) {
            best_cost = cost;
            best = s;
        }
    }
    return best;
}

int64_t lin_ws_floats(int M, int N, int K) {
    // v2 needs lda/ldb % 4 == 0, which every caller guarantees (lin_validate rejects the rest)
    const int s = lin_v2_ok(N, K, 4, 4) ? lin_nsplit2(M, N, K) : lin_nsplit(M, N, K);
    return s > 1 ? (int64_t)s * M * N : 0;
}

#ifndef SMC_LIN_BT
#define SMC_LIN_BT 1
#endif
// bt (optional): the same B transposed, [N][K] row-major with row pitch K; used by the v2 kernel (SMC_LIN_BT)
int lin_launch(const float* a, int lda, const float* b, int ldb, float* c, int ldc, int M, int N, int K,
               const smc_linear_epilogue* epi, float* ws, int64_t ws_bytes, hipStream_t st, int* counters = nullptr,
               const short* bx3 = nullptr, const float* bt = nullptr) {
    int rc = lin_validate(a, lda, b, ldb, c, ldc, M, N, K);
    if (rc != SMC_OK) return rc;
    LinParams p{};
    p.a = a; p.lda = lda; p.b = b; p.ldb = ldb; p.c = c; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
    if (epi) p.e = *epi;
    const bool v2 = lin_v2_ok(N, K, lda, ldb);
    p.nsplit = v2 ? lin_nsplit2(M, N, K) : lin_nsplit(M, N, K);
    if (p.nsplit > 1) {
        const int64_t need = (int64_t)p.nsplit * M * N * (int64_t)sizeof(float);
        SMC_CHECK(ws && ws_bytes >= need, "smc_linear_f32: workspace %lld < %lld bytes", (long long)ws_bytes,
                  (long long)need);
        p.ws = ws;
        p.counters = counters;
    }
    if (v2 && bx3) {  // split-bf16 products (B given as planes over the same [K][N])
        const int mt = (int)smc::ceil_div(M, L2M), ntl = N / L2N;
        hipLaunchKernelGGL(lin_gemm2_x3_kernel, dim3((unsigned)(mt * ntl * p.nsplit)), dim3(256), 0, st, p, bx3, mt, ntl);
    } else if (v2) {
        const int mt = (int)smc::ceil_div(M, L2M), ntl = N / L2N;
        if (SMC_LIN_BT && bt && K % 4 == 0 && (reinterpret_cast<uintptr_t>(bt) & 15) == 0) {
            LinParams q = p;
            q.b = bt;
            q.ldb = K;
            hipLaunchKernelGGL((lin_gemm2_kernel<SMC_LIN_NST, SMC_LIN_KW, true>), dim3((unsigned)(mt * ntl * p.nsplit)),
                               dim3(256 * SMC_LIN_KW), 0, st, q, mt, ntl);
        } else {
            hipLaunchKernelGGL((lin_gemm2_kernel<SMC_LIN_NST, SMC_LIN_KW, false>), dim3((unsigned)(mt * ntl * p.nsplit)),
                               dim3(256 * SMC_LIN_KW), 0, st, p, mt, ntl);
        }
    } else {
        dim3 grid((unsigned)smc::ceil_div(M, LBM), (unsigned)smc::ceil_div(N, LBN), (unsigned)p.nsplit);
        hipLaunchKernelGGL(lin_gemm_kernel, grid, dim3(LNT), 0, st, p);
    }
    rc = smc::check_launch("smc_linear_f32");
    if (rc != SMC_OK || p.nsplit == 1 || p.counters) return rc;
    const int64_t nv = (int64_t)M * (N / 4);
    const int blocks = (int)std::min<int64_t>(smc::ceil_div(nv, 256), 4096);
    hipLaunchKernelGGL(lin_splitk_epilogue_kernel, dim3(blocks), dim3(256), 0, st, ws, p.nsplit, c, ldc, M, N, p.e);
    return smc::check_launch("smc_linear_f32 (split-K epilogue)");
}

// ------------------------------------------------------------------------------------------ LayerNorm
// One wave per row, D <= 1024 (D % 64 == 0): the row sits in registers, two-pass mean / variance
// (biased, as nn.LayerNorm), y = (x - mean) * rstd * w + b.  Backward (data gradient only):
//   dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w,  plus an optional residual gradient.

constexpr int LN_MAXV = 16;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* x, int64_t ldx, const float* w, const float* b,
                                                     float* y, int64_t ldy, float* mean_out, float* rstd_out, int M,
                                                     int D, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    const int nv = D >> 6;
    const float* xr = x + row * ldx;
    // every load issued before the first add (clamped column, zeroed past the row): loaded under a `t < nv`
    // branch, each add waited out its own load
    float v[LN_MAXV];
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) v[t] = xr[lane + 64 * min(t, nv - 1)];
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
        v[t] = t < nv ? v[t] : 0.f;
        s += v[t];
    }
    const float mean = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
        const float d = t < nv ? v[t] - mean : 0.f;
        q += d * d;
    }
    const float rstd = rsqrtf(wave_sum(q) / D + eps);
    // the affine parameters loaded before the first store (loaded next to each store, every column waited out the
    // previous column's store: vmcnt counts both)
    float wv[LN_MAXV], bv[LN_MAXV];
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
        const int c = lane + 64 * min(t, nv - 1);
        wv[t] = w[c];
        bv[t] = b[c];
    }
    float* yr = y + row * ldy;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
        if (t >= nv) break;
        const int c = lane + 64 * t;
        yr[c] = (v[t] - mean) * rstd * wv[t] + bv[t];
    }
    if (lane == 0) {
        if (mean_out) mean_out[row] = mean;
        if (rstd_out) rstd_out[row] = rstd;
    }
}

__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                                     const float* mean_in, const float* rstd_in, const float* w,
                                                     const float* dres, int64_t ldres, float* dx, int64_t lddx, int M,
                                                     int D) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    const int nv = D >> 6;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float g[LN_MAXV], xh[LN_MAXV];
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {  // all loads first (clamped column), as in ln_fwd_kernel
        const int c = lane + 64 * min(t, nv - 1);
        g[t] = dy[row * lddy + c] * w[c];
        xh[t] = (x[row * ldx + c] - mean) * rstd;
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
        g[t] = t < nv ? g[t] : 0.f;
        xh[t] = t < nv ? xh[t] : 0.f;
        s1 += g[t];
        s2 += g[t] * xh[t];
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
    float rv[LN_MAXV];  // the residual gradient loaded before the first store (as in ln_fwd_kernel)
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) rv[t] = dres ? dres[row * ldres + lane + 64 * min(t, nv - 1)] : 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
        if (t >= nv) break;
        const int c = lane + 64 * t;
        float v = rstd * (g[t] - m1 - xh[t] * m2);
        if (dres) v += rv[t];
        dx[row * lddx + c] = v;
    }
}

// ------------------------------------------------------------------------------------------ attention
// softmax(Q K^T * scale) V per (image, head), head dim 64, Q/K/V read from the fused projection
// qkv[M][3D] (nn.MultiheadAttention in_proj order q | k | v, head h at columns h*64).  A workgroup owns
// AQB query rows of one (image, head) with the whole K and V of that head in LDS (row pitch 65: the
// column-walking reads of the dot products hit 32 distinct banks).  scale = 1/8 is a power of two, so
// scaling Q before the product is bit-identical to scaling the logits.  P is saved for the backward.

constexpr int HD = 64, HP = 65, AQB = 16, AQB_BWD_SINGLE = 64;

// Stage `rows` rows of 64 floats (global row stride ld) into LDS rows of pitch HP, times `mul`; rows >= valid
// are zero.  Eight elements per thread are loaded before any is written: written as they arrive, every LDS
// store waited out its own global round trip (the staging was most of the attention kernels' time).
__device__ __forceinline__ void stage_rows64(float* dst, const float* src, int64_t ld, int rows, int valid, float mul) {
    constexpr int CH = 8;
    const int n = rows * HD;
    for (int i0 = threadIdx.x; i0 < n; i0 += 256 * CH) {
        float v[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int idx = i0 + 256 * k;
            v[k] = src[(int64_t)min(idx >> 6, valid - 1) * ld + (idx & 63)];
        }
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int idx = i0 + 256 * k, j = idx >> 6;
            if (idx < n) dst[j * HP + (idx & 63)] = j < valid ? v[k] * mul : 0.f;
        }
    }
}

// Several row blocks of 64 floats (16-B aligned rows, ld % 4 == 0) into LDS rows of pitch HP in ONE batch of 16-B
// loads: up to KMAX float4 per thread are in flight before the first LDS store (the K, V, Q, dO blocks of an attention
// backward workgroup: one global round trip instead of one per 2048-element chunk of each block; 28.8 -> 27.8 us per
// launch, profiles/r05/attn_stage/).
struct StageSeg {
    float* dst;
    const float* src;
    int64_t ld;
    int rows, valid;
    float mul;
};

typedef __attribute__((address_space(3))) float lds_float;

// The segment fields of global float4 index g, selected by compares over the unrolled segment list (constant indices
// only: a dynamically indexed StageSeg array lives in scratch, and its LDS pointers then come back as generic pointers,
// so the stores below became flat_store_dwordx4 at 4-B aligned LDS addresses -- the HP = 65 pitch -- which corrupted
// one dword of a staged float4 now and then while other kernels shared the CU (round 6)).
template <int NSEG>
__device__ __forceinline__ void stage_pick(const StageSeg (&s)[NSEG], const int (&start)[NSEG + 1], int g, int& si,
                                           int& loc) {
    si = 0;
#pragma unroll
    for (int i = 1; i < NSEG; ++i) si = g >= start[i] ? i : si;
    int base = start[0];
#pragma unroll
    for (int i = 1; i < NSEG; ++i) base = si == i ? start[i] : base;
    loc = g - base;
}

template <int NSEG, int KMAX>
__device__ __forceinline__ void stage_segs(const StageSeg (&s)[NSEG]) {
    int start[NSEG + 1];
    start[0] = 0;
#pragma unroll
    for (int i = 0; i < NSEG; ++i) start[i + 1] = start[i] + s[i].rows * (HD / 4);
    const int total = start[NSEG];
    for (int g0 = 0; g0 < total; g0 += 256 * KMAX) {
        float4 v[KMAX];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int g = min(g0 + (int)threadIdx.x + 256 * k, total - 1);
            int si, loc;
            stage_pick<NSEG>(s, start, g, si, loc);
            const float* src = s[0].src;
            int64_t ld = s[0].ld;
            int valid = s[0].valid;
#pragma unroll
            for (int i = 1; i < NSEG; ++i) {
                src = si == i ? s[i].src : src;
                ld = si == i ? s[i].ld : ld;
                valid = si == i ? s[i].valid : valid;
            }
            const int row = min(loc >> 4, valid - 1);
            v[k] = *reinterpret_cast<const float4*>(src + (int64_t)row * ld + 4 * (loc & 15));
        }
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int g = g0 + (int)threadIdx.x + 256 * k;
            if (g >= total) continue;
            int si, loc;
            stage_pick<NSEG>(s, start, g, si, loc);
            float* dst = s[0].dst;
            int valid = s[0].valid;
            float m = s[0].mul;
#pragma unroll
            for (int i = 1; i < NSEG; ++i) {
                dst = si == i ? s[i].dst : dst;
                valid = si == i ? s[i].valid : valid;
                m = si == i ? s[i].mul : m;
            }
            const int row = loc >> 4, c = 4 * (loc & 15);
            const bool ok = row < valid;
            // dword LDS stores through an LDS-typed pointer (row pitch HP = 65 floats: 4-B alignment only)
            lds_float* d = (lds_float*)(dst + row * HP + c);
            d[0] = ok ? v[k].x * m : 0.f;
            d[1] = ok ? v[k].y * m : 0.f;
            d[2] = ok ? v[k].z * m : 0.f;
            d[3] = ok ? v[k].w * m : 0.f;
        }
    }
}

__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* qkv, float* out, float* psave, int L, int H,
                                                       float scale, int causal) {
    extern __shared__ float sm[];
    float* Ks = sm;
    float* Vs = Ks + L * HP;
    float* Qs = Vs + L * HP;
    float* Ss = Qs + AQB * HP;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q0 = blockIdx.x * AQB, h = blockIdx.y, b = blockIdx.z;
    const int D = H * HD, ld = 3 * D;
    const float* base = qkv + (int64_t)b * L * ld + h * HD;
    const int nq = min(AQB, L - q0);
    // (row staging: the one-batch 16-B staging of the backward measured slower here, 17.4 -> 20.7 us per launch,
    // profiles/r05/attn_stage/)
    stage_rows64(Ks, base + D, ld, L, L, 1.f);
    stage_rows64(Vs, base + 2 * D, ld, L, L, 1.f);
    stage_rows64(Qs, base + (int64_t)q0 * ld, ld, AQB, nq, scale);
    __syncthreads();
    for (int idx = tid; idx < nq * L; idx += 256) {
        const int i = idx / L, j = idx - i * L;
        float s = 0.f;
#pragma unroll 16
        for (int d = 0; d < HD; ++d) s = fmaf(Qs[i * HP + d], Ks[j * HP + d], s);
        // causal: the -inf upper triangle of CLIP's text mask (attn_mask triu(1)); exp -> exactly 0
        Ss[i * L + j] = (causal && j > q0 + i) ? -INFINITY : s;
    }
    __syncthreads();
    for (int i = wave; i < nq; i += 4) {
        float mx = -INFINITY;
        for (int j = lane; j < L; j += 64) mx = fmaxf(mx, Ss[i * L + j]);
        mx = wave_max(mx);
        float sum = 0.f;
        for (int j = lane; j < L; j += 64) {
            const float e = expf(Ss[i * L + j] - mx);
            Ss[i * L + j] = e;
            sum += e;
        }
        const float inv = 1.f / wave_sum(sum);
        float* prow = psave ? psave + (((int64_t)b * H + h) * L + q0 + i) * L : nullptr;
        for (int j = lane; j < L; j += 64) {
            const float pv = Ss[i * L + j] * inv;
            Ss[i * L + j] = pv;
            if (prow) prow[j] = pv;
        }
    }
    __syncthreads();
    for (int idx = tid; idx < nq * HD; idx += 256) {
        const int i = idx >> 6, d = idx & 63;
        float o = 0.f;
        for (int j = 0; j < L; ++j) o = fmaf(Ss[i * L + j], Vs[j * HP + d], o);
        out[((int64_t)b * L + q0 + i) * D + h * HD + d] = o;
    }
}

// Backward: dP = dO V^T, dS = P * (dP - rowsum(dP * P)), dQ = scale dS K, dK = dS^T (scale Q), dV = P^T dO.
// QB query rows per workgroup; with one query block per head (L <= 64) dK/dV are plain stores,
// otherwise the blocks add into a zeroed dqkv with float atomics.
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float* dout, const float* qkv, const float* psave,
                                                       float* dqkv, int L, int H, float scale, int QB, int atomic) {
    extern __shared__ float sm[];
    float* Ks = sm;
    float* Vs = Ks + L * HP;
    float* Qs = Vs + L * HP;
    float* dOs = Qs + QB * HP;
    float* Ps = dOs + QB * HP;
    float* dSs = Ps + QB * L;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q0 = blockIdx.x * QB, h = blockIdx.y, b = blockIdx.z;
    const int D = H * HD, ld = 3 * D;
    const int nq = min(QB, L - q0);
    const float* base = qkv + (int64_t)b * L * ld + h * HD;
    const float* pbase = psave + (((int64_t)b * H + h) * L + q0) * L;
    // P block (contiguous, not 16-B aligned): its first 8 loads per thread are issued before the K / V / Q / dO batch
    float pv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) pv[k] = pbase[min(tid + 256 * k, nq * L - 1)];
    {
        const StageSeg segs[4] = {{Ks, base + D, ld, L, L, 1.f},
                                  {Vs, base + 2 * D, ld, L, L, 1.f},
                                  {Qs, base + (int64_t)q0 * ld, ld, QB, nq, scale},
                                  {dOs, dout + ((int64_t)b * L + q0) * D + h * HD, D, QB, nq, 1.f}};
        stage_segs<4, 10>(segs);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int idx = tid + 256 * k;
        if (idx < QB * L) Ps[idx] = idx < nq * L ? pv[k] : 0.f;
    }
    for (int i0 = tid + 256 * 8; i0 < QB * L; i0 += 256 * 8) {  // the rest of P (QB * L > 2048: long sequences)
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = pbase[min(i0 + 256 * k, nq * L - 1)];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int idx = i0 + 256 * k;
            if (idx < QB * L) Ps[idx] = idx < nq * L ? v[k] : 0.f;
        }
    }
    __syncthreads();
    for (int idx = tid; idx < nq * L; idx += 256) {
        const int i = idx / L, j = idx - i * L;
        float s = 0.f;
#pragma unroll 16
        for (int d = 0; d < HD; ++d) s = fmaf(dOs[i * HP + d], Vs[j * HP + d], s);
        dSs[idx] = s;
    }
    __syncthreads();
    for (int i = wave; i < nq; i += 4) {
        float t = 0.f;
        for (int j = lane; j < L; j += 64) t += dSs[i * L + j] * Ps[i * L + j];
        t = wave_sum(t);
        for (int j = lane; j < L; j += 64) dSs[i * L + j] = Ps[i * L + j] * (dSs[i * L + j] - t);
    }
    for (int idx = tid; idx < (QB - nq) * L; idx += 256) dSs[nq * L + idx] = 0.f;  // rows past L: no contribution
    __syncthreads();
    float* dbase = dqkv + (int64_t)b * L * ld + h * HD;
    for (int idx = tid; idx < nq * HD; idx += 256) {
        const int i = idx >> 6, d = idx & 63;
        float g = 0.f;
        for (int j = 0; j < L; ++j) g = fmaf(dSs[i * L + j], Ks[j * HP + d], g);
        dbase[(int64_t)(q0 + i) * ld + d] = g * scale;
    }
    for (int idx = tid; idx < L * HD; idx += 256) {
        const int j = idx >> 6, d = idx & 63;
        float gk = 0.f, gv = 0.f;
        for (int i = 0; i < nq; ++i) {
            gk = fmaf(dSs[i * L + j], Qs[i * HP + d], gk);
            gv = fmaf(Ps[i * L + j], dOs[i * HP + d], gv);
        }
        float* dk = dbase + (int64_t)j * ld + D + d;
        float* dv = dbase + (int64_t)j * ld + 2 * D + d;
        if (atomic) {
            atomicAdd(dk, gk);
            atomicAdd(dv, gv);
        } else {
            *dk = gk;
            *dv = gv;
        }
    }
}

size_t attn_fwd_lds(int L) { return sizeof(float) * (size_t)(2 * L * HP + AQB * HP + AQB * L); }
size_t attn_bwd_lds(int L, int QB) { return sizeof(float) * (size_t)(2 * L * HP + 2 * QB * HP + 2 * QB * L); }
// L <= 64: two query blocks per head (two adds onto zero commute, so the atomics stay deterministic)
// and the LDS image stays under 64 KiB; longer sequences: 16-row blocks.
#ifndef SMC_ATTN_BWD_ONEBLOCK
#define SMC_ATTN_BWD_ONEBLOCK 0
#endif
int attn_bwd_qb(int L) { return L <= AQB_BWD_SINGLE ? (SMC_ATTN_BWD_ONEBLOCK ? L : (L + 1) / 2) : AQB; }

int attn_check_lds(size_t bytes, const void* fn) {
    if (bytes > 160 * 1024) {
        smc::set_error("attention: sequence too long for the LDS-resident kernel (%zu bytes)", bytes);
        return SMC_ERR_UNSUPPORTED;
    }
    if (bytes > 64 * 1024 &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
        smc::set_error("attention: cannot raise the dynamic LDS limit to %zu bytes", bytes);
        return SMC_ERR_LAUNCH;
    }
    return SMC_OK;
}

int attn_fwd_launch(const float* qkv, float* out, float* psave, int B, int L, int H, float scale, hipStream_t st,
                    int causal = 0) {
    const size_t lds = attn_fwd_lds(L);
    int rc = attn_check_lds(lds, reinterpret_cast<const void*>(attn_fwd_kernel));
    if (rc != SMC_OK) return rc;
    hipLaunchKernelGGL(attn_fwd_kernel, dim3((unsigned)smc::ceil_div(L, AQB), H, B), dim3(256), lds, st, qkv, out,
                       psave, L, H, scale, causal);
    return smc::check_launch("smc_attention_fwd_f32");
}

int attn_bwd_launch(const float* dout, const float* qkv, const float* psave, float* dqkv, int B, int L, int H,
                    float scale, hipStream_t st) {
    const int QB = attn_bwd_qb(L);
    const int nqb = (int)smc::ceil_div(L, QB);
    const size_t lds = attn_bwd_lds(L, QB);
    SMC_CHECK((reinterpret_cast<uintptr_t>(qkv) & 15) == 0 && (reinterpret_cast<uintptr_t>(dout) & 15) == 0,
              "smc_attention_bwd_f32: qkv and dout must be 16-byte aligned");
    int rc = attn_check_lds(lds, reinterpret_cast<const void*>(attn_bwd_kernel));
    if (rc != SMC_OK) return rc;
    if (nqb > 1) SMC_TRY_MEMSET(dqkv, sizeof(float) * (size_t)B * L * 3 * H * HD, st, "smc_attention_bwd_f32: memset");
    hipLaunchKernelGGL(attn_bwd_kernel, dim3(nqb, H, B), dim3(256), lds, st, dout, qkv, psave, dqkv, L, H, scale, QB,
                       nqb > 1 ? 1 : 0);
    return smc::check_launch("smc_attention_bwd_f32");
}

// ------------------------------------------------------------------------------------ patch embedding
// conv1 (kernel = stride = patch, no bias) is a GEMM over non-overlapping patches: im2col is a pure
// permutation, so its adjoint (col2im) is the inverse permutation.
//   patches[b*G*G + gy*G + gx][c*p*p + py*p + px] = img[b][c][gy*p + py][gx*p + px]

__global__ void patch_perm_kernel(const float* src, float* dst, int B, int C, int G, int p, int to_patches) {
    const int64_t n = (int64_t)B * C * G * p * G * p;
    const int img_w = G * p;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        // i walks the image (NCHW): consecutive lanes read/write consecutive pixels of a patch row
        int64_t t = i;
        const int x = (int)(t % img_w); t /= img_w;
        const int y = (int)(t % img_w); t /= img_w;
        const int c = (int)(t % C);
        const int b = (int)(t / C);
        const int gy = y / p, py = y - gy * p, gx = x / p, px = x - gx * p;
        const int64_t pi = ((int64_t)b * G * G + gy * G + gx) * ((int64_t)C * p * p) + (int64_t)c * p * p + py * p + px;
        if (to_patches) dst[pi] = src[i];
        else dst[i] = src[pi];
    }
}

// x_pre[b][t] = (t == 0 ? cls : tok[b*(L-1) + t-1]) + pos[t]
__global__ void embed_fwd_kernel(const float* tok, const float* cls, const float* pos, float* x, int B, int L, int D) {
    const int64_t n = (int64_t)B * L * D;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int d = (int)(i % D);
        const int64_t r = i / D;
        const int t = (int)(r % L), b = (int)(r / L);
        const float v = t == 0 ? cls[d] : tok[((int64_t)b * (L - 1) + t - 1) * D + d];
        x[i] = v + pos[(int64_t)t * D + d];
    }
}

// dtok[b*(L-1) + t-1] = dx[b][t] for t >= 1
__global__ void embed_bwd_kernel(const float* dx, float* dtok, int B, int L, int D) {
    const int64_t n = (int64_t)B * (L - 1) * D;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int d = (int)(i % D);
        const int64_t r = i / D;
        const int t = (int)(r % (L - 1)) + 1, b = (int)(r / (L - 1));
        dtok[i] = dx[((int64_t)b * L + t) * D + d];
    }
}

inline unsigned ew_blocks(int64_t n) { return (unsigned)std::min<int64_t>(smc::ceil_div(n, 256), 8192); }

int ln_fwd_launch(const float* x, int64_t ldx, const float* w, const float* b, float* y, int64_t ldy, float* mean,
                  float* rstd, int M, int D, float eps, hipStream_t st) {
    if (D % 64 != 0 || D > 64 * LN_MAXV) {
        smc::set_error("layernorm: D=%d must be a multiple of 64 and <= %d", D, 64 * LN_MAXV);
        return SMC_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)smc::ceil_div(M, 4)), dim3(256), 0, st, x, ldx, w, b, y, ldy,
                       mean, rstd, M, D, eps);
    return smc::check_launch("smc_layernorm_fwd_f32");
}

int ln_bwd_launch(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* mean, const float* rstd,
                  const float* w, const float* dres, int64_t ldres, float* dx, int64_t lddx, int M, int D,
                  hipStream_t st) {
    if (D % 64 != 0 || D > 64 * LN_MAXV) {
        smc::set_error("layernorm: D=%d must be a multiple of 64 and <= %d", D, 64 * LN_MAXV);
        return SMC_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(ln_bwd_kernel, dim3((unsigned)smc::ceil_div(M, 4)), dim3(256), 0, st, dy, lddy, x, ldx, mean,
                       rstd, w, dres, ldres, dx, lddx, M, D);
    return smc::check_launch("smc_layernorm_bwd_f32");
}

// ------------------------------------------------------------------------------- packed weight layout
// Every segment starts on a 64-float boundary (16-B aligned float4 loads).

inline int64_t rnd(int64_t n) { return (n + 63) & ~int64_t(63); }

struct VitDims {
    int D, NL, H, p, G, E, C, L, P;  // P = C*p*p
    int x3;                          // split-bf16 products: the packed buffer also holds every projection's planes
};

VitDims dims(const smc_vit_config& c) {
    VitDims d;
    d.D = c.width; d.NL = c.layers; d.H = c.heads; d.p = c.patch; d.G = c.grid; d.E = c.out_dim; d.C = c.in_ch;
    d.L = c.grid * c.grid + 1;
    d.P = c.in_ch * c.patch * c.patch;
    d.x3 = c.products == 1;
    return d;
}

struct LayerW {
    const float *ln1_w, *ln1_b, *qkv_wt, *qkv_w, *qkv_b, *out_wt, *out_w, *out_b, *ln2_w, *ln2_b, *fc_wt, *fc_w,
        *fc_b, *pr_wt, *pr_w, *pr_b;
    // split-bf16 planes of the eight projections (nullptr: exact-fp32 products)
    const short *qkv_wt3, *qkv_w3, *out_wt3, *out_w3, *fc_wt3, *fc_w3, *pr_wt3, *pr_w3;
};

struct VitW {
    const float *conv_wt, *conv_w, *cls, *pos, *lnpre_w, *lnpre_b, *lnpost_w, *lnpost_b, *proj, *proj_t;
    const float* layers;  // start of layer 0
    int64_t layer_stride;
    const short *conv_wt3, *conv_w3, *proj3, *proj_t3;
    const float* layers3;  // start of layer 0's planes
    int64_t layer3_stride;
};

// floats of the split planes of a [K][N] matrix (3 bf16 terms per element), 64-float aligned
inline int64_t planes_floats(int64_t K, int64_t N) { return (K * N * 3 + 1) / 2; }

int64_t layer_floats(const VitDims& d) {
    const int64_t D = d.D;
    return 4 * rnd(D) + 2 * rnd(D * 3 * D) + rnd(3 * D) + 2 * rnd(D * D) + rnd(D) + 2 * rnd(D * 4 * D) + rnd(4 * D) +
           2 * rnd(4 * D * D) + rnd(D);
}

// Walks the layout; with base == nullptr it only counts.
int64_t layout(const VitDims& d, const float* base, VitW* w) {
    int64_t off = 0;
    auto seg = [&](int64_t n) {
        const float* ptr = base ? base + off : nullptr;
        off += rnd(n);
        return ptr;
    };
    const int64_t D = d.D;
    VitW t{};
    t.conv_wt = seg((int64_t)d.P * D);
    t.conv_w = seg(D * d.P);
    t.cls = seg(D);
    t.pos = seg((int64_t)d.L * D);
    t.lnpre_w = seg(D);
    t.lnpre_b = seg(D);
    t.layers = base ? base + off : nullptr;
    t.layer_stride = layer_floats(d);
    off += t.layer_stride * d.NL;
    t.lnpost_w = seg(D);
    t.lnpost_b = seg(D);
    t.proj = seg(D * d.E);
    t.proj_t = seg((int64_t)d.E * D);
    if (d.x3) {  // the planes region after the fp32 segments (smc_vit_pack_x3 fills it from them)
        auto pseg = [&](int64_t K, int64_t N) { return reinterpret_cast<const short*>(seg(planes_floats(K, N))); };
        t.conv_wt3 = pseg(d.P, D);
        t.conv_w3 = pseg(D, d.P);
        t.layers3 = base ? base + off : nullptr;
        t.layer3_stride = rnd(planes_floats(D, 3 * D)) + rnd(planes_floats(3 * D, D)) + 2 * rnd(planes_floats(D, D)) +
                          2 * rnd(planes_floats(D, 4 * D)) + 2 * rnd(planes_floats(4 * D, D));
        off += t.layer3_stride * d.NL;
        t.proj3 = pseg(D, d.E);
        t.proj_t3 = pseg(d.E, D);
    }
    if (w) *w = t;
    return off;
}

LayerW layer_w(const VitDims& d, const VitW& w, int l) {
    const float* base = w.layers + w.layer_stride * l;
    int64_t off = 0;
    auto seg = [&](int64_t n) {
        const float* ptr = base + off;
        off += rnd(n);
        return ptr;
    };
    const int64_t D = d.D;
    LayerW t;
    t.ln1_w = seg(D); t.ln1_b = seg(D);
    t.qkv_wt = seg(D * 3 * D); t.qkv_w = seg(3 * D * D); t.qkv_b = seg(3 * D);
    t.out_wt = seg(D * D); t.out_w = seg(D * D); t.out_b = seg(D);
    t.ln2_w = seg(D); t.ln2_b = seg(D);
    t.fc_wt = seg(D * 4 * D); t.fc_w = seg(4 * D * D); t.fc_b = seg(4 * D);
    t.pr_wt = seg(4 * D * D); t.pr_w = seg(D * 4 * D); t.pr_b = seg(D);
    t.qkv_wt3 = t.qkv_w3 = t.out_wt3 = t.out_w3 = t.fc_wt3 = t.fc_w3 = t.pr_wt3 = t.pr_w3 = nullptr;
    if (d.x3) {
        const float* b3 = w.layers3 + w.layer3_stride * l;
        int64_t o3 = 0;
        auto pseg = [&](int64_t K, int64_t N) {
            const short* ptr = reinterpret_cast<const short*>(b3 + o3);
            o3 += rnd(planes_floats(K, N));
            return ptr;
        };
        // [K][N] of each B operand: forward W^T [in][out], backward W [out][in]
        t.qkv_wt3 = pseg(D, 3 * D); t.qkv_w3 = pseg(3 * D, D);
        t.out_wt3 = pseg(D, D); t.out_w3 = pseg(D, D);
        t.fc_wt3 = pseg(D, 4 * D); t.fc_w3 = pseg(4 * D, D);
        t.pr_wt3 = pseg(4 * D, D); t.pr_w3 = pseg(D, 4 * D);
    }
    return t;
}

// ------------------------------------------------------------------------------- saved activations
struct LayerS {
    float *x_in, *mu1, *rs1, *qkv, *P, *x_mid, *mu2, *rs2, *G;
};

struct VitS {
    float *x_pre, *mu0, *rs0, *x_out, *mupost, *rspost;  // x_out: final stream (ln_post input, CLS rows used)
    float* layers;
    int64_t layer_stride;
};

int64_t saved_layer_floats(const VitDims& d, int B) {
    const int64_t M = (int64_t)B * d.L, D = d.D;
    return rnd(M * D) + 2 * rnd(M) + rnd(M * 3 * D) + rnd((int64_t)B * d.H * d.L * d.L) + rnd(M * D) + 2 * rnd(M) +
           rnd(M * 4 * D);
}

int64_t saved_layout(const VitDims& d, int B, float* base, VitS* s) {
    const int64_t M = (int64_t)B * d.L, D = d.D;
    int64_t off = 0;
    auto seg = [&](int64_t n) {
        float* ptr = base ? base + off : nullptr;
        off += rnd(n);
        return ptr;
    };
    VitS t{};
    t.x_pre = seg(M * D);
    t.mu0 = seg(M);
    t.rs0 = seg(M);
    t.x_out = seg(M * D);
    t.mupost = seg(B);
    t.rspost = seg(B);
    t.layers = base ? base + off : nullptr;
    t.layer_stride = saved_layer_floats(d, B);
    off += t.layer_stride * d.NL;
    if (s) *s = t;
    return off;
}

LayerS saved_layer(const VitDims& d, int B, const VitS& s, int l) {
    const int64_t M = (int64_t)B * d.L, D = d.D;
    float* base = s.layers + s.layer_stride * l;
    int64_t off = 0;
    auto seg = [&](int64_t n) {
        float* ptr = base + off;
        off += rnd(n);
        return ptr;
    };
    LayerS t;
    t.x_in = seg(M * D); t.mu1 = seg(M); t.rs1 = seg(M); t.qkv = seg(M * 3 * D);
    t.P = seg((int64_t)B * d.H * d.L * d.L); t.x_mid = seg(M * D); t.mu2 = seg(M); t.rs2 = seg(M);
    t.G = seg(M * 4 * D);
    return t;
}

#ifndef SMC_VIT_TRACE
#define SMC_VIT_TRACE 0
#endif
__global__ __launch_bounds__(256) void trace_copy_kernel(const float* src, float* dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

// ---------------------------------------------------------------------------------------- workspace
struct VitWs {
    float *h, *o, *big, *qkv, *P, *xa, *xb, *tok, *patches, *dx, *dh, *mu, *rs, *split;
    int64_t split_bytes;
    int* counters;           // split-K tile counters: one slice per GEMM of a pass, zeroed per pass
    int64_t counter_slice;   // ints per GEMM call
    int64_t counter_ints;
    float* trace;            // SMC_VIT_TRACE builds: intermediates of the backward (tools/det_stage.py)
};

int64_t max_tiles(const VitDims& d, int B) {
    const int M = B * d.L, D = d.D, Mt = B * d.G * d.G;
    int64_t m = 0;
    for (int64_t t : {lin_tiles(Mt, D), lin_tiles(Mt, d.P), lin_tiles(M, 3 * D), lin_tiles(M, D), lin_tiles(M, 4 * D),
                      lin_tiles(B, d.E), lin_tiles(B, D)})
        m = std::max(m, t);
    return m;
}

int gemms_per_pass(const VitDims& d) { return 4 * d.NL + 2; }

int64_t split_need(const VitDims& d, int B) {
    const int M = B * d.L, D = d.D, Mt = B * d.G * d.G;
    int64_t m = 0;
    auto upd = [&](int MM, int N, int K) { m = std::max(m, lin_ws_floats(MM, N, K)); };
    upd(Mt, D, d.P); upd(Mt, d.P, D);                 // patch embedding fwd / bwd
    upd(M, 3 * D, D); upd(M, D, 3 * D);               // qkv
    upd(M, D, D);                                     // out proj (fwd and bwd)
    upd(M, 4 * D, D); upd(M, D, 4 * D);               // fc / proj
    upd(B, d.E, D); upd(B, D, d.E);                   // head
    return m;
}

int64_t ws_layout(const VitDims& d, int B, float* base, VitWs* w) {
    const int64_t M = (int64_t)B * d.L, D = d.D, Mt = (int64_t)B * d.G * d.G;
    int64_t off = 0;
    auto seg = [&](int64_t n) {
        float* ptr = base ? base + off : nullptr;
        off += rnd(n);
        return ptr;
    };
    VitWs t{};
    t.h = seg(M * D);
    t.o = seg(M * D);
    t.big = seg(M * 4 * D);
    t.qkv = seg(M * 3 * D);
    t.P = seg((int64_t)B * d.H * d.L * d.L);
    t.xa = seg(M * D);
    t.xb = seg(M * D);
    t.tok = seg(Mt * D);
    t.patches = seg(Mt * d.P);
    t.dx = seg(M * D);
    t.dh = seg(M * D);
    t.mu = seg(M);
    t.rs = seg(M);
    const int64_t sp = split_need(d, B);
    t.split = seg(sp);
    t.split_bytes = sp * (int64_t)sizeof(float);
    t.counter_slice = max_tiles(d, B);
    t.counter_ints = t.counter_slice * gemms_per_pass(d);
    t.counters = reinterpret_cast<int*>(seg(t.counter_ints));
#if SMC_VIT_TRACE
    // A/B debug builds only (tools/det_stage.py): snapshots of the backward's intermediates, in execution order
    t.trace = seg(2 * M * D + (int64_t)d.NL * 12 * M * D + M * D + Mt * D + Mt * d.P);
#endif
    if (w) *w = t;
    return off;
}

int vit_validate(const smc_vit_config* cfg, int B) {
    SMC_CHECK(cfg, "smc_vit: null config");
    SMC_CHECK(B >= 1, "smc_vit: batch %d", B);
    SMC_CHECK(cfg->width >= 64 && cfg->layers >= 1 && cfg->heads >= 1 && cfg->patch >= 1 && cfg->grid >= 1 &&
                  cfg->out_dim >= 4 && cfg->in_ch >= 1,
              "smc_vit: bad config");
    SMC_CHECK(cfg->products == 0 || cfg->products == 1, "smc_vit: products %d (0: fp32 MFMA, 1: split-bf16)",
              cfg->products);
    if (cfg->width != cfg->heads * HD || cfg->width % 64 != 0 || cfg->width > 64 * LN_MAXV ||
        (cfg->in_ch * cfg->patch * cfg->patch) % LBK != 0 || cfg->width % LBK != 0 || cfg->out_dim % LBK != 0) {
        smc::set_error("smc_vit: unsupported config (head dim must be 64, width %% 64 == 0 <= 1024, "
                       "patch dim / out_dim %% 32 == 0)");
        return SMC_ERR_UNSUPPORTED;
    }
    return SMC_OK;
}

#define SMC_TRY(expr)                  \
    do {                               \
        const int rc_ = (expr);        \
        if (rc_ != SMC_OK) return rc_; \
    } while (0)

smc_linear_epilogue epi_none() { return smc_linear_epilogue{}; }

// Split-K partials are reduced by a separate epilogue kernel: measured on MI355X (B=4 ViT-B/32,
// tools/bench_vit.py) the in-launch hand-off's per-workgroup L2 write-back of the freshly written slabs costs
// more than the extra launch (fwd 3.06 vs 1.77 ms).
}  // namespace

// =================================================================================== C ABI: primitives

SMC_API int64_t smc_linear_workspace_size(int M, int N, int K) {
    if (M < 1 || N < 1 || K < 1 || K % LBK != 0) return 0;
    return lin_ws_floats(M, N, K) * (int64_t)sizeof(float);
}

SMC_API int smc_linear_f32(const float* a, int lda, const float* b, int ldb, float* c, int ldc, int M, int N, int K,
                           const smc_linear_epilogue* epi, float* workspace, int64_t workspace_bytes, void* stream) {
    return lin_launch(a, lda, b, ldb, c, ldc, M, N, K, epi, workspace, workspace_bytes, smc::as_stream(stream));
}

SMC_API int smc_layernorm_fwd_f32(const float* x, int64_t ldx, const float* w, const float* b, float* y, int64_t ldy,
                                  float* mean, float* rstd, int rows, int dim, float eps, void* stream) {
    SMC_CHECK(x && w && b && y && rows >= 1, "smc_layernorm_fwd_f32: bad arguments");
    return ln_fwd_launch(x, ldx, w, b, y, ldy, mean, rstd, rows, dim, eps, smc::as_stream(stream));
}

SMC_API int smc_layernorm_bwd_f32(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* mean,
                                  const float* rstd, const float* w, const float* dres, int64_t ldres, float* dx,
                                  int64_t lddx, int rows, int dim, void* stream) {
    SMC_CHECK(dy && x && mean && rstd && w && dx && rows >= 1, "smc_layernorm_bwd_f32: bad arguments");
    return ln_bwd_launch(dy, lddy, x, ldx, mean, rstd, w, dres, ldres, dx, lddx, rows, dim, smc::as_stream(stream));
}

SMC_API int smc_attention_fwd_f32(const float* qkv, float* out, float* p_save, int batch, int tokens, int heads,
                                  int head_dim, float scale, void* stream) {
    SMC_CHECK(qkv && out && batch >= 1 && tokens >= 1 && heads >= 1, "smc_attention_fwd_f32: bad arguments");
    if (head_dim != HD) {
        smc::set_error("smc_attention_fwd_f32: head_dim %d (only 64)", head_dim);
        return SMC_ERR_UNSUPPORTED;
    }
    return attn_fwd_launch(qkv, out, p_save, batch, tokens, heads, scale, smc::as_stream(stream));
}

SMC_API int smc_attention_causal_fwd_f32(const float* qkv, float* out, int batch, int tokens, int heads,
                                         int head_dim, float scale, void* stream) {
    SMC_CHECK(qkv && out && batch >= 1 && tokens >= 1 && heads >= 1, "smc_attention_causal_fwd_f32: bad arguments");
    if (head_dim != HD) {
        smc::set_error("smc_attention_causal_fwd_f32: head_dim %d (only 64)", head_dim);
        return SMC_ERR_UNSUPPORTED;
    }
    return attn_fwd_launch(qkv, out, nullptr, batch, tokens, heads, scale, smc::as_stream(stream), 1);
}

SMC_API int smc_attention_bwd_f32(const float* dout, const float* qkv, const float* p_save, float* dqkv, int batch,
                                  int tokens, int heads, int head_dim, float scale, void* stream) {
    SMC_CHECK(dout && qkv && p_save && dqkv && batch >= 1 && tokens >= 1 && heads >= 1,
              "smc_attention_bwd_f32: bad arguments");
    if (head_dim != HD) {
        smc::set_error("smc_attention_bwd_f32: head_dim %d (only 64)", head_dim);
        return SMC_ERR_UNSUPPORTED;
    }
    return attn_bwd_launch(dout, qkv, p_save, dqkv, batch, tokens, heads, scale, smc::as_stream(stream));
}

SMC_API int smc_patch_im2col_f32(const float* img, float* patches, int batch, int channels, int grid, int patch,
                                 int inverse, void* stream) {
    SMC_CHECK(img && patches && batch >= 1 && channels >= 1 && grid >= 1 && patch >= 1,
              "smc_patch_im2col_f32: bad arguments");
    const int64_t n = (int64_t)batch * channels * grid * patch * grid * patch;
    hipStream_t st = smc::as_stream(stream);
    if (inverse)
        hipLaunchKernelGGL(patch_perm_kernel, dim3(ew_blocks(n)), dim3(256), 0, st, patches, const_cast<float*>(img),
                           batch, channels, grid, patch, 0);
    else
        hipLaunchKernelGGL(patch_perm_kernel, dim3(ew_blocks(n)), dim3(256), 0, st, img, patches, batch, channels,
                           grid, patch, 1);
    return smc::check_launch("smc_patch_im2col_f32");
}

// =================================================================================== C ABI: executor

SMC_API int64_t smc_vit_packed_floats(const smc_vit_config* cfg) {
    if (vit_validate(cfg, 1) != SMC_OK) return -1;
    return layout(dims(*cfg), nullptr, nullptr);
}

SMC_API int smc_vit_pack_x3(const smc_vit_config* cfg, float* packed, void* stream) {
    SMC_TRY(vit_validate(cfg, 1));
    SMC_CHECK(packed, "smc_vit_pack_x3: null pointer");
    const VitDims d = dims(*cfg);
    SMC_CHECK(d.x3, "smc_vit_pack_x3: config has products = 0 (no planes region)");
    VitW w;
    layout(d, packed, &w);
    hipStream_t st = smc::as_stream(stream);
    auto planes = [&](const float* b, int K, int N, const short* out) {
        const int64_t total = (int64_t)K * N;
        hipLaunchKernelGGL(lin_x3_planes_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(total, 256), 8192)),
                           dim3(256), 0, st, b, N, K, N, const_cast<short*>(out));
    };
    const int D = d.D;
    planes(w.conv_wt, d.P, D, w.conv_wt3);
    planes(w.conv_w, D, d.P, w.conv_w3);
    for (int l = 0; l < d.NL; ++l) {
        const LayerW lw = layer_w(d, w, l);
        planes(lw.qkv_wt, D, 3 * D, lw.qkv_wt3);
        planes(lw.qkv_w, 3 * D, D, lw.qkv_w3);
        planes(lw.out_wt, D, D, lw.out_wt3);
        planes(lw.out_w, D, D, lw.out_w3);
        planes(lw.fc_wt, D, 4 * D, lw.fc_wt3);
        planes(lw.fc_w, 4 * D, D, lw.fc_w3);
        planes(lw.pr_wt, 4 * D, D, lw.pr_wt3);
        planes(lw.pr_w, D, 4 * D, lw.pr_w3);
    }
    planes(w.proj, D, d.E, w.proj3);
    planes(w.proj_t, d.E, D, w.proj_t3);
    return smc::check_launch("smc_vit_pack_x3");
}

SMC_API int64_t smc_vit_saved_floats(const smc_vit_config* cfg, int batch) {
    if (vit_validate(cfg, batch) != SMC_OK) return -1;
    return saved_layout(dims(*cfg), batch, nullptr, nullptr);
}

SMC_API int64_t smc_vit_workspace_bytes(const smc_vit_config* cfg, int batch) {
    if (vit_validate(cfg, batch) != SMC_OK) return -1;
    return ws_layout(dims(*cfg), batch, nullptr, nullptr) * (int64_t)sizeof(float);
}

SMC_API int smc_vit_forward_f32(const smc_vit_config* cfg, const float* packed, const float* image, int batch,
                                float* out, float* saved, float* workspace, int64_t workspace_bytes, void* stream) {
    SMC_TRY(vit_validate(cfg, batch));
    SMC_CHECK(packed && image && out && workspace, "smc_vit_forward_f32: null pointer");
    const VitDims d = dims(*cfg);
    const int B = batch, M = B * d.L, D = d.D, Mt = B * d.G * d.G;
    SMC_CHECK(workspace_bytes >= ws_layout(d, B, nullptr, nullptr) * (int64_t)sizeof(float),
              "smc_vit_forward_f32: workspace too small");
    hipStream_t st = smc::as_stream(stream);
    VitW w;
    layout(d, packed, &w);
    VitWs ws;
    ws_layout(d, B, workspace, &ws);
    VitS sv{};
    if (saved) saved_layout(d, B, saved, &sv);
    const float eps = cfg->ln_eps;
    int64_t cursor = 0;
    auto lin = [&](const float* a, int lda, const float* bw, int ldb, float* c, int ldc, int MM, int N, int K,
                   const smc_linear_epilogue& e, const short* bx3, const float* bt) {
        int* ctr = SMC_LIN_INLAUNCH ? ws.counters + cursor : nullptr;
        cursor += ws.counter_slice;
        if (cursor > ws.counter_ints) {
            smc::set_error("smc_vit: split-K counter slices exhausted");
            return SMC_ERR_INVALID;
        }
        return lin_launch(a, lda, bw, ldb, c, ldc, MM, N, K, &e, ws.split, ws.split_bytes, st, ctr, bx3, bt);
    };
    SMC_TRY_MEMSET(ws.counters, sizeof(int) * (size_t)ws.counter_ints, st, "smc_vit: counter memset");

    // patch embedding + class token + positional embedding, ln_pre
    SMC_TRY(smc_patch_im2col_f32(image, ws.patches, B, d.C, d.G, d.p, 0, stream));
    SMC_TRY(lin(ws.patches, d.P, w.conv_wt, D, ws.tok, D, Mt, D, d.P, epi_none(), w.conv_wt3, w.conv_w));
    float* x_pre = saved ? sv.x_pre : ws.xb;
    hipLaunchKernelGGL(embed_fwd_kernel, dim3(ew_blocks((int64_t)M * D)), dim3(256), 0, st, ws.tok, w.cls, w.pos,
                       x_pre, B, d.L, D);
    SMC_TRY(smc::check_launch("vit embed"));
    float* x = saved ? saved_layer(d, B, sv, 0).x_in : ws.xa;
    SMC_TRY(ln_fwd_launch(x_pre, D, w.lnpre_w, w.lnpre_b, x, D, saved ? sv.mu0 : nullptr, saved ? sv.rs0 : nullptr, M,
                          D, eps, st));

    const float scale = 1.f / sqrtf((float)HD);
    for (int l = 0; l < d.NL; ++l) {
        const LayerW lw = layer_w(d, w, l);
        LayerS ls{};
        if (saved) ls = saved_layer(d, B, sv, l);
        float* x_in = x;
        float* x_mid = saved ? ls.x_mid : (x_in == ws.xa ? ws.xb : ws.xa);
        float* x_out = saved ? (l + 1 < d.NL ? saved_layer(d, B, sv, l + 1).x_in : sv.x_out) : x_in;
        float* qkv = saved ? ls.qkv : ws.qkv;
        // attention block: x_mid = x_in + out_proj(attn(ln_1(x_in)))
        SMC_TRY(ln_fwd_launch(x_in, D, lw.ln1_w, lw.ln1_b, ws.h, D, saved ? ls.mu1 : nullptr,
                              saved ? ls.rs1 : nullptr, M, D, eps, st));
        smc_linear_epilogue e = epi_none();
        e.bias = lw.qkv_b;
        SMC_TRY(lin(ws.h, D, lw.qkv_wt, 3 * D, qkv, 3 * D, M, 3 * D, D, e, lw.qkv_wt3, lw.qkv_w));
        SMC_TRY(attn_fwd_launch(qkv, ws.o, saved ? ls.P : nullptr, B, d.L, d.H, scale, st));
        e = epi_none();
        e.bias = lw.out_b;
        e.residual = x_in;
        e.ld_res = D;
        SMC_TRY(lin(ws.o, D, lw.out_wt, D, x_mid, D, M, D, D, e, lw.out_wt3, lw.out_w));
        // MLP block: x_out = x_mid + c_proj(QuickGELU(c_fc(ln_2(x_mid))))
        SMC_TRY(ln_fwd_launch(x_mid, D, lw.ln2_w, lw.ln2_b, ws.h, D, saved ? ls.mu2 : nullptr,
                              saved ? ls.rs2 : nullptr, M, D, eps, st));
        e = epi_none();
        e.bias = lw.fc_b;
        e.act = SMC_LIN_ACT_QUICKGELU;
        e.pre_save = saved ? ls.G : nullptr;
        e.ld_pre = 4 * D;
        SMC_TRY(lin(ws.h, D, lw.fc_wt, 4 * D, ws.big, 4 * D, M, 4 * D, D, e, lw.fc_wt3, lw.fc_w));
        e = epi_none();
        e.bias = lw.pr_b;
        e.residual = x_mid;
        e.ld_res = D;
        SMC_TRY(lin(ws.big, 4 * D, lw.pr_wt, D, x_out, D, M, D, 4 * D, e, lw.pr_wt3, lw.pr_w));
        x = x_out;
    }
    // head: ln_post(x[:, 0]) @ proj   (CLS rows, stride L*D)
    SMC_TRY(ln_fwd_launch(x, (int64_t)d.L * D, w.lnpost_w, w.lnpost_b, ws.h, D, saved ? sv.mupost : nullptr,
                          saved ? sv.rspost : nullptr, B, D, eps, st));
    return lin(ws.h, D, w.proj, d.E, out, d.E, B, d.E, D, epi_none(), w.proj3, w.proj_t);
}

SMC_API int smc_vit_backward_f32(const smc_vit_config* cfg, const float* packed, const float* dout, int batch,
                                 int batch_run, const float* saved, float* dimage, float* workspace,
                                 int64_t workspace_bytes, void* stream) {
    SMC_TRY(vit_validate(cfg, batch));
    SMC_CHECK(packed && dout && saved && dimage && workspace, "smc_vit_backward_f32: null pointer");
    SMC_CHECK(batch_run >= 1 && batch_run <= batch, "smc_vit_backward_f32: batch_run %d not in [1, %d]", batch_run,
              batch);
    const VitDims d = dims(*cfg);
    // the saved activations are laid out for `batch` images; the leading `batch_run` of them are
    // differentiated (every per-image block of the layout is a prefix of its [batch * ...] tensor)
    const int B = batch_run, M = B * d.L, D = d.D, Mt = B * d.G * d.G;
    SMC_CHECK(workspace_bytes >= ws_layout(d, B, nullptr, nullptr) * (int64_t)sizeof(float),
              "smc_vit_backward_f32: workspace too small");
    hipStream_t st = smc::as_stream(stream);
    VitW w;
    layout(d, packed, &w);
    VitWs ws;
    ws_layout(d, B, workspace, &ws);
    VitS sv;
    saved_layout(d, batch, const_cast<float*>(saved), &sv);
    int64_t cursor = 0;
    auto lin = [&](const float* a, int lda, const float* bw, int ldb, float* c, int ldc, int MM, int N, int K,
                   const smc_linear_epilogue& e, const short* bx3, const float* bt) {
        int* ctr = SMC_LIN_INLAUNCH ? ws.counters + cursor : nullptr;
        cursor += ws.counter_slice;
        if (cursor > ws.counter_ints) {
            smc::set_error("smc_vit: split-K counter slices exhausted");
            return SMC_ERR_INVALID;
        }
        return lin_launch(a, lda, bw, ldb, c, ldc, MM, N, K, &e, ws.split, ws.split_bytes, st, ctr, bx3, bt);
    };
    int64_t toff = 0;
    auto snap = [&](const float* src, int64_t n) {
        if (SMC_VIT_TRACE) {
            hipLaunchKernelGGL(trace_copy_kernel, dim3(256), dim3(256), 0, st, src, ws.trace + toff, n);
            toff += n;
        }
    };
    SMC_TRY_MEMSET(ws.counters, sizeof(int) * (size_t)ws.counter_ints, st, "smc_vit: counter memset");

    // head: d(ln_post out) = dout @ proj^T, then ln_post backward into the CLS rows of a zeroed dx
    SMC_TRY(lin(dout, d.E, w.proj_t, D, ws.h, D, B, D, d.E, epi_none(), w.proj_t3, w.proj));
    SMC_TRY_MEMSET(ws.dx, sizeof(float) * (size_t)M * D, st, "smc_vit_backward_f32: memset");
    SMC_TRY(ln_bwd_launch(ws.h, D, sv.x_out, (int64_t)d.L * D, sv.mupost, sv.rspost, w.lnpost_w, nullptr, 0, ws.dx,
                          (int64_t)d.L * D, B, D, st));
    snap(ws.h, (int64_t)M * D);  // (the head's B rows; M * D keeps the snapshot sizes uniform)
    snap(ws.dx, (int64_t)M * D);

    const float scale = 1.f / sqrtf((float)HD);
    float* dx = ws.dx;  // gradient w.r.t. the current layer's output stream (updated in place)
    for (int l = d.NL - 1; l >= 0; --l) {
        const LayerW lw = layer_w(d, w, l);
        const LayerS ls = saved_layer(d, batch, sv, l);
        // MLP block
        smc_linear_epilogue e = epi_none();
        e.dact_pre = ls.G;
        e.ld_dact = 4 * D;
        SMC_TRY(lin(dx, D, lw.pr_w, 4 * D, ws.big, 4 * D, M, 4 * D, D, e, lw.pr_w3, lw.pr_wt));   // dG = (dx @ W_proj) * gelu'(G)
        snap(ws.big, (int64_t)M * 4 * D);
        SMC_TRY(lin(ws.big, 4 * D, lw.fc_w, D, ws.dh, D, M, D, 4 * D, epi_none(), lw.fc_w3, lw.fc_wt));  // dh2 = dG @ W_fc
        snap(ws.dh, (int64_t)M * D);
        SMC_TRY(ln_bwd_launch(ws.dh, D, ls.x_mid, D, ls.mu2, ls.rs2, lw.ln2_w, dx, D, dx, D, M, D, st));
        snap(dx, (int64_t)M * D);
        // attention block
        SMC_TRY(lin(dx, D, lw.out_w, D, ws.o, D, M, D, D, epi_none(), lw.out_w3, lw.out_wt));       // dO = dx_mid @ W_out
        snap(ws.o, (int64_t)M * D);
        SMC_TRY(attn_bwd_launch(ws.o, ls.qkv, ls.P, ws.qkv, B, d.L, d.H, scale, st));
        snap(ws.qkv, (int64_t)M * 3 * D);
        SMC_TRY(lin(ws.qkv, 3 * D, lw.qkv_w, D, ws.dh, D, M, D, 3 * D, epi_none(), lw.qkv_w3, lw.qkv_wt));  // dh1 = dqkv @ W_in
        snap(ws.dh, (int64_t)M * D);
        SMC_TRY(ln_bwd_launch(ws.dh, D, ls.x_in, D, ls.mu1, ls.rs1, lw.ln1_w, dx, D, dx, D, M, D, st));
        snap(dx, (int64_t)M * D);
    }
    // ln_pre backward, drop the class-token row, patch GEMM adjoint, col2im
    SMC_TRY(ln_bwd_launch(dx, D, sv.x_pre, D, sv.mu0, sv.rs0, w.lnpre_w, nullptr, 0, ws.dh, D, M, D, st));
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(ew_blocks((int64_t)Mt * D)), dim3(256), 0, st, ws.dh, ws.tok, B, d.L, D);
    SMC_TRY(smc::check_launch("vit embed bwd"));
    snap(ws.dh, (int64_t)M * D);
    snap(ws.tok, (int64_t)Mt * D);
    SMC_TRY(lin(ws.tok, D, w.conv_w, d.P, ws.patches, d.P, Mt, d.P, D, epi_none(), w.conv_w3, w.conv_wt));
    snap(ws.patches, (int64_t)Mt * d.P);
    return smc_patch_im2col_f32(dimage, ws.patches, B, d.C, d.G, d.p, 1, stream);
}
