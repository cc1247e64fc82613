// bf16 GEMM for the frozen Swin trunk's projections, gfx950:  C[M x N] = A[M x K] · B[N x K]ᵀ (+ bias)
//
// Both operands K-contiguous (A = the activations, B = a PyTorch Linear weight (out, in) as stored,
// or its transpose made once for the backward's dX = dY·W, the trunk being frozen), bf16 in, fp32
// accumulate, bf16 out.  The FFN's erf GELU (mmcv FFN of swin.py:586-601) rides in the epilogue:
//   EPI_BIAS  C = bf16(acc + bias)                        (qkv / proj / fc2 forward, dX GEMMs)
//   EPI_GELU  U = bf16(acc + b1), G = bf16(GELU(U))       (fc1 forward: U kept for the backward)
//   EPI_DGELU C = bf16(bf16(acc) · GELU'(U))              (fc2 dgrad: dU without dG ever in HBM)
// with swinblock.hip's element formulas, so given the same accumulated value the outputs are bit for
// bit those of the unfused GEMM + irads_gelu_fwd / irads_gelu_bwd.
//
// Structure (cdna_hip_programming.md §5, "glds, 2 LDS buffers, BK=64"):
//   * 256 x 128 output tile per 8-wave workgroup, each wave 64 x 64 = 4 x 4 MFMA 16x16x32 blocks;
//     the MFMA's first operand is the B fragment, so every lane ends with 4 consecutive columns of
//     one row (8-byte stores);
//   * A and B tiles of 64 k reach LDS by global_load_lds_dwordx4 (1 KiB = 8 rows x 128 B per wave
//     instruction, no staging registers), the 16-B chunks of a row XOR-swizzled by (row & 7) on the
//     global side: every ds_read_b128 fragment read is bank-conflict free;
//   * two LDS buffers (96 KiB, ONE __shared__ array), the next k-step's loads issued right after the
//     barrier that retires the previous step's reads, so they fly under this step's 32 MFMAs per wave;
//   * tiles of one M row-band on one XCD (xcd_remap), so its A rows are read from HBM once.
// Shapes: K % 64 == 0, N % 128 == 0, lda / ldb / ldc multiples of 8; M free (rows past M clamped on
// load, masked on store).
#include "common.h"
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace irads {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 gbf16x8;
typedef __attribute__((ext_vector_type(8))) unsigned short gu16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short gu16x4;
typedef __attribute__((address_space(3))) void g_lds_void;
typedef __attribute__((address_space(1))) void g_glb_void;

constexpr int GBN = 128, GBK = 64;  // GBN: the column granule every tiling takes (N % 128 == 0)
enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_DGELU = 2 };

__device__ __forceinline__ float g_gelu(float x) { return x * 0.5f * (1.f + erf_f32(x * 0.70710678118654752440f)); }
__device__ __forceinline__ float g_gelu_grad(float x) {
    const float cdf = 0.5f * (1.f + erf_f32(x * 0.70710678118654752440f));
    const float pdf = __expf(-0.5f * x * x) * 0.39894228040143267794f;
    return cdf + x * pdf;
}

// R rows x 64 k of a K-contiguous matrix into the LDS image at dst (row r: 128 B, chunk c at slot
// c ^ (r & 7)).  Wave w fills 8-row pieces w, w + 8, ...: lane l -> row 8·piece + (l >> 3), LDS slot
// l & 7 (the wave-uniform base + 16·lane destination of global_load_lds) <- chunk (l & 7) ^ (row & 7).
// (NW waves: wave w fills pieces w, w + NW, ...)
template <int R, int NW>
__device__ __forceinline__ void g_stage(const unsigned short *__restrict__ src, long ld, int r0, int rmax, int k0,
                                        unsigned char *dst, int wave, int lane) {
    constexpr int PER_WAVE = R / (8 * NW);  // 8-row pieces per wave
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
        const int piece = i * NW + wave;
        const int row = piece * 8 + (lane >> 3);
        const int c = (lane & 7) ^ (row & 7);
        const int gr = min(r0 + row, rmax);
        __builtin_amdgcn_global_load_lds((g_glb_void *)(src + (long)gr * ld + k0 + c * 8),
                                         (g_lds_void *)(dst + piece * 1024), 16, 0, 0);
    }
}

// MFMA fragment of rows rb .. rb + 15, k-chunk c (8 k) of an LDS image: lane -> row rb + (lane & 15)
__device__ __forceinline__ gbf16x8 g_frag(const unsigned char *img, int rb, int c, int lane) {
    const int row = rb + (lane & 15);
    return *(const gbf16x8 *)(img + row * 128 + ((c ^ (row & 7)) << 4));
}

// GELU / GELU' by table in the 256 x 256 tiling's epilogues: for every bf16 U whose exponent field is
// in [kTabE0, kTabE0 + kTabNE) (|U| in [2^-23, 2^9)), bf16(GELU(U)) and the fp32 GELU'(U) are
// precomputed by gemm_gelu_table_kernel with the epilogue's own g_gelu / g_gelu_grad — so a lookup is
// bit for bit the formula — and staged in LDS beside the k-step buffers; other U (zero, tiny, huge,
// Inf / NaN) take the formula.  The erf formula cost ~20 (GELU) / ~27 (GELU') VALU instructions per
// element, at 2 waves per SIMD the longest phase of a 256 x 256 tile.
constexpr int kTabE0 = 104, kTabNE = 32, kTabN = 2 * kTabNE * 128;  // entries: sign x exponent x mantissa
__device__ __forceinline__ int gelu_tab_index(unsigned b, bool &in) {
    const int ex = (int)((b >> 7) & 0xFF) - kTabE0;
    in = (unsigned)ex < (unsigned)kTabNE;
    return (int)((b >> 15) << 12) | (ex << 7) | (int)(b & 0x7F);
}

__global__ void gemm_gelu_table_kernel(unsigned short *__restrict__ g, float *__restrict__ dg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kTabN) return;
    const unsigned b = ((unsigned)(i >> 12) << 15) | ((unsigned)(((i >> 7) & (kTabNE - 1)) + kTabE0) << 7) | (i & 0x7F);
    const float u = bf2f((unsigned short)b);
    g[i] = f2bf(g_gelu(u));
    dg[i] = g_gelu_grad(u);
}

// BMT x BNT tile on (BMT / WR) x (BNT / 64) waves, each WR x 64 (WR / 16 x 4 MFMA blocks)
template <int EPI, int NS, int BMT, int BNT, int WR, bool TR = false>
__global__ void __launch_bounds__((BMT / WR) * (BNT / 64) * 64) gemm_nt_bf16(const unsigned short *__restrict__ A, long lda,
                                                    const unsigned short *__restrict__ B, long ldb,
                                                    const float *__restrict__ bias,
                                                    const unsigned short *__restrict__ U, long ldu,
                                                    unsigned short *__restrict__ C0, unsigned short *__restrict__ C1,
                                                    long ldc, int M, int N, int K, long long *trace = nullptr,
                                                    const unsigned char *__restrict__ gtab = nullptr) {
    // TR: wave 0 of every workgroup logs wall_clock64() at entry, after each k-step's barrier, after the
    // main loop and at exit into trace[blockIdx.x * (K / 64 + 3) ...] (irads_gemm_nt_trace, A/B only)
    constexpr int NWN = BNT / 64, NW = (BMT / WR) * NWN, MI = WR / 16;
    constexpr int G_A_BYTES = BMT * GBK * 2, G_STAGE = G_A_BYTES + BNT * GBK * 2;
    long long *tr = TR ? trace + (long)blockIdx.x * (K / GBK + 3) : nullptr;
    if (TR && threadIdx.x == 0) tr[0] = wall_clock64();
    // !TR: `trace` is irads_stamp_next's region (or null): this workgroup's entry clock, written at its
    // exit (bench.py times the window-attention launch before this GEMM up to this GEMM's start)
    unsigned long long *stamp = TR ? nullptr : (unsigned long long *)trace;
    const unsigned long long t_entry = stamp_clock(stamp);
    // the GELU / GELU' table (256 x 256 tiles, gtab given): 16 KiB of bf16 GELU or 32 KiB of fp32 GELU'
    // after the k-step buffers, in the same array; copied by LDS-DMA, retired by the first k-step's wait
    constexpr bool TAB = EPI != EPI_BIAS && BMT == 256 && BNT == 256 && NS == 2 && !TR;
    constexpr int TAB_BYTES = !TAB ? 0 : EPI == EPI_GELU ? kTabN * 2 : kTabN * 4;
    __shared__ __attribute__((aligned(16))) unsigned char smem[NS * G_STAGE + TAB_BYTES];  // ONE array (glds wait trap)
    const bool use_tab = TAB && gtab != nullptr;
    if (use_tab) {
        const unsigned char *src = gtab + (EPI == EPI_GELU ? 0 : kTabN * 2);  // [kTabN bf16 GELU][kTabN fp32 GELU']
#pragma unroll
        for (int c0 = 0; c0 < TAB_BYTES / 16; c0 += NW * 64)
            __builtin_amdgcn_global_load_lds((g_glb_void *)(src + (c0 + (int)threadIdx.x) * 16),
                                             (g_lds_void *)(smem + NS * G_STAGE + (c0 + (int)(threadIdx.x & ~63)) * 16),
                                             16, 0, 0);
    }
    const int nbn = N / BNT;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);  // the N tiles of an M row-band on one XCD
    const int bm = lid / nbn, bn = lid - bm * nbn;
    const int m0 = bm * BMT, n0 = bn * BNT;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave / NWN, wn = wave % NWN;
    const int grp = lane >> 4;
    f32x4 acc[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / GBK;
    // the epilogue's bias columns, loaded now: their latency hides under the first stage's
    // (unconditionally, from B's first row when there is none — N·K·2 ≥ N·4 bytes — so no branch joins
    // on a loaded value and forces an early vmcnt wait; the select happens at the use)
    const bool hasb = EPI != EPI_DGELU && bias;
    const float *bsrc = hasb ? bias : (const float *)B;
    f32x4 bq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bq[j] = *(const f32x4 *)(bsrc + n0 + wn * 64 + j * 16 + grp * 4);
    // NS-buffer ring, NS - 1 k-steps in flight: step ks waits (counted vmcnt, G_LOADS global_load_lds per
    // wave and stage) for its own stage only, the barrier after it publishes every wave's DMA and retires
    // every read of buffer (ks - 1) % NS, which then takes stage ks + NS - 1.
    constexpr int G_LOADS = (BMT + BNT) / (8 * NW);
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) {
            g_stage<BMT, NW>(A, lda, m0, M - 1, s * GBK, smem + s * G_STAGE, wave, lane);
            g_stage<BNT, NW>(B, ldb, n0, N - 1, s * GBK, smem + s * G_STAGE + G_A_BYTES, wave, lane);
        }
    for (int ks = 0; ks < nk; ++ks) {
        if (NS == 3 && ks + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G_LOADS) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (TR && tid == 0) tr[1 + ks] = wall_clock64();
        const unsigned char *As = smem + (ks % NS) * G_STAGE, *Bs = As + G_A_BYTES;
        if (ks + NS - 1 < nk) {
            unsigned char *nx = smem + ((ks + NS - 1) % NS) * G_STAGE;
            g_stage<BMT, NW>(A, lda, m0, M - 1, (ks + NS - 1) * GBK, nx, wave, lane);
            g_stage<BNT, NW>(B, ldb, n0, N - 1, (ks + NS - 1) * GBK, nx + G_A_BYTES, wave, lane);
        }
        // 64 x 64 waves: all 16 fragment reads of the step up front (the second half's land under the
        // first half's MFMAs); 128 x 64 waves (128 accumulator registers) read one half at a time
        constexpr int KU = MI == 4 ? 2 : 1;
#pragma unroll
        for (int k0 = 0; k0 < 2; k0 += KU) {
            gbf16x8 af[KU][MI], bf[KU][4];
#pragma unroll
            for (int kk = 0; kk < KU; ++kk) {
#pragma unroll
                for (int j = 0; j < 4; ++j) bf[kk][j] = g_frag(Bs, wn * 64 + j * 16, (k0 + kk) * 4 + grp, lane);
#pragma unroll
                for (int i = 0; i < MI; ++i) af[kk][i] = g_frag(As, wm * WR + i * 16, (k0 + kk) * 4 + grp, lane);
            }
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int kk = 0; kk < KU; ++kk)
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[kk][j], af[kk][i], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
    }
    // Epilogue through LDS: the wave's 64 x 64 tile, rounded to bf16 in the MFMA layout (lane: row
    // 16 i + (lane & 15), columns 16 j + 4 grp .. + 3), goes to its own 8 KiB LDS region, then back as
    // whole 128-B rows (lane: 16 B of row 8 it + (lane >> 3)) for full-line global stores (and, for
    // EPI_DGELU, full-line loads of U).  Rows of the region: 128 B with 16-B chunk c at slot
    // c ^ (row & 7), so the row-wise reads are conflict free.
    // EPI_DGELU: this lane's 8 rows x 8 columns of U (the row-wise layout below), issued before the LDS
    // round trip so their latency hides under it (rows past M clamped: loaded, never stored).
    // (WR = 128: two 64-row halves through the same region, one after the other)
    const int lr = lane >> 3, lc = lane & 7;
    // every wave's last fragment reads of the main loop are done (consumed by its MFMAs); a raw barrier,
    // as __syncthreads() would also wait for the U loads in flight
    unsigned char *reg = smem + wave * 8192;
#pragma unroll
    for (int h = 0; h < WR / 64; ++h) {
        const int mh = m0 + wm * WR + h * 64;  // first row of this half
        gu16x8 uq[8];
        if (EPI == EPI_DGELU) {
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int m = min(mh + it * 8 + lr, M - 1);
                uq[it] = *(const gu16x8 *)(U + (long)m * ldu + n0 + wn * 64 + lc * 8);
            }
        }
        if (h == 0) {
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (TR && tid == 0) tr[1 + nk] = wall_clock64();
        } else {
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the previous half's row reads are done
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int nl = j * 16 + grp * 4;  // column within the wave tile
            const f32x4 b4 = hasb ? bq[j] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = i * 16 + (lane & 15);
                gu16x4 w;
#pragma unroll
                for (int r = 0; r < 4; ++r) w[r] = f2bf(acc[h * 4 + i][j][r] + b4[r]);  // EPI_DGELU: b4 = 0
                const int c = nl >> 3, half = (nl >> 2) & 1;  // 16-B chunk and its 8-B half
                *(gu16x4 *)(reg + row * 128 + ((c ^ (row & 7)) << 4) + half * 8) = w;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done (own region only)
        __builtin_amdgcn_wave_barrier();
        gu16x8 v[8];
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int row = it * 8 + lr;
            v[it] = *(const gu16x8 *)(reg + row * 128 + ((lc ^ (row & 7)) << 4));
        }
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int m = mh + it * 8 + lr;
            const long o = (long)m * ldc + n0 + wn * 64 + lc * 8;
            if (EPI == EPI_BIAS) {
                if (m < M) *(gu16x8 *)(C0 + o) = v[it];
            } else if (EPI == EPI_GELU) {
                gu16x8 g;
                int ti[8];
                bool all_in = use_tab;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    bool in = false;
                    ti[e] = gelu_tab_index(v[it][e], in);
                    all_in = all_in && in;
                }
                if (__builtin_amdgcn_ballot_w64(!all_in) == 0) {  // uniform: every lane's 8 values in the table
#pragma unroll
                    for (int e = 0; e < 8; ++e) g[e] = ((const unsigned short *)(smem + NS * G_STAGE))[ti[e]];
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) g[e] = f2bf(g_gelu(bf2f(v[it][e])));
                }
                if (m < M) {
                    *(gu16x8 *)(C0 + o) = v[it];
                    *(gu16x8 *)(C1 + o) = g;
                }
            } else {
                gu16x8 d;
                int ti[8];
                bool all_in = use_tab;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    bool in = false;
                    ti[e] = gelu_tab_index(uq[it][e], in);
                    all_in = all_in && in;
                }
                if (__builtin_amdgcn_ballot_w64(!all_in) == 0) {  // uniform: every lane's 8 values in the table
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        d[e] = f2bf(bf2f(v[it][e]) * ((const float *)(smem + NS * G_STAGE))[ti[e]]);
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) d[e] = f2bf(bf2f(v[it][e]) * g_gelu_grad(bf2f(uq[it][e])));
                }
                if (m < M) *(gu16x8 *)(C0 + o) = d;
            }
        }
    }
    if (TR) {
        __syncthreads();
        if (tid == 0) tr[2 + nk] = wall_clock64();
    }
    stamp_write(stamp, t_entry, false);
}

}  // namespace
}  // namespace irads

using namespace irads;

// variant: 0 = 256 x 128 tiles, 2 buffers; 1 = 256 x 128, 3 buffers (1 workgroup per CU either way);
// 2 = 128 x 128 tiles on 4 waves, 2 buffers (64 KiB: 2 workgroups per CU); 3 = 128 x 128, 3 buffers;
// 4 = 256 x 256 tiles on 8 waves of 128 x 64, 2 buffers (128 KiB; N % 256 == 0)
// The GELU / GELU' tables ([kTabN bf16][kTabN fp32]), built once on the device by the first call that
// is not inside a stream capture (stream-ordered, then a device sync, so every later stream sees them);
// null until then (the epilogues then evaluate the formula).  IRADS_GEMM_GELU_TABLE=0 keeps the formula.
const unsigned char *gelu_tables(hipStream_t st) {
    static unsigned char *tab = nullptr;
    static bool failed = false;
    static std::mutex mu;
    static const bool off = [] {
        const char *e = getenv("IRADS_GEMM_GELU_TABLE");
        return e && !strcmp(e, "0");
    }();
    if (off) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!tab && !failed) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
        unsigned char *p = nullptr;
        if (hipMalloc(&p, kTabN * 6) != hipSuccess) {
            (void)hipGetLastError();
            failed = true;
            return nullptr;
        }
        gemm_gelu_table_kernel<<<(kTabN + 255) / 256, 256, 0, st>>>((unsigned short *)p, (float *)(p + kTabN * 2));
        if (hipStreamSynchronize(st) != hipSuccess) {
            (void)hipGetLastError();
            failed = true;
            return nullptr;
        }
        tab = p;
    }
    return tab;
}

template <int EPI, int V, bool TR = false>
static void gemm_launch(const uint16_t *A, long lda, const uint16_t *B, long ldb, const float *bias, const uint16_t *U,
                        long ldu, uint16_t *C0, uint16_t *C1, long ldc, int M, int N, int K, long long *trace,
                        hipStream_t st) {
    constexpr int BMT = (V < 2 || V == 4) ? 256 : 128, NS = (V & 1) ? 3 : 2, BNT = V == 4 ? 256 : 128;
    constexpr int WR = V == 4 ? 128 : 64;
    const unsigned nwg = (unsigned)(((M + BMT - 1) / BMT) * (N / BNT));
    const unsigned char *tab = (V == 4 && EPI != EPI_BIAS && !TR) ? gelu_tables(st) : nullptr;
    gemm_nt_bf16<EPI, NS, BMT, BNT, WR, TR><<<nwg, (BMT / WR) * (BNT / 64) * 64, 0, st>>>(
        (const unsigned short *)A, lda, (const unsigned short *)B, ldb, bias, (const unsigned short *)U, ldu,
        (unsigned short *)C0, (unsigned short *)C1, ldc, M, N, K, trace, tab);
}

template <int EPI>
static void gemm_dispatch(int variant, const uint16_t *A, long lda, const uint16_t *B, long ldb, const float *bias,
                          const uint16_t *U, long ldu, uint16_t *C0, uint16_t *C1, long ldc, int M, int N, int K,
                          long long *stamp, hipStream_t st) {
    switch (variant) {
    case 0: gemm_launch<EPI, 0>(A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stamp, st); break;
    case 1: gemm_launch<EPI, 1>(A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stamp, st); break;
    case 2: gemm_launch<EPI, 2>(A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stamp, st); break;
    case 3: gemm_launch<EPI, 3>(A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stamp, st); break;
    default: gemm_launch<EPI, 4>(A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stamp, st); break;
    }
}

extern "C" int irads_gemm_nt_variant(int variant, int epilogue, const uint16_t *A, long lda, const uint16_t *B,
                                     long ldb, const float *bias, const uint16_t *U, long ldu, uint16_t *C0,
                                     uint16_t *C1, long ldc, int M, int N, int K, void *stream) {
    long long *stamp = (long long *)take_stamp();  // irads_stamp_next's region for this launch, or null
    IRADS_REQUIRE(epilogue >= 0 && epilogue <= 2, "irads_gemm_nt: epilogue %d", epilogue);
    IRADS_REQUIRE(variant >= 0 && variant <= 4, "irads_gemm_nt: variant %d", variant);
    IRADS_REQUIRE(variant != 4 || N % 256 == 0, "irads_gemm_nt: the 256 x 256 tiling needs N %% 256 == 0 (N=%d)", N);
    IRADS_REQUIRE(M >= 0 && N > 0 && K > 0 && N % GBN == 0 && K % GBK == 0,
                  "irads_gemm_nt: needs N %% 128 == 0 and K %% 64 == 0 (M=%d N=%d K=%d)", M, N, K);
    IRADS_REQUIRE(A && B && C0 && (epilogue != 1 || C1) && (epilogue != 2 || U), "irads_gemm_nt: null pointer");
    IRADS_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 && (epilogue != 2 || ldu % 8 == 0) && lda >= K &&
                      ldb >= K && ldc >= N,
                  "irads_gemm_nt: leading dimensions must be multiples of 8 and cover the rows");
    IRADS_REQUIRE(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C0 | (uintptr_t)C1 | (uintptr_t)U | (uintptr_t)bias) % 16 == 0,
                  "irads_gemm_nt: pointers must be 16-byte aligned");
    IRADS_REQUIRE((long)((M + 127) / 128) * (N / GBN) < (1L << 31), "irads_gemm_nt: grid too large");
    if (M == 0) return IRADS_OK;
    hipStream_t st = (hipStream_t)stream;
    if (epilogue == EPI_BIAS)
        gemm_dispatch<EPI_BIAS>(variant, A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stamp, st);
    else if (epilogue == EPI_GELU)
        gemm_dispatch<EPI_GELU>(variant, A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stamp, st);
    else
        gemm_dispatch<EPI_DGELU>(variant, A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stamp, st);
    return check_launch("irads_gemm_nt");
}

extern "C" int irads_gemm_nt(int epilogue, const uint16_t *A, long lda, const uint16_t *B, long ldb, const float *bias,
                             const uint16_t *U, long ldu, uint16_t *C0, uint16_t *C1, long ldc, int M, int N, int K,
                             void *stream) {
    return irads_gemm_nt_variant(2, epilogue, A, lda, B, ldb, bias, U, ldu, C0, C1, ldc, M, N, K, stream);
}

extern "C" int irads_gemm_nt_trace(int variant, const uint16_t *A, long lda, const uint16_t *B, long ldb,
                                   const float *bias, uint16_t *C0, long ldc, int M, int N, int K, long long *trace,
                                   void *stream) {
    IRADS_REQUIRE(M > 0 && N > 0 && K > 0 && N % GBN == 0 && K % GBK == 0 && trace && variant >= 0 && variant <= 4 &&
                      (variant != 4 || N % 256 == 0),
                  "irads_gemm_nt_trace: shape / variant");
    hipStream_t st = (hipStream_t)stream;
    switch (variant) {
    case 0: gemm_launch<EPI_BIAS, 0, true>(A, lda, B, ldb, bias, nullptr, 0, C0, nullptr, ldc, M, N, K, trace, st); break;
    case 1: gemm_launch<EPI_BIAS, 1, true>(A, lda, B, ldb, bias, nullptr, 0, C0, nullptr, ldc, M, N, K, trace, st); break;
    case 2: gemm_launch<EPI_BIAS, 2, true>(A, lda, B, ldb, bias, nullptr, 0, C0, nullptr, ldc, M, N, K, trace, st); break;
    case 3: gemm_launch<EPI_BIAS, 3, true>(A, lda, B, ldb, bias, nullptr, 0, C0, nullptr, ldc, M, N, K, trace, st); break;
    default: gemm_launch<EPI_BIAS, 4, true>(A, lda, B, ldb, bias, nullptr, 0, C0, nullptr, ldc, M, N, K, trace, st); break;
    }
    return check_launch("irads_gemm_nt_trace");
}
