// Weight-gradient GEMM for the trainable Linears of the training step, gfx950.
//
//   D (m x n) fp32 = alpha * A^T B  (+ D if accumulate),   A (K x m), B (K x n) bf16 row-major
//   optionally colsum_A (m) / colsum_B (n) fp32 (the bias gradients), same alpha/accumulate
//
// In TRAIN_TYPE Adapter (optimizers.py:7-30) every trainable Linear — the 48 MAPA Adapters
// (swin.py:472-502), the MPG / DeformMPG fusion projections (swin.py:1045-1091), the
// SegFormer MLPs (segformer.py:11-18) — has a weight gradient of this shape: m, n = 8 ... 1024
// channels, K = tokens of the whole batch (up to 2^17).  A library GEMM tiles the m x n
// output and runs it on a handful of workgroups (8 x 128 output = one tile), so these were
// ~6 ms of the 60 ms step.  This kernel splits K instead:
//
//   * grid = output tiles x K-splits (~2048 workgroups); a workgroup streams its K-range once,
//     both operands staged through LDS, v_mfma_f32_16x16x32_bf16 accumulating in registers;
//   * both MFMA operands want 8 consecutive k per lane at a fixed column, i.e. the transpose
//     of the row-major HBM layout: tiles are stored in LDS as 16-column blocks of 32-byte rows
//     (each block a conflict-free [k][16] image) and read with ds_read_b64_tr_b16;
//   * the bias gradients (column sums) ride on the global loads: each thread owns a fixed
//     8-column group for the whole K-range, so the sums cost 8 adds per 16-byte load;
//   * per-split partials go to a workspace and a second kernel sums them in a fixed order:
//     deterministic, no atomics.
// The problem is HBM-bound (A and B are each read once: 2(m+n)K bytes for 2mnK flops).
#include <type_traits>

#include "common.h"

namespace irads {
namespace {

typedef unsigned short u16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

__device__ __forceinline__ u16x4 tr_read(const u16 *p) {
    return __builtin_bit_cast(u16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4 *)p));
}

constexpr int KS = 32;  // k per step = one 16x16x32 MFMA

// LDS image of a KS x T tile: block b (columns 16b..16b+15) is a [KS][16] row-major image,
// element (k, c) of the tile at b*KS*16 + k*16 + (c & 15).
template <int T> struct Tile {
    static constexpr int ELEMS = KS * T;
    static constexpr int LOADS = ELEMS / 8 / 256 > 0 ? ELEMS / 8 / 256 : 1;  // 16-B loads per thread
    static constexpr int THREADS = ELEMS / 8 < 256 ? ELEMS / 8 : 256;       // threads that load
};

template <int T>
__device__ __forceinline__ void load_tile(const u16 *__restrict__ g, long ld, int k0, int kend, int c0, int cols,
                                          u16x8 *reg, float *csum) {
    const int t = threadIdx.x;
#pragma unroll
    for (int s = 0; s < Tile<T>::LOADS; ++s) {
        const int e = (s * 256 + t) * 8;  // element index in the KS x T tile, row-major
        const int k = e / T, c = e % T;
        u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (t < Tile<T>::THREADS && k0 + k < kend && c0 + c < cols)
            v = *reinterpret_cast<const u16x8 *>(g + (long)(k0 + k) * ld + c0 + c);
        reg[s] = v;
        if (csum) {
#pragma unroll
            for (int j = 0; j < 8; ++j) csum[s * 8 + j] += bf2f(v[j]);
        }
    }
}

template <int T>
__device__ __forceinline__ void store_tile(u16 *lds, const u16x8 *reg) {
    const int t = threadIdx.x;
#pragma unroll
    for (int s = 0; s < Tile<T>::LOADS; ++s) {
        const int e = (s * 256 + t) * 8;
        const int k = e / T, c = e % T;
        if (t < Tile<T>::THREADS) *reinterpret_cast<u16x8 *>(lds + (c >> 4) * KS * 16 + k * 16 + (c & 15)) = reg[s];
    }
}

// operand fragment of 16-column block b: lane l = 16g + i gets column i, k slots
// {4g..4g+3, 16+4g..16+4g+3} (any k permutation works as long as A and B share it)
__device__ __forceinline__ bf16x8_t frag(const u16 *lds, int b, int lane) {
    const int g = lane >> 4, l16 = lane & 15;
    const u16 *p = lds + b * KS * 16 + (4 * g + (l16 >> 2)) * 16 + 4 * (l16 & 3);
    const u16x4 lo = tr_read(p), hi = tr_read(p + 16 * 16);
    return __builtin_bit_cast(bf16x8_t, u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

// TI x TJ output tile per workgroup, 4 waves as WI x WJ, each wave (TI/WI) x (TJ/WJ)
template <int TI, int TJ, int WI>
__global__ __launch_bounds__(256) void wgrad_partial_kernel(const u16 *__restrict__ A, long lda,
                                                            const u16 *__restrict__ B, long ldb, int K, int m,
                                                            int n, int chunk, int tiles_j, float *__restrict__ ws,
                                                            float *__restrict__ ws_sa, float *__restrict__ ws_sb) {
    constexpr int WJ = 4 / WI;
    constexpr int BI = TI / WI / 16, BJ = TJ / WJ / 16;  // MFMA blocks per wave
    __shared__ __attribute__((aligned(16))) u16 lA[KS * TI];
    __shared__ __attribute__((aligned(16))) u16 lB[KS * TJ];
    __shared__ float red[KS * (TI > TJ ? TI : TJ)];
    const int tile = blockIdx.x, split = blockIdx.y;
    const int ti = tile / tiles_j, tj = tile % tiles_j;
    const int i0 = ti * TI, j0 = tj * TJ;
    const int k0 = split * chunk, kend = min(K, k0 + chunk);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wi = wave / WJ, wj = wave % WJ;
    const bool sum_a = ws_sa != nullptr && tj == 0, sum_b = ws_sb != nullptr && ti == 0;
    constexpr int LA = Tile<TI>::LOADS, LB = Tile<TJ>::LOADS;
    float csa[LA * 8], csb[LB * 8];
#pragma unroll
    for (int j = 0; j < LA * 8; ++j) csa[j] = 0.f;
#pragma unroll
    for (int j = 0; j < LB * 8; ++j) csb[j] = 0.f;
    f32x4 acc[BI][BJ];
#pragma unroll
    for (int a = 0; a < BI; ++a)
#pragma unroll
        for (int b = 0; b < BJ; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    u16x8 ra[LA], rb[LB];
    load_tile<TI>(A, lda, k0, kend, i0, m, ra, sum_a ? csa : nullptr);
    load_tile<TJ>(B, ldb, k0, kend, j0, n, rb, sum_b ? csb : nullptr);
    for (int k = k0; k < kend; k += KS) {
        store_tile<TI>(lA, ra);
        store_tile<TJ>(lB, rb);
        __syncthreads();
        if (k + KS < kend) {  // prefetch the next step while this one computes
            load_tile<TI>(A, lda, k + KS, kend, i0, m, ra, sum_a ? csa : nullptr);
            load_tile<TJ>(B, ldb, k + KS, kend, j0, n, rb, sum_b ? csb : nullptr);
        }
        bf16x8_t fa[BI], fb[BJ];
#pragma unroll
        for (int a = 0; a < BI; ++a) fa[a] = frag(lA, wi * BI + a, lane);
#pragma unroll
        for (int b = 0; b < BJ; ++b) fb[b] = frag(lB, wj * BJ + b, lane);
#pragma unroll
        for (int a = 0; a < BI; ++a)
#pragma unroll
            for (int b = 0; b < BJ; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
        __syncthreads();
    }
    // partial tile -> workspace (split, m, n); lane owns column j = lane%16, rows 4(lane/16)..+3
    float *w = ws + (long)split * m * n;
#pragma unroll
    for (int a = 0; a < BI; ++a)
#pragma unroll
        for (int b = 0; b < BJ; ++b) {
            const int j = j0 + (wj * BJ + b) * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + (wi * BI + a) * 16 + 4 * (lane >> 4) + r;
                if (i < m && j < n) w[(long)i * n + j] = acc[a][b][r];
            }
        }
    // column sums: the KS threads sharing a column group (one per tile row) park their
    // partials in LDS; one thread per column adds them in row order (deterministic)
    auto colsum = [&](const float *cs, auto tag, int c0, int cols, float *out) {
        constexpr int T = decltype(tag)::value;
        __syncthreads();
#pragma unroll
        for (int s = 0; s < Tile<T>::LOADS; ++s) {
            const int e = (s * 256 + threadIdx.x) * 8;
            if (threadIdx.x < Tile<T>::THREADS)
#pragma unroll
                for (int j = 0; j < 8; ++j) red[e + j] = cs[s * 8 + j];  // e = row * T + col
        }
        __syncthreads();
        for (int c = threadIdx.x; c < T; c += 256) {
            float t = 0.f;
            for (int k = 0; k < KS; ++k) t += red[k * T + c];
            if (c0 + c < cols) out[c0 + c] = t;
        }
    };
    if (sum_a) colsum(csa, std::integral_constant<int, TI>{}, i0, m, ws_sa + (long)split * m);
    if (sum_b) colsum(csb, std::integral_constant<int, TJ>{}, j0, n, ws_sb + (long)split * n);
}

// sum the per-split partials: out[e] = alpha * sum_s ws[s][e] (+ out[e]), for the weight
// block and the two column-sum vectors in one launch (segments by blockIdx).  A workgroup
// owns 64 consecutive elements (coalesced across lanes); its 4 waves take the splits
// s = w, w+4, ... and are combined in wave order through LDS: a fixed summation order.
struct Seg {
    const float *ws;
    float *out;
    long count;
    int blocks, transpose;
};
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(Seg s0, Seg s1, Seg s2, int nsplit, float alpha,
                                                           int accumulate, int m, int n) {
    __shared__ float part[4][64];
    int blk = blockIdx.x;
    const Seg &sg = blk < s0.blocks ? s0 : (blk < s0.blocks + s1.blocks ? s1 : s2);
    blk -= blk < s0.blocks ? 0 : (blk < s0.blocks + s1.blocks ? s0.blocks : s0.blocks + s1.blocks);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long e = (long)blk * 64 + lane;
    const long count = sg.count;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (e < count) {
        int p = w;
        for (; p + 12 < nsplit; p += 16) {  // 4 independent loads in flight per lane
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] += sg.ws[(long)(p + 4 * u) * count + e];
        }
        for (; p < nsplit; p += 4) acc[0] += sg.ws[(long)p * count + e];
    }
    part[w][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    if (w == 0 && e < count) {
        float t = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
        t *= alpha;
        long o = e;
        if (sg.transpose) {  // element (i, j) of the m x n result stored at (j, i)
            const long i = e / n, j = e % n;
            o = j * m + i;
        }
        sg.out[o] = accumulate ? sg.out[o] + t : t;
    }
}

template <int TI, int TJ, int WI>
int launch_partial(const u16 *A, long lda, const u16 *B, long ldb, int K, int m, int n, int nsplit, int chunk,
                   float *ws, float *ws_sa, float *ws_sb, hipStream_t st) {
    const int tiles_i = (m + TI - 1) / TI, tiles_j = (n + TJ - 1) / TJ;
    dim3 grid(tiles_i * tiles_j, nsplit), block(256);
    hipLaunchKernelGGL((wgrad_partial_kernel<TI, TJ, WI>), grid, block, 0, st, A, lda, B, ldb, K, m, n, chunk, tiles_j,
                       ws, ws_sa, ws_sb);
    return check_launch("irads_wgrad partial");
}

}  // namespace
}  // namespace irads

using namespace irads;

extern "C" long irads_wgrad_workspace(int K, int m, int n) {
    // splits chosen below; workspace = nsplit * (m*n + m + n) floats
    const int TI = m <= 16 ? 16 : (m <= 32 ? 32 : (m <= 64 ? 64 : 128));
    const int TJ = 128;
    const long tiles = (long)((m + TI - 1) / TI) * ((n + TJ - 1) / TJ);
    long nsplit = (1024 + tiles - 1) / tiles;  // ~4 workgroups per CU
    const long maxsplit = (K + 63) / 64;      // >= 64 rows (2 MFMA steps) per workgroup
    if (nsplit > maxsplit) nsplit = maxsplit;
    if (nsplit < 1) nsplit = 1;
    return nsplit * ((long)m * n + m + n);
}

extern "C" int irads_wgrad(const uint16_t *A, long lda, const uint16_t *B, long ldb, int K, int m, int n, float alpha,
                           int accumulate, int transpose_out, float *D, float *colsum_a, float *colsum_b,
                           float *workspace, void *stream) {
    IRADS_REQUIRE(A && B && D && workspace, "irads_wgrad: null pointer");
    IRADS_REQUIRE(K >= 0 && m > 0 && n > 0 && m % 8 == 0 && n % 8 == 0,
                  "irads_wgrad: need m, n multiples of 8 (m=%d n=%d)", m, n);
    IRADS_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && lda >= m && ldb >= n &&
                      ((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0,
                  "irads_wgrad: rows must be 16-byte aligned (lda=%ld ldb=%ld)", lda, ldb);
    hipStream_t st = (hipStream_t)stream;
    const int TI = m <= 16 ? 16 : (m <= 32 ? 32 : (m <= 64 ? 64 : 128));
    const int TJ = 128;
    const long tiles = (long)((m + TI - 1) / TI) * ((n + TJ - 1) / TJ);
    long nsplit = (1024 + tiles - 1) / tiles;  // ~4 workgroups per CU
    const long maxsplit = (K + 63) / 64;      // >= 64 rows (2 MFMA steps) per workgroup
    if (nsplit > maxsplit) nsplit = maxsplit;
    if (nsplit < 1) nsplit = 1;
    long chunk = (K + nsplit - 1) / nsplit;
    chunk = (chunk + KS - 1) / KS * KS;
    nsplit = chunk > 0 ? (K + chunk - 1) / chunk : 1;
    if (nsplit < 1) nsplit = 1;
    if (chunk == 0) chunk = KS;
    float *ws = workspace;
    float *ws_sa = colsum_a ? ws + nsplit * (long)m * n : nullptr;
    float *ws_sb = colsum_b ? ws + nsplit * ((long)m * n + m) : nullptr;
    if (K == 0) {
        (void)hipMemsetAsync(ws, 0, sizeof(float) * nsplit * ((long)m * n + m + n), st);
    } else {
        int rc;
        if (TI == 16)
            rc = launch_partial<16, 128, 1>(A, lda, B, ldb, K, m, n, (int)nsplit, (int)chunk, ws, ws_sa, ws_sb, st);
        else if (TI == 32)
            rc = launch_partial<32, 128, 1>(A, lda, B, ldb, K, m, n, (int)nsplit, (int)chunk, ws, ws_sa, ws_sb, st);
        else if (TI == 64)
            rc = launch_partial<64, 128, 2>(A, lda, B, ldb, K, m, n, (int)nsplit, (int)chunk, ws, ws_sa, ws_sb, st);
        else
            rc = launch_partial<128, 128, 2>(A, lda, B, ldb, K, m, n, (int)nsplit, (int)chunk, ws, ws_sa, ws_sb, st);
        if (rc) return rc;
    }
    const long cnt = (long)m * n;
    Seg s0{ws, D, cnt, (int)((cnt + 63) / 64), transpose_out};
    Seg s1{ws_sa, colsum_a, m, colsum_a ? (m + 63) / 64 : 0, 0};
    Seg s2{ws_sb, colsum_b, n, colsum_b ? (n + 63) / 64 : 0, 0};
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(s0.blocks + s1.blocks + s2.blocks), dim3(256), 0, st, s0, s1, s2,
                       (int)nsplit, alpha, accumulate, m, n);
    return check_launch("irads_wgrad reduce");
}
