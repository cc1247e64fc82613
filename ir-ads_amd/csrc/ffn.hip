// Swin FFN GEMMs with the GELU fused into their epilogues (mmcv FFN of swin.py:586-601:
// Linear(C, 4C) -> GELU(erf) -> Linear(4C, C)) for gfx950.
//
// The reference runs GELU as its own pass over the 4C-wide hidden tensor each way; here the two
// GEMMs that produce that tensor own it:
//   forward   irads_ffn_fc1_gelu:  u = bf16(X W1ᵀ + b1) and g = bf16(GELU(u)) written by the same
//             epilogue (u is kept for the backward, g feeds fc2);
//   backward  irads_ffn_fc2_dgrad_dgelu:  du = bf16(bf16(dF W2) * GELU'(u)), the fc2 input-gradient
//             GEMM's epilogue reading u (dF W2 is rounded to bf16 first, as the autocast GEMM's
//             output is, so the arithmetic is the unfused path's: elem_kernel<0> / <1> of
//             swinblock.hip, bit for bit given the same GEMM sums).
// One GEMM, C[M x N] = A[M x K] · B[N x K]ᵀ (both operands K-contiguous: X and W1 as stored, W2
// transposed once by the caller), bf16 in, fp32 accumulate:
//   * 128 x 128 workgroup tile, 4 waves of 64 x 64, MFMA v_mfma_f32_16x16x32_bf16 with the weight
//     rows as the MFMA A operand, so each lane ends with 4 consecutive N outputs of one row
//     (8-byte stores; 4 lanes fill 32 B of a row);
//   * A / B tiles of 64 k staged in LDS by LDS-DMA (global_load_lds_dwordx4: no staging
//     registers), two buffers, the next tile's DMA issued right after the barrier that retires
//     the previous reads; the 16-B chunks of a 128-B row XOR-swizzled by (row & 7), applied on
//     the global side, so the ds_read_b128 fragment reads spread over the banks;
//   * tiles of one M row-block (the same A rows) run on one XCD, which keeps A in its L2.
// Shapes: K % 64 == 0, N % 128 == 0 (every Swin-B/L stage: K = C in {128 .. 1536}, N = 4C);
// M is free (rows past M are clamped on load and masked on store).
#include "common.h"

namespace irads {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE = BM * BK;  // bf16 elements of one A (or B) tile

__device__ __forceinline__ f32x4 mfma16(const bf16x8_t &a, const bf16x8_t &b, const f32x4 &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// the erf GELU of swinblock.hip's element kernels (same expressions, same rounding)
__device__ __forceinline__ float gelu_erf(float x) { return x * 0.5f * (1.f + erff(x * 0.70710678118654752440f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
    const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752440f));
    const float pdf = expf(-0.5f * x * x) * 0.39894228040143267794f;
    return cdf + x * pdf;
}

// one 128 x 64 tile (rows r0.., k0..) of a K-contiguous matrix into LDS: wave w issues rows
// (4 w + i) * 8 .. + 8, lane L row + L / 8, LDS slot L % 8 <- global chunk (L % 8) ^ (row & 7)
__device__ __forceinline__ void stage_tile(const unsigned short *__restrict__ src, int ld, int r0, int rmax, int k0,
                                           unsigned short *dst, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rb = (4 * wave + i) * 8, row = rb + (lane >> 3);
        const int c = (lane & 7) ^ (row & 7);
        const int gr = min(r0 + row, rmax);
        const unsigned short *p = src + (long)gr * ld + k0 + c * 8;
        __builtin_amdgcn_global_load_lds((glb_void *)p, (lds_void *)(dst + rb * BK), 16, 0, 0);
    }
}

template <int EPI>  // 0: + bias, store u and GELU(u); 1: store bf16(acc) * GELU'(u)
__global__ void __launch_bounds__(256, 2) ffn_gemm_nt(const unsigned short *__restrict__ A,
                                                      const unsigned short *__restrict__ Bw,
                                                      const float *__restrict__ bias,
                                                      const unsigned short *__restrict__ U, unsigned short *__restrict__ out0,
                                                      unsigned short *__restrict__ out1, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) unsigned short smem[4 * TILE];  // [buf][A, B][128][64]
    const int nbn = N / BN;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);  // the N tiles of an M row-block on one XCD
    const int bm = lid / nbn, bn = lid - bm * nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int l16 = lane & 15, grp = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
    stage_tile(A, K, m0, M - 1, 0, smem, wave, lane);
    stage_tile(Bw, K, n0, N - 1, 0, smem + TILE, wave, lane);
    for (int kt = 0; kt < nk; ++kt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMAs of tile kt landed
        __syncthreads();  // ... everyone's; and every read of the other buffer (tile kt - 1) is done
        const unsigned short *As = smem + (kt & 1) * 2 * TILE, *Bs = As + TILE;
        if (kt + 1 < nk) {
            unsigned short *nxt = smem + ((kt + 1) & 1) * 2 * TILE;
            stage_tile(A, K, m0, M - 1, (kt + 1) * BK, nxt, wave, lane);
            stage_tile(Bw, K, n0, N - 1, (kt + 1) * BK, nxt + TILE, wave, lane);
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int ch = ks * 4 + grp;
            bf16x8_t af[4], bf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wm * 64 + i * 16 + l16;
                af[i] = *(const bf16x8_t *)(As + r * BK + ((ch ^ (r & 7)) * 8));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = wn * 64 + j * 16 + l16;
                bf[j] = *(const bf16x8_t *)(Bs + r * BK + ((ch ^ (r & 7)) * 8));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);  // Cᵀ tile: lane = row m
        }
    }
    // epilogue: lane holds C[m][n4 .. n4 + 3], m = m0 + wm 64 + 16 i + l16, n4 = n0 + wn 64 + 16 j + 4 grp
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n4 = n0 + wn * 64 + j * 16 + grp * 4;
        f32x4 b4 = {0.f, 0.f, 0.f, 0.f};
        if (EPI == 0) b4 = *(const f32x4 *)(bias + n4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + wm * 64 + i * 16 + l16;
            if (m >= M) continue;
            const long o = (long)m * N + n4;
            u16x4 w0, w1;
            if (EPI == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const unsigned short ub = f2bf(acc[i][j][r] + b4[r]);
                    w0[r] = ub;
                    w1[r] = f2bf(gelu_erf(bf2f(ub)));
                }
                *(u16x4 *)(out0 + o) = w0;
                *(u16x4 *)(out1 + o) = w1;
            } else {
                const u16x4 uu = *(const u16x4 *)(U + o);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float d = bf2f(f2bf(acc[i][j][r]));
                    w0[r] = f2bf(d * gelu_erf_grad(bf2f(uu[r])));
                }
                *(u16x4 *)(out0 + o) = w0;
            }
        }
    }
}

int check_shape(const char *what, int M, int N, int K) {
    IRADS_REQUIRE(M >= 0 && N > 0 && K > 0, "%s: bad sizes M=%d N=%d K=%d", what, M, N, K);
    IRADS_REQUIRE(K % BK == 0 && N % BN == 0, "%s: needs K %% 64 == 0 and N %% 128 == 0 (K=%d, N=%d)", what, K, N);
    IRADS_REQUIRE((long)((M + BM - 1) / BM) * (N / BN) < (1L << 31), "%s: grid too large", what);
    return IRADS_OK;
}

}  // namespace
}  // namespace irads

using namespace irads;

extern "C" int irads_ffn_fc1_gelu(const uint16_t *x, const uint16_t *w1, const float *b1, int M, int K, int N,
                                  uint16_t *u, uint16_t *g, void *stream) {
    if (int e = check_shape("irads_ffn_fc1_gelu", M, N, K)) return e;
    IRADS_REQUIRE(x && w1 && b1 && u && g, "irads_ffn_fc1_gelu: null pointer");
    IRADS_REQUIRE(((uintptr_t)x | (uintptr_t)w1 | (uintptr_t)b1 | (uintptr_t)u | (uintptr_t)g) % 16 == 0,
                  "irads_ffn_fc1_gelu: pointers must be 16-byte aligned");
    if (M == 0) return IRADS_OK;
    const unsigned nwg = (unsigned)(((M + BM - 1) / BM) * (N / BN));
    ffn_gemm_nt<0><<<nwg, 256, 0, (hipStream_t)stream>>>(x, w1, b1, nullptr, u, g, M, N, K);
    return check_launch("irads_ffn_fc1_gelu");
}

extern "C" int irads_ffn_fc2_dgrad_dgelu(const uint16_t *dy, const uint16_t *w2t, const uint16_t *u, int M, int K,
                                         int N, uint16_t *du, void *stream) {
    if (int e = check_shape("irads_ffn_fc2_dgrad_dgelu", M, N, K)) return e;
    IRADS_REQUIRE(dy && w2t && u && du, "irads_ffn_fc2_dgrad_dgelu: null pointer");
    IRADS_REQUIRE(((uintptr_t)dy | (uintptr_t)w2t | (uintptr_t)u | (uintptr_t)du) % 16 == 0,
                  "irads_ffn_fc2_dgrad_dgelu: pointers must be 16-byte aligned");
    if (M == 0) return IRADS_OK;
    const unsigned nwg = (unsigned)(((M + BM - 1) / BM) * (N / BN));
    ffn_gemm_nt<1><<<nwg, 256, 0, (hipStream_t)stream>>>(dy, w2t, nullptr, u, du, nullptr, M, N, K);
    return check_launch("irads_ffn_fc2_dgrad_dgelu");
}
