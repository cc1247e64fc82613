// Row and element kernels of the fused Swin block (SwinBlockAdapter, reference
// semseg/models/backbones/swin.py:505-610 around ShiftWindowMSA :180-254 and mmcv FFN),
// gfx950.
//
// Under bf16 autocast the reference block is
//     X1   = X + DropPath(proj(attn(qkv(LN1(X)))))                       (fp32 residual)
//     Xout = (X1 + DropPath(fc2(GELU(fc1(LN2(X1)))))) + 0.5 * Adapter(X1)
// with the Linears in bf16 and LayerNorm / the residual stream in fp32.  Run op by op,
// that is ~25 separate launches per block each way (LN, casts fp32<->bf16, DropPath
// div/mul, adds, GELU, ReLU/dropout, gradient accumulation), every one a full pass
// over an (M, C) tensor in HBM.  Here the non-GEMM work between two GEMMs is ONE pass:
//
//   resln_fwd  : x (+ DropPath(a1)) (+ mult * a2)  ->  fp32 residual out, bf16 copy,
//                LayerNorm -> bf16 GEMM operand (+ mean / rstd for the backward)
//   resln_bwd  : g_res + g_add + LayerNorm-backward(dy)  ->  fp32 residual grad, and the
//                bf16 GEMM operands of the two branches that forked off the residual
//                (DropPath-backward, 0.5 * for the adapter)
//   gelu_fwd / gelu_bwd, relu_dropout_fwd / relu_dropout_bwd : bf16 element passes
//
// One wave64 per row for the row kernels (C = 64 * VPT, VPT in {2,3,4,6,8,12,16,24,32,48}
// covers Swin-B and Swin-L, including the 4C rows of PatchMerging), the row held in registers: reductions are wave shuffles, and
// every tensor is touched exactly once.  All kernels are HBM-bound streaming passes.
//
// Rounding follows the autocast reference op by op: DropPath on a bf16 branch is
// bf16(v * (1/keep)) * mask (torch's GPU div-by-scalar is a multiply by the fp32
// reciprocal), the residual add is fp32, the adapter term is bf16(0.5 * d), GELU is the
// exact erf form computed in fp32 and rounded to bf16, dropout keeps with probability
// 1-p and scales by 1/(1-p).
#include "common.h"

namespace irads {
namespace {

typedef unsigned short u16;

// ------------------------------------------------------------------ vector helpers
template <int VW> struct VecF;
template <> struct VecF<1> {
    static __device__ __forceinline__ void ld(const float *p, float *v) { v[0] = p[0]; }
    static __device__ __forceinline__ void st(float *p, const float *v) { p[0] = v[0]; }
};
template <> struct VecF<2> {
    static __device__ __forceinline__ void ld(const float *p, float *v) {
        float2 t = *reinterpret_cast<const float2 *>(p);
        v[0] = t.x, v[1] = t.y;
    }
    static __device__ __forceinline__ void st(float *p, const float *v) {
        *reinterpret_cast<float2 *>(p) = make_float2(v[0], v[1]);
    }
};
template <> struct VecF<4> {
    static __device__ __forceinline__ void ld(const float *p, float *v) {
        float4 t = *reinterpret_cast<const float4 *>(p);
        v[0] = t.x, v[1] = t.y, v[2] = t.z, v[3] = t.w;
    }
    static __device__ __forceinline__ void st(float *p, const float *v) {
        *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
};
template <int VW> struct VecB;
template <> struct VecB<1> {
    static __device__ __forceinline__ void ld(const u16 *p, float *v) { v[0] = bf2f(p[0]); }
    static __device__ __forceinline__ void st(u16 *p, const float *v) { p[0] = f2bf(v[0]); }
};
template <> struct VecB<2> {
    static __device__ __forceinline__ void ld(const u16 *p, float *v) {
        unsigned t = *reinterpret_cast<const unsigned *>(p);
        v[0] = __uint_as_float(t << 16), v[1] = __uint_as_float(t & 0xffff0000u);
    }
    static __device__ __forceinline__ void st(u16 *p, const float *v) {
        *reinterpret_cast<unsigned *>(p) = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
    }
};
template <> struct VecB<4> {
    static __device__ __forceinline__ void ld(const u16 *p, float *v) {
        uint2 t = *reinterpret_cast<const uint2 *>(p);
        v[0] = __uint_as_float(t.x << 16), v[1] = __uint_as_float(t.x & 0xffff0000u);
        v[2] = __uint_as_float(t.y << 16), v[3] = __uint_as_float(t.y & 0xffff0000u);
    }
    static __device__ __forceinline__ void st(u16 *p, const float *v) {
        uint2 t;
        t.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
        t.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2 *>(p) = t;
    }
};

__device__ __forceinline__ float round_bf(float v) { return bf2f(f2bf(v)); }

// DropPath on a bf16 branch value (common.py DropPath: x.div(keep) * mask), per-sample
// factor s = mask ? fp32(1/keep) : 0; no factor array = identity.
__device__ __forceinline__ float droppath(float v, bool has, float s) {
    if (!has) return v;
    return s == 0.f ? 0.f : round_bf(v * s);
}

constexpr int kRowsPerBlock = 4;  // one wave64 per row, 256 threads

// ------------------------------------------------------------------ forward row kernel
template <int VPT, bool A1, bool A2, bool LN, bool XOUT, bool XB>
__global__ __launch_bounds__(256) void resln_fwd_kernel(const float *__restrict__ x, const u16 *__restrict__ a1,
                                                        const float *__restrict__ a1s, const u16 *__restrict__ a2,
                                                        float a2m, int M, int rps, const float *__restrict__ gamma,
                                                        const float *__restrict__ beta, float eps,
                                                        float *__restrict__ xo, u16 *__restrict__ lo,
                                                        u16 *__restrict__ xbo, float *__restrict__ mean_o,
                                                        float *__restrict__ rstd_o) {
    constexpr int VW = (VPT % 4 == 0) ? 4 : (VPT % 2 == 0 ? 2 : 1);
    constexpr int NCH = VPT / VW;
    constexpr int C = VPT * 64;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
    if (row >= M) return;
    const long base = (long)row * C;
    float v[VPT];
#pragma unroll
    for (int k = 0; k < NCH; ++k) VecF<VW>::ld(x + base + (k * 64 + lane) * VW, v + k * VW);
    if (A1) {
        const bool has = a1s != nullptr;
        const float s = has ? a1s[row / rps] : 1.f;
        float t[VPT];
#pragma unroll
        for (int k = 0; k < NCH; ++k) VecB<VW>::ld(a1 + base + (k * 64 + lane) * VW, t + k * VW);
#pragma unroll
        for (int j = 0; j < VPT; ++j) v[j] += droppath(t[j], has, s);
    }
    if (A2) {
        float t[VPT];
#pragma unroll
        for (int k = 0; k < NCH; ++k) VecB<VW>::ld(a2 + base + (k * 64 + lane) * VW, t + k * VW);
#pragma unroll
        for (int j = 0; j < VPT; ++j) v[j] += round_bf(t[j] * a2m);
    }
    if (XOUT) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) VecF<VW>::st(xo + base + (k * 64 + lane) * VW, v + k * VW);
    }
    if (XB) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) VecB<VW>::st(xbo + base + (k * 64 + lane) * VW, v + k * VW);
    }
    if (LN) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < VPT; ++j) s += v[j];
        const float mu = wave_sum(s) * (1.f / C);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
            const float d = v[j] - mu;
            q += d * d;
        }
        const float rs = rsqrtf(wave_sum(q) * (1.f / C) + eps);
        float y[VPT];
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
#pragma unroll
            for (int e = 0; e < VW; ++e) {
                const int c = (k * 64 + lane) * VW + e;
                y[k * VW + e] = gamma[c] * (rs * (v[k * VW + e] - mu)) + beta[c];
            }
            VecB<VW>::st(lo + base + (k * 64 + lane) * VW, y + k * VW);
        }
        if (lane == 0) {
            mean_o[row] = mu;
            rstd_o[row] = rs;
        }
    }
}

// ------------------------------------------------------------------ backward row kernel
template <int VPT, bool LN, bool GRES, bool GADD, bool DXOUT, bool B1, bool B2>
__global__ __launch_bounds__(256) void resln_bwd_kernel(const u16 *__restrict__ dy, const float *__restrict__ x,
                                                        const float *__restrict__ mean, const float *__restrict__ rstd,
                                                        const float *__restrict__ gamma, const float *__restrict__ gres,
                                                        const u16 *__restrict__ gadd, int M, int rps,
                                                        float *__restrict__ dxo, u16 *__restrict__ b1o,
                                                        const float *__restrict__ b1s, u16 *__restrict__ b2o,
                                                        float b2m) {
    constexpr int VW = (VPT % 4 == 0) ? 4 : (VPT % 2 == 0 ? 2 : 1);
    constexpr int NCH = VPT / VW;
    constexpr int C = VPT * 64;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
    if (row >= M) return;
    const long base = (long)row * C;
    float dx[VPT];
#pragma unroll
    for (int j = 0; j < VPT; ++j) dx[j] = 0.f;
    if (LN) {
        float g[VPT], xv[VPT];
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            VecB<VW>::ld(dy + base + (k * 64 + lane) * VW, g + k * VW);
            VecF<VW>::ld(x + base + (k * 64 + lane) * VW, xv + k * VW);
        }
        const float mu = mean[row], rs = rstd[row];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
#pragma unroll
            for (int e = 0; e < VW; ++e) {
                const int j = k * VW + e;
                const int c = (k * 64 + lane) * VW + e;
                g[j] *= gamma[c];              // d xhat
                xv[j] = (xv[j] - mu) * rs;     // xhat
                s1 += g[j];
                s2 += g[j] * xv[j];
            }
        }
        const float m1 = wave_sum(s1) * (1.f / C), m2 = wave_sum(s2) * (1.f / C);
#pragma unroll
        for (int j = 0; j < VPT; ++j) dx[j] = rs * (g[j] - m1 - xv[j] * m2);
    }
    if (GRES) {
        float t[VPT];
#pragma unroll
        for (int k = 0; k < NCH; ++k) VecF<VW>::ld(gres + base + (k * 64 + lane) * VW, t + k * VW);
#pragma unroll
        for (int j = 0; j < VPT; ++j) dx[j] += t[j];
    }
    if (GADD) {
        float t[VPT];
#pragma unroll
        for (int k = 0; k < NCH; ++k) VecB<VW>::ld(gadd + base + (k * 64 + lane) * VW, t + k * VW);
#pragma unroll
        for (int j = 0; j < VPT; ++j) dx[j] += t[j];
    }
    if (DXOUT) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) VecF<VW>::st(dxo + base + (k * 64 + lane) * VW, dx + k * VW);
    }
    if (B1 || B2) {
        float gb[VPT];
#pragma unroll
        for (int j = 0; j < VPT; ++j) gb[j] = round_bf(dx[j]);  // grad cast to the bf16 branch
        if (B1) {
            const bool has = b1s != nullptr;
            const float s = has ? b1s[row / rps] : 1.f;
            float t[VPT];
#pragma unroll
            for (int j = 0; j < VPT; ++j) t[j] = droppath(gb[j], has, s);
#pragma unroll
            for (int k = 0; k < NCH; ++k) VecB<VW>::st(b1o + base + (k * 64 + lane) * VW, t + k * VW);
        }
        if (B2) {
            float t[VPT];
#pragma unroll
            for (int j = 0; j < VPT; ++j) t[j] = gb[j] * b2m;
#pragma unroll
            for (int k = 0; k < NCH; ++k) VecB<VW>::st(b2o + base + (k * 64 + lane) * VW, t + k * VW);
        }
    }
}

// ------------------------------------------------------------------ element kernels
// 8 bf16 per thread (16-byte accesses); the tail is handled element-wise.
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ void unpack8(u32x4 w, float *f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
__device__ __forceinline__ u32x4 pack8(const float *f) {
    u32x4 w;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (unsigned)f2bf(f[2 * i]) | ((unsigned)f2bf(f[2 * i + 1]) << 16);
    return w;
}

__device__ __forceinline__ float gelu_f(float x) { return x * 0.5f * (1.f + erf_f32(x * 0.70710678118654752440f)); }
__device__ __forceinline__ float gelu_grad(float x) {
    const float cdf = 0.5f * (1.f + erf_f32(x * 0.70710678118654752440f));
    const float pdf = __expf(-0.5f * x * x) * 0.39894228040143267794f;
    return cdf + x * pdf;
}

template <int OP>  // 0 gelu fwd, 1 gelu bwd, 2 relu+dropout fwd, 3 relu+dropout bwd
__global__ __launch_bounds__(256) void elem_kernel(const u16 *__restrict__ a, const u16 *__restrict__ b,
                                                   u16 *__restrict__ out, long n, float p, float scale,
                                                   unsigned long long salt,
                                                   const unsigned long long *__restrict__ seed_dev) {
    const long i8 = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
    if (i8 >= n) return;
    // the draw's seed lives in device memory (written by the torch generator on the same
    // stream), so a captured HIP graph draws a fresh mask on every replay
    const unsigned long long seed = (OP == 2 && seed_dev != nullptr) ? (*seed_dev ^ salt) : salt;
    auto f = [&](float av, float bv, long i) -> float {
        if (OP == 0) return gelu_f(av);
        if (OP == 1) return bv * gelu_grad(av);
        if (OP == 2) {
            const float r = av > 0.f ? av : 0.f;
            if (p <= 0.f) return r;
            return uniform01(seed, (unsigned long long)i) >= p ? r * scale : 0.f;
        }
        return av > 0.f ? bv * scale : 0.f;  // a = saved dropout output, b = grad
    };
    if (i8 + 8 <= n) {
        float av[8], bv[8], o[8];
        unpack8(*reinterpret_cast<const u32x4 *>(a + i8), av);
        if (OP == 1 || OP == 3) unpack8(*reinterpret_cast<const u32x4 *>(b + i8), bv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f(av[e], (OP == 1 || OP == 3) ? bv[e] : 0.f, i8 + e);
        *reinterpret_cast<u32x4 *>(out + i8) = pack8(o);
    } else {
        for (long i = i8; i < n; ++i) out[i] = f2bf(f(bf2f(a[i]), (OP == 1 || OP == 3) ? bf2f(b[i]) : 0.f, i));
    }
}

// ------------------------------------------------------------------ dispatch
template <int VPT>
int resln_fwd_vpt(const float *x, const u16 *a1, const float *a1s, const u16 *a2, float a2m, int M, int rps,
                  const float *gamma, const float *beta, float eps, float *xo, u16 *lo, u16 *xbo, float *mean,
                  float *rstd, hipStream_t st) {
    dim3 grid((M + kRowsPerBlock - 1) / kRowsPerBlock), block(256);
    const bool ln = gamma != nullptr;
#define IRADS_RESLN_F(A1_, A2_, LN_, XO_, XB_)                                                             \
    if ((a1 != nullptr) == A1_ && (a2 != nullptr) == A2_ && ln == LN_ && (xo != nullptr) == XO_ &&           \
        (xbo != nullptr) == XB_) {                                                                          \
        hipLaunchKernelGGL((resln_fwd_kernel<VPT, A1_, A2_, LN_, XO_, XB_>), grid, block, 0, st, x, a1, a1s, a2, \
                           a2m, M, rps, gamma, beta, eps, xo, lo, xbo, mean, rstd);                         \
        return check_launch("irads_resln_fwd");                                                             \
    }
    // the combinations the block sequence uses
    IRADS_RESLN_F(false, false, true, false, false)  // first LN1 of a stage
    IRADS_RESLN_F(true, false, true, true, true)     // X1 = X + dp(o); LN2; bf16(X1)
    IRADS_RESLN_F(true, true, true, true, false)     // Xout = X1 + dp(f) + 0.5 d; next LN1
    IRADS_RESLN_F(true, true, false, true, false)    // last block of a stage
    IRADS_RESLN_F(false, false, true, false, true)
    IRADS_RESLN_F(true, false, true, true, false)
    IRADS_RESLN_F(true, false, false, true, false)
#undef IRADS_RESLN_F
    set_error("irads_resln_fwd: unsupported combination of optional tensors");
    return IRADS_EINVAL;
}

template <int VPT>
int resln_bwd_vpt(const u16 *dy, const float *x, const float *mean, const float *rstd, const float *gamma,
                  const float *gres, const u16 *gadd, int M, int rps, float *dxo, u16 *b1o, const float *b1s,
                  u16 *b2o, float b2m, hipStream_t st) {
    dim3 grid((M + kRowsPerBlock - 1) / kRowsPerBlock), block(256);
    const bool ln = dy != nullptr;
#define IRADS_RESLN_B(LN_, GR_, GA_, DX_, B1_, B2_)                                                           \
    if (ln == LN_ && (gres != nullptr) == GR_ && (gadd != nullptr) == GA_ && (dxo != nullptr) == DX_ &&        \
        (b1o != nullptr) == B1_ && (b2o != nullptr) == B2_) {                                                 \
        hipLaunchKernelGGL((resln_bwd_kernel<VPT, LN_, GR_, GA_, DX_, B1_, B2_>), grid, block, 0, st, dy, x, mean, \
                           rstd, gamma, gres, gadd, M, rps, dxo, b1o, b1s, b2o, b2m);                          \
        return check_launch("irads_resln_bwd");                                                               \
    }
    IRADS_RESLN_B(false, true, false, false, true, true)  // block output grad -> ffn / adapter operands
    IRADS_RESLN_B(true, true, true, true, true, false)    // dX1 = g + g_adapter + LN2'(dy); d(o) operand
    IRADS_RESLN_B(true, true, false, true, true, true)    // dX = dX1 + LN1'(dy); previous block's operands
    IRADS_RESLN_B(true, true, false, true, false, false)  // first block: dX only
    IRADS_RESLN_B(true, false, false, true, false, false)
    IRADS_RESLN_B(true, true, true, true, false, false)
    IRADS_RESLN_B(true, true, true, true, true, true)
#undef IRADS_RESLN_B
    set_error("irads_resln_bwd: unsupported combination of optional tensors");
    return IRADS_EINVAL;
}

// DropPath factors of a whole stage in one launch (semseg/models/layers/common.py DropPath in bf16 under
// autocast: x.div(keep) * floor(keep + U), U ~ torch.rand in bf16 — 8 random bits, multiples of 2^-8):
// out[slot][s] = floor(bf16(keep[slot] + U)) * inv[slot] for an active slot (keep < 1), 1 otherwise.
// U is drawn from the stage's device seed (the Adapter dropout's, ^ salt), so a captured graph draws
// fresh factors on every replay; the keep + U sum is formed in fp64 and rounded fp32 -> bf16 like
// torch's (u.double() + keep).to(bfloat16).
__global__ __launch_bounds__(256) void droppath_kernel(const unsigned long long *__restrict__ seed_dev,
                                                       unsigned long long salt, const double *__restrict__ keep,
                                                       const float *__restrict__ inv, int n_slots, int S,
                                                       float *__restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_slots * S) return;
    const int slot = i / S;
    const double k = keep[slot];
    if (!(k < 1.0)) {
        out[i] = 1.f;
        return;
    }
    const float u = floorf(uniform01(*seed_dev ^ salt, (unsigned long long)i) * 256.f) * (1.f / 256.f);
    const float t = bf2f(f2bf((float)((double)u + k)));
    out[i] = floorf(t) * inv[slot];
}

}  // namespace
}  // namespace irads

using namespace irads;

#define IRADS_VPT_SWITCH(C, CALL)                         \
    switch ((C) / 64) {                                   \
        case 2: return CALL(2);                           \
        case 3: return CALL(3);                           \
        case 4: return CALL(4);                           \
        case 6: return CALL(6);                           \
        case 8: return CALL(8);                           \
        case 12: return CALL(12);                         \
        case 16: return CALL(16);                         \
        case 24: return CALL(24);                         \
        case 32: return CALL(32);                         \
        case 48: return CALL(48);                         \
        default: break;                                   \
    }

extern "C" int irads_resln_fwd(const float *x, const uint16_t *add1, const float *add1_scale, const uint16_t *add2,
                               float add2_mult, int M, int C, int rows_per_sample, const float *gamma,
                               const float *beta, float eps, float *x_out, uint16_t *ln_out, uint16_t *xb_out,
                               float *mean, float *rstd, void *stream) {
    IRADS_REQUIRE(x != nullptr && M >= 0 && C % 64 == 0, "irads_resln_fwd: need x and C %% 64 == 0 (C=%d)", C);
    IRADS_REQUIRE(rows_per_sample > 0, "irads_resln_fwd: rows_per_sample must be > 0");
    IRADS_REQUIRE(gamma == nullptr || (beta && ln_out && mean && rstd),
                  "irads_resln_fwd: LayerNorm needs gamma, beta, ln_out, mean and rstd");
    if (M == 0) return IRADS_OK;
    hipStream_t st = (hipStream_t)stream;
#define CALL(V) resln_fwd_vpt<V>(x, add1, add1_scale, add2, add2_mult, M, rows_per_sample, gamma, beta, eps, x_out, \
                                 ln_out, xb_out, mean, rstd, st)
    IRADS_VPT_SWITCH(C, CALL)
#undef CALL
    set_error("irads_resln_fwd: C=%d not supported (C/64 in {2,3,4,6,8,12,16,24,32,48})", C);
    return IRADS_EINVAL;
}

extern "C" int irads_resln_bwd(const uint16_t *dy, const float *x, const float *mean, const float *rstd,
                               const float *gamma, const float *g_res, const uint16_t *g_add, int M, int C,
                               int rows_per_sample, float *dx_out, uint16_t *b1_out, const float *b1_scale,
                               uint16_t *b2_out, float b2_mult, void *stream) {
    IRADS_REQUIRE(M >= 0 && C % 64 == 0, "irads_resln_bwd: C %% 64 != 0 (C=%d)", C);
    IRADS_REQUIRE(rows_per_sample > 0, "irads_resln_bwd: rows_per_sample must be > 0");
    IRADS_REQUIRE(dy == nullptr || (x && mean && rstd && gamma),
                  "irads_resln_bwd: LayerNorm backward needs x, mean, rstd and gamma");
    if (M == 0) return IRADS_OK;
    hipStream_t st = (hipStream_t)stream;
#define CALL(V) resln_bwd_vpt<V>(dy, x, mean, rstd, gamma, g_res, g_add, M, rows_per_sample, dx_out, b1_out, b1_scale, \
                                 b2_out, b2_mult, st)
    IRADS_VPT_SWITCH(C, CALL)
#undef CALL
    set_error("irads_resln_bwd: C=%d not supported (C/64 in {2,3,4,6,8,12,16,24,32,48})", C);
    return IRADS_EINVAL;
}

static int elem_launch(int op, const uint16_t *a, const uint16_t *b, uint16_t *out, long n, float p, float scale,
                       unsigned long long seed, void *stream, const uint64_t *seed_dev = nullptr) {
    const unsigned long long *sd = reinterpret_cast<const unsigned long long *>(seed_dev);
    if (n <= 0) return IRADS_OK;
    const long threads = (n + 7) / 8;
    dim3 grid((unsigned)((threads + 255) / 256)), block(256);
    hipStream_t st = (hipStream_t)stream;
    switch (op) {
        case 0: hipLaunchKernelGGL(elem_kernel<0>, grid, block, 0, st, a, b, out, n, p, scale, seed, sd); break;
        case 1: hipLaunchKernelGGL(elem_kernel<1>, grid, block, 0, st, a, b, out, n, p, scale, seed, sd); break;
        case 2: hipLaunchKernelGGL(elem_kernel<2>, grid, block, 0, st, a, b, out, n, p, scale, seed, sd); break;
        default: hipLaunchKernelGGL(elem_kernel<3>, grid, block, 0, st, a, b, out, n, p, scale, seed, sd); break;
    }
    return check_launch("irads_elementwise");
}

extern "C" int irads_gelu_fwd(const uint16_t *u, uint16_t *g, long n, void *stream) {
    IRADS_REQUIRE(u && g, "irads_gelu_fwd: null pointer");
    return elem_launch(0, u, nullptr, g, n, 0.f, 1.f, 0, stream);
}
extern "C" int irads_gelu_bwd(const uint16_t *u, const uint16_t *dg, uint16_t *du, long n, void *stream) {
    IRADS_REQUIRE(u && dg && du, "irads_gelu_bwd: null pointer");
    return elem_launch(1, u, dg, du, n, 0.f, 1.f, 0, stream);
}
extern "C" int irads_relu_dropout_fwd(const uint16_t *a, uint16_t *r, long n, float p, uint64_t seed,
                                      const uint64_t *seed_dev, void *stream) {
    IRADS_REQUIRE(a && r && p >= 0.f && p < 1.f, "irads_relu_dropout_fwd: bad arguments (p=%f)", (double)p);
    return elem_launch(2, a, nullptr, r, n, p, 1.f / (1.f - p), seed, stream, seed_dev);
}
extern "C" int irads_relu_dropout_bwd(const uint16_t *r, const uint16_t *dr, uint16_t *da, long n, float p,
                                      void *stream) {
    IRADS_REQUIRE(r && dr && da && p >= 0.f && p < 1.f, "irads_relu_dropout_bwd: bad arguments");
    return elem_launch(3, r, dr, da, n, p, p > 0.f ? 1.f / (1.f - p) : 1.f, 0, stream);
}

extern "C" int irads_droppath_scales(const uint64_t *seed_dev, uint64_t salt, const double *keep, const float *inv,
                                     int n_slots, int S, float *out, void *stream) {
    IRADS_REQUIRE(seed_dev && keep && inv && out && n_slots >= 1 && S >= 1, "irads_droppath_scales: bad arguments");
    const int n = n_slots * S;
    hipLaunchKernelGGL(droppath_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const unsigned long long *>(seed_dev), (unsigned long long)salt, keep, inv,
                       n_slots, S, out);
    return check_launch("irads_droppath_scales");
}
