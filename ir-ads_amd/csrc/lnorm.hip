// Trainable LayerNorm on bf16 rows with an fp32 result: the patch embeddings' norm
// (reference semseg/models/backbones/swin.py PatchEmbed -> mmcv build_norm_layer LN, run by
// autocast in fp32 on the bf16 projection output).  torch runs it as a cast kernel, its
// generic LayerNorm kernel and three backward kernels (input, partial and final gamma/beta
// reductions) over 128-wide rows; here it is one pass each way.
//
// Forward: one wave per row, C/64 values per lane held in registers; mean and variance in
//   fp32 (two passes over the registers, biased variance like torch), y = (x - mean) * rstd
//   * gamma + beta in fp32; mean / rstd saved.
// Backward: one wave per row again; dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat))
//   written as bf16 (the input's dtype), and per-workgroup partial sums of dy*xhat (dgamma)
//   and dy (dbeta) in a fixed order, summed over workgroups by the caller (deterministic).
#include "common.h"

namespace irads {
namespace {

constexpr int kWaves = 4;  // rows in flight per workgroup (one wave per row)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ void store_out(float *y, long i, float v) { y[i] = v; }
__device__ __forceinline__ void store_out(unsigned short *y, long i, float v) { y[i] = f2bf(v); }
__device__ __forceinline__ float load_in(const float *p, long i) { return p[i]; }
__device__ __forceinline__ float load_in(const unsigned short *p, long i) { return bf2f(p[i]); }

// V = C / 64 values per lane (lane owns channels lane + 64 k); TO = float (PatchEmbed norm)
// or bf16 storage (a frozen norm on a bf16 tensor whose consumers are Linears)
template <int V, typename TO>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const unsigned short *__restrict__ x, const float *__restrict__ g,
                                                     const float *__restrict__ b, long M, float eps,
                                                     TO *__restrict__ y, float *__restrict__ mean,
                                                     float *__restrict__ rstd) {
    constexpr int C = 64 * V;
    const int lane = threadIdx.x & 63;
    float gv[V], bv[V];
#pragma unroll
    for (int k = 0; k < V; ++k) gv[k] = g[lane + 64 * k], bv[k] = b[lane + 64 * k];
    for (long r = (long)blockIdx.x * kWaves + (threadIdx.x >> 6); r < M; r += (long)gridDim.x * kWaves) {
        float v[V];
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < V; ++k) {
            v[k] = bf2f(x[r * C + lane + 64 * k]);
            s += v[k];
        }
        const float mu = wave_sum(s) / (float)C;
        float q = 0.f;
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const float d = v[k] - mu;
            q += d * d;
        }
        const float rs = rsqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
        for (int k = 0; k < V; ++k) store_out(y, r * C + lane + 64 * k, (v[k] - mu) * rs * gv[k] + bv[k]);
        if (lane == 0) {
            mean[r] = mu;
            rstd[r] = rs;
        }
    }
}

// TD = dy storage (fp32 / bf16); part == nullptr: frozen affine, no gamma / beta sums
template <int V, typename TD>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const TD *__restrict__ dy, const unsigned short *__restrict__ x,
                                                     const float *__restrict__ mean, const float *__restrict__ rstd,
                                                     const float *__restrict__ g, long M,
                                                     unsigned short *__restrict__ dx, float *__restrict__ part) {
    constexpr int C = 64 * V;
    __shared__ float red[kWaves][2][C];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float gv[V], sg[V], sb[V];
#pragma unroll
    for (int k = 0; k < V; ++k) gv[k] = g[lane + 64 * k], sg[k] = sb[k] = 0.f;
    for (long r = (long)blockIdx.x * kWaves + wv; r < M; r += (long)gridDim.x * kWaves) {
        const float mu = mean[r], rs = rstd[r];
        float xh[V], d[V];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const long i = r * C + lane + 64 * k;
            xh[k] = (bf2f(x[i]) - mu) * rs;
            const float dyk = load_in(dy, i);
            d[k] = dyk * gv[k];
            s1 += d[k];
            s2 += d[k] * xh[k];
            sg[k] += dyk * xh[k];
            sb[k] += dyk;
        }
        const float m1 = wave_sum(s1) / (float)C, m2 = wave_sum(s2) / (float)C;
#pragma unroll
        for (int k = 0; k < V; ++k) dx[r * C + lane + 64 * k] = f2bf(rs * (d[k] - m1 - xh[k] * m2));
    }
    if (part == nullptr) return;  // uniform over the grid
#pragma unroll
    for (int k = 0; k < V; ++k) {
        red[wv][0][lane + 64 * k] = sg[k];
        red[wv][1][lane + 64 * k] = sb[k];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) {
        const int q = c / C, cc = c % C;
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) t += red[w][q][cc];
        part[((long)blockIdx.x * 2 + q) * C + cc] = t;
    }
}

// ---------------------------------------------------------------- PatchMerging gather + norm
// PatchMerging (reference mmcv PatchMerging in semseg/models/backbones/swin.py: nn.Unfold
// 2x2/2 + LayerNorm(4C) + Linear): the 2x2 unfold as the LayerNorm's read pattern.  Output
// token (b, oh, ow) is the row p = 4c + 2i + j <- x[b, 2oh+i, 2ow+j, c] (nn.Unfold's
// channel-major order), normalised in fp32 with the frozen affine and written as the bf16
// operand of the reduction GEMM.  Lane l owns channels c = l + 64k (k < V) and all four
// (i, j) of each: every load is a 256-B row segment of one source token, every store 8 B per
// lane over a contiguous 512-B run.  The backward recomputes xhat from the same gather and
// scatters dx (fp32) back to the source tokens: each source element is written exactly once.
template <int V>
__global__ __launch_bounds__(256) void merge_ln_fwd_kernel(const float *__restrict__ x, int Bt, int H, int W,
                                                           const float *__restrict__ g, const float *__restrict__ b,
                                                           float eps, unsigned short *__restrict__ y,
                                                           float *__restrict__ mean, float *__restrict__ rstd) {
    constexpr int C = 64 * V, C4 = 4 * C;
    const int lane = threadIdx.x & 63;
    const int Ho = H / 2, Wo = W / 2;
    const long M = (long)Bt * Ho * Wo;
    for (long r = (long)blockIdx.x * kWaves + (threadIdx.x >> 6); r < M; r += (long)gridDim.x * kWaves) {
        const int ow = (int)(r % Wo), oh = (int)((r / Wo) % Ho);
        const long bb = r / ((long)Wo * Ho);
        const float *src = x + ((bb * H + 2 * oh) * W + 2 * ow) * C + lane;
        float v[V][4];
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < V; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // q = 2i + j
                v[k][q] = src[((q >> 1) * W + (q & 1)) * C + 64 * k];
                s += v[k][q];
            }
        const float mu = wave_sum(s) / (float)C4;
        float ss = 0.f;
#pragma unroll
        for (int k = 0; k < V; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float d = v[k][q] - mu;
                ss += d * d;
            }
        const float rs = rsqrtf(wave_sum(ss) / (float)C4 + eps);
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const int p = 4 * (lane + 64 * k);
            const float4 gg = *reinterpret_cast<const float4 *>(g + p), be = *reinterpret_cast<const float4 *>(b + p);
            const float gq[4] = {gg.x, gg.y, gg.z, gg.w}, bq[4] = {be.x, be.y, be.z, be.w};
            unsigned short o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = f2bf((v[k][q] - mu) * rs * gq[q] + bq[q]);
            uint2 w;
            w.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
            w.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
            *reinterpret_cast<uint2 *>(y + r * C4 + p) = w;
        }
        if (lane == 0) {
            mean[r] = mu;
            rstd[r] = rs;
        }
    }
}

template <int V, bool ACC>  // ACC: add into dx (the stage output's other consumers already wrote it)
__global__ __launch_bounds__(256) void merge_ln_bwd_kernel(const unsigned short *__restrict__ dy,
                                                           const float *__restrict__ x, int Bt, int H, int W,
                                                           const float *__restrict__ mean,
                                                           const float *__restrict__ rstd,
                                                           const float *__restrict__ g, float *__restrict__ dx) {
    constexpr int C = 64 * V, C4 = 4 * C;
    const int lane = threadIdx.x & 63;
    const int Ho = H / 2, Wo = W / 2;
    const long M = (long)Bt * Ho * Wo;
    for (long r = (long)blockIdx.x * kWaves + (threadIdx.x >> 6); r < M; r += (long)gridDim.x * kWaves) {
        const int ow = (int)(r % Wo), oh = (int)((r / Wo) % Ho);
        const long bb = r / ((long)Wo * Ho);
        const long base = ((bb * H + 2 * oh) * W + 2 * ow) * C + lane;
        const float mu = mean[r], rs = rstd[r];
        float xh[V][4], d[V][4];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const int p = 4 * (lane + 64 * k);
            const uint2 w = *reinterpret_cast<const uint2 *>(dy + r * C4 + p);
            const float4 gg = *reinterpret_cast<const float4 *>(g + p);
            const float dq[4] = {bf2f((unsigned short)(w.x & 0xffffu)), bf2f((unsigned short)(w.x >> 16)),
                                 bf2f((unsigned short)(w.y & 0xffffu)), bf2f((unsigned short)(w.y >> 16))};
            const float gq[4] = {gg.x, gg.y, gg.z, gg.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                xh[k][q] = (x[base + ((q >> 1) * W + (q & 1)) * C + 64 * k] - mu) * rs;
                d[k][q] = dq[q] * gq[q];
                s1 += d[k][q];
                s2 += d[k][q] * xh[k][q];
            }
        }
        const float m1 = wave_sum(s1) / (float)C4, m2 = wave_sum(s2) / (float)C4;
#pragma unroll
        for (int k = 0; k < V; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q)
            {
                const long i = base + ((q >> 1) * W + (q & 1)) * C + 64 * k;
                const float v = rs * (d[k][q] - m1 - xh[k][q] * m2);
                dx[i] = ACC ? __fadd_rn(dx[i], v) : v;  // separately rounded: the fp32 sum autograd would form
            }
    }
}

int ln_blocks(long M) {
    const long b = (M + kWaves - 1) / kWaves;
    return (int)(b < 2048 ? b : 2048);  // ~8 workgroups per CU, each walking M / (2048·4) rows
}

}  // namespace
}  // namespace irads

using namespace irads;

#define IRADS_LN_CHECK(fn)                                                                                 \
    IRADS_REQUIRE(M > 0 && (C == 64 || C == 128 || C == 192 || C == 256),                                  \
                  fn ": need M > 0 and C in {64, 128, 192, 256} (M=%ld C=%d)", M, C)

extern "C" long irads_ln_bf16_partials(long M, int C) { return (long)ln_blocks(M) * 2 * C; }

extern "C" int irads_ln_bf16_fwd(const uint16_t *x, const float *gamma, const float *beta, long M, int C, float eps,
                                 float *y, float *mean, float *rstd, void *stream) {
    IRADS_LN_CHECK("irads_ln_bf16_fwd");
    IRADS_REQUIRE(x && gamma && beta && y && mean && rstd, "irads_ln_bf16_fwd: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(ln_blocks(M));
    switch (C / 64) {
        case 1: ln_fwd_kernel<1, float><<<grid, 256, 0, st>>>(x, gamma, beta, M, eps, y, mean, rstd); break;
        case 2: ln_fwd_kernel<2, float><<<grid, 256, 0, st>>>(x, gamma, beta, M, eps, y, mean, rstd); break;
        case 3: ln_fwd_kernel<3, float><<<grid, 256, 0, st>>>(x, gamma, beta, M, eps, y, mean, rstd); break;
        default: ln_fwd_kernel<4, float><<<grid, 256, 0, st>>>(x, gamma, beta, M, eps, y, mean, rstd); break;
    }
    return check_launch("irads_ln_bf16_fwd");
}

extern "C" int irads_ln_bf16_bwd(const float *dy, const uint16_t *x, const float *mean, const float *rstd,
                                 const float *gamma, long M, int C, uint16_t *dx, float *partials, void *stream) {
    IRADS_LN_CHECK("irads_ln_bf16_bwd");
    IRADS_REQUIRE(dy && x && mean && rstd && gamma && dx && partials, "irads_ln_bf16_bwd: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(ln_blocks(M));
    switch (C / 64) {
        case 1: ln_bwd_kernel<1, float><<<grid, 256, 0, st>>>(dy, x, mean, rstd, gamma, M, dx, partials); break;
        case 2: ln_bwd_kernel<2, float><<<grid, 256, 0, st>>>(dy, x, mean, rstd, gamma, M, dx, partials); break;
        case 3: ln_bwd_kernel<3, float><<<grid, 256, 0, st>>>(dy, x, mean, rstd, gamma, M, dx, partials); break;
        default: ln_bwd_kernel<4, float><<<grid, 256, 0, st>>>(dy, x, mean, rstd, gamma, M, dx, partials); break;
    }
    return check_launch("irads_ln_bf16_bwd");
}

#define IRADS_MERGE_CHECK(fn)                                                                                     \
    IRADS_REQUIRE(Bt > 0 && H > 0 && W > 0 && H % 2 == 0 && W % 2 == 0 &&                                         \
                      (C == 128 || C == 192 || C == 256 || C == 384 || C == 512 || C == 768),                     \
                  fn ": need even H, W and C in {128, 192, 256, 384, 512, 768} (H=%d W=%d C=%d)", H, W, C)

extern "C" int irads_merge_ln_fwd(const float *x, int Bt, int H, int W, int C, const float *gamma, const float *beta,
                                  float eps, uint16_t *y, float *mean, float *rstd, void *stream) {
    IRADS_MERGE_CHECK("irads_merge_ln_fwd");
    IRADS_REQUIRE(x && gamma && beta && y && mean && rstd, "irads_merge_ln_fwd: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(ln_blocks((long)Bt * (H / 2) * (W / 2)));
#define IRADS_MF(VV) merge_ln_fwd_kernel<VV><<<grid, 256, 0, st>>>(x, Bt, H, W, gamma, beta, eps, y, mean, rstd)
    switch (C / 64) {
        case 2: IRADS_MF(2); break;
        case 3: IRADS_MF(3); break;
        case 4: IRADS_MF(4); break;
        case 6: IRADS_MF(6); break;
        case 8: IRADS_MF(8); break;
        default: IRADS_MF(12); break;
    }
#undef IRADS_MF
    return check_launch("irads_merge_ln_fwd");
}

extern "C" int irads_merge_ln_bwd(const uint16_t *dy, const float *x, int Bt, int H, int W, int C, const float *mean,
                                  const float *rstd, const float *gamma, float *dx, int accumulate, void *stream) {
    IRADS_MERGE_CHECK("irads_merge_ln_bwd");
    IRADS_REQUIRE(dy && x && mean && rstd && gamma && dx, "irads_merge_ln_bwd: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(ln_blocks((long)Bt * (H / 2) * (W / 2)));
#define IRADS_MB(VV)                                                                                    \
    (accumulate ? merge_ln_bwd_kernel<VV, true><<<grid, 256, 0, st>>>(dy, x, Bt, H, W, mean, rstd, gamma, dx) \
                : merge_ln_bwd_kernel<VV, false><<<grid, 256, 0, st>>>(dy, x, Bt, H, W, mean, rstd, gamma, dx))
    switch (C / 64) {
        case 2: IRADS_MB(2); break;
        case 3: IRADS_MB(3); break;
        case 4: IRADS_MB(4); break;
        case 6: IRADS_MB(6); break;
        case 8: IRADS_MB(8); break;
        default: IRADS_MB(12); break;
    }
#undef IRADS_MB
    return check_launch("irads_merge_ln_bwd");
}

// frozen LayerNorm, bf16 in -> bf16 out (DeformMPG's fuse_norm on the bf16 U_fc1 output, whose
// consumers are the heads' Linears); backward bf16 dy -> bf16 dx, no affine gradients.
#define IRADS_LNB_CHECK(fn)                                                                                \
    IRADS_REQUIRE(M > 0 && C % 64 == 0 && (C / 64 <= 4 || C / 64 == 8 || C / 64 == 16),                    \
                  fn ": need M > 0 and C / 64 in {1, 2, 3, 4, 8, 16} (M=%ld C=%d)", M, C)

extern "C" int irads_ln_bf16_bf16_fwd(const uint16_t *x, const float *gamma, const float *beta, long M, int C,
                                      float eps, uint16_t *y, float *mean, float *rstd, void *stream) {
    IRADS_LNB_CHECK("irads_ln_bf16_bf16_fwd");
    IRADS_REQUIRE(x && gamma && beta && y && mean && rstd, "irads_ln_bf16_bf16_fwd: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(ln_blocks(M));
#define IRADS_LF(VV) ln_fwd_kernel<VV, unsigned short><<<grid, 256, 0, st>>>(x, gamma, beta, M, eps, y, mean, rstd)
    switch (C / 64) {
        case 1: IRADS_LF(1); break;
        case 2: IRADS_LF(2); break;
        case 3: IRADS_LF(3); break;
        case 4: IRADS_LF(4); break;
        case 8: IRADS_LF(8); break;
        default: IRADS_LF(16); break;
    }
#undef IRADS_LF
    return check_launch("irads_ln_bf16_bf16_fwd");
}

extern "C" int irads_ln_bf16_bf16_bwd(const uint16_t *dy, const uint16_t *x, const float *mean, const float *rstd,
                                      const float *gamma, long M, int C, uint16_t *dx, void *stream) {
    IRADS_LNB_CHECK("irads_ln_bf16_bf16_bwd");
    IRADS_REQUIRE(dy && x && mean && rstd && gamma && dx, "irads_ln_bf16_bf16_bwd: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(ln_blocks(M));
#define IRADS_LB(VV) \
    ln_bwd_kernel<VV, unsigned short><<<grid, 256, 0, st>>>(dy, x, mean, rstd, gamma, M, dx, nullptr)
    switch (C / 64) {
        case 1: IRADS_LB(1); break;
        case 2: IRADS_LB(2); break;
        case 3: IRADS_LB(3); break;
        case 4: IRADS_LB(4); break;
        case 8: IRADS_LB(8); break;
        default: IRADS_LB(16); break;
    }
#undef IRADS_LB
    return check_launch("irads_ln_bf16_bf16_bwd");
}
