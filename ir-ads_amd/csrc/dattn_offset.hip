// Offset networks of DAttentionMM (reference semseg/models/backbones/swin.py:777-786, applied at
// :880-905), both modalities in one launch:
//
//   pos_m = clamp(bf16(Conv1x1_{gc->2}(GELU(LN_gc(DWConv_{ks x ks, stride s}(x_m)))) + ref), -1, 1)
//
// per (map n = b*G + g, key cell (oy, ox)), m in {x, y} with its own weights.  The maps are
// tiny (16 x 16 key cells for every stage of the Swin-B config) and the whole network is
// ~1.3k MACs per cell, so as MIOpen convolutions (a grouped 9x9 conv without a tuned solver:
// naive kernels; NCHW <-> NHWC transposes; separate LayerNorm, GELU, 1x1, add, clamp and a
// weight cast per parameter) it cost ~1.5 ms of the step; here it is one launch forward and
// three backward.
//
// Rounding follows the autocast module path op by op: the depthwise conv and the 1x1 conv
// take bf16 operands (weights rounded from the fp32 parameters here) with fp32 accumulation
// and a bf16 result; the conv bias is added to the rounded conv output and rounded again
// (MIOpen adds it as a separate bf16 tensor op); LayerNorm and GELU run in fp32 on the bf16
// conv output; the offset is added to the bf16 reference points in bf16.
//
// Lanes: GCP consecutive lanes (GCP = 16 or 32 >= gc) hold the channels of one key cell, so
// the channel reductions of LayerNorm and the 1x1 conv are in-wave butterflies (their result
// is broadcast from the group's first lane so every lane uses the same value).
//
// Backward recomputes the forward (cheaper than saving it) and:
//   k1  per cell/channel: the gradient chain down to the conv output dV (bf16 values, kept as
//       fp32), plus per-block partial sums of the 1x1 weight, LayerNorm affine and conv bias
//       gradients (summed in a fixed order; the host adds the block partials);
//   k2  the depthwise weight gradient dW[c][ky][kx] = sum_{n,cell} dV * x, one block per
//       (channel, ky), a fixed-order block reduction;
//   k3  the input gradient, gathered per input pixel from the <= ceil(ks/s)^2 cells covering it.
#include "common.h"

namespace irads {
namespace {

typedef unsigned short u16;

__device__ __forceinline__ float rbf(float v) { return bf2f(f2bf(v)); }
__device__ __forceinline__ float gelu_f(float x) { return x * 0.5f * (1.f + erff(x * 0.70710678118654752440f)); }
__device__ __forceinline__ float gelu_grad(float x) {
    const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752440f));
    const float pdf = expf(-0.5f * x * x) * 0.39894228040143267794f;
    return cdf + x * pdf;
}

struct OffNet {
    const float *w;   // (gc, 1, ks, ks) depthwise weight
    const float *b;   // (gc) depthwise bias
    const float *lg;  // (gc) LayerNorm weight
    const float *lb;  // (gc) LayerNorm bias
    const float *w2;  // (2, gc) 1x1 conv weight (no bias)
};

struct OffArgs {
    const u16 *x[2];
    long sb[2], sc[2], sh[2], sw[2];  // element strides of x_m viewed as (B, G*gc, H, W)
    OffNet net[2];
    const u16 *ref;  // (Hk*Wk, 2) bf16 reference points (y, x)
    int B, G, gc, H, W, Hk, Wk, stride, pad;
    float eps;
};

template <int GCP>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = GCP / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return __shfl(v, (threadIdx.x & 63) & ~(GCP - 1), 64);
}

// depthwise weights of both modalities, bf16-rounded, into LDS: wl[m][c][k]
template <int KS>
__device__ __forceinline__ void load_weights(const OffArgs &a, float *wl) {
    const int per = a.gc * KS * KS;
    for (int i = threadIdx.x; i < 2 * per; i += blockDim.x) {
        const int m = i / per;
        wl[i] = rbf(a.net[m].w[i - m * per]);
    }
}

struct Cell {
    float v, rstd, xhat, ln, gb, r0, r1;
};

// forward of one (cell, channel); every lane of the group must call it (shuffles)
template <int GCP, int KS>
__device__ __forceinline__ Cell cell_forward(const OffArgs &a, int m, bool pv, int n, int oy, int ox, int c,
                                             const float *wl) {
    const OffNet &net = a.net[m];
    const bool cv = pv && c < a.gc;
    float acc = 0.f;
    if (cv) {
        const int b = n / a.G, gi = n - b * a.G;
        const u16 *xp = a.x[m] + b * a.sb[m] + (long)(gi * a.gc + c) * a.sc[m];
        const float *w = wl + (m * a.gc + c) * KS * KS;
#pragma unroll
        for (int ky = 0; ky < KS; ++ky) {
            const int iy = oy * a.stride - a.pad + ky;
            if (iy < 0 || iy >= a.H) continue;
#pragma unroll
            for (int kx = 0; kx < KS; ++kx) {
                const int ix = ox * a.stride - a.pad + kx;
                if (ix < 0 || ix >= a.W) continue;
                acc += bf2f(xp[iy * a.sh[m] + ix * a.sw[m]]) * w[ky * KS + kx];
            }
        }
    }
    Cell s;
    s.v = cv ? rbf(rbf(acc) + rbf(net.b[c])) : 0.f;
    const float inv = 1.f / (float)a.gc;
    const float mean = group_sum<GCP>(s.v) * inv;
    const float d = cv ? s.v - mean : 0.f;
    const float var = group_sum<GCP>(d * d) * inv;
    s.rstd = rsqrtf(var + a.eps);
    s.xhat = d * s.rstd;
    s.ln = cv ? s.xhat * net.lg[c] + net.lb[c] : 0.f;
    s.gb = cv ? rbf(gelu_f(s.ln)) : 0.f;
    const float o0 = rbf(group_sum<GCP>(cv ? s.gb * rbf(net.w2[c]) : 0.f));
    const float o1 = rbf(group_sum<GCP>(cv ? s.gb * rbf(net.w2[a.gc + c]) : 0.f));
    const int p = oy * a.Wk + ox;
    s.r0 = pv ? rbf(o0 + bf2f(a.ref[2 * p])) : 0.f;
    s.r1 = pv ? rbf(o1 + bf2f(a.ref[2 * p + 1])) : 0.f;
    return s;
}

template <int GCP, int KS>
__global__ __launch_bounds__(256) void offset_fwd_kernel(OffArgs a, float *__restrict__ pos0,
                                                         float *__restrict__ pos1) {
    __shared__ float wl[2 * 32 * KS * KS];
    load_weights<KS>(a, wl);
    __syncthreads();
    constexpr int PPB = 256 / GCP;
    const int m = blockIdx.y;
    const long cells = (long)a.B * a.G * a.Hk * a.Wk;
    const long pix = (long)blockIdx.x * PPB + threadIdx.x / GCP;
    const int c = threadIdx.x % GCP;
    const bool pv = pix < cells;
    const int hw = a.Hk * a.Wk;
    const int n = pv ? (int)(pix / hw) : 0, p = pv ? (int)(pix % hw) : 0;
    const Cell s = cell_forward<GCP, KS>(a, m, pv, n, p / a.Wk, p % a.Wk, c, wl);
    if (pv && c == 0) {
        float *pos = m ? pos1 : pos0;
        pos[2 * pix] = fminf(fmaxf(s.r0, -1.f), 1.f);
        pos[2 * pix + 1] = fminf(fmaxf(s.r1, -1.f), 1.f);
    }
}

// k1: gradient down to the conv output + block partials of (dW2[0], dW2[1], dLNw, dLNb, db)
template <int GCP, int KS>
__global__ __launch_bounds__(256) void offset_bwd_cell_kernel(OffArgs a, const float *__restrict__ gpos0,
                                                              const float *__restrict__ gpos1,
                                                              float *__restrict__ dv0, float *__restrict__ dv1,
                                                              float *__restrict__ part) {
    constexpr int PPB = 256 / GCP;
    __shared__ float wl[2 * 32 * KS * KS];
    __shared__ float red[5][PPB][GCP];
    load_weights<KS>(a, wl);
    __syncthreads();
    const int m = blockIdx.y;
    const OffNet &net = a.net[m];
    const long cells = (long)a.B * a.G * a.Hk * a.Wk;
    const int pl = threadIdx.x / GCP, c = threadIdx.x % GCP;
    const long pix = (long)blockIdx.x * PPB + pl;
    const bool pv = pix < cells, cv = pv && c < a.gc;
    const int hw = a.Hk * a.Wk;
    const int n = pv ? (int)(pix / hw) : 0, p = pv ? (int)(pix % hw) : 0;
    const Cell s = cell_forward<GCP, KS>(a, m, pv, n, p / a.Wk, p % a.Wk, c, wl);
    const float *gpos = m ? gpos1 : gpos0;
    // .float() backward -> bf16 gradient; clamp passes it where -1 <= r <= 1
    const float gp0 = pv ? rbf(gpos[2 * pix]) : 0.f, gp1 = pv ? rbf(gpos[2 * pix + 1]) : 0.f;
    const float go0 = (s.r0 >= -1.f && s.r0 <= 1.f) ? gp0 : 0.f;
    const float go1 = (s.r1 >= -1.f && s.r1 <= 1.f) ? gp1 : 0.f;
    float dgb = 0.f, dln = 0.f;
    if (cv) {
        dgb = rbf(go0 * rbf(net.w2[c]) + go1 * rbf(net.w2[a.gc + c]));  // 1x1 conv dgrad (bf16)
        dln = dgb * gelu_grad(s.ln);
    }
    const float t = cv ? dln * net.lg[c] : 0.f;
    const float inv = 1.f / (float)a.gc;
    const float mt = group_sum<GCP>(t) * inv;
    const float mtx = group_sum<GCP>(t * s.xhat) * inv;
    const float dvb = cv ? rbf(s.rstd * (t - mt - s.xhat * mtx)) : 0.f;  // LN input is bf16
    if (cv) (m ? dv1 : dv0)[pix * a.gc + c] = dvb;
    red[0][pl][c] = go0 * s.gb;
    red[1][pl][c] = go1 * s.gb;
    red[2][pl][c] = dln * s.xhat;
    red[3][pl][c] = dln;
    red[4][pl][c] = dvb;
    __syncthreads();
    if (threadIdx.x < 5 * GCP) {
        const int q = threadIdx.x / GCP, cc = threadIdx.x % GCP;
        float acc = 0.f;
        for (int i = 0; i < PPB; ++i) acc += red[q][i][cc];
        if (cc < a.gc) part[(((long)m * gridDim.x + blockIdx.x) * 5 + q) * a.gc + cc] = acc;
    }
}

// k2: depthwise weight gradient, block (c, ky, m), threads stride over cells
template <int KS>
__global__ __launch_bounds__(256) void offset_bwd_weight_kernel(OffArgs a, const float *__restrict__ dv0,
                                                                const float *__restrict__ dv1,
                                                                float *__restrict__ dw) {
    __shared__ float red[4][KS];
    const int c = blockIdx.x, ky = blockIdx.y, m = blockIdx.z;
    const float *dv = m ? dv1 : dv0;
    const long cells = (long)a.B * a.G * a.Hk * a.Wk;
    const int hw = a.Hk * a.Wk;
    float acc[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) acc[k] = 0.f;
    for (long pix = threadIdx.x; pix < cells; pix += blockDim.x) {
        const int n = (int)(pix / hw), p = (int)(pix % hw);
        const int oy = p / a.Wk, ox = p % a.Wk;
        const int iy = oy * a.stride - a.pad + ky;
        if (iy < 0 || iy >= a.H) continue;
        const float d = dv[pix * a.gc + c];
        const int b = n / a.G, gi = n - b * a.G;
        const u16 *xp = a.x[m] + b * a.sb[m] + (long)(gi * a.gc + c) * a.sc[m] + iy * a.sh[m];
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
            const int ix = ox * a.stride - a.pad + kx;
            if (ix >= 0 && ix < a.W) acc[kx] += d * bf2f(xp[ix * a.sw[m]]);
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        const float v = wave_sum(acc[k]);  // butterfly: every lane holds the same bits only up to order;
        if (lane == 0) red[wave][k] = v;  // lane 0's value is the one kept
    }
    __syncthreads();
    if (threadIdx.x < KS) {
        const int k = threadIdx.x;
        dw[(((long)m * a.gc + c) * KS + ky) * KS + k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    }
}

// k3: input gradient, thread per (m, n, iy, ix, c), channel fastest
template <int KS>
__global__ __launch_bounds__(256) void offset_bwd_input_kernel(OffArgs a, const float *__restrict__ dv0,
                                                               const float *__restrict__ dv1, u16 *__restrict__ dx0,
                                                               u16 *__restrict__ dx1) {
    __shared__ float wl[2 * 32 * KS * KS];
    load_weights<KS>(a, wl);
    __syncthreads();
    const int m = blockIdx.y;
    const long total = (long)a.B * a.G * a.H * a.W * a.gc;
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const int c = (int)(e % a.gc);
    long r = e / a.gc;
    const int ix = (int)(r % a.W);
    r /= a.W;
    const int iy = (int)(r % a.H);
    const int n = (int)(r / a.H);
    const float *dv = m ? dv1 : dv0;
    const float *w = wl + (m * a.gc + c) * KS * KS;
    // cells with oy*s - pad <= iy <= oy*s - pad + KS - 1
    const int s = a.stride;
    const int oy_lo = max(0, (iy + a.pad - KS + 1 + s - 1 + s * KS) / s - KS), oy_hi = min(a.Hk - 1, (iy + a.pad) / s);
    const int ox_lo = max(0, (ix + a.pad - KS + 1 + s - 1 + s * KS) / s - KS), ox_hi = min(a.Wk - 1, (ix + a.pad) / s);
    float acc = 0.f;
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
        const int ky = iy + a.pad - oy * s;
        for (int ox = ox_lo; ox <= ox_hi; ++ox) {
            const int kx = ix + a.pad - ox * s;
            acc += dv[((long)n * a.Hk * a.Wk + oy * a.Wk + ox) * a.gc + c] * w[ky * KS + kx];
        }
    }
    const int b = n / a.G, gi = n - b * a.G;
    u16 *dx = m ? dx1 : dx0;
    dx[b * a.sb[m] + (long)(gi * a.gc + c) * a.sc[m] + iy * a.sh[m] + ix * a.sw[m]] = f2bf(acc);
}

int fill_args(OffArgs &a, const uint16_t *x, const long *xs, const uint16_t *y, const long *ys, const float *const *px,
              const float *const *py, const uint16_t *ref, int B, int G, int gc, int H, int W, int ks, int stride,
              int pad, float eps) {
    IRADS_REQUIRE(x && y && xs && ys && px && py && ref, "irads_dattn_offset: null pointer");
    IRADS_REQUIRE(B > 0 && G > 0 && gc > 0 && gc <= 32 && H > 0 && W > 0 && stride > 0 && pad >= 0,
                  "irads_dattn_offset: bad shape (B=%d G=%d gc=%d H=%d W=%d stride=%d pad=%d)", B, G, gc, H, W, stride,
                  pad);
    IRADS_REQUIRE(ks == 3 || ks == 5 || ks == 7 || ks == 9, "irads_dattn_offset: ks=%d not in {3, 5, 7, 9}", ks);
    a.x[0] = x, a.x[1] = y;
    for (int m = 0; m < 2; ++m) {
        const long *s = m ? ys : xs;
        a.sb[m] = s[0], a.sc[m] = s[1], a.sh[m] = s[2], a.sw[m] = s[3];
        const float *const *pp = m ? py : px;
        for (int i = 0; i < 5; ++i) IRADS_REQUIRE(pp[i], "irads_dattn_offset: null parameter %d", i);
        a.net[m] = OffNet{pp[0], pp[1], pp[2], pp[3], pp[4]};
    }
    a.ref = ref;
    a.B = B, a.G = G, a.gc = gc, a.H = H, a.W = W, a.stride = stride, a.pad = pad, a.eps = eps;
    a.Hk = (H + 2 * pad - ks) / stride + 1;
    a.Wk = (W + 2 * pad - ks) / stride + 1;
    IRADS_REQUIRE(a.Hk > 0 && a.Wk > 0, "irads_dattn_offset: empty output (%dx%d)", a.Hk, a.Wk);
    return IRADS_OK;
}

#define IRADS_OFF_KS(KS_, ...)                 \
    switch (KS_) {                             \
        case 3: { constexpr int KS = 3; __VA_ARGS__; } break; \
        case 5: { constexpr int KS = 5; __VA_ARGS__; } break; \
        case 7: { constexpr int KS = 7; __VA_ARGS__; } break; \
        default: { constexpr int KS = 9; __VA_ARGS__; } break; \
    }

}  // namespace
}  // namespace irads

using namespace irads;

extern "C" long irads_dattn_offset_partials(int B, int G, int gc, int H, int W, int ks, int stride, int pad) {
    const long hk = (H + 2 * pad - ks) / stride + 1, wk = (W + 2 * pad - ks) / stride + 1;
    const long cells = (long)B * G * hk * wk;
    const int ppb = gc <= 16 ? 16 : 8;
    return 2 * ((cells + ppb - 1) / ppb) * 5 * gc;
}

extern "C" int irads_dattn_offset_fwd(const uint16_t *x, const long *x_strides, const uint16_t *y,
                                      const long *y_strides, const float *const *params_x,
                                      const float *const *params_y, const uint16_t *ref, int B, int G, int gc, int H,
                                      int W, int ks, int stride, int pad, float eps, float *pos_x, float *pos_y,
                                      void *stream) {
    OffArgs a;
    int rc = fill_args(a, x, x_strides, y, y_strides, params_x, params_y, ref, B, G, gc, H, W, ks, stride, pad, eps);
    if (rc) return rc;
    IRADS_REQUIRE(pos_x && pos_y, "irads_dattn_offset_fwd: null output");
    const long cells = (long)B * G * a.Hk * a.Wk;
    hipStream_t st = (hipStream_t)stream;
    if (gc <= 16) {
        dim3 grid((unsigned)((cells + 15) / 16), 2);
        IRADS_OFF_KS(ks, hipLaunchKernelGGL((offset_fwd_kernel<16, KS>), grid, dim3(256), 0, st, a, pos_x, pos_y));
    } else {
        dim3 grid((unsigned)((cells + 7) / 8), 2);
        IRADS_OFF_KS(ks, hipLaunchKernelGGL((offset_fwd_kernel<32, KS>), grid, dim3(256), 0, st, a, pos_x, pos_y));
    }
    return check_launch("irads_dattn_offset_fwd");
}

extern "C" int irads_dattn_offset_bwd(const uint16_t *x, const long *x_strides, const uint16_t *y,
                                      const long *y_strides, const float *const *params_x,
                                      const float *const *params_y, const uint16_t *ref, int B, int G, int gc, int H,
                                      int W, int ks, int stride, int pad, float eps, const float *gpos_x,
                                      const float *gpos_y, float *dv_x, float *dv_y, float *partials, float *dw,
                                      uint16_t *dx, uint16_t *dy, void *stream) {
    OffArgs a;
    int rc = fill_args(a, x, x_strides, y, y_strides, params_x, params_y, ref, B, G, gc, H, W, ks, stride, pad, eps);
    if (rc) return rc;
    IRADS_REQUIRE(gpos_x && gpos_y && dv_x && dv_y && partials && dw && dx && dy, "irads_dattn_offset_bwd: null");
    const long cells = (long)B * G * a.Hk * a.Wk;
    hipStream_t st = (hipStream_t)stream;
    if (gc <= 16) {
        dim3 grid((unsigned)((cells + 15) / 16), 2);
        IRADS_OFF_KS(ks, hipLaunchKernelGGL((offset_bwd_cell_kernel<16, KS>), grid, dim3(256), 0, st, a, gpos_x,
                                            gpos_y, dv_x, dv_y, partials));
    } else {
        dim3 grid((unsigned)((cells + 7) / 8), 2);
        IRADS_OFF_KS(ks, hipLaunchKernelGGL((offset_bwd_cell_kernel<32, KS>), grid, dim3(256), 0, st, a, gpos_x,
                                            gpos_y, dv_x, dv_y, partials));
    }
    rc = check_launch("irads_dattn_offset_bwd cells");
    if (rc) return rc;
    IRADS_OFF_KS(ks, hipLaunchKernelGGL((offset_bwd_weight_kernel<KS>), dim3(gc, KS, 2), dim3(256), 0, st, a, dv_x,
                                        dv_y, dw));
    rc = check_launch("irads_dattn_offset_bwd weight");
    if (rc) return rc;
    const long total = (long)B * G * H * W * gc;
    IRADS_OFF_KS(ks, hipLaunchKernelGGL((offset_bwd_input_kernel<KS>), dim3((unsigned)((total + 255) / 256), 2),
                                        dim3(256), 0, st, a, dv_x, dv_y, dx, dy));
    return check_launch("irads_dattn_offset_bwd input");
}
