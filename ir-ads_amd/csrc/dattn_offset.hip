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
// A block owns one output row of one map: the ks input rows it reads are staged in LDS
// channel-fastest (coalesced global reads, conflict-free taps), so each input value is read
// from HBM once per row instead of once per tap (81x at stride 1).
//
// Backward recomputes the forward (cheaper than saving it) and:
//   k1  per cell/channel: the gradient chain down to the conv output dV (bf16 values, kept as
//       fp32), plus per-block partial sums of the 1x1 weight, LayerNorm affine and conv bias
//       gradients and of the depthwise weight gradient (dV x the staged taps), in fixed orders;
//       the host adds the block partials;
//   k2  the input gradient, gathered per input pixel from the <= ceil(ks/s)^2 cells covering it.
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

// depthwise weights of modality m, bf16-rounded, into LDS: wl[c][k]
template <int KS>
__device__ __forceinline__ void load_weights(const OffArgs &a, int m, float *wl) {
    const int per = a.gc * KS * KS;
    for (int i = threadIdx.x; i < per; i += blockDim.x) wl[i] = rbf(a.net[m].w[i]);
}

// The KS input rows output row oy of map n reads, into LDS as [r][ix][c] (channel fastest:
// the GCP lanes of a cell read one 2*GCP-byte run).  Rows outside the map are zero, so the
// taps only test the column.  Global reads run along the unit-stride dimension of x.
template <int GCP, int KS>
__device__ __forceinline__ void stage_rows(const OffArgs &a, int m, int n, int oy, u16 *rows) {
    const int b = n / a.G, gi = n - b * a.G;
    const u16 *xb = a.x[m] + b * a.sb[m] + (long)gi * a.gc * a.sc[m];
    const int W = a.W, gc = a.gc;
    const int total = KS * W * gc;
    const bool cfast = a.sc[m] == 1;  // channels-last memory: read channel-fastest
    if (!cfast && a.sw[m] == 1 && W % 8 == 0 && (((uintptr_t)xb) & 15) == 0 && a.sh[m] % 8 == 0 &&
        a.sc[m] % 8 == 0) {
        // NCHW rows: 16-byte loads of 8 columns, scattered channel-fastest into LDS
        const int groups = KS * gc * (W / 8);
        for (int e = threadIdx.x; e < groups; e += blockDim.x) {
            const int ix0 = (e % (W / 8)) * 8, c = (e / (W / 8)) % gc, r = e / ((W / 8) * gc);
            const int iy = oy * a.stride - a.pad + r;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (iy >= 0 && iy < a.H) v = *reinterpret_cast<const uint4 *>(xb + c * a.sc[m] + iy * a.sh[m] + ix0);
            const unsigned w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 8; ++j)
                rows[(r * W + ix0 + j) * GCP + c] = (u16)(j & 1 ? w4[j >> 1] >> 16 : w4[j >> 1] & 0xffffu);
        }
        return;
    }
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
        int r, ix, c;
        if (cfast) {
            c = e % gc;
            ix = (e / gc) % W;
            r = e / (gc * W);
        } else {
            ix = e % W;
            c = (e / W) % gc;
            r = e / (W * gc);
        }
        const int iy = oy * a.stride - a.pad + r;
        u16 v = 0;
        if (iy >= 0 && iy < a.H) v = xb[c * a.sc[m] + iy * a.sh[m] + ix * a.sw[m]];
        rows[(r * W + ix) * GCP + c] = v;
    }
}

struct Cell {
    float v, rstd, xhat, ln, gb, r0, r1;
};

// forward of one (cell, channel) from the staged rows; every lane of the group must call it
template <int GCP, int KS>
__device__ __forceinline__ Cell cell_forward(const OffArgs &a, int m, bool pv, int oy, int ox, int c,
                                             const float *wl, const u16 *rows) {
    const OffNet &net = a.net[m];
    const bool cv = pv && c < a.gc;
    float acc = 0.f;
    if (cv) {
        const float *w = wl + c * KS * KS;
#pragma unroll
        for (int ky = 0; ky < KS; ++ky) {
#pragma unroll
            for (int kx = 0; kx < KS; ++kx) {
                const int ix = ox * a.stride - a.pad + kx;
                if (ix < 0 || ix >= a.W) continue;
                acc += bf2f(rows[(ky * a.W + ix) * GCP + c]) * w[ky * KS + kx];
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

// dynamic LDS: staged rows (u16) after the fixed arrays
template <int GCP, int KS>
__host__ __device__ constexpr int rows_offset_bytes() {
    return 32 * KS * KS * 4;
}

// block = (map n, output row oy), blockIdx.y = modality; cells ox in chunks of 256 / GCP
template <int GCP, int KS>
__global__ __launch_bounds__(256) void offset_fwd_kernel(OffArgs a, float *__restrict__ pos0,
                                                         float *__restrict__ pos1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *wl = reinterpret_cast<float *>(smem);
    u16 *rows = reinterpret_cast<u16 *>(smem + rows_offset_bytes<GCP, KS>());
    constexpr int PPB = 256 / GCP;
    const int m = blockIdx.y, n = blockIdx.x / a.Hk, oy = blockIdx.x % a.Hk;
    load_weights<KS>(a, m, wl);
    stage_rows<GCP, KS>(a, m, n, oy, rows);
    __syncthreads();
    const int pl = threadIdx.x / GCP, c = threadIdx.x % GCP;
    float *pos = m ? pos1 : pos0;
    for (int ox0 = 0; ox0 < a.Wk; ox0 += PPB) {
        const int ox = ox0 + pl;
        const bool pv = ox < a.Wk;
        const Cell s = cell_forward<GCP, KS>(a, m, pv, oy, pv ? ox : 0, c, wl, rows);
        if (pv && c == 0) {
            const long pix = ((long)n * a.Hk + oy) * a.Wk + ox;
            pos[2 * pix] = fminf(fmaxf(s.r0, -1.f), 1.f);
            pos[2 * pix + 1] = fminf(fmaxf(s.r1, -1.f), 1.f);
        }
    }
}

// backward, block = (map n, output row oy) as the forward: the gradient chain down to the conv
// output dV (kept for the input gradient, and in LDS), then this block's partial sums of the
// 1x1 weight, LN affine and conv bias gradients ([5][gc]) and of the depthwise weight gradient
// ([gc][KS*KS]: dV x the staged taps, summed over the row's cells).  Fixed summation orders.
template <int GCP, int KS>
__global__ __launch_bounds__(256) void offset_bwd_cell_kernel(OffArgs a, const float *__restrict__ gpos0,
                                                              const float *__restrict__ gpos1,
                                                              float *__restrict__ dv0, float *__restrict__ dv1,
                                                              float *__restrict__ part, float *__restrict__ wpart) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *wl = reinterpret_cast<float *>(smem);
    u16 *rows = reinterpret_cast<u16 *>(smem + rows_offset_bytes<GCP, KS>());
    constexpr int PPB = 256 / GCP;
    constexpr int MAXW = 64;  // cells per row held in LDS for the weight-gradient pass
    __shared__ float red[5][PPB][GCP];
    __shared__ float dvl[MAXW][GCP];
    const int m = blockIdx.y, n = blockIdx.x / a.Hk, oy = blockIdx.x % a.Hk;
    const OffNet &net = a.net[m];
    load_weights<KS>(a, m, wl);
    stage_rows<GCP, KS>(a, m, n, oy, rows);
    __syncthreads();
    const int pl = threadIdx.x / GCP, c = threadIdx.x % GCP;
    const float *gpos = m ? gpos1 : gpos0;
    float *dvg = m ? dv1 : dv0;
    float acc5[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int ox0 = 0; ox0 < a.Wk; ox0 += PPB) {
        const int ox = ox0 + pl;
        const bool pv = ox < a.Wk, cv = pv && c < a.gc;
        const Cell s = cell_forward<GCP, KS>(a, m, pv, oy, pv ? ox : 0, c, wl, rows);
        const long pix = ((long)n * a.Hk + oy) * a.Wk + (pv ? ox : 0);
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
        if (cv) dvg[pix * a.gc + c] = dvb;
        if (pv && ox < MAXW) dvl[ox][c] = dvb;
        acc5[0] += go0 * s.gb;
        acc5[1] += go1 * s.gb;
        acc5[2] += dln * s.xhat;
        acc5[3] += dln;
        acc5[4] += dvb;
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) red[q][pl][c] = acc5[q];
    __syncthreads();
    const long blk = (long)m * gridDim.x + blockIdx.x;
    if (threadIdx.x < 5 * GCP) {
        const int q = threadIdx.x / GCP, cc = threadIdx.x % GCP;
        float acc = 0.f;
        for (int i = 0; i < PPB; ++i) acc += red[q][i][cc];
        if (cc < a.gc) part[(blk * 5 + q) * a.gc + cc] = acc;
    }
    // depthwise weight gradient of this row: pair (c, ky, kx) per thread iteration
    const int KK = KS * KS, pairs = a.gc * KK, wk = min(a.Wk, MAXW);
    for (int pr = threadIdx.x; pr < pairs; pr += blockDim.x) {
        const int cc = pr / KK, k = pr - cc * KK, ky = k / KS, kx = k - ky * KS;
        float acc = 0.f;
        for (int ox = 0; ox < wk; ++ox) {
            const int ix = ox * a.stride - a.pad + kx;
            if (ix >= 0 && ix < a.W) acc += dvl[ox][cc] * bf2f(rows[(ky * a.W + ix) * GCP + cc]);
        }
        wpart[blk * pairs + pr] = acc;
    }
}

// input gradient, thread per (m, n, c, iy, ix) in the order of x's unit-stride dimension
template <int KS>
__global__ __launch_bounds__(256) void offset_bwd_input_kernel(OffArgs a, const float *__restrict__ dv0,
                                                               const float *__restrict__ dv1, u16 *__restrict__ dx0,
                                                               u16 *__restrict__ dx1) {
    __shared__ float wl[32 * KS * KS];
    const int m = blockIdx.y;
    load_weights<KS>(a, m, wl);
    __syncthreads();
    const long total = (long)a.B * a.G * a.H * a.W * a.gc;
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    int c, ix, iy, n;
    // channel fastest when x is channels-last, or at stride 1 (each pixel gathers up to ks^2
    // cells: coalesced dV reads dominate); else column fastest (coalesced dx stores)
    if (a.sc[m] == 1 || a.stride == 1) {
        c = (int)(e % a.gc);
        long r = e / a.gc;
        ix = (int)(r % a.W);
        r /= a.W;
        iy = (int)(r % a.H);
        n = (int)(r / a.H);
    } else {  // NCHW: column fastest
        ix = (int)(e % a.W);
        long r = e / a.W;
        iy = (int)(r % a.H);
        r /= a.H;
        c = (int)(r % a.gc);
        n = (int)(r / a.gc);
    }
    const float *dv = m ? dv1 : dv0;
    const float *w = wl + c * KS * KS;
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

// dynamic LDS above the 64 KiB default needs the per-kernel opt-in (gfx950: 160 KiB per
// workgroup, static arrays included; those are < 16 KiB here)
static int allow_lds(const void *kernel, size_t bytes) {
    if (bytes <= 64 * 1024) return IRADS_OK;
    if (bytes > 144 * 1024) return IRADS_EINVAL;
    return hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess
               ? IRADS_OK
               : IRADS_EINVAL;
}

template <int GCP, int KS>
size_t smem_bytes(int W) {
    return rows_offset_bytes<GCP, KS>() + (size_t)KS * W * GCP * 2;
}

extern "C" long irads_dattn_offset_partials(int B, int G, int gc, int H, int W, int ks, int stride, int pad) {
    const long hk = (H + 2 * pad - ks) / stride + 1;
    const long nblk = (long)B * G * hk;
    return 2 * nblk * (5 * gc + (long)gc * ks * ks);
}

#define IRADS_OFF_LAUNCH(KERNEL, ...)                                                                             \
    do {                                                                                                         \
        dim3 grid((unsigned)(B * G * a.Hk), 2);                                                                  \
        if (gc <= 16) {                                                                                          \
            IRADS_OFF_KS(ks, {                                                                                   \
                const size_t sm = smem_bytes<16, KS>(W);                                                         \
                IRADS_REQUIRE(allow_lds((const void *)KERNEL<16, KS>, sm) == IRADS_OK,                             \
                              "irads_dattn_offset: row tile %zu B exceeds the LDS (W=%d)", sm, W);               \
                hipLaunchKernelGGL((KERNEL<16, KS>), grid, dim3(256), sm, st, a, __VA_ARGS__);                   \
            });                                                                                                  \
        } else {                                                                                                 \
            IRADS_OFF_KS(ks, {                                                                                   \
                const size_t sm = smem_bytes<32, KS>(W);                                                         \
                IRADS_REQUIRE(allow_lds((const void *)KERNEL<32, KS>, sm) == IRADS_OK,                             \
                              "irads_dattn_offset: row tile %zu B exceeds the LDS (W=%d)", sm, W);               \
                hipLaunchKernelGGL((KERNEL<32, KS>), grid, dim3(256), sm, st, a, __VA_ARGS__);                   \
            });                                                                                                  \
        }                                                                                                        \
    } while (0)

extern "C" int irads_dattn_offset_fwd(const uint16_t *x, const long *x_strides, const uint16_t *y,
                                      const long *y_strides, const float *const *params_x,
                                      const float *const *params_y, const uint16_t *ref, int B, int G, int gc, int H,
                                      int W, int ks, int stride, int pad, float eps, float *pos_x, float *pos_y,
                                      void *stream) {
    OffArgs a;
    int rc = fill_args(a, x, x_strides, y, y_strides, params_x, params_y, ref, B, G, gc, H, W, ks, stride, pad, eps);
    if (rc) return rc;
    IRADS_REQUIRE(pos_x && pos_y, "irads_dattn_offset_fwd: null output");
    hipStream_t st = (hipStream_t)stream;
    IRADS_OFF_LAUNCH(offset_fwd_kernel, pos_x, pos_y);
    return check_launch("irads_dattn_offset_fwd");
}

extern "C" int irads_dattn_offset_bwd(const uint16_t *x, const long *x_strides, const uint16_t *y,
                                      const long *y_strides, const float *const *params_x,
                                      const float *const *params_y, const uint16_t *ref, int B, int G, int gc, int H,
                                      int W, int ks, int stride, int pad, float eps, const float *gpos_x,
                                      const float *gpos_y, float *dv_x, float *dv_y, float *partials, uint16_t *dx,
                                      uint16_t *dy, void *stream) {
    OffArgs a;
    int rc = fill_args(a, x, x_strides, y, y_strides, params_x, params_y, ref, B, G, gc, H, W, ks, stride, pad, eps);
    if (rc) return rc;
    IRADS_REQUIRE(gpos_x && gpos_y && dv_x && dv_y && partials && dx && dy, "irads_dattn_offset_bwd: null");
    IRADS_REQUIRE(a.Wk <= 64, "irads_dattn_offset_bwd: %d key cells per row > 64", a.Wk);
    hipStream_t st = (hipStream_t)stream;
    const long nblk = (long)B * G * a.Hk;
    float *wpart = partials + 2 * nblk * 5 * gc;
    IRADS_OFF_LAUNCH(offset_bwd_cell_kernel, gpos_x, gpos_y, dv_x, dv_y, partials, wpart);
    rc = check_launch("irads_dattn_offset_bwd cells");
    if (rc) return rc;
    const long total = (long)B * G * H * W * gc;
    IRADS_OFF_KS(ks, hipLaunchKernelGGL((offset_bwd_input_kernel<KS>), dim3((unsigned)((total + 255) / 256), 2),
                                        dim3(256), 0, st, a, dv_x, dv_y, dx, dy));
    return check_launch("irads_dattn_offset_bwd input");
}
