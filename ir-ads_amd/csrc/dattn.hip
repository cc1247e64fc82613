// DSCF cross-modal deformable attention (DAttentionMM, swin.py:726-1025) for gfx950.
//
// Two kernel families replace the grid_sample / einsum / softmax core (swin.py:911-1016):
//
// 1. Feature sampling (swin.py:911-944): x, y and q (B, C, H, W) sampled at the per-group
//    offset positions pos_x and pos_y (B*G, n, 2; (y, x) order) with bilinear
//    align_corners=True zero padding.  The six reference grid_sample calls become one
//    launch; the sampled tensors are tiny (B, C, 2n).  Corner indices use the CPU
//    grid_sample arithmetic ix = (gx + 1) * ((W-1)/2) (no FMA) — bit-exact with the
//    reference (oracle/csrc/sampling_oracle.c).
//
// 2. Fused attention with an on-the-fly bilinear relative-position bias
//    (swin.py:950-1016): out = softmax(scale·qᵀk + rpe_bias) v over 2n keys per query,
//    where rpe_bias = grid_sample(rpe_table[h] (119x159), 0.5·(q_grid − pos)).  The
//    reference materialises attn (B·h, HW, 2n) and two bias tensors of that size
//    (16.8 M entries per image at stage 0); here one thread owns one query, streams the
//    2n keys from LDS (broadcast reads) with an online softmax, and reads the whole
//    per-head table from LDS (75.7 KB fp32).  head_dim is 8 (Swin-B) / 12 (Swin-L):
//    too small for MFMA, so this is an fp32-VALU-bound kernel.
//    Backward: pass Q (thread per query) recomputes the row and writes dq and
//    delta = dO·O; pass K (thread per key) loops over a query chunk staged in LDS,
//    accumulates dk, dv and d(pos) in registers and the table gradient in LDS
//    (lanes = different keys hit scattered table cells: low atomic contention), then
//    flushes per-workgroup partial sums with one atomic per element.
#include "common.h"

namespace irads {
namespace {

struct Corner {
    int x0, y0;
    float fx, fy, nw, ne, sw, se;
};

// align_corners=True grid_sample arithmetic (CPU reference): ix = (g + 1) * ((size-1)/2)
__device__ __forceinline__ Corner corner_ac(float gx, float gy, int H, int W) {
    Corner c;
    const float sx = ((float)W - 1.0f) / 2.0f, sy = ((float)H - 1.0f) / 2.0f;
    const float ix = (gx + 1.0f) * sx, iy = (gy + 1.0f) * sy;
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    c.x0 = (int)fx0;
    c.y0 = (int)fy0;
    c.fx = ix - fx0;
    c.fy = iy - fy0;
    c.nw = (1.0f - c.fx) * (1.0f - c.fy);
    c.ne = c.fx * (1.0f - c.fy);
    c.sw = (1.0f - c.fx) * c.fy;
    c.se = c.fx * c.fy;
    return c;
}

struct Taps {
    float nw, ne, sw, se;
};

__device__ __forceinline__ Taps taps(const float *plane, int H, int W, const Corner &c) {
    Taps t;
    const bool xl = c.x0 >= 0 && c.x0 < W, xh = c.x0 + 1 >= 0 && c.x0 + 1 < W;
    const bool yl = c.y0 >= 0 && c.y0 < H, yh = c.y0 + 1 >= 0 && c.y0 + 1 < H;
    const long o = (long)c.y0 * W + c.x0;
    t.nw = (yl && xl) ? plane[o] : 0.f;
    t.ne = (yl && xh) ? plane[o + 1] : 0.f;
    t.sw = (yh && xl) ? plane[o + W] : 0.f;
    t.se = (yh && xh) ? plane[o + W + 1] : 0.f;
    return t;
}

__device__ __forceinline__ float interp(const Taps &t, const Corner &c) {
    float v = t.nw * c.nw;
    v = fmaf(t.ne, c.ne, v);
    v = fmaf(t.sw, c.sw, v);
    v = fmaf(t.se, c.se, v);
    return v;
}

__device__ __forceinline__ void scatter(float *plane, int H, int W, const Corner &c, float g) {
    const bool xl = c.x0 >= 0 && c.x0 < W, xh = c.x0 + 1 >= 0 && c.x0 + 1 < W;
    const bool yl = c.y0 >= 0 && c.y0 < H, yh = c.y0 + 1 >= 0 && c.y0 + 1 < H;
    const long o = (long)c.y0 * W + c.x0;
    if (yl && xl) atomicAdd(plane + o, c.nw * g);
    if (yl && xh) atomicAdd(plane + o + 1, c.ne * g);
    if (yh && xl) atomicAdd(plane + o + W, c.sw * g);
    if (yh && xh) atomicAdd(plane + o + W + 1, c.se * g);
}

// ---------------------------------------------------------------- feature sampling
__global__ void dattn_sample_fwd_kernel(const float *__restrict__ x, const float *__restrict__ y,
                                        const float *__restrict__ q, const float *__restrict__ px,
                                        const float *__restrict__ py, int B, int C, int H, int W, int G, int n,
                                        float *__restrict__ xs, float *__restrict__ ys, float *__restrict__ qs) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long total = (long)B * C * 2 * n;
    if (i >= total) return;
    const int j2 = (int)(i % (2 * n));
    const int c = (int)((i / (2 * n)) % C);
    const int b = (int)(i / (2L * n * C));
    const int gc = C / G, gi = c / gc, j = j2 % n;
    const float *pos = (j2 < n ? px : py) + ((long)(b * G + gi) * n + j) * 2;
    const Corner cr = corner_ac(pos[1], pos[0], H, W);  // grid = pos[..., (1, 0)]
    const long plane = ((long)b * C + c) * H * W;
    xs[i] = interp(taps(x + plane, H, W, cr), cr);
    ys[i] = interp(taps(y + plane, H, W, cr), cr);
    qs[i] = interp(taps(q + plane, H, W, cr), cr);
}

__device__ __forceinline__ void dsample(const Taps &t, const Corner &c, float g, float &dix, float &diy) {
    dix += g * ((t.ne - t.nw) * (1.0f - c.fy) + (t.se - t.sw) * c.fy);
    diy += g * ((t.sw - t.nw) * (1.0f - c.fx) + (t.se - t.ne) * c.fx);
}

// thread per (b, group, key, channel-in-group); the GP lanes of one (b, group, key) hold
// its channels, so d(pos) is a shuffle reduction over GP lanes (no atomics on pos)
template <int GP>
__global__ void dattn_sample_bwd_kernel(const float *__restrict__ x, const float *__restrict__ y,
                                        const float *__restrict__ q, const float *__restrict__ px,
                                        const float *__restrict__ py, const float *__restrict__ gxs,
                                        const float *__restrict__ gys, const float *__restrict__ gqs, int B, int C,
                                        int H, int W, int G, int n, float *__restrict__ gx, float *__restrict__ gy,
                                        float *__restrict__ gq, float *__restrict__ gpx, float *__restrict__ gpy) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long total = (long)B * G * 2 * n * GP;
    if (i >= total) return;  // total is a multiple of GP: whole groups exit together
    const int cc = (int)(i % GP);
    const long r = i / GP;
    const int j2 = (int)(r % (2 * n));
    const int gi = (int)((r / (2 * n)) % G);
    const int b = (int)(r / (2L * n * G));
    const int gc = C / G, j = j2 % n;
    const long pidx = ((long)(b * G + gi) * n + j) * 2;
    const float *pos = (j2 < n ? px : py) + pidx;
    const Corner cr = corner_ac(pos[1], pos[0], H, W);
    float dix = 0.f, diy = 0.f;
    if (cc < gc) {
        const int c = gi * gc + cc;
        const long plane = ((long)b * C + c) * H * W;
        const long oi = ((long)b * C + c) * 2 * n + j2;
        const float g1 = gxs[oi], g2 = gys[oi], g3 = gqs[oi];
        dsample(taps(x + plane, H, W, cr), cr, g1, dix, diy);
        dsample(taps(y + plane, H, W, cr), cr, g2, dix, diy);
        dsample(taps(q + plane, H, W, cr), cr, g3, dix, diy);
        scatter(gx + plane, H, W, cr, g1);
        scatter(gy + plane, H, W, cr, g2);
        scatter(gq + plane, H, W, cr, g3);
    }
#pragma unroll
    for (int o = GP / 2; o > 0; o >>= 1) {
        dix += __shfl_xor(dix, o, GP);
        diy += __shfl_xor(diy, o, GP);
    }
    if (cc == 0) {
        float *gp = (j2 < n ? gpx : gpy) + pidx;
        gp[0] = diy * (((float)H - 1.0f) / 2.0f);
        gp[1] = dix * (((float)W - 1.0f) / 2.0f);
    }
}

// ---------------------------------------------------------------- fused attention
struct AttnArgs {
    const float *q, *k, *v, *px, *py, *rpe, *qgy, *qgx;
    int B, nH, G, hc, H, W, n, Ht, Wt;
    float scale;
};

// bias of (query at grid (gy, gx)) for a key at pos (py, px): table sampled at
// 0.5 * (q_grid - pos) (swin.py:983-1007), align_corners=True, zero padding.
__device__ __forceinline__ float rpe_bias(const float *tab, int Ht, int Wt, float qgy, float qgx, float pyk, float pxk,
                                          Corner &cr, Taps &tp) {
    const float dy = (qgy - pyk) * 0.5f, dx = (qgx - pxk) * 0.5f;
    cr = corner_ac(dx, dy, Ht, Wt);
    tp = taps(tab, Ht, Wt, cr);
    return interp(tp, cr);
}

// LDS layout (floats): table[Ht*Wt] | kv[2n][2*HC] (k then v per key) | pos[2n][2]
template <int HC>
__global__ void __launch_bounds__(1024) dattn_attn_fwd_kernel(AttnArgs a, float *__restrict__ out,
                                                              float *__restrict__ lse) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int n2 = 2 * a.n, HW = a.H * a.W, TT = a.Ht * a.Wt;
    float *tab = sm, *kv = sm + TT, *pos = kv + n2 * 2 * HC;
    const int bh = blockIdx.y, b = bh / a.nH, h = bh % a.nH;
    const int gi = h / (a.nH / a.G);
    for (int i = threadIdx.x; i < TT; i += blockDim.x) tab[i] = a.rpe[(long)h * TT + i];
    for (int i = threadIdx.x; i < n2 * HC; i += blockDim.x) {
        const int c = i / n2, j = i % n2;
        kv[j * 2 * HC + c] = a.k[((long)bh * HC + c) * n2 + j];
        kv[j * 2 * HC + HC + c] = a.v[((long)bh * HC + c) * n2 + j];
    }
    for (int j = threadIdx.x; j < n2; j += blockDim.x) {
        const float *p = (j < a.n ? a.px : a.py) + ((long)(b * a.G + gi) * a.n + (j % a.n)) * 2;
        pos[2 * j] = p[0];
        pos[2 * j + 1] = p[1];
    }
    __syncthreads();
    const int qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= HW) return;
    const float qgy = a.qgy[qi / a.W], qgx = a.qgx[qi % a.W];
    float qv[HC], acc[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) {
        qv[c] = a.q[((long)bh * HC + c) * HW + qi];
        acc[c] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int j = 0; j < n2; ++j) {
        const float *kr = kv + j * 2 * HC;
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < HC; ++c) s = fmaf(qv[c], kr[c], s);
        Corner cr;
        Taps tp;
        s = s * a.scale + rpe_bias(tab, a.Ht, a.Wt, qgy, qgx, pos[2 * j], pos[2 * j + 1], cr, tp);
        const float mn = fmaxf(m, s);
        const float corr = __expf(m - mn), p = __expf(s - mn);
        l = l * corr + p;
#pragma unroll
        for (int c = 0; c < HC; ++c) acc[c] = fmaf(p, kr[HC + c], acc[c] * corr);
        m = mn;
    }
    const float inv = 1.f / l;
#pragma unroll
    for (int c = 0; c < HC; ++c) out[((long)bh * HC + c) * HW + qi] = acc[c] * inv;
    lse[(long)bh * HW + qi] = m + __logf(l);
}

// Pass Q (thread per query): dq, delta = dO·O, and the rpe-table gradient.
//  * The table gradient is accumulated per workgroup in LDS in FIXED POINT with integer
//    atomics: on gfx950 ds_add_f32 retires ~0.3 lanes/clk/CU whatever the address
//    pattern, ds_add_u32 ~4 (scripts/microbench/lds_atomic.hip).  The scale is a power of
//    two per workgroup chosen from a bound on its total contribution: for query q,
//    Σ_k |ds_qk| = Σ_k p_qk |dp_qk − δ_q| ≤ |δ_q| + Σ_c |dO_qc| · max_k |v_kc|, and the four
//    bilinear weights of a sample sum to 1, so no cell can exceed B = Σ_q bound_q;
//    scale = 2^(30 − ⌈log2 B⌉) keeps every partial sum inside int32 with a resolution of
//    B·2^-31 (fp32 accumulation of the same sums carries 2^-24 relative error).  Each
//    workgroup flushes its non-zero cells with one float atomic each (consecutive cells:
//    the coalesced atomic pattern).
//  * k, v and the key positions are read with wave-uniform addresses (scalar loads), so
//    LDS holds only the gradient table and two workgroups fit per CU.
__device__ __forceinline__ void scatter_fx(int *tg, int Ht, int Wt, const Corner &cr, float dsq) {
    const bool xl = cr.x0 >= 0 && cr.x0 < Wt, xh = cr.x0 + 1 >= 0 && cr.x0 + 1 < Wt;
    const bool yl = cr.y0 >= 0 && cr.y0 < Ht, yh = cr.y0 + 1 >= 0 && cr.y0 + 1 < Ht;
    const int o = cr.y0 * Wt + cr.x0;
    if (yl && xl) atomicAdd(&tg[o], __float2int_rn(cr.nw * dsq));
    if (yl && xh) atomicAdd(&tg[o + 1], __float2int_rn(cr.ne * dsq));
    if (yh && xl) atomicAdd(&tg[o + Wt], __float2int_rn(cr.sw * dsq));
    if (yh && xh) atomicAdd(&tg[o + Wt + 1], __float2int_rn(cr.se * dsq));
}

__device__ __forceinline__ float block_sum_f(float v, float *red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    float s = 0.f;
    for (int k = 0; k < nw; ++k) s += red[k];
    return s;
}

// LDS: tgrad[TT] (int32 fixed point)
template <int HC>
__global__ void __launch_bounds__(512) dattn_attn_bwd_q_kernel(AttnArgs a, const float *__restrict__ out,
                                                               const float *__restrict__ lse,
                                                               const float *__restrict__ gout,
                                                               float *__restrict__ delta, float *__restrict__ gq,
                                                               float *__restrict__ grpe) {
    extern __shared__ __attribute__((aligned(16))) int tgi[];
    __shared__ float red[8], vmx[8][HC];
    const int n2 = 2 * a.n, HW = a.H * a.W, TT = a.Ht * a.Wt;
    const int bh = blockIdx.y, b = bh / a.nH, h = bh % a.nH;
    const int gi = h / (a.nH / a.G);
    const float *tab = a.rpe + (long)h * TT;
    const float *kb = a.k + (long)bh * HC * n2, *vb = a.v + (long)bh * HC * n2;
    const float *pxb = a.px + (long)(b * a.G + gi) * a.n * 2, *pyb = a.py + (long)(b * a.G + gi) * a.n * 2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < TT; i += blockDim.x) tgi[i] = 0;
    // max_k |v_kc| per channel
    float vm[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) vm[c] = 0.f;
    for (int j = tid; j < n2; j += blockDim.x)
#pragma unroll
        for (int c = 0; c < HC; ++c) vm[c] = fmaxf(vm[c], fabsf(vb[c * n2 + j]));
#pragma unroll
    for (int c = 0; c < HC; ++c) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) vm[c] = fmaxf(vm[c], __shfl_xor(vm[c], o, 64));
        if (lane == 0) vmx[wave][c] = vm[c];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < HC; ++c) {
        vm[c] = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) vm[c] = fmaxf(vm[c], vmx[w][c]);
    }
    const int qi = blockIdx.x * blockDim.x + tid;
    const bool valid = qi < HW;
    float qv[HC], dq[HC], dov[HC];
    float dl = 0.f, bound = 0.f, qgy = 0.f, qgx = 0.f, ls = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c) {
        qv[c] = dov[c] = dq[c] = 0.f;
        if (valid) {
            const long o = ((long)bh * HC + c) * HW + qi;
            qv[c] = a.q[o];
            dov[c] = gout[o];
            dl = fmaf(dov[c], out[o], dl);
        }
    }
    if (valid) {
        qgy = a.qgy[qi / a.W];
        qgx = a.qgx[qi % a.W];
        ls = lse[(long)bh * HW + qi];
        bound = fabsf(dl);
#pragma unroll
        for (int c = 0; c < HC; ++c) bound = fmaf(fabsf(dov[c]), vm[c], bound);
    }
    const float btot = block_sum_f(bound, red);
    // fixed-point scale 2^e with btot·2^e <= 2^30 (exact power of two: scaling and unscaling are exact)
    const int e = (btot > 0.f && btot < 1e30f) ? min(100, 30 - (int)ceilf(log2f(btot))) : 0;
    const float fx = ldexpf(1.f, e), inv_fx = ldexpf(1.f, -e);
    if (valid) {
        for (int j = 0; j < n2; ++j) {
            float kr[HC], s = 0.f, dp = 0.f;
#pragma unroll
            for (int c = 0; c < HC; ++c) {
                kr[c] = kb[c * n2 + j];
                s = fmaf(qv[c], kr[c], s);
                dp = fmaf(dov[c], vb[c * n2 + j], dp);
            }
            const float *pp = (j < a.n ? pxb : pyb) + 2 * (j < a.n ? j : j - a.n);
            Corner cr;
            Taps tp;
            s = s * a.scale + rpe_bias(tab, a.Ht, a.Wt, qgy, qgx, pp[0], pp[1], cr, tp);
            const float p = __expf(s - ls);
            const float ds = p * (dp - dl);
            const float dss = ds * a.scale;
#pragma unroll
            for (int c = 0; c < HC; ++c) dq[c] = fmaf(dss, kr[c], dq[c]);
            scatter_fx(tgi, a.Ht, a.Wt, cr, ds * fx);
        }
#pragma unroll
        for (int c = 0; c < HC; ++c) gq[((long)bh * HC + c) * HW + qi] = dq[c];
        delta[(long)bh * HW + qi] = dl;
    }
    __syncthreads();
    for (int i = tid; i < TT; i += blockDim.x) {
        const int v = tgi[i];
        if (v != 0) atomicAdd(&grpe[(long)h * TT + i], (float)v * inv_fx);
    }
}

constexpr int QCH = 64;  // queries staged per LDS round in pass K

// Pass K (thread per key): loops over a chunk of queries staged in LDS and keeps dk, dv
// and d(pos) of its key in registers (no reduction over lanes).  The bias is recomputed
// from the table through L1/L2; LDS is only the query staging, so several workgroups
// share a CU.  LDS: qst[QCH][2*HC + 4] (q, dO, lse, delta, qgy, qgx)
template <int HC>
__global__ void __launch_bounds__(1024) dattn_attn_bwd_k_kernel(AttnArgs a, const float *__restrict__ lse,
                                                                const float *__restrict__ delta,
                                                                const float *__restrict__ gout, int q_per_block,
                                                                float *__restrict__ gk, float *__restrict__ gv,
                                                                float *__restrict__ gpx, float *__restrict__ gpy) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int n2 = 2 * a.n, HW = a.H * a.W, TT = a.Ht * a.Wt;
    constexpr int QS = 2 * HC + 4;
    float *qst = sm;
    const int bh = blockIdx.y, b = bh / a.nH, h = bh % a.nH;
    const int gi = h / (a.nH / a.G);
    const float *tab = a.rpe + (long)h * TT;
    const int j = threadIdx.x;
    const bool active = j < n2;
    float kr[HC], vr[HC], dk[HC], dv[HC];
    float pyk = 0.f, pxk = 0.f, dpy = 0.f, dpx = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c) kr[c] = vr[c] = dk[c] = dv[c] = 0.f;
    if (active) {
#pragma unroll
        for (int c = 0; c < HC; ++c) {
            kr[c] = a.k[((long)bh * HC + c) * n2 + j];
            vr[c] = a.v[((long)bh * HC + c) * n2 + j];
        }
        const float *p = (j < a.n ? a.px : a.py) + ((long)(b * a.G + gi) * a.n + (j % a.n)) * 2;
        pyk = p[0];
        pxk = p[1];
    }
    const int q_begin = blockIdx.x * q_per_block;
    const int q_end = min(HW, q_begin + q_per_block);
    const float sxt = ((float)a.Wt - 1.0f) / 2.0f, syt = ((float)a.Ht - 1.0f) / 2.0f;
    for (int q0 = q_begin; q0 < q_end; q0 += QCH) {
        const int nq = min(QCH, q_end - q0);
        __syncthreads();
        for (int i = threadIdx.x; i < nq * QS; i += blockDim.x) {
            const int qq = i / QS, f = i % QS, qi = q0 + qq;
            float val;
            if (f < HC)
                val = a.q[((long)bh * HC + f) * HW + qi];
            else if (f < 2 * HC)
                val = gout[((long)bh * HC + (f - HC)) * HW + qi];
            else if (f == 2 * HC)
                val = lse[(long)bh * HW + qi];
            else if (f == 2 * HC + 1)
                val = delta[(long)bh * HW + qi];
            else if (f == 2 * HC + 2)
                val = a.qgy[qi / a.W];
            else
                val = a.qgx[qi % a.W];
            qst[qq * QS + f] = val;
        }
        __syncthreads();
        if (active) {
            for (int qq = 0; qq < nq; ++qq) {
                const float *qs = qst + qq * QS;
                float s = 0.f, dp = 0.f;
#pragma unroll
                for (int c = 0; c < HC; ++c) {
                    s = fmaf(qs[c], kr[c], s);
                    dp = fmaf(qs[HC + c], vr[c], dp);
                }
                Corner cr;
                Taps tp;
                s = s * a.scale + rpe_bias(tab, a.Ht, a.Wt, qs[2 * HC + 2], qs[2 * HC + 3], pyk, pxk, cr, tp);
                const float p = __expf(s - qs[2 * HC]);
                const float ds = p * (dp - qs[2 * HC + 1]);
                const float dss = ds * a.scale;
#pragma unroll
                for (int c = 0; c < HC; ++c) {
                    dk[c] = fmaf(dss, qs[c], dk[c]);
                    dv[c] = fmaf(p, qs[HC + c], dv[c]);
                }
                float dix = 0.f, diy = 0.f;  // d bias / d disp; disp = 0.5 (q_grid - pos)
                dsample(tp, cr, ds, dix, diy);
                dpx -= 0.5f * dix * sxt;
                dpy -= 0.5f * diy * syt;
            }
        }
    }
    if (active) {
#pragma unroll
        for (int c = 0; c < HC; ++c) {
            atomicAdd(&gk[((long)bh * HC + c) * n2 + j], dk[c]);
            atomicAdd(&gv[((long)bh * HC + c) * n2 + j], dv[c]);
        }
        float *gp = (j < a.n ? gpx : gpy) + ((long)(b * a.G + gi) * a.n + (j % a.n)) * 2;
        atomicAdd(gp, dpy);
        atomicAdd(gp + 1, dpx);
    }
}

__global__ void sample_index_kernel(const float *__restrict__ grid, int N, int H, int W, int32_t *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const Corner c = corner_ac(grid[2 * i], grid[2 * i + 1], H, W);
    out[2 * i] = c.x0;
    out[2 * i + 1] = c.y0;
}

int check_attn(const AttnArgs &a) {
    IRADS_REQUIRE(a.B >= 0 && a.nH > 0 && a.G > 0 && a.nH % a.G == 0, "dattn: heads must be a multiple of groups");
    IRADS_REQUIRE(a.H > 0 && a.W > 0 && a.n > 0 && a.Ht > 0 && a.Wt > 0, "dattn: bad sizes");
    IRADS_REQUIRE(2 * a.n <= 1024, "dattn: 2*n_sample must be <= 1024 (got %d)", 2 * a.n);
    IRADS_REQUIRE(a.hc == 2 || a.hc == 4 || a.hc == 8 || a.hc == 12 || a.hc == 16 || a.hc == 24,
                  "dattn: head channels %d unsupported (2, 4, 8, 12, 16, 24)", a.hc);
    return IRADS_OK;
}

size_t fwd_smem(const AttnArgs &a) {
    return ((size_t)a.Ht * a.Wt + (size_t)2 * a.n * 2 * a.hc + (size_t)2 * a.n * 2) * sizeof(float);
}

}  // namespace
}  // namespace irads

using namespace irads;

#define IRADS_HC_DISPATCH(HCV, ...)                  \
    switch (HCV) {                                   \
        case 2: { constexpr int HC = 2; __VA_ARGS__; } break;   \
        case 4: { constexpr int HC = 4; __VA_ARGS__; } break;   \
        case 8: { constexpr int HC = 8; __VA_ARGS__; } break;   \
        case 12: { constexpr int HC = 12; __VA_ARGS__; } break; \
        case 16: { constexpr int HC = 16; __VA_ARGS__; } break; \
        case 24: { constexpr int HC = 24; __VA_ARGS__; } break; \
    }

extern "C" int irads_dattn_sample_fwd(const float *x, const float *y, const float *q, const float *pos_x,
                                      const float *pos_y, int B, int C, int H, int W, int G, int n, float *xs,
                                      float *ys, float *qs, void *stream) {
    IRADS_REQUIRE(B >= 0 && C > 0 && G > 0 && C % G == 0 && n > 0 && H > 0 && W > 0, "dattn_sample: bad sizes");
    const long total = (long)B * C * 2 * n;
    if (total == 0) return IRADS_OK;
    dattn_sample_fwd_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        x, y, q, pos_x, pos_y, B, C, H, W, G, n, xs, ys, qs);
    return check_launch("irads_dattn_sample_fwd");
}

extern "C" int irads_dattn_sample_bwd(const float *x, const float *y, const float *q, const float *pos_x,
                                      const float *pos_y, const float *gxs, const float *gys, const float *gqs, int B,
                                      int C, int H, int W, int G, int n, float *grad_x, float *grad_y, float *grad_q,
                                      float *grad_pos_x, float *grad_pos_y, void *stream) {
    IRADS_REQUIRE(B >= 0 && C > 0 && G > 0 && C % G == 0 && n > 0 && H > 0 && W > 0, "dattn_sample: bad sizes");
    const int gc = C / G;
    IRADS_REQUIRE(gc <= 64, "dattn_sample: group channels %d > 64", gc);
    int GP = 1;
    while (GP < gc) GP <<= 1;
    const long total = (long)B * G * 2 * n * GP;
    if (total == 0) return IRADS_OK;
    const unsigned grid = (unsigned)((total + 255) / 256);
    hipStream_t st = (hipStream_t)stream;
#define IRADS_SB(P)                                                                                             \
    case P:                                                                                                     \
        dattn_sample_bwd_kernel<P><<<grid, 256, 0, st>>>(x, y, q, pos_x, pos_y, gxs, gys, gqs, B, C, H, W, G, n, \
                                                         grad_x, grad_y, grad_q, grad_pos_x, grad_pos_y);       \
        break;
    switch (GP) { IRADS_SB(1) IRADS_SB(2) IRADS_SB(4) IRADS_SB(8) IRADS_SB(16) IRADS_SB(32) IRADS_SB(64) }
#undef IRADS_SB
    return check_launch("irads_dattn_sample_bwd");
}

static int attn_block(int HW) {
    int t = ((HW + 63) / 64) * 64;
    return t > 1024 ? 1024 : t;
}

extern "C" int irads_dattn_attn_fwd(const float *q, const float *k, const float *v, const float *pos_x,
                                    const float *pos_y, const float *rpe, const float *qgrid_y, const float *qgrid_x,
                                    int B, int nH, int G, int hc, int H, int W, int n, int Ht, int Wt, float scale,
                                    float *out, float *lse, void *stream) {
    AttnArgs a{q, k, v, pos_x, pos_y, rpe, qgrid_y, qgrid_x, B, nH, G, hc, H, W, n, Ht, Wt, scale};
    if (int e = check_attn(a)) return e;
    if (B == 0) return IRADS_OK;
    const size_t sh = fwd_smem(a);
    IRADS_REQUIRE(sh <= 160 * 1024, "dattn_attn: LDS request %zu exceeds 160 KiB", sh);
    const int HW = H * W, bs = attn_block(HW);
    dim3 grid((HW + bs - 1) / bs, B * nH);
    hipStream_t st = (hipStream_t)stream;
    IRADS_HC_DISPATCH(hc, {
        (void)hipFuncSetAttribute((const void *)dattn_attn_fwd_kernel<HC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sh);
        dattn_attn_fwd_kernel<HC><<<grid, bs, sh, st>>>(a, out, lse);
    })
    return check_launch("irads_dattn_attn_fwd");
}

extern "C" int irads_dattn_attn_bwd(const float *q, const float *k, const float *v, const float *pos_x,
                                    const float *pos_y, const float *rpe, const float *qgrid_y, const float *qgrid_x,
                                    int B, int nH, int G, int hc, int H, int W, int n, int Ht, int Wt, float scale,
                                    const float *out, const float *lse, const float *grad_out, float *delta,
                                    float *grad_q, float *grad_k, float *grad_v, float *grad_rpe, float *grad_pos_x,
                                    float *grad_pos_y, void *stream) {
    AttnArgs a{q, k, v, pos_x, pos_y, rpe, qgrid_y, qgrid_x, B, nH, G, hc, H, W, n, Ht, Wt, scale};
    if (int e = check_attn(a)) return e;
    if (B == 0) return IRADS_OK;
    hipStream_t st = (hipStream_t)stream;
    const int HW = H * W;
    const size_t sh_q = (size_t)Ht * Wt * sizeof(int);
    const size_t sh_k = (size_t)QCH * (2 * hc + 4) * sizeof(float);
    IRADS_REQUIRE(sh_q <= 160 * 1024 && sh_k <= 160 * 1024, "dattn_attn_bwd: LDS request exceeds 160 KiB");
    // pass Q: 512 queries per workgroup, or 256 when that leaves the chip under-filled
    const int bs = ((long)((HW + 511) / 512) * B * nH >= 512) ? 512 : 256;
    dim3 gq_grid((HW + bs - 1) / bs, B * nH);
    // pass K: one thread per key; enough query chunks per (b, h) to fill the chip
    const int kthreads = ((2 * n + 63) / 64) * 64;
    int qpb = 1024;
    while (qpb > QCH && (long)((HW + qpb - 1) / qpb) * B * nH < 1024) qpb /= 2;
    dim3 gk_grid((HW + qpb - 1) / qpb, B * nH);
    IRADS_HC_DISPATCH(hc, {
        (void)hipFuncSetAttribute((const void *)dattn_attn_bwd_q_kernel<HC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)sh_q);
        dattn_attn_bwd_q_kernel<HC><<<gq_grid, bs, sh_q, st>>>(a, out, lse, grad_out, delta, grad_q, grad_rpe);
        dattn_attn_bwd_k_kernel<HC><<<gk_grid, kthreads, sh_k, st>>>(a, lse, delta, grad_out, qpb, grad_k, grad_v,
                                                                     grad_pos_x, grad_pos_y);
    })
    return check_launch("irads_dattn_attn_bwd");
}

extern "C" int irads_dattn_sample_index(const float *grid, int N, int H, int W, int32_t *corners, void *stream) {
    IRADS_REQUIRE(N >= 0 && H > 0 && W > 0, "dattn_sample_index: bad sizes");
    if (N == 0) return IRADS_OK;
    sample_index_kernel<<<(N + 255) / 256, 256, 0, (hipStream_t)stream>>>(grid, N, H, W, corners);
    return check_launch("irads_dattn_sample_index");
}
