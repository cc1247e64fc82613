// Swin shifted-window attention (W-MSA / SW-MSA) forward and backward for gfx950.
//
// Replaces swin.py:180-254 (ShiftWindowMSA.forward: pad, roll, region mask, partition,
// reverse, un-roll, crop) fused with swin.py:95-116 (WindowMSA core: q*scale·kᵀ +
// relative-position bias + mask, softmax, ·v).  The qkv / proj Linears stay on
// hipBLASLt; this kernel reads the qkv Linear's output in TOKEN order (B, H, W, 3C) and
// writes attention output in token order (B, H, W, C), so the pad/roll/partition copies
// of the reference never touch HBM.  Pad tokens carry q = k = v = qkv bias (the
// reference pads after norm1 and before the Linear, swin.py:186-190 / :90).
//
// One workgroup = one (window, head): 144 tokens x head_dim 32.  Block ids are remapped
// so the heads of one window run on one XCD (shared L2 lines of the 3C-wide token rows).
//
// bf16 path (the training path): 3 waves; MFMA v_mfma_f32_16x16x32_bf16.
//   forward: Sᵀ = K·Qᵀ per 16x16 tile (query on the lane), so each lane owns whole
//   softmax rows (reduced over 4 registers x 9 tiles + 2 xor-shuffles) and the Pᵀ
//   accumulator registers are directly the B operand of Oᵀ = Vᵀ·Pᵀ (k order permuted
//   consistently in Vᵀ's LDS reads) — P never leaves registers.
//   backward: key-on-lane (S = Q·Kᵀ); dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS take P / dS straight
//   from the accumulators; dS crosses LDS once for dQᵀ = Kᵀ·dSᵀ.  LSE from the forward.
// fp32 path (parity / reference-precision mode): exact fp32 VALU kernels, thread per
//   query (dQ) and thread per key (dK, dV).
#include "common.h"

namespace irads {
namespace {

constexpr int WS = 12, NT = 144, HD = 32, TBL = 23 * 23;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;

struct Geo {
    int B, H, W, C, nH, shift, Hp, Wp, nWh, nWw, nW, n_mask;
    float scale;
};

// token t (0..143) of window w -> global token index (or -1 for a pad token) and region id
__device__ __forceinline__ void token_info(const Geo &g, int w, int t, int b, int &tok, int &region) {
    const int wr = w / g.nWw, wc = w % g.nWw;
    const int r = wr * WS + t / WS, c = wc * WS + t % WS;  // rolled (shifted) frame
    int oh = r + g.shift, ow = c + g.shift;
    if (oh >= g.Hp) oh -= g.Hp;
    if (ow >= g.Wp) ow -= g.Wp;
    tok = (oh < g.H && ow < g.W) ? (b * g.H + oh) * g.W + ow : -1;
    if (g.shift > 0) {
        const int hr = r < g.Hp - WS ? 0 : (r < g.Hp - g.shift ? 1 : 2);
        const int wrg = c < g.Wp - WS ? 0 : (c < g.Wp - g.shift ? 1 : 2);
        region = hr * 3 + wrg;
    } else {
        region = 0;
    }
}

__device__ __forceinline__ int rel_idx(int qi, int ki) {
    return (qi / WS - ki / WS + WS - 1) * (2 * WS - 1) + (qi % WS - ki % WS + WS - 1);
}

__device__ __forceinline__ float mask_val(const Geo &g, const float *mask, int wimg, const int *region, int qi, int ki) {
    if (mask) return mask[((long)(wimg % g.n_mask) * NT + qi) * NT + ki];
    if (g.shift > 0 && region[qi] != region[ki]) return -100.0f;
    return 0.0f;
}

__device__ __forceinline__ void decode_block(const Geo &g, int &b, int &w, int &h) {
    const int nwg = gridDim.x;
    const int lid = xcd_remap(blockIdx.x, nwg);
    h = lid % g.nH;
    const int bw = lid / g.nH;
    w = bw % g.nW;
    b = bw / g.nW;
}

// ====================================================================== fp32 path
__global__ void __launch_bounds__(256) winattn_fwd_f32(const float *__restrict__ qkv, const float *__restrict__ qbias,
                                                        const float *__restrict__ table, const float *__restrict__ mask,
                                                        Geo g, float *__restrict__ out, float *__restrict__ lse) {
    __shared__ float Ks[NT][HD + 1], Vs[NT][HD];
    __shared__ float tb[TBL];
    __shared__ int tokS[NT], regS[NT];
    int b, w, h;
    decode_block(g, b, w, h);
    const int C3 = 3 * g.C;
    for (int t = threadIdx.x; t < NT; t += blockDim.x) {
        int tok, reg;
        token_info(g, w, t, b, tok, reg);
        tokS[t] = tok;
        regS[t] = reg;
    }
    for (int i = threadIdx.x; i < TBL; i += blockDim.x) tb[i] = table[i * g.nH + h];
    __syncthreads();
    for (int e = threadIdx.x; e < NT * HD; e += blockDim.x) {
        const int t = e / HD, d = e % HD, tok = tokS[t];
        const int ck = g.C + h * HD + d, cv = 2 * g.C + h * HD + d;
        Ks[t][d] = tok >= 0 ? qkv[(long)tok * C3 + ck] : (qbias ? qbias[ck] : 0.f);
        Vs[t][d] = tok >= 0 ? qkv[(long)tok * C3 + cv] : (qbias ? qbias[cv] : 0.f);
    }
    __syncthreads();
    const int qi = threadIdx.x;
    if (qi >= NT) return;
    const int tok = tokS[qi];
    float q[HD], acc[HD];
    for (int d = 0; d < HD; ++d) {
        const int cq = h * HD + d;
        q[d] = (tok >= 0 ? qkv[(long)tok * C3 + cq] : (qbias ? qbias[cq] : 0.f)) * g.scale;
        acc[d] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int ki = 0; ki < NT; ++ki) {
        float s = 0.f;
        for (int d = 0; d < HD; ++d) s = fmaf(q[d], Ks[ki][d], s);
        s += tb[rel_idx(qi, ki)];
        s += mask_val(g, mask, b * g.nW + w, regS, qi, ki);
        const float mn = fmaxf(m, s);
        const float corr = expf(m - mn), p = expf(s - mn);
        l = l * corr + p;
        for (int d = 0; d < HD; ++d) acc[d] = fmaf(p, Vs[ki][d], acc[d] * corr);
        m = mn;
    }
    const float inv = 1.f / l;
    if (tok >= 0)
        for (int d = 0; d < HD; ++d) out[(long)tok * g.C + h * HD + d] = acc[d] * inv;
    lse[(((long)b * g.nW + w) * g.nH + h) * NT + qi] = m + logf(l);
}

__global__ void __launch_bounds__(256) winattn_bwd_f32(const float *__restrict__ qkv, const float *__restrict__ qbias,
                                                        const float *__restrict__ table, const float *__restrict__ mask,
                                                        Geo g, const float *__restrict__ out, const float *__restrict__ lse,
                                                        const float *__restrict__ gout, float *__restrict__ gqkv,
                                                        float *__restrict__ gtable, float *__restrict__ gbias) {
    __shared__ float Qs[NT][HD + 1], Ks[NT][HD + 1], Vs[NT][HD + 1], dOs[NT][HD + 1];
    __shared__ float tb[TBL], tg[TBL];
    __shared__ float lseS[NT], dlt[NT];
    __shared__ int tokS[NT], regS[NT];
    int b, w, h;
    decode_block(g, b, w, h);
    const int C3 = 3 * g.C;
    const long rowbase = (((long)b * g.nW + w) * g.nH + h) * NT;
    for (int t = threadIdx.x; t < NT; t += blockDim.x) {
        int tok, reg;
        token_info(g, w, t, b, tok, reg);
        tokS[t] = tok;
        regS[t] = reg;
        lseS[t] = lse[rowbase + t];
    }
    for (int i = threadIdx.x; i < TBL; i += blockDim.x) {
        tb[i] = table[i * g.nH + h];
        tg[i] = 0.f;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < NT * HD; e += blockDim.x) {
        const int t = e / HD, d = e % HD, tok = tokS[t];
        const int cq = h * HD + d, ck = g.C + cq, cv = 2 * g.C + cq;
        Qs[t][d] = (tok >= 0 ? qkv[(long)tok * C3 + cq] : (qbias ? qbias[cq] : 0.f)) * g.scale;
        Ks[t][d] = tok >= 0 ? qkv[(long)tok * C3 + ck] : (qbias ? qbias[ck] : 0.f);
        Vs[t][d] = tok >= 0 ? qkv[(long)tok * C3 + cv] : (qbias ? qbias[cv] : 0.f);
        // dO of a pad/cropped token is zero (its output is discarded by the crop, swin.py:248-249)
        dOs[t][d] = tok >= 0 ? gout[(long)tok * g.C + cq] : 0.f;
    }
    __syncthreads();
    // delta_q = dO_q · O_q
    for (int t = threadIdx.x; t < NT; t += blockDim.x) {
        const int tok = tokS[t];
        float s = 0.f;
        if (tok >= 0)
            for (int d = 0; d < HD; ++d) s = fmaf(dOs[t][d], out[(long)tok * g.C + h * HD + d], s);
        dlt[t] = s;
    }
    __syncthreads();
    const int me = threadIdx.x;
    if (me < NT) {
        // pass 1: thread per query -> dQ (and the bias-table gradient)
        const int qi = me;
        float dq[HD];
        for (int d = 0; d < HD; ++d) dq[d] = 0.f;
        for (int ki = 0; ki < NT; ++ki) {
            float s = 0.f, dp = 0.f;
            for (int d = 0; d < HD; ++d) {
                s = fmaf(Qs[qi][d], Ks[ki][d], s);
                dp = fmaf(dOs[qi][d], Vs[ki][d], dp);
            }
            const int ri = rel_idx(qi, ki);
            s += tb[ri] + mask_val(g, mask, b * g.nW + w, regS, qi, ki);
            const float p = expf(s - lseS[qi]);
            const float ds = p * (dp - dlt[qi]);
            for (int d = 0; d < HD; ++d) dq[d] = fmaf(ds, Ks[ki][d], dq[d]);
            if (gtable) atomicAdd(&tg[ri], ds);
        }
        const int tok = tokS[qi];
        for (int d = 0; d < HD; ++d) {
            const float v = dq[d] * g.scale;
            if (tok >= 0)
                gqkv[(long)tok * C3 + h * HD + d] = v;
            else if (gbias)
                atomicAdd(&gbias[h * HD + d], v);
        }
        // pass 2: thread per key -> dK, dV
        const int ki = me;
        float dk[HD], dv[HD];
        for (int d = 0; d < HD; ++d) dk[d] = dv[d] = 0.f;
        for (int qj = 0; qj < NT; ++qj) {
            float s = 0.f, dp = 0.f;
            for (int d = 0; d < HD; ++d) {
                s = fmaf(Qs[qj][d], Ks[ki][d], s);
                dp = fmaf(dOs[qj][d], Vs[ki][d], dp);
            }
            s += tb[rel_idx(qj, ki)] + mask_val(g, mask, b * g.nW + w, regS, qj, ki);
            const float p = expf(s - lseS[qj]);
            const float ds = p * (dp - dlt[qj]);
            for (int d = 0; d < HD; ++d) {
                dv[d] = fmaf(p, dOs[qj][d], dv[d]);
                dk[d] = fmaf(ds, Qs[qj][d], dk[d]);
            }
        }
        const int tk = tokS[ki];
        for (int d = 0; d < HD; ++d) {
            const int ck = g.C + h * HD + d, cv = 2 * g.C + h * HD + d;
            if (tk >= 0) {
                gqkv[(long)tk * C3 + ck] = dk[d];
                gqkv[(long)tk * C3 + cv] = dv[d];
            } else if (gbias) {
                atomicAdd(&gbias[ck], dk[d]);
                atomicAdd(&gbias[cv], dv[d]);
            }
        }
    }
    if (gtable) {
        __syncthreads();
        for (int i = threadIdx.x; i < TBL; i += blockDim.x) atomicAdd(&gtable[i * g.nH + h], tg[i]);
    }
}

// ====================================================================== bf16 MFMA path
__device__ __forceinline__ f32x4 mfma16(const bf16x8_t &a, const bf16x8_t &b, const f32x4 &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t as_bf(u16x8 v) { return __builtin_bit_cast(bf16x8_t, v); }

__device__ __forceinline__ u16x8 bias_frag(const float *qbias, int c0) {
    u16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = qbias ? f2bf(qbias[c0 + j]) : (unsigned short)0;
    return r;
}

__device__ __forceinline__ u16x8 load_frag(const unsigned short *qkv, const float *qbias, int tok, long C3, int c0) {
    if (tok >= 0) return *(const u16x8 *)(qkv + (long)tok * C3 + c0);
    return bias_frag(qbias, c0);
}

constexpr int KROW = 40;   // Ks row stride (bf16): 80 B, conflict-free 16-B reads
constexpr int VTROW = 168; // Vt row stride (forward): keys 0..159 (+8 pad)

// MM: 0 = no mask, 1 = shift-region mask computed in-kernel, 2 = explicit mask tensor
template <int MM>
__global__ void __launch_bounds__(192, 2) winattn_fwd_bf16(const unsigned short *__restrict__ qkv,
                                                         const float *__restrict__ qbias,
                                                         const float *__restrict__ table,
                                                         const float *__restrict__ mask, Geo g,
                                                         unsigned short *__restrict__ out, float *__restrict__ lse) {
    __shared__ __attribute__((aligned(16))) unsigned short Ks[NT * KROW];
    __shared__ __attribute__((aligned(16))) unsigned short Vt[HD * VTROW];
    __shared__ float tb[TBL];
    __shared__ int tokS[NT], kinf[NT];  // kinf = (row*23 + col) | region << 16
    int b, w, h;
    decode_block(g, b, w, h);
    const long C3 = 3 * g.C;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int t = tid; t < NT; t += 192) {
        int tok, reg;
        token_info(g, w, t, b, tok, reg);
        tokS[t] = tok;
        kinf[t] = ((t / WS) * (2 * WS - 1) + t % WS) | (reg << 16);
    }
    for (int i = tid; i < TBL; i += 192) tb[i] = table[i * g.nH + h];
    for (int i = tid; i < HD * (VTROW - NT); i += 192) Vt[(i / (VTROW - NT)) * VTROW + NT + i % (VTROW - NT)] = 0;
    __syncthreads();
    // K rows -> Ks, V rows -> Vt (transposed), 16 B per thread-iteration
    for (int e = tid; e < NT * 4; e += 192) {
        const int t = e >> 2, ch = e & 3, tok = tokS[t];
        const u16x8 kf = load_frag(qkv, qbias, tok, C3, g.C + h * HD + ch * 8);
        const u16x8 vf = load_frag(qkv, qbias, tok, C3, 2 * g.C + h * HD + ch * 8);
        *(u16x8 *)(Ks + t * KROW + ch * 8) = kf;
#pragma unroll
        for (int j = 0; j < 8; ++j) Vt[(ch * 8 + j) * VTROW + t] = vf[j];
    }
    __syncthreads();
    const int l16 = lane & 15, grp = lane >> 4;
    const long rowbase = (((long)b * g.nW + w) * g.nH + h) * NT;
    const bool lastH = (w / g.nWw) == g.nWh - 1, lastW = (w % g.nWw) == g.nWw - 1;
#pragma unroll 1
    for (int qq = 0; qq < 3; ++qq) {
        const int qt = wave * 3 + qq;
        const int qi = qt * 16 + l16;  // this lane's query (column of Sᵀ)
        const int qtok = tokS[qi];
        const bf16x8_t qf = as_bf(load_frag(qkv, qbias, qtok, C3, h * HD + grp * 8));
        const int qinfo = kinf[qi];
        const int qbase = (qinfo & 0xffff) + 264, qreg = qinfo >> 16;
        f32x4 s[9];
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 9; ++kt) {
            const bf16x8_t kf = as_bf(*(const u16x8 *)(Ks + (kt * 16 + l16) * KROW + grp * 8));
            s[kt] = mfma16(kf, qf, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ki = kt * 16 + grp * 4 + r;
                const int kh = ki / WS, kw = ki - kh * WS;  // arithmetic, no LDS round trip
                float v = s[kt][r] * g.scale + tb[qbase - (kh * (2 * WS - 1) + kw)];
                if (MM == 1) {
                    const int hr = lastH ? (kh < WS - g.shift ? 1 : 2) : 0;
                    const int wrg = lastW ? (kw < WS - g.shift ? 1 : 2) : 0;
                    v += (hr * 3 + wrg != qreg) ? -100.0f : 0.0f;
                }
                if (MM == 2) v += mask[((long)((b * g.nW + w) % g.n_mask) * NT + qi) * NT + ki];
                s[kt][r] = v;
                mx = fmaxf(mx, v);
            }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float sum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 9; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = __expf(s[kt][r] - mx);
                s[kt][r] = p;
                sum += p;
            }
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        // Oᵀ = Vᵀ · Pᵀ over 5 k-steps of 32 keys (keys 144..159 are zero)
        f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            bf16x8_t pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pb[r] = (__bf16)s[2 * ks][r];
                pb[4 + r] = (2 * ks + 1 < 9) ? (__bf16)s[2 * ks + 1][r] : (__bf16)0.f;
            }
            const int k0 = 32 * ks + 4 * grp, k1 = k0 + 16;
            u16x8 a0, a1;
            const u16x4 x00 = *(const u16x4 *)(Vt + l16 * VTROW + k0);
            const u16x4 x01 = *(const u16x4 *)(Vt + l16 * VTROW + k1);
            const u16x4 x10 = *(const u16x4 *)(Vt + (16 + l16) * VTROW + k0);
            const u16x4 x11 = *(const u16x4 *)(Vt + (16 + l16) * VTROW + k1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a0[j] = x00[j];
                a0[4 + j] = x01[j];
                a1[j] = x10[j];
                a1[4 + j] = x11[j];
            }
            o0 = mfma16(as_bf(a0), pb, o0);
            o1 = mfma16(as_bf(a1), pb, o1);
        }
        const float inv = 1.f / sum;
        if (qtok >= 0) {
            u16x4 w0, w1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w0[r] = f2bf(o0[r] * inv);
                w1[r] = f2bf(o1[r] * inv);
            }
            unsigned short *op = out + (long)qtok * g.C + h * HD;
            *(u16x4 *)(op + grp * 4) = w0;
            *(u16x4 *)(op + 16 + grp * 4) = w1;
        }
        if (grp == 0) lse[rowbase + qi] = mx + __logf(sum);
    }
}

constexpr int TROW = 152;  // Qt / dOt / Kt / dS row stride (bf16): 304 B, conflict-free

template <int MM>
__global__ void __launch_bounds__(192, 2) winattn_bwd_bf16(
    const unsigned short *__restrict__ qkv, const float *__restrict__ qbias, const float *__restrict__ table,
    const float *__restrict__ mask, Geo g, const unsigned short *__restrict__ out, const float *__restrict__ lse,
    const unsigned short *__restrict__ gout, unsigned short *__restrict__ gqkv, float *__restrict__ gtable,
    float *__restrict__ gbias) {
    __shared__ __attribute__((aligned(16))) unsigned short Qt[HD * TROW];
    __shared__ __attribute__((aligned(16))) unsigned short dOt[HD * TROW];
    __shared__ __attribute__((aligned(16))) unsigned short Kt[HD * TROW];
    __shared__ __attribute__((aligned(16))) unsigned short dS[NT * TROW];
    __shared__ float tb[TBL];
    __shared__ float lseS[NT], dlt[NT];
    __shared__ int tokS[NT], kinf[NT];  // kinf = (row*23 + col) | region << 16
    int b, w, h;
    decode_block(g, b, w, h);
    const long C3 = 3 * g.C;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, grp = lane >> 4;
    const long rowbase = (((long)b * g.nW + w) * g.nH + h) * NT;
    for (int t = tid; t < NT; t += 192) {
        int tok, reg;
        token_info(g, w, t, b, tok, reg);
        tokS[t] = tok;
        kinf[t] = ((t / WS) * (2 * WS - 1) + t % WS) | (reg << 16);
        lseS[t] = lse[rowbase + t];
    }
    for (int i = tid; i < TBL; i += 192) tb[i] = table[i * g.nH + h];
    __syncthreads();
    for (int e = tid; e < NT * 4; e += 192) {
        const int t = e >> 2, ch = e & 3, tok = tokS[t];
        const u16x8 qf = load_frag(qkv, qbias, tok, C3, h * HD + ch * 8);
        const u16x8 kf = load_frag(qkv, qbias, tok, C3, g.C + h * HD + ch * 8);
        u16x8 df;
        if (tok >= 0)
            df = *(const u16x8 *)(gout + (long)tok * g.C + h * HD + ch * 8);
        else
            df = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            Qt[(ch * 8 + j) * TROW + t] = qf[j];
            Kt[(ch * 8 + j) * TROW + t] = kf[j];
            dOt[(ch * 8 + j) * TROW + t] = df[j];
        }
    }
    // delta_q = dO_q · O_q (fp32)
    for (int t = tid; t < NT; t += 192) {
        const int tok = tokS[t];
        float s = 0.f;
        if (tok >= 0) {
            const unsigned short *dp = gout + (long)tok * g.C + h * HD;
            const unsigned short *op = out + (long)tok * g.C + h * HD;
            for (int d = 0; d < HD; ++d) s = fmaf(bf2f(dp[d]), bf2f(op[d]), s);
        }
        dlt[t] = s;
    }
    __syncthreads();
    // ---------------- phase 1: key tiles 3*wave .. 3*wave+2, key on the lane
    bf16x8_t kb[3], vb[3];
    int ktok[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int ki = (wave * 3 + j) * 16 + l16;
        ktok[j] = tokS[ki];
        kb[j] = as_bf(load_frag(qkv, qbias, ktok[j], C3, g.C + h * HD + grp * 8));
        vb[j] = as_bf(load_frag(qkv, qbias, ktok[j], C3, 2 * g.C + h * HD + grp * 8));
    }
    f32x4 dv[3][2], dk[3][2];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) dv[j][dt] = dk[j][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int ks = 0; ks < 5; ++ks) {
        bf16x8_t pb[3], sb[3];
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int qt = 2 * ks + half;
            if (qt >= 9) {
#pragma unroll
                for (int j = 0; j < 3; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        pb[j][4 * half + r] = (__bf16)0.f;
                        sb[j][4 * half + r] = (__bf16)0.f;
                    }
                continue;
            }
            const int qa = qt * 16 + l16;  // A-operand row (query) for this lane
            const int qtokA = tokS[qa];
            const bf16x8_t qf = as_bf(load_frag(qkv, qbias, qtokA, C3, h * HD + grp * 8));
            u16x8 dof;
            if (qtokA >= 0)
                dof = *(const u16x8 *)(gout + (long)qtokA * g.C + h * HD + grp * 8);
            else
                dof = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            const bf16x8_t df = as_bf(dof);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int ki = (wave * 3 + j) * 16 + l16;
                const int kinfo = kinf[ki];
                const int kpos = (kinfo & 0xffff) - 264, kreg = kinfo >> 16;
                f32x4 sa = mfma16(qf, kb[j], f32x4{0.f, 0.f, 0.f, 0.f});  // S[q][key]
                f32x4 da = mfma16(df, vb[j], f32x4{0.f, 0.f, 0.f, 0.f});  // dP[q][key]
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int qi = qt * 16 + grp * 4 + r;
                    const int qinfo = kinf[qi];
                    const int ri = (qinfo & 0xffff) - kpos;
                    float sv = sa[r] * g.scale + tb[ri];
                    if (MM == 1) sv += ((qinfo >> 16) != kreg) ? -100.0f : 0.0f;
                    if (MM == 2) sv += mask[((long)((b * g.nW + w) % g.n_mask) * NT + qi) * NT + ki];
                    const float p = __expf(sv - lseS[qi]);
                    const float ds = p * (da[r] - dlt[qi]);
                    pb[j][4 * half + r] = (__bf16)p;
                    sb[j][4 * half + r] = (__bf16)ds;
                    dS[qi * TROW + ki] = f2bf(ds);
                    if (gtable) atomicAdd(&gtable[ri * g.nH + h], ds);
                }
            }
        }
        // dVᵀ += dOᵀ·P ; dKᵀ += Qᵀ·dS   (k = 32 queries, permuted order shared by A and B)
        const int k0 = 32 * ks + 4 * grp, k1 = k0 + 16;
        const bool second = (k1 < NT);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const int d = dt * 16 + l16;
            u16x8 ao, aq;
            const u16x4 o_a = *(const u16x4 *)(dOt + d * TROW + k0);
            const u16x4 q_a = *(const u16x4 *)(Qt + d * TROW + k0);
            u16x4 o_b = {0, 0, 0, 0}, q_b = {0, 0, 0, 0};
            if (second) {
                o_b = *(const u16x4 *)(dOt + d * TROW + k1);
                q_b = *(const u16x4 *)(Qt + d * TROW + k1);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                ao[j] = o_a[j];
                ao[4 + j] = o_b[j];
                aq[j] = q_a[j];
                aq[4 + j] = q_b[j];
            }
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                dv[j][dt] = mfma16(as_bf(ao), pb[j], dv[j][dt]);
                dk[j][dt] = mfma16(as_bf(aq), sb[j], dk[j][dt]);
            }
        }
    }
    // write dK, dV (lane: 4 consecutive channels of one key)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int tk = ktok[j];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const int c0 = h * HD + dt * 16 + grp * 4;
            if (tk >= 0) {
                u16x4 wk, wv;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    wk[r] = f2bf(dk[j][dt][r] * g.scale);
                    wv[r] = f2bf(dv[j][dt][r]);
                }
                *(u16x4 *)(gqkv + (long)tk * C3 + g.C + c0) = wk;
                *(u16x4 *)(gqkv + (long)tk * C3 + 2 * g.C + c0) = wv;
            } else if (gbias) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    atomicAdd(&gbias[g.C + c0 + r], dk[j][dt][r] * g.scale);
                    atomicAdd(&gbias[2 * g.C + c0 + r], dv[j][dt][r]);
                }
            }
        }
    }
    __syncthreads();
    // ---------------- phase 2: dQᵀ = Kᵀ·dSᵀ for query tiles 3*wave .. 3*wave+2
#pragma unroll 1
    for (int qq = 0; qq < 3; ++qq) {
        const int qt = wave * 3 + qq;
        const int qi = qt * 16 + l16;
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            const int k0 = 32 * ks + 8 * grp;
            u16x8 bs, kt0, kt1;
            if (k0 < NT) {
                bs = *(const u16x8 *)(dS + qi * TROW + k0);
                kt0 = *(const u16x8 *)(Kt + l16 * TROW + k0);
                kt1 = *(const u16x8 *)(Kt + (16 + l16) * TROW + k0);
            } else {
                bs = kt0 = kt1 = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            }
            a0 = mfma16(as_bf(kt0), as_bf(bs), a0);
            a1 = mfma16(as_bf(kt1), as_bf(bs), a1);
        }
        const int qtok = tokS[qi];
        const int c0 = h * HD + grp * 4;
        if (qtok >= 0) {
            u16x4 w0, w1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w0[r] = f2bf(a0[r] * g.scale);
                w1[r] = f2bf(a1[r] * g.scale);
            }
            *(u16x4 *)(gqkv + (long)qtok * C3 + c0) = w0;
            *(u16x4 *)(gqkv + (long)qtok * C3 + c0 + 16) = w1;
        } else if (gbias) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                atomicAdd(&gbias[c0 + r], a0[r] * g.scale);
                atomicAdd(&gbias[c0 + 16 + r], a1[r] * g.scale);
            }
        }
    }
}

int make_geo(Geo &g, int dtype, int B, int H, int W, int C, int nH, int shift, float scale, const float *mask,
             int n_mask) {
    IRADS_REQUIRE(dtype == IRADS_F32 || dtype == IRADS_BF16, "winattn: dtype must be float32 or bfloat16");
    IRADS_REQUIRE(B >= 0 && H > 0 && W > 0 && nH > 0, "winattn: bad sizes");
    IRADS_REQUIRE(C == nH * HD, "winattn: head_dim must be 32 (embed_dims %d, heads %d)", C, nH);
    IRADS_REQUIRE(shift >= 0 && shift < WS, "winattn: shift must be in [0, 12)");
    IRADS_REQUIRE(!mask || n_mask > 0, "winattn: n_mask must be positive with a mask");
    g.B = B;
    g.H = H;
    g.W = W;
    g.C = C;
    g.nH = nH;
    g.shift = shift;
    g.Hp = (H + WS - 1) / WS * WS;
    g.Wp = (W + WS - 1) / WS * WS;
    g.nWh = g.Hp / WS;
    g.nWw = g.Wp / WS;
    g.nW = g.nWh * g.nWw;
    g.n_mask = n_mask;
    g.scale = scale;
    IRADS_REQUIRE((long)B * g.nW * nH < (1L << 31), "winattn: grid too large");
    return IRADS_OK;
}

}  // namespace
}  // namespace irads

using namespace irads;

extern "C" int irads_winattn_fwd(int dtype, const void *qkv, const float *qkv_bias, const float *rel_table,
                                 const float *mask, int n_mask, int B, int H, int W, int C, int nH, int shift,
                                 float scale, void *out, float *lse, void *stream) {
    Geo g;
    if (int e = make_geo(g, dtype, B, H, W, C, nH, shift, scale, mask, n_mask)) return e;
    if (B == 0) return IRADS_OK;
    hipStream_t st = (hipStream_t)stream;
    const unsigned nblk = (unsigned)(B * g.nW * nH);
    if (dtype == IRADS_F32)
        winattn_fwd_f32<<<nblk, 256, 0, st>>>((const float *)qkv, qkv_bias, rel_table, mask, g, (float *)out, lse);
    else
    {
        const int mm = mask ? 2 : (shift > 0 ? 1 : 0);
#define IRADS_WF(M) winattn_fwd_bf16<M><<<nblk, 192, 0, st>>>((const unsigned short *)qkv, qkv_bias, rel_table, mask, \
                                                              g, (unsigned short *)out, lse)
        if (mm == 0) IRADS_WF(0); else if (mm == 1) IRADS_WF(1); else IRADS_WF(2);
#undef IRADS_WF
    }
    return check_launch("irads_winattn_fwd");
}

extern "C" int irads_winattn_bwd(int dtype, const void *qkv, const float *qkv_bias, const float *rel_table,
                                 const float *mask, int n_mask, int B, int H, int W, int C, int nH, int shift,
                                 float scale, const void *out, const float *lse, const void *grad_out, void *grad_qkv,
                                 float *grad_table, float *grad_bias_pad, void *stream) {
    Geo g;
    if (int e = make_geo(g, dtype, B, H, W, C, nH, shift, scale, mask, n_mask)) return e;
    if (B == 0) return IRADS_OK;
    hipStream_t st = (hipStream_t)stream;
    const unsigned nblk = (unsigned)(B * g.nW * nH);
    if (dtype == IRADS_F32)
        winattn_bwd_f32<<<nblk, 256, 0, st>>>((const float *)qkv, qkv_bias, rel_table, mask, g, (const float *)out,
                                              lse, (const float *)grad_out, (float *)grad_qkv, grad_table,
                                              grad_bias_pad);
    else
    {
        const int mm = mask ? 2 : (shift > 0 ? 1 : 0);
#define IRADS_WB(M)                                                                                              \
    winattn_bwd_bf16<M><<<nblk, 192, 0, st>>>((const unsigned short *)qkv, qkv_bias, rel_table, mask, g,         \
                                              (const unsigned short *)out, lse, (const unsigned short *)grad_out, \
                                              (unsigned short *)grad_qkv, grad_table, grad_bias_pad)
        if (mm == 0) IRADS_WB(0); else if (mm == 1) IRADS_WB(1); else IRADS_WB(2);
#undef IRADS_WB
    }
    return check_launch("irads_winattn_bwd");
}
