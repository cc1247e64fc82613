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
#include <type_traits>

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
// Persistent-chunk design: one workgroup = 9 waves = one head x a contiguous chunk of
// windows (grid ~ one workgroup per CU).  Per workgroup the 36 relative-position biases
// each lane needs are gathered ONCE into registers (pre-scaled by log2 e: softmax runs in
// base 2 with v_exp_f32), so the per-window work is MFMA + a handful of VALU ops per
// score.  K/V (and Q/dO in backward) rows are staged into LDS row-major with plain 16-B
// copies; the transposed MFMA operands (Vᵀ, dOᵀ, Qᵀ, Kᵀ) are read with ds_read_b64_tr_b16.
// The next window's tiles are loaded into registers while the current one computes.
__device__ __forceinline__ f32x4 mfma16(const bf16x8_t &a, const bf16x8_t &b, const f32x4 &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t as_bf(u16x8 v) { return __builtin_bit_cast(bf16x8_t, v); }

typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

// 4 rows x 16 columns block, column-major per lane (cdna_hip_programming.md T10)
__device__ __forceinline__ u16x4 tr_read(const unsigned short *p) {
    return __builtin_bit_cast(u16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4 *)p));
}

__device__ __forceinline__ u16x8 cat4(u16x4 a, u16x4 b) {
    return u16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

constexpr int NR = 160;   // rows incl. zero padding to 5 k-steps of 32
constexpr float LOG2E = 1.4426950408889634f;
// Relative-position biases live in registers as fp16 pairs (pre-scaled by log2 e): abs
// error <= 2^-11 |b|, far below the bf16 rounding the reference's AMP applies to the
// q·kᵀ logits themselves; forward and backward use the same rounded values.
typedef __attribute__((ext_vector_type(2))) _Float16 h2;

struct Chunk {
    int h, w_begin, w_end;
};

__device__ __forceinline__ Chunk decode_chunk(const Geo &g, int cw) {
    const int lid = xcd_remap(blockIdx.x, gridDim.x);  // heads of one chunk on one XCD
    Chunk c;
    c.h = lid % g.nH;
    c.w_begin = (lid / g.nH) * cw;
    c.w_end = min(g.B * g.nW, c.w_begin + cw);
    return c;
}


// class bits of token t inside a boundary window: row / column in the second shift region
__device__ __forceinline__ bool hi_row(const Geo &g, int t) { return t / WS >= WS - g.shift; }
__device__ __forceinline__ bool hi_col(const Geo &g, int t) { return t % WS >= WS - g.shift; }
__device__ __forceinline__ int tok_a(int t) { return 23 * (t / WS) + t % WS; }  // A(t) of the bias index

// Window origin of one (image, window) work item, decoded once per workgroup (the runtime
// divisions by nW / nWw are the expensive part); tok() is then divide-free per token.
struct WinOrigin {
    int r0, c0, base;  // rolled-frame row / column of the window's first token, image token offset
    __device__ __forceinline__ WinOrigin(const Geo &g, int bw) {
        const int b = bw / g.nW, w = bw - b * g.nW;
        const int wr = w / g.nWw;
        r0 = wr * WS;
        c0 = (w - wr * g.nWw) * WS;
        base = b * g.H * g.W;
    }
    __device__ __forceinline__ int tok(const Geo &g, int t) const {
        const int tr = t / WS;  // constant divisor: multiply-shift
        int oh = r0 + tr + g.shift, ow = c0 + (t - tr * WS) + g.shift;
        if (oh >= g.Hp) oh -= g.Hp;
        if (ow >= g.Wp) ow -= g.Wp;
        return (oh < g.H && ow < g.W) ? base + oh * g.W + ow : -1;
    }
};

// ---------------------------------------------------------------------------------------------
// Forward, one workgroup per (window, head): 3 waves, wave w owns query tiles 3w..3w+2.
//
// The relative-position biases come from LDS as the MFMA accumulator seed itself: for a lane's
// query and its 4 consecutive keys (one row of the window, since 4 | 12) the 4 biases are 4
// consecutive entries of the reversed 23x23 table, so the head's table is staged as 16-byte
// quads F[si] = (R[si], R[si+1], R[si+2], R[si+3]) and each seed is ONE ds_read_b128 at a
// per-lane byte offset.  A workgroup is one (window, head); all of its global loads are issued
// up front and retire behind one wait (no load waits on another), 5 workgroups share a CU (LDS
// 31.5 KB, <= 128 VGPRs), so one workgroup's load latency is covered by the others' MFMA /
// softmax work.
//
// Scale folding: the MFMA computes s' = q·k + b / scale on the raw bf16 q (the quads hold the
// table divided by scale), and the softmax runs in base 2 on s'·(scale·log2 e): one fma per
// score turns s' into the exponent, no per-element q·scale pass.  (The reference's AMP rounds
// q·scale to bf16 before the product; here q·k is accumulated in fp32 from the unscaled bf16 q,
// one bf16 rounding closer to the fp32 module.)
constexpr int QF_STRIDE = 28;  // row stride of the (dr, dc) quad grids (23 x 28)
constexpr int QF = 23 * QF_STRIDE;
constexpr int QH = 2 * QF;     // quads per head: forward grid, then backward grid

// quads (nH, QH, 4) fp32, pre-divided by scale.
//   forward, a query's 4 consecutive keys of one window row: F[28 (dr + 11) + (dc + 11)][r] =
//     T[(11 - dr) * 23 + (11 - dc - r)] with dr = row(k) - row(q), dc = col(k0) - col(q).  The row
//     stride 28 (not 23) spreads the 16 lanes of each ds_read_b128 group over the LDS bank slots
//     (1.4-way on average instead of 2.1-way for the 81 (query tile, key tile) pairs).
//   backward (offset QF), a key's 4 consecutive queries of one window row: B[28 (dr + 11) + (dc + 11)][r]
//     = T[(dr + 11) * 23 + (dc + r + 11)] with dr = row(q) - row(k), dc = col(q0) - col(k).
// 0 outside the table.  One launch per (table version, scale).
// After the nH quad grids: each head's table REVERSED and divided by scale, R[e] = T[528 - e] / scale
// (RT floats per head, zero past 528).  A query's seed over 4 consecutive keys of one window row is
// then 4 consecutive entries R[264 + A(k0) - A(q) + r] (A(t) = 23 row(t) + col(t)), and a key's seed
// over 4 consecutive queries is the same 4 entries read backwards from R[264 + A(k) - A(q0)]:
// one 2.1 KB LDS image serves both orientations (the backward kernel winattn_bwd_bf16_rc).
constexpr int RT = 544;
__global__ void winattn_bias_quads_kernel(const float *__restrict__ table, int nH, float inv_scale,
                                          float *__restrict__ quads) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nH * QH * 4) {
        const int j = i - nH * QH * 4;
        if (j >= nH * RT) return;
        const int h = j / RT, e = j % RT;
        quads[i] = e < TBL ? table[(TBL - 1 - e) * nH + h] * inv_scale : 0.f;
        return;
    }
    const int h = i / (QH * 4), e = (i / 4) % QH, r = i % 4;
    const int eg = e < QF ? e : e - QF;
    const int dr = eg / QF_STRIDE - 11, dc = eg % QF_STRIDE - 11;
    int idx;
    if (e < QF) {
        const int tc = 11 - dc - r;
        idx = (dc <= 11 && tc >= 0 && tc < 23) ? (11 - dr) * 23 + tc : -1;
    } else {
        const int tc = dc + r + 11;
        idx = (dc <= 11 && tc >= 0 && tc < 23) ? (dr + 11) * 23 + tc : -1;
    }
    quads[i] = (idx >= 0 && idx < TBL) ? table[idx * nH + h] * inv_scale : 0.f;
}

// K / V tiles of the bf16 forward: 144 rows x 64 B, the four 16-B chunks of row t stored at chunk
// position c ^ kv_swz(t), kv_swz = {0, 2, 3, 1}[(t >> 2) & 3]: conflict-free for the ds_read_b128
// K-fragment reads (each 16-lane group covers all 16 slots of a 256-B bank row) and for the
// ds_read_b64_tr_b16 Vᵀ reads (the 8 rows a half-wave reads land on disjoint 32-B bank spans).
__device__ __forceinline__ int kv_swz(int t) { return (0x78 >> (2 * ((t >> 2) & 3))) & 3; }

// Shift-region class bits of a lane's 36 keys (key tiles kt, keys kt*16 + 4 grp + r, bit kt*4 + r):
// hbits = key row in the second region (k / 12 >= 12 - shift, a threshold on k: the low n bits
// clear), wbits = key column in the second region ((k % 12) >= 12 - shift: the 4 keys of a group
// are one row segment starting at column 4 ((kt + grp) % 3), so the pattern repeats every 3 tiles).
__device__ __forceinline__ void key_class_bits(int shift, int grp, unsigned long long &hbits,
                                               unsigned long long &wbits) {
    const int u = WS * (WS - shift) - 4 * grp;  // keys below the row threshold, counted from this group
    const int n = u <= 0 ? 0 : min(36, 4 * (u >> 4) + min(u & 15, 4));
    hbits = (n >= 64 ? 0ull : (~0ull << n)) & ((1ull << 36) - 1);
    unsigned m[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) m[c] = 0xFu & (0xFu << min(4, max(0, WS - shift - 4 * c)));
    const int g3 = grp % 3;
    const unsigned long long P = m[g3] | (m[(g3 + 1) % 3] << 4) | (m[(g3 + 2) % 3] << 8);
    wbits = P | (P << 12) | (P << 24);
}

// mneg100 where bit j of the mask is set, else 0: sign-extended one-bit field ANDed with the value
__device__ __forceinline__ float mask_term(unsigned long long mbits, int j, float mneg100) {
    const unsigned w = j < 32 ? (unsigned)mbits : (unsigned)(mbits >> 32);
    const int all = __builtin_amdgcn_sbfe((int)w, j & 31, 1);
    return __uint_as_float((unsigned)all & __float_as_uint(mneg100));
}

// wave-uniform "any lane true"
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0ull; }

// bf16 pad-token fragment (the qkv bias, swin.py:186-190) of 8 channels starting at c0
__device__ __forceinline__ u16x8 pad_frag(const float *qbias, int c0) {
    if (!qbias) return u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    const f32x4 a = *(const f32x4 *)(qbias + c0), b = *(const f32x4 *)(qbias + c0 + 4);
    u16x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        r[j] = f2bf(a[j]);
        r[4 + j] = f2bf(b[j]);
    }
    return r;
}

// One (window, head) item of the forward once its Q / K / V tiles are in LDS (Qs, Ks, Vs swizzled
// as kv_swz) and the head's quads in Bq: wave `wave` computes query tiles 3 wave .. 3 wave + 2 and
// writes their O rows (token tok[j], -1 = pad: not written) and base-2 LSE.
template <int MM>
__device__ __forceinline__ void fwd_item(const Geo &g, int bw, int h, const unsigned short *Qs,
                                         const unsigned short *Ks, const unsigned short *Vs, const f32x4 *Bq,
                                         const int (&tok)[3], int wave, int lane, const float *__restrict__ mask,
                                         float c2, unsigned short *__restrict__ out, float *__restrict__ lse) {
    const int l16 = lane & 15, grp = lane >> 4;
    const int swz_l = kv_swz(l16);
    int kofs[9];  // (28 row(k0) + col(k0)) * 16 B
#pragma unroll
    for (int kt = 0; kt < 9; ++kt) {
        const int k0 = kt * 16 + grp * 4;
        kofs[kt] = (QF_STRIDE * (k0 / WS) + k0 % WS) * 16;
    }
    unsigned long long hbits = 0, wbits = 0;
    bool lastH = false, lastW = false;
    if (MM == 1) {
        key_class_bits(g.shift, grp, hbits, wbits);
        const int wi = bw % g.nW;
        lastH = wi / g.nWw == g.nWh - 1;
        lastW = wi % g.nWw == g.nWw - 1;
    }
    const float mneg100 = -100.0f / g.scale;
    const bf16x8_t ones = as_bf(u16x8{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});
    const int vsw = kv_swz(4 * grp), vch = ((l16 & 3) >> 1), vin = (l16 & 1) * 4;
    const int vrow = 4 * grp + (l16 >> 2);
    const unsigned short *vb0 = Vs + vrow * HD + ((vch ^ vsw) * 8) + vin;
    const unsigned short *vb1 = Vs + vrow * HD + (((vch ^ 2) ^ vsw) * 8) + vin;
    const int rfrag = l16 * HD + (grp ^ swz_l) * 8;  // row 16 n + l16, chunk grp
    const char *bqb = (const char *)Bq;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        asm volatile("" ::: "memory");  // re-read the K fragments per tile (no 36-VGPR hoist)
        const int qi = (3 * wave + j) * 16 + l16;
        const bf16x8_t qf = as_bf(*(const u16x8 *)(Qs + (3 * wave + j) * 16 * HD + rfrag));
        const char *bq_q = bqb + (QF_STRIDE * 11 + 11 - (QF_STRIDE * (qi / WS) + qi % WS)) * 16;
        f32x4 s[9];
#pragma unroll
        for (int kt = 0; kt < 9; ++kt) {
            const f32x4 b4 = *(const f32x4 *)(bq_q + kofs[kt]);
            const bf16x8_t kf = as_bf(*(const u16x8 *)(Ks + kt * 16 * HD + rfrag));
            s[kt] = mfma16(kf, qf, b4);
            if (MM == 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    s[kt][r] = fmaf(mask[((long)(bw % g.n_mask) * NT + qi) * NT + kt * 16 + grp * 4 + r], 1.0f / g.scale,
                                    s[kt][r]);
            }
        }
        if (MM == 1 && (lastH || lastW)) {
            unsigned long long mbits = 0;
            if (lastH) mbits |= hi_row(g, qi) ? ~hbits : hbits;
            if (lastW) mbits |= hi_col(g, qi) ? ~wbits : wbits;
#pragma unroll
            for (int kt = 0; kt < 9; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) s[kt][r] += mask_term(mbits, kt * 4 + r, mneg100);
        }
        float mx = s[0][0];
#pragma unroll
        for (int kt = 0; kt < 9; ++kt)
#pragma unroll
            for (int r = (kt == 0); r < 4; ++r) mx = fmaxf(mx, s[kt][r]);
        mx = max_xor16_32(mx);
        const float mneg = -mx * c2;
#pragma unroll
        for (int kt = 0; kt < 9; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[kt][r] = fast_exp2(fmaf(s[kt][r], c2, mneg));
        f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0, os = o0;
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            bf16x8_t pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pb[r] = (__bf16)s[2 * ks][r];
                pb[4 + r] = (2 * ks + 1 < 9) ? (__bf16)s[2 * ks + 1][r] : (__bf16)0.f;
            }
            const int r0 = 32 * ks * HD, r1 = ks < 4 ? r0 + 16 * HD : r0;
            const u16x8 a0 = cat4(tr_read(vb0 + r0), tr_read(vb0 + r1));
            const u16x8 a1 = cat4(tr_read(vb1 + r0), tr_read(vb1 + r1));
            o0 = mfma16(as_bf(a0), pb, o0);
            o1 = mfma16(as_bf(a1), pb, o1);
            os = mfma16(ones, pb, os);
        }
        const float inv = __builtin_amdgcn_rcpf(os[0]);
        if (tok[j] >= 0) {
            u16x4 w0, w1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w0[r] = f2bf(o0[r] * inv);
                w1[r] = f2bf(o1[r] * inv);
            }
            unsigned short *op = out + (long)tok[j] * g.C + h * HD;
            *(u16x4 *)(op + grp * 4) = w0;
            *(u16x4 *)(op + 16 + grp * 4) = w1;
        }
        if (grp == 0) lse[((long)bw * g.nH + h) * NT + qi] = mx * c2 + __log2f(os[0]);
    }
}

// Persistent forward: one workgroup (3 waves) = one head x a contiguous chunk of windows, several
// workgroups per CU.  The next window's q, k, v are loaded into registers while the current one
// computes (the load is issued right after the current window's tiles reach LDS), so each
// workgroup keeps ~27 KB of loads in flight through its whole chunk instead of one
// load-then-compute burst per (window, head).  The head's quads are staged once per workgroup.
template <int MM>
__global__ void __launch_bounds__(192) winattn_fwd_bf16_pc(const unsigned short *__restrict__ qkv, const float *__restrict__ qbias,
                    const float *__restrict__ quads, const float *__restrict__ mask, Geo g, int cw, float c2,
                    unsigned short *__restrict__ out, float *__restrict__ lse) {
    __shared__ __attribute__((aligned(16))) unsigned short Qs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short Ks[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short Vs[NT * HD];
    __shared__ __attribute__((aligned(16))) f32x4 Bq[QF];
    const Chunk ck = decode_chunk(g, cw);
    const int h = ck.h;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, grp = lane >> 4;
    const char *base = (const char *)qkv;
    const unsigned rowb = 6u * (unsigned)g.C, cb = 2u * (unsigned)g.C, hb = (unsigned)(h * HD + grp * 8) * 2u;
    int tok[3];
    u16x8 qreg[3], kreg[3], vreg[3];
    auto prefetch = [&](int bw) {
        const WinOrigin wo(g, bw);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            tok[j] = wo.tok(g, (3 * wave + j) * 16 + l16);
            const unsigned off = (unsigned)max(tok[j], 0) * rowb + hb;
            qreg[j] = *(const u16x8 *)(base + off);
            kreg[j] = *(const u16x8 *)(base + off + cb);
            vreg[j] = *(const u16x8 *)(base + off + 2 * cb);
        }
    };
    if (ck.w_begin >= ck.w_end) return;
    prefetch(ck.w_begin);
    {
        const f32x4 *qsrc = (const f32x4 *)quads + (long)h * QH;
        f32x4 bq[3];
        f32x4 bq4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 3; ++j) bq[j] = qsrc[tid + 192 * j];
        if (tid < QF - 576) bq4 = qsrc[576 + tid];
#pragma unroll
        for (int j = 0; j < 3; ++j) Bq[tid + 192 * j] = bq[j];
        if (tid < QF - 576) Bq[576 + tid] = bq4;
    }
    const int c0 = h * HD + grp * 8;
    const int swz_l = kv_swz(l16);
    for (int bw = ck.w_begin; bw < ck.w_end; ++bw) {
        if (wave_any(tok[0] < 0 || tok[1] < 0 || tok[2] < 0)) {
            const u16x8 qp = pad_frag(qbias, c0), kp = pad_frag(qbias, g.C + c0), vp = pad_frag(qbias, 2 * g.C + c0);
#pragma unroll
            for (int j = 0; j < 3; ++j)
                if (tok[j] < 0) {
                    qreg[j] = qp;
                    kreg[j] = kp;
                    vreg[j] = vp;
                }
        }
        __syncthreads();  // the previous window's tile reads are done
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int o = ((3 * wave + j) * 16 + l16) * HD + (grp ^ swz_l) * 8;
            *(u16x8 *)(Qs + o) = qreg[j];
            *(u16x8 *)(Ks + o) = kreg[j];
            *(u16x8 *)(Vs + o) = vreg[j];
        }
        const int tcur[3] = {tok[0], tok[1], tok[2]};
        __syncthreads();
        if (bw + 1 < ck.w_end) prefetch(bw + 1);
        fwd_item<MM>(g, bw, h, Qs, Ks, Vs, Bq, tcur, wave, lane, mask, c2, out, lse);
    }
}

template <int MM>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(4))) winattn_fwd_bf16_wg(const unsigned short *__restrict__ qkv,
                                                            const float *__restrict__ qbias,
                                                            const float *__restrict__ quads,
                                                            const float *__restrict__ mask, Geo g, float c2,
                                                            unsigned short *__restrict__ out, float *__restrict__ lse) {
    __shared__ __attribute__((aligned(16))) unsigned short Ks[NT * HD];  // swizzled 64-B rows (kv_swz)
    __shared__ __attribute__((aligned(16))) unsigned short Vs[NT * HD];
    __shared__ __attribute__((aligned(16))) f32x4 Bq[QF];  // forward quads of this head
    const int lid = xcd_remap(blockIdx.x, gridDim.x);      // the heads of one window on one XCD
    const int h = lid % g.nH, bw = lid / g.nH;
    const WinOrigin wo(g, bw);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, grp = lane >> 4;
    // ---- every global load of the workgroup first.  Thread (wave, l16, grp) owns tokens
    // t_j = (3 wave + j) 16 + l16 and 16-B chunk grp of their q, k and v: its q rows are exactly
    // its MFMA B fragments, its k / v chunks are staged to LDS.  32-bit byte offsets (< 4 GiB).
    const char *base = (const char *)qkv;
    const unsigned rowb = 6u * (unsigned)g.C, cb = 2u * (unsigned)g.C, hb = (unsigned)(h * HD + grp * 8) * 2u;
    int tok[3];
    u16x8 qreg[3], kreg[3], vreg[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        tok[j] = wo.tok(g, (3 * wave + j) * 16 + l16);
        const unsigned off = (unsigned)max(tok[j], 0) * rowb + hb;
        qreg[j] = *(const u16x8 *)(base + off);
        kreg[j] = *(const u16x8 *)(base + off + cb);
        vreg[j] = *(const u16x8 *)(base + off + 2 * cb);
    }
    f32x4 bq[3];
    f32x4 bq4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 *qsrc = (const f32x4 *)quads + (long)h * QH;
#pragma unroll
    for (int j = 0; j < 3; ++j) bq[j] = qsrc[tid + 192 * j];  // QF = 644 >= 3 * 192
    if (tid < QF - 576) bq4 = qsrc[576 + tid];
    if (wave_any(tok[0] < 0 || tok[1] < 0 || tok[2] < 0)) {  // uniform: only waves holding pad tokens
        const int c0 = h * HD + grp * 8;
        const u16x8 qp = pad_frag(qbias, c0), kp = pad_frag(qbias, g.C + c0), vp = pad_frag(qbias, 2 * g.C + c0);
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (tok[j] < 0) {
                qreg[j] = qp;
                kreg[j] = kp;
                vreg[j] = vp;
            }
    }
    const int swz_l = kv_swz(l16);  // rows t = 16 n + l16 all have the swizzle of l16
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int t = (3 * wave + j) * 16 + l16;
        *(u16x8 *)(Ks + t * HD + (grp ^ swz_l) * 8) = kreg[j];
        *(u16x8 *)(Vs + t * HD + (grp ^ swz_l) * 8) = vreg[j];
        Bq[tid + 192 * j] = bq[j];
    }
    if (tid < QF - 576) Bq[576 + tid] = bq4;
    __syncthreads();
    // ---- per-lane constants: byte offset of the key group of every key tile (keys kt*16 + 4 grp + r,
    // one window row) in the quads, and the key class bits (MM == 1)
    int kofs[9];  // (28 row(k0) + col(k0)) * 16 B
#pragma unroll
    for (int kt = 0; kt < 9; ++kt) {
        const int k0 = kt * 16 + grp * 4;
        kofs[kt] = (QF_STRIDE * (k0 / WS) + k0 % WS) * 16;
    }
    unsigned long long hbits = 0, wbits = 0;
    if (MM == 1) key_class_bits(g.shift, grp, hbits, wbits);
    bool lastH = false, lastW = false;
    if (MM == 1) {
        const int wi = bw % g.nW;
        lastH = wi / g.nWw == g.nWh - 1;
        lastW = wi % g.nWw == g.nWw - 1;
    }
    const float mneg100 = -100.0f / g.scale;  // the region mask in s' units
    const bf16x8_t ones = as_bf(u16x8{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});
    // Vᵀ transposed reads: rows 32 ks + 4 grp + (l16 >> 2) (+16), all with the swizzle of grp; elements
    // 4 (l16 & 3) .. +3 of d-half 0 (chunk (l16 & 3) >> 1) and of d-half 1 (that chunk ^ 2)
    const int vsw = kv_swz(4 * grp), vch = ((l16 & 3) >> 1), vin = (l16 & 1) * 4;
    const int vrow = 4 * grp + (l16 >> 2);
    const unsigned short *vb0 = Vs + vrow * HD + ((vch ^ vsw) * 8) + vin;
    const unsigned short *vb1 = Vs + vrow * HD + (((vch ^ 2) ^ vsw) * 8) + vin;
    const unsigned short *kb = Ks + l16 * HD + (grp ^ swz_l) * 8;
    const char *bqb = (const char *)Bq;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int qi = (3 * wave + j) * 16 + l16;
        const bf16x8_t qf = as_bf(qreg[j]);
        const char *bq_q = bqb + (QF_STRIDE * 11 + 11 - (QF_STRIDE * (qi / WS) + qi % WS)) * 16;  // + key offset
        f32x4 s[9];
#pragma unroll
        for (int kt = 0; kt < 9; ++kt) {
            const f32x4 b4 = *(const f32x4 *)(bq_q + kofs[kt]);
            const bf16x8_t kf = as_bf(*(const u16x8 *)(kb + kt * 16 * HD));
            s[kt] = mfma16(kf, qf, b4);  // s'ᵀ (key rows, query on the lane), bias seeded
            if (MM == 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    s[kt][r] = fmaf(mask[((long)(bw % g.n_mask) * NT + qi) * NT + kt * 16 + grp * 4 + r], 1.0f / g.scale,
                                    s[kt][r]);
            }
        }
        if (MM == 1 && (lastH || lastW)) {  // uniform branch: only edge windows of the shifted grid
            unsigned long long mbits = 0;
            if (lastH) mbits |= hi_row(g, qi) ? ~hbits : hbits;
            if (lastW) mbits |= hi_col(g, qi) ? ~wbits : wbits;
#pragma unroll
            for (int kt = 0; kt < 9; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) s[kt][r] += mask_term(mbits, kt * 4 + r, mneg100);
        }
        float mx = s[0][0];
#pragma unroll
        for (int kt = 0; kt < 9; ++kt)
#pragma unroll
            for (int r = (kt == 0); r < 4; ++r) mx = fmaxf(mx, s[kt][r]);
        mx = max_xor16_32(mx);
        const float mneg = -mx * c2;
#pragma unroll
        for (int kt = 0; kt < 9; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[kt][r] = fast_exp2(fmaf(s[kt][r], c2, mneg));
        f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0, os = o0;
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            bf16x8_t pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pb[r] = (__bf16)s[2 * ks][r];
                pb[4 + r] = (2 * ks + 1 < 9) ? (__bf16)s[2 * ks + 1][r] : (__bf16)0.f;
            }
            // keys 144..159 do not exist: their P is 0, so any finite rows serve (tile 8 again)
            const int r0 = 32 * ks * HD, r1 = ks < 4 ? r0 + 16 * HD : r0;
            const u16x8 a0 = cat4(tr_read(vb0 + r0), tr_read(vb0 + r1));
            const u16x8 a1 = cat4(tr_read(vb1 + r0), tr_read(vb1 + r1));
            o0 = mfma16(as_bf(a0), pb, o0);
            o1 = mfma16(as_bf(a1), pb, o1);
            os = mfma16(ones, pb, os);
        }
        const float inv = __builtin_amdgcn_rcpf(os[0]);
        if (tok[j] >= 0) {
            u16x4 w0, w1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w0[r] = f2bf(o0[r] * inv);
                w1[r] = f2bf(o1[r] * inv);
            }
            unsigned short *op = out + (long)tok[j] * g.C + h * HD;
            *(u16x4 *)(op + grp * 4) = w0;
            *(u16x4 *)(op + 16 + grp * 4) = w1;
        }
        if (grp == 0) lse[((long)bw * g.nH + h) * NT + qi] = mx * c2 + __log2f(os[0]);  // base-2 LSE of s'·scale
    }
}

// As winattn_fwd_bf16_wg with the bias seeds read from the head's reversed table (2.1 KB of LDS
// instead of the 10 KB quad grid): 20.6 KB per workgroup, 6 workgroups per CU (VGPR-bound).
template <int MM>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(4))) winattn_fwd_bf16_rt(const unsigned short *__restrict__ qkv,
                                                            const float *__restrict__ qbias,
                                                            const float *__restrict__ quads,
                                                            const float *__restrict__ mask, Geo g, float c2,
                                                            unsigned short *__restrict__ out, float *__restrict__ lse) {
    __shared__ __attribute__((aligned(16))) unsigned short Ks[NT * HD];  // swizzled 64-B rows (kv_swz)
    __shared__ __attribute__((aligned(16))) unsigned short Vs[NT * HD];
    __shared__ __attribute__((aligned(16))) float Rs[RT];  // reversed, scaled table of this head
    const int lid = xcd_remap(blockIdx.x, gridDim.x);      // the heads of one window on one XCD
    const int h = lid % g.nH, bw = lid / g.nH;
    const WinOrigin wo(g, bw);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, grp = lane >> 4;
    // ---- every global load of the workgroup first.  Thread (wave, l16, grp) owns tokens
    // t_j = (3 wave + j) 16 + l16 and 16-B chunk grp of their q, k and v: its q rows are exactly
    // its MFMA B fragments, its k / v chunks are staged to LDS.  32-bit byte offsets (< 4 GiB).
    const char *base = (const char *)qkv;
    const unsigned rowb = 6u * (unsigned)g.C, cb = 2u * (unsigned)g.C, hb = (unsigned)(h * HD + grp * 8) * 2u;
    int tok[3];
    u16x8 qreg[3], kreg[3], vreg[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        tok[j] = wo.tok(g, (3 * wave + j) * 16 + l16);
        const unsigned off = (unsigned)max(tok[j], 0) * rowb + hb;
        qreg[j] = *(const u16x8 *)(base + off);
        kreg[j] = *(const u16x8 *)(base + off + cb);
        vreg[j] = *(const u16x8 *)(base + off + 2 * cb);
    }
    f32x4 rt = {0.f, 0.f, 0.f, 0.f};
    if (tid < RT / 4) rt = ((const f32x4 *)(quads + (long)g.nH * QH * 4 + (long)h * RT))[tid];
    if (wave_any(tok[0] < 0 || tok[1] < 0 || tok[2] < 0)) {  // uniform: only waves holding pad tokens
        const int c0 = h * HD + grp * 8;
        const u16x8 qp = pad_frag(qbias, c0), kp = pad_frag(qbias, g.C + c0), vp = pad_frag(qbias, 2 * g.C + c0);
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (tok[j] < 0) {
                qreg[j] = qp;
                kreg[j] = kp;
                vreg[j] = vp;
            }
    }
    const int swz_l = kv_swz(l16);  // rows t = 16 n + l16 all have the swizzle of l16
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int t = (3 * wave + j) * 16 + l16;
        *(u16x8 *)(Ks + t * HD + (grp ^ swz_l) * 8) = kreg[j];
        *(u16x8 *)(Vs + t * HD + (grp ^ swz_l) * 8) = vreg[j];
    }
    if (tid < RT / 4) ((f32x4 *)Rs)[tid] = rt;
    __syncthreads();
    // ---- per-lane constants: byte offset of the key group of every key tile (keys kt*16 + 4 grp + r,
    // one window row) in the quads, and the key class bits (MM == 1)
    int part3[3];  // A(16 j + 4 grp); key group of tile 3a + j: part3[j] + 92 a
#pragma unroll
    for (int j = 0; j < 3; ++j) part3[j] = tok_a(16 * j + 4 * grp);
    unsigned long long hbits = 0, wbits = 0;
    if (MM == 1) key_class_bits(g.shift, grp, hbits, wbits);
    bool lastH = false, lastW = false;
    if (MM == 1) {
        const int wi = bw % g.nW;
        lastH = wi / g.nWw == g.nWh - 1;
        lastW = wi % g.nWw == g.nWw - 1;
    }
    const float mneg100 = -100.0f / g.scale;  // the region mask in s' units
    const bf16x8_t ones = as_bf(u16x8{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});
    // Vᵀ transposed reads: rows 32 ks + 4 grp + (l16 >> 2) (+16), all with the swizzle of grp; elements
    // 4 (l16 & 3) .. +3 of d-half 0 (chunk (l16 & 3) >> 1) and of d-half 1 (that chunk ^ 2)
    const int vsw = kv_swz(4 * grp), vch = ((l16 & 3) >> 1), vin = (l16 & 1) * 4;
    const int vrow = 4 * grp + (l16 >> 2);
    const unsigned short *vb0 = Vs + vrow * HD + ((vch ^ vsw) * 8) + vin;
    const unsigned short *vb1 = Vs + vrow * HD + (((vch ^ 2) ^ vsw) * 8) + vin;
    const unsigned short *kb = Ks + l16 * HD + (grp ^ swz_l) * 8;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int qi = (3 * wave + j) * 16 + l16;
        const bf16x8_t qf = as_bf(qreg[j]);
        const float *rq = Rs + 264 - tok_a(qi);  // + A(k0): the seed over keys k0 .. k0 + 3
        f32x4 s[9];
#pragma unroll
        for (int kt = 0; kt < 9; ++kt) {
            const float *rb = rq + part3[kt % 3] + 92 * (kt / 3);
            const f32x4 b4 = {rb[0], rb[1], rb[2], rb[3]};
            const bf16x8_t kf = as_bf(*(const u16x8 *)(kb + kt * 16 * HD));
            s[kt] = mfma16(kf, qf, b4);  // s'ᵀ (key rows, query on the lane), bias seeded
            if (MM == 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    s[kt][r] = fmaf(mask[((long)(bw % g.n_mask) * NT + qi) * NT + kt * 16 + grp * 4 + r], 1.0f / g.scale,
                                    s[kt][r]);
            }
        }
        if (MM == 1 && (lastH || lastW)) {  // uniform branch: only edge windows of the shifted grid
            unsigned long long mbits = 0;
            if (lastH) mbits |= hi_row(g, qi) ? ~hbits : hbits;
            if (lastW) mbits |= hi_col(g, qi) ? ~wbits : wbits;
#pragma unroll
            for (int kt = 0; kt < 9; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) s[kt][r] += mask_term(mbits, kt * 4 + r, mneg100);
        }
        float mx = s[0][0];
#pragma unroll
        for (int kt = 0; kt < 9; ++kt)
#pragma unroll
            for (int r = (kt == 0); r < 4; ++r) mx = fmaxf(mx, s[kt][r]);
        mx = max_xor16_32(mx);
        const float mneg = -mx * c2;
#pragma unroll
        for (int kt = 0; kt < 9; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[kt][r] = fast_exp2(fmaf(s[kt][r], c2, mneg));
        f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0, os = o0;
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            bf16x8_t pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pb[r] = (__bf16)s[2 * ks][r];
                pb[4 + r] = (2 * ks + 1 < 9) ? (__bf16)s[2 * ks + 1][r] : (__bf16)0.f;
            }
            // keys 144..159 do not exist: their P is 0, so any finite rows serve (tile 8 again)
            const int r0 = 32 * ks * HD, r1 = ks < 4 ? r0 + 16 * HD : r0;
            const u16x8 a0 = cat4(tr_read(vb0 + r0), tr_read(vb0 + r1));
            const u16x8 a1 = cat4(tr_read(vb1 + r0), tr_read(vb1 + r1));
            o0 = mfma16(as_bf(a0), pb, o0);
            o1 = mfma16(as_bf(a1), pb, o1);
            os = mfma16(ones, pb, os);
        }
        const float inv = __builtin_amdgcn_rcpf(os[0]);
        if (tok[j] >= 0) {
            u16x4 w0, w1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w0[r] = f2bf(o0[r] * inv);
                w1[r] = f2bf(o1[r] * inv);
            }
            unsigned short *op = out + (long)tok[j] * g.C + h * HD;
            *(u16x4 *)(op + grp * 4) = w0;
            *(u16x4 *)(op + 16 + grp * 4) = w1;
        }
        if (grp == 0) lse[((long)bw * g.nH + h) * NT + qi] = mx * c2 + __log2f(os[0]);  // base-2 LSE of s'·scale
    }
}

// Backward: persistent-chunk workgroups of 9 waves (one head x a contiguous chunk of windows,
// ~one workgroup per CU), phase 1 key-on-lane (s' = q·kᵀ + b/scale, dP = dO·Vᵀ - δ; dVᵀ += dOᵀ·P and
// dKᵀ += qᵀ·dS straight from the accumulators; dS to LDS), phase 2 dQᵀ = Kᵀ·dSᵀ.  The biases are the
// forward's values, seeded into the s' accumulator as there: for a key and 4 consecutive queries of
// one window row they are 4 consecutive table entries, one ds_read_b128 from the head's backward
// quads (the stride-28 (dr, dc) grid) staged once per workgroup.  Q, dO, K and V tiles are 64-B rows
// swizzled as the forward's (kv_swz), dSᵀ rows are 160 bf16 with 8-B pieces XOR-placed by
// ds_swz(row): conflict-free both for the dS stores (key on the lane) and for phase 2's transposed
// reads.  The next window's q, k, v, dO, O and LSE are prefetched into registers while this one
// computes.
// EX: support the optional rel-table / pad-bias gradient accumulators (frozen in IR-ADS's
// Adapter training, so the default instantiation compiles them out)
constexpr int DST = 160;  // dSᵀ row stride (bf16)
__device__ __forceinline__ int ds_swz(int row) { return 4 * ((row >> 1) & 7); }

template <int MM, bool EX>
__global__ void __launch_bounds__(576) winattn_bwd_bf16(
    const unsigned short *__restrict__ qkv, const float *__restrict__ qbias, const float *__restrict__ quads,
    const float *__restrict__ mask, Geo g, int cw, float c2, const unsigned short *__restrict__ out,
    const float *__restrict__ lse,
    const unsigned short *__restrict__ gout, unsigned short *__restrict__ gqkv, float *__restrict__ gtable,
    float *__restrict__ gbias) {
    __shared__ __attribute__((aligned(16))) f32x4 Bf[QF];  // backward quads (stride-28 grid) of this head
    __shared__ __attribute__((aligned(16))) unsigned short Qs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short dOs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short Ks[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short Vs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short dSt[NR * DST];  // dSᵀ: [key][query], keys >= 144 zero
    __shared__ __attribute__((aligned(16))) float lseS[NT], dltS[NT];
    __shared__ int tokS[NT];
    __shared__ __attribute__((aligned(16))) unsigned short padS[3 * HD];  // pad-token q, k, v (bf16)
    __shared__ float tgS[EX ? TBL : 1];  // EX: this workgroup's rel-table gradient, flushed once
    const Chunk ck = decode_chunk(g, cw);
    const int h = ck.h;
    const float mneg100 = -100.0f / g.scale;  // the region mask in s' units
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, grp = lane >> 4;
    {  // the head's backward quads (16-B loads, both issued before either store)
        const f32x4 *src = (const f32x4 *)quads + (long)h * QH + QF;
        const f32x4 b0 = src[tid];
        f32x4 b1 = {0.f, 0.f, 0.f, 0.f};
        if (tid < QF - 576) b1 = src[576 + tid];
        Bf[tid] = b0;
        if (tid < QF - 576) Bf[576 + tid] = b1;
    }
    for (int i = tid; i < (NR - NT) * DST; i += 576) dSt[NT * DST + i] = 0;
    if (EX)
        for (int i = tid; i < TBL; i += 576) tgS[i] = 0.f;
    if (tid < 3 * HD) padS[tid] = qbias ? f2bf(qbias[(tid / HD) * g.C + h * HD + tid % HD]) : (unsigned short)0;
    // ---- lane constants.  Key kkey = 16 wave + l16 on the lane; queries 16 qt + 4 grp + r.
    const int kkey = wave * 16 + l16;
    const int swz_l = kv_swz(l16);
    // bias quad of (kkey, q0 = 16 qt + 4 grp) at 28 (row(q0) - row(k) + 11) + (col(q0) - col(k) + 11);
    // q0 + 48 is 4 rows further, so qt and qt + 3 differ by the constant 4 * 28 quads
    const char *bbase = (const char *)Bf + (QF_STRIDE * 11 + 11 - (QF_STRIDE * (kkey / WS) + kkey % WS)) * 16;
    int qpart[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int q0 = 16 * j + 4 * grp;
        qpart[j] = (QF_STRIDE * (q0 / WS) + q0 % WS) * 16;
    }
    unsigned long long hb = 0, wb = 0;  // query class bits (MM == 1): the forward's key pattern
    if (MM == 1) key_class_bits(g.shift, grp, hb, wb);
    const bool k_hr = kkey >= WS * (WS - g.shift), k_hc = kkey % WS >= WS - g.shift;
    // row-fragment bases (row 16 n + l16, chunk grp) and transposed-read bases (rows 4 grp + (l16 >> 2),
    // 4 elements at 4 (l16 & 3) of d-half 0 / 1), as the forward's
    const int rfrag = l16 * HD + (grp ^ swz_l) * 8;
    const int vsw = kv_swz(4 * grp), vch = ((l16 & 3) >> 1), vin = (l16 & 1) * 4;
    const int trow = (4 * grp + (l16 >> 2)) * HD;
    const int tc0 = ((vch ^ vsw) * 8) + vin, tc1 = (((vch ^ 2) ^ vsw) * 8) + vin;
    const int dsx = ds_swz(kkey);  // this lane's dS row placement
    // phase 2: rows k0 + (l16 >> 2) and + 4 with k0 = 32 ks + 8 grp; dSᵀ columns 16 wave + 4 (l16 & 3)
    const int p2c = wave * 16 + 4 * (l16 & 3);
    const int p2r = 8 * grp + (l16 >> 2);
    const int dsc0 = p2c ^ ds_swz(p2r), dsc1 = p2c ^ ds_swz(p2r + 4);
    const int ksw0 = kv_swz(8 * grp), ksw1 = kv_swz(8 * grp + 4);
    const int kc00 = ((vch ^ ksw0) * 8) + vin, kc01 = (((vch ^ 2) ^ ksw0) * 8) + vin;
    const int kc10 = ((vch ^ ksw1) * 8) + vin, kc11 = (((vch ^ 2) ^ ksw1) * 8) + vin;
    // staging: thread = (token tid / 4, chunk tid % 4)
    const int st_t = tid >> 2, st_ch = tid & 3;
    const int st_off = st_t * HD + (st_ch ^ kv_swz(st_t)) * 8;
    const char *qkvb = (const char *)qkv;
    const unsigned rowb = 6u * (unsigned)g.C, cb = 2u * (unsigned)g.C, orow = 2u * (unsigned)g.C;
    const unsigned hcb = (unsigned)(h * HD + st_ch * 8) * 2u;
    u16x8 qreg, oreg, dreg, kreg, vreg;
    __syncthreads();  // padS, Bf
    float lreg = 0.f;
    int tok_next = -1;
    auto prefetch = [&](int bw) {
        const WinOrigin wo(g, bw);
        const int tok = wo.tok(g, st_t);
        tok_next = tok;
        const unsigned off = (unsigned)max(tok, 0) * rowb + hcb;
        qreg = *(const u16x8 *)(qkvb + off);
        kreg = *(const u16x8 *)(qkvb + off + cb);
        vreg = *(const u16x8 *)(qkvb + off + 2 * cb);
        // pad / cropped tokens read token 0 and are replaced (their dO and O by zero: no gradient)
        const unsigned so = (unsigned)max(tok, 0) * orow + hcb;
        dreg = *(const u16x8 *)((const char *)gout + so);
        oreg = *(const u16x8 *)((const char *)out + so);
        if (tid < NT) lreg = lse[((long)bw * g.nH + h) * NT + tid];
    };
    if (ck.w_begin < ck.w_end) prefetch(ck.w_begin);
    for (int bw = ck.w_begin; bw < ck.w_end; ++bw) {
        if (wave_any(tok_next < 0)) {  // uniform: only waves staging pad tokens
            const u16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
            if (tok_next < 0) {
                qreg = *(const u16x8 *)(padS + st_ch * 8);
                kreg = *(const u16x8 *)(padS + HD + st_ch * 8);
                vreg = *(const u16x8 *)(padS + 2 * HD + st_ch * 8);
                dreg = zero;
                oreg = zero;
            }
        }
        __syncthreads();
        *(u16x8 *)(Qs + st_off) = qreg;  // raw q: the scale is folded into c2, as forward
        *(u16x8 *)(dOs + st_off) = dreg;
        *(u16x8 *)(Ks + st_off) = kreg;
        *(u16x8 *)(Vs + st_off) = vreg;
        {
            float part = 0.f;  // delta_q = dO_q · O_q, 4 lanes per token (stored negated)
#pragma unroll
            for (int j = 0; j < 8; ++j) part = fmaf(bf2f(dreg[j]), bf2f(oreg[j]), part);
            part += __shfl_xor(part, 1, 64);
            part += __shfl_xor(part, 2, 64);
            if (st_ch == 0) {
                dltS[st_t] = -part;
                tokS[st_t] = tok_next;
            }
            if (tid < NT) lseS[tid] = lreg;
        }
        __syncthreads();
        if (bw + 1 < ck.w_end) prefetch(bw + 1);
        unsigned long long mbits = 0;
        bool edge = false;  // uniform: window on the last row / column of the shifted grid
        if (MM == 1) {
            const int wi = bw % g.nW;
            const bool lastH = wi / g.nWw == g.nWh - 1, lastW = wi % g.nWw == g.nWw - 1;
            edge = lastH || lastW;
            if (lastH) mbits |= k_hr ? ~hb : hb;
            if (lastW) mbits |= k_hc ? ~wb : wb;
        }
        // ---------------- phase 1: key tile = wave (key on the lane)
        const bf16x8_t kb = as_bf(*(const u16x8 *)(Ks + wave * 16 * HD + rfrag));
        const bf16x8_t vb = as_bf(*(const u16x8 *)(Vs + wave * 16 * HD + rfrag));
        f32x4 dv0 = {0.f, 0.f, 0.f, 0.f}, dv1 = dv0, dk0 = dv0, dk1 = dv0;
        // two copies of the phase, picked by a uniform branch, so interior windows skip the mask test
        auto phase1 = [&](auto masked) {
        constexpr bool MASKED = decltype(masked)::value;
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            bf16x8_t pb, sb;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const int qt = 2 * ks + half;
                if (qt >= 9) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        pb[4 * half + r] = (__bf16)0.f;
                        sb[4 * half + r] = (__bf16)0.f;
                    }
                    continue;
                }
                const bf16x8_t qa = as_bf(*(const u16x8 *)(Qs + qt * 16 * HD + rfrag));
                const bf16x8_t da = as_bf(*(const u16x8 *)(dOs + qt * 16 * HD + rfrag));
                const f32x4 l4 = *(const f32x4 *)(lseS + qt * 16 + grp * 4);
                const f32x4 nd4 = *(const f32x4 *)(dltS + qt * 16 + grp * 4);
                const f32x4 b4 = *(const f32x4 *)(bbase + qpart[qt % 3] + (qt / 3) * (4 * QF_STRIDE * 16));
                const f32x4 sa = mfma16(qa, kb, b4);   // s'[q][key] = q·k + b / scale, as the forward's s'ᵀ
                const f32x4 dpa = mfma16(da, vb, nd4);  // dP[q][key] - delta_q
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = sa[r];
                    if (MASKED) v += mask_term(mbits, qt * 4 + r, mneg100);
                    if (MM == 2)
                        v = fmaf(mask[((long)(bw % g.n_mask) * NT + qt * 16 + grp * 4 + r) * NT + kkey], 1.0f / g.scale, v);
                    const float p = fast_exp2(fmaf(v, c2, -l4[r]));
                    const float ds = p * dpa[r];
                    pb[4 * half + r] = (__bf16)p;
                    sb[4 * half + r] = (__bf16)ds;
                    if (EX && gtable) atomicAdd(&tgS[rel_idx(qt * 16 + grp * 4 + r, kkey)], ds);  // LDS atomic
                }
                const u16x8 sbits = __builtin_bit_cast(u16x8, sb);
                *(u16x4 *)(dSt + kkey * DST + ((qt * 16 + grp * 4) ^ dsx)) =
                    u16x4{sbits[4 * half], sbits[4 * half + 1], sbits[4 * half + 2], sbits[4 * half + 3]};
            }
            // dVᵀ += dOᵀ·P ; dKᵀ += qᵀ·dS   (k = 32 queries; A via transposed LDS reads; queries
            // 144..159 carry P = dS = 0, so ks = 4 re-reads rows 128..143 for them)
            const int r0 = 32 * ks * HD + trow, r1 = ks < 4 ? r0 + 16 * HD : r0;
            const u16x8 ao0 = cat4(tr_read(dOs + r0 + tc0), tr_read(dOs + r1 + tc0));
            const u16x8 ao1 = cat4(tr_read(dOs + r0 + tc1), tr_read(dOs + r1 + tc1));
            const u16x8 aq0 = cat4(tr_read(Qs + r0 + tc0), tr_read(Qs + r1 + tc0));
            const u16x8 aq1 = cat4(tr_read(Qs + r0 + tc1), tr_read(Qs + r1 + tc1));
            dv0 = mfma16(as_bf(ao0), pb, dv0);
            dv1 = mfma16(as_bf(ao1), pb, dv1);
            dk0 = mfma16(as_bf(aq0), sb, dk0);
            dk1 = mfma16(as_bf(aq1), sb, dk1);
            __builtin_amdgcn_sched_barrier(0);  // keep the next q pair's LDS reads from being hoisted
        }
        };
        if (MM == 1 && edge)
            phase1(std::true_type{});
        else
            phase1(std::false_type{});
        {
            const int tk = tokS[kkey];
            const int c0 = h * HD + grp * 4;
            if (tk >= 0) {
                u16x4 k0, k1, v0, v1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    k0[r] = f2bf(dk0[r] * g.scale);  // dK = scale · dSᵀ·q
                    k1[r] = f2bf(dk1[r] * g.scale);
                    v0[r] = f2bf(dv0[r]);
                    v1[r] = f2bf(dv1[r]);
                }
                unsigned short *gp = gqkv + (long)tk * 3 * g.C;
                *(u16x4 *)(gp + g.C + c0) = k0;
                *(u16x4 *)(gp + g.C + c0 + 16) = k1;
                *(u16x4 *)(gp + 2 * g.C + c0) = v0;
                *(u16x4 *)(gp + 2 * g.C + c0 + 16) = v1;
            } else if (EX && gbias) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    atomicAdd(&gbias[g.C + c0 + r], dk0[r] * g.scale);
                    atomicAdd(&gbias[g.C + c0 + 16 + r], dk1[r] * g.scale);
                    atomicAdd(&gbias[2 * g.C + c0 + r], dv0[r]);
                    atomicAdd(&gbias[2 * g.C + c0 + 16 + r], dv1[r]);
                }
            }
        }
        __syncthreads();
        // ---------------- phase 2: dQᵀ = Kᵀ·dSᵀ for query tile = wave (keys >= 144: dSᵀ rows are zero,
        // K rows 32 lower are read in their place)
        {
            const int qq = wave * 16 + l16;
            f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
            for (int ks = 0; ks < 5; ++ks) {
                const int kr0 = 32 * ks + p2r, kr1 = kr0 + 4;
                const u16x8 bs = cat4(tr_read(dSt + kr0 * DST + dsc0), tr_read(dSt + kr1 * DST + dsc1));
                const int kk0 = (ks == 4 && kr0 >= NT) ? kr0 - 32 : kr0;
                const int kk1 = (ks == 4 && kr1 >= NT) ? kr1 - 32 : kr1;
                const u16x8 ak0 = cat4(tr_read(Ks + kk0 * HD + kc00), tr_read(Ks + kk1 * HD + kc10));
                const u16x8 ak1 = cat4(tr_read(Ks + kk0 * HD + kc01), tr_read(Ks + kk1 * HD + kc11));
                a0 = mfma16(as_bf(ak0), as_bf(bs), a0);
                a1 = mfma16(as_bf(ak1), as_bf(bs), a1);
            }
            const int qtok = tokS[qq];
            const int c0 = h * HD + grp * 4;
            if (qtok >= 0) {
                u16x4 w0, w1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    w0[r] = f2bf(a0[r] * g.scale);
                    w1[r] = f2bf(a1[r] * g.scale);
                }
                *(u16x4 *)(gqkv + (long)qtok * 3 * g.C + c0) = w0;
                *(u16x4 *)(gqkv + (long)qtok * 3 * g.C + c0 + 16) = w1;
            } else if (EX && gbias) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    atomicAdd(&gbias[c0 + r], a0[r] * g.scale);
                    atomicAdd(&gbias[c0 + 16 + r], a1[r] * g.scale);
                }
            }
        }
    }
    if (EX && gtable) {
        __syncthreads();
        for (int i = tid; i < TBL; i += 576) atomicAdd(&gtable[i * g.nH + h], tgS[i]);
    }
}

// Backward, one workgroup (4 waves) per (window, head), ~4 workgroups per CU.  dS never crosses LDS:
// key-tile jobs (key on the lane) form S, dP, P, dS and accumulate dVᵀ += dOᵀ·P, dKᵀ += Qᵀ·dS as
// the persistent kernel's phase 1 does; query-tile jobs (query on the lane, the forward's Sᵀ = K·Qᵀ
// orientation) recompute Sᵀ and dPᵀ and accumulate dQᵀ += Kᵀ·dSᵀ with dSᵀ straight from the
// accumulators (as the forward's Pᵀ feeds Oᵀ).  That costs two more 144x144x32 products and a second
// exp per score, and buys an LDS image of 40 KB (Q, dO, K, V, the reversed bias table, LSE, δ)
// instead of ~100 KB, so 4 workgroups share a CU and hide each other's load latency, with no
// barrier between the two kinds of job.  The 18 jobs (9 key tiles ≈ 38 MFMA each, 9 query tiles
// ≈ 28) are dealt to the 4 waves in fixed lists that are balanced to 93 %.
// EX (trainable table / pad bias) keeps the persistent kernel.
// job lists packed 5 bits a job (count in bits 25..27): kept in scalar registers, no private array
__device__ __forceinline__ unsigned rc_jobs(int wave) {  // job 0..8: key tile, 9..17: query tile job - 9
    constexpr unsigned w0 = 4u << 25 | 0u | 4u << 5 | 8u << 10 | 12u << 15;                // K0 K4 K8 Q3
    constexpr unsigned w1 = 5u << 25 | 1u | 5u << 5 | 9u << 10 | 13u << 15 | 17u << 20;   // K1 K5 Q0 Q4 Q8
    constexpr unsigned w2 = 4u << 25 | 2u | 6u << 5 | 10u << 10 | 14u << 15;               // K2 K6 Q1 Q5
    constexpr unsigned w3 = 5u << 25 | 3u | 7u << 5 | 11u << 10 | 15u << 15 | 16u << 20;  // K3 K7 Q2 Q6 Q7
    return wave == 0 ? w0 : wave == 1 ? w1 : wave == 2 ? w2 : w3;
}


template <int MM>
__global__ void __launch_bounds__(256) winattn_bwd_bf16_rc(
    const unsigned short *__restrict__ qkv, const float *__restrict__ qbias, const float *__restrict__ rtab,
    const float *__restrict__ mask, Geo g, float c2, const unsigned short *__restrict__ out,
    const float *__restrict__ lse, const unsigned short *__restrict__ gout, unsigned short *__restrict__ gqkv) {
    __shared__ __attribute__((aligned(16))) unsigned short Qs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short dOs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short Ks[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short Vs[NT * HD];
    __shared__ __attribute__((aligned(16))) float Rs[RT];
    __shared__ __attribute__((aligned(16))) float lseS[NT], ndS[NT];  // ndS = -δ
    const int lid = xcd_remap(blockIdx.x, gridDim.x);  // the heads of one window on one XCD
    const int h = lid % g.nH, bw = lid / g.nH;
    const WinOrigin wo(g, bw);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, grp = lane >> 4;
    // ---- staging: thread (token t = i / 4, 16-B chunk c = i % 4) for i = tid, tid + 256, tid + 512 (< 576);
    // every load issued before the first use
    const char *qkvb = (const char *)qkv;
    const unsigned rowb = 6u * (unsigned)g.C, cb = 2u * (unsigned)g.C, orow = 2u * (unsigned)g.C;
    u16x8 qr[3], kr[3], vr[3], dr[3], orr[3];
    int tk[3];
    const int nst = wave == 0 ? 3 : 2;  // 576 = 2 x 256 + 64: the third chunk is wave 0's
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (j < nst) {
            const int i = tid + 256 * j, t = i >> 2, c = i & 3;
            tk[j] = wo.tok(g, t);
            const unsigned hcb = (unsigned)(h * HD + c * 8) * 2u;
            const unsigned off = (unsigned)max(tk[j], 0) * rowb + hcb;
            qr[j] = *(const u16x8 *)(qkvb + off);
            kr[j] = *(const u16x8 *)(qkvb + off + cb);
            vr[j] = *(const u16x8 *)(qkvb + off + 2 * cb);
            const unsigned so = (unsigned)max(tk[j], 0) * orow + hcb;
            dr[j] = *(const u16x8 *)((const char *)gout + so);
            orr[j] = *(const u16x8 *)((const char *)out + so);
        }
    }
    f32x4 rt = {0.f, 0.f, 0.f, 0.f};
    if (tid < RT / 4) rt = ((const f32x4 *)(rtab + (long)h * RT))[tid];
    float lv = 0.f;
    if (tid < NT) lv = lse[((long)bw * g.nH + h) * NT + tid];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (j < nst) {
            const int i = tid + 256 * j, t = i >> 2, c = i & 3;
            if (wave_any(tk[j] < 0)) {  // uniform: only waves staging pad tokens
                if (tk[j] < 0) {
                    const int c0 = h * HD + c * 8;
                    const u16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
                    qr[j] = pad_frag(qbias, c0);
                    kr[j] = pad_frag(qbias, g.C + c0);
                    vr[j] = pad_frag(qbias, 2 * g.C + c0);
                    dr[j] = zero;  // a cropped token's output carries no gradient
                    orr[j] = zero;
                }
            }
            const int o = t * HD + (c ^ kv_swz(t)) * 8;
            *(u16x8 *)(Qs + o) = qr[j];  // raw q: the scale is folded into c2, as the forward
            *(u16x8 *)(Ks + o) = kr[j];
            *(u16x8 *)(Vs + o) = vr[j];
            *(u16x8 *)(dOs + o) = dr[j];
            float part = 0.f;  // δ_t = dO_t · O_t, 4 lanes per token
#pragma unroll
            for (int e = 0; e < 8; ++e) part = fmaf(bf2f(dr[j][e]), bf2f(orr[j][e]), part);
            part += __shfl_xor(part, 1, 64);
            part += __shfl_xor(part, 2, 64);
            if (c == 0) ndS[t] = -part;
        }
    }
    if (tid < RT / 4) ((f32x4 *)Rs)[tid] = rt;
    if (tid < NT) lseS[tid] = lv;
    __syncthreads();

    // ---- lane constants shared by both job kinds
    const int swz_l = kv_swz(l16);
    const int rfrag = l16 * HD + (grp ^ swz_l) * 8;  // row fragment: row 16 n + l16, chunk grp
    const int vsw = kv_swz(4 * grp), vch = ((l16 & 3) >> 1), vin = (l16 & 1) * 4;
    const int trow = (4 * grp + (l16 >> 2)) * HD;
    const int tc0 = ((vch ^ vsw) * 8) + vin, tc1 = (((vch ^ 2) ^ vsw) * 8) + vin;  // transposed reads, d-half 0 / 1
    int part3[3];  // A(16 j + 4 grp): A of a 4-token group of tile 3a + j is part3[j] + 92 a
#pragma unroll
    for (int j = 0; j < 3; ++j) part3[j] = tok_a(16 * j + 4 * grp);
    const float mneg100 = -100.0f / g.scale;
    unsigned long long hb = 0, wb = 0;  // class bits of the 36 tokens 16 n + 4 grp + r (MM == 1)
    bool lastH = false, lastW = false;
    if (MM == 1) {
        key_class_bits(g.shift, grp, hb, wb);
        const int wi = bw % g.nW;
        lastH = wi / g.nWw == g.nWh - 1;
        lastW = wi % g.nWw == g.nWw - 1;
    }
    const unsigned jobs = rc_jobs(__builtin_amdgcn_readfirstlane(wave));
    const int njobs = (int)(jobs >> 25);
    for (int jj = 0; jj < njobs; ++jj) {
        const int job = (int)((jobs >> (5 * jj)) & 31u);
        if (job < 9) {
            // ---------------- key tile `job`: key on the lane
            const int kt = job, kkey = kt * 16 + l16;
            const bf16x8_t kb = as_bf(*(const u16x8 *)(Ks + kt * 16 * HD + rfrag));
            const bf16x8_t vb = as_bf(*(const u16x8 *)(Vs + kt * 16 * HD + rfrag));
            // seed of (kkey, queries q0 .. q0 + 3): R[264 + A(k) - A(q0) - r], read backwards
            const float *rk = Rs + 264 + tok_a(kkey) - 3;
            unsigned long long mbits = 0;
            if (MM == 1) {
                const bool k_hr = kkey >= WS * (WS - g.shift), k_hc = kkey % WS >= WS - g.shift;
                if (lastH) mbits |= k_hr ? ~hb : hb;
                if (lastW) mbits |= k_hc ? ~wb : wb;
            }
            f32x4 dv0 = {0.f, 0.f, 0.f, 0.f}, dv1 = dv0, dk0 = dv0, dk1 = dv0;
#pragma unroll
            for (int ks = 0; ks < 5; ++ks) {
                bf16x8_t pb, sb;
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    const int qt = 2 * ks + half;
                    if (qt >= 9) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            pb[4 * half + r] = (__bf16)0.f;
                            sb[4 * half + r] = (__bf16)0.f;
                        }
                        continue;
                    }
                    const bf16x8_t qa = as_bf(*(const u16x8 *)(Qs + qt * 16 * HD + rfrag));
                    const bf16x8_t da = as_bf(*(const u16x8 *)(dOs + qt * 16 * HD + rfrag));
                    const f32x4 l4 = *(const f32x4 *)(lseS + qt * 16 + grp * 4);
                    const f32x4 nd4 = *(const f32x4 *)(ndS + qt * 16 + grp * 4);
                    const float *rb = rk - (part3[qt % 3] + 92 * (qt / 3));
                    const f32x4 b4 = {rb[3], rb[2], rb[1], rb[0]};
                    const f32x4 sa = mfma16(qa, kb, b4);    // s'[q][key] = q·k + b / scale
                    const f32x4 dpa = mfma16(da, vb, nd4);  // dP[q][key] - δ_q
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float v = sa[r];
                        if (MM == 1) v += mask_term(mbits, qt * 4 + r, mneg100);
                        if (MM == 2)
                            v = fmaf(mask[((long)(bw % g.n_mask) * NT + qt * 16 + grp * 4 + r) * NT + kkey], 1.0f / g.scale, v);
                        const float p = fast_exp2(fmaf(v, c2, -l4[r]));
                        pb[4 * half + r] = (__bf16)p;
                        sb[4 * half + r] = (__bf16)(p * dpa[r]);
                    }
                }
                const int r0 = 32 * ks * HD + trow, r1 = ks < 4 ? r0 + 16 * HD : r0;
                const u16x8 ao0 = cat4(tr_read(dOs + r0 + tc0), tr_read(dOs + r1 + tc0));
                const u16x8 ao1 = cat4(tr_read(dOs + r0 + tc1), tr_read(dOs + r1 + tc1));
                const u16x8 aq0 = cat4(tr_read(Qs + r0 + tc0), tr_read(Qs + r1 + tc0));
                const u16x8 aq1 = cat4(tr_read(Qs + r0 + tc1), tr_read(Qs + r1 + tc1));
                dv0 = mfma16(as_bf(ao0), pb, dv0);
                dv1 = mfma16(as_bf(ao1), pb, dv1);
                dk0 = mfma16(as_bf(aq0), sb, dk0);
                dk1 = mfma16(as_bf(aq1), sb, dk1);
            }
            const int tkk = wo.tok(g, kkey);
            if (tkk >= 0) {
                const int c0 = h * HD + grp * 4;
                u16x4 k0, k1, v0, v1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    k0[r] = f2bf(dk0[r] * g.scale);  // dK = scale · dSᵀ·q
                    k1[r] = f2bf(dk1[r] * g.scale);
                    v0[r] = f2bf(dv0[r]);
                    v1[r] = f2bf(dv1[r]);
                }
                unsigned short *gp = gqkv + (long)tkk * 3 * g.C;
                *(u16x4 *)(gp + g.C + c0) = k0;
                *(u16x4 *)(gp + g.C + c0 + 16) = k1;
                *(u16x4 *)(gp + 2 * g.C + c0) = v0;
                *(u16x4 *)(gp + 2 * g.C + c0 + 16) = v1;
            }
        } else {
            // ---------------- query tile `job - 9`: query on the lane (the forward's orientation)
            const int qt = job - 9, qi = qt * 16 + l16;
            const bf16x8_t qf = as_bf(*(const u16x8 *)(Qs + qt * 16 * HD + rfrag));
            const bf16x8_t df = as_bf(*(const u16x8 *)(dOs + qt * 16 * HD + rfrag));
            const float lq = lseS[qi], nd = ndS[qi];
            const f32x4 nd4 = {nd, nd, nd, nd};
            const float *rq = Rs + 264 - tok_a(qi);  // + A(k0): the seed over keys k0 .. k0 + 3
            unsigned long long mbits = 0;
            if (MM == 1) {
                if (lastH) mbits |= hi_row(g, qi) ? ~hb : hb;
                if (lastW) mbits |= hi_col(g, qi) ? ~wb : wb;
            }
            f32x4 dq0 = {0.f, 0.f, 0.f, 0.f}, dq1 = dq0;
#pragma unroll
            for (int ks = 0; ks < 5; ++ks) {
                bf16x8_t sbq;
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    const int kt = 2 * ks + half;
                    if (kt >= 9) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) sbq[4 * half + r] = (__bf16)0.f;
                        continue;
                    }
                    const bf16x8_t kf = as_bf(*(const u16x8 *)(Ks + kt * 16 * HD + rfrag));
                    const bf16x8_t vf = as_bf(*(const u16x8 *)(Vs + kt * 16 * HD + rfrag));
                    const float *rb = rq + part3[kt % 3] + 92 * (kt / 3);
                    const f32x4 b4 = {rb[0], rb[1], rb[2], rb[3]};
                    const f32x4 st = mfma16(kf, qf, b4);    // s'ᵀ[key][q]
                    const f32x4 dpt = mfma16(vf, df, nd4);  // dPᵀ[key][q] - δ_q
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float v = st[r];
                        if (MM == 1) v += mask_term(mbits, kt * 4 + r, mneg100);
                        if (MM == 2)
                            v = fmaf(mask[((long)(bw % g.n_mask) * NT + qi) * NT + kt * 16 + grp * 4 + r], 1.0f / g.scale, v);
                        const float p = fast_exp2(fmaf(v, c2, -lq));
                        sbq[4 * half + r] = (__bf16)(p * dpt[r]);
                    }
                }
                // Kᵀ (d x 32 keys) by transposed reads, keys permuted as dSᵀ's rows (the forward's Vᵀ)
                const int r0 = 32 * ks * HD + trow, r1 = ks < 4 ? r0 + 16 * HD : r0;
                const u16x8 a0 = cat4(tr_read(Ks + r0 + tc0), tr_read(Ks + r1 + tc0));
                const u16x8 a1 = cat4(tr_read(Ks + r0 + tc1), tr_read(Ks + r1 + tc1));
                dq0 = mfma16(as_bf(a0), sbq, dq0);
                dq1 = mfma16(as_bf(a1), sbq, dq1);
            }
            const int tq = wo.tok(g, qi);
            if (tq >= 0) {
                const int c0 = h * HD + grp * 4;
                u16x4 w0, w1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    w0[r] = f2bf(dq0[r] * g.scale);  // dQ = scale · dS·k
                    w1[r] = f2bf(dq1[r] * g.scale);
                }
                *(u16x4 *)(gqkv + (long)tq * 3 * g.C + c0) = w0;
                *(u16x4 *)(gqkv + (long)tq * 3 * g.C + c0 + 16) = w1;
            }
        }
    }
}

int chunk_windows(int total_windows, int nH, long target = 256) {  // target: persistent workgroups
    long cw = ((long)total_windows * nH + target - 1) / target;
    return (int)(cw < 1 ? 1 : cw);
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

extern "C" int irads_winattn_bias_quads(const float *rel_table, int nH, float scale, float *quads, void *stream) {
    IRADS_REQUIRE(rel_table && quads && nH > 0, "irads_winattn_bias_quads: null pointer / nH=%d", nH);
    IRADS_REQUIRE(scale > 0.f, "irads_winattn_bias_quads: scale must be positive (%g)", scale);
    const int n = nH * (QH * 4 + RT);
    winattn_bias_quads_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(rel_table, nH, 1.0f / scale, quads);
    return check_launch("irads_winattn_bias_quads");
}

extern "C" long irads_winattn_bias_quads_size(int nH) { return (long)nH * (QH * 4 + RT); }

extern "C" int irads_winattn_fwd(int dtype, const void *qkv, const float *qkv_bias, const float *rel_table,
                                 const float *bias_quads, const float *mask, int n_mask, int B, int H, int W, int C, int nH, int shift,
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
        IRADS_REQUIRE(bias_quads, "irads_winattn_fwd: bf16 needs bias_quads (irads_winattn_bias_quads)");
        IRADS_REQUIRE(scale > 0.f, "irads_winattn_fwd: scale must be positive (%g)", scale);
        const float c2 = scale * LOG2E;
        static const int pc_wg = [] {  // A/B switch while the persistent variant is measured
            const char *e = getenv("IRADS_WINATTN_FWD_PC");
            return e ? atoi(e) : 0;
        }();
        if (pc_wg > 0) {
            const int cw = chunk_windows(B * g.nW, nH, 256 * pc_wg);
            const unsigned nwg = (unsigned)(((B * g.nW + cw - 1) / cw) * nH);
#define IRADS_WF(M) winattn_fwd_bf16_pc<M><<<nwg, 192, 0, st>>>((const unsigned short *)qkv, qkv_bias, bias_quads, \
                                                                 mask, g, cw, c2, (unsigned short *)out, lse)
            if (mm == 0) IRADS_WF(0); else if (mm == 1) IRADS_WF(1); else IRADS_WF(2);
#undef IRADS_WF
        } else if (pc_wg < 0) {
#define IRADS_WF(M) winattn_fwd_bf16_rt<M><<<nblk, 192, 0, st>>>((const unsigned short *)qkv, qkv_bias, bias_quads, \
                                                                  mask, g, c2, (unsigned short *)out, lse)
            if (mm == 0) IRADS_WF(0); else if (mm == 1) IRADS_WF(1); else IRADS_WF(2);
#undef IRADS_WF
        } else {
#define IRADS_WF(M) winattn_fwd_bf16_wg<M><<<nblk, 192, 0, st>>>((const unsigned short *)qkv, qkv_bias, bias_quads, \
                                                                  mask, g, c2, (unsigned short *)out, lse)
            if (mm == 0) IRADS_WF(0); else if (mm == 1) IRADS_WF(1); else IRADS_WF(2);
#undef IRADS_WF
        }
    }
    return check_launch("irads_winattn_fwd");
}

extern "C" int irads_winattn_bwd(int dtype, const void *qkv, const float *qkv_bias, const float *rel_table,
                                 const float *bias_quads, const float *mask, int n_mask, int B, int H, int W, int C,
                                 int nH, int shift, float scale, const void *out, const float *lse,
                                 const void *grad_out, void *grad_qkv, float *grad_table, float *grad_bias_pad,
                                 void *stream) {
    Geo g;
    if (int e = make_geo(g, dtype, B, H, W, C, nH, shift, scale, mask, n_mask)) return e;
    if (B == 0) return IRADS_OK;
    hipStream_t st = (hipStream_t)stream;
    const unsigned nblk = (unsigned)(B * g.nW * nH);
    const int mm = mask ? 2 : (shift > 0 ? 1 : 0);
    const bool ex = grad_table || grad_bias_pad;
    if (dtype == IRADS_F32) {
        winattn_bwd_f32<<<nblk, 256, 0, st>>>((const float *)qkv, qkv_bias, rel_table, mask, g, (const float *)out,
                                              lse, (const float *)grad_out, (float *)grad_qkv, grad_table,
                                              grad_bias_pad);
    } else {
        IRADS_REQUIRE(bias_quads, "irads_winattn_bwd: bf16 needs bias_quads (irads_winattn_bias_quads)");
        IRADS_REQUIRE(scale > 0.f, "irads_winattn_bwd: scale must be positive (%g)", scale);
        const int cw = chunk_windows(B * g.nW, nH);
        const unsigned nwg = (unsigned)(((B * g.nW + cw - 1) / cw) * nH);
#define IRADS_WB(M, X)                                                                                            \
    winattn_bwd_bf16<M, X><<<nwg, 576, 0, st>>>((const unsigned short *)qkv, qkv_bias, bias_quads, mask, g, cw,   \
                                                scale * LOG2E,                                                    \
                                                (const unsigned short *)out, lse, (const unsigned short *)grad_out, \
                                                (unsigned short *)grad_qkv, grad_table, grad_bias_pad)
        static const int rc = [] {  // A/B switch while the per-item kernel is measured
            const char *e = getenv("IRADS_WINATTN_BWD_RC");
            return e ? atoi(e) : 0;
        }();
        if (ex) {
            if (mm == 0) IRADS_WB(0, true); else if (mm == 1) IRADS_WB(1, true); else IRADS_WB(2, true);
        } else if (rc) {
            const float *rtab = bias_quads + (long)nH * QH * 4;
#define IRADS_WR(M)                                                                                                 \
    winattn_bwd_bf16_rc<M><<<nblk, 256, 0, st>>>((const unsigned short *)qkv, qkv_bias, rtab, mask, g, scale * LOG2E, \
                                                 (const unsigned short *)out, lse, (const unsigned short *)grad_out,    \
                                                 (unsigned short *)grad_qkv)
            if (mm == 0) IRADS_WR(0); else if (mm == 1) IRADS_WR(1); else IRADS_WR(2);
#undef IRADS_WR
        } else {
            if (mm == 0) IRADS_WB(0, false); else if (mm == 1) IRADS_WB(1, false); else IRADS_WB(2, false);
        }
#undef IRADS_WB
    }
    return check_launch("irads_winattn_bwd");
}
