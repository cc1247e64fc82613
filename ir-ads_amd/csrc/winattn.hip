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
// Block ids are remapped so the heads of one window run on one XCD (shared L2 lines of the
// 3C-wide token rows).
//
// bf16 path (the training path): MFMA v_mfma_f32_16x16x32_bf16.
//   forward: Sᵀ = K·Qᵀ per 16x16 tile (query on the lane), so each lane owns whole softmax rows
//   and the Pᵀ accumulator registers are directly the B operand of Oᵀ = Vᵀ·Pᵀ (k order permuted
//   consistently in Vᵀ's LDS reads) — P never leaves registers.
//   backward: key-on-lane (S = Q·Kᵀ); dVᵀ += dOᵀ·P and dKᵀ += Qᵀ·dS take P / dS straight
//   from the accumulators; dS crosses LDS once for dQᵀ = Kᵀ·dSᵀ.  LSE from the forward.
// fp32 path (parity / reference-precision mode): exact fp32 VALU kernels, thread per
//   query (dQ) and thread per key (dK, dV).
#include "common.h"
#include <type_traits>
#include <cstdlib>
#include <cstring>

namespace irads {
namespace {

constexpr int WS = 12, NT = 144, HD = 32, TBL = 23 * 23;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;

struct Geo {
    int B, H, W, C, nH, shift, Hp, Wp, nWh, nWw, nW, n_mask;
    float scale;
    unsigned long long *stamp;  // irads_stamp_next's slot for this launch, or null
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
// Forward: one 3-wave workgroup per (window, head), ~6 per CU; backward: persistent 9-wave
// workgroups over a chunk of windows of one head.  K/V (and Q/dO in backward) rows are staged into
// LDS row-major with plain 16-B copies; the transposed MFMA operands (Vᵀ, dOᵀ, Qᵀ, Kᵀ) are read
// with ds_read_b64_tr_b16.  Scores are in base-2 units: q is rounded to bf16(q·scale·log2 e) when
// staged and the bias table is seeded as T·log2 e, so the softmax is v_exp_f32 of the MFMA output.
__device__ __forceinline__ f32x4 mfma16(const bf16x8_t &a, const bf16x8_t &b, const f32x4 &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t as_bf(u16x8 v) { return __builtin_bit_cast(bf16x8_t, v); }

typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
// fp32 -> bf16 (round to nearest even, as f2bf) as whole vectors: one v_cvt_pk_bf16_f32 per PAIR.
// Element-by-element f2bf made hipcc convert every value alone and v_perm the halves together
// (108 cvt + 54 perm per lane in the forward instead of 54 cvt).
__device__ __forceinline__ bf16x8_t pack_bf16(f32x4 lo, f32x4 hi) {
    return __builtin_convertvector((f32x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]}, bf16x8_t);
}
__device__ __forceinline__ u16x4 pack_bf16x4(f32x4 v) {
    return __builtin_bit_cast(u16x4, __builtin_convertvector(v, bf16x4_t));
}

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
typedef __attribute__((ext_vector_type(2))) float f2v;

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
// Relative-position biases enter both directions as the MFMA accumulator seed: for one query and 4
// consecutive keys of one window row (or one key and 4 consecutive queries) the 4 biases are 4
// consecutive entries of a (reversed) 23x23 table, so each seed is ONE 16-B LDS read.
//
// Bias buffer per head (irads_winattn_bias_quads; one launch per (table version, scale)): two grids
// of 16-B quads, fp32 and divided by scale (the kernels multiply by c2 = scale·log2 e while staging,
// giving T·log2 e).  A 4-token group always starts at column 0, 4 or 8 of a window row, so the
// column offset dc lies in [-11, 8] and a grid is 23 rows of QF_STRIDE = 20 quads:
//   [0, QB)   forward, a query's 4 consecutive keys k0 .. k0 + 3 of one window row:
//             F[20 (dr + 11) + (dc + 11)][r] = T[(11 - dr) * 23 + (11 - dc - r)],
//             dr = row(k0) - row(q), dc = col(k0) - col(q);
//   [QB, 2QB) backward, a key's 4 consecutive queries q0 .. q0 + 3 of one window row:
//             B[20 (dr + 11) + (dc + 11)][r] = T[(dr + 11) * 23 + (dc + r + 11)],
//             dr = row(q0) - row(k), dc = col(q0) - col(k).
// Row stride 20: the smallest grid on which the 16 lanes of each ds_read_b128 group spread over
// the bank slots as well as any injective linear layout does (5.8 LDS cycles per read against 4
// conflict-free, over all 81 (query tile, key tile) pairs; searched exhaustively with the lane
// groups of MI355X_MICROARCH.md §LDS), in 7.4 KB per grid.
constexpr int QF_STRIDE = 20;
constexpr int QB = 23 * QF_STRIDE;  // quads per grid
constexpr int QH = 8 * QB;          // floats per head (both grids)

__global__ void winattn_bias_quads_kernel(const float *__restrict__ table, int nH, float inv_scale,
                                          float *__restrict__ quads) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nH * QH) return;
    const int h = i / QH, f = i % QH;
    const bool fwd = f < 4 * QB;
    const int e = (fwd ? f : f - 4 * QB) / 4, r = f % 4;
    const int dr = e / QF_STRIDE - 11, dc = e % QF_STRIDE - 11;
    int idx;
    if (fwd) {
        const int tc = 11 - dc - r;
        idx = (tc >= 0 && tc < 23) ? (11 - dr) * 23 + tc : -1;
    } else {
        const int tc = dc + r + 11;
        idx = (tc >= 0 && tc < 23) ? (dr + 11) * 23 + tc : -1;
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

// bf16 fragment x c2, rounded to bf16
__device__ __forceinline__ u16x8 scale_frag(u16x8 v, float c) {
    f32x4 lo, hi;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        lo[e] = bf2f(v[e]) * c;
        hi[e] = bf2f(v[4 + e]) * c;
    }
    return __builtin_bit_cast(u16x8, pack_bf16(lo, hi));
}

// Forward, one workgroup per (window, head): 3 waves, wave w owns query tiles 3w..3w+2.  All global
// loads of the workgroup are issued up front and retire behind one wait; 25 KB of LDS and <= 96
// VGPRs let 6 workgroups share a CU, so one workgroup's load latency is covered by the others'
// MFMA / softmax work.  Each 4-key seed is one ds_read_b128 of the head's stride-20 quad grid.
// Scores are formed directly in base-2 units: q is pre-multiplied by c2 = scale·log2 e when it is
// loaded (one bf16 rounding of q·c2, where the reference's AMP rounds q·scale, swin.py:95) and the
// table by log2 e, so s'' = q''·k + T·log2 e and P = 2^s'' needs no scaling fma per score.  The
// row maximum is still formed; only a wave holding a row whose maximum lies outside [-60, 60]
// (where 2^s'' could overflow, or lose precision to underflow) shifts its scores, by one more MFMA
// per key tile that adds 32·bf16(-max/32) to every score of the row (exact, so the LSE records the
// shift that was applied).
template <int MM>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(MM == 2 ? 4 : 5))) winattn_fwd_bf16_rt(const unsigned short *__restrict__ qkv,
                                                            const float *__restrict__ qbias,
                                                            const float *__restrict__ quads,
                                                            const float *__restrict__ mask, Geo g, float c2,
                                                            unsigned short *__restrict__ out, float *__restrict__ lse) {
    __shared__ __attribute__((aligned(16))) unsigned short Ks[NT * HD];  // swizzled 64-B rows (kv_swz)
    __shared__ __attribute__((aligned(16))) unsigned short Vs[NT * HD];
    __shared__ __attribute__((aligned(16))) f32x4 Bq[QB];  // forward quads of this head x c2
    const unsigned long long t_entry = stamp_clock(g.stamp);
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
    f32x4 bq[3];  // QB = 460 <= 3 x 192 quads
    const f32x4 *qsrc = (const f32x4 *)(quads + (long)h * QH);
#pragma unroll
    for (int j = 0; j < 3; ++j) bq[j] = (tid + 192 * j < QB) ? qsrc[tid + 192 * j] : f32x4{0.f, 0.f, 0.f, 0.f};
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
#pragma unroll
    for (int j = 0; j < 3; ++j)
        if (tid + 192 * j < QB) Bq[tid + 192 * j] = bq[j] * c2;  // T / scale -> T·log2 e
#pragma unroll
    for (int j = 0; j < 3; ++j) qreg[j] = scale_frag(qreg[j], c2);
    __syncthreads();
    int part3[3];  // quad offset 20 row + col of key group 16 j + 4 grp; tile 3a + j adds 80 a
#pragma unroll
    for (int j = 0; j < 3; ++j) part3[j] = QF_STRIDE * ((16 * j + 4 * grp) / WS) + (16 * j + 4 * grp) % WS;
    unsigned long long hbits = 0, wbits = 0;
    if (MM == 1) key_class_bits(g.shift, grp, hbits, wbits);
    bool lastH = false, lastW = false;
    if (MM == 1) {
        const int wi = bw % g.nW;
        lastH = wi / g.nWw == g.nWh - 1;
        lastW = wi % g.nWw == g.nWw - 1;
    }
    const float mneg100 = -100.0f * LOG2E;  // the region mask in s'' units
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
        // seed of keys k0 .. k0 + 3: quad 20 (row(k0) - row(qi) + 11) + (col(k0) - col(qi) + 11)
        const f32x4 *bqq = Bq + (QF_STRIDE * 11 + 11 - (QF_STRIDE * (qi / WS) + qi % WS));
        f32x4 s[9];
#pragma unroll
        for (int kt = 0; kt < 9; ++kt) {
            const f32x4 b4 = bqq[part3[kt % 3] + 4 * QF_STRIDE * (kt / 3)];
            const bf16x8_t kf = as_bf(*(const u16x8 *)(kb + kt * 16 * HD));
            s[kt] = mfma16(kf, qf, b4);  // s''ᵀ (key rows, query on the lane), bias seeded
            if (MM == 2) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    s[kt][r] = fmaf(mask[((long)(bw % g.n_mask) * NT + qi) * NT + kt * 16 + grp * 4 + r], LOG2E, s[kt][r]);
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
        float shift = 0.f;
        if (wave_any(!(mx >= -60.f && mx <= 60.f))) {  // rare: shift the row by -max (NaN rows too)
            const unsigned short sh = f2bf(-mx * (1.0f / 32.0f));
            shift = -32.0f * bf2f(sh);
            const bf16x8_t shb = as_bf(u16x8{sh, sh, sh, sh, sh, sh, sh, sh});
#pragma unroll
            for (int kt = 0; kt < 9; ++kt) s[kt] = mfma16(ones, shb, s[kt]);
        }
#pragma unroll
        for (int kt = 0; kt < 9; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[kt][r] = fast_exp2(s[kt][r]);
        f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = o0, os = o0;
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
            const bf16x8_t pb = pack_bf16(s[2 * ks], (2 * ks + 1 < 9) ? s[2 * ks + 1] : f32x4{0.f, 0.f, 0.f, 0.f});
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
            const u16x4 w0 = pack_bf16x4(o0 * inv), w1 = pack_bf16x4(o1 * inv);
            unsigned short *op = out + (long)tok[j] * g.C + h * HD;
            *(u16x4 *)(op + grp * 4) = w0;
            *(u16x4 *)(op + 16 + grp * 4) = w1;
        }
        if (grp == 0) lse[((long)bw * g.nH + h) * NT + qi] = __log2f(os[0]) + shift;  // base-2 LSE of s''
    }
    stamp_end(g.stamp, t_entry);
}

// ---------------------------------------------------------------------------------------------
// Forward, persistent and pipelined: one 3-wave workgroup per (head, chunk of consecutive windows),
// ~3 per CU.  While a window's scores / softmax / PV run out of one LDS stage, the next window's
// q / k / v rows stream into the other stage by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no
// staging instructions), so HBM traffic overlaps the MFMA / VALU work of the previous window
// instead of alternating with it (the per-item kernel above starts every workgroup with all its
// loads outstanding and nothing to compute).  The head's bias quads are staged once per
// workgroup.  LDS: quads 7.4 KB + q 9 KB (one stage: read into registers before the next DMA)
// + 2 x (k + v) 36 KB + pad rows = 53.6 KB, 3 workgroups per CU.  Arithmetic per window is the
// per-item kernel's, instruction for instruction (same rounding, same LSE).
//
// LDS-DMA writes a wave-uniform base + 16 x lane: the 16 rows x 4 chunks of a row block are
// contiguous, and the kv_swz chunk swizzle is applied on the GLOBAL side (LDS slot s of row t
// receives chunk s ^ kv_swz(t)).  Pad tokens (no global row) DMA token 0 of the image and are
// overwritten from the pad rows by the lane that issued their slot, after its own vmcnt wait.
// Ordering: each window's DMA is issued after the barrier that ends every wave's reads of the
// stage and q buffer it overwrites, and waited for (s_waitcnt vmcnt(0)) before the barrier that
// publishes it; no DMA is in flight across a __syncthreads().
constexpr int PP_WG_PER_CU = 3;
constexpr int PP_LDS_BQ = QB * 16, PP_LDS_T = NT * HD * 2;  // bytes: quads, one 144-row tile
constexpr int PP_LDS = PP_LDS_BQ + 5 * PP_LDS_T + 3 * HD * 2;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

__device__ __forceinline__ void dma16(const char *g, unsigned short *lds_block) {
    __builtin_amdgcn_global_load_lds((glb_void *)g, (lds_void *)lds_block, 16, 0, 0);
}

template <int MM>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(3)))
winattn_fwd_bf16_pp(const unsigned short *__restrict__ qkv, const float *__restrict__ qbias,
                    const float *__restrict__ quads, const float *__restrict__ mask, Geo g, int cw, float c2,
                    unsigned short *__restrict__ out, float *__restrict__ lse) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[PP_LDS];  // ONE array (glds wait trap)
    f32x4 *Bq = (f32x4 *)smem;
    unsigned short *Qs = (unsigned short *)(smem + PP_LDS_BQ);
    unsigned short *KVs = Qs + NT * HD;                      // [stage][k, v][NT * HD]
    unsigned short *padS = KVs + 4 * NT * HD;                // pad-token q, k, v rows (bf16)
    const Chunk ck = decode_chunk(g, cw);                    // the heads of one chunk on one XCD
    const int h = ck.h;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, grp = lane >> 4;
    if (ck.w_begin >= ck.w_end) return;
    const char *base = (const char *)qkv;
    const unsigned rowb = 6u * (unsigned)g.C, cb = 2u * (unsigned)g.C;
    // ---- once per workgroup: the head's quads (x c2) and the pad rows
    {
        const f32x4 *qsrc = (const f32x4 *)(quads + (long)h * QH);
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (tid + 192 * j < QB) Bq[tid + 192 * j] = qsrc[tid + 192 * j] * c2;  // T / scale -> T·log2 e
        if (tid < 12) {  // (q, k, v) x 4 chunks of 8 channels
            const int m = tid >> 2, c = tid & 3;
            *(u16x8 *)(padS + m * HD + c * 8) = pad_frag(qbias, m * g.C + h * HD + c * 8);
        }
    }
    // DMA slot of this lane: row block rb = 3 wave + j (16 rows), row t = 16 rb + lane / 4, LDS slot
    // lane % 4 holding global chunk (lane % 4) ^ kv_swz(t)
    const int dslot = lane & 3;
    auto issue = [&](int bw, int stage, int (&dtok)[3]) {
        const WinOrigin wo(g, bw);
        unsigned short *Kd = KVs + (2 * stage) * NT * HD, *Vd = Kd + NT * HD;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int rb = 3 * wave + j, t = 16 * rb + (lane >> 2);
            dtok[j] = wo.tok(g, t);
            const int c = dslot ^ kv_swz(t);
            const int src = dtok[j] >= 0 ? dtok[j] : wo.base;  // pad: any valid row, overwritten below
            const char *p = base + (unsigned)src * rowb + (unsigned)(h * HD + c * 8) * 2u;
            const int o = rb * 16 * HD;  // wave-uniform LDS base of the row block
            dma16(p, Qs + o);
            dma16(p + cb, Kd + o);
            dma16(p + 2 * cb, Vd + o);
        }
    };
    auto fix_pads = [&](int stage, const int (&dtok)[3]) {  // after this wave's vmcnt wait
        unsigned short *Kd = KVs + (2 * stage) * NT * HD, *Vd = Kd + NT * HD;
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (dtok[j] < 0) {
                const int t = 16 * (3 * wave + j) + (lane >> 2), c = dslot ^ kv_swz(t);
                const int o = t * HD + dslot * 8;
                *(u16x8 *)(Kd + o) = *(const u16x8 *)(padS + HD + c * 8);
                *(u16x8 *)(Vd + o) = *(const u16x8 *)(padS + 2 * HD + c * 8);
            }
    };
    int dtok[3];
    __syncthreads();  // pad rows visible before any fix-up
    issue(ck.w_begin, 0, dtok);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fix_pads(0, dtok);
    __syncthreads();
    // ---- per-workgroup constants of the arithmetic (the per-item kernel's)
    int part3[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) part3[j] = QF_STRIDE * ((16 * j + 4 * grp) / WS) + (16 * j + 4 * grp) % WS;
    unsigned long long hbits = 0, wbits = 0;
    if (MM == 1) key_class_bits(g.shift, grp, hbits, wbits);
    const float mneg100 = -100.0f * LOG2E;
    const bf16x8_t ones = as_bf(u16x8{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80});
    const int swz_l = kv_swz(l16);
    const int vsw = kv_swz(4 * grp), vch = ((l16 & 3) >> 1), vin = (l16 & 1) * 4;
    const int vrow = 4 * grp + (l16 >> 2);
    int stage = 0;
    for (int bw = ck.w_begin; bw < ck.w_end; ++bw, stage ^= 1) {
        const WinOrigin wo(g, bw);
        int tok[3];
        u16x8 qreg[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int t = (3 * wave + j) * 16 + l16;
            tok[j] = wo.tok(g, t);
            qreg[j] = tok[j] >= 0 ? *(const u16x8 *)(Qs + t * HD + (grp ^ swz_l) * 8) : *(const u16x8 *)(padS + grp * 8);
            qreg[j] = scale_frag(qreg[j], c2);
        }
        __syncthreads();  // q buffer and the other stage are free
        const bool more = bw + 1 < ck.w_end;
        if (more) issue(bw + 1, stage ^ 1, dtok);
        bool lastH = false, lastW = false;
        if (MM == 1) {
            const int wi = bw % g.nW;
            lastH = wi / g.nWw == g.nWh - 1;
            lastW = wi % g.nWw == g.nWw - 1;
        }
        const unsigned short *Ks = KVs + (2 * stage) * NT * HD, *Vs = Ks + NT * HD;
        const unsigned short *vb0 = Vs + vrow * HD + ((vch ^ vsw) * 8) + vin;
        const unsigned short *vb1 = Vs + vrow * HD + (((vch ^ 2) ^ vsw) * 8) + vin;
        const unsigned short *kb = Ks + l16 * HD + (grp ^ swz_l) * 8;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int qi = (3 * wave + j) * 16 + l16;
            const bf16x8_t qf = as_bf(qreg[j]);
            const f32x4 *bqq = Bq + (QF_STRIDE * 11 + 11 - (QF_STRIDE * (qi / WS) + qi % WS));
            f32x4 s[9];
#pragma unroll
            for (int kt = 0; kt < 9; ++kt) {
                const f32x4 b4 = bqq[part3[kt % 3] + 4 * QF_STRIDE * (kt / 3)];
                const bf16x8_t kf = as_bf(*(const u16x8 *)(kb + kt * 16 * HD));
                s[kt] = mfma16(kf, qf, b4);
                if (MM == 2) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        s[kt][r] = fmaf(mask[((long)(bw % g.n_mask) * NT + qi) * NT + kt * 16 + grp * 4 + r], LOG2E, s[kt][r]);
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
            float shift = 0.f;
            if (wave_any(!(mx >= -60.f && mx <= 60.f))) {
                const unsigned short sh = f2bf(-mx * (1.0f / 32.0f));
                shift = -32.0f * bf2f(sh);
                const bf16x8_t shb = as_bf(u16x8{sh, sh, sh, sh, sh, sh, sh, sh});
#pragma unroll
                for (int kt = 0; kt < 9; ++kt) s[kt] = mfma16(ones, shb, s[kt]);
            }
#pragma unroll
            for (int kt = 0; kt < 9; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) s[kt][r] = fast_exp2(s[kt][r]);
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
            if (tok[j] >= 0) {  // stores need no wait: issuing them beside the DMAs is safe
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
            if (grp == 0) lse[((long)bw * g.nH + h) * NT + qi] = __log2f(os[0]) + shift;
        }
        if (more) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of window bw + 1 landed
            fix_pads(stage ^ 1, dtok);
        }
        __syncthreads();  // publishes the next stage and q rows
    }
}

// Backward: persistent-chunk workgroups of 9 waves (one head x a contiguous chunk of windows,
// ~one workgroup per CU), phase 1 key-on-lane (s' = q·kᵀ + b/scale, dP = dO·Vᵀ - δ; dVᵀ += dOᵀ·P and
// dKᵀ += qᵀ·dS straight from the accumulators; dS to LDS), phase 2 dQᵀ = Kᵀ·dSᵀ.  The biases are the
// forward's values, seeded into the s' accumulator as there: for a key and 4 consecutive queries of
// one window row they are 4 consecutive table entries, one ds_read_b128 from the head's backward
// quads (the stride-20 (dr, dc) grid) staged once per workgroup.  Q, dO, K and V tiles are 64-B rows
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
    __shared__ __attribute__((aligned(16))) f32x4 Bf[QB];  // backward quads (stride-20 grid) of this head
    __shared__ __attribute__((aligned(16))) unsigned short Qs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short dOs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short Ks[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short Vs[NT * HD];
    __shared__ __attribute__((aligned(16))) unsigned short dSt[NR * DST];  // dSᵀ: [key][query], keys >= 144 zero
    __shared__ __attribute__((aligned(16))) float lseS[NT], dltS[NT];
    __shared__ int tokS[NT];
    __shared__ __attribute__((aligned(16))) unsigned short padS[3 * HD];  // pad-token q, k, v (bf16)
    __shared__ float tgS[EX ? TBL : 1];  // EX: this workgroup's rel-table gradient, flushed once
    const unsigned long long t_entry = stamp_clock(g.stamp);
    const Chunk ck = decode_chunk(g, cw);
    const int h = ck.h;
    const float mneg100 = -100.0f * LOG2E;  // the region mask in s'' units
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, grp = lane >> 4;
    {  // the head's backward quads (16-B loads, both issued before either store)
        const f32x4 *src = (const f32x4 *)(quads + (long)h * QH) + QB;
        if (tid < QB) Bf[tid] = src[tid] * c2;  // T / scale -> T·log2 e: scores in base-2 units s''
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
        *(u16x8 *)(Qs + st_off) = scale_frag(qreg, c2);  // q'' = bf16(q·c2), as the forward
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
                        v = fmaf(mask[((long)(bw % g.n_mask) * NT + qt * 16 + grp * 4 + r) * NT + kkey], LOG2E, v);
                    const float p = fast_exp2(v - l4[r]);
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
                    k0[r] = f2bf(dk0[r] * (1.0f / LOG2E));  // dK = scale · dSᵀ·q = dSᵀ·q'' / log2 e
                    k1[r] = f2bf(dk1[r] * (1.0f / LOG2E));
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
                    atomicAdd(&gbias[g.C + c0 + r], dk0[r] * (1.0f / LOG2E));
                    atomicAdd(&gbias[g.C + c0 + 16 + r], dk1[r] * (1.0f / LOG2E));
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
    stamp_end(g.stamp, t_entry);
}

// Forward kernel choice: 0 = one workgroup per (window, head) (winattn_fwd_bf16_rt), 1 = persistent
// LDS-DMA pipelined (winattn_fwd_bf16_pp).  IRADS_WINATTN_FWD=rt|pp overrides (A/B measurements).
int g_fwd_variant = -1;  // -1: not chosen yet

int fwd_variant() {
    if (g_fwd_variant < 0) {
        const char *e = getenv("IRADS_WINATTN_FWD");
        g_fwd_variant = (e && !strcmp(e, "pp")) ? 1 : 0;
    }
    return g_fwd_variant;
}

// persistent forward workgroups: PP_WG_PER_CU per CU (LDS-limited), IRADS_WINATTN_PP_WGS overrides
int pp_slots() {
    static int n = [] {
        const char *e = getenv("IRADS_WINATTN_PP_WGS");
        if (e && atoi(e) > 0) return atoi(e);
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return PP_WG_PER_CU * cus;
    }();
    return n;
}

long bwd_target() {  // persistent backward workgroups per launch; IRADS_WINATTN_BWD_WGS overrides (A/B)
    static const long t = [] {
        const char *e = getenv("IRADS_WINATTN_BWD_WGS");
        const long v = e ? atol(e) : 0;
        return v > 0 ? v : 256L;
    }();
    return t;
}

int chunk_windows(int total_windows, int nH, long target = 256) {  // target: persistent workgroups
    long cw = ((long)total_windows * nH + target - 1) / target;
    return (int)(cw < 1 ? 1 : cw);
}

int make_geo(Geo &g, int dtype, int B, int H, int W, int C, int nH, int shift, float scale, const float *mask,
             int n_mask) {
    g.stamp = take_stamp();  // taken (disarmed) whatever follows; the bf16 kernels write it
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
    const int n = nH * QH;
    winattn_bias_quads_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(rel_table, nH, 1.0f / scale, quads);
    return check_launch("irads_winattn_bias_quads");
}

extern "C" long irads_winattn_bias_quads_size(int nH) { return (long)nH * QH; }

extern "C" int irads_winattn_fwd_variant(int variant) {
    const int prev = fwd_variant();
    if (variant == 0 || variant == 1) g_fwd_variant = variant;
    return prev;
}

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
        if (fwd_variant() == 1) {  // persistent, LDS-DMA pipelined (winattn_fwd_bf16_pp)
            const int n_wg = pp_slots();
            const long items = (long)B * g.nW * nH;
            const int cw = (int)((items + n_wg - 1) / n_wg);
            const unsigned nwg = (unsigned)(((B * g.nW + cw - 1) / cw) * nH);
#define IRADS_WP(M) winattn_fwd_bf16_pp<M><<<nwg, 192, 0, st>>>((const unsigned short *)qkv, qkv_bias, bias_quads, \
                                                                 mask, g, cw, c2, (unsigned short *)out, lse)
            if (mm == 0) IRADS_WP(0); else if (mm == 1) IRADS_WP(1); else IRADS_WP(2);
#undef IRADS_WP
        } else {
#define IRADS_WF(M) winattn_fwd_bf16_rt<M><<<nblk, 192, 0, st>>>((const unsigned short *)qkv, qkv_bias, bias_quads, \
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
        const int cw = chunk_windows(B * g.nW, nH, bwd_target());
        const unsigned nwg = (unsigned)(((B * g.nW + cw - 1) / cw) * nH);
#define IRADS_WB(M, X)                                                                                            \
    winattn_bwd_bf16<M, X><<<nwg, 576, 0, st>>>((const unsigned short *)qkv, qkv_bias, bias_quads, mask, g, cw,   \
                                                scale * LOG2E,                                                    \
                                                (const unsigned short *)out, lse, (const unsigned short *)grad_out, \
                                                (unsigned short *)grad_qkv, grad_table, grad_bias_pad)
        if (ex) {
            if (mm == 0) IRADS_WB(0, true); else if (mm == 1) IRADS_WB(1, true); else IRADS_WB(2, true);
        } else {
            if (mm == 0) IRADS_WB(0, false); else if (mm == 1) IRADS_WB(1, false); else IRADS_WB(2, false);
        }
#undef IRADS_WB
    }
    return check_launch("irads_winattn_bwd");
}
