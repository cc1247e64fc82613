/*
 * TEST INFRASTRUCTURE ONLY — CPU restatement (oracle) of the reference's bilinear
 * sampling arithmetic.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product path never links it.
 *
 * What it restates:
 *   - F.grid_sample(mode='bilinear', padding_mode='zeros') on CPU as the reference's
 *     PyTorch paths call it:
 *       * align_corners=False: multi_scale_deformable_attn_pytorch
 *         (detrex/layers/multi_scale_deform_attn.py:96-136, grid = 2*loc-1 at :106)
 *       * align_corners=True : DAttentionMM (semseg/models/backbones/swin.py:911-934,
 *         995-1007)
 *   - the integer corner indices floor(ix), floor(iy) those calls use.
 *
 * Arithmetic pinned to torch 2.10's CPU kernel (AVX512 path; SURVEY.md §7 "hard parts"),
 * and re-checked against the reference's own outputs by tests/test_oracle_golden.py:
 *   align_corners=False : ix = fmaf(gx + 1, W/2, -0.5)      (unnormalize)
 *   align_corners=True  : ix = (gx + 1) * ((W-1)/2)          (no FMA)
 *   corners x0 = floor(ix), y0 = floor(iy); fx = ix - x0, fy = iy - y0
 *   nw=(1-fx)(1-fy) ne=fx(1-fy) sw=(1-fx)fy se=fx*fy ; OOB corners contribute 0
 *   out = fmaf(v_se, se, fmaf(v_sw, sw, fmaf(v_ne, ne, v_nw*nw)))
 * Compile with -ffp-contract=off so only the explicit fmaf() calls fuse.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline float unnormalize(float g, int size, int align_corners) {
    if (align_corners) {
        float s = ((float)size - 1.0f) / 2.0f;
        return (g + 1.0f) * s;
    }
    float s = (float)size / 2.0f;
    return fmaf(g + 1.0f, s, -0.5f);
}

static inline float tap(const float *plane, int H, int W, int y, int x) {
    if (x < 0 || x >= W || y < 0 || y >= H) return 0.0f;
    return plane[(int64_t)y * W + x];
}

/* Sample one (C, H, W) image at n grid points (x, y) interleaved.
 * out: (C, n) ; corners (optional): (n, 2) int32 = (x0, y0). */
void oracle_grid_sample(const float *img, int C, int H, int W, const float *grid, int n,
                        int align_corners, float *out, int32_t *corners) {
    for (int p = 0; p < n; ++p) {
        float gx = grid[2 * p], gy = grid[2 * p + 1];
        float ix = unnormalize(gx, W, align_corners);
        float iy = unnormalize(gy, H, align_corners);
        float fx0 = floorf(ix), fy0 = floorf(iy);
        int x0 = (int)fx0, y0 = (int)fy0;
        float fx = ix - fx0, fy = iy - fy0;
        float nw = (1.0f - fx) * (1.0f - fy);
        float ne = fx * (1.0f - fy);
        float sw = (1.0f - fx) * fy;
        float se = fx * fy;
        if (corners) {
            corners[2 * p] = x0;
            corners[2 * p + 1] = y0;
        }
        for (int c = 0; c < C; ++c) {
            const float *pl = img + (int64_t)c * H * W;
            float v = tap(pl, H, W, y0, x0) * nw;
            v = fmaf(tap(pl, H, W, y0, x0 + 1), ne, v);
            v = fmaf(tap(pl, H, W, y0 + 1, x0), sw, v);
            v = fmaf(tap(pl, H, W, y0 + 1, x0 + 1), se, v);
            out[(int64_t)c * n + p] = v;
        }
    }
}

/* MSDA forward restatement (multi_scale_deform_attn.py:96-136).
 * value (bs, S, M, D); shapes (L, 2) int64 (H, W); loc (bs, Q, M, L, P, 2) x-first;
 * aw (bs, Q, M, L, P); out (bs, Q, M*D); corners (optional) (bs, Q, M, L, P, 2) int32.
 * Sum over (l, p) in sequential order (the reference's .sum(-1) order is a reduction
 * detail; values are compared with a tolerance, corner indices bit-exactly). */
void oracle_msda_fwd(const float *value, const int64_t *shapes, int bs, int S, int M, int D,
                     int L, int Q, int P, const float *loc, const float *aw, float *out,
                     int32_t *corners) {
    memset(out, 0, sizeof(float) * (size_t)bs * Q * M * D);
    for (int b = 0; b < bs; ++b)
        for (int q = 0; q < Q; ++q)
            for (int m = 0; m < M; ++m) {
                int64_t start = 0;
                for (int l = 0; l < L; ++l) {
                    int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1];
                    for (int p = 0; p < P; ++p) {
                        int64_t li = ((((int64_t)b * Q + q) * M + m) * L + l) * P + p;
                        float gx = 2.0f * loc[2 * li] - 1.0f;
                        float gy = 2.0f * loc[2 * li + 1] - 1.0f;
                        float ix = unnormalize(gx, W, 0), iy = unnormalize(gy, H, 0);
                        float fx0 = floorf(ix), fy0 = floorf(iy);
                        int x0 = (int)fx0, y0 = (int)fy0;
                        float fx = ix - fx0, fy = iy - fy0;
                        float nw = (1.0f - fx) * (1.0f - fy), ne = fx * (1.0f - fy);
                        float sw = (1.0f - fx) * fy, se = fx * fy;
                        if (corners) {
                            corners[2 * li] = x0;
                            corners[2 * li + 1] = y0;
                        }
                        float w = aw[li];
                        for (int d = 0; d < D; ++d) {
                            /* value_l as (M*D plane-major) view: element (y, x) of head m, chan d */
#define V(yy, xx) (((xx) < 0 || (xx) >= W || (yy) < 0 || (yy) >= H) ? 0.0f : \
    value[(((int64_t)b * S + start + (int64_t)(yy) * W + (xx)) * M + m) * D + d])
                            float v = V(y0, x0) * nw;
                            v = fmaf(V(y0, x0 + 1), ne, v);
                            v = fmaf(V(y0 + 1, x0), sw, v);
                            v = fmaf(V(y0 + 1, x0 + 1), se, v);
#undef V
                            out[(((int64_t)b * Q + q) * M + m) * D + d] += v * w;
                        }
                    }
                    start += (int64_t)H * W;
                }
            }
}
