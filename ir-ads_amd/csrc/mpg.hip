// MAPA prompt residual of the two-stream Swin (reference semseg/models/backbones/swin.py:1045-1068
// and the stage loop that adds its outputs, :1455-1460), fused with the rgb/dte batching:
//
//   x    = U_fc1(P_fc2(cat[D_fc1(x_rgb), D_fc2(x_dte)]))            (bf16, the GEMMs stay on hipBLASLt)
//   out  = cat[x_rgb + (x + (x*g_rgb + b_rgb)),  x_dte + (x + (x*g_dte + b_dte))]   (fp32, 2R x C)
//
// The reference runs this as 2 multiplies, 4 adds and a concatenation over (B, N, C) fp32
// tensors, and its backward as as many again plus four column reductions; here it is one
// pass each way.  Arithmetic is the reference's under autocast op by op: x is bf16, the
// tfts parameters fp32, every op an fp32 op rounded on its own (built with
// -ffp-contract=off: no FMA contraction, so the forward is bit-identical to torch's).
// Backward: g = dL/d out; dx_rgb, dx_dte are the two halves of g (views, no kernel);
//   dx    = bf16((g_r + g_r*g_rgb) + (g_d + g_d*g_dte))   (one rounding; the reference
//           accumulates four bf16-rounded terms, within one bf16 ulp of this)
//   dg_*  = sum_rows g_* * x,  db_* = sum_rows g_*        (per-block partials, added by the host)
#include "common.h"

namespace irads {
namespace {

typedef unsigned short u16;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ void unpack8(u32x4 w, float *f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}

// one thread = 8 consecutive channels of one row; a block walks rows with stride
// (256 / (C/8)) rows per iteration
// 8 consecutive stream values as fp32: fp32 rows (stage 0: the patch embedding's output) or
// bf16 rows (stages 1-3: PatchMerging's reduction GEMM output), upcast exactly as torch's
// bf16 + fp32 type promotion does
__device__ __forceinline__ void load8(const float *p, float *f) {
    const float4 a = reinterpret_cast<const float4 *>(p)[0], b = reinterpret_cast<const float4 *>(p)[1];
    f[0] = a.x, f[1] = a.y, f[2] = a.z, f[3] = a.w, f[4] = b.x, f[5] = b.y, f[6] = b.z, f[7] = b.w;
}
__device__ __forceinline__ void load8(const u16 *p, float *f) { unpack8(*reinterpret_cast<const u32x4 *>(p), f); }

template <typename TS>
__global__ __launch_bounds__(256) void mpg_fwd_kernel(const u16 *__restrict__ x, const TS *__restrict__ xr,
                                                      const TS *__restrict__ xd, const float *__restrict__ gr,
                                                      const float *__restrict__ br, const float *__restrict__ gd,
                                                      const float *__restrict__ bd, long R, int C,
                                                      float *__restrict__ out) {
    const int groups = C / 8;
    const int rpi = 256 / groups;  // rows per iteration
    const int cg = threadIdx.x % groups, rl = threadIdx.x / groups;
    if (rl >= rpi) return;
    const int c0 = cg * 8;
    float Gr[8], Br[8], Gd[8], Bd[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Gr[j] = gr[c0 + j], Br[j] = br[c0 + j], Gd[j] = gd[c0 + j], Bd[j] = bd[c0 + j];
    for (long r = (long)blockIdx.x * rpi + rl; r < R; r += (long)gridDim.x * rpi) {
        float xv[8];
        unpack8(*reinterpret_cast<const u32x4 *>(x + r * C + c0), xv);
        float av[8], dv[8];
        load8(xr + r * C + c0, av);
        load8(xd + r * C + c0, dv);
        float orr[8], odd[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float pr_ = __fadd_rn(__fmul_rn(xv[j], Gr[j]), Br[j]);  // apply_tfts
            const float pd_ = __fadd_rn(__fmul_rn(xv[j], Gd[j]), Bd[j]);
            orr[j] = __fadd_rn(av[j], __fadd_rn(xv[j], pr_));  // x_rgb + (x + p_rgb)
            odd[j] = __fadd_rn(dv[j], __fadd_rn(xv[j], pd_));
        }
        float4 *qr = reinterpret_cast<float4 *>(out + r * C + c0);
        float4 *qd = reinterpret_cast<float4 *>(out + (R + r) * C + c0);
        qr[0] = make_float4(orr[0], orr[1], orr[2], orr[3]);
        qr[1] = make_float4(orr[4], orr[5], orr[6], orr[7]);
        qd[0] = make_float4(odd[0], odd[1], odd[2], odd[3]);
        qd[1] = make_float4(odd[4], odd[5], odd[6], odd[7]);
    }
}

// partials: [block][4][C] = (sum g_r*x, sum g_r, sum g_d*x, sum g_d) over this block's rows,
// combined across the block's row lanes in a fixed order through LDS
__global__ __launch_bounds__(256) void mpg_bwd_kernel(const float *__restrict__ g, const u16 *__restrict__ x,
                                                      const float *__restrict__ gr, const float *__restrict__ gd,
                                                      long R, int C, u16 *__restrict__ gx,
                                                      float *__restrict__ part) {
    __shared__ float red[4][256 * 8 / 8];  // per thread: 4 quantities x 8 channels, staged 1 channel at a time
    const int groups = C / 8;
    const int rpi = 256 / groups;
    const int cg = threadIdx.x % groups, rl = threadIdx.x / groups;
    const bool act = rl < rpi;
    const int c0 = cg * 8;
    float Gr[8], Gd[8], s[4][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        Gr[j] = act ? gr[c0 + j] : 0.f;
        Gd[j] = act ? gd[c0 + j] : 0.f;
        s[0][j] = s[1][j] = s[2][j] = s[3][j] = 0.f;
    }
    if (act) {
        for (long r = (long)blockIdx.x * rpi + rl; r < R; r += (long)gridDim.x * rpi) {
            float xv[8];
            unpack8(*reinterpret_cast<const u32x4 *>(x + r * C + c0), xv);
            const float4 *pr = reinterpret_cast<const float4 *>(g + r * C + c0);
            const float4 *pd = reinterpret_cast<const float4 *>(g + (R + r) * C + c0);
            const float4 a0 = pr[0], a1 = pr[1], d0 = pd[0], d1 = pd[1];
            const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
            u32x4 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float t = __fadd_rn(__fadd_rn(av[j], __fmul_rn(av[j], Gr[j])),
                                          __fadd_rn(dv[j], __fmul_rn(dv[j], Gd[j])));
                const unsigned short b = f2bf(t);
                if (j & 1)
                    o[j >> 1] |= (unsigned)b << 16;
                else
                    o[j >> 1] = b;
                s[0][j] += av[j] * xv[j];
                s[1][j] += av[j];
                s[2][j] += dv[j] * xv[j];
                s[3][j] += dv[j];
            }
            *reinterpret_cast<u32x4 *>(gx + r * C + c0) = o;
        }
    }
    // fixed-order reduction over the rpi row lanes of each channel group, one channel at a time
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int q = 0; q < 4; ++q) red[q][threadIdx.x] = s[q][j];
        __syncthreads();
        for (int qc = threadIdx.x; qc < 4 * groups; qc += blockDim.x) {
            const int q = qc / groups, cc = qc % groups;
            float t = 0.f;
            for (int i = 0; i < rpi; ++i) t += red[q][i * groups + cc];
            part[((long)blockIdx.x * 4 + q) * C + cc * 8 + j] = t;
        }
        __syncthreads();
    }
}

int mpg_blocks(long R, int C) {
    const int rpi = 256 / (C / 8);
    long b = (R + rpi - 1) / rpi;
    const long target = 1024;  // ~4 workgroups per CU; each walks R / (blocks * rpi) rows
    return (int)(b < target ? b : target);
}

}  // namespace
}  // namespace irads

using namespace irads;

#define IRADS_MPG_CHECK(fn)                                                                                       \
    IRADS_REQUIRE(R > 0 && C >= 8 && C % 8 == 0 && C <= 2048, fn ": need R > 0 and C a multiple of 8 in [8, 2048] " \
                                                               "(R=%ld C=%d)", R, C)

extern "C" long irads_mpg_partials(long R, int C) { return (long)mpg_blocks(R, C) * 4 * C; }

extern "C" int irads_mpg_fwd(const uint16_t *x, const float *x_rgb, const float *x_dte, const float *gamma_rgb,
                             const float *beta_rgb, const float *gamma_dte, const float *beta_dte, long R, int C,
                             float *out, void *stream) {
    IRADS_MPG_CHECK("irads_mpg_fwd");
    IRADS_REQUIRE(x && x_rgb && x_dte && gamma_rgb && beta_rgb && gamma_dte && beta_dte && out,
                  "irads_mpg_fwd: null pointer");
    hipLaunchKernelGGL(mpg_fwd_kernel<float>, dim3(mpg_blocks(R, C)), dim3(256), 0, (hipStream_t)stream, x, x_rgb,
                       x_dte, gamma_rgb, beta_rgb, gamma_dte, beta_dte, R, C, out);
    return check_launch("irads_mpg_fwd");
}
extern "C" int irads_mpg_fwd_bf16(const uint16_t *x, const uint16_t *x_rgb, const uint16_t *x_dte,
                                  const float *gamma_rgb, const float *beta_rgb, const float *gamma_dte,
                                  const float *beta_dte, long R, int C, float *out, void *stream) {
    IRADS_MPG_CHECK("irads_mpg_fwd_bf16");
    IRADS_REQUIRE(x && x_rgb && x_dte && gamma_rgb && beta_rgb && gamma_dte && beta_dte && out,
                  "irads_mpg_fwd_bf16: null pointer");
    hipLaunchKernelGGL(mpg_fwd_kernel<u16>, dim3(mpg_blocks(R, C)), dim3(256), 0, (hipStream_t)stream, x, x_rgb,
                       x_dte, gamma_rgb, beta_rgb, gamma_dte, beta_dte, R, C, out);
    return check_launch("irads_mpg_fwd_bf16");
}

extern "C" int irads_mpg_bwd(const float *grad, const uint16_t *x, const float *gamma_rgb, const float *gamma_dte,
                             long R, int C, uint16_t *grad_x, float *partials, void *stream) {
    IRADS_MPG_CHECK("irads_mpg_bwd");
    IRADS_REQUIRE(grad && x && gamma_rgb && gamma_dte && grad_x && partials, "irads_mpg_bwd: null pointer");
    hipLaunchKernelGGL(mpg_bwd_kernel, dim3(mpg_blocks(R, C)), dim3(256), 0, (hipStream_t)stream, grad, x, gamma_rgb,
                       gamma_dte, R, C, grad_x, partials);
    return check_launch("irads_mpg_bwd");
}
