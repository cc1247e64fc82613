// AdamW update of a list of fp32 parameters (torch.optim.AdamW's fused / capturable step, the
// reference's optimizer, semseg/optimizers.py:33-49) in a few launches instead of PyTorch's
// multi-tensor chunks: the tensors go to the kernel as arguments in batches of kBatch (one learning
// rate and weight decay per launch), and each
// launch gives every tensor blocks in proportion to its size (4096 elements per block), so one big
// tensor no longer leaves a launch nearly idle.  The step count and learning rate are read on the
// device (per tensor), so the launches can be captured in a HIP graph and replayed.
//
// Per element, as ATen's fused Adam in ADAMW mode (decoupled weight decay):
//   p -= lr * wd * p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps),   bc_i = 1 - b_i^step.
#include "common.h"

namespace irads {
namespace {

constexpr int kBatch = 72;       // tensors per launch (kernel arguments stay under 4 KiB)
constexpr int kChunk = 4096;     // elements per block
constexpr int kThreads = 256;

// one launch: tensors sharing a learning rate and weight decay (a param group)
struct AdamWBatch {
    float *p[kBatch];
    const float *g[kBatch];
    float *m[kBatch];
    float *v[kBatch];
    const float *step[kBatch];
    int numel[kBatch];
    int first_block[kBatch + 1];  // block range of tensor t: [first_block[t], first_block[t + 1])
    const float *lr;
    float wd;
    int n;
    double beta1, beta2;       // the bias corrections are formed from these
    float b1, omb1, b2, omb2;  // beta_i and 1 - beta_i (taken in double), rounded once
    float eps;
};
static_assert(sizeof(AdamWBatch) <= 4096, "kernel arguments are limited to 4 KiB");

__device__ __forceinline__ void adamw_elem(float &p, float g, float &m, float &v, float lr, float wd, float b1,
                                           float omb1, float b2, float omb2, float eps, float step_size,
                                           float bc2s) {
    p -= lr * wd * p;
    m = b1 * m + omb1 * g;
    v = b2 * v + omb2 * g * g;
    const float denom = sqrtf(v) / bc2s + eps;
    p -= step_size * m / denom;
}

__global__ void __launch_bounds__(kThreads) adamw_kernel(const AdamWBatch B) {
    // the block's tensor: binary search over the batch's block ranges (uniform per block)
    int lo = 0, hi = B.n - 1;
    const int blk = blockIdx.x;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (B.first_block[mid] <= blk) lo = mid;
        else hi = mid - 1;
    }
    const int t = lo;
    float *__restrict__ p = B.p[t];
    const float *__restrict__ g = B.g[t];
    float *__restrict__ m = B.m[t];
    float *__restrict__ v = B.v[t];
    const long n = B.numel[t];
    const long begin = (long)(blk - B.first_block[t]) * kChunk;
    const long end = min(n, begin + kChunk);
    const float lr = *B.lr, step = *B.step[t], wd = B.wd;
    const float b1 = B.b1, omb1 = B.omb1, b2 = B.b2, omb2 = B.omb2, eps = B.eps;
    // bias corrections in double, as ATen forms them from the double betas
    const float bc1 = (float)(1.0 - pow(B.beta1, (double)step));
    const float bc2 = (float)(1.0 - pow(B.beta2, (double)step));
    const float step_size = lr / bc1, bc2s = sqrtf(bc2);
    const bool vec = ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0);
    if (vec) {
        const long nv = (end - begin) / 4;
        for (long i = threadIdx.x; i < nv; i += kThreads) {
            const long e = begin + 4 * i;
            const f32x4 p4 = *(const f32x4 *)(p + e), g4 = *(const f32x4 *)(g + e);
            const f32x4 m4 = *(const f32x4 *)(m + e), v4 = *(const f32x4 *)(v + e);
            float pp[4], mm[4], vv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pp[j] = p4[j];
                mm[j] = m4[j];
                vv[j] = v4[j];
                adamw_elem(pp[j], g4[j], mm[j], vv[j], lr, wd, b1, omb1, b2, omb2, eps, step_size, bc2s);
            }
            *(f32x4 *)(p + e) = f32x4{pp[0], pp[1], pp[2], pp[3]};
            *(f32x4 *)(m + e) = f32x4{mm[0], mm[1], mm[2], mm[3]};
            *(f32x4 *)(v + e) = f32x4{vv[0], vv[1], vv[2], vv[3]};
        }
        for (long e = begin + 4 * nv + threadIdx.x; e < end; e += kThreads) {
            float pp = p[e], mm = m[e], vv = v[e];
            adamw_elem(pp, g[e], mm, vv, lr, wd, b1, omb1, b2, omb2, eps, step_size, bc2s);
            p[e] = pp;
            m[e] = mm;
            v[e] = vv;
        }
    } else {
        for (long e = begin + threadIdx.x; e < end; e += kThreads) {
            float pp = p[e], mm = m[e], vv = v[e];
            adamw_elem(pp, g[e], mm, vv, lr, wd, b1, omb1, b2, omb2, eps, step_size, bc2s);
            p[e] = pp;
            m[e] = mm;
            v[e] = vv;
        }
    }
}

}  // namespace
}  // namespace irads

using namespace irads;

extern "C" int irads_adamw(int n, float *const *p, const float *const *g, float *const *m, float *const *v,
                           const float *const *step, const float *const *lr, const float *wd, const long *numel,
                           double beta1, double beta2, double eps, void *stream) {
    IRADS_REQUIRE(n >= 0, "adamw: bad tensor count");
    if (n == 0) return IRADS_OK;
    IRADS_REQUIRE(p && g && m && v && step && lr && wd && numel, "adamw: null array");
    hipStream_t st = (hipStream_t)stream;
    int t = 0;
    while (t < n) {  // a launch per run of up to kBatch tensors with one learning rate and weight decay
        AdamWBatch B;
        B.n = 0;
        B.lr = lr[t];
        B.wd = wd[t];
        B.beta1 = beta1;
        B.beta2 = beta2;
        B.b1 = (float)beta1;
        B.omb1 = (float)(1.0 - beta1);
        B.b2 = (float)beta2;
        B.omb2 = (float)(1.0 - beta2);
        B.eps = (float)eps;
        int blocks = 0;
        for (; t < n && B.n < kBatch && lr[t] == B.lr && wd[t] == B.wd; ++t) {
            IRADS_REQUIRE(p[t] && g[t] && m[t] && v[t] && step[t] && lr[t], "adamw: null pointer for tensor %d", t);
            IRADS_REQUIRE(numel[t] >= 0 && numel[t] < (1L << 31), "adamw: bad size for tensor %d", t);
            const long nb = (numel[t] + kChunk - 1) / kChunk;
            IRADS_REQUIRE(blocks + nb < (1L << 30), "adamw: too many elements in one launch");
            const int i = B.n++;
            B.p[i] = p[t];
            B.g[i] = g[t];
            B.m[i] = m[t];
            B.v[i] = v[t];
            B.step[i] = step[t];
            B.numel[i] = (int)numel[t];
            B.first_block[i] = blocks;
            blocks += (int)nb;
        }
        B.first_block[B.n] = blocks;
        if (blocks == 0) continue;
        adamw_kernel<<<blocks, kThreads, 0, st>>>(B);
        if (int e = check_launch("irads_adamw")) return e;
    }
    return IRADS_OK;
}
