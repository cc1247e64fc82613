// Greedy non-maximum suppression for the vCLR DINO inference, gfx950.
//
// Reference: projects/vCLR_deformable_mask/modeling/dino.py:1245 (nms_inference keeps
// batched_nms(box, score, label, 0.7) of the 300 best-scored queries) -> detectron2
// layers/nms.py batched_nms -> torchvision.ops.batched_nms (a third-party dependency, absent
// here): below 20 000 boxes its "coordinate trick" shifts every box by label x (max coordinate + 1)
// so boxes of different labels never overlap, then runs nms: boxes in decreasing score order, a
// box is dropped when its IoU with an earlier KEPT box exceeds the threshold, with
// IoU = inter / (area_a + area_b - inter) on xyxy boxes (no +1 pixel convention).
//
// One workgroup per image: the sorted boxes and their keep flags live in LDS; box i is decided once
// every earlier box is (the barrier of step i), then its row of IoUs against the later boxes is
// spread over the workgroup's lanes.  n <= kNmsMax (the inference passes 300).  The IoU is formed
// with the reference's operation order and no contraction into fused multiply-adds, so a tie at
// the threshold decides as the unfused arithmetic does.
#include "common.h"

namespace irads {
namespace {

constexpr int kNmsMax = 4096, kNmsThreads = 256;

__device__ __forceinline__ bool iou_above(float4 a, float sa, float4 b, float thr) {
#pragma clang fp contract(off)
    const float w = fmaxf(fminf(a.z, b.z) - fmaxf(a.x, b.x), 0.f);
    const float h = fmaxf(fminf(a.w, b.w) - fmaxf(a.y, b.y), 0.f);
    const float inter = w * h;
    const float sb = (b.z - b.x) * (b.w - b.y);
    return inter / (sa + sb - inter) > thr;
}

__global__ void __launch_bounds__(kNmsThreads) nms_kernel(const float4 *__restrict__ boxes, int n, float thr,
                                                          unsigned char *__restrict__ keep) {
#pragma clang fp contract(off)
    __shared__ float4 bx[kNmsMax];
    __shared__ unsigned char kp[kNmsMax];
    for (int i = threadIdx.x; i < n; i += kNmsThreads) {
        bx[i] = boxes[i];
        kp[i] = 1;
    }
    __syncthreads();
    for (int i = 0; i < n; ++i) {
        if (kp[i]) {  // uniform: every lane reads it after the same barrier
            const float4 a = bx[i];
            const float sa = (a.z - a.x) * (a.w - a.y);
            for (int j = i + 1 + threadIdx.x; j < n; j += kNmsThreads)
                if (kp[j] && iou_above(a, sa, bx[j], thr)) kp[j] = 0;
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < n; i += kNmsThreads) keep[i] = kp[i];
}

}  // namespace
}  // namespace irads

using namespace irads;

extern "C" int irads_nms(const float *boxes, int n, float iou_threshold, unsigned char *keep, void *stream) {
    IRADS_REQUIRE(n >= 0 && n <= kNmsMax, "irads_nms: %d boxes (at most %d)", n, kNmsMax);
    if (n == 0) return IRADS_OK;
    IRADS_REQUIRE(boxes && keep && ((uintptr_t)boxes & 15) == 0, "irads_nms: null / unaligned boxes");
    nms_kernel<<<1, kNmsThreads, 0, (hipStream_t)stream>>>((const float4 *)boxes, n, iou_threshold, keep);
    return check_launch("irads_nms");
}
