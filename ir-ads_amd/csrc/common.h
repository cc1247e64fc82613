// Shared helpers for the gfx950 kernels of libirads.so.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/irads.h"

namespace irads {

void set_error(const char *fmt, ...);
// In-step kernel spans (bench.py's roofline lines): the slot irads_stamp_next() armed for the
// calling thread's next stamped launch, or null; taking it disarms.
unsigned long long *take_stamp();

#define IRADS_REQUIRE(cond, ...)          \
    do {                                  \
        if (!(cond)) {                    \
            ::irads::set_error(__VA_ARGS__); \
            return IRADS_EINVAL;          \
        }                                 \
    } while (0)

inline int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return IRADS_ELAUNCH;
    }
    return IRADS_OK;
}

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float bf2f(unsigned short u) {
    return __uint_as_float(((unsigned)u) << 16);
}
// round-to-nearest-even f32 -> bf16; gfx950 has it in hardware (v_cvt_pk_bf16_f32, NaN stays NaN)
__device__ __forceinline__ unsigned short f2bf(float f) {
    return __builtin_bit_cast(unsigned short, (__bf16)f);
}

// erf in fp32 within 1 ulp (0.97 ulp measured against libm's erf in fp64 over [-6, 6] on a 6e-6
// grid, with an exact exp; the hardware exp adds < 1 ulp of exp(r) on the |x| > 0.9277 branch):
// x·P(x²) below 0.9277, 1 - exp(t·Q(t)) above, both minimax fits.  Straight-line FMAs and one
// v_exp_f32, about half the VALU of the libdevice erff, which the GELU passes (FFN, swin.py:597)
// are bound by.  NaN propagates, erf(±inf) = ±1.
__device__ __forceinline__ float erf_f32(float a) {
    const float t = fabsf(a), s = a * a;
    float r = fmaf(-1.72853470e-5f, t, 3.83197126e-4f);
    const float u = fmaf(-3.88396438e-3f, t, 2.42546219e-2f);
    r = fmaf(r, s, u);
    r = fmaf(r, t, -1.06777877e-1f);
    r = fmaf(r, t, -6.34846687e-1f);
    r = fmaf(r, t, -1.28717512e-1f);
    r = fmaf(r, t, -t);
    const float big = copysignf(1.0f - __expf(r), a);
    float q = -5.96761703e-4f;
    q = fmaf(q, s, 4.99119423e-3f);
    q = fmaf(q, s, -2.67681349e-2f);
    q = fmaf(q, s, 1.12819925e-1f);
    q = fmaf(q, s, -3.76125336e-1f);
    q = fmaf(q, s, 1.28379166e-1f);
    const float small = fmaf(q, a, a);
    return t > 0.927734375f ? big : small;
}

template <typename T> struct io;
template <> struct io<float> {
    static __device__ __forceinline__ float ld(const float *p, long i) { return p[i]; }
    static __device__ __forceinline__ void st(float *p, long i, float v) { p[i] = v; }
};
template <> struct io<unsigned short> {  // bf16 storage
    static __device__ __forceinline__ float ld(const unsigned short *p, long i) { return bf2f(p[i]); }
    static __device__ __forceinline__ void st(unsigned short *p, long i, float v) { p[i] = f2bf(v); }
};

// XCD-aware, bijective remap of a linear block id (cdna_hip_programming.md §5, T1):
// consecutive logical ids land on the same XCD (each XCD has its own L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int nx = 8;
    int q = nwg / nx, r = nwg % nx, x = orig % nx;
    int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
    return base + orig / nx;
}

// Raw v_exp_f32 (2^x): no denormal range fix-up. Softmax arguments are <= 0 and results
// below 2^-126 only ever feed bf16 operands, so flushing them to zero is harmless.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// max over lanes l, l ^ 16, l ^ 32, l ^ 48 with the gfx950 lane-swap VALU ops (no LDS round trip,
// unlike __shfl_xor's ds_bpermute): each swap hands every lane its partner's value in one of the
// two results, the other result being its own
__device__ __forceinline__ float max_xor16_32(float v) {
    auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float sum_xor16_32(float v) {
    auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Kernel span stamps (bench.py's in-step roofline): a stamped launch gets a region of STAMP_CAP
// (start, end) pairs; workgroup w (linear block id) writes its entry clock to region[2w] and its exit
// clock to region[2w + 1] on the device's constant-rate wall clock (s_memrealtime); the host reads
// min(start) .. max(end) = the launch's span inside the step.  Plain vector stores, one lane per
// workgroup, no shared address (a single min/max atomic address serialised every workgroup across
// the 8 XCDs: ~14 ns each, doubling the window-attention forward).  A null region (every launch but
// the stamped ones) is a uniform branch.
constexpr unsigned STAMP_CAP = IRADS_STAMP_CAP;
// The entry clock is READ at entry (stamp_clock: a scalar clock read, no memory write) and written
// with the exit clock at the end: a global store at entry would count as clobbering every later
// load, so the compiler would stop fetching the kernels' wave-uniform data through scalar loads
// (measured: DAttn forward 54 -> 130 VGPRs, 7 -> 3 waves per SIMD).
__device__ __forceinline__ unsigned stamp_wg() { return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); }
__device__ __forceinline__ unsigned long long stamp_clock(const unsigned long long *s) {
    return s ? (unsigned long long)wall_clock64() : 0ull;
}
__device__ __forceinline__ void stamp_write(unsigned long long *s, unsigned long long t0, bool with_end) {
    if (s && threadIdx.x == 0) {
        const unsigned w = stamp_wg();
        if (w < STAMP_CAP) {
            s[2 * w] = t0;
            if (with_end) s[2 * w + 1] = (unsigned long long)wall_clock64();
        }
    }
}
// exit stamp after a workgroup barrier: call it where every thread arrives
__device__ __forceinline__ void stamp_end(unsigned long long *s, unsigned long long t0) {
    if (s) {
        __syncthreads();
        stamp_write(s, t0, true);
    }
}
// exit clock only, lane 0 of the workgroup, no barrier (one-pass kernels ending a stamped entry)
__device__ __forceinline__ void stamp_end_lane0(unsigned long long *s) {
    if (s && threadIdx.x == 0) {
        const unsigned w = stamp_wg();
        if (w < STAMP_CAP) s[2 * w + 1] = (unsigned long long)wall_clock64();
    }
}

// counter-based dropout draw: splitmix64 of (seed, element index) -> uniform [0, 1)
// (the Adapter dropout of swinblock.hip and adapter.hip draw from the same stream)
__device__ __forceinline__ float uniform01(unsigned long long seed, unsigned long long i) {
    unsigned long long z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(unsigned)(z >> 40) * (1.f / 16777216.f);
}

}  // namespace irads
