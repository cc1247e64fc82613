// LDS float-atomic throughput by address pattern (gfx950), 16 waves per CU.
// Addresses are precomputed per lane, so the loop is one LDS op plus ~2 VALU ops;
// "ds_write" is the same loop with a plain store (baseline).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x) (void)(x)

// atomic: 0 = ds_write, 1 = ds_add_f32, 2 = ds_add_u32, 3 = ds_add_u64,
//         4 = global_atomic_add_f32 (no return) into a per-CU 19200-float slab,
//         5 = global_atomic_add_f32 into ONE slab shared by all CUs
__global__ void __launch_bounds__(1024) k(int pattern, int atomic, int iters, float *out, long long *cyc,
                                          float *gslab) {
    __shared__ float tg[19200];
    unsigned *tu = (unsigned *)tg;
    unsigned long long *tl = (unsigned long long *)tg;
    float *gs = gslab + (atomic == 4 ? (long)blockIdx.x * 19200 : 0);
    for (int i = threadIdx.x; i < 19200; i += 1024) tg[i] = 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int addr[8];
    unsigned h = threadIdx.x * 2654435761u + 12345u;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        int a;
        const int base = (u * 2371 + wave * 211) % 18000;
        if (pattern == 0) a = base + lane;                       // consecutive
        else if (pattern == 1) a = base + (lane * 5) / 8;        // ~0.62 cell/lane (DAttn pass Q)
        else if (pattern == 2) { h = h * 1664525u + 1013904223u; a = (h >> 8) % 18000; }  // scattered
        else if (pattern == 3) a = base;                         // same address
        else a = (base + lane * 159) % 18000;                    // stride Wt
        addr[u] = a;
    }
    long long t0 = clock64();
    for (int it = 0; it < iters; it += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int a = addr[u] + (it & 63);
            if (atomic == 0) tg[a] = (float)it;
            else if (atomic == 1) atomicAdd(&tg[a], 1.0f);
            else if (atomic == 2) atomicAdd(&tu[a], 3u);
            else if (atomic == 3) atomicAdd(&tl[a >> 1], 3ull);
            else __hip_atomic_fetch_add(&gs[a], 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    long long t1 = clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    float s = 0.f;
    for (int i = threadIdx.x; i < 19200; i += 1024) s += tg[i];
    if (s == 12345.f) out[0] = s;
}

int main() {
    float *out, *gslab;
    long long *cyc;
    CHECK(hipMalloc(&out, 4));
    CHECK(hipMalloc(&cyc, 256 * 8));
    CHECK(hipMalloc(&gslab, 256L * 19200 * 4));
    const char *ops[] = {"ds_write", "ds_add_f32", "ds_add_u32", "ds_add_u64", "glb_add_f32", "glb_shared"};
    const char *names[] = {"consecutive", "0.62 cell/lane", "scattered", "same address", "stride 159"};
    for (int atomic = 0; atomic < 6; ++atomic)
        for (int p = 0; p < 5; ++p) {
            const int iters = atomic >= 4 ? 1024 : 8192;
            k<<<256, 1024>>>(p, atomic, 64, out, cyc, gslab);
            k<<<256, 1024>>>(p, atomic, iters, out, cyc, gslab);
            CHECK(hipDeviceSynchronize());
            long long c;
            CHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            printf("%-10s %-16s %7.1f cycles per wave-instruction per CU  (%5.1f lanes/clk/CU)\n",
                   ops[atomic], names[p], (double)c / (16.0 * iters),
                   16.0 * iters * 64 / (double)c);
        }
    return 0;
}
