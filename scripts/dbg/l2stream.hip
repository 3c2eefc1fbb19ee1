// Microbenchmark: per-CU streaming rate of L2-resident weights (the fused kernels' A
// operands) vs loads in flight per thread.  256 workgroups x 256 threads; every
// workgroup streams the same S-byte buffer (each wave a contiguous quarter) as 1 KiB
// coalesced wave loads, D loads in flight per lane; STAG=1 staggers each workgroup's start.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int D>
__global__ void __launch_bounds__(256) stream(const f32x4* __restrict__ W, size_t n4, int stag, float* out) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const size_t per_w = n4 / 4;                 // f32x4 per wave
    const size_t chunks = per_w / 64;            // 1 KiB chunks per wave
    const size_t start = stag ? (size_t)(blockIdx.x * 37) % chunks : 0;
    const f32x4* base = W + w * per_w + l;
    f32x4 acc = {0, 0, 0, 0};
    for (size_t c0 = 0; c0 < chunks; c0 += D) {
        f32x4 v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            size_t c = c0 + d + start;
            if (c >= chunks) c -= chunks;
            v[d] = base[c * 64];
        }
#pragma unroll
        for (int d = 0; d < D; ++d) acc += v[d];
    }
    if (acc[0] == 1.2345f) out[0] = acc[1];
}

// the same stream as LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction into a
// per-wave LDS ring of D KiB): does the per-wave rate differ from register loads?
template <int D>
__global__ void __launch_bounds__(256) stream_lds(const f32x4* __restrict__ W, size_t n4, int stag, float* out) {
    __shared__ __attribute__((aligned(16))) char ring[4][D][1024];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const size_t per_w = n4 / 4;
    const size_t chunks = per_w / 64;
    const f32x4* base = W + w * per_w + l;
    for (size_t c0 = 0; c0 < chunks; c0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            size_t c = c0 + d;
            if (c >= chunks) c -= chunks;
            __builtin_amdgcn_global_load_lds((const void*)(base + c * 64), (__attribute__((address_space(3))) void*)&ring[w][d][0], 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (reinterpret_cast<float*>(ring[w][0])[l] == 1.2345f) out[0] = 1.f;
}

int main() {
    const size_t S = 3400 * 1024;                // bytes (SE weights, bf16)
    const size_t n4 = S / 16;
    f32x4* W;
    float* out;
    hipMalloc(&W, S);
    hipMalloc(&out, 4);
    hipMemset(W, 0, S);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int G = 256;   // workgroups (one per CU at 256)
    auto run = [&](auto kern, int D, int stag) {
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, 0, W, n4, stag, out);
        hipEventRecord(a);
        const int R = 10;
        for (int i = 0; i < R; ++i) hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, 0, W, n4, stag, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / R;
        printf("G=%3d D=%2d stag=%d: %.1f us per pass, %.1f GB/s per workgroup, %.2f TB/s aggregate\n", G, D, stag, us,
               S / (us * 1e-6) / 1e9, (double)G * S / (us * 1e-6) / 1e12);
    };
    // all CUs, half of them (one workgroup on every other CU slot), a quarter: is the shared
    // stream bound per CU or by the XCD L2s together?
    for (int g : {256, 128, 64, 512}) {
        G = g;
        run(stream<8>, 8, 0);
        run(stream<16>, 16, 0);
        run(stream<16>, 16, 1);
        run(stream_lds<8>, -8, 0);
        run(stream_lds<16>, -16, 0);
    }
    return 0;
}
