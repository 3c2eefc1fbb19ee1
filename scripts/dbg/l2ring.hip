// Microbenchmark: per-CU streaming rate of an L2-resident weight set (the fused kernels' A operands)
// through a CONTINUOUS register ring -- D 1-KiB wave loads in flight per wave at all times, each
// consumed D loads after its issue (a counted vmcnt wait, never a drain) -- for W waves per
// workgroup, one workgroup per CU.  (scripts/dbg/l2stream.hip drained every batch of D loads, so it
// measured latency-bound batches, not the stream.)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int D, int W>
__global__ void __launch_bounds__(64 * W) ring(const f32x4* __restrict__ Wt, size_t n4, float* out) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const size_t per_w = n4 / W;
    const int chunks = (int)(per_w / 64);                    // 1 KiB chunks per wave
    const f32x4* base = Wt + w * per_w + l;
    f32x4 r[D];
    f32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int d = 0; d < D; ++d) r[d] = base[(size_t)d * 64];
    for (int c = D; c < chunks + D; c += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            acc += r[d];                                     // waits for the oldest load only
            const int cc = c + d < chunks ? c + d : chunks - 1;
            r[d] = base[(size_t)cc * 64];
        }
    }
    if (acc[0] == 1.2345f) out[0] = acc[1];
}

int main() {
    const size_t S = 3400 * 1024;
    const size_t n4 = S / 16;
    f32x4* Wt;
    float* out;
    hipMalloc(&Wt, S);
    hipMalloc(&out, 4);
    hipMemset(Wt, 0, S);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](auto kern, int D, int W, int G) {
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(G), dim3(64 * W), 0, 0, Wt, n4, out);
        hipEventRecord(a);
        const int R = 10;
        for (int i = 0; i < R; ++i) hipLaunchKernelGGL(kern, dim3(G), dim3(64 * W), 0, 0, Wt, n4, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / R;
        printf("waves/WG=%d D=%2d G=%d: %.1f us per pass, %.1f GB/s per workgroup (%.1f B/clk at 2.4 GHz), %.2f TB/s\n",
               W, D, G, us, S / (us * 1e-6) / 1e9, S / (us * 1e-6) / 2.4e9, (double)G * S / (us * 1e-6) / 1e12);
    };
    run(ring<4, 4>, 4, 4, 256);
    run(ring<8, 4>, 8, 4, 256);
    run(ring<16, 4>, 16, 4, 256);
    run(ring<24, 4>, 24, 4, 256);
    run(ring<32, 4>, 32, 4, 256);
    run(ring<8, 8>, 8, 8, 256);
    run(ring<16, 8>, 16, 8, 256);
    run(ring<16, 4>, 16, 4, 64);
    run(ring<32, 4>, 32, 4, 64);
    return 0;
}
