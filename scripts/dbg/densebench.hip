// Microbenchmark: where dense_mfma's ~9.5 us per conv_affine call (M=3072, K=128, B=256 fp32,
// avc_vc.hip) goes.  The kernel body is dense_mfma's (16 rows x 16 NJ utterances per wave, U 16-k
// steps per load round); MODE strips parts of it: 0 full, 1 loads + stores only (no MFMA),
// 2 MFMA + stores only (operands from the lane id), 3 stores only; plus bf16 16x16x32 and an
// empty kernel.  Each variant: 200 back-to-back launches timed by events, and a 50-launch graph.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstring>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct DA { const float* A; const float* X; const float* bias; float* Y; int M, K, B; };

template <int NJ, int U, int MODE>
__global__ void __launch_bounds__(256) dense(DA D) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r16 = l & 15, kq = l >> 4;
    const int m0 = blockIdx.x * 64 + 16 * w, b0 = blockIdx.y * 16 * NJ;
    const int kb = 0, ke = D.K;
    const float* Ar = D.A + (size_t)min(m0 + r16, D.M - 1) * D.K;
    const float* Xr[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) Xr[j] = D.X + (size_t)min(b0 + 16 * j + r16, D.B - 1) * D.K;
    f32x4 ca[U], cx[NJ][U], na[U], nx[NJ][U];
    auto load = [&](int s0, f32x4 (&a)[U], f32x4 (&x)[NJ][U]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = kb + 16 * (s0 + u) + 4 * kq;
            if (MODE == 0 || MODE == 1) {
                a[u] = *reinterpret_cast<const f32x4*>(Ar + k);
#pragma unroll
                for (int j = 0; j < NJ; ++j) x[j][u] = *reinterpret_cast<const f32x4*>(Xr[j] + k);
            } else {
                a[u] = f32x4{(float)l, (float)k, 1.f, 2.f};
#pragma unroll
                for (int j = 0; j < NJ; ++j) x[j][u] = f32x4{(float)j, (float)k, 1.f, 2.f};
            }
        }
    };
    f32x4 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int ns = (ke - kb + 15) / 16;
    load(0, ca, cx);
    for (int s = 0; s < ns; s += U) {
        if (s + U < ns) load(s + U, na, nx);
        if (MODE == 0 || MODE == 2) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[u][e], cx[j][u][e], acc[j], 0, 0, 0);
        } else if (MODE == 1) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[j] += ca[u] * cx[j][u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ca[u] = na[u];
#pragma unroll
            for (int j = 0; j < NJ; ++j) cx[j][u] = nx[j][u];
        }
    }
    const int m = m0 + 4 * kq;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int bb = b0 + 16 * j + r16;
        if (bb >= D.B) continue;
        *reinterpret_cast<f32x4*>(D.Y + (size_t)bb * D.M + m) = acc[j] + f32x4{D.bias[m], D.bias[m + 1], D.bias[m + 2], D.bias[m + 3]};
    }
}

// bf16 operands (converted on load), 16x16x32 MFMA: 4 MFMAs per tile over K = 128
template <int NJ>
__global__ void __launch_bounds__(256) dense_bf(DA D) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r16 = l & 15, kq = l >> 4;
    const int m0 = blockIdx.x * 64 + 16 * w, b0 = blockIdx.y * 16 * NJ;
    const float* Ar = D.A + (size_t)min(m0 + r16, D.M - 1) * D.K;
    f32x4 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < D.K; k0 += 32) {
        const int k = k0 + 8 * kq;
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(Ar + k), a1 = *reinterpret_cast<const f32x4*>(Ar + k + 4);
        bf16x8 a;
        for (int e = 0; e < 4; ++e) { a[e] = (__bf16)a0[e]; a[4 + e] = (__bf16)a1[e]; }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const float* xr = D.X + (size_t)min(b0 + 16 * j + r16, D.B - 1) * D.K + k;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(xr), x1 = *reinterpret_cast<const f32x4*>(xr + 4);
            bf16x8 x;
            for (int e = 0; e < 4; ++e) { x[e] = (__bf16)x0[e]; x[4 + e] = (__bf16)x1[e]; }
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, x, acc[j], 0, 0, 0);
        }
    }
    const int m = m0 + 4 * kq;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int bb = b0 + 16 * j + r16;
        if (bb >= D.B) continue;
        *reinterpret_cast<f32x4*>(D.Y + (size_t)bb * D.M + m) = acc[j];
    }
}


// X and A tiles staged through LDS by contiguous 16-B loads (one round, each byte once per
// workgroup), then dense_mfma's exact MFMA sequence from LDS fragments
constexpr int LKC = 128, LST = LKC + 4;
template <int NJ>
__global__ void __launch_bounds__(256) dense_lds(DA D) {
    extern __shared__ float lds[];
    float* As = lds;
    float* Xs = lds + 64 * LST;
    const int t = threadIdx.x, w = t >> 6, l = t & 63, r16 = l & 15, kq = l >> 4;
    const int mb = blockIdx.x * 64, b0 = blockIdx.y * 16 * NJ;
    const int kb = 0, ke = D.K, kc = ke - kb;
    constexpr int NA = 64 * LKC / 4, NX = 16 * NJ * LKC / 4, NT = (NA + NX) / 256;
    f32x4 v[NT];
#pragma unroll
    for (int r = 0; r < NT; ++r) {
        const int i = t + 256 * r;
        const bool isA = i < NA;
        const int ii = isA ? i : i - NA, row = ii / (LKC / 4), k = 4 * (ii % (LKC / 4));
        const float* src = isA ? D.A + (size_t)min(mb + row, D.M - 1) * D.K
                               : D.X + (size_t)min(b0 + row, D.B - 1) * D.K;
        v[r] = k + 4 <= kc ? *reinterpret_cast<const f32x4*>(src + kb + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int r = 0; r < NT; ++r) {
        const int i = t + 256 * r;
        const bool isA = i < NA;
        const int ii = isA ? i : i - NA, row = ii / (LKC / 4), k = 4 * (ii % (LKC / 4));
        *reinterpret_cast<f32x4*>((isA ? As : Xs) + row * LST + k) = v[r];
    }
    __syncthreads();
    f32x4 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* ar = As + (16 * w + r16) * LST + 4 * kq;
    const int ns = (kc + 15) / 16;
#pragma unroll 4
    for (int s = 0; s < ns; ++s) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(ar + 16 * s);
        f32x4 x[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) x[j] = *reinterpret_cast<const f32x4*>(Xs + (16 * j + r16) * LST + 16 * s + 4 * kq);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], x[j][e], acc[j], 0, 0, 0);
    }
    const int m = mb + 16 * w + 4 * kq;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int bb = b0 + 16 * j + r16;
        if (bb >= D.B) continue;
        *reinterpret_cast<f32x4*>(D.Y + (size_t)bb * D.M + m) = acc[j] + f32x4{D.bias[m], D.bias[m + 1], D.bias[m + 2], D.bias[m + 3]};
    }
}

__global__ void empty_k(DA D) { if (D.M < 0) D.Y[0] = 1.f; }

template <typename F>
static int timeit(const char* name, F launch, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipEventRecord(a, s));
    for (int i = 0; i < 200; ++i) launch();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 50; ++i) launch();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float gms = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float t; CK(hipEventElapsedTime(&t, a, b));
        gms = t < gms ? t : gms;
    }
    printf("%-28s stream %7.2f us/launch   graph %7.2f us/launch\n", name, ms * 1e3f / 200, gms * 1e3f / 50);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    return 0;
}

int main() {
    const int M = 3072, K = 128, B = 256;
    float *A, *X, *bias, *Y;
    CK(hipMalloc(&A, (size_t)M * K * 4)); CK(hipMalloc(&X, (size_t)B * K * 4));
    CK(hipMalloc(&bias, M * 4)); CK(hipMalloc(&Y, (size_t)B * M * 4));
    std::vector<float> h((size_t)M * K);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
    CK(hipMemcpy(A, h.data(), (size_t)M * K * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(X, h.data(), (size_t)B * K * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(bias, h.data(), M * 4, hipMemcpyHostToDevice));
    hipStream_t s; CK(hipStreamCreate(&s));
    DA d{A, X, bias, Y, M, K, B};
#define RUN(NAME, KER, NJ) timeit(NAME, [&] { hipLaunchKernelGGL(KER, dim3(M / 64, B / (16 * NJ)), dim3(256), 0, s, d); }, s)
    RUN("empty (grid 48x4)", empty_k, 4);
    RUN("f32 NJ4 U4 full", (dense<4, 4, 0>), 4);
    RUN("f32 NJ2 U4 full", (dense<2, 4, 0>), 2);
    RUN("f32 NJ1 U4 full", (dense<1, 4, 0>), 1);
    RUN("f32 NJ4 U8 full", (dense<4, 8, 0>), 4);
    RUN("f32 NJ4 loads+stores", (dense<4, 4, 1>), 4);
    RUN("f32 NJ4 mfma+stores", (dense<4, 4, 2>), 4);
    RUN("f32 NJ2 mfma+stores", (dense<2, 4, 2>), 2);
    RUN("f32 NJ4 stores only", (dense<4, 4, 3>), 4);
    RUN("bf16 NJ4", dense_bf<4>, 4);
    RUN("bf16 NJ2", dense_bf<2>, 2);
    RUN("bf16 NJ1", dense_bf<1>, 1);
#define RUNL(NAME, NJ) timeit(NAME, [&] { hipLaunchKernelGGL(dense_lds<NJ>, dim3(M / 64, B / (16 * NJ)), dim3(256), (64 + 16 * NJ) * LST * 4, s, d); }, s)
    RUNL("lds NJ4", 4);
    RUNL("lds NJ2", 2);
    RUNL("lds NJ1", 1);
    // bitwise check of the LDS kernels against dense<4,4,0>
    std::vector<float> y0((size_t)B * M), y1((size_t)B * M);
    hipLaunchKernelGGL((dense<4, 4, 0>), dim3(M / 64, B / 64), dim3(256), 0, s, d);
    CK(hipMemcpy(y0.data(), Y, y0.size() * 4, hipMemcpyDeviceToHost));
    for (int nj : {1, 2, 4}) {
        CK(hipMemset(Y, 0, y1.size() * 4));
        if (nj == 1) hipLaunchKernelGGL(dense_lds<1>, dim3(M / 64, B / 16), dim3(256), (64 + 16) * LST * 4, s, d);
        if (nj == 2) hipLaunchKernelGGL(dense_lds<2>, dim3(M / 64, B / 32), dim3(256), (64 + 32) * LST * 4, s, d);
        if (nj == 4) hipLaunchKernelGGL(dense_lds<4>, dim3(M / 64, B / 64), dim3(256), (64 + 64) * LST * 4, s, d);
        CK(hipMemcpy(y1.data(), Y, y1.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < y0.size(); ++i) bad += memcmp(&y0[i], &y1[i], 4) != 0;
        printf("lds NJ%d vs dense<4,4,0>: %zu differing of %zu\n", nj, bad, y0.size());
    }
    CK(hipDeviceSynchronize());
    printf("DONE\n");
    return 0;
}
