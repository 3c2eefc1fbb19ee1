// HIP kernels for the AdaIN-VC embedding attack on MI355X (gfx950 / CDNA4),
// besides the Conv1d GEMM engine (avc_gemm.hip):
//
// se_head: mean pool + 6 dense blocks + output Linear + MSE loss + their input
//   gradient for 16 utterances per workgroup, on v_mfma_f32_16x16x4_f32.
//
// attack_init: ptb <- ptb0, m = v = 0, adv = vc + eps*tanh(ptb) (attack_utils.py:68,78).
#include <hip/hip_runtime.h>

#include "avc_device.h"
#include "avc_kernels.h"

namespace avc {

// ---------------------------------------------------------------------------------
// se_head
// ---------------------------------------------------------------------------------
constexpr int HU = 16;   // utterances per workgroup (the N of the 16x16x4 MFMA)

// Y[row][u] = act(sum_k W[row][k] X[k][u] + bias[row]) for rows of wave `wave`.
// Wpk: fragment-packed A, [M/16][K/4][64] with A[16*mt + (l&15)][4*kk + (l>>4)].
// mode: 0 = ReLU/LReLU (act), 2 = identity.
__device__ __forceinline__ void head_gemm(const float* __restrict__ Wpk, int M, int K,
                                          const float* X, float* Y, const float* __restrict__ bias,
                                          int act, bool apply_act, int wave, int lane) {
    if (wave * 16 >= M) return;
    const float* Wt = Wpk + (size_t)wave * (K / 4) * 64;
    // all of this wave's A fragments in flight at once (K <= 128 -> <= 32 per lane)
    float a[32];
#pragma unroll
    for (int kk = 0; kk < 32; ++kk) a[kk] = (4 * kk < K) ? Wt[kk * 64 + lane] : 0.f;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const int hh = lane >> 4, col = lane & 15;
#pragma unroll
    for (int kk = 0; kk < 32; kk += 2) {
        if (4 * kk < K) {
            const float b0 = X[(4 * kk + hh) * HU + col];
            const float b1 = X[(4 * kk + 4 + hh) * HU + col];
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk + 1], b1, acc1, 0, 0, 0);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = wave * 16 + 4 * hh + r;
        float v = acc0[r] + acc1[r];
        if (bias) v += bias[row];
        if (apply_act) v = act_f(v, act);
        Y[row * HU + col] = v;
    }
}

__global__ void __launch_bounds__(512) se_head(HeadArgs A) {
    extern __shared__ float smem[];
    const int C = A.C, D = A.D, nd = A.n_dense;
    const int CM = C > D ? C : D;
    const int S = CM * HU;
    float* E = smem;                 // running dense-block state e
    float* Ys = E + S;               // stash: y1_l, y2_l for l < nd
    float* EMB = Ys + 2 * nd * S;
    float* GA = EMB + S;
    float* GB = GA + S;
    float* GC = GB + S;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int u0 = blockIdx.x * HU;

    // AdaptiveAvgPool1d(1) (models.py:275,340)
    for (int idx = tid; idx < C * HU; idx += blockDim.x) {
        const int u = idx / C, c = idx - u * C;
        const int b = u0 + u;
        float s = 0.f;
        if (b < A.B) {
            const float* p = A.hN + ((size_t)b * C + c) * A.TN;
            for (int t = 0; t < A.TN; ++t) s += p[t];
            s = s / (float)A.TN;
        }
        E[c * HU + u] = s;
    }
    __syncthreads();

    // dense_blocks (models.py:307-325)
    const size_t CC = (size_t)C * C;
    for (int l = 0; l < nd; ++l) {
        float* Y1 = Ys + (2 * l) * S;
        float* Y2 = Ys + (2 * l + 1) * S;
        head_gemm(A.Wp + (2 * l) * CC, C, C, E, Y1, A.bias + (2 * l) * C, A.act, true, wave, lane);
        __syncthreads();
        head_gemm(A.Wp + (2 * l + 1) * CC, C, C, Y1, Y2, A.bias + (2 * l + 1) * C, A.act, true, wave, lane);
        __syncthreads();
        for (int idx = tid; idx < C * HU; idx += blockDim.x) E[idx] = Y2[idx] + E[idx];
        __syncthreads();
    }
    // output_layer (models.py:342)
    head_gemm(A.Wp + 2 * nd * CC, D, C, E, EMB, A.bias + 2 * nd * C, A.act, false, wave, lane);
    __syncthreads();

    if (A.mode == 0) {
        for (int idx = tid; idx < D * HU; idx += blockDim.x) {
            const int u = idx / D, d = idx - u * D;
            const int b = u0 + u;
            if (b < A.B) A.emb_out[(size_t)b * D + d] = EMB[d * HU + u];
        }
        return;
    }

    // loss = MSE(emb, tgt) - 0.1*MSE(emb, org) (attack_utils.py:81) and its gradient
    const int step = *A.step;
    if (tid < HU) {
        const int b = u0 + tid;
        if (b < A.B && A.losses && step >= 1 && step <= A.loss_len) {
            float s1 = 0.f, s2 = 0.f;
            for (int d = 0; d < D; ++d) {
                const float e = EMB[d * HU + tid];
                const float d1 = e - A.tgt[(size_t)b * D + d];
                const float d2 = e - A.org[(size_t)b * D + d];
                s1 += d1 * d1;
                s2 += d2 * d2;
            }
            A.losses[(size_t)(step - 1) * A.B + b] = s1 / (float)D - 0.1f * (s2 / (float)D);
        }
    }
    const float gscale = A.scal[1];
    for (int idx = tid; idx < D * HU; idx += blockDim.x) {
        const int d = idx / HU, u = idx - d * HU;
        const int b = u0 + u;
        float g = 0.f;
        if (b < A.B) {
            const float e = EMB[idx];
            g = gscale * (e - A.tgt[(size_t)b * D + d]) + gscale * (e - A.org[(size_t)b * D + d]) * -0.1f;
        }
        GA[idx] = g;
    }
    __syncthreads();

    // backward through output_layer and the dense blocks (input gradient only)
    const size_t offT_out = 2 * nd * CC;
    head_gemm(A.WpT + offT_out, C, D, GA, GB, nullptr, 0, false, wave, lane);   // g_e
    __syncthreads();
    for (int l = nd - 1; l >= 0; --l) {
        const float* Y1 = Ys + (2 * l) * S;
        const float* Y2 = Ys + (2 * l + 1) * S;
        for (int idx = tid; idx < C * HU; idx += blockDim.x) GC[idx] = GB[idx] * act_d(Y2[idx], A.act);
        __syncthreads();
        head_gemm(A.WpT + (2 * l + 1) * CC, C, C, GC, GA, nullptr, 0, false, wave, lane);
        __syncthreads();
        for (int idx = tid; idx < C * HU; idx += blockDim.x) GA[idx] = GA[idx] * act_d(Y1[idx], A.act);
        __syncthreads();
        head_gemm(A.WpT + (2 * l) * CC, C, C, GA, GC, nullptr, 0, false, wave, lane);
        __syncthreads();
        for (int idx = tid; idx < C * HU; idx += blockDim.x) GB[idx] = GB[idx] + GC[idx];
        __syncthreads();
    }
    // d/d hN of the mean over time
    const int TN = A.TN;
    for (int u = 0; u < HU && u0 + u < A.B; ++u) {
        const size_t off = (size_t)(u0 + u) * C * TN;
        for (int idx = tid; idx < C * TN; idx += blockDim.x) {
            const int c = idx / TN;
            const float g = GB[c * HU + u] / (float)TN;
            A.g_hN[off + idx] = g;
            A.g_hN_masked[off + idx] = g * act_d(A.mask_hN[off + idx], A.act);
        }
    }
}

__global__ void attack_init(const float* __restrict__ vc, const float* __restrict__ ptb0, float* ptb, float* m,
                            float* v, float* adv, float eps, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float p = ptb0[i];
    ptb[i] = p;
    m[i] = 0.f;
    v[i] = 0.f;
    adv[i] = vc[i] + eps * tanhf(p);
}

}  // namespace avc
