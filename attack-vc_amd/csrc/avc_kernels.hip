// HIP kernels for the AdaIN-VC embedding attack on MI355X (gfx950 / CDNA4).
//
// conv_gemm_f32<WM,WN>: every Conv1d of the SpeakerEncoder (models.py:82-104,
//   265-305) and every input-gradient (dgrad) of one, as an implicit GEMM on the
//   exact-f32 matrix cores (v_mfma_f32_32x32x2_f32):
//       C[M][N] = A[M][K] * B[K][N]     M = output channels, N = (utterance, t),
//                                       K = (input channel, tap)
//   A is a pre-packed weight matrix stored K-major ([K][Mpad]); B is the im2col
//   tile, never materialised in HBM: each K chunk is gathered straight into LDS
//   from the [B][C][T] activations, with reflect padding (forward), or with the
//   zero-dilated / tap-flipped / reflect-folded adjoint (dgrad).  Bias, ReLU,
//   residual avg-pool, ReLU' masks and the Adam update are fused into epilogues.
//   One launch can run several independent problems (blockIdx.z), e.g. all 8
//   conv-bank kernels of models.py:100-103.
//
// se_head: mean pool + 6 dense blocks + output Linear + MSE loss + their input
//   gradient for 16 utterances per workgroup, on v_mfma_f32_16x16x4_f32.
//
// attack_init: ptb <- ptb0, m = v = 0, adv = vc + eps*tanh(ptb) (attack_utils.py:68,78).
#include <hip/hip_runtime.h>

#include "avc_kernels.h"

namespace avc {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// get_act (models.py:107-118): 0 = ReLU, 1 = LeakyReLU(0.01)
__device__ __forceinline__ float act_f(float x, int act) {
    return x > 0.f ? x : (act ? 0.01f * x : 0.f);
}
// derivative expressed through the activation OUTPUT (same sign as its input)
__device__ __forceinline__ float act_d(float y, int act) {
    return y > 0.f ? 1.f : (act ? 0.01f : 0.f);
}

// Global-address-space views: pointers read out of the Problem table are generic,
// which would make every gather a flat_load (counted on lgkmcnt as well).
typedef const float __attribute__((address_space(1)))* gcptr;
__device__ __forceinline__ gcptr as_global(const float* p) { return (gcptr)p; }

// Index of dY for padded-output coordinate q of a stride-s conv; `ok` is false
// where the zero-dilation leaves a hole or q falls outside [0, T).  The caller
// loads row[idx] unconditionally (idx is clamped in range) and selects later, so
// no load waits inside the gather loop.  STRIDE = 0: runtime stride `rs`.
template <int STRIDE>
__device__ __forceinline__ int dy_index(int q, int rs, int T, bool& ok) {
    int qq = q;
    ok = q >= 0;
    if (STRIDE == 2) {
        ok = ok && !(q & 1);
        qq = q >> 1;
    } else if (STRIDE == 0 && rs != 1) {
        qq = q / rs;
        ok = ok && qq * rs == q;
    }
    ok = ok && qq < T;
    return ok ? qq : 0;
}

__device__ __forceinline__ void epilogue(const Problem& P, int m, int b, int t, float acc) {
    const int T = P.T_out;
    switch (P.epi) {
    case EPI_ACT: {
        float y = act_f(acc + P.bias[m], P.act);
        P.out0[((size_t)b * P.out0_C + P.out0_coff + m) * T + t] = y;
        break;
    }
    case EPI_BLOCK: {  // conv_blocks (models.py:299-304): y=act(conv2); out = y + avgpool(out)
        float a2 = act_f(acc + P.bias[m], P.act);
        P.out0[((size_t)b * P.out0_C + m) * T + t] = a2;
        const float* hin = P.aux0 + ((size_t)b * P.aux0_C + m) * P.aux0_T;
        float res;
        if (P.pool_s > 1) {
            const int lo = t * P.pool_s;
            const int hi = min(lo + P.pool_s, P.aux0_T);
            float s = 0.f;
            for (int q = lo; q < hi; ++q) s += hin[q];
            res = s / (float)(hi - lo);
        } else {
            res = hin[t];
        }
        P.out1[((size_t)b * P.out1_C + m) * T + t] = a2 + res;
        break;
    }
    case EPI_MASK: {
        float y = P.aux0[((size_t)b * P.aux0_C + m) * P.aux0_T + t];
        P.out0[((size_t)b * P.out0_C + m) * T + t] = acc * act_d(y, P.act);
        break;
    }
    case EPI_POOLT: {  // + d(avg_pool1d ceil_mode)/d(input) of the residual branch
        const float* g = P.aux0 + ((size_t)b * P.aux0_C + m) * P.aux0_T;
        float r;
        if (P.pool_s > 1) {
            const int q = t / P.pool_s;
            const int cnt = min(P.pool_s, T - q * P.pool_s);
            r = g[q] / (float)cnt;
        } else {
            r = g[t];
        }
        const float gv = acc + r;
        const size_t o = ((size_t)b * P.out0_C + m) * T + t;
        if (P.out0) P.out0[o] = gv;
        // masked copy = the next dgrad's dY (ReLU' of the forward activation aux1)
        if (P.out1) P.out1[o] = gv * act_d(P.aux1[o], P.act);
        break;
    }
    case EPI_INCONV_T: {  // split d(cat)/d: bank part gated by its ReLU, x part passes through
        if (m < P.split) {
            float y = P.aux0[((size_t)b * P.aux0_C + m) * P.aux0_T + t];
            P.out0[((size_t)b * P.out0_C + m) * T + t] = acc * act_d(y, P.act);
        } else {
            P.out1[((size_t)b * P.out1_C + (m - P.split)) * T + t] = acc;
        }
        break;
    }
    case EPI_ADAM: {
        // adv = vc + eps*tanh(ptb) backward (attack_utils.py:78) then torch.optim.Adam
        // _single_tensor_adam (torch/optim/adam.py): m.lerp_(g,1-b1);
        // v.mul_(b2).addcmul_(g,g,1-b2); p.addcdiv_(m, sqrt(v)/sqrt(bc2)+eps, -lr/bc1)
        const AdamArgs& A = P.adam;
        const size_t idx = ((size_t)b * P.M + m) * T + t;
        const float gadv = acc + P.aux0[idx];
        float p = A.ptb[idx];
        const float th = tanhf(p);
        const float eps = P.scal[0];
        const float g = (gadv * eps) * (1.f - th * th);
        const int step = min(max(*P.step, 1), P.table_len);
        if (A.grad0 && step == 1) A.grad0[idx] = g;
        float mm = A.m[idx];
        mm = mm + A.b1c * (g - mm);
        float vv = A.v[idx] * A.b2;
        vv = vv + A.b2c * g * g;
        const float nstep = A.table[2 * (step - 1)];
        const float bc2s = A.table[2 * (step - 1) + 1];
        const float denom = sqrtf(vv) / bc2s + A.adam_eps;
        p = p + nstep * (mm / denom);
        A.ptb[idx] = p;
        A.m[idx] = mm;
        A.v[idx] = vv;
        A.adv[idx] = A.vc[idx] + eps * tanhf(p);
        break;
    }
    default:
        break;
    }
}

template <int WM, int WN, int KC, int MODE, int STRIDE>
__global__ void __launch_bounds__(256) conv_gemm_f32(const Problem* __restrict__ probs) {
    constexpr int MT = 64 * WM, NT = 64 * WN;
    const Problem& P = probs[blockIdx.z];
    const int m0 = blockIdx.y * MT, n0 = blockIdx.x * NT;
    if (P.tick && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(P.tick, 1);
    if (m0 >= P.M || n0 >= P.N) return;

    constexpr int LDS_MAIN = KC * (MT + NT);
    __shared__ float lds[LDS_MAIN > 4096 ? LDS_MAIN : 4096];
    float* ldsA = lds;
    float* ldsB = lds + KC * MT;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int r32 = lane & 31, h = lane >> 5;

    const int N = P.N, T_out = P.T_out, Kend = P.K, Mpad = P.Mpad, nseg = P.nseg, act = P.act;
    const float* __restrict__ At = P.At;

    // B loader: lanes <-> columns n; each thread owns BPASS consecutive K rows of the
    // chunk, so (segment, c, j) is wave-uniform and advances by one tap per row.
    constexpr int BROWS = 256 / NT;
    constexpr int BPASS = KC / BROWS;
    const int nl = tid % NT;
    const int rg = __builtin_amdgcn_readfirstlane(tid / NT);
    const int n = n0 + nl;
    const bool nvalid = n < N;
    const int bb = nvalid ? n / T_out : 0;
    const int tt = nvalid ? n - bb * T_out : 0;

    constexpr int AF4 = KC * MT / 4 / 256;
    static_assert(BPASS <= 16, "validity mask packs 16 rows");
    f32x4 areg[AF4];
    float breg[BPASS];
    float ereg[MODE == SEG_BWD ? BPASS : 1];   // reflect-fold term of the adjoint gather
    unsigned vmask = 0u;                       // bit p: main term valid; bit 16+p: fold term valid
    const bool both_edges = MODE == SEG_BWD && P.both_edges;

    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const gcptr gAt = as_global(At);
    auto load_chunk = [&](int kc) {
        const int k0 = kc * KC;
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int f = tid + i * 256;
            const int r = f / (MT / 4), c4 = f % (MT / 4);
            areg[i] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
                gAt + (size_t)(k0 + r) * Mpad + m0 + 4 * c4);
        }
        // chunks never straddle segments (segments are padded to KSEG rows)
        int si = 0;
        while (si + 1 < nseg && k0 >= P.seg[si + 1].k0) ++si;
        const Seg& S = P.seg[si];
        const int ks = S.ks, pl = S.pl, srcT = S.src_T, C = S.C;
        const gcptr base = as_global(S.src) + ((size_t)bb * S.src_C + S.c_off) * srcT;
        const int kk0 = k0 - S.k0 + rg * BPASS;
        int c = kk0 / ks;
        int j = kk0 - c * ks;
        vmask = 0u;
#pragma unroll
        for (int p = 0; p < BPASS; ++p) {
            const bool live = c < C;                        // wave-uniform (padded rows are 0)
            const gcptr row = base + (size_t)(live ? c : 0) * srcT;
            if (MODE == SEG_FWD) {
                // x_pad[c][t*stride + j] of F.pad(mode="reflect") (models.py:23-29)
                const int st = STRIDE ? STRIDE : S.stride;
                int q = tt * st + j - pl;
                q = q < 0 ? -q : q;
                q = q >= srcT ? 2 * srcT - 2 - q : q;
                breg[p] = row[q];
                vmask |= (live ? 1u : 0u) << p;
            } else {
                // adjoint: dX[c][t] = sum_{co,j} W[co][c][j] sum_{p in pad^-1(t)} dY[co][(p-j)/s]
                // pad^-1(t) = {t+pl} u {pl-t : 1<=t<=pl} u {pl+2T-2-t : T-1-pr<=t<=T-2}
                const int rs = S.stride, pr = S.pr;
                bool ok0, ok1;
                const int i0 = dy_index<STRIDE>(tt + pl - j, rs, srcT, ok0);
                const bool left = tt >= 1 && tt <= pl;
                const bool right = tt >= T_out - 1 - pr && tt <= T_out - 2;
                // one fold term per lane (the left one if a tiny T_out <= pl+pr+1 gives both)
                const int qe = left ? pl - tt - j : (right ? pl + 2 * T_out - 2 - tt - j : -1);
                const int i1 = dy_index<STRIDE>(qe, rs, srcT, ok1);
                breg[p] = row[i0];
                ereg[p] = row[i1];
                if (both_edges) {   // tiny T only: here a waited load is acceptable
                    bool ok2;
                    const int i2 = dy_index<STRIDE>(left && right ? pl + 2 * T_out - 2 - tt - j : -1, rs, srcT, ok2);
                    const float e2 = row[i2];
                    ereg[p] = (ok1 ? ereg[p] : 0.f) + (ok2 ? e2 : 0.f);
                    ok1 = true;
                }
                vmask |= ((live && ok0) ? 1u : 0u) << p;
                vmask |= ((live && ok1) ? 1u : 0u) << (16 + p);
            }
            if (++j == ks) {
                j = 0;
                ++c;
            }
        }
    };
    auto store_chunk = [&]() {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int f = tid + i * 256;
            const int r = f / (MT / 4), c4 = f % (MT / 4);
            *reinterpret_cast<f32x4*>(&ldsA[r * MT + 4 * c4]) = areg[i];
        }
#pragma unroll
        for (int p = 0; p < BPASS; ++p) {
            float v = ((vmask >> p) & 1u) ? breg[p] : 0.f;
            if (MODE == SEG_BWD) v += ((vmask >> (16 + p)) & 1u) ? ereg[p] : 0.f;
            ldsB[(rg * BPASS + p) * NT + nl] = nvalid ? v : 0.f;
        }
    };

    const int nchunks = (Kend + KC - 1) / KC;
    load_chunk(0);
    for (int kc = 0; kc < nchunks; ++kc) {
        __syncthreads();
        store_chunk();
        __syncthreads();
        if (kc + 1 < nchunks) load_chunk(kc + 1);
#pragma unroll
        for (int s = 0; s < KC / 2; ++s) {
            const int kr = 2 * s + h;
            float a[WM], bv[WN];
#pragma unroll
            for (int i = 0; i < WM; ++i) a[i] = ldsA[kr * MT + wm * 32 * WM + 32 * i + r32];
#pragma unroll
            for (int j = 0; j < WN; ++j) bv[j] = ldsB[kr * NT + wn * 32 * WN + 32 * j + r32];
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int j = 0; j < WN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bv[j], acc[i][j], 0, 0, 0);
        }
    }

    // Epilogue through a per-wave 32x32 LDS stage: the C/D register map of the
    // 32x32 tile is col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5); staging
    // lets one compact (not unrolled) loop visit the tile row by row.
    __syncthreads();
    float* stage = lds + wave * 1024;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
#pragma unroll
        for (int j = 0; j < WN; ++j) {
#pragma unroll
            for (int r = 0; r < 16; ++r) stage[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + r32] = acc[i][j][r];
            const int ncol = n0 + wn * 32 * WN + 32 * j + r32;
            const bool cv = ncol < P.N;
            const int b = cv ? ncol / T_out : 0;
            const int t = ncol - b * T_out;
            const int mbase = m0 + wm * 32 * WM + 32 * i;
#pragma unroll 1
            for (int pass = 0; pass < 16; ++pass) {
                const int row = 2 * pass + h;
                const float v = stage[row * 32 + r32];
                if (cv && mbase + row < P.M) epilogue(P, mbase + row, b, t, v);
            }
        }
    }
}

#define AVC_INST_T(WM, WN, KC)                                                     \
    template __global__ void conv_gemm_f32<WM, WN, KC, SEG_FWD, 1>(const Problem*); \
    template __global__ void conv_gemm_f32<WM, WN, KC, SEG_FWD, 2>(const Problem*); \
    template __global__ void conv_gemm_f32<WM, WN, KC, SEG_FWD, 0>(const Problem*); \
    template __global__ void conv_gemm_f32<WM, WN, KC, SEG_BWD, 1>(const Problem*); \
    template __global__ void conv_gemm_f32<WM, WN, KC, SEG_BWD, 2>(const Problem*); \
    template __global__ void conv_gemm_f32<WM, WN, KC, SEG_BWD, 0>(const Problem*);
AVC_INST_T(2, 2, 32)
AVC_INST_T(2, 2, 16)
AVC_INST_T(2, 1, 32)
AVC_INST_T(1, 1, 32)
AVC_INST_T(1, 1, 16)
#undef AVC_INST_T

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
