// The embedding head of the fused SpeakerEncoder kernels (avc_fused.hip): the standard shape's
// compile-time constants and the in-kernel head chain
// (time-mean -> dense blocks -> output Linear -> loss -> backward); see avc_fused.hip.
#pragma once
#include "avc_fused_core.h"

namespace avc {

struct StdSE {
    static constexpr int T = 128, NB = 8, KSZ = 5, NBLK = 6, NDENSE = 6;
    static constexpr int sub(int l) { return (l & 1) ? 2 : 1; }
    static constexpr int Tl(int l) {
        int t = T;
        for (int i = 0; i < l; ++i) t = (t + sub(i) - 1) / sub(i);
        return t;
    }
    static constexpr int nf(int frames) { return (frames + 15) / 16; }
    // block l's input length for an utterance of T frames (a ragged batch's per-workgroup length)
    __host__ __device__ static constexpr int Tl_of(int T, int l) {
        int t = T;
        for (int i = 0; i < l; ++i) t = (t + sub(i) - 1) / sub(i);
        return t;
    }
};


// ---------------------------------------------------------------------------------
// Embedding-attack head in the forward's tail (bf16 mode, c_h = c_out = 128): time-mean
// -> 2*nd dense layers -> output Linear -> loss (attack_utils.py:81-82) -> backward to
// d loss / d time-mean, for THIS workgroup's utterance.  The same chain, per-element
// arithmetic and summation order as se_head_v mode 1 (avc_kernels.hip), which it
// replaces for the emb attack: that launch is a latency-bound 26-step chain on 128 CUs
// between the two conv kernels; here every CU streams the 13 matrices itself (832 KB of
// bf16 per utterance) while its conv-stack LDS is dead.  Thread u owns rows u/4 and
// u/4 + 64 with K slice u%4 -- se_head_v's threads u and u + 256 -- so se_head_v's
// packed bf16 weights are used as they are.
// ---------------------------------------------------------------------------------
typedef unsigned hu32x4 __attribute__((ext_vector_type(4)));
struct HW16 {
    hu32x4 r[4];   // 32 bf16 weights of one row slice, 8 per 16-byte chunk
};
__device__ __forceinline__ float hw16_w(const HW16& hw, int e, int j) {
    const int f = 4 * e + j, cc = f >> 3, i = f & 7;
    const unsigned word = hw.r[cc][i >> 1];
    return __builtin_bit_cast(float, (i & 1) ? (word & 0xffff0000u) : (word << 16));
}
// Head vectors in LDS are stored slice-major: element k at hpos(k) = q*36 + 2i + e
// (k = 8i + 2q + e), so slice q's 32 inputs are one contiguous run read as eight
// 16-byte loads; the 36-float slice stride puts the four slices of a wave's broadcast
// reads on distinct banks.
constexpr int HVS = 4 * 36;   // floats per head vector
__device__ __forceinline__ int hpos(int k) { return ((k >> 1) & 3) * 36 + 2 * (k >> 3) + (k & 1); }
// sum_k W[m][k] X[k] over this lane's K slice, then over the row's 4 slices (DPP)
__device__ __forceinline__ float head_dot(const HW16& hw, const float* X, int q) {
#pragma clang fp contract(off)
    // the even / odd k of each pair accumulate separately (se_head_v's order) -- as the two
    // lanes of one packed fma (v_pk_fma_f32: each lane an IEEE fma, so bitwise the same sums)
    f32x2 acc2v = {0.f, 0.f};
    const f32x4* X4 = reinterpret_cast<const f32x4*>(X + q * 36);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const f32x4 x = X4[e];     // pairs i = 2e (x0, x1) and i = 2e + 1 (x2, x3), k = 8i + 2q
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f32x2 wv = {hw16_w(hw, e, 2 * h), hw16_w(hw, e, 2 * h + 1)};
            acc2v = __builtin_elementwise_fma(wv, f32x2{x[2 * h], x[2 * h + 1]}, acc2v);
        }
    }
    float acc = acc2v[0] + acc2v[1];
    acc += dpp_mov<0xB1>(acc);
    acc += dpp_mov<0x4E>(acc);
    return acc;
}
// sm: LDS floats, E (the time-mean, [128]) already written by the caller.  ND = n_dense
// (compile-time: the 2*(2*ND+1) chain steps are straight-line code, so the 3-step weight
// ring stays in flight across the per-step barriers -- a runtime loop made the compiler
// copy the ring registers at the loop head and drain it with vmcnt(0) every iteration).
// Per-row state a thread needs again (biases, targets, the forward activations for the
// act' masks, E and GB of its own rows) stays in registers; LDS only carries the vectors
// every thread reads (E, Y_i, GA, GM).
// MODE 1: the emb attack's chain (forward, loss, backward to g_pooled);  MODE 0: forward only
// (e2e / fb: the embedding for the Decoder), storing the dense activations for MODE 3;
// MODE 3: backward only, from d loss / d emb (the split-K slices at H.tgt, summed in slice
// order) with the MODE-0 activations, leaving g_pooled in sm[hpos(c)] (se_head_v modes 1/0/3).
// NTH = 256 (a 4-wave workgroup: thread u owns rows u/4 and u/4 + 64) or 512 (8 waves: row u/4 only,
// se_head_v's own mapping); the per-row arithmetic and summation order are the same either way.
template <int ND, int MODE = 1, int NTH = 256>
__device__ __forceinline__ void se_head_fused(const HeadArgs& H, int b, float* sm, float* loss_cur) {
#pragma clang fp contract(off)
    static_assert(NTH == 256 || NTH == 512, "head thread count");
    constexpr int HR = 512 / NTH;                   // rows per thread
    constexpr int C = FZ_C, D = FZ_C;
    constexpr size_t CC = (size_t)C * C;
    constexpr int NF = 2 * ND + 1, NL = 2 * NF;
    constexpr int I0 = MODE == 3 ? NF : 0;          // first chain step
    constexpr int I1 = MODE == 0 ? NF : NL;         // one past the last
    const int act = H.act;
    const int tid = threadIdx.x, q = tid & 3, m0 = tid >> 2, ln = tid & 63, wv = tid >> 6;
    const bool own = q == 0;
    float* E = sm;                     // head vectors: HVS floats each, slice-major (hpos)
    float* Ys = E + HVS;               // [2ND][HVS]
    float* GA = Ys + 2 * ND * HVS;
    float* GB = GA + HVS;              // loss scratch only
    float* GM = GB + HVS;
    float* LS = GM + HVS;
    const uint16_t* __restrict__ W16 = H.Wr16;
    const uint16_t* __restrict__ WT16 = H.WrT16;
    // rows m0 + 64 h (se_head_v thread tid + 256 h: wave wv + 4 h), h < HR
    auto load_w = [&](HW16 (&hw)[HR], auto I) __attribute__((always_inline)) {
        constexpr int i = decltype(I)::value;
        constexpr int j = i - NF - 1, l = ND - 1 - j / 2;
        const uint16_t* base = i < NF ? W16 + (size_t)i * CC                       // dense, then output
                                      : (i == NF ? WT16 + (size_t)(2 * ND) * CC     // output^T
                                                 : WT16 + (size_t)(j % 2 == 0 ? 2 * l + 1 : 2 * l) * CC);
#pragma unroll
        for (int h = 0; h < HR; ++h)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
#if AVC_FZ_ABLATE & 16
                hw[h].r[cc] = hu32x4{(unsigned)i, 3u, 5u, (unsigned)cc};   // timing only: no weight loads
#else
                hw[h].r[cc] = gload<hu32x4>(reinterpret_cast<const float*>(
                    base + ((size_t)((wv + 4 * h) * 4 + cc) * 64 + ln) * 8));
#endif
    };
    float bias[NF][HR] = {}, tg[HR] = {}, og[HR] = {};
    float e_own[HR] = {}, gb_own[HR] = {}, ys[2 * ND][HR];
#pragma unroll
    for (int h = 0; h < HR; ++h) {
        const int m = m0 + 64 * h;
        if constexpr (MODE != 3) {
#pragma unroll
            for (int i = 0; i < NF; ++i) bias[i][h] = H.bias[i * C + m];
        }
        if constexpr (MODE == 1) {
            tg[h] = H.tgt[(size_t)b * D + m];
            og[h] = H.org[(size_t)b * D + m];
        }
        if constexpr (MODE == 3) {
#pragma unroll
            for (int i = 0; i < 2 * ND; ++i) ys[i][h] = H.act_in[((size_t)b * 2 * ND + i) * C + m];
            if (own) {   // d loss / d emb: the slices summed in order (se_head_v mode 3)
                const int np = H.tgt_parts > 0 ? H.tgt_parts : 1;
                float g = 0.f;
                for (int q2 = 0; q2 < np; ++q2) g += H.tgt[((size_t)q2 * H.B + b) * D + m];
                GA[hpos(m)] = g;
            }
        }
    }
    const float gscale = MODE == 1 ? H.scal[1] : 0.f;
    const float lam = MODE == 1 ? H.scal[4] : 0.f;   // weight of the org term (0.1 in the attacks)
    HW16 w0[HR], w1[HR], w2[HR];
    load_w(w0, IC<I0>{});
    load_w(w1, IC<I0 + 1>{});
    load_w(w2, IC<I0 + 2>{});
    __syncthreads();
    if constexpr (MODE != 3) {
#pragma unroll
        for (int h = 0; h < HR; ++h) e_own[h] = E[hpos(m0 + 64 * h)];
    }

    auto run_step = [&](auto I, const HW16 (&hw)[HR]) __attribute__((always_inline)) {
        constexpr int i = decltype(I)::value;
        constexpr int j = i - NF - 1, l = ND - 1 - j / 2;
        const float* X = i < 2 * ND ? ((i % 2 == 0) ? E : Ys + (i - 1) * HVS)
                                    : (i == 2 * ND ? E : (i == NF ? GA : (j % 2 == 0 ? GM : GA)));
        float o[HR];
#pragma unroll
        for (int h = 0; h < HR; ++h) o[h] = head_dot(hw[h], X, q);
#pragma unroll
        for (int h = 0; h < HR; ++h) {
            const int m = m0 + 64 * h;
            if constexpr (i < 2 * ND) {
                const float y = act_f(o[h] + bias[i][h], act);
                ys[i][h] = y;
                if (own) Ys[i * HVS + hpos(m)] = y;
                if constexpr (MODE == 0)
                    if (own) H.act_out[((size_t)b * 2 * ND + i) * C + m] = y;
                if constexpr (i % 2 == 1) {
                    e_own[h] = y + e_own[h];
                    if (own) E[hpos(m)] = e_own[h];
                }
            } else if constexpr (i == 2 * ND && MODE == 0) {
                if (own) H.emb_out[(size_t)b * D + m] = o[h] + bias[2 * ND][h];
            } else if constexpr (i == 2 * ND) {
                // loss = MSE(emb, tgt) - 0.1 MSE(emb, org) (attack_utils.py:81-82)
                const float e = o[h] + bias[2 * ND][h];
                const float d1 = e - tg[h], d2 = e - og[h];
                if (own) {
                    GA[hpos(m)] = gscale * d1 + gscale * d2 * -lam;
                    GB[hpos(m)] = d1 * d1;
                    GM[hpos(m)] = d2 * d2;
                }
            } else if constexpr (i == NF) {
                gb_own[h] = o[h];
                if (own) GM[hpos(m)] = o[h] * act_d(ys[2 * ND - 1][h], act);
            } else if constexpr (j % 2 == 0) {
                if (own) GA[hpos(m)] = o[h] * act_d(ys[2 * l][h], act);
            } else {
                gb_own[h] = gb_own[h] + o[h];
                if constexpr (l > 0)
                    if (own) GM[hpos(m)] = gb_own[h] * act_d(ys[2 * l - 1][h], act);
            }
        }
        if constexpr (i == 2 * ND && MODE == 1) {
            __syncthreads();
            if (tid < 64) {   // per-utterance loss, fixed summation order (se_head_v's)
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int d = 0; d < D; d += 64) {
                    s1 += GB[hpos(d + tid)];
                    s2 += GM[hpos(d + tid)];
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) {
                    s1 += __shfl_xor(s1, off);
                    s2 += __shfl_xor(s2, off);
                }
                if (tid == 0) LS[0] = s1 / (float)D - lam * (s2 / (float)D);
            }
        }
        __syncthreads();
    };
    // 3-step register ring: slot (i - I0) % 3 holds step i and is refilled with step i + 3
    static_for<I0, I1>([&](auto I) __attribute__((always_inline)) {
        constexpr int i = decltype(I)::value;
        auto step = [&](HW16 (&slot)[HR]) __attribute__((always_inline)) {
            run_step(I, slot);
            if constexpr (i + 3 < I1) load_w(slot, IC<i + 3>{});
        };
        if constexpr ((i - I0) % 3 == 0) step(w0);
        else if constexpr ((i - I0) % 3 == 1) step(w1);
        else step(w2);
    });
    if constexpr (MODE == 1) {
        if (own)
#pragma unroll
            for (int h = 0; h < HR; ++h) H.g_pooled[(size_t)b * C + m0 + 64 * h] = gb_own[h];
        if (tid == 0) loss_cur[b] = LS[0];
    } else if constexpr (MODE == 3) {
        if (own)   // g_pooled for the conv stack's backward, in LDS (E is dead); caller syncs
#pragma unroll
            for (int h = 0; h < HR; ++h) E[hpos(m0 + 64 * h)] = gb_own[h];
    }
}


}  // namespace avc
