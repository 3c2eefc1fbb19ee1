// 8-wave fused SpeakerEncoder forward (bf16, the config.yaml shape at T = 128): the 4-wave engine of
// avc_fused.hip with two waves per SIMD.
//
// Why: one workgroup owns one utterance and B = 256 puts exactly one on every CU, so the 4-wave
// engine runs ONE wave per SIMD.  Its GEMMs are co-bound by MFMA and by the per-wave L2 weight
// stream (~8.5 B/clk per wave, DESIGN.md 9: 4 waves pull ~34 B/clk per CU, 8 waves ~50), and nothing
// hides an epilogue, a barrier or an L2 round trip behind another wave's matrix work.
//
// Mapping: wave wv = 4 hh + w.  w (0..3) owns output channels [32 w, 32 w + 32) of every 128-channel
// layer, as before; hh (0, 1) owns HALF of the layer's 16-frame fragments (frames [64 hh, 64 hh + 64)
// at T = 128, halving with every stride-2 block).  Waves w and w + 4 share a SIMD and stream the same
// A tiles (the second read is an L1 hit); each B fragment is read by one wave only.  A stride-2
// block's pooled residual for output half hh comes from input half hh, except in the last block
// (32 -> 16 frames, one output fragment), whose odd input fragment is handed over through LDS.
//
// Every output element is accumulated by one wave with the same MFMA sequence over K as in the
// 4-wave kernel, the epilogues are the same per-element operations and the head is se_head_fused
// with one row per thread (its per-row arithmetic unchanged): the results are bitwise those of
// se_fwd_fused<bf16, 0>.  The ReLU' bits go out in se_bwd8's layout: per (layer, wave) one u32 per
// lane, bit 16 i + 4 f + r for tile i, local fragment f, row r.
#include "avc_fused_core.h"
#include "avc_se_head.h"

#ifndef AVC_FZ8_RD
#define AVC_FZ8_RD 8
#endif

namespace avc {

constexpr int F8_MASK_U32_PER_LAYER = 2 * FZ_MASK_WORDS_PER_LAYER;   // a layer's slot of the mask words, as u32

// ReLU' bits of one (layer, wave) for the 8-wave kernels: bit 16 i + 4 f + r, f < 4 local fragments
struct MaskAcc8 {
    unsigned m = 0;
    __device__ __forceinline__ void put(int i, int f, int r, float y) {
        unsigned bit;
        asm("v_med3_i32 %0, %1, 0, 1" : "=v"(bit) : "v"(y));
        m |= bit << (16 * i + 4 * f + r);
    }
    __device__ __forceinline__ void store(u64* mbase, int layer, int wv) const {
        reinterpret_cast<unsigned*>(mbase)[(size_t)layer * F8_MASK_U32_PER_LAYER + wv * 64 + (threadIdx.x & 63)] = m;
    }
};

template <int PREC>
__global__ void __launch_bounds__(512, 1) se_fwd8(FusedArgs A) {
    static_assert(PREC == PREC_BF16, "the 8-wave engine is the bf16 bench path");
    using S = StdSE;
    using E = typename Fz<PREC>::E;
    constexpr int RS = Fz<PREC>::RS;
    constexpr int ESZ = (int)sizeof(E);
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int T = S::T, P = S::KSZ / 2;
    constexpr int NH = 4;                        // fragments per half at T = 128
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wv & 3, hh = wv >> 2;
    const int c = lane & 15, kq = lane >> 4;
    const int ch0 = 32 * w + 4 * kq;
    if (A.tick && b == 0 && tid == 0) atomicAdd(A.tick, 1);
    FZ_PH_DECL
    FZ_PH();

    char* XB = fz_lds;                                  // x image [T+8][80], pad 4
    char* BK0 = XB + (T + 8) * RS;                      // bank output [T][128], double-buffered
    char* BK1 = BK0 + T * RS;
    char* HB = fz_lds;                                  // block input image [T+2P][128]
    char* YB = HB + (T + 2 * P) * RS;                   // conv1 output image
    // last block's stride-2 pool: the odd input fragment of half 1, fp32 [wave w][2][64 lanes]
    f32x4* XCH = reinterpret_cast<f32x4*>(YB + (T + 2 * P) * RS);
    u64* mbase = A.masks + (size_t)b * A.mask_words;
    const bool wm = A.write_masks != 0;

    const int ns_c = S::KSZ * FZ_C / KS;
    auto op_bank = [&](int kb) __attribute__((always_inline)) {
        const int ns = (FZ_CIN * (kb + 1) + KS - 1) / KS;
        return aop(A.w.bank[kb], 2 * w, 2, ns, ns);
    };
    auto op_inb = [&](int kb) __attribute__((always_inline)) { return aop(A.w.in_b[kb], 2 * w, 2, FZ_C / KS, FZ_C / KS); };
    auto op_inx = [&]() __attribute__((always_inline)) {
        const int ns = (FZ_CIN + KS - 1) / KS;
        return aop(A.w.in_x, 2 * w, 2, ns, ns);
    };
    auto op_c1 = [&](int l) __attribute__((always_inline)) { return aop(A.w.c1[l], 2 * w, 2, ns_c, ns_c); };
    auto op_c2 = [&](int l) __attribute__((always_inline)) { return aop(A.w.c2[l], 2 * w, 2, ns_c, ns_c); };
    ARing<2, AVC_FZ8_RD> ring;
    ring_fill(ring, op_bank(0));
    // ---- x -> XB (transposed, reflect rows): the 4-wave kernel's conflict-free load, by waves 0-3
    constexpr int NGX = FZ_CIN / VE;
    constexpr int GPT = NGX / 2;
    if (wv < 4) {
        const int xt = 32 * wv + (lane >> 1), xh = lane & 1;
        float xv[GPT][VE];
        const float* xs = A.x + (size_t)b * FZ_CIN * T + xt;
#pragma unroll
        for (int m = 0; m < GPT; ++m)
#pragma unroll
            for (int e = 0; e < VE; ++e) xv[m][e] = xs[(size_t)((2 * m + xh) * VE + e) * T];
#pragma unroll
        for (int m = 0; m < GPT; ++m) {
            const f32x4 v = pk_bf16x8([&](int e) { return xv[m][e]; });
            const int cb = (2 * m + xh) * 16;
            *reinterpret_cast<f32x4*>(XB + (4 + xt) * RS + cb) = v;
            if (xt >= 1 && xt <= 4) *reinterpret_cast<f32x4*>(XB + (4 - xt) * RS + cb) = v;
            if (xt >= T - 5 && xt <= T - 2) *reinterpret_cast<f32x4*>(XB + (4 + 2 * T - 2 - xt) * RS + cb) = v;
        }
    }
    __syncthreads();
    FZ_PH();
    const int t0 = 64 * hh;                             // first frame of this wave's half (T = 128 layers)
    int rb[NH];
    f32x4 acc_h[2][NH];
    zero_acc(acc_h);
    f32x4 b_in[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) b_in[i] = *reinterpret_cast<const f32x4*>(A.w.b_in + ch0 + 16 * i);
    auto bank_fwd = [&](auto KB) __attribute__((always_inline)) {
        constexpr int kb = decltype(KB)::value;
        constexpr int pl = (kb + 1) / 2;
        f32x4 bkb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) bkb[i] = *reinterpret_cast<const f32x4*>(A.w.b_bank[kb] + ch0 + 16 * i);
        f32x4 acc[2][NH];
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NH; ++f) rb[f] = t0 + 16 * f + c + 4 - pl;
        fz_gemm<PREC, 2, NH, FZ_CIN, 1>(acc, IC<NH>{}, ring, op_bank(kb), op_inb(kb), XB, rb);
        char* BK = (kb & 1) ? BK1 : BK0;
        MaskAcc8 mk;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int f = 0; f < NH; ++f) {
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = act_f(acc[i][f][r] + bkb[i][r], 0);
                    mk.put(i, f, r, y[r]);
                }
                st4<PREC>(BK + (t0 + 16 * f + c) * RS + (ch0 + 16 * i) * ESZ, y);
            }
        if (wm) mk.store(mbase, kb, wv);
        __syncthreads();
        // in_conv over this bank block (K = 128 channels of the block) for this half's frames
#pragma unroll
        for (int f = 0; f < NH; ++f) rb[f] = t0 + 16 * f + c;
        fz_gemm<PREC, 2, NH, FZ_C, 1>(acc_h, IC<NH>{}, ring, op_inb(kb), kb + 1 < S::NB ? op_bank(kb + 1) : op_inx(), BK,
                                      rb);
        FZ_PH();
    };
    static_for<0, S::NB>([&](auto KB) __attribute__((always_inline)) { bank_fwd(KB); });
    {   // in_conv, x block (K = 80)
#pragma unroll
        for (int f = 0; f < NH; ++f) rb[f] = t0 + 16 * f + c + 4;
        fz_gemm<PREC, 2, NH, FZ_CIN, 1>(acc_h, IC<NH>{}, ring, op_inx(), op_c1(0), XB, rb);
    }
    __syncthreads();   // XB / BK are dead: HB and YB alias them
    FZ_PH();

    // h0 = act(in_conv + b): fp32 residual stream in registers, operand image in HB
    f32x4 hres[2][NH];
    {
        MaskAcc8 mk;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int f = 0; f < NH; ++f) {
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = act_f(acc_h[i][f][r] + b_in[i][r], 0);
                    mk.put(i, f, r, y[r]);
                }
                hres[i][f] = y;
                put_reflect<PREC>(HB, t0 + 16 * f + c, T, P, (ch0 + 16 * i) * ESZ, y);
            }
        if (wm) mk.store(mbase, S::NB, wv);
    }
    __syncthreads();

    // one conv block (models.py:285-305).  NI / NO: fragments of this half's input / output frames
    // (NO = 0: the half has no output fragment -- the last block's 16 frames sit in half 0)
    auto block = [&](auto LL) __attribute__((always_inline)) {
        constexpr int l = decltype(LL)::value;
        constexpr int Ti = S::Tl(l), To = S::Tl(l + 1), s = S::sub(l);
        constexpr int NI = S::nf(Ti) / 2;                     // 4, 4, 2, 2, 1, 1
        constexpr int NO1 = (S::nf(To) + 1) / 2;               // half 0's output fragments
        constexpr int NO0 = S::nf(To) - NO1;                   // half 1's
        const int ti0 = 16 * NI * hh, to0 = 16 * NO1 * hh;   // first frame of this half (in / out)
        f32x4 bc1[2], bc2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            bc1[i] = *reinterpret_cast<const f32x4*>(A.w.b_c1[l] + ch0 + 16 * i);
            bc2[i] = *reinterpret_cast<const f32x4*>(A.w.b_c2[l] + ch0 + 16 * i);
        }
        // conv1 (stride 1): y1 = act(conv1(h) + b1) -> YB
        f32x4 acc[2][NH];
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NH; ++f) rb[f] = min(ti0 + 16 * f + c, Ti - 1);
        fz_gemm<PREC, 2, NH, FZ_C, 1>(acc, IC<NI>{}, ring, op_c1(l), op_c2(l), HB, rb);
        {
            MaskAcc8 mk;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < NI; ++f) {
                    f32x4 y;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        y[r] = act_f(acc[i][f][r] + bc1[i][r], 0);
                        mk.put(i, f, r, y[r]);
                    }
                    put_reflect<PREC>(YB, ti0 + 16 * f + c, Ti, P, (ch0 + 16 * i) * ESZ, y);
                }
            if (wm) mk.store(mbase, S::NB + 1 + 2 * l, wv);
        }
        if constexpr (To < 32 && s == 2) {
            // the last block: half 1 hands its input fragment (frames 16..31) to half 0's pool
            if (hh == 1)
#pragma unroll
                for (int i = 0; i < 2; ++i) XCH[(w * 2 + i) * 64 + lane] = hres[i][0];
        }
        __syncthreads();
        // conv2 (stride s): y2 = act(conv2(y1) + b2); h = y2 + avg_pool1d(h, s, ceil_mode)
        const int no = hh == 0 ? NO1 : NO0;
        if (no == 0) {
            // (half 1 of the last block has no output: its ring is not used again)
            return;
        }
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NH; ++f) rb[f] = min(to0 + 16 * f + c, To - 1) * s;
        if constexpr (l + 1 < S::NBLK) {
            fz_gemm<PREC, 2, NH, FZ_C, 1>(acc, IC<(NO1 > 0 ? NO1 : 1)>{}, ring, op_c2(l), op_c1(l + 1), YB, rb);
        } else {
            fz_gemm<PREC, 2, NH, FZ_C, 1>(acc, IC<(NO1 > 0 ? NO1 : 1)>{}, ring, op_c2(l), op_c2(l), YB, rb);
        }
        if constexpr (s == 2) {
            // pooled[t'] = (h[2t'] + h[2t'+1]) / cnt: sources in local frags 2f', 2f'+1 (the last
            // block's f' = 0 takes frag 1 from half 1 through XCH)
            f32x4 hx[2];
            if constexpr (To < 32) {
#pragma unroll
                for (int i = 0; i < 2; ++i) hx[i] = XCH[(w * 2 + i) * 64 + lane];
            }
            const int src0 = (lane & 48) | ((2 * c) & 15), src1 = (lane & 48) | ((2 * c + 1) & 15);
#pragma unroll
            for (int fo = 0; fo < NO1; ++fo) {
                const int t = to0 + 16 * fo + c;
                const bool two = 2 * t + 1 < Ti;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x4 sa = hres[i][2 * fo < NH ? 2 * fo : NH - 1];
                    f32x4 sb;
                    if constexpr (To < 32) sb = hx[i];
                    else sb = hres[i][(2 * fo + 1) < NH ? 2 * fo + 1 : NH - 1];
                    f32x4 pv;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float a0 = __shfl(sa[r], src0), a1 = __shfl(sa[r], src1);
                        const float b0 = __shfl(sb[r], src0), b1 = __shfl(sb[r], src1);
                        const float x0 = c < 8 ? a0 : b0, x1 = c < 8 ? a1 : b1;
                        pv[r] = two ? (x0 + x1) / 2.f : x0;
                    }
                    hres[i][fo] = pv;
                }
            }
        }
        {
            MaskAcc8 mk;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < NO1; ++f) {
                    f32x4 y, h;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        y[r] = act_f(acc[i][f][r] + bc2[i][r], 0);
                        mk.put(i, f, r, y[r]);
                        h[r] = y[r] + hres[i][f][r];
                    }
                    hres[i][f] = h;
                    if constexpr (l + 1 < S::NBLK) put_reflect<PREC>(HB, to0 + 16 * f + c, To, P, (ch0 + 16 * i) * ESZ, h);
                }
            if (wm) mk.store(mbase, S::NB + 2 + 2 * l, wv);
        }
    };
    static_for<0, S::NBLK>([&](auto L) __attribute__((always_inline)) {
        block(L);
        __syncthreads();
        FZ_PH();
    });

    // AdaptiveAvgPool1d(1) over the TN = 16 frames (half 0's one fragment), then the head
    constexpr int TN = S::Tl(S::NBLK);
    float* hsm = reinterpret_cast<float*>(fz_lds);      // the head's LDS (conv images dead)
    const bool fh = A.fuse_head != 0;
    if (hh == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            f32x4 s4 = hres[i][0];
            row16_sum(s4);
            if (c == 0) {
                f32x4 m;
#pragma unroll
                for (int r = 0; r < 4; ++r) m[r] = s4[r] / (float)TN;
                *reinterpret_cast<f32x4*>(A.pooled + (size_t)b * FZ_C + ch0 + 16 * i) = m;
                if (fh)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) hsm[hpos(ch0 + 16 * i + rr)] = m[rr];
            }
        }
    }
    if (fh) {
        if (A.fuse_head == 2) se_head_fused<S::NDENSE, 0, 512>(A.head, b, hsm, A.loss_cur);
        else se_head_fused<S::NDENSE, 1, 512>(A.head, b, hsm, A.loss_cur);
    }
    FZ_PH();
    FZ_PH_DUMP("fwd");
}

// ---------------------------------------------------------------------------------
// backward + Adam (se_bwd_fused<bf16, 0> with two waves per SIMD)
// ---------------------------------------------------------------------------------
// ReLU' bits of a layer as written by se_fwd8: both halves' words of this channel quarter (the bank
// phase needs one fragment of the other half)
struct MaskRd8 {
    unsigned m[2];
    __device__ __forceinline__ void load(const u64* mbase, int layer, int w) {
        const unsigned* p = reinterpret_cast<const unsigned*>(mbase) + (size_t)layer * F8_MASK_U32_PER_LAYER + w * 64 +
                            (threadIdx.x & 63);
        m[0] = p[0];
        m[1] = p[4 * 64];
        __builtin_amdgcn_sched_barrier(0);
    }
    // g * act'(y) of element (i, local fragment f of half h, r): the bit sign-extended to a lane
    // mask ANDed onto g (ReLU; the standard shape)
    __device__ __forceinline__ float gate(int h, int i, int f, int r, float g) const {
        int mk;
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(mk) : "v"(m[h]), "s"(16 * i + 4 * f + r));
        return __builtin_bit_cast(float, __builtin_bit_cast(int, g) & mk);
    }
};

// reflect-pad adjoint on the accumulators of local fragments whose columns start at cb[f] (interior
// frames, or the pad-position columns Tin .. Tin + 2E - 1 of the edge fragment): the sum at pad
// position v folds onto -v (left) or 2 (Tin - 1) - v (right).  Wave-local (this wave's scratch).
template <int MT, int NF>
__device__ __forceinline__ void fold_edges8(f32x4 (&acc)[MT][NF], const int (&cb)[NF], int Tin, int E, float* scr) {
    const int lane = threadIdx.x & 63, c = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        const int e = cb[f] + c - Tin;
        if (e >= 0 && e < 2 * E) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) scr[(16 * i + 4 * kq + r) * 8 + e] = acc[i][f][r];
        }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int g = 0; g < NF; ++g) {
        const int t = cb[g] + c;
        const int el = (t >= 1 && t <= E) ? E - t : -1;
        const int er = (t >= Tin - 1 - E && t <= Tin - 2) ? Tin - 2 - t + E : -1;
        if (t < Tin && (el >= 0 || er >= 0)) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float* row = scr + (16 * i + 4 * kq + r) * 8;
                    float add = el >= 0 ? row[el] : 0.f;
                    if (er >= 0) add += row[er];
                    acc[i][g][r] += add;
                }
        }
    }
}

template <int PREC>
__global__ void __launch_bounds__(512, 1) se_bwd8(FusedArgs A) {
    static_assert(PREC == PREC_BF16, "the 8-wave engine is the bf16 bench path");
    using S = StdSE;
    using E = typename Fz<PREC>::E;
    constexpr int RS = Fz<PREC>::RS;
    constexpr int ESZ = (int)sizeof(E);
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int T = S::T, P = S::KSZ / 2;
    constexpr int NH = 4;                        // interior fragments per half at T = 128
    constexpr int ZP = 4;                        // zero rows around a block dY image
    constexpr int ZPB = 8;                       // ... around a bank g(b_k) image
    constexpr int EB = 4;                        // bank dgrad edge columns per side
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wv & 3, hh = wv >> 2;
    const int c = lane & 15, kq = lane >> 4;
    const int ch0 = 32 * w + 4 * kq;
    const u64* mbase = A.masks + (size_t)b * A.mask_words;
    constexpr int TN = S::Tl(S::NBLK);
    FZ_PH_DECL
    FZ_PH();

    char* GB = fz_lds;                                  // dilated dY image [T+2ZP] rows; later g_pre0
    char* GB2 = GB + (T + 2 * ZP) * RS;                 // stride-1 dY image [T+2ZP] rows
    char* GBK[2] = {GB2, GB2 + (T + 2 * ZPB) * RS};     // per-half g(b_k) images (bank phase; alias GB2)
    float* FSCR = reinterpret_cast<float*>(GB2 + 2 * (T + 2 * ZPB) * RS) + wv * (5 * 16 * 8);
    f32x4* XCH = reinterpret_cast<f32x4*>(reinterpret_cast<char*>(FSCR) + (8 - wv) * (5 * 16 * 8 * 4));

    f32x4 gp[2];
    if (A.fuse_head == 3) {   // e2e / fb: the head's backward (se_head_v mode 3) runs here
        float* hsm = reinterpret_cast<float*>(fz_lds);
        se_head_fused<S::NDENSE, 3, 512>(A.head, b, hsm, nullptr);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) gp[i][r] = hsm[hpos(ch0 + 16 * i + r)];
        __syncthreads();
    } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) gp[i] = *reinterpret_cast<const f32x4*>(A.g_pooled + (size_t)b * FZ_C + ch0 + 16 * i);
    }
    const int ns_c = S::KSZ * FZ_C / KS;
    auto op_c1T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c1T[l], 2 * w, 2, ns_c, ns_c); };
    auto op_c2T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c2T[l], 2 * w, 2, ns_c, ns_c); };
    ARing<2, AVC_FZ8_RD> ring;
    ring_fill(ring, op_c2T(S::NBLK - 1));
    MaskRd8 mnext;
    mnext.load(mbase, S::NB + 2 + 2 * (S::NBLK - 1), w);
    {   // zero both dY images (pad rows and dilation holes must read as 0)
        constexpr int n16 = 2 * (T + 2 * ZP) * RS / 16;
        for (int i = tid; i < n16; i += 512) reinterpret_cast<f32x4*>(fz_lds)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // g(h_N): d mean / d h = 1/TN on the TN = 16 frames: half 0's one fragment
    f32x4 gh[2][NH];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x4 g = gp[i];
#pragma unroll
        for (int r = 0; r < 4; ++r) g[r] = g[r] / (float)TN;
#pragma unroll
        for (int f = 0; f < NH; ++f) gh[i][f] = (hh == 0 && f == 0) ? g : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();

    int rb[NH + 1], cb[NH + 1];
    // backward of one conv block: NI interior fragments of this half at Ti (+ the edge fragment
    // of the pad positions, computed by both halves), NO output fragments at To
    auto block = [&](auto LL) __attribute__((always_inline)) {
        constexpr int l = decltype(LL)::value;
        constexpr int Ti = S::Tl(l), To = S::Tl(l + 1), s = S::sub(l);
        constexpr int NI = S::nf(Ti) / 2;
        constexpr int NO1 = (S::nf(To) + 1) / 2;      // half 0's output fragments (half 1: nf - NO1)
        const int no = hh == 0 ? NO1 : S::nf(To) - NO1;
        const int ti0 = 16 * NI * hh, to0 = 16 * NO1 * hh;
        // dY of conv2 = g(h_{l+1}) * act'(y2_l), written dilated by s into GB
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int f = 0; f < NH; ++f) {
                if (f >= no) continue;
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = mnext.gate(hh, i, f, r, gh[i][f][r]);
                const int t = to0 + 16 * f + c;
                st4<PREC>(GB + (ZP + s * t) * RS + (ch0 + 16 * i) * ESZ, v);
                if (s == 2) st4<PREC>(GB + (ZP + 2 * t + 1) * RS + (ch0 + 16 * i) * ESZ, f32x4{0.f, 0.f, 0.f, 0.f});
            }
        if constexpr (To < 32 && s == 2) {
            // the last block's pool adjoint: half 1's frames 16..31 take g(h_{l+1}) of half 0's fragment
            if (hh == 0)
#pragma unroll
                for (int i = 0; i < 2; ++i) XCH[(w * 2 + i) * 64 + lane] = gh[i][0];
        }
        __syncthreads();
        // conv2^T over this half's interior columns and the edge columns
#pragma unroll
        for (int f = 0; f <= NH; ++f) {   // fragments past the edge one: outside every fold range
            cb[f] = f < NI ? ti0 + 16 * f : (f == NI ? Ti : -1024);
            const int n = cb[f] + c;
            rb[f] = ZP + (n >= 0 && n < Ti + 2 * P ? vpos(n, Ti, P) : 0) + P;
        }
        f32x4 acc[2][NH + 1];
        zero_acc(acc);
        MaskRd8 m1;
        m1.load(mbase, S::NB + 1 + 2 * l, w);
        fz_gemm<PREC, 2, NH + 1, FZ_C, -1>(acc, IC<NI + 1>{}, ring, op_c2T(l), op_c1T(l), GB, rb);
        fold_edges8(acc, cb, Ti, P, FSCR);
        // * act'(y1_l) -> GB2 (stride 1)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int f = 0; f < NI; ++f) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = m1.gate(hh, i, f, r, acc[i][f][r]);
                st4<PREC>(GB2 + (ZP + ti0 + 16 * f + c) * RS + (ch0 + 16 * i) * ESZ, v);
            }
        __syncthreads();
        // conv1^T (+ fold) + avg_pool^T of g(h_{l+1}) -> g(h_l)
        zero_acc(acc);
        if constexpr (l > 0) mnext.load(mbase, S::NB + 2 + 2 * (l - 1), w);   // next block's conv2
        else mnext.load(mbase, S::NB, w);                                     // or h0
        if constexpr (l > 0) {
            fz_gemm<PREC, 2, NH + 1, FZ_C, -1>(acc, IC<NI + 1>{}, ring, op_c1T(l), op_c2T(l - 1), GB2, rb);
        } else {
            fz_gemm<PREC, 2, NH + 1, FZ_C, -1>(acc, IC<NI + 1>{}, ring, op_c1T(l), op_c1T(l), GB2, rb);
        }
        fold_edges8(acc, cb, Ti, P, FSCR);
        if constexpr (s == 2) {
            // g_h[t] += g_{l+1}[t/2] / cnt(t/2) (torch avg_pool backward: grad / divide_factor);
            // decreasing f keeps the in-place update safe (frag f reads local frag f/2)
            f32x4 gx[2];
            if constexpr (To < 32) {
#pragma unroll
                for (int i = 0; i < 2; ++i) gx[i] = XCH[(w * 2 + i) * 64 + lane];
            }
#pragma unroll
            for (int f = NI - 1; f >= 0; --f) {
                const int g = NI * hh + f;                     // global fragment
                const int t = 16 * g + c;
                const bool two = 2 * (t >> 1) + 1 < Ti;
                const int srcl = (lane & 48) | (8 * (g & 1) + (c >> 1));
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    f32x4 sv;
                    if constexpr (To < 32) sv = gx[i];
                    else sv = gh[i][f >> 1];
                    f32x4 ng;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float gg = __shfl(sv[r], srcl);
                        ng[r] = acc[i][f][r] + (two ? gg / 2.f : gg);
                    }
                    gh[i][f] = ng;
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < NI; ++f) gh[i][f] = acc[i][f] + gh[i][f];
        }
    };
    FZ_PH();
    static_for<0, S::NBLK>([&](auto L) __attribute__((always_inline)) {
        block(IC<S::NBLK - 1 - decltype(L)::value>{});
        FZ_PH();
    });

    // g_pre0 = g(h0) * act'(h0) -> GP (= GB image, rows ZP + t; pad rows are zero)
    char* GP = GB;
    const int t0 = 64 * hh;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int f = 0; f < NH; ++f) {
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = mnext.gate(hh, i, f, r, gh[i][f][r]);
            st4<PREC>(GP + (ZP + t0 + 16 * f + c) * RS + (ch0 + 16 * i) * ESZ, v);
        }
    __syncthreads();

    // bank dgrad, K split over the 4 channel quarters: wave (w, hh) sums over bank channels
    // [32w, 32w+32) of every bank kernel for its half's x-gradient columns (+ the edge columns).
    // g(b_k) of those channels over the frames the half reads (fragments 0-4 / 3-7) goes to the
    // half's own GBK image, so the hand-off stays wave-local (no barrier), as in se_bwd_fused.
    char* GBKh = GBK[hh];
    {   // zero this wave's channel slice of its GBK pad rows
        constexpr int V16 = 32 * ESZ / 16;
        for (int idx = lane; idx < 2 * ZPB * V16; idx += 64) {
            const int rr = idx / V16, part = idx - rr * V16;
            const int row = rr < ZPB ? rr : T + rr;
            *reinterpret_cast<f32x4*>(GBKh + row * RS + 32 * w * ESZ + part * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    f32x4 accx[5][NH + 1];
    zero_acc(accx);
    constexpr int SPW = 32 / KS;                // K steps of one wave's 32-channel quarter
    constexpr int SPT = FZ_C / KS;              // K steps per tap
    constexpr int LG = SPW == 1 ? 0 : 1;
    auto op_inTb = [&](int kb) __attribute__((always_inline)) { return aop(A.w.inT_b[kb], 2 * w, 2, SPT, SPT); };
    auto op_bankT = [&](int kb) __attribute__((always_inline)) {
        return aop(A.w.bankT[kb], 0, 5, (kb + 1) * SPT, (kb + 1) * SPW, LG, SPW - 1, SPT, w * SPW);
    };
    // one A stream for the whole phase: in_conv^T (2 tiles) and bank^T (5 tiles) steps alternate in
    // the 5-tile ring (the in_conv^T steps re-read their last tile in the 3 spare slots: L1 hits);
    // at two waves per SIMD the 4-wave kernel's register-resident in_conv^T operand does not fit
    ARing<5, 2> ring5;
    MaskRd8 mbn;                                // ReLU' words of the next bank kernel, a GEMM ahead
    mbn.load(mbase, 0, w);
#pragma unroll
    for (int f = 0; f <= NH; ++f) cb[f] = f < NH ? t0 + 16 * f : T;
    {   // x passthrough of the cat: W_in[:, x block]^T g_pre0 (interior columns only)
#pragma unroll
        for (int f = 0; f <= NH; ++f) {
            const int n = cb[f] + c;
            rb[f] = n < T ? ZP + n : 0;
        }
        const AOp opx = aop(A.w.inT_x, 0, 5, SPT, SPW, 30, -1, 0, w * SPW);
        ring_fill(ring5, opx);
        fz_gemm<PREC, 5, NH + 1, FZ_C, 1>(accx, IC<NH + 1>{}, ring5, opx, op_inTb(0), GP, rb);
    }
    FZ_PH();
    const int fb0 = hh == 0 ? 0 : 3;            // first g(b_k) fragment this half computes (5 of them)
    auto bank_bwd = [&](auto KB) __attribute__((always_inline)) {
        constexpr int kb = decltype(KB)::value;
        constexpr int pl = (kb + 1) / 2;
        const MaskRd8 mb = mbn;
        // g(b_k) for this wave's 32 bank channels = (W_in[:, kb]^T g_pre0) * act'(b_k), fragments
        // fb0 .. fb0 + 4 in two groups (3 + 2: fewer live registers)
        auto gbk = [&](auto F0, auto NFG, const AOp& nxt) __attribute__((always_inline)) {
            constexpr int f0 = decltype(F0)::value, nfg = decltype(NFG)::value;
            f32x4 acc[2][nfg];
            zero_acc(acc);
            int rt[nfg];
#pragma unroll
            for (int f = 0; f < nfg; ++f) rt[f] = ZP + 16 * (fb0 + f0 + f) + c;
            fz_gemm<PREC, 2, nfg, FZ_C, 1>(acc, IC<nfg>{}, ring5, op_inTb(kb), nxt, GP, rt);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < nfg; ++f) {
                    const int g = fb0 + f0 + f;            // global fragment; its bits: half g / 4, local g % 4
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = mb.gate(g >> 2, i, g & 3, r, acc[i][f][r]);
                    st4<PREC>(GBKh + (ZPB + 16 * g + c) * RS + (ch0 + 16 * i) * ESZ, v);
                }
        };
        gbk(IC<0>{}, IC<3>{}, op_inTb(kb));
        gbk(IC<3>{}, IC<2>{}, op_bankT(kb));
        FZ_PH();
        asm volatile("" ::: "memory");   // wave-local hand-off: program order only
        if constexpr (kb + 1 < S::NB) mbn.load(mbase, kb + 1, w);
        // bank_k^T over this wave's channel quarter: rows q = v + pl - j of g(b_k)
#pragma unroll
        for (int f = 0; f <= NH; ++f) {
            const int n = cb[f] + c;
            rb[f] = ZPB + (n < T + 2 * EB ? vpos(n, T, EB) : 0) + pl;
        }
        const AOp opn = kb + 1 < S::NB ? op_inTb(kb + 1) : op_bankT(kb);
        fz_gemm<PREC, 5, NH + 1, FZ_C, -1>(accx, IC<NH + 1>{}, ring5, op_bankT(kb), opn, GBKh, rb);
        asm volatile("" ::: "memory");
        FZ_PH();
    };
    static_for<0, S::NB>([&](auto KB) __attribute__((always_inline)) { bank_bwd(KB); });
    fold_edges8(accx, cb, T, EB, FSCR);
    __syncthreads();   // every GEMM's LDS reads done: R0 / R1 alias the images
    FZ_PH();

    // deterministic cross-wave sum ((p0 + p2) + (p1 + p3)) per half, then tanh' + Adam
    constexpr int TP = T + 4;
    auto rq = [&](int q) __attribute__((always_inline)) { return q + q / (T / 4); };
    float* R0 = reinterpret_cast<float*>(fz_lds);
    float* R1 = R0 + FZ_CIN * TP;
    for (int phase = 0; phase < 2; ++phase) {
        // phase 0: waves 2, 3 (of each half) store p2 -> R0, p3 -> R1;  phase 1: waves 0, 1 add p0, p1
        if ((phase == 0) == (w >= 2)) {
            float* R = (w & 1) ? R1 : R0;
#pragma unroll
            for (int i = 0; i < 5; ++i)
#pragma unroll
                for (int f = 0; f < NH; ++f) {
                    const int t = t0 + 16 * f + c;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float* p = R + (16 * i + 4 * kq + r) * TP + t;
                        *p = phase ? accx[i][f][r] + *p : accx[i][f][r];
                    }
                }
        }
        __syncthreads();
    }
    FZ_PH();

    if (A.gx_out && A.losses && tid == 0) {   // fb: the fused head's loss of SE(dec) -> history row
        const int sn = *A.step;
        if (sn >= 1 && sn <= A.loss_len) A.losses[(size_t)(sn - 1) * A.B + b] = A.loss_cur[b];
    }
    if (A.gx_out) {   // d loss / d x handed on (fb: the decoder output's gradient)
        f32x4* gx = reinterpret_cast<f32x4*>(A.gx_out + (size_t)b * FZ_CIN * T);
        const f32x4* R04 = reinterpret_cast<const f32x4*>(R0);
        const f32x4* R14 = reinterpret_cast<const f32x4*>(R1);
        for (int q = tid; q < FZ_CIN * T / 4; q += 512) gx[q] = R04[rq(q)] + R14[rq(q)];
        return;
    }
    const AdamArgs& Ad = A.adam;
    const float eps = A.scal[0];
    if (A.losses && tid == 0) {   // the fused head's loss of this iteration -> history row step-1
        const int sn = *A.step;
        if (sn >= 1 && sn <= A.loss_len) A.losses[(size_t)(sn - 1) * A.B + b] = A.loss_cur[b];
    }
    const int step = min(max(*A.step, 1), A.table_len);
    const float nstep = Ad.table[2 * (step - 1)];
    const float bc2s = Ad.table[2 * (step - 1) + 1];
    const float rbc2s = 1.f / bc2s;
    const AdamStep St{nstep, bc2s, rbc2s, eps, A.scal[3]};
    const size_t base4 = (size_t)b * FZ_CIN * T / 4;
    f32x4* __restrict__ ptb4 = reinterpret_cast<f32x4*>(Ad.ptb) + base4;
    f32x4* __restrict__ m4 = reinterpret_cast<f32x4*>(Ad.m) + base4;
    f32x4* __restrict__ v4 = reinterpret_cast<f32x4*>(Ad.v) + base4;
    const f32x4* __restrict__ vc4 = reinterpret_cast<const f32x4*>(Ad.vc) + base4;
    f32x4* __restrict__ adv4 = reinterpret_cast<f32x4*>(Ad.adv) + base4;
    f32x4* __restrict__ g04 = Ad.grad0 && step == 1 ? reinterpret_cast<f32x4*>(Ad.grad0) + base4 : nullptr;
    const f32x4* R04 = reinterpret_cast<const f32x4*>(R0);
    const f32x4* R14 = reinterpret_cast<const f32x4*>(R1);
    constexpr int n4 = FZ_CIN * T / 4;
    constexpr int AB = n4 / 512;                // 5: one batch of 16-byte accesses covers the utterance
    static_assert(AB * 512 == n4, "Adam batch");
    f32x4 sP[AB], sM[AB], sV[AB], sX[AB];
#pragma unroll
    for (int k = 0; k < AB; ++k) {
        const int q = tid + 512 * k;
        sP[k] = ptb4[q];
        sM[k] = m4[q];
        sV[k] = v4[q];
        sX[k] = vc4[q];
    }
#pragma unroll
    for (int k = 0; k < AB; ++k) {
        const int q = tid + 512 * k;
        const f32x4 gsum = R04[rq(q)] + R14[rq(q)];
        f32x4 p = sP[k], mm = sM[k], vv = sV[k], g, ad;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float pe = p[e], me = mm[e], ve = vv[e], ge, ae;
            adam_elem<PREC>(Ad, St, gsum[e], sX[k][e], pe, me, ve, ge, ae);
            p[e] = pe;
            mm[e] = me;
            vv[e] = ve;
            g[e] = ge;
            ad[e] = ae;
        }
        if (g04) g04[q] = g;
        ptb4[q] = p;
        m4[q] = mm;
        v4[q] = vv;
        adv4[q] = ad;
    }
    FZ_PH();
    FZ_PH_DUMP("bwd");
}

template __global__ void se_fwd8<PREC_BF16>(FusedArgs);
template __global__ void se_bwd8<PREC_BF16>(FusedArgs);

}  // namespace avc
