// Fused per-utterance SpeakerEncoder engine for the embedding attack on gfx950.
//
// One workgroup (4 waves, 256 threads) owns ONE utterance for a whole
// forward or backward pass; every activation of the conv stack lives in LDS
// and every Conv1d (and every Conv1d input-gradient) runs on the matrix cores
// straight out of LDS:
//
//   se_fwd_fused  adv -> conv bank (models.py:82-104) -> in_conv 1x1 (337-338)
//                 -> 6 conv blocks (285-305) -> time-mean (275,340)   [+ ReLU' bit masks]
//   se_head       (avc_kernels.hip, batched over utterances) dense blocks, output
//                 Linear, MSE loss and its gradient back to the time-mean
//   se_bwd_fused  that gradient -> block dgrads -> in_conv dgrad -> bank dgrad
//                 -> tanh' -> Adam (attack_utils.py:78-84, torch _single_tensor_adam)
//                 -> next adv = vc + eps*tanh(ptb)
//
// GEMM shape per layer: C[M = out channels][N = frames] = A[M][K = (tap, in channel)] * B.
// Wave w owns the 32 output channels [32w, 32w+32) of a 128-channel layer (two 16-row
// M tiles) and all N columns (16-column fragments), so the weights of a layer are read
// from L2 exactly once per workgroup and never duplicated across waves.
//   A: packed in fragment order in HBM (one 16-byte load per lane per M tile per K step),
//      prefetched three K steps ahead in registers.
//   B: activations in LDS as [frame row][channel] (channels contiguous, rows of 288 B
//      bf16 / 544 B fp32 -- a row stride of 2 mod 16 16-byte slots makes every
//      ds_read_b128 of a fragment conflict-free for any tap shift).  With K ordered
//      (tap, channel), a lane's 8 (bf16) or 4 (fp32) consecutive K values are one
//      16-byte read of one row: tap j of output frame t is row t*stride + j (padded
//      coordinates), so reflect padding is just extra rows written by the producer.
//   MFMA: v_mfma_f32_16x16x32_bf16 (bf16 in, fp32 acc) or v_mfma_f32_16x16x4_f32
//      (exact fp32; the 4 K values of a 16-byte read are 4 MFMAs).
// Dgrads use the same loop with the B rows running backwards (q = p - j over a
// zero-padded, stride-dilated dY image) and the reflect-pad adjoint done on the
// accumulators: the pad positions are extra "edge" columns whose sums are shuffled
// onto the reflected interior columns.  ReLU' is kept from the forward as 64-bit
// ballot words per (tile, fragment, register) -- the bwd tests the same lane bit.
//
// The residual stream h and its gradient stay fp32 in registers in the MFMA C/D
// layout (col = lane&15, row = 4*(lane>>4)+reg); avg_pool1d(ceil_mode) and its
// adjoint are lane shuffles.  Only the bf16/fp32 operand copies go through LDS.
#include "avc_fused_core.h"
#include "avc_ktime.h"
#include "avc_se_head.h"

AVC_KTIME_DEFINE(fused)   // se_fwd_fused / se_bwd_fused, per precision (avc_ktime.h)

namespace avc {
// shape-generic kernels: the fragment-count class of a block k stride-2 blocks below an input of
// class G (an upper bound of its true count: the dead fragments compute on clamped rows, never stored)
__host__ __device__ constexpr int fz_cls(int G, int k) { return (G >> k) > 0 ? (G >> k) : 1; }
// the config's blocks subsample as the AdaIN-VC default: 6 blocks, stride 2 on the odd ones
__device__ __forceinline__ bool fz_std_sub(const FusedArgs& A) {
    bool s = A.nblk == 6;
#pragma unroll
    for (int l = 0; l < 6; ++l) s = s && A.sub[l] == ((l & 1) ? 2 : 1);
    return s;
}
}  // namespace avc

// A-ring depth of the standard-shape kernels' 2-tile GEMMs (the generic shapes keep 4: their
// step counts are runtime values, and the ring's end-of-GEMM rotation would not fold away)
#ifndef AVC_FZ_RD_FWD
#define AVC_FZ_RD_FWD 8
#endif
// round-5 epilogue VALU cuts (A/B on the emb iteration, bit-identical results): the stride-2 pool from
// DPP pair sums (2 lane shuffles per element instead of 4) and the bank / conv1 ReLU on packed bf16 pairs
// -- 0.1768 -> 0.1756 ms together
#ifndef AVC_FZ_POOLDPP
#define AVC_FZ_POOLDPP 1
#endif
#ifndef AVC_FZ_PKRELU
#define AVC_FZ_PKRELU 1
#endif
#ifndef AVC_FZ_RD_BWD
#define AVC_FZ_RD_BWD 8
#endif

namespace avc {

// ---------------------------------------------------------------------------------
// shapes (kernel template parameter SH):
//   SH = 0        : the AdaIN-VC speaker encoder at its config.yaml defaults (bank 1..8,
//                   kernel 5, six blocks with subsample [1,2,1,2,1,2]) at T = 128 -- every
//                   layer's frame and fragment count is a compile-time constant;
//   SH = 1,2,4,8  : any eligible config and T <= 16*SH; every layer runs SH fragments
//                   (SH + 1 for dgrad outputs, which carry the pad-position columns).
//   SH = 16       : the config.yaml model at any T in (64, 128] (round 6): the standard kernels'
//                   compile-time fragment classes (8, 8, 4, 4, 2, 2, 1 -- upper bounds of every such
//                   T's layer lengths) with the frame counts as runtime values; odd block lengths
//                   take the ceil-mode pooling tail.  Real utterances of 65-127 frames then run at the
//                   128-frame kernels' cost instead of the generic instances' ~2x.
// Fragment counts are never runtime values: MFMA code under runtime per-fragment
// guards produced wrong results on gfx950 for one-fragment layers.
// ---------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------
// The two passes are device functions: launched on their own (se_fwd_fused / se_bwd_fused) or back to back per
// iteration inside the persistent attack kernel (se_attack_fused, KT = false: no per-pass kernel stamps).
template <int PREC, int SH, bool KT>
__device__ __forceinline__ void se_fwd_body(const FusedArgs& A) {
    constexpr int STD = (SH == 0 || SH == 16) ? 1 : 0;
    constexpr bool RT = SH == 16;               // standard classes, runtime frame counts
    constexpr int G = STD ? 8 : SH;             // fragments per (non-dgrad) layer
    using E = typename Fz<PREC>::E;
    constexpr int RS = Fz<PREC>::RS;
    constexpr int ESZ = (int)sizeof(E);
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int NF = 8;
    constexpr bool DBUF = PREC == PREC_BF16;   // double-buffered bank output (LDS room)
    // bf16, standard shape (ReLU, no ContentEncoder InstanceNorm there): bank / conv1 epilogues pack first
    constexpr bool PKRELU = AVC_FZ_PKRELU && PREC == PREC_BF16 && STD != 0;
    int b = blockIdx.x;
    if constexpr (!KT) asm volatile("" : "+s"(b));   // (persistent kernel: nothing derived from it crosses a pass)
    // a ragged batch (runtime-length kernels only): this workgroup's own length and packed offset
    // (per-pass launches only: with it the persistent shape-16 instance crashed the backend's AGPR-copy pass)
    const RagUtt* const ru = (RT && KT && A.rag) ? A.rag + b : nullptr;
    const int T = (STD && !RT) ? StdSE::T : (ru ? ru->T : A.T);
    const size_t xoff = ru ? (size_t)ru->xoff : (size_t)b * FZ_CIN * T;
    auto TLr = [&](int l) __attribute__((always_inline)) { return ru ? StdSE::Tl_of(T, l) : A.Tl[l]; };
    const int nb = STD ? StdSE::NB : A.nb;
    const int nblk = STD ? StdSE::NBLK : A.nblk;
    const int ks = STD ? StdSE::KSZ : A.ks;
    const int P = ks / 2;
    int tid = threadIdx.x;
    // (persistent kernel: the lane index made opaque per pass, so LICM cannot hoist the lane-derived LDS / HBM
    // offsets of both passes out of the iteration loop -- live across it they spilled ~1k VGPRs)
    if constexpr (!KT) asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, kq = lane >> 4;
    const int act = STD ? 0 : A.act;                   // the standard shape is ReLU (host-checked)
    FZ_PH_DECL
    FZ_PH();
    KTime* const kt = &g_ktime_fused[KT_FUSED_FWD + (PREC == PREC_BF16)];
    const KtStart kts = KT ? ktime_begin(kt) : KtStart{0ull, false};
    if (A.tick && b == 0 && tid == 0) atomicAdd(A.tick, 1);

    char* XB = fz_lds;                                  // x image [T+8][80], pad 4
    char* BK0 = XB + (T + 8) * RS;                      // bank output [T][128]
    char* BK1 = DBUF ? BK0 + T * RS : BK0;
    char* HB = fz_lds;                                  // block input image [T+2P][128]
    char* YB = HB + (T + 2 * P) * RS;                   // conv1 output image

    const bool ce = A.ce_mode != 0;                     // ContentEncoder pass
    u64* mbase = A.masks + (size_t)b * A.mask_words;
    const bool wm = A.write_masks != 0 && !ce;
    const int ch0 = 32 * w + 4 * kq;                    // + 16*i + r
    constexpr int WPL = FZ_MASK_WORDS_PER_LAYER / 4;    // mask words per (layer, wave)

    const auto nf0 = IC<G>{};
    const int ns_c = ks * FZ_C / KS;
    // the A operands of the pass, in launch order (each GEMM prefetches the next one's)
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
    auto op_mean = [&]() __attribute__((always_inline)) { return aop(A.w.mean_w, 2 * w, 2, FZ_C / KS, FZ_C / KS); };
    ARing<2, STD ? AVC_FZ_RD_FWD : 4> ring;
    ring_fill(ring, op_bank(0));
    // ---- x -> XB (transposed, reflect rows).  Lane (t, half) of the 128 frame slots reads
    // x[ci][t] for the VE channels of every other channel group (coalesced: two 128-B runs
    // per wave load) and writes each group as ONE 16-byte LDS store.  A row is 2 mod 16
    // 16-byte slots long, so the 16 lanes (8 frames x 2 halves) of a store phase hit 16
    // distinct slots: conflict-free.  All loads are issued before any store (one HBM round
    // trip); the first GEMM's weight ring is filled before them and lands meanwhile.
    constexpr int NGX = FZ_CIN / VE;                    // 16-byte channel groups of a row
    constexpr int GPT = NGX / 2;                        // groups per thread
    static_assert(NGX % 2 == 0, "channel groups split over two lanes");
    const int xt = 32 * w + (lane >> 1), xh = lane & 1;
    float xv[GPT][VE];
    {
        const float* xs = A.x + xoff + xt;
        if (xt < T) {
#pragma unroll
            for (int m = 0; m < GPT; ++m)
#pragma unroll
                for (int e = 0; e < VE; ++e) xv[m][e] = xs[(size_t)((2 * m + xh) * VE + e) * T];
        }
    }
    if (xt < T) {
#pragma unroll
        for (int m = 0; m < GPT; ++m) {
            f32x4 v;
            if constexpr (PREC == PREC_F32) {
                v = f32x4{xv[m][0], xv[m][1], xv[m][2], xv[m][3]};
            } else {
                v = pk_bf16x8([&](int e) { return xv[m][e]; });
            }
            const int cb = (2 * m + xh) * 16;
            *reinterpret_cast<f32x4*>(XB + (4 + xt) * RS + cb) = v;
            if (xt >= 1 && xt <= 4) *reinterpret_cast<f32x4*>(XB + (4 - xt) * RS + cb) = v;
            if (xt >= T - 5 && xt <= T - 2) *reinterpret_cast<f32x4*>(XB + (4 + 2 * T - 2 - xt) * RS + cb) = v;
        }
    }
    __syncthreads();
    FZ_PH();
    int rb[NF];
    f32x4 acc_h[2][NF];
    zero_acc(acc_h);
    MaskAcc mk;
    // biases are loaded ahead of the GEMM that precedes their epilogue (their latency
    // then hides under it instead of stalling the epilogue)
    f32x4 b_in[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) b_in[i] = *reinterpret_cast<const f32x4*>(A.w.b_in + ch0 + 16 * i);
    // one bank kernel + its in_conv block; compile-time kb for the standard shape (every
    // GEMM's step count and operand map a constant: the runtime loop's K loops carried ~4x
    // the VALU/SALU work per step)
    auto bank_fwd = [&](auto KB) __attribute__((always_inline)) {
        const int kb = KB;
        const int k = kb + 1;
        const int pl = k / 2;
        f32x4 bkb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) bkb[i] = *reinterpret_cast<const f32x4*>(A.w.b_bank[kb] + ch0 + 16 * i);
        f32x4 acc[2][NF];
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, T - 1) + 4 - pl;
        fz_gemm<PREC, 2, NF, FZ_CIN, 1>(acc, nf0, ring, op_bank(kb), op_inb(kb), XB, rb);
        FZ_PH();
        char* BK = (kb & 1) ? BK1 : BK0;
        mk = MaskAcc();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const f32x4 bi = bkb[i];
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if (f >= nf0) continue;
                const int t = 16 * f + c;
                if constexpr (PKRELU) {   // ReLU' bit from the pre-activation, ReLU on the packed bf16 pairs
                    const f32x4 x = acc[i][f] + bi;
#pragma unroll
                    for (int r = 0; r < 4; ++r) mk.put(i, f, r, x[r]);
                    if (t < T) *reinterpret_cast<u32x2*>(BK + t * RS + (ch0 + 16 * i) * ESZ) = relu_pk_bf16x4(x);
                } else {
                    f32x4 y;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        y[r] = act_f(acc[i][f][r] + bi[r], act);
                        mk.put(i, f, r, y[r]);
                    }
                    if (t < T) st4<PREC>(BK + t * RS + (ch0 + 16 * i) * ESZ, y);
                }
            }
        }
        if (wm) mk.store(mbase + (size_t)(kb * 4 + w) * WPL);
        __syncthreads();
        FZ_PH();
        // in_conv over this bank block (K = 128 channels of the block)
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, T - 1);
        fz_gemm<PREC, 2, NF, FZ_C, 1>(acc_h, nf0, ring, op_inb(kb), kb + 1 < nb ? op_bank(kb + 1) : op_inx(), BK, rb);
        if (!DBUF) __syncthreads();
        FZ_PH();
    };
    if constexpr (STD != 0) {
        static_for<0, StdSE::NB>([&](auto KB) __attribute__((always_inline)) { bank_fwd(KB); });
    } else {
        for (int kb = 0; kb < nb; ++kb) bank_fwd(kb);
    }
    {   // in_conv, x block (K = 80)
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, T - 1) + 4;
        fz_gemm<PREC, 2, NF, FZ_CIN, 1>(acc_h, nf0, ring, op_inx(), op_c1(0), XB, rb);
    }
    __syncthreads();   // XB / BK are dead: HB and YB alias them
    FZ_PH();

    // h0 = act(in_conv + b): fp32 residual stream in registers, operand image in HB
    f32x4 hres[2][NF];
    {
        mk = MaskAcc();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int f = 0; f < NF; ++f) acc_h[i][f] += b_in[i];
        }
        if (ce) {   // ContentEncoder: InstanceNorm before the act (models.py:199-200)
            f32x4 is[2];
            inorm_rows(acc_h, nf0, T, is);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = act_f(acc_h[i][f][r], act);
                    mk.put(i, f, r, y[r]);
                }
                hres[i][f] = y;
                const int t = 16 * f + c;
                if (f < nf0 && t < T) put_reflect<PREC>(HB, t, T, P, (ch0 + 16 * i) * ESZ, y);
            }
        }
        if (wm) mk.store(mbase + (size_t)(nb * 4 + w) * WPL);
    }
    __syncthreads();
    FZ_PH();

    // one conv block (models.py:285-305); nfi / nfo: fragments of its input / output frames
    auto block = [&](auto nfi, auto nfo, int l, int Ti, int To, int s) __attribute__((always_inline)) {
        f32x4 acc[2][NF];
        f32x4 bc1[2], bc2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            bc1[i] = *reinterpret_cast<const f32x4*>(A.w.b_c1[l] + ch0 + 16 * i);
            bc2[i] = *reinterpret_cast<const f32x4*>(A.w.b_c2[l] + ch0 + 16 * i);
        }
        // conv1 (stride 1): y1 = act(conv1(h) + b1) -> YB
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, Ti - 1);
        fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, nfi, ring, op_c1(l), op_c2(l), HB, rb);
        FZ_PH();
        mk = MaskAcc();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int f = 0; f < NF; ++f) acc[i][f] += bc1[i];
        }
        if (ce) {
            f32x4 is[2];
            inorm_rows(acc, nfi, Ti, is);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if (f >= nfi) continue;
                const int t = 16 * f + c;
                if constexpr (PKRELU) {   // as in the bank epilogue (the conv1 output only feeds conv2's image)
#pragma unroll
                    for (int r = 0; r < 4; ++r) mk.put(i, f, r, acc[i][f][r]);
                    if (t < Ti) put_reflect_pk(YB, t, Ti, P, (ch0 + 16 * i) * ESZ, relu_pk_bf16x4(acc[i][f]));
                } else {
                    f32x4 y;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        y[r] = act_f(acc[i][f][r], act);
                        mk.put(i, f, r, y[r]);
                    }
                    if (t < Ti) put_reflect<PREC>(YB, t, Ti, P, (ch0 + 16 * i) * ESZ, y);
                }
            }
        }
        if (wm) mk.store(mbase + (size_t)((nb + 1 + 2 * l) * 4 + w) * WPL);
        __syncthreads();
        FZ_PH();
        // conv2 (stride s): y2 = act(conv2(y1) + b2); h = y2 + avg_pool1d(h, s, ceil_mode)
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, To - 1) * s;
        fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, nfo, ring, op_c2(l),
                                      l + 1 < nblk ? op_c1(l + 1) : (ce ? op_mean() : op_c2(l)), YB, rb);
        FZ_PH();
        if (AVC_FZ_POOLDPP && STD != 0 && s == 2 && (!RT || (Ti & 1) == 0)) {
            // the standard shape's stride-2 layers have even input lengths: every pooled frame averages a
            // pair.  The pair sum h[2t'] + h[2t'+1] is formed in place by a quad-permute DPP add (lane 2k
            // holds it; the same bits as the add below, fp addition being commutative), then one lane
            // shuffle per source fragment compacts it -- 2 ds_bpermute per element instead of 4.
            const int src0 = (lane & 48) | ((2 * c) & 15);
#pragma unroll
            for (int fo = 0; fo < NF; ++fo) {
                if (fo >= nfo) continue;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x4 sa = hres[i][(2 * fo) < NF ? 2 * fo : NF - 1];
                    const f32x4 sb = hres[i][(2 * fo + 1) < NF ? 2 * fo + 1 : NF - 1];
                    f32x4 pv;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float pa = sa[r] + dpp_mov<0xB1>(sa[r]), pb = sb[r] + dpp_mov<0xB1>(sb[r]);
                        const float a = __shfl(pa, src0), bb = __shfl(pb, src0);
                        pv[r] = (c < 8 ? a : bb) / 2.f;
                    }
                    hres[i][fo] = pv;
                }
            }
        } else if (s == 2) {
            // pooled[t'] = (h[2t'] + h[2t'+1]) / cnt : sources in frags 2f', 2f'+1; increasing f'
            // order keeps the in-place update safe (frag f' is read before it is written)
            const int src0 = (lane & 48) | ((2 * c) & 15), src1 = (lane & 48) | ((2 * c + 1) & 15);
#pragma unroll
            for (int fo = 0; fo < NF; ++fo) {
                if (fo >= nfo) continue;
                const int t = 16 * fo + c;
                const bool two = 2 * t + 1 < Ti;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x4 sa = hres[i][(2 * fo) < NF ? 2 * fo : NF - 1];
                    const f32x4 sb = hres[i][(2 * fo + 1) < NF ? 2 * fo + 1 : NF - 1];
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
        mk = MaskAcc();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int f = 0; f < NF; ++f) acc[i][f] += bc2[i];
        }
        if (ce) {
            f32x4 is[2];
            inorm_rows(acc, nfo, To, is);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if (f >= nfo) continue;
                f32x4 y, h;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = act_f(acc[i][f][r], act);
                    mk.put(i, f, r, y[r]);
                    h[r] = y[r] + hres[i][f][r];
                }
                hres[i][f] = h;
                const int t = 16 * f + c;
                if (t < To) put_reflect<PREC>(HB, t, To, P, (ch0 + 16 * i) * ESZ, h);
            }
        }
        if (wm) mk.store(mbase + (size_t)((nb + 2 + 2 * l) * 4 + w) * WPL);
        __syncthreads();
        FZ_PH();
    };
    int TN;
    if constexpr (STD != 0) {
        static_for<0, StdSE::NBLK>([&](auto L) __attribute__((always_inline)) {
            constexpr int l = decltype(L)::value;
            block(IC<StdSE::nf(StdSE::Tl(l))>{}, IC<StdSE::nf(StdSE::Tl(l + 1))>{}, l, RT ? TLr(l) : StdSE::Tl(l),
                  RT ? TLr(l + 1) : StdSE::Tl(l + 1), StdSE::sub(l));
        });
        TN = RT ? TLr(StdSE::NBLK) : StdSE::Tl(StdSE::NBLK);
    } else if (fz_std_sub(A)) {
        // the standard subsample pattern at another length: each block on the fragment count of its
        // own frames (G >> stride-2 blocks before it, at least 1) instead of the input's G -- the deeper
        // blocks computed 2-8x the fragments they hold (T = 120: se_fwd_fused 126 us against 84 us)
        static_for<0, 6>([&](auto L) __attribute__((always_inline)) {
            constexpr int l = decltype(L)::value;
            block(IC<fz_cls(G, l / 2)>{}, IC<fz_cls(G, (l + 1) / 2)>{}, l, A.Tl[l], A.Tl[l + 1], A.sub[l]);
        });
        TN = A.Tl[6];
    } else {
        for (int l = 0; l < A.nblk; ++l)
            block(IC<G>{}, IC<G>{}, l, A.Tl[l], A.Tl[l + 1], A.sub[l]);
        TN = A.Tl[A.nblk];
    }

    if (ce) {
        // mean_layer (1x1, models.py:207): mu = W_mean h_N + b over the TN frames of HB
        f32x4 acc[2][NF];
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = P + min(16 * f + c, TN - 1);
        fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, nf0, ring, op_mean(), op_mean(), HB, rb);
        float* mu = A.mu_out + (size_t)b * FZ_C * TN;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const f32x4 bi = *reinterpret_cast<const f32x4*>(A.w.b_mean + ch0 + 16 * i);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = 16 * f + c;
                if (t < TN)
#pragma unroll
                    for (int r = 0; r < 4; ++r) mu[(size_t)(ch0 + 16 * i + r) * TN + t] = acc[i][f][r] + bi[r];
            }
        }
        ktime_end(kt, kts);
        return;
    }
    // AdaptiveAvgPool1d(1): mean over the TN frames of each channel
    float* hsm = reinterpret_cast<float*>(fz_lds);      // fused head's LDS (conv images dead)
    const bool fh = PREC == PREC_BF16 && A.fuse_head != 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int f = 0; f < NF; ++f)
            if (16 * f + c < TN) s4 += hres[i][f];
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
    FZ_PH();
    if constexpr (PREC == PREC_BF16) {
        if (fh) {
            if constexpr (STD != 0) {
                if (A.fuse_head == 2) se_head_fused<StdSE::NDENSE, 0>(A.head, b, hsm, A.loss_cur);
                else se_head_fused<StdSE::NDENSE, 1>(A.head, b, hsm, A.loss_cur);
            }
            FZ_PH();
        }
    }
    FZ_PH_DUMP("fwd");
    ktime_end(kt, kts);
}

// ---------------------------------------------------------------------------------
// backward + Adam
// ---------------------------------------------------------------------------------
// sraw: the Adam step counter as the iteration sees it (1-based; the loss-history row and the grad0 test)
template <int PREC, int SH, bool KT>
__device__ __forceinline__ void se_bwd_body(const FusedArgs& A, const int sraw) {
    constexpr int STD = (SH == 0 || SH == 16) ? 1 : 0;
    constexpr bool RT = SH == 16;               // standard classes, runtime frame counts
    // the 128-frame LDS layout with unconditional stores (bf16; the fp32 instance of it crashes the gfx950
    // backend's AGPR-copy rewrite, so fp32 keeps the guarded stores)
    constexpr bool RTU = RT && PREC == PREC_BF16;
    constexpr int G = STD ? 8 : SH;
    using E = typename Fz<PREC>::E;
    constexpr int RS = Fz<PREC>::RS;
    constexpr int ESZ = (int)sizeof(E);
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int NF = FZ_MAXNF;
    constexpr int ZP = 4;          // zero rows around a block dY image
    constexpr int ZPB = 8;         // ... around a bank dY image
    constexpr int EB = 4;          // bank dgrad edge columns per side
    constexpr int WPL = FZ_MASK_WORDS_PER_LAYER / 4;
    int b = blockIdx.x;
    if constexpr (!KT) asm volatile("" : "+s"(b));   // (persistent kernel: nothing derived from it crosses a pass)
    // a ragged batch (runtime-length kernels only): this workgroup's own length and packed offset
    // (per-pass launches only: with it the persistent shape-16 instance crashed the backend's AGPR-copy pass)
    const RagUtt* const ru = (RT && KT && A.rag) ? A.rag + b : nullptr;
    const int T = (STD && !RT) ? StdSE::T : (ru ? ru->T : A.T);
    const size_t xoff = ru ? (size_t)ru->xoff : (size_t)b * FZ_CIN * T;
    auto TLr = [&](int l) __attribute__((always_inline)) { return ru ? StdSE::Tl_of(T, l) : A.Tl[l]; };
    const int nb = STD ? StdSE::NB : A.nb;
    const int ks = STD ? StdSE::KSZ : A.ks;
    const int P = ks / 2;
    int tid = threadIdx.x;
    // (persistent kernel: the lane index made opaque per pass, so LICM cannot hoist the lane-derived LDS / HBM
    // offsets of both passes out of the iteration loop -- live across it they spilled ~1k VGPRs)
    if constexpr (!KT) asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, kq = lane >> 4;
    const int act = STD ? 0 : A.act;                   // the standard shape is ReLU (host-checked)
    const int ch0 = 32 * w + 4 * kq;
    FZ_PH_DECL
    FZ_PH();
    KTime* const kt = &g_ktime_fused[KT_FUSED_BWD + (PREC == PREC_BF16)];
    const KtStart kts = KT ? ktime_begin(kt) : KtStart{0ull, false};
    const u64* mbase = A.masks + (size_t)b * A.mask_words;
    // Shape-generic bf16 kernels read the ReLU' words from an LDS copy of the utterance's set (made once,
    // below): their K loops have runtime step counts, so the waitcnt pass cannot count the weight-ring loads
    // issued after a word's global load and waited for it with vmcnt(0) -- draining the next GEMM's ring
    // at every masked epilogue (T = 120: se_bwd_fused 184 us against 84 us for the standard shape).
    constexpr bool MLDS = STD == 0 && PREC == PREC_BF16;
    u64* const MKL = reinterpret_cast<u64*>(fz_lds + fz_lds_bwd(PREC, T));   // (fz_lds_bwd_masks)
    auto mwords = [&](int layer) __attribute__((always_inline)) {
        if constexpr (MLDS) return (const u64*)(MKL + (size_t)(layer * 4 + w) * WPL);
        else return mbase + (size_t)(layer * 4 + w) * WPL;
    };

    // g_pooled, then the first GEMM's weight ring and mask words, are issued before the
    // LDS clearing so their latency hides under it
    const int TN = (STD && !RT) ? StdSE::Tl(StdSE::NBLK) : (RT ? TLr(StdSE::NBLK) : A.Tl[A.nblk]);
    f32x4 gp[2];
    if constexpr (PREC == PREC_BF16 && STD != 0) {
        if (A.fuse_head == 3) {   // e2e / fb: the head's backward (se_head_v mode 3) runs here
            float* hsm = reinterpret_cast<float*>(fz_lds);
            se_head_fused<StdSE::NDENSE, 3>(A.head, b, hsm, nullptr);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) gp[i][r] = hsm[hpos(ch0 + 16 * i + r)];
            __syncthreads();
            FZ_PH();
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i)
                gp[i] = *reinterpret_cast<const f32x4*>(A.g_pooled + (size_t)b * FZ_C + ch0 + 16 * i);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) gp[i] = *reinterpret_cast<const f32x4*>(A.g_pooled + (size_t)b * FZ_C + ch0 + 16 * i);
    }
    const int ns_c = ks * FZ_C / KS;
    const int nblk = STD ? StdSE::NBLK : A.nblk;
    auto op_c1T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c1T[l], 2 * w, 2, ns_c, ns_c); };
    auto op_c2T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c2T[l], 2 * w, 2, ns_c, ns_c); };
    ARing<2, STD ? AVC_FZ_RD_BWD : 4> ring;
    ring_fill(ring, op_c2T(nblk - 1));
    if constexpr (MLDS) {   // the utterance's ReLU' words -> LDS: every 16-byte piece in flight at once
        const int n16 = A.mask_words / 2;                        // (288 words per layer: even)
        constexpr int MKP = 16;                                  // 64 KB >= the largest set (25 layers: 57.6 KB)
        const f32x4* src = reinterpret_cast<const f32x4*>(mbase);
        f32x4* dst = reinterpret_cast<f32x4*>(MKL);
        f32x4 v[MKP];
#pragma unroll
        for (int k = 0; k < MKP; ++k) v[k] = src[min(tid + 256 * k, n16 - 1)];
#pragma unroll
        for (int k = 0; k < MKP; ++k)
            if (tid + 256 * k < n16) dst[tid + 256 * k] = v[k];
    }
    // ReLU' words of the next layer whose mask is applied, loaded one GEMM ahead
    MaskRd mnext;
    if constexpr (!MLDS) mnext.load(mwords(nb + 2 + 2 * (nblk - 1)));

    // Runtime lengths (RT): the LDS images are laid out for the classes' bound (128 frames), so every store of
    // a fragment's frames can be unconditional -- a frame past a layer's end stores a zero, which is what
    // the zero-padded dgrad images hold there.  (Per-lane `t < T` store guards under runtime lengths cost
    // exec-mask branches whose joins the waitcnt pass answers with full drains: the 36 us the SH = 16
    // backward took over SH = 0 at the same T = 128, round-6 ablation.)
    const int TL = RTU ? StdSE::T : T;
    char* GB = fz_lds;                          // dilated dY image [TL+2ZP] rows
    char* GB2 = GB + (TL + 2 * ZP) * RS;        // stride-1 dY image [TL+2ZP] rows
    float* FSCR = reinterpret_cast<float*>(fz_lds + fz_lds_bwd_main(PREC, TL)) + w * (5 * 16 * 8);
    {   // zero both images (pad rows and dilation holes must read as 0)
        const int n16 = 2 * (TL + 2 * ZP) * RS / 16;
        for (int i = tid; i < n16; i += 256) reinterpret_cast<f32x4*>(fz_lds)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // g(h_N): d mean / d h = 1/TN on the TN valid frames
    f32x4 gh[2][NF];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x4 g = gp[i];
#pragma unroll
        for (int r = 0; r < 4; ++r) g[r] = g[r] / (float)TN;
#pragma unroll
        for (int f = 0; f < NF; ++f) gh[i][f] = (16 * f + c < TN) ? g : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    if constexpr (MLDS) mnext.load(mwords(nb + 2 + 2 * (nblk - 1)));   // (the LDS copy is complete)
    FZ_PH();

    int rb[NF];
    // backward of one conv block; nfo: fragments of its output frames, nfc: of the
    // dgrad columns (Ti interior frames + 2P pad positions)
    auto block = [&](auto nfo, auto nfc, int l, int Ti, int To, int s) __attribute__((always_inline)) {
        // dY of conv2 = g(h_{l+1}) * act'(y2_l), written dilated by s into GB
        {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < 8; ++f) {
                    if (f >= nfo) continue;
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        v[r] = mnext.gate(i, f, r, gh[i][f][r], act);
                    const int t = 16 * f + c;
                    if (RTU || t < To) {   // RTU: g(h_{l+1}) is zero past To (the row gets its zero)
                        st4<PREC>(GB + (ZP + s * t) * RS + (ch0 + 16 * i) * ESZ, v);
                        if (s == 2)
                            st4<PREC>(GB + (ZP + 2 * t + 1) * RS + (ch0 + 16 * i) * ESZ, f32x4{0.f, 0.f, 0.f, 0.f});
                    }
                }
        }
        __syncthreads();
        FZ_PH();
        // conv2^T
        const int ncol = Ti + 2 * P;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const int n = 16 * f + c;
            rb[f] = ZP + (n < ncol ? vpos(n, Ti, P) : 0) + P;
        }
        f32x4 acc[2][NF];
        zero_acc(acc);
        MaskRd m1;
        m1.load(mwords(nb + 1 + 2 * l));
        fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, nfc, ring, op_c2T(l), op_c1T(l), GB, rb);
        FZ_PH();
        // wave-local fold: GB2 (written next) was last read before this block's first barrier
        fold_edges<false>(acc, Ti, P, FSCR);
        FZ_PH();
        {   // * act'(y1_l) -> GB2 (stride 1)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < 8; ++f) {
                    if (16 * f >= Ti) continue;
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        v[r] = m1.gate(i, f, r, acc[i][f][r], act);
                    const int t = 16 * f + c;
                    if constexpr (RTU) {
                        st4<PREC>(GB2 + (ZP + t) * RS + (ch0 + 16 * i) * ESZ, t < Ti ? v : f32x4{0.f, 0.f, 0.f, 0.f});
                    } else {
                        if (t < Ti) st4<PREC>(GB2 + (ZP + t) * RS + (ch0 + 16 * i) * ESZ, v);
                    }
                }
        }
        __syncthreads();
        FZ_PH();
        // conv1^T (+ fold) + avg_pool^T of g(h_{l+1}) -> g(h_l)
        zero_acc(acc);
        mnext.load(mwords(l > 0 ? nb + 2 + 2 * (l - 1) : nb));   // next block's conv2, or h0
        fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, nfc, ring, op_c1T(l), l > 0 ? op_c2T(l - 1) : op_c1T(l), GB2, rb);
        FZ_PH();
        // wave-local fold: GB (written next) was last read before the act' barrier above
        fold_edges<false>(acc, Ti, P, FSCR);
        if (s == 2) {
            // g_h[t] += g_{l+1}[t/2] / cnt(t/2) (torch avg_pool backward: grad / divide_factor);
            // decreasing f keeps the in-place update safe (frag f reads frag f/2)
#pragma unroll
            for (int f = 7; f >= 0; --f) {
                const int t = 16 * f + c;
                const bool two = 2 * (t >> 1) + 1 < Ti;
                const int srcl = (lane & 48) | (8 * (f & 1) + (c >> 1));
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x4 sv = gh[i][f >> 1];
                    f32x4 ng;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float g = __shfl(sv[r], srcl);
                        ng[r] = t < Ti ? acc[i][f][r] + (two ? g / 2.f : g) : 0.f;
                    }
                    gh[i][f] = ng;
                }
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) gh[i][8] = f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const int t = 16 * f + c;
                    gh[i][f] = t < Ti ? acc[i][f] + gh[i][f] : f32x4{0.f, 0.f, 0.f, 0.f};
                }
        }
        FZ_PH();
    };
    if constexpr (STD != 0) {
        static_for<0, StdSE::NBLK>([&](auto L) __attribute__((always_inline)) {
            constexpr int l = StdSE::NBLK - 1 - decltype(L)::value;
            constexpr int Tic = StdSE::Tl(l), Toc = StdSE::Tl(l + 1);   // the classes' bounds
            block(IC<StdSE::nf(Toc)>{}, IC<StdSE::nf(Tic + 2 * (StdSE::KSZ / 2))>{}, l, RT ? TLr(l) : Tic,
                  RT ? TLr(l + 1) : Toc, StdSE::sub(l));
        });
    } else if (fz_std_sub(A)) {   // per-block fragment counts, as in the forward
        static_for<0, 6>([&](auto L) __attribute__((always_inline)) {
            constexpr int l = 5 - decltype(L)::value;
            block(IC<fz_cls(G, (l + 1) / 2)>{}, IC<fz_cls(G, l / 2) + 1>{}, l, A.Tl[l], A.Tl[l + 1], A.sub[l]);
        });
    } else {
        for (int l = A.nblk - 1; l >= 0; --l)
            block(IC<G>{}, IC<G + 1>{}, l, A.Tl[l], A.Tl[l + 1], A.sub[l]);
    }

    // g_pre0 = g(h0) * act'(h0) -> GP (= GB image, rows ZP + t; pad rows are zero)
    char* GP = GB;
    const auto nf0 = IC<G>{};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            if (f >= nf0) continue;
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = mnext.gate(i, f, r, gh[i][f][r], act);
            const int t = 16 * f + c;
            if (RTU || t < T) st4<PREC>(GP + (ZP + t) * RS + (ch0 + 16 * i) * ESZ, v);   // (RT: g(h0) zero past T)
        }
    __syncthreads();
    FZ_PH();

    // bank dgrad, K split over waves: wave w sums over bank channels [32w, 32w+32) of
    // every bank kernel and produces a partial g(x) over all 80 x (T + 2*EB) columns.
    char* GBK = GB2;                            // per-wave channel slices, [T+2ZPB] rows
    {   // zero this wave's channel slice of the GBK pad rows
        constexpr int V16 = 32 * ESZ / 16;
        for (int idx = lane; idx < 2 * ZPB * V16; idx += 64) {
            const int rr = idx / V16, part = idx - rr * V16;
            const int row = rr < ZPB ? rr : T + rr;
            *reinterpret_cast<f32x4*>(GBK + row * RS + 32 * w * ESZ + part * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    const auto nfx = IC<STD ? StdSE::nf(StdSE::T + 2 * EB) : G + 1>{};
    f32x4 accx[5][NF];
    zero_acc(accx);
    constexpr int SPW = 32 / KS;                // K steps of one wave's 32-channel quarter
    constexpr int SPT = FZ_C / KS;              // K steps per tap
    constexpr int LG = SPW == 1 ? 0 : 1;
    auto op_inTb = [&](int kb) __attribute__((always_inline)) { return aop(A.w.inT_b[kb], 2 * w, 2, SPT, SPT); };
    auto op_bankT = [&](int kb) __attribute__((always_inline)) {
        return aop(A.w.bankT[kb], 0, 5, (kb + 1) * SPT, (kb + 1) * SPW, LG, SPW - 1, SPT, w * SPW);
    };
    // The bank phase is wave-local: wave w writes g(b_k) for ITS 32 bank channels into GBK and
    // its bank_k^T GEMM reads only those channels (K split over waves), and g_pre0 (GP) is
    // read-only here -- so no workgroup barrier between the phases of a bank kernel: a wave's
    // own LDS accesses are executed in order, and a compiler fence keeps them in program order.
    // The in_conv^T GEMMs (4 bf16 K steps) take their whole A operand from registers loaded one
    // GEMM ahead (ARes); the wide 2-slot ring carries only the bank_k^T steps, prefetched across
    // in_conv^T and the gate.
    // 2 slots: see ARing (a fully unrolled 2- or 3-slot variant of this phase spilled and ran
    // slower: 99 -> 107 us per launch, A/B)
    ARing<5, 2> ring5;
    constexpr int NSI = FZ_C / KS;              // in_conv^T K steps
    ARes<NSI, 2> resi;
    MaskRd mbn;                                 // ReLU' words of the next bank kernel, a GEMM ahead
    mbn.load(mwords(0));
    {   // x passthrough of the cat: W_in[:, x block]^T g_pre0 (interior columns only)
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const int n = 16 * f + c;
            rb[f] = n < T ? ZP + n : 0;
        }
        const AOp opx = aop(A.w.inT_x, 0, 5, SPT, SPW, 30, -1, 0, w * SPW);
        ring_fill(ring5, opx);
        res_load(resi, op_inTb(0));
        fz_gemm<PREC, 5, NF, FZ_C, 1>(accx, nfx, ring5, opx, op_bankT(0), GP, rb);
    }
    FZ_PH();
    auto bank_bwd = [&](auto KB) __attribute__((always_inline)) {
        const int kb = KB;
        const int k = kb + 1, pl = k / 2;
        // g(b_k) for this wave's 32 bank channels = (W_in[:, kb]^T g_pre0) * act'(b_k)
        f32x4 acc[2][8];
        zero_acc(acc);
        const MaskRd mb = mbn;
        int rt[8];
#pragma unroll
        for (int f = 0; f < 8; ++f) rt[f] = ZP + min(16 * f + c, T - 1);
        fz_gemm_res<PREC, 2, 8, NSI, FZ_C, 1>(acc, nf0, resi, GP, rt);
        FZ_PH();
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int f = 0; f < 8; ++f) {
                if (f >= nf0) continue;
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = mb.gate(i, f, r, acc[i][f][r], act);
                const int t = 16 * f + c;
                if constexpr (RTU) {
                    st4<PREC>(GBK + (ZPB + t) * RS + (ch0 + 16 * i) * ESZ, t < T ? v : f32x4{0.f, 0.f, 0.f, 0.f});
                } else {
                    if (t < T) st4<PREC>(GBK + (ZPB + t) * RS + (ch0 + 16 * i) * ESZ, v);
                }
            }
        asm volatile("" ::: "memory");   // wave-local hand-off (see above): program order only
        if (kb + 1 < nb) {
            res_load(resi, op_inTb(kb + 1));
            mbn.load(mwords(kb + 1));
        }
        FZ_PH();
        // bank_k^T over this wave's channel quarter: rows q = v + pl - j of g(b_k)
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const int n = 16 * f + c;
            rb[f] = ZPB + (n < T + 2 * EB ? vpos(n, T, EB) : 0) + pl;
        }
        const AOp opn = kb + 1 < nb ? op_bankT(kb + 1) : op_bankT(kb);
        fz_gemm<PREC, 5, NF, FZ_C, -1>(accx, nfx, ring5, op_bankT(kb), opn, GBK, rb);
        asm volatile("" ::: "memory");
        FZ_PH();
    };
    if constexpr (STD != 0) {
        static_for<0, StdSE::NB>([&](auto KB) __attribute__((always_inline)) { bank_bwd(KB); });
    } else {
        // (a compile-time bank loop here for the default bank at other lengths: 512 VGPRs with 164
        // spilled in the bf16 instance, se_bwd_fused 176 -> 210 us at T = 120; the fp32 instance
        // crashes the gfx950 backend)
        for (int kb = 0; kb < nb; ++kb) bank_bwd(kb);
    }
    fold_edges(accx, T, EB, FSCR);
    FZ_PH();

    // deterministic cross-wave sum: ((p0 + p2) + (p1 + p3)), then tanh' + Adam
    // rows padded by 4 floats at T = 128: the 4 lane groups (kq) of a store then start 16
    // banks apart instead of on the same 16 banks (a 4-way conflict)
    // (RT: the same padded layout of the classes' bound -- 132-float rows -- every column stored)
    const int TP = (STD && !RT) || RTU ? TL + 4 : T;
    auto rq = [&](int q) __attribute__((always_inline)) { return (STD && !RT) ? q + q / (StdSE::T / 4) : q; };
    float* R0 = reinterpret_cast<float*>(fz_lds);
    float* R1 = R0 + FZ_CIN * TP;
    for (int phase = 0; phase < 2; ++phase) {
        // phase 0: waves 2, 3 store p2 -> R0, p3 -> R1;  phase 1: waves 0, 1 add p0, p1
        if ((phase == 0) == (w >= 2)) {
            float* R = (w & 1) ? R1 : R0;
#pragma unroll
            for (int i = 0; i < 5; ++i)
#pragma unroll
                for (int f = 0; f < 8; ++f) {
                    const int t = 16 * f + c;
                    if (!RTU && t >= T) continue;
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
        const int sn = sraw;
        if (sn >= 1 && sn <= A.loss_len) A.losses[(size_t)(sn - 1) * A.B + b] = A.loss_cur[b];
    }
    // RT: item k of a thread is (row ci, frames 4g .. 4g+3) of the padded [80][132] rows, g < 32; its frames
    // t < T are element (ci, t) of the utterance's [80][T] arrays (16-byte accesses when T is a multiple of 4)
    const bool vec4 = (T & 3) == 0;
    const size_t xbase = xoff;
    auto rt_item = [&](int k, int& ci, int& g4, int& nok) __attribute__((always_inline)) {
        const int it = tid + 256 * k;          // < 80 * 32 = 2560 = 10 * 256
        ci = it >> 5;
        g4 = 4 * (it & 31);
        nok = max(0, min(4, T - g4));
    };
    auto rt_ld = [&](const float* a, size_t q) __attribute__((always_inline)) {
        if (vec4) return *reinterpret_cast<const f32x4*>(a + q);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = a[min(q + e, xbase + (size_t)FZ_CIN * T - 1)];
        return v;
    };
    auto rt_st = [&](float* a, size_t q, f32x4 v, int nok) __attribute__((always_inline)) {
        if (vec4) {
            *reinterpret_cast<f32x4*>(a + q) = v;
            return;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (e < nok) a[q + e] = v[e];
    };
    if (RTU && A.gx_out) {
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            int ci, g4, nok;
            rt_item(k, ci, g4, nok);
            if (nok == 0) continue;
            const int lo = ci * TP + g4;
            rt_st(A.gx_out, xbase + (size_t)ci * T + g4,
                  *reinterpret_cast<const f32x4*>(R0 + lo) + *reinterpret_cast<const f32x4*>(R1 + lo), nok);
        }
        ktime_end(kt, kts);
        return;
    }
    if (A.gx_out) {   // d loss / d x handed on (fb: the decoder output's gradient)
        f32x4* gx = reinterpret_cast<f32x4*>(A.gx_out + xoff);
        const f32x4* R04 = reinterpret_cast<const f32x4*>(R0);
        const f32x4* R14 = reinterpret_cast<const f32x4*>(R1);
        for (int q = tid; q < FZ_CIN * T / 4; q += 256) gx[q] = R04[rq(q)] + R14[rq(q)];
        ktime_end(kt, kts);
        return;
    }
    // Adam tail (reads ptb, m, v, vc, writes ptb, m, v, adv: 320 KB per utterance, every
    // workgroup at once -- the chip's burst rate bounds it).  Hoisting the reads ahead of the
    // fold / cross-wave sum measured no gain: the loaded registers were parked in AGPRs at once
    // (a vmcnt wait there) under the bank phase's register pressure.
    const AdamArgs& Ad = A.adam;
    const float eps = A.scal[0];
    if (A.losses && tid == 0) {   // the fused head's loss of this iteration -> history row step-1
        const int sn = sraw;
        if (sn >= 1 && sn <= A.loss_len) A.losses[(size_t)(sn - 1) * A.B + b] = A.loss_cur[b];
    }
    const int step = min(max(sraw, 1), A.table_len);
    const float nstep = Ad.table[2 * (step - 1)];
    const float bc2s = Ad.table[2 * (step - 1) + 1];
    const float rbc2s = 1.f / bc2s;
    const AdamStep S{nstep, bc2s, rbc2s, eps, A.scal[3]};
    const size_t base4 = xoff / 4;
    f32x4* __restrict__ ptb4 = reinterpret_cast<f32x4*>(Ad.ptb) + base4;
    f32x4* __restrict__ m4 = reinterpret_cast<f32x4*>(Ad.m) + base4;
    f32x4* __restrict__ v4 = reinterpret_cast<f32x4*>(Ad.v) + base4;
    const f32x4* __restrict__ vc4 = reinterpret_cast<const f32x4*>(Ad.vc) + base4;
    f32x4* __restrict__ adv4 = reinterpret_cast<f32x4*>(Ad.adv) + base4;
    f32x4* __restrict__ g04 = Ad.grad0 && step == 1 ? reinterpret_cast<f32x4*>(Ad.grad0) + base4 : nullptr;
    const f32x4* R04 = reinterpret_cast<const f32x4*>(R0);
    const f32x4* R14 = reinterpret_cast<const f32x4*>(R1);
    if constexpr (RTU) {   // the class-layout items (see rt_item): one batch, loads first
        constexpr int AB = 10;
        f32x4 sP[AB], sM[AB], sV[AB], sX[AB];
        size_t qa[AB];
        int nk[AB], lo[AB];
#pragma unroll
        for (int k = 0; k < AB; ++k) {
            int ci, g4;
            rt_item(k, ci, g4, nk[k]);
            qa[k] = xbase + (size_t)ci * T + min(g4, T - (vec4 ? 4 : 1));
            lo[k] = ci * TP + g4;
            sP[k] = rt_ld(Ad.ptb, qa[k]);
            sM[k] = rt_ld(Ad.m, qa[k]);
            sV[k] = rt_ld(Ad.v, qa[k]);
            sX[k] = rt_ld(Ad.vc, qa[k]);
        }
#pragma unroll
        for (int k = 0; k < AB; ++k) {
            if (nk[k] == 0) continue;
            const f32x4 gsum = *reinterpret_cast<const f32x4*>(R0 + lo[k]) + *reinterpret_cast<const f32x4*>(R1 + lo[k]);
            f32x4 p = sP[k], mm = sM[k], vv = sV[k], g, ad;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float pe = p[e], me = mm[e], ve = vv[e], ge, ae;
                adam_elem<PREC>(Ad, S, gsum[e], sX[k][e], pe, me, ve, ge, ae);
                p[e] = pe;
                mm[e] = me;
                vv[e] = ve;
                g[e] = ge;
                ad[e] = ae;
            }
            if (Ad.grad0 && step == 1) rt_st(Ad.grad0, qa[k], g, nk[k]);
            rt_st(Ad.ptb, qa[k], p, nk[k]);
            rt_st(Ad.m, qa[k], mm, nk[k]);
            rt_st(Ad.v, qa[k], vv, nk[k]);
            rt_st(Ad.adv, qa[k], ad, nk[k]);
        }
        FZ_PH();
        FZ_PH_DUMP("bwd");
        ktime_end(kt, kts);
        return;
    }
    // one batch of 16-byte accesses covers the utterance (80 x T / 4 <= 256 * AB at T <= 128);
    // all its loads are issued before its arithmetic (one HBM round trip)
    const int n4 = FZ_CIN * T / 4;
    constexpr int AB = 10;
    f32x4 sP[AB], sM[AB], sV[AB], sX[AB];
#pragma unroll
    for (int k = 0; k < AB; ++k) {
        const int q = min(tid + 256 * k, n4 - 1);
        sP[k] = ptb4[q];
        sM[k] = m4[q];
        sV[k] = v4[q];
        sX[k] = vc4[q];
    }
#pragma unroll
    for (int k = 0; k < AB; ++k) {
        const int q = tid + 256 * k;
        if (q >= n4) continue;
        const f32x4 gsum = R04[rq(q)] + R14[rq(q)];
        f32x4 p = sP[k], mm = sM[k], vv = sV[k], g, ad;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float pe = p[e], me = mm[e], ve = vv[e], ge, ae;
            adam_elem<PREC>(Ad, S, gsum[e], sX[k][e], pe, me, ve, ge, ae);
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
    ktime_end(kt, kts);
}

template <int PREC, int SH>
__global__ void __launch_bounds__(256, 1) se_fwd_fused(FusedArgs A) {
    se_fwd_body<PREC, SH, true>(A);
}
template <int PREC, int SH>
__global__ void __launch_bounds__(256, 1) se_bwd_fused(FusedArgs A) {
    se_bwd_body<PREC, SH, true>(A, *A.step);
}

// ---------------------------------------------------------------------------------
// Persistent emb attack: n_iters iterations (forward + fused head + backward + Adam) of ONE utterance per
// workgroup in one launch.  The utterances share nothing inside an iteration (per-utterance loss, gradient
// and Adam state), so a workgroup runs its utterance's iterations back to back: no kernel boundary per pass
// (where every workgroup waited for the slowest one and the next launch's ramp-up) -- the separate launches
// spent ~5 us per emb iteration between kernels.  Everything a pass hands to the next (adv, ReLU' words,
// pooled / g_pooled, the loss) is this workgroup's own and goes through its CU's write-through L1, so a
// workgroup-scope fence and barrier order it.  The step counter is read once (every workgroup, at its start)
// and advanced by fz_step_add after the launch, so the launch never races its own reads of it.
// ---------------------------------------------------------------------------------
template <int PREC, int SH>
__global__ void __launch_bounds__(256, 1) se_attack_fused(AtkArgs A) {
    // (the launch's start stamp parked in LDS and the loop bound re-read per iteration: the bodies run at the
    // scalar register limit, and every SGPR live across the loop spilled into VGPR lanes inside them)
    __shared__ unsigned long long kt_t0, kt_on;
    {
        const KtStart k0 = ktime_begin(&g_ktime_fused[KT_FUSED_ATK + (PREC == PREC_BF16)]);
        if (threadIdx.x == 0) {
            kt_t0 = k0.t0;
            kt_on = k0.on ? 1ull : 0ull;
        }
    }
    const int s0 = *A.b.step;
    // the arguments read through the kernarg pointer made opaque per iteration: no field load (or address
    // derived from one) is loop-invariant, so none is hoisted and kept live across the loop (taking the
    // parameter's address instead would make a private copy of it)
    for (int st = s0 + 1;; ++st) {
        auto kp = __builtin_amdgcn_kernarg_segment_ptr();   // (constant address space: scalar loads)
        asm volatile("" : "+s"(kp));
        const AtkArgs* ap = (const AtkArgs*)kp;
        if (st > s0 + ap->n_iters) break;
        se_fwd_body<PREC, SH, false>(ap->f);
        __threadfence_block();
        __syncthreads();
        se_bwd_body<PREC, SH, false>(ap->b, st);
        __threadfence_block();
        __syncthreads();
    }
    ktime_end(&g_ktime_fused[KT_FUSED_ATK + (PREC == PREC_BF16)], KtStart{kt_t0, kt_on != 0ull});
}
__global__ void fz_step_add(int32_t* step, int n) {
    if (threadIdx.x == 0) step[0] += n;
}

#define AVC_FZ_INST(P, S)                                        \
    template __global__ void se_fwd_fused<P, S>(FusedArgs);     \
    template __global__ void se_bwd_fused<P, S>(FusedArgs);
AVC_FZ_INST(PREC_F32, 0)
AVC_FZ_INST(PREC_F32, 1)
AVC_FZ_INST(PREC_F32, 2)
AVC_FZ_INST(PREC_F32, 4)
AVC_FZ_INST(PREC_F32, 8)
AVC_FZ_INST(PREC_F32, 16)
AVC_FZ_INST(PREC_BF16, 0)
AVC_FZ_INST(PREC_BF16, 1)
AVC_FZ_INST(PREC_BF16, 2)
AVC_FZ_INST(PREC_BF16, 4)
AVC_FZ_INST(PREC_BF16, 8)
AVC_FZ_INST(PREC_BF16, 16)
template __global__ void se_attack_fused<PREC_BF16, 0>(AtkArgs);
template __global__ void se_attack_fused<PREC_BF16, 16>(AtkArgs);
#undef AVC_FZ_INST

}  // namespace avc
