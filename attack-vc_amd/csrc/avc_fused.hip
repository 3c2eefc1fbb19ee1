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
#include <hip/hip_runtime.h>

#include <type_traits>

#include "avc_device.h"
#include "avc_kernels.h"
#include "avc_fused_lds.h"

namespace avc {

template <int PREC>
struct Fz;
template <>
struct Fz<PREC_F32> {
    using E = float;
    static constexpr int RS = 544;    // 128 ch * 4 B + 32 B
};
template <>
struct Fz<PREC_BF16> {
    using E = __bf16;
    static constexpr int RS = 288;    // 128 ch * 2 B + 32 B
};

extern __shared__ __attribute__((aligned(16))) char fz_lds[];

#ifndef AVC_FZ_ABLATE          // timing experiments only: 1 = no A loads, 2 = no mask bookkeeping
#define AVC_FZ_ABLATE 0
#endif

typedef unsigned long long u64;


__device__ __forceinline__ f32x4 lds16(const char* p) { return *reinterpret_cast<const f32x4*>(p); }

template <int PREC>
__device__ __forceinline__ void st4(char* p, f32x4 v) {
    if constexpr (PREC == PREC_F32) {
        *reinterpret_cast<f32x4*>(p) = v;
    } else {
        bf16x4 b;
#pragma unroll
        for (int e = 0; e < 4; ++e) b[e] = (__bf16)v[e];
        *reinterpret_cast<bf16x4*>(p) = b;
    }
}

template <int PREC>
__device__ __forceinline__ void st1(char* p, float v) {
    *reinterpret_cast<typename Fz<PREC>::E*>(p) = (typename Fz<PREC>::E)v;
}

template <int PREC>
__device__ __forceinline__ void mma(f32x4& acc, const f32x4& a, const f32x4& b) {
    if constexpr (PREC == PREC_F32) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], b[e], acc, 0, 0, 0);
    } else {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                      acc, 0, 0, 0);
    }
}

template <int MT, int NF>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[MT][NF]) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// ---------------------------------------------------------------------------------
// A operands and the cross-GEMM prefetch ring
// ---------------------------------------------------------------------------------
// One GEMM's A as seen by this wave: packed base at the wave's first M tile (lane offset
// applied), mt own tiles amt f32x4 apart, ns K steps with the step map
// ps = (s >> lg)*spt + soff + (s & msk) (identity, or a K-split over waves).
struct AOp {
    const f32x4* p;
    int amt, mt, ns, lg, msk, spt, soff;
};
__device__ __forceinline__ AOp aop(const void* packed, int tile0, int mt, int nst, int ns, int lg = 30, int msk = -1,
                                   int spt = 0, int soff = 0) {
    AOp o;
    o.p = reinterpret_cast<const f32x4*>(packed) + (size_t)tile0 * nst * 64 + (threadIdx.x & 63);
    o.amt = nst * 64;
    o.mt = mt;
    o.ns = ns;
    o.lg = lg;
    o.msk = msk;
    o.spt = spt;
    o.soff = soff;
    return o;
}
__device__ __forceinline__ const f32x4* a_step(const AOp& o, int s) {
    s = s < o.ns ? s : o.ns - 1;
    return o.p + (size_t)((s >> o.lg) * o.spt + o.soff + (s & o.msk)) * 64;
}
// Four K steps of A in flight: slot u of the ring holds step s+u.  A GEMM refills a slot
// right after using it, and the refills that run past its last step fetch the NEXT
// GEMM's first steps instead, so no GEMM starts with an exposed L2/MALL round trip.
template <int MTR>
struct ARing {
    f32x4 a[4][MTR];
};
// slot <- step s of A (s < A.ns) or step s - A.ns of N; branch-free (uniform selects);
// tiles beyond an operand's own count re-read its last tile (an L1 hit, never used)
template <int MTR>
__device__ __forceinline__ void ring_load(f32x4 (&slot)[MTR], const AOp& A, const AOp& N, int s) {
#if AVC_FZ_ABLATE & 4
    const bool own = true;   // debug: no cross-GEMM prefetch (N's steps loaded as A's last)
#else
    const bool own = s < A.ns;
#endif
    const f32x4* base = own ? a_step(A, s) : a_step(N, s - A.ns > 0 ? s - A.ns : 0);
    const int amt = own ? A.amt : N.amt;
    const int mt = own ? A.mt : N.mt;
#pragma unroll
    for (int i = 0; i < MTR; ++i)
        slot[i] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
            (const __attribute__((address_space(1))) f32x4*)(base + (size_t)(i < mt ? i : mt - 1) * amt));
#if AVC_FZ_ABLATE & 1
#pragma unroll
    for (int i = 0; i < MTR; ++i) slot[i] = f32x4{0.001f * s, 0.f, 0.f, 0.f};
#endif
}
template <int MTR>
__device__ __forceinline__ void ring_fill(ARing<MTR>& R, const AOp& A) {
#pragma unroll
    for (int u = 0; u < 4; ++u) ring_load<MTR>(R.a[u], A, A, u);
}

// acc[MT][NF] += A x B; the ring holds A's steps 0..3 on entry and N's steps 0..3 on exit.
//   B  : LDS base of the operand image; rb[f] = row of tap 0 for this lane's column
//   DJ : +1 forward (row = rb + j), -1 adjoint (row = rb - j)
// B fragments are read one step ahead into two alternating register sets.  The loop
// body has no early exits and issues every load unconditionally (steps past the end
// are clamped), so accumulators keep their registers across the back edge and the
// waitcnt pass sees a fixed number of loads in flight.
// NFC > 0: the live fragment count is the compile-time NFC (straight-line K loop);
// NFC == 0: up to NF fragments, the first `nf` live (runtime guards; generic shapes).
template <int PREC, int MT, int MTR, int NF, int NFC, int CINB, int DJ>
__device__ __forceinline__ void fz_gemm_impl(f32x4 (&acc)[MT][NF], int nf, ARing<MTR>& R, const AOp& A,
                                             const AOp& N, const char* B, const int (&rb)[NF]) {
    static_assert(MT <= MTR, "ring narrower than the GEMM");
    constexpr int NL = NFC ? NFC : NF;                 // fragments the loops run over
    auto live = [&](int f) __attribute__((always_inline)) { return NFC ? f < NFC : f < nf; };
    using E = typename Fz<PREC>::E;
    constexpr int RS = Fz<PREC>::RS;
    constexpr int VE = 16 / (int)sizeof(E);
    constexpr int KS = 4 * VE;
    const int kq = (threadIdx.x & 63) >> 4;
    const int ns = A.ns;
    int rbo[NL];
#pragma unroll
    for (int f = 0; f < NL; ++f) rbo[f] = rb[f] * RS;
    auto read_b = [&](f32x4 (&b)[NL], int s) __attribute__((always_inline)) {
        s = s < ns ? s : ns - 1;
        const int kl = KS * ((s >> A.lg) * A.spt + A.soff + (s & A.msk)) + VE * kq;
        const int j = kl / CINB;
        const int ci = kl - j * CINB;
        const char* Bs = B + ci * (int)sizeof(E) + DJ * j * RS;
#pragma unroll
        for (int f = 0; f < NL; ++f)
            if (live(f)) b[f] = lds16(Bs + rbo[f]);
    };
    auto mma_all = [&](const f32x4 (&a)[MTR], const f32x4 (&b)[NL]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int f = 0; f < NL; ++f)
                if (live(f)) mma<PREC>(acc[i][f], a[i], b[f]);
    };
    f32x4 bA[NL], bB[NL];
    read_b(bA, 0);
    const int nfull = ns & ~3;
#pragma unroll 1
    for (int s = 0; s < nfull; s += 4) {
        read_b(bB, s + 1);
        mma_all(R.a[0], bA);
        ring_load<MTR>(R.a[0], A, N, s + 4);
        read_b(bA, s + 2);
        mma_all(R.a[1], bB);
        ring_load<MTR>(R.a[1], A, N, s + 5);
        read_b(bB, s + 3);
        mma_all(R.a[2], bA);
        ring_load<MTR>(R.a[2], A, N, s + 6);
        read_b(bA, s + 4);
        mma_all(R.a[3], bB);
        ring_load<MTR>(R.a[3], A, N, s + 7);
    }
    // remainder (0..3 steps): slots hold steps nfull..nfull+3 (slot u = step nfull+u),
    // bA holds step nfull.  Afterwards rotate so that slot u = N's step u again.
    const int rem = ns - nfull;
#if AVC_FZ_ABLATE & 4
    // debug: no cross-GEMM prefetch -- finish this GEMM's own steps, then load N afresh
    if (rem >= 1) mma_all(R.a[0], bA);
    if (rem >= 2) {
        read_b(bB, nfull + 1);
        mma_all(R.a[1], bB);
    }
    if (rem >= 3) {
        read_b(bA, nfull + 2);
        mma_all(R.a[2], bA);
    }
    ring_fill(R, N);
    return;
#endif
    if (rem == 0) return;
    mma_all(R.a[0], bA);
    ring_load<MTR>(R.a[0], A, N, nfull + 4);
    if (rem >= 2) {
        read_b(bB, nfull + 1);
        mma_all(R.a[1], bB);
        ring_load<MTR>(R.a[1], A, N, nfull + 5);
    }
    if (rem >= 3) {
        read_b(bA, nfull + 2);
        mma_all(R.a[2], bA);
        ring_load<MTR>(R.a[2], A, N, nfull + 6);
    }
    // a GEMM shorter than the ring (ns < 4) entered with slots u >= ns holding clamped
    // copies of its own last step (its predecessor could not know this GEMM's successor):
    // those slots get N's steps u - rem now
    if (nfull == 0)
        for (int u = rem; u < 4; ++u) {
#pragma unroll
            for (int v = 0; v < 4; ++v)
                if (v == u) ring_load<MTR>(R.a[v], N, N, u - rem);
        }
    // slot u now holds step nfull + u + 4*(u < rem) of the A|N stream, i.e. N's step
    // (u - rem) mod 4: rotate left by rem
    f32x4 t[4][MTR];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < MTR; ++i) t[u][i] = R.a[u][i];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < MTR; ++i)
            R.a[u][i] = rem == 1 ? t[(u + 1) & 3][i] : (rem == 2 ? t[(u + 2) & 3][i] : t[(u + 3) & 3][i]);
}

template <int V>
using IC = std::integral_constant<int, V>;

// fz_gemm: the fragment count is either a compile-time IC<N> (specialised shapes) or a
// runtime int (generic shapes)
template <int PREC, int MT, int NF, int CINB, int DJ, int MTR, int NFC>
__device__ __forceinline__ void fz_gemm(f32x4 (&acc)[MT][NF], IC<NFC>, ARing<MTR>& R, const AOp& A, const AOp& N,
                                        const char* B, const int (&rb)[NF]) {
    static_assert(NFC >= 1 && NFC <= NF, "fragment count");
    fz_gemm_impl<PREC, MT, MTR, NF, NFC, CINB, DJ>(acc, NFC, R, A, N, B, rb);
}
template <int PREC, int MT, int NF, int CINB, int DJ, int MTR>
__device__ __forceinline__ void fz_gemm(f32x4 (&acc)[MT][NF], int nf, ARing<MTR>& R, const AOp& A, const AOp& N,
                                        const char* B, const int (&rb)[NF]) {
    fz_gemm_impl<PREC, MT, MTR, NF, 0, CINB, DJ>(acc, nf, R, A, N, B, rb);
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(IC<I>{});
        static_for<I + 1, N>(f);
    }
}

// position of dgrad output column n in input coordinates: interior n < Tin -> n;
// then E left pad positions -E..-1, then E right pad positions Tin..Tin+E-1
__device__ __forceinline__ int vpos(int n, int Tin, int E) {
    return n < Tin ? n : (n < Tin + E ? n - Tin - E : n - E);
}

// reflect-pad adjoint on the accumulators: the sum at pad position v folds onto
// interior frame -v (left) or 2(Tin-1)-v (right)   (F.pad mode="reflect", models.py:23-29).
// Edge column e (n = Tin + e) is staged through this wave's LDS scratch [MT*16 ch][8]
// and pulled by its target lane: fragment indices stay compile-time (no dynamic
// register indexing).  Called by all waves at the same point (contains a barrier).
template <int MT, int NF>
__device__ __forceinline__ void fold_edges(f32x4 (&acc)[MT][NF], int Tin, int E, float* scr) {
    const int lane = threadIdx.x & 63, c = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        const int e = 16 * f + c - Tin;
        if (e >= 0 && e < 2 * E) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) scr[(16 * i + 4 * kq + r) * 8 + e] = acc[i][f][r];
        }
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < NF; ++g) {
        const int t = 16 * g + c;
        const int el = (t >= 1 && t <= E) ? E - t : -1;                          // v = -t
        const int er = (t >= Tin - 1 - E && t <= Tin - 2) ? Tin - 2 - t + E : -1; // v = 2(Tin-1)-t
        if (el >= 0 || er >= 0) {
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

// 64-bit ReLU' ballot words of one layer for this wave: word (i*FZ_MAXNF + f)*4 + r
// lives in lane word%64 of lo (words < 64) or hi (words >= 64)
struct MaskAcc {
    u64 lo = 0, hi = 0;
    __device__ __forceinline__ void put(int widx, u64 word) {
        if (AVC_FZ_ABLATE & 2) return;
        const int lane = threadIdx.x & 63;
        if (widx < 64) {
            if (lane == widx) lo = word;
        } else {
            if (lane == widx - 64) hi = word;
        }
    }
    __device__ __forceinline__ void store(u64* base) const {
        const int lane = threadIdx.x & 63;
        base[lane] = lo;
        if (lane < FZ_MASK_WORDS_PER_LAYER / 4 - 64) base[64 + lane] = hi;
    }
};

__device__ __forceinline__ float act_bit(u64 word, int lane, int act) {
    return ((word >> lane) & 1ull) ? 1.f : (act ? 0.01f : 0.f);
}

// write 4 consecutive channels of frame t of a padded operand image (pad P rows each
// side, reflect): row P+t, plus its mirror rows (F.pad reflect)
template <int PREC>
__device__ __forceinline__ void put_reflect(char* img, int t, int T, int P, int chbyte, f32x4 v) {
    constexpr int RS = Fz<PREC>::RS;
    st4<PREC>(img + (P + t) * RS + chbyte, v);
    if (t >= 1 && t <= P) st4<PREC>(img + (P - t) * RS + chbyte, v);
    if (t >= T - 1 - P && t <= T - 2) st4<PREC>(img + (P + 2 * T - 2 - t) * RS + chbyte, v);
}

// ---------------------------------------------------------------------------------
// shapes (kernel template parameter SH):
//   SH = 0        : the AdaIN-VC speaker encoder at its config.yaml defaults (bank 1..8,
//                   kernel 5, six blocks with subsample [1,2,1,2,1,2]) at T = 128 -- every
//                   layer's frame and fragment count is a compile-time constant;
//   SH = 1,2,4,8  : any eligible config and T <= 16*SH; every layer runs SH fragments
//                   (SH + 1 for dgrad outputs, which carry the pad-position columns).
// Fragment counts are never runtime values: MFMA code under runtime per-fragment
// guards produced wrong results on gfx950 for one-fragment layers.
// ---------------------------------------------------------------------------------
struct StdSE {
    static constexpr int T = 128, NB = 8, KSZ = 5, NBLK = 6;
    static constexpr int sub(int l) { return (l & 1) ? 2 : 1; }
    static constexpr int Tl(int l) {
        int t = T;
        for (int i = 0; i < l; ++i) t = (t + sub(i) - 1) / sub(i);
        return t;
    }
    static constexpr int nf(int frames) { return (frames + 15) / 16; }
};


// ---------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------
template <int PREC, int SH>
__global__ void __launch_bounds__(256, 1) se_fwd_fused(FusedArgs A) {
    constexpr int STD = SH == 0 ? 1 : 0;
    constexpr int G = SH == 0 ? 8 : SH;         // fragments per (non-dgrad) layer
    using E = typename Fz<PREC>::E;
    constexpr int RS = Fz<PREC>::RS;
    constexpr int ESZ = (int)sizeof(E);
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int NF = 8;
    constexpr bool DBUF = PREC == PREC_BF16;   // double-buffered bank output (LDS room)
    const int b = blockIdx.x;
    const int T = STD ? StdSE::T : A.T;
    const int nb = STD ? StdSE::NB : A.nb;
    const int nblk = STD ? StdSE::NBLK : A.nblk;
    const int ks = STD ? StdSE::KSZ : A.ks;
    const int P = ks / 2;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, kq = lane >> 4;
    const int act = A.act;
    if (A.tick && b == 0 && tid == 0) atomicAdd(A.tick, 1);

    char* XB = fz_lds;                                  // x image [T+8][80], pad 4
    char* BK0 = XB + (T + 8) * RS;                      // bank output [T][128]
    char* BK1 = DBUF ? BK0 + T * RS : BK0;
    char* HB = fz_lds;                                  // block input image [T+2P][128]
    char* YB = HB + (T + 2 * P) * RS;                   // conv1 output image

    u64* mbase = A.masks + (size_t)b * A.mask_words;
    const bool wm = A.write_masks != 0;
    const int ch0 = 32 * w + 4 * kq;                    // + 16*i + r
    constexpr int WPL = FZ_MASK_WORDS_PER_LAYER / 4;    // mask words per (layer, wave)

    // ---- x -> XB (transposed, reflect rows)
    {
        const float* x = A.x + (size_t)b * FZ_CIN * T;
        for (int idx = tid; idx < FZ_CIN * T; idx += 256) {
            const int ci = idx / T, t = idx - ci * T;
            const float v = x[idx];
            st1<PREC>(XB + (4 + t) * RS + ci * ESZ, v);
            if (t >= 1 && t <= 4) st1<PREC>(XB + (4 - t) * RS + ci * ESZ, v);
            if (t >= T - 5 && t <= T - 2) st1<PREC>(XB + (4 + 2 * T - 2 - t) * RS + ci * ESZ, v);
        }
    }
    __syncthreads();

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
    ARing<2> ring;
    ring_fill(ring, op_bank(0));
    int rb[NF];
    f32x4 acc_h[2][NF];
    zero_acc(acc_h);
    MaskAcc mk;
    for (int kb = 0; kb < nb; ++kb) {
        const int k = kb + 1;
        const int pl = k / 2;
        f32x4 acc[2][NF];
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, T - 1) + 4 - pl;
        fz_gemm<PREC, 2, NF, FZ_CIN, 1>(acc, nf0, ring, op_bank(kb), op_inb(kb), XB, rb);
        char* BK = (kb & 1) ? BK1 : BK0;
        const float* bias = A.w.b_bank[kb];
        mk = MaskAcc();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const f32x4 bi = *reinterpret_cast<const f32x4*>(bias + ch0 + 16 * i);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if (f >= nf0) continue;
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = act_f(acc[i][f][r] + bi[r], act);
                    mk.put((i * FZ_MAXNF + f) * 4 + r, __ballot(y[r] > 0.f));
                }
                const int t = 16 * f + c;
                if (t < T) st4<PREC>(BK + t * RS + (ch0 + 16 * i) * ESZ, y);
            }
        }
        if (wm) mk.store(mbase + (size_t)(kb * 4 + w) * WPL);
        __syncthreads();
        // in_conv over this bank block (K = 128 channels of the block)
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, T - 1);
        fz_gemm<PREC, 2, NF, FZ_C, 1>(acc_h, nf0, ring, op_inb(kb), kb + 1 < nb ? op_bank(kb + 1) : op_inx(), BK, rb);
        if (!DBUF) __syncthreads();
    }
    {   // in_conv, x block (K = 80)
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, T - 1) + 4;
        fz_gemm<PREC, 2, NF, FZ_CIN, 1>(acc_h, nf0, ring, op_inx(), op_c1(0), XB, rb);
    }
    __syncthreads();   // XB / BK are dead: HB and YB alias them

    // h0 = act(in_conv + b): fp32 residual stream in registers, operand image in HB
    f32x4 hres[2][NF];
    {
        mk = MaskAcc();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const f32x4 bi = *reinterpret_cast<const f32x4*>(A.w.b_in + ch0 + 16 * i);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = act_f(acc_h[i][f][r] + bi[r], act);
                    mk.put((i * FZ_MAXNF + f) * 4 + r, __ballot(y[r] > 0.f));
                }
                hres[i][f] = y;
                const int t = 16 * f + c;
                if (f < nf0 && t < T) put_reflect<PREC>(HB, t, T, P, (ch0 + 16 * i) * ESZ, y);
            }
        }
        if (wm) mk.store(mbase + (size_t)(nb * 4 + w) * WPL);
    }
    __syncthreads();

    // one conv block (models.py:285-305); nfi / nfo: fragments of its input / output frames
    auto block = [&](auto nfi, auto nfo, int l, int Ti, int To, int s) __attribute__((always_inline)) {
        f32x4 acc[2][NF];
        // conv1 (stride 1): y1 = act(conv1(h) + b1) -> YB
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, Ti - 1);
        fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, nfi, ring, op_c1(l), op_c2(l), HB, rb);
        mk = MaskAcc();
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const f32x4 bi = *reinterpret_cast<const f32x4*>(A.w.b_c1[l] + ch0 + 16 * i);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if (f >= nfi) continue;
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = act_f(acc[i][f][r] + bi[r], act);
                    mk.put((i * FZ_MAXNF + f) * 4 + r, __ballot(y[r] > 0.f));
                }
                const int t = 16 * f + c;
                if (t < Ti) put_reflect<PREC>(YB, t, Ti, P, (ch0 + 16 * i) * ESZ, y);
            }
        }
        if (wm) mk.store(mbase + (size_t)((nb + 1 + 2 * l) * 4 + w) * WPL);
        __syncthreads();
        // conv2 (stride s): y2 = act(conv2(y1) + b2); h = y2 + avg_pool1d(h, s, ceil_mode)
        zero_acc(acc);
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(16 * f + c, To - 1) * s;
        fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, nfo, ring, op_c2(l), l + 1 < nblk ? op_c1(l + 1) : op_c2(l), YB, rb);
        if (s == 2) {
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
            const f32x4 bi = *reinterpret_cast<const f32x4*>(A.w.b_c2[l] + ch0 + 16 * i);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                if (f >= nfo) continue;
                f32x4 y, h;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = act_f(acc[i][f][r] + bi[r], act);
                    mk.put((i * FZ_MAXNF + f) * 4 + r, __ballot(y[r] > 0.f));
                    h[r] = y[r] + hres[i][f][r];
                }
                hres[i][f] = h;
                const int t = 16 * f + c;
                if (t < To) put_reflect<PREC>(HB, t, To, P, (ch0 + 16 * i) * ESZ, h);
            }
        }
        if (wm) mk.store(mbase + (size_t)((nb + 2 + 2 * l) * 4 + w) * WPL);
        __syncthreads();
    };
    int TN;
    if constexpr (STD != 0) {
        static_for<0, StdSE::NBLK>([&](auto L) __attribute__((always_inline)) {
            constexpr int l = decltype(L)::value;
            block(IC<StdSE::nf(StdSE::Tl(l))>{}, IC<StdSE::nf(StdSE::Tl(l + 1))>{}, l, StdSE::Tl(l),
                  StdSE::Tl(l + 1), StdSE::sub(l));
        });
        TN = StdSE::Tl(StdSE::NBLK);
    } else {
        for (int l = 0; l < A.nblk; ++l)
            block(IC<G>{}, IC<G>{}, l, A.Tl[l], A.Tl[l + 1], A.sub[l]);
        TN = A.Tl[A.nblk];
    }

    // AdaptiveAvgPool1d(1): mean over the TN frames of each channel
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int f = 0; f < NF; ++f)
            if (16 * f + c < TN) s4 += hres[i][f];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1)
#pragma unroll
            for (int r = 0; r < 4; ++r) s4[r] += __shfl_xor(s4[r], o);
        if (c == 0) {
            f32x4 m;
#pragma unroll
            for (int r = 0; r < 4; ++r) m[r] = s4[r] / (float)TN;
            *reinterpret_cast<f32x4*>(A.pooled + (size_t)b * FZ_C + ch0 + 16 * i) = m;
        }
    }
}

// ---------------------------------------------------------------------------------
// backward + Adam
// ---------------------------------------------------------------------------------
template <int PREC, int SH>
__global__ void __launch_bounds__(256, 1) se_bwd_fused(FusedArgs A) {
    constexpr int STD = SH == 0 ? 1 : 0;
    constexpr int G = SH == 0 ? 8 : SH;
    using E = typename Fz<PREC>::E;
    constexpr int RS = Fz<PREC>::RS;
    constexpr int ESZ = (int)sizeof(E);
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int NF = FZ_MAXNF;
    constexpr int ZP = 4;          // zero rows around a block dY image
    constexpr int ZPB = 8;         // ... around a bank dY image
    constexpr int EB = 4;          // bank dgrad edge columns per side
    constexpr int WPL = FZ_MASK_WORDS_PER_LAYER / 4;
    const int b = blockIdx.x;
    const int T = STD ? StdSE::T : A.T;
    const int nb = STD ? StdSE::NB : A.nb;
    const int ks = STD ? StdSE::KSZ : A.ks;
    const int P = ks / 2;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, kq = lane >> 4;
    const int act = A.act;
    const int ch0 = 32 * w + 4 * kq;
    const u64* mbase = A.masks + (size_t)b * A.mask_words;
    auto mword = [&](int layer, int widx) __attribute__((always_inline)) -> u64 {
        return mbase[(size_t)(layer * 4 + w) * WPL + widx];
    };

    char* GB = fz_lds;                          // dilated dY image [T+2ZP] rows
    char* GB2 = GB + (T + 2 * ZP) * RS;         // stride-1 dY image [T+2ZP] rows
    float* FSCR = reinterpret_cast<float*>(fz_lds + fz_lds_bwd_main(PREC, T)) + w * (5 * 16 * 8);
    {   // zero both images (pad rows and dilation holes must read as 0)
        const int n16 = 2 * (T + 2 * ZP) * RS / 16;
        for (int i = tid; i < n16; i += 256) reinterpret_cast<f32x4*>(fz_lds)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // g(h_N): d mean / d h = 1/TN on the TN valid frames
    const int TN = STD ? StdSE::Tl(StdSE::NBLK) : A.Tl[A.nblk];
    f32x4 gh[2][NF];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x4 g = *reinterpret_cast<const f32x4*>(A.g_pooled + (size_t)b * FZ_C + ch0 + 16 * i);
#pragma unroll
        for (int r = 0; r < 4; ++r) g[r] = g[r] / (float)TN;
#pragma unroll
        for (int f = 0; f < NF; ++f) gh[i][f] = (16 * f + c < TN) ? g : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();

    const int ns_c = ks * FZ_C / KS;
    const int nblk = STD ? StdSE::NBLK : A.nblk;
    auto op_c1T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c1T[l], 2 * w, 2, ns_c, ns_c); };
    auto op_c2T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c2T[l], 2 * w, 2, ns_c, ns_c); };
    ARing<2> ring;
    ring_fill(ring, op_c2T(nblk - 1));
    int rb[NF];
    // backward of one conv block; nfo: fragments of its output frames, nfc: of the
    // dgrad columns (Ti interior frames + 2P pad positions)
    auto block = [&](auto nfo, auto nfc, int l, int Ti, int To, int s) __attribute__((always_inline)) {
        // dY of conv2 = g(h_{l+1}) * act'(y2_l), written dilated by s into GB
        {
            const int L2 = nb + 2 + 2 * l;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < 8; ++f) {
                    if (f >= nfo) continue;
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        v[r] = gh[i][f][r] * act_bit(mword(L2, (i * FZ_MAXNF + f) * 4 + r), lane, act);
                    const int t = 16 * f + c;
                    if (t < To) {
                        st4<PREC>(GB + (ZP + s * t) * RS + (ch0 + 16 * i) * ESZ, v);
                        if (s == 2)
                            st4<PREC>(GB + (ZP + 2 * t + 1) * RS + (ch0 + 16 * i) * ESZ, f32x4{0.f, 0.f, 0.f, 0.f});
                    }
                }
        }
        __syncthreads();
        // conv2^T
        const int ncol = Ti + 2 * P;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const int n = 16 * f + c;
            rb[f] = ZP + (n < ncol ? vpos(n, Ti, P) : 0) + P;
        }
        f32x4 acc[2][NF];
        zero_acc(acc);
        fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, nfc, ring, op_c2T(l), op_c1T(l), GB, rb);
        fold_edges(acc, Ti, P, FSCR);
        {   // * act'(y1_l) -> GB2 (stride 1)
            const int L1 = nb + 1 + 2 * l;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < 8; ++f) {
                    if (16 * f >= Ti) continue;
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        v[r] = acc[i][f][r] * act_bit(mword(L1, (i * FZ_MAXNF + f) * 4 + r), lane, act);
                    const int t = 16 * f + c;
                    if (t < Ti) st4<PREC>(GB2 + (ZP + t) * RS + (ch0 + 16 * i) * ESZ, v);
                }
        }
        __syncthreads();
        // conv1^T (+ fold) + avg_pool^T of g(h_{l+1}) -> g(h_l)
        zero_acc(acc);
        fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, nfc, ring, op_c1T(l), l > 0 ? op_c2T(l - 1) : op_c1T(l), GB2, rb);
        fold_edges(acc, Ti, P, FSCR);
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
    };
    if constexpr (STD != 0) {
        static_for<0, StdSE::NBLK>([&](auto L) __attribute__((always_inline)) {
            constexpr int l = StdSE::NBLK - 1 - decltype(L)::value;
            constexpr int Ti = StdSE::Tl(l), To = StdSE::Tl(l + 1);
            block(IC<StdSE::nf(To)>{}, IC<StdSE::nf(Ti + 2 * (StdSE::KSZ / 2))>{}, l, Ti, To, StdSE::sub(l));
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
            for (int r = 0; r < 4; ++r) v[r] = gh[i][f][r] * act_bit(mword(nb, (i * FZ_MAXNF + f) * 4 + r), lane, act);
            const int t = 16 * f + c;
            if (t < T) st4<PREC>(GP + (ZP + t) * RS + (ch0 + 16 * i) * ESZ, v);
        }
    __syncthreads();

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
    ARing<5> ring5;
    {   // x passthrough of the cat: W_in[:, x block]^T g_pre0 (interior columns only)
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const int n = 16 * f + c;
            rb[f] = n < T ? ZP + n : 0;
        }
        const AOp opx = aop(A.w.inT_x, 0, 5, SPT, SPW, 30, -1, 0, w * SPW);
        ring_fill(ring5, opx);
        fz_gemm<PREC, 5, NF, FZ_C, 1>(accx, nfx, ring5, opx, op_inTb(0), GP, rb);
    }
    for (int kb = 0; kb < nb; ++kb) {
        const int k = kb + 1, pl = k / 2;
        // g(b_k) for this wave's 32 bank channels = (W_in[:, kb]^T g_pre0) * act'(b_k)
        f32x4 acc[2][8];
        zero_acc(acc);
        int rt[8];
#pragma unroll
        for (int f = 0; f < 8; ++f) rt[f] = ZP + min(16 * f + c, T - 1);
        fz_gemm<PREC, 2, 8, FZ_C, 1>(acc, nf0, ring5, op_inTb(kb), op_bankT(kb), GP, rt);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int f = 0; f < 8; ++f) {
                if (f >= nf0) continue;
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[i][f][r] * act_bit(mword(kb, (i * FZ_MAXNF + f) * 4 + r), lane, act);
                const int t = 16 * f + c;
                if (t < T) st4<PREC>(GBK + (ZPB + t) * RS + (ch0 + 16 * i) * ESZ, v);
            }
        __syncthreads();
        // bank_k^T over this wave's channel quarter: rows q = v + pl - j of g(b_k)
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const int n = 16 * f + c;
            rb[f] = ZPB + (n < T + 2 * EB ? vpos(n, T, EB) : 0) + pl;
        }
        fz_gemm<PREC, 5, NF, FZ_C, -1>(accx, nfx, ring5, op_bankT(kb), kb + 1 < nb ? op_inTb(kb + 1) : op_bankT(kb), GBK, rb);
        __syncthreads();
    }
    fold_edges(accx, T, EB, FSCR);

    // deterministic cross-wave sum: ((p0 + p2) + (p1 + p3)), then tanh' + Adam
    float* R0 = reinterpret_cast<float*>(fz_lds);
    float* R1 = R0 + FZ_CIN * T;
    for (int phase = 0; phase < 2; ++phase) {
        // phase 0: waves 2, 3 store p2 -> R0, p3 -> R1;  phase 1: waves 0, 1 add p0, p1
        if ((phase == 0) == (w >= 2)) {
            float* R = (w & 1) ? R1 : R0;
#pragma unroll
            for (int i = 0; i < 5; ++i)
#pragma unroll
                for (int f = 0; f < 8; ++f) {
                    const int t = 16 * f + c;
                    if (t >= T) continue;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float* p = R + (16 * i + 4 * kq + r) * T + t;
                        *p = phase ? accx[i][f][r] + *p : accx[i][f][r];
                    }
                }
        }
        __syncthreads();
    }

    const AdamArgs& Ad = A.adam;
    const float eps = A.scal[0];
    const int step = min(max(*A.step, 1), A.table_len);
    const float nstep = Ad.table[2 * (step - 1)];
    const float bc2s = Ad.table[2 * (step - 1) + 1];
    const size_t base = (size_t)b * FZ_CIN * T;
    for (int idx = tid; idx < FZ_CIN * T; idx += 256) {
        const size_t o = base + idx;
        const float gsum = R0[idx] + R1[idx];
        float p = Ad.ptb[o];
        const float th = tanhf(p);
        const float g = (gsum * eps) * (1.f - th * th);
        if (Ad.grad0 && step == 1) Ad.grad0[o] = g;
        float mm = Ad.m[o];
        mm = mm + Ad.b1c * (g - mm);
        float vv = Ad.v[o] * Ad.b2;
        vv = vv + Ad.b2c * g * g;
        p = p + nstep * (mm / (sqrtf(vv) / bc2s + Ad.adam_eps));
        Ad.ptb[o] = p;
        Ad.m[o] = mm;
        Ad.v[o] = vv;
        Ad.adv[o] = Ad.vc[o] + eps * tanhf(p);
    }
}

#define AVC_FZ_INST(P, S)                                        \
    template __global__ void se_fwd_fused<P, S>(FusedArgs);     \
    template __global__ void se_bwd_fused<P, S>(FusedArgs);
AVC_FZ_INST(PREC_F32, 0)
AVC_FZ_INST(PREC_F32, 1)
AVC_FZ_INST(PREC_F32, 2)
AVC_FZ_INST(PREC_F32, 4)
AVC_FZ_INST(PREC_F32, 8)
AVC_FZ_INST(PREC_BF16, 0)
AVC_FZ_INST(PREC_BF16, 1)
AVC_FZ_INST(PREC_BF16, 2)
AVC_FZ_INST(PREC_BF16, 4)
AVC_FZ_INST(PREC_BF16, 8)
#undef AVC_FZ_INST

}  // namespace avc
