// Shared device machinery of the fused per-utterance engines (SpeakerEncoder in
// avc_fused.hip, ContentEncoder/Decoder in avc_vc.hip): LDS operand images, the MFMA
// step, the cross-GEMM weight prefetch ring, the K loop, the reflect-pad adjoint fold
// and ReLU' ballot masks.  See avc_fused.hip for the design.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "avc_device.h"
#include "avc_fused_lds.h"
#include "avc_kernels.h"

#ifndef AVC_FZ_ABLATE          // timing experiments only: 1 = no A loads, 2 = no mask bookkeeping
#define AVC_FZ_ABLATE 0
#endif

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

typedef unsigned long long u64;
template <int V>
using IC = std::integral_constant<int, V>;


__device__ __forceinline__ f32x4 lds16(const char* p) { return *reinterpret_cast<const f32x4*>(p); }

// f32 -> bf16 in pairs (one v_cvt_pk_bf16_f32 each); element-wise casts made the compiler
// convert one element per instruction and re-pair them with v_perm / v_alignbit
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ u32x2 pk_bf16x4(const f32x4& v) { return u32x2{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])}; }
// 8 floats -> 8 bf16 in one 16-byte register quad (as f32x4 bits)
template <class F>
__device__ __forceinline__ f32x4 pk_bf16x8(F&& x) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    return __builtin_bit_cast(f32x4, u32x4{pk_bf16(x(0), x(1)), pk_bf16(x(2), x(3)), pk_bf16(x(4), x(5)), pk_bf16(x(6), x(7))});
}

template <int PREC>
__device__ __forceinline__ void st4(char* p, f32x4 v) {
    if constexpr (PREC == PREC_F32) {
        *reinterpret_cast<f32x4*>(p) = v;
    } else {
        *reinterpret_cast<u32x2*>(p) = pk_bf16x4(v);
    }
}

// ReLU on two packed bf16 values (v_pk_max_i16 against 0: a negative bf16 is a negative int16, -0 becomes
// +0): bf16(relu(x)) == relu(bf16(x)) bit for bit, so an epilogue whose output only feeds an operand
// image (no fp32 copy kept) packs first and applies the ReLU to pairs -- half the instructions
__device__ __forceinline__ unsigned relu_pk_bf16(unsigned v) {
    unsigned r;
    asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(v));
    return r;
}
__device__ __forceinline__ u32x2 relu_pk_bf16x4(const f32x4& x) {
    const u32x2 p = pk_bf16x4(x);
    return u32x2{relu_pk_bf16(p[0]), relu_pk_bf16(p[1])};
}
// write 4 packed bf16 channels of frame t of a padded operand image (pad P rows each side, reflect)
__device__ __forceinline__ void put_reflect_pk(char* img, int t, int T, int P, int chbyte, u32x2 v) {
    constexpr int RS = 288;
    *reinterpret_cast<u32x2*>(img + (P + t) * RS + chbyte) = v;
    if (t >= 1 && t <= P) *reinterpret_cast<u32x2*>(img + (P - t) * RS + chbyte) = v;
    if (t >= T - 1 - P && t <= T - 2) *reinterpret_cast<u32x2*>(img + (P + 2 * T - 2 - t) * RS + chbyte) = v;
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
// RD slots: 4 by default; 2 where a step already carries many MFMAs (the bank backward's
// 5-tile x 9-fragment steps: 720 MFMA cycles per step cover an L2 round trip with one
// spare slot, and the 4-slot ring's 80 extra VGPRs made the compiler collapse the ring into
// load -> wait -> use on every step)
template <int MTR, int RD = 4>
struct ARing {
    static_assert(RD == 2 || RD == 4 || RD == 8, "ring depth");
    f32x4 a[RD][MTR];
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
template <int MTR, int RD>
__device__ __forceinline__ void ring_fill(ARing<MTR, RD>& R, const AOp& A) {
#pragma unroll
    for (int u = 0; u < RD; ++u) ring_load<MTR>(R.a[u], A, A, u);
}

// acc[MT][NF] += A x B; the ring holds A's steps 0..RD-1 on entry and N's steps 0..RD-1 on exit.
//   B  : LDS base of the operand image; rb[f] = row of tap 0 for this lane's column
//   DJ : +1 forward (row = rb + j), -1 adjoint (row = rb - j)
// B fragments are read one step ahead into two alternating register sets.  The loop
// body has no early exits and issues every load unconditionally (steps past the end
// are clamped), so accumulators keep their registers across the back edge and the
// waitcnt pass sees a fixed number of loads in flight.
// NFC > 0: the live fragment count is the compile-time NFC (straight-line K loop);
// NFC == 0: up to NF fragments, the first `nf` live (runtime guards; generic shapes).
template <int PREC, int MT, int MTR, int RD, int NF, int NFC, int CINB, int DJ>
__device__ __forceinline__ void fz_gemm_impl(f32x4 (&acc)[MT][NF], int nf, ARing<MTR, RD>& R, const AOp& A,
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
    const int nfull = ns & ~(RD - 1);
    // slot u of an iteration: B of step s+u+1 into the idle buffer, MFMAs of step s+u, then the
    // slot refilled with step s+u+RD
#pragma unroll 1
    for (int s = 0; s < nfull; s += RD) {
#pragma unroll
        for (int u = 0; u < RD; ++u) {
            if (u & 1) {
                read_b(bA, s + u + 1);
                mma_all(R.a[u], bB);
            } else {
                read_b(bB, s + u + 1);
                mma_all(R.a[u], bA);
            }
            ring_load<MTR>(R.a[u], A, N, s + RD + u);
#if !(AVC_FZ_ABLATE & 8) && !defined(AVC_FZ_RING_FREE)
            // keep each refill in its own step: left alone, the scheduler sinks all RD refills to
            // the end of the iteration (the loaded registers are consumed a whole iteration
            // later, so the refills look like the least critical work), and the first MFMAs of
            // the next iteration then wait for an L2 round trip -- the ring's prefetch collapses
            // (AVC_FZ_RING_FREE: the long engine, whose chunked GEMMs measured 3 % faster without)
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
    }
    // remainder (0..RD-1 steps): slots hold steps nfull..nfull+RD-1 (slot u = step nfull+u),
    // bA holds step nfull.  Afterwards rotate so that slot u = N's step u again.
    const int rem = ns - nfull;
#if AVC_FZ_ABLATE & 4
    // debug: no cross-GEMM prefetch -- finish this GEMM's own steps, then load N afresh
#pragma unroll
    for (int u = 0; u < RD - 1; ++u)
        if (u < rem) {
            if (u & 1) read_b(bB, nfull + u);
            else if (u) read_b(bA, nfull + u);
            mma_all(R.a[u], (u & 1) ? bB : bA);
        }
    ring_fill(R, N);
    return;
#endif
    if (rem == 0) return;
#pragma unroll
    for (int u = 0; u < RD - 1; ++u)
        if (u < rem) {
            if (u & 1) read_b(bB, nfull + u);
            else if (u) read_b(bA, nfull + u);
            mma_all(R.a[u], (u & 1) ? bB : bA);
            ring_load<MTR>(R.a[u], A, N, nfull + RD + u);
        }
    // a GEMM shorter than the ring (ns < RD) entered with slots u >= ns holding clamped
    // copies of its own last step (its predecessor could not know this GEMM's successor):
    // those slots get N's steps u - rem now
    if (nfull == 0)
#pragma unroll
        for (int u = 0; u < RD; ++u)
            if (u >= rem) ring_load<MTR>(R.a[u], N, N, u - rem);
    // slot u now holds step nfull + u + RD*(u < rem) of the A|N stream, i.e. N's step
    // (u - rem) mod RD: rotate left by rem (rem is a compile-time constant wherever the
    // shape is, and the selects fold away)
    f32x4 t[RD][MTR];
#pragma unroll
    for (int u = 0; u < RD; ++u)
#pragma unroll
        for (int i = 0; i < MTR; ++i) t[u][i] = R.a[u][i];
#pragma unroll
    for (int u = 0; u < RD; ++u)
#pragma unroll
        for (int i = 0; i < MTR; ++i) {
            f32x4 v = t[(u + 1) % RD][i];
#pragma unroll
            for (int r = 2; r < RD; ++r)
                if (rem == r) v = t[(u + r) % RD][i];
            R.a[u][i] = v;
        }
}

// A GEMM whose whole A operand (NS K steps x MT tiles, identity step map) sits in registers
// before it starts: loaded by res_load one GEMM ahead, so a short GEMM (the bank backward's
// in_conv^T: 4 bf16 steps) never waits on L2 and needs no slot of the wide ring.
template <int NS, int MT>
struct ARes {
    f32x4 a[NS][MT];
};
template <int NS, int MT>
__device__ __forceinline__ void res_load(ARes<NS, MT>& R, const AOp& A) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < MT; ++i)
            R.a[s][i] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
                (const __attribute__((address_space(1))) f32x4*)(A.p + (size_t)s * 64 + (size_t)i * A.amt));
}
template <int PREC, int MT, int NF, int NS, int CINB, int DJ, int NFC>
__device__ __forceinline__ void fz_gemm_res(f32x4 (&acc)[MT][NF], IC<NFC>, const ARes<NS, MT>& R, const char* B,
                                            const int (&rb)[NF]) {
    using E = typename Fz<PREC>::E;
    constexpr int RS = Fz<PREC>::RS;
    constexpr int VE = 16 / (int)sizeof(E);
    constexpr int KS = 4 * VE;
    const int kq = (threadIdx.x & 63) >> 4;
    auto read_b = [&](f32x4 (&bs)[NFC], int s) __attribute__((always_inline)) {
        const int kl = KS * s + VE * kq;
        const int j = kl / CINB, ci = kl - j * CINB;
        const char* Bs = B + ci * (int)sizeof(E) + DJ * j * RS;
#pragma unroll
        for (int f = 0; f < NFC; ++f) bs[f] = lds16(Bs + rb[f] * RS);
    };
    f32x4 b[2][NFC];
    read_b(b[0], 0);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s + 1 < NS) read_b(b[(s + 1) & 1], s + 1);   // next step's B ahead of this step's MFMAs
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int f = 0; f < NFC; ++f) mma<PREC>(acc[i][f], R.a[s][i], b[s & 1][f]);
    }
}

// Diagnostic build only (-DAVC_FZ_PHASES): per-wave cycle stamps at phase boundaries,
// printed by workgroup 0 at the end of the kernel (scripts/dbg/phases.sh).
#ifdef AVC_FZ_PHASES
#ifndef FZ_PH_MAX
#define FZ_PH_MAX 96
#endif
#define FZ_PH_DECL          \
    unsigned long long fz_ph[FZ_PH_MAX]; \
    int fz_phn = 0;
#define FZ_PH()                                                            \
    do {                                                                   \
        if (fz_phn < FZ_PH_MAX) fz_ph[fz_phn++] = __builtin_readcyclecounter();   \
    } while (0)
#define FZ_PH_DUMP(tag)                                                                            \
    do {                                                                                           \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)                                            \
            for (int i_ = 1; i_ < fz_phn; ++i_)                                                    \
                printf("%s w%d %d %llu\n", tag, (int)(threadIdx.x >> 6), i_, fz_ph[i_] - fz_ph[i_ - 1]); \
    } while (0)
#else
#define FZ_PH_DECL
#define FZ_PH() \
    do {        \
    } while (0)
#define FZ_PH_DUMP(tag) \
    do {                \
    } while (0)
#endif


// fz_gemm: the fragment count is either a compile-time IC<N> (specialised shapes) or a
// runtime int (generic shapes)
template <int PREC, int MT, int NF, int CINB, int DJ, int MTR, int RD, int NFC>
__device__ __forceinline__ void fz_gemm(f32x4 (&acc)[MT][NF], IC<NFC>, ARing<MTR, RD>& R, const AOp& A, const AOp& N,
                                        const char* B, const int (&rb)[NF]) {
    static_assert(NFC >= 1 && NFC <= NF, "fragment count");
    fz_gemm_impl<PREC, MT, MTR, RD, NF, NFC, CINB, DJ>(acc, NFC, R, A, N, B, rb);
}
template <int PREC, int MT, int NF, int CINB, int DJ, int MTR, int RD>
__device__ __forceinline__ void fz_gemm(f32x4 (&acc)[MT][NF], int nf, ARing<MTR, RD>& R, const AOp& A, const AOp& N,
                                        const char* B, const int (&rb)[NF]) {
    fz_gemm_impl<PREC, MT, MTR, RD, NF, 0, CINB, DJ>(acc, nf, R, A, N, B, rb);
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
// register indexing).  The scratch is the wave's own, so the hand-off needs no workgroup
// barrier (a wave's LDS accesses execute in order); BAR = true keeps one for callers that
// use it to free other LDS (every wave must then call it at the same point).
template <bool BAR = true, int MT, int NF>
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
    if constexpr (BAR) __syncthreads();
    else asm volatile("" ::: "memory");
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

// Sum over the 16 lanes of each row (lane group) of a wave, every lane receiving the
// result, on DPP moves (no LDS round trip): rotate by 8 and 4 inside the row, then the
// quad permutations lane^2 and lane^1.  Each step adds (own + partner) == (partner + own),
// so all 16 lanes hold bitwise the same sum.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_mov<0x128>(v);   // row_ror:8
    v += dpp_mov<0x124>(v);   // row_ror:4
    v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
    return v;
}
__device__ __forceinline__ void row16_sum(f32x4& v) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = row16_sum(v[r]);
}

// InstanceNorm1d (affine=False, eps 1e-5; models.py:176,396) of the rows this wave owns:
// row (i, r) of v is one channel over the frames t = 16f + c < T (lanes of a 16-lane
// group x fragments).  Two-pass mean / biased variance like ATen's batch_norm_cpu
// statistics; v <- (v - mean) * invstd.  invstd[i][r] returned for the backward.
template <int MT, int NF>
__device__ __forceinline__ void inorm_rows(f32x4 (&v)[MT][NF], int nf, int T, f32x4 (&invstd)[MT]) {
    const int c = threadIdx.x & 15;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int f = 0; f < NF; ++f)
            if (f < nf && 16 * f + c < T) s += v[i][f];
        row16_sum(s);
        f32x4 mean;
#pragma unroll
        for (int r = 0; r < 4; ++r) mean[r] = s[r] / (float)T;
        f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int f = 0; f < NF; ++f)
            if (f < nf && 16 * f + c < T) {
                const f32x4 d = v[i][f] - mean;
                q += d * d;
            }
        row16_sum(q);
#pragma unroll
        for (int r = 0; r < 4; ++r) invstd[i][r] = 1.f / sqrtf(q[r] / (float)T + 1e-5f);
#pragma unroll
        for (int f = 0; f < NF; ++f) v[i][f] = (v[i][f] - mean) * invstd[i];
    }
}

// ReLU' masks of one layer for this wave, per lane: bit 4f + r of word i is
// (y[i][f][r] > 0) for this lane's element (tile i, fragment f < 8, row r).  Built with
// lane-local ops only and stored as one u64 per lane (lo = tile 0, hi = tile 1): a
// coalesced 512-B row per (layer, wave); the backward reads its own lane's word back.
struct MaskAcc {
    unsigned lo = 0, hi = 0;
    // bit = (y > 0) in VALU only: a float is > 0 exactly when its bit pattern is a positive
    // int, so med3(bits, 0, 1) is the bit (a compare would park one SGPR pair per element:
    // 64 live lane masks per epilogue spilled through v_writelane / v_readlane)
    __device__ __forceinline__ void put(int i, int f, int r, float y) {
        if (AVC_FZ_ABLATE & 2) return;
        // (inline asm: otherwise LLVM proves the bit equal to the act's own compare and
        // re-materialises exactly that SGPR-pair compare)
        unsigned bit;
        asm("v_med3_i32 %0, %1, 0, 1" : "=v"(bit) : "v"(y));
        // one v_lshl_or_b32 per bit: LLVM otherwise emits a shift per bit plus a v_or3 per two (1.5 VALU
        // per bit; an epilogue sets 64) -- measured 0.1782 -> 0.1766 ms per emb iteration (A/B, round 5)
        if (i == 0) asm("v_lshl_or_b32 %0, %1, %2, %0" : "+v"(lo) : "v"(bit), "i"(4 * f + r));
        else asm("v_lshl_or_b32 %0, %1, %2, %0" : "+v"(hi) : "v"(bit), "i"(4 * f + r));
    }
    __device__ __forceinline__ void store(u64* base) const {
        base[threadIdx.x & 63] = ((u64)hi << 32) | lo;
    }
};

// The same words read back for a backward pass: one coalesced load per (layer, wave),
// issued ahead of the GEMM that precedes their use.
struct MaskRd {
    unsigned lo = 0, hi = 0;
    // The scheduling barrier keeps the load where it is written (ahead of the GEMM that
    // precedes the words' use): the scheduler otherwise sank it to just before the use, where
    // its wait (vmcnt(0): the youngest load) also drained the GEMM's whole weight prefetch ring
    // -- measured 7-9k cycles per bank kernel in the backward's bank phase.
    __device__ __forceinline__ void load(const u64* base) {
        const u64 v = base[threadIdx.x & 63];
        lo = (unsigned)v;
        hi = (unsigned)(v >> 32);
        __builtin_amdgcn_sched_barrier(0);
    }
    // act'(y) of element (i, f, r): 1 where y > 0, else 0 (ReLU) or 0.01 (LeakyReLU)
    __device__ __forceinline__ float act(int i, int f, int r, int actk) const {
        const unsigned w = i == 0 ? lo : hi;
        return ((w >> (4 * f + r)) & 1u) ? 1.f : (actk ? 0.01f : 0.f);
    }
    // g * act'(y) of element (i, f, r).  ReLU: the bit sign-extended to a lane mask ANDed
    // onto g (VALU only; a select would park one SGPR-pair compare per element); the result
    // differs from g * 0 only in the sign of a zero.  LeakyReLU: g or 0.01 g.
    __device__ __forceinline__ float gate(int i, int f, int r, float g, int actk) const {
        const unsigned w = i == 0 ? lo : hi;
        if (actk) return ((w >> (4 * f + r)) & 1u) ? g : 0.01f * g;
        int m;
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(w), "s"(4 * f + r));
        return __builtin_bit_cast(float, __builtin_bit_cast(int, g) & m);
    }
};

// tanh for the bf16 mode's Adam tail (attack_utils.py:77-78,86: eps * tanh(ptb)) on the
// hardware exp2 / reciprocal instead of the libm sequence (the tail was VALU-bound on it:
// 2 tanh + sqrt + 2 IEEE divisions per element at one wave per SIMD).  |x| < 0.625: odd
// polynomial x + x^3 P(x^2) (least-squares fit in relative error, <= 0.9 ulp in f32);
// otherwise 1 - 2 / (1 + e^{2|x|}) (<= 2 ulp).  The fp32 mode keeps tanhf / sqrtf / IEEE
// division (torch's arithmetic).  Parity: tests/test_gpu_*.py tolerances.
// (every rounding step written out: no contraction left to the compiler)
__device__ __forceinline__ float fast_tanh(float x) {
#pragma clang fp contract(off)
    const float a = __builtin_fabsf(x);
    const float x2 = x * x;
    float p = -0.005691935773938894f;
    p = __builtin_fmaf(p, x2, 0.02062624879181385f);
    p = __builtin_fmaf(p, x2, -0.05373530462384224f);
    p = __builtin_fmaf(p, x2, 0.13331380486488342f);
    p = __builtin_fmaf(p, x2, -0.3333328068256378f);
    const float small = __builtin_fmaf(x * x2, p, x);
    const float e = __builtin_amdgcn_exp2f(a * 2.8853900817779268f);   // 2 log2(e)
    const float big = __builtin_copysignf(__builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + e), 1.f), x);
    return a < 0.625f ? small : big;
}
// One element of the Adam tail (attack_utils.py:78-86, torch _single_tensor_adam): tanh'
// of the reparameterisation, Adam moments and step, next adv = vc + eps*tanh(ptb).  One
// definition for every engine, with the contraction pinned, so the fused and long engines
// round identically (the compiler otherwise contracts vector and scalar copies differently).
//   fp32 mode: torch's per-operation IEEE arithmetic (tanhf, sqrt(v) / sqrt(bc2) + eps, m / den)
//   bf16 mode: hardware exp2 / rcp / sqrt and explicit fmas (the tail is VALU-bound)
struct AdamStep {
    float nstep, bc2s, rbc2s, eps;
    float pgd;           // > 0: the opt-in sign-gradient update with this step (avc_attack_opts.update)
};
// the attack input of a perturbation state p (attack_utils.py:78): vc + eps * tanh(p) -- a multiply, then an
// add, as the reference evaluates it -- or vc + p for the opt-in PGD update
template <int PREC>
__device__ __forceinline__ float adv_of(float x, float p, float eps, bool pgd) {
#pragma clang fp contract(off)
    if (pgd) return x + p;
    if constexpr (PREC == PREC_F32) return x + eps * tanhf(p);
    else return __builtin_fmaf(eps, fast_tanh(p), x);
}

template <int PREC>
__device__ __forceinline__ void adam_elem(const AdamArgs& Ad, const AdamStep& S, float gsum, float x, float& p,
                                          float& mm, float& vv, float& g, float& ad) {
#pragma clang fp contract(off)
    if (S.pgd > 0.f) {
        // PGD: ptb holds the perturbation delta itself (adv = vc + delta); delta <-
        // clamp(delta - step * sign(d loss / d delta), -eps, eps) -- north_star's "sign-grad +
        // eps-clamp" update (the reference's header optimiser clamps the same way,
        // models/header_model.py:65); not the reference's attack update (Adam + tanh)
        g = gsum;
        const float sg = gsum > 0.f ? 1.f : (gsum < 0.f ? -1.f : 0.f);
        p = fminf(fmaxf(p - S.pgd * sg, -S.eps), S.eps);
        ad = adv_of<PREC>(x, p, S.eps, true);
        return;
    }
    if constexpr (PREC == PREC_F32) {
        const float th = tanhf(p);
        g = (gsum * S.eps) * (1.f - th * th);
        mm = mm + Ad.b1c * (g - mm);
        vv = vv * Ad.b2;
        vv = vv + Ad.b2c * g * g;
        p = p + S.nstep * (mm / (sqrtf(vv) / S.bc2s + Ad.adam_eps));
        ad = adv_of<PREC>(x, p, S.eps, false);
    } else {
        const float th = fast_tanh(p);
        g = (gsum * S.eps) * __builtin_fmaf(-th, th, 1.f);
        mm = __builtin_fmaf(Ad.b1c, g - mm, mm);
        vv = __builtin_fmaf(Ad.b2c * g, g, vv * Ad.b2);
        const float den = __builtin_fmaf(__builtin_amdgcn_sqrtf(vv), S.rbc2s, Ad.adam_eps);
        p = __builtin_fmaf(S.nstep, mm * __builtin_amdgcn_rcpf(den), p);
        ad = adv_of<PREC>(x, p, S.eps, false);
    }
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


}  // namespace avc
