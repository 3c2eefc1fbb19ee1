// Long-utterance engine: the SpeakerEncoder / ContentEncoder forward, the SpeakerEncoder
// input-gradient + Adam, for ANY number of frames T (real utterances are 128-600 frames;
// the fused engine's LDS-resident images stop at T = 128).
//
// Same mapping as the fused engine (avc_fused.hip): one workgroup of 4 waves owns one
// utterance; wave w owns output channels [32w, 32w+32) of every 128-channel layer; every
// Conv1d and Conv1d input-gradient is a GEMM C[out ch][frames] = A[out ch][(tap, in ch)] x
// B on v_mfma_f32_16x16x32_bf16 (bf16) / v_mfma_f32_16x16x4_f32 (fp32), with A streamed
// from L2 through the cross-GEMM register ring (avc_fused_core.h).  What changes:
//
//  * activations live in per-utterance global scratch (LongArgs, avc_kernels.h): operand
//    images [pad rows | frames | pad rows][128 ch] (reflect-mirror rows for a forward
//    conv, zero rows for an input-gradient), and fp32 streams (the residual h, its
//    gradient) in the MFMA C/D fragment layout, so an epilogue moves one coalesced 1 KiB
//    run per wave instruction;
//  * every layer runs over chunks of 128 output columns: the chunk's input rows (+ the
//    conv halo) are staged into an LDS image with the fused engine's conflict-free row
//    stride, then the fused engine's K loop runs unchanged.  The last chunk of a layer is
//    moved back to end at the layer's last fragment (it overlaps its predecessor; columns
//    are recomputed bitwise identically and only the owning chunk accumulates sums);
//  * an input-gradient's columns are the reflect-PADDED input positions v = n - OFF, so
//    the pad positions' sums sit in the same chunk as the interior frames they fold onto
//    (models.py:23-29 adjoint, lz_fold), for any T;
//  * ReLU' masks are 64-bit ballots per 16-frame fragment (chunking-independent).
//
// Per-layer frame counts are runtime values, but every GEMM runs a compile-time number of
// fragments (8 per chunk; columns past the layer are clamped reads and dropped writes).
#ifndef LZ_ABL
#define LZ_ABL 0             // timing ablations only (wrong results): 1 = no bank-forward mask stores
#endif
#ifndef LZ_RD
#define LZ_RD 4              // weight-ring depth of the block / bank-forward GEMMs
#endif
#ifdef LZ_RING_FREE
#define AVC_FZ_RING_FREE 1   // no per-step scheduling barrier in the ring (fz_gemm_impl).  Round 6 A/B at T = 400:
                             // the pinned ring (default) is 1.6 % faster per emb iteration (1.1047 -> 1.0870 ms)
#endif
#include "avc_fused_core.h"
#include "avc_ktime.h"
AVC_KTIME_DEFINE(long)   // lz_se_fwd, lz_se_bwd, lz_dec_fwd, lz_dec_bwd per precision (avc_ktime.h)

namespace avc {

constexpr int LZ_CHF = 8;           // fragments per chunk (128 columns)
constexpr int LZ_FB = 4;            // fragments per batch of the per-frame passes (loads, then stores)
// finer stamps inside the bank phases (diagnostic builds with -DAVC_LZ_BANK_PHASES only)
#ifdef AVC_LZ_BANK_PHASES
#define FZ_PHB() FZ_PH()
#else
#define FZ_PHB() \
    do {         \
    } while (0)
#endif

template <int PREC>
struct Lz {
    using E = typename Fz<PREC>::E;
    static constexpr int ESZ = (int)sizeof(E);
    static constexpr int RS = Fz<PREC>::RS;     // LDS row stride
    static constexpr int GRB = 128 * ESZ;       // global image row bytes
};

__device__ __forceinline__ int lz_nf(int frames) { return (frames + 15) >> 4; }

// Chunk k of a layer of nfrag fragments: starts at fragment chf*k, except the last, which
// is moved back to end at nfrag.  A chunk owns the columns [16 f0, own_hi) up to the next
// chunk's start (the last one owns to the end), so every column is owned exactly once and
// a reflect-pad fold (whose sources and targets share the last / first chunk) is always
// complete in the chunk that owns its targets.  Returns false past the last chunk.
struct LzChunk {
    int f0, own_hi;
    bool last;
    __device__ __forceinline__ bool owns(int col) const { return col >= 16 * f0 && col < own_hi; }
};
__device__ __forceinline__ bool lz_chunk(int k, int nfrag, int chf, LzChunk& ch) {
    const int f = k * chf;
    if (k > 0 && f >= nfrag) return false;
    // the moved-back last chunk never starts before fragment 2: the first chunk keeps the
    // left reflect pads' targets (frames <= 4, columns <= 20) together with their sources
    const int flast = nfrag > chf ? max(nfrag - chf, 2) : 0;
    ch.last = f + chf >= nfrag;
    ch.f0 = ch.last ? flast : f;
    const int fn = f + chf;
    ch.own_hi = ch.last ? 1 << 30 : 16 * (fn + chf >= nfrag ? flast : fn);
    return true;
}

// rows [r0, r0 + n) of a global operand image -> LDS rows [0, n) (stride RS); whole
// workgroup, 16-byte pieces, U pieces per thread in flight
template <int PREC>
__device__ __forceinline__ void lz_stage(char* lds, const char* img, int r0, int n) {
    constexpr int GRB = Lz<PREC>::GRB, RS = Lz<PREC>::RS;
    constexpr int PPR = GRB / 16;
    constexpr int U = 8;
    const int tot = n * PPR;
    const char* src = img + (size_t)r0 * GRB;
    for (int base = 0; base < tot; base += 256 * U) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int idx = min(base + threadIdx.x + 256 * u, tot - 1);
            v[u] = *reinterpret_cast<const f32x4*>(src + (size_t)idx * 16);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int idx = base + threadIdx.x + 256 * u;
            if (idx < tot) {
                const int r = idx / PPR, p = idx - r * PPR;
                *reinterpret_cast<f32x4*>(lds + r * RS + p * 16) = v[u];
            }
        }
    }
}

// rows of one operand image of this workspace (fp32-sized rows serve both precisions)
template <int PREC>
__device__ __forceinline__ int lz_img_rows(const LongArgs& L) { return (int)(L.img_stride / Lz<PREC>::GRB); }
// lz_stage of rows [r0, r0 + n) clipped to the image's allocated rows (see LzPipe::rows)
template <int PREC>
__device__ __forceinline__ void lz_stage_cap(char* lds, const char* img, int r0, int n, const LongArgs& L) {
    lz_stage<PREC>(lds, img, r0, min(n, lz_img_rows<PREC>(L) - r0));
}

// rows [r0, r0 + n) of a global operand image -> LDS rows [0, n) (stride RS) by LDS-DMA
// (global_load_lds_dwordx4), NOT waited for: every wave issues NI 1-KB pieces of the padded
// LDS layout (a piece's lanes that fall on a row's pad slots or past row n load a duplicate
// that is never read).  A compile-time piece count keeps the waitcnt bookkeeping of the
// K loops that follow exact.  n <= NRMAX.
template <int PREC, int NRMAX>
struct LzDma {
    static constexpr int SPR = Lz<PREC>::RS / 16, PPR = Lz<PREC>::GRB / 16;
    static constexpr int NI = (NRMAX * SPR + 255) / 256;    // pieces per wave
    static constexpr int BUFB = NI * 256 * 16;               // LDS bytes a stage buffer spans
};
template <int PREC, int NRMAX>
__device__ __forceinline__ void lz_stage_dma(char* lds, const char* img, int r0, int n) {
    using D = LzDma<PREC, NRMAX>;
    constexpr int GRB = Lz<PREC>::GRB;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const char* src = img + (size_t)r0 * GRB;
#pragma unroll
    for (int i = 0; i < D::NI; ++i) {
        const int base = (i * 4 + w) * 64;                   // the piece's first slot (wave-uniform)
        const int q = base + lane;
        int r = q / D::SPR, p = q - r * D::SPR;
        r = r < n ? r : n - 1;
        p = p < D::PPR ? p : 0;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (size_t)r * GRB + p * 16),
                                         (__attribute__((address_space(3))) void*)(lds + (size_t)base * 16), 16, 0,
                                         0);
    }
}

// Chunk-input staging of one layer.  bf16 with every window <= NRMAX rows: two LDS buffers;
// chunk k+1's rows are issued by LDS-DMA right after chunk k's GEMM (issue_next), so the
// global round trip hides under chunk k's epilogue.  (Issued any earlier, the compiler puts
// a full vmcnt(0) before the GEMM's first LDS read -- it cannot tell the DMA's LDS target
// from the buffer being read -- and its weight-ring waits would over-wait on the DMA.)
// Otherwise the synchronous lz_stage.
template <int PREC, int NRMAX>
struct LzPipe {
    char* b0;
    int boff;                                                // second buffer at b0 + boff (0: one buffer)
    bool dma;
    int nfrag;
    int cap;                                                 // rows of an operand image (LongArgs::img_stride)
    // rows [r0, r0 + n) of the window, never past the image's last allocated row (a window is sized
    // for the longest layer; the rows past a short layer's extent are never read by an owned column)
    __device__ __forceinline__ int rows(int r0, int n) const { return min(n, cap - r0); }
    __device__ __forceinline__ LzPipe(char* WB, int nfrag_, int nr_bound, int cap_) : nfrag(nfrag_), cap(cap_) {
        dma = PREC == PREC_BF16 && nr_bound <= NRMAX;
        b0 = WB;
        boff = dma ? LzDma<PREC, NRMAX>::BUFB : 0;
    }
    template <class R0F, class NRF>
    __device__ __forceinline__ void prime(const char* img, R0F r0f, NRF nrf) {
        if (!dma) return;
        LzChunk c0;
        lz_chunk(0, nfrag, LZ_CHF, c0);
        __syncthreads();                                     // earlier readers of b0 are done
        lz_stage_dma<PREC, NRMAX>(b0, img, r0f(c0), rows(r0f(c0), nrf(c0)));
    }
    // the staged rows of chunk k (all waves may read them on return)
    template <class R0F, class NRF>
    __device__ __forceinline__ const char* next(int k, const LzChunk& chk, const char* img, R0F r0f, NRF nrf) {
        if (dma) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();                                 // chunk k landed everywhere; chunk k-1 read
            // (buffers by offset arithmetic: a select of two pointers became a scratch-indexed load)
            return b0 + (k & 1) * boff;
        }
        __syncthreads();
        lz_stage<PREC>(b0, img, r0f(chk), rows(r0f(chk), nrf(chk)));
        __syncthreads();
        return b0;
    }
    // after chunk k's last LDS read of this pass: chunk k+1's rows into the other buffer
    template <class R0F, class NRF>
    __device__ __forceinline__ void issue_next(int k, const char* img, R0F r0f, NRF nrf) {
        if (!dma) return;
        LzChunk nx;
        if (lz_chunk(k + 1, nfrag, LZ_CHF, nx))
            lz_stage_dma<PREC, NRMAX>(b0 + ((k + 1) & 1) * boff, img, r0f(nx), rows(r0f(nx), nrf(nx)));
    }
};

// x [80][T] frames u0 .. u0 + n - 1 -> LDS rows [0, n) (stride RS), transposed, frames outside
// [0, T) by the bank's reflect pad (models.py:23-29; pads <= 4, rows further out are clamped
// copies no owned column reads).  The fused engine's conflict-free mapping (lane (frame, half)
// stores every other 16-byte channel group of its frame, avc_fused.hip), and all of a
// thread's loads are issued before its first store: one HBM round trip.  n <= 256.
template <int PREC>
__device__ __forceinline__ void lz_x_window(char* XB, const float* xs, int T, int u0, int n) {
    constexpr int RS = Lz<PREC>::RS, VE = 16 / Lz<PREC>::ESZ;
    constexpr int NGX = FZ_CIN / VE, GPT = NGX / 2;
    static_assert(NGX % 2 == 0, "channel groups split over two lanes");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, xh = lane & 1;
    float xv[2][GPT][VE];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int r = 128 * p + 32 * w + (lane >> 1);
        int u = u0 + r;
        u = u < 0 ? -u : (u >= T ? 2 * T - 2 - u : u);
        u = min(max(u, 0), T - 1);
        if (r < n)
#pragma unroll
            for (int m = 0; m < GPT; ++m)
#pragma unroll
                for (int e = 0; e < VE; ++e) xv[p][m][e] = xs[(size_t)((2 * m + xh) * VE + e) * T + u];
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int r = 128 * p + 32 * w + (lane >> 1);
        if (r < n)
#pragma unroll
            for (int m = 0; m < GPT; ++m) {
                f32x4 v;
                if constexpr (PREC == PREC_F32) {
                    v = f32x4{xv[p][m][0], xv[p][m][1], xv[p][m][2], xv[p][m][3]};
                } else {
                    v = pk_bf16x8([&](int e) { return xv[p][m][e]; });
                }
                *reinterpret_cast<f32x4*>(XB + r * RS + (2 * m + xh) * 16) = v;
            }
    }
}

// zero image rows [r0, r0 + n) (whole workgroup)
template <int PREC>
__device__ __forceinline__ void lz_zero_rows(char* img, int r0, int n) {
    constexpr int GRB = Lz<PREC>::GRB;
    const int tot = n * GRB / 16;
    f32x4* p = reinterpret_cast<f32x4*>(img + (size_t)r0 * GRB);
    for (int i = threadIdx.x; i < tot; i += 256) p[i] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// wait for every vector-memory operation of this wave (s_waitcnt vmcnt(0), gfx9 encoding:
// expcnt / lgkmcnt left at their maxima).  The builtin, unlike inline asm, is seen by the
// compiler's waitcnt pass, so registers loaded before it need no further wait -- in particular
// none behind the epilogue's branchy stores, where the pass can only wait for everything
__device__ __forceinline__ void lz_vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// global stores of this workgroup visible to its other waves
__device__ __forceinline__ void lz_publish() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// this lane's f32x4 of frame t (channels 32w + 16i + 4kq .. +3) in a fragment-layout stream.
// A global-address-space pointer: the streams are picked from pointer pairs (ping-pong), and a
// generic pointer made every access a flat load / store, which waits on LDS traffic too
// (vmcnt AND lgkmcnt) -- one full round trip per fragment in the epilogues
typedef __attribute__((address_space(1))) f32x4 gf32x4;
__device__ __forceinline__ gf32x4* lz_fl(float* buf, int t, int w, int i) {
    const int kq = (threadIdx.x & 63) >> 4;
    return (gf32x4*)(buf) + ((((t >> 4) * 4 + w) * 2 + i) * 64 + ((t & 15) | (kq << 4)));
}

// The Decoder's stash of normalised activations (written by the forward, read twice by the
// backward: its dominant HBM stream at long T) in the fragment layout of lz_fl: fp32, or in bf16
// mode packed bf16 (8 bytes per lane and fragment) -- the values the fused engine stashes too
template <int PREC>
__device__ __forceinline__ void lz_stash_put(float* buf, int t, int w, int i, const f32x4& v) {
    if constexpr (PREC == PREC_F32) {
        *lz_fl(buf, t, w, i) = v;
    } else {
        const size_t k = (size_t)(lz_fl(buf, t, w, i) - (gf32x4*)buf);
        ((__attribute__((address_space(1))) u32x2*)buf)[k] = pk_bf16x4(v);
    }
}
template <int PREC>
__device__ __forceinline__ f32x4 lz_stash_get(const float* buf, int t, int w, int i) {
    if constexpr (PREC == PREC_F32) {
        return *lz_fl(const_cast<float*>(buf), t, w, i);
    } else {
        const size_t k = (size_t)(lz_fl(const_cast<float*>(buf), t, w, i) - (gf32x4*)buf);
        const u32x2 v = ((const __attribute__((address_space(1))) u32x2*)buf)[k];
        // bf16 -> f32 is exact: the bf16 bits in the high half
        return f32x4{__builtin_bit_cast(float, v[0] << 16), __builtin_bit_cast(float, v[0] & 0xffff0000u),
                     __builtin_bit_cast(float, v[1] << 16), __builtin_bit_cast(float, v[1] & 0xffff0000u)};
    }
}

// frame t of an operand image, 4 consecutive channels at byte offset chb; mirror rows of
// the reflect pad (F.pad mode="reflect", models.py:23-29) for pads up to 4
template <int PREC>
__device__ __forceinline__ void lz_put(char* img, int t, int T, int chb, f32x4 v) {
    constexpr int GRB = Lz<PREC>::GRB;
    st4<PREC>(img + (size_t)(LZ_ZR + t) * GRB + chb, v);
    if (t >= 1 && t <= 4) st4<PREC>(img + (size_t)(LZ_ZR - t) * GRB + chb, v);
    if (t >= T - 5 && t <= T - 2) st4<PREC>(img + (size_t)(LZ_ZR + 2 * T - 2 - t) * GRB + chb, v);
}

// ReLU' bits of one fragment, one byte per lane: bit 4i + r = (y[i][r] > 0), the lane's own
// elements.  Layout [layer][fragment][wave][lane] bytes per utterance (a wave's 64 bytes of a
// fragment are one coalesced access).  VALU only (med3 of the float's bits, as MaskAcc): the former 64-bit ballots
// parked one SGPR pair per element and stored through lane 0 under a branch, and were read back
// per fragment with a scalar load whose lgkmcnt(0) wait also drained the LDS queue
__device__ __forceinline__ unsigned lz_mask_bits(const f32x4 (&y)[2]) {
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            unsigned bit;
            asm("v_med3_i32 %0, %1, 0, 1" : "=v"(bit) : "v"(y[i][r]));
            m |= bit << (4 * i + r);
        }
    return m;
}
struct LzMask {
    unsigned bits;
    __device__ __forceinline__ void load(const unsigned char* p) { bits = *p; }
    __device__ __forceinline__ void none() { bits = 0; }
    __device__ __forceinline__ float act(int i, int r, int actk) const {
        return ((bits >> (4 * i + r)) & 1u) ? 1.f : (actk ? 0.01f : 0.f);
    }
};

// Reflect-pad adjoint inside a chunk of an input-gradient over padded positions
// v = n - OFF (column n = 16 (f0 + f) + c): the sum at pad position v in [-E, 0) folds onto
// frame -v, at v in [Tin, Tin + E) onto 2 (Tin - 1) - v.  Pads and targets of one side
// always share a chunk (the domain starts OFF >= E columns early and the last chunk is
// moved back).  Per-wave scratch [MT*16 rows][2E]; contains a barrier (all waves call it).
template <int MT, int NFL = LZ_CHF>
__device__ __forceinline__ void lz_fold(f32x4 (&acc)[MT][LZ_CHF], int f0, int OFF, int Tin, int E, float* scr) {
    const int lane = threadIdx.x & 63, c = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int f = 0; f < NFL; ++f) {
        const int v = 16 * (f0 + f) + c - OFF;
        const int e = v < 0 ? v + E : v - Tin + E;
        if ((v < 0 && v >= -E) || (v >= Tin && v < Tin + E)) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) scr[(16 * i + 4 * kq + r) * 8 + e] = acc[i][f][r];
        }
    }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < NFL; ++f) {
        const int t = 16 * (f0 + f) + c - OFF;
        const int el = (t >= 1 && t <= E) ? E - t : -1;
        const int er = (t >= Tin - 1 - E && t <= Tin - 2) ? E + Tin - 2 - t : -1;
        if (el >= 0 || er >= 0) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float* row = scr + (16 * i + 4 * kq + r) * 8;
                    float add = el >= 0 ? row[el] : 0.f;
                    if (er >= 0) add += row[er];
                    acc[i][f][r] += add;
                }
        }
    }
    __syncthreads();
}

// InstanceNorm statistics (affine=False, eps 1e-5, biased variance; models.py:176) of the
// rows this wave owns over the Tl frames of a fragment-layout raw stream: s = sum of the
// rows (accumulated by the GEMM epilogues over owned columns), then the centred second
// moment in a second pass.  mean / invstd per (tile, row).
__device__ __forceinline__ void lz_in_stats(const float* raw, int Tl, int w, f32x4 (&s)[2], f32x4 (&mean)[2],
                                            f32x4 (&invstd)[2]) {
    const int c = threadIdx.x & 15;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        row16_sum(s[i]);
#pragma unroll
        for (int r = 0; r < 4; ++r) mean[i][r] = s[i][r] / (float)Tl;
    }
    f32x4 q[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int nf = lz_nf(Tl);
    // LZ_FB fragments' loads in flight at a time (a runtime loop of load -> use waited a round
    // trip per fragment); the sum runs in the same fragment order
    for (int F0 = 0; F0 < nf; F0 += LZ_FB) {
        f32x4 v[LZ_FB][2];
#pragma unroll
        for (int u = 0; u < LZ_FB; ++u)
#pragma unroll
            for (int i = 0; i < 2; ++i) v[u][i] = *lz_fl(const_cast<float*>(raw), min(16 * (F0 + u) + c, Tl - 1), w, i);
#pragma unroll
        for (int u = 0; u < LZ_FB; ++u) {
            const int t = 16 * (F0 + u) + c;
            if (t < Tl)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x4 d = v[u][i] - mean[i];
                    q[i] += d * d;
                }
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        row16_sum(q[i]);
#pragma unroll
        for (int r = 0; r < 4; ++r) invstd[i][r] = 1.f / sqrtf(q[i][r] / (float)Tl + 1e-5f);
    }
}

// Running InstanceNorm statistics of a layer computed chunk by chunk from the GEMM epilogue's
// registers (the long Decoder): each chunk's owned frames give a count, a mean and a centred
// second moment (two passes over registers), merged into the running ones by Chan, Golub and
// LeVeque's pairwise update -- so no pass re-reads the raw fp32 stream for the variance (one
// HBM read of it per IN layer instead of two).  A layer of one chunk gets exactly
// lz_in_stats's arithmetic (the same sums in the same order).
struct LzMom {
    float n;
    f32x4 mean[2], m2[2];
};
template <int NF, class Own>
__device__ __forceinline__ void lz_mom_add(LzMom& M, const f32x4 (&y)[2][NF], Own own) {
    f32x4 s[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    f32x4 cnt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < NF; ++f)
        if (own(f)) {
            s[0] += y[0][f];
            s[1] += y[1][f];
            cnt[0] += 1.f;
        }
    row16_sum(s[0]);
    row16_sum(s[1]);
    const float nc = row16_sum(cnt[0]);
    if (nc == 0.f) return;
    f32x4 mc[2], q[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) mc[i][r] = s[i][r] / nc;
#pragma unroll
    for (int f = 0; f < NF; ++f)
        if (own(f))
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const f32x4 d = y[i][f] - mc[i];
                q[i] += d * d;
            }
    row16_sum(q[0]);
    row16_sum(q[1]);
    if (M.n == 0.f) {
        M.n = nc;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            M.mean[i] = mc[i];
            M.m2[i] = q[i];
        }
        return;
    }
    const float n = M.n + nc, wa = nc / n, wb = M.n * nc / n;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float d = mc[i][r] - M.mean[i][r];
            M.mean[i][r] += d * wa;
            M.m2[i][r] += q[i][r] + d * d * wb;
        }
    M.n = n;
}
// mean / invstd of the merged statistics over Tl frames (biased variance, eps 1e-5); resets M
__device__ __forceinline__ void lz_mom_get(LzMom& M, int Tl, f32x4 (&mean)[2], f32x4 (&invstd)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        mean[i] = M.mean[i];
#pragma unroll
        for (int r = 0; r < 4; ++r) invstd[i][r] = 1.f / sqrtf(M.m2[i][r] / (float)Tl + 1e-5f);
    }
    M.n = 0.f;
}

// Input length of conv block l for T frames: ceil-mode pooling halves it at every stride-2 block
// (models.py:303; the host's enc_block_lengths checks conv and pool agree).  Computed from the workgroup's
// own T (a ragged batch has one per utterance) instead of indexing A.Tl: a select between a kernarg array
// and a per-utterance global one made the compiler copy the whole FusedArgs to scratch (1.3 KB per lane).
__device__ __forceinline__ int lz_tl(const FusedArgs& A, int T, int l) {
    int t = T;
    for (int k = 0; k < l; ++k) t = A.sub[k] == 2 ? (t + 1) >> 1 : t;
    return t;
}

// ---------------------------------------------------------------------------------
// forward: SpeakerEncoder (models.py:327-343) or, in ce_mode, ContentEncoder (181-210)
// ---------------------------------------------------------------------------------
template <int PREC>
__device__ __forceinline__ void lz_se_fwd_body(FusedArgs A, LongArgs L) {
    using Z = Lz<PREC>;
    constexpr int RS = Z::RS, ESZ = Z::ESZ, GRB = Z::GRB;
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int NF = LZ_CHF;
    constexpr bool DBUF = PREC == PREC_BF16;
    const int b = blockIdx.x;
    const RagUtt* const ru = A.rag ? A.rag + b : nullptr;   // ragged batch: this utterance's own length
    const int T = ru ? ru->T : A.T, nb = A.nb, nblk = A.nblk, ks = A.ks, P = ks / 2, act = A.act;
    auto Tl = [&](int l) __attribute__((always_inline)) { return lz_tl(A, T, l); };
    const size_t xb = ru ? (size_t)ru->xoff : (size_t)b * FZ_CIN * T;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, kq = lane >> 4;
    const int ch0 = 32 * w + 4 * kq;
    const bool ce = A.ce_mode != 0;
    const bool wm = A.write_masks != 0 && !ce;
    if (A.tick && b == 0 && tid == 0) atomicAdd(A.tick, 1);
    FZ_PH_DECL
    FZ_PH();

    char* imgh = L.img[1] + (size_t)b * L.img_stride;
    char* imgy = L.img[2] + (size_t)b * L.img_stride;
    float* hf[2] = {L.fl[0] + (size_t)b * L.fl_stride, L.fl[1] + (size_t)b * L.fl_stride};
    float* raw = L.fl[2] + (size_t)b * L.fl_stride;
    unsigned char* mk = reinterpret_cast<unsigned char*>(L.masks + (size_t)b * L.mask_stride);
    auto mbyte = [&](int layer, int F) __attribute__((always_inline)) {
        return mk + ((size_t)(layer * L.nFmax + F) * 4 + w) * 64 + lane;
    };

    const int ns_c = ks * FZ_C / KS;
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
    ARing<2, LZ_RD> ring;
    ring_fill(ring, op_bank(0));

    FZ_PH();

    int rb[NF];
    f32x4 in_s[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};   // ContentEncoder: IN row sums
    // ---- conv bank (models.py:82-104) + in_conv (337-338), chunk by chunk: the bank
    // outputs of a chunk never leave LDS (in_conv consumes them block by block)
    {
        constexpr int NXR = 128 + 10;                   // x window: frames n0-4 .. n0+131 (+1)
        char* XB = fz_lds;
        char* BK0 = XB + NXR * RS;
        char* BK1 = DBUF ? BK0 + 128 * RS : BK0;
        const int nf0 = lz_nf(T);
        f32x4 b_in[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) b_in[i] = *reinterpret_cast<const f32x4*>(A.w.b_in + ch0 + 16 * i);
        LzChunk chk;
        for (int k = 0; lz_chunk(k, nf0, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            __syncthreads();                             // the previous chunk's readers are done
            lz_x_window<PREC>(XB, A.x + xb, T, n0 - 4, NXR);
            __syncthreads();
            FZ_PH();
            f32x4 acc_h[2][NF];
            zero_acc(acc_h);
            auto bank_step = [&](auto KB) __attribute__((always_inline)) {
                const int kb = KB;
                const int kk = kb + 1, pl = kk / 2;
                f32x4 bkb[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) bkb[i] = *reinterpret_cast<const f32x4*>(A.w.b_bank[kb] + ch0 + 16 * i);
                f32x4 acc[2][NF];
                zero_acc(acc);
#pragma unroll
                for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, T - 1) - n0 + 4 - pl;
                fz_gemm<PREC, 2, NF, FZ_CIN, 1>(acc, IC<NF>{}, ring, op_bank(kb), op_inb(kb), XB, rb);
                FZ_PHB();
                char* BK = (kb & 1) ? BK1 : BK0;
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    f32x4 y[2];
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int r = 0; r < 4; ++r) y[i][r] = act_f(acc[i][f][r] + bkb[i][r], act);
                    if (!(LZ_ABL & 1) && wm && chk.f0 + f < nf0 && chk.owns(16 * (chk.f0 + f)))
                        *mbyte(kb, chk.f0 + f) = (unsigned char)lz_mask_bits(y);
#pragma unroll
                    for (int i = 0; i < 2; ++i) st4<PREC>(BK + (16 * f + c) * RS + (ch0 + 16 * i) * ESZ, y[i]);
                }
                __syncthreads();
#pragma unroll
                for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, T - 1) - n0;
                const AOp nxt = kb + 1 < nb ? op_bank(kb + 1) : op_inx();
                FZ_PHB();
                fz_gemm<PREC, 2, NF, FZ_C, 1>(acc_h, IC<NF>{}, ring, op_inb(kb), nxt, BK, rb);
                if (!DBUF) __syncthreads();
                FZ_PHB();
            };
            for (int kb = 0; kb < nb; ++kb) bank_step(kb);
            FZ_PH();
#pragma unroll
            for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, T - 1) - n0 + 4;
            fz_gemm<PREC, 2, NF, FZ_CIN, 1>(acc_h, IC<NF>{}, ring, op_inx(), chk.last ? op_c1(0) : op_bank(0), XB, rb);
            FZ_PH();
            // h0 = act(in_conv + b) (SpeakerEncoder) / raw in_conv + b (ContentEncoder: IN next)
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = n0 + 16 * f + c;
                f32x4 y[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    y[i] = acc_h[i][f] + b_in[i];
                    if (!ce)
#pragma unroll
                        for (int r = 0; r < 4; ++r) y[i][r] = act_f(y[i][r], act);
                }
                if (wm && chk.f0 + f < nf0 && chk.owns(16 * (chk.f0 + f))) *mbyte(nb, chk.f0 + f) = (unsigned char)lz_mask_bits(y);
                if (t < T)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (ce) {
                            *lz_fl(raw, t, w, i) = y[i];
                            if (chk.owns(t)) in_s[i] += y[i];
                        } else {
                            *lz_fl(hf[0], t, w, i) = y[i];
                            lz_put<PREC>(imgh, t, T, (ch0 + 16 * i) * ESZ, y[i]);
                        }
                    }
            }
            FZ_PH();
        }
    }
    // ContentEncoder: h0 = act(IN(in_conv + b)) (models.py:195-200)
    // (LZ_FB fragments at a time: their loads -- raw and ex = ld(t, i), the residual or nothing --
    // then one drain, then the stores; as the decoder's in_pass)
    auto in_apply = [&](int Tl, auto&& ld, auto&& out) __attribute__((always_inline)) {
        lz_publish();
        f32x4 mean[2], inv[2];
        lz_in_stats(raw, Tl, w, in_s, mean, inv);
        for (int F0 = 0; F0 < lz_nf(Tl); F0 += LZ_FB) {
            f32x4 rv[LZ_FB][2], ex[LZ_FB][2];
#pragma unroll
            for (int u = 0; u < LZ_FB; ++u) {
                const int tc = min(16 * (F0 + u) + c, Tl - 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    rv[u][i] = *lz_fl(raw, tc, w, i);
                    ex[u][i] = ld(tc, i);
                }
            }
            lz_vm_drain();
#pragma unroll
            for (int u = 0; u < LZ_FB; ++u) {
                const int t = 16 * (F0 + u) + c;
                if (t < Tl)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        f32x4 v = (rv[u][i] - mean[i]) * inv[i];
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = act_f(v[r], act);
                        out(t, i, v, ex[u][i]);
                    }
            }
        }
        in_s[0] = in_s[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    auto no_ld = [](int, int) __attribute__((always_inline)) { return f32x4{0.f, 0.f, 0.f, 0.f}; };
    if (ce)
        in_apply(T, no_ld, [&](int t, int i, f32x4 v, f32x4) __attribute__((always_inline)) {
            *lz_fl(hf[0], t, w, i) = v;
            lz_put<PREC>(imgh, t, T, (ch0 + 16 * i) * ESZ, v);
        });

    // ---- conv blocks (models.py:285-305)
    int cur = 0;
    f32x4 tmean[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    char* WB = fz_lds;
    for (int l = 0; l < nblk; ++l) {
        const int Ti = Tl(l), To = Tl(l + 1), s = A.sub[l];
        const bool lastblk = l + 1 == nblk;
        f32x4 bc1[2], bc2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            bc1[i] = *reinterpret_cast<const f32x4*>(A.w.b_c1[l] + ch0 + 16 * i);
            bc2[i] = *reinterpret_cast<const f32x4*>(A.w.b_c2[l] + ch0 + 16 * i);
        }
        lz_publish();                                   // imgh of this block complete
        FZ_PH();
        // conv1 (stride 1): y1 = act(conv1(h) + b1)
        LzChunk chk;
        const int nfi = lz_nf(Ti);
        auto r0_c1 = [=](const LzChunk& ch) __attribute__((always_inline)) { return LZ_ZR + 16 * ch.f0 - P; };
        auto nr_c1 = [=](const LzChunk&) __attribute__((always_inline)) { return 127 + ks + 2; };
        LzPipe<PREC, 136> pipe1(WB, nfi, 127 + ks + 2, lz_img_rows<PREC>(L));
        pipe1.prime(imgh, r0_c1, nr_c1);
        for (int k = 0; lz_chunk(k, nfi, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            const char* SB = pipe1.next(k, chk, imgh, r0_c1, nr_c1);
            FZ_PH();
#pragma unroll
            for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, Ti - 1) - n0;
            f32x4 acc[2][NF];
            zero_acc(acc);
            fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, IC<NF>{}, ring, op_c1(l), chk.last ? op_c2(l) : op_c1(l), SB, rb);
            FZ_PH();
            pipe1.issue_next(k, imgh, r0_c1, nr_c1);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = n0 + 16 * f + c;
                f32x4 y[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    y[i] = acc[i][f] + bc1[i];
                    if (!ce)
#pragma unroll
                        for (int r = 0; r < 4; ++r) y[i][r] = act_f(y[i][r], act);
                }
                if (wm && chk.f0 + f < nfi && chk.owns(16 * (chk.f0 + f))) *mbyte(nb + 1 + 2 * l, chk.f0 + f) = (unsigned char)lz_mask_bits(y);
                if (t < Ti)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (ce) {
                            *lz_fl(raw, t, w, i) = y[i];
                            if (chk.owns(t)) in_s[i] += y[i];
                        } else {
                            lz_put<PREC>(imgy, t, Ti, (ch0 + 16 * i) * ESZ, y[i]);
                        }
                    }
            }
            FZ_PH();
        }
        if (ce)
            in_apply(Ti, no_ld, [&](int t, int i, f32x4 v, f32x4) __attribute__((always_inline)) {
                lz_put<PREC>(imgy, t, Ti, (ch0 + 16 * i) * ESZ, v);
            });
        lz_publish();                                   // imgy complete
        FZ_PH();
        // conv2 (stride s): y2 = act(conv2(y1) + b2); h = y2 + avg_pool1d(h, s, ceil_mode)
        float* hin = hf[cur];
        float* hout = hf[cur ^ 1];
        const int nfo = lz_nf(To);
        auto pool = [&](int t, int i) __attribute__((always_inline)) -> f32x4 {
            if (s == 1) return *lz_fl(hin, t, w, i);
            const f32x4 a = *lz_fl(hin, 2 * t, w, i);
            if (2 * t + 1 < Ti) return (a + *lz_fl(hin, 2 * t + 1, w, i)) / 2.f;
            return a;
        };
        auto r0_c2 = [=](const LzChunk& ch) __attribute__((always_inline)) { return LZ_ZR + s * 16 * ch.f0 - P; };
        auto nr_c2 = [=](const LzChunk&) __attribute__((always_inline)) { return s * 127 + ks + 2; };
        LzPipe<PREC, 264> pipe2(WB, nfo, s * 127 + ks + 2, lz_img_rows<PREC>(L));
        pipe2.prime(imgy, r0_c2, nr_c2);
        for (int k = 0; lz_chunk(k, nfo, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            const char* SB = pipe2.next(k, chk, imgy, r0_c2, nr_c2);
            FZ_PH();
#pragma unroll
            for (int f = 0; f < NF; ++f) rb[f] = s * (min(n0 + 16 * f + c, To - 1) - n0);
            f32x4 acc[2][NF];
            zero_acc(acc);
            const AOp nxt = chk.last ? (!lastblk ? op_c1(l + 1) : (ce ? op_mean() : op_c2(l))) : op_c2(l);
            fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, IC<NF>{}, ring, op_c2(l), nxt, SB, rb);
            FZ_PH();
            // the pooled residual of the whole chunk is loaded AND reduced before any of the
            // epilogue's stores and before the next chunk's DMA: a load consumed after a store (or
            // behind a branch that stores) waits for that store too (vmcnt counts both), which cost
            // a round trip per fragment
            f32x4 pv[NF][2];
            if (!ce) {
                f32x4 pb[NF][2];
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const int t = min(n0 + 16 * f + c, To - 1);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        pv[f][i] = *lz_fl(hin, s * t, w, i);
                        pb[f][i] = *lz_fl(hin, min(2 * t + 1, Ti - 1), w, i);
                    }
                }
                lz_vm_drain();
                // avg_pool1d(h, s, ceil_mode): (h[2t] + h[2t+1]) / 2, a lone tail frame as is
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const int t = n0 + 16 * f + c;
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        if (s == 2 && 2 * t + 1 < Ti) pv[f][i] = (pv[f][i] + pb[f][i]) / 2.f;
                }
            }
            pipe2.issue_next(k, imgy, r0_c2, nr_c2);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = n0 + 16 * f + c;
                f32x4 y[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    y[i] = acc[i][f] + bc2[i];
                    if (!ce)
#pragma unroll
                        for (int r = 0; r < 4; ++r) y[i][r] = act_f(y[i][r], act);
                }
                if (wm && chk.f0 + f < nfo && chk.owns(16 * (chk.f0 + f))) *mbyte(nb + 2 + 2 * l, chk.f0 + f) = (unsigned char)lz_mask_bits(y);
                if (t < To)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (ce) {
                            *lz_fl(raw, t, w, i) = y[i];
                            if (chk.owns(t)) in_s[i] += y[i];
                        } else {
                            const f32x4 h = y[i] + pv[f][i];
                            *lz_fl(hout, t, w, i) = h;
                            lz_put<PREC>(imgh, t, To, (ch0 + 16 * i) * ESZ, h);
                            if (lastblk && chk.owns(t)) tmean[i] += h;
                        }
                    }
            }
            FZ_PH();
        }
        if (ce)
            in_apply(To, pool, [&](int t, int i, f32x4 v, f32x4 pv) __attribute__((always_inline)) {
                const f32x4 h = v + pv;
                *lz_fl(hout, t, w, i) = h;
                lz_put<PREC>(imgh, t, To, (ch0 + 16 * i) * ESZ, h);
            });
        cur ^= 1;
    }
    const int TN = Tl(nblk);
    if (ce) {
        // mean_layer (1x1, models.py:207): mu = W_mean h_N + b -> [128][TN]
        lz_publish();
        f32x4 bm[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) bm[i] = *reinterpret_cast<const f32x4*>(A.w.b_mean + ch0 + 16 * i);
        float* mu = A.mu_out + (size_t)b * FZ_C * TN;
        LzChunk chk;
        const int nfn = lz_nf(TN);
        for (int k = 0; lz_chunk(k, nfn, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            __syncthreads();
            lz_stage_cap<PREC>(WB, imgh, LZ_ZR + n0, 129, L);
            __syncthreads();
#pragma unroll
            for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, TN - 1) - n0;
            f32x4 acc[2][NF];
            zero_acc(acc);
            fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, IC<NF>{}, ring, op_mean(), op_mean(), WB, rb);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = n0 + 16 * f + c;
                if (t < TN)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int r = 0; r < 4; ++r) mu[(size_t)(ch0 + 16 * i + r) * TN + t] = acc[i][f][r] + bm[i][r];
            }
        }
        return;
    }
    // AdaptiveAvgPool1d(1) (models.py:275,340): mean over the TN frames
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x4 s4 = tmean[i];
        row16_sum(s4);
        if (c == 0) {
            f32x4 m;
#pragma unroll
            for (int r = 0; r < 4; ++r) m[r] = s4[r] / (float)TN;
            *reinterpret_cast<f32x4*>(A.pooled + (size_t)b * FZ_C + ch0 + 16 * i) = m;
        }
    }
    FZ_PH();
    FZ_PH_DUMP("lfwd");
}
template <int PREC>
__global__ void __launch_bounds__(256, 1) lz_se_fwd(FusedArgs A, LongArgs L) {
    const KtStart kts = ktime_begin(&g_ktime_long[KT_LZ_SE_FWD + (PREC == PREC_BF16)]);
    lz_se_fwd_body<PREC>(A, L);
    ktime_end(&g_ktime_long[KT_LZ_SE_FWD + (PREC == PREC_BF16)], kts);
}

// ---------------------------------------------------------------------------------
// backward: d loss / d pooled -> conv blocks^T -> in_conv^T -> bank^T -> tanh' + Adam
// (attack_utils.py:78-84, torch _single_tensor_adam) or d loss / d x (gx_out)
// ---------------------------------------------------------------------------------
// Bank input-gradient chunk width: 128 columns in bf16; 64 in fp32 (its g_pre0 and g(b_k)
// LDS windows at 544 B per row would not fit beside each other at 128)
template <int PREC>
struct LzBank {
    static constexpr int CHF = PREC == PREC_BF16 ? 8 : 4;
};

template <int PREC>
__device__ __forceinline__ void lz_se_bwd_body(FusedArgs A, LongArgs L) {
    using Z = Lz<PREC>;
    using E = typename Z::E;
    constexpr int RS = Z::RS, ESZ = Z::ESZ, GRB = Z::GRB;
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int NF = LZ_CHF;
    const int b = blockIdx.x;
    const RagUtt* const ru = A.rag ? A.rag + b : nullptr;   // ragged batch: this utterance's own length
    const int T = ru ? ru->T : A.T, nb = A.nb, nblk = A.nblk, ks = A.ks, P = ks / 2, act = A.act;
    auto Tl = [&](int l) __attribute__((always_inline)) { return lz_tl(A, T, l); };
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, kq = lane >> 4;
    const int ch0 = 32 * w + 4 * kq;

    char* imgp = L.img[0] + (size_t)b * L.img_stride;   // g_pre0 (= g(h0) * act'(h0))
    char* imgg = L.img[1] + (size_t)b * L.img_stride;   // dilated dY of a conv2
    char* imgg2 = L.img[2] + (size_t)b * L.img_stride;  // dY of a conv1
    float* gh[2] = {L.fl[0] + (size_t)b * L.fl_stride, L.fl[1] + (size_t)b * L.fl_stride};
    const unsigned char* mk = reinterpret_cast<const unsigned char*>(L.masks + (size_t)b * L.mask_stride);
    auto mbyte = [&](int layer, int F) __attribute__((always_inline)) {
        return mk + ((size_t)(layer * L.nFmax + F) * 4 + w) * 64 + lane;
    };
    float* FSCR = reinterpret_cast<float*>(fz_lds + 150 * 1024) + w * (5 * 16 * 8);
    FZ_PH_DECL
    FZ_PH();

    const int ns_c = ks * FZ_C / KS;
    auto op_c1T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c1T[l], 2 * w, 2, ns_c, ns_c); };
    auto op_c2T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c2T[l], 2 * w, 2, ns_c, ns_c); };
    constexpr int SPW = 32 / KS;                        // K steps of one wave's 32-channel quarter
    constexpr int SPT = FZ_C / KS;                      // K steps per tap
    constexpr int LG = SPW == 1 ? 0 : 1;
    auto op_inTb = [&](int kb) __attribute__((always_inline)) { return aop(A.w.inT_b[kb], 2 * w, 2, SPT, SPT); };
    auto op_inTx = [&]() __attribute__((always_inline)) { return aop(A.w.inT_x, 0, 5, SPT, SPW, 30, -1, 0, w * SPW); };
    auto op_bankT = [&](int kb) __attribute__((always_inline)) {
        return aop(A.w.bankT[kb], 0, 5, (kb + 1) * SPT, (kb + 1) * SPW, LG, SPW - 1, SPT, w * SPW);
    };
    ARing<2, LZ_RD> ring;
    ring_fill(ring, op_c2T(nblk - 1));

    // g(h_N) = d loss / d pooled / TN on every frame (AdaptiveAvgPool1d backward)
    const int TN = Tl(nblk);
    f32x4 gN[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        gN[i] = *reinterpret_cast<const f32x4*>(A.g_pooled + (size_t)b * FZ_C + ch0 + 16 * i);
#pragma unroll
        for (int r = 0; r < 4; ++r) gN[i][r] = gN[i][r] / (float)TN;
    }
    // dY of the last block's conv2 = g(h_N) * act'(y2): dilated image rows LZ_ZR + s*t
    {
        const int l = nblk - 1, To = Tl(l + 1), s = A.sub[l];
        for (int F = 0; F < lz_nf(To); ++F) {
            LzMask m;
            m.load(mbyte(nb + 2 + 2 * l, F));
            const int t = 16 * F + c;
            if (t < To)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = gN[i][r] * m.act(i, r, act);
                    st4<PREC>(imgg + (size_t)(LZ_ZR + s * t) * GRB + (ch0 + 16 * i) * ESZ, v);
                    if (s == 2)
                        st4<PREC>(imgg + (size_t)(LZ_ZR + 2 * t + 1) * GRB + (ch0 + 16 * i) * ESZ,
                                  f32x4{0.f, 0.f, 0.f, 0.f});
                }
        }
    }
    int rb[NF];
    char* WB = fz_lds;
    int cur = 0;
    for (int l = nblk - 1; l >= 0; --l) {
        const int Ti = Tl(l), To = Tl(l + 1), s = A.sub[l];
        // zero rows around the dY2 image: before frame 0 and after frame s*To
        lz_zero_rows<PREC>(imgg, 0, LZ_ZR);
        lz_zero_rows<PREC>(imgg, LZ_ZR + s * To, LZ_ZR);
        lz_publish();
        FZ_PH();
        // conv2^T over padded positions v = n - 16 of the Ti input frames, * act'(y1) -> imgg2
        const int nfc = lz_nf(Ti + 16 + P);
        LzChunk chk;
        // rows of a chunk's input-gradient window: padded positions v in [vlo, vhi] + taps
        auto r0_g = [=](const LzChunk& ch) __attribute__((always_inline)) {
            return LZ_ZR + max(16 * ch.f0 - 16, -P) + P - ks - 1;
        };
        auto nr_g = [=](const LzChunk& ch) __attribute__((always_inline)) {
            return min(16 * ch.f0 + 111, Ti + P - 1) - max(16 * ch.f0 - 16, -P) + ks + 2;
        };
        LzPipe<PREC, 136> pipeg(WB, nfc, 127 + ks + 2, lz_img_rows<PREC>(L));
        pipeg.prime(imgg, r0_g, nr_g);
        for (int k = 0; lz_chunk(k, nfc, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            const int r0 = r0_g(chk);
            const char* SB = pipeg.next(k, chk, imgg, r0_g, nr_g);
            FZ_PH();
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int v = min(max(n0 + 16 * f + c - 16, -P), Ti + P - 1);
                rb[f] = LZ_ZR + v + P - r0;
            }
            f32x4 acc[2][NF];
            zero_acc(acc);
            fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, IC<NF>{}, ring, op_c2T(l), chk.last ? op_c1T(l) : op_c2T(l), SB, rb);
            FZ_PH();
            LzMask mv[NF];   // the chunk's ReLU' bytes, loaded before the epilogue's stores
#pragma unroll
            for (int f = 0; f < NF; ++f) mv[f].load(mbyte(nb + 1 + 2 * l, min(max(chk.f0 + f - 1, 0), lz_nf(Ti) - 1)));
            lz_vm_drain();
            lz_fold<2>(acc, chk.f0, 16, Ti, P, FSCR);
            pipeg.issue_next(k, imgg, r0_g, nr_g);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int F = chk.f0 + f - 1, t = 16 * F + c;   // frame of the column
                if (F < 0 || 16 * F >= Ti || !chk.owns(16 * (F + 1))) continue;
                const LzMask m = mv[f];
                if (t < Ti)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        f32x4 v;
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = acc[i][f][r] * m.act(i, r, act);
                        st4<PREC>(imgg2 + (size_t)(LZ_ZR + t) * GRB + (ch0 + 16 * i) * ESZ, v);
                    }
            }
            FZ_PH();
        }
        lz_zero_rows<PREC>(imgg2, 0, LZ_ZR);
        lz_zero_rows<PREC>(imgg2, LZ_ZR + Ti, LZ_ZR);
        lz_publish();
        FZ_PH();
        // conv1^T (+ fold) + avg_pool^T of g(h_{l+1}) -> g(h_l); then the next dY: the dilated
        // dY2 of block l-1 = g(h_l) * act'(y2_{l-1}), or g_pre0 = g(h_0) * act'(h0)
        const int sp = l > 0 ? A.sub[l - 1] : 1;
        const int mlayer = l > 0 ? nb + 2 + 2 * (l - 1) : nb;
        char* nimg = l > 0 ? imgg : imgp;
        float* gprev = gh[cur];
        float* gnew = gh[cur ^ 1];
        LzPipe<PREC, 136> pipeg2(WB, nfc, 127 + ks + 2, lz_img_rows<PREC>(L));
        pipeg2.prime(imgg2, r0_g, nr_g);
        for (int k = 0; lz_chunk(k, nfc, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            const int r0 = r0_g(chk);
            const char* SB = pipeg2.next(k, chk, imgg2, r0_g, nr_g);
            FZ_PH();
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int v = min(max(n0 + 16 * f + c - 16, -P), Ti + P - 1);
                rb[f] = LZ_ZR + v + P - r0;
            }
            f32x4 acc[2][NF];
            zero_acc(acc);
            const AOp nxt = chk.last ? (l > 0 ? op_c2T(l - 1) : op_inTx()) : op_c1T(l);
            if (chk.last && l == 0) {
                // the bank phase runs on a 5-tile ring: refill the 2-tile ring with a dummy
                fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, IC<NF>{}, ring, op_c1T(l), op_c1T(l), SB, rb);
            } else {
                fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, IC<NF>{}, ring, op_c1T(l), nxt, SB, rb);
            }
            FZ_PH();
            // g(h_{l+1}) of the chunk's frames, loaded before the epilogue's stores (see the
            // forward's conv2 epilogue)
            f32x4 gq[NF][2];
            if (l == nblk - 1) {
#pragma unroll
                for (int f = 0; f < NF; ++f)
#pragma unroll
                    for (int i = 0; i < 2; ++i) gq[f][i] = gN[i];
            } else {
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const int t = min(max(16 * (chk.f0 + f - 1) + c, 0), Ti - 1);
#pragma unroll
                    for (int i = 0; i < 2; ++i) gq[f][i] = *lz_fl(gprev, s == 2 ? t >> 1 : t, w, i);
                }
            }
            LzMask mv[NF];
#pragma unroll
            for (int f = 0; f < NF; ++f) mv[f].load(mbyte(mlayer, min(max(chk.f0 + f - 1, 0), lz_nf(Ti) - 1)));
            lz_vm_drain();
            // torch avg_pool backward: grad / divide_factor (2, or 1 for a ceil tail)
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = 16 * (chk.f0 + f - 1) + c;
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    if (s == 2 && 2 * (t >> 1) + 1 < Ti) gq[f][i] = gq[f][i] / 2.f;
            }
            lz_fold<2>(acc, chk.f0, 16, Ti, P, FSCR);
            pipeg2.issue_next(k, imgg2, r0_g, nr_g);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int F = chk.f0 + f - 1, t = 16 * F + c;
                if (F < 0 || 16 * F >= Ti || !chk.owns(16 * (F + 1))) continue;
                const LzMask m = mv[f];
                if (t < Ti)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const f32x4 g = acc[i][f] + gq[f][i];
                        if (l > 0) *lz_fl(gnew, t, w, i) = g;
                        f32x4 v;
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = g[r] * m.act(i, r, act);
                        st4<PREC>(nimg + (size_t)(LZ_ZR + sp * t) * GRB + (ch0 + 16 * i) * ESZ, v);
                        if (sp == 2)
                            st4<PREC>(nimg + (size_t)(LZ_ZR + 2 * t + 1) * GRB + (ch0 + 16 * i) * ESZ,
                                      f32x4{0.f, 0.f, 0.f, 0.f});
                    }
            }
            FZ_PH();
        }
        cur ^= 1;
    }

    // ---- in_conv^T and conv bank^T (models.py:82-104, 337-338) chunk by chunk over the
    // x-gradient's padded positions v = n - 4 (the bank's reflect pads are <= 4).  K of the
    // bank^T split over waves: wave w sums over bank channels [32w, 32w+32) of every bank
    // kernel into a partial g(x) [80][chunk]; g(b_k) for those channels is recomputed per
    // chunk over the frames the chunk needs (in_conv^T, * act'(b_k)).
    constexpr int CHF = LzBank<PREC>::CHF, CH = 16 * CHF;
    constexpr int NFW = CHF + 1;                        // g(b_k) window: frames n0-16 .. n0+CH-1
    constexpr int ZPB = 8;
    ARing<5, 2> ring5;   // 2 slots: see ARing
    ring_fill(ring5, op_inTx());
    lz_zero_rows<PREC>(imgp, 0, LZ_ZR);
    lz_zero_rows<PREC>(imgp, LZ_ZR + T, LZ_ZR);
    lz_publish();
    FZ_PH();
    char* GP = fz_lds;                                  // g_pre0 rows of frames n0-16 .. n0+CH-1
    char* GBK = GP + NFW * 16 * RS;                     // per-wave g(b_k) slices, ZPB + NFW*16 + ZPB rows
    static_assert((NFW * 16 + NFW * 16 + 2 * ZPB) * RS <= 150 * 1024, "bank windows overlap the fold scratch");
    static_assert(2 * FZ_CIN * CH * 4 <= 150 * 1024, "reduction rows overlap the fold scratch");
    float* R0 = reinterpret_cast<float*>(fz_lds);       // cross-wave partial sums (alias GP / GBK)
    float* R1 = R0 + FZ_CIN * CH;
    // column of row ci rotated by 16 (ci / 4 mod 4): the 4 lane groups (kq) of a store then hit
    // distinct banks instead of the same 16 (rows of CH floats all start on bank 0: a 4-way
    // conflict).  (Padding the rows instead made the compiler spill the accumulators.)
    auto rcol = [](int ci, int col) __attribute__((always_inline)) { return (col + 16 * ((ci >> 2) & 3)) & (CH - 1); };
    const int nfx = lz_nf(T + 8);
    const AdamArgs& Ad = A.adam;
    // gx_out mode (fb: d loss / d x handed on) has no Adam state: its AdamArgs are empty
    const bool adam = A.gx_out == nullptr;
    const float eps = adam ? A.scal[0] : 0.f;
    const int step = adam ? min(max(*A.step, 1), A.table_len) : 1;
    const float nstep = adam ? Ad.table[2 * (step - 1)] : 0.f;
    const float bc2s = adam ? Ad.table[2 * (step - 1) + 1] : 1.f;
    const float rbc2s = 1.f / bc2s;
    const AdamStep S{nstep, bc2s, rbc2s, eps, adam ? A.scal[3] : 0.f};
    const size_t xb = ru ? (size_t)ru->xoff : (size_t)b * FZ_CIN * T;
    LzChunk chk;
    for (int k = 0; lz_chunk(k, nfx, CHF, chk); ++k) {
        const int n0 = 16 * chk.f0;
        const int W0 = n0 - 16;                         // first frame of the g(b_k) window
        __syncthreads();
        lz_stage_cap<PREC>(GP, imgp, LZ_ZR + W0, NFW * 16, L);
        {   // this wave's slice of the GBK margins: zero
            constexpr int V16 = 32 * ESZ / 16;
            for (int idx = lane; idx < 2 * ZPB * V16; idx += 64) {
                const int rr = idx / V16, part = idx - rr * V16;
                const int row = rr < ZPB ? rr : NFW * 16 + rr;
                *reinterpret_cast<f32x4*>(GBK + row * RS + 32 * w * ESZ + part * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
        __syncthreads();
        FZ_PH();
        f32x4 accx[5][LZ_CHF];
        zero_acc(accx);
        // x passthrough of the cat: W_in[:, x block]^T g_pre0.  Pad columns read g_pre0 rows of
        // frames outside [0, T), which are zero rows of the image: they get nothing.
        int rbx[LZ_CHF];
#pragma unroll
        for (int f = 0; f < LZ_CHF; ++f) rbx[f] = min(max(n0 + 16 * f + c - 4, -4), T + 3) - W0;
        if constexpr (CHF == LZ_CHF) {
            fz_gemm<PREC, 5, LZ_CHF, FZ_C, 1>(accx, IC<LZ_CHF>{}, ring5, op_inTx(), op_inTb(0), GP, rbx);
        } else {
            fz_gemm<PREC, 5, LZ_CHF, FZ_C, 1>(accx, IC<CHF>{}, ring5, op_inTx(), op_inTb(0), GP, rbx);
        }
        auto bank_step = [&](auto KB) __attribute__((always_inline)) {
            const int kb = KB;
            const int kk = kb + 1, pl = kk / 2;
            // g(b_k) for this wave's 32 bank channels over the window = (W_in[:, kb]^T g_pre0) * act'(b_k)
            f32x4 acc[2][NFW];
            zero_acc(acc);
            int rt[NFW];
#pragma unroll
            for (int f = 0; f < NFW; ++f) rt[f] = 16 * f + c;
            LzMask mv[NFW];   // loaded ahead of the GEMM (they land under it)
#pragma unroll
            for (int f = 0; f < NFW; ++f) mv[f].load(mbyte(kb, min(max(W0 / 16 + f, 0), lz_nf(T) - 1)));
            fz_gemm<PREC, 2, NFW, FZ_C, 1>(acc, IC<NFW>{}, ring5, op_inTb(kb), op_bankT(kb), GP, rt);
            FZ_PHB();
#pragma unroll
            for (int f = 0; f < NFW; ++f) {
                const int F = W0 / 16 + f, u = 16 * F + c;
                LzMask m = mv[f];
                if (!(F >= 0 && 16 * F < T)) m.none();
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = (u >= 0 && u < T) ? acc[i][f][r] * m.act(i, r, act) : 0.f;
                    st4<PREC>(GBK + (ZPB + 16 * f + c) * RS + (ch0 + 16 * i) * ESZ, v);
                }
            }
            // wave-local hand-off (as in se_bwd_fused): the bank^T below reads only this wave's
            // g(b_k) channels, and GP is read-only here -- program order, no workgroup barrier
            asm volatile("" ::: "memory");
            FZ_PHB();
            // bank_k^T over this wave's channel quarter: rows u = v + pl - j of g(b_k)
#pragma unroll
            for (int f = 0; f < LZ_CHF; ++f) {
                const int v = min(max(n0 + 16 * f + c - 4, -4), T + 3);
                rb[f] = ZPB + (v + pl) - W0;
            }
            const AOp nxt = kb + 1 < nb ? op_inTb(kb + 1) : op_bankT(kb);
            if constexpr (CHF == LZ_CHF) {
                fz_gemm<PREC, 5, LZ_CHF, FZ_C, -1>(accx, IC<LZ_CHF>{}, ring5, op_bankT(kb), nxt, GBK, rb);
            } else {
                fz_gemm<PREC, 5, LZ_CHF, FZ_C, -1>(accx, IC<CHF>{}, ring5, op_bankT(kb), nxt, GBK, rb);
            }
            asm volatile("" ::: "memory");   // (the next gate rewrites this wave's slice: in order)
            FZ_PHB();
        };
        FZ_PH();
        for (int kb = 0; kb < nb; ++kb) bank_step(kb);
        FZ_PH();
        if (!chk.last) {   // ring5 now holds op_bankT(nb-1) prefetches; the next chunk starts at in_x^T
            ring_fill(ring5, op_inTx());
        }
        lz_fold<5, CHF>(accx, chk.f0, 4, T, 4, FSCR);
        FZ_PH();
        // deterministic cross-wave sum ((p0 + p2) + (p1 + p3)) into R0 / R1 [80][CH]
        for (int phase = 0; phase < 2; ++phase) {
            if ((phase == 0) == (w >= 2)) {
                float* R = (w & 1) ? R1 : R0;
#pragma unroll
                for (int i = 0; i < 5; ++i)
#pragma unroll
                    for (int f = 0; f < CHF; ++f)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            float* p = R + (16 * i + 4 * kq + r) * CH + ((16 * f + c + 16 * kq) & (CH - 1));
                            *p = phase ? accx[i][f][r] + *p : accx[i][f][r];
                        }
            }
            __syncthreads();
        }
        FZ_PH();
        // owned interior columns: t = n - 4 in [0, T), in groups of 4 consecutive frames of one mel row.  The
        // frame start n0 - 4 and the chunk's owned range are multiples of 4 (16), the utterance's offset xb a
        // multiple of 80: with T a multiple of 4 (vec) a group is entirely owned and inside [0, T) or not at
        // all, and every access is one 16-byte load / store; otherwise four 4-byte ones, each frame checked.
        // UB4 groups per thread per round, their state loads issued before any arithmetic (one round trip
        // per round; more groups per round spilled: the next chunk's ring5 prefetch is live here).  Same
        // per-element arithmetic (adam_elem) either way.  (Round 6: the former per-element 4-byte loop took
        // 31-56k cycles per 128-frame chunk at T = 400, 1.5-2x the fused engine's whole tail.)
        const bool vec = (T & 3) == 0;
        constexpr int NG = FZ_CIN * CH / 4, GPR = CH / 4, UG = (NG + 255) / 256, UB4 = 3;
        auto ld4 = [&](const float* a, size_t q) __attribute__((always_inline)) {
            if (vec) return ((const gf32x4*)(a))[q >> 2];
            const __attribute__((address_space(1))) float* g = (const __attribute__((address_space(1))) float*)(a);
            f32x4 r;
#pragma unroll
            for (int e = 0; e < 4; ++e) r[e] = g[min(q + e, xb + (size_t)FZ_CIN * T - 1)];
            return r;
        };
        auto st4g = [&](float* a, size_t q, f32x4 v, int nok) __attribute__((always_inline)) {
            if (vec) {
                ((gf32x4*)(a))[q >> 2] = v;
                return;
            }
            __attribute__((address_space(1))) float* g = (__attribute__((address_space(1))) float*)(a);
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e < nok) g[q + e] = v[e];
        };
#pragma unroll 1
        for (int u0 = 0; u0 < UG; u0 += UB4) {
            f32x4 gs4[UB4], P4[UB4], M4[UB4], V4[UB4], X4[UB4];
            size_t q4[UB4];
            int nok[UB4];      // frames of the group to update (0..4)
#pragma unroll
            for (int u = 0; u < UB4; ++u) {
                const int gi = tid + 256 * (u0 + u);
                const int ci = min(gi / GPR, FZ_CIN - 1), col = 4 * (gi - (gi / GPR) * GPR);
                const int n = n0 + col, t = n - 4;
                nok[u] = (gi < NG && chk.owns(n) && t >= 0 && t < T) ? min(4, T - t) : 0;
                q4[u] = xb + (size_t)ci * T + (size_t)min(max(t, 0), T - (vec ? 4 : 1));
                const int lo = ci * CH + rcol(ci, col);
                gs4[u] = *reinterpret_cast<const f32x4*>(R0 + lo) + *reinterpret_cast<const f32x4*>(R1 + lo);
                if (adam) {
                    P4[u] = ld4(Ad.ptb, q4[u]);
                    M4[u] = ld4(Ad.m, q4[u]);
                    V4[u] = ld4(Ad.v, q4[u]);
                    X4[u] = ld4(Ad.vc, q4[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < UB4; ++u) {
                if (nok[u] == 0) continue;
                if (!adam) {
                    st4g(A.gx_out, q4[u], gs4[u], nok[u]);
                    continue;
                }
                f32x4 p = P4[u], mm = M4[u], vv = V4[u], g, ad;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float pe = p[e], me = mm[e], ve = vv[e], ge, ae;
                    adam_elem<PREC>(Ad, S, gs4[u][e], X4[u][e], pe, me, ve, ge, ae);
                    p[e] = pe;
                    mm[e] = me;
                    vv[e] = ve;
                    g[e] = ge;
                    ad[e] = ae;
                }
                if (Ad.grad0 && step == 1) st4g(Ad.grad0, q4[u], g, nok[u]);
                st4g(Ad.ptb, q4[u], p, nok[u]);
                st4g(Ad.m, q4[u], mm, nok[u]);
                st4g(Ad.v, q4[u], vv, nok[u]);
                st4g(Ad.adv, q4[u], ad, nok[u]);
            }
        }
        FZ_PH();
    }
    FZ_PH_DUMP("lbwd");
}
template <int PREC>
__global__ void __launch_bounds__(256, 1) lz_se_bwd(FusedArgs A, LongArgs L) {
    const KtStart kts = ktime_begin(&g_ktime_long[KT_LZ_SE_BWD + (PREC == PREC_BF16)]);
    lz_se_bwd_body<PREC>(A, L);
    ktime_end(&g_ktime_long[KT_LZ_SE_BWD + (PREC == PREC_BF16)], kts);
}

// ---------------------------------------------------------------------------------
// Decoder (models.py:403-435) for any length: forward (+ e2e loss) and backward to
// d loss / d [mean | std] of every AdaIN (dec_fwd_fused / dec_bwd_fused in avc_vc.hip for
// the T <= 128 engine).  InstanceNorm statistics span all chunks: a layer's GEMM writes its
// raw output (+ bias) as an fp32 fragment-layout stream and accumulates the row sums over
// the columns each chunk owns; a second pass takes the centred second moment, a third
// normalises (AdaIN, act, residual) into the next operand image.  A x2 pixel-shuffle conv
// runs as two half-GEMMs over the even / odd output channels of one staged window: half s
// of channel c is frame 2t + s of the shuffled output (models.py:33-49).
// LongArgs: img[0] block input (h), img[1] conv1 output / dY images, img[2] second dY image,
// fl[0], fl[1] residual stream / its gradient (ping-pong), fl[2] raw / temporary gradients.
// The forward stashes each InstanceNorm's normalised output (fp32, fragment layout over
// the layer's frames, at stash + stash_off[q]) and 1/std for the backward.
// ---------------------------------------------------------------------------------

// [C][T] fp32 (a [B][C][T] tensor's utterance) -> image rows LZ_ZR + t, channels [0, C)
template <int PREC, int C>
__device__ __forceinline__ void lz_ct_to_img(char* img, const float* src, int T) {
    using Z = Lz<PREC>;
    constexpr int VE = 16 / Z::ESZ, NG = C / VE;
    constexpr int U = 4;   // slots per thread in flight: their loads, one drain, then the stores
    const int n = NG * T;
    for (int base = threadIdx.x; base < n; base += 256 * U) {
        float x[U][VE];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int idx = min(base + 256 * u, n - 1);
            const int g = idx / T, t = idx - g * T;
#pragma unroll
            for (int e = 0; e < VE; ++e) x[u][e] = src[(size_t)(VE * g + e) * T + t];
        }
        lz_vm_drain();
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int idx = base + 256 * u;
            if (idx >= n) continue;
            const int g = idx / T, t = idx - g * T;
            f32x4 v;
            if constexpr (PREC == PREC_F32) {
                v = f32x4{x[u][0], x[u][1], x[u][2], x[u][3]};
            } else {
                v = pk_bf16x8([&](int e) { return x[u][e]; });
            }
            *reinterpret_cast<f32x4*>(img + (size_t)(LZ_ZR + t) * Z::GRB + 16 * g) = v;
        }
    }
}

template <int PREC>
__device__ __forceinline__ void lz_dec_fwd_body(DecArgs A, LongArgs L) {
    using Z = Lz<PREC>;
    constexpr int RS = Z::RS, ESZ = Z::ESZ;
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int NF = LZ_CHF;
    const int b = blockIdx.x;
    const int nblk = A.nblk, ks = A.ks, P = ks / 2, act = A.act;
    const int T0 = A.Tl[0], Tn = A.Tl[nblk];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, kq = lane >> 4;
    const int ch0 = 32 * w + 4 * kq;
    const float* cond = A.cond + (size_t)b * (2 * nblk) * 256;
    const bool stash = A.stash_per_utt > 0;
    float* stb = A.stash + (size_t)b * A.stash_per_utt;

    char* imgh = L.img[0] + (size_t)b * L.img_stride;
    char* imgy = L.img[1] + (size_t)b * L.img_stride;
    float* hf[2] = {L.fl[0] + (size_t)b * L.fl_stride, L.fl[1] + (size_t)b * L.fl_stride};
    float* raw = L.fl[2] + (size_t)b * L.fl_stride;

    const int ns_c = ks * FZ_C / KS;
    const int ns_1 = FZ_C / KS;
    auto op_in = [&]() __attribute__((always_inline)) { return aop(A.w.in, 2 * w, 2, ns_1, ns_1); };
    auto op_c1 = [&](int l) __attribute__((always_inline)) { return aop(A.w.c1[l], 2 * w, 2, ns_c, ns_c); };
    auto op_c2 = [&](int l, int s) __attribute__((always_inline)) { return aop(A.w.c2[l][s], 2 * w, 2, ns_c, ns_c); };
    // out_conv: 80 rows = 5 tiles; waves take tiles {0,1}, {2,3}, {3,4}, {3,4}
    auto op_out = [&]() __attribute__((always_inline)) { return aop(A.w.out, w < 2 ? 2 * w : 3, 2, ns_1, ns_1); };
    ARing<2> ring;
    ring_fill(ring, op_in());
    int rb[NF];
    char* WB = fz_lds;
    LzMom mom;
    mom.n = 0.f;

    lz_ct_to_img<PREC, FZ_C>(imgy, A.mu + (size_t)b * FZ_C * T0, T0);   // mu -> in_conv operand
    lz_publish();
    // in_conv (1x1) + b -> raw
    {
        f32x4 bi[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) bi[i] = *reinterpret_cast<const f32x4*>(A.w.b_in + ch0 + 16 * i);
        LzChunk chk;
        for (int k = 0; lz_chunk(k, lz_nf(T0), NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            __syncthreads();
            lz_stage_cap<PREC>(WB, imgy, LZ_ZR + n0, 129, L);
            __syncthreads();
#pragma unroll
            for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, T0 - 1) - n0;
            f32x4 acc[2][NF];
            zero_acc(acc);
            fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, IC<NF>{}, ring, op_in(), chk.last ? op_c1(0) : op_in(), WB, rb);
            auto own = [&](int f) __attribute__((always_inline)) {
                const int t = n0 + 16 * f + c;
                return t < T0 && chk.owns(t);
            };
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i][f] += bi[i];
#pragma unroll
            for (int f = 0; f < NF; ++f)
                if (own(f))
#pragma unroll
                    for (int i = 0; i < 2; ++i) *lz_fl(raw, n0 + 16 * f + c, w, i) = acc[i][f];
            lz_mom_add(mom, acc, own);
        }
    }
    // InstanceNorm over the Tl frames of raw, then out(t, i, yhat, invstd, ex) with ex = ld(t, i)
    // (the residual, or nothing).  LZ_FB fragments at a time: all their loads, one drain, then the
    // stores (a load consumed behind a store waits for the store: a round trip per fragment)
    auto in_pass = [&](int Tl, auto&& ld, auto&& out) __attribute__((always_inline)) {
        lz_publish();
        f32x4 mean[2], inv[2];
        lz_mom_get(mom, Tl, mean, inv);
        for (int F0 = 0; F0 < lz_nf(Tl); F0 += LZ_FB) {
            f32x4 v[LZ_FB][2], ex[LZ_FB][2];
#pragma unroll
            for (int u = 0; u < LZ_FB; ++u) {
                const int tc = min(16 * (F0 + u) + c, Tl - 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    v[u][i] = *lz_fl(raw, tc, w, i);
                    ex[u][i] = ld(tc, i);
                }
            }
            lz_vm_drain();
#pragma unroll
            for (int u = 0; u < LZ_FB; ++u) {
                const int t = 16 * (F0 + u) + c;
                if (t < Tl)
#pragma unroll
                    for (int i = 0; i < 2; ++i) out(t, i, (v[u][i] - mean[i]) * inv[i], inv[i], ex[u][i]);
            }
        }
    };
    auto no_ld = [](int, int) __attribute__((always_inline)) { return f32x4{0.f, 0.f, 0.f, 0.f}; };
    auto put_inv = [&](int q, const f32x4& inv, int i) __attribute__((always_inline)) {
        if (stash && c == 0)
            *reinterpret_cast<f32x4*>(A.invstd + ((size_t)b * 2 * nblk + q) * 128 + ch0 + 16 * i) = inv;
    };
    in_pass(T0, no_ld, [&](int t, int i, f32x4 v, f32x4, f32x4) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_f(v[r], act);
        *lz_fl(hf[0], t, w, i) = v;
        lz_put<PREC>(imgh, t, T0, (ch0 + 16 * i) * ESZ, v);
    });

    int cur = 0;
    for (int l = 0; l < nblk; ++l) {
        const int Ti = A.Tl[l], up = A.up[l], To = Ti * up;
        f32x4 b1[2], b2[2][2], mn1[2], sd1[2], mn2[2], sd2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            b1[i] = *reinterpret_cast<const f32x4*>(A.w.b_c1[l] + ch0 + 16 * i);
            b2[0][i] = *reinterpret_cast<const f32x4*>(A.w.b_c2[l][0] + ch0 + 16 * i);
            b2[1][i] = *reinterpret_cast<const f32x4*>(A.w.b_c2[l][1] + ch0 + 16 * i);
            mn1[i] = *reinterpret_cast<const f32x4*>(cond + (2 * l) * 256 + ch0 + 16 * i);
            sd1[i] = *reinterpret_cast<const f32x4*>(cond + (2 * l) * 256 + 128 + ch0 + 16 * i);
            mn2[i] = *reinterpret_cast<const f32x4*>(cond + (2 * l + 1) * 256 + ch0 + 16 * i);
            sd2[i] = *reinterpret_cast<const f32x4*>(cond + (2 * l + 1) * 256 + 128 + ch0 + 16 * i);
        }
        lz_publish();
        // conv1 -> raw -> IN -> AdaIN(2l) -> act -> imgy
        LzChunk chk;
        const int nfi = lz_nf(Ti);
        // chunk windows staged by LDS-DMA one chunk ahead (LzPipe, as the SpeakerEncoder blocks)
        auto r0_w = [=](const LzChunk& ch) __attribute__((always_inline)) { return LZ_ZR + 16 * ch.f0 - P; };
        auto nr_w = [=](const LzChunk&) __attribute__((always_inline)) { return 127 + ks + 2; };
        LzPipe<PREC, 136> pipe1(WB, nfi, 127 + ks + 2, lz_img_rows<PREC>(L));
        pipe1.prime(imgh, r0_w, nr_w);
        for (int k = 0; lz_chunk(k, nfi, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            const char* SB = pipe1.next(k, chk, imgh, r0_w, nr_w);
#pragma unroll
            for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, Ti - 1) - n0;
            f32x4 acc[2][NF];
            zero_acc(acc);
            fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, IC<NF>{}, ring, op_c1(l), chk.last ? op_c2(l, 0) : op_c1(l), SB, rb);
            pipe1.issue_next(k, imgh, r0_w, nr_w);
            auto own = [&](int f) __attribute__((always_inline)) {
                const int t = n0 + 16 * f + c;
                return t < Ti && chk.owns(t);
            };
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int i = 0; i < 2; ++i) acc[i][f] += b1[i];
#pragma unroll
            for (int f = 0; f < NF; ++f)
                if (own(f))
#pragma unroll
                    for (int i = 0; i < 2; ++i) *lz_fl(raw, n0 + 16 * f + c, w, i) = acc[i][f];
            lz_mom_add(mom, acc, own);
        }
        float* st1 = stb + A.stash_off[2 * l];
        in_pass(Ti, no_ld, [&](int t, int i, f32x4 yh, f32x4 inv, f32x4) __attribute__((always_inline)) {
            if (stash) lz_stash_put<PREC>(st1, t, w, i, yh);
            if (t == c) put_inv(2 * l, inv, i);
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = act_f(yh[r] * sd1[i][r] + mn1[i][r], act);
            lz_put<PREC>(imgy, t, Ti, (ch0 + 16 * i) * ESZ, v);
        });
        lz_publish();
        // conv2 (up = 1: one GEMM; up = 2: the even / odd half-GEMMs) -> raw over To frames
        const AOp nxt = l + 1 < nblk ? op_c1(l + 1) : op_out();
        LzPipe<PREC, 136> pipe2(WB, nfi, 127 + ks + 2, lz_img_rows<PREC>(L));
        pipe2.prime(imgy, r0_w, nr_w);
        for (int k = 0; lz_chunk(k, nfi, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            const char* SB = pipe2.next(k, chk, imgy, r0_w, nr_w);
#pragma unroll
            for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, Ti - 1) - n0;
            for (int s = 0; s < up; ++s) {
                f32x4 acc[2][NF];
                zero_acc(acc);
                const AOp nx = s + 1 < up ? op_c2(l, 1) : (chk.last ? nxt : op_c2(l, 0));
                fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, IC<NF>{}, ring, op_c2(l, s), nx, SB, rb);
                if (s + 1 == up) pipe2.issue_next(k, imgy, r0_w, nr_w);
                auto own = [&](int f) __attribute__((always_inline)) {
                    const int t = n0 + 16 * f + c;
                    return t < Ti && chk.owns(t);
                };
#pragma unroll
                for (int f = 0; f < NF; ++f)
#pragma unroll
                    for (int i = 0; i < 2; ++i) acc[i][f] += b2[s][i];
#pragma unroll
                for (int f = 0; f < NF; ++f)
                    if (own(f))
#pragma unroll
                        for (int i = 0; i < 2; ++i) *lz_fl(raw, up * (n0 + 16 * f + c) + s, w, i) = acc[i][f];
                lz_mom_add(mom, acc, own);
            }
        }
        float* st2 = stb + A.stash_off[2 * l + 1];
        float* hin = hf[cur];
        float* hout = hf[cur ^ 1];
        // IN over the To frames -> AdaIN(2l+1) -> act -> + (nearest-upsampled) residual
        in_pass(To, [&](int t, int i) __attribute__((always_inline)) { return f32x4(*lz_fl(hin, up == 2 ? t >> 1 : t, w, i)); },
                [&](int t, int i, f32x4 yh, f32x4 inv, f32x4 res) __attribute__((always_inline)) {
            if (stash) lz_stash_put<PREC>(st2, t, w, i, yh);
            if (t == c) put_inv(2 * l + 1, inv, i);
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = act_f(yh[r] * sd2[i][r] + mn2[i][r], act);
            const f32x4 h = v + res;
            *lz_fl(hout, t, w, i) = h;
            lz_put<PREC>(imgh, t, To, (ch0 + 16 * i) * ESZ, h);
        });
        cur ^= 1;
    }
    lz_publish();
    // out_conv (1x1, 128 -> 80) + b -> out [80][Tn]; e2e: MSE(out, tgt) - 0.1 MSE(out, org)
    // (attack_utils.py:41-43), its gradient and the per-utterance loss
    const bool e2e = A.tgt_out != nullptr;
    const float gscale = e2e ? A.scal[2] : 0.f;
    float q1 = 0.f, q2 = 0.f;
    float* OS = reinterpret_cast<float*>(fz_lds + 80 * 1024);   // [80][128] fp32 chunk of out
    const int tile0 = w < 2 ? 2 * w : 3;
    LzChunk chk;
    for (int k = 0; lz_chunk(k, lz_nf(Tn), NF, chk); ++k) {
        const int n0 = 16 * chk.f0;
        __syncthreads();
        lz_stage_cap<PREC>(WB, imgh, LZ_ZR + n0, 129, L);
        __syncthreads();
#pragma unroll
        for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, Tn - 1) - n0;
        f32x4 acc[2][NF];
        zero_acc(acc);
        fz_gemm<PREC, 2, NF, FZ_C, 1>(acc, IC<NF>{}, ring, op_out(), op_out(), WB, rb);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int tile = tile0 + i;
            const bool mine = w < 2 || (w == 2 && i == 1);
            if (!mine) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = 16 * tile + 4 * kq + r;
                const float bo = A.w.b_out[co];
#pragma unroll
                for (int f = 0; f < NF; ++f) OS[co * 128 + 16 * f + c] = acc[i][f][r] + bo;
            }
        }
        __syncthreads();
        float* outb = A.out + (size_t)b * DZ_COUT * Tn;
        // UO elements per thread at a time: the targets' loads, one drain, then the stores (the
        // same per-thread order of the loss sums)
        constexpr int UO = 10;
        for (int i0 = tid; i0 < DZ_COUT * 128; i0 += 256 * UO) {
            float tg[UO], og[UO];
            if (e2e) {
#pragma unroll
                for (int u = 0; u < UO; ++u) {
                    const int idx = min(i0 + 256 * u, DZ_COUT * 128 - 1);
                    const int co = idx >> 7, t = min(n0 + (idx & 127), Tn - 1);
                    const size_t qb = (size_t)b * DZ_COUT * Tn + (size_t)co * Tn + t;
                    tg[u] = A.tgt_out[qb];
                    og[u] = A.org_out[qb];
                }
                lz_vm_drain();
            }
#pragma unroll
            for (int u = 0; u < UO; ++u) {
                const int idx = i0 + 256 * u;
                if (idx >= DZ_COUT * 128) continue;
                const int co = idx >> 7, col = idx & 127;
                const int t = n0 + col;
                if (t >= Tn || !chk.owns(t)) continue;
                const float o = OS[idx];
                const size_t q = (size_t)co * Tn + t;
                outb[q] = o;
                if (e2e) {
                    const size_t qb = (size_t)b * DZ_COUT * Tn + q;
                    const float d1 = o - tg[u], d2 = o - og[u];
                    A.g_out[qb] = gscale * d1 + gscale * d2 * -0.1f;
                    q1 += d1 * d1;
                    q2 += d2 * d2;
                }
            }
        }
    }
    if (e2e && A.losses) {
        // per-utterance loss: wave partial sums (fixed butterfly) then a fixed-order sum
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            q1 += __shfl_xor(q1, o);
            q2 += __shfl_xor(q2, o);
        }
        float* lsum = reinterpret_cast<float*>(fz_lds + 150 * 1024);
        __syncthreads();
        if (lane == 0) {
            lsum[2 * w] = q1;
            lsum[2 * w + 1] = q2;
        }
        __syncthreads();
        const int step = *A.step;
        if (tid == 0 && step >= 1 && step <= A.loss_len) {
            const float n = (float)(DZ_COUT * Tn);
            const float s1 = (lsum[0] + lsum[2]) + (lsum[4] + lsum[6]);
            const float s2 = (lsum[1] + lsum[3]) + (lsum[5] + lsum[7]);
            A.losses[(size_t)(step - 1) * A.B + b] = s1 / n - 0.1f * (s2 / n);
        }
    }
}
template <int PREC>
__global__ void __launch_bounds__(256, 1) lz_dec_fwd(DecArgs A, LongArgs L) {
    const KtStart kts = ktime_begin(&g_ktime_long[KT_LZ_DEC_FWD + (PREC == PREC_BF16)]);
    lz_dec_fwd_body<PREC>(A, L);
    ktime_end(&g_ktime_long[KT_LZ_DEC_FWD + (PREC == PREC_BF16)], kts);
}

template <int PREC>
__device__ __forceinline__ void lz_dec_bwd_body(DecArgs A, LongArgs L) {
    using Z = Lz<PREC>;
    constexpr int RS = Z::RS, ESZ = Z::ESZ, GRB = Z::GRB;
    constexpr int VE = 16 / ESZ, KS = 4 * VE;
    constexpr int NF = LZ_CHF;
    const int b = blockIdx.x;
    const int nblk = A.nblk, ks = A.ks, P = ks / 2, act = A.act;
    const int Tn = A.Tl[nblk];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, kq = lane >> 4;
    const int ch0 = 32 * w + 4 * kq;
    const float* cond = A.cond + (size_t)b * (2 * nblk) * 256;
    float* gcond = A.g_cond + (size_t)b * (2 * nblk) * 256;
    const float* stb = A.stash + (size_t)b * A.stash_per_utt;

    char* imgg = L.img[1] + (size_t)b * L.img_stride;    // dY image (half 0), the out_conv^T operand
    char* imgg2 = L.img[2] + (size_t)b * L.img_stride;   // dY image of half 1
    float* gh[2] = {L.fl[0] + (size_t)b * L.fl_stride, L.fl[1] + (size_t)b * L.fl_stride};
    float* tmp = L.fl[2] + (size_t)b * L.fl_stride;
    float* FSCR = reinterpret_cast<float*>(fz_lds + 150 * 1024) + w * (5 * 16 * 8);

    const int ns_c = ks * FZ_C / KS;
    const int ns_o = (DZ_COUT + KS - 1) / KS;
    auto op_outT = [&]() __attribute__((always_inline)) { return aop(A.w.outT, 2 * w, 2, ns_o, ns_o); };
    auto op_c1T = [&](int l) __attribute__((always_inline)) { return aop(A.w.c1T[l], 2 * w, 2, ns_c, ns_c); };
    auto op_c2T = [&](int l, int s) __attribute__((always_inline)) { return aop(A.w.c2T[l][s], 2 * w, 2, ns_c, ns_c); };
    ARing<2> ring;
    ring_fill(ring, op_outT());
    int rb[NF];
    char* WB = fz_lds;

    // g_in [80][Tn] -> image (channels 80..127 of each row zero: the K padding of out_conv^T)
    lz_zero_rows<PREC>(imgg, 0, LZ_ZR + Tn + 2 * LZ_ZR);
    lz_publish();
    lz_ct_to_img<PREC, DZ_COUT>(imgg, A.g_in + (size_t)b * DZ_COUT * Tn, Tn);
    lz_publish();
    // g(h_N) = out_conv^T g_out -> gh[0]
    {
        LzChunk chk;
        for (int k = 0; lz_chunk(k, lz_nf(Tn), NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            __syncthreads();
            lz_stage_cap<PREC>(WB, imgg, LZ_ZR + n0, 130, L);
            __syncthreads();
#pragma unroll
            for (int f = 0; f < NF; ++f) rb[f] = min(n0 + 16 * f + c, Tn - 1) - n0;
            f32x4 acc[2][NF];
            zero_acc(acc);
            fz_gemm<PREC, 2, NF, DZ_COUT, 1>(acc, IC<NF>{}, ring, op_outT(),
                                            chk.last ? op_c2T(nblk - 1, 0) : op_outT(), WB, rb);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = n0 + 16 * f + c;
                if (t < Tn && chk.owns(t))
#pragma unroll
                    for (int i = 0; i < 2; ++i) *lz_fl(gh[0], t, w, i) = acc[i][f];
            }
        }
    }
    // act + AdaIN + InstanceNorm backward of IN layer q over Tl frames (models.py:66-79, 176):
    //   z = yhat*std + mean, g_z = g * act'(z);  d/dmean = sum g_z,  d/dstd = sum g_z yhat;
    //   d/dx = invstd std (g_z - (sum g_z)/n - yhat (sum g_z yhat)/n).
    // gsrc(t, i) -> g; pass 1 keeps g_z in tmp and writes d/d cond[q]; pass 2 hands
    // (t, i, d/dx) to out.
    // pass 2 (and the d/d cond[q] store) from the pass-1 sums gm / gs
    auto adain_in_bwd_tail = [&](int q, int Tl, f32x4 (&gm)[2], f32x4 (&gs)[2], auto&& out) __attribute__((always_inline)) {
        const float* yq = stb + A.stash_off[q];
        f32x4 sd[2], is[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            sd[i] = *reinterpret_cast<const f32x4*>(cond + q * 256 + 128 + ch0 + 16 * i);
            is[i] = *reinterpret_cast<const f32x4*>(A.invstd + ((size_t)b * 2 * nblk + q) * 128 + ch0 + 16 * i);
        }
        f32x4 k1[2], k2[2], k3[2];
        const float inv_n = 1.f / (float)Tl;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            row16_sum(gm[i]);
            row16_sum(gs[i]);
            if (c == 0) {
                *reinterpret_cast<f32x4*>(gcond + q * 256 + ch0 + 16 * i) = gm[i];
                *reinterpret_cast<f32x4*>(gcond + q * 256 + 128 + ch0 + 16 * i) = gs[i];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                k1[i][r] = is[i][r] * sd[i][r];
                k2[i][r] = gm[i][r] * inv_n;
                k3[i][r] = gs[i][r] * inv_n;
            }
        }
        lz_publish();
        for (int F0 = 0; F0 < lz_nf(Tl); F0 += LZ_FB) {
            f32x4 zv[LZ_FB][2], yv[LZ_FB][2];
#pragma unroll
            for (int u = 0; u < LZ_FB; ++u) {
                const int tc = min(16 * (F0 + u) + c, Tl - 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    zv[u][i] = *lz_fl(tmp, tc, w, i);
                    yv[u][i] = lz_stash_get<PREC>(yq, tc, w, i);
                }
            }
            lz_vm_drain();
#pragma unroll
            for (int u = 0; u < LZ_FB; ++u) {
                const int t = 16 * (F0 + u) + c;
                if (t < Tl)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const f32x4 z = zv[u][i], yh = yv[u][i];
                        f32x4 d;
#pragma unroll
                        for (int r = 0; r < 4; ++r) d[r] = k1[i][r] * (z[r] - k2[i][r] - yh[r] * k3[i][r]);
                        out(t, i, d);
                    }
            }
        }
    };
    auto adain_in_bwd = [&](int q, int Tl, auto&& gsrc, auto&& out) __attribute__((always_inline)) {
        const float* yq = stb + A.stash_off[q];
        f32x4 mn[2], sd[2], gm[2], gs[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            mn[i] = *reinterpret_cast<const f32x4*>(cond + q * 256 + ch0 + 16 * i);
            sd[i] = *reinterpret_cast<const f32x4*>(cond + q * 256 + 128 + ch0 + 16 * i);
            gm[i] = gs[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        lz_publish();
        // LZ_FB fragments at a time: loads, one drain, then arithmetic and stores (in_pass)
        for (int F0 = 0; F0 < lz_nf(Tl); F0 += LZ_FB) {
            f32x4 gv[LZ_FB][2], yv[LZ_FB][2];
#pragma unroll
            for (int u = 0; u < LZ_FB; ++u) {
                const int tc = min(16 * (F0 + u) + c, Tl - 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    gv[u][i] = gsrc(tc, i);
                    yv[u][i] = lz_stash_get<PREC>(yq, tc, w, i);
                }
            }
            lz_vm_drain();
#pragma unroll
            for (int u = 0; u < LZ_FB; ++u) {
                const int t = 16 * (F0 + u) + c;
                if (t < Tl)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const f32x4 g = gv[u][i], yh = yv[u][i];
                        f32x4 z;
#pragma unroll
                        for (int r = 0; r < 4; ++r) z[r] = g[r] * act_d(yh[r] * sd[i][r] + mn[i][r], act);
                        *lz_fl(tmp, t, w, i) = z;
                        gm[i] += z;
                        gs[i] += z * yh;
                    }
            }
        }
        adain_in_bwd_tail(q, Tl, gm, gs, out);
    };

    int cur = 0;
    // pass-1 sums of the next conv2 branch's IN backward, accumulated by the conv1^T epilogue
    // that produces its input gradient (every block but the last, which starts from out_conv^T)
    f32x4 gm2[2], gs2[2];
    for (int l = nblk - 1; l >= 0; --l) {
        const int Ti = A.Tl[l], up = A.up[l], To = Ti * up;
        float* gin = gh[cur];            // g(h_{l+1}) over To frames
        float* gout = gh[cur ^ 1];       // g(h_l) over Ti frames
        // conv2 branch: act, AdaIN(2l+1), IN backward over To frames -> dY image(s): frame
        // 2t + s of the shuffled output is half s of frame t
        auto dy2 = [&](int t, int i, f32x4 d) __attribute__((always_inline)) {
            char* im = (up == 2 && (t & 1)) ? imgg2 : imgg;
            const int tt = up == 2 ? t >> 1 : t;
            st4<PREC>(im + (size_t)(LZ_ZR + tt) * GRB + (ch0 + 16 * i) * ESZ, d);
        };
        if (l == nblk - 1)
            adain_in_bwd(2 * l + 1, To, [&](int t, int i) __attribute__((always_inline)) { return f32x4(*lz_fl(gin, t, w, i)); },
                         dy2);
        else
            adain_in_bwd_tail(2 * l + 1, To, gm2, gs2, dy2);
        lz_zero_rows<PREC>(imgg, 0, LZ_ZR);
        lz_zero_rows<PREC>(imgg, LZ_ZR + Ti, LZ_ZR);
        if (up == 2) {
            lz_zero_rows<PREC>(imgg2, 0, LZ_ZR);
            lz_zero_rows<PREC>(imgg2, LZ_ZR + Ti, LZ_ZR);
        }
        lz_publish();
        // conv2^T (both halves) over padded positions of the Ti frames = g of conv1's output, and in
        // the same epilogue the first pass of conv1's act + AdaIN(2l) + IN backward on the chunk's
        // owned frames: g_z -> tmp and its two row sums (the sums in the order a separate pass over
        // the frames would take: bitwise the same, one fp32 stream write + read fewer)
        const int nfc = lz_nf(Ti + 16 + P);
        const float* yq1 = stb + A.stash_off[2 * l];
        f32x4 mn1[2], sd1[2], gm1[2], gs1[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            mn1[i] = *reinterpret_cast<const f32x4*>(cond + (2 * l) * 256 + ch0 + 16 * i);
            sd1[i] = *reinterpret_cast<const f32x4*>(cond + (2 * l) * 256 + 128 + ch0 + 16 * i);
            gm1[i] = gs1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        LzChunk chk;
        for (int k = 0; lz_chunk(k, nfc, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            const int vlo = max(n0 - 16, -P), vhi = min(n0 + 111, Ti + P - 1);
            const int r0 = LZ_ZR + vlo + P - ks - 1;
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int v = min(max(n0 + 16 * f + c - 16, -P), Ti + P - 1);
                rb[f] = LZ_ZR + v + P - r0;
            }
            f32x4 acc[2][NF];
            zero_acc(acc);
            for (int s = 0; s < up; ++s) {
                __syncthreads();
                lz_stage_cap<PREC>(WB, s ? imgg2 : imgg, r0, vhi - vlo + ks + 2, L);
                __syncthreads();
                const AOp nx = s + 1 < up ? op_c2T(l, 1) : (chk.last ? (l > 0 ? op_c1T(l) : op_c2T(l, 0)) : op_c2T(l, 0));
                fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, IC<NF>{}, ring, op_c2T(l, s), nx, WB, rb);
            }
            f32x4 yv[NF][2];   // the stash rows of the chunk's frames, loaded before any store
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = min(max(16 * (chk.f0 + f - 1) + c, 0), Ti - 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) yv[f][i] = lz_stash_get<PREC>(yq1, t, w, i);
            }
            lz_vm_drain();
            lz_fold<2>(acc, chk.f0, 16, Ti, P, FSCR);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int F = chk.f0 + f - 1, t = 16 * F + c;
                if (F < 0 || 16 * F >= Ti || !chk.owns(16 * (F + 1))) continue;
                if (t < Ti)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const f32x4 yh = yv[f][i];
                        f32x4 z;
#pragma unroll
                        for (int r = 0; r < 4; ++r) z[r] = acc[i][f][r] * act_d(yh[r] * sd1[i][r] + mn1[i][r], act);
                        *lz_fl(tmp, t, w, i) = z;
                        gm1[i] += z;
                        gs1[i] += z * yh;
                    }
            }
        }
        // conv1 branch: the rest of its IN backward -> dY of conv1 (the first block stops: mu is
        // constant in the attacks)
        if (l == 0) {
            adain_in_bwd_tail(0, Ti, gm1, gs1, [&](int, int, f32x4) __attribute__((always_inline)) {});
            break;
        }
        adain_in_bwd_tail(2 * l, Ti, gm1, gs1, [&](int t, int i, f32x4 d) __attribute__((always_inline)) {
            st4<PREC>(imgg + (size_t)(LZ_ZR + t) * GRB + (ch0 + 16 * i) * ESZ, d);
        });
        lz_zero_rows<PREC>(imgg, 0, LZ_ZR);
        lz_zero_rows<PREC>(imgg, LZ_ZR + Ti, LZ_ZR);
        lz_publish();
        // conv1^T (+ fold) + the residual branch (adjoint of the x2 nearest upsample) -> g(h_l),
        // and on it the first pass of block l-1's conv2-branch IN backward (AdaIN(2l-1) over the
        // same Ti frames): g_z -> tmp, its row sums -> gm2 / gs2
        const float* yq2 = stb + A.stash_off[2 * l - 1];
        f32x4 mn2[2], sd2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            mn2[i] = *reinterpret_cast<const f32x4*>(cond + (2 * l - 1) * 256 + ch0 + 16 * i);
            sd2[i] = *reinterpret_cast<const f32x4*>(cond + (2 * l - 1) * 256 + 128 + ch0 + 16 * i);
            gm2[i] = gs2[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        auto r0_g = [=](const LzChunk& ch) __attribute__((always_inline)) {
            return LZ_ZR + max(16 * ch.f0 - 16, -P) + P - ks - 1;
        };
        auto nr_g = [=](const LzChunk& ch) __attribute__((always_inline)) {
            return min(16 * ch.f0 + 111, Ti + P - 1) - max(16 * ch.f0 - 16, -P) + ks + 2;
        };
        LzPipe<PREC, 136> pipeg(WB, nfc, 127 + ks + 2, lz_img_rows<PREC>(L));
        pipeg.prime(imgg, r0_g, nr_g);
        for (int k = 0; lz_chunk(k, nfc, NF, chk); ++k) {
            const int n0 = 16 * chk.f0;
            const int r0 = r0_g(chk);
            const char* SB = pipeg.next(k, chk, imgg, r0_g, nr_g);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int v = min(max(n0 + 16 * f + c - 16, -P), Ti + P - 1);
                rb[f] = LZ_ZR + v + P - r0;
            }
            f32x4 acc[2][NF];
            zero_acc(acc);
            fz_gemm<PREC, 2, NF, FZ_C, -1>(acc, IC<NF>{}, ring, op_c1T(l), chk.last ? op_c2T(l - 1, 0) : op_c1T(l),
                                           SB, rb);
            // the residual branch's gradient of the chunk, loaded and summed before the stores
            f32x4 res[NF][2];
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = min(max(16 * (chk.f0 + f - 1) + c, 0), Ti - 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) res[f][i] = *lz_fl(gin, up * t, w, i);
            }
            if (up == 2) {
                f32x4 r1[NF][2];
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const int t = min(max(16 * (chk.f0 + f - 1) + c, 0), Ti - 1);
#pragma unroll
                    for (int i = 0; i < 2; ++i) r1[f][i] = *lz_fl(gin, 2 * t + 1, w, i);
                }
                lz_vm_drain();
#pragma unroll
                for (int f = 0; f < NF; ++f)
#pragma unroll
                    for (int i = 0; i < 2; ++i) res[f][i] = res[f][i] + r1[f][i];
            }
            f32x4 yv[NF][2];   // block l-1's conv2-branch stash rows of the chunk's frames
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int t = min(max(16 * (chk.f0 + f - 1) + c, 0), Ti - 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) yv[f][i] = lz_stash_get<PREC>(yq2, t, w, i);
            }
            lz_vm_drain();
            pipeg.issue_next(k, imgg, r0_g, nr_g);   // after the drain: it would wait for the DMA too
            lz_fold<2>(acc, chk.f0, 16, Ti, P, FSCR);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const int F = chk.f0 + f - 1, t = 16 * F + c;
                if (F < 0 || 16 * F >= Ti || !chk.owns(16 * (F + 1))) continue;
                if (t < Ti)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const f32x4 g = res[f][i] + acc[i][f], yh = yv[f][i];
                        *lz_fl(gout, t, w, i) = g;
                        f32x4 z;
#pragma unroll
                        for (int r = 0; r < 4; ++r) z[r] = g[r] * act_d(yh[r] * sd2[i][r] + mn2[i][r], act);
                        *lz_fl(tmp, t, w, i) = z;
                        gm2[i] += z;
                        gs2[i] += z * yh;
                    }
            }
        }
        cur ^= 1;
    }
}
template <int PREC>
__global__ void __launch_bounds__(256, 1) lz_dec_bwd(DecArgs A, LongArgs L) {
    const KtStart kts = ktime_begin(&g_ktime_long[KT_LZ_DEC_BWD + (PREC == PREC_BF16)]);
    lz_dec_bwd_body<PREC>(A, L);
    ktime_end(&g_ktime_long[KT_LZ_DEC_BWD + (PREC == PREC_BF16)], kts);
}

// LDS bytes of the long kernels (the host sets the same)
constexpr int LZ_LDS_BYTES = 160 * 1024;

#define AVC_LZ_INST(P)                                                    \
    template __global__ void lz_se_fwd<P>(FusedArgs, LongArgs);          \
    template __global__ void lz_se_bwd<P>(FusedArgs, LongArgs);          \
    template __global__ void lz_dec_fwd<P>(DecArgs, LongArgs);           \
    template __global__ void lz_dec_bwd<P>(DecArgs, LongArgs);
AVC_LZ_INST(PREC_F32)
AVC_LZ_INST(PREC_BF16)
#undef AVC_LZ_INST

}  // namespace avc
