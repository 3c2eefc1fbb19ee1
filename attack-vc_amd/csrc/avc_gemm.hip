// conv_gemm: every Conv1d of the SpeakerEncoder (models.py:82-104, 265-305) and
// every input-gradient (dgrad) of one, as an implicit GEMM on the CDNA4 matrix
// cores of gfx950:
//     C[M][N] = A[M][K] * B[K][N]    M = output channels, N = (utterance, t),
//                                    K = (input channel, tap)
//   PREC_F32 : v_mfma_f32_32x32x2_f32   (f32 in / f32 acc, bitwise a k-ordered fma chain)
//   PREC_BF16: v_mfma_f32_32x32x16_bf16 (bf16 in / f32 acc)
// Both produce the same 32x32 C/D register map, so staging and epilogues are shared.
//
// A (weights) is pre-packed row-major [Mpad][Kld] (k contiguous, zero padded),
// in fp32 or bf16.  B, the im2col tile, never exists in HBM: each K chunk is
// gathered from the [B][C][T] activations (reflect padding forward; zero
// dilation + flipped taps + reflect fold for the dgrad) into registers one
// chunk ahead and stored to a double-buffered LDS tile [N][K] (k contiguous),
// so one barrier per chunk separates "compute chunk k" from "store chunk k+1".
// Epilogues are fused and vectorised (4 consecutive frames per lane).
#include <hip/hip_runtime.h>

#include "avc_device.h"
#include "avc_kernels.h"

#ifndef AVC_ABLATE
#define AVC_ABLATE 0
#endif

namespace avc {

template <int PREC>
struct PrecT;
template <>
struct PrecT<PREC_F32> {
    using T = float;
    static constexpr int KPAD = 4;   // +16 B per LDS row: distinct bank slots for ds_read_b128
};
template <>
struct PrecT<PREC_BF16> {
    using T = __bf16;
    static constexpr int KPAD = 8;   // +16 B per LDS row
};

// Index of dY for padded-output coordinate q of a stride-s conv; `ok` is false
// where the zero-dilation leaves a hole or q falls outside [0, T).  The caller
// loads row[idx] unconditionally (idx is clamped in range) and selects later.
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

// ---------------------------------------------------------------------------------
// epilogues
// ---------------------------------------------------------------------------------

// one element (general path: any T, tile edges)
__device__ __forceinline__ void epilogue1(const Problem& P, int m, int b, int t, float acc) {
    const int T = P.T_out;
    switch (P.epi) {
    case EPI_ACT: {
        P.out0[((size_t)b * P.out0_C + P.out0_coff + m) * T + t] = act_f(acc + P.bias[m], P.act);
        break;
    }
    case EPI_BLOCK: {  // conv_blocks (models.py:299-304): y = act(conv2); out = y + avgpool(out)
        const float a2 = act_f(acc + P.bias[m], P.act);
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
        const float y = P.aux0[((size_t)b * P.aux0_C + m) * P.aux0_T + t];
        P.out0[((size_t)b * P.out0_C + m) * T + t] = acc * act_d(y, P.act);
        break;
    }
    case EPI_POOLT: {  // + d(avg_pool1d ceil_mode)/d(input); masked copy = next dgrad's dY
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
        if (P.out1) P.out1[o] = gv * act_d(P.aux1[o], P.act);
        break;
    }
    case EPI_INCONV_T: {  // d(cat)/d: bank part gated by its ReLU, x part passes through
        if (m < P.split) {
            const float y = P.aux0[((size_t)b * P.aux0_C + m) * P.aux0_T + t];
            P.out0[((size_t)b * P.out0_C + m) * T + t] = acc * act_d(y, P.act);
        } else {
            P.out1[((size_t)b * P.out1_C + (m - P.split)) * T + t] = acc;
        }
        break;
    }
    case EPI_ADAM: {
        // adv = vc + eps*tanh(ptb) backward (attack_utils.py:78), then torch.optim.Adam
        // _single_tensor_adam: m.lerp_(g,1-b1); v.mul_(b2).addcmul_(g,g,1-b2);
        // p.addcdiv_(m, sqrt(v)/sqrt(bc2)+eps, -lr/bc1); next adv = vc + eps*tanh(p)
        const AdamArgs& A = P.adam;
        const size_t idx = ((size_t)b * P.M + m) * T + t;
        const float eps = P.scal[0];
        const int step = min(max(*P.step, 1), P.table_len);
        const float nstep = A.table[2 * (step - 1)];
        const float bc2s = A.table[2 * (step - 1) + 1];
        float p = A.ptb[idx];
        const float pgd = P.scal[3];
        if (pgd > 0.f) {   // opt-in sign-gradient update (see adam_elem, avc_fused_core.h)
            const float gs = acc + P.aux0[idx];
            if (A.grad0 && step == 1) A.grad0[idx] = gs;
            p = fminf(fmaxf(p - pgd * (gs > 0.f ? 1.f : (gs < 0.f ? -1.f : 0.f)), -eps), eps);
            A.ptb[idx] = p;
            A.adv[idx] = A.vc[idx] + p;
            break;
        }
        const float th = tanhf(p);
        const float g = ((acc + P.aux0[idx]) * eps) * (1.f - th * th);
        if (A.grad0 && step == 1) A.grad0[idx] = g;
        float mm = A.m[idx];
        mm = mm + A.b1c * (g - mm);
        float vv = A.v[idx] * A.b2;
        vv = vv + A.b2c * g * g;
        p = p + nstep * (mm / (sqrtf(vv) / bc2s + A.adam_eps));
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

// four consecutive frames t..t+3 of one utterance (T % 4 == 0, t % 4 == 0):
// 16-byte loads/stores throughout; returns false if this element group must
// take the scalar path (ceil-mode pooling tail).
__device__ __forceinline__ bool epilogue4(const Problem& P, int m, int b, int t, f32x4 v) {
    const int T = P.T_out;
    switch (P.epi) {
    case EPI_ACT: {
        const float bi = P.bias[m];
        f32x4 y;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = act_f(v[e] + bi, P.act);
        gstore<f32x4>(P.out0 + ((size_t)b * P.out0_C + P.out0_coff + m) * T + t, y);
        return true;
    }
    case EPI_BLOCK: {
        const float* hin = P.aux0 + ((size_t)b * P.aux0_C + m) * P.aux0_T;
        f32x4 res;
        if (P.pool_s == 1) {
            res = gload<f32x4>(hin + t);
        } else if (P.pool_s == 2 && 2 * t + 8 <= P.aux0_T) {
            const f32x4 lo = gload<f32x4>(hin + 2 * t), hi = gload<f32x4>(hin + 2 * t + 4);
            res = f32x4{(lo[0] + lo[1]) / 2.f, (lo[2] + lo[3]) / 2.f, (hi[0] + hi[1]) / 2.f, (hi[2] + hi[3]) / 2.f};
        } else {
            return false;
        }
        const float bi = P.bias[m];
        f32x4 a2, o1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            a2[e] = act_f(v[e] + bi, P.act);
            o1[e] = a2[e] + res[e];
        }
        gstore<f32x4>(P.out0 + ((size_t)b * P.out0_C + m) * T + t, a2);
        gstore<f32x4>(P.out1 + ((size_t)b * P.out1_C + m) * T + t, o1);
        return true;
    }
    case EPI_MASK: {
        const f32x4 y = gload<f32x4>(P.aux0 + ((size_t)b * P.aux0_C + m) * P.aux0_T + t);
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = v[e] * act_d(y[e], P.act);
        gstore<f32x4>(P.out0 + ((size_t)b * P.out0_C + m) * T + t, o);
        return true;
    }
    case EPI_POOLT: {
        const float* g = P.aux0 + ((size_t)b * P.aux0_C + m) * P.aux0_T;
        f32x4 gv;
        if (P.pool_s == 1) {
            const f32x4 r = gload<f32x4>(g + t);
            gv = v + r;
        } else if (P.pool_s == 2) {   // T even here, every window has 2 inputs
            const f32x2 r = gload<f32x2>(g + t / 2);
            gv = f32x4{v[0] + r[0] / 2.f, v[1] + r[0] / 2.f, v[2] + r[1] / 2.f, v[3] + r[1] / 2.f};
        } else {
            return false;
        }
        const size_t o = ((size_t)b * P.out0_C + m) * T + t;
        if (P.out0) gstore<f32x4>(P.out0 + o, gv);
        if (P.out1) {
            const f32x4 y = gload<f32x4>(P.aux1 + o);
            f32x4 mk;
#pragma unroll
            for (int e = 0; e < 4; ++e) mk[e] = gv[e] * act_d(y[e], P.act);
            gstore<f32x4>(P.out1 + o, mk);
        }
        return true;
    }
    case EPI_INCONV_T: {
        if (m < P.split) {
            const f32x4 y = gload<f32x4>(P.aux0 + ((size_t)b * P.aux0_C + m) * P.aux0_T + t);
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = v[e] * act_d(y[e], P.act);
            gstore<f32x4>(P.out0 + ((size_t)b * P.out0_C + m) * T + t, o);
        } else {
            gstore<f32x4>(P.out1 + ((size_t)b * P.out1_C + (m - P.split)) * T + t, v);
        }
        return true;
    }
    case EPI_ADAM: {
        const AdamArgs& A = P.adam;
        const size_t idx = ((size_t)b * P.M + m) * T + t;
        const float eps = P.scal[0];
        const int step = min(max(*P.step, 1), P.table_len);
        const float nstep = A.table[2 * (step - 1)];
        const float bc2s = A.table[2 * (step - 1) + 1];
        f32x4 p = gload<f32x4>(A.ptb + idx);
        const f32x4 gx = gload<f32x4>(P.aux0 + idx);
        f32x4 mm = gload<f32x4>(A.m + idx);
        f32x4 vv = gload<f32x4>(A.v + idx);
        const f32x4 vc = gload<f32x4>(A.vc + idx);
        f32x4 g, adv;
        const float pgd = P.scal[3];
        if (pgd > 0.f) {   // opt-in sign-gradient update (see adam_elem, avc_fused_core.h)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                g[e] = v[e] + gx[e];
                p[e] = fminf(fmaxf(p[e] - pgd * (g[e] > 0.f ? 1.f : (g[e] < 0.f ? -1.f : 0.f)), -eps), eps);
                adv[e] = vc[e] + p[e];
            }
            if (A.grad0 && step == 1) gstore<f32x4>(A.grad0 + idx, g);
            gstore<f32x4>(A.ptb + idx, p);
            gstore<f32x4>(A.adv + idx, adv);
            return true;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float th = tanhf(p[e]);
            g[e] = ((v[e] + gx[e]) * eps) * (1.f - th * th);
            mm[e] = mm[e] + A.b1c * (g[e] - mm[e]);
            float w = vv[e] * A.b2;
            vv[e] = w + A.b2c * g[e] * g[e];
            p[e] = p[e] + nstep * (mm[e] / (sqrtf(vv[e]) / bc2s + A.adam_eps));
            adv[e] = vc[e] + eps * tanhf(p[e]);
        }
        if (A.grad0 && step == 1) gstore<f32x4>(A.grad0 + idx, g);
        gstore<f32x4>(A.ptb + idx, p);
        gstore<f32x4>(A.m + idx, mm);
        gstore<f32x4>(A.v + idx, vv);
        gstore<f32x4>(A.adv + idx, adv);
        return true;
    }
    default:
        return true;
    }
}

// ---------------------------------------------------------------------------------
// the GEMM
// ---------------------------------------------------------------------------------

// WM x WN 32x32 fragments per wave, WGM x WGN waves per workgroup, K chunk KC.
template <int PREC, int WM, int WN, int WGM, int WGN, int KC, int MODE, int STRIDE>
__global__ void __launch_bounds__(64 * WGM * WGN) conv_gemm(const Problem* __restrict__ probs, int ksplit) {
    using E = typename PrecT<PREC>::T;
    constexpr int NTHR = 64 * WGM * WGN;
    constexpr int MT = 32 * WM * WGM, NT = 32 * WN * WGN;
    constexpr int KP = KC + PrecT<PREC>::KPAD;           // LDS row length (elements)
    constexpr int STAGE = (MT + NT) * KP;                 // elements per LDS stage
    constexpr int EW = 32 * WN + 4;                       // epilogue stage row (floats)
    constexpr int EPI_FLOATS = WGM * WGN * 32 * WM * EW;
    constexpr int LDS_BYTES_MAIN = 2 * STAGE * (int)sizeof(E);
    constexpr int LDS_BYTES = LDS_BYTES_MAIN > EPI_FLOATS * 4 ? LDS_BYTES_MAIN : EPI_FLOATS * 4;
    constexpr int BROWS = NTHR / NT;                      // K rows gathered per thread-row group
    constexpr int BPASS = KC / BROWS;                     // K rows gathered per thread
    constexpr int AVEC = 16 / (int)sizeof(E);             // A elements per 16-byte load
    constexpr int ALOADS = MT * KC / AVEC / NTHR;         // A 16-byte loads per thread per chunk
    static_assert(NTHR % NT == 0 && KC % BROWS == 0 && BPASS % 4 == 0 && BPASS <= 16, "B loader shape");
    static_assert((MT * KC / AVEC) % NTHR == 0, "A loader shape");
    static_assert(PREC == PREC_F32 ? KC % 8 == 0 : KC % 16 == 0, "K chunk vs MFMA K");

    // blockIdx.z = problem * ksplit + split (split-K: this WG sums K rows
    // [split*ksplit_rows, (split+1)*ksplit_rows) into a slab; splitk_reduce finishes)
    const int split = blockIdx.z % ksplit;
    const Problem& P = probs[blockIdx.z / ksplit];
    const int m0 = blockIdx.y * MT, n0 = blockIdx.x * NT;
    if (P.tick && split == 0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(P.tick, 1);
    if (m0 >= P.M || n0 >= P.N) return;

    __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES];
    E* const lds = reinterpret_cast<E*>(lds_raw);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WGN, wn = wave % WGN;
    const int r32 = lane & 31, h = lane >> 5;

    const int N = P.N, T_out = P.T_out, Kend = P.K, Kld = P.Kld, nseg = P.nseg, act = P.act, Mpad = P.Mpad;
    const E* __restrict__ Ag = reinterpret_cast<const E*>(PREC == PREC_F32 ? (const void*)P.At : P.Ab);

    // B loader: lanes <-> columns n; each thread owns BPASS consecutive K rows of the
    // chunk, so (segment, c, j) is wave-uniform and advances by one tap per row.
    const int nl = tid % NT;
    const int rg = __builtin_amdgcn_readfirstlane(tid / NT);
    const int n = n0 + nl;
    const bool nvalid = n < N;
    const int bb = nvalid ? n / T_out : 0;
    const int tt = nvalid ? n - bb * T_out : 0;

    f32x4 areg[ALOADS];                                   // 16 bytes each (4 f32 or 8 bf16)
    float breg[BPASS];
    float ereg[MODE == SEG_BWD ? BPASS : 1];              // reflect-fold term of the adjoint gather
    unsigned vmask = 0u;                                  // bit p: main term valid; 16+p: fold term
    const bool both_edges = MODE == SEG_BWD && P.both_edges;

    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto load_chunk = [&](int kc) {
        const int k0 = kc * KC;
#pragma unroll
        for (int i = 0; i < ALOADS; ++i) {
            const int f = tid + i * NTHR;
            const int r = f / (KC / AVEC), c = f % (KC / AVEC);
            if (AVC_ABLATE & 4) {
                areg[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            } else {
                // rows past Mpad are never allocated: clamp (their outputs are discarded)
                const E* src = Ag + (size_t)min(m0 + r, Mpad - 1) * Kld + k0 + c * AVEC;
                areg[i] = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(
                    (const __attribute__((address_space(1))) E*)src);
            }
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
            const bool live = c < C;                      // wave-uniform (padded rows are 0)
            const gcptr row = base + (size_t)(live ? c : 0) * srcT;
            if (MODE == SEG_FWD) {
                // x_pad[c][t*stride + j] of F.pad(mode="reflect") (models.py:23-29)
                const int st = STRIDE ? STRIDE : S.stride;
                int q = tt * st + j - pl;
                q = q < 0 ? -q : q;
                q = q >= srcT ? 2 * srcT - 2 - q : q;
                breg[p] = (AVC_ABLATE & 1) ? 0.f : row[q];
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
                breg[p] = (AVC_ABLATE & 1) ? 0.f : row[i0];
                ereg[p] = (AVC_ABLATE & 1) ? 0.f : row[i1];
                if (both_edges) {   // tiny T only: a waited load is acceptable there
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

    auto store_chunk = [&](int stage) {
        E* ldsA = lds + stage * STAGE;
        E* ldsB = ldsA + MT * KP;
#pragma unroll
        for (int i = 0; i < ALOADS; ++i) {
            const int f = tid + i * NTHR;
            const int r = f / (KC / AVEC), c = f % (KC / AVEC);
            *reinterpret_cast<f32x4*>(&ldsA[r * KP + c * AVEC]) = areg[i];
        }
#pragma unroll
        for (int p4 = 0; p4 < BPASS; p4 += 4) {
            f32x4 w;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int p = p4 + e;
                float v = ((vmask >> p) & 1u) ? breg[p] : 0.f;
                if (MODE == SEG_BWD) v += ((vmask >> (16 + p)) & 1u) ? ereg[p] : 0.f;
                w[e] = nvalid ? v : 0.f;
            }
            if (PREC == PREC_F32) {
                *reinterpret_cast<f32x4*>(&ldsB[nl * KP + rg * BPASS + p4]) = w;
            } else {
                bf16x4 wb;
#pragma unroll
                for (int e = 0; e < 4; ++e) wb[e] = (__bf16)w[e];
                *reinterpret_cast<bf16x4*>(&ldsB[nl * KP + rg * BPASS + p4]) = wb;
            }
        }
    };

    auto compute = [&](int stage) {
        const E* ldsA = lds + stage * STAGE;
        const E* ldsB = ldsA + MT * KP;
        if (PREC == PREC_F32) {
            // K permutation inside the chunk: k-step s of lane half h uses chunk row
            // h*KC/2 + s for both operands -> 4 k-steps per ds_read_b128.
#pragma unroll
            for (int q = 0; q < KC / 8; ++q) {
                f32x4 a[WM], bv[WN];
#pragma unroll
                for (int i = 0; i < WM; ++i)
                    a[i] = *reinterpret_cast<const f32x4*>(
                        &ldsA[(wm * 32 * WM + 32 * i + r32) * KP + h * (KC / 2) + 4 * q]);
#pragma unroll
                for (int j = 0; j < WN; ++j)
                    bv[j] = *reinterpret_cast<const f32x4*>(
                        &ldsB[(wn * 32 * WN + 32 * j + r32) * KP + h * (KC / 2) + 4 * q]);
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < WM; ++i)
#pragma unroll
                        for (int j = 0; j < WN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][e], bv[j][e], acc[i][j], 0, 0, 0);
            }
        } else {
            // bf16 32x32x16: lane (row r32, half h) holds k = 8h .. 8h+7 of each 16-deep step
#pragma unroll
            for (int s = 0; s < KC / 16; ++s) {
                bf16x8 a[WM], bv[WN];
#pragma unroll
                for (int i = 0; i < WM; ++i)
                    a[i] = *reinterpret_cast<const bf16x8*>(
                        &ldsA[(wm * 32 * WM + 32 * i + r32) * KP + 16 * s + 8 * h]);
#pragma unroll
                for (int j = 0; j < WN; ++j)
                    bv[j] = *reinterpret_cast<const bf16x8*>(
                        &ldsB[(wn * 32 * WN + 32 * j + r32) * KP + 16 * s + 8 * h]);
#pragma unroll
                for (int i = 0; i < WM; ++i)
#pragma unroll
                    for (int j = 0; j < WN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], bv[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    // software pipeline: LDS double buffer, gathers one chunk ahead in registers,
    // one barrier per chunk
    int c_begin = 0, c_end = (Kend + KC - 1) / KC;
    if (ksplit > 1) {
        c_begin = split * (P.ksplit_rows / KC);
        c_end = min(c_end, c_begin + P.ksplit_rows / KC);
    }
    if (c_begin < c_end) {
        load_chunk(c_begin);
        store_chunk(0);
        if (c_begin + 1 < c_end) load_chunk(c_begin + 1);
        __syncthreads();
        for (int kc = c_begin; kc < c_end; ++kc) {
            const int st = (kc - c_begin) & 1;
            if (!(AVC_ABLATE & 16)) compute(st);
            if (kc + 1 < c_end) store_chunk(st ^ 1);
            if (kc + 2 < c_end) load_chunk(kc + 2);
            __syncthreads();
        }
    }

    // Epilogue: each wave stages its accumulators as [32*WM rows][32*WN (+4) cols]
    // floats (C/D map of the 32x32 tiles: col = lane&31, row = (r&3)+8*(r>>2)+4*(lane>>5)),
    // then walks them 4 consecutive columns per lane.
    float* stg = reinterpret_cast<float*>(lds_raw) + wave * (32 * WM * EW);
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                stg[(32 * i + (r & 3) + 8 * (r >> 2) + 4 * h) * EW + 32 * j + r32] = acc[i][j][r];
    __builtin_amdgcn_wave_barrier();
    if (AVC_ABLATE & 2) return;
    constexpr int C4 = 8 * WN;                            // float4 groups per staged row
    const int mw = m0 + wm * 32 * WM, nw = n0 + wn * 32 * WN;
    if (ksplit > 1) {   // raw partial sums; the epilogue runs in splitk_reduce
        float* slab = P.slab + (size_t)split * P.M * N;
        const bool v4 = (N & 3) == 0;
#pragma unroll 1
        for (int idx = lane; idx < 32 * WM * C4; idx += 64) {
            const int row = idx / C4, c4 = idx - row * C4;
            const int m = mw + row, nc = nw + 4 * c4;
            if (m >= P.M || nc >= N) continue;
            const f32x4 v = *reinterpret_cast<const f32x4*>(&stg[row * EW + 4 * c4]);
            if (v4) {
                gstore<f32x4>(slab + (size_t)m * N + nc, v);
            } else {
                for (int e = 0; e < 4 && nc + e < N; ++e) slab[(size_t)m * N + nc + e] = v[e];
            }
        }
        return;
    }
    const bool vec_ok = (T_out & 3) == 0;
#pragma unroll 1
    for (int idx = lane; idx < 32 * WM * C4; idx += 64) {
        const int row = idx / C4, c4 = idx - row * C4;
        const int m = mw + row;
        const int nc = nw + 4 * c4;
        if (m >= P.M || nc >= N) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(&stg[row * EW + 4 * c4]);
        const int b = nc / T_out, t = nc - b * T_out;
        if (vec_ok && nc + 3 < N && epilogue4(P, m, b, t, v)) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int ne = nc + e;
            if (ne >= N) break;
            const int be = ne / T_out;
            epilogue1(P, m, be, ne - be * T_out, v[e]);
        }
    }
}

// Split-K finish: sum the slabs in split order (deterministic; the split
// boundaries are multiples of KALIGN rows, independent of the tile variant)
// and apply the problem's fused epilogue, 4 consecutive columns per thread.
__global__ void __launch_bounds__(256) splitk_reduce(const Problem* __restrict__ probs, int ksplit) {
    const Problem& P = probs[blockIdx.z];
    const int N = P.N, M = P.M, T = P.T_out;
    const int ng = (N + 3) / 4;
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)M * ng) return;
    const int m = (int)(gid / ng), nc = (int)(gid - (long)m * ng) * 4;
    const size_t plane = (size_t)M * N;
    const float* base = P.slab + (size_t)m * N + nc;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    const bool v4 = (N & 3) == 0;
    for (int s = 0; s < ksplit; ++s) {
        if (v4) {
            v += gload<f32x4>(base + s * plane);
        } else {
            for (int e = 0; e < 4 && nc + e < N; ++e) v[e] += base[s * plane + e];
        }
    }
    const int b = nc / T, t = nc - b * T;
    if ((T & 3) == 0 && nc + 3 < N && epilogue4(P, m, b, t, v)) return;
    for (int e = 0; e < 4; ++e) {
        const int ne = nc + e;
        if (ne >= N) break;
        const int be = ne / T;
        epilogue1(P, m, be, ne - be * T, v[e]);
    }
}

#define AVC_GEMM_MS(PREC, WM, WN, WGM, WGN, KC)                                                        \
    template __global__ void conv_gemm<PREC, WM, WN, WGM, WGN, KC, SEG_FWD, 1>(const Problem*, int); \
    template __global__ void conv_gemm<PREC, WM, WN, WGM, WGN, KC, SEG_FWD, 2>(const Problem*, int); \
    template __global__ void conv_gemm<PREC, WM, WN, WGM, WGN, KC, SEG_FWD, 0>(const Problem*, int); \
    template __global__ void conv_gemm<PREC, WM, WN, WGM, WGN, KC, SEG_BWD, 1>(const Problem*, int); \
    template __global__ void conv_gemm<PREC, WM, WN, WGM, WGN, KC, SEG_BWD, 2>(const Problem*, int); \
    template __global__ void conv_gemm<PREC, WM, WN, WGM, WGN, KC, SEG_BWD, 0>(const Problem*, int);
#define AVC_GEMM_VARIANT(I, PREC, WM, WN, WGM, WGN, KC, NAME) AVC_GEMM_MS(PREC, WM, WN, WGM, WGN, KC)
#include "avc_gemm_variants.h"
#undef AVC_GEMM_VARIANT
#undef AVC_GEMM_MS

}  // namespace avc
