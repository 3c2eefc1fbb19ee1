// VSMask PredictiveModel forward (/root/reference/models/predictive_model.py:6-110,
// BASELINE config 5) on gfx950: every layer is one implicit-GEMM launch
//   Y[Cout][n] = A[Cout][K] . B[K][n],  n = (window, output pixel)
// with B gathered on the fly from the NCHW activation:
//   mode 0  ReflectionPad2d(1) + Conv2d 3x3 stride (sh, sw): K = (ci, ky, kx), reflect
//           indexing of the input (the pad is never materialised); BatchNorm2d (eval)
//           folded into A and the bias on the host; PReLU (one slope) in the epilogue.
//   mode 1  ConvTranspose2d 3x3 stride 2 as four gather convolutions, one per output
//           parity class (oy & 1, ox & 1) = blockIdx.z: class (py, px) only meets taps
//           ky = 2a (py = 0, a = 0, 1) or 1 (py = 1), likewise kx, at input rows
//           qy - a (py = 0) / qy (py = 1) -- no multiply by an inserted zero.
//           LeakyReLU(0.2) (+ tanh on the last layer) in the epilogue.
// fp32 FMA on the VALU (the fp32 VALU and matrix rates are equal on gfx950): 64 x 64
// output tile per 256-thread workgroup, 4 x 4 per thread, K in chunks of 16 staged
// through LDS.
#include <hip/hip_runtime.h>

#include "avc_kernels.h"

namespace avc {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float pm_act(float v, const PmConvArgs& P) {
    if (P.act == 0) return v >= 0.f ? v : P.slope * v;                // PReLU
    v = v >= 0.f ? v : 0.2f * v;                                      // LeakyReLU(0.2)
    return P.act == 2 ? tanhf(v) : v;                                 // final tanh
}

__global__ void __launch_bounds__(256) pm_conv(PmConvArgs P) {
    constexpr int TM = 64, TN = 64, TK = 16;
    __shared__ float As[TK][TM + 4];
    __shared__ float Bs[TK][TN + 4];
    const int tid = threadIdx.x;
    const int ks = P.ksplit > 1 ? P.ksplit : 1;
    const int cls = blockIdx.z / ks, slice = blockIdx.z - cls * ks;
    const int py = cls >> 1, px = cls & 1;
    const int nty = P.mode == 1 ? (py == 0 ? 2 : 1) : 3;
    const int ntx = P.mode == 1 ? (px == 0 ? 2 : 1) : 3;
    const int Hq = P.mode == 1 ? (P.Ho - py + 1) / 2 : P.Ho;   // output rows of this class
    const int Wq = P.mode == 1 ? (P.Wo - px + 1) / 2 : P.Wo;
    const int N = P.B * Hq * Wq;
    const int K = P.Cin * nty * ntx;
    const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM;
    if (n0 >= N) return;                        // (uniform: class grids are padded to the largest)
    // this slice's K range, whole chunks
    const int nch = (K + TK - 1) / TK, cps = (nch + ks - 1) / ks;
    const int kbeg = slice * cps * TK, kend = min(K, (slice + 1) * cps * TK);
    const float* __restrict__ A = P.w + P.woff[cls];

    // this thread's gather column (fixed over K): n -> (window, qy, qx)
    const int gn = tid & 63;
    const int n = n0 + gn;
    const bool nval = n < N;
    int b = 0, qy = 0, qx = 0;
    if (nval) {
        b = n / (Hq * Wq);
        const int r = n - b * Hq * Wq;
        qy = r / Wq;
        qx = r - qy * Wq;
    }
    const float* __restrict__ xb = P.x + (size_t)b * P.Cin * P.Hin * P.Win;
    // the 4 A and 4 B elements this thread stages per chunk
    auto load_a = [&](int k0, float (&ra)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = tid + 256 * j, m = m0 + (e >> 4), k = k0 + (e & 15);
            ra[j] = (m < P.Cout && k < kend) ? A[(size_t)m * K + k] : 0.f;
        }
    };
    auto load_b = [&](int k0, float (&rb)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + (tid >> 6) + 4 * j;
            float v = 0.f;
            if (nval && k < kend) {
                const int ci = k / (nty * ntx);
                const int t = k - ci * nty * ntx;
                const int a = t / ntx, bb = t - a * ntx;
                int iy, ix;
                bool ok = true;
                if (P.mode == 0) {
                    iy = qy * P.sh + a - 1;
                    ix = qx * P.sw + bb - 1;
                    iy = iy < 0 ? -iy : (iy >= P.Hin ? 2 * (P.Hin - 1) - iy : iy);
                    ix = ix < 0 ? -ix : (ix >= P.Win ? 2 * (P.Win - 1) - ix : ix);
                } else {
                    iy = py == 0 ? qy - a : qy;
                    ix = px == 0 ? qx - bb : qx;
                    ok = iy >= 0 && iy < P.Hin && ix >= 0 && ix < P.Win;
                }
                if (ok) v = P.in_nhwc ? xb[((size_t)iy * P.Win + ix) * P.Cin + ci] : xb[((size_t)ci * P.Hin + iy) * P.Win + ix];
            }
            rb[j] = v;
        }
    };

    const int ty = tid >> 4, tx = tid & 15;     // 4 x 4 micro-tile: rows 4ty.., cols 4tx..
    float acc[4][4] = {};
    float ra[4], rb[4];
    load_a(kbeg, ra);
    load_b(kbeg, rb);
    for (int k0 = kbeg; k0 < kend; k0 += TK) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = tid + 256 * j;
            As[e & 15][e >> 4] = ra[j];
            Bs[(tid >> 6) + 4 * j][gn] = rb[j];
        }
        __syncthreads();
        // next chunk's global loads in flight during this chunk's FMAs
        if (k0 + TK < kend) {
            load_a(k0 + TK, ra);
            load_b(k0 + TK, rb);
        }
#pragma unroll
        for (int kk = 0; kk < TK; ++kk) {
            float a4[4], b4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a4[i] = As[kk][4 * ty + i];
                b4[i] = Bs[kk][4 * tx + i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a4[i], b4[j], acc[i][j]);
        }
        __syncthreads();
    }
    // epilogue: bias (BN folded) + activation, NCHW store -- or the raw slice partial
    const size_t per = (size_t)P.B * P.Cout * P.Ho * P.Wo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int nn = n0 + 4 * tx + j;
        if (nn >= N) continue;
        const int ob = nn / (Hq * Wq);
        const int r = nn - ob * Hq * Wq;
        const int oqy = r / Wq, oqx = r - oqy * Wq;
        const int oy = P.mode == 1 ? 2 * oqy + py : oqy;
        const int ox = P.mode == 1 ? 2 * oqx + px : oqx;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = m0 + 4 * ty + i;
            if (co >= P.Cout) continue;
            const size_t o = P.out_nhwc ? (((size_t)ob * P.Ho + oy) * P.Wo + ox) * P.Cout + co
                                        : (((size_t)ob * P.Cout + co) * P.Ho + oy) * P.Wo + ox;
            if (ks > 1) P.part[(size_t)slice * per + o] = acc[i][j];
            else P.y[o] = pm_act(acc[i][j] + P.bias[co], P);
        }
    }
}

// ---------------------------------------------------------------------------------
// The network's two edge layers, whose GEMM shapes waste pm_conv's 64 x 64 tiles: the first
// (Cin = 1: K = 9) and the last (Cout = 1: one row of 64 used, 98 % of the tile's MACs
// discarded -- 0.45 ms of a 1.5 ms forward at B = 256).  One thread per output pixel; the
// per-output arithmetic is pm_conv's: the same fmaf chain over k in pm_conv's K order
// (ci-major, taps inner), the same K slices summed in slice order as pm_reduce does, then
// bias + activation -- the results are pm_conv's bit for bit, and batch-invariant.
// ---------------------------------------------------------------------------------
// mode 0, Cin = 1, Cout = CO (BN folded, PReLU), NHWC (== NCHW) input, NHWC output: the
// thread's 9 reflect-gathered inputs, every output channel, staged through LDS so the
// workgroup's 256 pixels x CO channels (contiguous in NHWC) leave as coalesced 16-byte stores
template <int CO>
__global__ void __launch_bounds__(256) pm_cin1(PmConvArgs P) {
    __shared__ float Ws[CO * 9];
    __shared__ float Bs[CO];
    __shared__ float Ys[256 * (CO + 4)];
    for (int i = threadIdx.x; i < CO * 9; i += 256) Ws[i] = P.w[i];
    for (int i = threadIdx.x; i < CO; i += 256) Bs[i] = P.bias[i];
    __syncthreads();
    const int N = P.B * P.Ho * P.Wo;
    const int n0 = blockIdx.x * 256, n = n0 + threadIdx.x;
    if (n < N) {
        const int b = n / (P.Ho * P.Wo);
        const int r = n - b * P.Ho * P.Wo;
        const int oy = r / P.Wo, ox = r - oy * P.Wo;
        const float* __restrict__ xb = P.x + (size_t)b * P.Hin * P.Win;
        float xv[9];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                int iy = oy * P.sh + a - 1, ix = ox * P.sw + c - 1;
                iy = iy < 0 ? -iy : (iy >= P.Hin ? 2 * (P.Hin - 1) - iy : iy);
                ix = ix < 0 ? -ix : (ix >= P.Win ? 2 * (P.Win - 1) - ix : ix);
                xv[3 * a + c] = xb[(size_t)iy * P.Win + ix];
            }
#pragma unroll
        for (int co = 0; co < CO; ++co) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < 9; ++k) acc = fmaf(Ws[co * 9 + k], xv[k], acc);
            Ys[threadIdx.x * (CO + 4) + co] = pm_act(acc + Bs[co], P);
        }
    }
    __syncthreads();
    const int nv = min(256, N - n0);
    f32x4* __restrict__ yo = reinterpret_cast<f32x4*>(P.y + (size_t)n0 * CO);
    for (int i = threadIdx.x; i < nv * CO / 4; i += 256) {
        const int px = i / (CO / 4), q = i - px * (CO / 4);
        yo[i] = *reinterpret_cast<const f32x4*>(&Ys[px * (CO + 4) + 4 * q]);
    }
}

// mode 1 (ConvTranspose2d 3x3 stride 2), Cout = 1, NHWC input with CI channels: one thread per
// 2 x 2 output block (2qy + py, 2qx + px) -- the four parity classes, which together read only
// the input pixels (qy - {0,1}, qx - {0,1}), loaded once as 16-byte channel vectors -- then per
// class pm_conv's fma chain over k = ci * nt + t in its K slices, summed in pm_reduce's order.
// Output [B][1][Ho][Wo]
template <int CI>
__global__ void __launch_bounds__(256) pm_cout1(PmConvArgs P) {
    // the workgroup's input pixels (a contiguous NHWC range: its quads' rows qy-1 .. qy), staged
    // with coalesced 16-byte loads; pixel stride CI + 4 floats, so the 16-lane groups of a
    // ds_read_b128 (consecutive pixels) cover the 64 banks once.  Per-lane 16-byte global reads
    // of 128-byte pixels touched 64 cache lines per instruction: 64.6 us of the ~1.1 ms forward.
    constexpr int XS = CI + 4, XCAP = 384;
    __shared__ float Ws[4][4 * CI];
    __shared__ __attribute__((aligned(16))) float xs[XCAP * XS];
    for (int c = 0; c < 4; ++c) {
        const int K = CI * ((c >> 1) == 0 ? 2 : 1) * ((c & 1) == 0 ? 2 : 1);
        for (int i = threadIdx.x; i < K; i += 256) Ws[c][i] = P.w[P.woff[c] + i];
    }
    const int Hq = (P.Ho + 1) / 2, Wq = (P.Wo + 1) / 2;   // class (0, 0): the most blocks
    const int N = P.B * Hq * Wq, HWq = Hq * Wq, HWin = P.Hin * P.Win;
    const int n0 = blockIdx.x * 256, n1 = min(N - 1, n0 + 255);
    const int bf = n0 / HWq, qyf = (n0 - bf * HWq) / Wq, bl = n1 / HWq, qyl = (n1 - bl * HWq) / Wq;
    const long p_lo = (long)bf * HWin + (long)max(qyf - 1, 0) * P.Win;
    const long p_hi = (long)bl * HWin + (long)min(qyl, P.Hin - 1) * P.Win + P.Win - 1;
    const int cnt = (int)(p_hi - p_lo + 1);
    const bool staged = cnt <= XCAP;                    // workgroup-uniform
    if (staged) {
        const f32x4* src = reinterpret_cast<const f32x4*>(P.x + p_lo * CI);
        for (int i = threadIdx.x; i < cnt * (CI / 4); i += 256) {
            const int pix = i / (CI / 4), q = i - pix * (CI / 4);
            *reinterpret_cast<f32x4*>(xs + pix * XS + 4 * q) = src[i];
        }
    }
    __syncthreads();
    const int n = n0 + threadIdx.x;
    if (n >= N) return;
    const int b = n / HWq;
    const int r = n - b * HWq;
    const int qy = r / Wq, qx = r - qy * Wq;
    const float* __restrict__ xb = P.x + (size_t)b * CI * HWin;
    // xv[dy][dx] = input (qy - dy, qx - dx), zero outside
    f32x4 xv[2][2][CI / 4];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
            const int iy = qy - dy, ix = qx - dx;
            const bool ok = iy >= 0 && iy < P.Hin && ix >= 0 && ix < P.Win;
            const int pi = ok ? iy * P.Win + ix : 0;
            const int li = ok ? (int)((long)b * HWin + pi - p_lo) : 0;   // in [0, cnt) when ok
            const f32x4* src = staged ? reinterpret_cast<const f32x4*>(xs + li * XS)
                                      : reinterpret_cast<const f32x4*>(xb + (size_t)pi * CI);
#pragma unroll
            for (int q = 0; q < CI / 4; ++q) xv[dy][dx][q] = ok ? src[q] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    const int ks = P.ksplit > 1 ? P.ksplit : 1;
#pragma unroll
    for (int cls = 0; cls < 4; ++cls) {
        const int py = cls >> 1, px = cls & 1;
        const int oy = 2 * qy + py, ox = 2 * qx + px;
        if (oy >= P.Ho || ox >= P.Wo) continue;
        const int nty = py == 0 ? 2 : 1, ntx = px == 0 ? 2 : 1, nt = nty * ntx;
        const int K = CI * nt;
        const int nch = (K + 15) / 16, cps = (nch + ks - 1) / ks;
        float s = 0.f, acc = 0.f;
        for (int sl = 0; sl < ks; ++sl) {
            const int cb = sl * cps * 16 / nt, ce = min(CI, (sl + 1) * cps * 16 / nt);
            acc = 0.f;
#pragma unroll
            for (int ci = 0; ci < CI; ++ci) {
                if (ci < cb || ci >= ce) continue;
                // tap t = a * ntx + c reads input (qy - a [py = 0], qx - c [px = 0])
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (t >= nt) continue;
                    const int ta = ntx == 2 ? t >> 1 : t, tc = ntx == 2 ? t & 1 : 0;
                    const int dy = py == 0 ? ta : 0, dx = px == 0 ? tc : 0;
                    acc = fmaf(Ws[cls][ci * nt + t], xv[dy][dx][ci >> 2][ci & 3], acc);
                }
            }
            s += acc;
        }
        const float v = ks > 1 ? s : acc;
        P.y[((size_t)b * P.Ho + oy) * P.Wo + ox] = pm_act(v + P.bias[0], P);
    }
}
// pm_cout1 when its two K slices split every class at ci = CI / 2 (CI = 32, ksplit 2: the
// reference network at any batch): the input channels in two halves, slice h = channels of half h,
// so a workgroup stages and holds half the pixel vectors at a time -- 33 KB of LDS and ~100
// registers instead of 57 KB and 260 (four workgroups per CU instead of one, so one workgroup's
// staging round trip runs under another's FMA chains).  Per output the same fmaf chains and the
// same slice sum (0 + slice 0) + slice 1 as pm_cout1: bitwise the same results.
template <int CI>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) pm_cout1h(PmConvArgs P) {
    constexpr int CH = CI / 2, XS = CH + 4, XCAP = 384;
    __shared__ float Ws[4][4 * CI];
    __shared__ __attribute__((aligned(16))) float xs[XCAP * XS];
    for (int c = 0; c < 4; ++c) {
        const int K = CI * ((c >> 1) == 0 ? 2 : 1) * ((c & 1) == 0 ? 2 : 1);
        for (int i = threadIdx.x; i < K; i += 256) Ws[c][i] = P.w[P.woff[c] + i];
    }
    const int Hq = (P.Ho + 1) / 2, Wq = (P.Wo + 1) / 2;
    const int N = P.B * Hq * Wq, HWq = Hq * Wq, HWin = P.Hin * P.Win;
    const int n0 = blockIdx.x * 256, n1 = min(N - 1, n0 + 255);
    const int bf = n0 / HWq, qyf = (n0 - bf * HWq) / Wq, bl = n1 / HWq, qyl = (n1 - bl * HWq) / Wq;
    const long p_lo = (long)bf * HWin + (long)max(qyf - 1, 0) * P.Win;
    const long p_hi = (long)bl * HWin + (long)min(qyl, P.Hin - 1) * P.Win + P.Win - 1;
    const int cnt = (int)(p_hi - p_lo + 1);
    const bool staged = cnt <= XCAP;                    // workgroup-uniform
    const int n = n0 + threadIdx.x;
    const bool live = n < N;
    const int nn = live ? n : N - 1;
    const int b = nn / HWq;
    const int r = nn - b * HWq;
    const int qy = r / Wq, qx = r - qy * Wq;
    const float* __restrict__ xb = P.x + (size_t)b * CI * HWin;
    float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
        if (h) __syncthreads();                         // every lane is done with half 0
        if (staged) {
            const f32x4* src = reinterpret_cast<const f32x4*>(P.x + p_lo * CI + h * CH);
            for (int i = threadIdx.x; i < cnt * (CH / 4); i += 256) {
                const int pix = i / (CH / 4), q = i - pix * (CH / 4);
                *reinterpret_cast<f32x4*>(xs + pix * XS + 4 * q) = src[pix * (CI / 4) + q];
            }
        }
        __syncthreads();
        f32x4 xv[2][2][CH / 4];
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                const int iy = qy - dy, ix = qx - dx;
                const bool ok = iy >= 0 && iy < P.Hin && ix >= 0 && ix < P.Win;
                const int pi = ok ? iy * P.Win + ix : 0;
                const int li = ok ? (int)((long)b * HWin + pi - p_lo) : 0;
                const f32x4* src = staged ? reinterpret_cast<const f32x4*>(xs + li * XS)
                                          : reinterpret_cast<const f32x4*>(xb + (size_t)pi * CI + h * CH);
#pragma unroll
                for (int q = 0; q < CH / 4; ++q) xv[dy][dx][q] = ok ? src[q] : f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
        for (int cls = 0; cls < 4; ++cls) {
            const int py = cls >> 1, px = cls & 1;
            const int nty = py == 0 ? 2 : 1, ntx = px == 0 ? 2 : 1, nt = nty * ntx;
            float acc = 0.f;
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int ci = h * CH + c;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (t >= nt) continue;
                    const int ta = ntx == 2 ? t >> 1 : t, tc = ntx == 2 ? t & 1 : 0;
                    const int dy = py == 0 ? ta : 0, dx = px == 0 ? tc : 0;
                    acc = fmaf(Ws[cls][ci * nt + t], xv[dy][dx][c >> 2][c & 3], acc);
                }
            }
            part[cls] += acc;                           // (0 + slice 0) + slice 1, as pm_cout1
        }
    }
    if (!live) return;
#pragma unroll
    for (int cls = 0; cls < 4; ++cls) {
        const int oy = 2 * qy + (cls >> 1), ox = 2 * qx + (cls & 1);
        if (oy >= P.Ho || ox >= P.Wo) continue;
        P.y[((size_t)b * P.Ho + oy) * P.Wo + ox] = pm_act(part[cls] + P.bias[0], P);
    }
}
template __global__ void pm_cout1h<32>(PmConvArgs);
template __global__ void pm_cin1<32>(PmConvArgs);
template __global__ void pm_cout1<32>(PmConvArgs);

// split-K finish: y = act(sum of the K-slice partials in slice order + bias)
__global__ void __launch_bounds__(256) pm_reduce(PmConvArgs P) {
    const size_t per = (size_t)P.B * P.Cout * P.Ho * P.Wo;
    const size_t o = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= per) return;
    float s = 0.f;
    for (int q = 0; q < P.ksplit; ++q) s += P.part[(size_t)q * per + o];
    const int co = P.out_nhwc ? (int)(o % P.Cout) : (int)((o / ((size_t)P.Ho * P.Wo)) % P.Cout);
    P.y[o] = pm_act(s + P.bias[co], P);
}

// ---------------------------------------------------------------------------------
// The same layers on the matrix cores: v_mfma_f32_16x16x4_f32 (exact fp32, the fp32 peak).
// Activations NHWC, K ordered (tap, input channel) with Cin % 16 == 0, so one 16-wide K chunk
// is ONE input pixel's 16 consecutive channels: a lane's B fragment (column = output pixel,
// 4 consecutive K) is one 16-byte load, and the reflect (mode 0) / parity-class (mode 1) index
// arithmetic runs once per tap, not per element.  A comes pre-packed in fragment order (one
// 16-byte load per lane per M tile per chunk).  Within a chunk the four MFMA steps take K
// values 4q + s of lane group q (a permutation of the chunk, applied to A and B alike).
// Workgroup: 4 waves side by side over N, each MT x 16 rows by 32 columns (two N tiles); no
// LDS -- A is shared by the 4 waves through L1, B by the M tiles of a wave in registers.  The
// next chunk's fragments are in flight during the current chunk's MFMAs.  Per output the
// summation order is fixed by the layer's (geometry-only) K split: batch-invariant.
// ---------------------------------------------------------------------------------
// The K loop keeps the next chunk's fragments in flight under the current chunk's MFMAs only if
// the waitcnt pass can count them: no branch inside the loop (the mode is a template parameter,
// every load is unconditional -- invalid taps read a clamped in-range address and are zeroed after
// the load, the last prefetch re-reads the final chunk).  With the mode a runtime value and
// conditional loads, every wait in the loop was vmcnt(0): the prefetch waited for itself.
#ifndef AVC_PM_PF
#define AVC_PM_PF 1
#endif
// occupancy cap (amdgpu_waves_per_eu): off -- forcing 4 waves per SIMD (<= 128 VGPRs; the MT = 4 forms
// take 116-130 unconstrained) measured 291.7k vs 295.8k windows/s unconstrained
#ifndef AVC_PM_WPE
#define AVC_PM_WPE 0
#endif
#if AVC_PM_WPE
#define PM_MFMA_ATTR __attribute__((amdgpu_waves_per_eu(AVC_PM_WPE)))
#else
#define PM_MFMA_ATTR
#endif
template <int MT, int MODE, int NT>
__global__ void __launch_bounds__(256) PM_MFMA_ATTR pm_mfma(PmConvArgs P) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 15, q = lane >> 4;
    const int ks = P.ksplit > 1 ? P.ksplit : 1;
    const int cls = blockIdx.z / ks, slice = blockIdx.z - cls * ks;
    const int py = cls >> 1, px = cls & 1;
    const int nty = MODE == 1 ? (py == 0 ? 2 : 1) : 3;
    const int ntx = MODE == 1 ? (px == 0 ? 2 : 1) : 3;
    const int Hq = MODE == 1 ? (P.Ho - py + 1) / 2 : P.Ho;
    const int Wq = MODE == 1 ? (P.Wo - px + 1) / 2 : P.Wo;
    const int N = P.B * Hq * Wq;
    const int nbase = blockIdx.x * 64 * NT;
    if (nbase >= N) return;                     // (uniform: class grids are padded to the largest)
    const int ccpt = P.Cin >> 4;                // K chunks per tap
    const int nchunk = nty * ntx * ccpt;
    const int cps = (nchunk + ks - 1) / ks;
    const int kc0 = slice * cps, kc1 = min(nchunk, kc0 + cps);
    const int mt0 = blockIdx.y * MT;            // first M tile of this workgroup
    const int nmt = (P.Cout + 15) >> 4;
    // this lane's two output columns (an invalid column computes on column 0 and is not stored)
    int cb[NT], cy[NT], cx[NT];
    bool cv[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int n = nbase + 16 * NT * w + 16 * j + c;
        cv[j] = n < N;
        const int nn = cv[j] ? n : 0;
        cb[j] = nn / (Hq * Wq);
        const int r = nn - cb[j] * Hq * Wq;
        cy[j] = r / Wq;
        cx[j] = r - cy[j] * Wq;
    }
    const f32x4* __restrict__ Aw = reinterpret_cast<const f32x4*>(P.wm + P.wmoff[cls]);
    auto load_a = [&](int kc, f32x4 (&a)[MT]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int mt = min(mt0 + i, nmt - 1);
            a[i] = Aw[((size_t)mt * nchunk + kc) * 64 + lane];
        }
    };
    auto load_b = [&](int kc, f32x4 (&b)[NT]) __attribute__((always_inline)) {
        const int tap = kc / ccpt, ci = ((kc - tap * ccpt) << 4) + 4 * q;
        const int a = tap / ntx, bb = tap - a * ntx;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            int iy, ix;
            bool ok = true;
            if constexpr (MODE == 0) {
                iy = cy[j] * P.sh + a - 1;
                ix = cx[j] * P.sw + bb - 1;
                iy = iy < 0 ? -iy : (iy >= P.Hin ? 2 * (P.Hin - 1) - iy : iy);
                ix = ix < 0 ? -ix : (ix >= P.Win ? 2 * (P.Win - 1) - ix : ix);
            } else {
                iy = py == 0 ? cy[j] - a : cy[j];
                ix = px == 0 ? cx[j] - bb : cx[j];
                ok = iy >= 0 && iy < P.Hin && ix >= 0 && ix < P.Win;
                iy = min(max(iy, 0), P.Hin - 1);
                ix = min(max(ix, 0), P.Win - 1);
            }
            const f32x4 v = *reinterpret_cast<const f32x4*>(P.x + (((size_t)cb[j] * P.Hin + iy) * P.Win + ix) * P.Cin + ci);
            b[j] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mma = [&](const f32x4 (&a)[MT], const f32x4 (&b)[NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
    };
    // the epilogue's biases, loaded now so their round trip is hidden by the K loop
    f32x4 bias4[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
        bias4[i] = *reinterpret_cast<const f32x4*>(P.bias + min((mt0 + i) * 16 + 4 * q, P.Cout - 4));
    if (kc0 < kc1) {   // (uniform; an empty K slice stores its zeros like any other)
        // ring of PF + 1 chunk buffers, PF chunks in flight ahead of the one being multiplied;
        // prefetch indices clamped to the slice (the last rounds re-read its final chunk)
        constexpr int PF = AVC_PM_PF, NB = PF + 1;
        f32x4 ra[NB][MT], rb[NB][NT];
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            load_a(min(kc0 + p, kc1 - 1), ra[p]);
            load_b(min(kc0 + p, kc1 - 1), rb[p]);
        }
        int kc = kc0;
        for (; kc + NB <= kc1; kc += NB) {
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const int kn = min(kc + u + PF, kc1 - 1);
                load_a(kn, ra[(u + PF) % NB]);
                load_b(kn, rb[(u + PF) % NB]);
                mma(ra[u], rb[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < PF; ++u)   // the last kc1 - kc <= PF chunks, already in flight
            if (kc + u < kc1) mma(ra[u], rb[u]);
    }
    // epilogue: rows 4q + r of M tile i = 4 consecutive output channels of column (j, c): NHWC
    const size_t per = (size_t)P.B * P.Cout * P.Ho * P.Wo;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        if (!cv[j]) continue;
        const int oy = MODE == 1 ? 2 * cy[j] + py : cy[j];
        const int ox = MODE == 1 ? 2 * cx[j] + px : cx[j];
        const size_t pix = ((size_t)cb[j] * P.Ho + oy) * P.Wo + ox;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int co = (mt0 + i) * 16 + 4 * q;
            if (co >= P.Cout) continue;
            const size_t o = pix * P.Cout + co;
            if (ks > 1) {
                *reinterpret_cast<f32x4*>(P.part + (size_t)slice * per + o) = acc[i][j];
            } else {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = pm_act(acc[i][j][r] + bias4[i][r], P);
                *reinterpret_cast<f32x4*>(P.y + o) = v;
            }
        }
    }
}
#define AVC_PM_INST(MT, NT)                                    \
    template __global__ void pm_mfma<MT, 0, NT>(PmConvArgs);   \
    template __global__ void pm_mfma<MT, 1, NT>(PmConvArgs);
AVC_PM_INST(2, 1)
AVC_PM_INST(2, 2)
AVC_PM_INST(4, 1)
AVC_PM_INST(4, 2)
AVC_PM_INST(4, 4)
#undef AVC_PM_INST

// ---- VSMask protect loop (/root/reference/vsmask.py:177-208) ----------------------------
// The reference walks start = 0, S, 2S, ... < T - W, feeds mel[..., start:start+W] (always the
// UNPERTURBED mel) to the predictor and adds its output at frames [start+W, start+W+Wo).  The
// windows are independent, so they are gathered into one batch (vsm_gather), predicted by one
// batched PredictiveModel forward, and summed per element in the reference's order by
// vsm_combine: acc = mel (+ header) (+ window 0) (+ window 1) ...; pert = acc - mel; band clamp
// (utils/audio.py:77-116); out = mel + pert.  Every element repeats the reference's fp32 adds
// in the same order, so the combine is bit-exact given the same predictor outputs.

__global__ void __launch_bounds__(256) vsm_gather(VsmArgs A) {
    const size_t n = (size_t)A.B * A.nw * A.F * A.W;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const int j = (int)(i % A.W);
        const size_t r = i / A.W;
        const int f = (int)(r % A.F);
        const size_t bk = r / A.F;
        const int k = (int)(bk % A.nw);
        const size_t b = bk / A.nw;
        A.win[i] = A.mel[(b * A.F + f) * A.T + (size_t)k * A.S + j];
    }
}

__global__ void __launch_bounds__(256) vsm_combine(VsmArgs A) {
    const size_t n = (size_t)A.B * A.F * A.T;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const int t = (int)(i % A.T);
        const size_t r = i / A.T;
        const int f = (int)(r % A.F);
        const size_t b = r / A.F;
        const float m = A.mel[i];
        float acc = m;
        if (A.header && t < A.Th) acc += A.header[(size_t)f * A.Th + t];
        if (A.mode == 1) {
            A.out[i] = fminf(fmaxf(acc, -1.f), 1.f);
            continue;
        }
        if (A.mode == 2) {   // apply_weighted_constraint (utils/audio.py:77-116) of the input itself
            const float e = f < A.low_end ? A.eps1 : (f < A.high_start ? A.eps2 : A.eps3);
            A.out[i] = fminf(fmaxf(m, -e), e);
            continue;
        }
        if (A.nw > 0 && f < A.rows && t >= A.W) {
            // windows k with k*S + W <= t < k*S + W + Wo, ascending k (the reference's order)
            const int u = t - A.W;
            int klo = u - A.Wo + 1;
            klo = klo <= 0 ? 0 : (klo + A.S - 1) / A.S;
            const int khi = min(A.nw - 1, u / A.S);
            for (int k = klo; k <= khi; ++k)
                acc += A.y[(((b * A.nw + k) * A.Ho) + f) * (size_t)A.Wo + (u - k * A.S)];
        }
        const float e = f < A.low_end ? A.eps1 : (f < A.high_start ? A.eps2 : A.eps3);
        const float p = fminf(fmaxf(acc - m, -e), e);
        A.out[i] = m + p;
    }
}

}  // namespace avc
