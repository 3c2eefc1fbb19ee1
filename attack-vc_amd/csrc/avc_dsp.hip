// Mel front / back end of the reference (data_utils.py:16-197; flavor 1: utils/audio.py:8-76,
// the torchaudio MelSpectrogram / InverseMelScale / GriffinLim of the VSMask converter) on gfx950:
//   dsp_wav2mel    file2mel after load + trim (data_utils.py:99-118): pre-emphasis,
//                  centered STFT, |X|, mel projection, dB, clip (+ normalize, 35-47)
//   dsp_mel2mag    mel2wav's front (150-157): (denormalize,) clip, dB^-1, inv_mel_matrix
//   dsp_gl_frames  one Griffin-Lim projection (168-197) per frame pair: STFT of the
//                  current signal, X = S * est / max(1e-8, |est|), inverse FFT x window
//   dsp_ola        librosa.istft's overlap-add / window-sum-square / center trim
//   dsp_deemph     lfilter([1], [1, -preemph]) (161) as a one-pass tiled affine scan
// STFT frames are the bandwidth unit: every frame kernel is one workgroup per PAIR of
// real frames, packed as the real / imaginary parts of one complex N-point FFT
// (Stockham radix-8 passes in LDS, natural order, twiddles staged in LDS) and separated with
// the conjugate-symmetry identities; the inverse transform of two Hermitian spectra is
// the same FFT run on conj(X0 + i X1).  HBM traffic per Griffin-Lim iteration and frame:
// the frame written once (N floats) and read by dsp_ola, the signal read back through L2.
#include <hip/hip_runtime.h>

#include "avc_kernels.h"
#include "avc_device.h"

namespace avc {

namespace {
constexpr int DSP_THREADS = 256;
constexpr int DSP_MT = 8;          // dsp_mel2mag: frames per workgroup

__device__ __forceinline__ int zp(int i) { return dsp_zp(i); }
__device__ __forceinline__ int tp(int i) { return dsp_tp(i); }
constexpr int zlen(int N) { return dsp_zlen(N); }

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// Forward FFT of Z[N] in place, natural order in and out: Stockham auto-sort passes of radix 8
// (then one of 4 or 2), each thread one or two butterflies per pass -- its R inputs at stride
// N/R (consecutive across lanes: conflict-free reads), the twiddles W_{R Ns}^{k m} from the
// padded table (W^(e + N/2) = -W^e), an in-register radix-R DFT, a barrier, the R outputs to
// (j / Ns) R Ns + j % Ns + r Ns, a barrier.  2048 points: 4 passes of 16-22 LDS accesses per
// thread (the radix-4 DIT with bit-reversed input took 6 passes and ~130, with 8-32-way
// conflicted strided twiddle and butterfly accesses: 1.9 bank-conflict cycles per LDS cycle).
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }   // -i a

template <int R>
__device__ __forceinline__ void dft_r(float2 (&a)[R]) {
    if constexpr (R == 2) {
        const float2 t = a[0];
        a[0] = cadd(t, a[1]);
        a[1] = csub(t, a[1]);
    } else if constexpr (R == 4) {
        const float2 t0 = cadd(a[0], a[2]), t1 = csub(a[0], a[2]), t2 = cadd(a[1], a[3]),
                     t3 = mul_mi(csub(a[1], a[3]));
        a[0] = cadd(t0, t2);
        a[1] = cadd(t1, t3);
        a[2] = csub(t0, t2);
        a[3] = csub(t1, t3);
    } else {   // R == 8: one radix-2 DIF stage (W8^m on the differences), two radix-4 DFTs
        constexpr float S2 = 0.70710678118654752f;
        float2 u[4], v[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            u[m] = cadd(a[m], a[m + 4]);
            v[m] = csub(a[m], a[m + 4]);
        }
        v[1] = make_float2((v[1].x + v[1].y) * S2, (v[1].y - v[1].x) * S2);
        v[2] = mul_mi(v[2]);
        v[3] = make_float2((v[3].y - v[3].x) * S2, -(v[3].x + v[3].y) * S2);
        dft_r<4>(u);
        dft_r<4>(v);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            a[2 * r] = u[r];
            a[2 * r + 1] = v[r];
        }
    }
}

template <int R, int LR, int LOGN, int LOGNS>
__device__ __forceinline__ void fft_pass(float2* Z, const float2* TW) {
    constexpr int N = 1 << LOGN, NB = N >> LR, NS = 1 << LOGNS, SH = LOGN - LOGNS - LR;
    constexpr int U = NB > DSP_THREADS ? NB / DSP_THREADS : 1;   // butterflies per thread
    float2 a[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int j = threadIdx.x + DSP_THREADS * u;
        if (NB < DSP_THREADS && j >= NB) continue;
        const int k = j & (NS - 1);
#pragma unroll
        for (int m = 0; m < R; ++m) a[u][m] = Z[zp(j + m * NB)];
#pragma unroll
        for (int m = 1; m < R; ++m) {
            const int e = (k * m) << SH;
            float2 t = TW[tp(e & (N / 2 - 1))];
            if (e >= N / 2) t = make_float2(-t.x, -t.y);
            a[u][m] = cmul(a[u][m], t);
        }
        dft_r<R>(a[u]);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int j = threadIdx.x + DSP_THREADS * u;
        if (NB < DSP_THREADS && j >= NB) continue;
        const int idx = ((j >> LOGNS) << (LOGNS + LR)) + (j & (NS - 1));
#pragma unroll
        for (int r = 0; r < R; ++r) Z[zp(idx + r * NS)] = a[u][r];
    }
    __syncthreads();
}

// radix 8 while three or more factors of two remain, then one pass of 4 or 2 (compile-time
// n_fft: each kernel is instantiated per log2 n_fft, so the registers are those of its passes)
template <int LOGN, int LOGNS = 0>
__device__ __forceinline__ void fft_lds(float2* Z, const float2* TW) {
    if constexpr (LOGNS < LOGN) {
        constexpr int REM = LOGN - LOGNS, LR = REM >= 3 ? 3 : REM;
        fft_pass<1 << LR, LR, LOGN, LOGNS>(Z, TW);
        fft_lds<LOGN, LOGNS + LR>(Z, TW);
    }
}

// sum over the 16 lanes of a row, every lane receiving it (DPP: rotate 8, 4 in the row, quad swaps 2, 1)
template <int CTRL>
__device__ __forceinline__ float dsp_dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float dsp_row16_sum(float v) {
    v += dsp_dpp<0x128>(v);
    v += dsp_dpp<0x124>(v);
    v += dsp_dpp<0x4E>(v);
    v += dsp_dpp<0xB1>(v);
    return v;
}

// numpy.pad(mode='reflect') index into [0, L) (no edge repeat; any overhang), or -1 (constant)
__device__ __forceinline__ int pad_index(int s, int L, int pad_mode) {
    if (s >= 0 && s < L) return s;
    if (pad_mode == 1) return -1;
    if (L == 1) return 0;
    const int period = 2 * (L - 1);
    s %= period;
    if (s < 0) s += period;
    return s >= L ? period - s : s;
}

// X0 / X1 of the two real frames packed in Z (k in [0, N/2])
__device__ __forceinline__ void split_pair(const float2* Z, int N, int k, float2& X0, float2& X1) {
    const float2 a = Z[zp(k & (N - 1))], c = Z[zp((N - k) & (N - 1))];
    X0 = make_float2(0.5f * (a.x + c.x), 0.5f * (a.y - c.y));
    X1 = make_float2(0.5f * (a.y + c.y), -0.5f * (a.x - c.x));
}

__device__ __forceinline__ void stage_twiddles(float2* TW, const float* tw, int N) {
    for (int k = threadIdx.x; k < (N >> 1); k += DSP_THREADS)
        TW[tp(k)] = reinterpret_cast<const float2*>(tw)[k];
}
}  // namespace

// grid (ceil(Tf / 2), B): frames 2p, 2p + 1 of utterance b -> mel [B][Tf][n_mels] or
// [B][n_mels][Tf] (transpose), normalized with (mean, std) when given
template <int LOGN>
__global__ void __launch_bounds__(DSP_THREADS) dsp_wav2mel(DspArgs A) {
    extern __shared__ float2 dsm[];
    constexpr int N = 1 << LOGN;
    const int F = A.F, Tf = A.Tf, L = A.L, b = blockIdx.y;
    float2* Z = dsm;                 // [zlen(N)]
    float2* TW = Z + zlen(N);        // [dsp_twlen(N)]
    float* MAG = reinterpret_cast<float*>(TW + dsp_twlen(N));   // [2][F]
    stage_twiddles(TW, A.twiddle, N);
    const int t0 = 2 * blockIdx.x, t1 = t0 + 1;
    const float* x = A.x + (size_t)b * L;
    const float a = A.preemph;
    auto sample = [&](int t, int n) -> float {
        if (t >= Tf) return 0.f;
        const int s = pad_index(t * A.hop + n - N / 2, L, A.pad_mode);
        if (s < 0) return 0.f;
        // wav = append(wav[0], wav[1:] - preemph * wav[:-1]) (data_utils.py:101)
        return s == 0 ? x[0] : x[s] - a * x[s - 1];
    };
    for (int n = threadIdx.x; n < N; n += DSP_THREADS) {
        const float w = A.window[n];
        Z[zp(n)] = make_float2(sample(t0, n) * w, sample(t1, n) * w);
    }
    __syncthreads();
    fft_lds<LOGN>(Z, TW);
    for (int k = threadIdx.x; k < F; k += DSP_THREADS) {
        float2 X0, X1;
        split_pair(Z, N, k, X0, X1);
        const float p0 = X0.x * X0.x + X0.y * X0.y, p1 = X1.x * X1.x + X1.y * X1.y;
        MAG[k] = A.flavor ? p0 : sqrtf(p0);            // torchaudio MelSpectrogram: power 2
        MAG[F + k] = A.flavor ? p1 : sqrtf(p1);
    }
    __syncthreads();
    // one (frame, mel) dot product per 16-lane row: lane l sums the filter's bins f = lo + l, lo + l + 16, ..
    // (coalesced reads of the filter row and of MAG), then a fixed-order DPP reduction over the row --
    // round 4 ran each dot product serially in one thread (up to ~60 dependent L2 loads for the top mels:
    // the kernel's critical path)
    const int l16 = threadIdx.x & 15;
    for (int idx = threadIdx.x >> 4; idx < 2 * A.n_mels; idx += DSP_THREADS / 16) {
        const int fr = idx / A.n_mels, m = idx - fr * A.n_mels, t = t0 + fr;
        const float* row = A.mel_basis + (size_t)m * F;
        const float* mg = MAG + fr * F;
        float s = 0.f;
        for (int f = A.mel_range[2 * m] + l16; f < A.mel_range[2 * m + 1]; f += 16) s = fmaf(row[f], mg[f], s);
        s = dsp_row16_sum(s);
        if (t >= Tf || l16 != 0) continue;
        float v;
        if (A.flavor) {
            v = log10f(fmaxf(s, 1e-5f));                   // log10(clamp(mel, 1e-5)) (utils/audio.py:55-56)
        } else {
            // 20 log10(max(1e-5, mel)); clip((mel - ref_db + max_db) / max_db, 1e-8, 1) (111-112)
            v = 20.f * log10f(fmaxf(1e-5f, s));
            v = fminf(fmaxf((v - A.ref_db + A.max_db) / A.max_db, 1e-8f), 1.f);
            if (A.mean) v = (v - A.mean[m]) / A.std[m];    // normalize (data_utils.py:35-47)
        }
        const size_t o = A.transpose ? ((size_t)b * A.n_mels + m) * Tf + t : ((size_t)b * Tf + t) * A.n_mels + m;
        A.mel_out[o] = v;
    }
}

// grid (Tf, B): spect_out[b][t][f] = sum_m inv_mel[f][m] * 10^((clip(mel, 0, 1) * max_db
// - max_db + ref_db) * 0.05)  (data_utils.py:150-157), mel denormalized first when given
// DSP_MT frames per workgroup: each inv_mel element read from L2 serves DSP_MT frames (one frame
// per workgroup re-read the whole [n_mels][F] matrix per frame: 0.43 ms per call at B=256)
__global__ void __launch_bounds__(DSP_THREADS) dsp_mel2mag(DspArgs A) {
    extern __shared__ float2 dsm[];
    float* lin = reinterpret_cast<float*>(dsm);            // [DSP_MT][n_mels]
    const int t0 = blockIdx.x * DSP_MT, b = blockIdx.y, nm = A.n_mels, Tf = A.Tf;
    for (int idx = threadIdx.x; idx < DSP_MT * nm; idx += DSP_THREADS) {
        const int tt = idx / nm, m = idx - tt * nm, t = min(t0 + tt, Tf - 1);
        float v = A.mel_in[A.transpose ? ((size_t)b * nm + m) * Tf + t : ((size_t)b * Tf + t) * nm + m];
        if (A.flavor) {                                    // pow(10, mel) (utils/audio.py:70)
            lin[idx] = exp10f(v);
            continue;
        }
        if (A.mean) v = v * A.std[m] + A.mean[m];          // denormalize (data_utils.py:50-62)
        v = fminf(fmaxf(v, 0.f), 1.f) * A.max_db - A.max_db + A.ref_db;
        lin[idx] = exp10f(v * 0.05f);
    }
    __syncthreads();
    for (int f = threadIdx.x; f < A.F; f += DSP_THREADS) {
        // inv_mel stored transposed [n_mels][F]: consecutive threads read consecutive bins
        float s[DSP_MT];
#pragma unroll
        for (int tt = 0; tt < DSP_MT; ++tt) s[tt] = 0.f;
        for (int m = 0; m < nm; ++m) {
            const float w = A.inv_mel[(size_t)m * A.F + f];
#pragma unroll
            for (int tt = 0; tt < DSP_MT; ++tt) s[tt] = fmaf(w, lin[tt * nm + m], s[tt]);
        }
        // flavor 1: InverseMelScale's relu of the least-squares solution, then GriffinLim's
        // specgram.pow(1 / power) (power 2): the magnitude
#pragma unroll
        for (int tt = 0; tt < DSP_MT; ++tt)
            if (t0 + tt < Tf)
                A.spect_out[((size_t)b * Tf + t0 + tt) * A.F + f] = A.flavor ? sqrtf(fmaxf(s[tt], 0.f)) : s[tt];
    }
}

// grid (ceil(F / 256), Tf, B): [B][F][Tf] (the reference's magnitude layout) -> [B][Tf][F]
__global__ void __launch_bounds__(DSP_THREADS) dsp_transpose(DspArgs A) {
    const int f = blockIdx.x * DSP_THREADS + threadIdx.x, t = blockIdx.y, b = blockIdx.z;
    if (f < A.F) A.spect_out[((size_t)b * A.Tf + t) * A.F + f] = A.spect[((size_t)b * A.F + f) * A.Tf + t];
}

// grid (ceil(Tf / 2), B): one Griffin-Lim step for frames 2p, 2p + 1 (data_utils.py:190-195):
//   init: X = S;  else X = S * est / max(1e-8, |est|), est = STFT(y) (center, pad_mode)
//   frames[t] = window * irfft(X[:, t])
template <int LOGN>
__global__ void __launch_bounds__(DSP_THREADS) dsp_gl_frames(DspArgs A) {
    // bins per thread: k = tid + 256 i, i < KPT covers F = N/2 + 1;
    // both spectra stay in registers between the forward and inverse transforms, so the
    // LDS holds only the FFT buffer and the twiddles (more workgroups per CU)
    constexpr int N = 1 << LOGN;
    constexpr int KPT = (N / 2 + 1 + DSP_THREADS - 1) / DSP_THREADS;
    extern __shared__ float2 dsm[];
    const int F = A.F, Tf = A.Tf, b = blockIdx.y, tid = threadIdx.x;
    float2* Z = dsm;                 // [zlen(N)]
    float2* TW = Z + zlen(N);        // [dsp_twlen(N)]
    const int t0 = 2 * blockIdx.x, t1 = t0 + 1;
    const bool has1 = t1 < Tf;
    const float* S0 = A.spect + ((size_t)b * Tf + t0) * F;
    const float* S1 = has1 ? S0 + F : S0;
    // target magnitudes first: their loads are in flight during the gather and forward FFT
    float m0[KPT], m1[KPT];
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
        const int k = tid + DSP_THREADS * i;
        m0[i] = k < F ? S0[k] : 0.f;
        m1[i] = (k < F && has1) ? S1[k] : 0.f;
    }
    float2 X0[KPT], X1[KPT];
    // flavor 1: the previous rebuilt spectra of the two frames
    float2* P0 = A.flavor ? reinterpret_cast<float2*>(A.tprev) + ((size_t)b * Tf + t0) * F : nullptr;
    float2* P1 = A.flavor ? P0 + F : nullptr;
    if (A.init) {
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
            const int k = tid + DSP_THREADS * i;
            X0[i] = make_float2(m0[i], 0.f);
            X1[i] = make_float2(m1[i], 0.f);
            if (A.flavor && k < F) {
                // X = |S| * angles0 (torch.rand complex: NOT unit modulus); tprev = 0
                if (A.angles0) {
                    const float2* a0 = reinterpret_cast<const float2*>(A.angles0) + ((size_t)b * F + k) * Tf;
                    const float2 u = a0[t0], v = has1 ? a0[t1] : make_float2(0.f, 0.f);
                    X0[i] = make_float2(m0[i] * u.x, m0[i] * u.y);
                    X1[i] = make_float2(m1[i] * v.x, m1[i] * v.y);
                }
                P0[k] = make_float2(0.f, 0.f);
                if (has1) P1[k] = make_float2(0.f, 0.f);
            }
        }
        stage_twiddles(TW, A.twiddle, N);
    } else {
        const float* y = A.y + (size_t)b * A.L;
        if (A.vec4) {   // hop, L and y 16-byte aligned: four samples per 16-byte load off the edges
            for (int n = 4 * tid; n < N; n += 4 * DSP_THREADS) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(A.window + n);
                const int b0 = t0 * A.hop + n - N / 2, b1 = t1 * A.hop + n - N / 2;
                f32x4 v0, v1;
                if (b0 >= 0 && b0 + 3 < A.L) {
                    v0 = *reinterpret_cast<const f32x4*>(y + b0);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int s0 = pad_index(b0 + e, A.L, A.pad_mode);
                        v0[e] = s0 < 0 ? 0.f : y[s0];
                    }
                }
                if (!has1) {
                    v1 = f32x4{0.f, 0.f, 0.f, 0.f};
                } else if (b1 >= 0 && b1 + 3 < A.L) {
                    v1 = *reinterpret_cast<const f32x4*>(y + b1);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int s1 = pad_index(b1 + e, A.L, A.pad_mode);
                        v1[e] = s1 < 0 ? 0.f : y[s1];
                    }
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) Z[zp(n + e)] = make_float2(v0[e] * w[e], v1[e] * w[e]);
            }
        } else {
            for (int n = tid; n < N; n += DSP_THREADS) {
                const float w = A.window[n];
                const int s0 = pad_index(t0 * A.hop + n - N / 2, A.L, A.pad_mode);
                const int s1 = pad_index(t1 * A.hop + n - N / 2, A.L, A.pad_mode);
                const float v0 = s0 < 0 ? 0.f : y[s0];
                const float v1 = (!has1 || s1 < 0) ? 0.f : y[s1];
                Z[zp(n)] = make_float2(v0 * w, v1 * w);
            }
        }
        stage_twiddles(TW, A.twiddle, N);
        __syncthreads();
        fft_lds<LOGN>(Z, TW);
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
            const int k = tid + DSP_THREADS * i;
            X0[i] = X1[i] = make_float2(0.f, 0.f);
            if (k < F) {
                float2 E0, E1;
                split_pair(Z, N, k, E0, E1);
                if (A.flavor) {
                    // torchaudio griffinlim: angles = rebuilt - alpha * tprev; angles /= |angles| +
                    // 1e-16; tprev = rebuilt; X = |S| * angles
                    const float al = A.momentum / (1.f + A.momentum);
                    const float2 q0 = P0[k], q1 = has1 ? P1[k] : make_float2(0.f, 0.f);
                    const float2 a0 = make_float2(E0.x - al * q0.x, E0.y - al * q0.y);
                    const float2 a1 = make_float2(E1.x - al * q1.x, E1.y - al * q1.y);
                    const float s0 = m0[i] / (sqrtf(a0.x * a0.x + a0.y * a0.y) + 1e-16f);
                    const float s1 = has1 ? m1[i] / (sqrtf(a1.x * a1.x + a1.y * a1.y) + 1e-16f) : 0.f;
                    X0[i] = make_float2(a0.x * s0, a0.y * s0);
                    X1[i] = make_float2(a1.x * s1, a1.y * s1);
                    P0[k] = E0;
                    if (has1) P1[k] = E1;
                } else {
                    const float s0 = m0[i] / fmaxf(1e-8f, sqrtf(E0.x * E0.x + E0.y * E0.y));
                    const float s1 = has1 ? m1[i] / fmaxf(1e-8f, sqrtf(E1.x * E1.x + E1.y * E1.y)) : 0.f;
                    X0[i] = make_float2(E0.x * s0, E0.y * s0);
                    X1[i] = make_float2(E1.x * s1, E1.y * s1);
                }
            }
        }
    }
    __syncthreads();   // every read of the forward spectrum is done
    // conj(X0 + i X1) over the full Hermitian extension (bins k and N - k from the same
    // thread), in natural order; irfft ignores the imaginary parts of the DC and Nyquist bins
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
        const int k = tid + DSP_THREADS * i;
        if (k < F) {
            float2 a = X0[i], c = X1[i];
            if (k == 0 || k == N / 2) a.y = c.y = 0.f;
            // Z = X0 + i X1 = (X0.x - X1.y) + i (X0.y + X1.x); store conj(Z)
            Z[zp(k)] = make_float2(a.x - c.y, -(a.y + c.x));
            if (k != 0 && k != N / 2)   // bin N - k: conj(X0) + i conj(X1)
                Z[zp(N - k)] = make_float2(a.x + c.y, a.y - c.x);
        }
    }
    __syncthreads();
    fft_lds<LOGN>(Z, TW);
    // z = conj(FFT(conj Z)) / N: frame0 = Re z, frame1 = Im z
    const float invN = 1.f / (float)N;
    float* f0 = A.frames + ((size_t)b * Tf + t0) * N;
    for (int n = 4 * tid; n < N; n += 4 * DSP_THREADS) {   // N >= 16: four per thread, 16-byte stores
        f32x4 w = *reinterpret_cast<const f32x4*>(A.window + n), o0, o1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float2 z = Z[zp(n + e)];
            w[e] = w[e] * invN;
            o0[e] = z.x * w[e];
            o1[e] = -z.y * w[e];
        }
        *reinterpret_cast<f32x4*>(f0 + n) = o0;
        if (has1) *reinterpret_cast<f32x4*>(f0 + N + n) = o1;
    }
}

// grid (ceil(Ly / 256)): wss[j] = sum over the frames t covering s = j + N/2 of window[s - t*hop]^2,
// once per call (the same sum, in the same order, that dsp_ola computed per sample and iteration)
__global__ void __launch_bounds__(DSP_THREADS) dsp_wss(DspArgs A) {
    const int j = blockIdx.x * DSP_THREADS + threadIdx.x;
    if (j >= A.Ly) return;
    const int N = A.N, hop = A.hop, s = j + N / 2;
    const int tlo = s - N + 1 <= 0 ? 0 : (s - N + hop) / hop, thi = min(A.Tf - 1, s / hop);
    float wss = 0.f;
    for (int t = tlo; t <= thi; ++t) {
        const float w = A.window[s - t * hop];
        wss += w * w;
    }
    A.wss[j] = wss;
}

// grid (ceil(Ly / 1024), B) when hop % 4 == 0: four consecutive samples per thread.  With N/2 and
// hop multiples of 4, the four samples' positions n..n+3 in a frame are all inside it or all
// outside, so each covering frame is one 16-byte load; per sample the frames are summed in the
// same (ascending) order as dsp_ola, and divided by the precomputed window sum-square.
__global__ void __launch_bounds__(DSP_THREADS) dsp_ola4(DspArgs A) {
    const int j = 4 * (blockIdx.x * DSP_THREADS + threadIdx.x), b = blockIdx.y;
    if (j >= A.Ly) return;
    const int N = A.N, hop = A.hop, s = j + N / 2;
    const int tlo = s - N + 4 <= 0 ? 0 : (s - N + 3 + hop) / hop, thi = min(A.Tf - 1, s / hop);
    const float* fr = A.frames + (size_t)b * A.Tf * N;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int t = tlo; t <= thi; ++t) acc += *reinterpret_cast<const f32x4*>(fr + (size_t)t * N + (s - t * hop));
    const f32x4 w = *reinterpret_cast<const f32x4*>(A.wss + j);
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = w[e] > 1.17549435e-38f ? acc[e] / w[e] : acc[e];
    *reinterpret_cast<f32x4*>(A.y + (size_t)b * A.Ly + j) = y;
}

// grid (ceil(Ly / 256), B): y[j] = sum_t frames[t][s - t*hop] / wss[s], s = j + N/2
// (librosa.istft, center=True, length=None: Ly = hop * (Tf - 1))
__global__ void __launch_bounds__(DSP_THREADS) dsp_ola(DspArgs A) {
    const int j = blockIdx.x * DSP_THREADS + threadIdx.x, b = blockIdx.y;
    if (j >= A.Ly) return;
    const int N = A.N, hop = A.hop, s = j + N / 2;
    const int tlo = s - N + 1 <= 0 ? 0 : (s - N + hop) / hop, thi = min(A.Tf - 1, s / hop);
    const float* fr = A.frames + (size_t)b * A.Tf * N;
    float acc = 0.f, wss = 0.f;
    // independent frame loads: unrolled so several are in flight per thread (the sum
    // stays in frame order, like librosa's sequential overlap-add)
#pragma unroll 8
    for (int t = tlo; t <= thi; ++t) {
        const int n = s - t * hop;
        acc += fr[(size_t)t * N + n];
        const float w = A.window[n];
        wss += w * w;
    }
    A.y[(size_t)b * A.Ly + j] = wss > 1.17549435e-38f ? acc / wss : acc;
}

// grid (B), 1024 threads: wav = lfilter([1], [1, -a], y) in ONE pass over HBM.  Tiles of
// 1024 x DE samples are staged through LDS with coalesced loads; thread t runs the
// recurrence over its DE consecutive samples from zero (affine map c -> e + a^DE c), an
// inclusive scan composes the maps across threads (fixed order: deterministic), the tile's
// carry enters from the previous tile, and the finished samples leave with coalesced stores.
constexpr int DE = 8;
__global__ void __launch_bounds__(1024) dsp_deemph(DspArgs A) {
    __shared__ float Ts[1024 * DE + 1024 * DE / 32];   // tile, one pad float per 32 (stride-DE reads)
    __shared__ float Ps[1024], Es[1024];
    const int b = blockIdx.x, tid = threadIdx.x, Ly = A.Ly;
    const float a = A.preemph;
    const float* y = A.y + (size_t)b * Ly;
    float* w = A.wav + (size_t)b * Ly;
    auto tp = [](int i) { return i + (i >> 5); };
    float aD = 1.f;
    for (int i = 0; i < DE; ++i) aD *= a;
    float carry = 0.f;   // wav[tile start - 1]
    for (int t0 = 0; t0 < Ly; t0 += 1024 * DE) {
        const int n = min(1024 * DE, Ly - t0);
#pragma unroll
        for (int i = 0; i < DE; ++i) {
            const int k = tid + 1024 * i;
            Ts[tp(k)] = k < n ? y[t0 + k] : 0.f;
        }
        __syncthreads();
        float e = 0.f;
#pragma unroll
        for (int i = 0; i < DE; ++i) e = fmaf(a, e, Ts[tp(DE * tid + i)]);
        Ps[tid] = aD;
        Es[tid] = e;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            float pl = 1.f, el = 0.f;
            if (tid >= off) {
                pl = Ps[tid - off];
                el = Es[tid - off];
            }
            __syncthreads();
            if (tid >= off) {
                Es[tid] = fmaf(Ps[tid], el, Es[tid]);   // (left then this segment): c -> E + P (el + pl c)
                Ps[tid] = Ps[tid] * pl;
            }
            __syncthreads();
        }
        // this segment's incoming value: the scan of the segments before it, fed the tile carry
        float c = tid == 0 ? carry : fmaf(Ps[tid - 1], carry, Es[tid - 1]);
        const float next_carry = fmaf(Ps[1023], carry, Es[1023]);
#pragma unroll
        for (int i = 0; i < DE; ++i) {
            const int k = DE * tid + i;
            c = fmaf(a, c, Ts[tp(k)]);
            Ts[tp(k)] = c;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < DE; ++i) {
            const int k = tid + 1024 * i;
            if (k < n) w[t0 + k] = Ts[tp(k)];
        }
        carry = next_carry;
        __syncthreads();
    }
}

#define AVC_DSP_INST(LG)                                          \
    template __global__ void dsp_wav2mel<LG>(DspArgs);            \
    template __global__ void dsp_gl_frames<LG>(DspArgs);
AVC_DSP_INST(4) AVC_DSP_INST(5) AVC_DSP_INST(6) AVC_DSP_INST(7) AVC_DSP_INST(8)
AVC_DSP_INST(9) AVC_DSP_INST(10) AVC_DSP_INST(11) AVC_DSP_INST(12)
#undef AVC_DSP_INST

}  // namespace avc
