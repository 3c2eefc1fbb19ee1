// Device-side problem descriptors shared by the kernels (avc_kernels.hip) and
// the host planner (avc_api.hip).  Everything is plain-old-data so the plan for
// one (B, T) workspace can be uploaded to HBM once and replayed every iteration
// (and captured into a hipGraph) with no per-iteration host work.
#pragma once
#include <stdint.h>

namespace avc {

constexpr int KSEG = 64;        // K-segment granule: a segment's rows are padded to it, so no K chunk
                                // (32 or 64 rows) ever straddles two segments
constexpr int KALIGN = 64;      // A matrices carry zero rows up to a multiple of the largest K chunk
constexpr int MAX_SEGS = 8;
constexpr int KSPLIT_MAX = 4;    // largest split-K factor (slab planes)

// How the im2col B-operand rows of one K segment are gathered from HBM.
enum Prec : int32_t { PREC_F32 = 0, PREC_BF16 = 1 };

enum SegMode : int32_t {
    SEG_FWD = 0,   // x_pad[c][t*stride + j] with reflect padding (models.py:10-30)
    SEG_BWD = 1,   // adjoint: zero-dilated dY, flipped taps, reflect-pad fold (dY already
                   // gated by ReLU' by its producer)
};

struct Seg {
    const float* src;    // [B][src_C][src_T]
    int32_t k0;          // first K row of the segment (multiple of KSEG)
    int32_t kpad;        // rows (C*ks rounded up to KSEG)
    int32_t C;           // channels gathered
    int32_t c_off;       // first channel inside src
    int32_t src_C, src_T;
    int32_t ks, stride, pl, pr;
    int32_t mode;
    int32_t pad_[3];
};

enum Epi : int32_t {
    EPI_ACT = 0,       // out0 = act(acc + bias)
    EPI_BLOCK = 1,     // a2 = act(acc + bias) -> out0 ; out1 = a2 + avgpool_s(aux0)
    EPI_MASK = 2,      // out0 = acc * act'(aux0)
    EPI_POOLT = 3,     // g = acc + avgpool_s^T(aux0); out0 = g (if set); out1 = g*act'(aux1) (if set)
    EPI_INCONV_T = 4,  // rows < split: out0 = acc*act'(aux0) ; rows >= split: out1 = acc
    EPI_ADAM = 5,      // g = acc + aux0 ; tanh backward ; Adam ; adv = vc + eps*tanh(p)
};

struct AdamArgs {
    float* ptb;
    float* m;
    float* v;
    const float* vc;
    float* adv;            // next-iteration input (== caller's out_adv)
    const float* table;    // [n_iters][2] = {-lr/(1-b1^t), sqrt(1-b2^t)}
    float* grad0;          // optional: dL/dptb at t == 1
    float b1c, b2, b2c;    // 1-beta1, beta2, 1-beta2 (as fp32, like torch's scalar casts)
    float adam_eps;
    int32_t pad_[4];
};

struct Problem {
    int32_t M, Mpad, N, K;     // GEMM: C[M][N] = A[M][K] * B[K][N]; K = end of the last segment
    int32_t T_out;             // columns per utterance (N = B*T_out)
    int32_t nseg;
    int32_t Kld;               // row stride of A (K rounded up to KALIGN; zero columns)
    int32_t ksplit_rows;       // split-K: rows per split (multiple of KALIGN); 0 = no split
    int32_t epi, act;
    const float* At;           // A row-major [Mpad][Kld] (k contiguous), fp32
    const void* Ab;            // the same A in bf16 (round-to-nearest-even)
    const float* bias;         // [M] or null
    float* out0; int32_t out0_C, out0_coff;
    float* out1; int32_t out1_C, split;
    const float* aux0; int32_t aux0_C, aux0_T;
    const float* aux1;         // EPI_POOLT: ReLU'-mask source of the masked output out1
    int32_t pool_s;
    int32_t both_edges;        // BWD gather: T_out <= pl+pr+1, a column may fold from both ends
    int32_t* tick;             // if set, block (0,0) thread 0 increments it (Adam step counter)
    const int32_t* step;       // Adam step counter (read by EPI_ADAM)
    const float* scal;         // per-call scalars: [0] = attack eps, [1] = loss-grad scale, [3] = PGD step (0: Adam)
    int32_t table_len;         // Adam table entries (step is clamped into [1, table_len])
    int32_t pad2_;
    float* slab;               // split-K partial sums [ksplit][M][N] (fp32), reduced in order
    AdamArgs adam;
    Seg seg[MAX_SEGS];
};

// Fused SpeakerEncoder head: mean pool -> dense blocks -> output Linear
// (models.py:275,307-325,340-342) [-> loss + its input-gradient back to the
// pooled features, attack_utils.py:81-83].  U utterances per workgroup.
struct HeadArgs {
    const float* hN;          // [B][C][TN]
    float* g_hN;              // [B][C][TN]   (attack mode)
    float* g_hN_masked;       // [B][C][TN]   g_hN * act'(mask_hN): the next dgrad's dY
    const float* mask_hN;     // [B][C][TN]
    const float* Wp;          // packed A fragments, forward
    const float* WpT;         // packed A fragments, backward (transposed)
    const float* bias;        // concatenated biases: dense(2*nd)*C, output D
    float* emb_out;           // [B][D]       (forward mode)
    const float* tgt;         // [B][D]
    const float* org;         // [B][D]
    float* losses;            // [n_iters][B] or null
    const int32_t* step;      // 1-based iteration counter (attack mode)
    const float* scal;        // [1] = 2 / n_elems of the MSE mean (per call)
    int32_t loss_len;         // rows of `losses` (iterations); writes beyond are dropped
    int32_t B, C, TN, D, n_dense, act, mode;
    const float* pooled_in;   // fused path: [B][C] time-mean of h_N (replaces the hN pooling)
    float* g_pooled;          // fused path: [B][C] d loss / d pooled (replaces the g_hN expansion)
    const float* Wr;          // se_head_v: row-major dense [2nd][C][C], output [D][C]
    const float* WrT;         // se_head_v: their transposes [2nd][C][C], output^T [C][D]
    int32_t tgt_parts;        // mode 3: d loss / d emb = sum of this many [B][D] slices at tgt
    const uint16_t* Wr16;     // se_head_v<true> (bf16 mode): Wr / WrT as bf16, 16-byte chunk layout
    const uint16_t* WrT16;
    float* act_out;           // fused mode 0: [B][2nd][C] the dense activations (for a later mode 3)
    const float* act_in;      // fused mode 3: the same, written by the mode-0 forward
};

// ---------------------------------------------------------------------------------
// Fused per-utterance SpeakerEncoder engine (avc_fused.hip): one workgroup of 4
// waves owns one utterance; every activation of the conv stack stays in LDS.
// Wave w owns output channels [32w, 32w+32) of every 128-channel layer.
// ---------------------------------------------------------------------------------
constexpr int FZ_MAXNB = 8;       // bank kernels
constexpr int FZ_MAXBLK = 8;      // conv blocks
constexpr int FZ_MAXNF = 9;       // 16-column fragments per layer (T <= 128, + edge columns)
constexpr int FZ_CIN = 80;        // mel bins (the only c_in the fused path is built for)
constexpr int FZ_C = 128;         // c_h == c_bank == c_out
constexpr int FZ_MASK_WORDS_PER_LAYER = 4 * 2 * FZ_MAXNF * 4;   // u64 ballot words (4 waves)

// Packed A operands: [m_tile(16 rows)][k_step][64 lanes][16 bytes]; lane (r = l&15,
// q = l>>4) holds A[16*mt + r][KS*step + VE*q + e], e < VE (VE = 4 fp32 / 8 bf16, KS = 4*VE).
// The K index of a conv is (tap j, input channel c) -> j*Cin + c.
struct FusedW {
    const void* bank[FZ_MAXNB];       // fwd: M=128, K=k*80
    const void* in_b[FZ_MAXNB];       // fwd in_conv, bank block kb: M=128, K=128
    const void* in_x;                 // fwd in_conv, x block: M=128, K=80
    const void* c1[FZ_MAXBLK];        // fwd conv1: M=128, K=ks*128
    const void* c2[FZ_MAXBLK];
    const void* c1T[FZ_MAXBLK];       // dgrad: A[ci][j*128+co] = W[co][ci][j]
    const void* c2T[FZ_MAXBLK];
    const void* inT_b[FZ_MAXNB];      // in_conv^T, bank block: A[ci'][co] = W_in[co][kb*128+ci']
    const void* inT_x;                // in_conv^T, x block: M=80, K=128
    const void* bankT[FZ_MAXNB];      // bank^T: M=80, K=k*128
    const float* b_bank[FZ_MAXNB];
    const float* b_in;
    const float* b_c1[FZ_MAXBLK];
    const float* b_c2[FZ_MAXBLK];
    const void* mean_w;               // ContentEncoder mean_layer 1x1: M=128, K=128 (CE packs only)
    const float* b_mean;
};

// Ragged batch (long engine, emb attack; avc_emb_attack_ragged): every workgroup's utterance has its own
// length.  Its input / Adam state start at float offset xoff of the packed arrays ([80][T_b] blocks, one
// after the other); the scratch slots (LongArgs) are sized for the longest.
// (The block lengths follow from T: Tl[l+1] = ceil(Tl[l] / sub[l]), avc_long.hip lz_tl.)
struct RagUtt {
    int32_t T;
    int32_t pad_;
    int64_t xoff;
};

struct FusedArgs {
    int32_t B, T, nb, ks, nblk, act;
    int32_t sub[FZ_MAXBLK];
    int32_t Tl[FZ_MAXBLK + 1];
    int32_t mask_words;               // u64 words per utterance
    int32_t write_masks;              // fwd: store ReLU' ballot masks (attack iterations)
    const float* x;                   // fwd input [B][80][T]
    float* pooled;                    // fwd output [B][128]: mean over T of h_N
    unsigned long long* masks;        // [B][mask_words]
    const float* g_pooled;            // bwd input [B][128]
    int32_t* tick;                    // fwd: block 0 advances the Adam step counter
    const int32_t* step;              // bwd: Adam step (1-based)
    const float* scal;                // [0] = attack eps, [3] = PGD step (0: Adam)
    int32_t table_len;
    int32_t ce_mode;                  // fwd: ContentEncoder (InstanceNorm before every act after the
                                      // bank, mean_layer output to mu_out instead of the time-mean)
    float* mu_out;                    // fwd, ce_mode: [B][128][T_N]
    float* gx_out;                    // bwd: if set, write d loss / d x [B][80][T] here (no Adam)
    AdamArgs adam;                    // bwd: Adam update + next adv
    FusedW w;
    // emb attack, bf16: the head chain (se_head_v mode 1) runs in the forward's tail
    int32_t fuse_head;                // fwd: run `head` for this workgroup's utterance in mode 1 (emb
                                      // loss + backward) or 2 (mode 0: embedding + activations out);
                                      // bwd: 3 = mode 3 (d loss / d emb -> g_pooled) before the stack
    int32_t loss_len;                 // bwd: rows of `losses`
    float* loss_cur;                  // fwd writes / bwd reads: [B] this iteration's per-utterance loss
    float* losses;                    // bwd: [loss_len][B] loss history (row = step - 1), or null
    HeadArgs head;                    // fwd (fuse_head): weights, biases, targets, g_pooled out
    const RagUtt* rag;                // long engine: per-workgroup lengths / offsets (null: every utterance
                                      // T frames at b * 80 * T)
};

// persistent emb attack (se_attack_fused): the forward's and the backward's arguments and the iteration count
struct AtkArgs {
    FusedArgs f, b;
    int32_t n_iters;
};

// ---------------------------------------------------------------------------------
// Long-utterance engine (avc_long.hip): any T (the fused engine's LDS images stop at 128
// frames).  Still one workgroup of 4 waves per utterance and wave w owns channels
// [32w, 32w+32), but the activations live in per-utterance global scratch (L2 / MALL):
//   operand images  [LZ_ZR pad rows | frames | pad rows][128 channels] of the operand type
//                   (bf16 / fp32), reflect-mirror or zero pad rows written by the producer;
//   fp32 streams    the residual h, its gradient and raw GEMM outputs, in the MFMA C/D
//                   "fragment layout" [16-frame fragment][wave][tile][64 lanes] f32x4, so an
//                   epilogue reads / writes one coalesced 1 KiB run per wave instruction;
//   ReLU' masks     64-bit ballots per (layer, 16-frame fragment, wave, tile, row), so any
//                   16-aligned frame chunking reads them back.
// Each layer runs over chunks of 128 output frames: the chunk's input rows are staged into
// LDS and the layer's GEMM runs on MFMA exactly as in the fused engine.
// ---------------------------------------------------------------------------------
constexpr int LZ_ZR = 16;         // pad rows before frame 0 / after the last frame of an image
constexpr int LZ_FL_EXTRA = 4;    // fragments beyond ceil(T/16) in a fragment-layout stream

struct LongArgs {
    char* img[3];                     // operand images, per utterance img_stride bytes each
    int64_t img_stride;
    float* fl[3];                     // fp32 fragment-layout streams, fl_stride floats per utterance
    int64_t fl_stride;
    unsigned long long* masks;        // ballot words [B][layer][nFmax][wave][tile*4 + row]
    int64_t mask_stride;              // words per utterance
    int32_t nFmax;                    // fragments per layer in the mask layout
    int32_t pad_;
};

// ---------------------------------------------------------------------------------
// Fused per-utterance Decoder (avc_vc.hip, models.py:346-435) for the e2e / feedback
// attacks.  Same layout rules as the SpeakerEncoder engine: wave w owns channels
// [32w, 32w+32) of every 128-channel layer.  A x2 pixel-shuffle conv (128 -> 256
// channels) runs as two half-GEMMs over its even (s = 0) and odd (s = 1) output
// channels: half s of channel c is the frame 2t+s of the shuffled output.
// ---------------------------------------------------------------------------------
constexpr int DZ_MAXBLK = 8;
constexpr int DZ_COUT = 80;

struct DecW {
    const void* in;                   // in_conv 1x1: M=128, K=128
    const void* c1[DZ_MAXBLK];        // M=128, K=ks*128, K index (tap, channel)
    const void* c2[DZ_MAXBLK][2];     // half s: rows 2c+s of second_conv (up=1: [0] only)
    const void* out;                  // out_conv 1x1: M=80, K=128
    const void* c1T[DZ_MAXBLK];       // dgrad: A[ci][(j, co)] = W1[co][ci][j]
    const void* c2T[DZ_MAXBLK][2];    // dgrad of half s: A[ci][(j, c)] = W2[2c+s][ci][j]
    const void* outT;                 // M=128, K=80: A[ci][co] = Wout[co][ci]
    const float* b_in;
    const float* b_c1[DZ_MAXBLK];
    const float* b_c2[DZ_MAXBLK][2];  // bias of half s
    const float* b_out;
};

struct DecArgs {
    int32_t B, ks, nblk, act;
    int32_t up[DZ_MAXBLK];
    int32_t Tl[DZ_MAXBLK + 1];        // lengths: Tl[0] = content length, Tl[l+1] = Tl[l] * up[l]
    int32_t stash_off[2 * DZ_MAXBLK]; // per InstanceNorm layer q = 2l (conv1), 2l+1 (conv2): float offset
    int32_t stash_per_utt;            // floats per utterance (0: no stash, forward only)
    const float* mu;                  // [B][128][Tl[0]] ContentEncoder mean
    const float* cond;                // [B][2*nblk][256] conv_affine outputs (mean | std)
    float* out;                       // [B][80][Tl[nblk]]
    float* stash;                     // [B][stash_per_utt] normalised activations (fwd -> bwd)
    float* invstd;                    // [B][2*nblk][128]
    // e2e loss (fwd): MSE(out, tgt_out) - 0.1 MSE(out, org_out) and its gradient
    const float* tgt_out;
    const float* org_out;
    float* g_out;                     // [B][80][Tl[nblk]]
    float* losses;                    // [n_iters][B] or null
    const int32_t* step;
    const float* scal;                // [2] = 2 / n_elems of the output MSE
    int32_t loss_len, pad_;
    // bwd
    const float* g_in;                // [B][80][Tl[nblk]] d loss / d out
    float* g_cond;                    // [B][2*nblk][256]
    DecW w;
};

// Batched dense layer over utterances: Y[b][m] = sum_k A[m][k] X[b][k] (+ bias[m])
// (the decoder's conv_affine Linear layers and their transposes).
// Split-K (gridDim.z = K / kchunk slices): slice z sums k in [z*kchunk, (z+1)*kchunk) into
// Y + z*B*M; the consumer adds the slices in a fixed order (deterministic, no atomics).
enum { DZ_VALU = 0, DZ_MFMA = 1, DZ_LDS = 2 };
struct DenseArgs {
    const float* A;                   // [M][K] row-major
    const float* X;                   // [B][K]
    const float* bias;                // [M] or null (added by slice 0 only)
    float* Y;                         // [gridDim.z][B][M]
    int32_t M, K, B, kchunk;
    int32_t variant;                  // DZ_VALU / DZ_MFMA / DZ_LDS (host-chosen; fixes the grid)
};

// Spectral-norm Decoder (sn=True, models.py:382: torch.nn.utils.spectral_norm, train mode since the
// reference never calls .eval()): before every Decoder forward, sn_power runs one power iteration per
// layer on W = weight_orig.reshape(out, -1) (v = normalize(W^T u), u = normalize(W v), sigma = u.(W v))
// and sn_scale rewrites every packed copy of the layer's weights as weight_orig / sigma (avc_vc.hip).
constexpr int SN_MAXDIM = 1024;   // largest out / in*k of a spectral-normed layer
struct SnLayer {
    int32_t h, w;                     // W is [h][w] row-major at raw + raw_off
    int64_t raw_off, u_off, v_off;    // u [h], v [w] at uv + u_off / v_off
};
struct SnChunk {                      // <= SN_CHUNK elements of one packed copy of one layer
    void* dst;                        // fp32 or bf16 (packed operand, same element order as src)
    const float* src;                 // the same elements of weight_orig (fp32)
    int32_t n, layer, bf16, pad;
};
constexpr int SN_CHUNK = 4096;
struct SnArgs {
    const SnLayer* layers;
    const float* raw;
    float* uv;
    float* sigma;                     // [layers]
    const SnChunk* chunks;
    const int* train;                 // device flag: 1 = train-mode hook (power iteration, u / v updated),
                                      // 0 = eval mode (sigma = u.(W v) from the stored u / v, nothing written)
};

// VSMask PredictiveModel layer (avc_pm.hip): implicit GEMM over NCHW activations.
struct PmConvArgs {
    const float* x;                   // [B][Cin][Hin][Win]
    const float* w;                   // packed A: mode 0 [Cout][Cin*9] (BN folded); mode 1 class c at woff[c]:
                                      // [Cout][Cin*nty*ntx]
    const float* bias;                // [Cout]
    float* y;                         // [B][Cout][Ho][Wo]
    int32_t B, Cin, Hin, Win, Cout, Ho, Wo, sh, sw;
    int32_t mode;                     // 0: reflect-pad conv 3x3 stride (sh, sw); 1: ConvTranspose2d 3x3 s2
    int32_t act;                      // 0: PReLU(slope); 1: LeakyReLU(0.2); 2: LeakyReLU(0.2) then tanh
    float slope;
    int32_t woff[4];
    int32_t ksplit;                   // > 1: K slices (blockIdx.z = class * ksplit + slice) write raw
    float* part;                      //      partial sums to part[slice][B*Cout*Ho*Wo]; pm_reduce finishes
    int32_t in_nhwc, out_nhwc;        // activation layouts (pm_conv): 0 = NCHW, 1 = NHWC (pm_mfma: both NHWC)
    const float* wm;                  // pm_mfma: A in MFMA fragment order, class c at wmoff[c] floats:
    int32_t wmoff[4];                 //   [m tile][K chunk of 16][64 lanes][4], K = (tap, ci)
};

// DSP frame kernels (avc_dsp.hip): LDS slot of complex element i of the FFT buffer,
// i + 2 floor(i/32) + floor(i/64).  Chosen by simulating the ds_read_b64 / ds_write_b64 lane
// groups of every access pattern at N = 2048 (worst extra-cycle factor per instruction:
// bit-reversed store 1, radix-4 passes 1 / 2 / 2 / 1 / 1; the former one-per-32 pad had
// 2 / 1 / 4 / 2 / 1 / 1 -- PMC: 2.85 conflict cycles per LDS instruction in the early passes)
// FFT buffer padding: one pad entry per 8 -- the Stockham passes' stride-8 output writes
// (radix 8 at sub-transform size 1) then cover 32 distinct bank pairs per 32 lanes
__host__ __device__ constexpr int dsp_zp(int i) { return i + (i >> 3); }
__host__ __device__ constexpr int dsp_zlen(int N) { return dsp_zp(N - 1) + 1; }
// twiddle table in LDS: one pad entry per 32, so the strided reads TW[k * (N >> s)] of the FFT
// passes (strides 64 / 16 / 4 entries across lanes) spread over the banks instead of a few
__host__ __device__ constexpr int dsp_tp(int i) { return i + (i >> 5); }
__host__ __device__ constexpr int dsp_twlen(int N) { return dsp_tp(N / 2 - 1) + 1; }

// UniversalPerturbationHeader.optimize (models/header_model.py:40-65), one iteration's
// elementwise ends around the SpeakerEncoder forward / input-gradient passes
struct HdrArgs {
    const float* src;                 // [N][F*T] source mels (constant)
    float* hdr;                       // [F*T] the header (in place)
    float* m;                         // [F*T] Adam state
    float* v;
    float* x;                         // compose: [N][F*T] = clamp(src + hdr, -1, 1)
    const float* gx;                  // update: [N][F*T] d loss / d x
    const float* table;               // Adam table [iters][2] (-lr / bc1, sqrt(bc2))
    const int32_t* step;              // 1-based step (advanced by the forward)
    int32_t table_len, N, FT;
    float b1c, b2, b2c, adam_eps;     // 1 - beta1, beta2, 1 - beta2, eps
    float clamp_eps;                  // header clamp (epsilon)
};

// VSMask protect loop (/root/reference/vsmask.py:177-208): window gather + combine/clamp.
struct VsmArgs {
    const float* mel;                 // [B][F][T] log-mel (the 4-D [B,1,F,T] view)
    const float* header;              // [F][Th] universal perturbation header (nullptr: none)
    const float* y;                   // [B*nw][Ho][Wo] predictor output per window (nw = 0: none)
    float* win;                       // gather: [B*nw][F][W] windows
    float* out;                       // [B][F][T]
    int B, F, T, Th, W, S, nw, Ho, Wo, rows;   // rows = min(F, Ho): predicted rows that land on the mel
    int low_end, high_start;          // band edges int(F*0.3), int(F*0.7) (utils/audio.py:97-98)
    float eps1, eps2, eps3;
    int mode;                         // 0 = protect (band clamp of the summed perturbation),
                                      // 1 = header_model.apply_header (clamp the sum to [-1, 1]),
                                      // 2 = apply_weighted_constraint alone (band clamp of mel)
};

// Mel front / back end (avc_dsp.hip; data_utils.py:16-197).  One workgroup per pair of
// STFT frames: the two real frames are the real and imaginary parts of ONE complex
// n_fft-point FFT in LDS (radix-2, bit-reversed load, twiddles staged in LDS).
struct DspArgs {
    int32_t B, N, logN, F, hop, Tf;    // F = N/2 + 1 bins, Tf frames per utterance
    int32_t L;                         // samples per utterance of the signal framed (x)
    int32_t Ly;                        // samples per utterance of the OLA output (y)
    int32_t n_mels, pad_mode;          // pad_mode 0: reflect (librosa 0.8 default), 1: constant
    int32_t init;                      // dsp_gl_frames: 1 = X = spect (zero phase), 0 = project
    int32_t transpose;                 // mel layout: 0 [B][Tf][n_mels], 1 [B][n_mels][Tf]
    float preemph, ref_db, max_db;
    const float* window;               // [N] periodic Hann(win_length) zero-padded to N
    const float* twiddle;              // [N/2][2]: exp(-2 pi i k / N)
    const float* x;                    // framed signal [B][L]
    const float* mel_basis;            // [n_mels][F]
    const int32_t* mel_range;          // [n_mels][2]: non-zero bins [lo, hi) of each filter
    const float* inv_mel;              // [n_mels][F]: inv_mel_matrix^T (data_utils.py:16-32)
    const float* mean;                 // [n_mels] normalize / denormalize statistics, or null
    const float* std;
    const float* mel_in;               // dsp_mel2mag input
    float* mel_out;                    // dsp_wav2mel output
    const float* spect;                // [B][Tf][F] target magnitude (Griffin-Lim)
    float* spect_out;                  // dsp_mel2mag / dsp_transpose output
    float* frames;                     // [B][Tf][N] windowed inverse-FFT frames
    float* y;                          // [B][Ly] overlap-added signal
    float* wav;                        // [B][Ly] de-emphasised output
    float* wss;                        // [Ly] window sum-square of the output samples (dsp_wss)
    int32_t vec4;                      // hop % 4 == 0 and y 16-byte aligned: 16-byte sample accesses
    // flavor 1: utils/audio.py's torchaudio converter (power-2 STFT, log10 mel, pinv inverse,
    // Griffin-Lim with momentum from given initial angles); 0: data_utils.py's librosa pipeline
    int32_t flavor;
    float momentum;                    // flavor 1 Griffin-Lim: alpha = momentum / (1 + momentum)
    const float* angles0;              // [B][F][Tf] complex64 initial angles (torch layout), or null: 1
    float* tprev;                      // [B][Tf][F] complex: the previous rebuilt spectrum
};

}  // namespace avc
