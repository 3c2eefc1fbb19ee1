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
    const float* scal;         // per-call scalars: [0] = attack eps, [1] = loss-grad scale
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
};

}  // namespace avc
