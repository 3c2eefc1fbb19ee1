// Device-side problem descriptors shared by the kernels (avc_kernels.hip) and
// the host planner (avc_api.hip).  Everything is plain-old-data so the plan for
// one (B, T) workspace can be uploaded to HBM once and replayed every iteration
// (and captured into a hipGraph) with no per-iteration host work.
#pragma once
#include <stdint.h>

namespace avc {

constexpr int KC = 16;          // K rows staged per chunk (fp32 path)
constexpr int MAX_SEGS = 8;

// How the im2col B-operand rows of one K segment are gathered from HBM.
enum SegMode : int32_t {
    SEG_FWD = 0,   // x_pad[c][t*stride + j] with reflect padding (models.py:10-30)
    SEG_BWD = 1,   // adjoint: zero-dilated dY, flipped taps, reflect-pad fold
};

struct Seg {
    const float* src;    // [B][src_C][src_T]
    const float* mask;   // BWD: activation whose sign gates dY (act'), or null
    int32_t k0;          // first K row of the segment (multiple of KC)
    int32_t kpad;        // rows (C*ks rounded up to KC)
    int32_t C;           // channels gathered
    int32_t c_off;       // first channel inside src
    int32_t src_C, src_T;
    int32_t ks, stride, pl, pr;
    int32_t mode;
    int32_t pad_;
};

enum Epi : int32_t {
    EPI_ACT = 0,       // out0 = act(acc + bias)
    EPI_BLOCK = 1,     // a2 = act(acc + bias) -> out0 ; out1 = a2 + avgpool_s(aux0)
    EPI_MASK = 2,      // out0 = acc * act'(aux0)
    EPI_POOLT = 3,     // out0 = acc + avgpool_s^T(aux0)
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
    int32_t M, Mpad, N, K;     // GEMM: C[M][N] = A[M][K] * B[K][N], K padded
    int32_t T_out;             // columns per utterance (N = B*T_out)
    int32_t nseg;
    int32_t epi, act;
    const float* At;           // [K][Mpad]
    const float* bias;         // [M] or null
    float* out0; int32_t out0_C, out0_coff;
    float* out1; int32_t out1_C, split;
    const float* aux0; int32_t aux0_C, aux0_T;
    int32_t pool_s;
    int32_t* tick;             // if set, block (0,0) thread 0 increments it (Adam step counter)
    const int32_t* step;       // Adam step counter (read by EPI_ADAM)
    const float* scal;         // per-call scalars: [0] = attack eps, [1] = loss-grad scale
    AdamArgs adam;
    Seg seg[MAX_SEGS];
};

// Fused SpeakerEncoder head: mean pool -> dense blocks -> output Linear
// (models.py:275,307-325,340-342) [-> loss + its input-gradient back to the
// pooled features, attack_utils.py:81-83].  U utterances per workgroup.
struct HeadArgs {
    const float* hN;          // [B][C][TN]
    float* g_hN;              // [B][C][TN]   (attack mode)
    const float* Wp;          // packed A fragments, forward
    const float* WpT;         // packed A fragments, backward (transposed)
    const float* bias;        // concatenated biases: dense(2*nd)*C, output D
    float* emb_out;           // [B][D]       (forward mode)
    const float* tgt;         // [B][D]
    const float* org;         // [B][D]
    float* losses;            // [n_iters][B] or null
    const int32_t* step;      // 1-based iteration counter (attack mode)
    const float* scal;        // [1] = 2 / n_elems of the MSE mean (per call)
    int32_t B, C, TN, D, n_dense, act, mode;
};

}  // namespace avc
