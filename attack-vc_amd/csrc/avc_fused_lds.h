// LDS budget of the fused per-utterance engine (avc_fused.hip) at frame count T;
// shared by the kernels (buffer placement) and the host planner (launch shmem).
#pragma once
#include "avc_kernels.h"

namespace avc {
// LDS bytes of each kernel at frame count T (the host planner uses the same formulas)
__host__ __device__ constexpr int fz_rs(int prec) { return prec == PREC_F32 ? 544 : 288; }
__host__ __device__ constexpr int fz_max2(int a, int b) { return a > b ? a : b; }
__host__ __device__ constexpr int fz_lds_fwd(int prec, int T, int ks) {
    return fz_max2((T + 8) * fz_rs(prec) + (prec == PREC_BF16 ? 2 : 1) * T * fz_rs(prec),
                   2 * (T + 2 * (ks / 2)) * fz_rs(prec));
}
// blocks: two dY images; bank: g_pre0 image + bank dY image; reduction: two [80][T] fp32
__host__ __device__ constexpr int fz_lds_bwd_main(int prec, int T) {
    return fz_max2(fz_max2(2 * (T + 8) * fz_rs(prec), (T + 8) * fz_rs(prec) + (T + 16) * fz_rs(prec)),
                   2 * FZ_CIN * (T + 4) * 4);   // rows padded at T = 128 (avc_fused.hip)
}
// + per-wave fold scratch [5*16 ch][8 edge columns] fp32
__host__ __device__ constexpr int fz_lds_bwd(int prec, int T) { return fz_lds_bwd_main(prec, T) + 4 * 5 * 16 * 8 * 4; }
// launch size: the shape-generic bf16 backward (shape != 0) also holds the utterance's ReLU' words
// (mask_words u64) after that (avc_fused.hip: MLDS) -- at most 94.7 + 57.6 KB at T = 128
__host__ __device__ constexpr int fz_lds_bwd_launch(int prec, int T, int shape, int mask_words) {
    return fz_lds_bwd(prec, T) + (shape != 0 && shape != 16 && prec == PREC_BF16 ? 8 * mask_words : 0);
}

// fused Decoder (avc_vc.hip) at output length Tn: forward = block-input image + conv1
// output image, (Tn + 2P) rows each; backward = two dY images (Tn + 8 rows) + per-wave
// fold scratch [2*16 ch][8 edge columns] fp32.  (+ 32 B static LDS in the forward)
constexpr int DZ_FOLD_FLOATS = 2 * 16 * 8;
__host__ __device__ constexpr int dz_lds_fwd(int prec, int Tn, int ks) { return 2 * (Tn + 2 * (ks / 2)) * fz_rs(prec); }
__host__ __device__ constexpr int dz_lds_bwd(int prec, int Tn) {
    return 2 * (Tn + 8) * fz_rs(prec) + 4 * DZ_FOLD_FLOATS * 4;
}
}  // namespace avc
