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
                   2 * FZ_CIN * T * 4);
}
// + per-wave fold scratch [5*16 ch][8 edge columns] fp32
__host__ __device__ constexpr int fz_lds_bwd(int prec, int T) { return fz_lds_bwd_main(prec, T) + 4 * 5 * 16 * 8 * 4; }
}  // namespace avc
