// In-graph kernel timing (bench.py's roofline): the durations of the hot kernels as they run
// inside the captured attack-loop graphs, with no profiler attached.  Each workgroup stamps the
// device's constant-rate wall clock (100 MHz) when it starts and when its last wave is done; the
// launch lasts from the earliest start to the latest end, and the workgroup that finishes last
// adds that span to a running sum (and resets the launch's min / max for the next launch, which
// stream order keeps behind it).  Off by default: a disabled record costs a clock read and a scalar
// load per workgroup (an earlier version that tested the flag with a vector load at the kernel's
// start and end cost 1.2 % of an emb iteration: two exposed HBM round trips per kernel).
//
// A record lives in the translation unit of the kernels it times (a __device__ symbol cannot be
// shared across hipcc objects without relocatable device code); each unit exports its records'
// device address through a host function, and avc_ktime (avc_api.hip) reads them.
#pragma once
#include <hip/hip_runtime.h>

namespace avc {

struct KTime {
    unsigned long long on;        // 0: not recording
    unsigned long long t0, t1;    // current launch: earliest start, latest end (wall-clock ticks)
    unsigned long long done;      // workgroups of the current launch that finished
    unsigned long long sum, n;    // summed launch spans (ticks) and launches
    unsigned long long pad[2];
};
constexpr int KT_SLOTS = 8;       // records per translation unit: kernel k at 2k (fp32) and 2k + 1 (bf16)
constexpr int KT_FUSED_FWD = 0, KT_FUSED_BWD = 2, KT_FUSED_ATK = 4;           // avc_fused.hip
constexpr int KT_LZ_SE_FWD = 0, KT_LZ_SE_BWD = 2, KT_LZ_DEC_FWD = 4, KT_LZ_DEC_BWD = 6;   // avc_long.hip
constexpr int KT_DEC_FWD = 0, KT_DEC_BWD = 2;                                  // avc_vc.hip

// Taken as the kernel's first action: the workgroup's start time and whether recording is on.  The flag
// is a scalar load whose wait lands on the first LDS / barrier wait of the kernel (no stall of its own).
struct KtStart {
    unsigned long long t0;
    bool on;
};
__device__ __forceinline__ KtStart ktime_begin(const KTime* k) {
    return KtStart{(unsigned long long)wall_clock64(), k->on != 0ull};
}
// every thread of the workgroup calls this as its last action
__device__ __forceinline__ void ktime_end(KTime* k, const KtStart& s) {
    if (!s.on) return;                        // the same value for every thread: a uniform branch
    __syncthreads();
    if (threadIdx.x != 0) return;
    const unsigned long long t1 = (unsigned long long)wall_clock64();
    atomicMin(&k->t0, s.t0);
    atomicMax(&k->t1, t1);
    __threadfence();
    const unsigned long long nwg = (unsigned long long)gridDim.x * gridDim.y * gridDim.z;
    if (atomicAdd(&k->done, 1ull) == nwg - 1) {
        __threadfence();
        const unsigned long long a = atomicAdd(&k->t0, 0ull), b = atomicAdd(&k->t1, 0ull);
        atomicAdd(&k->sum, b > a ? b - a : 0ull);
        atomicAdd(&k->n, 1ull);
        atomicExch(&k->t0, ~0ull);
        atomicExch(&k->t1, 0ull);
        atomicExch(&k->done, 0ull);
    }
}

}  // namespace avc

// one record array per translation unit and its host-side accessor
#define AVC_KTIME_DEFINE(UNIT)                                          \
    namespace avc {                                                     \
    __device__ KTime g_ktime_##UNIT[KT_SLOTS];                          \
    }                                                                   \
    extern "C" avc::KTime* avc_ktime_records_##UNIT() {                 \
        void* p = nullptr;                                              \
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(avc::g_ktime_##UNIT)) != hipSuccess) return nullptr; \
        return reinterpret_cast<avc::KTime*>(p);                        \
    }
