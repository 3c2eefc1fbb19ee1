// In-graph kernel timing (bench.py's roofline): the durations of the hot kernels as they run
// inside the captured attack-loop graphs, with no profiler attached.  Each workgroup stamps the
// device's constant-rate wall clock (100 MHz) when it starts and when its last wave is done; the
// launch lasts from the earliest start to the latest end, and the workgroup that finishes last
// adds that span to a running sum (and resets the launch's min / max for the next launch, which
// stream order keeps behind it).  Off by default: a disabled record costs one load per workgroup.
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
constexpr int KT_SLOTS = 4;       // records per translation unit

__device__ __forceinline__ bool ktime_on(const KTime* k) {
    return __builtin_nontemporal_load(&k->on) != 0ull;
}
__device__ __forceinline__ void ktime_begin(KTime* k) {
    if (threadIdx.x == 0 && ktime_on(k)) atomicMin(&k->t0, (unsigned long long)wall_clock64());
}
// every thread of the workgroup calls this as its last action
__device__ __forceinline__ void ktime_end(KTime* k) {
    if (!ktime_on(k)) return;                 // the same value for every thread: a uniform branch
    __syncthreads();
    if (threadIdx.x != 0) return;
    atomicMax(&k->t1, (unsigned long long)wall_clock64());
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
