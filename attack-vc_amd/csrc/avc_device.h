// Device helpers shared by the libavc kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace avc {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Global-address-space views: pointers read out of the Problem table are
// generic, which would make every access a flat_* op (also counted on lgkmcnt).
typedef const float __attribute__((address_space(1)))* gcptr;
typedef float __attribute__((address_space(1)))* gptr;
__device__ __forceinline__ gcptr as_global(const float* p) { return (gcptr)p; }
__device__ __forceinline__ gptr as_global_w(float* p) { return (gptr)p; }

template <class V>
__device__ __forceinline__ V gload(const float* p) {
    return *reinterpret_cast<const __attribute__((address_space(1))) V*>(as_global(p));
}
template <class V>
__device__ __forceinline__ void gstore(float* p, V v) {
    *reinterpret_cast<__attribute__((address_space(1))) V*>(as_global_w(p)) = v;
}

// get_act (models.py:107-118): 0 = ReLU, 1 = LeakyReLU(0.01)
__device__ __forceinline__ float act_f(float x, int act) { return x > 0.f ? x : (act ? 0.01f * x : 0.f); }
// derivative expressed through the activation OUTPUT (same sign as its input)
__device__ __forceinline__ float act_d(float y, int act) { return y > 0.f ? 1.f : (act ? 0.01f : 0.f); }

}  // namespace avc
