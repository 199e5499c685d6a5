// Shared helpers for the libic2ops HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>
#include "../../include/ic2ops.h"

namespace ic2 {

// ------------------------------------------------------------------------------------------------
// error reporting: every entry point returns IC2_OK or an IC2_E_* code; the message is thread-local
// ------------------------------------------------------------------------------------------------
void set_error(const char* fmt, ...);

// development knob `name` (integer env var), read only when IC2_DEV=1, else `dflt` (errors.hip)
int knob(const char* name, int dflt);

#define IC2_CHECK_ARG(cond, ...)                      \
  do {                                                \
    if (!(cond)) {                                    \
      ::ic2::set_error(__VA_ARGS__);                  \
      return IC2_E_INVALID;                           \
    }                                                 \
  } while (0)

#define IC2_CHECK_LAUNCH(name)                                                    \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) {                                                       \
      ::ic2::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));     \
      return IC2_E_LAUNCH;                                                        \
    }                                                                             \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------------------------------------
// bf16 <-> f32 (bf16 carried as raw uint16 in memory)
// ------------------------------------------------------------------------------------------------
typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  // round-to-nearest-even; NaN kept a NaN (plain cast lowers to v_cvt_pk_bf16_f32 on gfx950)
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  __device__ static __forceinline__ float load(const float* p) { return *p; }
  __device__ static __forceinline__ void store(float* p, float v) { *p = v; }
};
template <> struct Elem<bf16_t> {
  __device__ static __forceinline__ float load(const bf16_t* p) { return bf2f(*p); }
  __device__ static __forceinline__ void store(bf16_t* p, float v) { *p = f2bf(v); }
};

// f16 elements (the synthesis's f16 mode): stores saturate to the f16 range instead of overflowing to inf
template <> struct Elem<_Float16> {
  __device__ static __forceinline__ float load(const _Float16* p) { return (float)*p; }
  __device__ static __forceinline__ void store(_Float16* p, float v) {
    *p = (_Float16)__builtin_amdgcn_fmed3f(v, -65504.f, 65504.f);
  }
};

template <typename T> __device__ __forceinline__ float ld(const T* p) { return Elem<T>::load(p); }
template <typename T> __device__ __forceinline__ void st(T* p, float v) { Elem<T>::store(p, v); }

__device__ __forceinline__ float lrelu_gain_clamp(float v, float slope, float gain, float clamp) {
  v = v < 0.f ? v * slope : v;
  v = v * gain;
  if (clamp >= 0.f) v = fminf(fmaxf(v, -clamp), clamp);
  return v;
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// A zeroed 64-byte line in the code object: out-of-image loads read it instead of branching around
// the load (a per-load branch makes hipcc wait vmcnt(0) per element -> serialised round trips).
static __device__ __attribute__((aligned(64))) uint32_t g_zero_line[16] = {0};
__device__ __forceinline__ const void* zero_line() { return g_zero_line; }

}  // namespace ic2
