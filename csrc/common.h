// dgraph_amd — device-side helpers shared by the gfx950 (CDNA4) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace dgraph {

constexpr int kWave = 64;  // CDNA wavefront width; never 32.

// ---------------------------------------------------------------------------
// bf16 <-> f32. bf16 payloads are stored as raw uint16 (layout-identical to
// at::BFloat16); arithmetic is always fp32.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  // Plain conversion: hipcc emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving).
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}

// Element traits: storage type, and vector load/store of VEC elements.
template <typename T> struct Elem;
template <> struct Elem<float> {
  using storage = float;
  __device__ __forceinline__ static float to_f32(float v) { return v; }
  __device__ __forceinline__ static float from_f32(float v) { return v; }
};
template <> struct Elem<uint16_t> {  // bf16
  using storage = uint16_t;
  __device__ __forceinline__ static float to_f32(uint16_t v) { return bf16_to_f32(v); }
  __device__ __forceinline__ static uint16_t from_f32(float v) { return f32_to_bf16(v); }
};

// Raw byte vectors used for 4/8/16-byte per-lane loads.
template <int BYTES> struct RawVec;
template <> struct RawVec<2> { using type = uint16_t; };
template <> struct RawVec<4> { using type = uint32_t; };
template <> struct RawVec<8> { using type = uint2; };
template <> struct RawVec<16> { using type = uint4; };

// Load VEC elements of T starting at p (aligned to VEC*sizeof(T)) into fp32 regs.
template <typename T, int VEC>
__device__ __forceinline__ void load_vec_f32(const T* __restrict__ p, float (&o)[VEC]) {
  using R = typename RawVec<VEC * sizeof(T)>::type;
  R r = *reinterpret_cast<const R*>(p);
  const T* e = reinterpret_cast<const T*>(&r);
#pragma unroll
  for (int i = 0; i < VEC; ++i) o[i] = Elem<T>::to_f32(e[i]);
}

template <typename T, int VEC>
__device__ __forceinline__ void store_vec_f32(T* __restrict__ p, const float (&v)[VEC]) {
  using R = typename RawVec<VEC * sizeof(T)>::type;
  R r;
  T* e = reinterpret_cast<T*>(&r);
#pragma unroll
  for (int i = 0; i < VEC; ++i) e[i] = Elem<T>::from_f32(v[i]);
  *reinterpret_cast<R*>(p) = r;
}

// Grid sizing for grid-stride, memory-bound kernels: enough waves to fill
// 256 CUs x 8 waves, never more than needed.
inline int64_t cap_blocks(int64_t want, int64_t cap = 256 * 16) {
  if (want < 1) return 1;
  return want < cap ? want : cap;
}

}  // namespace dgraph
