// Shared device/host helpers for libdv_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <type_traits>

#include "../../include/dv_hip.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

namespace dv {

// thread-local last-error message surfaced by dv_last_error()
void set_error(const std::string& msg);
int check_launch(const char* what);
// zero n floats on `st` with a kernel (used instead of hipMemsetAsync so that
// zeroing is an ordinary kernel node when the stream is captured into a graph)
void zero_f32(float* p, long long n, hipStream_t st);

#define DV_REQUIRE(cond, msg)                      \
  do {                                             \
    if (!(cond)) {                                 \
      ::dv::set_error(std::string(__func__) + ": " + (msg)); \
      return DV_ERR_INVALID;                       \
    }                                              \
  } while (0)

// LDS-DMA through a raw buffer resource: a lane whose byte offset is out of
// range (DMA_OOB) writes 16 zero bytes to its LDS slot WITHOUT a memory
// access -- halo / pad slots must not all hit one shared zero line (a single
// hot L2 channel per XCD).  Resource size must stay below DMA_OOB.
constexpr unsigned DMA_OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dma_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
// 16 B per lane to LDS (lds + 16 * lane: `lds` must be wave-uniform)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff, 0, 0, 0);
}

// as dma16 with a wave-uniform byte offset added to every lane's address
// (the instruction's SGPR soffset: a per-chunk offset costs no VALU)
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff, (int)soff, 0, 0);
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// LDS byte address of a generic pointer into __shared__ memory
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// ds_read_b128 outside hipcc's waitcnt tracking: the caller waits with
// lgkm_wait_tied before using the result
template <int OFF>
__device__ __forceinline__ u32x4 ds_read_b128_off(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16 bits");
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}

// s_waitcnt lgkmcnt(N), tied to `v` so no use of v is scheduled above it
template <int N>
__device__ __forceinline__ void lgkm_wait_tied(u32x4& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v) { return (T)v; }

// v_exp_f32 + v_rcp_f32 (1 ulp), not the ~10-instruction IEEE divide: these
// sit in the per-element loops of the GroupNorm passes and conv epilogues,
// which are VALU-bound at their occupancy.  Large |x| saturates correctly
// (rcp(inf) = 0).
__device__ __forceinline__ float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float silu_f(float x) { return x * sigmoid_f(x); }

// wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x == NT (multiple of 64); `sh` holds NT/64 floats
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += sh[i];
  return r;
}

// 16-byte vector <-> T[16/sizeof(T)] helpers
template <typename T> struct Vec { };
template <> struct Vec<float> {
  static constexpr int N = 4;
  // NB: cast the whole vector; bit-casting single u32x4 elements in an
  // unrolled loop miscompiles on hipcc 7.2 (every element reads element 0).
  __device__ static inline void to_f(u32x4 v, float* o) {
    const f32x4 f = __builtin_bit_cast(f32x4, v);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = f[i];
  }
};
template <> struct Vec<bf16> {
  static constexpr int N = 8;
  __device__ static inline void to_f(u32x4 v, float* o) {
    const f32x4 lo = __builtin_bit_cast(f32x4, v << 16);
    const f32x4 hi = __builtin_bit_cast(f32x4, v & 0xffff0000u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = lo[i];
      o[2 * i + 1] = hi[i];
    }
  }
};

// ---- OCP MX-fp8 (e4m3 elements, one e8m0 scale per 32 channels): shared by
// the quantiser (dv_mx8.hip) and the GroupNorm apply's fused quantiser ----
// scale exponent E of a block with max |v| = amax: every v * 2^-E lies in the
// e4m3 range (<= 448) and the largest uses its top binade where it fits
__device__ __forceinline__ int mx_exp(float amax) {
  const unsigned b = __float_as_uint(amax);
  const int eb = (int)((b >> 23) & 255);
  const int E = eb - 135 + ((b & 0x7fffffu) > 0x600000u ? 1 : 0);
  return E < -127 ? -127 : E;
}
__device__ __forceinline__ float mx_inv(int E) { return __uint_as_float((unsigned)(127 - E) << 23); }

}  // namespace dv
