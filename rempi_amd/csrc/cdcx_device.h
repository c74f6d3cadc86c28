// cdcx_device.h -- device-side building blocks shared by the CDC encode/decode kernels:
// wave64/block scans, key packing, error reporting.  gfx950 only (wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cdcx_layout.h"

namespace cdcx {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / kWave; }

// Report an error code into the batch error word (first error wins on the host side; all
// bits are kept for diagnostics).
__device__ __forceinline__ void raise_error(uint32_t* err, uint32_t code) {
  atomicOr(err, 1u << code);
}

// Inclusive wave scan (Hillis-Steele over 64 lanes with __shfl_up).
template <class T, class Op>
__device__ __forceinline__ T wave_inclusive_scan(T v, Op op) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    T o = __shfl_up(v, d, kWave);
    if (l >= d) v = op(v, o);
  }
  return v;
}

template <class T, class Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
#pragma unroll
  for (int d = kWave / 2; d >= 1; d >>= 1) v = op(v, __shfl_xor(v, d, kWave));
  return v;
}

struct OpAdd {
  template <class T> __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
  template <class T> __device__ __forceinline__ T operator()(T a, T b) const { return a > b ? a : b; }
};
struct OpMin {
  template <class T> __device__ __forceinline__ T operator()(T a, T b) const { return a < b ? a : b; }
};

// Block-wide exclusive scan for BLOCK threads (multiple of 64).  `lds` needs BLOCK/64
// entries.  Returns the exclusive prefix; *total receives the block aggregate.  Must be
// called by all threads.
template <int BLOCK, class T, class Op>
__device__ __forceinline__ T block_exclusive_scan(T v, T identity, Op op, T* lds, T* total) {
  constexpr int NW = BLOCK / kWave;
  T inc = wave_inclusive_scan(v, op);
  if (lane_id() == kWave - 1) lds[wave_id()] = inc;
  __syncthreads();
  if (threadIdx.x < kWave) {
    T w = (threadIdx.x < NW) ? lds[threadIdx.x] : identity;
    T wi = wave_inclusive_scan(w, op);
    if (threadIdx.x < NW) lds[threadIdx.x] = wi;
  }
  __syncthreads();
  T wave_prefix = (wave_id() == 0) ? identity : lds[wave_id() - 1];
  T excl_in_wave = __shfl_up(inc, 1, kWave);
  if (lane_id() == 0) excl_in_wave = identity;
  T r = op(wave_prefix, excl_in_wave);
  *total = lds[NW - 1];
  __syncthreads();
  return r;
}

template <int BLOCK, class T>
__device__ __forceinline__ T block_sum(T v, T* lds) {
  T t;
  (void)block_exclusive_scan<BLOCK>(v, T(0), OpAdd(), lds, &t);
  return t;
}

// (clock, source) sort key of rempi_encoder_cdc.cpp:152-162 as an unsigned 64-bit value:
// signed clock in the high half, signed source in the low half, both bias-flipped so that
// unsigned comparison equals the reference's signed (clock, source) order.
__device__ __host__ __forceinline__ uint64_t pack_key(int32_t clk, int32_t src) {
  return ((uint64_t)((uint32_t)clk ^ 0x80000000u) << 32) | (uint64_t)((uint32_t)src ^ 0x80000000u);
}
__device__ __host__ __forceinline__ int32_t key_clock(uint64_t k) { return (int32_t)((uint32_t)(k >> 32) ^ 0x80000000u); }
__device__ __host__ __forceinline__ int32_t key_source(uint64_t k) { return (int32_t)((uint32_t)k ^ 0x80000000u); }

// For kernels of a few waves whose run time is a chain of dependent steps (scans over the unit
// list, list walks): their waves issue ahead of the throughput kernels of other streams that
// share the SIMD.  Without it a 70 us scan takes milliseconds while a chain kernel runs.
__device__ __forceinline__ void latency_kernel() { __builtin_amdgcn_s_setprio(3); }

// The same key as the two signed words {source, clock} (an int2 in memory): the form in which
// a unit's keys are kept in clock order, at Unit::key_off, and handed to the replay side.
constexpr uint64_t kKeyBias = 0x8000000080000000ull;
__device__ __host__ __forceinline__ uint64_t key_words(uint64_t k) { return k ^ kKeyBias; }

__device__ __forceinline__ uint64_t sext(int32_t v) { return (uint64_t)(int64_t)v; }

// Where a unit's epoch line (sources and their last clocks, at most kMaxUnitSources entries)
// sits in the epoch scratch arrays: kMaxUnitSources entries per unit when the batch's units are
// few and large (stride != 0), else at the unit's T-order start (a unit has at least as many
// records as sources).
__device__ __forceinline__ int64_t epoch_slot(int64_t unit, int64_t a, int64_t stride) {
  return stride ? unit * stride : a;
}

// Unaligned-safe 8-byte little-endian store into the byte output (all CDC sections are
// 8-byte multiples and every unit starts 8-aligned, so these are aligned in practice).
__device__ __forceinline__ void st_u64(uint8_t* p, uint64_t v) { *reinterpret_cast<uint64_t*>(p) = v; }
__device__ __forceinline__ void st_u32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }
__device__ __forceinline__ uint64_t ld_u64(const uint8_t* p) { return *reinterpret_cast<const uint64_t*>(p); }
__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

}  // namespace cdcx
