// wave.hpp -- wave64 helpers (CDNA: 64 lanes, 64-bit ballots).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hrf {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Add `val` at base[key] for every active lane with one atomic per distinct key per wave
// (labels are piecewise constant along a raster row, so a wave usually holds 1-3 keys).
// All 64 lanes must call it (uniform control flow); inactive lanes pass active=false.
template <class T>
__device__ __forceinline__ void agg_atomic_add(T *base, int64_t key, T val, bool active) {
  unsigned long long pending = __ballot(active);
  const int lane = lane_id();
  while (pending) {
    const int leader = __ffsll((long long)pending) - 1;
    const int64_t k = __shfl(key, leader, 64);
    const bool mine = active && key == k;
    const unsigned long long same = __ballot(mine);
    const T s = wave_sum<T>(mine ? val : T(0));
    if (lane == leader) atomicAdd(base + k, s);
    if (mine) active = false;
    pending &= ~same;
  }
}

// Inclusive prefix sum across the wave (Hillis-Steele with shuffles).
template <class T>
__device__ __forceinline__ T wave_inclusive_scan(T v) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

}  // namespace hrf
