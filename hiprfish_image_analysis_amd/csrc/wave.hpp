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

// Count equal keys over the contiguous range [first, first + 64*STEPS) with coalesced loads:
// the wave keeps one uniform run (key, count); a step whose valid keys all equal the run just
// adds its popcount, any other step flushes the run and aggregates its own keys per distinct
// key (agg_atomic_add), then the run restarts at the key of lane 63.  A component spanning
// the range costs one atomic per wave instead of one per pixel.  key(i) < 0 = no key.
// All lanes of the wave must call it.
template <int STEPS, class KeyF>
__device__ __forceinline__ void wave_run_count(int32_t *base, int64_t first, int64_t n, KeyF key) {
  const int lane = lane_id();
  int32_t run = -1, cnt = 0;  // wave-uniform
#pragma unroll 1
  for (int i = 0; i < STEPS; ++i) {
    const int64_t e = first + (int64_t)i * 64 + lane;
    if (first + (int64_t)i * 64 >= n) break;
    const int32_t k = e < n ? key(e) : -1;
    const unsigned long long valid = __ballot(k >= 0);
    const unsigned long long same = __ballot(k >= 0 && k == run);
    if (same == valid) {
      cnt += __popcll(valid);
      continue;
    }
    if (run >= 0 && cnt && lane == 0) atomicAdd(base + run, cnt);
    agg_atomic_add<int32_t>(base, k >= 0 ? k : 0, 1, k >= 0);
    run = __shfl(k, 63, 64);
    cnt = 0;
  }
  if (run >= 0 && cnt && lane == 0) atomicAdd(base + run, cnt);
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
