// Device-side building blocks shared by the gfx950 kernels: MurmurHash2, wave64 ballot/prefix primitives,
// workgroup prefix sums and the decoupled look-back status words.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hyrise_amd.h"

namespace hyk {

constexpr int WAVE = 64;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------------------
// MurmurHash2 (32 bit), as reference src/lib/utils/murmur_hash.cpp:21-75 computes it over the sizeof(T) bytes of
// an arithmetic key (murmur_hash.hpp:11-14). Only 4- and 8-byte keys occur on the device path, so the tail switch
// of the byte loop is never taken.
// ------------------------------------------------------------------------------------------------------------
__host__ __device__ inline uint32_t murmur_mix_word(uint32_t h, uint32_t k) {
  const uint32_t m = 0x5bd1e995u;
  k *= m;
  k ^= k >> 24;
  k *= m;
  h *= m;
  h ^= k;
  return h;
}

__host__ __device__ inline uint32_t murmur_final(uint32_t h) {
  const uint32_t m = 0x5bd1e995u;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return h;
}

__host__ __device__ inline uint32_t murmur2_u32(uint32_t key_bits, uint32_t seed) {
  uint32_t h = seed ^ 4u;
  h = murmur_mix_word(h, key_bits);
  return murmur_final(h);
}

__host__ __device__ inline uint32_t murmur2_u64(uint64_t key_bits, uint32_t seed) {
  uint32_t h = seed ^ 8u;
  h = murmur_mix_word(h, static_cast<uint32_t>(key_bits));
  h = murmur_mix_word(h, static_cast<uint32_t>(key_bits >> 32));
  return murmur_final(h);
}

template <typename T>
__host__ __device__ inline uint32_t murmur2(T key, uint32_t seed) {
  if constexpr (sizeof(T) == 4) {
    uint32_t bits;
    __builtin_memcpy(&bits, &key, 4);
    return murmur2_u32(bits, seed);
  } else {
    uint64_t bits;
    __builtin_memcpy(&bits, &key, 8);
    return murmur2_u64(bits, seed);
  }
}

// Predicate of one row (HY_OP_*): value compare of the reference's with_comparator (type_comparison.hpp:100-123), or
// the value-id compare of the dictionary rewrite (single_column_table_scan_impl.hpp:52-76).
// Branch-free: the op selects which of (v < c, v == c, v > c) accept and whether the result is inverted (one nibble
// per op of CMP_OP_CODES: bit 0 <, bit 1 ==, bit 2 >, bit 3 invert; != is "not ==", so NaN != c holds as in C++,
// ALL / IS NOT NULL accept every row, NONE / IS NULL / anything else none). A switch here compiled to a scalar branch
// tree per element of the scans' unrolled 16-row loops (~10,000 instructions for one 4-tile u8 scan; round-6
// tools/scan_probe.hip: the count pass alone took 47 us against a 10 us read ceiling).
constexpr uint64_t CMP_OP_CODES = 0x80086431A2ull;  // ops 0..9: EQ NE LT LE GT GE ALL NONE IS_NULL IS_NOT_NULL
__device__ __forceinline__ uint32_t cmp_op_code(int op) {
  return static_cast<uint32_t>(op) < 10u ? static_cast<uint32_t>(CMP_OP_CODES >> (4 * op)) & 15u : 0u;
}
template <typename T>
__device__ __forceinline__ bool cmp_code(uint32_t code, T v, T c) {
  const bool r = ((code & 1u) != 0 & (v < c)) | ((code & 2u) != 0 & (v == c)) | ((code & 4u) != 0 & (v > c));
  return r != ((code & 8u) != 0);
}
template <typename T>
__device__ __forceinline__ bool cmp_op(int op, T v, T c) {
  return cmp_code<T>(cmp_op_code(op), v, c);
}

// A dictionary predicate (op, search value id s) of the host's rewrite over value ids whose NULL id is dsize (the
// dictionary size, reference dictionary_encoder.hpp: null_value_id = dictionary.size()), as one id range and one
// excluded id: a row matches iff (id - lo) < span and id != except. EQ [s, s+1), LT [0, s), LE [0, s+1), GT [s+1,
// dsize), GE [s, dsize), ALL / IS NOT NULL [0, dsize), IS NULL [dsize, dsize+1), NE [0, dsize) except s, NONE and
// the rest nothing; every range is clipped to [0, dsize] so the NULL id only ever matches IS NULL. Two compares per
// row instead of a compare per op: the scans' unrolled 16-row loops measured 25 -> 12 us for the count of config 2's
// 60 M u8 ids (round-6 tools/scan_probe.hip, seg_count_var3 vs _var1). Ids are compared as read (E-width, widened).
struct DictPred {
  uint32_t lo, span, except;
};
__device__ __forceinline__ DictPred dict_pred(int op, uint32_t s, uint32_t dsize) {
  const uint32_t s1 = s < dsize ? s + 1 : dsize;  // min(s + 1, dsize)
  const uint32_t s0 = s < dsize ? s : dsize;      // min(s, dsize)
  switch (op) {
    case HY_OP_EQ:
      return {s0, s1 - s0, dsize};
    case HY_OP_NE:
      return {0u, dsize, s};
    case HY_OP_LT:
      return {0u, s0, dsize};
    case HY_OP_LE:
      return {0u, s1, dsize};
    case HY_OP_GT:
      return {s1, dsize - s1, dsize};
    case HY_OP_GE:
      return {s0, dsize - s0, dsize};
    case HY_OP_ALL:
    case HY_OP_IS_NOT_NULL:
      return {0u, dsize, dsize};
    case HY_OP_IS_NULL:
      return {dsize, 1u, dsize + 1u};
    default:
      return {0u, 0u, 0u};
  }
}
__device__ __forceinline__ bool dict_match(const DictPred& p, uint32_t id) {
  return (id - p.lo < p.span) & (id != p.except);
}

// ------------------------------------------------------------------------------------------------------------
// std::string values on the device: packed string arrays (include/hyrise_amd.h, "Column chunk descriptors").
// ------------------------------------------------------------------------------------------------------------
struct DevString {
  const unsigned char* p;
  uint32_t n;
};

// String i of a packed string array of `count` strings
__device__ inline DevString packed_string(const void* packed, uint32_t count, uint32_t i) {
  const uint32_t* off = static_cast<const uint32_t*>(packed);
  const uint32_t b = off[i], e = off[i + 1];
  const uintptr_t bytes = (reinterpret_cast<uintptr_t>(packed) + 4ull * (count + 1) + 15) & ~uintptr_t(15);
  return DevString{reinterpret_cast<const unsigned char*>(bytes) + b, e - b};
}

// std::string::compare (char_traits<char>::compare: bytes as unsigned char, then the length): <0, 0, >0
__device__ inline int string_compare(DevString a, DevString b) {
  const uint32_t n = a.n < b.n ? a.n : b.n;
  for (uint32_t i = 0; i < n; ++i)
    if (a.p[i] != b.p[i]) return a.p[i] < b.p[i] ? -1 : 1;
  return a.n < b.n ? -1 : (a.n > b.n ? 1 : 0);
}

// HY_OP_EQ..HY_OP_GE applied to a three-way comparison result
__device__ inline bool cmp_result(int op, int c) {
  switch (op) {
    case HY_OP_EQ:
      return c == 0;
    case HY_OP_NE:
      return c != 0;
    case HY_OP_LT:
      return c < 0;
    case HY_OP_LE:
      return c <= 0;
    case HY_OP_GT:
      return c > 0;
    default:
      return c >= 0;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Wave64 helpers.
// ------------------------------------------------------------------------------------------------------------
__device__ inline int lane_id() { return __lane_id(); }

// XCD-aware workgroup -> tile map. Workgroups are dispatched round-robin over the 8 XCDs (workgroup b on XCD b % 8);
// this hands XCD x a contiguous range of tiles, taken in order. Neighbouring tiles then run on the same XCD at about
// the same time, so the 128-B lines they share at the edges of their output runs are completed in one L2 instead of
// being written back half-filled from two. A bijection on [0, n) for any n.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
  constexpr uint32_t X = 8;
  const uint32_t q = n / X, r = n % X, x = b % X;
  return x * q + min(x, r) + b / X;
}

__device__ inline uint64_t lanemask_lt() {
  const int l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Inclusive prefix sum over the 64 lanes of a wave.
__device__ inline uint32_t wave_inclusive_sum(uint32_t v) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint32_t o = __shfl_up(v, d, WAVE);
    if (__lane_id() >= d) v += o;
  }
  return v;
}

__device__ inline uint64_t wave_inclusive_sum64(uint64_t v) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const uint64_t o = __shfl_up(v, d, WAVE);
    if (__lane_id() >= d) v += o;
  }
  return v;
}

__device__ inline uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, WAVE);
  return v;
}

// Exclusive prefix over a workgroup of NT threads. Returns the exclusive prefix of v; *total = sum over the group.
// scratch: NT/64 + 1 uint32 in LDS.
template <int NT>
__device__ inline uint32_t block_exclusive_sum(uint32_t v, uint32_t* scratch, uint32_t* total) {
  constexpr int NW = NT / WAVE;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint32_t incl = wave_inclusive_sum(v);
  if (__lane_id() == WAVE - 1) scratch[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const uint32_t t = scratch[i];
      scratch[i] = run;
      run += t;
    }
    scratch[NW] = run;
  }
  __syncthreads();
  const uint32_t res = scratch[w] + incl - v;
  *total = scratch[NW];
  __syncthreads();
  return res;
}

// ------------------------------------------------------------------------------------------------------------
// Decoupled look-back status words (single-pass chained scan across workgroups).
//
// Each word is one naturally aligned 8-byte {flag, value} granule written by ONE agent-scope relaxed atomic store
// and polled by agent-scope relaxed atomic loads: the data is the flag, so no release/acquire fence is needed
// (MI355X_MICROARCH.md "Valid forms", R2 granule). Words are zeroed by a memset before every launch. Tile ids are
// handed out by an atomic ticket so a workgroup only ever waits on workgroups that are already running.
// ------------------------------------------------------------------------------------------------------------
constexpr uint64_t LB_FLAG_AGG = 1ull << 62;
constexpr uint64_t LB_FLAG_PREFIX = 2ull << 62;
constexpr uint64_t LB_VALUE_MASK = (1ull << 62) - 1;
constexpr uint32_t LB_MAX_SPINS = 1u << 22;

__device__ inline void lb_publish(uint64_t* word, uint64_t flag, uint64_t value) {
  __hip_atomic_store(word, flag | value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline uint64_t lb_poll(const uint64_t* word) {
  return __hip_atomic_load(const_cast<uint64_t*>(word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix for tile `tile`, looking back over tiles [first_tile, tile). Executed by one lane.
// Returns false (and sets *error) if a predecessor never published within the spin bound.
__device__ inline bool lb_lookback(const uint64_t* status, uint64_t first_tile, uint64_t tile, uint64_t* prefix,
                                   uint32_t* error) {
  uint64_t acc = 0;
  uint64_t j = tile;
  uint32_t spins = 0;
  while (j > first_tile) {
    const uint64_t s = lb_poll(&status[j - 1]);
    const uint64_t flag = s & ~LB_VALUE_MASK;
    if (flag == 0) {
      if (++spins > LB_MAX_SPINS) {
        __hip_atomic_store(error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *prefix = acc;
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    acc += s & LB_VALUE_MASK;
    if (flag == LB_FLAG_PREFIX) break;
    --j;
  }
  *prefix = acc;
  return true;
}

__device__ inline uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, WAVE);
  return v;
}

// Wave-parallel look-back: executed by ALL 64 lanes of one wave. Each round polls the 64 nearest unresolved
// predecessors at once; it stops at the nearest inclusive PREFIX (or the segment start [first_tile]) and sums the
// aggregates in between. Returns the exclusive prefix of `tile` (same value in every lane).
__device__ inline uint64_t lb_lookback_wave(const uint64_t* status, uint64_t first_tile, uint64_t tile,
                                            uint32_t* error) {
  const int lane = __lane_id();
  uint64_t acc = 0;
  int64_t hi = static_cast<int64_t>(tile) - 1;
  uint32_t spins = 0;
  while (hi >= static_cast<int64_t>(first_tile)) {
    const int64_t j = hi - lane;
    uint64_t v = LB_FLAG_PREFIX;  // before the segment start: inclusive prefix 0
    if (j >= static_cast<int64_t>(first_tile)) v = lb_poll(&status[j]);
    const uint64_t flag = v & ~LB_VALUE_MASK;
    const uint64_t pmask = __ballot(flag == LB_FLAG_PREFIX);
    const int stop = pmask ? __builtin_ctzll(pmask) : 63;
    const uint64_t upto = stop == 63 ? ~0ull : ((2ull << stop) - 1);
    if (__ballot(flag == 0) & upto) {
      if (++spins > LB_MAX_SPINS) {
        if (lane == 0) __hip_atomic_store(error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return acc;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const uint64_t mine = (lane <= stop && j >= static_cast<int64_t>(first_tile)) ? (v & LB_VALUE_MASK) : 0;
    acc += wave_sum64(mine);
    if (pmask) break;
    hi -= WAVE;
  }
  return acc;
}

// owner[t] = c for every tile t in [begin[c], begin[c+1]), c < n: lets a workgroup find its chunk / segment with one
// load instead of a dependent binary search over the prefix (each step of which is a global-memory round trip).
static __global__ void fill_tile_owner(const uint64_t* __restrict__ begin, uint32_t n, uint32_t* __restrict__ owner) {
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x)
    for (uint64_t t = begin[c]; t < begin[c + 1]; ++t) owner[t] = c;
}

}  // namespace hyk
