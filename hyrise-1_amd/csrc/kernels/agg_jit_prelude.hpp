// Device prelude of the plan-compiled aggregation kernels (agg_jit, hyrise_amd_agg_jit.cpp). This file is compiled
// twice: by hipcc into the library (the host side uses JitArgs and checks the mirrored layouts) and, embedded as text,
// by hiprtc together with the source generated for one plan. It is self-contained (hiprtc has no system headers):
// the chunk descriptors mirror include/hyrise_amd.h (static_asserts in hyrise_amd_agg_jit.cpp), and the device
// helpers restate the ones of aggregate_stream.hip / aggregate_fused.hip that the generated kernel uses.
#pragma once

#ifdef __HIPCC_RTC__
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
using __hip_internal::uint8_t;
#else
#include <hip/hip_runtime.h>

#include <cstdint>
#endif

namespace hyj {

constexpr int WAVE = 64;
constexpr int R = 4;                    // rows per lane per step (consecutive rows)
constexpr int WAVES = 4;                // waves per workgroup
constexpr int STEPS = 16;               // 256-row steps of a 4096-row tile
constexpr int TILE = WAVE * R * STEPS;  // 4096 rows
constexpr int GROUPS = 4;               // table entries a wave accumulates at once
constexpr int CODES = 64;               // group codes of the per-wave entry table
constexpr int DICT_MAX = 63;            // dictionary entries a decode table holds
constexpr int PLIST = 64;               // tiles recorded per flush period
constexpr int FLUSH_STEPS = 512;        // 4 rows per lane per step: <= 2048 values per lane and period
constexpr int WINDOW = 18;              // binades a period's values may span (exact double partial sums)
constexpr int BASE_MAX = 200;           // fold pieces stay inside the 9 float limbs
constexpr int HDR_FIRST = 1, HDR_LAST = 2, HDR_ROWS = 3;  // record header words after the key words
enum : int32_t { OP_EQ = 0, OP_NE = 1, OP_LT = 2, OP_LE = 3, OP_GT = 4, OP_GE = 5, OP_ALL = 6, OP_NONE = 7,
                 OP_IS_NOT_NULL = 9 };

// mirrors of hy_column_chunk / hy_scan_chunk (include/hyrise_amd.h)
struct ColumnChunk {
  const void* data;
  const uint8_t* nulls;
  const void* dictionary;
  uint32_t size;
  uint32_t dictionary_size;
  int32_t kind;
  int32_t vid_width;
};
struct ScanChunk {
  ColumnChunk column;
  int32_t op;
  uint32_t search_vid;
  uint64_t out_begin;
  const uint32_t* vid_set;
};

constexpr int MAX_COLS = 8;
// One launch's run-time arguments (by value); everything about the plan's shape is compiled into the kernel.
struct JitArgs {
  const ColumnChunk* cols[MAX_COLS];  // per loaded column: its chunk descriptors (device)
  const ScanChunk* filter;            // fused TableScan: per chunk (device), or null
  const uint32_t* tile_chunk;
  const uint64_t* chunk_tile_begin;
  const uint32_t* chunk_size;
  const uint64_t* chunk_row_begin;
  unsigned long long* records;        // dense group records (initialised)
  uint32_t* deferred;                 // steps for agg_dense_fused, and their count
  uint32_t* n_deferred;
  uint32_t* error;
  uint64_t n_tiles;
};

#if defined(__HIPCC_RTC__) || defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) void lds_t;
typedef const __attribute__((address_space(1))) void gptr_t;

// lane id recomputed where used (not kept live across a step)
__device__ __forceinline__ uint32_t lane_id() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// 256 rows [base, base + 256) of a W-byte column into `lds` in row order (LDS-DMA, dword pieces; 16-byte pieces for
// 4-byte elements); at a chunk's end a piece is clamped to the last aligned piece holding a row of the chunk.
template <int W>
__device__ __forceinline__ void load_column(const void* data, uint32_t base, uint32_t size, unsigned char* lds) {
  const uint32_t lane = lane_id();
  const char* p = static_cast<const char*>(data);
  const uint64_t last = uint64_t(size - 1u) * W;
  const uint64_t b = uint64_t(base) * W;
  if constexpr (W == 4) {
    __builtin_amdgcn_global_load_lds((gptr_t*)(p + min(b + 16u * lane, last & ~uint64_t(15))), (lds_t*)lds, 16, 0, 0);
  } else if constexpr (W == 2) {
    __builtin_amdgcn_global_load_lds((gptr_t*)(p + min(b + 4u * lane, last & ~uint64_t(3))), (lds_t*)lds, 4, 0, 0);
    __builtin_amdgcn_global_load_lds((gptr_t*)(p + min(b + 256u + 4u * lane, last & ~uint64_t(3))),
                                     (lds_t*)(lds + 256), 4, 0, 0);
  } else {
    __builtin_amdgcn_global_load_lds((gptr_t*)(p + min(b + 4u * lane, last & ~uint64_t(3))), (lds_t*)lds, 4, 0, 0);
  }
}

// The same for a step that lies inside its chunk (no clamping): the column's uniform base plus 32-bit lane offsets
// (one SGPR base per column, the lane offsets shared by all columns of the same width).
template <int W>
__device__ __forceinline__ void load_column_inside(const void* data, uint32_t base, uint32_t lane, unsigned char* lds) {
  const char* pb = static_cast<const char*>(data) + uint64_t(base) * W;
  if constexpr (W == 4) {
    __builtin_amdgcn_global_load_lds((gptr_t*)(pb + 16u * lane), (lds_t*)lds, 16, 0, 0);
  } else if constexpr (W == 2) {
    __builtin_amdgcn_global_load_lds((gptr_t*)(pb + 4u * lane), (lds_t*)lds, 4, 0, 0);
    __builtin_amdgcn_global_load_lds((gptr_t*)(pb + 256u + 4u * lane), (lds_t*)(lds + 256), 4, 0, 0);
  } else {
    __builtin_amdgcn_global_load_lds((gptr_t*)(pb + 4u * lane), (lds_t*)lds, 4, 0, 0);
  }
}

// a lane's 4 rows of a staged W-byte column, zero-extended
template <int W>
__device__ __forceinline__ void read4(const unsigned char* col, uint32_t lane, uint32_t (&v)[R]) {
  if constexpr (W == 1) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(col + 4u * lane);
#pragma unroll
    for (int k = 0; k < R; ++k) v[k] = (w >> (8 * k)) & 0xFFu;
  } else if constexpr (W == 2) {
    const uint2 w = *reinterpret_cast<const uint2*>(col + 8u * lane);
    v[0] = w.x & 0xFFFFu;
    v[1] = w.x >> 16;
    v[2] = w.y & 0xFFFFu;
    v[3] = w.y >> 16;
  } else {
    const uint4 w = *reinterpret_cast<const uint4*>(col + 16u * lane);
    v[0] = w.x;
    v[1] = w.y;
    v[2] = w.z;
    v[3] = w.w;
  }
}

// ((id - lo) < span) != neg, and id < dsize (a NULL id never matches): the dictionary predicate as an id range
struct IdRange {
  uint32_t lo, span, neg, dsize;
};
__device__ __forceinline__ IdRange id_range(int32_t op, uint32_t svid, uint32_t dsize) {
  IdRange r{0u, 0u, 0u, dsize};
  switch (op) {
    case OP_EQ: r.lo = svid; r.span = 1; break;
    case OP_NE: r.lo = svid; r.span = 1; r.neg = 1; break;
    case OP_LT: r.span = svid; break;
    case OP_LE: r.span = svid + 1; break;
    case OP_GT: r.span = svid + 1; r.neg = 1; break;
    case OP_GE: r.span = svid; r.neg = 1; break;
    case OP_ALL:
    case OP_IS_NOT_NULL: r.neg = 1; break;
    default: break;  // OP_NONE (the host admits no other op)
  }
  return r;
}
__device__ __forceinline__ bool id_in_range(const IdRange& r, uint32_t id) {
  return ((id - r.lo < r.span) != (r.neg != 0)) && id < r.dsize;
}

__device__ __forceinline__ uint32_t wave_max_u(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), d, WAVE)));
  return v;
}
__device__ __forceinline__ uint32_t wave_min_u(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = min(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), d, WAVE)));
  return v;
}
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v |= __shfl_xor(v, d, WAVE);
  return v;
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// wave sum of 64-bit values through DPP (the total is read from lane 63)
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(v), CTRL, ROW_MASK, 0xf, false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(v >> 32), CTRL, ROW_MASK, 0xf, false);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  v += dpp64<0x111, 0xf>(v);
  v += dpp64<0x112, 0xf>(v);
  v += dpp64<0x114, 0xf>(v);
  v += dpp64<0x118, 0xf>(v);
  v += dpp64<0x142, 0xa>(v);
  v += dpp64<0x143, 0xc>(v);
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), 63);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), 63);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// adds the signed integer S * 2^p to a record's 32-bit-weighted limbs
__device__ __forceinline__ void add_scaled(unsigned long long* limbs, int n_limbs, int64_t S, int p) {
  if (S == 0) return;
  const bool neg = S < 0;
  const unsigned __int128 u =
      static_cast<unsigned __int128>(neg ? 0ull - static_cast<uint64_t>(S) : static_cast<uint64_t>(S)) << (p & 31);
  const int i = p >> 5;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int64_t piece = static_cast<int64_t>(static_cast<uint32_t>(u >> (32 * q)));
    if (piece && i + q < n_limbs) atomicAdd(limbs + i + q, static_cast<unsigned long long>(neg ? -piece : piece));
  }
}

__device__ __forceinline__ void defer_step(const JitArgs& a, uint32_t step_id) {
  if (lane_id() == 0) a.deferred[atomicAdd(a.n_deferred, 1u)] = step_id;
}
#endif

}  // namespace hyj
