// TableScan probe (config 2 shape: SF10 l_quantity, u8 value ids, 100,000-row chunks, RowID output): the product's
// scan_kernel (csrc/kernels/scan.hip: 4-tile segments, workgroup-staged stores) against scan_dict8_kernel below
// (dword loads, ballot-placed matches, wave-private LDS staging), on the same descriptors; outputs and per-chunk
// counts compared. Measured (profiles/r05_scan_probe.jsonl): 0.108 vs 0.142 ms (0.165 ms storing from registers).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o tools/scan_probe tools/scan_probe.hip
#include "../hyrise-1_amd/csrc/kernels/scan.hip"

namespace hyk {
// ------------------------------------------------------------------------------------------------------------
// 1-byte value ids without LDS staging (an alternative to scan_kernel for u8 ids; measured slower, not in the product): lane l of wave w reads dword i * 64 + l of the wave's span, i.e. rows
// span + 256 i + 4 l + j (j = 0..3, one 256-byte coalesced load per wave and group). A lane's <= 4 matches of group i
// go to consecutive positions at the lane's prefix - three ballots over the bits of its count give it - of the wave's
// own LDS slice, which the wave then stores coalesced (8-byte RowIDs, streaming). One barrier pair per workgroup (the
// segment's look-back), no per-tile block scans or workgroup barriers around the staging (scan_kernel's LDS stores
// conflicted about once per instruction, profiles/r04_pmc_scan_kernel_sq.txt). Storing each lane's matches straight
// from registers measured 0.165 ms against 0.108 (tools/scan_probe.hip): the partial lines cost more than the LDS.
// G groups of 256 rows per wave: a workgroup (segment) covers 4 * 256 * G rows, G = 16 -> 16384 = scan_kernel's
// 4-tile segment, so the host's segment geometry is unchanged.
// ------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t match4_dict(const hy_scan_chunk& ch, uint32_t v, uint32_t valid) {
  const uint32_t null_vid = static_cast<uint32_t>(ch.column.dictionary_size);
  const uint32_t s = static_cast<uint32_t>(ch.search_vid);
  const int op = ch.op;
  uint32_t m = 0;
  if (op == HY_OP_IS_NULL) {
#pragma unroll
    for (int j = 0; j < 4; ++j) m |= static_cast<uint32_t>(((v >> (8 * j)) & 0xFFu) == null_vid) << j;
  } else if (op == HY_OP_VID_SET) {
    const uint32_t* __restrict__ set = ch.vid_set;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t vid = (v >> (8 * j)) & 0xFFu;
      m |= static_cast<uint32_t>(vid != null_vid && ((set[vid >> 5] >> (vid & 31)) & 1u)) << j;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t vid = (v >> (8 * j)) & 0xFFu;
      m |= static_cast<uint32_t>(vid != null_vid && cmp_op<uint32_t>(op, vid, s)) << j;
    }
  }
  return m & valid;
}

// LDS written by some lanes of a wave and read by others: the wave's own ordering point (no workgroup barrier).
__device__ __forceinline__ void scan_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool OUT_ROWID, int G>
__global__ __launch_bounds__(SCAN_THREADS) void scan_dict8_kernel(ScanLaunchDesc d, void* __restrict__ out_any,
                                                                  uint32_t* __restrict__ counts) {
  constexpr uint32_t NW = SCAN_THREADS / WAVE;
  __shared__ uint32_t s_w[NW + 1];
  __shared__ uint32_t s_stage[NW][256];
  __shared__ uint64_t s_tile;
  __shared__ uint32_t s_chunk;
  __shared__ uint64_t s_prefix;
  if (threadIdx.x == 0) {
    const uint64_t tile = atomicAdd(d.ticket, 1u);
    s_tile = tile;
    s_chunk = tile < d.n_tiles ? d.tile_chunk[tile] : 0u;
  }
  __syncthreads();
  const uint64_t tile = s_tile;
  if (tile >= d.n_tiles) return;
  const uint32_t c = s_chunk;
  const hy_scan_chunk ch = d.chunks[c];
  const uint64_t first_tile = d.chunk_tile_begin[c];
  const uint32_t n = ch.column.size;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = __lane_id();
  const uint32_t wrow0 = static_cast<uint32_t>(tile - first_tile) * (NW * 256u * G) + w * (256u * G);
  const uint8_t* __restrict__ data = static_cast<const uint8_t*>(ch.column.data);
  uint32_t m[G];
  {
    uint32_t v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {  // all loads in flight first; the chunk's last dword is read byte by byte
      const uint32_t r = wrow0 + g * 256u + lane * 4u;
      if (r + 4 <= n) {
        v[g] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(data + r));
      } else {
        v[g] = 0;
        for (uint32_t j = 0; j < 4 && r + j < n; ++j) v[g] |= static_cast<uint32_t>(data[r + j]) << (8 * j);
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t r = wrow0 + g * 256u + lane * 4u;
      const uint32_t valid = r >= n ? 0u : (n - r >= 4 ? 0xFu : (1u << (n - r)) - 1u);
      m[g] = ch.op == HY_OP_NONE ? 0u : match4_dict(ch, v[g], valid);
    }
  }
  uint32_t mine = 0;
#pragma unroll
  for (int g = 0; g < G; ++g) mine += __popc(m[g]);
  const uint32_t wave_total = static_cast<uint32_t>(wave_sum64(mine));
  if (lane == 0) s_w[w] = wave_total;
  __syncthreads();
  if (threadIdx.x < WAVE) {  // wave 0: the segment's total, its look-back, the waves' offsets
    uint32_t seg_total = 0;
#pragma unroll
    for (uint32_t i = 0; i < NW; ++i) seg_total += s_w[i];
    uint64_t prefix = 0;
    if (tile == first_tile) {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, seg_total);
    } else {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_AGG, seg_total);
      prefix = lb_lookback_wave(d.status, first_tile, tile, d.error);
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, prefix + seg_total);
    }
    if (threadIdx.x == 0) {
      s_prefix = prefix;
      if (tile == d.chunk_tile_begin[c + 1] - 1) counts[d.chunk_index[c]] = static_cast<uint32_t>(prefix + seg_total);
    }
  }
  __syncthreads();
  uint64_t run = ch.out_begin + s_prefix;
  for (uint32_t i = 0; i < w; ++i) run += s_w[i];
  const uint64_t lt = lanemask_lt();
  const uint32_t cid = OUT_ROWID ? d.chunk_ids[c] : 0u;
  // per group: the lanes' matches staged in the wave's own LDS slice in row order, then stored coalesced (no
  // workgroup barrier: the slice is the wave's)
  uint32_t* stage = s_stage[w];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint32_t cnt = __popc(m[g]);  // 0..4: its prefix over the lanes from the ballots of its three bits
    const uint64_t b0 = __ballot(cnt & 1u), b1 = __ballot(cnt & 2u), b2 = __ballot(cnt & 4u);
    const uint32_t pre = __popcll(b0 & lt) + 2u * __popcll(b1 & lt) + 4u * __popcll(b2 & lt);
    const uint32_t tot = __popcll(b0) + 2u * __popcll(b1) + 4u * __popcll(b2);
    const uint32_t r = wrow0 + g * 256u + lane * 4u;
    uint32_t k = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((m[g] >> j) & 1u) stage[pre + k++] = r + j;
    scan_wave_sync();
    for (uint32_t i = lane; i < tot; i += WAVE) {
      if constexpr (OUT_ROWID)
        __builtin_nontemporal_store(static_cast<uint64_t>(cid) | (static_cast<uint64_t>(stage[i]) << 32),
                                    static_cast<uint64_t*>(out_any) + run + i);
      else
        static_cast<uint32_t*>(out_any)[run + i] = stage[i];
    }
    scan_wave_sync();  // the slice is rewritten by the next group
    run += tot;
  }
}


// Variant of scan_kernel<u8, DICT, RowID, SEG=4>: the four tiles' per-thread counts packed 16 bits each into one 64-bit
// value, so one workgroup scan gives every tile's positions (one barrier set per segment instead of one per tile), and
// the matches staged by 16 predicated LDS stores at popcount positions instead of a loop over the set bits.
constexpr int P_SEG = 4;
__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(8)))
void scan_packed_kernel(ScanLaunchDesc d, void* __restrict__ out_any, uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_stage[SCAN_TILE];
  __shared__ uint64_t s_w64[SCAN_THREADS / WAVE + 1];
  __shared__ uint64_t s_tile;
  __shared__ uint32_t s_chunk;
  __shared__ uint64_t s_prefix;
  if (threadIdx.x == 0) {
    const uint64_t tile = atomicAdd(d.ticket, 1u);
    s_tile = tile;
    s_chunk = tile < d.n_tiles ? d.tile_chunk[tile] : 0u;
  }
  __syncthreads();
  const uint64_t tile = s_tile;
  if (tile >= d.n_tiles) return;
  const uint32_t c = s_chunk;
  const hy_scan_chunk ch = d.chunks[c];
  const uint64_t first_tile = d.chunk_tile_begin[c];
  const uint32_t tile_row0 = static_cast<uint32_t>(tile - first_tile) * (P_SEG * SCAN_TILE);
  const uint32_t n = ch.column.size;
  uint32_t masks[P_SEG];
  {
    uint8_t v[P_SEG][16];
    u32x4 nl[P_SEG];
#pragma unroll
    for (int t = 0; t < P_SEG; ++t) {
      const uint32_t r0 = tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
      nl[t] = u32x4{0u, 0u, 0u, 0u};
      if (r0 < n && ch.op != HY_OP_NONE) load16(reinterpret_cast<const uint8_t*>(ch.column.data), r0, v[t]);
    }
#pragma unroll
    for (int t = 0; t < P_SEG; ++t)
      masks[t] = match_mask<uint8_t, MODE_DICT, uint8_t>(ch, tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD,
                                                         v[t], nl[t], ScanConst<uint8_t>{});
  }
  uint64_t packed = 0;
#pragma unroll
  for (int t = 0; t < P_SEG; ++t) packed |= static_cast<uint64_t>(__popc(masks[t])) << (16 * t);
  // workgroup exclusive scan of the packed counts (fields never carry: <= 4096 per tile)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint64_t incl = wave_inclusive_sum64(packed);
  if (__lane_id() == WAVE - 1) s_w64[w] = incl;
  __syncthreads();
  uint64_t before = 0, total = 0;
#pragma unroll
  for (int i = 0; i < SCAN_THREADS / WAVE; ++i) {
    const uint64_t x = s_w64[i];
    if (i < w) before += x;
    total += x;
  }
  const uint64_t excl = before + incl - packed;
  uint32_t seg_total = 0;
#pragma unroll
  for (int t = 0; t < P_SEG; ++t) seg_total += static_cast<uint32_t>((total >> (16 * t)) & 0xFFFFu);
  if (threadIdx.x < WAVE) {
    uint64_t prefix = 0;
    if (tile == first_tile) {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, seg_total);
    } else {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_AGG, seg_total);
      prefix = lb_lookback_wave(d.status, first_tile, tile, d.error);
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, prefix + seg_total);
    }
    if (threadIdx.x == 0) {
      s_prefix = prefix;
      if (tile == d.chunk_tile_begin[c + 1] - 1) counts[d.chunk_index[c]] = static_cast<uint32_t>(prefix + seg_total);
    }
  }
  __syncthreads();
  uint64_t run = ch.out_begin + s_prefix;
  const uint32_t cid = d.chunk_ids[c];
#pragma unroll
  for (int t = 0; t < P_SEG; ++t) {
    if (tile_row0 + t * SCAN_TILE >= n) break;  // uniform
    const uint32_t r0 = tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
    const uint32_t tile_total = static_cast<uint32_t>((total >> (16 * t)) & 0xFFFFu);
    const uint32_t pos = static_cast<uint32_t>((excl >> (16 * t)) & 0xFFFFu);
    const uint32_t m = masks[t];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) s_stage[pos + __popc(m & ((1u << i) - 1u))] = r0 + i;
    __syncthreads();
    uint64_t* out64 = static_cast<uint64_t*>(out_any) + run;
    for (uint32_t i = threadIdx.x; i < tile_total; i += SCAN_THREADS)
      out64[i] = static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[i]) << 32);  // plain stores (L2 / MALL)
    run += tile_total;
    __syncthreads();
  }
}

__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(8)))
void scan_seg_stage_kernel(ScanLaunchDesc d, void* __restrict__ out_any, uint32_t* __restrict__ counts) {
  __shared__ uint16_t s_stage[P_SEG * SCAN_TILE];  // the segment's match offsets (segment-relative, 16 bits)
  __shared__ uint64_t s_w64[SCAN_THREADS / WAVE + 1];
  __shared__ uint64_t s_tile;
  __shared__ uint32_t s_chunk;
  __shared__ uint64_t s_prefix;
  if (threadIdx.x == 0) {
    const uint64_t tile = atomicAdd(d.ticket, 1u);
    s_tile = tile;
    s_chunk = tile < d.n_tiles ? d.tile_chunk[tile] : 0u;
  }
  __syncthreads();
  const uint64_t tile = s_tile;
  if (tile >= d.n_tiles) return;
  const uint32_t c = s_chunk;
  const hy_scan_chunk ch = d.chunks[c];
  const uint64_t first_tile = d.chunk_tile_begin[c];
  const uint32_t tile_row0 = static_cast<uint32_t>(tile - first_tile) * (P_SEG * SCAN_TILE);
  const uint32_t n = ch.column.size;
  uint32_t masks[P_SEG];
  {
    uint8_t v[P_SEG][16];
    u32x4 nl[P_SEG];
#pragma unroll
    for (int t = 0; t < P_SEG; ++t) {
      const uint32_t r0 = tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
      nl[t] = u32x4{0u, 0u, 0u, 0u};
      if (r0 < n && ch.op != HY_OP_NONE) load16(reinterpret_cast<const uint8_t*>(ch.column.data), r0, v[t]);
    }
#pragma unroll
    for (int t = 0; t < P_SEG; ++t)
      masks[t] = match_mask<uint8_t, MODE_DICT, uint8_t>(ch, tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD,
                                                         v[t], nl[t], ScanConst<uint8_t>{});
  }
  uint64_t packed = 0;
#pragma unroll
  for (int t = 0; t < P_SEG; ++t) packed |= static_cast<uint64_t>(__popc(masks[t])) << (16 * t);
  // workgroup exclusive scan of the packed counts (fields never carry: <= 4096 per tile)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint64_t incl = wave_inclusive_sum64(packed);
  if (__lane_id() == WAVE - 1) s_w64[w] = incl;
  __syncthreads();
  uint64_t before = 0, total = 0;
#pragma unroll
  for (int i = 0; i < SCAN_THREADS / WAVE; ++i) {
    const uint64_t x = s_w64[i];
    if (i < w) before += x;
    total += x;
  }
  const uint64_t excl = before + incl - packed;
  uint32_t seg_total = 0;
#pragma unroll
  for (int t = 0; t < P_SEG; ++t) seg_total += static_cast<uint32_t>((total >> (16 * t)) & 0xFFFFu);
  if (threadIdx.x < WAVE) {
    uint64_t prefix = 0;
    if (tile == first_tile) {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, seg_total);
    } else {
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_AGG, seg_total);
      prefix = lb_lookback_wave(d.status, first_tile, tile, d.error);
      if (threadIdx.x == 0) lb_publish(&d.status[tile], LB_FLAG_PREFIX, prefix + seg_total);
    }
    if (threadIdx.x == 0) {
      s_prefix = prefix;
      if (tile == d.chunk_tile_begin[c + 1] - 1) counts[d.chunk_index[c]] = static_cast<uint32_t>(prefix + seg_total);
    }
  }
  __syncthreads();
  const uint64_t run = ch.out_begin + s_prefix;
  const uint32_t cid = d.chunk_ids[c];
  // every tile's matches staged at once (positions from the packed scan), one barrier, then the segment's stores
  uint32_t tbase = 0;
#pragma unroll
  for (int t = 0; t < P_SEG; ++t) {
    const uint32_t pos = tbase + static_cast<uint32_t>((excl >> (16 * t)) & 0xFFFFu);
    const uint32_t m = masks[t];
    const uint32_t o0 = t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((m >> i) & 1u) s_stage[pos + __popc(m & ((1u << i) - 1u))] = static_cast<uint16_t>(o0 + i);
    tbase += static_cast<uint32_t>((total >> (16 * t)) & 0xFFFFu);
  }
  __syncthreads();
  uint64_t* out64 = static_cast<uint64_t*>(out_any) + run;
  for (uint32_t i = threadIdx.x; i < seg_total; i += SCAN_THREADS)
    __builtin_nontemporal_store(static_cast<uint64_t>(cid) | (static_cast<uint64_t>(tile_row0 + s_stage[i]) << 32),
                                out64 + i);
}

// Ceilings for the same grid: every workgroup only streams its share of the output (27.6 M 8-byte RowIDs, coalesced,
// streaming stores), or only loads its 16384 ids and counts the matches (no stores but the count).
__global__ __launch_bounds__(SCAN_THREADS) void store_only_kernel(uint64_t n_out, uint32_t n_wg, uint64_t* __restrict__ out) {
  const uint64_t per = (n_out + n_wg - 1) / n_wg;
  const uint64_t b = per * blockIdx.x, e = min(n_out, b + per);
  for (uint64_t i = b + threadIdx.x; i < e; i += SCAN_THREADS) __builtin_nontemporal_store(i, out + i);
}
__global__ __launch_bounds__(SCAN_THREADS) void store16_only_kernel(uint64_t n_out, uint32_t n_wg, uint64_t* __restrict__ out) {
  const uint64_t per = ((n_out + n_wg - 1) / n_wg + 1) & ~uint64_t(1);  // even: 16-byte aligned pairs
  const uint64_t b = per * blockIdx.x, e = min(n_out, b + per);
  for (uint64_t i = b + 2 * threadIdx.x; i + 1 < e; i += 2 * SCAN_THREADS) {
    u32x4 v = {static_cast<uint32_t>(i), 7u, static_cast<uint32_t>(i + 1), 7u};
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + i));
  }
}
__global__ __launch_bounds__(SCAN_THREADS) void store_plain_kernel(uint64_t n_out, uint32_t n_wg, uint64_t* __restrict__ out) {
  const uint64_t per = (n_out + n_wg - 1) / n_wg;
  const uint64_t b = per * blockIdx.x, e = min(n_out, b + per);
  for (uint64_t i = b + threadIdx.x; i < e; i += SCAN_THREADS) out[i] = i;
}
__global__ __launch_bounds__(SCAN_THREADS) void load_count_kernel(const uint8_t* __restrict__ v, uint64_t n,
                                                                  uint32_t* __restrict__ sink) {
  const uint64_t r0 = static_cast<uint64_t>(blockIdx.x) * 16384 + threadIdx.x * 16;
  uint32_t c = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint64_t r = r0 + t * 4096;
    if (r + 16 <= n) {
      const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(v + r));
      const uint32_t w[4] = {x[0], x[1], x[2], x[3]};
#pragma unroll
      for (int i = 0; i < 16; ++i) c += ((w[i >> 2] >> (8 * (i & 3))) & 0xFFu) < 23u;
    }
  }
  if (c == 0xFFFFFFFFu) sink[0] = c;
}
// Two-pass form (round 6): seg_count_kernel counts each 4-tile segment's matches (ids read once), scan_write_kernel
// re-reads the ids and takes its segment's output position from the counts of the <= 6 segments before it in its
// chunk (no look-back, no ticket: every workgroup stores as soon as its own loads are back).
__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(8)))
void seg_count_kernel(ScanLaunchDesc d, uint32_t* __restrict__ seg_cnt) {
  __shared__ uint32_t s_scratch[SCAN_THREADS / WAVE + 1];
  const uint64_t tile = blockIdx.x;
  const uint32_t c = d.tile_chunk[tile];
  const hy_scan_chunk ch = d.chunks[c];
  const uint32_t row0 = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * (4 * SCAN_TILE);
  const uint32_t n = ch.column.size;
  uint32_t mine = 0;
  uint8_t v[4][16];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t r0 = row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
    if (r0 < n) load16(reinterpret_cast<const uint8_t*>(ch.column.data), r0, v[t]);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t r0 = row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
    if (r0 < n) mine += __popc(match_mask<uint8_t, MODE_DICT, uint8_t>(ch, r0, v[t], u32x4{0u, 0u, 0u, 0u}, {}));
  }
  uint32_t total;
  block_exclusive_sum<SCAN_THREADS>(mine, s_scratch, &total);
  if (threadIdx.x == 0) seg_cnt[tile] = total;
}

__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(8)))
void scan_write_kernel(ScanLaunchDesc d, const uint32_t* __restrict__ seg_cnt, uint64_t* __restrict__ out_any,
                       uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_stage[SCAN_TILE];
  __shared__ uint32_t s_scratch[SCAN_THREADS / WAVE + 1];
  __shared__ uint32_t s_prefix;
  const uint64_t tile = blockIdx.x;
  const uint32_t c = d.tile_chunk[tile];
  const hy_scan_chunk ch = d.chunks[c];
  const uint64_t first_tile = d.chunk_tile_begin[c];
  const uint32_t tile_row0 = static_cast<uint32_t>(tile - first_tile) * (4 * SCAN_TILE);
  const uint32_t n = ch.column.size;
  uint32_t masks[4];
  {
    uint8_t v[4][16];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t r0 = tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
      if (r0 < n) load16(reinterpret_cast<const uint8_t*>(ch.column.data), r0, v[t]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t r0 = tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
      masks[t] = r0 < n ? match_mask<uint8_t, MODE_DICT, uint8_t>(ch, r0, v[t], u32x4{0u, 0u, 0u, 0u}, {}) : 0u;
    }
  }
  if (threadIdx.x < WAVE) {
    const uint64_t before = tile - first_tile;
    uint32_t p = threadIdx.x < before ? seg_cnt[first_tile + threadIdx.x] : 0u;
    for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
    if (threadIdx.x == 0) {
      s_prefix = p;
      if (tile + 1 == d.chunk_tile_begin[c + 1]) counts[d.chunk_index[c]] = p + seg_cnt[tile];
    }
  }
  __syncthreads();
  uint64_t run = ch.out_begin + s_prefix;
  const uint32_t cid = d.chunk_ids[c];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (tile_row0 + t * SCAN_TILE >= n) break;
    const uint32_t r0 = tile_row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
    uint32_t tile_total;
    uint32_t pos = block_exclusive_sum<SCAN_THREADS>(__popc(masks[t]), s_scratch, &tile_total);
    uint32_t m = masks[t];
    while (m) {
      const int i = __builtin_ctz(m);
      m &= m - 1;
      s_stage[pos++] = r0 + i;
    }
    __syncthreads();
    uint64_t* out64 = out_any + run;
    const uint32_t lead = (reinterpret_cast<uintptr_t>(out64) & 15u) ? 1u : 0u;
    if (lead && threadIdx.x == 0 && tile_total)
      __builtin_nontemporal_store(static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[0]) << 32), out64);
    const uint32_t body = tile_total > lead ? tile_total - lead : 0u;
    u64x2* out128 = reinterpret_cast<u64x2*>(out64 + lead);
    for (uint32_t p = threadIdx.x; p < body / 2; p += SCAN_THREADS) {
      const uint32_t i = lead + 2 * p;
      u64x2 v;
      v.x = static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[i]) << 32);
      v.y = static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[i + 1]) << 32);
      __builtin_nontemporal_store(v, out128 + p);
    }
    if ((body & 1u) && threadIdx.x == SCAN_THREADS - 1)
      __builtin_nontemporal_store(static_cast<uint64_t>(cid) | (static_cast<uint64_t>(s_stage[tile_total - 1]) << 32),
                                  out64 + tile_total - 1);
    run += tile_total;
    __syncthreads();
  }
}
// Read ceilings (round 6): 4,201 workgroups read the 60 MB of ids in the product's tile layout (lane l of a tile
// reads bytes [16 l, 16 l + 16) of each 4096-byte tile) or contiguously, with streaming or plain loads, and count
// matches; the sink store depends on a runtime key so the loads stay.
template <int VARIANT>
__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(8)))
void read_probe_kernel(ScanLaunchDesc d, const uint8_t* __restrict__ v, uint64_t n, uint32_t key,
                       uint32_t* __restrict__ sink) {
  const uint8_t* base = v;
  uint64_t seg0 = static_cast<uint64_t>(blockIdx.x) * 16384;
  if (VARIANT == 4) {  // through the product's descriptor chain
    const uint32_t c = d.tile_chunk[blockIdx.x];
    base = static_cast<const uint8_t*>(d.chunks[c].column.data);
    seg0 = static_cast<uint64_t>(blockIdx.x - d.chunk_tile_begin[c]) * 16384;
  }
  uint32_t acc = 0;
  u32x4 x[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint64_t r = VARIANT == 2 ? seg0 + threadIdx.x * 64 + t * 16 : seg0 + t * 4096 + threadIdx.x * 16;
    const u32x4* p = reinterpret_cast<const u32x4*>(base + r);
    if (VARIANT == 0) x[t] = __builtin_nontemporal_load(p);
    else x[t] = *p;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t w = x[t][i];
      acc += ((w & 0xFFu) < 23u) + (((w >> 8) & 0xFFu) < 23u) + (((w >> 16) & 0xFFu) < 23u) + ((w >> 24) < 23u);
      acc ^= w;
    }
  if (acc == key) sink[threadIdx.x] = acc;
}
// Count-pass variants: VARIANT 1 = product loads + a plain u8 "< search_vid" compare (no match_mask), block sum;
// VARIANT 2 = as 1 with a wave reduction and one atomicAdd per wave (no barrier); VARIANT 3 = match_mask, wave reduce.
template <int VARIANT>
__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(8)))
void seg_count_var_kernel(ScanLaunchDesc d, uint32_t* __restrict__ seg_cnt) {
  __shared__ uint32_t s_scratch[SCAN_THREADS / WAVE + 1];
  const uint64_t tile = blockIdx.x;
  const uint32_t c = d.tile_chunk[tile];
  const hy_scan_chunk ch = d.chunks[c];
  const uint32_t row0 = static_cast<uint32_t>(tile - d.chunk_tile_begin[c]) * (4 * SCAN_TILE);
  const uint32_t n = ch.column.size;
  uint32_t mine = 0;
  u32x4 x[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t r0 = row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
    x[t] = r0 < n ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                        static_cast<const uint8_t*>(ch.column.data) + r0))
                  : u32x4{0u, 0u, 0u, 0u};
  }
  const uint32_t sv = static_cast<uint32_t>(ch.search_vid);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t r0 = row0 + t * SCAN_TILE + threadIdx.x * SCAN_ROWS_PER_THREAD;
    if (VARIANT == 3) {
      uint8_t v[16];
      __builtin_memcpy(v, &x[t], 16);
      mine += __popc(match_mask<uint8_t, MODE_DICT, uint8_t>(ch, r0, v, u32x4{0u, 0u, 0u, 0u}, {}));
    } else {
      const uint32_t valid = r0 >= n ? 0u : (n - r0) >= 16 ? 0xFFFFu : ((1u << (n - r0)) - 1u);
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) m |= static_cast<uint32_t>(((x[t][i >> 2] >> (8 * (i & 3))) & 0xFFu) < sv) << i;
      mine += __popc(m & valid);
    }
  }
  if (VARIANT == 1) {
    uint32_t total;
    block_exclusive_sum<SCAN_THREADS>(mine, s_scratch, &total);
    if (threadIdx.x == 0) seg_cnt[tile] = total;
  } else {
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(&seg_cnt[tile], mine);
  }
}
// One workgroup per chunk (round 6): 1024 threads walk the chunk in passes of 16384 rows (one 16-byte load per lane,
// the next pass's load issued before this pass's stores), so a chunk's output position is just the running count -
// no look-back, no ticket. Offsets are staged as u16 within the pass (32 KB LDS), then stored as 16-byte RowID pairs.
constexpr int CS_THREADS = 1024;
constexpr uint32_t CS_PASS = CS_THREADS * 16;
__global__ __launch_bounds__(CS_THREADS) void chunk_scan_kernel(const hy_scan_chunk* __restrict__ chunks,
                                                                const uint32_t* __restrict__ chunk_ids,
                                                                uint64_t* __restrict__ out_any,
                                                                uint32_t* __restrict__ counts) {
  __shared__ uint16_t s_stage[CS_PASS];
  __shared__ uint32_t s_scratch[CS_THREADS / WAVE + 1];
  const uint32_t c = blockIdx.x;
  const hy_scan_chunk ch = chunks[c];
  const uint32_t n = ch.column.size;
  const uint32_t cid = chunk_ids[c];
  const uint8_t* data = static_cast<const uint8_t*>(ch.column.data);
  uint64_t run = ch.out_begin;
  u32x4 nxt = {0u, 0u, 0u, 0u};
  if (threadIdx.x * 16 < n) nxt = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(data + threadIdx.x * 16));
  for (uint32_t p0 = 0; p0 < n; p0 += CS_PASS) {
    const u32x4 cur = nxt;
    const uint32_t rn = p0 + CS_PASS + threadIdx.x * 16;
    if (rn < n) nxt = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(data + rn));
    const uint32_t r0 = p0 + threadIdx.x * 16;
    uint8_t v[16];
    __builtin_memcpy(v, &cur, 16);
    uint32_t m = match_mask<uint8_t, MODE_DICT, uint8_t>(ch, r0, v, u32x4{0u, 0u, 0u, 0u}, {});
    uint32_t total;
    uint32_t pos = block_exclusive_sum<CS_THREADS>(__popc(m), s_scratch, &total);
    while (m) {
      const int i = __builtin_ctz(m);
      m &= m - 1;
      s_stage[pos++] = static_cast<uint16_t>(threadIdx.x * 16 + i);
    }
    __syncthreads();
    uint64_t* out64 = out_any + run;
    const uint32_t lead = (reinterpret_cast<uintptr_t>(out64) & 15u) ? 1u : 0u;
    if (lead && threadIdx.x == 0 && total)
      __builtin_nontemporal_store(static_cast<uint64_t>(cid) | (static_cast<uint64_t>(p0 + s_stage[0]) << 32), out64);
    const uint32_t body = total > lead ? total - lead : 0u;
    u64x2* out128 = reinterpret_cast<u64x2*>(out64 + lead);
    for (uint32_t q = threadIdx.x; q < body / 2; q += CS_THREADS) {
      const uint32_t i = lead + 2 * q;
      u64x2 w;
      w.x = static_cast<uint64_t>(cid) | (static_cast<uint64_t>(p0 + s_stage[i]) << 32);
      w.y = static_cast<uint64_t>(cid) | (static_cast<uint64_t>(p0 + s_stage[i + 1]) << 32);
      __builtin_nontemporal_store(w, out128 + q);
    }
    if ((body & 1u) && threadIdx.x == CS_THREADS - 1)
      __builtin_nontemporal_store(static_cast<uint64_t>(cid) | (static_cast<uint64_t>(p0 + s_stage[total - 1]) << 32),
                                  out64 + total - 1);
    run += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) counts[c] = static_cast<uint32_t>(run - ch.out_begin);
}
}  // namespace hyk

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 60007078ull;
  const uint32_t chunk = 100000;
  const uint32_t nc = static_cast<uint32_t>((n + chunk - 1) / chunk);
  std::vector<uint8_t> vids(n);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& b : vids) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    b = static_cast<uint8_t>(x % 50);
  }
  uint8_t* d_v;
  CK(hipMalloc(&d_v, n + 64));
  CK(hipMemcpy(d_v, vids.data(), n, hipMemcpyHostToDevice));
  std::vector<hy_scan_chunk> ch(nc);
  std::vector<uint64_t> seg_begin(nc + 1);
  std::vector<uint32_t> idx(nc), cid(nc);
  uint64_t run = 0;
  for (uint32_t c = 0; c < nc; ++c) {
    const uint32_t size = static_cast<uint32_t>(std::min<uint64_t>(chunk, n - uint64_t(c) * chunk));
    ch[c] = hy_scan_chunk{};
    ch[c].column.data = d_v + uint64_t(c) * chunk;
    ch[c].column.size = size;
    ch[c].column.dictionary_size = 50;
    ch[c].column.kind = HY_COL_DICT;
    ch[c].column.vid_width = 1;
    ch[c].search_vid = 23;
    ch[c].op = HY_OP_LT;
    ch[c].out_begin = uint64_t(c) * chunk;
    seg_begin[c] = run;
    run += ((size + hyk::SCAN_TILE - 1) / hyk::SCAN_TILE + 3) / 4;
    idx[c] = c;
    cid[c] = c + 7;
  }
  seg_begin[nc] = run;
  std::vector<uint32_t> owner(run);
  for (uint32_t c = 0; c < nc; ++c)
    for (uint64_t t = seg_begin[c]; t < seg_begin[c + 1]; ++t) owner[t] = c;
  hy_scan_chunk* d_ch;
  uint64_t *d_sb, *d_status, *d_out;
  uint32_t *d_owner, *d_idx, *d_cid, *d_ticket, *d_err, *d_counts;
  CK(hipMalloc(&d_ch, sizeof(hy_scan_chunk) * nc));
  CK(hipMalloc(&d_sb, 8 * (nc + 1)));
  CK(hipMalloc(&d_status, 8 * (run + 1)));
  CK(hipMalloc(&d_out, 8 * (n + 64)));
  CK(hipMalloc(&d_owner, 4 * run));
  CK(hipMalloc(&d_idx, 4 * nc));
  CK(hipMalloc(&d_cid, 4 * nc));
  CK(hipMalloc(&d_ticket, 4));
  CK(hipMalloc(&d_err, 4));
  CK(hipMalloc(&d_counts, 4 * nc));
  CK(hipMemcpy(d_ch, ch.data(), sizeof(hy_scan_chunk) * nc, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sb, seg_begin.data(), 8 * (nc + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_owner, owner.data(), 4 * run, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_idx, idx.data(), 4 * nc, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_cid, cid.data(), 4 * nc, hipMemcpyHostToDevice));
  CK(hipMemset(d_err, 0, 4));
  hyk::ScanLaunchDesc d{};
  d.chunks = d_ch;
  d.chunk_tile_begin = d_sb;
  d.tile_chunk = d_owner;
  d.chunk_index = d_idx;
  d.chunk_ids = d_cid;
  d.n_rows = n;
  d.n_chunks = nc;
  d.n_tiles = run;
  d.status = d_status;
  d.ticket = d_ticket;
  d.error = d_err;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<uint64_t> ref;
  std::vector<uint32_t> ref_counts;
  for (int v = 0; v < 4; ++v) {
    auto launch = [&]() {
      CK(hipMemsetAsync(d_status, 0, 8 * (run + 1)));
      CK(hipMemsetAsync(d_ticket, 0, 4));
      if (v == 0)
        hyk::scan_kernel<uint8_t, hyk::MODE_DICT, true, uint8_t, 4><<<run, hyk::SCAN_THREADS>>>(d, {}, d_out, d_counts);
      else if (v == 1)
        hyk::scan_dict8_kernel<true, 16><<<run, hyk::SCAN_THREADS>>>(d, d_out, d_counts);
      else if (v == 2)
        hyk::scan_packed_kernel<<<run, hyk::SCAN_THREADS>>>(d, d_out, d_counts);
      else
        hyk::scan_seg_stage_kernel<<<run, hyk::SCAN_THREADS>>>(d, d_out, d_counts);
    };
    CK(hipMemset(d_out, 0xFF, 8 * n));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> out(n);
    std::vector<uint32_t> counts(nc);
    CK(hipMemcpy(out.data(), d_out, 8 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(counts.data(), d_counts, 4 * nc, hipMemcpyDeviceToHost));
    if (v == 0) {
      ref = out;
      ref_counts = counts;
    }
    // events around each kernel: the memsets stay outside
    float total = 0;
    for (int r = 0; r < 20; ++r) {
      CK(hipMemsetAsync(d_status, 0, 8 * (run + 1)));
      CK(hipMemsetAsync(d_ticket, 0, 4));
      CK(hipEventRecord(a));
      if (v == 0)
        hyk::scan_kernel<uint8_t, hyk::MODE_DICT, true, uint8_t, 4><<<run, hyk::SCAN_THREADS>>>(d, {}, d_out, d_counts);
      else if (v == 1)
        hyk::scan_dict8_kernel<true, 16><<<run, hyk::SCAN_THREADS>>>(d, d_out, d_counts);
      else if (v == 2)
        hyk::scan_packed_kernel<<<run, hyk::SCAN_THREADS>>>(d, d_out, d_counts);
      else
        hyk::scan_seg_stage_kernel<<<run, hyk::SCAN_THREADS>>>(d, d_out, d_counts);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      total += ms;
    }
    uint64_t matches = 0;
    for (auto c : counts) matches += c;
    uint32_t err = 0;
    CK(hipMemcpy(&err, d_err, 4, hipMemcpyDeviceToHost));
    const double bytes = double(n) + 8.0 * double(matches);
    std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"matches\": %llu, \"alg_GBps\": %.1f, \"frac_spec\": %.3f, "
                "\"equal\": %d, \"error\": %u}\n",
                v == 0 ? "scan_kernel_seg4" : v == 1 ? "scan_dict8_kernel_g16" : v == 2 ? "scan_packed_kernel_plain_stores" : "scan_seg_stage_kernel", total / 20, (unsigned long long)matches,
                bytes / (total / 20 * 1e-3) / 1e9, bytes / (total / 20 * 1e-3) / 8e12,
                int(out == ref && counts == ref_counts), err);
  }
  {
    uint32_t* d_seg;
    CK(hipMalloc(&d_seg, 4 * run));
    CK(hipMemset(d_out, 0xFF, 8 * n));
    hyk::seg_count_kernel<<<run, hyk::SCAN_THREADS>>>(d, d_seg);
    hyk::scan_write_kernel<<<run, hyk::SCAN_THREADS>>>(d, d_seg, d_out, d_counts);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> out(n);
    std::vector<uint32_t> counts(nc);
    CK(hipMemcpy(out.data(), d_out, 8 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(counts.data(), d_counts, 4 * nc, hipMemcpyDeviceToHost));
    hipEvent_t m;
    CK(hipEventCreate(&m));
    float ta = 0, tb = 0;
    for (int r = 0; r < 20; ++r) {
      CK(hipEventRecord(a));
      hyk::seg_count_kernel<<<run, hyk::SCAN_THREADS>>>(d, d_seg);
      CK(hipEventRecord(m));
      hyk::scan_write_kernel<<<run, hyk::SCAN_THREADS>>>(d, d_seg, d_out, d_counts);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float x = 0, y = 0;
      CK(hipEventElapsedTime(&x, a, m));
      CK(hipEventElapsedTime(&y, m, b));
      ta += x;
      tb += y;
    }
    std::printf("{\"kernel\": \"two_pass\", \"count_ms\": %.4f, \"write_ms\": %.4f, \"ms\": %.4f, \"equal\": %d}\n",
                ta / 20, tb / 20, (ta + tb) / 20, int(out == ref && counts == ref_counts));
  }
  for (int v = 0; v < 5; ++v) {
    float total = 0;
    const uint64_t n_full = (n / 16384) * 16384;  // whole segments only (the probe reads 16384 bytes per workgroup)
    const uint32_t wgs = static_cast<uint32_t>(n_full / 16384);
    for (int r = 0; r < 20; ++r) {
      CK(hipMemset(d_out, 0, 8 * n));  // evict the ids from the Infinity Cache as the pipeline's writes would
      CK(hipEventRecord(a));
      if (v == 0) hyk::read_probe_kernel<0><<<wgs, hyk::SCAN_THREADS>>>(d, d_v, n, 0xFFFFFFFFu, d_counts);
      else if (v == 1) hyk::read_probe_kernel<1><<<wgs, hyk::SCAN_THREADS>>>(d, d_v, n, 0xFFFFFFFFu, d_counts);
      else if (v == 2) hyk::read_probe_kernel<2><<<wgs, hyk::SCAN_THREADS>>>(d, d_v, n, 0xFFFFFFFFu, d_counts);
      else if (v == 3) hyk::read_probe_kernel<1><<<wgs, hyk::SCAN_THREADS>>>(d, d_v, n, 0xFFFFFFFFu, d_counts);
      else hyk::read_probe_kernel<4><<<wgs, hyk::SCAN_THREADS>>>(d, d_v, n, 0xFFFFFFFFu, d_counts);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      total += ms;
    }
    static const char* names[] = {"read_tile_nt", "read_tile_plain", "read_contig_plain", "read_tile_plain_again",
                                  "read_tile_plain_descchain"};
    std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", names[v], total / 20,
                double(n_full) / (total / 20 * 1e-3) / 1e9);
  }
  {
    uint32_t* d_seg;
    CK(hipMalloc(&d_seg, 4 * run));
    for (int v = 1; v <= 3; ++v) {
      float total = 0;
      for (int r = 0; r < 20; ++r) {
        CK(hipMemset(d_out, 0, 8 * n));
        CK(hipMemset(d_seg, 0, 4 * run));
        CK(hipEventRecord(a));
        if (v == 1) hyk::seg_count_var_kernel<1><<<run, hyk::SCAN_THREADS>>>(d, d_seg);
        else if (v == 2) hyk::seg_count_var_kernel<2><<<run, hyk::SCAN_THREADS>>>(d, d_seg);
        else hyk::seg_count_var_kernel<3><<<run, hyk::SCAN_THREADS>>>(d, d_seg);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        total += ms;
      }
      std::vector<uint32_t> seg(run);
      CK(hipMemcpy(seg.data(), d_seg, 4 * run, hipMemcpyDeviceToHost));
      uint64_t sum = 0;
      for (auto x : seg) sum += x;
      std::printf("{\"kernel\": \"seg_count_var%d\", \"ms\": %.4f, \"matches\": %llu}\n", v, total / 20,
                  (unsigned long long)sum);
    }
  }
  {
    CK(hipMemset(d_out, 0xFF, 8 * n));
    hyk::chunk_scan_kernel<<<nc, hyk::CS_THREADS>>>(d_ch, d_cid, d_out, d_counts);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> out(n);
    std::vector<uint32_t> counts(nc);
    CK(hipMemcpy(out.data(), d_out, 8 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(counts.data(), d_counts, 4 * nc, hipMemcpyDeviceToHost));
    float total = 0;
    for (int r = 0; r < 20; ++r) {
      CK(hipEventRecord(a));
      hyk::chunk_scan_kernel<<<nc, hyk::CS_THREADS>>>(d_ch, d_cid, d_out, d_counts);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      total += ms;
    }
    std::printf("{\"kernel\": \"chunk_scan_1024\", \"ms\": %.4f, \"equal\": %d}\n", total / 20,
                int(out == ref && counts == ref_counts));
  }
  for (int v = 4; v < 8; ++v) {
    float total = 0;
    for (int r = 0; r < 20; ++r) {
      CK(hipEventRecord(a));
      if (v == 4)
        hyk::store_only_kernel<<<run, hyk::SCAN_THREADS>>>(27602404ull, static_cast<uint32_t>(run), d_out);
      else if (v == 6)
        hyk::store16_only_kernel<<<run, hyk::SCAN_THREADS>>>(27602404ull, static_cast<uint32_t>(run), d_out);
      else if (v == 7)
        hyk::store_plain_kernel<<<run, hyk::SCAN_THREADS>>>(27602404ull, static_cast<uint32_t>(run), d_out);
      else
        hyk::load_count_kernel<<<run, hyk::SCAN_THREADS>>>(d_v, n, d_counts);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      total += ms;
    }
    std::printf("{\"kernel\": \"%s\", \"ms\": %.4f}\n", v == 4 ? "store_only_221MB" : v == 5 ? "load_count_60MB" : v == 6 ? "store16_nt_221MB" : "store8_plain_221MB", total / 20);
  }
  return 0;
}
