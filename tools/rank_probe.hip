// Stable in-wave ranking probe for the radix partition passes (join.hip): an item's rank among the same-digit items
// of its wave that precede it in (item k, lane) order.
//   1. order check: does one ds_add_rtn_u32 per item (atomicAdd returning the old count) hand out its values to the
//      lanes that hit the same counter in ascending lane order, and do consecutive instructions of a wave apply in
//      order? If so, rank = the returned value, with all 16 items' atomics issued back to back.
//   2. throughput of that ranking against the mask ranking (wave_rank_lds: or / read / clear the digit's lane mask,
//      read / advance its counter) over the same items.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/rank_probe tools/rank_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

constexpr int ITEMS = 16;
constexpr int WAVES = 4;

__device__ inline uint64_t lanemask_lt() {
  const int l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

__device__ __forceinline__ uint32_t rank_mask(uint32_t digit, bool active, uint64_t* wave_mask, uint32_t* wave_cnt) {
  uint32_t rank = 0;
  if (active) {
    const uint64_t me = 1ull << __lane_id();
    __hip_atomic_fetch_or(&wave_mask[digit], me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t peers = __hip_atomic_load(&wave_mask[digit], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(&wave_mask[digit], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t c = __hip_atomic_load(&wave_cnt[digit], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    rank = c + static_cast<uint32_t>(__popcll(peers & (me - 1)));
    if ((peers & ~((me << 1) - 1)) == 0)
      __hip_atomic_store(&wave_cnt[digit], c + static_cast<uint32_t>(__popcll(peers)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  return rank;
}

// MODE 0: mask ranking; 1: atomic-return ranking. digits: n items laid out tile-major (wave w, item k, lane l).
// active: items whose digit < 256 (>= 256 marks an inactive row). Writes each item's rank (order check) or a
// checksum (throughput).
template <int MODE, bool WRITE_RANKS>
__global__ __launch_bounds__(256) void rank_kernel(const uint32_t* __restrict__ digits, uint64_t n_tiles,
                                                   uint32_t* __restrict__ ranks, uint32_t* __restrict__ sink) {
  __shared__ uint32_t s_cnt[WAVES][256];
  __shared__ uint64_t s_mask[WAVES][256];
  const int w = threadIdx.x / 64, lane = __lane_id();
  uint32_t acc = 0;
  for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    for (int i = lane; i < 256; i += 64) {
      s_cnt[w][i] = 0;
      s_mask[w][i] = 0;
    }
    const uint32_t* d = digits + (t * WAVES + w) * (ITEMS * 64);
    uint32_t dg[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) dg[k] = d[k * 64 + lane];
    uint32_t r[ITEMS];
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < ITEMS; ++k) r[k] = rank_mask(dg[k] & 255u, dg[k] < 256u, s_mask[w], s_cnt[w]);
    } else {
#pragma unroll
      for (int k = 0; k < ITEMS; ++k)
        r[k] = dg[k] < 256u ? __hip_atomic_fetch_add(&s_cnt[w][dg[k]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                            : 0u;
    }
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
      if (WRITE_RANKS)
        ranks[(t * WAVES + w) * (ITEMS * 64) + k * 64 + lane] = r[k];
      else
        acc += r[k] * (k + 1);
    }
  }
  if (!WRITE_RANKS && acc == 0x9E3779B9u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t n_tiles = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 65536;
  const uint64_t n = n_tiles * WAVES * ITEMS * 64;
  const bool uniform = argc > 2;  // only uniform digits (the partition passes' case): throughput without collisions
  std::vector<uint32_t> h(n);
  uint64_t x = 88172645463325252ull;
  auto rnd = [&] {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  // per tile a distribution: uniform 256 digits / 4 digits (heavy collisions) / 1 digit, 50 % or 100 % active
  for (uint64_t t = 0; t < n_tiles * WAVES; ++t) {
    const int kind = uniform ? static_cast<int>(3 * (t % 2)) : static_cast<int>(t % 6);
    const uint32_t span = kind % 3 == 0 ? 256 : kind % 3 == 1 ? 4 : 1;
    const bool half = kind >= 3;
    for (int i = 0; i < ITEMS * 64; ++i) {
      const uint64_t v = rnd();
      uint32_t dig = static_cast<uint32_t>(v % span) * (256 / span);
      if (half && ((v >> 40) & 1)) dig = 256;
      h[t * ITEMS * 64 + i] = dig;
    }
  }
  uint32_t *d, *r, *sink;
  CK(hipMalloc(&d, n * 4));
  CK(hipMalloc(&r, n * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  // 1. order check against the expected stable ranks
  hipLaunchKernelGGL((rank_kernel<1, true>), dim3(2048), dim3(256), 0, 0, d, n_tiles, r, sink);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> got(n);
  CK(hipMemcpy(got.data(), r, n * 4, hipMemcpyDeviceToHost));
  uint64_t bad = 0, checked = 0;
  for (uint64_t t = 0; t < n_tiles * WAVES; ++t) {
    uint32_t cnt[256] = {0};
    for (int i = 0; i < ITEMS * 64; ++i) {  // (k, lane) order = index order
      const uint32_t dig = h[t * ITEMS * 64 + i];
      if (dig >= 256) continue;
      ++checked;
      if (got[t * ITEMS * 64 + i] != cnt[dig]) ++bad;
      ++cnt[dig];
    }
  }
  std::printf("{\"check\": \"atomic-return ranks == stable (item, lane) ranks\", \"items\": %llu, \"mismatches\": %llu}\n",
              (unsigned long long)checked, (unsigned long long)bad);
  hipLaunchKernelGGL((rank_kernel<0, true>), dim3(2048), dim3(256), 0, 0, d, n_tiles, r, sink);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(got.data(), r, n * 4, hipMemcpyDeviceToHost));
  bad = 0;
  for (uint64_t t = 0; t < n_tiles * WAVES; ++t) {
    uint32_t cnt[256] = {0};
    for (int i = 0; i < ITEMS * 64; ++i) {
      const uint32_t dig = h[t * ITEMS * 64 + i];
      if (dig >= 256) continue;
      if (got[t * ITEMS * 64 + i] != cnt[dig]) ++bad;
      ++cnt[dig];
    }
  }
  std::printf("{\"check\": \"mask ranks == stable ranks\", \"mismatches\": %llu}\n", (unsigned long long)bad);
  // 2. throughput
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {
    for (int grid : {1024, 2048, 4096}) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0));
        if (mode == 0)
          hipLaunchKernelGGL((rank_kernel<0, false>), dim3(grid), dim3(256), 0, 0, d, n_tiles, r, sink);
        else
          hipLaunchKernelGGL((rank_kernel<1, false>), dim3(grid), dim3(256), 0, 0, d, n_tiles, r, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
      }
      std::printf("{\"mode\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"items_per_ns\": %.1f, \"read_TBps\": %.2f}\n",
                  mode ? "atomic_rtn" : "mask", grid, best, n / (best * 1e6), n * 4 / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
