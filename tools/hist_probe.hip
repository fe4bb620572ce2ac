// Digit-byte histogram probe for part2_hist_bytes (join.hip): per 4096-byte tile, the 256-bin histogram of its bytes,
// written digit-major (hist[d * n_tiles + tile], the radix passes' layout) or tile-major. Variants:
//   0: one tile per workgroup, one LDS histogram, 16 ds_add per thread (the round-4 kernel)
//   1: eight tiles per workgroup, all loads first (the round-5 kernel)
//   2: one tile per workgroup, one histogram per wave (summed at the end)
//   3: one tile per workgroup, 8 copies per bin interleaved (bin * 8 + lane % 8)
//   4: variant 0 without the atomics (loads + histogram writes only)
//   5: variant 0 written tile-major (contiguous histogram rows)
//   6: eight tiles per workgroup, the radix passes' segmented layout (263-tile segments, entry (d, t) at
//      seg * 263 * 256 + d * 263 + t), XCD-contiguous groups
//   7: one tile per workgroup, the same layout, XCD-contiguous tiles (the round-4 kernel's geometry)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hist_probe tools/hist_probe.hip
#include <hip/hip_runtime.h>

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

constexpr uint32_t TILE = 4096;
constexpr uint32_t THREADS = 256;

__device__ __forceinline__ void count16(uint32_t* h, const uint4& u, uint32_t mul, uint32_t add) {
  const uint32_t words[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 16; ++i) atomicAdd(&h[((words[i >> 2] >> (8 * (i & 3))) & 0xFFu) * mul + add], 1u);
}

__device__ __forceinline__ uint32_t xcd_map(uint32_t b, uint32_t n) {
  const uint32_t q = n / 8, r = n % 8, x = b % 8;
  return x * q + min(x, r) + b / 8;
}
constexpr uint32_t SEG = 263;

template <int TPW>
__global__ __launch_bounds__(THREADS) void hist_seg_kernel(const uint8_t* __restrict__ dig, uint32_t n_tiles,
                                                           uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_h[TPW * 256];
  const uint32_t n_groups = (n_tiles + TPW - 1) / TPW;
  const uint32_t t0 = xcd_map(blockIdx.x, n_groups) * TPW;
  const uint32_t nt = min(static_cast<uint32_t>(TPW), n_tiles - t0);
  for (uint32_t i = threadIdx.x; i < TPW * 256; i += THREADS) s_h[i] = 0;
  __syncthreads();
  uint4 u[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
    if (i < nt) u[i] = reinterpret_cast<const uint4*>(dig + static_cast<uint64_t>(t0 + i) * TILE)[threadIdx.x];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
    if (i < nt) count16(s_h + i * 256, u[i], 1, 0);
  __syncthreads();
  for (uint32_t i = 0; i < nt; ++i) {
    const uint32_t t = t0 + i, sg = t / SEG, tin = t % SEG, st = min(SEG, n_tiles - sg * SEG);
    hist[static_cast<uint64_t>(sg) * SEG * 256 + threadIdx.x * st + tin] = s_h[i * 256 + threadIdx.x];
  }
}

template <int V>
__global__ __launch_bounds__(THREADS) void hist_kernel(const uint8_t* __restrict__ dig, uint32_t n_tiles,
                                                       uint32_t* __restrict__ hist) {
  constexpr int TPW = V == 1 ? 8 : 1;
  constexpr int COPIES = V == 2 ? 4 : V == 3 ? 8 : 1;
  __shared__ uint32_t s_h[TPW * 256 * COPIES];
  const uint32_t t0 = blockIdx.x * TPW;
  if (t0 >= n_tiles) return;
  for (uint32_t i = threadIdx.x; i < TPW * 256 * COPIES; i += THREADS) s_h[i] = 0;
  __syncthreads();
  uint4 u[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
    u[i] = reinterpret_cast<const uint4*>(dig + static_cast<uint64_t>(t0 + i) * TILE)[threadIdx.x];
  if constexpr (V == 4) {
    if (u[0].x == 0x12345678u) s_h[0] = 1;  // keep the load
  } else if constexpr (V == 2) {
    count16(s_h + (threadIdx.x / 64) * 256, u[0], 1, 0);
  } else if constexpr (V == 3) {
    count16(s_h, u[0], 8, threadIdx.x & 7u);
  } else {
#pragma unroll
    for (int i = 0; i < TPW; ++i) count16(s_h + i * 256, u[i], 1, 0);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const uint32_t d = threadIdx.x;
    uint32_t c = 0;
    if constexpr (COPIES > 1 && V == 2) {
      for (int k = 0; k < COPIES; ++k) c += s_h[k * 256 + d];
    } else if constexpr (V == 3) {
      for (int k = 0; k < COPIES; ++k) c += s_h[d * 8 + k];
    } else {
      c = s_h[i * 256 + d];
    }
    if constexpr (V == 5)
      hist[static_cast<uint64_t>(t0 + i) * 256 + d] = c;
    else
      hist[static_cast<uint64_t>(d) * n_tiles + t0 + i] = c;
  }
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 276000000ull;
  const uint32_t n_tiles = static_cast<uint32_t>(n / TILE) & ~7u;
  std::vector<uint8_t> h(uint64_t(n_tiles) * TILE);
  uint64_t x = 88172645463325252ull;
  for (auto& b : h) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    b = static_cast<uint8_t>(x);
  }
  uint8_t* d_dig;
  uint32_t* d_hist;
  CK(hipMalloc(&d_dig, h.size()));
  CK(hipMalloc(&d_hist, uint64_t(n_tiles) * 256 * 4));
  CK(hipMemcpy(d_dig, h.data(), h.size(), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](int v) {
    auto launch = [&]() {
      switch (v) {
        case 0: hist_kernel<0><<<n_tiles, THREADS>>>(d_dig, n_tiles, d_hist); break;
        case 1: hist_kernel<1><<<(n_tiles + 7) / 8, THREADS>>>(d_dig, n_tiles, d_hist); break;
        case 2: hist_kernel<2><<<n_tiles, THREADS>>>(d_dig, n_tiles, d_hist); break;
        case 3: hist_kernel<3><<<n_tiles, THREADS>>>(d_dig, n_tiles, d_hist); break;
        case 4: hist_kernel<4><<<n_tiles, THREADS>>>(d_dig, n_tiles, d_hist); break;
        case 5: hist_kernel<5><<<n_tiles, THREADS>>>(d_dig, n_tiles, d_hist); break;
        case 6: hist_seg_kernel<8><<<(n_tiles + 7) / 8, THREADS>>>(d_dig, n_tiles, d_hist); break;
        default: hist_seg_kernel<1><<<n_tiles, THREADS>>>(d_dig, n_tiles, d_hist); break;
      }
    };
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < 10; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    // check: total count of tile 0 .. = TILE per tile (variants 0-3, 5)
    std::vector<uint32_t> hh(uint64_t(n_tiles) * 256);
    CK(hipMemcpy(hh.data(), d_hist, hh.size() * 4, hipMemcpyDeviceToHost));
    uint64_t tot = 0;
    for (auto c : hh) tot += c;
    std::printf("{\"variant\": %d, \"ms\": %.4f, \"GBps_bytes\": %.1f, \"count_ok\": %d}\n", v, ms / 10,
                double(h.size()) / (ms / 10 * 1e-3) / 1e9, v == 4 ? -1 : int(tot == h.size()));
  };
  for (int v = 0; v <= 7; ++v) run(v);
  CK(hipFree(d_dig));
  CK(hipFree(d_hist));
  return 0;
}
