// Infinity Cache (MALL) round-trip probe: does a produce -> consume hand-off through a REUSED staging buffer of
// B bytes stay on-die? For a total volume N, each block i runs
//   produce: src[i*B .. (i+1)*B) -> stage      (streaming read + write)
//   consume: stage -> dst[i*B .. (i+1)*B)      (read + streaming write)
// with stage reused by every block (B < N) or a fresh N-byte stage (B = N, the HBM round trip). The block loop is
// captured into one hipGraph so launch gaps are as in a prepared plan. Output: one line per (B, policy) with the
// time per GB of N and the rate over the four streams.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mall_probe tools/mall_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

template <bool NT_SRC>
__global__ __launch_bounds__(256) void produce(const uint4* __restrict__ src, uint4* __restrict__ stage, uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride) {
    uint4 v;
    if constexpr (NT_SRC) {
      v.x = __builtin_nontemporal_load(&src[i].x);
      v.y = __builtin_nontemporal_load(&src[i].y);
      v.z = __builtin_nontemporal_load(&src[i].z);
      v.w = __builtin_nontemporal_load(&src[i].w);
    } else {
      v = src[i];
    }
    v.x += 1u;
    stage[i] = v;
  }
}

template <bool NT_DST>
__global__ __launch_bounds__(256) void consume(const uint4* __restrict__ stage, uint4* __restrict__ dst, uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride) {
    uint4 v = stage[i];
    v.y ^= 3u;
    if constexpr (NT_DST) {
      __builtin_nontemporal_store(v.x, &dst[i].x);
      __builtin_nontemporal_store(v.y, &dst[i].y);
      __builtin_nontemporal_store(v.z, &dst[i].z);
      __builtin_nontemporal_store(v.w, &dst[i].w);
    } else {
      dst[i] = v;
    }
  }
}

// Re-read mode: kernel A reads a block of src (a histogram-like pass), kernel B reads the same block again and writes
// it to dst. Blocked (B < N): is B's re-read served on-die?
__global__ __launch_bounds__(256) void read_only(const uint4* __restrict__ src, uint64_t n, uint32_t* __restrict__ sink) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride) {
    const uint4 v = src[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t N = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4096ull) << 20;
  uint4 *src, *dst, *big;
  CK(hipMalloc(&src, N));
  CK(hipMalloc(&dst, N));
  CK(hipMalloc(&big, N));
  CK(hipMemset(src, 1, N));
  CK(hipMemset(dst, 0, N));
  CK(hipMemset(big, 0, N));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint64_t MB = 1ull << 20;
  std::vector<uint64_t> blocks = {16 * MB, 32 * MB, 64 * MB, 96 * MB, 128 * MB, 192 * MB, 256 * MB, 512 * MB, N};
  uint32_t* sink;
  CK(hipMalloc(&sink, 64));
  for (int ntd = 0; ntd < 2; ++ntd) {
    for (uint64_t B : blocks) {
      const uint64_t nb = N / B, n = B / 16;
      const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((n + 255) / 256, 256 * 16));
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (uint64_t i = 0; i < nb; ++i) {
        hipLaunchKernelGGL(read_only, dim3(grid), dim3(256), 0, s, src + i * n, n, sink);
        if (ntd)
          hipLaunchKernelGGL(consume<true>, dim3(grid), dim3(256), 0, s, src + i * n, dst + i * n, n);
        else
          hipLaunchKernelGGL(consume<false>, dim3(grid), dim3(256), 0, s, src + i * n, dst + i * n, n);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      float best = 1e30f;
      for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) best = std::min(best, ms);
      }
      std::printf("{\"mode\": \"reread\", \"block_MB\": %llu, \"nt_dst\": %d, \"ms\": %.4f, \"ms_per_GB\": %.4f}\n",
                  (unsigned long long)(B / MB), ntd, best, best / (N / 1e9));
      std::fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  if (argc > 2) return 0;
  for (int pol = 0; pol < 4; ++pol) {
    const bool nts = pol & 1, ntd = pol & 2;
    for (uint64_t B : blocks) {
      if (B > N) continue;
      const uint64_t nb = N / B;
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (uint64_t i = 0; i < nb; ++i) {
        uint4* stage = (B == N) ? big : big;  // the same region: reused when B < N
        const uint64_t n = B / 16;
        const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>((n + 255) / 256, 256 * 16));
        if (nts)
          hipLaunchKernelGGL(produce<true>, dim3(grid), dim3(256), 0, s, src + i * n, stage, n);
        else
          hipLaunchKernelGGL(produce<false>, dim3(grid), dim3(256), 0, s, src + i * n, stage, n);
        if (ntd)
          hipLaunchKernelGGL(consume<true>, dim3(grid), dim3(256), 0, s, stage, dst + i * n, n);
        else
          hipLaunchKernelGGL(consume<false>, dim3(grid), dim3(256), 0, s, stage, dst + i * n, n);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      float best = 1e30f;
      for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) best = std::min(best, ms);
      }
      std::printf("{\"block_MB\": %llu, \"nt_src\": %d, \"nt_dst\": %d, \"ms\": %.4f, \"ms_per_GB\": %.4f, "
                  "\"four_stream_TBps\": %.3f, \"launches\": %llu}\n",
                  (unsigned long long)(B / MB), nts ? 1 : 0, ntd ? 1 : 0, best, best / (N / 1e9),
                  4.0 * N / (best * 1e-3) / 1e12, (unsigned long long)(2 * nb));
      std::fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
