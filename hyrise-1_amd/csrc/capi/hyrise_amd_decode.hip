// Device decoding of SIMD-BP128 attribute vectors into FixedSizeByteAligned id mirrors, and of the RunLength and
// FrameOfReference encodings into value-column mirrors. The host holds the
// encoded chunk (reference storage/run_length_column.hpp, frame_of_reference_column.hpp); its compressed arrays are
// uploaded once and expanded in HBM, so every scan / join / aggregate kernel reads the chunk as a value chunk
// (HBM holds decoded mirrors - 288 GB leaves room for them - and the PCIe transfer stays compressed).
#include <hip/hip_runtime.h>

#include "hyrise_amd.h"
#include "capi_common.hpp"

using namespace hyc;

namespace {

constexpr int DEC_THREADS = 256;

// Row i lies in the first run r with end_positions[r] >= i (run_length_column.cpp:24-36); one binary search per row.
template <typename T>
__global__ __launch_bounds__(DEC_THREADS) void decode_run_length_kernel(const T* __restrict__ values,
                                                                        const uint8_t* __restrict__ run_nulls,
                                                                        const uint32_t* __restrict__ ends,
                                                                        uint32_t n_runs, uint32_t n_rows,
                                                                        T* __restrict__ out,
                                                                        uint8_t* __restrict__ out_nulls) {
  const uint32_t i = blockIdx.x * DEC_THREADS + threadIdx.x;
  if (i >= n_rows) return;
  uint32_t lo = 0, hi = n_runs - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ends[mid] < i)
      lo = mid + 1;
    else
      hi = mid;
  }
  out[i] = values[lo];
  if (out_nulls) out_nulls[i] = run_nulls[lo];
}

// value = block_minima[i / 2048] + offset[i] (frame_of_reference_column.cpp:25-37)
template <typename T>
__global__ __launch_bounds__(DEC_THREADS) void decode_frame_of_reference_kernel(const T* __restrict__ minima,
                                                                                const void* __restrict__ offsets,
                                                                                int width, uint32_t n_rows,
                                                                                T* __restrict__ out) {
  const uint32_t i = blockIdx.x * DEC_THREADS + threadIdx.x;
  if (i >= n_rows) return;
  const uint32_t off = width == 1   ? static_cast<const uint8_t*>(offsets)[i]
                       : width == 2 ? static_cast<const uint16_t*>(offsets)[i]
                                    : static_cast<const uint32_t*>(offsets)[i];
  out[i] = static_cast<T>(minima[i >> 11] + static_cast<T>(off));
}

// SIMD-BP128 (reference vector_compression/simd_bp128/simd_bp128_packing.cpp:22-157, simd_bp128_decompressor.cpp):
// one thread per id. Id i sits in meta block i / 2048 (header word meta[m]: 16 byte-sized bit widths), block
// (i / 128) % 16, whose words follow the header after the widths of the blocks before it; inside the block id j lives
// in 32-bit lane j % 4 at bit (j / 4) * w of that lane's bit stream (low bits first, split across two words when it
// straddles one). Four neighbouring threads read the four lanes of one 16-byte word: the loads coalesce into the
// block's w words. Reads w / 8 bytes per id (+ the header, cached), writes the id in the mirror's width.
template <typename O>
__global__ __launch_bounds__(DEC_THREADS) void decode_simd_bp128_kernel(const uint32_t* __restrict__ words,
                                                                        const uint32_t* __restrict__ meta,
                                                                        uint32_t n_rows, O* __restrict__ out) {
  const uint32_t i = blockIdx.x * DEC_THREADS + threadIdx.x;
  if (i >= n_rows) return;
  const uint32_t m = i >> 11, b = (i >> 7) & 15u, j = i & 127u;
  const uint32_t h = meta[m];
  uint32_t word = h + 1, w = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint32_t wk = (words[4ull * h + (k >> 2)] >> (8 * (k & 3))) & 0xFFu;
    if (k < b) word += wk;
    if (k == b) w = wk;
  }
  uint32_t v = 0;
  if (w) {
    const uint32_t lane = j & 3u, bit = (j >> 2) * w, wi = bit >> 5, shift = bit & 31u;
    uint64_t x = words[4ull * (word + wi) + lane] >> shift;
    if (shift + w > 32) x |= static_cast<uint64_t>(words[4ull * (word + wi + 1) + lane]) << (32 - shift);
    v = w == 32 ? static_cast<uint32_t>(x) : static_cast<uint32_t>(x) & ((1u << w) - 1u);
  }
  out[i] = static_cast<O>(v);
}

}  // namespace

extern "C" {

hy_status hy_decode_simd_bp128(const void* words, const uint32_t* meta_offsets, uint32_t n_rows, int32_t out_width,
                               void* out, hy_stream_t stream) {
  if (n_rows == 0) return HY_OK;
  if (!words || !meta_offsets || !out) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (!aligned16(words)) return fail(HY_ERR_ALIGNMENT, "SIMD-BP128 words not 16-byte aligned");
  const dim3 grid((n_rows + DEC_THREADS - 1) / DEC_THREADS);
  hipStream_t s = S(stream);
  const auto* wd = static_cast<const uint32_t*>(words);
  KTimer kt("decode_simd_bp128", s, n_rows);
  switch (out_width) {
    case 1:
      hipLaunchKernelGGL(decode_simd_bp128_kernel<uint8_t>, grid, dim3(DEC_THREADS), 0, s, wd, meta_offsets, n_rows,
                         static_cast<uint8_t*>(out));
      break;
    case 2:
      hipLaunchKernelGGL(decode_simd_bp128_kernel<uint16_t>, grid, dim3(DEC_THREADS), 0, s, wd, meta_offsets, n_rows,
                         static_cast<uint16_t*>(out));
      break;
    case 4:
      hipLaunchKernelGGL(decode_simd_bp128_kernel<uint32_t>, grid, dim3(DEC_THREADS), 0, s, wd, meta_offsets, n_rows,
                         static_cast<uint32_t*>(out));
      break;
    default:
      return fail(HY_ERR_INVALID_ARGUMENT, "output width");
  }
  kt.done();
  HY_HIP(hipGetLastError());
  return HY_OK;
}

hy_status hy_decode_run_length(const void* values, const uint8_t* run_nulls, const uint32_t* end_positions,
                               uint32_t n_runs, uint32_t value_bytes, uint32_t n_rows, void* out_values,
                               uint8_t* out_nulls, hy_stream_t stream) {
  if (n_rows == 0) return HY_OK;
  if (!values || !end_positions || !out_values || n_runs == 0 || (out_nulls && !run_nulls))
    return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  const dim3 grid((n_rows + DEC_THREADS - 1) / DEC_THREADS);
  hipStream_t s = S(stream);
  if (value_bytes == 4)
    hipLaunchKernelGGL(decode_run_length_kernel<uint32_t>, grid, dim3(DEC_THREADS), 0, s,
                       static_cast<const uint32_t*>(values), run_nulls, end_positions, n_runs, n_rows,
                       static_cast<uint32_t*>(out_values), out_nulls);
  else if (value_bytes == 8)
    hipLaunchKernelGGL(decode_run_length_kernel<uint64_t>, grid, dim3(DEC_THREADS), 0, s,
                       static_cast<const uint64_t*>(values), run_nulls, end_positions, n_runs, n_rows,
                       static_cast<uint64_t*>(out_values), out_nulls);
  else
    return fail(HY_ERR_UNSUPPORTED, "run-length value width");
  HY_HIP(hipGetLastError());
  return HY_OK;
}

hy_status hy_decode_frame_of_reference(const void* block_minima, int32_t value_type, const void* offsets,
                                       int32_t offset_width, uint32_t n_rows, void* out_values, hy_stream_t stream) {
  if (n_rows == 0) return HY_OK;
  if (!block_minima || !offsets || !out_values) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (offset_width != 1 && offset_width != 2 && offset_width != 4) return fail(HY_ERR_INVALID_ARGUMENT, "offset width");
  const dim3 grid((n_rows + DEC_THREADS - 1) / DEC_THREADS);
  hipStream_t s = S(stream);
  if (value_type == HY_TYPE_INT32)
    hipLaunchKernelGGL(decode_frame_of_reference_kernel<int32_t>, grid, dim3(DEC_THREADS), 0, s,
                       static_cast<const int32_t*>(block_minima), offsets, offset_width, n_rows,
                       static_cast<int32_t*>(out_values));
  else if (value_type == HY_TYPE_INT64)
    hipLaunchKernelGGL(decode_frame_of_reference_kernel<int64_t>, grid, dim3(DEC_THREADS), 0, s,
                       static_cast<const int64_t*>(block_minima), offsets, offset_width, n_rows,
                       static_cast<int64_t*>(out_values));
  else
    return fail(HY_ERR_UNSUPPORTED, "FrameOfReference supports int32 / int64");
  HY_HIP(hipGetLastError());
  return HY_OK;
}

}  // extern "C"
