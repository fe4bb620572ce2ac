// Device decoding of the RunLength and FrameOfReference encodings into value-column mirrors. The host holds the
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

}  // namespace

extern "C" {

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
