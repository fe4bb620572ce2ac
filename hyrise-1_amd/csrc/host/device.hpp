// Device residency owned by host objects (the MI355X analogue of the reference's NUMA placement: chunk columns are
// mirrored into HBM on first GPU use and kept there while the column lives; reference
// src/lib/storage/numa_placement_manager.cpp:48-52, Chunk::migrate chunk.cpp:148-160).
//
// Everything here goes through the C-ABI (include/hyrise_amd.h); hy_status failures become std::logic_error,
// like the reference's Fail (src/lib/utils/assert.hpp:49-70).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "hyrise_amd.h"
#include "storage.hpp"

namespace hyrise {

inline void hy_check(hy_status st, const char* what) {
  if (st != HY_OK) Fail(std::string(what) + " failed (" + std::to_string(st) + "): " + hy_last_error_message());
}

// Owning device allocation.
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes) : _bytes(bytes) {
    if (bytes) hy_check(hy_malloc(&_ptr, bytes), "hy_malloc");
  }
  ~DeviceBuffer() {
    if (_ptr) hy_free(_ptr);
  }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  void* get() const { return _ptr; }
  template <typename T>
  T* as() const {
    return static_cast<T*>(_ptr);
  }
  size_t bytes() const { return _bytes; }

 private:
  void* _ptr = nullptr;
  size_t _bytes = 0;
};

// Per-thread stream for operator execution (operators may run concurrently on scheduler workers).
hy_stream_t operator_stream();

// Is a usable device present? Throws with a clear message if the HIP library reports none.
void require_device();

// Device mirror of one Value/Dictionary column chunk.
struct DeviceColumn {
  std::shared_ptr<DeviceBuffer> data, nulls, dictionary;
  hy_column_chunk desc{};
};

// Device mirror of a PosList (same 8-byte RowID layout).
struct DevicePosList {
  std::shared_ptr<DeviceBuffer> rows;  // may be shared by several PosLists (views)
  uint64_t size = 0;
  uint64_t view_offset = 0;            // in RowIDs
  const hy_row_id* ptr() const { return rows ? rows->as<hy_row_id>() + view_offset : nullptr; }
};

// Returns (creating on first use) the device mirror of a data column chunk. String columns are only resident as
// dictionary attribute vectors (dictionary stays on the host).
std::shared_ptr<DeviceColumn> device_column(const BaseColumn& column);

// Returns (uploading on first use) the device mirror of a PosList.
std::shared_ptr<DevicePosList> device_pos_list(const PosList& pos_list);

// Creates a PosList whose host content and device mirror are both filled from a device RowID array.
std::shared_ptr<PosList> pos_list_from_device(std::shared_ptr<DeviceBuffer> rows, uint64_t offset, uint64_t n);

int32_t hy_type_of(DataType t);

}  // namespace hyrise
