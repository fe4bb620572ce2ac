// Device residency owned by host objects (the MI355X analogue of the reference's NUMA placement: chunk columns are
// mirrored into HBM on first GPU use and kept there while the column lives; reference
// src/lib/storage/numa_placement_manager.cpp:48-52, Chunk::migrate chunk.cpp:148-160).
//
// Everything here goes through the C-ABI (include/hyrise_amd.h); hy_status failures become std::logic_error,
// like the reference's Fail (src/lib/utils/assert.hpp:49-70).
#pragma once

#include <atomic>
#include <deque>
#include <new>
#include <mutex>
#include <memory>
#include <string>
#include <vector>

#include "hyrise_amd.h"
#include "storage.hpp"

namespace hyrise {

inline void hy_check(hy_status st, const char* what) {
  if (st != HY_OK) Fail(std::string(what) + " failed (" + std::to_string(st) + "): " + hy_last_error_message());
}

// Per-thread cache of device blocks for operator-scoped temporaries (workspaces, offsets, counts). A block goes
// back to the cache of the thread that releases it and is only handed out again on that thread, whose operator work
// is ordered on that thread's stream - so a reused block is never written before the kernels that read it finished,
// and releasing it neither frees device memory nor waits for the device (hipFree synchronises the whole device).
void* temp_block_acquire(size_t bytes, size_t* block_bytes);
hy_stream_t operator_stream();
void temp_block_release(void* ptr, size_t block_bytes);
// Returns a long-lived buffer to the device pool once every operator stream of the process has finished the work
// enqueued so far (the operator streams are non-blocking: a free on the null stream would not be ordered after them).
// The free is enqueued on the releasing thread's operator stream, so that thread's next output allocation reuses the
// block (same-stream reuse needs no cross-stream dependency in the pool).
void device_buffer_free(void* ptr);

// Owning device allocation. Temporary (the `stream` constructor): a block of the calling thread's cache, for buffers
// used only by that thread's operator stream while the operator runs; otherwise a plain allocation for buffers that
// outlive the operator (column mirrors, the RowIDs behind output PosLists).
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  // long-lived buffers (operator outputs): stream-ordered on this thread's operator stream, from the device pool
  explicit DeviceBuffer(size_t bytes) : _bytes(bytes) {
    if (bytes) hy_check(hy_malloc_async(&_ptr, bytes, operator_stream()), "hy_malloc_async");
  }
  DeviceBuffer(size_t bytes, hy_stream_t /*operator stream*/) : _bytes(bytes), _temp(true) {
    if (bytes) _ptr = temp_block_acquire(bytes, &_block);
  }
  ~DeviceBuffer() {
    // ordered after the work of every operator stream that may still read it
    if (_ptr) _temp ? temp_block_release(_ptr, _block) : device_buffer_free(_ptr);
  }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  void* get() const { return _ptr; }
  template <typename T>
  T* as() const {
    return static_cast<T*>(_ptr);
  }
  size_t bytes() const { return _bytes; }
  // exchanges the allocations (views that hold this object see the new one: an output's RowIDs sized after the
  // PosLists over them were created)
  void swap(DeviceBuffer& o) {
    std::swap(_ptr, o._ptr);
    std::swap(_bytes, o._bytes);
    std::swap(_block, o._block);
    std::swap(_temp, o._temp);
  }

 private:
  void* _ptr = nullptr;
  size_t _bytes = 0;
  size_t _block = 0;
  bool _temp = false;
};

// Per-thread stream for operator execution (operators may run concurrently on scheduler workers).
hy_stream_t operator_stream();
// Waits for the calling thread's operator stream, if the thread has one (no stream is created).
void operator_stream_synchronize_if_used();

// Is a usable device present? Throws with a clear message if the HIP library reports none.
void require_device();

// Device mirror of one column chunk. desc: what the row-wise kernels read (values / dictionary ids). RunLength and
// FrameOfReference chunks also keep their compressed arrays in HBM (`compressed`, HY_COL_RLE / HY_COL_FOR), which
// TableScans read directly; their value mirror (desc) is decoded from those on the first row-wise use only.
struct DeviceColumn {
  std::shared_ptr<DeviceBuffer> data, nulls, dictionary;
  hy_column_chunk desc{};
  std::shared_ptr<DeviceBuffer> c_data, c_nulls, c_aux;
  hy_column_chunk compressed{};
  bool has_compressed = false;
  std::atomic<bool> decoded{true};
  std::mutex decode_mutex;
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
// The descriptor a TableScan reads: the compressed form of RunLength / FrameOfReference chunks (no value mirror is
// decoded for them), device_column(column)->desc otherwise.
hy_column_chunk device_scan_chunk(const BaseColumn& column);

// Output objects of an operator that emits many chunks (JoinHash: one per radix partition, 65,536 at SF100): the
// chunks, their columns, PosLists and the PosLists' device mirrors live in four arenas (slabs: elements never move);
// the shared_ptrs handed out alias an arena's control block (no allocation, no control block per object). The arenas
// own each other in one direction only - chunks -> columns -> PosLists -> mirrors - so the last chunk released frees
// them all.
//
// The arenas' memory comes in 1 MiB host blocks that are recycled process-wide (up to SLAB_POOL_BYTES): an operator
// that emits 65,536 chunks per execution would otherwise free its pages to the OS and fault them in again on the next
// execution, and page faults from several builder threads serialise in the kernel.
void* slab_block_acquire();
void slab_block_release(void* block);
constexpr size_t SLAB_BLOCK_BYTES = size_t(1) << 20;

// Append-only sequence of T in recycled blocks (elements never move; destroyed in order with the slab).
template <typename T>
class Slab {
 public:
  static constexpr size_t PER_BLOCK = SLAB_BLOCK_BYTES / sizeof(T);
  static_assert(PER_BLOCK >= 64 && alignof(T) <= 16, "slab element too large");
  Slab() = default;
  Slab(const Slab&) = delete;
  Slab& operator=(const Slab&) = delete;
  ~Slab() {
    for (size_t i = 0; i < _n; ++i) at(i).~T();
    for (void* b : _blocks) slab_block_release(b);
  }
  template <typename... A>
  T& emplace_back(A&&... a) {
    if (_n == _blocks.size() * PER_BLOCK) _blocks.push_back(slab_block_acquire());
    T* p = new (static_cast<T*>(_blocks.back()) + _n % PER_BLOCK) T(std::forward<A>(a)...);
    ++_n;
    return *p;
  }

 private:
  T& at(size_t i) { return static_cast<T*>(_blocks[i / PER_BLOCK])[i % PER_BLOCK]; }
  std::vector<void*> _blocks;
  size_t _n = 0;
};

struct OutputArena {
  std::shared_ptr<Slab<DevicePosList>> mirrors = std::make_shared<Slab<DevicePosList>>();
  std::shared_ptr<Slab<PosList>> lists = std::make_shared<Slab<PosList>>();
  std::shared_ptr<Slab<ReferenceColumn>> columns = std::make_shared<Slab<ReferenceColumn>>();
  std::shared_ptr<Slab<Chunk>> chunks = std::make_shared<Slab<Chunk>>();
};
// A lazy PosList in the arena over rows [offset, offset + n) of a device RowID array; *mirror (if given) receives its
// device mirror, whose view the producer may still move (with PosList::set_lazy_size) before publishing the list.
std::shared_ptr<PosList> pos_list_from_device(OutputArena& arena, std::shared_ptr<DeviceBuffer> rows, uint64_t offset,
                                              uint64_t n, DevicePosList** mirror = nullptr);
inline std::shared_ptr<ReferenceColumn> arena_reference_column(OutputArena& arena, std::shared_ptr<const Table> table,
                                                               ColumnID column, std::shared_ptr<const PosList> pos_list) {
  return std::shared_ptr<ReferenceColumn>(arena.columns,
                                         &arena.columns->emplace_back(std::move(table), column, std::move(pos_list)));
}
inline std::shared_ptr<Chunk> arena_chunk(OutputArena& arena, ChunkColumns columns) {
  return std::shared_ptr<Chunk>(arena.chunks, &arena.chunks->emplace_back(std::move(columns)));
}

// Returns (uploading on first use) the device mirror of a PosList.
std::shared_ptr<DevicePosList> device_pos_list(const PosList& pos_list);

// Creates a lazy PosList over a device RowID array (its device mirror; host RowIDs copied on first host access).
std::shared_ptr<PosList> pos_list_from_device(std::shared_ptr<DeviceBuffer> rows, uint64_t offset, uint64_t n);

int32_t hy_type_of(DataType t);

}  // namespace hyrise
