#include "device.hpp"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace hyrise {

namespace {
// Every live operator stream of the process (one per thread that ran an operator), for device_buffer_free.
struct StreamRegistry {
  std::mutex m;
  std::vector<hy_stream_t> streams;
};
StreamRegistry& stream_registry() {
  static StreamRegistry* r = new StreamRegistry;  // (never destroyed: buffers may be released during exit)
  return *r;
}

struct StreamHolder {
  hy_stream_t stream = nullptr;
  ~StreamHolder() {
    if (!stream) return;
    auto& r = stream_registry();
    std::lock_guard<std::mutex> lock(r.m);
    r.streams.erase(std::remove(r.streams.begin(), r.streams.end(), stream), r.streams.end());
    hy_stream_destroy(stream);  // (its pending work still completes)
    // a DeviceBuffer freed later on this thread (another thread_local's destructor) must not name the destroyed
    // stream: device_buffer_free then falls back to a registered stream or the null stream
    stream = nullptr;
  }
};
thread_local StreamHolder t_stream;

std::shared_ptr<DeviceBuffer> upload(const void* host, size_t bytes, hy_stream_t s) {
  auto buf = std::make_shared<DeviceBuffer>(std::max<size_t>(bytes, 16));
  if (bytes) hy_check(hy_memcpy_htod(buf->get(), host, bytes, s), "hy_memcpy_htod");
  return buf;
}
}  // namespace

namespace {
// size classes: powers of two from 4 KiB, cached per thread; at most temp_cache_bytes() kept by ALL threads together
// (g_temp_cached: an eighth of the device's memory, 36 GiB on MI355X, at least 8 GiB) - enough to keep a JoinHash
// workspace of an SF100 join (a 16 GiB block): freeing it after every execution costs a hipFree (a device-wide
// synchronisation and an unmap) per operator call. A failed allocation frees the thread's cached blocks and retries.
std::atomic<size_t> g_temp_cached{0};
size_t temp_cache_bytes() {
  static const size_t bytes = [] {
    uint64_t free_b = 0, total_b = 0;
    if (hy_device_memory(&free_b, &total_b) != HY_OK || total_b == 0) return size_t(8) << 30;
    return std::max<size_t>(size_t(8) << 30, static_cast<size_t>(total_b / 8));
  }();
  return bytes;
}
struct TempCache {
  std::vector<std::pair<size_t, void*>> free_blocks;  // (block bytes, ptr)
  size_t cached = 0;
  void trim() {
    for (auto& b : free_blocks) hy_free(b.second);
    free_blocks.clear();
    g_temp_cached -= cached;
    cached = 0;
  }
  ~TempCache() { trim(); }
};
TempCache& temp_cache() {
  thread_local TempCache c;
  return c;
}
}  // namespace

namespace {
constexpr size_t SLAB_POOL_BYTES = size_t(1) << 30;
struct SlabPool {
  std::mutex m;
  std::vector<void*> free_blocks;
};
SlabPool& slab_pool() {
  static SlabPool* p = new SlabPool;  // (never destroyed: arenas may be released during static destruction)
  return *p;
}
}  // namespace

void* slab_block_acquire() {
  auto& p = slab_pool();
  {
    std::lock_guard<std::mutex> lock(p.m);
    if (!p.free_blocks.empty()) {
      void* b = p.free_blocks.back();
      p.free_blocks.pop_back();
      return b;
    }
  }
  void* b = ::operator new(SLAB_BLOCK_BYTES, std::align_val_t(64));
  return b;
}

void slab_block_release(void* block) {
  auto& p = slab_pool();
  {
    std::lock_guard<std::mutex> lock(p.m);
    if (p.free_blocks.size() * SLAB_BLOCK_BYTES < SLAB_POOL_BYTES) {
      p.free_blocks.push_back(block);
      return;
    }
  }
  ::operator delete(block, std::align_val_t(64));
}

void* temp_block_acquire(size_t bytes, size_t* block_bytes) {
  size_t b = 4096;
  while (b < bytes) b <<= 1;
  auto& c = temp_cache();
  for (size_t i = 0; i < c.free_blocks.size(); ++i) {
    if (c.free_blocks[i].first == b) {
      void* p = c.free_blocks[i].second;
      c.free_blocks[i] = c.free_blocks.back();
      c.free_blocks.pop_back();
      c.cached -= b;
      g_temp_cached -= b;
      *block_bytes = b;
      return p;
    }
  }
  void* p = nullptr;
  if (hy_malloc(&p, b) != HY_OK) {  // device memory short: give back this thread's cached blocks, then retry once
    c.trim();
    hy_check(hy_malloc(&p, b), "hy_malloc");
  }
  *block_bytes = b;
  return p;
}

void temp_block_release(void* ptr, size_t block_bytes) {
  auto& c = temp_cache();
  // reserve the block's bytes in the process-wide budget; over it, the block goes back to the device
  size_t cur = g_temp_cached.load();
  do {
    if (cur + block_bytes > temp_cache_bytes()) {
      hy_free(ptr);
      return;
    }
  } while (!g_temp_cached.compare_exchange_weak(cur, cur + block_bytes));
  c.free_blocks.emplace_back(block_bytes, ptr);
  c.cached += block_bytes;
}

void require_device() {
  int n = 0;
  hy_get_device_count(&n);
  if (n <= 0) Fail("hyrise-amd: no HIP device available — the GPU operators have no CPU fallback");
}

hy_stream_t operator_stream() {
  if (!t_stream.stream) {
    require_device();
    hy_check(hy_stream_create(&t_stream.stream), "hy_stream_create");
    auto& r = stream_registry();
    std::lock_guard<std::mutex> lock(r.m);
    r.streams.push_back(t_stream.stream);
  }
  return t_stream.stream;
}

void operator_stream_synchronize_if_used() {
  if (t_stream.stream) hy_check(hy_stream_synchronize(t_stream.stream), "hy_stream_synchronize");
}

void device_buffer_free(void* ptr) {
  auto& r = stream_registry();
  std::lock_guard<std::mutex> lock(r.m);
  // a thread without an operator stream (the chunk reaper, an embedding's own threads) frees on a stream of its own
  // kind, not on another thread's operator stream (which would then wait for every other stream's work)
  static hy_stream_t release_stream = [] {
    hy_stream_t x = nullptr;
    return hy_stream_create(&x) == HY_OK ? x : nullptr;
  }();
  hy_stream_t s = t_stream.stream ? t_stream.stream : release_stream;
  // (a destructor: a failure cannot be reported; the pool keeps the block then)
  static_cast<void>(hy_free_async_after(ptr, s, r.streams.data(), static_cast<uint32_t>(r.streams.size())));
}

unsigned host_cpu_share() {
  static const unsigned share = [] {
    long n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = static_cast<long>(std::max(1u, std::thread::hardware_concurrency()));
    auto cap = [&](long c) {
      if (c > 0) n = std::min(n, c);
    };
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2: "<quota> <period>" or "max <period>"
      char q[32] = {0};
      long period = 0;
      if (std::fscanf(f, "%31s %ld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
        cap((std::strtol(q, nullptr, 10) + period - 1) / period);
      std::fclose(f);
    } else if (FILE* fq = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {  // cgroup v1
      long quota = -1, period = 0;
      if (std::fscanf(fq, "%ld", &quota) != 1) quota = -1;
      std::fclose(fq);
      if (FILE* fp = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
        if (std::fscanf(fp, "%ld", &period) == 1 && quota > 0 && period > 0) cap((quota + period - 1) / period);
        std::fclose(fp);
      }
    }
    if (const char* e = std::getenv("OMP_NUM_THREADS")) cap(std::strtol(e, nullptr, 10));
    return static_cast<unsigned>(std::max(1L, n));
  }();
  return share;
}

int32_t hy_type_of(DataType t) {
  switch (t) {
    case DataType::Int:
      return HY_TYPE_INT32;
    case DataType::Long:
      return HY_TYPE_INT64;
    case DataType::Float:
      return HY_TYPE_FLOAT;
    case DataType::Double:
      return HY_TYPE_DOUBLE;
    default:
      return 0;
  }
}

// A packed string array (include/hyrise_amd.h, "Column chunk descriptors"): uint32 offsets[n + 1], then the bytes
// at the next 16-byte boundary.
std::shared_ptr<DeviceBuffer> upload_strings(const std::vector<std::string>& v, hy_stream_t s) {
  const size_t n = v.size();
  const size_t head = ((4 * (n + 1)) + 15) & ~size_t(15);
  size_t bytes = 0;
  for (const auto& x : v) bytes += x.size();
  Assert(bytes < 0xFFFFFFFFull, "hyrise-amd: a string chunk exceeds 4 GiB");
  std::vector<char> packed(head + bytes + 16, 0);
  auto* off = reinterpret_cast<uint32_t*>(packed.data());
  size_t at = 0;
  for (size_t i = 0; i < n; ++i) {
    off[i] = static_cast<uint32_t>(at);
    std::memcpy(packed.data() + head + at, v[i].data(), v[i].size());
    at += v[i].size();
  }
  off[n] = static_cast<uint32_t>(at);
  auto buf = upload(packed.data(), packed.size(), s);
  hy_check(hy_stream_synchronize(s), "hy_stream_synchronize");  // `packed` is pageable and local
  return buf;
}

namespace {
// The column's device residency (created on first use); RunLength / FrameOfReference chunks hold only their compressed
// arrays until device_column() decodes their value mirror.
std::shared_ptr<DeviceColumn> resident(const BaseColumn& column) {
  return column.device_mirror_or_create([&]() {
    hy_stream_t s = operator_stream();
    auto d = std::make_shared<DeviceColumn>();
    d->desc.size = static_cast<uint32_t>(column.size());
    if (const auto* dict = dynamic_cast<const BaseDictionaryColumn*>(&column)) {
      const auto& av = dict->attribute_vector();
      if (av.compression() == VectorCompressionType::SimdBp128) {
        // the packed words cross PCIe; the kernels read the FixedSizeByteAligned ids decoded from them in HBM
        const auto words = upload(av.bytes().data(), av.bytes().size(), s);
        const auto meta = upload(av.meta_offsets().data(), av.meta_offsets().size() * 4, s);
        d->data = std::make_shared<DeviceBuffer>(std::max<size_t>(av.size(), 1) * av.width() + 16);
        hy_check(hy_decode_simd_bp128(words->get(), meta->as<uint32_t>(), static_cast<uint32_t>(av.size()), av.width(),
                                      d->data->get(), s),
                 "hy_decode_simd_bp128");
        hy_check(hy_stream_synchronize(s), "sync");  // words / meta are released at scope end
      } else {
        d->data = upload(av.bytes().data(), av.bytes().size(), s);
      }
      d->desc.kind = HY_COL_DICT;
      d->desc.vid_width = av.width();
      d->desc.dictionary_size = static_cast<uint32_t>(dict->unique_values_count());
      d->desc.data = d->data->get();
      resolve_data_type(column.data_type(), [&](auto tag) {
        using T = decltype(tag);
        const auto& dv = static_cast<const DictionaryColumn<T>&>(column).dictionary();
        if constexpr (!std::is_same_v<T, std::string>)
          d->dictionary = upload(dv.data(), dv.size() * sizeof(T), s);
        else  // the dictionary's strings, packed (column comparisons and reference scans read them)
          d->dictionary = upload_strings(dv, s);
        d->desc.dictionary = d->dictionary->get();
      });
    } else if (column.encoding_type() == EncodingType::RunLength ||
               column.encoding_type() == EncodingType::FrameOfReference) {
      // encoded chunk: its compressed arrays go to HBM as they are (the TableScans' HY_COL_RLE / HY_COL_FOR form);
      // the value mirror is decoded from them on the first row-wise use (decode_mirror)
      resolve_data_type(column.data_type(), [&](auto tag) {
        using T = decltype(tag);
        if constexpr (std::is_same_v<T, std::string>) {
          // RunLength strings (FrameOfReference takes integers only): the runs' values as one packed string array,
          // their end positions and NULL flags - the string TableScans evaluate the predicate once per run
          const auto* rl = dynamic_cast<const RunLengthColumn<std::string>*>(&column);
          Assert(rl != nullptr, "device_column: unknown encoded string column");
          hy_column_chunk& c = d->compressed;
          c.size = static_cast<uint32_t>(column.size());
          d->c_data = upload_strings(rl->values(), s);
          d->c_aux = upload(rl->end_positions().data(), rl->end_positions().size() * 4, s);
          if (std::find(rl->null_values().begin(), rl->null_values().end(), uint8_t{1}) != rl->null_values().end())
            d->c_nulls = upload(rl->null_values().data(), rl->null_values().size(), s);
          c.kind = HY_COL_RLE;
          c.dictionary_size = static_cast<uint32_t>(rl->end_positions().size());
          c.data = d->c_data->get();
          c.dictionary = d->c_aux->get();
          c.nulls = d->c_nulls ? d->c_nulls->as<uint8_t>() : nullptr;
        } else {
          hy_column_chunk& c = d->compressed;
          c.size = static_cast<uint32_t>(column.size());
          if (const auto* rl = dynamic_cast<const RunLengthColumn<T>*>(&column)) {
            d->c_data = upload(rl->values().data(), rl->values().size() * sizeof(T), s);
            d->c_aux = upload(rl->end_positions().data(), rl->end_positions().size() * 4, s);
            if (std::find(rl->null_values().begin(), rl->null_values().end(), uint8_t{1}) != rl->null_values().end())
              d->c_nulls = upload(rl->null_values().data(), rl->null_values().size(), s);
            c.kind = HY_COL_RLE;
            c.dictionary_size = static_cast<uint32_t>(rl->end_positions().size());
          } else if constexpr (std::is_same_v<T, int32_t> || std::is_same_v<T, int64_t>) {
            const auto* fr = dynamic_cast<const FrameOfReferenceColumn<T>*>(&column);
            Assert(fr != nullptr, "device_column: unknown encoded column");
            const auto& ov = fr->offset_values();
            d->c_data = upload(ov.bytes().data(), ov.bytes().size(), s);
            d->c_aux = upload(fr->block_minima().data(), fr->block_minima().size() * sizeof(T), s);
            if (std::find(fr->null_values().begin(), fr->null_values().end(), uint8_t{1}) != fr->null_values().end())
              d->c_nulls = upload(fr->null_values().data(), fr->null_values().size(), s);
            c.kind = HY_COL_FOR;
            c.vid_width = ov.width();
            c.dictionary_size = static_cast<uint32_t>(fr->block_minima().size());
          } else {
            Fail("device_column: unknown encoded column");
          }
          c.data = d->c_data->get();
          c.dictionary = d->c_aux->get();
          c.nulls = d->c_nulls ? d->c_nulls->as<uint8_t>() : nullptr;
        }
      });
      d->has_compressed = true;
      d->decoded = false;
      d->desc.kind = column.data_type() == DataType::String ? HY_COL_STRING : HY_COL_VALUE;
    } else {
      Assert(!column.is_reference(), "device_column of a ReferenceColumn");
      resolve_data_type(column.data_type(), [&](auto tag) {
        using T = decltype(tag);
        const auto& vc = static_cast<const ValueColumn<T>&>(column);
        if constexpr (!std::is_same_v<T, std::string>)
          d->data = upload(vc.values().data(), vc.values().size() * sizeof(T), s);
        else  // ValueColumn<std::string>: the chunk's strings as one packed array
          d->data = upload_strings(vc.values(), s);
        d->desc.data = d->data->get();
        if (vc.is_nullable()) {
          d->nulls = upload(vc.null_values().data(), vc.null_values().size(), s);
          d->desc.nulls = d->nulls->as<uint8_t>();
        }
      });
      d->desc.kind = column.data_type() == DataType::String ? HY_COL_STRING : HY_COL_VALUE;
    }
    hy_check(hy_stream_synchronize(s), "hy_stream_synchronize");
    return d;
  });
}

// The value mirror of a RunLength / FrameOfReference chunk, decoded in HBM from its compressed arrays.
void decode_mirror(DeviceColumn& d, const BaseColumn& column) {
  hy_stream_t s = operator_stream();
  const hy_column_chunk& c = d.compressed;
  const uint32_t n = c.size;
  resolve_data_type(column.data_type(), [&](auto tag) {
    using T = decltype(tag);
    if constexpr (std::is_same_v<T, std::string>) {
      // RunLength strings row-wise (column compares, projections): the runs expanded on the host into a packed string
      // array per row (string rows are not a device-decoded format), NULL flags per row
      const auto& rl = static_cast<const RunLengthColumn<std::string>&>(column);
      std::vector<std::string> rows(n);
      std::vector<uint8_t> nulls(std::max<size_t>(n, 1) + 16, 0);
      bool any_null = false;
      size_t r = 0;
      for (uint32_t i = 0; i < n; ++i) {
        while (rl.end_positions()[r] < i) ++r;
        if (rl.null_values()[r]) {
          nulls[i] = 1;
          any_null = true;
        } else {
          rows[i] = rl.values()[r];
        }
      }
      d.data = upload_strings(rows, s);
      if (any_null) {
        d.nulls = upload(nulls.data(), nulls.size(), s);
        hy_check(hy_stream_synchronize(s), "hy_stream_synchronize");  // `nulls` is pageable and local
      }
    } else {
      d.data = std::make_shared<DeviceBuffer>(std::max<size_t>(n, 1) * sizeof(T) + 16);
      if (c.kind == HY_COL_RLE) {
        if (c.nulls) d.nulls = std::make_shared<DeviceBuffer>(std::max<size_t>(n, 1) + 16);
        if (n)
          hy_check(hy_decode_run_length(c.data, c.nulls, static_cast<const uint32_t*>(c.dictionary), c.dictionary_size,
                                        sizeof(T), n, d.data->get(), d.nulls ? d.nulls->as<uint8_t>() : nullptr, s),
                   "hy_decode_run_length");
      } else {
        if (n)
          hy_check(hy_decode_frame_of_reference(c.dictionary, hy_type_of(column.data_type()), c.data, c.vid_width, n,
                                                d.data->get(), s),
                   "hy_decode_frame_of_reference");
        d.nulls = d.c_nulls;  // the row NULL flags are the same array
      }
    }
  });
  hy_check(hy_stream_synchronize(s), "hy_stream_synchronize");
  d.desc.data = d.data->get();
  d.desc.nulls = d.nulls ? d.nulls->as<uint8_t>() : nullptr;
}
}  // namespace

std::shared_ptr<DeviceColumn> device_column(const BaseColumn& column) {
  auto d = resident(column);
  if (!d->decoded.load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lock(d->decode_mutex);
    if (!d->decoded.load(std::memory_order_relaxed)) {
      decode_mirror(*d, column);
      d->decoded.store(true, std::memory_order_release);
    }
  }
  return d;
}

hy_column_chunk device_scan_chunk(const BaseColumn& column) {
  const auto d = resident(column);
  return d->has_compressed ? d->compressed : d->desc;
}

std::shared_ptr<DevicePosList> device_pos_list(const PosList& pos_list) {
  if (auto d = pos_list.device_mirror()) return d;
  hy_stream_t s = operator_stream();
  auto d = std::make_shared<DevicePosList>();
  d->size = pos_list.size();
  d->rows = upload(pos_list.data(), pos_list.size() * sizeof(RowID), s);
  hy_check(hy_stream_synchronize(s), "hy_stream_synchronize");
  pos_list.set_device_mirror(d);
  return d;
}

namespace {
// the lazy PosLists' host copy (PosList::host): after the kernels that wrote the RowIDs (their operator synchronised its
// stream before execute() returned; on the producer's own thread the copy is stream-ordered after them as well)
void fetch_pos_list(const PosList& pos_list, RowID* dst) {
  const auto d = pos_list.device_mirror();
  if (!d) throw std::logic_error("lazy PosList without a device mirror");
  hy_stream_t s = operator_stream();
  hy_check(hy_memcpy_dtoh(dst, d->ptr(), pos_list.size() * sizeof(RowID), s), "hy_memcpy_dtoh");
  hy_check(hy_stream_synchronize(s), "hy_stream_synchronize");
}
}  // namespace

std::shared_ptr<PosList> pos_list_from_device(std::shared_ptr<DeviceBuffer> rows, uint64_t offset, uint64_t n) {
  auto pl = PosList::lazy(n, &fetch_pos_list);  // host RowIDs copied on first host access
  // device mirror: a view into the shared buffer (kept alive by the shared_ptr)
  auto d = std::make_shared<DevicePosList>();
  d->size = n;
  d->rows = std::move(rows);
  d->view_offset = offset;
  pl->set_device_mirror(d);
  return pl;
}

std::shared_ptr<PosList> pos_list_from_device(OutputArena& arena, std::shared_ptr<DeviceBuffer> rows, uint64_t offset,
                                              uint64_t n, DevicePosList** mirror) {
  DevicePosList& d = arena.mirrors->emplace_back();
  d.size = n;
  d.rows = std::move(rows);
  d.view_offset = offset;
  if (mirror) *mirror = &d;
  PosList& pl = arena.lists->emplace_back();
  // (not through set_device_mirror: libstdc++'s atomic shared_ptr store takes a mutex from a global pool, which
  // serialised the output builder threads)
  pl.make_lazy(n, &fetch_pos_list, std::shared_ptr<DevicePosList>(arena.mirrors, &d));
  return std::shared_ptr<PosList>(arena.lists, &pl);
}

}  // namespace hyrise
