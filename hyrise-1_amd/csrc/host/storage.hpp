// Columnar storage mirror: Table -> Chunk -> {ValueColumn<T>, DictionaryColumn<T>, ReferenceColumn}.
//
// Same public surface and semantics as the reference's storage layer (the parts the hot path touches):
//   Table          reference src/lib/storage/table.hpp:26-175, append_chunk table.cpp:143-170
//   Chunk          reference src/lib/storage/chunk.hpp:41-160
//   ValueColumn    reference src/lib/storage/value_column.hpp:15-73 (append: value_column.cpp:78-90)
//   DictionaryColumn + DictionaryEncoder + FixedSizeByteAligned attribute vectors
//                  reference src/lib/storage/dictionary_column.hpp:20-72, dictionary_column.cpp:75-95,
//                  dictionary_column/dictionary_encoder.hpp:57-130, fixed_size_byte_aligned_compressor.cpp:21-43
//   ReferenceColumn reference src/lib/storage/reference_column.hpp:19-50, reference_column.cpp:23-33
//   load_table     reference src/lib/utils/load_table.cpp:14-62
// Every column can carry a device-resident mirror (device.hpp) that GPU operators create on first use.
#pragma once

#include <cstring>
#include <limits>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "types.hpp"

namespace hyrise {

// CPUs this process may use: the affinity mask, capped by a cgroup CPU quota (cpu.max) and OMP_NUM_THREADS - a GPU
// box grants one GPU's share of a larger machine, which std::thread::hardware_concurrency() does not see.
unsigned host_cpu_share();

class Table;
struct DeviceColumn;  // device.hpp

// No enable_shared_from_this: operator outputs hold columns in arenas behind aliasing shared_ptrs (device.hpp), and
// pybind11 would wrap such an object in a fresh owning pointer (then delete an arena element) for that base.
class BaseColumn {
 public:
  explicit BaseColumn(DataType data_type) : _data_type(data_type) {}
  virtual ~BaseColumn();

  DataType data_type() const { return _data_type; }
  virtual size_t size() const = 0;
  virtual AllTypeVariant operator[](ChunkOffset chunk_offset) const = 0;
  virtual void append(const AllTypeVariant& value) { Fail("Column is immutable"); }
  virtual EncodingType encoding_type() const = 0;
  virtual bool is_reference() const { return false; }

  // Lazily created device mirror (owned by the column; invalidated by mutation).
  std::shared_ptr<DeviceColumn> device_mirror() const {
    std::lock_guard<std::mutex> lock(_device_mutex);
    return _device;
  }
  void set_device_mirror(std::shared_ptr<DeviceColumn> d) const {
    std::lock_guard<std::mutex> lock(_device_mutex);
    _device = std::move(d);
  }
  // Returns the device mirror, creating it with create() under the column's lock on first use.
  template <typename F>
  std::shared_ptr<DeviceColumn> device_mirror_or_create(F&& create) const {
    std::lock_guard<std::mutex> lock(_device_mutex);
    if (!_device) _device = create();
    return _device;
  }

 protected:
  void invalidate_device() {
    std::lock_guard<std::mutex> lock(_device_mutex);
    _device.reset();
  }
  const DataType _data_type;
  mutable std::mutex _device_mutex;
  mutable std::shared_ptr<DeviceColumn> _device;
};

template <typename T>
class ValueColumn final : public BaseColumn {
 public:
  explicit ValueColumn(bool nullable = false) : BaseColumn(data_type_from_type<T>()) {
    if (nullable) _nulls.emplace();
  }
  ValueColumn(std::vector<T>&& values, std::optional<std::vector<uint8_t>>&& nulls)
      : BaseColumn(data_type_from_type<T>()), _values(std::move(values)), _nulls(std::move(nulls)) {}

  size_t size() const override { return _values.size(); }
  EncodingType encoding_type() const override { return EncodingType::Unencoded; }

  AllTypeVariant operator[](ChunkOffset o) const override {
    if (_nulls && (*_nulls).at(o)) return NullValue{};
    return _values.at(o);
  }

  void append(const AllTypeVariant& v) override {
    invalidate_device();
    const bool is_null = variant_is_null(v);
    if (_nulls) {
      _nulls->push_back(is_null ? 1 : 0);
      _values.push_back(is_null ? T{} : type_cast<T>(v));
      return;
    }
    Assert(!is_null, "ValueColumns is not nullable but value passed is null.");
    _values.push_back(type_cast<T>(v));
  }

  bool is_nullable() const { return _nulls.has_value(); }
  bool is_null(ChunkOffset o) const { return _nulls && (*_nulls)[o]; }
  const std::vector<T>& values() const { return _values; }
  std::vector<T>& values() {
    invalidate_device();
    return _values;
  }
  const std::vector<uint8_t>& null_values() const {
    Assert(is_nullable(), "This ValueColumn does not support null values.");
    return *_nulls;
  }
  std::vector<uint8_t>& null_values() {
    Assert(is_nullable(), "This ValueColumn does not support null values.");
    invalidate_device();
    return *_nulls;
  }

 private:
  std::vector<T> _values;
  std::optional<std::vector<uint8_t>> _nulls;
};

// Attribute vector of value ids, in one of the reference's two compressions:
//   FixedSizeByteAligned  uint8 / uint16 / uint32 per id, the narrowest that holds max_value
//                         (reference fixed_size_byte_aligned_compressor.cpp:21-30)
//   SimdBp128             the reference's SIMD-BP128 bit packing (vector_compression/simd_bp128/): 16-byte words;
//                         per meta block of 16 x 128 ids one word of 16 bit widths, then per block `width` words in
//                         which id i of the block sits in 32-bit lane i % 4, at bit (i / 4) * width of that lane's
//                         little-endian bit stream (simd_bp128_packing.cpp:22-157, simd_bp128_compressor.cpp:13-120).
//                         meta_offsets()[m] = index of meta block m's header word (host-side index, from the sizes).
//                         width() is the byte width of the id's FixedSizeByteAligned form (the device mirror's).
class AttributeVector {
 public:
  AttributeVector() = default;
  AttributeVector(const std::vector<uint32_t>& vids, uint32_t max_value,
                  VectorCompressionType compression = VectorCompressionType::FixedSizeByteAligned);
  AttributeVector(std::vector<uint8_t>&& bytes, int width, size_t size)
      : _bytes(std::move(bytes)), _width(width), _size(size) {}

  uint32_t get(size_t i) const {
    if (_compression == VectorCompressionType::SimdBp128) return bp128_get(i);
    switch (_width) {
      case 1:
        return _bytes[i];
      case 2: {
        uint16_t v;
        std::memcpy(&v, _bytes.data() + 2 * i, 2);
        return v;
      }
      default: {
        uint32_t v;
        std::memcpy(&v, _bytes.data() + 4 * i, 4);
        return v;
      }
    }
  }
  int width() const { return _width; }
  size_t size() const { return _size; }
  VectorCompressionType compression() const { return _compression; }
  // FixedSizeByteAligned: the ids; SimdBp128: the packed 16-byte words
  const std::vector<uint8_t>& bytes() const { return _bytes; }
  const std::vector<uint32_t>& meta_offsets() const { return _meta; }

  static constexpr uint32_t BP128_BLOCK = 128, BP128_BLOCKS = 16, BP128_META = BP128_BLOCK * BP128_BLOCKS;

 private:
  uint32_t bp128_get(size_t i) const;

  std::vector<uint8_t> _bytes;
  int _width = 1;
  size_t _size = 0;
  VectorCompressionType _compression = VectorCompressionType::FixedSizeByteAligned;
  std::vector<uint32_t> _meta;
};

// RunLengthColumn (reference storage/run_length_column.hpp): one value + NULL flag per run, end_positions[r] = last
// offset of run r. On the device it is decoded once into a value mirror (hy_decode_run_length).
template <typename T>
class RunLengthColumn final : public BaseColumn {
 public:
  RunLengthColumn(std::vector<T> values, std::vector<uint8_t> null_values, std::vector<ChunkOffset> end_positions)
      : BaseColumn(data_type_from_type<T>()),
        _values(std::move(values)),
        _null_values(std::move(null_values)),
        _end_positions(std::move(end_positions)) {}
  size_t size() const override { return _end_positions.empty() ? 0 : _end_positions.back() + 1u; }
  EncodingType encoding_type() const override { return EncodingType::RunLength; }
  AllTypeVariant operator[](ChunkOffset o) const override {  // run_length_column.cpp:24-36
    const auto run = static_cast<size_t>(
        std::distance(_end_positions.cbegin(), std::lower_bound(_end_positions.cbegin(), _end_positions.cend(), o)));
    if (_null_values.at(run)) return NullValue{};
    return _values.at(run);
  }
  const std::vector<T>& values() const { return _values; }
  const std::vector<uint8_t>& null_values() const { return _null_values; }
  const std::vector<ChunkOffset>& end_positions() const { return _end_positions; }

 private:
  std::vector<T> _values;
  std::vector<uint8_t> _null_values;
  std::vector<ChunkOffset> _end_positions;
};

// FrameOfReferenceColumn (reference storage/frame_of_reference_column.hpp): per block of 2048 rows a minimum, per row
// an unsigned offset (FixedSizeByteAligned u8/u16/u32) and a NULL flag; int32 / int64 only. Decoded on the device
// once into a value mirror (hy_decode_frame_of_reference).
template <typename T>
class FrameOfReferenceColumn final : public BaseColumn {
 public:
  static constexpr uint32_t block_size = 2048u;
  FrameOfReferenceColumn(std::vector<T> block_minima, std::vector<uint8_t> null_values,
                         std::shared_ptr<const AttributeVector> offset_values)
      : BaseColumn(data_type_from_type<T>()),
        _block_minima(std::move(block_minima)),
        _null_values(std::move(null_values)),
        _offset_values(std::move(offset_values)) {}
  size_t size() const override { return _null_values.size(); }
  EncodingType encoding_type() const override { return EncodingType::FrameOfReference; }
  AllTypeVariant operator[](ChunkOffset o) const override {  // frame_of_reference_column.cpp:25-37
    if (_null_values.at(o)) return NullValue{};
    return static_cast<T>(_block_minima.at(o / block_size) + static_cast<T>(_offset_values->get(o)));
  }
  const std::vector<T>& block_minima() const { return _block_minima; }
  const std::vector<uint8_t>& null_values() const { return _null_values; }
  const AttributeVector& offset_values() const { return *_offset_values; }

 private:
  std::vector<T> _block_minima;
  std::vector<uint8_t> _null_values;
  std::shared_ptr<const AttributeVector> _offset_values;
};

class BaseDictionaryColumn : public BaseColumn {
 public:
  using BaseColumn::BaseColumn;
  virtual ValueID lower_bound(const AllTypeVariant& value) const = 0;
  virtual ValueID upper_bound(const AllTypeVariant& value) const = 0;
  virtual size_t unique_values_count() const = 0;
  virtual ValueID null_value_id() const = 0;
  virtual const AttributeVector& attribute_vector() const = 0;
};

template <typename T>
class DictionaryColumn : public BaseDictionaryColumn {
 public:
  DictionaryColumn(std::shared_ptr<const std::vector<T>> dictionary, std::shared_ptr<const AttributeVector> av,
                   ValueID null_value_id)
      : BaseDictionaryColumn(data_type_from_type<T>()),
        _dictionary(std::move(dictionary)),
        _attribute_vector(std::move(av)),
        _null_value_id(null_value_id) {}

  size_t size() const override { return _attribute_vector->size(); }
  EncodingType encoding_type() const override { return EncodingType::Dictionary; }

  AllTypeVariant operator[](ChunkOffset o) const override {
    const ValueID vid = _attribute_vector->get(o);
    if (vid == _null_value_id) return NullValue{};
    return (*_dictionary)[vid];
  }

  // reference dictionary_column.cpp:75-95
  ValueID lower_bound(const AllTypeVariant& value) const override {
    Assert(!variant_is_null(value), "Null value passed.");
    const T typed = type_cast<T>(value);
    auto it = std::lower_bound(_dictionary->cbegin(), _dictionary->cend(), typed);
    if (it == _dictionary->cend()) return INVALID_VALUE_ID;
    return static_cast<ValueID>(std::distance(_dictionary->cbegin(), it));
  }
  ValueID upper_bound(const AllTypeVariant& value) const override {
    Assert(!variant_is_null(value), "Null value passed.");
    const T typed = type_cast<T>(value);
    auto it = std::upper_bound(_dictionary->cbegin(), _dictionary->cend(), typed);
    if (it == _dictionary->cend()) return INVALID_VALUE_ID;
    return static_cast<ValueID>(std::distance(_dictionary->cbegin(), it));
  }
  size_t unique_values_count() const override { return _dictionary->size(); }
  ValueID null_value_id() const override { return _null_value_id; }
  const AttributeVector& attribute_vector() const override { return *_attribute_vector; }
  const std::vector<T>& dictionary() const { return *_dictionary; }

 private:
  std::shared_ptr<const std::vector<T>> _dictionary;
  std::shared_ptr<const AttributeVector> _attribute_vector;
  ValueID _null_value_id;
};

// FixedStringDictionaryColumn (reference storage/fixed_string_dictionary_column.hpp, fixed_string_vector.hpp): a string
// dictionary stored as one char array of fixed-width entries (every entry padded with '\0' to the longest value's
// length, dictionary_encoder.hpp:132-138), plus the attribute vector. An entry reads as its chars up to the first
// '\0' (FixedString::string, fixed_string.cpp), so values are compared, bounded and returned exactly as the
// reference's. It is a DictionaryColumn<std::string> over those decoded entries: scans rewrite predicates to value ids
// and the device reads the attribute vector as for Dictionary; encoding_type() tells the two apart.
class FixedStringDictionaryColumn final : public DictionaryColumn<std::string> {
 public:
  FixedStringDictionaryColumn(std::vector<char> chars, size_t string_length, size_t n_entries,
                              std::shared_ptr<const AttributeVector> av, ValueID null_value_id)
      : DictionaryColumn<std::string>(decode(chars, string_length, n_entries), std::move(av), null_value_id),
        _chars(std::move(chars)),
        _string_length(string_length) {}
  EncodingType encoding_type() const override { return EncodingType::FixedStringDictionary; }
  // the fixed-width entries (string_length() bytes each; one '\0' byte when every value is empty)
  const std::vector<char>& fixed_string_chars() const { return _chars; }
  size_t string_length() const { return _string_length; }

 private:
  static std::shared_ptr<const std::vector<std::string>> decode(const std::vector<char>& chars, size_t len, size_t n) {
    auto v = std::make_shared<std::vector<std::string>>();
    v->reserve(n);
    for (size_t i = 0; i < n; ++i) {
      const char* p = chars.data() + i * len;
      v->emplace_back(p, len ? strnlen(p, len) : 0);
    }
    return v;
  }
  std::vector<char> _chars;
  size_t _string_length;
};

class ReferenceColumn final : public BaseColumn {
 public:
  ReferenceColumn(std::shared_ptr<const Table> referenced_table, ColumnID referenced_column_id,
                  std::shared_ptr<const PosList> pos);

  size_t size() const override { return _pos_list->size(); }
  EncodingType encoding_type() const override { return EncodingType::Unencoded; }
  bool is_reference() const override { return true; }
  AllTypeVariant operator[](ChunkOffset o) const override;

  const std::shared_ptr<const PosList>& pos_list() const { return _pos_list; }
  const std::shared_ptr<const Table>& referenced_table() const { return _referenced_table; }
  ColumnID referenced_column_id() const { return _referenced_column_id; }

 private:
  std::shared_ptr<const Table> _referenced_table;
  ColumnID _referenced_column_id;
  std::shared_ptr<const PosList> _pos_list;
};

using ChunkColumns = std::vector<std::shared_ptr<BaseColumn>>;

// MVCC columns of a data chunk (reference storage/mvcc_columns.hpp:15-45): per row the id of the transaction holding
// its lock (0 if none), the commit id of its insert and of its delete.
struct MvccColumns {
  static constexpr uint32_t MAX_COMMIT_ID = std::numeric_limits<uint32_t>::max() - 1;
  std::vector<uint32_t> tids, begin_cids, end_cids;
  // HBM copy (tids | begin_cids | end_cids), made on first Validate; the vectors are not mutated after
  // Chunk::set_mvcc_columns (a new MVCC state is a new MvccColumns object), so the copy stays valid
  mutable std::mutex device_mutex;
  mutable std::shared_ptr<void> device;
  mutable uint64_t device_rows = 0;  // rows the copy holds (the chunk's size when it was made)
};

class Chunk {
 public:
  explicit Chunk(ChunkColumns columns) : _columns(std::move(columns)) {}
  bool has_mvcc_columns() const { return _mvcc != nullptr; }
  std::shared_ptr<const MvccColumns> mvcc_columns() const { return _mvcc; }
  void set_mvcc_columns(std::shared_ptr<const MvccColumns> m) {
    // every row of the chunk needs its MVCC entries (validate.cpp:101 iterates chunk_in->size() rows)
    if (m && (m->tids.size() < size() || m->begin_cids.size() < size() || m->end_cids.size() < size()))
      throw std::logic_error("MVCC columns shorter than the chunk");
    _mvcc = std::move(m);
  }
  size_t size() const { return _columns.empty() ? 0 : _columns[0]->size(); }
  uint16_t column_count() const { return static_cast<uint16_t>(_columns.size()); }
  std::shared_ptr<BaseColumn> get_column(ColumnID id) const { return _columns.at(id); }
  const ChunkColumns& columns() const { return _columns; }
  // reference chunk.cpp:39-41
  void replace_column(ColumnID id, std::shared_ptr<BaseColumn> c) { _columns.at(id) = std::move(c); }
  void append(const std::vector<AllTypeVariant>& values);

 private:
  ChunkColumns _columns;
  std::shared_ptr<const MvccColumns> _mvcc;
};

struct TableColumnDefinition {
  TableColumnDefinition() = default;
  TableColumnDefinition(std::string n, DataType t, bool null = false) : name(std::move(n)), data_type(t), nullable(null) {}
  std::string name;
  DataType data_type = DataType::Int;
  bool nullable = false;
};
using TableColumnDefinitions = std::vector<TableColumnDefinition>;

class Table {
 public:
  Table(TableColumnDefinitions defs, TableType type, uint32_t max_chunk_size = CHUNK_MAX_SIZE)
      : _defs(std::move(defs)), _type(type), _max_chunk_size(max_chunk_size) {}
  // A table of many chunks (a JoinHash output has one per radix partition: 65,536 at SF100, ~8 allocations each) hands
  // its chunks to a background thread to destroy: dropping an operator's output costs the dropping thread a move
  // instead of ~7 ms of frees. release_drain() waits until every handed-over chunk is destroyed.
  ~Table();
  Table(const Table&) = delete;
  Table& operator=(const Table&) = delete;

  const TableColumnDefinitions& column_definitions() const { return _defs; }
  TableType type() const { return _type; }
  uint16_t column_count() const { return static_cast<uint16_t>(_defs.size()); }
  const std::string& column_name(ColumnID id) const { return _defs.at(id).name; }
  DataType column_data_type(ColumnID id) const { return _defs.at(id).data_type; }
  bool column_is_nullable(ColumnID id) const { return _defs.at(id).nullable; }
  ColumnID column_id_by_name(const std::string& name) const;
  std::vector<std::string> column_names() const;

  uint32_t max_chunk_size() const { return _max_chunk_size; }
  uint32_t chunk_count() const {
    resolve();
    return static_cast<uint32_t>(_chunks.size());
  }
  uint64_t row_count() const;
  std::shared_ptr<Chunk> get_chunk(ChunkID id) const {
    resolve();
    return _chunks.at(id);
  }
  const std::vector<std::shared_ptr<Chunk>>& chunks() const {
    resolve();
    return _chunks;
  }

  // A table whose chunks are produced on first access: an operator's output computed lazily, so that the consumer
  // that reads it next can produce it as a by-product of its own work (a TableScan whose JoinHash evaluates the scan
  // predicate inside its first radix pass, operators.cpp). Every accessor of the chunks resolves the table first; the
  // producer runs once, on the first accessing thread. A consumer that produces the chunks itself takes the producer
  // (take_pending) and installs them with fulfil().
  struct Producer {
    virtual ~Producer() = default;
    virtual std::vector<std::shared_ptr<Chunk>> produce() = 0;
  };
  void set_pending(std::shared_ptr<Producer> producer);
  std::shared_ptr<Producer> pending() const;  // the unresolved producer, or null
  // takes the producer if it is still pending (null otherwise): the caller must fulfil() the table
  std::shared_ptr<Producer> take_pending();
  void fulfil(std::vector<std::shared_ptr<Chunk>>&& chunks);

  // reference table.cpp: append a row, opening a new chunk when the last one is full
  void append(const std::vector<AllTypeVariant>& values);
  void append_chunk(const ChunkColumns& columns);
  // chunks an operator built (possibly on several threads), appended in order; same checks as append_chunk
  void append_chunks(std::vector<std::shared_ptr<Chunk>>&& chunks);
  void append_mutable_chunk();

  AllTypeVariant get_value(ColumnID column_id, uint64_t row) const;

  static std::shared_ptr<Table> create_dummy_table(const TableColumnDefinitions& defs) {
    return std::make_shared<Table>(defs, TableType::Data);
  }

 private:
  void resolve() const {
    if (_pending_flag.load(std::memory_order_acquire)) resolve_slow();
  }
  void resolve_slow() const;
  TableColumnDefinitions _defs;
  TableType _type;
  uint32_t _max_chunk_size;
  mutable std::vector<std::shared_ptr<Chunk>> _chunks;
  mutable std::mutex _pending_m;
  mutable std::condition_variable _pending_cv;
  mutable std::shared_ptr<Producer> _pending;
  mutable bool _taken = false;  // a consumer took the producer and will fulfil() the table
  mutable std::atomic<bool> _pending_flag{false};
};

void release_drain();

// Creates an empty ValueColumn<T> for a data type.
std::shared_ptr<BaseColumn> make_value_column(DataType t, bool nullable);

// Dictionary encoding of one value column (reference dictionary_encoder.hpp:57-130).
std::shared_ptr<BaseColumn> encode_dictionary(
    const BaseColumn& value_column, VectorCompressionType compression = VectorCompressionType::FixedSizeByteAligned);

// ChunkEncoder (reference src/lib/storage/chunk_encoder.cpp): encode chunks of a data table. Only Unencoded and
// Dictionary exist on the device path; other encodings are rejected.
// The vector compression applies to Dictionary's attribute vectors (reference ChunkEncodingSpec's
// vector_compression_type); the other encodings keep FixedSizeByteAligned.
struct ChunkEncoder {
  static void encode_chunks(const std::shared_ptr<Table>& table, const std::vector<ChunkID>& chunk_ids,
                            EncodingType encoding,
                            VectorCompressionType compression = VectorCompressionType::FixedSizeByteAligned);
  static void encode_all_chunks(const std::shared_ptr<Table>& table, EncodingType encoding,
                                VectorCompressionType compression = VectorCompressionType::FixedSizeByteAligned);
  // every chunk's columns column_ids (the others stay as they are); chunks in parallel
  static void encode_columns(const std::shared_ptr<Table>& table, const std::vector<ColumnID>& column_ids,
                             EncodingType encoding,
                             VectorCompressionType compression = VectorCompressionType::FixedSizeByteAligned);
};

std::shared_ptr<Table> load_table(const std::string& file_name, uint32_t chunk_size = CHUNK_MAX_SIZE);

}  // namespace hyrise
