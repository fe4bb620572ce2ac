#include "storage.hpp"

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>

#include <fstream>
#include <sstream>

namespace hyrise {

BaseColumn::~BaseColumn() = default;

ReferenceColumn::ReferenceColumn(std::shared_ptr<const Table> referenced_table, ColumnID referenced_column_id,
                                 std::shared_ptr<const PosList> pos)
    : BaseColumn(referenced_table->column_data_type(referenced_column_id)),
      _referenced_table(std::move(referenced_table)),
      _referenced_column_id(referenced_column_id),
      _pos_list(std::move(pos)) {}

// reference reference_column.cpp:23-33
AllTypeVariant ReferenceColumn::operator[](ChunkOffset o) const {
  const RowID row_id = _pos_list->at(o);
  if (row_id.is_null()) return NullValue{};
  const auto chunk = _referenced_table->get_chunk(row_id.chunk_id);
  return (*chunk->get_column(_referenced_column_id))[row_id.chunk_offset];
}

void Chunk::append(const std::vector<AllTypeVariant>& values) {
  Assert(values.size() == _columns.size(), "append: wrong number of values");
  for (size_t i = 0; i < values.size(); ++i) _columns[i]->append(values[i]);
}

ColumnID Table::column_id_by_name(const std::string& name) const {
  for (ColumnID i = 0; i < _defs.size(); ++i)
    if (_defs[i].name == name) return i;
  Fail("Couldn't find column '" + name + "'");
}

std::vector<std::string> Table::column_names() const {
  std::vector<std::string> out;
  for (const auto& d : _defs) out.push_back(d.name);
  return out;
}

uint64_t Table::row_count() const {
  resolve();
  uint64_t n = 0;
  for (const auto& c : _chunks) n += c->size();
  return n;
}

std::shared_ptr<BaseColumn> make_value_column(DataType t, bool nullable) {
  std::shared_ptr<BaseColumn> out;
  resolve_data_type(t, [&](auto tag) {
    using T = decltype(tag);
    out = std::make_shared<ValueColumn<T>>(nullable);
  });
  return out;
}

void Table::append_mutable_chunk() {
  resolve();
  ChunkColumns cols;
  for (const auto& d : _defs) cols.push_back(make_value_column(d.data_type, d.nullable));
  _chunks.push_back(std::make_shared<Chunk>(std::move(cols)));
}

void Table::append(const std::vector<AllTypeVariant>& values) {
  resolve();
  if (_chunks.empty() || _chunks.back()->size() >= _max_chunk_size) append_mutable_chunk();
  _chunks.back()->append(values);
}

void Table::append_chunk(const ChunkColumns& columns) {
  resolve();
  Assert(columns.size() == _defs.size(), "append_chunk: wrong number of columns");
  const size_t n = columns.empty() ? 0 : columns[0]->size();
  for (const auto& c : columns) {
    Assert(c->size() == n, "Columns don't have the same length");
    Assert(c->is_reference() == (_type == TableType::References), "Invalid column type");
  }
  _chunks.push_back(std::make_shared<Chunk>(columns));
}

// The bulk form operators use for outputs they built consistent by construction (a JoinHash's 65,536 chunks at
// SF100): the per-column checks are debug-only here, as the reference's DebugAssert, because walking every chunk's
// columns and PosLists right after other threads built them costs several milliseconds of cache misses.
namespace {

// Destroys handed-over chunk lists on one background thread (never joined: the process-exit hook drains it while the
// HIP runtime is still up, since the hook is registered after the first device allocation it frees).
class ChunkReaper {
 public:
  void push(std::vector<std::shared_ptr<Chunk>>&& chunks) {
    std::lock_guard<std::mutex> lock(_m);
    if (!_started) {
      _started = true;
      std::thread([this] { run(); }).detach();
      std::atexit([] { chunk_reaper().drain(); });
    }
    _queue.push_back(std::move(chunks));
    _cv.notify_all();
  }
  void drain() {
    std::unique_lock<std::mutex> lock(_m);
    _cv.wait(lock, [&] { return _queue.empty() && _busy == 0; });
  }
  static ChunkReaper& chunk_reaper() {
    static ChunkReaper* r = new ChunkReaper;  // (leaked: outlives static destruction)
    return *r;
  }

 private:
  void run() {
    for (;;) {
      std::vector<std::shared_ptr<Chunk>> chunks;
      {
        std::unique_lock<std::mutex> lock(_m);
        _cv.wait(lock, [&] { return !_queue.empty(); });
        chunks = std::move(_queue.front());
        _queue.pop_front();
        ++_busy;
      }
      chunks.clear();
      std::lock_guard<std::mutex> lock(_m);
      --_busy;
      _cv.notify_all();
    }
  }
  std::mutex _m;
  std::condition_variable _cv;
  std::deque<std::vector<std::shared_ptr<Chunk>>> _queue;
  size_t _busy = 0;
  bool _started = false;
};

constexpr size_t BACKGROUND_RELEASE_CHUNKS = 1024;

}  // namespace

void Table::set_pending(std::shared_ptr<Producer> producer) {
  std::lock_guard<std::mutex> lock(_pending_m);
  _pending = std::move(producer);
  _taken = false;
  _pending_flag.store(_pending != nullptr, std::memory_order_release);
  _pending_cv.notify_all();
}

std::shared_ptr<Table::Producer> Table::pending() const {
  std::lock_guard<std::mutex> lock(_pending_m);
  return _taken ? nullptr : _pending;
}

std::shared_ptr<Table::Producer> Table::take_pending() {
  std::lock_guard<std::mutex> lock(_pending_m);
  if (!_pending || _taken) return nullptr;
  _taken = true;
  return _pending;
}

void Table::fulfil(std::vector<std::shared_ptr<Chunk>>&& chunks) {
  std::lock_guard<std::mutex> lock(_pending_m);
  _chunks = std::move(chunks);
  _pending = nullptr;
  _taken = false;
  _pending_flag.store(false, std::memory_order_release);
  _pending_cv.notify_all();
}

void Table::resolve_slow() const {
  std::unique_lock<std::mutex> lock(_pending_m);
  // a consumer that took the producer fulfils the table: other accessors wait for it
  _pending_cv.wait(lock, [&] { return !_taken || !_pending; });
  if (!_pending) return;
  // the producer stays pending until produce() succeeds: a failing scan (Fail in produce) leaves the table pending,
  // so the error reaches every accessor instead of an empty table that looks valid
  const auto producer = _pending;
  auto chunks = producer->produce();
  _chunks = std::move(chunks);
  _pending = nullptr;
  _pending_flag.store(false, std::memory_order_release);
  _pending_cv.notify_all();
}

Table::~Table() {
  if (_chunks.size() >= BACKGROUND_RELEASE_CHUNKS) ChunkReaper::chunk_reaper().push(std::move(_chunks));
}

void release_drain() { ChunkReaper::chunk_reaper().drain(); }

void Table::append_chunks(std::vector<std::shared_ptr<Chunk>>&& chunks) {
  resolve();
#ifdef HYRISE_DEBUG  // (reference: DebugAssert, active in HYRISE_DEBUG builds)
  for (const auto& ch : chunks) {
    Assert(ch->column_count() == _defs.size(), "append_chunk: wrong number of columns");
    for (const auto& c : ch->columns()) {
      Assert(c->size() == ch->size(), "Columns don't have the same length");
      Assert(c->is_reference() == (_type == TableType::References), "Invalid column type");
    }
  }
#endif
  if (_chunks.empty()) {
    _chunks = std::move(chunks);
  } else {
    _chunks.reserve(_chunks.size() + chunks.size());
    for (auto& ch : chunks) _chunks.push_back(std::move(ch));
  }
}

AllTypeVariant Table::get_value(ColumnID column_id, uint64_t row) const {
  resolve();
  for (const auto& c : _chunks) {
    if (row < c->size()) return (*c->get_column(column_id))[static_cast<ChunkOffset>(row)];
    row -= c->size();
  }
  Fail("Row does not exist.");
}

AttributeVector::AttributeVector(const std::vector<uint32_t>& vids, uint32_t max_value,
                                 VectorCompressionType compression)
    : _compression(compression) {
  // reference fixed_size_byte_aligned_compressor.cpp:21-30: narrowest width that holds max_value
  _width = max_value <= 0xFFu ? 1 : (max_value <= 0xFFFFu ? 2 : 4);
  _size = vids.size();
  if (compression == VectorCompressionType::FixedSizeByteAligned) {
    _bytes.resize(_size * _width);
    for (size_t i = 0; i < _size; ++i) {
      const uint32_t v = vids[i];
      std::memcpy(_bytes.data() + i * _width, &v, _width);  // little endian
    }
    return;
  }
  // SIMD-BP128 (simd_bp128_compressor.cpp:13-120): meta blocks of 16 x 128 ids, the last one zero-padded; a meta
  // block's header word holds the 16 blocks' bit widths (the bits of the OR of the block's ids); then each of the
  // first ceil(ids left / 128) blocks packed into `width` words.
  std::vector<uint32_t> words;  // 4 per 16-byte word
  for (size_t m0 = 0; m0 < _size; m0 += BP128_META) {
    _meta.push_back(static_cast<uint32_t>(words.size() / 4));
    const size_t in_meta = std::min<size_t>(BP128_META, _size - m0);
    uint32_t widths[BP128_BLOCKS] = {0};
    for (uint32_t b = 0; b < BP128_BLOCKS; ++b) {
      uint32_t acc = 0;
      for (uint32_t i = 0; i < BP128_BLOCK; ++i) {
        const size_t k = m0 + b * BP128_BLOCK + i;
        if (k < _size) acc |= vids[k];
      }
      while (acc) {
        ++widths[b];
        acc >>= 1;
      }
    }
    uint32_t header[4] = {0, 0, 0, 0};
    uint8_t wb[16];
    for (uint32_t b = 0; b < BP128_BLOCKS; ++b) wb[b] = static_cast<uint8_t>(widths[b]);
    std::memcpy(header, wb, 16);
    words.insert(words.end(), header, header + 4);
    const uint32_t blocks = static_cast<uint32_t>((in_meta + BP128_BLOCK - 1) / BP128_BLOCK);
    for (uint32_t b = 0; b < blocks; ++b) {
      const uint32_t w = widths[b];
      const size_t base = words.size();
      words.resize(base + 4 * w, 0u);
      for (uint32_t i = 0; i < BP128_BLOCK && w; ++i) {
        const size_t k = m0 + b * BP128_BLOCK + i;
        const uint64_t v = k < _size ? vids[k] : 0u;
        const uint32_t lane = i & 3u, bit = (i >> 2) * w, word = bit >> 5, shift = bit & 31u;
        words[base + 4 * word + lane] |= static_cast<uint32_t>(v << shift);
        if (shift + w > 32) words[base + 4 * (word + 1) + lane] |= static_cast<uint32_t>(v >> (32 - shift));
      }
    }
  }
  _bytes.resize(words.size() * 4);
  if (!words.empty()) std::memcpy(_bytes.data(), words.data(), _bytes.size());
}

uint32_t AttributeVector::bp128_get(size_t i) const {
  const size_t m = i / BP128_META;
  const uint32_t b = static_cast<uint32_t>((i % BP128_META) / BP128_BLOCK), j = static_cast<uint32_t>(i % BP128_BLOCK);
  const uint8_t* header = _bytes.data() + 16ull * _meta[m];
  size_t word = _meta[m] + 1;
  for (uint32_t k = 0; k < b; ++k) word += header[k];
  const uint32_t w = header[b];
  if (w == 0) return 0;
  const uint32_t lane = j & 3u, bit = (j >> 2) * w, wi = bit >> 5, shift = bit & 31u;
  auto lane_word = [&](size_t k) {
    uint32_t v;
    std::memcpy(&v, _bytes.data() + 16 * k + 4 * lane, 4);
    return v;
  };
  uint64_t v = lane_word(word + wi) >> shift;
  if (shift + w > 32) v |= static_cast<uint64_t>(lane_word(word + wi + 1)) << (32 - shift);
  return w == 32 ? static_cast<uint32_t>(v) : static_cast<uint32_t>(v & ((1u << w) - 1u));
}

// reference dictionary_column/dictionary_encoder.hpp:57-130
std::shared_ptr<BaseColumn> encode_dictionary(const BaseColumn& base, VectorCompressionType compression) {
  std::shared_ptr<BaseColumn> out;
  resolve_data_type(base.data_type(), [&](auto tag) {
    using T = decltype(tag);
    const auto* vc = dynamic_cast<const ValueColumn<T>*>(&base);
    Assert(vc != nullptr, "encode_dictionary needs a ValueColumn");
    const auto& values = vc->values();
    std::vector<T> dict;
    dict.reserve(values.size());
    for (size_t i = 0; i < values.size(); ++i)
      if (!vc->is_null(static_cast<ChunkOffset>(i))) dict.push_back(values[i]);
    std::sort(dict.begin(), dict.end());
    dict.erase(std::unique(dict.begin(), dict.end()), dict.end());
    dict.shrink_to_fit();
    const auto null_value_id = static_cast<uint32_t>(dict.size());
    std::vector<uint32_t> vids(values.size());
    for (size_t i = 0; i < values.size(); ++i) {
      if (vc->is_null(static_cast<ChunkOffset>(i))) {
        vids[i] = null_value_id;
      } else {
        vids[i] = static_cast<uint32_t>(std::distance(dict.cbegin(), std::lower_bound(dict.cbegin(), dict.cend(), values[i])));
      }
    }
    const uint32_t max_value = static_cast<uint32_t>(dict.size() + 1u);
    auto av = std::make_shared<const AttributeVector>(vids, max_value, compression);
    out = std::make_shared<DictionaryColumn<T>>(std::make_shared<const std::vector<T>>(std::move(dict)), std::move(av),
                                                null_value_id);
  });
  return out;
}

// reference run_length_column/run_length_encoder.hpp:22-66: a new run starts when NULL-ness or the value changes
std::shared_ptr<BaseColumn> encode_run_length(const BaseColumn& base) {
  std::shared_ptr<BaseColumn> out;
  resolve_data_type(base.data_type(), [&](auto tag) {
    using T = decltype(tag);
    const auto* vc = dynamic_cast<const ValueColumn<T>*>(&base);
    Assert(vc != nullptr, "encode_run_length needs a ValueColumn");
    std::vector<T> values;
    std::vector<uint8_t> nulls;
    std::vector<ChunkOffset> ends;
    for (ChunkOffset i = 0; i < vc->size(); ++i) {
      const bool n = vc->is_null(i);
      const T v = n ? T{} : vc->values()[i];
      if (!ends.empty() && static_cast<bool>(nulls.back()) == n && (n || values.back() == v)) {
        ends.back() = i;
      } else {
        values.push_back(v);
        nulls.push_back(n ? 1 : 0);
        ends.push_back(i);
      }
    }
    out = std::make_shared<RunLengthColumn<T>>(std::move(values), std::move(nulls), std::move(ends));
  });
  return out;
}

// reference frame_of_reference/frame_of_reference_encoder.hpp:27-86 (NULL rows count as 0 for the block minimum)
std::shared_ptr<BaseColumn> encode_frame_of_reference(const BaseColumn& base) {
  std::shared_ptr<BaseColumn> out;
  resolve_data_type(base.data_type(), [&](auto tag) {
    using T = decltype(tag);
    if constexpr (std::is_same_v<T, int32_t> || std::is_same_v<T, int64_t>) {
      const auto* vc = dynamic_cast<const ValueColumn<T>*>(&base);
      Assert(vc != nullptr, "encode_frame_of_reference needs a ValueColumn");
      constexpr uint32_t B = FrameOfReferenceColumn<T>::block_size;
      const size_t n = vc->size();
      std::vector<T> minima;
      std::vector<uint8_t> nulls(n);
      std::vector<uint32_t> offsets(n);
      uint32_t max_offset = 0;
      for (size_t b = 0; b < n; b += B) {
        const size_t e = std::min(n, b + B);
        T mn = std::numeric_limits<T>::max(), mx = std::numeric_limits<T>::lowest();
        for (size_t i = b; i < e; ++i) {
          const T v = vc->is_null(static_cast<ChunkOffset>(i)) ? T{0} : vc->values()[i];
          mn = std::min(mn, v);
          mx = std::max(mx, v);
        }
        Assert(static_cast<std::make_unsigned_t<T>>(mx - mn) <= std::numeric_limits<uint32_t>::max(),
               "Value range in block must fit into uint32_t.");
        minima.push_back(mn);
        for (size_t i = b; i < e; ++i) {
          const bool isn = vc->is_null(static_cast<ChunkOffset>(i));
          nulls[i] = isn ? 1 : 0;
          offsets[i] = static_cast<uint32_t>((isn ? T{0} : vc->values()[i]) - mn);
          max_offset = std::max(max_offset, offsets[i]);
        }
      }
      auto av = std::make_shared<const AttributeVector>(offsets, max_offset);
      out = std::make_shared<FrameOfReferenceColumn<T>>(std::move(minima), std::move(nulls), std::move(av));
    } else {
      Fail("FrameOfReference encoding supports int and long columns only");
    }
  });
  return out;
}

// reference dictionary_column/dictionary_encoder.hpp:36-48, 132-138 with EncodingType::FixedStringDictionary: the
// values as FixedStrings of the longest value's length (a value reads back up to its first '\0'), sorted and unique;
// std::string columns only.
std::shared_ptr<BaseColumn> encode_fixed_string_dictionary(const BaseColumn& base, VectorCompressionType compression) {
  const auto* vc = dynamic_cast<const ValueColumn<std::string>*>(&base);
  if (!vc) Fail("FixedStringDictionary encoding supports string columns only");
  const auto& values = vc->values();
  size_t len = 0;
  for (const auto& v : values) len = std::max(len, v.size());
  auto fixed = [&](const std::string& v) { return std::string(v.data(), strnlen(v.data(), v.size())); };
  std::vector<std::string> dict;
  dict.reserve(values.size());
  for (size_t i = 0; i < values.size(); ++i)
    if (!vc->is_null(static_cast<ChunkOffset>(i))) dict.push_back(fixed(values[i]));
  std::sort(dict.begin(), dict.end());
  dict.erase(std::unique(dict.begin(), dict.end()), dict.end());
  const auto null_value_id = static_cast<uint32_t>(dict.size());
  std::vector<uint32_t> vids(values.size());
  for (size_t i = 0; i < values.size(); ++i)
    vids[i] = vc->is_null(static_cast<ChunkOffset>(i))
                  ? null_value_id
                  : static_cast<uint32_t>(std::lower_bound(dict.cbegin(), dict.cend(), fixed(values[i])) - dict.cbegin());
  std::vector<char> chars(len ? len * dict.size() : 1, '\0');  // (fixed_string_vector.hpp:27-33: one byte if len 0)
  for (size_t i = 0; i < dict.size() && len; ++i) std::memcpy(chars.data() + i * len, dict[i].data(), dict[i].size());
  auto av = std::make_shared<const AttributeVector>(vids, static_cast<uint32_t>(dict.size() + 1u), compression);
  return std::make_shared<FixedStringDictionaryColumn>(std::move(chars), len, dict.size(), std::move(av), null_value_id);
}

namespace {
std::shared_ptr<BaseColumn> encode_column(const BaseColumn& col, EncodingType encoding,
                                          VectorCompressionType compression) {
  switch (encoding) {
    case EncodingType::Dictionary:
      return encode_dictionary(col, compression);
    case EncodingType::FixedStringDictionary:
      return encode_fixed_string_dictionary(col, compression);
    case EncodingType::RunLength:
      return encode_run_length(col);
    case EncodingType::FrameOfReference:
      return encode_frame_of_reference(col);
    default:
      Fail("Encoding type not supported by the device path");
  }
}
}  // namespace

void ChunkEncoder::encode_chunks(const std::shared_ptr<Table>& table, const std::vector<ChunkID>& chunk_ids,
                                 EncodingType encoding, VectorCompressionType compression) {
  Assert(table->type() == TableType::Data, "Only data tables can be encoded");
  if (encoding == EncodingType::Unencoded) return;
  for (const auto chunk_id : chunk_ids) {
    const auto chunk = table->get_chunk(chunk_id);
    for (ColumnID c = 0; c < chunk->column_count(); ++c) {
      const auto col = chunk->get_column(c);
      if (col->encoding_type() != EncodingType::Unencoded) continue;  // already encoded
      // the reference's ChunkEncoder leaves string columns FrameOfReference cannot encode to the caller's spec;
      // here FrameOfReference on a non-integer column keeps it unencoded
      if (encoding == EncodingType::FrameOfReference && col->data_type() != DataType::Int &&
          col->data_type() != DataType::Long)
        continue;
      // likewise FixedStringDictionary (a string-only encoding) keeps numeric columns unencoded
      if (encoding == EncodingType::FixedStringDictionary && col->data_type() != DataType::String) continue;
      chunk->replace_column(c, encode_column(*col, encoding, compression));
    }
  }
}

void ChunkEncoder::encode_columns(const std::shared_ptr<Table>& table, const std::vector<ColumnID>& column_ids,
                                  EncodingType encoding, VectorCompressionType compression) {
  Assert(table->type() == TableType::Data, "Only data tables can be encoded");
  if (encoding == EncodingType::Unencoded) return;
  // chunks are independent: encoded in parallel (the reference encodes chunk by chunk in jobs as well)
  const ChunkID n = table->chunk_count();
  const unsigned workers = std::max(1u, std::min(16u, host_cpu_share()));
  std::atomic<ChunkID> next{0};
  auto work = [&]() {
    for (ChunkID c; (c = next.fetch_add(1)) < n;) {
      const auto chunk = table->get_chunk(c);
      for (const auto col_id : column_ids) {
        const auto col = chunk->get_column(col_id);
        // (the reference's per-column ChunkEncodingSpec, chunk_encoder.cpp: a column already in `encoding` stays)
        if (col->encoding_type() == encoding) continue;
        if (col->encoding_type() != EncodingType::Unencoded) Fail("encode_columns re-encodes unencoded columns only");
        chunk->replace_column(col_id, encode_column(*col, encoding, compression));
      }
    }
  };
  std::vector<std::thread> pool;
  for (unsigned i = 1; i < workers; ++i) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
}

void ChunkEncoder::encode_all_chunks(const std::shared_ptr<Table>& table, EncodingType encoding,
                                     VectorCompressionType compression) {
  std::vector<ChunkID> ids(table->chunk_count());
  for (ChunkID i = 0; i < ids.size(); ++i) ids[i] = i;
  encode_chunks(table, ids, encoding, compression);
}

namespace {
std::vector<std::string> split(const std::string& s, char delim) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, delim)) out.push_back(item);
  return out;
}
}  // namespace

// reference src/lib/utils/load_table.cpp:14-62
std::shared_ptr<Table> load_table(const std::string& file_name, uint32_t chunk_size) {
  std::ifstream infile(file_name);
  Assert(infile.is_open(), "load_table: Could not find file " + file_name);
  std::string line;
  std::getline(infile, line);
  const auto names = split(line, '|');
  std::getline(infile, line);
  auto types = split(line, '|');
  TableColumnDefinitions defs;
  std::vector<bool> nullable;
  for (size_t i = 0; i < names.size(); ++i) {
    const auto parts = split(types.at(i), '_');
    const bool is_nullable = parts.size() > 1 && parts[1] == "null";
    nullable.push_back(is_nullable);
    defs.emplace_back(names[i], data_type_from_string(parts[0]), is_nullable);
  }
  auto table = std::make_shared<Table>(defs, TableType::Data, chunk_size);
  while (std::getline(infile, line)) {
    auto fields = split(line, '|');
    std::vector<AllTypeVariant> values;
    for (size_t i = 0; i < fields.size(); ++i) {
      if (nullable[i] && fields[i] == "null")
        values.emplace_back(NullValue{});
      else
        values.emplace_back(fields[i]);
    }
    // a trailing empty string field is dropped by getline-split; restore it
    while (values.size() < defs.size()) values.emplace_back(std::string{});
    table->append(values);
  }
  return table;
}

}  // namespace hyrise
