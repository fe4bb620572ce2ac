// Binary table files (the reference's ImportBinary / ExportBinary, src/lib/operators/import_binary.cpp and
// export_binary.cpp, format in export_binary.hpp:38-171): the way Hyrise persists and reloads encoded tables.
// Importing keeps every chunk in its stored encoding - a dictionary column's FixedSizeByteAligned attribute vector is
// the file's bytes - so load_to_device() then uploads exactly those bytes to HBM (the same 1 B/row l_quantity the
// scan kernels read), with no re-encoding between disk and device.
//
//   header  chunk size (u32) | chunk count (u32) | column count (u16) | type names (size_t lengths + chars) |
//           nullable flags (u8 each) | column names (size_t lengths + chars)
//   chunk   row count (u32), then per column: BinaryColumnType (u8: 0 value, 1 dictionary) and
//           value:      [null flags, u8 per row, if the column is nullable] values (T per row; strings: size_t
//                       lengths then chars)
//           dictionary: attribute-vector width (u8) | dictionary size (u32) | dictionary values | attribute vector
#include <cstring>
#include <fstream>
#include <numeric>

#include "device.hpp"
#include "storage.hpp"

namespace hyrise {

namespace {

enum class BinaryColumnType : uint8_t { value_column = 0, dictionary_column = 1 };

template <typename T>
T read_value(std::ifstream& f) {
  T v;
  f.read(reinterpret_cast<char*>(&v), sizeof(T));
  return v;
}

template <typename T>
std::vector<T> read_values(std::ifstream& f, size_t n) {
  std::vector<T> v(n);
  if (n) f.read(reinterpret_cast<char*>(v.data()), n * sizeof(T));
  return v;
}

std::vector<std::string> read_strings(std::ifstream& f, size_t n) {
  const auto lengths = read_values<size_t>(f, n);
  const auto chars = read_values<char>(f, std::accumulate(lengths.begin(), lengths.end(), size_t{0}));
  std::vector<std::string> out(n);
  size_t at = 0;
  for (size_t i = 0; i < n; ++i) {
    out[i].assign(chars.data() + at, lengths[i]);
    at += lengths[i];
  }
  return out;
}

template <typename T>
std::vector<T> read_typed(std::ifstream& f, size_t n) {
  if constexpr (std::is_same_v<T, std::string>)
    return read_strings(f, n);
  else
    return read_values<T>(f, n);
}

template <typename T>
std::shared_ptr<BaseColumn> import_column(std::ifstream& f, uint32_t rows, bool nullable) {
  const auto kind = read_value<BinaryColumnType>(f);
  if (kind == BinaryColumnType::value_column) {  // import_binary.cpp:200-215
    std::optional<std::vector<uint8_t>> nulls;
    if (nullable) nulls = read_values<uint8_t>(f, rows);
    auto values = read_typed<T>(f, rows);
    return std::make_shared<ValueColumn<T>>(std::move(values), std::move(nulls));
  }
  if (kind == BinaryColumnType::dictionary_column) {  // import_binary.cpp:217-227
    const auto width = read_value<uint8_t>(f);
    const auto dict_size = read_value<uint32_t>(f);
    auto dictionary = std::make_shared<std::vector<T>>(read_typed<T>(f, dict_size));
    if (width != 1 && width != 2 && width != 4) Fail("Cannot import attribute vector with width: " + std::to_string(width));
    auto bytes = read_values<uint8_t>(f, size_t(rows) * width);
    auto av = std::make_shared<AttributeVector>(std::move(bytes), width, rows);
    return std::make_shared<DictionaryColumn<T>>(dictionary, av, dict_size);
  }
  Fail("Cannot import column: invalid column type");
}

template <typename T>
void write_value(std::ofstream& f, const T& v) {
  f.write(reinterpret_cast<const char*>(&v), sizeof(T));
}

template <typename T>
void write_values(std::ofstream& f, const std::vector<T>& v) {
  if constexpr (std::is_same_v<T, std::string>) {
    std::vector<size_t> lengths(v.size());
    std::string chars;
    for (size_t i = 0; i < v.size(); ++i) {
      lengths[i] = v[i].size();
      chars += v[i];
    }
    write_values(f, lengths);
    if (!chars.empty()) f.write(chars.data(), static_cast<std::streamsize>(chars.size()));
  } else {
    if (!v.empty()) f.write(reinterpret_cast<const char*>(v.data()), static_cast<std::streamsize>(v.size() * sizeof(T)));
  }
}

template <typename T>
void export_column(std::ofstream& f, const BaseColumn& column) {
  if (const auto* vc = dynamic_cast<const ValueColumn<T>*>(&column)) {  // export_binary.cpp:148-158
    write_value(f, BinaryColumnType::value_column);
    if (vc->is_nullable()) write_values(f, vc->null_values());
    write_values(f, vc->values());
    return;
  }
  if (const auto* dc = dynamic_cast<const DictionaryColumn<T>*>(&column)) {  // export_binary.cpp:186-219
    write_value(f, BinaryColumnType::dictionary_column);
    const auto& av = dc->attribute_vector();
    Assert(av.compression() == VectorCompressionType::FixedSizeByteAligned,  // export_binary.cpp:243-254
           "Does only support fixed-size byte-aligned compressed attribute vectors.");
    write_value(f, static_cast<uint8_t>(av.width()));
    write_value(f, static_cast<uint32_t>(dc->dictionary().size()));
    write_values(f, dc->dictionary());
    const auto& bytes = av.bytes();
    if (!bytes.empty()) f.write(reinterpret_cast<const char*>(bytes.data()), static_cast<std::streamsize>(bytes.size()));
    return;
  }
  if (column.is_reference()) {  // export_binary.cpp:160-184: materialised values, no NULL flags
    write_value(f, BinaryColumnType::value_column);
    std::vector<T> values(column.size());
    for (ChunkOffset r = 0; r < column.size(); ++r) values[r] = type_cast<T>(column[r]);
    write_values(f, values);
    return;
  }
  Fail("ExportBinary: unsupported column encoding");
}

}  // namespace

// reference import_binary.cpp:62-133
std::shared_ptr<Table> import_binary(const std::string& filename) {
  std::ifstream f(filename, std::ios::binary);
  Assert(f.is_open(), "ImportBinary: Could not find file " + filename);
  f.exceptions(std::ifstream::failbit | std::ifstream::badbit);
  const auto chunk_size = read_value<uint32_t>(f);
  const auto chunk_count = read_value<uint32_t>(f);
  const auto column_count = read_value<uint16_t>(f);
  const auto types = read_strings(f, column_count);
  const auto nullable = read_values<uint8_t>(f, column_count);
  const auto names = read_strings(f, column_count);
  TableColumnDefinitions defs;
  for (uint16_t c = 0; c < column_count; ++c) defs.emplace_back(names[c], data_type_from_string(types[c]), nullable[c] != 0);
  auto table = std::make_shared<Table>(defs, TableType::Data, chunk_size);
  for (uint32_t k = 0; k < chunk_count; ++k) {
    const auto rows = read_value<uint32_t>(f);
    ChunkColumns cols;
    for (uint16_t c = 0; c < column_count; ++c) {
      resolve_data_type(defs[c].data_type, [&](auto tag) {
        using T = decltype(tag);
        cols.push_back(import_column<T>(f, rows, defs[c].nullable));
      });
    }
    table->append_chunk(cols);
  }
  return table;
}

// reference export_binary.cpp:86-146
void export_binary(const std::shared_ptr<const Table>& table, const std::string& filename) {
  std::ofstream f;
  f.exceptions(std::ofstream::failbit | std::ofstream::badbit);
  f.open(filename, std::ios::binary);
  write_value(f, static_cast<uint32_t>(table->max_chunk_size()));
  write_value(f, static_cast<uint32_t>(table->chunk_count()));
  write_value(f, static_cast<uint16_t>(table->column_count()));
  std::vector<std::string> types, names;
  std::vector<uint8_t> nullable;
  for (ColumnID c = 0; c < table->column_count(); ++c) {
    types.push_back(data_type_to_string(table->column_data_type(c)));
    names.push_back(table->column_name(c));
    nullable.push_back(table->column_is_nullable(c) ? 1 : 0);
  }
  write_values(f, types);
  write_values(f, nullable);
  write_values(f, names);
  for (ChunkID k = 0; k < table->chunk_count(); ++k) {
    const auto chunk = table->get_chunk(k);
    write_value(f, static_cast<uint32_t>(chunk->size()));
    for (ColumnID c = 0; c < table->column_count(); ++c) {
      resolve_data_type(table->column_data_type(c), [&](auto tag) {
        using T = decltype(tag);
        export_column<T>(f, *chunk->get_column(c));
      });
    }
  }
}

// The HBM mirrors of every numeric column chunk of a data table (string columns stay host-side: the device path
// takes them as dictionary codes), created now instead of on first use.
void load_to_device(const std::shared_ptr<const Table>& table) {
  for (ChunkID k = 0; k < table->chunk_count(); ++k)
    for (ColumnID c = 0; c < table->column_count(); ++c)
      if (table->column_data_type(c) != DataType::String) device_column(*table->get_chunk(k)->get_column(c));
  hy_check(hy_stream_synchronize(operator_stream()), "hy_stream_synchronize");
}

}  // namespace hyrise
