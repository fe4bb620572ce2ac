// Core vocabulary of the host-side operator layer.
//
// Mirrors the reference's row addressing and type system so that operator outputs are byte-identical:
//   RowID / PosList / ChunkID / ChunkOffset / ValueID / NULL_ROW_ID / INVALID_VALUE_ID
//       -> reference src/lib/types.hpp:38-43, 92, 97-131, 138, 150-155
//   AllTypeVariant (Null, int32, int64, float, double, string)
//       -> reference src/lib/all_type_variant.hpp (data_types list)
//   type_cast<T>(AllTypeVariant) semantics (lexical cast; integral targets truncate through double)
//       -> reference src/lib/type_cast.hpp:39-58
//
// Boost and TBB are not available, so std::variant replaces boost::variant and std::vector replaces
// tbb::concurrent_vector / pmr vectors. Only the observable semantics are kept.
#pragma once

#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <initializer_list>
#include <iterator>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <string>
#include <variant>
#include <vector>

namespace hyrise {

using ChunkID = uint32_t;
using ChunkOffset = uint32_t;
using ColumnID = uint16_t;
using ValueID = uint32_t;

constexpr ChunkOffset INVALID_CHUNK_OFFSET = std::numeric_limits<ChunkOffset>::max();
constexpr ChunkID INVALID_CHUNK_ID = std::numeric_limits<ChunkID>::max();
constexpr ValueID INVALID_VALUE_ID = std::numeric_limits<ValueID>::max();
constexpr ValueID NULL_VALUE_ID = std::numeric_limits<ValueID>::max();
constexpr ColumnID INVALID_COLUMN_ID = std::numeric_limits<ColumnID>::max();
// reference chunk.hpp:44
constexpr ChunkOffset CHUNK_MAX_SIZE = std::numeric_limits<ChunkOffset>::max() - 1;

// 8-byte row address, identical layout to the reference's RowID {ChunkID chunk_id; ChunkOffset chunk_offset;}.
struct RowID {
  ChunkID chunk_id{INVALID_CHUNK_ID};
  ChunkOffset chunk_offset{INVALID_CHUNK_OFFSET};

  RowID() = default;
  RowID(ChunkID c, ChunkOffset o) : chunk_id(c), chunk_offset(o) {}

  bool is_null() const { return chunk_offset == INVALID_CHUNK_OFFSET; }
  bool operator==(const RowID& o) const { return chunk_id == o.chunk_id && chunk_offset == o.chunk_offset; }
  bool operator!=(const RowID& o) const { return !(*this == o); }
  bool operator<(const RowID& o) const {
    return chunk_id < o.chunk_id || (chunk_id == o.chunk_id && chunk_offset < o.chunk_offset);
  }
};
static_assert(sizeof(RowID) == 8, "RowID must be 8 bytes like the reference");

inline const RowID NULL_ROW_ID = RowID{INVALID_CHUNK_ID, INVALID_CHUNK_OFFSET};

struct DevicePosList;  // device.hpp

class PosList;
// Copies a device-produced PosList's RowIDs to `dst` (the device layer's function, device.cpp). Carried by each lazy
// PosList, so code in another shared object (the oracle module) reading it calls the producer's copy routine.
using PosListFetch = void (*)(const PosList& pos_list, RowID* dst);

// PosList: the reference's `using PosList = pmr_vector<RowID>` (types.hpp:138) as a class with the same vector
// interface (every member the reference's operators call on a PosList: size / empty / operator[] / at / data /
// begin / end / cbegin / cend / front / back / push_back / emplace_back / reserve / resize / shrink_to_fit / clear /
// insert / capacity / ==) plus an optional device-resident mirror in the same 8-byte layout, so that a downstream GPU
// operator does not re-upload what an upstream GPU operator produced. A PosList a GPU operator produces is lazy: it
// knows its size and holds only the device mirror; the host RowIDs are copied down on the first host access through
// ANY member. The vector is a private member, not a base class: no access path can see the unfilled storage of a
// lazy list. Code that needs the std::vector itself takes vector() (host copy made first). INTEGRATION.md 2 lists
// this as the one type change of the drop-in.
class PosList {
  using Vec = std::vector<RowID>;

 public:
  using value_type = RowID;
  using size_type = Vec::size_type;
  using difference_type = Vec::difference_type;
  using reference = RowID&;
  using const_reference = const RowID&;
  using pointer = RowID*;
  using const_pointer = const RowID*;
  using iterator = Vec::iterator;
  using const_iterator = Vec::const_iterator;

  PosList() = default;
  explicit PosList(size_t n) : _v(n) {}
  PosList(size_t n, const RowID& value) : _v(n, value) {}
  PosList(std::initializer_list<RowID> l) : _v(l) {}
  template <typename It, typename = typename std::iterator_traits<It>::iterator_category>
  PosList(It first, It last) : _v(first, last) {}
  explicit PosList(Vec&& v) : _v(std::move(v)) {}
  PosList(const PosList& o) : _v(o.host()), _single_chunk_id(o._single_chunk_id) {}
  PosList& operator=(const PosList& o) {
    if (this != &o) {
      Vec copy = o.host();
      _v = std::move(copy);
      _state.store(HOST, std::memory_order_relaxed);
      _device.reset();
      _single_chunk_id = o._single_chunk_id;
    }
    return *this;
  }

  // A PosList of n RowIDs that live on the device (its mirror is set by the producer; fetch copies them down).
  static std::shared_ptr<PosList> lazy(size_t n, PosListFetch fetch) {
    auto p = std::make_shared<PosList>();
    p->_lazy_size = n;
    p->_state.store(n > 0 ? LAZY : HOST, std::memory_order_relaxed);
    p->_fetch = fetch;
    return p;
  }
  bool is_lazy() const { return _state.load(std::memory_order_acquire) != HOST; }
  // makes an empty list lazy in place (lists allocated in an operator's output arena)
  // with its device mirror (a plain store: the list is not shared with any other thread yet)
  void make_lazy(size_t n, PosListFetch fetch, std::shared_ptr<DevicePosList> mirror) {
    _v.clear();
    _lazy_size = n;
    _state.store(n > 0 ? LAZY : HOST, std::memory_order_relaxed);
    _fetch = fetch;
    _device = std::move(mirror);
  }
  // the size of a lazy list that is not shared yet (its producer learns the sizes after creating the lists)
  void set_lazy_size(size_t n) {
    _lazy_size = n;
    _state.store(n > 0 ? LAZY : HOST, std::memory_order_relaxed);
  }

  // sizes need no host copy
  size_t size() const { return is_lazy() ? _lazy_size : _v.size(); }
  bool empty() const { return size() == 0; }
  size_t capacity() const { return is_lazy() ? _lazy_size : _v.capacity(); }
  // element and iterator access: the host RowIDs (copied down first when lazy)
  const RowID& operator[](size_t i) const { return host()[i]; }
  RowID& operator[](size_t i) { return host()[i]; }
  const RowID& at(size_t i) const { return host().at(i); }
  RowID& at(size_t i) { return host().at(i); }
  const RowID* data() const { return host().data(); }
  RowID* data() { return host().data(); }
  const_iterator begin() const { return host().begin(); }
  const_iterator end() const { return host().end(); }
  const_iterator cbegin() const { return host().cbegin(); }
  const_iterator cend() const { return host().cend(); }
  iterator begin() { return host().begin(); }
  iterator end() { return host().end(); }
  const RowID& front() const { return host().front(); }
  const RowID& back() const { return host().back(); }
  RowID& front() { return host().front(); }
  RowID& back() { return host().back(); }
  const Vec& vector() const { return host(); }
  // modifiers: the list becomes a plain host list; a device mirror no longer matches it and is dropped
  void push_back(const RowID& r) { mutate().push_back(r); }
  template <typename... A>
  RowID& emplace_back(A&&... a) {
    return mutate().emplace_back(std::forward<A>(a)...);
  }
  void reserve(size_t n) { host_mut().reserve(n); }
  void shrink_to_fit() { host_mut().shrink_to_fit(); }
  void resize(size_t n) { mutate().resize(n); }
  void resize(size_t n, const RowID& v) { mutate().resize(n, v); }
  void clear() { mutate().clear(); }
  template <typename It>
  iterator insert(const_iterator pos, It first, It last) {
    const auto off = pos - host().cbegin();
    auto& v = mutate();
    return v.insert(v.cbegin() + off, first, last);
  }
  bool operator==(const PosList& o) const { return host() == o.host(); }
  bool operator!=(const PosList& o) const { return !(*this == o); }

  std::shared_ptr<DevicePosList> device_mirror() const { return std::atomic_load(&_device); }
  void set_device_mirror(std::shared_ptr<DevicePosList> d) const { std::atomic_store(&_device, std::move(d)); }

  // The only chunk every non-NULL RowID points into, when the producer knows it (a TableScan over a data table emits
  // one PosList per input chunk); INVALID_CHUNK_ID when unknown or mixed. Lets GPU consumers read that chunk's
  // descriptor once per workgroup instead of once per row.
  ChunkID single_chunk_id() const { return _single_chunk_id; }
  void set_single_chunk_id(ChunkID c) { _single_chunk_id = c; }

 private:
  // The first host access of a lazy list copies it down; concurrent readers of the same list wait for that copy, readers
  // of other lists are not involved (the state is per list: LAZY -> FETCHING -> HOST).
  Vec& host() const {
    auto& self = const_cast<PosList&>(*this);
    if (_state.load(std::memory_order_acquire) != HOST) self.fetch_once();
    return self._v;
  }
  void fetch_once() {
    uint8_t expected = LAZY;
    if (_state.compare_exchange_strong(expected, FETCHING, std::memory_order_acq_rel)) {
      try {
        _v.resize(_lazy_size);
        _fetch(*this, _v.data());
      } catch (...) {
        _state.store(LAZY, std::memory_order_release);
        throw;
      }
      _state.store(HOST, std::memory_order_release);
      return;
    }
    while (_state.load(std::memory_order_acquire) == FETCHING) std::this_thread::yield();
    if (_state.load(std::memory_order_acquire) == LAZY) fetch_once();  // (the fetching reader failed: try again)
  }
  Vec& host_mut() { return host(); }
  Vec& mutate() {
    Vec& v = host();
    if (_device) set_device_mirror(nullptr);
    _single_chunk_id = INVALID_CHUNK_ID;
    return v;
  }

  Vec _v;
  mutable std::shared_ptr<DevicePosList> _device;
  ChunkID _single_chunk_id = INVALID_CHUNK_ID;
  size_t _lazy_size = 0;
  static constexpr uint8_t HOST = 0, LAZY = 1, FETCHING = 2;
  mutable std::atomic<uint8_t> _state{HOST};
  PosListFetch _fetch = nullptr;
};

enum class DataType : uint8_t { Null, Int, Long, Float, Double, String };

enum class PredicateCondition {
  Equals,
  NotEquals,
  LessThan,
  LessThanEquals,
  GreaterThan,
  GreaterThanEquals,
  Between,
  In,
  Like,
  NotLike,
  IsNull,
  IsNotNull
};

enum class JoinMode { Inner, Left, Right, Outer, Cross, Semi, Anti };
enum class TableType { References, Data };
enum class EncodingType : uint8_t { Unencoded, Dictionary, RunLength, FixedStringDictionary, FrameOfReference };
// reference storage/vector_compression/vector_compression.hpp: how a DictionaryColumn's attribute vector is stored
enum class VectorCompressionType : uint8_t { FixedSizeByteAligned, SimdBp128 };
enum class AggregateFunction { Min, Max, Sum, Avg, Count, CountDistinct };

struct NullValue {
  bool operator==(const NullValue&) const { return true; }
};

using AllTypeVariant = std::variant<NullValue, int32_t, int64_t, float, double, std::string>;

inline bool variant_is_null(const AllTypeVariant& v) { return v.index() == 0; }

// Errors: the reference's Fail/Assert throw std::logic_error (src/lib/utils/assert.hpp:49-70).
[[noreturn]] inline void Fail(const std::string& msg) { throw std::logic_error(msg); }
inline void Assert(bool cond, const std::string& msg) {
  if (!cond) Fail(msg);
}

template <typename T>
constexpr DataType data_type_from_type() {
  if constexpr (std::is_same_v<T, int32_t>) return DataType::Int;
  if constexpr (std::is_same_v<T, int64_t>) return DataType::Long;
  if constexpr (std::is_same_v<T, float>) return DataType::Float;
  if constexpr (std::is_same_v<T, double>) return DataType::Double;
  if constexpr (std::is_same_v<T, std::string>) return DataType::String;
  return DataType::Null;
}

inline size_t data_type_size(DataType t) {
  switch (t) {
    case DataType::Int:
    case DataType::Float:
      return 4;
    case DataType::Long:
    case DataType::Double:
      return 8;
    default:
      return 0;
  }
}

inline std::string data_type_to_string(DataType t) {
  switch (t) {
    case DataType::Int:
      return "int";
    case DataType::Long:
      return "long";
    case DataType::Float:
      return "float";
    case DataType::Double:
      return "double";
    case DataType::String:
      return "string";
    default:
      return "null";
  }
}

inline DataType data_type_from_string(const std::string& s) {
  if (s == "int") return DataType::Int;
  if (s == "long") return DataType::Long;
  if (s == "float") return DataType::Float;
  if (s == "double") return DataType::Double;
  if (s == "string") return DataType::String;
  Fail("Invalid data type " + s);
}

// Calls f(T{}) with the C++ type of the data type (reference resolve_type.hpp resolve_data_type).
template <typename F>
void resolve_data_type(DataType t, F&& f) {
  switch (t) {
    case DataType::Int:
      f(int32_t{});
      return;
    case DataType::Long:
      f(int64_t{});
      return;
    case DataType::Float:
      f(float{});
      return;
    case DataType::Double:
      f(double{});
      return;
    case DataType::String:
      f(std::string{});
      return;
    default:
      Fail("Cannot resolve Null data type");
  }
}

namespace detail {

// boost::lexical_cast<Target>(AllTypeVariant) streams the held value with precision
// max(precision(variant)=6, precision(Target)): Target float -> 9, double -> 17, otherwise 6 (boost
// lcast_set_precision). Default float formatting of an ostream at precision p is printf's %.<p>g.
inline std::string to_lexical_string(const AllTypeVariant& v, int precision) {
  char buf[64];
  switch (v.index()) {
    case 1:
      return std::to_string(std::get<int32_t>(v));
    case 2:
      return std::to_string(std::get<int64_t>(v));
    case 3:
      std::snprintf(buf, sizeof(buf), "%.*g", precision, static_cast<double>(std::get<float>(v)));
      return buf;
    case 4:
      std::snprintf(buf, sizeof(buf), "%.*g", precision, std::get<double>(v));
      return buf;
    case 5:
      return std::get<std::string>(v);
    default:
      Fail("Cannot cast NULL");
  }
}

// boost::lexical_cast<Integral>(string): the whole string must be an integer within range.
template <typename T>
bool try_parse_integral(const std::string& s, T& out) {
  if (s.empty()) return false;
  errno = 0;
  char* end = nullptr;
  long long val = std::strtoll(s.c_str(), &end, 10);
  if (end != s.c_str() + s.size() || errno == ERANGE) return false;
  if (val < static_cast<long long>(std::numeric_limits<T>::min()) ||
      val > static_cast<long long>(std::numeric_limits<T>::max()))
    return false;
  // lexical_cast rejects leading whitespace / '+' differently; fixture values never use them.
  out = static_cast<T>(val);
  return true;
}

}  // namespace detail

// type_cast<T>(AllTypeVariant): reference type_cast.hpp:39-58.
//  * same type -> the value itself
//  * non-integral target -> lexical_cast (via the round-trip text of the source)
//  * integral target -> try_lexical_convert, else numeric_cast<T>(lexical_cast<double>(v)), which truncates
//    toward zero and throws on overflow (boost::numeric::bad_numeric_cast -> mapped to std::logic_error here).
template <typename T>
T type_cast(const AllTypeVariant& v) {
  if (const T* p = std::get_if<T>(&v)) return *p;
  if (variant_is_null(v)) Fail("type_cast of NULL");
  if constexpr (std::is_same_v<T, std::string>) {
    return detail::to_lexical_string(v, 6);
  } else if constexpr (std::is_floating_point_v<T>) {
    const std::string text = detail::to_lexical_string(v, std::is_same_v<T, float> ? 9 : 17);
    char* end = nullptr;
    T out;
    if constexpr (std::is_same_v<T, float>) {
      out = std::strtof(text.c_str(), &end);
    } else {
      out = std::strtod(text.c_str(), &end);
    }
    if (end != text.c_str() + text.size() || text.empty()) Fail("bad lexical cast: " + text);
    return out;
  } else {
    T out;
    if (detail::try_parse_integral<T>(detail::to_lexical_string(v, 6), out)) return out;
    const std::string text = detail::to_lexical_string(v, 17);
    char* end = nullptr;
    const double d = std::strtod(text.c_str(), &end);
    if (end != text.c_str() + text.size() || text.empty()) Fail("bad lexical cast: " + text);
    const double t = std::trunc(d);
    if (!(t >= static_cast<double>(std::numeric_limits<T>::min()) &&
          t <= static_cast<double>(std::numeric_limits<T>::max())))
      Fail("bad numeric cast: overflow");
    return static_cast<T>(t);
  }
}

inline DataType variant_data_type(const AllTypeVariant& v) {
  switch (v.index()) {
    case 1:
      return DataType::Int;
    case 2:
      return DataType::Long;
    case 3:
      return DataType::Float;
    case 4:
      return DataType::Double;
    case 5:
      return DataType::String;
    default:
      return DataType::Null;
  }
}

inline std::string predicate_condition_to_string(PredicateCondition c) {
  switch (c) {
    case PredicateCondition::Equals:
      return "=";
    case PredicateCondition::NotEquals:
      return "!=";
    case PredicateCondition::LessThan:
      return "<";
    case PredicateCondition::LessThanEquals:
      return "<=";
    case PredicateCondition::GreaterThan:
      return ">";
    case PredicateCondition::GreaterThanEquals:
      return ">=";
    case PredicateCondition::Between:
      return "BETWEEN";
    case PredicateCondition::In:
      return "IN";
    case PredicateCondition::Like:
      return "LIKE";
    case PredicateCondition::NotLike:
      return "NOT LIKE";
    case PredicateCondition::IsNull:
      return "IS NULL";
    case PredicateCondition::IsNotNull:
      return "IS NOT NULL";
  }
  return "?";
}

}  // namespace hyrise
