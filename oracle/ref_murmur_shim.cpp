// C entry points over the reference's own murmur_hash.cpp (compiled from /root/reference, never copied).
#include "utils/murmur_hash.hpp"
#include <cstdint>
#include <string>
extern "C" {
unsigned int ref_murmur2_int32(int32_t v, unsigned int seed) { return opossum::murmur2<int32_t>(v, seed); }
unsigned int ref_murmur2_int64(int64_t v, unsigned int seed) { return opossum::murmur2<int64_t>(v, seed); }
unsigned int ref_murmur2_float(float v, unsigned int seed) { return opossum::murmur2<float>(v, seed); }
unsigned int ref_murmur2_double(double v, unsigned int seed) { return opossum::murmur2<double>(v, seed); }
unsigned int ref_murmur_hash2(const char* s, unsigned int len, unsigned int seed) {
  return opossum::murmur2<std::string>(std::string(s, len), seed);
}
}
