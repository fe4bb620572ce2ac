// Native check of the C-ABI's RCCL exchange (hy_comm_*, hy_join_exchange_counts / _records) in a process without
// any other runtime - the way a C++ Hyrise process links libhyrise_amd.so. One rank (RCCL refuses two ranks on one
// device): counts all-gathered unchanged, records routed to the rank's own buckets in bucket order, the counts matrix
// for step 2, HY_ERR_CAPACITY with the exact row count for a too-small buffer. Prints "exchange_check ok".
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "hyrise_amd.h"

#define CHECK(x)                                                                       \
  do {                                                                                 \
    const hy_status s_ = (x);                                                          \
    if (s_ != HY_OK) {                                                                 \
      std::printf("FAIL %s -> %d: %s\n", #x, static_cast<int>(s_), hy_last_error_message()); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

int main() {
  CHECK(hy_set_device(0));
  hy_comm_id id;
  CHECK(hy_comm_get_unique_id(&id));
  hy_comm_t comm = nullptr;
  CHECK(hy_comm_init(&comm, 1, &id, 0));
  const uint32_t nb = 64;
  std::vector<uint64_t> counts(nb);
  uint64_t total = 0;
  for (uint32_t b = 0; b < nb; ++b) total += counts[b] = (b * 37u + 11u) % 300u;
  std::vector<uint64_t> recs(total * 2);
  for (size_t i = 0; i < recs.size(); ++i) recs[i] = 0x9E3779B97F4A7C15ull * (i + 1);
  void *d_in = nullptr, *d_out = nullptr;
  CHECK(hy_malloc(&d_in, recs.size() * 8));
  CHECK(hy_malloc(&d_out, recs.size() * 8 + 64));
  CHECK(hy_memcpy_htod(d_in, recs.data(), recs.size() * 8, nullptr));
  std::vector<uint64_t> all(nb), rc(nb);
  CHECK(hy_join_exchange_counts(comm, counts.data(), nb, all.data(), nullptr));
  if (all != counts) return std::printf("FAIL all-gathered counts\n"), 1;
  uint64_t rows = 0;
  if (hy_join_exchange_records(comm, d_in, 16, all.data(), nb, d_out, 3, rc.data(), &rows, nullptr) != HY_ERR_CAPACITY ||
      rows != total)
    return std::printf("FAIL capacity check\n"), 1;
  CHECK(hy_join_exchange_records(comm, d_in, 16, all.data(), nb, d_out, total + 4, rc.data(), &rows, nullptr));
  std::vector<uint64_t> got(recs.size());
  CHECK(hy_memcpy_dtoh(got.data(), d_out, got.size() * 8, nullptr));
  CHECK(hy_stream_synchronize(nullptr));
  if (rows != total || rc != counts || got != recs) return std::printf("FAIL routed records\n"), 1;
  CHECK(hy_free(d_in));
  CHECK(hy_free(d_out));
  CHECK(hy_comm_destroy(comm));
  std::printf("exchange_check ok (%llu records)\n", static_cast<unsigned long long>(total));
  return 0;
}
