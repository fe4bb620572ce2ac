// The distributed JoinHash's exchange step inside the product boundary: an RCCL communicator (one process per GPU,
// xGMI point-to-point links) and the two collectives between hy_*_exchange_partition (step 1) and
// hy_join_exchange_join(_rows) (step 2), so that a C++ Hyrise process linking libhyrise_amd.so runs the whole
// distributed join without Python (the reference has no distributed join - it is the
// MI355X-native scale-out of join_hash.cpp's partition -> build/probe split).
//
//   counts  ncclAllGather of every rank's B first-digit bucket counts (B <= 256 uint64 per rank)
//   records one ncclGroupStart/End round of ncclSend / ncclRecv: rank r sends each destination d the contiguous run
//           of its records whose buckets d owns ([d * B / N, (d + 1) * B / N), the plan of include/hyrise_amd.h) and
//           receives, sender after sender, the runs of its own buckets. One message per (sender, destination) pair
//           and side: on xGMI's seven point-to-point links every pair is a direct link, so the all-to-all is one
//           round with no relaying. The rank's own run is a device copy.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "hyrise_amd.h"
#include "capi_common.hpp"

using namespace hyc;

struct hy_comm_s {
  ncclComm_t nccl = nullptr;
  int32_t n_ranks = 0;
  int32_t rank = 0;
  uint64_t* counts = nullptr;  // device scratch: n_ranks * 256 gathered bucket counts
  uint32_t* flag = nullptr;    // device scratch: the exchange's all-reduced abort flag
};

namespace {

hy_status nccl_fail(ncclResult_t r, const char* what) {
  return fail(HY_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}

#define HY_NCCL(call)                                  \
  do {                                                 \
    const ncclResult_t r_ = (call);                    \
    if (r_ != ncclSuccess) return nccl_fail(r_, #call); \
  } while (0)

// An RCCL call inside ncclGroupStart/End. Every argument of the point-to-point calls is validated (collectively, by the
// abort verdict) before the group opens, so a failure here is RCCL's own. Closing the group would launch the part
// already queued while peers wait on the sends and receives never queued, so the communicator is aborted instead: the
// peers' calls then fail rather than wait, and this handle answers every later call with an error.
#define HY_NCCL_IN_GROUP(comm, call)                 \
  do {                                               \
    const ncclResult_t r_ = (call);                  \
    if (r_ != ncclSuccess) {                         \
      (void)ncclCommAbort((comm)->nccl);             \
      (comm)->nccl = nullptr;                        \
      return nccl_fail(r_, #call);                   \
    }                                                \
  } while (0)

hy_status comm_usable(hy_comm_t comm) {
  return comm->nccl ? HY_OK : fail(HY_ERR_DEVICE, "communicator was aborted by an earlier failed exchange");
}

uint32_t owner_begin(uint32_t n_buckets, int32_t d, int32_t n) {
  return static_cast<uint32_t>(uint64_t(d) * n_buckets / uint32_t(n));
}

}  // namespace

extern "C" {

hy_status hy_comm_get_unique_id(hy_comm_id* id) {
  if (!id) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  static_assert(sizeof(ncclUniqueId) == HY_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  HY_NCCL(ncclGetUniqueId(&u));
  std::memcpy(id->bytes, &u, HY_COMM_ID_BYTES);
  return HY_OK;
}

hy_status hy_comm_init(hy_comm_t* comm, int32_t n_ranks, const hy_comm_id* id, int32_t rank) {
  if (!comm || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(HY_ERR_INVALID_ARGUMENT, "comm init");
  auto* c = new hy_comm_s();
  ncclUniqueId u;
  std::memcpy(&u, id->bytes, HY_COMM_ID_BYTES);
  const ncclResult_t r = ncclCommInitRank(&c->nccl, n_ranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  c->n_ranks = n_ranks;
  c->rank = rank;
  if (hipMalloc(&c->counts, sizeof(uint64_t) * 256 * n_ranks) != hipSuccess ||
      hipMalloc(&c->flag, sizeof(uint32_t)) != hipSuccess) {
    if (c->counts) (void)hipFree(c->counts);
    ncclCommDestroy(c->nccl);
    delete c;
    return fail(HY_ERR_DEVICE, "hipMalloc");
  }
  *comm = c;
  return HY_OK;
}

hy_status hy_comm_destroy(hy_comm_t comm) {
  if (!comm) return HY_OK;
  if (comm->counts) (void)hipFree(comm->counts);
  if (comm->flag) (void)hipFree(comm->flag);
  const ncclResult_t r = comm->nccl ? ncclCommDestroy(comm->nccl) : ncclSuccess;
  delete comm;
  return r == ncclSuccess ? HY_OK : nccl_fail(r, "ncclCommDestroy");
}

hy_status hy_join_exchange_counts(hy_comm_t comm, const uint64_t* bucket_counts, uint32_t n_buckets,
                                  uint64_t* all_counts, hy_stream_t stream) {
  if (!comm || !bucket_counts || !all_counts || n_buckets == 0 || n_buckets > 256)
    return fail(HY_ERR_INVALID_ARGUMENT, "exchange counts");
  if (const hy_status st = comm_usable(comm); st != HY_OK) return st;
  hipStream_t s = S(stream);
  uint64_t* mine = comm->counts + uint64_t(comm->rank) * n_buckets;
  HY_HIP(hipMemcpyAsync(mine, bucket_counts, 8ull * n_buckets, hipMemcpyHostToDevice, s));
  HY_NCCL(ncclAllGather(mine, comm->counts, n_buckets, ncclUint64, comm->nccl, s));
  HY_HIP(hipMemcpyAsync(all_counts, comm->counts, 8ull * n_buckets * comm->n_ranks, hipMemcpyDeviceToHost, s));
  HY_HIP(hipStreamSynchronize(s));
  return HY_OK;
}

hy_status hy_join_exchange_records(hy_comm_t comm, const void* records, uint32_t record_bytes,
                                   const uint64_t* all_counts, uint32_t n_buckets, void* recv_records,
                                   uint64_t recv_capacity, uint64_t* recv_counts, uint64_t* recv_rows,
                                   hy_stream_t stream) {
  if (!comm || !all_counts || !recv_counts || !recv_rows || n_buckets == 0 || record_bytes == 0)
    return fail(HY_ERR_INVALID_ARGUMENT, "exchange records");
  if (const hy_status st = comm_usable(comm); st != HY_OK) return st;
  const int32_t n = comm->n_ranks, me = comm->rank;
  if (n_buckets < static_cast<uint32_t>(n)) return fail(HY_ERR_INVALID_ARGUMENT, "fewer buckets than ranks");
  // this rank's runs per destination (its records are grouped by bucket, buckets ascending), and what it receives
  std::vector<uint64_t> send(n, 0), send_off(n + 1, 0), recv(n, 0), recv_off(n + 1, 0);
  for (int32_t d = 0; d < n; ++d) {
    for (uint32_t b = owner_begin(n_buckets, d, n); b < owner_begin(n_buckets, d + 1, n); ++b)
      send[d] += all_counts[uint64_t(me) * n_buckets + b];
    send_off[d + 1] = send_off[d] + send[d];
  }
  const uint32_t lo = owner_begin(n_buckets, me, n), hi = owner_begin(n_buckets, me + 1, n);
  for (int32_t src = 0; src < n; ++src) {
    for (uint32_t b = lo; b < hi; ++b) {
      const uint64_t cnt = all_counts[uint64_t(src) * n_buckets + b];
      recv_counts[uint64_t(src) * (hi - lo) + (b - lo)] = cnt;
      recv[src] += cnt;
    }
    recv_off[src + 1] = recv_off[src] + recv[src];
  }
  *recv_rows = recv_off[n];
  // The abort decision is collective: a rank that returned early here would leave its peers blocked in their sends to
  // it. Every rank contributes its own verdict (1: receive buffer too small, 2: null buffer) and all take the max.
  uint32_t mine = recv_off[n] > recv_capacity ? 1u : 0u;
  if ((recv_off[n] && !recv_records) || (send_off[n] && !records)) mine = 2u;
  hipStream_t s = S(stream);
  uint32_t verdict = 0;
  HY_HIP(hipMemcpyAsync(comm->flag, &mine, 4, hipMemcpyHostToDevice, s));
  HY_NCCL(ncclAllReduce(comm->flag, comm->flag, 1, ncclUint32, ncclMax, comm->nccl, s));
  HY_HIP(hipMemcpyAsync(&verdict, comm->flag, 4, hipMemcpyDeviceToHost, s));
  HY_HIP(hipStreamSynchronize(s));
  if (verdict == 1)
    return fail(HY_ERR_CAPACITY, mine ? "exchange receive buffer too small"
                                      : "exchange receive buffer of another rank too small");
  if (verdict != 0) return fail(HY_ERR_INVALID_ARGUMENT, mine ? "null exchange buffer" : "null exchange buffer on another rank");
  const auto* src = static_cast<const char*>(records);
  auto* dst = static_cast<char*>(recv_records);
  const uint64_t rb = record_bytes;
  if (send[me])
    HY_HIP(hipMemcpyAsync(dst + recv_off[me] * rb, src + send_off[me] * rb, send[me] * rb, hipMemcpyDeviceToDevice, s));
  HY_NCCL(ncclGroupStart());
  for (int32_t k = 1; k < n; ++k) {  // peers in a rotating order, so that every link carries one message per round
    const int32_t to = (me + k) % n, from = (me - k + n) % n;
    if (send[to]) HY_NCCL_IN_GROUP(comm, ncclSend(src + send_off[to] * rb, send[to] * rb, ncclUint8, to, comm->nccl, s));
    if (recv[from])
      HY_NCCL_IN_GROUP(comm, ncclRecv(dst + recv_off[from] * rb, recv[from] * rb, ncclUint8, from, comm->nccl, s));
  }
  const ncclResult_t end = ncclGroupEnd();
  if (end != ncclSuccess) {
    (void)ncclCommAbort(comm->nccl);
    comm->nccl = nullptr;
    return nccl_fail(end, "ncclGroupEnd");
  }
  return HY_OK;
}

}  // extern "C"
