// C entry points of JoinHash (include/hyrise_amd.h): argument checks and the dispatch on the hashed type to the
// per-type translation units (hyrise_amd_join_*.hip, join_host.hpp).
#include <cstdio>
#include <cstring>
#include "join_host.hpp"

#include <memory>
#include <mutex>

using namespace hyc;
using namespace hyj;

namespace {

hy_status prepare(const hy_join_side* build, const hy_join_filter* build_filter, const hy_join_side* probe,
                  const hy_join_filter* probe_filter, const hy_join_params* params, SidePlan& bp, SidePlan& pp) {
  if (!params) return fail(HY_ERR_INVALID_ARGUMENT, "params");
  if (params->radix_bits > 24) return fail(HY_ERR_UNSUPPORTED, "radix_bits > 24");
  if (!(params->mode == HY_JOIN_INNER || params->mode == HY_JOIN_LEFT || params->mode == HY_JOIN_RIGHT ||
        params->mode == HY_JOIN_SEMI || params->mode == HY_JOIN_ANTI))
    return fail(HY_ERR_UNSUPPORTED, "join mode");
  hy_status st = plan_side(build, bp);
  if (st != HY_OK) return st;
  st = plan_side(probe, pp);
  if (st != HY_OK) return st;
  st = plan_filter(build_filter, bp, build->value_type, params->hashed_type);
  if (st != HY_OK) return st;
  st = plan_filter(probe_filter, pp, probe->value_type, params->hashed_type);
  if (st != HY_OK) return st;
  // fuse the dereference when the side is a reference table (one PosList per chunk shared by the join column)
  bp.fuse = (!bp.referenced.empty() && build->fuse_dereference) ? 1 : 0;
  pp.fuse = (!pp.referenced.empty() && probe->fuse_dereference) ? 1 : 0;
  if (!type_bytes(build->value_type) || !type_bytes(probe->value_type) || !type_bytes(params->hashed_type))
    return fail(HY_ERR_UNSUPPORTED, "join column type");
  return HY_OK;
}

size_t join_bytes_any(int32_t hashed, const SidePlan& bp, const SidePlan& pp, uint32_t bits) {
  switch (hashed) {
    case HY_TYPE_INT32:
      return join_bytes_i32(bp, pp, bits);
    case HY_TYPE_INT64:
      return join_bytes_i64(bp, pp, bits);
    case HY_TYPE_FLOAT:
      return join_bytes_f32(bp, pp, bits);
    default:
      return join_bytes_f64(bp, pp, bits);
  }
}

}  // namespace

extern "C" {

hy_status hy_scan_join_hash_workspace_size(const hy_join_side* build, const hy_join_filter* build_filter,
                                           const hy_join_side* probe, const hy_join_filter* probe_filter,
                                           const hy_join_params* params, size_t* bytes) {
  KnobScope knob_scope;
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "bytes");
  SidePlan bp, pp;
  hy_status st = prepare(build, build_filter, probe, probe_filter, params, bp, pp);
  if (st != HY_OK) return st;
  *bytes = join_bytes_any(params->hashed_type, bp, pp, params->radix_bits);
  return HY_OK;
}

hy_status hy_scan_join_hash(const hy_join_side* build, const hy_join_filter* build_filter, const hy_join_side* probe,
                            const hy_join_filter* probe_filter, const hy_join_params* params, hy_row_id* out_build,
                            hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                            uint32_t* partition_counts, hy_join_result* result, void* workspace,
                            size_t workspace_bytes, hy_stream_t stream) {
  KnobScope knob_scope;
  SidePlan bp, pp;
  hy_status st = prepare(build, build_filter, probe, probe_filter, params, bp, pp);
  if (st != HY_OK) return st;
  if (!partition_begin || !partition_counts) return fail(HY_ERR_INVALID_ARGUMENT, "partition arrays");
  if (params->key_hash && params->hashed_type != HY_TYPE_INT32)
    return fail(HY_ERR_INVALID_ARGUMENT, "key_hash needs int32 key ids");
  hipStream_t s = S(stream);
  struct KeyHashScope {  // the kernels' Digit carries it (join_host.hpp)
    explicit KeyHashScope(const uint32_t* k) { g_key_hash = k; }
    ~KeyHashScope() { g_key_hash = nullptr; }
  } key_hash_scope(params->key_hash);
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      return join_i32(bp, pp, build->value_type, probe->value_type, params, out_build, out_probe, out_capacity,
                      partition_begin, partition_counts, result, workspace, workspace_bytes, s);
    case HY_TYPE_INT64:
      return join_i64(bp, pp, build->value_type, probe->value_type, params, out_build, out_probe, out_capacity,
                      partition_begin, partition_counts, result, workspace, workspace_bytes, s);
    case HY_TYPE_FLOAT:
      return join_f32(bp, pp, build->value_type, probe->value_type, params, out_build, out_probe, out_capacity,
                      partition_begin, partition_counts, result, workspace, workspace_bytes, s);
    default:
      return join_f64(bp, pp, build->value_type, probe->value_type, params, out_build, out_probe, out_capacity,
                      partition_begin, partition_counts, result, workspace, workspace_bytes, s);
  }
}

}  // extern "C"

// A prepared fused TableScan -> JoinHash (include/hyrise_amd.h, "Prepared plans"): the validated side plans, the
// params and a workspace of its own, so that the descriptors are staged to HBM once.
struct hy_join_plan_s {
  SidePlan bp, pp;
  hy_join_params params{};
  int32_t build_type = 0, probe_type = 0;
  void* workspace = nullptr;
  size_t workspace_bytes = 0;
  // the captured launch sequence (every kernel and memset of one execution) for the output buffers it was captured
  // with; replayed by later executions with the same buffers
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipStream_t graph_stream = nullptr;
  const void* graph_args[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  uint64_t graph_capacity = 0;
  const uint32_t* misc = nullptr;   // the captured join's flags / total (device)
  const uint64_t* totals = nullptr;
  const uint32_t* direct_overflow = nullptr;  // the captured direct pass's region-overflow flag, or null
  bool no_graph = false;
  JoinKnobs knobs;  // the environment's knobs when the plan was created; every execution runs under them
  ~hy_join_plan_s() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
  }
};

namespace {

hy_status run_plan(hy_join_plan_s* plan, hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,
                   uint64_t* partition_begin, uint32_t* partition_counts, hy_join_result* result, hipStream_t s) {
  const hy_join_params* prm = &plan->params;
  switch (prm->hashed_type) {
    case HY_TYPE_INT32:
      return join_i32(plan->bp, plan->pp, plan->build_type, plan->probe_type, prm, out_build, out_probe, out_capacity,
                      partition_begin, partition_counts, result, plan->workspace, plan->workspace_bytes, s);
    case HY_TYPE_INT64:
      return join_i64(plan->bp, plan->pp, plan->build_type, plan->probe_type, prm, out_build, out_probe, out_capacity,
                      partition_begin, partition_counts, result, plan->workspace, plan->workspace_bytes, s);
    case HY_TYPE_FLOAT:
      return join_f32(plan->bp, plan->pp, plan->build_type, plan->probe_type, prm, out_build, out_probe, out_capacity,
                      partition_begin, partition_counts, result, plan->workspace, plan->workspace_bytes, s);
    default:
      return join_f64(plan->bp, plan->pp, plan->build_type, plan->probe_type, prm, out_build, out_probe, out_capacity,
                      partition_begin, partition_counts, result, plan->workspace, plan->workspace_bytes, s);
  }
}

// After a replay: the join's flags and total, exactly as run_join_partitions reads them after an eager execution.
// *direct_overflow: a direct pass's region overflowed (the output is invalid; the caller reruns on the classic passes).
hy_status finish_replay(const hy_join_plan_s* plan, uint64_t out_capacity, hy_join_result* result, hipStream_t s,
                        bool* direct_overflow) {
  uint32_t flags[4] = {0, 0, 0, 0};
  uint32_t dflag = 0;
  uint64_t total = 0;
  HY_HIP(hipMemcpyAsync(flags, plan->misc, 16, hipMemcpyDeviceToHost, s));
  HY_HIP(hipMemcpyAsync(&total, plan->totals + 1, 8, hipMemcpyDeviceToHost, s));
  if (plan->direct_overflow) HY_HIP(hipMemcpyAsync(&dflag, plan->direct_overflow, 4, hipMemcpyDeviceToHost, s));
  HY_HIP(hipStreamSynchronize(s));
  *direct_overflow = dflag != 0;
  if (dflag) return HY_OK;
  if (flags[1]) return fail(HY_ERR_KERNEL, "join look-back did not complete");
  if (result) {
    result->total_pairs = total;
    result->capacity_required = total;
  }
  if (flags[2] || total > out_capacity) return fail(HY_ERR_CAPACITY, "join output needs " + std::to_string(total) + " pairs");
  return HY_OK;
}

bool graphs_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("HY_PLAN_GRAPH");
    return !e || std::strtol(e, nullptr, 10) != 0;
  }();
  return v;
}

}  // namespace

extern "C" {

hy_status hy_scan_join_plan_create(const hy_join_side* build, const hy_join_filter* build_filter,
                                   const hy_join_side* probe, const hy_join_filter* probe_filter,
                                   const hy_join_params* params, hy_join_plan_t* plan) {
  KnobScope knob_scope;
  if (!plan) return fail(HY_ERR_INVALID_ARGUMENT, "plan");
  *plan = nullptr;
  auto p = std::make_unique<hy_join_plan_s>();
  hy_status st = prepare(build, build_filter, probe, probe_filter, params, p->bp, p->pp);
  if (st != HY_OK) return st;
  if (params->key_hash && params->hashed_type != HY_TYPE_INT32)
    return fail(HY_ERR_INVALID_ARGUMENT, "key_hash needs int32 key ids");
  p->params = *params;
  p->knobs = knobs();
  p->build_type = build->value_type;
  p->probe_type = probe->value_type;
  p->workspace_bytes = join_bytes_any(params->hashed_type, p->bp, p->pp, params->radix_bits);
  HY_HIP(hipMalloc(&p->workspace, std::max<size_t>(p->workspace_bytes, 256)));
  *plan = p.release();
  return HY_OK;
}

hy_status hy_scan_join_plan_execute(hy_join_plan_t plan, hy_row_id* out_build, hy_row_id* out_probe,
                                    uint64_t out_capacity, uint64_t* partition_begin, uint32_t* partition_counts,
                                    hy_join_result* result, hy_stream_t stream) {
  if (!plan) return fail(HY_ERR_INVALID_ARGUMENT, "plan");
  if (!partition_begin || !partition_counts) return fail(HY_ERR_INVALID_ARGUMENT, "partition arrays");
  hipStream_t s = S(stream);
  KnobScope knob_scope(plan->knobs);
  struct KeyHashScope {
    explicit KeyHashScope(const uint32_t* k) { g_key_hash = k; }
    ~KeyHashScope() { g_key_hash = nullptr; }
  } key_hash_scope(plan->params.key_hash);
  const void* args[5] = {out_build, out_probe, partition_begin, partition_counts, plan->workspace};
  bool timing;
  {
    std::lock_guard<std::mutex> lock(g_kt_mutex);
    timing = g_kt_enabled;  // per-kernel event timing needs the eager launches
  }
  const bool same = plan->exec && plan->graph_stream == s && plan->graph_capacity == out_capacity &&
                    std::equal(args, args + 5, plan->graph_args);
  // a direct pass that overflowed a region: the plan keeps the classic passes from now on (its graph is dropped and
  // its descriptors staged again by the eager execution below, whose carve is the classic one)
  auto drop_direct = [&]() {
    plan->knobs.direct = false;
    knob_scope.own.direct = false;
    if (plan->exec) (void)hipGraphExecDestroy(plan->exec);
    if (plan->graph) (void)hipGraphDestroy(plan->graph);
    plan->exec = nullptr;
    plan->graph = nullptr;
    plan->direct_overflow = nullptr;
    plan->bp.device_ready = plan->pp.device_ready = false;
  };
  if (same && !timing) {  // replay the captured launches
    HY_HIP(hipGraphLaunch(plan->exec, s));
    bool ovf = false;
    const hy_status st = finish_replay(plan, out_capacity, result, s, &ovf);
    if (!ovf) return st;
    drop_direct();
  }
  if (plan->bp.device_ready && plan->pp.device_ready && !timing && !plan->no_graph && graphs_enabled() &&
      s != nullptr) {
    // capture one execution (descriptors are already in the plan's workspace: nothing is staged from the host)
    if (plan->exec) (void)hipGraphExecDestroy(plan->exec);
    if (plan->graph) (void)hipGraphDestroy(plan->graph);
    plan->exec = nullptr;
    plan->graph = nullptr;
    hy_status st = HY_OK;
    std::unique_lock<std::recursive_mutex> capture_lock(g_capture_m);  // (no free orders itself after s meanwhile)
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess) {
      capture_state() = CaptureState{true, nullptr, nullptr};
      st = run_plan(plan, out_build, out_probe, out_capacity, partition_begin, partition_counts, result, s);
      const CaptureState cs = capture_state();
      capture_state() = CaptureState{};
      hipGraph_t g = nullptr;
      const hipError_t e = hipStreamEndCapture(s, &g);
      capture_lock.unlock();
      if (std::getenv("HY_DEBUG_RING")) {
        hipStreamCaptureStatus after = hipStreamCaptureStatusNone;
        const hipError_t qe = hipStreamIsCapturing(s, &after);
        std::fprintf(stderr, "hyrise-amd capture: stream %p run_plan %d (%s) end %s graph %p misc %p; after: %s %d\n",
                     static_cast<void*>(s), int(st), st == HY_OK ? "" : g_last_error.c_str(), hipGetErrorString(e),
                     static_cast<void*>(g), static_cast<const void*>(cs.misc), hipGetErrorString(qe), int(after));
      }
      if (st == HY_OK && e == hipSuccess && g && cs.misc &&
          hipGraphInstantiate(&plan->exec, g, nullptr, nullptr, 0) == hipSuccess) {
        plan->graph = g;
        plan->graph_stream = s;
        plan->graph_capacity = out_capacity;
        std::copy(args, args + 5, plan->graph_args);
        plan->misc = cs.misc;
        plan->totals = cs.totals;
        plan->direct_overflow = cs.direct_overflow;
        HY_HIP(hipGraphLaunch(plan->exec, s));
        bool ovf = false;
        const hy_status st2 = finish_replay(plan, out_capacity, result, s, &ovf);
        if (!ovf) return st2;
        drop_direct();
        return run_plan(plan, out_build, out_probe, out_capacity, partition_begin, partition_counts, result, s);
      }
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
    } else {
      (void)hipGetLastError();
    }
    plan->no_graph = true;  // capture is not available here: execute eagerly from now on
  }
  direct_fell_back() = false;
  const hy_status st =
      run_plan(plan, out_build, out_probe, out_capacity, partition_begin, partition_counts, result, s);
  if (direct_fell_back()) plan->knobs.direct = false;  // (the classic carve's descriptors are staged now)
  // from now on the plan's workspace holds both sides' descriptors (the single-pass variant carves the workspace
  // differently and may fall back within a call: it keeps staging every time)
  if ((st == HY_OK || st == HY_ERR_CAPACITY) && !onepass_enabled()) plan->bp.device_ready = plan->pp.device_ready = true;
  return st;
}

hy_status hy_scan_join_plan_rebind(hy_join_plan_t plan, const hy_join_filter* build_filter,
                                   const hy_join_filter* probe_filter) {
  if (!plan) return fail(HY_ERR_INVALID_ARGUMENT, "plan");
  // validate both sides before changing either
  struct Bind {
    uint32_t* offsets;
    uint64_t* begin;
    hy_row_id* rows;
  } bind[2] = {};
  const SidePlan* sides[2] = {&plan->bp, &plan->pp};
  const hy_join_filter* filters[2] = {build_filter, probe_filter};
  for (int i = 0; i < 2; ++i) {
    const SidePlan& p = *sides[i];
    const hy_join_filter* f = filters[i];
    if (!p.filtered) {
      if (f) return fail(HY_ERR_INVALID_ARGUMENT, "rebind: a filter for a side the plan does not filter");
      continue;
    }
    if (!f) return fail(HY_ERR_INVALID_ARGUMENT, "rebind: the plan filters this side");
    if (f->n_chunks < p.chunks.size() || (p.chunks.size() && !f->chunks) || f->value_type != p.filter_type)
      return fail(HY_ERR_INVALID_ARGUMENT, "rebind: the filter differs from the plan's");
    if (p.chunks.size() && std::memcmp(f->chunks, p.filter.data(), sizeof(hy_scan_chunk) * p.chunks.size()) != 0)
      return fail(HY_ERR_INVALID_ARGUMENT, "rebind: the predicate chunks differ from the plan's");
    if (f->out_row_ids && (!f->out_offsets || !f->out_chunk_begin))
      return fail(HY_ERR_INVALID_ARGUMENT, "out_row_ids needs out_offsets and out_chunk_begin");
    // which outputs exist shapes the plan's workspace carve: only the pointers may change
    if ((f->out_offsets != nullptr) != (p.scan_out != nullptr) ||
        (f->out_chunk_begin != nullptr) != (p.scan_chunk_begin != nullptr))
      return fail(HY_ERR_INVALID_ARGUMENT, "rebind: out_offsets / out_chunk_begin must stay set (or unset) as at create");
    bind[i] = Bind{f->out_offsets, f->out_chunk_begin, f->out_row_ids};
  }
  SidePlan* mut[2] = {&plan->bp, &plan->pp};
  bool changed = false;
  for (int i = 0; i < 2; ++i) {
    if (!mut[i]->filtered) continue;
    changed |= mut[i]->scan_out != bind[i].offsets || mut[i]->scan_chunk_begin != bind[i].begin ||
               mut[i]->scan_rows != bind[i].rows;
    mut[i]->scan_out = bind[i].offsets;
    mut[i]->scan_chunk_begin = bind[i].begin;
    mut[i]->scan_rows = bind[i].rows;
  }
  // a rebound plan runs its launches eagerly from now on: a captured graph holds the old pointers, and an operator that
  // rebinds per execution (its outputs are new buffers each time) would capture again on every call - and capture on a
  // stream while other threads' operators launch, allocate and free
  if (changed) {
    if (plan->exec) (void)hipGraphExecDestroy(plan->exec);
    if (plan->graph) (void)hipGraphDestroy(plan->graph);
    plan->exec = nullptr;
    plan->graph = nullptr;
  }
  plan->no_graph = true;
  return HY_OK;
}

hy_status hy_scan_join_plan_destroy(hy_join_plan_t plan) {
  if (!plan) return HY_OK;
  if (plan->workspace) HY_HIP(hipFree(plan->workspace));
  delete plan;
  return HY_OK;
}

hy_status hy_join_hash_workspace_size(const hy_join_side* build, const hy_join_side* probe,
                                      const hy_join_params* params, size_t* bytes) {
  KnobScope knob_scope;
  return hy_scan_join_hash_workspace_size(build, nullptr, probe, nullptr, params, bytes);
}

hy_status hy_join_hash(const hy_join_side* build, const hy_join_side* probe, const hy_join_params* params,
                       hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                       uint32_t* partition_counts, hy_join_result* result, void* workspace, size_t workspace_bytes,
                       hy_stream_t stream) {
  KnobScope knob_scope;
  return hy_scan_join_hash(build, nullptr, probe, nullptr, params, out_build, out_probe, out_capacity,
                           partition_begin, partition_counts, result, workspace, workspace_bytes, stream);
}

hy_status hy_join_exchange_partition_workspace_size(const hy_join_side* side, const hy_join_params* params,
                                                    uint32_t n_ranks, size_t* bytes) {
  KnobScope knob_scope;
  if (!bytes || !params || n_ranks == 0) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  SidePlan p;
  hy_status st = plan_side(side, p);
  if (st != HY_OK) return st;
  const auto w = digit_plan(params->radix_bits, ceil_log2(n_ranks));
  if (w.empty() || (1u << w[0]) < n_ranks) return fail(HY_ERR_UNSUPPORTED, "radix bits too few for the ranks");
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      *bytes = exchange_partition_bytes_i32(p, params->radix_bits, w);
      break;
    case HY_TYPE_INT64:
      *bytes = exchange_partition_bytes_i64(p, params->radix_bits, w);
      break;
    case HY_TYPE_FLOAT:
      *bytes = exchange_partition_bytes_f32(p, params->radix_bits, w);
      break;
    case HY_TYPE_DOUBLE:
      *bytes = exchange_partition_bytes_f64(p, params->radix_bits, w);
      break;
    default:
      return fail(HY_ERR_UNSUPPORTED, "hashed type");
  }
  return HY_OK;
}

hy_status hy_join_exchange_partition(const hy_join_side* side, const hy_join_params* params, int32_t keep_nulls,
                                     uint32_t n_ranks, void* out_records, uint64_t* bucket_counts, void* workspace,
                                     size_t workspace_bytes, hy_stream_t stream) {
  KnobScope knob_scope;
  if (!params || !bucket_counts || n_ranks == 0) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (params->radix_bits > 24) return fail(HY_ERR_UNSUPPORTED, "radix_bits > 24");
  if (params->key_hash) return fail(HY_ERR_UNSUPPORTED, "string join keys in the distributed join");
  SidePlan p;
  hy_status st = plan_side(side, p);
  if (st != HY_OK) return st;
  p.fuse = (!p.referenced.empty() && side->fuse_dereference) ? 1 : 0;
  const auto w = digit_plan(params->radix_bits, ceil_log2(n_ranks));
  if (w.empty() || (1u << w[0]) < n_ranks) return fail(HY_ERR_UNSUPPORTED, "radix bits too few for the ranks");
  if (p.n_rows && !out_records) return fail(HY_ERR_INVALID_ARGUMENT, "out_records");
  hipStream_t s = S(stream);
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      return exchange_partition_i32(p, side->value_type, params, keep_nulls, w, out_records, bucket_counts, workspace,
                                    workspace_bytes, s);
    case HY_TYPE_INT64:
      return exchange_partition_i64(p, side->value_type, params, keep_nulls, w, out_records, bucket_counts, workspace,
                                    workspace_bytes, s);
    case HY_TYPE_FLOAT:
      return exchange_partition_f32(p, side->value_type, params, keep_nulls, w, out_records, bucket_counts, workspace,
                                    workspace_bytes, s);
    case HY_TYPE_DOUBLE:
      return exchange_partition_f64(p, side->value_type, params, keep_nulls, w, out_records, bucket_counts, workspace,
                                    workspace_bytes, s);
  }
  return fail(HY_ERR_UNSUPPORTED, "hashed type");
}

hy_status hy_join_exchange_join_workspace_size(const uint64_t* build_counts, const uint64_t* probe_counts,
                                               uint32_t n_senders, uint32_t n_buckets, const hy_join_params* params,
                                               size_t* bytes) {
  KnobScope knob_scope;
  if (!bytes || !params || !build_counts || !probe_counts || n_senders == 0)
    return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  const uint32_t bits = params->radix_bits;
  const auto w = digit_plan(bits, ceil_log2(n_senders));
  if (w.empty()) return fail(HY_ERR_UNSUPPORTED, "radix_bits 0");
  const uint32_t digits = 1u << (w.size() > 1 ? w[1] : 0);
  const RecvPlan rb = recv_plan(build_counts, n_senders, n_buckets, digits);
  const RecvPlan rp = recv_plan(probe_counts, n_senders, n_buckets, digits);
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      *bytes = exchange_join_bytes_i32(rb, rp, bits, w, n_buckets, n_senders);
      break;
    case HY_TYPE_INT64:
      *bytes = exchange_join_bytes_i64(rb, rp, bits, w, n_buckets, n_senders);
      break;
    case HY_TYPE_FLOAT:
      *bytes = exchange_join_bytes_f32(rb, rp, bits, w, n_buckets, n_senders);
      break;
    case HY_TYPE_DOUBLE:
      *bytes = exchange_join_bytes_f64(rb, rp, bits, w, n_buckets, n_senders);
      break;
    default:
      return fail(HY_ERR_UNSUPPORTED, "hashed type");
  }
  return HY_OK;
}

hy_status hy_join_exchange_join(const void* build_records, const uint64_t* build_counts, const void* probe_records,
                                const uint64_t* probe_counts, uint32_t n_senders, uint32_t first_bucket,
                                uint32_t n_buckets, const hy_join_params* params, hy_row_id* out_build,
                                hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                                uint32_t* partition_counts, hy_join_result* result, void* workspace,
                                size_t workspace_bytes, hy_stream_t stream) {
  KnobScope knob_scope;
  if (!params || !build_counts || !probe_counts || n_senders == 0 || !partition_begin || !partition_counts)
    return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (params->radix_bits > 24) return fail(HY_ERR_UNSUPPORTED, "radix_bits > 24");
  if (!(params->mode == HY_JOIN_INNER || params->mode == HY_JOIN_LEFT || params->mode == HY_JOIN_RIGHT ||
        params->mode == HY_JOIN_SEMI || params->mode == HY_JOIN_ANTI))
    return fail(HY_ERR_UNSUPPORTED, "join mode");
  const uint32_t bits = params->radix_bits;
  const auto w = digit_plan(bits, ceil_log2(n_senders));
  if (w.empty() || first_bucket + n_buckets > (1u << w[0])) return fail(HY_ERR_INVALID_ARGUMENT, "bucket range");
  const uint32_t digits = 1u << (w.size() > 1 ? w[1] : 0);
  const RecvPlan rbp = recv_plan(build_counts, n_senders, n_buckets, digits);
  const RecvPlan rpp = recv_plan(probe_counts, n_senders, n_buckets, digits);
  if (rbp.rows >= 0xFFFFFFFFull || rpp.rows >= 0xFFFFFFFFull)
    return fail(HY_ERR_UNSUPPORTED, "received side exceeds 2^32-1 rows");
  hipStream_t s = S(stream);
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      return exchange_join_i32(build_records, probe_records, rbp, rpp, n_senders, n_buckets, w, params, out_build,
                               out_probe, out_capacity, partition_begin, partition_counts, result, workspace,
                               workspace_bytes, s);
    case HY_TYPE_INT64:
      return exchange_join_i64(build_records, probe_records, rbp, rpp, n_senders, n_buckets, w, params, out_build,
                               out_probe, out_capacity, partition_begin, partition_counts, result, workspace,
                               workspace_bytes, s);
    case HY_TYPE_FLOAT:
      return exchange_join_f32(build_records, probe_records, rbp, rpp, n_senders, n_buckets, w, params, out_build,
                               out_probe, out_capacity, partition_begin, partition_counts, result, workspace,
                               workspace_bytes, s);
    case HY_TYPE_DOUBLE:
      return exchange_join_f64(build_records, probe_records, rbp, rpp, n_senders, n_buckets, w, params, out_build,
                               out_probe, out_capacity, partition_begin, partition_counts, result, workspace,
                               workspace_bytes, s);
  }
  return fail(HY_ERR_UNSUPPORTED, "hashed type");
}

// ---- row-index exchange records {key, uint32 global row} ----
uint32_t hy_join_exchange_row_record_bytes(int32_t hashed_type) {
  return (hashed_type == HY_TYPE_INT32 || hashed_type == HY_TYPE_FLOAT) ? 8u : 16u;
}

namespace {

hy_status plan_row_side(const hy_join_side* side, const hy_join_filter* filter, const hy_join_params* params,
                        uint32_t n_ranks, uint64_t row_base, SidePlan& p, std::vector<uint32_t>& w) {
  if (!params || n_ranks == 0) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if (params->radix_bits > 24) return fail(HY_ERR_UNSUPPORTED, "radix_bits > 24");
  hy_status st = plan_side(side, p);
  if (st != HY_OK) return st;
  // A reference side (a PosList per chunk, e.g. an earlier join's output) takes part with its rows dereferenced
  // (write_output_columns, join_hash.cpp:584-592): the payload is then the row of the referenced data table.
  const bool ref = !p.referenced.empty();
  if (ref && !side->fuse_dereference)
    return fail(HY_ERR_UNSUPPORTED, "row-index exchange records of a reference side need fuse_dereference");
  if (ref && filter) return fail(HY_ERR_UNSUPPORTED, "a fused scan needs a data-table side");
  p.fuse = ref ? 1 : 0;
  st = plan_filter(filter, p, side->value_type, params->hashed_type);
  if (st != HY_OK) return st;
  if (p.scan_rows)
    return fail(HY_ERR_UNSUPPORTED, "out_row_ids on an exchange side (expand out_offsets: hy_expand_chunk_row_ids)");
  const uint64_t rows = ref ? p.ref_row_begin.back() : p.n_rows;
  if (rows + row_base >= (p.filtered ? 0x7FFFFFFFull : 0xFFFFFFFFull))
    return fail(HY_ERR_UNSUPPORTED, "global row indexes exceed the 32-bit record payload");
  if (ref) {
    for (auto& r : p.ref_row_begin) r += row_base;  // payload = global row of the referenced table
  } else {
    for (auto& c : p.chunks) c.row_begin += row_base;  // payload = global row index
  }
  w = digit_plan(params->radix_bits, ceil_log2(n_ranks));
  if (w.empty() || (1u << w[0]) < n_ranks) return fail(HY_ERR_UNSUPPORTED, "radix bits too few for the ranks");
  return HY_OK;
}

}  // namespace

hy_status hy_scan_join_exchange_partition_workspace_size(const hy_join_side* side, const hy_join_filter* filter,
                                                         const hy_join_params* params, uint32_t n_ranks,
                                                         size_t* bytes) {
  KnobScope knob_scope;
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "bytes");
  SidePlan p;
  std::vector<uint32_t> w;
  hy_status st = plan_row_side(side, filter, params, n_ranks, 0, p, w);
  if (st != HY_OK) return st;
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      *bytes = exchange_partition_rows_bytes_i32(p, params->radix_bits, w);
      return HY_OK;
    case HY_TYPE_INT64:
      *bytes = exchange_partition_rows_bytes_i64(p, params->radix_bits, w);
      return HY_OK;
    case HY_TYPE_FLOAT:
      *bytes = exchange_partition_rows_bytes_f32(p, params->radix_bits, w);
      return HY_OK;
    case HY_TYPE_DOUBLE:
      *bytes = exchange_partition_rows_bytes_f64(p, params->radix_bits, w);
      return HY_OK;
  }
  return fail(HY_ERR_UNSUPPORTED, "hashed type");
}

hy_status hy_scan_join_exchange_partition(const hy_join_side* side, const hy_join_filter* filter,
                                          const hy_join_params* params, int32_t keep_nulls, uint32_t n_ranks,
                                          uint64_t row_base, void* out_records, uint64_t* bucket_counts,
                                          void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  KnobScope knob_scope;
  if (!bucket_counts) return fail(HY_ERR_INVALID_ARGUMENT, "bucket_counts");
  if (params && params->key_hash) return fail(HY_ERR_UNSUPPORTED, "string join keys in the distributed join");
  SidePlan p;
  std::vector<uint32_t> w;
  hy_status st = plan_row_side(side, filter, params, n_ranks, row_base, p, w);
  if (st != HY_OK) return st;
  if (p.n_rows && !out_records) return fail(HY_ERR_INVALID_ARGUMENT, "out_records");
  hipStream_t s = S(stream);
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      return exchange_partition_rows_i32(p, side->value_type, params, keep_nulls, w, out_records, bucket_counts,
                                         workspace, workspace_bytes, s);
    case HY_TYPE_INT64:
      return exchange_partition_rows_i64(p, side->value_type, params, keep_nulls, w, out_records, bucket_counts,
                                         workspace, workspace_bytes, s);
    case HY_TYPE_FLOAT:
      return exchange_partition_rows_f32(p, side->value_type, params, keep_nulls, w, out_records, bucket_counts,
                                         workspace, workspace_bytes, s);
    case HY_TYPE_DOUBLE:
      return exchange_partition_rows_f64(p, side->value_type, params, keep_nulls, w, out_records, bucket_counts,
                                         workspace, workspace_bytes, s);
  }
  return fail(HY_ERR_UNSUPPORTED, "hashed type");
}

namespace {

hy_status plan_row_join(const uint64_t* build_counts, const uint64_t* probe_counts, uint32_t n_senders,
                        uint32_t first_bucket, uint32_t n_buckets, const hy_join_params* params,
                        const uint32_t* build_chunk_sizes, uint32_t n_build_chunks, const uint32_t* probe_chunk_sizes,
                        uint32_t n_probe_chunks, RecvPlan& rbp, RecvPlan& rpp, std::vector<uint32_t>& w, Layouts& lay) {
  if (!params || !build_counts || !probe_counts || n_senders == 0) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  if ((n_build_chunks && !build_chunk_sizes) || (n_probe_chunks && !probe_chunk_sizes))
    return fail(HY_ERR_INVALID_ARGUMENT, "chunk layouts");
  if (params->radix_bits > 24) return fail(HY_ERR_UNSUPPORTED, "radix_bits > 24");
  if (!(params->mode == HY_JOIN_INNER || params->mode == HY_JOIN_LEFT || params->mode == HY_JOIN_RIGHT ||
        params->mode == HY_JOIN_SEMI || params->mode == HY_JOIN_ANTI))
    return fail(HY_ERR_UNSUPPORTED, "join mode");
  w = digit_plan(params->radix_bits, ceil_log2(n_senders));
  if (w.empty() || first_bucket + n_buckets > (1u << w[0])) return fail(HY_ERR_INVALID_ARGUMENT, "bucket range");
  const uint32_t digits = 1u << (w.size() > 1 ? w[1] : 0);
  rbp = recv_plan(build_counts, n_senders, n_buckets, digits);
  rpp = recv_plan(probe_counts, n_senders, n_buckets, digits);
  if (rbp.rows >= 0xFFFFFFFFull || rpp.rows >= 0xFFFFFFFFull)
    return fail(HY_ERR_UNSUPPORTED, "received side exceeds 2^32-1 rows");
  lay.build_rows = layout_rows(build_chunk_sizes, n_build_chunks);
  lay.probe_rows = layout_rows(probe_chunk_sizes, n_probe_chunks);
  return HY_OK;
}

}  // namespace

hy_status hy_join_exchange_join_rows_workspace_size(const uint64_t* build_counts, const uint64_t* probe_counts,
                                                    uint32_t n_senders, uint32_t n_buckets,
                                                    const hy_join_params* params, const uint32_t* build_chunk_sizes,
                                                    uint32_t n_build_chunks, const uint32_t* probe_chunk_sizes,
                                                    uint32_t n_probe_chunks, size_t* bytes) {
  KnobScope knob_scope;
  if (!bytes) return fail(HY_ERR_INVALID_ARGUMENT, "bytes");
  RecvPlan rb, rp;
  std::vector<uint32_t> w;
  Layouts lay;
  hy_status st = plan_row_join(build_counts, probe_counts, n_senders, 0, n_buckets, params, build_chunk_sizes,
                               n_build_chunks, probe_chunk_sizes, n_probe_chunks, rb, rp, w, lay);
  if (st != HY_OK) return st;
  const uint32_t bits = params->radix_bits;
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      *bytes = exchange_join_rows_bytes_i32(rb, rp, bits, w, n_buckets, n_senders, lay);
      return HY_OK;
    case HY_TYPE_INT64:
      *bytes = exchange_join_rows_bytes_i64(rb, rp, bits, w, n_buckets, n_senders, lay);
      return HY_OK;
    case HY_TYPE_FLOAT:
      *bytes = exchange_join_rows_bytes_f32(rb, rp, bits, w, n_buckets, n_senders, lay);
      return HY_OK;
    case HY_TYPE_DOUBLE:
      *bytes = exchange_join_rows_bytes_f64(rb, rp, bits, w, n_buckets, n_senders, lay);
      return HY_OK;
  }
  return fail(HY_ERR_UNSUPPORTED, "hashed type");
}

hy_status hy_join_exchange_join_rows(const void* build_records, const uint64_t* build_counts,
                                     const void* probe_records, const uint64_t* probe_counts, uint32_t n_senders,
                                     uint32_t first_bucket, uint32_t n_buckets, const hy_join_params* params,
                                     const uint32_t* build_chunk_sizes, uint32_t n_build_chunks,
                                     const uint32_t* probe_chunk_sizes, uint32_t n_probe_chunks,
                                     hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,
                                     uint64_t* partition_begin, uint32_t* partition_counts, hy_join_result* result,
                                     void* workspace, size_t workspace_bytes, hy_stream_t stream) {
  KnobScope knob_scope;
  if (!partition_begin || !partition_counts) return fail(HY_ERR_INVALID_ARGUMENT, "partition arrays");
  RecvPlan rb, rp;
  std::vector<uint32_t> w;
  Layouts lay;
  hy_status st = plan_row_join(build_counts, probe_counts, n_senders, first_bucket, n_buckets, params,
                               build_chunk_sizes, n_build_chunks, probe_chunk_sizes, n_probe_chunks, rb, rp, w, lay);
  if (st != HY_OK) return st;
  hipStream_t s = S(stream);
  switch (params->hashed_type) {
    case HY_TYPE_INT32:
      return exchange_join_rows_i32(build_records, probe_records, rb, rp, n_senders, n_buckets, w, params, out_build,
                                    out_probe, out_capacity, partition_begin, partition_counts, result, workspace,
                                    workspace_bytes, s, lay);
    case HY_TYPE_INT64:
      return exchange_join_rows_i64(build_records, probe_records, rb, rp, n_senders, n_buckets, w, params, out_build,
                                    out_probe, out_capacity, partition_begin, partition_counts, result, workspace,
                                    workspace_bytes, s, lay);
    case HY_TYPE_FLOAT:
      return exchange_join_rows_f32(build_records, probe_records, rb, rp, n_senders, n_buckets, w, params, out_build,
                                    out_probe, out_capacity, partition_begin, partition_counts, result, workspace,
                                    workspace_bytes, s, lay);
    case HY_TYPE_DOUBLE:
      return exchange_join_rows_f64(build_records, probe_records, rb, rp, n_senders, n_buckets, w, params, out_build,
                                    out_probe, out_capacity, partition_begin, partition_counts, result, workspace,
                                    workspace_bytes, s, lay);
  }
  return fail(HY_ERR_UNSUPPORTED, "hashed type");
}

uint32_t hy_join_exchange_bucket_bits(uint32_t radix_bits, uint32_t n_ranks) {
  const auto w = digit_plan(radix_bits, ceil_log2(std::max<uint32_t>(1, n_ranks)));
  return w.empty() ? 0u : w[0];
}

}  // extern "C"

// ---- columns carried with the exchange (include/hyrise_amd.h) ----
namespace {

__global__ void record_row_ids_kernel(const uint32_t* __restrict__ payloads, uint32_t stride_words, uint64_t n,
                                      uint64_t row_base, hyk::RowMap m, hy_row_id* __restrict__ out) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t p = payloads[i * stride_words];
    out[i] = p == hyk::NULL_PAYLOAD ? hy_row_id{0xFFFFFFFFu, 0xFFFFFFFFu}
                                    : hyk::map_row(m, static_cast<uint32_t>(p - row_base));
  }
}

template <typename K>
__global__ void localize_kernel(char* __restrict__ records, uint32_t record_bytes, uint64_t n, K* __restrict__ keys,
                                uint32_t* __restrict__ old_payloads) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    char* r = records + i * record_bytes;
    uint32_t* pay = reinterpret_cast<uint32_t*>(r + record_bytes / 2);
    if (keys) keys[i] = *reinterpret_cast<const K*>(r);
    if (old_payloads) old_payloads[i] = *pay;
    *pay = static_cast<uint32_t>(i);
  }
}

}  // namespace

extern "C" {

hy_status hy_exchange_record_row_ids(const void* records, uint64_t n, uint32_t record_bytes, uint64_t row_base,
                                     const uint32_t* chunk_sizes, uint32_t n_chunks, hy_row_id* out_row_ids,
                                     hy_stream_t stream) {
  if (record_bytes != 8 && record_bytes != 16) return fail(HY_ERR_INVALID_ARGUMENT, "record_bytes");
  if (n == 0) return HY_OK;
  if (!records || !out_row_ids || !chunk_sizes || n_chunks == 0) return fail(HY_ERR_INVALID_ARGUMENT, "null argument");
  hipStream_t s = S(stream);
  const std::vector<uint64_t> rb = layout_rows(chunk_sizes, n_chunks);
  if (rb.back() >= 0xFFFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "table exceeds 2^32-1 rows");
  // the chunk prefix lives on the device for the non-uniform case; a small allocation per call
  void* d_rb = nullptr;
  HY_HIP(hipMallocAsync(&d_rb, 8 * rb.size(), s));
  HY_STAGE(d_rb, rb.data(), 8 * rb.size(), s);
  const hyk::RowMap m = make_map(static_cast<const uint64_t*>(d_rb), rb);
  const auto* pay = reinterpret_cast<const uint32_t*>(static_cast<const char*>(records) + record_bytes / 2);
  hipLaunchKernelGGL(record_row_ids_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, pay, record_bytes / 4, n, row_base,
                     m, out_row_ids);
  HY_HIP(hipGetLastError());
  HY_HIP(hipFreeAsync(d_rb, s));
  return HY_OK;
}

hy_status hy_exchange_records_localize(void* records, uint64_t n, uint32_t record_bytes, void* keys,
                                       uint32_t* old_payloads, hy_stream_t stream) {
  if (record_bytes != 8 && record_bytes != 16) return fail(HY_ERR_INVALID_ARGUMENT, "record_bytes");
  if (n == 0) return HY_OK;
  if (!records) return fail(HY_ERR_INVALID_ARGUMENT, "records");
  if (n >= 0xFFFFFFFFull) return fail(HY_ERR_UNSUPPORTED, "more than 2^32-1 records");
  hipStream_t s = S(stream);
  auto* r = static_cast<char*>(records);
  if (record_bytes == 8)
    hipLaunchKernelGGL(localize_kernel<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0, s, r, 8u, n,
                       static_cast<uint32_t*>(keys), old_payloads);
  else
    hipLaunchKernelGGL(localize_kernel<uint64_t>, dim3(grid_for(n, 256)), dim3(256), 0, s, r, 16u, n,
                       static_cast<uint64_t*>(keys), old_payloads);
  HY_HIP(hipGetLastError());
  return HY_OK;
}

}  // extern "C"
