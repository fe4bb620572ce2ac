// Host-side concurrency checks of the operator layer's shared objects, built with -fsanitize=thread (Makefile target
// host_concurrency_check_tsan) and run by tests/test_host_concurrency.py on the CPU: no GPU is involved, so the races
// a GPU run can only show as a fault are exercised under ThreadSanitizer here.
//   1. a deferred table whose producer throws stays pending: every accessor sees the error, a later producer runs
//      (storage.cpp Table::resolve_slow);
//   2. many threads reading one deferred table: the producer runs once and every reader sees its chunks;
//   3. a consumer that took the producer fulfils the table while readers wait for it (the fused TableScan), and a
//      consumer that gives the producer back (JoinHash's Untake) lets a waiting reader produce it;
//   4. operators that wait for their own jobs while running as jobs of a pool with fewer workers than waiters
//      (JobGroup::wait runs unclaimed jobs itself; before, every worker blocked and the process hung);
//   5. a job's exception reaches wait(); tables of >= 1024 chunks dropped on several threads (the ChunkReaper).
// Prints "host_concurrency_check ok" and exits 0, or names the failed check and exits 1.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <future>
#include <stdexcept>
#include <thread>
#include <vector>

#include "scheduler.hpp"
#include "storage.hpp"

using namespace hyrise;

// (device.cpp defines it for the product library; this check links storage.cpp and scheduler.cpp alone)
unsigned hyrise::host_cpu_share() { return 4; }

namespace {

int g_failures = 0;
#define CHECK(cond, what)                                   \
  do {                                                      \
    if (!(cond)) {                                          \
      std::fprintf(stderr, "FAILED: %s (%s)\n", what, #cond); \
      ++g_failures;                                         \
    }                                                       \
  } while (0)

std::vector<std::shared_ptr<Chunk>> make_chunks(size_t n) {
  std::vector<std::shared_ptr<Chunk>> v;
  for (size_t i = 0; i < n; ++i) v.push_back(std::make_shared<Chunk>(ChunkColumns{make_value_column(DataType::Int, false)}));
  return v;
}

std::shared_ptr<Table> empty_table() {
  return std::make_shared<Table>(TableColumnDefinitions{TableColumnDefinition("a", DataType::Int)}, TableType::Data);
}

struct Throwing final : Table::Producer {
  std::atomic<int> calls{0};
  std::vector<std::shared_ptr<Chunk>> produce() override {
    ++calls;
    throw std::logic_error("scan failed");
  }
};

struct Slow final : Table::Producer {
  std::atomic<int> calls{0};
  size_t n;
  explicit Slow(size_t chunks) : n(chunks) {}
  std::vector<std::shared_ptr<Chunk>> produce() override {
    ++calls;
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    return make_chunks(n);
  }
};

void throwing_producer_stays_pending() {
  auto t = empty_table();
  auto bad = std::make_shared<Throwing>();
  t->set_pending(bad);
  for (int i = 0; i < 2; ++i) {
    bool threw = false;
    try {
      (void)t->chunk_count();
    } catch (const std::logic_error&) {
      threw = true;
    }
    CHECK(threw, "a failing producer's error reaches every accessor");
  }
  CHECK(bad->calls == 2, "the failed producer stays pending and runs again on the next access");
  t->set_pending(std::make_shared<Slow>(3));
  CHECK(t->chunk_count() == 3, "a later producer resolves the table");
}

void concurrent_readers_produce_once() {
  for (int round = 0; round < 20; ++round) {
    auto t = empty_table();
    auto p = std::make_shared<Slow>(4);
    t->set_pending(p);
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int i = 0; i < 8; ++i)
      th.emplace_back([&] {
        if (t->chunk_count() != 4 || t->get_chunk(3) == nullptr) ++bad;
      });
    for (auto& x : th) x.join();
    CHECK(bad == 0, "every concurrent reader sees the produced chunks");
    CHECK(p->calls == 1, "the producer runs once");
  }
}

void taken_producer_fulfilled_while_readers_wait() {
  for (int round = 0; round < 20; ++round) {
    auto t = empty_table();
    auto p = std::make_shared<Slow>(2);
    t->set_pending(p);
    auto taken = t->take_pending();
    CHECK(taken == p, "take_pending hands out the producer");
    CHECK(t->take_pending() == nullptr, "the producer is taken once");
    std::atomic<int> bad{0};
    std::vector<std::thread> readers;
    for (int i = 0; i < 6; ++i)
      readers.emplace_back([&] {
        if (t->chunk_count() != 5) ++bad;
      });
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    t->fulfil(make_chunks(5));
    for (auto& x : readers) x.join();
    CHECK(bad == 0, "readers waiting on a taken producer see the consumer's chunks");
    CHECK(p->calls == 0, "a taken producer is not run by the readers");
  }
  // a consumer that fails gives the producer back: a waiting reader produces the table itself
  auto t = empty_table();
  auto p = std::make_shared<Slow>(3);
  t->set_pending(p);
  auto taken = t->take_pending();
  std::atomic<uint32_t> seen{0};
  std::thread reader([&] { seen = t->chunk_count(); });
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  t->set_pending(taken);
  reader.join();
  CHECK(seen == 3 && p->calls == 1, "an untaken producer is run by the waiting reader");
}

void nested_job_waits_do_not_deadlock() {
  set_job_scheduler(make_pool_scheduler(2));
  std::atomic<int> inner_runs{0};
  auto body = [&] {
    JobGroup outer;
    for (int i = 0; i < 6; ++i)
      outer.schedule([&] {  // an "operator" running on a worker, waiting for its own jobs
        JobGroup inner;
        for (int k = 0; k < 4; ++k) inner.schedule([&] { ++inner_runs; });
        inner.wait();
      });
    outer.wait();
  };
  auto f = std::async(std::launch::async, body);
  if (f.wait_for(std::chrono::seconds(60)) != std::future_status::ready) {
    std::fprintf(stderr, "FAILED: nested JobGroup waits deadlocked on a 2-worker pool\n");
    std::fflush(stderr);
    std::_Exit(1);  // (the hung workers cannot be joined)
  }
  f.get();
  CHECK(inner_runs == 24, "every inner job ran exactly once");
  // a job's exception reaches wait()
  {
    JobGroup g;
    g.schedule([] { throw std::runtime_error("job failed"); });
    g.schedule([] {});
    bool threw = false;
    try {
      g.wait();
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw, "a job's exception is rethrown by wait()");
  }
  set_job_scheduler(nullptr);
}

void large_tables_dropped_concurrently() {
  std::vector<std::thread> th;
  for (int i = 0; i < 4; ++i)
    th.emplace_back([] {
      for (int r = 0; r < 3; ++r) {
        auto t = empty_table();
        t->append_chunks(make_chunks(1500));  // >= 1024 chunks: released by the background reaper
      }
    });
  for (auto& x : th) x.join();
  release_drain();
}

}  // namespace

int main() {
  throwing_producer_stays_pending();
  concurrent_readers_produce_once();
  taken_producer_fulfilled_while_readers_wait();
  nested_job_waits_do_not_deadlock();
  large_tables_dropped_concurrently();
  if (g_failures) {
    std::printf("host_concurrency_check: %d failure(s)\n", g_failures);
    return 1;
  }
  std::printf("host_concurrency_check ok\n");
  return 0;
}
