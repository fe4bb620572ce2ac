// Job submission to the host's scheduler (scheduler.hpp; reference scheduler/current_scheduler.cpp,
// scheduler/node_queue_scheduler.cpp, scheduler/job_task.cpp).
#include "scheduler.hpp"

#include <deque>

namespace hyrise {

namespace {

std::mutex g_scheduler_m;
std::shared_ptr<JobScheduler> g_scheduler;

// One queue, n workers (a single-node NodeQueueScheduler: node_queue_scheduler.cpp:26-60, task_queue.cpp).
class PoolScheduler final : public JobScheduler {
 public:
  explicit PoolScheduler(unsigned workers) : _n(workers ? workers : 1) {
    for (unsigned i = 0; i < _n; ++i) _workers.emplace_back([this] { run(); });
  }
  ~PoolScheduler() override {
    {
      std::lock_guard<std::mutex> lock(_m);
      _stop = true;
    }
    _cv.notify_all();
    for (auto& t : _workers) t.join();
  }
  void schedule(std::function<void()> job) override {
    {
      std::lock_guard<std::mutex> lock(_m);
      _queue.push_back(std::move(job));
    }
    _cv.notify_one();
  }
  unsigned concurrency() const override { return _n; }

 private:
  void run() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lock(_m);
        _cv.wait(lock, [&] { return _stop || !_queue.empty(); });
        if (_queue.empty()) return;  // (stopping, and every queued job has run)
        job = std::move(_queue.front());
        _queue.pop_front();
      }
      job();
    }
  }
  const unsigned _n;
  std::mutex _m;
  std::condition_variable _cv;
  std::deque<std::function<void()>> _queue;
  bool _stop = false;
  std::vector<std::thread> _workers;
};

// No workers: a job runs when it is scheduled (the reference without a scheduler, abstract_task.cpp).
class InlineScheduler final : public JobScheduler {
 public:
  void schedule(std::function<void()> job) override { job(); }
  unsigned concurrency() const override { return 1; }
};

}  // namespace

void set_job_scheduler(std::shared_ptr<JobScheduler> scheduler) {
  std::lock_guard<std::mutex> lock(g_scheduler_m);
  g_scheduler = std::move(scheduler);
}

std::shared_ptr<JobScheduler> job_scheduler() {
  std::lock_guard<std::mutex> lock(g_scheduler_m);
  return g_scheduler;
}

std::shared_ptr<JobScheduler> make_pool_scheduler(unsigned workers) { return std::make_shared<PoolScheduler>(workers); }
std::shared_ptr<JobScheduler> make_inline_scheduler() { return std::make_shared<InlineScheduler>(); }

JobGroup::JobGroup() : _scheduler(job_scheduler()) {}

JobGroup::~JobGroup() {
  try {
    wait();
  } catch (...) {  // (a job's exception is only reported by an explicit wait())
  }
}

unsigned JobGroup::concurrency(unsigned dflt) const { return _scheduler ? _scheduler->concurrency() : dflt; }

void JobGroup::finish_one(std::exception_ptr e) {
  std::lock_guard<std::mutex> lock(_m);
  if (e && !_error) _error = e;
  --_pending;
  _cv.notify_all();
}

void JobGroup::schedule(std::function<void()> job) {
  {
    std::lock_guard<std::mutex> lock(_m);
    ++_pending;
  }
  auto wrapped = [this, job = std::move(job)] {
    std::exception_ptr e;
    try {
      job();
    } catch (...) {
      e = std::current_exception();
    }
    finish_one(e);
  };
  if (_scheduler) {
    // The job runs once, on whichever takes it first: a worker of the scheduler, or wait() on the waiting thread
    // (the worker's queue entry holds only the claim, never `this`).
    auto claim = std::make_shared<Claimable>();
    claim->run = std::move(wrapped);
    _claims.push_back(claim);
    _scheduler->schedule([claim] {
      if (!claim->taken.exchange(true)) claim->run();
    });
  } else {
    _threads.emplace_back(std::move(wrapped));
  }
}

void JobGroup::wait() {
  // Jobs no worker has started yet run here, on the waiting thread (CurrentScheduler::wait_for_tasks lets the waiting
  // worker make progress the same way, worker.cpp _wait_for_tasks): operators that wait for their jobs while running on
  // the scheduler's own workers cannot deadlock when every worker is such a waiter.
  for (auto& claim : _claims)
    if (!claim->taken.exchange(true)) claim->run();
  _claims.clear();
  for (auto& t : _threads)
    if (t.joinable()) t.join();
  _threads.clear();
  std::unique_lock<std::mutex> lock(_m);
  _cv.wait(lock, [&] { return _pending == 0; });
  if (_error) {
    std::exception_ptr e = _error;
    _error = nullptr;
    std::rethrow_exception(e);
  }
}

}  // namespace hyrise
