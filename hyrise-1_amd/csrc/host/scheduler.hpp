// Intra-operator parallelism through the host's scheduler. The reference's operators split their work into JobTasks
// and wait for them in CurrentScheduler::wait_for_tasks (scheduler/current_scheduler.hpp:16-50, scheduler/job_task.hpp;
// JoinHash: join_hash.cpp:139-182); with a NodeQueueScheduler set, the jobs run on its workers, and without one each
// job runs when it is scheduled (abstract_task.cpp: schedule() without a scheduler executes the task). Here an
// integration registers its scheduler once (set_job_scheduler; INTEGRATION.md shows the NodeQueueScheduler adapter),
// and the operators' host-side jobs - JoinHash's output chunk builders - are submitted to it, so that operators
// executing concurrently share its workers instead of each spawning threads. Without a registered scheduler a job runs
// on a thread of its own, joined by wait() (the behaviour before the hook existed).
#pragma once

#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace hyrise {

class JobScheduler {
 public:
  virtual ~JobScheduler() = default;
  // runs `job` on some worker - or right away on the calling thread (a scheduler without workers)
  virtual void schedule(std::function<void()> job) = 0;
  // how many jobs a caller should split its work into
  virtual unsigned concurrency() const = 0;
};

void set_job_scheduler(std::shared_ptr<JobScheduler> scheduler);  // CurrentScheduler::set
std::shared_ptr<JobScheduler> job_scheduler();                    // CurrentScheduler::get (null: none registered)

// Schedulers for tests and simple embeddings: a fixed pool of worker threads fed from one queue (the shape of a
// single-node NodeQueueScheduler), and one that runs every job on the scheduling thread.
std::shared_ptr<JobScheduler> make_pool_scheduler(unsigned workers);
std::shared_ptr<JobScheduler> make_inline_scheduler();

// Jobs submitted together and waited for (CurrentScheduler::wait_for_tasks). A job's exception is rethrown by wait();
// the destructor waits too, so nothing a job references goes away under it.
class JobGroup {
 public:
  JobGroup();
  ~JobGroup();
  JobGroup(const JobGroup&) = delete;
  JobGroup& operator=(const JobGroup&) = delete;

  void schedule(std::function<void()> job);
  void wait();
  // jobs the group's scheduler wants (its concurrency; without one `dflt`)
  unsigned concurrency(unsigned dflt) const;

 private:
  struct Claimable {
    std::atomic<bool> taken{false};
    std::function<void()> run;
  };
  void finish_one(std::exception_ptr e);
  std::shared_ptr<JobScheduler> _scheduler;
  std::vector<std::shared_ptr<Claimable>> _claims;  // jobs handed to _scheduler (wait() runs those not yet taken)
  std::vector<std::thread> _threads;
  std::mutex _m;
  std::condition_variable _cv;
  size_t _pending = 0;
  std::exception_ptr _error;
};

}  // namespace hyrise
