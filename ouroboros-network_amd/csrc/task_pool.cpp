// task_pool.cpp -- see task_pool.h.
//
// A job is the caller's loop over [0, ntasks): an atomic cursor hands out
// task indices to whoever takes part -- the caller itself and any workers
// that pick the job off the queue -- so a job finishes even with no worker at
// all.  The job lives on the caller's stack; the caller unlinks it from the
// queue and waits until no worker still holds it before returning.
#include "task_pool.h"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace ouro_pool {
namespace {

struct Job {
  const std::function<void(size_t)>* fn = nullptr;
  size_t ntasks = 0;
  int helpers = 0;                // workers that may still join (width - 1)
  std::atomic<size_t> next{0};    // next task index to hand out
  int active = 0;                 // workers inside run() (guarded by Pool::mu)
  std::atomic<bool> threw{false};
};

void run(Job* j) {
  for (;;) {
    const size_t k = j->next.fetch_add(1, std::memory_order_relaxed);
    if (k >= j->ntasks) return;
    try {
      (*j->fn)(k);
    } catch (...) {
      j->threw.store(true, std::memory_order_relaxed);
    }
  }
}

struct Pool {
  std::mutex mu;
  std::condition_variable work, idle;
  std::deque<Job*> q;
  int started = 0;
  bool spawn_failed = false;
  int max_workers = 0;

  void loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      work.wait(lk, [&] { return !q.empty(); });
      Job* j = q.front();
      if (j->helpers <= 0 || j->next.load(std::memory_order_relaxed) >= j->ntasks) {
        q.pop_front();  // nothing left to take part in: its owner finishes it
        continue;
      }
      j->helpers--;
      j->active++;
      lk.unlock();
      run(j);
      lk.lock();
      if (--j->active == 0) idle.notify_all();
    }
  }

  // start workers until `want` exist (under mu); a failed start is final
  void grow(int want) {
    want = std::min(want, max_workers);
    while (started < want && !spawn_failed) {
      try {
        std::thread([this] { loop(); }).detach();
        started++;
      } catch (...) {
        spawn_failed = true;
      }
    }
  }
};

Pool& pool() {
  // leaked on purpose: workers block on its condition variables until exit
  static Pool* p = [] {
    Pool* q = new Pool;
    q->max_workers = std::min(64, usable_cpus()) - 1;
    if (const char* e = getenv("OURO_HOST_THREADS")) q->max_workers = std::max(0, atoi(e) - 1);
    return q;
  }();
  return *p;
}

}  // namespace

int usable_cpus() {
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) return std::max(1, CPU_COUNT(&set));
  return 1;
}

int workers() {
  Pool& P = pool();
  std::lock_guard<std::mutex> g(P.mu);
  return P.started;
}

int parallel_for(size_t ntasks, int width, const std::function<void(size_t)>& fn) {
  if (ntasks == 0) return 0;
  Pool& P = pool();
  Job j;
  j.fn = &fn;
  j.ntasks = ntasks;
  const int w = width <= 0 ? P.max_workers + 1 : width;
  j.helpers = (int)std::min<size_t>((size_t)std::max(0, w - 1), ntasks - 1);
  bool queued = false;
  if (j.helpers > 0) {
    std::lock_guard<std::mutex> g(P.mu);
    P.grow(j.helpers);
    if (P.started > 0) {
      try {
        P.q.push_back(&j);
        queued = true;
      } catch (...) {
        // no memory for the queue node: the caller runs it alone
      }
    }
  }
  if (queued) P.work.notify_all();
  run(&j);
  if (queued) {
    std::unique_lock<std::mutex> lk(P.mu);
    auto it = std::find(P.q.begin(), P.q.end(), &j);
    if (it != P.q.end()) P.q.erase(it);
    P.idle.wait(lk, [&] { return j.active == 0; });
  }
  return j.threw.load() ? -1 : 0;
}

}  // namespace ouro_pool
