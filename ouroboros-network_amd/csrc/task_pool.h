// task_pool.h -- the library's one persistent pool of host worker threads.
//
// Every host-side parallel loop of the product goes through it: the host
// path's item loops (host_path.hip), the CBOR slicer (pack.cpp) and the
// gather of raw headers into pinned staging (kernels.hip, the raw-CBOR
// pipeline).  Threads are started once, on first use, and live until the
// process exits, so a batch never pays for thread creation and a call
// behind the C ABI never lets std::system_error or std::bad_alloc escape:
// when no worker can be started (or none is free) the calling thread runs
// the tasks itself, and a task that throws is reported, not propagated.
#pragma once
#include <stddef.h>

#include <functional>

namespace ouro_pool {

// Runs fn(k) for every k in [0, ntasks), on the calling thread plus up to
// width - 1 pool workers (width <= 0: every worker).  Concurrent callers
// share the workers; each call returns once all of ITS tasks have run.
// Returns 0, or -1 if any task threw (the other tasks still ran).
int parallel_for(size_t ntasks, int width, const std::function<void(size_t)>& fn);

// Workers the pool has started so far (0 before the first parallel_for).
int workers();

// The CPUs this process may run on (sched_getaffinity), at least 1.
int usable_cpus();

}  // namespace ouro_pool
