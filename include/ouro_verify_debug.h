/*
 * ouro_verify_debug.h -- diagnostics and timing probes of libouro_verify.so.
 *
 * NOT part of the drop-in boundary (include/ouro_verify.h): nothing the
 * reference binds is here.  bench.py, tools/ and tests/ use these to read
 * counters, per-phase timings and the placement of the library's threads; a
 * node never needs them.  Every call is host-only and verifies nothing.
 */
#ifndef OURO_VERIFY_DEBUG_H
#define OURO_VERIFY_DEBUG_H

#include "ouro_verify.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Items the host path has verified since the process started -- single items
 * routed there, and host-buffer batches recomputed there after a device
 * error. */
int ouro_debug_host_path(unsigned long long *single_items,
                         unsigned long long *recomputed_batches);

/* Re-read the library's environment switches (OURO_SINGLE_ITEM,
 * OURO_ON_DEVICE_ERROR, OURO_WIDE_SMALL_MAX, OURO_HOST_*, OURO_CBOR_*,
 * OURO_LAT_*, OURO_PLAN_*; csrc/knobs.h).  The library reads them once, on
 * first use, and never on a call path: a process that changes one (tests,
 * bench.py A/B passes) calls this afterwards.  Plans keep the values they
 * were created with. */
void ouro_debug_reload_knobs(void);

/* TIMING PROBE (bench.py latency phases) of the plan's last waited-for
 * window, when OURO_PLAN_TIMING was set in the environment when the plan was
 * created (-1 otherwise): gpu_ms = the window's GPU span, from the input copy
 * kernel's start to the last header's end, read from s_memrealtime stamps the
 * kernels write into the plan's pinned done block (no runtime events: events
 * recorded every window made the runtime stall one submit in ~250 for ~125
 * us); the forms without the done word (OURO_PLAN_FLAG=0 / OURO_PLAN_STAGE
 * != 2) time it with events around the launches instead.  copy_us /
 * launch_us = host time of submit's copy into the pinned block and of the
 * launch calls.  Any pointer may be NULL. */
int ouro_debug_plan_timing(ouro_tpraos_plan *plan, float *gpu_ms, float *copy_us,
                           float *launch_us);

/* Per-thread contexts (stream, scratch, staging) are pooled per device; a
 * thread borrows one on its first call and returns it when it exits.
 * created = contexts made so far on `device`, idle = returned ones waiting in
 * the pool. */
int ouro_debug_contexts(int device, size_t *created, size_t *idle);

/* TIMING PROBE (tools/lat_stamps.py): header 0's per-item stamps of the last
 * fused latency launch, 16 items x 24 tags of s_memrealtime (100 MHz), for a
 * library built with -DOURO_LAT_STAMPS=1 and run with OURO_LAT_STAMPS set.
 * Returns the number of stamps written to out, or -1 (the product build). */
int ouro_debug_lat_stamps(unsigned long long *out);

/* CLOCK PROBE (bench.py roofline.frac_clock): the shader clock the header
 * kernel ran at, from per-workgroup s_memtime / s_memrealtime stamps at entry
 * and exit of the last k_tpraos_verify launch (4 values per workgroup, up to
 * max_slots rows), in a library built with -DOURO_CLOCK_STAMPS=1
 * (lib/libouro_verify_clock.so).  Returns the rows written, or -1 (the
 * product build, in which no stamp executes). */
int ouro_debug_clock_stamps(unsigned long long *out, int max_slots);

/* Workers of ouro_tpraos_verify_batch_multi: per worker its device, NUMA node
 * and the CPUs it is bound to (0 = unbound); returns the worker count. */
int ouro_debug_multi_workers(int *devices, int *nodes, int *cpus, int max);

/* (no device) bind the calling thread to a PCI bus id's node as read from
 * OURO_SYSFS_ROOT (default /sys); returns the node, *ncpus the CPUs bound.
 * ouro_debug_thread_cpus: the CPUs the caller may run on. */
int ouro_debug_numa_bind_pci(const char *busid, int *ncpus);
int ouro_debug_thread_cpus(int *cpus, int max);

/* 1 in the test build (lib/libouro_verify_test.so, -DOURO_TEST_HOOKS=1), whose
 * launches honour OURO_TEST_DEVICE_ERROR (every launch then reports a device
 * error) and whose plans honour OURO_TEST_PLAN_POISON; 0 in the product, which
 * reads neither variable. */
int ouro_debug_test_hooks(void);

/* The calling thread's last raw-CBOR call (ouro_tpraos_verify_cbor /
 * ouro_integrity_verify_cbor): out6 = {total ms, ms gathering header bytes
 * into pinned staging, ms waiting for finished chunks, chunks, slots in
 * flight, gather threads}; -1 before the first call. */
int ouro_debug_cbor_stats(double *out6);

#ifdef __cplusplus
}
#endif
#endif /* OURO_VERIFY_DEBUG_H */
