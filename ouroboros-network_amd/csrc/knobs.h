// The library's environment switches, read ONCE (VERDICT r05 item 7,
// ADVICE r05): at the first call that needs one, and again only when the
// embedding process asks for it with ouro_debug_reload_knobs()
// (include/ouro_verify_debug.h; tests and bench.py call it after they change
// the environment).  No per-call path of the library calls getenv: a
// setenv racing a getenv in the embedding process is undefined behaviour,
// and a stray variable must not change the product's kernels between calls
// (tests/test_abi.py::test_no_getenv_on_call_paths greps for it).
//
// Every field is an atomic so a reload racing a call is well defined (the
// call sees either value).  Defaults are the product's; the A/B-only
// switches are documented where they are used (kernels.hip).
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>

namespace ouro_knobs {

struct Knobs {
  // product behaviour (include/ouro_verify.h documents each)
  std::atomic<int> on_device_error_fail{0};  // OURO_ON_DEVICE_ERROR=fail
  std::atomic<int> single_on_gpu{0};         // OURO_SINGLE_ITEM=gpu
  std::atomic<size_t> wide_small_max{2048};  // OURO_WIDE_SMALL_MAX
  std::atomic<long long> host_chunk{-1};     // OURO_HOST_CHUNK (-1: one resident grid)
  std::atomic<int> host_threads{0};          // OURO_HOST_THREADS (0: the default cap)
  std::atomic<int> host_lanes{0};            // OURO_HOST_IMPL=lanes (A/B, bench single_item)
  // raw CBOR engine (0: the default; range-checked where used)
  std::atomic<size_t> cbor_chunk{0};         // OURO_CBOR_CHUNK
  std::atomic<size_t> cbor_slots{0};         // OURO_CBOR_SLOTS
  std::atomic<size_t> cbor_copy_threads{0};  // OURO_CBOR_COPY_THREADS
  std::atomic<int> cbor_ramp{0};             // OURO_CBOR_RAMP (A/B, rejected)
  // latency mode (A/B forms, bit-exact; read when a plan / launch shape is made)
  std::atomic<int> lat_block{0};             // OURO_LAT_BLOCK (0: kLatBlock)
  std::atomic<int> lat_quad{1};              // OURO_LAT_QUAD
  std::atomic<int> lat_wide{0xff};           // OURO_LAT_WIDE
  std::atomic<int> lat_fuse{1};              // OURO_LAT_FUSE
  std::atomic<int> lat_stamps{0};            // OURO_LAT_STAMPS (a -DOURO_LAT_STAMPS build only)
  // plans (read at ouro_tpraos_plan_create)
  std::atomic<int> plan_stage{2};            // OURO_PLAN_STAGE
  std::atomic<int> plan_spin{0};             // OURO_PLAN_SPIN
  std::atomic<int> plan_graph{0};            // OURO_PLAN_GRAPH
  std::atomic<int> plan_trim{1};             // OURO_PLAN_TRIM
  std::atomic<int> plan_flag{1};             // OURO_PLAN_FLAG
  std::atomic<int> plan_launcher{1};         // OURO_PLAN_LAUNCHER (0: launches on the caller)
  std::atomic<int> plan_timing{0};           // OURO_PLAN_TIMING (timing probe)
  // honoured by the test-hook build only (-DOURO_TEST_HOOKS=1)
  std::atomic<int> split{0};                 // OURO_SPLIT (the split kernels, rejected)
  std::atomic<int> lat_skip{0};              // OURO_LAT_SKIP (timing probe: wrong verdicts)
  std::atomic<int> test_device_error{0};     // OURO_TEST_DEVICE_ERROR
  std::atomic<int> test_plan_poison{0};      // OURO_TEST_PLAN_POISON
  std::atomic<int> test_plan_sentinel{0};    // OURO_TEST_PLAN_SENTINEL
};

// the switches, loaded from the environment on first use
const Knobs& get();
// re-read the environment (ouro_debug_reload_knobs)
void reload();

}  // namespace ouro_knobs
