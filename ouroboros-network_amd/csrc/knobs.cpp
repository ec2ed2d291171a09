// The one place the library reads its environment switches (knobs.h).
#include "knobs.h"

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace ouro_knobs {
namespace {

Knobs g_knobs;
std::once_flag g_once;
std::mutex g_reload;

bool str_is(const char* name, const char* v) {
  const char* e = getenv(name);
  return e && strcmp(e, v) == 0;
}
template <class T>
void read_int(std::atomic<T>& f, const char* name, T dflt) {
  const char* e = getenv(name);
  f.store(e ? (T)strtoll(e, nullptr, 0) : dflt, std::memory_order_relaxed);
}
template <class T>
void read_size(std::atomic<T>& f, const char* name, T dflt) {
  const char* e = getenv(name);
  f.store(e ? (T)strtoull(e, nullptr, 10) : dflt, std::memory_order_relaxed);
}

void load(Knobs& k) {
  k.on_device_error_fail.store(str_is("OURO_ON_DEVICE_ERROR", "fail"), std::memory_order_relaxed);
  k.single_on_gpu.store(str_is("OURO_SINGLE_ITEM", "gpu"), std::memory_order_relaxed);
  {
    const char* e = getenv("OURO_WIDE_SMALL_MAX");
    k.wide_small_max.store(e ? (size_t)strtoull(e, nullptr, 0) : 2048, std::memory_order_relaxed);
  }
  read_size<long long>(k.host_chunk, "OURO_HOST_CHUNK", -1);
  read_int(k.host_threads, "OURO_HOST_THREADS", 0);
  k.host_lanes.store(str_is("OURO_HOST_IMPL", "lanes"), std::memory_order_relaxed);
  read_size<size_t>(k.cbor_chunk, "OURO_CBOR_CHUNK", 0);
  read_size<size_t>(k.cbor_slots, "OURO_CBOR_SLOTS", 0);
  read_size<size_t>(k.cbor_copy_threads, "OURO_CBOR_COPY_THREADS", 0);
  read_int(k.cbor_ramp, "OURO_CBOR_RAMP", 0);
  read_int(k.lat_block, "OURO_LAT_BLOCK", 0);
  read_int(k.lat_quad, "OURO_LAT_QUAD", 1);
  read_int(k.lat_wide, "OURO_LAT_WIDE", 0xff);
  read_int(k.lat_fuse, "OURO_LAT_FUSE", 1);
  k.lat_stamps.store(getenv("OURO_LAT_STAMPS") != nullptr, std::memory_order_relaxed);
  read_int(k.plan_stage, "OURO_PLAN_STAGE", 2);
  read_int(k.plan_spin, "OURO_PLAN_SPIN", 0);
  read_int(k.plan_graph, "OURO_PLAN_GRAPH", 0);
  read_int(k.plan_trim, "OURO_PLAN_TRIM", 1);
  read_int(k.plan_flag, "OURO_PLAN_FLAG", 1);
  read_int(k.plan_launcher, "OURO_PLAN_LAUNCHER", 1);
  k.plan_timing.store(getenv("OURO_PLAN_TIMING") != nullptr, std::memory_order_relaxed);
  read_int(k.split, "OURO_SPLIT", 0);
  read_int(k.lat_skip, "OURO_LAT_SKIP", 0);
  k.test_device_error.store(getenv("OURO_TEST_DEVICE_ERROR") != nullptr,
                            std::memory_order_relaxed);
  k.test_plan_poison.store(getenv("OURO_TEST_PLAN_POISON") != nullptr, std::memory_order_relaxed);
  k.test_plan_sentinel.store(getenv("OURO_TEST_PLAN_SENTINEL") != nullptr,
                             std::memory_order_relaxed);
}

}  // namespace

const Knobs& get() {
  std::call_once(g_once, [] { load(g_knobs); });
  return g_knobs;
}

void reload() {
  std::call_once(g_once, [] {});
  std::lock_guard<std::mutex> lk(g_reload);
  load(g_knobs);
}

}  // namespace ouro_knobs
