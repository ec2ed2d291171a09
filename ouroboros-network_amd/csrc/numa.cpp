// numa.cpp -- NUMA placement of the host side of a GPU's pipeline (SURVEY.md
// §8(e): "each GPU has its own HIP stream and pinned-host staging
// (NUMA-local)").
//
// A device's NUMA node is the `numa_node` file of its PCI function in sysfs
// (the PCI bus id comes from hipDeviceGetPCIBusId in kernels.hip); the node's
// CPUs are its `cpulist`.  Binding a thread = restricting its affinity to
// those CPUs (intersected with what the process may use: a container's
// cpuset is honoured, and an empty intersection leaves the thread alone) and
// setting its memory policy to prefer that node, so the pinned staging it
// allocates afterwards (hipHostMalloc with hipHostMallocNumaUser, which
// follows the calling thread's policy) lands there.  The sysfs root is
// OURO_SYSFS_ROOT (default /sys): tests/test_numa.py mocks it.
//
// Plain host C++: no HIP here.
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ouro_verify.h"

namespace {

std::string sysfs_root() {
  const char* e = getenv("OURO_SYSFS_ROOT");
  return e && *e ? std::string(e) : std::string("/sys");
}

bool read_file(const std::string& path, std::string* out) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096];
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  *out = buf;
  return true;
}

// "0-3,8,10-11\n" -> {0,1,2,3,8,10,11}; false on a malformed list
bool parse_cpulist(const std::string& s, std::vector<int>* cpus) {
  size_t i = 0;
  while (i < s.size()) {
    if (s[i] == ',' || isspace((unsigned char)s[i])) {
      i++;
      continue;
    }
    char* end = nullptr;
    const long a = strtol(s.c_str() + i, &end, 10);
    if (end == s.c_str() + i || a < 0 || a >= CPU_SETSIZE) return false;
    i = (size_t)(end - s.c_str());
    long b = a;
    if (i < s.size() && s[i] == '-') {
      const char* p = s.c_str() + i + 1;
      b = strtol(p, &end, 10);
      if (end == p || b < a || b >= CPU_SETSIZE) return false;
      i = (size_t)(end - s.c_str());
    }
    for (long c = a; c <= b; c++) cpus->push_back((int)c);
  }
  return true;
}

}  // namespace

namespace ouro_numa {

// the NUMA node of a PCI function ("0000:C1:00.0" in any case), -1 if sysfs
// does not say (no file, or the firmware's -1)
int node_of_pci(const char* busid) {
  if (!busid || !*busid) return -1;
  std::string id(busid);
  for (char& c : id) c = (char)tolower((unsigned char)c);
  std::string v;
  if (!read_file(sysfs_root() + "/bus/pci/devices/" + id + "/numa_node", &v)) return -1;
  return atoi(v.c_str());
}

// the CPUs of a node, empty if unknown
std::vector<int> cpus_of_node(int node) {
  std::vector<int> cpus;
  std::string v;
  if (node < 0 ||
      !read_file(sysfs_root() + "/devices/system/node/node" + std::to_string(node) + "/cpulist", &v))
    return cpus;
  if (!parse_cpulist(v, &cpus)) cpus.clear();
  return cpus;
}

// Bind the calling thread to `node`: affinity to the node's CPUs that the
// process may use, memory policy preferring the node.  Returns the number of
// CPUs the thread is bound to, 0 if it was left alone.
int bind_thread(int node) {
  const std::vector<int> cpus = cpus_of_node(node);
  if (cpus.empty()) return 0;
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return 0;
  int k = 0;
  for (int c : cpus)
    if (CPU_ISSET(c, &allowed)) {
      CPU_SET(c, &want);
      k++;
    }
  if (k == 0) return 0;  // the node's CPUs are outside this process's cpuset
  if (sched_setaffinity(0, sizeof(want), &want) != 0) return 0;  // 0 = this thread
  // MPOL_PREFERRED (1) for this thread; best effort (no libnuma in the image)
  unsigned long mask[16] = {0};
  if (node < (int)(sizeof(mask) * 8)) {
    mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
    (void)syscall(SYS_set_mempolicy, 1, mask, sizeof(mask) * 8);
  }
  return k;
}

}  // namespace ouro_numa

extern "C" {

// Diagnostics / the mocked-sysfs test (tests/test_numa.py): bind the calling
// thread to the NUMA node of a PCI function given by its bus id; returns the
// node (-1: unknown, nothing changed) and the CPUs bound in *ncpus.
int ouro_debug_numa_bind_pci(const char* busid, int* ncpus) {
  const int node = ouro_numa::node_of_pci(busid);
  const int k = node >= 0 ? ouro_numa::bind_thread(node) : 0;
  if (ncpus) *ncpus = k;
  return node;
}

// The CPUs the calling thread may run on (ascending), at most max; returns
// the count.
int ouro_debug_thread_cpus(int* cpus, int max) {
  cpu_set_t s;
  if (sched_getaffinity(0, sizeof(s), &s) != 0) return -1;
  int k = 0;
  for (int c = 0; c < CPU_SETSIZE; c++)
    if (CPU_ISSET(c, &s)) {
      if (cpus && k < max) cpus[k] = c;
      k++;
    }
  return k;
}

}  // extern "C"
