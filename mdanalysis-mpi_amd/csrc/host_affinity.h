// Host threads next to the GPU: the CPUs of the NUMA node the device's PCIe
// root sits on (sysfs), restricted to the CPUs this process may use.  The
// XTC read pool and the stager's gather pool run there: their host copies
// and the DMA that follows share that socket's memory (C5 on a 2-socket EPYC
// host: 36-37k frames/s with the readers on the GPU's node vs 32-33k on the
// other one).
// RMSF_READ_AFFINITY=0 disables it.
#pragma once

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace rmsf_host {

// "0-63,128-191" -> set bits
inline bool parse_cpulist(const char *s, cpu_set_t *out) {
  CPU_ZERO(out);
  bool any = false;
  while (*s) {
    char *e;
    long a = std::strtol(s, &e, 10);
    if (e == s) break;
    long b = a;
    s = e;
    if (*s == '-') {
      b = std::strtol(s + 1, &e, 10);
      s = e;
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) {
      CPU_SET((int)c, out);
      any = true;
    }
    while (*s == ',' || std::isspace((unsigned char)*s)) ++s;
  }
  return any;
}

inline bool read_line(const std::string &path, char *buf, size_t n) {
  FILE *f = std::fopen(path.c_str(), "r");
  if (!f) return false;
  const bool ok = std::fgets(buf, (int)n, f) != nullptr;
  std::fclose(f);
  return ok;
}

// CPUs of the device's NUMA node that this process may run on; false when
// unknown (no sysfs entry, node -1, empty intersection, or disabled).
inline bool device_cpus(int dev, cpu_set_t *out) {
  const char *env = std::getenv("RMSF_READ_AFFINITY");
  if (env && env[0] == '0') return false;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) return false;
  for (char *p = bus; *p; ++p) *p = (char)std::tolower((unsigned char)*p);
  char line[4096];
  if (!read_line(std::string("/sys/bus/pci/devices/") + bus + "/numa_node", line, sizeof(line))) return false;
  const int node = std::atoi(line);
  if (node < 0) return false;
  if (!read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", line, sizeof(line)))
    return false;
  cpu_set_t near, allowed;
  if (!parse_cpulist(line, &near)) return false;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
  CPU_AND(out, &near, &allowed);
  return CPU_COUNT(out) > 0;
}

// Pin the calling thread (best effort).
inline void pin_self(const cpu_set_t &cpus) { (void)pthread_setaffinity_np(pthread_self(), sizeof(cpus), &cpus); }

}  // namespace rmsf_host
