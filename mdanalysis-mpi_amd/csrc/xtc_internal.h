// xtc_internal.h -- state shared by the host XTC codec (xtc.cpp) and the
// GPU decoder (xtc_gpu.hip).  Not part of the public ABI.
#pragma once

#include <cstdint>
#include <vector>

struct rmsf_xtc {
  uint64_t serial = 0;          // unique per open (a freed handle's address may be reused)
  int fd = -1;
  int64_t n_atoms = 0;
  std::vector<int64_t> offset;  // byte offset of each frame record (a multiple of 4)
  std::vector<int64_t> size;    // bytes of each frame record
  int64_t max_size = 0;         // largest record
  std::vector<int32_t> step;
  std::vector<float> time;
  std::vector<float> box;       // 9 per frame (nm)
};

// pread until n bytes arrived (false on EOF / error)
bool rmsf_internal_pread_all(int fd, void *dst, size_t n, int64_t off);
