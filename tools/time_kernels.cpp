// Times the library's C2 Welford accumulate, C3 superposition sums and the
// aligned accumulators (Welford, sum) from a
// plain C++ process (no torch), HIP events, 100k atoms x 20k frames -- to
// compare with the same entry points driven from Python (tools/tune_stats.py,
// bench.py).  Not product code.
//   hipcc -O2 -std=c++17 -Iinclude tools/time_kernels.cpp -Lmdanalysis-mpi_amd/lib -lrmsf_hip \
//         -Wl,-rpath,$PWD/mdanalysis-mpi_amd/lib -o tools/time_kernels
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "rmsf_hip.h"

#define OK(x)                                                          \
  do {                                                                 \
    int rc_ = (x);                                                     \
    if (rc_) {                                                         \
      printf("%s failed: %d %s\n", #x, rc_, rmsf_last_error());       \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

int main() {
  const int64_t n = 100000, nf = 20000;
  float *x;
  double *ref, *info, *xf, *mean, *m2;
  void *work, *acc;
  OK(rmsf_malloc((void **)&x, sizeof(float) * 3 * n * nf));
  OK(rmsf_malloc((void **)&ref, sizeof(double) * 3 * n));
  OK(rmsf_malloc((void **)&info, sizeof(double) * RMSF_REFINFO_DOUBLES));
  OK(rmsf_malloc((void **)&xf, sizeof(double) * RMSF_XFORM_DOUBLES * nf));
  OK(rmsf_malloc((void **)&mean, sizeof(double) * 3 * n));
  OK(rmsf_malloc((void **)&m2, sizeof(double) * 3 * n));
  const size_t wb = rmsf_superpose_workspace_bytes(n, nf);
  OK(rmsf_malloc(&work, wb));
  const size_t ab = rmsf_accumulate_balanced_workspace_bytes(n, nf, 0);
  OK(rmsf_malloc(&acc, ab));
  // rigid motion per frame: identity rotation + small shifts (the kernels' cost does not depend on it)
  std::vector<double> motion(12 * nf, 0.0);
  for (int64_t f = 0; f < nf; ++f) {
    motion[12 * f + 0] = motion[12 * f + 4] = motion[12 * f + 8] = 1.0;
    motion[12 * f + 9] = 0.001 * (f % 7);
  }
  double *dm;
  OK(rmsf_malloc((void **)&dm, sizeof(double) * motion.size()));
  OK(rmsf_memcpy_h2d(dm, motion.data(), sizeof(double) * motion.size(), nullptr));
  OK(rmsf_synth_frames(x, 3 * n, n, 0, nf, 0, dm, nullptr));
  OK(rmsf_reference_setup(x, nullptr, n, nullptr, nullptr, ref, info, nullptr));
  OK(rmsf_stream_synchronize(nullptr));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    for (int k = 0; k < 4; ++k) {
      float ms[5];
      for (int i = 0; i < 5; ++i) {
        hipEventRecord(a, nullptr);
        if (k == 0)
          OK(rmsf_superpose(x, 3 * n, nf, n, nullptr, nullptr, ref, info, xf, work, wb, nullptr));
        else if (k == 1)
          OK(rmsf_accumulate_balanced(x, 3 * n, nf, n, nullptr, nullptr, nullptr, RMSF_MODE_WELFORD, 0, acc, ab,
                                      nullptr));
        else  // aligned (C3 / RMSF.py sweep 2, sweep 1): transform records from the superposition above
          OK(rmsf_accumulate_balanced(x, 3 * n, nf, n, nullptr, xf, info, k == 2 ? RMSF_MODE_WELFORD : RMSF_MODE_SUM,
                                      0, acc, ab, nullptr));
        hipEventRecord(b, nullptr);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms[i], a, b);
      }
      std::sort(ms, ms + 5);
      static const char *name[4] = {"rmsf_superpose", "accumulate_balanced", "accumulate_balanced align",
                                     "accumulate_balanced align sum"};
      printf("%-30s median %.3f ms  min %.3f ms\n", name[k], ms[2], ms[0]);
      fflush(stdout);
    }
  }
  return 0;
}
