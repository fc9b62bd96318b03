// Frame-pitch probe: the library's superposition sums (rmsf_superpose), the
// aligned Welford accumulate and the unaligned Welford stream over the same
// 100k-atom x 20k-frame trajectory laid out with different frame pitches
// (bytes between consecutive frames).  The lanes-over-frames superposition
// kernel reads 64 frames per workgroup at the same column, so the pitch
// decides how those rows spread over HBM channels.  Not product code.
//   hipcc -O2 -std=c++17 -Iinclude tools/stride_probe.cpp -Lmdanalysis-mpi_amd/lib -lrmsf_hip \
//         -Wl,-rpath,$PWD/mdanalysis-mpi_amd/lib -o tools/stride_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rmsf_hip.h"

#define OK(x)                                                    \
  do {                                                           \
    int rc_ = (x);                                               \
    if (rc_) {                                                   \
      printf("%s failed: %d %s\n", #x, rc_, rmsf_last_error()); \
      exit(1);                                                   \
    }                                                            \
  } while (0)

int main(int argc, char **argv) {
  const int64_t n = 100000, nf = 20000;
  std::vector<int64_t> pads = {0, 32, 64, 544, 1024, 32 + 1024};  // extra floats per frame
  if (argc > 1) {
    pads.clear();
    for (int i = 1; i < argc; ++i) pads.push_back(atoll(argv[i]));
  }
  const int64_t maxpad = *std::max_element(pads.begin(), pads.end());
  float *x;
  double *ref, *info, *xf, *mean, *m2;
  void *work, *acc;
  OK(rmsf_malloc((void **)&x, sizeof(float) * (3 * n + maxpad) * nf));
  OK(rmsf_malloc((void **)&ref, sizeof(double) * 3 * n));
  OK(rmsf_malloc((void **)&info, sizeof(double) * RMSF_REFINFO_DOUBLES));
  OK(rmsf_malloc((void **)&xf, sizeof(double) * RMSF_XFORM_DOUBLES * nf));
  OK(rmsf_malloc((void **)&mean, sizeof(double) * 3 * n));
  OK(rmsf_malloc((void **)&m2, sizeof(double) * 3 * n));
  const size_t wb = rmsf_superpose_workspace_bytes(n, nf);
  OK(rmsf_malloc(&work, wb));
  const size_t ab = rmsf_accumulate_balanced_workspace_bytes(n, nf, 0);
  OK(rmsf_malloc(&acc, ab));
  std::vector<double> motion(12 * nf, 0.0);
  for (int64_t f = 0; f < nf; ++f) {
    motion[12 * f + 0] = motion[12 * f + 4] = motion[12 * f + 8] = 1.0;
    motion[12 * f + 9] = 0.001 * (f % 7);
  }
  double *dm;
  OK(rmsf_malloc((void **)&dm, sizeof(double) * motion.size()));
  OK(rmsf_memcpy_h2d(dm, motion.data(), sizeof(double) * motion.size(), nullptr));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto t = [&](auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    float best = 1e9, sum = 0;
    const int R = 5;
    for (int i = 0; i < R; ++i) {
      hipEventRecord(a, nullptr);
      launch();
      hipEventRecord(b, nullptr);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
      sum += ms;
    }
    return std::make_pair(sum / R, best);
  };
  printf("%-10s %-12s %-8s %18s %18s %18s\n", "pad_f32", "pitch_B", "pitch%4K", "superpose ms", "align-welford ms",
         "welford ms");
  for (int rep = 0; rep < 2; ++rep) {
    for (int64_t pad : pads) {
      const int64_t fs = 3 * n + pad;
      OK(rmsf_synth_frames(x, fs, n, 0, nf, 0, dm, nullptr));
      OK(rmsf_reference_setup(x, nullptr, n, nullptr, nullptr, ref, info, nullptr));
      OK(rmsf_stream_synchronize(nullptr));
      auto sp = t([&] { OK(rmsf_superpose(x, fs, nf, n, nullptr, nullptr, ref, info, xf, work, wb, nullptr)); });
      auto aw = t([&] {
        OK(rmsf_accumulate_balanced(x, fs, nf, n, nullptr, xf, info, RMSF_MODE_WELFORD, 0, acc, ab, nullptr));
      });
      auto wf = t([&] {
        OK(rmsf_accumulate_balanced(x, fs, nf, n, nullptr, nullptr, nullptr, RMSF_MODE_WELFORD, 0, acc, ab, nullptr));
      });
      printf("%-10lld %-12lld %-8lld %8.3f (%6.3f) %8.3f (%6.3f) %8.3f (%6.3f)\n", (long long)pad,
             (long long)(4 * fs), (long long)((4 * fs) % 4096), sp.first, sp.second, aw.first, aw.second, wf.first,
             wf.second);
      fflush(stdout);
    }
  }
  return 0;
}
