// The superposition sums (k_frame_stats) + per-frame QCP (k_qcp_frames) at
// the strong-scaling shares (100k atoms x 20k/N frames) for several fixed
// workgroup counts of the balanced stats grid, each kernel timed on its own
// (HIP events).  Not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_stats3.hip -o tools/ubench_stats3
#include "../mdanalysis-mpi_amd/csrc/rmsf_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

int main() {
  const int64_t n = 100000, nf_max = 20000, fs = 3 * n;
  float *x;
  double *ref, *info, *xf;
  CK(hipMalloc(&x, sizeof(float) * fs * nf_max));
  CK(hipMalloc(&ref, sizeof(double) * 3 * n));
  CK(hipMalloc(&info, sizeof(double) * RMSF_REFINFO_DOUBLES));
  CK(hipMalloc(&xf, sizeof(double) * RMSF_XFORM_DOUBLES * nf_max));
  std::vector<double> motion(12 * nf_max, 0.0);
  for (int64_t f = 0; f < nf_max; ++f) {
    const double an = 0.01 * (f % 97);
    motion[12 * f + 0] = std::cos(an), motion[12 * f + 1] = -std::sin(an);
    motion[12 * f + 3] = std::sin(an), motion[12 * f + 4] = std::cos(an);
    motion[12 * f + 8] = 1.0;
    motion[12 * f + 9] = 50.0 + 0.001 * (f % 7), motion[12 * f + 10] = 50.0, motion[12 * f + 11] = 50.0;
  }
  double *dm;
  CK(hipMalloc(&dm, sizeof(double) * motion.size()));
  CK(hipMemcpy(dm, motion.data(), sizeof(double) * motion.size(), hipMemcpyHostToDevice));
  if (rmsf_synth_frames(x, fs, n, 0, nf_max, 0, dm, nullptr) ||
      rmsf_reference_setup(x, nullptr, n, nullptr, nullptr, ref, info, nullptr)) {
    printf("setup failed: %s\n", rmsf_last_error());
    return 1;
  }
  double *part;
  CK(hipMalloc(&part, (size_t)1 << 30));
  hipEvent_t e[3];
  for (auto &ev : e) CK(hipEventCreate(&ev));
  for (int rep = 0; rep < 2; ++rep) {
    for (int64_t nf : {2500, 5000, 20000}) {
      for (int G : {768, 1536, 2304, 3072, 4608}) {
        StatsPlan pl = stats_plan(n, nf);
        pl.G = G;
        const int64_t len = (pl.T + pl.G - 1) / pl.G;
        pl.P = (int)((len + pl.ntiles - 1) / pl.ntiles + 1);
        const unsigned gq = (unsigned)((nf + 3) / 4);
        auto launch = [&](bool timed) {
          if (timed) CK(hipEventRecord(e[0]));
          hipLaunchKernelGGL((k_frame_stats<false, false, true>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs, nf, n,
                             nullptr, nullptr, ref, pl, part);
          if (timed) CK(hipEventRecord(e[1]));
          hipLaunchKernelGGL((k_qcp_frames<false, false>), dim3(gq), dim3(kBlock), 0, 0, part, pl, nf, x, fs, nullptr,
                             info, xf);
          if (timed) CK(hipEventRecord(e[2]));
        };
        for (int i = 0; i < 2; ++i) launch(false);
        CK(hipDeviceSynchronize());
        float s1 = 0, s2 = 0;
        const int R = 10;
        for (int i = 0; i < R; ++i) {
          launch(true);
          CK(hipEventSynchronize(e[2]));
          float a, b;
          CK(hipEventElapsedTime(&a, e[0], e[1]));
          CK(hipEventElapsedTime(&b, e[1], e[2]));
          s1 += a, s2 += b;
        }
        printf("frames %6ld G %5d P %d  stats %8.4f ms (%5.0f GB/s)  qcp %7.4f ms  sum %8.4f\n", (long)nf, G, pl.P,
               s1 / R, 12.0 * n * nf / (s1 / R) / 1e6, s2 / R, (s1 + s2) / R);
        fflush(stdout);
      }
    }
  }
  return 0;
}
