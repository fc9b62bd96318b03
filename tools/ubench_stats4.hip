// The superposition sums (k_frame_stats, VEC4 path) built for different
// minimum occupancies (amdgpu_waves_per_eu: 1 = the library's 164 VGPRs,
// 3 waves/SIMD; 4 / 5 force fewer registers) and run on balanced grids of
// several workgroup counts, A/B in one process (HIP events, 100k atoms x
// 20k and 2,500 frames); partials compared bitwise against the library
// build.  Not product code.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude tools/ubench_stats4.hip -o tools/ubench_stats4
#include "../mdanalysis-mpi_amd/csrc/rmsf_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

template <int W>
void launch(dim3 g, const float *x, int64_t fs, int64_t nf, int64_t n, const double *ref, StatsPlan pl, double *part) {
  hipLaunchKernelGGL((k_frame_stats<false, false, true, W>), g, dim3(kBlock), 0, 0, x, fs, nf, n, nullptr, nullptr,
                     ref, pl, part);
}

int main() {
  const int64_t n = 100000, nf_max = 20000, fs = 3 * n;
  float *x;
  double *ref, *info;
  CK(hipMalloc(&x, sizeof(float) * fs * nf_max));
  CK(hipMalloc(&ref, sizeof(double) * 3 * n));
  CK(hipMalloc(&info, sizeof(double) * RMSF_REFINFO_DOUBLES));
  if (rmsf_synth_frames(x, fs, n, 0, nf_max, 0, nullptr, nullptr) ||
      rmsf_reference_setup(x, nullptr, n, nullptr, nullptr, ref, info, nullptr)) {
    printf("setup failed: %s\n", rmsf_last_error());
    return 1;
  }
  const size_t pbytes = (size_t)1 << 28;
  double *part, *part0;
  CK(hipMalloc(&part, pbytes));
  CK(hipMalloc(&part0, pbytes));
  std::vector<char> ha(pbytes), hb(pbytes);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep) {
    for (int64_t nf : {20000, 2500}) {
      for (int G : {768, 1024, 1280, 1536, 2048, 3072, 4096}) {
        StatsPlan pl = stats_plan(n, nf);
        pl.G = G;
        const int64_t len = (pl.T + pl.G - 1) / pl.G;
        pl.P = (int)((len + pl.ntiles - 1) / pl.ntiles + 1);
        const size_t used = (size_t)pl.G * pl.P * kStats * kTF * sizeof(double);
        if (used > pbytes) continue;
        CK(hipMemset(part0, 0, used));
        launch<1>(dim3(pl.G), x, fs, nf, n, ref, pl, part0);
        CK(hipMemcpy(ha.data(), part0, used, hipMemcpyDeviceToHost));
        for (int W : {1, 4, 5}) {
          auto go = [&]() {
            if (W == 1) launch<1>(dim3(pl.G), x, fs, nf, n, ref, pl, part);
            else if (W == 4) launch<4>(dim3(pl.G), x, fs, nf, n, ref, pl, part);
            else launch<5>(dim3(pl.G), x, fs, nf, n, ref, pl, part);
          };
          CK(hipMemset(part, 0, used));
          go();
          CK(hipMemcpy(hb.data(), part, used, hipMemcpyDeviceToHost));
          const bool same = std::memcmp(ha.data(), hb.data(), used) == 0;
          for (int i = 0; i < 2; ++i) go();
          CK(hipDeviceSynchronize());
          const int R = nf > 5000 ? 10 : 40;
          std::vector<float> ts;
          for (int i = 0; i < R; ++i) {
            CK(hipEventRecord(e0));
            go();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float a;
            CK(hipEventElapsedTime(&a, e0, e1));
            ts.push_back(a);
          }
          std::sort(ts.begin(), ts.end());
          const float med = ts[ts.size() / 2];
          printf("rep %d frames %6ld G %5d waves_per_eu %d: stats %8.4f ms (%5.0f GB/s)  bitwise %s\n", rep,
                 (long)nf, G, W, med, 12.0 * n * nf / med / 1e6, same ? "equal" : "DIFFERENT");
          fflush(stdout);
        }
      }
    }
  }
  return 0;
}
