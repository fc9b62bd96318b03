// The float4 Welford stream (k_welford_flat_sk) at the per-GPU shares of the
// strong-scaling bench (100k atoms x 20k/N frames): time per launch against
// frames, and the balanced grid's workgroups per CU at each share.  Finds the
// fixed part of a launch that the 1/N shares expose.  Not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_short.hip -o tools/ubench_short
#include "../mdanalysis-mpi_amd/csrc/rmsf_kernels.hip"

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

int main(int argc, char **argv) {
  // ubench_short [n_atoms [frames...]]: default 100k atoms at 2,500-20,000 frames
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000;
  std::vector<int64_t> frames_list;
  for (int i = 2; i < argc; ++i) frames_list.push_back(atoll(argv[i]));
  if (frames_list.empty()) frames_list = {2500, 5000, 10000, 20000};
  int64_t nf_max = 0;
  for (int64_t f : frames_list) nf_max = std::max(nf_max, f);
  const int64_t fs = 3 * n;
  float *x;
  CK(hipMalloc(&x, sizeof(float) * fs * nf_max));
  if (rmsf_synth_frames(x, fs, n, 0, nf_max, 0, nullptr, nullptr)) return 1;
  const size_t ab = (size_t)1 << 30;
  void *acc;
  CK(hipMalloc(&acc, ab));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // S > 0: chunk-aligned frame ranges, S per chunk, split-major (the plan's
  // many-chunks cut, forced)
  auto plan_s = [&](int64_t nf, int S) {
    SkPlan p = sk_plan(3 * n / 4, 4, nf, 1, RMSF_MODE_WELFORD, 1);
    p.S = S;
    p.G = (int)(p.C * S);
    const int64_t W = (p.T + p.G - 1) / p.G;
    p.P = (int)((W + kCoefN - 1) / kCoefN + (W - 1) / nf + 2);
    if (nf % S == 0) p.P = (int)((nf / S + kCoefN - 1) / kCoefN);
    return p;
  };
  auto launch = [&](int64_t nf, int per_cu, int groups, int S = 0) {
    const SkPlan pl = S > 0 ? plan_s(nf, S) : sk_plan(3 * n / 4, 4, nf, groups, RMSF_MODE_WELFORD, per_cu);
    if (sk_bytes(pl, true) > ab) {  // never launch past the workspace
      printf("skip: G %d needs %zu B of partials (> %zu)\n", pl.G, sk_bytes(pl, true), ab);
      return -1;
    }
    int64_t *hdr = static_cast<int64_t *>(acc);
    double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
    double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 4;
    hipLaunchKernelGGL((k_welford_flat_sk<4>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs / 4, pl, hdr, p0, p1);
    return pl.G;
  };
  for (int rep = 0; rep < 2; ++rep) {
    for (int64_t nf : frames_list) {
      for (int v = 0; v < 12; ++v) {
        static const int kG[] = {512, 768, 1024, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        static const int kS[] = {0, 0, 0, 1, 2, 3, 4, 5, 7, 10, 13, 20};
        const int groups = kG[v], S = kS[v];
        int G = 0;
        for (int i = 0; i < 3; ++i) G = launch(nf, 3, groups, S);
        if (G < 0) continue;
        CK(hipDeviceSynchronize());
        float best = 1e9, sum = 0;
        const int R = 20;
        for (int i = 0; i < R; ++i) {
          CK(hipEventRecord(a));
          launch(nf, 3, groups, S);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          best = std::min(best, ms);
          sum += ms;
        }
        const double bytes = 12.0 * n * nf;
        printf("frames %6ld G %5d S %2d  %8.4f ms (min %8.4f)  %6.0f GB/s  frac %.3f\n", (long)nf, G, S, sum / R,
               best, bytes / (sum / R) / 1e6, bytes / (sum / R) / 1e6 / 8000.0);
      }
    }
  }
  // back-to-back launches (a step loop): the gap between dependent launches
  for (int64_t nf : frames_list) {
    const int K = 20;
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < K; ++i) launch(nf, 3, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("back-to-back x%d frames %ld: %.4f ms per launch\n", K, (long)nf, ms / K);
  }
  return 0;
}
