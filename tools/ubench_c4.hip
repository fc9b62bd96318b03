// The float4 Welford stream at C4's per-GPU share (1M atoms = 12 MB frames x
// 2,500 frames, 30 GB): 0.80 of peak against 0.85 at C2 (100k atoms = 1.2 MB
// frames).  Is it the frame size (page locality of the 4 KB chunk columns) or
// the plan?  Times, in one process: the library launch (chunk-aligned S = 2),
// the same plan with the math removed (pure read of the same pattern), a
// 512-lane variant (two adjacent chunks per workgroup: 8 KB contiguous per
// frame), and the 100k-atom x 25k-frame stream of the same 30 GB.  Not
// product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_c4.hip -o tools/ubench_c4
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

namespace ub {
// the library's segment walk, cw lanes per chunk, blockDim = CW; READ_ONLY:
// the loads without the statistics (sum of the floats, one store per segment)
template <int CW, bool READ_ONLY>
__global__ __launch_bounds__(CW) void stream(const float *__restrict__ xyz, int64_t stride4, SkPlan pl,
                                             double *__restrict__ parts0, double *__restrict__ parts1) {
  const int b = sk_range(pl, blockIdx.x);
  int64_t lo = sk_lo(pl, b);
  const int64_t hi = sk_lo(pl, b + 1);
  int64_t slot = (int64_t)b * pl.P;
  while (lo < hi) {
    int64_t c, f0;
    const int len = (int)sk_seg_len(pl, lo, hi, &c, &f0);
    const int64_t i4 = c * CW + threadIdx.x;
    if (i4 < pl.lanes) {
      const f32x4 *p = reinterpret_cast<const f32x4 *>(xyz) + f0 * stride4 + i4;
      const int64_t o = slot * (CW * 4) + 4 * threadIdx.x;
      if (READ_ONLY) {
        float s = 0.f;
        int k = 0;
        for (; k + 4 <= len; k += 4) {
          f32x4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(p + (int64_t)(k + u) * stride4);
#pragma unroll
          for (int u = 0; u < 4; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
        }
        for (; k < len; ++k) {
          const f32x4 v = __builtin_nontemporal_load(p + (int64_t)k * stride4);
          s += v.x + v.y + v.z + v.w;
        }
        __builtin_nontemporal_store((double)s, parts0 + o);
      } else {
        double m[4], q[4];
        wel_flat_run<4>(p, stride4, len, m, q);
        store4(parts0 + o, parts1 + o, m, q);
      }
    }
    lo += len;
    ++slot;
  }
}
}  // namespace ub

int main() {
  const size_t ab = (size_t)2 << 30;
  void *acc;
  CK(hipMalloc(&acc, ab));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct Case { int64_t n, nf; };
  const Case cases[] = {{1000000, 2500}, {100000, 25000}};
  float *x;
  CK(hipMalloc(&x, sizeof(float) * 3 * (size_t)1000000 * 2500));
  for (int rep = 0; rep < 2; ++rep)
    for (const Case &cs : cases) {
      const int64_t n = cs.n, nf = cs.nf, fs = 3 * n;
      if (rmsf_synth_frames(x, fs, n, 0, nf, 0, nullptr, nullptr)) return 1;
      CK(hipDeviceSynchronize());
      auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 2; ++i) launch();
        CK(hipDeviceSynchronize());
        float best = 1e9, sum = 0;
        const int R = 8;
        for (int i = 0; i < R; ++i) {
          CK(hipEventRecord(a));
          launch();
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          best = std::min(best, ms);
          sum += ms;
        }
        const double bytes = 12.0 * n * nf;
        printf("%7ld atoms x %5ld frames %-44s %7.4f ms (min %7.4f)  frac %.3f\n", (long)n, (long)nf, name, sum / R,
               best, bytes / (sum / R) / 1e6 / 8000.0);
        fflush(stdout);
      };
      int64_t *hdr = static_cast<int64_t *>(acc);
      double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
      run("library rmsf_accumulate_balanced", [&] {
        rmsf_accumulate_balanced(x, fs, nf, n, nullptr, nullptr, nullptr, RMSF_MODE_WELFORD, 0, acc, ab, nullptr);
      });
      const SkPlan pl = sk_plan(3 * n / 4, 4, nf, 0, RMSF_MODE_WELFORD, kSkPerCuFlat);
      double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 4;
      char nm[96];
      snprintf(nm, sizeof nm, "same plan (G %d S %d), pure read", pl.G, pl.S);
      run(nm, [&] { hipLaunchKernelGGL((ub::stream<256, true>), dim3(pl.G), dim3(256), 0, 0, x, fs / 4, pl, p0, p1); });
      // 512 lanes per chunk (two library chunks side by side)
      SkPlan pw = sk_plan(3 * n / 4, 4, nf, 0, RMSF_MODE_WELFORD, kSkPerCuFlat, 512);
      if (pw.S == 0 && pw.C > 256) {  // many chunks: force the chunk-aligned cut as the library does
        pw.S = std::max<int64_t>(1, pl.S);
        pw.G = (int)(pw.C * pw.S);
        pw.P = (int)((nf / pw.S + kCoefN - 1) / kCoefN);
      }
      double *q1 = p0 + (size_t)pw.G * pw.P * 512 * 4;
      if (sk_bytes(pw, true) <= ab) {
        snprintf(nm, sizeof nm, "512 lanes/chunk (G %d S %d) Welford", pw.G, pw.S);
        run(nm, [&] { hipLaunchKernelGGL((ub::stream<512, false>), dim3(pw.G), dim3(512), 0, 0, x, fs / 4, pw, p0, q1); });
        snprintf(nm, sizeof nm, "512 lanes/chunk (G %d S %d) pure read", pw.G, pw.S);
        run(nm, [&] { hipLaunchKernelGGL((ub::stream<512, true>), dim3(pw.G), dim3(512), 0, 0, x, fs / 4, pw, p0, q1); });
      }
    }
  return 0;
}
