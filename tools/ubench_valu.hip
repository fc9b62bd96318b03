// VALU ceiling of the per-atom-frame bodies, no frame loads (not product code).
// Frames are synthesised in registers; the per-frame transform still comes by
// scalar loads, so only the trajectory stream is missing.  100k atoms x 20k
// frames, same grid as the product kernels.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_valu.hip -o tools/ubench_valu
// B0  apply (3 f32 rounding points) + Welford   (k_accum_atoms<WELFORD, ALIGN>)
// B1  Welford only                              (k_welford_flat body, 1 coord)
// B2  superposition sums (covariance, COM, |x|^2)  (k_frame_stats body)
// B3  B2 + B0                                   (a fused single-read sweep)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

struct WCoef {
  double a, b;
};
__constant__ WCoef g_coef[4096];

__device__ __forceinline__ void welford(double &m, double &q, double x, const WCoef c) {
  const double d = x - m;
  q = fma(c.a * d, d, q);
  m = fma(c.b, d, m);
}

__device__ __forceinline__ void apply_xform(float &x, float &y, float &z, const double *__restrict__ t, double rc0,
                                            double rc1, double rc2) {
  const float p0 = (float)((double)x - t[9]);
  const float p1 = (float)((double)y - t[10]);
  const float p2 = (float)((double)z - t[11]);
  const double d0 = p0, d1 = p1, d2 = p2;
  const float r0 = (float)(d0 * t[0] + d1 * t[3] + d2 * t[6]);
  const float r1 = (float)(d0 * t[1] + d1 * t[4] + d2 * t[7]);
  const float r2 = (float)(d0 * t[2] + d1 * t[5] + d2 * t[8]);
  x = (float)((double)r0 + rc0);
  y = (float)((double)r1 + rc1);
  z = (float)((double)r2 + rc2);
}

template <int B>
__global__ __launch_bounds__(256) void k_body(int64_t n_sel, int64_t nf, int S, const double *__restrict__ xform,
                                              const double *__restrict__ ref, double *__restrict__ out) {
  const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (a >= n_sel) return;
  const int s = blockIdx.y;
  const int64_t fb = nf * s / S;
  const int n = (int)(nf * (s + 1) / S - fb);
  const double *xf = xform + fb * 16;
  const double r0 = ref[0], r1 = ref[1], r2 = ref[2];
  float bx = 20.f + (float)(a & 1023) * 0.05f, by = bx + 1.f, bz = bx + 2.f;
  double m0 = 0, m1 = 0, m2 = 0, q0 = 0, q1 = 0, q2 = 0;
  double acc[13] = {};
#pragma unroll 4
  for (int k = 0; k < n; ++k) {
    float x = bx + (float)k * 1e-3f, y = by - (float)k * 1e-3f, z = bz + (float)(k & 7);
    if (B == 2 || B == 3) {
      const double X = x, Y = y, Z = z;
      acc[0] += X;
      acc[1] += Y;
      acc[2] += Z;
      acc[3] = fma(X, r0, acc[3]);
      acc[4] = fma(X, r1, acc[4]);
      acc[5] = fma(X, r2, acc[5]);
      acc[6] = fma(Y, r0, acc[6]);
      acc[7] = fma(Y, r1, acc[7]);
      acc[8] = fma(Y, r2, acc[8]);
      acc[9] = fma(Z, r0, acc[9]);
      acc[10] = fma(Z, r1, acc[10]);
      acc[11] = fma(Z, r2, acc[11]);
      acc[12] = fma(X, X, fma(Y, Y, fma(Z, Z, acc[12])));
    }
    if (B == 0 || B == 3) apply_xform(x, y, z, xf + (int64_t)k * 16, 50.0, 49.0, 51.0);
    if (B != 2) {
      const WCoef c = g_coef[k & 4095];
      welford(m0, q0, (double)x, c);
      if (B != 1) {
        welford(m1, q1, (double)y, c);
        welford(m2, q2, (double)z, c);
      }
    }
  }
  double t = m0 + m1 + m2 + q0 + q1 + q2;
  for (int j = 0; j < 13; ++j) t += acc[j];
  out[a + s * n_sel] = t;
}

__global__ void k_fill_xform(double *xf, int64_t nf) {
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= nf) return;
  double *t = xf + 16 * f;
  const double c = cos(0.001 * f), s = sin(0.001 * f);
  const double R[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
  for (int j = 0; j < 9; ++j) t[j] = R[j];
  t[9] = 50.0;
  t[10] = 49.0;
  t[11] = 51.0;
}

int main() {
  const int64_t n = 100000, nf = 20000;
  const int S = 12;
  double *xf, *ref, *out;
  CK(hipMalloc(&xf, sizeof(double) * 16 * nf));
  CK(hipMalloc(&ref, sizeof(double) * 16));
  CK(hipMalloc(&out, sizeof(double) * n * S));
  CK(hipMemset(ref, 0, sizeof(double) * 16));
  hipLaunchKernelGGL(k_fill_xform, dim3((nf + 255) / 256), dim3(256), 0, 0, xf, nf);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char *name, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 5;
    CK(hipEventRecord(a));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= R;
    printf("%-44s %7.3f ms  %.3e atom-frames/s  (12 B/af at 8 TB/s: %.3f ms)\n", name, ms, n * nf / (ms * 1e-3),
           12.0 * n * nf / 8e12 * 1e3);
  };
#define B(V, name) run(name, [&] { hipLaunchKernelGGL((k_body<V>), dim3((n + 255) / 256, S), dim3(256), 0, 0, n, nf, S, xf, ref, out); })
  for (int rep = 0; rep < 2; ++rep) {
    B(0, "B0 apply + Welford (3 coords)");
    B(1, "B1 Welford (1 coord)");
    B(2, "B2 superposition sums");
    B(3, "B3 sums + apply + Welford (fused body)");
  }
  return 0;
}
