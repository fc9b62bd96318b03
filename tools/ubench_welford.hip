// Micro-benchmark of the C2 streaming Welford accumulator (k_welford_flat)
// against a pure-read ceiling, on the full 100k atoms x 20k frames (24 GB).
// Not product code.   hipcc -O3 --offload-arch=gfx950 tools/ubench_welford.hip -o tools/ubench_welford
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

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kCoefN = 16384;
struct WCoef {
  double a, b;
};
struct WCoefTable {
  WCoef v[kCoefN];
};
constexpr WCoefTable make_coef_table() {
  WCoefTable t{};
  for (int k = 0; k < kCoefN; ++k) {
    t.v[k].a = double(k) / double(k + 1);
    t.v[k].b = 1.0 / double(k + 1);
  }
  return t;
}
__constant__ WCoefTable g_coef = make_coef_table();

__device__ __forceinline__ void welford(double &m, double &q, double x, const WCoef c) {
  const double d = x - m;
  q = fma(c.a * d, d, q);
  m = fma(c.b, d, m);
}

template <bool NT>
__device__ __forceinline__ f4 ld(const f4 *p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}

// pure read ceiling: fp32 sums only
template <int U, int BS>
__global__ __launch_bounds__(BS) void k_read(const f4 *__restrict__ x, int64_t stride4, int64_t n4, int64_t nf, int S,
                                             float *out) {
  const int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n4) return;
  const int s = blockIdx.y;
  const int64_t fb = nf * s / S, fe = nf * (s + 1) / S;
  const f4 *p = x + fb * stride4 + i;
  f4 acc = {0, 0, 0, 0};
  int64_t k = 0;
  const int nfl = (int)(fe - fb);
  for (; k + U <= nfl; k += U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + (k + u) * stride4);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x == 1234.5f) out[i] = acc.y;
}

template <int U, int BS, bool NT>
__global__ __launch_bounds__(BS) void k_wel(const f4 *__restrict__ x, int64_t stride4, int64_t n4, int64_t nf, int S,
                                            double *__restrict__ om, double *__restrict__ oq) {
  const int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n4) return;
  const int s = blockIdx.y;
  const int64_t fb = nf * s / S, fe = nf * (s + 1) / S;
  const int nfl = (int)(fe - fb);
  const f4 *p = x + fb * stride4 + i;
  double m0 = 0, m1 = 0, m2 = 0, m3 = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0;
  int k = 0;
  for (; k + U <= nfl; k += U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(p + (int64_t)(k + u) * stride4);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const WCoef c = g_coef.v[k + u];
      welford(m0, q0, (double)v[u].x, c);
      welford(m1, q1, (double)v[u].y, c);
      welford(m2, q2, (double)v[u].z, c);
      welford(m3, q3, (double)v[u].w, c);
    }
  }
  for (; k < nfl; ++k) {
    const f4 v = ld<NT>(p + (int64_t)k * stride4);
    const WCoef c = g_coef.v[k];
    welford(m0, q0, (double)v.x, c);
    welford(m1, q1, (double)v.y, c);
    welford(m2, q2, (double)v.z, c);
    welford(m3, q3, (double)v.w, c);
  }
  const int64_t o = (int64_t)s * n4 * 4 + 4 * i;
  om[o] = m0;
  om[o + 1] = m1;
  om[o + 2] = m2;
  om[o + 3] = m3;
  oq[o] = q0;
  oq[o + 1] = q1;
  oq[o + 2] = q2;
  oq[o + 3] = q3;
}


// software-pipelined: the next U frames' loads are issued before the current
// U frames are consumed
template <int U, int BS>
__global__ __launch_bounds__(BS) void k_wel_sp(const f4 *__restrict__ x, int64_t stride4, int64_t n4, int64_t nf, int S,
                                               double *__restrict__ om, double *__restrict__ oq) {
  const int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n4) return;
  const int s = blockIdx.y;
  const int64_t fb = nf * s / S, fe = nf * (s + 1) / S;
  const int nfl = (int)(fe - fb);
  const f4 *p = x + fb * stride4 + i;
  double m0 = 0, m1 = 0, m2 = 0, m3 = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0;
  f4 cur[U], nxt[U];
  const int nfu = nfl / U * U;
#pragma unroll
  for (int u = 0; u < U; ++u) cur[u] = (u < nfu) ? __builtin_nontemporal_load(p + (int64_t)u * stride4) : f4{0, 0, 0, 0};
  for (int k = 0; k < nfu; k += U) {
    const bool more = k + U < nfu;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (more) nxt[u] = __builtin_nontemporal_load(p + (int64_t)(k + U + u) * stride4);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const WCoef c = g_coef.v[k + u];
      welford(m0, q0, (double)cur[u].x, c);
      welford(m1, q1, (double)cur[u].y, c);
      welford(m2, q2, (double)cur[u].z, c);
      welford(m3, q3, (double)cur[u].w, c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = nxt[u];
  }
  for (int k = nfu; k < nfl; ++k) {
    const f4 v = __builtin_nontemporal_load(p + (int64_t)k * stride4);
    const WCoef c = g_coef.v[k];
    welford(m0, q0, (double)v.x, c);
    welford(m1, q1, (double)v.y, c);
    welford(m2, q2, (double)v.z, c);
    welford(m3, q3, (double)v.w, c);
  }
  const int64_t o = (int64_t)s * n4 * 4 + 4 * i;
  om[o] = m0;
  om[o + 1] = m1;
  om[o + 2] = m2;
  om[o + 3] = m3;
  oq[o] = q0;
  oq[o + 1] = q1;
  oq[o + 2] = q2;
  oq[o + 3] = q3;
}

// balanced ("stream-K") decomposition: the (column chunk, frame) space is
// linearised chunk-major and cut into G equal ranges, one per workgroup, so
// every workgroup streams the same number of bytes and the grid has no tail
// wave.  A range spans at most a few chunks; each (chunk, range) segment
// writes one partial (slot 2b + j).
template <int U, int BS, bool READ_ONLY>
__global__ __launch_bounds__(BS) void k_wel_sk(const f4 *__restrict__ x, int64_t stride4, int64_t n4, int64_t nf,
                                               int G, double *__restrict__ om, double *__restrict__ oq) {
  const int64_t C = (n4 + BS - 1) / BS;
  const int64_t T = C * nf;
  const int b = blockIdx.x;
  int64_t lo = T * b / G;
  const int64_t hi = T * (b + 1) / G;
  int j = 0;
  while (lo < hi) {
    const int64_t c = lo / nf, f0 = lo % nf;
    const int64_t f1 = f0 + (hi - lo) < nf ? f0 + (hi - lo) : nf;
    const int nfl = (int)(f1 - f0);
    const int64_t i = c * BS + threadIdx.x;
    if (i < n4) {
      const f4 *p = x + f0 * stride4 + i;
      double m0 = 0, m1 = 0, m2 = 0, m3 = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0;
      f4 acc = {0, 0, 0, 0};
      int k = 0;
      for (; k + U <= nfl; k += U) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + (int64_t)(k + u) * stride4);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (READ_ONLY) {
            acc += v[u];
          } else {
            const WCoef cf = g_coef.v[k + u];
            welford(m0, q0, (double)v[u].x, cf);
            welford(m1, q1, (double)v[u].y, cf);
            welford(m2, q2, (double)v[u].z, cf);
            welford(m3, q3, (double)v[u].w, cf);
          }
        }
      }
      for (; k < nfl; ++k) {
        const f4 v = __builtin_nontemporal_load(p + (int64_t)k * stride4);
        const WCoef cf = g_coef.v[k];
        welford(m0, q0, (double)v.x, cf);
        welford(m1, q1, (double)v.y, cf);
        welford(m2, q2, (double)v.z, cf);
        welford(m3, q3, (double)v.w, cf);
      }
      if (READ_ONLY) m0 = acc.x + acc.y + acc.z + acc.w;
      const int64_t o = ((int64_t)(2 * b + j) * BS + threadIdx.x) * 4;
      if (!READ_ONLY || m0 == 1234.5) {
        om[o] = m0;
        om[o + 1] = m1;
        om[o + 2] = m2;
        om[o + 3] = m3;
        oq[o] = q0;
        oq[o + 1] = q1;
        oq[o + 2] = q2;
        oq[o + 3] = q3;
      }
    }
    lo += nfl;
    j = j < 1 ? j + 1 : 1;
  }
}

int main() {
  const int64_t n = 100000, nf = 20000, n4 = 3 * n / 4;
  const size_t bytes = sizeof(float) * 3 * n * nf;
  f4 *x;
  double *om, *oq;
  float *out;
  CK(hipMalloc(&x, bytes));
  CK(hipMemset(x, 0x3f, bytes));
  const int Smax = 256;
  CK(hipMalloc(&om, sizeof(double) * 3 * n * Smax));
  CK(hipMalloc(&oq, sizeof(double) * 3 * n * Smax));
  CK(hipMalloc(&out, sizeof(float) * 3 * n));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char *name, int S, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 8;
    CK(hipEventRecord(a));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= R;
    printf("%-34s S=%4d %7.3f ms %7.0f GB/s  frac %.3f\n", name, S, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 8000.0);
  };
#define RD(U, BS, S) \
  run("read U=" #U " BS=" #BS, S, [&] { hipLaunchKernelGGL((k_read<U, BS>), dim3((n4 + BS - 1) / BS, S), dim3(BS), 0, 0, x, n4, n4, nf, S, out); })
#define WL(U, BS, NT, S) \
  run("welford U=" #U " BS=" #BS " NT=" #NT, S, [&] { hipLaunchKernelGGL((k_wel<U, BS, NT>), dim3((n4 + BS - 1) / BS, S), dim3(BS), 0, 0, x, n4, n4, nf, S, om, oq); })
#define SP(U, BS, S) \
  run("welford-sp U=" #U " BS=" #BS, S, [&] { hipLaunchKernelGGL((k_wel_sp<U, BS>), dim3((n4 + BS - 1) / BS, S), dim3(BS), 0, 0, x, n4, n4, nf, S, om, oq); })
  const char *set = getenv("UB_SET");
  for (int rep = 0; rep < 2; ++rep) {
    if (set && set[0] == 'K') {  // balanced (stream-K) grid vs the split grid
#define SK(U, BS, RO, G) \
  run("sk U=" #U " BS=" #BS " RO=" #RO, G, [&] { hipLaunchKernelGGL((k_wel_sk<U, BS, RO>), dim3(G), dim3(BS), 0, 0, x, n4, n4, nf, G, om, oq); })
      RD(4, 256, 56);
      WL(4, 256, true, 12);
      for (int G : {512, 1024}) SK(4, 256, true, G);
      for (int G : {384, 512, 640, 768, 896, 1024, 1280, 1536}) SK(4, 256, false, G);
      for (int G : {512, 768, 1024}) SK(8, 256, false, G);
      for (int G : {256, 384, 512}) SK(4, 512, false, G);
      for (int G : {128, 256, 512}) SK(4, 1024, false, G);
      continue;
    }
    if (set && set[0] == 'S') {  // split-count sweep
      RD(4, 256, 12);
      RD(4, 256, 56);
      for (int S : {10, 12, 13, 20, 24, 28, 32, 40}) WL(4, 256, true, S);
      for (int S : {12, 24, 40}) WL(8, 256, true, S);
      for (int S : {12, 24}) WL(4, 512, true, S);
      continue;
    }
    RD(4, 256, 56);
    for (int S : {8, 12, 16, 56}) WL(4, 256, true, S);
    for (int S : {8, 12, 16, 56}) SP(4, 256, S);
    for (int S : {8, 16}) SP(2, 256, S);
  }
  return 0;
}
