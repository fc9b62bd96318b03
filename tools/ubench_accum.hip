// Ablation of the aligned per-atom accumulator (k_accum_atoms<WELFORD, ALIGN>)
// on 100k atoms x 20k frames (24 GB).  Not product code.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_accum.hip -o tools/ubench_accum
// V0  product: f32-faithful transform + Welford           (U frames in flight)
// V1  no transform, Welford                                (dwordx3 stream floor)
// V2  transform + f64 sum only (SUM mode)
// V3  transform + shifted sums (s1, s2 about a per-atom shift; 3 ops/coord)
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

constexpr int kCoefN = 4096;
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

template <int V, int U, int BS>
__global__ __launch_bounds__(BS) void k_acc(const float *__restrict__ xyz, int64_t fstride, int64_t n_sel, int64_t nf,
                                            int S, const double *__restrict__ xform, const double *__restrict__ refinfo,
                                            const double *__restrict__ shift, double *__restrict__ o0,
                                            double *__restrict__ o1) {
  const int64_t a = (int64_t)blockIdx.x * BS + threadIdx.x;
  if (a >= n_sel) return;
  const int s = blockIdx.y;
  const int64_t fb = nf * s / S;
  const int n = (int)(nf * (s + 1) / S - fb);
  const float *p = xyz + fb * fstride + 3 * a;
  const double *xf = xform + fb * 16;
  const double rc0 = refinfo[0], rc1 = refinfo[1], rc2 = refinfo[2];
  double h0 = 0, h1 = 0, h2 = 0;
  if (V == 3) {
    h0 = shift[3 * a];
    h1 = shift[3 * a + 1];
    h2 = shift[3 * a + 2];
  }
  double m0 = 0, m1 = 0, m2 = 0, q0 = 0, q1 = 0, q2 = 0;
  auto consume = [&](float x, float y, float z, int k) {
    if (V != 1) apply_xform(x, y, z, xf + (int64_t)k * 16, rc0, rc1, rc2);
    if (V == 0 || V == 1) {
      const WCoef c = g_coef.v[k];
      welford(m0, q0, (double)x, c);
      welford(m1, q1, (double)y, c);
      welford(m2, q2, (double)z, c);
    } else if (V == 2) {
      m0 += (double)x;
      m1 += (double)y;
      m2 += (double)z;
    } else {
      const double e0 = (double)x - h0, e1 = (double)y - h1, e2 = (double)z - h2;
      m0 += e0;
      m1 += e1;
      m2 += e2;
      q0 = fma(e0, e0, q0);
      q1 = fma(e1, e1, q1);
      q2 = fma(e2, e2, q2);
    }
  };
  int k = 0;
  for (; k + U <= n; k += U) {
    float vx[U], vy[U], vz[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float *q = p + (int64_t)(k + u) * fstride;
      vx[u] = __builtin_nontemporal_load(q);
      vy[u] = __builtin_nontemporal_load(q + 1);
      vz[u] = __builtin_nontemporal_load(q + 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) consume(vx[u], vy[u], vz[u], k + u);
  }
  for (; k < n; ++k) {
    const float *q = p + (int64_t)k * fstride;
    consume(q[0], q[1], q[2], k);
  }
  const int64_t o = (int64_t)s * 3 * n_sel + 3 * a;
  o0[o] = m0;
  o0[o + 1] = m1;
  o0[o + 2] = m2;
  o1[o] = q0;
  o1[o + 1] = q1;
  o1[o + 2] = q2;
}

// V0 with a register ring: the loads of frame k+D are issued while frame k
// is consumed (D frames in flight per lane at all times).  XS: the per-frame
// transform comes by scalar loads (0) or is staged in LDS in 64-frame chunks (1).
template <int D, int BS, int XS>
__global__ __launch_bounds__(BS) void k_acc_pf(const float *__restrict__ xyz, int64_t fstride, int64_t n_sel,
                                               int64_t nf, int S, const double *__restrict__ xform,
                                               const double *__restrict__ refinfo, double *__restrict__ o0,
                                               double *__restrict__ o1) {
  __shared__ double xl[XS ? 64 * 12 : 1];
  const int64_t a = (int64_t)blockIdx.x * BS + threadIdx.x;
  const bool live = a < n_sel;
  const int64_t ac = live ? a : n_sel - 1;
  const int s = blockIdx.y;
  const int64_t fb = nf * s / S;
  const int n = (int)(nf * (s + 1) / S - fb);
  const float *p = xyz + fb * fstride + 3 * ac;
  const double *xf = xform + fb * 16;
  const double rc0 = refinfo[0], rc1 = refinfo[1], rc2 = refinfo[2];
  double m0 = 0, m1 = 0, m2 = 0, q0 = 0, q1 = 0, q2 = 0;
  float bx[D], by[D], bz[D];
#pragma unroll
  for (int u = 0; u < D; ++u) {
    const float *q = p + (int64_t)min(u, n - 1) * fstride;
    bx[u] = __builtin_nontemporal_load(q);
    by[u] = __builtin_nontemporal_load(q + 1);
    bz[u] = __builtin_nontemporal_load(q + 2);
  }
  for (int k = 0; k < n; k += D) {
    if (XS && (k & 63) == 0) {
      __syncthreads();
      for (int i = threadIdx.x; i < 64 * 12; i += BS) {
        const int f = k + i / 12;
        xl[i] = f < n ? xf[(int64_t)f * 16 + i % 12] : 0.0;
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < D; ++u) {
      float x = bx[u], y = by[u], z = bz[u];
      const float *q = p + (int64_t)min(k + D + u, n - 1) * fstride;
      bx[u] = __builtin_nontemporal_load(q);
      by[u] = __builtin_nontemporal_load(q + 1);
      bz[u] = __builtin_nontemporal_load(q + 2);
      if (k + u < n) {
        const double *t = XS ? xl + ((k + u) & 63) * 12 : xf + (int64_t)(k + u) * 16;
        apply_xform(x, y, z, t, rc0, rc1, rc2);
        const WCoef c = g_coef.v[k + u];
        welford(m0, q0, (double)x, c);
        welford(m1, q1, (double)y, c);
        welford(m2, q2, (double)z, c);
      }
    }
  }
  if (!live) return;
  const int64_t o = (int64_t)s * 3 * n_sel + 3 * a;
  o0[o] = m0;
  o0[o + 1] = m1;
  o0[o + 2] = m2;
  o1[o] = q0;
  o1[o + 1] = q1;
  o1[o + 2] = q2;
}


// V4: 4 atoms per lane from three float4 loads at a 48-B lane stride.
// V5: three fully coalesced float4 loads per wave-frame (768 floats = 256
//     atoms), transposed through LDS so each lane gets its 4 atoms.
typedef float f4 __attribute__((ext_vector_type(4)));
template <int V, int U, int BS>
__global__ __launch_bounds__(BS) void k_acc4(const float *__restrict__ xyz, int64_t fstride, int64_t n_sel, int64_t nf,
                                             int S, const double *__restrict__ xform, const double *__restrict__ refinfo,
                                             double *__restrict__ o0, double *__restrict__ o1) {
  __shared__ __attribute__((aligned(16))) float lds[(V == 5) ? (BS / 64) * U * 768 : 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t a0 = ((int64_t)blockIdx.x * BS + (threadIdx.x & ~63)) * 4;  // wave's first atom
  const int64_t a = a0 + 4 * lane;                                          // lane's first atom
  if (a0 >= n_sel) return;  // n_sel is a multiple of 256 here
  const int s = blockIdx.y;
  const int64_t fb = nf * s / S;
  const int n = (int)(nf * (s + 1) / S - fb);
  const double *xf = xform + fb * 16;
  const double rc0 = refinfo[0], rc1 = refinfo[1], rc2 = refinfo[2];
  double m[12], q[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) m[j] = q[j] = 0.0;
  int k = 0;
  for (; k + U <= n; k += U) {
    f4 v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float *fr = xyz + (fb + k + u) * fstride;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (V == 4) v[u][j] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(fr + 3 * a) + j);
        else v[u][j] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(fr + 3 * a0) + j * 64 + lane);
      }
    }
    if (V == 5) {
      float *L = lds + w * U * 768;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 3; ++j) *reinterpret_cast<f4 *>(L + u * 768 + 4 * (j * 64 + lane)) = v[u][j];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's own LDS region, no barrier needed
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 3; ++j) v[u][j] = *reinterpret_cast<const f4 *>(L + u * 768 + 12 * lane + 4 * j);
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float c[12] = {v[u][0].x, v[u][0].y, v[u][0].z, v[u][0].w, v[u][1].x, v[u][1].y,
                     v[u][1].z, v[u][1].w, v[u][2].x, v[u][2].y, v[u][2].z, v[u][2].w};
      const double *t = xf + (int64_t)(k + u) * 16;
      const WCoef cf = g_coef.v[k + u];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        apply_xform(c[3 * i], c[3 * i + 1], c[3 * i + 2], t, rc0, rc1, rc2);
        welford(m[3 * i], q[3 * i], (double)c[3 * i], cf);
        welford(m[3 * i + 1], q[3 * i + 1], (double)c[3 * i + 1], cf);
        welford(m[3 * i + 2], q[3 * i + 2], (double)c[3 * i + 2], cf);
      }
    }
  }
  const int64_t o = (int64_t)s * 3 * n_sel + 3 * a;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    o0[o + j] = m[j];
    o1[o + j] = q[j];
  }
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

__global__ void k_fill_xyz(float *x, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] = 20.0f + 60.0f * (float)((i * 2654435761ull) % 1000003) / 1000003.0f;
}

int main() {
  const int64_t n = 100096, nf = 20000, fs = 3 * n;  // multiple of 256 atoms (V4/V5 have no tail)
  const size_t bytes = sizeof(float) * fs * nf;
  float *x;
  double *xf, *ri, *sh, *o0, *o1;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&xf, sizeof(double) * 16 * nf));
  CK(hipMalloc(&ri, sizeof(double) * 16));
  CK(hipMalloc(&sh, sizeof(double) * 3 * n));
  const int Smax = 128;
  CK(hipMalloc(&o0, sizeof(double) * 3 * n * Smax));
  CK(hipMalloc(&o1, sizeof(double) * 3 * n * Smax));
  hipLaunchKernelGGL(k_fill_xyz, dim3((fs * nf + 255) / 256), dim3(256), 0, 0, x, fs * nf);
  hipLaunchKernelGGL(k_fill_xform, dim3((nf + 255) / 256), dim3(256), 0, 0, xf, nf);
  CK(hipMemset(ri, 0, sizeof(double) * 16));
  CK(hipMemset(sh, 0, sizeof(double) * 3 * n));
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char *name, int S, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 6;
    CK(hipEventRecord(a));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= R;
    printf("%-36s S=%3d %7.3f ms %7.0f GB/s  frac %.3f\n", name, S, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 8000.0);
  };
#define AC(V, U, BS, S)                                                                                           \
  run("V" #V " U=" #U " BS=" #BS, S, [&] {                                                                         \
    hipLaunchKernelGGL((k_acc<V, U, BS>), dim3((n + BS - 1) / BS, S), dim3(BS), 0, 0, x, fs, n, nf, S, xf, ri, sh, \
                       o0, o1);                                                                                    \
  })
#define AC4(V, U, BS, S)                                                                                           \
  run("V" #V " 4 atoms/lane U=" #U " BS=" #BS, S, [&] {                                                            \
    hipLaunchKernelGGL((k_acc4<V, U, BS>), dim3((n / 4 + BS - 1) / BS, S), dim3(BS), 0, 0, x, fs, n, nf, S, xf, ri, \
                       o0, o1);                                                                                     \
  })
#define PF(D, BS, XS, S)                                                                                    \
  run("V0 ring D=" #D " BS=" #BS " XS=" #XS, S, [&] {                                                       \
    hipLaunchKernelGGL((k_acc_pf<D, BS, XS>), dim3((n + BS - 1) / BS, S), dim3(BS), 0, 0, x, fs, n, nf, S, xf, \
                       ri, o0, o1);                                                                        \
  })
  const char *which = getenv("UB_SET");
  const bool layouts = which && which[0] == 'L';
  for (int rep = 0; rep < 2; ++rep) {
    AC(0, 4, 256, 12);
    AC(1, 4, 256, 12);
    if (layouts) {
      AC4(4, 2, 256, 12);
      AC4(4, 2, 256, 48);
      AC4(4, 1, 256, 48);
      AC4(5, 2, 256, 12);
      AC4(5, 2, 256, 48);
      AC4(5, 1, 256, 48);
      AC4(5, 2, 128, 48);
      continue;
    }
    AC(0, 2, 256, 12);
    AC(0, 8, 256, 12);
    PF(2, 256, 0, 12);
    PF(4, 256, 0, 12);
    PF(4, 256, 0, 24);
    PF(8, 256, 0, 12);
    PF(4, 256, 1, 12);
    PF(8, 256, 1, 12);
    PF(4, 512, 1, 12);
  }
  return 0;
}
