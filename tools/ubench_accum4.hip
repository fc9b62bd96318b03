// Aligned Welford accumulate (k_accum_split_sk<WELFORD, ALIGN, Q = 2>, the
// C3 / RMSF.py sweep-2 kernel, 1.08-1.11x the unaligned stream) against
// variants aimed at its memory-level parallelism: more waves per SIMD
// (amdgpu_waves_per_eu 6 / 8 caps the VGPRs), software-pipelined loads (the
// next U frames in flight while the current U are transformed), U = 2.
// The unaligned float4 Welford stream (k_welford_flat_sk) of the same bytes
// is timed in the same process as the floor.  Not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_accum4.hip -o tools/ubench_accum4
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

namespace ub {

template <int U>
__device__ __forceinline__ void consume1(float x, float y, float z, const double *__restrict__ t, double rc0,
                                         double rc1, double rc2, const double (&sh)[3], double (&m)[3],
                                         double (&q)[3]) {
  apply_xform(x, y, z, t, rc0, rc1, rc2);
  const double d0 = (double)x - sh[0], d1 = (double)y - sh[1], d2 = (double)z - sh[2];
  m[0] += d0, m[1] += d1, m[2] += d2;
  q[0] = fma(d0, d0, q[0]), q[1] = fma(d1, d1, q[1]), q[2] = fma(d2, d2, q[2]);
}

// PIPE = 0: the library's loop (U loads, then U transforms); 1: double-buffered
template <int U, int PIPE>
__device__ __forceinline__ void span(const float *__restrict__ p, int64_t fstride, int nf,
                                     const double *__restrict__ xf, double rc0, double rc1, double rc2,
                                     const double (&sh)[3], double (&m)[3], double (&q)[3]) {
  int k = 0;
  if (PIPE && nf >= U) {
    float cx[U], cy[U], cz[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float *r = p + (int64_t)u * fstride;
      cx[u] = __builtin_nontemporal_load(r), cy[u] = __builtin_nontemporal_load(r + 1),
      cz[u] = __builtin_nontemporal_load(r + 2);
    }
    for (; k + 2 * U <= nf; k += U) {
      float nx[U], ny[U], nz[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float *r = p + (int64_t)(k + U + u) * fstride;
        nx[u] = __builtin_nontemporal_load(r), ny[u] = __builtin_nontemporal_load(r + 1),
        nz[u] = __builtin_nontemporal_load(r + 2);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) consume1<U>(cx[u], cy[u], cz[u], xf + (int64_t)(k + u) * kXform, rc0, rc1, rc2, sh, m, q);
#pragma unroll
      for (int u = 0; u < U; ++u) cx[u] = nx[u], cy[u] = ny[u], cz[u] = nz[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) consume1<U>(cx[u], cy[u], cz[u], xf + (int64_t)(k + u) * kXform, rc0, rc1, rc2, sh, m, q);
    k += U;
  } else {
    for (; k + U <= nf; k += U) {
      float vx[U], vy[U], vz[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float *r = p + (int64_t)(k + u) * fstride;
        vx[u] = __builtin_nontemporal_load(r), vy[u] = __builtin_nontemporal_load(r + 1),
        vz[u] = __builtin_nontemporal_load(r + 2);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) consume1<U>(vx[u], vy[u], vz[u], xf + (int64_t)(k + u) * kXform, rc0, rc1, rc2, sh, m, q);
    }
  }
  for (; k < nf; ++k) {
    const float *r = p + (int64_t)k * fstride;
    consume1<U>(r[0], r[1], r[2], xf + (int64_t)k * kXform, rc0, rc1, rc2, sh, m, q);
  }
}

template <int U, int PIPE>
__device__ __forceinline__ void body(const float *__restrict__ xyz, int64_t fstride, const double *__restrict__ xform,
                                     const double *__restrict__ refinfo, const SkPlan &pl, int64_t *__restrict__ hdr,
                                     double *__restrict__ parts0, double *__restrict__ parts1, double *red) {
  constexpr int Q = 2, NV = 6;
  const int b = sk_range(pl, blockIdx.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) sk_write_header(hdr, pl);
  const int li = threadIdx.x % kBlock;
  const int qd = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kBlock));
  const double rc0 = refinfo[0], rc1 = refinfo[1], rc2 = refinfo[2];
  int64_t lo = uni64(sk_lo(pl, b));
  const int64_t hi = uni64(sk_lo(pl, b + 1));
  int64_t slot = (int64_t)b * pl.P;
  while (lo < hi) {
    int64_t c, f0;
    const int len = __builtin_amdgcn_readfirstlane((int)sk_seg_len(pl, lo, hi, &c, &f0));
    c = uni64(c);
    f0 = uni64(f0);
    const int64_t a = c * kBlock + li;
    const bool live = a < pl.lanes;
    const int s0 = (int)((int64_t)len * qd / Q), s1 = (int)((int64_t)len * (qd + 1) / Q);
    double m[3] = {0.0, 0.0, 0.0}, q[3] = {0.0, 0.0, 0.0}, sh[3] = {0.0, 0.0, 0.0};
    if (live) {
      const float *p = xyz + f0 * fstride + 3 * a;
      float x = p[0], y = p[1], z = p[2];
      apply_xform(x, y, z, xform + f0 * kXform, rc0, rc1, rc2);
      sh[0] = (double)x, sh[1] = (double)y, sh[2] = (double)z;
      span<U, PIPE>(p + (int64_t)s0 * fstride, fstride, s1 - s0, xform + (f0 + s0) * kXform, rc0, rc1, rc2, sh, m, q);
    }
    if (qd > 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) red[((qd - 1) * NV + j) * kBlock + li] = m[j], red[((qd - 1) * NV + 3 + j) * kBlock + li] = q[j];
    }
    __syncthreads();
    if (qd == 0 && live) {
#pragma unroll
      for (int j = 0; j < 3; ++j) m[j] += red[j * kBlock + li], q[j] += red[(3 + j) * kBlock + li];
      const double inv = g_coef.v[len - 1].b;
#pragma unroll
      for (int j = 0; j < 3; ++j) shifted_to_moments(m[j], q[j], sh[j], inv);
      const int64_t o = slot * (kBlock * 3) + 3 * li;
      store3<RMSF_MODE_WELFORD>(parts0 + o, parts1 + o, m, q);
    }
    __syncthreads();
    lo += len;
    ++slot;
  }
}

#define UB_ARGS const float *__restrict__ xyz, int64_t fstride, const double *__restrict__ xform, \
  const double *__restrict__ refinfo, SkPlan pl, int64_t *__restrict__ hdr, double *__restrict__ parts0, \
  double *__restrict__ parts1
#define UB_KERNEL(NAME, U, PIPE, ATTR)                                                   \
  __global__ __launch_bounds__(512) ATTR void NAME(UB_ARGS) {                            \
    __shared__ double red[6 * kBlock];                                                   \
    body<U, PIPE>(xyz, fstride, xform, refinfo, pl, hdr, parts0, parts1, red);           \
  }
UB_KERNEL(k_base, 4, 0, )
UB_KERNEL(k_w6, 4, 0, __attribute__((amdgpu_waves_per_eu(6))))
UB_KERNEL(k_w8, 4, 0, __attribute__((amdgpu_waves_per_eu(8))))
UB_KERNEL(k_pipe, 4, 1, )
UB_KERNEL(k_pipe_w6, 4, 1, __attribute__((amdgpu_waves_per_eu(6))))
UB_KERNEL(k_u2_w8, 2, 0, __attribute__((amdgpu_waves_per_eu(8))))
UB_KERNEL(k_pipe2_w8, 2, 1, __attribute__((amdgpu_waves_per_eu(8))))
}  // namespace ub

int main() {
  const int64_t n = 100000, nf_max = 20000, fs = 3 * n;
  float *x;
  double *ref, *info, *xf, *out0, *out1;
  CK(hipMalloc(&x, sizeof(float) * fs * nf_max));
  CK(hipMalloc(&ref, sizeof(double) * 3 * n));
  CK(hipMalloc(&info, sizeof(double) * RMSF_REFINFO_DOUBLES));
  CK(hipMalloc(&xf, sizeof(double) * RMSF_XFORM_DOUBLES * nf_max));
  CK(hipMalloc(&out0, sizeof(double) * fs));
  CK(hipMalloc(&out1, sizeof(double) * fs));
  std::vector<double> motion(12 * nf_max, 0.0);
  for (int64_t f = 0; f < nf_max; ++f) {  // small rotations about z + shifts
    const double an = 0.01 * (f % 97);
    motion[12 * f + 0] = std::cos(an), motion[12 * f + 1] = -std::sin(an);
    motion[12 * f + 3] = std::sin(an), motion[12 * f + 4] = std::cos(an);
    motion[12 * f + 8] = 1.0;
    motion[12 * f + 9] = 50.0 + 0.001 * (f % 7), motion[12 * f + 10] = 50.0, motion[12 * f + 11] = 50.0;
  }
  double *dm;
  CK(hipMalloc(&dm, sizeof(double) * motion.size()));
  CK(hipMemcpy(dm, motion.data(), sizeof(double) * motion.size(), hipMemcpyHostToDevice));
  const size_t wb = rmsf_superpose_workspace_bytes(n, nf_max);
  void *work;
  CK(hipMalloc(&work, wb));
  if (rmsf_synth_frames(x, fs, n, 0, nf_max, 0, dm, nullptr) ||
      rmsf_reference_setup(x, nullptr, n, nullptr, nullptr, ref, info, nullptr) ||
      rmsf_superpose(x, fs, nf_max, n, nullptr, nullptr, ref, info, xf, work, wb, nullptr)) {
    printf("setup failed: %s\n", rmsf_last_error());
    return 1;
  }
  CK(hipDeviceSynchronize());
  const size_t ab = (size_t)2 << 30;
  void *acc;
  CK(hipMalloc(&acc, ab));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char *name, int64_t nf, auto launch) {
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
    printf("frames %5ld %-40s %7.4f ms (min %7.4f)  %6.0f GB/s\n", (long)nf, name, sum / R, best,
           bytes / (sum / R) / 1e6);
    fflush(stdout);
  };
  auto lib = [&](int mode, int64_t nf) {
    rmsf_accumulate_balanced(x, fs, nf, n, nullptr, xf, info, mode, 0, acc, ab, nullptr);
  };
  auto stream = [&](int64_t nf) {  // the unaligned float4 stream of the same bytes
    rmsf_accumulate_balanced(x, fs, nf, n, nullptr, nullptr, nullptr, RMSF_MODE_WELFORD, 0, acc, ab, nullptr);
  };
  auto fold = [&] { rmsf_fold_balanced(acc, fs, RMSF_MODE_WELFORD, 0, out0, out1, nullptr); };
  typedef void (*KFn)(const float *, int64_t, const double *, const double *, SkPlan, int64_t *, double *, double *);
  auto var = [&](KFn k, int64_t nf, int per_cu) {
    SkPlan pl = sk_plan(n, 3, nf, 0, RMSF_MODE_WELFORD, per_cu);
    int64_t *hdr = static_cast<int64_t *>(acc);
    double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
    double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 3;
    hipLaunchKernelGGL(k, dim3(pl.G), dim3(512), 0, 0, x, fs, xf, info, pl, hdr, p0, p1);
  };
  struct V { const char *name; KFn k; };
  const V vs[] = {{"base (library copy)", ub::k_base}, {"waves_per_eu 6", ub::k_w6}, {"waves_per_eu 8", ub::k_w8},
                  {"pipelined U=4", ub::k_pipe}, {"pipelined U=4 wpe 6", ub::k_pipe_w6}, {"U=2 wpe 8", ub::k_u2_w8},
                  {"pipelined U=2 wpe 8", ub::k_pipe2_w8}};
  {  // agreement with the library (identical code paths but the loop shape: rounding-identical expected)
    std::vector<double> a0(fs), q0(fs), a1(fs), q1(fs);
    lib(RMSF_MODE_WELFORD, 2500);
    fold();
    CK(hipMemcpy(a0.data(), out0, 8 * fs, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q0.data(), out1, 8 * fs, hipMemcpyDeviceToHost));
    for (const V &v : vs) {
      var(v.k, 2500, 8);
      fold();
      CK(hipMemcpy(a1.data(), out0, 8 * fs, hipMemcpyDeviceToHost));
      CK(hipMemcpy(q1.data(), out1, 8 * fs, hipMemcpyDeviceToHost));
      double d = 0;
      for (int64_t i = 0; i < fs; ++i) d = std::max(d, std::max(std::fabs(a0[i] - a1[i]), std::fabs(q0[i] - q1[i])));
      printf("%-24s max |diff| vs library %.3e\n", v.name, d);
    }
  }
  char nm[128];
  for (int rep = 0; rep < 2; ++rep) {
    for (int64_t nf : {2500, 20000}) {
      run("STREAM unaligned float4 (floor)", nf, [&] { stream(nf); });
      run("library k_accum_split_sk", nf, [&] { lib(RMSF_MODE_WELFORD, nf); });
      for (const V &v : vs)
        for (int per_cu : {8, 16}) {
          snprintf(nm, sizeof nm, "%s %d/CU", v.name, per_cu);
          run(nm, nf, [&] { var(v.k, nf, per_cu); });
        }
    }
  }
  return 0;
}
