// The aligned accumulator with the frames of each segment split over Q
// sub-blocks of one workgroup (Q x 256 threads, the 256 atoms of a chunk in
// every sub-block, a common shift, the Q shifted sums added in LDS before
// ONE partial is stored) against the library kernel (one 256-thread
// workgroup per range, one partial per segment).  Q x fewer partials for the
// same number of waves; the question is whether the partial traffic (196 MB
// per launch at 8,192 ranges = 6 % of a 2,500-frame share) and the launch
// tail are what the library kernel pays at small shares.  Not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_accum3.hip -o tools/ubench_accum3
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

// shifted sums (WELFORD) or sums (SUM) of nf aligned frames from p, shift given
template <int MODE, int U>
__device__ __forceinline__ void accum_span(const float *__restrict__ p, int64_t fstride, int nf,
                                           const double *__restrict__ xf, double rc0, double rc1, double rc2,
                                           const double (&sh)[3], double (&m)[3], double (&q)[3]) {
  auto consume = [&](float x, float y, float z, int k) {
    apply_xform(x, y, z, xf + (int64_t)k * kXform, rc0, rc1, rc2);
    if (MODE == RMSF_MODE_WELFORD) {
      const double d0 = (double)x - sh[0], d1 = (double)y - sh[1], d2 = (double)z - sh[2];
      m[0] += d0, m[1] += d1, m[2] += d2;
      q[0] = fma(d0, d0, q[0]), q[1] = fma(d1, d1, q[1]), q[2] = fma(d2, d2, q[2]);
    } else {
      m[0] += (double)x, m[1] += (double)y, m[2] += (double)z;
    }
  };
  int k = 0;
  for (; k + U <= nf; k += U) {
    float vx[U], vy[U], vz[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float *r = p + (int64_t)(k + u) * fstride;
      vx[u] = __builtin_nontemporal_load(r);
      vy[u] = __builtin_nontemporal_load(r + 1);
      vz[u] = __builtin_nontemporal_load(r + 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) consume(vx[u], vy[u], vz[u], k + u);
  }
  for (; k < nf; ++k) {
    const float *r = p + (int64_t)k * fstride;
    consume(r[0], r[1], r[2], k);
  }
}

template <int MODE, int Q, int U>
__global__ __launch_bounds__(kBlock *Q) void accum_q(const float *__restrict__ xyz, int64_t fstride,
                                                     const double *__restrict__ xform,
                                                     const double *__restrict__ refinfo, SkPlan pl,
                                                     int64_t *__restrict__ hdr, double *__restrict__ parts0,
                                                     double *__restrict__ parts1) {
  constexpr int NV = MODE == RMSF_MODE_WELFORD ? 6 : 3;
  __shared__ double red[(Q > 1 ? Q - 1 : 1) * NV * kBlock];
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
      if (MODE == RMSF_MODE_WELFORD) {  // common shift: the segment's first frame, transformed
        float x = p[0], y = p[1], z = p[2];
        apply_xform(x, y, z, xform + f0 * kXform, rc0, rc1, rc2);
        sh[0] = (double)x, sh[1] = (double)y, sh[2] = (double)z;
      }
      accum_span<MODE, U>(p + (int64_t)s0 * fstride, fstride, s1 - s0, xform + (f0 + s0) * kXform, rc0, rc1, rc2,
                          sh, m, q);
    }
    if (Q > 1) {
      if (qd > 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          red[((qd - 1) * NV + j) * kBlock + li] = m[j];
          if (MODE == RMSF_MODE_WELFORD) red[((qd - 1) * NV + 3 + j) * kBlock + li] = q[j];
        }
      }
      __syncthreads();
    }
    if (qd == 0 && live) {
#pragma unroll
      for (int v = 1; v < Q; ++v) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          m[j] += red[((v - 1) * NV + j) * kBlock + li];
          if (MODE == RMSF_MODE_WELFORD) q[j] += red[((v - 1) * NV + 3 + j) * kBlock + li];
        }
      }
      if (MODE == RMSF_MODE_WELFORD) {
        const double inv = g_coef.v[len - 1].b;
#pragma unroll
        for (int j = 0; j < 3; ++j) shifted_to_moments(m[j], q[j], sh[j], inv);
      }
      const int64_t o = slot * (kBlock * 3) + 3 * li;
      store3<MODE>(parts0 + o, parts1 + o, m, q);
    }
    if (Q > 1) __syncthreads();
    lo += len;
    ++slot;
  }
}
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
  auto qsplit = [&](int mode, int64_t nf, int per_cu, auto qq) {
    constexpr int Q = decltype(qq)::value;
    SkPlan pl = sk_plan(n, 3, nf, 0, mode, per_cu);
    int64_t *hdr = static_cast<int64_t *>(acc);
    double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
    double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 3;
    if (mode == RMSF_MODE_WELFORD)
      hipLaunchKernelGGL((ub::accum_q<RMSF_MODE_WELFORD, Q, 4>), dim3(pl.G), dim3(kBlock * Q), 0, 0, x, fs, xf, info,
                         pl, hdr, p0, p1);
    else
      hipLaunchKernelGGL((ub::accum_q<RMSF_MODE_SUM, Q, 4>), dim3(pl.G), dim3(kBlock * Q), 0, 0, x, fs, xf, info, pl,
                         hdr, p0, p1);
    return pl.G;
  };
  using Q2 = std::integral_constant<int, 2>;
  using Q4 = std::integral_constant<int, 4>;
  for (int64_t nf : {2500, 20000}) {  // agreement with the library (fold orders differ: rounding only)
    for (int mode : {RMSF_MODE_WELFORD, RMSF_MODE_SUM}) {
      std::vector<double> a0(fs), q0(fs), a1(fs), q1(fs);
      lib(mode, nf);
      rmsf_fold_balanced(acc, fs, mode, 0, out0, out1, nullptr);
      CK(hipMemcpy(a0.data(), out0, 8 * fs, hipMemcpyDeviceToHost));
      CK(hipMemcpy(q0.data(), out1, 8 * fs, hipMemcpyDeviceToHost));
      qsplit(mode, nf, 8, Q4{});
      rmsf_fold_balanced(acc, fs, mode, 0, out0, out1, nullptr);
      CK(hipMemcpy(a1.data(), out0, 8 * fs, hipMemcpyDeviceToHost));
      CK(hipMemcpy(q1.data(), out1, 8 * fs, hipMemcpyDeviceToHost));
      double da = 0, dq = 0;
      for (int64_t i = 0; i < fs; ++i) {
        da = std::max(da, std::fabs(a0[i] - a1[i]) / std::max(1.0, std::fabs(a0[i])));
        if (mode == RMSF_MODE_WELFORD) dq = std::max(dq, std::fabs(q0[i] - q1[i]) / std::max(1.0, std::fabs(q0[i])));
      }
      printf("frames %5ld mode %d  Q=4 vs library: max rel |d acc0| %.3e, max rel |d M2| %.3e\n", (long)nf, mode, da,
             dq);
    }
  }
  // accumulate + fold (the fold reads every partial: its cost grows with G*P)
  auto libg = [&](int mode, int64_t nf, int groups) {
    SkPlan pl = sk_plan(n, 3, nf, groups, mode, kSkPerCuAligned);
    int64_t *hdr = static_cast<int64_t *>(acc);
    double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
    double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 3;
    if (mode == RMSF_MODE_WELFORD)
      hipLaunchKernelGGL((k_accum_atoms_sk<RMSF_MODE_WELFORD, true, false, 4>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs,
                         nullptr, xf, info, pl, hdr, p0, p1);
    else
      hipLaunchKernelGGL((k_accum_atoms_sk<RMSF_MODE_SUM, true, false, 4>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs,
                         nullptr, xf, info, pl, hdr, p0, p1);
  };
  auto fold = [&](int mode) { rmsf_fold_balanced(acc, fs, mode, 0, out0, out1, nullptr); };
  char nm[96];
  for (int rep = 0; rep < 2; ++rep) {
    for (int64_t nf : {2500, 5000, 20000}) {
      for (int mode : {RMSF_MODE_WELFORD, RMSF_MODE_SUM}) {
        const char *mn = mode == RMSF_MODE_WELFORD ? "WEL" : "SUM";
        snprintf(nm, sizeof nm, "%s lib 32/CU x256 +fold", mn);
        run(nm, nf, [&] { lib(mode, nf); fold(mode); });
        for (int groups : {2048, 4096}) {
          snprintf(nm, sizeof nm, "%s lib G=%d x256 +fold", mn, groups);
          run(nm, nf, [&] { libg(mode, nf, groups); fold(mode); });
        }
        for (int per_cu : {8, 16, 32}) {
          snprintf(nm, sizeof nm, "%s Q=2 %d/CU x512 +fold", mn, per_cu);
          run(nm, nf, [&] { qsplit(mode, nf, per_cu, Q2{}); fold(mode); });
        }
        for (int per_cu : {4, 8}) {
          snprintf(nm, sizeof nm, "%s Q=4 %d/CU x1024 +fold", mn, per_cu);
          run(nm, nf, [&] { qsplit(mode, nf, per_cu, Q4{}); fold(mode); });
        }
      }
    }
  }
  return 0;
}
