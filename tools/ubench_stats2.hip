// Ablation of the superposition-sums kernel AS BUILT IN THE LIBRARY
// (k_frame_stats, included from csrc/rmsf_kernels.hip into this TU) against
// the round-1 micro-benchmark twin V11 and candidate variants, in one
// process, on the C3 shape (100k atoms x 20k frames, contiguous selection,
// frame pitch 1.2 MB).  Not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_stats2.hip -o tools/ubench_stats2
//
// Variants:
//   lib(chunk)       the library kernel k_frame_stats<false,false,true>
//   v11(chunk)       round-1 twin (no tail checks, no partial writes)
//   copy<T,E>(chunk) a copy of the library kernel: T = tail checks on/off,
//                    E = epilogue (wave fold + partial store) on/off
//   sk<E>(G)         balanced ("stream-K") grid: G workgroups, each one equal
//                    contiguous range of (64-frame group, 32-atom tile) units
#include "../mdanalysis-mpi_amd/csrc/rmsf_kernels.hip"

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

namespace ub {
using ::f32x4;

// --- V11 (tools/ubench_stats.hip k_lanes_frames2<32>) -----------------------
__global__ __launch_bounds__(kBlock) void v11(const float *__restrict__ xyz, int64_t fstride, int64_t n_frames,
                                              int64_t n, int64_t chunk, const double *__restrict__ ref,
                                              double *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) float tile[kTF * kPitch];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t f0 = (int64_t)blockIdx.x * kTF;
  const int64_t a_beg = (int64_t)blockIdx.y * chunk, a_end = min(n, a_beg + chunk);
  const int64_t f = f0 + lane;
  const float *myfr = xyz + min(f, n_frames - 1) * fstride;
  const double px = myfr[0], py = myfr[1], pz = myfr[2];
  double acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = 0;
  f32x4 pre[kNPre];
  auto gload = [&](int64_t t0) {
#pragma unroll
    for (int k = 0; k < kNPre; ++k) {
      const int idx = threadIdx.x + k * kBlock;
      const int row = idx / kRow4, col = idx % kRow4;
      const int64_t fr = min(f0 + row, n_frames - 1);
      pre[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(xyz + fr * fstride + 3 * t0) + col);
    }
  };
  gload(a_beg);
  for (int64_t t0 = a_beg; t0 < a_end; t0 += kTA) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kNPre; ++k) {
      const int idx = threadIdx.x + k * kBlock;
      const int row = idx / kRow4, col = idx % kRow4;
      *reinterpret_cast<f32x4 *>(tile + row * kPitch + 4 * col) = pre[k];
    }
    __syncthreads();
    if (t0 + kTA < a_end) gload(t0 + kTA);
    const f32x4 *my = reinterpret_cast<const f32x4 *>(tile + lane * kPitch + w * 3 * kAPW);
#pragma unroll 1
    for (int g = 0; g < kAPW / 4; ++g) {
      const f32x4 q0 = my[3 * g], q1 = my[3 * g + 1], q2 = my[3 * g + 2];
      const float c[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
      const double *rr = ref + 3 * (t0 + w * kAPW + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double r0 = rr[3 * i], r1 = rr[3 * i + 1], r2 = rr[3 * i + 2];
        const double x = (double)c[3 * i] - px, y = (double)c[3 * i + 1] - py, z = (double)c[3 * i + 2] - pz;
        acc[0] += x;
        acc[1] += y;
        acc[2] += z;
        acc[6] = fma(x, r0, acc[6]);
        acc[7] = fma(x, r1, acc[7]);
        acc[8] = fma(x, r2, acc[8]);
        acc[9] = fma(y, r0, acc[9]);
        acc[10] = fma(y, r1, acc[10]);
        acc[11] = fma(y, r2, acc[11]);
        acc[12] = fma(z, r0, acc[12]);
        acc[13] = fma(z, r1, acc[13]);
        acc[14] = fma(z, r2, acc[14]);
        acc[15] = fma(x, x, fma(y, y, fma(z, z, acc[15])));
      }
    }
  }
  double t = 0;
  for (int j = 0; j < 16; ++j) t += acc[j];
  if (t == 12345.678) out[f] = t;
}

// --- tile body shared by copy<> and sk<>: tiles [a_beg, a_end) of frames f0.. --
template <bool TAIL>
__device__ __forceinline__ void tiles(const float *__restrict__ xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                      const double *__restrict__ ref, int64_t f0, int64_t a_beg, int64_t a_end,
                                      float *tile, double (&acc)[kStats], double px, double py, double pz) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t last = n_frames - 1;
  f32x4 pre[kNPre];
  const int64_t lim = 3 * n_sel;
  auto gload = [&](int64_t t0) {
#pragma unroll
    for (int k = 0; k < kNPre; ++k) {
      const int idx = threadIdx.x + k * kBlock;
      const int row = idx / kRow4, col = idx % kRow4;
      const float *src = xyz + min(f0 + row, last) * fstride;
      const int64_t e = 3 * t0 + 4 * col;
      if (!TAIL || e + 3 < lim) {
        pre[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(src + e));
      } else {
        pre[k] = f32x4{e < lim ? src[e] : 0.f, e + 1 < lim ? src[e + 1] : 0.f, e + 2 < lim ? src[e + 2] : 0.f, 0.f};
      }
    }
  };
  gload(a_beg);
  for (int64_t t0 = a_beg; t0 < a_end; t0 += kTA) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kNPre; ++k) {
      const int idx = threadIdx.x + k * kBlock;
      const int row = idx / kRow4, col = idx % kRow4;
      *reinterpret_cast<f32x4 *>(tile + row * kPitch + 4 * col) = pre[k];
    }
    __syncthreads();
    if (t0 + kTA < a_end) gload(t0 + kTA);
    const f32x4 *my = reinterpret_cast<const f32x4 *>(tile + lane * kPitch + w * 3 * kAPW);
    const int64_t ab = t0 + w * kAPW;
#pragma unroll 1
    for (int g = 0; g < kAPW / 4; ++g) {
      const int64_t a4 = ab + 4 * g;
      if (TAIL && a4 >= a_end) break;
      const f32x4 q0 = my[3 * g], q1 = my[3 * g + 1], q2 = my[3 * g + 2];
      const float c[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
      const double *rr = ref + 3 * a4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (TAIL && a4 + i >= a_end) break;
        const double r0 = rr[3 * i], r1 = rr[3 * i + 1], r2 = rr[3 * i + 2];
        const double x = (double)c[3 * i] - px, y = (double)c[3 * i + 1] - py, z = (double)c[3 * i + 2] - pz;
        acc[0] += x;
        acc[1] += y;
        acc[2] += z;
        acc[6] = fma(x, r0, acc[6]);
        acc[7] = fma(x, r1, acc[7]);
        acc[8] = fma(x, r2, acc[8]);
        acc[9] = fma(y, r0, acc[9]);
        acc[10] = fma(y, r1, acc[10]);
        acc[11] = fma(y, r2, acc[11]);
        acc[12] = fma(z, r0, acc[12]);
        acc[13] = fma(z, r1, acc[13]);
        acc[14] = fma(z, r2, acc[14]);
        acc[15] = fma(x, x, fma(y, y, fma(z, z, acc[15])));
      }
    }
  }
}

template <bool EPI>
__device__ __forceinline__ void epilogue(float *tile, double (&acc)[kStats], double *__restrict__ o_base,
                                         bool valid) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (!EPI) {
    double t = 0;
    for (int j = 0; j < kStats; ++j) t += acc[j];
    if (t == 12345.678) o_base[lane] = t;
    return;
  }
  __syncthreads();
  double *red = reinterpret_cast<double *>(tile);
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < kStats; ++j) red[((w - 1) * kStats + j) * 64 + lane] = acc[j];
  }
  __syncthreads();
  if (w == 0 && valid) {
    double *o = o_base + lane * kStats;
#pragma unroll
    for (int j = 0; j < kStats; ++j) {
      double t = acc[j];
#pragma unroll
      for (int v = 0; v < kBlock / 64 - 1; ++v) t += red[(v * kStats + j) * 64 + lane];
      o[j] = t;
    }
  }
  __syncthreads();
}

template <bool TAIL, bool EPI>
__global__ __launch_bounds__(kBlock) void copy(const float *__restrict__ xyz, int64_t fstride, int64_t n_frames,
                                               int64_t n_sel, const double *__restrict__ ref, int64_t chunk,
                                               int n_chunks, double *__restrict__ part) {
  __shared__ __attribute__((aligned(16))) float tile[kTF * kPitch];
  const int lane = threadIdx.x & 63;
  const int64_t f0 = (int64_t)blockIdx.x * kTF;
  const int64_t a_beg = (int64_t)blockIdx.y * chunk, a_end = min(n_sel, a_beg + chunk);
  const float *myfr = xyz + min(f0 + lane, n_frames - 1) * fstride;
  const double px = myfr[0], py = myfr[1], pz = myfr[2];
  double acc[kStats];
#pragma unroll
  for (int j = 0; j < kStats; ++j) acc[j] = 0.0;
  tiles<TAIL>(xyz, fstride, n_frames, n_sel, ref, f0, a_beg, a_end, tile, acc, px, py, pz);
  // partial of (frame group, chunk): 64 frames x 16 doubles
  epilogue<EPI>(tile, acc, part + ((int64_t)blockIdx.x * n_chunks + blockIdx.y) * 64 * kStats, true);
}

template <bool EPI>
__global__ __launch_bounds__(kBlock) void sk(const float *__restrict__ xyz, int64_t fstride, int64_t n_frames,
                                             int64_t n_sel, const double *__restrict__ ref, int64_t ntiles,
                                             int64_t ngroups, int G, int P, double *__restrict__ part) {
  __shared__ __attribute__((aligned(16))) float tile[kTF * kPitch];
  const int lane = threadIdx.x & 63;
  const int64_t T = ngroups * ntiles;
  const int b = blockIdx.x;
  int64_t lo = uni64(T * b / G);
  const int64_t hi = uni64(T * (b + 1) / G);
  int64_t slot = (int64_t)b * P;
  while (lo < hi) {
    const int64_t g = uni64(lo / ntiles);
    const int64_t t_lo = lo - g * ntiles;
    const int64_t t_hi = min(ntiles, t_lo + (hi - lo));
    const int64_t f0 = g * kTF;
    const float *myfr = xyz + min(f0 + lane, n_frames - 1) * fstride;
    const double px = myfr[0], py = myfr[1], pz = myfr[2];
    double acc[kStats];
#pragma unroll
    for (int j = 0; j < kStats; ++j) acc[j] = 0.0;
    tiles<true>(xyz, fstride, n_frames, n_sel, ref, f0, t_lo * kTA, min(n_sel, t_hi * kTA), tile, acc, px, py, pz);
    epilogue<EPI>(tile, acc, part + slot * 64 * kStats, true);
    lo += t_hi - t_lo;
    ++slot;
  }
}
}  // namespace ub

int main() {
  const int64_t n = 100000, nf = 20000, fs = 3 * n;
  float *x;
  double *ref, *info, *out, *part;
  CK(hipMalloc(&x, sizeof(float) * fs * nf));
  CK(hipMalloc(&ref, sizeof(double) * 3 * n));
  CK(hipMalloc(&info, sizeof(double) * RMSF_REFINFO_DOUBLES));
  CK(hipMalloc(&out, sizeof(double) * nf));
  const size_t part_bytes = (size_t)1 << 30;
  CK(hipMalloc(&part, part_bytes));
  std::vector<double> motion(12 * nf, 0.0);
  for (int64_t f = 0; f < nf; ++f) {
    motion[12 * f + 0] = motion[12 * f + 4] = motion[12 * f + 8] = 1.0;
    motion[12 * f + 9] = 0.001 * (f % 7);
  }
  double *dm;
  CK(hipMalloc(&dm, sizeof(double) * motion.size()));
  CK(hipMemcpy(dm, motion.data(), sizeof(double) * motion.size(), hipMemcpyHostToDevice));
  if (rmsf_synth_frames(x, fs, n, 0, nf, 0, dm, nullptr) || rmsf_reference_setup(x, nullptr, n, nullptr, nullptr, ref, info, nullptr)) {
    printf("setup failed: %s\n", rmsf_last_error());
    return 1;
  }
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = 12.0 * n * nf;
  auto run = [&](const char *name, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    float best = 1e9, sum = 0;
    const int R = 5;
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
    printf("%-34s %7.3f ms (min %7.3f)  %6.0f GB/s\n", name, sum / R, best, bytes / (sum / R) / 1e6);
    fflush(stdout);
  };
  const unsigned ng = (unsigned)((nf + kTF - 1) / kTF);
  const int64_t ntiles = (n + kTA - 1) / kTA;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int rep = 0; rep < 2; ++rep) {
    char nm[96];
    for (int64_t chunk : {7168, 1024}) {
      const int nch = (int)((n + chunk - 1) / chunk);
      snprintf(nm, sizeof nm, "v11 chunk=%lld", (long long)chunk);
      run(nm, [&] { hipLaunchKernelGGL(ub::v11, dim3(ng, nch), dim3(kBlock), 0, 0, x, fs, nf, n, chunk, ref, out); });
      snprintf(nm, sizeof nm, "copy<tail,epi> chunk=%lld", (long long)chunk);
      run(nm, [&] {
        hipLaunchKernelGGL((ub::copy<true, true>), dim3(ng, nch), dim3(kBlock), 0, 0, x, fs, nf, n, ref, chunk, nch, part);
      });
      snprintf(nm, sizeof nm, "copy<tail,noepi> chunk=%lld", (long long)chunk);
      run(nm, [&] {
        hipLaunchKernelGGL((ub::copy<true, false>), dim3(ng, nch), dim3(kBlock), 0, 0, x, fs, nf, n, ref, chunk, nch, part);
      });
    }
    std::vector<int> Gs = {768, 1536, 2304, 3072, 4608, 6144};
    if (getenv("UB_G")) {  // comma-separated workgroup counts
      Gs.clear();
      for (char *t = strtok(strdup(getenv("UB_G")), ","); t; t = strtok(nullptr, ",")) Gs.push_back(atoi(t));
    }
    for (int G : Gs) {
      StatsPlan pl = stats_plan(n, nf);
      pl.G = G;
      const int64_t len = (pl.T + G - 1) / G;
      pl.P = (int)((len + pl.ntiles - 1) / pl.ntiles + 1);
      if ((size_t)G * pl.P * 64 * kStats * 8 > part_bytes) continue;
      snprintf(nm, sizeof nm, "lib k_frame_stats G=%d P=%d", G, pl.P);
      run(nm, [&] {
        hipLaunchKernelGGL((k_frame_stats<false, false, true>), dim3(G), dim3(kBlock), 0, 0, x, fs, nf, n, nullptr,
                           nullptr, ref, pl, part);
      });
    }
    run("lib rmsf_superpose (default plan)", [&] {
      static double *xf = nullptr;
      if (!xf) CK(hipMalloc(&xf, sizeof(double) * RMSF_XFORM_DOUBLES * nf));
      rmsf_superpose(x, fs, nf, n, nullptr, nullptr, ref, info, xf, part, part_bytes, nullptr);
    });
    {
      const int nch = (int)((n + 7167) / 7168);
      run("welford flat (reference stream)", [&] {
        static void *acc = nullptr;
        static size_t ab = 0;
        if (!acc) {
          ab = rmsf_accumulate_balanced_workspace_bytes(n, nf, 0);
          CK(hipMalloc(&acc, ab));
        }
        rmsf_accumulate_balanced(x, fs, nf, n, nullptr, nullptr, nullptr, RMSF_MODE_WELFORD, 0, acc, ab, nullptr);
      });
      (void)nch;
    }
  }
  return 0;
}
