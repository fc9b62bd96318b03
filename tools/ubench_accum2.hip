// The aligned accumulator (RMSF.py:99-103 / 133-138: f32-faithful transform
// + f64 statistics) as built in the library (k_accum_atoms_sk: one atom per
// lane, global_load_dwordx3 per frame) against a candidate that stages
// frame tiles through LDS with float4 loads -- the staging that brought the
// superposition sums to ~1.02x the Welford stream -- and reads lane = atom
// from LDS.  C3 shape (100k atoms x 20k frames), same process.  Not product
// code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_accum2.hip -o tools/ubench_accum2
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
using ::f32x4;

// tile = TF frames x 64 atoms (192 floats = 48 float4 per row), staged with
// float4 loads (next tile in flight); wave w takes rows w*TF/4 .. of every
// tile, lane = atom; shifted sums with one shift per segment (the segment's
// first frame after the transform) so the waves' sums add.
constexpr int kA = 64;               // atoms per chunk
constexpr int kRowF = 3 * kA;        // floats per tile row
constexpr int kRowP = kRowF + 4;     // LDS row pitch
constexpr int kRow4 = kRowF / 4;     // float4 per row

template <int MODE, int TF>
__global__ __launch_bounds__(kBlock) void accum_tiles(const float *__restrict__ xyz, int64_t fstride,
                                                      const double *__restrict__ xform,
                                                      const double *__restrict__ refinfo, SkPlan pl,
                                                      int64_t n_sel, int64_t *__restrict__ hdr,
                                                      double *__restrict__ parts0, double *__restrict__ parts1) {
  constexpr int NPRE = TF * kRow4 / kBlock;
  constexpr int RPW = TF / 4;  // rows per wave
  __shared__ __attribute__((aligned(16))) float tile[TF * kRowP];
  const int b = sk_range(pl, blockIdx.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) sk_write_header(hdr, pl);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double rc0 = refinfo[0], rc1 = refinfo[1], rc2 = refinfo[2];
  const int64_t lim = 3 * n_sel;
  int64_t lo = uni64(sk_lo(pl, b));
  const int64_t hi = uni64(sk_lo(pl, b + 1));
  int64_t slot = (int64_t)b * pl.P;
  while (lo < hi) {
    int64_t c, f0;
    const int len = __builtin_amdgcn_readfirstlane((int)sk_seg_len(pl, lo, hi, &c, &f0));
    c = uni64(c);
    f0 = uni64(f0);
    const int64_t e0 = 3 * c * kA, fend = f0 + len;
    f32x4 pre[NPRE];
    auto gload = [&](int64_t t0) {
#pragma unroll
      for (int k = 0; k < NPRE; ++k) {
        const int idx = threadIdx.x + k * kBlock;
        const int row = idx / kRow4, col = idx % kRow4;
        const float *src = xyz + min(t0 + row, fend - 1) * fstride;
        const int64_t e = e0 + 4 * col;
        if (e + 3 < lim) {
          pre[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(src + e));
        } else {
          pre[k] = f32x4{e < lim ? src[e] : 0.f, e + 1 < lim ? src[e + 1] : 0.f, e + 2 < lim ? src[e + 2] : 0.f, 0.f};
        }
      }
    };
    double m[3] = {0, 0, 0}, q[3] = {0, 0, 0}, sh[3] = {0, 0, 0};
    gload(f0);
    for (int64_t t0 = f0; t0 < fend; t0 += TF) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < NPRE; ++k) {
        const int idx = threadIdx.x + k * kBlock;
        const int row = idx / kRow4, col = idx % kRow4;
        *reinterpret_cast<f32x4 *>(tile + row * kRowP + 4 * col) = pre[k];
      }
      __syncthreads();
      if (t0 + TF < fend) gload(t0 + TF);
      if (MODE == RMSF_MODE_WELFORD && t0 == f0) {  // the shift: frame f0 transformed (every wave)
        float x = tile[3 * lane], y = tile[3 * lane + 1], z = tile[3 * lane + 2];
        apply_xform(x, y, z, xform + f0 * kXform, rc0, rc1, rc2);
        sh[0] = (double)x, sh[1] = (double)y, sh[2] = (double)z;
      }
      const int nfr = (int)min((int64_t)TF, fend - t0);
      const int r0 = w * RPW;
#pragma unroll 2
      for (int j = 0; j < RPW; ++j) {
        const int r = r0 + j;
        if (r >= nfr) break;  // uniform
        float x = tile[r * kRowP + 3 * lane], y = tile[r * kRowP + 3 * lane + 1], z = tile[r * kRowP + 3 * lane + 2];
        apply_xform(x, y, z, xform + (t0 + r) * kXform, rc0, rc1, rc2);
        if (MODE == RMSF_MODE_WELFORD) {
          const double d0 = (double)x - sh[0], d1 = (double)y - sh[1], d2 = (double)z - sh[2];
          m[0] += d0, m[1] += d1, m[2] += d2;
          q[0] = fma(d0, d0, q[0]), q[1] = fma(d1, d1, q[1]), q[2] = fma(d2, d2, q[2]);
        } else {
          m[0] += (double)x, m[1] += (double)y, m[2] += (double)z;
        }
      }
    }
    // fold the waves (same shift), convert, store the segment's partial
    __syncthreads();
    double *red = reinterpret_cast<double *>(tile);  // [6][4][64]
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      red[(k * 4 + w) * 64 + lane] = m[k];
      red[((3 + k) * 4 + w) * 64 + lane] = q[k];
    }
    __syncthreads();
    if (w == 0 && c * kA + lane < n_sel) {
      const double inv = g_coef.v[len - 1].b;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        double a = red[(k * 4) * 64 + lane], qq = red[((3 + k) * 4) * 64 + lane];
#pragma unroll
        for (int v = 1; v < 4; ++v) {
          a += red[(k * 4 + v) * 64 + lane];
          qq += red[((3 + k) * 4 + v) * 64 + lane];
        }
        if (MODE == RMSF_MODE_WELFORD) shifted_to_moments(a, qq, sh[k], inv);
        const int64_t o = slot * (kA * 3) + 3 * lane + k;
        __builtin_nontemporal_store(a, parts0 + o);
        if (MODE == RMSF_MODE_WELFORD) __builtin_nontemporal_store(qq, parts1 + o);
      }
    }
    lo += len;
    ++slot;
  }
}
}  // namespace ub

int main() {
  const int64_t n = 100000, nf = 20000, fs = 3 * n;
  float *x;
  double *ref, *info, *xf, *out0, *out1;
  CK(hipMalloc(&x, sizeof(float) * fs * nf));
  CK(hipMalloc(&ref, sizeof(double) * 3 * n));
  CK(hipMalloc(&info, sizeof(double) * RMSF_REFINFO_DOUBLES));
  CK(hipMalloc(&xf, sizeof(double) * RMSF_XFORM_DOUBLES * nf));
  CK(hipMalloc(&out0, sizeof(double) * fs));
  CK(hipMalloc(&out1, sizeof(double) * fs));
  std::vector<double> motion(12 * nf, 0.0);
  for (int64_t f = 0; f < nf; ++f) {  // small rotations about z + shifts: realistic R
    const double a = 0.01 * (f % 97);
    motion[12 * f + 0] = std::cos(a), motion[12 * f + 1] = -std::sin(a);
    motion[12 * f + 3] = std::sin(a), motion[12 * f + 4] = std::cos(a);
    motion[12 * f + 8] = 1.0;
    motion[12 * f + 9] = 50.0 + 0.001 * (f % 7), motion[12 * f + 10] = 50.0, motion[12 * f + 11] = 50.0;
  }
  double *dm;
  CK(hipMalloc(&dm, sizeof(double) * motion.size()));
  CK(hipMemcpy(dm, motion.data(), sizeof(double) * motion.size(), hipMemcpyHostToDevice));
  const size_t wb = rmsf_superpose_workspace_bytes(n, nf);
  void *work;
  CK(hipMalloc(&work, wb));
  if (rmsf_synth_frames(x, fs, n, 0, nf, 0, dm, nullptr) ||
      rmsf_reference_setup(x, nullptr, n, nullptr, nullptr, ref, info, nullptr) ||
      rmsf_superpose(x, fs, nf, n, nullptr, nullptr, ref, info, xf, work, wb, nullptr)) {
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
    printf("%-44s %7.3f ms (min %7.3f)  %6.0f GB/s\n", name, sum / R, best, bytes / (sum / R) / 1e6);
    fflush(stdout);
  };
  auto lib = [&](int mode) {
    rmsf_accumulate_balanced(x, fs, nf, n, nullptr, xf, info, mode, 0, acc, ab, nullptr);
  };
  auto tiles = [&](int mode, int groups, auto tf) {  // groups 0 = the library's auto plan at 32/CU
    constexpr int TF = decltype(tf)::value;
    SkPlan pl = sk_plan(n, 3, nf, groups, mode, kSkPerCuAligned, ub::kA);
    int64_t *hdr = static_cast<int64_t *>(acc);
    double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
    double *p1 = p0 + (size_t)pl.G * pl.P * ub::kA * 3;
    if (mode == RMSF_MODE_WELFORD)
      hipLaunchKernelGGL((ub::accum_tiles<RMSF_MODE_WELFORD, TF>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs, xf, info,
                         pl, n, hdr, p0, p1);
    else
      hipLaunchKernelGGL((ub::accum_tiles<RMSF_MODE_SUM, TF>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs, xf, info, pl,
                         n, hdr, p0, p1);
  };
  using T32 = std::integral_constant<int, 32>;
  using T16 = std::integral_constant<int, 16>;
  {  // agreement with the library (different fold orders: rounding only)
    std::vector<double> a0(fs), q0(fs), a1(fs), q1(fs);
    lib(RMSF_MODE_WELFORD);
    rmsf_fold_balanced(acc, fs, RMSF_MODE_WELFORD, 0, out0, out1, nullptr);
    CK(hipMemcpy(a0.data(), out0, 8 * fs, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q0.data(), out1, 8 * fs, hipMemcpyDeviceToHost));
    tiles(RMSF_MODE_WELFORD, 3072, T32{});
    rmsf_fold_balanced(acc, fs, RMSF_MODE_WELFORD, 0, out0, out1, nullptr);
    CK(hipMemcpy(a1.data(), out0, 8 * fs, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q1.data(), out1, 8 * fs, hipMemcpyDeviceToHost));
    double dm = 0, dq = 0;
    for (int64_t i = 0; i < fs; ++i) {
      dm = std::max(dm, std::fabs(a0[i] - a1[i]));
      dq = std::max(dq, std::fabs(q0[i] - q1[i]) / std::max(1.0, std::fabs(q0[i])));
    }
    printf("tiles vs library (aligned Welford): max |d mean| %.3e A, max rel |d M2| %.3e\n", dm, dq);
  }
  // the library kernel's knobs: grid size and frame unroll
  auto atoms = [&](int mode, int groups, auto u) {
    constexpr int U = decltype(u)::value;
    SkPlan pl = sk_plan(n, 3, nf, groups, mode, kSkPerCuAligned);
    int64_t *hdr = static_cast<int64_t *>(acc);
    double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
    double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 3;
    if (mode == RMSF_MODE_WELFORD)
      hipLaunchKernelGGL((k_accum_atoms_sk<RMSF_MODE_WELFORD, true, false, U>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs,
                         nullptr, xf, info, pl, hdr, p0, p1);
    else
      hipLaunchKernelGGL((k_accum_atoms_sk<RMSF_MODE_SUM, true, false, U>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs,
                         nullptr, xf, info, pl, hdr, p0, p1);
  };
  using U2 = std::integral_constant<int, 2>;
  using U4 = std::integral_constant<int, 4>;
  using U8 = std::integral_constant<int, 8>;
  for (int rep = 0; rep < 2; ++rep) {
    run("lib k_accum_atoms_sk<WELFORD,ALIGN>", [&] { lib(RMSF_MODE_WELFORD); });
    run("lib k_accum_atoms_sk<SUM,ALIGN>", [&] { lib(RMSF_MODE_SUM); });
    run("lib welford flat (stream reference)", [&] {
      rmsf_accumulate_balanced(x, fs, nf, n, nullptr, nullptr, nullptr, RMSF_MODE_WELFORD, 0, acc, ab, nullptr);
    });
    char nm[96];
    for (int groups : {0, 4096, 6144}) {
      snprintf(nm, sizeof nm, "atoms U=8 WELFORD G=%d", groups);
      run(nm, [&] { atoms(RMSF_MODE_WELFORD, groups, U8{}); });
      snprintf(nm, sizeof nm, "atoms U=4 WELFORD G=%d", groups);
      run(nm, [&] { atoms(RMSF_MODE_WELFORD, groups, U4{}); });
      snprintf(nm, sizeof nm, "atoms U=8 SUM G=%d", groups);
      run(nm, [&] { atoms(RMSF_MODE_SUM, groups, U8{}); });
    }
  }
  return 0;
}
