// Micro-benchmark / ablation of the per-frame covariance reduction
// (k_frame_stats) on synthetic 100k atoms x 2000 frames.  Not product code.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_stats.hip -o /tmp/ubench_stats
// Variants (template V):
//   0  product-like: frame nt loads + ref (f64, L2) + 16 fp64 sums
//   1  no ref loads (r := x): tests the L2 ref stream
//   2  ref + frame, only 3 sums: tests fp64 VALU issue
//   3  frame loads only, 3 sums (pure streaming floor)
//   4  lanes-over-frames: lane = frame, wave = 16-atom slab of a 64-atom
//      tile staged through LDS; ref via scalar loads; no cross-lane reduce
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int B = 256;

template <int V>
__global__ __launch_bounds__(B) void k_rowwise(const float *__restrict__ xyz, int64_t fstride, int64_t n, const double *__restrict__ ref,
                                             double *__restrict__ out) {
  const int64_t f = blockIdx.x;
  const float *fr = xyz + f * fstride;
  const double px = fr[0], py = fr[1], pz = fr[2];
  double acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = 0;
  constexpr int U = 4;
  int64_t a = threadIdx.x;
  for (; a + (U - 1) * B < n; a += U * B) {
    float vx[U], vy[U], vz[U];
    double r0[U], r1[U], r2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t b = a + u * B;
      vx[u] = __builtin_nontemporal_load(fr + 3 * b);
      vy[u] = __builtin_nontemporal_load(fr + 3 * b + 1);
      vz[u] = __builtin_nontemporal_load(fr + 3 * b + 2);
      if (V == 0 || V == 2) {
        r0[u] = ref[3 * b];
        r1[u] = ref[3 * b + 1];
        r2[u] = ref[3 * b + 2];
      } else {
        r0[u] = vx[u];
        r1[u] = vy[u];
        r2[u] = vz[u];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double x = (double)vx[u] - px, y = (double)vy[u] - py, z = (double)vz[u] - pz;
      if (V == 2 || V == 3) {
        acc[0] = fma(x, r0[u], acc[0]);
        acc[1] = fma(y, r1[u], acc[1]);
        acc[2] = fma(z, r2[u], acc[2]);
      } else {
        acc[0] += x;
        acc[1] += y;
        acc[2] += z;
        acc[6] = fma(x, r0[u], acc[6]);
        acc[7] = fma(x, r1[u], acc[7]);
        acc[8] = fma(x, r2[u], acc[8]);
        acc[9] = fma(y, r0[u], acc[9]);
        acc[10] = fma(y, r1[u], acc[10]);
        acc[11] = fma(y, r2[u], acc[11]);
        acc[12] = fma(z, r0[u], acc[12]);
        acc[13] = fma(z, r1[u], acc[13]);
        acc[14] = fma(z, r2[u], acc[14]);
        acc[15] = fma(x, x, fma(y, y, fma(z, z, acc[15])));
      }
    }
  }
  double t = 0;
  for (int j = 0; j < 16; ++j) t += acc[j];
  // cheap sink (not a real reduction): keeps the work alive
  if (t == 12345.678) out[f] = t;
}


// V5: SoA reference (three f64 arrays, coalesced 8 B/lane loads)
// V7: f32 AoS reference (12 B/lane; bandwidth probe only)
// V8: 2 frames per lane share each AoS f64 ref load
template <int V>
__global__ __launch_bounds__(B) void k_rowwise2(const float *__restrict__ xyz, int64_t fstride, int64_t n, const double *__restrict__ ref,
                                              double *__restrict__ out) {
  constexpr int F = (V == 8) ? 2 : 1;
  const int64_t f = (int64_t)blockIdx.x * F;
  const float *fr = xyz + f * fstride;
  double acc[F][13];
  for (int q = 0; q < F; ++q)
    for (int j = 0; j < 13; ++j) acc[q][j] = 0;
  constexpr int U = (V == 8) ? 2 : 4;
  const double *rx = ref, *ry = ref + n, *rz = ref + 2 * n;
  const float *rf = reinterpret_cast<const float *>(ref);
  int64_t a = threadIdx.x;
  for (; a + (U - 1) * B < n; a += U * B) {
    float vx[F][U], vy[F][U], vz[F][U];
    double r0[U], r1[U], r2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t b = a + u * B;
#pragma unroll
      for (int q = 0; q < F; ++q) {
        vx[q][u] = __builtin_nontemporal_load(fr + q * fstride + 3 * b);
        vy[q][u] = __builtin_nontemporal_load(fr + q * fstride + 3 * b + 1);
        vz[q][u] = __builtin_nontemporal_load(fr + q * fstride + 3 * b + 2);
      }
      if (V == 5) {
        r0[u] = rx[b];
        r1[u] = ry[b];
        r2[u] = rz[b];
      } else if (V == 7) {
        r0[u] = rf[3 * b];
        r1[u] = rf[3 * b + 1];
        r2[u] = rf[3 * b + 2];
      } else {
        r0[u] = ref[3 * b];
        r1[u] = ref[3 * b + 1];
        r2[u] = ref[3 * b + 2];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int q = 0; q < F; ++q) {
        const double x = (double)vx[q][u], y = (double)vy[q][u], z = (double)vz[q][u];
        double *c = acc[q];
        c[0] += x;
        c[1] += y;
        c[2] += z;
        c[3] = fma(x, r0[u], c[3]);
        c[4] = fma(x, r1[u], c[4]);
        c[5] = fma(x, r2[u], c[5]);
        c[6] = fma(y, r0[u], c[6]);
        c[7] = fma(y, r1[u], c[7]);
        c[8] = fma(y, r2[u], c[8]);
        c[9] = fma(z, r0[u], c[9]);
        c[10] = fma(z, r1[u], c[10]);
        c[11] = fma(z, r2[u], c[11]);
        c[12] = fma(x, x, fma(y, y, fma(z, z, c[12])));
      }
    }
  }
  double t = 0;
  for (int q = 0; q < F; ++q)
    for (int j = 0; j < 13; ++j) t += acc[q][j];
  if (t == 12345.678) out[f] = t;
}

// lanes over frames.  Block = 4 waves, 64 frames; tile = 64 atoms; wave w
// handles tile atoms [16w, 16w+16) for frame (group*64 + lane).
constexpr int TF = 64, TA = 64, PITCH = TA * 3 + 1;  // dwords per LDS row (193: conflict-free b32 column reads)
__global__ __launch_bounds__(B) void k_lanes_frames(const float *__restrict__ xyz, int64_t fstride, int64_t n_frames, int64_t n,
                                                  int64_t chunk, const double *__restrict__ ref, double *__restrict__ out) {
  __shared__ float tile[TF * PITCH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t f0 = (int64_t)blockIdx.x * TF;
  const int64_t a_beg = (int64_t)blockIdx.y * chunk, a_end = min(n, a_beg + chunk);
  const int64_t f = f0 + lane;
  const bool fvalid = f < n_frames;
  const float *myfr = xyz + (fvalid ? f : f0) * fstride;
  const double px = myfr[0], py = myfr[1], pz = myfr[2];
  double acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = 0;
  for (int64_t t0 = a_beg; t0 < a_end; t0 += TA) {
    // stage: 64 rows x 192 floats = 64 x 48 float4 -> 12 float4 per thread
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const int idx = threadIdx.x + k * B;  // 0..3071
      const int row = idx / 48, col = idx % 48;
      const int64_t fr = min(f0 + row, n_frames - 1);
      const float4 v = *reinterpret_cast<const float4 *>(xyz + fr * fstride + 3 * t0 + 4 * col);
      float *d = tile + row * PITCH + 4 * col;
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
    __syncthreads();
    const float *my = tile + lane * PITCH;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int at = w * 16 + i;
      const int64_t ga = t0 + at;
      const double r0 = ref[3 * ga], r1 = ref[3 * ga + 1], r2 = ref[3 * ga + 2];  // uniform -> s_load
      const double x = (double)my[3 * at] - px, y = (double)my[3 * at + 1] - py, z = (double)my[3 * at + 2] - pz;
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
  double t = 0;
  for (int j = 0; j < 16; ++j) t += acc[j];
  if (t == 12345.678) out[f] = t;
}


// V10: lanes-over-frames, tuned.  Tile = 64 frames x TA2 atoms; LDS row
// pitch 3*TA2+4 dwords (16-B aligned rows: conflict-free ds_read_b128 column
// reads, ds_write_b128 staging); next tile prefetched into registers while the
// current one is consumed; ref wave-uniform -> scalar loads, one 4-atom group
// per iteration (bounded SGPR use).
template <int TA2, bool NOMATH = false>
__global__ __launch_bounds__(B) void k_lanes_frames2(const float *__restrict__ xyz, int64_t fstride, int64_t n_frames, int64_t n,
                                                   int64_t chunk, const double *__restrict__ ref, double *__restrict__ out) {
  constexpr int P2 = 3 * TA2 + 4;
  constexpr int ROW4 = 3 * TA2 / 4;              // float4 per row
  constexpr int NPRE = TF * ROW4 / B;            // float4 per thread per tile
  constexpr int APW = TA2 / 4;                   // atoms per wave per tile
  __shared__ __attribute__((aligned(16))) float tile[TF * P2];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t f0 = (int64_t)blockIdx.x * TF;
  const int64_t a_beg = (int64_t)blockIdx.y * chunk, a_end = min(n, a_beg + chunk);
  const int64_t f = f0 + lane;
  const float *myfr = xyz + min(f, n_frames - 1) * fstride;
  const double px = myfr[0], py = myfr[1], pz = myfr[2];
  double acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = 0;
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 pre[NPRE];
  auto gload = [&](int64_t t0) {
#pragma unroll
    for (int k = 0; k < NPRE; ++k) {
      const int idx = threadIdx.x + k * B;
      const int row = idx / ROW4, col = idx % ROW4;
      const int64_t fr = min(f0 + row, n_frames - 1);
      pre[k] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(xyz + fr * fstride + 3 * t0) + col);
    }
  };
  gload(a_beg);
  for (int64_t t0 = a_beg; t0 < a_end; t0 += TA2) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPRE; ++k) {
      const int idx = threadIdx.x + k * B;
      const int row = idx / ROW4, col = idx % ROW4;
      *reinterpret_cast<f4 *>(tile + row * P2 + 4 * col) = pre[k];
    }
    __syncthreads();
    if (t0 + TA2 < a_end) gload(t0 + TA2);
    const f4 *my = reinterpret_cast<const f4 *>(tile + lane * P2 + w * 3 * APW);
    if (NOMATH) {  // staging floor: keep one LDS read so the tile is consumed
      acc[0] += my[0].x;
      continue;
    }
#pragma unroll 1
    for (int g = 0; g < APW / 4; ++g) {
      const f4 q0 = my[3 * g], q1 = my[3 * g + 1], q2 = my[3 * g + 2];
      const float c[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
      const double *rr = ref + 3 * (t0 + w * APW + 4 * g);
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

// pseudo-random coordinates in [0, 100): real-looking bit patterns (the
// memset pattern toggles few bits -- HBM/DVFS behaviour may depend on it)
__global__ void k_fill_random(float *x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    x[i] = (float)(h & 0xffffff) * (100.0f / 16777216.0f);
  }
}

int main() {
  const bool occ = getenv("UB_SET") && getenv("UB_SET")[0] == 'O';
  const int64_t n = getenv("UB_N") ? atoll(getenv("UB_N")) : 100352, nf = occ ? 20000 : 2000, fs = 3 * n;  // n: multiple of the 64-atom tile (no tail handling in V4)
  float *x;
  double *ref, *out;
  // UB_ALIGN=<bytes>: over-allocate and start the trajectory at that
  // virtual-address alignment (placement probe); UB_SHIFT=<bytes>: plus an offset
  const size_t ub_align = getenv("UB_ALIGN") ? strtoull(getenv("UB_ALIGN"), nullptr, 0) : 0;
  const size_t ub_shift = getenv("UB_SHIFT") ? strtoull(getenv("UB_SHIFT"), nullptr, 0) : 0;
  {
    char *raw;
    CK(hipMalloc(&raw, sizeof(float) * fs * nf + ub_align + ub_shift));
    uintptr_t p = (uintptr_t)raw;
    if (ub_align) p = (p + ub_align - 1) / ub_align * ub_align;
    p += ub_shift;
    x = (float *)p;
    printf("trajectory base %p (raw %p) mod 1 GiB = %zu MiB\n", (void *)x, (void *)raw,
           (size_t)(((uintptr_t)x) % (1ull << 30)) >> 20);
  }
  CK(hipMalloc(&ref, sizeof(double) * 3 * n));
  CK(hipMalloc(&out, sizeof(double) * nf));
  CK(hipMemset(x, 0x3f, sizeof(float) * fs * nf));  // non-zero operands (DVFS)
  CK(hipMemset(ref, 0x3f, sizeof(double) * 3 * n));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double bytes = 12.0 * n * nf;
  auto run = [&](const char *name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    const int R = 10;
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= R;
    printf("%-44s %8.3f ms  %7.0f GB/s (12 B/atom-frame)\n", name, ms, bytes / ms / 1e6);
  };
  if (occ) {  // full C3 size: occupancy (blocks per CU via dynamic LDS) x chunk
    int lds_max = 0;
    CK(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0));
    const int stat = 64 * (3 * 32 + 4) * 4;
    for (int rep = 0; rep < 2; ++rep)
      for (int64_t chunk : {1024, 1888, 2048}) {
        if (rep == 1 && chunk == 1024) {
          hipLaunchKernelGGL(k_fill_random, dim3(8192), dim3(256), 0, 0, x, fs * nf);
          CK(hipDeviceSynchronize());
          printf("-- random coordinates from here on --\n");
        }
        const int64_t nchunk = (n + chunk - 1) / chunk;
        for (int k : {0, 2, 3, 4}) {
          const int dyn = k ? lds_max / k - stat - 512 : 0;
          char nm[80];
          snprintf(nm, sizeof nm, "V11 TA=32 chunk=%lld blocks/CU<=%d", (long long)chunk, k ? k : 6);
          run(nm, [&] {
            hipLaunchKernelGGL((k_lanes_frames2<32>), dim3((nf + TF - 1) / TF, nchunk), dim3(B), dyn, 0, x, fs, nf, n, chunk, ref, out);
          });
        }
        {
          char nm2[80];
          snprintf(nm2, sizeof nm2, "V10 TA=64 chunk=%lld", (long long)chunk);
          run(nm2, [&] {
            hipLaunchKernelGGL((k_lanes_frames2<64>), dim3((nf + TF - 1) / TF, nchunk), dim3(B), 0, 0, x, fs, nf, n, chunk, ref, out);
          });
          snprintf(nm2, sizeof nm2, "V12 TA=16 chunk=%lld", (long long)chunk);
          run(nm2, [&] {
            hipLaunchKernelGGL((k_lanes_frames2<16>), dim3((nf + TF - 1) / TF, nchunk), dim3(B), 0, 0, x, fs, nf, n, chunk, ref, out);
          });
        }
        char nm[80];
        snprintf(nm, sizeof nm, "V11 staging only chunk=%lld", (long long)chunk);
        run(nm, [&] {
          hipLaunchKernelGGL((k_lanes_frames2<32, true>), dim3((nf + TF - 1) / TF, nchunk), dim3(B), 0, 0, x, fs, nf, n, chunk, ref, out);
        });
      }
    return 0;
  }
  run("V0 rowwise full (nt frame + ref)", [&] { hipLaunchKernelGGL(k_rowwise<0>, dim3(nf), dim3(B), 0, 0, x, fs, n, ref, out); });
  run("V1 rowwise, no ref loads", [&] { hipLaunchKernelGGL(k_rowwise<1>, dim3(nf), dim3(B), 0, 0, x, fs, n, ref, out); });
  run("V2 rowwise, ref, 3 sums", [&] { hipLaunchKernelGGL(k_rowwise<2>, dim3(nf), dim3(B), 0, 0, x, fs, n, ref, out); });
  run("V3 rowwise, frame only, 3 sums", [&] { hipLaunchKernelGGL(k_rowwise<3>, dim3(nf), dim3(B), 0, 0, x, fs, n, ref, out); });
  run("V5 rowwise, SoA f64 ref", [&] { hipLaunchKernelGGL(k_rowwise2<5>, dim3(nf), dim3(B), 0, 0, x, fs, n, ref, out); });
  run("V7 rowwise, f32 AoS ref (probe)", [&] { hipLaunchKernelGGL(k_rowwise2<7>, dim3(nf), dim3(B), 0, 0, x, fs, n, ref, out); });
  run("V8 rowwise, 2 frames/lane share ref", [&] { hipLaunchKernelGGL(k_rowwise2<8>, dim3(nf / 2), dim3(B), 0, 0, x, fs, n, ref, out); });
  run("V9 rowwise2<0> AoS f64 ref (control)", [&] { hipLaunchKernelGGL(k_rowwise2<0>, dim3(nf), dim3(B), 0, 0, x, fs, n, ref, out); });
  for (int64_t chunk : {512, 1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "V10 lanes-over-frames TA=64 chunk=%lld", (long long)chunk);
    const int64_t nchunk = (n + chunk - 1) / chunk;
    run(nm, [&] {
      hipLaunchKernelGGL(k_lanes_frames2<64>, dim3((nf + TF - 1) / TF, nchunk), dim3(B), 0, 0, x, fs, nf, n, chunk, ref, out);
    });
    snprintf(nm, sizeof nm, "V11 lanes-over-frames TA=32 chunk=%lld", (long long)chunk);
    run(nm, [&] {
      hipLaunchKernelGGL(k_lanes_frames2<32>, dim3((nf + TF - 1) / TF, nchunk), dim3(B), 0, 0, x, fs, nf, n, chunk, ref, out);
    });
  }
  for (int64_t chunk : {1024, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "V4 lanes-over-frames chunk=%lld", (long long)chunk);
    const int64_t nchunk = (n + chunk - 1) / chunk;
    run(nm, [&] {
      hipLaunchKernelGGL(k_lanes_frames, dim3((nf + TF - 1) / TF, nchunk), dim3(B), 0, 0, x, fs, nf, n, chunk, ref, out);
    });
  }
  return 0;
}
