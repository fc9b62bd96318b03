// Gathered-read micro-benchmark (round 6): does the cache policy of a sparse
// gather change the L2's fetch size from memory?  Each selected atom's row
// costs a whole 128-B line at 1 in 10 or sparser (DESIGN section 4 "Sparse
// selections"); a 64-B or 32-B fetch would cut that traffic.  One thread per
// (selected atom, frame split) sums its atom's coordinates over its frames
// with one load flavour:
//   0 plain global loads, 1 nontemporal global loads,
//   2.. raw buffer loads with cache-policy bits aux (gfx94x/gfx950: sc0 = 1,
//   nt = 2, sc1 = 16).
// Run plain for times, and under rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum
// TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum for the fetch sizes.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_gather_policy.hip -o /tmp/ugp
//   /tmp/ugp [stride] [n_frames]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

constexpr int kSplits = 64;

template <int P>
__global__ __launch_bounds__(256) void k_gather(const float *__restrict__ xyz, int64_t fstride, int64_t nf,
                                                int64_t n_sel, const int32_t *__restrict__ sel,
                                                float *__restrict__ out) {
  const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (a >= n_sel) return;
  const int64_t f0 = nf * blockIdx.y / kSplits, f1 = nf * (blockIdx.y + 1) / kSplits;
  const uint32_t off = 12u * (uint32_t)sel[a];
  float sx = 0.f, sy = 0.f, sz = 0.f;
#pragma unroll 4
  for (int64_t f = f0; f < f1; ++f) {
    const float *row = xyz + f * fstride;
    float x, y, z;
    if constexpr (P == 0) {
      const float *p = row + off / 4;
      x = p[0], y = p[1], z = p[2];
    } else if constexpr (P == 1) {
      const float *p = row + off / 4;
      x = __builtin_nontemporal_load(p), y = __builtin_nontemporal_load(p + 1), z = __builtin_nontemporal_load(p + 2);
    } else {
      constexpr int aux = P == 2 ? 0 : P == 3 ? 1 : P == 4 ? 2 : P == 5 ? 16 : P == 6 ? 17 : 3;
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(row), 0, (int)(4 * fstride), 0x00020000);
      x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, aux));
      y = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off + 4, 0, aux));
      z = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off + 8, 0, aux));
    }
    sx += x, sy += y, sz += z;
  }
  float *o = out + 3 * (blockIdx.y * n_sel + a);
  o[0] = sx, o[1] = sy, o[2] = sz;
}

__global__ void k_fill(float *p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (float)(i % 1000) * 0.01f;
}

int main(int argc, char **argv) {
  const int stride = argc > 1 ? std::atoi(argv[1]) : 10;
  const int64_t nf = argc > 2 ? std::atoll(argv[2]) : 4000;
  const int64_t n_atoms = 100000, fstride = 3 * n_atoms;
  const int64_t n_sel = (n_atoms + stride - 1) / stride;
  float *xyz, *out;
  int32_t *sel;
  CHECK(hipMalloc(&xyz, sizeof(float) * fstride * nf));
  CHECK(hipMalloc(&out, sizeof(float) * 3 * n_sel * kSplits));
  CHECK(hipMalloc(&sel, sizeof(int32_t) * n_sel));
  std::vector<int32_t> h(n_sel);
  for (int64_t i = 0; i < n_sel; ++i) h[i] = (int32_t)(i * stride);
  CHECK(hipMemcpy(sel, h.data(), sizeof(int32_t) * n_sel, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, xyz, fstride * nf);
  CHECK(hipDeviceSynchronize());
  const dim3 grid((unsigned)((n_sel + 255) / 256), kSplits);
  const char *names[] = {"plain", "nontemporal", "buffer aux=0", "buffer sc0", "buffer nt", "buffer sc1",
                         "buffer sc0|sc1", "buffer sc0|nt"};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double lines = (double)nf * n_sel * 128.0;  // one line per selected atom per frame (stride >= 11)
  for (int p = 0; p < 8; ++p) {
    auto launch = [&]() {
      switch (p) {
        case 0: hipLaunchKernelGGL(k_gather<0>, grid, dim3(256), 0, 0, xyz, fstride, nf, n_sel, sel, out); break;
        case 1: hipLaunchKernelGGL(k_gather<1>, grid, dim3(256), 0, 0, xyz, fstride, nf, n_sel, sel, out); break;
        case 2: hipLaunchKernelGGL(k_gather<2>, grid, dim3(256), 0, 0, xyz, fstride, nf, n_sel, sel, out); break;
        case 3: hipLaunchKernelGGL(k_gather<3>, grid, dim3(256), 0, 0, xyz, fstride, nf, n_sel, sel, out); break;
        case 4: hipLaunchKernelGGL(k_gather<4>, grid, dim3(256), 0, 0, xyz, fstride, nf, n_sel, sel, out); break;
        case 5: hipLaunchKernelGGL(k_gather<5>, grid, dim3(256), 0, 0, xyz, fstride, nf, n_sel, sel, out); break;
        case 6: hipLaunchKernelGGL(k_gather<6>, grid, dim3(256), 0, 0, xyz, fstride, nf, n_sel, sel, out); break;
        default: hipLaunchKernelGGL(k_gather<7>, grid, dim3(256), 0, 0, xyz, fstride, nf, n_sel, sel, out); break;
      }
    };
    launch();
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    std::printf("1 in %d, %ld frames, %-15s: %8.3f ms  (%6.0f GB/s of 128-B lines, %6.0f GB/s selected)\n", stride,
                (long)nf, names[p], best, lines / (best * 1e6), 12.0 * nf * n_sel / (best * 1e6));
  }
  CHECK(hipFree(xyz));
  CHECK(hipFree(out));
  CHECK(hipFree(sel));
  return 0;
}
