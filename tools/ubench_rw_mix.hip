// Read stream with a small write stream mixed in (round 6): what do writes
// of ~10 % of the read bytes cost beside a saturating HBM read stream?  The
// sparse-selection compaction writes 2.43 GB beside a 24 GB gathered read
// and costs 1.4-1.8 ms, where the bytes alone would take 0.4 ms
// (DESIGN section 4 "Sparse selections").  Each thread sums float4 over a
// grid-stride read of A (nontemporal loads); with W > 0 every W-th float4
// read is also written to B (nontemporal stores, contiguous), so B gets
// 1/W of A's bytes.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_rw_mix.hip -o /tmp/urw && /tmp/urw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int W>
__global__ __launch_bounds__(256) void k_rw(const f4 *__restrict__ a, f4 *__restrict__ b, long n4, float *out) {
  f4 acc = {0, 0, 0, 0};
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    const f4 v = __builtin_nontemporal_load(a + i);
    acc += v;
    if constexpr (W > 0) {
      if (i % W == 0) __builtin_nontemporal_store(v, b + i / W);
    }
  }
  if (acc.x == 1234.5f) out[0] = acc.y;
}

int main() {
  const long bytes = 12L << 30;  // 12 GiB read
  const long n4 = bytes / 16;
  f4 *a, *b;
  float *out;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes / 4) != hipSuccess || hipMalloc(&out, 64) != hipSuccess)
    return 1;
  (void)hipMemset(a, 0x3f, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const dim3 grid(256 * 32), blk(256);
  for (int w : {0, 40, 20, 10, 5}) {
    auto launch = [&]() {
      switch (w) {
        case 0: hipLaunchKernelGGL(k_rw<0>, grid, blk, 0, 0, a, b, n4, out); break;
        case 40: hipLaunchKernelGGL(k_rw<40>, grid, blk, 0, 0, a, b, n4, out); break;
        case 20: hipLaunchKernelGGL(k_rw<20>, grid, blk, 0, 0, a, b, n4, out); break;
        case 10: hipLaunchKernelGGL(k_rw<10>, grid, blk, 0, 0, a, b, n4, out); break;
        default: hipLaunchKernelGGL(k_rw<5>, grid, blk, 0, 0, a, b, n4, out); break;
      }
    };
    launch();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    const double wb = w ? (double)bytes / w : 0.0;
    std::printf("read 12 GiB%s: %.3f ms  (read %.0f GB/s, read+write %.0f GB/s)\n",
                w ? (std::string(" + write 1/") + std::to_string(w)).c_str() : "", best, bytes / (best * 1e6),
                (bytes + wb) / (best * 1e6));
  }
  return 0;
}
