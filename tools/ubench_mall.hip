// Read bandwidth vs working-set size (L2 / Infinity Cache / HBM) for
// coalesced float4 streaming reads.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_read(const f4 *__restrict__ x, int64_t n4, float *out) {
  f4 acc = {0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) acc += x[i];
  if (acc.x == 1234.5f) out[0] = acc.y;
}
int main() {
  const size_t maxb = (size_t)2 << 30;
  f4 *x; float *out;
  hipMalloc(&x, maxb); hipMalloc(&out, 64); hipMemset(x, 0x3f, maxb);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (size_t mb : {16, 64, 128, 192, 256, 384, 512, 2048}) {
    const int64_t n4 = mb * (1 << 20) / 16;
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_read, dim3(8192), dim3(256), 0, 0, x, n4, out);
    hipDeviceSynchronize();
    const int R = 20;
    hipEventRecord(a);
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL(k_read, dim3(8192), dim3(256), 0, 0, x, n4, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ms /= R;
    printf("working set %5zu MB: %.4f ms  %7.0f GB/s\n", mb, ms, mb * 1048576.0 / ms / 1e6);
  }
  return 0;
}
