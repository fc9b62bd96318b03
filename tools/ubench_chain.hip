// Dependent-add latency (round 6): how fast can one wave run an in-order f64
// add chain -- the floor of wave_seq_sum's serial part (rmsf_kernels.hip).
//   1. registers only: s = s + t_i over 64 values held in VGPRs, repeated;
//   2. terms read from LDS (broadcast ds_read_b128, 16 in flight), as in
//      wave_seq_sum.
// One wave on the whole GPU; cycles from s_memtime-free HIP events.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_chain.hip -o /tmp/uch && /tmp/uch
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(64) void k_reg(double *out, int reps, double seed) {
  double t[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) t[i] = seed * (i + 1);
  double s = 0.0;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int i = 0; i < 64; ++i) s = s + t[i];
  }
  if (threadIdx.x == 0) out[0] = s;
}

__global__ __launch_bounds__(64) void k_lds(double *out, int reps, double seed) {
  __shared__ double lds[256];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = seed * (i + 1);
  __syncthreads();
  double s = 0.0;
  for (int r = 0; r < reps; ++r) {
    constexpr int G = 16;
    double ta[G], tb[G];
    auto rd = [&](double(&tt)[G], int i0) {
#pragma unroll
      for (int k = 0; k < G; ++k) tt[k] = lds[i0 + k];
    };
    auto add = [&](const double(&tt)[G]) {
#pragma unroll
      for (int k = 0; k < G; ++k) s = s + tt[k];
    };
    rd(ta, 0);
#pragma unroll
    for (int i0 = 0; i0 < 256; i0 += 2 * G) {
      rd(tb, i0 + G);
      add(ta);
      if (i0 + 2 * G < 256) rd(ta, i0 + 2 * G);
      add(tb);
    }
  }
  if (threadIdx.x == 0) out[0] = s;
}

// 3. as 2, the chain in lane 0 alone (exec = 1 lane for the reads and adds)
__global__ __launch_bounds__(64) void k_lds1(double *out, int reps, double seed) {
  __shared__ double lds[256];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = seed * (i + 1);
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int r = 0; r < reps; ++r) {
      constexpr int G = 16;
      double ta[G], tb[G];
      auto rd = [&](double(&tt)[G], int i0) {
#pragma unroll
        for (int k = 0; k < G; ++k) tt[k] = lds[i0 + k];
      };
      auto add = [&](const double(&tt)[G]) {
#pragma unroll
        for (int k = 0; k < G; ++k) s = s + tt[k];
      };
      rd(ta, 0);
#pragma unroll
      for (int i0 = 0; i0 < 256; i0 += 2 * G) {
        rd(tb, i0 + G);
        add(ta);
        if (i0 + 2 * G < 256) rd(ta, i0 + 2 * G);
        add(tb);
      }
    }
    out[0] = s;
  }
}

// 4. terms held by the lanes, read into the chain by v_readlane (two 32-bit
// halves per f64) -- no LDS round trip
__global__ __launch_bounds__(64) void k_readlane(double *out, int reps, double seed) {
  double t[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = seed * (threadIdx.x + 64 * j + 1);
  double s = 0.0;
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned long long u = __builtin_bit_cast(unsigned long long, t[j]);
      const int lo = (int)(u & 0xffffffffu), hi = (int)(u >> 32);
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const unsigned long long v = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(hi, i) << 32) |
                                     (unsigned)__builtin_amdgcn_readlane(lo, i);
        s = s + __builtin_bit_cast(double, v);
      }
    }
  }
  if (threadIdx.x == 0) out[0] = s;
}

int main() {
  double *out;
  hipMalloc(&out, 64);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int dev = 0, clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
  const int reps = 20000;
  for (int which = 0; which < 4; ++which) {
    const long adds = (long)reps * (which == 0 ? 64 : 256);
    for (int it = 0; it < 2; ++it) {
      hipEventRecord(a);
      if (which == 0)
        hipLaunchKernelGGL(k_reg, dim3(1), dim3(64), 0, 0, out, reps, 1.0000001);
      else if (which == 1)
        hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, out, reps / 4, 1.0000001);
      else if (which == 2)
        hipLaunchKernelGGL(k_lds1, dim3(1), dim3(64), 0, 0, out, reps / 4, 1.0000001);
      else
        hipLaunchKernelGGL(k_readlane, dim3(1), dim3(64), 0, 0, out, reps / 4, 1.0000001);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const long n = which == 0 ? adds : adds / 4;
      if (it)
        std::printf("%s: %ld dependent f64 adds in %.3f ms = %.2f ns per add = %.1f cycles at the %.0f MHz peak clock\n",
                    which == 0 ? "registers" : which == 1 ? "LDS terms" : which == 2 ? "LDS terms, lane 0 only" : "readlane terms", n, ms, ms * 1e6 / n, ms * 1e6 / n * clk / 1e6,
                    clk / 1e3);
    }
  }
  hipFree(out);
  return 0;
}
