// The in-order f64 add chain of wave_seq_sum (rmsf_kernels.hip), measured
// as the product runs it (round 6, second study): one wave per chain, its
// 1,024 terms parked in the wave's LDS slice, W waves per CU at once.  The
// first study (ubench_chain.hip) let the compiler hoist the LDS reads out of
// the repeat loop into AGPRs, so its "LDS terms" figure timed AGPR copies;
// here a compiler barrier per block keeps the reads in the loop.
//   V0  the product's form: all 64 lanes read each 16-term group (broadcast
//       ds_read_b128), the next group's reads in flight while one is added;
//   V1  as V0, the reads D groups ahead, pinned by sched_barrier;
//   V2  as V1, the chain in lane 0 alone (exec = 1 lane: each read returns
//       16 B instead of 1 KiB);
//   V3  registers only (the floor): the same adds over values already held;
//   V4  the chain in every lane at once, each 16-lane row holding 16 terms
//       per register pair (lane l of a row: terms 2l, 2l + 1 of a 32-term
//       group, one ds_read_b128 per lane), each add a v_fmac_f64 by 1.0 of
//       the term broadcast from lane j of the row (DPP row_newbcast:j) --
//       fma(t, 1.0, s) rounds once, as s + t does, so the bits are the add's;
//   V5  as V4, each group's 32 adds in one asm statement opening with s_nop 1
//       (a term just written by a VALU needs 2 wait states before a DPP
//       read), with D - 1 = 0 or 1 s_nop 0 between consecutive adds: the
//       accumulator's own hazard measured (a stale read would lose an add
//       and change the printed sum).
// Prints ns per add per chain for W = 1, 2, 4, 8 waves per CU.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_chain2.hip -o /tmp/uch2 && /tmp/uch2
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kBlk = 1024, G = 16, NG = kBlk / G;

template <int V, int D>
__global__ __launch_bounds__(64) void k_chain(double *out, int reps, double seed) {
  __shared__ double lds[kBlk];
  const int lane = threadIdx.x;
  for (int i = lane; i < kBlk; i += 64) lds[i] = seed * (i + 1);
  __syncthreads();
  double s = 0.0;
  auto rd = [&](double(&t)[G], int i0) {
#pragma unroll
    for (int k = 0; k < G; ++k) t[k] = lds[i0 + k];
  };
  auto add = [&](const double(&t)[G]) {
#pragma unroll
    for (int k = 0; k < G; ++k) s = s + t[k];
  };
  if constexpr (V == 5) {
    double one = 1.0;
    asm volatile("" : "+v"(one));
    for (int r = 0; r < reps; ++r) {
      asm volatile("" ::: "memory");
      constexpr int NG2 = kBlk / 32;
      double2 t[3];
      const double2 *l2 = reinterpret_cast<const double2 *>(lds) + (lane & 15);
#pragma unroll
      for (int g = 0; g < 2; ++g) t[g] = l2[16 * g];
#pragma unroll
      for (int g = 0; g < NG2; ++g) {
        if (g + 2 < NG2) t[(g + 2) % 3] = l2[16 * (g + 2)];
        __builtin_amdgcn_sched_barrier(0);
        const double2 &u = t[g % 3];
#define RMSF_X(J, R) "v_fmac_f64_dpp %0, %" #R ", %3 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n" NOP
#define RMSF_XY(J) RMSF_X(J, 1) RMSF_X(J, 2)
#define RMSF_ROW32                                                                                           \
  asm volatile("s_nop 1\n" RMSF_XY(0) RMSF_XY(1) RMSF_XY(2) RMSF_XY(3) RMSF_XY(4) RMSF_XY(5) RMSF_XY(6)      \
               RMSF_XY(7) RMSF_XY(8) RMSF_XY(9) RMSF_XY(10) RMSF_XY(11) RMSF_XY(12) RMSF_XY(13) RMSF_XY(14)  \
               RMSF_XY(15)                                                                                   \
               : "+v"(s) : "v"(u.x), "v"(u.y), "v"(one));
        if constexpr (D == 1) {
#define NOP ""
          RMSF_ROW32
#undef NOP
        } else {
#define NOP "s_nop 0\n"
          RMSF_ROW32
#undef NOP
        }
#undef RMSF_ROW32
#undef RMSF_XY
#undef RMSF_X
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else if constexpr (V == 4) {
    double one = 1.0;
    asm volatile("" : "+v"(one));
    for (int r = 0; r < reps; ++r) {
      asm volatile("" ::: "memory");
      constexpr int NG2 = kBlk / 32;
      double2 t[D + 1];
      const double2 *l2 = reinterpret_cast<const double2 *>(lds) + (lane & 15);
#pragma unroll
      for (int g = 0; g < D; ++g) t[g] = l2[16 * g];
#pragma unroll
      for (int g = 0; g < NG2; ++g) {
        if (g + D < NG2) t[(g + D) % (D + 1)] = l2[16 * (g + D)];
        __builtin_amdgcn_sched_barrier(0);
        const double2 &u = t[g % (D + 1)];
#define RMSF_FMAC_BCAST(J)                                                                                 \
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(s)      \
               : "v"(u.x), "v"(one));                                                                     \
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(s)      \
               : "v"(u.y), "v"(one));
        RMSF_FMAC_BCAST(0) RMSF_FMAC_BCAST(1) RMSF_FMAC_BCAST(2) RMSF_FMAC_BCAST(3)
        RMSF_FMAC_BCAST(4) RMSF_FMAC_BCAST(5) RMSF_FMAC_BCAST(6) RMSF_FMAC_BCAST(7)
        RMSF_FMAC_BCAST(8) RMSF_FMAC_BCAST(9) RMSF_FMAC_BCAST(10) RMSF_FMAC_BCAST(11)
        RMSF_FMAC_BCAST(12) RMSF_FMAC_BCAST(13) RMSF_FMAC_BCAST(14) RMSF_FMAC_BCAST(15)
#undef RMSF_FMAC_BCAST
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else if constexpr (V == 3) {
    double t[G];
    rd(t, 0);
    for (int r = 0; r < reps; ++r) {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
#pragma unroll
        for (int k = 0; k < G; ++k) asm volatile("" : "+v"(t[k]));
        add(t);
      }
    }
  } else if constexpr (V == 0) {
    for (int r = 0; r < reps; ++r) {
      asm volatile("" ::: "memory");
      double ta[G], tb[G];
      rd(ta, 0);
#pragma unroll
      for (int i0 = 0; i0 < kBlk; i0 += 2 * G) {
        rd(tb, i0 + G);
        add(ta);
        if (i0 + 2 * G < kBlk) rd(ta, i0 + 2 * G);
        add(tb);
      }
    }
  } else {
    if (V == 2 && lane != 0) return;
    for (int r = 0; r < reps; ++r) {
      asm volatile("" ::: "memory");
      double t[D + 1][G];
#pragma unroll
      for (int g = 0; g < D; ++g) rd(t[g], g * G);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if (g + D < NG) rd(t[(g + D) % (D + 1)], (g + D) * G);
        __builtin_amdgcn_sched_barrier(0);
        add(t[g % (D + 1)]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  if (lane == 0) out[blockIdx.x] = s;
}

template <int V, int D>
void run(const char *name, double *out, hipEvent_t a, hipEvent_t b) {
  const int reps = 200;
  for (int w : {1, 2, 4, 8}) {
    const dim3 grid(256 * w);
    float best = 1e30f;
    for (int it = 0; it < 3; ++it) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL((k_chain<V, D>), grid, dim3(64), 0, 0, out, reps, 1.0000001);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (it && ms < best) best = ms;
    }
    double h;
    (void)hipMemcpy(&h, out, sizeof h, hipMemcpyDeviceToHost);
    std::printf("%-44s W=%d per CU: %.2f ns per add per chain  (sum %a)\n", name, w, best * 1e6 / ((double)reps * kBlk), h);
  }
}

int main() {
  double *out;
  (void)hipMalloc(&out, 256 * 8 * 8 * sizeof(double));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  run<3, 1>("V3 registers (floor)", out, a, b);
  run<0, 1>("V0 product: 64 lanes, next group in flight", out, a, b);
  run<1, 2>("V1 64 lanes, 2 groups ahead, pinned", out, a, b);
  run<1, 3>("V1 64 lanes, 3 groups ahead, pinned", out, a, b);
  run<2, 1>("V2 lane 0, 1 group ahead, pinned", out, a, b);
  run<2, 2>("V2 lane 0, 2 groups ahead, pinned", out, a, b);
  run<2, 3>("V2 lane 0, 3 groups ahead, pinned", out, a, b);
  run<4, 1>("V4 DPP broadcast fmac, 1 group ahead", out, a, b);
  run<4, 2>("V4 DPP broadcast fmac, 2 groups ahead", out, a, b);
  run<4, 3>("V4 DPP broadcast fmac, 3 groups ahead", out, a, b);
  run<5, 1>("V5 32 adds per asm, no nop between", out, a, b);
  run<5, 2>("V5 32 adds per asm, s_nop 0 between", out, a, b);
  (void)hipFree(out);
  return 0;
}
