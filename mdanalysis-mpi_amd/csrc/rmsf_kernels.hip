// rmsf_kernels.hip -- hand-written HIP kernels for gfx950 (MI355X, CDNA4) and
// the extern "C" launchers declared in include/rmsf_hip.h.
//
// Hot path of /root/reference/RMSF.py (cited as RMSF.py:N):
//   * k_welford_flat     RMSF.py:137-138, no alignment, contiguous selection.
//                        HBM-bound stream: 12 B per atom-frame, one float4 per
//                        lane per frame, fp64 mean/M2 in registers across a
//                        frame tile (split).
//   * k_accum_atoms      RMSF.py:99-103 (SUM) and RMSF.py:133-138 (WELFORD)
//                        with the f32-faithful superposition transform; one
//                        atom (12 B, global_load_dwordx3) per lane per frame.
//   * k_frame_stats      per-(frame, atom chunk) reduction of the mobile COM
//                        and the qcprot inner product (RMSF.py:94-97,127-131).
//   * k_qcp_frames       per-frame QCP (qcprot FastCalcRMSDAndRotation, the
//                        published Theobald/Liu algorithm), one wave per frame.
//   * k_ref_com/center/finish  RMSF.py:80-87 / 113-118 reference centring.
//   * k_chan_merge       second_order_moments, RMSF.py:36-41.
//   * k_finalize         RMSF.py:146.
//   * k_synth            counter-based synthetic trajectory generator.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "rmsf_hip.h"
#include "rmsf_device.h"

#define RMSF_EXPORT __attribute__((visibility("default")))
#ifndef RMSF_SHIFTED_SUMS
#define RMSF_SHIFTED_SUMS 1  // per-frame statistics as shifted sums (0: Welford updates, for A/B)
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

int hip_fail(const char *what, hipError_t e) {
  return fail(RMSF_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                  \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hip_fail(#expr, e_);  \
  } while (0)

int after_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(what, e);
  return RMSF_OK;
}

inline hipStream_t S(void *stream) { return reinterpret_cast<hipStream_t>(stream); }

constexpr int kBlock = 256;
constexpr int kXform = RMSF_XFORM_DOUBLES;
constexpr int kStats = 16;       // doubles per (frame, chunk) partial
constexpr int64_t kAccumBlocks = 3584;       // target workgroups, k_welford_flat
constexpr int64_t kAccumBlocksAtom = 4608;   // target workgroups, k_accum_atoms
constexpr int64_t kStatsGroups = 3072;  // k_frame_stats workgroups at most (balanced grid; 4 rounds of 3 per CU on MI355X)
constexpr int64_t kStatsRound = 768;    // ... in whole rounds of this many (3 resident per CU x 256 CUs)
constexpr int64_t kStatsRoundUnits = 768 * 160;  // ... one round per this many (64-frame, 32-atom) units
constexpr int64_t kStatsMinUnits = 1;   // ... at least this many units each

// ---------------------------------------------------------------------------
// Welford coefficients a_k = k/(k+1), b_k = 1/(k+1) (RMSF.py:137-138), folded
// at compile time (IEEE division, identical to numpy's) into a constant table
// read with scalar loads.  A split never exceeds kCoefN frames.
constexpr int kCoefN = RMSF_MAX_SPLIT_FRAMES;
struct WCoef {
  double a, b;
};
struct WCoefTable {
  WCoef v[kCoefN];
};
constexpr WCoefTable make_coef_table() {
  WCoefTable t{};
  for (int k = 0; k < kCoefN; ++k) {
    t.v[k].a = double(k) / double(k + 1);
    t.v[k].b = 1.0 / double(k + 1);
  }
  return t;
}
__constant__ WCoefTable g_coef = make_coef_table();

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

[[maybe_unused]] __device__ __forceinline__ void welford(double &m, double &q, double x, const WCoef c) {
  // M2 += k/(k+1) (x-mean)^2 ; mean = (k mean + x)/(k+1) == mean + (x-mean)/(k+1)
  const double d = x - m;
  q = fma(c.a * d, d, q);
  m = fma(c.b, d, m);
}

// (S1, S2) of n values shifted by sh -> (mean, M2); inv = 1/n.  M2 is
// clamped at 0 (S2 - S1^2/n can round below it only when M2 ~ 0) -- by a
// comparison, not fmax, so a NaN (e.g. the undefined rotation of a
// one-atom superposition, NaN in qcprot too) stays NaN as in RMSF.py.
__device__ __forceinline__ double clamp0(double v) { return v > 0.0 ? v : (v == v ? 0.0 : v); }

[[maybe_unused]] __device__ __forceinline__ void shifted_to_moments(double &s1, double &s2, double sh, double inv) {
  const double d = s1 * inv;
  s2 = clamp0(fma(-s1, d, s2));
  s1 = sh + d;
}

__device__ __forceinline__ int64_t split_begin(int64_t n_frames, int n_splits, int s) {
  return (n_frames * s) / n_splits;
}

// ---------------------------------------------------------------------------
// Streaming bodies.  One lane walks `nf` consecutive frames of its column and
// keeps the statistics in registers; U frames of loads are in flight.
//
// wel_flat_run: 4 consecutive coordinates (one float4) per lane, no
// alignment, contiguous selection (config C2).
template <int U>
__device__ __forceinline__ void wel_flat_run(const f32x4 *__restrict__ p, int64_t stride4, int nf, double (&m)[4],
                                             double (&q)[4]) {
#if RMSF_SHIFTED_SUMS
  // Shifted sums: S1 = sum d, S2 = sum d^2 with d = x - x_first (the
  // segment's first frame), converted to (mean, M2) at the end -- 3 VALU ops
  // per coordinate against Welford's 4, and no per-frame coefficients.  Same
  // statistics as RMSF.py:137-138's Welford to f64 rounding (the shift keeps
  // S1 small, so M2 = S2 - S1^2/n does not cancel).
  double sh[4];
  if (nf <= 0) {  // an empty split: nothing to read
#pragma unroll
    for (int c = 0; c < 4; ++c) m[c] = q[c] = 0.0;
    return;
  }
  {
    const f32x4 v0 = p[0];
    sh[0] = (double)v0.x, sh[1] = (double)v0.y, sh[2] = (double)v0.z, sh[3] = (double)v0.w;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) m[c] = q[c] = 0.0;
  auto acc = [&](const f32x4 v) {
    const double d0 = (double)v.x - sh[0], d1 = (double)v.y - sh[1];
    const double d2 = (double)v.z - sh[2], d3 = (double)v.w - sh[3];
    m[0] += d0, m[1] += d1, m[2] += d2, m[3] += d3;
    q[0] = fma(d0, d0, q[0]), q[1] = fma(d1, d1, q[1]), q[2] = fma(d2, d2, q[2]), q[3] = fma(d3, d3, q[3]);
  };
  int k = 0;
  for (; k + U <= nf; k += U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + (int64_t)(k + u) * stride4);
#pragma unroll
    for (int u = 0; u < U; ++u) acc(v[u]);
  }
  for (; k < nf; ++k) acc(__builtin_nontemporal_load(p + (int64_t)k * stride4));
  const double inv = g_coef.v[nf - 1].b;  // 1/nf
#pragma unroll
  for (int c = 0; c < 4; ++c) shifted_to_moments(m[c], q[c], sh[c], inv);
#else
#pragma unroll
  for (int c = 0; c < 4; ++c) m[c] = q[c] = 0.0;
  int k = 0;
  for (; k + U <= nf; k += U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + (int64_t)(k + u) * stride4);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const WCoef c = g_coef.v[k + u];
      welford(m[0], q[0], (double)v[u].x, c);
      welford(m[1], q[1], (double)v[u].y, c);
      welford(m[2], q[2], (double)v[u].z, c);
      welford(m[3], q[3], (double)v[u].w, c);
    }
  }
  for (; k < nf; ++k) {
    const f32x4 v = __builtin_nontemporal_load(p + (int64_t)k * stride4);
    const WCoef c = g_coef.v[k];
    welford(m[0], q[0], (double)v.x, c);
    welford(m[1], q[1], (double)v.y, c);
    welford(m[2], q[2], (double)v.z, c);
    welford(m[3], q[3], (double)v.w, c);
  }
#endif
}

// Partials are written with nontemporal stores: beside the nt-load streams,
// plain stores of a few percent of the bytes cost 2-8 % of the stream's time
// on gfx950, nt stores about a third of that (tools/ubench_welford2.hip).
__device__ __forceinline__ void nt_store(double v, double *p) { __builtin_nontemporal_store(v, p); }

__device__ __forceinline__ void store4(double *__restrict__ om, double *__restrict__ oq, const double (&m)[4],
                                       const double (&q)[4]) {
  f64x2 *a = reinterpret_cast<f64x2 *>(om);
  f64x2 *b = reinterpret_cast<f64x2 *>(oq);
  __builtin_nontemporal_store(f64x2{m[0], m[1]}, a);
  __builtin_nontemporal_store(f64x2{m[2], m[3]}, a + 1);
  __builtin_nontemporal_store(f64x2{q[0], q[1]}, b);
  __builtin_nontemporal_store(f64x2{q[2], q[3]}, b + 1);
}

// k_welford_flat (split grid): grid = (ceil(n4/256), n_splits).
template <int U>
__global__ __launch_bounds__(kBlock) void k_welford_flat(
    const float *__restrict__ xyz, int64_t stride4, int64_t n4, int64_t n_frames,
    int n_splits, double *__restrict__ out_mean, double *__restrict__ out_m2,
    int64_t n_coord) {
  const int64_t i4 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i4 >= n4) return;
  const int s = blockIdx.y;
  const int64_t fb = split_begin(n_frames, n_splits, s);
  const int nf = (int)(split_begin(n_frames, n_splits, s + 1) - fb);
  double m[4], q[4];
  wel_flat_run<U>(reinterpret_cast<const f32x4 *>(xyz) + fb * stride4 + i4, stride4, nf, m, q);
  store4(out_mean + (int64_t)s * n_coord + 4 * i4, out_m2 + (int64_t)s * n_coord + 4 * i4, m, q);
}

// accum_atoms_run: one selected atom (12 B) per lane; MODE 0 = WELFORD
// (m = mean, q = M2), 1 = SUM (m = sum).  xf = the first frame's transform.
template <int MODE, bool ALIGN, int U, bool PLANES = false>
__device__ __forceinline__ void accum_atoms_run(const float *__restrict__ p, int64_t fstride, int nf,
                                                const double *__restrict__ xf, double rc0, double rc1, double rc2,
                                                double (&m)[3], double (&q)[3], int64_t ps = 0) {
  const int64_t cs = PLANES ? ps : 1;  // x -> y -> z of the lane's atom (coordinate planes: ps floats)
#pragma unroll
  for (int c = 0; c < 3; ++c) m[c] = q[c] = 0.0;
#if RMSF_SHIFTED_SUMS
  // WELFORD as shifted sums (see wel_flat_run): the shift is the segment's
  // first frame after the transform
  double sh[3] = {0.0, 0.0, 0.0};
  if (MODE == RMSF_MODE_WELFORD && nf > 0) {
    float x = p[0], y = p[cs], z = p[2 * cs];
    if (ALIGN) apply_xform(x, y, z, xf, rc0, rc1, rc2);
    sh[0] = (double)x, sh[1] = (double)y, sh[2] = (double)z;
  }
#endif
  auto consume = [&](float x, float y, float z, int k) {
    if (ALIGN) apply_xform(x, y, z, xf + (int64_t)k * kXform, rc0, rc1, rc2);
    if (MODE == RMSF_MODE_WELFORD) {
#if RMSF_SHIFTED_SUMS
      const double d0 = (double)x - sh[0], d1 = (double)y - sh[1], d2 = (double)z - sh[2];
      m[0] += d0, m[1] += d1, m[2] += d2;
      q[0] = fma(d0, d0, q[0]), q[1] = fma(d1, d1, q[1]), q[2] = fma(d2, d2, q[2]);
#else
      const WCoef c = g_coef.v[k];
      welford(m[0], q[0], (double)x, c);
      welford(m[1], q[1], (double)y, c);
      welford(m[2], q[2], (double)z, c);
#endif
    } else {
      m[0] += (double)x;
      m[1] += (double)y;
      m[2] += (double)z;
    }
  };
  int k = 0;
  for (; k + U <= nf; k += U) {
    float vx[U], vy[U], vz[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float *r = p + (int64_t)(k + u) * fstride;
      vx[u] = __builtin_nontemporal_load(r);
      vy[u] = __builtin_nontemporal_load(r + cs);
      vz[u] = __builtin_nontemporal_load(r + 2 * cs);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) consume(vx[u], vy[u], vz[u], k + u);
  }
  for (; k < nf; ++k) {
    const float *r = p + (int64_t)k * fstride;
    consume(r[0], r[cs], r[2 * cs], k);
  }
#if RMSF_SHIFTED_SUMS
  if (MODE == RMSF_MODE_WELFORD && nf > 0) {
    const double inv = g_coef.v[nf - 1].b;  // 1/nf
#pragma unroll
    for (int c = 0; c < 3; ++c) shifted_to_moments(m[c], q[c], sh[c], inv);
  }
#endif
}

template <int MODE>
__device__ __forceinline__ void store3(double *__restrict__ o0, double *__restrict__ o1, const double (&m)[3],
                                       const double (&q)[3]) {
  nt_store(m[0], o0);
  nt_store(m[1], o0 + 1);
  nt_store(m[2], o0 + 2);
  if (MODE == RMSF_MODE_WELFORD) {
    nt_store(q[0], o1);
    nt_store(q[1], o1 + 1);
    nt_store(q[2], o1 + 2);
  }
}

// k_accum_atoms (split grid): one selected atom per lane, frames of split
// blockIdx.y.  MODE 0 = WELFORD (out0 = mean, out1 = M2), 1 = SUM (out0 = sum).
template <int MODE, bool ALIGN, bool GATHER, int U>
__global__ __launch_bounds__(kBlock) void k_accum_atoms(
    const float *__restrict__ xyz, int64_t fstride, int64_t n_sel, const int32_t *__restrict__ sel,
    int64_t n_frames, int n_splits, const double *__restrict__ xform, const double *__restrict__ refinfo,
    double *__restrict__ out0, double *__restrict__ out1) {
  const int64_t a = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a >= n_sel) return;
  const int s = blockIdx.y;
  const int64_t fb = split_begin(n_frames, n_splits, s);
  const int nf = (int)(split_begin(n_frames, n_splits, s + 1) - fb);
  const int64_t off = GATHER ? 3 * (int64_t)sel[a] : 3 * a;
  const double rc0 = ALIGN ? refinfo[0] : 0.0, rc1 = ALIGN ? refinfo[1] : 0.0, rc2 = ALIGN ? refinfo[2] : 0.0;
  double m[3], q[3];
  accum_atoms_run<MODE, ALIGN, U>(xyz + fb * fstride + off, fstride, nf, ALIGN ? xform + fb * kXform : nullptr,
                                  rc0, rc1, rc2, m, q);
  const int64_t o = (int64_t)s * 3 * n_sel + 3 * a;
  store3<MODE>(out0 + o, out1 + o, m, q);
}

// ---------------------------------------------------------------------------
// Balanced ("stream-K") grid.  The batch's (lane chunk, frame) space --
// chunk c = lanes [256c, 256c+256), frames 0..nf-1 -- is linearised
// chunk-major and cut into G equal ranges, one per workgroup (G = a multiple
// of the CU count, kSkPerCu* below), so every workgroup streams the same
// bytes and no tail wave exists.  A workgroup walks its range as segments:
// maximal runs inside one chunk, at most kCoefN frames (the coefficient
// table); each segment writes one partial into slot b*P + j (j = segment
// index within workgroup b).  Measured on MI355X (tools/ubench_welford.hip,
// 100k atoms x 20k frames): 3.48 ms at G = 512 vs 3.67-3.75 ms for the best
// split grid, against a 3.47 ms pure-read ceiling.  The gain varies by box:
// where the split grid already streams at ~3.67 ms the two tie.
//
// Workspace = header (kSkHdr int64) + parts0[G*P][256*cpl] (+ parts1).
constexpr int kSkHdr = 16;
constexpr int64_t kSkMinSeg = 32;  // auto grid: ranges of >= this many frames
constexpr int64_t kSkMaxSegsPerChunk = 64;  // auto grid: ranges per chunk at most (sk_plan)
struct SkPlan {
  int64_t lanes, C, nf, T;
  int G, P, cpl, mode;
  int S;   // > 0: chunk-aligned ranges, S per chunk, dispatched split-major
  int cw;  // lanes per chunk (kBlock; 16 for the tiled float4 stream)
  // launch subset (chunk-aligned plans): chunks [c0, c0 + Cs) -- an atom slab
  // whose ranges and segments are exactly the whole plan's (not in the header)
  int64_t c0, Cs;
};

// range processed by hardware workgroup `hw`: with chunk-aligned ranges the
// dispatch is split-major (consecutive workgroups = consecutive chunks of
// the same frames, as the split grid's), otherwise the identity
__device__ __forceinline__ int sk_range(const SkPlan &p, int hw) {
  return p.S > 0 ? (int)((p.c0 + (int64_t)hw % p.Cs) * p.S + hw / p.Cs) : hw;
}

__host__ __device__ inline int64_t sk_lo(const SkPlan &p, int64_t b) { return p.T * b / p.G; }

__host__ __device__ inline int64_t sk_seg_len(const SkPlan &p, int64_t lo, int64_t hi, int64_t *c, int64_t *f0) {
  *c = lo / p.nf;
  *f0 = lo - *c * p.nf;
  int64_t len = hi - lo;
  if (p.nf - *f0 < len) len = p.nf - *f0;
  if (len > kCoefN) len = kCoefN;
  return len;
}

// The segment walk is wave-uniform, but 64-bit division runs on the VALU:
// pin the results to SGPRs so the per-frame transform records and the
// coefficient table keep arriving by scalar loads.
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ void sk_write_header(int64_t *hdr, const SkPlan &p) {
  hdr[0] = p.lanes;
  hdr[1] = p.C;
  hdr[2] = p.nf;
  hdr[3] = p.T;
  hdr[4] = p.G;
  hdr[5] = p.P;
  hdr[6] = p.cpl;
  hdr[7] = p.mode;
  hdr[8] = p.S;
  hdr[9] = p.cw;
}

template <int U>
__global__ __launch_bounds__(kBlock) void k_welford_flat_sk(const float *__restrict__ xyz, int64_t stride4,
                                                            SkPlan pl, int64_t *__restrict__ hdr,
                                                            double *__restrict__ parts0,
                                                            double *__restrict__ parts1) {
  const int b = sk_range(pl, blockIdx.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) sk_write_header(hdr, pl);
  int64_t lo = sk_lo(pl, b);
  const int64_t hi = sk_lo(pl, b + 1);
  int64_t slot = (int64_t)b * pl.P;
  while (lo < hi) {
    int64_t c, f0;
    const int len = (int)sk_seg_len(pl, lo, hi, &c, &f0);
    const int64_t i4 = c * kBlock + threadIdx.x;
    if (i4 < pl.lanes) {
      double m[4], q[4];
      wel_flat_run<U>(reinterpret_cast<const f32x4 *>(xyz) + f0 * stride4 + i4, stride4, len, m, q);
      const int64_t o = slot * (kBlock * 4) + 4 * threadIdx.x;
      store4(parts0 + o, parts1 + o, m, q);
    }
    lo += len;
    ++slot;
  }
}

// ---------------------------------------------------------------------------
// RMSF.py:137-138 as written (round 4, the sequential Welford): for every
// coordinate, the batch's frames in order, k = k0 + f,
//   sumsquares += (k / (k + 1.0)) * (x - mean)**2
//   mean = (k * mean + x) / (k + 1)
// with numpy's operations and roundings (no contraction, csrc/Makefile), so
// the running (mean, sumsquares) are the reference recurrence's own values
// bit for bit.  Parallel over coordinates only: a lane carries one
// coordinate through every frame, with the next U frames' loads in flight
// while it folds the current U.  The per-frame constants come from a table
// (k_seq_coef) read by scalar loads: c_k = k / (k + 1.0), and r_k, 1 / (k + 1)
// refined as the hardware division refines it, so the division costs a mul
// and two FMAs per coordinate -- q0 = num r_k, q = fma(fma(-(k+1), q0, num),
// r_k, q0), the closing steps of the IEEE division sequence (v_div_scale /
// v_div_fmas / v_div_fixup change nothing for a finite numerator in normal
// range; seq_div covers the rest).
struct SeqCoef {
  double c, r;
};

__global__ __launch_bounds__(kBlock) void k_seq_coef(int64_t k0, int64_t nf, SeqCoef *__restrict__ out) {
  const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (f >= nf) return;
  const double k = (double)(k0 + f), k1 = k + 1.0;
  double r = __builtin_amdgcn_rcp(k1);
  double e = __builtin_fma(-k1, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-k1, r, 1.0);
  r = __builtin_fma(r, e, r);
  out[f] = SeqCoef{k / k1, r};
}

// num / k1 for k1 = k + 1 >= 1 and r = k_seq_coef's refined 1/k1.  The
// fast form is the hardware division's own closing steps; it is exact
// whenever v_div_scale would not rescale, i.e. for every finite nonzero
// numerator that f32 coordinates can produce (|num| between ~2^-201 and
// 2^181, far inside the 2^-968 .. 2^1023 band).  Zero and infinity divide
// to themselves, and a NaN stays NaN, so one select covers the rest.
__device__ __forceinline__ double seq_div(double num, double k1, double r) {
  const double q0 = num * r;
  const double q = __builtin_fma(__builtin_fma(-k1, q0, num), r, q0);
  return (num == 0.0 || __builtin_isinf(num)) ? num : q;
}

template <int U, bool GATHER>
__global__ __launch_bounds__(kBlock) void k_welford_seq(const float *__restrict__ xyz, int64_t fstride, int64_t nf,
                                                        int64_t n_coord, const int32_t *__restrict__ sel,
                                                        int64_t k0, const SeqCoef *__restrict__ coef,
                                                        double *__restrict__ mean, double *__restrict__ ss) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n_coord) return;
  // RMSF.py:119-120: np.zeros; later batches continue the running state
  double m = k0 > 0 ? mean[j] : 0.0, q = k0 > 0 ? ss[j] : 0.0;
  const float *__restrict__ p = xyz + (GATHER ? 3 * (int64_t)sel[j / 3] + j % 3 : j);
  // k = k0 + f and k1 = k + 1 exactly (integers below 2^53)
  auto step = [&](float v, const SeqCoef cf, double k, double k1) {
    const double x = (double)v;
    const double d = x - m;
    q = q + cf.c * (d * d);
    m = seq_div(k * m + x, k1, cf.r);
  };
  auto load = [&](float (&v)[U], SeqCoef (&c)[U], int64_t f) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = __builtin_nontemporal_load(p + (f + u) * fstride);
      c[u] = coef[f + u];
    }
  };
  // A block whose coordinates are all nonzero and finite, entered with a
  // finite running mean, needs no select: every numerator k*mean + x is then
  // finite and nonzero, or an exact cancellation to +0 that the closing steps
  // also return as +0 (-0 needs x = -0).  Checked once per block and wave:
  // 2 % faster at 100k x 20k, the same bits (tools/ab_seq_hoist.py).
  auto step_fast = [&](float v, const SeqCoef cf, double k, double k1) {
    const double x = (double)v;
    const double d = x - m;
    q = q + cf.c * (d * d);
    const double num = k * m + x;
    const double q0 = num * cf.r;
    m = __builtin_fma(__builtin_fma(-k1, q0, num), cf.r, q0);
  };
  // kb = k0 + f carried across blocks: the block's U + 1 frame counts cost U
  // adds (frame u's k + 1 is frame u + 1's k), not a 64-bit conversion and
  // 2U - 1 adds
  auto run = [&](const float (&v)[U], const SeqCoef (&c)[U], double &kb) {
    double kk[U + 1];
    kk[0] = kb;
#pragma unroll
    for (int u = 1; u <= U; ++u) kk[u] = kb + (double)u;
    kb = kk[U];
    bool special = __builtin_isinf(m);
#pragma unroll
    for (int u = 0; u < U; ++u) special |= (v[u] == 0.0f) | __builtin_isinf(v[u]);
    if (!__any((int)special)) {
#pragma unroll
      for (int u = 0; u < U; ++u) step_fast(v[u], c[u], kk[u], kk[u + 1]);
      return;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) step(v[u], c[u], kk[u], kk[u + 1]);
  };
  // two register blocks in turn, one always loading while the other folds
  // (no copies between them: a copy makes the compiler wait on the
  // coefficients' scalar loads where it is made).  The coefficients stay a
  // table read by scalar loads: computing each 64-frame window's c and r in
  // the wave (one division per lane) and broadcasting them by v_readlane is
  // bit-identical but slower -- 4.98 vs 4.20 ms at 100k x 20k
  // (tools/ab_seq_lane.py, profiles/r05_workloads/seq_welford_lane.txt).
  // A ring of 2-6 blocks (more loads in flight while one folds) spills
  // SGPRs and loses 10-17 % (tools/ab_seq_ring.py, seq_welford_ring.txt);
  // the same ring over raw buffer loads (no per-frame address SGPRs, no
  // spills) ties with this form, -1.3 to +4 % (seq_welford_buf.txt), and so
  // do this form's two blocks read by buffer loads (+1 %, 7 % fewer VALU
  // instructions, seq_welford_kk.txt).
  int64_t f = 0;
  double kb = (double)k0;
  if (nf >= U) {
    float a[U], b[U];
    SeqCoef ca[U], cb[U];
    load(a, ca, 0);
    for (;;) {
      if (f + 2 * U > nf) {
        run(a, ca, kb);
        f += U;
        break;
      }
      load(b, cb, f + U);
      run(a, ca, kb);
      f += U;
      if (f + 2 * U > nf) {
        run(b, cb, kb);
        f += U;
        break;
      }
      load(a, ca, f + U);
      run(b, cb, kb);
      f += U;
    }
  }
  for (; f < nf; ++f, kb += 1.0) step(__builtin_nontemporal_load(p + f * fstride), coef[f], kb, kb + 1.0);
  mean[j] = m;
  ss[j] = q;
}

// The gathered recurrence with one selected atom per lane (round 5): its
// three coordinates are three independent chains, the frame's row is one
// dwordx3 load per atom, and a wave gathers 64 atoms per load instruction
// instead of 21 -- a third of the address work for the texture path, which
// bounds the coordinate-per-lane gather (0.47 of HBM at 100k of 120k atoms).
// A third of the waves, too: it pays from ~50k selected atoms (0.75 waves
// per SIMD) and loses below (profiles/r05_workloads/seq_welford_atoms.txt).
// Same operations per coordinate as k_welford_seq, so the same bits.
template <int U>
__global__ __launch_bounds__(kBlock) void k_welford_seq_atoms(const float *__restrict__ xyz, int64_t fstride,
                                                              int64_t nf, int64_t n_sel,
                                                              const int32_t *__restrict__ sel, int64_t k0,
                                                              const SeqCoef *__restrict__ coef,
                                                              double *__restrict__ mean, double *__restrict__ ss) {
  const int64_t a = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a >= n_sel) return;
  double m[3], q[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    m[c] = k0 > 0 ? mean[3 * a + c] : 0.0;
    q[c] = k0 > 0 ? ss[3 * a + c] : 0.0;
  }
  const float *__restrict__ p = xyz + 3 * (int64_t)sel[a];
  auto step = [&](int c, float v, const SeqCoef cf, double k, double k1) {
    const double x = (double)v;
    const double d = x - m[c];
    q[c] = q[c] + cf.c * (d * d);
    m[c] = seq_div(k * m[c] + x, k1, cf.r);
  };
  auto step_fast = [&](int c, float v, const SeqCoef cf, double k, double k1) {
    const double x = (double)v;
    const double d = x - m[c];
    q[c] = q[c] + cf.c * (d * d);
    const double num = k * m[c] + x;
    const double q0 = num * cf.r;
    m[c] = __builtin_fma(__builtin_fma(-k1, q0, num), cf.r, q0);
  };
  auto load = [&](float (&v)[U][3], SeqCoef (&cc)[U], int64_t f) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float *r = p + (f + u) * fstride;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[u][c] = __builtin_nontemporal_load(r + c);
      cc[u] = coef[f + u];
    }
  };
  auto run = [&](const float (&v)[U][3], const SeqCoef (&cc)[U], double &kb) {
    double kk[U + 1];
    kk[0] = kb;
#pragma unroll
    for (int u = 1; u <= U; ++u) kk[u] = kb + (double)u;
    kb = kk[U];
    bool special = __builtin_isinf(m[0]) | __builtin_isinf(m[1]) | __builtin_isinf(m[2]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) special |= (v[u][c] == 0.0f) | __builtin_isinf(v[u][c]);
    if (!__any((int)special)) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < 3; ++c) step_fast(c, v[u][c], cc[u], kk[u], kk[u + 1]);
      return;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) step(c, v[u][c], cc[u], kk[u], kk[u + 1]);
  };
  int64_t f = 0;
  double kb = (double)k0;
  if (nf >= U) {
    float va[U][3], vb[U][3];
    SeqCoef ca[U], cb[U];
    load(va, ca, 0);
    for (;;) {
      if (f + 2 * U > nf) {
        run(va, ca, kb);
        f += U;
        break;
      }
      load(vb, cb, f + U);
      run(va, ca, kb);
      f += U;
      if (f + 2 * U > nf) {
        run(vb, cb, kb);
        f += U;
        break;
      }
      load(va, ca, f + U);
      run(vb, cb, kb);
      f += U;
    }
  }
  for (; f < nf; ++f, kb += 1.0) {
    const float *r = p + f * fstride;
#pragma unroll
    for (int c = 0; c < 3; ++c) step(c, __builtin_nontemporal_load(r + c), coef[f], kb, kb + 1.0);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    mean[3 * a + c] = m[c];
    ss[3 * a + c] = q[c];
  }
}

// ---------------------------------------------------------------------------
// exact=True on the ALIGNED path (round 6): RMSF.py:84-85, 94-97, 99-103,
// 111, 117-118, 127-138 with the reference's own summation orders, so each
// frame's rotation, every f32 rounding point of the transform, the sweep-1
// sum, the average and the Welford state are the script's own values bit
// for bit (on the restated upstream orders: AtomGroup.center_of_mass =
// einsum('ij,ij->j', x, m[:, None]) / m.sum(), sequential over the atoms
// with the caller's numpy m.sum(); qcprot's InnerProduct loop; both as
// oracle/rmsf_oracle.py restates them -- upstream, unverified here).  The
// frame-parallel kernels above reassociate these sums, so their rotations
// can differ in the last bits, which flips an f32 rounding point of an
// aligned coordinate now and then -- a cost of |x - mean| ulp / (N RMSF)
// that only a few-frame run can push past 1e-6 A.
//
// wave_seq_sum: s = ((t_0 + t_1) + t_2) + ... over atoms 0..n-1, the
// reference's order, by one wave.  Its 64 lanes form the terms of a block
// of kSeqBlk atoms at once (lane i: atoms a0 + i + 64 j -- coalesced loads,
// elementwise terms with the same roundings as the serial statement) and
// park them in the wave's LDS slice; then the chain adds them in order, 32
// at a time: each lane reads two consecutive terms of the group (lane i of
// every 16-lane row: terms 2i and 2i + 1, one ds_read_b128), and each add is
// a v_fmac_f64 of the term broadcast from lane j of the row (DPP
// row_newbcast:j) times 1.0 -- fma(t, 1.0, s) rounds once, exactly as s + t
// does, so the bits are the serial sum's (every lane carries the same s).
// The next block's loads are issued before the chain runs.  The adds are the
// only serial work, at the dependent f64 add's own floor: 2.05 ns per add,
// against 4.3-4.6 when every lane read each term by a broadcast LDS read
// (the LDS's return bandwidth bound that form; tools/ubench_chain2.hip,
// profiles/r06_workloads/chain2.txt).  (The first round-6 form walked every
// chain in one lane per frame: ~500 cycles per atom, 24 ms for one sweep's
// superposition of 100k atoms x 100 frames; a form with four frames' chains
// per wave, one per row, and the terms in registers lost to load latency:
// profiles/r06_workloads/probe_exact_aligned.txt.)  Atoms past n enter as
// +0.0: s is never -0.0 (it starts at +0.0, and x + (-x) is +0.0), so
// s + 0.0 == s bit for bit and a ragged last group needs no branch.
// load(a) issues atom a's loads (a clamped to the last atom: every block
// issues the same count), term(raw, a) forms t_a.  lds: kSeqBlk doubles
// private to the wave.
constexpr int kSeqK = 16;             // atoms per lane per block (4 / 8 / 16 measured: 16 ~7 % faster)
constexpr int kSeqBlk = 64 * kSeqK;   // atoms per block
// A chain is issue-bound: two chain waves on one SIMD run at half speed each
// (ubench_chain2 V5: 2.05 -> 3.8 ns per add).  So the reference's workgroup
// (four chains) holds nearly all of its CU's LDS, and a launch of at most
// kSeqReserveMax chain waves reserves kSeqReserve bytes of LDS per wave
// beside its 8 KB slice (40 KB in all), so at most four share a CU, one per
// SIMD.  Above that the reservation cost more than it saved (the waves fill
// the CUs unevenly and some wait a whole chain): 100k atoms x 100 frames'
// 1,000 InnerProduct chains 0.96 ms unreserved against 1.2, 1M x 32's 320
// 5.7 against 7.3 ms (profiles/r06_workloads/exact_chain_dpp.txt).
constexpr int kRefSlice = 4 * kSeqBlk + kSeqBlk / 2;
// At most kSeqPcMax chains a launch runs each chain as a two-wave workgroup
// (pc_seq_sum: one wave forms the terms, one adds them) with 16 KB + 56 KB of
// LDS, at most two per CU; up to kSeqReserveMax as one wave with 8 KB + 32 KB,
// at most four per CU; above that one wave, unreserved.  (Two-wave chains
// at 1M atoms x 32 frames: 5.54 against 5.91 ms; at 100k x 100's 1,000
// InnerProduct chains, where the doubled wave count shares SIMDs, 1.16
// against 1.10: profiles/r06_workloads/exact_pc_ab.txt.)
constexpr int64_t kSeqPcMax = 512;
constexpr size_t kSeqPcReserve = 7 * kSeqBlk * sizeof(double);
constexpr size_t kSeqReserve = 4 * kSeqBlk * sizeof(double);
constexpr int64_t kSeqReserveMax = 768;
inline bool seq_pc(int64_t chains) { return chains <= kSeqPcMax; }
inline size_t seq_reserve(int64_t chains) {
  return seq_pc(chains) ? kSeqPcReserve : chains <= kSeqReserveMax ? kSeqReserve : 0;
}
// s += the group's 32 terms (lane 0's pair first), in order.  The opening
// s_nop 1: a DPP read of a VGPR needs 2 wait states after a VALU write, and
// hipcc pads nothing inside an asm string.  The adds follow each other with
// none: back to back, each reads the accumulator the previous one wrote
// (measured: the sum of 2e5 chained adds bit-equal to the plain chain's;
// 2.05 ns per add, against 3.6 with an s_nop 0 between; ubench_chain2 V5).
#define RMSF_ROW_FMAC(J)                                                \
  "v_fmac_f64_dpp %0, %1, %3 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t" \
  "v_fmac_f64_dpp %0, %2, %3 row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ double row_add32(double s, const double2 &u, double one) {
  asm("s_nop 1\n\t" RMSF_ROW_FMAC(0) RMSF_ROW_FMAC(1) RMSF_ROW_FMAC(2) RMSF_ROW_FMAC(3) RMSF_ROW_FMAC(4)
          RMSF_ROW_FMAC(5) RMSF_ROW_FMAC(6) RMSF_ROW_FMAC(7) RMSF_ROW_FMAC(8) RMSF_ROW_FMAC(9) RMSF_ROW_FMAC(10)
              RMSF_ROW_FMAC(11) RMSF_ROW_FMAC(12) RMSF_ROW_FMAC(13) RMSF_ROW_FMAC(14) RMSF_ROW_FMAC(15)
      : "+v"(s)
      : "v"(u.x), "v"(u.y), "v"(one));
  return s;
}
#undef RMSF_ROW_FMAC
// The chain over one parked block: s += its cnt terms in order (whole
// groups of 32; the caller pads the last group with +0.0).  Lane i of a row
// reads the pair 2i, 2i + 1 of each group.
__device__ __forceinline__ double chain_block(double s, const double *lds, int cnt) {
  const double one = 1.0;
  const double2 *pair = reinterpret_cast<const double2 *>(lds) + (threadIdx.x & 15);
  constexpr int NG = kSeqBlk / 32;
  if (cnt == kSeqBlk) {  // two groups' reads in flight while one is added
    double2 u[3];
    u[0] = pair[0];
    u[1] = pair[16];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g + 2 < NG) u[(g + 2) % 3] = pair[16 * (g + 2)];
      __builtin_amdgcn_sched_barrier(0);
      s = row_add32(s, u[g % 3], one);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {  // the ragged last block: its groups, the last one padded with +0.0
    const int ng = (cnt + 31) / 32;
    double2 u = pair[0];
    for (int g = 0; g < ng; ++g) {
      const double2 w = u;
      if (g + 1 < ng) u = pair[16 * (g + 1)];
      s = row_add32(s, w, one);
    }
  }
  return s;
}
template <class Load, class Term>
__device__ __forceinline__ double wave_seq_sum(int64_t n, double *lds, Load load, Term term) {
  using Raw = decltype(load(int64_t(0)));
  const int lane = threadIdx.x & 63;
  Raw va[kSeqK], vb[kSeqK];
  double s = 0.0;
  // whole blocks: unclamped indices, so one base and constant offsets per
  // lane address the block (no 64-bit index arithmetic per load)
  auto fill = [&](Raw(&v)[kSeqK], int64_t a0) {
    const int64_t b = a0 + lane;
    if (a0 + kSeqBlk <= n) {
#pragma unroll
      for (int j = 0; j < kSeqK; ++j) v[j] = load(b + 64 * j);
    } else {
#pragma unroll
      for (int j = 0; j < kSeqK; ++j) v[j] = load(min(b + 64 * j, n - 1));
    }
    __builtin_amdgcn_sched_barrier(0);  // issued before the chain below
  };
  auto run = [&](const Raw(&v)[kSeqK], int64_t a0) {
    const int64_t b = a0 + lane;
    if (a0 + kSeqBlk <= n) {
#pragma unroll
      for (int j = 0; j < kSeqK; ++j) lds[lane + 64 * j] = term(v[j], b + 64 * j);
    } else {
#pragma unroll
      for (int j = 0; j < kSeqK; ++j) lds[lane + 64 * j] = b + 64 * j < n ? term(v[j], b + 64 * j) : 0.0;
    }
    __builtin_amdgcn_wave_barrier();  // one wave: its LDS operations complete in order
    s = chain_block(s, lds, (int)min((int64_t)kSeqBlk, n - a0));
    __builtin_amdgcn_wave_barrier();  // the slice is rewritten by the next block
  };
  fill(va, 0);
  int64_t a0 = 0;
  for (; a0 + 2 * kSeqBlk < n; a0 += 2 * kSeqBlk) {
    fill(vb, a0 + kSeqBlk);
    run(va, a0);
    fill(va, a0 + 2 * kSeqBlk);
    run(vb, a0 + kSeqBlk);
  }
  fill(vb, a0 + kSeqBlk);
  run(va, a0);
  if (a0 + kSeqBlk < n) run(vb, a0 + kSeqBlk);
  return s;
}

// pc_seq_sum: wave_seq_sum split over a workgroup of two waves (round 6).
// Wave 1 loads block b + 1 and parks its terms in one LDS buffer while wave
// 0 adds block b's from the other, so the chain wave issues nothing but its
// reads and adds; one barrier per block.  Same loads, terms and order, so
// the same bits.  s is the chain wave's.  buf: two kSeqBlk-double buffers.
// chain: whether this wave adds (wave-uniform); several pairs may share a
// workgroup, each with its own buf, as long as every pair has the same n
// (the barriers are the workgroup's).
template <class Load, class Term>
__device__ __forceinline__ double pc_seq_sum(int64_t n, double (*buf)[kSeqBlk], Load load, Term term,
                                             bool chain = threadIdx.x < 64) {
  using Raw = decltype(load(int64_t(0)));
  const int lane = threadIdx.x & 63;
  const int64_t nb = (n + kSeqBlk - 1) / kSeqBlk;
  Raw va[kSeqK], vb[kSeqK];
  double s = 0.0;
  auto fill = [&](Raw(&v)[kSeqK], int64_t blk) {
    const int64_t a0 = blk * kSeqBlk, b = a0 + lane;
    if (a0 + kSeqBlk <= n) {
#pragma unroll
      for (int j = 0; j < kSeqK; ++j) v[j] = load(b + 64 * j);
    } else {
#pragma unroll
      for (int j = 0; j < kSeqK; ++j) v[j] = load(min(b + 64 * j, n - 1));
    }
  };
  auto park = [&](const Raw(&v)[kSeqK], int64_t blk) {
    double *lds = buf[blk & 1];
    const int64_t a0 = blk * kSeqBlk, b = a0 + lane;
    if (a0 + kSeqBlk <= n) {
#pragma unroll
      for (int j = 0; j < kSeqK; ++j) lds[lane + 64 * j] = term(v[j], b + 64 * j);
    } else {
#pragma unroll
      for (int j = 0; j < kSeqK; ++j) lds[lane + 64 * j] = b + 64 * j < n ? term(v[j], b + 64 * j) : 0.0;
    }
  };
  auto cnt = [&](int64_t blk) { return (int)min((int64_t)kSeqBlk, n - blk * kSeqBlk); };
  if (!chain) {
    fill(va, 0);
    fill(vb, 1);
    park(va, 0);
    fill(va, 2);
  }
  __syncthreads();
  // step b: the chain adds block b; wave 1 parks block b + 1 (loaded two
  // steps ago) and issues block b + 3's loads into the same registers
  for (int64_t b = 0; b < nb; b += 2) {
    if (chain) {
      s = chain_block(s, buf[b & 1], cnt(b));
    } else if (b + 1 < nb) {
      park(vb, b + 1);
      fill(vb, b + 3);
    }
    __syncthreads();
    if (b + 1 >= nb) break;
    if (chain) {
      s = chain_block(s, buf[(b + 1) & 1], cnt(b + 1));
    } else if (b + 2 < nb) {
      park(va, b + 2);
      fill(va, b + 4);
    }
    __syncthreads();
  }
  return s;
}

struct SeqF1D {  // a coordinate and an f64 factor (mass / reference)
  float x;
  double d;
};
struct SeqF3 {
  float x, y, z;
};
struct SeqD1D {
  double x, d;
};
struct SeqD3 {
  double x, y, z;
};

// The centred reference of exact=True (RMSF.py:84-85 / 111 + 117-118) and
// its record, in parts:
//   1. x = frame[sel[a]] (f32 -> f64) or avg[a] / div (RMSF.py:111, also to
//      avg_out) into ref;
//   2. com_c = (sum_a x_ac m_a, atom by atom) / mass_total (RMSF.py:84/117),
//      wave c's chain, to the record's [0..2];
//   3. ref = x - com in place (RMSF.py:85/118);
//   4. the rest of the record: sum r (waves 0-2), G2 = sum_a ((r0 r0 + r1
//      r1) + r2 r2) in qcprot's per-atom order (wave 3; the G2 of every
//      InnerProduct call against this reference), mass_total, n_sel.
// k_ref_seq runs them in one workgroup of four waves (PART kRefAll), or
// 1-3 (kRefCentre), 2 alone (kRefCom) or 4 alone (kRefSums).  From
// kRefGridMin atoms, 1 and 3 run as grid-wide launches (k_ref_fill,
// k_ref_centre_grid) instead: one workgroup streamed them at one CU's rate,
// ~4 ms of a 1M-atom setup's 8.5 (profiles/r06_workloads/exact_chain_dpp.txt).
constexpr int kRefAll = 0, kRefCentre = 1, kRefCom = 2, kRefSums = 3;
constexpr int64_t kRefGridMin = 16384;
constexpr size_t kRefPairsLds = 144 * 1024 - 3 * 2 * 1024 * sizeof(double);  // k_ref_com_pairs' dynamic LDS
template <bool FROM_F32, bool GATHER>
__device__ __forceinline__ void ref_fill_atom(int64_t a, const float *__restrict__ frame,
                                              const double *__restrict__ avg, double div,
                                              const int32_t *__restrict__ sel, double *__restrict__ avg_out,
                                              double *__restrict__ ref) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double x;
    if (FROM_F32) {
      x = (double)frame[3 * (GATHER ? (int64_t)sel[a] : a) + c];
    } else {
      x = avg[3 * a + c] / div;
      if (avg_out) avg_out[3 * a + c] = x;
    }
    ref[3 * a + c] = x;
  }
}
template <bool FROM_F32, bool GATHER>
__global__ __launch_bounds__(kBlock) void k_ref_fill(const float *__restrict__ frame, const double *__restrict__ avg,
                                                     double div, int64_t n_sel, const int32_t *__restrict__ sel,
                                                     double *__restrict__ avg_out, double *__restrict__ ref) {
  const int64_t a = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a < n_sel) ref_fill_atom<FROM_F32, GATHER>(a, frame, avg, div, sel, avg_out, ref);
}
__global__ __launch_bounds__(kBlock) void k_ref_centre_grid(int64_t n_coord, const double *__restrict__ info,
                                                            double *__restrict__ ref) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n_coord) ref[i] = ref[i] - info[i % 3];
}
// k_ref_com_pairs: k_ref_seq's part 2 (the reference's three COM chains,
// which the InnerProduct waits for) from kRefGridMin atoms, each chain a
// pair of waves (pc_seq_sum: wave c adds, wave c + 3 forms the terms; the
// adding waves must not share a SIMD, and a CU's waves are dealt to its
// SIMDs in turn -- pairs as waves 2c / 2c + 1 put two chains on one SIMD
// and ran 1.25x slower).
// Launched with kRefPairsLds of LDS so its CU runs nothing else.  Same bits
// as k_ref_seq's one-wave chains.  (The sums of r and G2 run beside the
// InnerProduct, off the critical path, and keep one wave each.)
template <bool MASSES>
__global__ __launch_bounds__(384) void k_ref_com_pairs(int64_t n_sel, const double *__restrict__ masses,
                                                       double mass_total, const double *__restrict__ ref,
                                                       double *__restrict__ info) {
  __shared__ double buf[3][2][kSeqBlk];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = w % 3;
  const bool chain = w < 3;  // waves 0-2 add, on three SIMDs; 3-5 form the terms
  const double s = pc_seq_sum(
      n_sel, buf[c], [&](int64_t a) { return SeqD1D{ref[3 * a + c], MASSES ? masses[a] : 1.0}; },
      [&](const SeqD1D &v, int64_t) { return v.x * v.d; }, chain);
  if (chain && (threadIdx.x & 63) == 0) info[c] = s / mass_total;
}

template <bool FROM_F32, bool GATHER, bool MASSES, int PART>
__global__ __launch_bounds__(kBlock) void k_ref_seq(const float *__restrict__ frame, const double *__restrict__ avg,
                                                    double div, int64_t n_sel, const int32_t *__restrict__ sel,
                                                    const double *__restrict__ masses, double mass_total,
                                                    double *__restrict__ avg_out, double *__restrict__ ref,
                                                    double *__restrict__ info) {
  __shared__ double com[3];
  __shared__ double slice[kBlock / 64][kRefSlice];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool lead = (threadIdx.x & 63) == 0;
  if (PART == kRefAll || PART == kRefCentre) {
    for (int64_t a = threadIdx.x; a < n_sel; a += kBlock)
      ref_fill_atom<FROM_F32, GATHER>(a, frame, avg, div, sel, avg_out, ref);
    __syncthreads();
  }
  if (PART != kRefSums) {
    if (w < 3) {  // three independent chains, one per axis
      const int c = w;
      const double s = wave_seq_sum(
          n_sel, slice[w], [&](int64_t a) { return SeqD1D{ref[3 * a + c], MASSES ? masses[a] : 1.0}; },
          [&](const SeqD1D &v, int64_t) { return v.x * v.d; });
      if (lead) info[c] = com[c] = s / mass_total;
    }
    if (PART == kRefCom) return;
    __syncthreads();
    const double c0 = com[0], c1 = com[1], c2 = com[2];
    for (int64_t a = threadIdx.x; a < n_sel; a += kBlock) {
      ref[3 * a] = ref[3 * a] - c0;
      ref[3 * a + 1] = ref[3 * a + 1] - c1;
      ref[3 * a + 2] = ref[3 * a + 2] - c2;
    }
    if (PART == kRefCentre) return;
    __syncthreads();
  }
  if (w < 3) {  // the sums of r, in order
    const int c = w;
    const double s = wave_seq_sum(
        n_sel, slice[w], [&](int64_t a) { return ref[3 * a + c]; }, [&](double r, int64_t) { return r; });
    if (lead) info[3 + c] = s;
  } else {
    const double g = wave_seq_sum(
        n_sel, slice[w], [&](int64_t a) { return SeqD3{ref[3 * a], ref[3 * a + 1], ref[3 * a + 2]}; },
        [&](const SeqD3 &r, int64_t) { return r.x * r.x + r.y * r.y + r.z * r.z; });
    if (lead) {
      info[6] = g;
      info[7] = mass_total;
      info[8] = (double)n_sel;
      for (int j = 9; j < 16; ++j) info[j] = 0.0;
    }
  }
}

// The per-frame superposition of exact=True (RMSF.py:94-97 / 127-131 +
// get_rotation_matrix, RMSF.py:43-51), one wave per (frame, chain):
//   k_seq_com: the frame's mobile COM (RMSF.py:94 / 127), atom by atom, chain
//     c the axis c; written to the record's [9..11];
//   k_seq_ip: qcprot's InnerProduct loop against the reference, chain j < 9
//     A[j] = sum_a x1_a[j/3] r_a[j%3], chain 9 G1 = sum_a ((x1 x1 + y1 y1) +
//     z1 z1), x1 = f64(x) - com (RMSF.py:95 / 128); A parked in the record's
//     [0..8], G1 in [13];
//   k_seq_qcp: E0 = (G1 + G2) * 0.5 and the QCP solve -> R in [0..8], rmsd in
//     [12], [13..15] zero.
// the frames' chains: seq_sum_in(slice, n, load, term), two waves (PC) or one
template <class Load, class Term>
__device__ __forceinline__ double seq_sum_in(double (*buf)[kSeqBlk], int64_t n, Load load, Term term) {
  return pc_seq_sum(n, buf, load, term);
}
template <class Load, class Term>
__device__ __forceinline__ double seq_sum_in(double *buf, int64_t n, Load load, Term term) {
  return wave_seq_sum(n, buf, load, term);
}
#define RMSF_SEQ_SUM(...) seq_sum_in(slice, __VA_ARGS__)
#define RMSF_SEQ_SLICE __shared__ std::conditional_t<PC, double[2][kSeqBlk], double[kSeqBlk]> slice

template <bool GATHER, bool MASSES, bool PC>
__global__ __launch_bounds__(PC ? 128 : 64) void k_seq_com(const float *__restrict__ xyz, int64_t fstride,
                                                           int64_t n_sel, const int32_t *__restrict__ sel,
                                                           const double *__restrict__ masses, double mass_total,
                                                           double *__restrict__ xform) {
  RMSF_SEQ_SLICE;
  const int64_t f = blockIdx.x;
  const int c = blockIdx.y;
  const float *__restrict__ fr = xyz + f * fstride + c;
  const double s = RMSF_SEQ_SUM(
      n_sel, [&](int64_t a) { return SeqF1D{fr[3 * (GATHER ? (int64_t)sel[a] : a)], MASSES ? masses[a] : 1.0}; },
      [&](const SeqF1D &v, int64_t) { return (double)v.x * v.d; });
  if (threadIdx.x == 0) xform[f * kXform + 9 + c] = s / mass_total;
}

template <bool GATHER, bool PC>
__global__ __launch_bounds__(PC ? 128 : 64) void k_seq_ip(const float *__restrict__ xyz, int64_t fstride,
                                                          int64_t n_sel, const int32_t *__restrict__ sel,
                                                          const double *__restrict__ ref, double *__restrict__ xform) {
  RMSF_SEQ_SLICE;
  const int64_t f = blockIdx.x;
  const int j = blockIdx.y;
  const float *__restrict__ fr = xyz + f * fstride;
  const double *t = xform + f * kXform;
  auto row = [&](int64_t a) -> int64_t { return 3 * (GATHER ? (int64_t)sel[a] : a); };
  double s;
  if (j < 9) {
    const int ax = j / 3, rb = j % 3;
    const double cx = t[9 + ax];
    s = RMSF_SEQ_SUM(
        n_sel, [&](int64_t a) { return SeqF1D{fr[row(a) + ax], ref[3 * a + rb]}; },
        [&](const SeqF1D &v, int64_t) { return ((double)v.x - cx) * v.d; });
  } else {
    const double c0 = t[9], c1 = t[10], c2 = t[11];
    s = RMSF_SEQ_SUM(
        n_sel,
        [&](int64_t a) {
          const float *p = fr + row(a);
          return SeqF3{p[0], p[1], p[2]};
        },
        [&](const SeqF3 &v, int64_t) {
          const double x1 = (double)v.x - c0, y1 = (double)v.y - c1, z1 = (double)v.z - c2;
          return x1 * x1 + y1 * y1 + z1 * z1;
        });
  }
  if (threadIdx.x == 0) xform[f * kXform + (j < 9 ? j : 13)] = s;
}
#undef RMSF_SEQ_SUM
#undef RMSF_SEQ_SLICE

__global__ __launch_bounds__(64) void k_seq_qcp(int64_t n_frames, int64_t n_sel, const double *__restrict__ refinfo,
                                                double *__restrict__ xform) {
  const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (f >= n_frames) return;
  double *t = xform + f * kXform;
  double A[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) A[j] = t[j];
  const double E0 = (t[13] + refinfo[6]) * 0.5;
  double rot[9], rmsd;
  qcp_solve(A, E0, (double)n_sel, rot, &rmsd);
#pragma unroll
  for (int j = 0; j < 9; ++j) t[j] = rot[j];
  t[12] = rmsd;
  t[13] = t[14] = t[15] = 0.0;
}

// k_accum_seq: one selected atom per lane, the batch's frames in order
// (k = k0 + f), each frame's transform applied (ALIGN, RMSF.py:99-101 /
// 133-135) and then
//   SUM:     pos += x                                  (RMSF.py:103)
//   WELFORD: sumsquares += (k / (k + 1.0)) * (x - mean)**2 ;
//            mean = (k * mean + x) / (k + 1)            (RMSF.py:137-138)
// with numpy's operations and roundings -- k_welford_seq_atoms' recurrence,
// the running state continued from acc0/acc1 when k0 > 0.  U frames' loads
// are issued before they are consumed.
template <int MODE, bool ALIGN, bool GATHER, int U>
__global__ __launch_bounds__(kBlock) void k_accum_seq(const float *__restrict__ xyz, int64_t fstride, int64_t nf,
                                                      int64_t n_sel, const int32_t *__restrict__ sel,
                                                      const double *__restrict__ xform,
                                                      const double *__restrict__ refinfo, int64_t k0,
                                                      const SeqCoef *__restrict__ coef, double *__restrict__ acc0,
                                                      double *__restrict__ acc1) {
  const int64_t a = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a >= n_sel) return;
  const double rc0 = ALIGN ? refinfo[0] : 0.0, rc1 = ALIGN ? refinfo[1] : 0.0, rc2 = ALIGN ? refinfo[2] : 0.0;
  double m[3], q[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    m[c] = k0 > 0 ? acc0[3 * a + c] : 0.0;
    if (MODE == RMSF_MODE_WELFORD && k0 > 0) q[c] = acc1[3 * a + c];
  }
  const float *__restrict__ p = xyz + 3 * (GATHER ? (int64_t)sel[a] : a);
  auto consume = [&](float x, float y, float z, int64_t f, double k) {
    if (ALIGN) apply_xform(x, y, z, xform + f * kXform, rc0, rc1, rc2);
    const float v[3] = {x, y, z};
    if (MODE == RMSF_MODE_SUM) {
#pragma unroll
      for (int c = 0; c < 3; ++c) m[c] = m[c] + (double)v[c];
    } else {
      const SeqCoef cf = coef[f];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const double xx = (double)v[c];
        const double d = xx - m[c];
        q[c] = q[c] + cf.c * (d * d);
        m[c] = seq_div(k * m[c] + xx, k + 1.0, cf.r);
      }
    }
  };
  int64_t f = 0;
  double kb = (double)k0;
  for (; f + U <= nf; f += U) {
    float v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float *r = p + (f + u) * fstride;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[u][c] = __builtin_nontemporal_load(r + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u, kb += 1.0) consume(v[u][0], v[u][1], v[u][2], f + u, kb);
  }
  for (; f < nf; ++f, kb += 1.0) {
    const float *r = p + f * fstride;
    consume(r[0], r[1], r[2], f, kb);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    acc0[3 * a + c] = m[c];
    if (MODE == RMSF_MODE_WELFORD) acc1[3 * a + c] = q[c];
  }
}

template <int MODE, bool ALIGN, bool GATHER, int U, bool PLANES = false>
__global__ __launch_bounds__(kBlock) void k_accum_atoms_sk(const float *__restrict__ xyz, int64_t fstride,
                                                           const int32_t *__restrict__ sel,
                                                           const double *__restrict__ xform,
                                                           const double *__restrict__ refinfo, SkPlan pl,
                                                           int64_t *__restrict__ hdr, double *__restrict__ parts0,
                                                           double *__restrict__ parts1, int64_t ps = 0) {
  const int b = sk_range(pl, blockIdx.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) sk_write_header(hdr, pl);
  const double rc0 = ALIGN ? refinfo[0] : 0.0, rc1 = ALIGN ? refinfo[1] : 0.0, rc2 = ALIGN ? refinfo[2] : 0.0;
  int64_t lo = uni64(sk_lo(pl, b));
  const int64_t hi = uni64(sk_lo(pl, b + 1));
  int64_t slot = (int64_t)b * pl.P;
  while (lo < hi) {
    int64_t c, f0;
    const int len = __builtin_amdgcn_readfirstlane((int)sk_seg_len(pl, lo, hi, &c, &f0));
    c = uni64(c);
    f0 = uni64(f0);
    const int64_t a = c * kBlock + threadIdx.x;
    if (a < pl.lanes) {
      const int64_t off = (PLANES ? 1 : 3) * (GATHER ? (int64_t)sel[a] : a);
      double m[3], q[3];
      accum_atoms_run<MODE, ALIGN, U, PLANES>(xyz + f0 * fstride + off, fstride, len,
                                              ALIGN ? xform + f0 * kXform : nullptr, rc0, rc1, rc2, m, q, ps);
      const int64_t o = slot * (kBlock * 3) + 3 * threadIdx.x;
      store3<MODE>(parts0 + o, parts1 + o, m, q);
    }
    lo += len;
    ++slot;
  }
}

// accum_span: frames [0, nf) from p (one selected atom per lane), adding to
// m/q: WELFORD shifted sums (S1 += d, S2 += d^2, d = x - sh), SUM plain sums.
// xf = frame 0's transform record.
template <int MODE, bool ALIGN, int U, bool PLANES = false>
__device__ __forceinline__ void accum_span(const float *__restrict__ p, int64_t fstride, int nf,
                                           const double *__restrict__ xf, double rc0, double rc1, double rc2,
                                           const double (&sh)[3], double (&m)[3], double (&q)[3], int64_t ps = 0) {
  const int64_t cs = PLANES ? ps : 1;  // x -> y -> z of the lane's atom
  auto consume = [&](float x, float y, float z, int k) {
    if (ALIGN) apply_xform(x, y, z, xf + (int64_t)k * kXform, rc0, rc1, rc2);
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
      vy[u] = __builtin_nontemporal_load(r + cs);
      vz[u] = __builtin_nontemporal_load(r + 2 * cs);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) consume(vx[u], vy[u], vz[u], k + u);
  }
  for (; k < nf; ++k) {
    const float *r = p + (int64_t)k * fstride;
    consume(r[0], r[cs], r[2 * cs], k);
  }
}

// k_accum_split_sk: the balanced grid of k_accum_atoms_sk with the frames of
// every segment split over Q sub-blocks of Q*256 threads (each sub-block the
// chunk's 256 atoms, a contiguous Q-th of the segment's frames).  The
// sub-blocks share one shift (the segment's first frame after the
// transform), so their shifted sums add: sub-blocks 1..Q-1 leave theirs in
// LDS and sub-block 0 adds them in that order (deterministic) and stores ONE
// partial per segment.  Q x fewer partials at the same wave count: at 8,192
// ranges x 2 segments the partials are 196 MB per launch, which the fold
// reads back -- 6 % of a 2,500-frame share (tools/ubench_accum3.hip).
template <int MODE, bool ALIGN, bool GATHER, int U, int Q, bool PLANES = false>
__global__ __launch_bounds__(kBlock *Q) void k_accum_split_sk(const float *__restrict__ xyz, int64_t fstride,
                                                              const int32_t *__restrict__ sel,
                                                              const double *__restrict__ xform,
                                                              const double *__restrict__ refinfo, SkPlan pl,
                                                              int64_t *__restrict__ hdr,
                                                              double *__restrict__ parts0,
                                                              double *__restrict__ parts1, int64_t ps = 0) {
  static_assert(Q > 1 && RMSF_SHIFTED_SUMS, "k_accum_split_sk combines shifted sums of Q > 1 sub-blocks");
  constexpr int NV = MODE == RMSF_MODE_WELFORD ? 6 : 3;  // doubles per lane handed over
  __shared__ double red[(Q - 1) * NV * kBlock];
  const int b = sk_range(pl, blockIdx.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) sk_write_header(hdr, pl);
  const int li = threadIdx.x % kBlock;
  const int qd = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kBlock));
  const double rc0 = ALIGN ? refinfo[0] : 0.0, rc1 = ALIGN ? refinfo[1] : 0.0, rc2 = ALIGN ? refinfo[2] : 0.0;
  int64_t lo = uni64(sk_lo(pl, b));
  const int64_t hi = uni64(sk_lo(pl, b + 1));
  int64_t slot = (int64_t)b * pl.P;
  while (lo < hi) {
    int64_t c, f0;
    const int len = __builtin_amdgcn_readfirstlane((int)sk_seg_len(pl, lo, hi, &c, &f0));
    c = uni64(c);
    f0 = uni64(f0);
    const int64_t a = c * kBlock + li;
    const bool live = a < pl.lanes;  // no early exit: every thread meets the barriers
    const int s0 = (int)((int64_t)len * qd / Q), s1 = (int)((int64_t)len * (qd + 1) / Q);
    double m[3] = {0.0, 0.0, 0.0}, q[3] = {0.0, 0.0, 0.0}, sh[3] = {0.0, 0.0, 0.0};
    if (live) {
      const float *p = xyz + f0 * fstride + (PLANES ? 1 : 3) * (GATHER ? (int64_t)sel[a] : a);
      if (MODE == RMSF_MODE_WELFORD) {
        const int64_t cs = PLANES ? ps : 1;
        float x = p[0], y = p[cs], z = p[2 * cs];
        if (ALIGN) apply_xform(x, y, z, xform + f0 * kXform, rc0, rc1, rc2);
        sh[0] = (double)x, sh[1] = (double)y, sh[2] = (double)z;
      }
      accum_span<MODE, ALIGN, U, PLANES>(p + (int64_t)s0 * fstride, fstride, s1 - s0,
                                         ALIGN ? xform + (f0 + s0) * kXform : nullptr, rc0, rc1, rc2, sh, m, q, ps);
    }
    if (qd > 0) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        red[((qd - 1) * NV + j) * kBlock + li] = m[j];
        if (MODE == RMSF_MODE_WELFORD) red[((qd - 1) * NV + 3 + j) * kBlock + li] = q[j];
      }
    }
    __syncthreads();
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
        const double inv = g_coef.v[len - 1].b;  // 1/len
#pragma unroll
        for (int j = 0; j < 3; ++j) shifted_to_moments(m[j], q[j], sh[j], inv);
      }
      const int64_t o = slot * (kBlock * 3) + 3 * li;
      store3<MODE>(parts0 + o, parts1 + o, m, q);
    }
    __syncthreads();  // red is rewritten by the next segment
    lo += len;
    ++slot;
  }
}

// Fold the balanced partials of one batch, in frame order, into the running
// result (acc_n frames already in acc0/acc1; 0 = overwrite): Chan's merge
// (second_order_moments, RMSF.py:36-41) for WELFORD, a sum for SUM.  One
// thread per lane (its cpl = 3 or 4 coordinates, which share the segment
// walk); it replays the walk of the workgroups that cover its chunk in a
// fixed order (bitwise reproducible) and loads the partials of up to
// kFoldBatch segments before folding any of them, so a chunk covered by a
// few ranges costs one memory round trip, not one per segment.  The walk is
// uniform per wave (a chunk is 256 lanes), its divisions stay off the
// critical path of the loads.
//
// PACK (N > 1, WELFORD only): the fold also writes the moments about the
// merge's shift c that the one-all-reduce merge sums (k_chan_shift_pack's
// T1/T2, same arithmetic: shift_moments), so the pack needs no launch of its
// own.  PACK = 1: float32 shift, 2: float64 shift; c = shift[j] (+ off3[j % 3]).
constexpr int kFoldBatch = 4;

// T1 = n (mean - c), T2 = M2 + n (mean - c)^2, the rounding fixed by explicit
// operations (the standalone pack and the fused fold must agree bit for bit)
__device__ __forceinline__ void shift_moments(double mu, double M2, double c, double nk, double *t1, double *t2) {
  const double d = mu - c;
  *t1 = nk * d;
  *t2 = __builtin_fma(nk, d * d, M2);
}

// Where coordinate j's T1 goes in a merge buffer: the plain layout [T1 | T2]
// (t_slice = 0: T1 at j, T2 at j + n), or the atom-sliced layout of the
// reduce-scatter merge (t_slice = 3 x atoms per rank): slice r = j / t_slice
// holds [T1 | T2] of its t_slice coordinates, T2 t_slice after T1.
__device__ __forceinline__ int64_t slice_t1(int64_t j, int64_t t_slice) {
  const int64_t r = j / t_slice;
  return 2 * r * t_slice + (j - r * t_slice);
}

// FIN: also the finalise of RMSF.py:146 for an atom plan (cpl = 3: lane l is
// atom l), rmsf[l] = sqrt((M2x + M2y + M2z) / n_total) -- k_finalize's
// expression on the values just stored, so bit-identical to it, one launch
// fewer.  A flat plan (cpl = 4: an atom's coordinates span two lanes) writes
// no RMSF here; k_finalize_flat, launched after it, finalises that plan.
template <int PACK, bool FIN = false>
__global__ __launch_bounds__(kBlock) void k_fold_sk(const int64_t *__restrict__ hdr,
                                                    const double *__restrict__ parts0, int64_t n_coord,
                                                    double acc_n, double *__restrict__ acc0,
                                                    double *__restrict__ acc1, const void *__restrict__ shift,
                                                    const double *__restrict__ off3, double *__restrict__ t,
                                                    int64_t l_off, int64_t l_end, int64_t t_n, int64_t t_slice,
                                                    double *__restrict__ rmsf = nullptr, double n_total = 0.0) {
  // lanes [l_off, l_end) (an atom slab; 0, INT64_MAX = all).  T1/T2 of the
  // slab's coordinates go to t[j - j_lo] and t[t_n + j - j_lo]; with t_slice
  // (whole range only) to the atom-sliced layout of slice_t1.
  const int64_t l = l_off + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  SkPlan pl;
  pl.lanes = hdr[0];
  pl.C = hdr[1];
  pl.nf = hdr[2];
  pl.T = hdr[3];
  pl.G = (int)hdr[4];
  pl.P = (int)hdr[5];
  pl.cpl = (int)hdr[6];
  pl.mode = (int)hdr[7];
  pl.S = (int)hdr[8];
  pl.cw = (int)hdr[9];
  if (l >= pl.lanes || l >= l_end) return;
  const int cpl = pl.cpl;
  const int64_t j0 = l * cpl;  // first coordinate of the lane
  const int nx = (int)(n_coord - j0 < cpl ? n_coord - j0 : cpl);
  const int64_t c = l / pl.cw;
  const int64_t slot_d = (int64_t)pl.cw * pl.cpl;
  const int64_t off = j0 - c * slot_d;
  const int64_t clo = c * pl.nf, chi = clo + pl.nf;
  const double *__restrict__ parts1 = parts0 + (int64_t)pl.G * pl.P * slot_d;
  const bool wel = pl.mode == RMSF_MODE_WELFORD;
  // the merge's shift, loaded before the walk so its latency hides behind it
  double cs[4] = {0.0, 0.0, 0.0, 0.0};
  if (PACK) {
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      if (x < nx) {
        const int64_t j = j0 + x;
        double c = PACK == 1 ? (double)static_cast<const float *>(shift)[j] : static_cast<const double *>(shift)[j];
        if (off3) c += off3[j % 3];
        cs[x] = c;
      }
    }
  }
  double n1 = acc_n, mu[4] = {0.0, 0.0, 0.0, 0.0}, M[4] = {0.0, 0.0, 0.0, 0.0};
  if (acc_n > 0) {
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      if (x < nx) {
        mu[x] = acc0[j0 + x];
        if (wel) M[x] = acc1[j0 + x];
      }
    }
  }
  // first range whose end is past the chunk's start, walked from its start
  int64_t b = clo * pl.G / pl.T;
  while (b > 0 && sk_lo(pl, b) > clo) --b;
  while (sk_lo(pl, b + 1) <= clo) ++b;
  int64_t lo = sk_lo(pl, b), hi = sk_lo(pl, b + 1), slot = b * pl.P;
  while (lo < clo) {
    int64_t cc, f0;
    lo += sk_seg_len(pl, lo, hi, &cc, &f0);
    ++slot;
  }
  for (;;) {
    int64_t sl[kFoldBatch];
    double ln[kFoldBatch];
    int n = 0;
    while (n < kFoldBatch) {
      if (lo >= hi) {
        if (++b >= pl.G) break;
        lo = sk_lo(pl, b);
        hi = sk_lo(pl, b + 1);
        slot = b * pl.P;
      }
      if (lo >= chi) break;
      int64_t cc, f0;
      const int64_t len = sk_seg_len(pl, lo, hi, &cc, &f0);
      sl[n] = slot;
      ln[n] = (double)len;
      ++n;
      lo += len;
      ++slot;
    }
    double pm[kFoldBatch][4], pq[kFoldBatch][4];
#pragma unroll
    for (int k = 0; k < kFoldBatch; ++k) {
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        if (k < n && x < nx) {
          const int64_t o = sl[k] * slot_d + off + x;
          pm[k][x] = parts0[o];
          pq[k][x] = wel ? parts1[o] : 0.0;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kFoldBatch; ++k) {
      if (k < n) {
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          if (x >= nx) continue;
          if (!wel) {
            mu[x] += pm[k][x];
          } else if (n1 <= 0) {
            mu[x] = pm[k][x];
            M[x] = pq[k][x];
          } else {
            const double n2 = ln[k], mu2 = pm[k][x], M2 = pq[k][x];
            const double T = n1 + n2;
            const double d = mu2 - mu[x];
            const double mun = (n1 * mu[x] + n2 * mu2) / T;
            M[x] = M[x] + M2 + (n1 * n2 / T) * (d * d);
            mu[x] = mun;
          }
        }
        if (wel) n1 = n1 <= 0 ? ln[k] : n1 + ln[k];
      }
    }
    if (n < kFoldBatch) break;
  }
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    if (x < nx) {
      acc0[j0 + x] = mu[x];
      if (wel) acc1[j0 + x] = M[x];
    }
  }
  if (FIN && cpl == 3 && nx == 3) rmsf[l] = sqrt((M[0] + M[1] + M[2]) / n_total);
  if (PACK) {
    const double nk = acc_n + (double)pl.nf;  // frames folded in: this rank's n_k
    if (t_slice > 0) {
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        if (x < nx) {
          double *t1 = t + slice_t1(j0 + x, t_slice);
          shift_moments(mu[x], M[x], cs[x], nk, t1, t1 + t_slice);
        }
      }
    } else {
      double *t1 = t + (j0 - l_off * cpl), *t2 = t1 + t_n;
#pragma unroll
      for (int x = 0; x < 4; ++x)
        if (x < nx) shift_moments(mu[x], M[x], cs[x], nk, t1 + x, t2 + x);
    }
  }
}

// ---------------------------------------------------------------------------
// Wave / block reductions (64-wide waves).
template <int N>
__device__ __forceinline__ void wave_sum(double (&v)[N]) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] += __shfl_xor(v[j], off, 64);
  }
}

// k_frame_stats -- "lanes over frames" on a balanced grid.
// Work units: (64-frame group g, 32-atom tile t); unit u = g*ntiles + t
// (group-major).  Workgroup b takes the equal contiguous range
// [T b / G, T (b+1) / G) of the T = ngroups*ntiles units and walks it as
// segments (maximal runs inside one frame group); each segment writes one
// partial -- 16 sums x 64 frames -- into slot b*P + j (j = segment index in
// the workgroup).  Equal ranges leave no tail wave, and the partials stay
// small (G*P slots, independent of the trajectory length).
// Inside a segment: lane = frame, the 4 waves of the block split each
// 32-atom tile that is staged HBM -> registers -> LDS (pitch 100 dwords:
// 16-B rows, conflict-free ds_read_b128 column reads), with the next tile's
// loads in flight.  The atom index is wave-uniform, so the f64 reference and
// masses arrive by scalar loads and no per-atom cross-lane reduction exists:
// each lane owns its frame's sums.  Sums are relative to a per-frame pivot p
// (the frame's first selected atom, for conditioning):
//   [0..2]  sum x'            [3..5]  sum m x'   (only with masses)
//   [6..14] sum x'_a r_b      [15]    sum |x'|^2
// Epilogue: the 4 waves' sums meet in LDS and all 256 threads add them (wave
// order 0..3, fixed) and store the partial stat-major, [16][64] -- every
// store instruction writes 512 contiguous bytes.  (The former epilogue, wave
// 0 alone storing 16 doubles per lane at a 128-B lane stride, cost 3-18 % of
// the kernel: tools/ubench_stats2.hip.)
// VEC4: contiguous selection, 16-B aligned frames -> float4 staging loads;
// otherwise (gathered selection / odd strides) element-wise staging loads.
constexpr int kTF = 64;                    // frames per block (one per lane)
constexpr int kTA = 32;                    // atoms per tile
constexpr int kPitch = 3 * kTA + 4;        // LDS row pitch (dwords): 16-B rows, conflict-free b128 column reads
constexpr int kRow4 = 3 * kTA / 4;         // float4 per tile row
constexpr int kNPre = kTF * kRow4 / kBlock;  // float4 per thread per tile (VEC4)
constexpr int kNEl = kTF * kTA / kBlock;     // atoms per thread per tile (element path)
constexpr int kAPW = kTA / 4;              // atoms per wave per tile
constexpr int kStatsLds = (kTF * kPitch > 2 * (kBlock / 64) * kStats * kTF) ? kTF * kPitch : 2 * (kBlock / 64) * kStats * kTF;
static_assert(kTF * kRow4 % kBlock == 0 && kTF * kTA % kBlock == 0, "tile shape");
static_assert(kStats * kTF % kBlock == 0, "epilogue: whole outputs per thread");

// balanced-grid plan of k_frame_stats (computed identically on the host for
// the launch and for k_qcp_frames' fold)
struct StatsPlan {
  int64_t ntiles, ngroups, T;
  int G, P;
};

__host__ __device__ inline int64_t st_lo(const StatsPlan &p, int64_t b) { return p.T * b / p.G; }

// PLANES: frames stored as coordinate planes (x[n], y[n], z[n], ps floats
// apart; SoA).  The element path gathers each atom's three plane values into
// the same (atom, xyz) tile rows; the VEC4 path stages each tile row as
// [x(32) | y(32) | z(32)] (three 128-B plane segments per frame, the same
// 24 float4 per row) and its 4-atom groups read one float4 of each plane.
template <bool GATHER, bool MASSES, bool VEC4, int WPE = 1, bool PLANES = false, int DENSE = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void k_frame_stats(
    const float *__restrict__ xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
    const int32_t *__restrict__ sel, const double *__restrict__ masses, const double *__restrict__ ref,
    StatsPlan pl, double *__restrict__ part, int64_t ps = 0, float *__restrict__ dense = nullptr,
    int64_t dpitch = 0) {
  static_assert(DENSE == 0 || (GATHER && !PLANES && !VEC4), "the dense copy is of gathered (frame, atom, xyz) rows");
  __shared__ __attribute__((aligned(16))) float tile[kStatsLds];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t last = n_frames - 1;
  const int64_t o0 = GATHER ? (PLANES ? 1 : 3) * (int64_t)sel[0] : 0;
  const int64_t cs = PLANES ? ps : 1;  // x -> y -> z of one atom
  const int64_t lim = 3 * n_sel;  // floats of the selection inside a frame row (VEC4)
  int64_t lo = uni64(st_lo(pl, blockIdx.x));
  const int64_t hi = uni64(st_lo(pl, blockIdx.x + 1));
  int64_t slot = (int64_t)blockIdx.x * pl.P;
  while (lo < hi) {
    const int64_t g = uni64(lo / pl.ntiles);
    const int64_t t_lo = lo - g * pl.ntiles;
    const int64_t t_hi = min(pl.ntiles, t_lo + (hi - lo));
    const int64_t f0 = g * kTF;
    const int64_t a_beg = t_lo * kTA, a_end = min(n_sel, t_hi * kTA);
    const float *myfr = xyz + min(f0 + lane, last) * fstride;
    const double px = myfr[o0], py = myfr[o0 + cs], pz = myfr[o0 + 2 * cs];
    double acc[kStats];
#pragma unroll
    for (int j = 0; j < kStats; ++j) acc[j] = 0.0;

    f32x4 pre[VEC4 ? kNPre : 1];
    float pel[VEC4 ? 1 : 3 * kNEl];
    // element path: this thread's atom of the tile at t0 (clamped to the
    // segment's last atom), as its index in the frame rows.  Loaded one tile
    // ahead and scaled only where gload uses it: scaling it right after the
    // load would make the wave wait for that load -- and so for every store
    // issued before it -- at the end of each tile.
    using EAtom = std::conditional_t<GATHER, int32_t, int64_t>;
    auto elem_atom = [&](int64_t t0) -> EAtom {
      const int64_t a = min(t0 + (int64_t)(threadIdx.x % kTA), a_end - 1);
      if constexpr (GATHER) return sel[a];
      else return a;
    };
    EAtom eatom = VEC4 ? 0 : elem_atom(a_beg);
    auto gload = [&](int64_t t0) {
      if (VEC4) {
#pragma unroll
        for (int k = 0; k < kNPre; ++k) {
          const int idx = threadIdx.x + k * kBlock;
          const int row = idx / kRow4, col = idx % kRow4;
          const float *src = xyz + min(f0 + row, last) * fstride;
          if (PLANES) {  // col 0-7: x plane, 8-15: y, 16-23: z; 4 atoms each
            const int64_t a = t0 + 4 * (col % 8);
            const float *q = src + (col / 8) * ps + a;
            if (a + 3 < n_sel) {
              pre[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(q));
            } else {  // selection tail
              pre[k] = f32x4{a < n_sel ? q[0] : 0.f, a + 1 < n_sel ? q[1] : 0.f, a + 2 < n_sel ? q[2] : 0.f, 0.f};
            }
            continue;
          }
          const int64_t e = 3 * t0 + 4 * col;
          if (e + 3 < lim) {
            pre[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(src + e));
          } else {  // selection tail: never read past the selection
            pre[k] = f32x4{e < lim ? src[e] : 0.f, e + 1 < lim ? src[e + 1] : 0.f, e + 2 < lim ? src[e + 2] : 0.f, 0.f};
          }
        }
      } else {
        // kBlock % kTA == 0: a thread stages the same atom j of every row it
        // loads, so one offset serves its kNEl rows.  The offset (the
        // selection index) was loaded one tile ahead (eatom), and no load is
        // conditional: past the segment's last atom the thread re-reads that
        // atom, whose tile slots neither the sums nor the dense copy read.
        // (The per-row `if (a < a_end)` form compiled to an index load, a
        // vmcnt(0), the coordinate load and another vmcnt(0) per row: 16
        // serial round trips per tile.)
        // (the empty asm pins the first use of the loaded index here, so its
        // widening is not hoisted to the load)
        if constexpr (GATHER) asm volatile("" : "+v"(eatom));
        const int64_t off = (PLANES ? 1 : 3) * (int64_t)eatom;
#pragma unroll
        for (int k = 0; k < kNEl; ++k) {
          const int row = (threadIdx.x + k * kBlock) / kTA;
          const float *src = xyz + min(f0 + row, last) * fstride + off;
          pel[3 * k] = __builtin_nontemporal_load(src);
          pel[3 * k + 1] = __builtin_nontemporal_load(src + cs);
          pel[3 * k + 2] = __builtin_nontemporal_load(src + 2 * cs);
        }
        eatom = elem_atom(t0 + kTA);
      }
    };
    auto lstore = [&]() {
      if (VEC4) {
#pragma unroll
        for (int k = 0; k < kNPre; ++k) {
          const int idx = threadIdx.x + k * kBlock;
          const int row = idx / kRow4, col = idx % kRow4;
          *reinterpret_cast<f32x4 *>(tile + row * kPitch + 4 * col) = pre[k];
        }
      } else {
#pragma unroll
        for (int k = 0; k < kNEl; ++k) {
          const int idx = threadIdx.x + k * kBlock;
          const int row = idx / kTA, j = idx % kTA;
          float *d = tile + row * kPitch + 3 * j;
          d[0] = pel[3 * k];
          d[1] = pel[3 * k + 1];
          d[2] = pel[3 * k + 2];
        }
      }
    };
    // Compaction (rmsf_superpose_compact, DENSE): every (frame, selected
    // atom) is staged exactly once over the grid, so the staged tile goes
    // out once too, to the dense copy the later passes read instead of
    // re-gathering (an exact copy: same bits).  From LDS, after the next
    // tile's loads are issued: a frame's 32 atoms are 384 contiguous bytes of
    // the copy.  Writing the copy here beats a stand-alone gather before a
    // dense covariance pass (ratios to re-gathering on one box,
    // profiles/r06_workloads/).
    // The copy costs +1.4-1.8 ms at 10k of 100k atoms x 20k frames for its
    // 2.43 GB (3.8e7 64-B writes) beside the gathered read, where the bytes
    // alone would take 0.4 ms.  None of the kernel-side levers moved it:
    // store forms and row pitches, storing before or after the next tile's
    // loads or after the tile's sums, from one wave or all, keeping the
    // stores in flight across the next wait (a fixed count per tile), and 2
    // or 3 waves per SIMD all measured the same
    // (profiles/r06_workloads/ab_dense_store_split.txt, pmc_dense_store.txt:
    // instruction-issue waits +1.6e9 cycles and L1 pending stalls +46 %).
    // the segment's last tile, whole or not
    auto dense_last = [&](int64_t t0) {
      const int nfl = 3 * (int)min((int64_t)kTA, a_end - t0);
      for (int idx = threadIdx.x; idx < kTF * 3 * kTA; idx += kBlock) {
        const int row = idx / (3 * kTA), e = idx - row * (3 * kTA);
        if (e < nfl && f0 + row <= last)
          __builtin_nontemporal_store(tile[row * kPitch + e], dense + (f0 + row) * dpitch + 3 * t0 + e);
      }
    };
    // DENSE 2: threads 0..239 own one float4 column (t % 24) of rows t / 24 +
    // 10 k, so a thread's copy addresses are one base plus constant strides:
    // few registers, and the kernel keeps 3 waves per SIMD (WPE 3) as the
    // re-gathering kernel does.  (Measured equal to 2 waves per SIMD with
    // per-row addresses, ab_dense_store_split.txt: the copy's cost is not
    // occupancy.)  DENSE 1 (a copy pitch not 16-B aligned; only through the
    // ABI) takes the general loop.
    auto dense_whole = [&](int64_t t0) {
      if constexpr (DENSE == 2) {
        constexpr int kRows = kBlock / kRow4;  // 10 rows per pass
        if (threadIdx.x < kRows * kRow4) {
          const int col = threadIdx.x % kRow4, r0 = threadIdx.x / kRow4;
          const float *src = tile + r0 * kPitch + 4 * col;
          f32x4 *dst = reinterpret_cast<f32x4 *>(dense + (f0 + r0) * dpitch + 3 * t0) + col;
          const int64_t step4 = kRows * dpitch / 4;
#pragma unroll
          for (int k = 0; k < (kTF + kRows - 1) / kRows; ++k) {
            const int row = r0 + kRows * k;
            if (row < kTF && f0 + row <= last)
              __builtin_nontemporal_store(*reinterpret_cast<const f32x4 *>(src + kRows * kPitch * k), dst + step4 * k);
          }
        }
      } else {
        dense_last(t0);
      }
    };
    // one 4-atom group of this wave's slab (atoms a4..a4+3, a wave-uniform index)
    auto group = [&](const f32x4 *my, int gi, int64_t a4, int n_at) {
      float c[12];
      if (PLANES && VEC4) {  // my = the row; this wave's group gi = float4 (2w + gi) of each plane segment
        const f32x4 qx = my[2 * w + gi], qy = my[8 + 2 * w + gi], qz = my[16 + 2 * w + gi];
        const float cp[12] = {qx.x, qy.x, qz.x, qx.y, qy.y, qz.y, qx.z, qy.z, qz.z, qx.w, qy.w, qz.w};
#pragma unroll
        for (int j = 0; j < 12; ++j) c[j] = cp[j];
      } else {
        const f32x4 q0 = my[3 * gi], q1 = my[3 * gi + 1], q2 = my[3 * gi + 2];
        const float cr[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
#pragma unroll
        for (int j = 0; j < 12; ++j) c[j] = cr[j];
      }
      const double *rr = ref + 3 * a4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i >= n_at) break;  // uniform; n_at < 4 only in the selection's last tile
        const double r0 = rr[3 * i], r1 = rr[3 * i + 1], r2 = rr[3 * i + 2];
        const double x = (double)c[3 * i] - px, y = (double)c[3 * i + 1] - py, z = (double)c[3 * i + 2] - pz;
        acc[0] += x;
        acc[1] += y;
        acc[2] += z;
        if (MASSES) {
          const double m = masses[a4 + i];
          acc[3] = fma(m, x, acc[3]);
          acc[4] = fma(m, y, acc[4]);
          acc[5] = fma(m, z, acc[5]);
        }
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
    };

    const f32x4 *my = reinterpret_cast<const f32x4 *>(tile + lane * kPitch + (PLANES && VEC4 ? 0 : w * 3 * kAPW));
    // The segment's last tile is peeled, so the next tile's loads in the
    // loop are unconditional.  (Behind an `if (t0 + kTA < a_end)` the
    // element path's loaded values met the loop-carried ones in a phi, and
    // the copies resolving it waited for the loads right after issuing
    // them: no load was in flight across the tile's sums.)
    auto step = [&](int64_t t0) {  // a whole tile with a successor
      __syncthreads();
      lstore();
      __syncthreads();
      gload(t0 + kTA);
      if constexpr (DENSE != 0) dense_whole(t0);
      const int64_t ab = t0 + w * kAPW;  // first atom of this wave's slab (uniform)
#pragma unroll 1
      for (int gi = 0; gi < kAPW / 4; ++gi) group(my, gi, ab + 4 * gi, 4);
    };
    gload(a_beg);
    int64_t t0 = a_beg;
    for (; t0 + kTA < a_end; t0 += kTA) step(t0);
    {  // the last tile, whole or not
      __syncthreads();
      lstore();
      __syncthreads();
      if constexpr (DENSE != 0) dense_last(t0);
      const int64_t ab = t0 + w * kAPW;
#pragma unroll 1
      for (int gi = 0; gi < kAPW / 4; ++gi) {
        const int64_t a4 = ab + 4 * gi;
        if (a4 >= a_end) break;  // uniform
        group(my, gi, a4, (int)min((int64_t)4, a_end - a4));
      }
    }
    // the 4 waves' sums meet in LDS (the tile buffer is free after this
    // barrier); thread t then adds outputs o = t + 256 k (o = stat*64 + frame)
    __syncthreads();
    double *red = reinterpret_cast<double *>(tile);
#pragma unroll
    for (int j = 0; j < kStats; ++j) red[(w * kStats + j) * kTF + lane] = acc[j];
    __syncthreads();
    double *out = part + slot * (kStats * kTF);
#pragma unroll
    for (int k = 0; k < kStats * kTF / kBlock; ++k) {
      const int o = threadIdx.x + k * kBlock;
      double t = red[o];
#pragma unroll
      for (int v = 1; v < kBlock / 64; ++v) t += red[v * kStats * kTF + o];
      nt_store(t, out + o);
    }
    lo += t_hi - t_lo;
    ++slot;
  }
}

// k_qcp_frames: one wave per frame.  Folds the chunk partials in a fixed
// order (deterministic), forms COM / A / E0 and solves QCP on lane 0.
template <bool GATHER, bool MASSES, bool PLANES = false>
__global__ __launch_bounds__(kBlock) void k_qcp_frames(
    const double *__restrict__ part, StatsPlan pl, int64_t n_frames, const float *__restrict__ xyz,
    int64_t fstride, const int32_t *__restrict__ sel, const double *__restrict__ refinfo,
    double *__restrict__ xform, int64_t ps = 0) {
  const int64_t f = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (f >= n_frames) return;
  // the workgroups whose ranges cover frame group g (units [g*ntiles,
  // (g+1)*ntiles)): b0.. while their range starts inside it; workgroup b's
  // segment for g is its (g - first group of b)-th
  const int64_t g = f / kTF, fl = f - g * kTF;
  const int64_t ulo = g * pl.ntiles, uhi = ulo + pl.ntiles;
  int64_t b0 = ulo * pl.G / pl.T;
  while (b0 > 0 && st_lo(pl, b0) > ulo) --b0;
  while (st_lo(pl, b0 + 1) <= ulo) ++b0;
  double s[kStats];
#pragma unroll
  for (int j = 0; j < kStats; ++j) s[j] = 0.0;
  for (int64_t b = b0 + lane; b < pl.G; b += 64) {
    const int64_t blo = st_lo(pl, b);
    if (blo >= uhi) break;
    if (st_lo(pl, b + 1) <= blo) continue;  // an empty range writes nothing
    const int64_t seg = g - blo / pl.ntiles;
    const double *pp = part + ((int64_t)b * pl.P + seg) * (kStats * kTF) + fl;
#pragma unroll
    for (int j = 0; j < kStats; ++j) s[j] += pp[j * kTF];
  }
  wave_sum(s);
  if (lane != 0) return;

  const double nsel = refinfo[7 + 1];  // n_sel
  const double mtot = refinfo[7];      // total mass (n_sel without masses)
  const int64_t o0 = GATHER ? (PLANES ? 1 : 3) * (int64_t)sel[0] : 0;
  const int64_t cs = PLANES ? ps : 1;
  const float *fr = xyz + f * fstride;
  const double px = fr[o0], py = fr[o0 + cs], pz = fr[o0 + 2 * cs];
  // COM relative to the pivot
  const double cx = (MASSES ? s[3] : s[0]) / mtot;
  const double cy = (MASSES ? s[4] : s[1]) / mtot;
  const double cz = (MASSES ? s[5] : s[2]) / mtot;
  // sum of centred reference coordinates (0 for unit masses up to rounding)
  const double sr0 = refinfo[3], sr1 = refinfo[4], sr2 = refinfo[5];
  double A[9];
  A[0] = s[6] - cx * sr0;
  A[1] = s[7] - cx * sr1;
  A[2] = s[8] - cx * sr2;
  A[3] = s[9] - cy * sr0;
  A[4] = s[10] - cy * sr1;
  A[5] = s[11] - cy * sr2;
  A[6] = s[12] - cz * sr0;
  A[7] = s[13] - cz * sr1;
  A[8] = s[14] - cz * sr2;
  const double gmob = s[15] - 2.0 * (cx * s[0] + cy * s[1] + cz * s[2]) + nsel * (cx * cx + cy * cy + cz * cz);
  const double E0 = 0.5 * (gmob + refinfo[6]);
  double *t = xform + f * kXform;
  double rot[9], rmsd;
  qcp_solve(A, E0, nsel, rot, &rmsd);
#pragma unroll
  for (int j = 0; j < 9; ++j) t[j] = rot[j];
  t[9] = px + cx;
  t[10] = py + cy;
  t[11] = pz + cz;
  t[12] = rmsd;
  t[13] = t[14] = t[15] = 0.0;
}

// ---------------------------------------------------------------------------
// Reference setup, RMSF.py:84-85 / 117-118, as three launches over
// kRefBlocks-bounded grids with fixed-order (deterministic) reductions whose
// per-block partials live in the scratch tail of the caller's refinfo record:
//   k_ref_com     per-block sum m x, sum m            -> scratch1[b][4]
//   k_ref_center  COM from scratch1 (same order in every block), r = x - com
//                 -> d_ref; per-block sum r, sum |r|^2 -> scratch2[b][4]
//   k_ref_finish  one block folds scratch2            -> info[0..8]
constexpr int kRefBlocks = 256;
constexpr int kRefThreads = 256;
static_assert(RMSF_REFINFO_DOUBLES >= 16 + 2 * 4 * kRefBlocks, "refinfo scratch");

// f64 path: avg[] / div -- the sweep-1 sums divided by the frame count as
// they are read (RMSF.py:111, the same IEEE division as k_divide; div = 1 is
// exact for an average passed in)
template <bool FROM_F32, bool GATHER>
__device__ __forceinline__ void ref_load(const float *__restrict__ frame, const double *__restrict__ avg,
                                         const int32_t *__restrict__ sel, int64_t a, double &x, double &y,
                                         double &z, double div = 1.0) {
  if (FROM_F32) {
    const float *p = frame + (GATHER ? 3 * (int64_t)sel[a] : 3 * a);
    x = (double)p[0];
    y = (double)p[1];
    z = (double)p[2];
  } else {
    x = avg[3 * a] / div;
    y = avg[3 * a + 1] / div;
    z = avg[3 * a + 2] / div;
  }
}

__device__ __forceinline__ void block_sum4(double (&v)[4], double *out) {
  __shared__ double red[kRefThreads / 64][4];
  wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0)
    for (int j = 0; j < 4; ++j) red[w][j] = v[j];
  __syncthreads();
  if (threadIdx.x < 4) {
    double t = 0.0;
    for (int i = 0; i < kRefThreads / 64; ++i) t += red[i][threadIdx.x];
    out[threadIdx.x] = t;
  }
}

// One wave folds nb [4]-partials: lane-strided sums, then the xor butterfly
// (fixed order, every lane ends with the same totals).
__device__ __forceinline__ void fold_partials(const double *__restrict__ p, int nb, double (&t)[4]) {
  const int lane = threadIdx.x & 63;
  for (int j = 0; j < 4; ++j) t[j] = 0.0;
  for (int b = lane; b < nb; b += 64)
    for (int j = 0; j < 4; ++j) t[j] += p[4 * b + j];
  wave_sum(t);
}

template <bool FROM_F32, bool GATHER, bool MASSES>
__device__ __forceinline__ void ref_com_body(const float *__restrict__ frame, const double *__restrict__ avg,
                                             int64_t n_sel, const int32_t *__restrict__ sel,
                                             const double *__restrict__ masses, double *__restrict__ info, int blk,
                                             int nblk, double div = 1.0) {
  double v[4] = {0, 0, 0, 0};
  const int64_t stride = (int64_t)nblk * kRefThreads;
  for (int64_t a = (int64_t)blk * kRefThreads + threadIdx.x; a < n_sel; a += stride) {
    double x, y, z;
    ref_load<FROM_F32, GATHER>(frame, avg, sel, a, x, y, z, div);
    const double m = MASSES ? masses[a] : 1.0;
    v[0] = fma(x, m, v[0]);
    v[1] = fma(y, m, v[1]);
    v[2] = fma(z, m, v[2]);
    v[3] += m;
  }
  block_sum4(v, info + 16 + 4 * blk);
}

template <bool FROM_F32, bool GATHER>
__device__ __forceinline__ void ref_center_body(const float *__restrict__ frame, const double *__restrict__ avg,
                                                int64_t n_sel, const int32_t *__restrict__ sel,
                                                double *__restrict__ ref, double *__restrict__ info, int blk,
                                                int nblk, double div = 1.0, double *__restrict__ avg_out = nullptr) {
  __shared__ double com[4];
  if (threadIdx.x < 64) {
    double t[4];
    fold_partials(info + 16, nblk, t);
    if (threadIdx.x < 4) com[threadIdx.x] = t[threadIdx.x];
  }
  __syncthreads();
  const double c0 = com[0] / com[3], c1 = com[1] / com[3], c2 = com[2] / com[3];
  double w[4] = {0, 0, 0, 0};
  const int64_t stride = (int64_t)nblk * kRefThreads;
  for (int64_t a = (int64_t)blk * kRefThreads + threadIdx.x; a < n_sel; a += stride) {
    double x, y, z;
    ref_load<FROM_F32, GATHER>(frame, avg, sel, a, x, y, z, div);
    if (avg_out) {
      avg_out[3 * a] = x;
      avg_out[3 * a + 1] = y;
      avg_out[3 * a + 2] = z;
    }
    const double r0 = x - c0, r1 = y - c1, r2 = z - c2;
    ref[3 * a] = r0;
    ref[3 * a + 1] = r1;
    ref[3 * a + 2] = r2;
    w[0] += r0;
    w[1] += r1;
    w[2] += r2;
    w[3] = fma(r0, r0, fma(r1, r1, fma(r2, r2, w[3])));
  }
  block_sum4(w, info + 16 + 4 * kRefBlocks + 4 * blk);
  if (blk == 0 && threadIdx.x < 3) info[threadIdx.x] = threadIdx.x == 0 ? c0 : (threadIdx.x == 1 ? c1 : c2);
  if (blk == 0 && threadIdx.x == 3) info[7] = com[3];
}

// one wave
__device__ __forceinline__ void ref_finish_body(int nb, int64_t n_sel, double *__restrict__ info) {
  double t[4];
  fold_partials(info + 16 + 4 * kRefBlocks, nb, t);
  if (threadIdx.x < 4) info[3 + threadIdx.x] = t[threadIdx.x];  // sum r (3), sum |r|^2
  if (threadIdx.x == 0) {
    info[8] = (double)n_sel;
    for (int j = 9; j < 16; ++j) info[j] = 0.0;
  }
}

template <bool FROM_F32, bool GATHER, bool MASSES>
__global__ __launch_bounds__(kRefThreads) void k_ref_com(const float *__restrict__ frame,
                                                         const double *__restrict__ avg, int64_t n_sel,
                                                         const int32_t *__restrict__ sel,
                                                         const double *__restrict__ masses,
                                                         double *__restrict__ info) {
  ref_com_body<FROM_F32, GATHER, MASSES>(frame, avg, n_sel, sel, masses, info, blockIdx.x, gridDim.x);
}

template <bool FROM_F32, bool GATHER>
__global__ __launch_bounds__(kRefThreads) void k_ref_center(const float *__restrict__ frame,
                                                            const double *__restrict__ avg, int64_t n_sel,
                                                            const int32_t *__restrict__ sel,
                                                            double *__restrict__ ref, double *__restrict__ info) {
  ref_center_body<FROM_F32, GATHER>(frame, avg, n_sel, sel, ref, info, blockIdx.x, gridDim.x);
}

__global__ __launch_bounds__(64) void k_ref_finish(int nb, int64_t n_sel, double *__restrict__ info) {
  ref_finish_body(nb, n_sel, info);
}

// The three steps of a one-workgroup grid (n_sel <= 4 x 256) in ONE launch:
// the same code in the same order, the partials passed through the same
// scratch (each read by the wave that wrote it), so the record is
// bit-identical to the three launches' -- two launch boundaries fewer per
// reference (RMSF.py's two sweeps at config C1's size run two of them).
// With div != 1 (rmsf_reference_setup_mean) it also absorbs k_divide: the
// average is avg[] / div, written to avg_out as it is read.
template <bool FROM_F32, bool GATHER, bool MASSES>
__global__ __launch_bounds__(kRefThreads) void k_ref_setup1(const float *__restrict__ frame,
                                                            const double *__restrict__ avg, int64_t n_sel,
                                                            const int32_t *__restrict__ sel,
                                                            const double *__restrict__ masses,
                                                            double *__restrict__ ref, double *__restrict__ info,
                                                            double div = 1.0, double *__restrict__ avg_out = nullptr) {
  ref_com_body<FROM_F32, GATHER, MASSES>(frame, avg, n_sel, sel, masses, info, 0, 1, div);
  __syncthreads();
  ref_center_body<FROM_F32, GATHER>(frame, avg, n_sel, sel, ref, info, 0, 1, div, avg_out);
  __syncthreads();
  if (threadIdx.x < 64) ref_finish_body(1, n_sel, info);
}

// ---------------------------------------------------------------------------
constexpr int kMergeGroup = 128;
struct MergeCounts {
  double n[kMergeGroup];
  double w[kMergeGroup];  // n1 n2 / T of the step that merges part s (RMSF.py:39), exact on the host
};

// second_order_moments(S1, S2), RMSF.py:36-41, one coordinate, with the
// script's operations in its order (the library is built without FP
// contraction): T = n1 + n2; mu = (n1 mu1 + n2 mu2) / T;
// M = M1 + M2 + (n1 n2 / T) (mu2 - mu1)**2.  n1, n2 are the frame counts
// (Python ints in RMSF.py: n1 n2 is an exact integer product, then one
// correctly rounded division -- the same as (double)(n1 n2) / T below 2^53).
// The caller guarantees T > 0 (RMSF.py:39 raises ZeroDivisionError at T = 0).
__device__ __forceinline__ void som(double n1, double mu1, double M1, double n1n2_over_T, double n2, double mu2,
                                    double M2, double T, double &mu, double &M) {
  const double d = mu2 - mu1;
  mu = (n1 * mu1 + n2 * mu2) / T;
  M = M1 + M2 + n1n2_over_T * (d * d);
}

// Fold (acc) + parts[0..np) in order (mpi4py's _py_reduce shape: res = S0,
// res = op(res, S_i)): second_order_moments, RMSF.py:36-41.  first_verbatim:
// the state starts as part 0 itself (no op applied, as the fold's first
// element); else as (acc_n, acc) -- acc_n = 0: the empty state (0, zeros,
// zeros) RMSF.py:119-121 gives a rank without frames.  An empty partial is
// (0, zeros, zeros) too (its memory is not read); a merge of two empty states
// (T = 0, where RMSF.py:39 raises) is skipped.
__global__ __launch_bounds__(kBlock) void k_chan_merge(const double *__restrict__ acc_mean,
                                                       const double *__restrict__ acc_m2, double acc_n,
                                                       const double *__restrict__ mp,
                                                       const double *__restrict__ qp, MergeCounts cnt,
                                                       int np, int first_verbatim, int64_t n, double *mo, double *qo) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  double n1 = acc_n, mu = 0.0, M = 0.0;
  int s0 = 0;
  if (first_verbatim) {
    n1 = cnt.n[0];
    if (n1 > 0) {
      mu = mp[j];
      M = qp[j];
    }
    s0 = 1;
  } else if (acc_n > 0) {
    mu = acc_mean[j];
    M = acc_m2[j];
  }
  for (int s = s0; s < np; ++s) {
    const double n2 = cnt.n[s];
    const double T = n1 + n2;
    if (T <= 0) continue;  // two empty states (RMSF.py:39's ZeroDivisionError)
    double mu2 = 0.0, M2 = 0.0;
    if (n2 > 0) {
      mu2 = mp[(int64_t)s * n + j];
      M2 = qp[(int64_t)s * n + j];
    }
    som(n1, mu, M, cnt.w[s], n2, mu2, M2, T, mu, M);
    n1 = T;
  }
  mo[j] = mu;
  qo[j] = M;
}

// A reduction schedule of second_order_moments steps over the partials, run
// in place: step i is S[dst] = op(S[dst], S[src]) with the host-known counts
// (n_dst, n_src) of that moment.  Every thread owns one coordinate of every
// partial and walks the steps in order (no cross-thread dependence); the
// partials' memory is the schedule's working storage, as each mpi4py rank's
// `result` is (parts of empty states are not read).  last: write S[0] to
// (mo, qo) after the steps.
constexpr int kMaxSteps = 96;
struct ChanSteps {
  int dst[kMaxSteps], src[kMaxSteps];
  double n1[kMaxSteps], n2[kMaxSteps], w[kMaxSteps];
};

__global__ __launch_bounds__(kBlock) void k_chan_steps(double *mp, double *qp, ChanSteps st, int n_steps,
                                                       double n0_final, int64_t n, double *mo, double *qo) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  for (int i = 0; i < n_steps; ++i) {
    const double n1 = st.n1[i], n2 = st.n2[i], T = n1 + n2;
    const int64_t a = (int64_t)st.dst[i] * n + j, b = (int64_t)st.src[i] * n + j;
    double mu1 = 0.0, M1 = 0.0, mu2 = 0.0, M2 = 0.0;
    if (n1 > 0) {
      mu1 = mp[a];
      M1 = qp[a];
    }
    if (n2 > 0) {
      mu2 = mp[b];
      M2 = qp[b];
    }
    double mu, M;
    som(n1, mu1, M1, st.w[i], n2, mu2, M2, T, mu, M);
    mp[a] = mu;
    qp[a] = M;
  }
  if (mo) {
    double mu = 0.0, M = 0.0;
    if (n0_final > 0) {
      mu = mp[j];
      M = qp[j];
    }
    mo[j] = mu;
    qo[j] = M;
  }
}

// S1 = op(S1, S2) in place, two separate buffers (one pairwise step of a
// distributed reduction: S2 just arrived from another rank or device).
__global__ __launch_bounds__(kBlock) void k_chan_pair(double *m1, double *q1, const double *__restrict__ m2,
                                                      const double *__restrict__ q2, double n1, double n2, double w,
                                                      int64_t n) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  double mu1 = 0.0, M1 = 0.0, mu2 = 0.0, M2 = 0.0;
  if (n1 > 0) {
    mu1 = m1[j];
    M1 = q1[j];
  }
  if (n2 > 0) {
    mu2 = m2[j];
    M2 = q2[j];
  }
  double mu, M;
  som(n1, mu1, M1, w, n2, mu2, M2, n1 + n2, mu, M);
  m1[j] = mu;
  q1[j] = M;
}

__global__ __launch_bounds__(kBlock) void k_sum_splits(const double *__restrict__ parts, int np, int64_t n,
                                                       double *__restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  double t = 0.0;
  for (int s = 0; s < np; ++s) t += parts[(int64_t)s * n + j];
  out[j] = t;
}

__global__ __launch_bounds__(kBlock) void k_divide(const double *__restrict__ x, double d, int64_t n,
                                                   double *__restrict__ y) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n) y[j] = x[j] / d;
}

__global__ __launch_bounds__(kBlock) void k_chan_weight(const double *__restrict__ m, double w, int64_t n,
                                                        double *__restrict__ y) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n) y[j] = w * m[j];
}

__global__ __launch_bounds__(kBlock) void k_chan_deviation(const double *__restrict__ mk,
                                                           const double *__restrict__ qk,
                                                           const double *__restrict__ mean, double nk,
                                                           int64_t n, double *__restrict__ y) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const double d = mk[j] - mean[j];
  y[j] = qk[j] + nk * (d * d);
}

// One-collective cross-rank merge (RMSF.py:140-143 + 146): moments about a
// shift c that every rank holds (the reference structure, the sweep-1
// average, or trajectory frame 0 broadcast during the sweep).  Per rank
//   T1 = n_k (mean_k - c),   T2 = M2_k + n_k (mean_k - c)^2
// summed over ranks in ONE all-reduce; then mean = c + T1/n and
// M2 = T2 - T1^2/n -- Chan's k-way formula in exact arithmetic, and with c
// near the data (|mean - c| ~ the fluctuation) free of cancellation.
template <typename ShiftT>
__global__ __launch_bounds__(kBlock) void k_chan_shift_pack(const double *__restrict__ mk,
                                                            const double *__restrict__ qk,
                                                            const ShiftT *__restrict__ shift,
                                                            const double *__restrict__ off3, double nk, int64_t n,
                                                            double *__restrict__ t, int64_t t_slice) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  double c = (double)shift[j];
  if (off3) c += off3[j % 3];
  if (t_slice > 0) {
    double *t1 = t + slice_t1(j, t_slice);
    shift_moments(mk[j], qk[j], c, nk, t1, t1 + t_slice);
  } else {
    shift_moments(mk[j], qk[j], c, nk, t + j, t + n + j);
  }
}

template <typename ShiftT>
__global__ __launch_bounds__(kBlock) void k_chan_shift_finish(const double *__restrict__ t,
                                                              const ShiftT *__restrict__ shift,
                                                              const double *__restrict__ off3, int64_t n_sel,
                                                              double nf, double *__restrict__ mean,
                                                              double *__restrict__ m2, double *__restrict__ rmsf,
                                                              int64_t t2_off) {
  // T2 at t + t2_off (3 n_sel for [T1 | T2]; the slice width for a
  // reduce-scatter slice whose last rank holds fewer atoms)
  const int64_t a = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a >= n_sel) return;
  const int64_t n = t2_off;
  double q[3];
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    const int64_t j = 3 * a + x;
    double c = (double)shift[j];
    if (off3) c += off3[x];
    const double t1 = t[j];
    mean[j] = c + t1 / nf;
    // the two sums are of non-negative terms whose difference rounds to
    // >= -eps * T2: clamp so that sqrt below never sees a negative zero-sum
    q[x] = clamp0(t[n + j] - t1 * (t1 / nf));
    m2[j] = q[x];
  }
  if (rmsf) rmsf[a] = sqrt((q[0] + q[1] + q[2]) / nf);
}

__global__ __launch_bounds__(kBlock) void k_finalize(const double *__restrict__ m2, int64_t n_sel, double nf,
                                                     double *__restrict__ out) {
  const int64_t a = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a >= n_sel) return;
  out[a] = sqrt((m2[3 * a] + m2[3 * a + 1] + m2[3 * a + 2]) / nf);
}

// k_finalize behind rmsf_fold_balanced_finalize for the plan the workspace
// header names: a flat plan (hdr[6] = 4 coordinates per lane, whose fold
// cannot finalise per lane) is finalised here from the M2 the fold just
// stored; an atom plan (finalised in the fold) leaves at once.  The decision
// is the workspace's own, read on the device -- no host record of plans.
__global__ __launch_bounds__(kBlock) void k_finalize_flat(const int64_t *__restrict__ hdr,
                                                          const double *__restrict__ m2, int64_t n_sel, double nf,
                                                          double *__restrict__ out) {
  if (hdr[6] != 4) return;
  for (int64_t a = (int64_t)blockIdx.x * kBlock + threadIdx.x; a < n_sel; a += (int64_t)gridDim.x * kBlock)
    out[a] = sqrt((m2[3 * a] + m2[3 * a + 1] + m2[3 * a + 2]) / nf);
}

__global__ __launch_bounds__(kBlock) void k_qcp_batch(const double *__restrict__ A, const double *__restrict__ E0,
                                                      const double *__restrict__ N, int64_t n,
                                                      double *__restrict__ rot, double *__restrict__ rmsd) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double r[9], d;
  qcp_solve(A + 9 * i, E0[i], N[i], r, &d);
  for (int j = 0; j < 9; ++j) rot[9 * i + j] = r[j];
  rmsd[i] = d;
}

// qcprot InnerProduct (weights optional): A (9) and E0, in the published
// loop's order -- one pass over the atoms, every accumulator updated per atom
// (Theobald's qcprot.c, restated by MDAnalysis.lib.qcprot; upstream,
// unverified here; oracle/rmsf_oracle.py:inner_product).  One lane: the
// host-pointer CalcRMSDRotationalMatrix replaces a single-threaded call, and
// its A / E0 are then the loop's own bits (no contraction, csrc/Makefile).
__global__ __launch_bounds__(64) void k_inner_product(const double *__restrict__ ref,
                                                      const double *__restrict__ conf,
                                                      const double *__restrict__ w, int64_t N,
                                                      double *__restrict__ out) {
  if (threadIdx.x != 0) return;
  double A[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, G1 = 0.0, G2 = 0.0;
  for (int64_t i = 0; i < N; ++i) {
    const double cx = conf[3 * i], cy = conf[3 * i + 1], cz = conf[3 * i + 2];
    const double wi = w ? w[i] : 1.0;
    const double x1 = w ? wi * cx : cx, y1 = w ? wi * cy : cy, z1 = w ? wi * cz : cz;
    G1 = G1 + (x1 * cx + y1 * cy + z1 * cz);
    const double x2 = ref[3 * i], y2 = ref[3 * i + 1], z2 = ref[3 * i + 2];
    const double g2 = x2 * x2 + y2 * y2 + z2 * z2;
    G2 = G2 + (w ? wi * g2 : g2);
    A[0] = A[0] + x1 * x2;
    A[1] = A[1] + x1 * y2;
    A[2] = A[2] + x1 * z2;
    A[3] = A[3] + y1 * x2;
    A[4] = A[4] + y1 * y2;
    A[5] = A[5] + y1 * z2;
    A[6] = A[6] + z1 * x2;
    A[7] = A[7] + z1 * y2;
    A[8] = A[8] + z1 * z2;
  }
  for (int j = 0; j < 9; ++j) out[j] = A[j];
  out[9] = (G1 + G2) * 0.5;
}

// ---------------------------------------------------------------------------
// Synthetic generator.  Every f64 op is a single IEEE-rounded op (no FMA
// contraction), so oracle/synth.py reproduces the frames bit-for-bit.
__host__ __device__ inline uint64_t sm64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t skey(uint64_t seed, uint64_t stream, uint64_t i, uint64_t j) {
  return sm64(sm64(sm64(seed ^ (stream * 0xD1B54A32D192ED03ull)) + i) + j);
}

// k_gather_frames: compact batch of frames (a scattered run(frames=...) list,
// or the dense copy of a sparse selection's rows, pipeline._Compactor):
// dst[k][j] = the selected atom j of frame src + frames[k]*fstride, one float
// per thread, grid = (coordinate blocks, frames).  Round 6 A/B at 10k, 455 and
// 50k of 100k atoms x 20k frames (profiles/r06_workloads/ab_gather.txt):
// this form is the fastest at CA-like densities -- one atom per thread with
// three strided stores is 3-12 % slower there (13 % faster at 1 in 2, where
// compaction does not run), 16 frames per block row 12 % slower.
template <bool GATHER>
__global__ __launch_bounds__(kBlock) void k_gather_frames(const float *__restrict__ src, int64_t fstride,
                                                          const int64_t *__restrict__ frames, int64_t n_sel,
                                                          const int32_t *__restrict__ sel, float *__restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= 3 * n_sel) return;
  const int64_t k = blockIdx.y;
  const float *fr = src + frames[k] * fstride;
  const int64_t a = i / 3, c = i - 3 * a;
  dst[k * 3 * n_sel + i] = __builtin_nontemporal_load(fr + (GATHER ? 3 * (int64_t)sel[a] + c : i));
}

// k_gather_planes: the same compact batch from frames stored as coordinate
// planes (SoA: x[n], y[n], z[n] at plane_stride floats apart, HBM-resident):
// one selected atom per thread, its three plane values (consecutive lanes
// read consecutive -- or gathered -- atoms of each plane) interleaved into
// dst's (frame, atom, xyz) rows.  grid = (atom blocks, frames).
template <bool GATHER>
__global__ __launch_bounds__(kBlock) void k_gather_planes(const float *__restrict__ src, int64_t fstride,
                                                          int64_t pstride, const int64_t *__restrict__ frames,
                                                          int64_t n_sel, const int32_t *__restrict__ sel,
                                                          float *__restrict__ dst) {
  const int64_t a = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a >= n_sel) return;
  const int64_t k = blockIdx.y;
  const float *fr = src + frames[k] * fstride + (GATHER ? (int64_t)sel[a] : a);
  float *o = dst + k * 3 * n_sel + 3 * a;
  o[0] = __builtin_nontemporal_load(fr);
  o[1] = __builtin_nontemporal_load(fr + pstride);
  o[2] = __builtin_nontemporal_load(fr + 2 * pstride);
}

// k_planes_to_rows: per-coordinate f64 statistics kept in plane order
// (x[n], y[n], z[n] -- what the unaligned kernels produce when they read
// coordinate planes in place) to (atom, xyz) order: dst[3a + c] = src[c n + a].
__global__ __launch_bounds__(kBlock) void k_planes_to_rows(const double *__restrict__ src, int64_t n,
                                                           double *__restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // destination index: coalesced stores
  if (i >= 3 * n) return;
  const int64_t a = i / 3, c = i - 3 * a;
  dst[i] = src[c * n + a];
}

// The generator's per-atom noise scale sigma(a) (k_synth's expression): the
// expected RMSF of an unaligned synthetic atom is sqrt(3) sigma(a), the
// reference figure of the bench's sanity check (rmsf_amd.synth).
__global__ __launch_bounds__(kBlock) void k_synth_sigma(double *__restrict__ out, int64_t a0, int64_t n,
                                                        uint64_t seed) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const double two53 = 1.1102230246251565e-16;  // 2^-53
  out[i] = 0.2 + (double)(skey(seed, 2, (uint64_t)(a0 + i), 0) >> 11) * two53 * 1.8;
}

__global__ __launch_bounds__(kBlock) void k_synth(float *__restrict__ out, int64_t fstride, int64_t n_atoms,
                                                  int64_t f0, int64_t nf, uint64_t seed,
                                                  const double *__restrict__ motion) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= nf * n_atoms) return;
  const int64_t fl = t / n_atoms, a = t - fl * n_atoms;
  const int64_t f = f0 + fl;
  const double two24 = 5.9604644775390625e-08;   // 2^-24
  const double two53 = 1.1102230246251565e-16;   // 2^-53
  const double sqrt6 = 2.449489742783178;
  const double sigma = 0.2 + (double)(skey(seed, 2, (uint64_t)a, 0) >> 11) * two53 * 1.8;
  double p[3];
  for (int c = 0; c < 3; ++c) {
    const double base = (double)(skey(seed, 1, (uint64_t)a, (uint64_t)c) >> 11) * two53 * 100.0;
    const uint64_t h = skey(seed, 3, (uint64_t)f, (uint64_t)(3 * a + c));
    const uint64_t u = (h >> 40) + ((h >> 16) & 0xFFFFFFull);
    const double g = ((double)u * two24 - 1.0) * sqrt6;
    const double s = sigma * g;
    p[c] = base + s;
  }
  float *o = out + fl * fstride + 3 * a;
  if (motion) {
    const double *M = motion + 12 * f;
    const double d0 = p[0] - 50.0, d1 = p[1] - 50.0, d2 = p[2] - 50.0;
    for (int b = 0; b < 3; ++b) {
      const double e0 = d0 * M[b];
      const double e1 = d1 * M[3 + b];
      const double e2 = d2 * M[6 + b];
      const double y = ((e0 + e1) + e2) + M[9 + b];
      o[b] = (float)y;
    }
  } else {
    o[0] = (float)p[0];
    o[1] = (float)p[1];
    o[2] = (float)p[2];
  }
}

inline unsigned grid1(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// Balanced grid of k_frame_stats: whole rounds of kStatsRound workgroups, up
// to kStatsGroups, by the batch's unit count -- a function of the shape only,
// so the summation order (hence the bits) does not depend on the device.
// P = the most segments any workgroup's range can cross: ceil(len/ntiles)+1.
StatsPlan stats_plan(int64_t n_sel, int64_t n_frames) {
  StatsPlan p;
  p.ntiles = (n_sel + kTA - 1) / kTA;
  p.ngroups = std::max<int64_t>(1, (n_frames + kTF - 1) / kTF);
  p.T = p.ntiles * p.ngroups;
  // whole rounds, ~160 units per workgroup, at most kStatsGroups: fewer
  // workgroups at short batches cut both the per-workgroup fixed cost and the
  // partials k_qcp_frames folds (tools/ubench_stats3.hip, 100k atoms: 2,500
  // frames 0.478 vs 0.516 ms for stats + QCP at 768 vs 3,072 workgroups;
  // 5,000 frames 0.945 vs 0.988 at 1,536; 20,000 frames best at 3,072)
  const int64_t rounds = std::min<int64_t>(kStatsGroups / kStatsRound,
                                           std::max<int64_t>(1, (p.T + kStatsRoundUnits / 2) / kStatsRoundUnits));
  p.G = (int)std::max<int64_t>(1, std::min<int64_t>(kStatsRound * rounds, p.T / kStatsMinUnits));
  const int64_t len = (p.T + p.G - 1) / p.G;
  p.P = (int)((len + p.ntiles - 1) / p.ntiles + 1);
  return p;
}

}  // namespace

// ===========================================================================
// extern "C" ABI
// ===========================================================================
extern "C" {

RMSF_EXPORT int rmsf_abi_version(void) { return RMSF_ABI_VERSION; }

// error hook used by stager.cpp (not part of the public header)
RMSF_EXPORT int rmsf_internal_set_error(int code, const char *msg) { return fail(code, msg ? msg : ""); }

RMSF_EXPORT const char *rmsf_last_error(void) { return g_err.c_str(); }

RMSF_EXPORT int rmsf_device_count(int *n) {
  if (!n) return fail(RMSF_EINVAL, "rmsf_device_count: null");
  HIP_TRY(hipGetDeviceCount(n));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_set_device(int dev) {
  HIP_TRY(hipSetDevice(dev));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_malloc(void **p, size_t bytes) {
  if (!p) return fail(RMSF_EINVAL, "rmsf_malloc: null");
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return fail(RMSF_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_free(void *p) {
  HIP_TRY(hipFree(p));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_memcpy_h2d(void *d, const void *h, size_t bytes, void *stream) {
  HIP_TRY(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, S(stream)));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_memcpy_d2h(void *h, const void *d, size_t bytes, void *stream) {
  HIP_TRY(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, S(stream)));
  HIP_TRY(hipStreamSynchronize(S(stream)));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_memcpy2d_d2d(void *d_dst, size_t dpitch, const void *d_src, size_t spitch, size_t width,
                                 size_t height, void *stream) {
  if (!d_dst || !d_src || width > dpitch || width > spitch) return fail(RMSF_EINVAL, "rmsf_memcpy2d_d2d: bad arguments");
  if (width == 0 || height == 0) return RMSF_OK;
  HIP_TRY(hipMemcpy2DAsync(d_dst, dpitch, d_src, spitch, width, height, hipMemcpyDeviceToDevice, S(stream)));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_stream_synchronize(void *stream) {
  HIP_TRY(hipStreamSynchronize(S(stream)));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_block_range(int64_t n_frames, int size, int rank, int64_t *start, int64_t *stop) {
  if (n_frames < 0 || size < 1 || rank < 0 || rank >= size || !start || !stop)
    return fail(RMSF_EINVAL, "rmsf_block_range: bad arguments");
  const int64_t per = n_frames / size;  // RMSF.py:64 (floor division)
  if (rank < size - 1) {                // RMSF.py:65
    *start = rank * per;
    *stop = (rank + 1) * per;
  } else {                              // RMSF.py:66
    *start = (int64_t)(size - 1) * per;
    *stop = n_frames;
  }
  return RMSF_OK;
}

}  // extern "C"

namespace {

int reference_setup_impl(const float *d_frame, const double *d_avg, int64_t n_sel, const int32_t *d_sel,
                         const double *d_masses, double *d_ref, double *d_refinfo, void *stream, bool one_launch,
                         double div = 1.0, double *d_avg_out = nullptr) {
  if ((d_frame == nullptr) == (d_avg == nullptr))
    return fail(RMSF_EINVAL, "rmsf_reference_setup: exactly one of d_frame / d_avg");
  if (n_sel < 1 || !d_ref || !d_refinfo) return fail(RMSF_EINVAL, "rmsf_reference_setup: bad arguments");
  const bool g = d_sel != nullptr, m = d_masses != nullptr;
  hipStream_t s = S(stream);
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(kRefBlocks, (n_sel + 4 * kRefThreads - 1) / (4 * kRefThreads)));
  const dim3 grid(nb), block(kRefThreads);
  if (nb == 1 && one_launch) {  // one launch, bit-identical to the three below
#define ONE_LAUNCH(F, G, M) hipLaunchKernelGGL((k_ref_setup1<F, G, M>), dim3(1), block, 0, s, d_frame, d_avg, n_sel, d_sel, d_masses, d_ref, d_refinfo, div, d_avg_out)
    if (d_frame) {
      if (g && m) ONE_LAUNCH(true, true, true);
      else if (g) ONE_LAUNCH(true, true, false);
      else if (m) ONE_LAUNCH(true, false, true);
      else ONE_LAUNCH(true, false, false);
    } else {
      if (m) ONE_LAUNCH(false, false, true);
      else ONE_LAUNCH(false, false, false);
    }
#undef ONE_LAUNCH
    return after_launch("k_ref_setup1");
  }
  if (d_avg_out) {  // more than one workgroup: the average first (k_divide), then the setup from it
    hipLaunchKernelGGL(k_divide, dim3(grid1(3 * n_sel)), dim3(kBlock), 0, s, d_avg, div, 3 * n_sel, d_avg_out);
    d_avg = d_avg_out;
  }
#define COM_LAUNCH(F, G, M) hipLaunchKernelGGL((k_ref_com<F, G, M>), grid, block, 0, s, d_frame, d_avg, n_sel, d_sel, d_masses, d_refinfo)
#define CEN_LAUNCH(F, G) hipLaunchKernelGGL((k_ref_center<F, G>), grid, block, 0, s, d_frame, d_avg, n_sel, d_sel, d_ref, d_refinfo)
  if (d_frame) {
    if (g && m) COM_LAUNCH(true, true, true);
    else if (g) COM_LAUNCH(true, true, false);
    else if (m) COM_LAUNCH(true, false, true);
    else COM_LAUNCH(true, false, false);
    if (g) CEN_LAUNCH(true, true);
    else CEN_LAUNCH(true, false);
  } else {
    if (m) COM_LAUNCH(false, false, true);
    else COM_LAUNCH(false, false, false);
    CEN_LAUNCH(false, false);
  }
#undef COM_LAUNCH
#undef CEN_LAUNCH
  hipLaunchKernelGGL(k_ref_finish, dim3(1), dim3(64), 0, s, nb, n_sel, d_refinfo);
  return after_launch("k_ref_*");
}

}  // namespace

extern "C" {

RMSF_EXPORT int rmsf_reference_setup(const float *d_frame, const double *d_avg, int64_t n_sel,
                                     const int32_t *d_sel, const double *d_masses, double *d_ref,
                                     double *d_refinfo, void *stream) {
  return reference_setup_impl(d_frame, d_avg, n_sel, d_sel, d_masses, d_ref, d_refinfo, stream, true);
}

RMSF_EXPORT int rmsf_reference_setup_mean(const double *d_sum, double n_frames, int64_t n_sel,
                                          const double *d_masses, double *d_avg, double *d_ref, double *d_refinfo,
                                          void *stream) {
  if (!d_sum || !d_avg || !(n_frames > 0)) return fail(RMSF_EINVAL, "rmsf_reference_setup_mean: bad arguments");
  return reference_setup_impl(nullptr, d_sum, n_sel, nullptr, d_masses, d_ref, d_refinfo, stream, true, n_frames,
                              d_avg);
}

// test hook (not in the public header): always the three launches, for the
// bit-identity test of k_ref_setup1
RMSF_EXPORT int rmsf_internal_reference_setup3(const float *d_frame, const double *d_avg, int64_t n_sel,
                                               const int32_t *d_sel, const double *d_masses, double *d_ref,
                                               double *d_refinfo, void *stream) {
  return reference_setup_impl(d_frame, d_avg, n_sel, d_sel, d_masses, d_ref, d_refinfo, stream, false);
}

RMSF_EXPORT size_t rmsf_superpose_workspace_bytes(int64_t n_sel, int64_t n_frames) {
  if (n_sel < 1 || n_frames < 0) return 0;
  const StatsPlan p = stats_plan(n_sel, n_frames);
  return (size_t)p.G * (size_t)p.P * kStats * kTF * sizeof(double);
}

}  // extern "C"

namespace {

// rmsf_superpose(_planes): ps = 0 for (frame, atom, xyz) rows, else the
// coordinate-plane stride of SoA frames (PLANES kernels)
int superpose_impl(const char *who, const float *d_xyz, int64_t fstride, int64_t ps, int64_t n_frames, int64_t n_sel,
                   const int32_t *d_sel, const double *d_masses, const double *d_ref, const double *d_refinfo,
                   double *d_xform, void *d_work, size_t work_bytes, hipStream_t s, float *d_dense = nullptr,
                   int64_t dense_pitch = 0) {
  if (n_frames == 0) return RMSF_OK;
  const bool planes = ps > 0;
  if (!d_xyz || !d_ref || !d_refinfo || !d_xform || !d_work || n_sel < 1 || n_frames < 0 ||
      (planes ? (ps < (d_sel ? 1 : n_sel) || fstride < 3 * ps) : fstride < (d_sel ? 3 : 3 * n_sel)))
    return fail(RMSF_EINVAL, std::string(who) + ": bad arguments");
  const StatsPlan plan = stats_plan(n_sel, n_frames);
  if (work_bytes < rmsf_superpose_workspace_bytes(n_sel, n_frames))
    return fail(RMSF_ENOMEM, std::string(who) + ": workspace too small");
  double *part = static_cast<double *>(d_work);
  const bool g = d_sel != nullptr, m = d_masses != nullptr;
  const bool vec4 = !g && fstride % 4 == 0 && (!planes || ps % 4 == 0) &&
                    reinterpret_cast<uintptr_t>(d_xyz) % 16 == 0;
  dim3 grid((unsigned)plan.G);
  auto stats = [&](auto P) {
    constexpr bool PL = decltype(P)::value;
#define ST_LAUNCH(G, M, V) \
  hipLaunchKernelGGL((k_frame_stats<G, M, V, 1, PL>), grid, dim3(kBlock), 0, s, d_xyz, fstride, n_frames, n_sel, d_sel, d_masses, d_ref, plan, part, ps)
#define ST_DENSE(M, D) \
  hipLaunchKernelGGL((k_frame_stats<true, M, false, 3, false, D>), grid, dim3(kBlock), 0, s, d_xyz, fstride, n_frames, n_sel, d_sel, d_masses, d_ref, plan, part, ps, d_dense, dense_pitch)
    if (d_dense) {
      if constexpr (!PL) {
        const bool dv = dense_pitch % 4 == 0 && reinterpret_cast<uintptr_t>(d_dense) % 16 == 0;
        if (m && dv) ST_DENSE(true, 2);
        else if (m) ST_DENSE(true, 1);
        else if (dv) ST_DENSE(false, 2);
        else ST_DENSE(false, 1);
      }
    } else if (g && m) ST_LAUNCH(true, true, false);
    else if (g) ST_LAUNCH(true, false, false);
    else if (m && vec4) ST_LAUNCH(false, true, true);
    else if (m) ST_LAUNCH(false, true, false);
    else if (vec4) ST_LAUNCH(false, false, true);
    else ST_LAUNCH(false, false, false);
#undef ST_LAUNCH
#undef ST_DENSE
  };
  if (planes) stats(std::true_type{});
  else stats(std::false_type{});
  int rc = after_launch("k_frame_stats");
  if (rc) return rc;
  const unsigned gq = (unsigned)((n_frames + 3) / 4);
  auto qcp = [&](auto P) {
    constexpr bool PL = decltype(P)::value;
#define QCP_LAUNCH(G, M) \
  hipLaunchKernelGGL((k_qcp_frames<G, M, PL>), dim3(gq), dim3(kBlock), 0, s, part, plan, n_frames, d_xyz, fstride, d_sel, d_refinfo, d_xform, ps)
    if (g && m) QCP_LAUNCH(true, true);
    else if (g) QCP_LAUNCH(true, false);
    else if (m) QCP_LAUNCH(false, true);
    else QCP_LAUNCH(false, false);
#undef QCP_LAUNCH
  };
  if (planes) qcp(std::true_type{});
  else qcp(std::false_type{});
  return after_launch("k_qcp_frames");
}

}  // namespace

extern "C" {

RMSF_EXPORT int rmsf_superpose(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                               const int32_t *d_sel, const double *d_masses, const double *d_ref,
                               const double *d_refinfo, double *d_xform, void *d_work, size_t work_bytes,
                               void *stream) {
  return superpose_impl("rmsf_superpose", d_xyz, fstride, 0, n_frames, n_sel, d_sel, d_masses, d_ref, d_refinfo,
                        d_xform, d_work, work_bytes, S(stream));
}

RMSF_EXPORT int rmsf_superpose_compact(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                       const int32_t *d_sel, const double *d_masses, const double *d_ref,
                                       const double *d_refinfo, double *d_xform, void *d_work, size_t work_bytes,
                                       float *d_dense_out, int64_t dense_stride, void *stream) {
  if (!d_sel || !d_dense_out) return fail(RMSF_EINVAL, "rmsf_superpose_compact: needs a selection and an output");
  if (dense_stride == 0) dense_stride = 3 * n_sel;
  if (dense_stride < 3 * n_sel) return fail(RMSF_EINVAL, "rmsf_superpose_compact: dense_stride < 3 n_sel");
  return superpose_impl("rmsf_superpose_compact", d_xyz, fstride, 0, n_frames, n_sel, d_sel, d_masses, d_ref,
                        d_refinfo, d_xform, d_work, work_bytes, S(stream), d_dense_out, dense_stride);
}

RMSF_EXPORT int rmsf_superpose_planes(const float *d_xyz, int64_t fstride, int64_t pstride, int64_t n_frames,
                                      int64_t n_sel, const int32_t *d_sel, const double *d_masses,
                                      const double *d_ref, const double *d_refinfo, double *d_xform, void *d_work,
                                      size_t work_bytes, void *stream) {
  if (pstride < 1) return fail(RMSF_EINVAL, "rmsf_superpose_planes: plane stride < 1");
  return superpose_impl("rmsf_superpose_planes", d_xyz, fstride, pstride, n_frames, n_sel, d_sel, d_masses, d_ref,
                        d_refinfo, d_xform, d_work, work_bytes, S(stream));
}

RMSF_EXPORT int64_t rmsf_split_count(int64_t n_frames, int n_splits, int s) {
  if (n_splits < 1 || s < 0 || s >= n_splits) return -1;
  return (n_frames * (s + 1)) / n_splits - (n_frames * s) / n_splits;
}

RMSF_EXPORT int rmsf_accumulate_splits(int64_t n_sel, int64_t n_frames, int aligned) {
  if (n_frames <= 0) return 1;
  // Frame tiles ("splits") per launch.  Measured on MI355X (tools/
  // ubench_welford.hip, 100k atoms x 20k frames): for k_welford_flat long
  // tiles win -- 12 splits (3.5k workgroups, ~1.75 waves of the 2048 resident
  // slots) stream at 6.45 TB/s, 56 splits (16k workgroups) at 6.1 TB/s; the
  // aligned k_accum_atoms (tools/ubench_accum.hip, same-process A/B) runs
  // 3.96 ms at 12 splits vs 4.08 ms at 42.  Splits never exceed kCoefN frames.
  const int64_t lanes = aligned ? n_sel : (3 * n_sel + 3) / 4;
  const int64_t blocks_x = std::max<int64_t>(1, (lanes + kBlock - 1) / kBlock);
  const int64_t target = aligned ? kAccumBlocksAtom : kAccumBlocks;
  int64_t want = (target + blocks_x - 1) / blocks_x;
  want = std::min<int64_t>(want, std::max<int64_t>(1, n_frames / 32));  // tiles of >= 32 frames
  want = std::max<int64_t>(want, (n_frames + kCoefN - 1) / kCoefN);
  want = std::min<int64_t>(want, 65535);
  return (int)std::max<int64_t>(1, want);
}

RMSF_EXPORT int rmsf_accumulate(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                const int32_t *d_sel, const double *d_xform, const double *d_refinfo, int mode,
                                int n_splits, double *d_out0, double *d_out1, void *stream) {
  if (mode != RMSF_MODE_WELFORD && mode != RMSF_MODE_SUM) return fail(RMSF_EINVAL, "rmsf_accumulate: bad mode");
  if (!d_xyz || !d_out0 || (mode == RMSF_MODE_WELFORD && !d_out1) || n_sel < 1 || n_frames < 1 ||
      fstride < (d_sel ? 3 : 3 * n_sel))
    return fail(RMSF_EINVAL, "rmsf_accumulate: bad arguments");
  if (d_xform && !d_refinfo) return fail(RMSF_EINVAL, "rmsf_accumulate: aligned mode needs d_refinfo");
  if (n_splits <= 0) n_splits = rmsf_accumulate_splits(n_sel, n_frames, d_xform != nullptr);
  if (n_splits > 65535) return fail(RMSF_EINVAL, "rmsf_accumulate: n_splits > 65535");
  if ((n_frames + n_splits - 1) / n_splits > kCoefN)
    return fail(RMSF_EINVAL, "rmsf_accumulate: a split exceeds RMSF_MAX_SPLIT_FRAMES frames; raise n_splits");
  hipStream_t s = S(stream);
  const int64_t n_coord = 3 * n_sel;
  const bool flat_ok = !d_xform && !d_sel && mode == RMSF_MODE_WELFORD && (n_coord % 4 == 0) &&
                       (fstride % 4 == 0) && (reinterpret_cast<uintptr_t>(d_xyz) % 16 == 0) &&
                       (reinterpret_cast<uintptr_t>(d_out0) % 16 == 0) &&
                       (reinterpret_cast<uintptr_t>(d_out1) % 16 == 0);
  if (flat_ok) {
    const int64_t n4 = n_coord / 4;
    dim3 grid(grid1(n4), (unsigned)n_splits);
    hipLaunchKernelGGL((k_welford_flat<4>), grid, dim3(kBlock), 0, s, d_xyz, fstride / 4, n4, n_frames, n_splits,
                       d_out0, d_out1, n_coord);
    return after_launch("k_welford_flat");
  }
  dim3 grid(grid1(n_sel), (unsigned)n_splits);
  const bool g = d_sel != nullptr, al = d_xform != nullptr;
#define AC_LAUNCH(M, A, G) \
  hipLaunchKernelGGL((k_accum_atoms<M, A, G, 4>), grid, dim3(kBlock), 0, s, d_xyz, fstride, n_sel, d_sel, n_frames, n_splits, d_xform, d_refinfo, d_out0, d_out1)
  if (mode == RMSF_MODE_WELFORD) {
    if (al && g) AC_LAUNCH(0, true, true);
    else if (al) AC_LAUNCH(0, true, false);
    else if (g) AC_LAUNCH(0, false, true);
    else AC_LAUNCH(0, false, false);
  } else {
    if (al && g) AC_LAUNCH(1, true, true);
    else if (al) AC_LAUNCH(1, true, false);
    else if (g) AC_LAUNCH(1, false, true);
    else AC_LAUNCH(1, false, false);
  }
#undef AC_LAUNCH
  return after_launch("k_accum_atoms");
}

}  // extern "C"

namespace {

int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  const int slot = dev < 64 ? dev : 63;
  if (cached[slot] > 0) return cached[slot];
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cached[slot] = n;
  return n;
}

// Auto workgroups per CU of the balanced grid, by kernel (tools/tune_groups.py,
// 100k atoms x 20k frames, same-process sweeps on MI355X): the float4 Welford
// streams best with 2-3 resident workgroups per CU (3.58 ms at 3/CU vs 3.75 ms
// split grid on the same box); one atom per lane without the transform at 1-2;
// the aligned (transform) kernels are VALU-heavy (~48 fp64 ops per
// atom-frame, 99 VGPRs) and want many short ranges: 3.90 vs 4.06 ms (Welford),
// 3.73 vs 3.77 ms (sum) at 32/CU -- round 2 replaced them by the frame-split
// kernel (k_accum_split_sk) below.  Round 2 (tools/ubench_short.hip, five
// boxes, the strong-scaling shares 100k x 20k/N): the float4 Welford at
// 2/CU = 512 workgroups is the fastest count at every share -- 8 % under
// 3/CU at 2,500 frames (0.444-0.454 vs 0.480-0.494 ms), 2 % at 5,000, within
// +0.4/-1 % at 10,000-20,000 -- so 2/CU, not 3.
constexpr int kSkPerCuFlat = 2, kSkPerCuAtoms = 2, kSkPerCuAligned = 32;
// Aligned accumulate, frame-split (k_accum_split_sk; tools/ubench_accum3.hip,
// accumulate + fold at 100k atoms): Welford Q = 2 at 8 workgroups/CU, sum
// Q = 4 at 4/CU -- against the one-sub-block kernel at 32/CU, 17-20 % less
// time at 2,500 frames, 11-12 % at 5,000, 2-3 % at 20,000.
constexpr int kQWel = 2, kSkPerCuSplitWel = 8, kQSum = 4, kSkPerCuSplitSum = 4;
// Sequential Welford (k_welford_seq): frames per register block (two blocks
// in turn: 8 frames folding while the next 8 load; 4, 6 and 12 are slower).
constexpr int kSeqU = 8;
// gathered selections of >= kSeqAtomsMinSel atoms: one atom per lane, blocks
// of 4 frames (100k of 120k atoms x 20k frames: 5.01 ms against 6.30 for the
// coordinate-per-lane gather; 8 frames 5.28, 2 frames 5.18; 20k atoms: 2x
// slower, too few waves -- profiles/r05_workloads/seq_welford_atoms.txt)
constexpr int kSeqAtomsU = 4;
constexpr int64_t kSeqAtomsMinSel = 49152;


// Balanced-grid plan for `lanes` lanes (cpl coordinates each) over nf frames.
SkPlan sk_plan(int64_t lanes, int cpl, int64_t nf, int n_groups, int mode, int per_cu, int cw = kBlock) {
  SkPlan p{};
  p.lanes = lanes;
  p.cw = cw;
  p.C = (lanes + cw - 1) / cw;
  p.nf = nf;
  p.T = p.C * nf;
  p.cpl = cpl;
  p.mode = mode;
  p.c0 = 0;
  int64_t G = n_groups > 0 ? n_groups : (int64_t)per_cu * cu_count();
  int64_t S = 0;  // > 0: chunk-aligned ranges, S per chunk
  if (n_groups <= 0 && p.C > G) {
    // Many chunks (large frames, e.g. 1M atoms = 12 MB): ranges spanning
    // several chunks put the resident workgroups on far-apart frames (a TLB
    // page per wave).  Cut every chunk into S equal frame ranges instead and
    // order them chunk-major, so resident workgroups share frame rows --
    // the split grid's locality (C4 at 1M x 20k: 38.1 vs 39.0 ms).  At C4's
    // per-rank share (1M x 2,500) S = 1..4 are within 1 %, whole or in the
    // merge's two slabs; S = 6 loses 4 % (profiles/r05_workloads/c4_share_s.txt).
    S = std::max<int64_t>((nf + kCoefN - 1) / kCoefN, (kAccumBlocks + p.C - 1) / p.C);
    S = std::min<int64_t>(S, std::max<int64_t>(1, nf / kSkMinSeg));
    G = p.C * S;
  } else if (n_groups <= 0) {
    G = std::min<int64_t>(G, std::max<int64_t>(1, p.T / kSkMinSeg));
    // Few chunks over many frames (a sparse selection: RMSF.py's 214 CA, the
    // adk density 1 in 220): at most kSkMaxSegsPerChunk ranges per chunk.
    // The fold walks a chunk's segments one after another (a memory round
    // trip per kFoldBatch of them), so hundreds of 32-frame segments cost
    // more than the parallelism they buy.
    // 64 of 16 / 64 / 256 / unlimited measured at 455 of 100k atoms x 20k
    // frames (RMSF.py's two sweeps 2.16 -> 0.75 ms; 10k atoms unchanged;
    // profiles/r06_workloads/sparse_segs.txt)
    G = std::min<int64_t>(G, std::max<int64_t>(1, p.C * kSkMaxSegsPerChunk));
  }
  G = std::max<int64_t>(1, std::min<int64_t>({G, p.T, (int64_t)INT32_MAX}));
  p.G = (int)G;
  // segments per workgroup: a range of W frames meets at most (W-1)/nf + 2
  // chunks and each chunk piece adds at most one cut at kCoefN
  const int64_t W = (p.T + G - 1) / G;
  p.P = (int)((W + kCoefN - 1) / kCoefN + (W - 1) / nf + 2);
  if (S > 0 && G == p.C * S) {
    p.S = (int)S;
    if (nf % S == 0) p.P = (int)((nf / S + kCoefN - 1) / kCoefN);  // exact: one chunk per range
  }
  p.Cs = p.C;
  return p;
}

size_t sk_bytes(const SkPlan &p, bool two) {
  const size_t part = (size_t)p.G * (size_t)p.P * (size_t)p.cw * (size_t)p.cpl * sizeof(double);
  return kSkHdr * sizeof(int64_t) + part * (two ? 2 : 1);
}

bool flat_layout(const float *d_xyz, int64_t fstride, int64_t n_sel, const int32_t *d_sel, const double *d_xform,
                 int mode) {
  return !d_xform && !d_sel && mode == RMSF_MODE_WELFORD && (3 * n_sel) % 4 == 0 && fstride % 4 == 0 &&
         reinterpret_cast<uintptr_t>(d_xyz) % 16 == 0;
}

int fold_shift_launch(const int64_t *hdr, const double *p0, int64_t n_coord, int64_t acc_n, double *acc0, double *acc1,
                      const void *shift, int shift_is_f32, const double *off3, double *t, int64_t l0, int64_t l1,
                      int64_t t_n, int64_t threads, hipStream_t s, int64_t t_slice = 0) {
  if (shift_is_f32)
    hipLaunchKernelGGL(k_fold_sk<1>, dim3(grid1(threads)), dim3(kBlock), 0, s, hdr, p0, n_coord, (double)acc_n, acc0,
                       acc1, shift, off3, t, l0, l1, t_n, t_slice);
  else
    hipLaunchKernelGGL(k_fold_sk<2>, dim3(grid1(threads)), dim3(kBlock), 0, s, hdr, p0, n_coord, (double)acc_n, acc0,
                       acc1, shift, off3, t, l0, l1, t_n, t_slice);
  return after_launch("k_fold_sk");
}

// n1 n2 / T of RMSF.py:39 (`S1[0] * S2[0]/T`: an exact integer product, one
// correctly rounded division -- exact as computed here while n1 n2 < 2^53);
// 0 for T = 0, a step that is never launched.
double merge_weight(int64_t n1, int64_t n2) {
  const int64_t T = n1 + n2;
  return T > 0 ? (double)(n1 * n2) / (double)T : 0.0;
}

// The order in which RMSF.py:143's comm.reduce(S, op=second_order_moments)
// applies its op over the ranks' partials, as (dst, src) steps
// S[dst] = op(S[dst], S[src]); S[0] is the result.
//   RMSF_MERGE_MPI4PY: mpi4py's object reduce with rc.fast_reduce (its
//     default) -- PyMPI_reduce_p2p's binomial tree: for mask = 1, 2, 4, ...
//     rank r with r % (2 mask) == 0 receives S[r + mask] (if that rank
//     exists) and computes op(result, received); ranks with the mask bit set
//     send and stop.  (mpi4py is upstream, not vendored here: restated from
//     its published source, unverified in this container.)
//   RMSF_MERGE_RANK: res = S0, res = op(res, S_i) for i = 1..P-1 -- mpi4py's
//     naive reduce (rc.fast_reduce = False: a gather, then _py_reduce).
std::vector<std::pair<int, int>> reduce_schedule(int n_parts, int order) {
  std::vector<std::pair<int, int>> st;
  if (order == RMSF_MERGE_RANK) {
    for (int i = 1; i < n_parts; ++i) st.push_back({0, i});
    return st;
  }
  for (int64_t mask = 1; mask < n_parts; mask <<= 1)
    for (int64_t r = 0; r + mask < n_parts; r += 2 * mask) st.push_back({(int)r, (int)(r + mask)});
  return st;
}

}  // namespace

extern "C" {

RMSF_EXPORT size_t rmsf_accumulate_balanced_workspace_bytes(int64_t n_sel, int64_t n_frames, int n_groups) {
  if (n_sel < 1 || n_frames < 1) return 0;
  // the larger of the two layouts (float4 columns / one atom per lane), WELFORD
  size_t m = 0;
  for (int per_cu : {kSkPerCuFlat, kSkPerCuAtoms, kSkPerCuAligned, kSkPerCuSplitWel, kSkPerCuSplitSum}) {
    m = std::max(m, sk_bytes(sk_plan((3 * n_sel + 3) / 4, 4, n_frames, n_groups, RMSF_MODE_WELFORD, per_cu), true));
    m = std::max(m, sk_bytes(sk_plan(n_sel, 3, n_frames, n_groups, RMSF_MODE_WELFORD, per_cu), true));
  }
  return m;
}

RMSF_EXPORT int rmsf_accumulate_balanced(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                         const int32_t *d_sel, const double *d_xform, const double *d_refinfo,
                                         int mode, int n_groups, void *d_work, size_t work_bytes, void *stream) {
  if (mode != RMSF_MODE_WELFORD && mode != RMSF_MODE_SUM)
    return fail(RMSF_EINVAL, "rmsf_accumulate_balanced: bad mode");
  if (!d_xyz || !d_work || n_sel < 1 || n_frames < 1 || fstride < (d_sel ? 3 : 3 * n_sel) ||
      reinterpret_cast<uintptr_t>(d_work) % 16 != 0)
    return fail(RMSF_EINVAL, "rmsf_accumulate_balanced: bad arguments");
  if (d_xform && !d_refinfo) return fail(RMSF_EINVAL, "rmsf_accumulate_balanced: aligned mode needs d_refinfo");
  hipStream_t s = S(stream);
  const bool two = mode == RMSF_MODE_WELFORD;
  int64_t *hdr = static_cast<int64_t *>(d_work);
  if (flat_layout(d_xyz, fstride, n_sel, d_sel, d_xform, mode)) {
    const SkPlan pl = sk_plan(3 * n_sel / 4, 4, n_frames, n_groups, mode, kSkPerCuFlat);
    if (work_bytes < sk_bytes(pl, two)) return fail(RMSF_ENOMEM, "rmsf_accumulate_balanced: workspace too small");
    double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
    double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 4;
    hipLaunchKernelGGL((k_welford_flat_sk<4>), dim3(pl.G), dim3(kBlock), 0, s, d_xyz, fstride / 4, pl, hdr, p0, p1);
    return after_launch("k_welford_flat_sk");
  }
  const bool g = d_sel != nullptr, al = d_xform != nullptr;
  const bool split = al && RMSF_SHIFTED_SUMS;  // aligned: the frame-split kernel
  const int per_cu = !al ? kSkPerCuAtoms : !split ? kSkPerCuAligned : two ? kSkPerCuSplitWel : kSkPerCuSplitSum;
  const SkPlan pl = sk_plan(n_sel, 3, n_frames, n_groups, mode, per_cu);
  if (work_bytes < sk_bytes(pl, two)) return fail(RMSF_ENOMEM, "rmsf_accumulate_balanced: workspace too small");
  double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
  double *p1 = two ? p0 + (size_t)pl.G * pl.P * kBlock * 3 : nullptr;
#if RMSF_SHIFTED_SUMS
  if (split) {
#define SPLIT_LAUNCH(M_, G_, Q_) \
  hipLaunchKernelGGL((k_accum_split_sk<M_, true, G_, 4, Q_>), dim3(pl.G), dim3(kBlock * Q_), 0, s, d_xyz, fstride, d_sel, d_xform, d_refinfo, pl, hdr, p0, p1)
    if (two) {
      if (g) SPLIT_LAUNCH(0, true, kQWel);
      else SPLIT_LAUNCH(0, false, kQWel);
    } else {
      if (g) SPLIT_LAUNCH(1, true, kQSum);
      else SPLIT_LAUNCH(1, false, kQSum);
    }
#undef SPLIT_LAUNCH
    return after_launch("k_accum_split_sk");
  }
#endif
#define SK_LAUNCH(M_, A_, G_) \
  hipLaunchKernelGGL((k_accum_atoms_sk<M_, A_, G_, 4>), dim3(pl.G), dim3(kBlock), 0, s, d_xyz, fstride, d_sel, d_xform, d_refinfo, pl, hdr, p0, p1)
  if (two) {
    if (al && g) SK_LAUNCH(0, true, true);
    else if (al) SK_LAUNCH(0, true, false);
    else if (g) SK_LAUNCH(0, false, true);
    else SK_LAUNCH(0, false, false);
  } else {
    if (al && g) SK_LAUNCH(1, true, true);
    else if (al) SK_LAUNCH(1, true, false);
    else if (g) SK_LAUNCH(1, false, true);
    else SK_LAUNCH(1, false, false);
  }
#undef SK_LAUNCH
  return after_launch("k_accum_atoms_sk");
}

RMSF_EXPORT int rmsf_accumulate_balanced_planes(const float *d_xyz, int64_t fstride, int64_t pstride,
                                                int64_t n_frames, int64_t n_sel, const int32_t *d_sel,
                                                const double *d_xform, const double *d_refinfo, int mode,
                                                int n_groups, void *d_work, size_t work_bytes, void *stream) {
#if RMSF_SHIFTED_SUMS
  if (mode != RMSF_MODE_WELFORD && mode != RMSF_MODE_SUM)
    return fail(RMSF_EINVAL, "rmsf_accumulate_balanced_planes: bad mode");
  if (!d_xyz || !d_work || (d_xform && !d_refinfo) || n_sel < 1 || n_frames < 1 || pstride < (d_sel ? 1 : n_sel) ||
      fstride < 3 * pstride || reinterpret_cast<uintptr_t>(d_work) % 16 != 0)
    return fail(RMSF_EINVAL, "rmsf_accumulate_balanced_planes: bad arguments");
  hipStream_t s = S(stream);
  const bool two = mode == RMSF_MODE_WELFORD, g = d_sel != nullptr;
  const int per_cu = !d_xform ? kSkPerCuAtoms : two ? kSkPerCuSplitWel : kSkPerCuSplitSum;
  const SkPlan pl = sk_plan(n_sel, 3, n_frames, n_groups, mode, per_cu);
  if (work_bytes < sk_bytes(pl, two)) return fail(RMSF_ENOMEM, "rmsf_accumulate_balanced_planes: workspace too small");
  int64_t *hdr = static_cast<int64_t *>(d_work);
  double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
  double *p1 = two ? p0 + (size_t)pl.G * pl.P * kBlock * 3 : nullptr;
  if (!d_xform) {  // unaligned: one atom per lane (k_accum_atoms_sk), the row form's kernel for a selection
#define SK_LAUNCH(M_, G_) \
  hipLaunchKernelGGL((k_accum_atoms_sk<M_, false, G_, 4, true>), dim3(pl.G), dim3(kBlock), 0, s, d_xyz, fstride, d_sel, nullptr, nullptr, pl, hdr, p0, p1, pstride)
    if (two && g) SK_LAUNCH(0, true);
    else if (two) SK_LAUNCH(0, false);
    else if (g) SK_LAUNCH(1, true);
    else SK_LAUNCH(1, false);
#undef SK_LAUNCH
    return after_launch("k_accum_atoms_sk");
  }
#define SPLIT_LAUNCH(M_, G_, Q_) \
  hipLaunchKernelGGL((k_accum_split_sk<M_, true, G_, 4, Q_, true>), dim3(pl.G), dim3(kBlock * Q_), 0, s, d_xyz, fstride, d_sel, d_xform, d_refinfo, pl, hdr, p0, p1, pstride)
  if (two) {
    if (g) SPLIT_LAUNCH(0, true, kQWel);
    else SPLIT_LAUNCH(0, false, kQWel);
  } else {
    if (g) SPLIT_LAUNCH(1, true, kQSum);
    else SPLIT_LAUNCH(1, false, kQSum);
  }
#undef SPLIT_LAUNCH
  return after_launch("k_accum_split_sk");
#else
  return fail(RMSF_EINVAL, "rmsf_accumulate_balanced_planes: needs the shifted-sums build");
#endif
}

RMSF_EXPORT int rmsf_fold_balanced(const void *d_work, int64_t n_coord, int mode, int64_t acc_n, double *d_acc0,
                                   double *d_acc1, void *stream) {
  if (mode != RMSF_MODE_WELFORD && mode != RMSF_MODE_SUM) return fail(RMSF_EINVAL, "rmsf_fold_balanced: bad mode");
  if (!d_work || !d_acc0 || (mode == RMSF_MODE_WELFORD && !d_acc1) || n_coord < 1 || acc_n < 0)
    return fail(RMSF_EINVAL, "rmsf_fold_balanced: bad arguments");
  const int64_t *hdr = static_cast<const int64_t *>(d_work);
  const double *p0 = reinterpret_cast<const double *>(hdr + kSkHdr);
  // the plan (and where parts1 starts) is read from the header the
  // accumulate kernel wrote
  // one thread per lane of >= 3 coordinates (the plan's cpl is on the device)
  hipLaunchKernelGGL(k_fold_sk<0>, dim3(grid1((n_coord + 2) / 3)), dim3(kBlock), 0, S(stream), hdr, p0, n_coord,
                     (double)acc_n, d_acc0, d_acc1, nullptr, nullptr, nullptr, (int64_t)0, INT64_MAX, n_coord,
                     (int64_t)0);
  return after_launch("k_fold_sk");
}

RMSF_EXPORT int rmsf_fold_balanced_finalize(const void *d_work, int64_t n_coord, int64_t acc_n, double *d_acc0,
                                            double *d_acc1, int64_t n_total, double *d_rmsf, void *stream) {
  if (!d_work || !d_acc0 || !d_acc1 || !d_rmsf || n_coord < 3 || n_coord % 3 != 0 || acc_n < 0 || n_total < 1)
    return fail(RMSF_EINVAL, "rmsf_fold_balanced_finalize: bad arguments");
  const int64_t *hdr = static_cast<const int64_t *>(d_work);
  const double *p0 = reinterpret_cast<const double *>(hdr + kSkHdr);
  hipLaunchKernelGGL((k_fold_sk<0, true>), dim3(grid1((n_coord + 2) / 3)), dim3(kBlock), 0, S(stream), hdr, p0,
                     n_coord, (double)acc_n, d_acc0, d_acc1, nullptr, nullptr, nullptr, (int64_t)0, INT64_MAX, n_coord,
                     (int64_t)0, d_rmsf, (double)n_total);
  int rc = after_launch("k_fold_sk<FIN>");
  if (rc) return rc;
  // the workspace's plan decides on the device (hdr[6]); an atom plan exits here
  const int64_t n_sel = n_coord / 3;
  hipLaunchKernelGGL(k_finalize_flat, dim3((unsigned)std::min<int64_t>(grid1(n_sel), 1024)), dim3(kBlock), 0,
                     S(stream), hdr, d_acc1, n_sel, (double)n_total, d_rmsf);
  return after_launch("k_finalize_flat");
}

RMSF_EXPORT int rmsf_fold_balanced_shift(const void *d_work, int64_t n_coord, int64_t acc_n, double *d_acc0,
                                         double *d_acc1, const void *d_shift, int shift_is_f32, const double *d_off3,
                                         double *d_t, void *stream) {
  if (!d_work || !d_acc0 || !d_acc1 || !d_shift || !d_t || n_coord < 1 || acc_n < 0)
    return fail(RMSF_EINVAL, "rmsf_fold_balanced_shift: bad arguments");
  const int64_t *hdr = static_cast<const int64_t *>(d_work);
  const double *p0 = reinterpret_cast<const double *>(hdr + kSkHdr);
  return fold_shift_launch(hdr, p0, n_coord, acc_n, d_acc0, d_acc1, d_shift, shift_is_f32, d_off3, d_t, 0, INT64_MAX,
                           n_coord, (n_coord + 2) / 3, S(stream));
}

RMSF_EXPORT int rmsf_fold_balanced_shift_sliced(const void *d_work, int64_t n_coord, int64_t acc_n, double *d_acc0,
                                                double *d_acc1, const void *d_shift, int shift_is_f32,
                                                const double *d_off3, int64_t slice_coords, double *d_t,
                                                void *stream) {
  if (!d_work || !d_acc0 || !d_acc1 || !d_shift || !d_t || n_coord < 1 || acc_n < 0 || slice_coords < 3 ||
      slice_coords % 3)
    return fail(RMSF_EINVAL, "rmsf_fold_balanced_shift_sliced: bad arguments");
  const int64_t *hdr = static_cast<const int64_t *>(d_work);
  const double *p0 = reinterpret_cast<const double *>(hdr + kSkHdr);
  return fold_shift_launch(hdr, p0, n_coord, acc_n, d_acc0, d_acc1, d_shift, shift_is_f32, d_off3, d_t, 0, INT64_MAX,
                           n_coord, (n_coord + 2) / 3, S(stream), slice_coords);
}

// ---- atom slabs of the flat balanced plan (C4's merge overlap) ------------
RMSF_EXPORT int rmsf_balanced_slab_chunks(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                          int64_t *h_chunks) {
  if (!h_chunks || n_sel < 1 || n_frames < 1) return fail(RMSF_EINVAL, "rmsf_balanced_slab_chunks: bad arguments");
  *h_chunks = 0;
  if (!flat_layout(d_xyz, fstride, n_sel, nullptr, nullptr, RMSF_MODE_WELFORD)) return RMSF_OK;
  const SkPlan pl = sk_plan(3 * n_sel / 4, 4, n_frames, 0, RMSF_MODE_WELFORD, kSkPerCuFlat);
  if (pl.S > 0) *h_chunks = pl.C;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_accumulate_balanced_slab(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                              int64_t c0, int64_t c1, void *d_work, size_t work_bytes,
                                              void *stream) {
  if (!d_xyz || !d_work || n_sel < 1 || n_frames < 1 || reinterpret_cast<uintptr_t>(d_work) % 16 != 0)
    return fail(RMSF_EINVAL, "rmsf_accumulate_balanced_slab: bad arguments");
  if (!flat_layout(d_xyz, fstride, n_sel, nullptr, nullptr, RMSF_MODE_WELFORD))
    return fail(RMSF_EINVAL, "rmsf_accumulate_balanced_slab: needs the flat float4 layout (no selection, aligned)");
  SkPlan pl = sk_plan(3 * n_sel / 4, 4, n_frames, 0, RMSF_MODE_WELFORD, kSkPerCuFlat);
  if (pl.S <= 0) return fail(RMSF_EINVAL, "rmsf_accumulate_balanced_slab: the plan is not chunk-aligned");
  if (c0 < 0 || c1 <= c0 || c1 > pl.C) return fail(RMSF_EINVAL, "rmsf_accumulate_balanced_slab: bad chunk range");
  if (work_bytes < sk_bytes(pl, true)) return fail(RMSF_ENOMEM, "rmsf_accumulate_balanced_slab: workspace too small");
  pl.c0 = c0;
  pl.Cs = c1 - c0;
  int64_t *hdr = static_cast<int64_t *>(d_work);
  double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
  double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 4;
  hipLaunchKernelGGL((k_welford_flat_sk<4>), dim3((unsigned)(pl.Cs * pl.S)), dim3(kBlock), 0, S(stream), d_xyz,
                     fstride / 4, pl, hdr, p0, p1);
  return after_launch("k_welford_flat_sk");
}

RMSF_EXPORT int rmsf_fold_balanced_shift_slab(const void *d_work, int64_t n_coord, int64_t acc_n, double *d_acc0,
                                              double *d_acc1, const void *d_shift, int shift_is_f32,
                                              const double *d_off3, double *d_t, int64_t c0, int64_t c1,
                                              void *stream) {
  if (!d_work || !d_acc0 || !d_acc1 || !d_shift || !d_t || n_coord < 4 || acc_n < 0 || c0 < 0 || c1 <= c0)
    return fail(RMSF_EINVAL, "rmsf_fold_balanced_shift_slab: bad arguments");
  // flat plan: 256-lane chunks of 4 coordinates
  const int64_t l0 = c0 * kBlock, l1 = c1 * kBlock;
  const int64_t j0 = 4 * l0, j1 = std::min(4 * l1, n_coord);
  if (j0 >= n_coord) return fail(RMSF_EINVAL, "rmsf_fold_balanced_shift_slab: bad chunk range");
  const int64_t *hdr = static_cast<const int64_t *>(d_work);
  const double *p0 = reinterpret_cast<const double *>(hdr + kSkHdr);
  return fold_shift_launch(hdr, p0, n_coord, acc_n, d_acc0, d_acc1, d_shift, shift_is_f32, d_off3, d_t, l0, l1,
                           j1 - j0, l1 - l0, S(stream));
}

RMSF_EXPORT int rmsf_chan_merge(const double *d_mean_parts, const double *d_m2_parts, const int64_t *h_counts,
                                int n_parts, int64_t n_coord, double *d_mean, double *d_m2, void *stream) {
  if (!d_mean_parts || !d_m2_parts || !h_counts || n_parts < 1 || n_coord < 1 || !d_mean || !d_m2)
    return fail(RMSF_EINVAL, "rmsf_chan_merge: bad arguments");
  int64_t total = 0;
  for (int i = 0; i < n_parts; ++i) {
    if (h_counts[i] < 0) return fail(RMSF_EINVAL, "rmsf_chan_merge: negative count");
    total += h_counts[i];
  }
  if (total == 0) return fail(RMSF_EEMPTY, "rmsf_chan_merge: every partial is empty (no frames)");
  hipStream_t s = S(stream);
  int64_t acc_n = 0;
  for (int g0 = 0; g0 < n_parts; g0 += kMergeGroup) {
    const int np = std::min(kMergeGroup, n_parts - g0);
    MergeCounts c{};
    int64_t run = acc_n;  // the running count before part g0 + i
    for (int i = 0; i < np; ++i) {
      const int64_t n2 = h_counts[g0 + i];
      c.n[i] = (double)n2;
      c.w[i] = merge_weight(run, n2);
      run = (g0 == 0 && i == 0) ? n2 : run + n2;
    }
    hipLaunchKernelGGL(k_chan_merge, dim3(grid1(n_coord)), dim3(kBlock), 0, s, d_mean, d_m2, (double)acc_n,
                       d_mean_parts + (int64_t)g0 * n_coord, d_m2_parts + (int64_t)g0 * n_coord, c, np,
                       g0 == 0 ? 1 : 0, n_coord, d_mean, d_m2);
    int rc = after_launch("k_chan_merge");
    if (rc) return rc;
    acc_n = run;
  }
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_chan_merge_pair(double *d_mean1, double *d_m21, int64_t n1, const double *d_mean2,
                                     const double *d_m22, int64_t n2, int64_t n_coord, void *stream) {
  if (!d_mean1 || !d_m21 || !d_mean2 || !d_m22 || n1 < 0 || n2 < 0 || n_coord < 1)
    return fail(RMSF_EINVAL, "rmsf_chan_merge_pair: bad arguments");
  if (n1 + n2 == 0)
    return fail(RMSF_EEMPTY, "rmsf_chan_merge_pair: both partials are empty (RMSF.py:39 ZeroDivisionError)");
  hipLaunchKernelGGL(k_chan_pair, dim3(grid1(n_coord)), dim3(kBlock), 0, S(stream), d_mean1, d_m21, d_mean2, d_m22,
                     (double)n1, (double)n2, merge_weight(n1, n2), n_coord);
  return after_launch("k_chan_pair");
}

RMSF_EXPORT int rmsf_chan_reduce_steps(int n_parts, int order, int *h_dst, int *h_src, int capacity) {
  if (n_parts < 1 || (order != RMSF_MERGE_RANK && order != RMSF_MERGE_MPI4PY) || capacity < 0)
    return fail(RMSF_EINVAL, "rmsf_chan_reduce_steps: bad arguments");
  const std::vector<std::pair<int, int>> st = reduce_schedule(n_parts, order);
  if ((h_dst || h_src) && capacity < (int)st.size())
    return fail(RMSF_EINVAL, "rmsf_chan_reduce_steps: capacity below n_parts - 1");
  for (size_t i = 0; i < st.size() && (h_dst || h_src); ++i) {
    if (h_dst) h_dst[i] = st[i].first;
    if (h_src) h_src[i] = st[i].second;
  }
  return (int)st.size();
}

RMSF_EXPORT int rmsf_chan_reduce(double *d_mean_parts, double *d_m2_parts, const int64_t *h_counts, int n_parts,
                                 int64_t n_coord, int order, double *d_mean, double *d_m2, void *stream) {
  if (!d_mean_parts || !d_m2_parts || !h_counts || n_parts < 1 || n_coord < 1 || !d_mean || !d_m2 ||
      (order != RMSF_MERGE_RANK && order != RMSF_MERGE_MPI4PY))
    return fail(RMSF_EINVAL, "rmsf_chan_reduce: bad arguments");
  std::vector<int64_t> cnt(h_counts, h_counts + n_parts);
  int64_t total = 0;
  for (int64_t v : cnt) {
    if (v < 0) return fail(RMSF_EINVAL, "rmsf_chan_reduce: negative count");
    total += v;
  }
  if (total == 0) return fail(RMSF_EEMPTY, "rmsf_chan_reduce: every partial is empty (no frames)");
  // the schedule with its counts, on the host; T = 0 steps (two empty
  // states, where RMSF.py:39 raises) are dropped: their dst stays empty
  const std::vector<std::pair<int, int>> sched = reduce_schedule(n_parts, order);
  std::vector<std::pair<int, int>> keep;
  std::vector<int64_t> n1s, n2s;
  for (const auto &p : sched) {
    const int64_t a = cnt[p.first], b = cnt[p.second];
    if (a + b == 0) continue;
    keep.push_back(p);
    n1s.push_back(a);
    n2s.push_back(b);
    cnt[p.first] = a + b;
  }
  hipStream_t s = S(stream);
  const size_t ns = keep.size();
  size_t i0 = 0;
  do {
    const int k = (int)std::min<size_t>(kMaxSteps, ns - i0);
    ChanSteps st{};
    for (int i = 0; i < k; ++i) {
      st.dst[i] = keep[i0 + i].first;
      st.src[i] = keep[i0 + i].second;
      st.n1[i] = (double)n1s[i0 + i];
      st.n2[i] = (double)n2s[i0 + i];
      st.w[i] = merge_weight(n1s[i0 + i], n2s[i0 + i]);
    }
    const bool last = i0 + k >= ns;
    hipLaunchKernelGGL(k_chan_steps, dim3(grid1(n_coord)), dim3(kBlock), 0, s, d_mean_parts, d_m2_parts, st, k,
                       (double)cnt[0], n_coord, last ? d_mean : nullptr, last ? d_m2 : nullptr);
    const int rc = after_launch("k_chan_steps");
    if (rc) return rc;
    i0 += k;
  } while (i0 < ns);
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_sum_splits(const double *d_parts, int n_parts, int64_t n, double *d_sum, void *stream) {
  if (!d_parts || !d_sum || n_parts < 1 || n < 1) return fail(RMSF_EINVAL, "rmsf_sum_splits: bad arguments");
  hipLaunchKernelGGL(k_sum_splits, dim3(grid1(n)), dim3(kBlock), 0, S(stream), d_parts, n_parts, n, d_sum);
  return after_launch("k_sum_splits");
}

RMSF_EXPORT int rmsf_divide(const double *d_x, double divisor, int64_t n, double *d_y, void *stream) {
  if (!d_x || !d_y || n < 1) return fail(RMSF_EINVAL, "rmsf_divide: bad arguments");
  if (divisor == 0.0) return fail(RMSF_EEMPTY, "rmsf_divide: divisor is zero (no frames)");
  hipLaunchKernelGGL(k_divide, dim3(grid1(n)), dim3(kBlock), 0, S(stream), d_x, divisor, n, d_y);
  return after_launch("k_divide");
}

RMSF_EXPORT int rmsf_chan_weight(const double *d_mean_k, double w, int64_t n, double *d_out, void *stream) {
  if (!d_mean_k || !d_out || n < 1) return fail(RMSF_EINVAL, "rmsf_chan_weight: bad arguments");
  hipLaunchKernelGGL(k_chan_weight, dim3(grid1(n)), dim3(kBlock), 0, S(stream), d_mean_k, w, n, d_out);
  return after_launch("k_chan_weight");
}

RMSF_EXPORT int rmsf_chan_deviation(const double *d_mean_k, const double *d_m2_k, const double *d_mean, double n_k,
                                    int64_t n, double *d_out, void *stream) {
  if (!d_mean_k || !d_m2_k || !d_mean || !d_out || n < 1)
    return fail(RMSF_EINVAL, "rmsf_chan_deviation: bad arguments");
  hipLaunchKernelGGL(k_chan_deviation, dim3(grid1(n)), dim3(kBlock), 0, S(stream), d_mean_k, d_m2_k, d_mean, n_k, n,
                     d_out);
  return after_launch("k_chan_deviation");
}

namespace {
int shift_pack(const double *d_mean_k, const double *d_m2_k, const void *d_shift, int shift_is_f32,
               const double *d_off3, double n_k, int64_t n, double *d_t, int64_t t_slice, void *stream) {
  if (!d_mean_k || !d_m2_k || !d_shift || !d_t || n < 1 || n_k < 0 || t_slice < 0)
    return fail(RMSF_EINVAL, "rmsf_chan_shift_pack: bad arguments");
  if (shift_is_f32)
    hipLaunchKernelGGL(k_chan_shift_pack<float>, dim3(grid1(n)), dim3(kBlock), 0, S(stream), d_mean_k, d_m2_k,
                       static_cast<const float *>(d_shift), d_off3, n_k, n, d_t, t_slice);
  else
    hipLaunchKernelGGL(k_chan_shift_pack<double>, dim3(grid1(n)), dim3(kBlock), 0, S(stream), d_mean_k, d_m2_k,
                       static_cast<const double *>(d_shift), d_off3, n_k, n, d_t, t_slice);
  return after_launch("k_chan_shift_pack");
}

int shift_finish(const double *d_t, int64_t t2_off, const void *d_shift, int shift_is_f32, const double *d_off3,
                 int64_t n_sel, int64_t n_frames, double *d_mean, double *d_m2, double *d_rmsf, void *stream) {
  if (!d_t || !d_shift || !d_mean || !d_m2 || n_sel < 1 || t2_off < 3 * n_sel)
    return fail(RMSF_EINVAL, "rmsf_chan_shift_finish: bad arguments");
  if (n_frames < 1) return fail(RMSF_EEMPTY, "rmsf_chan_shift_finish: no frames");
  if (shift_is_f32)
    hipLaunchKernelGGL(k_chan_shift_finish<float>, dim3(grid1(n_sel)), dim3(kBlock), 0, S(stream), d_t,
                       static_cast<const float *>(d_shift), d_off3, n_sel, (double)n_frames, d_mean, d_m2, d_rmsf,
                       t2_off);
  else
    hipLaunchKernelGGL(k_chan_shift_finish<double>, dim3(grid1(n_sel)), dim3(kBlock), 0, S(stream), d_t,
                       static_cast<const double *>(d_shift), d_off3, n_sel, (double)n_frames, d_mean, d_m2, d_rmsf,
                       t2_off);
  return after_launch("k_chan_shift_finish");
}
}  // namespace

RMSF_EXPORT int rmsf_chan_shift_pack(const double *d_mean_k, const double *d_m2_k, const void *d_shift,
                                     int shift_is_f32, const double *d_off3, double n_k, int64_t n, double *d_t,
                                     void *stream) {
  return shift_pack(d_mean_k, d_m2_k, d_shift, shift_is_f32, d_off3, n_k, n, d_t, 0, stream);
}

RMSF_EXPORT int rmsf_chan_shift_pack_sliced(const double *d_mean_k, const double *d_m2_k, const void *d_shift,
                                            int shift_is_f32, const double *d_off3, double n_k, int64_t n,
                                            int64_t slice_coords, double *d_t, void *stream) {
  if (slice_coords < 3 || slice_coords % 3) return fail(RMSF_EINVAL, "rmsf_chan_shift_pack_sliced: bad slice width");
  return shift_pack(d_mean_k, d_m2_k, d_shift, shift_is_f32, d_off3, n_k, n, d_t, slice_coords, stream);
}

RMSF_EXPORT int rmsf_chan_shift_finish(const double *d_t, const void *d_shift, int shift_is_f32, const double *d_off3,
                                       int64_t n_sel, int64_t n_frames, double *d_mean, double *d_m2,
                                       double *d_rmsf, void *stream) {
  return shift_finish(d_t, 3 * n_sel, d_shift, shift_is_f32, d_off3, n_sel, n_frames, d_mean, d_m2, d_rmsf, stream);
}

RMSF_EXPORT int rmsf_chan_shift_finish_slice(const double *d_t, int64_t slice_coords, const void *d_shift,
                                             int shift_is_f32, const double *d_off3, int64_t n_sel, int64_t n_frames,
                                             double *d_mean, double *d_m2, double *d_rmsf, void *stream) {
  return shift_finish(d_t, slice_coords, d_shift, shift_is_f32, d_off3, n_sel, n_frames, d_mean, d_m2, d_rmsf,
                      stream);
}

RMSF_EXPORT size_t rmsf_welford_sequential_workspace_bytes(int64_t n_frames) {
  return n_frames < 1 ? 0 : (size_t)n_frames * sizeof(SeqCoef);
}

RMSF_EXPORT int rmsf_welford_sequential(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                        const int32_t *d_sel, int64_t k0, double *d_mean, double *d_sumsquares,
                                        void *d_work, size_t work_bytes, void *stream) {
  if (!d_xyz || !d_mean || !d_sumsquares || !d_work || n_sel < 1 || (!d_sel && fstride < 3 * n_sel) ||
      n_frames < 0 || k0 < 0 || k0 + n_frames > (int64_t(1) << 53))
    return fail(RMSF_EINVAL, "rmsf_welford_sequential: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  if (work_bytes < rmsf_welford_sequential_workspace_bytes(n_frames))
    return fail(RMSF_EINVAL, "rmsf_welford_sequential: workspace too small");
  hipStream_t s = S(stream);
  SeqCoef *coef = static_cast<SeqCoef *>(d_work);
  hipLaunchKernelGGL(k_seq_coef, dim3(grid1(n_frames)), dim3(kBlock), 0, s, k0, n_frames, coef);
  if (int rc = after_launch("k_seq_coef")) return rc;
  // one coordinate per lane: the recurrence is serial in frames, so the
  // coordinates are the only parallelism, and more waves beat wider loads
  // (100k x 20k: 4.25 ms at 1 coordinate per lane, 4.74 at 2, 5.45 at 4;
  // DESIGN section 4) -- except a large gathered selection, where the
  // gather's address work bounds the stream and one atom per lane wins
  const int64_t n_coord = 3 * n_sel;
  if (d_sel && n_sel >= kSeqAtomsMinSel) {
    hipLaunchKernelGGL((k_welford_seq_atoms<kSeqAtomsU>), dim3(grid1(n_sel)), dim3(kBlock), 0, s, d_xyz, fstride,
                       n_frames, n_sel, d_sel, k0, coef, d_mean, d_sumsquares);
    return after_launch("k_welford_seq_atoms");
  }
  if (d_sel)
    hipLaunchKernelGGL((k_welford_seq<kSeqU, true>), dim3(grid1(n_coord)), dim3(kBlock), 0, s, d_xyz, fstride,
                       n_frames, n_coord, d_sel, k0, coef, d_mean, d_sumsquares);
  else
    hipLaunchKernelGGL((k_welford_seq<kSeqU, false>), dim3(grid1(n_coord)), dim3(kBlock), 0, s, d_xyz, fstride,
                       n_frames, n_coord, nullptr, k0, coef, d_mean, d_sumsquares);
  return after_launch("k_welford_seq");
}

}  // extern "C"

namespace {
bool ref_seq_args_ok(const float *d_frame, const double *d_avg, double avg_divisor, int64_t n_sel,
                     const int32_t *d_sel, const double *d_ref, const double *d_refinfo) {
  return (d_frame == nullptr) != (d_avg == nullptr) && n_sel >= 1 && d_ref && d_refinfo &&
         !(d_avg && !(avg_divisor > 0.0)) && !(d_avg && d_sel);
}
// one k_ref_seq launch of part PART
template <int PART>
void ref_seq_launch(const float *d_frame, const double *d_avg, double div, int64_t n_sel, const int32_t *d_sel,
                    const double *d_masses, double mass_total, double *d_avg_out, double *d_ref, double *d_refinfo,
                    hipStream_t s) {
  const bool g = d_sel != nullptr, m = d_masses != nullptr;
#define SEQREF(F, G, M)                                                                                          \
  hipLaunchKernelGGL((k_ref_seq<F, G, M, PART>), dim3(1), dim3(kBlock), 0, s, d_frame, d_avg, div, n_sel, d_sel, \
                     d_masses, mass_total, d_avg_out, d_ref, d_refinfo)
  if (d_frame) {
    if (g && m) SEQREF(true, true, true);
    else if (g) SEQREF(true, true, false);
    else if (m) SEQREF(true, false, true);
    else SEQREF(true, false, false);
  } else {
    if (m) SEQREF(false, false, true);
    else SEQREF(false, false, false);
  }
#undef SEQREF
}
// RMSF.py:84-85 / 111 + 117-118: ref centred, the record's [0..2]
int ref_centre_seq(const float *d_frame, const double *d_avg, double div, int64_t n_sel, const int32_t *d_sel,
                   const double *d_masses, double mass_total, double *d_avg_out, double *d_ref, double *d_refinfo,
                   hipStream_t s) {
  if (n_sel < kRefGridMin) {
    ref_seq_launch<kRefCentre>(d_frame, d_avg, div, n_sel, d_sel, d_masses, mass_total, d_avg_out, d_ref, d_refinfo,
                               s);
    return after_launch("k_ref_seq");
  }
  if (d_frame && d_sel)
    hipLaunchKernelGGL((k_ref_fill<true, true>), dim3(grid1(n_sel)), dim3(kBlock), 0, s, d_frame, d_avg, div, n_sel,
                       d_sel, d_avg_out, d_ref);
  else if (d_frame)
    hipLaunchKernelGGL((k_ref_fill<true, false>), dim3(grid1(n_sel)), dim3(kBlock), 0, s, d_frame, d_avg, div, n_sel,
                       d_sel, d_avg_out, d_ref);
  else
    hipLaunchKernelGGL((k_ref_fill<false, false>), dim3(grid1(n_sel)), dim3(kBlock), 0, s, d_frame, d_avg, div,
                       n_sel, d_sel, d_avg_out, d_ref);
  if (int rc = after_launch("k_ref_fill")) return rc;
  if (d_masses)
    hipLaunchKernelGGL((k_ref_com_pairs<true>), dim3(1), dim3(384), kRefPairsLds, s, n_sel, d_masses, mass_total,
                       d_ref, d_refinfo);
  else
    hipLaunchKernelGGL((k_ref_com_pairs<false>), dim3(1), dim3(384), kRefPairsLds, s, n_sel, d_masses, mass_total,
                       d_ref, d_refinfo);
  if (int rc = after_launch("k_ref_com_pairs")) return rc;
  hipLaunchKernelGGL(k_ref_centre_grid, dim3(grid1(3 * n_sel)), dim3(kBlock), 0, s, 3 * n_sel, d_refinfo, d_ref);
  return after_launch("k_ref_centre_grid");
}
}  // namespace

extern "C" {

RMSF_EXPORT int rmsf_reference_centre_sequential(const float *d_frame, const double *d_avg, double avg_divisor,
                                                 int64_t n_sel, const int32_t *d_sel, const double *d_masses,
                                                 double mass_total, double *d_avg_out, double *d_ref,
                                                 double *d_refinfo, void *stream) {
  if (!ref_seq_args_ok(d_frame, d_avg, avg_divisor, n_sel, d_sel, d_ref, d_refinfo))
    return fail(RMSF_EINVAL, "rmsf_reference_centre_sequential: bad arguments (exactly one of d_frame / d_avg)");
  return ref_centre_seq(d_frame, d_avg, avg_divisor, n_sel, d_sel, d_masses, mass_total, d_avg_out, d_ref, d_refinfo,
                        S(stream));
}

RMSF_EXPORT int rmsf_reference_sums_sequential(int64_t n_sel, double mass_total, const double *d_ref,
                                               double *d_refinfo, void *stream) {
  if (n_sel < 1 || !d_ref || !d_refinfo) return fail(RMSF_EINVAL, "rmsf_reference_sums_sequential: bad arguments");
  ref_seq_launch<kRefSums>(nullptr, nullptr, 1.0, n_sel, nullptr, nullptr, mass_total, nullptr,
                           const_cast<double *>(d_ref), d_refinfo, S(stream));
  return after_launch("k_ref_seq");
}

RMSF_EXPORT int rmsf_reference_setup_sequential(const float *d_frame, const double *d_avg, double avg_divisor,
                                                int64_t n_sel, const int32_t *d_sel, const double *d_masses,
                                                double mass_total, double *d_avg_out, double *d_ref,
                                                double *d_refinfo, void *stream) {
  if (!ref_seq_args_ok(d_frame, d_avg, avg_divisor, n_sel, d_sel, d_ref, d_refinfo))
    return fail(RMSF_EINVAL, "rmsf_reference_setup_sequential: bad arguments (exactly one of d_frame / d_avg)");
  hipStream_t s = S(stream);
  if (n_sel < kRefGridMin) {  // one launch
    ref_seq_launch<kRefAll>(d_frame, d_avg, avg_divisor, n_sel, d_sel, d_masses, mass_total, d_avg_out, d_ref,
                            d_refinfo, s);
    return after_launch("k_ref_seq");
  }
  if (int rc = ref_centre_seq(d_frame, d_avg, avg_divisor, n_sel, d_sel, d_masses, mass_total, d_avg_out, d_ref,
                              d_refinfo, s))
    return rc;
  return rmsf_reference_sums_sequential(n_sel, mass_total, d_ref, d_refinfo, stream);
}

RMSF_EXPORT int rmsf_frame_com_sequential(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                          const int32_t *d_sel, const double *d_masses, double mass_total,
                                          double *d_xform, void *stream) {
  if (!d_xyz || !d_xform || n_sel < 1 || n_frames < 0 || fstride < (d_sel ? 3 : 3 * n_sel))
    return fail(RMSF_EINVAL, "rmsf_frame_com_sequential: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  hipStream_t s = S(stream);
  const bool g = d_sel != nullptr, m = d_masses != nullptr;
  const dim3 gc((unsigned)n_frames, 3);
  const size_t lds = seq_reserve(3 * n_frames);
#define SEQCOM(G, M)                                                                                         \
  do {                                                                                                       \
    if (seq_pc(3 * n_frames))                                                                                \
      hipLaunchKernelGGL((k_seq_com<G, M, true>), gc, dim3(128), lds, s, d_xyz, fstride, n_sel, d_sel, d_masses, \
                         mass_total, d_xform);                                                               \
    else                                                                                                     \
      hipLaunchKernelGGL((k_seq_com<G, M, false>), gc, dim3(64), lds, s, d_xyz, fstride, n_sel, d_sel,       \
                         d_masses, mass_total, d_xform);                                                     \
  } while (0)
  if (g && m) SEQCOM(true, true);
  else if (g) SEQCOM(true, false);
  else if (m) SEQCOM(false, true);
  else SEQCOM(false, false);
#undef SEQCOM
  return after_launch("k_seq_com");
}

RMSF_EXPORT int rmsf_inner_product_sequential(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                              const int32_t *d_sel, const double *d_ref, double *d_xform,
                                              void *stream) {
  if (!d_xyz || !d_ref || !d_xform || n_sel < 1 || n_frames < 0 || fstride < (d_sel ? 3 : 3 * n_sel))
    return fail(RMSF_EINVAL, "rmsf_inner_product_sequential: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  hipStream_t s = S(stream);
  const dim3 gi((unsigned)n_frames, 10);
  const size_t lds = seq_reserve(10 * n_frames);
#define SEQIP(G, PC) \
  hipLaunchKernelGGL((k_seq_ip<G, PC>), gi, dim3(PC ? 128 : 64), lds, s, d_xyz, fstride, n_sel, d_sel, d_ref, d_xform)
  if (seq_pc(10 * n_frames)) {
    if (d_sel) SEQIP(true, true);
    else SEQIP(false, true);
  } else {
    if (d_sel) SEQIP(true, false);
    else SEQIP(false, false);
  }
#undef SEQIP
  return after_launch("k_seq_ip");
}

RMSF_EXPORT int rmsf_superpose_sequential_qcp(int64_t n_frames, int64_t n_sel, const double *d_refinfo,
                                              double *d_xform, void *stream) {
  if (!d_refinfo || !d_xform || n_sel < 1 || n_frames < 0)
    return fail(RMSF_EINVAL, "rmsf_superpose_sequential_qcp: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  const unsigned fb = (unsigned)((n_frames + 63) / 64);
  hipLaunchKernelGGL(k_seq_qcp, dim3(fb), dim3(64), 0, S(stream), n_frames, n_sel, d_refinfo, d_xform);
  return after_launch("k_seq_qcp");
}

RMSF_EXPORT int rmsf_superpose_sequential_from_com(const float *d_xyz, int64_t fstride, int64_t n_frames,
                                                   int64_t n_sel, const int32_t *d_sel, const double *d_ref,
                                                   const double *d_refinfo, double *d_xform, void *stream) {
  if (!d_xyz || !d_ref || !d_refinfo || !d_xform || n_sel < 1 || n_frames < 0 || fstride < (d_sel ? 3 : 3 * n_sel))
    return fail(RMSF_EINVAL, "rmsf_superpose_sequential_from_com: bad arguments");
  if (int rc = rmsf_inner_product_sequential(d_xyz, fstride, n_frames, n_sel, d_sel, d_ref, d_xform, stream))
    return rc;
  return rmsf_superpose_sequential_qcp(n_frames, n_sel, d_refinfo, d_xform, stream);
}

RMSF_EXPORT int rmsf_superpose_sequential(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                          const int32_t *d_sel, const double *d_masses, double mass_total,
                                          const double *d_ref, const double *d_refinfo, double *d_xform,
                                          void *stream) {
  if (!d_xyz || !d_ref || !d_refinfo || !d_xform || n_sel < 1 || n_frames < 0 || fstride < (d_sel ? 3 : 3 * n_sel))
    return fail(RMSF_EINVAL, "rmsf_superpose_sequential: bad arguments");
  if (int rc = rmsf_frame_com_sequential(d_xyz, fstride, n_frames, n_sel, d_sel, d_masses, mass_total, d_xform,
                                         stream))
    return rc;
  return rmsf_superpose_sequential_from_com(d_xyz, fstride, n_frames, n_sel, d_sel, d_ref, d_refinfo, d_xform,
                                            stream);
}

RMSF_EXPORT int rmsf_accumulate_sequential(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                           const int32_t *d_sel, const double *d_xform, const double *d_refinfo,
                                           int mode, int64_t k0, double *d_acc0, double *d_acc1, void *d_work,
                                           size_t work_bytes, void *stream) {
  const bool wel = mode == RMSF_MODE_WELFORD;
  if ((mode != RMSF_MODE_WELFORD && mode != RMSF_MODE_SUM) || !d_xyz || !d_acc0 || (wel && (!d_acc1 || !d_work)) ||
      n_sel < 1 || n_frames < 0 || k0 < 0 || k0 + n_frames > (int64_t(1) << 53) ||
      fstride < (d_sel ? 3 : 3 * n_sel) || (d_xform != nullptr) != (d_refinfo != nullptr))
    return fail(RMSF_EINVAL, "rmsf_accumulate_sequential: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  hipStream_t s = S(stream);
  const SeqCoef *coef = nullptr;
  if (wel) {
    if (work_bytes < rmsf_welford_sequential_workspace_bytes(n_frames))
      return fail(RMSF_EINVAL, "rmsf_accumulate_sequential: workspace too small");
    hipLaunchKernelGGL(k_seq_coef, dim3(grid1(n_frames)), dim3(kBlock), 0, s, k0, n_frames,
                       static_cast<SeqCoef *>(d_work));
    if (int rc = after_launch("k_seq_coef")) return rc;
    coef = static_cast<const SeqCoef *>(d_work);
  }
  const bool al = d_xform != nullptr, g = d_sel != nullptr;
  const dim3 grid((unsigned)grid1(n_sel));
#define SEQACC(MO, A, G)                                                                                    \
  hipLaunchKernelGGL((k_accum_seq<MO, A, G, 4>), grid, dim3(kBlock), 0, s, d_xyz, fstride, n_frames, n_sel, d_sel, \
                     d_xform, d_refinfo, k0, coef, d_acc0, d_acc1)
  auto launch = [&](auto MOc) {
    constexpr int MO = decltype(MOc)::value;
    if (al && g) SEQACC(MO, true, true);
    else if (al) SEQACC(MO, true, false);
    else if (g) SEQACC(MO, false, true);
    else SEQACC(MO, false, false);
  };
#undef SEQACC
  if (wel) launch(std::integral_constant<int, RMSF_MODE_WELFORD>{});
  else launch(std::integral_constant<int, RMSF_MODE_SUM>{});
  return after_launch("k_accum_seq");
}

RMSF_EXPORT int rmsf_finalize(const double *d_m2, int64_t n_sel, int64_t n_frames, double *d_rmsf, void *stream) {
  if (!d_m2 || !d_rmsf || n_sel < 1) return fail(RMSF_EINVAL, "rmsf_finalize: bad arguments");
  if (n_frames < 1) return fail(RMSF_EEMPTY, "rmsf_finalize: no frames");
  hipLaunchKernelGGL(k_finalize, dim3(grid1(n_sel)), dim3(kBlock), 0, S(stream), d_m2, n_sel, (double)n_frames,
                     d_rmsf);
  return after_launch("k_finalize");
}

RMSF_EXPORT int rmsf_qcp_batch(const double *d_A, const double *d_E0, const double *d_N, int64_t n, double *d_rot,
                               double *d_rmsd, void *stream) {
  if (!d_A || !d_E0 || !d_N || !d_rot || !d_rmsd || n < 0) return fail(RMSF_EINVAL, "rmsf_qcp_batch: bad arguments");
  if (n == 0) return RMSF_OK;
  hipLaunchKernelGGL(k_qcp_batch, dim3(grid1(n)), dim3(kBlock), 0, S(stream), d_A, d_E0, d_N, n, d_rot, d_rmsd);
  return after_launch("k_qcp_batch");
}

RMSF_EXPORT int rmsf_calc_rmsd_rotational_matrix(const double *h_ref, const double *h_conf, int64_t N, double *h_rot,
                                                 const double *h_weights, double *rmsd_out) {
  if (!h_ref || !h_conf || !h_rot || N < 1) return fail(RMSF_EINVAL, "CalcRMSDRotationalMatrix: bad arguments");
  const size_t cb = (size_t)N * 3 * sizeof(double);
  double *d = nullptr;
  const size_t total = 2 * cb + (size_t)N * sizeof(double) + 32 * sizeof(double);
  HIP_TRY(hipMalloc(&d, total));
  double *dref = d, *dconf = d + 3 * N, *dw = d + 6 * N, *dio = d + 7 * N;
  int rc = RMSF_OK;
  do {
    hipError_t e;
    if ((e = hipMemcpy(dref, h_ref, cb, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail("memcpy", e); break; }
    if ((e = hipMemcpy(dconf, h_conf, cb, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail("memcpy", e); break; }
    if (h_weights && (e = hipMemcpy(dw, h_weights, N * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess) {
      rc = hip_fail("memcpy", e);
      break;
    }
    hipLaunchKernelGGL(k_inner_product, dim3(1), dim3(64), 0, 0, dref, dconf, h_weights ? dw : nullptr, N, dio);
    if ((rc = after_launch("k_inner_product"))) break;
    const double nd = (double)N;
    if ((e = hipMemcpy(dio + 10, &nd, sizeof nd, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail("memcpy", e); break; }
    hipLaunchKernelGGL(k_qcp_batch, dim3(1), dim3(kBlock), 0, 0, dio, dio + 9, dio + 10, (int64_t)1, dio + 11, dio + 20);
    if ((rc = after_launch("k_qcp_batch"))) break;
    double h[10];
    if ((e = hipMemcpy(h, dio + 11, sizeof h, hipMemcpyDeviceToHost)) != hipSuccess) { rc = hip_fail("memcpy", e); break; }
    for (int j = 0; j < 9; ++j) h_rot[j] = h[j];
    if (rmsd_out) *rmsd_out = h[9];
  } while (0);
  (void)hipFree(d);
  return rc;
}

RMSF_EXPORT int rmsf_gather_frames(const float *d_src, int64_t fstride, const int64_t *d_frames, int64_t n_frames,
                                   int64_t n_sel, const int32_t *d_sel, float *d_dst, void *stream) {
  if (!d_src || !d_frames || !d_dst || n_frames < 0 || n_sel < 1 || fstride < (d_sel ? 3 : 3 * n_sel))
    return fail(RMSF_EINVAL, "rmsf_gather_frames: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  if (n_frames > 65535) return fail(RMSF_EINVAL, "rmsf_gather_frames: at most 65535 frames per call");
  const dim3 grid((unsigned)grid1(3 * n_sel), (unsigned)n_frames);
  if (d_sel)
    hipLaunchKernelGGL(k_gather_frames<true>, grid, dim3(kBlock), 0, S(stream), d_src, fstride, d_frames, n_sel, d_sel,
                       d_dst);
  else
    hipLaunchKernelGGL(k_gather_frames<false>, grid, dim3(kBlock), 0, S(stream), d_src, fstride, d_frames, n_sel,
                       d_sel, d_dst);
  return after_launch("k_gather_frames");
}

RMSF_EXPORT int rmsf_gather_planes(const float *d_src, int64_t fstride, int64_t pstride, const int64_t *d_frames,
                                   int64_t n_frames, int64_t n_sel, const int32_t *d_sel, float *d_dst,
                                   void *stream) {
  if (!d_src || !d_frames || !d_dst || n_frames < 0 || n_sel < 1 || pstride < (d_sel ? 1 : n_sel) ||
      fstride < 3 * pstride)
    return fail(RMSF_EINVAL, "rmsf_gather_planes: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  if (n_frames > 65535) return fail(RMSF_EINVAL, "rmsf_gather_planes: at most 65535 frames per call");
  const dim3 grid((unsigned)grid1(n_sel), (unsigned)n_frames);
  if (d_sel)
    hipLaunchKernelGGL(k_gather_planes<true>, grid, dim3(kBlock), 0, S(stream), d_src, fstride, pstride, d_frames,
                       n_sel, d_sel, d_dst);
  else
    hipLaunchKernelGGL(k_gather_planes<false>, grid, dim3(kBlock), 0, S(stream), d_src, fstride, pstride, d_frames,
                       n_sel, d_sel, d_dst);
  return after_launch("k_gather_planes");
}

RMSF_EXPORT int rmsf_planes_to_rows(const double *d_src, int64_t n, double *d_dst, void *stream) {
  if (!d_src || !d_dst || n < 1 || d_src == d_dst) return fail(RMSF_EINVAL, "rmsf_planes_to_rows: bad arguments");
  hipLaunchKernelGGL(k_planes_to_rows, dim3(grid1(3 * n)), dim3(kBlock), 0, S(stream), d_src, n, d_dst);
  return after_launch("k_planes_to_rows");
}

RMSF_EXPORT int rmsf_synth_sigma(double *d_sigma, int64_t a0, int64_t n, uint64_t seed, void *stream) {
  if (!d_sigma || a0 < 0 || n < 1) return fail(RMSF_EINVAL, "rmsf_synth_sigma: bad arguments");
  hipLaunchKernelGGL(k_synth_sigma, dim3(grid1(n)), dim3(kBlock), 0, S(stream), d_sigma, a0, n, seed);
  return after_launch("k_synth_sigma");
}

RMSF_EXPORT int rmsf_synth_frames(float *d_out, int64_t fstride, int64_t n_atoms, int64_t f0, int64_t nf,
                                  uint64_t seed, const double *d_motion, void *stream) {
  if (!d_out || n_atoms < 1 || nf < 0 || f0 < 0 || fstride < 3 * n_atoms)
    return fail(RMSF_EINVAL, "rmsf_synth_frames: bad arguments");
  if (nf == 0) return RMSF_OK;
  // One work-item per (frame, atom).  An AQL dispatch's grid size is a 32-bit
  // count of WORK-ITEMS (blocks x 256), not of blocks: a 1M-atom x 20k-frame
  // trajectory (2e10 items) in one launch wraps modulo 2^32 and leaves most
  // frames unwritten.  Each launch covers at most 2^31 items.
  const int64_t per_launch = int64_t(1) << 31;
  for (int64_t done = 0; done < nf;) {
    int64_t fchunk = std::max<int64_t>(1, per_launch / n_atoms);
    fchunk = std::min(fchunk, nf - done);
    hipLaunchKernelGGL(k_synth, dim3(grid1(fchunk * n_atoms)), dim3(kBlock), 0, S(stream), d_out + done * fstride,
                       fstride, n_atoms, f0 + done, fchunk, seed, d_motion);
    int rc = after_launch("k_synth");
    if (rc) return rc;
    done += fchunk;
  }
  return RMSF_OK;
}

}  // extern "C"
