// Read-pattern probe for the C2 Welford stream, in one process with the
// library kernels (csrc/rmsf_kernels.hip included): does the access pattern
// of the superposition-sums kernel (64-frame x narrow-column tiles staged
// through LDS, which streamed at ~6.9 TB/s in tools/ubench_stats2.hip) beat
// the flat float4 stream (lane = 4 coordinates, frames walked per lane)?
// Finding (profiles/r02_workloads/ubench_welford2*.txt): the tiled reads are
// not faster once results are written -- but the partial STORES were the
// cost: plain stores beside the nt-load stream cost 2-8 %, nontemporal
// stores a third of that, which made the library's flat kernel 3.58 -> 3.49
// ms.  100k atoms x 20k frames.  Not product code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_welford2.hip -o tools/ubench_welford2
#include "../mdanalysis-mpi_amd/csrc/rmsf_kernels.hip"

// ---- candidate stream kernels measured here and NOT adopted (the library keeps
// k_welford_flat_sk, which streams as fast once its partials are written with
// nontemporal stores): moved out of csrc/rmsf_kernels.hip in round 2 ----
namespace {
// k_welford_tiles_sk -- the C2 stream (contiguous selection, no alignment,
// float4-aligned rows) on the balanced grid with chunks of kTW = 64
// coordinates: a workgroup walks its range's segments (one chunk, <= kCoefN
// frames each) in tiles of 64 frames x 64 coordinates staged HBM -> registers
// -> LDS (next tile in flight), and wave w keeps the shifted sums of tile rows
// 16w..16w+15 for lane = coordinate; the 4 waves' sums (one shift per
// segment: they add) are folded in LDS and stored as one (mean, M2) partial
// per segment, exactly the layout k_fold_sk replays (cw = 16 lanes of 4).
// Versus k_welford_flat_sk (lane = 4 coordinates walking frames): the
// resident workgroups read the same few frames at once, 256 B of each per
// workgroup -- 3.44-3.50 ms vs 3.58-3.69 ms for 100k atoms x 20k frames in
// the same process (tools/ubench_welford2.hip).
constexpr int kTW = 64;                       // coordinates per chunk (a 256-B frame-row column)
constexpr int kTWL = kTW / 4;                 // float4 lanes per chunk
constexpr int kTWF = 64;                      // frames per tile
constexpr int kTWP = kTW + 4;                 // LDS row pitch (floats): 16-B rows
constexpr int kTWH = kBlock / kTW;            // waves = frame parts of a tile
constexpr int kTWPre = kTWF * kTWL / kBlock;  // float4 staging loads per thread per tile
static_assert(kTWH * kTW == kBlock && kTWF % kTWH == 0 && kTWF * kTWL % kBlock == 0, "tile shape");
static_assert(2 * kTWH * kTW * 2 <= kTWF * kTWP, "part fold (doubles) fits in the tile buffer (floats)");

__global__ __launch_bounds__(kBlock) void k_welford_tiles_sk(const float *__restrict__ xyz, int64_t stride4,
                                                             SkPlan pl, int64_t *__restrict__ hdr,
                                                             double *__restrict__ parts0,
                                                             double *__restrict__ parts1) {
  __shared__ __attribute__((aligned(16))) float tile[kTWF * kTWP];
  const int b = sk_range(pl, blockIdx.x);
  if (blockIdx.x == 0 && threadIdx.x == 0) sk_write_header(hdr, pl);
  const int cc = threadIdx.x % kTW;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x / kTW);  // = the wave
  const f32x4 *__restrict__ x4 = reinterpret_cast<const f32x4 *>(xyz);
  int64_t lo = uni64(sk_lo(pl, b));
  const int64_t hi = uni64(sk_lo(pl, b + 1));
  int64_t slot = (int64_t)b * pl.P;
  while (lo < hi) {
    int64_t c, f0;
    const int len = __builtin_amdgcn_readfirstlane((int)sk_seg_len(pl, lo, hi, &c, &f0));
    c = uni64(c);
    f0 = uni64(f0);
    const int64_t l0 = c * kTWL, fend = f0 + len;
    f32x4 pre[kTWPre];
    auto gload = [&](int64_t t0) {
#pragma unroll
      for (int k = 0; k < kTWPre; ++k) {
        const int idx = threadIdx.x + k * kBlock;
        const int row = idx / kTWL, col = idx % kTWL;
        const int64_t f = min(t0 + row, fend - 1);
        const int64_t lane = l0 + col;
        pre[k] = lane < pl.lanes ? __builtin_nontemporal_load(x4 + f * stride4 + lane) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    };
    double sh = 0.0, s1 = 0.0, s2 = 0.0;
    gload(f0);
    for (int64_t t0 = f0; t0 < fend; t0 += kTWF) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kTWPre; ++k) {
        const int idx = threadIdx.x + k * kBlock;
        const int row = idx / kTWL, col = idx % kTWL;
        *reinterpret_cast<f32x4 *>(tile + row * kTWP + 4 * col) = pre[k];
      }
      __syncthreads();
      if (t0 + kTWF < fend) gload(t0 + kTWF);
      if (t0 == f0) sh = (double)tile[cc];  // the segment's first frame: the shift
      const int nf = (int)min((int64_t)kTWF, fend - t0);
      const int r0 = h * (kTWF / kTWH);
      if (r0 + kTWF / kTWH <= nf) {  // wave-uniform
#pragma unroll
        for (int j = 0; j < kTWF / kTWH; ++j) {
          const double d = (double)tile[(r0 + j) * kTWP + cc] - sh;
          s1 += d;
          s2 = fma(d, d, s2);
        }
      } else {
        for (int r = r0; r < nf; ++r) {
          const double d = (double)tile[r * kTWP + cc] - sh;
          s1 += d;
          s2 = fma(d, d, s2);
        }
      }
    }
    // the waves' sums share the shift: add them, convert, store one partial
    __syncthreads();
    double *red = reinterpret_cast<double *>(tile);
    red[h * kTW + cc] = s1;
    red[(kTWH + h) * kTW + cc] = s2;
    __syncthreads();
    if (h == 0) {
      double a = red[cc], q = red[kTWH * kTW + cc];
#pragma unroll
      for (int v = 1; v < kTWH; ++v) {
        a += red[v * kTW + cc];
        q += red[(kTWH + v) * kTW + cc];
      }
      shifted_to_moments(a, q, sh, g_coef.v[len - 1].b);
      nt_store(a, parts0 + slot * kTW + cc);
      nt_store(q, parts1 + slot * kTW + cc);
    }
    lo += len;
    ++slot;
  }
}

// k_welford_sweep -- the C2 stream with the whole chip sweeping the frames
// together.  Workgroup b owns K consecutive 64-coordinate chunks for ALL
// frames of the batch and walks them window by window (64 frames): window w
// of chunk 0, of chunk 1, ..., then window w+1 -- every workgroup does the
// same work per window, so the resident workgroups stay on nearby frames
// (short frame splits of the tiled kernel streamed 3.39-3.49 ms vs 3.58-3.64
// for the flat kernel, but paid for it in partial stores:
// tools/ubench_welford2.hip).  Per chunk the statistics stay in registers
// (shifted sums, one shift per kCoefN-frame segment) and one (mean, M2)
// partial per segment is stored -- the layout of the balanced plan with one
// range per chunk (S = 1, cw = 16 lanes of 4), so k_fold_sk folds it.
template <int KMAX>
__global__ __launch_bounds__(kBlock) void k_welford_sweep(const float *__restrict__ xyz, int64_t stride4, SkPlan pl,
                                                          int K, int64_t *__restrict__ hdr,
                                                          double *__restrict__ parts0, double *__restrict__ parts1) {
  __shared__ __attribute__((aligned(16))) float tile[kTWF * kTWP];
  if (blockIdx.x == 0 && threadIdx.x == 0) sk_write_header(hdr, pl);
  const int cc = threadIdx.x % kTW;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x / kTW);  // = the wave
  const f32x4 *__restrict__ x4 = reinterpret_cast<const f32x4 *>(xyz);
  const int64_t cbeg = (int64_t)blockIdx.x * K;
  const int nk = (int)min((int64_t)K, pl.C - cbeg);
  const int64_t nf = pl.nf;
  double sh[KMAX], s1[KMAX], s2[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) sh[k] = s1[k] = s2[k] = 0.0;
  f32x4 pre[kTWPre];
  auto gload = [&](int64_t t0, int k) {
    const int64_t l0 = (cbeg + k) * kTWL;
#pragma unroll
    for (int q = 0; q < kTWPre; ++q) {
      const int idx = threadIdx.x + q * kBlock;
      const int row = idx / kTWL, col = idx % kTWL;
      const int64_t f = min(t0 + row, nf - 1);
      const int64_t lane = l0 + col;
      pre[q] = lane < pl.lanes ? __builtin_nontemporal_load(x4 + f * stride4 + lane) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (nk > 0) gload(0, 0);
  for (int64_t w0 = 0; w0 < nf; w0 += kTWF) {
    const int nfr = (int)min((int64_t)kTWF, nf - w0);
    const bool seg_start = w0 % kCoefN == 0;
    const bool seg_end = (w0 + kTWF) % kCoefN == 0 || w0 + kTWF >= nf;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k >= nk) break;  // uniform
      __syncthreads();
#pragma unroll
      for (int q = 0; q < kTWPre; ++q) {
        const int idx = threadIdx.x + q * kBlock;
        const int row = idx / kTWL, col = idx % kTWL;
        *reinterpret_cast<f32x4 *>(tile + row * kTWP + 4 * col) = pre[q];
      }
      __syncthreads();
      if (k + 1 < nk) gload(w0, k + 1);
      else if (w0 + kTWF < nf) gload(w0 + kTWF, 0);
      if (seg_start) {
        sh[k] = (double)tile[cc];  // the segment's first frame: the shift
        s1[k] = s2[k] = 0.0;
      }
      const int r0 = h * (kTWF / kTWH);
      if (r0 + kTWF / kTWH <= nfr) {  // wave-uniform
#pragma unroll
        for (int j = 0; j < kTWF / kTWH; ++j) {
          const double d = (double)tile[(r0 + j) * kTWP + cc] - sh[k];
          s1[k] += d;
          s2[k] = fma(d, d, s2[k]);
        }
      } else {
        for (int r = r0; r < nfr; ++r) {
          const double d = (double)tile[r * kTWP + cc] - sh[k];
          s1[k] += d;
          s2[k] = fma(d, d, s2[k]);
        }
      }
      if (seg_end) {  // the waves' sums share the shift: add, convert, store the segment's partial
        __syncthreads();
        double *red = reinterpret_cast<double *>(tile);
        red[h * kTW + cc] = s1[k];
        red[(kTWH + h) * kTW + cc] = s2[k];
        __syncthreads();
        if (h == 0) {
          double a = red[cc], qq = red[kTWH * kTW + cc];
#pragma unroll
          for (int v = 1; v < kTWH; ++v) {
            a += red[v * kTW + cc];
            qq += red[(kTWH + v) * kTW + cc];
          }
          const int64_t seg = w0 / kCoefN;
          const int len = (int)min((int64_t)kCoefN, nf - seg * kCoefN);
          shifted_to_moments(a, qq, sh[k], g_coef.v[len - 1].b);
          const int64_t slot = (cbeg + k) * pl.P + seg;
          nt_store(a, parts0 + slot * kTW + cc);
          nt_store(qq, parts1 + slot * kTW + cc);
        }
      }
    }
  }
}

// Plan of k_welford_sweep: one logical range per 64-coordinate chunk (S = 1:
// segments of <= kCoefN frames, slots chunk*P + segment), so k_fold_sk
// replays it; *k_out = chunks per workgroup (<= kSweepK), *g_out = workgroups.
constexpr int kSweepK = 8;
SkPlan sweep_plan(int64_t lanes, int64_t nf, int mode, int per_cu, int *k_out, int *g_out) {
  SkPlan p{};
  p.lanes = lanes;
  p.cw = kTWL;
  p.cpl = 4;
  p.C = (lanes + kTWL - 1) / kTWL;
  p.nf = nf;
  p.T = p.C * nf;
  p.G = (int)p.C;
  p.S = 1;
  p.P = (int)((nf + kCoefN - 1) / kCoefN);
  p.mode = mode;
  const int64_t slots = (int64_t)per_cu * cu_count();
  const int64_t K = std::max<int64_t>(1, std::min<int64_t>(kSweepK, (p.C + slots - 1) / slots));
  *k_out = (int)K;
  *g_out = (int)((p.C + K - 1) / K);
  return p;
}

}  // namespace

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

// k_welford_flat_sk with the round-1 plain partial stores (A/B of the store kind)
__global__ __launch_bounds__(kBlock) void flat_plain(const float *__restrict__ xyz, int64_t stride4, SkPlan pl,
                                                    int64_t *__restrict__ hdr, double *__restrict__ parts0,
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
      wel_flat_run<4>(reinterpret_cast<const f32x4 *>(xyz) + f0 * stride4 + i4, stride4, len, m, q);
      const int64_t o = slot * (kBlock * 4) + 4 * threadIdx.x;
      f64x2 *a = reinterpret_cast<f64x2 *>(parts0 + o);
      f64x2 *bb = reinterpret_cast<f64x2 *>(parts1 + o);
      a[0] = f64x2{m[0], m[1]};
      a[1] = f64x2{m[2], m[3]};
      bb[0] = f64x2{q[0], q[1]};
      bb[1] = f64x2{q[2], q[3]};
    }
    lo += len;
    ++slot;
  }
}

// tile = 64 frames x W floats (W/4 float4 per row), staged HBM -> regs -> LDS
// (next tile in flight); thread t owns coordinate c = t % W of frame half
// h = t / W (W = 128: 2 halves of 32 frames; W = 256: 1 half of 64 frames)
// and keeps shifted sums over its frames of every tile.  Blocks = (column
// block, frame split).
template <int W, bool WRITE = false, bool STORE = true, bool NTS = false>
__global__ __launch_bounds__(256) void welford_tiles(const float *__restrict__ xyz, int64_t fstride, int64_t n_frames,
                                                     int64_t n_cols, int n_splits, double *__restrict__ out) {
  constexpr int TF = 64, R4 = W / 4, NPRE = TF * R4 / 256, H = 256 / W, FPH = TF / H;
  constexpr int P = W + 4;  // row pitch (floats): 16-B rows
  __shared__ __attribute__((aligned(16))) float tile[TF * P];
  const int64_t c0 = (int64_t)blockIdx.x * W;
  const int64_t fb = n_frames * blockIdx.y / n_splits, fe = n_frames * (blockIdx.y + 1) / n_splits;
  const int c = threadIdx.x % W, h = threadIdx.x / W;
  f32x4 pre[NPRE];
  auto gload = [&](int64_t f0) {
#pragma unroll
    for (int k = 0; k < NPRE; ++k) {
      const int idx = threadIdx.x + k * 256;
      const int row = idx / R4, col = idx % R4;
      const int64_t f = min(f0 + row, fe - 1);
      pre[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(xyz + f * fstride + c0) + col);
    }
  };
  double sh = 0, s1 = 0, s2 = 0;
  bool first = true;
  gload(fb);
  for (int64_t f0 = fb; f0 < fe; f0 += TF) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPRE; ++k) {
      const int idx = threadIdx.x + k * 256;
      const int row = idx / R4, col = idx % R4;
      *reinterpret_cast<f32x4 *>(tile + row * P + 4 * col) = pre[k];
    }
    __syncthreads();
    if (f0 + TF < fe) gload(f0 + TF);
    const int nf = (int)min((int64_t)TF, fe - f0);
    if (first) {  // one shift per coordinate for the whole block (row 0): the H parts' sums add
      sh = (double)tile[c];
      first = false;
    }
#pragma unroll 8
    for (int j = 0; j < FPH; ++j) {
      const int r = h * FPH + j;
      if (r >= nf) break;
      const double d = (double)tile[r * P + c] - sh;
      s1 += d;
      s2 = fma(d, d, s2);
    }
  }
  if (WRITE) {  // the H frame parts add in LDS; one (mean, M2) per coordinate per split
    __syncthreads();
    double *red = reinterpret_cast<double *>(tile);  // [2][H][W] doubles <= the tile buffer
    red[h * W + c] = s1;
    red[(H + h) * W + c] = s2;
    __syncthreads();
    if (h == 0) {
      double a = 0, q = 0;
      for (int k = 0; k < H; ++k) a += red[k * W + c], q += red[(H + k) * W + c];
      const double n = (double)(fe - fb), d = a / n;
      double *o = out + (int64_t)blockIdx.y * 2 * n_cols;
      if (!STORE) {  // combine + convert, but store only conditionally: the store's own cost
        if (q == 12345.678) o[c0 + c] = sh + d;
      } else if (c0 + c < n_cols) {
        if (NTS) {
          __builtin_nontemporal_store(sh + d, o + c0 + c);
          __builtin_nontemporal_store(fmax(0.0, q - a * d), o + n_cols + c0 + c);
        } else {
          o[c0 + c] = sh + d;
          o[n_cols + c0 + c] = fmax(0.0, q - a * d);
        }
      }
    }
  } else if (s1 + s2 == 12345.678) {
    out[c0 + c] = sh;
  }
}
}  // namespace ub

int main() {
  const int64_t n = 100000, nf = 20000, fs = 3 * n;
  float *x;
  double *out;
  CK(hipMalloc(&x, sizeof(float) * (fs * nf + 1024)));  // + the last column block's overhang
  CK(hipMalloc(&out, sizeof(double) * (fs + 1024)));
  double *part;  // partials: up to 128 splits x 4 frame parts x 2 x n_cols
  CK(hipMalloc(&part, sizeof(double) * 128 * 4 * 2 * (fs + 64)));
  if (rmsf_synth_frames(x, fs, n, 0, nf, 0, nullptr, nullptr)) {
    printf("synth failed\n");
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
    printf("%-40s %7.3f ms (min %7.3f)  %6.0f GB/s\n", name, sum / R, best, bytes / (sum / R) / 1e6);
    fflush(stdout);
  };
  const size_t ab = rmsf_accumulate_balanced_workspace_bytes(n, nf, 0);
  const size_t ab2 = std::max(ab, (size_t)1 << 30);
  void *acc;
  CK(hipMalloc(&acc, ab2));
  const int64_t n4 = fs / 4;
  auto tiles_sk = [&](const SkPlan &pl) {
    int64_t *hdr = static_cast<int64_t *>(acc);
    double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
    double *p1 = p0 + (size_t)pl.G * pl.P * kTW;
    if (sk_bytes(pl, true) > ab2) {
      printf("workspace too small\n");
      exit(1);
    }
    hipLaunchKernelGGL(k_welford_tiles_sk, dim3(pl.G), dim3(kBlock), 0, 0, x, fs / 4, pl, hdr, p0, p1);
    hipLaunchKernelGGL(k_fold_sk, dim3(grid1(fs)), dim3(kBlock), 0, 0, hdr, p0, fs, 0.0, out, part);
  };
  {  // agreement of the two decompositions (different fold orders: rounding only)
    std::vector<double> m0(fs), q0(fs), m1(fs), q1(fs);
    rmsf_accumulate_balanced(x, fs, nf, n, nullptr, nullptr, nullptr, RMSF_MODE_WELFORD, 0, acc, ab, nullptr);
    rmsf_fold_balanced(acc, fs, RMSF_MODE_WELFORD, 0, out, part, nullptr);
    CK(hipMemcpy(m0.data(), out, 8 * fs, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q0.data(), part, 8 * fs, hipMemcpyDeviceToHost));
    tiles_sk(sk_plan(n4, 4, nf, 0, RMSF_MODE_WELFORD, 3, kTWL));
    CK(hipMemcpy(m1.data(), out, 8 * fs, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q1.data(), part, 8 * fs, hipMemcpyDeviceToHost));
    double dm = 0, dq = 0;
    for (int64_t i = 0; i < fs; ++i) {
      dm = std::max(dm, std::fabs(m0[i] - m1[i]));
      dq = std::max(dq, std::fabs(q0[i] - q1[i]) / std::max(1.0, std::fabs(q0[i])));
    }
    printf("tiles_sk vs flat: max |d mean| %.3e A, max rel |d M2| %.3e\n", dm, dq);
    int K = 0, Gw = 0;
    const SkPlan sp = sweep_plan(n4, nf, RMSF_MODE_WELFORD, 3, &K, &Gw);
    {
      int64_t *hdr = static_cast<int64_t *>(acc);
      double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
      double *p1 = p0 + (size_t)sp.G * sp.P * kTW;
      hipLaunchKernelGGL((k_welford_sweep<kSweepK>), dim3(Gw), dim3(kBlock), 0, 0, x, fs / 4, sp, K, hdr, p0, p1);
      hipLaunchKernelGGL(k_fold_sk, dim3(grid1(fs)), dim3(kBlock), 0, 0, hdr, p0, fs, 0.0, out, part);
    }
    CK(hipMemcpy(m1.data(), out, 8 * fs, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q1.data(), part, 8 * fs, hipMemcpyDeviceToHost));
    dm = dq = 0;
    for (int64_t i = 0; i < fs; ++i) {
      dm = std::max(dm, std::fabs(m0[i] - m1[i]));
      dq = std::max(dq, std::fabs(q0[i] - q1[i]) / std::max(1.0, std::fabs(q0[i])));
    }
    printf("sweep vs flat: max |d mean| %.3e A, max rel |d M2| %.3e\n", dm, dq);
  }
  for (int rep = 0; rep < 2; ++rep) {
    run("lib k_welford_flat_sk (+fold)", [&] {
      rmsf_accumulate_balanced(x, fs, nf, n, nullptr, nullptr, nullptr, RMSF_MODE_WELFORD, 0, acc, ab, nullptr);
      rmsf_fold_balanced(acc, fs, RMSF_MODE_WELFORD, 0, out, part, nullptr);
    });
    char nm[96];
    {
      const SkPlan pl = sk_plan(n4, 4, nf, 0, RMSF_MODE_WELFORD, kSkPerCuFlat);
      for (int ab_rep = 0; ab_rep < 2; ++ab_rep) {
        run("A/B: flat, nontemporal partial stores", [&] {
          int64_t *hdr = static_cast<int64_t *>(acc);
          double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
          double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 4;
          hipLaunchKernelGGL((k_welford_flat_sk<4>), dim3(pl.G), dim3(kBlock), 0, 0, x, fs / 4, pl, hdr, p0, p1);
        });
        run("A/B: flat, plain partial stores", [&] {
          int64_t *hdr = static_cast<int64_t *>(acc);
          double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
          double *p1 = p0 + (size_t)pl.G * pl.P * kBlock * 4;
          hipLaunchKernelGGL(ub::flat_plain, dim3(pl.G), dim3(kBlock), 0, 0, x, fs / 4, pl, hdr, p0, p1);
        });
      }
    }
    for (int S : {5, 16, 32}) {
      snprintf(nm, sizeof nm, "probe W=64 splits=%d no epilogue", S);
      run(nm, [&] {
        hipLaunchKernelGGL((ub::welford_tiles<64>), dim3((unsigned)(fs / 64 + (fs % 64 != 0)), S), dim3(256), 0, 0,
                           x, fs, nf, fs, S, out);
      });
      snprintf(nm, sizeof nm, "probe W=64 splits=%d combine, no store", S);
      run(nm, [&] {
        hipLaunchKernelGGL((ub::welford_tiles<64, true, false>), dim3((unsigned)(fs / 64 + (fs % 64 != 0)), S),
                           dim3(256), 0, 0, x, fs, nf, fs, S, part);
      });
      snprintf(nm, sizeof nm, "probe W=64 splits=%d combine + nt store", S);
      run(nm, [&] {
        hipLaunchKernelGGL((ub::welford_tiles<64, true, true, true>), dim3((unsigned)(fs / 64 + (fs % 64 != 0)), S),
                           dim3(256), 0, 0, x, fs, nf, fs, S, part);
      });
      snprintf(nm, sizeof nm, "probe W=64 splits=%d combine + store", S);
      run(nm, [&] {
        hipLaunchKernelGGL((ub::welford_tiles<64, true, true>), dim3((unsigned)(fs / 64 + (fs % 64 != 0)), S),
                           dim3(256), 0, 0, x, fs, nf, fs, S, part);
      });
    }
    for (int per_cu : {3}) {
      int K = 0, Gw = 0;
      const SkPlan pl = sweep_plan(n4, nf, RMSF_MODE_WELFORD, per_cu, &K, &Gw);
      snprintf(nm, sizeof nm, "sweep per_cu=%d K=%d G=%d P=%d", per_cu, K, Gw, pl.P);
      run(nm, [&] {
        int64_t *hdr = static_cast<int64_t *>(acc);
        double *p0 = reinterpret_cast<double *>(hdr + kSkHdr);
        double *p1 = p0 + (size_t)pl.G * pl.P * kTW;
        hipLaunchKernelGGL((k_welford_sweep<kSweepK>), dim3(Gw), dim3(kBlock), 0, 0, x, fs / 4, pl, K, hdr, p0, p1);
        hipLaunchKernelGGL(k_fold_sk, dim3(grid1(fs)), dim3(kBlock), 0, 0, hdr, p0, fs, 0.0, out, part);
      });
    }
    for (int per_cu : {3}) {
      const SkPlan pl = sk_plan(n4, 4, nf, 0, RMSF_MODE_WELFORD, per_cu, kTWL);
      snprintf(nm, sizeof nm, "tiles_sk auto per_cu=%d G=%d S=%d P=%d", per_cu, pl.G, pl.S, pl.P);
      run(nm, [&] { tiles_sk(pl); });
    }
    for (int G : {6144}) {
      const SkPlan pl = sk_plan(n4, 4, nf, G, RMSF_MODE_WELFORD, 3, kTWL);
      snprintf(nm, sizeof nm, "tiles_sk G=%d S=%d P=%d", pl.G, pl.S, pl.P);
      run(nm, [&] { tiles_sk(pl); });
    }
  }
  return 0;
}
