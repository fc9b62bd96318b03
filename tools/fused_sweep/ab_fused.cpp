// A/B of the aligned sweeps in ONE process (not product code): the two-pass
// path (rmsf_superpose + rmsf_accumulate_balanced + rmsf_fold_balanced) vs the
// single-read fused sweep (rmsf_sweep_fused) on the same synthetic frames
// (random rotation + translation per frame, reference = frame 0 -- config
// C3), alternating A/B/A, HIP events on one stream.  Checks the fused result
// against the two-pass one (RMSF, mean, M2, per-frame rmsd) and reports the
// fused kernel's status words (timeouts, compute-wave stalls).
// TRACE=1 adds per-frame hand-off latencies and per-workgroup lags; PRESET=1
// also times the fused sweep with every rotation known in advance (no chain).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Wno-unused-value -Iinclude \
//         -Imdanalysis-mpi_amd/csrc tools/fused_sweep/ab_fused.cpp tools/fused_sweep/fused_sweep.hip \
//         -Lmdanalysis-mpi_amd/lib -lrmsf_hip -Wl,-rpath,'$ORIGIN/../../mdanalysis-mpi_amd/lib' \
//         -o tools/fused_sweep/ab_fused
//   tools/fused_sweep/ab_fused [n_sel] [n_frames] [reps] [mode: 0 welford, 1 sum]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "rmsf_hip.h"

#define OK(x)                                                    \
  do {                                                           \
    int rc_ = (x);                                               \
    if (rc_) {                                                   \
      printf("%s failed: %d %s\n", #x, rc_, rmsf_last_error());  \
      exit(1);                                                   \
    }                                                            \
  } while (0)

extern "C" int rmsf_sweep_fused_supported(int64_t n_sel);
extern "C" size_t rmsf_sweep_fused_workspace_bytes(int64_t n_sel);
extern "C" int rmsf_sweep_fused(const float *, int64_t, int64_t, int64_t, const int32_t *, const double *,
                                const double *, const double *, int, int64_t, double *, double *, double *, void *,
                                size_t, void *);
extern "C" int rmsf_sweep_fused_status(const void *, uint32_t *, void *);
extern "C" int rmsf_sweep_fused_trace(uint64_t *);
extern "C" int rmsf_sweep_fused_preset(const double *, void *);

// per-frame hand-off latencies from the fused kernel's trace (s_memrealtime, 100 MHz)
static void report_trace(const std::vector<uint64_t> &t, int64_t nf) {
  const char *name[] = {"sums(wg0)", "publish(wg0)", "progress(all)", "gathered", "R published", "R in LDS(wg0)", "applied(wg0)"};
  auto ev = [&](int e, int64_t f) { return (double)t[e * nf + f]; };
  const int64_t lo = nf / 4, hi = nf - nf / 4;
  if (hi - lo < 8) return;
  auto pct = [&](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (v.size() - 1))];
  };
  printf("trace (frames %lld..%lld, us): stage delta to previous stage  p10 / p50 / p90\n", (long long)lo, (long long)hi);
  for (int e = 1; e < 7; ++e) {
    std::vector<double> d;
    for (int64_t f = lo; f < hi; ++f) d.push_back((ev(e, f) - ev(e - 1, f)) / 100.0);
    printf("  %-14s - %-14s %8.2f %8.2f %8.2f\n", name[e], name[e - 1], pct(d, 0.1), pct(d, 0.5), pct(d, 0.9));
  }
  std::vector<double> per, lat;
  for (int64_t f = lo + 1; f < hi; ++f) per.push_back((ev(4, f) - ev(4, f - 1)) / 100.0);
  for (int64_t f = lo; f < hi; ++f) lat.push_back((ev(5, f) - ev(1, f)) / 100.0);
  printf("  R-publish period per frame p50 %.3f us; publish(wg0) -> R in LDS(wg0) p50 %.2f us p90 %.2f us\n",
         pct(per, 0.5), pct(lat, 0.5), pct(lat, 0.9));
}

// per-workgroup publish lag at sample frames (relative to the earliest
// publisher of that frame), with the workgroup's hardware placement
static void report_wg(const std::vector<uint64_t> &t) {
  int GS = 0;
  while (GS < 512 && t[GS]) ++GS;
  if (!GS) return;
  std::vector<double> lag(GS, 0.0);
  for (int k = 0; k < 8; ++k) {
    uint64_t mn = ~0ull;
    for (int c = 0; c < GS; ++c) mn = std::min(mn, t[k * 512 + c]);
    for (int c = 0; c < GS; ++c) lag[c] += (t[k * 512 + c] - mn) / 100.0 / 8;
  }
  std::vector<int> idx(GS);
  for (int c = 0; c < GS; ++c) idx[c] = c;
  std::sort(idx.begin(), idx.end(), [&](int x, int y) { return lag[x] > lag[y]; });
  printf("stream workgroups: %d; mean publish lag behind the first, us (wg: lag xcc se/sh/cu stalls end)\n", GS);
  auto show = [&](int c) {
    const uint64_t id = t[8 * 512 + c];
    printf("  wg %3d: %8.2f  xcc %llu se %llu sh %llu cu %2llu  stalls %6llu  wait us/wave load %7.1f piv %7.1f slot %7.1f R %7.1f\n", c, lag[c],
           (unsigned long long)(t[9 * 512 + c] & 15), (unsigned long long)((id >> 13) & 7),
           (unsigned long long)((id >> 12) & 1), (unsigned long long)((id >> 8) & 15),
           (unsigned long long)t[10 * 512 + c], t[12 * 512 + c] / 700.0, t[13 * 512 + c] / 700.0,
           t[14 * 512 + c] / 700.0, t[15 * 512 + c] / 700.0);
  };
  for (int i = 0; i < 12 && i < GS; ++i) show(idx[i]);
  printf("  ...\n");
  for (int i = std::max(12, GS - 4); i < GS; ++i) show(idx[i]);
  // lag histogram by xcc
  double sx[16] = {0};
  int nx[16] = {0};
  for (int c = 0; c < GS; ++c) sx[t[9 * 512 + c] & 15] += lag[c], nx[t[9 * 512 + c] & 15]++;
  printf("  mean lag by xcc:");
  for (int x = 0; x < 16; ++x)
    if (nx[x]) printf(" %d:%.1f(%d)", x, sx[x] / nx[x], nx[x]);
  printf("\n");
}

static std::vector<double> motion_table(int64_t nf, uint64_t seed) {
  std::mt19937_64 g(seed);
  std::normal_distribution<double> nd;
  std::uniform_real_distribution<double> ud(-5.0, 5.0);
  std::vector<double> m(12 * nf);
  for (int64_t f = 0; f < nf; ++f) {
    double q[4], n = 0;
    for (double &v : q) v = nd(g), n += v * v;
    n = std::sqrt(n);
    for (double &v : q) v /= n;
    const double a = q[0], b = q[1], c = q[2], d = q[3];
    double R[9] = {a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c),
                   2 * (b * c + a * d), a * a - b * b + c * c - d * d, 2 * (c * d - a * b),
                   2 * (b * d - a * c), 2 * (c * d + a * b), a * a - b * b - c * c + d * d};
    for (int k = 0; k < 9; ++k) m[12 * f + k] = R[k];
    for (int k = 0; k < 3; ++k) m[12 * f + 9 + k] = 50.0 + ud(g);
  }
  return m;
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000;
  const int64_t nf = argc > 2 ? atoll(argv[2]) : 20000;
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  const int which = argc > 4 ? atoi(argv[4]) : 0;
  if (!rmsf_sweep_fused_supported(n)) {
    printf("fused sweep does not support n_sel=%lld\n", (long long)n);
    return 1;
  }
  const int mode = which == 1 ? RMSF_MODE_SUM : RMSF_MODE_WELFORD;
  float *x;
  double *ref, *info, *xf, *xf2, *m0, *q0, *m1, *q1, *rmsf0, *rmsf1, *dm;
  void *work, *acc, *fw;
  OK(rmsf_malloc((void **)&x, sizeof(float) * 3 * n * nf));
  OK(rmsf_malloc((void **)&ref, sizeof(double) * 3 * n));
  OK(rmsf_malloc((void **)&info, sizeof(double) * RMSF_REFINFO_DOUBLES));
  OK(rmsf_malloc((void **)&xf, sizeof(double) * RMSF_XFORM_DOUBLES * nf));
  OK(rmsf_malloc((void **)&xf2, sizeof(double) * RMSF_XFORM_DOUBLES * nf));
  for (double **p : {&m0, &q0, &m1, &q1}) OK(rmsf_malloc((void **)p, sizeof(double) * 3 * n));
  OK(rmsf_malloc((void **)&rmsf0, sizeof(double) * n));
  OK(rmsf_malloc((void **)&rmsf1, sizeof(double) * n));
  const size_t wb = rmsf_superpose_workspace_bytes(n, nf);
  OK(rmsf_malloc(&work, std::max<size_t>(wb, 16)));
  const size_t ab = rmsf_accumulate_balanced_workspace_bytes(n, nf, 0);
  OK(rmsf_malloc(&acc, ab));
  const size_t fb = rmsf_sweep_fused_workspace_bytes(n);
  OK(rmsf_malloc(&fw, fb));
  std::vector<double> mot = motion_table(nf, 7);
  OK(rmsf_malloc((void **)&dm, sizeof(double) * mot.size()));
  OK(rmsf_memcpy_h2d(dm, mot.data(), sizeof(double) * mot.size(), nullptr));
  OK(rmsf_synth_frames(x, 3 * n, n, 0, nf, 1, dm, nullptr));
  OK(rmsf_reference_setup(x, nullptr, n, nullptr, nullptr, ref, info, nullptr));
  OK(rmsf_stream_synchronize(nullptr));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto two_pass = [&](double *mo, double *qo, double *xfo) {
    OK(rmsf_superpose(x, 3 * n, nf, n, nullptr, nullptr, ref, info, xfo, work, wb, nullptr));
    OK(rmsf_accumulate_balanced(x, 3 * n, nf, n, nullptr, xfo, info, mode, 0, acc, ab, nullptr));
    OK(rmsf_fold_balanced(acc, 3 * n, mode, 0, mo, mode == RMSF_MODE_WELFORD ? qo : nullptr, nullptr));
  };
  auto fused = [&](double *mo, double *qo, double *xfo) {
    OK(rmsf_sweep_fused(x, 3 * n, nf, n, nullptr, nullptr, ref, info, mode, 0, mo, qo, xfo, fw, fb, nullptr));
  };
  auto timeit = [&](auto &&fn, double *mo, double *qo, double *xfo) {
    hipEventRecord(a, nullptr);
    fn(mo, qo, xfo);
    hipEventRecord(b, nullptr);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
  };
  // correctness first (one of each); the fused launch traced when TRACE is set
  uint64_t *dtr = nullptr;
  if (getenv("TRACE")) {
    OK(rmsf_malloc((void **)&dtr, sizeof(uint64_t) * (7 * nf + 16 * 512)));
    hipMemset(dtr, 0, sizeof(uint64_t) * (7 * nf + 16 * 512));
    OK(rmsf_sweep_fused_trace(dtr));
  }
  two_pass(m0, q0, xf);
  fused(m1, q1, xf2);
  if (dtr) {
    std::vector<uint64_t> ht(7 * nf);
    OK(rmsf_memcpy_d2h(ht.data(), dtr, sizeof(uint64_t) * 7 * nf, nullptr));
    report_trace(ht, nf);
    std::vector<uint64_t> wg(16 * 512);
    OK(rmsf_memcpy_d2h(wg.data(), dtr + 7 * nf, sizeof(uint64_t) * wg.size(), nullptr));
    report_wg(wg);
    OK(rmsf_sweep_fused_trace(nullptr));
  }
  OK(rmsf_stream_synchronize(nullptr));
  uint32_t st[4];
  OK(rmsf_sweep_fused_status(fw, st, nullptr));
  printf("n_sel=%lld n_frames=%lld mode=%d  fused status: timeout=%u abort=%u stalls=%u\n", (long long)n,
         (long long)nf, mode, st[0], st[1], st[2]);
  if (st[0]) {
    printf("FUSED TIMEOUT code %u\n", st[0]);
    return 2;
  }
  std::vector<double> hm0(3 * n), hm1(3 * n), hq0(3 * n), hq1(3 * n), hx0(16 * nf), hx1(16 * nf);
  OK(rmsf_memcpy_d2h(hm0.data(), m0, 24 * n, nullptr));
  OK(rmsf_memcpy_d2h(hm1.data(), m1, 24 * n, nullptr));
  OK(rmsf_memcpy_d2h(hx0.data(), xf, 128 * nf, nullptr));
  OK(rmsf_memcpy_d2h(hx1.data(), xf2, 128 * nf, nullptr));
  double dmean = 0, drmsf = 0, drot = 0, drmsd = 0, dcom = 0;
  for (int64_t i = 0; i < 3 * n; ++i) dmean = std::max(dmean, std::fabs(hm0[i] - hm1[i]));
  if (mode == RMSF_MODE_WELFORD) {
    OK(rmsf_memcpy_d2h(hq0.data(), q0, 24 * n, nullptr));
    OK(rmsf_memcpy_d2h(hq1.data(), q1, 24 * n, nullptr));
    for (int64_t i = 0; i < n; ++i) {
      const double r0 = std::sqrt((hq0[3 * i] + hq0[3 * i + 1] + hq0[3 * i + 2]) / nf);
      const double r1 = std::sqrt((hq1[3 * i] + hq1[3 * i + 1] + hq1[3 * i + 2]) / nf);
      drmsf = std::max(drmsf, std::fabs(r0 - r1));
    }
  }
  for (int64_t f = 0; f < nf; ++f) {
    for (int k = 0; k < 9; ++k) drot = std::max(drot, std::fabs(hx0[16 * f + k] - hx1[16 * f + k]));
    for (int k = 9; k < 12; ++k) dcom = std::max(dcom, std::fabs(hx0[16 * f + k] - hx1[16 * f + k]));
    drmsd = std::max(drmsd, std::fabs(hx0[16 * f + 12] - hx1[16 * f + 12]));
  }
  printf("fused vs two-pass: max|dmean|=%.3e max|dRMSF|=%.3e max|dR|=%.3e max|dCOM|=%.3e max|drmsd|=%.3e  rmsd[0..2]=%.4f %.4f %.4f\n",
         dmean, drmsf, drot, dcom, drmsd, hx1[12], hx1[16 + 12], hx1[32 + 12]);
  const double gb = 12.0 * n * nf / 1e9;
  for (int r = 0; r < reps; ++r) {
    const float t0 = timeit(two_pass, m0, q0, xf);
    const float t1 = timeit(fused, m1, q1, xf2);
    const float t2 = timeit(two_pass, m0, q0, xf);
    OK(rmsf_sweep_fused_status(fw, st, nullptr));
    printf("rep %d: two-pass %.3f ms | fused %.3f ms (%.2f TB/s single-read, %.3f of 8 TB/s; stalls %u, timeout %u) | two-pass %.3f ms\n",
           r, t0, t1, gb / t1, gb / t1 / 8.0, st[2], st[0], t2);
  }
  if (getenv("PRESET")) {
    // the single-read sweep with every rotation known (no chain), beside the
    // two passes of the two-pass path timed alone
    void *big;
    OK(rmsf_malloc(&big, (size_t)256 * nf));
    auto sup = [&](double *, double *, double *xfo) {
      OK(rmsf_superpose(x, 3 * n, nf, n, nullptr, nullptr, ref, info, xfo, work, wb, nullptr));
    };
    auto accf = [&](double *mo, double *qo, double *xfo) {
      OK(rmsf_accumulate_balanced(x, 3 * n, nf, n, nullptr, xfo, info, mode, 0, acc, ab, nullptr));
      OK(rmsf_fold_balanced(acc, 3 * n, mode, 0, mo, mode == RMSF_MODE_WELFORD ? qo : nullptr, nullptr));
    };
    two_pass(m0, q0, xf);
    OK(rmsf_sweep_fused_preset(xf, big));
    for (int r = 0; r < reps; ++r) {
      const float t1 = timeit(fused, m1, q1, xf2);
      const float ts = timeit(sup, m0, q0, xf);
      const float ta = timeit(accf, m0, q0, xf);
      OK(rmsf_sweep_fused_status(fw, st, nullptr));
      printf("preset rep %d: fused with rotations known %.3f ms (%.2f TB/s; stalls %u timeout %u) | superpose pass %.3f ms | accumulate+fold pass %.3f ms\n",
             r, t1, gb / t1, st[2], st[0], ts, ta);
    }
    OK(rmsf_sweep_fused_preset(nullptr, nullptr));
    OK(rmsf_memcpy_d2h(hm0.data(), m0, 24 * n, nullptr));
    OK(rmsf_memcpy_d2h(hm1.data(), m1, 24 * n, nullptr));
    double dm = 0;
    for (int64_t i = 0; i < 3 * n; ++i) dm = std::max(dm, std::fabs(hm0[i] - hm1[i]));
    printf("preset fused vs two-pass: max|dmean|=%.3e\n", dm);
  }
  return 0;
}
