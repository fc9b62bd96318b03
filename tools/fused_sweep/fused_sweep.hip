// fused_sweep.hip -- EXPERIMENT, NOT IN THE PRODUCT LIBRARY (measured and
// rejected in round 3; numbers in DESIGN.md "What did not pay"): the
// single-read aligned sweep, RMSF.py:91-103 (align + sum) and RMSF.py:123-138
// (align + Welford) in ONE pass over the frames.  Built only into the A/B
// harness beside it (ab_fused.cpp; build line there, run.sh runs it).
//
// The two-pass path (rmsf_kernels.hip) reads every frame twice per aligned
// sweep: once for the superposition sums (k_frame_stats, RMSF.py:94-97 +
// qcprot InnerProduct), once to transform and accumulate (k_accum_split_sk,
// RMSF.py:99-103 / 133-138), because a frame's rotation depends on ALL of
// its selected atoms.  Here each frame is read from HBM once and kept on chip
// until its rotation is known.  One persistent launch, one workgroup per CU,
// two roles:
//
//   * GS "stream" workgroups: workgroup c owns the atom slice [c*apw,
//     (c+1)*apw) for the whole launch, one atom per lane of its `nw` compute
//     waves, with the atom's centred reference, mass and running statistics
//     in registers.  Compute waves stream the slice of every frame (12 B per
//     lane, kPF frames of loads in flight), form the frame's 16
//     superposition sums (pivot-relative, as k_frame_stats), reduce them
//     across the wave (permlane32/16 swaps + xor shuffles: lane L ends with
//     value L>>2) and stage the frame in an LDS ring.  The last wave to
//     finish a frame adds the waves' sums in wave order and publishes the
//     workgroup's record -- 16 doubles as 32 tagged 8-B granules ({tag =
//     frame+1, 32-bit half}) stored sc1 (write-through): the data is its own
//     flag -- and raises the workgroup's progress word.  A poller wave
//     fetches the transform records in frame order into LDS (and the
//     frames' pivots ahead of use); the compute waves apply RMSF.py's three
//     f32 rounding points (apply_xform: the two-pass kernel's code) to the
//     staged frame and accumulate shifted sums (shift = the atom's reference
//     position: aligned frames sit on it) or plain sums;
//   * GO "owner" workgroups on the remaining CUs (no stream of their own, so
//     their polls do not queue behind frame loads): owner workgroup k owns
//     the frames f = k (mod GO), alternately to its two groups of four waves.
//     A group waits for every stream workgroup's progress word, gathers the
//     GS records with sc1 loads (re-reading any granule whose tag has not
//     landed), adds them in workgroup order (fixed: bitwise reproducible),
//     solves QCP on one lane (qcp_solve, the published Theobald/Liu
//     algorithm of qcprot) and publishes the 13-double transform record (R,
//     mobile COM, rmsd) the same tagged way, plus the plain per-frame record
//     d_xform[f] for callers.
//
// Every hand-off is placement-independent (MI355X_MICROARCH.md, "Valid
// forms": sc1 granule stores + sc1 loads, every granule's tag checked);
// every spin is bounded (a timeout sets status[0] and every wave leaves).
// The launcher zeroes the per-launch sync state (granule rings, progress
// words, status) with one hipMemsetAsync.  All G workgroups must be
// co-resident: G = the CU count, one workgroup per CU (the LDS ring keeps it
// so).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "rmsf_device.h"
#include "rmsf_hip.h"

#define RMSF_EXPORT __attribute__((visibility("default")))

extern "C" int rmsf_internal_set_error(int code, const char *msg);

namespace {

int ffail(int code, const std::string &m) { return rmsf_internal_set_error(code, m.c_str()); }

constexpr int kThreads = 512;      // 8 waves: <= 7 compute + 1 poller (stream); 2 x 4 owner waves (owner)
constexpr int kMaxCompute = 7;     // compute waves (one atom per lane: <= 448 atoms per stream workgroup)
constexpr int kOwnerWaves = 4;     // waves per owner group (each gathers a quarter of a frame's records)
constexpr int kPF = 16;            // frames of loads in flight per compute lane
constexpr int kNsb = 8;            // frames of per-wave sums staged in LDS
constexpr int kNrs = 64;           // frames of transform records staged in LDS
constexpr int kNrf = 64;           // frames of the per-workgroup record ring (HBM)
constexpr int kNrr = 64;           // frames of the transform-record ring (HBM)
constexpr int kMaxRing = 48;       // LDS frame ring; < kNrf, kNrr, kNrs (ring reuse argument below)
constexpr int kMinRing = 4;
constexpr int kPiv = 128;          // frames of pivots staged in LDS by the poller
constexpr int kRecChunks = 16;     // 16-B chunks per record (one double each)
constexpr int kRChunks = 13;       // transform record: R (9), mobile COM (3), rmsd
constexpr int kPollFrames = 8;     // transform records fetched per poller round
constexpr int kMaxGS = 256;        // stream workgroups at most
constexpr unsigned kSpinMax = 1u << 22;
constexpr int kLdsMax = 160 * 1024;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x3 __attribute__((ext_vector_type(3)));

struct FusedArgs {
  const float *xyz;
  int64_t fstride, nf, n_sel, apw;
  const int32_t *sel;
  const double *masses, *ref, *refinfo;
  double *xform, *acc0, *acc1;
  double acc_n;
  uint32_t *status;  // [0] timeout code, [1] abort flag, [2] compute-wave stalls
  uint32_t *prog;    // [GS] frames whose record each stream workgroup published (monotone)
  uint64_t *rec;     // [kNrf][GS][kRecChunks] chunks of two granules
  uint64_t *rrec;    // [kNrr][kRecChunks]
  uint32_t rec_bytes, rrec_bytes, prog_bytes;
  int GS, GO, nw, ring;
  int64_t fb;        // LDS bytes per staged frame (12 * apw, 16-B aligned)
  int64_t off0;      // offset of the pivot atom (the first selected) in a frame
  uint64_t *trace;   // optional [kTraceEvents][nf] s_memrealtime stamps (tools/ab_fused)
  int preset;        // debug: rrec holds every frame's rotation (index f); no owners
};
// trace events: stream workgroup 0 (compute wave 0 / poller) and the owners
enum { T_SUMS = 0, T_PUB, T_PROG, T_GATH, T_RPUB, T_RDY, T_APPLY, kTraceEvents };
__device__ __forceinline__ void stamp(const FusedArgs &a, int ev, int f) {
  if (a.trace) a.trace[(int64_t)ev * a.nf + f] = __builtin_amdgcn_s_memrealtime();
}
// per-workgroup tail of the trace, rows of kTraceWG words indexed by blockIdx:
// rows 0..7 publish time of sample frames nf/2 + 8k, 8 HW_ID1, 9 XCC_ID,
// 10 stalls, 11 end time, 12..15 ticks waiting for loads / pivots / part
// slots / rotations (summed over compute waves)
constexpr int kTraceWG = 512;
__device__ __forceinline__ uint64_t *trace_wg(const FusedArgs &a, int row) {
  return a.trace + (int64_t)kTraceEvents * a.nf + row * kTraceWG + blockIdx.x;
}

// LDS layout (dynamic shared memory, offsets in bytes)
struct LdsLayout {
  int hdr, part, rs, own, piv, ring, total;
};
// header words
enum {
  H_SUMS = 0,                   // [kNsb] cumulative arrivals of compute waves per sums slot
  H_PUB = H_SUMS + kNsb,        // [kNsb] frame+1 whose sums were published from that slot
  H_RREADY = H_PUB + kNsb,      // [kNrs] frame+1 whose transform record is in rs[]
  H_APPLIED = H_RREADY + kNrs,  // [kMaxCompute] frames applied by each compute wave
  H_PUBLISHED = H_APPLIED + kMaxCompute + 1,  // frames whose record this workgroup published (max)
  H_PIVHI,                      // frames < H_PIVHI have their pivot in the LDS pivot ring
  H_OWNCNT,                     // [2] owner groups: partial arrivals (cumulative)
  H_OWNDONE = H_OWNCNT + 2,     // [2] owner groups: frames finished by the group's wave 0
  H_ABORT = H_OWNDONE + 2,
  H_WORDS
};

__host__ __device__ inline LdsLayout lds_layout(int nw, int ring, int64_t fb) {
  LdsLayout L;
  L.hdr = 0;
  L.part = ((H_WORDS * 4) + 15) / 16 * 16;
  L.rs = L.part + kNsb * nw * 16 * 8;
  L.own = L.rs + kNrs * 16 * 8;
  L.piv = L.own + 2 * kOwnerWaves * 16 * 8;
  L.ring = L.piv + kPiv * 16;
  L.total = L.ring + (int)(ring * fb);
  return L;
}

__device__ __forceinline__ uint32_t *hw(char *s) { return reinterpret_cast<uint32_t *>(s); }

// LDS flag words: acquire loads / release stores (the data they guard is
// plain LDS, read after the flag matched)
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// global abort: any wave that timed out sets it; spinning waves check it
__device__ __forceinline__ bool aborted(const FusedArgs &a, char *s) {
  if (lds_ld(hw(s) + H_ABORT)) return true;
  const uint32_t g = __hip_atomic_load(a.status + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (g) lds_st(hw(s) + H_ABORT, 1u);
  return g != 0;
}
__device__ __forceinline__ void give_up(uint32_t *status, char *s, uint32_t code) {
  __hip_atomic_store(status + 0, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(status + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  lds_st(hw(s) + H_ABORT, 1u);
}
// compute waves: the same, with no global memory access (the poller mirrors
// the global abort flag into LDS), so that no vector-memory instruction sits
// on a spin path of the streaming loop
__device__ __forceinline__ bool spin_lds(unsigned &n, const FusedArgs &a, char *s, uint32_t code) {
  __builtin_amdgcn_s_sleep(2);
  if ((++n & 255u) == 0 && lds_ld(hw(s) + H_ABORT)) return false;
  if (n > kSpinMax) {
    give_up(a.status, s, code);
    return false;
  }
  return true;
}
// one bounded-spin step; false = give up (wave-uniform)
__device__ __forceinline__ bool spin(unsigned &n, const FusedArgs &a, char *s, uint32_t code) {
  __builtin_amdgcn_s_sleep(2);
  if ((++n & 255u) == 0 && aborted(a, s)) return false;
  if (n > kSpinMax) {
    give_up(a.status, s, code);
    return false;
  }
  return true;
}

// ---- granules ---------------------------------------------------------------
// a chunk = one double as two 8-B granules {lo, tag} {hi, tag}, stored by ONE
// 16-B sc1 store; each granule is checked on its own (halves of a 16-B sc1
// store are observed untorn, the 16 B as a whole are not relied upon)
__device__ __forceinline__ u32x4 chunk_of(double v, uint32_t tag) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  return u32x4{(uint32_t)b, tag, (uint32_t)(b >> 32), tag};
}
__device__ __forceinline__ bool chunk_ok(const u32x4 c, uint32_t tag) { return c.y == tag && c.w == tag; }
__device__ __forceinline__ double chunk_val(const u32x4 c) {
  return __longlong_as_double((long long)(((uint64_t)c.z << 32) | c.x));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
constexpr int kSc1 = 16;  // cache-policy bits: sc1 (write-through / L1-bypassing, agent-coherent)
__device__ __forceinline__ void chunk_store(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 c) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, c), r, off, 0, kSc1);
}
__device__ __forceinline__ u32x4 chunk_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
}

// ---- wave reduction of 16 doubles -------------------------------------------
// Transposed butterfly: each step halves the values per lane (permlane32 /
// permlane16 swaps for lane bits 5 and 4, xor shuffles for bits 3 and 2),
// then bits 1 and 0 are folded; lane L ends with the wave total of value
// L >> 2.  The instruction sequence is fixed, so the sums are reproducible.
__device__ __forceinline__ double swap32_add(double a, double b) {
  // v_permlane32_swap exchanges lanes 32-63 of a with lanes 0-31 of b:
  // lanes 0-31 end with a[l] + a[l+32], lanes 32-63 with b[l-32] + b[l]
  const uint32_t al = __double2loint(a), ah = __double2hiint(a);
  const uint32_t bl = __double2loint(b), bh = __double2hiint(b);
  const auto lo = __builtin_amdgcn_permlane32_swap(al, bl, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(ah, bh, false, false);
  return __hiloint2double((int)hi[0], (int)lo[0]) + __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ double swap16_add(double a, double b) {
  // the same over lane bit 4 (odd rows of a <-> even rows of b)
  const uint32_t al = __double2loint(a), ah = __double2hiint(a);
  const uint32_t bl = __double2loint(b), bh = __double2hiint(b);
  const auto lo = __builtin_amdgcn_permlane16_swap(al, bl, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
  return __hiloint2double((int)hi[0], (int)lo[0]) + __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ double xor_step(double a, double b, int bit, int lane) {
  // lanes with `bit` clear keep a and take the partner's a; set: keep b
  const bool up = (lane & bit) != 0;
  const double keep = up ? b : a, send = up ? a : b;
  return keep + __shfl_xor(send, bit, 64);
}
__device__ __forceinline__ double wave_reduce16(const double (&v)[16], int lane) {
  double u[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) u[k] = swap32_add(v[k], v[k + 8]);
  double w4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) w4[k] = swap16_add(u[k], u[k + 4]);
  const double x0 = xor_step(w4[0], w4[2], 8, lane), x1 = xor_step(w4[1], w4[3], 8, lane);
  double y = xor_step(x0, x1, 4, lane);
  y += __shfl_xor(y, 2, 64);
  y += __shfl_xor(y, 1, 64);
  return y;
}

// ---- stream workgroups: compute waves -----------------------------------------
template <int MODE, bool MASSES, bool GATHER>
__device__ void compute_wave(const FusedArgs &a, char *s, int w, int lane) {
  const LdsLayout L = lds_layout(a.nw, a.ring, a.fb);
  uint32_t *H = hw(s);
  double *part = reinterpret_cast<double *>(s + L.part);
  const double *rs = reinterpret_cast<const double *>(s + L.rs);
  const float *piv = reinterpret_cast<const float *>(s + L.piv);
  float *ring = reinterpret_cast<float *>(s + L.ring);
  const int cu = blockIdx.x;
  const int64_t a_lo = (int64_t)cu * a.apw;
  const int64_t n_loc = max((int64_t)0, min(a.apw, a.n_sel - a_lo));
  const int la = w * 64 + lane;
  const bool act = la < n_loc;
  const int64_t atom = act ? a_lo + la : 0;
  const int64_t off = GATHER ? 3 * (int64_t)a.sel[atom] : 3 * atom;
  const double r0 = act ? a.ref[3 * atom] : 0.0, r1 = act ? a.ref[3 * atom + 1] : 0.0,
               r2 = act ? a.ref[3 * atom + 2] : 0.0;
  const double ms = (MASSES && act) ? a.masses[atom] : 0.0;
  const double rc0 = a.refinfo[0], rc1 = a.refinfo[1], rc2 = a.refinfo[2];
  const double sh0 = r0 + rc0, sh1 = r1 + rc1, sh2 = r2 + rc2;  // shift: the atom's reference position
  double S1[3] = {0.0, 0.0, 0.0}, S2[3] = {0.0, 0.0, 0.0};
  const int nf = (int)a.nf;
  const uint32_t nwu = (uint32_t)a.nw;
  const __amdgpu_buffer_rsrc_t rrec = rsrc(a.rec, a.rec_bytes);
  float *my_ring = ring + 3 * la;
  const int fbf = (int)(a.fb / 4);  // floats per staged frame
  const int ring_n = a.ring;
  int g = 0;                        // next frame to apply
  int gslot = 0;                    // g % ring_n
  bool dead = false;
  const bool tr = cu == 0 && w == 0 && lane == 0;  // tracing wave (when a.trace is set)
  uint32_t stalls = 0;  // frames whose rotation was not yet known when their ring slot was needed
  uint64_t tw[4] = {0, 0, 0, 0};  // trace only: ticks waiting for loads, pivots, part slots, rotations
  const bool tt = a.trace != nullptr;
  auto now = []() { return __builtin_amdgcn_s_memrealtime(); };

  auto apply = [&]() {
    const double *t = rs + (g % kNrs) * 16;
    double tt[13];
#pragma unroll
    for (int j = 0; j < 13; ++j) tt[j] = t[j];
    const float *p = my_ring + gslot * fbf;
    float x = p[0], y = p[1], z = p[2];
    apply_xform(x, y, z, tt, rc0, rc1, rc2);
    if (MODE == RMSF_MODE_WELFORD) {
      const double d0 = (double)x - sh0, d1 = (double)y - sh1, d2 = (double)z - sh2;
      S1[0] += d0, S1[1] += d1, S1[2] += d2;
      S2[0] = fma(d0, d0, S2[0]), S2[1] = fma(d1, d1, S2[1]), S2[2] = fma(d2, d2, S2[2]);
    } else {
      S1[0] += (double)x, S1[1] += (double)y, S1[2] += (double)z;
    }
    if (tr) stamp(a, T_APPLY, g);
    ++g;
    gslot = gslot + 1 == ring_n ? 0 : gslot + 1;
    // the poller reuses a record slot once every wave applied its frame
    if (lane == 0) lds_st(H + H_APPLIED + w, (uint32_t)g);
  };
  auto rready = [&](int fr) { return lds_ld(H + H_RREADY + (fr % kNrs)) == (uint32_t)(fr + 1); };

  auto frame = [&](int f, int fslot, float x, float y, float z) {
    if (tr) stamp(a, T_SUMS, f);
    // pivot = the frame's first selected atom, staged in LDS by the poller
    if (lds_ld(H + H_PIVHI) <= (uint32_t)f) {
      const uint64_t t0 = tt ? now() : 0;
      unsigned sp = 0;
      while (lds_ld(H + H_PIVHI) <= (uint32_t)f) {
        if (!spin_lds(sp, a, s, 10)) {
          dead = true;
          return;
        }
      }
      if (tt) tw[1] += now() - t0;
    }
    const float *pv = piv + (f % kPiv) * 4;
    const double P0 = pv[0], P1 = pv[1], P2 = pv[2];
    if (!act) x = (float)P0, y = (float)P1, z = (float)P2;  // contributes 0 to every sum
    const double d0 = (double)x - P0, d1 = (double)y - P1, d2 = (double)z - P2;
    double v[16];
    v[0] = d0, v[1] = d1, v[2] = d2;
    v[3] = ms * d0, v[4] = ms * d1, v[5] = ms * d2;
    v[6] = d0 * r0, v[7] = d0 * r1, v[8] = d0 * r2;
    v[9] = d1 * r0, v[10] = d1 * r1, v[11] = d1 * r2;
    v[12] = d2 * r0, v[13] = d2 * r1, v[14] = d2 * r2;
    v[15] = fma(d0, d0, fma(d1, d1, d2 * d2));
    const double tot = wave_reduce16(v, lane);
    const int slot = f % kNsb;
    // the slot is free once frame f - kNsb was published from it
    if (f >= kNsb && lds_ld(H + H_PUB + slot) != (uint32_t)(f - kNsb + 1)) {
      const uint64_t t0 = tt ? now() : 0;
      unsigned sp = 0;
      while (lds_ld(H + H_PUB + slot) != (uint32_t)(f - kNsb + 1)) {
        if (!spin_lds(sp, a, s, 1)) {
          dead = true;
          return;
        }
      }
      if (tt) tw[2] += now() - t0;
    }
    if ((lane & 3) == 0) part[(slot * a.nw + w) * 16 + (lane >> 2)] = tot;
    uint32_t old = 0;
    if (lane == 0)
      old = __hip_atomic_fetch_add(H + H_SUMS + slot, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old == nwu * (uint32_t)(f / kNsb + 1) - 1) {
      // the last wave of this workgroup for frame f: the workgroup's record
      if (lane < 16) {
        double r = 0.0;
        for (int k = 0; k < a.nw; ++k) r += part[(slot * a.nw + k) * 16 + lane];
        const uint32_t o = (uint32_t)((((f % kNrf) * a.GS + cu) * kRecChunks + lane) * 16);
        chunk_store(rrec, o, chunk_of(r, (uint32_t)(f + 1)));
      }
      if (lane == 0) {
        // progress word: a hint for the owners (the granules' tags are the truth)
        __hip_atomic_fetch_max(a.prog + cu, (uint32_t)(f + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cu == 0) stamp(a, T_PUB, f);
        if (a.trace && f >= (int)a.nf / 2 && f < (int)a.nf / 2 + 64 && (f - (int)a.nf / 2) % 8 == 0)
          *trace_wg(a, (f - (int)a.nf / 2) / 8) = __builtin_amdgcn_s_memrealtime();
        lds_st(H + H_PUB + slot, (uint32_t)(f + 1));
        __hip_atomic_fetch_max(H + H_PUBLISHED, (uint32_t)(f + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    // ring slot fslot holds frame f - ring until it is applied
    while (g <= f - ring_n) {
      unsigned sp = 0;
      const uint64_t t0 = tt && !rready(g) ? now() : 0;
      while (!rready(g)) {
        if (!spin_lds(sp, a, s, 2)) {
          dead = true;
          return;
        }
      }
      if (t0) tw[3] += now() - t0;
      if (lane == 0 && sp) ++stalls;
      apply();
    }
    if (act) {
      float *p = my_ring + fslot * fbf;
      p[0] = x, p[1] = y, p[2] = z;
    }
    while (g <= f && rready(g)) apply();
  };

  // Software pipeline: frame f's 12 B are loaded kPF frames ahead, by plain
  // loads whose waits the compiler places (conservatively: it waits for all of
  // them at the top of each unrolled trip).  (An inline-asm variant with
  // counted waits ran faster but is unsound: the compiler may copy or reuse a
  // register whose load is still in flight -- it faulted the GPU once.)
  float PX[kPF], PY[kPF], PZ[kPF];
  const float *base = a.xyz + off;
  auto issue = [&](float &x, float &y, float &z, const float *q) {
    x = __builtin_nontemporal_load(q);
    y = __builtin_nontemporal_load(q + 1);
    z = __builtin_nontemporal_load(q + 2);
  };
#pragma unroll
  for (int u = 0; u < kPF; ++u)
    if (u < nf) issue(PX[u], PY[u], PZ[u], base + (int64_t)u * a.fstride);
  int fslot = 0;  // f % ring_n
  for (int f0 = 0; f0 < nf && !dead; f0 += kPF) {
#pragma unroll
    for (int u = 0; u < kPF; ++u) {
      const int f = f0 + u;
      if (f < nf && !dead) {
        const uint64_t t0 = tt ? now() : 0;
        const float x = PX[u], y = PY[u], z = PZ[u];
        if (tt) tw[0] += now() - t0;
        if (f + kPF < nf) issue(PX[u], PY[u], PZ[u], base + (int64_t)(f + kPF) * a.fstride);
        frame(f, fslot, x, y, z);
        fslot = fslot + 1 == ring_n ? 0 : fslot + 1;
      }
    }
  }
  // drain: apply what is left
  while (!dead && g < nf) {
    unsigned sp = 0;
    while (!rready(g)) {
      if (!spin_lds(sp, a, s, 3)) {
        dead = true;
        break;
      }
    }
    if (dead) break;
    apply();
  }
  if (lane == 0 && stalls) __hip_atomic_fetch_add(a.status + 2, stalls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 0 && a.trace) {
    __hip_atomic_fetch_add(trace_wg(a, 10), (uint64_t)stalls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(trace_wg(a, 11), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = 0; k < 4; ++k) __hip_atomic_fetch_add(trace_wg(a, 12 + k), tw[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (dead || !act) return;
  // epilogue: this launch's statistics of the atom, folded into the running
  // result (Chan, RMSF.py:36-41; a sum for SUM)
  const double n2 = (double)nf, n1 = a.acc_n;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int64_t o = 3 * atom + j;
    if (MODE == RMSF_MODE_WELFORD) {
      const double shj = j == 0 ? sh0 : (j == 1 ? sh1 : sh2);
      const double dm = S1[j] / n2;
      const double mu2 = shj + dm;
      const double M2 = fmax(0.0, fma(-S1[j], dm, S2[j]));
      if (n1 > 0) {
        const double mu1 = a.acc0[o], M1 = a.acc1[o];
        const double T = n1 + n2, d = mu2 - mu1;
        a.acc0[o] = (n1 * mu1 + n2 * mu2) / T;
        a.acc1[o] = M1 + M2 + (n1 * n2 / T) * (d * d);
      } else {
        a.acc0[o] = mu2;
        a.acc1[o] = M2;
      }
    } else {
      a.acc0[o] = (n1 > 0 ? a.acc0[o] : 0.0) + S1[j];
    }
  }
}

// ---- stream workgroups: poller wave (transform records HBM -> LDS, in frame
// order; pivots ahead of the compute waves) -----------------------------------
__device__ void poller_wave(const FusedArgs &a, char *s, int lane) {
  const LdsLayout L = lds_layout(a.nw, a.ring, a.fb);
  uint32_t *H = hw(s);
  double *rs = reinterpret_cast<double *>(s + L.rs);
  float *piv = reinterpret_cast<float *>(s + L.piv);
  const __amdgpu_buffer_rsrc_t rr = rsrc(a.rrec, a.rrec_bytes);
  const int fk = lane >> 4, v = lane & 15;  // frame offset (0..3) and value of this lane, per load
  const int nf = (int)a.nf;
  int next = 0, pivhi = 0;
  uint32_t have = 0;  // frames next + k (k < kPollFrames) already in LDS
  unsigned spins = 0, rounds = 0;
  while (next < nf) {
    // the global abort flag, mirrored into LDS for the compute waves (one
    // extra round trip, so not every round)
    if ((++rounds & 63u) == 0 && aborted(a, s)) return;
    // pivots of the next 64 frames (one frame per lane), once the compute
    // waves are past the frames whose slots they reuse: every wave has
    // summed the frames below H_PUBLISHED
    if (pivhi < nf && pivhi + 64 <= (int)lds_ld(H + H_PUBLISHED) + kPiv) {
      const int f = pivhi + lane;
      if (f < nf) {
        const float *pv = a.xyz + (int64_t)f * a.fstride + a.off0;
        float *d = piv + (f % kPiv) * 4;
        d[0] = pv[0], d[1] = pv[1], d[2] = pv[2];
      }
      pivhi = min(nf, pivhi + 64);
      if (lane == 0) lds_st(H + H_PIVHI, (uint32_t)pivhi);
    }
    // rs slot of frame f is reused once every compute wave applied f - kNrs
    uint32_t amin = 0xffffffffu;
    for (int k = 0; k < a.nw; ++k) amin = min(amin, lds_ld(H + H_APPLIED + k));
    const int W = min(kPollFrames, min(nf - next, (int)amin + kNrs - next));
    if (W <= 0) {
      if (!spin(spins, a, s, 4)) return;
      continue;
    }
    // poll every frame of the window not yet delivered; deliver each one
    // that is complete (the compute waves check frames one by one)
    bool ok[kPollFrames / 4];
    double val[kPollFrames / 4];
#pragma unroll
    for (int h = 0; h < kPollFrames / 4; ++h) {
      const int k = h * 4 + fk;
      ok[h] = false;
      val[h] = 0.0;
      if (k < W && v < kRChunks && !((have >> k) & 1u)) {
        const int f = next + k;
        const u32x4 c = chunk_load(rr, (uint32_t)((((a.preset ? f : f % kNrr)) * kRecChunks + v) * 16));
        ok[h] = chunk_ok(c, (uint32_t)(f + 1));
        val[h] = chunk_val(c);
      }
    }
    uint32_t got = 0;
#pragma unroll
    for (int h = 0; h < kPollFrames / 4; ++h) {
      const uint64_t good = __ballot(ok[h] && v < kRChunks);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = h * 4 + q;
        if (k < W && !((have >> k) & 1u) && ((good >> (16 * q)) & 0x1fffull) == 0x1fffull) got |= 1u << k;
      }
    }
    if (got == 0) {
      if (!spin(spins, a, s, 5)) return;
      continue;
    }
    spins = 0;
#pragma unroll
    for (int h = 0; h < kPollFrames / 4; ++h) {
      const int k = h * 4 + fk;
      if (((got >> k) & 1u) && v < kRChunks) rs[((next + k) % kNrs) * 16 + v] = val[h];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane < kPollFrames && ((got >> lane) & 1u)) {
      lds_st(H + H_RREADY + ((next + lane) % kNrs), (uint32_t)(next + lane + 1));
      if (blockIdx.x == 0) stamp(a, T_RDY, next + lane);
    }
    have |= got;
    // advance past the delivered prefix
    const int adv = __builtin_ctz(~have);
    next += adv;
    have >>= adv;
  }
}

// ---- owner workgroups ------------------------------------------------------------
// Owner workgroup k owns frames f = k (mod GO); its group q (waves 4q..4q+3)
// takes every other one.  Wave o of a group, lane (i, v) = (lane >> 4,
// lane & 15) loads value v of the records of stream workgroups
// c = i + 4 (kOwnerWaves j + o).  Sum order (fixed, reproducible): j
// ascending, then i (xor 16, 32), then waves o = 0..3.
template <bool MASSES>
__device__ void owner_wave(const FusedArgs &a, char *s, int k, int q, int o, int lane) {
  const LdsLayout L = lds_layout(a.nw, a.ring, a.fb);
  uint32_t *H = hw(s);
  double *own = reinterpret_cast<double *>(s + L.own) + q * kOwnerWaves * 16;  // [0..15] record, [16 o ..] partials
  const __amdgpu_buffer_rsrc_t rrec = rsrc(a.rec, a.rec_bytes);
  const __amdgpu_buffer_rsrc_t rr = rsrc(a.rrec, a.rrec_bytes);
  const __amdgpu_buffer_rsrc_t rprog = rsrc(a.prog, a.prog_bytes);
  const int GS = a.GS, GO = a.GO;
  const int v = lane & 15, i = lane >> 4;
  constexpr int kJ = kMaxGS / (4 * kOwnerWaves);  // records per lane
  const int nf = (int)a.nf;
  if (a.preset) return;
  int it = 0;
  for (int f = k + GO * q; f < nf; f += 2 * GO, ++it) {
    unsigned spins = 0;
    const uint32_t tag = (uint32_t)(f + 1);
    // every stream workgroup's progress word >= f + 1 (4 words per lane)
    for (;;) {
      bool ok = true;
      if (4 * lane < GS) {
        const u32x4 p = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rprog, 16 * lane, 0, kSc1));
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * lane + e < GS) ok = ok && ((e == 0 ? p.x : e == 1 ? p.y : e == 2 ? p.z : p.w) >= tag);
      }
      if (__all(ok)) break;
      if (!spin(spins, a, s, 6)) return;
    }
    if (o == 0 && lane == 0) stamp(a, T_PROG, f);
    double val[kJ];
    uint32_t need = 0;
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      val[j] = 0.0;
      const int c = i + 4 * (kOwnerWaves * j + o);
      if (c < GS) need |= 1u << j;
    }
    for (;;) {
      u32x4 ch[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        if (need & (1u << j)) {
          const int c = i + 4 * (kOwnerWaves * j + o);
          ch[j] = chunk_load(rrec, (uint32_t)((((f % kNrf) * GS + c) * kRecChunks + v) * 16));
        }
      }
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        if ((need & (1u << j)) && chunk_ok(ch[j], tag)) {
          val[j] = chunk_val(ch[j]);
          need &= ~(1u << j);
        }
      }
      if (!__any(need != 0)) break;
      if (!spin(spins, a, s, 7)) return;
    }
    if (o == 0 && lane == 0) stamp(a, T_GATH, f);
    double t = 0.0;
#pragma unroll
    for (int j = 0; j < kJ; ++j) t += val[j];
    t += __shfl_xor(t, 16, 64);
    t += __shfl_xor(t, 32, 64);
    if (o > 0) {
      // hand the partial to wave 0 (the slot is reused once wave 0 is done)
      while (lds_ld(H + H_OWNDONE + q) != (uint32_t)it) {
        if (!spin(spins, a, s, 8)) return;
      }
      if (lane < 16) own[16 * o + v] = t;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_fetch_add(H + H_OWNCNT + q, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    }
    while (lds_ld(H + H_OWNCNT + q) != (uint32_t)((kOwnerWaves - 1) * (it + 1))) {
      if (!spin(spins, a, s, 9)) return;
    }
    for (int w2 = 1; w2 < kOwnerWaves; ++w2) t += lane < 16 ? own[16 * w2 + v] : 0.0;
    if (lane < 16) own[v] = t;  // the frame's 16 sums
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    if (lane == 0) {
      double S[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) S[e] = own[e];
      const double *ri = a.refinfo;
      const double nsel = ri[8], mtot = ri[7];
      const float *pv = a.xyz + (int64_t)f * a.fstride + a.off0;
      const double px = pv[0], py = pv[1], pz = pv[2];
      // COM relative to the pivot, A = sum (x - c) (x) r, E0 (as k_qcp_frames)
      const double cx = (MASSES ? S[3] : S[0]) / mtot;
      const double cy = (MASSES ? S[4] : S[1]) / mtot;
      const double cz = (MASSES ? S[5] : S[2]) / mtot;
      const double sr0 = ri[3], sr1 = ri[4], sr2 = ri[5];
      double A[9];
      A[0] = S[6] - cx * sr0;
      A[1] = S[7] - cx * sr1;
      A[2] = S[8] - cx * sr2;
      A[3] = S[9] - cy * sr0;
      A[4] = S[10] - cy * sr1;
      A[5] = S[11] - cy * sr2;
      A[6] = S[12] - cz * sr0;
      A[7] = S[13] - cz * sr1;
      A[8] = S[14] - cz * sr2;
      const double gmob = S[15] - 2.0 * (cx * S[0] + cy * S[1] + cz * S[2]) + nsel * (cx * cx + cy * cy + cz * cz);
      const double E0 = 0.5 * (gmob + ri[6]);
      double rot[9], rmsd;
      qcp_solve(A, E0, nsel, rot, &rmsd);
#pragma unroll
      for (int e = 0; e < 9; ++e) own[e] = rot[e];
      own[9] = px + cx;
      own[10] = py + cy;
      own[11] = pz + cz;
      own[12] = rmsd;
      own[13] = own[14] = own[15] = 0.0;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    const double res = lane < 16 ? own[v] : 0.0;
    if (lane < kRChunks) chunk_store(rr, (uint32_t)(((f % kNrr) * kRecChunks + lane) * 16), chunk_of(res, tag));
    if (lane < 16) a.xform[(int64_t)f * 16 + lane] = res;
    if (lane == 0) stamp(a, T_RPUB, f);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) lds_st(H + H_OWNDONE + q, (uint32_t)(it + 1));
  }
}

template <int MODE, bool MASSES, bool GATHER>
__global__ __launch_bounds__(kThreads) void k_fused_sweep(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t *H = hw(smem);
  for (int i = threadIdx.x; i < H_WORDS; i += blockDim.x) H[i] = 0u;
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (a.trace && threadIdx.x == 0) {
    *trace_wg(a, 8) = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID (cu, sh, se)
    *trace_wg(a, 9) = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
  }
  if ((int)blockIdx.x < a.GS) {
    if (w < a.nw) compute_wave<MODE, MASSES, GATHER>(a, smem, w, lane);
    else if (w == kThreads / 64 - 1) poller_wave(a, smem, lane);
  } else {
    owner_wave<MASSES>(a, smem, (int)blockIdx.x - a.GS, w / kOwnerWaves, w % kOwnerWaves, lane);
  }
}

int cu_count_fused() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  return n;
}

struct FusedPlan {
  int GS, GO, nw, ring;
  int64_t apw, fb;
  size_t lds, ws_status, ws_prog, ws_rec, ws_rrec;
  bool ok;
};

// GS stream workgroups of <= 7 x 64 atoms, GO = the remaining CUs (8..32)
FusedPlan fused_plan(int64_t n_sel) {
  FusedPlan p{};
  const int G = std::min(cu_count_fused(), kMaxGS + 32);
  const int64_t per = 64LL * kMaxCompute;
  const int64_t need = (n_sel + per - 1) / per;  // stream workgroups at least
  p.GO = (int)std::max<int64_t>(8, std::min<int64_t>(32, G - need));
  p.GS = std::min(kMaxGS, G - p.GO);
  p.apw = (n_sel + p.GS - 1) / p.GS;
  p.nw = (int)((p.apw + 63) / 64);
  p.fb = (12 * p.apw + 15) / 16 * 16;
  const LdsLayout L0 = lds_layout(p.nw, 0, p.fb);
  p.ring = (int)std::min<int64_t>(kMaxRing, (kLdsMax - L0.total) / std::max<int64_t>(16, p.fb));
  p.lds = (size_t)lds_layout(p.nw, p.ring, p.fb).total;
  p.ws_status = 256;
  p.ws_prog = (size_t)(kMaxGS * 4 + 255) / 256 * 256;
  p.ws_rec = (size_t)kNrf * p.GS * kRecChunks * 16;
  p.ws_rrec = (size_t)kNrr * kRecChunks * 16;
  p.ok = n_sel >= 1 && p.GS >= 1 && p.nw >= 1 && p.nw <= kMaxCompute && p.ring >= kMinRing;
  return p;
}

}  // namespace

extern "C" {

RMSF_EXPORT int rmsf_sweep_fused_supported(int64_t n_sel) {
  if (n_sel < 1) return 0;
  return fused_plan(n_sel).ok ? 1 : 0;
}

RMSF_EXPORT size_t rmsf_sweep_fused_workspace_bytes(int64_t n_sel) {
  if (n_sel < 1) return 0;
  const FusedPlan p = fused_plan(n_sel);
  return p.ws_status + p.ws_prog + p.ws_rec + p.ws_rrec;
}

// debug: s_memrealtime stamps of every frame's hand-offs into d_trace
// ([kTraceEvents][n_frames] u64) on the next launches (NULL = off)
static uint64_t *g_trace = nullptr;
RMSF_EXPORT int rmsf_sweep_fused_trace(uint64_t *d_trace) {
  g_trace = d_trace;
  return RMSF_OK;
}

// debug: the next launches take every frame's rotation from d_known (16
// doubles per frame, as d_xform) instead of computing it (d_big: 256 B per
// frame), so that they time the single-read sweep without the rotation chain
static const double *g_known = nullptr;
static uint64_t *g_big = nullptr;
RMSF_EXPORT int rmsf_sweep_fused_preset(const double *d_known, void *d_big) {
  g_known = d_known;
  g_big = static_cast<uint64_t *>(d_big);
  return RMSF_OK;
}
__global__ void k_preset_fill(const double *known, int64_t nf, uint64_t *big) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nf * kRecChunks) return;
  const int64_t f = i / kRecChunks, v = i % kRecChunks;
  const u32x4 c = chunk_of(v < kRChunks ? known[f * 16 + v] : 0.0, (uint32_t)(f + 1));
  *reinterpret_cast<u32x4 *>(big + 2 * i) = c;
}

RMSF_EXPORT int rmsf_sweep_fused(const float *d_xyz, int64_t fstride, int64_t n_frames, int64_t n_sel,
                                 const int32_t *d_sel, const double *d_masses, const double *d_ref,
                                 const double *d_refinfo, int mode, int64_t acc_n, double *d_acc0, double *d_acc1,
                                 double *d_xform, void *d_work, size_t work_bytes, void *stream) {
  if (mode != RMSF_MODE_WELFORD && mode != RMSF_MODE_SUM) return ffail(RMSF_EINVAL, "rmsf_sweep_fused: bad mode");
  if (n_frames == 0) return RMSF_OK;
  if (!d_xyz || !d_ref || !d_refinfo || !d_acc0 || (mode == RMSF_MODE_WELFORD && !d_acc1) || !d_xform || !d_work ||
      n_sel < 1 || n_frames < 0 || acc_n < 0 || fstride < (d_sel ? 3 : 3 * n_sel) ||
      reinterpret_cast<uintptr_t>(d_work) % 16 != 0)
    return ffail(RMSF_EINVAL, "rmsf_sweep_fused: bad arguments");
  if (n_frames >= (int64_t)INT32_MAX) return ffail(RMSF_EINVAL, "rmsf_sweep_fused: n_frames >= 2^31 - 1");
  const FusedPlan p = fused_plan(n_sel);
  if (!p.ok) return ffail(RMSF_EINVAL, "rmsf_sweep_fused: selection too large for the on-chip slice");
  const size_t ws = p.ws_status + p.ws_prog + p.ws_rec + p.ws_rrec;
  if (work_bytes < ws) return ffail(RMSF_ENOMEM, "rmsf_sweep_fused: workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char *w = static_cast<char *>(d_work);
  hipError_t e = hipMemsetAsync(w, 0, ws, s);
  if (e != hipSuccess) return ffail(RMSF_EHIP, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
  FusedArgs a{};
  a.xyz = d_xyz;
  a.fstride = fstride;
  a.nf = n_frames;
  a.n_sel = n_sel;
  a.apw = p.apw;
  a.sel = d_sel;
  a.masses = d_masses;
  a.ref = d_ref;
  a.refinfo = d_refinfo;
  a.xform = d_xform;
  a.acc0 = d_acc0;
  a.acc1 = d_acc1;
  a.acc_n = (double)acc_n;
  a.status = reinterpret_cast<uint32_t *>(w);
  a.prog = reinterpret_cast<uint32_t *>(w + p.ws_status);
  a.rec = reinterpret_cast<uint64_t *>(w + p.ws_status + p.ws_prog);
  a.rrec = reinterpret_cast<uint64_t *>(w + p.ws_status + p.ws_prog + p.ws_rec);
  a.prog_bytes = (uint32_t)p.ws_prog;
  a.rec_bytes = (uint32_t)p.ws_rec;
  a.rrec_bytes = (uint32_t)p.ws_rrec;
  a.GS = p.GS;
  a.GO = p.GO;
  a.nw = p.nw;
  a.ring = p.ring;
  a.fb = p.fb;
  int32_t s0 = 0;
  if (d_sel) {
    e = hipMemcpyAsync(&s0, d_sel, sizeof s0, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return ffail(RMSF_EHIP, std::string("rmsf_sweep_fused: selection read: ") + hipGetErrorString(e));
  }
  a.off0 = 3 * (int64_t)s0;
  a.trace = g_trace;
  if (g_known && g_big) {
    hipLaunchKernelGGL(k_preset_fill, dim3((unsigned)((n_frames * kRecChunks + 255) / 256)), dim3(256), 0, s, g_known,
                       n_frames, g_big);
    a.rrec = g_big;
    a.rrec_bytes = (uint32_t)(n_frames * kRecChunks * 16);
    a.preset = 1;
  }
  const dim3 grid((unsigned)(p.GS + p.GO)), block((unsigned)kThreads);
  const bool g = d_sel != nullptr, m = d_masses != nullptr;
#define FU_LAUNCH(M_, MS_, G_)                                                                          \
  do {                                                                                                  \
    e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_fused_sweep<M_, MS_, G_>),                \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds);                    \
    if (e == hipSuccess) hipLaunchKernelGGL((k_fused_sweep<M_, MS_, G_>), grid, block, p.lds, s, a);    \
  } while (0)
  if (mode == RMSF_MODE_WELFORD) {
    if (g && m) FU_LAUNCH(RMSF_MODE_WELFORD, true, true);
    else if (g) FU_LAUNCH(RMSF_MODE_WELFORD, false, true);
    else if (m) FU_LAUNCH(RMSF_MODE_WELFORD, true, false);
    else FU_LAUNCH(RMSF_MODE_WELFORD, false, false);
  } else {
    if (g && m) FU_LAUNCH(RMSF_MODE_SUM, true, true);
    else if (g) FU_LAUNCH(RMSF_MODE_SUM, false, true);
    else if (m) FU_LAUNCH(RMSF_MODE_SUM, true, false);
    else FU_LAUNCH(RMSF_MODE_SUM, false, false);
  }
#undef FU_LAUNCH
  if (e != hipSuccess) return ffail(RMSF_EHIP, std::string("k_fused_sweep: ") + hipGetErrorString(e));
  e = hipGetLastError();
  if (e != hipSuccess) return ffail(RMSF_EHIP, std::string("k_fused_sweep: ") + hipGetErrorString(e));
  return RMSF_OK;
}

// status words of the last launch on d_work: [0] timeout code (0 = none),
// [1] abort flag, [2] compute-wave stalls (a frame's rotation not yet known
// when its ring slot was needed).  Synchronises `stream`.
RMSF_EXPORT int rmsf_sweep_fused_status(const void *d_work, uint32_t *h_status4, void *stream) {
  if (!d_work || !h_status4) return ffail(RMSF_EINVAL, "rmsf_sweep_fused_status: null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = hipMemcpyAsync(h_status4, d_work, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return ffail(RMSF_EHIP, std::string("rmsf_sweep_fused_status: ") + hipGetErrorString(e));
  return RMSF_OK;
}

}  // extern "C"
