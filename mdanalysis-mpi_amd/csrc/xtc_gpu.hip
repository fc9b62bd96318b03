// xtc_gpu.hip -- XTC decompression on the GPU (config C5).
//
// The host decoder (xtc.cpp) replaces libxdrfile behind MDAnalysis'
// XTCReader, i.e. what `universe.trajectory[frame]` runs at RMSF.py:92,124;
// it is bound by host cores (~2k frames/s of 250k atoms on 16 threads).  Here
// the compressed frame records themselves are streamed: read from the file
// into a pinned slot (pread, host threads), copied to HBM (about 1/6 of the
// decoded bytes), and decompressed on the device, one wave per frame, frames
// in parallel.  A frame's xdr3dfcoord stream is sequential only in its bit
// offsets, so the decode is two passes (see "two-pass frame decode" below):
// a wave-uniform walk that reads just the 1-6 flag bits per atom group, and
// a lane-parallel decode of 64 recorded groups at a time.  Output: float32
// [n][n_atoms][3] Angstrom frames in HBM with MDAnalysis' rounding
// f32(f32(int * f32(1/prec)) * 10), bit-identical to the host decoder.  The
// selection is applied downstream (the accumulate kernels gather it
// in-kernel), as for any HBM-resident trajectory.
//
// Packed triples of <= 52 bits are split with two exact double-precision
// divisions (quotient estimate by reciprocal, one correction step); wider
// ones use the byte-wise long division of the published algorithm.  Every
// read is bounded by the record length; a corrupt frame sets its status and
// is filled with NaN.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <mutex>
#include <memory>
#include <functional>
#include <condition_variable>
#include <string>
#include <thread>
#include <vector>

#include "rmsf_hip.h"
#include "xtc_internal.h"
#include "host_affinity.h"

#define RMSF_EXPORT __attribute__((visibility("default")))

extern "C" int rmsf_internal_set_error(int code, const char *msg);

namespace {

int fail(int code, const std::string &m) { return rmsf_internal_set_error(code, m.c_str()); }

#define XD_HIP(expr)                                                                                  \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess) return fail(RMSF_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr int kMagic = 1995;
constexpr int kFirstIdx = 9;
constexpr int kLastIdx = 73;
struct MagicTable {
  int v[kLastIdx];
};
struct InvTable {
  double v[kLastIdx];
};
constexpr MagicTable make_magic() {
  return MagicTable{{0,        0,        0,        0,        0,        0,       0,       0,       0,       8,
                     10,       12,       16,       20,       25,       32,      40,      50,      64,      80,
                     101,      128,      161,      203,      256,      322,     406,     512,     645,     812,
                     1024,     1290,     1625,     2048,     2580,     3250,    4096,    5060,    6501,    8192,
                     10321,    13003,    16384,    20642,    26007,    32768,   41285,   52015,   65536,   82570,
                     104031,   131072,   165140,   208063,   262144,   330280,  416127,  524287,  660561,  832255,
                     1048576,  1321122,  1664510,  2097152,  2642245,  3329021, 4194304, 5284491, 6658042, 8388607,
                     10568983, 13316085, 16777216}};
}
constexpr InvTable make_inv() {
  InvTable t{};
  const MagicTable m = make_magic();
  for (int i = 0; i < kLastIdx; ++i) t.v[i] = m.v[i] ? 1.0 / (double)m.v[i] : 0.0;
  return t;
}
__constant__ MagicTable g_magic = make_magic();
__constant__ InvTable g_inv = make_inv();
constexpr MagicTable h_magic = make_magic();
constexpr InvTable h_inv = make_inv();

// status codes per frame
constexpr int32_t kOk = 0, kShort = 1, kBadMagic = 2, kBadNatoms = 3, kBadHeader = 4, kCorrupt = 5;

__host__ __device__ inline uint32_t be32w(uint32_t w) { return __builtin_bswap32(w); }

// ---- bit windows ------------------------------------------------------------
// A window yields the 64 stream bits at its read position, MSB first
// (peek64), and advances (skip).  Words past the stream read as 0;
// consumed() > 8*nbytes flags an overrun, checked once per atom.  Both reads
// are branch-free: of the 96 bits w0:w1:w2 around the position, bits
// [sh, sh+64) are (w0:w1 << sh) | ((w1:w2 << sh) >> 32).
__host__ __device__ inline uint64_t bits64(uint32_t w0, uint32_t w1, uint32_t w2, int sh) {
  const uint64_t hi = (uint64_t)w0 << 32 | w1, lo = (uint64_t)w1 << 32 | w2;
  return (hi << sh) | ((lo << sh) >> 32);
}

// host: straight from memory
struct MemWindow {
  const uint32_t *s;
  int64_t nw, pos;
  __host__ __device__ inline void start(const uint32_t *p, int64_t n_words) {
    s = p;
    nw = n_words;
    pos = 0;
  }
  __host__ __device__ inline uint32_t at(int64_t j) const { return j < nw ? be32w(s[j]) : 0u; }
  __host__ __device__ inline uint64_t peek64() const {
    const int64_t i = pos >> 5;
    return bits64(at(i), at(i + 1), at(i + 2), (int)(pos & 31));
  }
  __host__ __device__ inline void skip(int k) { pos += k; }
  __host__ __device__ inline void advance(int64_t k) { pos += k; }
  __host__ __device__ inline void skip64(int64_t k) { pos += k; }
  __host__ __device__ inline int64_t consumed() const { return pos; }
  __host__ __device__ static inline int uni(int v) { return v; }
  __host__ __device__ inline void uniformize() {}
};

template <class W>
__host__ __device__ inline uint64_t take(W &w, int k) {  // 1 <= k <= 64
  const uint64_t v = w.peek64() >> (64 - k);
  w.skip(k);
  return v;
}

// receiveints' byte order: the packed value's bytes arrive least significant
// first (8 bits each), the last (1..8 bits) carrying the top.  One read of
// all nbits (<= 64), then the q full bytes are reversed.
__host__ __device__ inline uint64_t unpack(uint64_t x, int nbits) {  // x: the nbits as read, MSB first
  const int q = (nbits - 1) >> 3, r = nbits - 8 * q;  // q full bytes, r (1..8) top bits
  const uint64_t top = x & ((1ull << r) - 1ull);
  const uint64_t low = (__builtin_bswap64(x >> r) >> (63 - 8 * q)) >> 1;
  return (top << (8 * q)) | low;
}

// value = (n0*s1 + n1)*s2 + n2, value < 2^52: exact double arithmetic, the
// quotient estimate corrected by at most one, without branches.
__host__ __device__ inline void split_f64(uint64_t v, const unsigned s[3], const double inv[3], int out[3]) {
  double d = (double)v;
  for (int i = 2; i >= 1; --i) {
    const double si = (double)s[i];
    double q = floor(d * inv[i]);
    double r = fma(-q, si, d);  // exact: |r| < 2 s
    const double adj = (r >= si ? 1.0 : 0.0) - (r < 0.0 ? 1.0 : 0.0);
    q += adj;
    r = fma(-adj, si, r);
    out[i] = (int)r;
    d = q;
  }
  out[0] = (int)fmin(d, 2147483647.0);  // < s0 <= 2^24 for a valid stream
}

// the published byte-wise long division, for packed values wider than 52 bits
template <class W>
__host__ __device__ inline bool split_bytes(W &w, int nbits, const unsigned s[3], int out[3]) {
  if (nbits > 96 || s[1] == 0 || s[2] == 0 || s[1] > (1u << 24) || s[2] > (1u << 24)) return false;
  unsigned bytes[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int nb = 0;
  while (nbits > 8) {
    bytes[nb++] = (unsigned)take(w, 8);
    nbits -= 8;
  }
  if (nbits > 0) bytes[nb++] = (unsigned)take(w, nbits);
  for (int i = 2; i > 0; --i) {
    unsigned num = 0;
    for (int j = nb - 1; j >= 0; --j) {
      num = (num << 8) | bytes[j];
      const unsigned p = num / s[i];
      bytes[j] = p;
      num -= p * s[i];
    }
    out[i] = (int)num;
  }
  out[0] = (int)(bytes[0] | bytes[1] << 8 | bytes[2] << 16 | bytes[3] << 24);
  return true;
}

__host__ __device__ inline int sizeofint_hd(unsigned size) {
  unsigned num = 1;
  int nbits = 0;
  while (size >= num && nbits < 32) {
    nbits++;
    num <<= 1;
  }
  return nbits;
}

__host__ __device__ inline int sizeofints_hd(const unsigned sizes[3]) {
  unsigned bytes[32];
  int nb = 1, nbits = 0;
  bytes[0] = 1;
  for (int i = 0; i < 3; ++i) {
    unsigned tmp = 0;
    int bc;
    for (bc = 0; bc < nb; ++bc) {
      tmp = bytes[bc] * sizes[i] + tmp;
      bytes[bc] = tmp & 0xff;
      tmp >>= 8;
    }
    while (tmp != 0 && bc < 32) {
      bytes[bc++] = tmp & 0xff;
      tmp >>= 8;
    }
    nb = bc;
  }
  unsigned num = 1;
  nb--;
  while (bytes[nb] >= num && nbits < 32) {
    nbits++;
    num *= 2;
  }
  return nbits + nb * 8;
}

__host__ __device__ inline float f32_bits(uint32_t u) { return __builtin_bit_cast(float, u); }

// xdrfile scales to nm in f32; MDAnalysis then multiplies by 10 in f32
__host__ __device__ inline void to_angstrom(int c0, int c1, int c2, float invp, float &a, float &b, float &c) {
#pragma clang fp contract(off)
  const float x = (float)c0 * invp, y = (float)c1 * invp, z = (float)c2 * invp;
  a = x * 10.0f;
  b = y * 10.0f;
  c = z * 10.0f;
}

// ---- two-pass frame decode ---------------------------------------------------
// The stream is a sequence of groups: one "large" atom (an absolute packed
// triple) followed by the run of small triples its flag announced (run/3
// atoms, each relative to the previous one).  Only the bit offsets are
// sequential: a group's length is fixed by the header (large triple), its
// flag/run code and the current small-integer index.  Pass 1 walks the
// stream reading nothing but the 1-6 flag bits per group and records each
// group's (bit offset, atom index, small index, run); pass 2 decodes the
// recorded groups independently -- on the device one group per lane, 64 at a
// time -- reading the triples straight from memory.  Groups are independent
// because smallnum == magicints[smallidx]/2 in every state a run can use and a
// large atom resets `prev`.  Corruption is detected in pass 1, in the order
// of the sequential algorithm, so the status is identical.
struct XtcFrame {
  const uint32_t *s;  // compressed stream (big-endian words)
  int64_t nw, nbits;
  int natoms, bitsize, large_bits, smallidx0;
  unsigned bitsizeint[3], sizeint[3];
  double invint[3];
  int minint[3];
  float inv_precision;
};

struct XtcGroup {
  int64_t pos;   // bit offset of the large triple
  int32_t idx;   // index of the group's first output atom
  uint32_t meta; // small-integer index (bits per small triple) | run/3 << 8 | flag bits (1 or 6) << 16
  __host__ __device__ inline int sidx() const { return (int)(meta & 0xff); }
  __host__ __device__ inline int nsmall() const { return (int)((meta >> 8) & 0xff); }
  __host__ __device__ inline int fbits() const { return (int)(meta >> 16); }
};

__host__ __device__ inline uint32_t stream_word(const uint32_t *s, int64_t nw, int64_t j) {
  return j < nw ? be32w(s[j]) : 0u;
}

__host__ __device__ inline bool split_bytes_ok(int nbits, const unsigned s[3]) {
  return !(nbits > 96 || s[1] == 0 || s[2] == 0 || s[1] > (1u << 24) || s[2] > (1u << 24));
}

// stream words for pass 2: straight from memory (host) ...
struct MemSrc {
  const uint32_t *s;
  int64_t nw;
  __host__ __device__ inline uint32_t at(int64_t j) const { return stream_word(s, nw, j); }
};

// ... or from the wave's LDS ring (device): kRing words of the stream up
// to the fill point, byte-swapped, zero past the stream
constexpr int kRing = 4096;
struct LdsSrc {
  const uint32_t *ring;
  __device__ inline uint32_t at(int64_t j) const { return ring[j & (kRing - 1)]; }
};

template <class Src>
__host__ __device__ inline void triple_at(const XtcFrame &F, const Src &src, int64_t pos, int nbits,
                                          const unsigned s[3], const double inv[3], int out[3]) {
  if (nbits <= 52) {
    const int64_t i = pos >> 5;
    const uint64_t v = bits64(src.at(i), src.at(i + 1), src.at(i + 2), (int)(pos & 31)) >> (64 - nbits);
    split_f64(unpack(v, nbits), s, inv, out);
  } else {
    MemWindow w;
    w.start(F.s, F.nw);
    w.skip64(pos);
    (void)split_bytes(w, nbits, s, out);  // the widths were validated (header / pass 1)
  }
}

__host__ __device__ inline void put_atom(float *o, int64_t idx, int c0, int c1, int c2, float invp) {
  float a, b, c;
  to_angstrom(c0, c1, c2, invp, a, b, c);
  o[3 * idx] = a;
  o[3 * idx + 1] = b;
  o[3 * idx + 2] = c;
}

// pass 2: one group
template <class Src>
__host__ __device__ inline void decode_group(const XtcFrame &F, const XtcGroup &g, const int *magic,
                                             const double *inv_magic, float *o, const Src &src) {
  int cur[3];
  if (F.bitsize == 0) {
    int64_t p = g.pos;
    for (int c = 0; c < 3; ++c) {
      const int64_t i = p >> 5;
      cur[c] = (int)(bits64(src.at(i), src.at(i + 1), src.at(i + 2), (int)(p & 31)) >> (64 - F.bitsizeint[c]));
      p += F.bitsizeint[c];
    }
  } else {
    triple_at(F, src, g.pos, F.bitsize, F.sizeint, F.invint, cur);
  }
  for (int c = 0; c < 3; ++c) cur[c] += F.minint[c];
  const int nsmall = g.nsmall(), sidx = g.sidx();
  if (nsmall == 0) {
    put_atom(o, g.idx, cur[0], cur[1], cur[2], F.inv_precision);
    return;
  }
  const unsigned m = (unsigned)magic[sidx];
  const unsigned ss[3] = {m, m, m};
  const double iv = inv_magic[sidx];
  const double is[3] = {iv, iv, iv};
  const int smallnum = magic[sidx] / 2;
  int prev[3] = {cur[0], cur[1], cur[2]};
  int64_t p = g.pos + F.large_bits + g.fbits();
  for (int k = 0; k < nsmall; ++k) {
    int t[3];
    triple_at(F, src, p, sidx, ss, is, t);
    p += sidx;
    for (int c = 0; c < 3; ++c) t[c] += prev[c] - smallnum;
    if (k == 0) {  // the writer swapped the first two atoms (water)
      put_atom(o, g.idx, t[0], t[1], t[2], F.inv_precision);
      put_atom(o, g.idx + 1, prev[0], prev[1], prev[2], F.inv_precision);
    } else {
      put_atom(o, g.idx + 1 + k, t[0], t[1], t[2], F.inv_precision);
    }
    prev[0] = t[0];
    prev[1] = t[1];
    prev[2] = t[2];
  }
}

// Frame header of one XTC record (starting at its magic word, `words`
// long): the raw form (<= 9 atoms) is decoded here (*raw = true); otherwise
// F describes the compressed stream.  Mirrors decode_coords() of xtc.cpp.
__host__ __device__ inline int32_t parse_header(const uint32_t *rec, int64_t words, int64_t n_atoms, float *o,
                                                XtcFrame &F, bool *raw) {
#pragma clang fp contract(off)
  *raw = false;
  if (words < 14) return kShort;
  if ((int)be32w(rec[0]) != kMagic) return kBadMagic;
  const int natoms = (int)be32w(rec[1]);
  if (natoms != n_atoms || (int)be32w(rec[13]) != natoms) return kBadNatoms;
  const uint32_t *p = rec + 14;  // magic natoms step time box[9] lsize
  int64_t left = words - 14;
  if (natoms <= 9) {
    if (left < 3 * natoms) return kShort;
    for (int a = 0; a < natoms; ++a)  // raw floats (nm) x 10, as MDAnalysis
      for (int c = 0; c < 3; ++c) o[3 * a + c] = f32_bits(be32w(p[3 * a + c])) * 10.0f;
    *raw = true;
    return kOk;
  }
  if (left < 9) return kShort;
  F.natoms = natoms;
  const float precision = f32_bits(be32w(p[0]));
  int maxint[3];
  for (int c = 0; c < 3; ++c) {
    F.minint[c] = (int)be32w(p[1 + c]);
    maxint[c] = (int)be32w(p[4 + c]);
  }
  const int smallidx = (int)be32w(p[7]);
  const int nbytes = (int)be32w(p[8]);
  p += 9;
  left -= 9;
  if (smallidx < kFirstIdx || smallidx >= kLastIdx || nbytes < 0 || ((int64_t)nbytes + 3) / 4 > left)
    return kBadHeader;
  for (int c = 0; c < 3; ++c) {
    F.sizeint[c] = (unsigned)(maxint[c] - F.minint[c]) + 1u;
    if (F.sizeint[c] == 0) return kBadHeader;  // a wrapped range
    F.invint[c] = 1.0 / (double)F.sizeint[c];
    F.bitsizeint[c] = 0;
  }
  F.bitsize = 0;
  if ((F.sizeint[0] | F.sizeint[1] | F.sizeint[2]) > 0xffffff) {
    for (int c = 0; c < 3; ++c) F.bitsizeint[c] = sizeofint_hd(F.sizeint[c]);
    F.large_bits = (int)(F.bitsizeint[0] + F.bitsizeint[1] + F.bitsizeint[2]);
  } else {
    F.bitsize = sizeofints_hd(F.sizeint);
    F.large_bits = F.bitsize;
    // the sequential decoder fails on its first large triple
    if (F.bitsize > 52 && !split_bytes_ok(F.bitsize, F.sizeint)) return kCorrupt;
  }
  F.inv_precision = (float)(1.0 / (double)precision);
  F.s = p;
  F.nw = ((int64_t)nbytes + 3) / 4;
  F.nbits = 8 * (int64_t)nbytes;
  F.smallidx0 = smallidx;
  return kOk;
}

// one step of pass 1, shared by host and device: from the group's flag
// peek (p6 = the 6 bits after its large triple) to its record.  Returns
// false on a corrupt stream (the sequential algorithm's checks, in order).
__host__ __device__ inline bool group_step(const XtcFrame &F, const int *magic, uint32_t p6, int &i, int &run,
                                           int &sidx, int &adv, uint32_t &meta) {
  const bool flag = (p6 >> 5) != 0;
  const int rc = (int)(p6 & 31), rm = rc % 3;
  run = flag ? rc - rm : run;
  const int is_smaller = flag ? rm - 1 : 0;
  ++i;
  int nsmall = 0;
  adv = flag ? 6 : 1;
  if (run > 0) {
    nsmall = run / 3;
    if (i + nsmall > F.natoms || magic[sidx] == 0) return false;
    adv += nsmall * sidx;
    i += nsmall;
  }
  meta = (uint32_t)sidx | (uint32_t)nsmall << 8 | (flag ? 6u : 1u) << 16;
  sidx += is_smaller;
  return !(sidx < kFirstIdx - 1 || sidx >= kLastIdx);
}

// host: pass 1 and pass 2 interleaved group by group
inline int32_t scan_host(const XtcFrame &F, const int *magic, const double *inv, float *o) {
  const MemSrc src{F.s, F.nw};
  MemWindow b;
  b.start(F.s, F.nw);
  int i = 0, run = 0, sidx = F.smallidx0;
  while (i < F.natoms) {
    XtcGroup g;
    g.pos = b.consumed();
    g.idx = i;
    b.advance(F.large_bits);
    const uint32_t p6 = (uint32_t)(b.peek64() >> 58);
    int adv;
    if (!group_step(F, magic, p6, i, run, sidx, adv, g.meta)) return kCorrupt;
    b.advance(adv);
    if (b.consumed() > F.nbits) return kCorrupt;
    decode_group(F, g, magic, inv, o, src);
  }
  return kOk;
}

// v_writelane_b32 (the LLVM intrinsic; this clang has no builtin for it):
// lane `lane` of `old` := the uniform `value`
extern "C" __device__ int llvm_amdgcn_writelane(int value, int lane, int old) __asm("llvm.amdgcn.writelane");
__device__ inline uint32_t writelane(uint32_t old, uint32_t value, int lane) {
  return (uint32_t)llvm_amdgcn_writelane((int)value, lane, (int)old);
}
__device__ inline int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Stream words for the device passes come from an LDS ring filled in stages
// of 512 words (8 per lane), one stage in flight ahead of the fill point.
// (Loads hidden from the compiler with inline asm were measured wrong: its
// register allocator copies the destination registers before the data
// lands.)
__device__ inline uint32_t ld_word(const uint32_t *s, int64_t nw, int64_t j) { return j < nw ? s[j] : 0u; }

constexpr int kStage = 512;
struct RingFill {
  const uint32_t *s;
  int64_t nw;
  uint32_t *ring;
  int lane;
  int64_t hi;       // the ring holds stream words [hi - kRing, hi)
  uint32_t st[8];   // in flight: words hi + 64 v + lane
  __device__ inline void issue() {
#pragma unroll
    for (int v = 0; v < 8; ++v) st[v] = ld_word(s, nw, hi + 64 * v + lane);
  }
  __device__ inline void advance() {
#pragma unroll
    for (int v = 0; v < 8; ++v) ring[(hi + 64 * v + lane) & (kRing - 1)] = be32w(st[v]);
    hi += kStage;
    issue();
  }
  __device__ inline void ensure(int64_t word) {  // word < hi afterwards (uniform)
    while (word >= hi) advance();
  }
};

// device: one wave per frame.  Pass 1 (wave-uniform, SGPR state) alternates
// two steps.  (a) A lane-parallel scan: while the flag bit is 0 a group's
// length is constant (D = large bits + 1 + run/3 * smallidx), so lane m tests
// the flag bit of group m at pos + m*D + large bits, and a ballot gives the
// count K of clean groups ahead (flag 0, inside the stream, the atom count
// and the ring); their records are written lane-parallel.  (b) For the
// group the scan stopped at (a set flag, the frame's end, or a corrupt
// stream) the sequential step: a 6-bit peek and group_step(), exactly as on
// the host.  Group k of a batch of 64 lives in lane k; a full batch is
// decoded lane-parallel (pass 2) from the LDS ring.
__device__ int32_t scan_wave(const XtcFrame &F, const int *magic, const double *inv, float *o,
                             uint32_t *ring) {
  const int lane = (int)(threadIdx.x & 63);
  RingFill rf{F.s, F.nw, ring, lane, 0, {}};
  rf.issue();
  rf.advance();  // words [0, 512) in the ring, [512, 1024) in flight
  const LdsSrc src{ring};
  uint32_t r_lo = 0, r_hi = 0, r_idx = 0, r_meta = 0;
  auto flush = [&](int n) {
    if (lane < n) {
      XtcGroup g;
      g.pos = (int64_t)((uint64_t)r_hi << 32 | r_lo);
      g.idx = (int32_t)r_idx;
      g.meta = r_meta;
      decode_group(F, g, magic, inv, o, src);
    }
  };
  auto rd = [&](int64_t j) { return (uint32_t)uni((int)ring[j & (kRing - 1)]); };
  int64_t pos = 0;
  int i = 0, run = 0, sidx = F.smallidx0, n = 0;
  const int natoms = F.natoms, lb = F.large_bits;
  const int64_t nbits = F.nbits;
  int32_t st = kOk;
  while (i < natoms) {
    i = uni(i);
    run = uni(run);
    sidx = uni(sidx);
    n = uni(n);
    // (a) scan of clean (flag 0) groups; run is 0 or a multiple of 3
    const int ns = (int)(((uint32_t)run * 0x56u) >> 8);
    const int D = lb + 1 + ns * sidx;
    int K = 0;
    if (!(ns > 0 && sidx <= kFirstIdx - 1)) {  // magicints[8] == 0: a run there is corrupt
      rf.ensure((pos >> 5) + 192);
      const int64_t P = pos + (int64_t)lane * D + lb;                // flag bit of group `lane`
      const int64_t endb = P + 1 + (int64_t)ns * sidx;                // end of its small triples
      const int64_t im = (int64_t)i + (int64_t)lane * (1 + ns);      // its first atom
      bool stop = im + 1 + ns > natoms || endb > nbits || ((endb + 95) >> 5) >= rf.hi;
      if (!stop) stop = ((ring[(P >> 5) & (kRing - 1)] >> (31 - (int)(P & 31))) & 1u) != 0;
      const uint64_t m = __ballot(stop);
      K = uni(m ? (int)__builtin_ctzll(m) : 64);
    }
    if (K > 0) {
      const uint32_t meta0 = (uint32_t)sidx | (uint32_t)ns << 8 | 1u << 16;
      for (int done = 0; done < K;) {
        const int take = min(K - done, 64 - n);
        if (lane >= n && lane < n + take) {
          const int mm = done + (lane - n);
          const int64_t gp = pos + (int64_t)mm * D;
          r_lo = (uint32_t)gp;
          r_hi = (uint32_t)((uint64_t)gp >> 32);
          r_idx = (uint32_t)(i + mm * (1 + ns));
          r_meta = meta0;
        }
        n += take;
        done += take;
        if (n == 64) {
          flush(64);
          n = 0;
        }
      }
      pos += (int64_t)K * D;
      i += K * (1 + ns);
      continue;
    }
    // (b) sequential step for the group at pos
    const int64_t q = pos + lb;
    rf.ensure(((q + 6 + 720 + 95) >> 5) + 1);  // flag bits and up to 10 small triples of <= 72 bits
    const uint32_t p6 = (uint32_t)((((uint64_t)rd(q >> 5) << 32 | rd((q >> 5) + 1)) << (q & 31)) >> 58);
    int adv;
    uint32_t meta;
    const int idx = i;
    if (!group_step(F, magic, p6, i, run, sidx, adv, meta)) {
      st = kCorrupt;
      break;
    }
    const int64_t gpos = pos;
    pos = q + adv;
    if (pos > nbits) {
      st = kCorrupt;
      break;
    }
    r_lo = writelane(r_lo, (uint32_t)uni((int)(uint32_t)gpos), n);
    r_hi = writelane(r_hi, (uint32_t)uni((int)(uint32_t)((uint64_t)gpos >> 32)), n);
    r_idx = writelane(r_idx, (uint32_t)uni(idx), n);
    r_meta = writelane(r_meta, (uint32_t)uni((int)meta), n);
    if (++n == 64) {
      flush(64);
      n = 0;
    }
  }
  if (st == kOk) flush(n);
  return st;
}

// One wave per frame (grid = n_frames blocks of 64).
__global__ __launch_bounds__(64) void k_xtc_decode(const uint32_t *__restrict__ words,
                                                   const int64_t *__restrict__ rec_off,
                                                   const int64_t *__restrict__ rec_len, int64_t n_atoms,
                                                   float *__restrict__ out, int64_t out_stride,
                                                   int32_t *__restrict__ status) {
  __shared__ uint32_t ring[kRing];
  const int64_t f = blockIdx.x;
  float *o = out + f * out_stride;
  XtcFrame F;
  bool raw;
  int32_t st = parse_header(words + rec_off[f], rec_len[f], n_atoms, o, F, &raw);
  if (st == kOk && !raw) st = scan_wave(F, g_magic.v, g_inv.v, o, ring);
  if (st != kOk) {
    for (int64_t k = threadIdx.x; k < 3 * n_atoms; k += 64) o[k] = __builtin_nanf("");
  }
  if (threadIdx.x == 0) status[f] = st;
}

const char *status_text(int32_t s) {
  switch (s) {
    case kShort: return "truncated frame record";
    case kBadMagic: return "bad magic number";
    case kBadNatoms: return "atom count differs from the file's";
    case kBadHeader: return "bad compression header";
    case kCorrupt: return "corrupt compressed coordinates";
    default: return "unknown error";
  }
}

constexpr size_t kReadSub = 4u << 20;     // bytes per pread task (read contiguous batches)
constexpr size_t kCopyMin = 64u << 20;    // host->device copies of at least this many bytes

// Persistent worker threads for the file reads (spawning threads per read
// cost ~0.2 ms each).  launch(n, fn) hands fn(0..n-1) to the workers (in
// increasing k) and returns; wait() returns when all are done; run() = both.
class ReadPool {
 public:
  // cpus != nullptr: every worker runs on those CPUs (rmsf_host::device_cpus)
  explicit ReadPool(int n, const cpu_set_t *cpus = nullptr) {
    for (int i = 0; i < n; ++i) {
      if (cpus) {
        const cpu_set_t c = *cpus;
        th_.emplace_back([this, c] {
          rmsf_host::pin_self(c);
          loop();
        });
      } else {
        th_.emplace_back([this] { loop(); });
      }
    }
  }
  ~ReadPool() {
    wait();
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  void launch(int64_t n, std::function<void(int64_t)> fn) {
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return left_ == 0; });
    fn_ = std::move(fn);
    next_ = 0;
    total_ = n;
    left_ = n;
    ++gen_;
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return left_ == 0; });
  }
  void run(int64_t n, std::function<void(int64_t)> fn) {
    launch(n, std::move(fn));
    wait();
  }

 private:
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [&] { return stop_ || (gen_ != seen && next_ < total_); });
      if (stop_) return;
      while (next_ < total_) {
        const int64_t i = next_++;
        const std::function<void(int64_t)> *fn = &fn_;  // not replaced before left_ reaches 0
        g.unlock();
        (*fn)(i);
        g.lock();
        if (--left_ == 0) done_.notify_all();
      }
      seen = gen_;
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  std::function<void(int64_t)> fn_;
  int64_t next_ = 0, total_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Waits for a launched pool on every exit path of the scope (its tasks
// reference the caller's locals).
struct PoolWait {
  ReadPool &p;
  ~PoolWait() { p.wait(); }
};

}  // namespace

struct rmsf_xtcdec {
  const rmsf_xtc *x = nullptr;
  int64_t batch = 0, n_atoms = 0;
  int n_threads = 1;
  std::unique_ptr<ReadPool> pool;
  struct Slot {
    unsigned char *h_raw = nullptr;
    int64_t *h_tab = nullptr;  // [2][batch]: record offset (words), record length (words)
    int32_t *h_status = nullptr;
    unsigned char *d_raw = nullptr;
    int64_t *d_tab = nullptr;
    int32_t *d_status = nullptr;
    float *d_frames = nullptr;
    size_t raw_cap = 0;
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr, released = nullptr;
    int64_t pending = 0;  // frames whose status is not yet checked
    int64_t f0 = 0, step = 1;
    std::vector<int64_t> list;  // the frames of a list decode (else f0 + k*step)
  };
  std::vector<Slot> slots;
  int next = 0;
};

namespace {

int check_slot(rmsf_xtcdec *d, rmsf_xtcdec::Slot &s) {
  if (s.pending == 0) return RMSF_OK;
  XD_HIP(hipEventSynchronize(s.done));
  const int64_t n = s.pending;
  s.pending = 0;
  for (int64_t k = 0; k < n; ++k)
    if (s.h_status[k] != kOk)
      return fail(RMSF_EINVAL, "xtc (GPU decode): frame " +
                                   std::to_string(s.list.empty() ? s.f0 + k * s.step : s.list[k]) + ": " +
                                   status_text(s.h_status[k]));
  return RMSF_OK;
}

void free_slot(rmsf_xtcdec::Slot &s) {
  if (s.s) (void)hipStreamSynchronize(s.s);
  if (s.h_raw) (void)hipHostFree(s.h_raw);
  if (s.h_tab) (void)hipHostFree(s.h_tab);
  if (s.h_status) (void)hipHostFree(s.h_status);
  if (s.d_raw) (void)hipFree(s.d_raw);
  if (s.d_tab) (void)hipFree(s.d_tab);
  if (s.d_status) (void)hipFree(s.d_status);
  if (s.d_frames) (void)hipFree(s.d_frames);
  if (s.done) (void)hipEventDestroy(s.done);
  if (s.released) (void)hipEventDestroy(s.released);
  if (s.s) (void)hipStreamDestroy(s.s);
  s = rmsf_xtcdec::Slot{};
}

}  // namespace

extern "C" {

RMSF_EXPORT int rmsf_xtc_decode_records(const void *d_records, const int64_t *d_rec_off, const int64_t *d_rec_len,
                                        int64_t n_frames, int64_t n_atoms, float *d_out, int64_t out_stride,
                                        int32_t *d_status, void *stream) {
  if (!d_records || !d_rec_off || !d_rec_len || !d_out || !d_status || n_frames < 0 || n_atoms < 1 ||
      out_stride < 3 * n_atoms ||
      (reinterpret_cast<uintptr_t>(d_records) & 3))
    return fail(RMSF_EINVAL, "rmsf_xtc_decode_records: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  if (n_frames > 0x7fffffffLL) return fail(RMSF_EINVAL, "rmsf_xtc_decode_records: too many frames");
  hipLaunchKernelGGL(k_xtc_decode, dim3((unsigned)n_frames), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const uint32_t *>(d_records), d_rec_off, d_rec_len, n_atoms, d_out, out_stride,
                     d_status);
  XD_HIP(hipGetLastError());
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_xtc_decode_records_host(const void *h_records, const int64_t *h_rec_off,
                                             const int64_t *h_rec_len, int64_t n_frames, int64_t n_atoms,
                                             float *h_out, int64_t out_stride, int32_t *h_status) {
  if (!h_records || !h_rec_off || !h_rec_len || !h_out || !h_status || n_frames < 0 || n_atoms < 1 ||
      out_stride < 3 * n_atoms || (reinterpret_cast<uintptr_t>(h_records) & 3))
    return fail(RMSF_EINVAL, "rmsf_xtc_decode_records_host: bad arguments");
  const uint32_t *w = static_cast<const uint32_t *>(h_records);
  for (int64_t f = 0; f < n_frames; ++f) {
    float *o = h_out + f * out_stride;
    XtcFrame F;
    bool raw;
    int32_t st = parse_header(w + h_rec_off[f], h_rec_len[f], n_atoms, o, F, &raw);
    if (st == kOk && !raw) st = scan_host(F, h_magic.v, h_inv.v, o);
    h_status[f] = st;
  }
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_xtcdec_create(const rmsf_xtc *x, int64_t batch_frames, int n_slots, int n_threads,
                                   rmsf_xtcdec **out) {
  if (!x || !out || batch_frames < 1 || n_slots < 1 || n_slots > 16 || n_threads < 1)
    return fail(RMSF_EINVAL, "rmsf_xtcdec_create: bad arguments");
  *out = nullptr;
  auto *d = new rmsf_xtcdec();
  d->x = x;
  d->batch = batch_frames;
  d->n_atoms = x->n_atoms;
  d->n_threads = n_threads;
  // read threads on the GPU's NUMA node when it is known
  int dev = 0;
  cpu_set_t near;
  const bool pin = hipGetDevice(&dev) == hipSuccess && rmsf_host::device_cpus(dev, &near);
  d->pool = std::make_unique<ReadPool>(n_threads, pin ? &near : nullptr);
  d->slots.resize(n_slots);
  const size_t raw = (size_t)batch_frames * (size_t)x->max_size;
  for (auto &s : d->slots) {
    s.raw_cap = raw;
    hipError_t e = hipHostMalloc((void **)&s.h_raw, raw, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void **)&s.h_tab, 2 * batch_frames * sizeof(int64_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void **)&s.h_status, batch_frames * sizeof(int32_t), hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void **)&s.d_raw, raw);
    if (e == hipSuccess) e = hipMalloc((void **)&s.d_tab, 2 * batch_frames * sizeof(int64_t));
    if (e == hipSuccess) e = hipMalloc((void **)&s.d_status, batch_frames * sizeof(int32_t));
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.released, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(s.released, s.s);  // initially free
    if (e == hipSuccess) e = hipEventRecord(s.done, s.s);
    if (e != hipSuccess) {
      for (auto &t : d->slots) free_slot(t);
      delete d;
      return fail(RMSF_ENOMEM, std::string("rmsf_xtcdec_create: ") + hipGetErrorString(e));
    }
  }
  *out = d;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_xtcdec_destroy(rmsf_xtcdec *d) {
  if (d) {
    for (auto &s : d->slots) free_slot(s);
    delete d;
  }
  return RMSF_OK;
}

}  // extern "C"

namespace {

// out == nullptr: into the slot's own frame buffer (allocated on first use),
// reused once the consumer released the slot; otherwise into the caller's
// buffer, frame k at out + k*out_stride.
// list != nullptr: the frames list[0..n) in that order (f0/step unused).
int xtcdec_decode(rmsf_xtcdec *d, int64_t f0, int64_t n, int64_t step, float *out, int64_t out_stride,
                  void *consumer_stream, int *slot, float **d_frames, const int64_t *list = nullptr) {
  const int si = d->next;
  d->next = (d->next + 1) % (int)d->slots.size();
  auto &s = d->slots[si];
  int rc = check_slot(d, s);  // the pinned buffers are rewritten below: the previous use must be over
  if (rc) return rc;
  XD_HIP(hipEventSynchronize(s.done));
  const rmsf_xtc *x = d->x;
  int64_t *off = s.h_tab, *len = s.h_tab + d->batch;
  size_t total = 0;
  bool copied = false;
  auto frame = [&](int64_t k) { return list ? list[k] : f0 + k * step; };
  if (!list && step == 1) {
    const int64_t a = x->offset[f0], e = x->offset[f0 + n - 1] + x->size[f0 + n - 1];
    total = (size_t)(e - a);
    if (total > s.raw_cap) return fail(RMSF_EINVAL, "rmsf_xtcdec_decode: batch larger than the slot");
    // read in 4 MiB tasks over the pool with no barrier between them; this
    // thread copies every completed prefix of >= 64 MiB to the device as it
    // forms, so the DMA overlaps the rest of the read
    const int64_t pieces = (int64_t)((total + kReadSub - 1) / kReadSub);
    std::unique_ptr<std::atomic<char>[]> st(new std::atomic<char>[pieces]);  // 0 pending, 1 read, 2 failed
    for (int64_t k = 0; k < pieces; ++k) st[k].store(0);
    std::mutex mu;
    std::condition_variable cv;
    unsigned char *h = s.h_raw;
    const int fd = x->fd;
    d->pool->launch(pieces, [&, h, fd, a, total](int64_t k) {
      const size_t o = (size_t)k * kReadSub, len = std::min(kReadSub, total - o);
      st[k].store(rmsf_internal_pread_all(fd, h + o, len, a + (int64_t)o) ? 1 : 2);
      { std::lock_guard<std::mutex> g(mu); }
      cv.notify_one();
    });
    PoolWait pw{*d->pool};
    size_t sent = 0;
    for (int64_t next = 0; next < pieces;) {
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return st[next].load() != 0; });
      }
      for (; next < pieces && st[next].load() != 0; ++next)
        if (st[next].load() == 2) return fail(RMSF_EINVAL, "xtc: read failed");
      const size_t ready = std::min(total, (size_t)next * kReadSub);
      if (ready - sent >= kCopyMin || ready == total) {
        XD_HIP(hipMemcpyAsync(s.d_raw + sent, s.h_raw + sent, ready - sent, hipMemcpyHostToDevice, s.s));
        sent = ready;
      }
    }
    copied = true;
    for (int64_t k = 0; k < n; ++k) {
      off[k] = (x->offset[f0 + k] - a) / 4;
      len[k] = x->size[f0 + k] / 4;
    }
  } else {
    for (int64_t k = 0; k < n; ++k) {
      const int64_t f = frame(k);
      off[k] = (int64_t)(total / 4);
      len[k] = x->size[f] / 4;
      total += (size_t)x->size[f];
    }
    if (total > s.raw_cap) return fail(RMSF_EINVAL, "rmsf_xtcdec_decode: batch larger than the slot");
    std::vector<char> ok(n, 1);
    d->pool->run(n, [&](int64_t k) {
      const int64_t f = frame(k);
      ok[k] = rmsf_internal_pread_all(x->fd, s.h_raw + 4 * off[k], (size_t)x->size[f], x->offset[f]);
    });
    for (char c : ok)
      if (!c) return fail(RMSF_EINVAL, "xtc: read failed");
  }
  if (!copied) XD_HIP(hipMemcpyAsync(s.d_raw, s.h_raw, total, hipMemcpyHostToDevice, s.s));
  XD_HIP(hipMemcpyAsync(s.d_tab, s.h_tab, 2 * d->batch * sizeof(int64_t), hipMemcpyHostToDevice, s.s));
  if (!out) {
    if (!s.d_frames) {
      const size_t bytes = (size_t)d->batch * 3 * (size_t)d->n_atoms * sizeof(float);
      hipError_t e = hipMalloc((void **)&s.d_frames, bytes);
      if (e != hipSuccess) return fail(RMSF_ENOMEM, std::string("rmsf_xtcdec_decode: ") + hipGetErrorString(e));
    }
    XD_HIP(hipStreamWaitEvent(s.s, s.released, 0));  // the consumer is done with the previous frames
    out = s.d_frames;
    out_stride = 3 * d->n_atoms;
  }
  rc = rmsf_xtc_decode_records(s.d_raw, s.d_tab, s.d_tab + d->batch, n, d->n_atoms, out, out_stride, s.d_status,
                               s.s);
  if (rc) return rc;
  XD_HIP(hipMemcpyAsync(s.h_status, s.d_status, n * sizeof(int32_t), hipMemcpyDeviceToHost, s.s));
  XD_HIP(hipEventRecord(s.done, s.s));
  XD_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(consumer_stream), s.done, 0));
  s.pending = n;
  s.f0 = f0;
  s.step = step;
  if (list) s.list.assign(list, list + n);
  else s.list.clear();
  *slot = si;
  if (d_frames) *d_frames = out;
  return RMSF_OK;
}

}  // namespace

extern "C" {

RMSF_EXPORT int rmsf_xtcdec_decode(rmsf_xtcdec *d, int64_t f0, int64_t n, int64_t step, void *consumer_stream,
                                   int *slot, float **d_frames) {
  if (!d || !slot || !d_frames || n < 1 || n > d->batch || step < 1 || f0 < 0 ||
      f0 + (n - 1) * step >= (int64_t)d->x->offset.size())
    return fail(RMSF_EINVAL, "rmsf_xtcdec_decode: bad arguments");
  return xtcdec_decode(d, f0, n, step, nullptr, 0, consumer_stream, slot, d_frames);
}

RMSF_EXPORT int rmsf_xtcdec_decode_into(rmsf_xtcdec *d, int64_t f0, int64_t n, int64_t step, float *d_out,
                                        int64_t out_stride, void *consumer_stream, int *slot) {
  if (!d || !slot || !d_out || out_stride < 3 * d->n_atoms || n < 1 || n > d->batch || step < 1 || f0 < 0 ||
      f0 + (n - 1) * step >= (int64_t)d->x->offset.size())
    return fail(RMSF_EINVAL, "rmsf_xtcdec_decode_into: bad arguments");
  return xtcdec_decode(d, f0, n, step, d_out, out_stride, consumer_stream, slot, nullptr);
}

RMSF_EXPORT int rmsf_xtcdec_decode_list(rmsf_xtcdec *d, const int64_t *h_frames, int64_t n, void *consumer_stream,
                                        int *slot, float **d_frames) {
  if (!d || !h_frames || !slot || !d_frames || n < 1 || n > d->batch)
    return fail(RMSF_EINVAL, "rmsf_xtcdec_decode_list: bad arguments");
  const int64_t nf = (int64_t)d->x->offset.size();
  for (int64_t k = 0; k < n; ++k)
    if (h_frames[k] < 0 || h_frames[k] >= nf)
      return fail(RMSF_EINVAL, "rmsf_xtcdec_decode_list: frame " + std::to_string(h_frames[k]) + " out of range");
  return xtcdec_decode(d, 0, n, 1, nullptr, 0, consumer_stream, slot, d_frames, h_frames);
}

RMSF_EXPORT int rmsf_xtcdec_release(rmsf_xtcdec *d, int slot, void *consumer_stream) {
  if (!d || slot < 0 || slot >= (int)d->slots.size()) return fail(RMSF_EINVAL, "rmsf_xtcdec_release: bad slot");
  XD_HIP(hipEventRecord(d->slots[slot].released, reinterpret_cast<hipStream_t>(consumer_stream)));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_xtcdec_synchronize(rmsf_xtcdec *d) {
  if (!d) return fail(RMSF_EINVAL, "rmsf_xtcdec_synchronize: null");
  int first = RMSF_OK;
  for (auto &s : d->slots) {
    const int rc = check_slot(d, s);
    if (rc && !first) first = rc;
  }
  return first;
}

}  // extern "C"
