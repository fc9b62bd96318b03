// xtc.cpp -- GROMACS XTC trajectory reader/writer (host C++).
//
// Replaces the libxdrfile decode behind MDAnalysis' XTCReader, i.e. what
// `universe.trajectory[frame]` runs at RMSF.py:92,124 for the reference's
// GRO/XTC input (RMSF.py:34,56); SURVEY.md 8(f) row 2.  The format is the
// published xdrfile one: big-endian XDR records, magic 1995, and the
// xdr3dfcoord integer compression (mixed-radix packed triples, run-length
// coded "small" differences, water-pair swap, adaptive magicints index).
// This is a restatement from the published algorithm: no third-party code is
// vendored, and no reference XTC file exists in this environment, so format
// parity is UNPINNED (tested by write/read round trips and an independent
// Python decoder, oracle/xtc_py.py).
//
// Frames are indexed once (offsets), then decoded frame-parallel by a thread
// pool with pread() -- independent frames, no shared state.  Positions are
// returned in Angstrom with MDAnalysis' rounding: f32(f32(i*f32(1/prec))*10).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rmsf_hip.h"
#include "xtc_internal.h"

#define RMSF_EXPORT __attribute__((visibility("default")))

extern "C" int rmsf_internal_set_error(int code, const char *msg);

namespace {

int fail(int code, const std::string &m) { return rmsf_internal_set_error(code, m.c_str()); }

constexpr int kMagic = 1995;
constexpr int magicints[] = {
    0,       0,       0,       0,       0,       0,       0,       0,        0,        8,        10,
    12,      16,      20,      25,      32,      40,      50,      64,       80,       101,      128,
    161,     203,     256,     322,     406,     512,     645,     812,      1024,     1290,     1625,
    2048,    2580,    3250,    4096,    5060,    6501,    8192,    10321,    13003,    16384,    20642,
    26007,   32768,   41285,   52015,   65536,   82570,   104031,  131072,   165140,   208063,   262144,
    330280,  416127,  524287,  660561,  832255,  1048576, 1321122, 1664510,  2097152,  2642245,  3329021,
    4194304, 5284491, 6658042, 8388607, 10568983, 13316085, 16777216};
constexpr int FIRSTIDX = 9;
constexpr int LASTIDX = sizeof(magicints) / sizeof(magicints[0]);

// ---- XDR primitives (big-endian) -------------------------------------------
inline uint32_t be32(const unsigned char *p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | (uint32_t)p[3];
}
inline int32_t rd_i(const unsigned char *&p) {
  const int32_t v = (int32_t)be32(p);
  p += 4;
  return v;
}
inline float rd_f(const unsigned char *&p) {
  const uint32_t u = be32(p);
  p += 4;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline void wr_u(std::vector<unsigned char> &o, uint32_t v) {
  o.push_back((unsigned char)(v >> 24));
  o.push_back((unsigned char)(v >> 16));
  o.push_back((unsigned char)(v >> 8));
  o.push_back((unsigned char)v);
}
inline void wr_i(std::vector<unsigned char> &o, int32_t v) { wr_u(o, (uint32_t)v); }
inline void wr_f(std::vector<unsigned char> &o, float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  wr_u(o, u);
}

// ---- bit-level codec ---------------------------------------------------------
// MSB-first bit reader with a 64-bit reservoir.  Bit-for-bit the xdrfile
// receivebits / receiveints semantics, but a triple is rebuilt as one integer
// (64-bit, or 128-bit when the packed size exceeds 64 bits) and split with
// two hardware divisions instead of byte-wise long division.  (A double-
// reciprocal quotient estimate measured ~10% slower than 64-bit div here.)
struct BitReader {
  const unsigned char *p, *end;
  uint64_t acc = 0;
  int nacc = 0;
  size_t bits_left;
  BitReader(const unsigned char *b, size_t len) : p(b), end(b + len), bits_left(8 * len) {}
  bool overrun = false;
  inline uint32_t bits(int n) {  // 0 <= n <= 32
    if (n == 0) return 0;
    if ((size_t)n > bits_left) {
      overrun = true;
      bits_left = 0;
      return 0;
    }
    bits_left -= (size_t)n;
    if (nacc < n) {
      while (nacc <= 56) {
        acc = (acc << 8) | (p < end ? *p++ : 0u);
        nacc += 8;
      }
    }
    nacc -= n;
    return (uint32_t)((acc >> nacc) & ((n == 32) ? 0xffffffffull : ((1ull << n) - 1)));
  }
  // receiveints: the value's bytes arrive least significant first, the
  // last (partial) one carrying the top bits; value = (n0*s1 + n1)*s2 + n2
  inline void ints(int nbits, const unsigned sizes[3], int nums[3]) {
    if (nbits <= 64) {
      uint64_t v = 0;
      int sh = 0;
      while (nbits > 8) {
        v |= (uint64_t)bits(8) << sh;
        sh += 8;
        nbits -= 8;
      }
      if (nbits > 0) v |= (uint64_t)bits(nbits) << sh;
      nums[2] = (int)(v % sizes[2]);
      v /= sizes[2];
      nums[1] = (int)(v % sizes[1]);
      v /= sizes[1];
      nums[0] = (int)(uint32_t)v;
    } else {
      unsigned __int128 v = 0;
      int sh = 0;
      while (nbits > 8) {
        v |= (unsigned __int128)bits(8) << sh;
        sh += 8;
        nbits -= 8;
      }
      if (nbits > 0) v |= (unsigned __int128)bits(nbits) << sh;
      nums[2] = (int)(uint32_t)(v % sizes[2]);
      v /= sizes[2];
      nums[1] = (int)(uint32_t)(v % sizes[1]);
      v /= sizes[1];
      nums[0] = (int)(uint32_t)v;
    }
  }
};

struct BitWriter {
  std::vector<unsigned char> out;
  unsigned lastbits = 0, lastbyte = 0;
  void bits(int n, int num) {
    while (n >= 8) {
      lastbyte = (lastbyte << 8) | (unsigned)((num >> (n - 8)) & 0xff);
      out.push_back((unsigned char)(lastbyte >> lastbits));
      n -= 8;
    }
    if (n > 0) {
      lastbyte = (lastbyte << n) | (unsigned)(num & ((1 << n) - 1));
      lastbits += n;
      if (lastbits >= 8) {
        lastbits -= 8;
        out.push_back((unsigned char)(lastbyte >> lastbits));
      }
    }
  }
  void flush() {
    if (lastbits > 0) out.push_back((unsigned char)(lastbyte << (8 - lastbits)));
  }
  bool ints(int nbits, const unsigned sizes[3], const unsigned nums[3]) {
    unsigned bytes[32];
    int nb = 0;
    unsigned tmp = nums[0];
    do {
      bytes[nb++] = tmp & 0xff;
      tmp >>= 8;
    } while (tmp != 0);
    for (int i = 1; i < 3; ++i) {
      if (nums[i] >= sizes[i]) return false;
      tmp = nums[i];
      int bc;
      for (bc = 0; bc < nb; ++bc) {
        tmp = bytes[bc] * sizes[i] + tmp;
        bytes[bc] = tmp & 0xff;
        tmp >>= 8;
      }
      while (tmp != 0) {
        bytes[bc++] = tmp & 0xff;
        tmp >>= 8;
      }
      nb = bc;
    }
    if (nbits >= nb * 8) {
      for (int i = 0; i < nb; ++i) bits(8, (int)bytes[i]);
      bits(nbits - nb * 8, 0);
    } else {
      int i;
      for (i = 0; i < nb - 1; ++i) bits(8, (int)bytes[i]);
      bits(nbits - (nb - 1) * 8, (int)bytes[i]);
    }
    return true;
  }
};

int sizeofint(unsigned size) {
  unsigned num = 1;
  int nbits = 0;
  while (size >= num && nbits < 32) {
    nbits++;
    num <<= 1;
  }
  return nbits;
}

int sizeofints(const unsigned sizes[3]) {
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
    while (tmp != 0) {
      bytes[bc++] = tmp & 0xff;
      tmp >>= 8;
    }
    nb = bc;
  }
  unsigned num = 1;
  nb--;
  while (bytes[nb] >= num) {
    nbits++;
    num *= 2;
  }
  return nbits + nb * 8;
}

// Decode one coordinate block (after the frame header and box) into nm
// floats, MDAnalysis/xdrfile rounding: f32(int) * f32(1/precision).
// Returns bytes consumed or -1.
long decode_coords(const unsigned char *p0, size_t avail, int natoms, float *xyz_nm) {
  const unsigned char *p = p0;
  auto need = [&](size_t n) { return (size_t)(p - p0) + n <= avail; };
  if (!need(4)) return -1;
  const int lsize = rd_i(p);
  if (lsize != natoms) return -1;
  if (natoms <= 9) {
    if (!need(12 * (size_t)natoms)) return -1;
    for (int i = 0; i < 3 * natoms; ++i) xyz_nm[i] = rd_f(p);
    return p - p0;
  }
  if (!need(4 + 24 + 4 + 4)) return -1;
  const float precision = rd_f(p);
  int minint[3], maxint[3];
  for (int i = 0; i < 3; ++i) minint[i] = rd_i(p);
  for (int i = 0; i < 3; ++i) maxint[i] = rd_i(p);
  unsigned sizeint[3], bitsizeint[3] = {0, 0, 0};
  for (int i = 0; i < 3; ++i) sizeint[i] = (unsigned)(maxint[i] - minint[i]) + 1u;
  if (!sizeint[0] || !sizeint[1] || !sizeint[2]) return -1;  // a wrapped range: corrupt header
  int bitsize = 0;
  if ((sizeint[0] | sizeint[1] | sizeint[2]) > 0xffffff) {
    for (int i = 0; i < 3; ++i) bitsizeint[i] = sizeofint(sizeint[i]);
  } else {
    bitsize = sizeofints(sizeint);
  }
  int smallidx = rd_i(p);
  if (smallidx < FIRSTIDX || smallidx >= LASTIDX) return -1;
  int smaller = magicints[std::max(FIRSTIDX, smallidx - 1)] / 2;
  int smallnum = magicints[smallidx] / 2;
  unsigned sizesmall[3];
  sizesmall[0] = sizesmall[1] = sizesmall[2] = magicints[smallidx];
  const int nbytes = rd_i(p);
  if (nbytes < 0 || !need(((size_t)nbytes + 3) & ~(size_t)3)) return -1;
  BitReader br(p, (size_t)nbytes);
  const float inv_precision = (float)(1.0 / precision);
  float *lfp = xyz_nm;
  int prevcoord[3] = {0, 0, 0};
  int run = 0;
  int i = 0;
  int cur[3];
  while (i < lsize) {
    if (bitsize == 0) {
      cur[0] = br.bits(bitsizeint[0]);
      cur[1] = br.bits(bitsizeint[1]);
      cur[2] = br.bits(bitsizeint[2]);
    } else {
      br.ints(bitsize, sizeint, cur);
    }
    i++;
    cur[0] += minint[0];
    cur[1] += minint[1];
    cur[2] += minint[2];
    prevcoord[0] = cur[0];
    prevcoord[1] = cur[1];
    prevcoord[2] = cur[2];
    const int flag = br.bits(1);
    int is_smaller = 0;
    if (flag == 1) {
      run = br.bits(5);
      is_smaller = run % 3;
      run -= is_smaller;
      is_smaller--;
    }
    if (run > 0) {
      if (i + run / 3 > lsize || sizesmall[0] == 0) return -1;  // smallidx below the magicints table
      for (int k = 0; k < run; k += 3) {
        int t[3];
        br.ints(smallidx, sizesmall, t);
        i++;
        t[0] += prevcoord[0] - smallnum;
        t[1] += prevcoord[1] - smallnum;
        t[2] += prevcoord[2] - smallnum;
        if (k == 0) {  // the first two atoms were swapped by the writer (water)
          std::swap(t[0], prevcoord[0]);
          std::swap(t[1], prevcoord[1]);
          std::swap(t[2], prevcoord[2]);
          *lfp++ = (float)prevcoord[0] * inv_precision;
          *lfp++ = (float)prevcoord[1] * inv_precision;
          *lfp++ = (float)prevcoord[2] * inv_precision;
        } else {
          prevcoord[0] = t[0];
          prevcoord[1] = t[1];
          prevcoord[2] = t[2];
        }
        *lfp++ = (float)t[0] * inv_precision;
        *lfp++ = (float)t[1] * inv_precision;
        *lfp++ = (float)t[2] * inv_precision;
      }
    } else {
      *lfp++ = (float)cur[0] * inv_precision;
      *lfp++ = (float)cur[1] * inv_precision;
      *lfp++ = (float)cur[2] * inv_precision;
    }
    smallidx += is_smaller;
    if (smallidx < FIRSTIDX - 1 || smallidx >= LASTIDX) return -1;
    if (is_smaller < 0) {
      smallnum = smaller;
      smaller = smallidx > FIRSTIDX ? magicints[smallidx - 1] / 2 : 0;
    } else if (is_smaller > 0) {
      smaller = smallnum;
      smallnum = magicints[smallidx] / 2;
    }
    sizesmall[0] = sizesmall[1] = sizesmall[2] = magicints[smallidx];
  }
  if (br.overrun) return -1;
  p += ((size_t)nbytes + 3) & ~(size_t)3;
  return p - p0;
}

// Encode one coordinate block (nm floats) -- the xdrfile compressor.
bool encode_coords(const float *ptr, int size, float precision, std::vector<unsigned char> &o) {
#pragma clang fp contract(off)
  wr_i(o, size);
  if (size <= 9) {
    for (int i = 0; i < 3 * size; ++i) wr_f(o, ptr[i]);
    return true;
  }
  if (precision <= 0) precision = 1000;
  wr_f(o, precision);
  std::vector<int> ip(3 * (size_t)size + 3 * 9, 0);  // slack: the run loop peeks one atom ahead
  int minint[3] = {INT_MAX, INT_MAX, INT_MAX}, maxint[3] = {INT_MIN, INT_MIN, INT_MIN};
  int mindiff = INT_MAX, old[3] = {0, 0, 0};
  for (int i = 0; i < size; ++i) {
    int l[3];
    for (int c = 0; c < 3; ++c) {
      const float v = ptr[3 * i + c];
      const float lf = v >= 0.0f ? v * precision + 0.5f : v * precision - 0.5f;
      if (std::fabs(lf) > (float)(INT_MAX - 2)) return false;
      l[c] = (int)lf;
      minint[c] = std::min(minint[c], l[c]);
      maxint[c] = std::max(maxint[c], l[c]);
      ip[3 * i + c] = l[c];
    }
    const int diff = std::abs(old[0] - l[0]) + std::abs(old[1] - l[1]) + std::abs(old[2] - l[2]);
    if (diff < mindiff && i >= 1) mindiff = diff;
    old[0] = l[0];
    old[1] = l[1];
    old[2] = l[2];
  }
  for (int c = 0; c < 3; ++c) wr_i(o, minint[c]);
  for (int c = 0; c < 3; ++c) wr_i(o, maxint[c]);
  for (int c = 0; c < 3; ++c)
    if ((float)maxint[c] - (float)minint[c] >= (float)(INT_MAX - 2)) return false;
  unsigned sizeint[3], bitsizeint[3] = {0, 0, 0};
  for (int c = 0; c < 3; ++c) sizeint[c] = (unsigned)(maxint[c] - minint[c]) + 1u;
  int bitsize = 0;
  if ((sizeint[0] | sizeint[1] | sizeint[2]) > 0xffffff) {
    for (int c = 0; c < 3; ++c) bitsizeint[c] = sizeofint(sizeint[c]);
  } else {
    bitsize = sizeofints(sizeint);
  }
  // (the published loop can run to LASTIDX and then read magicints[LASTIDX]
  // when no two consecutive atoms are close; clamp to the table instead)
  int smallidx = FIRSTIDX;
  while (smallidx < LASTIDX - 1 && magicints[smallidx] < mindiff) smallidx++;
  wr_i(o, smallidx);
  const int maxidx = std::min(LASTIDX - 1, smallidx + 8);
  const int minidx = maxidx - 8;
  int smaller = magicints[std::max(FIRSTIDX, smallidx - 1)] / 2;
  int smallnum = magicints[smallidx] / 2;
  unsigned sizesmall[3];
  sizesmall[0] = sizesmall[1] = sizesmall[2] = magicints[smallidx];
  const int larger = magicints[maxidx] / 2;
  BitWriter bw;
  int prevcoord[3] = {0, 0, 0};
  int prevrun = -1;
  int i = 0;
  unsigned tmpcoord[30];
  while (i < size) {
    int is_small = 0, is_smaller;
    int *thiscoord = ip.data() + 3 * (size_t)i;
    if (smallidx < maxidx && i >= 1 && std::abs(thiscoord[0] - prevcoord[0]) < larger &&
        std::abs(thiscoord[1] - prevcoord[1]) < larger && std::abs(thiscoord[2] - prevcoord[2]) < larger) {
      is_smaller = 1;
    } else if (smallidx > minidx) {
      is_smaller = -1;
    } else {
      is_smaller = 0;
    }
    if (i + 1 < size) {
      if (std::abs(thiscoord[0] - thiscoord[3]) < smallnum && std::abs(thiscoord[1] - thiscoord[4]) < smallnum &&
          std::abs(thiscoord[2] - thiscoord[5]) < smallnum) {
        std::swap(thiscoord[0], thiscoord[3]);  // water: swap the first two atoms
        std::swap(thiscoord[1], thiscoord[4]);
        std::swap(thiscoord[2], thiscoord[5]);
        is_small = 1;
      }
    }
    const unsigned tc[3] = {(unsigned)(thiscoord[0] - minint[0]), (unsigned)(thiscoord[1] - minint[1]),
                            (unsigned)(thiscoord[2] - minint[2])};
    if (bitsize == 0) {
      bw.bits(bitsizeint[0], (int)tc[0]);
      bw.bits(bitsizeint[1], (int)tc[1]);
      bw.bits(bitsizeint[2], (int)tc[2]);
    } else if (!bw.ints(bitsize, sizeint, tc)) {
      return false;
    }
    prevcoord[0] = thiscoord[0];
    prevcoord[1] = thiscoord[1];
    prevcoord[2] = thiscoord[2];
    thiscoord += 3;
    i++;
    int run = 0;
    if (is_small == 0 && is_smaller == -1) is_smaller = 0;
    while (is_small && run < 8 * 3) {
      long tmpsum = 0;
      for (int j = 0; j < 3; ++j) {
        const long t = thiscoord[j] - prevcoord[j];
        tmpsum += t * t;
      }
      if (is_smaller == -1 && tmpsum >= (long)smaller * smaller) is_smaller = 0;
      tmpcoord[run++] = (unsigned)(thiscoord[0] - prevcoord[0] + smallnum);
      tmpcoord[run++] = (unsigned)(thiscoord[1] - prevcoord[1] + smallnum);
      tmpcoord[run++] = (unsigned)(thiscoord[2] - prevcoord[2] + smallnum);
      prevcoord[0] = thiscoord[0];
      prevcoord[1] = thiscoord[1];
      prevcoord[2] = thiscoord[2];
      i++;
      thiscoord += 3;
      is_small = 0;
      if (i < size && std::abs(thiscoord[0] - prevcoord[0]) < smallnum &&
          std::abs(thiscoord[1] - prevcoord[1]) < smallnum && std::abs(thiscoord[2] - prevcoord[2]) < smallnum) {
        is_small = 1;
      }
    }
    if (run != prevrun || is_smaller != 0) {
      prevrun = run;
      bw.bits(1, 1);
      bw.bits(5, run + is_smaller + 1);
    } else {
      bw.bits(1, 0);
    }
    for (int k = 0; k < run; k += 3)
      if (!bw.ints(smallidx, sizesmall, &tmpcoord[k])) return false;
    if (is_smaller != 0) {
      smallidx += is_smaller;
      if (is_smaller < 0) {
        smallnum = smaller;
        smaller = magicints[smallidx - 1] / 2;
      } else {
        smaller = smallnum;
        smallnum = magicints[smallidx] / 2;
      }
      sizesmall[0] = sizesmall[1] = sizesmall[2] = magicints[smallidx];
    }
  }
  bw.flush();
  wr_i(o, (int)bw.out.size());
  o.insert(o.end(), bw.out.begin(), bw.out.end());
  while (o.size() % 4) o.push_back(0);
  return true;
}

}  // namespace

bool rmsf_internal_pread_all(int fd, void *dst, size_t n, int64_t off) {
  char *d = static_cast<char *>(dst);
  while (n > 0) {
    const ssize_t r = pread(fd, d, n, (off_t)off);
    if (r <= 0) return false;
    d += r;
    n -= (size_t)r;
    off += r;
  }
  return true;
}

namespace {

// decode frame f of x into `dst` (Angstrom), selecting `sel` rows
bool decode_frame(const rmsf_xtc *x, int64_t f, const int32_t *sel, int64_t n_sel, float *dst,
                  std::vector<unsigned char> &raw, std::vector<float> &nm) {
  raw.resize((size_t)x->size[f]);
  if (!rmsf_internal_pread_all(x->fd, raw.data(), raw.size(), x->offset[f])) return false;
  nm.resize(3 * (size_t)x->n_atoms);
  const size_t hdr = 4 * 4 + 9 * 4;
  if (decode_coords(raw.data() + hdr, raw.size() - hdr, (int)x->n_atoms, nm.data()) < 0) return false;
  if (sel) {
    for (int64_t a = 0; a < n_sel; ++a)
      for (int c = 0; c < 3; ++c) dst[3 * a + c] = nm[3 * (size_t)sel[a] + c] * 10.0f;
  } else {
    for (int64_t k = 0; k < 3 * x->n_atoms; ++k) dst[k] = nm[k] * 10.0f;
  }
  return true;
}

}  // namespace

// Frame-parallel decode used by the stager (stager.cpp) and rmsf_xtc_read.
extern "C" int rmsf_internal_xtc_decode(const rmsf_xtc *x, int64_t f0, int64_t n, int64_t step, const int32_t *sel,
                                        int64_t n_sel, float *out, int64_t out_stride, int n_threads) {
  std::atomic<int64_t> next{0};
  std::atomic<bool> bad{false};
  auto work = [&] {
    std::vector<unsigned char> raw;
    std::vector<float> nm;
    for (;;) {
      const int64_t k = next.fetch_add(1);
      if (k >= n || bad.load()) return;
      if (!decode_frame(x, f0 + k * step, sel, n_sel, out + k * out_stride, raw, nm)) bad.store(true);
    }
  };
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(n_threads, n));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto &t : th) t.join();
  return bad.load() ? fail(RMSF_EINVAL, "xtc: corrupt frame") : RMSF_OK;
}

extern "C" int64_t rmsf_internal_xtc_natoms(const rmsf_xtc *x) { return x ? x->n_atoms : 0; }
extern "C" int64_t rmsf_internal_xtc_nframes(const rmsf_xtc *x) { return x ? (int64_t)x->offset.size() : 0; }

extern "C" {

RMSF_EXPORT int rmsf_xtc_open(const char *path, rmsf_xtc **out, int64_t *n_atoms, int64_t *n_frames) {
  if (!path || !out) return fail(RMSF_EINVAL, "rmsf_xtc_open: bad arguments");
  *out = nullptr;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(RMSF_EINVAL, std::string("rmsf_xtc_open: cannot open ") + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return fail(RMSF_EINVAL, "rmsf_xtc_open: stat failed");
  }
  static std::atomic<uint64_t> next_serial{1};
  auto *x = new rmsf_xtc();
  x->serial = next_serial.fetch_add(1);
  x->fd = fd;
  const int64_t fsize = st.st_size;
  int64_t off = 0;
  unsigned char h[4 * 4 + 9 * 4 + 4 + 4 + 24 + 4 + 4];
  while (off < fsize) {
    const size_t want = (size_t)std::min<int64_t>((int64_t)sizeof h, fsize - off);
    if (want < 4 * 4 + 9 * 4 + 4 || !rmsf_internal_pread_all(fd, h, want, off)) break;
    const unsigned char *p = h;
    const int magic = rd_i(p), na = rd_i(p), stp = rd_i(p);
    const float tm = rd_f(p);
    float box[9];
    for (float &b : box) b = rd_f(p);
    const int lsize = rd_i(p);
    if (magic != kMagic || na <= 0 || lsize != na || (x->n_atoms && na != x->n_atoms)) {
      rmsf_xtc_close(x);
      return fail(RMSF_EINVAL, "rmsf_xtc_open: not an XTC file or inconsistent atom count at byte " +
                                   std::to_string(off));
    }
    int64_t sz = 4 * 4 + 9 * 4 + 4;
    if (na <= 9) {
      sz += 12 * (int64_t)na;
    } else {
      if (want < sizeof h) break;
      p += 4 + 24 + 4;  // precision, minint, maxint, smallidx
      const int nbytes = rd_i(p);
      if (nbytes < 0) break;
      sz += 4 + 24 + 4 + 4 + ((nbytes + 3) & ~3);
    }
    if (off + sz > fsize) break;  // truncated last frame: ignored, as readers do
    x->n_atoms = na;
    x->offset.push_back(off);
    x->size.push_back(sz);
    x->max_size = std::max(x->max_size, sz);
    x->step.push_back(stp);
    x->time.push_back(tm);
    x->box.insert(x->box.end(), box, box + 9);
    off += sz;
  }
  if (x->offset.empty()) {
    rmsf_xtc_close(x);
    return fail(RMSF_EINVAL, "rmsf_xtc_open: no complete frame");
  }
  *out = x;
  if (n_atoms) *n_atoms = x->n_atoms;
  if (n_frames) *n_frames = (int64_t)x->offset.size();
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_xtc_close(rmsf_xtc *x) {
  if (x) {
    if (x->fd >= 0) close(x->fd);
    delete x;
  }
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_xtc_frame_info(const rmsf_xtc *x, int64_t f, int32_t *step, float *time, float *box9) {
  if (!x || f < 0 || f >= (int64_t)x->offset.size()) return fail(RMSF_EINVAL, "rmsf_xtc_frame_info: bad frame");
  if (step) *step = x->step[f];
  if (time) *time = x->time[f];
  if (box9) std::memcpy(box9, &x->box[9 * f], 9 * sizeof(float));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_xtc_frame_record(const rmsf_xtc *x, int64_t f, int64_t *offset, int64_t *bytes) {
  if (!x || f < 0 || f >= (int64_t)x->offset.size()) return fail(RMSF_EINVAL, "rmsf_xtc_frame_record: bad frame");
  if (offset) *offset = x->offset[f];
  if (bytes) *bytes = x->size[f];
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_xtc_read(const rmsf_xtc *x, int64_t f0, int64_t n, int64_t step, const int32_t *h_sel,
                              int64_t n_sel, float *h_out, int n_threads) {
  if (!x || !h_out || n < 0 || step < 1 || f0 < 0 || (n > 0 && f0 + (n - 1) * step >= (int64_t)x->offset.size()))
    return fail(RMSF_EINVAL, "rmsf_xtc_read: bad arguments");
  if (h_sel)
    for (int64_t a = 0; a < n_sel; ++a)
      if (h_sel[a] < 0 || h_sel[a] >= x->n_atoms) return fail(RMSF_EINVAL, "rmsf_xtc_read: selection out of range");
  const int64_t rows = h_sel ? n_sel : x->n_atoms;
  return rmsf_internal_xtc_decode(x, f0, n, step, h_sel, rows, h_out, 3 * rows, n_threads);
}

RMSF_EXPORT int rmsf_xtc_write(const char *path, const float *xyz, int64_t n_frames, int64_t n_atoms, float precision,
                               const float *box9, int append) {
  if (!path || !xyz || n_frames < 0 || n_atoms < 1 || n_atoms > INT_MAX / 3)
    return fail(RMSF_EINVAL, "rmsf_xtc_write: bad arguments");
  FILE *fp = std::fopen(path, append ? "ab" : "wb");
  if (!fp) return fail(RMSF_EINVAL, std::string("rmsf_xtc_write: cannot open ") + path);
  // frames are encoded independently on a few threads, written in order
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({n_frames, 16, (int64_t)std::thread::hardware_concurrency()}));
  int rc = RMSF_OK;
  std::vector<std::vector<unsigned char>> enc((size_t)nt);
  for (int64_t f0 = 0; f0 < n_frames && rc == RMSF_OK; f0 += nt) {
    const int64_t n = std::min<int64_t>(nt, n_frames - f0);
    std::atomic<bool> bad{false};
    auto work = [&](int64_t k) {
      std::vector<unsigned char> &o = enc[(size_t)k];
      std::vector<float> nm(3 * (size_t)n_atoms);
      const float *src = xyz + (f0 + k) * 3 * n_atoms;
      for (size_t i = 0; i < nm.size(); ++i) nm[i] = src[i] * 0.1f;  // Angstrom -> nm (MDAnalysis writer)
      o.clear();
      wr_i(o, kMagic);
      wr_i(o, (int)n_atoms);
      wr_i(o, (int)(f0 + k));
      wr_f(o, (float)(f0 + k));
      for (int j = 0; j < 9; ++j) wr_f(o, box9 ? box9[j] * 0.1f : 0.0f);
      if (!encode_coords(nm.data(), (int)n_atoms, precision, o)) bad.store(true);
    };
    std::vector<std::thread> th;
    for (int64_t k = 1; k < n; ++k) th.emplace_back(work, k);
    work(0);
    for (auto &t : th) t.join();
    if (bad.load()) {
      rc = fail(RMSF_EINVAL, "rmsf_xtc_write: coordinates out of range for this precision");
      break;
    }
    for (int64_t k = 0; k < n; ++k)
      if (std::fwrite(enc[(size_t)k].data(), 1, enc[(size_t)k].size(), fp) != enc[(size_t)k].size()) {
        rc = fail(RMSF_EINVAL, "rmsf_xtc_write: write failed");
        break;
      }
  }
  std::fclose(fp);
  return rc;
}

}  // extern "C"
