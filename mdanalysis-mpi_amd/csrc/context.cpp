// context.cpp -- the RMSF context (rmsf_ctx_*, rmsf_push_*, rmsf_get_*,
// rmsf_multi_*): RMSF.py's whole per-rank loop (RMSF.py:80-146) behind one
// opaque handle, for hosts that bring neither torch nor a device allocator.
//
// Host-side orchestration only -- every device step is one of the kernel
// entry points of rmsf_kernels.hip (reference setup, superpose, accumulate,
// Chan merge, ...), the stager of stager.cpp, or an RCCL all-reduce.
//
// State on the context's device:
//   sel[n_sel] int32 (NULL = contiguous), masses[n_sel] f64 (NULL = uniform)
//   ref[3 n_sel] + refinfo[RMSF_REFINFO_DOUBLES]      centred reference
//   wel: parts [1+S][3 n_sel] x2 (slot 0 = running mean / M2, 1..S = the
//        current chunk's split partials), n               (RMSF.py:120-138)
//   sum: parts [1+S][3 n_sel] (slot 0 = running sum), n   (RMSF.py:89-105)
//   xform[chunk][16] + superpose workspace, exchange buffers, rmsf[n_sel]
//   shift[3 n_sel] f32: the unaligned merge's shift frame (selected rows)
//
// Laziness (round 4), invisible to every entry point: a push's fold is
// deferred until the running state is next used (the shifted merge then
// folds and packs in one launch); a reset only marks the state, which is
// zeroed if it is read before a fold overwrites it; rmsf_multi_push_frames
// may record a push for the atom-slab merge, which any other call runs whole.
// Host side: one worker thread per device for the rmsf_multi_* calls, a side
// stream for digests and the shift frame's gather, a communicator stream for
// the slab merge's collectives.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "rmsf_hip.h"
#include "xtc_internal.h"

#define RMSF_EXPORT __attribute__((visibility("default")))

extern "C" int rmsf_internal_set_error(int code, const char *msg);

namespace {

int fail(int code, const std::string &m) { return rmsf_internal_set_error(code, m.c_str()); }

#define CX_HIP(expr)                                                                                \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess) return fail(RMSF_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define CX_OK(expr)              \
  do {                           \
    int rc_ = (expr);            \
    if (rc_ != RMSF_OK) return rc_; \
  } while (0)

constexpr int64_t kChunkFrames = 16384;         // frames per superpose/accumulate launch group
constexpr int64_t kSlabMinAtoms = 1000000;      // auto atom slabs from 1M atoms (pipeline.SLAB_MIN_ATOMS)
constexpr int kSlabsAuto = 2;                   // pipeline.SLABS_AUTO
constexpr int64_t kStageBytes = 64ll << 20;     // default pinned slot size

// ---- RCCL, resolved at first use (the library torch already loaded, if any,
// shares the soname and is reused) -------------------------------------------
struct Rccl {
  ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                         hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char *(*GetErrorString)(ncclResult_t) = nullptr;
  bool ok = false;
  std::string why;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      r.why = std::string("cannot load librccl.so.1: ") + dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](auto &fp, const char *name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
      if (!fp) all = false;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommInitAll, "ncclCommInitAll");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.AllReduce, "ncclAllReduce");
    sym(r.Reduce, "ncclReduce");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    r.ok = all;
    if (!all) r.why = "librccl.so.1 lacks a required symbol";
  });
  return r;
}

int nccl_fail(const char *what, ncclResult_t e) {
  const Rccl &r = rccl();
  return fail(RMSF_EHIP, std::string(what) + ": " + (r.GetErrorString ? r.GetErrorString(e) : "rccl error"));
}

// Make `dev` current for a scope, restoring the caller's device.
struct DeviceScope {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  // grow to >= need bytes; work queued on `s` may still use the old buffer,
  // so it is drained first (keep: the old contents are carried over)
  int ensure(size_t need, hipStream_t s, bool keep = false) {
    if (need <= bytes) return RMSF_OK;
    // the buffer is allocated on the current device: it must be the stream's
    // (a context's buffers live on its own device; a caller that forgot its
    // DeviceScope would hand the kernels another device's pointer)
    int cur = -1;
    hipDevice_t sd = -1;
    if (s && hipGetDevice(&cur) == hipSuccess && hipStreamGetDevice(s, &sd) == hipSuccess && sd != cur)
      return fail(RMSF_EHIP, "internal: buffer for a device-" + std::to_string(sd) + " stream allocated while device " +
                                 std::to_string(cur) + " is current");
    if (p) {
      hipError_t e0 = hipStreamSynchronize(s);
      if (e0 != hipSuccess) return fail(RMSF_EHIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e0));
    }
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, need);
    if (e != hipSuccess) return fail(RMSF_ENOMEM, std::string("hipMalloc(") + std::to_string(need) + "): " + hipGetErrorString(e));
    if (keep && p && bytes) (void)hipMemcpy(q, p, bytes, hipMemcpyDeviceToDevice);
    if (p) (void)hipFree(p);
    p = q;
    bytes = need;
    return RMSF_OK;
  }
  double *d() const { return static_cast<double *>(p); }
};

// Running partial over pushed chunks: parts0/parts1 hold the result (mean/sum, M2).
struct Running {
  DevBuf parts0, parts1;
  int64_t n = 0;
  bool stale = false;  // reset lazily: zeroed only if read before a fold overwrites it
};

// One host thread per context for the multi-context calls
// (rmsf_multi_push_frames, the slab merge): each context's launches are
// enqueued from its own thread, so N devices start their sweeps together
// instead of one after another behind a single thread's launch latency.
struct Worker {
  std::thread th;
  std::mutex m;
  std::condition_variable cv;
  std::function<int()> job;
  bool has = false, done = true, quit = false;
  int rc = 0;
  std::string err;
  Worker() : th([this] { loop(); }) {}
  ~Worker() {
    {
      std::lock_guard<std::mutex> lk(m);
      quit = true;
    }
    cv.notify_all();
    th.join();
  }
  void loop() {
    for (;;) {
      std::function<int()> j;
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return has || quit; });
        if (!has) return;
        j = std::move(job);
        has = false;
      }
      const int r = j();
      std::string e = r ? std::string(rmsf_last_error()) : std::string();
      {
        std::lock_guard<std::mutex> lk(m);
        rc = r;
        err = std::move(e);
        done = true;
      }
      cv.notify_all();
    }
  }
  void post(std::function<int()> f) {
    {
      std::lock_guard<std::mutex> lk(m);
      job = std::move(f);
      has = true;
      done = false;
    }
    cv.notify_all();
  }
  int wait(std::string *e) {
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [&] { return done; });
    *e = err;
    return rc;
  }
};

// Order-independent 64-bit digest of a reference structure: the bit patterns
// of the centred reference ref[0..n) and of its COM info[0..3) (what the
// shifted merge uses as its shift, k_chan_shift_pack), each word mixed with
// its position and summed mod 2^64.  Two contexts whose digests differ hold
// different references; equal digests mean identical bits up to a 2^-64
// collision.  rmsf_multi_chan_merge takes the one-all-reduce shifted merge
// only when every context's digest is equal.
__host__ __device__ inline uint64_t dig_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <class W>
__global__ __launch_bounds__(256) void k_digest(const W *__restrict__ a, int64_t n, const uint64_t *__restrict__ info,
                                                int64_t n_info, unsigned long long *__restrict__ out) {
  uint64_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n + n_info; j += stride) {
    const uint64_t w = j < n ? (uint64_t)a[j] : info[j - n];
    acc += dig_mix(w ^ dig_mix((uint64_t)j));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += (uint64_t)__shfl_xor((unsigned long long)acc, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

}  // namespace

struct rmsf_ctx {
  int dev = 0;
  int64_t n_atoms = 0, n_sel = 0, n_coord = 0;
  std::vector<int32_t> h_sel;  // empty = contiguous
  bool has_masses = false;
  std::vector<double> h_masses;
  hipStream_t stream = nullptr;
  DevBuf sel, masses, ref, refinfo, xform, work, accwork, frame, avg, rmsf, xa, xb, cnt, refdig;
  DevBuf seqwork;  // the sequential Welford's per-frame coefficients (RMSF_PUSH_EXACT)
  bool ref_set = false;
  Running wel, sum;
  rmsf_stager *stager = nullptr;
  rmsf_xtcdec *xdec = nullptr;  // GPU XTC decoder, bound to the file of serial xdec_serial
  uint64_t xdec_serial = 0;
  int64_t stage_batch = 0;  // 0 = auto
  int stage_slots = 2, stage_threads = 4;
  bool stager_dirty = true;
  ncclComm_t comm = nullptr;
  int comm_size = 0;  // ranks of `comm` (0 = none)
  // measurement (rmsf_ctx_set_timing): HIP events around each superpose /
  // accumulate launch on the context stream, with the atom-frames it covered
  struct Span {
    hipEvent_t a, b;
    int which;  // RMSF_TIME_ACCUMULATE / RMSF_TIME_SUPERPOSE / RMSF_TIME_MERGE
    int64_t atom_frames;
    bool closed;  // b recorded
  };
  bool timing = false;
  std::vector<Span> spans;
  int open_merge = -1;  // index of the merge span awaiting its end event
  std::vector<hipEvent_t> event_pool;  // events of read spans, reused by the next ones
  // per-frame QCP rmsd of the aligned Welford pushes (rmsf_ctx_collect_rmsd)
  bool collect_rmsd = false;
  DevBuf rmsd;
  int64_t n_rmsd = 0;
  // the merge's shift for unaligned Welford state (rmsf_set_merge_shift_frame):
  // a selected frame, f32 [n_sel][3], with its digest
  DevBuf shift, zidx, shiftdig;
  bool shift_set = false, zidx_set = false;
  // each digest is also copied to pinned host memory, an event after it: the
  // merge reads it without waiting for the sweep queued behind the setter
  unsigned long long *h_dig[2] = {nullptr, nullptr};  // [reference, shift frame]
  hipEvent_t ev_dig[2] = {nullptr, nullptr};
  // side stream for the digests and the shift frame's gather: they run beside
  // the sweep instead of in front of it (the merge waits for ev_dig[1])
  hipStream_t side = nullptr;
  hipEvent_t ev_main = nullptr;
  bool wel_aligned = false;  // the Welford state came from aligned pushes
  // the last balanced accumulate's fold, deferred until the state is next
  // used, so a merge can fold and pack in one launch (rmsf_fold_balanced_shift)
  struct PendingFold {
    bool on = false, welford = false;
    int mode_k = 0;
    int64_t acc_n = 0;
  } pend;
  // a device push recorded by rmsf_multi_push_frames for the atom-slab merge
  // (run by the next rmsf_multi_chan_merge_root, or whole by any other call)
  struct SlabPush {
    bool on = false;
    const float *d = nullptr;
    int64_t stride = 0, n_frames = 0, chunks = 0;
    int k = 0;
  } slab;
  bool merged_away = false;  // a reduce-to-root merge left the result on another context
  bool rmsf_valid = false;   // rmsf holds the finalised result of the current state
  int transport = RMSF_TRANSPORT_AUTO;
  hipStream_t comm_stream = nullptr;  // the slab merge's RCCL calls (beside the next slab)
  std::vector<hipEvent_t> ev_pack, ev_done;
  hipEvent_t ev_sent = nullptr;  // the exact merge: this context's state is ready to be read by a peer
  hipEvent_t ev_pulled = nullptr;  // ... and a peer's copy of it (on this context's stream) has completed
  // exact=True for aligned pushes (rmsf_ctx_set_exact): references, pushes and
  // the sweep-1 sum exchange in the reference's own summation orders
  bool exact = false;
  double mass_total = 0.0;  // numpy's masses.sum() (pairwise), the COM divisor
  bool ref_exact = false;   // the current reference record came from the sequential setup
  Worker *worker = nullptr;

  const int32_t *d_sel() const { return h_sel.empty() ? nullptr : static_cast<const int32_t *>(sel.p); }
  const double *d_masses() const { return has_masses ? masses.d() : nullptr; }
};

namespace {

int check_ctx(const rmsf_ctx *c, const char *fn) {
  if (!c) return fail(RMSF_EINVAL, std::string(fn) + ": null context");
  return RMSF_OK;
}

// Every stream, event and buffer a context owns lives on the context's
// device.  The creation sites check that this device is current (a missing
// DeviceScope on a worker thread would otherwise create them on device 0:
// the bug class of ADVICE r4) -- DevBuf::ensure checks the same against its
// stream's device.  A one-GPU box never trips these; they guard the
// multi-device paths that have not run on distinct devices here.
int on_device(const rmsf_ctx *c, const char *what) {
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != c->dev)
    return fail(RMSF_EHIP, std::string("internal: ") + what + " for a device-" + std::to_string(c->dev) +
                               " context created while device " + std::to_string(cur) + " is current");
  return RMSF_OK;
}

// the context stream and its side stream (a shift frame's gather reads a
// caller's frame there): what a getter waits for before the caller may free
// what it pushed
int sync_streams(rmsf_ctx *c) {
  CX_HIP(hipStreamSynchronize(c->stream));
  if (c->side) CX_HIP(hipStreamSynchronize(c->side));
  return RMSF_OK;
}

int zero_running(rmsf_ctx *c, Running &r, bool two) {
  const size_t row = sizeof(double) * c->n_coord;
  CX_OK(r.parts0.ensure(row, c->stream, true));
  CX_HIP(hipMemsetAsync(r.parts0.p, 0, row, c->stream));
  if (two) {
    CX_OK(r.parts1.ensure(row, c->stream, true));
    CX_HIP(hipMemsetAsync(r.parts1.p, 0, row, c->stream));
  }
  r.n = 0;
  r.stale = false;
  return RMSF_OK;
}

// A reset state is zeroed only when it is read with no frame folded in (an
// empty block): the first balanced fold of a push overwrites it otherwise.
int ensure_zeroed(rmsf_ctx *c, Running &r, bool two) {
  if (r.parts0.bytes == 0 || (r.n == 0 && r.stale)) return zero_running(c, r, two);
  return RMSF_OK;
}

// Brackets `launch` with timing events on the context stream when timing is on.
template <class F>
int timed(rmsf_ctx *c, int which, int64_t atom_frames, F &&launch) {
  if (!c->timing) return launch();
  rmsf_ctx::Span sp{nullptr, nullptr, which, atom_frames, true};
  if (c->event_pool.size() < 2) CX_OK(on_device(c, "a timing event"));
  auto take = [c](hipEvent_t *e) -> hipError_t {
    if (c->event_pool.empty()) return hipEventCreate(e);
    *e = c->event_pool.back();
    c->event_pool.pop_back();
    return hipSuccess;
  };
  CX_HIP(take(&sp.a));
  if (take(&sp.b) != hipSuccess) {
    c->event_pool.push_back(sp.a);
    return fail(RMSF_EHIP, "hipEventCreate failed");
  }
  c->spans.push_back(sp);  // owned by the context from here on
  CX_HIP(hipEventRecord(sp.a, c->stream));
  CX_OK(launch());
  CX_HIP(hipEventRecord(sp.b, c->stream));
  return RMSF_OK;
}

// The merge's span (RMSF_TIME_MERGE): opened on `s` where the context's
// exchange starts (its moments packed), closed on `s2` where its result is
// finished -- the collective, the wait for the slowest rank and the unpack,
// as each device's stream sees them.
int merge_open(rmsf_ctx *c, hipStream_t s) {
  if (!c->timing) return RMSF_OK;
  if (c->event_pool.size() < 2) CX_OK(on_device(c, "a merge timing event"));
  hipEvent_t a = nullptr, b = nullptr;
  auto take = [c](hipEvent_t *e) -> hipError_t {
    if (c->event_pool.empty()) return hipEventCreate(e);
    *e = c->event_pool.back();
    c->event_pool.pop_back();
    return hipSuccess;
  };
  CX_HIP(take(&a));
  if (take(&b) != hipSuccess) {
    c->event_pool.push_back(a);
    return fail(RMSF_EHIP, "hipEventCreate failed");
  }
  c->spans.push_back({a, b, RMSF_TIME_MERGE, 0, false});
  c->open_merge = (int)c->spans.size() - 1;
  CX_HIP(hipEventRecord(a, s));
  return RMSF_OK;
}

int merge_close(rmsf_ctx *c, hipStream_t s) {
  if (!c->timing || c->open_merge < 0) return RMSF_OK;
  rmsf_ctx::Span &sp = c->spans[c->open_merge];
  c->open_merge = -1;
  CX_HIP(hipEventRecord(sp.b, s));
  sp.closed = true;
  return RMSF_OK;
}

// which >= 0: the spans of that family are read -- their events go back to
// the pool; which < 0: the context is destroyed -- every event is released
void drop_spans(rmsf_ctx *c, int which) {
  std::vector<rmsf_ctx::Span> keep;
  for (auto &sp : c->spans) {
    if (which < 0) {
      (void)hipEventDestroy(sp.a);
      (void)hipEventDestroy(sp.b);
    } else if (sp.which == which) {
      c->event_pool.push_back(sp.a);
      c->event_pool.push_back(sp.b);
    } else {
      keep.push_back(sp);
    }
  }
  c->spans.swap(keep);
  c->open_merge = -1;
  for (size_t i = 0; i < c->spans.size(); ++i)
    if (c->spans[i].which == RMSF_TIME_MERGE && !c->spans[i].closed) c->open_merge = (int)i;
  if (which < 0) {
    for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
    c->event_pool.clear();
  }
}

// the deferred fold of the last accumulate (plain: into the running state)
int flush_fold(rmsf_ctx *c) {
  if (!c->pend.on) return RMSF_OK;
  c->pend.on = false;
  Running &r = c->pend.welford ? c->wel : c->sum;
  return rmsf_fold_balanced(c->accwork.p, c->n_coord, c->pend.mode_k, c->pend.acc_n, r.parts0.d(),
                            c->pend.welford ? r.parts1.d() : nullptr, c->stream);
}

// exact mode, aligned or summing pushes: RMSF.py:94-103 / 127-138 with the
// reference's summation orders -- rmsf_superpose_sequential for the frames'
// records, rmsf_accumulate_sequential continuing the running state at k = n
int process_exact(rmsf_ctx *c, const float *d_xyz, int64_t stride, int64_t n_frames, const int32_t *d_sel, int mode) {
  const bool aligned = mode == RMSF_PUSH_ALIGN_SUM || mode == RMSF_PUSH_ALIGN_WELFORD;
  const bool welford = mode == RMSF_PUSH_ALIGN_WELFORD;
  const double *xf = nullptr;
  if (aligned) {
    if (!c->ref_set) return fail(RMSF_EINVAL, "rmsf_push: aligned mode before a reference was set");
    if (!c->ref_exact)
      return fail(RMSF_EINVAL, "rmsf_push: exact mode needs its reference set after rmsf_ctx_set_exact "
                               "(the sequential setup's record)");
    CX_OK(c->xform.ensure(sizeof(double) * RMSF_XFORM_DOUBLES * (size_t)n_frames, c->stream));
    CX_OK(timed(c, RMSF_TIME_SUPERPOSE, c->n_sel * n_frames, [&] {
      return rmsf_superpose_sequential(d_xyz, stride, n_frames, c->n_sel, d_sel, c->d_masses(), c->mass_total,
                                       c->ref.d(), c->refinfo.d(), c->xform.d(), c->stream);
    }));
    xf = c->xform.d();
    if (welford && c->collect_rmsd) {
      const size_t need = sizeof(double) * (size_t)(c->n_rmsd + n_frames);
      CX_OK(c->rmsd.ensure(need > c->rmsd.bytes ? std::max(need, 2 * c->rmsd.bytes) : need, c->stream, true));
      CX_HIP(hipMemcpy2DAsync(c->rmsd.d() + c->n_rmsd, sizeof(double), c->xform.d() + 12,
                              sizeof(double) * RMSF_XFORM_DOUBLES, sizeof(double), (size_t)n_frames,
                              hipMemcpyDeviceToDevice, c->stream));
      c->n_rmsd += n_frames;
    }
  }
  Running &r = welford ? c->wel : c->sum;
  const size_t row = sizeof(double) * c->n_coord;
  CX_OK(r.parts0.ensure(row, c->stream, true));
  if (welford) {
    CX_OK(r.parts1.ensure(row, c->stream, true));
    const size_t wb = rmsf_welford_sequential_workspace_bytes(n_frames);
    CX_OK(c->seqwork.ensure(std::max<size_t>(wb, 16), c->stream));
  }
  CX_OK(timed(c, RMSF_TIME_ACCUMULATE, c->n_sel * n_frames, [&] {
    return rmsf_accumulate_sequential(d_xyz, stride, n_frames, c->n_sel, d_sel, xf, aligned ? c->refinfo.d() : nullptr,
                                      welford ? RMSF_MODE_WELFORD : RMSF_MODE_SUM, r.n, r.parts0.d(),
                                      welford ? r.parts1.d() : nullptr, welford ? c->seqwork.p : nullptr,
                                      welford ? c->seqwork.bytes : 0, c->stream);
  }));
  r.n += n_frames;
  r.stale = false;
  if (welford) {
    c->wel_aligned = aligned;
    c->rmsf_valid = false;
    c->merged_away = false;
  }
  return RMSF_OK;
}

// one launch group over n_frames device frames: [superpose] + accumulate; its
// fold is deferred (flush_fold / the merge's fused fold + pack)
int process(rmsf_ctx *c, const float *d_xyz, int64_t stride, int64_t n_frames, const int32_t *d_sel, int mode) {
  const bool aligned = mode == RMSF_PUSH_ALIGN_SUM || mode == RMSF_PUSH_ALIGN_WELFORD;
  const bool welford = mode == RMSF_PUSH_WELFORD || mode == RMSF_PUSH_ALIGN_WELFORD;
  CX_OK(flush_fold(c));  // the workspace is about to be rewritten
  if (c->exact && mode == RMSF_PUSH_WELFORD) mode = RMSF_PUSH_EXACT;  // the sequential Welford
  if (c->exact && mode != RMSF_PUSH_EXACT) return process_exact(c, d_xyz, stride, n_frames, d_sel, mode);
  if (mode == RMSF_PUSH_EXACT) {
    // RMSF.py:137-138 as written, continuing the running state at k = n (a
    // reset state has n = 0: the kernel starts from zeros); the recurrence
    // updates (mean, sumsquares) in place, nothing to fold
    Running &r = c->wel;
    const size_t row = sizeof(double) * c->n_coord;
    CX_OK(r.parts0.ensure(row, c->stream, true));
    CX_OK(r.parts1.ensure(row, c->stream, true));
    const size_t wb = rmsf_welford_sequential_workspace_bytes(n_frames);
    CX_OK(c->seqwork.ensure(std::max<size_t>(wb, 16), c->stream));
    CX_OK(timed(c, RMSF_TIME_ACCUMULATE, c->n_sel * n_frames, [&] {
      return rmsf_welford_sequential(d_xyz, stride, n_frames, c->n_sel, d_sel, r.n, r.parts0.d(), r.parts1.d(),
                                     c->seqwork.p, c->seqwork.bytes, c->stream);
    }));
    r.n += n_frames;
    r.stale = false;
    c->wel_aligned = false;
    c->rmsf_valid = false;
    c->merged_away = false;
    return RMSF_OK;
  }
  const double *xf = nullptr;
  if (aligned) {
    if (!c->ref_set) return fail(RMSF_EINVAL, "rmsf_push: aligned mode before a reference was set");
    CX_OK(c->xform.ensure(sizeof(double) * RMSF_XFORM_DOUBLES * (size_t)n_frames, c->stream));
    const size_t wb = rmsf_superpose_workspace_bytes(c->n_sel, n_frames);
    CX_OK(c->work.ensure(std::max<size_t>(wb, 8), c->stream));
    CX_OK(timed(c, RMSF_TIME_SUPERPOSE, c->n_sel * n_frames, [&] {
      return rmsf_superpose(d_xyz, stride, n_frames, c->n_sel, d_sel, c->d_masses(), c->ref.d(), c->refinfo.d(),
                            c->xform.d(), c->work.p, c->work.bytes, c->stream);
    }));
    xf = c->xform.d();
  }
  if (aligned && welford && c->collect_rmsd) {
    // the rmsd RMSF.py:48 discards: element 12 of each frame's transform record
    // grown geometrically: one reallocation (and stream sync) per doubling,
    // not per batch
    const size_t need = sizeof(double) * (size_t)(c->n_rmsd + n_frames);
    CX_OK(c->rmsd.ensure(need > c->rmsd.bytes ? std::max(need, 2 * c->rmsd.bytes) : need, c->stream, true));
    CX_HIP(hipMemcpy2DAsync(c->rmsd.d() + c->n_rmsd, sizeof(double), c->xform.d() + 12,
                            sizeof(double) * RMSF_XFORM_DOUBLES, sizeof(double), (size_t)n_frames,
                            hipMemcpyDeviceToDevice, c->stream));
    c->n_rmsd += n_frames;
  }
  Running &r = welford ? c->wel : c->sum;
  const int mode_k = welford ? RMSF_MODE_WELFORD : RMSF_MODE_SUM;
  // balanced grid: equal (lane chunk, frame) ranges per workgroup, folded in
  // frame order into the running slot 0
  const size_t wb = rmsf_accumulate_balanced_workspace_bytes(c->n_sel, n_frames, 0);
  CX_OK(c->accwork.ensure(std::max<size_t>(wb, 16), c->stream));
  CX_OK(timed(c, RMSF_TIME_ACCUMULATE, c->n_sel * n_frames, [&] {
    return rmsf_accumulate_balanced(d_xyz, stride, n_frames, c->n_sel, d_sel, xf,
                                    aligned ? c->refinfo.d() : nullptr, mode_k, 0, c->accwork.p, c->accwork.bytes,
                                    c->stream);
  }));
  c->pend.on = true;
  c->pend.welford = welford;
  c->pend.mode_k = mode_k;
  c->pend.acc_n = r.n;
  r.n += n_frames;
  r.stale = false;  // the (deferred) fold with acc_n = 0 overwrites the state
  if (welford) {
    c->wel_aligned = aligned;
    c->rmsf_valid = false;
    c->merged_away = false;
  }
  return RMSF_OK;
}

// a recorded slab push that no slab merge consumed runs whole
int flush_slab(rmsf_ctx *c) {
  if (!c->slab.on) return RMSF_OK;
  c->slab.on = false;
  return process(c, c->slab.d, c->slab.stride, c->slab.n_frames, c->d_sel(), RMSF_PUSH_WELFORD);
}

// everything queued for the running state is in it
int settle(rmsf_ctx *c) {
  CX_OK(flush_slab(c));
  return flush_fold(c);
}

// order the side stream after everything queued on the context stream so far
int side_begin(rmsf_ctx *c) {
  if (!c->side || !c->ev_main) CX_OK(on_device(c, "the side stream / its event"));
  if (!c->side) CX_HIP(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
  if (!c->ev_main) CX_HIP(hipEventCreateWithFlags(&c->ev_main, hipEventDisableTiming));
  CX_HIP(hipEventRecord(c->ev_main, c->stream));
  CX_HIP(hipStreamWaitEvent(c->side, c->ev_main, 0));
  return RMSF_OK;
}

// queue, on the side stream (after side_begin), the digest of a reference
// (which = 0) or merge shift frame (1), its copy to pinned host memory and an
// event after them
int digest_into(rmsf_ctx *c, int which, const void *a, bool words32, int64_t n, const void *info, int64_t n_info) {
  DevBuf &out = which ? c->shiftdig : c->refdig;
  CX_OK(out.ensure(sizeof(unsigned long long), c->side));
  if (!c->h_dig[which]) {
    void *h = nullptr;
    CX_HIP(hipHostMalloc(&h, sizeof(unsigned long long), hipHostMallocDefault));
    c->h_dig[which] = static_cast<unsigned long long *>(h);
  }
  if (!c->ev_dig[which]) {
    CX_OK(on_device(c, "a digest event"));
    CX_HIP(hipEventCreateWithFlags(&c->ev_dig[which], hipEventDisableTiming));
  }
  CX_HIP(hipMemsetAsync(out.p, 0, sizeof(unsigned long long), c->side));
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(256, (n + n_info + 1023) / 1024));
  auto *o = static_cast<unsigned long long *>(out.p);
  auto *in = static_cast<const uint64_t *>(info);
  if (words32)
    hipLaunchKernelGGL(k_digest<uint32_t>, dim3(blocks), dim3(256), 0, c->side, static_cast<const uint32_t *>(a), n,
                       in, n_info, o);
  else
    hipLaunchKernelGGL(k_digest<uint64_t>, dim3(blocks), dim3(256), 0, c->side, static_cast<const uint64_t *>(a), n,
                       in, n_info, o);
  CX_HIP(hipGetLastError());
  CX_HIP(hipMemcpyAsync(c->h_dig[which], out.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->side));
  CX_HIP(hipEventRecord(c->ev_dig[which], c->side));
  return RMSF_OK;
}

// queue the digest of the context's current reference (after every setter):
// the centred reference and its COM, what the shifted merge uses as its shift
int digest_reference(rmsf_ctx *c) {
  CX_OK(side_begin(c));
  return digest_into(c, 0, c->ref.p, false, c->n_coord, c->refinfo.p, 3);
}

// the merge shift frame's gather (selected rows of device frame d, f32) and
// digest on the side stream, whose ordering the caller set up (side_begin)
int shift_frame_on_side(rmsf_ctx *c, const float *d) {
  if (!c->shift.p) CX_OK(c->shift.ensure(sizeof(float) * c->n_coord, c->side));
  if (!c->zidx_set) {
    CX_OK(c->zidx.ensure(sizeof(int64_t), c->side));
    CX_HIP(hipMemsetAsync(c->zidx.p, 0, sizeof(int64_t), c->side));
    c->zidx_set = true;
  }
  CX_OK(rmsf_gather_frames(d, 3 * c->n_atoms, static_cast<const int64_t *>(c->zidx.p), 1, c->n_sel, c->d_sel(),
                           static_cast<float *>(c->shift.p), c->side));
  c->shift_set = true;
  return digest_into(c, 1, c->shift.p, true, c->n_coord, nullptr, 0);
}

// true when every context holds a reference (shift = false) or a merge shift
// frame (shift = true) with the same digest; waits for the digests only
int same_digests(rmsf_ctx **cs, int n, bool shift, bool *same) {
  *same = true;
  unsigned long long d0 = 0;
  const int w = shift ? 1 : 0;
  for (int i = 0; i < n; ++i) {
    const bool set = shift ? cs[i]->shift_set : cs[i]->ref_set;
    if (!set || !cs[i]->ev_dig[w]) {
      *same = false;
      return RMSF_OK;
    }
    DeviceScope ds(cs[i]->dev);
    CX_HIP(hipEventSynchronize(cs[i]->ev_dig[w]));
    const unsigned long long d = *cs[i]->h_dig[w];
    if (i == 0) d0 = d;
    else if (d != d0) *same = false;
  }
  return RMSF_OK;
}

int check_mode(int mode, const char *fn) {
  if (mode < RMSF_PUSH_WELFORD || mode > RMSF_PUSH_EXACT) return fail(RMSF_EINVAL, std::string(fn) + ": bad mode");
  return RMSF_OK;
}

int ensure_stager(rmsf_ctx *c) {
  if (c->stager && !c->stager_dirty) return RMSF_OK;
  if (c->stager) {
    CX_OK(rmsf_stager_destroy(c->stager));
    c->stager = nullptr;
  }
  int64_t batch = c->stage_batch;
  if (batch <= 0) batch = std::max<int64_t>(1, std::min<int64_t>(4096, kStageBytes / (12 * std::max<int64_t>(1, c->n_sel))));
  CX_OK(rmsf_stager_create(c->n_atoms, c->n_sel, c->h_sel.empty() ? nullptr : c->h_sel.data(), batch, c->stage_slots,
                           c->stage_threads, &c->stager));
  c->stage_batch = batch;
  c->stager_dirty = false;
  return RMSF_OK;
}

// fn(i) for every context, one host thread per DEVICE: the contexts of one
// device run in context order on one thread (the worker of the device's
// first context; context 0's device on the calling thread) -- they share that
// device's queues, so more threads would only contend for them -- and the
// devices' threads run at once, so N devices start their work together
// instead of one after another behind a single thread's launch latency.  The
// first failure (in context order) is reported on the calling thread.
int for_each_ctx(rmsf_ctx **cs, int n, const std::function<int(int)> &fn) {
  if (n == 1) return fn(0);
  std::vector<std::vector<int>> groups;  // per device, in order of first appearance
  std::vector<int> gdev;
  for (int i = 0; i < n; ++i) {
    size_t g = 0;
    while (g < gdev.size() && gdev[g] != cs[i]->dev) ++g;
    if (g == gdev.size()) {
      gdev.push_back(cs[i]->dev);
      groups.emplace_back();
    }
    groups[g].push_back(i);
  }
  std::vector<int> rcs(n, RMSF_OK);
  std::vector<std::string> msgs(n);
  auto run_group = [&](const std::vector<int> &grp) -> int {
    for (int i : grp) {
      rcs[i] = fn(i);
      if (rcs[i] != RMSF_OK) {
        msgs[i] = rmsf_last_error();
        return rcs[i];
      }
    }
    return RMSF_OK;
  };
  // every worker exists before any job is posted: a job must never outlive
  // this frame (it refers to fn and the vectors above)
  for (size_t g = 1; g < groups.size(); ++g) {
    rmsf_ctx *c = cs[groups[g][0]];
    if (!c->worker) c->worker = new (std::nothrow) Worker;
    if (!c->worker) return fail(RMSF_ENOMEM, "rmsf_multi: cannot start a worker thread");
  }
  for (size_t g = 1; g < groups.size(); ++g)
    cs[groups[g][0]]->worker->post([&run_group, &groups, g] { return run_group(groups[g]); });
  run_group(groups[0]);
  for (size_t g = 1; g < groups.size(); ++g) {
    std::string e;
    (void)cs[groups[g][0]]->worker->wait(&e);
  }
  for (int i = 0; i < n; ++i)
    if (rcs[i] != RMSF_OK) return fail(rcs[i], msgs[i]);
  return RMSF_OK;
}

// ---- cross-rank exchange ----------------------------------------------------
// reduce(count, bufs, root): sum bufs[i][0..count) over all ranks, in place,
// for the n local contexts (each buffer on its context's stream); root >= 0:
// only that rank's buffer must hold the sum afterwards.
using Reduce = std::function<int(int64_t, double *const *, int)>;

// The contexts of this process are every rank of the exchange (RCCL
// communicators of size n from rmsf_multi_init_all, or no communicator at
// all): the frame counts are all known on the host, no device exchange needed.
bool whole_group_here(rmsf_ctx *const *cs, int n) {
  for (int i = 0; i < n; ++i)
    if (cs[i]->comm ? cs[i]->comm_size != n : false) return false;
  return true;
}

int count_exchange(rmsf_ctx **cs, int n, const Reduce &red, const std::vector<int64_t> &local, int64_t *total,
                   bool host_counts) {
  if (host_counts) {
    int64_t t = 0;
    for (int64_t v : local) t += v;
    *total = t;
    return RMSF_OK;
  }
  std::vector<double *> bufs(n);
  for (int i = 0; i < n; ++i) {
    DeviceScope ds(cs[i]->dev);
    CX_OK(cs[i]->cnt.ensure(sizeof(double), cs[i]->stream));
    double v = (double)local[i];
    CX_HIP(hipMemcpyAsync(cs[i]->cnt.p, &v, sizeof(double), hipMemcpyHostToDevice, cs[i]->stream));
    CX_HIP(hipStreamSynchronize(cs[i]->stream));
    bufs[i] = cs[i]->cnt.d();
  }
  CX_OK(red(1, bufs.data(), -1));
  double t = 0.0;
  for (int i = 0; i < n; ++i) {
    DeviceScope ds(cs[i]->dev);
    double v = 0.0;
    CX_HIP(hipMemcpyAsync(&v, cs[i]->cnt.p, sizeof(double), hipMemcpyDeviceToHost, cs[i]->stream));
    CX_HIP(hipStreamSynchronize(cs[i]->stream));
    if (i == 0) t = v;
    else if (v != t) return fail(RMSF_EINVAL, "exchange: ranks disagree on the frame count");
  }
  *total = (int64_t)t;
  return RMSF_OK;
}

int exchange_sum(rmsf_ctx **cs, int n, const Reduce &red, bool host_counts) {
  std::vector<int64_t> local(n);
  for (int i = 0; i < n; ++i) {
    DeviceScope ds(cs[i]->dev);
    CX_OK(settle(cs[i]));
    CX_OK(ensure_zeroed(cs[i], cs[i]->sum, false));
    local[i] = cs[i]->sum.n;
  }
  int64_t total = 0;
  CX_OK(count_exchange(cs, n, red, local, &total, host_counts));
  std::vector<double *> bufs(n);
  for (int i = 0; i < n; ++i) bufs[i] = cs[i]->sum.parts0.d();
  CX_OK(red(cs[0]->n_coord, bufs.data(), -1));
  for (int i = 0; i < n; ++i) cs[i]->sum.n = total;
  return RMSF_OK;
}

int exchange_chan(rmsf_ctx **cs, int n, const Reduce &red, bool host_counts) {
  std::vector<int64_t> local(n);
  for (int i = 0; i < n; ++i) {
    DeviceScope ds(cs[i]->dev);
    CX_OK(settle(cs[i]));
    CX_OK(ensure_zeroed(cs[i], cs[i]->wel, true));
    local[i] = cs[i]->wel.n;
  }
  int64_t total = 0;
  CX_OK(count_exchange(cs, n, red, local, &total, host_counts));
  if (total == 0) return fail(RMSF_EEMPTY, "rmsf chan merge: no frames on any rank (RMSF.py:39 ZeroDivisionError)");
  const int64_t nc = cs[0]->n_coord;
  std::vector<double *> a(n), b(n);
  // step 1: global mean = sum_k (n_k/n) mean_k
  for (int i = 0; i < n; ++i) {
    rmsf_ctx *c = cs[i];
    DeviceScope ds(c->dev);
    CX_OK(c->xa.ensure(sizeof(double) * nc, c->stream));
    CX_OK(c->xb.ensure(sizeof(double) * nc, c->stream));
    CX_OK(merge_open(c, c->stream));
    CX_OK(rmsf_chan_weight(c->wel.parts0.d(), (double)local[i] / (double)total, nc, c->xa.d(), c->stream));
    a[i] = c->xa.d();
    b[i] = c->xb.d();
  }
  CX_OK(red(nc, a.data(), -1));
  // step 2: global M2 = sum_k M2_k + n_k (mean_k - mean)^2
  for (int i = 0; i < n; ++i) {
    rmsf_ctx *c = cs[i];
    DeviceScope ds(c->dev);
    CX_OK(rmsf_chan_deviation(c->wel.parts0.d(), c->wel.parts1.d(), c->xa.d(), (double)local[i], nc, c->xb.d(),
                              c->stream));
  }
  CX_OK(red(nc, b.data(), -1));
  for (int i = 0; i < n; ++i) {
    rmsf_ctx *c = cs[i];
    DeviceScope ds(c->dev);
    CX_HIP(hipMemcpyAsync(c->wel.parts0.p, c->xa.p, sizeof(double) * nc, hipMemcpyDeviceToDevice, c->stream));
    CX_HIP(hipMemcpyAsync(c->wel.parts1.p, c->xb.p, sizeof(double) * nc, hipMemcpyDeviceToDevice, c->stream));
    c->wel.n = total;
    c->rmsf_valid = false;
    CX_OK(merge_close(c, c->stream));
  }
  return RMSF_OK;
}

// What the one-collective merge shifts the moments by: the contexts' common
// reference structure (centred reference + its COM), which every rank of
// RMSF.py holds identically (the frame-0 reference, RMSF.py:80-87, or the
// average, :113-118), or -- unaligned Welford state -- a common merge shift
// frame (rmsf_set_merge_shift_frame: frame 0 of the frame list, f32).
enum class Shift { REF, FRAME };

struct ShiftArgs {
  const void *p;
  int f32;
  const double *off3;
};

ShiftArgs shift_of(rmsf_ctx *c, Shift kind) {
  if (kind == Shift::REF) return {c->ref.p, 0, c->refinfo.d()};
  return {c->shift.p, 1, nullptr};
}

// The k-way Chan merge in ONE data collective (rmsf_chan_shift_pack/_finish):
// T1 = sum n_k (mean_k - c), T2 = sum M2_k + n_k (mean_k - c)^2 about the
// common shift c.  A context whose last fold is still deferred folds and
// packs in one launch (rmsf_fold_balanced_shift).  root >= 0: a reduce to
// that context (RMSF.py:143); the others are left `merged_away`.  The caller
// guarantees that every context holds the same shift.
int exchange_chan_shifted(rmsf_ctx **cs, int n, const Reduce &red, bool host_counts, Shift kind, int root) {
  std::vector<int64_t> local(n);
  for (int i = 0; i < n; ++i) {
    if (kind == Shift::REF && !cs[i]->ref_set)
      return fail(RMSF_EINVAL, "rmsf shifted chan merge: a context holds no reference");
    if (kind == Shift::FRAME && !cs[i]->shift_set)
      return fail(RMSF_EINVAL, "rmsf shifted chan merge: a context holds no merge shift frame");
    DeviceScope ds(cs[i]->dev);
    CX_OK(flush_slab(cs[i]));
    if (!(cs[i]->pend.on && cs[i]->pend.welford)) {
      CX_OK(flush_fold(cs[i]));
      CX_OK(ensure_zeroed(cs[i], cs[i]->wel, true));
    }
    local[i] = cs[i]->wel.n;
  }
  int64_t total = 0;
  CX_OK(count_exchange(cs, n, red, local, &total, host_counts));
  if (total == 0) return fail(RMSF_EEMPTY, "rmsf chan merge: no frames on any rank (RMSF.py:39 ZeroDivisionError)");
  const int64_t nc = cs[0]->n_coord;
  std::vector<double *> t(n);
  // each context's pack (and below its finish) from its device's host thread:
  // with one device per context the launches leave in parallel
  CX_OK(for_each_ctx(cs, n, [&](int i) -> int {
    rmsf_ctx *c = cs[i];
    DeviceScope ds(c->dev);
    const ShiftArgs sh = shift_of(c, kind);
    CX_OK(c->xa.ensure(sizeof(double) * 2 * nc, c->stream));
    if (kind == Shift::FRAME) CX_HIP(hipStreamWaitEvent(c->stream, c->ev_dig[1], 0));  // the side gather
    if (c->pend.on && c->pend.welford) {  // fold + pack, one launch
      c->pend.on = false;
      CX_OK(rmsf_fold_balanced_shift(c->accwork.p, nc, c->pend.acc_n, c->wel.parts0.d(), c->wel.parts1.d(), sh.p,
                                     sh.f32, sh.off3, c->xa.d(), c->stream));
    } else {
      CX_OK(rmsf_chan_shift_pack(c->wel.parts0.d(), c->wel.parts1.d(), sh.p, sh.f32, sh.off3, (double)local[i], nc,
                                 c->xa.d(), c->stream));
    }
    t[i] = c->xa.d();
    return merge_open(c, c->stream);
  }));
  CX_OK(red(2 * nc, t.data(), root));
  return for_each_ctx(cs, n, [&](int i) -> int {
    rmsf_ctx *c = cs[i];
    DeviceScope ds(c->dev);
    if (root >= 0 && i != root) {
      c->merged_away = true;
      c->rmsf_valid = false;
      return merge_close(c, c->stream);  // its part of the reduce was queued on its stream
    }
    const ShiftArgs sh = shift_of(c, kind);
    CX_OK(c->rmsf.ensure(sizeof(double) * c->n_sel, c->stream));
    CX_OK(rmsf_chan_shift_finish(c->xa.d(), sh.p, sh.f32, sh.off3, c->n_sel, total, c->wel.parts0.d(),
                                 c->wel.parts1.d(), c->rmsf.d(), c->stream));
    c->wel.n = total;
    c->rmsf_valid = true;
    c->merged_away = false;
    return merge_close(c, c->stream);
  });
}

Reduce callback_reduce(rmsf_ctx *c, rmsf_allreduce_fn fn, void *user) {
  return [c, fn, user](int64_t count, double *const *bufs, int) -> int {
    DeviceScope ds(c->dev);
    int rc = fn(bufs[0], count, (void *)c->stream, user);
    if (rc != 0) return fail(RMSF_EINVAL, "allreduce callback returned " + std::to_string(rc));
    return RMSF_OK;
  };
}

// one RCCL collective per context on `streams[i]` (the context streams, or
// the slab merge's comm streams), grouped: one thread drives every device
int rccl_collective(rmsf_ctx **cs, int n, int64_t count, double *const *bufs, int root, const hipStream_t *streams) {
  const Rccl &r = rccl();
  ncclResult_t e = r.GroupStart();
  if (e != ncclSuccess) return nccl_fail("ncclGroupStart", e);
  for (int i = 0; i < n; ++i) {
    DeviceScope ds(cs[i]->dev);
    e = root < 0 ? r.AllReduce(bufs[i], bufs[i], (size_t)count, ncclFloat64, ncclSum, cs[i]->comm, streams[i])
                 : r.Reduce(bufs[i], bufs[i], (size_t)count, ncclFloat64, ncclSum, root, cs[i]->comm, streams[i]);
    if (e != ncclSuccess) {
      (void)r.GroupEnd();
      return nccl_fail(root < 0 ? "ncclAllReduce" : "ncclReduce", e);
    }
  }
  e = r.GroupEnd();
  if (e != ncclSuccess) return nccl_fail("ncclGroupEnd", e);
  return RMSF_OK;
}

Reduce rccl_reduce(rmsf_ctx **cs, int n) {
  return [cs, n](int64_t count, double *const *bufs, int root) -> int {
    std::vector<hipStream_t> st(n);
    for (int i = 0; i < n; ++i) st[i] = cs[i]->stream;
    return rccl_collective(cs, n, count, bufs, root, st.data());
  };
}

// contexts of one process, no communicator: fold on the host in context order
Reduce local_reduce(rmsf_ctx **cs, int n) {
  return [cs, n](int64_t count, double *const *bufs, int root) -> int {
    std::vector<double> acc((size_t)count, 0.0), tmp((size_t)count);
    for (int i = 0; i < n; ++i) {
      DeviceScope ds(cs[i]->dev);
      CX_HIP(hipMemcpyAsync(tmp.data(), bufs[i], sizeof(double) * count, hipMemcpyDeviceToHost, cs[i]->stream));
      CX_HIP(hipStreamSynchronize(cs[i]->stream));
      for (int64_t j = 0; j < count; ++j) acc[j] += tmp[j];
    }
    for (int i = 0; i < n; ++i) {
      if (root >= 0 && i != root) continue;
      DeviceScope ds(cs[i]->dev);
      CX_HIP(hipMemcpyAsync(bufs[i], acc.data(), sizeof(double) * count, hipMemcpyHostToDevice, cs[i]->stream));
      CX_HIP(hipStreamSynchronize(cs[i]->stream));
    }
    return RMSF_OK;
  };
}

// timing rehearsal (RMSF_TRANSPORT_NOOP): the exchanges move nothing
Reduce noop_reduce() {
  return [](int64_t, double *const *, int) -> int { return RMSF_OK; };
}

int multi_reduce(rmsf_ctx **cs, int n, const char *fn, Reduce *out, int *kind = nullptr) {
  if (!cs || n <= 0) return fail(RMSF_EINVAL, std::string(fn) + ": no contexts");
  int with = 0, noop = 0;
  for (int i = 0; i < n; ++i) {
    CX_OK(check_ctx(cs[i], fn));
    if (cs[i]->n_coord != cs[0]->n_coord) return fail(RMSF_EINVAL, std::string(fn) + ": contexts differ in n_sel");
    for (int j = 0; j < i; ++j)
      if (cs[j] == cs[i]) return fail(RMSF_EINVAL, std::string(fn) + ": a context is listed twice");
    with += cs[i]->comm != nullptr;
    noop += cs[i]->transport == RMSF_TRANSPORT_NOOP;
  }
  if (noop && noop != n) return fail(RMSF_EINVAL, std::string(fn) + ": mixed transports");
  int k = 0;
  if (noop) {
    *out = noop_reduce();
    k = 2;
  } else if (with == n) {
    *out = rccl_reduce(cs, n);
    k = 1;
  } else if (with == 0) {
    *out = local_reduce(cs, n);
  } else {
    return fail(RMSF_EINVAL, std::string(fn) + ": some contexts have an RCCL communicator and some do not");
  }
  if (kind) *kind = k;
  return RMSF_OK;
}

// k atom slabs of a flat plan's chunks, cut at multiples of 3 chunks (3 x 1024
// coordinates = whole atoms) -- pipeline._slab_bounds
std::vector<std::pair<int64_t, int64_t>> slab_bounds(int64_t n_chunks, int k) {
  std::vector<int64_t> cuts;
  for (int i = 1; i < k; ++i) {
    double x = (double)i * (double)n_chunks / k / 3.0;
    int64_t c = 3 * (int64_t)std::nearbyint(x);
    c = std::min(n_chunks, std::max<int64_t>(0, c));
    if (c > 0 && c < n_chunks && (cuts.empty() || cuts.back() != c)) cuts.push_back(c);
  }
  std::sort(cuts.begin(), cuts.end());
  cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
  std::vector<std::pair<int64_t, int64_t>> out;
  int64_t lo = 0;
  for (int64_t c : cuts) {
    out.push_back({lo, c});
    lo = c;
  }
  out.push_back({lo, n_chunks});
  return out;
}

// The recorded slab pushes of every context and the merge, slab by slab
// (pipeline._slab_sweep): slab s's accumulate + fold-pack on each context
// stream, then its collective -- RCCL: on the context's comm stream after an
// event, so slab s+1 streams while slab s's reduce runs; host transports: in
// turn -- and the finish of every slab.  Bit-identical per rank to the
// unslabbed fold + pack (every slab replays the whole plan's segments).
int slab_merge(rmsf_ctx **cs, int n, int kind, const Reduce &red, int root) {
  const int64_t nc = cs[0]->n_coord;
  const auto bounds = slab_bounds(cs[0]->slab.chunks, cs[0]->slab.k);
  const size_t ns = bounds.size();
  int64_t total = 0;
  for (int i = 0; i < n; ++i) total += cs[i]->wel.n + cs[i]->slab.n_frames;
  if (total == 0) return fail(RMSF_EEMPTY, "rmsf chan merge: no frames on any rank (RMSF.py:39 ZeroDivisionError)");
  const bool rc_l = kind == 1;
  CX_OK(for_each_ctx(cs, n, [&](int i) -> int {
    rmsf_ctx *c = cs[i];
    DeviceScope ds(c->dev);
    CX_OK(flush_fold(c));
    CX_OK(ensure_zeroed(c, c->wel, true));
    const auto sp = c->slab;
    c->slab.on = false;
    const size_t wb = rmsf_accumulate_balanced_workspace_bytes(c->n_sel, sp.n_frames, 0);
    CX_OK(c->accwork.ensure(std::max<size_t>(wb, 16), c->stream));
    CX_OK(c->xa.ensure(sizeof(double) * 2 * nc, c->stream));
    if (rc_l) {
      if (!c->comm_stream) {
        CX_OK(on_device(c, "the slab merge's stream"));
        CX_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
      }
      if (c->ev_pack.size() < ns) CX_OK(on_device(c, "the slab merge's events"));
      while (c->ev_pack.size() < ns) {
        hipEvent_t a = nullptr, b = nullptr;
        CX_HIP(hipEventCreateWithFlags(&a, hipEventDisableTiming));
        CX_HIP(hipEventCreateWithFlags(&b, hipEventDisableTiming));
        c->ev_pack.push_back(a);
        c->ev_done.push_back(b);
      }
    }
    for (size_t s = 0; s < ns; ++s) {
      const int64_t c0 = bounds[s].first, c1 = bounds[s].second;
      const int64_t j0 = 1024 * c0, j1 = std::min(1024 * c1, nc);
      CX_OK(timed(c, RMSF_TIME_ACCUMULATE, sp.n_frames * (j1 - j0) / 3, [&] {
        return rmsf_accumulate_balanced_slab(sp.d, sp.stride, sp.n_frames, c->n_sel, c0, c1, c->accwork.p,
                                             c->accwork.bytes, c->stream);
      }));
      if (s == 0) CX_HIP(hipStreamWaitEvent(c->stream, c->ev_dig[1], 0));  // the side gather, before the first pack
      CX_OK(rmsf_fold_balanced_shift_slab(c->accwork.p, nc, c->wel.n, c->wel.parts0.d(), c->wel.parts1.d(),
                                          c->shift.p, 1, nullptr, c->xa.d() + 2 * j0, c0, c1, c->stream));
      if (rc_l) CX_HIP(hipEventRecord(c->ev_pack[s], c->stream));
    }
    c->wel.n += sp.n_frames;
    c->wel.stale = false;
    c->wel_aligned = false;
    return merge_open(c, c->stream);  // the exposed part: after the last slab's pack
  }));
  std::vector<double *> bufs(n);
  std::vector<hipStream_t> st(n);
  for (size_t s = 0; s < ns; ++s) {
    const int64_t j0 = 1024 * bounds[s].first, j1 = std::min(1024 * bounds[s].second, nc);
    for (int i = 0; i < n; ++i) {
      bufs[i] = cs[i]->xa.d() + 2 * j0;
      st[i] = cs[i]->comm_stream;
      if (rc_l) {
        DeviceScope ds(cs[i]->dev);
        CX_HIP(hipStreamWaitEvent(cs[i]->comm_stream, cs[i]->ev_pack[s], 0));
      }
    }
    if (rc_l) {
      CX_OK(rccl_collective(cs, n, 2 * (j1 - j0), bufs.data(), root, st.data()));
      for (int i = 0; i < n; ++i) {
        DeviceScope ds(cs[i]->dev);
        CX_HIP(hipEventRecord(cs[i]->ev_done[s], cs[i]->comm_stream));
      }
    } else {
      CX_OK(red(2 * (j1 - j0), bufs.data(), root));
    }
  }
  for (int i = 0; i < n; ++i) {
    rmsf_ctx *c = cs[i];
    DeviceScope ds(c->dev);
    if (root >= 0 && i != root) {
      c->merged_away = true;
      c->rmsf_valid = false;
      CX_OK(merge_close(c, rc_l ? c->comm_stream : c->stream));  // after its last slab's collective
      continue;
    }
    CX_OK(c->rmsf.ensure(sizeof(double) * c->n_sel, c->stream));
    for (size_t s = 0; s < ns; ++s) {
      const int64_t j0 = 1024 * bounds[s].first, j1 = std::min(1024 * bounds[s].second, nc);
      if (rc_l) CX_HIP(hipStreamWaitEvent(c->stream, c->ev_done[s], 0));
      CX_OK(rmsf_chan_shift_finish(c->xa.d() + 2 * j0, static_cast<const float *>(c->shift.p) + j0, 1, nullptr,
                                   (j1 - j0) / 3, total, c->wel.parts0.d() + j0, c->wel.parts1.d() + j0,
                                   c->rmsf.d() + j0 / 3, c->stream));
    }
    c->wel.n = total;
    c->rmsf_valid = true;
    c->merged_away = false;
    CX_OK(merge_close(c, c->stream));
  }
  return RMSF_OK;
}

// RMSF.py:141-143 with second_order_moments' own arithmetic over contexts of
// this process (each holding a rank's S of RMSF.py:140, e.g. from
// RMSF_PUSH_EXACT), device to device: the reduction schedule of `order`
// (rmsf_chan_reduce_steps) run as mpi4py runs it -- for each step
// S[dst] = op(S[dst], S[src]), src's state is copied to dst's device
// (hipMemcpyPeerAsync on dst's stream, after an event on src's stream; xGMI
// between devices, a device copy on one) and merged there by
// rmsf_chan_merge_pair.  The tree's steps at one level run on different
// streams concurrently.  The result lands in context 0, then goes to `root`
// (root >= 0, as mpi4py forwards 0's result to root; the others are left
// merged_away) or to every context (root = -1).
int ensure_event(const rmsf_ctx *c, hipEvent_t *e) {
  if (!*e) {
    CX_OK(on_device(c, "an exact-merge event"));
    CX_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  return RMSF_OK;
}

// d's device may read s's memory directly (xGMI peer mapping) where the
// platform allows; otherwise hipMemcpyPeerAsync stages the copy itself
void enable_peer(int dev, int peer) {
  if (dev == peer) return;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, dev, peer) != hipSuccess || !can) return;
  DeviceScope ds(dev);
  if (hipDeviceEnablePeerAccess(peer, 0) != hipSuccess) (void)hipGetLastError();  // already enabled: fine
}

// d's stream copies s's Welford state (mean, M2) into d->xb after s's queued
// work; s's stream then waits for that copy, so nothing s does next (a reset,
// a push, its destruction's drain) can overwrite or free the state while the
// peer copy is in flight -- rmsf_ctx_synchronize(s) then covers the read too
int pull_state(rmsf_ctx *d, rmsf_ctx *s, int64_t nc) {
  enable_peer(d->dev, s->dev);
  {
    DeviceScope ds(s->dev);
    CX_OK(ensure_event(s, &s->ev_sent));
    CX_HIP(hipEventRecord(s->ev_sent, s->stream));
  }
  {
    DeviceScope dd(d->dev);
    CX_OK(d->xb.ensure(sizeof(double) * 2 * nc, d->stream));
    CX_HIP(hipStreamWaitEvent(d->stream, s->ev_sent, 0));
    const size_t row = sizeof(double) * nc;
    CX_HIP(hipMemcpyPeerAsync(d->xb.p, d->dev, s->wel.parts0.p, s->dev, row, d->stream));
    CX_HIP(hipMemcpyPeerAsync(d->xb.d() + nc, d->dev, s->wel.parts1.p, s->dev, row, d->stream));
    CX_OK(ensure_event(d, &d->ev_pulled));
    CX_HIP(hipEventRecord(d->ev_pulled, d->stream));
  }
  DeviceScope ds(s->dev);
  CX_HIP(hipStreamWaitEvent(s->stream, d->ev_pulled, 0));  // the wait binds this record (reuse is safe)
  return RMSF_OK;
}

int exact_merge(rmsf_ctx **cs, int n, int root, int order) {
  std::vector<int64_t> cnt(n);
  for (int i = 0; i < n; ++i) {
    DeviceScope ds(cs[i]->dev);
    CX_OK(settle(cs[i]));
    CX_OK(ensure_zeroed(cs[i], cs[i]->wel, true));
    cnt[i] = cs[i]->wel.n;
  }
  int64_t total = 0;
  for (int64_t v : cnt) total += v;
  if (total == 0) return fail(RMSF_EEMPTY, "rmsf exact merge: no frames on any rank (RMSF.py:39 ZeroDivisionError)");
  const int64_t nc = cs[0]->n_coord;
  for (int i = 0; i < n; ++i) {
    DeviceScope ds(cs[i]->dev);
    CX_OK(merge_open(cs[i], cs[i]->stream));
  }
  const int ns = rmsf_chan_reduce_steps(n, order, nullptr, nullptr, 0);
  if (ns < 0) return ns;
  std::vector<int> dst(std::max(ns, 1)), src(std::max(ns, 1));
  if (ns > 0) CX_OK(rmsf_chan_reduce_steps(n, order, dst.data(), src.data(), ns) < 0 ? RMSF_EINVAL : RMSF_OK);
  for (int k = 0; k < ns; ++k) {
    rmsf_ctx *d = cs[dst[k]], *s = cs[src[k]];
    const int64_t n1 = cnt[dst[k]], n2 = cnt[src[k]];
    if (n1 + n2 == 0) continue;  // two empty states (where RMSF.py:39 raises): dst stays empty
    CX_OK(pull_state(d, s, nc));
    DeviceScope dd(d->dev);
    CX_OK(rmsf_chan_merge_pair(d->wel.parts0.d(), d->wel.parts1.d(), n1, d->xb.d(), d->xb.d() + nc, n2, nc,
                               d->stream));
    cnt[dst[k]] = n1 + n2;
  }
  // S[0] is comm.reduce's result; forward it as mpi4py forwards rank 0's
  for (int i = 0; i < n; ++i) {
    rmsf_ctx *c = cs[i];
    if (i != 0 && root >= 0 && i != root) {
      c->merged_away = true;
      c->rmsf_valid = false;
      continue;
    }
    if (i != 0) {
      CX_OK(pull_state(c, cs[0], nc));
      DeviceScope dc(c->dev);
      CX_HIP(hipMemcpyAsync(c->wel.parts0.p, c->xb.p, sizeof(double) * nc, hipMemcpyDeviceToDevice, c->stream));
      CX_HIP(hipMemcpyAsync(c->wel.parts1.p, c->xb.d() + nc, sizeof(double) * nc, hipMemcpyDeviceToDevice,
                            c->stream));
    }
    c->wel.n = total;
    c->wel_aligned = false;
    c->rmsf_valid = false;
    c->merged_away = false;
  }
  if (root > 0) {  // rank 0 only sent its result on
    cs[0]->merged_away = true;
    cs[0]->rmsf_valid = false;
  }
  for (int i = 0; i < n; ++i) {
    DeviceScope ds(cs[i]->dev);
    CX_OK(merge_close(cs[i], cs[i]->stream));
  }
  return RMSF_OK;
}

}  // namespace

// ============================================================================
extern "C" {

RMSF_EXPORT int rmsf_ctx_create(int device, int64_t n_atoms, int64_t n_sel, const int64_t *h_sel,
                                const double *h_masses, int flags, rmsf_ctx **out) {
  if (!out) return fail(RMSF_EINVAL, "rmsf_ctx_create: out is NULL");
  *out = nullptr;
  if (flags != 0) return fail(RMSF_EINVAL, "rmsf_ctx_create: flags must be 0");
  if (n_atoms <= 0 || n_sel <= 0 || n_atoms > (int64_t)INT32_MAX)
    return fail(RMSF_EINVAL, "rmsf_ctx_create: n_atoms/n_sel must be positive (n_atoms < 2^31)");
  if (!h_sel && n_sel > n_atoms) return fail(RMSF_EINVAL, "rmsf_ctx_create: n_sel > n_atoms without a selection");
  int nd = 0;
  CX_HIP(hipGetDeviceCount(&nd));
  if (device < 0 || device >= nd) return fail(RMSF_EINVAL, "rmsf_ctx_create: no such device");
  rmsf_ctx *c = new (std::nothrow) rmsf_ctx;
  if (!c) return fail(RMSF_ENOMEM, "rmsf_ctx_create: out of host memory");
  c->dev = device;
  c->n_atoms = n_atoms;
  c->n_sel = n_sel;
  c->n_coord = 3 * n_sel;
  auto bail = [&](int rc) {
    rmsf_ctx_destroy(c);
    return rc;
  };
  if (h_sel) {
    c->h_sel.resize(n_sel);
    bool identity = true;
    for (int64_t i = 0; i < n_sel; ++i) {
      if (h_sel[i] < 0 || h_sel[i] >= n_atoms)
        return bail(fail(RMSF_EINVAL, "rmsf_ctx_create: selection index " + std::to_string(h_sel[i]) + " out of range"));
      c->h_sel[i] = (int32_t)h_sel[i];
      identity = identity && h_sel[i] == i;
    }
    if (identity) c->h_sel.clear();  // atoms 0..n_sel-1: the contiguous path
  }
  DeviceScope ds(device);
  if (ds.err != hipSuccess) return bail(fail(RMSF_EHIP, "rmsf_ctx_create: hipSetDevice failed"));
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(RMSF_EHIP, "rmsf_ctx_create: hipStreamCreate failed"));
  int rc;
  if (!c->h_sel.empty()) {
    if ((rc = c->sel.ensure(sizeof(int32_t) * n_sel, c->stream)) != RMSF_OK) return bail(rc);
    if (hipMemcpy(c->sel.p, c->h_sel.data(), sizeof(int32_t) * n_sel, hipMemcpyHostToDevice) != hipSuccess)
      return bail(fail(RMSF_EHIP, "rmsf_ctx_create: selection upload failed"));
  }
  if (h_masses) {
    c->has_masses = true;
    c->h_masses.assign(h_masses, h_masses + n_sel);
    if ((rc = c->masses.ensure(sizeof(double) * n_sel, c->stream)) != RMSF_OK) return bail(rc);
    if (hipMemcpy(c->masses.p, h_masses, sizeof(double) * n_sel, hipMemcpyHostToDevice) != hipSuccess)
      return bail(fail(RMSF_EHIP, "rmsf_ctx_create: masses upload failed"));
  }
  if ((rc = c->ref.ensure(sizeof(double) * c->n_coord, c->stream)) != RMSF_OK) return bail(rc);
  if ((rc = c->refinfo.ensure(sizeof(double) * RMSF_REFINFO_DOUBLES, c->stream)) != RMSF_OK) return bail(rc);
  if ((rc = zero_running(c, c->wel, true)) != RMSF_OK) return bail(rc);
  if ((rc = zero_running(c, c->sum, false)) != RMSF_OK) return bail(rc);
  *out = c;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_destroy(rmsf_ctx *c) {
  if (!c) return RMSF_OK;
  {
    DeviceScope ds(c->dev);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->side) (void)hipStreamSynchronize(c->side);  // digests copy into pinned memory freed below
    if (c->stager) rmsf_stager_destroy(c->stager);
    if (c->xdec) rmsf_xtcdec_destroy(c->xdec);
    delete c->worker;  // joins its thread
    c->worker = nullptr;
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    if (c->comm && rccl().ok) rccl().CommDestroy(c->comm);
    drop_spans(c, -1);
    for (hipEvent_t e : c->ev_pack) (void)hipEventDestroy(e);
    for (int w = 0; w < 2; ++w) {
      if (c->ev_dig[w]) (void)hipEventDestroy(c->ev_dig[w]);
      if (c->h_dig[w]) (void)hipHostFree(c->h_dig[w]);
    }
    for (hipEvent_t e : c->ev_done) (void)hipEventDestroy(e);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->ev_main) (void)hipEventDestroy(c->ev_main);
    if (c->ev_sent) (void)hipEventDestroy(c->ev_sent);
    if (c->ev_pulled) (void)hipEventDestroy(c->ev_pulled);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;  // DevBufs free on the context's device
  }
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_stream(rmsf_ctx *c, void **stream) {
  CX_OK(check_ctx(c, "rmsf_ctx_stream"));
  if (!stream) return fail(RMSF_EINVAL, "rmsf_ctx_stream: stream is NULL");
  *stream = (void *)c->stream;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_synchronize(rmsf_ctx *c) {
  CX_OK(check_ctx(c, "rmsf_ctx_synchronize"));
  DeviceScope ds(c->dev);
  // a push recorded for the slab merge still reads the caller's frames: it
  // runs (whole) now, so the frames are free once this returns, as promised
  CX_OK(flush_slab(c));
  CX_HIP(hipStreamSynchronize(c->stream));
  if (c->side) CX_HIP(hipStreamSynchronize(c->side));  // a shift frame's gather reads the caller's frame
  if (c->comm_stream) CX_HIP(hipStreamSynchronize(c->comm_stream));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_set_staging(rmsf_ctx *c, int64_t batch_frames, int n_slots, int n_threads) {
  CX_OK(check_ctx(c, "rmsf_ctx_set_staging"));
  if (n_slots < 1 || n_threads < 0) return fail(RMSF_EINVAL, "rmsf_ctx_set_staging: n_slots >= 1, n_threads >= 0");
  c->stage_batch = batch_frames > 0 ? batch_frames : 0;
  c->stage_slots = n_slots;
  c->stage_threads = n_threads;
  c->stager_dirty = true;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_set_timing(rmsf_ctx *c, int on) {
  CX_OK(check_ctx(c, "rmsf_ctx_set_timing"));
  c->timing = on != 0;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_kernel_time(rmsf_ctx *c, int which, int64_t *launches, double *ms, double *atom_frames) {
  CX_OK(check_ctx(c, "rmsf_ctx_kernel_time"));
  if (which != RMSF_TIME_ACCUMULATE && which != RMSF_TIME_SUPERPOSE && which != RMSF_TIME_MERGE)
    return fail(RMSF_EINVAL, "rmsf_ctx_kernel_time: bad kernel");
  DeviceScope ds(c->dev);
  CX_OK(flush_slab(c));  // a recorded slab push is part of what was timed
  CX_OK(sync_streams(c));
  int64_t k = 0;
  double t = 0.0, af = 0.0;
  for (auto &sp : c->spans) {
    if (sp.which != which || !sp.closed) continue;
    float e = 0.f;
    CX_HIP(hipEventElapsedTime(&e, sp.a, sp.b));
    ++k;
    t += e;
    af += (double)sp.atom_frames;
  }
  drop_spans(c, which);
  if (launches) *launches = k;
  if (ms) *ms = t;
  if (atom_frames) *atom_frames = af;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_collect_rmsd(rmsf_ctx *c, int on) {
  CX_OK(check_ctx(c, "rmsf_ctx_collect_rmsd"));
  c->collect_rmsd = on != 0;
  c->n_rmsd = 0;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_get_rmsd(rmsf_ctx *c, int64_t *n, double *h_rmsd, int64_t capacity) {
  CX_OK(check_ctx(c, "rmsf_get_rmsd"));
  if (n) *n = c->n_rmsd;
  if (!h_rmsd || c->n_rmsd == 0) return RMSF_OK;
  if (capacity < c->n_rmsd) return fail(RMSF_EINVAL, "rmsf_get_rmsd: output holds fewer than n frames");
  DeviceScope ds(c->dev);
  CX_HIP(hipMemcpyAsync(h_rmsd, c->rmsd.p, sizeof(double) * c->n_rmsd, hipMemcpyDeviceToHost, c->stream));
  CX_HIP(hipStreamSynchronize(c->stream));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_reset(rmsf_ctx *c, int what) {
  CX_OK(check_ctx(c, "rmsf_ctx_reset"));
  // lazily: a reset state is zeroed only if it is read before a fold
  // overwrites it (ensure_zeroed); queued work for it is dropped
  if (what & 1) {
    c->n_rmsd = 0;
    c->wel.n = 0;
    c->wel.stale = true;
    c->wel_aligned = false;
    c->merged_away = false;
    c->rmsf_valid = false;
    c->slab.on = false;
    if (c->pend.on && c->pend.welford) c->pend.on = false;
  }
  if (what & 2) {
    c->sum.n = 0;
    c->sum.stale = true;
    if (c->pend.on && !c->pend.welford) c->pend.on = false;
  }
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_set_reference(rmsf_ctx *c, const double *h_ref, const double *h_com) {
  CX_OK(check_ctx(c, "rmsf_set_reference"));
  if (!h_ref || !h_com) return fail(RMSF_EINVAL, "rmsf_set_reference: NULL reference");
  // the record rmsf_reference_setup() would write (RMSF.py:84-86)
  double info[16] = {0};
  info[0] = h_com[0];
  info[1] = h_com[1];
  info[2] = h_com[2];
  for (int64_t a = 0; a < c->n_sel; ++a) {
    const double *r = h_ref + 3 * a;
    info[3] += r[0];
    info[4] += r[1];
    info[5] += r[2];
    info[6] += r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
    info[7] += c->has_masses ? c->h_masses[a] : 1.0;
  }
  info[8] = (double)c->n_sel;
  DeviceScope ds(c->dev);
  CX_HIP(hipMemcpyAsync(c->ref.p, h_ref, sizeof(double) * c->n_coord, hipMemcpyHostToDevice, c->stream));
  CX_HIP(hipMemcpyAsync(c->refinfo.p, info, sizeof(info), hipMemcpyHostToDevice, c->stream));
  CX_HIP(hipStreamSynchronize(c->stream));  // the host sources are the caller's / on this stack
  c->ref_set = true;
  c->ref_exact = true;  // G_ref above is qcprot's per-atom order already
  return digest_reference(c);
}

RMSF_EXPORT int rmsf_set_reference_frame(rmsf_ctx *c, const float *xyz, int is_device_ptr) {
  CX_OK(check_ctx(c, "rmsf_set_reference_frame"));
  if (!xyz) return fail(RMSF_EINVAL, "rmsf_set_reference_frame: NULL frame");
  DeviceScope ds(c->dev);
  const float *d = xyz;
  if (!is_device_ptr) {
    const size_t bytes = sizeof(float) * 3 * (size_t)c->n_atoms;
    CX_OK(c->frame.ensure(bytes, c->stream));
    CX_HIP(hipMemcpyAsync(c->frame.p, xyz, bytes, hipMemcpyHostToDevice, c->stream));
    CX_HIP(hipStreamSynchronize(c->stream));
    d = static_cast<const float *>(c->frame.p);
  }
  if (c->exact)
    CX_OK(rmsf_reference_setup_sequential(d, nullptr, 1.0, c->n_sel, c->d_sel(), c->d_masses(), c->mass_total,
                                          nullptr, c->ref.d(), c->refinfo.d(), c->stream));
  else
    CX_OK(rmsf_reference_setup(d, nullptr, c->n_sel, c->d_sel(), c->d_masses(), c->ref.d(), c->refinfo.d(),
                               c->stream));
  c->ref_set = true;
  c->ref_exact = c->exact;
  return digest_reference(c);
}

RMSF_EXPORT int rmsf_set_reference_average(rmsf_ctx *c) {
  CX_OK(check_ctx(c, "rmsf_set_reference_average"));
  if (c->sum.n <= 0) return fail(RMSF_EEMPTY, "rmsf_set_reference_average: no frames summed (RMSF.py:111)");
  DeviceScope ds(c->dev);
  CX_OK(settle(c));
  CX_OK(c->avg.ensure(sizeof(double) * c->n_coord, c->stream));
  if (c->exact)
    CX_OK(rmsf_reference_setup_sequential(nullptr, c->sum.parts0.d(), (double)c->sum.n, c->n_sel, nullptr,
                                          c->d_masses(), c->mass_total, c->avg.d(), c->ref.d(), c->refinfo.d(),
                                          c->stream));
  else
    CX_OK(rmsf_reference_setup_mean(c->sum.parts0.d(), (double)c->sum.n, c->n_sel, c->d_masses(), c->avg.d(),
                                    c->ref.d(), c->refinfo.d(), c->stream));
  c->ref_set = true;
  c->ref_exact = c->exact;
  return digest_reference(c);
}

RMSF_EXPORT int rmsf_ctx_set_exact(rmsf_ctx *c, int on, double mass_total) {
  CX_OK(check_ctx(c, "rmsf_ctx_set_exact"));
  if (on && !(mass_total > 0.0)) return fail(RMSF_EINVAL, "rmsf_ctx_set_exact: mass_total must be > 0");
  c->exact = on != 0;
  c->mass_total = on ? mass_total : 0.0;
  c->ref_exact = false;  // a reference set before does not carry the sequential record's bits
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_push_frames(rmsf_ctx *c, const float *xyz, int64_t n_frames, int64_t stride, int mode,
                                 int is_device_ptr) {
  CX_OK(check_ctx(c, "rmsf_push_frames"));
  CX_OK(check_mode(mode, "rmsf_push_frames"));
  if (n_frames < 0) return fail(RMSF_EINVAL, "rmsf_push_frames: n_frames < 0");
  if (n_frames == 0) return RMSF_OK;
  if (!xyz) return fail(RMSF_EINVAL, "rmsf_push_frames: NULL frames");
  if (stride == 0) stride = 3 * c->n_atoms;
  if (stride < 3 * c->n_atoms) return fail(RMSF_EINVAL, "rmsf_push_frames: frame_stride < 3*n_atoms");
  DeviceScope ds(c->dev);
  if (ds.err != hipSuccess) return fail(RMSF_EHIP, "rmsf_push_frames: hipSetDevice failed");
  CX_OK(flush_slab(c));  // an earlier recorded slab push comes first
  if (is_device_ptr) {
    for (int64_t f = 0; f < n_frames; f += kChunkFrames) {
      const int64_t nf = std::min(kChunkFrames, n_frames - f);
      CX_OK(process(c, xyz + f * stride, stride, nf, c->d_sel(), mode));
    }
    return RMSF_OK;
  }
  CX_OK(ensure_stager(c));
  for (int64_t f = 0; f < n_frames; f += c->stage_batch) {
    const int64_t nf = std::min(c->stage_batch, n_frames - f);
    int slot = -1;
    float *d = nullptr;
    CX_OK(rmsf_stager_stage(c->stager, xyz + f * stride, stride, nf, c->stream, &slot, &d));
    int rc = process(c, d, 3 * c->n_sel, nf, nullptr, mode);
    int rc2 = rmsf_stager_release(c->stager, slot, c->stream);
    CX_OK(rc);
    CX_OK(rc2);
  }
  // the host buffer is free once the gathers returned; copies run from pinned slots
  return RMSF_OK;
}

}  // extern "C"

namespace {

// The context's GPU XTC decoder for file x (made on first use, remade for another file).
int ensure_xdec(rmsf_ctx *c, const rmsf_xtc *x, int n_slots, int64_t *batch) {
  *batch = std::max<int64_t>(1, std::min<int64_t>(4096, (int64_t(2) << 30) / (12 * c->n_atoms)));
  if (!c->xdec || c->xdec_serial != x->serial) {
    if (c->xdec) CX_OK(rmsf_xtcdec_destroy(c->xdec));
    c->xdec = nullptr;
    CX_OK(rmsf_xtcdec_create(x, *batch, n_slots, 16, &c->xdec));
    c->xdec_serial = x->serial;
  }
  return RMSF_OK;
}

// Decode n_frames frames batch by batch (decode(i, n, &slot, &d) queues batch
// frames i..i+n) with up to kSlots decodes in flight ahead of the kernels,
// then wait once and report corrupt frames.
template <class Decode>
int push_decoded(rmsf_ctx *c, int64_t n_frames, int64_t batch, int mode, Decode &&decode) {
  constexpr size_t kSlots = 3;
  struct Pending {
    int slot;
    float *d;
    int64_t n;
  };
  std::vector<Pending> q;
  size_t head = 0;
  auto consume = [&]() -> int {
    const Pending p = q[head++];
    const int rc = process(c, p.d, 3 * c->n_atoms, p.n, c->d_sel(), mode);
    const int rc2 = rmsf_xtcdec_release(c->xdec, p.slot, c->stream);
    return rc ? rc : rc2;
  };
  for (int64_t i = 0; i < n_frames; i += batch) {
    Pending p{-1, nullptr, std::min(batch, n_frames - i)};
    CX_OK(decode(i, p.n, &p.slot, &p.d));
    q.push_back(p);
    if (q.size() - head >= kSlots) CX_OK(consume());
  }
  while (head < q.size()) CX_OK(consume());
  return rmsf_xtcdec_synchronize(c->xdec);
}

}  // namespace

extern "C" {

RMSF_EXPORT int rmsf_push_xtc(rmsf_ctx *c, const rmsf_xtc *x, int64_t f0, int64_t n_frames, int64_t step, int mode) {
  CX_OK(check_ctx(c, "rmsf_push_xtc"));
  CX_OK(check_mode(mode, "rmsf_push_xtc"));
  if (!x || n_frames < 0 || step < 1 || f0 < 0) return fail(RMSF_EINVAL, "rmsf_push_xtc: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  if (x->n_atoms != c->n_atoms) return fail(RMSF_EINVAL, "rmsf_push_xtc: the file's atom count differs");
  DeviceScope ds(c->dev);
  CX_OK(flush_slab(c));
  // the records are decompressed on the GPU (csrc/xtc_gpu.hip) into full
  // frames; the accumulate kernels gather the selection
  int64_t batch = 0;
  CX_OK(ensure_xdec(c, x, 3, &batch));
  return push_decoded(c, n_frames, batch, mode, [&](int64_t i, int64_t n, int *slot, float **d) {
    return rmsf_xtcdec_decode(c->xdec, f0 + i * step, n, step, c->stream, slot, d);
  });
}

RMSF_EXPORT int rmsf_push_xtc_frames(rmsf_ctx *c, const rmsf_xtc *x, const int64_t *h_frames, int64_t n_frames,
                                     int mode) {
  CX_OK(check_ctx(c, "rmsf_push_xtc_frames"));
  CX_OK(check_mode(mode, "rmsf_push_xtc_frames"));
  if (!x || n_frames < 0 || (n_frames > 0 && !h_frames)) return fail(RMSF_EINVAL, "rmsf_push_xtc_frames: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  if (x->n_atoms != c->n_atoms) return fail(RMSF_EINVAL, "rmsf_push_xtc_frames: the file's atom count differs");
  DeviceScope ds(c->dev);
  CX_OK(flush_slab(c));
  int64_t batch = 0;
  CX_OK(ensure_xdec(c, x, 3, &batch));
  return push_decoded(c, n_frames, batch, mode, [&](int64_t i, int64_t n, int *slot, float **d) {
    return rmsf_xtcdec_decode_list(c->xdec, h_frames + i, n, c->stream, slot, d);
  });
}

RMSF_EXPORT int rmsf_push_frame_ptrs(rmsf_ctx *c, const float *const *h_ptrs, int64_t n_frames, int mode) {
  CX_OK(check_ctx(c, "rmsf_push_frame_ptrs"));
  CX_OK(check_mode(mode, "rmsf_push_frame_ptrs"));
  if (n_frames < 0 || (n_frames > 0 && !h_ptrs)) return fail(RMSF_EINVAL, "rmsf_push_frame_ptrs: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  DeviceScope ds(c->dev);
  if (ds.err != hipSuccess) return fail(RMSF_EHIP, "rmsf_push_frame_ptrs: hipSetDevice failed");
  CX_OK(flush_slab(c));
  CX_OK(ensure_stager(c));
  for (int64_t f = 0; f < n_frames; f += c->stage_batch) {
    const int64_t nf = std::min(c->stage_batch, n_frames - f);
    int slot = -1;
    float *d = nullptr;
    CX_OK(rmsf_stager_stage_ptrs(c->stager, h_ptrs + f, nf, c->stream, &slot, &d));
    int rc = process(c, d, 3 * c->n_sel, nf, nullptr, mode);
    int rc2 = rmsf_stager_release(c->stager, slot, c->stream);
    CX_OK(rc);
    CX_OK(rc2);
  }
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_push_frame_planes(rmsf_ctx *c, const float *const *h_ptrs, int64_t plane_stride,
                                       int64_t n_frames, int mode) {
  CX_OK(check_ctx(c, "rmsf_push_frame_planes"));
  CX_OK(check_mode(mode, "rmsf_push_frame_planes"));
  if (n_frames < 0 || (n_frames > 0 && !h_ptrs) || plane_stride < c->n_atoms)
    return fail(RMSF_EINVAL, "rmsf_push_frame_planes: bad arguments");
  if (n_frames == 0) return RMSF_OK;
  DeviceScope ds(c->dev);
  if (ds.err != hipSuccess) return fail(RMSF_EHIP, "rmsf_push_frame_planes: hipSetDevice failed");
  CX_OK(flush_slab(c));
  CX_OK(ensure_stager(c));
  for (int64_t f = 0; f < n_frames; f += c->stage_batch) {
    const int64_t nf = std::min(c->stage_batch, n_frames - f);
    int slot = -1;
    float *d = nullptr;
    CX_OK(rmsf_stager_stage_planes(c->stager, h_ptrs + f, plane_stride, nf, c->stream, &slot, &d));
    int rc = process(c, d, 3 * c->n_sel, nf, nullptr, mode);
    int rc2 = rmsf_stager_release(c->stager, slot, c->stream);
    CX_OK(rc);
    CX_OK(rc2);
  }
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_get_partial(rmsf_ctx *c, int64_t *n, double *h_mean, double *h_m2) {
  CX_OK(check_ctx(c, "rmsf_get_partial"));
  if (c->merged_away)
    return fail(RMSF_EINVAL, "rmsf_get_partial: a reduce-to-root merge left the result on another context");
  DeviceScope ds(c->dev);
  CX_OK(settle(c));
  CX_OK(ensure_zeroed(c, c->wel, true));
  const size_t row = sizeof(double) * c->n_coord;
  if (h_mean) CX_HIP(hipMemcpyAsync(h_mean, c->wel.parts0.p, row, hipMemcpyDeviceToHost, c->stream));
  if (h_m2) CX_HIP(hipMemcpyAsync(h_m2, c->wel.parts1.p, row, hipMemcpyDeviceToHost, c->stream));
  CX_OK(sync_streams(c));
  if (n) *n = c->wel.n;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_get_sum(rmsf_ctx *c, int64_t *n, double *h_sum) {
  CX_OK(check_ctx(c, "rmsf_get_sum"));
  DeviceScope ds(c->dev);
  CX_OK(settle(c));
  CX_OK(ensure_zeroed(c, c->sum, false));
  if (h_sum)
    CX_HIP(hipMemcpyAsync(h_sum, c->sum.parts0.p, sizeof(double) * c->n_coord, hipMemcpyDeviceToHost, c->stream));
  CX_OK(sync_streams(c));
  if (n) *n = c->sum.n;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_get_average(rmsf_ctx *c, double *h_avg) {
  CX_OK(check_ctx(c, "rmsf_get_average"));
  if (!h_avg) return fail(RMSF_EINVAL, "rmsf_get_average: NULL output");
  if (c->sum.n <= 0) return fail(RMSF_EEMPTY, "rmsf_get_average: no frames summed");
  DeviceScope ds(c->dev);
  CX_OK(settle(c));
  CX_OK(c->avg.ensure(sizeof(double) * c->n_coord, c->stream));
  CX_OK(rmsf_divide(c->sum.parts0.d(), (double)c->sum.n, c->n_coord, c->avg.d(), c->stream));
  CX_HIP(hipMemcpyAsync(h_avg, c->avg.p, sizeof(double) * c->n_coord, hipMemcpyDeviceToHost, c->stream));
  CX_OK(sync_streams(c));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_get_rmsf(rmsf_ctx *c, double *h_rmsf) {
  CX_OK(check_ctx(c, "rmsf_get_rmsf"));
  if (!h_rmsf) return fail(RMSF_EINVAL, "rmsf_get_rmsf: NULL output");
  if (c->merged_away)
    return fail(RMSF_EINVAL, "rmsf_get_rmsf: a reduce-to-root merge left the result on another context");
  if (c->wel.n <= 0 && !c->slab.on) return fail(RMSF_EEMPTY, "rmsf_get_rmsf: no frames accumulated");
  DeviceScope ds(c->dev);
  CX_OK(settle(c));
  if (!c->rmsf_valid) {  // the shifted merges finalise as they unpack
    CX_OK(c->rmsf.ensure(sizeof(double) * c->n_sel, c->stream));
    CX_OK(rmsf_finalize(c->wel.parts1.d(), c->n_sel, c->wel.n, c->rmsf.d(), c->stream));
    c->rmsf_valid = true;
  }
  CX_HIP(hipMemcpyAsync(h_rmsf, c->rmsf.p, sizeof(double) * c->n_sel, hipMemcpyDeviceToHost, c->stream));
  CX_OK(sync_streams(c));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_set_partial(rmsf_ctx *c, int64_t n, const double *h_mean, const double *h_m2) {
  CX_OK(check_ctx(c, "rmsf_set_partial"));
  if (n < 0 || (n > 0 && (!h_mean || !h_m2))) return fail(RMSF_EINVAL, "rmsf_set_partial: bad arguments");
  DeviceScope ds(c->dev);
  c->slab.on = false;  // the state is replaced: queued work for it is moot
  if (c->pend.on && c->pend.welford) c->pend.on = false;
  c->merged_away = false;
  c->rmsf_valid = false;
  CX_OK(zero_running(c, c->wel, true));
  if (n > 0) {
    const size_t row = sizeof(double) * c->n_coord;
    CX_HIP(hipMemcpyAsync(c->wel.parts0.p, h_mean, row, hipMemcpyHostToDevice, c->stream));
    CX_HIP(hipMemcpyAsync(c->wel.parts1.p, h_m2, row, hipMemcpyHostToDevice, c->stream));
    CX_HIP(hipStreamSynchronize(c->stream));
  }
  c->wel.n = n;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_ctx_allreduce_sum(rmsf_ctx *c, rmsf_allreduce_fn fn, void *user) {
  CX_OK(check_ctx(c, "rmsf_ctx_allreduce_sum"));
  if (!fn) return fail(RMSF_EINVAL, "rmsf_ctx_allreduce_sum: NULL callback");
  return exchange_sum(&c, 1, callback_reduce(c, fn, user), false);
}

RMSF_EXPORT int rmsf_ctx_chan_merge(rmsf_ctx *c, rmsf_allreduce_fn fn, void *user) {
  CX_OK(check_ctx(c, "rmsf_ctx_chan_merge"));
  if (!fn) return fail(RMSF_EINVAL, "rmsf_ctx_chan_merge: NULL callback");
  return exchange_chan(&c, 1, callback_reduce(c, fn, user), false);
}

RMSF_EXPORT int rmsf_ctx_chan_merge_shifted(rmsf_ctx *c, rmsf_allreduce_fn fn, void *user) {
  CX_OK(check_ctx(c, "rmsf_ctx_chan_merge_shifted"));
  if (!fn) return fail(RMSF_EINVAL, "rmsf_ctx_chan_merge_shifted: NULL callback");
  return exchange_chan_shifted(&c, 1, callback_reduce(c, fn, user), false, Shift::REF, -1);
}

RMSF_EXPORT int rmsf_multi_unique_id(void *id_out) {
  if (!id_out) return fail(RMSF_EINVAL, "rmsf_multi_unique_id: NULL output");
  const Rccl &r = rccl();
  if (!r.ok) return fail(RMSF_EHIP, r.why);
  static_assert(sizeof(ncclUniqueId) == RMSF_UNIQUE_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  ncclResult_t e = r.GetUniqueId(&id);
  if (e != ncclSuccess) return nccl_fail("ncclGetUniqueId", e);
  std::memcpy(id_out, &id, sizeof(id));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_multi_init(rmsf_ctx *c, const void *id, int nranks, int rank) {
  CX_OK(check_ctx(c, "rmsf_multi_init"));
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail(RMSF_EINVAL, "rmsf_multi_init: bad arguments");
  if (c->comm) return fail(RMSF_EINVAL, "rmsf_multi_init: context already has a communicator");
  const Rccl &r = rccl();
  if (!r.ok) return fail(RMSF_EHIP, r.why);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  DeviceScope ds(c->dev);
  ncclResult_t e = r.CommInitRank(&c->comm, nranks, uid, rank);
  if (e != ncclSuccess) {
    c->comm = nullptr;
    return nccl_fail("ncclCommInitRank", e);
  }
  c->comm_size = nranks;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_multi_init_all(rmsf_ctx **cs, int n) {
  if (!cs || n < 1) return fail(RMSF_EINVAL, "rmsf_multi_init_all: no contexts");
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) {
    CX_OK(check_ctx(cs[i], "rmsf_multi_init_all"));
    if (cs[i]->comm) return fail(RMSF_EINVAL, "rmsf_multi_init_all: a context already has a communicator");
    devs[i] = cs[i]->dev;
  }
  const Rccl &r = rccl();
  if (!r.ok) return fail(RMSF_EHIP, r.why);
  std::vector<ncclComm_t> comms(n, nullptr);
  ncclResult_t e = r.CommInitAll(comms.data(), n, devs.data());
  if (e != ncclSuccess) return nccl_fail("ncclCommInitAll", e);
  for (int i = 0; i < n; ++i) {
    cs[i]->comm = comms[i];
    cs[i]->comm_size = n;
  }
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_multi_allreduce_sum(rmsf_ctx **cs, int n) {
  Reduce red;
  int kind = 0;
  CX_OK(multi_reduce(cs, n, "rmsf_multi_allreduce_sum", &red, &kind));
  bool exact = true;
  for (int i = 0; i < n; ++i) exact = exact && cs[i]->exact;
  // exact contexts of this process: RMSF.py:110's sums added in rank order,
  // ((s_0 + s_1) + s_2) + ... (local_reduce), not in RCCL's ring order --
  // the same bits as any order for two ranks, this build's order beyond
  if (exact && kind == 1 && whole_group_here(cs, n)) red = local_reduce(cs, n);
  return exchange_sum(cs, n, red, whole_group_here(cs, n));
}

RMSF_EXPORT int rmsf_multi_chan_merge_root(rmsf_ctx **cs, int n, int root) {
  Reduce red;
  int kind = 0;
  CX_OK(multi_reduce(cs, n, "rmsf_multi_chan_merge_root", &red, &kind));
  if (root < -1 || root >= n) return fail(RMSF_EINVAL, "rmsf_multi_chan_merge_root: root outside the contexts");
  // Every rank of the exchange is a context of this process: the merge is ONE
  // data collective of moments about a shift every context holds -- the
  // reference of aligned state (RMSF.py's ranks hold the same one), or the
  // merge shift frame of unaligned state -- with the reference / frame
  // digests compared here (k_digest: one shift c for T1 = sum n_k (mean_k -
  // c)).  Ranks in other processes could decide differently, so a
  // communicator spanning processes keeps the two-pass form
  // (rmsf_ctx_chan_merge_shifted is the explicit choice there), as do
  // contexts without a common shift.  The two-pass form leaves the result on
  // every context whatever `root` asks.
  const bool here = whole_group_here(cs, n);
  bool unaligned = true;  // the Welford state of every context came from unaligned pushes
  for (int i = 0; i < n; ++i) unaligned = unaligned && (cs[i]->slab.on || !cs[i]->wel_aligned);
  bool use_ref = false, use_frame = false;
  if (here && unaligned) CX_OK(same_digests(cs, n, true, &use_frame));
  if (here && !use_frame) CX_OK(same_digests(cs, n, false, &use_ref));
  if (use_frame) {
    bool slabs = true;
    for (int i = 0; i < n; ++i)
      slabs = slabs && cs[i]->slab.on && cs[i]->slab.chunks == cs[0]->slab.chunks && cs[i]->slab.k == cs[0]->slab.k;
    if (slabs) return slab_merge(cs, n, kind, red, root);
    return exchange_chan_shifted(cs, n, red, here, Shift::FRAME, root);
  }
  if (use_ref) return exchange_chan_shifted(cs, n, red, here, Shift::REF, root);
  return exchange_chan(cs, n, red, here);
}

RMSF_EXPORT int rmsf_multi_chan_merge(rmsf_ctx **cs, int n) { return rmsf_multi_chan_merge_root(cs, n, -1); }

RMSF_EXPORT int rmsf_multi_chan_merge_exact(rmsf_ctx **cs, int n, int root, int order) {
  if (!cs || n < 1) return fail(RMSF_EINVAL, "rmsf_multi_chan_merge_exact: no contexts");
  if (root < -1 || root >= n) return fail(RMSF_EINVAL, "rmsf_multi_chan_merge_exact: root outside the contexts");
  if (order != RMSF_MERGE_RANK && order != RMSF_MERGE_MPI4PY)
    return fail(RMSF_EINVAL, "rmsf_multi_chan_merge_exact: unknown order");
  for (int i = 0; i < n; ++i) {
    CX_OK(check_ctx(cs[i], "rmsf_multi_chan_merge_exact"));
    if (cs[i]->n_coord != cs[0]->n_coord) return fail(RMSF_EINVAL, "rmsf_multi_chan_merge_exact: contexts differ in n_sel");
    for (int j = 0; j < i; ++j)
      if (cs[j] == cs[i]) return fail(RMSF_EINVAL, "rmsf_multi_chan_merge_exact: a context is listed twice");
    if (cs[i]->merged_away)
      return fail(RMSF_EINVAL, "rmsf_multi_chan_merge_exact: a context's state was merged away (reset it first)");
  }
  if (!whole_group_here(cs, n))
    return fail(RMSF_EINVAL, "rmsf_multi_chan_merge_exact: the communicator spans other processes; merge their "
                             "rmsf_get_partial states with rmsf_chan_reduce / rmsf_chan_merge_pair over the host's "
                             "transport");
  return exact_merge(cs, n, root, order);
}

RMSF_EXPORT int rmsf_multi_set_transport(rmsf_ctx **cs, int n, int transport) {
  if (!cs || n < 1) return fail(RMSF_EINVAL, "rmsf_multi_set_transport: no contexts");
  if (transport != RMSF_TRANSPORT_AUTO && transport != RMSF_TRANSPORT_NOOP)
    return fail(RMSF_EINVAL, "rmsf_multi_set_transport: unknown transport");
  for (int i = 0; i < n; ++i) CX_OK(check_ctx(cs[i], "rmsf_multi_set_transport"));
  for (int i = 0; i < n; ++i) cs[i]->transport = transport;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_set_merge_shift_frame(rmsf_ctx *c, const float *xyz, int is_device_ptr) {
  CX_OK(check_ctx(c, "rmsf_set_merge_shift_frame"));
  if (!xyz) return fail(RMSF_EINVAL, "rmsf_set_merge_shift_frame: NULL frame");
  DeviceScope ds(c->dev);
  const float *d = xyz;
  if (!is_device_ptr) {
    const size_t bytes = sizeof(float) * 3 * (size_t)c->n_atoms;
    CX_OK(c->frame.ensure(bytes, c->stream));
    CX_HIP(hipMemcpyAsync(c->frame.p, xyz, bytes, hipMemcpyHostToDevice, c->stream));
    CX_HIP(hipStreamSynchronize(c->stream));
    d = static_cast<const float *>(c->frame.p);
  }
  // on the side stream, after the work queued so far (a previous merge still
  // reading the old shift); the merge waits for ev_dig[1]
  CX_OK(side_begin(c));
  CX_OK(shift_frame_on_side(c, d));
  // a host frame was staged in c->frame, which the next host setter reuses:
  // the gather from it finishes here
  if (!is_device_ptr) CX_HIP(hipStreamSynchronize(c->side));
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_multi_push_frames(rmsf_ctx **cs, int n, const float *const *d_frames, const int64_t *n_frames,
                                       int64_t frame_stride, int mode, int flags, const float *const *d_ref_frames,
                                       const float *const *d_shift_frames, int merge_slabs) {
  if (!cs || n < 1 || !d_frames || !n_frames) return fail(RMSF_EINVAL, "rmsf_multi_push_frames: bad arguments");
  CX_OK(check_mode(mode, "rmsf_multi_push_frames"));
  if (merge_slabs < 0) return fail(RMSF_EINVAL, "rmsf_multi_push_frames: merge_slabs < 0");
  for (int i = 0; i < n; ++i) {
    CX_OK(check_ctx(cs[i], "rmsf_multi_push_frames"));
    if (n_frames[i] < 0 || (n_frames[i] > 0 && !d_frames[i]))
      return fail(RMSF_EINVAL, "rmsf_multi_push_frames: bad frames");
    for (int j = 0; j < i; ++j)
      if (cs[j] == cs[i]) return fail(RMSF_EINVAL, "rmsf_multi_push_frames: a context is listed twice");
  }
  return for_each_ctx(cs, n, [&](int i) -> int {
    rmsf_ctx *c = cs[i];
    // the job runs on a worker thread whose current device is not c's: every
    // stream, event and buffer below (side_begin, the shift frame's gather)
    // belongs on c's device
    DeviceScope ds(c->dev);
    if (ds.err != hipSuccess) return fail(RMSF_EHIP, "rmsf_multi_push_frames: hipSetDevice failed");
    if (flags & RMSF_MULTI_RESET)
      CX_OK(rmsf_ctx_reset(c, (mode == RMSF_PUSH_WELFORD || mode == RMSF_PUSH_ALIGN_WELFORD ||
                               mode == RMSF_PUSH_EXACT) ? 1 : 2));
    if (d_ref_frames && d_ref_frames[i]) CX_OK(rmsf_set_reference_frame(c, d_ref_frames[i], 1));
    // the shift frame is needed only by the merge: its gather is queued on
    // the side stream AFTER this push's launches (so they leave the host
    // first) but ordered after the work queued BEFORE them (a previous merge
    // still reading the old shift), not after the sweep
    const bool shift_after = d_shift_frames && d_shift_frames[i];
    if (shift_after) CX_OK(side_begin(c));
    const int64_t nf = n_frames[i];
    if (nf == 0) return shift_after ? shift_frame_on_side(c, d_shift_frames[i]) : RMSF_OK;
    const int64_t stride = frame_stride ? frame_stride : 3 * c->n_atoms;
    // the atom-slab merge (C4's size): a single unaligned launch group over
    // all atoms whose flat plan is chunk-aligned, recorded here and streamed
    // slab by slab by the next rmsf_multi_chan_merge_root
    const int k = merge_slabs == 0 ? (c->n_sel >= kSlabMinAtoms ? kSlabsAuto : 1) : merge_slabs;
    if (k >= 2 && mode == RMSF_PUSH_WELFORD && !c->d_sel() && (c->shift_set || shift_after) && nf <= kChunkFrames &&
        c->wel.n == 0 && !c->slab.on && stride >= 3 * c->n_atoms) {
      int64_t chunks = 0;
      CX_OK(rmsf_balanced_slab_chunks(d_frames[i], stride, nf, c->n_sel, &chunks));
      if (chunks >= 2 * 3) {
        CX_OK(flush_fold(c));
        c->slab = {true, d_frames[i], stride, nf, chunks, k};
        c->rmsf_valid = false;
        c->merged_away = false;
        return shift_after ? shift_frame_on_side(c, d_shift_frames[i]) : RMSF_OK;
      }
    }
    CX_OK(rmsf_push_frames(c, d_frames[i], nf, stride, mode, 1));
    return shift_after ? shift_frame_on_side(c, d_shift_frames[i]) : RMSF_OK;
  });
}

}  // extern "C"
