// stager.cpp -- pinned-host, multi-buffered host->device frame stager.
//
// Replaces the per-frame `universe.trajectory[frame]` -> `ts.positions` read
// of RMSF.py:92,124 as the source of device frame blocks (north star
// subsystem 1).  Frames arrive as host float32 [n_atoms_frame][3] arrays; the
// selection (RMSF.py:77,126 -- only these rows are ever consumed, SURVEY
// Appendix B Q3) is gathered by a small thread pool straight into a pinned
// slot, the slot is copied with hipMemcpyAsync on the stager's own copy
// stream, and the consumer stream waits on the copy event.  With >= 2 slots
// the host gather of batch i+1 and the DMA of batch i overlap the kernels of
// batch i-1.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rmsf_hip.h"
#include "host_affinity.h"

#define RMSF_EXPORT __attribute__((visibility("default")))

// error reporting shared with rmsf_kernels.hip through this small hook
extern "C" int rmsf_internal_set_error(int code, const char *msg);
extern "C" int rmsf_internal_xtc_decode(const rmsf_xtc *x, int64_t f0, int64_t n, int64_t step, const int32_t *sel,
                                        int64_t n_sel, float *out, int64_t out_stride, int n_threads);
extern "C" int64_t rmsf_internal_xtc_natoms(const rmsf_xtc *x);
extern "C" int64_t rmsf_internal_xtc_nframes(const rmsf_xtc *x);

namespace {

int fail(int code, const std::string &m) { return rmsf_internal_set_error(code, m.c_str()); }

#define ST_HIP(expr)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(RMSF_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Fixed pool: run(n, fn) calls fn(i) for i in [0, n) on the workers + caller.
class Pool {
 public:
  // cpus != nullptr: the workers run on those CPUs (rmsf_host::device_cpus)
  explicit Pool(int n, const cpu_set_t *cpus = nullptr) {
    for (int i = 0; i < n; ++i) {
      if (cpus) {
        const cpu_set_t c = *cpus;
        workers_.emplace_back([this, c] {
          rmsf_host::pin_self(c);
          loop();
        });
      } else {
        workers_.emplace_back([this] { loop(); });
      }
    }
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  void run(int64_t n, const std::function<void(int64_t)> &fn) {
    if (workers_.empty() || n <= 1) {
      for (int64_t i = 0; i < n; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      n_ = n;
      next_ = 0;
      busy_ = (int)workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void drain() {
    for (;;) {
      int64_t i;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (next_ >= n_) return;
        i = next_++;
      }
      (*fn_)(i);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      drain();
      {
        std::lock_guard<std::mutex> g(mu_);
        if (--busy_ == 0) done_cv_.notify_all();
      }
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t)> *fn_ = nullptr;
  int64_t n_ = 0, next_ = 0;
  int busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace

struct rmsf_stager {
  int64_t n_atoms_frame = 0, n_sel = 0, batch = 0;
  std::vector<int32_t> sel;  // empty = identity
  int n_slots = 0, next = 0;
  std::vector<float *> h_slot, d_slot;
  std::vector<hipEvent_t> copied, released;
  std::vector<char> copy_pending, release_pending;
  hipStream_t copy_stream = nullptr;
  Pool *pool = nullptr;
  int n_threads = 1;
};

namespace {

void destroy(rmsf_stager *st) {
  if (!st) return;
  if (st->copy_stream) (void)hipStreamSynchronize(st->copy_stream);
  for (auto p : st->h_slot)
    if (p) (void)hipHostFree(p);
  for (auto p : st->d_slot)
    if (p) (void)hipFree(p);
  for (auto e : st->copied)
    if (e) (void)hipEventDestroy(e);
  for (auto e : st->released)
    if (e) (void)hipEventDestroy(e);
  if (st->copy_stream) (void)hipStreamDestroy(st->copy_stream);
  delete st->pool;
  delete st;
}

// Take the next slot, let `fill(dst)` write n_frames compact frames into its
// pinned buffer, then queue the DMA and make the consumer wait for it.
int fill_and_copy(rmsf_stager *st, int64_t n_frames, const std::function<int(float *)> &fill, void *consumer_stream,
                  int *slot, float **d_batch) {
  if (n_frames < 1 || n_frames > st->batch)
    return fail(RMSF_EINVAL, "rmsf_stager_stage: n_frames must be in [1, batch_frames]");
  const int s = st->next;
  st->next = (st->next + 1) % st->n_slots;
  // the pinned slot may still be feeding an earlier DMA
  if (st->copy_pending[s]) {
    ST_HIP(hipEventSynchronize(st->copied[s]));
    st->copy_pending[s] = 0;
  }
  const int rc = fill(st->h_slot[s]);
  if (rc != RMSF_OK) return rc;
  // the device slot may still be read by the consumer's kernels
  if (st->release_pending[s]) {
    ST_HIP(hipStreamWaitEvent(st->copy_stream, st->released[s], 0));
    st->release_pending[s] = 0;
  }
  const int64_t row = 3 * st->n_sel;
  ST_HIP(hipMemcpyAsync(st->d_slot[s], st->h_slot[s], (size_t)n_frames * row * sizeof(float), hipMemcpyHostToDevice,
                        st->copy_stream));
  ST_HIP(hipEventRecord(st->copied[s], st->copy_stream));
  st->copy_pending[s] = 1;
  ST_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(consumer_stream), st->copied[s], 0));
  *slot = s;
  *d_batch = st->d_slot[s];
  return RMSF_OK;
}

// Gather the selection rows of host frames into dst; `frame(i)` yields frame i.
int gather(rmsf_stager *st, int64_t n_frames, const std::function<const float *(int64_t)> &frame, float *dst) {
  const int64_t row = 3 * st->n_sel;
  const int32_t *sel = st->sel.empty() ? nullptr : st->sel.data();
  const int64_t n_sel = st->n_sel;
  // split work into (frame, atom-range) pieces so one big frame still spreads
  const int64_t piece = 1 << 16;
  const int64_t per_frame = (n_sel + piece - 1) / piece;
  std::atomic<bool> bad{false};
  st->pool->run(n_frames * per_frame, [&](int64_t w) {
    const int64_t f = w / per_frame, a0 = (w % per_frame) * piece, a1 = std::min(n_sel, a0 + piece);
    const float *src = frame(f);
    if (!src) {
      bad = true;
      return;
    }
    float *o = dst + f * row;
    if (!sel) {
      std::memcpy(o + 3 * a0, src + 3 * a0, (size_t)(a1 - a0) * 3 * sizeof(float));
    } else {
      for (int64_t a = a0; a < a1; ++a) {
        const float *q = src + 3 * (int64_t)sel[a];
        o[3 * a] = q[0];
        o[3 * a + 1] = q[1];
        o[3 * a + 2] = q[2];
      }
    }
  });
  return bad ? fail(RMSF_EINVAL, "rmsf_stager_stage: null frame pointer") : RMSF_OK;
}

// Gather the selection of host frames stored as coordinate planes (SoA: x[n],
// y[n], z[n] at plane(f), plane(f) + plane_stride, plane(f) + 2 plane_stride
// floats -- a DCD frame's X/Y/Z records, or a synthetic [F][3][n] array) and
// interleave them into dst's (frame, atom, xyz) rows on the way into the
// pinned slot: the device sees the same frame blocks as for [F][n][3] input,
// and the bytes over PCIe stay 12 per selected atom.
int gather_planes(rmsf_stager *st, int64_t n_frames, const std::function<const float *(int64_t)> &frame,
                  int64_t plane_stride, float *dst) {
  const int64_t row = 3 * st->n_sel;
  const int32_t *sel = st->sel.empty() ? nullptr : st->sel.data();
  const int64_t n_sel = st->n_sel;
  const int64_t piece = 1 << 16;
  const int64_t per_frame = (n_sel + piece - 1) / piece;
  std::atomic<bool> bad{false};
  st->pool->run(n_frames * per_frame, [&](int64_t w) {
    const int64_t f = w / per_frame, a0 = (w % per_frame) * piece, a1 = std::min(n_sel, a0 + piece);
    const float *x = frame(f);
    if (!x) {
      bad = true;
      return;
    }
    const float *y = x + plane_stride, *z = y + plane_stride;
    float *o = dst + f * row;
    if (!sel) {
      for (int64_t a = a0; a < a1; ++a) {
        o[3 * a] = x[a];
        o[3 * a + 1] = y[a];
        o[3 * a + 2] = z[a];
      }
    } else {
      for (int64_t a = a0; a < a1; ++a) {
        const int64_t i = sel[a];
        o[3 * a] = x[i];
        o[3 * a + 1] = y[i];
        o[3 * a + 2] = z[i];
      }
    }
  });
  return bad ? fail(RMSF_EINVAL, "rmsf_stager_stage_planes: null frame pointer") : RMSF_OK;
}

}  // namespace

extern "C" {

RMSF_EXPORT int rmsf_stager_create(int64_t n_atoms_frame, int64_t n_sel, const int32_t *h_sel, int64_t batch_frames,
                                   int n_slots, int n_threads, rmsf_stager **out) {
  if (!out || n_atoms_frame < 1 || n_sel < 1 || batch_frames < 1 || n_slots < 1 || n_slots > 64 ||
      (!h_sel && n_sel > n_atoms_frame))
    return fail(RMSF_EINVAL, "rmsf_stager_create: bad arguments");
  *out = nullptr;
  auto *st = new rmsf_stager();
  st->n_atoms_frame = n_atoms_frame;
  st->n_sel = n_sel;
  st->batch = batch_frames;
  st->n_slots = n_slots;
  if (h_sel) {
    st->sel.assign(h_sel, h_sel + n_sel);
    for (int32_t i : st->sel)
      if (i < 0 || i >= n_atoms_frame) {
        destroy(st);
        return fail(RMSF_EINVAL, "rmsf_stager_create: selection index out of range");
      }
  }
  const size_t bytes = (size_t)batch_frames * (size_t)n_sel * 3 * sizeof(float);
  st->h_slot.assign(n_slots, nullptr);
  st->d_slot.assign(n_slots, nullptr);
  st->copied.assign(n_slots, nullptr);
  st->released.assign(n_slots, nullptr);
  st->copy_pending.assign(n_slots, 0);
  st->release_pending.assign(n_slots, 0);
  hipError_t e = hipStreamCreateWithFlags(&st->copy_stream, hipStreamNonBlocking);
  for (int i = 0; e == hipSuccess && i < n_slots; ++i) {
    e = hipHostMalloc(reinterpret_cast<void **>(&st->h_slot[i]), bytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&st->d_slot[i]), bytes);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&st->copied[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&st->released[i], hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    destroy(st);
    return fail(RMSF_ENOMEM, std::string("rmsf_stager_create: ") + hipGetErrorString(e));
  }
  int dev = 0;
  cpu_set_t near;
  const bool pin = hipGetDevice(&dev) == hipSuccess && rmsf_host::device_cpus(dev, &near);
  st->pool = new Pool(std::max(0, n_threads - 1), pin ? &near : nullptr);
  st->n_threads = std::max(1, n_threads);
  *out = st;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_stager_destroy(rmsf_stager *st) {
  destroy(st);
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_stager_stage(rmsf_stager *st, const float *h_frames, int64_t h_frame_stride, int64_t n_frames,
                                  void *consumer_stream, int *slot, float **d_batch) {
  if (!st || !h_frames || !slot || !d_batch || h_frame_stride < 3 * st->n_atoms_frame)
    return fail(RMSF_EINVAL, "rmsf_stager_stage: bad arguments");
  return fill_and_copy(
      st, n_frames, [&](float *dst) { return gather(st, n_frames, [&](int64_t f) { return h_frames + f * h_frame_stride; }, dst); },
      consumer_stream, slot, d_batch);
}

RMSF_EXPORT int rmsf_stager_stage_ptrs(rmsf_stager *st, const float *const *h_frame_ptrs, int64_t n_frames,
                                       void *consumer_stream, int *slot, float **d_batch) {
  if (!st || !h_frame_ptrs || !slot || !d_batch) return fail(RMSF_EINVAL, "rmsf_stager_stage_ptrs: bad arguments");
  return fill_and_copy(
      st, n_frames, [&](float *dst) { return gather(st, n_frames, [&](int64_t f) { return h_frame_ptrs[f]; }, dst); },
      consumer_stream, slot, d_batch);
}

RMSF_EXPORT int rmsf_stager_stage_planes(rmsf_stager *st, const float *const *h_frame_ptrs, int64_t h_plane_stride,
                                         int64_t n_frames, void *consumer_stream, int *slot, float **d_batch) {
  if (!st || !h_frame_ptrs || !slot || !d_batch || h_plane_stride < st->n_atoms_frame)
    return fail(RMSF_EINVAL, "rmsf_stager_stage_planes: bad arguments");
  return fill_and_copy(
      st, n_frames,
      [&](float *dst) {
        return gather_planes(st, n_frames, [&](int64_t f) { return h_frame_ptrs[f]; }, h_plane_stride, dst);
      },
      consumer_stream, slot, d_batch);
}

RMSF_EXPORT int rmsf_stager_stage_xtc(rmsf_stager *st, const rmsf_xtc *x, int64_t f0, int64_t n_frames, int64_t step,
                                      void *consumer_stream, int *slot, float **d_batch) {
  if (!st || !x || !slot || !d_batch || step < 1 || f0 < 0)
    return fail(RMSF_EINVAL, "rmsf_stager_stage_xtc: bad arguments");
  if (rmsf_internal_xtc_natoms(x) != st->n_atoms_frame)
    return fail(RMSF_EINVAL, "rmsf_stager_stage_xtc: atom count differs from the stager's frame size");
  if (n_frames > 0 && f0 + (n_frames - 1) * step >= rmsf_internal_xtc_nframes(x))
    return fail(RMSF_EINVAL, "rmsf_stager_stage_xtc: frame out of range");
  const int32_t *sel = st->sel.empty() ? nullptr : st->sel.data();
  const int nt = st->n_threads;
  return fill_and_copy(
      st, n_frames,
      [&](float *dst) { return rmsf_internal_xtc_decode(x, f0, n_frames, step, sel, st->n_sel, dst, 3 * st->n_sel, nt); },
      consumer_stream, slot, d_batch);
}

RMSF_EXPORT int rmsf_stager_release(rmsf_stager *st, int slot, void *consumer_stream) {
  if (!st || slot < 0 || slot >= st->n_slots) return fail(RMSF_EINVAL, "rmsf_stager_release: bad slot");
  ST_HIP(hipEventRecord(st->released[slot], reinterpret_cast<hipStream_t>(consumer_stream)));
  st->release_pending[slot] = 1;
  return RMSF_OK;
}

RMSF_EXPORT int rmsf_stager_synchronize(rmsf_stager *st) {
  if (!st) return fail(RMSF_EINVAL, "rmsf_stager_synchronize: null");
  ST_HIP(hipStreamSynchronize(st->copy_stream));
  for (int i = 0; i < st->n_slots; ++i) st->copy_pending[i] = 0;
  return RMSF_OK;
}

}  // extern "C"
