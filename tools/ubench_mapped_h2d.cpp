// Feasibility/timing probe for the C5 host path: can the page cache of an
// XTC file be DMA'd to HBM straight from a registered (pinned) read-only
// mapping, skipping the pread copy into a pinned slot?
//
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 -x hip ubench_mapped_h2d.cpp -o ubench_mapped_h2d -lpthread
//   ./ubench_mapped_h2d [GB] [path]
//
// Prints: file write; mmap + hipHostRegister time; H2D from the registered
// mapping (1 stream, 3 streams); pread(16 threads) -> pinned -> H2D pieces
// (the current decoder's path) for comparison.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 2.7;
  const char *path = argc > 2 ? argv[2] : "/tmp/ubench_mapped_h2d.bin";
  const size_t n = (size_t)(gb * 1e9) & ~(size_t)4095;
  {
    std::vector<unsigned char> buf(64 << 20);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (unsigned char)(i * 2654435761u >> 13);
    int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0600);
    if (fd < 0) { std::perror("open"); return 1; }
    double t = now();
    for (size_t o = 0; o < n; o += buf.size()) {
      size_t len = std::min(buf.size(), n - o);
      if (write(fd, buf.data(), len) != (ssize_t)len) { std::perror("write"); return 1; }
    }
    close(fd);
    std::printf("write %.2f GB: %.3f s\n", n / 1e9, now() - t);
  }
  int fd = open(path, O_RDONLY);
  unsigned char *d = nullptr;
  CK(hipMalloc((void **)&d, n));
  hipStream_t st[3];
  for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipDeviceSynchronize());

  // (a) current path: pread into pinned, H2D in 128 MB pieces
  {
    const size_t piece = 128u << 20;
    unsigned char *h = nullptr;
    CK(hipHostMalloc((void **)&h, n, hipHostMallocDefault));
    for (int rep = 0; rep < 3; ++rep) {
      double t = now();
      for (size_t o = 0; o < n; o += piece) {
        size_t len = std::min(piece, n - o);
        const int T = 16;
        size_t ch = (len + T - 1) / T;
        std::vector<std::thread> th;
        for (int k = 0; k < T; ++k)
          th.emplace_back([&, k] {
            size_t s = k * ch;
            if (s >= len) return;
            size_t l = std::min(ch, len - s);
            while (l) {
              ssize_t r = pread(fd, h + o + s, l, (off_t)(o + s));
              if (r <= 0) return;
              s += r;
              l -= r;
            }
          });
        for (auto &x : th) x.join();
        CK(hipMemcpyAsync(d + o, h + o, len, hipMemcpyHostToDevice, st[0]));
      }
      CK(hipStreamSynchronize(st[0]));
      double dt = now() - t;
      std::printf("pread16+pinned+H2D: %.2f ms  %.1f GB/s\n", dt * 1e3, n / dt / 1e9);
    }
    CK(hipHostFree(h));
  }

  // (b) registered read-only mapping of the file
  double t = now();
  void *m = mmap(nullptr, n, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
  if (m == MAP_FAILED) { std::perror("mmap"); return 1; }
  double t_map = now() - t;
  t = now();
  hipError_t e = hipHostRegister(m, n, hipHostRegisterReadOnly);
  double t_reg = now() - t;
  std::printf("mmap(POPULATE) %.2f ms, hipHostRegister(ReadOnly) %.2f ms -> %s\n", t_map * 1e3, t_reg * 1e3,
              hipGetErrorString(e));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    t = now();
    e = hipHostRegister(m, n, hipHostRegisterDefault);
    std::printf("hipHostRegister(Default) %.2f ms -> %s\n", (now() - t) * 1e3, hipGetErrorString(e));
    if (e != hipSuccess) return 0;
  }
  for (int rep = 0; rep < 3; ++rep) {
    t = now();
    CK(hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, st[0]));
    CK(hipStreamSynchronize(st[0]));
    double dt = now() - t;
    std::printf("mapped H2D 1 copy: %.2f ms  %.1f GB/s\n", dt * 1e3, n / dt / 1e9);
  }
  for (int rep = 0; rep < 3; ++rep) {
    t = now();
    size_t third = (n / 3) & ~(size_t)4095;
    for (int k = 0; k < 3; ++k) {
      size_t o = k * third, len = k == 2 ? n - o : third;
      CK(hipMemcpyAsync(d + o, (unsigned char *)m + o, len, hipMemcpyHostToDevice, st[k]));
    }
    for (auto &s : st) CK(hipStreamSynchronize(s));
    double dt = now() - t;
    std::printf("mapped H2D 3 streams: %.2f ms  %.1f GB/s\n", dt * 1e3, n / dt / 1e9);
  }
  // verify a few bytes
  std::vector<unsigned char> chk(4096);
  CK(hipMemcpy(chk.data(), d + n - 4096, 4096, hipMemcpyDeviceToHost));
  std::printf("tail bytes match: %d\n", std::memcmp(chk.data(), (unsigned char *)m + n - 4096, 4096) == 0);
  t = now();
  CK(hipHostUnregister(m));
  std::printf("hipHostUnregister %.2f ms\n", (now() - t) * 1e3);
  munmap(m, n);
  close(fd);
  unlink(path);
  return 0;
}
