// Self-test driver for the host runtime (libbe_runtime sources linked in directly), built by
// tools/sanitize_runtime.py under AddressSanitizer + UndefinedBehaviorSanitizer and, separately,
// ThreadSanitizer (SURVEY.md §5 "Race detection / sanitizers": the reference has none).
//
//  * watershed: 2-D two-basin image and a 3-D random image; checks every in-mask voxel is labelled
//    by a marker label and out-of-mask voxels stay 0.
//  * ensure_spacing: random 2-D/3-D points vs an O(N^2) oracle.
//  * shm ring: producer and consumer threads (TSan sees every cross-thread access) streaming
//    variable-size multi-frame messages through a small ring that wraps many times, plus a
//    forked consumer process (cross-process futex wake-ups), full/timeout/too-large/closed paths.
#include <sys/wait.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int be_rt_watershed(const float*, const int*, const unsigned char*, int, int, int, int, int*);
int be_rt_ensure_spacing(const int*, int, int, int, unsigned char*);
int be_rt_ring_create(const char*, int64_t, void**);
int be_rt_ring_open(const char*, void**);
int be_rt_ring_unlink(const char*);
int be_rt_ring_shutdown(void*);
int be_rt_ring_close(void*);
int be_rt_ring_write(void*, const void*, const int64_t*, int, int64_t);
int be_rt_ring_next_len(void*, int64_t*, int64_t);
int be_rt_ring_read(void*, void*, int64_t);
int be_rt_ring_stats(void*, int64_t*);
}

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

static void test_watershed() {
  // 2-D: two markers in two valleys separated by a ridge at x = 8
  const int H = 12, W = 17;
  std::vector<float> img(H * W);
  std::vector<int> mk(H * W, 0), out(H * W, -1);
  std::vector<unsigned char> mask(H * W, 1);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) img[y * W + x] = x == 8 ? 10.f : float(std::abs(x - (x < 8 ? 3 : 13)));
  mk[5 * W + 3] = 1;
  mk[5 * W + 13] = 2;
  mask[0] = 0;
  CHECK(be_rt_watershed(img.data(), mk.data(), mask.data(), 1, H, W, 1, out.data()) == 0);
  CHECK(out[0] == 0);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      if (!mask[y * W + x]) continue;
      if (x < 8) CHECK(out[y * W + x] == 1);
      if (x > 8) CHECK(out[y * W + x] == 2);
    }
  // 3-D random, 26-connectivity, no mask
  const int D = 9, H3 = 13, W3 = 11, N = D * H3 * W3;
  std::mt19937 g(1);
  std::vector<float> im3(N);
  std::vector<int> m3(N, 0), o3(N);
  for (auto& v : im3) v = float(g() % 1000) / 7.f;
  for (int k = 1; k <= 6; ++k) m3[g() % N] = k;
  CHECK(be_rt_watershed(im3.data(), m3.data(), nullptr, D, H3, W3, 3, o3.data()) == 0);
  for (int i = 0; i < N; ++i) CHECK(o3[i] >= 1 && o3[i] <= 6);
}

static void test_spacing() {
  std::mt19937 g(7);
  for (int ndim = 2; ndim <= 3; ++ndim) {
    const int N = 500, sp = 5;
    std::vector<int> c(N * ndim);
    for (auto& v : c) v = int(g() % 60);
    std::vector<unsigned char> keep(N);
    CHECK(be_rt_ensure_spacing(c.data(), N, ndim, sp, keep.data()) == 0);
    std::vector<unsigned char> ref(N, 0);
    for (int i = 0; i < N; ++i) {
      bool ok = true;
      for (int j = 0; j < i && ok; ++j) {
        if (!ref[j]) continue;
        int cheb = 0;
        for (int d = 0; d < ndim; ++d) cheb = std::max(cheb, std::abs(c[i * ndim + d] - c[j * ndim + d]));
        if (cheb < sp) ok = false;
      }
      ref[i] = ok;
    }
    for (int i = 0; i < N; ++i) CHECK(keep[i] == ref[i]);
  }
}

static std::vector<unsigned char> payload(uint64_t seed, size_t n) {
  std::vector<unsigned char> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = (unsigned char)((seed * 131 + i * 7) & 0xff);
  return v;
}

static void produce(void* r, int msgs) {
  for (int m = 0; m < msgs; ++m) {
    const int nf = 1 + m % 3;
    std::vector<std::vector<unsigned char>> f(nf);
    std::vector<const void*> ptr(nf);
    std::vector<int64_t> len(nf);
    for (int i = 0; i < nf; ++i) {
      f[i] = payload(m * 3 + i, (size_t)((m * 977 + i * 131) % 20000));
      ptr[i] = f[i].data();
      len[i] = (int64_t)f[i].size();
    }
    CHECK(be_rt_ring_write(r, ptr.data(), len.data(), nf, 5000000) == 0);
  }
}

static void consume(void* r, int msgs) {
  std::vector<unsigned char> buf(1 << 16);
  for (int m = 0; m < msgs; ++m) {
    const int nf = 1 + m % 3;
    for (int i = 0; i < nf; ++i) {
      int64_t n = -1;
      CHECK(be_rt_ring_next_len(r, &n, 5000000) == 0);
      CHECK(n == (m * 977 + i * 131) % 20000);
      CHECK(be_rt_ring_read(r, buf.data(), (int64_t)buf.size()) == 0);
      auto ref = payload(m * 3 + i, (size_t)n);
      CHECK(n == 0 || std::memcmp(buf.data(), ref.data(), (size_t)n) == 0);
    }
  }
}

static void test_ring_threads() {
  std::string name = "/be-ring-selftest-t-" + std::to_string(getpid());
  void *w = nullptr, *r = nullptr;
  CHECK(be_rt_ring_create(name.c_str(), 1 << 16, &w) == 0);
  CHECK(be_rt_ring_open(name.c_str(), &r) == 0);
  CHECK(be_rt_ring_unlink(name.c_str()) == 0);
  const int msgs = 3000;
  std::thread c(consume, r, msgs);
  produce(w, msgs);
  c.join();
  int64_t st[5];
  CHECK(be_rt_ring_stats(w, st) == 0);
  CHECK(st[0] == 65536 && st[1] == 0 && st[2] == 6000);
  // edge cases: empty wait times out, oversized message refused, full ring times out, closed wakes
  int64_t n;
  CHECK(be_rt_ring_next_len(r, &n, 1000) == -2);
  std::vector<unsigned char> big(1 << 17);
  const void* bp = big.data();
  int64_t bl = (int64_t)big.size();
  CHECK(be_rt_ring_write(w, &bp, &bl, 1, 0) == -3);
  bl = 40000;
  CHECK(be_rt_ring_write(w, &bp, &bl, 1, 0) == 0);
  CHECK(be_rt_ring_write(w, &bp, &bl, 1, 1000) == -2);
  std::thread waiter([&] {
    int64_t l2 = 40000;
    CHECK(be_rt_ring_write(w, &bp, &l2, 1, -1) == -4);
  });
  usleep(20000);
  CHECK(be_rt_ring_shutdown(r) == 0);
  waiter.join();
  CHECK(be_rt_ring_close(r) == 0);
  CHECK(be_rt_ring_close(w) == 0);
}

// Frames past the parallel-copy threshold (512 KiB): the payload copies run on the helper pool, from
// the producer and the consumer thread at once, across the wrap point of a 4 MiB ring; then a
// forked child (whose pool must be its own: the parent's helper threads do not exist there)
// streams more of them back.
static void large_roundtrip(void* w, void* r, int msgs, uint64_t salt) {
  std::thread c([&] {
    std::vector<unsigned char> buf(3 << 20);
    for (int m = 0; m < msgs; ++m) {
      int64_t n = -1;
      CHECK(be_rt_ring_next_len(r, &n, 5000000) == 0);
      CHECK(n == (int64_t)((600 << 10) + (m * 104729) % (2 << 20)));
      CHECK(be_rt_ring_read(r, buf.data(), (int64_t)buf.size()) == 0);
      auto ref = payload(salt + m, (size_t)n);
      CHECK(std::memcmp(buf.data(), ref.data(), (size_t)n) == 0);
    }
  });
  for (int m = 0; m < msgs; ++m) {
    auto f = payload(salt + m, (size_t)((600 << 10) + (m * 104729) % (2 << 20)));
    const void* p = f.data();
    int64_t l = (int64_t)f.size();
    CHECK(be_rt_ring_write(w, &p, &l, 1, 5000000) == 0);
  }
  c.join();
}

static void test_ring_large(bool fork_ok) {
  std::string name = "/be-ring-selftest-l-" + std::to_string(getpid());
  void *w = nullptr, *r = nullptr;
  CHECK(be_rt_ring_create(name.c_str(), 4 << 20, &w) == 0);
  CHECK(be_rt_ring_open(name.c_str(), &r) == 0);
  large_roundtrip(w, r, 40, 11);
  if (fork_ok) {
    pid_t pid = fork();
    CHECK(pid >= 0);
    if (pid == 0) {
      large_roundtrip(w, r, 20, 77);
      _exit(0);
    }
    int status = 0;
    CHECK(waitpid(pid, &status, 0) == pid);
    CHECK(WIFEXITED(status) && WEXITSTATUS(status) == 0);
  }
  CHECK(be_rt_ring_unlink(name.c_str()) == 0);
  CHECK(be_rt_ring_close(r) == 0);
  CHECK(be_rt_ring_close(w) == 0);
}

static void test_ring_fork() {
  std::string name = "/be-ring-selftest-p-" + std::to_string(getpid());
  void* w = nullptr;
  CHECK(be_rt_ring_create(name.c_str(), 1 << 16, &w) == 0);
  const int msgs = 2000;
  pid_t pid = fork();
  CHECK(pid >= 0);
  if (pid == 0) {
    void* r = nullptr;
    if (be_rt_ring_open(name.c_str(), &r) != 0) _exit(3);
    consume(r, msgs);
    be_rt_ring_close(r);
    _exit(0);
  }
  produce(w, msgs);
  int status = 0;
  CHECK(waitpid(pid, &status, 0) == pid);
  CHECK(WIFEXITED(status) && WEXITSTATUS(status) == 0);
  CHECK(be_rt_ring_unlink(name.c_str()) == 0);
  CHECK(be_rt_ring_close(w) == 0);
}

int main(int argc, char** argv) {
  const bool fork_ok = !(argc > 1 && std::strcmp(argv[1], "--no-fork") == 0);
  test_watershed();
  test_spacing();
  test_ring_threads();
  if (fork_ok) test_ring_fork();
  test_ring_large(fork_ok);
  std::printf("runtime selftest ok\n");
  return 0;
}
