// Cross-process single-producer / single-consumer byte ring in POSIX shared memory.
//
// Used as the bulk-data lane between the serving router (worker process) and the per-GPU replica
// processes (bioengine_worker_amd/serve/replica.py): the Unix-socket connection carries the small
// pickle header of each request/result, the out-of-band tensor/ndarray buffers travel through two of
// these rings (router->replica, replica->router).  This replaces what the reference does with Ray's
// plasma object store between the proxy/entry/runtime deployments (SURVEY.md §2.6 C4, §5 "Distributed
// communication backend" (b); reference bioengine/apps/proxy_deployment.py:522-554).
//
// Layout: one 4 KiB header page (magic, capacity, producer/consumer cursors on separate cache
// lines, two futex words) followed by `capacity` data bytes (power of two).  A message is a run of
// frames [u64 length][payload, padded to 8 bytes]; cursors are monotonically increasing 64-bit
// byte counts, so full/empty need no extra flag and a frame header never straddles the wrap point
// (every position is 8-aligned and the capacity is a multiple of 8).  Payload copies split at the
// wrap into at most two memcpys.
//
// Blocking: the producer waits on `space_seq`, the consumer on `data_seq`, with a short spin and then
// FUTEX_WAIT on the shared mapping (not FUTEX_PRIVATE: the waiter and the waker are different
// processes).  Every publish/consume bumps the sequence word and issues FUTEX_WAKE.
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <mutex>
#include <thread>
#include <linux/futex.h>
#include <new>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

namespace {

constexpr uint64_t kMagic = 0x42455249'4e473031ull;  // "BERING01"
constexpr int64_t kHeader = 4096;

struct alignas(64) Header {
  uint64_t magic;
  uint64_t capacity;
  alignas(64) std::atomic<uint64_t> head;  // producer cursor (bytes published)
  alignas(64) std::atomic<uint64_t> tail;  // consumer cursor (bytes released)
  alignas(64) std::atomic<uint32_t> data_seq;
  alignas(64) std::atomic<uint32_t> space_seq;
  alignas(64) std::atomic<uint64_t> frames_written;
  std::atomic<uint64_t> bytes_written;
  std::atomic<uint32_t> closed;
};
static_assert(sizeof(Header) <= kHeader, "header page");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "lock-free 64-bit atomics across processes");

struct Ring {
  Header* h;
  unsigned char* data;
  uint64_t mask;
  size_t map_len;
};

inline uint64_t align8(uint64_t v) { return (v + 7) & ~uint64_t(7); }

long futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

void wake(std::atomic<uint32_t>* seq) {
  seq->fetch_add(1, std::memory_order_release);
  futex(seq, FUTEX_WAKE, INT32_MAX, nullptr);
}

// Wait until pred() holds; returns 0, or -2 on timeout (timeout_us < 0 = forever), -4 if closed.
template <class Pred>
int wait_for(Ring* r, std::atomic<uint32_t>* seq, int64_t timeout_us, Pred pred) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (int spin = 0; spin < 256; ++spin) {
    if (pred()) return 0;
  }
  for (;;) {
    uint32_t s = seq->load(std::memory_order_acquire);
    if (pred()) return 0;
    if (r->h->closed.load(std::memory_order_acquire)) return -4;
    timespec ts{0, 50 * 1000 * 1000};  // re-check at least every 50 ms (closed flag, timeout)
    if (timeout_us >= 0) {
      int64_t left = timeout_us - std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t0).count();
      if (left <= 0) return -2;
      if (left < 50000) ts = timespec{0, static_cast<long>(left) * 1000};
    }
    futex(seq, FUTEX_WAIT, s, &ts);
  }
}

// Large payload copies are split over the calling thread plus a few persistent helpers: one core's
// memcpy of a 2 MiB image is ~0.1-0.2 ms, on the critical path of every served request (once into
// the ring in the sender, once out in the receiver).  BE_RING_COPY_THREADS (default 4, 1 = off) is
// the total number of threads per copy; helpers sleep on a condition variable between copies.
constexpr uint64_t kParMin = 512 << 10;

struct CopyPool {
  std::mutex use;  // one parallel copy at a time per process
  std::mutex mu;
  std::condition_variable cv;
  unsigned char* dst = nullptr;
  const unsigned char* src = nullptr;
  uint64_t chunk = 0, n = 0;
  uint64_t gen = 0;
  std::atomic<int> pending{0};
  int helpers = 0;
  pid_t pid = 0;
};

int copy_threads() {
  static const int t = [] {
    const char* e = getenv("BE_RING_COPY_THREADS");
    const int v = e ? atoi(e) : 4;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  return t;
}

void helper_main(CopyPool* p, int idx) {
  uint64_t seen = 0;
  for (;;) {
    unsigned char* d;
    const unsigned char* s;
    uint64_t lo, hi;
    {
      std::unique_lock<std::mutex> lk(p->mu);
      p->cv.wait(lk, [&] { return p->gen != seen; });
      seen = p->gen;
      d = p->dst;
      s = p->src;
      lo = (uint64_t)(idx + 1) * p->chunk;
      hi = lo + p->chunk < p->n ? lo + p->chunk : p->n;
    }
    if (lo < hi) std::memcpy(d + lo, s + lo, hi - lo);
    p->pending.fetch_sub(1, std::memory_order_acq_rel);
  }
}

// One pool per process (a forked child starts its own: the parent's helper threads do not exist
// there, and the parent's mutexes may have been held at the fork).  Copies are serialised by the
// pool's `use`: the ring's two directions may copy from two threads.
CopyPool* pool() {
  static std::mutex init_mu;
  static CopyPool* p = nullptr;
  std::lock_guard<std::mutex> g(init_mu);
  if (p == nullptr || p->pid != getpid()) {
    p = new CopyPool;  // a pre-fork pool is leaked on purpose: its mutex may be held by a dead thread
    p->pid = getpid();
    p->helpers = copy_threads() - 1;
    for (int i = 0; i < p->helpers; ++i) std::thread(helper_main, p, i).detach();
  }
  return p;
}

void par_memcpy(void* dst, const void* src, uint64_t n) {
  if (n < kParMin || copy_threads() <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  CopyPool* p = pool();
  std::lock_guard<std::mutex> g(p->use);
  const int parts = p->helpers + 1;
  const uint64_t chunk = ((n + parts - 1) / parts + 63) & ~uint64_t(63);
  {
    std::lock_guard<std::mutex> lk(p->mu);
    p->dst = static_cast<unsigned char*>(dst);
    p->src = static_cast<const unsigned char*>(src);
    p->chunk = chunk;
    p->n = n;
    p->pending.store(p->helpers, std::memory_order_relaxed);
    ++p->gen;
  }
  p->cv.notify_all();
  std::memcpy(dst, src, chunk < n ? chunk : n);
  while (p->pending.load(std::memory_order_acquire) > 0) std::this_thread::yield();
}

void copy_in(Ring* r, uint64_t pos, const void* src, uint64_t n) {
  uint64_t off = pos & r->mask;
  uint64_t first = r->mask + 1 - off;
  if (first >= n) {
    par_memcpy(r->data + off, src, n);
  } else {
    par_memcpy(r->data + off, src, first);
    par_memcpy(r->data, static_cast<const unsigned char*>(src) + first, n - first);
  }
}

void copy_out(Ring* r, uint64_t pos, void* dst, uint64_t n) {
  uint64_t off = pos & r->mask;
  uint64_t first = r->mask + 1 - off;
  if (first >= n) {
    par_memcpy(dst, r->data + off, n);
  } else {
    par_memcpy(dst, r->data + off, first);
    par_memcpy(static_cast<unsigned char*>(dst) + first, r->data, n - first);
  }
}

// populate: pre-fault the whole mapping (MAP_POPULATE).  A ring is written front to back, so until it
// first wraps every message lands on pages this process has never touched; on the VM hosts the
// serving boxes run on a first touch costs ~1 ms per MiB (measured: a 1 MiB echo through a cold
// 512 MiB ring 4.3 ms vs 0.75 ms for 4 KiB), more than the copy itself.
int map_ring(int fd, size_t len, Ring** out, bool populate) {
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, 0);
  if (p == MAP_FAILED) return -errno;
  Ring* r = new (std::nothrow) Ring;
  if (!r) {
    munmap(p, len);
    return -ENOMEM;
  }
  r->h = static_cast<Header*>(p);
  r->data = static_cast<unsigned char*>(p) + kHeader;
  r->map_len = len;
  r->mask = 0;
  *out = r;
  return 0;
}

}  // namespace

extern "C" {

// Create the segment `name` ("/be-ring-..."), capacity rounded up to a power of two >= 64 KiB.
int be_rt_ring_create(const char* name, int64_t capacity, void** out, int populate) {
  if (!name || !out || capacity <= 0) return -EINVAL;
  uint64_t cap = 65536;
  while (cap < static_cast<uint64_t>(capacity)) cap <<= 1;
  int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return -errno;
  size_t len = kHeader + cap;
  if (ftruncate(fd, static_cast<off_t>(len)) != 0) {
    int e = errno;
    close(fd);
    shm_unlink(name);
    return -e;
  }
  Ring* r = nullptr;
  int rc = map_ring(fd, len, &r, populate != 0);
  close(fd);
  if (rc != 0) {
    shm_unlink(name);
    return rc;
  }
  Header* h = new (r->h) Header();  // value-initialises the atomics in place
  h->capacity = cap;
  r->mask = cap - 1;
  std::atomic_thread_fence(std::memory_order_release);
  h->magic = kMagic;
  *out = r;
  return 0;
}

int be_rt_ring_open(const char* name, void** out, int populate) {
  if (!name || !out) return -EINVAL;
  int fd = shm_open(name, O_RDWR, 0600);
  if (fd < 0) return -errno;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < kHeader) {
    close(fd);
    return -EINVAL;
  }
  Ring* r = nullptr;
  int rc = map_ring(fd, static_cast<size_t>(st.st_size), &r, populate != 0);
  close(fd);
  if (rc != 0) return rc;
  if (r->h->magic != kMagic || kHeader + r->h->capacity != static_cast<uint64_t>(st.st_size)) {
    munmap(r->h, r->map_len);
    delete r;
    return -EINVAL;
  }
  r->mask = r->h->capacity - 1;
  *out = r;
  return 0;
}

int be_rt_ring_unlink(const char* name) { return shm_unlink(name) == 0 ? 0 : -errno; }

// Mark closed (wakes both sides: pending waits return -4) without unmapping.
int be_rt_ring_shutdown(void* ring) {
  Ring* r = static_cast<Ring*>(ring);
  if (!r) return -EINVAL;
  r->h->closed.store(1, std::memory_order_release);
  wake(&r->h->data_seq);
  wake(&r->h->space_seq);
  return 0;
}

int be_rt_ring_close(void* ring) {
  Ring* r = static_cast<Ring*>(ring);
  if (!r) return -EINVAL;
  munmap(r->h, r->map_len);
  delete r;
  return 0;
}

// Bytes one message of n payloads of the given lengths occupies in the ring.
int be_rt_ring_message_bytes(const int64_t* lens, int n, int64_t* out) {
  if (!out || n < 0 || (n > 0 && !lens)) return -EINVAL;
  uint64_t total = 0;
  for (int i = 0; i < n; ++i) {
    if (lens[i] < 0) return -EINVAL;
    total += 8 + align8(static_cast<uint64_t>(lens[i]));
  }
  *out = static_cast<int64_t>(total);
  return 0;
}

// Producer: publish one message of n frames (bufs[i], lens[i]) atomically — the consumer sees all
// of them or none.  Returns 0, -2 timeout, -3 message larger than the ring, -4 closed.
int be_rt_ring_write(void* ring, const void* bufs, const int64_t* lens, int n, int64_t timeout_us) {
  Ring* r = static_cast<Ring*>(ring);
  if (!r || (n > 0 && (!bufs || !lens))) return -EINVAL;
  const void* const* b = static_cast<const void* const*>(bufs);
  int64_t need = 0;
  if (be_rt_ring_message_bytes(lens, n, &need) != 0) return -EINVAL;
  const uint64_t cap = r->mask + 1;
  if (static_cast<uint64_t>(need) > cap) return -3;
  Header* h = r->h;
  if (h->closed.load(std::memory_order_acquire)) return -4;
  const uint64_t head = h->head.load(std::memory_order_relaxed);
  int rc = wait_for(r, &h->space_seq, timeout_us, [&] {
    return head + static_cast<uint64_t>(need) - h->tail.load(std::memory_order_acquire) <= cap;
  });
  if (rc != 0) return rc;
  uint64_t pos = head;
  for (int i = 0; i < n; ++i) {
    uint64_t len = static_cast<uint64_t>(lens[i]);
    std::memcpy(r->data + (pos & r->mask), &len, 8);
    pos += 8;
    if (len) copy_in(r, pos, b[i], len);
    pos += align8(len);
  }
  h->frames_written.fetch_add(static_cast<uint64_t>(n), std::memory_order_relaxed);
  h->bytes_written.fetch_add(static_cast<uint64_t>(need), std::memory_order_relaxed);
  h->head.store(pos, std::memory_order_release);
  wake(&h->data_seq);
  return 0;
}

// Consumer: wait for the next frame and report its payload length (the frame stays queued until
// be_rt_ring_read).  Returns 0, -2 timeout, -4 closed and drained.
int be_rt_ring_next_len(void* ring, int64_t* len, int64_t timeout_us) {
  Ring* r = static_cast<Ring*>(ring);
  if (!r || !len) return -EINVAL;
  Header* h = r->h;
  const uint64_t tail = h->tail.load(std::memory_order_relaxed);
  int rc = wait_for(r, &h->data_seq, timeout_us, [&] { return h->head.load(std::memory_order_acquire) != tail; });
  if (rc != 0) return rc;
  uint64_t l;
  std::memcpy(&l, r->data + (tail & r->mask), 8);
  *len = static_cast<int64_t>(l);
  return 0;
}

// Consumer: copy the next frame (announced by be_rt_ring_next_len) into dst (cap >= its length)
// and release its space to the producer.
int be_rt_ring_read(void* ring, void* dst, int64_t cap) {
  Ring* r = static_cast<Ring*>(ring);
  if (!r) return -EINVAL;
  Header* h = r->h;
  const uint64_t tail = h->tail.load(std::memory_order_relaxed);
  if (h->head.load(std::memory_order_acquire) == tail) return -5;  // nothing queued
  uint64_t l;
  std::memcpy(&l, r->data + (tail & r->mask), 8);
  if (static_cast<uint64_t>(cap) < l || (l && !dst)) return -EINVAL;
  if (l) copy_out(r, tail + 8, dst, l);
  h->tail.store(tail + 8 + align8(l), std::memory_order_release);
  wake(&h->space_seq);
  return 0;
}

// out[0..4] = capacity, bytes queued, frames written, bytes written (lifetime), closed
int be_rt_ring_stats(void* ring, int64_t* out) {
  Ring* r = static_cast<Ring*>(ring);
  if (!r || !out) return -EINVAL;
  Header* h = r->h;
  out[0] = static_cast<int64_t>(h->capacity);
  out[1] = static_cast<int64_t>(h->head.load(std::memory_order_acquire) - h->tail.load(std::memory_order_acquire));
  out[2] = static_cast<int64_t>(h->frames_written.load(std::memory_order_relaxed));
  out[3] = static_cast<int64_t>(h->bytes_written.load(std::memory_order_relaxed));
  out[4] = static_cast<int64_t>(h->closed.load(std::memory_order_relaxed));
  return 0;
}

}  // extern "C"
