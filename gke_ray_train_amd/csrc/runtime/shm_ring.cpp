// Shared-memory SPSC ring buffer: the zero-copy hand-off of input batches between processes.
//
// Reference role: Ray's plasma object store + Ray Data's streaming_split feeding each training
// worker (the reference's DataLoader workers pickle every batch through a
// pipe, ray-jobs/pytorch_llm_ray.py:206-216). Here a producer process (the data pipeline)
// writes whole batches into fixed-size slots of a POSIX shared-memory segment and the training
// rank reads them in place (or memcpys them straight into a pinned staging buffer for the async
// H2D copy): no pickling, no per-batch syscalls, one segment per (producer, rank) pair.
//
// Layout: [Header (4 KiB)][slot 0][slot 1]...; slot = [uint64 nbytes][payload, slot_size bytes].
// head (next slot to write) and tail (next slot to read) are monotonically increasing 64-bit
// counters on separate cache lines; the producer publishes a slot with a release store of head,
// the consumer frees it with a release store of tail. Waiting spins briefly, then sleeps with an
// exponential backoff capped at 200 us (no futex: the segment may be mapped at different addresses,
// and the hand-off rate is a few thousand batches per second at most).
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <new>

namespace {

constexpr uint64_t kMagic = 0x47525452494e4731ull;  // "GRTRING1"
constexpr size_t kHeader = 4096;

struct alignas(64) Header {
  uint64_t magic;
  uint64_t slot_size;
  uint64_t n_slots;
  uint64_t total_bytes;
  alignas(64) std::atomic<uint64_t> head;
  alignas(64) std::atomic<uint64_t> tail;
  alignas(64) std::atomic<uint32_t> closed;
};

struct Ring {
  Header* h;
  char* base;
  size_t map_bytes;
  int owner;
};

inline char* slot_ptr(Ring* r, uint64_t idx) {
  return r->base + kHeader + (idx % r->h->n_slots) * (r->h->slot_size + 64);
}

inline int64_t now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

inline void backoff(int& spins) {
  if (spins < 64) {
    ++spins;
    return;
  }
  const long us = spins < 80 ? 2 : (spins < 120 ? 20 : 200);
  if (spins < 200) ++spins;
  timespec ts{0, us * 1000};
  nanosleep(&ts, nullptr);
}

// wait until pred() or timeout (ms, <0 = forever); returns 0 ok, -1 timeout, -2 closed
template <typename Pred>
int wait_for(Ring* r, Pred pred, int64_t timeout_ms, bool closed_aborts) {
  const int64_t t0 = timeout_ms >= 0 ? now_ms() : 0;
  int spins = 0;
  while (!pred()) {
    if (closed_aborts && r->h->closed.load(std::memory_order_acquire)) return -2;
    if (timeout_ms >= 0 && now_ms() - t0 > timeout_ms) return -1;
    backoff(spins);
  }
  return 0;
}

}  // namespace

extern "C" {

// Create (or replace) a ring named `name` (/dev/shm/<name>). Returns an opaque handle or null.
void* grt_ring_create(const char* name, uint64_t slot_size, uint64_t n_slots) {
  if (n_slots < 2 || slot_size == 0) return nullptr;
  slot_size = (slot_size + 63) / 64 * 64;
  const size_t bytes = kHeader + n_slots * (slot_size + 64);
  shm_unlink(name);
  int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return nullptr;
  if (ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    shm_unlink(name);
    return nullptr;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(name);
    return nullptr;
  }
  Header* h = new (p) Header();
  h->slot_size = slot_size;
  h->n_slots = n_slots;
  h->total_bytes = bytes;
  h->head.store(0, std::memory_order_relaxed);
  h->tail.store(0, std::memory_order_relaxed);
  h->closed.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  h->magic = kMagic;
  return new Ring{h, (char*)p, bytes, 1};
}

void* grt_ring_open(const char* name) {
  int fd = shm_open(name, O_RDWR, 0600);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < kHeader) {
    close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  Header* h = (Header*)p;
  if (h->magic != kMagic || h->total_bytes != (uint64_t)st.st_size) {
    munmap(p, (size_t)st.st_size);
    return nullptr;
  }
  return new Ring{h, (char*)p, (size_t)st.st_size, 0};
}

uint64_t grt_ring_slot_size(void* hd) { return ((Ring*)hd)->h->slot_size; }
uint64_t grt_ring_capacity(void* hd) { return ((Ring*)hd)->h->n_slots; }
uint64_t grt_ring_size(void* hd) {
  Ring* r = (Ring*)hd;
  return r->h->head.load(std::memory_order_acquire) - r->h->tail.load(std::memory_order_acquire);
}

// Producer, zero-copy: pointer to the next free slot's payload (wait up to timeout_ms), or null
// with *err = -1 timeout / -2 closed.
void* grt_ring_acquire_write(void* hd, int64_t timeout_ms, int* err) {
  Ring* r = (Ring*)hd;
  const uint64_t head = r->h->head.load(std::memory_order_relaxed);
  const int rc = wait_for(r, [&] { return head - r->h->tail.load(std::memory_order_acquire) < r->h->n_slots; },
                          timeout_ms, true);
  if (err) *err = rc;
  if (rc != 0) return nullptr;
  return slot_ptr(r, head) + 64;
}

int grt_ring_commit_write(void* hd, uint64_t nbytes) {
  Ring* r = (Ring*)hd;
  if (nbytes > r->h->slot_size) return -3;
  const uint64_t head = r->h->head.load(std::memory_order_relaxed);
  *(uint64_t*)slot_ptr(r, head) = nbytes;
  r->h->head.store(head + 1, std::memory_order_release);
  return 0;
}

int grt_ring_push(void* hd, const void* data, uint64_t nbytes, int64_t timeout_ms) {
  Ring* r = (Ring*)hd;
  if (nbytes > r->h->slot_size) return -3;
  int err = 0;
  void* dst = grt_ring_acquire_write(hd, timeout_ms, &err);
  if (!dst) return err;
  memcpy(dst, data, nbytes);
  return grt_ring_commit_write(hd, nbytes);
}

// Consumer, zero-copy: payload pointer of the oldest filled slot (its size in *nbytes); the slot
// stays owned by the reader until grt_ring_release_read. Null with *err = -1 timeout / -2 closed
// and drained.
const void* grt_ring_acquire_read(void* hd, int64_t timeout_ms, uint64_t* nbytes, int* err) {
  Ring* r = (Ring*)hd;
  const uint64_t tail = r->h->tail.load(std::memory_order_relaxed);
  const int64_t t0 = timeout_ms >= 0 ? now_ms() : 0;
  int spins = 0;
  while (r->h->head.load(std::memory_order_acquire) <= tail) {
    // closed only ends the stream once it is drained
    if (r->h->closed.load(std::memory_order_acquire) && r->h->head.load(std::memory_order_acquire) <= tail) {
      if (err) *err = -2;
      return nullptr;
    }
    if (timeout_ms >= 0 && now_ms() - t0 > timeout_ms) {
      if (err) *err = -1;
      return nullptr;
    }
    backoff(spins);
  }
  if (err) *err = 0;
  const char* s = slot_ptr(r, tail);
  if (nbytes) *nbytes = *(const uint64_t*)s;
  return s + 64;
}

int grt_ring_release_read(void* hd) {
  Ring* r = (Ring*)hd;
  const uint64_t tail = r->h->tail.load(std::memory_order_relaxed);
  if (r->h->head.load(std::memory_order_acquire) <= tail) return -1;
  r->h->tail.store(tail + 1, std::memory_order_release);
  return 0;
}

// Copying pop; returns payload size, or -1 timeout, -2 closed and drained, -3 buffer too small.
int64_t grt_ring_pop(void* hd, void* out, uint64_t cap, int64_t timeout_ms) {
  Ring* r = (Ring*)hd;
  const uint64_t tail = r->h->tail.load(std::memory_order_relaxed);
  const int64_t t0 = timeout_ms >= 0 ? now_ms() : 0;
  int spins = 0;
  while (r->h->head.load(std::memory_order_acquire) <= tail) {
    if (r->h->closed.load(std::memory_order_acquire) && r->h->head.load(std::memory_order_acquire) <= tail)
      return -2;
    if (timeout_ms >= 0 && now_ms() - t0 > timeout_ms) return -1;
    backoff(spins);
  }
  const char* s = slot_ptr(r, tail);
  const uint64_t n = *(const uint64_t*)s;
  if (n > cap) return -3;
  memcpy(out, s + 64, n);
  r->h->tail.store(tail + 1, std::memory_order_release);
  return (int64_t)n;
}

void grt_ring_close(void* hd) { ((Ring*)hd)->h->closed.store(1, std::memory_order_release); }
int grt_ring_closed(void* hd) { return (int)((Ring*)hd)->h->closed.load(std::memory_order_acquire); }

// Unmap; `unlink` also removes the segment name (creator side, at the end of the run).
void grt_ring_destroy(void* hd, const char* name, int unlink_name) {
  Ring* r = (Ring*)hd;
  if (!r) return;
  munmap(r->base, r->map_bytes);
  if (unlink_name && name) shm_unlink(name);
  delete r;
}

}  // extern "C"
