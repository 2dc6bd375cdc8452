// Host-side race / memory-error stress of the native runtime: built by
// tests/test_build.py with -fsanitize=thread and, separately, -fsanitize=address,undefined, and
// run on the CPU (GPU sanitizers are not available; the runtime has no device code).
//
// * shared-memory SPSC ring: a producer thread and a consumer thread on two independent mappings
//   of one segment (as two processes would have), mixing copying push/pop with the zero-copy
//   acquire/commit and acquire/release paths, backpressure on a 4-slot ring, payload integrity
//   (sequence + checksum per message), timeout and close-drains-then-ends semantics;
// * batch gather (multi-threaded window copy) and pad-collate on random shapes, checked exactly.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

extern "C" {
void* grt_ring_create(const char* name, uint64_t slot_size, uint64_t n_slots);
void* grt_ring_open(const char* name);
void* grt_ring_acquire_write(void* hd, int64_t timeout_ms, int* err);
int grt_ring_commit_write(void* hd, uint64_t nbytes);
int grt_ring_push(void* hd, const void* data, uint64_t nbytes, int64_t timeout_ms);
const void* grt_ring_acquire_read(void* hd, int64_t timeout_ms, uint64_t* nbytes, int* err);
int grt_ring_release_read(void* hd);
int64_t grt_ring_pop(void* hd, void* out, uint64_t cap, int64_t timeout_ms);
void grt_ring_close(void* hd);
void grt_ring_destroy(void* hd, const char* name, int unlink_name);
int grt_gather_windows_i64(const int64_t* tokens, int64_t n, const int64_t* starts, int64_t B, int64_t S,
                           int64_t* out_x, int64_t* out_y, int nthreads);
int grt_gather_windows_i32(const int32_t* tokens, int64_t n, const int64_t* starts, int64_t B, int64_t S,
                           int64_t* out_x, int64_t* out_y, int nthreads);
int grt_pad_collate(const int64_t* flat, const int64_t* offsets, const int64_t* prompt_len, int64_t B, int64_t S,
                    int64_t pad_id, int64_t* ids, int64_t* labels, int64_t* mask);
}

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

static uint64_t fill(uint8_t* p, uint64_t seq, uint64_t n) {
  uint64_t sum = 0;
  for (uint64_t i = 0; i < n; ++i) {
    p[i] = (uint8_t)((seq * 131 + i * 7) & 0xff);
    sum += p[i];
  }
  return sum;
}

static void ring_stress(int messages) {
  char name[64];
  snprintf(name, sizeof name, "/grt_sanitize_%d", (int)getpid());
  const uint64_t slot = 4096;
  void* prod = grt_ring_create(name, slot, 4);
  CHECK(prod);
  void* cons = grt_ring_open(name);
  CHECK(cons);
  // empty ring: a bounded read times out
  int err = 0;
  CHECK(grt_ring_acquire_read(cons, 5, nullptr, &err) == nullptr && err == -1);

  std::thread producer([&] {
    std::vector<uint8_t> buf(slot);
    for (int s = 0; s < messages; ++s) {
      const uint64_t n = 16 + (uint64_t)(s * 97) % (slot - 16);
      if (s % 2 == 0) {  // zero-copy write
        int e = 0;
        uint8_t* dst = (uint8_t*)grt_ring_acquire_write(prod, 10000, &e);
        CHECK(dst && e == 0);
        memcpy(dst, &s, sizeof s);
        fill(dst + 8, (uint64_t)s, n - 8);
        CHECK(grt_ring_commit_write(prod, n) == 0);
      } else {
        memcpy(buf.data(), &s, sizeof s);
        fill(buf.data() + 8, (uint64_t)s, n - 8);
        CHECK(grt_ring_push(prod, buf.data(), n, 10000) == 0);
      }
    }
    grt_ring_close(prod);
  });

  std::vector<uint8_t> out(slot), ref(slot);
  int got = 0;
  for (;;) {
    uint64_t n = 0;
    const uint8_t* p = nullptr;
    int64_t rc = 0;
    if (got % 3 == 0) {  // zero-copy read
      int e = 0;
      p = (const uint8_t*)grt_ring_acquire_read(cons, 10000, &n, &e);
      if (!p) {
        CHECK(e == -2);
        break;
      }
    } else {
      rc = grt_ring_pop(cons, out.data(), out.size(), 10000);
      if (rc == -2) break;
      CHECK(rc > 0);
      n = (uint64_t)rc;
      p = out.data();
    }
    int seq = -1;
    memcpy(&seq, p, sizeof seq);
    CHECK(seq == got);
    CHECK(n == 16 + (uint64_t)(got * 97) % (slot - 16));
    fill(ref.data(), (uint64_t)got, n - 8);
    CHECK(memcmp(ref.data(), p + 8, n - 8) == 0);
    if (got % 3 == 0) CHECK(grt_ring_release_read(cons) == 0);
    ++got;
  }
  producer.join();
  CHECK(got == messages);
  grt_ring_destroy(cons, name, 0);
  grt_ring_destroy(prod, name, 1);
}

static void gather_stress(std::mt19937_64& rng) {
  for (int it = 0; it < 20; ++it) {
    const int64_t n = 5000 + rng() % 100000, S = 1 + rng() % 300, B = 1 + rng() % 64;
    std::vector<int64_t> tok(n);
    std::vector<int32_t> tok32(n);
    for (int64_t i = 0; i < n; ++i) tok32[i] = (int32_t)(tok[i] = (int64_t)(rng() % 50000));
    std::vector<int64_t> st(B), x(B * S), y(B * S), x2(B * S), y2(B * S);
    for (auto& s : st) s = (int64_t)(rng() % (uint64_t)(n - S - 1));
    const int nth = 1 + (int)(rng() % 8);
    CHECK(grt_gather_windows_i64(tok.data(), n, st.data(), B, S, x.data(), y.data(), nth) == 0);
    CHECK(grt_gather_windows_i32(tok32.data(), n, st.data(), B, S, x2.data(), y2.data(), nth) == 0);
    for (int64_t b = 0; b < B; ++b)
      for (int64_t i = 0; i < S; ++i) {
        CHECK(x[b * S + i] == tok[st[b] + i] && y[b * S + i] == tok[st[b] + i + 1]);
        CHECK(x2[b * S + i] == x[b * S + i] && y2[b * S + i] == y[b * S + i]);
      }
    st[0] = n - S;  // runs one past the end: rejected without touching memory
    CHECK(grt_gather_windows_i64(tok.data(), n, st.data(), B, S, x.data(), y.data(), nth) == -1);
    // pad-collate
    std::vector<int64_t> off(B + 1, 0), pl(B);
    for (int64_t b = 0; b < B; ++b) {
      off[b + 1] = off[b] + (int64_t)(rng() % (uint64_t)(2 * S));
      pl[b] = (int64_t)(rng() % (uint64_t)(S + 1));
    }
    std::vector<int64_t> flat(off[B] + 1), ids(B * S), lab(B * S), msk(B * S);
    for (auto& v : flat) v = (int64_t)(rng() % 1000);
    CHECK(grt_pad_collate(flat.data(), off.data(), pl.data(), B, S, -7, ids.data(), lab.data(), msk.data()) == 0);
    for (int64_t b = 0; b < B; ++b) {
      const int64_t len = std::min<int64_t>(off[b + 1] - off[b], S);
      for (int64_t i = 0; i < S; ++i) {
        const bool v = i < len;
        CHECK(ids[b * S + i] == (v ? flat[off[b] + i] : -7));
        CHECK(msk[b * S + i] == (v ? 1 : 0));
        CHECK(lab[b * S + i] == ((v && i >= pl[b]) ? flat[off[b] + i] : -100));
      }
    }
  }
}

int main(int argc, char** argv) {
  const int messages = argc > 1 ? atoi(argv[1]) : 20000;
  std::mt19937_64 rng(1234);
  ring_stress(messages);
  gather_stress(rng);
  printf("sanitize_stress ok (%d ring messages)\n", messages);
  return 0;
}
