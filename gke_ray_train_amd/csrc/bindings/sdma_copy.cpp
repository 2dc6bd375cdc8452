// Device -> host copies on the SDMA engines, ordered with HIP streams.
//
// Why: on this ROCm image every device -> pinned-host copy that goes through HIP runs as a ROCclr
// blit kernel on the compute units, whatever the allocation type, copy kind (even
// hipMemcpyDeviceToDeviceNoCU) or engine knob (profiles/r6_offload_link.md). The offloaded AdamW
// (parallel/offload.py) writes its moments back to the host every step, so those blit kernels
// compete with the update and the forward GEMMs for CUs. The HSA runtime's async copy takes an
// SDMA engine for a copy between two different agents (GPU -> CPU), but it is not stream-ordered.
//
// Ordering (one worker thread per device):
//   d2h() on the caller's stream: records an event after the producer, queues a job, and makes the
//   stream wait (hipStreamWaitValue32, GTE) on a pinned host word until the worker has stored the
//   job's sequence number there. Work enqueued on the stream afterwards — or on any stream that
//   waits for an event recorded there afterwards — therefore runs after the copy has landed, as
//   with a stream-ordered copy.
//   worker: hipEventSynchronize(ready) -> hsa_amd_memory_async_copy_on_engine
//   (dst, cpu, src, gpu) with a completion signal -> wait bounded at 10 s + 1 s per GB -> store seq
//   (release). A failed or timed-out copy still stores seq (the stream must not hang) and leaves a
//   sticky error (sdma_stats()['error'], raised by the offloaded optimizer at its next step /
//   synchronize); every later copy then releases its stream at once instead of queueing behind it.
// Coherence: the event marker after the producer releases to system scope (L2 written back), so
// the SDMA engine reads the producer's data from memory; the host destination is read by later
// SDMA host -> device copies or by the CPU after a stream synchronisation.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "grt_sdma.h"

namespace grt {
namespace {

struct Job {
  hipEvent_t ready;
  void* dst;
  const void* src;
  size_t bytes;
  uint32_t seq;
};

hsa_status_t find_cpu(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(data) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

class Copier {
 public:
  explicit Copier(int dev) : dev_(dev) {
    const char* tr = getenv("GRT_SDMA_TRACE");  // 1: one stderr line per submitted / finished copy
    trace_ = tr && atoi(tr) != 0;
    if (hsa_init() != HSA_STATUS_SUCCESS) throw std::runtime_error("sdma: hsa_init failed");
    if (hsa_iterate_agents(find_cpu, &cpu_) != HSA_STATUS_INFO_BREAK) throw std::runtime_error("sdma: no CPU agent");
    if (hsa_signal_create(1, 0, nullptr, &sig_) != HSA_STATUS_SUCCESS) throw std::runtime_error("sdma: signal");
    void* f = nullptr;
    if (hipHostMalloc(&f, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
      throw std::runtime_error("sdma: hipHostMalloc of the completion word");
    flag_ = static_cast<uint32_t*>(f);
    __atomic_store_n(flag_, 0u, __ATOMIC_RELEASE);
    worker_ = std::thread([this] { run(); });
    worker_.detach();  // lives as long as the process (no teardown ordering against the HIP runtime)
  }

  void d2h(void* dst, const void* src, size_t bytes, hipStream_t s, hipStream_t producer) {
    std::lock_guard<std::mutex> g(submit_mu_);  // sequence numbers follow submission order
    if (!gpu_known_) {
      hsa_amd_pointer_info_t info{};
      info.size = sizeof(info);
      if (hsa_amd_pointer_info(const_cast<void*>(src), &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
          info.type == HSA_EXT_POINTER_TYPE_UNKNOWN || info.type == HSA_EXT_POINTER_TYPE_LOCKED)
        throw std::runtime_error("sdma_d2h: the source is not device memory of this process");
      gpu_ = info.agentOwner;
      gpu_known_ = true;
      pick_engine();
    }
    // the producer event is recorded on the producer's own stream when one is given: an event recorded
    // on `s` behind a cross-stream wait let copies read moments their update had not yet written
    // (full GPU suite with GRT_OFFLOAD_D2H=sdma, gpurun_out/r6sdma3)
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(ev, producer ? producer : s) != hipSuccess)
      throw std::runtime_error("sdma_d2h: event record failed");
    const uint32_t seq = ++next_seq_;
    if (trace_) fprintf(stderr, "sdma: submit seq=%u bytes=%zu\n", seq, bytes);
    {
      std::lock_guard<std::mutex> q(mu_);
      q_.push_back(Job{ev, dst, src, bytes, seq});
    }
    cv_.notify_one();
    if (hipStreamWaitValue32(s, flag_, seq, hipStreamWaitValueGte, 0xffffffffu) != hipSuccess)
      throw std::runtime_error("sdma_d2h: hipStreamWaitValue32 failed");
  }

  SdmaStats stats() {
    SdmaStats st;
    st.engine = engine_;
    st.engines_available = avail_;
    st.engines_preferred = pref_;
    st.copies = copies_.load();
    st.bytes = bytes_.load();
    st.busy_ns = busy_ns_.load();
    std::lock_guard<std::mutex> g(err_mu_);
    st.error = err_;
    return st;
  }

  void clear_error() {
    std::lock_guard<std::mutex> g(err_mu_);
    err_.clear();
    failed_ = false;
  }

 private:
  // GRT_SDMA_ENGINE: "auto" lets the HSA runtime assign the engine per copy; a number n pins engine n.
  // Default 2: engines 1-3 move device -> host at ~56 GB/s on MI355X, 8 and 15 at 7-9 GB/s
  // (xGMI-side engines; gpurun_out/r6sdmaeng). With runtime-assigned engines, shared with the HIP
  // runtime's own host -> device SDMA copies, one copy at full 70B offload depth never completed
  // (profiles/r6_offload_link.md); a pinned engine of our own avoids that.
  void pick_engine() {
    (void)hsa_amd_memory_copy_engine_status(cpu_, gpu_, &avail_);
    (void)hsa_amd_memory_get_preferred_copy_engine(cpu_, gpu_, &pref_);
    const char* e = getenv("GRT_SDMA_ENGINE");
    const std::string v = e ? e : "2";
    engine_ = v == "auto" ? 0u : 1u << (unsigned)atoi(v.c_str());
    if (engine_ && !(avail_ & engine_)) {  // not available for this direction: let the runtime pick
      if (trace_) fprintf(stderr, "sdma: engine 0x%x not in 0x%x, runtime-assigned\n", engine_, avail_);
      engine_ = 0;
    }
    if (trace_) fprintf(stderr, "sdma: engines available 0x%x preferred 0x%x using 0x%x\n", avail_, pref_, engine_);
  }

  void fail(const std::string& m) {
    std::lock_guard<std::mutex> g(err_mu_);
    if (err_.empty()) err_ = m;
    failed_ = true;
  }

  void run() {
    (void)hipSetDevice(dev_);
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> q(mu_);
        cv_.wait(q, [this] { return !q_.empty(); });
        j = q_.front();
        q_.pop_front();
      }
      const auto tq = std::chrono::steady_clock::now();
      // the producer. (Polling hipEventQuery from this thread instead let copies start before their
      // producer finished: the parity test read stale moments, gpurun_out/r6sdma3.)
      const hipError_t e = hipEventSynchronize(j.ready);
      (void)hipEventDestroy(j.ready);
      const auto t0 = std::chrono::steady_clock::now();
      if (failed_) {
        // an earlier copy failed: release the stream at once (the error is already recorded and the
        // host raises at its next check) instead of stalling every later copy behind a stuck engine
      } else if (e != hipSuccess) {
        fail(std::string("producer event failed: ") + hipGetErrorString(e));
      } else {
        hsa_signal_store_screlease(sig_, 1);
        const hsa_status_t st =
            engine_ ? hsa_amd_memory_async_copy_on_engine(j.dst, cpu_, j.src, gpu_, j.bytes, 0, nullptr, sig_,
                                                          (hsa_amd_sdma_engine_id_t)engine_, true)
                    : hsa_amd_memory_async_copy(j.dst, cpu_, j.src, gpu_, j.bytes, 0, nullptr, sig_);
        if (st != HSA_STATUS_SUCCESS) {
          fail("hsa_amd_memory_async_copy returned " + std::to_string((int)st));
        } else {
          // bounded: 10 s + 1 s per GB (the link moves ~56 GB/s) releases the stream with an error
          const uint64_t limit_ns = 10000000000ull + (uint64_t)j.bytes;
          const hsa_signal_value_t v = hsa_signal_wait_scacquire(sig_, HSA_SIGNAL_CONDITION_LT, 1, limit_ns,
                                                                 HSA_WAIT_STATE_BLOCKED);
          if (v != 0) fail(v < 0 ? "SDMA copy reported an error" : "SDMA copy timed out");
        }
      }
      const auto t1 = std::chrono::steady_clock::now();
      busy_ns_ += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
      if (trace_)
        fprintf(stderr, "sdma: done seq=%u ready-wait %.3f ms copy %.3f ms\n", j.seq,
                std::chrono::duration<double, std::milli>(t0 - tq).count(),
                std::chrono::duration<double, std::milli>(t1 - t0).count());
      copies_ += 1;
      bytes_ += j.bytes;
      __atomic_store_n(flag_, j.seq, __ATOMIC_RELEASE);  // the waiting stream proceeds
    }
  }

  int dev_;
  bool trace_ = false;
  hsa_agent_t cpu_{}, gpu_{};
  bool gpu_known_ = false;
  uint32_t engine_ = 0, avail_ = 0, pref_ = 0;
  hsa_signal_t sig_{};
  uint32_t* flag_ = nullptr;
  uint32_t next_seq_ = 0;
  std::mutex submit_mu_, mu_, err_mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  std::thread worker_;
  std::atomic<uint64_t> copies_{0}, bytes_{0}, busy_ns_{0};
  std::string err_;
  std::atomic<bool> failed_{false};  // set by fail(): later copies release their streams at once
};

constexpr int kMaxDev = 64;
Copier* g_copiers[kMaxDev] = {};
std::mutex g_mu;

Copier& copier(int dev) {
  if (dev < 0 || dev >= kMaxDev) throw std::runtime_error("sdma: device ordinal out of range");
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_copiers[dev]) g_copiers[dev] = new Copier(dev);  // process lifetime (see the worker)
  return *g_copiers[dev];
}

}  // namespace

void sdma_d2h(void* dst, const void* src, size_t bytes, int device, hipStream_t s, hipStream_t producer) {
  if (bytes == 0) return;
  copier(device).d2h(dst, src, bytes, s, producer);
}

SdmaStats sdma_stats(int device) { return copier(device).stats(); }

void sdma_clear_error(int device) { copier(device).clear_error(); }

}  // namespace grt
