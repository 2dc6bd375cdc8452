// Native batch assembler for token-window datasets (CPU side of the input pipeline).
//
// Reference role: TextDataset.__getitem__ + DataLoader collate of the BasicLLM job
// (reference ray-jobs/pytorch_llm_ray.py:107-119,206-216): every step Python indexes B windows
// of S+1 tokens one by one and stacks them. Here one call gathers a whole batch of windows
// (inputs and next-token targets) straight into a caller-provided (pinned) buffer with a small
// thread pool, so the host side of the loader is one memcpy-bound native call per batch and the
// H2D copy can be issued asynchronously from pinned memory.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

extern "C" {

// tokens: [n] int64 ; starts: [B] int64 window starts ; out_x/out_y: [B, S] int64
// Returns 0 on success, -1 if any window runs past the end.
int grt_gather_windows_i64(const int64_t* tokens, int64_t n, const int64_t* starts, int64_t B, int64_t S,
                           int64_t* out_x, int64_t* out_y, int nthreads) {
  for (int64_t b = 0; b < B; ++b)
    if (starts[b] < 0 || starts[b] + S + 1 > n) return -1;
  auto work = [&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b) {
      const int64_t* src = tokens + starts[b];
      memcpy(out_x + b * S, src, sizeof(int64_t) * S);
      if (out_y) memcpy(out_y + b * S, src + 1, sizeof(int64_t) * S);
    }
  };
  nthreads = std::max(1, std::min<int>(nthreads, (int)B));
  if (nthreads == 1 || B * S < (1 << 16)) {
    work(0, B);
    return 0;
  }
  std::vector<std::thread> th;
  const int64_t per = (B + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int64_t b0 = t * per, b1 = std::min(B, b0 + per);
    if (b0 < b1) th.emplace_back(work, b0, b1);
  }
  for (auto& x : th) x.join();
  return 0;
}

// Same for int32 token storage widened to int64 outputs (halves resident dataset memory).
int grt_gather_windows_i32(const int32_t* tokens, int64_t n, const int64_t* starts, int64_t B, int64_t S,
                           int64_t* out_x, int64_t* out_y, int nthreads) {
  for (int64_t b = 0; b < B; ++b)
    if (starts[b] < 0 || starts[b] + S + 1 > n) return -1;
  auto work = [&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b) {
      const int32_t* src = tokens + starts[b];
      int64_t* x = out_x + b * S;
      for (int64_t i = 0; i < S; ++i) x[i] = src[i];
      if (out_y) {
        int64_t* y = out_y + b * S;
        for (int64_t i = 0; i < S; ++i) y[i] = src[i + 1];
      }
    }
  };
  nthreads = std::max(1, std::min<int>(nthreads, (int)B));
  std::vector<std::thread> th;
  const int64_t per = (B + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int64_t b0 = t * per, b1 = std::min(B, b0 + per);
    if (b0 < b1) th.emplace_back(work, b0, b1);
  }
  for (auto& x : th) x.join();
  return 0;
}

// Right-padded packing of variable-length samples into [B, S] (SFT collator):
// concatenated tokens + offsets[B+1]; writes ids (pad_id), labels (-100 where padded or where
// mask_prompt[b] tokens are the prompt), attention mask (0/1). Truncates to S.
int grt_pad_collate(const int64_t* flat, const int64_t* offsets, const int64_t* prompt_len, int64_t B, int64_t S,
                    int64_t pad_id, int64_t* ids, int64_t* labels, int64_t* mask) {
  for (int64_t b = 0; b < B; ++b) {
    const int64_t len = std::min<int64_t>(offsets[b + 1] - offsets[b], S);
    if (len < 0) return -1;
    const int64_t* src = flat + offsets[b];
    const int64_t pl = prompt_len ? prompt_len[b] : 0;
    for (int64_t i = 0; i < S; ++i) {
      const bool v = i < len;
      ids[b * S + i] = v ? src[i] : pad_id;
      labels[b * S + i] = (v && i >= pl) ? src[i] : -100;
      mask[b * S + i] = v ? 1 : 0;
    }
  }
  return 0;
}

}  // extern "C"
