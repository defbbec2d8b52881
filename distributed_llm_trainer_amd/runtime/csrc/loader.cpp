// Native token-batch loader (host side of the input pipeline).
//
// Replaces the reference's DataLoader worker processes (ddp_trainer.py:460-487,
// tinystories.py:122-161: 2-4 forked Python workers per rank re-collating int64
// tensors) with one in-process C++ producer pool:
//
//   * the corpus is a flat little-endian token file (uint16 / uint32 / int64) mapped
//     read-only with mmap -- a multi-GB corpus costs page cache, not process RSS, and
//     every rank on the node shares the same pages;
//   * samples are the non-overlapping windows tokens[i*S:(i+1)*S] of the reference's
//     map-style datasets (tinystories.py:44-50); epoch order is a seeded Fisher-Yates
//     permutation (splitmix64) sharded rank-strided like DistributedSampler with
//     drop_last, so every rank sees a disjoint slice and runs are reproducible;
//   * "dummy" mode generates uniform token ids from a counter hash of
//     (seed, rank, step, position) -- the reference's synthetic dataset without the
//     262 MB per-rank randint tensor;
//   * N producer threads fill a ring of caller-owned (pinned) batch slots as int64
//     [batch, seq_len]; the consumer takes slots in step order and hands them back after
//     its H2D copy has completed.
//
// C ABI (ctypes), no torch / HIP dependency: the slots are host memory registered by
// the Python side (torch pinned tensors), so the H2D copy is a plain async memcpy.
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#define DLT_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

inline uint64_t mix3(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t s = a * 0xD6E8FEB86659FD93ull ^ (b + 0x9E3779B97F4A7C15ull) * 0xA0761D6478BD642Full ^ c;
  return splitmix64(s);
}

enum SlotState : int { FREE = 0, FILLING = 1, READY = 2, TAKEN = 3 };

struct Loader {
  // source
  const uint8_t* map = nullptr;
  size_t map_bytes = 0;
  int fd = -1;
  int elem = 0;         // bytes per token in the file (0 = dummy)
  int64_t n_tokens = 0;
  int64_t vocab = 0;    // dummy mode
  // geometry
  int64_t seq = 0, batch = 0;
  int rank = 0, world = 1;
  uint64_t seed = 0;
  bool shuffle = true;
  int64_t windows = 0;       // total windows in the file
  int64_t per_rank = 0;      // windows per rank per epoch (drop_last)
  int64_t steps_per_epoch = 0;
  // ring
  std::vector<int64_t*> slots;
  std::vector<int64_t> slot_step;
  std::vector<int> state;
  std::mutex mu;
  std::condition_variable cv_work, cv_ready;
  int64_t next_fill = 0;     // next step to assign to a producer
  int64_t next_take = 0;     // next step the consumer wants
  bool stop = false;
  std::vector<std::thread> workers;
  // epoch permutations, cached for two epochs.  Handed out as shared_ptr: a producer
  // filling epoch e keeps its permutation alive while another producer replaces the
  // cache entry with epoch e+2 (tiny corpora have ring-many epochs in flight; a plain
  // vector reference here was a data race, found by tests/native/loader_stress.cpp
  // under ThreadSanitizer).
  std::mutex perm_mu;
  int64_t perm_epoch[2] = {-1, -1};
  std::shared_ptr<const std::vector<int64_t>> perm[2];
  std::atomic<int64_t> produced{0};

  std::shared_ptr<const std::vector<int64_t>> epoch_perm(int64_t epoch) {
    const int k = (int)(epoch & 1);
    {
      std::lock_guard<std::mutex> g(perm_mu);
      if (perm_epoch[k] == epoch) return perm[k];
    }
    auto p = std::make_shared<std::vector<int64_t>>(windows);  // built outside the lock
    for (int64_t i = 0; i < windows; ++i) (*p)[i] = i;
    if (shuffle) {
      uint64_t s = seed ^ (0x5851F42D4C957F2Dull * (uint64_t)(epoch + 1));
      for (int64_t i = windows - 1; i > 0; --i) {
        const int64_t j = (int64_t)(splitmix64(s) % (uint64_t)(i + 1));
        std::swap((*p)[i], (*p)[j]);
      }
    }
    std::lock_guard<std::mutex> g(perm_mu);
    perm[k] = p;
    perm_epoch[k] = epoch;
    return p;
  }

  int64_t load_token(int64_t idx) const {
    const uint8_t* p = map + (size_t)idx * elem;
    switch (elem) {
      case 2: { uint16_t v; std::memcpy(&v, p, 2); return v; }
      case 4: { uint32_t v; std::memcpy(&v, p, 4); return v; }
      default: { int64_t v; std::memcpy(&v, p, 8); return v; }
    }
  }

  void fill(int64_t step, int64_t* out) {
    if (elem == 0) {  // dummy: counter-hash uniform ids in [0, vocab)
      for (int64_t b = 0; b < batch; ++b) {
        const uint64_t row = (uint64_t)step * (uint64_t)batch + (uint64_t)b;
        for (int64_t t = 0; t < seq; ++t)
          out[b * seq + t] = (int64_t)(mix3(seed, ((uint64_t)rank << 40) ^ row, (uint64_t)t) % (uint64_t)vocab);
      }
      return;
    }
    const int64_t epoch = step / steps_per_epoch;
    const int64_t within = step % steps_per_epoch;
    const auto perm_ref = epoch_perm(epoch);
    const std::vector<int64_t>& p = *perm_ref;
    for (int64_t b = 0; b < batch; ++b) {
      // DistributedSampler layout: rank r takes positions r, r+W, r+2W, ...
      const int64_t pos = (within * batch + b) * world + rank;
      const int64_t w = p[pos];
      const int64_t base = w * seq;
      if (elem == 8) {
        std::memcpy(out + b * seq, map + (size_t)base * 8, (size_t)seq * 8);
      } else if (elem == 2) {
        const uint16_t* src = reinterpret_cast<const uint16_t*>(map) + base;
        for (int64_t t = 0; t < seq; ++t) out[b * seq + t] = src[t];
      } else {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(map) + base;
        for (int64_t t = 0; t < seq; ++t) out[b * seq + t] = src[t];
      }
    }
  }

  void worker() {
    for (;;) {
      int slot = -1;
      int64_t step = 0;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_work.wait(lk, [&] {
          if (stop) return true;
          for (size_t i = 0; i < state.size(); ++i)
            if (state[i] == FREE) return true;
          return false;
        });
        if (stop) return;
        for (size_t i = 0; i < state.size(); ++i)
          if (state[i] == FREE) { slot = (int)i; break; }
        step = next_fill++;
        state[slot] = FILLING;
        slot_step[slot] = step;
      }
      fill(step, slots[slot]);
      produced.fetch_add(1, std::memory_order_relaxed);
      {
        std::lock_guard<std::mutex> lk(mu);
        state[slot] = READY;
      }
      cv_ready.notify_all();
    }
  }
};

}  // namespace

// Open a loader.  path == nullptr selects dummy mode (vocab ids uniform in [0, vocab)).
// token_bytes: 2 (uint16), 4 (uint32) or 8 (int64).  max_tokens <= 0: whole file.
// Returns nullptr on error (*err set: 1 open/mmap failed, 2 bad args, 3 too few tokens).
DLT_API void* dlt_loader_open(const char* path, int token_bytes, int64_t max_tokens, int64_t vocab, int64_t seq_len,
                              int64_t batch, int rank, int world, uint64_t seed, int shuffle, int n_slots,
                              int n_threads, int* err) {
  *err = 0;
  if (seq_len <= 0 || batch <= 0 || world <= 0 || rank < 0 || rank >= world || n_slots <= 0 || n_threads <= 0) {
    *err = 2;
    return nullptr;
  }
  auto* L = new Loader();
  L->seq = seq_len;
  L->batch = batch;
  L->rank = rank;
  L->world = world;
  L->seed = seed;
  L->shuffle = shuffle != 0;
  if (path == nullptr) {
    if (vocab <= 0) { delete L; *err = 2; return nullptr; }
    L->vocab = vocab;
    L->elem = 0;
    L->steps_per_epoch = INT64_MAX;
  } else {
    if (token_bytes != 2 && token_bytes != 4 && token_bytes != 8) { delete L; *err = 2; return nullptr; }
    L->fd = ::open(path, O_RDONLY);
    struct stat st;
    if (L->fd < 0 || fstat(L->fd, &st) != 0 || st.st_size <= 0) {
      if (L->fd >= 0) ::close(L->fd);
      delete L;
      *err = 1;
      return nullptr;
    }
    L->map_bytes = (size_t)st.st_size;
    void* m = mmap(nullptr, L->map_bytes, PROT_READ, MAP_SHARED, L->fd, 0);
    if (m == MAP_FAILED) { ::close(L->fd); delete L; *err = 1; return nullptr; }
    madvise(m, L->map_bytes, MADV_RANDOM);
    L->map = static_cast<const uint8_t*>(m);
    L->elem = token_bytes;
    L->n_tokens = (int64_t)(L->map_bytes / token_bytes);
    if (max_tokens > 0 && max_tokens < L->n_tokens) L->n_tokens = max_tokens;
    L->windows = (L->n_tokens - 1) / seq_len;  // tinystories.py:44-45
    L->per_rank = L->windows / world;           // DistributedSampler(drop_last=True)
    L->steps_per_epoch = L->per_rank / batch;   // DataLoader(drop_last=True)
    if (L->steps_per_epoch <= 0) {
      munmap(const_cast<uint8_t*>(L->map), L->map_bytes);
      ::close(L->fd);
      delete L;
      *err = 3;
      return nullptr;
    }
  }
  L->slots.assign(n_slots, nullptr);
  L->slot_step.assign(n_slots, -1);
  L->state.assign(n_slots, TAKEN);  // not producible until the caller registers memory
  (void)n_threads;
  return L;
}

// Register host memory (int64 [batch, seq_len]) for slot i.  Starts the producers once
// every slot has memory.
DLT_API int dlt_loader_set_slot(void* h, int i, int64_t* ptr, int n_threads) {
  auto* L = static_cast<Loader*>(h);
  if (i < 0 || i >= (int)L->slots.size() || ptr == nullptr) return -1;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->slots[i] = ptr;
    L->state[i] = FREE;
  }
  bool all = true;
  for (auto* p : L->slots) all = all && p != nullptr;
  if (all && L->workers.empty()) {
    for (int t = 0; t < n_threads; ++t) L->workers.emplace_back([L] { L->worker(); });
  }
  L->cv_work.notify_all();
  return 0;
}

// Start (or restart) the stream at a given step: used to resume mid-run.
DLT_API int dlt_loader_seek(void* h, int64_t step) {
  auto* L = static_cast<Loader*>(h);
  std::unique_lock<std::mutex> lk(L->mu);
  // wait until no slot is being filled, then drop all prefetched batches
  L->cv_ready.wait(lk, [&] {
    for (int s : L->state)
      if (s == FILLING) return false;
    return true;
  });
  for (size_t i = 0; i < L->state.size(); ++i)
    if (L->slots[i] != nullptr && L->state[i] == READY) L->state[i] = FREE;
  L->next_fill = step;
  L->next_take = step;
  lk.unlock();
  L->cv_work.notify_all();
  return 0;
}

// Block until the batch for the next step is ready; returns its slot (caller owns it
// until dlt_loader_release).  *step_out receives the step index.
DLT_API int dlt_loader_next(void* h, int64_t* step_out) {
  auto* L = static_cast<Loader*>(h);
  std::unique_lock<std::mutex> lk(L->mu);
  int slot = -1;
  L->cv_ready.wait(lk, [&] {
    for (size_t i = 0; i < L->state.size(); ++i)
      if (L->state[i] == READY && L->slot_step[i] == L->next_take) { slot = (int)i; return true; }
    return false;
  });
  L->state[slot] = TAKEN;
  *step_out = L->next_take++;
  return slot;
}

DLT_API int dlt_loader_release(void* h, int slot) {
  auto* L = static_cast<Loader*>(h);
  {
    std::lock_guard<std::mutex> lk(L->mu);
    if (slot < 0 || slot >= (int)L->state.size() || L->state[slot] != TAKEN) return -1;
    L->state[slot] = FREE;
  }
  L->cv_work.notify_one();
  return 0;
}

// Synchronous fill of one step into caller memory (no ring; used by tests / random access).
DLT_API int dlt_loader_fill(void* h, int64_t step, int64_t* out) {
  auto* L = static_cast<Loader*>(h);
  if (step < 0) return -1;
  L->fill(step, out);
  return 0;
}

DLT_API int64_t dlt_loader_steps_per_epoch(void* h) { return static_cast<Loader*>(h)->steps_per_epoch; }
DLT_API int64_t dlt_loader_num_windows(void* h) { return static_cast<Loader*>(h)->windows; }
DLT_API int64_t dlt_loader_produced(void* h) { return static_cast<Loader*>(h)->produced.load(); }

DLT_API void dlt_loader_close(void* h) {
  auto* L = static_cast<Loader*>(h);
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop = true;
  }
  L->cv_work.notify_all();
  L->cv_ready.notify_all();
  for (auto& t : L->workers) t.join();
  if (L->map) munmap(const_cast<uint8_t*>(L->map), L->map_bytes);
  if (L->fd >= 0) ::close(L->fd);
  delete L;
}
