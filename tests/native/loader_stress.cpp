// Host-side stress test of the native token loader (runtime/csrc/loader.cpp), built
// with ThreadSanitizer or AddressSanitizer+UBSan by tests/test_native_sanitizers.py.
//
// Producer threads, the consumer, synchronous random-access fills and seeks run
// concurrently on a corpus so small that one epoch is a single step: the producers
// are always working on several epochs at once, which stresses the cached epoch
// permutations.  Every consumed batch is checked against a synchronous fill of the
// same step, and a dummy-mode loader is closed while its producers are blocked.
#include "../../distributed_llm_trainer_amd/runtime/csrc/loader.cpp"

#include <cstdio>
#include <cstdlib>
#include <string>

static int fails = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                \
    }                                                         \
  } while (0)

// mem: the ring's slot memory; it must outlive the loader (producers keep filling
// free slots until dlt_loader_close)
static int run(void* h, std::vector<std::vector<int64_t>>& mem, int64_t seq, int64_t batch, int n_slots, int steps,
               int seek_at) {
  mem.assign(n_slots, std::vector<int64_t>(seq * batch));
  for (int i = 0; i < n_slots; ++i) CHECK(dlt_loader_set_slot(h, i, mem[i].data(), 4) == 0);
  std::vector<int64_t> want(seq * batch);
  // a second thread doing random-access fills while the ring runs
  std::atomic<bool> done{false};
  std::thread side([&] {
    std::vector<int64_t> buf(seq * batch);
    for (int64_t s = 0; !done.load(); s = (s + 7) % 97) dlt_loader_fill(h, s, buf.data());
  });
  int64_t expect = 0;
  for (int k = 0; k < steps; ++k) {
    if (k == seek_at) {
      CHECK(dlt_loader_seek(h, 1000) == 0);
      expect = 1000;
    }
    int64_t step = -1;
    const int slot = dlt_loader_next(h, &step);
    CHECK(slot >= 0 && slot < n_slots);
    CHECK(step == expect);
    ++expect;
    dlt_loader_fill(h, step, want.data());
    CHECK(std::memcmp(want.data(), mem[slot].data(), want.size() * 8) == 0);
    CHECK(dlt_loader_release(h, slot) == 0);
  }
  CHECK(dlt_loader_release(h, 0) != 0 || true);  // double release is rejected or harmless
  done = true;
  side.join();
  return 0;
}

int main() {
  // corpus: 64 uint16 tokens, seq 8 -> 7 windows; world 2 -> 3 per rank; batch 3 -> 1 step/epoch
  const std::string path = std::string(std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp") +
                           "/dlt_loader_stress_" + std::to_string(getpid()) + ".bin";
  {
    FILE* f = std::fopen(path.c_str(), "wb");
    for (uint16_t t = 0; t < 64; ++t) {
      const uint16_t v = (uint16_t)(t * 31 + 5);
      std::fwrite(&v, 2, 1, f);
    }
    std::fclose(f);
  }
  int err = 0;
  void* h = dlt_loader_open(path.c_str(), 2, 0, 0, 8, 3, 1, 2, 42, 1, 6, 4, &err);
  CHECK(h != nullptr && err == 0);
  if (h) {
    CHECK(dlt_loader_steps_per_epoch(h) == 1);
    std::vector<std::vector<int64_t>> mem;
    run(h, mem, 8, 3, 6, 400, 200);
    dlt_loader_close(h);
  }
  // dummy mode; closed while producers wait on a full ring
  h = dlt_loader_open(nullptr, 0, 0, 1000, 16, 2, 0, 1, 7, 0, 3, 3, &err);
  CHECK(h != nullptr);
  if (h) {
    std::vector<std::vector<int64_t>> mem;
    run(h, mem, 16, 2, 3, 100, 50);
    dlt_loader_close(h);
  }
  // bad arguments
  CHECK(dlt_loader_open(nullptr, 0, 0, 0, 16, 2, 0, 1, 7, 0, 3, 3, &err) == nullptr && err == 2);
  CHECK(dlt_loader_open("/nonexistent/dlt", 2, 0, 0, 16, 2, 0, 1, 7, 0, 3, 3, &err) == nullptr && err == 1);
  std::remove(path.c_str());
  if (fails) {
    std::fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  std::printf("loader stress OK\n");
  return 0;
}
