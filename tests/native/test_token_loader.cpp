// Standalone stress test of the native loader's threading core (csrc/token_loader.h), built by
// tests/test_native_sanitizers.py with -fsanitize=thread (data races, lock-order inversions) and
// with -fsanitize=address,undefined (out-of-bounds slot/mmap reads, use-after-free on restart).
//
// Exercises: many workers racing for few slots, consumer reading every batch while producers
// refill the others, set_state() restarts mid-stream (workers joined and re-spawned), epoch
// boundaries (shared permutation regenerated under the lock), destruction with producers blocked.
// Every batch is checked against the corpus (tokens are arange, so a window identifies itself).

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../neuronx_distributed_llama3_2_amd/csrc/token_loader.h"

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

static void check_batch(const int64_t* b, int64_t B, int64_t S, int64_t vocab) {
  for (int64_t r = 0; r < B; ++r) {
    const int64_t* row = b + r * (S + 1);
    for (int64_t i = 1; i <= S; ++i) CHECK(row[i] == (row[i - 1] + 1) % vocab);
  }
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/nxd_tl_test.bin";
  const int64_t ntok = 200003, vocab = 60000, S = 32, B = 4;
  {
    std::vector<uint32_t> toks(ntok);
    for (int64_t i = 0; i < ntok; ++i) toks[i] = (uint32_t)(i % vocab);
    FILE* f = std::fopen(path, "wb");
    CHECK(f);
    CHECK(std::fwrite(toks.data(), 4, toks.size(), f) == toks.size());
    std::fclose(f);
  }
  for (int nslots : {2, 3, 8}) {
    for (int threads : {1, 4, 8}) {
      std::vector<std::vector<int64_t>> bufs(nslots, std::vector<int64_t>(B * (S + 1)));
      std::vector<int64_t*> ptrs;
      for (auto& v : bufs) ptrs.push_back(v.data());
      nxd_data::TokenLoaderCore ld(path, 4, S, B, 1, 2, 17, threads, ptrs);
      const int64_t spe = ld.steps_per_epoch();
      CHECK(spe == ((ntok - 1) / S) / (2 * B));
      std::vector<std::vector<int64_t>> first;
      for (int64_t s = 0; s < spe + 7; ++s) {  // crosses an epoch boundary
        const int slot = ld.next_slot();
        check_batch(bufs[slot].data(), B, S, vocab);
        if (s >= 10 && s < 14) first.push_back(bufs[slot]);
        auto ids = ld.sample_ids(s);
        for (int64_t r = 0; r < B; ++r) CHECK(bufs[slot][r * (S + 1)] == (ids[r] * S) % vocab);
      }
      ld.set_state(0, 10);  // restart producers mid-stream: must replay steps 10..13 exactly
      for (int k = 0; k < 4; ++k) {
        const int slot = ld.next_slot();
        CHECK(bufs[slot] == first[k]);
      }
      ld.next_slot();  // leave producers running/blocked on full ring: destructor must join cleanly
    }
  }
  std::remove(path);
  std::printf("token_loader stress OK\n");
  return 0;
}
