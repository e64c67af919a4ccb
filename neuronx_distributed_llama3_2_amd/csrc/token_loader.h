// Torch-free core of the native token data loader (csrc/dataloader.cpp wraps it for Python).
//
// Kept free of ATen so the threading protocol (worker threads filling a ring of host batch slots,
// consumer handing slots back, set_state restarting the producers) can be compiled standalone with
// -fsanitize=thread / -fsanitize=address by tests/native/test_token_loader.cpp.  The reference has
// no race detection at all; its input pipeline is torch_xla's MpDeviceLoader
// (src/neuronx_distributed/pipeline/model.py:1590-1591).
//
// Corpus: flat little-endian uint16/uint32 token ids.  Sample i = tokens [i*S, i*S + S + 1).
// Every epoch the sample order is a seeded permutation; DP rank r of d takes positions r, r+d, ...
// (equal counts; the tail that does not fill a global batch is dropped).

#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace nxd_data {

class TokenLoaderCore {
 public:
  // slots: caller-owned buffers of batch * (seq_len + 1) int64 each (>= 2 of them); they must
  // outlive the loader.  The Python wrapper passes pinned tensors' data pointers.
  TokenLoaderCore(const std::string& path, int token_bytes, int64_t seq_len, int64_t batch, int64_t dp_rank,
                  int64_t dp_size, uint64_t seed, int threads, std::vector<int64_t*> slots)
      : seq_len_(seq_len), batch_(batch), dp_rank_(dp_rank), dp_size_(dp_size), seed_(seed), tb_(token_bytes),
        slots_(std::move(slots)) {
    if (token_bytes != 2 && token_bytes != 4) throw std::invalid_argument("token_bytes must be 2 or 4");
    if (seq_len <= 0 || batch <= 0 || dp_size <= 0 || dp_rank < 0 || dp_rank >= dp_size)
      throw std::invalid_argument("bad loader geometry");
    if (slots_.size() < 2) throw std::invalid_argument("need at least 2 batch slots");
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open token file " + path);
    struct stat st;
    if (fstat(fd_, &st) != 0) {
      release_file();
      throw std::runtime_error("stat failed on " + path);
    }
    bytes_ = (size_t)st.st_size;
    ntok_ = (int64_t)(bytes_ / tb_);
    if (ntok_ <= seq_len_) {
      release_file();
      throw std::runtime_error("token file shorter than one sample");
    }
    base_ = ::mmap(nullptr, bytes_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (base_ == MAP_FAILED) {
      base_ = nullptr;
      release_file();
      throw std::runtime_error("mmap failed on " + path);
    }
    ::madvise(base_, bytes_, MADV_RANDOM);
    nsamples_ = (ntok_ - 1) / seq_len_;
    const int64_t per_rank = nsamples_ / (dp_size_ * batch_) * batch_;  // whole local batches only
    if (per_rank <= 0) {
      release_file();
      throw std::runtime_error("corpus too small for one global batch");
    }
    steps_per_epoch_ = per_rank / batch_;
    nthreads_ = std::max(1, threads);
    start_workers();
  }

  TokenLoaderCore(const TokenLoaderCore&) = delete;
  TokenLoaderCore& operator=(const TokenLoaderCore&) = delete;

  ~TokenLoaderCore() {
    stop_workers();
    release_file();
  }

  int64_t num_samples() const { return nsamples_; }
  int64_t steps_per_epoch() const { return steps_per_epoch_; }

  // Index of the slot holding the next batch; the slot stays valid until the following call.
  int next_slot() {
    std::unique_lock<std::mutex> lk(mu_);
    if (held_ >= 0) {  // release the slot the consumer held
      free_.push_back(held_);
      held_ = -1;
      cv_work_.notify_all();
    }
    cv_ready_.wait(lk, [&] { return !ready_.empty() && ready_.front().first == consume_step_; });
    const int slot = ready_.front().second;
    ready_.pop_front();
    held_ = slot;
    ++consume_step_;
    return slot;
  }

  // (epoch, step within epoch) of the NEXT batch next_slot() returns
  std::vector<int64_t> state() {
    std::lock_guard<std::mutex> g(mu_);
    return {consume_step_ / steps_per_epoch_, consume_step_ % steps_per_epoch_};
  }

  void set_state(int64_t epoch, int64_t step) {
    stop_workers();
    {
      std::lock_guard<std::mutex> g(mu_);
      consume_step_ = epoch * steps_per_epoch_ + step;
    }
    start_workers();
  }

  // corpus window indices of the local batch at global step g (tests / resume checks)
  std::vector<int64_t> sample_ids(int64_t g) {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<int64_t> ids;
    batch_samples(g, ids);
    return ids;
  }

 private:
  void release_file() {
    if (base_) ::munmap(base_, bytes_);
    base_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }

  // global step g -> local sample ids of that batch (caller holds mu_: perm_ is shared)
  void batch_samples(int64_t g, std::vector<int64_t>& out) {
    const int64_t epoch = g / steps_per_epoch_, s = g % steps_per_epoch_;
    if (epoch != perm_epoch_) {
      perm_.resize(nsamples_);
      std::iota(perm_.begin(), perm_.end(), 0);
      std::mt19937_64 rng(seed_ * 0x9E3779B97F4A7C15ull + (uint64_t)epoch);
      std::shuffle(perm_.begin(), perm_.end(), rng);
      perm_epoch_ = epoch;
    }
    out.resize(batch_);
    for (int64_t b = 0; b < batch_; ++b) out[b] = perm_[(s * batch_ + b) * dp_size_ + dp_rank_];
  }

  void fill(int slot, const std::vector<int64_t>& ids) {
    int64_t* dst = slots_[slot];
    const int64_t L = seq_len_ + 1;
    for (size_t b = 0; b < ids.size(); ++b) {
      const int64_t off = ids[b] * seq_len_;
      if (tb_ == 2) {
        const uint16_t* src = reinterpret_cast<const uint16_t*>(base_) + off;
        for (int64_t i = 0; i < L; ++i) dst[b * L + i] = src[i];
      } else {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(base_) + off;
        for (int64_t i = 0; i < L; ++i) dst[b * L + i] = src[i];
      }
    }
  }

  void worker() {
    std::vector<int64_t> ids;
    while (true) {
      int slot;
      int64_t g;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_work_.wait(lk, [&] { return stop_ || !free_.empty(); });
        if (stop_) return;
        slot = free_.back();
        free_.pop_back();
        g = produce_step_++;
        batch_samples(g, ids);
      }
      fill(slot, ids);  // the copy runs outside the lock, in parallel across workers
      {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = ready_.begin();
        while (it != ready_.end() && it->first < g) ++it;
        ready_.insert(it, {g, slot});
      }
      cv_ready_.notify_all();
    }
  }

  void start_workers() {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = false;
    free_.clear();
    ready_.clear();
    held_ = -1;
    for (int i = 0; i < (int)slots_.size(); ++i) free_.push_back(i);
    produce_step_ = consume_step_;
    for (int i = 0; i < nthreads_; ++i) threads_.emplace_back(&TokenLoaderCore::worker, this);
  }

  void stop_workers() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_work_.notify_all();
    for (auto& t : threads_) t.join();
    threads_.clear();
  }

  int64_t seq_len_, batch_, dp_rank_, dp_size_;
  uint64_t seed_;
  int tb_;
  std::vector<int64_t*> slots_;
  int fd_ = -1;
  void* base_ = nullptr;
  size_t bytes_ = 0;
  int64_t ntok_ = 0, nsamples_ = 0, steps_per_epoch_ = 0;
  std::vector<int64_t> perm_;
  int64_t perm_epoch_ = -1;
  int nthreads_ = 1;
  std::mutex mu_;
  std::condition_variable cv_work_, cv_ready_;
  std::vector<int> free_;
  std::deque<std::pair<int64_t, int>> ready_;
  int held_ = -1;
  int64_t produce_step_ = 0, consume_step_ = 0;
  bool stop_ = false;
  std::vector<std::thread> threads_;
};

}  // namespace nxd_data
