// Native token data loader: memory-mapped pre-tokenized corpus -> shuffled, DP-sharded windows
// of seq_len+1 tokens assembled by worker threads into a ring of pinned host batches.
//
// The reference feeds the device through torch_xla's MpDeviceLoader (parallel_loader prefetch
// threads; src/neuronx_distributed/pipeline/model.py:1590-1591, tp_zero1_llama_hf_pretrain.py:425)
// on top of a Python HF-datasets DataLoader.  On MI355X the input pipeline is: this loader
// (C++ threads, no GIL, no per-sample Python objects) -> pinned batch -> H2D copy on a side HIP
// stream (utils/data_loader.py), overlapped with the previous step's compute.
//
// Corpus format: a flat little-endian file of uint16 or uint32 token ids (e.g. numpy .tofile of
// the concatenated tokenized dataset).  Sample i is tokens [i*seq_len, i*seq_len + seq_len + 1)
// (non-overlapping windows, the +1 token gives the shifted label).  Every epoch the sample order
// is a seeded permutation; DP rank r of d takes positions r, r+d, ... of it (equal counts; the
// tail that does not fill a global batch is dropped).  State (epoch, step) is exposed for exact
// resume from a checkpoint.

#include <ATen/ATen.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <torch/extension.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace nxd_data {

class TokenLoader {
 public:
  TokenLoader(const std::string& path, int token_bytes, int64_t seq_len, int64_t batch, int64_t dp_rank,
              int64_t dp_size, uint64_t seed, int threads, int prefetch, bool pin)
      : seq_len_(seq_len), batch_(batch), dp_rank_(dp_rank), dp_size_(dp_size), seed_(seed), tb_(token_bytes) {
    TORCH_CHECK(token_bytes == 2 || token_bytes == 4, "token_bytes must be 2 (uint16) or 4 (uint32)");
    TORCH_CHECK(seq_len > 0 && batch > 0 && dp_size > 0 && dp_rank >= 0 && dp_rank < dp_size, "bad loader geometry");
    fd_ = ::open(path.c_str(), O_RDONLY);
    TORCH_CHECK(fd_ >= 0, "cannot open token file ", path);
    struct stat st;
    TORCH_CHECK(fstat(fd_, &st) == 0, "stat failed on ", path);
    bytes_ = (size_t)st.st_size;
    ntok_ = (int64_t)(bytes_ / tb_);
    TORCH_CHECK(ntok_ > seq_len_, "token file shorter than one sample");
    base_ = ::mmap(nullptr, bytes_, PROT_READ, MAP_PRIVATE, fd_, 0);
    TORCH_CHECK(base_ != MAP_FAILED, "mmap failed on ", path);
    ::madvise(base_, bytes_, MADV_RANDOM);
    nsamples_ = (ntok_ - 1) / seq_len_;
    per_rank_ = nsamples_ / (dp_size_ * batch_) * batch_;  // whole local batches only
    TORCH_CHECK(per_rank_ > 0, "corpus too small for one global batch");
    steps_per_epoch_ = per_rank_ / batch_;
    auto opts = at::TensorOptions().dtype(at::kLong);
    nslots_ = std::max(2, prefetch);
    for (int i = 0; i < nslots_; ++i) {
      at::Tensor t = at::empty({batch_, seq_len_ + 1}, opts);
      if (pin) {
        try {
          t = t.pin_memory();
        } catch (...) {  // no device runtime (CPU-only host): plain pageable memory
        }
      }
      slots_.push_back(t);
    }
    nthreads_ = std::max(1, threads);
    start_workers();
  }

  ~TokenLoader() {
    stop_workers();
    if (base_ && base_ != MAP_FAILED) ::munmap(base_, bytes_);
    if (fd_ >= 0) ::close(fd_);
  }

  int64_t num_samples() const { return nsamples_; }
  int64_t steps_per_epoch() const { return steps_per_epoch_; }

  // next batch [batch, seq_len + 1] (int64); valid until the following next() call
  at::Tensor next() {
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
    return slots_[slot];
  }

  // (epoch, step within epoch) of the NEXT batch next() returns
  std::vector<int64_t> state() {
    std::lock_guard<std::mutex> g(mu_);
    return {consume_step_ / steps_per_epoch_, consume_step_ % steps_per_epoch_};
  }

  void set_state(int64_t epoch, int64_t step) {
    stop_workers();
    consume_step_ = epoch * steps_per_epoch_ + step;
    start_workers();
  }

 private:
  // global step g -> local sample ids of that batch
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
    int64_t* dst = slots_[slot].data_ptr<int64_t>();
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
        batch_samples(g, ids);  // permutation shared under the lock (cheap index math)
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
    for (int i = 0; i < nslots_; ++i) free_.push_back(i);
    produce_step_ = consume_step_;
    for (int i = 0; i < nthreads_; ++i) threads_.emplace_back(&TokenLoader::worker, this);
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
  int fd_ = -1;
  void* base_ = nullptr;
  size_t bytes_ = 0;
  int64_t ntok_ = 0, nsamples_ = 0, per_rank_ = 0, steps_per_epoch_ = 0;
  std::vector<int64_t> perm_;
  int64_t perm_epoch_ = -1;
  std::vector<at::Tensor> slots_;
  int nslots_ = 2, nthreads_ = 1;
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

void register_dataloader(pybind11::module& m) {
  pybind11::class_<nxd_data::TokenLoader>(m, "TokenLoader")
      .def(pybind11::init<const std::string&, int, int64_t, int64_t, int64_t, int64_t, uint64_t, int, int, bool>(),
           pybind11::arg("path"), pybind11::arg("token_bytes"), pybind11::arg("seq_len"), pybind11::arg("batch"),
           pybind11::arg("dp_rank") = 0, pybind11::arg("dp_size") = 1, pybind11::arg("seed") = 0,
           pybind11::arg("threads") = 4, pybind11::arg("prefetch") = 4, pybind11::arg("pin") = true)
      .def("next", &nxd_data::TokenLoader::next, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("state", &nxd_data::TokenLoader::state)
      .def("set_state", &nxd_data::TokenLoader::set_state, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("num_samples", &nxd_data::TokenLoader::num_samples)
      .def("steps_per_epoch", &nxd_data::TokenLoader::steps_per_epoch);
}
