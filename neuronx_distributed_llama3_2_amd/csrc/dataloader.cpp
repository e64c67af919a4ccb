// Native token data loader: memory-mapped pre-tokenized corpus -> shuffled, DP-sharded windows
// of seq_len+1 tokens assembled by worker threads into a ring of pinned host batches.
//
// The reference feeds the device through torch_xla's MpDeviceLoader (parallel_loader prefetch
// threads; src/neuronx_distributed/pipeline/model.py:1590-1591, tp_zero1_llama_hf_pretrain.py:425)
// on top of a Python HF-datasets DataLoader.  On MI355X the input pipeline is: this loader
// (C++ threads, no GIL, no per-sample Python objects) -> pinned batch -> H2D copy on a side HIP
// stream (utils/data_loader.py), overlapped with the previous step's compute.
//
// The threading core lives in token_loader.h (torch-free, sanitizer-tested standalone); this file
// only owns the pinned batch tensors and exposes the loader to Python.

#include <ATen/ATen.h>
#include <torch/extension.h>

#include <memory>

#include "token_loader.h"

namespace nxd_data {

class TokenLoader {
 public:
  TokenLoader(const std::string& path, int token_bytes, int64_t seq_len, int64_t batch, int64_t dp_rank,
              int64_t dp_size, uint64_t seed, int threads, int prefetch, bool pin) {
    TORCH_CHECK(seq_len > 0 && batch > 0, "bad loader geometry");
    auto opts = at::TensorOptions().dtype(at::kLong);
    const int nslots = std::max(2, prefetch);
    std::vector<int64_t*> ptrs;
    for (int i = 0; i < nslots; ++i) {
      at::Tensor t = at::empty({batch, seq_len + 1}, opts);
      if (pin) {
        try {
          t = t.pin_memory();
        } catch (...) {  // no device runtime (CPU-only host): plain pageable memory
        }
      }
      slots_.push_back(t);
      ptrs.push_back(t.data_ptr<int64_t>());
    }
    try {
      core_ = std::make_unique<TokenLoaderCore>(path, token_bytes, seq_len, batch, dp_rank, dp_size, seed, threads,
                                                std::move(ptrs));
    } catch (const std::exception& e) {
      TORCH_CHECK(false, e.what());
    }
  }

  ~TokenLoader() { core_.reset(); }  // joins the workers before the slot tensors go away

  // next batch [batch, seq_len + 1] (int64); valid until the following next() call
  at::Tensor next() { return slots_[core_->next_slot()]; }
  std::vector<int64_t> state() { return core_->state(); }
  void set_state(int64_t epoch, int64_t step) { core_->set_state(epoch, step); }
  int64_t num_samples() const { return core_->num_samples(); }
  int64_t steps_per_epoch() const { return core_->steps_per_epoch(); }

 private:
  std::vector<at::Tensor> slots_;
  std::unique_ptr<TokenLoaderCore> core_;
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
