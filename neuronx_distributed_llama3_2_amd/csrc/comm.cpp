// Python bindings of the direct-peer collectives (csrc/peer_allreduce.hip): the framework's native
// communication layer beside torch.distributed's RCCL (the reference drives its collectives
// through the Neuron runtime's CC layer, src/neuronx_distributed/parallel_layers/parallel_state.py:412-415,
// mappings.py:97-147).  Every rank exports one device region (its IPC handle exchanged once over the
// torch process group), maps every peer's, and one kernel per call moves or sums the data: the
// tensor-parallel decode all-reduces / vocabulary gather (default) and the sequence-parallel
// all-gather / reduce-scatter (NXD_SP_PEER).  The bulk collectives (DP buckets, SP at large sizes,
// PP send/recv) stay on torch's ProcessGroupNCCL = RCCL over xGMI.
// (Round 6 removed the native-RCCL communicator layer that used to live here: opt-in, never run with
// more than one rank, and a duplicate of what ProcessGroupNCCL already does.)
#include <torch/extension.h>
#include <hip/hip_runtime.h>
#include <ATen/hip/HIPContext.h>

#include <cstring>
#include <string>
#include <vector>

namespace nxd {
// peer_allreduce.hip: one-shot all-reduce over IPC-mapped peer buffers
void* peer_ar_create(int64_t, int*);
int peer_coll_run(void*, const void*, void*, int64_t, int, int, hipStream_t);
int peer_ar_ipc_handle(void*, void*);
int peer_ar_open(void*, int, int, const void*);
int peer_ar_run(void*, float*, int, int, int, float*, void*, const float*, int, hipStream_t);
int peer_ar_error(void*);
void peer_ar_set_error(void*, int);
void peer_ar_set_spin_limit(void*, int64_t);
void peer_ar_destroy(void*);
}

namespace {

// ---- one-shot peer all-reduce (csrc/peer_allreduce.hip) ---------------------------------------------
// Latency-class all-reduce of tensor-parallel decode partials: every rank exports one device region
// (IPC handle exchanged by the caller over the torch process group), maps every peer's, and one kernel
// per call publishes, waits for and sums all partials.  Modes: 0 out = sum, 1 residual fold
// res = bf16(bf16(res + bf16(xadd)) + bf16(sum)), 2 res = bf16(sum).
pybind11::tuple peer_ar_create(int64_t nmax) {
  int unc = 0;
  void* h = nxd::peer_ar_create(nmax, &unc);
  TORCH_CHECK(h, "peer all-reduce: device allocation failed");
  return pybind11::make_tuple(reinterpret_cast<int64_t>(h), unc != 0);
}

pybind11::bytes peer_ar_ipc_handle(int64_t h) {
  char buf[64] = {0};
  const int n = nxd::peer_ar_ipc_handle(reinterpret_cast<void*>(h), buf);
  TORCH_CHECK(n > 0, "peer all-reduce: hipIpcGetMemHandle failed");
  return pybind11::bytes(buf, 64);
}

void peer_ar_open(int64_t h, int64_t rank, std::vector<std::string> handles) {
  std::string all;
  for (auto& x : handles) {
    TORCH_CHECK(x.size() == 64, "peer all-reduce: 64-byte IPC handles expected");
    all += x;
  }
  const int rc = nxd::peer_ar_open(reinterpret_cast<void*>(h), (int)handles.size(), (int)rank, all.data());
  TORCH_CHECK(rc == 0, "peer all-reduce: opening the peers' IPC handles failed (", rc, ")");
}

void peer_ar_run(int64_t h, at::Tensor in, bool zero_in, int64_t mode, c10::optional<at::Tensor> out,
                 c10::optional<at::Tensor> res, c10::optional<at::Tensor> xadd) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kFloat && in.is_contiguous(), "peer all-reduce: fp32 input");
  const int64_t n = in.numel();
  float* op = nullptr;
  void* rp = nullptr;
  const float* xp = nullptr;
  if (out.has_value()) {
    TORCH_CHECK(out->scalar_type() == at::kFloat && out->is_contiguous() && out->numel() == n, "peer all-reduce: out");
    op = out->data_ptr<float>();
  }
  if (res.has_value()) {
    TORCH_CHECK(res->scalar_type() == at::kBFloat16 && res->is_contiguous() && res->numel() == n, "peer all-reduce: res");
    rp = res->data_ptr();
  }
  if (xadd.has_value()) {
    TORCH_CHECK(xadd->scalar_type() == at::kFloat && xadd->is_contiguous() && xadd->numel() >= n, "peer all-reduce: xadd");
    xp = xadd->data_ptr<float>();
  }
  const int rc = nxd::peer_ar_run(reinterpret_cast<void*>(h), in.data_ptr<float>(), zero_in ? 1 : 0, (int)mode, (int)n, op,
                                  rp, xp, 0, at::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(rc == 0, "peer all-reduce: launch failed (", rc, ")");
}

// sequence-parallel all-gather (mode 0: out = [world * n]) / reduce-scatter (mode 1: in = [world * n])
void peer_coll(int64_t h, at::Tensor in, at::Tensor out, int64_t mode) {
  TORCH_CHECK(in.is_cuda() && in.is_contiguous() && out.is_contiguous() && in.scalar_type() == out.scalar_type(),
              "peer collective: contiguous GPU tensors of one dtype");
  TORCH_CHECK(in.scalar_type() == at::kBFloat16 || in.scalar_type() == at::kFloat || mode == 0,
              "peer reduce-scatter: bf16 or fp32");
  const int es = (int)in.element_size();
  TORCH_CHECK(es == 2 || es == 4, "peer collective: 2- or 4-byte elements");
  const int64_t n = mode == 0 ? in.numel() : out.numel();
  const int rc = nxd::peer_coll_run(reinterpret_cast<void*>(h), in.data_ptr(), out.data_ptr(), n, es, (int)mode,
                                    at::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(rc == 0, "peer collective: launch failed (", rc, ")");
}

// all-gather of [rows, C] slices (any dtype; row bytes a multiple of 16) into [rows, world * C]
void peer_ar_gather(int64_t h, at::Tensor in, at::Tensor out, int64_t world) {
  TORCH_CHECK(in.is_cuda() && in.is_contiguous() && out.is_contiguous() && in.dim() == 2 && out.dim() == 2 &&
                  in.scalar_type() == out.scalar_type(),
              "peer gather: contiguous 2-D tensors of one dtype");
  const int64_t row_bytes = in.size(1) * in.element_size();
  TORCH_CHECK(row_bytes % 16 == 0 && out.size(0) == in.size(0) && out.size(1) == world * in.size(1),
              "peer gather: row bytes % 16, out [rows, world * C]");
  const int64_t nbytes = in.numel() * in.element_size();
  const int rc = nxd::peer_ar_run(reinterpret_cast<void*>(h), reinterpret_cast<float*>(in.data_ptr()), 0, 3,
                                  (int)(nbytes / 4), reinterpret_cast<float*>(out.data_ptr()), nullptr, nullptr,
                                  (int)(row_bytes / 16), at::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(rc == 0, "peer gather: launch failed (", rc, ")");
}

}  // namespace

void register_comm(pybind11::module& m) {
  m.def("peer_ar_create", &peer_ar_create);
  m.def("peer_ar_ipc_handle", &peer_ar_ipc_handle);
  m.def("peer_ar_open", &peer_ar_open);
  m.def("peer_ar_run", &peer_ar_run, pybind11::arg("h"), pybind11::arg("inp"), pybind11::arg("zero_in"),
        pybind11::arg("mode"), pybind11::arg("out") = pybind11::none(), pybind11::arg("res") = pybind11::none(),
        pybind11::arg("xadd") = pybind11::none());
  m.def("peer_ar_gather", &peer_ar_gather);
  m.def("peer_coll", &peer_coll);
  m.def("peer_ar_error", [](int64_t h) { return nxd::peer_ar_error(reinterpret_cast<void*>(h)); });
  m.def("peer_ar_set_spin_limit", [](int64_t h, int64_t v) { nxd::peer_ar_set_spin_limit(reinterpret_cast<void*>(h), v); });
  m.def("peer_ar_set_error", [](int64_t h, int v) { nxd::peer_ar_set_error(reinterpret_cast<void*>(h), v); });
  m.def("peer_ar_destroy", [](int64_t h) { nxd::peer_ar_destroy(reinterpret_cast<void*>(h)); });
}
