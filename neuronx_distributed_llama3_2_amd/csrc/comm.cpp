// Native collective layer over RCCL (the reference drives its collectives through the
// Neuron runtime's CC layer, src/neuronx_distributed/parallel_layers/parallel_state.py:412-415,
// mappings.py:97-147).  torch.distributed stays the default path; this layer adds what it does not
// expose, for the framework's own buckets:
//   * communicators created straight from RCCL (unique id exchanged over the torch process group),
//     with their environment (channels, protocol) applied by parallel/rccl_env.py before init;
//   * coalesced launches: a list of tensors -> ONE ncclGroupStart/End region (all-reduce,
//     reduce-scatter, all-gather, all-to-all, batched send/recv);
//   * bucketed all-reduce: many small tensors packed into a persistent staging buffer by one
//     kernel (csrc/comm_pack.hip), one all-reduce, one unpack;
//   * explicit streams: every call runs on the HIP stream it is given (the Python wrapper owns a
//     high-priority comm stream, event ordering and caching-allocator stream records).
#include <torch/extension.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <ATen/hip/HIPContext.h>

#include <dlfcn.h>

#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace nxd {
int multi_copy_launch(const void* const*, void* const*, const int64_t*, int, hipStream_t);
// peer_allreduce.hip: one-shot all-reduce over IPC-mapped peer buffers
void* peer_ar_create(int64_t, int*);
int peer_coll_run(void*, const void*, void*, int64_t, int, int, hipStream_t);
int peer_ar_ipc_handle(void*, void*);
int peer_ar_open(void*, int, int, const void*);
int peer_ar_run(void*, float*, int, int, int, float*, void*, const float*, int, hipStream_t);
int peer_ar_error(void*);
void peer_ar_set_error(void*, int);
void peer_ar_destroy(void*);
}

namespace {

// RCCL entry points resolved from the librccl.so torch already loaded (dlopen RTLD_NOLOAD of the
// same file): one RCCL instance per process, whichever RCCL build torch ships with.
struct Rccl {
  decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&::ncclCommInitRank) CommInitRank = nullptr;
  decltype(&::ncclCommDestroy) CommDestroy = nullptr;
  decltype(&::ncclAllReduce) AllReduce = nullptr;
  decltype(&::ncclReduceScatter) ReduceScatter = nullptr;
  decltype(&::ncclAllGather) AllGather = nullptr;
  decltype(&::ncclSend) Send = nullptr;
  decltype(&::ncclRecv) Recv = nullptr;
  decltype(&::ncclGroupStart) GroupStart = nullptr;
  decltype(&::ncclGroupEnd) GroupEnd = nullptr;
  decltype(&::ncclGetErrorString) GetErrorString = nullptr;
  decltype(&::ncclGetVersion) GetVersion = nullptr;
};
Rccl g_rccl;
bool g_loaded = false;

void load_rccl(const std::string& path) {
  if (g_loaded) return;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  TORCH_CHECK(h, "native comm: cannot load ", path, ": ", dlerror());
#define NXD_SYM(f) g_rccl.f = reinterpret_cast<decltype(g_rccl.f)>(dlsym(h, "nccl" #f)); \
  TORCH_CHECK(g_rccl.f, "native comm: symbol nccl" #f " missing in ", path)
  NXD_SYM(GetUniqueId);
  NXD_SYM(CommInitRank);
  NXD_SYM(CommDestroy);
  NXD_SYM(AllReduce);
  NXD_SYM(ReduceScatter);
  NXD_SYM(AllGather);
  NXD_SYM(Send);
  NXD_SYM(Recv);
  NXD_SYM(GroupStart);
  NXD_SYM(GroupEnd);
  NXD_SYM(GetErrorString);
  NXD_SYM(GetVersion);
#undef NXD_SYM
  g_loaded = true;
}

void need_rccl() { TORCH_CHECK(g_loaded, "native comm: call comm_load(<torch lib>/librccl.so) first"); }

#define NXD_NCCL_CHECK(cmd)                                                                      \
  do {                                                                                           \
    ncclResult_t r_ = (cmd);                                                                     \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error ", g_rccl.GetErrorString(r_), " at ", #cmd);      \
  } while (0)

struct Comm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
};

std::mutex g_mu;
std::vector<std::unique_ptr<Comm>> g_comms;

Comm& get(int64_t h) {
  need_rccl();
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h], "invalid native communicator handle ", h);
  return *g_comms[h];
}

ncclDataType_t dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "native comm: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

ncclRedOp_t op_of(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  if (op == "avg") return ncclAvg;
  TORCH_CHECK(false, "native comm: unknown reduce op ", op);
  return ncclSum;
}

void check_dev(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
}

hipStream_t as_stream(int64_t s) { return reinterpret_cast<hipStream_t>(static_cast<intptr_t>(s)); }

pybind11::bytes unique_id() {
  need_rccl();
  ncclUniqueId id;
  NXD_NCCL_CHECK(g_rccl.GetUniqueId(&id));
  return pybind11::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

int64_t init(pybind11::bytes id, int64_t nranks, int64_t rank, int64_t device) {
  need_rccl();
  std::string s = id;
  TORCH_CHECK(s.size() == NCCL_UNIQUE_ID_BYTES, "native comm: bad unique id");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "native comm: bad rank / size");
  TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "native comm: hipSetDevice failed");
  ncclUniqueId uid;
  std::memcpy(uid.internal, s.data(), NCCL_UNIQUE_ID_BYTES);
  auto c = std::make_unique<Comm>();
  NXD_NCCL_CHECK(g_rccl.CommInitRank(&c->comm, (int)nranks, uid, (int)rank));
  c->rank = (int)rank;
  c->nranks = (int)nranks;
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(std::move(c));
  return (int64_t)g_comms.size() - 1;
}

void destroy(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (h >= 0 && h < (int64_t)g_comms.size() && g_comms[h]) {
    g_rccl.CommDestroy(g_comms[h]->comm);
    g_comms[h].reset();
  }
}

// in-place all-reduce of every tensor, one group launch
void all_reduce(int64_t h, std::vector<at::Tensor> ts, const std::string& op, int64_t stream) {
  Comm& c = get(h);
  const ncclRedOp_t rop = op_of(op);
  for (auto& t : ts) check_dev(t, "tensor");   // validate everything before opening the group
  NXD_NCCL_CHECK(g_rccl.GroupStart());
  for (auto& t : ts) {
    NXD_NCCL_CHECK(g_rccl.AllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dtype_of(t), rop, c.comm, as_stream(stream)));
  }
  NXD_NCCL_CHECK(g_rccl.GroupEnd());
}

// out[i] (numel n) = reduce over ranks of in[i] chunk `rank` (in numel n * nranks)
void reduce_scatter(int64_t h, std::vector<at::Tensor> outs, std::vector<at::Tensor> ins, const std::string& op,
                    int64_t stream) {
  Comm& c = get(h);
  TORCH_CHECK(outs.size() == ins.size(), "reduce_scatter: list sizes differ");
  const ncclRedOp_t rop = op_of(op);
  for (size_t i = 0; i < outs.size(); ++i) {
    check_dev(outs[i], "out");
    check_dev(ins[i], "in");
    TORCH_CHECK(ins[i].numel() == outs[i].numel() * c.nranks && ins[i].scalar_type() == outs[i].scalar_type(),
                "reduce_scatter: in must be nranks x out");
  }
  NXD_NCCL_CHECK(g_rccl.GroupStart());
  for (size_t i = 0; i < outs.size(); ++i) {
    NXD_NCCL_CHECK(g_rccl.ReduceScatter(ins[i].data_ptr(), outs[i].data_ptr(), outs[i].numel(), dtype_of(outs[i]), rop,
                                     c.comm, as_stream(stream)));
  }
  NXD_NCCL_CHECK(g_rccl.GroupEnd());
}

void all_gather(int64_t h, std::vector<at::Tensor> outs, std::vector<at::Tensor> ins, int64_t stream) {
  Comm& c = get(h);
  TORCH_CHECK(outs.size() == ins.size(), "all_gather: list sizes differ");
  for (size_t i = 0; i < outs.size(); ++i) {
    check_dev(outs[i], "out");
    check_dev(ins[i], "in");
    TORCH_CHECK(outs[i].numel() == ins[i].numel() * c.nranks && ins[i].scalar_type() == outs[i].scalar_type(),
                "all_gather: out must be nranks x in");
  }
  NXD_NCCL_CHECK(g_rccl.GroupStart());
  for (size_t i = 0; i < outs.size(); ++i) {
    NXD_NCCL_CHECK(g_rccl.AllGather(ins[i].data_ptr(), outs[i].data_ptr(), ins[i].numel(), dtype_of(ins[i]), c.comm,
                                 as_stream(stream)));
  }
  NXD_NCCL_CHECK(g_rccl.GroupEnd());
}

// equal-split all-to-all: chunk j of `in` goes to rank j, chunk j of `out` comes from rank j
void all_to_all(int64_t h, at::Tensor out, at::Tensor in, int64_t stream) {
  Comm& c = get(h);
  check_dev(out, "out");
  check_dev(in, "in");
  TORCH_CHECK(in.numel() == out.numel() && in.numel() % c.nranks == 0 && in.scalar_type() == out.scalar_type(),
              "all_to_all: equal sizes divisible by nranks");
  const int64_t n = in.numel() / c.nranks;
  const int64_t eb = in.element_size();
  dtype_of(in);
  NXD_NCCL_CHECK(g_rccl.GroupStart());
  for (int j = 0; j < c.nranks; ++j) {
    NXD_NCCL_CHECK(g_rccl.Send(static_cast<const char*>(in.data_ptr()) + j * n * eb, n, dtype_of(in), j, c.comm,
                            as_stream(stream)));
    NXD_NCCL_CHECK(g_rccl.Recv(static_cast<char*>(out.data_ptr()) + j * n * eb, n, dtype_of(out), j, c.comm,
                            as_stream(stream)));
  }
  NXD_NCCL_CHECK(g_rccl.GroupEnd());
}

// batched point-to-point: sends[i] -> send_peers[i], recvs[i] <- recv_peers[i], one group
void batch_p2p(int64_t h, std::vector<at::Tensor> sends, std::vector<int64_t> send_peers, std::vector<at::Tensor> recvs,
               std::vector<int64_t> recv_peers, int64_t stream) {
  Comm& c = get(h);
  TORCH_CHECK(sends.size() == send_peers.size() && recvs.size() == recv_peers.size(), "batch_p2p: list sizes");
  for (size_t i = 0; i < sends.size(); ++i) {
    check_dev(sends[i], "send");
    TORCH_CHECK(send_peers[i] >= 0 && send_peers[i] < c.nranks, "batch_p2p: bad peer");
  }
  for (size_t i = 0; i < recvs.size(); ++i) {
    check_dev(recvs[i], "recv");
    TORCH_CHECK(recv_peers[i] >= 0 && recv_peers[i] < c.nranks, "batch_p2p: bad peer");
  }
  NXD_NCCL_CHECK(g_rccl.GroupStart());
  for (size_t i = 0; i < sends.size(); ++i) {
    NXD_NCCL_CHECK(g_rccl.Send(sends[i].data_ptr(), sends[i].numel(), dtype_of(sends[i]), (int)send_peers[i], c.comm,
                            as_stream(stream)));
  }
  for (size_t i = 0; i < recvs.size(); ++i) {
    NXD_NCCL_CHECK(g_rccl.Recv(recvs[i].data_ptr(), recvs[i].numel(), dtype_of(recvs[i]), (int)recv_peers[i], c.comm,
                            as_stream(stream)));
  }
  NXD_NCCL_CHECK(g_rccl.GroupEnd());
}

// Bucketed all-reduce: pack every tensor (same dtype) into `staging` (16-B aligned slots), one
// all-reduce over the used prefix, unpack.  Returns the bytes reduced.
int64_t bucketed_all_reduce(int64_t h, std::vector<at::Tensor> ts, at::Tensor staging, const std::string& op,
                            int64_t stream) {
  Comm& c = get(h);
  check_dev(staging, "staging");
  if (ts.empty()) return 0;
  const auto st = ts[0].scalar_type();
  const int64_t eb = ts[0].element_size();
  std::vector<const void*> src, cdst;
  std::vector<void*> dst, csrc_out;
  std::vector<int64_t> nb;
  int64_t off = 0;
  char* base = static_cast<char*>(staging.data_ptr());
  for (auto& t : ts) {
    check_dev(t, "tensor");
    TORCH_CHECK(t.scalar_type() == st, "bucketed_all_reduce: one dtype per bucket");
    const int64_t bytes = t.numel() * eb;
    src.push_back(t.data_ptr());
    dst.push_back(base + off);
    nb.push_back(bytes);
    off += (bytes + 15) / 16 * 16;
  }
  TORCH_CHECK(off <= staging.numel() * staging.element_size(), "bucketed_all_reduce: staging buffer too small (",
              off, " bytes needed)");
  const hipStream_t s = as_stream(stream);
  TORCH_CHECK(nxd::multi_copy_launch(src.data(), dst.data(), nb.data(), (int)ts.size(), s) == 0, "pack failed");
  NXD_NCCL_CHECK(g_rccl.AllReduce(base, base, off / eb, dtype_of(ts[0]), op_of(op), c.comm, s));
  std::vector<const void*> usrc;
  std::vector<void*> udst;
  for (size_t i = 0; i < ts.size(); ++i) {
    usrc.push_back(dst[i]);
    udst.push_back(ts[i].data_ptr());
  }
  TORCH_CHECK(nxd::multi_copy_launch(usrc.data(), udst.data(), nb.data(), (int)ts.size(), s) == 0, "unpack failed");
  return off;
}

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

std::string version() {
  int v = 0;
  need_rccl();
  g_rccl.GetVersion(&v);
  return std::to_string(v);
}

}  // namespace

void register_comm(pybind11::module& m) {
  m.def("comm_load", &load_rccl);
  m.def("comm_unique_id", &unique_id);
  m.def("comm_init", &init);
  m.def("comm_destroy", &destroy);
  m.def("comm_all_reduce", &all_reduce);
  m.def("comm_reduce_scatter", &reduce_scatter);
  m.def("comm_all_gather", &all_gather);
  m.def("comm_all_to_all", &all_to_all);
  m.def("comm_batch_p2p", &batch_p2p);
  m.def("comm_bucketed_all_reduce", &bucketed_all_reduce);
  m.def("comm_version", &version);
  m.def("peer_ar_create", &peer_ar_create);
  m.def("peer_ar_ipc_handle", &peer_ar_ipc_handle);
  m.def("peer_ar_open", &peer_ar_open);
  m.def("peer_ar_run", &peer_ar_run, pybind11::arg("h"), pybind11::arg("inp"), pybind11::arg("zero_in"),
        pybind11::arg("mode"), pybind11::arg("out") = pybind11::none(), pybind11::arg("res") = pybind11::none(),
        pybind11::arg("xadd") = pybind11::none());
  m.def("peer_ar_gather", &peer_ar_gather);
  m.def("peer_coll", &peer_coll);
  m.def("peer_ar_error", [](int64_t h) { return nxd::peer_ar_error(reinterpret_cast<void*>(h)); });
  m.def("peer_ar_set_error", [](int64_t h, int v) { nxd::peer_ar_set_error(reinterpret_cast<void*>(h), v); });
  m.def("peer_ar_destroy", [](int64_t h) { nxd::peer_ar_destroy(reinterpret_cast<void*>(h)); });
}
