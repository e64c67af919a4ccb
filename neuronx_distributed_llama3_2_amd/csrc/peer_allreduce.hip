// One-shot all-reduce over peer-mapped (IPC) device buffers for latency-bound messages: the
// tensor-parallel decode's row-parallel partial sums (o_proj, down: M x H fp32, a few KiB per layer).
//
// Reference: the fork's TP decode has its all-reduces compiled into one SPMD graph
// (examples/inference/modules/gqa.py:641-647, src/neuronx_distributed/trace/spmd.py:82-187).  A ring
// all-reduce through RCCL costs (2 (W - 1)) link latencies per call; at these sizes the data is
// nothing and the latency is everything, so here every rank publishes its partial once and every rank
// reads all W partials directly: ONE kernel launch per all-reduce, no host involvement, capturable in
// the decode hipGraph.
//
// Per rank, one IPC-exported region: a 4 KiB header of flags [2][kMaxBlocks] (uint64 epochs) + slots
// [2][nmax x 4 B].
// Call c of a rank has epoch e = ctr[0] + 1 (one device counter per rank, advanced by the last block of
// the call to finish -- an arrival ticket in ctr[1] -- so hipGraph replays keep counting) and parity
// e & 1; every block of a call uses the same epoch.  (Per-block counters broke the slot-reuse argument
// below once calls of different sizes, hence different block-to-chunk maps, alternate: a block's
// parity then no longer alternated with the call, and a rank could overwrite a slot region a peer
// was still reading for the previous call -- a reduce-scatter mismatch in the 4-rank GPU test.)
// Block b of every rank:
//   1. copies its chunk of the local partial into slot[parity] (and zeroes the partial when it is an
//      atomic accumulator that must start at zero for the next producer);
//   2. publishes: every wave drains its stores (vmcnt(0)), workgroup barrier, one system-scope release
//      (the region may be read from another GPU over xGMI), then the flag[parity][b] = e store;
//   3. waits for flag[parity][b] >= e of every peer (relaxed system-scope polls with s_sleep and a
//      bounded spin; the flag word also carries the call's signature, so peers whose call sequences
//      drifted apart are told from peers that are merely late), then one system-scope acquire and a
//      barrier.  A peer that never arrives, or whose
//      flag is PAST e (it skipped a call: the two ranks' call sequences diverged), marks the call
//      lost: *err (pinned host memory, read by the host without a sync) is set, every output of the
//      call is written as NaN (a missed check cannot pass stale slots off as a sum) and the rank's
//      flags are poisoned so its peers fail their next call as well;
//   4. sums the W chunks in rank order (bitwise identical on every rank: the residual stream stays
//      replicated) and applies the epilogue.
// A slot is rewritten two calls later; by then every peer has passed the intervening call, which it
// only enters after finishing its reads of this one (kernel order on its stream), so two slots
// suffice.
#include "common.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace nxd {
namespace par {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 128;
constexpr int kThreads = 256;

enum Mode { SUM = 0, FOLD_RES = 1, SET_RES = 2, GATHER = 3 };

struct Args {
  float* in;                                 // local partial [n] fp32
  int zero_in;                               // zero `in` after publishing it
  float* slot[2];                            // this rank's slots (IPC region)
  const float* peer_slot[kMaxRanks][2];      // every rank's slots (own included), as mapped here
  uint64_t* flag;                            // this rank's flags [2][kMaxBlocks] (IPC region)
  const uint64_t* peer_flag[kMaxRanks];      // every rank's flags, as mapped here
  uint64_t* ctr;                             // [0] epoch of the last call, [1] arrival ticket (local memory)
  int* err;                                  // != 0: a peer never arrived / diverged (host-mapped)
  int world, rank, n, chunk, mode;
  uint32_t sig;                              // call_sig(mode, n, 4)
  int64_t spin_limit;
  float* out;                                // SUM: [n] fp32
  uint16_t* res;                             // FOLD_RES / SET_RES: bf16 residual stream [n]
  const float* xadd;                         // FOLD_RES: pending fp32 sum folded first (o_proj)
  // GATHER: every rank's slice [rows][rowu x 16 B] (any dtype, moved as bytes) into
  // out [rows][world][rowu x 16 B] -- the vocab-parallel logits of TP decode
  int rowu;
};

// The last block of a call to finish (arrival ticket) publishes the call's epoch for the next call.
// Every block read ctr[0] at its start, before taking its ticket, so none reads the new value.
__device__ __forceinline__ void advance_epoch(uint64_t* ctr, uint64_t e) {
  const uint64_t t = __hip_atomic_fetch_add(ctr + 1, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == gridDim.x - 1) {
    __hip_atomic_store(ctr + 1, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ctr, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// A flag word is (epoch << 8) | signature of the call (its kind and size): ranks whose call sequences
// drifted apart by whole calls publish the expected epoch for a DIFFERENT call, which the signature
// exposes (epochs alone re-align after one skipped call).
__host__ __device__ __forceinline__ uint32_t call_sig(int mode, int64_t n, int es) {
  uint64_t h = (uint64_t)n * 0x9E3779B97F4A7C15ull ^ ((uint64_t)(mode + 1) << 40) ^ ((uint64_t)es << 48);
  h ^= h >> 29;
  return (uint32_t)(h & 0xFF);
}
__device__ __forceinline__ uint64_t flag_word(uint64_t e, uint32_t sig) { return (e << 8) | sig; }

// Poll a peer's flag for epoch e.  Legal values are those of e - 2 (the peer has not reached this call
// yet) and e with this call's signature; a later epoch, or epoch e for another kind / size of call,
// means the peers' call sequences diverged.  Returns false for a lost peer: bounded spin expired or
// diverged.
__device__ __forceinline__ bool wait_peer(const uint64_t* pf, uint64_t e, uint32_t sig, int64_t spin_limit) {
  int64_t it = 0;
  uint64_t v;
  while (((v = __hip_atomic_load(pf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >> 8) < e) {
    __builtin_amdgcn_s_sleep(2);
    if (++it > spin_limit) return false;
  }
  return v == flag_word(e, sig);
}

// A rank that lost a peer poisons ALL its flags (both parities, every block): a peer still running
// (or one that comes back late) then reads a value past its epoch on its next wait and fails that call
// too, instead of summing this rank's stale slot as if the sequences still matched.
__device__ __forceinline__ void poison_flags(uint64_t* flag, int tid) {
  static_assert(kThreads >= 2 * kMaxBlocks, "one flag per thread");
  if (tid < 2 * kMaxBlocks) __hip_atomic_store(flag + tid, ~(uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(kThreads) peer_allreduce_kernel(Args a) {
  __shared__ uint64_t e_s;
  __shared__ int lost_s;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int lo = b * a.chunk, hi = min(a.n, lo + a.chunk);
  if (tid == 0) e_s = __hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint64_t e = e_s;
  const int par = (int)(e & 1);
  float* mine = a.slot[par];
  for (int i = lo + tid * 4; i < hi; i += kThreads * 4) {
    if (i + 4 <= hi) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(a.in + i);
      *reinterpret_cast<f32x4_t*>(mine + i) = v;
      if (a.zero_in) *reinterpret_cast<f32x4_t*>(a.in + i) = f32x4_t{0.f, 0.f, 0.f, 0.f};
    } else {
      for (int j = i; j < hi; ++j) {
        mine[j] = a.in[j];
        if (a.zero_in) a.in[j] = 0.f;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: peers may sit on other GPUs
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.flag + par * kMaxBlocks + b, flag_word(e, a.sig), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // (rank loops unrolled with static indices: a runtime index into the kernel-argument arrays would
  // copy them to scratch)
  const uint64_t* pf = nullptr;
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r)
    if (r == tid) pf = a.peer_flag[r] + par * kMaxBlocks + b;
  if (tid == 0) lost_s = 0;
  __syncthreads();
  if (tid < a.world && tid != a.rank && !wait_peer(pf, e, a.sig, a.spin_limit)) {
    lost_s = 1;
    __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const bool lost = lost_s != 0;
  if (lost) poison_flags(a.flag, tid);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (a.mode == GATHER) {
    // 16-byte units u of this block's chunk: row m = u / rowu, unit j = u % rowu of rank r's slice
    const int u0 = lo / 4, u1 = hi / 4;
    for (int u = u0 + tid; u < u1; u += kThreads) {
      const int m = u / a.rowu, j = u - m * a.rowu;
#pragma unroll
      for (int r = 0; r < kMaxRanks; ++r) {
        if (r < a.world) {
          u32x4_t v = reinterpret_cast<const u32x4_t*>(par ? a.peer_slot[r][1] : a.peer_slot[r][0])[u];
          if (lost) v = u32x4_t{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};   // NaN in bf16 and fp32
          reinterpret_cast<u32x4_t*>(a.out)[((int64_t)m * a.world + r) * a.rowu + j] = v;
        }
      }
    }
    if (tid == 0) advance_epoch(a.ctr, e);
    return;
  }
  for (int i = lo + tid; i < hi; i += kThreads) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
      if (r < a.world) s += (par ? a.peer_slot[r][1] : a.peer_slot[r][0])[i];
    if (lost) s = __builtin_nanf("");
    if (a.mode == SUM) {
      a.out[i] = s;
    } else if (a.mode == FOLD_RES) {
      // the unfused TP = 1 rounding: y = bf16(bf16(y + bf16(o_proj)) + bf16(down))
      const float y = bf2f(f2bf(bf2f(a.res[i]) + bf2f(f2bf(a.xadd[i]))));
      a.res[i] = lost ? (uint16_t)0xFFFF : f2bf(y + bf2f(f2bf(s)));
    } else {
      a.res[i] = f2bf(s);
    }
  }
  if (tid == 0) advance_epoch(a.ctr, e);
}

struct Handle {
  char* base = nullptr;        // IPC region: flags, slot 0, slot 1
  size_t bytes = 0;
  int64_t nmax = 0;
  bool uncached = false;
  int world = 0, rank = 0;
  char* peer_base[kMaxRanks] = {};
  bool opened[kMaxRanks] = {};
  uint64_t* ctr = nullptr;
  int* err = nullptr;          // device-side pointer the kernels store to
  int* err_host = nullptr;     // the same word, host-mapped pinned memory (nullptr: device memory)
  int64_t spin_limit = -1;     // polls before a peer counts as lost (< 0: NXD_PEER_AR_SPIN_LIMIT)
};

int64_t env_spin_limit() {
  static const int64_t limit = [] {
    const char* e = getenv("NXD_PEER_AR_SPIN_LIMIT");
    return e ? atoll(e) : (int64_t)1 << 24;   // ~ seconds of s_sleep polling, then give up
  }();
  return limit;
}
int64_t spin_limit_of(const Handle* h) { return h->spin_limit >= 0 ? h->spin_limit : env_spin_limit(); }

constexpr size_t kFlagBytes = 2 * kMaxBlocks * sizeof(uint64_t);
constexpr size_t kHeader = 4096;

size_t slot_offset(int64_t nmax, int s) {
  const size_t slot_bytes = ((size_t)nmax * 4 + 255) / 256 * 256;
  return kHeader + (size_t)s * slot_bytes;
}

// ---- bandwidth-class collectives on the same region: all-gather and reduce-scatter of the
// sequence-parallel activations (a ring uses one xGMI link per hop; here every rank
// reads each peer's slot directly, all 7 links of a node at once).  Same epoch / parity / publish /
// wait protocol as peer_allreduce_kernel; elements per rank n and per block `chunk` are multiples
// of 8.  AG: out[r n + i] = in_r[i] (bytes).  RS: out[i] = sum_r in_r[rank n + i] (fp32 accumulate
// in rank order, bf16 or fp32 io).
struct CollArgs {
  const char* in;
  char* slot[2];
  const char* peer_slot[kMaxRanks][2];
  uint64_t* flag;
  const uint64_t* peer_flag[kMaxRanks];
  uint64_t* ctr;
  int* err;
  int world, rank, es, mode;   // es: element bytes (2 | 4); mode 0 AG, 1 RS
  uint32_t sig;                // call_sig(4 + mode, n, es)
  int64_t n, chunk, spin_limit;
  char* out;
};

__device__ __forceinline__ void copy16(const char* src, char* dst, int64_t b0, int64_t b1, int tid) {
  for (int64_t o = b0 + (int64_t)tid * 16; o < b1; o += (int64_t)kThreads * 16)
    *reinterpret_cast<u32x4_t*>(dst + o) = *reinterpret_cast<const u32x4_t*>(src + o);
}

__global__ void __launch_bounds__(kThreads) peer_coll_kernel(CollArgs a) {
  __shared__ uint64_t e_s;
  __shared__ int lost_s;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int64_t lo = (int64_t)b * a.chunk, hi = min(a.n, lo + a.chunk);
  if (tid == 0) e_s = __hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint64_t e = e_s;
  const int par = (int)(e & 1);
  char* mine = a.slot[par];
  if (a.mode == 0) {
    copy16(a.in, mine, lo * a.es, hi * a.es, tid);
  } else {
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
      if (r < a.world) copy16(a.in, mine, ((int64_t)r * a.n + lo) * a.es, ((int64_t)r * a.n + hi) * a.es, tid);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.flag + par * kMaxBlocks + b, flag_word(e, a.sig), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const uint64_t* pf = nullptr;
#pragma unroll
  for (int r = 0; r < kMaxRanks; ++r)
    if (r == tid) pf = a.peer_flag[r] + par * kMaxBlocks + b;
  if (tid == 0) lost_s = 0;
  __syncthreads();
  if (tid < a.world && tid != a.rank && !wait_peer(pf, e, a.sig, a.spin_limit)) {
    lost_s = 1;
    __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const bool lost = lost_s != 0;
  if (lost) poison_flags(a.flag, tid);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (a.mode == 0) {
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r) {
      if (r < a.world) {
        const char* src = par ? a.peer_slot[r][1] : a.peer_slot[r][0];
        for (int64_t o = lo * a.es + (int64_t)tid * 16; o < hi * a.es; o += (int64_t)kThreads * 16)
          *reinterpret_cast<u32x4_t*>(a.out + (int64_t)r * a.n * a.es + o) =
              lost ? u32x4_t{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu} : *reinterpret_cast<const u32x4_t*>(src + o);
      }
    }
  } else {
    const int64_t base = (int64_t)a.rank * a.n;
    const int per = 16 / a.es;   // elements per 16-byte vector
    for (int64_t i = lo + (int64_t)tid * per; i < hi; i += (int64_t)kThreads * per) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < kMaxRanks; ++r) {
        if (r < a.world) {
          const char* src = par ? a.peer_slot[r][1] : a.peer_slot[r][0];
          const u32x4_t v = *reinterpret_cast<const u32x4_t*>(src + (base + i) * a.es);
          if (a.es == 2) {
            float f[8];
            unpack8(v, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += f[j];
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] += __uint_as_float(v[j]);
          }
        }
      }
      if (lost) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = __builtin_nanf("");
      }
      if (a.es == 2) {
        *reinterpret_cast<u32x4_t*>(a.out + i * 2) = pack8(acc);
      } else {
        *reinterpret_cast<f32x4_t*>(a.out + i * 4) = f32x4_t{acc[0], acc[1], acc[2], acc[3]};
      }
    }
  }
  if (tid == 0) advance_epoch(a.ctr, e);
}

}  // namespace par

// ---- host API (comm.cpp binds it) ----------------------------------------------------------------

void* peer_ar_create(int64_t nmax, int* uncached) {
  auto* h = new par::Handle();
  h->nmax = nmax;
  h->bytes = par::slot_offset(nmax, 2);
  static_assert(par::kFlagBytes <= par::kHeader, "flag block");
  // fine-grained, uncached device memory: coherent for peers on other GPUs without relying on cache
  // maintenance; plain device memory if the runtime cannot export such an allocation
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, h->bytes, hipDeviceMallocUncached) == hipSuccess) {
    hipIpcMemHandle_t ih;
    if (hipIpcGetMemHandle(&ih, p) == hipSuccess) {
      h->uncached = true;
    } else {
      (void)hipGetLastError();
      (void)hipFree(p);
      p = nullptr;
    }
  } else {
    (void)hipGetLastError();
    p = nullptr;
  }
  if (!p && hipMalloc(&p, h->bytes) != hipSuccess) {
    delete h;
    return nullptr;
  }
  h->base = static_cast<char*>(p);
  if (hipMemset(h->base, 0, h->bytes) != hipSuccess || hipMalloc(&h->ctr, par::kMaxBlocks * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(h->ctr, 0, par::kMaxBlocks * sizeof(uint64_t)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    delete h;
    return nullptr;
  }
  // the lost-peer word in pinned, host-mapped memory: the host reads it after any step without a
  // device sync or a copy (device memory + hipMemcpy if the runtime refuses the mapping)
  void* hp = nullptr;
  if (hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, hp, 0) == hipSuccess) {
      h->err_host = static_cast<int*>(hp);
      h->err = static_cast<int*>(dp);
      *reinterpret_cast<volatile int*>(h->err_host) = 0;
    } else {
      (void)hipGetLastError();
      (void)hipHostFree(hp);
    }
  } else {
    (void)hipGetLastError();
  }
  if (!h->err && (hipMalloc(&h->err, sizeof(int)) != hipSuccess || hipMemset(h->err, 0, sizeof(int)) != hipSuccess ||
                  hipDeviceSynchronize() != hipSuccess)) {
    delete h;
    return nullptr;
  }
  *uncached = h->uncached ? 1 : 0;
  return h;
}

int peer_ar_ipc_handle(void* hv, void* out64) {
  auto* h = static_cast<par::Handle*>(hv);
  hipIpcMemHandle_t ih;
  if (hipIpcGetMemHandle(&ih, h->base) != hipSuccess) return -1;
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "ipc handle size");
  memcpy(out64, &ih, sizeof(ih));
  return (int)sizeof(ih);
}

// handles: world x 64 bytes (every rank's region, own included)
int peer_ar_open(void* hv, int world, int rank, const void* handles) {
  auto* h = static_cast<par::Handle*>(hv);
  if (world < 1 || world > par::kMaxRanks || rank < 0 || rank >= world) return -1;
  h->world = world;
  h->rank = rank;
  for (int r = 0; r < world; ++r) {
    if (r == rank) {
      h->peer_base[r] = h->base;
      continue;
    }
    hipIpcMemHandle_t ih;
    memcpy(&ih, static_cast<const char*>(handles) + 64 * r, sizeof(ih));
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, ih, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -2 - r;
    h->peer_base[r] = static_cast<char*>(p);
    h->opened[r] = true;
  }
  return 0;
}

int peer_ar_run(void* hv, float* in, int zero_in, int mode, int n, float* out, void* res, const float* xadd,
                int rowu, hipStream_t stream) {
  auto* h = static_cast<par::Handle*>(hv);
  if (n < 1 || n > h->nmax || h->world < 1) return -1;
  if (((mode == par::SUM || mode == par::GATHER) && !out) || ((mode == par::FOLD_RES || mode == par::SET_RES) && !res) ||
      (mode == par::FOLD_RES && !xadd) || (mode == par::GATHER && (rowu < 1 || (n / 4) % rowu)))
    return -2;
  if ((reinterpret_cast<uintptr_t>(in) & 15) || n % 4) return -3;
  par::Args a{};
  a.in = in;
  a.zero_in = zero_in;
  for (int s = 0; s < 2; ++s) a.slot[s] = reinterpret_cast<float*>(h->base + par::slot_offset(h->nmax, s));
  for (int r = 0; r < h->world; ++r) {
    for (int s = 0; s < 2; ++s) a.peer_slot[r][s] = reinterpret_cast<const float*>(h->peer_base[r] + par::slot_offset(h->nmax, s));
    a.peer_flag[r] = reinterpret_cast<const uint64_t*>(h->peer_base[r]);
  }
  a.flag = reinterpret_cast<uint64_t*>(h->base);
  a.ctr = h->ctr;
  a.err = h->err;
  a.world = h->world;
  a.rank = h->rank;
  a.n = n;
  a.mode = mode;
  a.sig = par::call_sig(mode, n, 4);
  // ~1 KiB of fp32 per block keeps every CU's share latency-sized; at most kMaxBlocks blocks
  int blocks = (n + 1023) / 1024;
  blocks = blocks < 1 ? 1 : (blocks > par::kMaxBlocks ? par::kMaxBlocks : blocks);
  a.chunk = ((n + blocks - 1) / blocks + 3) / 4 * 4;
  blocks = (n + a.chunk - 1) / a.chunk;
  a.spin_limit = par::spin_limit_of(h);
  a.out = out;
  a.res = static_cast<uint16_t*>(res);
  a.xadd = xadd;
  a.rowu = rowu;
  hipLaunchKernelGGL(par::peer_allreduce_kernel, dim3(blocks), dim3(par::kThreads), 0, stream, a);
  return (int)hipGetLastError();
}

// AG (mode 0): in [n] -> out [world * n]; RS (mode 1): in [world * n] -> out [n]; es = 2 (bf16) or 4 (fp32)
int peer_coll_run(void* hv, const void* in, void* out, int64_t n, int es, int mode, hipStream_t stream) {
  auto* h = static_cast<par::Handle*>(hv);
  if (h->world < 1 || n < 1 || n % 8 || (es != 2 && es != 4) || (mode != 0 && mode != 1)) return -1;
  const int64_t need = (mode == 0 ? n : (int64_t)h->world * n) * es;
  if (need > (int64_t)h->nmax * 4) return -2;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) return -3;
  par::CollArgs a{};
  a.in = static_cast<const char*>(in);
  for (int s = 0; s < 2; ++s) a.slot[s] = h->base + par::slot_offset(h->nmax, s);
  for (int r = 0; r < h->world; ++r) {
    for (int s = 0; s < 2; ++s) a.peer_slot[r][s] = h->peer_base[r] + par::slot_offset(h->nmax, s);
    a.peer_flag[r] = reinterpret_cast<const uint64_t*>(h->peer_base[r]);
  }
  a.flag = reinterpret_cast<uint64_t*>(h->base);
  a.ctr = h->ctr;
  a.err = h->err;
  a.world = h->world;
  a.rank = h->rank;
  a.es = es;
  a.mode = mode;
  a.n = n;
  a.sig = par::call_sig(4 + mode, n, es);
  // 64 KiB of this rank's elements per block (latency-bound below that), at most kMaxBlocks blocks
  int64_t blocks = (n * es + 65535) / 65536;
  blocks = blocks < 1 ? 1 : (blocks > par::kMaxBlocks ? par::kMaxBlocks : blocks);
  a.chunk = ((n + blocks - 1) / blocks + 7) / 8 * 8;
  blocks = (n + a.chunk - 1) / a.chunk;
  a.spin_limit = par::spin_limit_of(h);
  a.out = static_cast<char*>(out);
  hipLaunchKernelGGL(par::peer_coll_kernel, dim3((unsigned)blocks), dim3(par::kThreads), 0, stream, a);
  return (int)hipGetLastError();
}

// Non-zero once any call of this handle lost a peer.  Pinned word: reflects every call that has
// completed on the device (no sync here; callers check after their step's own synchronisation).
int peer_ar_error(void* hv) {
  auto* h = static_cast<par::Handle*>(hv);
  if (h->err_host) return *reinterpret_cast<volatile int*>(h->err_host);
  int v = 0;
  if (hipMemcpy(&v, h->err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v;
}

// Per-handle bound of the peer wait (< 0: back to NXD_PEER_AR_SPIN_LIMIT).  The init self-test runs
// with a generous one: the ranks' first launches (code-object load) can be milliseconds apart.
void peer_ar_set_spin_limit(void* hv, int64_t v) { static_cast<par::Handle*>(hv)->spin_limit = v; }

// Host-side test hook: a lost peer injected without a GPU fault (tests only).
void peer_ar_set_error(void* hv, int v) {
  auto* h = static_cast<par::Handle*>(hv);
  if (h->err_host) *reinterpret_cast<volatile int*>(h->err_host) = v;
  else (void)hipMemcpy(h->err, &v, sizeof(int), hipMemcpyHostToDevice);
}

void peer_ar_destroy(void* hv) {
  auto* h = static_cast<par::Handle*>(hv);
  if (!h) return;
  (void)hipDeviceSynchronize();
  for (int r = 0; r < par::kMaxRanks; ++r)
    if (h->opened[r]) (void)hipIpcCloseMemHandle(h->peer_base[r]);
  if (h->base) (void)hipFree(h->base);
  if (h->ctr) (void)hipFree(h->ctr);
  if (h->err_host) (void)hipHostFree(h->err_host);
  else if (h->err) (void)hipFree(h->err);
  delete h;
}

}  // namespace nxd
