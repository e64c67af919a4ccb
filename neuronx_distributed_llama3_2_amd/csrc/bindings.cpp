// Python bindings of the CDNA4 kernels (module `neuronx_distributed_llama3_2_amd._C`).
// Every entry point validates shapes/dtypes on the host BEFORE launching (a wrong shape must
// never reach a hand-written kernel), then launches on the caller's current HIP stream, so the
// ops compose with torch streams and hipGraph capture.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include "common.h"

#include <execinfo.h>
#include <csignal>
#include <cstdlib>
#include <unistd.h>

namespace nxd {
int flash_attn_fwd_launch(const void*, const void*, const void*, void*, float*, const int64_t*, const int64_t*,
                          const int64_t*, const int64_t*, int, int, int, int, int, int, float, int, int,
                          const DropoutArgs&, hipStream_t);
int64_t flash_attn_bwd_workspace(int, int, int, int, int, int, int, int);
void flash_attn_bwd_set_knob(int, int);
int transpose_bf16_launch(const void*, void*, int64_t, int64_t, int64_t, int64_t, hipStream_t);
void transpose_set_variant(int);
int flash_attn_bwd_launch(const void*, const void*, const void*, const void*, const void*, const float*, float*,
                          void*, void*, void*, const int64_t*, const int64_t*, const int64_t*, const int64_t*,
                          const int64_t*, const int64_t*, const int64_t*, const int64_t*, int, int, int, int, int, int,
                          float, int, int, const DropoutArgs&, hipStream_t);
int rmsnorm_fwd_launch(const void*, const void*, const void*, void*, void*, float*, int64_t, int, float, hipStream_t);
int rmsnorm_bwd_num_partials(int64_t);
void rmsnorm_set_rows_path(int);
int rmsnorm_bwd_launch(const void*, const void*, const void*, const float*, const void*, void*, float*, float*, int,
                       int64_t, int, hipStream_t);
int rope_inplace_launch(void*, int64_t, int64_t, int, int, int, const float*, const float*, const int64_t*, int64_t,
                        int64_t, float, hipStream_t);
int swiglu_fwd_launch(const void*, void*, int64_t, int, hipStream_t);
int swiglu_bwd_launch(const void*, const void*, void*, int64_t, int, hipStream_t);
int swiglu_bwd_dual_launch(const void*, const void*, void*, void*, int64_t, int, hipStream_t);
int swiglu_fwd_dual_launch(const void*, void*, void*, int64_t, int, hipStream_t);
int xent_stats_launch(const void*, int, const int64_t*, float*, int64_t, int, int64_t, int64_t, hipStream_t);
int xent_bwd_launch(const void*, int, const int64_t*, const float*, void*, int64_t, int, int64_t, int64_t, int64_t, float,
                    int64_t, hipStream_t);
int flat_reduce_launch(const void*, int, int64_t, int, float*, float*, int, hipStream_t);
int adamw_flat_launch(float*, const void*, int, float*, float*, void*, int64_t, float, float, float, float, float, float,
                      float, const float*, float, uint32_t, const float*, hipStream_t);
int clip_coef_launch(const float*, float*, float, int, hipStream_t);
int scale_flat_launch(float*, int64_t, const float*, hipStream_t);
int embedding_fwd_launch(const int64_t*, const void*, void*, int64_t, int, int64_t, int64_t, hipStream_t);
int embedding_bwd_launch(const int64_t*, const void*, float*, int64_t, int, int64_t, int64_t, hipStream_t);
int decode_attn_launch(const void*, const int64_t*, const void*, const void*, const int64_t*, const int*, const int*,
                       float*, float*, float*, int*, void*, const int64_t*, int, int, int, int, int, int, float, hipStream_t);
int kv_cache_write_launch(const void*, const void*, const int64_t*, void*, void*, const int64_t*, const int*, const int*,
                          int, int, int, int, int, hipStream_t);
int argmax_launch(const void*, int, int64_t, int, int, int64_t*, hipStream_t);
int greedy_advance_launch(const void*, int, int64_t, int, int, unsigned long long*, int64_t*, int64_t, int, int64_t*, int64_t*,
                          int64_t*, int*, hipStream_t);
int topk_sample_launch(const void*, int, int64_t, int, int, int, float, const float*, int64_t*, float*, int64_t*,
                       hipStream_t);
int gemv_launch(const void*, int64_t, const void*, int64_t, int, const float*, float, const void*, void*, int64_t, int, int,
                int, int, hipStream_t);
int dequant_int8_launch(const void*, int64_t, const float*, float, void*, int, int, hipStream_t);
int expert_gemv_launch(const void*, int64_t, const void*, int64_t, int64_t, const int32_t*, int, int, void*, int64_t, int,
                       int, int, hipStream_t);
void dgemv_set_knob(int, int);
void decode_attn_set_v2(int);
void decode_attn_set_prefetch(const void*, int64_t, const void*, int64_t, int);
void decode_attn_set_trace(uint64_t*);
int dgemv_launch(int, const void*, int64_t, const void*, float, const void*, int64_t, void*, int64_t, int, int, int, int,
                 int, int, const float*, const float*, const int64_t*, int, void*, void*, int64_t, int64_t, int64_t,
                 const int*, int, int, const float*, float*, hipStream_t, const int64_t*, int64_t, void*, float*);
int grouped_gemm_launch(int, const void*, const void*, void*, const int*, int, int, int, int, int, hipStream_t);
int wgrad_gemm_launch(const void*, int64_t, const void*, int64_t, float*, int64_t, int, int, int, int, hipStream_t);
int wgrad_gemm_choose_splits(int, int, int);
int decode_attn_oproj_launch(const void*, const int64_t*, const void*, const void*, const int64_t*, const int*, const int*,
                             const void*, int64_t, int, float*, float*, float*, float*, float*, int, int, int, int, int, int, float, hipStream_t);
int grouped_rowgemm_launch(int, const void*, const void*, void*, const int*, int, int, int, int, hipStream_t);
int wgrad_gemm_grouped_launch(const void*, int64_t, const void*, int64_t, float*, int64_t, int64_t, const int*, int, int,
                              int, int, hipStream_t);
void wgrad_gemm_set_ablate(int);
int dense_gemm_launch(int, int, const void*, int64_t, const void*, int64_t, void*, int64_t, int, int, int, int, hipStream_t);
int dense_gemm_choose_splits(int, int, int);
void dense_gemm_set_pipe(int);
void decode_attn_set_oproj_maxl(int);
int decode_attn_oproj_maxl();
int decode_attn_sync_error(bool);
void decode_attn_set_sync(int);
void grouped_rowgemm_set_pp(int);
void wgrad_gemm_set_pp(int);
int cu_stream_launch(const void*, void*, int64_t, int, int64_t, hipStream_t);
int moe_combine_fwd_launch(const void*, const int64_t*, const float*, void*, int64_t, int, int, hipStream_t);
int moe_combine_bwd_launch(const void*, const void*, const int64_t*, const float*, void*, float*, int64_t, int, int,
                           hipStream_t);
}  // namespace nxd

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

void check_rc(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed with code ", rc); }

void check_cuda(const at::Tensor& t, const char* n) { TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor"); }

void check_bf16(const at::Tensor& t, const char* n) {
  check_cuda(t, n);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, n, " must be bfloat16");
}

void check_aligned16(const at::Tensor& t, const char* n) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n, " must be 16-byte aligned");
}

// [B, S, H, D] view with unit stride on D and 16-B aligned rows
void bshd_strides(const at::Tensor& t, const char* n, int64_t* s) {
  check_bf16(t, n);
  TORCH_CHECK(t.dim() == 4, n, " must be [B, S, H, D]");
  TORCH_CHECK(t.stride(3) == 1, n, " must have unit stride on D");
  for (int i = 0; i < 3; ++i) TORCH_CHECK(t.stride(i) % 8 == 0 || t.size(i) == 1, n, " strides must be multiples of 8 elements");
  check_aligned16(t, n);
  s[0] = t.stride(0);
  s[1] = t.stride(1);
  s[2] = t.stride(2);
}

// dropout_p in [0, 1): keep iff hash >= p * 2^32 (truncated, as ops/attention_dropout.py), scale 1/(1-p)
nxd::DropoutArgs dropout_args(double p, int64_t seed, int64_t head_offset) {
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout_p must be in [0, 1)");
  nxd::DropoutArgs d;
  d.thresh = (uint32_t)(uint64_t)(p * 4294967296.0);
  d.scale = (float)(1.0 / (1.0 - p));
  d.seed = (uint32_t)(seed & 0xFFFFFFFFll);
  d.head_offset = (int)head_offset;
  return d;
}

void flash_attn_fwd(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor lse, double scale, bool causal,
                    int64_t causal_offset, double dropout_p, int64_t seed, int64_t head_offset) {
  int64_t qs[3], ks[3], vs[3], os[3];
  bshd_strides(q, "q", qs);
  bshd_strides(k, "k", ks);
  bshd_strides(v, "v", vs);
  bshd_strides(o, "o", os);
  const int B = q.size(0), Sq = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == Sk && v.size(2) == Hkv, "k/v shape mismatch");
  TORCH_CHECK(k.size(3) == D && v.size(3) == D && o.sizes() == q.sizes(), "head dim / output shape mismatch");
  TORCH_CHECK(D == 64 || D == 128, "head_dim must be 64 or 128");
  TORCH_CHECK(Hkv > 0 && Hq % Hkv == 0, "num q heads must be a multiple of num kv heads");
  TORCH_CHECK(Sk > 0, "empty key sequence");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == (int64_t)B * Hq * Sq,
              "lse must be contiguous fp32 [B, Hq, Sq]");
  check_rc(nxd::flash_attn_fwd_launch(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), qs, ks,
                                      vs, os, B, Sq, Sk, Hq, Hkv, D, (float)scale, causal ? 1 : 0, (int)causal_offset,
                                      dropout_args(dropout_p, seed, head_offset), cur_stream()),
           "flash_attn_fwd");
}

void flash_attn_bwd(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor dout, at::Tensor lse,
                    at::Tensor dq, at::Tensor dk, at::Tensor dv, double scale, bool causal, int64_t causal_offset,
                    double dropout_p, int64_t seed, int64_t head_offset) {
  int64_t qs[3], ks[3], vs[3], os[3], dos[3], dqs[3], dks[3], dvs[3];
  bshd_strides(q, "q", qs);
  bshd_strides(k, "k", ks);
  bshd_strides(v, "v", vs);
  bshd_strides(o, "o", os);
  bshd_strides(dout, "dout", dos);
  bshd_strides(dq, "dq", dqs);
  bshd_strides(dk, "dk", dks);
  bshd_strides(dv, "dv", dvs);
  const int B = q.size(0), Sq = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.sizes() == v.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "k/v/dk/dv shape mismatch");
  TORCH_CHECK(o.sizes() == q.sizes() && dout.sizes() == q.sizes() && dq.sizes() == q.sizes(), "q/o/dout/dq shape mismatch");
  TORCH_CHECK(k.size(0) == B && k.size(3) == D, "k shape mismatch");
  TORCH_CHECK(D == 64 || D == 128, "head_dim must be 64 or 128");
  TORCH_CHECK(Hkv > 0 && Hq % Hkv == 0, "num q heads must be a multiple of num kv heads");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == (int64_t)B * Hq * Sq, "bad lse");
  auto opts = q.options().dtype(at::kFloat);
  // fp32 workspace: dQ / dK / dV accumulators + per-row constants (sized by the kernel TU)
  at::Tensor ws = at::empty({nxd::flash_attn_bwd_workspace(B, Sq, Sk, Hq, Hkv, D, causal ? 1 : 0, (int)causal_offset)}, opts);
  check_rc(nxd::flash_attn_bwd_launch(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                                      lse.data_ptr<float>(), ws.data_ptr<float>(), dq.data_ptr(),
                                      dk.data_ptr(), dv.data_ptr(), qs, ks, vs, os, dos, dqs, dks, dvs, B, Sq, Sk, Hq, Hkv, D,
                                      (float)scale, causal ? 1 : 0, (int)causal_offset,
                                      dropout_args(dropout_p, seed, head_offset), cur_stream()),
           "flash_attn_bwd");
}

void rows_check(const at::Tensor& t, const char* n, int64_t H) {
  check_bf16(t, n);
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
  TORCH_CHECK(t.size(-1) == H, n, " last dim mismatch");
  check_aligned16(t, n);
}

void rmsnorm_fwd(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> h_out,
                 at::Tensor rstd, double eps) {
  const int64_t H = x.size(-1);
  const int64_t rows = x.numel() / H;
  rows_check(x, "x", H);
  rows_check(y, "y", H);
  check_bf16(w, "w");
  TORCH_CHECK(w.is_contiguous() && w.numel() == H, "w must be [H]");
  TORCH_CHECK(H % 8 == 0 && H <= 16384, "hidden size must be a multiple of 8 and <= 16384");
  TORCH_CHECK(rstd.scalar_type() == at::kFloat && rstd.numel() == rows, "rstd must be fp32 [rows]");
  const void* rp = nullptr;
  void* hp = nullptr;
  if (res.has_value()) {
    rows_check(*res, "residual", H);
    TORCH_CHECK(res->numel() == x.numel(), "residual shape mismatch");
    TORCH_CHECK(h_out.has_value(), "h_out required with residual");
    rows_check(*h_out, "h_out", H);
    rp = res->data_ptr();
    hp = h_out->data_ptr();
  }
  check_rc(nxd::rmsnorm_fwd_launch(x.data_ptr(), rp, w.data_ptr(), y.data_ptr(), hp, rstd.data_ptr<float>(), rows, (int)H,
                                   (float)eps, cur_stream()),
           "rmsnorm_fwd");
}

void rmsnorm_bwd(at::Tensor dy, at::Tensor h, at::Tensor w, at::Tensor rstd, c10::optional<at::Tensor> dres, at::Tensor dx,
                 at::Tensor dw, bool accumulate) {
  const int64_t H = h.size(-1);
  const int64_t rows = h.numel() / H;
  rows_check(dy, "dy", H);
  rows_check(h, "h", H);
  rows_check(dx, "dx", H);
  TORCH_CHECK(dy.numel() == h.numel() && dx.numel() == h.numel(), "shape mismatch");
  TORCH_CHECK(H % 8 == 0 && H <= 16384, "bad hidden size");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.is_contiguous() && dw.numel() == H, "dw must be fp32 [H]");
  TORCH_CHECK(rstd.scalar_type() == at::kFloat && rstd.numel() == rows, "rstd must be fp32 [rows]");
  const void* drp = nullptr;
  if (dres.has_value()) {
    rows_check(*dres, "dres", H);
    TORCH_CHECK(dres->numel() == h.numel(), "dres shape mismatch");
    drp = dres->data_ptr();
  }
  const int G = nxd::rmsnorm_bwd_num_partials(rows);
  at::Tensor part = at::empty({(int64_t)G * H}, h.options().dtype(at::kFloat));
  check_rc(nxd::rmsnorm_bwd_launch(dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), drp, dx.data_ptr(),
                                   part.data_ptr<float>(), dw.data_ptr<float>(), accumulate ? 1 : 0, rows, (int)H, cur_stream()),
           "rmsnorm_bwd");
}

void rope_inplace(at::Tensor buf, int64_t T, int64_t W, int64_t col0, int64_t nheads, int64_t D, at::Tensor cos_t,
                  at::Tensor sin_t, c10::optional<at::Tensor> pos, int64_t pos_div, int64_t pos_mod, double sign) {
  check_bf16(buf, "buf");
  check_aligned16(buf, "buf");
  TORCH_CHECK(D == 64 || D == 128 || D == 256, "rope head_dim must be 64/128/256");
  TORCH_CHECK(W % 8 == 0 && col0 % 8 == 0, "rope row stride / column offset must be multiples of 8");
  TORCH_CHECK(col0 + nheads * D <= W, "rope heads exceed the row");
  TORCH_CHECK(buf.storage().nbytes() >= (size_t)((T - 1) * W + W) * 2 + buf.storage_offset() * 2 || T == 0,
              "rope buffer too small");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                  sin_t.is_contiguous() && cos_t.size(-1) == D / 2 && sin_t.sizes() == cos_t.sizes(),
              "cos/sin tables must be contiguous fp32 [max_pos, D/2]");
  const int64_t* pp = nullptr;
  if (pos.has_value()) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->is_contiguous() && pos->numel() == T, "pos must be int64 [T]");
    pp = pos->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(pos_div > 0 && pos_mod > 0 && pos_mod <= cos_t.size(0), "bad implicit positions");
  }
  check_rc(nxd::rope_inplace_launch(buf.data_ptr(), T, W, (int)col0, (int)nheads, (int)D, cos_t.data_ptr<float>(),
                                    sin_t.data_ptr<float>(), pp, pos_div, pos_mod, (float)sign, cur_stream()),
           "rope");
}

// dst [C, R] = src [R, C]^T (bf16, unit inner strides, row strides multiples of 8 elements)
void transpose_bf16(at::Tensor src, at::Tensor dst) {
  check_bf16(src, "src");
  check_bf16(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2, "transpose_bf16: 2-D tensors");
  TORCH_CHECK(src.stride(1) == 1 && dst.stride(1) == 1, "transpose_bf16: unit inner stride");
  TORCH_CHECK(dst.size(0) == src.size(1) && dst.size(1) == src.size(0), "transpose_bf16: shape mismatch");
  check_aligned16(src, "src");
  check_aligned16(dst, "dst");
  check_rc(nxd::transpose_bf16_launch(src.data_ptr(), dst.data_ptr(), src.size(0), src.size(1), src.stride(0),
                                      dst.stride(0), cur_stream()),
           "transpose_bf16");
}

void swiglu_fwd(at::Tensor gu, at::Tensor h) {
  const int64_t I2 = gu.size(-1);
  TORCH_CHECK(I2 % 16 == 0, "gate_up width must be a multiple of 16");
  rows_check(gu, "gate_up", I2);
  rows_check(h, "h", I2 / 2);
  TORCH_CHECK(h.numel() * 2 == gu.numel(), "shape mismatch");
  check_rc(nxd::swiglu_fwd_launch(gu.data_ptr(), h.data_ptr(), gu.numel() / I2, (int)(I2 / 2), cur_stream()), "swiglu_fwd");
}

void swiglu_bwd(at::Tensor gu, at::Tensor dh, at::Tensor dgu) {
  const int64_t I2 = gu.size(-1);
  TORCH_CHECK(I2 % 16 == 0, "gate_up width must be a multiple of 16");
  rows_check(gu, "gate_up", I2);
  rows_check(dh, "dh", I2 / 2);
  rows_check(dgu, "dgu", I2);
  TORCH_CHECK(dh.numel() * 2 == gu.numel() && dgu.numel() == gu.numel(), "shape mismatch");
  check_rc(nxd::swiglu_bwd_launch(gu.data_ptr(), dh.data_ptr(), dgu.data_ptr(), gu.numel() / I2, (int)(I2 / 2), cur_stream()),
           "swiglu_bwd");
}

// h = silu(g) * u and its transpose h_t [I, rows] (contiguous); rows and I multiples of 64.
void swiglu_fwd_dual(at::Tensor gu, at::Tensor h, at::Tensor h_t) {
  const int64_t I2 = gu.size(-1);
  rows_check(gu, "gate_up", I2);
  rows_check(h, "h", I2 / 2);
  TORCH_CHECK(h.numel() * 2 == gu.numel(), "shape mismatch");
  const int64_t N = gu.numel() / I2;
  check_bf16(h_t, "h_t");
  TORCH_CHECK(h_t.dim() == 2 && h_t.size(0) == I2 / 2 && h_t.size(1) == N && h_t.is_contiguous(),
              "h_t must be contiguous [I, rows]");
  TORCH_CHECK(N % 64 == 0 && (I2 / 2) % 64 == 0, "swiglu_fwd_dual: rows and I must be multiples of 64");
  check_aligned16(h_t, "h_t");
  check_rc(nxd::swiglu_fwd_dual_launch(gu.data_ptr(), h.data_ptr(), h_t.data_ptr(), N, (int)(I2 / 2), cur_stream()),
           "swiglu_fwd_dual");
}

// dgu and its transpose dgu_t [2I, rows] (contiguous) in one kernel; rows and I multiples of 64.
void swiglu_bwd_dual(at::Tensor gu, at::Tensor dh, at::Tensor dgu, at::Tensor dgu_t) {
  const int64_t I2 = gu.size(-1);
  rows_check(gu, "gate_up", I2);
  rows_check(dh, "dh", I2 / 2);
  rows_check(dgu, "dgu", I2);
  TORCH_CHECK(dh.numel() * 2 == gu.numel() && dgu.numel() == gu.numel(), "shape mismatch");
  const int64_t N = gu.numel() / I2;
  check_bf16(dgu_t, "dgu_t");
  TORCH_CHECK(dgu_t.dim() == 2 && dgu_t.size(0) == I2 && dgu_t.size(1) == N && dgu_t.is_contiguous(),
              "dgu_t must be contiguous [2I, rows]");
  TORCH_CHECK(N % 64 == 0 && (I2 / 2) % 64 == 0, "swiglu_bwd_dual: rows and I must be multiples of 64");
  check_aligned16(dgu_t, "dgu_t");
  check_rc(nxd::swiglu_bwd_dual_launch(gu.data_ptr(), dh.data_ptr(), dgu.data_ptr(), dgu_t.data_ptr(), N, (int)(I2 / 2),
                                       cur_stream()),
           "swiglu_bwd_dual");
}

void logits_check(const at::Tensor& x) {
  check_cuda(x, "logits");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "logits must be [N, V] with unit column stride");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "logits must be bf16 or fp32");
  TORCH_CHECK(x.size(1) % 8 == 0 && x.stride(0) % 8 == 0, "vocab shard and row stride must be multiples of 8");
  check_aligned16(x, "logits");
}

void xent_stats(at::Tensor logits, at::Tensor labels, at::Tensor stats, int64_t vocab_start) {
  logits_check(logits);
  const int64_t N = logits.size(0);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == N, "labels must be int64 [N]");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.is_contiguous() && stats.numel() == N * 4, "stats must be fp32 [N,4]");
  check_rc(nxd::xent_stats_launch(logits.data_ptr(), logits.scalar_type() == at::kFloat, labels.data_ptr<int64_t>(),
                                  stats.data_ptr<float>(), N, (int)logits.size(1), logits.stride(0), vocab_start, cur_stream()),
           "xent_stats");
}

void xent_bwd(at::Tensor logits, at::Tensor labels, at::Tensor gstat, at::Tensor grad, int64_t vocab_start, double eps,
              int64_t vocab_total) {
  logits_check(logits);
  const int64_t N = logits.size(0);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == N, "labels must be int64 [N]");
  TORCH_CHECK(gstat.scalar_type() == at::kFloat && gstat.is_contiguous() && gstat.numel() == N * 4, "gstat must be fp32 [N,4]");
  check_bf16(grad, "grad");
  TORCH_CHECK(grad.dim() == 2 && grad.size(0) == N && grad.size(1) == logits.size(1) && grad.stride(1) == 1 &&
                  grad.stride(0) % 8 == 0,
              "grad must be bf16 [N, V]");
  check_aligned16(grad, "grad");
  check_rc(nxd::xent_bwd_launch(logits.data_ptr(), logits.scalar_type() == at::kFloat, labels.data_ptr<int64_t>(),
                                gstat.data_ptr<float>(), grad.data_ptr(), N, (int)logits.size(1), logits.stride(0),
                                grad.stride(0), vocab_start, (float)eps, vocab_total, cur_stream()),
           "xent_bwd");
}

void flat_check(const at::Tensor& t, const char* n) {
  check_cuda(t, n);
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
  check_aligned16(t, n);
}

void flat_reduce(at::Tensor x, int64_t mode, at::Tensor out, bool accumulate) {
  flat_check(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "x must be bf16/fp32");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 1, "out must be fp32");
  TORCH_CHECK(mode == 0 || mode == 1, "mode must be 0 (sumsq) or 1 (max abs)");
  at::Tensor part = at::empty({2048}, x.options().dtype(at::kFloat));
  check_rc(nxd::flat_reduce_launch(x.data_ptr(), x.scalar_type() == at::kBFloat16, x.numel(), (int)mode, part.data_ptr<float>(),
                                   out.data_ptr<float>(), accumulate ? 1 : 0, cur_stream()),
           "flat_reduce");
}

void adamw_flat(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, c10::optional<at::Tensor> p16, double lr, double b1,
                double b2, double eps, double wd, double bc1, double bc2, c10::optional<at::Tensor> gscale, double gscale_host,
                int64_t sr_seed, c10::optional<at::Tensor> hyper) {
  flat_check(p, "p");
  flat_check(g, "g");
  flat_check(m, "m");
  flat_check(v, "v");
  TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "p/m/v must be fp32");
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "g must be fp32/bf16");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "size mismatch");
  void* o = nullptr;
  if (p16.has_value()) {
    flat_check(*p16, "p16");
    TORCH_CHECK(p16->scalar_type() == at::kBFloat16 && p16->numel() == n, "p16 must be bf16 of the same size");
    o = p16->data_ptr();
  }
  const float* gs = nullptr;
  if (gscale.has_value()) {
    TORCH_CHECK(gscale->scalar_type() == at::kFloat && gscale->is_cuda(), "gscale must be a fp32 GPU tensor");
    gs = gscale->data_ptr<float>();
  }
  if (hyper.has_value()) {
    TORCH_CHECK(hyper->scalar_type() == at::kFloat && hyper->is_cuda() && hyper->numel() >= 3 && hyper->is_contiguous(),
                "hyper must be a contiguous fp32 GPU tensor [lr, bc1, bc2]");
  }
  check_rc(nxd::adamw_flat_launch(p.data_ptr<float>(), g.data_ptr(), g.scalar_type() == at::kBFloat16, m.data_ptr<float>(),
                                  v.data_ptr<float>(), o, n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1,
                                  (float)bc2, gs, (float)gscale_host, (uint32_t)(sr_seed & 0xffffffff),
                                  hyper.has_value() ? hyper->data_ptr<float>() : nullptr, cur_stream()),
           "adamw_flat");
}

void clip_coef(at::Tensor stat, at::Tensor coef, double max_norm, bool is_sumsq) {
  TORCH_CHECK(stat.scalar_type() == at::kFloat && coef.scalar_type() == at::kFloat && coef.numel() >= 2 && stat.is_cuda(),
              "clip_coef: fp32 GPU tensors, coef of size >= 2");
  check_rc(nxd::clip_coef_launch(stat.data_ptr<float>(), coef.data_ptr<float>(), (float)max_norm, is_sumsq ? 1 : 0, cur_stream()),
           "clip_coef");
}

void scale_flat(at::Tensor x, at::Tensor s) {
  flat_check(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && s.scalar_type() == at::kFloat && s.is_cuda(), "fp32 tensors required");
  check_rc(nxd::scale_flat_launch(x.data_ptr<float>(), x.numel(), s.data_ptr<float>(), cur_stream()), "scale_flat");
}

void embedding_fwd(at::Tensor ids, at::Tensor w, at::Tensor out, int64_t start) {
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.is_cuda(), "ids must be int64 contiguous");
  check_bf16(w, "w");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "w must be contiguous [V, H]");
  const int64_t H = w.size(1);
  TORCH_CHECK(H % 8 == 0, "embedding dim must be a multiple of 8");
  rows_check(out, "out", H);
  TORCH_CHECK(out.numel() == ids.numel() * H, "out shape mismatch");
  check_aligned16(w, "w");
  check_rc(nxd::embedding_fwd_launch(ids.data_ptr<int64_t>(), w.data_ptr(), out.data_ptr(), ids.numel(), (int)H, start,
                                     w.size(0), cur_stream()),
           "embedding_fwd");
}

void embedding_bwd(at::Tensor ids, at::Tensor dout, at::Tensor dw, int64_t start) {
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.is_cuda(), "ids must be int64 contiguous");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.dim() == 2 && dw.is_contiguous(), "dw must be fp32 [V, H]");
  const int64_t H = dw.size(1);
  rows_check(dout, "dout", H);
  TORCH_CHECK(dout.numel() == ids.numel() * H, "dout shape mismatch");
  check_rc(nxd::embedding_bwd_launch(ids.data_ptr<int64_t>(), dout.data_ptr(), dw.data_ptr<float>(), ids.numel(), (int)H,
                                     start, dw.size(0), cur_stream()),
           "embedding_bwd");
}

// q: [B, T, Hq, D] (strided), caches: [Bc, Hkv, Lmax, D] contiguous, out: [B, T, Hq, D]
// Zero-initialised split counters of the fused decode-attention kernel (the last workgroup of each
// (batch, kv head) resets its counter, so the buffer stays valid across launches and graph replays).
// Grown outside of stream capture only.
int* decode_counters(int dev, int64_t n) {
  static std::vector<at::Tensor> bufs;
  if ((int)bufs.size() <= dev) bufs.resize(dev + 1);
  if (!bufs[dev].defined() || bufs[dev].numel() < n) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(cur_stream(), &st);
    TORCH_CHECK(st == hipStreamCaptureStatusNone, "decode_attn: first call for this batch must happen before graph capture");
    bufs[dev] = at::zeros({std::max<int64_t>(n, 1024)}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev));
  }
  return bufs[dev].data_ptr<int>();
}

// Arm the NEXT decode_attn launch with up to two weight ranges to stream into the Infinity Cache
// from spare workgroups of its grid (o_proj and the head of gate_up in the fused decode layer).
void decode_attn_prefetch(c10::optional<at::Tensor> a, int64_t a_bytes, c10::optional<at::Tensor> b, int64_t b_bytes,
                          int64_t wgs) {
  auto rng = [](const c10::optional<at::Tensor>& t, int64_t n) -> std::pair<const void*, int64_t> {
    if (!t.has_value() || !t->defined()) return {nullptr, 0};
    check_cuda(*t, "prefetch range");
    TORCH_CHECK(t->is_contiguous(), "prefetch range must be contiguous");
    const int64_t total = t->numel() * t->element_size();
    return {t->data_ptr(), std::max<int64_t>(0, std::min(n < 0 ? total : n, total))};
  };
  const auto ra = rng(a, a_bytes), rb = rng(b, b_bytes);
  nxd::decode_attn_set_prefetch(ra.first, ra.second, rb.first, rb.second, (int)wgs);
}

// Fused decode attention + o_proj (csrc/decode_attn.hip FUSE): oacc [B*T, Hout] fp32 (zero on entry)
// += o_proj(attention).  Returns false (nothing launched) for shapes the fused kernel does not cover.
bool decode_attn_oproj(at::Tensor q, at::Tensor kc, at::Tensor vc, c10::optional<at::Tensor> cache_idx, at::Tensor seq_len,
                       at::Tensor wo, at::Tensor oacc, double scale) {
  int64_t qs[3];
  bshd_strides(q, "q", qs);
  check_bf16(kc, "k_cache");
  check_bf16(vc, "v_cache");
  check_bf16(wo, "wo");
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.sizes() == kc.sizes() && vc.is_contiguous(),
              "caches must be contiguous [B, Hkv, Lmax, D]");
  const int B = q.size(0), T = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Hkv = kc.size(1), Lmax = kc.size(2);
  TORCH_CHECK(kc.size(3) == D, "head dim mismatch");
  TORCH_CHECK(wo.dim() == 2 && wo.stride(1) == 1 && wo.size(1) == (int64_t)Hq * D, "wo must be [Hout, Hq * D]");
  check_aligned16(wo, "wo");
  const int64_t Hout = wo.size(0);
  TORCH_CHECK(oacc.scalar_type() == at::kFloat && oacc.is_cuda() && oacc.is_contiguous() && oacc.dim() == 2 &&
                  oacc.size(0) >= (int64_t)B * T && oacc.size(1) == Hout,
              "oacc must be fp32 contiguous [>= B*T, Hout]");
  TORCH_CHECK(seq_len.scalar_type() == at::kInt && seq_len.numel() == B && seq_len.is_contiguous(), "seq_len must be int32 [B]");
  const int* ci = nullptr;
  if (cache_idx.has_value()) {
    TORCH_CHECK(cache_idx->scalar_type() == at::kInt && cache_idx->numel() == B, "cache_idx must be int32 [B]");
    ci = cache_idx->data_ptr<int>();
  } else {
    TORCH_CHECK(kc.size(0) >= B, "cache batch too small");
  }
  if (Hkv <= 0 || Hq % Hkv || Hout > INT32_MAX) return false;
  const int64_t cs[3] = {kc.stride(0), kc.stride(1), kc.stride(2)};
  // past the fused kernel's one-pass limit: split attention partials (keys per split >= 128), merged
  // inside the o_proj launch
  at::Tensor part;
  float *po = nullptr, *pm = nullptr, *pl = nullptr, *mo = nullptr;
  if (Lmax > nxd::decode_attn_oproj_maxl()) {
    const int64_t M = (int64_t)(Hq / Hkv) * T;
    const int64_t rows = (int64_t)B * Hkv * ((Lmax + 127) / 128) * M;
    part = at::empty({rows * (D + 2) + (int64_t)B * Hkv * M * D}, q.options().dtype(at::kFloat));
    po = part.data_ptr<float>(); pm = po + rows * D; pl = pm + rows; mo = pl + rows;
  }
  const int rc = nxd::decode_attn_oproj_launch(q.data_ptr(), qs, kc.data_ptr(), vc.data_ptr(), cs, ci, seq_len.data_ptr<int>(),
                                               wo.data_ptr(), wo.stride(0), (int)Hout, oacc.data_ptr<float>(), po, pm, pl, mo, B, T,
                                               Hq, Hkv, D, Lmax, (float)scale, cur_stream());
  if (rc == -1) return false;
  check_rc(rc, "decode_attn_oproj");
  return true;
}

void decode_attn(at::Tensor q, at::Tensor kc, at::Tensor vc, c10::optional<at::Tensor> cache_idx, at::Tensor seq_len,
                 at::Tensor out, double scale, int64_t nsplit) {
  int64_t qs[3], os[3];
  bshd_strides(q, "q", qs);
  bshd_strides(out, "out", os);
  check_bf16(kc, "k_cache");
  check_bf16(vc, "v_cache");
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.sizes() == kc.sizes() && vc.is_contiguous(),
              "caches must be contiguous [B, Hkv, Lmax, D]");
  const int B = q.size(0), T = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Hkv = kc.size(1), Lmax = kc.size(2);
  TORCH_CHECK(kc.size(3) == D && (D == 64 || D == 128), "head dim mismatch (64/128)");
  TORCH_CHECK(Hkv > 0 && Hq % Hkv == 0, "q heads must be a multiple of kv heads");
  TORCH_CHECK((int64_t)(Hq / Hkv) * T <= 64, "decode supports (Hq/Hkv) * new_tokens <= 64");
  TORCH_CHECK(nsplit >= 1 && nsplit * 128 >= Lmax, "nsplit * 128 must cover the cache length");
  TORCH_CHECK(seq_len.scalar_type() == at::kInt && seq_len.numel() == B && seq_len.is_contiguous(), "seq_len must be int32 [B]");
  const int* ci = nullptr;
  if (cache_idx.has_value()) {
    TORCH_CHECK(cache_idx->scalar_type() == at::kInt && cache_idx->numel() == B, "cache_idx must be int32 [B]");
    ci = cache_idx->data_ptr<int>();
  } else {
    TORCH_CHECK(kc.size(0) >= B, "cache batch too small");
  }
  TORCH_CHECK(out.sizes() == q.sizes(), "out shape mismatch");
  const int M = (Hq / Hkv) * T;
  auto opts = q.options().dtype(at::kFloat);
  at::Tensor po = at::empty({(int64_t)B * Hkv * nsplit * M * D}, opts);
  at::Tensor pm = at::empty({(int64_t)B * Hkv * nsplit * M}, opts);
  at::Tensor pl = at::empty({(int64_t)B * Hkv * nsplit * M}, opts);
  const int64_t cs[3] = {kc.stride(0), kc.stride(1), kc.stride(2)};
  (void)Lmax;
  TORCH_CHECK(os[2] % 8 == 0 || Hq == 1, "out head stride must keep 16-byte alignment");
  int* counters = decode_counters(q.device().index(), (int64_t)B * Hkv);
  check_rc(nxd::decode_attn_launch(q.data_ptr(), qs, kc.data_ptr(), vc.data_ptr(), cs, ci, seq_len.data_ptr<int>(),
                                   po.data_ptr<float>(), pm.data_ptr<float>(), pl.data_ptr<float>(), counters, out.data_ptr(),
                                   os, B, T, Hq, Hkv, D, (int)nsplit, (float)scale, cur_stream()),
           "decode_attn");
  nxd::decode_attn_set_prefetch(nullptr, 0, nullptr, 0, 0);   // armed ranges never outlive one call
}

// k, v: [B, T, Hkv, D] strided; caches [Bc, Hkv, Lmax, D]; pos: int32 [B] position of token 0
void kv_cache_write(at::Tensor k, at::Tensor v, at::Tensor kc, at::Tensor vc, c10::optional<at::Tensor> cache_idx,
                    at::Tensor pos) {
  int64_t ks[3], vs[3];
  bshd_strides(k, "k", ks);
  bshd_strides(v, "v", vs);
  TORCH_CHECK(ks[0] == vs[0] && ks[1] == vs[1] && ks[2] == vs[2] && k.sizes() == v.sizes(), "k/v layouts must match");
  check_bf16(kc, "k_cache");
  check_bf16(vc, "v_cache");
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.sizes() == kc.sizes() && vc.is_contiguous(), "bad caches");
  const int B = k.size(0), T = k.size(1), H = k.size(2), D = k.size(3);
  TORCH_CHECK(kc.size(1) == H && kc.size(3) == D && D % 8 == 0, "cache / new kv mismatch");
  TORCH_CHECK(pos.scalar_type() == at::kInt && pos.numel() == B, "pos must be int32 [B]");
  const int* ci = nullptr;
  if (cache_idx.has_value()) {
    TORCH_CHECK(cache_idx->scalar_type() == at::kInt && cache_idx->numel() == B, "cache_idx must be int32 [B]");
    ci = cache_idx->data_ptr<int>();
  } else {
    TORCH_CHECK(kc.size(0) >= B, "cache batch too small");
  }
  const int64_t cs[3] = {kc.stride(0), kc.stride(1), kc.stride(2)};
  check_rc(nxd::kv_cache_write_launch(k.data_ptr(), v.data_ptr(), ks, kc.data_ptr(), vc.data_ptr(), cs, ci, pos.data_ptr<int>(),
                                      B, T, H, D, (int)kc.size(2), cur_stream()),
           "kv_cache_write");
}

void argmax_rows(at::Tensor x, at::Tensor out) {
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be [B, V]");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x must be fp32/bf16");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.numel() == x.size(0), "out must be int64 [B]");
  check_rc(nxd::argmax_launch(x.data_ptr(), x.scalar_type() == at::kFloat, x.stride(0), (int)x.size(0), (int)x.size(1),
                              out.data_ptr<int64_t>(), cur_stream()),
           "argmax");
}

// greedy decode tail: argmax of logits [B, V] -> out[:, step], tokens, positions + 1, cache_len + 1,
// step + 1 (the decode loop's feed-back, graph-capturable); slot: int64 [B] zeros between calls
void greedy_advance(at::Tensor logits, at::Tensor slot, at::Tensor out, at::Tensor step, at::Tensor tokens,
                    at::Tensor positions, at::Tensor cache_len) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [B, V] with unit stride");
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16, "logits must be fp32/bf16");
  const int64_t B = logits.size(0);
  TORCH_CHECK(slot.scalar_type() == at::kLong && slot.numel() == B && slot.is_contiguous(), "slot: int64 [B]");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.dim() == 2 && out.size(0) == B && out.stride(1) == 1, "out: int64 [B, S]");
  TORCH_CHECK(step.scalar_type() == at::kLong && step.numel() == 1, "step: int64 [1]");
  TORCH_CHECK(tokens.scalar_type() == at::kLong && tokens.numel() == B && tokens.is_contiguous(), "tokens: int64 [B]");
  TORCH_CHECK(positions.scalar_type() == at::kLong && positions.numel() == B && positions.is_contiguous(), "positions: int64 [B]");
  TORCH_CHECK(cache_len.scalar_type() == at::kInt && cache_len.numel() == B && cache_len.is_contiguous(), "cache_len: int32 [B]");
  for (const at::Tensor* t : {&slot, &out, &step, &tokens, &positions, &cache_len}) check_cuda(*t, "decode state");
  check_rc(nxd::greedy_advance_launch(logits.data_ptr(), logits.scalar_type() == at::kFloat, logits.stride(0), (int)B,
                                      (int)logits.size(1), reinterpret_cast<unsigned long long*>(slot.data_ptr<int64_t>()),
                                      out.data_ptr<int64_t>(), out.stride(0), (int)out.size(1), step.data_ptr<int64_t>(),
                                      tokens.data_ptr<int64_t>(), positions.data_ptr<int64_t>(), cache_len.data_ptr<int>(),
                                      cur_stream()),
           "greedy_advance");
}

void topk_sample(at::Tensor x, int64_t k, double temperature, c10::optional<at::Tensor> uniform, at::Tensor out,
                 c10::optional<at::Tensor> vals, c10::optional<at::Tensor> idx) {
  check_cuda(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be [B, V]");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x must be fp32/bf16");
  const int64_t B = x.size(0);
  TORCH_CHECK(k >= 1 && k <= 1024 && k <= x.size(1), "top_k must be in [1, 1024]");
  TORCH_CHECK(out.scalar_type() == at::kLong && out.numel() == B, "out must be int64 [B]");
  const float* u = nullptr;
  if (uniform.has_value()) {
    TORCH_CHECK(uniform->scalar_type() == at::kFloat && uniform->numel() == B, "uniform must be fp32 [B]");
    u = uniform->data_ptr<float>();
  }
  float* vp = nullptr;
  int64_t* ip = nullptr;
  if (vals.has_value()) {
    TORCH_CHECK(vals->scalar_type() == at::kFloat && vals->numel() == B * k, "vals must be fp32 [B, k]");
    vp = vals->data_ptr<float>();
  }
  if (idx.has_value()) {
    TORCH_CHECK(idx->scalar_type() == at::kLong && idx->numel() == B * k, "idx must be int64 [B, k]");
    ip = idx->data_ptr<int64_t>();
  }
  check_rc(nxd::topk_sample_launch(x.data_ptr(), x.scalar_type() == at::kFloat, x.stride(0), (int)B, (int)x.size(1), (int)k,
                                   (float)temperature, u, out.data_ptr<int64_t>(), vp, ip, cur_stream()),
           "topk_sample");
}

// y[M, N] = x[M, K] @ W^T (W bf16 or int8 [Nw, K], Nw = N or 2N with glu), optional per-row fp32
// scale / per-tensor scale, optional bias [Nw]; M <= 8.
void gemv(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> scale, double tscale, c10::optional<at::Tensor> bias,
          at::Tensor y, bool glu) {
  check_cuda(x, "x");
  check_bf16(x, "x");
  check_bf16(y, "y");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "gemv: 2-D operands");
  TORCH_CHECK(x.stride(1) == 1 && w.stride(1) == 1 && y.stride(1) == 1, "gemv: unit inner strides required");
  const bool i8 = w.scalar_type() == at::kChar;
  TORCH_CHECK(i8 || w.scalar_type() == at::kBFloat16, "gemv: weight must be bf16 or int8");
  const int M = x.size(0), K = x.size(1), N = y.size(1);
  TORCH_CHECK(M >= 1 && M <= 8 && y.size(0) == M, "gemv: 1 <= M <= 8");
  TORCH_CHECK(w.size(1) == K && w.size(0) == (glu ? 2 * N : N), "gemv: weight shape mismatch");
  const int epl = i8 ? 16 : 8;
  TORCH_CHECK(K % epl == 0 && x.stride(0) % 8 == 0 && w.stride(0) % epl == 0, "gemv: K / leading dims must be multiples of ",
              epl);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "gemv: 16-byte aligned operands required");
  const float* sp = nullptr;
  if (scale.has_value()) {
    TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->is_contiguous() && scale->numel() == w.size(0),
                "gemv: scale must be fp32 [Nw]");
    sp = scale->data_ptr<float>();
  }
  const void* bp = nullptr;
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == w.size(0), "gemv: bias must be [Nw]");
    bp = bias->data_ptr();
  }
  check_rc(nxd::gemv_launch(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), i8, sp, (float)tscale, bp,
                            y.data_ptr(), y.stride(0), M, N, K, glu, cur_stream()),
           "gemv");
}

// x [X, K] bf16, w [E, Nw, K] bf16 (unit inner stride), eidx [P] int32 (values < E), y [P, N]
void expert_gemv(at::Tensor x, at::Tensor w, at::Tensor eidx, int64_t xdiv, at::Tensor y, bool glu) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  check_cuda(eidx, "eidx");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 3 && y.dim() == 2, "expert_gemv: x [X, K], w [E, Nw, K], y [P, N]");
  TORCH_CHECK(x.stride(1) == 1 && w.stride(2) == 1 && y.stride(1) == 1, "expert_gemv: unit inner strides required");
  TORCH_CHECK(eidx.scalar_type() == at::kInt && eidx.dim() == 1 && eidx.is_contiguous(), "expert_gemv: eidx int32 [P]");
  const int P = eidx.size(0), K = x.size(1), N = y.size(1);
  TORCH_CHECK(xdiv >= 1 && y.size(0) == P && (P + xdiv - 1) / xdiv <= x.size(0), "expert_gemv: x/y rows vs pairs");
  TORCH_CHECK(w.size(2) == K && w.size(1) == (glu ? 2 * N : N), "expert_gemv: weight shape mismatch");
  TORCH_CHECK(K % 8 == 0 && x.stride(0) % 8 == 0 && w.stride(1) % 8 == 0 && w.stride(0) % 8 == 0,
              "expert_gemv: K / leading dims must be multiples of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "expert_gemv: 16-byte aligned operands required");
  TORCH_CHECK(P <= 65535, "expert_gemv: too many pairs");
  if (P == 0) return;
  check_rc(nxd::expert_gemv_launch(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(1), w.stride(0),
                                   eidx.data_ptr<int32_t>(), P, (int)xdiv, y.data_ptr(), y.stride(0), N, K, glu,
                                   cur_stream()),
           "expert_gemv");
}

void dequant_int8(at::Tensor w, c10::optional<at::Tensor> scale, double tscale, at::Tensor out) {
  check_cuda(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kChar && w.dim() == 2 && w.stride(1) == 1, "dequant: int8 [N, K] weight");
  check_bf16(out, "out");
  TORCH_CHECK(out.is_contiguous() && out.sizes() == w.sizes(), "dequant: out must be contiguous [N, K]");
  const int N = w.size(0), K = w.size(1);
  TORCH_CHECK(K % 16 == 0 && w.stride(0) % 16 == 0, "dequant: K must be a multiple of 16");
  const float* sp = nullptr;
  if (scale.has_value()) {
    TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->is_contiguous() && scale->numel() == N, "dequant: scale [N]");
    sp = scale->data_ptr<float>();
  }
  check_rc(nxd::dequant_int8_launch(w.data_ptr(), w.stride(0), sp, (float)tscale, out.data_ptr(), N, K, cur_stream()),
           "dequant_int8");
}

// main_grad [M, N] fp32 += dy [T, M]^T x [T, N] (csrc/wgrad_gemm.hip): token-major bf16 operands with
// unit inner strides, row strides multiples of 8 elements, T % 32 == 0; splits <= 0 -> auto.
void wgrad_gemm(at::Tensor mg, at::Tensor dy, at::Tensor x, int64_t splits) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  check_cuda(mg, "main_grad");
  TORCH_CHECK(mg.scalar_type() == at::kFloat, "wgrad_gemm: main_grad must be fp32");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && mg.dim() == 2, "wgrad_gemm: 2-D operands");
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1);
  TORCH_CHECK(x.size(0) == T && mg.size(0) == M && mg.size(1) == N, "wgrad_gemm: shape mismatch");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1 && mg.stride(1) == 1, "wgrad_gemm: unit inner strides");
  TORCH_CHECK(dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0, "wgrad_gemm: row strides must be multiples of 8");
  TORCH_CHECK(T % 32 == 0 && M % 8 == 0 && N % 8 == 0, "wgrad_gemm: T % 32, M % 8, N % 8 must be 0");
  TORCH_CHECK(T <= INT32_MAX && M <= INT32_MAX && N <= INT32_MAX, "wgrad_gemm: dims too large");
  check_aligned16(dy, "dy");
  check_aligned16(x, "x");
  check_rc(nxd::wgrad_gemm_launch(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), mg.data_ptr<float>(),
                                  mg.stride(0), (int)T, (int)M, (int)N, (int)splits, cur_stream()),
           "wgrad_gemm");
}

// Hand-written dense GEMM (csrc/dense_gemm.hip).  layout 0 (NT): c[M, N] = a[M, K] b[N, K]^T;
// layout 1 (TN): c[M, N] = a[K, M]^T b[K, N] (token-major weight gradient).  epi 0: c bf16 = result;
// 1: c fp32 += result (deterministic); 2: c fp32 += result by split-K atomics (splits <= 0: chosen).
void dense_gemm(int64_t layout, int64_t epi, at::Tensor a, at::Tensor b, at::Tensor c, int64_t splits) {
  check_bf16(a, "dense_gemm a");
  check_bf16(b, "dense_gemm b");
  check_cuda(c, "dense_gemm c");
  TORCH_CHECK(layout == 0 || layout == 1, "dense_gemm: layout must be 0 (NT) or 1 (TN)");
  TORCH_CHECK(epi >= 0 && epi <= 2, "dense_gemm: epi must be 0, 1 or 2");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "dense_gemm: 2-D operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1, "dense_gemm: unit inner strides");
  TORCH_CHECK(c.scalar_type() == (epi == 0 ? at::kBFloat16 : at::kFloat), "dense_gemm: c dtype must be ",
              epi == 0 ? "bfloat16" : "float32");
  int64_t M, N, K;
  if (layout == 0) {
    M = a.size(0); K = a.size(1); N = b.size(0);
    TORCH_CHECK(b.size(1) == K, "dense_gemm NT: a [M, K], b [N, K]");
  } else {
    K = a.size(0); M = a.size(1); N = b.size(1);
    TORCH_CHECK(b.size(0) == K, "dense_gemm TN: a [K, M], b [K, N]");
    TORCH_CHECK(M % 8 == 0, "dense_gemm TN: M % 8 must be 0");
  }
  TORCH_CHECK(c.size(0) == M && c.size(1) == N, "dense_gemm: c must be [M, N]");
  TORCH_CHECK(K % 64 == 0 && N % 8 == 0, "dense_gemm: K % 64 and N % 8 must be 0");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && c.stride(0) % (epi == 0 ? 8 : 4) == 0,
              "dense_gemm: row strides must be multiples of 8 elements (c fp32: 4)");
  TORCH_CHECK(M <= INT32_MAX && N <= INT32_MAX && K <= INT32_MAX, "dense_gemm: dims too large");
  check_aligned16(a, "dense_gemm a");
  check_aligned16(b, "dense_gemm b");
  check_aligned16(c, "dense_gemm c");
  check_rc(nxd::dense_gemm_launch((int)layout, (int)epi, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                                  c.data_ptr(), c.stride(0), (int)M, (int)N, (int)K, (int)splits, cur_stream()),
           "dense_gemm");
}

// MoE grouped GEMMs over expert-sorted rows (csrc/grouped_gemm.hip); offs int32 [E + 1] on device.
//   mode 0: a = x [M, K], b = W [E, K, N], c = y [M, N] bf16
//   mode 1: a = dy [M, N], b = W [E, K, N], c = dx [M, K] bf16
//   mode 2: a = x [M, K], b = dy [M, N], c = dW [E, K, N] fp32 (accumulate: +=)
void grouped_gemm(int64_t mode, at::Tensor a, at::Tensor b, at::Tensor offs, at::Tensor c, bool accumulate) {
  check_bf16(a, "a");
  check_bf16(b, "b");
  check_cuda(c, "c");
  check_cuda(offs, "offs");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && c.is_contiguous(), "grouped_gemm: contiguous operands");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.dim() == 1 && offs.is_contiguous(), "grouped_gemm: offs int32 [E+1]");
  check_aligned16(a, "a");
  check_aligned16(b, "b");
  check_aligned16(c, "c");
  TORCH_CHECK(a.dim() == 2, "grouped_gemm: a must be 2-D");
  const int64_t M = a.size(0);
  int64_t E, K, N;
  if (mode == 0 || mode == 1) {
    TORCH_CHECK(b.dim() == 3, "grouped_gemm: W must be [E, K, N]");
    E = b.size(0); K = b.size(1); N = b.size(2);
    check_bf16(c, "c");
    TORCH_CHECK(c.dim() == 2 && c.size(0) == M, "grouped_gemm: output rows");
    if (mode == 0) {
      TORCH_CHECK(a.size(1) == K && c.size(1) == N, "grouped_gemm fwd: x [M, K], y [M, N]");
    } else {
      TORCH_CHECK(a.size(1) == N && c.size(1) == K, "grouped_gemm dgrad: dy [M, N], dx [M, K]");
    }
  } else if (mode == 2) {
    TORCH_CHECK(b.dim() == 2 && b.size(0) == M, "grouped_gemm wgrad: dy [M, N]");
    TORCH_CHECK(c.scalar_type() == at::kFloat && c.dim() == 3, "grouped_gemm wgrad: dW fp32 [E, K, N]");
    E = c.size(0); K = a.size(1); N = b.size(1);
    TORCH_CHECK(c.size(1) == K && c.size(2) == N, "grouped_gemm wgrad: dW shape");
  } else {
    TORCH_CHECK(false, "grouped_gemm: mode must be 0, 1 or 2");
  }
  TORCH_CHECK(offs.size(0) == E + 1, "grouped_gemm: offs must have E + 1 entries");
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0, "grouped_gemm: K and N must be multiples of 8");
  TORCH_CHECK(M < (1LL << 31) && K < (1LL << 31) && N < (1LL << 31) && E < 65536, "grouped_gemm: sizes too large");
  static const bool wg_kernel = [] {
    const char* e = getenv("NXD_GG_WGRAD");
    return !(e && e[0] == '0');
  }();
  if (mode == 2 && wg_kernel) {
    // expert weight gradients on the token-major wgrad kernel (csrc/wgrad_gemm.hip, grouped mode):
    // dW[e] [K, N] += x_e^T dy_e
    if (!accumulate) c.zero_();
    if (M == 0) return;
    check_rc(nxd::wgrad_gemm_grouped_launch(a.data_ptr(), K, b.data_ptr(), N, c.data_ptr<float>(), N, K * N,
                                            offs.data_ptr<int32_t>(), (int)E, (int)M, (int)K, (int)N, cur_stream()),
             "grouped_gemm wgrad");
    return;
  }
  static const bool row_kernel = [] {
    const char* e = getenv("NXD_GG_ROW");
    return !(e && e[0] == '0');
  }();
  if ((mode == 0 || mode == 1) && row_kernel) {
    // 256 x 256 tiles (csrc/grouped_rowgemm.hip); -1 = shape it does not take (reduction % 32)
    const int rc = nxd::grouped_rowgemm_launch((int)mode, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                               offs.data_ptr<int32_t>(), (int)E, (int)M, (int)K, (int)N, cur_stream());
    if (rc != -1) {
      check_rc(rc, "grouped_gemm (256-tile)");
      return;
    }
  }
  check_rc(nxd::grouped_gemm_launch((int)mode, a.data_ptr(), b.data_ptr(), c.data_ptr(), offs.data_ptr<int32_t>(), (int)E,
                                    (int)M, (int)K, (int)N, accumulate ? 1 : 0, cur_stream()),
           "grouped_gemm");
}

// MoE un-permute + affinity-weighted combine (csrc/moe_combine.hip).  ys [T*k, H] bf16 in
// expert-sorted order, inv int64 [T*k], aff fp32 [T, k] (undefined tensor: unit weights), out [T, H].
void moe_combine_check(const at::Tensor& ys, const at::Tensor& inv, const at::Tensor& aff, int64_t T, int64_t k) {
  check_bf16(ys, "ys");
  check_cuda(inv, "inv");
  TORCH_CHECK(ys.dim() == 2 && ys.is_contiguous() && ys.size(0) == T * k, "moe_combine: ys must be contiguous [T*k, H]");
  TORCH_CHECK(ys.size(1) % 8 == 0 && ys.size(1) < (1LL << 31), "moe_combine: H must be a multiple of 8");
  TORCH_CHECK(inv.scalar_type() == at::kLong && inv.is_contiguous() && inv.numel() == T * k, "moe_combine: inv int64 [T*k]");
  TORCH_CHECK(k >= 1 && k <= 8, "moe_combine: top_k must be in [1, 8]");
  if (aff.defined()) {
    check_cuda(aff, "aff");
    TORCH_CHECK(aff.scalar_type() == at::kFloat && aff.is_contiguous() && aff.numel() == T * k, "moe_combine: aff fp32 [T, k]");
  }
  check_aligned16(ys, "ys");
}

void moe_combine_fwd(at::Tensor ys, at::Tensor inv, c10::optional<at::Tensor> aff, at::Tensor out) {
  const int64_t T = out.size(0), H = ys.size(1), k = T ? ys.size(0) / T : 1;
  const at::Tensor a = aff.has_value() ? *aff : at::Tensor();
  moe_combine_check(ys, inv, a, T, k);
  check_bf16(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && out.size(1) == H, "moe_combine: out must be contiguous [T, H]");
  check_aligned16(out, "out");
  check_rc(nxd::moe_combine_fwd_launch(ys.data_ptr(), inv.data_ptr<int64_t>(), a.defined() ? a.data_ptr<float>() : nullptr,
                                       out.data_ptr(), T, (int)k, (int)H, cur_stream()),
           "moe_combine_fwd");
}

void moe_combine_bwd(at::Tensor dout, at::Tensor ys, at::Tensor inv, at::Tensor aff, at::Tensor dys, at::Tensor daff) {
  const int64_t T = dout.size(0), H = ys.size(1), k = T ? ys.size(0) / T : 1;
  TORCH_CHECK(aff.defined(), "moe_combine_bwd: affinities required");
  moe_combine_check(ys, inv, aff, T, k);
  check_bf16(dout, "dout");
  check_bf16(dys, "dys");
  TORCH_CHECK(dout.dim() == 2 && dout.is_contiguous() && dout.size(1) == H, "moe_combine_bwd: dout [T, H]");
  TORCH_CHECK(dys.sizes() == ys.sizes() && dys.is_contiguous(), "moe_combine_bwd: dys like ys");
  TORCH_CHECK(daff.scalar_type() == at::kFloat && daff.is_contiguous() && daff.numel() == T * k && daff.is_cuda(),
              "moe_combine_bwd: daff fp32 [T, k]");
  check_aligned16(dout, "dout");
  check_aligned16(dys, "dys");
  check_rc(nxd::moe_combine_bwd_launch(dout.data_ptr(), ys.data_ptr(), inv.data_ptr<int64_t>(), aff.data_ptr<float>(),
                                       dys.data_ptr(), daff.data_ptr<float>(), T, (int)k, (int)H, cur_stream()),
           "moe_combine_bwd");
}

// Fused decode GEMV (csrc/decode_fused.hip).  epi: 0 plain, 1 residual add into y (in place),
// 2 SwiGLU on a fused [2N, K] gate/up weight, 3 QKV with RoPE + KV-cache write.  norm_w: RMSNorm
// of x fused as a prologue.  x [M, K], w [Nw, K], y [M, N] bf16, M <= 8.
void dgemv(int64_t epi, at::Tensor x, c10::optional<at::Tensor> norm_w, double eps, at::Tensor w, at::Tensor y,
           int64_t nq, int64_t nkv, int64_t D, c10::optional<at::Tensor> cos_t, c10::optional<at::Tensor> sin_t,
           c10::optional<at::Tensor> pos, int64_t T, c10::optional<at::Tensor> kc, c10::optional<at::Tensor> vc,
           c10::optional<at::Tensor> cache_idx, c10::optional<at::Tensor> xadd, c10::optional<at::Tensor> yadd,
           c10::optional<at::Tensor> xidx, c10::optional<at::Tensor> xcopy) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  // epi 0 with an fp32 y: the unrounded partial sum (row-parallel projection at TP > 1)
  float* yf = nullptr;
  if (epi == 0 && y.scalar_type() == at::kFloat) {
    TORCH_CHECK(y.is_cuda(), "dgemv: y must be a GPU tensor");
    yf = y.data_ptr<float>();
  } else {
    check_bf16(y, "y");
  }
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "dgemv: x [M, K], w [Nw, K], y [M, N]");
  TORCH_CHECK(x.stride(1) == 1 && w.stride(1) == 1 && y.stride(1) == 1, "dgemv: unit inner strides");
  // xidx (QKV only): x is an embedding table [V, K] and input row m is x[xidx[m]]; xcopy [M, K]
  // receives the gathered rows (the residual stream)
  const int64_t M = xidx.has_value() ? xidx->numel() : x.size(0), K = x.size(1), N = y.size(1);
  const int64_t* xi = nullptr;
  void* xc = nullptr;
  if (xidx.has_value()) {
    TORCH_CHECK(epi == 3 && norm_w.has_value(), "dgemv: xidx needs the QKV epilogue with the RMSNorm prologue");
    TORCH_CHECK(xidx->scalar_type() == at::kLong && xidx->is_contiguous() && xidx->is_cuda(), "dgemv: int64 xidx [M]");
    xi = xidx->data_ptr<int64_t>();
    if (xcopy.has_value()) {
      check_bf16(*xcopy, "xcopy");
      TORCH_CHECK(xcopy->is_contiguous() && xcopy->dim() == 2 && xcopy->size(0) == M && xcopy->size(1) == K,
                  "dgemv: xcopy bf16 contiguous [M, K]");
      check_aligned16(*xcopy, "xcopy");
      xc = xcopy->data_ptr();
    }
  }
  TORCH_CHECK(M >= 1 && M <= 8 && y.size(0) == M, "dgemv: 1..8 rows");
  TORCH_CHECK(K % 8 == 0 && x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && w.size(1) == K, "dgemv: K / strides");
  check_aligned16(x, "x");
  check_aligned16(w, "w");
  TORCH_CHECK(w.size(0) == (epi == 2 ? 2 * N : N), "dgemv: weight rows vs output columns");
  const void* nw = nullptr;
  if (norm_w.has_value()) {
    check_bf16(*norm_w, "norm_w");
    TORCH_CHECK(norm_w->is_contiguous() && norm_w->numel() == K, "dgemv: norm weight [K]");
    check_aligned16(*norm_w, "norm_w");
    TORCH_CHECK(M * K * 2 <= 65536, "dgemv: fused norm needs M * K <= 32768");
    nw = norm_w->data_ptr();
  }
  const float *cp = nullptr, *sp = nullptr;
  const int64_t* pp = nullptr;
  void *kp = nullptr, *vp = nullptr;
  const int* ci = nullptr;
  int64_t c_sb = 0, c_sh = 0, c_sl = 0;
  int Lmax = 0, max_pos = 0;
  if (epi == 3) {
    TORCH_CHECK(cos_t.has_value() && sin_t.has_value() && pos.has_value() && kc.has_value() && vc.has_value(),
                "dgemv rope_kv: cos, sin, pos, k/v cache required");
    TORCH_CHECK(D % 2 == 0 && D >= 2 && nq >= 1 && nkv >= 1 && N == (nq + 2 * nkv) * D, "dgemv rope_kv: head layout");
    TORCH_CHECK(cos_t->scalar_type() == at::kFloat && sin_t->scalar_type() == at::kFloat && cos_t->is_contiguous() &&
                    sin_t->is_contiguous() && cos_t->dim() == 2 && cos_t->size(1) == D / 2 && sin_t->sizes() == cos_t->sizes(),
                "dgemv rope_kv: fp32 cos/sin tables [P, D/2]");
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->is_contiguous() && pos->numel() == M, "dgemv rope_kv: int64 pos [M]");
    check_bf16(*kc, "k_cache");
    check_bf16(*vc, "v_cache");
    TORCH_CHECK(kc->dim() == 4 && kc->sizes() == vc->sizes() && kc->strides() == vc->strides() && kc->stride(3) == 1 &&
                    kc->size(1) == nkv && kc->size(3) == D,
                "dgemv rope_kv: caches [B, Hkv, Lmax, D]");
    TORCH_CHECK(T >= 1 && M % T == 0, "dgemv rope_kv: rows must be whole sequences of T tokens");
    if (cache_idx.has_value()) {
      TORCH_CHECK(cache_idx->scalar_type() == at::kInt && cache_idx->is_contiguous() && cache_idx->numel() == M / T,
                  "dgemv rope_kv: int32 cache_idx [B]");
      ci = cache_idx->data_ptr<int>();
    } else {
      TORCH_CHECK(kc->size(0) >= M / T, "dgemv rope_kv: cache batch");
    }
    cp = cos_t->data_ptr<float>();
    sp = sin_t->data_ptr<float>();
    pp = pos->data_ptr<int64_t>();
    kp = kc->data_ptr();
    vp = vc->data_ptr();
    c_sb = kc->stride(0);
    c_sh = kc->stride(1);
    c_sl = kc->stride(2);
    Lmax = kc->size(2);
    max_pos = cos_t->size(0);
  } else {
    TORCH_CHECK(epi >= 0 && epi <= 2, "dgemv: epi must be 0..3");
  }
  // fp32 pending-residual side inputs (fused attention + o_proj): xadd [M, K] for the NORM prologue,
  // yadd [M, N] for the RESID epilogue (zeroed by it)
  const float* xa = nullptr;
  float* ya = nullptr;
  if (xadd.has_value()) {
    TORCH_CHECK(nw != nullptr, "dgemv: xadd needs the fused RMSNorm prologue");
    TORCH_CHECK(xadd->scalar_type() == at::kFloat && xadd->is_contiguous() && xadd->dim() == 2 && xadd->size(0) >= M &&
                    xadd->size(1) == K && xadd->is_cuda(),
                "dgemv: xadd fp32 contiguous [>=M, K]");
    xa = xadd->data_ptr<float>();
  }
  if (yadd.has_value()) {
    TORCH_CHECK(epi == 1, "dgemv: yadd is the RESID epilogue's side input");
    TORCH_CHECK(yadd->scalar_type() == at::kFloat && yadd->is_contiguous() && yadd->dim() == 2 && yadd->size(0) >= M &&
                    yadd->size(1) == N && yadd->is_cuda(),
                "dgemv: yadd fp32 contiguous [>=M, N]");
    ya = yadd->data_ptr<float>();
  }
  check_rc(nxd::dgemv_launch((int)epi, x.data_ptr(), x.stride(0), nw, (float)eps, w.data_ptr(), w.stride(0), y.data_ptr(),
                             y.stride(0), (int)M, (int)N, (int)K, (int)nq, (int)nkv, (int)D, cp, sp, pp, (int)T, kp, vp,
                             c_sb, c_sh, c_sl, ci, Lmax, max_pos, xa, ya, cur_stream(), xi, x.size(0), xc, yf),
           "dgemv");
}

}  // namespace

void register_gemm(pybind11::module& m);  // gemm.cpp
void register_dataloader(pybind11::module& m);  // dataloader.cpp
void register_comm(pybind11::module& m);  // comm.cpp

// SIGABRT: print the native stack (backtrace_symbols_fd writes straight to fd 2, no allocation) and
// chain to the handler installed before us (Python's faulthandler prints the Python stacks, then the
// default action dumps core).  An abort raised inside a C++ destructor during garbage collection --
// an error from an earlier asynchronous GPU failure surfacing in a free -- otherwise shows only
// "Fatal Python error: Aborted ... Garbage-collecting" (profiles/r4_decode_attn_trace_abort.txt).
// NXD_ABORT_BACKTRACE=0 leaves SIGABRT alone.
static struct sigaction g_prev_abrt;
static void abort_backtrace(int sig) {
  static const char hdr[] = "[nxd] SIGABRT: native backtrace (neuronx_distributed_llama3_2_amd _C)\n";
  (void)!write(2, hdr, sizeof(hdr) - 1);
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  sigaction(SIGABRT, &g_prev_abrt, nullptr);
  raise(sig);
}
static void install_abort_backtrace() {
  const char* e = std::getenv("NXD_ABORT_BACKTRACE");
  if (e && e[0] == '0') return;
  struct sigaction sa {};
  sa.sa_handler = abort_backtrace;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESETHAND;
  sigaction(SIGABRT, &sa, &g_prev_abrt);
}

PYBIND11_MODULE(_C, m) {
  install_abort_backtrace();
  m.def("decode_attn_trace", [](c10::optional<at::Tensor> t) {
    if (!t.has_value()) {
      nxd::decode_attn_set_trace(nullptr);
      return;
    }
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->is_contiguous(), "trace: int64 GPU tensor");
    nxd::decode_attn_set_trace(reinterpret_cast<uint64_t*>(t->data_ptr<int64_t>()));
  }, "arm (tensor) / disarm (None) the decode attention phase trace");
  register_gemm(m);
  register_dataloader(m);
  register_comm(m);
  m.def("gemv", &gemv);
  m.def("dequant_int8", &dequant_int8);
  m.def("expert_gemv", &expert_gemv);
  m.def("grouped_gemm", &grouped_gemm);
  m.def("wgrad_gemm", &wgrad_gemm);
  m.def("dense_gemm", &dense_gemm, py::arg("layout"), py::arg("epi"), py::arg("a"), py::arg("b"), py::arg("c"),
        py::arg("splits") = 0);
  m.def("dense_gemm_set_pipe", [](int64_t v) { nxd::dense_gemm_set_pipe((int)v); });
  m.def("dense_gemm_splits", [](int64_t M, int64_t N, int64_t K) {
    return nxd::dense_gemm_choose_splits((int)M, (int)N, (int)K);
  });
  // diagnostics: copy kernel on exactly `blocks` workgroups (CU-interference measurements)
  // A HIP stream whose kernels may only use the CUs whose bits are NOT listed in `exclude`
  // (hipExtStreamCreateWithCUMask; the CUs left out stay free for the collectives' kernels, which
  // then never wait for a compute workgroup to retire).  Returns the raw stream handle for
  // torch.cuda.ExternalStream; the stream lives for the process.
  m.def("cu_masked_stream", [](std::vector<int64_t> exclude) {
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    TORCH_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0,
                "cu_masked_stream: CU count");
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
    for (int64_t c : exclude) {
      TORCH_CHECK(c >= 0 && c < ncu, "cu_masked_stream: CU index out of range");
      mask[c / 32] &= ~(1u << (c % 32));
    }
    hipStream_t st = nullptr;
    check_rc(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) == hipSuccess ? 0 : -1,
             "hipExtStreamCreateWithCUMask");
    return (int64_t)(uintptr_t)st;
  });
  m.def("cu_stream", [](at::Tensor src, at::Tensor dst, int64_t bytes_per_block, int64_t blocks, int64_t ticks) {
    check_cuda(src, "src");
    check_cuda(dst, "dst");
    TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && src.nbytes() == dst.nbytes(), "cu_stream: buffers");
    TORCH_CHECK(bytes_per_block * blocks <= (int64_t)src.nbytes(), "cu_stream: buffers too small");
    check_rc(nxd::cu_stream_launch(src.data_ptr(), dst.data_ptr(), bytes_per_block, (int)blocks, ticks, cur_stream()),
             "cu_stream");
  });
  m.def("wgrad_gemm_set_ablate", [](int64_t v) { nxd::wgrad_gemm_set_ablate((int)v); });
  // ping-pong (staggered wave-group) main loops of the two hand-written GEMMs, for in-process A/B
  m.def("grouped_rowgemm_set_pp", [](int64_t v) { nxd::grouped_rowgemm_set_pp((int)v); });
  m.def("wgrad_gemm_set_pp", [](int64_t v) { nxd::wgrad_gemm_set_pp((int)v); });
  m.def("wgrad_gemm_splits", [](int64_t T, int64_t M, int64_t N) { return nxd::wgrad_gemm_choose_splits((int)T, (int)M, (int)N); });
  m.def("moe_combine_fwd", &moe_combine_fwd);
  m.def("moe_combine_bwd", &moe_combine_bwd);
  m.def("dgemv", &dgemv, py::arg("epi"), py::arg("x"), py::arg("norm_w"), py::arg("eps"), py::arg("w"), py::arg("y"),
        py::arg("nq"), py::arg("nkv"), py::arg("D"), py::arg("cos_t"), py::arg("sin_t"), py::arg("pos"), py::arg("T"),
        py::arg("kc"), py::arg("vc"), py::arg("cache_idx"), py::arg("xadd") = py::none(), py::arg("yadd") = py::none(),
        py::arg("xidx") = py::none(), py::arg("xcopy") = py::none());
  // decode A/B knobs: 0 = GLU row pairs per wave, 1 = GEMV k-slices (0 auto), 2 = MFMA decode attention on/off,
  // 3 = GEMV early epilogue / prologue reads on/off, 5 = bs = 1 GEMV forced occupancy (0 natural | 7 | 8 waves / SIMD)
  m.def("decode_set_knob", [](int which, int value) {
    if (which == 2) nxd::decode_attn_set_v2(value);
    else if (which == 3) nxd::dgemv_set_knob(2, value);
    else nxd::dgemv_set_knob(which, value);
  });
  m.doc() = "CDNA4 (gfx950) kernels of neuronx_distributed_llama3_2_amd";
  m.def("flash_attn_fwd", &flash_attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("lse"),
        py::arg("scale"), py::arg("causal"), py::arg("causal_offset"), py::arg("dropout_p") = 0.0, py::arg("seed") = 0,
        py::arg("head_offset") = 0);
  m.def("flash_attn_bwd", &flash_attn_bwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("dout"),
        py::arg("lse"), py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("scale"), py::arg("causal"),
        py::arg("causal_offset"), py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("head_offset") = 0);
  // A/B knobs of the backward: 0 = ablation flags, 1 = chunk override (0 = auto)
  m.def("flash_attn_set_knob", [](int which, int value) { nxd::flash_attn_bwd_set_knob(which, value); });
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("transpose_set_variant", [](bool tr) { nxd::transpose_set_variant(tr ? 1 : 0); });
  m.def("rmsnorm_set_rows_path", [](bool on) { nxd::rmsnorm_set_rows_path(on ? 1 : 0); });
  m.def("rope_inplace", &rope_inplace);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("transpose_bf16", &transpose_bf16);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("swiglu_bwd_dual", &swiglu_bwd_dual);
  m.def("swiglu_fwd_dual", &swiglu_fwd_dual);
  m.def("xent_stats", &xent_stats);
  m.def("xent_bwd", &xent_bwd);
  m.def("flat_reduce", &flat_reduce);
  m.def("adamw_flat", &adamw_flat);
  m.def("clip_coef", &clip_coef);
  m.def("scale_flat", &scale_flat);
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("decode_attn", &decode_attn);
  m.def("decode_attn_oproj", &decode_attn_oproj);
  m.def("decode_attn_sync_error", [](bool reset) { return nxd::decode_attn_sync_error(reset); }, py::arg("reset") = false);
  m.def("decode_attn_set_sync", [](int64_t v) { nxd::decode_attn_set_sync((int)v); });
  m.def("decode_attn_set_oproj_maxl", [](int64_t v) { nxd::decode_attn_set_oproj_maxl((int)v); });
  m.def("decode_attn_prefetch", &decode_attn_prefetch);
  m.def("kv_cache_write", &kv_cache_write);
  m.def("argmax_rows", &argmax_rows);
  m.def("greedy_advance", &greedy_advance);
  m.def("topk_sample", &topk_sample);
  m.attr("ARCH") = "gfx950";
}
