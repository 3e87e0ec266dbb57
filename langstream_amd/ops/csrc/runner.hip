// Native model step executors: the whole Llama / BERT forward -- and for the LLM engine
// the whole step (input upload, token feedback, forward, sampling, result download) --
// issued from C++ with the GIL released.
//
// Why: in the streaming runtime the GPU engines share the Python GIL with agent
// threads.  Every torch op called from Python releases and re-acquires the GIL, and
// with busy agent threads each re-acquire waits up to the interpreter switch interval
// -- measured 1.6-1.8 s of host time per mixed prefill step on MI355X with a
// Python-driven forward, and still ~30 ms per decode step for the ~40 small ops of
// input upload + sampling (cProfile, engine thread).  Here a step is ONE call.
//
// LlamaRunner: packed weights per layer (qkv / o / gate_up / down, two norms), paged
//   KV caches, RoPE table; forward() handles decode rows, prefill rows or both in one
//   step; optional tensor parallelism through a c10d ProcessGroup (RCCL all-reduce
//   after o_proj and down_proj, all-gather of the vocab-sharded logits).
// BertRunner: packed-varlen encoder + pooling.
// StepExecutor: owns a ring of pinned host "arenas" (fixed layout, filled by the
//   Python scheduler through numpy views), one device arena, the token feedback buffer
//   and per-bucket HIP graphs.  launch(): one H2D copy of the arena, (TP: one RCCL
//   broadcast of it to the other ranks), on-device feedback of the previous step's
//   sampled tokens into this step's decode rows, forward, logit deltas, sampling, one
//   D2H copy into a pinned result slot, event.  Decode-only steps replay a captured
//   graph of gather+forward+deltas+sample; the counts those kernels need are read
//   from the device copy of the arena header, so one graph serves every step of its
//   bucket.  Non-zero TP ranks run worker_loop() entirely in C++.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/HIPGraph.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <map>
#include <mutex>
#include <thread>
#include <memory>
#include <string>
#include <vector>

namespace py = pybind11;

// Prefill routing of the plain projections (qkv / o / down): hipBLASLt's kernel choice is
// erratic across M -- 1.55 PFLOP/s at M = 8192 or 16384, 0.9-1.1 at some M in between --
// while gemm_pp_kernel holds 1.25-1.43 (profiles/pgemm_m2_r3c.log).  A per-(N, K) table of
// 256-row M buckets, measured on the target by tools/pgemm_route_tune.py and loaded at
// import (ops/pgemm_route_gfx950.csv), says where gemm_prefill is the faster one.
namespace pgemm_route {
std::mutex mu;
std::map<std::pair<int64_t, int64_t>, std::vector<uint8_t>> table;   // (N, K) -> use_pp per M/256
void set(int64_t N, int64_t K, std::vector<int64_t> use_pp) {
  std::lock_guard<std::mutex> lk(mu);
  std::vector<uint8_t> v(use_pp.begin(), use_pp.end());
  table[{N, K}] = std::move(v);
}
bool use_pp(int64_t T, int64_t N, int64_t K) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = table.find({N, K});
  if (it == table.end()) return false;
  const int64_t b = (T + 128) / 256;
  return b >= 0 && b < (int64_t)it->second.size() && it->second[b] != 0;
}
}  // namespace pgemm_route

void rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, double eps);
void fused_add_rmsnorm(at::Tensor x, at::Tensor residual, at::Tensor w, double eps);
void layernorm(at::Tensor out, at::Tensor x, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> residual,
               at::Tensor g, at::Tensor b, double eps);
void embed_layernorm(at::Tensor out, at::Tensor ids, at::Tensor pos_ids, c10::optional<at::Tensor> type_ids,
                     at::Tensor wte, at::Tensor wpe, at::Tensor wtt, at::Tensor g, at::Tensor b, double eps);
void silu_and_mul(at::Tensor out, at::Tensor x);
void bias_gelu(at::Tensor x, c10::optional<at::Tensor> bias);
void rope_and_cache(at::Tensor qkv, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots, at::Tensor k_cache,
                    at::Tensor v_cache, int64_t Hq, int64_t Hkv, bool apply_rope);
void paged_decode_attention(at::Tensor out, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                            at::Tensor block_tables, at::Tensor ctx_lens, double scale, int64_t nsplit,
                            int64_t blocks_per_split, at::Tensor workspace);
void paged_decode_attention_rope(at::Tensor out, at::Tensor qkv, at::Tensor pos, at::Tensor cos_sin,
                                 at::Tensor slots, at::Tensor k_cache, at::Tensor v_cache, at::Tensor block_tables,
                                 at::Tensor ctx_lens, double scale, int64_t nsplit, int64_t min_bps,
                                 at::Tensor workspace);
void paged_prefill_attention(at::Tensor out, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                             at::Tensor block_tables, at::Tensor q_start, at::Tensor q_len, at::Tensor ctx_len,
                             at::Tensor tiles, int64_t Hq, double scale);
void varlen_encoder_attention(at::Tensor out, at::Tensor qkv, at::Tensor q_start, at::Tensor q_len,
                              at::Tensor tiles, int64_t Hq, int64_t Hkv, double scale);
void pool_embeddings(at::Tensor out, at::Tensor x, at::Tensor start, at::Tensor len, int64_t mode, bool normalize);
void sample_tokens(at::Tensor logits, at::Tensor temperature, at::Tensor top_k, at::Tensor top_p, at::Tensor seeds,
                   at::Tensor steps, at::Tensor out_tok, at::Tensor out_lp, at::Tensor top_ids, at::Tensor top_lps,
                   int64_t n_top);
void tp_sample_stats(at::Tensor logits, int64_t vstart, at::Tensor stats);
void tp_sample_hist(at::Tensor logits, int64_t vtot, at::Tensor temperature, at::Tensor top_k, at::Tensor top_p,
                    at::Tensor stats_all, int64_t world, at::Tensor hist);
void tp_sample_pick(at::Tensor logits, int64_t vstart, int64_t vtot, at::Tensor temperature, at::Tensor top_k,
                    at::Tensor top_p, at::Tensor seeds, at::Tensor steps, at::Tensor stats_all, int64_t world,
                    at::Tensor hist_all, int64_t n_top, at::Tensor cand);
void tp_sample_final(at::Tensor stats_all, at::Tensor cand_all, int64_t world, int64_t rows, at::Tensor temperature,
                     int64_t n_top, at::Tensor out_tok, at::Tensor out_lp, at::Tensor top_ids, at::Tensor top_lps);

class OneShotAllReduce;
std::shared_ptr<OneShotAllReduce> make_oneshot_allreduce(c10::intrusive_ptr<::c10d::ProcessGroup> pg,
                                                         int64_t max_elems);
void oneshot_allreduce_run(const std::shared_ptr<OneShotAllReduce>& ar, at::Tensor t);
void oneshot_allreduce_i64(const std::shared_ptr<OneShotAllReduce>& ar, at::Tensor t);
void oneshot_allgather32(const std::shared_ptr<OneShotAllReduce>& ar, const at::Tensor& in, at::Tensor out);
int64_t oneshot_capacity_bytes(const std::shared_ptr<OneShotAllReduce>& ar);
bool oneshot_route_sum_i64(const std::shared_ptr<OneShotAllReduce>& ar,
                           const c10::intrusive_ptr<::c10d::ProcessGroup>& pg, at::Tensor t);
bool oneshot_route_gather32(const std::shared_ptr<OneShotAllReduce>& ar,
                            const c10::intrusive_ptr<::c10d::ProcessGroup>& pg, const at::Tensor& src,
                            const at::Tensor& dst);

void skinny_gemm(at::Tensor out, at::Tensor x, at::Tensor w);
void gemm_fused(at::Tensor out, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> bias, bool gelu,
                c10::optional<at::Tensor> residual, c10::optional<at::Tensor> ln_stats_in, int64_t ln_width,
                c10::optional<at::Tensor> c1, c10::optional<at::Tensor> c2, c10::optional<at::Tensor> res_g,
                c10::optional<at::Tensor> res_b, double eps, c10::optional<at::Tensor> stats_out);
void gemv(at::Tensor out, at::Tensor x, at::Tensor w);
void gemv_silu(at::Tensor out, at::Tensor x, at::Tensor w);
bool gemv_supported(const at::Tensor& w, bool silu);
void gemv_norm(at::Tensor out, at::Tensor o, at::Tensor res, at::Tensor res_out, at::Tensor norm_w, double eps,
               at::Tensor w);
void gemv_qkv(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots,
              at::Tensor k_cache, at::Tensor v_cache, int64_t Hq, int64_t Hkv, bool apply_rope,
              c10::optional<at::Tensor> o, c10::optional<at::Tensor> res, c10::optional<at::Tensor> res_out,
              c10::optional<at::Tensor> norm_w, double eps);
void gemv_silu_norm(at::Tensor out, at::Tensor o, at::Tensor res, at::Tensor res_out, at::Tensor norm_w, double eps,
                    at::Tensor w);
void skinny_gemm_add_rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor residual, at::Tensor norm_w,
                             double eps);
void gemm_prefill(at::Tensor out, at::Tensor x, at::Tensor w, bool silu, int64_t variant);
bool gemm_prefill_supported(const at::Tensor& w, bool silu);
void gemm_prefill_f32(at::Tensor out, at::Tensor x, at::Tensor w);
bool gemm_prefill_f32_supported(const at::Tensor& w);
bool decode_gemm_supported(const at::Tensor& w, bool silu);
int64_t decode_gemm_workspace(int64_t M, int64_t N, int64_t K, bool silu);
void decode_gemm_qkv_rope(at::Tensor qkv, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor pos,
                          at::Tensor cos_sin, at::Tensor slots, at::Tensor k_cache, at::Tensor v_cache, int64_t Hq,
                          int64_t Hkv);
bool decode_gemm_f32_supported(const at::Tensor& w, int64_t M);
void decode_gemm_f32(at::Tensor out, at::Tensor x, at::Tensor w, int64_t bn_force);
void decode_gemm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor workspace, c10::optional<at::Tensor> residual,
                 c10::optional<at::Tensor> norm_w, double eps, int64_t bn_force, int64_t splits_force);
void decode_gemm_silu(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor tickets,
                      at::Tensor err, int64_t splits);
const int* oneshot_allreduce_err(const std::shared_ptr<OneShotAllReduce>& ar);
int64_t decode_gemm_cmb_splits(int64_t N, int64_t K);
void decode_gemm_res(at::Tensor y_out, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor counters,
                     at::Tensor residual, at::Tensor norm_g, at::Tensor sumsq_out, at::Tensor err);
void decode_gemm_qkv_cmb(at::Tensor qkv, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor counters,
                         at::Tensor sumsq_in, double eps, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots,
                         at::Tensor k_cache, at::Tensor v_cache, int64_t Hq, int64_t Hkv, at::Tensor err);
void decode_gemm_silu_r(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor sumsq_in, double eps);
void rms_prep(at::Tensor y, at::Tensor sumsq, at::Tensor h, at::Tensor g);
void rows_rms_scale(at::Tensor out, at::Tensor y, at::Tensor sumsq, double eps);

#define HIP_OK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));          \
  } while (0)

namespace {

// Prefix KV reuse (engine/llm_engine.py PrefixCache): copy whole KV blocks (src -> dst
// pairs) in every layer's K and V cache.  grid = (pairs, 2 x layers); tab[t] is the base
// of cache tensor t ([NB, ...], block_bytes per block).  Pairs outside [0, NB) are skipped.
__global__ void __launch_bounds__(256) kv_block_copy_kernel(const int64_t* __restrict__ tab,
                                                             const int32_t* __restrict__ pairs, int64_t nb,
                                                             int64_t block_bytes) {
  const int32_t s = pairs[2 * blockIdx.x], d = pairs[2 * blockIdx.x + 1];
  if (s < 0 || d < 0 || s >= nb || d >= nb || s == d) return;
  char* base = reinterpret_cast<char*>(tab[blockIdx.y]);
  const uint4* src = reinterpret_cast<const uint4*>(base + (int64_t)s * block_bytes);
  uint4* dst = reinterpret_cast<uint4*>(base + (int64_t)d * block_bytes);
  for (int64_t i = threadIdx.x; i < block_bytes / 16; i += 256) dst[i] = src[i];
}

// ---------------------------------------------------------------------------- Llama
class LlamaRunner {
 public:
  LlamaRunner(at::Tensor embed, std::vector<at::Tensor> qkv_w, std::vector<at::Tensor> o_w,
              std::vector<at::Tensor> gate_up_w, std::vector<at::Tensor> down_w, std::vector<at::Tensor> in_norm,
              std::vector<at::Tensor> post_norm, at::Tensor final_norm, at::Tensor lm_head,
              std::vector<at::Tensor> k_caches, std::vector<at::Tensor> v_caches, at::Tensor cos_sin, int64_t hq,
              int64_t hkv, int64_t head_dim, double eps, double scale, int64_t vocab_size, int64_t vocab_start,
              py::object process_group)
      : embed_(embed), qkv_w_(qkv_w), o_w_(o_w), gate_up_w_(gate_up_w), down_w_(down_w), in_norm_(in_norm),
        post_norm_(post_norm), final_norm_(final_norm), lm_head_(lm_head), kc_(k_caches), vc_(v_caches),
        cos_sin_(cos_sin), hq_(hq), hkv_(hkv), d_(head_dim), eps_(eps), scale_(scale), vocab_(vocab_size),
        vocab_start_(vocab_start) {
    const size_t L = qkv_w_.size();
    TORCH_CHECK(L > 0 && o_w_.size() == L && gate_up_w_.size() == L && down_w_.size() == L &&
                in_norm_.size() == L && post_norm_.size() == L && kc_.size() == L && vc_.size() == L,
                "inconsistent layer lists");
    if (!process_group.is_none()) pg_ = py::cast<c10::intrusive_ptr<::c10d::ProcessGroup>>(process_group);
    // LS_ONESHOT_AR=1: decode-sized all-reduces (<= LS_ONESHOT_AR_MAX elements, default
    // 256 x 8192) through the one-shot IPC kernel (allreduce.hip) instead of RCCL
    if (pg_ && getenv("LS_ONESHOT_AR") && atoi(getenv("LS_ONESHOT_AR")) != 0) {
      const int64_t mx = getenv("LS_ONESHOT_AR_MAX") ? atoll(getenv("LS_ONESHOT_AR_MAX")) : 256 * 8192;
      oneshot_ = make_oneshot_allreduce(pg_, mx);
      oneshot_max_ = mx;
    }
    // device status words that must stay 0 (see status_ptrs) and the decode-GEMM
    // workspace: f32 split-K partials / the gate_up half exchange, sized once for the
    // largest decode batch so graph captures never allocate
    auto dev = embed_.options();
    status_ = at::zeros({4}, dev.dtype(at::kInt));
    if (dgemm_enabled()) {
      int64_t wsz = 1, fmax = 0;
      for (size_t l = 0; l < L; ++l) {
        const at::Tensor* ws[3] = {&qkv_w_[l], &o_w_[l], &down_w_[l]};
        for (auto* w : ws)
          if (decode_gemm_supported(*w, false))
            wsz = std::max(wsz, decode_gemm_workspace(kDgemmMaxM, w->size(0), w->size(1), false));
        if (decode_gemm_supported(gate_up_w_[l], true)) {
          wsz = std::max(wsz, decode_gemm_workspace(kDgemmMaxM, gate_up_w_[l].size(0), gate_up_w_[l].size(1), true));
          fmax = std::max(fmax, gate_up_w_[l].size(0) / 2);
        }
      }
      // the norm-deferred layer (forward_dgemm): combine-path splits must exist for qkv /
      // o / down, the head dim must be 128 (one head per 128-column tile)
      bool fz = !pg_ && head_dim == 128 && fused_env();
      const int64_t H = embed_.size(1);
      for (size_t l = 0; l < L && fz; ++l) {
        const at::Tensor* ws[3] = {&qkv_w_[l], &o_w_[l], &down_w_[l]};
        for (auto* w : ws) {
          const int64_t S = decode_gemm_cmb_splits(w->size(0), w->size(1));
          fz = fz && S > 0 && decode_gemm_supported(*w, false);
          if (S > 0) wsz = std::max(wsz, S * kDgemmMaxM * w->size(0) * 4);
        }
        fz = fz && decode_gemm_supported(gate_up_w_[l], true) && o_w_[l].size(0) == H && down_w_[l].size(0) == H;
      }
      dg_ws_ = at::empty({(wsz + 3) / 4}, dev.dtype(at::kFloat));
      dg_tickets_ = at::zeros({std::max<int64_t>(2, 2 * (fmax / 128))}, dev.dtype(at::kInt));
      if (fz) {
        auto bf = dev.dtype(at::kBFloat16);
        y_in_ = at::zeros({kDgemmMaxM, H}, bf);
        y_post_ = at::zeros({kDgemmMaxM, H}, bf);
        ss_in_ = at::zeros({kDgemmMaxM, H / 128}, dev.dtype(at::kFloat));
        ss_post_ = at::zeros({kDgemmMaxM, H / 128}, dev.dtype(at::kFloat));
        ss0_ = at::zeros({kDgemmMaxM, 1}, dev.dtype(at::kFloat));
        const int64_t maxt = std::max<int64_t>(qkv_w_[0].size(0), H) / 128;
        cnt_qkv_ = at::zeros({maxt}, dev.dtype(at::kLong));
        cnt_o_ = at::zeros({maxt}, dev.dtype(at::kLong));
        cnt_down_ = at::zeros({maxt}, dev.dtype(at::kLong));
      }
    }
  }

  // Copy `n` KV blocks (int32 (src, dst) pairs on the device) in every layer's K and V
  // cache, on the current stream: the prefix-cache copies a step carries ahead of its
  // forward (StepExecutor::run).
  void copy_kv_blocks(const int32_t* pairs, int64_t n) {
    if (n <= 0) return;
    if (!kv_tab_.defined()) {
      std::vector<int64_t> ptrs;
      for (size_t l = 0; l < kc_.size(); ++l) {
        TORCH_CHECK(kc_[l].is_contiguous() && vc_[l].is_contiguous() && kc_[l].size(0) == kc_[0].size(0) &&
                    vc_[l].size(0) == kc_[0].size(0) && kc_[l][0].numel() == vc_[l][0].numel(),
                    "KV caches: contiguous, one block count, K and V blocks of one size");
        ptrs.push_back(reinterpret_cast<int64_t>(kc_[l].data_ptr()));
        ptrs.push_back(reinterpret_cast<int64_t>(vc_[l].data_ptr()));
      }
      kv_tab_ = at::tensor(ptrs, at::TensorOptions().dtype(at::kLong)).to(embed_.device());
      kv_block_bytes_ = kc_[0][0].numel() * kc_[0].element_size();
      TORCH_CHECK(kv_block_bytes_ % 16 == 0);
    }
    kv_block_copy_kernel<<<dim3((unsigned)n, (unsigned)kv_tab_.numel()), 256, 0,
                           at::hip::getCurrentHIPStream()>>>(kv_tab_.data_ptr<int64_t>(), pairs, kc_[0].size(0),
                                                             kv_block_bytes_);
  }

  // Device int32 words that are 0 unless a step's results are invalid: [0] the gate_up
  // half-exchange of gemm_decode.hip timed out; the one-shot all-reduce's sticky timeout
  // word.  The step executor copies them next to every step's results and fails the step.
  std::vector<const int*> status_ptrs() const {
    // [0] gate_up half exchange, [1] combine rendezvous (forward_dgemm), then the
    // one-shot all-reduce's word
    std::vector<const int*> v{status_.data_ptr<int>(), status_.data_ptr<int>() + 1};
    if (oneshot_) v.push_back(oneshot_allreduce_err(oneshot_));
    return v;
  }

  // LM head with f32 OUTPUT straight from the GEMM (bf16 x bf16 -> f32): a bf16 logit
  // tensor quantises logits to 2^-7 relative steps (0.125 at |logit| ~ 20), which ties
  // near-equal tokens and coarsens the log-probs FLARE and `logprobs` consume.  Every row
  // count runs on the 256-row decode GEMM's f32 epilogue (gemm_decode.hip), in blocks of
  // 256 rows; only shapes it cannot take (vocab % 128, hidden % 64) fall back to the
  // library GEMM (LS_DGEMM_HEAD=0 forces the library).
  at::Tensor lm_head(const at::Tensor& x) {
    static const bool dg_head = [] {
      const char* e = getenv("LS_DGEMM_HEAD");
      return e == nullptr || e[0] != '0';
    }();
    const int64_t R = x.size(0);
    // LS_HEAD_PP_MIN_T = n > 0: batches of n+ rows on the ping-pong prefill kernel with an
    // f32 epilogue -- faster alone (261 vs 279 us at M = 256, 247 vs 268 at 192:
    // profiles/r5/head_pp_r5ag.log) but slower end to end: the RAG bench's closed-loop rate
    // was 1.8 % lower with it in all three rounds of a same-box A/B (ab_head_r5ak.log; it
    // streams the 1 GB head through the caches, where the decode GEMM's loads are
    // non-temporal).  Off by default.
    static const int64_t pp_min = [] {
      const char* e = getenv("LS_HEAD_PP_MIN_T");
      return e ? atoll(e) : 0;
    }();
    if (pp_min > 0 && R >= pp_min && gemm_prefill_f32_supported(lm_head_) &&
        (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && x.stride(1) == 1 && x.stride(0) % 8 == 0) {
      at::Tensor out = at::empty({R, lm_head_.size(0)}, x.options().dtype(at::kFloat));
      gemm_prefill_f32(out, x, lm_head_);
      return out;
    }
    if (dg_head && dgemm_enabled() && R >= 1 && decode_gemm_f32_supported(lm_head_, std::min<int64_t>(R, kDgemmMaxM))) {
      at::Tensor xc = x.contiguous();
      at::Tensor out = at::empty({R, lm_head_.size(0)}, x.options().dtype(at::kFloat));
      for (int64_t r0 = 0; r0 < R; r0 += kDgemmMaxM) {
        const int64_t n = std::min<int64_t>(kDgemmMaxM, R - r0);
        decode_gemm_f32(out.narrow(0, r0, n), xc.narrow(0, r0, n), lm_head_, 0);
      }
      return out;
    }
    if (f32_head_) {
      try {
        return at::mm(x, lm_head_.t(), at::kFloat);
      } catch (const c10::Error&) {
        f32_head_ = false;  // this torch build has no bf16->f32 mm: round through bf16
      }
    }
    return at::linear(x, lm_head_).to(at::kFloat);
  }

  // x . w^T on the hand-written kernels for any row count: the ping-pong prefill GEMM
  // (256 x 256 tiles) from LS_PGEMM_MIN_T rows, the 256-row decode GEMM (split-K, in
  // blocks of 256 rows) below that.  The library GEMM remains only for shapes neither
  // kernel takes (tiny test models: N % 128 or K % 64 != 0) or LS_PGEMM=lib.
  at::Tensor proj(const at::Tensor& x, const at::Tensor& w) {
    const int64_t T = x.size(0);
    at::Tensor out = at::empty({T, w.size(0)}, x.options());
    if (pgemm(T, w, false)) {
      gemm_prefill(out, x, w, false, -1);
    } else if (plib(T, w)) {
      at::linear_out(out, x, w);
    } else if (dgemm_blocks_ok(w, false) && x.stride(1) == 1) {
      for (int64_t r0 = 0; r0 < T; r0 += kDgemmMaxM) {
        const int64_t n = std::min<int64_t>(kDgemmMaxM, T - r0);
        decode_gemm(out.narrow(0, r0, n), x.narrow(0, r0, n), w, dg_ws_, c10::nullopt, c10::nullopt, eps_, 0, 0);
      }
    } else {
      out = at::linear(x, w);
    }
    return out;
  }

  // silu(x . w[:F]^T) * (x . w[F:]^T) for any row count (same routing as proj)
  at::Tensor proj_silu(const at::Tensor& x, const at::Tensor& w) {
    const int64_t T = x.size(0);
    at::Tensor a = at::empty({T, w.size(0) / 2}, x.options());
    if (pgemm(T, w, true)) {
      gemm_prefill(a, x, w, true, -1);
    } else if (dgemm_blocks_ok(w, true) && x.stride(1) == 1) {
      for (int64_t r0 = 0; r0 < T; r0 += kDgemmMaxM) {
        const int64_t n = std::min<int64_t>(kDgemmMaxM, T - r0);
        decode_gemm_silu(a.narrow(0, r0, n), x.narrow(0, r0, n), w, dg_ws_, dg_tickets_, status_.narrow(0, 0, 1), 0);
      }
    } else {
      at::Tensor gu = at::linear(x, w);
      silu_and_mul(a, gu);
    }
    return a;
  }

  // f32 logits [rows or T, vocab]; decode rows are [0, num_decode), prefill rows after.
  at::Tensor forward_impl(const at::Tensor& ids, const at::Tensor& pos, const at::Tensor& slots, int64_t num_decode,
                          const at::Tensor& d_bt, const at::Tensor& d_ctx, int64_t nsplit, int64_t bps,
                          const at::Tensor& ws, int64_t num_prefill, const at::Tensor& p_bt, const at::Tensor& q_start,
                          const at::Tensor& q_len, const at::Tensor& ctx_len, const at::Tensor& tiles,
                          const c10::optional<at::Tensor>& rows, bool gather_logits = true) {
    const int64_t T = ids.size(0);
    if (num_prefill == 0 && num_decode == T && fused_ready(T))
      return forward_dgemm(ids, pos, slots, d_bt, d_ctx, nsplit, bps, ws, rows);
    at::Tensor h = embed(ids);
    at::Tensor residual = h;
    at::Tensor x = at::empty_like(h);
    rmsnorm(x, h, in_norm_[0], eps_);
    const int64_t L = qkv_w_.size();
    // Decode-sized steps (5..256 rows) run on the 256-row decode GEMM (gemm_decode.hip,
    // dgemm()); the skinny ring (gemm_skinny.hip) remains the path for LS_DGEMM=0 or
    // shapes the decode GEMM does not take: qkv at T <= 32, o_proj at T <= 192 and
    // down_proj at 48 <= T <= 256, the last two with the residual add + RMSNorm fused into
    // the split-K reduction at TP=1; under TP the row-parallel partial sums are
    // all-reduced first, so o/down store the plain GEMM and the residual add + RMSNorm
    // runs after the all-reduce.
    const bool sk = skinny_enabled();
    // T <= 4 (single-stream / low-concurrency chat): the register-streaming GEMV
    // (ops/csrc/gemm_gemv.hip) for all four projections, gate_up with silu*up fused; it
    // fuses no residual, so it also serves tensor-parallel ranks.
    const bool gv = gemv_enabled() && T <= 4;
    auto attend = [&](int64_t l, const at::Tensor& qkv, bool roped) {
      if (!roped) rope_and_cache(qkv, pos, cos_sin_, slots, kc_[l], vc_[l], hq_, hkv_, true);
      at::Tensor q = qkv.narrow(1, 0, hq_ * d_);
      at::Tensor attn = at::empty({T, hq_ * d_}, qkv.options());
      if (num_decode > 0)
        paged_decode_attention(attn.narrow(0, 0, num_decode), q.narrow(0, 0, num_decode), kc_[l], vc_[l], d_bt,
                               d_ctx, scale_, nsplit, bps, ws);
      if (num_prefill > 0)
        paged_prefill_attention(attn, q, kc_[l], vc_[l], p_bt, q_start, q_len, ctx_len, tiles, hq_, scale_);
      return attn;
    };
    // TP = 1: the residual add + RMSNorm after o_proj and down_proj run in the PROLOGUE of
    // the next GEMV (gate_up / the next layer's qkv), which recomputes the norm per block
    // from the L2-resident activations -- no separate norm kernels or hand-offs.  (A
    // last-block add+norm epilogue with an agent-scope ticket measured slower: 3.72 vs
    // 3.48 ms per batch-1 step, the serial tail outweighs the launch it saves.)
    bool fused = gv && !pg_;
    for (int64_t l = 0; l < L && fused; ++l)
      fused = gemv_supported(qkv_w_[l], false) && gemv_supported(o_w_[l], false) &&
              gemv_supported(gate_up_w_[l], true) && gemv_supported(down_w_[l], false);
    if (fused) {
      at::Tensor dn;
      for (int64_t l = 0; l < L; ++l) {
        // qkv GEMV with RoPE + K/V cache writes in its epilogue (and, past layer 0, the
        // previous layer's residual add + RMSNorm in its prologue)
        at::Tensor qkv = at::empty({T, qkv_w_[l].size(0)}, x.options());
        if (l == 0) {
          gemv_qkv(qkv, x, qkv_w_[l], pos, cos_sin_, slots, kc_[l], vc_[l], hq_, hkv_, true, c10::nullopt,
                   c10::nullopt, c10::nullopt, c10::nullopt, eps_);
        } else if (T <= gemv_pro_max_t()) {
          at::Tensor rn = at::empty_like(residual);
          gemv_qkv(qkv, x, qkv_w_[l], pos, cos_sin_, slots, kc_[l], vc_[l], hq_, hkv_, true, dn, residual, rn,
                   in_norm_[l], eps_);
          residual = rn;
        } else {
          fused_add_rmsnorm(dn, residual, in_norm_[l], eps_);
          gemv_qkv(qkv, dn, qkv_w_[l], pos, cos_sin_, slots, kc_[l], vc_[l], hq_, hkv_, true, c10::nullopt,
                   c10::nullopt, c10::nullopt, c10::nullopt, eps_);
        }
        at::Tensor attn = attend(l, qkv, true);
        at::Tensor o = at::empty_like(residual);
        gemv(o, attn, o_w_[l]);
        at::Tensor a = at::empty({T, gate_up_w_[l].size(0) / 2}, o.options());
        if (T <= gemv_pro_max_t()) {
          at::Tensor rn = at::empty_like(residual);
          gemv_silu_norm(a, o, residual, rn, post_norm_[l], eps_, gate_up_w_[l]);
          residual = rn;
        } else {
          fused_add_rmsnorm(o, residual, post_norm_[l], eps_);
          gemv_silu(a, o, gate_up_w_[l]);
        }
        dn = at::empty_like(residual);
        gemv(dn, a, down_w_[l]);
      }
      fused_add_rmsnorm(dn, residual, final_norm_, eps_);
      x = dn;
    }
    const bool decode_only = num_prefill == 0 && num_decode == T;
    for (int64_t l = 0; l < L && !fused; ++l) {
      at::Tensor qkv;
      bool roped = false;   // RoPE + the K/V cache write already done by the qkv GEMM's reduction
      if (gv && gemv_supported(qkv_w_[l], false)) {
        qkv = at::empty({T, qkv_w_[l].size(0)}, x.options());
        gemv(qkv, x, qkv_w_[l]);
      } else if (dgemm(T, qkv_w_[l], false)) {
        qkv = at::empty({T, qkv_w_[l].size(0)}, x.options());
        if (decode_only && qkv_rope_fused()) {
          decode_gemm_qkv_rope(qkv, x, qkv_w_[l], dg_ws_, pos, cos_sin_, slots, kc_[l], vc_[l], hq_, hkv_);
          roped = true;
        } else {
          decode_gemm(qkv, x, qkv_w_[l], dg_ws_, c10::nullopt, c10::nullopt, eps_, 0, 0);
        }
      } else if (sk && T <= skinny_qkv_max() && skinny_shape(qkv_w_[l])) {
        qkv = at::empty({T, qkv_w_[l].size(0)}, x.options());
        skinny_gemm(qkv, x, qkv_w_[l]);
      } else {
        qkv = proj(x, qkv_w_[l]);
      }
      at::Tensor attn = at::empty({T, hq_ * d_}, qkv.options());
      at::Tensor q = qkv.narrow(1, 0, hq_ * d_);
      if (roped) {
        paged_decode_attention(attn, q, kc_[l], vc_[l], d_bt, d_ctx, scale_, nsplit, bps, ws);
      } else if (decode_only && rope_fused()) {
        // decode-only step: RoPE + K/V cache write inside the attention kernel
        paged_decode_attention_rope(attn, qkv, pos, cos_sin_, slots, kc_[l], vc_[l], d_bt, d_ctx, scale_, nsplit,
                                    bps, ws);
      } else {
        rope_and_cache(qkv, pos, cos_sin_, slots, kc_[l], vc_[l], hq_, hkv_, true);
        if (num_decode > 0)
          paged_decode_attention(attn.narrow(0, 0, num_decode), q.narrow(0, 0, num_decode), kc_[l], vc_[l], d_bt,
                                 d_ctx, scale_, nsplit, bps, ws);
      }
      if (num_prefill > 0)
        paged_prefill_attention(attn, q, kc_[l], vc_[l], p_bt, q_start, q_len, ctx_len, tiles, hq_, scale_);
      at::Tensor o;
      if (gv && gemv_supported(o_w_[l], false)) {
        o = at::empty_like(residual);
        gemv(o, attn, o_w_[l]);
        all_reduce(o);
        fused_add_rmsnorm(o, residual, post_norm_[l], eps_);
      } else if (dgemm(T, o_w_[l], false)) {
        o = at::empty_like(residual);
        if (!pg_) {
          decode_gemm(o, attn, o_w_[l], dg_ws_, residual, post_norm_[l], eps_, 0, 0);
        } else {
          decode_gemm(o, attn, o_w_[l], dg_ws_, c10::nullopt, c10::nullopt, eps_, 0, 0);
          all_reduce(o);
          fused_add_rmsnorm(o, residual, post_norm_[l], eps_);
        }
      } else if (sk && T <= 192 && skinny_shape(o_w_[l])) {
        o = at::empty_like(residual);
        if (!pg_) {
          skinny_gemm_add_rmsnorm(o, attn, o_w_[l], residual, post_norm_[l], eps_);
        } else {
          skinny_gemm(o, attn, o_w_[l]);
          all_reduce(o);
          fused_add_rmsnorm(o, residual, post_norm_[l], eps_);
        }
      } else {
        o = proj(attn, o_w_[l]);
        all_reduce(o);
        fused_add_rmsnorm(o, residual, post_norm_[l], eps_);
      }
      at::Tensor a;
      if (gv && gemv_supported(gate_up_w_[l], true)) {
        a = at::empty({T, gate_up_w_[l].size(0) / 2}, o.options());
        gemv_silu(a, o, gate_up_w_[l]);
      } else if (dgemm(T, gate_up_w_[l], true)) {
        // decode batch: SwiGLU in the epilogue after the in-launch combine of the K halves
        a = at::empty({T, gate_up_w_[l].size(0) / 2}, o.options());
        decode_gemm_silu(a, o, gate_up_w_[l], dg_ws_, dg_tickets_, status_.narrow(0, 0, 1), 0);
      } else {
        a = proj_silu(o, gate_up_w_[l]);
      }
      const at::Tensor& nxt = l + 1 < L ? in_norm_[l + 1] : final_norm_;
      at::Tensor dn;
      if (gv && gemv_supported(down_w_[l], false)) {
        dn = at::empty_like(residual);
        gemv(dn, a, down_w_[l]);
        all_reduce(dn);
        fused_add_rmsnorm(dn, residual, nxt, eps_);
      } else if (dgemm(T, down_w_[l], false)) {
        dn = at::empty_like(residual);
        if (!pg_) {
          decode_gemm(dn, a, down_w_[l], dg_ws_, residual, nxt, eps_, 0, 0);
        } else {
          decode_gemm(dn, a, down_w_[l], dg_ws_, c10::nullopt, c10::nullopt, eps_, 0, 0);
          all_reduce(dn);
          fused_add_rmsnorm(dn, residual, nxt, eps_);
        }
      } else if (sk && T >= 48 && T <= 256 && skinny_shape(down_w_[l])) {
        dn = at::empty_like(residual);
        if (!pg_) {
          skinny_gemm_add_rmsnorm(dn, a, down_w_[l], residual, nxt, eps_);
        } else {
          skinny_gemm(dn, a, down_w_[l]);
          all_reduce(dn);
          fused_add_rmsnorm(dn, residual, nxt, eps_);
        }
      } else {
        dn = proj(a, down_w_[l]);
        all_reduce(dn);
        fused_add_rmsnorm(dn, residual, nxt, eps_);
      }
      x = dn;
    }
    at::Tensor sel = rows.has_value() ? x.index_select(0, *rows) : x;
    at::Tensor lg = lm_head(sel);
    if (pg_ && !gather_logits) {
      // vocab-parallel sampling downstream: this rank's valid slice only
      const int64_t valid = std::max<int64_t>(0, std::min<int64_t>(lg.size(1), vocab_ - vocab_start_));
      return valid == lg.size(1) ? lg : lg.narrow(1, 0, valid);
    }
    if (pg_) {
      const int64_t world = pg_->getSize();
      std::vector<at::Tensor> parts;
      for (int64_t i = 0; i < world; ++i) parts.push_back(at::empty_like(lg));
      std::vector<std::vector<at::Tensor>> outs{parts};
      std::vector<at::Tensor> ins{lg.contiguous()};
      pg_->allgather(outs, ins)->wait();
      lg = at::cat(parts, 1);
    }
    if (lg.size(1) != vocab_) lg = lg.narrow(1, 0, vocab_).contiguous();
    return lg;
  }

  // Decode-only steps of 129..256 rows at TP = 1: the norm-deferred layer of
  // gemm_decode.hip (DgArgs).  Per layer 5 launches -- qkv (+ in-launch split-K combine,
  // 1/rms, RoPE, KV write), attention, o (+ combine, residual add, y = h * g, row sums of
  // h^2), gate_up (+ 1/rms, SwiGLU), down (+ combine ...) -- instead of 8.  The residual
  // stream h is updated in place; y_in_ / y_post_ hold bf16(h * g) for the next GEMM and
  // ss_in_ / ss_post_ the per-tile sums of h^2 its epilogue turns into 1/rms.
  at::Tensor forward_dgemm(const at::Tensor& ids, const at::Tensor& pos, const at::Tensor& slots,
                           const at::Tensor& d_bt, const at::Tensor& d_ctx, int64_t nsplit, int64_t bps,
                           const at::Tensor& ws, const c10::optional<at::Tensor>& rows) {
    const int64_t T = ids.size(0);
    at::Tensor h = embed(ids).contiguous();
    const int64_t L = qkv_w_.size();
    at::Tensor y = y_in_.narrow(0, 0, T), y2 = y_post_.narrow(0, 0, T);
    at::Tensor ss_in = ss_in_.narrow(0, 0, T), ss_post = ss_post_.narrow(0, 0, T), ss0 = ss0_.narrow(0, 0, T);
    at::Tensor err = status_.narrow(0, 1, 1);
    rms_prep(y, ss0, h, in_norm_[0]);
    for (int64_t l = 0; l < L; ++l) {
      at::Tensor qkv = at::empty({T, qkv_w_[l].size(0)}, h.options());
      decode_gemm_qkv_cmb(qkv, y, qkv_w_[l], dg_ws_, cnt_qkv_, l == 0 ? ss0 : ss_in, eps_, pos, cos_sin_, slots,
                          kc_[l], vc_[l], hq_, hkv_, err);
      at::Tensor attn = at::empty({T, hq_ * d_}, h.options());
      paged_decode_attention(attn, qkv.narrow(1, 0, hq_ * d_), kc_[l], vc_[l], d_bt, d_ctx, scale_, nsplit, bps, ws);
      decode_gemm_res(y2, attn, o_w_[l], dg_ws_, cnt_o_, h, post_norm_[l], ss_post, err);
      at::Tensor a = at::empty({T, gate_up_w_[l].size(0) / 2}, h.options());
      decode_gemm_silu_r(a, y2, gate_up_w_[l], ss_post, eps_);
      decode_gemm_res(y, a, down_w_[l], dg_ws_, cnt_down_, h, l + 1 < L ? in_norm_[l + 1] : final_norm_, ss_in, err);
    }
    at::Tensor x = at::empty_like(h);
    rows_rms_scale(x, y, ss_in, eps_);
    at::Tensor sel = rows.has_value() ? x.index_select(0, *rows) : x;
    at::Tensor lg = lm_head(sel);
    if (lg.size(1) != vocab_) lg = lg.narrow(1, 0, vocab_).contiguous();
    return lg;
  }

  at::Tensor forward(at::Tensor ids, at::Tensor pos, at::Tensor slots, int64_t num_decode,
                     c10::optional<at::Tensor> d_bt, c10::optional<at::Tensor> d_ctx, int64_t nsplit, int64_t bps,
                     c10::optional<at::Tensor> ws, int64_t num_prefill, c10::optional<at::Tensor> p_bt,
                     c10::optional<at::Tensor> q_start, c10::optional<at::Tensor> q_len,
                     c10::optional<at::Tensor> ctx_len, c10::optional<at::Tensor> tiles,
                     c10::optional<at::Tensor> rows) {
    at::Tensor none = at::empty({0}, ids.options().dtype(at::kInt));
    auto get = [&](const c10::optional<at::Tensor>& t) { return t.has_value() ? *t : none; };
    at::Tensor ws_t = ws.has_value() ? *ws : at::empty({0}, ids.options().dtype(at::kFloat));
    TORCH_CHECK(num_decode == 0 || (d_bt.has_value() && d_ctx.has_value()), "decode rows need block tables");
    TORCH_CHECK(num_prefill == 0 || (p_bt.has_value() && q_start.has_value() && q_len.has_value() &&
                                     ctx_len.has_value() && tiles.has_value()), "prefill rows need metadata");
    return forward_impl(ids, pos, slots, num_decode, get(d_bt), get(d_ctx), nsplit, bps, ws_t, num_prefill,
                        get(p_bt), get(q_start), get(q_len), get(ctx_len), get(tiles), rows);
  }

  int64_t hq() const { return hq_; }
  int64_t head_dim() const { return d_; }
  int64_t vocab() const { return vocab_; }
  int64_t vocab_start() const { return vocab_start_; }
  c10::intrusive_ptr<::c10d::ProcessGroup> pg() const { return pg_; }

  // The sampler's collectives on the one-shot buffers when LS_ONESHOT_AR=1 (and the
  // message fits), c10d otherwise: int64 sum in place, 32-bit all-gather.
  void allreduce_i64(at::Tensor t) { oneshot_route_sum_i64(oneshot_, pg_, t); }
  void allgather32(const at::Tensor& src, const at::Tensor& dst) { oneshot_route_gather32(oneshot_, pg_, src, dst); }

 private:
  at::Tensor embed(const at::Tensor& ids) {
    at::Tensor idl = ids.to(at::kLong);
    if (!pg_) return at::embedding(embed_, idl);
    const int64_t vpr = embed_.size(0);
    at::Tensor local = idl - vocab_start_;
    at::Tensor mask = (local < 0).logical_or(local >= vpr);
    at::Tensor h = at::embedding(embed_, local.clamp(0, vpr - 1));
    h.masked_fill_(mask.unsqueeze(1), 0);
    all_reduce(h);
    return h;
  }

  // LS_DGEMM_FUSED=1: the norm-deferred fused 129..256-row decode layer (in-launch
  // split-K combine).  Off by default: measured 9.43 vs 8.80 ms per B=256 decode step
  // (profiles/eng2_fused_r4.log) -- the 32 MB of slab writes + reads after the
  // rendezvous cost more than the reduce launches they replace.
  static bool fused_env() {
    static const bool on = [] {
      const char* e = getenv("LS_DGEMM_FUSED");
      return e != nullptr && e[0] == '1';
    }();
    return on;
  }
  bool fused_ready(int64_t T) const {
    return cnt_qkv_.defined() && dgemm_enabled() && T >= std::max(dgemm_min_t(), fused_min_t()) &&
           T <= kDgemmMaxM;
  }

  static bool gemv_enabled() {
    static const bool on = [] {
      const char* v = std::getenv("LS_GEMV");
      return !(v && std::string(v) == "0");
    }();
    return on;
  }

  // Largest T whose qkv / gate_up GEMVs recompute the add + RMSNorm in their prologue.  Each
  // block re-reads o and the residual (2 T K bf16 from L2), which at T = 4 equals the
  // block's 64 KB of weights: gate_up measured 62 us with the prologue against 41 us
  // plain + a separate fused_add_rmsnorm launch; batch-4 decode step 4.59 -> 4.15 ms
  // (tools/gemv_bench.py, tools/engine_bench.py; profiles/gemv_r4/gemv_ab_r4h.log).
  static int gemv_pro_max_t() {
    static const int t = [] {
      const char* e = getenv("LS_GEMV_PRO_MAX_T");
      return e ? atoi(e) : 2;
    }();
    return t;
  }

  // LS_ATTN_ROPE=0: separate rope_cache launch before decode attention (A/B switch)
  // Decode-only steps whose qkv runs on the split-K decode GEMM: RoPE + the K/V cache
  // write inside its reduction (LS_QKV_ROPE=0: the attention kernel's fused form instead).
  static bool qkv_rope_fused() {
    static const bool on = [] {
      const char* e = getenv("LS_QKV_ROPE");
      return e == nullptr || e[0] != '0';
    }();
    return on;
  }
  static bool rope_fused() {
    static const bool on = [] {
      const char* e = getenv("LS_ATTN_ROPE");
      return e == nullptr || e[0] != '0';
    }();
    return on;
  }

  static bool skinny_enabled() {
    static const bool on = [] {
      const char* e = getenv("LS_SKINNY_GEMM");
      return e == nullptr || e[0] != '0';
    }();
    return on;
  }
  // Prefill-sized steps (T >= LS_PGEMM_MIN_T, default 1024) run all four projections on
  // the 256 x 256-tile ping-pong GEMM (ops/csrc/gemm_prefill.hip), gate_up with SwiGLU in
  // its epilogue (no [T, 2F] round trip).  LS_PGEMM=lib: the library GEMM instead (A/B
  // switch); LS_PGEMM=route: qkv / o / down by the measured per-M-bucket table
  // (ops/pgemm_route_gfx950.csv, tools/pgemm_route_tune.py) between this kernel and the
  // library GEMM, gate_up always here.  (Until round 6 a "library" bucket fell through to
  // the 256-row decode GEMM blocks, so route-mode A/Bs before then measured those.)
  static bool pgemm(int64_t T, const at::Tensor& w, bool silu) { return prefill_route(T, w, silu) == 1; }
  // LS_PGEMM=route and the table says the library GEMM for this plain projection's M bucket
  static bool plib(int64_t T, const at::Tensor& w) { return prefill_route(T, w, false) == 2; }
  // 0: not a prefill-sized step (decode GEMM blocks / library below), 1: gemm_prefill,
  // 2: the library GEMM (route mode, where the table measured it faster)
  static int prefill_route(int64_t T, const at::Tensor& w, bool silu) {
    static const int mode = [] {
      const char* e = getenv("LS_PGEMM");
      if (e == nullptr) return 2;
      const std::string v(e);
      if (v == "lib" || v == "0") return 0;
      if (v == "route" || v == "1") return 1;
      return 2;
    }();
    static const int64_t min_t = [] {
      const char* e = getenv("LS_PGEMM_MIN_T");
      return e ? (int64_t)atoll(e) : (int64_t)1024;
    }();
    if (mode == 0 || !gemm_prefill_supported(w, silu) || T < min_t) return 0;
    if (silu || mode == 2) return 1;
    return pgemm_route::use_pp(T, w.size(0), w.size(1)) ? 1 : 2;
  }
  // rows below the prefill threshold: the decode GEMM in 256-row blocks
  bool dgemm_blocks_ok(const at::Tensor& w, bool silu) const {
    static const bool lib = [] {
      const char* e = getenv("LS_PGEMM");
      return e != nullptr && (std::string(e) == "lib" || std::string(e) == "0");
    }();
    return !lib && dgemm_enabled() && dg_ws_.defined() && decode_gemm_supported(w, silu);
  }
  // Fallback routing when the decode GEMM does not take a step (LS_DGEMM=0, or T below
  // LS_DGEMM_MIN_T): qkv rows up to this many go to the skinny ring.  With the default
  // routing the decode GEMM is tried FIRST and takes every qkv from 5 rows (it measured
  // faster than the skinny ring at every M from 5, profiles/dgemm_smallm_r4.log), so this
  // knob only matters for those A/B runs.
  static int64_t skinny_qkv_max() {
    static const int64_t v = [] {
      const char* e = getenv("LS_SKINNY_QKV_MAX");
      return e ? (int64_t)atoll(e) : (int64_t)32;
    }();
    return v;
  }
  static bool skinny_shape(const at::Tensor& w) { return w.size(0) % 128 == 0 && w.size(1) % 64 == 0; }

  // Decode batches of LS_DGEMM_MIN_T (default 5) .. 256 rows run all four projections
  // on the 256-row decode GEMM (ops/csrc/gemm_decode.hip) instead of hipBLASLt / the
  // skinny ring.  LS_DGEMM=0 turns it off (A/B switch).
  static constexpr int64_t kDgemmMaxM = 256;
  static bool dgemm_enabled() {
    static const bool on = [] {
      const char* e = getenv("LS_DGEMM");
      return e == nullptr || e[0] != '0';
    }();
    return on;
  }
  // From 5 rows (the GEMV takes 1..4): measured against hipBLASLt and the skinny ring at
  // 5..128 rows on the Llama-3-8B shapes (profiles/dgemm_smallm_r4.log): qkv 17-24.5 us
  // vs 28.8-31.1 (hipBLASLt) / 18.3-27.5 (skinny), gate_up + SwiGLU 52.4-54.3 vs
  // 53.8-62.7 / 57.7-59.3, down 30.5-37.8 vs 34.3-84.0 / 35.0-45.4.
  static int64_t dgemm_min_t() {
    static const int64_t min_t = [] {
      const char* e = getenv("LS_DGEMM_MIN_T");
      return e ? (int64_t)atoll(e) : (int64_t)5;
    }();
    return min_t;
  }
  // the norm-deferred layer from this many rows (LS_DGEMM_FUSED_MIN_T)
  static int64_t fused_min_t() {
    static const int64_t v = [] {
      const char* e = getenv("LS_DGEMM_FUSED_MIN_T");
      return e ? (int64_t)atoll(e) : (int64_t)129;
    }();
    return v;
  }
  bool dgemm(int64_t T, const at::Tensor& w, bool silu) const {
    return dgemm_enabled() && dg_ws_.defined() && T >= dgemm_min_t() && T <= kDgemmMaxM &&
           decode_gemm_supported(w, silu);
  }

  void all_reduce(at::Tensor& t) {
    if (!pg_) return;
    if (oneshot_ && t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.numel() <= oneshot_max_) {
      oneshot_allreduce_run(oneshot_, t);
      return;
    }
    std::vector<at::Tensor> v{t};
    pg_->allreduce(v)->wait();
  }

  std::shared_ptr<OneShotAllReduce> oneshot_;
  int64_t oneshot_max_ = 0;

  bool f32_head_ = true;
  at::Tensor status_, dg_ws_, dg_tickets_;
  at::Tensor y_in_, y_post_, ss_in_, ss_post_, ss0_, cnt_qkv_, cnt_o_, cnt_down_;   // forward_dgemm
  at::Tensor embed_;
  std::vector<at::Tensor> qkv_w_, o_w_, gate_up_w_, down_w_, in_norm_, post_norm_;
  at::Tensor final_norm_, lm_head_;
  std::vector<at::Tensor> kc_, vc_;
  at::Tensor kv_tab_;          // device [2 L] base pointers of the K / V caches (copy_kv_blocks)
  int64_t kv_block_bytes_ = 0;
  at::Tensor cos_sin_;
  int64_t hq_, hkv_, d_;
  double eps_, scale_;
  int64_t vocab_, vocab_start_;
  c10::intrusive_ptr<::c10d::ProcessGroup> pg_;
};

// ---------------------------------------------------------------------------- BERT
class BertRunner {
 public:
  // fused: empty, or per layer {qkv W' (W for layer 0), qkv c1, qkv c2, ff1 W', ff1 c1, ff1 c2}
  // -> the fused layer sequence of models/bert.py forward_fused (gemm_fused.hip epilogues).
  BertRunner(at::Tensor wte, at::Tensor wpe, at::Tensor wtt, at::Tensor emb_g, at::Tensor emb_b,
             std::vector<std::vector<at::Tensor>> layers, int64_t heads, double eps, double scale, int64_t pooling,
             bool normalize, std::vector<std::vector<at::Tensor>> fused)
      : wte_(wte), wpe_(wpe), wtt_(wtt), emb_g_(emb_g), emb_b_(emb_b), layers_(layers), heads_(heads), eps_(eps),
        scale_(scale), pooling_(pooling), normalize_(normalize), fused_(fused) {
    for (auto& l : layers_) TORCH_CHECK(l.size() == 12, "bert layer needs 12 tensors");
    TORCH_CHECK(fused_.empty() || fused_.size() == layers_.size(), "fused params: one entry per layer");
    for (auto& f : fused_) TORCH_CHECK(f.size() == 6, "fused layer needs 6 tensors");
  }

  at::Tensor forward(at::Tensor ids, at::Tensor pos, at::Tensor starts, at::Tensor lens, at::Tensor tiles,
                     bool out_f32) {
    const int64_t T = ids.size(0), H = wte_.size(1);
    at::Tensor x = at::empty({T, H}, wte_.options());
    embed_layernorm(x, ids, pos, c10::nullopt, wte_, wpe_, wtt_, emb_g_, emb_b_, eps_);
    if (!fused_.empty()) {
      x = forward_fused(x, starts, lens, tiles);
    } else {
      for (auto& l : layers_) {
        // qkv_w, qkv_b, o_w, o_b, ln1_g, ln1_b, ff1_w, ff1_b, ff2_w, ff2_b, ln2_g, ln2_b
        at::Tensor qkv = at::linear(x, l[0], l[1]);
        at::Tensor a = at::empty({T, H}, x.options());
        varlen_encoder_attention(a, qkv, starts, lens, tiles, heads_, heads_, scale_);
        at::Tensor o = at::linear(a, l[2]);
        at::Tensor x1 = at::empty_like(x);
        layernorm(x1, o, l[3], x, l[4], l[5], eps_);
        at::Tensor hdn = at::linear(x1, l[6]);
        bias_gelu(hdn, l[7]);
        at::Tensor o2 = at::linear(hdn, l[8]);
        at::Tensor x2 = at::empty_like(x);
        layernorm(x2, o2, l[9], x1, l[10], l[11], eps_);
        x = x2;
      }
    }
    at::Tensor out = at::empty({starts.size(0), H}, x.options().dtype(out_f32 ? at::kFloat : x.scalar_type()));
    pool_embeddings(out, x, starts, lens, pooling_, normalize_);
    return out;
  }

 private:
  at::Tensor forward_fused(at::Tensor x, const at::Tensor& starts, const at::Tensor& lens, const at::Tensor& tiles) {
    const int64_t T = x.size(0), H = x.size(1);
    auto st_opts = x.options().dtype(at::kFloat);
    at::Tensor xp2, st2;
    const at::Tensor* pg = nullptr;
    const at::Tensor* pb = nullptr;
    for (size_t i = 0; i < layers_.size(); ++i) {
      auto& l = layers_[i];
      auto& f = fused_[i];
      at::Tensor qkv = at::empty({T, f[0].size(0)}, x.options());
      if (i == 0)
        gemm_fused(qkv, x, f[0], l[1], false, c10::nullopt, c10::nullopt, 0, c10::nullopt, c10::nullopt,
                   c10::nullopt, c10::nullopt, eps_, c10::nullopt);
      else
        gemm_fused(qkv, xp2, f[0], l[1], false, c10::nullopt, st2, H, f[1], f[2], c10::nullopt, c10::nullopt, eps_,
                   c10::nullopt);
      at::Tensor a = at::empty({T, H}, x.options());
      varlen_encoder_attention(a, qkv, starts, lens, tiles, heads_, heads_, scale_);
      at::Tensor xp1 = at::empty({T, H}, x.options());
      at::Tensor st1 = at::empty({T, H / 64, 2}, st_opts);
      if (i == 0)
        gemm_fused(xp1, a, l[2], l[3], false, x, c10::nullopt, 0, c10::nullopt, c10::nullopt, c10::nullopt,
                   c10::nullopt, eps_, st1);
      else
        gemm_fused(xp1, a, l[2], l[3], false, xp2, st2, H, c10::nullopt, c10::nullopt, *pg, *pb, eps_, st1);
      at::Tensor hdn = at::empty({T, f[3].size(0)}, x.options());
      gemm_fused(hdn, xp1, f[3], l[7], true, c10::nullopt, st1, H, f[4], f[5], c10::nullopt, c10::nullopt, eps_,
                 c10::nullopt);
      at::Tensor nx = at::empty({T, H}, x.options());
      at::Tensor nst = at::empty({T, H / 64, 2}, st_opts);
      gemm_fused(nx, hdn, l[8], l[9], false, xp1, st1, H, c10::nullopt, c10::nullopt, l[4], l[5], eps_, nst);
      xp2 = nx;
      st2 = nst;
      pg = &l[10];
      pb = &l[11];
    }
    at::Tensor out = at::empty_like(xp2);
    layernorm(out, xp2, c10::nullopt, c10::nullopt, *pg, *pb, eps_);
    return out;
  }

  at::Tensor wte_, wpe_, wtt_, emb_g_, emb_b_;
  std::vector<std::vector<at::Tensor>> layers_;
  int64_t heads_;
  double eps_, scale_;
  int64_t pooling_;
  bool normalize_;
  std::vector<std::vector<at::Tensor>> fused_;
};

// ---------------------------------------------------------------------------- step executor
// Arena header (int32 words); must match langstream_amd/engine/arena.py.
enum Hdr : int {
  H_KIND = 0,     // 1 step, 3 stop, 4 capture bucket H_BUCKET
  H_T = 1,        // tokens in the step
  H_ND = 2,       // decode rows [0, nd)
  H_NPS = 3,      // prefill sequences
  H_NTILES = 4,   // prefill attention tiles
  H_NROWS = 5,    // rows to sample
  H_NGATHER = 6,  // decode rows whose input token is the previous step's sample
  H_NDELTA = 7,   // logit deltas (penalties / bias / min-tokens)
  H_NTOP = 8,     // top logprobs per row
  H_BUCKET = 9,   // >0: decode-only step replayed from the bucket's graph
  H_ROWS_ALL = 10, // 1: sample every row (rows == arange(T))
  H_NCOPY = 11    // KV block copies (prefix cache) ahead of the forward: kvcopy[0, n)
};
constexpr int kMaxKvCopies = 2048;   // must match MAX_KV_COPIES in engine/arena.py

// ids[gdst[i]] = tok_prev[gsrc[i]] for i < hdr[H_NGATHER]; count read on the device.
__global__ void gather_feedback_kernel(int32_t* __restrict__ ids, const int64_t* __restrict__ gdst,
                                       const int64_t* __restrict__ gsrc, const int32_t* __restrict__ tok_prev,
                                       const int32_t* __restrict__ hdr, int cap) {
  const int n = min(hdr[H_NGATHER], cap);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    ids[gdst[i]] = tok_prev[gsrc[i]];
}

// logits[row, tok] += val for each (row, tok, val) triple, count read on the device.
// Under TP the logits are this rank's vocabulary slice starting at voff.
__global__ void logit_delta_kernel(float* __restrict__ logits, int64_t ld, int V, int nrows,
                                   const int32_t* __restrict__ trip, const int32_t* __restrict__ hdr, int cap,
                                   int voff) {
  const int n = min(hdr[H_NDELTA], cap);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = trip[3 * i], t = trip[3 * i + 1] - voff;
    const float v = __int_as_float(trip[3 * i + 2]);
    if (r >= 0 && r < nrows && t >= 0 && t < V) atomicAdd(&logits[(int64_t)r * ld + t], v);
  }
}

constexpr int kMaxTop = 32;
using clk = std::chrono::steady_clock;

class StepExecutor {
 public:
  StepExecutor(std::shared_ptr<LlamaRunner> runner, std::map<std::string, int64_t> off, int64_t arena_bytes,
               int64_t fixed_bytes, int64_t max_tokens, int64_t max_seqs, int64_t max_blocks, int64_t max_tiles,
               int64_t max_deltas, int64_t nslots, int64_t nsplit, int64_t bps, bool use_graphs, int64_t device)
      : r_(std::move(runner)), off_(std::move(off)), arena_bytes_(arena_bytes), fixed_bytes_(fixed_bytes),
        maxT_(max_tokens), maxS_(max_seqs), maxB_(max_blocks), maxTiles_(max_tiles), maxD_(max_deltas),
        nsplit_(nsplit), bps_(bps), use_graphs_(use_graphs) {
    static const char* need[] = {"hdr", "ids", "pos", "slots", "dbt", "dctx", "pbt", "q_start", "q_len", "ctx_len",
                                 "tiles", "rows", "gdst", "gsrc", "temp", "top_p", "top_k", "seeds", "steps",
                                 "kvcopy", "deltas"};
    for (const char* k : need) TORCH_CHECK(off_.count(k), "arena layout lacks ", k);
    auto dev = at::TensorOptions().device(at::kCUDA, device);
    auto pin = at::TensorOptions().dtype(at::kByte).pinned_memory(true);
    for (int64_t i = 0; i < nslots; ++i) {
      host_.push_back(at::zeros({arena_bytes_}, pin));
      out_.push_back(at::zeros({out_bytes()}, pin));
      hipEvent_t a, b;
      HIP_OK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
      in_ev_.push_back(a);
      out_ev_.push_back(b);
      in_used_.push_back(false);
    }
    arena_ = at::zeros({arena_bytes_}, dev.dtype(at::kByte));
    status_ptrs_ = r_->status_ptrs();
    st_host_ = at::zeros({nslots, kStatusWords}, at::TensorOptions().dtype(at::kInt).pinned_memory(true));
    TORCH_CHECK((int64_t)status_ptrs_.size() <= kStatusWords);
    hdr_small_ = at::zeros({16 + kStatusWords}, at::TensorOptions().dtype(at::kInt).pinned_memory(true));
    tok_ = at::zeros({maxS_}, dev.dtype(at::kInt));
    lp_ = at::zeros({maxS_}, dev.dtype(at::kFloat));
    ti_ = at::zeros({maxS_ * kMaxTop}, dev.dtype(at::kInt));
    tl_ = at::zeros({maxS_ * kMaxTop}, dev.dtype(at::kFloat));
    ws_ = at::empty({std::max<int64_t>(1, maxS_ * r_->hq() * nsplit_ * (r_->head_dim() + 2))},
                    dev.dtype(at::kFloat));
    if (r_->pg()) {   // vocab-parallel sampling exchange buffers (tp_sample_* in sampling.hip)
      const int64_t W = r_->pg()->getSize(), cw = 3 + 2 * kMaxTop;
      tp_stats_ = at::zeros({maxS_ * 4}, dev.dtype(at::kFloat));
      tp_stats_all_ = at::zeros({W * maxS_ * 4}, dev.dtype(at::kFloat));
      tp_hist_ = at::zeros({maxS_ * 2 * 1024}, dev.dtype(at::kLong));
      tp_cand_ = at::zeros({maxS_ * cw}, dev.dtype(at::kFloat));
      tp_cand_all_ = at::zeros({W * maxS_ * cw}, dev.dtype(at::kFloat));
    }
    pool_ = at::cuda::graph_pool_handle();
    slot_job_.assign(nslots, -1);
    // Launcher thread (single-GPU executors): hipGraphLaunch of a ~300-node decode graph
    // returns only ~1 ms before the graph finishes (measured with --hip-trace,
    // tools/gap_analysis.py), so a launch issued from the engine thread came only after
    // the engine's own bookkeeping for the previous step -- the GPU idled ~0.5 ms per step
    // in the RAG pipeline.  A dedicated thread keeps the next step's launch queued.
    static const bool async_env = getenv("LS_ASYNC_LAUNCH") ? atoi(getenv("LS_ASYNC_LAUNCH")) != 0 : true;
    if (!r_->pg() && async_env) {
      stream_ = at::hip::getCurrentHIPStreamMasqueradingAsCUDA();
      launcher_ = std::thread([this] { launcher_loop(); });
    }
  }

  ~StepExecutor() {
    if (launcher_.joinable()) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
      }
      cv_.notify_all();
      launcher_.join();
    }
    for (auto e : in_ev_) (void)hipEventDestroy(e);
    for (auto e : out_ev_) (void)hipEventDestroy(e);
  }

  int64_t out_bytes() const { return maxS_ * 8 + maxS_ * kMaxTop * 8; }
  at::Tensor host_slot(int64_t i) { return host_.at(i); }
  at::Tensor out_slot(int64_t i) { return out_.at(i); }
  bool has_graph(int64_t B) const { return graphs_.count(B) > 0; }

  // Block until the H2D copy that last read host slot i has finished (slot reusable).
  void wait_in(int64_t i) {
    wait_submitted(i);
    if (in_used_.at(i)) HIP_OK(hipEventSynchronize(in_ev_[i]));
  }
  // Block until the results of the step that wrote out slot i are on the host.
  void wait_out(int64_t i) {
    wait_submitted(i);
    HIP_OK(hipEventSynchronize(out_ev_.at(i)));
    check_status(st_host_[i].data_ptr<int>());
  }

  // One scheduler round trip in a single GIL-released call: launch the step in host
  // slot `slot` (results -> out slot `slot`), then block until the previous step's
  // results (out slot `prev`, -1: none) are on the host, then until host slot `next`
  // is free for the scheduler to fill.
  void step(int64_t slot, int64_t prev, int64_t next) {
    if (launcher_.joinable()) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        rethrow_locked();
        slot_job_.at(slot) = issued_++;
        jobs_.push_back(slot);
      }
      cv_.notify_all();
    } else {
      launch(slot, slot);
    }
    auto t0 = clk::now();
    if (prev >= 0) wait_out(prev);
    auto t1 = clk::now();
    if (next >= 0) wait_in(next);
    t_wait_ += std::chrono::duration<double, std::milli>(t1 - t0).count();
  }

  // {upload, run (enqueue forward/graph), download, wait} milliseconds, cumulative.
  std::vector<double> timings() const { return {t_up_, t_run_, t_down_, t_wait_}; }

  // Python entry: launch synchronously, after anything the launcher thread still holds.
  void launch_sync(int64_t slot, int64_t oslot) {
    drain();
    launch(slot, oslot);
  }

  // Rank 0: run the step described by host slot `slot`; results land in out slot `oslot`.
  void launch(int64_t slot, int64_t oslot) {
    const int32_t* hdr = reinterpret_cast<const int32_t*>(host_.at(slot).data_ptr());
    TORCH_CHECK(hdr[H_KIND] == 1, "launch expects a step header");
    validate(hdr);
    auto t0 = clk::now();
    upload(slot);
    auto t1 = clk::now();
    run(hdr);
    auto t2 = clk::now();
    t_up_ += std::chrono::duration<double, std::milli>(t1 - t0).count();
    t_run_ += std::chrono::duration<double, std::milli>(t2 - t1).count();
    download(hdr, oslot);
    t_down_ += std::chrono::duration<double, std::milli>(clk::now() - t2).count();
  }

  // All ranks (rank 0 announces it to the workers): capture the decode graph for bucket B.
  void capture(int64_t B) {
    drain();
    if (graphs_.count(B)) return;
    if (r_->pg()) {
      int32_t* hdr = reinterpret_cast<int32_t*>(hdr_small_.data_ptr());
      for (int i = 0; i < 16; ++i) hdr[i] = 0;
      hdr[H_KIND] = 4;
      hdr[H_BUCKET] = (int32_t)B;
      announce(hdr);
    }
    do_capture(B);
  }

  void shutdown() {
    drain();
    if (!r_->pg()) return;
    int32_t* hdr = reinterpret_cast<int32_t*>(hdr_small_.data_ptr());
    for (int i = 0; i < 16; ++i) hdr[i] = 0;
    hdr[H_KIND] = 3;
    announce(hdr);
    HIP_OK(hipStreamSynchronize(stream()));
  }

  // Non-zero TP ranks: mirror rank 0's steps until told to stop.
  void worker_loop() {
    TORCH_CHECK(r_->pg(), "worker_loop needs a process group");
    int32_t* hdr = reinterpret_cast<int32_t*>(hdr_small_.data_ptr());
    while (true) {
      broadcast_arena();
      HIP_OK(hipMemcpyAsync(hdr, arena_.data_ptr(), 16 * sizeof(int32_t), hipMemcpyDeviceToHost, stream()));
      HIP_OK(hipStreamSynchronize(stream()));
      check_status(hdr + 16);   // the previous step's
      const int kind = hdr[H_KIND];
      if (kind == 3) return;
      if (kind == 4) {
        do_capture(hdr[H_BUCKET]);
      } else if (kind == 1) {
        validate(hdr);
        run(hdr);
        // a worker has no result slot: its status words land behind the step and are
        // checked after the next header's synchronisation (no extra sync per step)
        copy_status(hdr + 16);
      } else {
        TORCH_CHECK(false, "bad step kind ", kind);
      }
    }
  }

 private:
  hipStream_t stream() const { return at::hip::getCurrentHIPStream().stream(); }

  void rethrow_locked() {
    if (err_) {
      auto e = err_;
      err_ = nullptr;
      std::rethrow_exception(e);
    }
  }

  // The job that last used slot i has been handed to HIP (its events are recorded).
  void wait_submitted(int64_t i) {
    if (!launcher_.joinable()) return;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return err_ || done_ > slot_job_.at(i); });
    rethrow_locked();
  }

  void drain() {
    if (!launcher_.joinable()) return;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return err_ || done_ == issued_; });
    rethrow_locked();
  }

  void launcher_loop() {
    at::hip::HIPStreamGuardMasqueradingAsCUDA guard(*stream_);
    while (true) {
      int64_t slot;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
        if (jobs_.empty()) return;   // stop_ and nothing left to launch
        slot = jobs_.front();
        jobs_.pop_front();
      }
      try {
        launch(slot, slot);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        err_ = std::current_exception();
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        ++done_;
      }
      cv_.notify_all();
    }
  }

  template <typename T>
  at::Tensor view(const char* name, int64_t n, at::ScalarType st) {
    return arena_.narrow(0, off_.at(name), n * (int64_t)sizeof(T)).view(st);
  }

  void validate(const int32_t* h) const {
    TORCH_CHECK(h[H_T] >= 0 && h[H_T] <= maxT_, "step tokens out of range: ", h[H_T]);
    TORCH_CHECK(h[H_ND] >= 0 && h[H_ND] <= h[H_T] && h[H_ND] <= maxS_, "decode rows out of range");
    TORCH_CHECK(h[H_NPS] >= 0 && h[H_NPS] <= maxS_ && h[H_NTILES] >= 0 && h[H_NTILES] <= maxTiles_);
    TORCH_CHECK(h[H_NROWS] >= 0 && h[H_NROWS] <= maxS_ && h[H_NGATHER] >= 0 && h[H_NGATHER] <= maxS_);
    TORCH_CHECK(h[H_NDELTA] >= 0 && h[H_NDELTA] <= maxD_ && h[H_NTOP] >= 0 && h[H_NTOP] <= kMaxTop);
    TORCH_CHECK(h[H_BUCKET] >= 0 && h[H_BUCKET] <= maxS_);
    if (h[H_BUCKET] > 0)
      TORCH_CHECK(h[H_T] == h[H_ND] && h[H_ND] <= h[H_BUCKET] && h[H_NPS] == 0 && h[H_NTOP] == 0,
                  "graph steps are decode-only");
    TORCH_CHECK(h[H_NPS] == 0 || h[H_T] > h[H_ND], "prefill sequences without prefill tokens");
    TORCH_CHECK(h[H_NCOPY] >= 0 && h[H_NCOPY] <= kMaxKvCopies && (h[H_BUCKET] == 0 || h[H_NCOPY] == 0),
                "KV block copies out of range (or on a graph step)");
  }

  void upload(int64_t slot) {
    const int32_t* hdr = reinterpret_cast<const int32_t*>(host_[slot].data_ptr());
    const int64_t bytes = r_->pg() ? arena_bytes_ : fixed_bytes_ + 12 * (int64_t)hdr[H_NDELTA];
    HIP_OK(hipMemcpyAsync(arena_.data_ptr(), host_[slot].data_ptr(), bytes, hipMemcpyHostToDevice, stream()));
    HIP_OK(hipEventRecord(in_ev_[slot], stream()));
    in_used_[slot] = true;
    if (r_->pg()) broadcast_arena();
  }

  void announce(const int32_t* hdr) {
    HIP_OK(hipMemcpyAsync(arena_.data_ptr(), hdr, 16 * sizeof(int32_t), hipMemcpyHostToDevice, stream()));
    broadcast_arena();
  }

  void broadcast_arena() {
    std::vector<at::Tensor> t{arena_};
    c10d::BroadcastOptions o;
    o.rootRank = 0;
    r_->pg()->broadcast(t, o)->wait();
  }

  // The step body shared by eager launches and graph capture.
  void body(int64_t T, int64_t nd, int64_t nps, int64_t ntiles, int64_t nrows, bool rows_all, int64_t ntop) {
    const int32_t* dh = reinterpret_cast<const int32_t*>(arena_.data_ptr());
    at::Tensor ids = view<int32_t>("ids", T, at::kInt);
    gather_feedback_kernel<<<(int)std::max<int64_t>(1, (maxS_ + 255) / 256), 256, 0, stream()>>>(
        ids.data_ptr<int32_t>(), reinterpret_cast<const int64_t*>((char*)arena_.data_ptr() + off_.at("gdst")),
        reinterpret_cast<const int64_t*>((char*)arena_.data_ptr() + off_.at("gsrc")), tok_.data_ptr<int32_t>(), dh,
        (int)maxS_);
    at::Tensor pos = view<int32_t>("pos", T, at::kInt);
    at::Tensor slots = view<int64_t>("slots", T, at::kLong);
    at::Tensor dbt = view<int32_t>("dbt", std::max<int64_t>(nd, 1) * maxB_, at::kInt).view({-1, maxB_});
    at::Tensor dctx = view<int32_t>("dctx", std::max<int64_t>(nd, 1), at::kInt);
    at::Tensor pbt = view<int32_t>("pbt", std::max<int64_t>(nps, 1) * maxB_, at::kInt).view({-1, maxB_});
    at::Tensor qs = view<int32_t>("q_start", std::max<int64_t>(nps, 1), at::kInt);
    at::Tensor ql = view<int32_t>("q_len", std::max<int64_t>(nps, 1), at::kInt);
    at::Tensor cl = view<int32_t>("ctx_len", std::max<int64_t>(nps, 1), at::kInt);
    at::Tensor tiles = view<int32_t>("tiles", std::max<int64_t>(ntiles, 1) * 2, at::kInt).view({-1, 2});
    c10::optional<at::Tensor> rows;
    if (!rows_all) rows = view<int64_t>("rows", nrows, at::kLong);
    const bool tp = (bool)r_->pg();
    at::Tensor logits = r_->forward_impl(ids, pos, slots, nd, dbt, dctx, nsplit_, std::min(bps_, maxB_), ws_,
                                         T - nd, pbt, qs, ql, cl, tiles, rows, /*gather_logits=*/!tp);
    last_logits_ = logits;
    if (nrows == 0) return;
    const int V = (int)logits.size(1);
    logit_delta_kernel<<<(int)std::max<int64_t>(1, std::min<int64_t>((maxD_ + 255) / 256, 1024)), 256, 0,
                         stream()>>>(logits.data_ptr<float>(), logits.stride(0), V, (int)logits.size(0),
                                     reinterpret_cast<const int32_t*>((char*)arena_.data_ptr() + off_.at("deltas")),
                                     dh, (int)maxD_, tp ? (int)r_->vocab_start() : 0);
    at::Tensor lg = logits.narrow(0, 0, nrows);
    at::Tensor temp = view<float>("temp", nrows, at::kFloat), topk = view<int32_t>("top_k", nrows, at::kInt);
    at::Tensor topp = view<float>("top_p", nrows, at::kFloat), seeds = view<int64_t>("seeds", nrows, at::kLong);
    at::Tensor steps = view<int64_t>("steps", nrows, at::kLong);
    if (!tp) {
      sample_tokens(lg, temp, topk, topp, seeds, steps, tok_, lp_, ti_, tl_, ntop);
      return;
    }
    sample_vocab_parallel(lg, temp, topk, topp, seeds, steps, nrows, ntop);
  }

  // Vocab-parallel sampling: four tp_sample_* phases with an all-gather of [R, 4] row
  // statistics, an all-reduce of the [R, 2, 1024] top-k/top-p histograms and an
  // all-gather of [R, 3 + 2 n] candidates, instead of all-gathering f32 logit rows
  // ([R, vocab] x 4 B: 128 MiB per step at R = 256 on Llama-3).  Same tokens as the
  // single-GPU sampler on the same logits (sampling.hip).
  void sample_vocab_parallel(const at::Tensor& lg, const at::Tensor& temp, const at::Tensor& topk,
                             const at::Tensor& topp, const at::Tensor& seeds, const at::Tensor& steps, int64_t R,
                             int64_t ntop) {
    const int64_t W = r_->pg()->getSize(), cw = 3 + 2 * ntop;
    auto gather = [&](const at::Tensor& src, const at::Tensor& dst, int64_t per) {
      r_->allgather32(src.narrow(0, 0, per), dst);
    };
    at::Tensor stats = tp_stats_.narrow(0, 0, R * 4), stats_all = tp_stats_all_.narrow(0, 0, W * R * 4);
    tp_sample_stats(lg, r_->vocab_start(), stats);
    gather(tp_stats_, stats_all, R * 4);
    at::Tensor hist = tp_hist_.narrow(0, 0, R * 2 * 1024);
    tp_sample_hist(lg, r_->vocab(), temp, topk, topp, stats_all, W, hist);
    r_->allreduce_i64(hist);
    at::Tensor cand_all = tp_cand_all_.narrow(0, 0, W * R * cw);
    tp_sample_pick(lg, r_->vocab_start(), r_->vocab(), temp, topk, topp, seeds, steps, stats_all, W, hist, ntop,
                   tp_cand_);
    gather(tp_cand_, cand_all, R * cw);
    tp_sample_final(stats_all, cand_all, W, R, temp, ntop, tok_, lp_, ti_, tl_);
  }

  void run(const int32_t* h) {
    if (h[H_NCOPY] > 0)
      r_->copy_kv_blocks(reinterpret_cast<const int32_t*>((char*)arena_.data_ptr() + off_.at("kvcopy")), h[H_NCOPY]);
    const int64_t B = h[H_BUCKET];
    if (B > 0) {
      auto it = graphs_.find(B);
      TORCH_CHECK(it != graphs_.end(), "decode graph for bucket ", B, " was not captured");
      if (it->second) {
        it->second->replay();
        return;
      }
    }
    body(h[H_T], h[H_ND], h[H_NPS], h[H_NTILES], h[H_NROWS], h[H_ROWS_ALL] != 0, h[H_NTOP]);
  }

  void download(const int32_t* h, int64_t oslot) {
    const int64_t n = h[H_NROWS], ntop = h[H_NTOP];
    char* o = (char*)out_.at(oslot).data_ptr();
    if (n > 0) {
      HIP_OK(hipMemcpyAsync(o, tok_.data_ptr(), n * 4, hipMemcpyDeviceToHost, stream()));
      HIP_OK(hipMemcpyAsync(o + maxS_ * 4, lp_.data_ptr(), n * 4, hipMemcpyDeviceToHost, stream()));
      if (ntop > 0) {
        HIP_OK(hipMemcpyAsync(o + maxS_ * 8, ti_.data_ptr(), n * ntop * 4, hipMemcpyDeviceToHost, stream()));
        HIP_OK(hipMemcpyAsync(o + maxS_ * 8 + maxS_ * kMaxTop * 4, tl_.data_ptr(), n * ntop * 4,
                              hipMemcpyDeviceToHost, stream()));
      }
    }
    copy_status(st_host_[oslot].data_ptr<int>());
    HIP_OK(hipEventRecord(out_ev_[oslot], stream()));
  }

  // status words (LlamaRunner::status_ptrs) -> pinned host ints, in stream order after the step
  void copy_status(int* dst) {
    for (size_t k = 0; k < status_ptrs_.size(); ++k)
      HIP_OK(hipMemcpyAsync(dst + k, status_ptrs_[k], sizeof(int), hipMemcpyDeviceToHost, stream()));
  }
  void check_status(const int* st) {
    if (st[1] != 0) {
      // per step, like [0] below: clear and report once
      HIP_OK(hipMemsetAsync(const_cast<int*>(status_ptrs_[1]), 0, sizeof(int), stream()));
      TORCH_CHECK(false, "decode GEMM: a split-K combine rendezvous timed out (a K-slice workgroup never "
                  "arrived); this step's results are invalid");
    }
    if (st[0] != 0) {
      // the gate_up exchange word is per step: clear it (in stream order, after this
      // step) so the failed step is reported once and later steps run normally -- the
      // exchange's monotonic tickets stay consistent after a timeout.  The one-shot
      // all-reduce words below stay sticky: a peer that never arrived desynchronises
      // its epochs for good.
      if (!status_ptrs_.empty())
        HIP_OK(hipMemsetAsync(const_cast<int*>(status_ptrs_[0]), 0, sizeof(int), stream()));
      TORCH_CHECK(false, "decode GEMM: the gate_up K-half exchange timed out (partner workgroup never "
                  "published); this step's results are invalid");
    }
    for (int k = 2; k < kStatusWords; ++k)
      TORCH_CHECK(st[k] == 0, "one-shot all-reduce timed out: a tensor-parallel peer never arrived; this step's "
                  "results are invalid");
  }

  // Neutral inputs for graph warm-up: no KV writes (slot -1), empty contexts, no feedback.
  void neutralise(int64_t B) {
    char* base = (char*)arena_.data_ptr();
    hipStream_t s = stream();
    HIP_OK(hipMemsetAsync(base + off_.at("hdr"), 0, 16 * 4, s));
    HIP_OK(hipMemsetAsync(base + off_.at("ids"), 0, B * 4, s));
    HIP_OK(hipMemsetAsync(base + off_.at("pos"), 0, B * 4, s));
    HIP_OK(hipMemsetAsync(base + off_.at("slots"), 0xFF, B * 8, s));
    HIP_OK(hipMemsetAsync(base + off_.at("dbt"), 0, B * maxB_ * 4, s));
    HIP_OK(hipMemsetAsync(base + off_.at("dctx"), 0, B * 4, s));
    HIP_OK(hipMemsetAsync(base + off_.at("temp"), 0, B * 4, s));
    HIP_OK(hipMemsetAsync(base + off_.at("top_k"), 0, B * 4, s));
    HIP_OK(hipMemsetAsync(base + off_.at("seeds"), 0, B * 8, s));
    HIP_OK(hipMemsetAsync(base + off_.at("steps"), 0, B * 8, s));
    std::vector<float> ones(B, 1.0f);
    HIP_OK(hipMemcpy(base + off_.at("top_p"), ones.data(), B * 4, hipMemcpyHostToDevice));
  }

  void do_capture(int64_t B) {
    TORCH_CHECK(B > 0 && B <= maxS_, "bad graph bucket ", B);
    if (graphs_.count(B)) return;
    if (!use_graphs_) {
      graphs_.emplace(B, nullptr);
      return;
    }
    auto cur = at::hip::getCurrentHIPStreamMasqueradingAsCUDA();
    neutralise(B);
    HIP_OK(hipStreamSynchronize(cur.stream()));
    auto side = at::hip::getStreamFromPoolMasqueradingAsCUDA();
    auto g = std::make_unique<at::cuda::CUDAGraph>();
    {
      at::hip::HIPStreamGuardMasqueradingAsCUDA guard(side);
      for (int i = 0; i < 2; ++i) body(B, B, 0, 0, B, true, 0);  // allocator + hipBLASLt warm-up
      HIP_OK(hipStreamSynchronize(side.stream()));
      g->capture_begin(pool_);
      body(B, B, 0, 0, B, true, 0);
      g->capture_end();
    }
    HIP_OK(hipStreamSynchronize(side.stream()));
    graph_logits_[B] = last_logits_;
    graphs_.emplace(B, std::move(g));
  }

  std::shared_ptr<LlamaRunner> r_;
  std::map<std::string, int64_t> off_;
  int64_t arena_bytes_, fixed_bytes_, maxT_, maxS_, maxB_, maxTiles_, maxD_, nsplit_, bps_;
  bool use_graphs_;
  std::vector<at::Tensor> host_, out_;
  std::vector<hipEvent_t> in_ev_, out_ev_;
  static constexpr int kStatusWords = 4;
  std::vector<const int*> status_ptrs_;
  at::Tensor st_host_;
  std::vector<bool> in_used_;
  at::Tensor arena_, hdr_small_, tok_, lp_, ti_, tl_, ws_, last_logits_;
  at::Tensor tp_stats_, tp_stats_all_, tp_hist_, tp_cand_, tp_cand_all_;
  std::map<int64_t, std::unique_ptr<at::cuda::CUDAGraph>> graphs_;
  // launcher thread state (guarded by mu_): jobs in issue order, per-slot job index
  std::thread launcher_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<int64_t> jobs_;
  std::vector<int64_t> slot_job_;
  int64_t issued_ = 0, done_ = 0;
  bool stop_ = false;
  std::exception_ptr err_;
  c10::optional<at::hip::HIPStreamMasqueradingAsCUDA> stream_;
  std::map<int64_t, at::Tensor> graph_logits_;
  at::cuda::MempoolId_t pool_;
  double t_up_ = 0, t_run_ = 0, t_down_ = 0, t_wait_ = 0;
};

}  // namespace

void bind_runners(py::module_& m) {
  m.def("set_pgemm_route", &pgemm_route::set, "prefill routing table: use_pp[b] for M in [256 b - 128, 256 b + 128)");
  m.def("pgemm_route_uses_pp", &pgemm_route::use_pp);
  py::class_<LlamaRunner, std::shared_ptr<LlamaRunner>>(m, "LlamaRunner")
      .def(py::init<at::Tensor, std::vector<at::Tensor>, std::vector<at::Tensor>, std::vector<at::Tensor>,
                    std::vector<at::Tensor>, std::vector<at::Tensor>, std::vector<at::Tensor>, at::Tensor, at::Tensor,
                    std::vector<at::Tensor>, std::vector<at::Tensor>, at::Tensor, int64_t, int64_t, int64_t, double,
                    double, int64_t, int64_t, py::object>())
      .def("forward", &LlamaRunner::forward, py::call_guard<py::gil_scoped_release>());
  py::class_<BertRunner>(m, "BertRunner")
      .def(py::init<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, std::vector<std::vector<at::Tensor>>,
                    int64_t, double, double, int64_t, bool, std::vector<std::vector<at::Tensor>>>())
      .def("forward", &BertRunner::forward, py::call_guard<py::gil_scoped_release>());
  py::class_<StepExecutor>(m, "StepExecutor")
      .def(py::init<std::shared_ptr<LlamaRunner>, std::map<std::string, int64_t>, int64_t, int64_t, int64_t,
                    int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, bool, int64_t>())
      .def("host_slot", &StepExecutor::host_slot)
      .def("out_slot", &StepExecutor::out_slot)
      .def("has_graph", &StepExecutor::has_graph)
      .def("wait_in", &StepExecutor::wait_in, py::call_guard<py::gil_scoped_release>())
      .def("wait_out", &StepExecutor::wait_out, py::call_guard<py::gil_scoped_release>())
      .def("launch", &StepExecutor::launch_sync, py::call_guard<py::gil_scoped_release>())
      .def("step", &StepExecutor::step, py::call_guard<py::gil_scoped_release>())
      .def("timings", &StepExecutor::timings)
      .def("capture", &StepExecutor::capture, py::call_guard<py::gil_scoped_release>())
      .def("shutdown", &StepExecutor::shutdown, py::call_guard<py::gil_scoped_release>())
      .def("worker_loop", &StepExecutor::worker_loop, py::call_guard<py::gil_scoped_release>());
}
