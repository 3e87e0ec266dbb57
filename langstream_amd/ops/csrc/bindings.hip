// Python bindings for the langstream_amd HIP kernels (module `_hip_ops`).
#include <torch/extension.h>

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
void sample_tokens(at::Tensor logits, at::Tensor temperature, at::Tensor top_k, at::Tensor top_p, at::Tensor seeds,
                   at::Tensor steps, at::Tensor out_tok, at::Tensor out_lp, at::Tensor top_ids, at::Tensor top_lps,
                   int64_t n_top);
void apply_logit_deltas(at::Tensor logits, at::Tensor rows, at::Tensor toks, at::Tensor delta);
void pool_embeddings(at::Tensor out, at::Tensor x, at::Tensor start, at::Tensor len, int64_t mode, bool normalize);
void l2_normalize_rows(at::Tensor out, at::Tensor x);
void tp_sample_stats(at::Tensor logits, int64_t vstart, at::Tensor stats);
void tp_sample_hist(at::Tensor logits, int64_t vtot, at::Tensor temperature, at::Tensor top_k, at::Tensor top_p,
                    at::Tensor stats_all, int64_t world, at::Tensor hist);
void tp_sample_pick(at::Tensor logits, int64_t vstart, int64_t vtot, at::Tensor temperature, at::Tensor top_k,
                    at::Tensor top_p, at::Tensor seeds, at::Tensor steps, at::Tensor stats_all, int64_t world,
                    at::Tensor hist_all, int64_t n_top, at::Tensor cand);
void tp_sample_final(at::Tensor stats_all, at::Tensor cand_all, int64_t world, int64_t rows, at::Tensor temperature,
                     int64_t n_top, at::Tensor out_tok, at::Tensor out_lp, at::Tensor top_ids, at::Tensor top_lps);
std::vector<at::Tensor> oneshot_allreduce_sim(std::vector<at::Tensor> inputs, int64_t calls, int64_t stall_rank);
int64_t oneshot_allreduce_selftest(py::object process_group, at::Tensor t);
bool oneshot_flags_uncached(py::object process_group);
std::vector<at::Tensor> oneshot_collectives_selftest(py::object process_group, at::Tensor bf, at::Tensor g32,
                                                     at::Tensor i64, int64_t cap);
std::vector<at::Tensor> oneshot_route_selftest(py::object process_group, at::Tensor g32, at::Tensor i64, int64_t cap);
void knn_topk(at::Tensor X, at::Tensor Q, int64_t K, at::Tensor out_s, at::Tensor out_i, at::Tensor ws_s,
              at::Tensor ws_i, int64_t sample);
void knn_topk_ablate(at::Tensor X, at::Tensor Q, int64_t K, at::Tensor out_s, at::Tensor out_i, at::Tensor ws_s,
                     at::Tensor ws_i, int64_t sample, int64_t abl);
int64_t knn_default_sample();
void skinny_gemm(at::Tensor out, at::Tensor x, at::Tensor w);
void gemv(at::Tensor out, at::Tensor x, at::Tensor w);
bool gemv_supported(const at::Tensor& w, bool silu);
void gemv_silu(at::Tensor out, at::Tensor x, at::Tensor w);
void gemv_add_rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor residual, at::Tensor norm_w,
                      double eps, at::Tensor counter);
void gemv_norm(at::Tensor out, at::Tensor o, at::Tensor res, at::Tensor res_out, at::Tensor norm_w, double eps,
               at::Tensor w);
void gemv_silu_norm(at::Tensor out, at::Tensor o, at::Tensor res, at::Tensor res_out, at::Tensor norm_w, double eps,
                    at::Tensor w);
void gemv_qkv(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots,
              at::Tensor k_cache, at::Tensor v_cache, int64_t Hq, int64_t Hkv, bool apply_rope,
              c10::optional<at::Tensor> o, c10::optional<at::Tensor> res, c10::optional<at::Tensor> res_out,
              c10::optional<at::Tensor> norm_w, double eps);
void skinny_gemm_silu(at::Tensor out, at::Tensor x, at::Tensor w);
void gemm_fused(at::Tensor out, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> bias, bool gelu,
                c10::optional<at::Tensor> residual, c10::optional<at::Tensor> ln_stats_in, int64_t ln_width,
                c10::optional<at::Tensor> c1, c10::optional<at::Tensor> c2, c10::optional<at::Tensor> res_g,
                c10::optional<at::Tensor> res_b, double eps, c10::optional<at::Tensor> stats_out);
void skinny_gemm_add_rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor residual, at::Tensor norm_w,
                             double eps);
void gemm_prefill(at::Tensor out, at::Tensor x, at::Tensor w, bool silu, int64_t variant);
bool gemm_prefill_supported(const at::Tensor& w, bool silu);
void gemm_prefill_f32(at::Tensor out, at::Tensor x, at::Tensor w);
bool gemm_prefill_f32_supported(const at::Tensor& w);
bool decode_gemm_supported(const at::Tensor& w, bool silu);
int64_t decode_gemm_workspace(int64_t M, int64_t N, int64_t K, bool silu);
void decode_gemm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor workspace, c10::optional<at::Tensor> residual,
                 c10::optional<at::Tensor> norm_w, double eps, int64_t bn_force, int64_t splits_force);
void decode_gemm_qkv_rope(at::Tensor qkv, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor pos,
                          at::Tensor cos_sin, at::Tensor slots, at::Tensor k_cache, at::Tensor v_cache, int64_t Hq,
                          int64_t Hkv);
bool decode_gemm_f32_supported(const at::Tensor& w, int64_t M);
void decode_gemm_f32(at::Tensor out, at::Tensor x, at::Tensor w, int64_t bn_force);
void decode_gemm_silu(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor tickets,
                      at::Tensor err, int64_t splits);
void decode_gemm_ablate(at::Tensor x, at::Tensor w, at::Tensor workspace, int64_t abl, int64_t splits,
                        int64_t split_outer);
int64_t decode_gemm_cmb_splits(int64_t N, int64_t K);
void decode_gemm_res(at::Tensor y_out, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor counters,
                     at::Tensor residual, at::Tensor norm_g, at::Tensor sumsq_out, at::Tensor err);
void decode_gemm_qkv_cmb(at::Tensor qkv, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor counters,
                         at::Tensor sumsq_in, double eps, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots,
                         at::Tensor k_cache, at::Tensor v_cache, int64_t Hq, int64_t Hkv, at::Tensor err);
void decode_gemm_silu_r(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor sumsq_in, double eps);
pybind11::dict decode_gemm_launch_counts(bool reset);
void rms_prep(at::Tensor y, at::Tensor sumsq, at::Tensor h, at::Tensor g);
void rows_rms_scale(at::Tensor out, at::Tensor y, at::Tensor sumsq, double eps);
void bind_runners(pybind11::module_& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "langstream_amd CDNA4 (gfx950) kernels";
  m.def("rmsnorm", &rmsnorm);
  m.def("fused_add_rmsnorm", &fused_add_rmsnorm);
  m.def("layernorm", &layernorm);
  m.def("embed_layernorm", &embed_layernorm);
  m.def("silu_and_mul", &silu_and_mul);
  m.def("bias_gelu", &bias_gelu);
  m.def("rope_and_cache", &rope_and_cache);
  m.def("paged_decode_attention", &paged_decode_attention);
  m.def("paged_decode_attention_rope", &paged_decode_attention_rope);
  m.def("paged_prefill_attention", &paged_prefill_attention);
  m.def("varlen_encoder_attention", &varlen_encoder_attention);
  m.def("sample_tokens", &sample_tokens);
  m.def("apply_logit_deltas", &apply_logit_deltas);
  m.def("pool_embeddings", &pool_embeddings);
  m.def("l2_normalize_rows", &l2_normalize_rows);
  m.def("knn_topk", &knn_topk);
  m.def("oneshot_allreduce_sim", &oneshot_allreduce_sim, py::arg("inputs"), py::arg("calls"),
        py::arg("stall_rank") = -1);
  m.def("oneshot_allreduce_selftest", &oneshot_allreduce_selftest);
  m.def("oneshot_flags_uncached", &oneshot_flags_uncached);
  m.def("oneshot_collectives_selftest", &oneshot_collectives_selftest);
  m.def("oneshot_route_selftest", &oneshot_route_selftest);
  m.def("tp_sample_stats", &tp_sample_stats);
  m.def("tp_sample_hist", &tp_sample_hist);
  m.def("tp_sample_pick", &tp_sample_pick);
  m.def("tp_sample_final", &tp_sample_final);
  m.def("knn_default_sample", &knn_default_sample);
  m.def("knn_topk_ablate", &knn_topk_ablate);
  m.def("skinny_gemm", &skinny_gemm);
  m.def("gemv", &gemv);
  m.def("gemv_supported", &gemv_supported);
  m.def("gemv_silu", &gemv_silu);
  m.def("gemv_add_rmsnorm", &gemv_add_rmsnorm);
  m.def("gemv_norm", &gemv_norm);
  m.def("gemv_silu_norm", &gemv_silu_norm);
  m.def("gemv_qkv", &gemv_qkv);
  m.def("skinny_gemm_silu", &skinny_gemm_silu);
  m.def("gemm_fused", &gemm_fused, py::arg("out"), py::arg("x"), py::arg("w"), py::arg("bias") = py::none(),
        py::arg("gelu") = false, py::arg("residual") = py::none(), py::arg("ln_stats_in") = py::none(),
        py::arg("ln_width") = 0, py::arg("c1") = py::none(), py::arg("c2") = py::none(),
        py::arg("res_g") = py::none(), py::arg("res_b") = py::none(), py::arg("eps") = 1e-12,
        py::arg("stats_out") = py::none());
  m.def("skinny_gemm_add_rmsnorm", &skinny_gemm_add_rmsnorm);
  m.def("gemm_prefill", &gemm_prefill, py::arg("out"), py::arg("x"), py::arg("w"), py::arg("silu"), py::arg("variant") = -1);
  m.def("gemm_prefill_supported", &gemm_prefill_supported);
  m.def("gemm_prefill_f32", &gemm_prefill_f32, "out[M, N] (f32) = x . w^T on the ping-pong MFMA kernel");
  m.def("gemm_prefill_f32_supported", &gemm_prefill_f32_supported);
  m.def("decode_gemm_supported", &decode_gemm_supported);
  m.def("decode_gemm_workspace", &decode_gemm_workspace);
  m.def("decode_gemm", &decode_gemm, py::arg("out"), py::arg("x"), py::arg("w"), py::arg("workspace"),
        py::arg("residual") = py::none(), py::arg("norm_w") = py::none(), py::arg("eps") = 1e-5,
        py::arg("bn") = 0, py::arg("splits") = 0);
  m.def("decode_gemm_ablate", &decode_gemm_ablate);
  m.def("decode_gemm_qkv_rope", &decode_gemm_qkv_rope);
  m.def("decode_gemm_f32_supported", &decode_gemm_f32_supported);
  m.def("decode_gemm_f32", &decode_gemm_f32, py::arg("out"), py::arg("x"), py::arg("w"), py::arg("bn") = 0);
  m.def("decode_gemm_silu", &decode_gemm_silu, py::arg("out"), py::arg("x"), py::arg("w"), py::arg("workspace"),
        py::arg("tickets"), py::arg("err"), py::arg("splits") = 0);
  m.def("decode_gemm_cmb_splits", &decode_gemm_cmb_splits);
  m.def("decode_gemm_res", &decode_gemm_res);
  m.def("decode_gemm_qkv_cmb", &decode_gemm_qkv_cmb);
  m.def("decode_gemm_silu_r", &decode_gemm_silu_r);
  m.def("decode_gemm_launch_counts", &decode_gemm_launch_counts, py::arg("reset") = false);
  m.def("rms_prep", &rms_prep);
  m.def("rows_rms_scale", &rows_rms_scale);
  bind_runners(m);
}
