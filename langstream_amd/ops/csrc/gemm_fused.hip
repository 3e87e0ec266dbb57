// General-M MFMA GEMM with fused epilogues for gfx950:  C[M, N] = X[M, K] . W[N, K]^T
// (the nn.Linear layout: both operands K-contiguous), built for the embedding encoder
// (bge-small QKV [T,384]x[384,1152], O [T,384]x[384,384], FFN1
// [T,384]x[384,1536], FFN2 [T,1536]x[1536,384]) where the library path pays a separate
// bias / GELU / residual+LayerNorm pass after every GEMM.
//
// Main loop: the glds ring of gemm_skinny.hip generalised to any M -- BM(M) x 128(N)
// workgroup tiles, one wave per 64 x 64 sub-tile (4 x 4 MFMA 16x16x32 accumulators),
// both operands global -> LDS by global_load_lds_dwordx4 into an S-deep ring of 32-deep
// K stages (64-B rows, source-side bank swizzle), one raw s_barrier per K step behind a
// counted vmcnt, XCD-aware tile order (the M tiles of one W tile share an L2).
//
// LayerNorm folded into the neighbouring GEMMs (no normalisation pass at all): a GEMM
// whose output feeds a LayerNorm stores the UN-normalised row v (bias + residual added)
// plus per-row partial statistics (sum v, sum v^2 over each 64-column sub-tile, from the
// bf16-rounded values).  Its consumers finish the statistics (mean, rstd) per row in
// their prologue and apply the LayerNorm algebraically:
//   * as the INPUT of the next GEMM:  LN(x) . W^T = r (x . W'^T) - r mu c1 + c2, with
//     W' = W * gamma (columns of K), c1 = rowsum(W'), c2 = W . beta precomputed at load
//     time (flag LNIN; the GEMM streams the un-normalised x);
//   * as the RESIDUAL of the next residual add: (res - mu) r gamma + beta, elementwise
//     in the epilogue (flag RESLN).
// Epilogue order: v = acc; LNIN: v = r (v - mu c1) + c2; BIAS: v += b; GELU (erf);
// RES: v += res [normalised when RESLN]; store bf16; STATS: per-row partial sums.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

constexpr int BN = 128;
constexpr int GBK = 32;

enum : int { F_BIAS = 1, F_LNIN = 2, F_GELU = 4, F_RES = 8, F_RESLN = 16, F_STATS = 32 };

struct Epi {
  const bf16* bias;     // [N]
  const float* c1;      // [N]   rowsum of W'            (LNIN)
  const float* c2;      // [N]   W . beta                 (LNIN)
  const float* st_in;   // [M][nts_in][2] partial (sum, sumsq) of the LayerNorm input rows
  int nts_in;
  int n_in;             // LayerNorm row width
  float eps;
  const bf16* res;      // [M, N] residual (row stride ldr)
  int64_t ldr;
  const bf16* g;        // [N] gamma / beta of the residual's LayerNorm (RESLN)
  const bf16* be;
  float* st_out;        // [M][N / 64][2]
};

__device__ __forceinline__ float gelu_erf(float v) { return 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); }

template <int BM, int S, int FL>
__global__ void __launch_bounds__(BM * 2) gemm_fused_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                            const bf16* __restrict__ w, int M, int N, int K,
                                                            bf16* __restrict__ out, int64_t ldo, int MT, Epi e) {
  constexpr int NW = BM / 32;                 // waves (BM/64 x 2)
  constexpr int XB = BM * GBK * 2, WB = BN * GBK * 2, SB = XB + WB;
  constexpr int XPW = BM / 16 / NW;           // 16-row X pieces per wave (= 2)
  constexpr int WPW = 8 / NW;                 // 16-row W pieces per wave
  constexpr int PER = XPW + WPW;              // LDS-DMA instructions per wave per stage
  static_assert(XPW * NW * 16 == BM && WPW * NW == 8, "piece split");
  constexpr int LDS_BYTES = S * SB > BM * 8 ? S * SB : BM * 8;
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = logical % MT, nt = logical / MT;
  const int m0 = mt * BM;
  const int nk = K / GBK;

  const int prow = lane >> 2;
  const int sck = ((lane & 3) ^ swz_g(lane >> 4)) * 8;
  const bf16* xs[XPW];
#pragma unroll
  for (int j = 0; j < XPW; ++j) {
    const int row = 16 * (wid * XPW + j) + prow;
    xs[j] = x + (int64_t)min(m0 + row, M - 1) * ldx + sck;   // rows >= M: any valid row, never stored
  }
  const bf16* wsrc[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) wsrc[j] = w + (int64_t)(nt * BN + 16 * (wid * WPW + j) + prow) * K + sck;
  auto issue = [&](int kt, int buf) {
    const int ko = kt * GBK;
    char* base = lds + buf * SB;
#pragma unroll
    for (int j = 0; j < XPW; ++j) glds16(xs[j] + ko, base + (wid * XPW + j) * 1024);
#pragma unroll
    for (int j = 0; j < WPW; ++j) glds16(wsrc[j] + ko, base + XB + (wid * WPW + j) * 1024);
  };

  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, h = lane >> 4;
  const int swz = 16 * (h ^ swz_g(fr >> 2));
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(min(s, nk - 1), s);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    wait_vmcnt<(S - 2) * PER>();          // this wave's DMA of stage kt has landed
    __builtin_amdgcn_s_barrier();         // ... and every other wave's; step kt-1's reads are done
    int nb = buf + S - 1;
    if (nb >= S) nb -= S;
    issue(min(kt + S - 1, nk - 1), nb);
    const char* lx = lds + buf * SB;
    const char* lw = lx + XB;
    bf16x8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = __builtin_bit_cast(bf16x8, ld16(lx + (64 * wm + 16 * i + fr) * 64 + swz));
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = __builtin_bit_cast(bf16x8, ld16(lw + (64 * wn + 16 * j + fr) * 64 + swz));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    buf = buf + 1 == S ? 0 : buf + 1;
  }
  wait_vmcnt<0>();  // no LDS-DMA may outlive the main loop
  __syncthreads();  // every wave is done reading the ring: reuse it for the row statistics

  // (mean, rstd) of this tile's rows from the partial statistics of the LayerNorm input
  float* rowst = reinterpret_cast<float*>(lds);
  if constexpr ((FL & (F_LNIN | F_RESLN)) != 0) {
    for (int r = threadIdx.x; r < BM; r += BM * 2) {
      const int m = min(m0 + r, M - 1);
      const float* p = e.st_in + (int64_t)m * e.nts_in * 2;
      float s = 0.f, ss = 0.f;
      for (int t = 0; t < e.nts_in; ++t) { s += p[2 * t]; ss += p[2 * t + 1]; }
      const float mu = s / e.n_in;
      const float var = fmaxf(ss / e.n_in - mu * mu, 0.f);
      rowst[2 * r] = mu;
      rowst[2 * r + 1] = rsqrtf(var + e.eps);
    }
    __syncthreads();
  }

  // per-column constants of this lane's 4 columns
  float cb[4] = {0.f, 0.f, 0.f, 0.f}, cc1[4] = {0.f, 0.f, 0.f, 0.f}, cc2[4] = {0.f, 0.f, 0.f, 0.f};
  float cg[4] = {1.f, 1.f, 1.f, 1.f}, cbe[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nt * BN + 64 * wn + 16 * j + fr;
    if constexpr ((FL & F_BIAS) != 0) cb[j] = (float)e.bias[n];
    if constexpr ((FL & F_LNIN) != 0) { cc1[j] = e.c1[n]; cc2[j] = e.c2[n]; }
    if constexpr ((FL & F_RESLN) != 0) { cg[j] = (float)e.g[n]; cbe[j] = (float)e.be[n]; }
  }
  const int rbase = 64 * wm + 4 * h;
  const int nts_out = N / 64;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = rbase + 16 * i + r;
      const int m = m0 + lr;
      float mu = 0.f, rs = 1.f;
      if constexpr ((FL & (F_LNIN | F_RESLN)) != 0) { mu = rowst[2 * lr]; rs = rowst[2 * lr + 1]; }
      float s = 0.f, ss = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nt * BN + 64 * wn + 16 * j + fr;
        float v = acc[i][j][r];
        if constexpr ((FL & F_LNIN) != 0) v = rs * (v - mu * cc1[j]) + cc2[j];
        v += cb[j];
        if constexpr ((FL & F_GELU) != 0) v = gelu_erf(v);
        if constexpr ((FL & F_RES) != 0) {
          if (m < M) {
            float rv = (float)e.res[(int64_t)m * e.ldr + n];
            if constexpr ((FL & F_RESLN) != 0) rv = (rv - mu) * rs * cg[j] + cbe[j];
            v += rv;
          }
        }
        const bf16 o = (bf16)v;
        if (m < M) out[(int64_t)m * ldo + n] = o;
        const float vr = (float)o;
        s += vr;
        ss += vr * vr;
      }
      if constexpr ((FL & F_STATS) != 0) {
        // reduce over the 16 lanes (columns) that share this row
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s += __shfl_xor(s, o, 64);
          ss += __shfl_xor(ss, o, 64);
        }
        if (fr == 0 && m < M) {
          float* p = e.st_out + ((int64_t)m * nts_out + nt * 2 + wn) * 2;
          p[0] = s;
          p[1] = ss;
        }
      }
    }
}

// ring depth: the LDS ring bounds workgroups per CU (BM=256: 24 KB per stage), so a short
// K (encoder: 12-48 stages) runs a 3-deep ring at 2 workgroups per CU, overlapping one
// workgroup's prologue / epilogue with another's main loop; LS_GEMM_RING overrides.
int ring_depth(int bm, int nk) {
  static const int env = [] {
    const char* v = getenv("LS_GEMM_RING");
    return v ? atoi(v) : 0;
  }();
  if (env == 3 || env == 4 || env == 6) return env;
  if (bm == 256) return nk <= 48 ? 3 : 6;
  return nk <= 48 ? 3 : 4;
}

template <int FL>
void launch_fl(int bm, dim3 grid, hipStream_t st, const at::Tensor& x, const at::Tensor& w, int M, int N, int K,
               at::Tensor& out, int MT, const Epi& e) {
#define L(BMV, SV)                                                                                            \
  gemm_fused_kernel<BMV, SV, FL><<<grid, BMV * 2, 0, st>>>((const bf16*)x.data_ptr(), x.stride(0),            \
                                                          (const bf16*)w.data_ptr(), M, N, K,                 \
                                                          (bf16*)out.data_ptr(), out.stride(0), MT, e)
#define LS(BMV)                      \
  switch (ring_depth(BMV, K / GBK)) { \
    case 3: L(BMV, 3); break;        \
    case 4: L(BMV, 4); break;        \
    default: L(BMV, 6); break;       \
  }
  if (bm == 64) { LS(64) }
  else if (bm == 128) { LS(128) }
  else { LS(256) }
#undef LS
#undef L
}

void launch(int flags, int bm, dim3 grid, hipStream_t st, const at::Tensor& x, const at::Tensor& w, int M, int N,
            int K, at::Tensor& out, int MT, const Epi& e) {
  switch (flags) {
#define C(F) case F: launch_fl<F>(bm, grid, st, x, w, M, N, K, out, MT, e); break;
    C(0)
    C(F_BIAS)
    C(F_BIAS | F_GELU)
    C(F_BIAS | F_RES)
    C(F_BIAS | F_RES | F_STATS)
    C(F_BIAS | F_RES | F_RESLN | F_STATS)
    C(F_LNIN | F_BIAS)
    C(F_LNIN | F_BIAS | F_GELU)
    C(F_RES)
    C(F_RES | F_STATS)
#undef C
    default: TORCH_CHECK(false, "unsupported gemm_fused epilogue flags ", flags);
  }
}

}  // namespace

// out[M, N] = epilogue(x[M, K] . w[N, K]^T).  Optional tensors select the epilogue:
//   bias [N]; ln_stats_in [M, T, 2] f32 partial (sum, sumsq) rows of the LayerNorm input
//   (width ln_width) with c1/c2 [N] f32 -> LNIN, or with res_g/res_b [N] -> RESLN;
//   gelu; residual [M, N]; stats_out [M, N/64, 2] f32.
void gemm_fused(at::Tensor out, at::Tensor x, at::Tensor w, c10::optional<at::Tensor> bias, bool gelu,
                c10::optional<at::Tensor> residual, c10::optional<at::Tensor> ln_stats_in, int64_t ln_width,
                c10::optional<at::Tensor> c1, c10::optional<at::Tensor> c2, c10::optional<at::Tensor> res_g,
                c10::optional<at::Tensor> res_b, double eps, c10::optional<at::Tensor> stats_out) {
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x must be [M, K] with unit column stride");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) == K, "w must be contiguous [N, K]");
  TORCH_CHECK(K % GBK == 0 && N % BN == 0, "gemm_fused needs K % 32 == 0 and N % 128 == 0");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.dim() == 2 && out.size(0) == M && out.size(1) == N &&
              out.stride(1) == 1);
  TORCH_CHECK(M < (1LL << 31) / 256);
  Epi e{};
  int flags = 0;
  auto f32n = [&](const c10::optional<at::Tensor>& t, const char* what) {
    TORCH_CHECK(t.has_value() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == N, what,
                " must be f32 [N]");
    return t->data_ptr<float>();
  };
  auto bf16n = [&](const c10::optional<at::Tensor>& t, const char* what) {
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->numel() == N, what, " must be bf16 [N]");
    return (const bf16*)t->data_ptr();
  };
  if (bias.has_value()) {
    e.bias = bf16n(bias, "bias");
    flags |= F_BIAS;
  }
  if (gelu) flags |= F_GELU;
  if (residual.has_value()) {
    TORCH_CHECK(residual->scalar_type() == at::kBFloat16 && residual->dim() == 2 && residual->size(0) == M &&
                residual->size(1) == N && residual->stride(1) == 1, "residual must be bf16 [M, N]");
    e.res = (const bf16*)residual->data_ptr();
    e.ldr = residual->stride(0);
    flags |= F_RES;
  }
  if (ln_stats_in.has_value()) {
    TORCH_CHECK(ln_stats_in->scalar_type() == at::kFloat && ln_stats_in->is_contiguous() && ln_stats_in->dim() == 3 &&
                ln_stats_in->size(0) == M && ln_stats_in->size(2) == 2, "ln_stats_in must be f32 [M, T, 2]");
    e.st_in = ln_stats_in->data_ptr<float>();
    e.nts_in = (int)ln_stats_in->size(1);
    e.n_in = (int)ln_width;
    e.eps = (float)eps;
    TORCH_CHECK(ln_width > 0);
    if (res_g.has_value()) {
      TORCH_CHECK(residual.has_value() && res_b.has_value(), "RESLN needs residual, res_g and res_b");
      e.g = bf16n(res_g, "res_g");
      e.be = bf16n(res_b, "res_b");
      flags |= F_RESLN;
    } else {
      e.c1 = f32n(c1, "c1");
      e.c2 = f32n(c2, "c2");
      flags |= F_LNIN;
    }
  }
  if (stats_out.has_value()) {
    TORCH_CHECK(stats_out->scalar_type() == at::kFloat && stats_out->is_contiguous() &&
                stats_out->numel() == M * (N / 64) * 2, "stats_out must be f32 [M, N/64, 2]");
    e.st_out = stats_out->data_ptr<float>();
    flags |= F_STATS;
  }
  if (M == 0) return;
  // tile height: the tallest that still gives >= ~1 workgroup per CU
  const int64_t NT = N / BN;
  int bm = 256;
  while (bm > 64 && ((M + bm - 1) / bm) * NT < 256) bm /= 2;
  const int MT = (int)((M + bm - 1) / bm);
  auto stream = at::hip::getCurrentHIPStream();
  launch(flags, bm, dim3((unsigned)(MT * NT)), stream, x, w, (int)M, (int)N, (int)K, out, MT, e);
}
