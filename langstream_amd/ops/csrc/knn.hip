// Brute-force k-nearest-neighbour search for the local vector store
// (query-vector-db / `ORDER BY cosine_similarity(...) DESC LIMIT k`).
//
// Stage 1 (fused GEMM + chunk top-k): grid = N/1024 row chunks x ceil(Q/16) query
// groups, flattened and XCD-remapped (groups of a chunk share an XCD's L2).  Each wave streams 256 store rows through mfma_f32_16x16x32_bf16 as the
// A operand (one 16-B load per lane per MFMA, straight from HBM: the rows are read
// once per query group) against the 16 queries' Q^T fragments held in LDS.  Scores
// for the 1024 x 16 block go to LDS; each wave then extracts the top-k of 4 queries
// by k rounds of wave-argmax (k <= 64), writing (score, row) candidates.
// Stage 2: one workgroup per query selects the global top-k from all chunk
// candidates (k rounds of block-argmax over an L2-resident candidate list).
//
// Scores are raw dot products; the store keeps rows L2-normalised so this is
// cosine similarity.  Rows >= N (tail chunk) score -inf.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

constexpr int CH = 1024;  // store rows per workgroup
constexpr int QG = 16;    // queries per workgroup (one MFMA column group)

// Bitonic sort of one (value, index) pair per lane across a 64-wide wave, descending by
// value with ties broken towards the lower index (the order the argmax path produces):
// afterwards lane L holds the L-th largest.  6*7/2 = 21 xor-shuffle compare-exchanges.
__device__ __forceinline__ void wave_sort_desc(float& v, int& i, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const float ov = __shfl_xor(v, j, 64);
      const int oi = __shfl_xor(i, j, 64);
      const bool other_first = ov > v || (ov == v && oi < i);
      // descending blocks where (lane & k) == 0; the lower lane of a pair keeps the "first"
      const bool lower = (lane & j) == 0;
      const bool desc = (lane & k) == 0;
      const bool take = (lower == desc) ? other_first : !other_first;
      if (take) { v = ov; i = oi; }
    }
  }
}

template <int DIM>
__global__ void __launch_bounds__(256) knn_stage1_kernel(const bf16* __restrict__ X, int64_t N,
                                                         const bf16* __restrict__ Qm, int Qn, int K,
                                                         float* __restrict__ cand_s, int32_t* __restrict__ cand_i,
                                                         int nchunks) {
  constexpr int KS = DIM / 32;
  __shared__ __attribute__((aligned(16))) bf16 q_lds[QG * DIM];
  __shared__ float sc[QG][CH + 1];
  // 1-D grid, XCD-aware: the query groups of one row chunk are consecutive logical ids
  // on one XCD, so the chunk's rows come from HBM once and from that XCD's L2 after
  // (with grid (chunks, groups) every group re-streamed the whole store from HBM).
  const int nqg = gridDim.x / nchunks;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = logical / nqg, qg = logical - chunk * nqg;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, h = lane >> 4;
  // stage the 16 queries (zero rows past Qn)
  for (int c = threadIdx.x; c < QG * DIM / 8; c += 256) {
    const int qq = c / (DIM / 8), cc = c - qq * (DIM / 8);
    const int qi = qg * QG + qq;
    *reinterpret_cast<uint4*>(&q_lds[qq * DIM + cc * 8]) =
        qi < Qn ? ld16(Qm + (int64_t)qi * DIM + cc * 8) : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  const int64_t row0 = (int64_t)chunk * CH + wid * 256;
  for (int st = 0; st < 16; ++st) {
    const int64_t r = row0 + st * 16 + i16;
    const bool valid = r < N;
    const bf16* xr = X + (valid ? r : 0) * DIM + 8 * h;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 a = __builtin_bit_cast(bf16x8, ld16(xr + 32 * ks));
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(&q_lds[i16 * DIM + 32 * ks + 8 * h]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
    // acc[rr] = score(row 4h+rr of the subtile, query i16)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int lr = wid * 256 + st * 16 + 4 * h + rr;
      const bool ok = row0 + st * 16 + 4 * h + rr < N;
      sc[i16][lr] = ok ? acc[rr] : -INFINITY;
    }
  }
  __syncthreads();
  // top-K per query: wave w handles queries w, w+4, w+8, w+12.
  // Fast path (threshold + sort): every lane holds 16 of the 1024 scores in registers;
  // the K-th largest of the 64 lane maxima, T, lower-bounds the K-th largest score (the
  // K lanes owning those maxima each hold a score >= T), so only scores >= T can be in
  // the top-K.  They are compacted by ballot into a 64-slot LDS list and bitonic-sorted
  // across the wave (21 shuffle stages) -- instead of K rounds of a 1024-wide argmax.
  // When more than 64 scores reach T (heavy ties, or a tail chunk where T = -inf) the
  // wave falls back to the K-round argmax over LDS.
  __shared__ float cv_lds[4][64];
  __shared__ int ci_lds[4][64];
  for (int qq = wid; qq < QG; qq += 4) {
    const int qi = qg * QG + qq;
    if (qi >= Qn) continue;
    float* outs = cand_s + ((int64_t)qi * nchunks + chunk) * K;
    int32_t* outi = cand_i + ((int64_t)qi * nchunks + chunk) * K;
    float v[CH / 64];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < CH / 64; ++j) {
      v[j] = sc[qq][lane + 64 * j];
      m = fmaxf(m, v[j]);
    }
    float tv = m;
    int ti = lane;
    wave_sort_desc(tv, ti, lane);
    const float T = __shfl(tv, K - 1, 64);
    int count = 0;
    if (T > -INFINITY) {
#pragma unroll
      for (int j = 0; j < CH / 64; ++j) {
        const bool p = v[j] >= T;
        const uint64_t mask = __ballot(p);
        const int pos = count + __popcll(mask & ((1ull << lane) - 1ull));
        if (p && pos < 64) {
          cv_lds[wid][pos] = v[j];
          ci_lds[wid][pos] = lane + 64 * j;
        }
        count += __popcll(mask);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (T > -INFINITY && count <= 64) {
      float cvv = lane < count ? cv_lds[wid][lane] : -INFINITY;
      int cii = lane < count ? ci_lds[wid][lane] : CH;
      wave_sort_desc(cvv, cii, lane);
      if (lane < K) {
        outs[lane] = cvv;
        outi[lane] = cii < CH ? (int32_t)((int64_t)chunk * CH + cii) : -1;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      continue;
    }
    for (int k = 0; k < K; ++k) {
      float bv = -INFINITY;
      int bi = CH;
      for (int j = lane; j < CH; j += 64) {
        const float v = sc[qq][j];
        if (v > bv) { bv = v; bi = j; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      if (lane == 0) {
        outs[k] = bv;
        outi[k] = bi < CH ? (int32_t)((int64_t)chunk * CH + bi) : -1;
        if (bi < CH) sc[qq][bi] = -INFINITY;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

__global__ void __launch_bounds__(256) knn_stage2_kernel(float* __restrict__ cand_s, const int32_t* __restrict__ cand_i,
                                                         int ncand, int K, float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_i) {
  __shared__ float rv[4];
  __shared__ int ri[4];
  const int qi = blockIdx.x;
  float* cs = cand_s + (int64_t)qi * ncand;
  const int32_t* ci = cand_i + (int64_t)qi * ncand;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int k = 0; k < K; ++k) {
    float bv = -INFINITY;
    int bi = ncand;
    for (int j = threadIdx.x; j < ncand; j += 256) {
      const float v = cs[j];
      if (v > bv) { bv = v; bi = j; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { rv[wid] = bv; ri[wid] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float b = rv[0];
      int bb = ri[0];
      for (int w = 1; w < 4; ++w)
        if (rv[w] > b || (rv[w] == b && ri[w] < bb)) { b = rv[w]; bb = ri[w]; }
      out_s[(int64_t)qi * K + k] = b;
      out_i[(int64_t)qi * K + k] = bb < ncand ? ci[bb] : -1;
      if (bb < ncand) cs[bb] = -INFINITY;
    }
    __syncthreads();
  }
}

}  // namespace

// X: [N, dim] bf16 (rows L2-normalised), Q: [Qn, dim] bf16.  Returns via out tensors
// the top-K scores (f32 [Qn, K]) and row indices (int32 [Qn, K], -1 if N < K).
// workspace: f32 [Qn * nchunks * K] and int32 same count.
void knn_topk(at::Tensor X, at::Tensor Q, int64_t K, at::Tensor out_s, at::Tensor out_i, at::Tensor ws_s,
              at::Tensor ws_i) {
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 && Q.scalar_type() == at::kBFloat16);
  TORCH_CHECK(X.is_contiguous() && Q.is_contiguous() && X.dim() == 2 && Q.dim() == 2);
  const int dim = X.size(1);
  TORCH_CHECK(Q.size(1) == dim);
  TORCH_CHECK(K >= 1 && K <= 64);
  const int64_t N = X.size(0);
  const int Qn = Q.size(0);
  const int nchunks = (int)((N + CH - 1) / CH);
  TORCH_CHECK(ws_s.numel() >= (int64_t)Qn * nchunks * K && ws_i.numel() >= (int64_t)Qn * nchunks * K);
  TORCH_CHECK(out_s.numel() >= (int64_t)Qn * K && out_i.numel() >= (int64_t)Qn * K);
  if (Qn == 0 || N == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  TORCH_CHECK((int64_t)nchunks * ((Qn + QG - 1) / QG) < (1LL << 31), "kNN grid too large");
  dim3 grid(nchunks * ((Qn + QG - 1) / QG));
#define LAUNCH(DD)                                                                                          \
  knn_stage1_kernel<DD><<<grid, 256, 0, stream>>>((const bf16*)X.data_ptr(), N, (const bf16*)Q.data_ptr(), \
                                                  Qn, (int)K, ws_s.data_ptr<float>(), ws_i.data_ptr<int32_t>(), \
                                                  nchunks)
  switch (dim) {
    case 128: LAUNCH(128); break;
    case 256: LAUNCH(256); break;
    case 384: LAUNCH(384); break;
    case 512: LAUNCH(512); break;
    case 768: LAUNCH(768); break;
    case 1024: LAUNCH(1024); break;
    case 1536: LAUNCH(1536); break;
    case 2048: LAUNCH(2048); break;
    default: TORCH_CHECK(false, "unsupported embedding dim ", dim);
  }
#undef LAUNCH
  knn_stage2_kernel<<<Qn, 256, 0, stream>>>(ws_s.data_ptr<float>(), ws_i.data_ptr<int32_t>(), nchunks * (int)K,
                                            (int)K, out_s.data_ptr<float>(), out_i.data_ptr<int32_t>());
}
