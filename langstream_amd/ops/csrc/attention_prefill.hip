// Flash-style prefill / encoder attention on MFMA (gfx950, mfma_f32_16x16x32_bf16).
//
// Variable-length batches; GQA handled by packing the G query heads of one kv head
// as extra rows (row = token*G + g), so every staged K/V tile is reused by G heads.
//
//  * PAGED=true  (Llama prefill, incl. chunked prefill with a cached prefix):
//      K from k_cache [NB, Hkv, 64, D], V^T from v_cache [NB, Hkv, 8, D, 8] (8-key groups,
//      common.h vt_off), causal.
//  * PAGED=false (BERT encoder): K and V read from the packed QKV projection,
//      bidirectional, keys limited to the sequence (padding-free varlen).
//
// Workgroup = 4 waves x 32 query rows (two 16-row MFMA subtiles per wave), KV tile
// = 64 keys staged in LDS (register-staged: issue the next tile's global loads
// before computing the current one, write LDS after the barrier -- guide T14).
// Scores are computed swapped (S^T = K Q^T) with the K-row permutation described in
// attention_decode.hip, so softmax stats and the P^T operand are lane-local and V^T
// rows are read with ds_read_b128.  LDS images are XOR-swizzled per 16-B chunk so
// both fragment reads are bank-conflict-free (derivation in the comments below).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

constexpr int KVT = 64;   // keys per tile (== KV cache block size)
constexpr int ROWS = 128; // query rows per workgroup
constexpr float LOG2E_P = 1.4426950408889634f;

// K tile: [64 keys][D], 16-B chunk c of row `key` stored at chunk c ^ kswz(key).
// The 16 rows read by one ds_read_b128 lane group are keys base + 8a + b (a,b in 0..3,
// base multiple of 4) -> kswz = b | a<<2 takes 16 distinct values: conflict-free.
template <int D>
__device__ __forceinline__ int kswz(int key) {
  constexpr int NCH = D / 8;
  return ((key & 3) | (((key >> 3) & 3) << 2)) & (NCH - 1);
}
// V^T tile: [D][64 keys] (128-B rows, two rows per 256-B bank row) -> chunk c of row d
// at c ^ ((d>>1)&7): the 8 same-parity rows of a lane group hit 8 distinct chunks.
__device__ __forceinline__ int vswz(int d) { return (d >> 1) & 7; }

struct SeqMeta {
  const int32_t* q_start;  // first token of the sequence in the Q/out tensors
  const int32_t* q_len;    // new (query) tokens
  const int32_t* ctx_len;  // total keys visible (prefix + q_len)
};

template <int D, bool PAGED>
__global__ void __launch_bounds__(256, 2) prefill_attn_kernel(
    bf16* __restrict__ out, const bf16* __restrict__ q, int64_t q_stride, const bf16* __restrict__ kc,
    const bf16* __restrict__ vc, const int32_t* __restrict__ block_tables, int max_blocks, int NB,
    SeqMeta meta, const int32_t* __restrict__ tiles, int Hq, int Hkv, float scale_log2, int64_t out_stride) {
  constexpr int KS = D / 32;
  constexpr int DT = D / 16;
  constexpr int NCH = D / 8;           // 16-B chunks per K row
  constexpr int KCH = KVT * NCH;       // chunks per K tile
  constexpr int VCH = D * (KVT / 8);   // chunks per V^T tile
  constexpr int KPT = KCH / 256;       // K chunks per thread
  constexpr int VPT = VCH / 256;
  static_assert(KCH % 256 == 0 && VCH % 256 == 0, "tile must split evenly over 256 threads");
  __shared__ __attribute__((aligned(16))) bf16 ks_lds[KVT * D];
  __shared__ __attribute__((aligned(16))) bf16 vs_lds[D * KVT];

  const int G = Hq / Hkv;
  const int kvh = blockIdx.y;
  const int seq = tiles[2 * blockIdx.x];
  const int r0 = tiles[2 * blockIdx.x + 1];
  const int qs = meta.q_start[seq], ql = meta.q_len[seq], cl = meta.ctx_len[seq];
  const int prefix = cl - ql;
  const int nrows = ql * G;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, h = lane >> 4;

  // ---- Q^T fragments for this wave's two 16-row subtiles
  bf16x8 qf[2][KS];
  int rowpos[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int row = r0 + wid * 32 + n * 16 + i16;
    const bool valid = row < nrows;
    const int tq = valid ? row / G : 0, g = valid ? row - (row / G) * G : 0;
    rowpos[n] = valid ? prefix + tq : -1;  // -1: masks every key (row produces nothing)
    const bf16* qp = q + (int64_t)(qs + tq) * q_stride + (int64_t)(kvh * G + g) * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[n][ks] = __builtin_bit_cast(bf16x8, valid ? ld16(qp + 32 * ks) : make_uint4(0, 0, 0, 0));
  }
  // last row of this tile decides how many keys the workgroup must visit
  const int last_row = min(r0 + ROWS, nrows) - 1;
  const int kmax = PAGED ? min(cl, prefix + last_row / G + 1) : cl;
  const int ntiles = (kmax + KVT - 1) / KVT;

  f32x4 o[2][DT];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[n][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-1e30f, -1e30f}, l[2] = {0.f, 0.f};

  uint4 kreg[KPT], vreg[VPT];
  auto load_tile = [&](int t) {
    if constexpr (PAGED) {
      const int blk = min(max(block_tables[(int64_t)seq * max_blocks + min(t, max_blocks - 1)], 0), NB - 1);
      const bf16* kb = kc + ((int64_t)blk * Hkv + kvh) * KVT * D;
      const bf16* vb = vc + ((int64_t)blk * Hkv + kvh) * D * KVT;
#pragma unroll
      for (int i = 0; i < KPT; ++i) kreg[i] = ld16(kb + (threadIdx.x + 256 * i) * 8);
#pragma unroll
      for (int i = 0; i < VPT; ++i) vreg[i] = ld16(vb + (threadIdx.x + 256 * i) * 8);
    } else {
      // K rows / V rows straight from the packed QKV tensor (keys beyond the sequence -> 0)
#pragma unroll
      for (int i = 0; i < KPT; ++i) {
        const int qi = threadIdx.x + 256 * i, key = qi / NCH, c = qi - key * NCH;
        const int kk = t * KVT + key;
        kreg[i] = kk < cl ? ld16(kc + (int64_t)(qs + kk) * q_stride + (int64_t)(Hq + kvh) * D + c * 8)
                          : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int qi = threadIdx.x + 256 * i, key = qi / NCH, c = qi - key * NCH;
        const int kk = t * KVT + key;
        vreg[i] = kk < cl ? ld16(vc + (int64_t)(qs + kk) * q_stride + (int64_t)(Hq + Hkv + kvh) * D + c * 8)
                          : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int qi = threadIdx.x + 256 * i, key = qi / NCH, c = qi - key * NCH;
      *reinterpret_cast<uint4*>(&ks_lds[key * D + 8 * (c ^ kswz<D>(key))]) = kreg[i];
    }
    if constexpr (PAGED) {
      // source already V^T in 8-key groups: chunk qi = (key group c, dim d)
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int qi = threadIdx.x + 256 * i, c = qi / D, d = qi - c * D;
        *reinterpret_cast<uint4*>(&vs_lds[d * KVT + 8 * (c ^ vswz(d))]) = vreg[i];
      }
    } else {
      // source is V[key][d]: transpose while writing (2-B LDS stores)
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int qi = threadIdx.x + 256 * i, key = qi / NCH, c = qi - key * NCH;
        const bf16x8 v = __builtin_bit_cast(bf16x8, vreg[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int d = c * 8 + j;
          vs_lds[d * KVT + 8 * ((key >> 3) ^ vswz(d)) + (key & 7)] = v[j];
        }
      }
    }
  };

  if (ntiles > 0) load_tile(0);
  for (int t = 0; t < ntiles; ++t) {
    __syncthreads();  // everyone finished reading the previous tile
    store_tile();
    __syncthreads();
    if (t + 1 < ntiles) load_tile(t + 1);  // in flight during this tile's MFMAs
    const int kbase = t * KVT;
    // ---- S^T = K Q^T : 4 key subtiles x KS k-steps, K fragment shared by both row subtiles
    f32x4 s[2][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const int key = 32 * (kt >> 1) + 8 * (i16 >> 2) + 4 * (kt & 1) + (i16 & 3);
      const int sw = kswz<D>(key);
      s[0][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      s[1][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&ks_lds[key * D + 8 * ((4 * ks + h) ^ sw)]);
        s[0][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[0][ks], s[0][kt], 0, 0, 0);
        s[1][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[1][ks], s[1][kt], 0, 0, 0);
      }
    }
    // ---- online softmax per row subtile
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kbase + 32 * (kt >> 1) + 8 * h + 4 * (kt & 1) + r;
          float v = s[n][kt][r] * scale_log2;
          const bool ok = PAGED ? (key <= rowpos[n]) : (key < cl && rowpos[n] >= 0);
          v = ok ? v : -INFINITY;
          s[n][kt][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m[n], mx);
      const float alpha = exp2f(m[n] - mnew);
      float ps = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[n][kt][r] - mnew);
          s[n][kt][r] = p;
          ps += p;
        }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l[n] = l[n] * alpha + ps;
      m[n] = mnew;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[n][dt] *= alpha;
    }
    // ---- O^T += V^T P^T
#pragma unroll
    for (int kg = 0; kg < 2; ++kg) {
      bf16x8 pf[2];
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pf[n][j] = (bf16)s[n][2 * kg][j];
          pf[n][4 + j] = (bf16)s[n][2 * kg + 1][j];
        }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int d = 16 * dt + i16;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&vs_lds[d * KVT + 8 * ((4 * kg + h) ^ vswz(d))]);
        o[0][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pf[0], o[0][dt], 0, 0, 0);
        o[1][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pf[1], o[1][dt], 0, 0, 0);
      }
    }
  }
  // ---- epilogue: O[row i16][d = 16dt + 4h + r] / l
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int row = r0 + wid * 32 + n * 16 + i16;
    if (row < nrows) {
      const int tq = row / G, g = row - tq * G;
      const float inv = l[n] > 0.f ? 1.f / l[n] : 0.f;
      bf16* op = out + (int64_t)(qs + tq) * out_stride + (int64_t)(kvh * G + g) * D + 4 * h;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[n][dt][r] * inv);
        *reinterpret_cast<bf16x4*>(op + 16 * dt) = v;
      }
    }
  }
}

}  // namespace

// Paged causal prefill.  q: [T, >=Hq*D] view with row stride; out: [T, Hq*D].
// tiles: [ntiles, 2] int32 (seq, first row) with rows = token*G + g, 128 rows per tile.
void paged_prefill_attention(at::Tensor out, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                             at::Tensor block_tables, at::Tensor q_start, at::Tensor q_len, at::Tensor ctx_len,
                             at::Tensor tiles, int64_t Hq, double scale) {
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16 && q.stride(-1) == 1);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == KVT && v_cache.dim() == 5 && v_cache.size(2) == KVT / 8 &&
              v_cache.size(4) == 8, "KV block size must be 64 (v_cache [NB, Hkv, 8, D, 8])");
  const int Hkv = k_cache.size(1), D = k_cache.size(3);
  TORCH_CHECK(Hq % Hkv == 0 && v_cache.size(3) == D);
  for (auto* t : {&block_tables, &q_start, &q_len, &ctx_len, &tiles})
    TORCH_CHECK(t->scalar_type() == at::kInt && t->is_contiguous());
  TORCH_CHECK(out.stride(-1) == 1 && q.stride(0) % 8 == 0 && out.stride(0) % 4 == 0);
  const int ntiles = tiles.size(0);
  if (ntiles == 0) return;
  SeqMeta meta{q_start.data_ptr<int32_t>(), q_len.data_ptr<int32_t>(), ctx_len.data_ptr<int32_t>()};
  dim3 grid(ntiles, Hkv);
  auto stream = at::hip::getCurrentHIPStream();
  const float sl2 = (float)scale * LOG2E_P;
#define LAUNCH(DD)                                                                                                   \
  prefill_attn_kernel<DD, true><<<grid, 256, 0, stream>>>(                                                          \
      (bf16*)out.data_ptr(), (const bf16*)q.data_ptr(), q.stride(0), (const bf16*)k_cache.data_ptr(),              \
      (const bf16*)v_cache.data_ptr(), block_tables.data_ptr<int32_t>(), (int)block_tables.size(1),                 \
      (int)k_cache.size(0), meta, tiles.data_ptr<int32_t>(), (int)Hq, Hkv, sl2, out.stride(0))
  if (D == 128) LAUNCH(128);
  else if (D == 64) LAUNCH(64);
  else TORCH_CHECK(false, "unsupported head dim ", D);
#undef LAUNCH
}

// Dense bidirectional varlen attention over a packed QKV tensor [T, (Hq+2Hkv)*D]
// (BERT encoder).  out: [T, Hq*D].  seq arrays: q_start == k_start, q_len == ctx_len.
void varlen_encoder_attention(at::Tensor out, at::Tensor qkv, at::Tensor q_start, at::Tensor q_len,
                              at::Tensor tiles, int64_t Hq, int64_t Hkv, double scale) {
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && qkv.is_contiguous() && out.is_contiguous());
  for (auto* t : {&q_start, &q_len, &tiles}) TORCH_CHECK(t->scalar_type() == at::kInt && t->is_contiguous());
  const int D = qkv.size(-1) / (Hq + 2 * Hkv);
  TORCH_CHECK(D * (Hq + 2 * Hkv) == qkv.size(-1));
  const int ntiles = tiles.size(0);
  if (ntiles == 0) return;
  SeqMeta meta{q_start.data_ptr<int32_t>(), q_len.data_ptr<int32_t>(), q_len.data_ptr<int32_t>()};
  dim3 grid(ntiles, Hkv);
  auto stream = at::hip::getCurrentHIPStream();
  const float sl2 = (float)scale * LOG2E_P;
  const bf16* base = (const bf16*)qkv.data_ptr();
#define LAUNCH(DD)                                                                                       \
  prefill_attn_kernel<DD, false><<<grid, 256, 0, stream>>>((bf16*)out.data_ptr(), base, qkv.stride(0),  \
                                                           base, base, nullptr, 1, 1, meta,             \
                                                           tiles.data_ptr<int32_t>(), (int)Hq, (int)Hkv, \
                                                           sl2, out.stride(0))
  if (D == 32) LAUNCH(32);
  else if (D == 64) LAUNCH(64);
  else if (D == 128) LAUNCH(128);
  else TORCH_CHECK(false, "unsupported head dim ", D);
#undef LAUNCH
}
