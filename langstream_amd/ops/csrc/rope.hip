// RoPE + paged-KV cache write, fused (one pass over the QKV projection output).
//
// qkv      : [T, (Hq + 2*Hkv) * D] bf16, rotated IN PLACE for the q and k heads
// pos      : [T] int32 absolute positions
// cos_sin  : [max_pos, D] f32 table; cols [0, D/2) = cos, [D/2, D) = sin (host-built,
//            includes any rope scaling; no device trig -- guide App. B "element-wise")
// slots    : [T] int64 cache slot = block * BS + offset (-1 = do not cache)
// k_cache  : [NB, Hkv, BS, D]   (token-major rows: 256-B contiguous per token & head)
// v_cache  : [NB, Hkv, BS/8, D, 8]   (TRANSPOSED in 8-key groups: 8 keys of one dim are
//            16 contiguous bytes, so attention reads V^T MFMA fragments with one 16-B load
//            per lane; a token's V lands at a 16-B stride -- common.h vt_off)
//
// Grid: x = tiles of TOK tokens, y = head groups.  y < nq: rotate HG query heads;
// nq <= y < nq+nk: rotate HG key heads and store them to the K cache; the last Hkv
// y-slices write one kv head of V transposed, with lane == token inside a tile so a
// wave's 2-B stores for one head-dim row land on consecutive cache addresses.
// Many small workgroups: a decode step (T = batch) still spreads over
// (T/16) x (Hq/8 + Hkv/8 + Hkv) workgroups instead of one.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

// Tokens per workgroup tile: 16 for prefill-sized T; 2 for decode-sized T, so a
// B=256 decode step launches ~1.7k workgroups with one task per thread instead of
// 208 workgroups looping over dependent pos -> cos/sin loads (12 us -> latency of one).
constexpr int TOK_LARGE = 16;
constexpr int TOK_SMALL = 2;
constexpr int64_t SMALL_T = 2048;
constexpr int HG = 8;    // heads per rotate workgroup

template <int D, int TOK>
__global__ void __launch_bounds__(256) rope_cache_kernel(bf16* __restrict__ qkv, const int32_t* __restrict__ pos,
                                                         const float* __restrict__ cos_sin,
                                                         const int64_t* __restrict__ slots, bf16* __restrict__ kc,
                                                         bf16* __restrict__ vc, int64_t T, int Hq, int Hkv, int BS,
                                                         int max_pos, int apply_rope, int64_t nslots) {
  constexpr int HALF = D / 2;
  constexpr int VPH = HALF / 8;  // 16-B vectors per half head
  const int64_t t0 = (int64_t)blockIdx.x * TOK;
  const int ntok = (int)min((int64_t)TOK, T - t0);
  const int row_elems = (Hq + 2 * Hkv) * D;
  const int nq = (Hq + HG - 1) / HG, nk = (Hkv + HG - 1) / HG;
  const int y = blockIdx.y;
  if (y < nq + nk) {
    // ---- rotate a group of q (or k) heads for the tile's tokens
    const bool is_k = y >= nq;
    const int h0 = is_k ? Hq + (y - nq) * HG : y * HG;
    const int hend = is_k ? Hq + Hkv : Hq;
    const int nh = min(HG, hend - h0);
    const int tasks = ntok * nh * VPH;
    for (int i = threadIdx.x; i < tasks; i += blockDim.x) {
      const int tl = i / (nh * VPH);
      const int rem = i - tl * nh * VPH;
      const int h = h0 + rem / VPH, c = rem % VPH;
      const int64_t t = t0 + tl;
      bf16* base = qkv + t * row_elems + h * D;
      float a[8], b[8];
      unpack8(ld16(base + c * 8), a);
      unpack8(ld16(base + HALF + c * 8), b);
      if (apply_rope) {
        const int p = min(max(pos[t], 0), max_pos - 1);
        const float* cs = cos_sin + (int64_t)p * D;
        float co[8], si[8];
        *reinterpret_cast<float4*>(co) = *reinterpret_cast<const float4*>(cs + c * 8);
        *reinterpret_cast<float4*>(co + 4) = *reinterpret_cast<const float4*>(cs + c * 8 + 4);
        *reinterpret_cast<float4*>(si) = *reinterpret_cast<const float4*>(cs + HALF + c * 8);
        *reinterpret_cast<float4*>(si + 4) = *reinterpret_cast<const float4*>(cs + HALF + c * 8 + 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x1 = a[j], x2 = b[j];
          a[j] = x1 * co[j] - x2 * si[j];
          b[j] = x2 * co[j] + x1 * si[j];
        }
      }
      const uint4 pa = pack8(a), pb = pack8(b);
      st16(base + c * 8, pa);
      st16(base + HALF + c * 8, pb);
      if (is_k) {
        const int64_t s = slots[t];
        if (s >= 0 && s < nslots) {
          const int64_t blk = s / BS, off = s - blk * BS;
          bf16* kd = kc + ((blk * Hkv + (h - Hq)) * BS + off) * D;
          st16(kd + c * 8, pa);
          st16(kd + HALF + c * 8, pb);
        }
      }
    }
    return;
  }
  // ---- V of one kv head, transposed into the cache.  thread -> (token lane, d-row)
  const int hv = y - nq - nk;
  const int tl = threadIdx.x % TOK;
  const int dr = threadIdx.x / TOK;  // 0..256/TOK-1
  if (tl >= ntok) return;
  const int64_t t = t0 + tl;
  const int64_t s = slots[t];
  if (s < 0 || s >= nslots) return;
  const int64_t blk = s / BS, off = s - blk * BS;
  const bf16* src = qkv + t * row_elems + (Hq + Hkv + hv) * D;
  bf16* vd = vc + ((blk * Hkv + hv) * (int64_t)D) * BS;
  for (int d = dr; d < D; d += 256 / TOK) vd[vt_off(d, (int)off, D)] = src[d];
}

}  // namespace

void rope_and_cache(at::Tensor qkv, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots, at::Tensor k_cache,
                    at::Tensor v_cache, int64_t Hq, int64_t Hkv, bool apply_rope) {
  TORCH_CHECK(qkv.is_cuda() && qkv.scalar_type() == at::kBFloat16 && qkv.is_contiguous());
  TORCH_CHECK(pos.scalar_type() == at::kInt && slots.scalar_type() == at::kLong);
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous());
  TORCH_CHECK(k_cache.scalar_type() == at::kBFloat16 && v_cache.scalar_type() == at::kBFloat16);
  TORCH_CHECK(k_cache.dim() == 4 && v_cache.dim() == 5, "k_cache [NB, Hkv, BS, D], v_cache [NB, Hkv, BS/8, D, 8]");
  const int D = k_cache.size(3);
  const int BS = k_cache.size(2);
  TORCH_CHECK(k_cache.size(1) == Hkv && v_cache.size(1) == Hkv && v_cache.size(2) == BS / 8 && v_cache.size(3) == D &&
              v_cache.size(4) == 8);
  TORCH_CHECK(qkv.size(-1) == (Hq + 2 * Hkv) * D);
  const int64_t T = qkv.numel() / qkv.size(-1);
  TORCH_CHECK(pos.numel() == T && slots.numel() == T);
  TORCH_CHECK(cos_sin.size(1) == D);
  if (T == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const int nq = (int)((Hq + HG - 1) / HG), nk = (int)((Hkv + HG - 1) / HG);
  const bool small = T <= SMALL_T;
  const int tok = small ? TOK_SMALL : TOK_LARGE;
  dim3 grid((unsigned)((T + tok - 1) / tok), nq + nk + (int)Hkv);
#define LAUNCH(DD, TT)                                                                                      \
  rope_cache_kernel<DD, TT><<<grid, 256, 0, stream>>>((bf16*)qkv.data_ptr(), pos.data_ptr<int32_t>(),      \
                                                      cos_sin.data_ptr<float>(), slots.data_ptr<int64_t>(), \
                                                      (bf16*)k_cache.data_ptr(), (bf16*)v_cache.data_ptr(), T, \
                                                      (int)Hq, (int)Hkv, BS, (int)cos_sin.size(0),          \
                                                      apply_rope ? 1 : 0, (int64_t)k_cache.size(0) * BS)
  if (D == 128) { if (small) LAUNCH(128, TOK_SMALL); else LAUNCH(128, TOK_LARGE); }
  else if (D == 64) { if (small) LAUNCH(64, TOK_SMALL); else LAUNCH(64, TOK_LARGE); }
  else TORCH_CHECK(false, "unsupported head dim ", D);
#undef LAUNCH
}
