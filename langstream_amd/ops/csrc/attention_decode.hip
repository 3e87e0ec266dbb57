// Paged GQA decode attention on MFMA (gfx950, mfma_f32_16x16x32_bf16).
//
// One query token per sequence.  Work unit = one (sequence, kv-head) pair; its G
// query heads (G = Hq/Hkv <= 16) are the 16 MFMA "rows" (padded with zero rows).
//
// Layout trick (no LDS, no transposes): with the V cache stored transposed in 8-key
// groups ([NB, Hkv, BS/8, D, 8], common.h vt_off) and the scores computed SWAPPED (S^T = K * Q^T), every MFMA
// operand of both products is one 16-B contiguous global load per lane and the
// softmax statistics stay lane-local:
//   S^T tile kt=(2*kg+e):  A = K rows, lane i=l&15 loads key 32kg + 8(i>>2) + 4e + (i&3)
//                          B = Q^T (registers), acc[r] = S[key 32kg+8h+4e+r][qrow l&15]
//   O^T tile dt:           A = V^T rows d=16dt+i, keys 32kg+8h..+7 (16 B)
//                          B = P^T: element j of lane-group h is key 32kg+8h+j, which is
//                          exactly acc(kt=2kg+(j>>2))[j&3] of the same lane.
// The K-row permutation above is what makes the P^T fragment lane-local.
//
// Grid: (B*Hkv, S splits).  WPP waves per workgroup stride over the split's KV blocks:
// WPP = 1 (one wave owns a (seq, kv-head) pair, writes straight from its accumulators)
// once the pairs alone fill every wave slot of the chip (B*Hkv >= 2048, no split);
// otherwise WPP = 4, merged through LDS, and with S > 1 a second kernel merges splits
// (a sequence whose context fits in one split is finished by split 0 and skipped by
// the merge: short chats at small batch pay no partial round trip).
//
// Split policy (decided per launch, so it is fixed inside a captured HIP graph):
// S = min(nsplit_max, ceil(TARGET_WG / (B*Hkv))).  At large batch the (seq, kv-head)
// pairs alone fill the chip, S = 1, and there are no partials and no merge launch; at
// small batch a long context is cut into S pieces.  Each sequence divides its OWN
// context evenly over the S splits (bps = max(min_bps, ceil(nblk / S)), computed on
// the device), so the grid carries no idle workgroups for short sequences.
//
// Memory path: K and V fragments are raw buffer loads through per-block descriptors
// (wave-uniform, readfirstlane'd).  The K descriptor covers only the block's valid
// keys and masked V groups get an out-of-range offset, so the tail of a sequence's
// last block is never fetched (the hardware range check returns zeros).  Per wave, all
// 32 KiB of a block's K and V are in flight before its first MFMA; with PIPE the next
// block's K is issued right after the scores and its V right after O += V P (same
// registers), so a wave keeps streaming through its softmax.  250 VGPRs, 2 waves/SIMD.
//
// Measured on MI355X (tools/attn_bench.py, 32 q / 8 kv heads x 128, scattered blocks;
// profiles/decode_attn_*_r2i.log), B=256:
//   ctx 448: 89.8 us (flat loads, r1) -> 84.3 (buffer loads) -> 80.0 us = 5.9 TB/s
//            (WPP=1 + PIPE); ctx 1024: 176 us = 6.1 TB/s; ctx 410 (ragged tail) 77 us.
// Ragged contexts (uniform +-30 %) cost ~12 % at WPP=1 (the launch ends with the
// longest sequence: 2048 waves fill the 2048 slots, nothing rebalances) and ~11 % at
// WPP=4; forcing 2-3 KV splits to rebalance was slower still (107 vs 94 us,
// profiles/decode_attn_ragged_split_ab_r2i.log).
// Rejected: nt loads (+7%, back-to-back replays lose the L2/MALL reuse), a select on
// the loaded data for the tail mask (139 us: each load waited before the next issued),
// next-block prefetch into extra registers (1 wave/SIMD, 103 us), 125 VGPRs / 4 waves
// (106 us), amdgpu_waves_per_eu(3) (106.9 us).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

constexpr int BS = 64;            // tokens per KV block (engine-wide constant)
constexpr int TARGET_WG = 512;    // ~2 workgroups per CU before contexts are split (1024 measured
                                  // 13-17 % slower at B = 32-64, ctx 600: profiles/attn_split_r4l.log)
constexpr int WAVE_SLOTS = 2048;  // 256 CUs x 4 SIMDs x 2 waves/SIMD
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ int split_blocks(int nblk, int nsplit, int min_bps) {
  return max(min_bps, (nblk + nsplit - 1) / nsplit);
}

// Fused RoPE + KV write (ROPE = true, decode-only steps): q holds the UN-rotated QKV
// projection rows [B, (Hq + 2 Hkv) D].  Every wave rotates its Q^T fragments in
// registers (a lane's dims 32ks + 8h + j, ks < KS/2, pair with the +D/2 dims of ks + KS/2
// in the same lane).  The step's new token (position pos[b] = ctx - 1) is NOT read back
// from the cache: waves attend over the ctx - 1 cached keys, and the owner wave (wave 0
// of split 0) rotates the new key, writes K and V^T into the paged cache for later steps
// and seeds its softmax state with the new token itself (m = s_new, l = 1, O = v_new).
// This removes the separate rope_cache launch (~11 us per layer at B = 256 in the RAG
// bench, profiles/rag_bench_kernel_stats_r2m.csv) from every decode step.
struct RopeArgs {
  const float* cos_sin;    // [max_pos, D]: cos in [0, D/2), sin in [D/2, D)
  const int32_t* pos;      // [B]
  int max_pos;
  const int64_t* slots;    // [B] cache slot of the new token (-1: do not cache)
  int64_t nslots;
  bf16* kc;                // writable views of the caches
  bf16* vc;
};

template <int D, int WPP, bool PIPE, bool ROPE, int AUX = 0>
__global__ void __launch_bounds__(64 * WPP) __attribute__((amdgpu_waves_per_eu(2, 2))) decode_attn_kernel(
    bf16* __restrict__ out, const bf16* __restrict__ q, int64_t q_stride, const bf16* __restrict__ kc,
    const bf16* __restrict__ vc, const int32_t* __restrict__ block_tables, int max_blocks,
    const int32_t* __restrict__ ctx_lens, int Hkv, int G, int NB, float scale_log2, int min_bps,
    float* __restrict__ part_o, float* __restrict__ part_ml, RopeArgs ra) {
  constexpr int KS = D / 32;  // k-steps over the head dim
  constexpr int DT = D / 16;  // 16-wide output tiles over the head dim
  constexpr int HALF = D / 2;

  const int pair = blockIdx.x;
  const int b = pair / Hkv, kvh = pair - b * Hkv;
  const int split = blockIdx.y, nsplit = gridDim.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, h = lane >> 4;

  const int ctx_all = ctx_lens[b];
  const int p_new = ROPE ? min(max(ra.pos[b], 0), ra.max_pos - 1) : 0;
  // keys read from the cache: with ROPE the new token (the last one) comes from registers
  const int ctx = ROPE ? max(ctx_all - 1, 0) : ctx_all;
  const int nblk = min((ctx + BS - 1) / BS, max_blocks);
  const int bps = split_blocks(nblk, nsplit, min_bps);
  const int bstart = split * bps;
  const int bend = min(nblk, bstart + bps);
  // splits past this sequence's context exit at once; the merge kernel only reads
  // the ceil(nblk / bps) splits that exist.
  if (split > 0 && bstart >= nblk) return;
  // a context that fits in one split (short chats at small batch) is finished here:
  // split 0 writes the normalised bf16 row and the merge kernel skips it
  const bool single = nsplit == 1 || nblk <= bps;

  // Q^T fragments (B operand): lane holds Q[head kvh*G + i16][32ks + 8h .. +7]
  bf16x8 qf[KS];
  const bool qrow_valid = i16 < G;
  const bf16* qp = q + (int64_t)b * q_stride + (int64_t)(kvh * G + (qrow_valid ? i16 : 0)) * D + 8 * h;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    uint4 v = qrow_valid ? ld16(qp + 32 * ks) : make_uint4(0, 0, 0, 0);
    qf[ks] = __builtin_bit_cast(bf16x8, v);
  }

  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, l = 0.f;

  const int32_t* bt = block_tables + (int64_t)b * max_blocks;
  auto block_of = [&](int bi) { return min(max(bt[bi], 0), NB - 1); };
  // Keys at or past the context are never fetched (the last block of a sequence is
  // partly filled).  K and V go through per-block buffer descriptors: a K descriptor
  // covers exactly the valid rows, so the hardware range check returns zeros for the
  // rest without touching memory; a V^T group whose 8 keys all lie past the context
  // gets an out-of-range offset.  (A select on the loaded data instead made every
  // load wait before the next one issued: 139 vs 90 us at B=256.)
  constexpr int OOB = 1 << 30;
  // AUX: buffer-load cache policy, 0 or 2 (nt).  KV bytes have no reuse within a decode
  // step: in the RAG bench nt loads take the in-engine kernel from 84.5 to 73.5 us per
  // layer (the activations and split-K slabs stay cached; profiles/nt_r3c/).  Back-to-back
  // isolated calls over one pool re-read the same cache and measure nt slower, so
  // tools/attn_bench.py runs with a ring of pools.  LS_ATTN_NT=0 turns it off.
  const int kbyte = 8 * h * 2;

  // AUX 3 (LS_ATTN_NT=2, the default): the FIRST block of a sequence loaded with the
  // cached policy, for template-prefix blocks shared by every prompt (engine/
  // prefix_cache.py); see the launch site for the measurements behind the default.
  auto issue_k_p = [&](int bi, uint4(&kf)[4][KS], auto polc) {
    constexpr int POL = decltype(polc)::value;
    const int blk = __builtin_amdgcn_readfirstlane(block_of(bi));
    const int lim = __builtin_amdgcn_readfirstlane(min(ctx - bi * BS, BS));   // valid keys here (>= 1)
    const int64_t boff = ((int64_t)blk * Hkv + kvh) * BS * D;
    auto krs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(kc + boff), 0, lim * D * 2, 0x00020000);
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const int key = 32 * (kt >> 1) + 8 * (i16 >> 2) + 4 * (kt & 1) + (i16 & 3);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        kf[kt][ks] = __builtin_bit_cast(
            uint4, __builtin_amdgcn_raw_buffer_load_b128(krs, key * D * 2 + 64 * ks + kbyte, 0, POL));
    }
  };
  auto issue_v_p = [&](int bi, uint4(&vf)[2][DT], auto polc) {
    constexpr int POL = decltype(polc)::value;
    const int blk = __builtin_amdgcn_readfirstlane(block_of(bi));
    const int lim = __builtin_amdgcn_readfirstlane(min(ctx - bi * BS, BS));
    const int64_t boff = ((int64_t)blk * Hkv + kvh) * BS * D;
    auto vrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(vc + boff), 0, BS * D * 2, 0x00020000);
#pragma unroll
    for (int kg = 0; kg < 2; ++kg) {
      const bool vok = 32 * kg + 8 * h < lim;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int off = (int)vt_off(16 * dt + i16, 32 * kg + 8 * h, D) * 2;
        vf[kg][dt] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(vrs, vok ? off : OOB, 0, POL));
      }
    }
  };
  // AUX 3: nt loads except for a sequence's first block (cached)
  constexpr bool FIRST_CACHED = AUX == 3;
  constexpr int POLX = AUX == 3 ? 2 : AUX;
  auto issue_k = [&](int bi, uint4(&kf)[4][KS]) {
    if (FIRST_CACHED && bi == 0) issue_k_p(bi, kf, std::integral_constant<int, 0>());
    else issue_k_p(bi, kf, std::integral_constant<int, POLX>());
  };
  auto issue_v = [&](int bi, uint4(&vf)[2][DT]) {
    if (FIRST_CACHED && bi == 0) issue_v_p(bi, vf, std::integral_constant<int, 0>());
    else issue_v_p(bi, vf, std::integral_constant<int, POLX>());
  };

  // K and V of block i are in flight together; with PIPE, block i+1's K loads are
  // issued as soon as the scores of block i are computed (its K registers are free) and
  // its V loads right after O += V P (same registers, no extra VGPRs), so a wave keeps
  // streaming while it does the softmax and the PV products.
  uint4 kf[4][KS];
  uint4 vf[2][DT];
  if (PIPE && bstart + wid < bend) {
    issue_k(bstart + wid, kf);
    issue_v(bstart + wid, vf);
  }
  // RoPE after the first block's K/V loads are issued: its loads and math hide
  // behind that fetch, which the first MFMA waits for anyway
  if constexpr (ROPE) {
    // cos / sin of this lane's low-half dims c = 32ks + 8h + j (ks < KS/2)
    const float* cs = ra.cos_sin + (int64_t)p_new * D;
    float co[KS / 2][8], si[KS / 2][8];
#pragma unroll
    for (int ks = 0; ks < KS / 2; ++ks) {
      const int c = 32 * ks + 8 * h;
      *reinterpret_cast<float4*>(co[ks]) = *reinterpret_cast<const float4*>(cs + c);
      *reinterpret_cast<float4*>(co[ks] + 4) = *reinterpret_cast<const float4*>(cs + c + 4);
      *reinterpret_cast<float4*>(si[ks]) = *reinterpret_cast<const float4*>(cs + HALF + c);
      *reinterpret_cast<float4*>(si[ks] + 4) = *reinterpret_cast<const float4*>(cs + HALF + c + 4);
    }
    auto rotate = [&](bf16x8 (&f)[KS]) {
#pragma unroll
      for (int ks = 0; ks < KS / 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x1 = (float)f[ks][j], x2 = (float)f[ks + KS / 2][j];
          f[ks][j] = (bf16)(x1 * co[ks][j] - x2 * si[ks][j]);
          f[ks + KS / 2][j] = (bf16)(x2 * co[ks][j] + x1 * si[ks][j]);
        }
    };
    rotate(qf);
    if (split == 0 && wid == 0 && ctx_all >= 1) {
      // the new token: rotated key (every lane group h holds dims 32ks + 8h .. +7)
      const bf16* kp = q + (int64_t)b * q_stride + (int64_t)(Hkv * G + kvh) * D + 8 * h;
      const bf16* vp = q + (int64_t)b * q_stride + (int64_t)(Hkv * G + Hkv + kvh) * D;
      bf16x8 kn[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kn[ks] = __builtin_bit_cast(bf16x8, ld16(kp + 32 * ks));
      rotate(kn);
      // O^T layout: lane holds O[qrow][16dt + 4h + r]; the new token's V for those dims
      bf16x4 vn[DT];
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) vn[dt] = *reinterpret_cast<const bf16x4*>(vp + 16 * dt + 4 * h);
      float dot = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) dot += (float)qf[ks][j] * (float)kn[ks][j];
      dot += __shfl_xor(dot, 16, 64);
      dot += __shfl_xor(dot, 32, 64);
      // first element of the online softmax: m = s_new, l = 1, O = v_new
      m = dot * scale_log2;
      l = 1.f;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[dt][r] = (float)vn[dt][r];
      const int64_t sl = ra.slots[b];
      if (sl >= 0 && sl < ra.nslots) {
        const int64_t blk = sl / BS, off = sl - blk * BS;
        if (i16 == 0) {
          bf16* kd = ra.kc + ((blk * Hkv + kvh) * BS + off) * D + 8 * h;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) st16(kd + 32 * ks, __builtin_bit_cast(uint4, kn[ks]));
        }
        if (i16 < DT) {
          // V^T: lane (i16, h) stores dims 16 i16 + 4h + r (2-B stores at a 16-B stride)
          bf16* vd = ra.vc + ((blk * Hkv + kvh) * (int64_t)D) * BS;
          bf16x4 vv = vn[0];
#pragma unroll
          for (int dt = 1; dt < DT; ++dt) if (i16 == dt) vv = vn[dt];
#pragma unroll
          for (int r = 0; r < 4; ++r) vd[vt_off(16 * i16 + 4 * h + r, (int)off, D)] = vv[r];
        }
      }
    }
  }

  for (int bi = bstart + wid; bi < bend; bi += WPP) {
    const bool more = bi + WPP < bend;
    if (!PIPE) {
      issue_k(bi, kf);
      issue_v(bi, vf);
    }
    // all 32 KiB of the block in flight before the first MFMA (the scheduler would
    // otherwise sink the V loads past the softmax to raise occupancy)
    __builtin_amdgcn_sched_barrier(0);
    // ---- S^T = K Q^T for the 64 keys of this block (4 tiles of 16 keys)
    f32x4 s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf[kt][ks]), qf[ks], acc, 0, 0, 0);
      s[kt] = acc;
    }
    // ---- online softmax (row = qrow = lane&15; this lane holds 16 of the 64 keys)
    const int kbase = bi * BS;
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kbase + 32 * (kt >> 1) + 8 * h + 4 * (kt & 1) + r;
        float v = s[kt][r] * scale_log2;
        v = key < ctx ? v : -INFINITY;
        s[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx);
    const float alpha = exp2f(m - mnew);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[kt][r] - mnew);
        s[kt][r] = p;
        psum += p;
      }
    }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mnew;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    if (PIPE && more) issue_k(bi + WPP, kf);
    __builtin_amdgcn_sched_barrier(0);
    // ---- O^T += V^T P^T
#pragma unroll
    for (int kg = 0; kg < 2; ++kg) {
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = (bf16)s[2 * kg][j];
        pf[4 + j] = (bf16)s[2 * kg + 1][j];
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vf[kg][dt]), pf, o[dt], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (PIPE && more) issue_v(bi + WPP, vf);
  }

  // o[dt][r] = O[qrow i16][d = 16dt + 4h + r]
  if constexpr (WPP == 1) {
    // one wave owns the (pair, split): write straight from the accumulators
    if (i16 < G) {
      const int64_t row = (int64_t)b * Hkv * G + kvh * G + i16;
      if (single) {
        const float inv = l > 0.f ? 1.f / l : 0.f;
        bf16* op = out + row * D + 4 * h;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[dt][r] * inv);
          *reinterpret_cast<bf16x4*>(op + 16 * dt) = v;
        }
      } else {
        const int64_t pi = row * nsplit + split;
        float* po = part_o + pi * D + 4 * h;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) *reinterpret_cast<f32x4*>(po + 16 * dt) = o[dt];
        if (h == 0) {
          part_ml[pi * 2] = m;
          part_ml[pi * 2 + 1] = l;
        }
      }
    }
  } else {
  static_assert(WPP == 4, "the LDS merge maps 256 threads onto (16 rows x 16 chunks)");
  // ---- merge the WPP waves through LDS
  __shared__ float sh_o[WPP][16][D + 4];
  __shared__ float sh_m[WPP][16], sh_l[WPP][16];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) sh_o[wid][i16][16 * dt + 4 * h + r] = o[dt][r];
  if (h == 0) {
    sh_m[wid][i16] = m;
    sh_l[wid][i16] = l;
  }
  __syncthreads();
  // 256 threads: thread -> (qrow, d-chunk of D/16)
  const int row = threadIdx.x >> 4;   // 0..15
  const int dc = threadIdx.x & 15;    // chunk of D/16 elements
  constexpr int CH = D / 16;
  if (row < G) {
    float mw[WPP], mstar = -1e30f;
#pragma unroll
    for (int w = 0; w < WPP; ++w) { mw[w] = sh_m[w][row]; mstar = fmaxf(mstar, mw[w]); }
    float lt = 0.f, f[WPP];
#pragma unroll
    for (int w = 0; w < WPP; ++w) { f[w] = exp2f(mw[w] - mstar); lt += sh_l[w][row] * f[w]; }
    float acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < WPP; ++w) a += sh_o[w][row][dc * CH + c] * f[w];
      acc[c] = a;
    }
    const int head = kvh * G + row;
    if (single) {
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      bf16* op = out + ((int64_t)b * Hkv * G + head) * D + dc * CH;
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] *= inv;
#pragma unroll
      for (int c = 0; c < CH; c += 8) st16(op + c, pack8(acc + c));
    } else {
      const int64_t pi = (((int64_t)b * Hkv * G + head) * nsplit + split);
      float* po = part_o + pi * D + dc * CH;
#pragma unroll
      for (int c = 0; c < CH; ++c) po[c] = acc[c];
      if (dc == 0) {
        part_ml[pi * 2] = mstar;
        part_ml[pi * 2 + 1] = lt;
      }
    }
  }
  }
}

template <int D>
__global__ void __launch_bounds__(256) decode_merge_kernel(bf16* __restrict__ out, const float* __restrict__ part_o,
                                                           const float* __restrict__ part_ml, int nsplit_grid, int nrows,
                                                           const int32_t* __restrict__ ctx_lens, int Hq, int min_bps,
                                                           int max_blocks, int ctx_adj) {
  // one wave per (b, head) row; lanes over d
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  // ctx_adj = 1 under ROPE: the split kernel covered the ctx - 1 cached keys
  const int nblk = min((max(ctx_lens[row / Hq] - ctx_adj, 0) + BS - 1) / BS, max_blocks);
  const int bps = split_blocks(nblk, nsplit_grid, min_bps);
  const int nsplit = max(1, min(nsplit_grid, (nblk + bps - 1) / bps));
  if (nblk <= bps) return;   // one split: the attention kernel wrote the row itself
  const float* ml = part_ml + (int64_t)row * nsplit_grid * 2;
  float mstar = -1e30f;
  for (int s = 0; s < nsplit; ++s) mstar = fmaxf(mstar, ml[2 * s]);
  float lt = 0.f;
  for (int s = 0; s < nsplit; ++s) lt += ml[2 * s + 1] * exp2f(ml[2 * s] - mstar);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  for (int d = lane; d < D; d += 64) {
    float a = 0.f;
    for (int s = 0; s < nsplit; ++s) a += part_o[((int64_t)row * nsplit_grid + s) * D + d] * exp2f(ml[2 * s] - mstar);
    out[(int64_t)row * D + d] = (bf16)(a * inv);
  }
}

}  // namespace

// Number of KV splits a decode launch over B sequences uses (<= nsplit_max).
int64_t decode_nsplit(int64_t B, int64_t Hkv, int64_t nsplit_max) {
  static const int64_t target = getenv("LS_ATTN_TARGET_WG") ? atoll(getenv("LS_ATTN_TARGET_WG")) : TARGET_WG;
  const int64_t pairs = std::max<int64_t>(1, B * Hkv);
  return std::max<int64_t>(1, std::min<int64_t>(nsplit_max, (target + pairs - 1) / pairs));
}

// q: [B, Hq*D] view (row stride q_stride elements), out: [B, Hq, D] contiguous.
// nsplit: the MAXIMUM split count (the workspace is sized for it); a launch uses
// decode_nsplit(B, Hkv, nsplit).  min_bps: the fewest KV blocks one split covers.
// workspace: f32 tensor with >= B*Hq*S*(D+2) elements when the launch splits (S > 1).
static void decode_attention_launch(at::Tensor& out, const at::Tensor& q, const at::Tensor& k_cache,
                                    const at::Tensor& v_cache, const at::Tensor& block_tables,
                                    const at::Tensor& ctx_lens, double scale, int64_t nsplit, int64_t min_bps,
                                    const at::Tensor& workspace, const RopeArgs* ra) {
  TORCH_CHECK(q.is_cuda() && q.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16);
  TORCH_CHECK(out.is_contiguous() && q.stride(-1) == 1);
  TORCH_CHECK(k_cache.dim() == 4 && v_cache.dim() == 5, "k_cache [NB, Hkv, 64, D], v_cache [NB, Hkv, 8, D, 8]");
  const int Hkv = k_cache.size(1), D = k_cache.size(3);
  TORCH_CHECK(k_cache.size(2) == BS && v_cache.size(1) == Hkv && v_cache.size(2) == BS / 8 && v_cache.size(3) == D &&
              v_cache.size(4) == 8, "KV block size must be 64");
  const int B = ctx_lens.numel();
  TORCH_CHECK(out.numel() % ((int64_t)B * D) == 0);
  const int Hq = out.numel() / ((int64_t)B * D);
  TORCH_CHECK(Hq % Hkv == 0);
  const int G = Hq / Hkv;
  TORCH_CHECK(G <= 16, "GQA group too large for the 16-row MFMA tile");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && block_tables.is_contiguous() && block_tables.size(0) == B);
  TORCH_CHECK(ctx_lens.scalar_type() == at::kInt && ctx_lens.is_contiguous());
  TORCH_CHECK(nsplit >= 1 && min_bps >= 1);
  const int64_t q_stride = q.dim() >= 2 ? q.stride(0) : (int64_t)Hq * D;
  TORCH_CHECK(q_stride % 8 == 0);
  if (B == 0) return;
  const int64_t ns = decode_nsplit(B, Hkv, nsplit);
  float* po = nullptr;
  float* pml = nullptr;
  if (ns > 1) {
    TORCH_CHECK(workspace.scalar_type() == at::kFloat && workspace.numel() >= (int64_t)B * Hq * ns * (D + 2),
                "decode workspace too small");
    po = workspace.data_ptr<float>();
    pml = po + (int64_t)B * Hq * ns * D;
  }
  auto stream = at::hip::getCurrentHIPStream();
  // Wave-per-pair (WPP=1) once the (seq, kv-head) pairs alone fill every wave slot of
  // the chip (256 CUs x 8 resident waves): each wave then streams its whole context
  // with no LDS merge and no idle waves in a workgroup whose block count is not a
  // multiple of 4.  Smaller batches keep 4 waves per pair (and split long contexts).
  static const int env_wpp = getenv("LS_ATTN_WPP") ? atoi(getenv("LS_ATTN_WPP")) : 0;
  static const bool pipe = getenv("LS_ATTN_PIPE") ? atoi(getenv("LS_ATTN_PIPE")) != 0 : true;
  const bool rope = ra != nullptr;
  // LS_ATTN_NT (read per launch, A/B inside one process): 0 cached loads, 1 all nt, 2
  // (default) nt except each sequence's first block (the shared template-prefix block).
  // The attention kernel alone is faster all-nt (B = 256 ctx 270..550, one shared first
  // block, cold caches: 67.2 / 72.2 / 73.5 us for 1 / 2 / 0,
  // profiles/r5/attn_shared_first_block_r5ab.log; bench timeline 67.7 vs 70.7 us), but the
  // whole RAG bench ran less GPU time with 2 in both rounds of a same-box A/B (16.55 /
  // 16.63 s vs 16.74 / 17.25 s, ab_head_attn_r5ai.log): the decode GEMMs that follow
  // lose more than the attention gains.
  const char* ent = getenv("LS_ATTN_NT");
  const int attn_nt = ent ? atoi(ent) : 2;
  const RopeArgs rargs = rope ? *ra : RopeArgs{};
  const int wpp = env_wpp == 1 || env_wpp == 4 ? env_wpp : ((int64_t)B * Hkv >= WAVE_SLOTS && ns == 1 ? 1 : 4);
  dim3 grid(B * Hkv, ns);
  const float sl2 = (float)scale * LOG2E;
#define LAUNCH_R(DD, W, P, R)                                                                                 \
  if (attn_nt == 2) LAUNCH_A(DD, W, P, R, 3); else if (attn_nt) LAUNCH_A(DD, W, P, R, 2); else LAUNCH_A(DD, W, P, R, 0)
#define LAUNCH_A(DD, W, P, R, A)                                                                              \
  decode_attn_kernel<DD, W, P, R, A><<<grid, 64 * W, 0, stream>>>(                                            \
      (bf16*)out.data_ptr(), (const bf16*)q.data_ptr(), q_stride, (const bf16*)k_cache.data_ptr(),            \
      (const bf16*)v_cache.data_ptr(), block_tables.data_ptr<int32_t>(), (int)block_tables.size(1),          \
      ctx_lens.data_ptr<int32_t>(), Hkv, G, (int)k_cache.size(0), sl2, (int)min_bps, po, pml, rargs)
#define LAUNCH_P(DD, W, P) \
  if (rope) LAUNCH_R(DD, W, P, true); else LAUNCH_R(DD, W, P, false)
#define LAUNCH_K(DD, W) \
  if (pipe) LAUNCH_P(DD, W, true); else LAUNCH_P(DD, W, false)
#define LAUNCH(DD)                                                                                            \
  if (wpp == 1) { LAUNCH_K(DD, 1); } else { LAUNCH_K(DD, 4); }                                                \
  if (ns > 1)                                                                                                 \
    decode_merge_kernel<DD><<<(B * Hq + 3) / 4, 256, 0, stream>>>((bf16*)out.data_ptr(), po, pml, (int)ns,    \
                                                                  B * Hq, ctx_lens.data_ptr<int32_t>(), Hq,    \
                                                                  (int)min_bps, (int)block_tables.size(1), rope ? 1 : 0)
  if (D == 128) { LAUNCH(128); }
  else if (D == 64) { LAUNCH(64); }
  else TORCH_CHECK(false, "unsupported head dim ", D);
  (void)rope;
#undef LAUNCH_K
#undef LAUNCH_P
#undef LAUNCH_R
#undef LAUNCH_A
#undef LAUNCH
}

void paged_decode_attention(at::Tensor out, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                            at::Tensor block_tables, at::Tensor ctx_lens, double scale, int64_t nsplit,
                            int64_t min_bps, at::Tensor workspace) {
  decode_attention_launch(out, q, k_cache, v_cache, block_tables, ctx_lens, scale, nsplit, min_bps, workspace,
                          nullptr);
}

// Decode-only step with RoPE and the KV-cache write fused in (see RopeArgs above).
// qkv: [B, (Hq + 2 Hkv) D] un-rotated projection rows (not modified); ctx_lens count the
// new token; pos [B] int32 its position; slots [B] int64 its cache slot (-1: not cached).
void paged_decode_attention_rope(at::Tensor out, at::Tensor qkv, at::Tensor pos, at::Tensor cos_sin,
                                 at::Tensor slots, at::Tensor k_cache, at::Tensor v_cache, at::Tensor block_tables,
                                 at::Tensor ctx_lens, double scale, int64_t nsplit, int64_t min_bps,
                                 at::Tensor workspace) {
  TORCH_CHECK(qkv.is_cuda() && qkv.dim() == 2 && qkv.stride(1) == 1, "qkv must be [B, (Hq + 2 Hkv) D]");
  const int64_t Hkv = k_cache.size(1), D = k_cache.size(3), B = ctx_lens.numel();
  TORCH_CHECK(qkv.size(0) == B && out.numel() % (B * D) == 0);
  const int64_t Hq = out.numel() / (B * D);
  TORCH_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "qkv width must be (Hq + 2 Hkv) * D");
  TORCH_CHECK(pos.scalar_type() == at::kInt && pos.is_contiguous() && pos.numel() >= B);
  TORCH_CHECK(slots.scalar_type() == at::kLong && slots.is_contiguous() && slots.numel() >= B);
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() && cos_sin.dim() == 2 &&
              cos_sin.size(1) == D && cos_sin.size(0) >= 1);
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous());
  RopeArgs ra{cos_sin.data_ptr<float>(), pos.data_ptr<int32_t>(), (int)cos_sin.size(0), slots.data_ptr<int64_t>(),
              k_cache.size(0) * BS, (bf16*)k_cache.data_ptr(), (bf16*)v_cache.data_ptr()};
  decode_attention_launch(out, qkv, k_cache, v_cache, block_tables, ctx_lens, scale, nsplit, min_bps, workspace,
                          &ra);
}
