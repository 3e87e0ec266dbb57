// Small-batch decode projection GEMV: out[T, N] = x[T, K] @ W[N, K]^T for T <= 4 (bf16).
//
// At batch 1-4 a decode step is pure weight streaming (Llama-3-8B: 15 GB of bf16 weights
// per step, 2.4 ms at HBM speed).  hipBLASLt's small-M tiles and the MFMA skinny kernel
// (gemm_skinny.hip, which stages x through LDS for M >= 16) reach 3-5 TB/s here
// (profiles/prof_b1_kernel_stats.csv); this kernel follows the guide's GEMV row
// (cdna_hip_programming.md, "GEMV / M <= 16 decode weights"): every W byte is loaded once,
// straight into VGPRs with non-temporal 16-B loads, all of a block's loads issued before
// the first use (deep MLP, one late vmcnt), x kept in registers for the whole block, and
// the dot products on v_dot2c_f32_bf16.
//
// Decomposition: a 256-thread workgroup owns RB rows of W.  K is cut into 512-element
// chunks (64 lanes x 8 bf16 = 1 KB per wave load); chunk c belongs to wave c % 4, so the
// four waves of a block stream four adjacent KBs of every row.  Each lane accumulates
// RB x TR partial sums; a 64-lane xor-shuffle reduction and a 4-wave LDS combine finish
// them.  Grid = N / RB blocks (>= 512 for every Llama projection: qkv 768, o 512,
// gate_up 3584, down 1024).
//
// Epilogues: EPI_NONE writes bf16 rows; EPI_SILU treats W as the fused [gate; up]
// projection [2F, K], gives each block RB/2 gate rows and the matching RB/2 up rows and
// writes silu(gate) * up as [T, F] (replacing the gate_up GEMM + silu_and_mul pair).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int EPI_NONE = 0, EPI_SILU = 1, EPI_ADDNORM = 2, EPI_QKV = 3;

// EPI_ADDNORM operands: after the projection, residual = bf16(out + residual) and
// out = bf16(rmsnorm(residual) * norm_w) -- the fused_add_rmsnorm of norm.hip -- done by
// the block that finishes last (agent-scope release/acquire ticket on `counter`, which the
// last block resets to 0 for the next launch; the buffer is zero-initialised once).
struct AddNorm {
  bf16* residual;
  const bf16* norm_w;
  unsigned int* counter;
  float eps;
};

// PRO (prologue) operands: the GEMV input is x = rmsnorm(o + res) * norm_w, computed in
// the kernel; block 0 writes res_out = bf16(o + res) (a different buffer than res: the
// other blocks are still reading res).
struct ProNorm {
  const bf16* o;
  const bf16* res;
  bf16* res_out;
  const bf16* norm_w;
  float eps;
};

// EPI_QKV operands: W is the fused qkv projection [(Hq + 2 Hkv) * D, K]; each block owns
// RB/2 rotary pairs (d, d + D/2) of one head, so the epilogue applies RoPE to q and k heads
// and writes k to the paged K cache [NB, Hkv, BS, D] and v transposed to the V cache
// [NB, Hkv, BS/8, D, 8] -- the rope_cache kernel of rope.hip, fused (same bf16 rounding).
struct QkvEpi {
  const int32_t* pos;
  const float* cos_sin;  // [max_pos, D]: cols [0, D/2) cos, [D/2, D) sin
  const int64_t* slots;  // [T] cache slot, -1 = not cached
  bf16* kc;
  bf16* vc;
  int64_t nslots;
  int Hq, Hkv, BS, D, max_pos, apply_rope;
};

// 8-element bf16 dot on v_dot2c_f32_bf16.  The pairs are taken with shufflevector on the
// whole 16-B value: bit-casting extracted u32 elements (a.y, a[1], ...) is miscompiled by
// this hipcc (every pair reads element 0; checked in the ISA).
__device__ __forceinline__ float dot8(u32x4 a, u32x4 b, float acc) {
  const bf16x8 av = __builtin_bit_cast(bf16x8, a), bv = __builtin_bit_cast(bf16x8, b);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av, av, 0, 1), __builtin_shufflevector(bv, bv, 0, 1),
                                        acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av, av, 2, 3), __builtin_shufflevector(bv, bv, 2, 3),
                                        acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av, av, 4, 5), __builtin_shufflevector(bv, bv, 4, 5),
                                        acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av, av, 6, 7), __builtin_shufflevector(bv, bv, 6, 7),
                                        acc, false);
  return acc;
}

// TR: rows of x handled (x rows >= T are clamped to T-1 and not stored); KCH: 512-element
// chunks per wave (ceil(K / 2048)); RB: W rows per block.
template <int TR, int KCH, int RB, int EPI, bool PRO>
__global__ void __launch_bounds__(256) gemv_kernel(const bf16* __restrict__ x, int T, const bf16* __restrict__ W,
                                                   int N, int K, bf16* __restrict__ out, int ldo, AddNorm an,
                                                   ProNorm pro, QkvEpi qe) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nchunk = K >> 9;  // K % 512 == 0 (host-checked)
  constexpr int HALF = RB / 2;
  const int F = N >> 1;
  const int base = blockIdx.x * (EPI == EPI_SILU ? HALF : RB);
  // EPI_QKV: head and first rotary index of this block's HALF pairs
  const int qk_bph = EPI == EPI_QKV ? (qe.D / 2) / HALF : 1;
  const int qk_head = blockIdx.x / qk_bph, qk_j0 = (blockIdx.x % qk_bph) * HALF;
  auto w_row = [&](int r) -> int {
    if constexpr (EPI == EPI_SILU) return r < HALF ? base + r : F + base + r - HALF;
    else if constexpr (EPI == EPI_QKV) return qk_head * qe.D + (r < HALF ? qk_j0 + r : qe.D / 2 + qk_j0 + r - HALF);
    else return base + r;
  };
  u32x4 wr[RB][KCH];
  u32x4 xr[TR][KCH];
  if constexpr (PRO) {
    // ---- prologue: x = rmsnorm(o + residual) * norm_w, recomputed by every block from
    // the L2-resident [T, K] operands (16 KB per token at K = 4096 against >= 64 KB of W
    // per block); block 0 also writes the new residual stream.  Load order matters: vmcnt
    // retires loads in issue order, so the o / residual / norm_w fragments are all loaded
    // BEFORE the W stream is issued -- an operand loaded after W cannot be waited for
    // without draining every W load first (that order, with the residual store inside the
    // loop, measured 67 us for gate_up at T = 4 against 42 us without a prologue).
    u32x4 ov[TR][KCH], rv[TR][KCH];
    uint4 nv[KCH];
#pragma unroll
    for (int m = 0; m < TR; ++m) {
      const int64_t mo = (int64_t)min(m, T - 1) * K;
#pragma unroll
      for (int c = 0; c < KCH; ++c) {
        const int off = (min(c * 4 + wv, nchunk - 1) << 9) + lane * 8;
        ov[m][c] = *reinterpret_cast<const u32x4*>(pro.o + mo + off);
        rv[m][c] = *reinterpret_cast<const u32x4*>(pro.res + mo + off);
      }
    }
#pragma unroll
    for (int c = 0; c < KCH; ++c) nv[c] = ld16(pro.norm_w + (min(c * 4 + wv, nchunk - 1) << 9) + lane * 8);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int row = w_row(r);
      const bf16* wrow = W + (int64_t)row * K + lane * 8;
#pragma unroll
      for (int c = 0; c < KCH; ++c)
        wr[r][c] =
            __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow + (min(c * 4 + wv, nchunk - 1) << 9)));
    }
    // pin the issue order: the scheduler otherwise hoists the norm arithmetic (and with it
    // the wait for o / residual) above the W loads, exposing one L2 round trip per block;
    // the empty asm "redefines" the fragments after the W stream is out
    asm volatile("" ::: "memory");
#pragma unroll
    for (int m = 0; m < TR; ++m)
#pragma unroll
      for (int c = 0; c < KCH; ++c) asm volatile("" : "+v"(ov[m][c]), "+v"(rv[m][c]));
    __shared__ float pro_red[4][TR];
    float ss[TR];
#pragma unroll
    for (int m = 0; m < TR; ++m) {
      ss[m] = 0.f;
#pragma unroll
      for (int c = 0; c < KCH; ++c) {
        float a[8], b[8];
        unpack8(__builtin_bit_cast(uint4, ov[m][c]), a);
        unpack8(__builtin_bit_cast(uint4, rv[m][c]), b);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += b[j];
        const uint4 packed = pack8(a);  // the residual stream stays bf16: round once
        unpack8(packed, a);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += a[j] * a[j];
        ss[m] += c * 4 + wv < nchunk ? s : 0.f;
        xr[m][c] = __builtin_bit_cast(u32x4, packed);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int m = 0; m < TR; ++m) ss[m] += __shfl_xor(ss[m], o, 64);
    if (lane == 0) {
#pragma unroll
      for (int m = 0; m < TR; ++m) pro_red[wv][m] = ss[m];
    }
    if (blockIdx.x == 0) {
#pragma unroll
      for (int m = 0; m < TR; ++m)
#pragma unroll
        for (int c = 0; c < KCH; ++c) {
          const int g = c * 4 + wv;
          if (m < T && g < nchunk)
            st16(pro.res_out + (int64_t)m * K + (g << 9) + lane * 8, __builtin_bit_cast(uint4, xr[m][c]));
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int m = 0; m < TR; ++m)
      ss[m] = rsqrtf((pro_red[0][m] + pro_red[1][m] + pro_red[2][m] + pro_red[3][m]) / K + pro.eps);
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      const int g = c * 4 + wv;
      float wf[8];
      unpack8(nv[c], wf);
#pragma unroll
      for (int m = 0; m < TR; ++m) {
        float a[8];
        unpack8(__builtin_bit_cast(uint4, xr[m][c]), a);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[j] * ss[m] * wf[j];
        xr[m][c] = g < nchunk ? __builtin_bit_cast(u32x4, pack8(a)) : u32x4{0, 0, 0, 0};
      }
    }
  } else {
    // ---- x fragments: chunk c of this wave = global chunk c*4 + wv
#pragma unroll
    for (int m = 0; m < TR; ++m) {
      const bf16* xm = x + (int64_t)min(m, T - 1) * K;
#pragma unroll
      for (int c = 0; c < KCH; ++c) {
        // branch-free tail: a chunk past K reloads the last one and is zeroed by a select, so
        // no load sits behind control flow (which made the compiler drain vmcnt per row)
        xr[m][c] = *reinterpret_cast<const u32x4*>(xm + (min(c * 4 + wv, nchunk - 1) << 9) + lane * 8);
      }
    }
    // ---- W rows of this block
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int row = w_row(r);
      const bf16* wrow = W + (int64_t)row * K + lane * 8;
#pragma unroll
      for (int c = 0; c < KCH; ++c)
        wr[r][c] =
            __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow + (min(c * 4 + wv, nchunk - 1) << 9)));
    }
    // Left alone, the scheduler interleaves the dots with the W loads (a rolling window of
    // ~4-8 loads per wave behind the TR x fragments), which at TR = 4 halves the bytes in
    // flight: qkv / o at T = 4 ran at ~3 TB/s.  Where x + W fit in ~128 VGPRs, every W load
    // is issued before the first dot (the empty asm "redefines" the fragments after them).
    if constexpr ((RB + TR) * KCH * 4 <= 128) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int c = 0; c < KCH; ++c) asm volatile("" : "+v"(wr[r][c]));
#pragma unroll
      for (int m = 0; m < TR; ++m)
#pragma unroll
        for (int c = 0; c < KCH; ++c) asm volatile("" : "+v"(xr[m][c]));
    }
#pragma unroll
    for (int m = 0; m < TR; ++m)
#pragma unroll
      for (int c = 0; c < KCH; ++c) xr[m][c] = c * 4 + wv < nchunk ? xr[m][c] : u32x4{0, 0, 0, 0};
  }
  float acc[RB][TR];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int m = 0; m < TR; ++m) {
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < KCH; ++c) a = dot8(wr[r][c], xr[m][c], a);
      acc[r][m] = a;
    }
  // ---- reduce over the 64 lanes, then over the 4 waves through LDS
  // all RB * TR sums advance one xor step together: one LDS round trip per step
  __shared__ float red[4][RB * TR];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int m = 0; m < TR; ++m) acc[r][m] += __shfl_xor(acc[r][m], o, 64);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int m = 0; m < TR; ++m) red[wv][r * TR + m] = acc[r][m];
  }
  __syncthreads();
  if constexpr (EPI == EPI_QKV) {
    const int t = threadIdx.x;
    if (t < HALF * TR) {
      const int u = t / TR, m = t % TR;
      if (m < T) {
        const int hd = qe.D / 2;
        const int i1 = u * TR + m, i2 = (u + HALF) * TR + m;
        // the unfused path rounds the projection to bf16 before rotating
        float a = (float)(bf16)(red[0][i1] + red[1][i1] + red[2][i1] + red[3][i1]);
        float b = (float)(bf16)(red[0][i2] + red[1][i2] + red[2][i2] + red[3][i2]);
        const int d1 = qk_j0 + u, d2 = hd + qk_j0 + u;
        const bool rot = qe.apply_rope && qk_head < qe.Hq + qe.Hkv;
        if (rot) {
          const int p = min(max(qe.pos[m], 0), qe.max_pos - 1);
          const float co = qe.cos_sin[(int64_t)p * qe.D + d1], si = qe.cos_sin[(int64_t)p * qe.D + hd + d1];
          const float x1 = a, x2 = b;
          a = x1 * co - x2 * si;
          b = x2 * co + x1 * si;
        }
        const bf16 ab = (bf16)a, bb = (bf16)b;
        bf16* orow = out + (int64_t)m * ldo + qk_head * qe.D;
        orow[d1] = ab;
        orow[d2] = bb;
        const int64_t s = qe.slots[m];
        if (qk_head >= qe.Hq && s >= 0 && s < qe.nslots) {
          const int64_t blk = s / qe.BS, off = s - blk * qe.BS;
          if (qk_head < qe.Hq + qe.Hkv) {
            bf16* kd = qe.kc + ((blk * qe.Hkv + (qk_head - qe.Hq)) * qe.BS + off) * qe.D;
            kd[d1] = ab;
            kd[d2] = bb;
          } else {
            bf16* vd = qe.vc + (blk * qe.Hkv + (qk_head - qe.Hq - qe.Hkv)) * (int64_t)qe.D * qe.BS;
            vd[vt_off(d1, (int)off, qe.D)] = ab;
            vd[vt_off(d2, (int)off, qe.D)] = bb;
          }
        }
      }
    }
  } else if (EPI == EPI_SILU) {
    const int t = threadIdx.x;
    if (t < HALF * TR) {
      const int r = t / TR, m = t % TR;
      if (m < T) {
        const float g = red[0][r * TR + m] + red[1][r * TR + m] + red[2][r * TR + m] + red[3][r * TR + m];
        const int ru = (r + HALF) * TR + m;
        const float u = red[0][ru] + red[1][ru] + red[2][ru] + red[3][ru];
        const float gb = (float)(bf16)g, ub = (float)(bf16)u;  // round as the unfused GEMM output would
        out[(int64_t)m * ldo + base + r] = (bf16)(gb / (1.f + __expf(-gb)) * ub);
      }
    }
  } else if (EPI == EPI_ADDNORM) {
    // hand-off payload stored write-through (sc1: 8-byte agent-scope atomic stores of 4 packed
    // bf16), so no block needs a release fence (an agent release = an L2 writeback in each of
    // the 512-1024 blocks measured 4.3 vs 3.5 ms per batch-1 step); guide §6 Guideline 16 R1
    const int t = threadIdx.x;
    constexpr int G = RB / 4;  // 8-byte groups per output row
    if (t < TR * G) {
      const int m = t / G, gq = t % G;
      if (m < T) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = (gq * 4 + j) * TR + m;
          v[j] = (bf16)(red[0][i] + red[1][i] + red[2][i] + red[3][i]);
        }
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(out + (int64_t)m * ldo + base + gq * 4),
                           __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
    const int t = threadIdx.x;
    if (t < RB * TR) {
      const int r = t / TR, m = t % TR;
      if (m < T) out[(int64_t)m * ldo + base + r] = (bf16)(red[0][t] + red[1][t] + red[2][t] + red[3][t]);
    }
  }
  if constexpr (EPI == EPI_ADDNORM) {
    // ---- ticket: every storing wave drains, then one relaxed agent-scope add; the last
    // block acquires and runs the add + RMSNorm
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned int prev = __hip_atomic_fetch_add(an.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      red[0][0] = (prev == gridDim.x - 1) ? 1.f : 0.f;  // "I am last", through the one LDS array
      if (prev == gridDim.x - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (red[0][0] == 0.f) return;
    __syncthreads();  // every thread has read the flag before red is reused below
    for (int m = 0; m < T; ++m) {
      bf16* orow = out + (int64_t)m * ldo;
      bf16* rrow = an.residual + (int64_t)m * N;
      float ss = 0.f;
      for (int c = threadIdx.x; c < (N >> 3); c += blockDim.x) {
        float a[8], b[8];
        unpack8(ld16(orow + c * 8), a);
        unpack8(ld16(rrow + c * 8), b);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += b[j];
        const uint4 packed = pack8(a);
        st16(rrow + c * 8, packed);
        unpack8(packed, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
      }
      ss = wave_sum(ss);
      __syncthreads();
      if (lane == 0) red[1][wv] = ss;
      __syncthreads();
      const float inv = rsqrtf((red[1][0] + red[1][1] + red[1][2] + red[1][3]) / N + an.eps);
      for (int c = threadIdx.x; c < (N >> 3); c += blockDim.x) {
        float a[8], wf[8];
        unpack8(ld16(rrow + c * 8), a);  // this thread's own rounded residual
        unpack8(ld16(an.norm_w + c * 8), wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[j] * inv * wf[j];
        st16(orow + c * 8, pack8(a));
      }
    }
    if (threadIdx.x == 0) __hip_atomic_store(an.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct Extra {
  AddNorm an{};
  ProNorm pro{};
  QkvEpi qe{};
};

template <int TR, int KCH, int EPI, bool PRO>
void launch_rb(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, int T, int N, int K, hipStream_t st,
               const Extra& ex) {
  // RB sets the rows sharing one x fetch + reduction.  Where x + W fit in ~128 VGPRs
  // (K <= 4096 at T <= 4) every W load is pinned ahead of the dots (see the kernel); at
  // larger K the compiler streams W through a rolling window of loads per wave instead,
  // so RB does not set the VGPR count there (RB = 2 at K = 14336, T = 4 measured 0.7x
  // hipBLASLt; profiles/gemv_bench.log)
  constexpr int RB = KCH <= 3 ? 8 : 4;
  const int rows_per_block = EPI == EPI_SILU ? RB / 2 : RB;
  const int nrows = EPI == EPI_SILU ? N / 2 : N;
  TORCH_CHECK(nrows % rows_per_block == 0, "gemv: output rows must be a multiple of ", rows_per_block);
  if (EPI == EPI_QKV) TORCH_CHECK((ex.qe.D / 2) % (RB / 2) == 0, "gemv_qkv: head_dim / 2 must divide by ", RB / 2);
  gemv_kernel<TR, KCH, RB, EPI, PRO><<<nrows / rows_per_block, 256, 0, st>>>(
      (const bf16*)x.data_ptr(), T, (const bf16*)w.data_ptr(), N, K, (bf16*)out.data_ptr(), (int)out.stride(0), ex.an,
      ex.pro, ex.qe);
}

template <int TR, int EPI, bool PRO>
void launch_k(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, int T, int N, int K, hipStream_t st,
              const Extra& ex) {
  switch ((K + 2047) / 2048) {
    case 1: return launch_rb<TR, 1, EPI, PRO>(x, w, out, T, N, K, st, ex);
    case 2: return launch_rb<TR, 2, EPI, PRO>(x, w, out, T, N, K, st, ex);
    case 3: return launch_rb<TR, 3, EPI, PRO>(x, w, out, T, N, K, st, ex);
    case 4: return launch_rb<TR, 4, EPI, PRO>(x, w, out, T, N, K, st, ex);
    case 5: return launch_rb<TR, 5, EPI, PRO>(x, w, out, T, N, K, st, ex);
    case 6: return launch_rb<TR, 6, EPI, PRO>(x, w, out, T, N, K, st, ex);
    case 7: return launch_rb<TR, 7, EPI, PRO>(x, w, out, T, N, K, st, ex);
    default: TORCH_CHECK(false, "gemv: K = ", K, " > 14336 is not supported");
  }
}

template <int EPI, bool PRO = false>
void gemv_dispatch(at::Tensor out, const at::Tensor& x, const at::Tensor& w, const Extra& ex = Extra{}) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && out.is_cuda(), "gemv: CUDA tensors expected");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  out.scalar_type() == at::kBFloat16, "gemv: bf16 tensors expected");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && x.stride(0) == x.size(1) && w.is_contiguous(),
              "gemv: contiguous x [T, K] and W [N, K] expected");
  const int T = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemv: K mismatch");
  TORCH_CHECK(T >= 1 && T <= 4, "gemv: 1 <= T <= 4");
  TORCH_CHECK(K % 512 == 0, "gemv: K must be a multiple of 512");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == T && out.stride(1) == 1 &&
                  out.size(1) == (EPI == EPI_SILU ? N / 2 : N), "gemv: bad output shape");
  auto st = at::hip::getCurrentHIPStream();
  switch (T) {
    case 1: return launch_k<1, EPI, PRO>(x, w, out, T, N, K, st, ex);
    case 2: return launch_k<2, EPI, PRO>(x, w, out, T, N, K, st, ex);
    default: return launch_k<4, EPI, PRO>(x, w, out, T, N, K, st, ex);
  }
}

ProNorm make_pro(const at::Tensor& o, const at::Tensor& res, const at::Tensor& res_out, const at::Tensor& norm_w,
                 double eps) {
  TORCH_CHECK(res.scalar_type() == at::kBFloat16 && res_out.scalar_type() == at::kBFloat16 &&
                  norm_w.scalar_type() == at::kBFloat16, "gemv_norm: bf16 operands");
  TORCH_CHECK(res.is_contiguous() && res_out.is_contiguous() && norm_w.is_contiguous() && o.is_contiguous(),
              "gemv_norm: contiguous operands");
  TORCH_CHECK(res.sizes() == o.sizes() && res_out.sizes() == o.sizes() && norm_w.numel() == o.size(1),
              "gemv_norm: o / residual / norm shapes");
  TORCH_CHECK(res_out.data_ptr() != res.data_ptr(), "gemv_norm: res_out must not alias res");
  return ProNorm{(const bf16*)o.data_ptr(), (const bf16*)res.data_ptr(), (bf16*)res_out.data_ptr(),
                 (const bf16*)norm_w.data_ptr(), (float)eps};
}

QkvEpi make_qkv(const at::Tensor& out, const at::Tensor& pos, const at::Tensor& cos_sin, const at::Tensor& slots,
                const at::Tensor& kc, const at::Tensor& vc, int64_t Hq, int64_t Hkv, bool apply_rope) {
  TORCH_CHECK(pos.scalar_type() == at::kInt && slots.scalar_type() == at::kLong && cos_sin.scalar_type() == at::kFloat &&
                  cos_sin.is_contiguous(), "gemv_qkv: pos int32, slots int64, cos_sin f32");
  TORCH_CHECK(kc.dim() == 4 && vc.dim() == 5 && kc.scalar_type() == at::kBFloat16 && vc.scalar_type() == at::kBFloat16,
              "gemv_qkv: paged caches [NB, Hkv, BS, D] / [NB, Hkv, BS/8, D, 8] bf16");
  const int D = kc.size(3), BS = kc.size(2);
  TORCH_CHECK(kc.size(1) == Hkv && vc.size(1) == Hkv && vc.size(2) == BS / 8 && vc.size(3) == D && vc.size(4) == 8 &&
                  cos_sin.size(1) == D, "gemv_qkv: cache / rope table shapes");
  TORCH_CHECK(out.size(1) == (Hq + 2 * Hkv) * D && pos.numel() == out.size(0) && slots.numel() == out.size(0),
              "gemv_qkv: qkv / pos / slots shapes");
  return QkvEpi{pos.data_ptr<int32_t>(), cos_sin.data_ptr<float>(), slots.data_ptr<int64_t>(), (bf16*)kc.data_ptr(),
                (bf16*)vc.data_ptr(), kc.size(0) * (int64_t)BS, (int)Hq, (int)Hkv, BS, D, (int)cos_sin.size(0),
                apply_rope ? 1 : 0};
}

template <int EPI>
void gemv_norm_dispatch(at::Tensor out, const at::Tensor& o, const at::Tensor& res, at::Tensor res_out,
                        const at::Tensor& norm_w, double eps, const at::Tensor& w) {
  Extra ex;
  ex.pro = make_pro(o, res, res_out, norm_w, eps);
  gemv_dispatch<EPI, true>(out, o, w, ex);
}

}  // namespace

// out[T, N] = x @ w^T for 1 <= T <= 4 (bf16, K % 512 == 0, K <= 14336, N % 8 == 0).
void gemv(at::Tensor out, at::Tensor x, at::Tensor w) { gemv_dispatch<EPI_NONE>(out, x, w); }

// out[T, F] = silu(x @ w[:F]^T) * (x @ w[F:]^T) for the fused gate_up weight w [2F, K].
void gemv_silu(at::Tensor out, at::Tensor x, at::Tensor w) { gemv_dispatch<EPI_SILU>(out, x, w); }

// Prologue-fused forms: the input is x = rmsnorm(o + res) * norm_w (the fused_add_rmsnorm
// that follows the previous projection), res_out = bf16(o + res).
void gemv_norm(at::Tensor out, at::Tensor o, at::Tensor res, at::Tensor res_out, at::Tensor norm_w, double eps,
               at::Tensor w) {
  gemv_norm_dispatch<EPI_NONE>(out, o, res, res_out, norm_w, eps, w);
}
void gemv_silu_norm(at::Tensor out, at::Tensor o, at::Tensor res, at::Tensor res_out, at::Tensor norm_w, double eps,
                    at::Tensor w) {
  gemv_norm_dispatch<EPI_SILU>(out, o, res, res_out, norm_w, eps, w);
}

// out = rmsnorm(residual += x @ w^T) * norm_w with the rounding of gemv + fused_add_rmsnorm;
// `counter` is a zero-initialised int32 word owned by the caller (one launch at a time).
void gemv_add_rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor residual, at::Tensor norm_w,
                      double eps, at::Tensor counter) {
  TORCH_CHECK(residual.scalar_type() == at::kBFloat16 && norm_w.scalar_type() == at::kBFloat16 &&
                  residual.is_contiguous() && norm_w.is_contiguous() && out.is_contiguous(),
              "gemv_add_rmsnorm: bf16 contiguous operands");
  TORCH_CHECK(residual.numel() == out.numel() && norm_w.numel() == w.size(0), "gemv_add_rmsnorm: shapes");
  TORCH_CHECK(counter.is_cuda() && counter.scalar_type() == at::kInt && counter.numel() >= 1, "counter: int32");
  Extra ex;
  ex.an = AddNorm{(bf16*)residual.data_ptr(), (const bf16*)norm_w.data_ptr(), (unsigned int*)counter.data_ptr(),
                  (float)eps};
  gemv_dispatch<EPI_ADDNORM>(out, x, w, ex);
}

// qkv projection with RoPE + paged K/V cache writes fused into the epilogue (rope_and_cache
// of rope.hip).  With `o` given (defined tensor), the input is the prologue norm of
// gemv_norm (x ignored); else x is the normalised input.
void gemv_qkv(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots,
              at::Tensor k_cache, at::Tensor v_cache, int64_t Hq, int64_t Hkv, bool apply_rope,
              c10::optional<at::Tensor> o, c10::optional<at::Tensor> res, c10::optional<at::Tensor> res_out,
              c10::optional<at::Tensor> norm_w, double eps) {
  Extra ex;
  ex.qe = make_qkv(out, pos, cos_sin, slots, k_cache, v_cache, Hq, Hkv, apply_rope);
  if (o.has_value()) {
    TORCH_CHECK(res.has_value() && res_out.has_value() && norm_w.has_value(), "gemv_qkv: prologue operands");
    ex.pro = make_pro(*o, *res, *res_out, *norm_w, eps);
    gemv_dispatch<EPI_QKV, true>(out, *o, w, ex);
  } else {
    gemv_dispatch<EPI_QKV, false>(out, x, w, ex);
  }
}

// Whether the GEMV path supports this weight (host-side shape rule used by the runner).
bool gemv_supported(const at::Tensor& w, bool silu) {
  const int64_t N = w.size(0), K = w.size(1);
  return K % 512 == 0 && K <= 14336 && (silu ? (N % 8 == 0) : (N % 8 == 0));
}
