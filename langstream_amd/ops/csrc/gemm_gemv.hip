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

constexpr int EPI_NONE = 0, EPI_SILU = 1;

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
template <int TR, int KCH, int RB, int EPI>
__global__ void __launch_bounds__(256) gemv_kernel(const bf16* __restrict__ x, int T, const bf16* __restrict__ W,
                                                   int N, int K, bf16* __restrict__ out, int ldo) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nchunk = K >> 9;  // K % 512 == 0 (host-checked)
  // ---- x fragments: chunk c of this wave = global chunk c*4 + wv
  u32x4 xr[TR][KCH];
#pragma unroll
  for (int m = 0; m < TR; ++m) {
    const bf16* xm = x + (int64_t)min(m, T - 1) * K;
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      // branch-free tail: a chunk past K reloads the last one and is zeroed by a select, so
      // no load sits behind control flow (which made the compiler drain vmcnt per row)
      const int g = c * 4 + wv;
      const u32x4 v = *reinterpret_cast<const u32x4*>(xm + (min(g, nchunk - 1) << 9) + lane * 8);
      xr[m][c] = g < nchunk ? v : u32x4{0, 0, 0, 0};
    }
  }
  // ---- W rows of this block
  constexpr int HALF = RB / 2;
  const int F = N >> 1;
  const int base = blockIdx.x * (EPI == EPI_SILU ? HALF : RB);
  u32x4 wr[RB][KCH];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int row = EPI == EPI_SILU ? (r < HALF ? base + r : F + base + r - HALF) : base + r;
    const bf16* wrow = W + (int64_t)row * K + lane * 8;
#pragma unroll
    for (int c = 0; c < KCH; ++c)
      wr[r][c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow + (min(c * 4 + wv, nchunk - 1) << 9)));
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
  if (EPI == EPI_SILU) {
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
  } else {
    const int t = threadIdx.x;
    if (t < RB * TR) {
      const int r = t / TR, m = t % TR;
      if (m < T) out[(int64_t)m * ldo + base + r] = (bf16)(red[0][t] + red[1][t] + red[2][t] + red[3][t]);
    }
  }
}

template <int TR, int KCH, int EPI>
void launch_rb(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, int T, int N, int K, hipStream_t st) {
  // the compiler streams W through a rolling window of ~8 loads per wave, so RB sets the
  // rows sharing one x fetch + reduction, not the VGPR count (RB = 2 at K = 14336, T = 4
  // measured 0.7x hipBLASLt; profiles/gemv_bench.log)
  constexpr int RB = KCH <= 3 ? 8 : 4;
  const int rows_per_block = EPI == EPI_SILU ? RB / 2 : RB;
  const int nrows = EPI == EPI_SILU ? N / 2 : N;
  TORCH_CHECK(nrows % rows_per_block == 0, "gemv: output rows must be a multiple of ", rows_per_block);
  gemv_kernel<TR, KCH, RB, EPI><<<nrows / rows_per_block, 256, 0, st>>>(
      (const bf16*)x.data_ptr(), T, (const bf16*)w.data_ptr(), N, K, (bf16*)out.data_ptr(), (int)out.stride(0));
}

template <int TR, int EPI>
void launch_k(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, int T, int N, int K, hipStream_t st) {
  switch ((K + 2047) / 2048) {
    case 1: return launch_rb<TR, 1, EPI>(x, w, out, T, N, K, st);
    case 2: return launch_rb<TR, 2, EPI>(x, w, out, T, N, K, st);
    case 3: return launch_rb<TR, 3, EPI>(x, w, out, T, N, K, st);
    case 4: return launch_rb<TR, 4, EPI>(x, w, out, T, N, K, st);
    case 5: return launch_rb<TR, 5, EPI>(x, w, out, T, N, K, st);
    case 6: return launch_rb<TR, 6, EPI>(x, w, out, T, N, K, st);
    case 7: return launch_rb<TR, 7, EPI>(x, w, out, T, N, K, st);
    default: TORCH_CHECK(false, "gemv: K = ", K, " > 14336 is not supported");
  }
}

template <int EPI>
void gemv_dispatch(at::Tensor out, const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && out.is_cuda(), "gemv: CUDA tensors expected");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  out.scalar_type() == at::kBFloat16, "gemv: bf16 tensors expected");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && x.stride(0) == x.size(1) && w.is_contiguous(),
              "gemv: contiguous x [T, K] and W [N, K] expected");
  const int T = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemv: K mismatch");
  TORCH_CHECK(T >= 1 && T <= 4, "gemv: 1 <= T <= 4");
  TORCH_CHECK(K % 512 == 0, "gemv: K must be a multiple of 512");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == T && out.stride(1) == 1 && out.size(1) == (EPI ? N / 2 : N),
              "gemv: bad output shape");
  auto st = at::hip::getCurrentHIPStream();
  switch (T) {
    case 1: return launch_k<1, EPI>(x, w, out, T, N, K, st);
    case 2: return launch_k<2, EPI>(x, w, out, T, N, K, st);
    default: return launch_k<4, EPI>(x, w, out, T, N, K, st);
  }
}

}  // namespace

// out[T, N] = x @ w^T for 1 <= T <= 4 (bf16, K % 512 == 0, K <= 14336, N % 8 == 0).
void gemv(at::Tensor out, at::Tensor x, at::Tensor w) { gemv_dispatch<EPI_NONE>(out, x, w); }

// out[T, F] = silu(x @ w[:F]^T) * (x @ w[F:]^T) for the fused gate_up weight w [2F, K].
void gemv_silu(at::Tensor out, at::Tensor x, at::Tensor w) { gemv_dispatch<EPI_SILU>(out, x, w); }

// Whether the GEMV path supports this weight (host-side shape rule used by the runner).
bool gemv_supported(const at::Tensor& w, bool silu) {
  const int64_t N = w.size(0), K = w.size(1);
  return K % 512 == 0 && K <= 14336 && (silu ? (N % 8 == 0) : (N % 8 == 0));
}
