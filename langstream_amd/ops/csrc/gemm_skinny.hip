// Decode-shaped ("skinny") GEMM on MFMA for gfx950:  C[M, N] = X[M, K] . W[N, K]^T
// with M <= 256 (one decode step's tokens) and a large weight W streamed from HBM once.
//
// Why not hipBLASLt here: at M = 256 its picks for the Llama-3-8B projections leave the
// chip under-filled (qkv N=6144 -> 192 long-K workgroups, o/down N=4096 -> 128-256)
// and run 3-4.6x above the weight-streaming floor (tools/gemm_tune.py,
// profiles/gemm_tune_decode_shapes.log).  This kernel:
//   * tiles BM(M) x 128(N) x 64(K), BM = 64/128/256 by batch; one wave per 64x64 sub-tile
//     (4x4 MFMA 16x16x32 accumulators), so the whole decode batch shares each W tile;
//   * both operands are K-contiguous (W is [N, K], the natural B^T layout), so every
//     MFMA fragment is one 16-B ds_read_b128 from a padded LDS row (144 B: the 16 rows
//     a quarter-wave reads land on 16 disjoint 4-bank groups);
//   * global -> registers -> LDS, double-buffered LDS with the next tile's global loads
//     in flight during the MFMAs: one barrier per K-step (a second register set that
//     issues loads two steps ahead measured 5-40 % SLOWER: profiles/skinny_gemm_v3_*);
//   * split-K over gridDim.y so small-N shapes still launch >= 512 workgroups; partials
//     go to an f32 workspace and the reduction kernel applies the epilogue;
//   * XCD-aware order: the M-tiles of one N-tile (which read the same W tile) are
//     consecutive logical ids on one XCD, so W comes from HBM once and then from L2;
//   * fused epilogues: SiLU(gate) * up for the gate_up projection (the workgroup's 128
//     columns are 64 gate rows + the matching 64 up rows of W), and residual-add +
//     RMSNorm in the split-K reduction for o_proj / down_proj.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

constexpr int BN = 128, BK = 64;
constexpr int LDA = BK + 8;             // padded LDS row, elements (144 B)

enum { EPI_STORE = 0, EPI_PARTIAL = 1, EPI_SILU = 2 };

// Workgroup tile BM x 128 (BM = 64 / 128 / 256), one wave per 64 x 64 sub-tile
// (BM/64 x 2 waves), each wave 4 x 4 MFMA 16x16x32 accumulators.
template <int BM, int EPI>
__global__ void __launch_bounds__(BM * 2) skinny_gemm_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                             const bf16* __restrict__ w, int M, int N, int K,
                                                             int k_per_split, bf16* __restrict__ out, int64_t ldo,
                                                             float* __restrict__ part, int MT, int silu_F) {
  constexpr int NT_ = BM * 2;                 // threads
  constexpr int XS = BM * LDA, WS = BN * LDA;
  constexpr int XC = BM * 8 / NT_;            // 16-B X chunks per thread per K-step (= 4)
  constexpr int WC = BN * 8 / NT_;            // 16-B W chunks per thread per K-step
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * (XS + WS)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = logical % MT, nt = logical / MT;
  const int m0 = mt * BM;
  const int kbeg = blockIdx.y * k_per_split;
  const int nk = k_per_split / BK;

  const bf16* xp[XC];
  bool xok[XC];
#pragma unroll
  for (int i = 0; i < XC; ++i) {
    const int q = tid + NT_ * i, row = q >> 3, kc = q & 7;
    xok[i] = m0 + row < M;
    xp[i] = x + (int64_t)(xok[i] ? m0 + row : 0) * ldx + kbeg + kc * 8;
  }
  const bf16* wp[WC];
#pragma unroll
  for (int i = 0; i < WC; ++i) {
    const int q = tid + NT_ * i, row = q >> 3, kc = q & 7;
    int wrow;
    if (EPI == EPI_SILU) wrow = row < 64 ? nt * 64 + row : silu_F + nt * 64 + (row - 64);
    else wrow = nt * BN + row;
    wp[i] = w + (int64_t)wrow * K + kbeg + kc * 8;
  }
  uint4 rx[XC], rw[WC];
  auto gload = [&](int kt) {
    const int ko = kt * BK;
#pragma unroll
    for (int i = 0; i < XC; ++i) rx[i] = xok[i] ? ld16(xp[i] + ko) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < WC; ++i) rw[i] = ld16(wp[i] + ko);
  };
  auto lstore = [&](int buf) {
    bf16* lx = lds + buf * (XS + WS);
    bf16* lw = lx + XS;
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const int q = tid + NT_ * i;
      st16(lx + (q >> 3) * LDA + (q & 7) * 8, rx[i]);
    }
#pragma unroll
    for (int i = 0; i < WC; ++i) {
      const int q = tid + NT_ * i;
      st16(lw + (q >> 3) * LDA + (q & 7) * 8, rw[i]);
    }
  };

  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  // local W row (= output column inside the tile) of this lane's B fragment for col tile j.
  // SILU: tiles 0,1 are gate columns 32wn..+31 and tiles 2,3 the matching up columns, so
  // acc[i][j] and acc[i][j+2] hold gate and up of the same output element.
  auto bcol = [&](int j) {
    if (EPI == EPI_SILU) return (j < 2 ? 32 * wn + 16 * j : 64 + 32 * wn + 16 * (j - 2)) + fr;
    return 64 * wn + 16 * j + fr;
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  if (nk > 1) gload(1);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const bf16* lx = lds + (kt & 1) * (XS + WS);
    const bf16* lw = lx + XS;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = __builtin_bit_cast(bf16x8, ld16(lx + (64 * wm + 16 * i + fr) * LDA + 32 * ks + fk));
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = __builtin_bit_cast(bf16x8, ld16(lw + bcol(j) * LDA + 32 * ks + fk));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      lstore((kt + 1) & 1);
      if (kt + 2 < nk) gload(kt + 2);
    }
    __syncthreads();
  }

  // acc[i][j][r] = C[64wm + 16i + 4(lane>>4) + r][bcol(j)] (tile-local)
  const int rbase = 64 * wm + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + rbase + 16 * i + r;
      if (m >= M) continue;
      if (EPI == EPI_SILU) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float g = acc[i][j][r], u = acc[i][j + 2][r];
          out[(int64_t)m * ldo + nt * 64 + 32 * wn + 16 * j + fr] = (bf16)(g / (1.f + __expf(-g)) * u);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = nt * BN + bcol(j);
          if (EPI == EPI_STORE) out[(int64_t)m * ldo + n] = (bf16)acc[i][j][r];
          else part[((int64_t)blockIdx.y * M + m) * N + n] = acc[i][j][r];
        }
      }
    }
}

// out[m, n] = bf16(sum_s part[s, m, n]); 4 columns per thread
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                                            bf16* __restrict__ out, int64_t ldo) {
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t total = (int64_t)M * N;
  if (idx >= total) return;
  const int m = idx / N, n = idx - (int64_t)m * N;
  constexpr int SMAX = 8;  // loads of the first 8 partials issued together (see below)
  float4 b[SMAX];
#pragma unroll
  for (int s = 0; s < SMAX; ++s)
    if (s < S) b[s] = *reinterpret_cast<const float4*>(part + (int64_t)s * total + idx);
  float4 a = b[0];
#pragma unroll
  for (int s = 1; s < SMAX; ++s)
    if (s < S) { a.x += b[s].x; a.y += b[s].y; a.z += b[s].z; a.w += b[s].w; }
  for (int s = SMAX; s < S; ++s) {
    const float4 c = *reinterpret_cast<const float4*>(part + (int64_t)s * total + idx);
    a.x += c.x; a.y += c.y; a.z += c.z; a.w += c.w;
  }
  bf16x4 o = {(bf16)a.x, (bf16)a.y, (bf16)a.z, (bf16)a.w};
  *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = o;
}

// One row per workgroup:  v = sum_s part[s, m, :] + residual[m, :];  residual = bf16(v);
// out[m, :] = rmsnorm(bf16(v)) * w.  (Same rounding as fused_add_rmsnorm in norm.hip.)
// NT threads per row: 512 at the decode width (H = 4096, NV = 1) puts the whole row's
// partials (S x 16 KB) in flight at once -- one memory round trip per row instead of two.
template <int NV, int SMAX = 8, int NT = 256>
__global__ void __launch_bounds__(NT) splitk_add_rmsnorm_kernel(const float* __restrict__ part, int S, int M, int H,
                                                                 bf16* __restrict__ residual,
                                                                 const bf16* __restrict__ w, float eps,
                                                                 bf16* __restrict__ out) {
  __shared__ float red[NT / 64];
  const int m = blockIdx.x;
  const int64_t total = (int64_t)M * H;
  float v[NV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (threadIdx.x + NT * i) * 8;
    if (c < H) {
      const float* p = part + (int64_t)m * H + c;
      // Issue the first SMAX partials' loads together (independent, predicated), then
      // reduce: one memory latency instead of S back-to-back ones (S = 8 at decode M).
      float4 b0[SMAX], b1[SMAX];
#pragma unroll
      for (int s = 0; s < SMAX; ++s) {
        if (s < S) {
          b0[s] = *reinterpret_cast<const float4*>(p + s * total);
          b1[s] = *reinterpret_cast<const float4*>(p + s * total + 4);
        }
      }
      float4 a0 = b0[0], a1 = b1[0];
#pragma unroll
      for (int s = 1; s < SMAX; ++s) {
        if (s < S) {
          a0.x += b0[s].x; a0.y += b0[s].y; a0.z += b0[s].z; a0.w += b0[s].w;
          a1.x += b1[s].x; a1.y += b1[s].y; a1.z += b1[s].z; a1.w += b1[s].w;
        }
      }
      for (int s = SMAX; s < S; ++s) {
        const float4 c0 = *reinterpret_cast<const float4*>(p + s * total);
        const float4 c1 = *reinterpret_cast<const float4*>(p + s * total + 4);
        a0.x += c0.x; a0.y += c0.y; a0.z += c0.z; a0.w += c0.w;
        a1.x += c1.x; a1.y += c1.y; a1.z += c1.z; a1.w += c1.w;
      }
      float r[8];
      unpack8(ld16(residual + (int64_t)m * H + c), r);
      v[i][0] = a0.x + r[0]; v[i][1] = a0.y + r[1]; v[i][2] = a0.z + r[2]; v[i][3] = a0.w + r[3];
      v[i][4] = a1.x + r[4]; v[i][5] = a1.y + r[5]; v[i][6] = a1.z + r[6]; v[i][7] = a1.w + r[7];
      const uint4 packed = pack8(v[i]);
      st16(residual + (int64_t)m * H + c, packed);
      unpack8(packed, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / H + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (threadIdx.x + NT * i) * 8;
    if (c < H) {
      float wf[8], o[8];
      unpack8(ld16(w + c), wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * wf[j];
      st16(out + (int64_t)m * H + c, pack8(o));
    }
  }
}

// ---------------------------------------------------------------------------------
// LDS-DMA pipelined variant.  The register-staged kernel above keeps ONE K-step of W in
// flight per CU (16 KB): by Little's law at ~1.5 us loaded HBM latency that streams
// ~10 GB/s per CU, well under the ~24 GB/s a CU can pull (MI355X_MICROARCH 'global_load
// dwordx4 ~10 B/cyc/CU'), so every M = 256 shape was latency-bound.  Here both tiles go
// global -> LDS by global_load_lds_dwordx4 (no VGPRs) into an S-deep ring of 32-deep
// K-stages with S-1 stages in flight (5 x 8 KB of W per CU at BM = 256).
//   * LDS image: rows of 64 B (32 bf16); one wave-instruction fills 16 rows (1 KiB,
//     lane-linear), so the bank swizzle goes on the SOURCE address: LDS chunk p of row r
//     holds global k-chunk p ^ g((r >> 2) & 3) with g = {0, 2, 3, 1}; a fragment read
//     (lane = 16h + fr reads row fr, chunk h) then puts the 16 lanes of each ds_read_b128
//     bank group ({0-3,12-15,20-27}, ... MI355X_MICROARCH LDS table) on 16 distinct
//     16-B bank slots: conflict-free;
//   * one raw s_barrier per K-step after a counted `s_waitcnt vmcnt((S-2) x pieces)`;
//     never __syncthreads() in the loop, which would drain every DMA in flight;
//   * the refill of the buffer read in step kt-1 is issued right after that barrier;
//     past the last stage it re-loads the last stage into a buffer nobody reads again,
//     so the wait count stays a compile-time constant.
constexpr int GBK = 32;

template <int BM, int S, int EPI>
__global__ void __launch_bounds__(BM * 2) skinny_glds_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                             const bf16* __restrict__ w, int M, int N, int K,
                                                             int k_per_split, bf16* __restrict__ out, int64_t ldo,
                                                             float* __restrict__ part, int MT, int silu_F) {
  constexpr int NW = BM / 32;                 // waves
  constexpr int XB = BM * GBK * 2, WB = BN * GBK * 2, SB = XB + WB;
  constexpr int WPW = 8 / NW;                 // 16-row W pieces per wave (X: 2 per wave)
  constexpr int PER = 2 + WPW;                // LDS-DMA instructions per wave per stage
  __shared__ __attribute__((aligned(1024))) char lds[S * SB];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = logical % MT, nt = logical / MT;
  const int m0 = mt * BM;
  const int kbeg = blockIdx.y * k_per_split;
  const int nk = k_per_split / GBK;

  // this lane's source row / swizzled k-chunk inside each 16-row piece
  const int prow = lane >> 2;
  const int sck = ((lane & 3) ^ swz_g(lane >> 4)) * 8;
  const bf16* xs[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 16 * (2 * wid + j) + prow;
    xs[j] = x + (int64_t)min(m0 + row, M - 1) * ldx + kbeg + sck;   // rows >= M: any valid row, never stored
  }
  const bf16* wsrc[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int row = 16 * (wid * WPW + j) + prow;
    int wrow;
    if (EPI == EPI_SILU) wrow = row < 64 ? nt * 64 + row : silu_F + nt * 64 + (row - 64);
    else wrow = nt * BN + row;
    wsrc[j] = w + (int64_t)wrow * K + kbeg + sck;
  }
  auto issue = [&](int kt, int buf) {
    const int ko = kt * GBK;
    char* base = lds + buf * SB;
#pragma unroll
    for (int j = 0; j < 2; ++j) glds16(xs[j] + ko, base + (2 * wid + j) * 1024);
#pragma unroll
    for (int j = 0; j < WPW; ++j) glds16(wsrc[j] + ko, base + XB + (wid * WPW + j) * 1024);
  };

  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, h = lane >> 4;
  const int swz = 16 * (h ^ swz_g(fr >> 2));   // byte offset of this lane's chunk in a 64-B row
  auto bcol = [&](int j) {
    if (EPI == EPI_SILU) return (j < 2 ? 32 * wn + 16 * j : 64 + 32 * wn + 16 * (j - 2)) + fr;
    return 64 * wn + 16 * j + fr;
  };
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
    for (int j = 0; j < 4; ++j) b[j] = __builtin_bit_cast(bf16x8, ld16(lw + bcol(j) * 64 + swz));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    buf = buf + 1 == S ? 0 : buf + 1;
  }
  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup

  const int rbase = 64 * wm + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + rbase + 16 * i + r;
      if (m >= M) continue;
      if (EPI == EPI_SILU) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float g = acc[i][j][r], u = acc[i][j + 2][r];
          out[(int64_t)m * ldo + nt * 64 + 32 * wn + 16 * j + fr] = (bf16)(g / (1.f + __expf(-g)) * u);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = nt * BN + bcol(j);
          if (EPI == EPI_STORE) out[(int64_t)m * ldo + n] = (bf16)acc[i][j][r];
          else part[((int64_t)blockIdx.y * M + m) * N + n] = acc[i][j][r];
        }
      }
    }
}

bool use_glds() {
  static const bool on = [] {
    const char* e = getenv("LS_SKINNY_GLDS");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

int pick_bm(int64_t M) { return M <= 64 ? 64 : (M <= 128 ? 128 : 256); }

// split-K so that (M-tiles x N-tiles x S) workgroups cover the CUs: 256-row tiles are
// 8-wave workgroups (1 per CU), smaller ones run 2 per CU.
int pick_splitk(int bm, int tiles, int K) {
  const int target = bm == 256 ? 256 : 512;
  int s = 1;
  while (tiles * s < target && (K / BK) % (2 * s) == 0 && K / (2 * s) >= 512) s *= 2;
  return s;
}

template <int EPI>
void launch(int bm, dim3 grid, hipStream_t st, const at::Tensor& x, const at::Tensor& w, int M, int N, int K, int kps,
            bf16* out, int64_t ldo, float* part, int MT, int F) {
#define L(KERNEL, BMV, ...)                                                                                    \
  KERNEL<BMV, __VA_ARGS__><<<grid, BMV * 2, 0, st>>>((const bf16*)x.data_ptr(), x.stride(0),                  \
                                                     (const bf16*)w.data_ptr(), M, N, K, kps, out, ldo, part, MT, F)
  if (use_glds()) {
    // ring depth by LDS budget: BM=256 -> 6 x 24 KB (1 WG/CU); 128 -> 4 x 16 KB and 64 -> 4 x 12 KB (2-3 WG/CU)
    if (bm == 64) L(skinny_glds_kernel, 64, 4, EPI);
    else if (bm == 128) L(skinny_glds_kernel, 128, 4, EPI);
    else L(skinny_glds_kernel, 256, 6, EPI);
  } else {
    if (bm == 64) L(skinny_gemm_kernel, 64, EPI);
    else if (bm == 128) L(skinny_gemm_kernel, 128, EPI);
    else L(skinny_gemm_kernel, 256, EPI);
  }
#undef L
}

void check_operands(const at::Tensor& x, const at::Tensor& w, int64_t K) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x must be [M, K] with unit column stride");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) == K, "w must be contiguous [N, K]");
  TORCH_CHECK(K % BK == 0, "K must be a multiple of 64");
  TORCH_CHECK(x.size(0) <= 65536, "skinny GEMM: M too large");
}

}  // namespace

// out[M, N] (bf16, row stride out.stride(0)) = x[M, K] . w[N, K]^T
void skinny_gemm(at::Tensor out, at::Tensor x, at::Tensor w) {
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  check_operands(x, w, K);
  TORCH_CHECK(N % BN == 0, "N must be a multiple of 128");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1);
  TORCH_CHECK(out.stride(0) % 4 == 0);
  if (M == 0) return;
  const int BM = pick_bm(M);
  const int MT = (M + BM - 1) / BM, NT = N / BN;
  const int S = pick_splitk(BM, MT * NT, K);
  auto stream = at::hip::getCurrentHIPStream();
  dim3 grid(MT * NT, S);
  if (S == 1) {
    launch<EPI_STORE>(BM, grid, stream, x, w, M, N, K, K, (bf16*)out.data_ptr(), out.stride(0), nullptr, MT, 0);
    return;
  }
  at::Tensor part = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  launch<EPI_PARTIAL>(BM, grid, stream, x, w, M, N, K, K / S, nullptr, 0, part.data_ptr<float>(), MT, 0);
  const int64_t total4 = M * N / 4;
  splitk_reduce_kernel<<<(int)((total4 + 255) / 256), 256, 0, stream>>>(part.data_ptr<float>(), S, M, N,
                                                                       (bf16*)out.data_ptr(), out.stride(0));
}

// out[M, F] = silu(x . w[:F]^T) * (x . w[F:]^T), w = the fused gate_up weight [2F, K]
void skinny_gemm_silu(at::Tensor out, at::Tensor x, at::Tensor w) {
  const int64_t M = x.size(0), K = x.size(1), F = w.size(0) / 2;
  check_operands(x, w, K);
  TORCH_CHECK(w.size(0) == 2 * F && F % 64 == 0, "gate_up rows must be 2F with F % 64 == 0");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.size(0) == M && out.size(1) == F);
  if (M == 0) return;
  const int BM = pick_bm(M);
  const int MT = (M + BM - 1) / BM, NT = F / 64;
  auto stream = at::hip::getCurrentHIPStream();
  launch<EPI_SILU>(BM, dim3(MT * NT, 1), stream, x, w, M, (int)(2 * F), K, K, (bf16*)out.data_ptr(), out.stride(0),
                   nullptr, MT, (int)F);
}

// residual += x . w^T ; out = rmsnorm(residual) * norm_w   (out, residual: [M, N] bf16)
void skinny_gemm_add_rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor residual, at::Tensor norm_w,
                             double eps) {
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  check_operands(x, w, K);
  TORCH_CHECK(N % BN == 0 && N <= 256 * 8 * 8, "N must be a multiple of 128 and <= 16384");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.size(0) == M && out.size(1) == N);
  TORCH_CHECK(residual.scalar_type() == at::kBFloat16 && residual.is_contiguous() && residual.numel() == M * N);
  TORCH_CHECK(norm_w.scalar_type() == at::kBFloat16 && norm_w.numel() == N);
  if (M == 0) return;
  const int BM = pick_bm(M);
  const int MT = (M + BM - 1) / BM, NT = N / BN;
  const int S = pick_splitk(BM, MT * NT, K);
  auto stream = at::hip::getCurrentHIPStream();
  at::Tensor part = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  launch<EPI_PARTIAL>(BM, dim3(MT * NT, S), stream, x, w, M, N, K, K / S, nullptr, 0, part.data_ptr<float>(), MT, 0);
  const int nv = (int)((N / 8 + 255) / 256);
#define RED(NV)                                                                                          \
  splitk_add_rmsnorm_kernel<NV><<<(int)M, 256, 0, stream>>>(part.data_ptr<float>(), S, M, N,             \
                                                            (bf16*)residual.data_ptr(),                  \
                                                            (const bf16*)norm_w.data_ptr(), (float)eps,  \
                                                            (bf16*)out.data_ptr())
  if (nv <= 1) RED(1);
  else if (nv <= 2) RED(2);
  else if (nv <= 4) RED(4);
  else RED(8);
#undef RED
}

// Launch helpers for the split-K reductions, shared with gemm_decode.hip.
void splitk_reduce_launch(const float* part, int S, int M, int N, bf16* out, int64_t ldo, hipStream_t st) {
  const int64_t total4 = (int64_t)M * N / 4;
  splitk_reduce_kernel<<<(int)((total4 + 255) / 256), 256, 0, st>>>(part, S, M, N, out, ldo);
}

void splitk_add_rmsnorm_launch(const float* part, int S, int M, int N, bf16* residual, const bf16* norm_w, float eps,
                               bf16* out, hipStream_t st) {
  const int nv = (N / 8 + 255) / 256;
  TORCH_CHECK(nv <= 8, "splitk_add_rmsnorm: N <= 16384");
  const char* e = getenv("LS_NORM_NT512");   // 0: the 256-thread form (read per launch, A/B in one process)
  if ((e ? atoi(e) : 1) != 0 && N / 8 <= 512) {
    splitk_add_rmsnorm_kernel<1, 8, 512><<<M, 512, 0, st>>>(part, S, M, N, residual, norm_w, eps, out);
    return;
  }
#define RED(NV) splitk_add_rmsnorm_kernel<NV><<<M, 256, 0, st>>>(part, S, M, N, residual, norm_w, eps, out)
  if (nv <= 1) RED(1);
  else if (nv <= 2) RED(2);
  else if (nv <= 4) RED(4);
  else RED(8);
#undef RED
}
