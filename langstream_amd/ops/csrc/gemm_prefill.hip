// Prefill-sized GEMM on MFMA for gfx950:  C[M, N] = X[M, K] . W[N, K]^T  (M in the
// thousands: one chunked-prefill step of the LLM engine), optionally with the Llama
// SwiGLU fused into the epilogue so the [T, 2F] gate_up product never reaches HBM.
//
// Why a second big-M kernel next to gemm_fused.hip: that one tiles 256 x 128 with one
// 64 x 64 sub-tile per wave, which moves (64 + 64) x 32 x 2 B through LDS per 16 MFMAs.
// Here the workgroup tile is 256 x 256 with one 128 x 64 sub-tile per wave (8 waves,
// 2 per SIMD): 12 ds_read_b128 per 32 MFMA 16x16x32, i.e. per K step the CU reads
// 96 KB of LDS (~384 cycles at 256 B/clk) under ~1030 cycles of MFMA per SIMD, so the
// matrix cores, not the LDS array, set the pace (MI355X_MICROARCH LDS table).
//   * both operands global -> LDS by global_load_lds_dwordx4 (no VGPR staging) into an
//     S-deep ring of 32-deep K stages (32 KB each), S-1 stages in flight, one raw
//     s_barrier per K step behind a counted vmcnt (same ring protocol as gemm_skinny.hip);
//   * 64-B LDS rows with the source-side bank swizzle of common.h (conflict-free
//     fragment reads);
//   * grouped tile order on top of the XCD remap: the ~32 workgroups an XCD runs at once
//     cover GROUP_M M-tiles x (32 / GROUP_M) N-tiles, so both the X and the W tiles they
//     stream are shared through that XCD's L2 (a 1-D order would re-stream X from HBM
//     once per N tile);
//   * SILU epilogue: a tile's 256 W rows are 128 gate rows + the matching 128 up rows,
//     laid out so every wave holds gate and up of the same output element in its own
//     accumulators; out = silu(g) * u is stored as bf16 [M, F].
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

constexpr int TM = 256, TN = 256, GBK = 32;
constexpr int XB = TM * GBK * 2, WB = TN * GBK * 2, SB = XB + WB;  // 16 KB + 16 KB per stage

enum { EPI_STORE = 0, EPI_SILU = 1 };

// NWV = 8: 2 x 4 waves of 128 x 64 (2 waves per SIMD, 8 x 4 accumulators each);
// NWV = 4: 2 x 2 waves of 128 x 128 (1 wave per SIMD, 8 x 8 accumulators in AGPRs), a
// third less LDS read traffic per K step and no SIMD-sharing wave at the barrier.
// (A register-staged ring -- global_load_dwordx4 + ds_write_b128 instead of LDS-DMA --
// measured 10-15 % slower on every Llama shape: profiles/pgemm_bench_v3_rs.log.)
// ABL (diagnostic ablation builds, wrong results, timing only; LS_PGEMM_ABL):
// bit 0 drops the in-loop waits + barrier, bit 1 the in-loop LDS-DMA issue,
// bit 2 the in-loop fragment reads.
// SP (8-wave layout): the step's 4 LDS-DMA pieces are spread over the MFMA stream, one
// per quarter (3 fragment reads + 8 MFMAs + 1 piece, sched_barrier-fenced), instead of
// issued back to back after the barrier.
template <int S, int EPI, int NWV, int ABL = 0, bool SP = false>
__global__ void __launch_bounds__(NWV * 64) gemm_prefill_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                                const bf16* __restrict__ w, int M, int K,
                                                                bf16* __restrict__ out, int64_t ldo, int MT,
                                                                int NTL, int F, int group_m) {
  static_assert(S >= 3, "the ring keeps stage kt+1 readable while kt+2.. are in flight");
  constexpr int PPW = 16 / NWV;           // 16-row X pieces (and W pieces) per wave per stage
  constexpr int PER = 2 * PPW;            // LDS-DMA instructions per wave per stage
  constexpr int WCOLS = 512 / NWV;        // columns per wave (64 / 128)
  constexpr int JT = WCOLS / 16;          // 16-column MFMA tiles per wave
  constexpr int NRD = 8 + JT;             // fragment reads per wave per K step
  __shared__ __attribute__((aligned(1024))) char lds[S * SB];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = group_m * NTL;
  const int grp = logical / per_group, first = grp * group_m;
  const int gsz = min(MT - first, group_m);
  const int rem = logical - grp * per_group;
  const int mt = first + rem % gsz, nt = rem / gsz;
  const int m0 = mt * TM;
  const int nk = K / GBK;

  // LDS-DMA sources: wave w fills X pieces PPW*w.. and W pieces PPW*w.. (16 rows each)
  const int prow = lane >> 2;
  const int sck = ((lane & 3) ^ swz_g(lane >> 4)) * 8;
  const bf16* xs[PPW];
  const bf16* wsrc[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int row = 16 * (PPW * wid + j) + prow;
    xs[j] = x + (int64_t)min(m0 + row, M - 1) * ldx + sck;   // rows >= M: any valid row, never stored
    int wrow;
    if (EPI == EPI_SILU) wrow = row < 128 ? nt * 128 + row : F + nt * 128 + (row - 128);
    else wrow = nt * TN + row;
    wsrc[j] = w + (int64_t)wrow * K + sck;
  }
  auto issue = [&](int kt, int slot) {
    const int ko = kt * GBK;
    char* base = lds + slot * SB;
#pragma unroll
    for (int j = 0; j < PPW; ++j) glds16(xs[j] + ko, base + (PPW * wid + j) * 1024);
#pragma unroll
    for (int j = 0; j < PPW; ++j) glds16(wsrc[j] + ko, base + XB + (PPW * wid + j) * 1024);
  };

  const int wm = wid / (NWV / 2), wn = wid % (NWV / 2);
  const int fr = lane & 15, h = lane >> 4;
  const int swz = 16 * (h ^ swz_g(fr >> 2));
  // tile-local W row (= output column) of this lane's B fragment for column tile j.
  // SILU: tiles [0, JT/2) are gate columns, [JT/2, JT) the matching up columns.
  auto bcol = [&](int j) {
    if (EPI == EPI_SILU)
      return (j < JT / 2 ? (WCOLS / 2) * wn + 16 * j : 128 + (WCOLS / 2) * wn + 16 * (j - JT / 2)) + fr;
    return WCOLS * wn + 16 * j + fr;
  };
  f32x4 acc[8][JT];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Fragments are double-buffered in registers: step kt's MFMAs run on fragments read
  // during step kt-1, while this step's ds_reads fetch stage kt+1 (left to itself hipcc
  // reuses two fragment registers and exposes the LDS latency four times per K step).
  auto load_frags = [&](int slot, bf16x8 (&a)[8], bf16x8 (&b)[JT]) {
    const char* lx = lds + slot * SB;
    const char* lw = lx + XB;
#pragma unroll
    for (int j = 0; j < JT; ++j) b[j] = __builtin_bit_cast(bf16x8, ld16(lw + bcol(j) * 64 + swz));
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = __builtin_bit_cast(bf16x8, ld16(lx + (128 * wm + 16 * i + fr) * 64 + swz));
  };
  auto mma = [&](const bf16x8 (&a)[8], const bf16x8 (&b)[JT]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < JT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  };
  int buf = 0;                            // ring slot of stage kt
  // one K step: stage kt+1 visible to every wave -> refill the slot of stage kt-1 (its
  // fragments were consumed by step kt-1's MFMAs, which waited for them) -> read stage
  // kt+1's fragments into `nxt` -> MFMAs on `cur`.
  auto step = [&](int kt, const bf16x8 (&ca)[8], const bf16x8 (&cb)[JT], bf16x8 (&na)[8], bf16x8 (&nb)[JT]) {
    // stage kt's fragment reads (all but the NRD newest LDS ops) are complete before this
    // wave joins the barrier after which another wave may refill their slot
    if constexpr ((ABL & 1) == 0) {
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NRD < 15 ? NRD : 15) : "memory");  // counter max 15
      wait_vmcnt<(S - 3) * PER>();        // this wave's DMA of stage kt+1 has landed
      __builtin_amdgcn_s_barrier();       // ... and every other wave's
    }
    int rs = buf + S - 1;
    if (rs >= S) rs -= S;
    const int b1 = buf + 1 == S ? 0 : buf + 1;
    if constexpr (SP && NWV == 8) {
      const char* lx = lds + b1 * SB;
      const char* lw = lx + XB;
      const int ko = min(kt + S - 1, nk - 1) * GBK;   // past the end: re-load the last stage into a dead slot
      char* dst = lds + rs * SB;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr ((ABL & 4) == 0) {
          nb[q] = __builtin_bit_cast(bf16x8, ld16(lw + bcol(q) * 64 + swz));
#pragma unroll
          for (int i = 2 * q; i < 2 * q + 2; ++i)
            na[i] = __builtin_bit_cast(bf16x8, ld16(lx + (128 * wm + 16 * i + fr) * 64 + swz));
        }
#pragma unroll
        for (int i = 2 * q; i < 2 * q + 2; ++i)
#pragma unroll
          for (int j = 0; j < JT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[i], cb[j], acc[i][j], 0, 0, 0);
        if constexpr ((ABL & 2) == 0) {
          if (q < 2) glds16(xs[q] + ko, dst + (2 * wid + q) * 1024);
          else glds16(wsrc[q - 2] + ko, dst + XB + (2 * wid + q - 2) * 1024);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      if constexpr ((ABL & 2) == 0) issue(min(kt + S - 1, nk - 1), rs);  // past the end: re-load the last stage into a dead slot
      if constexpr ((ABL & 4) == 0) load_frags(b1, na, nb);  // past the end: reads a dead slot, never used
      mma(ca, cb);
      constexpr int PERRD = 8 * JT / NRD;   // MFMAs between consecutive fragment reads
#pragma unroll
      for (int g = 0; g < NRD; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);       // 1 ds_read
        __builtin_amdgcn_sched_group_barrier(0x008, PERRD, 0);   // PERRD MFMAs
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8 * JT - PERRD * NRD, 0);
    }
    buf = b1;
  };

#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(min(s, nk - 1), s);
  wait_vmcnt<(S - 2) * PER>();
  __builtin_amdgcn_s_barrier();
  bf16x8 a0[8], b0[JT], a1[8], b1[JT];
  load_frags(0, a0, b0);
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, a0, b0, a1, b1);
    step(kt + 1, a1, b1, a0, b0);
  }
  if (kt < nk) step(kt, a0, b0, a1, b1);
  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup

  // acc[i][j][r] = C[128wm + 16i + 4h + r][bcol(j)] (tile-local)
  const int rbase = m0 + 128 * wm + 4 * h;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = rbase + 16 * i + r;
      if (m >= M) continue;
      bf16* orow = out + (int64_t)m * ldo;
      if (EPI == EPI_SILU) {
#pragma unroll
        for (int j = 0; j < JT / 2; ++j) {
          const float g = acc[i][j][r], u = acc[i][j + JT / 2][r];
          orow[nt * 128 + (WCOLS / 2) * wn + 16 * j + fr] = (bf16)(g / (1.f + __expf(-g)) * u);
        }
      } else {
#pragma unroll
        for (int j = 0; j < JT; ++j) orow[nt * TN + WCOLS * wn + 16 * j + fr] = (bf16)acc[i][j][r];
      }
    }
}

// ---------------------------------------------------------------------------------
// 64-deep K stages with 128-B LDS rows.  The SQ/TCC counters of the 32-deep kernel show
// the same L2 misses as hipBLASLt's MT256x256x64 but TWICE its TCP->TCC read requests
// (profiles/pmc_pgemm_v2): a 32-deep stage loads half of each 128-B line per DMA
// instruction, so every line costs two requests, and the request rate -- not MFMA, LDS
// or HBM -- bounded the loop (ablation: no in-loop DMA 1.2 -> 1.78 PFLOP/s).  Here one
// LDS-DMA instruction fills 8 rows x 128 B (one request per line).
//   * LDS image: 128-B rows; chunk p of row r holds global k-chunk p ^ ((r >> 1) & 7),
//     which puts the 16 lanes of each ds_read_b128 lane group on 16 distinct 16-B bank
//     slots (MI355X_MICROARCH LDS table; exhaustively checked for both k halves);
//   * 2 slots of 64 KB: stage p+2 is issued when every wave has read stage p, i.e. two
//     32-deep half-steps before it is needed; one barrier per 64-deep stage;
//   * compute is unchanged: half-steps of 32 MFMA 16x16x32 per wave on fragments read
//     during the previous half-step.
constexpr int SB64 = 65536, XB64 = 32768;

template <int EPI>
__global__ void __launch_bounds__(512) gemm_prefill64_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                             const bf16* __restrict__ w, int M, int K,
                                                             bf16* __restrict__ out, int64_t ldo, int MT, int NTL,
                                                             int F, int group_m) {
  constexpr int JT = 4;
  __shared__ __attribute__((aligned(1024))) char lds[2 * SB64];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = group_m * NTL;
  const int grp = logical / per_group, first = grp * group_m;
  const int gsz = min(MT - first, group_m);
  const int rem = logical - grp * per_group;
  const int mt = first + rem % gsz, nt = rem / gsz;
  const int m0 = mt * TM;
  const int np = K / 64;                  // 64-deep stages

  // LDS-DMA: wave w fills rows 32w..32w+31 of the X and the W image, 4 pieces of 8 rows
  // each; lane l loads row (l >> 3) of a piece, swizzled chunk (l & 7) ^ ((row >> 1) & 7)
  const int prow = lane >> 3;
  const int row0 = 32 * wid + prow;      // this lane's row in piece 0 (pieces step 8 rows)
  // ((row0 + 8j) >> 1) & 7 = ((row0 >> 1) + 4j) & 7: one chunk order for even j, one for odd
  const int sck = ((lane & 7) ^ ((row0 >> 1) & 7)) * 8;
  const int sck1 = ((lane & 7) ^ (((row0 >> 1) + 4) & 7)) * 8;
  const bf16* xsrc = x + (int64_t)min(m0 + row0, M - 1) * ldx;
  int wrow0;
  if (EPI == EPI_SILU) wrow0 = row0 < 128 ? nt * 128 + row0 : F + nt * 128 + (row0 - 128);
  else wrow0 = nt * TN + row0;
  const bf16* wsrc = w + (int64_t)wrow0 * K;
  auto issue = [&](int p, int slot) {
    const int ko = p * 64;
    char* base = lds + slot * SB64 + (4 * wid) * 1024;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int mrow = min(m0 + row0 + 8 * j, M - 1) - min(m0 + row0, M - 1);   // rows >= M: any valid row
      glds16(xsrc + (int64_t)mrow * ldx + ko + ((j & 1) ? sck1 : sck), base + j * 1024);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      glds16(wsrc + (int64_t)(8 * j) * K + ko + ((j & 1) ? sck1 : sck), base + XB64 + j * 1024);
  };

  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, h = lane >> 4;
  const int fsw = (fr >> 1) & 7;          // = (row >> 1) & 7 for every fragment row (rows are 16-aligned + fr)
  auto bcol = [&](int j) {
    if (EPI == EPI_SILU) return (j < 2 ? 32 * wn + 16 * j : 128 + 32 * wn + 16 * (j - 2)) + fr;
    return 64 * wn + 16 * j + fr;
  };
  f32x4 acc[8][JT];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // half-step t reads k-chunks 4 (t & 1) + h of stage t >> 1 from slot (t >> 1) & 1
  auto load_frags = [&](int t, bf16x8 (&a)[8], bf16x8 (&b)[JT]) {
    const char* lx = lds + ((t >> 1) & 1) * SB64;
    const char* lw = lx + XB64;
    const int off = 16 * ((4 * (t & 1) + h) ^ fsw);
#pragma unroll
    for (int j = 0; j < JT; ++j) b[j] = __builtin_bit_cast(bf16x8, ld16(lw + bcol(j) * 128 + off));
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = __builtin_bit_cast(bf16x8, ld16(lx + (128 * wm + 16 * i + fr) * 128 + off));
  };
  const int nh = 2 * np;
  auto half = [&](int t, const bf16x8 (&ca)[8], const bf16x8 (&cb)[JT], bf16x8 (&na)[8], bf16x8 (&nb)[JT]) {
    if (t & 1) {
      // next half-step opens stage p+1 = (t+1)/2: every wave's reads of stage p (the
      // newest LDS ops, issued one half-step ago) are done and stage p+1 has landed ->
      // barrier -> stage p+2 into stage p's slot
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      const int p = t >> 1;
      if (p + 2 < np) issue(p + 2, p & 1);
    }
    if (t + 1 < nh) load_frags(t + 1, na, nb);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < JT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[i], cb[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int g = 0; g < 12; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
  };

  issue(0, 0);
  issue(min(1, np - 1), 1);
  wait_vmcnt<8>();                        // stage 0 (this wave's 8 pieces) landed
  __builtin_amdgcn_s_barrier();
  bf16x8 a0[8], b0[JT], a1[8], b1[JT];
  load_frags(0, a0, b0);
  for (int t = 0; t < nh; t += 2) {       // nh is even
    half(t, a0, b0, a1, b1);
    half(t + 1, a1, b1, a0, b0);
  }
  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup

  const int rbase = m0 + 128 * wm + 4 * h;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = rbase + 16 * i + r;
      if (m >= M) continue;
      bf16* orow = out + (int64_t)m * ldo;
      if (EPI == EPI_SILU) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float g = acc[i][j][r], u = acc[i][j + 2][r];
          orow[nt * 128 + 32 * wn + 16 * j + fr] = (bf16)(g / (1.f + __expf(-g)) * u);
        }
      } else {
#pragma unroll
        for (int j = 0; j < JT; ++j) orow[nt * TN + 64 * wn + 16 * j + fr] = (bf16)acc[i][j][r];
      }
    }
}

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

template <int EPI>
void launch(int ring, int nwv, bool sp, dim3 grid, hipStream_t st, const at::Tensor& x, const at::Tensor& w, int M, int K,
            at::Tensor& out, int MT, int NTL, int F, int gm) {
#define L(SV, NW, ...)                                                                                         \
  gemm_prefill_kernel<SV, EPI, NW, ##__VA_ARGS__><<<grid, NW * 64, 0, st>>>((const bf16*)x.data_ptr(), x.stride(0),                  \
                                                     (const bf16*)w.data_ptr(), M, K, (bf16*)out.data_ptr(),  \
                                                     out.stride(0), MT, NTL, F, gm)
  static const bool k64 = env_int("LS_PGEMM_K64", 0) != 0;   // measured equal, 2-slot ring: off
  if (k64 && K % 64 == 0) {
    gemm_prefill64_kernel<EPI><<<grid, 512, 0, st>>>((const bf16*)x.data_ptr(), x.stride(0),
                                                    (const bf16*)w.data_ptr(), M, K, (bf16*)out.data_ptr(),
                                                    out.stride(0), MT, NTL, F, gm);
    return;
  }
  static const int abl = env_int("LS_PGEMM_ABL", 0);
  if (abl != 0 && EPI == EPI_STORE && nwv == 8 && ring == 4) {   // diagnostic ablations
    auto* xp = (const bf16*)x.data_ptr();
    auto* wp = (const bf16*)w.data_ptr();
    auto* op = (bf16*)out.data_ptr();
    if (abl == 1) gemm_prefill_kernel<4, EPI, 8, 1><<<grid, 512, 0, st>>>(xp, x.stride(0), wp, M, K, op, out.stride(0), MT, NTL, F, gm);
    else if (abl == 2) gemm_prefill_kernel<4, EPI, 8, 2><<<grid, 512, 0, st>>>(xp, x.stride(0), wp, M, K, op, out.stride(0), MT, NTL, F, gm);
    else if (abl == 3) gemm_prefill_kernel<4, EPI, 8, 3><<<grid, 512, 0, st>>>(xp, x.stride(0), wp, M, K, op, out.stride(0), MT, NTL, F, gm);
    else if (abl == 4) gemm_prefill_kernel<4, EPI, 8, 4><<<grid, 512, 0, st>>>(xp, x.stride(0), wp, M, K, op, out.stride(0), MT, NTL, F, gm);
    else gemm_prefill_kernel<4, EPI, 8, 7><<<grid, 512, 0, st>>>(xp, x.stride(0), wp, M, K, op, out.stride(0), MT, NTL, F, gm);
    return;
  }
  if (nwv == 4) {
    if (ring == 3) L(3, 4);
    else if (ring == 5) L(5, 4);
    else L(4, 4);
  } else if (sp) {
    if (ring == 3) L(3, 8, 0, true);
    else if (ring == 5) L(5, 8, 0, true);
    else L(4, 8, 0, true);
  } else {
    if (ring == 3) L(3, 8);
    else if (ring == 5) L(5, 8);
    else L(4, 8);
  }
#undef L
}

}  // namespace

// Shapes the kernel takes: K % 32 == 0 and N % 256 == 0 (silu: the fused [2F, K] gate_up
// weight with F % 128 == 0).
bool gemm_prefill_supported(const at::Tensor& w, bool silu) {
  if (w.dim() != 2 || w.scalar_type() != at::kBFloat16 || !w.is_contiguous() || w.size(1) % GBK != 0) return false;
  return silu ? (w.size(0) % 256 == 0) : (w.size(0) % TN == 0);
}

// silu == false: out[M, N] = x . w^T;  silu == true: out[M, F] = silu(x . w[:F]^T) * (x . w[F:]^T)
void gemm_prefill(at::Tensor out, at::Tensor x, at::Tensor w, bool silu) {
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16, "x must be bf16 on the GPU");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x must be [M, K] with unit column stride");
  TORCH_CHECK(w.size(1) == K && gemm_prefill_supported(w, silu), "gemm_prefill: unsupported weight shape");
  TORCH_CHECK(x.device() == w.device() && out.device() == x.device(), "gemm_prefill: tensors on different devices");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0,
              "gemm_prefill: x and w must be 16-byte aligned (16-B LDS-DMA rows)");
  const int64_t NO = silu ? N / 2 : N;
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.dim() == 2 && out.size(0) == M && out.size(1) == NO &&
              out.stride(1) == 1, "out must be bf16 [M, ", NO, "]");
  TORCH_CHECK(M < (1LL << 31) / TM);
  if (M == 0) return;
  const int MT = (int)((M + TM - 1) / TM), NTL = (int)(silu ? N / 2 / 128 : N / TN);
  static const int ring = env_int("LS_PGEMM_RING", 4);
  static const int gm_env = env_int("LS_PGEMM_GROUP", 8);
  static const int nwv = env_int("LS_PGEMM_WAVES", 8) == 4 ? 4 : 8;
  static const bool sp = env_int("LS_PGEMM_SPREAD", 1) != 0;
  const int gm = std::max(1, std::min(gm_env, MT));
  auto stream = at::hip::getCurrentHIPStream();
  const dim3 grid((unsigned)(MT * NTL));
  if (silu) launch<EPI_SILU>(ring, nwv, sp, grid, stream, x, w, (int)M, (int)K, out, MT, NTL, (int)(N / 2), gm);
  else launch<EPI_STORE>(ring, nwv, sp, grid, stream, x, w, (int)M, (int)K, out, MT, NTL, 0, gm);
}
