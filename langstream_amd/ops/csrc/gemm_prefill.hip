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
#include <type_traits>

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

// ---------------------------------------------------------------------------------
// Ping-pong kernel: 64-deep K tiles cut into four 16 KB HALF-TILES (128 LDS rows x 128 B)
// -- A-q0 = tile rows {0..63, 128..191}, A-q1 = rows {64..127, 192..255}, B-q0 / B-q1 =
// the first / second 32 of each wave's 64 columns -- in an 8-slot LDS ring (128 KB).
// Every K tile is four PHASES, one C quadrant (qm, qn) of the wave's 128 x 64 each:
//
//   phase  quadrant  fragment reads        LDS-DMA issued            vmcnt before barrier
//   0      (0, 0)    A-q0 -> a, B-q0 -> b0  B-q1 of tile t+1        8 (B-q1 of t landed)
//   1      (0, 1)    B-q1 -> b1             A-q1 of tile t+1        8 (A-q1 of t)
//   2      (1, 1)    A-q1 -> a              A-q0 of tile t+2        -
//   3      (1, 0)    -                      B-q0 of tile t+2        8 (A-q0, B-q0 of t+1)
//
// A phase is { fragment reads, one half-tile of LDS-DMA (2 per lane), counted vmcnt } ->
// s_barrier -> { lgkmcnt(0), 16 MFMA 16x16x32 } -> s_barrier, and the two wave groups that
// share each SIMD (wm = 0: waves 0-3, wm = 1: waves 4-7) run one barrier apart, so one
// group's MFMA cluster overlaps the other's LDS reads and DMA issue (cdna_hip_programming
// §5 "256^2 8-phase template", T3-T5).  Hazards, by barrier count: a half-tile is waited
// for (every wave, its own DMA) in the phase BEFORE its first read, and re-filled no
// earlier than two phases after its last read (the staggered group finishes reading
// one barrier late); each half-tile spends 4-5 phases in flight (4 half-tiles = 64 KB per CU).
// LDS rows hold k-chunk c ^ ((row >> 1) & 7) at chunk c (source-side swizzle, conflict-free
// ds_read_b128 for the 16 rows of a fragment lane group).
constexpr int HT = 16384;

// Epilogue forms of the ping-pong kernel (EPS):
//   0: each lane stores its accumulators as 2-byte scalars straight from the MFMA layout
//      (a wave-instruction writes 4 rows x 32 B: partial lines);
//   1: the tile goes through LDS as bf16 rows (the ring is dead after the K loop) and
//      leaves in 16-B stores of whole 512-B rows -- full 128-B lines per instruction;
//   2: timing ablation, no stores at all (results garbage; LS_PGEMM_KERNEL=4).
constexpr int EPI_ROW = 256 + 8;          // staged row pitch in bf16 (528 B: 4-bank shift per row)
constexpr int PP_LDS = 256 * EPI_ROW * 2 > 8 * HT ? 256 * EPI_ROW * 2 : 8 * HT;

// Split-K (S > 1, plain GEMM only): the grid is S x the tile grid; split s takes K tiles
// [2 floor(s P / S), 2 floor((s + 1) P / S)) of the P = K / 128 tile pairs and stores its
// f32 partial tile to part[s][M][N] (a reduction kernel sums the S slabs into bf16).  For
// mid-size steps whose tile grid leaves CUs idle: T = 1024 gives o / down 4 x 16 = 64
// tiles on 256 CUs.  Consecutive logical ids share a split (one XCD streams one K range).
template <int EPI, int EPS = 0>
__global__ void __launch_bounds__(512) gemm_pp_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                      const bf16* __restrict__ w, int M, int K,
                                                      bf16* __restrict__ out, int64_t ldo, int MT, int NTL, int F,
                                                      int group_m, int S = 1, float* __restrict__ part = nullptr) {
  __shared__ __attribute__((aligned(1024))) char lds[EPS == 1 ? PP_LDS : 8 * HT];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = gridDim.x / S;
  const int split = logical / ntiles;
  logical -= split * ntiles;
  const int per_group = group_m * NTL;
  const int grp = logical / per_group, first = grp * group_m;
  const int gsz = min(MT - first, group_m);
  const int rem = logical - grp * per_group;
  const int mt = first + rem % gsz, nt = rem / gsz;
  const int m0 = mt * TM;
  const int npairs = K / 128;
  const int kt0 = 2 * (int)(((int64_t)split * npairs) / S);
  const int nk = 2 * (int)(((int64_t)(split + 1) * npairs) / S) - kt0;
  x += (int64_t)kt0 * 64;
  w += (int64_t)kt0 * 64;

  // LDS-DMA sources: wave w fills LDS rows 16w..16w+15 of every half-tile (2 pieces of
  // 8 rows x 128 B); lane l loads row 8e + (l >> 3) of piece e, swizzled chunk l & 7.
  const bf16* src[4][2];   // [A-q0, A-q1, B-q0, B-q1][piece]
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int r = 16 * wid + 8 * e + (lane >> 3);
    const int koff = ((lane & 7) ^ ((r >> 1) & 7)) * 8;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int arow = m0 + (r & 63) + 128 * (r >> 6) + 64 * q;
      src[q][e] = x + (int64_t)min(arow, M - 1) * ldx + koff;   // rows >= M: any valid row, never stored
      int wrow;
      if (EPI == EPI_SILU) wrow = (q == 0 ? 0 : F) + nt * 128 + r;
      else wrow = nt * TN + 64 * (r >> 5) + 32 * q + (r & 31);
      src[2 + q][e] = w + (int64_t)wrow * K + koff;
    }
  }
  auto issue = [&](int type, int tile, int slot) {
    const int ko = min(tile, nk - 1) * 64;   // past the end: re-load the last tile into a dead slot
#pragma unroll
    for (int e = 0; e < 2; ++e) glds16(src[type][e] + ko, lds + slot * HT + (2 * wid + e) * 1024);
  };

  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, h = lane >> 4;
  const int fsw = (fr >> 1) & 7;
  // byte offsets of this lane's fragment rows for k-steps 0 / 1 inside a half-tile
  const int aoff0 = (64 * wm + fr) * 128 + 16 * (h ^ fsw), aoff1 = (64 * wm + fr) * 128 + 16 * ((4 + h) ^ fsw);
  const int boff0 = (32 * wn + fr) * 128 + 16 * (h ^ fsw), boff1 = (32 * wn + fr) * 128 + 16 * ((4 + h) ^ fsw);
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  auto read_a = [&](int slot) {
    const char* base = lds + slot * HT;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i][0] = __builtin_bit_cast(bf16x8, ld16(base + aoff0 + i * 2048));
      a[i][1] = __builtin_bit_cast(bf16x8, ld16(base + aoff1 + i * 2048));
    }
  };
  auto read_b = [&](int slot, bf16x8 (&b)[2][2]) {
    const char* base = lds + slot * HT;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b[j][0] = __builtin_bit_cast(bf16x8, ld16(base + boff0 + j * 2048));
      b[j][1] = __builtin_bit_cast(bf16x8, ld16(base + boff1 + j * 2048));
    }
  };
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[qm][qn][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&](f32x4 (&c)[4][2], const bf16x8 (&bb)[2][2]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], bb[j][ks], c[i][j], 0, 0, 0);
  };
  // the MFMA half of a phase: barrier -> wait this wave's fragment reads -> cluster -> barrier
  auto compute = [&](f32x4 (&c)[4][2], const bf16x8 (&bb)[2][2]) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma(c, bb);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // one K tile t whose half-tiles sit in slots 4P..4P+3 (P = t & 1, compile-time)
  auto ktile = [&](int t, auto Pc) {
    constexpr int P = decltype(Pc)::value;
    constexpr int Q = 1 - P;
    read_a(4 * P + 0);
    read_b(4 * P + 1, b0);
    issue(3, t + 1, 4 * Q + 2);     // B-q1 of t+1
    wait_vmcnt<8>();
    compute(acc[0][0], b0);
    read_b(4 * P + 2, b1);
    issue(1, t + 1, 4 * Q + 3);     // A-q1 of t+1
    wait_vmcnt<8>();
    compute(acc[0][1], b1);
    read_a(4 * P + 3);
    issue(0, t + 2, 4 * P + 0);     // A-q0 of t+2
    compute(acc[1][1], b1);
    issue(2, t + 2, 4 * P + 1);     // B-q0 of t+2
    wait_vmcnt<8>();
    compute(acc[1][0], b0);
  };

  // prologue, in steady-state issue order: A-q0, B-q0, B-q1, A-q1 of tile 0, A-q0, B-q0 of tile 1
  issue(0, 0, 0);
  issue(2, 0, 1);
  issue(3, 0, 2);
  issue(1, 0, 3);
  issue(0, 1, 4);
  issue(2, 1, 5);
  wait_vmcnt<8>();
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one barrier behind
  for (int t = 0; t < nk; t += 2) {   // nk even
    ktile(t, std::integral_constant<int, 0>());
    ktile(t + 1, std::integral_constant<int, 1>());
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();
  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup

  if constexpr (EPS == 2) {
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[qm][qn][i][j]));
    return;
  }
  if constexpr (EPS == 1) {
    // stage: every wave's fragments -> bf16 rows of the tile image (OC columns wide),
    // then whole rows leave with 16-B stores
    constexpr int OC = EPI == EPI_SILU ? 128 : 256;          // output columns of the tile
    constexpr int RP = EPI == EPI_SILU ? 128 + 8 : EPI_ROW;  // row pitch (bf16)
    bf16* T = reinterpret_cast<bf16*>(lds);
    __syncthreads();                                         // every wave's ring reads are done
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bf16* trow = T + (128 * wm + 64 * qm + 16 * i + 4 * h + r) * RP;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if constexpr (EPI == EPI_SILU) {
              const float g = acc[qm][0][i][j][r], u = acc[qm][1][i][j][r];
              trow[32 * wn + 16 * j + fr] = (bf16)(g / (1.f + __expf(-g)) * u);
            } else {
#pragma unroll
              for (int qn = 0; qn < 2; ++qn) trow[64 * wn + 32 * qn + 16 * j + fr] = (bf16)acc[qm][qn][i][j][r];
            }
          }
        }
    __syncthreads();
    constexpr int CPR = OC / 8;                              // 16-B chunks per row
    const int rows = min(256, M - m0);
    const int col0 = EPI == EPI_SILU ? nt * 128 : nt * TN;
    for (int q = threadIdx.x; q < rows * CPR; q += 512) {
      const int rr = q / CPR, c = (q - rr * CPR) * 8;
      st16(out + (int64_t)(m0 + rr) * ldo + col0 + c, ld16(reinterpret_cast<const char*>(T + rr * RP + c)));
    }
    return;
  }

  // acc[qm][qn][i][j][r] = C[128 wm + 64 qm + 16 i + 4 h + r][64 wn + 32 qn + 16 j + fr] (tile-local;
  // SILU: qn = 0 gate, qn = 1 up of feature nt*128 + 32 wn + 16 j + fr)
  if constexpr (EPI == EPI_STORE) {
    if (part != nullptr) {   // split-K: this split's f32 partial tile (S = 1: an f32 GEMM, gemm_prefill_f32)
      const int64_t N = (int64_t)NTL * TN;
#pragma unroll
      for (int qm = 0; qm < 2; ++qm)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + 128 * wm + 64 * qm + 16 * i + 4 * h + r;
            if (m >= M) continue;
            float* prow = part + ((int64_t)split * M + m) * N;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int qn = 0; qn < 2; ++qn) prow[nt * TN + 64 * wn + 32 * qn + 16 * j + fr] = acc[qm][qn][i][j][r];
          }
      return;
    }
  }
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 128 * wm + 64 * qm + 16 * i + 4 * h + r;
        if (m >= M) continue;
        bf16* orow = out + (int64_t)m * ldo;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (EPI == EPI_SILU) {
            const float g = acc[qm][0][i][j][r], u = acc[qm][1][i][j][r];
            orow[nt * 128 + 32 * wn + 16 * j + fr] = (bf16)(g / (1.f + __expf(-g)) * u);
          } else {
#pragma unroll
            for (int qn = 0; qn < 2; ++qn) orow[nt * TN + 64 * wn + 32 * qn + 16 * j + fr] = (bf16)acc[qm][qn][i][j][r];
          }
        }
      }
}

// ---------------------------------------------------------------------------------
// Persistent form of the ping-pong kernel: one workgroup per CU walks its tiles (round r
// of G = gridDim.x tiles: logical tile r*G + xcd_remap(blockIdx)) as ONE stream of K tiles,
// so the ring's prefetch runs straight across tile boundaries -- the next tile's first
// half-tiles are in flight while this tile finishes and stores -- and no tile pays a
// cold prologue.  Operands are read by buffer_load ... lds through per-tile buffer
// resources: the per-lane offsets are tile-independent (8 VGPRs instead of 8 pointers),
// rows past M fall outside the X resource's range and read zeros, and the "tile" after
// a workgroup's last one has an empty resource (its dummy prefetches move no bytes).
// (make_rsrc / blds16: common.h)

template <int EPI>
__global__ void __launch_bounds__(512) gemm_pp2_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                       const bf16* __restrict__ w, int64_t w_elems, int M, int K,
                                                       bf16* __restrict__ out, int64_t ldo, int MT, int NTL, int F,
                                                       int group_m, int ntiles) {
  __shared__ __attribute__((aligned(1024))) char lds[8 * HT];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = gridDim.x;
  const int g = xcd_remap(blockIdx.x, G);
  const int my_n = g < ntiles ? (ntiles - 1 - g) / G + 1 : 0;
  if (my_n == 0) return;
  const int nk = K / 64;
  const int per_group = group_m * NTL;
  auto coords = [&](int j, int& m0, int& nt) {
    const int logical = j * G + g;
    const int grp = logical / per_group, first = grp * group_m;
    const int gsz = min(MT - first, group_m);
    const int rem = logical - grp * per_group;
    m0 = (first + rem % gsz) * TM;
    nt = rem / gsz;
  };
  constexpr int WROWS = EPI == EPI_SILU ? 128 : TN;   // W rows per tile from the tile's W base
  auto rsrc_a = [&](int j) {
    if (j >= my_n) return make_rsrc(x, 0);
    int m0, nt;
    coords(j, m0, nt);
    return make_rsrc(x + (int64_t)m0 * ldx, (uint32_t)(((int64_t)(M - m0 - 1) * ldx + K) * 2));
  };
  auto rsrc_w = [&](int j) {
    if (j >= my_n) return make_rsrc(w, 0);
    int m0, nt;
    coords(j, m0, nt);
    const int64_t off = (int64_t)nt * WROWS * K;
    return make_rsrc(w + off, (uint32_t)((w_elems - off) * 2));
  };
  // tile-independent per-lane byte offsets: [A-q0, A-q1, B-q0, B-q1][piece]
  int voff[4][2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int r = 16 * wid + 8 * e + (lane >> 3);
    const int kb = ((lane & 7) ^ ((r >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      voff[q][e] = (int)(((r & 63) + 128 * (r >> 6) + 64 * q) * ldx * 2) + kb;
      if (EPI == EPI_SILU) voff[2 + q][e] = (int)(((int64_t)(q == 0 ? 0 : F) + r) * K * 2) + kb;
      else voff[2 + q][e] = (64 * (r >> 5) + 32 * q + (r & 31)) * K * 2 + kb;
    }
  }
  i32x4 ra_cur = rsrc_a(0), rw_cur = rsrc_w(0), ra_nxt = rsrc_a(1), rw_nxt = rsrc_w(1);
  const unsigned lds_u32 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  // K tile tr of the current tile (tr >= nk: tile tr - nk of the next one)
  auto issue = [&](int type, int tr, int slot) {
    const bool nxt = tr >= nk;
    const int soff = (nxt ? tr - nk : tr) * 128;
    const i32x4 rs = type < 2 ? (nxt ? ra_nxt : ra_cur) : (nxt ? rw_nxt : rw_cur);
#pragma unroll
    for (int e = 0; e < 2; ++e) blds16(rs, voff[type][e], soff, lds_u32 + slot * HT + (2 * wid + e) * 1024);
  };

  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, h = lane >> 4;
  const int fsw = (fr >> 1) & 7;
  const int aoff0 = (64 * wm + fr) * 128 + 16 * (h ^ fsw), aoff1 = (64 * wm + fr) * 128 + 16 * ((4 + h) ^ fsw);
  const int boff0 = (32 * wn + fr) * 128 + 16 * (h ^ fsw), boff1 = (32 * wn + fr) * 128 + 16 * ((4 + h) ^ fsw);
  bf16x8 a[4][2], b0[2][2], b1[2][2];
  auto read_a = [&](int slot) {
    const char* base = lds + slot * HT;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i][0] = __builtin_bit_cast(bf16x8, ld16(base + aoff0 + i * 2048));
      a[i][1] = __builtin_bit_cast(bf16x8, ld16(base + aoff1 + i * 2048));
    }
  };
  auto read_b = [&](int slot, bf16x8 (&b)[2][2]) {
    const char* base = lds + slot * HT;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b[j][0] = __builtin_bit_cast(bf16x8, ld16(base + boff0 + j * 2048));
      b[j][1] = __builtin_bit_cast(bf16x8, ld16(base + boff1 + j * 2048));
    }
  };
  f32x4 acc[2][2][4][2];
  auto zero = [&]() {
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[qm][qn][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto compute = [&](f32x4 (&c)[4][2], const bf16x8 (&bb)[2][2]) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][ks], bb[j][ks], c[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // same phase table as gemm_pp_kernel
  auto ktile = [&](int t, auto Pc) {
    constexpr int P = decltype(Pc)::value;
    constexpr int Q = 1 - P;
    read_a(4 * P + 0);
    read_b(4 * P + 1, b0);
    issue(3, t + 1, 4 * Q + 2);
    wait_vmcnt<8>();
    compute(acc[0][0], b0);
    read_b(4 * P + 2, b1);
    issue(1, t + 1, 4 * Q + 3);
    wait_vmcnt<8>();
    compute(acc[0][1], b1);
    read_a(4 * P + 3);
    issue(0, t + 2, 4 * P + 0);
    compute(acc[1][1], b1);
    issue(2, t + 2, 4 * P + 1);
    wait_vmcnt<8>();
    compute(acc[1][0], b0);
  };

  zero();
  issue(0, 0, 0);
  issue(2, 0, 1);
  issue(3, 0, 2);
  issue(1, 0, 3);
  issue(0, 1, 4);
  issue(2, 1, 5);
  wait_vmcnt<8>();
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one barrier behind
  for (int j = 0; j < my_n; ++j) {
    for (int t = 0; t < nk; t += 2) {   // nk even
      ktile(t, std::integral_constant<int, 0>());
      ktile(t + 1, std::integral_constant<int, 1>());
    }
    int m0, nt;
    coords(j, m0, nt);
#pragma unroll
    for (int qm = 0; qm < 2; ++qm)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + 128 * wm + 64 * qm + 16 * i + 4 * h + r;
          if (m >= M) continue;
          bf16* orow = out + (int64_t)m * ldo;
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            if (EPI == EPI_SILU) {
              const float gg = acc[qm][0][i][jj][r], u = acc[qm][1][i][jj][r];
              orow[nt * 128 + 32 * wn + 16 * jj + fr] = (bf16)(gg / (1.f + __expf(-gg)) * u);
            } else {
#pragma unroll
              for (int qn = 0; qn < 2; ++qn)
                orow[nt * TN + 64 * wn + 32 * qn + 16 * jj + fr] = (bf16)acc[qm][qn][i][jj][r];
            }
          }
        }
    zero();
    ra_cur = ra_nxt;
    rw_cur = rw_nxt;
    ra_nxt = rsrc_a(j + 2);
    rw_nxt = rsrc_w(j + 2);
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();
  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup
}

int num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

template <int EPI>
void launch(int variant, int ring, int nwv, bool sp, dim3 grid, hipStream_t st, const at::Tensor& x, const at::Tensor& w, int M, int K,
            at::Tensor& out, int MT, int NTL, int F, int gm) {
#define L(SV, NW, ...)                                                                                         \
  gemm_prefill_kernel<SV, EPI, NW, ##__VA_ARGS__><<<grid, NW * 64, 0, st>>>((const bf16*)x.data_ptr(), x.stride(0),                  \
                                                     (const bf16*)w.data_ptr(), M, K, (bf16*)out.data_ptr(),  \
                                                     out.stride(0), MT, NTL, F, gm)
  if (variant == 2 && K % 128 == 0) {
    const int ntiles = (int)grid.x;
    const int G = std::min(ntiles, num_cus());
    TORCH_CHECK((int64_t)x.size(0) * x.stride(0) * 2 < (1LL << 32) && w.numel() * 2 < (1LL << 32),
                "gemm_prefill: operands over 4 GB (32-bit buffer ranges)");
    gemm_pp2_kernel<EPI><<<G, 512, 0, st>>>((const bf16*)x.data_ptr(), x.stride(0), (const bf16*)w.data_ptr(),
                                           w.numel(), M, K, (bf16*)out.data_ptr(), out.stride(0), MT, NTL, F, gm,
                                           ntiles);
    return;
  }
  if ((variant == 1 || variant == 3 || variant == 4) && K % 128 == 0) {
    auto* xp = (const bf16*)x.data_ptr();
    auto* wp = (const bf16*)w.data_ptr();
    auto* op = (bf16*)out.data_ptr();
    if (variant == 3)
      gemm_pp_kernel<EPI, 1><<<grid, 512, 0, st>>>(xp, x.stride(0), wp, M, K, op, out.stride(0), MT, NTL, F, gm);
    else if (variant == 4)
      gemm_pp_kernel<EPI, 2><<<grid, 512, 0, st>>>(xp, x.stride(0), wp, M, K, op, out.stride(0), MT, NTL, F, gm);
    else
      gemm_pp_kernel<EPI, 0><<<grid, 512, 0, st>>>(xp, x.stride(0), wp, M, K, op, out.stride(0), MT, NTL, F, gm);
    return;
  }
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
void splitk_reduce_launch(const float* part, int S, int M, int N, bf16* out, int64_t ldo, hipStream_t st);

bool gemm_prefill_supported(const at::Tensor& w, bool silu) {
  if (w.dim() != 2 || w.scalar_type() != at::kBFloat16 || !w.is_contiguous() || w.size(1) % GBK != 0) return false;
  return silu ? (w.size(0) % 256 == 0) : (w.size(0) % TN == 0);
}

// silu == false: out[M, N] = x . w^T;  silu == true: out[M, F] = silu(x . w[:F]^T) * (x . w[F:]^T)
// variant: -1 = LS_PGEMM_KERNEL (default 1); 0 = the 32-deep ring kernel; 1 = the ping-pong kernel;
// 2 = its persistent form (the same schedule on 32x32x16 MFMA measured 1.27-1.29 PFLOP/s,
// 13-15 % below 16x16x32: profiles/pgemm_ab_r3_mfma32_v3.log, removed)
void gemm_prefill(at::Tensor out, at::Tensor x, at::Tensor w, bool silu, int64_t variant) {
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
  // default: the ping-pong kernel (1.48-1.50 PFLOP/s on the Llama-3-8B shapes at M = 16384,
  // 1.23-1.30 for kernel 0; the persistent form 2 measured 1-5 % slower than 1:
  // profiles/pgemm_ab_r3_pingpong_v1.log, pgemm_ab_r3_persistent_v2.log)
  static const int var_env = env_int("LS_PGEMM_KERNEL", 1);
  const int var = variant < 0 ? var_env : (int)variant;
  // Split-K for under-filled plain GEMMs on the ping-pong kernel (LS_PGEMM_SPLITK=0: off):
  // fewer than ~200 tiles on 256 CUs, S = min(4, 256 / tiles) K ranges of >= 8 tile
  // pairs.  Llama-3-8B at T = 1024 (profiles/r5/pgemm_midm_*): down 231 -> 102 us (S = 4,
  // 1.18 PFLOP/s), o 78 -> 51, qkv 78 -> 62; T = 2048: down 236 -> 175, o 76 -> 71
  static const int splitk_env = env_int("LS_PGEMM_SPLITK", 1);
  static const int splitk_min_k = env_int("LS_PGEMM_SPLITK_MIN_K", 4096);
  const int tiles = MT * NTL;
  int S = 1;
  if (!silu && var == 1 && splitk_env && K % 128 == 0 && K >= splitk_min_k && tiles < 200) {
    S = std::max(1, std::min({4, 256 / tiles, (int)(K / 128) / 8}));
  }
  if (S > 1) {
    at::Tensor part = at::empty({S, M, N}, x.options().dtype(at::kFloat));
    gemm_pp_kernel<EPI_STORE, 0><<<dim3((unsigned)(tiles * S)), 512, 0, stream>>>(
        (const bf16*)x.data_ptr(), x.stride(0), (const bf16*)w.data_ptr(), (int)M, (int)K, nullptr, 0, MT, NTL, 0, gm,
        S, part.data_ptr<float>());
    splitk_reduce_launch(part.data_ptr<float>(), S, (int)M, (int)N, (bf16*)out.data_ptr(), out.stride(0), stream);
    return;
  }
  if (silu) launch<EPI_SILU>(var, ring, nwv, sp, grid, stream, x, w, (int)M, (int)K, out, MT, NTL, (int)(N / 2), gm);
  else launch<EPI_STORE>(var, ring, nwv, sp, grid, stream, x, w, (int)M, (int)K, out, MT, NTL, 0, gm);
}

// out[M, N] (f32) = x . w^T on the ping-pong kernel (its split-K partial-tile epilogue with
// one split).  The LM head of decode batches of 129..256 rows: at M = 256, N = 128256 the
// head is MFMA-bound (269 GFLOP); 261 us here vs 279 on the bandwidth-shaped decode GEMM
// (profiles/r5/head_pp_r5ag.log).  Shapes: K % 128 == 0, N % 256 == 0.
bool gemm_prefill_f32_supported(const at::Tensor& w) {
  return w.dim() == 2 && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.size(1) % 128 == 0 &&
         w.size(0) % TN == 0;
}

void gemm_prefill_f32(at::Tensor out, at::Tensor x, at::Tensor w) {
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 &&
              x.stride(0) % 8 == 0, "x must be bf16 [M, K] with unit column stride");
  TORCH_CHECK(w.size(1) == K && gemm_prefill_f32_supported(w), "gemm_prefill_f32: unsupported weight shape");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.dim() == 2 && out.size(0) == M && out.size(1) == N &&
              out.is_contiguous(), "out must be a contiguous f32 [M, N]");
  TORCH_CHECK(x.device() == w.device() && out.device() == x.device(), "gemm_prefill_f32: tensors on different devices");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0,
              "gemm_prefill_f32: x and w must be 16-byte aligned");
  TORCH_CHECK(M < (1LL << 31) / TM);
  if (M == 0) return;
  const int MT = (int)((M + TM - 1) / TM), NTL = (int)(N / TN);
  static const int gm_env = env_int("LS_PGEMM_GROUP", 8);
  const int gm = std::max(1, std::min(gm_env, MT));
  gemm_pp_kernel<EPI_STORE, 0><<<dim3((unsigned)(MT * NTL)), 512, 0, at::hip::getCurrentHIPStream()>>>(
      (const bf16*)x.data_ptr(), x.stride(0), (const bf16*)w.data_ptr(), (int)M, (int)K, nullptr, 0, MT, NTL, 0, gm,
      1, out.data_ptr<float>());
}
