// Brute-force k-nearest-neighbour search for the local vector store
// (query-vector-db / `ORDER BY cosine_similarity(...) DESC LIMIT k`).
//
// Stage 1 (fused GEMM + chunk top-k): grid = N/1024 row chunks x ceil(Q/16) query
// groups, flattened and XCD-remapped (groups of a chunk share an XCD's L2).  Each wave streams 256 store rows through mfma_f32_16x16x32_bf16 as the
// A operand (one 16-B load per lane per MFMA, straight from HBM: the rows are read
// once per query group) against the 16 queries' Q^T fragments held in LDS.  Scores
// for the 1024 x 16 block go to LDS; each wave then extracts the top-k of 4 queries,
// filtered by a per-query score threshold (the K-th best of an exact search over a
// sample of the store; see the top-k comment in the kernel), appending (score, row)
// candidates to a per-query list.
// Select: one workgroup per query selects the global top-k from its candidates
// (k rounds of block-argmax over a short, L2-resident list).
//
// Measured (tools/engine_bench.py --what knn, 1M x 384, k=20; profiles/knn_*):
// per-chunk exact top-k (before) Q=256 1.96 ms; with a running atomic-max threshold
// 1.81 ms (stage 1 1.49 ms + select 0.33 ms: contention on the per-query atomics and
// long candidate lists).
//
// Scores are raw dot products; the store keeps rows L2-normalised so this is
// cosine similarity.  Rows >= N (tail chunk) score -inf.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

constexpr int CH = 1024;  // store rows per workgroup
constexpr int QG = 16;    // queries per workgroup (one MFMA column group)
// queries per workgroup of the thresholded main pass (their rows staged in LDS)
constexpr int qf_of(int dim) { return dim <= 512 ? 64 : dim <= 1024 ? 32 : 16; }
constexpr int SAMPLE_CHUNKS = 32;  // chunks searched exactly first, to set the per-query thresholds

// order-preserving float <-> int key (for atomic max on a float threshold)
__device__ __forceinline__ int f2key(float f) {
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float key2f(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF); }

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
__global__ void __launch_bounds__(256) knn_exact_kernel(const bf16* __restrict__ X, int64_t N,
                                                         const bf16* __restrict__ Qm, int Qn, int K,
                                                         float* __restrict__ cand_s, int32_t* __restrict__ cand_i,
                                                         int* __restrict__ ctrl, int nchunks_total, int chunk0,
                                                         int nchunks) {
  constexpr int KS = DIM / 32;
  constexpr int QROW = DIM + 8;   // +16 B per query row: the 16 lanes i16 of a B-fragment read hit distinct banks
  constexpr int KB = KS < 32 ? KS : 32;   // k-steps per load batch (DIM 2048: two batches)
  // subtiles whose A fragments are in flight together (<= 48 16-B loads per lane)
  constexpr int U = (48 / KB) >= 8 ? 8 : (48 / KB) >= 4 ? 4 : (48 / KB) >= 2 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) bf16 q_lds[QG * QROW];
  __shared__ float sc[QG][CH + 1];
  __shared__ float sh_thr[QG];
  // 1-D grid, XCD-aware: the query groups of one row chunk are consecutive logical ids
  // on one XCD, so the chunk's rows come from HBM once and from that XCD's L2 after
  // (with grid (chunks, groups) every group re-streamed the whole store from HBM).
  const int nqg = gridDim.x / nchunks;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int lchunk = logical / nqg, qg = logical - lchunk * nqg;
  const int chunk = chunk0 + lchunk;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, h = lane >> 4;
  // stage the 16 queries (zero rows past Qn) and their score thresholds
  for (int c = threadIdx.x; c < QG * DIM / 8; c += 256) {
    const int qq = c / (DIM / 8), cc = c - qq * (DIM / 8);
    const int qi = qg * QG + qq;
    *reinterpret_cast<uint4*>(&q_lds[qq * QROW + cc * 8]) =
        qi < Qn ? ld16(Qm + (int64_t)qi * DIM + cc * 8) : make_uint4(0, 0, 0, 0);
  }
  if (threadIdx.x < QG) {
    const int qi = qg * QG + threadIdx.x;
    sh_thr[threadIdx.x] = qi < Qn ? key2f(ctrl[Qn + qi]) : INFINITY;
  }
  __syncthreads();
  const int64_t row0 = (int64_t)chunk * CH + wid * 256;
  for (int st0 = 0; st0 < 16; st0 += U) {
    f32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KS; kb += KB) {
      uint4 af[U][KB];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = row0 + (st0 + u) * 16 + i16;
        const bf16* xr = X + (r < N ? r : 0) * DIM + 8 * h + 32 * kb;
#pragma unroll
        for (int ks = 0; ks < KB; ++ks) af[u][ks] = ld16(xr + 32 * ks);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int ks = 0; ks < KB; ++ks) {
          const bf16x8 bq = *reinterpret_cast<const bf16x8*>(&q_lds[i16 * QROW + 32 * (kb + ks) + 8 * h]);
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[u][ks]), bq, acc[u], 0, 0, 0);
        }
    }
    // acc[u][rr] = score(row 4h+rr of subtile st0+u, query i16)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int lr = wid * 256 + (st0 + u) * 16 + 4 * h + rr;
        sc[i16][lr] = row0 + (st0 + u) * 16 + 4 * h + rr < N ? acc[u][rr] : -INFINITY;
      }
  }
  __syncthreads();
  // top-K per query: wave w handles queries w, w+4, w+8, w+12.  Every lane holds 16 of
  // the chunk's 1024 scores in registers.
  //
  // Threshold: thr[q] is the K-th best score over a SAMPLE of the store (the first
  // chunks, searched exactly by an earlier launch), so it lower-bounds the final K-th
  // best and scores below it can never be in the answer.  Almost every (chunk, query)
  // of the main pass then finds no score >= thr and costs one ballot per register; the
  // few chunks that can contribute append at most K candidates to the query's list
  // (one atomic slot reservation per chunk; capacity nchunks*K can never overflow).
  // The sample launch itself runs with thr = -inf.
  //
  // Selection inside a contributing chunk: if more than 64 scores pass, the K-th
  // largest of the 64 lane maxima, Tl, is a second lower bound (the K lanes owning
  // those maxima each hold a score >= Tl); scores >= max(thr, Tl) are compacted by
  // ballot into a 64-slot LDS list and bitonic-sorted across the wave.  When more than
  // 64 still pass (heavy ties, or a tail chunk of -inf rows) the wave falls back to K
  // rounds of argmax over LDS.
  __shared__ float cv_lds[4][64];
  __shared__ int ci_lds[4][64];
  const int64_t cap = (int64_t)nchunks_total * K;
  for (int qq = wid; qq < QG; qq += 4) {
    const int qi = qg * QG + qq;
    if (qi >= Qn) continue;
    int* cnt = ctrl + qi;
    float* outs = cand_s + (int64_t)qi * cap;
    int32_t* outi = cand_i + (int64_t)qi * cap;
    float v[CH / 64];
#pragma unroll
    for (int j = 0; j < CH / 64; ++j) v[j] = sc[qq][lane + 64 * j];
    const float T0 = sh_thr[qq];
    int count = 0;
#pragma unroll
    for (int j = 0; j < CH / 64; ++j) count += __popcll(__ballot(v[j] >= T0));
    if (count == 0) continue;
    float T = T0;
    if (count > 64) {
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < CH / 64; ++j) m = fmaxf(m, v[j]);
      int ti = lane;
      wave_sort_desc(m, ti, lane);
      T = fmaxf(T0, __shfl(m, K - 1, 64));
    }
    int count2 = 0;
    if (T > -INFINITY) {
#pragma unroll
      for (int j = 0; j < CH / 64; ++j) {
        const bool p = v[j] >= T;
        const uint64_t mask = __ballot(p);
        const int pos = count2 + __popcll(mask & ((1ull << lane) - 1ull));
        if (p && pos < 64) {
          cv_lds[wid][pos] = v[j];
          ci_lds[wid][pos] = lane + 64 * j;
        }
        count2 += __popcll(mask);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (T > -INFINITY && count2 <= 64) {
      float cvv = lane < count2 ? cv_lds[wid][lane] : -INFINITY;
      int cii = lane < count2 ? ci_lds[wid][lane] : CH;
      const int n = min(count2, K);
      if (count2 > K) wave_sort_desc(cvv, cii, lane);
      int base = 0;
      if (lane == 0) base = __hip_atomic_fetch_add(cnt, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      base = __shfl(base, 0, 64);
      if (lane < n) {
        outs[base + lane] = cvv;
        outi[base + lane] = (int32_t)((int64_t)chunk * CH + cii);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      continue;
    }
    int base = 0;
    if (lane == 0) base = __hip_atomic_fetch_add(cnt, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    base = __shfl(base, 0, 64);
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
        outs[base + k] = bv;
        outi[base + k] = bi < CH ? (int32_t)((int64_t)chunk * CH + bi) : -1;
        if (bi < CH) sc[qq][bi] = -INFINITY;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}


// Main pass: the rows of the chunks after the sample, 64 queries per workgroup at
// dim <= 512 (four MFMA column groups share every A fragment, so the store streams
// through L2 a quarter as often as with 16), scores stay in the MFMA accumulators and only those strictly
// above the query's sample threshold are appended to its list.  Strict: a row outside
// the sample that TIES the sample's K-th best loses to it on row index, since the
// sample is the lowest rows.  A list that fills up (adversarial data: many rows above
// the sample's K-th best) sets the query's overflow flag; the host then reruns the
// search exactly.
template <int DIM>
__global__ void __launch_bounds__(256) knn_filter_kernel(const bf16* __restrict__ X, int64_t N,
                                                         const bf16* __restrict__ Qm, int Qn,
                                                         float* __restrict__ cand_s, int32_t* __restrict__ cand_i,
                                                         int* __restrict__ ctrl, int64_t cap, int chunk0,
                                                         int nchunks) {
  constexpr int KS = DIM / 32;
  constexpr int QROW = DIM + 8;
  constexpr int KB = KS < 32 ? KS : 32;
  constexpr int U = KB <= 6 ? 4 : KB <= 12 ? 2 : 1;
  constexpr int QF = qf_of(DIM);
  __shared__ __attribute__((aligned(16))) bf16 q_lds[QF * QROW];
  const int nqf = gridDim.x / nchunks;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int lchunk = logical / nqf, qf = logical - lchunk * nqf;
  const int chunk = chunk0 + lchunk;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i16 = lane & 15, h = lane >> 4;
  for (int c = threadIdx.x; c < QF * DIM / 8; c += 256) {
    const int qq = c / (DIM / 8), cc = c - qq * (DIM / 8);
    const int qi = qf * QF + qq;
    *reinterpret_cast<uint4*>(&q_lds[qq * QROW + cc * 8]) =
        qi < Qn ? ld16(Qm + (int64_t)qi * DIM + cc * 8) : make_uint4(0, 0, 0, 0);
  }
  // this lane's 4 queries: column i16 of each group g
  float thr[QF / 16];
#pragma unroll
  for (int g = 0; g < QF / 16; ++g) {
    const int qi = qf * QF + 16 * g + i16;
    thr[g] = qi < Qn ? key2f(ctrl[Qn + qi]) : INFINITY;
  }
  __syncthreads();
  const int64_t row0 = (int64_t)chunk * CH + wid * 256;
  for (int st0 = 0; st0 < 16; st0 += U) {
    f32x4 acc[U][QF / 16];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int g = 0; g < QF / 16; ++g) acc[u][g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KS; kb += KB) {
      uint4 af[U][KB];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = row0 + (st0 + u) * 16 + i16;
        const bf16* xr = X + (r < N ? r : 0) * DIM + 8 * h + 32 * kb;
#pragma unroll
        for (int ks = 0; ks < KB; ++ks) af[u][ks] = ld16(xr + 32 * ks);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KB; ++ks)
#pragma unroll
        for (int g = 0; g < QF / 16; ++g) {
          const bf16x8 bq = *reinterpret_cast<const bf16x8*>(&q_lds[(16 * g + i16) * QROW + 32 * (kb + ks) + 8 * h]);
#pragma unroll
          for (int u = 0; u < U; ++u)
            acc[u][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[u][ks]), bq, acc[u][g],
                                                                0, 0, 0);
        }
    }
    // acc[u][g][rr] = score(row 4h+rr of subtile st0+u, query 16g+i16)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int g = 0; g < QF / 16; ++g)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int64_t row = row0 + (st0 + u) * 16 + 4 * h + rr;
          if (acc[u][g][rr] > thr[g] && row < N) {
            const int qi = qf * QF + 16 * g + i16;
            const int slot = __hip_atomic_fetch_add(ctrl + qi, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (slot < cap) {
              cand_s[(int64_t)qi * cap + slot] = acc[u][g][rr];
              cand_i[(int64_t)qi * cap + slot] = (int32_t)row;
            } else {
              ctrl[2 * Qn + qi] = 1;
            }
          }
        }
  }
}

// Main pass for large query batches (Q >= 128, dim <= 512): 256 queries per workgroup,
// 8 waves x 32 queries whose Q^T fragments stay in REGISTERS for the whole launch, and
// the workgroup's row range streamed ONCE through a ring of LDS stages (64 rows each,
// LDS-DMA) that all 8 waves read.  knn_filter_kernel instead re-reads every row from L2
// per 64 queries straight into registers, which bounded it by the L2 -> CU path at
// Q = 1024 (412 GB/s effective over 1M x 384; profiles/knn_filter64_r2i.log).
//   * LDS image: row r's 16-B chunk p holds the row's chunk p ^ (r & 15) (rows are a
//     multiple of 256 B, so without it the 16 rows of an A-fragment lane group would
//     sit on the same banks); the LDS-DMA writes lane-linear, so the permutation is
//     applied to the SOURCE address (cdna_hip_programming §5.4 rule 21);
//   * per 64-row tile a wave reads 4 x KS A fragments and issues 8 x KS MFMAs (two
//     16-query groups share each fragment);
//   * scores above the query's sample threshold are appended exactly as in
//     knn_filter_kernel (same candidate lists, counters and overflow flags).
// Ablations at Q = 2048 (profiles/knn_ablation_r4.txt): with reads pinned ahead of each
// subtile, dropping the MFMAs left 523 of 1625 us (reads and MFMAs ran in phases, not
// overlapped); interleaved (below) the pass takes 1572 us and 1337 without MFMAs -- the
// fragment-read stream, not the MFMA pipe or the DMA / barrier (1378 without them), now
// bounds it.
// Measured at Q = 2048 over 1M x 384 (profiles/knn_pmc_r4/): MFMA busy ~41 %, waves
// parked in waitcnt / barrier ~49 %, L2 hit 85 %, LDS array ~23 % busy.  Dead ends: a
// one-ballot epilogue test + buffer-resource DMA addressing + pinned fragment reads (VALU
// per MFMA 5.7 -> ~1.5 in the loop: no change in time), moving the barrier to mid-tile
// so the next tile's first fragments load under this tile's last MFMAs (1.607 vs 1.598 ms).
//
// MODE 0: append scores > thr (the rows after an exact sample, see above);
// MODE 1: append scores >= thr over the WHOLE store (thr from a MODE 2 pass: a lower
//         bound attained by K distinct rows, so every row of the answer is >= thr);
// MODE 2: no appends -- the running max of every (lane, accumulator register) slot,
//         i.e. of 16 disjoint row groups per query per workgroup, written to
//         gmax[q * G + 16 * rb + 4h + rr] (knn_group_thr_kernel turns them into thr).
// NW: waves per workgroup -- 8 (two per SIMD, 32 queries per wave; launched) or 4 (one
// per SIMD, 64 queries per wave: each A fragment feeds 4 query groups, half the LDS reads
// per MFMA, up to 512 registers).  NW = 4 measured 2.62 vs 1.61 ms at Q = 2048: with one
// wave per SIMD nothing covers a wave's waits (profiles/knn_nw_r4v/).
// ABL (timing-only diagnosis, wrong results): 1 drops the in-loop vmcnt wait + barrier,
// 2 also the LDS-DMA issue, 3 drops the MFMAs instead.
template <int DIM, int MODE, int NW = 8, int ABL = 0>
__global__ void __launch_bounds__(NW * 64, 1) knn_filter_q256_kernel(const bf16* __restrict__ X, int64_t N,
                                                              const bf16* __restrict__ Qm, int Qn,
                                                              float* __restrict__ cand_s, int32_t* __restrict__ cand_i,
                                                              int* __restrict__ ctrl, int64_t cap, int64_t row_begin,
                                                              int rows_per_wg, int nqb, float* __restrict__ gmax,
                                                              int G, int prio) {
  constexpr int KS = DIM / 32;
  constexpr int RB = DIM * 2;                    // bytes per row
  constexpr int TR = 64;                         // rows per LDS stage
  constexpr int SB = TR * RB;                    // stage bytes
  constexpr int CAPW = 128;                      // per-wave LDS candidate buffer entries
  constexpr int QGW = 256 / NW / 16;             // 16-query groups per wave
  constexpr int CBYTES = NW * CAPW * 12;
  constexpr int NST = 3 * SB + CBYTES <= 160 * 1024 ? 3 : 2;
  constexpr int GPW = SB / (NW * 1024);          // LDS-DMA instructions per wave per stage
  static_assert(NW == 8 || NW == 4, "waves per workgroup");
  static_assert(RB % 256 == 0 && SB % 8192 == 0, "rows must be a multiple of 256 B");
  __shared__ __attribute__((aligned(1024))) char lds[NST * SB + CBYTES];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, h = lane >> 4;
  // prio 1: the second half of the waves (one per SIMD) at raised priority for the whole
  // launch, so the two waves of a SIMD drift out of lockstep; prio 2: MFMA clusters at
  // raised priority (cdna_hip_programming T5)
  if (prio == 1 && wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  // candidates above the threshold go to this wave's LDS buffer (ballot-compacted, no
  // atomics) and reach the global lists only in flush(): a returning global atomic inside
  // the tile loop made hipcc drain vmcnt(0) every tile, i.e. the whole LDS-DMA ring
  float* c_s = reinterpret_cast<float*>(lds + NST * SB) + wid * CAPW;
  int* c_r = reinterpret_cast<int*>(lds + NST * SB + NW * CAPW * 4) + wid * CAPW;
  int* c_q = reinterpret_cast<int*>(lds + NST * SB + NW * CAPW * 8) + wid * CAPW;
  int ccount = 0;   // wave-uniform
  auto flush = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int e = lane; e < ccount; e += 64) {
      const int qi = c_q[e];
      const int slot = __hip_atomic_fetch_add(ctrl + qi, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (slot < cap) {
        cand_s[(int64_t)qi * cap + slot] = c_s[e];
        cand_i[(int64_t)qi * cap + slot] = c_r[e];
      } else {
        ctrl[2 * Qn + qi] = 1;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    ccount = 0;
  };
  // XCD-aware: the query blocks of one row range are consecutive logical ids
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int rb = logical / nqb, qb = logical - rb * nqb;
  const int64_t r0 = row_begin + (int64_t)rb * rows_per_wg;
  const int64_t r1 = min(N, r0 + rows_per_wg);
  if (r0 >= r1) return;
  const int nrows = (int)(r1 - r0);
  const int ntile = (nrows + TR - 1) / TR;

  // this wave's 16 QGW queries: groups g of 16; lane (fr, h) holds query 16g + fr, dims 32ks + 8h..
  const int q0 = qb * 256 + wid * (16 * QGW);
  bf16x8 qf[QGW][KS];
  float thr[QGW];
#pragma unroll
  for (int g = 0; g < QGW; ++g) {
    const int qi = q0 + 16 * g + fr;
    const bool ok = qi < Qn;
    const bf16* qp = Qm + (int64_t)(ok ? qi : 0) * DIM + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[g][ks] = __builtin_bit_cast(bf16x8, ok ? ld16(qp + 32 * ks) : make_uint4(0, 0, 0, 0));
    thr[g] = MODE == 2 ? -INFINITY : ok ? key2f(ctrl[Qn + qi]) : INFINITY;
  }
  // consume the query fragments here: otherwise hipcc places their vmcnt wait at the first
  // MFMA inside the tile loop, where a vmcnt(0) also drains the LDS-DMA ring every tile
#pragma unroll
  for (int g = 0; g < QGW; ++g) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(qf[g][ks]));
    asm volatile("" ::"v"(thr[g]));
  }
  // LDS-DMA: instruction j of wave w fills bytes [(w*GPW + j) * 1024, +1024) of a stage,
  // through a buffer resource over this workgroup's rows: the per-lane offsets are
  // tile-invariant (a tile adds t * SB), no 64-bit address math per load, and rows past
  // the range read as zeros (their scores are masked by lr < nrows).
  const i32x4 rsrc = make_rsrc((const char*)X + r0 * RB, (uint32_t)nrows * RB);
  int voff[GPW];
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const int o = (wid * GPW + j) * 1024 + lane * 16;
    const int r = o / RB, p = (o % RB) / 16;
    voff[j] = r * RB + ((p ^ (r & 15)) * 16);
  }
  const unsigned lds_base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  auto issue = [&](int t, int slot) {
    const int toff = min(t, ntile - 1) * SB;   // past the end: reload the last tile (dead slot)
#pragma unroll
    for (int j = 0; j < GPW; ++j)
      blds16(rsrc, voff[j] + toff, 0, lds_base + slot * SB + (wid * GPW + j) * 1024);
  };
  // A fragment of 16-row subtile i, k-step ks: row 16i + fr, chunk 4ks + h (swizzled)
  int aoff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) aoff[ks] = fr * RB + (((4 * ks + h) ^ fr) * 16);

  // Score epilogues run one subtile behind the MFMAs that produce them: subtile i's
  // compare / ballot / append is issued after subtile i+1's MFMAs, so the wave never waits
  // on an MFMA result it has just requested (two accumulator sets alternate; the last
  // subtile of a tile is checked after the next tile's first MFMAs).
  auto mm = [&](const bf16x8 (&f)[KS], f32x4 (&acc)[QGW]) {
    if (prio == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int g = 0; g < QGW; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int g = 0; g < QGW; ++g) {
        if constexpr (ABL == 3) {
          asm volatile("" ::"v"(f[ks]));
        } else {
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[ks], qf[g][ks], acc[g], 0, 0, 0);
        }
      }
    if (prio == 2) __builtin_amdgcn_s_setprio(0);
  };
  // acc[g][rr] = score(row r0 + sr0 + 4h + rr, query q0 + 16g + fr); sr0 = subtile's first row.
  // Fast test first: one ballot over the subtile's 8 scores per lane (hits are rare -- only
  // rows above the query's sample threshold), the per-score ballots only when it fires.
  float gm[QGW][4];   // MODE 2: running max per (query group, accumulator register)
#pragma unroll
  for (int g = 0; g < QGW; ++g)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) gm[g][rr] = -INFINITY;
  auto pass = [&](float v, float t) { return MODE == 0 ? v > t : v >= t; };
  auto epi = [&](int sr0, const f32x4 (&acc)[QGW]) {
    if constexpr (MODE == 2) {
      const bool tail = sr0 + 16 > nrows;   // wave-uniform
#pragma unroll
      for (int g = 0; g < QGW; ++g)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          gm[g][rr] = fmaxf(gm[g][rr], tail && sr0 + 4 * h + rr >= nrows ? -INFINITY : acc[g][rr]);
      return;
    }
    bool any = false;
#pragma unroll
    for (int g = 0; g < QGW; ++g)
      any |= pass(fmaxf(fmaxf(acc[g][0], acc[g][1]), fmaxf(acc[g][2], acc[g][3])), thr[g]);
    if (__ballot(any) == 0) return;
#pragma unroll
    for (int g = 0; g < QGW; ++g)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int lr = sr0 + 4 * h + rr;
        const bool hit = pass(acc[g][rr], thr[g]) && lr < nrows;
        const uint64_t mask = __ballot(hit);
        if (mask == 0) continue;
        const int nh = __popcll(mask);
        if (ccount + nh > CAPW) flush();   // rare: drains the DMA ring once
        const int pos = ccount + __popcll(mask & ((1ull << lane) - 1ull));
        if (hit) {
          c_s[pos] = acc[g][rr];
          c_r[pos] = (int)(r0 + lr);
          c_q[pos] = q0 + 16 * g + fr;
        }
        ccount += nh;
      }
  };
  f32x4 accA[QGW], accB[QGW];
  int pend = -1;   // first row of the subtile whose scores wait in accB (-1: none)
  for (int s = 0; s < NST - 1; ++s) issue(s, s);
  for (int t = 0; t < ntile; ++t) {
    if constexpr (ABL != 1 && ABL != 2) {
      wait_vmcnt<(NST - 2) * GPW>();   // this wave's DMA of tile t landed (tiles t+1.. may be in flight)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();    // every wave's part of tile t landed; tile t-1's slot is free
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (ABL != 2) issue(t + NST - 1, (t + NST - 1) % NST);
    const char* st = lds + (t % NST) * SB;
    const int tl0 = t * TR;   // tile's first row, relative to r0
    // A fragments double-buffered across the tile's four 16-row subtiles: subtile i+1's
    // LDS reads are in flight while subtile i's MFMAs run
    bf16x8 fa[KS], fb[KS];
    auto rd = [&](int i, bf16x8 (&f)[KS]) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) f[ks] = __builtin_bit_cast(bf16x8, ld16(st + i * 16 * RB + aoff[ks]));
    };
    if constexpr (DIM > 384) {
      // one fragment set: two of them beside the query fragments exceed 256 VGPRs
      rd(0, fa);
      mm(fa, accA);
      if (pend >= 0) epi(pend, accB);
      rd(1, fa);
      mm(fa, accB);
      epi(tl0, accA);
      rd(2, fa);
      mm(fa, accA);
      epi(tl0 + 16, accB);
      rd(3, fa);
      mm(fa, accB);
      epi(tl0 + 32, accA);
      pend = tl0 + 48;
      continue;
    }
    if constexpr (DIM <= 384) {
      // instruction-level interleave: the next subtile's fragment reads ride between this
      // subtile's MFMAs (per k-step one ds_read, QGW MFMAs), so a wave is never in an
      // all-read or all-MFMA phase (sched_group_barrier, one sync group).  Q = 2048: 1.585
      // vs 1.635 ms for reads pinned ahead of each subtile (profiles/knn_ilv_r4y/, with the
      // MFMA clusters at raised priority)
      auto mmrd = [&](const bf16x8 (&f)[KS], f32x4 (&acc)[QGW], bf16x8 (&nf)[KS], int inext) {
        if (prio == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int g = 0; g < QGW; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          nf[ks] = __builtin_bit_cast(bf16x8, ld16(st + inext * 16 * RB + aoff[ks]));
#pragma unroll
          for (int g = 0; g < QGW; ++g)
            acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[ks], qf[g][ks], acc[g], 0, 0, 0);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);     // 1 ds_read
          __builtin_amdgcn_sched_group_barrier(0x008, QGW, 0);   // QGW MFMAs
        }
        if (prio == 2) __builtin_amdgcn_s_setprio(0);
      };
      rd(0, fa);
      mmrd(fa, accA, fb, 1);              // subtile 0, reads 1
      if (pend >= 0) epi(pend, accB);
      mmrd(fb, accB, fa, 2);              // subtile 1, reads 2
      epi(tl0, accA);
      mmrd(fa, accA, fb, 3);              // subtile 2, reads 3
      epi(tl0 + 16, accB);
      mm(fb, accB);                       // subtile 3
      epi(tl0 + 32, accA);
      pend = tl0 + 48;
      continue;
    }
    // sched_barriers pin each subtile's reads ahead of the previous subtile's MFMAs:
    // left alone, hipcc sinks every read to just before its MFMA behind an lgkmcnt wait
#define KNN_SB __builtin_amdgcn_sched_barrier(0)
    rd(0, fa);
    rd(1, fb);
    KNN_SB;
    mm(fa, accA);                       // subtile 0
    if (pend >= 0) epi(pend, accB);     // the previous tile's subtile 3
    KNN_SB;
    rd(2, fa);
    KNN_SB;
    mm(fb, accB);                       // subtile 1
    epi(tl0, accA);
    KNN_SB;
    rd(3, fb);
    KNN_SB;
    mm(fa, accA);                       // subtile 2
    epi(tl0 + 16, accB);
    KNN_SB;
    mm(fb, accB);                       // subtile 3
    epi(tl0 + 32, accA);
#undef KNN_SB
    pend = tl0 + 48;
  }
  if (pend >= 0) epi(pend, accB);
  wait_vmcnt<0>();   // no LDS-DMA may outlive the workgroup
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (MODE == 2) {
#pragma unroll
    for (int g = 0; g < QGW; ++g) {
      const int qi = q0 + 16 * g + fr;
      if (qi < Qn)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) gmax[(int64_t)qi * G + 16 * rb + 4 * h + rr] = gm[g][rr];
    }
    return;
  }
  flush();
}

// thr[q] = the K-th largest of 64 group maxima (lane l: max over groups l, l+64, ...):
// K disjoint row groups each hold a row scoring >= thr, so the answer's K-th best is
// >= thr (a lower bound attained by K distinct rows).  One wave per query.
__global__ void __launch_bounds__(256) knn_group_thr_kernel(const float* __restrict__ gmax, int G, int Qn, int K,
                                                            int* __restrict__ ctrl) {
  const int lane = threadIdx.x & 63;
  const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= Qn) return;
  float m = -INFINITY;
  for (int j = lane; j < G; j += 64) m = fmaxf(m, gmax[(int64_t)qi * G + j]);
  int idx = lane;
  wave_sort_desc(m, idx, lane);
  const float t = __shfl(m, K - 1, 64);
  if (lane == 0) ctrl[Qn + qi] = f2key(t);
}

template <int DD, int MM>
void launch_q256(int abl, dim3 grid, hipStream_t stream, const bf16* X, int64_t N, const bf16* Q, int Qn, float* ws_s,
                 int32_t* ws_i, int* ctrl, int64_t cap, int64_t row_begin, int rpw, int nqb, int G) {
  // LS_KNN_PRIO: 2 (default) MFMA clusters at raised priority, 1 half the waves raised, 0 none
  static const int prio = getenv("LS_KNN_PRIO") ? atoi(getenv("LS_KNN_PRIO")) : 2;
  // the timing-only ablations exist for the bench's shape (384 dims, main pass) only
  if constexpr (DD == 384 && MM == 1) {
    switch (abl) {
      case 1:
        knn_filter_q256_kernel<DD, MM, 8, 1><<<grid, 512, 0, stream>>>(X, N, Q, Qn, ws_s, ws_i, ctrl, cap, row_begin,
                                                                       rpw, nqb, ws_s, G, prio);
        return;
      case 2:
        knn_filter_q256_kernel<DD, MM, 8, 2><<<grid, 512, 0, stream>>>(X, N, Q, Qn, ws_s, ws_i, ctrl, cap, row_begin,
                                                                       rpw, nqb, ws_s, G, prio);
        return;
      case 3:
        knn_filter_q256_kernel<DD, MM, 8, 3><<<grid, 512, 0, stream>>>(X, N, Q, Qn, ws_s, ws_i, ctrl, cap, row_begin,
                                                                       rpw, nqb, ws_s, G, prio);
        return;
      default:
        break;
    }
  }
  knn_filter_q256_kernel<DD, MM, 8><<<grid, 512, 0, stream>>>(X, N, Q, Qn, ws_s, ws_i, ctrl, cap, row_begin, rpw, nqb,
                                                              ws_s, G, prio);
}

__global__ void knn_init_kernel(int* __restrict__ ctrl, int Qn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < Qn) {
    ctrl[i] = 0;
    ctrl[Qn + i] = f2key(-INFINITY);
    ctrl[2 * Qn + i] = 0;
  }
}

// Bitonic merge of a bitonic 64-sequence into descending order (ties: lower index first).
__device__ __forceinline__ void wave_merge_desc(float& v, int& i, int lane) {
#pragma unroll
  for (int j = 32; j > 0; j >>= 1) {
    const float ov = __shfl_xor(v, j, 64);
    const int oi = __shfl_xor(i, j, 64);
    const bool other_first = ov > v || (ov == v && oi < i);
    const bool lower = (lane & j) == 0;
    if (lower ? other_first : !other_first) { v = ov; i = oi; }
  }
}

// One wave per query: the top-K of the query's candidate list, ordered by score then
// row index (so the answer does not depend on the order candidates were appended).
// The wave keeps its best 64 sorted across lanes; each batch of 64 candidates is
// skipped when none beats the current K-th best, else sorted and merged (max of best[i]
// and batch[63-i] is bitonic and holds the top 64 of both).
// write_thr: store the K-th best score as the query's threshold instead of the answer.
__global__ void __launch_bounds__(256) knn_select_kernel(const float* __restrict__ cand_s,
                                                         const int32_t* __restrict__ cand_i, int* __restrict__ ctrl,
                                                         int Qn, int64_t cap, int K, float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_i, int write_thr) {
  const int lane = threadIdx.x & 63;
  const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= Qn) return;
  const int n = (int)min((int64_t)ctrl[qi], cap);
  const float* cs = cand_s + (int64_t)qi * cap;
  const int32_t* ci = cand_i + (int64_t)qi * cap;
  float bv = -INFINITY;
  int br = INT_MAX;
  float nv = -INFINITY;
  int nr = INT_MAX;
  if (lane < n) {
    nv = cs[lane];
    nr = ci[lane];
  }
  for (int base = 0; base < n; base += 64) {
    float v = nv;
    int r = nr < 0 || v == -INFINITY ? INT_MAX : nr;
    nv = -INFINITY;
    nr = INT_MAX;
    if (base + 64 + lane < n) {   // prefetch the next batch
      nv = cs[base + 64 + lane];
      nr = ci[base + 64 + lane];
    }
    const float kv = __shfl(bv, K - 1, 64);
    const int kr = __shfl(br, K - 1, 64);
    if (__ballot(v > kv || (v == kv && r < kr)) == 0) continue;
    wave_sort_desc(v, r, lane);
    const float ov = __shfl(v, 63 - lane, 64);
    const int orr = __shfl(r, 63 - lane, 64);
    if (ov > bv || (ov == bv && orr < br)) { bv = ov; br = orr; }
    wave_merge_desc(bv, br, lane);
  }
  if (write_thr) {
    const float kv = __shfl(bv, K - 1, 64);
    if (lane == 0) ctrl[Qn + qi] = f2key(kv);   // -inf when the sample holds fewer than K rows
  } else if (lane < K) {
    out_s[(int64_t)qi * K + lane] = bv;
    out_i[(int64_t)qi * K + lane] = bv > -INFINITY && br != INT_MAX ? br : -1;
  }
}

// Long candidate lists (the group-max path: ~K * N / sample-rows per query): one
// WORKGROUP per query, its 4 waves each keep the best 64 of every 4th batch (the loop of
// knn_select_kernel), then wave 0 merges the four sorted lists from LDS.  A quarter of
// the serial batch chain per wave, and 4x the waves in flight.
__global__ void __launch_bounds__(256) knn_select4_kernel(const float* __restrict__ cand_s,
                                                          const int32_t* __restrict__ cand_i,
                                                          const int* __restrict__ ctrl, int Qn, int64_t cap, int K,
                                                          float* __restrict__ out_s, int32_t* __restrict__ out_i) {
  __shared__ float lv[4][64];
  __shared__ int lr[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int qi = blockIdx.x;
  const int n = (int)min((int64_t)ctrl[qi], cap);
  const float* cs = cand_s + (int64_t)qi * cap;
  const int32_t* ci = cand_i + (int64_t)qi * cap;
  float bv = -INFINITY;
  int br = INT_MAX;
  float nv = -INFINITY;
  int nr = INT_MAX;
  if (wid * 64 + lane < n) {
    nv = cs[wid * 64 + lane];
    nr = ci[wid * 64 + lane];
  }
  for (int base = wid * 64; base < n; base += 256) {
    float v = nv;
    int r = nr < 0 || v == -INFINITY ? INT_MAX : nr;
    nv = -INFINITY;
    nr = INT_MAX;
    if (base + 256 + lane < n) {
      nv = cs[base + 256 + lane];
      nr = ci[base + 256 + lane];
    }
    const float kv = __shfl(bv, K - 1, 64);
    const int kr = __shfl(br, K - 1, 64);
    if (__ballot(v > kv || (v == kv && r < kr)) == 0) continue;
    wave_sort_desc(v, r, lane);
    const float ov = __shfl(v, 63 - lane, 64);
    const int orr = __shfl(r, 63 - lane, 64);
    if (ov > bv || (ov == bv && orr < br)) { bv = ov; br = orr; }
    wave_merge_desc(bv, br, lane);
  }
  lv[wid][lane] = bv;
  lr[wid][lane] = br;
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int w = 1; w < 4; ++w) {
    const float ov = lv[w][63 - lane];
    const int orr = lr[w][63 - lane];
    if (ov > bv || (ov == bv && orr < br)) { bv = ov; br = orr; }
    wave_merge_desc(bv, br, lane);
  }
  if (lane < K) {
    out_s[(int64_t)qi * K + lane] = bv;
    out_i[(int64_t)qi * K + lane] = bv > -INFINITY && br != INT_MAX ? br : -1;
  }
}

}  // namespace

// X: [N, dim] bf16 (rows L2-normalised), Q: [Qn, dim] bf16.  Returns via out tensors
// the top-K scores (f32 [Qn, K]) and row indices (int32 [Qn, K], -1 if N < K).
// workspace: f32 [Qn * nchunks * K] and int32 [Qn * nchunks * K + 3 * Qn] (candidate
// lists, then per-query candidate counts, thresholds and overflow flags).
//
// Launch sequence: init; exact per-chunk top-K over the first `sample` chunks; select
// (K-th best of the sample -> threshold); thresholded main pass over the rest; select
// (answer).  sample <= 0 or >= nchunks: every chunk is searched exactly.  The caller
// checks the overflow flags (ws_i tail) and reruns exactly if any is set.
namespace {
void knn_topk_impl(at::Tensor X, at::Tensor Q, int64_t K, at::Tensor out_s, at::Tensor out_i, at::Tensor ws_s,
                   at::Tensor ws_i, int64_t sample, int abl_req) {
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 && Q.scalar_type() == at::kBFloat16);
  TORCH_CHECK(X.is_contiguous() && Q.is_contiguous() && X.dim() == 2 && Q.dim() == 2);
  const int dim = X.size(1);
  TORCH_CHECK(Q.size(1) == dim);
  TORCH_CHECK(K >= 1 && K <= 64);
  const int64_t N = X.size(0);
  const int Qn = Q.size(0);
  const int nchunks = (int)((N + CH - 1) / CH);
  TORCH_CHECK(ws_s.numel() >= (int64_t)Qn * nchunks * K && ws_i.numel() >= (int64_t)Qn * nchunks * K + 3 * Qn,
              "kNN workspace too small");
  TORCH_CHECK(out_s.numel() >= (int64_t)Qn * K && out_i.numel() >= (int64_t)Qn * K);
  if (Qn == 0 || N == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const int nqg = (Qn + QG - 1) / QG, nqf = (Qn + qf_of(dim) - 1) / qf_of(dim);
  TORCH_CHECK((int64_t)nchunks * nqg < (1LL << 31), "kNN grid too large");
  int* ctrl = ws_i.data_ptr<int32_t>() + (int64_t)Qn * nchunks * K;
  const int64_t cap = (int64_t)nchunks * K;
  knn_init_kernel<<<(Qn + 255) / 256, 256, 0, stream>>>(ctrl, Qn);
#define DISPATCH_DIM(LAUNCH)                                       \
  switch (dim) {                                                   \
    case 128: LAUNCH(128); break;                                  \
    case 256: LAUNCH(256); break;                                  \
    case 384: LAUNCH(384); break;                                  \
    case 512: LAUNCH(512); break;                                  \
    case 768: LAUNCH(768); break;                                  \
    case 1024: LAUNCH(1024); break;                                \
    case 1536: LAUNCH(1536); break;                                \
    case 2048: LAUNCH(2048); break;                                \
    default: TORCH_CHECK(false, "unsupported embedding dim ", dim); \
  }
  auto exact = [&](int nc) {
    dim3 grid(nc * nqg);
#define LAUNCH_E(DD)                                                                                          \
  knn_exact_kernel<DD><<<grid, 256, 0, stream>>>((const bf16*)X.data_ptr(), N, (const bf16*)Q.data_ptr(),    \
                                                 Qn, (int)K, ws_s.data_ptr<float>(), ws_i.data_ptr<int32_t>(), \
                                                 ctrl, nchunks, 0, nc)
    DISPATCH_DIM(LAUNCH_E)
#undef LAUNCH_E
  };
  static const int q256_min = getenv("LS_KNN_Q256_MIN") ? atoi(getenv("LS_KNN_Q256_MIN")) : 128;
  const bool q256 = Qn >= q256_min && (dim == 128 || dim == 256 || dim == 384 || dim == 512);
  // MODE: 0 strict filter after an exact sample, 1 non-strict filter over the whole store,
  // 2 group-max sample pass (gmax = ws_s scratch, G groups per query)
  auto filter_q256 = [&](int mode, int64_t row_begin, int64_t rows, int64_t nrb_target, int64_t min_rpw,
                         int* G_out) {
    if (rows <= 0) return;
    const int nqb = (Qn + 255) / 256;
    int64_t rpw = (rows + nrb_target - 1) / nrb_target;
    rpw = std::max<int64_t>(min_rpw, (rpw + 63) / 64 * 64);
    const int nrb = (int)((rows + rpw - 1) / rpw);
    const int G = 16 * nrb;
    if (G_out) *G_out = G;
    // abl_req (knn_topk_ablate only -- diagnosis, wrong results): the main pass without
    // its sync (1), without sync and DMA (2), without MFMAs (3); MODE 1, 384 dims only.
    // The serving entry point (knn_topk) always passes 0.
    const int abl = mode == 1 && dim == 384 ? abl_req : 0;
    dim3 grid(nrb * nqb);
#define LAUNCH_Q(DD, MM)                                                                                         \
  launch_q256<DD, MM>(abl, grid, stream, (const bf16*)X.data_ptr(), N, (const bf16*)Q.data_ptr(), Qn,            \
                      ws_s.data_ptr<float>(), ws_i.data_ptr<int32_t>(), ctrl, cap, row_begin, (int)rpw, nqb, G)
#define LAUNCH_QM(DD)                     \
  switch (mode) {                         \
    case 0: LAUNCH_Q(DD, 0); break;       \
    case 1: LAUNCH_Q(DD, 1); break;       \
    default: LAUNCH_Q(DD, 2); break;      \
  }
    switch (dim) {
      case 128: LAUNCH_QM(128); break;
      case 256: LAUNCH_QM(256); break;
      case 384: LAUNCH_QM(384); break;
      case 512: LAUNCH_QM(512); break;
      default: break;
    }
#undef LAUNCH_QM
#undef LAUNCH_Q
  };
  auto filter = [&](int c0, int nc) {
    if (q256) {
      // ~1024 workgroups (4 per CU) over rows x query blocks, whole 64-row tiles per workgroup
      const int64_t row_begin = (int64_t)c0 * CH;
      filter_q256(0, row_begin, std::min<int64_t>(N, (int64_t)(c0 + nc) * CH) - row_begin,
                  std::max(1, 1024 / ((Qn + 255) / 256)), 256, nullptr);
      return;
    }
    dim3 grid(nc * nqf);
#define LAUNCH_F(DD)                                                                                            \
  knn_filter_kernel<DD><<<grid, 256, 0, stream>>>((const bf16*)X.data_ptr(), N, (const bf16*)Q.data_ptr(), Qn, \
                                                  ws_s.data_ptr<float>(), ws_i.data_ptr<int32_t>(), ctrl, cap, c0, \
                                                  nc)
    DISPATCH_DIM(LAUNCH_F)
#undef LAUNCH_F
  };
#undef DISPATCH_DIM
  auto select = [&](int write_thr) {
    knn_select_kernel<<<(Qn + 3) / 4, 256, 0, stream>>>(ws_s.data_ptr<float>(), ws_i.data_ptr<int32_t>(), ctrl, Qn,
                                                        cap, (int)K, out_s.data_ptr<float>(),
                                                        out_i.data_ptr<int32_t>(), write_thr);
  };
  const int ns = sample <= 0 ? nchunks : (int)std::min<int64_t>(nchunks, sample);
  // Large batches: the thresholds come from a group-max pass over the sample rows (an
  // MFMA pass with a running-max epilogue, ~10x cheaper than the exact per-chunk top-K
  // of the sample) and the filter then covers the whole store with scores >= thr.
  const int64_t S = (int64_t)ns * CH;
  if (q256 && ns < nchunks && K <= 64 && N >= 2 * S && !getenv("LS_KNN_EXACT_SAMPLE")) {
    const int nqb = (Qn + 255) / 256;
    const int64_t nrb_target = std::min<int64_t>(256, std::max<int64_t>(32, 256 / nqb));
    const int64_t rpw = std::max<int64_t>(64, ((S + nrb_target - 1) / nrb_target + 63) / 64 * 64);
    const int64_t G = 16 * ((S + rpw - 1) / rpw);
    if ((int64_t)Qn * G <= ws_s.numel()) {
      int Gk = 0;
      filter_q256(2, 0, S, nrb_target, 64, &Gk);
      knn_group_thr_kernel<<<(Qn + 3) / 4, 256, 0, stream>>>(ws_s.data_ptr<float>(), Gk, Qn, (int)K, ctrl);
      filter_q256(1, 0, N, std::max(1, 1024 / nqb), 256, nullptr);
      knn_select4_kernel<<<Qn, 256, 0, stream>>>(ws_s.data_ptr<float>(), ws_i.data_ptr<int32_t>(), ctrl, Qn, cap,
                                                 (int)K, out_s.data_ptr<float>(), out_i.data_ptr<int32_t>());
      return;
    }
  }
  exact(ns);
  if (ns < nchunks) {
    select(1);
    filter(ns, nchunks - ns);
  }
  select(0);
}
}  // namespace

void knn_topk(at::Tensor X, at::Tensor Q, int64_t K, at::Tensor out_s, at::Tensor out_i, at::Tensor ws_s,
              at::Tensor ws_i, int64_t sample) {
  knn_topk_impl(X, Q, K, out_s, out_i, ws_s, ws_i, sample, 0);
}

// Timing-only ablations of the large-batch main pass (tools/engine_bench.py --knn-ablate):
// the results are WRONG by design, so this is a separate entry point the serving path
// never calls (no environment switch on knn_topk).
void knn_topk_ablate(at::Tensor X, at::Tensor Q, int64_t K, at::Tensor out_s, at::Tensor out_i, at::Tensor ws_s,
                     at::Tensor ws_i, int64_t sample, int64_t abl) {
  TORCH_CHECK(abl >= 0 && abl <= 3, "knn_topk_ablate: abl 0..3");
  knn_topk_impl(X, Q, K, out_s, out_i, ws_s, ws_i, sample, (int)abl);
}

int64_t knn_default_sample() { return SAMPLE_CHUNKS; }
