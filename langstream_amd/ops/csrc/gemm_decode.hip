// Decode-step GEMM on MFMA for gfx950:  C[M, N] = X[M, K] . W[N, K]^T  with the whole
// decode batch (129 <= M <= 256 rows) in ONE 256-row workgroup tile.
//
// Replaces hipBLASLt on the Llama decode projections (qkv, o, gate_up + SwiGLU, down);
// the reference's inference call site is ChatCompletionsStep.java:132-155 (remote
// OpenAI / Ollama completions), which this engine serves locally.
//
// Why this shape of kernel.  At M = 256 a projection is neither HBM- nor MFMA-bound: it
// is bound by what each CU can pull through its load path (~60-70 GB/s per CU,
// MI355X_MICROARCH 'ring-gemm'), and every workgroup re-reads the activations X from L2.
// The chip-wide bytes a CU must ingest are  (1 + M / BN) x W  plus, with K split S ways,
// S x M x N x 4 of f32 partial sums.  So:
//   * all 256 rows in one tile (X re-read N / BN times, never W);
//   * BN = 128 or 256 output columns; split-K only as far as needed to put ~1 workgroup
//     on every CU (qkv/o/down), and for gate_up a 2-way split whose halves are combined
//     inside the launch (below) so SwiGLU stays in the epilogue;
//   * 64-deep K stages with 128-B LDS rows filled by LDS-DMA (global_load_lds_dwordx4):
//     one DMA instruction = 8 full 128-B lines (the 64-B rows of gemm_skinny.hip's ring
//     issue two requests per line: twice the TA traffic for the same bytes);
//   * separate rings: X (L2-resident, short latency) 2 slots, issued 1 stage ahead; W
//     (HBM, long latency) 3 slots, issued 2 stages ahead.  One raw s_barrier per stage
//     behind a counted vmcnt -- never __syncthreads() in the loop (it would drain the
//     DMAs in flight);
//   * bank swizzle on the SOURCE address (the DMA image is lane-linear): chunk p of LDS
//     row r holds global k-chunk p ^ ((r >> 1) & 7), conflict-free ds_read_b128 fragments;
//   * 8 waves as 4 (rows) x 2 (columns), 64 x BN/2 per wave, MFMA 16x16x32 bf16.
//
// gate_up (EPI_SILU2): tile = 128 gate + the matching 128 up rows of W, K split in two.
// The two halves of a tile sit on one XCD.  The first to finish (ticket parity of a
// monotonic per-tile counter, so no per-call reset) publishes its f32 accumulators
// (plain stores -> agent release -> flag), the second waits for the flag (the first is
// running: it already took its ticket, so no co-residency assumption), acquires, adds the
// partner's half to its own registers (f32 a + b == b + a: the result does not depend on
// which half came first) and writes silu(g) * u.  The wait is bounded; a timeout sets
// err[0] and the host checks it (ops.decode_gemm_error).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <atomic>
#include <string>
#include "common.h"

void splitk_reduce_launch(const float* part, int S, int M, int N, bf16* out, int64_t ldo, hipStream_t st);
void splitk_add_rmsnorm_launch(const float* part, int S, int M, int N, bf16* residual, const bf16* norm_w, float eps,
                               bf16* out, hipStream_t st);

namespace {

constexpr int BM = 256, BK = 64;
constexpr int XSTAGE = BM * BK * 2;    // 32 KB
constexpr int LDS_MAX = 160 * 1024;

// s_waitcnt vmcnt(n) for a run-time n (the instruction takes an immediate)
__device__ __forceinline__ void wait_vmcnt_dyn(int n) {
  switch (n) {
#define W_(k) case k: wait_vmcnt<k>(); break;
    W_(0) W_(1) W_(2) W_(3) W_(4) W_(5) W_(6) W_(7) W_(8) W_(9) W_(10) W_(11) W_(12) W_(13) W_(14) W_(15)
    W_(16) W_(17) W_(18) W_(19) W_(20) W_(21) W_(22) W_(23) W_(24) W_(25) W_(26) W_(27) W_(28) W_(29) W_(30)
#undef W_
    default: wait_vmcnt<0>(); break;
  }
}

enum { EPI_STORE = 0, EPI_PARTIAL = 1, EPI_SILU = 2, EPI_SILU2 = 3, EPI_CMB_RES = 4, EPI_CMB_QKV = 5,
       EPI_SILU_R = 6 };

// ---- the norm-deferred decode layer (TP = 1, 129..256 rows; LlamaRunner::forward_dgemm)
//
// RMSNorm needs whole rows, which is what forced a separate split-K reduce kernel (with
// its launch and its slab round trip) behind o / down.  Here the norm is split in two:
//   rmsnorm(h) . W^T = r_m * ((h * g) . W^T),   r_m = 1 / sqrt(mean_k h[m,k]^2 + eps)
// The producer's combine writes y = bf16(h * g) -- elementwise, no row dependency -- and
// per-(row, tile) partial sums of h^2; the consumer GEMM runs on y and multiplies its
// output rows by r_m (gate_up: in its SwiGLU epilogue; qkv: in its combine, before RoPE).
// With that, the split-K reduction of qkv / o / down happens INSIDE the GEMM launch:
// the S K-slices of a tile write their f32 partial tiles, meet at a per-tile counter
// (all tiles x S <= CUs workgroups are co-resident: one 160 KB-LDS workgroup per CU), and
// each slice then reduces 1/S of the tile's rows (cdna_hip_programming "Projection GEMM
// at M = 256", item 2: plain slab stores -> agent release -> counter; counter poll ->
// agent acquire -> plain loads).  Counters are 64-bit and monotonic per call site
// (never reset; a launch advances each of its tiles by exactly S).
struct DgArgs {
  unsigned long long* counters = nullptr;  // [tiles] per call site
  int* err = nullptr;                      // set when a rendezvous times out
  bf16* residual = nullptr;                // CMB_RES: h, updated in place (h += x . w^T)
  const bf16* norm_g = nullptr;            // CMB_RES: the next RMSNorm's weight [N]
  bf16* y_out = nullptr;                   // CMB_RES: bf16(h * g) [M, N]
  float* sumsq_out = nullptr;              // CMB_RES: [M][tiles] partial sums of h^2
  const float* sumsq_in = nullptr;         // CMB_QKV / SILU_R: the producer's partials [M][npart]
  int npart = 0;
  float eps = 1e-5f, inv_h = 0.f;          // inv_h = 1 / hidden size (the mean of h^2)
  const int32_t* pos = nullptr;            // CMB_QKV: RoPE + paged KV write
  const float* cos_sin = nullptr;
  int max_pos = 0;
  const int64_t* slots = nullptr;
  int64_t nslots = 0;
  bf16* kc = nullptr;
  bf16* vc = nullptr;
  int Hq = 0, Hkv = 0, BS = 0;
};

// 1 / rms of one row from its npart partial sums of squares.  The partials were written by
// the previous launch from every XCD, so each load is a MALL / cross-XCD round trip: the
// loads go out together as float4s (a dependent scalar loop cost ~1 us per partial).
__device__ __forceinline__ float rms_scale(const float* __restrict__ part, int npart, float inv_h, float eps) {
  float s = 0.f;
  int t = 0;
  if ((npart & 3) == 0 && (reinterpret_cast<uintptr_t>(part) & 15) == 0) {
    const float4* p4 = reinterpret_cast<const float4*>(part);
    const int n4 = npart >> 2;
    for (; t + 8 <= n4; t += 8) {
      float4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = p4[t + j];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    }
    for (; t < n4; ++t) {
      const float4 v = p4[t];
      s += (v.x + v.y) + (v.z + v.w);
    }
    t = npart;
  }
  for (; t < npart; ++t) s += part[t];
  return rsqrtf(s * inv_h + eps);
}

// 8-row x 128-B piece p of an image: lane l fills row 8p + (l >> 3), LDS chunk l & 7
// with global chunk (l & 7) ^ ((row >> 1) & 7).
__device__ __forceinline__ int piece_chunk(int lane, int row) { return ((lane & 7) ^ ((row >> 1) & 7)) * 8; }

// XS / WS: ring slots of X / W; stage t of X is issued XS-1 steps ahead, of W WS-1 ahead.
// ABL (timing-only ablations, wrong results; tools/dgemm_bench.py --ablate): bit 0 drops
// the MFMAs, bit 1 the fragment reads, bit 2 the LDS-DMA issue, bit 3 the W DMA only;
// bit 4 (a real variant, results valid) streams W with the non-temporal hint; bit 5 uses 4
// dedicated loader waves; bit 6 skips the partial-slab stores; bit 7 (a real variant)
// writes the partial slabs with non-temporal stores.
// LD: dedicated loader waves (0 or 4).  With LD = 4 the workgroup is 8 compute + 4
// loader waves: only the loaders issue LDS-DMA.  Measured (tools/dgemm_bench.py
// --ablate, profiles/dgemm_ablation_r3a.log, dgemm_ablation_r3b_loaders.log): with every wave issuing its share of the
// stage right after the barrier, a full DMA queue blocks the issuing wave before its
// MFMAs, so a step costs DMA + compute instead of max(DMA, compute).
template <int BN, int XS, int WS, int EPI, int ABL = 0, int LD = 0, int BMT = BM, int SPB = 1>
__global__ void __launch_bounds__(LD ? 768 : 512) dgemm_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                   const bf16* __restrict__ w, int M, int N, int K, int S,
                                                   bf16* __restrict__ out, int64_t ldo, float* __restrict__ part,
                                                   int F, unsigned* __restrict__ tickets, float* __restrict__ xchg,
                                                   int* __restrict__ err, int split_outer, DgArgs ga) {
  constexpr int WSTAGE = BN * BK * 2;
  // BMT: rows of the tile (256, or 128 / 64 for small batches: rows past M are zeros the
  // DMA still moves and the MFMAs still multiply, so a 64-row batch in a 256-row tile
  // pays the 256-row X stream).  8 compute waves as WM x WN, IT x 16 rows each.
  constexpr int IT = BMT == 64 ? 2 : 4;    // 16-row tiles per wave
  constexpr int WM = BMT / (16 * IT);      // wave rows
  constexpr int WN = 8 / WM;               // wave columns
  constexpr int XST = BMT * BK * 2;        // X stage bytes
  static_assert(BMT == 256 || BMT == 128 || BMT == 64, "tile rows");
  constexpr bool CMB = EPI == EPI_CMB_RES || EPI == EPI_CMB_QKV;
  static_assert(BMT == 256 || !(CMB || EPI == EPI_SILU2 || EPI == EPI_SILU_R), "fused paths: 256-row tiles");
  constexpr bool SILU_LIKE = EPI == EPI_SILU || EPI == EPI_SILU_R;
  static_assert(!(CMB || EPI == EPI_SILU_R) || (BN == 128 && LD == 4), "fused epilogues: BN 128 + loader waves");
  constexpr int JT = BN / (16 * WN);       // 16-col tiles per wave (wave = 16 IT rows x BN / WN cols)
  static_assert(JT >= 2 || !(EPI == EPI_SILU || EPI == EPI_SILU2 || EPI == EPI_SILU_R), "SwiGLU pairs");
  constexpr int NLW = LD ? LD : 8;         // waves that issue the DMAs
  constexpr int PX = BMT / 8 / NLW;        // X pieces per issuing wave per stage (BMT / 8 per stage)
  constexpr int PW = BN / 8 / NLW;         // W pieces per issuing wave per stage
  // SPB: 64-deep K stages per barrier.  At small M a stage is a few MFMAs per wave and the
  // barrier + LDS-read round trip per stage sets the rate; SPB = 2 halves the barriers
  // (the ring then keeps SPB stages being read, so XS - SPB / WS - SPB are issued ahead).
  constexpr int XA = XS - SPB, WA = WS - SPB;  // stages issued ahead
  static_assert(SPB == 1 || SPB == 2, "stages per barrier");
  static_assert(SPB == 1 || (ABL & ~(16 | 128)) == 0, "ablations: one stage per barrier");
  static_assert(XA >= 1 && WA >= XA, "W is issued at least as far ahead as X");
  static_assert(XS * XST + WS * WSTAGE <= LDS_MAX, "LDS budget");
  __shared__ __attribute__((aligned(1024))) char lds[XS * XST + WS * WSTAGE];
  char* const lx0 = lds;
  char* const lw0 = lds + XS * XST;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = LD == 0 || wid >= 8;   // issues DMAs (every wave when LD == 0)
  const bool computer = LD == 0 || wid < 8;
  const int lw = LD ? (wid >= 8 ? wid - 8 : 0) : wid;   // index among the issuing waves
  // the S splits of one tile are consecutive logical ids: same XCD (speed only)
  // split_outer: consecutive logical ids (one XCD) share the K split, i.e. the same X
  // slice, which then stays in that XCD's L2; otherwise the S splits of one tile are
  // adjacent (the gate_up exchange pairs sit on one XCD).
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = gridDim.x / S;
  const int tile = split_outer ? logical % ntiles : logical / S;
  const int split = split_outer ? logical / ntiles : logical - tile * S;
  const int nk = K / BK;
  const int kb = (int)(((int64_t)split * nk) / S), ke = (int)(((int64_t)(split + 1) * nk) / S);
  const int nks = ke - kb;

  // ---- LDS-DMA sources: buffer resources from this split's first K column (X rows at
  // or past M fall outside the X resource and read zeros; they are never stored).  X
  // pieces keep one per-lane byte offset each (the row decides the range check); a W
  // piece is 8 consecutive rows, so its row base and the K stage go in the scalar
  // offset and only two per-lane offsets remain (the swizzle depends on the piece's row
  // parity) -- 64-bit pointers per piece cost BN = 256 its third wave per SIMD.
  const i32x4 xrs = make_rsrc(x + (int64_t)kb * BK, (uint32_t)((((int64_t)(M - 1) * ldx + K) - (int64_t)kb * BK) * 2));
  const i32x4 wrs = make_rsrc(w + (int64_t)kb * BK, (uint32_t)(((int64_t)N * K - (int64_t)kb * BK) * 2));
  int xvo[PX];
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const int row = (8 * PX) * lw + 8 * j + (lane >> 3);
    xvo[j] = (row * (int)ldx + piece_chunk(lane, row)) * 2;
  }
  int wvo[2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
    wvo[p] = ((lane >> 3) * K + (((lane & 7) ^ ((4 * p + (lane >> 4)) & 7)) * 8)) * 2;
  auto wrow0 = [&](int j) -> uint32_t {   // first W row of piece j (uniform)
    const int lr = (8 * PW) * lw + 8 * j;
    if constexpr (EPI == EPI_SILU || EPI == EPI_SILU2 || EPI == EPI_SILU_R)
      return lr < BN / 2 ? tile * (BN / 2) + lr : F + tile * (BN / 2) + (lr - BN / 2);
    return tile * BN + lr;
  };
  const unsigned lxa = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lx0;
  const unsigned lwa = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lw0;
  auto issue_x = [&](int t) {
    const unsigned dst = lxa + (t % XS) * XST + (PX * lw) * 1024;
#pragma unroll
    for (int j = 0; j < PX; ++j) blds16<false>(xrs, xvo[j], t * BK * 2, dst + j * 1024);
  };
  auto issue_w = [&](int t) {
    const unsigned dst = lwa + (t % WS) * WSTAGE + (PW * lw) * 1024;
#pragma unroll
    for (int j = 0; j < PW; ++j)
      blds16<(ABL & 16) != 0>(wrs, wvo[(PW * lw + j) & 1], (int)(wrow0(j) * (uint32_t)K * 2u + (uint32_t)(t * BK * 2)),
                              dst + j * 1024);
  };

  // ---- fragments
  const int cw = computer ? wid : 0;       // loaders: any valid layout, never used
  const int wm = cw / WN, wn = cw % WN;
  const int fr = lane & 15, h = lane >> 4;
  const int fsw = (fr >> 1) & 7;           // = (row >> 1) & 7 of every fragment row
  auto bcol = [&](int j) {                 // tile-local W row of this lane's B fragment
    if constexpr (EPI == EPI_SILU || EPI == EPI_SILU2 || EPI == EPI_SILU_R)
      return (j < JT / 2 ? (BN / (2 * WN)) * wn + 16 * j : BN / 2 + (BN / (2 * WN)) * wn + 16 * (j - JT / 2)) + fr;
    return (BN / WN) * wn + 16 * j + fr;
  };
  int aoff[IT], boff[JT];
#pragma unroll
  for (int i = 0; i < IT; ++i) aoff[i] = (16 * IT * wm + 16 * i + fr) * 128;
#pragma unroll
  for (int j = 0; j < JT; ++j) boff[j] = bcol(j) * 128;

  f32x4 acc[IT][JT];
#pragma unroll
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Issue order: pseudo-steps u = -WA .. -1 (prologue), then steps u = 0 .. nks-1, each
  // issuing X(u + XA) then W(u + WA) (stages outside [0, nks) are skipped).  X(t) is
  // issued at step t - XA and W(t) at step t - WA <= t - XA, before it, so once X(t) has
  // landed so has W(t).  The DMAs issued AFTER X(t) are W(t - XA + WA) and, for the steps
  // in between, X(t+1 .. t+XA-1) and W(t+WA-XA+1 .. t+WA-1): at the top of step t the
  // wait is vmcnt(that count), computed exactly (the tail skips issues).
  auto issue_step = [&](int u) {
    if (!loader) return;
    if constexpr ((ABL & 4) == 0) {
      if (u + XA >= 0 && u + XA < nks) issue_x(u + XA);
      if constexpr ((ABL & 8) == 0)
        if (u + WA >= 0 && u + WA < nks) issue_w(u + WA);
    }
  };
  for (int u = -WA; u < 0; ++u) issue_step(u);
  for (int t = 0; t < nks; t += SPB) {
    if (loader) {
      if constexpr (SPB == 1) {
        const int nx = max(0, min(t + XA - 1, nks - 1) - t);                       // X(t+1 .. t+XA-1)
        const int nw = max(0, min(t + WA - 1, nks - 1) - (t - XA + WA) + 1);       // W(t-XA+WA .. t+WA-1)
        if constexpr ((ABL & 12) == 0) wait_vmcnt_dyn(PX * nx + PW * nw);
        else if constexpr ((ABL & 4) == 0) wait_vmcnt_dyn(PX * nx);
      } else {
        // stages t .. t+SPB-1 must have landed: the last of their DMAs is X(t+SPB-1),
        // issued by step u0; count what was issued after it (W(u0+WA), steps u0+1 .. t-1)
        const int u0 = t + SPB - 1 - XA;
        int cnt = (u0 + WA >= 0 && u0 + WA < nks) ? PW : 0;
        for (int u = u0 + 1; u < t; ++u)
          cnt += ((u + XA >= 0 && u + XA < nks) ? PX : 0) + ((u + WA >= 0 && u + WA < nks) ? PW : 0);
        wait_vmcnt_dyn(cnt);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous stages' fragment reads are done
    __builtin_amdgcn_s_barrier();                         // every wave: stages t.. landed, t-SPB.. read
#pragma unroll
    for (int sp = 0; sp < SPB; ++sp) issue_step(t + sp);  // into the slots of stages t-SPB ..
    if (!computer) continue;
#pragma unroll
    for (int sp = 0; sp < SPB; ++sp) {
    if (t + sp >= nks) break;
    const char* lx = lx0 + ((t + sp) % XS) * XST;
    const char* lw = lw0 + ((t + sp) % WS) * WSTAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int off = 16 * ((4 * ks + h) ^ fsw);
      bf16x8 a[IT], b[JT];
      if constexpr ((ABL & 2) == 0) {
#pragma unroll
        for (int j = 0; j < JT; ++j) b[j] = __builtin_bit_cast(bf16x8, ld16(lw + boff[j] + off));
#pragma unroll
        for (int i = 0; i < IT; ++i) a[i] = __builtin_bit_cast(bf16x8, ld16(lx + aoff[i] + off));
      } else {
#pragma unroll
        for (int j = 0; j < JT; ++j) b[j] = bf16x8{} + (bf16)(float)(t + ks + j);
#pragma unroll
        for (int i = 0; i < IT; ++i) a[i] = bf16x8{} + (bf16)(float)(t + i);
      }
      if constexpr ((ABL & 1) == 0) {
#pragma unroll
        for (int i = 0; i < IT; ++i)
#pragma unroll
          for (int j = 0; j < JT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < IT; ++i) asm volatile("" ::"v"(a[i]));
#pragma unroll
        for (int j = 0; j < JT; ++j) asm volatile("" ::"v"(b[j]));
      }
    }
    }
  }
  wait_vmcnt<0>();  // no LDS-DMA may outlive the workgroup

  // acc[i][j][r] = C[16 IT wm + 16i + 4h + r][tile col of bcol(j)]
  const int rbase = 16 * IT * wm + 4 * h;
  if constexpr (EPI == EPI_SILU2) {
    // ---- in-launch combine of the two K halves (see the header); with loader waves
    // (LD = 4) only the 512 compute threads hold accumulators, the loaders only join
    // the workgroup barriers
    __syncthreads();                                      // ring reads done: LDS reusable
    unsigned* sh = reinterpret_cast<unsigned*>(lds);
    if (threadIdx.x == 0) sh[0] = __hip_atomic_fetch_add(&tickets[2 * tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned tk = sh[0];
    const unsigned gen = tk / 2 + 1;                      // this call's generation for the tile
    float* xb = xchg + (int64_t)tile * (BM * BN);
    if ((tk & 1u) == 0) {
      // first half: publish the accumulators in a thread-linear, coalesced layout
      if (computer) {
#pragma unroll
        for (int i = 0; i < IT; ++i)
#pragma unroll
          for (int j = 0; j < JT; ++j)
            *reinterpret_cast<f32x4*>(xb + ((int64_t)(i * JT + j) * 512 + threadIdx.x) * 4) = acc[i][j];
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&tickets[2 * tile + 1], gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (threadIdx.x == 0) {
      int spins = 0;
      while (__hip_atomic_load(&tickets[2 * tile + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1 << 22)) {   // ~0.5 s: the partner never published -- flag it, never hang
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (!computer) return;
    // combine + SwiGLU + store one 16-row tile at a time (bounded live registers)
#pragma unroll
    for (int i = 0; i < IT; ++i) {
#pragma unroll
      for (int j = 0; j < JT / 2; ++j) {
        // gate column j and its up column j + JT/2, one pair at a time (bounded registers)
        const f32x4 g = acc[i][j] + *reinterpret_cast<const f32x4*>(xb + ((int64_t)(i * JT + j) * 512 + threadIdx.x) * 4);
        const f32x4 u = acc[i][j + JT / 2] +
                        *reinterpret_cast<const f32x4*>(xb + ((int64_t)(i * JT + j + JT / 2) * 512 + threadIdx.x) * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rbase + 16 * i + r;
          if (m < M)
            out[(int64_t)m * ldo + tile * (BN / 2) + (BN / (2 * WN)) * wn + fr + 16 * j] =
                (bf16)(g[r] / (1.f + __expf(-g[r])) * u[r]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    return;
  }
  // ---- LDS-staged epilogue: the tile goes through LDS as f32 rows of BN + 4 (the ring
  // is dead now) and leaves in whole rows with 16-B stores -- every store instruction
  // writes full 128-B lines instead of 4 x 64-B row pieces per wave.  BN = 128 stages all
  // 256 rows at once (132 KB); BN = 256 in two passes of 128 rows.
  // CMB_QKV: this thread's row scale, fetched now so its latency hides behind the slab
  // stores and the rendezvous (nr <= NT rows per slice: thread i takes row rr0 + i)
  float r_pre = 1.f;
  if constexpr (EPI == EPI_CMB_QKV) {
    const int R = (M + S - 1) / S, rr0 = split * R;
    if ((int)threadIdx.x < min(R, M - rr0))
      r_pre = rms_scale(ga.sumsq_in + (int64_t)(rr0 + threadIdx.x) * ga.npart, ga.npart, ga.inv_h, ga.eps);
  }
  constexpr int TP = BN + 4;
  constexpr int PASS_ROWS = BMT * TP * 4 <= XS * XST + WS * WSTAGE ? BMT : BMT / 2;
  static_assert(PASS_ROWS * TP * 4 <= XS * XST + WS * WSTAGE, "epilogue pass must fit the ring's LDS");
  constexpr int NT = LD ? 768 : 512;
  float* T = reinterpret_cast<float*>(lds);
  // SILU_R: the row scales 1/rms(h) after T (LDS past 256 x 132 floats is free)
  float* rbuf = reinterpret_cast<float*>(lds + PASS_ROWS * TP * 4);
  if constexpr (EPI == EPI_SILU_R) static_assert(PASS_ROWS == BMT && BMT * TP * 4 + BMT * 4 <= LDS_MAX, "r buffer");
#pragma unroll
  for (int r0 = 0; r0 < BMT; r0 += PASS_ROWS) {
    __syncthreads();                                    // ring reads / the previous pass are done
    if (computer && 16 * IT * wm >= r0 && 16 * IT * wm < r0 + PASS_ROWS) {
#pragma unroll
      for (int i = 0; i < IT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* trow = T + (rbase + 16 * i + r - r0) * TP;
#pragma unroll
          for (int j = 0; j < JT; ++j) trow[bcol(j)] = acc[i][j][r];
        }
    }
    if constexpr (EPI == EPI_SILU_R) {
      // the loader waves (idle now) reduce the producer's per-tile partial sums of h^2
      // while the compute waves stage the tile
      if (!computer) {
        const int m = threadIdx.x - 512;
        if (m < M) rbuf[m] = rms_scale(ga.sumsq_in + (int64_t)m * ga.npart, ga.npart, ga.inv_h, ga.eps);
      }
    }
    __syncthreads();
    const int rows = min(PASS_ROWS, M - r0);
    if constexpr (CMB) {
      // slab stores WRITE-THROUGH (sc1): the K slices of this tile read them in this launch,
      // and a plain store would need an agent release fence that writes back every dirty
      // L2 line of the XCD (128 KB per workgroup here) -- MI355X_MICROARCH publish-large
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
          part, 0, (int)((int64_t)S * M * N * 4), 0x00020000);
      for (int q = threadIdx.x; q < rows * (BN / 4); q += NT) {
        const int m = q / (BN / 4), c = (q - m * (BN / 4)) * 4;
        const int off = (int)((((int64_t)split * M + r0 + m) * N + tile * BN + c) * 4);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, *reinterpret_cast<const f32x4*>(T + m * TP + c)),
                                               prs, off, 0, 16);
      }
    } else if constexpr (EPI == EPI_PARTIAL) {
      // part[split][m][tile * BN + c]: BN / 4 float4 per row
      for (int q = threadIdx.x; q < ((ABL & 64) ? 0 : rows * (BN / 4)); q += NT) {
        const int m = q / (BN / 4), c = (q - m * (BN / 4)) * 4;
        f32x4* dst = reinterpret_cast<f32x4*>(part + ((int64_t)split * M + r0 + m) * N + tile * BN + c);
        const f32x4 v = *reinterpret_cast<const f32x4*>(T + m * TP + c);
        if constexpr ((ABL & 128) != 0) __builtin_nontemporal_store(v, dst);
        else *dst = v;
      }
    } else if constexpr (EPI == EPI_STORE) {
      for (int q = threadIdx.x; q < rows * (BN / 8); q += NT) {
        const int m = q / (BN / 8), c = (q - m * (BN / 8)) * 8;
        const float* src = T + m * TP + c;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = src[e];
        st16(out + (int64_t)(r0 + m) * ldo + tile * BN + c, pack8(v));
      }
    } else {
      // EPI_SILU(_R): tile columns [0, BN/2) are gate, [BN/2, BN) the matching up columns
      for (int q = threadIdx.x; q < rows * (BN / 16); q += NT) {
        const int m = q / (BN / 16), c = (q - m * (BN / 16)) * 8;
        const float* g = T + m * TP + c;
        const float rs = EPI == EPI_SILU_R ? rbuf[r0 + m] : 1.f;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gg = g[e] * rs, uu = g[BN / 2 + e] * rs;
          v[e] = gg / (1.f + __expf(-gg)) * uu;
        }
        st16(out + (int64_t)(r0 + m) * ldo + tile * (BN / 2) + c, pack8(v));
      }
    }
  }
  if constexpr (CMB) {
    // ---- rendezvous of the tile's S slices: publish this slab, wait for the others
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's slab stores are done
    __syncthreads();
    if (threadIdx.x == 0) {
      // every storing wave drained its sc1 stores before the barrier above: no release
      unsigned long long* cnt = ga.counters + tile;
      const unsigned long long old = __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long target = old - old % (unsigned long long)S + (unsigned long long)S;
      int spins = 0;
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 23)) {   // ~1 s: a slice never arrived -- flag it, never hang
          __hip_atomic_store(ga.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // ---- this slice reduces rows [rr0, rr0 + nr) of the tile over the S slabs
    const int R = (M + S - 1) / S;
    const int rr0 = split * R, nr = min(R, M - rr0);
    if (nr <= 0) return;
    const int64_t MN = (int64_t)M * N;
    if constexpr (EPI == EPI_CMB_RES) {
      // h += sum; residual <- bf16(h); y <- bf16(bf16(h) * g); sumsq[m][tile] = sum_c h^2.
      // Thread = 8 consecutive columns of one row; the 16 threads of a row are 16
      // consecutive lanes of one wave (NT and 16 | 64), reduced with width-16 shuffles.
      const int ntiles = N / BN;
      for (int q = threadIdx.x; q < nr * (BN / 8); q += NT) {
        const int m = rr0 + q / (BN / 8), c = tile * BN + (q % (BN / 8)) * 8;
        const float* p = part + (int64_t)m * N + c;
        f32x4 a0 = *reinterpret_cast<const f32x4*>(p), a1 = *reinterpret_cast<const f32x4*>(p + 4);
        for (int s = 1; s < S; ++s) {
          a0 += *reinterpret_cast<const f32x4*>(p + s * MN);
          a1 += *reinterpret_cast<const f32x4*>(p + s * MN + 4);
        }
        bf16* rp = ga.residual + (int64_t)m * N + c;
        float h[8], y[8], g[8];
        unpack8(ld16(rp), h);
        unpack8(ld16(ga.norm_g + c), g);
        float ss = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float hv = (float)(bf16)(h[e] + (e < 4 ? a0[e] : a1[e - 4]));   // the bf16 residual stream
          h[e] = hv;
          y[e] = hv * g[e];
          ss += hv * hv;
        }
        st16(rp, pack8(h));
        st16(ga.y_out + (int64_t)m * N + c, pack8(y));
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 16);
        if ((q & 15) == 0) ga.sumsq_out[(int64_t)m * ntiles + tile] = ss;
      }
    } else {
      // qkv: the tile is one head (BN = D = 128).  Row scale r_m from the producer's
      // partials, then RoPE on q / k heads, the paged K / V write for k / v heads.
      constexpr int D = 128, HALF = 64, G4 = 16;
      float* rrow = reinterpret_cast<float*>(lds);   // LDS is free after the slab stores
      if (threadIdx.x < nr) rrow[threadIdx.x] = r_pre;
      __syncthreads();
      const int hd = tile;
      for (int q = threadIdx.x; q < nr * G4; q += NT) {
        const int i = q / G4, c4 = q % G4, m = rr0 + i;
        const int64_t e0 = (int64_t)m * N + (int64_t)hd * D + 4 * c4;
        f32x4 lo = *reinterpret_cast<const f32x4*>(part + e0), hi = *reinterpret_cast<const f32x4*>(part + e0 + HALF);
        for (int s = 1; s < S; ++s) {
          lo += *reinterpret_cast<const f32x4*>(part + s * MN + e0);
          hi += *reinterpret_cast<const f32x4*>(part + s * MN + e0 + HALF);
        }
        const float rs = rrow[i];
        float a[4], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = lo[j] * rs;
          b[j] = hi[j] * rs;
        }
        if (hd < ga.Hq + ga.Hkv) {
          const int pp = min(max(ga.pos[m], 0), ga.max_pos - 1);
          const float4 co = *reinterpret_cast<const float4*>(ga.cos_sin + (int64_t)pp * D + 4 * c4);
          const float4 si = *reinterpret_cast<const float4*>(ga.cos_sin + (int64_t)pp * D + HALF + 4 * c4);
          const float cv[4] = {co.x, co.y, co.z, co.w}, sv[4] = {si.x, si.y, si.z, si.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float x1 = a[j], x2 = b[j];
            a[j] = x1 * cv[j] - x2 * sv[j];
            b[j] = x2 * cv[j] + x1 * sv[j];
          }
        }
        const bf16x4 va = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
        const bf16x4 vb = {(bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
        bf16* orow = out + (int64_t)m * ldo + (int64_t)hd * D + 4 * c4;
        *reinterpret_cast<bf16x4*>(orow) = va;
        *reinterpret_cast<bf16x4*>(orow + HALF) = vb;
        if (hd < ga.Hq) continue;
        const int64_t sl = ga.slots[m];
        if (sl < 0 || sl >= ga.nslots) continue;
        const int64_t blk = sl / ga.BS, off = sl - blk * ga.BS;
        if (hd < ga.Hq + ga.Hkv) {
          bf16* kd = ga.kc + ((blk * ga.Hkv + (hd - ga.Hq)) * ga.BS + off) * D + 4 * c4;
          *reinterpret_cast<bf16x4*>(kd) = va;
          *reinterpret_cast<bf16x4*>(kd + HALF) = vb;
        } else {
          bf16* vd = ga.vc + ((blk * ga.Hkv + (hd - ga.Hq - ga.Hkv)) * (int64_t)D) * ga.BS;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            vd[vt_off(4 * c4 + j, (int)off, D)] = va[j];
            vd[vt_off(HALF + 4 * c4 + j, (int)off, D)] = vb[j];
          }
        }
      }
    }
  }
}

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}

// Splits so that tiles x S covers the chip about once (<= 256 + 8 workgroups, one per
// CU) with at least `min_steps` 64-deep stages per split.
int pick_split(int tiles, int K, int min_steps) {
  const int nk = K / BK;
  int best = 1;
  for (int s = 1; s <= 64; ++s) {
    if (tiles * s > 264 || nk / s < min_steps) break;
    best = s;
  }
  return best;
}

int split_outer_default() {
  static const int v = env_int("LS_DGEMM_SPLIT_OUTER", 1);
  return v;
}

// Cache policy of the decode GEMMs in an engine step (profiles/nt_r3c/, full RAG bench,
// per-layer kernel times): W loads non-temporal (LS_DGEMM_WNT, gate_up 66.5 -> 64.5 us)
// and the f32 split-K slabs stored non-temporally (LS_DGEMM_NTST); with the attention's
// nt KV loads the layer drops 256.8 -> 240.6 us.  Both default on; read per launch.
// LS_DGEMM_WNT = 2: nt only for weights past 64 MB (gate_up / down); qkv and o measured
// faster with cached weight loads in isolation (M = 256, weights cold: 27.3 vs 28.8 and
// 23.8 vs 26.5 us, profiles/r5/dgemm_cold_hot_r5q.log).
int wnt_default(int64_t wbytes) {
  const int v = env_int("LS_DGEMM_WNT", 1);
  return v == 2 ? wbytes > (int64_t(64) << 20) : v;
}
int ntst_default() { return env_int("LS_DGEMM_NTST", 1); }

// Host-side launch census per (BN, epilogue, tile rows, K splits): the tests read it to
// prove which kernel variant a shape was routed to (decode_gemm_launch_counts).
// Relaxed atomics on the host only; one increment per launch.
constexpr int kCensusBn = 3, kCensusEpi = 7, kCensusBm = 3, kCensusS = 17;
std::atomic<int64_t> g_census[kCensusBn][kCensusEpi][kCensusBm][kCensusS];
constexpr int census_bn(int bn) { return bn == 64 ? 0 : bn == 128 ? 1 : 2; }
constexpr int census_bm(int bm) { return bm == 64 ? 0 : bm == 128 ? 1 : 2; }

// ring shapes: BN = 128: X 3 slots (2 ahead) + W 4 slots (3 ahead) = 160 KB;
// BN = 256: X 2 + W 3 = 160 KB.
template <int BN, int EPI, int BMT>
void dgemm_launch_bm(int S, int tiles, hipStream_t st, const at::Tensor& x, const at::Tensor& w, int M, int N, int K,
                     bf16* out, int64_t ldo, float* part, int F, unsigned* tickets, float* xchg, int* err,
                     const DgArgs& ga) {
  g_census[census_bn(BN)][EPI][census_bm(BMT)][std::min(S, kCensusS - 1)].fetch_add(1, std::memory_order_relaxed);
  // small tiles: two stages per barrier and the LDS they leave as a deeper W ring (8 / 6
  // slots at 64 / 128 rows: 96 / 64 KB of weights issued ahead)
  constexpr int SPB = BMT == BM ? 1 : 2;
  // BN = 64 (256-row tiles only): 8 KB W stages, so the W ring runs 5 stages ahead
  constexpr int XS = BN == 256 ? 2 : BMT == BM ? 3 : 4;
  constexpr int WS = BN == 256 ? 3 : BN == 64 ? 6 : BMT == 64 ? 8 : BMT == 128 ? 6 : 4;
  // BN = 256: 8 compute waves need 128 accumulator VGPRs each, no room for a third wave
  // per SIMD.  (Streaming the B fragments one at a time fits 168 VGPRs with 4 loader
  // waves, but the gate_up K-half exchange form then measured 90 vs 82 us:
  // profiles/dgemm_r3c/silu2_loaders.log.)
  constexpr int LDW = BN <= 128 ? 4 : 0;
  // the gate_up exchange pairs and the in-launch combine slices of a tile sit on one XCD
  const int so = (EPI == EPI_SILU2 || EPI == EPI_CMB_RES || EPI == EPI_CMB_QKV) ? 0 : split_outer_default();
  // cache-policy variants (ABL bits 4 and 7, real variants): weights streamed with the
  // non-temporal hint -- 16 GB of weights per decode step have no reuse and should not
  // evict the activations and the split-K workspace -- and / or the f32 partial slabs
  // written non-temporally, so they do not sit dirty in L2 for the kernel-end write-back
  const int pol = LDW == 4 ? (wnt_default(w.numel() * 2) ? 16 : 0) | (ntst_default() ? 128 : 0) : 0;
#define POL_(A)                                                                                                  \
  case A:                                                                                                        \
    dgemm_kernel<BN, XS, WS, EPI, A, LDW, BMT, SPB><<<dim3(tiles * S), 768, 0, st>>>(                                 \
        (const bf16*)x.data_ptr(), x.stride(0), (const bf16*)w.data_ptr(), M, N, K, S, out, ldo, part, F, tickets, \
        xchg, err, so, ga);                                                                                      \
    return;
  if constexpr (BMT == BM) {
    switch (pol) { POL_(16) POL_(128) POL_(144) default: break; }
  } else {
    switch (pol) { POL_(144) default: break; }
  }
#undef POL_
  dgemm_kernel<BN, XS, WS, EPI, 0, LDW, BMT, SPB><<<dim3(tiles * S), LDW ? 768 : 512, 0, st>>>(
      (const bf16*)x.data_ptr(), x.stride(0), (const bf16*)w.data_ptr(), M, N, K, S, out, ldo, part, F, tickets, xchg,
      err, so, ga);
}

// Tile rows by batch: 64- and 128-row tiles for M <= 64 / <= 128 (BN = 128, plain /
// split-K / SwiGLU epilogues; LS_DGEMM_SMALL_BM=0 keeps every batch on 256-row tiles).
int small_bm_default() { return env_int("LS_DGEMM_SMALL_BM", 1); }

template <int BN, int EPI>
void dgemm_launch(int S, int tiles, hipStream_t st, const at::Tensor& x, const at::Tensor& w, int M, int N, int K,
                  bf16* out, int64_t ldo, float* part, int F, unsigned* tickets, float* xchg, int* err,
                  DgArgs ga = DgArgs()) {
  if constexpr (BN == 128 && (EPI == EPI_STORE || EPI == EPI_PARTIAL || EPI == EPI_SILU)) {
    if (small_bm_default()) {
      if (M <= 64) {
        dgemm_launch_bm<BN, EPI, 64>(S, tiles, st, x, w, M, N, K, out, ldo, part, F, tickets, xchg, err, ga);
        return;
      }
      if (M <= 128) {
        dgemm_launch_bm<BN, EPI, 128>(S, tiles, st, x, w, M, N, K, out, ldo, part, F, tickets, xchg, err, ga);
        return;
      }
    }
  }
  dgemm_launch_bm<BN, EPI, BM>(S, tiles, st, x, w, M, N, K, out, ldo, part, F, tickets, xchg, err, ga);
}

void check_xw(const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "decode_gemm: bf16 GPU tensors");
  TORCH_CHECK(x.device() == w.device(), "decode_gemm: tensors on different devices");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x must be [M, K] with unit column stride");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) == x.size(1), "w must be contiguous [N, K]");
  TORCH_CHECK(x.size(1) % BK == 0, "K must be a multiple of 64");
  TORCH_CHECK(x.size(0) >= 1 && x.size(0) <= BM, "decode_gemm: 1 <= M <= 256");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0,
              "decode_gemm: x and w must be 16-byte aligned (LDS-DMA rows)");
}

int pick_bn(int N) {
  static const int env = env_int("LS_DGEMM_BN", 0);
  if (env == 64 || env == 128 || env == 256) return N % env == 0 ? env : 128;
  return 128;
}

}  // namespace

// The launch census since the last reset: {"bn128_partial_bm64_s3": n, ...}.
pybind11::dict decode_gemm_launch_counts(bool reset) {
  static const char* epi_names[kCensusEpi] = {"store", "partial", "silu", "silu2", "cmb_res", "cmb_qkv", "silu_r"};
  static const int bns[kCensusBn] = {64, 128, 256}, bms[kCensusBm] = {64, 128, 256};
  pybind11::dict d;
  for (int a = 0; a < kCensusBn; ++a)
    for (int e = 0; e < kCensusEpi; ++e)
      for (int b = 0; b < kCensusBm; ++b)
        for (int s = 0; s < kCensusS; ++s) {
          const int64_t n = reset ? g_census[a][e][b][s].exchange(0) : g_census[a][e][b][s].load();
          if (n == 0) continue;
          const std::string key = "bn" + std::to_string(bns[a]) + "_" + epi_names[e] + "_bm" + std::to_string(bms[b]) +
                                  "_s" + std::to_string(s);
          d[pybind11::str(key)] = n;
        }
  return d;
}

// Shapes: K % 64 == 0, N % 128 == 0; silu: the fused [2F, K] gate_up weight, F % 128 == 0.
bool decode_gemm_supported(const at::Tensor& w, bool silu) {
  if (w.dim() != 2 || w.scalar_type() != at::kBFloat16 || !w.is_contiguous() || w.size(1) % BK != 0) return false;
  return silu ? (w.size(0) % 256 == 0) : (w.size(0) % 128 == 0);
}

// Workspace bytes a decode_gemm call needs (f32 partials / exchange) -- callers that
// capture graphs allocate it once.
int64_t decode_gemm_workspace(int64_t M, int64_t N, int64_t K, bool silu) {
  if (silu) return (N / 256) * (int64_t)BM * 256 * 4;
  const int bn = pick_bn((int)N);
  const int S = pick_split((int)(N / bn), (int)K, 4);
  return S > 1 ? (int64_t)S * M * N * 4 : 0;
}

// out[M, N] = x . w^T  (mode 0), or with the split-K reduction fused with
// residual += x . w^T; out = rmsnorm(residual) * norm_w  (mode 1).
// bn / splits: 0 = automatic (tests and tools/dgemm_bench.py force them).
void decode_gemm(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor workspace, c10::optional<at::Tensor> residual,
                 c10::optional<at::Tensor> norm_w, double eps, int64_t bn_force, int64_t splits_force) {
  check_xw(x, w);
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(N % 128 == 0, "decode_gemm: N % 128 == 0");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.size(0) == M && out.size(1) == N && out.stride(1) == 1);
  const bool norm = residual.has_value();
  TORCH_CHECK(!norm || (norm_w.has_value() && residual->is_contiguous() && residual->numel() == (int64_t)M * N &&
                        out.is_contiguous() && norm_w->numel() == N), "decode_gemm: residual/norm shapes");
  int bn = (bn_force == 64 || bn_force == 128 || bn_force == 256) && N % bn_force == 0 ? (int)bn_force : pick_bn(N);
  // o-shaped projections with the residual + RMSNorm reduction (K <= 4096): 64-column
  // tiles, half the K splits (4 instead of 8) and half the f32 slab bytes the reduction
  // reads -- 27.1 vs 31.4 us at M = 256 including the reduction (profiles/dgemm_bn64_r4r.log);
  // qkv and down stay on 128 (29.8 vs 32.9, 45.3 vs 51.8)
  static const int o_bn64 = env_int("LS_DGEMM_O_BN64", 1);
  if (bn_force == 0 && o_bn64 && norm && K <= 4096 && N % 64 == 0 && M > 128) bn = 64;
  const int tiles = N / bn;
  const int S = splits_force > 0 ? (int)std::min<int64_t>(splits_force, K / BK) : pick_split(tiles, K, 4);
  auto st = at::hip::getCurrentHIPStream();
  if (S == 1 && !norm) {
    if (bn == 256)
      dgemm_launch<256, EPI_STORE>(1, tiles, st, x, w, M, N, K, (bf16*)out.data_ptr(), out.stride(0), nullptr, 0,
                                   nullptr, nullptr, nullptr);
    else if (bn == 64)
      dgemm_launch<64, EPI_STORE>(1, tiles, st, x, w, M, N, K, (bf16*)out.data_ptr(), out.stride(0), nullptr, 0,
                                  nullptr, nullptr, nullptr);
    else
      dgemm_launch<128, EPI_STORE>(1, tiles, st, x, w, M, N, K, (bf16*)out.data_ptr(), out.stride(0), nullptr, 0,
                                   nullptr, nullptr, nullptr);
    return;
  }
  TORCH_CHECK(workspace.scalar_type() == at::kFloat && workspace.is_cuda() &&
              workspace.numel() >= (int64_t)S * M * N, "decode_gemm: workspace too small");
  float* part = workspace.data_ptr<float>();
  if (bn == 256)
    dgemm_launch<256, EPI_PARTIAL>(S, tiles, st, x, w, M, N, K, nullptr, 0, part, 0, nullptr, nullptr, nullptr);
  else if (bn == 64)
    dgemm_launch<64, EPI_PARTIAL>(S, tiles, st, x, w, M, N, K, nullptr, 0, part, 0, nullptr, nullptr, nullptr);
  else
    dgemm_launch<128, EPI_PARTIAL>(S, tiles, st, x, w, M, N, K, nullptr, 0, part, 0, nullptr, nullptr, nullptr);
  if (norm)
    splitk_add_rmsnorm_launch(part, S, M, N, (bf16*)residual->data_ptr(), (const bf16*)norm_w->data_ptr(), (float)eps,
                              (bf16*)out.data_ptr(), st);
  else
    splitk_reduce_launch(part, S, M, N, (bf16*)out.data_ptr(), out.stride(0), st);
}

// ---------------------------------------------------------------------------------
// qkv projection of a decode-only step: the split-K reduction fused with RoPE and the
// paged KV-cache write.  One thread per (row m, head hd, 4-dim group c < D/8): it sums
// the S partial slabs of dims 4c..4c+3 and D/2+4c..+3 (the RoPE pairs), rotates q and k
// heads in f32 (cos / sin of position pos[m]), stores the bf16 row, and for k / v heads
// writes the paged cache (K rows, V transposed: see rope.hip).  This replaces the plain
// split-K reduce + the separate RoPE/cache pass (the attention then runs its un-fused
// form: the fused-RoPE attention measured 91.6 vs 80.4 us at B = 256, ctx 410,
// profiles/decode_attn_rope_isolated_r3.log).
template <int D>
__global__ void __launch_bounds__(256) splitk_reduce_rope_kernel(
    const float* __restrict__ part, int S, int M, int N, bf16* __restrict__ out, int64_t ldo,
    const int32_t* __restrict__ pos, const float* __restrict__ cos_sin, int max_pos,
    const int64_t* __restrict__ slots, int64_t nslots, bf16* __restrict__ kc, bf16* __restrict__ vc, int Hq, int Hkv,
    int BS) {
  constexpr int HALF = D / 2, G4 = HALF / 4;
  const int H = Hq + 2 * Hkv;
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (tid >= (int64_t)M * H * G4) return;
  const int c = (int)(tid % G4);
  const int64_t rest = tid / G4;
  const int hd = (int)(rest % H);
  const int m = (int)(rest / H);
  const int64_t MN = (int64_t)M * N;
  const int64_t e0 = (int64_t)m * N + (int64_t)hd * D + 4 * c;
  constexpr int SMAX = 8;
  float4 lo[SMAX], hi[SMAX];
#pragma unroll
  for (int s = 0; s < SMAX; ++s)
    if (s < S) {
      lo[s] = *reinterpret_cast<const float4*>(part + s * MN + e0);
      hi[s] = *reinterpret_cast<const float4*>(part + s * MN + e0 + HALF);
    }
  float a[4] = {lo[0].x, lo[0].y, lo[0].z, lo[0].w}, b[4] = {hi[0].x, hi[0].y, hi[0].z, hi[0].w};
#pragma unroll
  for (int s = 1; s < SMAX; ++s)
    if (s < S) {
      a[0] += lo[s].x; a[1] += lo[s].y; a[2] += lo[s].z; a[3] += lo[s].w;
      b[0] += hi[s].x; b[1] += hi[s].y; b[2] += hi[s].z; b[3] += hi[s].w;
    }
  for (int s = SMAX; s < S; ++s) {
    const float4 x = *reinterpret_cast<const float4*>(part + s * MN + e0);
    const float4 y = *reinterpret_cast<const float4*>(part + s * MN + e0 + HALF);
    a[0] += x.x; a[1] += x.y; a[2] += x.z; a[3] += x.w;
    b[0] += y.x; b[1] += y.y; b[2] += y.z; b[3] += y.w;
  }
  if (hd < Hq + Hkv) {
    const int p = min(max(pos[m], 0), max_pos - 1);
    const float4 co = *reinterpret_cast<const float4*>(cos_sin + (int64_t)p * D + 4 * c);
    const float4 si = *reinterpret_cast<const float4*>(cos_sin + (int64_t)p * D + HALF + 4 * c);
    const float cv[4] = {co.x, co.y, co.z, co.w}, sv[4] = {si.x, si.y, si.z, si.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x1 = a[j], x2 = b[j];
      a[j] = x1 * cv[j] - x2 * sv[j];
      b[j] = x2 * cv[j] + x1 * sv[j];
    }
  }
  const bf16x4 va = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
  const bf16x4 vb = {(bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
  bf16* orow = out + (int64_t)m * ldo + (int64_t)hd * D + 4 * c;
  *reinterpret_cast<bf16x4*>(orow) = va;
  *reinterpret_cast<bf16x4*>(orow + HALF) = vb;
  if (hd < Hq) return;
  const int64_t sl = slots[m];
  if (sl < 0 || sl >= nslots) return;
  const int64_t blk = sl / BS, off = sl - blk * BS;
  if (hd < Hq + Hkv) {
    bf16* kd = kc + ((blk * Hkv + (hd - Hq)) * BS + off) * D + 4 * c;
    *reinterpret_cast<bf16x4*>(kd) = va;
    *reinterpret_cast<bf16x4*>(kd + HALF) = vb;
  } else {
    bf16* vd = vc + ((blk * Hkv + (hd - Hq - Hkv)) * (int64_t)D) * BS;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vd[vt_off(4 * c + j, (int)off, D)] = va[j];
      vd[vt_off(HALF + 4 * c + j, (int)off, D)] = vb[j];
    }
  }
}

void rope_and_cache(at::Tensor qkv, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots, at::Tensor k_cache,
                    at::Tensor v_cache, int64_t Hq, int64_t Hkv, bool apply_rope);

// qkv[M, (Hq + 2 Hkv) D] = RoPE(x . w^T) for q and k heads, with the step's K / V rows
// written to the paged cache (the same contract as decode_gemm + rope_and_cache).
void decode_gemm_qkv_rope(at::Tensor qkv, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor pos,
                          at::Tensor cos_sin, at::Tensor slots, at::Tensor k_cache, at::Tensor v_cache, int64_t Hq,
                          int64_t Hkv) {
  check_xw(x, w);
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  const int D = (int)k_cache.size(3), BSZ = (int)k_cache.size(2);
  TORCH_CHECK(N == (Hq + 2 * Hkv) * D && N % 128 == 0, "decode_gemm_qkv_rope: qkv width");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && qkv.size(0) == M && qkv.size(1) == N && qkv.stride(1) == 1);
  TORCH_CHECK(pos.scalar_type() == at::kInt && pos.numel() >= M && slots.scalar_type() == at::kLong &&
              slots.numel() >= M && cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
              cos_sin.size(1) == D, "decode_gemm_qkv_rope: pos / slots / cos_sin");
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous() && v_cache.dim() == 5 && v_cache.size(2) == BSZ / 8 &&
              v_cache.size(3) == D && v_cache.size(4) == 8, "decode_gemm_qkv_rope: v_cache [NB, Hkv, BS/8, D, 8]");
  const int bn = pick_bn(N), tiles = N / bn;
  // at most 4 K slices: the fused reduction reads every slab once more (qkv at M = 256:
  // 27.5 us with 4 slices vs 28.1 with the 5 pick_split chooses, profiles/dgemm_bench_r3b.log)
  const int S = std::min(4, pick_split(tiles, K, 4));
  if (S == 1 || D != 128) {
    decode_gemm(qkv, x, w, workspace, c10::nullopt, c10::nullopt, 1e-5, 0, 0);
    rope_and_cache(qkv, pos, cos_sin, slots, k_cache, v_cache, Hq, Hkv, true);
    return;
  }
  TORCH_CHECK(workspace.scalar_type() == at::kFloat && workspace.numel() >= (int64_t)S * M * N,
              "decode_gemm_qkv_rope: workspace too small");
  auto st = at::hip::getCurrentHIPStream();
  float* part = workspace.data_ptr<float>();
  if (bn == 256)
    dgemm_launch<256, EPI_PARTIAL>(S, tiles, st, x, w, M, N, K, nullptr, 0, part, 0, nullptr, nullptr, nullptr);
  else
    dgemm_launch<128, EPI_PARTIAL>(S, tiles, st, x, w, M, N, K, nullptr, 0, part, 0, nullptr, nullptr, nullptr);
  const int64_t threads = (int64_t)M * (Hq + 2 * Hkv) * (D / 8);
  splitk_reduce_rope_kernel<128><<<(unsigned)((threads + 255) / 256), 256, 0, st>>>(
      part, S, M, N, (bf16*)qkv.data_ptr(), qkv.stride(0), pos.data_ptr<int32_t>(), cos_sin.data_ptr<float>(),
      (int)cos_sin.size(0), slots.data_ptr<int64_t>(), k_cache.size(0) * BSZ, (bf16*)k_cache.data_ptr(),
      (bf16*)v_cache.data_ptr(), (int)Hq, (int)Hkv, BSZ);
}

// f32 OUTPUT (the LM head: logits the sampler reads in f32): out[M, N] f32 contiguous =
// x . w^T, no K split -- the EPI_PARTIAL epilogue with one split IS an f32 store.
// bn: 128 or 256 (0 = LS_DGEMM_HEAD_BN, default 128).
bool decode_gemm_f32_supported(const at::Tensor& w, int64_t M) {
  return M >= 1 && M <= BM && w.dim() == 2 && w.scalar_type() == at::kBFloat16 && w.is_contiguous() &&
         w.size(1) % BK == 0 && w.size(0) % 128 == 0;
}

void decode_gemm_f32(at::Tensor out, at::Tensor x, at::Tensor w, int64_t bn_force) {
  check_xw(x, w);
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(decode_gemm_f32_supported(w, M), "decode_gemm_f32: shape");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.size(0) == M && out.size(1) == N,
              "decode_gemm_f32: out must be f32 [M, N] contiguous");
  static const int bn_env = env_int("LS_DGEMM_HEAD_BN", 128);
  int bn = bn_force > 0 ? (int)bn_force : bn_env;
  if (bn != 256 || N % 256 != 0) bn = 128;
  auto st = at::hip::getCurrentHIPStream();
  if (bn == 256)
    dgemm_launch<256, EPI_PARTIAL>(1, N / 256, st, x, w, M, N, K, nullptr, 0, out.data_ptr<float>(), 0, nullptr,
                                   nullptr, nullptr);
  else
    dgemm_launch<128, EPI_PARTIAL>(1, N / 128, st, x, w, M, N, K, nullptr, 0, out.data_ptr<float>(), 0, nullptr,
                                   nullptr, nullptr);
}

// out[M, F] = silu(x . w[:F]^T) * (x . w[F:]^T).  tickets: int32 [2 * (F / 128)] zeros
// once at allocation (monotonic, never reset); err: int32 [1].
// splits: 0 = automatic (2 with the in-launch combine), 1 = one launch over full K.
void decode_gemm_silu(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor tickets,
                      at::Tensor err, int64_t splits) {
  check_xw(x, w);
  const int M = (int)x.size(0), K = (int)x.size(1), F = (int)(w.size(0) / 2);
  TORCH_CHECK(decode_gemm_supported(w, true), "decode_gemm_silu: gate_up rows must be 2F with F % 128 == 0");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.size(0) == M && out.size(1) == F && out.stride(1) == 1);
  const int tiles = F / 128;
  // default 1: one launch of 128-column tiles (64 gate + 64 up) with loader waves, full K
  // (66 us at M = 256 on Llama-3-8B, tools/dgemm_bench.py); 2: the 256-column tile with
  // the in-launch K-half exchange (82 us: 8 waves that also issue their DMAs)
  static const int split_env = env_int("LS_DGEMM_SILU_SPLIT", 1);
  const int sp = splits > 0 ? (int)splits : split_env;
  auto st = at::hip::getCurrentHIPStream();
  if (sp != 2 || K / BK < 8) {
    // one launch, no combine: 128-column tiles (64 gate + 64 up), full K
    dgemm_launch<128, EPI_SILU>(1, F / 64, st, x, w, M, 2 * F, K, (bf16*)out.data_ptr(), out.stride(0), nullptr, F,
                           nullptr, nullptr, nullptr);
    return;
  }
  TORCH_CHECK(tickets.scalar_type() == at::kInt && tickets.is_cuda() && tickets.numel() >= 2 * tiles,
              "decode_gemm_silu: tickets [2 * F / 128] int32");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.is_cuda() && err.numel() >= 1);
  TORCH_CHECK(workspace.scalar_type() == at::kFloat && workspace.is_cuda() &&
              workspace.numel() >= (int64_t)tiles * BM * 256, "decode_gemm_silu: workspace too small");
  dgemm_launch<256, EPI_SILU2>(2, tiles, st, x, w, M, 2 * F, K, (bf16*)out.data_ptr(), out.stride(0), nullptr, F,
                          reinterpret_cast<unsigned*>(tickets.data_ptr<int>()), workspace.data_ptr<float>(),
                          err.data_ptr<int>());
}

// Timing-only ablation builds of the plain split-K GEMM (EPI_PARTIAL, BN = 128): abl bits
// as documented at dgemm_kernel.  Results are garbage by design.
void decode_gemm_ablate(at::Tensor x, at::Tensor w, at::Tensor workspace, int64_t abl, int64_t splits,
                        int64_t split_outer) {
  check_xw(x, w);
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  const int tiles = N / 128;
  const int S = splits > 0 ? (int)splits : pick_split(tiles, K, 4);
  TORCH_CHECK(workspace.numel() >= (int64_t)S * M * N);
  auto st = at::hip::getCurrentHIPStream();
  const dim3 grid(tiles * S);
  float* part = workspace.data_ptr<float>();
#define A_(V)                                                                                          \
  case V:                                                                                              \
    dgemm_kernel<128, 3, 4, EPI_PARTIAL, (V & ~32), (V & 32) ? 4 : 0><<<grid, (V & 32) ? 768 : 512, 0, st>>>( \
        (const bf16*)x.data_ptr(), x.stride(0),                                                        \
                                                                  (const bf16*)w.data_ptr(), M, N, K, S,  \
                                                                  nullptr, 0, part, 0, nullptr, nullptr, \
                                                                  nullptr, (int)split_outer, DgArgs());  \
    break;
  switch (abl) {
    A_(0) A_(1) A_(2) A_(3) A_(4) A_(5) A_(7) A_(8) A_(9) A_(11) A_(16) A_(17)
    A_(32) A_(33) A_(35) A_(36) A_(39) A_(48) A_(64) A_(71)
    default: TORCH_CHECK(false, "unsupported ablation ", abl);
  }
#undef A_
}

// ---------------------------------------------------------------------------------
// Norm-deferred decode layer entry points (see DgArgs).  The combine path needs every
// workgroup of the launch co-resident (tiles x S <= CUs; one workgroup per CU by LDS).
namespace {
int device_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return v;
  }();
  return n;
}

void check_cmb_common(const at::Tensor& x, const at::Tensor& w, const at::Tensor& workspace, const at::Tensor& counters,
                      const at::Tensor& err, int S) {
  check_xw(x, w);
  const int64_t M = x.size(0), N = w.size(0);
  TORCH_CHECK(N % 128 == 0, "combine path: N % 128 == 0");
  TORCH_CHECK(S >= 1 && (N / 128) * S <= device_cus(), "combine path: tiles x splits exceeds the CU count");
  TORCH_CHECK(workspace.scalar_type() == at::kFloat && workspace.is_cuda() && workspace.numel() >= S * M * N,
              "combine path: workspace too small");
  TORCH_CHECK(counters.scalar_type() == at::kLong && counters.is_cuda() && counters.numel() >= N / 128,
              "combine path: counters int64 [tiles]");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.is_cuda() && err.numel() >= 1, "combine path: err int32 [1]");
}
}  // namespace

// K splits of the combine path for an [N, K] weight (0: not supported on this device).
int64_t decode_gemm_cmb_splits(int64_t N, int64_t K) {
  if (N % 128 != 0 || K % BK != 0) return 0;
  const int tiles = (int)(N / 128), cus = device_cus();
  if (cus <= 0 || tiles > cus) return 0;
  int best = 0;
  for (int s = 1; s <= 16; ++s) {
    if (tiles * s > cus || (K / BK) / s < 4) break;
    best = s;
  }
  return best;
}

// residual[M, N] += x . w^T  (in place, bf16 residual stream);  y_out = bf16(residual * norm_g);
// sumsq_out[M][N / 128] = per-tile sums of residual^2 (for the consumer's 1/rms).
void decode_gemm_res(at::Tensor y_out, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor counters,
                     at::Tensor residual, at::Tensor norm_g, at::Tensor sumsq_out, at::Tensor err) {
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  const int S = (int)decode_gemm_cmb_splits(N, K);
  check_cmb_common(x, w, workspace, counters, err, S);
  TORCH_CHECK(residual.scalar_type() == at::kBFloat16 && residual.is_contiguous() && residual.numel() == (int64_t)M * N,
              "decode_gemm_res: residual bf16 [M, N] contiguous");
  TORCH_CHECK(y_out.scalar_type() == at::kBFloat16 && y_out.is_contiguous() && y_out.numel() == (int64_t)M * N,
              "decode_gemm_res: y_out bf16 [M, N] contiguous");
  TORCH_CHECK(norm_g.scalar_type() == at::kBFloat16 && norm_g.is_contiguous() && norm_g.numel() == N,
              "decode_gemm_res: norm weight bf16 [N]");
  TORCH_CHECK(sumsq_out.scalar_type() == at::kFloat && sumsq_out.is_contiguous() &&
              sumsq_out.numel() >= (int64_t)M * (N / 128), "decode_gemm_res: sumsq_out f32 [M, N / 128]");
  DgArgs ga;
  ga.counters = reinterpret_cast<unsigned long long*>(counters.data_ptr<int64_t>());
  ga.err = err.data_ptr<int>();
  ga.residual = (bf16*)residual.data_ptr();
  ga.norm_g = (const bf16*)norm_g.data_ptr();
  ga.y_out = (bf16*)y_out.data_ptr();
  ga.sumsq_out = sumsq_out.data_ptr<float>();
  dgemm_launch<128, EPI_CMB_RES>(S, N / 128, at::hip::getCurrentHIPStream(), x, w, M, N, K, nullptr, 0,
                                 workspace.data_ptr<float>(), 0, nullptr, nullptr, nullptr, ga);
}

// qkv = RoPE(r_m * (x . w^T)) with the step's K / V rows written to the paged cache;
// r_m from sumsq_in [M, npart] (the producer's partials) over hidden size K.
void decode_gemm_qkv_cmb(at::Tensor qkv, at::Tensor x, at::Tensor w, at::Tensor workspace, at::Tensor counters,
                         at::Tensor sumsq_in, double eps, at::Tensor pos, at::Tensor cos_sin, at::Tensor slots,
                         at::Tensor k_cache, at::Tensor v_cache, int64_t Hq, int64_t Hkv, at::Tensor err) {
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  const int S = (int)decode_gemm_cmb_splits(N, K);
  check_cmb_common(x, w, workspace, counters, err, S);
  const int D = (int)k_cache.size(3), BSZ = (int)k_cache.size(2);
  TORCH_CHECK(D == 128 && N == (Hq + 2 * Hkv) * D, "decode_gemm_qkv_cmb: head dim 128, qkv width");
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && qkv.size(0) == M && qkv.size(1) == N && qkv.stride(1) == 1);
  TORCH_CHECK(sumsq_in.scalar_type() == at::kFloat && sumsq_in.is_contiguous() && sumsq_in.dim() == 2 &&
              sumsq_in.size(0) >= M, "decode_gemm_qkv_cmb: sumsq_in f32 [M, npart]");
  TORCH_CHECK(pos.scalar_type() == at::kInt && pos.numel() >= M && slots.scalar_type() == at::kLong &&
              slots.numel() >= M && cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
              cos_sin.size(1) == D, "decode_gemm_qkv_cmb: pos / slots / cos_sin");
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous() && v_cache.dim() == 5 && v_cache.size(2) == BSZ / 8 &&
              v_cache.size(3) == D && v_cache.size(4) == 8, "decode_gemm_qkv_cmb: v_cache [NB, Hkv, BS/8, D, 8]");
  DgArgs ga;
  ga.counters = reinterpret_cast<unsigned long long*>(counters.data_ptr<int64_t>());
  ga.err = err.data_ptr<int>();
  ga.sumsq_in = sumsq_in.data_ptr<float>();
  ga.npart = (int)sumsq_in.size(1);
  ga.eps = (float)eps;
  ga.inv_h = 1.f / (float)K;
  ga.pos = pos.data_ptr<int32_t>();
  ga.cos_sin = cos_sin.data_ptr<float>();
  ga.max_pos = (int)cos_sin.size(0);
  ga.slots = slots.data_ptr<int64_t>();
  ga.nslots = k_cache.size(0) * BSZ;
  ga.kc = (bf16*)k_cache.data_ptr();
  ga.vc = (bf16*)v_cache.data_ptr();
  ga.Hq = (int)Hq;
  ga.Hkv = (int)Hkv;
  ga.BS = BSZ;
  dgemm_launch<128, EPI_CMB_QKV>(S, N / 128, at::hip::getCurrentHIPStream(), x, w, M, N, K,
                                 (bf16*)qkv.data_ptr(), qkv.stride(0), workspace.data_ptr<float>(), 0, nullptr,
                                 nullptr, nullptr, ga);
}

// out[M, F] = silu(r_m * x . w[:F]^T) * (r_m * x . w[F:]^T), r_m from sumsq_in [M, npart].
void decode_gemm_silu_r(at::Tensor out, at::Tensor x, at::Tensor w, at::Tensor sumsq_in, double eps) {
  check_xw(x, w);
  const int M = (int)x.size(0), K = (int)x.size(1), F = (int)(w.size(0) / 2);
  TORCH_CHECK(decode_gemm_supported(w, true), "decode_gemm_silu_r: gate_up rows must be 2F with F % 128 == 0");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.size(0) == M && out.size(1) == F && out.stride(1) == 1);
  TORCH_CHECK(sumsq_in.scalar_type() == at::kFloat && sumsq_in.is_contiguous() && sumsq_in.dim() == 2 &&
              sumsq_in.size(0) >= M, "decode_gemm_silu_r: sumsq_in f32 [M, npart]");
  DgArgs ga;
  ga.sumsq_in = sumsq_in.data_ptr<float>();
  ga.npart = (int)sumsq_in.size(1);
  ga.eps = (float)eps;
  ga.inv_h = 1.f / (float)K;
  dgemm_launch<128, EPI_SILU_R>(1, F / 64, at::hip::getCurrentHIPStream(), x, w, M, 2 * F, K, (bf16*)out.data_ptr(),
                                out.stride(0), nullptr, F, nullptr, nullptr, nullptr, ga);
}

// ---------------------------------------------------------------------------------
// Row helpers of the norm-deferred layer: the first layer's input (y = bf16(h * g),
// sumsq[m] = sum h^2, one partial) and the final norm (out = bf16(y * r_m)).
namespace {
__global__ void __launch_bounds__(256) rms_prep_kernel(bf16* __restrict__ y, float* __restrict__ sumsq,
                                                       const bf16* __restrict__ h, const bf16* __restrict__ g, int N) {
  __shared__ float red[4];
  const int m = blockIdx.x;
  float ss = 0.f;
  for (int c = threadIdx.x * 8; c < N; c += 256 * 8) {
    float hv[8], gv[8], yv[8];
    unpack8(ld16(h + (int64_t)m * N + c), hv);
    unpack8(ld16(g + c), gv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ss += hv[e] * hv[e];
      yv[e] = hv[e] * gv[e];
    }
    st16(y + (int64_t)m * N + c, pack8(yv));
  }
  ss = block_sum(ss, red);
  if (threadIdx.x == 0) sumsq[m] = ss;
}

__global__ void __launch_bounds__(256) rows_rms_scale_kernel(bf16* __restrict__ out, const bf16* __restrict__ y,
                                                             const float* __restrict__ sumsq, int npart, float inv_h,
                                                             float eps, int N) {
  const int m = blockIdx.x;
  const float r = rms_scale(sumsq + (int64_t)m * npart, npart, inv_h, eps);
  for (int c = threadIdx.x * 8; c < N; c += 256 * 8) {
    float v[8];
    unpack8(ld16(y + (int64_t)m * N + c), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= r;
    st16(out + (int64_t)m * N + c, pack8(v));
  }
}
}  // namespace

void rms_prep(at::Tensor y, at::Tensor sumsq, at::Tensor h, at::Tensor g) {
  const int64_t M = h.size(0), N = h.size(1);
  TORCH_CHECK(h.is_contiguous() && y.is_contiguous() && h.scalar_type() == at::kBFloat16 &&
              y.scalar_type() == at::kBFloat16 && y.numel() == M * N && N % 8 == 0, "rms_prep: bf16 [M, N]");
  TORCH_CHECK(g.numel() == N && g.scalar_type() == at::kBFloat16 && sumsq.scalar_type() == at::kFloat &&
              sumsq.numel() >= M, "rms_prep: g [N] bf16, sumsq f32 [M]");
  if (M == 0) return;
  rms_prep_kernel<<<(unsigned)M, 256, 0, at::hip::getCurrentHIPStream()>>>(
      (bf16*)y.data_ptr(), sumsq.data_ptr<float>(), (const bf16*)h.data_ptr(), (const bf16*)g.data_ptr(), (int)N);
}

void rows_rms_scale(at::Tensor out, at::Tensor y, at::Tensor sumsq, double eps) {
  const int64_t M = y.size(0), N = y.size(1);
  TORCH_CHECK(y.is_contiguous() && out.is_contiguous() && y.scalar_type() == at::kBFloat16 &&
              out.scalar_type() == at::kBFloat16 && out.numel() == M * N && N % 8 == 0, "rows_rms_scale: bf16 [M, N]");
  TORCH_CHECK(sumsq.scalar_type() == at::kFloat && sumsq.is_contiguous() && sumsq.dim() == 2 && sumsq.size(0) >= M,
              "rows_rms_scale: sumsq f32 [M, npart]");
  if (M == 0) return;
  rows_rms_scale_kernel<<<(unsigned)M, 256, 0, at::hip::getCurrentHIPStream()>>>(
      (bf16*)out.data_ptr(), (const bf16*)y.data_ptr(), sumsq.data_ptr<float>(), (int)sumsq.size(1), 1.f / (float)N,
      (float)eps, (int)N);
}
