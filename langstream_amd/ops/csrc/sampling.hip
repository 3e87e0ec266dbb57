// Token sampling + log-probs for the decode loop (one workgroup of 1024 threads per
// sequence row; rows of 128K logits are swept 16 B per lane with 4 loads in flight per
// lane -- `sweep` below -- in 2-3 passes, L2/Infinity-Cache hot).  The first version
// loaded 4 B per lane per dependent iteration and was latency-bound: 342 us per row at
// batch 1 (profiles/prof_b1_kernel_stats.csv).
//
// Per row r (all params are device tensors so the launch is graph-capturable):
//   temperature[r] <= 0  -> greedy argmax
//   otherwise            -> Gumbel-max sampling from softmax(logits / T), optionally
//                           restricted by top_k[r] (>0) and top_p[r] (<1).  The cut is
//                           found with a 1024-bin LDS histogram of (logit - max)/T over
//                           [-32, 0] nats (8 lane-interleaved copies, merged by a
//                           block-wide suffix scan); the cutoff bin is kept whole
//                           (documented approximation: ties within 1/32 nat).
// Outputs: token[r] (int32), logprob[r] = log softmax(logits)[token] at T = 1 (what
// OpenAI-style `logprobs` and FLARE consume), and optionally the top-n alternatives.
//
// Vocab-parallel variant for tensor parallelism: tp_* kernels below (four phases with
// small exchanges instead of all-gathering the logit rows).
//
// apply_penalties: logits[row, tok] -= presence*(cnt>0) + frequency*cnt ; += bias
// (sparse triples; host builds them only for rows that use penalties / logit_bias).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

constexpr int NBINS = 1024;   // == blockDim.x: one bin per thread in the cut scan
constexpr int NCOPY = 8;      // histogram copies, picked by lane & 7 (LDS atomic contention / 8)
constexpr float RANGE = 32.f;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// Per-row 32-bit key from the 64-bit (seed, step) mix; per-element draws hash (key, index)
// with a 32-bit finaliser (two multiplies instead of two 64-bit mixes per element: the
// Gumbel pass is ALU-bound on a 128K-entry row).
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t row_key(uint64_t seed) {
  const uint64_t z = mix64(seed);
  return (uint32_t)z ^ (uint32_t)(z >> 32);
}

__device__ __forceinline__ float uniform01(uint32_t key, uint32_t idx) {
  const uint32_t z = hash32(idx * 0x9e3779b9U + key);
  // 24 random bits -> (0, 1)
  return ((float)(z >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

template <typename T>
__device__ __forceinline__ float ldf(const T* p) { return (float)(*p); }

// Calls fn(value, index) for every element of a row: 16-B vector loads (4 f32 / 8 bf16),
// four of them issued per lane before use; a scalar tail (and a scalar path for rows that
// are not 16-B aligned).  Each thread sees its elements in increasing index order.
template <typename T, typename Fn>
__device__ __forceinline__ void sweep(const T* __restrict__ lr, int V, bool aligned, Fn&& fn) {
  constexpr int N = 16 / sizeof(T);
  const int tid = threadIdx.x, nt = blockDim.x;
  int tail = 0;
  if (aligned) {
    const int nvec = V / N;
    const uint4* vp = reinterpret_cast<const uint4*>(lr);
    int v = tid;
    for (; v + 3 * nt < nvec; v += 4 * nt) {
      uint4 q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = vp[v + u * nt];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const T* e = reinterpret_cast<const T*>(&q[u]);
#pragma unroll
        for (int j = 0; j < N; ++j) fn((float)e[j], (v + u * nt) * N + j);
      }
    }
    for (; v < nvec; v += nt) {
      const uint4 q = vp[v];
      const T* e = reinterpret_cast<const T*>(&q);
#pragma unroll
      for (int j = 0; j < N; ++j) fn((float)e[j], v * N + j);
    }
    tail = nvec * N;
  }
  for (int i = tail + tid; i < V; i += nt) fn(ldf(lr + i), i);
}

struct ArgMax {
  float v;
  int i;
};
__device__ __forceinline__ ArgMax amax(ArgMax a, ArgMax b) {
  return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}
__device__ __forceinline__ ArgMax wave_argmax(ArgMax a) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = amax(a, b);
  }
  return a;
}

template <typename T>
__global__ void __launch_bounds__(1024) sample_kernel(const T* __restrict__ logits, int64_t row_stride, int V,
                                                      const float* __restrict__ temperature,
                                                      const int32_t* __restrict__ top_k,
                                                      const float* __restrict__ top_p,
                                                      const int64_t* __restrict__ seeds,
                                                      const int64_t* __restrict__ steps,
                                                      int32_t* __restrict__ out_tok, float* __restrict__ out_lp,
                                                      int n_top, int32_t* __restrict__ top_ids,
                                                      float* __restrict__ top_lps, bool aligned) {
  __shared__ float red_f[16];
  __shared__ int red_i[16];
  __shared__ unsigned long long hist_mass[NCOPY][NBINS];  // fixed point, 2^-24 units
  __shared__ int hist_cnt[NCOPY][NBINS];
  __shared__ int cut_bin;
  const int row = blockIdx.x;
  const T* lr = logits + (int64_t)row * row_stride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float temp = temperature[row];
  const bool greedy = !(temp > 0.f);
  const float invT = greedy ? 1.f : 1.f / temp;

  // ---- pass 1: max, argmax, sum exp (T = 1)
  ArgMax best{-INFINITY, 0x7fffffff};
  float mloc = -INFINITY, sloc = 0.f;
  sweep(lr, V, aligned, [&](float x, int i) {
    if (x > best.v) best = ArgMax{x, i};
    if (x > mloc) {
      sloc = sloc * __expf(mloc - x) + 1.f;
      mloc = x;
    } else {
      sloc += __expf(x - mloc);
    }
  });
  best = wave_argmax(best);
  // combine (m, s) across the wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(mloc, o, 64), so = __shfl_xor(sloc, o, 64);
    const float mn = fmaxf(mloc, mo);
    sloc = (mloc == -INFINITY ? 0.f : sloc * __expf(mloc - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
    mloc = mn;
  }
  __shared__ float red_m[16], red_s[16];
  if (lane == 0) {
    red_f[wid] = best.v;
    red_i[wid] = best.i;
    red_m[wid] = mloc;
    red_s[wid] = sloc;
  }
  __syncthreads();
  const int nw = blockDim.x >> 6;
  ArgMax gbest{-INFINITY, 0x7fffffff};
  float gm = -INFINITY;
  for (int w = 0; w < nw; ++w) {
    gbest = amax(gbest, ArgMax{red_f[w], red_i[w]});
    gm = fmaxf(gm, red_m[w]);
  }
  float gs = 0.f;
  for (int w = 0; w < nw; ++w) gs += red_m[w] == -INFINITY ? 0.f : red_s[w] * __expf(red_m[w] - gm);
  const float logZ = gm + __logf(gs);

  int token = gbest.i;
  if (!greedy) {
    const int k = top_k[row];
    const float p = top_p[row];
    const bool restrict_ = (k > 0 && k < V) || (p > 0.f && p < 1.f);
    float thresh = -INFINITY;  // in (x - max)/T units
    if (restrict_) {
      // ---- pass 2: histogram of scaled logits
      for (int b = tid; b < NCOPY * NBINS; b += blockDim.x) {
        (&hist_mass[0][0])[b] = 0ull;
        (&hist_cnt[0][0])[b] = 0;
      }
      if (tid == 0) cut_bin = 0;
      __syncthreads();
      const int cp = lane & (NCOPY - 1);
      const bool need_cnt = k > 0 && k < V, need_mass = p > 0.f && p < 1.f;
      sweep(lr, V, aligned, [&](float x, int) {
        const float z = (x - gm) * invT;
        if (z >= -RANGE) {
          const int b = min(NBINS - 1, (int)((z + RANGE) * (NBINS / RANGE)));
          // integer ds_add_u64: LDS float atomics measured ~6x slower here (sample_bench.log)
          if (need_mass) atomicAdd(&hist_mass[cp][b], (unsigned long long)(__expf(z) * 16777216.f));
          if (need_cnt) atomicAdd(&hist_cnt[cp][b], 1);
        }
      });
      __syncthreads();
      // suffix scan from the top bin: thread t owns bin NBINS-1-t (blockDim.x == NBINS)
      const int b = NBINS - 1 - tid;
      float m = 0.f;
      int c = 0;
#pragma unroll
      for (int q = 0; q < NCOPY; ++q) {
        m += (float)hist_mass[q][b] * (1.0f / 16777216.f);
        c += hist_cnt[q][b];
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {  // inclusive wave scan over increasing tid
        const float mo = __shfl_up(m, o, 64);
        const int co = __shfl_up(c, o, 64);
        if (lane >= o) {
          m += mo;
          c += co;
        }
      }
      __shared__ float wm[16];
      __shared__ int wc[16];
      if (lane == 63) {
        wm[wid] = m;
        wc[wid] = c;
      }
      __syncthreads();
      float tot = 0.f;
      for (int w = 0; w < nw; ++w) {
        if (w < wid) {
          m += wm[w];
          c += wc[w];
        }
        tot += wm[w];
      }
      const bool hit = (need_cnt && c >= k) || (need_mass && m >= p * tot);
      // the cut is the highest bin whose suffix satisfies the rule = the lowest such tid
      if (hit) atomicMax(&cut_bin, b);
      __syncthreads();
      thresh = cut_bin * (RANGE / NBINS) - RANGE;
    }
    // ---- pass 3: Gumbel-max among the kept tokens
    const uint32_t key = row_key((uint64_t)seeds[row] * 0x2545F4914F6CDD1DULL + (uint64_t)steps[row]);
    ArgMax g{-INFINITY, 0x7fffffff};
    const int cb = restrict_ ? cut_bin : -1;
    sweep(lr, V, aligned, [&](float x, int i) {
      const float z = (x - gm) * invT;
      if (restrict_) {
        const int b = z >= -RANGE ? min(NBINS - 1, (int)((z + RANGE) * (NBINS / RANGE))) : -1;
        if (b < cb) return;
      }
      const float u = uniform01(key, (uint32_t)i);
      const float gz = z - __logf(-__logf(u));
      if (gz > g.v) g = ArgMax{gz, i};
    });
    (void)thresh;
    g = wave_argmax(g);
    __syncthreads();
    if (lane == 0) {
      red_f[wid] = g.v;
      red_i[wid] = g.i;
    }
    __syncthreads();
    ArgMax gg{-INFINITY, 0x7fffffff};
    for (int w = 0; w < nw; ++w) gg = amax(gg, ArgMax{red_f[w], red_i[w]});
    token = gg.i < V ? gg.i : gbest.i;
  }
  if (tid == 0) {
    out_tok[row] = token;
    out_lp[row] = ldf(lr + token) - logZ;
  }
  // ---- optional top-n alternatives (n_top small): repeated block argmax excluding picks
  if (n_top > 0) {
    __shared__ int picked[32];
    for (int n = 0; n < n_top; ++n) {
      ArgMax bb{-INFINITY, 0x7fffffff};
      sweep(lr, V, aligned, [&](float x, int i) {
        bool skip = false;
        for (int j = 0; j < n; ++j) skip |= (picked[j] == i);
        if (!skip && x > bb.v) bb = ArgMax{x, i};
      });
      bb = wave_argmax(bb);
      __syncthreads();
      if (lane == 0) {
        red_f[wid] = bb.v;
        red_i[wid] = bb.i;
      }
      __syncthreads();
      if (tid == 0) {
        ArgMax t{-INFINITY, 0x7fffffff};
        for (int w = 0; w < nw; ++w) t = amax(t, ArgMax{red_f[w], red_i[w]});
        const int id = t.i < V ? t.i : 0;
        picked[n] = id;
        top_ids[row * n_top + n] = id;
        top_lps[row * n_top + n] = ldf(lr + id) - logZ;
      }
      __syncthreads();
    }
  }
}

template <typename T>
__global__ void penalty_kernel(T* __restrict__ logits, int64_t row_stride, int V, const int32_t* __restrict__ rows,
                               const int32_t* __restrict__ toks, const float* __restrict__ delta, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = toks[i];
  if (t < 0 || t >= V) return;
  T* p = logits + (int64_t)rows[i] * row_stride + t;
  *p = (T)((float)(*p) + delta[i]);
}


// ---------------------------------------------------------------------------------
// Vocab-parallel sampling (tensor parallelism: each rank holds logits for its slice
// [vstart, vstart + Vl) of the vocabulary).  The single-GPU kernel above decomposes into
// four per-rank phases with small exchanges in between, instead of all-gathering the
// full f32 logit rows (B x 128K x 4 B = 128 MiB per step at B = 256):
//   stats : local max / argmax (global index) and (m, s) for log-sum-exp    -> all-gather [W, R, 4]
//   hist  : local 1024-bin histogram (count, fixed-point mass) relative to
//           the GLOBAL max, for rows restricted by top-k / top-p            -> all-reduce  [R, 2, NBINS] i64
//   pick  : global cut bin from the summed histogram (the same suffix scan),
//           local Gumbel argmax with noise keyed by the GLOBAL token index,
//           the winner's raw logit, local top-n candidates                   -> all-gather [W, R, CW]
//   final : merge -> token, logprob = logit - logZ, top-n (ties: lower index)
// Histogram sums are integers and the noise depends only on (seed, step, global index),
// so every rank takes the same cut and the result equals the single-GPU kernel's on the
// same logits.  CW = 3 + 2 * n_top floats per row (idx stored as float bit patterns).
constexpr int TPS = 4;   // stats width

__device__ __forceinline__ void combine_ms(float& m, float& s, float mo, float so) {
  const float mn = fmaxf(m, mo);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
  m = mn;
}

__global__ void __launch_bounds__(1024) tp_stats_kernel(const float* __restrict__ logits, int64_t row_stride, int Vl,
                                                        int vstart, float* __restrict__ stats, bool aligned) {
  __shared__ float rf[16], rm[16], rs[16];
  __shared__ int ri[16];
  const int row = blockIdx.x;
  const float* lr = logits + (int64_t)row * row_stride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
  ArgMax best{-INFINITY, 0x7fffffff};
  float m = -INFINITY, sm = 0.f;
  sweep(lr, Vl, aligned, [&](float x, int i) {
    if (x > best.v) best = ArgMax{x, i};
    if (x > m) {
      sm = sm * __expf(m - x) + 1.f;
      m = x;
    } else {
      sm += __expf(x - m);
    }
  });
  best = wave_argmax(best);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) combine_ms(m, sm, __shfl_xor(m, o, 64), __shfl_xor(sm, o, 64));
  if (lane == 0) { rf[wid] = best.v; ri[wid] = best.i; rm[wid] = m; rs[wid] = sm; }
  __syncthreads();
  if (tid == 0) {
    ArgMax g{-INFINITY, 0x7fffffff};
    float gm = -INFINITY, gs = 0.f;
    for (int w = 0; w < nw; ++w) {
      g = amax(g, ArgMax{rf[w], ri[w]});
      combine_ms(gm, gs, rm[w], rs[w]);
    }
    float* o = stats + (int64_t)row * TPS;
    o[0] = g.v;
    o[1] = __int_as_float(g.i == 0x7fffffff ? 0x7fffffff : g.i + vstart);
    o[2] = gm;
    o[3] = gs;
  }
}

// global max, argmax and log Z of a row from the all-gathered stats [W, R, 4]
struct RowStats {
  ArgMax best;
  float logZ;
};
__device__ __forceinline__ RowStats row_stats(const float* __restrict__ stats_all, int W, int R, int row) {
  ArgMax g{-INFINITY, 0x7fffffff};
  float m = -INFINITY, sm = 0.f;
  for (int w = 0; w < W; ++w) {
    const float* p = stats_all + ((int64_t)w * R + row) * TPS;
    g = amax(g, ArgMax{p[0], __float_as_int(p[1])});
    combine_ms(m, sm, p[2], p[3]);
  }
  return RowStats{g, m + __logf(sm)};
}

__global__ void __launch_bounds__(1024) tp_hist_kernel(const float* __restrict__ logits, int64_t row_stride, int Vl,
                                                       int Vtot, const float* __restrict__ temperature,
                                                       const int32_t* __restrict__ top_k,
                                                       const float* __restrict__ top_p,
                                                       const float* __restrict__ stats_all, int W, int R,
                                                       int64_t* __restrict__ hist, bool aligned) {
  __shared__ unsigned long long hist_mass[NCOPY][NBINS];
  __shared__ int hist_cnt[NCOPY][NBINS];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  int64_t* ho = hist + (int64_t)row * 2 * NBINS;
  const float temp = temperature[row];
  const int k = top_k[row];
  const float p = top_p[row];
  const bool need_cnt = k > 0 && k < Vtot, need_mass = p > 0.f && p < 1.f;
  if (!(temp > 0.f) || !(need_cnt || need_mass)) {
    for (int b = tid; b < 2 * NBINS; b += blockDim.x) ho[b] = 0;
    return;
  }
  const float invT = 1.f / temp;
  const float gm = row_stats(stats_all, W, R, row).best.v;
  for (int b = tid; b < NCOPY * NBINS; b += blockDim.x) {
    (&hist_mass[0][0])[b] = 0ull;
    (&hist_cnt[0][0])[b] = 0;
  }
  __syncthreads();
  const int cp = lane & (NCOPY - 1);
  const float* lr = logits + (int64_t)row * row_stride;
  sweep(lr, Vl, aligned, [&](float x, int) {
    const float z = (x - gm) * invT;
    if (z >= -RANGE) {
      const int b = min(NBINS - 1, (int)((z + RANGE) * (NBINS / RANGE)));
      if (need_mass) atomicAdd(&hist_mass[cp][b], (unsigned long long)(__expf(z) * 16777216.f));
      if (need_cnt) atomicAdd(&hist_cnt[cp][b], 1);
    }
  });
  __syncthreads();
  for (int b = tid; b < NBINS; b += blockDim.x) {
    int64_t c = 0, ms = 0;
#pragma unroll
    for (int q = 0; q < NCOPY; ++q) {
      c += hist_cnt[q][b];
      ms += (int64_t)hist_mass[q][b];
    }
    ho[b] = c;
    ho[NBINS + b] = ms;
  }
}

__global__ void __launch_bounds__(1024) tp_pick_kernel(const float* __restrict__ logits, int64_t row_stride, int Vl,
                                                       int vstart, int Vtot, const float* __restrict__ temperature,
                                                       const int32_t* __restrict__ top_k,
                                                       const float* __restrict__ top_p,
                                                       const int64_t* __restrict__ seeds,
                                                       const int64_t* __restrict__ steps,
                                                       const float* __restrict__ stats_all, int W, int R,
                                                       const int64_t* __restrict__ hist_all, int n_top,
                                                       float* __restrict__ cand, bool aligned) {
  __shared__ float red_f[16], red_x[16];
  __shared__ int red_i[16];
  __shared__ int cut_bin;
  __shared__ float wm[16];
  __shared__ int wc[16];
  const int row = blockIdx.x;
  const float* lr = logits + (int64_t)row * row_stride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
  const int CW = 3 + 2 * n_top;
  float* co = cand + (int64_t)row * CW;
  const float temp = temperature[row];
  const bool greedy = !(temp > 0.f);
  if (!greedy) {
    const float invT = 1.f / temp;
    const float gm = row_stats(stats_all, W, R, row).best.v;
    const int k = top_k[row];
    const float p = top_p[row];
    const bool need_cnt = k > 0 && k < Vtot, need_mass = p > 0.f && p < 1.f;
    const bool restrict_ = need_cnt || need_mass;
    if (restrict_) {
      // the same suffix scan as sample_kernel, over the all-reduced histogram
      const int64_t* hr = hist_all + (int64_t)row * 2 * NBINS;
      const int b = NBINS - 1 - tid;
      float m = (float)hr[NBINS + b] * (1.0f / 16777216.f);
      int c = (int)hr[b];
      if (tid == 0) cut_bin = 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float mo = __shfl_up(m, o, 64);
        const int cc = __shfl_up(c, o, 64);
        if (lane >= o) {
          m += mo;
          c += cc;
        }
      }
      if (lane == 63) {
        wm[wid] = m;
        wc[wid] = c;
      }
      __syncthreads();
      float tot = 0.f;
      for (int w = 0; w < nw; ++w) {
        if (w < wid) {
          m += wm[w];
          c += wc[w];
        }
        tot += wm[w];
      }
      const bool hit = (need_cnt && c >= k) || (need_mass && m >= p * tot);
      if (hit) atomicMax(&cut_bin, b);
      __syncthreads();
    }
    const uint32_t key = row_key((uint64_t)seeds[row] * 0x2545F4914F6CDD1DULL + (uint64_t)steps[row]);
    ArgMax g{-INFINITY, 0x7fffffff};
    float gx = -INFINITY;
    const int cb = restrict_ ? cut_bin : -1;
    sweep(lr, Vl, aligned, [&](float x, int i) {
      const float z = (x - gm) * invT;
      if (restrict_) {
        const int b = z >= -RANGE ? min(NBINS - 1, (int)((z + RANGE) * (NBINS / RANGE))) : -1;
        if (b < cb) return;
      }
      const float u = uniform01(key, (uint32_t)(vstart + i));
      const float gz = z - __logf(-__logf(u));
      if (gz > g.v) {
        g = ArgMax{gz, vstart + i};
        gx = x;
      }
    });
    // wave argmax carrying the raw logit of the winner
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ArgMax b{__shfl_xor(g.v, o, 64), __shfl_xor(g.i, o, 64)};
      const float bx = __shfl_xor(gx, o, 64);
      if (b.v > g.v || (b.v == g.v && b.i < g.i)) {
        g = b;
        gx = bx;
      }
    }
    __syncthreads();
    if (lane == 0) {
      red_f[wid] = g.v;
      red_i[wid] = g.i;
      red_x[wid] = gx;
    }
    __syncthreads();
    if (tid == 0) {
      ArgMax gg{-INFINITY, 0x7fffffff};
      float xx = -INFINITY;
      for (int w = 0; w < nw; ++w)
        if (red_f[w] > gg.v || (red_f[w] == gg.v && red_i[w] < gg.i)) {
          gg = ArgMax{red_f[w], red_i[w]};
          xx = red_x[w];
        }
      co[0] = gg.v;
      co[1] = __int_as_float(gg.i);
      co[2] = xx;
    }
  } else if (tid == 0) {
    co[0] = -INFINITY;
    co[1] = __int_as_float(0x7fffffff);
    co[2] = -INFINITY;
  }
  // local top-n candidates (raw logits, global ids), as sample_kernel's repeated argmax
  if (n_top > 0) {
    __shared__ int picked[32];
    for (int n = 0; n < n_top; ++n) {
      ArgMax bb{-INFINITY, 0x7fffffff};
      sweep(lr, Vl, aligned, [&](float x, int i) {
        bool skip = false;
        for (int j = 0; j < n; ++j) skip |= (picked[j] == i);
        if (!skip && x > bb.v) bb = ArgMax{x, i};
      });
      bb = wave_argmax(bb);
      __syncthreads();
      if (lane == 0) {
        red_f[wid] = bb.v;
        red_i[wid] = bb.i;
      }
      __syncthreads();
      if (tid == 0) {
        ArgMax t{-INFINITY, 0x7fffffff};
        for (int w = 0; w < nw; ++w) t = amax(t, ArgMax{red_f[w], red_i[w]});
        picked[n] = t.i < Vl ? t.i : -1;
        co[3 + 2 * n] = t.v;
        co[4 + 2 * n] = __int_as_float(t.i < Vl ? t.i + vstart : 0x7fffffff);
      }
      __syncthreads();
    }
  }
}

// one thread per row: merge the W ranks' stats and candidates
__global__ void tp_final_kernel(const float* __restrict__ stats_all, const float* __restrict__ cand_all, int W, int R,
                                const float* __restrict__ temperature, int n_top, int32_t* __restrict__ out_tok,
                                float* __restrict__ out_lp, int32_t* __restrict__ top_ids,
                                float* __restrict__ top_lps) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= R) return;
  const int CW = 3 + 2 * n_top;
  const RowStats st = row_stats(stats_all, W, R, row);
  int token = st.best.i;
  float x = st.best.v;
  if (temperature[row] > 0.f) {
    ArgMax g{-INFINITY, 0x7fffffff};
    float gx = -INFINITY;
    for (int w = 0; w < W; ++w) {
      const float* c = cand_all + ((int64_t)w * R + row) * CW;
      const ArgMax b{c[0], __float_as_int(c[1])};
      if (b.v > g.v || (b.v == g.v && b.i < g.i)) {
        g = b;
        gx = c[2];
      }
    }
    if (g.i != 0x7fffffff) {
      token = g.i;
      x = gx;
    }
  }
  out_tok[row] = token;
  out_lp[row] = x - st.logZ;
  // top-n: repeated selection over the W x n_top candidates (each rank's list is sorted)
  int pos[64];
  for (int w = 0; w < W && w < 64; ++w) pos[w] = 0;
  for (int n = 0; n < n_top; ++n) {
    ArgMax t{-INFINITY, 0x7fffffff};
    int tw = -1;
    for (int w = 0; w < W && w < 64; ++w) {
      if (pos[w] >= n_top) continue;
      const float* c = cand_all + ((int64_t)w * R + row) * CW + 3 + 2 * pos[w];
      const ArgMax b{c[0], __float_as_int(c[1])};
      if (b.v > t.v || (b.v == t.v && b.i < t.i)) {
        t = b;
        tw = w;
      }
    }
    if (tw >= 0) ++pos[tw];
    top_ids[row * n_top + n] = t.i == 0x7fffffff ? 0 : t.i;
    top_lps[row * n_top + n] = t.v - st.logZ;
  }
}

}  // namespace

void sample_tokens(at::Tensor logits, at::Tensor temperature, at::Tensor top_k, at::Tensor top_p, at::Tensor seeds,
                   at::Tensor steps, at::Tensor out_tok, at::Tensor out_lp, at::Tensor top_ids, at::Tensor top_lps,
                   int64_t n_top) {
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1);
  const int B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && top_p.scalar_type() == at::kFloat);
  TORCH_CHECK(top_k.scalar_type() == at::kInt && seeds.scalar_type() == at::kLong && steps.scalar_type() == at::kLong);
  TORCH_CHECK(out_tok.scalar_type() == at::kInt && out_lp.scalar_type() == at::kFloat);
  TORCH_CHECK(temperature.numel() >= B && top_k.numel() >= B && top_p.numel() >= B && seeds.numel() >= B &&
              steps.numel() >= B && out_tok.numel() >= B && out_lp.numel() >= B);
  TORCH_CHECK(n_top >= 0 && n_top <= 32);
  if (n_top > 0) TORCH_CHECK(top_ids.numel() >= B * n_top && top_lps.numel() >= B * n_top);
  if (B == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const bool aligned = (reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0) &&
                       (logits.stride(0) * (int64_t)logits.element_size()) % 16 == 0;
#define LAUNCH(TT)                                                                                              \
  sample_kernel<TT><<<B, NBINS, 0, stream>>>(                                                                    \
      (const TT*)logits.data_ptr(), logits.stride(0), V, temperature.data_ptr<float>(), top_k.data_ptr<int32_t>(), \
      top_p.data_ptr<float>(), seeds.data_ptr<int64_t>(), steps.data_ptr<int64_t>(), out_tok.data_ptr<int32_t>(), \
      out_lp.data_ptr<float>(), (int)n_top, n_top > 0 ? top_ids.data_ptr<int32_t>() : nullptr,                  \
      n_top > 0 ? top_lps.data_ptr<float>() : nullptr, aligned)
  if (logits.scalar_type() == at::kFloat) LAUNCH(float);
  else if (logits.scalar_type() == at::kBFloat16) LAUNCH(bf16);
  else TORCH_CHECK(false, "logits must be f32 or bf16");
#undef LAUNCH
}

void apply_logit_deltas(at::Tensor logits, at::Tensor rows, at::Tensor toks, at::Tensor delta) {
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1);
  TORCH_CHECK(rows.scalar_type() == at::kInt && toks.scalar_type() == at::kInt && delta.scalar_type() == at::kFloat);
  const int n = rows.numel();
  TORCH_CHECK(toks.numel() == n && delta.numel() == n);
  if (n == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const int V = logits.size(1);
  if (logits.scalar_type() == at::kFloat)
    penalty_kernel<float><<<(n + 255) / 256, 256, 0, stream>>>(logits.data_ptr<float>(), logits.stride(0), V,
                                                               rows.data_ptr<int32_t>(), toks.data_ptr<int32_t>(),
                                                               delta.data_ptr<float>(), n);
  else
    penalty_kernel<bf16><<<(n + 255) / 256, 256, 0, stream>>>((bf16*)logits.data_ptr(), logits.stride(0), V,
                                                              rows.data_ptr<int32_t>(), toks.data_ptr<int32_t>(),
                                                              delta.data_ptr<float>(), n);
}

// ---- vocab-parallel sampling phases (see tp_stats_kernel); f32 logits [R, Vl] of this
// rank's vocabulary slice starting at vstart.
static bool rows_aligned(const at::Tensor& lg) {
  return (reinterpret_cast<uintptr_t>(lg.data_ptr()) % 16 == 0) && (lg.stride(0) * 4) % 16 == 0;
}

void tp_sample_stats(at::Tensor logits, int64_t vstart, at::Tensor stats) {
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.scalar_type() == at::kFloat);
  const int R = logits.size(0);
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.numel() >= (int64_t)R * TPS);
  if (R == 0) return;
  tp_stats_kernel<<<R, NBINS, 0, at::hip::getCurrentHIPStream()>>>(logits.data_ptr<float>(), logits.stride(0),
                                                                    (int)logits.size(1), (int)vstart,
                                                                    stats.data_ptr<float>(), rows_aligned(logits));
}

void tp_sample_hist(at::Tensor logits, int64_t vtot, at::Tensor temperature, at::Tensor top_k, at::Tensor top_p,
                    at::Tensor stats_all, int64_t world, at::Tensor hist) {
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.scalar_type() == at::kFloat);
  const int R = logits.size(0);
  TORCH_CHECK(stats_all.numel() >= world * R * TPS && hist.scalar_type() == at::kLong &&
              hist.numel() >= (int64_t)R * 2 * NBINS);
  if (R == 0) return;
  tp_hist_kernel<<<R, NBINS, 0, at::hip::getCurrentHIPStream()>>>(
      logits.data_ptr<float>(), logits.stride(0), (int)logits.size(1), (int)vtot, temperature.data_ptr<float>(),
      top_k.data_ptr<int32_t>(), top_p.data_ptr<float>(), stats_all.data_ptr<float>(), (int)world, R,
      hist.data_ptr<int64_t>(), rows_aligned(logits));
}

void tp_sample_pick(at::Tensor logits, int64_t vstart, int64_t vtot, at::Tensor temperature, at::Tensor top_k,
                    at::Tensor top_p, at::Tensor seeds, at::Tensor steps, at::Tensor stats_all, int64_t world,
                    at::Tensor hist_all, int64_t n_top, at::Tensor cand) {
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.scalar_type() == at::kFloat);
  const int R = logits.size(0);
  TORCH_CHECK(n_top >= 0 && n_top <= 32);
  TORCH_CHECK(cand.scalar_type() == at::kFloat && cand.numel() >= (int64_t)R * (3 + 2 * n_top));
  if (R == 0) return;
  tp_pick_kernel<<<R, NBINS, 0, at::hip::getCurrentHIPStream()>>>(
      logits.data_ptr<float>(), logits.stride(0), (int)logits.size(1), (int)vstart, (int)vtot,
      temperature.data_ptr<float>(), top_k.data_ptr<int32_t>(), top_p.data_ptr<float>(), seeds.data_ptr<int64_t>(),
      steps.data_ptr<int64_t>(), stats_all.data_ptr<float>(), (int)world, R, hist_all.data_ptr<int64_t>(),
      (int)n_top, cand.data_ptr<float>(), rows_aligned(logits));
}

void tp_sample_final(at::Tensor stats_all, at::Tensor cand_all, int64_t world, int64_t rows, at::Tensor temperature,
                     int64_t n_top, at::Tensor out_tok, at::Tensor out_lp, at::Tensor top_ids, at::Tensor top_lps) {
  TORCH_CHECK(world >= 1 && world <= 64);
  TORCH_CHECK(cand_all.numel() >= world * rows * (3 + 2 * n_top) && stats_all.numel() >= world * rows * TPS);
  if (rows == 0) return;
  tp_final_kernel<<<(int)((rows + 127) / 128), 128, 0, at::hip::getCurrentHIPStream()>>>(
      stats_all.data_ptr<float>(), cand_all.data_ptr<float>(), (int)world, (int)rows, temperature.data_ptr<float>(),
      (int)n_top, out_tok.data_ptr<int32_t>(), out_lp.data_ptr<float>(),
      n_top > 0 ? top_ids.data_ptr<int32_t>() : nullptr, n_top > 0 ? top_lps.data_ptr<float>() : nullptr);
}
