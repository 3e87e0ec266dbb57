// One-shot all-reduce for decode-sized tensor-parallel messages (bf16 sum), an
// alternative to the RCCL ring for the two per-layer all-reduces of a TP decode step
// (LlamaRunner::all_reduce; enabled with LS_ONESHOT_AR=1).
//
// Why: a decode step's all-reduce moves B x hidden bf16 (256 x 8192 x 2 B = 4 MiB at
// B = 256 on Llama-3-70B), and a ring pays 2(W-1) latency-bound hops for it.  On xGMI
// every GPU has a direct link to every other one (point-to-point, 8 GPUs fully
// connected), so one step suffices: every rank publishes its input in a buffer the
// others can read (IPC-mapped device memory), and every rank reads all W inputs and
// sums them itself -- (W-1) x message bytes in over W-1 links in parallel.
//
// Protocol (per workgroup b, which owns a fixed slice of the message):
//   e = ++epoch[b]                          (local counter, one per workgroup)
//   copy my slice of the input into my buffer half (e & 1)
//   system-scope release fence; store flag[peer][my rank][b] = e on every peer (vector
//     atomic stores -- never scalar stores)
//   wait until flag[me][src][b] >= e for every src (system-scope acquire loads; the spin
//     is bounded: on timeout *err is set (sticky), the workgroup writes NaN instead of a
//     sum of possibly stale peer buffers, and the kernel finishes instead of hanging.  The
//     step executor copies *err next to every step's results and fails the step when it
//     is set -- a stalled peer can never turn into silently wrong logits)
//   out slice = sum over w = 0..W-1 of rank w's buffer half (e & 1), same order on every
//     rank, so every rank produces bit-identical results
// Two buffer halves make back-to-back calls safe: a rank reaches call k+2 (which
// rewrites half k & 1) only after every peer has flagged call k+1, i.e. finished call k.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <hip/hip_runtime.h>
#include <vector>
#include "common.h"

namespace py = pybind11;

#define AR_OK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));           \
  } while (0)

namespace {

constexpr int kMaxRanks = 8;
constexpr int kBlocks = 64;          // workgroups (message slices) per call
constexpr int kThreads = 256;
constexpr long long kSpinLimit = 1LL << 21;   // ~seconds: a peer that never arrives sets *err

// Per-launch I/O of up to kMaxRanks ranks: a real call fills entry 0 (one rank per
// process); the single-GPU rehearsal launches every simulated rank in ONE grid
// (blockIdx.y = entry) so all of them are co-resident -- separate streams could share a
// hardware queue and serialise, leaving the first kernel waiting for the others.
struct IOTable {
  const bf16* in[kMaxRanks];
  bf16* out[kMaxRanks];
  int* epoch[kMaxRanks];
  int* err[kMaxRanks];
};

struct PeerTable {
  bf16* data[kMaxRanks];   // rank w's buffer base (two halves of `cap` elements)
  int* flags[kMaxRanks];   // rank w's flag array [kMaxRanks][kBlocks]
};

// in and out may alias (in place): a workgroup reads only its own slice of `in`, before
// its first barrier, and writes `out` after the exchange.
__global__ void __launch_bounds__(kThreads) oneshot_ar_kernel(IOTable io, int64_t n, int64_t cap, int rank0, int W,
                                                              PeerTable tbl, int stall_rank) {
  __shared__ int timed_out;
  const int b = blockIdx.x, tid = threadIdx.x, y = blockIdx.y;
  const int rank = rank0 + y;
  const bf16* in = io.in[y];
  bf16* out = io.out[y];
  int* epoch = io.epoch[y];
  const int e = epoch[b] + 1;
  const int64_t half = (int64_t)(e & 1) * cap;
  // slice of whole 8-element vectors owned by this workgroup
  const int64_t nvec = n / 8;
  const int64_t per = (nvec + kBlocks - 1) / kBlocks;
  const int64_t v0 = b * per, v1 = min(nvec, v0 + per);
  bf16* mine = tbl.data[rank] + half;
  for (int64_t v = v0 + tid; v < v1; v += kThreads) st16(mine + v * 8, ld16(in + v * 8));
  if (b == 0)   // ragged tail (n % 8 elements)
    for (int64_t i = nvec * 8 + tid; i < n; i += kThreads) mine[i] = in[i];
  if (tid == 0) timed_out = 0;
  __threadfence_system();
  __syncthreads();
  // stall_rank (rehearsal only): that simulated rank never publishes, like a peer that
  // hangs before its all-reduce
  if (tid < W && rank != stall_rank)
    __hip_atomic_store(tbl.flags[tid] + rank * kBlocks + b, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < W) {
    const int* f = tbl.flags[rank] + tid * kBlocks + b;
    long long spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (++spins > kSpinLimit) {
        __hip_atomic_store(io.err[y], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __threadfence_system();
  if (timed_out) {
    // never hand out a sum over buffers a peer may not have written yet
    const bf16 nan = (bf16)__builtin_nanf("");
    for (int64_t i = v0 * 8 + tid; i < v1 * 8; i += kThreads) out[i] = nan;
    if (b == 0)
      for (int64_t i = nvec * 8 + tid; i < n; i += kThreads) out[i] = nan;
    __syncthreads();
    if (tid == 0) epoch[b] = e;
    return;
  }
  for (int64_t v = v0 + tid; v < v1; v += kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < W; ++w) {
      float x[8];
      unpack8(ld16(tbl.data[w] + half + v * 8), x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
    st16(out + v * 8, pack8(acc));
  }
  if (b == 0)
    for (int64_t i = nvec * 8 + tid; i < n; i += kThreads) {
      float a = 0.f;
      for (int w = 0; w < W; ++w) a += (float)tbl.data[w][half + i];
      out[i] = (bf16)a;
    }
  __syncthreads();
  if (tid == 0) epoch[b] = e;
}

// The same protocol for the other collectives of a tensor-parallel decode step -- the
// vocab-parallel sampler's int64 histogram all-reduce (MODE 1) and its f32 row-statistics
// and candidate all-gathers (MODE 2, 4-byte words) -- so a TP decode step needs no c10d
// call and can be captured whole into a graph without RCCL (and without its ring hops).
// Units: MODE 1 int64 (2 per 16-B vector), MODE 2 32-bit words (4 per vector).  `n` is
// the per-rank unit count; MODE 2 writes rank w's units at out + w * n (word stores: the
// segments are not 16-B aligned in general).  A timed-out wait writes all-ones / NaN words.
template <int MODE>
__global__ void __launch_bounds__(kThreads) oneshot_x_kernel(const void* in_, void* out_, int* epoch, int* err, int64_t n,
                                                             int64_t half_bytes, int rank, int W, PeerTable tbl) {
  __shared__ int timed_out;
  constexpr int U = MODE == 1 ? 8 : 4;   // bytes per unit
  constexpr int VU = 16 / U;             // units per 16-B vector
  const int b = blockIdx.x, tid = threadIdx.x;
  const char* in = (const char*)in_;
  const int e = epoch[b] + 1;
  const int64_t half = (int64_t)(e & 1) * half_bytes;   // byte offset of this call's buffer half
  const int64_t nvec = n / VU;
  const int64_t per = (nvec + kBlocks - 1) / kBlocks;
  const int64_t v0 = b * per, v1 = min(nvec, v0 + per);
  char* mine = (char*)tbl.data[rank] + half;
  for (int64_t v = v0 + tid; v < v1; v += kThreads) st16(mine + v * 16, ld16(in + v * 16));
  if (b == 0)
    for (int64_t i = nvec * VU + tid; i < n; i += kThreads) {
      if constexpr (U == 8) reinterpret_cast<int64_t*>(mine)[i] = reinterpret_cast<const int64_t*>(in)[i];
      else reinterpret_cast<uint32_t*>(mine)[i] = reinterpret_cast<const uint32_t*>(in)[i];
    }
  if (tid == 0) timed_out = 0;
  __threadfence_system();
  __syncthreads();
  if (tid < W) __hip_atomic_store(tbl.flags[tid] + rank * kBlocks + b, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < W) {
    const int* f = tbl.flags[rank] + tid * kBlocks + b;
    long long spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (++spins > kSpinLimit) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __threadfence_system();
  // this workgroup's units: vectors [v0, v1) plus (block 0) the ragged tail
  auto for_units = [&](auto&& f) {
    for (int64_t i = v0 * VU + tid; i < v1 * VU; i += kThreads) f(i);
    if (b == 0)
      for (int64_t i = nvec * VU + tid; i < n; i += kThreads) f(i);
  };
  if constexpr (MODE == 1) {
    int64_t* out = (int64_t*)out_;
    if (timed_out) {
      for_units([&](int64_t i) { out[i] = -1; });
    } else {
      for (int64_t v = v0 + tid; v < v1; v += kThreads) {
        int64_t a0 = 0, a1 = 0;
        for (int w = 0; w < W; ++w) {
          const uint4 x = ld16((const char*)tbl.data[w] + half + v * 16);
          a0 += (int64_t)(((uint64_t)x.y << 32) | x.x);
          a1 += (int64_t)(((uint64_t)x.w << 32) | x.z);
        }
        out[v * 2] = a0;
        out[v * 2 + 1] = a1;
      }
      if (b == 0)
        for (int64_t i = nvec * VU + tid; i < n; i += kThreads) {
          int64_t a = 0;
          for (int w = 0; w < W; ++w) a += reinterpret_cast<const int64_t*>((const char*)tbl.data[w] + half)[i];
          out[i] = a;
        }
    }
  } else {
    uint32_t* out = (uint32_t*)out_;
    for (int w = 0; w < W; ++w) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>((const char*)tbl.data[w] + half);
      for_units([&](int64_t i) { out[w * n + i] = timed_out ? 0x7FC00000u : src[i]; });
    }
  }
  __syncthreads();
  if (tid == 0) epoch[b] = e;
}

void launch_oneshot(const IOTable& io, int ranks_in_grid, int64_t n, int64_t cap, int rank0, int W,
                    const PeerTable& tbl, hipStream_t stream, int stall_rank = -1) {
  oneshot_ar_kernel<<<dim3(kBlocks, ranks_in_grid), kThreads, 0, stream>>>(io, n, cap, rank0, W, tbl, stall_rank);
}

int64_t region_bytes(int64_t cap) { return 2 * cap * (int64_t)sizeof(bf16) + kMaxRanks * kBlocks * sizeof(int); }

}  // namespace

// ---------------------------------------------------------------------------------
// Multi-process form: one instance per TP rank, built collectively over the process
// group (IPC handles exchanged with an all-gather).
class OneShotAllReduce {
 public:
  OneShotAllReduce(c10::intrusive_ptr<::c10d::ProcessGroup> pg, int64_t max_elems)
      : pg_(std::move(pg)), cap_(max_elems) {
    W_ = pg_->getSize();
    rank_ = pg_->getRank();
    TORCH_CHECK(W_ >= 1 && W_ <= kMaxRanks, "one-shot all-reduce supports up to ", kMaxRanks, " ranks");
    // Data halves: plain device memory (written once by the owner, read once per call by
    // each peer over xGMI).  Flags: UNCACHED device memory -- peers on other GPUs spin on
    // them with system-scope acquires, and a coarse-grained allocation gives no coherence
    // guarantee for a remote writer's stores into a line this GPU's L2 may hold.  A driver
    // that cannot export uncached memory over IPC falls back to plain memory (warned).
    const int64_t dbytes = 2 * cap_ * (int64_t)sizeof(bf16);
    const int64_t fbytes = kMaxRanks * kBlocks * (int64_t)sizeof(int);
    AR_OK(hipMalloc(&base_, dbytes));
    AR_OK(hipMemset(base_, 0, dbytes));
    hipIpcMemHandle_t h[2];
    AR_OK(hipIpcGetMemHandle(&h[0], base_));
    if (hipExtMallocWithFlags(&flags_, fbytes, hipDeviceMallocUncached) == hipSuccess &&
        hipIpcGetMemHandle(&h[1], flags_) == hipSuccess) {
      flags_uncached_ = true;
    } else {
      if (flags_ != nullptr) (void)hipFree(flags_);
      (void)hipGetLastError();
      flags_ = nullptr;
      AR_OK(hipMalloc(&flags_, fbytes));
      AR_OK(hipIpcGetMemHandle(&h[1], flags_));
      TORCH_WARN_ONCE("one-shot all-reduce: uncached flag memory not exportable over IPC; using plain device memory");
    }
    AR_OK(hipMemset(flags_, 0, fbytes));
    AR_OK(hipMalloc(&epoch_, kBlocks * sizeof(int) + sizeof(int)));
    AR_OK(hipMemset(epoch_, 0, kBlocks * sizeof(int) + sizeof(int)));
    err_ = epoch_ + kBlocks;
    AR_OK(hipDeviceSynchronize());
    auto opts = at::TensorOptions().dtype(at::kByte).device(at::kCUDA, at::hip::current_device());
    at::Tensor mine = at::from_blob(h, {(int64_t)sizeof(h)}, at::kByte).to(opts);
    std::vector<at::Tensor> parts;
    for (int w = 0; w < W_; ++w) parts.push_back(at::empty({(int64_t)sizeof(h)}, opts));
    std::vector<std::vector<at::Tensor>> outs{parts};
    std::vector<at::Tensor> ins{mine};
    pg_->allgather(outs, ins)->wait();
    for (int w = 0; w < W_; ++w) {
      if (w == rank_) {
        tbl_.data[w] = (bf16*)base_;
        tbl_.flags[w] = (int*)flags_;
        continue;
      }
      hipIpcMemHandle_t hw[2];
      at::Tensor hb = parts[w].cpu();
      memcpy(hw, hb.data_ptr(), sizeof(hw));
      void* q = nullptr;
      AR_OK(hipIpcOpenMemHandle(&q, hw[0], hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(q);
      tbl_.data[w] = (bf16*)q;
      q = nullptr;
      AR_OK(hipIpcOpenMemHandle(&q, hw[1], hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(q);
      tbl_.flags[w] = (int*)q;
    }
  }

  ~OneShotAllReduce() {
    for (void* q : opened_) (void)hipIpcCloseMemHandle(q);
    (void)hipFree(base_);
    (void)hipFree(flags_);
    (void)hipFree(epoch_);
  }

  bool flags_uncached() const { return flags_uncached_; }

  int64_t capacity() const { return cap_; }

  // In place: t = sum over ranks of t (bf16, contiguous, numel <= capacity()).
  void run(at::Tensor& t) {
    TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.numel() <= cap_,
                "one-shot all-reduce: contiguous bf16 up to ", cap_, " elements");
    IOTable io{};
    io.in[0] = (const bf16*)t.data_ptr();
    io.out[0] = (bf16*)t.data_ptr();
    io.epoch[0] = epoch_;
    io.err[0] = err_;
    launch_oneshot(io, 1, t.numel(), cap_, rank_, W_, tbl_, at::hip::getCurrentHIPStream().stream());
  }

  // t = sum over ranks of t (int64, contiguous, up to 2 * capacity() / 8 elements).
  void run_sum_i64(at::Tensor& t) {
    TORCH_CHECK(t.scalar_type() == at::kLong && t.is_contiguous() && t.numel() * 8 <= 2 * cap_,
                "one-shot all-reduce: contiguous int64 up to ", 2 * cap_ / 8, " elements");
    oneshot_x_kernel<1><<<kBlocks, kThreads, 0, at::hip::getCurrentHIPStream().stream()>>>(
        t.data_ptr(), t.data_ptr(), epoch_, err_, t.numel(), cap_ * (int64_t)sizeof(bf16), rank_, W_, tbl_);
  }

  // out[w * n : (w + 1) * n] = rank w's `in` (4-byte elements, n = in.numel()).
  void run_gather32(const at::Tensor& in, at::Tensor& out) {
    TORCH_CHECK(in.element_size() == 4 && in.is_contiguous() && in.numel() * 4 <= 2 * cap_ && out.is_contiguous() &&
                    out.element_size() == 4 && out.numel() == W_ * in.numel() && out.data_ptr() != in.data_ptr(),
                "one-shot all-gather: contiguous 4-byte elements up to ", 2 * cap_ / 4, " per rank");
    oneshot_x_kernel<2><<<kBlocks, kThreads, 0, at::hip::getCurrentHIPStream().stream()>>>(
        in.data_ptr(), out.data_ptr(), epoch_, err_, in.numel(), cap_ * (int64_t)sizeof(bf16), rank_, W_, tbl_);
  }

  // Device word that becomes non-zero (and stays so) when a wait timed out.
  const int* err_ptr() const { return err_; }

  // Non-zero when a wait timed out (a peer never arrived): the results are invalid.
  int64_t error() {
    int e = 0;
    AR_OK(hipMemcpy(&e, err_, sizeof(int), hipMemcpyDeviceToHost));
    return e;
  }

 private:
  c10::intrusive_ptr<::c10d::ProcessGroup> pg_;
  int64_t cap_;
  int W_ = 1, rank_ = 0;
  void* base_ = nullptr;
  void* flags_ = nullptr;
  bool flags_uncached_ = false;
  int* epoch_ = nullptr;
  int* err_ = nullptr;
  PeerTable tbl_{};
  std::vector<void*> opened_;
};

std::shared_ptr<OneShotAllReduce> make_oneshot_allreduce(c10::intrusive_ptr<::c10d::ProcessGroup> pg,
                                                         int64_t max_elems) {
  return std::make_shared<OneShotAllReduce>(std::move(pg), max_elems);
}

void oneshot_allreduce_run(const std::shared_ptr<OneShotAllReduce>& ar, at::Tensor t) { ar->run(t); }
void oneshot_allreduce_i64(const std::shared_ptr<OneShotAllReduce>& ar, at::Tensor t) { ar->run_sum_i64(t); }
void oneshot_allgather32(const std::shared_ptr<OneShotAllReduce>& ar, const at::Tensor& in, at::Tensor out) {
  ar->run_gather32(in, out);
}
// Bytes ONE call may move (one buffer half: run_sum_i64 / run_gather32 accept up to
// capacity() bf16 elements' worth; the other half is the next call's).
int64_t oneshot_capacity_bytes(const std::shared_ptr<OneShotAllReduce>& ar) {
  return ar->capacity() * (int64_t)sizeof(bf16);
}

// The sampler's int64 sum: on the one-shot buffers when the message fits one call, c10d
// otherwise.  Returns true when the one-shot path ran.
bool oneshot_route_sum_i64(const std::shared_ptr<OneShotAllReduce>& ar,
                           const c10::intrusive_ptr<::c10d::ProcessGroup>& pg, at::Tensor t) {
  if (ar && t.numel() * 8 <= oneshot_capacity_bytes(ar)) {
    ar->run_sum_i64(t);
    return true;
  }
  std::vector<at::Tensor> v{t};
  pg->allreduce(v)->wait();
  return false;
}

// The sampler's 32-bit all-gather (dst = W x src), routed the same way.
bool oneshot_route_gather32(const std::shared_ptr<OneShotAllReduce>& ar,
                            const c10::intrusive_ptr<::c10d::ProcessGroup>& pg, const at::Tensor& src,
                            const at::Tensor& dst) {
  const int64_t W = pg->getSize(), per = src.numel();
  if (ar && per * 4 <= oneshot_capacity_bytes(ar)) {
    at::Tensor d = dst;
    ar->run_gather32(src, d);
    return true;
  }
  std::vector<at::Tensor> parts;
  for (int64_t w = 0; w < W; ++w) parts.push_back(dst.narrow(0, w * per, per));
  std::vector<std::vector<at::Tensor>> outs{parts};
  std::vector<at::Tensor> ins{src};
  pg->allgather(outs, ins)->wait();
  return false;
}
const int* oneshot_allreduce_err(const std::shared_ptr<OneShotAllReduce>& ar) { return ar->err_ptr(); }

// Single-GPU rehearsal of the protocol: W simulated ranks with their own buffers, flag
// arrays and epoch counters on one device, all launched in ONE grid (co-resident),
// `calls` back-to-back calls.  Returns the per-rank outputs of the last call and the
// per-rank error flags.  stall_rank >= 0: that rank never publishes its flags (a hung
// peer): every other rank must time out, flag the error and write NaN, not a sum.
std::vector<at::Tensor> oneshot_allreduce_sim(std::vector<at::Tensor> inputs, int64_t calls, int64_t stall_rank) {
  const int W = (int)inputs.size();
  TORCH_CHECK(W >= 1 && W <= kMaxRanks && calls >= 1);
  const int64_t n = inputs[0].numel();
  for (auto& t : inputs)
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.numel() == n);
  auto opts = inputs[0].options();
  std::vector<at::Tensor> regions, outs;
  at::Tensor epochs = at::zeros({W, kBlocks + 1}, opts.dtype(at::kInt));
  PeerTable tbl{};
  IOTable io{};
  for (int w = 0; w < W; ++w) {
    regions.push_back(at::zeros({region_bytes(n)}, opts.dtype(at::kByte)));
    outs.push_back(at::empty_like(inputs[w]));
    char* p = (char*)regions[w].data_ptr();
    tbl.data[w] = (bf16*)p;
    tbl.flags[w] = (int*)(p + 2 * n * sizeof(bf16));
    io.in[w] = (const bf16*)inputs[w].data_ptr();
    io.out[w] = (bf16*)outs[w].data_ptr();
    io.epoch[w] = epochs.data_ptr<int>() + w * (kBlocks + 1);
    io.err[w] = io.epoch[w] + kBlocks;
  }
  auto stream = at::hip::getCurrentHIPStream().stream();
  for (int64_t c = 0; c < calls; ++c) launch_oneshot(io, W, n, n, 0, W, tbl, stream, (int)stall_rank);
  AR_OK(hipStreamSynchronize(stream));
  outs.push_back(epochs.select(1, kBlocks).contiguous());
  return outs;
}

// Whether an instance built on this group got uncached (fine-grained) flag memory.
bool oneshot_flags_uncached(py::object process_group) {
  auto pg = py::cast<c10::intrusive_ptr<::c10d::ProcessGroup>>(process_group);
  return make_oneshot_allreduce(pg, 1024)->flags_uncached();
}

// World-size-agnostic self test over a real process group: build the instance, run one
// in-place all-reduce of t, return the error flag (0 = every peer arrived).
int64_t oneshot_allreduce_selftest(py::object process_group, at::Tensor t) {
  auto pg = py::cast<c10::intrusive_ptr<::c10d::ProcessGroup>>(process_group);
  auto ar = make_oneshot_allreduce(pg, t.numel());
  ar->run(t);
  AR_OK(hipStreamSynchronize(at::hip::getCurrentHIPStream().stream()));
  return ar->error();
}

// The int64 all-reduce and 32-bit all-gather forms, interleaved on ONE instance the way
// the vocab-parallel sampler calls them (bf16 sum, gather, int64 sum, gather): returns
// [bf16 result, gather result, int64 result, gather result] and the error flag.
std::vector<at::Tensor> oneshot_collectives_selftest(py::object process_group, at::Tensor bf, at::Tensor g32,
                                                     at::Tensor i64, int64_t cap) {
  auto pg = py::cast<c10::intrusive_ptr<::c10d::ProcessGroup>>(process_group);
  auto ar = make_oneshot_allreduce(pg, cap);
  const int64_t W = pg->getSize();
  at::Tensor g1 = at::empty({W * g32.numel()}, g32.options()), g2 = at::empty_like(g1);
  ar->run(bf);
  ar->run_gather32(g32, g1);
  ar->run_sum_i64(i64);
  ar->run_gather32(g32, g2);
  AR_OK(hipStreamSynchronize(at::hip::getCurrentHIPStream().stream()));
  return {bf, g1, i64, g2, at::full({1}, ar->error(), i64.options())};
}

// The runner's routing of the sampler collectives: returns {summed i64, gathered g32,
// [one-shot used for the sum, for the gather]}.  Messages past one call's capacity must
// fall back to c10d instead of failing the one-shot size check.
std::vector<at::Tensor> oneshot_route_selftest(py::object process_group, at::Tensor g32, at::Tensor i64, int64_t cap) {
  auto pg = py::cast<c10::intrusive_ptr<::c10d::ProcessGroup>>(process_group);
  auto ar = make_oneshot_allreduce(pg, cap);
  at::Tensor g = at::empty({pg->getSize() * g32.numel()}, g32.options());
  const bool a = oneshot_route_sum_i64(ar, pg, i64);
  const bool b = oneshot_route_gather32(ar, pg, g32, g);
  AR_OK(hipStreamSynchronize(at::hip::getCurrentHIPStream().stream()));
  at::Tensor used = at::tensor({(int64_t)a, (int64_t)b, ar->error()}, at::kLong);
  return {i64, g, used};
}
