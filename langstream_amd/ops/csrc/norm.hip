// Normalisation kernels (memory-bound, one workgroup per row, row held in
// registers, 16-B vector I/O).
//
//  rmsnorm            : y = x * rsqrt(mean(x^2) + eps) * w                 (Llama)
//  fused_add_rmsnorm  : r += x ; x = rmsnorm(r) * w   (in place, residual kept bf16)
//  layernorm          : y = LN(x [+ bias] [+ residual]) * g + b            (BERT)
//  embed_layernorm    : y = LN(word[id] + pos[p] + type[t]) * g + b        (BERT input)
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

template <int NV>
__global__ void __launch_bounds__(256) rmsnorm_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                      const bf16* __restrict__ w, int H, float eps,
                                                      int64_t x_stride, int64_t out_stride) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const bf16* xr = x + row * x_stride;
  bf16* orow = out + row * out_stride;
  float v[NV][8];
  float ss = 0.f;
  const int nvec = H >> 3;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      unpack8(ld16(xr + c * 8), v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / H + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float wf[8], o[8];
      unpack8(ld16(w + c * 8), wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * wf[j];
      st16(orow + c * 8, pack8(o));
    }
  }
}

template <int NV>
__global__ void __launch_bounds__(256) fused_add_rmsnorm_kernel(bf16* __restrict__ x, bf16* __restrict__ res,
                                                                const bf16* __restrict__ w, int H, float eps) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  bf16* xr = x + row * H;
  bf16* rr = res + row * H;
  float v[NV][8];
  float ss = 0.f;
  const int nvec = H >> 3;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float a[8], b[8];
      unpack8(ld16(xr + c * 8), a);
      unpack8(ld16(rr + c * 8), b);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = a[j] + b[j];
      // residual stream kept in bf16 (round once), norm computed on the rounded value
      const uint4 packed = pack8(v[i]);
      st16(rr + c * 8, packed);
      unpack8(packed, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / H + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float wf[8], o[8];
      unpack8(ld16(w + c * 8), wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv * wf[j];
      st16(xr + c * 8, pack8(o));
    }
  }
}

// LayerNorm over rows of H (H % 8 == 0).  Optional per-column bias (the
// preceding GEMM's bias, fused here) and residual.
template <int NV>
__global__ void __launch_bounds__(256) layernorm_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                        const bf16* __restrict__ bias, const bf16* __restrict__ res,
                                                        const bf16* __restrict__ g, const bf16* __restrict__ b,
                                                        int H, float eps) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int nvec = H >> 3;
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      unpack8(ld16(x + row * H + c * 8), v[i]);
      if (bias) {
        float t[8];
        unpack8(ld16(bias + c * 8), t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += t[j];
      }
      if (res) {
        float t[8];
        unpack8(ld16(res + row * H + c * 8), t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += t[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = block_sum(s, red) / H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        s2 += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum(s2, red) / H + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float gf[8], bf[8], o[8];
      unpack8(ld16(g + c * 8), gf);
      unpack8(ld16(b + c * 8), bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * inv * gf[j] + bf[j];
      st16(out + row * H + c * 8, pack8(o));
    }
  }
}

template <int NV>
__global__ void __launch_bounds__(256) embed_layernorm_kernel(bf16* __restrict__ out, const int32_t* __restrict__ ids,
                                                              const int32_t* __restrict__ pos_ids,
                                                              const int32_t* __restrict__ type_ids,
                                                              const bf16* __restrict__ wte, const bf16* __restrict__ wpe,
                                                              const bf16* __restrict__ wtt, const bf16* __restrict__ g,
                                                              const bf16* __restrict__ b, int H, float eps, int nV,
                                                              int nP, int nT) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  // clamp indices: an out-of-range id must never fault the GPU
  const int64_t id = min(max(ids[row], 0), nV - 1), p = min(max(pos_ids[row], 0), nP - 1),
                t = type_ids ? min(max(type_ids[row], 0), nT - 1) : 0;
  const int nvec = H >> 3;
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float a[8], pp[8], tt[8];
      unpack8(ld16(wte + id * H + c * 8), a);
      unpack8(ld16(wpe + p * H + c * 8), pp);
      unpack8(ld16(wtt + t * H + c * 8), tt);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = a[j] + pp[j] + tt[j];
        s += v[i][j];
      }
    }
  }
  const float mean = block_sum(s, red) / H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        s2 += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum(s2, red) / H + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float gf[8], bf[8], o[8];
      unpack8(ld16(g + c * 8), gf);
      unpack8(ld16(b + c * 8), bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * inv * gf[j] + bf[j];
      st16(out + row * H + c * 8, pack8(o));
    }
  }
}

inline int pick_threads(int H) {
  const int nvec = H / 8;
  int t = ((nvec + 63) / 64) * 64;
  return t > 256 ? 256 : t;
}

#define DISPATCH_NV(H, THREADS, ...)                                            \
  do {                                                                          \
    const int _nv = ((H) / 8 + (THREADS)-1) / (THREADS);                        \
    if (_nv <= 1) { constexpr int NV = 1; __VA_ARGS__; }                        \
    else if (_nv <= 2) { constexpr int NV = 2; __VA_ARGS__; }                   \
    else if (_nv <= 4) { constexpr int NV = 4; __VA_ARGS__; }                   \
    else if (_nv <= 8) { constexpr int NV = 8; __VA_ARGS__; }                   \
    else TORCH_CHECK(false, "hidden size too large: ", H);                      \
  } while (0)

inline void check_bf16(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
}

}  // namespace

void rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, double eps) {
  check_bf16(x, "x"); check_bf16(w, "w"); check_bf16(out, "out");
  const int H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && w.numel() == H && x.stride(-1) == 1 && out.stride(-1) == 1 && w.is_contiguous());
  const int64_t rows = x.numel() / H;
  TORCH_CHECK(x.dim() == 2 || x.is_contiguous(), "x must be 2-D or contiguous");
  const int64_t xs = x.dim() == 2 ? x.stride(0) : H, os = out.dim() == 2 ? out.stride(0) : H;
  TORCH_CHECK(xs % 8 == 0 && os % 8 == 0, "row strides must keep 16-B alignment");
  if (rows == 0) return;
  const int th = pick_threads(H);
  auto stream = at::hip::getCurrentHIPStream();
  DISPATCH_NV(H, th, rmsnorm_kernel<NV><<<rows, th, 0, stream>>>(
      (bf16*)out.data_ptr(), (const bf16*)x.data_ptr(), (const bf16*)w.data_ptr(), H, (float)eps, xs, os));
}

void fused_add_rmsnorm(at::Tensor x, at::Tensor residual, at::Tensor w, double eps) {
  check_bf16(x, "x"); check_bf16(residual, "residual"); check_bf16(w, "w");
  TORCH_CHECK(x.is_contiguous() && residual.is_contiguous() && x.sizes() == residual.sizes());
  const int H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && w.numel() == H);
  const int64_t rows = x.numel() / H;
  if (rows == 0) return;
  const int th = pick_threads(H);
  auto stream = at::hip::getCurrentHIPStream();
  DISPATCH_NV(H, th, fused_add_rmsnorm_kernel<NV><<<rows, th, 0, stream>>>(
      (bf16*)x.data_ptr(), (bf16*)residual.data_ptr(), (const bf16*)w.data_ptr(), H, (float)eps));
}

void layernorm(at::Tensor out, at::Tensor x, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> residual,
               at::Tensor g, at::Tensor b, double eps) {
  check_bf16(x, "x"); check_bf16(out, "out"); check_bf16(g, "g"); check_bf16(b, "b");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous());
  const int H = x.size(-1);
  TORCH_CHECK(H % 8 == 0 && g.numel() == H && b.numel() == H);
  const int64_t rows = x.numel() / H;
  const bf16* bp = nullptr;
  const bf16* rp = nullptr;
  if (bias.has_value()) { check_bf16(*bias, "bias"); TORCH_CHECK(bias->numel() == H); bp = (const bf16*)bias->data_ptr(); }
  if (residual.has_value()) {
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->is_contiguous() && residual->numel() == x.numel());
    rp = (const bf16*)residual->data_ptr();
  }
  if (rows == 0) return;
  const int th = pick_threads(H);
  auto stream = at::hip::getCurrentHIPStream();
  DISPATCH_NV(H, th, layernorm_kernel<NV><<<rows, th, 0, stream>>>(
      (bf16*)out.data_ptr(), (const bf16*)x.data_ptr(), bp, rp, (const bf16*)g.data_ptr(),
      (const bf16*)b.data_ptr(), H, (float)eps));
}

void embed_layernorm(at::Tensor out, at::Tensor ids, at::Tensor pos_ids, c10::optional<at::Tensor> type_ids,
                     at::Tensor wte, at::Tensor wpe, at::Tensor wtt, at::Tensor g, at::Tensor b, double eps) {
  check_bf16(out, "out"); check_bf16(wte, "wte"); check_bf16(wpe, "wpe"); check_bf16(wtt, "wtt");
  TORCH_CHECK(ids.scalar_type() == at::kInt && pos_ids.scalar_type() == at::kInt);
  TORCH_CHECK(ids.is_contiguous() && pos_ids.is_contiguous() && out.is_contiguous());
  const int H = wte.size(1);
  TORCH_CHECK(H % 8 == 0 && wpe.size(1) == H && wtt.size(1) == H && out.size(-1) == H);
  const int64_t rows = ids.numel();
  const int32_t* tp = nullptr;
  if (type_ids.has_value()) {
    TORCH_CHECK(type_ids->scalar_type() == at::kInt && type_ids->is_contiguous() && type_ids->numel() == rows);
    tp = type_ids->data_ptr<int32_t>();
  }
  if (rows == 0) return;
  const int th = pick_threads(H);
  auto stream = at::hip::getCurrentHIPStream();
  DISPATCH_NV(H, th, embed_layernorm_kernel<NV><<<rows, th, 0, stream>>>(
      (bf16*)out.data_ptr(), ids.data_ptr<int32_t>(), pos_ids.data_ptr<int32_t>(), tp, (const bf16*)wte.data_ptr(),
      (const bf16*)wpe.data_ptr(), (const bf16*)wtt.data_ptr(), (const bf16*)g.data_ptr(), (const bf16*)b.data_ptr(),
      H, (float)eps, (int)wte.size(0), (int)wpe.size(0), (int)wtt.size(0)));
}
