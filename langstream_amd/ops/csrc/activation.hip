// Elementwise activation kernels (memory-bound, 16-B vector I/O, grid-stride).
//
//  silu_and_mul : out[t, f] = silu(x[t, f]) * x[t, F + f]     (Llama SwiGLU, x = [T, 2F])
//  bias_gelu    : x[t, f]   = gelu_erf(x[t, f] + bias[f])      (BERT FFN1 epilogue, in place)
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) silu_and_mul_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                           int64_t T, int F) {
  const int fv = F >> 3;
  const int64_t total = T * fv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / fv;
    const int c = (int)(i - t * fv);
    float g[8], u[8], o[8];
    unpack8(ld16(x + t * 2 * F + c * 8), g);
    unpack8(ld16(x + t * 2 * F + F + c * 8), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
    st16(out + t * F + c * 8, pack8(o));
  }
}

__global__ void __launch_bounds__(256) bias_gelu_kernel(bf16* __restrict__ x, const bf16* __restrict__ bias,
                                                        int64_t T, int F) {
  const int fv = F >> 3;
  const int64_t total = T * fv;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = i / fv;
    const int c = (int)(i - t * fv);
    float v[8], b[8];
    unpack8(ld16(x + t * F + c * 8), v);
    if (bias) unpack8(ld16(bias + c * 8), b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float z = v[j] + (bias ? b[j] : 0.f);
      v[j] = 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
    }
    st16(x + t * F + c * 8, pack8(v));
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace

void silu_and_mul(at::Tensor out, at::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16);
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous());
  const int F = x.size(-1) / 2;
  TORCH_CHECK(F % 8 == 0 && out.size(-1) == F);
  const int64_t T = x.numel() / (2 * F);
  TORCH_CHECK(out.numel() == T * F);
  if (T == 0) return;
  silu_and_mul_kernel<<<grid_for(T * (F / 8)), 256, 0, at::hip::getCurrentHIPStream()>>>(
      (bf16*)out.data_ptr(), (const bf16*)x.data_ptr(), T, F);
}

void bias_gelu(at::Tensor x, c10::optional<at::Tensor> bias) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous());
  const int F = x.size(-1);
  TORCH_CHECK(F % 8 == 0);
  const bf16* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->numel() == F && bias->is_contiguous());
    bp = (const bf16*)bias->data_ptr();
  }
  const int64_t T = x.numel() / F;
  if (T == 0) return;
  bias_gelu_kernel<<<grid_for(T * (F / 8)), 256, 0, at::hip::getCurrentHIPStream()>>>((bf16*)x.data_ptr(), bp, T, F);
}
