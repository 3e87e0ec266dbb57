// Sentence-embedding pooling for the encoder (compute-ai-embeddings):
//   mode 0 = CLS  (first token of each sequence; bge family)
//   mode 1 = mean (mean over the sequence's tokens; e5 / sentence-transformers)
// followed by optional L2 normalisation.  Input is the packed (padding-free)
// hidden state [T, H] with per-sequence start/len; output [B, H] f32 or bf16.
// One workgroup (256 threads) per sequence, 16-B vector loads over H.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"

namespace {

template <typename TO>
__global__ void __launch_bounds__(256) pool_kernel(TO* __restrict__ out, const bf16* __restrict__ x,
                                                   const int32_t* __restrict__ start, const int32_t* __restrict__ len,
                                                   int H, int mode, int normalize) {
  __shared__ float red[16];
  __shared__ __attribute__((aligned(16))) float acc_sh[4][1024];
  const int b = blockIdx.x;
  const int s0 = start[b], n = max(len[b], 1);
  const int nvec = H >> 3;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // each wave sums a strided subset of the tokens for all H columns it owns
  for (int c = lane; c < nvec; c += 64) {
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int tend = mode == 0 ? 1 : n;
    for (int t = wid; t < tend; t += 4) {
      float v[8];
      unpack8(ld16(x + (int64_t)(s0 + t) * H + c * 8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc_sh[wid][c * 8 + j] = a[j];
  }
  __syncthreads();
  const float scale = mode == 0 ? 1.f : 1.f / n;
  float ss = 0.f;
  for (int i = threadIdx.x; i < H; i += blockDim.x) {
    const float v = (acc_sh[0][i] + acc_sh[1][i] + acc_sh[2][i] + acc_sh[3][i]) * scale;
    acc_sh[0][i] = v;
    ss += v * v;
  }
  ss = block_sum(ss, red);
  const float inv = normalize ? 1.f / fmaxf(sqrtf(ss), 1e-12f) : 1.f;
  for (int i = threadIdx.x; i < H; i += blockDim.x) out[(int64_t)b * H + i] = (TO)(acc_sh[0][i] * inv);
}

__global__ void __launch_bounds__(256) l2norm_rows_kernel(bf16* __restrict__ out, const bf16* __restrict__ x,
                                                          int64_t rows, int H) {
  // one wave per row
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float ss = 0.f;
  for (int c = lane; c < H / 8; c += 64) {
    float v[8];
    unpack8(ld16(x + row * H + c * 8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
  }
  ss = wave_sum(ss);
  const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  for (int c = lane; c < H / 8; c += 64) {
    float v[8];
    unpack8(ld16(x + row * H + c * 8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= inv;
    st16(out + row * H + c * 8, pack8(v));
  }
}

}  // namespace

void pool_embeddings(at::Tensor out, at::Tensor x, at::Tensor start, at::Tensor len, int64_t mode, bool normalize) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 2);
  TORCH_CHECK(start.scalar_type() == at::kInt && len.scalar_type() == at::kInt);
  const int H = x.size(1), B = start.numel();
  TORCH_CHECK(H % 8 == 0 && H <= 1024, "hidden size must be <= 1024 and a multiple of 8");
  TORCH_CHECK(out.is_contiguous() && out.numel() == (int64_t)B * H);
  TORCH_CHECK(mode == 0 || mode == 1);
  if (B == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  if (out.scalar_type() == at::kFloat)
    pool_kernel<float><<<B, 256, 0, stream>>>(out.data_ptr<float>(), (const bf16*)x.data_ptr(),
                                              start.data_ptr<int32_t>(), len.data_ptr<int32_t>(), H, (int)mode,
                                              normalize ? 1 : 0);
  else if (out.scalar_type() == at::kBFloat16)
    pool_kernel<bf16><<<B, 256, 0, stream>>>((bf16*)out.data_ptr(), (const bf16*)x.data_ptr(),
                                             start.data_ptr<int32_t>(), len.data_ptr<int32_t>(), H, (int)mode,
                                             normalize ? 1 : 0);
  else
    TORCH_CHECK(false, "out must be f32 or bf16");
}

void l2_normalize_rows(at::Tensor out, at::Tensor x) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16);
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.dim() == 2 && x.sizes() == out.sizes());
  const int H = x.size(1);
  TORCH_CHECK(H % 8 == 0);
  const int64_t rows = x.size(0);
  if (rows == 0) return;
  l2norm_rows_kernel<<<(rows + 3) / 4, 256, 0, at::hip::getCurrentHIPStream()>>>((bf16*)out.data_ptr(),
                                                                                 (const bf16*)x.data_ptr(), rows, H);
}
