// Per-CU ingest rate on gfx950: LDS-DMA (buffer_load ... lds) vs plain vector loads into
// VGPRs, from an L2-resident region every workgroup re-reads (a decode GEMM's activations)
// and from distinct HBM regions read once (its weights), alone and concurrently.
//
// Question it answers for the decode GEMM design (docs/ARCHITECTURE.md, round-4
// headroom): is the ~45-50 GB/s per CU the LDS-DMA path delivers in dgemm_kernel a limit
// of that path, or of the CU's vector memory pipeline as a whole?  If the two paths add,
// a kernel that streams the weights into registers beside an LDS-DMA activation ring can
// ingest faster.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ingest_bench.hip -o tools/bin/ingest_bench
// Run:   tools/bin/ingest_bench            (one line of JSON per mode)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../langstream_amd/ops/csrc/common.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int NT = 512;          // 8 waves
constexpr int RING = 64 * 1024;  // LDS ring (8 KB per wave)
constexpr int Q = 6;             // loads in flight per wave

enum { DMA = 0, VMEM = 1, IDLE = 2 };

// role of waves 0-3 / 4-7 and the region each reads: l2 = one shared region of
// `l2_bytes` re-read by every workgroup; hbm = a distinct `hbm_bytes` slice per workgroup
template <int ROLE_LO, int ROLE_HI, bool LO_HBM, bool HI_HBM>
__global__ void __launch_bounds__(NT) ingest_kernel(const char* __restrict__ l2src, int64_t l2_bytes,
                                                     const char* __restrict__ hbm, int64_t hbm_bytes,
                                                     uint4* __restrict__ sink, unsigned long long* __restrict__ cycles) {
  extern __shared__ __attribute__((aligned(1024))) char lds[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool hi = wid >= 4;
  const int role = hi ? ROLE_HI : ROLE_LO;
  const bool from_hbm = hi ? HI_HBM : LO_HBM;
  const char* base = from_hbm ? hbm + (int64_t)blockIdx.x * hbm_bytes : l2src;
  const int64_t bytes = from_hbm ? hbm_bytes : l2_bytes;
  // the 4 waves of a role split the region: wave w4 reads 1-KB pieces w4, w4 + 4, ...
  const int w4 = wid & 3;
  const int64_t pieces = bytes / 1024;
  const unsigned long long t0 = wall_clock64();
  if (role == DMA) {
    const i32x4 rs = make_rsrc(base, (uint32_t)bytes);
    const unsigned ring = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds + wid * (RING / 8);
    int slot = 0;
    for (int64_t p = w4; p < pieces; p += 4) {
      blds16<false>(rs, lane * 16, (int)(p * 1024), ring + slot * 1024);
      slot = (slot + 1) & 7;
      wait_vmcnt<Q>();
    }
    wait_vmcnt<0>();
  } else if (role == VMEM) {
    uint4 acc = {0, 0, 0, 0};
    const int64_t step = 4 * 1024;
    for (int64_t off = (int64_t)w4 * 1024; off + (Q - 1) * step < bytes; off += Q * step) {
      uint4 v[Q];
#pragma unroll
      for (int j = 0; j < Q; ++j) v[j] = ld16(base + off + j * step + lane * 16);
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        acc.x ^= v[j].x; acc.y ^= v[j].y; acc.z ^= v[j].z; acc.w ^= v[j].w;
      }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[blockIdx.x * NT + threadIdx.x] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) cycles[blockIdx.x] = wall_clock64() - t0;
}

template <int A, int B, bool AH, bool BH>
void run(const char* name, const char* l2src, int64_t l2_bytes, const char* hbm, int64_t hbm_bytes, uint4* sink,
         unsigned long long* cyc, int wgs, int reps) {
  auto k = ingest_kernel<A, B, AH, BH>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  // 160 KB of dynamic LDS: one workgroup per CU
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(wgs), dim3(NT), 160 * 1024, 0, l2src, l2_bytes, hbm,
                                                 hbm_bytes, sink, cyc);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL(k, dim3(wgs), dim3(NT), 160 * 1024, 0, l2src, l2_bytes, hbm, hbm_bytes, sink, cyc);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double t = ms / 1e3 / reps;
  auto bytes_of = [&](int role, bool h) { return role == IDLE ? 0.0 : (double)(h ? hbm_bytes : l2_bytes); };
  const double per_wg = bytes_of(A, AH) + bytes_of(B, BH);
  printf("{\"mode\": \"%s\", \"us\": %.2f, \"GB_s_per_CU\": %.1f, \"chip_TB_s\": %.2f}\n", name, t * 1e6,
         per_wg / t / 1e9, per_wg * wgs / t / 1e12);
  fflush(stdout);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int wgs = cus;
  const int64_t l2_bytes = 1 << 20;      // re-read by every workgroup (X slice)
  const int64_t hbm_bytes = 1 << 20;     // per workgroup, read once (W slice)
  char *l2src, *hbm;
  uint4* sink;
  unsigned long long* cyc;
  CK(hipMalloc(&l2src, l2_bytes));
  CK(hipMalloc(&hbm, hbm_bytes * wgs + (1 << 20)));
  CK(hipMalloc(&sink, (size_t)wgs * NT * 16));
  CK(hipMalloc(&cyc, wgs * 8));
  CK(hipMemset(l2src, 1, l2_bytes));
  CK(hipMemset(hbm, 2, hbm_bytes * wgs));
  const int reps = 20;
  run<DMA, IDLE, false, false>("dma_l2 (4 waves)", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<DMA, DMA, false, false>("dma_l2 (8 waves)", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<DMA, IDLE, true, false>("dma_hbm (4 waves)", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<VMEM, IDLE, false, false>("vmem_l2 (4 waves)", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<VMEM, VMEM, false, false>("vmem_l2 (8 waves)", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<VMEM, IDLE, true, false>("vmem_hbm (4 waves)", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<DMA, DMA, false, true>("dma_l2 + dma_hbm", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<DMA, VMEM, false, true>("dma_l2 + vmem_hbm", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<VMEM, DMA, false, true>("vmem_l2 + dma_hbm", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  run<VMEM, VMEM, false, true>("vmem_l2 + vmem_hbm", l2src, l2_bytes, hbm, hbm_bytes, sink, cyc, wgs, reps);
  return 0;
}
