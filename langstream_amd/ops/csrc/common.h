// Shared helpers for the langstream_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//  * bf16 tensors are handled as `__bf16` (clang native type); f32->bf16 uses the
//    plain cast, which hipcc lowers to v_cvt_pk_bf16_f32 on gfx950 (NaN-safe).
//  * memory-bound kernels move 16 B per lane (8 x bf16) per access (guide G13).
//  * wave = 64 lanes; reductions use __shfl_xor over 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LS_WAVE 64

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Paged V cache: [NB, Hkv, BS/8, D, 8] -- V^T of a (block, kv-head) in 8-key groups, each
// head dim's 8 keys one 16-B chunk.  The MFMA P.V operand (8 consecutive keys of one dim)
// is still one 16-B load, the 16 dims of a fragment are 256 contiguous bytes, and the
// step's new token lands as 2-B stores at a 16-B stride (16 lines per head instead of
// D lines of a [D, BS] image).  Element (d, key) of the image at:
__host__ __device__ __forceinline__ int64_t vt_off(int d, int key, int D) {
  return ((int64_t)(key >> 3) * D + d) * 8 + (key & 7);
}

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64).  `red` must hold
// blockDim.x/64 floats of LDS.  Result is broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

__device__ __forceinline__ uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ void st16(void* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// streamed-once data (KV cache, database rows): non-temporal load, keeps L2 for reused lines
__device__ __forceinline__ uint4 ld16_nt(const void* p) {
  return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
}

__device__ __forceinline__ void unpack8(uint4 v, float* f) {
  const bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)b[i];
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  bf16x8 b;
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (bf16)f[i];
  return __builtin_bit_cast(uint4, b);
}

// XCD-aware bijective remap of a linear workgroup id (guide §5 "XCD swizzle
// must be bijective"): consecutive logical tiles land on the same XCD so they
// share that XCD's L2.  Speed only -- never relied on for correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// ---------------------------------------------------------------------------------
// LDS-DMA helpers shared by the glds-ring GEMMs (gemm_skinny.hip, gemm_fused.hip).
// 64-B LDS rows of 32 bf16; chunk p of row r holds global k-chunk p ^ swz_g((r >> 2) & 3)
// so the 16 lanes of each ds_read_b128 bank group hit 16 distinct 16-B slots.
static __device__ __forceinline__ int swz_g(int q) { return (0x78 >> (2 * q)) & 3; }

// LDS-DMA through inline asm (cdna_hip_programming.md §5.7): with the builtin, hipcc sees
// an LDS write and puts `s_waitcnt vmcnt(0)` in front of the next ds_read, which drains
// the whole ring every K-step; the asm form is invisible to its wait insertion, and the
// kernel counts these loads itself (wait_vmcnt).
static __device__ __forceinline__ void glds16(const bf16* src, char* lds_wave_base) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds_wave_base);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}

// Same with the non-temporal hint (streamed-once operands: leave L2 to the re-read ones).
static __device__ __forceinline__ void glds16_nt(const bf16* src, char* lds_wave_base) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds_wave_base);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}

// Raw buffer resource over `bytes` bytes from p (stride 0): loads at or past `bytes`
// (voffset + instruction offset) return zeros without touching memory.
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}

// 16 B per lane from rsrc + voff + soff into LDS at lds_wave_base + 16 * lane (M0-based,
// as glds16; inline asm so hipcc does not drain vmcnt before the next ds_read).  The
// range check applies to voff only.  NT: the non-temporal hint.
template <bool NT = false>
static __device__ __forceinline__ void blds16(i32x4 rsrc, int voff, int soff, unsigned lds_addr) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(lds_addr);
  unsigned keep;
  if constexpr (NT)
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen nt lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
        : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(dst), "s"(soff)
        : "memory");
}

template <int N>
static __device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

