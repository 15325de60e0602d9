// MI355X (gfx950 / CDNA4) health canary, part 2: the low-precision matrix datapaths
// and the LDS.
//
// canary.hip checks HBM and the bf16 MFMA path.  CDNA4's low-precision throughput runs
// on other instructions: the block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (OCP fp8
// e4m3, bf8 e5m2 and fp4 e2m1 operands with one E8M0 scale per 32-element block; 2x and
// 4x the bf16 rate per clock, MI355X_MICROARCH.md "Matrix cores") and the non-scaled
// v_mfma_f32_32x32x16_fp8_fp8.  A pod that serves an fp8 or MXFP4 model computes on
// these, so a partition is advertised healthy only if they are exact too:
//
//   1. Exactness: one wave per block computes C[32x32] = A[32xK] * B[Kx32] from small
//      integers (exact in every format, canary_common.h) with per-lane power-of-two
//      block scales, then checks every accumulator register against a scalar integer
//      reference.  Blocks below `inject_blocks` perturb one operand: the fault
//      injection that proves the verifier sees a wrong result.
//   2. Rate: register-resident MFMA chains, 8 blocks of 4 waves per CU -> TFLOP/s.
//   3. LDS march: every workgroup takes its CU's whole LDS (160 KB on gfx950), writes
//      an address-derived pattern, reads it back in reverse order (words written by
//      another wave, so addressing faults show) while writing the complement, then
//      reads the complement (both polarities of every bit).
//
// Operand and scale layout of the scaled 32x32x64 form, measured on the MI355X with raw
// fragments (scripts/probe_lowp_layout.py, profiles/r2/lowp_layout_probe.json): lane l
// (r = l & 31, h = l >> 5) holds 32 elements of row r of A (column r of B), byte j of the
// 8-dword operand for fp8/bf8, nibble j of the low 4 dwords for fp4, and its scale
// operand (byte 0, op_sel 0) is the E8M0 exponent of k-block h of that row:
//   * fp4:     element j is k = 32 h + j (the lane's 32 elements are its own block);
//   * fp8/bf8: element j is k = 32 (j >> 4) + 16 h + (j & 15), i.e. two K=32 halves, each
//     in the 32x32x16 map, so block h spans elements 16h..16h+15 of BOTH lane halves.
// A and B use the same map, C/D the dtype-independent 32x32 one (cdna_hip_programming.md
// §3).  tests/test_gpu_datapath.py checks it against a PyTorch fp32 GEMM on random codes
// and random block scales, which only matches if both maps are right.
//
// C ABI for ctypes (k8s_gpu_device_plugin_amd/ops/canary.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "canary_common.h"

namespace {

using namespace canary;
using i32x8 = __attribute__((ext_vector_type(8))) int;

constexpr int kFp8 = 0, kBf8 = 1, kFp4 = 4;  // cbsz / blgp format codes
constexpr int kFp8Unscaled = 8;             // host-side id of v_mfma_f32_32x32x16_fp8_fp8

// OCP code of a small integer v in [-4, 4] (every one is exact in all three formats).
template <int FMT>
__device__ __forceinline__ uint32_t lowp_code(int v) {
  const uint32_t m = static_cast<uint32_t>(v < 0 ? -v : v);
  uint32_t c;
  if (FMT == kFp8) c = m == 0 ? 0u : m == 1 ? 0x38u : m == 2 ? 0x40u : m == 3 ? 0x44u : 0x48u;       // e4m3fn
  else if (FMT == kBf8) c = m == 0 ? 0u : m == 1 ? 0x3Cu : m == 2 ? 0x40u : m == 3 ? 0x42u : 0x44u;  // e5m2
  else c = m == 0 ? 0u : m == 1 ? 0x2u : m == 2 ? 0x4u : m == 3 ? 0x5u : 0x6u;                       // e2m1
  if (v < 0) c |= FMT == kFp4 ? 0x8u : 0x80u;
  return c;
}

template <int FMT>
constexpr int kBits = FMT == kFp4 ? 4 : 8;

// k (within one 64-deep step) of element j of a lane in half h (see the layout note above)
template <int FMT>
__device__ __forceinline__ int kmap(int h, int j) {
  return FMT == kFp4 ? 32 * h + j : 32 * (j >> 4) + 16 * h + (j & 15);
}

// element j (0..31) of a lane's operand
template <int FMT>
__device__ __forceinline__ void put(i32x8& x, int j, uint32_t code) {
  constexpr int b = kBits<FMT>;
  x[(j * b) >> 5] |= static_cast<int>(code << ((j * b) & 31));
}

// E8M0 block scale of (row or column `rc`, k-block `kb`, operand `which`) when varied:
// 2^0 or 2^1, so every product stays an exact small integer in fp32.
__device__ __forceinline__ int scale_exp(int vary, int rc, int kb, int which) {
  return vary ? static_cast<int>(mix32((static_cast<uint64_t>(which) << 48) ^ (static_cast<uint64_t>(rc) << 24) ^
                                       static_cast<uint64_t>(kb)) & 1u)
              : 0;
}

template <int FMT>
__global__ void __launch_bounds__(64) lowp_exact(int ksteps, int vary_scale, int inject_blocks,
                                                 unsigned long long* __restrict__ errors) {
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const uint32_t blk = blockIdx.x + (static_cast<uint32_t>(FMT + 1) << 20);  // distinct data per format
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int s = 0; s < ksteps; ++s) {
    i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const int k = 64 * s + kmap<FMT>(h, j);
      int av = a_val(blk, r, k);
      if (s == 0 && j == 0 && lane == 0 && static_cast<int>(blockIdx.x) < inject_blocks) av = av == 4 ? 3 : av + 1;
      put<FMT>(a, j, lowp_code<FMT>(av));
      put<FMT>(b, j, lowp_code<FMT>(b_val(blk, k, r)));
    }
    const int sa = 127 + scale_exp(vary_scale, r, 2 * s + h, 0);
    const int sb = 127 + scale_exp(vary_scale, r, 2 * s + h, 1);
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, FMT, FMT, 0, sa, 0, sb);
  }
  uint32_t bad = 0;
  const int col = lane & 31;
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    int ref = 0;
    for (int kb = 0; kb < 2 * ksteps; ++kb) {
      int part = 0;
      for (int j = 0; j < 32; ++j) part += a_val(blk, row, 32 * kb + j) * b_val(blk, 32 * kb + j, col);
      ref += part << (scale_exp(vary_scale, row, kb, 0) + scale_exp(vary_scale, col, kb, 1));
    }
    bad += acc[reg] != static_cast<float>(ref);
  }
  for (int off = kWave / 2; off > 0; off >>= 1) bad += __shfl_down(bad, off, kWave);
  if (lane == 0 && bad) atomicAdd(errors, static_cast<unsigned long long>(bad));
}

// Non-scaled fp8: lane l holds A[r][16 s + 8 h + j] / B[16 s + 8 h + j][r], byte j of a
// 2-dword operand (the bf16 32x32x16 map with one byte per element).
__global__ void __launch_bounds__(64) fp8_exact(int ksteps, int inject_blocks, unsigned long long* __restrict__ errors) {
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const uint32_t blk = blockIdx.x + (0x77u << 20);
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int s = 0; s < ksteps; ++s) {
    uint64_t a = 0, b = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * h + j;
      int av = a_val(blk, r, k);
      if (s == 0 && j == 0 && lane == 0 && static_cast<int>(blockIdx.x) < inject_blocks) av = av == 4 ? 3 : av + 1;
      a |= static_cast<uint64_t>(lowp_code<kFp8>(av)) << (8 * j);
      b |= static_cast<uint64_t>(lowp_code<kFp8>(b_val(blk, k, r))) << (8 * j);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(static_cast<long>(a), static_cast<long>(b), acc, 0, 0, 0);
  }
  uint32_t bad = 0;
  const int col = lane & 31;
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    int ref = 0;
    for (int k = 0; k < ksteps * 16; ++k) ref += a_val(blk, row, k) * b_val(blk, k, col);
    bad += acc[reg] != static_cast<float>(ref);
  }
  for (int off = kWave / 2; off > 0; off >>= 1) bad += __shfl_down(bad, off, kWave);
  if (lane == 0 && bad) atomicAdd(errors, static_cast<unsigned long long>(bad));
}

// Throughput: register-resident operands, two independent accumulator chains per wave.
template <int FMT>
__global__ void __launch_bounds__(256) lowp_rate(int iters, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    put<FMT>(a, j, lowp_code<FMT>(((lane + j) % 5) - 2));
    put<FMT>(b, j, lowp_code<FMT>(((lane * 3 + j) % 7) - 3));
  }
  f32x16 acc0, acc1;
  for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
  for (int it = 0; it < iters; ++it) {
    acc0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc0, FMT, FMT, 0, 127, 0, 127);
    acc1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a, acc1, FMT, FMT, 0, 127, 0, 127);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i];
  if (s == 1234.5f) sink[blockIdx.x * blockDim.x + threadIdx.x] = s;  // keeps the chains live
}

// C[MxN] (fp32) = dequant(A)[MxK] * dequant(Bt)[NxK]^T with one E8M0 scale per 32 k:
// A, Bt hold one OCP code per byte (fp4 in the low nibble), sa [M][K/32], sb [N][K/32].
// One wave per 32x32 output tile; M, N % 32 == 0 and K % 64 == 0 (host-checked).
template <int FMT>
__global__ void __launch_bounds__(64) lowp_gemm(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt,
                                                const uint8_t* __restrict__ sa, const uint8_t* __restrict__ sb,
                                                float* __restrict__ C, int M, int N, int K) {
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  const int kblocks = K / 32;
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int k0 = 0; k0 < K; k0 += 64) {
    const uint8_t* ap = A + static_cast<size_t>(m0 + r) * K + k0;
    const uint8_t* bp = Bt + static_cast<size_t>(n0 + r) * K + k0;
    i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      put<FMT>(a, j, ap[kmap<FMT>(h, j)] & (FMT == kFp4 ? 0xFu : 0xFFu));
      put<FMT>(b, j, bp[kmap<FMT>(h, j)] & (FMT == kFp4 ? 0xFu : 0xFFu));
    }
    const int ka = sa[static_cast<size_t>(m0 + r) * kblocks + k0 / 32 + h];
    const int kb = sb[static_cast<size_t>(n0 + r) * kblocks + k0 / 32 + h];
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, FMT, FMT, 0, ka, 0, kb);
  }
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    C[static_cast<size_t>(m0 + row) * N + n0 + (lane & 31)] = acc[reg];
  }
}

// One MFMA on raw fragments: lane l's operand element j is a[l * 32 + j] / b[l * 32 + j]
// (one code per byte), its scales sa[l] / sb[l]; C is written row-major with the 32x32
// C/D map.  For layout probes (scripts/probe_lowp_layout.py), not for the canary run.
template <int FMT>
__global__ void __launch_bounds__(64) lowp_raw(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                               const uint8_t* __restrict__ sa, const uint8_t* __restrict__ sb,
                                               float* __restrict__ C) {
  const int lane = threadIdx.x;
  i32x8 x = {0, 0, 0, 0, 0, 0, 0, 0}, y = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    put<FMT>(x, j, a[lane * 32 + j] & (FMT == kFp4 ? 0xFu : 0xFFu));
    put<FMT>(y, j, b[lane * 32 + j] & (FMT == kFp4 ? 0xFu : 0xFFu));
  }
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(x, y, acc, FMT, FMT, 0, sa[lane], 0, sb[lane]);
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    C[row * 32 + (lane & 31)] = acc[reg];
  }
}

__device__ __forceinline__ uint32_t lds_pat(uint32_t i, uint32_t seed) { return i * 0x9E3779B1u ^ seed; }

// March over `words` 4-byte LDS words (the whole dynamic allocation).  Block b < inject_blocks
// flips one bit between the write and the first read (verifier self-test: one mismatch each).
__global__ void __launch_bounds__(256) lds_march(int words, uint32_t seed, int inject_blocks,
                                                 unsigned long long* __restrict__ errors) {
  extern __shared__ uint32_t lds[];
  const uint32_t s = seed ^ mix32(blockIdx.x);
  const int t = threadIdx.x, nt = blockDim.x;
  for (int i = t; i < words; i += nt) lds[i] = lds_pat(i, s);
  __syncthreads();
  if (t == 0 && static_cast<int>(blockIdx.x) < inject_blocks) lds[words / 3] ^= 1u << (blockIdx.x & 31);
  __syncthreads();
  uint32_t bad = 0;
  for (int i = t; i < words; i += nt) {  // descending: thread t reads what thread nt-1-t wrote
    const int j = words - 1 - i;
    const uint32_t want = lds_pat(j, s);
    bad += lds[j] != want;
    lds[j] = ~want;
  }
  __syncthreads();
  for (int i = t; i < words; i += nt) bad += lds[i] != ~lds_pat(i, s);
  for (int off = kWave / 2; off > 0; off >>= 1) bad += __shfl_down(bad, off, kWave);
  // no __shared__ scratch: the dynamic allocation is the whole LDS
  if ((t & (kWave - 1)) == 0 && bad) atomicAdd(errors, static_cast<unsigned long long>(bad));
}

constexpr int kMaxLdsBytes = 160 * 1024;

// Launches lds_march over 2 workgroups per CU with the largest LDS allocation the device
// grants (160 KB on gfx950); returns its size in bytes, 0 on a HIP error.
unsigned long long launch_lds_march(const hipDeviceProp_t& prop, int inject_blocks, unsigned long long* d_err) {
  size_t bytes = prop.maxSharedMemoryPerMultiProcessor > 0 ? prop.maxSharedMemoryPerMultiProcessor : 0;
  if (bytes > static_cast<size_t>(kMaxLdsBytes)) bytes = kMaxLdsBytes;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (attempt == 1 || bytes == 0) bytes = prop.sharedMemPerBlock;
    bytes &= ~static_cast<size_t>(1023);
    if (bytes == 0) return 0;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(lds_march), hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(bytes));
    hipLaunchKernelGGL(lds_march, dim3(prop.multiProcessorCount * 2), dim3(256), bytes, 0,
                       static_cast<int>(bytes / 4), 0xC0FFEEu, inject_blocks, d_err);
    if (hipGetLastError() == hipSuccess) return bytes;
  }
  return 0;
}

template <int FMT>
float time_lowp_rate(int blocks, int iters, float* sink) {
  hipEvent_t e0, e1;
  float ms = 0;
  if (hipEventCreate(&e0) != hipSuccess) return 0;
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return 0;
  }
  hipLaunchKernelGGL(lowp_rate<FMT>, dim3(blocks), dim3(256), 0, 0, 16, sink);  // warm-up
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(lowp_rate<FMT>, dim3(blocks), dim3(256), 0, 0, iters, sink);
  (void)hipEventRecord(e1, 0);
  if (hipEventSynchronize(e1) != hipSuccess || hipGetLastError() != hipSuccess ||
      hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
    ms = 0;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms;
}

bool launch_lowp_exact(int fmt, int blocks, int ksteps, int vary, int inject, unsigned long long* d_err) {
  switch (fmt) {
    case kFp8: hipLaunchKernelGGL(lowp_exact<kFp8>, dim3(blocks), dim3(64), 0, 0, ksteps, vary, inject, d_err); break;
    case kBf8: hipLaunchKernelGGL(lowp_exact<kBf8>, dim3(blocks), dim3(64), 0, 0, ksteps, vary, inject, d_err); break;
    case kFp4: hipLaunchKernelGGL(lowp_exact<kFp4>, dim3(blocks), dim3(64), 0, 0, ksteps, vary, inject, d_err); break;
    case kFp8Unscaled:
      hipLaunchKernelGGL(fp8_exact, dim3(blocks), dim3(64), 0, 0, 4 * ksteps, inject, d_err);
      break;
    default: return false;
  }
  return hipGetLastError() == hipSuccess;
}

}  // namespace

extern "C" {

struct amdgpu_canary_datapath_result {
  double fp8_tflops;                // block-scaled fp8 (e4m3) MFMA, dense
  double fp4_tflops;                // block-scaled fp4 (e2m1) MFMA, dense
  unsigned long long lowp_errors;   // wrong accumulators over fp8 / bf8 / fp4 / unscaled fp8
  unsigned long long lds_errors;    // LDS march mismatches
  unsigned long long lds_bytes;     // LDS bytes per workgroup the march covered
};

// Exactness of every low-precision MFMA form (2 blocks per CU each, K = 256, varied block
// scales), the LDS march, and the fp8 / fp4 rates (`iters` MFMA pairs per wave).
int amdgpu_canary_datapaths(int device, int iters, amdgpu_canary_datapath_result* out, char* err, int err_len) {
  std::memset(out, 0, sizeof(*out));
  hipDeviceProp_t prop;
  unsigned long long* d_err = nullptr;
  float* sink = nullptr;
  unsigned long long h_err[2] = {0, 0};
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipGetDeviceProperties(&prop, device);
  if (e == hipSuccess) e = hipMalloc(&d_err, sizeof(h_err));
  if (e == hipSuccess) e = hipMemset(d_err, 0, sizeof(h_err));
  if (e == hipSuccess) e = hipMalloc(&sink, static_cast<size_t>(prop.multiProcessorCount) * 8 * 256 * sizeof(float));
  if (e == hipSuccess) {
    const int blocks = prop.multiProcessorCount * 2;
    for (int fmt : {kFp8, kBf8, kFp4, kFp8Unscaled})
      if (!launch_lowp_exact(fmt, blocks, 4, 1, 0, d_err)) {
        e = hipErrorLaunchFailure;
        break;
      }
  }
  if (e == hipSuccess) {
    out->lds_bytes = launch_lds_march(prop, 0, d_err + 1);
    if (out->lds_bytes == 0) e = hipErrorLaunchFailure;
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(h_err, d_err, sizeof(h_err), hipMemcpyDeviceToHost);
  if (e == hipSuccess) {
    out->lowp_errors = h_err[0];
    out->lds_errors = h_err[1];
    const int blocks = prop.multiProcessorCount * 8;
    if (iters < 1) iters = 1;
    const double flops = 2.0 * 32 * 32 * 64 * 2.0 /*chains*/ * iters * (blocks * 4.0 /*waves*/);
    const float t8 = time_lowp_rate<kFp8>(blocks, iters, sink);
    const float t4 = time_lowp_rate<kFp4>(blocks, iters, sink);
    out->fp8_tflops = t8 > 0 ? flops / (t8 * 1e-3) / 1e12 : 0;
    out->fp4_tflops = t4 > 0 ? flops / (t4 * 1e-3) / 1e12 : 0;
    e = hipGetLastError();
  }
  if (e != hipSuccess) std::snprintf(err, err_len, "datapaths: %s", hipGetErrorString(e));
  if (sink) (void)hipFree(sink);
  if (d_err) (void)hipFree(d_err);
  return e == hipSuccess ? 0 : -1;
}

// Wrong accumulator registers of one low-precision form (fmt 0 fp8, 1 bf8, 4 fp4: block
// scaled, K = 64 * ksteps; 8: unscaled fp8, K = 64 * ksteps too) over 2 blocks per CU, of
// which `inject_blocks` compute with one perturbed operand.  -1 on a HIP error.
long long amdgpu_canary_lowp_check(int device, int fmt, int ksteps, int vary_scale, int inject_blocks) {
  hipDeviceProp_t prop;
  unsigned long long* d_err = nullptr;
  unsigned long long h = 0;
  if (ksteps < 1 || ksteps > 64 || inject_blocks < 0 || hipSetDevice(device) != hipSuccess ||
      hipGetDeviceProperties(&prop, device) != hipSuccess)
    return -1;
  long long rc = -1;
  if (hipMalloc(&d_err, 8) == hipSuccess && hipMemset(d_err, 0, 8) == hipSuccess &&
      launch_lowp_exact(fmt, prop.multiProcessorCount * 2, ksteps, vary_scale, inject_blocks, d_err) &&
      hipDeviceSynchronize() == hipSuccess && hipMemcpy(&h, d_err, 8, hipMemcpyDeviceToHost) == hipSuccess)
    rc = static_cast<long long>(h);
  if (d_err) (void)hipFree(d_err);
  return rc;
}

// Dense TFLOP/s of the block-scaled form `fmt` (0 fp8, 1 bf8, 4 fp4); -1 on error.
int amdgpu_canary_lowp_rate(int device, int fmt, int iters, double* tflops) {
  hipDeviceProp_t prop;
  float* sink = nullptr;
  *tflops = 0;
  if (iters < 1 || hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  const int blocks = prop.multiProcessorCount * 8;
  if (hipMalloc(&sink, static_cast<size_t>(blocks) * 256 * sizeof(float)) != hipSuccess) return -1;
  float ms = 0;
  switch (fmt) {
    case kFp8: ms = time_lowp_rate<kFp8>(blocks, iters, sink); break;
    case kBf8: ms = time_lowp_rate<kBf8>(blocks, iters, sink); break;
    case kFp4: ms = time_lowp_rate<kFp4>(blocks, iters, sink); break;
    default: break;
  }
  (void)hipFree(sink);
  if (ms <= 0) return -1;
  *tflops = 2.0 * 32 * 32 * 64 * 2.0 * iters * (blocks * 4.0) / (ms * 1e-3) / 1e12;
  return 0;
}

// LDS march mismatches over 2 workgroups per CU (`inject_blocks` of them flip one bit);
// *bytes = LDS bytes per workgroup covered.  -1 on a HIP error.
long long amdgpu_canary_lds_check(int device, int inject_blocks, unsigned long long* bytes) {
  hipDeviceProp_t prop;
  unsigned long long* d_err = nullptr;
  unsigned long long h = 0;
  *bytes = 0;
  if (inject_blocks < 0 || hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess)
    return -1;
  long long rc = -1;
  if (hipMalloc(&d_err, 8) == hipSuccess && hipMemset(d_err, 0, 8) == hipSuccess) {
    *bytes = launch_lds_march(prop, inject_blocks, d_err);
    if (*bytes && hipDeviceSynchronize() == hipSuccess && hipMemcpy(&h, d_err, 8, hipMemcpyDeviceToHost) == hipSuccess)
      rc = static_cast<long long>(h);
  }
  if (d_err) (void)hipFree(d_err);
  return rc;
}

// Host wrapper for the numerics test (see lowp_gemm): all buffers in host memory.
int amdgpu_canary_lowp_gemm(int device, int fmt, const uint8_t* a_host, const uint8_t* bt_host, const uint8_t* sa_host,
                            const uint8_t* sb_host, float* c_host, int M, int N, int K, char* err, int err_len) {
  if (M <= 0 || N <= 0 || K <= 0 || M % 32 || N % 32 || K % 64 || (fmt != kFp8 && fmt != kBf8 && fmt != kFp4)) {
    std::snprintf(err, err_len, "fmt %d shape (%d,%d,%d): need fmt 0/1/4, M,N %% 32 == 0, K %% 64 == 0", fmt, M, N, K);
    return -1;
  }
  uint8_t *a = nullptr, *bt = nullptr, *sa = nullptr, *sb = nullptr;
  float* c = nullptr;
  const size_t na = static_cast<size_t>(M) * K, nb = static_cast<size_t>(N) * K, nsa = static_cast<size_t>(M) * (K / 32),
               nsb = static_cast<size_t>(N) * (K / 32), nc = static_cast<size_t>(M) * N * 4;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&a, na);
  if (e == hipSuccess) e = hipMalloc(&bt, nb);
  if (e == hipSuccess) e = hipMalloc(&sa, nsa);
  if (e == hipSuccess) e = hipMalloc(&sb, nsb);
  if (e == hipSuccess) e = hipMalloc(&c, nc);
  if (e == hipSuccess) e = hipMemcpy(a, a_host, na, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(bt, bt_host, nb, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(sa, sa_host, nsa, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(sb, sb_host, nsb, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    const dim3 grid(N / 32, M / 32);
    if (fmt == kFp8) hipLaunchKernelGGL(lowp_gemm<kFp8>, grid, dim3(64), 0, 0, a, bt, sa, sb, c, M, N, K);
    else if (fmt == kBf8) hipLaunchKernelGGL(lowp_gemm<kBf8>, grid, dim3(64), 0, 0, a, bt, sa, sb, c, M, N, K);
    else hipLaunchKernelGGL(lowp_gemm<kFp4>, grid, dim3(64), 0, 0, a, bt, sa, sb, c, M, N, K);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(c_host, c, nc, hipMemcpyDeviceToHost);
  if (e != hipSuccess) std::snprintf(err, err_len, "%s", hipGetErrorString(e));
  for (void* p : {static_cast<void*>(a), static_cast<void*>(bt), static_cast<void*>(sa), static_cast<void*>(sb),
                  static_cast<void*>(c)})
    if (p) (void)hipFree(p);
  return e == hipSuccess ? 0 : -1;
}

// Raw-fragment probe (see lowp_raw): a, b [64][32] codes, sa, sb [64], c [32][32].
int amdgpu_canary_lowp_raw(int device, int fmt, const uint8_t* a_host, const uint8_t* b_host, const uint8_t* sa_host,
                           const uint8_t* sb_host, float* c_host) {
  if (fmt != kFp8 && fmt != kBf8 && fmt != kFp4) return -1;
  uint8_t* buf = nullptr;
  float* c = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&buf, 2 * 2048 + 2 * 64);
  if (e == hipSuccess) e = hipMalloc(&c, 32 * 32 * 4);
  if (e == hipSuccess) e = hipMemcpy(buf, a_host, 2048, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(buf + 2048, b_host, 2048, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(buf + 4096, sa_host, 64, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(buf + 4160, sb_host, 64, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    if (fmt == kFp8) hipLaunchKernelGGL(lowp_raw<kFp8>, dim3(1), dim3(64), 0, 0, buf, buf + 2048, buf + 4096, buf + 4160, c);
    else if (fmt == kBf8) hipLaunchKernelGGL(lowp_raw<kBf8>, dim3(1), dim3(64), 0, 0, buf, buf + 2048, buf + 4096, buf + 4160, c);
    else hipLaunchKernelGGL(lowp_raw<kFp4>, dim3(1), dim3(64), 0, 0, buf, buf + 2048, buf + 4096, buf + 4160, c);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(c_host, c, 32 * 32 * 4, hipMemcpyDeviceToHost);
  if (c) (void)hipFree(c);
  if (buf) (void)hipFree(buf);
  return e == hipSuccess ? 0 : -1;
}

}  // extern "C"
