// MI355X (gfx950 / CDNA4) partition health canary.
//
// The reference has no device-level health check at all: its health channel has no
// producer (plugin/plugin.go:181, SURVEY.md defect D9).  Before a partition is
// advertised (and after a GPU_POST_RESET) the plugin can run this canary on it, in a
// short-lived child process so the plugin daemon itself never holds a HIP context:
//
//   1. HBM pattern test  - every 16-byte word gets an address-derived pattern
//      (catches stuck bits and aliasing/addressing faults), written and read back
//      with 16 B/lane vector accesses, block-contiguous chunks, 16 blocks per CU,
//      non-temporal loads on the verify pass (shapes chosen by the on-hardware sweep
//      below: ~6.0 TB/s write, ~6.8 TB/s read+verify on MI355X); mismatches are
//      reduced per wave (64-lane shuffles) then per block in LDS, one atomic/block.
//      Write and read passes are timed separately -> achieved HBM GB/s.
//   2. MFMA exactness    - v_mfma_f32_32x32x16_bf16 on small-integer operands
//      (exact in bf16 and fp32) checked lane-by-lane against a scalar reference
//      using the documented gfx950 fragment maps (cdna_hip_programming.md §3).
//   3. MFMA throughput   - register-resident 32x32x16 bf16 MFMA chains, 4 waves
//      per block (one per SIMD), 8 blocks per CU -> dense bf16 TFLOP/s.
//
// C ABI for ctypes (k8s_gpu_device_plugin_amd/ops/canary.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

// Address-derived 16-byte pattern, ~5 integer ops per word so the verify pass stays
// HBM-bound: lo * odd constant is a bijection mod 2^32, so no two words of a <=64 GiB
// buffer share a pattern (aliasing / addressing faults are caught), and every data bit
// takes both values across the buffer (stuck-at faults are caught).
__device__ __forceinline__ uint4 pattern(uint64_t idx, uint32_t seed) {
  const uint32_t lo = static_cast<uint32_t>(idx), hi = static_cast<uint32_t>(idx >> 32);
  const uint32_t b = lo * 0x9E3779B1u ^ (hi + seed) * 0x85EBCA77u;
  return make_uint4(b, b ^ 0xA5A5A5A5u, ~b, b * 3u + 0x6A09E667u);
}

__device__ __forceinline__ uint32_t diff(const uint4& a, const uint4& b) {
  return (a.x != b.x) + (a.y != b.y) + (a.z != b.z) + (a.w != b.w);
}

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x16 = __attribute__((ext_vector_type(16))) float;

// small integer in [-4, 4] from a hash: exactly representable in bf16
__device__ __forceinline__ int small_int(uint64_t key) { return static_cast<int>(mix32(key) % 9u) - 4; }

__device__ __forceinline__ short bf16_of_int(int v) {
  const float f = static_cast<float>(v);
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return static_cast<short>(u >> 16);  // exact for small integers
}

__device__ __forceinline__ int a_val(uint32_t blk, int row, int k) {
  return small_int((static_cast<uint64_t>(blk) << 40) ^ (static_cast<uint64_t>(row) << 20) ^ static_cast<uint64_t>(k));
}
__device__ __forceinline__ int b_val(uint32_t blk, int k, int col) {
  return small_int(0x5555ull ^ (static_cast<uint64_t>(blk) << 40) ^ (static_cast<uint64_t>(k) << 20) ^
                   static_cast<uint64_t>(col) ^ (1ull << 62));
}

// One wave per block computes C[32x32] = A[32xK] * B[Kx32] with K = 16 * ksteps, then
// every lane checks its 16 accumulator registers against a scalar integer reference.
// Blocks below `inject_blocks` perturb one A operand (lane 0, first k-step): the fault
// injection that proves the verifier sees a wrong matrix-core result.
__global__ void __launch_bounds__(64) mfma_exact(int ksteps, int inject_blocks,
                                                 unsigned long long* __restrict__ errors) {
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const uint32_t blk = blockIdx.x;
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int s = 0; s < ksteps; ++s) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      const int k = s * 16 + 8 * h + j;  // lane l holds A[r][8h+j], B[8h+j][r]
      a[j] = bf16_of_int(a_val(blk, r, k) + ((s == 0 && j == 0 && lane == 0 && static_cast<int>(blk) < inject_blocks)
                                                   ? 1 : 0));
      b[j] = bf16_of_int(b_val(blk, k, r));
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
  uint32_t bad = 0;
  const int col = lane & 31;
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);  // C/D map of 32x32x16
    int ref = 0;
    for (int k = 0; k < ksteps * 16; ++k) ref += a_val(blk, row, k) * b_val(blk, k, col);
    bad += acc[reg] != static_cast<float>(ref);
  }
  for (int off = kWave / 2; off > 0; off >>= 1) bad += __shfl_down(bad, off, kWave);
  if (lane == 0 && bad) atomicAdd(errors, static_cast<unsigned long long>(bad));
}

// Throughput: register-resident operands, two independent accumulator chains per wave.
__global__ void __launch_bounds__(256) mfma_rate(int iters, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = bf16_of_int(((lane + j) % 5) - 2);
    b[j] = bf16_of_int(((lane * 3 + j) % 7) - 3);
  }
  f32x16 acc0, acc1;
  for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
  for (int it = 0; it < iters; ++it) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc1, 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc0[i] + acc1[i];
  if (s == 1234.5f) sink[blockIdx.x * blockDim.x + threadIdx.x] = s;  // keeps the chain live
}

// Plain MFMA GEMM used by the numerics test: C[MxN] (fp32) = A[MxK] * B[KxN] (bf16,
// row-major).  One wave per 32x32 output tile, K stepped 16 at a time through
// v_mfma_f32_32x32x16_bf16 with the gfx950 operand maps: lane l (r = l&31, h = l>>5)
// feeds A[r][k0+8h+j] and B[k0+8h+j][r]; accumulator reg i of lane l is
// C[(i&3) + 8*(i>>2) + 4*h][l&31].  M, N multiples of 32, K multiple of 16 (host-checked).
__global__ void __launch_bounds__(64) mfma_gemm(const short* __restrict__ A, const short* __restrict__ B,
                                                float* __restrict__ C, int M, int N, int K) {
  const int lane = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const int tm = blockIdx.y * 32, tn = blockIdx.x * 32;
  if (tm + 32 > M || tn + 32 > N) return;  // host checks shapes; never touch memory past them
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int k0 = 0; k0 < K; k0 += 16) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = A[static_cast<size_t>(tm + r) * K + k0 + 8 * h + j];
      b[j] = B[static_cast<size_t>(k0 + 8 * h + j) * N + tn + r];
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
  for (int i = 0; i < 16; ++i) {
    const int row = tm + (i & 3) + 8 * (i >> 2) + 4 * h;
    C[static_cast<size_t>(row) * N + tn + r] = acc[i];
  }
}

// ---- HBM access-shape sweep (used to pick the canary's streaming shape on gfx950) ----
// UNROLL independent 16 B accesses in flight per lane; NT = non-temporal (streaming)
// loads/stores; CHUNKED = each block streams one contiguous chunk instead of a
// grid-stride walk.
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
__device__ __forceinline__ uint4 nt_load(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store(const uint4& v, uint4* p) {
  const u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
}

template <int UNROLL, bool NT, bool CHUNKED>
__global__ void __launch_bounds__(256) sweep_write(uint4* __restrict__ buf, uint64_t n, uint32_t seed) {
  uint64_t begin, end, step;
  if (CHUNKED) {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    begin = blockIdx.x * per + threadIdx.x;
    end = min<uint64_t>(n, (blockIdx.x + 1) * per);
    step = blockDim.x;
  } else {
    begin = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    end = n;
    step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  }
  uint64_t i = begin;
  for (; i + (UNROLL - 1) * step < end; i += UNROLL * step) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint4 v = pattern(i + u * step, seed);
      if (NT) nt_store(v, buf + i + u * step);
      else buf[i + u * step] = v;
    }
  }
  for (; i < end; i += step) buf[i] = pattern(i, seed);
}

template <int UNROLL, bool NT, bool CHUNKED>
__global__ void __launch_bounds__(256) sweep_verify(const uint4* __restrict__ buf, uint64_t n, uint32_t seed,
                                                    unsigned long long* __restrict__ errors) {
  uint64_t begin, end, step;
  if (CHUNKED) {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    begin = blockIdx.x * per + threadIdx.x;
    end = min<uint64_t>(n, (blockIdx.x + 1) * per);
    step = blockDim.x;
  } else {
    begin = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    end = n;
    step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  }
  uint32_t bad = 0;
  uint64_t i = begin;
  for (; i + (UNROLL - 1) * step < end; i += UNROLL * step) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = NT ? nt_load(buf + i + u * step) : buf[i + u * step];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) bad += diff(v[u], pattern(i + u * step, seed));
  }
  for (; i < end; i += step) bad += diff(buf[i], pattern(i, seed));
  for (int off = kWave / 2; off > 0; off >>= 1) bad += __shfl_down(bad, off, kWave);
  __shared__ uint32_t wave_bad[256 / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) wave_bad[wid] = bad;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < static_cast<int>(blockDim.x / kWave); ++w) t += wave_bad[w];
    if (t) atomicAdd(errors, static_cast<unsigned long long>(t));
  }
}

// Shapes picked from the on-hardware sweep (profiles/hbm_sweep_gpu.json, 4 GiB buffer):
// writes: block-contiguous chunks, plain stores (~6.0 TB/s); verify: block-contiguous
// chunks, non-temporal loads (~6.8 TB/s), both at 16 blocks of 256 threads per CU.
constexpr int kBlocksPerCu = 16;
#define hbm_write sweep_write<4, false, true>
#define hbm_verify sweep_verify<4, true, true>

template <int U, bool NT, bool CH>
float time_pair(uint4* buf, uint64_t n, int blocks, unsigned long long* err, int reps, float* t_read) {
  hipEvent_t a, b, c;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventCreate(&c);
  float tw = 0, tr = 0;
  for (int r = 0; r < reps + 1; ++r) {  // first repetition is warm-up
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((sweep_write<U, NT, CH>), dim3(blocks), dim3(256), 0, 0, buf, n, 9u + r);
    (void)hipEventRecord(b, 0);
    hipLaunchKernelGGL((sweep_verify<U, NT, CH>), dim3(blocks), dim3(256), 0, 0, buf, n, 9u + r, err);
    (void)hipEventRecord(c, 0);
    (void)hipEventSynchronize(c);
    float x = 0, y = 0;
    (void)hipEventElapsedTime(&x, a, b);
    (void)hipEventElapsedTime(&y, b, c);
    if (r) {
      tw += x;
      tr += y;
    }
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipEventDestroy(c);
  *t_read = tr / reps;
  return tw / reps;
}

}  // namespace

extern "C" {

struct amdgpu_canary_result {
  int ok;
  int device;
  unsigned long long hbm_bytes;
  unsigned long long hbm_errors;
  unsigned long long mfma_errors;
  double write_gbps;
  double read_gbps;
  double mfma_tflops;
  double elapsed_ms;
  int num_cus;
  char arch[64];
  char error[256];
};

int amdgpu_canary_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -1;
  return n;
}

#define CANARY_CHECK(expr)                                                                   \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) {                                                                  \
      std::snprintf(out->error, sizeof(out->error), "%s: %s", #expr, hipGetErrorString(e_)); \
      goto done;                                                                             \
    }                                                                                        \
  } while (0)

// hbm_bytes: size of the pattern buffer (rounded down to 16 B); passes: timed
// write+verify repetitions; mfma_iters: MFMA pairs per wave for the rate test.
int amdgpu_canary_run(int device, unsigned long long hbm_bytes, int passes, int mfma_iters,
                      amdgpu_canary_result* out) {
  std::memset(out, 0, sizeof(*out));
  out->device = device;
  uint4* buf = nullptr;
  unsigned long long* d_err = nullptr;
  float* sink = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
  hipDeviceProp_t prop;
  const uint64_t n = hbm_bytes / sizeof(uint4);
  unsigned long long h_err[2] = {0, 0};
  float t_write = 0, t_read = 0, t_mfma = 0;
  int blocks = 0;
  CANARY_CHECK(hipSetDevice(device));
  CANARY_CHECK(hipGetDeviceProperties(&prop, device));
  out->num_cus = prop.multiProcessorCount;
  std::snprintf(out->arch, sizeof(out->arch), "%s", prop.gcnArchName);
  out->hbm_bytes = n * sizeof(uint4);
  if (passes < 1) passes = 1;
  CANARY_CHECK(hipMalloc(&buf, n * sizeof(uint4) + 16));
  CANARY_CHECK(hipMalloc(&d_err, 2 * sizeof(unsigned long long)));
  CANARY_CHECK(hipMemset(d_err, 0, 2 * sizeof(unsigned long long)));
  CANARY_CHECK(hipEventCreate(&e0));
  CANARY_CHECK(hipEventCreate(&e1));
  CANARY_CHECK(hipEventCreate(&e2));
  blocks = prop.multiProcessorCount * kBlocksPerCu;  // >> #CUs
  // warm-up (first-touch page mapping) outside the timed region
  hipLaunchKernelGGL(hbm_write, dim3(blocks), dim3(256), 0, 0, buf, n, 0x1234u);
  CANARY_CHECK(hipGetLastError());
  CANARY_CHECK(hipDeviceSynchronize());
  for (int p = 0; p < passes; ++p) {
    const uint32_t seed = 0xA5A5u + p;
    float tw = 0, tr = 0;
    CANARY_CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(hbm_write, dim3(blocks), dim3(256), 0, 0, buf, n, seed);
    CANARY_CHECK(hipEventRecord(e1, 0));
    hipLaunchKernelGGL(hbm_verify, dim3(blocks), dim3(256), 0, 0, buf, n, seed, d_err);
    CANARY_CHECK(hipEventRecord(e2, 0));
    CANARY_CHECK(hipEventSynchronize(e2));
    CANARY_CHECK(hipGetLastError());
    CANARY_CHECK(hipEventElapsedTime(&tw, e0, e1));
    CANARY_CHECK(hipEventElapsedTime(&tr, e1, e2));
    t_write += tw;
    t_read += tr;
  }
  // MFMA exactness: 2 * #CUs single-wave blocks, K = 16 * 32
  hipLaunchKernelGGL(mfma_exact, dim3(prop.multiProcessorCount * 2), dim3(64), 0, 0, 32, 0, d_err + 1);
  CANARY_CHECK(hipGetLastError());
  // MFMA rate
  CANARY_CHECK(hipMalloc(&sink, static_cast<size_t>(prop.multiProcessorCount) * 8 * 256 * sizeof(float)));
  hipLaunchKernelGGL(mfma_rate, dim3(prop.multiProcessorCount * 8), dim3(256), 0, 0, 16, sink);  // warm-up
  CANARY_CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(mfma_rate, dim3(prop.multiProcessorCount * 8), dim3(256), 0, 0, mfma_iters, sink);
  CANARY_CHECK(hipEventRecord(e1, 0));
  CANARY_CHECK(hipEventSynchronize(e1));
  CANARY_CHECK(hipGetLastError());
  CANARY_CHECK(hipEventElapsedTime(&t_mfma, e0, e1));
  CANARY_CHECK(hipMemcpy(h_err, d_err, sizeof(h_err), hipMemcpyDeviceToHost));
  out->hbm_errors = h_err[0];
  out->mfma_errors = h_err[1];
  out->write_gbps = static_cast<double>(n) * sizeof(uint4) * passes / (t_write * 1e-3) / 1e9;
  out->read_gbps = static_cast<double>(n) * sizeof(uint4) * passes / (t_read * 1e-3) / 1e9;
  {
    const double flops = 2.0 * 32 * 32 * 16 * 2.0 /*chains*/ * mfma_iters * (prop.multiProcessorCount * 8.0 * 4 /*waves*/);
    out->mfma_tflops = flops / (t_mfma * 1e-3) / 1e12;
  }
  out->elapsed_ms = t_write + t_read + t_mfma;
  out->ok = (out->hbm_errors == 0 && out->mfma_errors == 0) ? 1 : 0;
done:
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (e2) (void)hipEventDestroy(e2);
  if (sink) (void)hipFree(sink);
  if (d_err) (void)hipFree(d_err);
  if (buf) (void)hipFree(buf);
  return out->error[0] ? -1 : 0;
}

// Fault-injection self-check of the HBM verifier: writes the pattern, corrupts
// `flips` 4-byte words at spread-out offsets behind the kernel's back (hipMemcpy), and
// returns how many mismatching words the verify kernel reports (expected == flips).
long long amdgpu_canary_detects_corruption(int device, unsigned long long hbm_bytes, int flips) {
  uint4* buf = nullptr;
  unsigned long long* d_err = nullptr;
  unsigned long long h_err = 0;
  const uint64_t n = hbm_bytes / sizeof(uint4);
  hipDeviceProp_t prop;
  if (n == 0 || flips < 0 || hipSetDevice(device) != hipSuccess ||
      hipGetDeviceProperties(&prop, device) != hipSuccess)
    return -1;
  const int blocks = prop.multiProcessorCount * kBlocksPerCu;
  long long rc = -1;
  if (hipMalloc(&buf, n * sizeof(uint4)) == hipSuccess && hipMalloc(&d_err, sizeof(h_err)) == hipSuccess &&
      hipMemset(d_err, 0, sizeof(h_err)) == hipSuccess) {
    hipLaunchKernelGGL(hbm_write, dim3(blocks), dim3(256), 0, 0, buf, n, 77u);
    bool ok = hipDeviceSynchronize() == hipSuccess;
    for (int f = 0; ok && f < flips; ++f) {
      const uint64_t word = (static_cast<uint64_t>(f) * 2654435761ull) % n;
      const uint32_t junk = 0xDEADBEEFu ^ static_cast<uint32_t>(f);
      ok = hipMemcpy(reinterpret_cast<char*>(buf + word) + 4 * (f & 3), &junk, 4, hipMemcpyHostToDevice) ==
           hipSuccess;
    }
    if (ok) {
      hipLaunchKernelGGL(hbm_verify, dim3(blocks), dim3(256), 0, 0, buf, n, 77u, d_err);
      if (hipDeviceSynchronize() == hipSuccess &&
          hipMemcpy(&h_err, d_err, sizeof(h_err), hipMemcpyDeviceToHost) == hipSuccess)
        rc = static_cast<long long>(h_err);
    }
  }
  if (d_err) (void)hipFree(d_err);
  if (buf) (void)hipFree(buf);
  return rc;
}

// Fault-injection check of the MFMA verifier: `inject_blocks` of the 2 * #CUs exactness
// blocks compute with one perturbed operand.  Returns the mismatching accumulator
// registers found (0 expected without injection), -1 on a HIP error.
long long amdgpu_canary_mfma_detects(int device, int inject_blocks) {
  unsigned long long* d_err = nullptr;
  unsigned long long h_err = 0;
  hipDeviceProp_t prop;
  if (inject_blocks < 0 || hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess)
    return -1;
  long long rc = -1;
  if (hipMalloc(&d_err, sizeof(h_err)) == hipSuccess && hipMemset(d_err, 0, sizeof(h_err)) == hipSuccess) {
    hipLaunchKernelGGL(mfma_exact, dim3(prop.multiProcessorCount * 2), dim3(64), 0, 0, 32, inject_blocks, d_err);
    if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(&h_err, d_err, sizeof(h_err), hipMemcpyDeviceToHost) == hipSuccess)
      rc = static_cast<long long>(h_err);
  }
  if (d_err) (void)hipFree(d_err);
  return rc;
}

// Host wrapper for the numerics test: inputs/outputs in host memory.
int amdgpu_canary_mfma_gemm(int device, const unsigned short* a_host, const unsigned short* b_host, float* c_host,
                            int M, int N, int K, char* err, int err_len) {
  if (M <= 0 || N <= 0 || K <= 0 || M % 32 || N % 32 || K % 16) {
    std::snprintf(err, err_len, "shape (%d,%d,%d) must be M,N %% 32 == 0 and K %% 16 == 0", M, N, K);
    return -1;
  }
  short *a = nullptr, *b = nullptr;
  float* c = nullptr;
  hipError_t e = hipSetDevice(device);
  const size_t sa = static_cast<size_t>(M) * K * 2, sb = static_cast<size_t>(K) * N * 2,
               sc = static_cast<size_t>(M) * N * 4;
  if (e == hipSuccess) e = hipMalloc(&a, sa);
  if (e == hipSuccess) e = hipMalloc(&b, sb);
  if (e == hipSuccess) e = hipMalloc(&c, sc);
  if (e == hipSuccess) e = hipMemcpy(a, a_host, sa, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(b, b_host, sb, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(mfma_gemm, dim3(N / 32, M / 32), dim3(64), 0, 0, a, b, c, M, N, K);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(c_host, c, sc, hipMemcpyDeviceToHost);
  if (e != hipSuccess) std::snprintf(err, err_len, "%s", hipGetErrorString(e));
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  if (c) (void)hipFree(c);
  return e == hipSuccess ? 0 : -1;
}

// variant: 0 U4 grid-stride, 1 U8 grid-stride, 2 U4 NT, 3 U8 NT, 4 U4 chunked, 5 U8 chunked,
// 6 U4 NT chunked, 7 U16 grid-stride.  blocks_per_cu scales the grid.
int amdgpu_canary_hbm_sweep(int device, unsigned long long bytes, int variant, int blocks_per_cu, int reps,
                            double* write_gbps, double* read_gbps, unsigned long long* errors) {
  hipDeviceProp_t prop;
  if (hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess) return -1;
  const uint64_t n = bytes / sizeof(uint4);
  uint4* buf = nullptr;
  unsigned long long* err = nullptr;
  if (hipMalloc(&buf, n * sizeof(uint4)) != hipSuccess) return -2;
  if (hipMalloc(&err, 8) != hipSuccess || hipMemset(err, 0, 8) != hipSuccess) {
    (void)hipFree(buf);
    return -2;
  }
  const int blocks = prop.multiProcessorCount * (blocks_per_cu > 0 ? blocks_per_cu : 8);
  float tw = 0, tr = 0;
  switch (variant) {
    case 0: tw = time_pair<4, false, false>(buf, n, blocks, err, reps, &tr); break;
    case 1: tw = time_pair<8, false, false>(buf, n, blocks, err, reps, &tr); break;
    case 2: tw = time_pair<4, true, false>(buf, n, blocks, err, reps, &tr); break;
    case 3: tw = time_pair<8, true, false>(buf, n, blocks, err, reps, &tr); break;
    case 4: tw = time_pair<4, false, true>(buf, n, blocks, err, reps, &tr); break;
    case 5: tw = time_pair<8, false, true>(buf, n, blocks, err, reps, &tr); break;
    case 6: tw = time_pair<4, true, true>(buf, n, blocks, err, reps, &tr); break;
    case 7: tw = time_pair<16, false, false>(buf, n, blocks, err, reps, &tr); break;
    default: break;
  }
  const hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(errors, err, 8, hipMemcpyDeviceToHost);
  *write_gbps = tw > 0 ? n * 16.0 / (tw * 1e-3) / 1e9 : 0;
  *read_gbps = tr > 0 ? n * 16.0 / (tr * 1e-3) / 1e9 : 0;
  (void)hipFree(err);
  (void)hipFree(buf);
  return e == hipSuccess ? 0 : -3;
}

}  // extern "C"
