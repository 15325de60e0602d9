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
//   4. Matrix path       - LDS-staged MFMA GEMM on exact integer data, ABFT-checked.
//   5. fp8 / bf8 / fp4 MFMA exactness and rate, LDS march (datapath.hip).
//
// C ABI for ctypes (k8s_gpu_device_plugin_amd/ops/canary.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "canary_common.h"

namespace {

using namespace canary;

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

__device__ __forceinline__ short bf16_of_int(int v) {
  const float f = static_cast<float>(v);
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return static_cast<short>(u >> 16);  // exact for small integers
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

// ---- LDS-staged MFMA GEMM: the matrix path a real workload takes --------------------
// C[MxN] (fp32) = A[MxK] * B, A row-major bf16, B given transposed (Bt[NxK] row-major,
// so both operands are K-contiguous).  A 128x128 block tile, BK = 64, 4 waves as 2x2,
// each wave 64x64 = 2x2 v_mfma_f32_32x32x16_bf16 tiles (64 accumulator registers).
// Operands stream HBM -> LDS with global_load_lds (16 B per lane, no VGPR round trip),
// double-buffered so tile t+1 lands while tile t is multiplied; fragments come out of
// LDS with one ds_read_b128 per operand per k-step.  Blocks are remapped XCD-aware so
// the tiles that share A rows share an XCD's L2.  Integer-valued operands make every
// result exact, so an ABFT row/column checksum (below) verifies the whole path - HBM,
// L2, the LDS DMA, LDS reads and the matrix cores - not just the MFMA unit.
constexpr int kTileM = 128, kTileN = 128, kTileK = 64;
constexpr int kTileBytes = kTileM * kTileK * 2;  // one operand tile, 16 KiB
typedef __attribute__((address_space(3))) void* lds_void_ptr;

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {  // bijective for any nwg
  const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__global__ void __launch_bounds__(256) gemm_lds(const short* __restrict__ A, const short* __restrict__ Bt,
                                               float* __restrict__ C, int M, int N, int K) {
  // one __shared__ array for everything (a second object can de-pipeline glds waits)
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * kTileBytes];  // [buf][A|B][128][64] bf16
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nbn = N / kTileN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / nbn) * kTileM, n0 = (wg % nbn) * kTileN;
  if (m0 + kTileM > M || n0 + kTileN > N) return;  // host checks shapes
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 31, h = lane >> 5;

  // staging: wave w issues 4 x 1 KiB per operand = rows (4w+i)*8 .. +7; lane l lands at
  // physical 16 B chunk l&7 of row l>>3.  LDS rows are 128 B, so the 16 lanes of one
  // ds_read_b128 cycle (rows r..r+15, same k chunk) would hit 2 of the 16 bank slots of
  // a 256 B bank row (8-way conflict).  The image is swizzled as physical chunk =
  // logical chunk ^ ((row >> 1) & 7): row parity picks the 128 B half of the bank row
  // and (row >> 1) & 7 the slot in it, so 16 consecutive rows cover all 16 slots
  // (conflict-free; `chunk ^ (row & 7)` measured 2-way, SQ_LDS_BANK_CONFLICT).  The
  // swizzle is applied on the per-lane global source address, since the glds
  // destination must stay lane-linear.
  auto stage = [&](int t, int buf) {
    const int k0 = t * kTileK;
    char* base = smem + buf * 2 * kTileBytes;
    for (int i = 0; i < 4; ++i) {
      const int row = (wave * 4 + i) * 8 + (lane >> 3), kc = ((lane & 7) ^ ((row >> 1) & 7)) * 8;
      __builtin_amdgcn_global_load_lds(A + static_cast<size_t>(m0 + row) * K + k0 + kc,
                                       (lds_void_ptr)(base + (wave * 4 + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(Bt + static_cast<size_t>(n0 + row) * K + k0 + kc,
                                       (lds_void_ptr)(base + kTileBytes + (wave * 4 + i) * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int T = K / kTileK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    if (t + 1 < T) stage(t + 1, cur ^ 1);
    const short* As = reinterpret_cast<const short*>(smem + cur * 2 * kTileBytes);
    const short* Bs = As + kTileM * kTileK;
#pragma unroll
    for (int kk = 0; kk < kTileK / 16; ++kk) {
      const int chunk = 2 * kk + h;  // logical 16 B chunk of this lane's 8 k values
      bf16x8 a[2], b[2];
      for (int i = 0; i < 2; ++i) {
        const int row = wr * 64 + i * 32 + r;
        a[i] = *reinterpret_cast<const bf16x8*>(As + row * kTileK + ((chunk ^ ((row >> 1) & 7)) << 3));
      }
      for (int j = 0; j < 2; ++j) {
        const int row = wc * 64 + j * 32 + r;
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + row * kTileK + ((chunk ^ ((row >> 1) & 7)) << 3));
      }
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 has landed
    __syncthreads();                                   // ... and nobody still reads tile t's buffer
  }
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        C[static_cast<size_t>(row) * N + n0 + wc * 64 + j * 32 + r] = acc[i][j][e];
      }
}

// ---- 256x256-tile GEMM, two wave groups in ping-pong: the fast matrix path ------------
// Same contract as gemm_lds (A [MxK], Bt [NxK] bf16, fp32 C), M, N % 256 == 0, K % 64 == 0.
// 8 waves = 2 groups (wr) x 4 (wc); a wave owns 128x64 of C as 2 halves x 4x4 tiles of
// v_mfma_f32_16x16x32_bf16 (128 accumulator registers).  Per K-tile (BK = 64) a wave runs
// four sections, each closed by a raw s_barrier:
//   L0: ds_read A half 0 + all of B (16 x b128)   M0: 32 MFMA into half 0
//   L1: ds_read A half 1 (8 x b128)               M1: 32 MFMA into half 1
// Group 1 executes one extra barrier first, so it runs one barrier interval behind group
// 0.  Waves w and w+4 share a SIMD, hence on every SIMD one wave is in an MFMA section
// while its partner reads LDS: the MFMA pipe does not wait for fragment loads.
// Operands stream in with global_load_lds into 2 LDS buffers (2 x 64 KiB, 1 block/CU).
// Interval i (between barriers i and i+1) holds group 0's section i and group 1's
// section i-1.  Tile t lives in buffer t&1 and is read in intervals 4t..4t+3; tile t+2
// is issued by both groups in interval 4t+4 (right after the barrier that ends the last
// read of tile t) and each wave retires its own copies with s_waitcnt vmcnt(0) before
// barrier 4t+8, which precedes the first read of tile t+2.  The DMA therefore stays in
// flight across three barriers (__syncthreads would drain it at each: vmcnt(0)).
// Write-after-read is covered by every reading section ending in lgkmcnt(0) before its
// barrier.  Row swizzle as in gemm_lds (chunk ^ ((row >> 1) & 7)): conflict-free for the
// 16x16x32 lane groups too.  Tiles are rastered in groups of 4 tile rows, so one XCD's
// consecutive workgroups share 4 A panels and a run of B panels in their L2.
constexpr int kBT = 256, kBK = 64;
constexpr int kBOp = kBT * kBK * 2;  // one operand tile, 32 KiB
constexpr int kBStage = 2 * kBOp;    // A + B of one K-tile, 64 KiB
using f32x4 = __attribute__((ext_vector_type(4))) float;

// Output tile of this workgroup: XCD-aware bijective remap, then tiles rastered in groups
// of `group` tile rows so one XCD's consecutive workgroups share A and B panels in L2.
__device__ __forceinline__ void tile_origin256(int M, int N, int group, int* m0, int* n0) {
  const int nbm = M / kBT, nbn = N / kBT;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = group * nbn, first_m = (wg / per_group) * group;
  const int gm = nbm - first_m < group ? nbm - first_m : group;
  *m0 = (first_m + (wg % per_group) % gm) * kBT;
  *n0 = ((wg % per_group) / gm) * kBT;
}

__device__ __forceinline__ void section_end() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this section's LDS reads are done
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);  // nothing crosses a section boundary
}

__global__ void __launch_bounds__(512) gemm256(const short* __restrict__ A, const short* __restrict__ Bt,
                                              float* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBStage];  // the only LDS object
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int m0, n0;
  tile_origin256(M, N, 4, &m0, &n0);
  if (m0 + kBT > M || n0 + kBT > N) return;  // host checks shapes (block-uniform exit)
  const int wr = wave >> 2, wc = wave & 3;
  const bool g1 = wr == 1;
  const int r16 = lane & 15, q = lane >> 4;

  auto stage = [&](int t) {  // 8 x 1 KiB pieces per wave: rows (4w+i)*8 .. +7 of A and of B
    const int k0 = t * kBK;
    char* base = smem + (t & 1) * kBStage;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (wave * 4 + i) * 8 + (lane >> 3), kc = ((lane & 7) ^ ((row >> 1) & 7)) * 8;
      __builtin_amdgcn_global_load_lds(A + static_cast<size_t>(m0 + row) * K + k0 + kc,
                                       (lds_void_ptr)(base + (wave * 4 + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(Bt + static_cast<size_t>(n0 + row) * K + k0 + kc,
                                       (lds_void_ptr)(base + kBOp + (wave * 4 + i) * 1024), 16, 0, 0);
    }
  };
  auto frag = [&](const short* S, int row, int chunk) {
    return *reinterpret_cast<const bf16x8*>(S + row * kBK + ((chunk ^ ((row >> 1) & 7)) << 3));
  };

  f32x4 acc[2][4][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4][2], b[4][2];

  const int T = K / kBK;
  stage(0);
  if (T > 1) {
    stage(1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 landed; tile 1 may fly on
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  section_end();
  if (g1) section_end();  // the one-interval stagger

  for (int t = 0; t < T; ++t) {
    const short* As = reinterpret_cast<const short*>(smem + (t & 1) * kBStage);
    const short* Bs = As + kBT * kBK;
    // L0
    if (!g1 && t >= 1 && t + 1 < T) stage(t + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j][s] = frag(Bs, wc * 64 + j * 16 + r16, 4 * s + q);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i][s] = frag(As, wr * 128 + i * 16 + r16, 4 * s + q);
    section_end();
    // M0
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s], b[j][s], acc[0][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    section_end();
    // L1
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i][s] = frag(As, wr * 128 + 64 + i * 16 + r16, 4 * s + q);
    if (g1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 (issued in interval 4t)
    section_end();
    // M1
    if (g1 && t + 2 < T) stage(t + 2);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s], b[j][s], acc[1][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (!g1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 (issued in interval 4t)
    section_end();
  }
  if (!g1) section_end();  // both groups pass the same number of barriers

#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wr * 128 + h * 64 + i * 16 + q * 4 + e;
          C[static_cast<size_t>(row) * N + n0 + wc * 64 + j * 16 + r16] = acc[h][i][j][e];
        }
}

// ---- gemm256 with region-wise staging: the DMA issued from LDS-read sections ----------
// gemm256 issues all eight 1 KiB pieces of a wave in one section, and a piece costs
// ~60-185 issue cycles (MI355X_MICROARCH.md, LDS-DMA piece row), so that section runs
// about twice as long as the others.  Here a tile's regions are refilled as soon as they
// are free: B and the A rows every wave reads in L0 ("A-h0": rows 0-63 and 128-191) are
// last read in interval 4t+1, so their refill for tile t+2 (6 pieces per wave) is issued
// in L(t,1); the A-h1 rows are last read in interval 4t+3, so theirs (2 pieces) is issued
// in L(t+1,0).  All DMA sits in L sections (which are shorter than the partner wave's
// MFMA section), and a tile is retired with vmcnt(6) before barrier 4t+8: the next
// tile's six younger pieces stay in flight.  Measured (4096^3 / 8192^3, integer data):
// 1254-1264 / 1308-1314 TFLOP/s vs gemm256's 1069-1084 / 1078-1090.
// kBEarly of a wave's 4 B pieces of tile t+2 go with its A-h0 pieces in L(t,1), the rest
// with the A-h1 pieces in L(t+1,0): the split balances DMA issue between the two L
// sections (L0 also carries twice L1's ds_reads).
// kG1Early: group 1 issues each refill from the MFMA section one interval earlier (the
// first interval its region is free) instead of from its next LDS-read section.
// kScalarWave: the wave index goes through readfirstlane, so everything derived from it
// (LDS piece addresses -> M0, group branches) is scalar instead of per-lane.
// kGroupM: tile rows per raster group; kPrio: raise wave priority around MFMA sections.
template <int kBEarly, bool kG1Early = false, bool kScalarWave = true, int kGroupM = 4, bool kPrio = true>
__global__ void __launch_bounds__(512) gemm256s(const short* __restrict__ A, const short* __restrict__ Bt,
                                               float* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBStage];  // the only LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = kScalarWave ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  int m0, n0;
  tile_origin256(M, N, kGroupM, &m0, &n0);
  if (m0 + kBT > M || n0 + kBT > N) return;  // host checks shapes (block-uniform exit)
  const int wr = wave >> 2, wc = wave & 3;
  const bool g1 = wr == 1;
  const int r16 = lane & 15, q = lane >> 4;

  // piece p = rows 8p .. 8p+7 of one operand (1 KiB, 128 B rows, swizzled source)
  auto piece = [&](const short* src, int r0, char* base, int p, int k0) {
    const int row = p * 8 + (lane >> 3), kc = ((lane & 7) ^ ((row >> 1) & 7)) * 8;
    __builtin_amdgcn_global_load_lds(src + static_cast<size_t>(r0 + row) * K + k0 + kc, (lds_void_ptr)(base + p * 1024),
                                     16, 0, 0);
  };
  // A-h0 pieces are 0-7 and 16-23, A-h1 pieces 8-15 and 24-31; wave w owns list entries 2w, 2w+1
  auto a_piece = [](int k, int half) { return (k < 8 ? k : k + 8) + 8 * half; };
  auto stage_b_ah0 = [&](int t) {  // kBEarly B + 2 A-h0 pieces
    char* base = smem + (t & 1) * kBStage;
#pragma unroll
    for (int i = 0; i < kBEarly; ++i) piece(Bt, n0, base + kBOp, wave * 4 + i, t * kBK);
#pragma unroll
    for (int i = 0; i < 2; ++i) piece(A, m0, base, a_piece(wave * 2 + i, 0), t * kBK);
  };
  auto stage_ah1 = [&](int t) {  // 4 - kBEarly B + 2 A-h1 pieces
    char* base = smem + (t & 1) * kBStage;
#pragma unroll
    for (int i = kBEarly; i < 4; ++i) piece(Bt, n0, base + kBOp, wave * 4 + i, t * kBK);
#pragma unroll
    for (int i = 0; i < 2; ++i) piece(A, m0, base, a_piece(wave * 2 + i, 1), t * kBK);
  };
  auto frag = [&](const short* S, int row, int chunk) {
    return *reinterpret_cast<const bf16x8*>(S + row * kBK + ((chunk ^ ((row >> 1) & 7)) << 3));
  };
  auto retire = [&](int t) {  // tile t+1 landed; tile t+2's 2 + kBEarly pieces may fly on
    if (t + 2 >= K / kBK)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (kBEarly == 4)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (kBEarly == 3)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if constexpr (kBEarly == 2)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (kBEarly == 1)
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  };

  f32x4 acc[2][4][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4][2], b[4][2];

  const int T = K / kBK;
  stage_b_ah0(0);
  stage_ah1(0);
  if (T > 1) {
    stage_b_ah0(1);
    stage_ah1(1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 landed; tile 1 may fly on
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  section_end();
  if (g1) section_end();  // the one-interval stagger

  for (int t = 0; t < T; ++t) {
    const short* As = reinterpret_cast<const short*>(smem + (t & 1) * kBStage);
    const short* Bs = As + kBT * kBK;
    // L0
    if ((!kG1Early || !g1) && t >= 1 && t + 1 < T) stage_ah1(t + 1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j][s2] = frag(Bs, wc * 64 + j * 16 + r16, 4 * s2 + q);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i][s2] = frag(As, wr * 128 + i * 16 + r16, 4 * s2 + q);
    section_end();
    // M0
    if (kG1Early && g1 && t + 2 < T) stage_b_ah0(t + 2);
    if constexpr (kPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], b[j][s2], acc[0][i][j], 0, 0, 0);
    if constexpr (kPrio) __builtin_amdgcn_s_setprio(0);
    section_end();
    // L1
    if ((!kG1Early || !g1) && t + 2 < T) stage_b_ah0(t + 2);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i][s2] = frag(As, wr * 128 + 64 + i * 16 + r16, 4 * s2 + q);
    if (g1) retire(t);
    section_end();
    // M1
    if (kG1Early && g1 && t + 2 < T) stage_ah1(t + 2);
    if constexpr (kPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], b[j][s2], acc[1][i][j], 0, 0, 0);
    if constexpr (kPrio) __builtin_amdgcn_s_setprio(0);
    if (!g1) retire(t);
    section_end();
  }
  if (!g1) section_end();  // both groups pass the same number of barriers

  // Epilogue through LDS: after the last barrier no wave reads a staging buffer and no DMA
  // is in flight, so each wave turns its 64x64 fp32 half-outputs into whole rows in a
  // 16 KiB region of its own (8 x 16 KiB = the whole 128 KiB; 256 B rows: a ds_write_b32
  // is 2-way, which costs nothing on that instruction, and the b128 read-back is
  // conflict-free) and stores them with dwordx4: 16 row-contiguous stores of 4 rows x
  // 256 B per half instead of 64 column-scattered dword stores.
  static_assert(8 * 64 * 64 * 4 <= 2 * kBStage, "epilogue regions fit the staging LDS");
  float* region = reinterpret_cast<float*>(smem + wave * (64 * 64 * 4));
  constexpr int kLd = 64;  // floats per row
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) region[(i * 16 + q * 4 + e) * kLd + j * 16 + r16] = acc[h][i][j][e];
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const int row = p * 4 + (lane >> 4), c4 = (lane & 15) * 4;
      const float4 v = *reinterpret_cast<const float4*>(region + row * kLd + c4);
      *reinterpret_cast<float4*>(C + static_cast<size_t>(m0 + wr * 128 + h * 64 + row) * N + n0 + wc * 64 + c4) = v;
    }
  }
}

// Integer operands in [-4, 4] (exact in bf16): element (i, k) of operand `which`.
__global__ void __launch_bounds__(256) gemm_fill(short* __restrict__ X, int rows, int K, uint32_t which) {
  const size_t n = static_cast<size_t>(rows) * K;
  for (size_t e = blockIdx.x * 256ull + threadIdx.x; e < n; e += static_cast<size_t>(gridDim.x) * 256)
    X[e] = bf16_of_int(small_int((static_cast<uint64_t>(which) << 56) ^ e));
}

// Uniform random bf16 in [-1, 1) (rate measurement on data with full mantissas: the
// clock the chip holds under MFMA load depends on operand bit activity).
__global__ void __launch_bounds__(256) gemm_fill_random(short* __restrict__ X, int rows, int K, uint32_t which) {
  const size_t n = static_cast<size_t>(rows) * K;
  for (size_t e = blockIdx.x * 256ull + threadIdx.x; e < n; e += static_cast<size_t>(gridDim.x) * 256) {
    const float f = static_cast<float>(mix32((static_cast<uint64_t>(which) << 56) ^ e) >> 8) * (2.0f / 16777216.0f) - 1.0f;
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    X[e] = static_cast<short>(u >> 16);
  }
}

__device__ __forceinline__ int bf16_to_int(short v) {
  const uint32_t u = static_cast<uint32_t>(static_cast<uint16_t>(v)) << 16;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return static_cast<int>(f);
}

// colsum[k] += sum over a 64-row slab of X[row][k]: threads over k (coalesced), blocks
// over (k range, row slab) so the whole chip takes part; out must be zeroed.  Two's-
// complement wrap-around makes the unsigned atomic add a signed one.
constexpr int kSlab = 64;
__global__ void __launch_bounds__(256) gemm_colsum(const short* __restrict__ X, int rows, int K,
                                                   long long* __restrict__ out) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  const int r0 = blockIdx.y * kSlab, r1 = r0 + kSlab < rows ? r0 + kSlab : rows;
  long long s = 0;
  for (int i = r0; i < r1; ++i) s += bf16_to_int(X[static_cast<size_t>(i) * K + k]);
  atomicAdd(reinterpret_cast<unsigned long long*>(out + k), static_cast<unsigned long long>(s));
}

// ABFT: for row i, sum_n C[i][n] must equal sum_k A[i][k] * (sum_n Bt[n][k]); for column
// n, sum_m C[m][n] must equal sum_k (sum_m A[m][k]) * Bt[n][k].  One block per row /
// column, int64 reductions (C holds exact integers).  mode 0 = rows, 1 = columns.
__global__ void __launch_bounds__(256) gemm_abft(const short* __restrict__ X, const float* __restrict__ C,
                                                 const long long* __restrict__ other_sum, int M, int N, int K,
                                                 int mode, unsigned long long* __restrict__ errors) {
  __shared__ long long red[2][256];
  const int idx = blockIdx.x, tid = threadIdx.x;
  long long expect = 0, got = 0;
  for (int k = tid; k < K; k += 256) expect += static_cast<long long>(bf16_to_int(X[static_cast<size_t>(idx) * K + k])) * other_sum[k];
  if (mode == 0)
    for (int n = tid; n < N; n += 256) got += static_cast<long long>(C[static_cast<size_t>(idx) * N + n]);
  else
    for (int m = tid; m < M; m += 256) got += static_cast<long long>(C[static_cast<size_t>(m) * N + idx]);
  red[0][tid] = expect;
  red[1][tid] = got;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      red[0][tid] += red[0][tid + s];
      red[1][tid] += red[1][tid + s];
    }
    __syncthreads();
  }
  if (tid == 0 && red[0][0] != red[1][0]) atomicAdd(errors, 1ull);
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

// Tile-stride: block b streams tiles b, b + G, b + 2G, ... of 256 * UNROLL contiguous
// 16 B elements, so every wave reads whole contiguous runs (like CHUNKED) while the grid
// sweeps the buffer front to back together (like grid-stride): no per-block tail.
template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) tile_write(uint4* __restrict__ buf, uint64_t n, uint32_t seed) {
  const uint64_t tile = 256ull * UNROLL;
  for (uint64_t t0 = blockIdx.x * tile; t0 < n; t0 += static_cast<uint64_t>(gridDim.x) * tile) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t i = t0 + u * 256ull + threadIdx.x;
      if (i < n) {
        const uint4 v = pattern(i, seed);
        if (NT) nt_store(v, buf + i);
        else buf[i] = v;
      }
    }
  }
}

template <int UNROLL, bool NT>
__global__ void __launch_bounds__(256) tile_verify(const uint4* __restrict__ buf, uint64_t n, uint32_t seed,
                                                   unsigned long long* __restrict__ errors) {
  const uint64_t tile = 256ull * UNROLL;
  uint32_t bad = 0;
  for (uint64_t t0 = blockIdx.x * tile; t0 < n; t0 += static_cast<uint64_t>(gridDim.x) * tile) {
    if (t0 + tile <= n) {
      uint4 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const uint64_t i = t0 + u * 256ull + threadIdx.x;
        v[u] = NT ? nt_load(buf + i) : buf[i];
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) bad += diff(v[u], pattern(t0 + u * 256ull + threadIdx.x, seed));
    } else {
      for (uint64_t i = t0 + threadIdx.x; i < n; i += 256) bad += diff(buf[i], pattern(i, seed));
    }
  }
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

template <int U, bool NT>
float time_tile(uint4* buf, uint64_t n, int blocks, unsigned long long* err, int reps, float* t_read) {
  hipEvent_t a, b, c;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventCreate(&c);
  float tw = 0, tr = 0;
  for (int r = 0; r < reps + 1; ++r) {  // first repetition is warm-up
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((tile_write<U, false>), dim3(blocks), dim3(256), 0, 0, buf, n, 9u + r);
    (void)hipEventRecord(b, 0);
    hipLaunchKernelGGL((tile_verify<U, NT>), dim3(blocks), dim3(256), 0, 0, buf, n, 9u + r, err);
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

// Shapes picked from the on-hardware sweep (profiles/hbm_sweep_gpu.json, 4 GiB buffer):
// writes: block-contiguous chunks, plain stores (~6.0 TB/s); verify: block-contiguous
// chunks, non-temporal loads (~6.8 TB/s), both at 16 blocks of 256 threads per CU.
// Re-swept at the canary's 1 GiB (profiles/r2/hbm_sweep_session4.json): behind plain
// stores the verify measures ~5.9 TB/s, since it also pays for the write-back of the lines
// the write phase left dirty in the caches; behind non-temporal stores it reads at 6.7 TB/s
// but the write drops to 5.6.  The write+verify pair takes the same time either way.
// Tile-stride (no per-block tail) was no faster than block-contiguous chunks.
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
  double gemm_tflops;                   // LDS-staged MFMA GEMM (matrix path) rate
  unsigned long long gemm_errors;       // ABFT row/column checksum mismatches
  double fp8_tflops;                    // block-scaled fp8 MFMA rate (datapath.hip)
  double fp4_tflops;                    // block-scaled fp4 MFMA rate
  unsigned long long lowp_errors;       // fp8 / bf8 / fp4 MFMA exactness mismatches
  unsigned long long lds_errors;        // LDS march mismatches
  unsigned long long lds_bytes;         // LDS bytes per workgroup the march covered
};

struct amdgpu_canary_datapath_result {  // datapath.hip
  double fp8_tflops;
  double fp4_tflops;
  unsigned long long lowp_errors;
  unsigned long long lds_errors;
  unsigned long long lds_bytes;
};
int amdgpu_canary_datapaths(int device, int iters, amdgpu_canary_datapath_result* out, char* err, int err_len);

int amdgpu_canary_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -1;
  return n;
}

int amdgpu_canary_gemm_rate(int device, int M, int N, int K, int iters, int inject, int kernel, double* tflops,
                            unsigned long long* errors, char* err, int err_len);

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
  // matrix path: HBM -> L2 -> LDS DMA -> ds_read -> MFMA, exact and checksummed.  4096^3
  // (256 tiles of 256x256: one per CU) takes ~0.5 ms; hbm_bytes < 256 MiB (fault-injection
  // runs) uses 1024^3 on the 128x128 kernel.
  {
    const int g = hbm_bytes >= (256ull << 20) ? 4096 : 1024;
    if (amdgpu_canary_gemm_rate(device, g, g, g, 4, 0, 0, &out->gemm_tflops, &out->gemm_errors, out->error,
                                sizeof(out->error)) != 0)
      goto done;
  }
  // low-precision datapaths (fp8 / bf8 / fp4 MFMA) and the LDS
  {
    amdgpu_canary_datapath_result dp;
    if (amdgpu_canary_datapaths(device, mfma_iters / 4 > 0 ? mfma_iters / 4 : 1, &dp, out->error,
                                sizeof(out->error)) != 0)
      goto done;
    out->fp8_tflops = dp.fp8_tflops;
    out->fp4_tflops = dp.fp4_tflops;
    out->lowp_errors = dp.lowp_errors;
    out->lds_errors = dp.lds_errors;
    out->lds_bytes = dp.lds_bytes;
  }
  out->ok = (out->hbm_errors == 0 && out->mfma_errors == 0 && out->gemm_errors == 0 && out->lowp_errors == 0 &&
             out->lds_errors == 0)
                ? 1
                : 0;
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

// GEMM kernel choice: 1 = gemm_lds (128x128 tiles), 2 = gemm256 (256x256 tiles, wave-group
// ping-pong), 3 = gemm256s (same, region-wise DMA from the LDS-read sections); 0 = gemm256s
// when the shape divides into 256x256 tiles and gives at least 256 of them (one per CU),
// else gemm_lds.  Returns 0 for a shape the kernel cannot take.
int pick_gemm(int M, int N, int K, int kernel) {
  if (M <= 0 || N <= 0 || K <= 0 || K % kTileK) return 0;
  const bool fits256 = M % kBT == 0 && N % kBT == 0, fits128 = M % kTileM == 0 && N % kTileN == 0;
  if (kernel >= 2 && kernel <= 11) return fits256 ? kernel : 0;
  if (kernel == 1) return fits128 ? 1 : 0;
  if (kernel != 0) return 0;
  if (fits256 && (M / kBT) * (N / kBT) >= 256) return 3;
  return fits128 ? 1 : 0;
}

void launch_gemm(int kind, const short* a, const short* b, float* c, int M, int N, int K) {
  const dim3 g256((M / kBT) * (N / kBT)), b256(512);
  if (kind == 3)
    hipLaunchKernelGGL(gemm256s<4>, g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 4)
    hipLaunchKernelGGL(gemm256s<2>, g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 5)
    hipLaunchKernelGGL(gemm256s<0>, g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 6)
    hipLaunchKernelGGL(gemm256s<3>, g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 7)
    hipLaunchKernelGGL((gemm256s<4, true>), g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 8)
    hipLaunchKernelGGL((gemm256s<4, false, false>), g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 9)
    hipLaunchKernelGGL((gemm256s<4, false, true, 2>), g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 10)
    hipLaunchKernelGGL((gemm256s<4, false, true, 8>), g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 11)
    hipLaunchKernelGGL((gemm256s<4, false, true, 4, false>), g256, b256, 0, 0, a, b, c, M, N, K);
  else if (kind == 2)
    hipLaunchKernelGGL(gemm256, dim3((M / kBT) * (N / kBT)), dim3(512), 0, 0, a, b, c, M, N, K);
  else
    hipLaunchKernelGGL(gemm_lds, dim3((M / kTileM) * (N / kTileN)), dim3(256), 0, 0, a, b, c, M, N, K);
}

// LDS-staged GEMM on host data (numerics test): A [MxK], Bt [NxK] bf16 row-major.
int amdgpu_canary_gemm(int device, const unsigned short* a_host, const unsigned short* bt_host, float* c_host, int M,
                       int N, int K, int kernel, char* err, int err_len) {
  const int kind = pick_gemm(M, N, K, kernel);
  if (kind == 0) {
    std::snprintf(err, err_len, "shape (%d,%d,%d) does not fit kernel %d (M,N %% 128 or 256, K %% 64)", M, N, K,
                  kernel);
    return -1;
  }
  short *a = nullptr, *b = nullptr;
  float* c = nullptr;
  hipError_t e = hipSetDevice(device);
  const size_t sa = static_cast<size_t>(M) * K * 2, sb = static_cast<size_t>(N) * K * 2,
               sc = static_cast<size_t>(M) * N * 4;
  if (e == hipSuccess) e = hipMalloc(&a, sa);
  if (e == hipSuccess) e = hipMalloc(&b, sb);
  if (e == hipSuccess) e = hipMalloc(&c, sc);
  if (e == hipSuccess) e = hipMemcpy(a, a_host, sa, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(b, bt_host, sb, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    launch_gemm(kind, a, b, c, M, N, K);
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

// Matrix-path canary: device-generated integer operands, `iters` timed GEMMs, then the
// ABFT row + column checksums of the result.  *tflops = dense bf16 rate achieved,
// *errors = rows + columns whose checksum is off (0 on a healthy partition).
// flags bit 0 corrupts one element of C before the check (verifier self-test); bit 1
// fills the operands with random bf16 in [-1, 1) instead and skips the (then inexact)
// checksums: the rate on full-mantissa data, comparable with a BLAS benchmark.
int amdgpu_canary_gemm_rate(int device, int M, int N, int K, int iters, int flags, int kernel, double* tflops,
                            unsigned long long* errors, char* err, int err_len) {
  const bool inject = flags & 1, random_data = flags & 2;
  *tflops = 0;
  *errors = 0;
  const int kind = pick_gemm(M, N, K, kernel);
  if (kind == 0 || K > 65536 || iters < 1) {
    std::snprintf(err, err_len, "shape (%d,%d,%d) does not fit kernel %d (M,N %% 128 or 256, K %% 64, K <= 65536)",
                  M, N, K, kernel);
    return -1;
  }
  short *a = nullptr, *b = nullptr;
  float* c = nullptr;
  long long *asum = nullptr, *bsum = nullptr;
  unsigned long long* d_err = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float ms = 0;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&a, static_cast<size_t>(M) * K * 2);
  if (e == hipSuccess) e = hipMalloc(&b, static_cast<size_t>(N) * K * 2);
  if (e == hipSuccess) e = hipMalloc(&c, static_cast<size_t>(M) * N * 4);
  if (e == hipSuccess) e = hipMalloc(&asum, static_cast<size_t>(K) * 8);
  if (e == hipSuccess) e = hipMalloc(&bsum, static_cast<size_t>(K) * 8);
  if (e == hipSuccess) e = hipMalloc(&d_err, 8);
  if (e == hipSuccess) e = hipMemset(d_err, 0, 8);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  if (e == hipSuccess) {
    if (random_data) {
      hipLaunchKernelGGL(gemm_fill_random, dim3(2048), dim3(256), 0, 0, a, M, K, 1u);
      hipLaunchKernelGGL(gemm_fill_random, dim3(2048), dim3(256), 0, 0, b, N, K, 2u);
    } else {
      hipLaunchKernelGGL(gemm_fill, dim3(2048), dim3(256), 0, 0, a, M, K, 1u);
      hipLaunchKernelGGL(gemm_fill, dim3(2048), dim3(256), 0, 0, b, N, K, 2u);
    }
    launch_gemm(kind, a, b, c, M, N, K);  // warm-up
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipEventRecord(e0, 0);
  for (int i = 0; e == hipSuccess && i < iters; ++i) launch_gemm(kind, a, b, c, M, N, K);
  if (e == hipSuccess) e = hipEventRecord(e1, 0);
  if (e == hipSuccess) e = hipEventSynchronize(e1);
  if (e == hipSuccess) e = hipGetLastError();
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  if (e == hipSuccess && inject) {
    const float junk = 12345.0f;
    e = hipMemcpy(c + static_cast<size_t>(M / 2) * N + N / 3, &junk, 4, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess && !random_data) {
    e = hipMemset(asum, 0, static_cast<size_t>(K) * 8);
    if (e == hipSuccess) e = hipMemset(bsum, 0, static_cast<size_t>(K) * 8);
    hipLaunchKernelGGL(gemm_colsum, dim3((K + 255) / 256, (M + kSlab - 1) / kSlab), dim3(256), 0, 0, a, M, K, asum);
    hipLaunchKernelGGL(gemm_colsum, dim3((K + 255) / 256, (N + kSlab - 1) / kSlab), dim3(256), 0, 0, b, N, K, bsum);
    hipLaunchKernelGGL(gemm_abft, dim3(M), dim3(256), 0, 0, a, c, bsum, M, N, K, 0, d_err);
    hipLaunchKernelGGL(gemm_abft, dim3(N), dim3(256), 0, 0, b, c, asum, M, N, K, 1, d_err);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(errors, d_err, 8, hipMemcpyDeviceToHost);
  if (e == hipSuccess && ms > 0) *tflops = 2.0 * M * N * K * iters / (ms * 1e-3) / 1e12;
  if (e != hipSuccess) std::snprintf(err, err_len, "%s", hipGetErrorString(e));
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (d_err) (void)hipFree(d_err);
  if (bsum) (void)hipFree(bsum);
  if (asum) (void)hipFree(asum);
  if (c) (void)hipFree(c);
  if (b) (void)hipFree(b);
  if (a) (void)hipFree(a);
  return e == hipSuccess ? 0 : -1;
}

// variant: 0 U4 grid-stride, 1 U8 grid-stride, 2 U4 NT, 3 U8 NT, 4 U4 chunked, 5 U8 chunked,
// 6 U4 NT chunked, 7 U16 grid-stride, 8 U8 NT chunked, 9 U2 NT chunked, 10 U4 tile-stride
// (NT verify), 11 U8 tile-stride (NT verify), 12 U8 tile-stride.  blocks_per_cu scales the grid.
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
    case 8: tw = time_pair<8, true, true>(buf, n, blocks, err, reps, &tr); break;
    case 9: tw = time_pair<2, true, true>(buf, n, blocks, err, reps, &tr); break;
    case 10: tw = time_tile<4, true>(buf, n, blocks, err, reps, &tr); break;
    case 11: tw = time_tile<8, true>(buf, n, blocks, err, reps, &tr); break;
    case 12: tw = time_tile<8, false>(buf, n, blocks, err, reps, &tr); break;
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
