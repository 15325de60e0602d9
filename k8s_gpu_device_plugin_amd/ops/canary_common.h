// Helpers shared by the gfx950 canary sources (canary.hip, datapath.hip): the hash
// that derives exact small-integer operands, and the MFMA register vector types.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace canary {

constexpr int kWave = 64;

using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return static_cast<uint32_t>(x);
}

// small integer in [-4, 4] from a hash: exactly representable in bf16, fp8 (e4m3 and
// e5m2) and fp4 (e2m1), so MFMA results on such operands are exact in fp32
__device__ __forceinline__ int small_int(uint64_t key) { return static_cast<int>(mix32(key) % 9u) - 4; }

// A[row][k] and B[k][col] of exactness block `blk`
__device__ __forceinline__ int a_val(uint32_t blk, int row, int k) {
  return small_int((static_cast<uint64_t>(blk) << 40) ^ (static_cast<uint64_t>(row) << 20) ^ static_cast<uint64_t>(k));
}
__device__ __forceinline__ int b_val(uint32_t blk, int k, int col) {
  return small_int(0x5555ull ^ (static_cast<uint64_t>(blk) << 40) ^ (static_cast<uint64_t>(k) << 20) ^
                   static_cast<uint64_t>(col) ^ (1ull << 62));
}

}  // namespace canary
