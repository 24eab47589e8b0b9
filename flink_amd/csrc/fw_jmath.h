// fw_jmath.h — Java arithmetic and key hashing shared by the HIP translation units (included inside their
// anonymous namespaces, after flink_window.h).
#pragma once

__device__ __forceinline__ int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
__device__ __forceinline__ int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// flink-core/src/main/java/org/apache/flink/util/MathUtils.java:191-198
__device__ __forceinline__ int32_t bit_mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return (int32_t)x;
}
// MathUtils.java:134-154
__device__ __forceinline__ int32_t murmur(int32_t code) {
  uint32_t c = (uint32_t)code;
  c *= 0xcc9e2d51u;
  c = rotl32(c, 15);
  c *= 0x1b873593u;
  c = rotl32(c, 13);
  c = c * 5u + 0xe6546b64u;
  c ^= 4u;
  int32_t r = bit_mix(c);
  return r >= 0 ? r : (r != INT32_MIN ? -r : 0);
}
__device__ __forceinline__ uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}
__device__ __forceinline__ int32_t key_hash_of(int32_t kind, int64_t key, const int32_t* kh, int64_t i) {
  if (kind == FW_KEY_HASHED) return kh[i];
  if (kind == FW_KEY_INT) return (int32_t)key;
  return (int32_t)(key ^ (int64_t)((uint64_t)key >> 32));  // Long.hashCode
}
// KeyGroupRangeAssignment.computeKeyGroupForKeyHash (KeyGroupRangeAssignment.java:69-71)
__device__ __forceinline__ int32_t key_group(int32_t h, int32_t max_par) { return murmur(h) % max_par; }
