// Ceiling of k_dt_aggregate's record phase on MI355X (not part of the product): 1024 workgroups of 1024 threads,
// each streams its own 16384 consecutive 16-byte records (2^24 in all, 256 MB) and, per mode, adds them into a
// 3488-slot LDS table the way the dense aggregate does (slot from a hash of the record's word, count / sum / min /
// max as 64-bit LDS atomics).  Reports ms and GB/s of records read for:
//   mode 0: loads only (RPT records per thread in flight, double-buffered as in the aggregate)
//   mode 1: loads + the four LDS atomics at a hashed slot (no probing)
//   mode 2: loads + a bucket read (two ds_read_b128) + the four atomics (the aggregate's lookup + add)
//   mode 3: loads + cnt/sum atomics only, min/max read first and raised only when needed
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int SLOTS = 3488, THREADS = 1024, PER_WG = 16384;
struct i64x2 { long long x, y; };
template <int MODE, int RPT>
__global__ __launch_bounds__(THREADS) void k_agg(const i64x2* __restrict__ rec, unsigned long long* out) {
  __shared__ unsigned long long kw[SLOTS], cnt[SLOTS];
  __shared__ long long sum[SLOTS], mn[SLOTS], mx[SLOTS];
  for (int h = threadIdx.x; h < SLOTS; h += THREADS) {
    kw[h] = h;
    cnt[h] = 0;
    sum[h] = 0;
    mn[h] = 1ll << 62;
    mx[h] = -(1ll << 62);
  }
  __syncthreads();
  const long long b0 = (long long)blockIdx.x * PER_WG, e0 = b0 + PER_WG;
  constexpr int RS = THREADS * RPT;
  unsigned long long acc = 0;
  auto load = [&](i64x2 (&d)[RPT], long long r0) {
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      const long long i = r0 + j * THREADS + threadIdx.x;
      d[j] = rec[i < e0 ? i : e0 - 1];
    }
  };
  auto add = [&](const i64x2 (&d)[RPT]) {
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      const unsigned long long w = (unsigned long long)d[j].x;
      const long long v = d[j].y;
      if (MODE == 0) {
        acc += w ^ (unsigned long long)v;
        continue;
      }
      uint32_t h = (uint32_t)(w >> 32) * 0x9E3779B1u ^ (uint32_t)w;
      h ^= h >> 15;
      const uint32_t s = (uint32_t)(((uint64_t)h * (SLOTS / 4)) >> 32) * 4u;
      uint32_t t = s;
      if (MODE == 2) {
        const i64x2 a = *reinterpret_cast<const i64x2*>(&kw[s]);
        const i64x2 b = *reinterpret_cast<const i64x2*>(&kw[s + 2]);
        t = (unsigned long long)a.x == w ? s : (unsigned long long)a.y == w ? s + 1 : (unsigned long long)b.x == w ? s + 2
            : (unsigned long long)b.y == w ? s + 3 : s + (uint32_t)(w & 3);
      }
      atomicAdd(&cnt[t], 1ull);
      atomicAdd((unsigned long long*)&sum[t], (unsigned long long)v);
      if (MODE == 3) {
        if (v < mn[t]) atomicMin(&mn[t], v);
        if (v > mx[t]) atomicMax(&mx[t], v);
      } else {
        atomicMin(&mn[t], v);
        atomicMax(&mx[t], v);
      }
    }
  };
  i64x2 ra[RPT], rb[RPT];
  load(ra, b0);
  for (long long r0 = b0; r0 < e0; r0 += 2 * RS) {
    load(rb, r0 + RS);
    add(ra);
    if (r0 + RS >= e0) break;
    load(ra, r0 + 2 * RS);
    add(rb);
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = cnt[7] + (unsigned long long)sum[5] + acc;
}
__global__ void k_init(i64x2* rec, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    rec[i] = i64x2{(long long)(z % 1048576ull * 0x2545F4914F6CDD1Dull), (long long)(int)(z >> 20)};
  }
}
template <int MODE, int RPT>
float run(const i64x2* rec, unsigned long long* out, int nwg) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL((k_agg<MODE, RPT>), dim3(nwg), dim3(THREADS), 0, 0, rec, out);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL((k_agg<MODE, RPT>), dim3(nwg), dim3(THREADS), 0, 0, rec, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}
int main() {
  const int nwg = 1024;
  const size_t n = (size_t)nwg * PER_WG;
  i64x2* rec;
  unsigned long long* out;
  CK(hipMalloc(&rec, n * sizeof(i64x2)));
  CK(hipMalloc(&out, nwg * sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, rec, n);
  CK(hipDeviceSynchronize());
  const double gb = n * 16.0 / 1e9;
  auto pr = [&](const char* name, float ms) { printf("%-34s %.4f ms  %.2f TB/s of records\n", name, ms, gb / ms); };
  pr("loads only, RPT 2", run<0, 2>(rec, out, nwg));
  pr("loads only, RPT 4", run<0, 4>(rec, out, nwg));
  pr("loads only, RPT 8", run<0, 8>(rec, out, nwg));
  pr("loads + 4 atomics, RPT 2", run<1, 2>(rec, out, nwg));
  pr("loads + 4 atomics, RPT 4", run<1, 4>(rec, out, nwg));
  pr("loads + bucket read + 4 atomics, RPT 2", run<2, 2>(rec, out, nwg));
  pr("loads + bucket read + 4 atomics, RPT 4", run<2, 4>(rec, out, nwg));
  pr("loads + 2 atomics + min/max if needed, RPT 2", run<3, 2>(rec, out, nwg));
  pr("loads + 2 atomics + min/max if needed, RPT 4", run<3, 4>(rec, out, nwg));
  return 0;
}
