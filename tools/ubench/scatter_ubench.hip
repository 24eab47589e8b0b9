// Microbenchmark of the partition scatter's cost structure on MI355X (not part of the product).
// n = 2^24 records (key, ts, val int64), P = 2048 partitions, 32768-record tiles; each variant timed over 20 launches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

constexpr int P = 2048, LOGP = 11, TILE = 32768, TPB = 1024;
struct alignas(16) i64x2 { long long x, y; };

__device__ __forceinline__ uint64_t fmix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}
__device__ __forceinline__ uint32_t part_of(int64_t k) { return (uint32_t)(fmix64((uint64_t)k) >> (64 - LOGP)); }

__global__ void k_gen(int64_t* key, int64_t* ts, int64_t* val, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t z = fmix64(i * 0x9E3779B97F4A7C15ull + 1);
  key[i] = (int64_t)(z % 1000000);
  ts[i] = 1000000 + i / 100;
  val[i] = (int64_t)(z >> 40);
}
// pure read of the three columns (pairs per lane, RPT records per thread per round)
template <int RPT>
__global__ __launch_bounds__(TPB) void k_read(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n, int64_t* out) {
  const int64_t t0 = (int64_t)blockIdx.x * TILE, t1 = min(n, t0 + TILE);
  int64_t acc = 0;
  for (int64_t b = t0; b < t1; b += (int64_t)TPB * RPT) {
    i64x2 k[RPT / 2], t[RPT / 2], v[RPT / 2];
#pragma unroll
    for (int j = 0; j < RPT / 2; j++) {
      int64_t i = b + 2 * ((int64_t)j * TPB + threadIdx.x);
      k[j] = *(const i64x2*)(key + i); t[j] = *(const i64x2*)(ts + i); v[j] = *(const i64x2*)(val + i);
    }
#pragma unroll
    for (int j = 0; j < RPT / 2; j++) acc += k[j].x ^ t[j].y ^ v[j].x ^ k[j].y ^ t[j].x ^ v[j].y;
  }
  if (acc == 42) out[0] = acc;
}
// MODE 0: linear 16-B store (copy); 1: + partition + LDS rank, linear store; 2: scattered into partition runs
template <int RPT, int MODE>
__global__ __launch_bounds__(TPB) void k_scat(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n, int T,
                                              const uint32_t* offs, i64x2* out) {
  __shared__ uint32_t base[P];
  const int tile = blockIdx.x;
  if (MODE == 2) for (int i = threadIdx.x; i < P; i += TPB) base[i] = offs[(int64_t)i * T + tile];
  else for (int i = threadIdx.x; i < P; i += TPB) base[i] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)tile * TILE, t1 = min(n, t0 + TILE);
  for (int64_t b = t0; b < t1; b += (int64_t)TPB * RPT) {
    i64x2 k[RPT / 2], t[RPT / 2], v[RPT / 2];
#pragma unroll
    for (int j = 0; j < RPT / 2; j++) {
      int64_t i = b + 2 * ((int64_t)j * TPB + threadIdx.x);
      k[j] = *(const i64x2*)(key + i); t[j] = *(const i64x2*)(ts + i); v[j] = *(const i64x2*)(val + i);
    }
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      const int64_t i = b + 2 * ((int64_t)(j >> 1) * TPB + threadIdx.x) + (j & 1);
      const int64_t kk = (j & 1) ? k[j >> 1].y : k[j >> 1].x, tt = (j & 1) ? t[j >> 1].y : t[j >> 1].x,
                    vv = (j & 1) ? v[j >> 1].y : v[j >> 1].x;
      int64_t pos = i;
      if (MODE >= 1) {
        const uint32_t p = part_of(kk);
        const uint32_t r = atomicAdd(&base[p], 1u);
        if (MODE == 2) pos = r; else asm volatile("" ::"v"(r));
      }
      out[pos] = i64x2{kk ^ (tt << 20), vv};
    }
  }
}
// LDS-staged: rounds of R records sorted by partition in LDS, then written as runs (MODE 0: into the global
// partition runs; MODE 1: linearly into the tile's own region)
template <int RPT, int MODE>
__global__ __launch_bounds__(TPB) void k_stage(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n, int T,
                                               const uint32_t* offs, i64x2* out) {
  constexpr int R = TPB * RPT;
  __shared__ i64x2 stg[R];
  __shared__ uint16_t sp[R];
  __shared__ uint32_t cnt[P], start[P], gb[P];
  __shared__ uint32_t wsum[TPB / 64 + 1];
  const int tile = blockIdx.x;
  for (int i = threadIdx.x; i < P; i += TPB) gb[i] = MODE == 0 ? offs[(int64_t)i * T + tile] : 0;
  const int64_t t0 = (int64_t)tile * TILE, t1 = min(n, t0 + TILE);
  uint32_t done = 0;
  for (int64_t b = t0; b < t1; b += R) {
    for (int i = threadIdx.x; i < P; i += TPB) cnt[i] = 0;
    __syncthreads();
    i64x2 k[RPT / 2], t[RPT / 2], v[RPT / 2];
#pragma unroll
    for (int j = 0; j < RPT / 2; j++) {
      int64_t i = b + 2 * ((int64_t)j * TPB + threadIdx.x);
      k[j] = *(const i64x2*)(key + i); t[j] = *(const i64x2*)(ts + i); v[j] = *(const i64x2*)(val + i);
    }
    uint32_t pp[RPT], rr[RPT];
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      const int64_t kk = (j & 1) ? k[j >> 1].y : k[j >> 1].x;
      pp[j] = part_of(kk);
      rr[j] = atomicAdd(&cnt[pp[j]], 1u);
    }
    __syncthreads();
    // exclusive scan of cnt (P = 2 per thread)
    const uint32_t a0 = cnt[2 * threadIdx.x], a1 = cnt[2 * threadIdx.x + 1];
    uint32_t x = a0 + a1;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) { uint32_t run = 0; for (int w = 0; w < TPB / 64; w++) { uint32_t q = wsum[w]; wsum[w] = run; run += q; } }
    __syncthreads();
    const uint32_t ex = wsum[wid] + x - (a0 + a1);
    start[2 * threadIdx.x] = ex;
    start[2 * threadIdx.x + 1] = ex + a0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      const int64_t kk = (j & 1) ? k[j >> 1].y : k[j >> 1].x, tt = (j & 1) ? t[j >> 1].y : t[j >> 1].x,
                    vv = (j & 1) ? v[j >> 1].y : v[j >> 1].x;
      const uint32_t s = start[pp[j]] + rr[j];
      stg[s] = i64x2{kk ^ (tt << 20), vv};
      sp[s] = (uint16_t)pp[j];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < R; i += TPB) {
      const uint32_t p = sp[i];
      const uint32_t g = MODE == 0 ? gb[p] + (i - start[p]) : (uint32_t)(t0 - 0) + done + i;
      out[g] = stg[i];
    }
    __syncthreads();
    if (MODE == 0) for (int i = threadIdx.x; i < P; i += TPB) gb[i] += cnt[i];
    done += R;
  }
}
__global__ void k_hist(const int64_t* key, int64_t n, int T, uint32_t* hist) {
  __shared__ uint32_t h[P];
  for (int i = threadIdx.x; i < P; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * TILE, t1 = min(n, t0 + TILE);
  for (int64_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) atomicAdd(&h[part_of(key[i])], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += blockDim.x) hist[(int64_t)i * T + blockIdx.x] = h[i];
}


// tile-local staging of 8192-record tiles (1 round per tile): sorted by partition in LDS, written linearly into the
// tile's region; the tile's partition starts go to st[t][p] (u16 pairs: start, count)
__global__ __launch_bounds__(TPB) void k_stage8k(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                                 i64x2* out, uint32_t* st) {
  constexpr int R = 8192, RPT = 8;
  __shared__ i64x2 stg[R];
  __shared__ uint32_t cnt[P], start[P];
  __shared__ uint32_t wsum[TPB / 64 + 1];
  const int tile = blockIdx.x;
  for (int i = threadIdx.x; i < P; i += TPB) cnt[i] = 0;
  __syncthreads();
  const int64_t b = (int64_t)tile * R;
  i64x2 k[RPT / 2], t[RPT / 2], v[RPT / 2];
#pragma unroll
  for (int j = 0; j < RPT / 2; j++) {
    int64_t i = b + 2 * ((int64_t)j * TPB + threadIdx.x);
    k[j] = *(const i64x2*)(key + i); t[j] = *(const i64x2*)(ts + i); v[j] = *(const i64x2*)(val + i);
  }
  uint32_t pp[RPT], rr[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    const int64_t kk = (j & 1) ? k[j >> 1].y : k[j >> 1].x;
    pp[j] = part_of(kk);
    rr[j] = atomicAdd(&cnt[pp[j]], 1u);
  }
  __syncthreads();
  const uint32_t a0 = cnt[2 * threadIdx.x], a1 = cnt[2 * threadIdx.x + 1];
  uint32_t x = a0 + a1;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) { uint32_t run = 0; for (int w = 0; w < TPB / 64; w++) { uint32_t q = wsum[w]; wsum[w] = run; run += q; } }
  __syncthreads();
  const uint32_t ex = wsum[wid] + x - (a0 + a1);
  start[2 * threadIdx.x] = ex;
  start[2 * threadIdx.x + 1] = ex + a0;
  st[(int64_t)tile * P + 2 * threadIdx.x] = ex | (a0 << 16);
  st[(int64_t)tile * P + 2 * threadIdx.x + 1] = (ex + a0) | (a1 << 16);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    const int64_t kk = (j & 1) ? k[j >> 1].y : k[j >> 1].x, tt = (j & 1) ? t[j >> 1].y : t[j >> 1].x,
                  vv = (j & 1) ? v[j >> 1].y : v[j >> 1].x;
    stg[start[pp[j]] + rr[j]] = i64x2{kk, vv ^ (tt << 20)};
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R; i += TPB) out[b + i] = stg[i];
}
// [t][p] -> [p][t], 64x64 tiles through LDS
__global__ void k_transpose(const uint32_t* in, uint32_t* outp, int T) {
  __shared__ uint32_t s[64][65];
  const int t0 = blockIdx.x * 64, p0 = blockIdx.y * 64;
  for (int r = threadIdx.y; r < 64; r += blockDim.y) s[r][threadIdx.x] = in[(int64_t)(t0 + r) * P + p0 + threadIdx.x];
  __syncthreads();
  for (int r = threadIdx.y; r < 64; r += blockDim.y) outp[(int64_t)(p0 + r) * T + t0 + threadIdx.x] = s[threadIdx.x][r];
}
// one workgroup (512 threads) per partition: gather its runs (start/count per tile) and fold the records
template <bool XCD>
__global__ __launch_bounds__(512) void k_gather(const i64x2* rec, const uint32_t* stT, int T, int64_t* sink) {
  __shared__ uint32_t pre[2048 + 1];
  __shared__ uint16_t s0[2048];
  __shared__ uint32_t wsum[9];
  // XCD: blocks b, b + 8, ... (one XCD) take consecutive partitions, whose runs sit side by side in every tile
  const int p = XCD ? (int)((blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3)) : (int)blockIdx.x;
  const uint32_t* row = stT + (int64_t)p * T;
  uint32_t c[4], tot = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int t = threadIdx.x * 4 + q;
    const uint32_t w = t < T ? row[t] : 0u;
    if (t < T) s0[t] = (uint16_t)(w & 0xffff);
    c[q] = w >> 16;
    tot += c[q];
  }
  uint32_t x = tot;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) { uint32_t run = 0; for (int w = 0; w < 8; w++) { uint32_t q = wsum[w]; wsum[w] = run; run += q; } wsum[8] = run; }
  __syncthreads();
  uint32_t e = wsum[wid] + x - tot;
#pragma unroll
  for (int q = 0; q < 4; q++) { pre[threadIdx.x * 4 + q] = e; e += c[q]; }
  if (threadIdx.x == 0) pre[T] = wsum[8];
  __syncthreads();
  const uint32_t total = wsum[8];
  int64_t acc = 0;
  for (uint32_t i0 = 0; i0 < total; i0 += 512 * 2) {
    i64x2 r[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t i = i0 + j * 512 + threadIdx.x;
      r[j] = i64x2{0, 0};
      if (i < total) {
        int lo = 0, hi = T - 1;  // last t with pre[t] <= i
        while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (pre[mid] <= i) lo = mid; else hi = mid - 1; }
        r[j] = rec[(int64_t)lo * 8192 + s0[lo] + (i - pre[lo])];
      }
    }
    acc += r[0].x ^ r[1].y ^ r[0].y ^ r[1].x;
  }
  if (acc == 42) sink[0] = acc;
}
// the same fold over partition-major runs (today's k_aggregate read)
__global__ __launch_bounds__(512) void k_linread(const i64x2* rec, const uint32_t* offs, int T, int64_t n, int64_t* sink) {
  const int p = blockIdx.x;
  const int64_t b = offs[(int64_t)p * T], e = p + 1 < P ? offs[(int64_t)(p + 1) * T] : n;
  int64_t acc = 0;
  for (int64_t i0 = b; i0 < e; i0 += 1024) {
    i64x2 r[2];
#pragma unroll
    for (int j = 0; j < 2; j++) { const int64_t i = i0 + j * 512 + threadIdx.x; r[j] = i < e ? rec[i] : i64x2{0, 0}; }
    acc += r[0].x ^ r[1].y ^ r[0].y ^ r[1].x;
  }
  if (acc == 42) sink[0] = acc;
}


// tile-local, no staging: pass 1 counts the tile's keys per partition, a scan gives the runs inside the tile's
// region, pass 2 re-reads the records and writes each at its run's cursor (scattered inside the region)
template <int TL>
__global__ __launch_bounds__(TPB) void k_tilelocal(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                                   i64x2* out, uint32_t* st) {
  __shared__ uint32_t cnt[P], cur[P];
  __shared__ uint32_t wsum[TPB / 64 + 1];
  const int tile = blockIdx.x;
  for (int i = threadIdx.x; i < P; i += TPB) cnt[i] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)tile * TL, t1 = min(n, t0 + TL);
  for (int64_t b = t0; b < t1; b += (int64_t)TPB * 8) {
    i64x2 k[4];
#pragma unroll
    for (int j = 0; j < 4; j++) k[j] = *(const i64x2*)(key + b + 2 * ((int64_t)j * TPB + threadIdx.x));
#pragma unroll
    for (int j = 0; j < 4; j++) { atomicAdd(&cnt[part_of(k[j].x)], 1u); atomicAdd(&cnt[part_of(k[j].y)], 1u); }
  }
  __syncthreads();
  const uint32_t a0 = cnt[2 * threadIdx.x], a1 = cnt[2 * threadIdx.x + 1];
  uint32_t x = a0 + a1;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) { uint32_t run = 0; for (int w = 0; w < TPB / 64; w++) { uint32_t q = wsum[w]; wsum[w] = run; run += q; } }
  __syncthreads();
  const uint32_t ex = wsum[wid] + x - (a0 + a1);
  cur[2 * threadIdx.x] = ex;
  cur[2 * threadIdx.x + 1] = ex + a0;
  st[(int64_t)tile * P + 2 * threadIdx.x] = ex;
  st[(int64_t)tile * P + 2 * threadIdx.x + 1] = ex + a0;
  __syncthreads();
  for (int64_t b = t0; b < t1; b += (int64_t)TPB * 8) {
    i64x2 k[4], t[4], v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int64_t i = b + 2 * ((int64_t)j * TPB + threadIdx.x);
      k[j] = *(const i64x2*)(key + i); t[j] = *(const i64x2*)(ts + i); v[j] = *(const i64x2*)(val + i);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int64_t kk = (j & 1) ? k[j >> 1].y : k[j >> 1].x, tt = (j & 1) ? t[j >> 1].y : t[j >> 1].x,
                    vv = (j & 1) ? v[j >> 1].y : v[j >> 1].x;
      const uint32_t pos = atomicAdd(&cur[part_of(kk)], 1u);
      out[t0 + pos] = i64x2{kk, vv ^ (tt << 20)};
    }
  }
}

int main() {
  const int64_t n = 1 << 24;
  const int T = (int)(n / TILE);
  int64_t *key, *ts, *val, *o;
  i64x2* out;
  uint32_t* offs;
  CK(hipMalloc(&key, n * 8)); CK(hipMalloc(&ts, n * 8)); CK(hipMalloc(&val, n * 8)); CK(hipMalloc(&o, 64));
  CK(hipMalloc(&out, n * 16)); CK(hipMalloc(&offs, (size_t)P * T * 4));
  hipLaunchKernelGGL(k_gen, dim3(n / 256), dim3(256), 0, 0, key, ts, val, n);
  hipLaunchKernelGGL(k_hist, dim3(T), dim3(1024), 0, 0, key, n, T, offs);
  std::vector<uint32_t> h((size_t)P * T);
  CK(hipMemcpy(h.data(), offs, h.size() * 4, hipMemcpyDeviceToHost));
  uint32_t run = 0;
  for (auto& x : h) { uint32_t c = x; x = run; run += c; }
  CK(hipMemcpy(offs, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 3; i++) launch();
    hipEventRecord(a, 0);
    for (int i = 0; i < 20; i++) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 20;
    printf("%-44s %8.4f ms  %6.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
  };
  const double rd = n * 24.0, wr = n * 16.0;
  timeit("read 24 B (RPT 8)", rd, [&] { hipLaunchKernelGGL((k_read<8>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, o); });
  timeit("read 24 B (RPT 4)", rd, [&] { hipLaunchKernelGGL((k_read<4>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, o); });
  timeit("copy 24->16 linear (RPT 8)", rd + wr, [&] { hipLaunchKernelGGL((k_scat<8, 0>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, T, offs, out); });
  timeit("copy 24->16 linear (RPT 4)", rd + wr, [&] { hipLaunchKernelGGL((k_scat<4, 0>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, T, offs, out); });
  timeit("+partition+LDS rank, linear (RPT 8)", rd + wr, [&] { hipLaunchKernelGGL((k_scat<8, 1>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, T, offs, out); });
  timeit("scatter into partition runs (RPT 8)", rd + wr, [&] { hipLaunchKernelGGL((k_scat<8, 2>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, T, offs, out); });
  timeit("scatter into partition runs (RPT 4)", rd + wr, [&] { hipLaunchKernelGGL((k_scat<4, 2>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, T, offs, out); });
  timeit("LDS-staged 4096 -> partition runs", rd + wr, [&] { hipLaunchKernelGGL((k_stage<4, 0>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, T, offs, out); });
  timeit("LDS-staged 4096 -> tile-local linear", rd + wr, [&] { hipLaunchKernelGGL((k_stage<4, 1>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, T, offs, out); });
  {
    const int T8 = (int)(n / 8192);
    uint32_t *st, *stT;
    CK(hipMalloc(&st, (size_t)T8 * P * 4)); CK(hipMalloc(&stT, (size_t)T8 * P * 4));
    timeit("LDS-staged 8192 tiles -> tile-local + table", rd + wr, [&] { hipLaunchKernelGGL(k_stage8k, dim3(T8), dim3(TPB), 0, 0, key, ts, val, n, out, st); });
    timeit("transpose start table", 2.0 * T8 * P * 4, [&] { hipLaunchKernelGGL(k_transpose, dim3(T8 / 64, P / 64), dim3(64, 16), 0, 0, st, stT, T8); });
    timeit("gather runs per partition (16 B/rec)", wr, [&] { hipLaunchKernelGGL(k_gather<false>, dim3(P), dim3(512), 0, 0, out, stT, T8, o); });
    timeit("gather runs, XCD-grouped partitions", wr, [&] { hipLaunchKernelGGL(k_gather<true>, dim3(P), dim3(512), 0, 0, out, stT, T8, o); });
  }
  {
    uint32_t* st;
    CK(hipMalloc(&st, (size_t)(n / 8192) * P * 4));
    timeit("tile-local 2-pass scattered, 32768 tiles", rd + wr + n * 8.0, [&] { hipLaunchKernelGGL((k_tilelocal<32768>), dim3(n / 32768), dim3(TPB), 0, 0, key, ts, val, n, out, st); });
    timeit("tile-local 2-pass scattered, 65536 tiles", rd + wr + n * 8.0, [&] { hipLaunchKernelGGL((k_tilelocal<65536>), dim3(n / 65536), dim3(TPB), 0, 0, key, ts, val, n, out, st); });
    timeit("tile-local 2-pass scattered, 16384 tiles", rd + wr + n * 8.0, [&] { hipLaunchKernelGGL((k_tilelocal<16384>), dim3(n / 16384), dim3(TPB), 0, 0, key, ts, val, n, out, st); });
    timeit("tile-local 2-pass scattered, 8192 tiles", rd + wr + n * 8.0, [&] { hipLaunchKernelGGL((k_tilelocal<8192>), dim3(n / 8192), dim3(TPB), 0, 0, key, ts, val, n, out, st); });
  }
  hipLaunchKernelGGL((k_scat<8, 2>), dim3(T), dim3(TPB), 0, 0, key, ts, val, n, T, offs, out);
  timeit("linear read of partition-major runs", wr, [&] { hipLaunchKernelGGL(k_linread, dim3(P), dim3(512), 0, 0, out, offs, T, n, o); });
  timeit("hist (keys only)", n * 8.0, [&] { hipLaunchKernelGGL(k_hist, dim3(T), dim3(1024), 0, 0, key, n, T, offs); });
  return 0;
}
