// Radix-sort microbenchmark for the t-digest key sort: 2^24 (u64 key, u32 payload) pairs, 64 key bits, rocPRIM
// onesweep with the gfx950 default (8 bits per place) and 10-bit digits (11 bits exceed the histogram kernel's LDS at 6 places). Prints ms per sort (median of 10).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 sort_ubench.hip -o sort_ubench
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void fill(uint64_t* k, uint32_t* v, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    k[i] = z;
    v[i] = (uint32_t)i;
  }
}
__global__ void check(const uint64_t* k, int64_t n, int* bad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x + 1; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (k[i - 1] > k[i]) atomicAdd(bad, 1);
}

template <class Cfg>
void run(const char* name, int64_t n, uint64_t* k0, uint64_t* k1, uint32_t* v0, uint32_t* v1, int* bad) {
  size_t bytes = 0;
  rocprim::double_buffer<uint64_t> kb(k0, k1);
  rocprim::double_buffer<uint32_t> vb(v0, v1);
  CK(rocprim::radix_sort_pairs<Cfg>(nullptr, bytes, kb, vb, (size_t)n, 0, 64));
  void* tmp;
  CK(hipMalloc(&tmp, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> t;
  for (int it = 0; it < 12; it++) {
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, k0, v0, n, 77ull + it);
    rocprim::double_buffer<uint64_t> kk(k0, k1);
    rocprim::double_buffer<uint32_t> vv(v0, v1);
    CK(hipEventRecord(a, 0));
    CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, kk, vv, (size_t)n, 0, 64, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 2) t.push_back(ms);
    if (it == 11) {
      CK(hipMemset(bad, 0, 4));
      hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, kk.current(), n, bad);
      int h = 0;
      CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
      std::sort(t.begin(), t.end());
      printf("%-10s median %.3f ms  min %.3f  unsorted %d  tmp %zu MB\n", name, t[t.size() / 2], t[0], h, bytes >> 20);
    }
  }
  CK(hipFree(tmp));
}

int main() {
  const int64_t n = int64_t(1) << 24;
  uint64_t *k0, *k1;
  uint32_t *v0, *v1;
  int* bad;
  CK(hipMalloc(&k0, n * 8));
  CK(hipMalloc(&k1, n * 8));
  CK(hipMalloc(&v0, n * 4));
  CK(hipMalloc(&v1, n * 4));
  CK(hipMalloc(&bad, 4));
  using rocprim::block_radix_rank_algorithm;
  using rocprim::kernel_config;
  using rocprim::radix_sort_onesweep_config;
  run<rocprim::default_config>("default", n, k0, k1, v0, v1, bad);
  run<rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                 radix_sort_onesweep_config<kernel_config<512, 32>, kernel_config<512, 12>, 8,
                                                            block_radix_rank_algorithm::match>>>("8b/512x12", n, k0, k1,
                                                                                                 v0, v1, bad);
  run<rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                 radix_sort_onesweep_config<kernel_config<256, 16>, kernel_config<512, 12>, 10,
                                                            block_radix_rank_algorithm::match>>>("10b/512x12", n, k0, k1,
                                                                                                 v0, v1, bad);
  run<rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                 radix_sort_onesweep_config<kernel_config<256, 16>, kernel_config<1024, 8>, 10,
                                                            block_radix_rank_algorithm::match>>>("10b/1024x8", n, k0, k1,
                                                                                                 v0, v1, bad);
  run<rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                 radix_sort_onesweep_config<kernel_config<256, 16>, kernel_config<256, 16>, 10,
                                                            block_radix_rank_algorithm::match>>>("10b/256x16", n, k0,
                                                                                                 k1, v0, v1, bad);
  return 0;
}
