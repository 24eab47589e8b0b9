// LDS atomic throughput on MI355X (not part of the product): per op, 1024-thread workgroups (one per CU) each
// issue ITER wave-instructions of random slots in a 4096-entry table; reports lane-ops per clock per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int S = 4096, ITER = 256;
template <int OP>
__global__ __launch_bounds__(1024) void k_lds(unsigned long long* out, int spread) {
  __shared__ unsigned long long t[S];
  for (int i = threadIdx.x; i < S; i += 1024) t[i] = i;
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x * 97u + 1;
  unsigned long long acc = 0;
  for (int it = 0; it < ITER; it++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const uint32_t s = spread ? (x & (S - 1)) : ((threadIdx.x + it) & (S - 1));
    if (OP == 0) atomicAdd((unsigned int*)&t[s], 1u);
    if (OP == 1) atomicAdd(&t[s], 1ull);
    if (OP == 2) atomicMin((long long*)&t[s], (long long)x);
    if (OP == 3) atomicAdd((double*)&t[s], 1.0);
    if (OP == 4) acc += __hip_atomic_load(&t[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (OP == 5) t[s] = x;
    if (OP == 6) { atomicAdd(&t[s], 1ull); atomicAdd(&t[(s + 1) & (S - 1)], 2ull); atomicMin((long long*)&t[(s + 2) & (S - 1)], (long long)x); atomicMax((long long*)&t[(s + 3) & (S - 1)], (long long)x); }
  }
  __syncthreads();
  if (acc == 12345) out[1] = acc;
  if (threadIdx.x == 0) out[0] += t[7];
}
int main() {
  unsigned long long* o;
  CK(hipMalloc(&o, 16));
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const char* names[] = {"ds_add_u32", "ds_add_u64", "ds_min_i64", "ds_add_f64", "ds_read_b64", "ds_write_b64", "4x 64-bit atomics"};
  for (int spread = 1; spread >= 0; spread--)
  for (int op = 0; op < 7; op++) {
    auto run = [&] {
      switch (op) {
        case 0: hipLaunchKernelGGL(k_lds<0>, dim3(256 * 4), dim3(1024), 0, 0, o, spread); break;
        case 1: hipLaunchKernelGGL(k_lds<1>, dim3(256 * 4), dim3(1024), 0, 0, o, spread); break;
        case 2: hipLaunchKernelGGL(k_lds<2>, dim3(256 * 4), dim3(1024), 0, 0, o, spread); break;
        case 3: hipLaunchKernelGGL(k_lds<3>, dim3(256 * 4), dim3(1024), 0, 0, o, spread); break;
        case 4: hipLaunchKernelGGL(k_lds<4>, dim3(256 * 4), dim3(1024), 0, 0, o, spread); break;
        case 5: hipLaunchKernelGGL(k_lds<5>, dim3(256 * 4), dim3(1024), 0, 0, o, spread); break;
        case 6: hipLaunchKernelGGL(k_lds<6>, dim3(256 * 4), dim3(1024), 0, 0, o, spread); break;
      }
    };
    run(); hipDeviceSynchronize();
    hipEventRecord(a); for (int r = 0; r < 5; r++) run(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
    const double lane_ops = 256.0 * 4 * 1024 * ITER * (op == 6 ? 4 : 1);
    // per CU: lane-ops / (time * 2.4 GHz) / 256 CUs (assumes ~2.4 GHz)
    printf("%-20s %s  %.4f ms  %.2f lane-ops/clk/CU (2.4 GHz)\n", names[op], spread ? "random" : "consecutive", ms,
           lane_ops / (ms * 1e-3 * 2.4e9) / 256);
  }
  return 0;
}
