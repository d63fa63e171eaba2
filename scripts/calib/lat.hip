// Latency probes (one workgroup): dependent random loads and returning device-scope
// atomics over tables of the multi BFS's sizes. Prints microseconds per dependent step.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_chain_load(const uint32_t* __restrict__ t, uint32_t mask, uint32_t steps, uint32_t* out,
                             unsigned long long* clk) {
  uint32_t x = threadIdx.x * 7919u;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  for (uint32_t i = 0; i < steps; ++i) x = t[((x + i * 40503u + threadIdx.x * 977u) * 2654435761u) & mask] + x;
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) clk[0] = t1 - t0;
  out[threadIdx.x] = x;
}

__global__ void k_chain_atomic(uint32_t* t, uint32_t mask, uint32_t steps, uint32_t* out, unsigned long long* clk) {
  uint32_t x = threadIdx.x * 7919u;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  for (uint32_t i = 0; i < steps; ++i) x = atomicOr(&t[((x + i * 40503u + threadIdx.x * 977u) * 2654435761u) & mask], 1u << (i & 31)) + x;
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) clk[0] = t1 - t0;
  out[threadIdx.x] = x;
}

__global__ void k_chain_store_barrier(uint32_t* t, uint32_t mask, uint32_t steps, uint32_t* out,
                                      unsigned long long* clk) {
  uint32_t x = threadIdx.x * 7919u;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  for (uint32_t i = 0; i < steps; ++i) {
    t[((x + i * 40503u + threadIdx.x * 977u) * 2654435761u) & mask] = x;
    __syncthreads();
    x += i;
  }
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) clk[0] = t1 - t0;
  out[threadIdx.x] = x;
}

__global__ void k_multi_atomic(uint32_t* t, uint32_t mask, uint32_t steps, uint32_t* out, unsigned long long* clk) {
  uint32_t x = threadIdx.x * 7919u;
  __syncthreads();
  const unsigned long long t0 = wall_clock64();
  for (uint32_t i = 0; i < steps; ++i) {
    uint32_t r[12];
#pragma unroll
    for (int s = 0; s < 12; ++s) r[s] = atomicOr(&t[((x + i * 40503u + threadIdx.x * 977u + s * 7u) * 2654435761u) & mask], 1u);
#pragma unroll
    for (int s = 0; s < 12; ++s) x += r[s];
  }
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) clk[0] = t1 - t0;
  out[threadIdx.x] = x;
}

int main() {
  int rate = 0;
  hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
  printf("wall clock rate %d kHz\n", rate);
  const size_t words[] = {1u << 20, 1u << 24, 1u << 26};  // 4 MB, 64 MB, 256 MB
  uint32_t *t, *out;
  unsigned long long* clk;
  hipMalloc(&t, (1u << 26) * 4);
  hipMemset(t, 0, (1u << 26) * 4);
  hipMalloc(&out, 4096 * 4);
  hipMalloc(&clk, 64);
  const uint32_t steps = 64;
  for (size_t w : words) {
    for (int th : {64, 1024}) {
      for (int kind = 0; kind < 4; ++kind) {
        for (int rep = 0; rep < 2; ++rep) {
          if (kind == 0) hipLaunchKernelGGL(k_chain_load, dim3(1), dim3(th), 0, 0, t, (uint32_t)(w - 1), steps, out, clk);
          if (kind == 1) hipLaunchKernelGGL(k_chain_atomic, dim3(1), dim3(th), 0, 0, t, (uint32_t)(w - 1), steps, out, clk);
          if (kind == 3) hipLaunchKernelGGL(k_multi_atomic, dim3(1), dim3(th), 0, 0, t, (uint32_t)(w - 1), steps, out, clk);
          if (kind == 2) hipLaunchKernelGGL(k_chain_store_barrier, dim3(1), dim3(th), 0, 0, t, (uint32_t)(w - 1), steps, out, clk);
          hipDeviceSynchronize();
          unsigned long long c = 0;
          hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
          if (rep == 1)
            printf("%-14s table %6zu KB threads %4d: %.3f us per dependent step\n",
                   kind == 0 ? "load" : kind == 1 ? "atomicOr-ret" : kind == 2 ? "store+barrier" : "12 atomicOr-ret", w * 4 / 1024, th,
                   c / (rate / 1000.0) / steps);
        }
      }
    }
  }
  return 0;
}
