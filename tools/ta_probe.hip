// Vector-memory (TA) cost of a uniform-address access: full-exec wave64 vs one active lane.
// Each wave walks a private 16 KB region (L2-resident) with dependent uniform loads (A/B) or
// issues uniform stores (C/D). Prints ms per kernel. hipcc --offload-arch=gfx950 -O3 ta_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#define N 4096
__global__ __launch_bounds__(64) void ld_full(const int* p, int* out) {
  const int* q = p + (size_t)blockIdx.x * 4096;
  int x = 0;
  for (int i = 0; i < N; i++) x = q[(x + i * 17) & 4095] + 1;  // uniform address, all lanes
  if (threadIdx.x == 0) out[blockIdx.x] = x;
}
__global__ __launch_bounds__(64) void ld_one(const int* p, int* out) {
  const int* q = p + (size_t)blockIdx.x * 4096;
  int x = 0;
  for (int i = 0; i < N; i++) {
    int v = 0;
    if (threadIdx.x == 0) v = q[(x + i * 17) & 4095];
    x = __builtin_amdgcn_readfirstlane(v) + 1;
  }
  if (threadIdx.x == 0) out[blockIdx.x] = x;
}
__global__ __launch_bounds__(64) void st_full(int* p) {
  int* q = p + (size_t)blockIdx.x * 4096;
  for (int i = 0; i < N; i++) q[(i * 17) & 4095] = i;
}
__global__ __launch_bounds__(64) void st_one(int* p) {
  int* q = p + (size_t)blockIdx.x * 4096;
  for (int i = 0; i < N; i++) if (threadIdx.x == 0) q[(i * 17) & 4095] = i;
}
int main() {
  int nb = 256 * 32;
  int *p, *out;
  hipMalloc(&p, (size_t)nb * 4096 * 4);
  hipMalloc(&out, nb * 4);
  hipMemset(p, 0, (size_t)nb * 4096 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 2; rep++) {
    float ms;
    hipEventRecord(a); ld_full<<<nb, 64>>>(p, out); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b); printf("ld_full %.3f ms\n", ms);
    hipEventRecord(a); ld_one<<<nb, 64>>>(p, out); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b); printf("ld_one  %.3f ms\n", ms);
    hipEventRecord(a); st_full<<<nb, 64>>>(p); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b); printf("st_full %.3f ms\n", ms);
    hipEventRecord(a); st_one<<<nb, 64>>>(p); hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b); printf("st_one  %.3f ms\n", ms);
  }
  return 0;
}
