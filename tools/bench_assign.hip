// Standalone micro-benchmark (tools only, not part of the library): variants
// of the radius graph's cell-assignment pass at the C2 shape (50k particles,
// frame T-1 of an [n][11][2] window), timed with hipEvents.
//   hipcc -O3 --offload-arch=gfx950 tools/bench_assign.hip -o /tmp/bench_assign && /tmp/bench_assign
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <math.h>

struct Grid { float lo[3]; float inv_cell; int g[3]; };

__device__ __forceinline__ int cell_of(float x, float lo, float inv, int g) {
  float q = floorf((x - lo) * inv);
  if (!(q == q)) q = 0.0f;
  q = fminf(fmaxf(q, 0.0f), (float)(g - 1));
  return (int)q;
}

// V0: as the library (runtime dim loop, Grid through a pointer)
__global__ void k_v0(const float* pos, int64_t stride, int64_t n, int dim, const Grid* gp, int* cell, int* count) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i0 < n;
  const int64_t i = active ? i0 : n - 1;
  const Grid G = *gp;
  const float* p = pos + i * stride;
  int c[3] = {0, 0, 0};
  for (int d = 0; d < dim; ++d) c[d] = cell_of(p[d], G.lo[d], G.inv_cell, G.g[d]);
  const int key = (c[2] * G.g[1] + c[1]) * G.g[0] + c[0];
  if (active) {
    cell[i] = key;
    atomicAdd(&count[key], 1);
  }
}

// V1: 2D unrolled loads issued together, no atomic
template <bool ATOMIC>
__global__ void k_v1(const float* pos, int64_t stride, int64_t n, const Grid* gp, int* cell, int* count) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i0 < n;
  const int64_t i = active ? i0 : n - 1;
  const float x = pos[i * stride], y = pos[i * stride + 1];
  const Grid G = *gp;
  const int key = cell_of(y, G.lo[1], G.inv_cell, G.g[1]) * G.g[0] + cell_of(x, G.lo[0], G.inv_cell, G.g[0]);
  if (active) {
    cell[i] = key;
    if (ATOMIC) atomicAdd(&count[key], 1);
  }
}

__global__ void k_empty(int* p) { if (p == nullptr && threadIdx.x == 1234) p[0] = 1; }

int main() {
  const int64_t n = 50000, T = 11, stride = T * 2;
  std::vector<float> h(n * stride);
  for (int64_t i = 0; i < n; ++i)
    for (int t = 0; t < T; ++t) {
      h[(i * T + t) * 2] = 0.25f + 0.5f * (i / 200);
      h[(i * T + t) * 2 + 1] = -9.75f + 0.5f * (i % 200);
    }
  float* pos; int *cell, *count; Grid* gp;
  hipMalloc(&pos, h.size() * 4); hipMalloc(&cell, n * 4); hipMalloc(&count, 4 << 20); hipMalloc(&gp, sizeof(Grid));
  hipMemcpy(pos, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  Grid G{{0.25f, -9.75f, 0.f}, 1.0f / 0.606f, {207, 166, 1}};
  hipMemcpy(gp, &G, sizeof(Grid), hipMemcpyHostToDevice);
  const float* last = pos + (T - 1) * 2;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const unsigned nb = (unsigned)((n + 255) / 256);
  auto timeit = [&](const char* name, auto fn) {
    for (int k = 0; k < 20; ++k) fn();
    hipEventRecord(a);
    for (int k = 0; k < 200; ++k) fn();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-40s %8.2f us/launch\n", name, ms * 1e3f / 200);
  };
  timeit("empty kernel", [&] { hipLaunchKernelGGL(k_empty, dim3(nb), dim3(256), 0, 0, cell); });
  timeit("memset 1 MB", [&] { hipMemsetAsync(count, 0, 1 << 20, 0); });
  timeit("v0 library form", [&] { hipLaunchKernelGGL(k_v0, dim3(nb), dim3(256), 0, 0, last, stride, n, 2, gp, cell, count); });
  timeit("memset + v0", [&] { hipMemsetAsync(count, 0, 1 << 20, 0); hipLaunchKernelGGL(k_v0, dim3(nb), dim3(256), 0, 0, last, stride, n, 2, gp, cell, count); });
  timeit("v1 2D unrolled, atomic", [&] { hipLaunchKernelGGL((k_v1<true>), dim3(nb), dim3(256), 0, 0, last, stride, n, gp, cell, count); });
  timeit("v1 2D unrolled, no atomic", [&] { hipLaunchKernelGGL((k_v1<false>), dim3(nb), dim3(256), 0, 0, last, stride, n, gp, cell, count); });
  return 0;
}
