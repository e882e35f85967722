// Round-6 experiment: the gap between two dependent ~50 us kernels on one stream, by what the kernels
// request: nothing / 80 KB dynamic LDS / LDS + a large register allocation.  Eager launches, then the
// same sequence captured in a hipGraph and replayed.  Run under rocprofv3 --kernel-trace.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ __launch_bounds__(256) void k_work(float* p, long n4, int iters) {
  extern __shared__ float lds[];
  float acc[MODE == 2 ? 64 : 4];
#pragma unroll
  for (int i = 0; i < (MODE == 2 ? 64 : 4); ++i) acc[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < iters; ++it) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
      float4 v = reinterpret_cast<float4*>(p)[i];
#pragma unroll
      for (int k = 0; k < (MODE == 2 ? 64 : 4); ++k) acc[k] = acc[k] * 0.999f + v.x;
      if (MODE >= 1) lds[(threadIdx.x * 4 + it) & 16383] = acc[0];
      v.y += acc[(MODE == 2 ? 63 : 3)];
      reinterpret_cast<float4*>(p)[i] = v;
    }
  }
  if (MODE >= 1) { __syncthreads(); if (threadIdx.x == 0) p[blockIdx.x] += lds[blockIdx.x & 255]; }
}
struct BigArgs { float* p; long n4; int iters; float pad[320]; };
__global__ __launch_bounds__(256) void k_work_big(BigArgs a) {
  for (int it = 0; it < a.iters; ++it)
    for (long i = blockIdx.x * 256L + threadIdx.x; i < a.n4; i += (long)gridDim.x * 256) {
      float4 v = reinterpret_cast<float4*>(a.p)[i];
      v.y += a.pad[threadIdx.x & 255];
      reinterpret_cast<float4*>(a.p)[i] = v;
    }
}
int main() {
  float* p;
  const long n4 = (64L << 20) / 16;
  hipMalloc(&p, 64L << 20);
  hipMemset(p, 0, 64L << 20);
  hipStream_t s;
  hipStreamCreate(&s);
  auto seq = [&](int mode) {
    for (int k = 0; k < 8; ++k) {
      if (mode == 0) hipLaunchKernelGGL(k_work<0>, dim3(512), dim3(256), 0, s, p, n4, 2);
      if (mode == 1) hipLaunchKernelGGL(k_work<1>, dim3(512), dim3(256), 80 * 1024, s, p, n4, 2);
      if (mode == 2) hipLaunchKernelGGL(k_work<2>, dim3(512), dim3(256), 80 * 1024, s, p, n4, 2);
      if (mode == 3) {
        BigArgs a{};
        a.p = p; a.n4 = n4; a.iters = 2;
        hipLaunchKernelGGL(k_work_big, dim3(512), dim3(256), 0, s, a);
      }
    }
  };
  hipFuncSetAttribute((const void*)k_work<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  hipFuncSetAttribute((const void*)k_work<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  for (int mode = 0; mode < 4; ++mode) {
    for (int r = 0; r < 3; ++r) seq(mode);   // eager
    hipStreamSynchronize(s);
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    seq(mode);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int r = 0; r < 3; ++r) hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    printf("mode %d done\n", mode);
  }
  return 0;
}
