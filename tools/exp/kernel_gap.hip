// Round-6 experiment: does the gap between two dependent kernels on one stream grow with the bytes the
// first one leaves dirty in L2 (plain stores) vs writes through (sc1 stores)?  Run under
// rocprofv3 --kernel-trace; the trace's start/end timestamps give the gaps.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int AUX>
__global__ void k_write(float* p, long n4) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, 0x7ffffff0, 0x00020000);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    u32x4 v = {(unsigned)i, 1u, 2u, 3u};
    if (AUX == 0) *reinterpret_cast<u32x4*>(p + 4 * i) = v;
    else __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(16 * (i % (1 << 26))), 0, AUX);
  }
}
__global__ void k_tiny(float* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.0f; }
int main() {
  float* p;
  const long maxb = 256L << 20;
  hipMalloc(&p, maxb);
  for (int rep = 0; rep < 3; ++rep)
    for (long mb : {1L, 8L, 32L, 128L, 256L}) {
      long n4 = (mb << 20) / 16;
      for (int k = 0; k < 4; ++k) {
        hipLaunchKernelGGL(k_write<0>, dim3(1024), dim3(256), 0, 0, p, n4);
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, 0, p);
        hipLaunchKernelGGL(k_write<16>, dim3(1024), dim3(256), 0, 0, p, n4);
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, 0, p);
      }
      hipDeviceSynchronize();
      printf("done %ld MB\n", mb);
    }
  hipFree(p);
  return 0;
}
