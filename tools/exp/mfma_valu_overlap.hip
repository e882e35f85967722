// Experiment: does one wave's f32 MFMA stream overlap another wave's (or its own) VALU stream on the
// same SIMD?  512 threads = 8 waves, waves w and w + 4 share a SIMD.  Per-wave s_memtime spans.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mfma_block(f32x4 (&acc)[4], float a, float b, int n) {
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
  }
}
__device__ __forceinline__ void valu_block(float (&v)[8], float a, int n) {
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = __builtin_fmaf(v[k], a, 0.5f);
  }
}
__device__ __forceinline__ void mixed_block(f32x4 (&acc)[4], float (&v)[8], float a, float b, int n) {
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
      v[2 * t] = __builtin_fmaf(v[2 * t], a, 0.5f);
      v[2 * t + 1] = __builtin_fmaf(v[2 * t + 1], a, 0.5f);
    }
  }
}

__global__ __launch_bounds__(512) void k(int mode, int nm, int nv, float* out, unsigned long long* tm) {
  const int w = threadIdx.x / 64;
  f32x4 acc[4] = {};
  float v[8];
  for (int k2 = 0; k2 < 8; ++k2) v[k2] = threadIdx.x * 1e-3f + k2;
  const float a = 0.999f + threadIdx.x * 1e-7f, b = 1.0001f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const bool lo = w < 4;
  if (mode == 0) { if (lo) mfma_block(acc, a, b, nm); }
  else if (mode == 1) { if (!lo) valu_block(v, a, nv); }
  else if (mode == 2) { if (lo) mfma_block(acc, a, b, nm); else valu_block(v, a, nv); }
  else if (mode == 3) { if (lo) mixed_block(acc, v, a, b, nm); }          // same counts in ONE wave
  else if (mode == 4) { if (lo) { mfma_block(acc, a, b, nm); valu_block(v, a, nm); } }  // serial, one wave (mode 3 counts)
  else if (mode == 5) { mfma_block(acc, a, b, nm); }                      // both waves MFMA
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int t = 0; t < 4; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  for (int k2 = 0; k2 < 8; ++k2) s += v[k2];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) tm[blockIdx.x * 8 + w] = t1 - t0;
}

int main() {
  const int nm = 256, nv = 4 * nm * 2 / 8 * 4;  // 1024 MFMAs (32k cyc); 8 * nv FMAs
  float* out; unsigned long long* tm;
  hipMalloc(&out, 256 * 512 * 4); hipMalloc(&tm, 256 * 8 * 8);
  const char* names[] = {"mfma only (w0-3)", "valu only (w4-7)", "mfma w0-3 + valu w4-7", "mixed in one wave (w0-3)",
                         "mfma then valu, one wave", "mfma on all 8 waves"};
  for (int mode = 0; mode < 6; ++mode) {
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, mode, nm, nv, out, tm);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(256 * 8);
    hipMemcpy(h.data(), tm, h.size() * 8, hipMemcpyDeviceToHost);
    double lo = 0, hi = 0;
    for (int bl = 0; bl < 256; ++bl)
      for (int w = 0; w < 8; ++w) (w < 4 ? lo : hi) += h[bl * 8 + w];
    printf("%-28s waves0-3 %8.0f  waves4-7 %8.0f cycles (s_memtime)\n", names[mode], lo / 1024, hi / 1024);
  }
  printf("counts: %d MFMA (16x16x4 f32) and %d v_fma_f32 per wave\n", 4 * nm, 8 * nv);
  return 0;
}
