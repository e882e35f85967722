// Round-6 experiment: the launch-stream gap an event record costs between two dependent kernels, by event
// flags (timing off; + no system fence; + device-scope release), with a second stream waiting on the event
// and running a kernel (the training step's side-stream pattern).  Run under rocprofv3 --kernel-trace.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void k_main(float* p, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 v = reinterpret_cast<float4*>(p)[i];
    v.y += 1.0f;
    reinterpret_cast<float4*>(p)[i] = v;
  }
}
__global__ __launch_bounds__(256) void k_side(float* p, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) p[4 * i + 1] += 0.5f;
}
int main() {
  float *p, *q;
  const long n4 = (64L << 20) / 16;
  (void)hipMalloc(&p, 64L << 20);
  (void)hipMalloc(&q, 64L << 20);
  hipStream_t s, s2;
  (void)hipStreamCreate(&s);
  (void)hipStreamCreate(&s2);
  const unsigned flags[3] = {hipEventDisableTiming, hipEventDisableTiming | hipEventDisableSystemFence,
                             hipEventDisableTiming | hipEventReleaseToDevice};
  for (int f = 0; f < 3; ++f) {
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, flags[f]);
    for (int k = 0; k < 16; ++k) {
      hipLaunchKernelGGL(k_main, dim3(512), dim3(256), 0, s, p, n4);
      (void)hipEventRecord(ev, s);
      (void)hipStreamWaitEvent(s2, ev, 0);
      hipLaunchKernelGGL(k_side, dim3(256), dim3(256), 0, s2, q, n4 / 4);
    }
    (void)hipDeviceSynchronize();
    (void)hipEventDestroy(ev);
    printf("flags %d done\n", f);
  }
  return 0;
}
