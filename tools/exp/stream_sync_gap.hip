// Round-6 experiment: what a cross-stream dependency costs the launch stream.  Main stream: 16 dependent
// ~25 us kernels; after each, the side stream is made to wait for it and runs a kernel of its own, by
//   0  hipEventRecord(main) + hipStreamWaitEvent(side)           (the training step's pattern)
//   1  hipStreamWriteValue32(main) + hipStreamWaitValue32(side)   (stream memory operations)
//   2  the main kernel's last workgroup bumps a counter itself (release fence + agent atomic) +
//      hipStreamWaitValue32(side) -- nothing queued on the main stream between the kernels
//   3  a one-wave signal kernel on the main stream stores the counter (system-scope release) +
//      hipStreamWaitValue32(side)
// and, for each, whether the side kernel saw the main kernel's writes (it checks a value the main kernel
// stored).  Run under rocprofv3 --kernel-trace: the main-stream gaps are the cost.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void k_main(float* p, long n4, unsigned* done, unsigned k, int mode) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 v = reinterpret_cast<float4*>(p)[i];
    v.y += 1.0f;
    reinterpret_cast<float4*>(p)[i] = v;
  }
  if (threadIdx.x == 0) p[0] = (float)k;   // the value the side kernel checks
  if (mode == 2) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();   // this workgroup's stores before its arrival
      const unsigned prev = atomicAdd(done + 1, 1u);
      if (prev == gridDim.x * (k + 1) - 1) {   // the last workgroup of launch k
        __threadfence();
        __hip_atomic_store(done, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}
__global__ __launch_bounds__(64) void k_signal(unsigned* done, unsigned v) {
  if (threadIdx.x == 0) __hip_atomic_store(done, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(256) void k_side(float* q, long n4, const float* p, unsigned k, unsigned* bad) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && p[0] < (float)k) atomicAdd(bad, 1u);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) q[4 * i + 1] += 0.5f;
}
int main() {
  float *p, *q;
  unsigned *done, *bad;
  const long n4 = (32L << 20) / 16;
  (void)hipMalloc(&p, 64L << 20);
  (void)hipMalloc(&q, 64L << 20);
  (void)hipMalloc(&done, 64);
  (void)hipMalloc(&bad, 64);
  hipStream_t s, s2;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  for (int mode = 0; mode < 4; ++mode) {
    (void)hipMemset(done, 0, 64);
    (void)hipMemset(bad, 0, 64);
    (void)hipMemset(p, 0, 64L << 20);
    (void)hipDeviceSynchronize();
    for (unsigned k = 0; k < 16; ++k) {
      hipLaunchKernelGGL(k_main, dim3(512), dim3(256), 0, s, p, n4, done, k, mode == 2 ? 2 : 0);
      if (mode == 0) {
        (void)hipEventRecord(ev, s);
        (void)hipStreamWaitEvent(s2, ev, 0);
      } else if (mode == 1) {
        (void)hipStreamWriteValue32(s, done, k + 1, 0);
        (void)hipStreamWaitValue32(s2, done, k + 1, hipStreamWaitValueGte, 0xffffffffu);
      } else {
        if (mode == 3) hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, s, done, k + 1);
        (void)hipStreamWaitValue32(s2, done, k + 1, hipStreamWaitValueGte, 0xffffffffu);
      }
      hipLaunchKernelGGL(k_side, dim3(256), dim3(256), 0, s2, q, n4 / 4, p, k, bad);
    }
    (void)hipDeviceSynchronize();
    unsigned b = 0;
    (void)hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
    printf("mode %d done, side kernels that saw a stale value: %u\n", mode, b);
  }
  return 0;
}
