// Fused Adam over the flat fp32 parameter buffer (replaces torch.optim.Adam's
// multi-tensor path used by sgnn/single_scale/train.py:199,271-273).
// Same arithmetic order as torch 2.x Adam (amsgrad=False, weight_decay=0):
//   m = lerp(m, g, 1-b1) ; v = v*b2 + (1-b2)*g*g
//   p += -step_size * m / (sqrt(v)/sqrt(1-b2^t) + eps),  step_size = lr/(1-b1^t)
#include "common.h"
#include "../../include/sgnn.h"
#include "sgnn_internal.h"

namespace {
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              int64_t n, float w1, float b2, float omb2,
                                              float neg_step, float bc2_sqrt, float eps) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    float mi = m[i];
    mi = __fadd_rn(mi, __fmul_rn(w1, __fsub_rn(gi, mi)));  // lerp, weight < 0.5 branch
    float vi = __fadd_rn(__fmul_rn(v[i], b2), __fmul_rn(omb2, __fmul_rn(gi, gi)));
    const float denom = __fadd_rn(__fdiv_rn(sqrtf(vi), bc2_sqrt), eps);
    p[i] = __fadd_rn(p[i], __fmul_rn(neg_step, __fdiv_rn(mi, denom)));
    m[i] = mi;
    v[i] = vi;
  }
}
}  // namespace

extern "C" int sgnn_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              int64_t n, float lr, float beta1, float beta2, float eps,
                              int64_t step, void* stream) {
  using namespace sgnn;
  if (!param || !grad || !exp_avg || !exp_avg_sq || n < 0 || step < 1)
    return set_error(SGNN_ERR_INVALID, "adam_step: bad arguments");
  if (!(1.0f - beta1 < 0.5f)) return set_error(SGNN_ERR_UNSUPPORTED, "adam_step: beta1 <= 0.5");
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float neg_step = (float)(-(double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 2048);
  if (n == 0) return SGNN_OK;
  hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), param,
                     grad, exp_avg, exp_avg_sq, n, 1.0f - beta1, beta2, 1.0f - beta2, neg_step,
                     bc2_sqrt, eps);
  return check_launch("adam_step");
}
