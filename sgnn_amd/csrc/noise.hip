// Random-walk position noise for training (sgnn/noise_utils.py:4-39), fused
// with the noisy window (learned_simulator.py:467):
//   n_v[t] ~ N(0, (std_last / sqrt(T-1))^2), t < T-1   (velocity increments)
//   v_noise = cumsum_t n_v ;  p_noise = [0, cumsum_t v_noise]
//   noise[i][t][c] = p_noise[t] ;  noisy = pos + noise
// The reference draws n_v on torch's CPU generator; here the normals come
// from a counter-based Philox4x32-10 stream keyed by seed and indexed by the
// GLOBAL (particle, coordinate): particle = offset + local index, so a rank
// that owns particles [offset, offset + n) of a data-parallel batch draws
// exactly the slice of the noise one process would draw for the whole
// concatenated batch (and ranks never share a stream).  Box-Muller transformed — the same
// distribution, reproducible for a given seed, one pass over the window
// instead of randn + two cumsums + cat + add.
#include "common.h"
#include "../../include/sgnn.h"
#include "sgnn_internal.h"

namespace {
struct u32x4 {
  uint32_t x, y, z, w;
};

SGNN_DEV u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// two standard normals from two uniform words (u1 in (0, 1], u2 in [0, 1))
SGNN_DEV void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float u1 = ((float)a + 1.0f) * 2.3283064365386963e-10f;
  const float u2 = (float)b * 2.3283064365386963e-10f;
  const float r = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincosf(6.283185307179586f * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

constexpr int kMaxT = 64;

__global__ __launch_bounds__(256) void k_random_walk_noise(const float* __restrict__ pos, int64_t n,
                                                           int T, int dim, float step_std,
                                                           uint64_t seed, uint64_t offset,
                                                           float* __restrict__ noise,
                                                           float* __restrict__ noisy) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (particle, coordinate)
  if (q >= n * dim) return;
  const int64_t i = q / dim;
  const int c = (int)(q - i * dim);
  const uint64_t g = (uint64_t)q + offset * (uint64_t)dim;   // global (particle, coordinate)
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  float acc_v = 0.0f, acc_p = 0.0f;
  const float* src = pos + i * T * dim + c;
  float* dn = noise + i * T * dim + c;
  float* dp = noisy + i * T * dim + c;
  dn[0] = 0.0f;
  dp[0] = src[0];
  float z[4];
  for (int t = 1; t < T; ++t) {
    const int k = t - 1;  // increment index
    if ((k & 3) == 0) {
      const u32x4 r = philox4x32_10(u32x4{(uint32_t)g, (uint32_t)(g >> 32), (uint32_t)(k >> 2), 0u}, k0, k1);
      box_muller(r.x, r.y, z[0], z[1]);
      box_muller(r.z, r.w, z[2], z[3]);
    }
    acc_v += z[k & 3] * step_std;   // cumsum of the velocity increments
    acc_p += acc_v;                 // cumsum again: position noise
    dn[t * dim] = acc_p;
    dp[t * dim] = src[t * dim] + acc_p;
  }
}
}  // namespace

extern "C" int sgnn_random_walk_noise(const float* pos_seq, int64_t n, int32_t T, int32_t dim,
                                      float noise_std_last_step, uint64_t seed, uint64_t offset,
                                      float* noise, float* noisy, void* stream) {
  using namespace sgnn;
  if (!pos_seq || !noise || !noisy || n < 0 || T < 2 || dim < 1 || dim > 3)
    return set_error(SGNN_ERR_INVALID, "random_walk_noise: bad arguments");
  if (T > kMaxT) return set_error(SGNN_ERR_UNSUPPORTED, "random_walk_noise: T > 64");
  if (n == 0) return SGNN_OK;
  const float step_std = noise_std_last_step / sqrtf((float)(T - 1));
  const int64_t items = n * dim;
  hipLaunchKernelGGL(k_random_walk_noise, dim3((unsigned)((items + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), pos_seq, n, T, dim, step_std, seed, offset, noise,
                     noisy);
  return check_launch("random_walk_noise");
}
