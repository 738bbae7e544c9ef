// qs_gae.h -- generalized advantage estimation over an HBM-resident rollout.
//
// Replaces stable_baselines3 RolloutBuffer.compute_returns_and_advantage (buffers.py, the SB3 PPO the
// reference trains with, swarm_rl/sb_train.py:53-64): for every agent column, backwards over time
//   delta_t = r_t + gamma * V_{t+1} * (1 - start_{t+1}) - V_t,   A_t = delta_t + gamma lambda (1 - start_{t+1}) A_{t+1}
// with V_T = last_values, start_T = last_dones; returns = A + V.
// Layout [T, I] row-major (time-major): at every t the I columns are one coalesced 4-byte-per-lane
// read per input and write per output; each lane carries its column's recurrence in registers.
// HBM-bound: 17 B per element (r, V, start byte in; A, returns out).
#pragma once
#ifndef __HIPCC_RTC__   // hipRTC (qs_specialize) provides these itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

namespace qs {

__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                  const uint8_t* __restrict__ starts,
                                                  const float* __restrict__ last_val,
                                                  const uint8_t* __restrict__ last_done, float* __restrict__ adv,
                                                  float* __restrict__ ret, int T, int I, float gamma, float lam) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= I) return;
    float nv = last_val[i];
    float nnt = 1.f - (float)last_done[i];
    float a = 0.f;
    const float gl = gamma * lam;
    for (int t = T - 1; t >= 0; --t) {
        const size_t k = (size_t)t * (size_t)I + (size_t)i;
        const float v = val[k];
        const float delta = rew[k] + gamma * nv * nnt - v;
        a = delta + gl * nnt * a;
        adv[k] = a;
        ret[k] = a + v;
        nnt = 1.f - (float)starts[k];
        nv = v;
    }
}

}  // namespace qs
