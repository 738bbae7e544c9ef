// qs_curriculum.h -- sb_train's capture-radius curriculum on the device (one launch per env step).
//
// Replaces CurriculumCallback._on_step (swarm_rl/custom_callbacks.py:441-468), which SB3 calls after every
// VecEnv step of the rollout: every env the step reset (reset_infos[e] not None, in env order) writes its
// {"success"} into a window of `window` outcomes at window_i % window and advances window_i; if any env was
// reset, sucess_rate = sum(window) / window, and when it exceeds capture_radius_sr the radius is multiplied by
// capture_radius_decay, set on every env (env_method("set_capture_radius", ...)) and the window cleared.
// Here the window, the radius and the counters live in device memory (qs_curriculum), the step's reset_info
// row [E] is read where the step kernel wrote it, and the new radius goes straight into every env's
// env_f[QS_ENVF_CAPTURE] row -- no host round trip; the host reads qs_curriculum once per rollout (to log and
// to save the reference's curriculum checkpoints).  fp64 like the reference's numpy / Python floats.
//
// One workgroup of QS_CUR_THREADS lanes: lane t owns a contiguous chunk of envs, the chunk's reset count is
// scanned across the workgroup (LDS), so each reset env knows its rank r among the step's c resets; only the
// last `window` of them survive sequential writes (r >= c - window), and their slots (window_i + r) % window
// are distinct, so they are written in parallel without a race.
//
// Data-parallel training: the reference runs ONE callback over all envs of its VecEnv.  With one rank
// per GPU, each rank's handle owns a contiguous block of the global envs; the ranks all-gather their reset_info rows
// (rank-major = global env order) and every rank runs this kernel over the concatenation (n_read = world * E), so
// every rank computes the same window and radius, and writes it into its own n_write envs.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif
#include "quadswarm.h"

namespace qs {

constexpr int QS_CUR_THREADS = 256;

__global__ __launch_bounds__(QS_CUR_THREADS) void curriculum_kernel(const uint8_t* __restrict__ reset_info,
                                                                     float* __restrict__ capture, int E,
                                                                     int n_write, qs_curriculum* __restrict__ cur) {
    // the window and every value passed between lanes stay in LDS for the launch; the device struct is read at
    // the start and written back at the end
    __shared__ int scan[QS_CUR_THREADS];
    __shared__ double win[QS_CUR_MAX_WINDOW];
    __shared__ int shrink;
    __shared__ float rad;
    const int t = threadIdx.x;
    const int W = cur->window;
    const long long wi = cur->window_i;
    if (t < W) win[t] = cur->past[t];
    const int chunk = (E + QS_CUR_THREADS - 1) / QS_CUR_THREADS;
    const int e0 = min(E, t * chunk), e1 = min(E, e0 + chunk);
    int n = 0;
    for (int e = e0; e < e1; ++e) n += reset_info[e] != 0;
    scan[t] = n;
    __syncthreads();
    // inclusive Hillis-Steele scan of the per-lane counts
    for (int off = 1; off < QS_CUR_THREADS; off <<= 1) {
        const int v = t >= off ? scan[t - off] : 0;
        __syncthreads();
        scan[t] += v;
        __syncthreads();
    }
    const int c = scan[QS_CUR_THREADS - 1];
    int r = scan[t] - n;   // rank of this lane's first reset env among the step's c resets
    for (int e = e0; e < e1; ++e) {
        const uint8_t v = reset_info[e];
        if (v == 0) continue;
        if (r >= c - W) win[(int)((wi + r) % W)] = v == 2 ? 1.0 : 0.0;
        ++r;
    }
    __syncthreads();
    if (t == 0) {
        int s = 0;
        if (c > 0) {
            cur->window_i = wi + c;
            double sum = 0.0;
            for (int k = 0; k < W; ++k) sum += win[k];   // 0/1 values: exact in any order, like np.sum
            const double sr = sum / (double)W;
            cur->success_rate = sr;
            if (sr > cur->sr_threshold) {
                const double nr = cur->decay * cur->radius;
                cur->radius = nr;
                cur->history[cur->n_shrinks % QS_CUR_MAX_HIST] = nr;
                cur->n_shrinks += 1;
                rad = (float)nr;
                s = 1;
            }
        }
        shrink = s;
    }
    __syncthreads();
    if (t < W) cur->past[t] = shrink ? 0.0 : win[t];
    if (shrink)
        for (int e = t; e < n_write; e += QS_CUR_THREADS) capture[e] = rad;
}

}  // namespace qs
