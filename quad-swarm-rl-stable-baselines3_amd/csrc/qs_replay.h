// qs_replay.h -- experience replay on device (flavor B).
//
// Replaces ExperienceReplayWrapper / ReplayBuffer (gym_art/quadrotor_multi/quad_experience_replay.py:16-216) and
// the env-side bookkeeping they read (quadrotor_multi.py:182-185 state, :382-388 can_drones_fly, :461-465 reset
// accounting, :722-725 crash accumulation).  replay_env() runs one env on RL of its lanes: fused into the tail
// of the flavor-B step kernel (the env's RL = Q * NPAD lanes, after the step's stores and a workgroup fence),
// and as replay_kernel<false> (RL = 16, 4 envs per wavefront) after qs_reset.  The decision logic is a handful of per-env
// integers: the env's lanes evaluate it redundantly from broadcast loads (no cross-lane exchange) and its
// first lane writes what changed; the RL lanes then move whole env snapshots (copy loops of snap_words
// 32-bit words) when a checkpoint is saved, an event is written or an episode is replayed.  A step with
// nothing to do (the common case) costs the env's ~10 loads and no store.  Snapshots are contiguous per (env, slot) in HBM
// ([E, keep + bufsz, W]) so each copy is a coalesced burst on the store side; the live side is the SoA state.
// CPU restatement: oracle/replay_oracle.py (pinned to the reference's wrapper by tests/golden/replay_*.npz).
#pragma once
#include "qs_common.h"
#include "qs_rng.h"

namespace qs {

enum : uint32_t { S_REPLAY = 25 };
constexpr int32_t LAST_ADD_NONE = -1000000000;   // last_tick_added_to_buffer = -1e9 (:91, :195)

struct RP {
    float prob;
    int bufsz, keep, steps_ago, cp_every, grace, gap, max_rep, hist_len, hist_min;
    int W;   // snapshot words
};

struct RBufs {
    int32_t* ri;       // [QS_NR, E]
    double* crash;     // [E]
    double* hist;      // [hist_len, E]
    int32_t* perm;     // [bufsz, E]
    int32_t* nrep;     // [bufsz, E]
    uint32_t* store;   // [E, keep + bufsz, W]
};

// the flavor-B step kernel's replay arguments, in device memory after the KP block (rargs_of): read at the two
// places that use them (the done path's stats row, the replay tail) instead of occupying 23 SGPRs (or, spilled,
// serialising the kernel's argument loads) for the whole step
struct RArgs {
    uint64_t ri, crash, hist, perm, nrep, store;   // the RBufs pointers as integers (ri == 0: replay off)
    RP p;
};
// an integer address -> a global (address space 1) pointer: the accesses through it stay global_* (a pointer loaded
// from memory would be generic -> flat_*)
template <class T>
__device__ __forceinline__ T* gptr(uint64_t x) {
    typedef __attribute__((address_space(1))) T GT;
    return (T*)(reinterpret_cast<GT*>(x));
}
__device__ __forceinline__ RBufs load_rbufs(const RArgs* a) {
    RBufs r;
    r.ri = gptr<int32_t>(a->ri); r.crash = gptr<double>(a->crash); r.hist = gptr<double>(a->hist);
    r.perm = gptr<int32_t>(a->perm); r.nrep = gptr<int32_t>(a->nrep); r.store = gptr<uint32_t>(a->store);
    return r;
}

// Word w of env e's snapshot -> its live location (layout in quadswarm.h qs_replay_buffers.snap_words).
// *episode is set for the env's episode counter, which a restore leaves alone.
__device__ __forceinline__ uint32_t* snap_word(const KP& kp, const Bufs& b, int e, int w, bool* episode) {
    const int N = kp.N;
    *episode = false;
    int n = QS_NF * N;
    if (w < n) { const int f = w / N; return reinterpret_cast<uint32_t*>(b.st + (size_t)f * kp.I + (size_t)e * N + (w - f * N)); }
    w -= n;
    n = QS_NI * N;
    if (w < n) { const int f = w / N; return reinterpret_cast<uint32_t*>(b.ist + (size_t)f * kp.I + (size_t)e * N + (w - f * N)); }
    w -= n;
    n = 3 * N;
    if (w < n) { const int f = w / N; return reinterpret_cast<uint32_t*>(b.stale + (size_t)f * kp.I + (size_t)e * N + (w - f * N)); }
    w -= n;
    if (w < QS_NE) { *episode = w == QS_E_EPISODE; return reinterpret_cast<uint32_t*>(b.env + (size_t)w * kp.E + e); }
    w -= QS_NE;
    if (w < QS_NENVF) {   // the scenario floats are env-major inside their block (quadswarm.h QS_SC_NF)
        if (w >= QS_ENVF_SC_SIZE && w < QS_ENVF_SC_SIZE + QS_SC_NF)
            return reinterpret_cast<uint32_t*>(b.envf + (size_t)QS_ENVF_SC_SIZE * kp.E + (size_t)QS_SC_NF * e +
                                               (w - QS_ENVF_SC_SIZE));
        return reinterpret_cast<uint32_t*>(b.envf + (size_t)w * kp.E + e);
    }
    w -= QS_NENVF;
    n = kp.obst ? 2 * kp.M : 0;
    if (w < n) return reinterpret_cast<uint32_t*>(b.obst) + (size_t)e * n + w;
    w -= n;
    return reinterpret_cast<uint32_t*>(b.obs) + (size_t)e * N * kp.obs_dim + w;
}

constexpr int RL = 16;   // lanes per env of the standalone replay kernel

__device__ __forceinline__ void snap_save(const KP& kp, const Bufs& b, int e, uint32_t* dst, int W, int lane, int RL) {
    for (int w = lane; w < W; w += RL) {
        bool ep;
        dst[w] = *snap_word(kp, b, e, w, &ep);
    }
}

__device__ __forceinline__ void snap_restore(const KP& kp, const Bufs& b, int e, const uint32_t* src, int W, int lane,
                                             int RL) {
    for (int w = lane; w < W; w += RL) {
        bool ep;
        uint32_t* p = snap_word(kp, b, e, w, &ep);
        if (!ep) *p = src[w];
    }
}

// crashes_in_recent_episodes.append(x); activate = can_drones_fly() (quadrotor_multi.py:382-388, 462-465)
__device__ __forceinline__ int hist_push(const RP& rp, const RBufs& r, int E, int e, double x, int& hn, int& hh, bool w0) {
    if (w0) r.hist[(size_t)hh * E + e] = x;
    hh = (hh + 1) % rp.hist_len;
    hn = min(hn + 1, rp.hist_len);
    double s = 0.0;
    for (int k = 0; k < hn; ++k) {   // oldest first
        const int p = (hh - hn + k + rp.hist_len) % rp.hist_len;
        s += (p == (hh - 1 + rp.hist_len) % rp.hist_len) ? x : r.hist[(size_t)p * E + e];
    }
    return (hn >= rp.hist_min && fabs(s / hn) < 1.0) ? 1 : 0;
}

// STEP: after step_kernel (one ExperienceReplayWrapper.step per env, :124-180).
// !STEP: after reset_kernel (ExperienceReplayWrapper.reset -> env.reset accounting, :109-122) of the masked envs.
// One env on RL of its lanes (lane in [0, RL)): no barriers or cross-lane exchange inside.
template <bool STEP>
__device__ __forceinline__ void replay_env(const KP& kp, const KPM& kpm, const Bufs& b, const RBufs& r, const RP& rp, uint32_t seed,
                                           int e, int lane, int RL) {
    const int E = kp.E;
    const bool w0 = lane == 0;
    int32_t* ri = r.ri;
    int active = ri[QS_R_ACTIVE * E + e];
    int hn = ri[QS_R_HIST_N * E + e], hh = ri[QS_R_HIST_HEAD * E + e];
    double crash = r.crash[e];
    const int ri0_active = active, ri0_hn = hn, ri0_hh = hh;
    const double crash0 = crash;

    if (!STEP) {
        if (b.mask != nullptr && b.mask[e] == 0) return;
        if (!active) {
            active = hist_push(rp, r, E, e, crash, hn, hh, w0);
            crash = 0.0;
        }
        if (w0) {
            ri[QS_R_ACTIVE * E + e] = active;
            ri[QS_R_HIST_N * E + e] = hn;
            ri[QS_R_HIST_HEAD * E + e] = hh;
            r.crash[e] = crash;
        }
        return;
    }

    const int N = kp.N, W = rp.W, slots = rp.keep + rp.bufsz;
    uint32_t* st = r.store + (size_t)e * slots * W;   // this env's slots
    const int32_t flags = b.env[QS_E_FLAGS * E + e];
    const bool done = b.done[(size_t)e * N] != 0;
    const int tick = b.env[QS_E_TICK * E + e];
    int saved = ri[QS_R_SAVED * E + e];
    int ck_n = ri[QS_R_CK_N * E + e], ck_head = ri[QS_R_CK_HEAD * E + e];
    int buf_n = ri[QS_R_BUF_N * E + e], buf_idx = ri[QS_R_BUF_IDX * E + e];
    int last_add = ri[QS_R_LAST_ADD * E + e];
    const int ri0_saved = saved, ri0_ck_n = ck_n, ri0_ck_head = ck_head, ri0_buf_n = buf_n, ri0_buf_idx = buf_idx,
              ri0_last_add = last_add;
    int restored = -1, pushed = -1;

    if (!active)   // crashes_last_episode += infos[0]["rewards"]["rew_crash"] = dt * -(crash * on_floor) (:725)
        crash += -(double)kp.dt * (double)kpm.rew_crash * ((flags & QS_EF_FLOOR0) ? 1.0 : 0.0);

    if (done) {
        // the env's own reset inside step (quadrotor_multi.py:836) ...
        if (!active) {
            active = hist_push(rp, r, E, e, crash, hn, hh, w0);
            crash = 0.0;
        }
        // ... then new_episode (:182-216); the step kernel already wrote the reset env
        int episodes = ri[QS_R_EPISODES * E + e] + 1;
        last_add = LAST_ADD_NONE;
        ck_n = 0;
        ck_head = 0;
        const Rng rng = env_rng(seed, tick, b.env[QS_E_EPISODE * E + e]);
        const W4 q = block(rng, kp.id0 + (uint32_t)(e * N), S_REPLAY | UNIF_BIT, 0);
        if (u01(q.w[0]) < rp.prob && buf_n > 0 && active) {
            // sample_event (:38-45): randint(0, len - 1) = floor(v * len), v = ((w >> 8) + 0.5) / 2^24
            const int pos = (int)(((2ull * (q.w[1] >> 8) + 1ull) * (uint64_t)buf_n) >> 25);
            const int phys = r.perm[(size_t)pos * E + e];
            const int nr = r.nrep[(size_t)phys * E + e] + 1;
            snap_restore(kp, b, e, st + (size_t)(rp.keep + phys) * W, W, lane, RL);
            // cleanup (:47-54) keeps the events replayed fewer than max_rep times, in order.  Every other
            // event is already below the limit, so only the sampled one can go: it moves to the first free
            // position and the later events shift down one.
            if (w0) {
                r.nrep[(size_t)phys * E + e] = nr;
                if (nr >= rp.max_rep) {
                    for (int p = pos; p + 1 < buf_n; ++p) r.perm[(size_t)p * E + e] = r.perm[(size_t)(p + 1) * E + e];
                    r.perm[(size_t)(buf_n - 1) * E + e] = phys;
                }
                ri[QS_R_REPLAYED * E + e] += 1;
            }
            if (nr >= rp.max_rep) buf_n -= 1;
            saved = 1;   // the stored env copy has saved_in_replay_buffer = True (:26)
            restored = phys;
        } else {
            if (!active) {   // env.reset() (:209): a second history entry, 0 after the in-env reset
                active = hist_push(rp, r, E, e, crash, hn, hh, w0);
                crash = 0.0;
            }
            saved = 0;
        }
        if (w0) ri[QS_R_EPISODES * E + e] = episodes;
    } else {
        if (active && !saved && tick % rp.cp_every == 0) {   // save_checkpoint (:97-102, :157-159)
            snap_save(kp, b, e, st + (size_t)ck_head * W, W, lane, RL);
            ck_head = (ck_head + 1) % rp.keep;
            ck_n = min(ck_n + 1, rp.keep);
        }
        if ((flags & QS_EF_NEWCOL) && active && tick > rp.grace && !saved && tick - last_add > rp.gap) {
            if (rp.steps_ago > ck_n) {
                if (w0) ri[QS_R_INDEX_ERR * E + e] += 1;   // the reference raises IndexError (:171-173)
            } else {
                const int src = (ck_head - rp.steps_ago + rp.keep) % rp.keep;   // episode_checkpoints[-steps_ago]
                int pos;
                if (buf_n < rp.bufsz) pos = buf_n++;   // write_cp_to_buffer (:24-36)
                else pos = buf_idx;
                const int phys = r.perm[(size_t)pos * E + e];
                const uint32_t* from = st + (size_t)src * W;
                uint32_t* to = st + (size_t)(rp.keep + phys) * W;
                for (int w = lane; w < W; w += RL) to[w] = from[w];
                // the wrapper returns the checkpoint's obs for this step (`obs` rebound at :175, returned :180)
                const int nod = N * kp.obs_dim;
                uint32_t* obs_w = reinterpret_cast<uint32_t*>(b.obs) + (size_t)e * nod;   // bit copies
                for (int k = lane; k < nod; k += RL) obs_w[k] = from[W - nod + k];
                if (w0) r.nrep[(size_t)phys * E + e] = 0;
                buf_idx = (buf_idx + 1) % rp.bufsz;
                last_add = tick;
                pushed = phys;
            }
        }
    }
    if (w0) {
        auto put = [&](int f, int v, int was) { if (v != was) ri[f * E + e] = v; };
        put(QS_R_ACTIVE, active, ri0_active);
        put(QS_R_SAVED, saved, ri0_saved);
        put(QS_R_CK_N, ck_n, ri0_ck_n);
        put(QS_R_CK_HEAD, ck_head, ri0_ck_head);
        put(QS_R_BUF_N, buf_n, ri0_buf_n);
        put(QS_R_BUF_IDX, buf_idx, ri0_buf_idx);
        put(QS_R_LAST_ADD, last_add, ri0_last_add);
        put(QS_R_HIST_N, hn, ri0_hn);
        put(QS_R_HIST_HEAD, hh, ri0_hh);
        put(QS_R_RESTORED, restored, ri[QS_R_RESTORED * E + e]);
        put(QS_R_PUSHED, pushed, ri[QS_R_PUSHED * E + e]);
        if (crash != crash0) r.crash[e] = crash;
    }
}

template <bool STEP>
__global__ __launch_bounds__(256) void replay_kernel(const KP* __restrict__ kpp, Bufs b, RBufs r, RP rp) {
    const KP& kp = *kpp;
    const KPM kpm = load_kpm(kpp);
    const uint32_t seed = kpm.seed;
    const int e = blockIdx.x * (256 / RL) + threadIdx.x / RL;
    if (e >= kp.E) return;   // no barriers: lanes of absent envs just leave
    replay_env<STEP>(kp, kpm, b, r, rp, seed, e, threadIdx.x % RL, RL);
}

}  // namespace qs
