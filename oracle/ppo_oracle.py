"""CPU restatement of the PPO-side math the GPU path replaces -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (quadswarm_amd.ppo) never does.

stable_baselines3 is not installed in this image and no reference test pins its outputs,
so these follow SB3's published algorithm and are pinned by known-answer tests (tests/test_ppo_cpu.py):
  * gae_np            <- RolloutBuffer.compute_returns_and_advantage (stable_baselines3/common/buffers.py),
                         as called from OnPolicyAlgorithm.collect_rollouts; driven by swarm_rl/sb_train.py:53-104
  * squashed_logp_np  <- SquashedDiagGaussianDistribution.log_prob (stable_baselines3/common/distributions.py),
                         the distribution of ActorCriticPolicyCustom.py:336-337
"""
import math

import numpy as np


def gae_np(rewards, values, episode_starts, last_values, dones, gamma=0.99, gae_lambda=0.95):
    """fp64 GAE over [T, I] arrays; returns (advantages, returns)."""
    rewards = np.asarray(rewards, np.float64)
    values = np.asarray(values, np.float64)
    starts = np.asarray(episode_starts, np.float64)
    T = rewards.shape[0]
    adv = np.zeros_like(rewards)
    last = np.zeros_like(rewards[0])
    for step in reversed(range(T)):
        if step == T - 1:
            next_non_terminal = 1.0 - np.asarray(dones, np.float64)
            next_values = np.asarray(last_values, np.float64)
        else:
            next_non_terminal = 1.0 - starts[step + 1]
            next_values = values[step + 1]
        delta = rewards[step] + gamma * next_values * next_non_terminal - values[step]
        last = delta + gamma * gae_lambda * next_non_terminal * last
        adv[step] = last
    return adv, adv + values


def squashed_logp_np(mean, log_std, actions, epsilon=1e-6):
    """fp64 log-prob of tanh-squashed diagonal Gaussian actions [B, A]."""
    mean = np.asarray(mean, np.float64)
    log_std = np.broadcast_to(np.asarray(log_std, np.float64), mean.shape)
    eps = float(np.finfo(np.asarray(actions).dtype).eps)   # TanhBijector.inverse: eps of the action dtype
    a = np.asarray(actions, np.float64)
    y = np.clip(a, -1 + eps, 1 - eps)
    g = np.arctanh(y)
    lp = -((g - mean) ** 2) / (2 * np.exp(2 * log_std)) - log_std - 0.5 * math.log(2 * math.pi)
    return lp.sum(1) - np.log(1 - a ** 2 + epsilon).sum(1)
